"""Device-resident batched seal/open over torch tensors (torch = HBM allocator + streams only).

All functions launch asynchronously on `stream` (default: torch's current
stream) and return immediately; the crypto runs in the gfx950 kernels of
libcurvezmq_mi355x.so.
"""
import ctypes

import numpy as np

from . import _lib


def _stream(stream):
    import torch
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    return getattr(stream, "cuda_stream", stream)


def _ptr(t):
    return None if t is None else t.data_ptr()


def _need_cuda_u8(t, what):
    import torch
    if t is None or not t.is_cuda:
        raise ValueError(f"{what} must be a CUDA (HIP) tensor")
    if t.dtype != torch.uint8 and what not in ("desc",):
        raise ValueError(f"{what} must be uint8")


def subkeys(precom, direction, stream=None):
    """precom: (nkeys, 32) uint8 device tensor -> (nkeys, 32) subkeys for `direction`."""
    import torch
    _need_cuda_u8(precom, "precom")
    out = torch.empty_like(precom)
    _lib.check(_lib.lib().cz_subkeys(_ptr(out), _ptr(precom), precom.shape[0], direction, _stream(stream)),
               "cz_subkeys")
    return out


def seal_uniform(inp, in_stride, out, out_stride, count, length, subkey, counter0, flags8=None, stream=None):
    """Seal `count` payloads of `length` bytes (frame i at in[i*in_stride]) into MESSAGE
    bodies; body i goes to slot i = out[i*out_stride : (i+1)*out_stride].  The batch owns
    whole slots: slot bytes past the body are written (as zeros)."""
    _need_cuda_u8(inp, "in")
    _need_cuda_u8(out, "out")
    need_in = (count - 1) * in_stride + length if count else 0
    need_out = count * out_stride if count else 0
    if out_stride < length + _lib.CZ_MESSAGE_OVERHEAD and count > 1:
        raise ValueError("out_stride smaller than a MESSAGE body")
    if inp.numel() < need_in or out.numel() < need_out:
        raise ValueError("buffer too small for the batch")
    if flags8 is not None and flags8.numel() < count:
        raise ValueError("flags8 too small")
    _lib.check(_lib.lib().cz_seal_uniform(count, length, _ptr(inp), in_stride, _ptr(out), out_stride, _ptr(subkey),
                                          counter0, _ptr(flags8), _stream(stream)), "cz_seal_uniform")


def seal_uniform_box(box, box_stride, out, out_stride, count, length, subkey, counter0, stream=None):
    """Uniform seal from the reference's box layout: slot i of `box` holds 0^32 || flags ||
    payload (length = payload bytes), as CurveClientMechanism.encode hands it to Curve.afternm."""
    _need_cuda_u8(box, "box")
    _need_cuda_u8(out, "out")
    if count:  # (like seal_uniform, the batch owns whole output slots)
        if box.numel() < (count - 1) * box_stride + length + 33 or out.numel() < count * out_stride:
            raise ValueError("seal_uniform_box: buffers smaller than the batch")
    _lib.check(_lib.lib().cz_seal_uniform_box(count, length, _ptr(box), box_stride, _ptr(out), out_stride,
                                              _ptr(subkey), counter0, _stream(stream)), "cz_seal_uniform_box")


def open_uniform(inp, in_stride, out, out_stride, count, size, subkey, floor0, status, check=True, stream=None):
    """Open `count` bodies of `size` bytes of one connection, in order; payload i goes to
    slot out[i*out_stride : (i+1)*out_stride] (whole slots owned by the batch)."""
    _need_cuda_u8(inp, "in")
    _need_cuda_u8(out, "out")
    if count and (inp.numel() < (count - 1) * in_stride + size or status.numel() < count):
        raise ValueError("buffer too small for the batch")
    if count and size >= 33 and out.numel() < count * out_stride:
        raise ValueError("output too small for the batch (needs count * out_stride bytes)")
    _lib.check(_lib.lib().cz_open_uniform(count, size, _ptr(inp), in_stride, _ptr(out), out_stride, _ptr(subkey),
                                          floor0, 1 if check else 0, _ptr(status), _stream(stream)),
               "cz_open_uniform")


def _check_desc_bounds(desc_np, in_bytes, out_bytes, nkeys, seal):
    ln = desc_np["len"].astype(np.uint64)
    olen = ln + np.uint64(33) if seal else np.where(ln >= 33, ln - np.uint64(33), 0).astype(np.uint64)
    if len(desc_np) and (np.any(desc_np["in_off"] + ln > np.uint64(in_bytes))
                         or np.any(desc_np["out_off"] + olen > np.uint64(out_bytes))
                         or np.any(desc_np["key_idx"] >= nkeys)):
        raise ValueError("descriptor out of bounds")


def seal_batch(desc, count, inp, out, subkeys_t, order=None, stream=None, desc_np=None):
    """desc: device tensor holding `count` cz_frame_desc (40 B each).  If desc_np (the host
    copy, numpy DESC dtype) is given, bounds are checked before the launch."""
    _need_cuda_u8(inp, "in")
    _need_cuda_u8(out, "out")
    if desc_np is not None:
        _check_desc_bounds(desc_np, inp.numel(), out.numel(), subkeys_t.shape[0], True)
    _lib.check(_lib.lib().cz_seal_batch(_ptr(desc), _ptr(order), count, _ptr(inp), _ptr(out), _ptr(subkeys_t),
                                        _stream(stream)), "cz_seal_batch")


def open_batch(desc, count, inp, out, subkeys_t, status, nonces=None, order=None, stream=None, desc_np=None):
    _need_cuda_u8(inp, "in")
    _need_cuda_u8(out, "out")
    if desc_np is not None:
        _check_desc_bounds(desc_np, inp.numel(), out.numel(), subkeys_t.shape[0], False)
    _lib.check(_lib.lib().cz_open_batch(_ptr(desc), _ptr(order), count, _ptr(inp), _ptr(out), _ptr(subkeys_t),
                                        _ptr(status), _ptr(nonces), _stream(stream)), "cz_open_batch")


def fill(buf, seed, stream=None):
    """Counter-based SplitMix64 synthetic bytes (tests/cz_testlib.py splitmix_words)."""
    _lib.check(_lib.lib().cz_fill(_ptr(buf), buf.numel() * buf.element_size(), seed, _stream(stream)), "cz_fill")


def plan_order(desc_np):
    """Frame indices sorted by decreasing length (balances lanes of a ragged batch)."""
    count = len(desc_np)
    order = np.zeros(count, dtype=np.uint32)
    d = np.ascontiguousarray(desc_np)
    _lib.check(_lib.lib().cz_plan_order(d.ctypes.data, count, order.ctypes.data), "cz_plan_order")
    return order


DESC_DTYPE = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("len", "<u4"), ("key_idx", "<u4"),
                       ("counter", "<u8"), ("flags", "<u4"), ("prev", "<i4")])

SEGMENT_DTYPE = np.dtype([("frame", "<u4"), ("first_block", "<u4"), ("nblocks", "<u4"), ("part", "<u4")])
COMBINE_DTYPE = np.dtype([("frame", "<u4"), ("part0", "<u4"), ("nseg", "<u4"), ("reserved", "<u4")])
SEG_BLOCKS = 128  # 8 KiB of box per lane (Zipf sweep: 64 -> 1664, 128 -> 1687-1709, 160 -> 1707, 192 -> 1671 GiB/s)


class SegmentPlan:
    """Host plan for a ragged batch: frames longer than 1.5 x seg_blocks are split
    into seg_blocks-block segments (cz_plan_segments).  `to(device)` uploads the
    segment and combine lists and allocates the partial-record workspace."""

    def __init__(self, desc_np, open_=False, seg_blocks=SEG_BLOCKS):
        d = np.ascontiguousarray(desc_np)
        count = len(d)
        nseg, ncomb, npart = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        L = _lib.lib()
        L.cz_plan_segments(d.ctypes.data, count, int(open_), seg_blocks, None, 0, ctypes.byref(nseg), None, 0,
                           ctypes.byref(ncomb), ctypes.byref(npart))
        self.segments = np.zeros(max(nseg.value, 1), dtype=SEGMENT_DTYPE)
        self.combines = np.zeros(max(ncomb.value, 1), dtype=COMBINE_DTYPE)
        _lib.check(L.cz_plan_segments(d.ctypes.data, count, int(open_), seg_blocks, self.segments.ctypes.data,
                                      len(self.segments), ctypes.byref(nseg), self.combines.ctypes.data,
                                      len(self.combines), ctypes.byref(ncomb), ctypes.byref(npart)),
                   "cz_plan_segments")
        self.nseg, self.ncomb, self.npart = nseg.value, ncomb.value, npart.value
        self.segments = self.segments[:self.nseg]
        self.combines = self.combines[:self.ncomb]
        self.d_seg = self.d_comb = self.d_work = None

    def to(self, device):
        import torch
        self.d_seg = torch.from_numpy(self.segments.view(np.uint8).copy()).to(device)
        self.d_comb = torch.from_numpy(self.combines.view(np.uint8).copy()).to(device)
        self.d_work = torch.empty(max(self.npart, 1) * 64, dtype=torch.uint8, device=device)
        return self


def seal_segments(desc, plan, inp, out, subkeys_t, stream=None, desc_np=None):
    """Ragged seal with long frames split across lanes (same output as seal_batch)."""
    _need_cuda_u8(inp, "in")
    _need_cuda_u8(out, "out")
    if desc_np is not None:
        _check_desc_bounds(desc_np, inp.numel(), out.numel(), subkeys_t.shape[0], True)
    _lib.check(_lib.lib().cz_seal_segments(_ptr(desc), _ptr(plan.d_seg), plan.nseg, _ptr(plan.d_comb), plan.ncomb,
                                           _ptr(inp), _ptr(out), _ptr(subkeys_t), _ptr(plan.d_work),
                                           _stream(stream)), "cz_seal_segments")


def open_segments(desc, plan, inp, out, subkeys_t, status, nonces=None, stream=None, desc_np=None):
    """Ragged open with long frames split across lanes (same output as open_batch)."""
    _need_cuda_u8(inp, "in")
    _need_cuda_u8(out, "out")
    if desc_np is not None:
        _check_desc_bounds(desc_np, inp.numel(), out.numel(), subkeys_t.shape[0], False)
    _lib.check(_lib.lib().cz_open_segments(_ptr(desc), _ptr(plan.d_seg), plan.nseg, _ptr(plan.d_comb), plan.ncomb,
                                           _ptr(inp), _ptr(out), _ptr(subkeys_t), _ptr(plan.d_work), _ptr(status),
                                           _ptr(nonces), _stream(stream)), "cz_open_segments")

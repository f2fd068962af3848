"""ZMTP v2 framing (zmq/io/coder/v2/V2Encoder.java, V2Decoder.java) over the C-ABI.

`parse` is the host V2Decoder walk (one header per frame, no device needed);
`copy` launches the device pack/unpack kernel (k_v2_copy) that moves bodies
between aligned slots and socket-ready wire streams.
"""
import ctypes

import numpy as np

from . import _lib

V2_FRAME_DTYPE = np.dtype([("body_off", "<u8"), ("size", "<u4"), ("msg_flags", "<u4")])
V2_ITEM_DTYPE = np.dtype([("src_off", "<u8"), ("dst_off", "<u8"), ("size", "<u4"), ("flags", "<u4")])


def header_size(size):
    """2, or 9 when the body exceeds 255 bytes (V2Encoder.java:33-55)."""
    return int(_lib.lib().cz_v2_header_size(size))


def parse(wire, maxmsgsize=-1, cap=None):
    """Parse whole frames of `wire` (bytes-like).  Returns (frames, consumed, rc): frames is a
    V2_FRAME_DTYPE array, consumed the bytes of whole frames, rc CZ_OK / CZ_EPROTO / CZ_EMSGSIZE
    for a bad header after the returned frames (V2Decoder.java:52-58, Decoder.java:76-98)."""
    buf = np.frombuffer(bytes(wire), dtype=np.uint8)
    if cap is None:
        cap = len(buf) // 2 + 1
    frames = np.zeros(max(cap, 1), dtype=V2_FRAME_DTYPE)
    nf, consumed = ctypes.c_uint32(), ctypes.c_uint64()
    rc = _lib.lib().cz_v2_parse(buf.ctypes.data if len(buf) else None, len(buf), maxmsgsize, frames.ctypes.data,
                                cap, ctypes.byref(nf), ctypes.byref(consumed))
    return frames[:nf.value], consumed.value, rc


def copy(items, src, dst, stream=None):
    """Device pack/unpack: items = device tensor of V2_ITEM_DTYPE records (24 B each)."""
    from .batch import _ptr, _stream
    count = items.numel() // V2_ITEM_DTYPE.itemsize
    _lib.check(_lib.lib().cz_v2_copy(_ptr(items), count, _ptr(src), _ptr(dst), _stream(stream)), "cz_v2_copy")

"""ctypes binding of libcurvezmq_mi355x.so (the C-ABI in include/curvezmq_mi355x.h).

The library is the product: every byte of ciphertext, plaintext and every tag
comes from its gfx950 kernels.  There is no CPU fallback -- if the shared
object is missing this module raises, and on a machine without a GPU the
compute entry points return CZ_EHIP.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CZ_LIB", os.path.join(HERE, "libcurvezmq_mi355x.so"))  # CZ_LIB: A/B builds only

CZ_OK = 0
CZ_EINVAL = -22
CZ_EHIP = -5
CZ_ENOMEM = -12
CZ_EPROTO = -71
CZ_EMSGSIZE = -90
CZ_EAGAIN = -11
CZ_MESSAGE_MAX = 0x7fffffff - 33

CZ_HS_HANDSHAKING = 0
CZ_HS_READY = 1
CZ_HS_ERROR = 2

CZ_STATUS_OK = 0
CZ_STATUS_CRYPTO = 1
CZ_STATUS_MALFORMED = 2
CZ_STATUS_COMMAND = 3
CZ_STATUS_SEQUENCE = 4

CZ_DIR_C2S = 0
CZ_DIR_S2C = 1
CZ_MSG_MORE = 0x01
CZ_MSG_COMMAND = 0x02
CZ_DESC_CHECK_NONCE = 0x100
CZ_MESSAGE_OVERHEAD = 33

CZ_V2_MORE = 0x01
CZ_V2_LARGE = 0x02
CZ_V2_COMMAND = 0x04
CZ_V2_ITEM_HEADER = 0x100

CZ_ZMTP_UNEXPECTED_COMMAND = 0x10000001
CZ_ZMTP_MALFORMED_COMMAND_MESSAGE = 0x10000012
CZ_ZMTP_INVALID_SEQUENCE = 0x10000002
CZ_ZMTP_CRYPTOGRAPHIC = 0x11000001
CZ_ZMTP_UNSPECIFIED = 0x10000000
CZ_ZMTP_KEY_EXCHANGE = 0x10000003
CZ_ZMTP_MALFORMED_COMMAND_HELLO = 0x10000013
CZ_ZMTP_MALFORMED_COMMAND_INITIATE = 0x10000014
CZ_ZMTP_MALFORMED_COMMAND_ERROR = 0x10000015
CZ_ZMTP_MALFORMED_COMMAND_READY = 0x10000016
CZ_ZAP_MALFORMED_REPLY = 0x20000001
CZ_ZAP_INVALID_STATUS_CODE = 0x20000004


class CzError(RuntimeError):
    pass


class cz_frame_desc(ctypes.Structure):
    _fields_ = [("in_off", ctypes.c_uint64), ("out_off", ctypes.c_uint64), ("len", ctypes.c_uint32),
                ("key_idx", ctypes.c_uint32), ("counter", ctypes.c_uint64), ("flags", ctypes.c_uint32),
                ("prev", ctypes.c_int32)]


assert ctypes.sizeof(cz_frame_desc) == 40


class cz_v2_frame(ctypes.Structure):
    _fields_ = [("body_off", ctypes.c_uint64), ("size", ctypes.c_uint32), ("msg_flags", ctypes.c_uint32)]


class cz_v2_item(ctypes.Structure):
    _fields_ = [("src_off", ctypes.c_uint64), ("dst_off", ctypes.c_uint64), ("size", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


assert ctypes.sizeof(cz_v2_frame) == 16 and ctypes.sizeof(cz_v2_item) == 24

_VP = ctypes.c_void_p
_P = ctypes.c_char_p
_U8P = ctypes.POINTER(ctypes.c_uint8)
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I = ctypes.c_int

# name -> (restype, argtypes); must cover every function in include/curvezmq_mi355x.h
SIGNATURES = {
    "cz_box_afternm": (_I, [_VP, _VP, _U64, _VP, _VP]),
    "cz_box_open_afternm": (_I, [_VP, _VP, _U64, _VP, _VP]),
    "cz_secretbox": (_I, [_VP, _VP, _U64, _VP, _VP]),
    "cz_secretbox_open": (_I, [_VP, _VP, _U64, _VP, _VP]),
    "cz_subkeys": (_I, [_VP, _VP, _U32, _I, _VP]),
    "cz_subkey": (_I, [_VP, _VP, _I]),
    "cz_seal_batch": (_I, [_VP, _VP, _U32, _VP, _VP, _VP, _VP]),
    "cz_open_batch": (_I, [_VP, _VP, _U32, _VP, _VP, _VP, _VP, _VP, _VP]),
    "cz_seal_uniform": (_I, [_U32, _U32, _VP, _U64, _VP, _U64, _VP, _U64, _VP, _VP]),
    "cz_seal_uniform_box": (_I, [_U32, _U32, _VP, _U64, _VP, _U64, _VP, _U64, _VP]),
    "cz_open_uniform": (_I, [_U32, _U32, _VP, _U64, _VP, _U64, _VP, _U64, _I, _VP, _VP]),
    "cz_plan_order": (_I, [_VP, _U32, _VP]),
    "cz_plan_segments": (_I, [_VP, _U32, _I, _U32, _VP, _U32, ctypes.POINTER(_U32), _VP, _U32,
                              ctypes.POINTER(_U32), ctypes.POINTER(_U32)]),
    "cz_seal_segments": (_I, [_VP, _VP, _U32, _VP, _U32, _VP, _VP, _VP, _VP, _VP]),
    "cz_open_segments": (_I, [_VP, _VP, _U32, _VP, _U32, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    "cz_fill": (_I, [_VP, _U64, _U64, _VP]),
    "cz_dev_copy": (_I, [_VP, _VP, _U64, _VP]),
    "cz_nacl_forget": (_I, []),
    "cz_ctx_create": (_I, [ctypes.POINTER(_VP), _I]),
    "cz_ctx_destroy": (None, [_VP]),
    "cz_ctx_set_keys": (_I, [_VP, _VP, _U32, _I]),
    "cz_ctx_seal": (_I, [_VP, _VP, _U32, _VP, _U64, _VP, _U64]),
    "cz_ctx_open": (_I, [_VP, _VP, _U32, _VP, _U64, _VP, _U64, _VP]),
    "cz_ctx_seal_uniform": (_I, [_VP, _U32, _U32, _VP, _U64, _VP, _U64, _U64, _VP, _U32]),
    "cz_ctx_open_uniform": (_I, [_VP, _U32, _U32, _VP, _U64, _VP, _U64, _U64, _I, _VP, _U32]),
    "cz_host_alloc": (_VP, [_U64]),
    "cz_host_free": (_I, [_VP]),
    "cz_nacl_thread_init": (_I, []),
    "cz_mech_create": (_VP, [_I, _VP, _U64, _U64, _I]),
    "cz_mech_destroy": (None, [_VP]),
    "cz_mech_encode": (ctypes.c_int64, [_VP, _VP, _U64, _I, _VP]),
    "cz_mech_decode": (ctypes.c_int64, [_VP, _VP, _U64, _VP, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "cz_mech_encode_batch": (_I, [_VP, _U32, _VP, _VP, _VP, _VP, _VP, _VP]),
    "cz_mech_decode_batch": (_I, [_VP, _U32, _VP, _VP, _VP, _VP, _VP, _VP, _VP, ctypes.POINTER(_I)]),
    "cz_mech_nonce": (_U64, [_VP]),
    "cz_mech_peer_nonce": (_U64, [_VP]),
    "cz_v2_header_size": (_U32, [_U64]),
    "cz_v2_parse": (_I, [_VP, _U64, ctypes.c_int64, _VP, _U32, ctypes.POINTER(_U32), ctypes.POINTER(_U64)]),
    "cz_v2_copy": (_I, [_VP, _U32, _VP, _VP, _VP]),
    "cz_engine_create": (_I, [ctypes.POINTER(_VP), _U64, _I]),
    "cz_engine_destroy": (None, [_VP]),
    "cz_engine_add_conn": (_I, [_VP, _I, _VP, _U64, _U64]),
    "cz_engine_remove_conn": (_I, [_VP, _I]),
    "cz_engine_msg_alloc": (_VP, [_VP, _U32]),
    "cz_engine_send": (_I, [_VP, _I, _VP, _U32, _I]),
    "cz_engine_flush_out": (_I, [_VP]),
    "cz_engine_wire_out": (_I, [_VP, _I, ctypes.POINTER(_VP), ctypes.POINTER(_U64)]),
    "cz_engine_wire_iov": (_I, [_VP, _I, _VP, _U32, ctypes.POINTER(_U32)]),
    "cz_engine_recv": (_I, [_VP, _I, _VP, _U64]),
    "cz_engine_recv_buffer": (_I, [_VP, _I, _U64, ctypes.POINTER(_VP), ctypes.POINTER(_U64)]),
    "cz_engine_recv_commit": (_I, [_VP, _I, _U64]),
    "cz_engine_flush_in": (_I, [_VP]),
    "cz_engine_msgs_in": (_I, [_VP, _I, ctypes.POINTER(_U32)]),
    "cz_engine_msg_in": (_I, [_VP, _I, _U32, ctypes.POINTER(_VP), ctypes.POINTER(_U32), ctypes.POINTER(_I)]),
    "cz_engine_conn_error": (_I, [_VP, _I, ctypes.POINTER(_I)]),
    "cz_engine_nonce": (_U64, [_VP, _I]),
    "cz_engine_peer_nonce": (_U64, [_VP, _I]),
    "cz_scalarmult": (_I, [_VP, _VP, _VP]),
    "cz_box_keypair": (_I, [_VP, _VP]),
    "cz_box_beforenm": (_I, [_VP, _VP, _VP]),
    "cz_box": (_I, [_VP, _VP, _U64, _VP, _VP, _VP]),
    "cz_box_open": (_I, [_VP, _VP, _U64, _VP, _VP, _VP]),
    "cz_x25519_batch": (_I, [_VP, _VP, _VP, _U32, _VP]),
    "cz_beforenm_batch": (_I, [_VP, _VP, _VP, _U32, _VP]),
    "cz_hs_create": (_I, [ctypes.POINTER(_VP), _I, _VP, _VP, _VP, _I, _VP, _U32, _VP, _VP, _U32]),
    "cz_hs_destroy": (None, [_VP]),
    "cz_hs_next_command": (_I, [_VP, _VP, _U32, ctypes.POINTER(_U32)]),
    "cz_hs_process_command": (_I, [_VP, _VP, _U64]),
    "cz_hs_status": (_I, [_VP]),
    "cz_hs_event": (_I, [_VP]),
    "cz_hs_error_status": (_I, [_VP]),
    "cz_hs_set_zap": (_I, [_VP, _I]),
    "cz_hs_zap_reply": (_I, [_VP, ctypes.c_char_p]),
    "cz_hs_client_key": (_I, [_VP, _VP]),
    "cz_hs_session": (_I, [_VP, _VP, ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    "cz_hs_peer_property": (_I, [_VP, ctypes.c_char_p, ctypes.POINTER(_VP), ctypes.POINTER(_U32)]),
    "cz_hs_mechanism": (_VP, [_VP, _I]),
    "cz_engine_add_session": (_I, [_VP, _VP]),
    "cz_zmtp_metadata_check": (_I, [_VP, _U64, _I]),
    "cz_zmtp_metadata": (_U32, [_I, _VP, _U32, _VP, _U32]),
    "cz_last_error": (ctypes.c_char_p, []),
    "cz_version": (ctypes.c_char_p, []),
    "cz_device_ok": (_I, []),
    "cz_tune": (_I, [ctypes.c_char_p, _I]),
}

_LIB = None


def _torch_runtime_first():
    """PyTorch bundles its own libamdhip64 / libhsa-runtime64, loaded into the global symbol scope by
    `import torch`.  Importing torch before the library binds the library's HIP calls to that same
    runtime: one runtime in the process.  Loaded the other way round, the process holds two, and
    whichever initializes second sees no device (tools/diag/hip_init_order.py,
    profiles/r06/hip_init_order.log).  torch is imported only, not initialized."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib():
    """Load the HIP library; raise loudly if it has not been built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise CzError(f"{LIB_PATH} is missing: run `python -m jeromq_amd.build` (hipcc, gfx950). "
                      "There is no CPU fallback for the CURVE path.")
    _torch_runtime_first()
    L = ctypes.CDLL(LIB_PATH)
    ab_variant = "CZ_LIB" in os.environ  # an older A/B build may predate a symbol; the product may not
    for name, (res, args) in SIGNATURES.items():
        if ab_variant and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    # A/B and profiling runs only: CZ_TUNE="open_seg_carry=0,pair=1" sets cz_tune knobs at load
    for kv in filter(None, os.environ.get("CZ_TUNE", "").split(",")):
        k, v = kv.split("=")
        if L.cz_tune(k.strip().encode(), int(v)) < 0:
            raise CzError(f"CZ_TUNE: unknown knob {k!r}")
    _LIB = L
    return L


def last_error():
    return lib().cz_last_error().decode(errors="replace")


def check(rc, what="cz call"):
    if rc != CZ_OK:
        raise CzError(f"{what} failed ({rc}): {last_error()}")
    return rc

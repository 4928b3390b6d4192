"""ctypes binding of libmec (include/mec.h).

The shared library is built in-tree by ``make -C memec_amd`` (or
``__graft_entry__.build()``).  There is no fallback: if libmec.so is missing
or cannot be loaded, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# MEMEC_LIBMEC: another build of the same library (the bounds-checked
# debug build, make -C memec_amd bounds); default the in-tree release build
LIB_PATH = os.environ.get("MEMEC_LIBMEC") or os.path.join(HERE, "libmec.so")

MEC_OK, MEC_EINVAL, MEC_ENOMEM, MEC_EHIP, MEC_ETOOMANY, MEC_ESINGULAR, MEC_ENODEV = 0, -1, -2, -3, -4, -5, -6
FAMILIES = {"rs": 0, "cauchy": 1, "isal_rs": 2, "isal_cauchy": 3}

# Exported symbols declared by include/mec.h (checked by tests/test_abi.py).
SYMBOLS = (
    "mec_abi_version", "mec_create", "mec_create_multi", "mec_destroy", "mec_last_error", "mec_get_info",
    "mec_get_matrix", "mec_get_bitmatrix", "mec_encode", "mec_decode", "mec_decode_split",
    "mec_encode_update", "mec_xor", "mec_fill_random", "mec_encode_host", "mec_decode_host",
    "mec_encode_update_host", "mec_encode_host_batch", "mec_host_register", "mec_host_unregister",
    "mec_encode_batch", "mec_decode_batch", "mec_encode_update_batch", "mec_set_coalescing", "mec_set_host_queue", "mec_get_stats",
    "mec_set_probe", "mec_set_knob", "mec_queue_trace_enable", "mec_queue_last_trace",
    "mec_encode_batch32", "mec_decode_batch32", "mec_encode_update_batch32",
)
NULL_OFF = 0xFFFFFFFF  # MEC_NULL_OFF
MEM_DEVICE, MEM_HOST = 0, 1


class MecError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libmec error %d: %s" % (code, msg))
        self.code = code


class MecInfo(ctypes.Structure):
    _fields_ = [("family", ctypes.c_int32), ("k", ctypes.c_uint32), ("m", ctypes.c_uint32),
                ("w", ctypes.c_uint32), ("chunk_size", ctypes.c_uint32),
                ("packet_size", ctypes.c_uint32), ("device", ctypes.c_int32)]


class MecStats(ctypes.Structure):
    _fields_ = [("coalesced_batches", ctypes.c_uint64), ("coalesced_requests", ctypes.c_uint64),
                ("cached_plans", ctypes.c_uint64), ("zero_copy_calls", ctypes.c_uint64),
                ("staged_calls", ctypes.c_uint64), ("queue_calls", ctypes.c_uint64),
                ("queue_launches", ctypes.c_uint64), ("queue_slots", ctypes.c_uint32),
                ("queue_parts", ctypes.c_uint32), ("queue_broken", ctypes.c_uint32), ("queue_devslot", ctypes.c_uint32),
                ("queue_timeouts", ctypes.c_uint64), ("mg_cache_bytes", ctypes.c_uint64),
                ("mg_cache_tables", ctypes.c_uint64), ("mg_cache_uncached", ctypes.c_uint64),
                ("jit_kernels", ctypes.c_uint64), ("jit_failed", ctypes.c_uint64), ("jit_pending", ctypes.c_uint64),
                ("jit_compile_ms", ctypes.c_uint64), ("jit_launches", ctypes.c_uint64)]


_lib = None
u8p = ctypes.POINTER(ctypes.c_uint8)
vp = ctypes.c_void_p
i64 = ctypes.c_int64
u32 = ctypes.c_uint32
u64 = ctypes.c_uint64


def lib():
    """Load libmec.so (raises if it is missing: no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MecError(MEC_ENODEV, "libmec.so not built at %s (run make -C memec_amd)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    L.mec_last_error.restype = ctypes.c_char_p
    L.mec_create.argtypes = [ctypes.c_int, u32, u32, u32, ctypes.c_int, ctypes.POINTER(vp)]
    L.mec_create_multi.argtypes = [ctypes.c_int, u32, u32, u32, ctypes.POINTER(ctypes.c_int), u32,
                                   ctypes.POINTER(vp)]
    L.mec_destroy.argtypes = [vp]
    L.mec_destroy.restype = None
    L.mec_get_info.argtypes = [vp, ctypes.POINTER(MecInfo)]
    L.mec_get_matrix.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), ctypes.c_size_t]
    L.mec_get_bitmatrix.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), ctypes.c_size_t]
    L.mec_encode.argtypes = [vp, vp, i64, i64, vp, i64, i64, u32, u32, vp]
    L.mec_decode.argtypes = [vp, vp, i64, i64, u32, u64, vp]
    L.mec_decode_split.argtypes = [vp, vp, i64, i64, vp, i64, i64, u32, u64, vp]
    L.mec_encode_update.argtypes = [vp, u32, vp, i64, vp, i64, i64, u32, u32, vp]
    L.mec_xor.argtypes = [vp, vp, vp, u64, vp]
    L.mec_fill_random.argtypes = [vp, u64, u64, u64, vp]
    L.mec_encode_host.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mec_decode_host.argtypes = [vp, ctypes.POINTER(vp), u64]
    L.mec_encode_update_host.argtypes = [vp, u32, vp, ctypes.POINTER(vp)]
    L.mec_encode_host_batch.argtypes = [vp, vp, vp, u32, u32]
    L.mec_host_register.argtypes = [vp, ctypes.c_size_t]
    L.mec_host_unregister.argtypes = [vp]
    pvp = ctypes.POINTER(vp)
    L.mec_encode_batch.argtypes = [vp, pvp, pvp, u32, u32, ctypes.c_int, vp]
    L.mec_decode_batch.argtypes = [vp, pvp, ctypes.POINTER(u64), u32, ctypes.POINTER(ctypes.c_int32),
                                   ctypes.c_int, vp]
    L.mec_encode_update_batch.argtypes = [vp, ctypes.POINTER(u32), pvp, pvp, u32, u32, ctypes.c_int, vp]
    pu32 = ctypes.POINTER(u32)
    L.mec_encode_batch32.argtypes = [vp, vp, u32, pu32, pu32, u32, u32, vp]
    L.mec_decode_batch32.argtypes = [vp, vp, u32, pu32, ctypes.POINTER(u64), u32, ctypes.POINTER(ctypes.c_int32), vp]
    L.mec_encode_update_batch32.argtypes = [vp, vp, u32, pu32, pu32, pu32, u32, u32, vp]
    L.mec_set_coalescing.argtypes = [vp, u32]
    L.mec_set_host_queue.argtypes = [vp, u32]
    L.mec_get_stats.argtypes = [vp, ctypes.POINTER(MecStats)]
    L.mec_set_probe.argtypes = [vp, ctypes.c_int]
    L.mec_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    _lib = L
    return L


def set_knob(name, value):
    """Change a launch-shape experiment knob at run time (mec_set_knob):
    name = the environment variable's name, value = its string syntax, None =
    back to the built-in rule."""
    check(lib().mec_set_knob(name.encode(), None if value is None else str(value).encode()))


def check(rc):
    if rc < 0:
        raise MecError(rc, lib().mec_last_error().decode(errors="replace"))
    return rc

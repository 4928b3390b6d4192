"""MemEC's own coding plugin, compiled from the reference sources into
oracle/_ref/ (oracle/Makefile `ref`), driven through ctypes — test
infrastructure only, the checker the random-shape sweeps compare against.

* Jerasure RS / Cauchy: `libmemec_ref.so` (oracle/ref_shim.cc) —
  `Coding::instantiate` (common/coding/coding.cc:12-54), `Coding::encode`
  one parity index per call (rscoding.cc:51-95, cauchycoding.cc:49-85) and
  `Coding::decode` in place (rscoding.cc:97-187, cauchycoding.cc:87-180).
* ISA-L RS / Cauchy: `libmemec_ref_isal.so` (oracle/ref_isal_plugin.cc), the
  same plugin built -DUSE_ISAL over ISA-L's ec_base.c (rscoding.cc:81-89,
  155-177).  Its decode of an erased PARITY chunk reads past the k x k
  inverse (rscoding.cc:173-175), so `decode` reports, for each
  erased parity chunk, the plugin's own encode of the decoded data instead
  (the engine's documented fix); erased data chunks are the plugin's bytes.

`available()` is False where oracle/_ref was not built (a fresh checkout):
tests that need it skip.  Each call instantiates, uses and destroys the
plugin (ChunkUtil's chunk size is process-global in the reference)."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libmemec_ref.so")
REFI_SO = os.path.join(ROOT, "oracle", "_ref", "libmemec_ref_isal.so")
CS_RS, CS_CAUCHY = 4, 7  # CodingScheme (coding_scheme.hh:4-13)
SCHEME = {"rs": CS_RS, "cauchy": CS_CAUCHY, "isal_rs": CS_RS, "isal_cauchy": CS_CAUCHY}

_libs = {}


def available():
    return os.path.exists(REF_SO) and os.path.exists(REFI_SO)


def _lib(fam):
    isal = fam.startswith("isal")
    key = "isal" if isal else "jer"
    if key in _libs:
        return _libs[key]
    vp, u32, u8p = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p
    L = ctypes.CDLL(REFI_SO if isal else REF_SO)
    pre = "refi_" if isal else "ref_"
    getattr(L, pre + "instantiate").restype = vp
    getattr(L, pre + "instantiate").argtypes = [ctypes.c_int, u32, u32, u32]
    getattr(L, pre + "destroy").argtypes = [vp]
    if isal:
        L.refi_encode.argtypes = [vp, u8p, u32, u8p, u32, u32, u32]
        L.refi_decode_poisoned.restype = ctypes.c_int
        L.refi_decode_poisoned.argtypes = [vp, u8p, ctypes.c_uint64, ctypes.c_uint8]
    else:
        L.ref_encode.argtypes = [vp, u8p, u32, u32, u8p]
        L.ref_decode.restype = ctypes.c_int
        L.ref_decode.argtypes = [vp, u8p, ctypes.c_uint64]
    _libs[key] = L
    return L


def _p(a):
    assert a.flags["C_CONTIGUOUS"] and a.dtype == np.uint8
    return ctypes.c_void_p(a.ctypes.data)


class _Handle:
    def __init__(self, fam, k, m, cs):
        self.fam, self.k, self.m, self.cs = fam, k, m, cs
        self.isal = fam.startswith("isal")
        self.L = _lib(fam)
        pre = "refi_" if self.isal else "ref_"
        self.h = ctypes.c_void_p(getattr(self.L, pre + "instantiate")(SCHEME[fam], k, m, cs))
        assert self.h.value, (fam, k, m, cs)
        self._destroy = getattr(self.L, pre + "destroy")

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self._destroy(self.h)

    def encode_one(self, data, index):
        """Parity `index` (1-based) of k dense data chunks."""
        out = np.zeros(self.cs, np.uint8)
        if self.isal:
            self.L.refi_encode(self.h, _p(data), 0, _p(out), index, 0, 0)
        else:
            self.L.ref_encode(self.h, _p(data), 0, index, _p(out))
        return out


def encode(fam, k, m, cs, data):
    """data: [k][cs] uint8 -> [m][cs], one Coding::encode call per parity
    (test/common/coding/coding.cc:150-152)."""
    d = np.ascontiguousarray(data, dtype=np.uint8).reshape(k * cs)
    with _Handle(fam, k, m, cs) as h:
        return np.stack([h.encode_one(d, i + 1) for i in range(m)])


def decode(fam, k, m, cs, chunks, erased):
    """chunks: [k+m][cs] (any contents, codeword or not); the erased chunks
    are cleared and rebuilt in place as Coding::decode does.  Returns (ok,
    out [k+m][cs]); ok False where the plugin's decode returns false (more
    than m erased, or ISA-L's singular survivor matrices)."""
    work = np.ascontiguousarray(chunks, dtype=np.uint8).reshape(k + m, cs).copy()
    for e in erased:
        work[e] = 0
    present = sum(1 << i for i in range(k + m) if i not in erased)
    with _Handle(fam, k, m, cs) as h:
        flat = work.reshape(-1)
        if h.isal:
            rc = h.L.refi_decode_poisoned(h.h, _p(flat), ctypes.c_uint64(present), 0xA5)
        else:
            rc = h.L.ref_decode(h.h, _p(flat), ctypes.c_uint64(present))
        if rc != 0:
            return False, None
        if h.isal:  # erased parity: the plugin's encode of the decoded data
            d = np.ascontiguousarray(work[:k]).reshape(-1)
            for e in erased:
                if e >= k:
                    work[e] = h.encode_one(d, e - k + 1)
    return True, work

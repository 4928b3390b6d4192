"""ctypes view of oracle/build/liboracle.so — the CPU restatement (checker).

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.
"""
import ctypes
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")

u8p = ctypes.POINTER(ctypes.c_uint8)
ip = ctypes.POINTER(ctypes.c_int)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(ORACLE_SO)
        L.orc_fill_splitmix.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_rs_encode.argtypes = [ctypes.c_int, ctypes.c_int, ip, ctypes.POINTER(u8p),
                                    ctypes.POINTER(u8p), ctypes.c_size_t]
        L.orc_rs_decode.argtypes = [ctypes.c_int, ctypes.c_int, ip, ip, ctypes.POINTER(u8p),
                                    ctypes.POINTER(u8p), ctypes.c_size_t]
        L.orc_crs_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ip, ctypes.c_int,
                                     ctypes.POINTER(u8p), ctypes.POINTER(u8p), ctypes.c_size_t,
                                     ctypes.c_size_t]
        L.orc_crs_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ip, ip,
                                     ctypes.POINTER(u8p), ctypes.POINTER(u8p), ctypes.c_size_t,
                                     ctypes.c_size_t]
        L.orc_isal_decode.argtypes = [ctypes.c_int, ctypes.c_int, u8p, ip, ctypes.POINTER(u8p),
                                      ctypes.c_size_t]
        L.orc_isal_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p,
                                      ctypes.POINTER(u8p), ctypes.POINTER(u8p)]
        L.orc_isal_encode_update.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             u8p, u8p, ctypes.POINTER(u8p)]
        L.orc_encode_batch_mt.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                          u8p, u8p, ctypes.c_uint32, ctypes.c_int]
        L.orc_decode_batch_mt.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                          u8p, ctypes.c_uint32, ip, ctypes.c_int]
        _lib = L
    return _lib


def ptr(a):
    return a.ctypes.data_as(u8p)


def fill(n, seed, word_offset=0):
    buf = np.empty(n, dtype=np.uint8)
    lib().orc_fill_splitmix(ptr(buf), n, seed, word_offset)
    return buf


def rs_getw(k, m, cs):
    return lib().orc_rs_getw(k, m, cs)


def cauchy_getw(k, m, cs):
    return lib().orc_cauchy_getw(k, m, cs)


def rs_matrix(k, m):
    out = (ctypes.c_int * (k * m))()
    assert lib().orc_rs_vandermonde_matrix(k, m, 8, out) == 0
    return list(out)


def cauchy_matrix(k, m, w):
    out = (ctypes.c_int * (k * m))()
    if lib().orc_cauchy_good_matrix(k, m, w, out) != 0:
        return None
    return list(out)


def bitmatrix(k, m, w, matrix):
    mat = (ctypes.c_int * (k * m))(*matrix)
    out = (ctypes.c_int * (k * m * w * w))()
    lib().orc_matrix_to_bitmatrix(k, m, w, mat, out)
    return list(out)


def smart_schedule(k, m, w, bm):
    b = (ctypes.c_int * len(bm))(*bm)
    mx = k * m * w * w + 1
    ops = (ctypes.c_int * (5 * mx))()
    n = lib().orc_smart_schedule(k, m, w, b, ops, mx)
    return list(ops)[:5 * n], n


def _ptrs(arrs):
    return (u8p * len(arrs))(*[ptr(a) for a in arrs])


def rs_encode(k, m, data_chunks, cs):
    """data_chunks: list of k uint8 arrays -> list of m parity arrays."""
    mat = (ctypes.c_int * (k * m))(*rs_matrix(k, m))
    par = [np.zeros(cs, np.uint8) for _ in range(m)]
    lib().orc_rs_encode(k, m, mat, _ptrs(data_chunks), _ptrs(par), cs)
    return par


def crs_encode(k, m, data_chunks, cs):
    w = cauchy_getw(k, m, cs)
    mat = cauchy_matrix(k, m, w)
    bm = bitmatrix(k, m, w, mat)
    ops, n = smart_schedule(k, m, w, bm)
    par = [np.zeros(cs, np.uint8) for _ in range(m)]
    o = (ctypes.c_int * len(ops))(*ops)
    lib().orc_crs_encode(k, m, w, o, n, _ptrs(data_chunks), _ptrs(par), cs, cs // w)
    return par


def encode(family, k, m, data_chunks, cs):
    if family == "rs":
        return rs_encode(k, m, data_chunks, cs)
    if family == "cauchy":
        return crs_encode(k, m, data_chunks, cs)
    enc = isal_matrix(family, k, m)
    par = [np.zeros(cs, np.uint8) for _ in range(m)]
    coef = np.ascontiguousarray(enc[k * k:])
    lib().orc_isal_encode(cs, k, m, ptr(coef), _ptrs(data_chunks), _ptrs(par))
    return par


def isal_matrix(family, k, m):
    a = np.zeros((k + m) * k, np.uint8)
    if family == "isal_rs":
        lib().orc_isal_gen_rs_matrix(ptr(a), k + m, k)
    else:
        lib().orc_isal_gen_cauchy1_matrix(ptr(a), k + m, k)
    return a


def decode(family, k, m, chunks, erased, cs):
    """chunks: list of k+m arrays (modified in place; erased ones are outputs)."""
    er = (ctypes.c_int * (k + m))(*[1 if i in erased else 0 for i in range(k + m)])
    for e in erased:
        chunks[e][:] = 0
    if family == "rs":
        mat = (ctypes.c_int * (k * m))(*rs_matrix(k, m))
        return lib().orc_rs_decode(k, m, mat, er, _ptrs(chunks[:k]), _ptrs(chunks[k:]), cs)
    if family == "cauchy":
        w = cauchy_getw(k, m, cs)
        bm = bitmatrix(k, m, w, cauchy_matrix(k, m, w))
        b = (ctypes.c_int * len(bm))(*bm)
        return lib().orc_crs_decode(k, m, w, b, er, _ptrs(chunks[:k]), _ptrs(chunks[k:]), cs, cs // w)
    enc = isal_matrix(family, k, m)
    return lib().orc_isal_decode(k, m, ptr(enc), er, _ptrs(chunks), cs)


def encode_batch_mt(family, k, m, cs, data, parity, n_stripes, threads):
    fam = 0 if family == "rs" else 1
    return lib().orc_encode_batch_mt(fam, k, m, cs, ptr(data), ptr(parity), n_stripes, threads)


def decode_batch_mt(family, k, m, cs, chunks, n_stripes, erased, threads):
    """In-place decode of dense [s][k+m][cs] stripes, one erasure pattern."""
    fam = 0 if family == "rs" else 1
    er = (ctypes.c_int * (k + m))(*[1 if i in erased else 0 for i in range(k + m)])
    return lib().orc_decode_batch_mt(fam, k, m, cs, ptr(chunks), n_stripes, er, threads)


_golden = None


def golden():
    global _golden
    if _golden is None:
        with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
            meta = json.load(f)
        npz = np.load(os.path.join(GOLDEN_DIR, "golden.npz"), allow_pickle=False)
        blobs = {k.replace("|", "/"): npz[k] for k in npz.files}
        _golden = (meta, blobs)
    return _golden

#!/usr/bin/env python3
"""Time the oracle restatement against the compiled reference, side by side,
single thread, same stripes (build container only: needs oracle/_ref).

The reference's Coding::encode computes all m parities per call
(jerasure_matrix_encode, rscoding.cc:91) and returns one; one call per stripe
is therefore one full-stripe encode, the same work as orc_rs_encode /
orc_crs_encode.  Reported as data GiB/s (k * chunk per stripe)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _oracle as O  # noqa: E402

REF = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libmemec_ref.so"))
u8p = ctypes.POINTER(ctypes.c_uint8)
REF.ref_instantiate.restype = ctypes.c_void_p
REF.ref_instantiate.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
REF.ref_encode.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint32, ctypes.c_uint32, u8p]
REF.ref_destroy.argtypes = [ctypes.c_void_p]
REF.ref_alloc_chunks.restype = ctypes.c_void_p
REF.ref_alloc_chunks.argtypes = [ctypes.c_uint32]
REF.ref_chunk_data.restype = ctypes.c_void_p
REF.ref_chunk_data.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
REF.ref_encode_chunks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]


def run(fam, k, m, cs, n, reps=3):
    data = O.fill(n * k * cs, 99)
    scheme = 4 if fam == "rs" else 7
    h = ctypes.c_void_p(REF.ref_instantiate(scheme, k, m, cs))
    chunks = REF.ref_alloc_chunks(n * (k + m))
    for s in range(n):
        for j in range(k):
            ctypes.memmove(REF.ref_chunk_data(chunks, s * (k + m) + j), O.ptr(data[(s * k + j) * cs:]), cs)
    best_ref = best_orc = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        for s in range(n):
            REF.ref_encode_chunks(h, chunks, s * (k + m), 1)
        best_ref = min(best_ref, time.perf_counter() - t0)
        par = np.zeros(n * m * cs, np.uint8)
        t0 = time.perf_counter()
        O.encode_batch_mt(fam, k, m, cs, data, par, n, 1)
        best_orc = min(best_orc, time.perf_counter() - t0)
    REF.ref_destroy(h)
    gib = n * k * cs / 2**30
    return gib / best_ref, gib / best_orc


if __name__ == "__main__":
    print("config, reference GiB/s, oracle GiB/s, oracle/reference")
    for fam, k, m, cs, n in [("rs", 4, 2, 4096, 20000), ("rs", 8, 2, 4096, 10000), ("rs", 10, 4, 1 << 20, 24),
                             ("cauchy", 12, 4, 65536, 400)]:
        r, o = run(fam, k, m, cs, n)
        print("%s(%d,%d)@%d, %.3f, %.3f, %.3f" % (fam, k, m, cs, r, o, o / r))

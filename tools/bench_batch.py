#!/usr/bin/env python3
"""Throughput of the pointer-array batch ABI and the coalescer (one GPU).

  device gather vs strided : same stripes, chunk pointers from a device table
                             vs base + stride (RS(10,4)@1MiB, RS(8,2)@4KiB
                             scattered over ChunkPool-like 8+cs slots)
  decode_batch             : mixed erasure patterns per stripe
  host batch               : mec_encode_batch on host memory (PCIe-inclusive)
  coalescer                : T threads issuing single-stripe mec_encode_host
                             calls, with and without coalescing

Prints one JSON object per measurement.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from memec_amd import Codec, fill_random, host_register, host_unregister  # noqa: E402


def timed(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def gib(x):
    return x / 2**30


def emit(**kw):
    print(json.dumps(kw), flush=True)


def device_gather(fam, k, m, cs, n, hdr, reps):
    c = Codec(fam, k, m, cs)
    slot = cs + hdr
    slab = torch.empty(n * (k + m) * slot, dtype=torch.uint8, device="cuda")
    fill_random(slab, 1)
    perm = np.random.default_rng(0).permutation(n * (k + m))
    base = slab.data_ptr()
    rows = perm.reshape(n, k + m).astype(np.uint64) * np.uint64(slot) + np.uint64(base + hdr)
    dptr = np.ascontiguousarray(rows[:, :k]).reshape(-1)
    pptr = np.ascontiguousarray(rows[:, k:]).reshape(-1)
    t_g = timed(lambda: c.encode_batch(dptr, pptr), reps)
    data = torch.empty(n, k, cs, dtype=torch.uint8, device="cuda")
    fill_random(data, 2)
    par = torch.empty(n, m, cs, dtype=torch.uint8, device="cuda")
    t_s = timed(lambda: c.encode(data, par), reps)
    alg = n * (k + m) * cs
    emit(test="device_gather_encode", family=fam, k=k, m=m, chunk=cs, stripes=n, slot_header=hdr,
         gather_ms=round(t_g * 1e3, 4), strided_ms=round(t_s * 1e3, 4),
         gather_GBps=round(alg / t_g / 1e9, 1), strided_GBps=round(alg / t_s / 1e9, 1),
         note="gather time includes host-side grouping + pointer-table upload")
    del slab, data, par


def decode_mixed(fam, k, m, cs, n, n_patterns, reps):
    c = Codec(fam, k, m, cs)
    stripe = torch.empty(n, k + m, cs, dtype=torch.uint8, device="cuda")
    fill_random(stripe, 3)
    rng = np.random.default_rng(1)
    pats = [sorted(rng.choice(k + m, size=m, replace=False).tolist()) for _ in range(n_patterns)]
    masks = [sum(1 << i for i in range(k + m) if i not in pats[s % n_patterns]) for s in range(n)]
    base = stripe.data_ptr()
    ptrs = np.uint64(base) + np.arange(n * (k + m), dtype=np.uint64) * np.uint64(cs)
    masks = np.asarray(masks, dtype=np.uint64)
    t = timed(lambda: c.decode_batch(ptrs, masks, as_array=True), reps)
    alg = n * (k + m) * cs
    emit(test="decode_batch_mixed", family=fam, k=k, m=m, chunk=cs, stripes=n, patterns=n_patterns,
         ms=round(t * 1e3, 4), GBps=round(alg / t / 1e9, 1), data_GiBps=round(gib(n * k * cs) / t, 1))
    del stripe


def aligned(nbytes, align=4096):
    raw = np.empty(nbytes + align, np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


def host_batch(fam, k, m, cs, n, reps, registered=False):
    c = Codec(fam, k, m, cs)
    slot = cs + 8
    slab = aligned(n * (k + m) * slot)
    slab[:] = np.random.default_rng(0).integers(0, 256, slab.size, dtype=np.uint8)
    if registered:
        host_register(slab)
    base = slab.ctypes.data
    rows = np.arange(n * (k + m), dtype=np.uint64).reshape(n, k + m) * np.uint64(slot) + np.uint64(base + 8)
    dptr = np.ascontiguousarray(rows[:, :k]).reshape(-1)
    pptr = np.ascontiguousarray(rows[:, k:]).reshape(-1)
    t = timed(lambda: c.encode_batch(dptr, pptr, mem="host"), reps, warm=1)
    st = c.stats()
    if registered:
        host_unregister(slab)
    emit(test="host_encode_batch", family=fam, k=k, m=m, chunk=cs, stripes=n,
         memory="registered (zero-copy)" if registered else "pageable",
         ms=round(t * 1e3, 3), data_GiBps=round(gib(n * k * cs) / t, 2),
         zero_copy_calls=st["zero_copy_calls"], staged_calls=st["staged_calls"])


def coalescer(fam, k, m, cs, threads, per_thread, max_batch, registered=False):
    """T threads issuing single-stripe mec_encode_host calls on their own
    k + m chunks (slots of 8 + cs bytes in one slab, as ChunkPool)."""
    import ctypes
    from memec_amd._lib import lib
    c = Codec(fam, k, m, cs)
    if max_batch:
        c.set_coalescing(max_batch)
    slot = cs + 8
    slab = aligned(threads * (k + m) * slot)
    slab[:] = np.random.default_rng(1).integers(0, 256, slab.size, dtype=np.uint8)
    if registered:
        host_register(slab)
    vp = ctypes.c_void_p
    base = slab.ctypes.data
    arrs = []
    for t in range(threads):
        a = [base + (t * (k + m) + i) * slot + 8 for i in range(k + m)]
        arrs.append(((vp * k)(*[vp(x) for x in a[:k]]), (vp * m)(*[vp(x) for x in a[k:]])))
    L = lib()

    def worker(t):
        dp, pp = arrs[t]
        for _ in range(per_thread):
            L.mec_encode_host(c._h, dp, pp)

    def run():
        th = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        for x in th:
            x.start()
        for x in th:
            x.join()

    run()  # warm
    t0 = time.perf_counter()
    run()
    dt = time.perf_counter() - t0
    st = c.stats()
    if registered:
        host_unregister(slab)
    n = threads * per_thread
    emit(test="coalescer_encode_host", family=fam, k=k, m=m, chunk=cs, threads=threads, calls=n,
         max_batch=max_batch, memory="registered (zero-copy)" if registered else "pageable",
         calls_per_s=round(n / dt, 1), data_GiBps=round(gib(n * k * cs) / dt, 3),
         mean_batch=round(st["coalesced_requests"] / st["coalesced_batches"], 2) if st["coalesced_batches"] else 1,
         zero_copy_calls=st["zero_copy_calls"], staged_calls=st["staged_calls"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="", help="comma list of test names to run")
    a = ap.parse_args()
    reps = 3 if a.quick else 10
    torch.cuda.set_device(0)
    tests = [
        ("gather_rs1m_h8", lambda: device_gather("rs", 10, 4, 1 << 20, 1024, 8, reps)),
        ("gather_rs1m_h256", lambda: device_gather("rs", 10, 4, 1 << 20, 1024, 256, reps)),
        ("gather_rs4k_h8", lambda: device_gather("rs", 8, 2, 4096, 65536, 8, reps)),
        ("gather_rs4k_h256", lambda: device_gather("rs", 8, 2, 4096, 65536, 256, reps)),
        ("gather_crs64k_h8", lambda: device_gather("cauchy", 12, 4, 65536, 4096, 8, reps)),
    ]
    tests += [("decode_mixed_%d" % n, (lambda n=n: decode_mixed("rs", 10, 4, 65536, 4096, n, reps)))
              for n in (1, 4, 14, 64)]
    # MemEC's default chunk (bin/config: chunk=4096): reconstruction batches of 4 KiB stripes
    tests += [("decode_mixed4k_%d" % n, (lambda n=n: decode_mixed("rs", 10, 4, 4096, 65536, n, reps)))
              for n in (1, 4, 14, 64)]
    tests += [
        ("decode_mixed_crs", lambda: decode_mixed("cauchy", 12, 4, 65536, 4096, 4, reps)),
        ("host_rs4k", lambda: host_batch("rs", 8, 2, 4096, 16384, reps)),
        ("host_rs1m", lambda: host_batch("rs", 10, 4, 1 << 20, 64, reps)),
        ("host_rs4k_reg", lambda: host_batch("rs", 8, 2, 4096, 16384, reps, True)),
        ("host_rs1m_reg", lambda: host_batch("rs", 10, 4, 1 << 20, 64, reps, True)),
        ("host_crs64k", lambda: host_batch("cauchy", 12, 4, 65536, 1024, reps)),
        ("host_crs64k_reg", lambda: host_batch("cauchy", 12, 4, 65536, 1024, reps, True)),
        ("coalesce_off", lambda: coalescer("rs", 8, 2, 4096, 16, 200, 0)),
        ("coalesce_on", lambda: coalescer("rs", 8, 2, 4096, 16, 200, 256)),
        ("coalesce_off_reg", lambda: coalescer("rs", 8, 2, 4096, 16, 200, 0, True)),
        ("coalesce_on_reg", lambda: coalescer("rs", 8, 2, 4096, 16, 200, 256, True)),
    ]
    only = set(x for x in a.only.split(",") if x)
    for name, fn in tests:
        if not only or name in only:
            fn()


if __name__ == "__main__":
    main()

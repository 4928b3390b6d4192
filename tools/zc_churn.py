#!/usr/bin/env python3
"""The zero-copy single-stripe test's sequence (tests/test_gpu_zerocopy.py
test_zc_single_stripe_calls), repeated on a FRESH slab every iteration —
allocated, registered, coded, unregistered and freed, so host virtual
addresses and pages are reused from one iteration to the next as they were
across the full suite's 328 earlier tests — optionally with other GPU work
running beside it.  Every output is checked after every call and a mismatch
is reported with its map (tests/_mismatch.py): byte ranges, pages, 1 KiB
tiles, and whether the wrong bytes are the pre-call contents.

  python tools/zc_churn.py [--iters N] [--fam rs] [--cs 65536] [--bg none|launch|queue|regchurn|all]

VERDICT r05 item 1 (profiles/r05/parity/pytest_gpu_r05a_zc_mismatch.log).
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import _oracle as O  # noqa: E402
from _mismatch import mismatch_map  # noqa: E402
from memec_amd import Codec, host_register, host_unregister  # noqa: E402


def aligned(nbytes, align=4096):
    raw = np.empty(nbytes + align, np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


def bg_launch(stop, errs):
    """Device-resident RS(10,4)@1 MiB encodes back to back (other streams,
    every CU busy, L2 churned)."""
    import torch
    c = Codec("rs", 10, 4, 1 << 20)
    d = torch.randint(0, 256, (64, 10, 1 << 20), dtype=torch.uint8, device="cuda:0")
    p = torch.empty(64, 4, 1 << 20, dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.Stream()
    n = 0
    with torch.cuda.stream(s):
        while not stop.is_set():
            c.encode(d, p)
            n += 1
            if n % 8 == 0:
                s.synchronize()
    s.synchronize()
    c.close()
    return n


def bg_queue(stop, errs):
    """Another context's resident queue serving single-stripe seals on its
    own registered slab (a resident grid polling host memory beside us), in
    bursts of 400 calls with 120 ms pauses: the grid then idles out between
    bursts (MEC_QUEUE_IDLE_MS, 50 ms), which the main loop's
    hipHostRegister / hipHostUnregister wait for — the runtime appears not
    to register or unregister host memory while a kernel is resident (a queue
    kept busy without pause held the main loop's registration for minutes,
    profiles/r06/parity/zc_churn_r06d_queue_busy.log)."""
    k, m, cs = 8, 2, 4096
    buf = aligned((k + m) * (cs + 8))
    buf[:] = np.random.default_rng(5).integers(0, 256, buf.size, dtype=np.uint8)
    host_register(buf)
    c = Codec("rs", k, m, cs)
    c.set_host_queue(4)
    view = [buf[i * (cs + 8) + 8:i * (cs + 8) + 8 + cs] for i in range(k + m)]
    want = O.encode("rs", k, m, [view[j].copy() for j in range(k)], cs)
    n = 0
    while not stop.is_set():
        for _ in range(400):
            view[k][:] = 0
            got = c.encode_host([view[j] for j in range(k)])
            if not np.array_equal(got[0], want[0]):
                errs.append("bg queue staged encode wrong")
            n += 1
        time.sleep(0.12)
    c.close()
    host_unregister(buf)
    return n


def bg_regchurn(stop, errs):
    """Register / unregister / free other buffers continuously."""
    n = 0
    rng = np.random.default_rng(9)
    while not stop.is_set():
        b = aligned(int(rng.integers(1, 64)) * 4096 + int(rng.integers(0, 4096)))
        host_register(b)
        b[:16] = 1
        host_unregister(b)
        del b
        n += 1
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--fam", default="rs")
    ap.add_argument("--cs", type=int, default=65536)
    ap.add_argument("--bg", default="none")
    a = ap.parse_args()
    k, m, cs = 10, 4, a.cs
    if a.fam == "cauchy" and O.cauchy_getw(k, m, cs) <= 0:
        cs = 4096
    slot = cs + 8
    stop, errs, counts = threading.Event(), [], {}
    kinds = ["launch", "queue", "regchurn"] if a.bg == "all" else ([] if a.bg == "none" else a.bg.split(","))
    if "launch" in kinds:  # torch's device init before libmec's, as in the test suite
        import torch
        torch.cuda.set_device(0)
    fns = {"launch": bg_launch, "queue": bg_queue, "regchurn": bg_regchurn}
    threads = []
    for kd in kinds:
        def run(kd=kd):
            try:
                counts[kd] = fns[kd](stop, errs)
            except Exception as e:  # noqa: BLE001
                errs.append("bg %s: %r" % (kd, e))
        t = threading.Thread(target=run)
        t.start()
        threads.append(t)
    c = Codec(a.fam, k, m, cs)
    rng = np.random.default_rng(1)
    reg_ms = []
    bad, first, addrs = [], None, set()
    t0 = time.time()
    pat = [0, 3, 10, 13]
    for it in range(a.iters):
        buf = aligned((k + m + 1) * slot)
        buf[:] = rng.integers(0, 256, buf.size, dtype=np.uint8)
        addrs.add(buf.ctypes.data)
        t_r = time.perf_counter()
        host_register(buf)
        reg_ms.append((time.perf_counter() - t_r) * 1e3)
        try:
            view = [buf[i * slot + 8:i * slot + 8 + cs] for i in range(k + m + 1)]
            want = O.encode(a.fam, k, m, [view[j].copy() for j in range(k)], cs)
            for i in range(m):
                view[k + i][:] = 0
            pre = [view[k + i].copy() for i in range(m)]
            c.encode_batch([buf.ctypes.data + j * slot + 8 for j in range(k)],
                           [buf.ctypes.data + (k + i) * slot + 8 for i in range(m)], mem="host")
            checks = [("encode", k + i, view[k + i], want[i], pre[i]) for i in range(m)]
            orig = [v.copy() for v in view[:k + m]]
            for e in pat:
                view[e][:] = 0
            pre_d = [v.copy() for v in view[:k + m]]
            c.decode_host(view[:k + m], sum(1 << i for i in range(k + m) if i not in pat))
            checks += [("decode", i, view[i], orig[i], pre_d[i]) for i in range(k + m)]
            for what, i, g, w, p in checks:
                if not np.array_equal(g, w):
                    rep = {"iter": it, "call": what, "chunk": i,
                           "map": mismatch_map(g, w, p, buf.ctypes.data + i * slot + 8)}
                    bad.append(rep)
                    print(json.dumps(rep), flush=True)
        finally:
            t_r = time.perf_counter()
            host_unregister(buf)
            reg_ms.append((time.perf_counter() - t_r) * 1e3)
        del buf
        if it % 50 == 0:
            print("iter %d %.1fs bad %d" % (it, time.time() - t0, len(bad)), flush=True)
    stop.set()
    for t in threads:
        t.join()
    st = c.stats()
    c.close()
    print(json.dumps({"fam": a.fam, "cs": cs, "iters": a.iters, "bg": a.bg, "bad_calls": len(bad),
                      "distinct_slab_addrs": len(addrs), "bg_counts": counts, "bg_errors": errs[:5],
                      "register_unregister_ms": {"median": round(float(np.median(reg_ms)), 3),
                                                 "max": round(float(np.max(reg_ms)), 3)},
                      "zero_copy_calls": st["zero_copy_calls"], "staged_calls": st["staged_calls"],
                      "seconds": round(time.time() - t0, 1)}), flush=True)
    return 1 if bad or errs else 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Zero-copy single-stripe decode on a registered ChunkPool-like slab,
repeated: every call's rebuilt chunks are compared with the originals right
after mec_decode_host returns, and a mismatch is classified (bytes still
zero = the GPU's stores to host memory not yet visible; other bytes =
wrong data).  Round-5 investigation of one mismatch in the full GPU suite
(profiles/r05/parity/pytest_gpu_r05a_zc_mismatch.log).

  python tools/zc_stress.py [--iters N] [--fam rs] [--cs 65536] [--queue SLOTS]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import _oracle as O  # noqa: E402
from memec_amd import Codec, host_register, host_unregister  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--fam", default="rs")
    ap.add_argument("--cs", type=int, default=65536)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--queue", type=int, default=0, help="resident queue slots (0: per-call launches, as the test)")
    a = ap.parse_args()
    k, m, cs = a.k, a.m, a.cs
    slot = cs + 8
    raw = np.empty((k + m) * slot + 4096, np.uint8)
    off = (-raw.ctypes.data) % 4096
    buf = raw[off:off + (k + m) * slot]
    buf[:] = O.fill(buf.nbytes, 9)
    host_register(buf)
    view = [buf[i * slot + 8:i * slot + 8 + cs] for i in range(k + m)]
    c = Codec(a.fam, k, m, cs)
    if a.queue:
        c.set_host_queue(a.queue)
    data = [view[j] for j in range(k)]
    par = O.encode(a.fam, k, m, [d.copy() for d in data], cs)
    for i in range(m):
        view[k + i][:] = par[i]
    orig = [v.copy() for v in view]
    pats = [[0, 3, 10, 13], [1, 2], [0], [4, 5, 6, 7], [k + m - 1]]
    bad = {"zero_bytes": 0, "wrong_bytes": 0, "calls_bad": 0}
    first = None
    for it in range(a.iters):
        pat = pats[it % len(pats)]
        for e in pat:
            view[e][:] = 0
        c.decode_host(view, sum(1 << i for i in range(k + m) if i not in pat))
        for e in pat:
            if not np.array_equal(view[e], orig[e]):
                diff = np.nonzero(view[e] != orig[e])[0]
                z = int((view[e][diff] == 0).sum())
                bad["zero_bytes"] += z
                bad["wrong_bytes"] += len(diff) - z
                bad["calls_bad"] += 1
                if first is None:
                    first = {"iter": it, "chunk": e, "pat": pat, "first": int(diff[0]), "last": int(diff[-1]),
                             "n": len(diff), "zeros": z}
                view[e][:] = orig[e]
    st = c.stats()
    c.close()
    host_unregister(buf)
    print(json.dumps({"fam": a.fam, "k": k, "m": m, "cs": cs, "iters": a.iters, "queue": a.queue, **bad, "first": first,
                      "zero_copy_calls": st["zero_copy_calls"], "staged_calls": st["staged_calls"],
                      "queue_calls": st["queue_calls"]}), flush=True)


if __name__ == "__main__":
    main()

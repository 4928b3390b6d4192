#!/usr/bin/env python3
"""Soak of the resident submission queue (memec_amd/csrc/queue.hip) under
the server's calling pattern: T threads share one context, each owns one
stripe of a registered ChunkPool-like slab (slots of 8 + chunk bytes) and
loops over random single-stripe calls for D seconds —

  encode(index)  one parity row, checked against the oracle's parity;
  decode         1..m random erasures restored in place, checked against
                 the original chunks;
  update twice   the same delta XORed into every parity twice must leave
                 the parity unchanged;

with random pauses longer than the queue's idle timeout (MEC_QUEUE_IDLE_MS,
set low here) and a quiet window for every thread each 250 ms, so the grid
idles out and is relaunched by the next callers many times a second.
Every call's bytes are checked; one JSON line per (family, shape).
Not product code.

  SOAK_SECONDS=60 SOAK_THREADS=16 [SOAK_STAGED=1] python3 tools/queue_soak.py
"""
import json
import os
import random
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("MEC_QUEUE_IDLE_MS", "3")
os.environ.setdefault("MEC_QUEUE_MAX_CHUNK", str(1 << 20))  # multi-part slots too
import torch  # noqa: E402

import _oracle as O  # noqa: E402
from test_gpu_queue import Slab, encode_index  # noqa: E402

from memec_amd import Codec  # noqa: E402

SHAPES = [("rs", 8, 2, 4096), ("cauchy", 12, 4, 4096), ("rs", 10, 4, 16384), ("cauchy", 6, 3, 8192),
          ("rs", 10, 4, 65536), ("cauchy", 12, 4, 65536)]  # the last two: 4-part slots
if os.environ.get("SOAK_SHAPES"):  # fam:k:m:chunk,...
    SHAPES = [(f, int(k), int(m), int(c)) for f, k, m, c in (x.split(":") for x in os.environ["SOAK_SHAPES"].split(","))]


def soak(fam, k, m, cs, threads, seconds, slots):
    n = k + m + 1  # + one delta slot per stripe
    slab = Slab(threads * n, cs, 7 + k)
    staged = os.environ.get("SOAK_STAGED") == "1"
    if staged:  # unregistered chunks: calls are staged through mapped pinned lanes
        slab.close()
    c = Codec(fam, k, m, cs)
    c.set_host_queue(slots)
    wants, origs = [], []
    for t in range(threads):
        base = t * n
        data = [slab.view(base + j).copy() for j in range(k)]
        par = O.encode(fam, k, m, [d.copy() for d in data], cs)
        for i in range(m):
            slab.view(base + k + i)[:] = par[i]
        wants.append(par)
        origs.append([slab.view(base + i).copy() for i in range(k + m)])
    st0 = c.stats()
    errs, counts = [], [0] * threads
    stop = time.time() + seconds

    def worker(t):
        rng = random.Random(1000 + t)
        base = t * n
        try:
            while time.time() < stop and len(errs) < 10:
                op = rng.random()
                if op < 0.4:
                    i = rng.randrange(m)
                    slab.view(base + k + i)[:] = 0
                    encode_index(c, slab, k, [base + j for j in range(k)], base + k + i, i + 1)
                    if not np.array_equal(slab.view(base + k + i), wants[t][i]):
                        errs.append(("encode", t, i))
                elif op < 0.8:
                    er = sorted(rng.sample(range(k + m), rng.randint(1, m)))
                    for e in er:
                        slab.view(base + e)[:] = 0
                    c.decode_host([slab.view(base + i) for i in range(k + m)],
                                  sum(1 << i for i in range(k + m) if i not in er))
                    for e in er:
                        if not np.array_equal(slab.view(base + e), origs[t][e]):
                            errs.append(("decode", t, er, e))
                else:
                    j = rng.randrange(k)
                    delta = slab.view(base + k + m)
                    pars = [slab.view(base + k + i) for i in range(m)]
                    c.encode_update_host(j, delta, pars)
                    c.encode_update_host(j, delta, pars)
                    for i in range(m):
                        if not np.array_equal(pars[i], wants[t][i]):
                            errs.append(("update", t, j, i))
                counts[t] += 1
                if rng.random() < 0.01:  # a pause past the idle timeout
                    time.sleep(rng.uniform(0.005, 0.03))
                if time.time() % 0.25 < 0.02:  # every thread quiet together: the grid idles out
                    time.sleep(0.02)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    t0 = time.time()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.time() - t0
    st = c.stats()
    c.close()
    if not staged:
        slab.close()
    return {"family": fam, "k": k, "m": m, "chunk": cs, "threads": threads, "slots": slots, "staged": staged,
            "seconds": round(dt, 1), "calls": sum(counts), "calls_per_s": round(sum(counts) / dt),
            "queue_calls": st["queue_calls"] - st0["queue_calls"],
            "queue_launches": st["queue_launches"] - st0["queue_launches"],
            "errors": len(errs), "first_errors": [str(e) for e in errs[:3]]}


def main():
    torch.cuda.set_device(0)
    seconds = float(os.environ.get("SOAK_SECONDS", "20"))
    threads = int(os.environ.get("SOAK_THREADS", "16"))
    slots = int(os.environ.get("SOAK_SLOTS", "8"))
    bad = 0
    for fam, k, m, cs in SHAPES:
        r = soak(fam, k, m, cs, threads, seconds, slots)
        bad += r["errors"]
        print(json.dumps(r), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

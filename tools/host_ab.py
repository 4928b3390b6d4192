#!/usr/bin/env python3
"""Interleaved A/B of launch knobs on the host-memory (PCIe-inclusive)
batch paths: mec_encode_host_batch on registered (zero-copy) and pageable
(staged) buffers, and mec_encode_batch over registered ChunkPool-like slots,
for the BASELINE shapes.  The kernels there stream host memory across PCIe,
whose latency (~2 us a read) is not HBM's, so the HBM-tuned wave caps may
not be the right ones.  One JSON line per (shape, mode): GiB/s of data per
arm, arms alternated `--rounds` times, outputs compared across arms.

  python tools/host_ab.py [--arms unset,wpc0,wpc24] [--rounds 2] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import memec_amd  # noqa: E402
from memec_amd import Codec, host_register, host_unregister  # noqa: E402

ARMS = {"unset": {}, "wpc0": {"MEC_WPC": "0"}, "wpc8": {"MEC_WPC": "8"}, "wpc16": {"MEC_WPC": "16"},
        "wpc24": {"MEC_WPC": "24"}, "wpc32": {"MEC_WPC": "32"}, "blk64": {"MEC_BLOCK": "64"},
        "blk256": {"MEC_BLOCK": "256"}, "gw0": {"MEC_GWPC": "0"}, "gw24": {"MEC_GWPC": "24"},
        "gw32": {"MEC_GWPC": "32"}, "gblk64": {"MEC_GBLOCK": "64"}, "gblk256": {"MEC_GBLOCK": "256"},
        "ct4": {"MEC_COPY_THREADS": "4"}, "ct8": {"MEC_COPY_THREADS": "8"}, "ct12": {"MEC_COPY_THREADS": "12"},
        "ct16": {"MEC_COPY_THREADS": "16"}}
KNOBS = sorted({k for a in ARMS.values() for k in a})
SHAPES = [("rs", 10, 4, 1 << 20, 292), ("cauchy", 12, 4, 65536, 4096), ("rs", 8, 2, 4096, 65536)]


def aligned(nbytes, align=4096):
    raw = np.empty(nbytes + align, np.uint8)
    off = (-raw.ctypes.data) % align
    return raw[off:off + nbytes]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="unset,wpc0,wpc24")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="registered,pageable,slots,pslots")
    a = ap.parse_args()
    arms = a.arms.split(",")
    for fam, k, m, cs, n in SHAPES:
        c = Codec(fam, k, m, cs)
        d = aligned(n * k * cs).reshape(n, k, cs)
        d[:] = np.random.default_rng(1).integers(0, 256, d.size, dtype=np.uint8).reshape(d.shape)
        p = aligned(n * m * cs).reshape(n, m, cs)
        for mode in a.modes.split(","):
            if mode in ("registered", "slots"):
                host_register(d)
                host_register(p)
            if mode in ("slots", "pslots"):  # pointer batch over the same buffers (one map); pslots unregistered
                dptr = (d.ctypes.data + np.arange(n * k, dtype=np.uint64) * np.uint64(cs)).astype(np.uint64)
                pptr = (p.ctypes.data + np.arange(n * m, dtype=np.uint64) * np.uint64(cs)).astype(np.uint64)
                step = lambda: c.encode_batch(dptr, pptr, mem="host")  # noqa: E731
            else:
                step = lambda: c.encode_host_batch(d, p)  # noqa: E731
            res, digests = {}, set()
            for _ in range(a.rounds):
                for arm in arms:
                    for kn in KNOBS:
                        memec_amd.set_knob(kn, ARMS[arm].get(kn))
                    step()
                    t0 = time.perf_counter()
                    for _ in range(a.reps):
                        step()
                    dt = (time.perf_counter() - t0) / a.reps
                    res.setdefault(arm, []).append(round(n * k * cs / dt / 2**30, 2))
                    digests.add(int(p.view(np.uint64)[::4097].sum()))
            for kn in KNOBS:
                memec_amd.set_knob(kn, None)
            if mode in ("registered", "slots"):
                host_unregister(d)
                host_unregister(p)
            st = c.stats()
            print(json.dumps({"family": fam, "k": k, "m": m, "chunk": cs, "stripes": n, "mode": mode,
                              "GiBps_data": res, "equal": len(digests) == 1,
                              "zero_copy_calls": st["zero_copy_calls"], "staged_calls": st["staged_calls"]}),
                  flush=True)
        c.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""2 vs 4 block windows (mec_set_knob MEC_WINDOWS) for in-place byte-wise
decodes whose stripes take 256-thread blocks (stripe stride >= 8 MiB, or
exactly 512 KiB / 1 MiB), on ~48 GiB batches, at two allocation offsets
(a dummy buffer first: the placement decides part of the rate,
tools/place_ab.py), interleaved, median of 5 rounds of best-of-2.  Prints
the box fingerprint first.  Not product code.

  python3 tools/win4_ab.py
"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from memec_amd import Codec, fill_random, set_knob  # noqa: E402

MIB = 1 << 20
SHAPES = [  # k, m, chunk, erased
    (10, 4, MIB, [0, 1, 2, 3]), (10, 4, MIB, [0, 5, 10, 13]), (12, 4, MIB, [0, 1, 2, 3]),
    (6, 3, MIB, [0, 1, 2]), (8, 4, MIB, [1, 3, 8, 9]), (4, 4, 128 << 10, [0, 1, 2, 3]),
    (10, 4, 768 << 10, [0, 1, 2, 3]),
]


def main():
    dev = torch.device("cuda", 0)
    print(json.dumps({"box": bench.box_info(dev)}), flush=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for k, m, cs, erased in SHAPES:
        n = (48 << 30) // ((k + m) * cs)
        c = Codec("rs", k, m, cs)
        present = sum(1 << i for i in range(k + m) if i not in erased)
        nbytes = (k + len(erased)) * cs * n
        for off in (0, 3):
            dummy = torch.empty(off << 30, dtype=torch.uint8, device=dev) if off else None
            st = torch.empty(n, k + m, cs, dtype=torch.uint8, device=dev)
            fill_random(st, 9)
            res = {w: [] for w in (2, 4)}
            for _ in range(5):
                for w in (2, 4):
                    set_knob("MEC_WINDOWS", str(w))
                    c.decode(st, present)
                    best = None
                    for _ in range(2):
                        ev[0].record()
                        c.decode(st, present)
                        ev[1].record()
                        ev[1].synchronize()
                        ms = ev[0].elapsed_time(ev[1])
                        best = ms if best is None else min(best, ms)
                    res[w].append(best)
            set_knob("MEC_WINDOWS", None)
            pct = {w: nbytes / (statistics.median(v) * 1e-3) / 8e12 * 100 for w, v in res.items()}
            print("RS(%d,%d)@%-5dKiB erased %-14s n=%-5d off %d GiB  win2 %5.2f%%  win4 %5.2f%%  (%+.2f)"
                  % (k, m, cs >> 10, erased, n, off, pct[2], pct[4], pct[4] - pct[2]), flush=True)
            del st, dummy
            torch.cuda.empty_cache()
        c.close()


if __name__ == "__main__":
    main()

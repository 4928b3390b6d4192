#!/usr/bin/env python3
"""Launch-shape sweep on the configs[2] buffer itself: RS(10,4) in-place
decode of erasures {0,1,2,3}, 1 MiB chunks, 4096 stripes (56 GiB), over
resident-wave caps x block sizes x windows (mec_set_knob), interleaved
round-robin, median of 5 rounds of best-of-2.  Not product code.

  python3 tools/dec_shape_ab.py [stripes] [erased, e.g. 0,1,2,3]
  DSA_WPC=-1,12,16,20,24 DSA_BLOCK=64,256 DSA_WIN=-1,1,2,4   (-1 = library default)
"""
import itertools
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from memec_amd import Codec, fill_random, set_knob  # noqa: E402

K, M, CS = 10, 4, 1 << 20


def lst(name, dflt):
    return [int(x) for x in os.environ.get(name, dflt).split(",")]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    erased = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2, 3]
    c = Codec("rs", K, M, CS)
    st = torch.empty(n, K + M, CS, dtype=torch.uint8, device="cuda")
    fill_random(st, 5)
    present = sum(1 << i for i in range(K + M) if i not in erased)
    nbytes = (K + len(erased)) * CS * n
    arms = list(itertools.product(lst("DSA_WPC", "-1,12,16,20,24"), lst("DSA_BLOCK", "-1,64,256"),
                                  lst("DSA_WIN", "-1,1,2,4")))
    res = {a: [] for a in arms}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def knob(name, v):
        set_knob(name, None if v < 0 else str(v))
    for rnd in range(5):
        for a in arms:
            knob("MEC_WPC", a[0])
            knob("MEC_BLOCK", a[1])
            knob("MEC_WINDOWS", a[2])
            c.decode(st, present)
            best = None
            for _ in range(2):
                ev[0].record()
                c.decode(st, present)
                ev[1].record()
                ev[1].synchronize()
                ms = ev[0].elapsed_time(ev[1])
                best = ms if best is None else min(best, ms)
            res[a].append(best)
        print("round %d" % rnd, file=sys.stderr, flush=True)
    for name in ("MEC_WPC", "MEC_BLOCK", "MEC_WINDOWS"):
        set_knob(name, None)
    pct = {a: nbytes / (statistics.median(v) * 1e-3) / 8e12 * 100 for a, v in res.items()}
    for a in sorted(pct, key=pct.get, reverse=True):
        print("wpc %3d block %3d win %2d  %5.2f %%" % (a[0], a[1], a[2], pct[a]), flush=True)


if __name__ == "__main__":
    main()

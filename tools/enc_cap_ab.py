#!/usr/bin/env python3
"""Wave caps for the split-layout Vandermonde encode at wide stripes (the
current rule gives ceil_even(64/K + R): 8 waves for k = 16..20), per shape:
default vs 10 / 12 / 14 / 16, ~8 GiB each, interleaved, median of 5 rounds
of best-of-3.  Not product code."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from memec_amd import Codec, fill_random, set_knob  # noqa: E402

SHAPES = [(16, 4, 256 << 10), (20, 4, 16384), (12, 4, 65536), (10, 4, 1 << 20), (24, 4, 65536), (8, 2, 4096),
          (28, 4, 4096), (12, 2, 1 << 20)]
if os.environ.get("ENC_SHAPES"):  # k:m:chunk,...
    SHAPES = [tuple(int(x) for x in t.split(":")) for t in os.environ["ENC_SHAPES"].split(",")]


def main():
    dev = torch.device("cuda", 0)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    arms = os.environ.get("ENC_ARMS", "-,10,12,14,16").split(",")
    for k, m, cs in SHAPES:
        n = max(1, (8 << 30) // ((k + m) * cs))
        data = torch.empty(n, k, cs, dtype=torch.uint8, device=dev)
        fill_random(data, 6)
        par = torch.empty(n, m, cs, dtype=torch.uint8, device=dev)
        c = Codec(os.environ.get("ENC_FAMILY", "rs"), k, m, cs)
        res = {a: [] for a in arms}
        for _ in range(5):
            for a in arms:
                set_knob("MEC_WPC", None if a == "-" else a)
                c.encode(data, par)
                best = None
                for _ in range(3):
                    ev[0].record()
                    c.encode(data, par)
                    ev[1].record()
                    ev[1].synchronize()
                    ms = ev[0].elapsed_time(ev[1])
                    best = ms if best is None else min(best, ms)
                res[a].append(best)
        set_knob("MEC_WPC", None)
        nb = (k + m) * cs * n
        print("RS(%2d,%d)@%-7d encode " % (k, m, cs) + "  ".join("wpc %-2s %5.2f%%" % (a, nb / (statistics.median(res[a]) * 1e-3) / 8e12 * 100) for a in arms), flush=True)
        c.close()
        del data, par
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

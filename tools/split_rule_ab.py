#!/usr/bin/env python3
"""The split-layout dense wave rule (gf8_target_waves) against the old
split count ceil_even(64/K + R), per shape: mec_decode_split of erasures
{0..m-1} (survivors read from [s][k+m], outputs to [s][m]) and the ISA-L
Cauchy encode (a dense matrix) into a separate parity buffer, ~8 GiB each,
interleaved, median of 5 rounds of best-of-3.  Not product code."""
import math
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from memec_amd import Codec, fill_random, set_knob  # noqa: E402

SHAPES = [(10, 4, 1 << 20), (8, 2, 4096), (4, 2, 4096), (12, 4, 65536), (6, 3, 1 << 20), (16, 4, 256 << 10),
          (10, 4, 65536), (20, 4, 16384)]


def old_cap(k, m):
    return min(20, max(6, 2 * math.ceil((64.0 / k + m) / 2)))


def main():
    dev = torch.device("cuda", 0)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for k, m, cs in SHAPES:
        n = max(1, (8 << 30) // ((k + m) * cs))
        st = torch.empty(n, k + m, cs, dtype=torch.uint8, device=dev)
        fill_random(st, 5)
        out = torch.empty(n, m, cs, dtype=torch.uint8, device=dev)
        pm = sum(1 << i for i in range(k + m) if i >= m)
        rs, ic = Codec("rs", k, m, cs), Codec("isal_cauchy", k, m, cs)
        cases = {"dec_split": (lambda: rs.decode_split(st, out, pm), (k + m) * cs * n),
                 "isal_cauchy_enc": (lambda: ic.encode(st[:, :k], out), (k + m) * cs * n)}
        arms = {"new": None, "old": str(old_cap(k, m))}
        res = {(c_, a): [] for c_ in cases for a in arms}
        for _ in range(5):
            for c_, (fn, _) in cases.items():
                for a, v in arms.items():
                    set_knob("MEC_WPC", v)
                    fn()
                    best = None
                    for _ in range(3):
                        ev[0].record()
                        fn()
                        ev[1].record()
                        ev[1].synchronize()
                        ms = ev[0].elapsed_time(ev[1])
                        best = ms if best is None else min(best, ms)
                    res[(c_, a)].append(best)
        set_knob("MEC_WPC", None)
        for c_, (_, nb) in cases.items():
            p = {a: nb / (statistics.median(res[(c_, a)]) * 1e-3) / 8e12 * 100 for a in arms}
            print("RS-shape (%2d,%d)@%-7d %-16s old(cap %s) %5.2f%%  new %5.2f%%  (%+.2f)"
                  % (k, m, cs, c_, arms["old"], p["old"], p["new"], p["new"] - p["old"]), flush=True)
        rs.close()
        ic.close()
        del st, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

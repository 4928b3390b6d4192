#!/usr/bin/env python3
"""Wave caps (MEC_WPC) for the dense (decode) matrix in a split layout:
survivors read from [s][k+m], the outputs to a separate [s][4] buffer
(mec_decode_split), next to the Vandermonde encode of the same layout and
the in-place decode.  RS(10,4) @ 1 MiB x 4096, interleaved, median of 5
rounds of best-of-3.  Not product code.

  python3 tools/split_cap_ab.py [caps, e.g. -,12,14,16,18,20]
"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from memec_amd import Codec, fill_random, set_knob  # noqa: E402

K, M, CS, N = 10, 4, 1 << 20, 4096


def main():
    caps = sys.argv[1].split(",") if len(sys.argv) > 1 else ["-", "12", "14", "16", "18", "20"]
    dev = torch.device("cuda", 0)
    c = Codec("rs", K, M, CS)
    st = torch.empty(N, K + M, CS, dtype=torch.uint8, device=dev)
    fill_random(st, 11)
    out = torch.empty(N, M, CS, dtype=torch.uint8, device=dev)
    pm = sum(1 << i for i in range(K + M) if i not in (0, 1, 2, 3))
    cases = {
        "enc_strided": lambda: c.encode(st[:, :K], out),
        "dec_split": lambda: c.decode_split(st, out, pm),
        "dec_inplace": lambda: c.decode(st, pm),
    }
    nbytes = (K + M) * CS * N
    res = {(nm, cap): [] for nm in cases for cap in caps}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for rnd in range(5):
        for nm, fn in cases.items():
            for cap in caps:
                set_knob("MEC_WPC", None if cap == "-" else cap)
                fn()
                best = None
                for _ in range(3):
                    ev[0].record()
                    fn()
                    ev[1].record()
                    ev[1].synchronize()
                    ms = ev[0].elapsed_time(ev[1])
                    best = ms if best is None else min(best, ms)
                res[(nm, cap)].append(best)
        set_knob("MEC_WPC", None)
        print("round %d done" % rnd, file=sys.stderr, flush=True)
    for nm in cases:
        print("%-12s " % nm + "  ".join("wpc %-2s %5.2f%%" % (cap, nbytes / (statistics.median(res[(nm, cap)]) * 1e-3) / 8e12 * 100)
                                        for cap in caps), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where does the in-place RS(10,4) decode lose to the encode?  The same
launches with the arithmetic removed (mec_set_probe XOR twin) and with it,
over the layouts the bench and a server could use, interleaved round-robin,
median of 5 rounds of best-of-3.

  enc_dense      encode, data [s][10] dense, parity [s][4] separate (configs[1])
  enc_strided    encode, data = chunks 0..9 of [s][14], parity separate
  enc_inplace    encode, parity written into chunks 10..13 of [s][14]
  dec_inplace    decode {0,1,2,3} in place in [s][14] (configs[2])
  dec_tail       decode {10,11,12,13} in place (writes after the reads)
  dec_mixed      decode {0,5,10,13} in place
  dec_split      decode {0,1,2,3}: survivors read from [s][14], outputs to a separate [s][4]

Usage: python3 tools/twin_layouts.py [stripes]
"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from memec_amd import Codec, fill_random  # noqa: E402

K, M, CS = 10, 4, 1 << 20


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev = torch.device("cuda", 0)
    c = Codec("rs", K, M, CS)
    st = torch.empty(n, K + M, CS, dtype=torch.uint8, device=dev)
    fill_random(st, 11)
    dense = torch.empty(n, K, CS, dtype=torch.uint8, device=dev)
    fill_random(dense, 12)
    out = torch.empty(n, M, CS, dtype=torch.uint8, device=dev)

    def pm(er):
        return sum(1 << i for i in range(K + M) if i not in er)

    cases = {
        "enc_dense": (lambda: c.encode(dense, out), (K + M) * CS * n),
        "enc_strided": (lambda: c.encode(st[:, :K], out), (K + M) * CS * n),
        "enc_inplace": (lambda: c.encode(st[:, :K], st[:, K:]), (K + M) * CS * n),
        "dec_inplace": (lambda: c.decode(st, pm([0, 1, 2, 3])), (K + 4) * CS * n),
        "dec_tail": (lambda: c.decode(st, pm([10, 11, 12, 13])), (K + 4) * CS * n),
        "dec_mixed": (lambda: c.decode(st, pm([0, 5, 10, 13])), (K + 4) * CS * n),
        "dec_split": (lambda: c.decode_split(st, out, pm([0, 1, 2, 3])), (K + 4) * CS * n),
    }
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(cases)
    res = {(nm, tw): [] for nm in names for tw in (False, True)}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for rnd in range(5):
        for nm in names:
            fn, _ = cases[nm]
            for tw in (False, True):
                c.set_probe(tw)
                fn()
                best = None
                for _ in range(3):
                    ev[0].record()
                    fn()
                    ev[1].record()
                    ev[1].synchronize()
                    ms = ev[0].elapsed_time(ev[1])
                    best = ms if best is None else min(best, ms)
                res[(nm, tw)].append(best)
        c.set_probe(False)
        print("round %d done" % rnd, file=sys.stderr, flush=True)
    rows = {}
    for nm in names:
        b = cases[nm][1]
        code = b / (statistics.median(res[(nm, False)]) * 1e-3) / 8e12 * 100
        twin = b / (statistics.median(res[(nm, True)]) * 1e-3) / 8e12 * 100
        rows[nm] = {"code_pct": round(code, 2), "twin_pct": round(twin, 2)}
        print("%-12s code %5.2f %%  twin %5.2f %%  (of 8 TB/s)" % (nm, code, twin), flush=True)
    print(json.dumps({"stripes": n, "rows": rows}))


if __name__ == "__main__":
    main()

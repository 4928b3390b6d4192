#!/usr/bin/env python3
"""One strided launch shape for a counter pass: R launches of
  enc_split    [s][k] data -> [s][m] parity
  enc_inplace  parity written inside [s][k+m]
  dec_inplace  erasures {0..m-1} of [s][k+m] restored in place
over ~GIB GiB of stripes, timed by HIP events (printed), for rocprofv3
--pmc comparisons between shapes (tools/exp_r03i.sh).  Not product code.

  python3 tools/shape_pmc.py fam k m chunk op [reps] [gib]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from memec_amd import Codec, fill_random  # noqa: E402


def main():
    fam, k, m, cs, op = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
    gib = float(sys.argv[7]) if len(sys.argv) > 7 else 8
    n = max(1, int(gib * (1 << 30)) // ((k + m) * cs))
    c = Codec(fam, k, m, cs)
    if os.environ.get("SHAPE_TWIN") == "1":  # the launch's XOR-only twin (mec_set_probe)
        c.set_probe(True)
    if op == "enc_split":
        data = torch.empty(n, k, cs, dtype=torch.uint8, device="cuda")
        fill_random(data, 1)
        par = torch.empty(n, m, cs, dtype=torch.uint8, device="cuda")
        step = lambda: c.encode(data, par)  # noqa: E731
    else:
        st = torch.empty(n, k + m, cs, dtype=torch.uint8, device="cuda")
        fill_random(st, 1)
        if op == "enc_inplace":
            step = lambda: c.encode(st[:, :k], st[:, k:])  # noqa: E731
        else:
            present = sum(1 << i for i in range(m, k + m))
            step = lambda: c.decode(st, present)  # noqa: E731
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    step()
    ms = []
    for _ in range(reps):
        ev[0].record()
        step()
        ev[1].record()
        ev[1].synchronize()
        ms.append(ev[0].elapsed_time(ev[1]))
    nbytes = (k + m) * cs * n
    print("%s %d %d %d %s%s n=%d best %.4f ms %.2f %%" % (fam, k, m, cs, op, " twin" if os.environ.get("SHAPE_TWIN") == "1" else "",
                                                         n, min(ms), nbytes / (min(ms) * 1e-3) / 8e12 * 100), flush=True)


if __name__ == "__main__":
    main()

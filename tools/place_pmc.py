#!/usr/bin/env python3
"""One placement of tools/place_ab.py for a counter pass: allocate a dummy
buffer of D GiB first, then time R in-place decodes of the configs[4]
shape (CRS(12,4) @ 64 KiB x 32768, erasures {0,1,2,3}) or, with
PLACE_CASE=rs, of configs[2] (RS(10,4) @ 1 MiB x 4096).  Run under
rocprofv3 --pmc to compare counters of a slow and a fast placement.
Not product code.

  python3 tools/place_pmc.py D [R]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from memec_amd import Codec, fill_random  # noqa: E402


def main():
    d = float(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    fam, k, m, cs, n = ("rs", 10, 4, 1 << 20, 4096) if os.environ.get("PLACE_CASE") == "rs" else \
        ("cauchy", 12, 4, 65536, 32768)
    erased = [0, 1, 2, 3]
    dev = torch.device("cuda", 0)
    dummy = torch.empty(int(d * (1 << 30)), dtype=torch.uint8, device=dev) if d else None
    st = torch.empty(n, k + m, cs, dtype=torch.uint8, device=dev)
    fill_random(st, 3)
    c = Codec(fam, k, m, cs)
    present = sum(1 << i for i in range(k + m) if i not in erased)
    nbytes = (k + len(erased)) * cs * n
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    c.decode(st, present)
    out = []
    for _ in range(reps):
        ev[0].record()
        c.decode(st, present)
        ev[1].record()
        ev[1].synchronize()
        out.append(ev[0].elapsed_time(ev[1]))
    print("%s offset %.1f GiB st %#x: %s  best %.2f %%" % (fam, d, st.data_ptr(), " ".join("%.3f" % x for x in out),
          nbytes / (min(out) * 1e-3) / 8e12 * 100), flush=True)
    del dummy
    c.close()


if __name__ == "__main__":
    main()

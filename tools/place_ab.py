#!/usr/bin/env python3
"""Is the box-to-box bimodality of the in-place decodes a property of the
box or of where the buffer lands?  For several offsets of the allocation
(a dummy buffer of D GiB allocated first), time the configs[2] RS(10,4)
decode (4096 x 1 MiB stripes) and the configs[4] CRS(12,4) decode (32768 x
64 KiB) at several window counts (mec_set_knob MEC_WINDOWS), interleaved,
median of 3 rounds of best-of-2.  Prints the box fingerprint first.  Not
product code.

  python3 tools/place_ab.py [D,D,...]   (default 0,1,3,7,12)
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

CASES = [("rs", 10, 4, 1 << 20, 4096, [0, 1, 2, 3]), ("cauchy", 12, 4, 65536, 32768, [0, 1, 2, 3])]
# arms: label -> knobs (MEC_WINDOWS / MEC_SGROUP through mec_set_knob)
ARMS = {"win2": {"MEC_WINDOWS": "2"}, "win4": {"MEC_WINDOWS": "4"}, "perm": {"MEC_SGROUP": "p"},
        "default": {}}
if os.environ.get("PLACE_ARMS"):
    ARMS = {a: ARMS[a] for a in os.environ["PLACE_ARMS"].split(",")}


def main():
    dev = torch.device("cuda", 0)
    print(json.dumps({"box": bench.box_info(dev)}), flush=True)
    offs = [float(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 3, 7, 12]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    wins = list(ARMS)
    for fam, k, m, cs, n, erased in CASES:
        c = Codec(fam, k, m, cs)
        present = sum(1 << i for i in range(k + m) if i not in erased)
        nbytes = (k + len(erased)) * cs * n
        for d in offs:
            dummy = torch.empty(int(d * (1 << 30)), dtype=torch.uint8, device=dev) if d else None
            st = torch.empty(n, k + m, cs, dtype=torch.uint8, device=dev)
            fill_random(st, 3)
            res = {w: [] for w in wins}
            for _ in range(3):
                for w in wins:
                    for kn in ("MEC_WINDOWS", "MEC_SGROUP"):
                        set_knob(kn, ARMS[w].get(kn))
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
            for kn in ("MEC_WINDOWS", "MEC_SGROUP"):
                set_knob(kn, None)
            pct = {w: nbytes / (statistics.median(v) * 1e-3) / 8e12 * 100 for w, v in res.items()}
            print("%-6s k=%-2d cs=%-7d n=%-5d offset %5.1f GiB (st at %#x)  " % (fam, k, cs, n, d, st.data_ptr()) +
                  "  ".join("%s %5.2f%%" % (w, pct[w]) for w in wins), flush=True)
            del st, dummy
            torch.cuda.empty_cache()
        c.close()


if __name__ == "__main__":
    main()

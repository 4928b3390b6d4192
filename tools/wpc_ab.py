#!/usr/bin/env python3
"""Interleaved sweep of MEC_WPC (resident waves per CU, capped through the
LDS each block reserves) for the strided gf8 / bitmatrix launches, over
codes, chunk sizes and both layouts: split-buffer encode ([s][k] data,
[s][m] parity) and in-place decode ([s][k+m] stripes).  ~2 GiB of stripes
per case, 8 launches per sample, 5 rounds; median % of 8 TB/s.  Not product
code.

  python3 tools/wpc_ab.py [encode|decode|both]   (WPC_SIZES=4096,65536 to narrow)
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from memec_amd import Codec, fill_random, set_knob  # noqa: E402

CASES = [("rs", 4, 2), ("rs", 8, 2), ("rs", 12, 2), ("rs", 10, 4), ("cauchy", 4, 2), ("cauchy", 8, 2),
         ("cauchy", 12, 4)]
SIZES = [4096, 8192, 16384, 32768, 65536, 262144, 1 << 20]
WPC = [0, 4, 6, 8, 12, 16, 24]
if os.environ.get("WPC_CASES"):  # fam:k:m,...
    CASES = [(c.split(":")[0], int(c.split(":")[1]), int(c.split(":")[2])) for c in os.environ["WPC_CASES"].split(",")]
if os.environ.get("WPC_LIST"):
    WPC = [int(x) for x in os.environ["WPC_LIST"].split(",")]
VAR = os.environ.get("WPC_VAR", "MEC_WPC")  # the knob swept (e.g. MEC_WINDOWS); 0 = unset


def main():
    ops = sys.argv[1] if len(sys.argv) > 1 else "both"
    ops = ["encode", "decode"] if ops == "both" else [ops]
    sizes = [int(x) for x in os.environ["WPC_SIZES"].split(",")] if os.environ.get("WPC_SIZES") else SIZES
    torch.cuda.set_device(0)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for op in ops:
        for fam, k, m in CASES:
            for cs in sizes:
                n = max(1, int(os.environ.get("WPC_GIB", "2")) * (1 << 30) // ((k + m) * cs))
                codec = Codec(fam, k, m, cs, device=0)
                erased = list(range(m))
                if op == "encode":
                    data = torch.empty(n, k, cs, dtype=torch.uint8, device="cuda")
                    fill_random(data, 1)
                    par = torch.empty(n, m, cs, dtype=torch.uint8, device="cuda")
                    step = lambda: codec.encode(data, par)  # noqa: E731
                    nbytes = (k + m) * cs * n
                else:
                    st = torch.empty(n, k + m, cs, dtype=torch.uint8, device="cuda")
                    fill_random(st, 1)
                    present = sum(1 << i for i in range(k + m) if i not in erased)
                    step = lambda: codec.decode(st, present)  # noqa: E731
                    nbytes = (k + m) * cs * n
                res = {w: [] for w in WPC}
                for _ in range(5):
                    for w in WPC:
                        if w < 0 or (VAR != "MEC_WPC" and w == 0):  # -1: the library's default
                            set_knob(VAR, None)
                        else:
                            set_knob(VAR, str(w))
                        step()
                        ev[0].record()
                        for _ in range(8):
                            step()
                        ev[1].record()
                        ev[1].synchronize()
                        res[w].append(ev[0].elapsed_time(ev[1]) / 8)
                set_knob(VAR, None)
                pct = {w: nbytes / (statistics.median(v) * 1e-3) / 8e12 * 100 for w, v in res.items()}
                best = max(pct, key=pct.get)
                print("%-6s %-6s k=%-2d m=%d cs=%-7d " % (op, fam, k, m, cs) +
                      " ".join("w%-2d %5.1f" % (w, pct[w]) for w in WPC) +
                      "  best w%d (+%.1f)" % (best, pct[best] - pct[0]), flush=True)
                del codec
                if op == "encode":
                    del data, par
                else:
                    del st
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

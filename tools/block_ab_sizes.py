#!/usr/bin/env python3
"""Interleaved A/B of MEC_BLOCK=64 vs 256 for in-place decodes (default) or
split-buffer encodes (AB_OP=encode) across chunk sizes (the block-size
rules).  ~4 GiB of stripe
per case, 10 launches per sample, 5 rounds; median kernel ms.  Not product
code."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from memec_amd import Codec, fill_random, set_knob  # noqa: E402

CASES = [("rs", 4, 2, [0, 1]), ("rs", 10, 4, [0, 1, 2, 3]), ("cauchy", 12, 4, [0, 1, 2, 3])]
SIZES = [4096, 16384, 65536, 262144, 1 << 20]


def main():
    global CASES, SIZES
    if os.environ.get("AB_CASES") == "cauchy":  # bitmatrix kernel, larger chunks
        CASES = [("cauchy", 12, 4, [0, 1, 2, 3]), ("cauchy", 4, 2, [0, 1])]
        SIZES = [65536, 131072, 262144, 524288, 1 << 20, 2 << 20]
    torch.cuda.set_device(0)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for fam, k, m, erased in CASES:
        for cs in SIZES:
            n = max(1, (4 << 30) // ((k + m) * cs))
            codec = Codec(fam, k, m, cs, device=0)
            if os.environ.get("AB_OP") == "encode":  # split data / parity buffers
                data = torch.empty(n, k, cs, dtype=torch.uint8, device="cuda")
                fill_random(data, 1)
                par = torch.empty(n, m, cs, dtype=torch.uint8, device="cuda")
                st = (data, par)
                nbytes = (k + m) * cs * n
            else:
                st = torch.empty(n, k + m, cs, dtype=torch.uint8, device="cuda")
                fill_random(st, 1)
                nbytes = (k + len(erased)) * cs * n
            present = sum(1 << i for i in range(k + m) if i not in erased)

            def step():
                if isinstance(st, tuple):
                    codec.encode(*st)
                else:
                    codec.decode(st, present)
            res = {64: [], 256: []}
            for _ in range(5):
                for b in (64, 256):
                    set_knob("MEC_BLOCK", str(b))
                    step()
                    ev[0].record()
                    for _ in range(10):
                        step()
                    ev[1].record()
                    ev[1].synchronize()
                    res[b].append(ev[0].elapsed_time(ev[1]) / 10)
            set_knob("MEC_BLOCK", None)
            line = "%s(%d,%d) cs=%7d n=%6d" % (fam, k, m, cs, n)
            for b in (64, 256):
                med = statistics.median(res[b])
                line += "  B%-3d %.4f ms %.1f%%" % (b, med, nbytes / med / 1e6 / 80)
            print(line, flush=True)
            del st
            codec.close()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

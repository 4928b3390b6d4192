#!/usr/bin/env python3
"""Interleaved A/B of launch shapes (MEC_BLOCK x MEC_WPC x MEC_BM_VW x
MEC_WINDOWS) for the strided
launches over three layouts: split-buffer encode ([s][k] data, [s][m]
parity), in-place encode (parity inside [s][k+m], as tools/perf_sweep.py)
and in-place decode of erasures {0..m-1}.  ~2 GiB of stripes per case, 8
launches per sample, 5 rounds; median % of 8 TB/s.  Not product code.

  AB_CASES=cauchy:12:2,... AB_SIZES=8192,... AB_ARMS=-:-,64:8,256:12:2 \
  AB_OPS=enc_split,enc_inplace,dec_inplace,update python3 tools/bm_small_ab.py
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from memec_amd import Codec, fill_random, set_knob  # noqa: E402


def env_list(name, default, conv=str):
    v = os.environ.get(name)
    return [conv(x) for x in v.split(",")] if v else default


CASES = [(c.split(":")[0], int(c.split(":")[1]), int(c.split(":")[2]))
         for c in env_list("AB_CASES", ["cauchy:12:2", "cauchy:8:2", "cauchy:12:4"])]
SIZES = env_list("AB_SIZES", [4096, 8192, 16384, 32768, 65536], int)
# block:wpc[:vw[:windows]] — MEC_BLOCK, MEC_WPC, MEC_BM_VW, MEC_WINDOWS ("-" leaves a knob unset)
KNOBS = ("MEC_BLOCK", "MEC_WPC", "MEC_BM_VW", "MEC_WINDOWS")
ARMS = [tuple((a + ":-:-:-").split(":")[:4])
        for a in env_list("AB_ARMS", ["-:-", "64:0", "64:8", "64:12", "64:16", "256:0", "256:8", "256:12", "256:16"])]
OPS = env_list("AB_OPS", ["enc_split", "enc_inplace", "dec_inplace"])


def setenv(name, v):
    if v == "-":
        set_knob(name, None)
    else:
        set_knob(name, v)


def main():
    torch.cuda.set_device(0)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    gib = float(os.environ.get("AB_GIB", "2"))
    for fam, k, m in CASES:
        for cs in SIZES:
            n = max(1, int(gib * (1 << 30)) // ((k + m) * cs))
            codec = Codec(fam, k, m, cs, device=0)
            for op in OPS:
                if op == "update":  # parity ^= A[:, j] * delta (the server's delta path)
                    data = torch.empty(n, cs, dtype=torch.uint8, device="cuda")
                    fill_random(data, 1)
                    par = torch.zeros(n, m, cs, dtype=torch.uint8, device="cuda")
                    bufs = [data, par]
                    step = lambda: codec.encode_update(min(3, k - 1), data, par)  # noqa: E731
                elif op == "enc_split":
                    data = torch.empty(n, k, cs, dtype=torch.uint8, device="cuda")
                    fill_random(data, 1)
                    par = torch.empty(n, m, cs, dtype=torch.uint8, device="cuda")
                    bufs = [data, par]
                    step = lambda: codec.encode(data, par)  # noqa: E731
                else:
                    st = torch.empty(n, k + m, cs, dtype=torch.uint8, device="cuda")
                    fill_random(st, 1)
                    bufs = [st]
                    if op == "enc_inplace":
                        step = lambda: codec.encode(st[:, :k], st[:, k:])  # noqa: E731
                    else:
                        present = sum(1 << i for i in range(m, k + m))
                        step = lambda: codec.decode(st, present)  # noqa: E731
                nbytes = (1 + 2 * m) * cs * n if op == "update" else (k + m) * cs * n
                res = {a: [] for a in ARMS}
                for _ in range(5):
                    for a in ARMS:
                        for knob, val in zip(KNOBS, a):
                            setenv(knob, val)
                        step()
                        ev[0].record()
                        for _ in range(8):
                            step()
                        ev[1].record()
                        ev[1].synchronize()
                        res[a].append(ev[0].elapsed_time(ev[1]) / 8)
                for knob in KNOBS:
                    setenv(knob, "-")
                pct = {a: nbytes / (statistics.median(v) * 1e-3) / 8e12 * 100 for a, v in res.items()}
                best = max(pct, key=pct.get)
                print("%-11s %-6s k=%-2d m=%d cs=%-7d " % (op, fam, k, m, cs) +
                      " ".join("%s %5.1f" % (":".join(a), pct[a]) for a in ARMS) +
                      "  best %s (+%.1f)" % (":".join(best), pct[best] - pct[ARMS[0]]), flush=True)
                del bufs, step
                data = par = st = None
                torch.cuda.empty_cache()
            codec.close()


if __name__ == "__main__":
    main()

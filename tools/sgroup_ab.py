#!/usr/bin/env python3
"""Interleaved A/B of the stripe-group block map (MEC_SGROUP, stream_common.hpp
stripe_tile) on RS(10,4) at ~56 GiB per launch: split-buffer encode at 64 KiB
.. 4 MiB chunks and in-place decode of {0,1,2,3} at 1 MiB.  Every grouped
run's output is checked against the identity map's.  Median kernel ms over
rounds x 10 launches (HIP events).  Not product code.

  SG_VALUES=0,16,32:64,d SG_CHUNKS_K=1024,4096 SG_DEC_K=1024 python3 tools/sgroup_ab.py [rounds=5]
  (value g[:run]; 0 = identity map, d = the library's default rule)
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from memec_amd import Codec, fill_random, set_knob  # noqa: E402

FAM, K, M = os.environ.get("SG_CODE", "rs,10,4").split(",")
K, M = int(K), int(M)
TOTAL = 56 << 30


def set_group(v):
    if v == "d":  # the library's own rule
        set_knob("MEC_SGROUP", None)
    else:
        set_knob("MEC_SGROUP", v)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    vals = os.environ.get("SG_VALUES", "0,16,32,64,128").split(",")
    torch.cuda.set_device(0)
    pool_d = torch.empty(TOTAL * K // (K + M), dtype=torch.uint8, device="cuda")
    pool_p = torch.empty(TOTAL * M // (K + M), dtype=torch.uint8, device="cuda")
    fill_random(pool_d, 5)
    cases = []
    for cs in [int(x) << 10 for x in os.environ.get("SG_CHUNKS_K", "64,256,1024,4096").split(",")]:
        n = TOTAL // ((K + M) * cs)
        c = Codec(FAM, K, M, cs)
        data = pool_d[: n * K * cs].view(n, K, cs)
        par = pool_p[: n * M * cs].view(n, M, cs)
        cases.append(("%s encode split %5d KiB" % (FAM, cs >> 10), c, (lambda c=c, d=data, p=par: c.encode(d, p)),
                      par, (K + M) * cs * n))
    dec = [int(x) << 10 for x in os.environ.get("SG_DEC_K", "1024").split(",") if x]
    if dec and os.environ.get("SG_DECODE", "1") == "1":
        whole = torch.cat([pool_d.view(-1), pool_p.view(-1)])
        for cs in dec:
            n = TOTAL // ((K + M) * cs)
            c = Codec(FAM, K, M, cs)
            st = whole[: n * (K + M) * cs].view(n, K + M, cs)
            present = sum(1 << i for i in range(K + M) if i not in (0, 1, 2, 3))
            cases.append(("%s decode in place %5d KiB" % (FAM, cs >> 10), c, (lambda c=c, st=st, p=present: c.decode(st, p)),
                          st[:, :4], (K + 4) * cs * n))
    # correctness: every group value gives the identity map's bytes
    for name, c, step, out, _ in cases:
        set_knob("MEC_SGROUP", "0")
        step()
        torch.cuda.synchronize()
        ref = out.clone()
        for v in vals:
            out.zero_()
            set_group(v)
            step()
            torch.cuda.synchronize()
            assert torch.equal(out, ref), (name, v)
        del ref
    print("all group values bit-exact vs the identity map", flush=True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name, c, step, out, nbytes in cases:
        res = {v: [] for v in vals}
        for _ in range(rounds):
            for v in vals:
                set_group(v)
                step()
                ev[0].record()
                for _ in range(10):
                    step()
                ev[1].record()
                ev[1].synchronize()
                res[v].append(ev[0].elapsed_time(ev[1]) / 10)
        line = "%-34s" % name
        for v in vals:
            med = statistics.median(res[v])
            line += "  g%-4s %5.1f %%" % (v, nbytes / med / 1e6 / 80)
        print(line, flush=True)


if __name__ == "__main__":
    main()

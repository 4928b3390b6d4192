#!/usr/bin/env python3
"""RS(10,4)@1 MiB x 4096 stripes, one arm per process, for per-channel EA
counters: run it under

  rocprofv3 -E tools/ea_channels.yaml --pmc MEC_EA_RD_CH0 ... -- python3 tools/channel_probe.py ARM

(tools/gpu_session.sh `channels`), where the derived counters select one
TCC instance of TCC_EA0_RDREQ / _WRREQ each, summed over the XCCs.
Arms: enc_split (configs[1]: data and parity buffers), dec_inplace
(configs[2]: erasures {0,1,2,3} rebuilt inside the stripe buffer),
dec_split (the same decode into a separate output buffer).  Prints the
kernel time per step."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from memec_amd import Codec, fill_random
    arm = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    k, m, cs, n = 10, 4, 1 << 20, 4096
    torch.cuda.set_device(0)
    c = Codec("rs", k, m, cs)
    erased = [0, 1, 2, 3]
    present = sum(1 << i for i in range(k + m) if i not in erased)
    if arm == "enc_split":
        data = torch.empty(n, k, cs, dtype=torch.uint8, device="cuda")
        fill_random(data, 5)
        par = torch.empty(n, m, cs, dtype=torch.uint8, device="cuda")
        step = lambda: c.encode(data, par)  # noqa: E731
    else:
        st = torch.empty(n, k + m, cs, dtype=torch.uint8, device="cuda")
        fill_random(st, 6)
        c.encode(st[:, :k], st[:, k:])
        if arm == "dec_inplace":
            st[:, erased] = 0
            step = lambda: c.decode(st, present)  # noqa: E731
        else:
            out = torch.empty(n, k + m, cs, dtype=torch.uint8, device="cuda")
            step = lambda: c.decode_split(st, out, present)  # noqa: E731
    step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / steps
    print(json.dumps({"arm": arm, "ms_per_step": round(ms, 4), "frac": round((k + m) * cs * n / (ms * 1e-3) / 8e12, 4)}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""RS(10,4)@1 MiB x 4096 stripes, one arm per process, for per-channel EA
counters: run it under

  python3 tools/channel_probe.py --write-yaml ea_channels.yaml
  rocprofv3 -E ea_channels.yaml --pmc MEC_EA_RD_CH0 ... -- python3 tools/channel_probe.py ARM

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


# Derived counters per TCC instance (rocprofv3 -E): MEC_EA_<KIND>_CH<i> =
# reduce(select(<counter>, [DIMENSION_INSTANCE=[i]]), sum), i.e. one TCC
# channel summed over the XCCs.
KINDS = {"RD": "TCC_EA0_RDREQ", "WR": "TCC_EA0_WRREQ", "RDLVL": "TCC_EA0_RDREQ_LEVEL",
         "RDSTALL": "TCC_EA0_RDREQ_DRAM_CREDIT_STALL", "WRSTALL": "TCC_EA0_WRREQ_DRAM_CREDIT_STALL"}


def write_yaml(path):
    out = ["rocprofiler-sdk:", "  counters-schema-version: 1", "  counters:"]
    for tag, ctr in KINDS.items():
        for i in range(16):
            out += [f"  - name: MEC_EA_{tag}_CH{i}",
                    f"    description: {ctr} of TCC instance (channel) {i}, summed over the XCCs",
                    "    properties: []", "    definitions:", "    - architectures:", "      - gfx950",
                    f"      expression: reduce(select({ctr},[DIMENSION_INSTANCE=[{i}]]),sum)"]
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")


def main():
    if sys.argv[1] == "--write-yaml":
        write_yaml(sys.argv[2])
        return
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

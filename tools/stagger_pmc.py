#!/usr/bin/env python3
"""Per-arm memory-side counters of tools/stagger_probe under rocprofv3 --pmc.

  python tools/stagger_pmc.py ARMS RUN_DIR [RUN_DIR ...]

ARMS is the probe's comma-separated arm list; each RUN_DIR holds one
rocprofv3 pass (run_counter_collection.csv).  Every arm is 6 dispatches of
probe_kernel in list order (one untimed, then 5 timed): the 5 timed ones are
summed.  Derived, as DESIGN §9's round-3 table: EA read latency =
TCC_EA0_RDREQ_LEVEL / RDREQ (cycles a read waits at the memory side), reads
in flight = RDREQ_LEVEL / GRBM_GUI_ACTIVE, and the same for writes.
Prints one JSON line per arm."""
import csv
import json
import os
import sys


def load(run_dir):
    per = {}  # dispatch id -> {counter: value}
    with open(os.path.join(run_dir, "run_counter_collection.csv")) as f:
        for row in csv.DictReader(f):
            if "probe_kernel" not in row["Kernel_Name"]:
                continue
            d = per.setdefault(int(row["Dispatch_Id"]), {})
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return [per[k] for k in sorted(per)]


def main():
    arms = sys.argv[1].split(",")
    sums = [dict() for _ in arms]
    for run_dir in sys.argv[2:]:
        rows = load(run_dir)
        if len(rows) != 6 * len(arms):
            raise SystemExit(f"{run_dir}: {len(rows)} probe dispatches, expected {6 * len(arms)}")
        for a in range(len(arms)):
            for r in rows[a * 6 + 1:a * 6 + 6]:
                for k, v in r.items():
                    sums[a][k] = sums[a].get(k, 0.0) + v
    for name, s in zip(arms, sums):
        out = {"arm": name, **{k: s[k] for k in sorted(s)}}
        rd, wr, g = s.get("TCC_EA0_RDREQ_sum"), s.get("TCC_EA0_WRREQ_sum"), s.get("GRBM_GUI_ACTIVE")
        if rd and "TCC_EA0_RDREQ_LEVEL_sum" in s:
            out["ea_read_latency"] = round(s["TCC_EA0_RDREQ_LEVEL_sum"] / rd, 1)
            if g:
                out["ea_reads_in_flight"] = round(s["TCC_EA0_RDREQ_LEVEL_sum"] / g, 1)
        if wr and "TCC_EA0_WRREQ_LEVEL_sum" in s:
            out["ea_write_latency"] = round(s["TCC_EA0_WRREQ_LEVEL_sum"] / wr, 1)
            if g:
                out["ea_writes_in_flight"] = round(s["TCC_EA0_WRREQ_LEVEL_sum"] / g, 1)
        print(json.dumps(out))


if __name__ == "__main__":
    main()

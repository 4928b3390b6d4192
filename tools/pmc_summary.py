#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into profiles/pmc_<config>.json.

Input: gpurun_out/<TAG>/pmc_fetch_<cfg>/run_counter_collection.csv
(FETCH_SIZE pass) and gpurun_out/<TAG>/pmc_write_<cfg>/run_counter_collection.csv
(WRITE_SIZE pass), produced by TAG=<TAG> tools/gpu_session.sh pmc
(PMC_DIR overrides the directory).  Corrections per
MI355X_MICROARCH.md §HBM: counters are in KiB; on gfx950 FETCH_SIZE reads
exactly half of a wide coalesced streaming read, so read bytes =
2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for 16-B-per-lane stores.
The tail kernels never run for these sizes; only the main coding kernel
(gf8_kernel / bm_kernel) is averaged.
"""
import csv
import json
import re
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, counter):
    """Average per launch of the dominant coding kernel (the one launched
    most often: the timed step), ignoring setup / verification launches."""
    by_name = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if row["Counter_Name"] != counter:
                continue
            # the coding kernels, not bench.py's XOR twin (gf8_kernel S = 2, kGf8Xor)
            if re.search(r"gf8_kernel<\d+, \d+, (true|false), 2,", name):
                continue
            if "gf8_kernel" in name or "gf8_mg_kernel" in name or "bm_kernel" in name:
                by_name.setdefault(name, []).append(float(row["Counter_Value"]))
    if not by_name:
        return None, 0, []
    name = max(by_name, key=lambda n: len(by_name[n]))
    vals = by_name[name]
    return sum(vals) / len(vals), len(vals), [name]


def main(cfgs, out_dir, tag):
    sys.path.insert(0, ROOT)
    from bench import CONFIGS
    for cfg in cfgs:
        # tools/gpu_session.sh writes under gpurun_out/<TAG>/ (older runs: gpurun_out/)
        base = os.environ.get("PMC_DIR") or os.path.join(ROOT, "gpurun_out", tag)
        if not os.path.isdir(base):
            base = os.path.join(ROOT, "gpurun_out")
        fpath = os.path.join(base, "pmc_fetch_%s" % cfg, "run_counter_collection.csv")
        wpath = os.path.join(base, "pmc_write_%s" % cfg, "run_counter_collection.csv")
        if not (os.path.exists(fpath) and os.path.exists(wpath)):
            print("missing", cfg)
            continue
        fetch_kib, nf, names = per_launch(fpath, "FETCH_SIZE")
        write_kib, nw, _ = per_launch(wpath, "WRITE_SIZE")
        fam, k, m, cs, stripes, op, erased = CONFIGS[cfg]
        if op == "update":  # read delta + m parities, write m parities
            read_alg = (1 + m) * cs * stripes
            write_alg = m * cs * stripes
        else:
            read_alg = (k * cs * stripes)
            write_alg = (m if op == "encode" else len(erased)) * cs * stripes
        rd = 2 * fetch_kib * 1024
        wr = write_kib * 1024
        rec = {"config": cfg, "round": tag, "kernels": names, "launches": [nf, nw],
               "FETCH_SIZE_kib_per_launch": fetch_kib, "WRITE_SIZE_kib_per_launch": write_kib,
               "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
               "hbm_bytes_per_launch": rd + wr,
               "algorithmic_read_bytes": read_alg, "algorithmic_write_bytes": write_alg,
               "traffic_over_algorithmic": (rd + wr) / (read_alg + write_alg),
               "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 wide-stream halving), write = WRITE_SIZE x 1024",
               "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, tag %s" % tag}
        with open(os.path.join(out_dir, "pmc_%s.json" % cfg), "w") as f:
            json.dump(rec, f, indent=1)
        print(cfg, "traffic/alg = %.4f" % rec["traffic_over_algorithmic"])


if __name__ == "__main__":
    tag = os.environ.get("TAG", "r01")
    main(sys.argv[1:] or ["rs_enc"], os.path.join(ROOT, "profiles"), tag)

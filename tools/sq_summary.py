#!/usr/bin/env python3
"""Summarise a rocprofv3 SQ_* counter pass (tools/gpu_session.sh sq) for the
coding kernels: per-launch counter averages plus derived ratios.

  VALU/wave       SQ_INSTS_VALU / SQ_WAVES (VALU instructions per wave)
  SALU/wave       SQ_INSTS_SALU / SQ_WAVES
  valu_busy       SQ_ACTIVE_INST_VALU * 4 / (GRBM_GUI_ACTIVE * 256 CUs * 4 SIMDs)
                  (ACTIVE_INST_VALU counts per-SIMD issue cycles in quads;
                  the ratio is a utilisation estimate, comparable between
                  variants of one kernel)
  issue_stall     SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  occupancy       SQ_WAVE_CYCLES / SQ_BUSY_CYCLES (mean resident waves)
"""
import csv
import json
import sys
from collections import defaultdict


def summarise(path):
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if "gf8_kernel" not in name and "bm_kernel" not in name:
                continue
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
            meta[name] = {"vgpr": int(row["VGPR_Count"]), "agpr": int(row["Accum_VGPR_Count"]),
                          "sgpr": int(row["SGPR_Count"]), "lds": int(row["LDS_Block_Size"]),
                          "grid": int(row["Grid_Size"])}
    out = {}
    for name, ctr in acc.items():
        avg = {c: sum(v) / len(v) for c, v in ctr.items()}
        waves = avg.get("SQ_WAVES", 0) or 1
        d = dict(meta[name])
        d["counters"] = avg
        d["valu_per_wave"] = avg.get("SQ_INSTS_VALU", 0) / waves
        d["salu_per_wave"] = avg.get("SQ_INSTS_SALU", 0) / waves
        if "GRBM_GUI_ACTIVE" in avg and "SQ_ACTIVE_INST_VALU" in avg:
            d["valu_busy"] = avg["SQ_ACTIVE_INST_VALU"] * 4 / (avg["GRBM_GUI_ACTIVE"] * 256 * 4)
        if "SQ_WAVE_CYCLES" in avg:
            d["issue_stall"] = avg.get("SQ_WAIT_INST_ANY", 0) / avg["SQ_WAVE_CYCLES"]
            if avg.get("SQ_BUSY_CYCLES"):
                d["mean_waves"] = avg["SQ_WAVE_CYCLES"] / avg["SQ_BUSY_CYCLES"]
        out[name] = d
    return out


if __name__ == "__main__":
    res = {p: summarise(p) for p in sys.argv[1:]}
    print(json.dumps(res, indent=1))

#!/usr/bin/env bash
# tools/lib_ab.sh — interleaved A/B of two libmec builds on the GPU box:
# memec_amd/libmec.so (new) against memec_amd/libmec_<OLD>.so, bench.py
# lines per config, ROUNDS alternations.  Restores the new build at the end.
# Not product code.
#   OLD=flat CFGS="rs_enc rs_dec" ROUNDS=2 EXTRA="--stripes 32768" bash tools/lib_ab.sh
set -u
cd "$(dirname "$0")/.."
OLD=${OLD:-flat}
CFGS=${CFGS:-rs_enc rs_dec crs_enc crs_dec rs8_small}
ROUNDS=${ROUNDS:-2}
mkdir -p gpurun_out/lib_ab
cp memec_amd/libmec.so /tmp/libmec_new.so || exit 1
rc=0
for r in $(seq 1 "$ROUNDS"); do
    for v in new "$OLD"; do
        if [ "$v" = new ]; then cp /tmp/libmec_new.so memec_amd/libmec.so; else cp "memec_amd/libmec_$v.so" memec_amd/libmec.so; fi
        for c in $CFGS; do
            timeout -k 10 200 python bench.py --config "$c" --no-cpu-baseline --no-extra-configs --steps 20 ${EXTRA:-} \
                > "gpurun_out/lib_ab/${v}_${c}_$r.json" 2> "gpurun_out/lib_ab/${v}_${c}_$r.err" || { rc=$?; break 3; }
            python - "$v" "$c" "$r" <<'PY'
import json, sys
v, c, r = sys.argv[1:]
d = json.loads(open("gpurun_out/lib_ab/%s_%s_%s.json" % (v, c, r)).read().strip().splitlines()[-1])
ro = d["roofline"]
print("%-6s %-10s round %s  kernel %.4f ms  %.1f %%  ceiling %s" % (v, c, r, ro["kernel_ms"], 100 * ro["frac"],
      ro.get("stream_ceiling_GBps")), flush=True)
PY
        done
    done
done
cp /tmp/libmec_new.so memec_amd/libmec.so
exit $rc

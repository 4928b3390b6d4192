#!/usr/bin/env bash
# tools/knob_ab.sh VAR "VALUES" "CONFIGS" [ROUNDS] — interleaved A/B of one
# launch knob over bench.py configs: for each round, config and value, one
# bench.py process with VAR=value (libmec reads it at first use; "unset"
# leaves the built-in rule), the value and the line appended to
# $OUT (default gpurun_out/knob_ab.jsonl).  Each run under its own limit;
# the script stops at the first failing run.
#   bash tools/knob_ab.sh MEC_TILE_SKEW "unset 0 8 64" "rs_dec crs_dec" 2
set -u
cd "$(dirname "$0")/.."
VAR=$1
VALUES=$2
CONFIGS=$3
ROUNDS=${4:-2}
OUT=${OUT:-gpurun_out/knob_ab.jsonl}
mkdir -p "$(dirname "$OUT")"
for r in $(seq 1 "$ROUNDS"); do
    for c in $CONFIGS; do
        for v in $VALUES; do
            echo "{\"round\": $r, \"config\": \"$c\", \"var\": \"$VAR\", \"value\": \"$v\"}" >> "$OUT"
            if [ "$v" = unset ]; then
                timeout -k 10 240 env -u "$VAR" python bench.py --config "$c" --no-cpu-baseline --no-extra-configs \
                    --no-pmc-live --no-ceiling --steps 10 >> "$OUT" 2>> "$OUT.err" || exit 1
            else
                timeout -k 10 240 env "$VAR=$v" python bench.py --config "$c" --no-cpu-baseline --no-extra-configs \
                    --no-pmc-live --no-ceiling --steps 10 >> "$OUT" 2>> "$OUT.err" || exit 1
            fi
        done
    done
done

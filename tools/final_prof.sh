#!/usr/bin/env bash
# Round-final profiler evidence: the exact default bench command under
# rocprofv3 --kernel-trace --stats (its bench line and kernel averages must
# agree), then tools/gpu_session.sh prof for every bench config.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o run \
    -- python3 bench.py > "$OUT/default_cmd_under_rocprof.json" 2> "$OUT/default_cmd_under_rocprof.err" || exit $?
PROF_CONFIGS="${PROF_CONFIGS:-rs_enc rs_dec rs_dec_mixed crs_enc crs_dec rs8_small rs42 rs42_dec rs_update rs8_update rs16_8 rs16_8_dec isal12_8}" bash tools/gpu_session.sh prof

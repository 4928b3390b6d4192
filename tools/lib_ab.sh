#!/bin/bash
# Build A/B of the host paths: libmec builds alternated process by process
# (MEMEC_LIBMEC), after the staged-path GPU tests on the in-tree build.
# ARMS = name=path[:ENV=VAL] list, "new" = the in-tree libmec.so; save a
# baseline first (`cp memec_amd/libmec.so memec_amd/ab/libmec_base.so`).
#   TAG=r06n MODES=pageable,pslots ARMS="base=memec_amd/ab/libmec_base.so new=" bash tools/lib_ab.sh
set -o pipefail
TAG=${TAG:-libab}
MODES=${MODES:-pageable,pslots}
ARMS=${ARMS:-"base=memec_amd/ab/libmec_base.so new="}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_multi.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || exit 1
for i in 1 2; do for A in $ARMS; do
  L=${A%%=*}; spec=${A#*=}; path=${spec%%:*}; envs=""
  [ "$spec" != "$path" ] && envs=${spec#*:}
  ( if [ -n "$path" ]; then export MEMEC_LIBMEC=$PWD/$path; fi
    [ -n "$envs" ] && export "$envs"
    timeout -k 10 240 python3 -u tools/host_ab.py --arms unset --rounds 2 --modes $MODES > gpurun_out/$TAG/ab_${L}_$i.jsonl 2>> gpurun_out/$TAG/ab.err ) || exit 1
done; done
python3 - "$TAG" $ARMS <<'PY'
import json, sys
tag, arms = sys.argv[1], [a.split("=")[0] for a in sys.argv[2:]]
rows = {}
for L in arms:
    for i in (1, 2):
        for line in open("gpurun_out/%s/ab_%s_%d.jsonl" % (tag, L, i)):
            d = json.loads(line)
            rows.setdefault("%s(%d,%d)@%d %s" % (d["family"], d["k"], d["m"], d["chunk"], d["mode"]), {}) \
                .setdefault(L, []).extend(d["GiBps_data"]["unset"])
with open("gpurun_out/%s/summary.json" % tag, "w") as f:
    json.dump(rows, f, indent=1)
for k, v in rows.items():
    print(k, v)
PY

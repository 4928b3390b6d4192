#!/bin/bash
# Back-to-back device batches (tools/wide_ab.py shapes) on two libmec builds,
# processes alternated, plus a kernel + memory-copy trace of each build on
# one shape (tools/trace_gaps.py: the gap between consecutive launches).
#   TAG=r06r VARIANT=memec_amd/ab/libmec_x.so VARIANT_ENV=MEC_X=1 SHAPES="32 33 36" bash tools/gap_ab.sh
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-gapab}
SHAPES=${SHAPES:-32 33 36}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2; do for L in base variant; do for s in $SHAPES; do
  ( if [ $L = variant ]; then export MEMEC_LIBMEC=$PWD/$VARIANT; [ -n "${VARIANT_ENV:-}" ] && export "$VARIANT_ENV"; fi
    timeout -k 10 200 python3 -u tools/wide_ab.py --arms auto --shape $s --steps 30 --warmup 20 > $OUT/ab_${L}_${s}_$i.log 2>&1 ) || exit 1
done; done; done
for L in base variant; do
  ( if [ $L = variant ]; then export MEMEC_LIBMEC=$PWD/$VARIANT; [ -n "${VARIANT_ENV:-}" ] && export "$VARIANT_ENV"; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_$L -o run \
      -- python3 tools/wide_ab.py --arms auto --shape ${TRACE_SHAPE:-33} --steps 30 --warmup 20 > $OUT/trace_$L.log 2>&1 ) || exit 1
  d=$(dirname $(find $OUT/trace_$L -name run_kernel_trace.csv | head -n 1))
  python3 tools/trace_gaps.py $d > $OUT/gaps_$L.txt || exit 1
done
for L in base variant; do for s in $SHAPES; do echo "$L $s: $(grep -h '^{' $OUT/ab_${L}_${s}_*.log | python3 -c "import sys, json; print([json.loads(l)['auto']['frac'] for l in sys.stdin])")"; done; done
cat $OUT/gaps_*.txt

#!/usr/bin/env bash
# tools/server_pattern.sh — MemEC's server calling pattern on the GPU box:
# W worker threads sharing one Coding, single-stripe calls (SEAL encode of
# every parity, UPDATE delta encode, degraded-read decode), timed for
#   reference   MemEC's own plugin on the box's CPU (oracle/_ref/coding_bench_ref,
#               built in the build container from the reference sources)
#   staged      the drop-in adapter over libmec, chunks in malloc'd memory
#               (copied through mapped pinned staging), resident queue on
#   registered  the same on a registered ChunkPool-like slab (zero-copy)
# from the same tools/coding_bench.cc, one JSON line per run into
# gpurun_out/server_pattern.jsonl.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p "$OUT"
g++ -std=c++11 -O2 -Wall -Imemec_amd/csrc/coding -Iinclude tools/coding_bench.cc memec_amd/csrc/coding/*.cc \
    -Lmemec_amd -lmec -Wl,-rpath,"$PWD/memec_amd" -lpthread -o tools/coding_bench || exit 1
SECS=${SECS:-2}
J=${J:-$OUT/server_pattern.jsonl}
: > "$J"
for c in ${CFGS:-rs,4,2,4096 rs,8,2,4096 cauchy,4,2,4096 rs,10,4,65536}; do  # scheme,k,m,chunk
  cfg="$(echo $c | tr , ' ')"
  for mode in seal delta decode; do
    for w in ${WORKERS:-1 4 16}; do
      timeout -k 10 60 oracle/_ref/coding_bench_ref $cfg $w $SECS $mode >> "$J" || exit $?
      for reg in ${REGS:-0 1}; do
        for push in ${PUSHES:-0}; do  # MEC_QUEUE_PUSH arms (sources through the BAR, §4.5)
          MEC_QUEUE_PUSH=$push MEMEC_GPU_REGISTER=$reg timeout -k 10 60 tools/coding_bench $cfg $w $SECS $mode >> "$J" || exit $?
        done
      done
      tail -n 3 "$J"
    done
  done
done
echo "server pattern done"

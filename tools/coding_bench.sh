#!/usr/bin/env bash
# Build tools/coding_bench against the in-tree adapter + libmec and run the
# server calling patterns with and without coalescing (one GPU).
set -euo pipefail
cd "$(dirname "$0")/.."
g++ -std=c++11 -O2 -Wall -Imemec_amd/csrc/coding -Iinclude tools/coding_bench.cc memec_amd/csrc/coding/*.cc \
    -Lmemec_amd -lmec -Wl,-rpath,"$PWD/memec_amd" -lpthread -o tools/coding_bench
SECS=${SECS:-3}
for cfg in "rs 8 2 4096" "rs 10 4 65536" "cauchy 12 4 65536"; do
  for mode in seal delta decode; do
    for w in 1 16; do
      for co in 0 256; do
        for reg in ${REGISTER:-0 1}; do
          MEMEC_GPU_REGISTER=$reg MEMEC_GPU_COALESCE=$co timeout -k 10 120 tools/coding_bench $cfg $w $SECS $mode
        done
      done
    done
  done
done

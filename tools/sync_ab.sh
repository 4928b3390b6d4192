#!/usr/bin/env bash
# A/B: polling vs blocking waits for single-stripe host calls (server pattern).
cd "$(dirname "$0")/.."
g++ -std=c++11 -O2 -Imemec_amd/csrc/coding -Iinclude tools/coding_bench.cc memec_amd/csrc/coding/*.cc \
    -Lmemec_amd -lmec -Wl,-rpath,"$PWD/memec_amd" -lpthread -o tools/coding_bench || exit 1
for spin in 0 1; do
  for w in 1 16; do
    for cfg in "rs 8 2 4096" "rs 10 4 65536"; do
      for reg in 0 1; do
        MEC_SYNC_SPIN=$spin MEMEC_GPU_REGISTER=$reg MEMEC_GPU_COALESCE=0 timeout -k 10 60 tools/coding_bench $cfg $w 2 seal | sed "s/^{/{\"spin\": $spin, /"
      done
    done
  done
done

#!/usr/bin/env bash
# A/B: MEC_QUEUE_SOLO_MAX (lone calls on chunks above it take the launch
# path) for the 8 and 16 KiB shapes, registered and staged, 1/4/16 workers.
set -o pipefail
cd "$(dirname "$0")/.."
g++ -std=c++11 -O2 -Imemec_amd/csrc/coding -Iinclude tools/coding_bench.cc memec_amd/csrc/coding/*.cc \
    -Lmemec_amd -lmec -Wl,-rpath,"$PWD/memec_amd" -lpthread -o tools/coding_bench || exit 1
for reg in 1 0; do
for solo in 16384 4096; do
  for w in 1 2 4 16; do
    for cfg in "rs 10 4 16384 decode" "rs 10 4 16384 seal" "rs 8 2 8192 seal"; do
      set -- $cfg
      MEC_QUEUE_SOLO_MAX=$solo MEMEC_GPU_QUEUE=32 MEMEC_GPU_REGISTER=$reg timeout -k 10 60 tools/coding_bench $1 $2 $3 $4 $w 2 $5 | sed "s/^{/{\"solo\": $solo, /"
      rc=$?
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
done

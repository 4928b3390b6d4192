#!/usr/bin/env bash
# Device sweep (tools/perf_sweep.py) + single-stripe host calls through the
# C++ adapter, one worker (performance.cc's Kop/s, test_coding.sh's grid).
set -o pipefail
cd "$(dirname "$0")/.."
g++ -std=c++11 -O2 -Imemec_amd/csrc/coding -Iinclude tools/coding_bench.cc memec_amd/csrc/coding/*.cc \
    -Lmemec_amd -lmec -Wl,-rpath,"$PWD/memec_amd" -lpthread -o tools/coding_bench || exit 1
timeout -k 10 300 python -u tools/perf_sweep.py || exit $?
for fam in rs cauchy; do
  for k in 4 6 8 12; do
    for cs in 2048 4096 8192 16384 32768 65536 131072; do
      for reg in 0 1; do
        MEMEC_GPU_REGISTER=$reg timeout -k 10 30 tools/coding_bench $fam $k 2 $cs 1 0.5 seal | sed "s/^{/{\"registered_env\": $reg, /"
        rc=$?  # a rejected (family, chunk) is a normal exit; a crash or timeout ends the sweep
        case $rc in 124|134|137|139) exit $rc;; esac
      done
    done
  done
done

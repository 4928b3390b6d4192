#!/usr/bin/env bash
# A/B: resident submission queue (MEMEC_GPU_QUEUE=slots) vs per-call launches
# for the server's single-stripe calls through the C++ adapter, registered
# ChunkPool slab (zero-copy) or, with REGS=0, unregistered chunks (staged
# through mapped pinned lanes), 1, 4 and 16 workers.  QCFGS overrides the
# configurations ("family k m chunk op;..."), e.g. the Cauchy-RS rows:
#   QCFGS="cauchy 12 4 4096 seal;cauchy 12 4 16384 seal;cauchy 12 4 4096 decode;cauchy 12 4 16384 decode"
set -o pipefail
cd "$(dirname "$0")/.."
g++ -std=c++11 -O2 -Imemec_amd/csrc/coding -Iinclude tools/coding_bench.cc memec_amd/csrc/coding/*.cc \
    -Lmemec_amd -lmec -Wl,-rpath,"$PWD/memec_amd" -lpthread -o tools/coding_bench || exit 1
for reg in ${REGS:-1}; do
for q in 0 32; do
  for w in 1 4 16; do
    IFS=';' read -r -a CFGS <<< "${QCFGS:-rs 8 2 4096 seal;rs 10 4 65536 seal;rs 10 4 4096 delta;rs 10 4 16384 decode}"
    for cfg in "${CFGS[@]}"; do
      set -- $cfg
      MEMEC_GPU_QUEUE=$q MEMEC_GPU_REGISTER=$reg timeout -k 10 60 tools/coding_bench $1 $2 $3 $4 $w 2 $5 | sed "s/^{/{\"queue\": $q, /"
      rc=$?
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
done

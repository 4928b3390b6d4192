#!/usr/bin/env bash
# A/B for chunks above 16 KiB on the resident queue: per-call launches vs the
# queue with one workgroup per slot vs the queue with one workgroup per 16 KiB
# of chunk (multi-part slots), server calling pattern through the C++ adapter
# on a registered slab (tools/coding_bench.cc), 1 / 4 / 16 workers, 2 s each.
#   QCFGS="rs 10 4 65536 decode;..."  WORKERS="1 4 16"
set -o pipefail
cd "$(dirname "$0")/.."
g++ -std=c++11 -O2 -Imemec_amd/csrc/coding -Iinclude tools/coding_bench.cc memec_amd/csrc/coding/*.cc \
    -Lmemec_amd -lmec -Wl,-rpath,"$PWD/memec_amd" -lpthread -o tools/coding_bench || exit 1
IFS=';' read -r -a CFGS <<< "${QCFGS:-rs 10 4 16384 decode;rs 10 4 32768 decode;rs 10 4 65536 decode;rs 10 4 65536 delta;cauchy 12 4 16384 seal;cauchy 12 4 65536 seal}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  for w in ${WORKERS:-1 4 16}; do
    for arm in ${ARMS:-launch q1 qparts}; do
      case $arm in
        launch) env="MEMEC_GPU_QUEUE=0" ;;
        q1) env="MEMEC_GPU_QUEUE=32 MEC_QUEUE_MAX_CHUNK=${QMAX:-131072} MEC_QUEUE_PARTS=1" ;;
        qparts) env="MEMEC_GPU_QUEUE=32 MEC_QUEUE_MAX_CHUNK=${QMAX:-131072}" ;;
        qp256) env="MEMEC_GPU_QUEUE=32 MEC_QUEUE_MAX_CHUNK=${QMAX:-131072} MEC_QUEUE_PART_THREADS=256" ;;
        qp64) env="MEMEC_GPU_QUEUE=32 MEC_QUEUE_MAX_CHUNK=${QMAX:-131072} MEC_QUEUE_PART_THREADS=64" ;;
      esac
      env $env MEMEC_GPU_REGISTER=1 timeout -k 10 60 tools/coding_bench $1 $2 $3 $4 $w 2 $5 | sed "s/^{/{\"arm\": \"$arm\", /"
      rc=$?
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done

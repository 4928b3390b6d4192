#!/usr/bin/env bash
# A/B of the staging copy threads for unregistered host batches.
cd "$(dirname "$0")/.."
for t in 4 8 16; do
  echo "MEC_COPY_THREADS=$t"
  MEC_COPY_THREADS=$t timeout -k 10 200 python tools/bench_batch.py --only host_rs1m,host_rs4k
done

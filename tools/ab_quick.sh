#!/usr/bin/env bash
# Quick kernel check: GPU tests, MEC_BLOCK A/B (64 vs 256) on the main configs.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
AB_VAR=MEC_BLOCK AB_VALUES=256,64 timeout -k 10 300 python -u tools/win_ab.py rs_enc rs_dec crs_enc crs_dec rs8_small rs_update > gpurun_out/block_ab3.log 2>&1

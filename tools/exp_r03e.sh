# queue at the 1 MiB default cut: GPU queue/zero-copy/adapter tests, soak, and the small-Cauchy window A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_zerocopy.py tests/test_coding_adapter.py tests/test_memec_tree.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_queue_cut.log 2>&1 || exit $?
SOAK_SECONDS=8 SOAK_SHAPES=rs:10:4:65536,cauchy:12:4:65536,rs:6:3:1048576,cauchy:6:3:1048576 timeout -k 10 200 python -u tools/queue_soak.py > gpurun_out/queue_soak_cut.log 2>&1 || exit $?
bash tools/exp_r03d.sh

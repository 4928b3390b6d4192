# queue completion/poll fences: GPU queue tests, then launches vs queue
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_zerocopy.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_queue.log 2>&1 || exit $?
QCFGS="rs 8 2 4096 seal;rs 10 4 16384 decode;rs 10 4 65536 decode;rs 10 4 65536 delta;cauchy 12 4 16384 seal;cauchy 12 4 65536 seal" WORKERS="1 4 16" ARMS="launch q1 qparts" timeout -k 10 500 bash tools/queue_parts_ab.sh > gpurun_out/queue_fence_ab.log 2>&1

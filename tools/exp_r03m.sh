# queue part size after the fence fix: 1024-thread parts (default) vs 256-thread parts vs launches
set -o pipefail
cd $GRAFT_REPO_ROOT
QMAX=1048576 QCFGS="rs 8 2 4096 seal;rs 10 4 16384 decode;rs 10 4 65536 decode;cauchy 12 4 16384 seal;cauchy 12 4 65536 seal;rs 10 4 262144 decode" WORKERS="1 4 16" ARMS="launch qparts qp256" timeout -k 10 500 bash tools/queue_parts_ab.sh > gpurun_out/queue_pthr2_ab.log 2>&1

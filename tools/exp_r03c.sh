# queue: chunk cut above 64 KiB, then a soak over multi-part slots
set -o pipefail
cd $GRAFT_REPO_ROOT
QMAX=2097152 QCFGS="rs 10 4 131072 decode;rs 10 4 262144 decode;rs 10 4 1048576 decode;cauchy 12 4 131072 seal;cauchy 12 4 262144 seal;cauchy 12 4 1048576 seal" WORKERS="1 4 16" ARMS="launch qparts" timeout -k 10 400 bash tools/queue_parts_ab.sh > gpurun_out/queue_cut_ab.log 2>&1 || exit $?
SOAK_SECONDS=10 timeout -k 10 300 python -u tools/queue_soak.py > gpurun_out/queue_soak3.log 2>&1

set -o pipefail
cd $GRAFT_REPO_ROOT
QCFGS="rs 10 4 65536 decode;cauchy 12 4 65536 seal" WORKERS="1 4 16" ARMS="launch qparts qp256 qp64" timeout -k 10 300 bash tools/queue_parts_ab.sh > gpurun_out/queue_pthr_ab.log 2>&1 || exit $?
AB_CASES=cauchy:12:2,cauchy:8:2,rs:12:2 AB_SIZES=2048,4096,8192,16384 AB_OPS=enc_inplace,dec_inplace AB_ARMS="-:-:-:-,-:-:-:1,-:-:-:4,-:-:-:8,-:-:-:16,-:16,-:20,64:16" timeout -k 10 400 python tools/bm_small_ab.py > gpurun_out/small_win_ab.log 2>&1

set -u
TAG=r06g bash tools/gpu_session.sh e2e batch || exit $?
mkdir -p gpurun_out/r06g
CFGS="rs,8,2,4096 rs,10,4,16384 rs,10,4,65536 cauchy,12,4,16384 cauchy,12,4,65536" WORKERS="1 4 16" REGS="0 1" \
  J=gpurun_out/r06g/server_queue_table.jsonl timeout -k 10 500 bash tools/server_pattern.sh > gpurun_out/r06g/server_queue_table.log 2>&1 || exit $?
CFGS="rs,4,2,4096 rs,8,2,4096 cauchy,4,2,4096" WORKERS="1 16" REGS="1" PUSHES="0 4096" \
  J=gpurun_out/r06g/server_push.jsonl timeout -k 10 400 bash tools/server_pattern.sh > gpurun_out/r06g/server_push.log 2>&1 || exit $?
echo all done

# HEAD after the queue cut and tiny-Cauchy rule: full GPU suite, smoke, then the reference's sweep grid (device + single-stripe host calls)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_session.sh tests smoke || exit $?
timeout -k 10 600 bash tools/perf_sweep.sh > gpurun_out/perf_sweep_r03.jsonl 2> gpurun_out/perf_sweep_r03.err

# two 16-byte units per lane for in-place dense decodes (MEC_UPT=2): parity, then A/B on the bench's decode configs
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_launch_knobs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_upt.log 2>&1 || exit $?
ENV_ARMS='default:;u2:MEC_UPT=2;u2w8:MEC_UPT=2+MEC_WPC=8;u2w0:MEC_UPT=2+MEC_WPC=0' timeout -k 10 500 python -u tools/env_ab.py rs_dec rs_dec_mixed rs42_dec > gpurun_out/upt_ab.log 2>&1

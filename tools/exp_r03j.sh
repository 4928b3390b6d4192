# LDS-staged bitmatrix kernel: parity tests, then A/B against bm_kernel on small in-place stripes
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_launch_knobs.py tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bml.log 2>&1 || exit $?
AB_CASES=cauchy:12:2,cauchy:8:2,cauchy:6:2,cauchy:4:2,cauchy:12:4 AB_SIZES=1024,2048,4096,8192,16384 AB_OPS=enc_inplace,dec_inplace AB_ARMS="-:-:-:-:-,-:-:-:-:1,-:12:-:-:1,-:16:-:-:1" timeout -k 10 400 python tools/bm_small_ab.py > gpurun_out/bml_ab.log 2>&1

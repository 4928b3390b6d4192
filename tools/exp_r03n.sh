# rotated source order for strided bitmatrix launches: parity, no-regression build A/B, placement A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_launch_knobs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rot.log 2>&1 || exit $?
OLD=base CFGS="crs_enc crs_dec" ROUNDS=2 timeout -k 10 400 bash tools/lib_ab.sh > gpurun_out/lib_ab_rot.log 2>&1 || exit $?
PLACE_ARMS=default,rot timeout -k 10 400 python -u tools/place_ab.py 0,1,3,7,12 > gpurun_out/place_rot.log 2>&1

# final check of the split wave rules: parity suites, then new default vs the old count on the wide m = 4 shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_launch_knobs.py tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_enc_rule.log 2>&1 || exit $?
for shp in 16:4:262144:8 20:4:16384:8 24:4:65536:8 28:4:4096:8 10:4:1048576:12 12:4:65536:10; do
  IFS=: read k m c old <<< "$shp"
  ENC_SHAPES=$k:$m:$c ENC_ARMS=-,$old timeout -k 10 200 python -u tools/enc_cap_ab.py >> gpurun_out/enc_rule_ab2.log 2>&1 || exit $?
done

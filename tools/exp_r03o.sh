# the wide-stripe floor of the split encode rule: new default vs the old count (ceil_even(64/K+R)) per shape
set -o pipefail
cd $GRAFT_REPO_ROOT
for shp in 16:4:262144:8 20:4:16384:8 24:4:65536:8 28:4:4096:8 30:2:65536:6 22:2:16384:6 14:2:1048576:8 18:2:4096:8; do
  IFS=: read k m c old <<< "$shp"
  ENC_SHAPES=$k:$m:$c ENC_ARMS=-,$old timeout -k 10 200 python -u tools/enc_cap_ab.py >> gpurun_out/enc_rule_ab.log 2>&1 || exit $?
  ENC_FAMILY=isal_rs ENC_SHAPES=$k:$m:$c ENC_ARMS=-,$old timeout -k 10 200 python -u tools/enc_cap_ab.py >> gpurun_out/enc_rule_ab_isal.log 2>&1 || exit $?
done

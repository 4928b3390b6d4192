# small in-place Cauchy: identity order + one-wave blocks + split caps (MEC_WINDOWS=1) vs the default, 2 rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
AB_CASES=cauchy:4:2,cauchy:6:2,cauchy:8:2,cauchy:12:2,cauchy:12:4,cauchy:10:4 AB_SIZES=1024,2048,4096 AB_OPS=enc_inplace,dec_inplace AB_ARMS="-:-:-:-,-:-:-:1" timeout -k 10 300 python tools/bm_small_ab.py > gpurun_out/small_win1_ab_$r.log 2>&1 || exit $?
done

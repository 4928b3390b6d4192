# counters of a slow (3 GiB offset) and a fast (7 GiB) placement of the configs[4] decode
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_avail.txt 2>&1
for off in 3 7 3 7; do timeout -k 10 90 python tools/place_pmc.py $off 6 >> gpurun_out/place_plain.log 2>&1 || exit $?; done
for off in 3 7; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --output-format csv -d gpurun_out/place_tlb_$off -o run -- python3 tools/place_pmc.py $off 4 >> gpurun_out/place_pmc.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/place_tcc_$off -o run -- python3 tools/place_pmc.py $off 4 >> gpurun_out/place_pmc.log 2>&1 || exit $?
done

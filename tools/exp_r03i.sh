# memory-pipeline counters of five shapes (fast split encodes vs slow in-place launches)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
while read -r shape; do
  i=$((i+1))
  timeout -k 10 60 python tools/shape_pmc.py $shape >> gpurun_out/shape_plain.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/shape_a_$i -o run -- python3 tools/shape_pmc.py $shape >> gpurun_out/shape_pmc.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum --output-format csv -d gpurun_out/shape_b_$i -o run -- python3 tools/shape_pmc.py $shape >> gpurun_out/shape_pmc.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum --output-format csv -d gpurun_out/shape_c_$i -o run -- python3 tools/shape_pmc.py $shape >> gpurun_out/shape_pmc.log 2>&1 || exit $?
done <<'SHAPES'
rs 10 4 1048576 enc_split
rs 10 4 1048576 dec_inplace
rs 8 2 4096 enc_split
rs 12 2 4096 enc_inplace
cauchy 12 2 4096 enc_inplace
SHAPES

# code vs XOR-only twin at the memory side: split RS(10,4) encode (code beats its twin) and in-place decode (it does not)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
while read -r twin shape; do
  i=$((i+1))
  SHAPE_TWIN=$twin timeout -k 10 60 python tools/shape_pmc.py $shape 5 16 >> gpurun_out/twin_plain.log 2>&1 || exit $?
  SHAPE_TWIN=$twin timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/twin_a_$i -o run -- python3 tools/shape_pmc.py $shape 5 16 >> gpurun_out/twin_pmc.log 2>&1 || exit $?
  SHAPE_TWIN=$twin timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/twin_b_$i -o run -- python3 tools/shape_pmc.py $shape 5 16 >> gpurun_out/twin_pmc.log 2>&1 || exit $?
done <<'SHAPES'
0 rs 10 4 1048576 enc_split
1 rs 10 4 1048576 enc_split
0 rs 10 4 1048576 dec_inplace
1 rs 10 4 1048576 dec_inplace
SHAPES

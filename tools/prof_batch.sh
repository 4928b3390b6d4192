set -e
cd /root/repo && export TMPDIR=/tmp
for t in gather_rs1m_h256 gather_rs1m_h8 gather_rs4k_h256 gather_crs64k_h8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pb_$t -o run -- python3 tools/bench_batch.py --quick --only $t > gpurun_out/pb_$t.log 2>&1
done
echo done

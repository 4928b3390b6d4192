set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config rs42 > gpurun_out/bench_rs42_twin.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --config rs42_dec > gpurun_out/bench_rs42_dec.json 2>/dev/null || exit 1
for c in rs42 rs42_dec; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$c -o run -- python3 bench.py --config $c --no-cpu-baseline --no-secondary --no-ceiling --steps 5 --warmup 1 > /dev/null 2>&1 || exit 2
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$c -o run -- python3 bench.py --config $c --no-cpu-baseline --no-secondary --no-ceiling --steps 5 --warmup 1 > /dev/null 2>&1 || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rs42 -o run -- python3 bench.py --config rs42 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_rs42_under_rocprof.json 2>/dev/null || exit 4
echo ok

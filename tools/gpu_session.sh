#!/usr/bin/env bash
# tools/gpu_session.sh STEP... — run GPU steps on the MI355X box, each under
# its own time limit, stopping at the first fault/abort/timeout.
#   tests   pytest -m gpu          smoke   __graft_entry__.smoke()
#   bench   bench.py (default)     prof    rocprofv3 --kernel-trace --stats of bench
#   benchall  bench.py for every config (no cpu baseline)
#   batch   tools/bench_batch.py (pointer batches, coalescer)
#   pmc     rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench
#   sq      rocprofv3 --pmc SQ_* pass (VALU/SALU instruction mix, occupancy)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
TAG=${TAG:-r01}

run() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "=== $name: $*" | tee -a "$OUT/session.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a "$OUT/session.log"
    tail -n 25 "$OUT/$name.log"
    if grep -q "illegal memory access\|Memory access fault\|hipErrorIllegalAddress\|HSA_STATUS_ERROR" "$OUT/$name.log"; then
        echo "stopping: $name hit a GPU fault"; exit 3
    fi
    case $rc in
        0|1|5) return 0 ;;   # pass / test failures / no tests: not a GPU fault
        *) echo "stopping: $name rc=$rc"; exit $rc ;;
    esac
}

for step in "$@"; do
    case $step in
        tests) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
        testsel)  # TESTSEL=group,group,...; a group is file[::test]+file...; one process per group
            i=0
            for grp in $(echo "$TESTSEL" | tr ',' ' '); do
                i=$((i + 1))
                run "pytest_sel_$i" 600 python -u -m pytest $(echo "$grp" | tr '+' ' ') -m gpu -x -v --timeout 120 --timeout-method thread
            done ;;
        bounds)  # the bounds-checked build (make -C memec_amd bounds) under the index-heavy suites
            run pytest_bounds 900 env MEMEC_LIBMEC=memec_amd/bounds/libmec.so python -u -m pytest tests/test_gpu_wide.py \
                tests/test_gpu_batch.py tests/test_gpu_sweep.py tests/test_gpu_queue.py tests/test_gpu_launch_knobs.py \
                tests/test_gpu_zerocopy.py \
                -m gpu -x -q --timeout 120 --timeout-method thread ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 400 python bench.py ;;
        benchdec) run bench_rs_dec 400 python bench.py --config rs_dec ;;
        benchall)
            for c in rs_enc rs_dec rs_dec_mixed rs8_small crs_enc crs_dec rs42 rs42_dec rs_update rs8_update; do
                run "bench_$c" 300 python bench.py --config "$c" --no-cpu-baseline --no-extra-configs --steps 10
            done ;;
        cpu256) run bench_cpu256 400 python bench.py --cpu-threads 256 --no-extra-configs --no-secondary --steps 10 ;;
        batch) run bench_batch 600 python tools/bench_batch.py ${BATCH_ONLY:+--only $BATCH_ONLY} ;;
        e2e)  # host-memory (PCIe-inclusive) dense batches, pageable and registered, per config
            for c in ${E2E_CONFIGS:-rs_enc crs_enc rs8_small}; do
                run "bench_e2e_$c" 400 python bench.py --config $c --e2e --no-cpu-baseline --no-extra-configs --steps 5
                grep -h '^{' "$OUT/bench_e2e_$c.log" >> "$OUT/bench_e2e.jsonl"
            done ;;
        prof)
            for c in ${PROF_CONFIGS:-rs_enc}; do
                run "prof_$c" 400 rocprofv3 --kernel-trace --stats --output-format csv \
                    -d "$OUT/prof_$c" -o run -- python3 bench.py --config "$c" --no-cpu-baseline --no-extra-configs --steps 10
            done ;;
        pmc)
            for c in ${PROF_CONFIGS:-rs_enc}; do
                run "pmc_fetch_$c" 400 rocprofv3 --pmc FETCH_SIZE --output-format csv \
                    -d "$OUT/pmc_fetch_$c" -o run -- python3 bench.py --config "$c" --no-cpu-baseline --no-extra-configs --steps 5 --warmup 1
                run "pmc_write_$c" 400 rocprofv3 --pmc WRITE_SIZE --output-format csv \
                    -d "$OUT/pmc_write_$c" -o run -- python3 bench.py --config "$c" --no-cpu-baseline --no-extra-configs --steps 5 --warmup 1
            done ;;
        sq)
            for c in ${PROF_CONFIGS:-rs_enc}; do
                run "pmc_sq_$c" 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU \
                    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
                    --output-format csv -d "$OUT/pmc_sq_$c" -o run -- python3 bench.py --config "$c" --no-cpu-baseline --no-extra-configs --steps 3 --warmup 1
            done ;;
        sqlds)
            for c in ${PROF_CONFIGS:-rs_enc}; do
                run "pmc_sqlds_$c" 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
                    SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
                    --output-format csv -d "$OUT/pmc_sqlds_$c" -o run -- python3 bench.py --config "$c" --no-cpu-baseline --no-extra-configs --no-ceiling --steps 3 --warmup 1
            done ;;
        wide) run wide_ab 600 python tools/wide_ab.py --bytewise --arms bs,mg --steps 10 ;;
        server) run server_pattern 900 bash tools/server_pattern.sh ;;
        zc)  # zero-copy single-stripe decodes in place, every call's bytes checked (tools/zc_stress.py)
            for a in "rs 65536 0" "cauchy 65536 0" "rs 65536 8" "rs 4096 0"; do
                set -- $a
                run "zc_$1_$2_q$3" 300 python3 tools/zc_stress.py --fam $1 --cs $2 --queue $3 --iters ${ZC_ITERS:-3000}
                grep -h '^{' "$OUT/zc_$1_$2_q$3.log" >> "$OUT/zc_stress.jsonl"
            done ;;
        zcchurn)  # the zero-copy test's sequence on a fresh slab per iteration, beside other GPU work (tools/zc_churn.py)
            for bg in ${ZC_BG:-none all}; do
                for fam in ${ZC_FAMS:-rs cauchy}; do
                    it=${ZC_ITERS:-1500}
                    [ "$bg" = none ] || it=${ZC_ITERS_BG:-120}  # beside other GPU work a call waits for CUs
                    run "zcchurn_${fam}_$bg" 300 python3 -u tools/zc_churn.py --fam $fam --bg $bg --iters $it
                    grep -h '^{' "$OUT/zcchurn_${fam}_$bg.log" >> "$OUT/zc_churn.jsonl"
                done
            done ;;
        batch32)  # RS(8,2)@4 KiB strided vs pointer rows vs 32-bit slab offsets on the same chunks, interleaved (tools/wide_ab.py)
            for rnd in 1 2; do
                for i in ${B32_SHAPES:-32 33 36 34 35 37 18 17 38}; do
                    run "b32_${rnd}_$i" 300 python3 tools/wide_ab.py --arms auto --shape $i --steps 30 --warmup 20
                    grep -h '^{' "$OUT/b32_${rnd}_$i.log" >> "$OUT/batch32_ab.jsonl"
                done
            done ;;
        wcap)  # bit-sliced wave caps per shape: default vs forced 4 / 5 / 6 waves per CU, interleaved (tools/wide_ab.py)
            for i in ${WCAP_SHAPES:-6 20 4}; do
                run "wcap_$i" 400 python3 tools/wide_ab.py --arms ${WCAP_ARMS:-bs,bsw4,bsw5,bsw6,bs} --shape $i --steps 20 --warmup 20
                grep -h '^{' "$OUT/wcap_$i.log" >> "$OUT/wcap.jsonl"
            done ;;
        knobab)  # interleaved bench A/B of one knob (tools/knob_ab.sh): KNOB_VAR, KNOB_VALUES, KNOB_CONFIGS, KNOB_ROUNDS
            run "knobab_${KNOB_VAR}" 1000 env OUT="$OUT/knob_ab_${KNOB_VAR}.jsonl" bash tools/knob_ab.sh "$KNOB_VAR" \
                "$KNOB_VALUES" "$KNOB_CONFIGS" "${KNOB_ROUNDS:-2}" ;;
        profab)  # kernel-trace of tools/wide_ab.py shapes (PROFAB_SHAPES): per-launch kernel time vs the step's wall time
            for i in ${PROFAB_SHAPES:-32 33 36}; do
                run "profab_$i" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profab_$i" -o run \
                    -- python3 tools/wide_ab.py --arms auto --shape $i --steps 30 --warmup 20
            done ;;
        profcopy)  # kernel + memory-copy trace of tools/wide_ab.py shapes: the per-call table copies beside the launches
            for i in ${PROFAB_SHAPES:-33 35 37}; do
                run "profcopy_$i" 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
                    -d "$OUT/profcopy_$i" -o run -- python3 tools/wide_ab.py --arms auto --shape $i --steps 30 --warmup 20
            done ;;
        widefull)  # every byte-wise wide shape on the default arm (the rule as built), one process per shape
            for i in ${WIDE_ALL:-$(python3 -c "import sys; sys.path.insert(0, 'tools'); import wide_ab as w; print(' '.join(str(i) for i, s in enumerate(w.SHAPES) if s[0] != 'cauchy' and s[2] > 4))")}; do
                run "widefull_$i" 200 python3 tools/wide_ab.py --arms auto --shape $i --steps 20 --warmup 20
                grep -h '^{' "$OUT/widefull_$i.log" >> "$OUT/widefull.jsonl"
            done ;;
        tabwait)  # device batches: launch waits for its table copy on the device vs on the host while the stream is busy
            for i in ${TW_SHAPES:-33 35 36 37 17 38}; do
                run "tabwait_$i" 300 python3 tools/wide_ab.py --arms tw0,tw1,tw0,tw1 --shape $i --steps 30 --warmup 20
                grep -h '^{' "$OUT/tabwait_$i.log" >> "$OUT/tabwait.jsonl"
            done ;;
        tsan)  # host-TSan build (tools/tsan_build.sh, built beforehand): concurrent callers
            export TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 exitcode=0 suppressions=$PWD/tools/tsan_suppressions.txt"
            for c in rs,8,2,4096 cauchy,4,2,4096 rs,10,4,65536; do
                for mode in seal decode; do
                    for reg in 0 1; do
                        run "tsan_$(echo $c | tr , _)_${mode}_r$reg" 120 env MEMEC_GPU_REGISTER=$reg \
                            tools/coding_bench_tsan $(echo $c | tr , ' ') 16 1 $mode
                    done
                done
            done
            grep -c "WARNING: ThreadSanitizer" "$OUT"/tsan_*.log > "$OUT/tsan_counts.txt" || true ;;
        asan)  # host-ASan build (tools/asan_build.sh, built beforehand): the server pattern and queue calls
            export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
            for c in rs,8,2,4096 cauchy,4,2,4096 rs,10,4,65536 rs,6,3,20504; do
                for mode in seal delta decode; do
                    for w in 1 16; do
                        for reg in 0 1; do
                            run "asan_$(echo $c | tr , _)_${mode}_w${w}_r$reg" 90 env MEMEC_GPU_REGISTER=$reg \
                                tools/coding_bench_asan $(echo $c | tr , ' ') $w 1 $mode
                        done
                    done
                done
            done
            run asan_latency_rs 120 tools/queue_latency_asan rs 8 2 4096 3000 1 1
            run asan_latency_cauchy 120 tools/queue_latency_asan cauchy 4 2 4096 3000 0 2
            grep -l "ERROR: AddressSanitizer" "$OUT"/asan_*.log > "$OUT/asan_errors.txt" || true ;;
        latency)  # single-caller queue latency, traced (tools/queue_latency.hip, built here)
            /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude tools/queue_latency.hip -Lmemec_amd -lmec \
                -Wl,-rpath,"$PWD/memec_amd" -o tools/queue_latency || exit 1
            for env in ${LAT_ENVS:-MEC_QUEUE_TIMEOUT_MS=5000}; do  # ','-separated settings per run
                for a in ${LAT_ARGS:-rs,8,2,4096,20000,1,1 rs,8,2,4096,20000,0,1 rs,4,2,4096,20000,1,1 \
                         rs,10,4,65536,5000,1,1 cauchy,4,2,4096,20000,1,1 rs,8,2,4096,20000,1,2}; do
                    args="$(echo $a | tr , ' ')"
                    env=$(echo $env | tr , ' ')
                    tag="$(echo $env $args | tr ' =' '__')"
                    run "latency_$tag" 120 env $env tools/queue_latency $args
                    sed "s/^{/{\"env\": \"$env\", /" "$OUT/latency_$tag.log" | grep '^{' >> "$OUT/latency.jsonl"
                done
            done ;;
        widepmc)  # HBM traffic of one wide shape per kernel arm (WIDE_SHAPES, WIDE_ARMS)
            for sh in ${WIDE_SHAPES:-0 1}; do
                for arm in ${WIDE_ARMS:-bs mg}; do
                    for ctr in FETCH_SIZE WRITE_SIZE; do
                        run "pmc_wide_${sh}_${arm}_${ctr}" 300 rocprofv3 --pmc $ctr --output-format csv \
                            -d "$OUT/pmc_wide_${sh}_${arm}_${ctr}" -o run -- python3 tools/wide_ab.py --arms $arm --shape $sh --steps 5 --warmup 1
                    done
                done
            done ;;
        widesq)  # VALU issue and occupancy of one wide shape per kernel arm (WIDE_SHAPES, WIDE_ARMS)
            for sh in ${WIDE_SHAPES:-0}; do
                for arm in ${WIDE_ARMS:-bs mg}; do
                    run "pmc_widesq_${sh}_${arm}" 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
                        SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
                        --output-format csv -d "$OUT/pmc_widesq_${sh}_${arm}" -o run -- python3 tools/wide_ab.py --arms $arm --shape $sh --steps 3 --warmup 1
                done
            done ;;
        channels)  # per-TCC-instance EA counters (CH_KINDS of tools/channel_probe.py KINDS) of RS(10,4)@1 MiB arms, 4 a pass
            python3 tools/channel_probe.py --write-yaml "$OUT/ea_channels.yaml" || exit 1
            for arm in ${CH_ARMS:-enc_split dec_inplace dec_split}; do
                run "ch_plain_$arm" 120 python3 tools/channel_probe.py $arm 5
                for kind in ${CH_KINDS:-RD WR}; do
                    for q in 0 4 8 12; do
                        ctrs="MEC_EA_${kind}_CH$q MEC_EA_${kind}_CH$((q + 1)) MEC_EA_${kind}_CH$((q + 2)) MEC_EA_${kind}_CH$((q + 3))"
                        run "ch_${arm}_${kind}_$q" 120 timeout -s KILL 100 rocprofv3 -E "$OUT/ea_channels.yaml" --pmc $ctrs \
                            --output-format csv -d "$OUT/ch_${arm}_${kind}_$q" -o run -- python3 tools/channel_probe.py $arm 3
                    done
                done
            done ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "session done"

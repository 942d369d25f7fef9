#!/bin/bash
# One GPU session: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash, abort or timeout ends the script.
# Test failures (pytest rc 1) do not stop the bench.  Usage: tools/gpu_round.sh [tag] [steps...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
shift || true
STEPS=${*:-"smoke pytest bench prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # name seconds cmd...
    local name=$1 t=$2
    shift 2
    echo "== $name: $*"
    local t0=$(date +%s)
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc ($(( $(date +%s) - t0 ))s)"
    tail -n 15 "$OUT/$name.log"
    return $rc
}

fatal() {  # rc: anything but 0/1 (crash, abort, timeout) ends the session
    [ "$1" -ne 0 ] && [ "$1" -ne 1 ] && { echo "== stopping after rc=$1"; exit "$1"; }
    return 0
}

for s in $STEPS; do
    case $s in
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; [ $rc -ne 0 ] && exit $rc ;;
        pytest) run pytest_gpu 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread; fatal $? ;;
        pytestall) run pytest_gpu 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread; fatal $? ;;
        bench) run bench 300 python bench.py; fatal $? ;;
        benchcplx) run bench_cplx 300 python bench.py --workload cplx_i16 --cpu-seconds 5; fatal $? ;;
        bench2d) run bench_2d 300 python bench.py --workload fir2d_u8 --cpu-seconds 5; fatal $? ;;
        prof) run prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
                  python bench.py --steps 200 --warmup 100 --cpu-seconds 0 --no-parity --no-configs; fatal $? ;;
        pmc) for c in FETCH_SIZE WRITE_SIZE; do
                 run "pmc_$c" 300 rocprofv3 --pmc "$c" --kernel-trace -d "$OUT/pmc_$c" -o run --output-format csv -- \
                     python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity --no-configs --roofline-launches 5 \
                     --roofline-ramp 0; fatal $? || exit
             done ;;
        bench_*) wl=${s#bench_}
             run "bench_$wl" 300 python bench.py --workload "$wl" --cpu-seconds 5; fatal $? ;;
        prof_*) wl=${s#prof_}
             run "prof_$wl" 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$wl" -o run --output-format csv -- \
                 python bench.py --workload "$wl" --steps 200 --warmup 100 --cpu-seconds 0 --no-parity; fatal $? ;;
        pmc_*) wl=${s#pmc_}
             for c in FETCH_SIZE WRITE_SIZE; do
                 run "pmc_${wl}_$c" 300 rocprofv3 --pmc "$c" --kernel-trace -d "$OUT/pmc_${wl}_$c" -o run \
                     --output-format csv -- python bench.py --workload "$wl" --steps 10 --warmup 2 --cpu-seconds 0 \
                     --no-parity --roofline-launches 5 --roofline-ramp 0; fatal $? || exit
             done ;;
        pytestsub) run pytest_sub 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 \
                 --timeout-method thread ${PYTEST_FILES}; fatal $? ;;
        benchdrv) run bench_drv 300 python bench.py --gpus 1 --steps 20 --warmup 5; fatal $? ;;
        launch2|launch4) n=${s#launch}
             run "launch$n" 400 python bench.py --gpus "$n" --steps 20 --warmup 5; fatal $? ;;
        self_serial|self_overlap) m=${s#self_}
             run "self_$m" 300 env FIR_SELF_HALO=1 FIR_HALO=xgmi FIR_GATE_MODE=$m python bench.py --cpu-seconds 0; fatal $? ;;
        self_rccl) run self_rccl 300 env FIR_SELF_HALO=1 FIR_HALO=rccl python bench.py --cpu-seconds 0; fatal $? ;;
        profself_serial|profself_overlap) m=${s#profself_}
             run "profself_$m" 300 env FIR_SELF_HALO=1 FIR_HALO=xgmi FIR_GATE_MODE=$m rocprofv3 --kernel-trace --stats \
                 -d "$OUT/profself_$m" -o run --output-format csv -- python bench.py --steps 200 --warmup 100 \
                 --cpu-seconds 0 --no-parity; fatal $? ;;
        metab) run metab 300 python tools/metrics_ab.py warmup-fir-filter_amd/fir_hip/libfir_hip.so abrun/libfir_hip_old.so \
                 abrun/libfir_hip_oldnoasm.so abrun/libfir_hip_glds0.so abrun/libfir_hip_glds768.so abrun/libfir_hip_glds256.so; fatal $? ;;
        rowlat) run rowlat 300 python tools/row_call_latency.py "$OUT/row_call_latency.json"; fatal $? ;;
        ltr) run long_taps_rate 300 python tools/long_taps_rate.py 31,64,65,66,128,257,450,500,1000,2048,4099; fatal $? ;;
        sq_*) wl=${s#sq_}
             run "sq_$wl" 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace \
                 -d "$OUT/sq_$wl" -o run --output-format csv -- python bench.py --workload "$wl" --steps 10 \
                 --warmup 2 --cpu-seconds 0 --no-parity --roofline-launches 5 --roofline-ramp 0; fatal $? ;;
        dist2prof_serial|dist2prof_overlap) m=${s#dist2prof_}
             run "dist2prof_$m" 300 tools/dist2_prof.sh "$OUT/dist2prof_$m" "$m"; fatal $? ;;
        banknc) run banknc 200 python tools/lib_ab.py warmup-fir-filter_amd/fir_hip/libfir_hip.so \
                     abrun/libfir_hip_sk0.so 10 bank; fatal $? ;;
        bankab) for v in u2 xcd persist u2xcd; do
                 run "bankab_$v" 200 python tools/lib_ab.py warmup-fir-filter_amd/fir_hip/libfir_hip.so \
                     abrun/libfir_hip_bank_$v.so 10 bank; fatal $? || exit
             done ;;
        probe) run probe 200 python tools/pipeline_probe.py; fatal $? ;;
        profwl_*) wl=${s#profwl_}
             run "profwl_$wl" 300 rocprofv3 --kernel-trace --stats -d "$OUT/profwl_$wl" -o run --output-format csv -- \
                 python bench.py --workload "$wl" --steps 200 --warmup 100 --cpu-seconds 0 --no-parity; fatal $? ;;
        libab_*) wl=${s#libab_}
             run "libab_$wl" 200 python tools/lib_ab.py warmup-fir-filter_amd/fir_hip/libfir_hip.so ${AB_LIB} 10 "$wl"; fatal $? ;;
        ltab_*) kind=${s#ltab_}
             run "ltab_$kind" 400 python tools/long_taps_ab.py ${LT_TAPS:-66,128,257,450,900} \
                 warmup-fir-filter_amd/fir_hip/libfir_hip.so ${LT_LIBS} --kind "$kind"; fatal $? ;;
        ltab) run long_taps_ab 400 python tools/long_taps_ab.py 66,128,257,450,500,1000,4099 \
                 warmup-fir-filter_amd/fir_hip/libfir_hip.so abrun/libfir_hip_mr_v1.so abrun/libfir_hip_mr_d1.so \
                 abrun/libfir_hip_mr_d3.so abrun/libfir_hip_mr_t4w1d2.so abrun/libfir_hip_mr_old.so; fatal $? ;;
        metab2) run metab2 300 python tools/metrics_ab.py warmup-fir-filter_amd/fir_hip/libfir_hip.so abrun/libfir_hip_mleaf0.so \
                 abrun/libfir_hip_mleaf1024.so abrun/libfir_hip_mleaf256.so; fatal $? ;;
        ltab2) run long_taps_ab2 400 python tools/long_taps_ab.py 66,128,257,450,500,1000,4099 \
                 warmup-fir-filter_amd/fir_hip/libfir_hip.so abrun/libfir_hip_prev.so; fatal $? ;;
        metab3) run metab3 300 python tools/metrics_ab.py warmup-fir-filter_amd/fir_hip/libfir_hip.so abrun/libfir_hip_prev.so \
                 abrun/libfir_hip_met_ng1.so abrun/libfir_hip_met_b256.so abrun/libfir_hip_met_b256t4k.so \
                 abrun/libfir_hip_met_t1k.so; fatal $? ;;
        ltexp) run long_taps_exp 400 python tools/long_taps_ab.py 66,257,1000,4099 \
                 warmup-fir-filter_amd/fir_hip/libfir_hip.so abrun/libfir_hip_lt_e2.so --no-check; fatal $? ;;
        lth) run long_taps_head 400 python tools/long_taps_ab.py 66,128,257,450,500,1000,2048,4099 \
                 warmup-fir-filter_amd/fir_hip/libfir_hip.so abrun/libfir_hip_head.so; fatal $? ;;
        ltd) run long_taps_d 400 python tools/long_taps_ab.py 66,128,162,200,257,500,1000,4099 \
                 warmup-fir-filter_amd/fir_hip/libfir_hip.so abrun/libfir_hip_lt_x6.so abrun/libfir_hip_lt_x4.so; fatal $? ;;
        metp) run metp 300 python tools/metrics_ab.py warmup-fir-filter_amd/fir_hip/libfir_hip.so \
                 abrun/libfir_hip_met_p256.so abrun/libfir_hip_met_p1024.so abrun/libfir_hip_met_np.so \
                 abrun/libfir_hip_met_npb256t4k.so; fatal $? ;;
        metp2) run metp2 300 python tools/metrics_ab.py warmup-fir-filter_amd/fir_hip/libfir_hip.so \
                 abrun/libfir_hip_prevmet.so; fatal $? ;;
        metexp) run metexp 300 python tools/metrics_ab.py warmup-fir-filter_amd/fir_hip/libfir_hip.so \
                 abrun/libfir_hip_met_e1.so abrun/libfir_hip_met_e2.so abrun/libfir_hip_met_e3.so \
                 abrun/libfir_hip_met_b256t4k.so --no-check; fatal $? ;;
        ktrace_*) wl=${s#ktrace_}
             run "ktrace_$wl" 150 rocprofv3 --kernel-trace -d "$OUT/ktrace_$wl" -o run --output-format csv -- \
                 python bench.py --workload "$wl" --steps 20 --warmup 10 --cpu-seconds 0 --no-parity \
                 --roofline-launches 20 --roofline-ramp 10; fatal $? ;;
        sqlt_*) kind=${s#sqlt_}
              run "sq_lt257_$kind" 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                 SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VALU --kernel-trace -d "$OUT/sq_lt257_$kind" \
                 -o run --output-format csv -- python tools/long_taps_one.py 257 u8 6 "$kind"; fatal $? || exit
              run "sq_lt257b_$kind" 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS \
                 SQ_INSTS_MFMA --kernel-trace -d "$OUT/sq_lt257b_$kind" -o run --output-format csv -- \
                 python tools/long_taps_one.py 257 u8 6 "$kind"; fatal $? ;;
        sqlt) run sq_lt257 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                 SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VALU --kernel-trace -d "$OUT/sq_lt257" \
                 -o run --output-format csv -- python tools/long_taps_one.py 257 u8 6; fatal $?
              run sq_lt257b 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS \
                 SQ_INSTS_MFMA --kernel-trace -d "$OUT/sq_lt257b" -o run --output-format csv -- \
                 python tools/long_taps_one.py 257 u8 6; fatal $? ;;
        asan) run asan 600 make -C warmup-fir-filter_amd/csrc asan-check; fatal $? ;;
        asanbin) run asan 300 env LD_LIBRARY_PATH=tools/asan_bin ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 \
                 tools/asan_bin/capi_check; fatal $? ;;
        stagemicro) run stage_micro 200 tools/microbench/stage_micro 15; fatal $? ;;
        pipetime) run pipeline_timing 300 python tools/pipeline_timing.py; fatal $? ;;
        pipecold) run pipeline_timing_cold 300 python tools/pipeline_timing.py --cold; fatal $? ;;
        stagewall) run stage_wall 300 python tools/stage_wall_probe.py; fatal $? ;;
        stagewall1) run stage_wall_1reader 300 env FIR_STAGE_READERS=1 FIR_STAGE_READ_CHUNK=0 python tools/stage_wall_probe.py; fatal $? ;;
        bigstage) run big_stage 300 python tools/big_stage_probe.py 40; fatal $? ;;
        restoreprobe) run restore_probe 300 python tools/restore_stage_probe.py; fatal $? ;;
        reportprobe) run report_probe 300 python tools/report_stage_probe.py; fatal $? ;;
        micro) run micro 300 tools/microbench/fir_micro 28 20; fatal $? ;;
        micro2d) run micro2d 300 tools/microbench/fir2d_micro 15; fatal $? ;;
        microideal) run microideal 300 tools/microbench/ideal_micro 15; fatal $? ;;
        microread) run microread 300 tools/microbench/read_micro 15; fatal $? ;;
        microu8) run microu8 300 tools/microbench/fir_u8_micro 15; fatal $? ;;
        dist2|dist4) n=${s#dist}
             run "dist$n" 300 env FIR_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
                 --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus "$n" \
                 --steps 5 --warmup 2 --cpu-seconds 0 --log2n 24; fatal $? ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "== done"

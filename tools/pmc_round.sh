#!/bin/bash
# PMC HBM traffic of the bench's BASELINE workloads on THIS build, summarised on the box with the
# build id (tools/pmc_summary.py), so bench.py attaches the traffic only to runs of this build.
# Two separate passes per workload (FETCH_SIZE, WRITE_SIZE: the TCC block takes at most 4 counters
# per pass), each under its own time limit; any failure ends the script.
# Usage: tools/pmc_round.sh <tag> [workload ...]   -> gpurun_out/<tag>/pmc_<workload>.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}
shift
WLS=${*:-"fir1d_i16 cplx_i16 fir2d_u8 pipeline_fixed3"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# the dominant kernel of each workload (bench.KERNELS) and its algorithmic bytes per launch
declare -A KERN=([fir1d_i16]=fir1d_reg_kernel [cplx_i16]=fir1d_reg_kernel [fir2d_u8]=fir2d_pk16_strip_kernel
                 [pipeline_fixed3]=fir1d_reg_batch_kernel [fir1d_u8]=fir1d_reg_kernel [bank_u8]=fir1d_reg_kernel
                 [ideal_u8]=fir1d_ideal_reg_kernel [restore_u8]=restore_map_kernel [metrics_u8]=metrics_leaf_kernel)
declare -A ALG=([fir1d_i16]=1610612736 [cplx_i16]=1610612736 [fir2d_u8]=536870912 [pipeline_fixed3]=84969065
                [fir1d_u8]=536870912 [bank_u8]=1342177280 [ideal_u8]=2415919104 [restore_u8]=2415919104
                [metrics_u8]=2415919104)
for wl in $WLS; do
    for c in FETCH_SIZE WRITE_SIZE; do
        echo "== $wl $c"
        timeout -s KILL 120 rocprofv3 --pmc "$c" --kernel-trace -d "$OUT/pmc_${wl}_$c" -o run --output-format csv -- \
            python bench.py --workload "$wl" --steps 10 --warmup 2 --cpu-seconds 0 --no-parity \
            --roofline-launches 5 --roofline-ramp 0 > "$OUT/pmc_${wl}_$c.log" 2>&1 || { echo "pass failed"; exit 1; }
    done
    python tools/pmc_summary.py "$OUT" "${KERN[$wl]}" "${ALG[$wl]}" "$OUT/pmc_$wl.json" "pmc_${wl}_" || exit 1
done
echo "== done"

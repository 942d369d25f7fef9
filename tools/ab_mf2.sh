#!/bin/bash
# Dev A/B of the step-form MFMA kernel (fir1d_mfma_step_kernel): parity of the long-filter tests
# with the shipped build, then tools/long_taps_rate.py per build in abrun/ (make ab1dm AB=...).
# Usage (GPU box): bash tools/ab_mf2.sh "tile s2a3 ..." [taps]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V=${1:-"tile"}
TAPS=${2:-17,31,64}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fir1d.py -x -q --timeout 120 --timeout-method thread \
    -k 'long or mfma or many_taps' > gpurun_out/mf2_parity.txt 2>&1 || { tail -30 gpurun_out/mf2_parity.txt; exit 1; }
tail -2 gpurun_out/mf2_parity.txt
echo "== step (shipped)" | tee gpurun_out/mf2_rates.txt
timeout -k 10 150 python -u tools/long_taps_rate.py $TAPS 2>&1 | tee -a gpurun_out/mf2_rates.txt || exit 1
for v in $V; do
    echo "== $v" | tee -a gpurun_out/mf2_rates.txt
    FIR_HIP_LIB=$PWD/abrun/libfir_hip_$v.so timeout -k 10 150 python -u tools/long_taps_rate.py $TAPS 2>&1 | tee -a gpurun_out/mf2_rates.txt || exit 1
done

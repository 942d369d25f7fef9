#!/bin/bash
# Per-rank kernel traces of the N = 2 sharded step (BASELINE configs[3] shape, 2^28 int16 per rank)
# on a one-GPU box: the two ranks share the GPU (gloo process group, halos through the gate's
# IPC-mapped mailboxes), each rank under its OWN rocprofv3 with the program directly after `--`
# (bash starts both; nothing execs from a process that has touched the GPU).
# Usage: tools/dist2_prof.sh <out dir> <serial|overlap> [steps]
set -u
OUT=$1
MODE=$2
STEPS=${3:-200}
mkdir -p "$OUT"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29600 + RANDOM % 300)) WORLD_SIZE=2 \
       FIR_DIST_BACKEND=gloo FIR_GATE_MODE=$MODE HSA_ENABLE_IPC_MODE_LEGACY=0
pids=()
for r in 0 1; do
    RANK=$r LOCAL_RANK=$r timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/rank$r" -o run \
        --output-format csv -- python3 bench.py --gpus 2 --steps "$STEPS" --warmup 100 --cpu-seconds 0 \
        > "$OUT/rank$r.log" 2>&1 &
    pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
exit $rc

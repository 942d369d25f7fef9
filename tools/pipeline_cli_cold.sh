#!/bin/bash
# The pipeline program end to end in fresh processes (python start, imports, device start, every
# stage, 112 PNGs), alternating the side-thread device start on and off; wall seconds per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$(mktemp -d)
for i in 1 2 3; do
  for w in 1 0; do
    t0=$(date +%s.%N)
    FIR_PIPELINE_START_DEVICES=$w timeout -k 10 120 python warmup-fir-filter_amd/pipeline_fir_1d.py --tap all \
        --overwrite-vectors --overwrite-images --vector-dir "$T/vec" --image-out-dir "$T/img" > "$T/log" 2>&1 || { cat "$T/log"; exit 1; }
    t1=$(date +%s.%N)
    echo "start_devices=$w wall_s=$(awk -v a="$t0" -v b="$t1" "BEGIN{printf \"%.3f\", b - a}") $(tail -1 "$T/log" | grep -o "elapsed=[0-9.]*s")"
  done
done
rm -rf "$T"

# A/B of the RCCL halo path on one GPU (FIR_SELF_HALO=1: the segment is its own neighbour, a
# ring of one): RCCL's internal stream at high vs default priority.  The default N > 1 path
# (xGMI peer reads) needs no per-step message; this measures the FIR_HALO=rccl fallback.
# Usage: bash tools/selfhalo_ab.sh <tag>
set -u
OUT=gpurun_out/${1:-selfhalo}; mkdir -p $OUT; export TMPDIR=/tmp
for hp in 1 0; do
  FIR_NCCL_HIPRI=$hp FIR_SELF_HALO=1 timeout -k 10 200 python -u bench.py --cpu-seconds 0 > $OUT/hp$hp.log 2>&1 || exit $?
  grep '^{' $OUT/hp$hp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('hipri $hp', d['ms_per_step'], d['host_issue_us_per_step'], d['parity'])"
done

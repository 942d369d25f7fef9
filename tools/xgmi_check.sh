set -u
mkdir -p gpurun_out/s09; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_restore_sharded.py -x -q --timeout 200 --timeout-method thread -k "xgmi or rccl" > gpurun_out/s09/t.log 2>&1; rc=$?; tail -3 gpurun_out/s09/t.log; [ $rc -ne 0 ] && exit $rc
for n in 2 4; do
  FIR_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --steps 20 --warmup 5 --cpu-seconds 0 --log2n 26 > gpurun_out/s09/dist$n.log 2>&1 || exit $?
  grep '^{' gpurun_out/s09/dist$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['parity'], d['config']['parallelism'])"
done

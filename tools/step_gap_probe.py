"""Dev probe: where does the sharded step lose time on one GPU?  Times `steps` back-to-back
steps of several compositions around the 2^28-sample int16 bulk kernel (HIP events on the
compute stream, clocks warmed first):

  bulk          the bulk kernel alone
  segment       one launch of the FIR kernel that reads the halos itself (the xGMI step)
  bulk+edge     + the one-block edge kernel (halos from a resident tensor)
  bulk+wait+edge  + a stream wait on an event recorded (once) on another stream
  bulk+xchg+edge  + the RCCL ring-of-one exchange posted every step (fir_hip.sharded)
  xchg-side     the same, exchange posted from an idle side stream
  xchg-first    exchange posted and waited on before the bulk (no overlap, one wait per step)
  side-edge     exchange, wait and edge kernel all on the side stream (bulk alone on the compute stream)

Usage: python tools/step_gap_probe.py [steps] [variant,...]   (needs a GPU; one line per variant)
"""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import fir_hip  # noqa: E402
from fir_hip import sharded, torch_ops  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, pg_options=opts)
    stream = torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    taps = torch_ops.Taps([-256, -1024, 6656, -1024, -256])
    x = torch.from_numpy(np.random.default_rng(1).integers(-32768, 32768, 1 << 28, dtype=np.int16)).to(dev)
    y = torch.empty(x.shape, dtype=torch.int32, device=dev)
    hl = x[-2:].clone()
    hr = x[:2].clone()
    ex = sharded.HaloExchange(x, 5, 1, self_ring=True)
    ev = torch.cuda.Event()
    with torch.cuda.stream(side):
        ev.record()

    def bulk():
        torch_ops.fir1d_fixed_rows_dev(x, taps, 12, 32, fir_hip.OUT_I32, out=y)

    def edge(l, r):
        torch_ops.fir1d_fixed_edges_dev(x, taps, y, l, r, 12, 32, fir_hip.OUT_I32)

    def v_bulk():
        bulk()

    def v_edge():
        bulk()
        edge(hl, hr)

    def v_wait():
        bulk()
        stream.wait_event(ev)
        edge(hl, hr)

    def v_xchg():
        works = ex.post()
        bulk()
        sharded.wait_all(works)
        edge(*ex.halos())

    def v_side():
        with torch.cuda.stream(side):
            works = ex.post()
        bulk()
        sharded.wait_all(works)
        edge(*ex.halos())

    def v_side_edge():  # timing only: the edge kernel races the bulk's provisional edge outputs here
        with torch.cuda.stream(side):
            works = ex.post()
            sharded.wait_all(works)
            torch_ops.fir1d_fixed_edges_dev(x, taps, y, *ex.halos(), 12, 32, fir_hip.OUT_I32, stream=side)
        bulk()

    def v_segment():  # the xGMI step's launch: halos read by the FIR kernel itself (local tensors here)
        torch_ops.fir1d_fixed_segment_dev(x, taps, hl, hr, 12, 32, fir_hip.OUT_I32, out=y)

    def v_xchg_first():  # exchange first, its wait before the bulk, then bulk + edge back to back
        works = ex.post()
        sharded.wait_all(works)
        bulk()
        edge(*ex.halos())

    variants = [("segment", v_segment), ("xchg-first", v_xchg_first), ("side-edge", v_side_edge), ("bulk", v_bulk), ("bulk+edge", v_edge), ("bulk+wait+edge", v_wait), ("bulk+xchg+edge", v_xchg),
                ("xchg-side", v_side)]
    if len(sys.argv) > 2:  # a subset, e.g. for a trace
        variants = [v for v in variants if v[0] in sys.argv[2].split(",")]
    for _ in range(100):
        v_bulk()
    torch.cuda.synchronize()
    res = {n: [] for n, _ in variants}
    for rep in range(3):
        for name, fn in variants:
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / steps * 1e6)
    for name, _ in variants:
        print(f"{name:16s} {min(res[name]):8.1f} us/step (best of 3 x {steps})", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

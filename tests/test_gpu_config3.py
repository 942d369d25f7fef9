"""GPU: BASELINE configs[3] on the HIP path — 5-tap FIR-1D over 2^31 int16 samples sharded as
8 ranks x 2^28 samples, the (L-1)-sample halo handed over between neighbours every step.

On a one-GPU box the 8 ranks are 8 processes sharing it (a gloo group for the host-side
collectives); with several GPUs rank r runs on device r % device_count.  Each rank owns its own 2^28-sample segment (512 MiB in, 1 GiB out) in HBM, and
EVERY step changes every segment (``seg.add_``, a different amount per rank and step) before
filtering it, so a halo read that is not ordered against the neighbours' writes would show up:

* ``xgmi``: fir_hip.sharded.XgmiHalo — the halo gate (csrc/halo_gate.hip) hands the edges over
  through IPC-mapped mailboxes with device atomics, then ONE FIR launch reads them;
* ``xgmi_overlap``: the same gate on a high-priority side stream while the bulk kernel runs
  (XgmiHalo.gate_async / join), then the edge kernel (bench.py with FIR_GATE_MODE=overlap; serial is
  its default);
* ``rccl``: fir_hip.sharded.HaloExchange — the message path (on this box over gloo, staged
  through the host, since RCCL refuses several ranks on one GPU; across GPUs the same op list
  runs on RCCL), bulk kernel then edge kernel.

Checked bit-exactly against the C oracle (oracle/fir_oracle.c): every step's first and last 64
outputs of every rank (the halo-dependent ones plus their neighbours) with the neighbours'
samples OF THAT STEP, and the final step's full 2^28-sample output of every rank.  Taps: the
BASELINE sharpen filter and 32-bit-wrap taps (|acc| up to 5.4e9).
"""
from __future__ import annotations

import numpy as np
import pytest

WORLD = 8
LOG2N = 28  # samples per rank: 8 x 2^28 = 2^31 = BASELINE configs[3]
STEPS = 4
EDGE = 64
TAPS = ([-256, -1024, 6656, -1024, -256], [32767, -32768, 32767, -32768, 32767])


def _add(r: int, s: int) -> int:
    """What rank r's segment has gained after steps 0..s (step t adds (t + 1) * (r + 1))."""
    return sum((t + 1) * (r + 1) for t in range(s + 1))


def _wrap16(a: np.ndarray, c: int) -> np.ndarray:
    return ((a.astype(np.int64) + c) & 0xFFFF).astype(np.uint16).view(np.int16)


def _worker(rank, world, port, kind, log2n, q):
    import os
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "warmup-fir-filter_amd")]
    import torch
    import torch.distributed as dist

    import fir_hip as fh
    from fir_hip import sharded, torch_ops as to
    from oracle import c_oracle, fir_oracle as fo

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    msgs = []
    try:
        # one GPU per rank when the box has several (the xGMI path then runs across GPUs); on a
        # one-GPU box every rank shares device 0
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.set_stream(stream)
        n = 1 << log2n
        x0 = np.random.default_rng(20260227 + rank).integers(-32768, 32768, n, dtype=np.int16)
        edges = [None] * world  # every rank's first / last EDGE samples of x0
        dist.all_gather_object(edges, (x0[:EDGE].copy(), x0[n - EDGE:].copy()))
        seg = torch.empty(n, dtype=torch.int16, device=dev)
        y = torch.empty(n, dtype=torch.int32, device=dev)
        co = c_oracle()
        for taps in TAPS:
            hl, hr = sharded.halo_sizes(len(taps))
            seg.copy_(torch.from_numpy(x0))
            torch.cuda.synchronize()
            dist.barrier()
            if kind.startswith("xgmi"):
                got_kind, src = sharded.make_halo_source(seg, len(taps))
                if got_kind != "xgmi":
                    msgs.append(f"rank {rank}: halo source {got_kind}, expected xgmi")
            else:
                src = sharded.HaloExchange(seg, len(taps))
            recorded = []
            for step in range(STEPS):
                seg.add_((step + 1) * (rank + 1))  # every segment changes every step
                if kind == "xgmi":  # serial: the gate, then one launch reading its halos
                    src.gate()
                    left, right = src.halos()
                    to.fir1d_fixed_segment_dev(seg, taps, left, right, 12, 32, fh.OUT_I32, out=y)
                elif kind == "xgmi_overlap":  # the gate on its side stream || the bulk kernel, then edges
                    src.gate_async()
                    to.fir1d_fixed_rows_dev(seg, taps, 12, 32, fh.OUT_I32, out=y)
                    src.join()
                    left, right = src.halos()
                    to.fir1d_fixed_edges_dev(seg, taps, y, left, right, 12, 32, fh.OUT_I32)
                else:
                    works = src.post()
                    to.fir1d_fixed_rows_dev(seg, taps, 12, 32, fh.OUT_I32, out=y)
                    sharded.wait_all(works)
                    left, right = src.halos()
                    to.fir1d_fixed_edges_dev(seg, taps, y, left, right, 12, 32, fh.OUT_I32)
                recorded.append(torch.cat([y[:EDGE], y[n - EDGE:]]).clone())  # stream-ordered snapshot
            torch.cuda.synchronize()
            if kind.startswith("xgmi"):
                src.check()
            for s in range(STEPS):  # every step's halo-dependent outputs, with that step's neighbours
                own_head = _wrap16(x0[:EDGE + hr], _add(rank, s))
                own_tail = _wrap16(x0[n - EDGE - hl:], _add(rank, s))
                lh = _wrap16(edges[rank - 1][1][EDGE - hl:], _add(rank - 1, s)) if rank > 0 and hl else None
                rh = _wrap16(edges[rank + 1][0][:hr], _add(rank + 1, s)) if rank < world - 1 and hr else None
                want = np.concatenate([fo.fir1d_i16_i32(own_head, taps, halo_left=lh)[:EDGE],
                                       fo.fir1d_i16_i32(own_tail, taps, halo_right=rh)[hl:]])
                got = recorded[s].cpu().numpy()
                if not np.array_equal(got, want):
                    bad = np.flatnonzero(got != want)
                    msgs.append(f"rank {rank} taps {taps} step {s}: edge outputs {bad.tolist()[:8]} differ")
            s = STEPS - 1  # the final step's full segment
            xf = _wrap16(x0, _add(rank, s))
            lh = _wrap16(edges[rank - 1][1][EDGE - hl:], _add(rank - 1, s)) if rank > 0 and hl else None
            rh = _wrap16(edges[rank + 1][0][:hr], _add(rank + 1, s)) if rank < world - 1 and hr else None
            full = co.fir1d_rows(xf, taps, 12, 32, co.OUT_I32, halo_left=lh, halo_right=rh, nthreads=2)
            if not np.array_equal(y.cpu().numpy(), full):
                msgs.append(f"rank {rank} taps {taps}: full final output differs from the oracle")
            del xf, full
            dist.barrier()  # nobody unmaps or reuses its segment while a neighbour may read it
            if kind.startswith("xgmi"):
                src.close()
        q.put((rank, msgs))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, msgs + [f"rank {rank}: {type(e).__name__}: {e}"]))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["xgmi", "xgmi_overlap", "rccl"])
def test_config3_8_ranks_2p28_changing_segments(kind):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, kind, LOG2N, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(WORLD):
            rank, msgs = q.get(timeout=110)
            results[rank] = msgs
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    assert sorted(results) == list(range(WORLD)), results
    problems = [m for r in sorted(results) for m in results[r]]
    assert not problems, problems
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]

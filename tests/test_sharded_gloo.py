"""Multi-rank long-vector sharding on CPU with the gloo backend.

The halo exchange of fir_hip.sharded is the product code under test; the per-segment
compute is injected as the oracle (test infrastructure), so the check is: segments +
exchanged halos reproduce the unsharded filter bit for bit, for odd/even tap counts,
complex interleaving and uneven segment sizes.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N = 10_007


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, hq, channels, q):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "warmup-fir-filter_amd")]
    from fir_hip import sharded
    from oracle import fir_oracle as fo

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(99)
        x = rng.integers(-32768, 32768, N * channels, dtype=np.int16)
        lo, hi = sharded.segment_bounds(N, world, rank)
        seg = torch.from_numpy(x[lo * channels:hi * channels].copy())
        out = torch.zeros(seg.shape, dtype=torch.int32)

        def bulk(s, o):
            o.copy_(torch.from_numpy(fo.fir1d_i16_i32(s.numpy(), hq, channels=channels)))

        def edges(s, o, left, right):
            y = fo.fir1d_i16_i32(s.numpy(), hq, channels=channels,
                                 halo_left=None if left is None else left.numpy(),
                                 halo_right=None if right is None else right.numpy())
            hl, hr = sharded.halo_sizes(len(hq), channels)
            o[:hl] = torch.from_numpy(y[:hl])
            if hr:
                o[o.numel() - hr:] = torch.from_numpy(y[y.size - hr:])

        sharded.sharded_fir1d_step(seg, hq, out, channels=channels, bulk_fn=bulk, edge_fn=edges)
        parts = [None] * world
        dist.all_gather_object(parts, out.numpy())
        if rank == 0:
            full = fo.fir1d_i16_i32(x, hq, channels=channels)
            q.put(bool(np.array_equal(np.concatenate(parts), full)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,hq,channels", [
    (2, [-256, -1024, 6656, -1024, -256], 1),
    (2, [1024, 2048, 1024], 2),
    (3, [5, -7, 9, 11], 1),
    (4, [32767, -32768, 32767, -32768, 32767], 1),
    (2, [4096], 1),
    (8, [-256, -1024, 6656, -1024, -256], 1),  # the 8-rank layout of BASELINE configs[3]
    (8, [3, -5, 7, -11, 13, -11, 7, -5, 3], 2),
])
def test_sharded_halo_exchange_matches_unsharded(world, hq, channels):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, hq, channels, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_segment_bounds_cover_exactly():
    from fir_hip import sharded

    for n, w in ((10, 3), (2 ** 31, 8), (7, 7), (5, 2)):
        spans = [sharded.segment_bounds(n, w, r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def _exchange_worker(rank, world, port, taps, channels, self_ring, q):
    """HaloExchange built once and posted on several steps (the bench's step loop)."""
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "warmup-fir-filter_amd")]
    from fir_hip import sharded

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 37 * channels
        seg = torch.arange(rank * 1000, rank * 1000 + n, dtype=torch.int16)
        ex = sharded.HaloExchange(seg, taps, channels, self_ring=self_ring)
        hl, hr = sharded.halo_sizes(taps, channels)
        ok = True
        for step in range(3):
            seg.add_(1)  # new data each step: the send views must see it
            sharded.wait_all(ex.post())
            left, right = ex.halos()
            lrank = rank - 1 if rank > 0 else (rank if self_ring else None)
            rrank = rank + 1 if rank < world - 1 else (rank if self_ring else None)
            base = step + 1
            if hl:
                want_l = None if lrank is None else torch.arange(lrank * 1000 + n - hl, lrank * 1000 + n) + base
                ok &= (left is None) if want_l is None else bool(torch.equal(left.long(), want_l))
            if hr:
                want_r = None if rrank is None else torch.arange(rrank * 1000, rrank * 1000 + hr) + base
                ok &= (right is None) if want_r is None else bool(torch.equal(right.long(), want_r))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,taps,channels,self_ring", [  # self_ring (RCCL only): test_gpu_restore_sharded
    (3, 5, 1, False),
    (4, 4, 2, False),
    (2, 4, 1, False),
])
def test_halo_exchange_object_reposts_fresh_halos(world, taps, channels, self_ring):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, taps, channels, self_ring, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get(timeout=5) for _ in range(world))
    assert all(got.values()), got


def _fallback_worker(rank, world, port, q):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "warmup-fir-filter_amd")]
    from fir_hip import sharded

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seg = torch.arange(rank * 100, rank * 100 + 40, dtype=torch.int16)
        kind, src = sharded.make_halo_source(seg, 5)  # host tensors cannot be mapped: every rank -> rccl
        left, right = (None, None)
        sharded.wait_all(src.post())
        left, right = src.halos()
        ok = kind == "rccl" and isinstance(src, sharded.HaloExchange)
        # every rank carries the same reason: the first refusing rank and its error
        ok &= src.fallback_reason.startswith("rank 0: ") and "XgmiHalo needs a contiguous device segment" in src.fallback_reason
        if rank > 0:
            ok &= left.tolist() == list(range((rank - 1) * 100 + 38, (rank - 1) * 100 + 40))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_halo_source_falls_back_to_rccl_on_every_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fallback_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get(timeout=5) for _ in range(3))
    assert all(got.values()), got

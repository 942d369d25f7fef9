"""GPU: the restore-stage u8 conversions and the one-process multi-device
entry fir1d_fixed_rows_sharded, both through the C ABI.

Restore: bit-exact against the reference's own _to_u8_clip / _to_u8_normalized outputs
(tests/golden/restore_u8.npz, made by tests/golden/make_golden.py) and against the oracle
on large random arrays (ties at every x.5, both signs of zero, values far out of range).
Sharded: the box has one GPU, so shards go to repeated ids of device 0 (each shard is its
own H2D / kernel / D2H with the halo taken from the host buffer); results must equal the
unsharded call and the oracle for rows split and single-row segments, every tap count the
register kernel covers, complex channels, and more shards than rows or samples.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import fir_hip
from conftest import GOLDEN
from fir_hip import torch_ops
from oracle import c_oracle, fir_oracle as fo

DEV = torch.device("cuda", 0)


def test_restore_reference_outputs_bit_exact():
    d = np.load(GOLDEN / "restore_u8.npz")
    names = [k[:-4] for k in d.files if k.endswith("__in")]
    assert len(names) == 22
    for name in names:
        a = d[name + "__in"]
        assert np.array_equal(fir_hip.restore_u8(a, fir_hip.RESTORE_CLIP), d[name + "__clip"]), name
        assert np.array_equal(fir_hip.restore_u8(a, fir_hip.RESTORE_NORMALIZE), d[name + "__normalize"]), name


@pytest.mark.parametrize("n", [1, 7, 1023, 1024, 1025, 4096 * 3 + 5, (1 << 22) + 333])
def test_restore_random_vs_oracle(n):
    rng = np.random.default_rng(n)
    a = rng.uniform(-400.0, 700.0, n)
    a[rng.integers(0, n, max(1, n // 10))] = rng.integers(-5, 262, max(1, n // 10)) + 0.5  # ties
    a[: min(n, 2)] = [-0.0, 0.0][: min(n, 2)]
    assert np.array_equal(fir_hip.restore_u8(a, fir_hip.RESTORE_CLIP), fo.to_u8_clip(a))
    assert np.array_equal(fir_hip.restore_u8(a, fir_hip.RESTORE_NORMALIZE), fo.to_u8_normalized(a))


def test_restore_shapes_constant_and_empty():
    a = np.full((33, 65), -7.0)
    assert np.array_equal(fir_hip.restore_u8(a, fir_hip.RESTORE_NORMALIZE), np.zeros((33, 65), np.uint8))
    assert fir_hip.restore_u8(a).shape == (33, 65)
    assert fir_hip.restore_u8(np.zeros((0, 4))).shape == (0, 4)
    with pytest.raises(ValueError, match="zero-size"):
        fir_hip.restore_u8(np.zeros(0), fir_hip.RESTORE_NORMALIZE)


def test_restore_dev_on_ideal_outputs(images):
    co = c_oracle()
    x = images["case_000_img_001_1280x853_gray"]
    yi = co.fir1d_ideal_rows(x, [-1 / 16, -4 / 16, 26 / 16, -4 / 16, -1 / 16])
    t = torch.from_numpy(yi).cuda()
    for pol, ref in ((fir_hip.RESTORE_CLIP, fo.to_u8_clip), (fir_hip.RESTORE_NORMALIZE, fo.to_u8_normalized)):
        got = torch_ops.restore_u8_dev(t, pol)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy(), ref(yi))


SHARD_DEVS = [[0], [0, 0], [0, 0, 0], [0] * 7]


@pytest.mark.parametrize("devs", SHARD_DEVS)
@pytest.mark.parametrize("L", [1, 2, 3, 5, 9, 12])
def test_sharded_single_row_i16(devs, L):
    rng = np.random.default_rng(100 + L * 10 + len(devs))
    n = 100_003
    x = rng.integers(-32768, 32768, n, dtype=np.int16)
    hq = rng.integers(-20000, 20000, L)
    got = fir_hip.fir1d_fixed_rows_sharded(x, hq, 12, 32, fir_hip.OUT_I32, devices=devs)
    assert np.array_equal(got, fo.fir1d_i16_i32(x, hq, 12, 32))


@pytest.mark.parametrize("devs", SHARD_DEVS)
def test_sharded_complex_and_u8_rows(devs, images):
    rng = np.random.default_rng(7)
    xc = rng.integers(-32768, 32768, 2 * 50_001, dtype=np.int16)
    got = fir_hip.fir1d_fixed_rows_sharded(xc, [1024, 2048, 1024], 12, 32, fir_hip.OUT_I32, channels=2,
                                           devices=devs)
    assert np.array_equal(got, fo.fir1d_i16_i32(xc, [1024, 2048, 1024], 12, 32, channels=2))
    x = images["case_005_img_006_4499x2999_gray"]
    hq = fo.quantize_h([-1 / 16, -4 / 16, 26 / 16, -4 / 16, -1 / 16])
    got = fir_hip.fir1d_fixed_rows_sharded(x, hq, 12, 32, fir_hip.OUT_U8_SAT, devices=devs)
    assert np.array_equal(got, fir_hip.fir1d_fixed_rows(x, hq, 12, 32, fir_hip.OUT_U8_SAT))


def test_sharded_more_shards_than_work():
    x = np.arange(3 * 40, dtype=np.uint8).reshape(3, 40)
    got = fir_hip.fir1d_fixed_rows_sharded(x, [256, 1024, 1536, 1024, 256], devices=[0] * 5)
    assert np.array_equal(got, fo.fir1d_rows(x, [256, 1024, 1536, 1024, 256], 12, 32, fo.OUT_U8_SAT))
    x1 = np.arange(3, dtype=np.int16)
    got = fir_hip.fir1d_fixed_rows_sharded(x1, [3, -7, 11], 4, 32, fir_hip.OUT_I32, devices=[0] * 5)
    assert np.array_equal(got, fo.fir1d_i16_i32(x1, [3, -7, 11], 4, 32))


def test_sharded_bad_device_is_an_error():
    with pytest.raises(fir_hip.FirHipError, match="out of range"):
        fir_hip.fir1d_fixed_rows_sharded(np.zeros(64, np.uint8), [1, 2, 1], devices=[0, 99])


def test_rccl_halo_exchange_ring_of_one():
    """The RCCL halo exchange of fir_hip.sharded on the box's one GPU: a world of one whose
    segment is its own left and right neighbour (bench.py's FIR_SELF_HALO rehearsal).  The
    grouped send/recv must deliver the segment's last HL samples as the left halo and its
    first HR samples as the right halo on every repost, and the edge kernel fed with them
    must match the oracle with the same halos."""
    import socket

    import torch.distributed as dist
    from fir_hip import sharded

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        for taps, ch in (([-256, -1024, 6656, -1024, -256], 1), ([5, -7, 9, 11], 1), ([1024, 2048, 1024], 2)):
            hl, hr = sharded.halo_sizes(len(taps), ch)
            rng = np.random.default_rng(len(taps) * 10 + ch)
            x = torch.from_numpy(rng.integers(-32768, 32768, 4099 * ch, dtype=np.int16)).to(dev)
            y = torch.empty(x.shape, dtype=torch.int32, device=dev)
            ex = sharded.HaloExchange(x, len(taps), ch, self_ring=True)
            for step in range(3):
                x.add_(step + 1)
                works = ex.post()
                torch_ops.fir1d_fixed_rows_dev(x, taps, 12, 32, fir_hip.OUT_I32, ch, out=y)
                sharded.wait_all(works)
                left, right = ex.halos()
                torch_ops.fir1d_fixed_edges_dev(x, taps, y, left, right, 12, 32, fir_hip.OUT_I32, ch)
                torch.cuda.synchronize()
                xs = x.cpu().numpy()
                assert np.array_equal(left.cpu().numpy(), xs[xs.size - hl:]), (taps, step)
                if hr:
                    assert np.array_equal(right.cpu().numpy(), xs[:hr]), (taps, step)
                want = c_oracle().fir1d_rows(xs, taps, 12, 32, c_oracle().OUT_I32, channels=ch,
                                             halo_left=xs[xs.size - hl:], halo_right=xs[:hr] if hr else None)
                assert np.array_equal(y.cpu().numpy(), want), (taps, step)
    finally:
        dist.destroy_process_group()


def _xgmi_worker(rank, world, port, taps, ch, q):
    import os
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "warmup-fir-filter_amd")]
    import torch.distributed as dist

    import fir_hip as fh
    from fir_hip import sharded, torch_ops as to
    from oracle import c_oracle as co

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        n = 50_003 if world != 2 else 65_536  # 2 ranks: whole vectors, the one-launch kernel path
        x = np.random.default_rng(7).integers(-32768, 32768, n * ch, dtype=np.int16)
        lo, hi = sharded.segment_bounds(n, world, rank)
        seg = torch.from_numpy(x[lo * ch:hi * ch].copy()).to(dev)
        y = torch.empty(seg.shape, dtype=torch.int32, device=dev)
        y2 = torch.full(seg.shape, -7, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        dist.barrier()  # every segment resident before it is mapped
        kind, src = sharded.make_halo_source(seg, len(taps), ch)
        for step in range(3):  # every segment changes every step; the gate orders the hand-off
            seg.add_(step + 1)
            src.gate()
            to.fir1d_fixed_rows_dev(seg, taps, 12, 32, fh.OUT_I32, ch, out=y)
            to.fir1d_fixed_edges_dev(seg, taps, y, *src.halos(), 12, 32, fh.OUT_I32, ch)
            # the one-launch form reads the same received halos inside the register kernel
            to.fir1d_fixed_segment_dev(seg, taps, *src.halos(), 12, 32, fh.OUT_I32, ch, out=y2)
        torch.cuda.synchronize()
        src.check()
        parts = [None] * world
        dist.all_gather_object(parts, y.cpu().numpy())
        flags = [None] * world
        dist.all_gather_object(flags, bool(torch.equal(y, y2)))
        dist.barrier()  # nobody unmaps / frees before every rank is done reading
        src.close()
        if rank == 0:
            xf = (x.astype(np.int32) + 6).astype(np.int16)  # + 1 + 2 + 3, int16 wrap
            full = co().fir1d_rows(xf, taps, 12, 32, co().OUT_I32, channels=ch)
            q.put((kind, bool(np.array_equal(np.concatenate(parts), full)) and all(flags)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,taps,ch", [(2, [-256, -1024, 6656, -1024, -256], 1), (3, [5, -7, 9, 11], 1),
                                           (4, [1024, 2048, 1024], 2)])
def test_xgmi_peer_halos_across_processes(world, taps, ch):
    """fir_hip.sharded.XgmiHalo: ranks (processes) map their neighbours' mailboxes through the
    C ABI's IPC entries and the halo gate hands the edges over every step while every segment
    changes.  On the one-GPU box the ranks share device 0 (the same mapping and atomics path
    as across GPUs, minus the xGMI hop)."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_xgmi_worker, args=(r, world, port, taps, ch, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    kind, ok = q.get(timeout=5)
    assert kind == "xgmi" and ok


def _gate_buffers(hl_bytes, hr_bytes):
    mb = torch.empty(fir_hip.halo_mailbox_bytes(hl_bytes, hr_bytes), dtype=torch.uint8, device=DEV)
    return torch_ops.halo_mailbox_init_dev(mb, hl_bytes, hr_bytes)


def test_halo_gate_two_streams_and_timeout():
    """The gate kernel itself (csrc/halo_gate.hip) in one process: two 'ranks' whose gates run
    concurrently on two streams hand their edges over for several epochs (changing segments);
    a gate whose neighbour never publishes reports FIR_GATE_TIMEOUT and leaves zero halos."""
    hl, hr = 2, 2  # int16 samples of a 5-tap filter
    hlb, hrb = 2 * hl, 2 * hr
    mb_a, mb_b = _gate_buffers(hlb, hrb), _gate_buffers(hlb, hrb)
    a = torch.arange(1000, dtype=torch.int16, device=DEV)
    b = torch.arange(5000, 6000, dtype=torch.int16, device=DEV)
    la = torch.empty(hl, dtype=torch.int16, device=DEV)  # a's left halo = b's tail (b sits left of a)
    rb = torch.empty(hr, dtype=torch.int16, device=DEV)  # b's right halo = a's head
    st_a = torch.full((1,), -1, dtype=torch.int32, device=DEV)
    st_b = torch.full((1,), -1, dtype=torch.int32, device=DEV)
    # the two gates wait on each other, so they must run at the same time: two streams of one
    # priority may share a hardware queue (GPU_MAX_HW_QUEUES, after the streams other tests made),
    # where the second gate would queue behind the first until it times out (seen once in a
    # subset run); a high-priority stream is served by a queue of its own priority
    s1, s2 = torch.cuda.Stream(device=DEV), torch.cuda.Stream(device=DEV, priority=-1)
    torch.cuda.synchronize()
    for step in range(5):
        a.add_(step + 1)
        b.sub_(step + 3)
        torch.cuda.synchronize()
        torch_ops.halo_gate_dev(a, hlb, hrb, mb_a, mb_b.data_ptr(), None, la, None, st_a, 5.0, stream=s1)
        torch_ops.halo_gate_dev(b, hlb, hrb, mb_b, None, mb_a.data_ptr(), None, rb, st_b, 5.0, stream=s2)
        torch.cuda.synchronize()
        assert st_a.item() == 0 and st_b.item() == 0, step
        assert torch.equal(la, b[-hl:]) and torch.equal(rb, a[:hr]), step
    # a neighbour that never publishes: bounded wait, reported, zero halos
    lone = _gate_buffers(hlb, hrb)
    never = _gate_buffers(hlb, hrb)
    la.fill_(7)
    torch_ops.halo_gate_dev(a, hlb, hrb, lone, never.data_ptr(), None, la, None, st_a, 0.05)
    torch.cuda.synchronize()
    assert st_a.item() == fir_hip.GATE_TIMEOUT
    assert int(la.abs().sum()) == 0


def test_peer_access_check():
    """The guard XgmiHalo runs before any kernel reads a neighbour: this GPU can read itself,
    and a bus id no visible GPU has is refused (that rank then takes the RCCL path)."""
    import fir_hip as fh

    bus = fh.device_bus_id(0)
    assert len(bus) >= 7 and ":" in bus
    assert fh.peer_access(0, bus)
    assert not fh.peer_access(0, "0000:ff:1f.7")
    for d in range(fh.device_count()):
        other = fh.device_bus_id(d)
        assert fh.peer_access(0, other) in (True, False)


@pytest.mark.parametrize("dtype,ch,stage", [(np.int16, 1, 1), (np.int16, 2, 1), (np.int16, 1, 0), (np.uint8, 1, 0),
                                            (np.uint8, 1, 1)])
@pytest.mark.parametrize("n", [8, 16, 4096, 4099, 1 << 20, (1 << 20) + 16, 3])
def test_segment_with_halos_matches_oracle(dtype, ch, stage, n):
    """fir1d_fixed_segment_dev: the register kernel with the halos in place of the zero padding
    (n*ch a whole number of vectors) or rows + edge kernels (otherwise), every tap count 1..9
    and a 12-tap generic case, one-sided and absent halos."""
    rng = np.random.default_rng(n + ch)
    lo, hi = (0, 256) if dtype == np.uint8 else (-32768, 32768)
    x = rng.integers(lo, hi, n * ch, dtype=dtype)
    xd = torch.from_numpy(x).to(DEV)
    for L in list(range(1, 10)) + [12]:
        hq = rng.integers(-3000, 3000, L) if dtype == np.int16 else rng.integers(-300, 900, L)
        hl_n, hr_n = (L - 1 - L // 2) * ch, (L // 2) * ch
        hlv = rng.integers(lo, hi, hl_n, dtype=dtype)
        hrv = rng.integers(lo, hi, hr_n, dtype=dtype)
        for use_l, use_r in ((True, True), (False, True), (True, False), (False, False)):
            left = torch.from_numpy(hlv).to(DEV) if use_l and hl_n else None
            right = torch.from_numpy(hrv).to(DEV) if use_r and hr_n else None
            y = torch_ops.fir1d_fixed_segment_dev(xd, hq, left, right, 12, 32, stage, ch)
            want = c_oracle().fir1d_rows(x, hq, 12, 32, stage, channels=ch,
                                         halo_left=hlv if left is not None else None,
                                         halo_right=hrv if right is not None else None)
            assert np.array_equal(y.cpu().numpy(), want), (L, use_l, use_r)

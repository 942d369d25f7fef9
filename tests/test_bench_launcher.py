"""bench.py's N > 1 self-launch (CPU, no GPU): `python bench.py --gpus N` started directly
spawns N ranks under torch.distributed.run as a child process, forwards rank 0's ONE JSON line
and exits with the ranks' status.  A stub rank script (gloo, CPU only) stands in for the GPU
workload; the launcher function is bench.launch_ranks itself."""
from __future__ import annotations

import json
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

STUB = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)   # the bench's max-over-ranks timing
    print(f"rank {rank} noise on stdout")      # not a result line: goes to stderr
    if rank == 0:   # bench.emit_result's protocol
        line = json.dumps({"metric": "stub", "value": float(t.item()), "n_gpus": world,
                           "argv": sys.argv[1:], "backend": os.environ.get("FIR_DIST_BACKEND")})
        open(os.environ["FIR_BENCH_RESULT"], "w").write(line + "\\n")
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(int(os.environ.get("STUB_EXIT_RANK", "-1")) == rank)
""")


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, str(ROOT))
    import bench as b

    return b


def _run(bench, tmp_path, n, env_extra=None, capsys=None):
    stub = tmp_path / "stub_rank.py"
    stub.write_text(STUB)
    import os

    env = dict(os.environ, FIR_DIST_BACKEND="gloo", **(env_extra or {}))
    return bench.launch_ranks(n, str(stub), ["--gpus", str(n), "--steps", "3"], env)


@pytest.mark.parametrize("n", [2, 3])
def test_launch_ranks_forwards_rank0_line(bench, tmp_path, capfd, n):
    rc = _run(bench, tmp_path, n)
    out, err = capfd.readouterr()
    assert rc == 0
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out  # exactly one JSON line on stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["value"] == float(n)  # the all-reduce saw every rank
    assert rec["argv"] == ["--gpus", str(n), "--steps", "3"]
    assert "rank 0 noise on stdout" in err and "rank 1 noise on stdout" in err  # ranks' stdout -> stderr


def test_launch_ranks_fails_when_a_rank_fails(bench, tmp_path, capfd):
    rc = _run(bench, tmp_path, 2, {"STUB_EXIT_RANK": "1"})
    capfd.readouterr()
    assert rc != 0


def test_bench_main_self_launches_before_any_gpu_call(bench, monkeypatch):
    """`--gpus 2` without WORLD_SIZE goes to launch_ranks with the same argv, choosing the gloo
    rehearsal when the host has fewer GPUs than ranks (here: none)."""
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("FIR_DIST_BACKEND", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "7", "--warmup", "1"])
    monkeypatch.setattr(bench, "launch_ranks", lambda n, script, argv, env: calls.append((n, script, argv, env)) or 0)
    assert bench.main() == 0
    (n, script, argv, env), = calls
    assert n == 2 and Path(script).name == "bench.py"
    assert argv == ["--gpus", "2", "--steps", "7", "--warmup", "1"]
    assert env["FIR_DIST_BACKEND"] == "gloo" and "2 ranks" in env["FIR_BENCH_REHEARSAL"]


def test_bench_rejects_world_mismatch(bench, monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "3")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit, match="WORLD_SIZE=3"):
        bench.main()


def test_bench_script_runs_launcher_end_to_end(tmp_path):
    """The real entry: `python bench.py --gpus 2` on a host without GPUs spawns 2 ranks; each
    fails at its first GPU call (no device here), so the parent exits non-zero and prints no
    result line — the launcher neither hangs nor claims a result."""
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--cpu-seconds", "0"], capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert p.stdout == ""


def _halo_report_worker(rank, world, port, q):
    import os
    import sys

    sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]
    import torch
    import torch.distributed as dist

    import bench as b
    from fir_hip import sharded

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seg = torch.arange(rank * 100, rank * 100 + 40, dtype=torch.int16)

        class WL:  # the fields halo_report / gate_failures read
            pass

        wl = WL()
        wl.halo_kind, wl.halo_src = sharded.make_halo_source(seg, 5)  # CPU tensors: RCCL path, with a reason
        info = b.halo_report(wl, world, dist.barrier, torch.device("cpu"), n=5)

        class StuckGate(sharded.XgmiHalo):  # a gate whose status word says "timed out" on rank 1
            def __init__(self):
                self.status = torch.tensor([1 if rank == 1 else 0], dtype=torch.int32)
                self.timeout_s = 10.0

        wl.halo_src = StuckGate()
        failed = b.gate_failures(wl, world, torch.device("cpu"))
        ranks = b.gather_floats(float(rank) + 0.5, world, torch.device("cpu"))
        q.put((rank, info, failed, ranks))
    finally:
        dist.destroy_process_group()


def test_halo_report_and_gate_failures_over_gloo():
    """The N > 1 bench line explains itself: config.halo names the source, why RCCL was chosen and
    the hand-off's own per-step cost (max / min over ranks); a timed-out gate on any rank is seen
    by every rank (the run then ends with a line and status 3, not a hang)."""
    import multiprocessing as mp
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_halo_report_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict((r, (i, f, k)) for r, i, f, k in (q.get(timeout=5) for _ in range(2)))
    for r in (0, 1):
        info, failed, ranks = got[r]
        assert info["source"] == "rccl"
        assert info["fallback_reason"].startswith("rank 0: ")
        assert set(info["exchange_us_per_step"]) == {"max", "min", "timing"}
        assert info["exchange_us_per_step"]["max"] >= info["exchange_us_per_step"]["min"] > 0
        assert failed == [1]
        assert ranks == [0.5, 1.5]


def _legs_worker(rank, world, port, q):
    """bench.halo_leg / run_halo_legs over gloo with the GPU parts stubbed: the xGMI leg's gate
    times out on rank 1 (an injected status word), the RCCL leg runs the real send/recv exchange."""
    import os
    import sys
    import types

    sys.path[:0] = [str(ROOT), str(ROOT / "warmup-fir-filter_amd")]
    import torch
    import torch.distributed as dist

    import bench as b
    from fir_hip import sharded

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        class StuckGate(sharded.XgmiHalo):  # mapped and probed fine, but a later gate times out on rank 1
            def __init__(self):
                self.status = torch.tensor([1 if rank == 1 else 0], dtype=torch.int32)
                self.timeout_s = 10.0
                self.closed = False

            def gate(self, stream=None):
                pass

            def close(self):
                self.closed = True

        stuck = StuckGate()
        real = sharded.make_halo_source
        sharded.make_halo_source = lambda *a, **k: ("xgmi", stuck) if k.get("prefer") == "xgmi" else real(*a, **k)
        b.measure = lambda wl, *a, **k: (0.01, 0.001, 1e-4)  # the GPU timing loops

        class WL:  # the fields halo_leg reads
            x = torch.arange(rank * 100, rank * 100 + 40, dtype=torch.int16)
            taps = types.SimpleNamespace(n=5)
            channels, units, unit, config = 1, 40, "Gsamples/s", {}
            halo_kind = halo_src = None

            def set_halo(self, kind, src):
                self.halo_kind, self.halo_src = kind, src
                self.config["parallelism"] = kind

            def oracle(self, nthreads):
                return None

            def matches(self, ref):
                return True

        args = types.SimpleNamespace(steps=10, warmup=0, roofline_ramp=0, roofline_launches=1)
        wl = WL()
        legs, head = b.run_halo_legs(["xgmi", "rccl"],
                                     lambda k: b.halo_leg(wl, k, args, world, dist.barrier, torch.device("cpu")))
        q.put((rank, legs, head, stuck.closed))
    finally:
        dist.destroy_process_group()


def test_gate_failure_leaves_the_rccl_leg_reported_over_gloo():
    """At N > 1 the bench times both halo sources; an xGMI gate that times out on one rank marks
    only that leg failed (its error names the rank) and the RCCL leg still yields the run's
    value, with bit-exact parity, so the first real multi-GPU run has a number either way."""
    import multiprocessing as mp
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_legs_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict((r, (legs, head, closed)) for r, legs, head, closed in (q.get(timeout=5) for _ in range(2)))
    for r in (0, 1):
        legs, head, closed = got[r]
        assert head == "rccl" and closed
        assert "timed out" in legs["xgmi"]["error"] and "[1]" in legs["xgmi"]["error"]
        rccl = legs["rccl"]
        assert rccl["value"] == round(80 * 10 / 0.01 / 1e9, 3) and rccl["parity"].startswith("bit-exact")
        assert rccl["halo"]["source"] == "rccl" and rccl["halo"]["exchange_us_per_step"]["max"] > 0


def test_run_halo_legs_headline_order():
    import bench as b

    def one(kind):
        if kind == "xgmi":
            raise b.LegFailed("xGMI halo path unavailable: rank 0: no peer access")
        return {"value": 1.0, "parity": "bit-exact"}

    legs, head = b.run_halo_legs(["xgmi", "rccl"], one)
    assert head == "rccl" and legs["xgmi"] == {"error": "xGMI halo path unavailable: rank 0: no peer access"}
    legs, head = b.run_halo_legs(["xgmi", "rccl"], lambda k: {"value": 2.0, "parity": "MISMATCH"})
    assert head is None
    legs, head = b.run_halo_legs(["xgmi", "rccl"], lambda k: {"value": 3.0, "parity": "bit-exact"})
    assert head == "xgmi"


def test_pmc_traffic_only_for_the_running_build(tmp_path):
    """roofline.traffic comes from a committed PMC summary only when that summary was taken on the
    build that is running (build_id == fir_build_id()) at this workload's size; a summary of
    another build, an old one without an id, or another size gives null."""
    import json
    import types

    import bench as b
    import fir_hip

    wl = types.SimpleNamespace(name="fir1d_i16", gen2d=False, alg_bytes=1610612736)
    (tmp_path / "profiles").mkdir()
    path = tmp_path / "profiles" / "pmc_fir1d_i16.json"
    assert b.pmc_traffic(wl, tmp_path) is None  # no summary
    base = {"algorithmic_bytes_per_launch": wl.alg_bytes, "hbm_bytes_per_launch": 1644000000}
    path.write_text(json.dumps(dict(base, build_id=fir_hip.build_id())))
    assert b.pmc_traffic(wl, tmp_path) == 1644000000
    path.write_text(json.dumps(dict(base, build_id="0" * 32)))
    assert b.pmc_traffic(wl, tmp_path) is None  # another build
    path.write_text(json.dumps(base))
    assert b.pmc_traffic(wl, tmp_path) is None  # no build id: taken before round 6
    path.write_text(json.dumps(dict(base, build_id=fir_hip.build_id(), algorithmic_bytes_per_launch=5)))
    assert b.pmc_traffic(wl, tmp_path) is None  # another size

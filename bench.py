#!/usr/bin/env python3
"""bench.py — Gsamples/s + %HBM roofline of the MI355X fixed-point FIR hot path.

Default workload (BASELINE.json configs[1]; configs[3] at --gpus 8): 5-tap int16 -> int32
FIR-1D (Q4.12 "sharpen" taps [-256,-1024,6656,-1024,-256], 32-bit wrap, round, no
saturation) over 2^28 synthetic samples PER GPU (weak scaling: 2^31 samples on 8 GPUs),
inputs resident in HBM before the timed region.  For N > 1 each rank owns one contiguous
segment; a step is a one-wave gate kernel that hands the 2+2-sample halo over through the
neighbours' HBM over xGMI, ordered per step (device atomics on mailboxes mapped once), then ONE
launch of the FIR kernel reading it (FIR_GATE_MODE=overlap: the gate beside the bulk kernel, then
an edge kernel; FIR_HALO=rccl: RCCL send/recv every step, overlapped with the bulk kernel, then an
edge kernel).

Contract: `python bench.py --gpus N --steps K --warmup W`; rank 0 prints ONE JSON line.  For
N > 1 either launch it under torch.distributed.run (RANK/WORLD_SIZE set), or run it as is: the
parent then starts `torch.distributed.run --nproc-per-node N` as a child process before any GPU
call of its own, forwards rank 0's JSON line and exits with the children's status.  A box with
fewer GPUs than ranks rehearses over gloo (ranks share devices; config.rehearsal says so).
Extra keys:
  roofline      dominant kernel's algorithmic bytes / its mean duration (HIP events on the
                stream it runs on: 100 untimed ramp launches and >= 50 ms of them, then 200 timed back to back,
                whatever --steps/--warmup are), vs the 8.0 TB/s HBM3E peak; `traffic` = PMC
                HBM bytes per launch from the committed rocprofv3 summary in profiles/, null if
                absent or taken on another build (its build_id must equal fir_build_id())
  cpu_baseline  the C oracle (oracle/fir_oracle.c, OpenMP) on this host's cores, same input;
                timed by rank 0 at every N, after the GPU legs, while the other ranks wait
  parity        every rank's full output compared bit-exactly with the C oracle
  cpu_baseline_numpy  the vectorised NumPy restatement (oracle/fir_oracle.py, one core) on a
                bounded leading slice of the same input (BASELINE.md's "NumPy CPU path")
  cpu_baseline_numpy_threads  the same NumPy path over contiguous slices on a thread pool of
                the host's cores (core count in `cores`)
  cpu_baseline_python_loop  the reference's own per-sample Python loop (restated in
                oracle.fir1d_loop) on 2^16 samples: what its CPU path costs (1-D workloads)
  host_issue_us_per_step  host time to enqueue one timed step (diagnostic: < ms_per_step
                means the GPU, not Python, sets the pace)
Other workloads: `cplx_i16` / `fir2d_u8` measure configs[2] / configs[4]; `fir1d_u8` the
reference's own u8 -> sat-u8 golden path (a1/a4) at scale; `ideal_u8` (the f64
ideal model), `bank_u8` (the fused 4-filter 3-tap bank, §8(f) 3) and
`restore_u8` (the f64 -> u8 clip conversion, §8(f) 4) and `metrics_u8` (the report's
_compute_metrics, §8(f) 2) measure the next rows on 2^28 samples (4096-sample rows for the
image workloads, the reference's row layout).  For workloads without a C oracle leg
(restore_u8, metrics_u8) cpu_baseline times the NumPy restatement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (ROOT, ROOT / "warmup-fir-filter_amd"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import fir_hip  # noqa: E402
from fir_hip import sharded, torch_ops  # noqa: E402

METRIC = "Gsamples/s + %HBM-roofline, 5-tap int16 FIR-1D, 2^28 samples @1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
SEED = 20260227
SHARPEN5 = [-256, -1024, 6656, -1024, -256]  # h_coeff_5tap_map["sharpen"] in Q4.12
SIMPLE_LP3 = [1024, 2048, 1024]              # h_coeff_3tap_map["simple_lp"] in Q4.12
SIMPLE_LP5 = [256, 1024, 1536, 1024, 256]    # h_coeff_5tap_map["simple_lp"] in Q4.12
SHARPEN5_F64 = [-1 / 16, -4 / 16, 26 / 16, -4 / 16, -1 / 16]  # h_coeff_5tap_map["sharpen"]
BANK3 = [[1365] * 3, [1024, 2048, 1024], [-4096, 0, 4096], [-512, 5120, -512]]  # h_coeff_3tap_map, Q4.12
BANK3_NAMES = ("moving_avg", "simple_lp", "edge", "sharpen")  # the bank's order (h_coeff.py:3-8)
ROW_W = 4096
PIPE_COPIES = max(1, int(os.environ.get("FIR_PIPE_COPIES", "4")))  # configs[0]: rotated buffer sets (> 256 MB)
IMAGES_NPZ = ROOT / "warmup-fir-filter_amd" / "fir_1d" / "sim" / "img_u8.npz"  # the 7 golden images, decoded
# FIR_SELF_HALO=1 (N = 1 only): post the RCCL halo exchange every step with the segment as its
# own neighbour (a ring of one), so the sharded step's exchange + edge kernel run and are timed
# on a single GPU.  Rehearsal only; the JSON line says so in config.rehearsal.
SELF_HALO = os.environ.get("FIR_SELF_HALO") == "1"
# N > 1 halo source: "xgmi" (default: neighbours' HBM mapped once, read by the edge kernel) or
# "rccl" (send/recv every step); xgmi falls back to rccl on every rank if any rank cannot map.
HALO_PREF = os.environ.get("FIR_HALO", "xgmi")
# xGMI step ordering: "serial" (the gate, then ONE segment launch reading its halos; default) or
# "overlap" (the gate on a high-priority side stream while the bulk kernel runs, then a 4-output edge
# kernel).  Measured (profiles/r04): serial 253.5 us per step against 268.5 us for
# overlap with the segment as its own neighbour, and 513 vs 608 us with 2 ranks sharing one GPU:
# a gate running beside the bulk kernel is slowed by it (9 -> 35 us, up to 320 us while it polls a
# neighbour) and the edge launch adds its own gap, so overlapping costs more than it hides.
GATE_MODE = os.environ.get("FIR_GATE_MODE", "serial")
KERNELS = {"fir1d_i16": "fir1d_reg_kernel", "cplx_i16": "fir1d_reg_kernel", "fir2d_u8": "fir2d_pk16_strip_kernel",
           "fir1d_u8": "fir1d_reg_kernel", "ideal_u8": "fir1d_ideal_kernel", "bank_u8": "fir1d_reg_kernel",
           "restore_u8": "restore_map_kernel",
           "pipeline_fixed3": "fir1d_reg_batch_kernel (4-filter bank, the 7 images in one launch)",
           "metrics_u8": "metrics_leaf_kernel (+ metrics_prep: unset markers; chain and final in the launch)"}
NUMPY_ONLY = ("restore_u8", "metrics_u8", "pipeline_fixed3")  # no C oracle leg: the NumPy restatement is the CPU baseline
ROOF_RAMP, ROOF_LAUNCHES = 100, 200  # roofline loop: untimed ramp, then timed launches of the dominant kernel


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def _cpu_threads() -> int:
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(16, _env_int("OMP_NUM_THREADS", n), n))


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def launch_ranks(n: int, script: str, argv: list[str], env: dict | None = None) -> int:
    """Run ``script argv`` as n ranks under torch.distributed.run (a CHILD process: the caller
    must not have touched the GPU, and nothing here execs).  Rank 0's JSON line is forwarded to
    stdout; everything else the ranks print goes to stderr.  Returns the launcher's exit status
    (non-zero if any rank failed, or if no JSON line came back)."""
    import subprocess
    import tempfile

    env = dict(os.environ if env is None else env)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    with tempfile.TemporaryDirectory(prefix="fir_bench_") as tmp:
        # rank 0 writes its line to a file (emit_result): torchrun runs the ranks unbuffered, so a
        # line on a shared stdout pipe can interleave with another rank's output
        result = Path(tmp) / "result.json"
        env["FIR_BENCH_RESULT"] = str(result)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), script, *argv]
        # the ranks' own output goes to stderr: stdout carries only the result line
        rc = subprocess.run(cmd, env=env, stdout=sys.stderr.fileno()).returncode
        line = result.read_text().strip() if result.exists() else ""
    if line:
        print(line, flush=True)
    elif rc == 0:
        print("bench.py: the ranks exited without a result line", file=sys.stderr)
        return 1
    return rc


def emit_result(line: str) -> None:
    """Rank 0's one JSON line: to the launcher's result file when started by launch_ranks, else
    stdout."""
    path = os.environ.get("FIR_BENCH_RESULT")
    if path:
        Path(path).write_text(line + "\n")
    else:
        print(line, flush=True)


class Workload:
    """One bench workload: host input, device buffers, one step, the oracle check."""

    def __init__(self, name: str, rank: int, world: int, dev: torch.device, log2n: int, n_total: int | None = None):
        """n_total (1-D workloads): the signal's total length split over the ranks (strong scaling)
        instead of 2^log2n samples per rank (weak scaling)."""
        self.name, self.rank, self.world, self.dev = name, rank, world, dev
        self.gen2d = False
        rng = np.random.default_rng(SEED + rank)
        if name == "fir1d_i16":
            lo, hi = sharded.segment_bounds(n_total, world, rank) if n_total else (0, 1 << log2n)
            self.n = hi - lo
            self.taps = torch_ops.Taps(SHARPEN5)
            self.channels = 1
            self.x_host = rng.integers(-32768, 32768, self.n, dtype=np.int16)
            self.bytes_per_unit = 2 + 4
            self.units = self.n
            self.unit = "Gsamples/s"
            self.dtype = "int32 (int16 in, int32 wrap-around acc, int32 out)"
            self.config = {"workload": "fir1d_int16_int32_5tap_sharpen_q4.12", "samples_per_gpu": self.n,
                           "total_samples": self.n * world, "taps": 5, "frac_bits": 12, "acc_bits": 32,
                           "parallelism": "single GPU"}  # sharded runs: set by the first step
        elif name == "cplx_i16":
            lo, hi = sharded.segment_bounds(n_total // 2, world, rank) if n_total else (0, 1 << (log2n - 1))
            self.n = hi - lo  # complex samples
            self.taps = torch_ops.Taps(SIMPLE_LP3)
            self.channels = 2
            self.x_host = rng.integers(-32768, 32768, 2 * self.n, dtype=np.int16)
            self.bytes_per_unit = 4 + 8
            self.units = self.n
            self.unit = "Gsamples/s (complex)"
            self.dtype = "int32 (complex int16 in, real Q4.12 taps, complex int32 out)"
            self.config = {"workload": "fir1d_complex_int16_3tap_simple_lp", "complex_samples_per_gpu": self.n,
                           "taps": 3, "parallelism": "single GPU" if world == 1 else f"contiguous shards x{world}"}
        elif name == "fir2d_u8":
            self.h = self.w = 8192
            h1 = np.array(SIMPLE_LP5, dtype=np.int64)
            self.hq2 = (np.outer(h1, h1) // 4096).astype(np.int64)  # unity-gain 5x5 Q4.12
            # FIR2D_TAPS=gen5x5: a non-separable signed 5x5 (the general packed-16 form) instead
            self.gen2d = os.environ.get("FIR2D_TAPS") == "gen5x5"
            if self.gen2d:
                self.hq2 = np.random.default_rng(55).integers(-4, 5, (5, 5)).astype(np.int64)
            # A step filters a batch of FIR2D_FRAMES distinct 8192x8192 frames in one launch
            # (fir2d_fixed_frames_dev).  One frame (64 MiB in + 64 MiB out) fits the 256 MB
            # Infinity Cache, so filtering the same frame step after step would be served partly
            # from it (profiles/r02/micro2d_cold.txt: 23.6 us back to back vs 29.5 us cold); 4
            # frames move 512 MiB per step, so every step streams from HBM, as a video pipeline
            # would, and one launch per batch spares the per-launch ramp (29.7 -> 26.1 us/frame).
            self.frames = max(1, _env_int("FIR2D_FRAMES", 4))
            self.frames_host = rng.integers(0, 256, (self.frames, self.h, self.w), dtype=np.uint8)
            self.x_host = self.frames_host[0]  # the CPU legs' NumPy restatement times frame 0
            self.bytes_per_unit = 1 + 1
            self.units = self.frames * self.h * self.w
            self.unit = "Gpixels/s"
            self.dtype = "int32 (u8 in, int32 wrap-around acc, u8 saturated out)"
            self.config = {"workload": "fir2d_u8_5x5_" + ("nonseparable_signed_seed55" if self.gen2d else
                                                          "simple_lp_outer_q4.12"), "frame": [self.h, self.w],
                           "frames_per_step": self.frames, "parallelism": "single GPU (replicas when N > 1)"}
        elif name in ("ideal_u8", "bank_u8", "fir1d_u8"):
            self.n = 1 << log2n
            self.x_host = rng.integers(0, 256, (self.n // ROW_W, ROW_W), dtype=np.uint8)
            self.units = self.n
            self.unit = "Gsamples/s"
            par = "single GPU (replicas when N > 1)"
            if name == "fir1d_u8":
                self.taps = torch_ops.Taps(SHARPEN5)
                self.bytes_per_unit = 1 + 1
                self.dtype = "int32 (u8 in, int32 wrap-around acc, u8 saturated out)"
                self.config = {"workload": "fir1d_u8_5tap_sharpen_q4.12_rows4096", "samples_per_gpu": self.n,
                               "row_width": ROW_W, "taps": 5, "parallelism": par}
            elif name == "ideal_u8":
                self.bytes_per_unit = 1 + 8
                self.dtype = "f64 (u8 in, f64 taps, per-op rounded k-order sums, f64 out)"
                self.config = {"workload": "fir1d_ideal_f64_5tap_sharpen_rows4096", "samples_per_gpu": self.n,
                               "row_width": ROW_W, "taps": 5, "parallelism": par}
            else:
                self.bytes_per_unit = 1 + len(BANK3)
                self.dtype = "int32 (u8 in, int32 wrap-around acc, u8 saturated out x 4 filters)"
                self.config = {"workload": "fir1d_u8_bank4_3tap_q4.12_rows4096", "samples_per_gpu": self.n,
                               "row_width": ROW_W, "filters": len(BANK3), "taps": 3, "parallelism": par}
        elif name == "restore_u8":
            self.n = 1 << log2n
            self.x_host = rng.uniform(-64.0, 320.0, (self.n // ROW_W, ROW_W))  # ideal-output-like f64 rows
            self.units = self.n
            self.unit = "Gsamples/s"
            self.bytes_per_unit = 8 + 1
            self.dtype = "f64 in, u8 out (rint, clip)"
            self.config = {"workload": "restore_f64_to_u8_clip_rows4096", "samples_per_gpu": self.n,
                           "parallelism": "single GPU (replicas when N > 1)"}
        elif name == "pipeline_fixed3":
            # configs[0]: the fixed 3-tap stage of pipeline_fir_1d.py on the 7 golden images (the
            # reference's decoded u8 inputs, warmup-fir-filter_amd/fir_1d/sim/img_u8.npz) x the 4 filters of
            # h_coeff_3tap_map: the 7 images in ONE fused 4-filter launch (fir1d_fixed_images_multi_dev)
            # per step
            with np.load(IMAGES_NPZ) as d:
                self.images = [(k, np.ascontiguousarray(d[k])) for k in sorted(d.files)]
            self.x_host = self.images[0][1]
            px = sum(a.size for _, a in self.images)
            self.units = px * len(BANK3)  # output samples per stage (67,975,252)
            self.bytes_per_unit = (1 + len(BANK3)) / len(BANK3)  # 1 B in per pixel, 1 B out per output
            self.unit = "Gsamples/s"
            self.dtype = "int32 (u8 in, int32 wrap-around acc, u8 saturated out x 4 filters)"
            self.config = {"workload": "pipeline_fixed_3tap_stage_7_golden_images_x4_filters",
                           "images": len(self.images), "pixels": px, "filters": len(BANK3),
                           "output_samples": self.units, "parallelism": "single GPU (replicas when N > 1)",
                           "buffer_sets": PIPE_COPIES,
                           "note": f"one stage moves 85 MB, which fits the 256 MB Infinity Cache (MALL): every "
                                   f"step and roofline launch works on the next of {PIPE_COPIES} resident copies of "
                                   f"the stage's inputs and outputs ({PIPE_COPIES} x 85 MB > 256 MB), so each "
                                   f"launch streams from HBM; roofline.mall_resident is the same launch replayed "
                                   f"on one set"}
        elif name == "metrics_u8":
            self.n = 1 << log2n
            self.x_host = rng.uniform(-64.0, 320.0, self.n)  # ideal-output-like f64
            self.fixed_host = np.clip(np.rint(self.x_host) + rng.integers(-3, 4, self.n), 0, 255).astype(np.uint8)
            self.fixed = torch.from_numpy(self.fixed_host).to(dev)
            self.work = torch.empty(int(fir_hip.lib().fir_metrics_work_bytes(self.n)), dtype=torch.uint8, device=dev)
            self.units = self.n
            self.unit = "Gsamples/s"
            self.bytes_per_unit = 8 + 1
            self.dtype = "f64 (sums in NumPy's order, bit-exact; counts and max exact)"
            self.config = {"workload": "compare_metrics_f64_u8", "samples_per_gpu": self.n,
                           "parallelism": "single GPU (replicas when N > 1)"}
        else:
            raise SystemExit(f"unknown workload {name}")
        self.plans, self.turn = [], 0
        if name == "pipeline_fixed3":
            # PIPE_COPIES sets of the stage's buffers, used in turn (see config.note).  One buffer per
            # (image, filter) output, as the reference keeps them: each plane starts on the allocator's
            # 512-byte boundary, so every wave stores whole 128-byte lines
            self.sets = []
            for _ in range(PIPE_COPIES):
                xs = [torch.from_numpy(a).to(dev) for _, a in self.images]
                ys = [[torch.empty(a.shape, dtype=torch.uint8, device=dev) for _ in BANK3] for _, a in self.images]
                self.sets.append((xs, ys))
            self.xs, self.ys = self.sets[0]
            self.x, self.y = self.xs[0], self.ys[0][0]
        elif name == "fir2d_u8":  # the resident batch of frames
            self.x = torch.from_numpy(self.frames_host).to(dev)
            self.y = torch.empty(self.x.shape, dtype=torch.uint8, device=dev)
        else:
            self.x = torch.from_numpy(self.x_host).to(dev)
            if name == "ideal_u8":
                self.y = torch.empty(self.x.shape, dtype=torch.float64, device=dev)
            elif name == "bank_u8":
                self.y = torch.empty((len(BANK3),) + tuple(self.x.shape), dtype=torch.uint8, device=dev)
            elif name == "restore_u8":
                self.y = torch.empty(self.x.shape, dtype=torch.uint8, device=dev)
            elif name == "metrics_u8":
                self.y = torch.empty(9, dtype=torch.float64, device=dev)
            else:
                u8 = name == "fir1d_u8"
                self.y = torch.empty(self.x.shape, dtype=torch.uint8 if u8 else torch.int32, device=dev)
        self.left = self.right = None  # the halos the last step used (host copies for the oracle)
        self.halo_src, self.halo_kind = None, None

    @property
    def sharded_1d(self) -> bool:
        # FIR_SELF_HALO=1 rehearses the RCCL exchange at N = 1 (the segment is its own neighbour)
        return (self.world > 1 or SELF_HALO) and self.name in ("fir1d_i16", "cplx_i16")

    @property
    def alg_bytes(self) -> int:
        """Algorithmic bytes of one step (in + out bytes per unit x units)."""
        return int(round(self.units * self.bytes_per_unit))

    def bulk(self):
        if self.name == "pipeline_fixed3":
            # the 7 images x 4 filters in ONE launch, its arguments marshalled once (a plan).  One
            # launch per image took 55.8 us per stage, 4.1-4.6 us for each small image; as 7
            # parallel graph branches 88.3 us (profiles/r05/pipeline_unaligned_ab.txt)
            if not self.plans:
                self.plans = [torch_ops.ImagesMultiPlan(xs, BANK3, 12, 32, fir_hip.OUT_U8_SAT, outs=ys)
                              for xs, ys in self.sets]
            self.plans[self.turn % len(self.plans)].launch()
            self.turn += 1
        elif self.name == "fir2d_u8":
            torch_ops.fir2d_fixed_dev(self.x, self.hq2, 12, 32, fir_hip.OUT_U8_SAT, out=self.y)
        elif self.name == "ideal_u8":
            torch_ops.fir1d_ideal_rows_dev(self.x, SHARPEN5_F64, out=self.y)
        elif self.name == "bank_u8":
            torch_ops.fir1d_fixed_rows_multi_dev(self.x, BANK3, 12, 32, fir_hip.OUT_U8_SAT, out=self.y)
        elif self.name == "fir1d_u8":
            torch_ops.fir1d_fixed_rows_dev(self.x, self.taps, 12, 32, fir_hip.OUT_U8_SAT, out=self.y)
        elif self.name == "restore_u8":
            torch_ops.restore_u8_dev(self.x, fir_hip.RESTORE_CLIP, out=self.y)
        elif self.name == "metrics_u8":
            torch_ops.compare_metrics_dev(self.x, self.fixed, out=self.y, work=self.work)
        else:
            torch_ops.fir1d_fixed_rows_dev(self.x, self.taps, 12, 32, fir_hip.OUT_I32, self.channels, out=self.y)

    def dominant(self):
        """The step's dominant kernel alone (roofline timing): the halo-reading launch of a serial
        xGMI-sharded step, else the bulk kernel."""
        if self.sharded_1d and self.halo_kind == "xgmi" and GATE_MODE == "serial":
            torch_ops.fir1d_fixed_segment_dev(self.x, self.taps, *self.halo_src.halos(), 12, 32, fir_hip.OUT_I32,
                                              self.channels, out=self.y)
        else:
            self.bulk()

    def step(self):
        """One pass of the hot path (for N > 1: bulk kernel, then the halo-dependent edges)."""
        if not self.sharded_1d:
            self.bulk()
            return
        if self.halo_src is None:  # set up once (collectively), used every step
            if self.world == 1:  # FIR_SELF_HALO rehearsal: a ring of one (RCCL, or the gate on its own mailbox)
                self.halo_kind = "xgmi" if HALO_PREF == "xgmi" else "rccl"
                self.halo_src = (sharded.XgmiHalo(self.x, self.taps.n, self.channels, self_ring=True)
                                 if self.halo_kind == "xgmi" else
                                 sharded.HaloExchange(self.x, self.taps.n, self.channels, self_ring=True))
            else:
                self.halo_kind, self.halo_src = sharded.make_halo_source(self.x, self.taps.n, self.channels,
                                                                         prefer=HALO_PREF)
            self.describe_parallelism()
        self._step_sharded()

    def set_halo(self, kind, src) -> None:
        """Use ``src`` (an XgmiHalo or HaloExchange over this rank's segment) from the next step on."""
        self.halo_kind, self.halo_src = kind, src
        self.left = self.right = None
        self.describe_parallelism()

    def describe_parallelism(self) -> None:
        self.config["parallelism"] = (
                f"contiguous shards x{self.world}, " + (
                    "halo handed over through the neighbours' HBM over xGMI, ordered per step: a one-wave gate "
                    "kernel publishes this rank's edge samples with the step's epoch, waits for both neighbours' "
                    "epoch (device atomics on IPC-mapped mailboxes) and copies their edges; " + (
                        "the gate runs on a high-priority side stream while the bulk FIR kernel runs, then a "
                        "4-output edge kernel reads the halos" if GATE_MODE == "overlap" else
                        "then one FIR launch reads them") if self.halo_kind == "xgmi"
                    else "halo exchanged by RCCL send/recv every step (ordered by the messages), overlapped with "
                         "the bulk kernel, then an edge kernel"))

    def _step_sharded(self):
        if self.halo_kind == "xgmi" and GATE_MODE == "overlap":  # gate || bulk, then the edge kernel
            self.halo_src.gate_async()
            self.bulk()
            self.halo_src.join()
            self.left, self.right = self.halo_src.halos()
            torch_ops.fir1d_fixed_edges_dev(self.x, self.taps, self.y, self.left, self.right, 12, 32, fir_hip.OUT_I32,
                                            self.channels)
            return
        if self.halo_kind == "xgmi":  # the ordered hand-off, then ONE FIR launch reading the received halos
            self.halo_src.gate()
            self.left, self.right = self.halo_src.halos()
            torch_ops.fir1d_fixed_segment_dev(self.x, self.taps, self.left, self.right, 12, 32, fir_hip.OUT_I32,
                                              self.channels, out=self.y)
            return
        works = self.halo_src.post()  # RCCL: bulk || exchange, then the edge kernel
        self.bulk()
        sharded.wait_all(works)
        left, right = self.halo_src.halos()
        self.left, self.right = left, right
        torch_ops.fir1d_fixed_edges_dev(self.x, self.taps, self.y, left, right, 12, 32, fir_hip.OUT_I32,
                                        self.channels)

    def oracle(self, nthreads: int, reps: int = 1):
        from oracle import c_oracle

        co = c_oracle()
        out = None
        for _ in range(reps):
            if self.name == "pipeline_fixed3":
                out = [np.stack([co.fir1d_rows(a, h, 12, 32, co.OUT_U8_SAT, nthreads=nthreads) for h in BANK3])
                       for _, a in self.images]
            elif self.name == "fir2d_u8":
                out = np.stack([co.fir2d(f, self.hq2, 12, 32, co.OUT_U8_SAT, nthreads=nthreads)
                                for f in self.frames_host])
            elif self.name == "ideal_u8":
                out = co.fir1d_ideal_rows(self.x_host, SHARPEN5_F64, nthreads=nthreads)
            elif self.name == "bank_u8":
                out = np.stack([co.fir1d_rows(self.x_host, h, 12, 32, co.OUT_U8_SAT, nthreads=nthreads)
                                for h in BANK3])
            elif self.name == "fir1d_u8":
                out = co.fir1d_rows(self.x_host, self.taps.h, 12, 32, co.OUT_U8_SAT, nthreads=nthreads)
            elif self.name == "restore_u8":
                from oracle import fir_oracle as fo

                out = fo.to_u8_clip(self.x_host)
            elif self.name == "metrics_u8":
                from oracle import fir_oracle as fo

                out = fo.compute_metrics(self.x_host, self.fixed_host)
            else:
                hl = None if self.left is None else np.asarray(self.left.cpu() if torch.is_tensor(self.left) else self.left)
                hr = None if self.right is None else np.asarray(self.right.cpu() if torch.is_tensor(self.right) else self.right)
                out = co.fir1d_rows(self.x_host, self.taps.h, 12, 32, co.OUT_I32, channels=self.channels,
                                    halo_left=hl, halo_right=hr, nthreads=nthreads)
        return out

    def numpy_oracle_threads(self, max_units: int, nthreads: int) -> int:
        """The NumPy restatement over the leading ``max_units`` units split into ``nthreads``
        contiguous slices on a thread pool (NumPy releases the GIL in its array loops); 1-D
        int16 slices carry their true halos, row workloads split on row boundaries.
        Returns the units done."""
        from concurrent.futures import ThreadPoolExecutor

        from oracle import fir_oracle as fo

        if nthreads <= 1:
            return self.numpy_oracle(max_units)
        if self.name == "pipeline_fixed3":  # the 28 (image, filter) outputs over the pool
            def job(i):
                done = 0
                for k, (_, a) in enumerate(self.images):
                    for f, h in enumerate(BANK3):
                        if (k * len(BANK3) + f) % nthreads == i:
                            fo.fir1d_rows(a, h, 12, 32, fo.OUT_U8_SAT)
                            done += a.size
                return done
        elif self.name in ("fir1d_i16", "cplx_i16"):
            n = min(self.units, max_units)
            ch = self.channels
            hl, hr = fo.halo_sizes(self.taps.n)
            x = self.x_host

            def job(i):
                lo, hi = n * i // nthreads, n * (i + 1) // nthreads
                a, b = lo * ch, hi * ch
                fo.fir1d_i16_i32(x[a:b], self.taps.h, 12, 32, channels=ch,
                                 halo_left=x[max(0, a - hl * ch):a] if a >= hl * ch else None,
                                 halo_right=x[b:b + hr * ch] if b + hr * ch <= x.size else None)
                return hi - lo
        else:
            unit_rows = self.w if self.name == "fir2d_u8" else (ROW_W if self.name in (
                "ideal_u8", "bank_u8", "fir1d_u8", "restore_u8") else 1)
            nrows = max(nthreads, min(self.units, max_units) // unit_rows)

            def job(i):
                r0, r1 = nrows * i // nthreads, nrows * (i + 1) // nthreads
                return self.numpy_oracle((r1 - r0) * unit_rows, offset=r0 * unit_rows)
        with ThreadPoolExecutor(nthreads) as pool:
            return sum(pool.map(job, range(nthreads)))

    def numpy_oracle(self, max_units: int, offset: int = 0):
        """The NumPy restatement on ``max_units`` units from unit ``offset`` (row-aligned for
        the row workloads); returns the units done."""
        from oracle import fir_oracle as fo

        if self.name == "pipeline_fixed3":  # whole stage (all 28 outputs), whatever max_units is
            for _, a in self.images:
                for h in BANK3:
                    fo.fir1d_rows(a, h, 12, 32, fo.OUT_U8_SAT)
            return self.units
        if self.name == "fir2d_u8":
            r0 = offset // self.w
            rows = max(1, min(self.h - r0, max_units // self.w))
            fo.fir2d_fixed(self.x_host[r0:r0 + rows], self.hq2, 12, 32, fo.OUT_U8_SAT)
            return rows * self.w
        if self.name == "metrics_u8":
            m = min(self.n - offset, max_units)
            fo.compute_metrics(self.x_host[offset:offset + m], self.fixed_host[offset:offset + m])
            return m
        if self.name in ("ideal_u8", "bank_u8", "fir1d_u8", "restore_u8"):
            r0 = offset // ROW_W
            rows = max(1, min(self.x_host.shape[0] - r0, max_units // ROW_W))
            xs = self.x_host[r0:r0 + rows]
            if self.name == "restore_u8":
                fo.to_u8_clip(xs)
            elif self.name == "fir1d_u8":
                fo.fir1d_rows(xs, self.taps.h, 12, 32, fo.OUT_U8_SAT)
            elif self.name == "ideal_u8":
                fo.fir1d_ideal_rows(xs, SHARPEN5_F64)
            else:
                for h in BANK3:
                    fo.fir1d_rows(xs, h, 12, 32, fo.OUT_U8_SAT)
            return rows * ROW_W
        n = min(self.units - offset, max_units)
        c = self.channels
        fo.fir1d_i16_i32(self.x_host[offset * c:(offset + n) * c], self.taps.h, 12, 32, channels=c)
        return n

    def matches_reference(self) -> bool:
        """pipeline_fixed3: the 28 outputs' SHA-256 against the reference's own (recorded by
        tests/golden/make_golden.py from gen_fixed_output._run_fixed_rowwise)."""
        import hashlib

        outs = json.loads((ROOT / "tests" / "golden" / "image_outputs.json").read_text())["outputs"]
        want = {(o["case_stem"], o["coeff_name"]): o["fixed_u8_sha256"] for o in outs if o["tap"] == "3tap"}
        names = list(BANK3_NAMES)
        for (stem, _), yh in zip(self.images, self._planes_np()):
            for f, name in enumerate(names):
                if hashlib.sha256(np.ascontiguousarray(yh[f]).tobytes()).hexdigest() != want[(stem, name)]:
                    return False
        return True

    def _planes_np(self, ys=None):
        """pipeline_fixed3's outputs (of buffer set ``ys``, default the first) as one (filters, h, w)
        array per image."""
        return [np.stack([p.cpu().numpy() for p in ps]) for ps in (self.ys if ys is None else ys)]

    def matches(self, ref) -> bool:
        """Full-output parity: every output, and every report metric, bit for bit."""
        if self.name == "pipeline_fixed3":  # every buffer set the steps rotated through
            return all(np.array_equal(y, r) for _, ys in self.sets for y, r in zip(self._planes_np(ys), ref)) \
                and self.matches_reference()
        got = self.y.cpu().numpy()
        if self.name != "metrics_u8":
            return bool(np.array_equal(got, ref))
        return fir_hip.metrics_from_sums(got, self.n) == ref


RAMP_MS = 50.0  # the roofline loop's untimed ramp lasts at least this much GPU time


def ramp_launches(wl: Workload, at_least: int, world: int = 1, red_dev=None) -> int:
    """Untimed launches of the dominant kernel for a ramp of >= RAMP_MS: short kernels need more
    than a count of launches gives them (fir_2d 4 x 8192^2 ran 94 us in its first 100 launches,
    83 in the next 200 and 78.9 after 300; the 16 us pipeline stage 17.5 before 300, 15.8 after;
    rocprofv3 traces in gpurun_out r05x)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        wl.dominant()
    e1.record()
    e1.synchronize()
    est_ms = max(e0.elapsed_time(e1) / 5, 1e-3)
    n = max(at_least, min(20000, int(RAMP_MS / est_ms) + 1))
    if world > 1:  # the same count on every rank
        t = torch.tensor([float(n)], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n = int(t.item())
    return n


def measure(wl: Workload, steps: int, warmup: int, ramp: int, launches: int, world: int = 1,
            barrier=lambda: None, red_dev=None):
    """Time ``steps`` steps after ``warmup`` untimed ones (barrier + synchronize on both sides, max
    over ranks), then the dominant kernel alone: ``ramp`` untimed launches and at least RAMP_MS of
    them (ramp_launches), then ``launches`` back to back on the stream it runs on, bracketed by
    two HIP events (events between launches would perturb the stream: each record adds a ~11 us
    gap).  Leaves the full step's output in place.  Returns (elapsed s, host issue s, mean
    dominant-kernel s)."""
    for _ in range(warmup):
        wl.step()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        wl.step()
    t_issue = time.perf_counter() - t0  # host time to issue the steps (diagnostic: host-bound?)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_avg_s = roofline_loop(wl, ramp, launches, world, red_dev)
    wl.step()  # restore the full step's output (the loop above ran the dominant kernel alone)
    torch.cuda.synchronize()
    return elapsed, t_issue, kern_avg_s


def roofline_loop(wl: Workload, ramp: int, launches: int, world: int = 1, red_dev=None) -> float:
    """Mean duration (s) of the dominant kernel: ``ramp`` untimed launches and at least RAMP_MS of
    them, then ``launches`` back to back between two HIP events on the stream it runs on."""
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n_roof = max(1, launches)
    for _ in range(ramp_launches(wl, max(0, ramp), world, red_dev) if ramp > 0 else 0):
        wl.dominant()
    torch.cuda.synchronize()
    ev0.record()
    for _ in range(n_roof):
        wl.dominant()
    ev1.record()
    ev1.synchronize()
    return ev0.elapsed_time(ev1) / 1e3 / n_roof


def _sync() -> None:
    if torch.cuda.is_available():  # (the CPU tests drive the collective helpers below over gloo)
        torch.cuda.synchronize()


def gather_floats(v: float, world: int, red_dev) -> list[float]:
    """Every rank's value of ``v`` (collective)."""
    if world == 1:
        return [v]
    t = torch.tensor([v], dtype=torch.float64, device=red_dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [float(p.item()) for p in parts]


def halo_report(wl: Workload, world: int, barrier, red_dev, n: int = 100) -> dict:
    """config.halo of a sharded run (collective: every rank runs it after the timed steps): the
    halo source, why RCCL was chosen if it was, and what the hand-off alone costs per step --
    the xGMI gate kernel timed by HIP events around ``n`` back-to-back gates on the step stream
    (every rank runs the same count, so every wait is met), or RCCL's post + wait timed on the
    host -- as the max and min over ranks."""
    src = wl.halo_src
    info = {"source": wl.halo_kind}
    if wl.halo_kind == "xgmi":
        info["gate_mode"] = GATE_MODE
        barrier()
        _sync()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(n):
            src.gate()
        ev1.record()
        ev1.synchronize()
        per = gather_floats(ev0.elapsed_time(ev1) * 1e3 / n, world, red_dev)
        info["gate_us_per_step"] = {"max": round(max(per), 2), "min": round(min(per), 2),
                                    "timing": f"HIP events around {n} gate launches alone"}
    else:
        info["fallback_reason"] = getattr(src, "fallback_reason", None)
        barrier()
        _sync()
        t0 = time.perf_counter()
        for _ in range(n):
            sharded.wait_all(src.post())
        _sync()
        per = gather_floats((time.perf_counter() - t0) * 1e6 / n, world, red_dev)
        info["exchange_us_per_step"] = {"max": round(max(per), 2), "min": round(min(per), 2),
                                        "timing": f"host clock around {n} post + wait alone"}
    barrier()
    return info


def gate_failures(wl: Workload, world: int, red_dev) -> list[int]:
    """Ranks whose gated hand-off timed out in this run (collective; [] for other sources).  The
    gate's waits are bounded (timeout_s), so this is reached even when a neighbour never
    published: the run then ends with a line and a non-zero status instead of hanging."""
    bad = int(isinstance(wl.halo_src, sharded.XgmiHalo) and int(wl.halo_src.status.item()) != 0)
    flags = gather_floats(float(bad), world, red_dev)
    return [r for r, f in enumerate(flags) if f]


def pmc_traffic(wl: Workload, root: Path = ROOT):
    """HBM bytes per launch (per step for pipeline_fixed3) from the committed rocprofv3 PMC summary
    profiles/pmc_<workload>.json -- only when it was taken at this workload's size AND on the build
    that is running (its build_id, written by tools/pmc_summary.py from fir_build_id() on the box,
    equals the loaded library's): a summary of another build describes other kernels.  Else None."""
    pmc = root / "profiles" / f"pmc_{wl.name}{'_gen5x5' if wl.gen2d else ''}.json"
    if not pmc.exists():
        return None
    try:
        summary = json.loads(pmc.read_text())
    except (ValueError, OSError):
        return None
    if summary.get("algorithmic_bytes_per_launch") != wl.alg_bytes:
        return None
    if summary.get("build_id") != fir_hip.build_id():
        return None
    return summary.get("hbm_bytes_per_launch")


# The other single-GPU BASELINE configs, timed after the headline when bench.py runs without
# --workload at N = 1 (the driver's own run): configs[2] complex int16 2^27, configs[4] fir_2d 5x5
# on 8192^2 frames, configs[0] the pipeline's fixed 3-tap stage on the 7 golden images.
SUB_CONFIGS = (("configs[2]", "cplx_i16"), ("configs[4]", "fir2d_u8"), ("configs[0]", "pipeline_fixed3"))


def pipeline_stage_wall(reps: int = 5) -> dict:
    """configs[0] end to end through the host API, as pipeline_fir_1d.py runs it:
    generate_fixed_3tap_output_vector over the 7 golden images in a scratch input dir (the stage
    plans, reads the 7 .npy inputs into page-locked staging, makes ONE device call -- upload, one
    batch launch, 28 plane downloads -- and writes the 28 .npy outputs while the later planes are
    in flight).  The first run (page-locked buffers allocated) is reported on its own; then the
    best of ``reps`` by wall time, with its breakdown (ms): plan, load (file reads), h2d / kernel /
    d2h (HIP events inside the call), call (the device call on the host clock, plane writes
    overlapping it), save_tail (writes still running after the call), wall.  The ideal 3-tap stage
    (28 float64 outputs, 544 MB) is timed the same way."""
    import shutil
    import tempfile

    from fir_1d.sim.vector.gen_fixed_output import generate_fixed_3tap_output_vector
    from fir_1d.sim.vector.gen_ideal_output import generate_ideal_3tap_output_vector

    def stage(fn, ind, root, n, fresh):
        """n runs; fresh: each into a new output tree (a clean pipeline run), else over the
        previous run's files (--overwrite-vectors)"""
        runs = []
        for k in range(n):
            outd = root / (f"out{k}" if fresh else "out")
            t: dict = {}
            files = fn(input_dir=ind, output_dir=outd, overwrite=True, timings=t)
            runs.append(dict(t, files=files))
            if fresh and k:
                shutil.rmtree(root / f"out{k - 1}")
        return runs

    with tempfile.TemporaryDirectory(prefix="fir_stage_") as tmp:
        ind = Path(tmp) / "input"
        ind.mkdir()
        with np.load(IMAGES_NPZ) as d:
            for k in d.files:
                np.save(ind / f"{k}_x_u8.npy", d[k])
        fixed = stage(generate_fixed_3tap_output_vector, ind, Path(tmp) / "f", reps + 1, True)
        fixed_ow = stage(generate_fixed_3tap_output_vector, ind, Path(tmp) / "fo", reps, False)
        ideal = stage(generate_ideal_3tap_output_vector, ind, Path(tmp) / "i", 3, True)
        ideal_ow = stage(generate_ideal_3tap_output_vector, ind, Path(tmp) / "io", 3, False)
    best = min(fixed[1:], key=lambda r: r["wall_ms"])
    best_i = min(ideal[1:], key=lambda r: r["wall_ms"])
    return {"ms": best["wall_ms"], "files": best["files"], "breakdown_ms": best,
            "gpu_work_ms": round(best["h2d_ms"] + best["kernel_ms"] + best["d2h_ms"], 3),
            "first_run_ms": fixed[0]["wall_ms"], "runs_ms": [r["wall_ms"] for r in fixed],
            "overwrite_ms": min(r["wall_ms"] for r in fixed_ow[1:]),
            "ideal_3tap_stage": {"ms": best_i["wall_ms"], "files": best_i["files"], "breakdown_ms": best_i,
                                 "first_run_ms": ideal[0]["wall_ms"],
                                 "overwrite_ms": min(r["wall_ms"] for r in ideal_ow[1:])},
            "what": "generate_fixed_3tap_output_vector (host API: .npy in -> 28 .npy out incl. PCIe copies and file "
                    f"I/O) into a fresh output tree, best of {reps} after a first run (page-locked staging "
                    "allocated); overwrite_ms: the same stage over its previous files (--overwrite-vectors); round "
                    "1's per-image form took 17.4 ms, the reference's own CPU stage 92.6 s (SURVEY §3.1)"}


def run_sub_configs(args, dev) -> tuple[dict, bool]:
    """Each SUB_CONFIGS workload on its own: step rate, dominant-kernel roofline, PMC traffic when a
    matching summary is committed, full-output parity against the C oracle (configs[0] also
    against the reference's own output digests), and the C oracle's rate as its CPU baseline."""
    out, all_ok = {}, True
    nthr = _cpu_threads()
    for label, name in SUB_CONFIGS:
        wl = Workload(name, 0, 1, dev, args.log2n)
        torch.cuda.synchronize()
        elapsed, _, kern = measure(wl, args.steps, args.warmup, args.roofline_ramp, args.roofline_launches)
        tc0 = time.perf_counter()
        ref = wl.oracle(nthr)
        tc = time.perf_counter() - tc0
        ok = wl.matches(ref)
        all_ok &= ok
        achieved = wl.alg_bytes / kern / 1e9
        entry = {
            "workload": wl.config["workload"], "value": round(wl.units * args.steps / elapsed / 1e9, 3),
            "unit": wl.unit, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "dtype": wl.dtype,
            "config": wl.config,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(wl),
                         "kernel": KERNELS[name], "kernel_avg_us": round(kern * 1e6, 2),
                         "algorithmic_bytes_per_launch": wl.alg_bytes},
            "parity": ("bit-exact vs oracle (full output)" + (" and the reference's 28 output SHA-256s"
                                                              if name == "pipeline_fixed3" else ""))
            if ok else "MISMATCH",
            "cpu_baseline": {"value": round(wl.units / tc / 1e9, 4), "unit": wl.unit, "cores": nthr, "kind": "port",
                             "sample": f"C oracle (oracle/fir_oracle.c, OpenMP {nthr} threads), the parity run on the "
                                       f"full workload ({wl.units} units), {tc:.2f} s"},
        }
        if name == "pipeline_fixed3":
            entry["roofline"]["kernel_avg_us_is"] = (f"one launch over the 7 images (one stage), each launch on "
                                                     f"the next of {len(wl.plans)} buffer sets (HBM-streaming)")
            wl.plans = wl.plans[:1]  # the same launch replayed on one set: inputs and outputs MALL-resident
            kern1 = roofline_loop(wl, args.roofline_ramp, args.roofline_launches)
            entry["roofline"]["mall_resident"] = {
                "kernel_avg_us": round(kern1 * 1e6, 2), "achieved": round(wl.alg_bytes / kern1 / 1e9, 1),
                "frac_of_hbm_peak": round(wl.alg_bytes / kern1 / 1e9 / HBM_PEAK_GBS, 4),
                "what": "one buffer set replayed: its 85 MB stay in the 256 MB Infinity Cache, so this is not an "
                        "HBM roofline number"}
            entry["stage_wall"] = pipeline_stage_wall()
        out[label] = entry
        del wl, ref
        torch.cuda.empty_cache()
    return out, all_ok


class LegFailed(Exception):
    """A halo source's leg of an N > 1 run could not produce a number (no xGMI path, a timed-out
    gate, a parity mismatch); the run goes on with the next source."""


def run_halo_legs(kinds, run_one) -> tuple[dict, str | None]:
    """Each halo source's leg in turn (collective: every rank runs the same legs in the same
    order).  ``run_one(kind)`` returns the leg's record or raises LegFailed, which is recorded as
    the leg's ``error`` while the next leg still runs.  Returns (legs, headline kind): the first
    leg in ``kinds`` order that measured with bit-exact parity, or None."""
    legs = {}
    for kind in kinds:
        try:
            legs[kind] = run_one(kind)
        except LegFailed as exc:
            legs[kind] = {"error": str(exc)}
    ok = [k for k in kinds if "error" not in legs[k] and legs[k].get("parity") != "MISMATCH"]
    return legs, (ok[0] if ok else None)


def halo_leg(wl: Workload, kind: str, args, world: int, barrier, red_dev, parity_check: bool = True) -> dict:
    """One N > 1 leg: set up ``kind``'s halo source over the resident segments (xGMI: mapped
    mailboxes, probed collectively; rccl: the send/recv exchange), time the steps and the dominant
    kernel, report the hand-off's own cost, check every rank's full output against the oracle,
    and release the source.  Raises LegFailed when the source cannot run."""
    if kind == "xgmi":
        got, src = sharded.make_halo_source(wl.x, wl.taps.n, wl.channels, prefer="xgmi")
        if got != "xgmi":
            raise LegFailed(f"xGMI halo path unavailable: {src.fallback_reason}")
    else:
        src = sharded.HaloExchange(wl.x, wl.taps.n, wl.channels)
    wl.set_halo(kind, src)
    try:
        barrier()
        elapsed, t_issue, kern = measure(wl, args.steps, args.warmup, args.roofline_ramp, args.roofline_launches,
                                         world, barrier, red_dev)
        kern_ranks = gather_floats(kern, world, red_dev)
        failed = gate_failures(wl, world, red_dev)
        if failed:
            raise LegFailed(f"halo gate timed out (a neighbour's epoch did not arrive within {src.timeout_s} s) on "
                            f"rank(s) {failed}")
        halo = halo_report(wl, world, barrier, red_dev)
        parity = "skipped"
        if parity_check:
            ok = wl.matches(wl.oracle(_cpu_threads()))
            f = torch.tensor([0 if ok else 1], device=red_dev)
            dist.all_reduce(f, op=dist.ReduceOp.MAX)
            parity = "bit-exact vs oracle (full output, every rank)" if int(f.item()) == 0 else "MISMATCH"
        units = gather_floats(float(wl.units), world, red_dev)
        return {"value": round(sum(units) * args.steps / elapsed / 1e9, 3), "unit": wl.unit,
                "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                "kernel_avg_us_ranks": {"max": round(max(kern_ranks) * 1e6, 2), "min": round(min(kern_ranks) * 1e6, 2)},
                "halo": halo, "parity": parity, "parallelism": wl.config["parallelism"],
                "_elapsed": elapsed, "_t_issue": t_issue, "_kern": max(kern_ranks)}
    finally:
        barrier()  # no rank unmaps or frees while a neighbour may still read its mailbox
        if isinstance(src, sharded.XgmiHalo):
            src.close()


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100, help="untimed steps (clocks take ~40 launches to ramp)")
    ap.add_argument("--workload", default=None, choices=tuple(KERNELS),
                    help="default fir1d_i16 (configs[1]); without this flag an N = 1 run also times "
                         "configs[2], [4] and [0] (the line's 'configs' key)")
    ap.add_argument("--no-configs", action="store_true", help="time the headline workload only")
    ap.add_argument("--log2n", type=int, default=28, help="int16 values per GPU (2^28 = BASELINE configs[1])")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline time budget (0 = skip)")
    ap.add_argument("--no-parity", action="store_true", help="skip the full-size oracle comparison")
    ap.add_argument("--roofline-launches", type=int, default=ROOF_LAUNCHES,
                    help="timed launches of the dominant kernel (after as many as --roofline-ramp untimed)")
    ap.add_argument("--roofline-ramp", type=int, default=ROOF_RAMP)
    args = ap.parse_args()
    sub_configs = args.workload is None and not args.no_configs and not SELF_HALO
    args.workload = args.workload or "fir1d_i16"

    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # started directly: spawn the ranks as children (nothing here has touched the GPU;
        # device_count() does not initialise it on this image)
        env = dict(os.environ)
        if "FIR_DIST_BACKEND" not in env and torch.cuda.device_count() < args.gpus:
            env["FIR_DIST_BACKEND"] = "gloo"
            env["FIR_BENCH_REHEARSAL"] = f"{args.gpus} ranks on {torch.cuda.device_count()} GPU(s)"
        return launch_ranks(args.gpus, str(Path(__file__).resolve()), sys.argv[1:], env)

    rank, world = _env_int("RANK", 0), _env_int("WORLD_SIZE", 1)
    local_rank = _env_int("LOCAL_RANK", 0)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # FIR_DIST_BACKEND=gloo rehearses the N>1 flow on a box with fewer GPUs than ranks (ranks
    # share devices, halos staged through the host); the real multi-GPU run uses nccl (= RCCL).
    # Started under torchrun with more ranks than GPUs, the same rehearsal is chosen here.
    backend = os.environ.get("FIR_DIST_BACKEND", "")
    if not backend:
        backend = "nccl" if world == 1 or torch.cuda.device_count() >= world else "gloo"
        if backend == "gloo":
            os.environ["FIR_BENCH_REHEARSAL"] = f"{world} ranks on {torch.cuda.device_count()} GPU(s)"
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if SELF_HALO and world != 1:
        raise SystemExit("FIR_SELF_HALO=1 rehearses the exchange at N = 1 only")
    if world > 1 or SELF_HALO:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        if backend == "nccl":
            # RCCL's internal stream at high priority: it gets its own hardware queue, so the
            # exchange's cross-stream wait does not block the queue the FIR kernels run on
            # (measured with FIR_SELF_HALO=1)
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = os.environ.get("FIR_NCCL_HIPRI", "1") == "1"
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev, pg_options=opts)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    stream = torch.cuda.Stream(device=dev)  # a dedicated (non-null) stream for every launch
    torch.cuda.set_stream(stream)
    wl = Workload(args.workload, rank, world, dev, args.log2n)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            if backend == "nccl":
                dist.barrier(device_ids=[dev_index])
            else:
                dist.barrier()

    barrier()  # every rank's segment is resident and its communicator up before the first step
    legs = strong = None
    if wl.sharded_1d and world > 1:
        # both halo sources, each its own leg with its own numbers (the first real multi-GPU run
        # then yields a value whichever source works); the headline is the first that worked
        kinds = ["xgmi", "rccl"] if HALO_PREF == "xgmi" else [HALO_PREF]
        legs, head = run_halo_legs(kinds, lambda k: halo_leg(wl, k, args, world, barrier, red_dev,
                                                             not args.no_parity))
        if head is None:
            if rank == 0:
                emit_result(json.dumps({"metric": METRIC, "value": None, "unit": wl.unit, "n_gpus": world,
                                        "error": "no halo source produced a result",
                                        "legs": legs, "config": wl.config}))
            print(f"bench.py: every halo leg failed: {legs}", file=sys.stderr)
            dist.destroy_process_group()
            return 3
        lead = legs[head]
        elapsed, t_issue, kern_avg_s = lead["_elapsed"], lead["_t_issue"], lead["_kern"]
        kern_ranks = [lead["kernel_avg_us_ranks"]["max"] / 1e6, lead["kernel_avg_us_ranks"]["min"] / 1e6]
        halo, parity = lead["halo"], lead["parity"]
        wl.config["parallelism"] = lead["parallelism"]
        # strong scaling beside the weak headline: the same total as one GPU's headline (2^log2n
        # samples) split over the N ranks, through the headline's halo source
        swl = Workload(args.workload, rank, world, dev, args.log2n, n_total=1 << args.log2n)
        torch.cuda.synchronize()
        try:
            srec = halo_leg(swl, head, args, world, barrier, red_dev, not args.no_parity)
            spans = gather_floats(float(swl.n), world, red_dev)
            strong = {"total_samples": 1 << args.log2n, "samples_per_rank": {"max": int(max(spans)),
                                                                              "min": int(min(spans))},
                      **{k: v for k, v in srec.items() if not k.startswith("_") and k != "parallelism"},
                      "scaling": "strong", "halo_source": head}
        except LegFailed as exc:
            strong = {"total_samples": 1 << args.log2n, "error": str(exc), "halo_source": head}
        del swl
        for rec in legs.values():
            for k in [k for k in rec if k.startswith("_")]:
                del rec[k]
    else:
        elapsed, t_issue, kern_avg_s = measure(wl, args.steps, args.warmup, args.roofline_ramp,
                                               args.roofline_launches, world, barrier, red_dev)
        kern_ranks = gather_floats(kern_avg_s, world, red_dev)
        halo = None
        failed = gate_failures(wl, world, red_dev) if wl.sharded_1d else []
        if failed:
            if rank == 0:
                timeout = wl.halo_src.timeout_s
                emit_result(json.dumps({"metric": METRIC, "value": None, "unit": wl.unit, "n_gpus": world,
                                        "error": f"halo gate timed out (a neighbour's epoch did not arrive within "
                                                 f"{timeout} s) on rank(s) {failed}", "config": wl.config}))
            print(f"bench.py: halo gate timed out on rank(s) {failed}", file=sys.stderr)
            if dist.is_initialized():
                dist.destroy_process_group()
            return 3
        # parity: full output vs the C oracle (every rank, its own segment with the received halos)
        parity = "skipped"
        if not args.no_parity:
            ok = wl.matches(wl.oracle(_cpu_threads()))
            if world > 1:
                f = torch.tensor([0 if ok else 1], device=red_dev)
                dist.all_reduce(f, op=dist.ReduceOp.MAX)
                ok = int(f.item()) == 0
            parity = "bit-exact vs oracle (full output, every rank)" if ok else "MISMATCH"
    n_roof = max(1, args.roofline_launches)

    # CPU legs: rank 0 only, at every N, after the GPU legs (the other ranks wait at the barrier below)
    cpu = cpu_np = cpu_np_mt = cpu_loop = None
    if rank == 0 and args.cpu_seconds > 0:
        nthr = _cpu_threads()
        wl.oracle(nthr)  # warm (page-in, thread pool)
        reps, tc0 = 0, time.perf_counter()
        while True:
            wl.oracle(nthr)
            reps += 1
            if time.perf_counter() - tc0 >= args.cpu_seconds:
                break
        tc = time.perf_counter() - tc0
        np_only = args.workload in NUMPY_ONLY
        what = "NumPy restatement (oracle/fir_oracle.py)" if np_only else \
            f"C oracle (oracle/fir_oracle.c, OpenMP {nthr} threads)"
        cpu = {"value": round(wl.units * reps / tc / 1e9, 4), "unit": wl.unit, "cores": 1 if np_only else nthr,
               "kind": "port", "sample": f"{what} on the full per-GPU workload ({wl.units} units) x {reps} "
                                         f"repetitions, {tc:.1f} s"}
        tn0 = time.perf_counter()
        done = wl.numpy_oracle(1 << 24)
        tn = time.perf_counter() - tn0
        cpu_np = {"value": round(done / tn / 1e9, 5), "unit": wl.unit, "cores": 1, "kind": "port",
                  "sample": f"NumPy restatement (oracle/fir_oracle.py, int64 accumulation) on the first {done} "
                            f"units of the same input, {tn:.1f} s"}
        # the same NumPy path on the host's cores (BASELINE.json: "NumPy CPU path timed on the host
        # cores (core count stated)"): contiguous slices on a thread pool
        tm0 = time.perf_counter()
        done_m = wl.numpy_oracle_threads(1 << 26, nthr)
        tm = time.perf_counter() - tm0
        cpu_np_mt = {"value": round(done_m / tm / 1e9, 5), "unit": wl.unit, "cores": nthr, "kind": "port",
                     "sample": f"NumPy restatement on the first {done_m} units, {nthr} slices on a thread pool, "
                               f"{tm:.1f} s"}
        if args.workload in ("fir1d_i16", "fir1d_u8"):  # the reference's own per-sample Python loop
            from oracle import fir_oracle as fo

            m = 1 << 16
            tl0 = time.perf_counter()
            fo.fir1d_loop(wl.x_host.reshape(-1)[:m], wl.taps.h, 12, 32,
                          fo.OUT_I32 if args.workload == "fir1d_i16" else fo.OUT_U8_SAT)
            tl = time.perf_counter() - tl0
            cpu_loop = {"value": round(m / tl / 1e9, 7), "unit": wl.unit, "cores": 1, "kind": "port",
                        "sample": f"the reference's per-sample x per-tap Python loop (oracle.fir1d_loop, "
                                  f"fir_1d_fixed_ref.py:94-128) on the first {m} samples, {tl:.2f} s"}

    barrier()  # rank 0's CPU legs are done

    traffic = pmc_traffic(wl)

    total_units = wl.units * world * args.steps
    value = total_units / elapsed / 1e9
    alg_bytes = wl.alg_bytes
    achieved = alg_bytes / kern_avg_s / 1e9
    line = {
        "metric": METRIC if args.workload == "fir1d_i16" else f"{wl.unit}, {wl.config['workload']}",
        "value": round(value, 3),
        "unit": wl.unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": wl.dtype,
        "data": "synthetic (numpy default_rng seed 20260227 + rank), resident in HBM before timing",
        "config": wl.config,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "fir2d_mfma_kernel" if wl.gen2d else KERNELS[args.workload],
                     "limiter": ("HBM (int8 MFMA Toeplitz rows, 32-row strips walking alternately down and up; "
                                 "PMC 1.008x, DESIGN.md §5)" if wl.gen2d else
                                 "HBM (separable packed-16 strips; alternate strips walk up so the rows two "
                                 "strips share are read once, PMC 1.001x; DESIGN.md §5)")
                     if args.workload == "fir2d_u8" else "HBM",
                     "kernel_avg_us": round(kern_avg_s * 1e6, 2), "algorithmic_bytes_per_launch": alg_bytes,
                     "kernel_avg_us_ranks": {"max": round(max(kern_ranks) * 1e6, 2),
                                             "min": round(min(kern_ranks) * 1e6, 2)},
                     "timing": f"HIP events around {n_roof} back-to-back launches of the kernel after "
                               f"{max(0, args.roofline_ramp)} untimed ones and at least {RAMP_MS:g} ms of them"
                               if args.roofline_ramp > 0 else
                               f"HIP events around {n_roof} back-to-back launches of the kernel, no ramp"},
        "cpu_baseline": cpu,
        "cpu_baseline_numpy": cpu_np,
        "cpu_baseline_numpy_threads": cpu_np_mt,
        "cpu_baseline_python_loop": cpu_loop,
        "parity": parity,
        "host_issue_us_per_step": round(t_issue / args.steps * 1e6, 1),
    }
    if os.environ.get("FIR_BENCH_REHEARSAL"):
        line["config"] = dict(line["config"], rehearsal=(
            f"{os.environ['FIR_BENCH_REHEARSAL']}: gloo process group, ranks share the GPU's HBM; not a "
            "scaling number"))
    if halo is not None:
        line["config"] = dict(line["config"], halo=halo)
    if legs is not None:
        line["legs"] = legs
        line["strong_scaling"] = strong
    if wl.sharded_1d and world == 1:
        line["config"] = dict(wl.config, rehearsal=f"FIR_SELF_HALO=1: {wl.halo_kind} halo hand-off with itself every "
                                                    f"step (ring of one), gate mode {GATE_MODE}")
    subs_ok = True
    if sub_configs and world == 1:
        line["configs"], subs_ok = run_sub_configs(args, dev)
    if rank == 0:
        emit_result(json.dumps(line))
    if dist.is_initialized():
        torch.cuda.synchronize()
        barrier()  # no rank unmaps or frees its segment while a neighbour may still read it
        if isinstance(wl.halo_src, sharded.XgmiHalo) and legs is None:
            wl.halo_src.close()
        dist.destroy_process_group()
    return 0 if parity != "MISMATCH" and subs_ok else 1


if __name__ == "__main__":
    raise SystemExit(main())

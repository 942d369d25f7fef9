"""Long-vector sharding across ranks with an (L-1)-sample halo.

One process per GPU (``torch.distributed``; backend "nccl" is RCCL on ROCm, "gloo" for the
CPU tests).  A signal of N samples is cut into contiguous segments, one per rank.  An L-tap
centre-aligned filter makes every segment need the last ``HL = L-1-L//2`` samples of its
left neighbour and the first ``HR = L//2`` samples of its right neighbour (times
``channels`` for interleaved complex samples); the global ends are zero padded.  That halo is
the only data that crosses GPUs.  Two sources:

* :class:`XgmiHalo` (default, :func:`make_halo_source`): each rank maps its neighbours'
  mailboxes once (HIP IPC through the C ABI); every pass is then a one-wave gate kernel that
  hands the edges over through the mailboxes (device atomics over xGMI, ordered per step, so
  segments may change every pass) followed by one launch of the FIR kernel reading the
  received halos (``torch_ops.fir1d_fixed_segment_dev``).
* :class:`HaloExchange` (fallback, ``FIR_HALO=rccl``): two point-to-point messages of a few
  bytes per neighbour pair every pass, one ``batch_isend_irecv`` group, overlapped with the
  bulk kernel; a one-block edge kernel then rewrites the HL + HR edge outputs
  (``sharded_fir1d_step`` is the one-shot form).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def halo_sizes(taps: int, channels: int = 1) -> tuple[int, int]:
    c = taps // 2
    return (taps - 1 - c) * channels, c * channels


def segment_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous split of n samples into `world` segments (the first n % world get one more)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class HaloExchange:
    """The neighbour exchange of one resident 1-D segment, set up once and posted every step.

    The receive buffers and the point-to-point op list are built once (the segment, and so
    the send views, stay the same between steps), so a step costs one ``batch_isend_irecv``
    call on the host.  ``self_ring=True`` with a world of one rehearses the exchange on a
    single device: the segment is its own left and right neighbour (a ring of one), so
    RCCL's grouped send/recv runs for real; the received halos are then the segment's own
    wrap-around samples, and the edge outputs are checked against them."""

    def __init__(self, seg: torch.Tensor, taps: int, channels: int = 1, group=None, self_ring: bool = False):
        seg = seg.reshape(-1)
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        hl, hr = halo_sizes(taps, channels)
        if seg.numel() < max(hl, hr):
            raise ValueError("segment shorter than the filter halo")
        if self_ring and (world != 1 or dist.get_backend(group) != "nccl"):
            raise ValueError("self_ring rehearses a world of one on RCCL (gloo has no send-to-self)")
        self.staged = seg.is_cuda and dist.get_backend(group) == "gloo"
        # gloo has no device point-to-point: the few halo samples are staged through the host
        # (only to rehearse the multi-rank flow on a single-GPU box; RCCL sends device buffers)
        buf_dev = torch.device("cpu") if self.staged else seg.device
        self.seg, self.group, self.hl, self.hr = seg, group, hl, hr
        self.left = self.right = None
        self.fallback_reason = None  # set by make_halo_source when the xGMI path was refused
        self._sends = []  # (device view, host staging buffer or None)
        ops = []
        left_peer = _peer(group, rank - 1) if rank > 0 else (_peer(group, rank) if self_ring else None)
        right_peer = _peer(group, rank + 1) if rank < world - 1 else (_peer(group, rank) if self_ring else None)
        # receives first, then sends; within one direction a message pair matches in order, so
        # with a ring of one (both peers = self) left <- seg[-hl:] and right <- seg[:hr] as intended
        # On the wire every halo is raw bytes (a uint8 view): RCCL's process group refuses int16.
        if left_peer is not None and hl:
            self.left = torch.empty(hl, dtype=seg.dtype, device=buf_dev)
            ops.append(dist.P2POp(dist.irecv, _wire(self.left), left_peer, group))
        if right_peer is not None and hr:
            self.right = torch.empty(hr, dtype=seg.dtype, device=buf_dev)
            ops.append(dist.P2POp(dist.irecv, _wire(self.right), right_peer, group))
        if right_peer is not None and hl:
            ops.append(dist.P2POp(dist.isend, _wire(self._send_buf(seg[seg.numel() - hl:])), right_peer, group))
        if left_peer is not None and hr:
            ops.append(dist.P2POp(dist.isend, _wire(self._send_buf(seg[:hr])), left_peer, group))
        self.ops = ops

    def _send_buf(self, view: torch.Tensor) -> torch.Tensor:
        if not self.staged:
            return view
        host = torch.empty(view.shape, dtype=view.dtype)
        self._sends.append((view, host))
        return host

    def post(self):
        """Post this step's exchange; returns the request handles (empty when staged)."""
        if not self.ops:
            return []
        for view, host in self._sends:
            host.copy_(view)
        works = dist.batch_isend_irecv(self.ops)
        if self.staged:
            wait_all(works)
            return []
        return works

    def halos(self):
        """(left, right) on the segment's device, after the works have been waited on."""
        if self.staged:
            d = self.seg.device
            return (None if self.left is None else self.left.to(d), None if self.right is None else self.right.to(d))
        return self.left, self.right


class XgmiHalo:
    """The halo hand-off over xGMI, ordered per step (the MI355X-native exchange).

    Set up once, collectively: every rank zeroes a small mailbox in its own HBM
    (``fir_halo_mailbox_init_dev``), exports it (fir_hip.ipc_export), the handles are
    all-gathered over the process group, and each rank maps its left and right neighbours'
    mailboxes (fir_hip.ipc_import).  Every step, :meth:`gate` enqueues ONE wave on this rank's
    stream (``fir_halo_gate_dev``, csrc/halo_gate.hip) after whatever wrote the step's segment:
    it publishes the segment's first HR and last HL samples with the step's epoch, waits until
    both neighbours have published the same epoch (device atomics over xGMI, no host round trip,
    no RCCL kernel), and copies their samples into the local halo buffers :meth:`halos` returns,
    which the FIR kernel then reads.  So the halos are those of THIS step even when every
    segment changes each step, and no rank overwrites what a neighbour has yet to read (two
    mailbox slots; the argument is in halo_gate.hip).  A wait is bounded (``timeout_s``); an
    expired one is reported by :meth:`check` (the halos are then zero, not stale).

    Requires peer access AND peer atomics to both neighbours' GPUs (checked before mapping;
    :func:`make_halo_source` falls back to RCCL on every rank otherwise, or if the first gated
    hand-off, checked against the edges every rank reported, does not arrive)."""

    def __init__(self, seg: torch.Tensor, taps: int, channels: int = 1, group=None, timeout_s: float | None = None,
                 self_ring: bool = False):
        import os

        import fir_hip

        from . import torch_ops

        seg = seg.reshape(-1)
        if not seg.is_cuda or not seg.is_contiguous():
            raise ValueError("XgmiHalo needs a contiguous device segment")
        # self_ring: a ring of one on one GPU (no process group needed): the rank is its own left and
        # right neighbour, its own mailbox stands in for both mapped ones, so the gate publishes,
        # waits and copies exactly as across GPUs (left <- seg[-HL:], right <- seg[:HR]); it times
        # the gate's per-step cost without other processes sharing the GPU
        world = 1 if self_ring else dist.get_world_size(group)
        rank = 0 if self_ring else dist.get_rank(group)
        hl, hr = halo_sizes(taps, channels)
        if seg.numel() < max(hl, hr):
            raise ValueError("segment shorter than the filter halo")
        self.seg, self.hl, self.hr = seg, hl, hr
        self.timeout_s = float(timeout_s if timeout_s is not None else os.environ.get("FIR_GATE_TIMEOUT_S", 10.0))
        elt = seg.element_size()
        self.hl_bytes, self.hr_bytes = hl * elt, hr * elt
        dev = seg.device.index
        self.mailbox = torch.empty(fir_hip.halo_mailbox_bytes(self.hl_bytes, self.hr_bytes), dtype=torch.uint8,
                                   device=seg.device)
        torch_ops.halo_mailbox_init_dev(self.mailbox, self.hl_bytes, self.hr_bytes)
        self.status = torch.zeros(1, dtype=torch.int32, device=seg.device)
        has_l, has_r = (rank > 0 or self_ring), (rank < world - 1 or self_ring)
        self.left = torch.zeros(hl, dtype=seg.dtype, device=seg.device) if has_l and hl else None
        self.right = torch.zeros(hr, dtype=seg.dtype, device=seg.device) if has_r and hr else None
        self._side = self._ev_seg = self._ev_gate = None  # overlapped form (gate_async / join)
        torch.cuda.synchronize(seg.device)  # zeroed before any neighbour can map it
        self._mapped = []
        if self_ring:
            own = self.mailbox.data_ptr()
            self.left_mb = own if has_l else None
            self.right_mb = own if has_r else None
            self._expect = (seg[seg.numel() - hl:].cpu().numpy().tobytes() if has_l else None,
                            seg[:hr].cpu().numpy().tobytes() if has_r else None)
            return
        handle, off = fir_hip.ipc_export(self.mailbox.data_ptr())
        mine = {"handle": handle, "offset": off, "bus": fir_hip.device_bus_id(dev),
                "first": seg[:hr].cpu().numpy().tobytes(), "last": seg[seg.numel() - hl:].cpu().numpy().tobytes()}
        infos = [None] * world
        dist.all_gather_object(infos, mine, group=group)
        self._expect = (infos[rank - 1]["last"] if rank > 0 else None, infos[rank + 1]["first"] if rank < world - 1 else None)
        self.left_mb = self.right_mb = None
        # the gate's kernel loads from and performs atomics on the neighbours' HBM: refuse (-> RCCL
        # on every rank) unless this process sees both GPUs with peer access and peer atomics
        for r in (rank - 1, rank + 1):
            if 0 <= r < world:
                bus = infos[r]["bus"]
                if not (fir_hip.peer_access(dev, bus) and fir_hip.peer_atomics(dev, bus)):
                    raise RuntimeError(f"no peer access / peer atomics from device {dev} to rank {r}'s GPU {bus}")
        try:
            if rank > 0:
                p = infos[rank - 1]
                self.left_mb = fir_hip.ipc_import(p["handle"], p["offset"], dev)
                self._mapped.append(self.left_mb)
            if rank < world - 1:
                p = infos[rank + 1]
                self.right_mb = fir_hip.ipc_import(p["handle"], p["offset"], dev)
                self._mapped.append(self.right_mb)
        except Exception:
            self.close()
            raise

    def gate(self, stream=None) -> None:
        """Enqueue this step's ordered hand-off (after the step's segment is written)."""
        from . import torch_ops

        torch_ops.halo_gate_dev(self.seg, self.hl_bytes, self.hr_bytes, self.mailbox, self.left_mb, self.right_mb,
                                self.left, self.right, self.status, self.timeout_s, stream)

    def gate_async(self, stream=None) -> None:
        """The overlapped form of :meth:`gate`: the gate runs on a high-priority side stream (its
        own hardware queue) after everything enqueued so far on ``stream`` (the step's segment is
        written), so the bulk kernel enqueued next on ``stream`` runs while the gate waits for the
        neighbours; :meth:`join` makes ``stream`` wait for the gate before the edge kernel."""
        main = stream if stream is not None else torch.cuda.current_stream(self.seg.device)
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.seg.device, priority=-1)
            self._ev_seg, self._ev_gate = torch.cuda.Event(), torch.cuda.Event()
        self._ev_seg.record(main)
        self._side.wait_event(self._ev_seg)
        self.gate(self._side)
        self._ev_gate.record(self._side)

    def join(self, stream=None) -> None:
        """``stream`` waits for the last :meth:`gate_async` (the halos are then this step's)."""
        main = stream if stream is not None else torch.cuda.current_stream(self.seg.device)
        main.wait_event(self._ev_gate)

    def halos(self):
        """(left, right) halo tensors of the last gate (None at the global ends)."""
        return self.left, self.right

    def check(self) -> None:
        """Synchronising check of the gate's status (raises if any wait timed out)."""
        import fir_hip

        if int(self.status.item()) != 0:
            raise fir_hip.FirHipError(f"halo gate: a neighbour's epoch did not arrive within {self.timeout_s} s")

    def probe(self) -> bool:
        """One gated hand-off of the resident segments (collective), checked against the edges the
        neighbours reported at setup: True when the xGMI path delivered them."""
        self.gate()
        torch.cuda.synchronize(self.seg.device)
        if int(self.status.item()) != 0:
            return False
        got = (None if self.left is None else self.left.cpu().numpy().tobytes(),
               None if self.right is None else self.right.cpu().numpy().tobytes())
        want = (self._expect[0] if self.left is not None else None, self._expect[1] if self.right is not None else None)
        return got == want

    def close(self) -> None:
        import fir_hip

        for p in self._mapped:
            fir_hip.ipc_close(p)
        self._mapped = []
        self.left_mb = self.right_mb = None


def make_halo_source(seg: torch.Tensor, taps: int, channels: int = 1, group=None, prefer: str = "xgmi"):
    """The per-step halo source for a resident segment: XgmiHalo when every rank can map its
    neighbours and the first gated hand-off arrives intact on every rank (decided collectively,
    so all ranks take the same path), else the RCCL HaloExchange, whose ``fallback_reason``
    then names the first rank that refused the xGMI path and why (the same text on every rank).
    Returns (kind, source) with kind "xgmi" or "rccl"."""
    world = dist.get_world_size(group)

    def agree(ok: int) -> bool:
        flags = [None] * world
        dist.all_gather_object(flags, ok, group=group)
        return all(flags)

    src, err = None, None
    if prefer == "xgmi":
        try:
            src = XgmiHalo(seg, taps, channels, group)
        except Exception as e:  # noqa: BLE001 - any failure selects the RCCL path on every rank
            err = e
        if agree(int(src is not None)):
            ok = 0
            try:
                ok = int(src.probe())
            except Exception as e:  # noqa: BLE001
                err = e
            if not ok and err is None:
                err = RuntimeError("the first gated hand-off did not deliver the neighbours' edges")
            if agree(ok):
                return "xgmi", src
        dist.barrier(group=group)  # every rank: no neighbour is still reading a mailbox
        if src is not None:
            src.close()
        if err is not None:
            import sys

            print(f"fir_hip.sharded: xGMI halo path unavailable ({err}); using RCCL", file=sys.stderr)
        errs = [None] * world
        dist.all_gather_object(errs, None if err is None else f"{type(err).__name__}: {err}", group=group)
        reason = next((f"rank {r}: {e}" for r, e in enumerate(errs) if e), "xGMI path refused")
    else:
        reason = f"FIR_HALO={prefer} requested"
    ex = HaloExchange(seg, taps, channels, group)
    ex.fallback_reason = reason
    return "rccl", ex


def post_halo_exchange(seg: torch.Tensor, taps: int, channels: int = 1, group=None):
    """Post the neighbour exchange for a 1-D segment.  Returns (left, right, works):
    `left` / `right` are the receive buffers (None at the global ends or when empty) and
    `works` the request handles to wait on before the halos are read.  One-shot form of
    :class:`HaloExchange` (which a step loop should build once and post every step)."""
    ex = HaloExchange(seg, taps, channels, group)
    works = ex.post()
    left, right = ex.halos()
    return left, right, works


def _wire(t: torch.Tensor) -> torch.Tensor:
    """The bytes of a contiguous tensor as uint8 (same storage)."""
    return t.view(torch.uint8)


def _peer(group, r: int) -> int:
    return r if group is None else dist.get_global_rank(group, r)


def wait_all(works) -> None:
    for w in works:
        w.wait()


def sharded_fir1d_step(seg: torch.Tensor, taps, out: torch.Tensor, *, frac_bits: int = 12, acc_bits: int = 32,
                       out_stage: int = 1, channels: int = 1, group=None, stream=None, edge_fn=None,
                       bulk_fn=None) -> torch.Tensor:
    """One sharded pass: bulk kernel || halo exchange, then the edge kernel.

    ``bulk_fn(seg, out)`` / ``edge_fn(seg, out, left, right)`` default to the HIP
    kernels of :mod:`fir_hip.torch_ops`; the CPU tests inject their own."""
    if bulk_fn is None or edge_fn is None:
        from . import torch_ops

        def bulk_fn(s, o):  # noqa: F811
            return torch_ops.fir1d_fixed_rows_dev(s, taps, frac_bits, acc_bits, out_stage, channels, out=o,
                                                  stream=stream)

        def edge_fn(s, o, left, right):  # noqa: F811
            return torch_ops.fir1d_fixed_edges_dev(s, taps, o, left, right, frac_bits, acc_bits, out_stage,
                                                   channels, stream=stream)
    ntaps = taps.n if hasattr(taps, "n") else len(taps)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return bulk_fn(seg, out)
    left, right, works = post_halo_exchange(seg.reshape(-1), ntaps, channels, group)
    bulk_fn(seg, out)
    wait_all(works)
    edge_fn(seg, out, left, right)
    return out

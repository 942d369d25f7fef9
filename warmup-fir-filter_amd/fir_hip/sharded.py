"""Long-vector sharding across ranks with an (L-1)-sample halo exchange.

One process per GPU (``torch.distributed``; backend "nccl" is RCCL over xGMI on ROCm,
"gloo" for the CPU tests).  A signal of N samples is cut into contiguous segments, one
per rank.  An L-tap centre-aligned filter makes every segment need the last
``HL = L-1-L//2`` samples of its left neighbour and the first ``HR = L//2`` samples of
its right neighbour (times ``channels`` for interleaved complex samples); the global
ends are zero padded.  That exchange is the only communication: two point-to-point
messages of a few bytes per neighbour pair, posted as one ``batch_isend_irecv`` group.

``sharded_fir1d_step`` overlaps the exchange with the bulk of the work: the full
segment kernel runs first (its zero-padded edge outputs are provisional), the halo
messages are in flight meanwhile, and a one-block edge kernel rewrites the HL + HR
edge outputs once the halos have arrived (same stream, so it is ordered after both).
"""
from __future__ import annotations

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


def post_halo_exchange(seg: torch.Tensor, taps: int, channels: int = 1, group=None):
    """Post the neighbour exchange for a 1-D segment.  Returns (left, right, works):
    `left` / `right` are the receive buffers (None at the global ends or when empty) and
    `works` the request handles to wait on before the halos are read."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    hl, hr = halo_sizes(taps, channels)
    if seg.numel() < max(hl, hr):
        raise ValueError("segment shorter than the filter halo")
    staged = seg.is_cuda and dist.get_backend(group) == "gloo"
    # gloo has no device point-to-point: the few halo samples are staged through the host
    # (only to rehearse the multi-rank flow on a single-GPU box; RCCL sends device buffers)
    buf_dev = torch.device("cpu") if staged else seg.device

    def _send(t):
        return t.cpu() if staged else t.contiguous()

    ops, left, right = [], None, None
    if rank > 0:
        if hl:
            left = torch.empty(hl, dtype=seg.dtype, device=buf_dev)
            ops.append(dist.P2POp(dist.irecv, left, _peer(group, rank - 1), group))
        if hr:
            ops.append(dist.P2POp(dist.isend, _send(seg[:hr]), _peer(group, rank - 1), group))
    if rank < world - 1:
        if hr:
            right = torch.empty(hr, dtype=seg.dtype, device=buf_dev)
            ops.append(dist.P2POp(dist.irecv, right, _peer(group, rank + 1), group))
        if hl:
            ops.append(dist.P2POp(dist.isend, _send(seg[seg.numel() - hl:]), _peer(group, rank + 1), group))
    works = dist.batch_isend_irecv(ops) if ops else []
    if staged:
        wait_all(works)
        return (None if left is None else left.to(seg.device), None if right is None else right.to(seg.device), [])
    return left, right, works


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

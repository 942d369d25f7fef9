"""The u8 metrics pass in one launch (metrics.hip, metrics_leaf_kernel): the streaming waves hand
every block's three sums and every workgroup's counts to the chain workgroup inside the launch,
each word its own ready flag (set to an unset signalling-NaN pattern by metrics_prep, published
once by a write-through atomic store, read by returning atomics until published).  A stale read
there shows as a sum off by whole blocks (or a count off by a workgroup's), so these tests re-run the pass on the SAME output and work buffers with
new data each time (consumer caches warm with the previous call's lines), in eager calls and in
graph replays, at sizes with and without a ragged last block and with one to many layers of
blocks per wave, and compare every report metric with the oracle bit for bit."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import fir_hip
from fir_hip import torch_ops
from oracle import fir_oracle as fo

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _case(rng, n):
    yi = rng.uniform(-64.0, 320.0, n)
    yf = np.clip(np.rint(yi) + rng.integers(-3, 4, n), 0, 255).astype(np.uint8)
    return yi, yf


@pytest.mark.parametrize("n", [8192, 9 * 8192 + 4352, 1000 * 8192 + 7, 2049 * 8192, 4500 * 8192 + 100])
def test_repeated_calls_same_buffers(n):
    rng = np.random.default_rng(n)
    ideal = torch.empty(n, dtype=torch.float64, device=DEV)
    fixed = torch.empty(n, dtype=torch.uint8, device=DEV)
    sums = torch.empty(9, dtype=torch.float64, device=DEV)
    work = torch.empty(int(fir_hip.lib().fir_metrics_work_bytes(n)), dtype=torch.uint8, device=DEV)
    for rep in range(4):
        yi, yf = _case(rng, n)
        ideal.copy_(torch.from_numpy(yi))
        fixed.copy_(torch.from_numpy(yf))
        torch_ops.compare_metrics_dev(ideal, fixed, out=sums, work=work)
        got = fir_hip.metrics_from_sums(sums.cpu().numpy(), n)
        assert got == fo.compute_metrics(yi, yf), (n, rep)


def test_graph_replays_new_data():
    n = 61 * 1280  # 9 full blocks + a ragged one: the graph test's image
    ideal = torch.zeros(n, dtype=torch.float64, device=DEV)
    fixed = torch.zeros(n, dtype=torch.uint8, device=DEV)
    sums = torch.empty(9, dtype=torch.float64, device=DEV)
    work = torch.empty(int(fir_hip.lib().fir_metrics_work_bytes(n)), dtype=torch.uint8, device=DEV)
    s = torch.cuda.Stream(device=DEV)
    with torch.cuda.stream(s):
        torch_ops.compare_metrics_dev(ideal, fixed, out=sums, work=work)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        torch_ops.compare_metrics_dev(ideal, fixed, out=sums, work=work)
    torch.cuda.synchronize()
    for seed in range(8):
        yi, yf = _case(np.random.default_rng(100 + seed), n)
        ideal.copy_(torch.from_numpy(yi))
        fixed.copy_(torch.from_numpy(yf))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert fir_hip.metrics_from_sums(sums.cpu().numpy(), n) == fo.compute_metrics(yi, yf), seed


def test_uneven_load_beside_other_streams():
    """The pass beside other kernels on a second stream (the producers and the chain see uneven
    load), repeated with new data."""
    n = 3000 * 8192 + 123
    rng = np.random.default_rng(7)
    ideal = torch.empty(n, dtype=torch.float64, device=DEV)
    fixed = torch.empty(n, dtype=torch.uint8, device=DEV)
    sums = torch.empty(9, dtype=torch.float64, device=DEV)
    work = torch.empty(int(fir_hip.lib().fir_metrics_work_bytes(n)), dtype=torch.uint8, device=DEV)
    other = torch.cuda.Stream(device=DEV)
    big = torch.empty(1 << 27, dtype=torch.uint8, device=DEV)
    for rep in range(3):
        yi, yf = _case(rng, n)
        ideal.copy_(torch.from_numpy(yi))
        fixed.copy_(torch.from_numpy(yf))
        torch.cuda.synchronize()
        with torch.cuda.stream(other):
            for _ in range(4):
                big.add_(1)
        torch_ops.compare_metrics_dev(ideal, fixed, out=sums, work=work)
        torch.cuda.synchronize()
        assert fir_hip.metrics_from_sums(sums.cpu().numpy(), n) == fo.compute_metrics(yi, yf), rep

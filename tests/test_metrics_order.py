"""The summation order metrics.hip restates, pinned against NumPy on the CPU.

_compute_metrics (gen_3tap_compare_report.py:84-92) takes np.mean of float64 arrays; the GPU
kernel reproduces NumPy's order of additions so that mae / rmse / mean_err are bit-identical.
This test states that order in Python (blocks of 8192 elements summed pairwise, block sums
added in order to 0.0; pairwise_sum: under 8 a loop from 0.0, up to 128 eight strided
accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus the tail in order, above that
halves at floor(n/2) rounded down to a multiple of 8) and checks it equals np.sum / np.mean for
sizes on every boundary and for image shapes.  If a NumPy upgrade changed the order, this
test fails first (CPU) and names the cause."""
from __future__ import annotations

import numpy as np
import pytest

BLOCK, LEAF = 8192, 128


def pairwise(a: np.ndarray) -> float:
    n = a.size
    if n < 8:
        res = 0.0
        for v in a.tolist():
            res += v
        return res
    if n <= LEAF:
        m = n - n % 8
        r = [float(v) for v in a[:8]]
        for i in range(8, m, 8):
            for j in range(8):
                r[j] += float(a[i + j])
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        for v in a[m:].tolist():
            res += v
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return pairwise(a[:n2]) + pairwise(a[n2:])


def numpy_order_sum(a: np.ndarray) -> float:
    flat = np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
    s = 0.0
    for b in range(0, flat.size, BLOCK):
        s += pairwise(flat[b:b + BLOCK])
    return s


@pytest.mark.parametrize("n", [1, 5, 7, 8, 9, 16, 17, 127, 128, 129, 136, 200, 255, 1000, 4095, 8191, 8192, 8193,
                               16_384 + 77, 40_003])
def test_order_equals_numpy_sum(n):
    rng = np.random.default_rng(n)
    a = rng.standard_normal(n) * np.exp2(rng.integers(-30, 31, n))
    assert numpy_order_sum(a) == np.sum(a)
    assert numpy_order_sum(a) / n == a.mean()
    assert numpy_order_sum(np.abs(a)) == np.abs(a).sum()


@pytest.mark.parametrize("shape", [(37, 1001), (120, 700), (3, 8192 + 5)])
def test_order_equals_numpy_on_images(shape):
    """2-D C-contiguous arrays: NumPy reduces the C-order flattening in the same blocks."""
    rng = np.random.default_rng(sum(shape))
    a = rng.standard_normal(shape) * np.exp2(rng.integers(-20, 21, shape))
    assert numpy_order_sum(a) == np.sum(a) == np.add.reduce(a, axis=None)
    assert numpy_order_sum(np.square(a)) / a.size == np.mean(np.square(a))


def test_sum_of_negative_zeros_is_positive_zero():
    """The reduction starts from +0.0 (so a sum of -0.0 is +0.0), as the kernel's chain does."""
    a = np.full(9000, -0.0)
    assert np.signbit(np.sum(a)) == np.signbit(numpy_order_sum(a)) == False  # noqa: E712

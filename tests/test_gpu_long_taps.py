"""GPU: filters of any length, as the reference accepts them (its MAC loop runs over any
len(h): fir_1d/model/python/fir_1d_fixed_ref.py:83-107, fir_1d/model/python/fir_1d_ref.py:49-63).

* the drop-in API (fir_1d_fixed_golden, fir_1d_ideal) with 257 / 1000 / 2048 / 4099 taps against
  the reference's own outputs (tests/golden/long_taps.npz, made by make_golden.py), x shorter
  and longer than h;
* the library entries past the old 256-tap / (L-1)*channels <= 1024 limits against the C
  oracle: L = 1000 over 2^24 int16 samples, long u8 rows, complex and many-channel signals,
  long-halo segments, fused banks, the f64 ideal rows and 2-D kernels of 17x17 and 300 taps;
* acc_bits >= 64 with a sum that could exceed 64 bits is refused, not wrapped.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import fir_hip
from conftest import GOLDEN
from fir_1d.model.python.fir_1d_fixed_ref import fir_1d_fixed_golden
from fir_1d.model.python.fir_1d_ref import fir_1d_ideal
from fir_hip import torch_ops
from oracle import c_oracle, fir_oracle as fo

DEV = torch.device("cuda:0")


def _long_cases(kind: str):
    with np.load(GOLDEN / "long_taps.npz") as d:
        xo, ho, yo = d[kind + "_x_off"], d[kind + "_h_off"], d[kind + "_y_off"]
        params = d["fixed_params"] if kind == "fixed" else None
        for i in range(len(xo) - 1):
            p = tuple(int(v) for v in params[i]) if params is not None else ()
            yield (d[kind + "_x"][xo[i]:xo[i + 1]], d[kind + "_h"][ho[i]:ho[i + 1]], p,
                   d[kind + "_y"][yo[i]:yo[i + 1]])


def test_fixed_golden_long_filters_reference_outputs():
    n = 0
    for x, h, (f, a, c), y in _long_cases("fixed"):
        got = fir_1d_fixed_golden(x.tolist(), h.tolist(), frac_bits=f, acc_bits=a, coeff_bits=c)
        assert np.array_equal(got, y), (len(h), len(x), f, a, c)
        n += 1
    assert n == 10


def test_ideal_long_filters_reference_outputs():
    n = 0
    for x, h, _, y in _long_cases("ideal"):
        got = np.asarray(fir_1d_ideal(x.tolist(), h.tolist()), dtype=np.float64)
        assert got.tobytes() == y.tobytes(), (len(h), len(x))
        n += 1
    assert n == 5


@pytest.mark.parametrize("L", [65, 257, 1000])
def test_int16_2p24_long_filter_vs_c_oracle(L):
    """L = 1000 over 2^24 int16 -> int32 (and the 64-tap boundary past it)."""
    rng = np.random.default_rng(L)
    x = rng.integers(-32768, 32768, 1 << 24, dtype=np.int16)
    hq = rng.integers(-3000, 3000, L)
    co = c_oracle()
    got = fir_hip.fir1d_fixed_rows(x, hq, 12, 32, fir_hip.OUT_I32)
    assert np.array_equal(got, co.fir1d_rows(x, hq, 12, 32, co.OUT_I32))


@pytest.mark.parametrize("L,shape,stage,dtype", [
    (257, (64, 4096), fir_hip.OUT_U8_SAT, np.uint8), (1000, (33, 1031), fir_hip.OUT_U8_SAT, np.uint8),
    (300, (17, 4096), fir_hip.OUT_I32, np.int16), (4099, (3, 5000), fir_hip.OUT_I32, np.int16),
    (513, (1, 777), fir_hip.OUT_U8_SAT, np.uint8), (4099, (2, 100), fir_hip.OUT_I32, np.int16)])
def test_long_filter_rows_vs_oracle(L, shape, stage, dtype):
    rng = np.random.default_rng(L + shape[1])
    lo, hi = (0, 256) if dtype == np.uint8 else (-32768, 32768)
    x = rng.integers(lo, hi, shape, dtype=dtype)
    hq = rng.integers(-400, 400, L)
    co = c_oracle()
    for frac, acc in ((12, 32), (16, 24), (20, 48)):
        got = fir_hip.fir1d_fixed_rows(x, hq, frac, acc, stage)
        assert np.array_equal(got, co.fir1d_rows(x, hq, frac, acc, stage)), (frac, acc)


@pytest.mark.parametrize("L,ch", [(700, 2), (3, 5000), (40, 64), (129, 16)])
def test_long_halo_channels_vs_oracle(L, ch):
    """(L-1) * channels far past the old 1024-sample halo limit."""
    rng = np.random.default_rng(L * ch)
    x = rng.integers(-32768, 32768, (3, 37 * ch), dtype=np.int16)
    hq = rng.integers(-2000, 2000, L)
    got = fir_hip.fir1d_fixed_rows(x, hq, 12, 32, fir_hip.OUT_I32, channels=ch)
    assert np.array_equal(got, fo.fir1d_rows(x, hq, 12, 32, fo.OUT_I32, channels=ch))


@pytest.mark.parametrize("L", [301, 1024])
def test_long_halo_segment_vs_oracle(L):
    """A sharded segment whose halos are hundreds of samples (fir1d_fixed_segment_dev)."""
    rng = np.random.default_rng(L)
    n = 20_000
    x = rng.integers(-32768, 32768, n, dtype=np.int16)
    hq = rng.integers(-2000, 2000, L)
    hl_n, hr_n = fo.halo_sizes(L)
    hlv = rng.integers(-32768, 32768, hl_n, dtype=np.int16)
    hrv = rng.integers(-32768, 32768, hr_n, dtype=np.int16)
    y = torch_ops.fir1d_fixed_segment_dev(torch.from_numpy(x).to(DEV), hq, torch.from_numpy(hlv).to(DEV),
                                          torch.from_numpy(hrv).to(DEV), 12, 32, fir_hip.OUT_I32)
    want = c_oracle().fir1d_rows(x, hq, 12, 32, c_oracle().OUT_I32, halo_left=hlv, halo_right=hrv)
    assert np.array_equal(y.cpu().numpy(), want)


def test_long_filter_bank_and_sharded_entries():
    rng = np.random.default_rng(5)
    x = rng.integers(0, 256, (9, 2048), dtype=np.uint8)
    bank = rng.integers(-300, 300, (3, 333))
    got = fir_hip.fir1d_fixed_rows_multi(x, bank, 12, 32, fir_hip.OUT_U8_SAT)
    for f in range(3):
        assert np.array_equal(got[f], fo.fir1d_rows(x, bank[f], 12, 32, fo.OUT_U8_SAT)), f
    x1 = rng.integers(-32768, 32768, 100_003, dtype=np.int16)
    hq = rng.integers(-2000, 2000, 999)
    got = fir_hip.fir1d_fixed_rows_sharded(x1, hq, 12, 32, fir_hip.OUT_I32, devices=[0, 0, 0])
    assert np.array_equal(got, c_oracle().fir1d_rows(x1, hq, 12, 32, c_oracle().OUT_I32))


@pytest.mark.parametrize("L", [10, 257, 1025, 4099])
def test_ideal_long_rows_vs_oracle(L):
    rng = np.random.default_rng(L)
    x = rng.integers(0, 256, (7, 3001), dtype=np.uint8)
    h = rng.uniform(-1.0, 1.0, L)
    got = fir_hip.fir1d_ideal_rows(x, h)
    assert got.tobytes() == c_oracle().fir1d_ideal_rows(x, h).tobytes()


@pytest.mark.parametrize("R,C,shape", [(17, 17, (300, 517)), (5, 60, (77, 256)), (33, 9, (70000, 16)),
                                       (1, 300, (40, 1000))])
def test_fir2d_many_taps_vs_oracle(R, C, shape):
    """2-D kernels past the old R*C <= 256 limit, and a frame taller than 65535 rows."""
    rng = np.random.default_rng(R * C)
    x = rng.integers(0, 256, shape, dtype=np.uint8)
    hq = rng.integers(-200, 200, (R, C))
    co = c_oracle()
    for stage in (fir_hip.OUT_U8_SAT, fir_hip.OUT_I32):
        got = fir_hip.fir2d_fixed(x, hq, 12, 32, stage)
        assert np.array_equal(got, co.fir2d(x, hq, 12, 32, stage)), stage


def _exact_out(x, h, idx, frac, acc_bits, stage):
    """The reference's arithmetic (fir_1d_fixed_ref.py:94-126, unbounded ints) at outputs idx:
    chunked int64 partial sums (each < 2^57) added as Python ints, masked to acc_bits, sign
    restored, rounded, staged (OUT_I32: the int32 the library stores, its low 32 bits)."""
    x = np.asarray(x, np.int64)
    h = np.asarray(h, np.int64)
    c, out = h.size // 2, []
    xp = np.concatenate([np.zeros(h.size, np.int64), x, np.zeros(h.size, np.int64)])
    for n in idx:
        # sum_k h[k] x[n - k + c]: window x[n + c - L + 1 .. n + c] reversed
        w = xp[h.size + n + c - h.size + 1:h.size + n + c + 1][::-1]
        acc = sum(int(np.dot(h[i:i + 1024], w[i:i + 1024])) for i in range(0, h.size, 1024))
        acc &= (1 << acc_bits) - 1
        if acc & (1 << (acc_bits - 1)):
            acc -= 1 << acc_bits
        v = (acc + (1 << (frac - 1))) >> frac
        out.append(min(max(v, 0), 255) if stage == fo.OUT_U8_SAT else ((v + (1 << 31)) & 0xFFFFFFFF) - (1 << 31))
    return out


def test_acc64_wide_sums_are_exact():
    """acc_bits >= 64 means the reference's unbounded sum (fir_1d_fixed_ref.py:94-115): past
    2^63 the library sums in 128 bits.  int16 samples of the taps' alternating sign times
    alternating taps of +-2^31 make every full-window sum about 2^63.1; checked against the
    reference's arithmetic on Python ints; then a shard's edges and the 2-D generic kernel."""
    rng = np.random.default_rng(64)
    L = (1 << 17) + 1001
    n = (1 << 17) + 2048
    hq = np.full(L, (1 << 31) - 1, np.int64)
    hq[1::2] = -(1 << 31)
    x = np.where(np.arange(n) % 2 == 0, 32767, -32768).astype(np.int16)
    x[rng.integers(0, n, 500)] = rng.integers(-32768, 32768, 500)
    idx = list(range(0, 32)) + list(range(n // 2 - 32, n // 2 + 32)) + list(range(n - 32, n))
    for frac, acc in ((12, 64), (12, 100), (40, 128), (70, 96), (12, 63)):
        for stage in (fir_hip.OUT_U8_SAT, fir_hip.OUT_I32):
            got = fir_hip.fir1d_fixed_rows(x, hq, frac, acc, stage)
            want = _exact_out(x, hq, idx, frac, acc, stage)
            assert [int(got[i]) for i in idx] == want, (frac, acc, stage)
    # a shard's edge outputs through the same 128-bit sums (fir1d_fixed_edges_dev)
    m = 4096
    hl_n, hr_n = fo.halo_sizes(L)
    full = np.where(np.arange(hl_n + m + hr_n) % 2 == 0, 32767, -32768).astype(np.int16)
    hlv, xs, hrv = full[:hl_n].copy(), full[hl_n:hl_n + m].copy(), full[hl_n + m:].copy()
    y = torch_ops.fir1d_fixed_segment_dev(torch.from_numpy(xs).to(DEV), hq, torch.from_numpy(hlv).to(DEV),
                                          torch.from_numpy(hrv).to(DEV), 12, 80, fir_hip.OUT_U8_SAT)
    eidx = list(range(0, 32)) + list(range(m - 32, m))
    want = _exact_out(full, hq, [hl_n + i for i in eidx], 12, 80, fo.OUT_U8_SAT)
    got = y.cpu().numpy()
    assert [int(got[i]) for i in eidx] == want
    # 2-D: 2^23 taps of near-2^31 on u8 pixels reach 2^62 * 255 > 2^63
    img = np.full((3, 5), 255, np.uint8)
    k2 = np.full((1 << 11, 1 << 12), (1 << 31) - 1, np.int64)
    got2 = fir_hip.fir2d_fixed(img, k2, 12, 100, fir_hip.OUT_I32)
    # every output sees the 3 x 5 frame (all 255) under taps of one value: sum = 15 * 255 * h
    s = 15 * 255 * ((1 << 31) - 1)
    q = ((s + (1 << 11)) >> 12) & 0xFFFFFFFF
    assert (got2 == (q - (1 << 32) if q >= (1 << 31) else q)).all()


def test_table_cache_evicts_only_idle_tables():
    """More distinct long tap tables than the per-device cache budget (256 MiB): 20 filters of
    2^22 taps (16 MiB each) on the generic kernel, plus MFMA fragment tables, from two host
    threads on two streams; every result bit-exact (dev_tables.hip frees a table only after the
    launches that used it completed, never under a launch in flight)."""
    import threading

    co = c_oracle()
    rng = np.random.default_rng(2222)
    x = rng.integers(0, 256, 96, dtype=np.uint8)
    L = 1 << 22
    results, errors = {}, []

    def worker(tid):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream(device=DEV)
            with torch.cuda.stream(s):
                xd = torch.from_numpy(x).to(DEV)
                for k in range(10):
                    hq = np.zeros(L, dtype=np.int32)
                    idx = np.random.default_rng(100 * tid + k).integers(0, L, 64)
                    hq[idx] = np.random.default_rng(7 + 100 * tid + k).integers(-4096, 4096, 64)
                    hq[L // 2 - 2:L // 2 + 3] += np.array([-256, -1024, 6656, -1024, -256], dtype=np.int32)
                    y = torch_ops.fir1d_fixed_rows_dev(xd, hq, 12, 32, fir_hip.OUT_U8_SAT)
                    results[(tid, k)] = (hq, y)
                s.synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    for (tid, k), (hq, y) in sorted(results.items(), key=lambda kv: kv[0]):
        want = co.fir1d_rows(x.reshape(1, -1), hq, 12, 32, co.OUT_U8_SAT).reshape(-1)
        assert np.array_equal(y.cpu().numpy(), want), (tid, k)
    # matrix-core fragment tables keyed by the taps: 300 distinct 257-tap filters, each exact
    xs = rng.integers(0, 256, (4, 4096), dtype=np.uint8)
    for k in range(300):
        hq = np.random.default_rng(9000 + k).integers(-300, 300, 257).astype(np.int32)
        if k % 37 == 0:
            got = fir_hip.fir1d_fixed_rows(xs, hq, 12, 32, fir_hip.OUT_U8_SAT)
            assert np.array_equal(got, co.fir1d_rows(xs, hq, 12, 32, co.OUT_U8_SAT)), k
        else:
            fir_hip.fir1d_fixed_rows(xs, hq, 12, 32, fir_hip.OUT_U8_SAT)


# every instantiation of fir1d_mfma_run_kernel: one chunk of 4 .. 12 k-steps (one tile per run,
# 290 / 322 taps: 11 / 12), 14, 16 (354-450 taps), u8 out 18 .. 32 (500-930 taps; int32 out: several
# chunks of 8 .. 16 past 16); several chunks of 6 and 8 (4-tile runs, u8 out past 32)
@pytest.mark.parametrize("L", [65, 66, 100, 129, 130, 162, 194, 257, 258, 290, 322, 354, 386, 449, 450, 500, 580, 660,
                               720, 800, 860, 900, 930, 1000, 2048,
                               2658, 4099])
def test_u8_long_filter_run_kernel_vs_oracle(L):
    """u8 filters past 64 taps (fir1d_mfma_run_kernel: runs of 1-2 tiles sharing each chunk of
    tap fragments, LDS-DMA windows): every chunk length and one- or several-chunk form, rows
    whose runs cross row ends, one long row, both stages, the no-wrap fast form, 24-bit wrap and
    32-bit taps near the int16 byte-split limit."""
    rng = np.random.default_rng(L)
    co = c_oracle()
    shapes = [(16, 4096), (5, 5 * 1024 + 8), (1, (1 << 18) + 64)]
    for shape in shapes:
        x = rng.integers(0, 256, shape, dtype=np.uint8)
        for frac, acc, amp in ((12, 32, 400), (16, 24, 3000), (12, 32, 32639)):
            hq = rng.integers(-amp, amp + 1, L)
            for stage in (fir_hip.OUT_U8_SAT, fir_hip.OUT_I32):
                got = fir_hip.fir1d_fixed_rows(x, hq, frac, acc, stage)
                want = co.fir1d_rows(x, hq, frac, acc, stage)
                assert np.array_equal(got, want), (shape, frac, acc, amp, stage)


def _hann_taps(L: int, kind: str, scale: float = 1.0) -> np.ndarray:
    w = np.hanning(L + 2)[1:-1]
    if kind == "smooth":
        h = w / w.sum()
    else:  # windowed low-pass sinc, cutoff 0.1
        n = np.arange(L) - (L - 1) / 2
        h = 0.2 * np.sinc(0.2 * n) * w
        h /= h.sum()
    return np.rint(h * 4096 * scale).astype(np.int64)


# One-chunk u8 filters whose high byte plane is zero in some k-steps (fir1d_mfma_run_kernel HN =
# 0 / 2 / 4: a Q4.12 filter's taps mostly fit a signed byte): all small taps, a large centre
# (the windowed sinc), two large taps one or several k-steps apart (past 4 k-steps: both planes
# everywhere), large taps at the filter's ends, and one large tap on the first / last k-step.
def _mixed_plane_filters(L: int, rng) -> dict:
    f = {"smooth": _hann_taps(L, "smooth"), "sinc": _hann_taps(L, "sinc"),
         "sinc_x3": _hann_taps(L, "sinc", 3.0)}
    small = rng.integers(-128, 128, L)
    for name, pos in (("spike_mid", [L // 2]), ("spikes_near", [L // 2, L // 2 + 40]),
                      ("spikes_far", [3, L - 4]), ("spike_first", [0]), ("spike_last", [L - 1]),
                      ("spikes_3steps", [L // 2 - 50, L // 2 + 50])):
        h = small.copy()
        h[np.clip(pos, 0, L - 1)] = rng.choice([-2000, 1500, 129, -129], len(pos))
        f[name] = h
    f["edge_127"] = np.where(rng.random(L) < 0.5, 127, -128)
    return f


@pytest.mark.parametrize("L", [66, 100, 129, 162, 257, 290, 386, 450, 580, 800, 930])
def test_u8_long_filter_high_plane_skip_vs_oracle(L):
    rng = np.random.default_rng(1000 + L)
    co = c_oracle()
    for shape in [(16, 4096), (3, 3 * 1024 + 24)]:
        x = rng.integers(0, 256, shape, dtype=np.uint8)
        x[0, :] = 255
        for name, hq in _mixed_plane_filters(L, rng).items():
            for frac, acc in ((12, 32), (14, 24)):
                got = fir_hip.fir1d_fixed_rows(x, hq, frac, acc, fir_hip.OUT_U8_SAT)
                want = co.fir1d_rows(x, hq, frac, acc, fir_hip.OUT_U8_SAT)
                assert np.array_equal(got, want), (shape, name, frac, acc)


def test_table_survives_its_stream_destroyed_mid_launch():
    """A tap table still read by launches on a stream that is destroyed while they run: a new
    stream (which may reuse the destroyed one's handle) uses the same table, then more distinct
    tables than the cache budget force eviction.  The cache keeps one event per use and never
    re-records a pending one (dev_tables.hip), so the table outlives every launch that reads it
    and all outputs equal the oracle (the old per-(table, stream) re-record trusted
    a reused handle)."""
    import ctypes
    from types import SimpleNamespace

    hip = ctypes.CDLL("libamdhip64.so")  # the HIP runtime already in the process (torch's / the library's)
    co = c_oracle()
    rng = np.random.default_rng(31)
    x = rng.integers(0, 256, 8192, dtype=np.uint8)
    L = 1 << 20  # generic kernel, taps read from a 4 MiB device table
    hq = np.zeros(L, dtype=np.int32)
    hq[rng.integers(0, L, 256)] = rng.integers(-4096, 4096, 256)
    hq[L // 2 - 1:L // 2 + 2] += np.array([1024, 2048, 1024], dtype=np.int32)
    want = co.fir1d_rows(x.reshape(1, -1), hq, 12, 32, co.OUT_U8_SAT).reshape(-1)
    torch.cuda.set_device(0)
    xd = torch.from_numpy(x).to(DEV)
    ys = [torch.full(x.shape, 7, dtype=torch.uint8, device=DEV) for _ in range(4)]
    torch.cuda.synchronize()

    def new_stream():
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        return SimpleNamespace(cuda_stream=h.value)

    sa = new_stream()
    for y in ys[:3]:  # queued work that reads the table for a while
        torch_ops.fir1d_fixed_rows_dev(xd, hq, 12, 32, fir_hip.OUT_U8_SAT, out=y, stream=sa)
    assert hip.hipStreamDestroy(ctypes.c_void_p(sa.cuda_stream)) == 0  # may return with the launches in flight
    sb = new_stream()
    torch_ops.fir1d_fixed_rows_dev(xd, hq, 12, 32, fir_hip.OUT_U8_SAT, out=ys[3], stream=sb)
    small = torch.from_numpy(rng.integers(0, 256, 96, dtype=np.uint8)).to(DEV)
    big = 1 << 22  # 16 MiB tables: 20 of them pass the 256 MiB budget, so idle tables are evicted
    outs = []
    for k in range(20):
        h2 = np.zeros(big, dtype=np.int32)
        h2[big // 2] = 4096 + k
        outs.append((h2, torch_ops.fir1d_fixed_rows_dev(small, h2, 12, 32, fir_hip.OUT_U8_SAT, stream=sb)))
    torch.cuda.synchronize()
    assert hip.hipStreamDestroy(ctypes.c_void_p(sb.cuda_stream)) == 0
    for y in ys:
        assert np.array_equal(y.cpu().numpy(), want)
    s = small.cpu().numpy().reshape(1, -1)
    for h2, y in outs[::5]:
        assert np.array_equal(y.cpu().numpy(), co.fir1d_rows(s, h2, 12, 32, co.OUT_U8_SAT).reshape(-1))

"""The device entries (`*_dev` in include/fir_hip.h) enqueue on the caller's stream and never
allocate or synchronise, so a whole device-resident pass can be captured once into a hipGraph
(torch.cuda.CUDAGraph on ROCm) and replayed for new data: here one image's fixed 4-filter bank,
float64 ideal outputs, report metrics and restore conversion, plus the int16 -> int32 path and a
2-D filter, replayed over three different inputs and checked against the C oracle each time.
"""
from __future__ import annotations

import numpy as np
import torch

import fir_hip
from fir_hip import torch_ops
from oracle import c_oracle, fir_oracle as fo

DEV = torch.device("cuda:0")
BANK3 = [[1365] * 3, [1024, 2048, 1024], [-4096, 0, 4096], [-512, 5120, -512]]  # h_coeff_3tap_map, Q4.12
SHARPEN5 = [-256, -1024, 6656, -1024, -256]
SHARPEN5_F64 = [-1 / 16, -4 / 16, 26 / 16, -4 / 16, -1 / 16]
K2D = (np.outer([1, 4, 6, 4, 1], [1, 4, 6, 4, 1]) * 16).tolist()


def test_captured_pipeline_replays_bit_exact():
    H, W, N16 = 61, 1280, 1 << 18
    s = torch.cuda.Stream(device=DEV)
    x = torch.zeros((H, W), dtype=torch.uint8, device=DEV)          # static inputs
    x16 = torch.zeros(N16, dtype=torch.int16, device=DEV)
    bank = torch.empty((4, H, W), dtype=torch.uint8, device=DEV)    # static outputs
    ideal = torch.empty((H, W), dtype=torch.float64, device=DEV)
    sums = torch.empty(9, dtype=torch.float64, device=DEV)
    rest = torch.empty((H, W), dtype=torch.uint8, device=DEV)
    y16 = torch.empty(N16, dtype=torch.int32, device=DEV)
    y2d = torch.empty((H, W), dtype=torch.uint8, device=DEV)
    mwork = torch.empty(int(fir_hip.lib().fir_metrics_work_bytes(H * W)), dtype=torch.uint8, device=DEV)
    rwork = torch.empty(int(fir_hip.lib().fir_restore_work_bytes()), dtype=torch.uint8, device=DEV)
    taps16 = torch_ops.Taps(SHARPEN5)

    def step():
        torch_ops.fir1d_fixed_rows_multi_dev(x, BANK3, 12, 32, fir_hip.OUT_U8_SAT, out=bank)
        torch_ops.fir1d_ideal_rows_dev(x, SHARPEN5_F64, out=ideal)
        torch_ops.compare_metrics_dev(ideal, bank[3], out=sums, work=mwork)
        torch_ops.restore_u8_dev(ideal, fir_hip.RESTORE_NORMALIZE, out=rest, work=rwork)
        torch_ops.fir1d_fixed_rows_dev(x16, taps16, 12, 32, fir_hip.OUT_I32, out=y16)
        torch_ops.fir2d_fixed_dev(x, K2D, 12, 32, fir_hip.OUT_U8_SAT, out=y2d)

    with torch.cuda.stream(s):  # warm the entry points outside the capture
        step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        step()
    torch.cuda.synchronize()

    co = c_oracle()
    for seed in (1, 2, 3):
        rng = np.random.default_rng(seed)
        xh = rng.integers(0, 256, (H, W), dtype=np.uint8)
        x16h = rng.integers(-32768, 32768, N16, dtype=np.int16)
        x.copy_(torch.from_numpy(xh))
        x16.copy_(torch.from_numpy(x16h))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        for f, h in enumerate(BANK3):
            assert np.array_equal(bank[f].cpu().numpy(), co.fir1d_rows(xh, h, 12, 32, 0)), (seed, f)
        ideal_ref = co.fir1d_ideal_rows(xh, SHARPEN5_F64)
        assert np.array_equal(ideal.cpu().numpy().view(np.uint64), ideal_ref.view(np.uint64))
        m = fir_hip.metrics_from_sums(sums.cpu().numpy(), H * W)
        ref = fo.compute_metrics(ideal_ref, co.fir1d_rows(xh, BANK3[3], 12, 32, 0))
        assert m == ref, seed  # every report metric bit for bit (NumPy's summation order)
        assert np.array_equal(rest.cpu().numpy(), fo.to_u8_normalized(ideal_ref))
        assert np.array_equal(y16.cpu().numpy(), fo.fir1d_i16_i32(x16h, SHARPEN5))
        assert np.array_equal(y2d.cpu().numpy(), co.fir2d(xh, np.asarray(K2D), 12, 32, 0))

"""fir1d_fixed_images_multi_dev: the pipeline stage's images in one call (one launch per 8 images
and 4 filters for u8 -> sat-u8 banks; fir1d_reg_batch_kernel) must equal the per-image calls and
the oracle, and the golden images must reproduce the reference's output hashes."""
import hashlib

import numpy as np
import pytest
import torch

import fir_hip
from fir_hip import torch_ops
from fir_1d.sim.vector.h_coeff import h_coeff_3tap_map, h_coeff_5tap_map
from oracle import fir_oracle as fo

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _want(x, hq, stage=fir_hip.OUT_U8_SAT, frac=12):
    return np.stack([fo.fir1d_rows(x, h, frac, 32, stage) for h in hq])


def _run(xs, hq, stage=fir_hip.OUT_U8_SAT, frac=12):
    outs = torch_ops.fir1d_fixed_images_multi_dev([torch.from_numpy(x).to(DEV) for x in xs], hq, frac, 32, stage)
    torch.cuda.synchronize()
    return [o.cpu().numpy() for o in outs]


def test_golden_images_match_reference_hashes(images, image_outputs):
    """The 7 golden images x each bank in one call: the reference's 56 fixed-output SHA-256s."""
    by_key = {(o["case_stem"], o["tap"], o["coeff_name"]): o["fixed_u8_sha256"] for o in image_outputs["outputs"]}
    stems = list(images)
    for tap, bank in (("3tap", h_coeff_3tap_map), ("5tap", h_coeff_5tap_map)):
        hq = np.stack([fo.quantize_h(h) for h in bank.values()])
        got = _run([images[s] for s in stems], hq)
        for s, ys in zip(stems, got):
            for name, y in zip(bank, ys):
                assert hashlib.sha256(np.ascontiguousarray(y).tobytes()).hexdigest() == by_key[(s, tap, name)], \
                    (s, tap, name)


@pytest.mark.parametrize("F", [1, 2, 4, 6])
def test_mixed_shapes_vs_oracle(F):
    """Aligned and ragged widths, one-row and tiny images, an empty image, a width below the
    register kernel's minimum (per-image path) and more than 8 images (two batch launches)."""
    rng = np.random.default_rng(F)
    shapes = [(37, 1280), (29, 4499), (1, 777), (3, 64), (0, 50), (5, 17), (11, 1283), (2, 9), (64, 64),
              (7, 100), (13, 4096), (1, 16)]
    xs = [rng.integers(0, 256, s, dtype=np.uint8) for s in shapes]
    for x in xs:
        if x.size:
            x[:, :3] = 255
            x[:, -3:] = 255
    hq = rng.integers(-3000, 3000, (F, 3))
    if F > 1:
        hq[1] = np.array([1, 2, 1]) << 10  # packed-16 form beside the v_dot2 ones
    got = _run(xs, hq)
    for s, x, y in zip(shapes, xs, got):
        assert y.shape == (F,) + s
        assert np.array_equal(y, _want(x, hq)), s


@pytest.mark.parametrize("L", [1, 2, 5, 9])
def test_tap_counts_and_stages_vs_per_image_calls(L):
    """Every tap count the register kernel takes; int32 stages and int16 images go image by image
    through the same entry, with identical results."""
    rng = np.random.default_rng(L + 40)
    xs = [rng.integers(0, 256, s, dtype=np.uint8) for s in ((17, 4499), (9, 1024), (4, 33))]
    hq = rng.integers(-2000, 2000, (3, L))
    for stage in (fir_hip.OUT_U8_SAT, fir_hip.OUT_I32):
        got = _run(xs, hq, stage)
        for x, y in zip(xs, got):
            assert np.array_equal(y, _want(x, hq, stage)), (L, stage)
    x16 = [rng.integers(-32768, 32768, s, dtype=np.int16) for s in ((5, 999), (3, 64))]
    got = _run(x16, hq[:1], fir_hip.OUT_I32)
    for x, y in zip(x16, got):
        assert np.array_equal(y, _want(x, hq[:1], fir_hip.OUT_I32))


def test_unaligned_image_pointer_takes_the_per_image_path():
    """An image that does not start on 16 bytes is filtered on its own (generic kernel), the others
    still in the batch launch; all equal the oracle."""
    rng = np.random.default_rng(5)
    base = torch.from_numpy(rng.integers(0, 256, 1 + 19 * 700, dtype=np.uint8)).to(DEV)
    xa = base[1:].view(19, 700)  # offset 1 byte
    xb = torch.from_numpy(rng.integers(0, 256, (23, 4499), dtype=np.uint8)).to(DEV)
    hq = np.array([[1365, 1365, 1365], [-512, 5120, -512]])
    outs = torch_ops.fir1d_fixed_images_multi_dev([xa, xb], hq)
    torch.cuda.synchronize()
    for x, y in zip((xa, xb), outs):
        assert np.array_equal(y.cpu().numpy(), _want(x.cpu().numpy(), hq))


def test_planes_in_their_own_buffers_at_any_byte():
    """outs[i] as a list of per-filter planes: 128-byte, 16-byte and odd plane starts, plane 0
    included (u8 planes may start at any byte, every one of them: the batch launch stores through
    byte-aligned vector types in gfx950's unaligned-access mode)."""
    rng = np.random.default_rng(9)
    shapes = [(31, 4499), (17, 1280), (1, 5000)]
    xs = [rng.integers(0, 256, sh, dtype=np.uint8) for sh in shapes]
    hq = np.array([[1365, 1365, 1365], [1024, 2048, 1024], [-4096, 0, 4096], [-512, 5120, -512]])
    keep, outs = [], []
    for n, sh in enumerate(shapes):
        ps = []
        for off in ((0, 16, 1, 7), (3, 0, 16, 5), (0, 0, 0, 0))[n]:  # image 1: plane 0 at an odd byte
            buf = torch.empty(sh[0] * sh[1] + off, dtype=torch.uint8, device=DEV)
            keep.append(buf)
            ps.append(buf[off:].view(sh))
        outs.append(ps)
    torch_ops.fir1d_fixed_images_multi_dev([torch.from_numpy(x).to(DEV) for x in xs], hq, outs=outs)
    torch.cuda.synchronize()
    for x, ps in zip(xs, outs):
        assert np.array_equal(np.stack([p.cpu().numpy() for p in ps]), _want(x, hq))


def test_errors_name_the_image_and_launch_nothing():
    x = torch.zeros((4, 64), dtype=torch.uint8, device=DEV)
    y = torch.full((1, 4, 64), 7, dtype=torch.uint8, device=DEV)
    with pytest.raises(fir_hip.FirHipError, match="outs\\[1\\]"):
        torch_ops.fir1d_fixed_images_multi_dev([x, x], [[1, 2, 1]], outs=[y, y[:, :2]])
    with pytest.raises(fir_hip.FirHipError, match="taps"):
        torch_ops.fir1d_fixed_images_multi_dev([x], np.zeros((1, 0), np.int64), outs=[y])
    torch.cuda.synchronize()
    assert int(y.min()) == 7  # nothing ran
    assert torch_ops.fir1d_fixed_images_multi_dev([], [[1, 2, 1]]) == []


def test_plan_replays_and_captures_into_a_graph():
    """ImagesMultiPlan.launch() re-issues the same call; captured into a hipGraph it replays to
    the same outputs after the inputs change in place (nothing allocated or synchronised)."""
    rng = np.random.default_rng(11)
    shapes = [(29, 4499), (5, 640), (64, 64)]
    xs = [torch.from_numpy(rng.integers(0, 256, sh, dtype=np.uint8)).to(DEV) for sh in shapes]
    hq = np.array([[1365, 1365, 1365], [1024, 2048, 1024], [-4096, 0, 4096], [-512, 5120, -512]])
    outs = [[torch.empty(sh, dtype=torch.uint8, device=DEV) for _ in range(4)] for sh in shapes]
    plan = torch_ops.ImagesMultiPlan(xs, hq, outs=outs)
    plan.launch()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):  # torch's capture stream is the current stream inside
        plan.launch()
    for trial in range(2):
        for x in xs:
            x.copy_(torch.from_numpy(rng.integers(0, 256, tuple(x.shape), dtype=np.uint8)))
        g.replay()
        torch.cuda.synchronize()
        for x, ps in zip(xs, outs):
            got = np.stack([p.cpu().numpy() for p in ps])
            assert np.array_equal(got, _want(x.cpu().numpy(), hq)), trial


def test_row_length_must_be_a_multiple_of_channels():
    """An odd-width int16 image with channels=2 is refused, as fir1d_fixed_rows_dev does,
    instead of filtering rows*(r-1) samples at row stride r-1."""
    x = torch.zeros((4, 9), dtype=torch.int16, device=DEV)
    with pytest.raises(fir_hip.FirHipError, match="multiple of channels"):
        torch_ops.fir1d_fixed_images_multi_dev([x], [[1, 2, 1]], 12, 32, fir_hip.OUT_I32, channels=2)
    ok = torch_ops.fir1d_fixed_images_multi_dev([x[:, :8].contiguous()], [[1, 2, 1]], 12, 32, fir_hip.OUT_I32,
                                                channels=2)
    torch.cuda.synchronize()
    assert ok[0].shape == (1, 4, 8)

"""pytest setup: import paths, the `gpu` marker, golden-fixture loaders.

`-m "not gpu"` runs here (no GPU): the oracle against the reference's golden vectors,
the host-side validation logic, the C-ABI exports and the sharded driver over gloo.
`-m gpu` runs on an MI355X: the HIP kernels against the oracle and the golden vectors.
"""
from __future__ import annotations

import functools
import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "warmup-fir-filter_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"
IMAGES = ROOT / "warmup-fir-filter_amd" / "fir_1d" / "sim" / "img_u8.npz"  # decoded golden inputs (package data)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libfir_hip.so")


def pytest_collection_modifyitems(config, items):
    # every test in a test_gpu_* module is a GPU test
    for item in items:
        if Path(str(item.fspath)).name.startswith("test_gpu_"):
            item.add_marker(pytest.mark.gpu)


def _unhex(v):
    return float.fromhex(v) if isinstance(v, str) else v


def load_kats(kind: str) -> list[dict]:
    recs = json.loads((GOLDEN / f"kat_{kind}.json").read_text())
    for r in recs:
        r["x"] = [_unhex(v) for v in r["x"]]
        r["h"] = [_unhex(v) for v in r["h"]]
        if "expect" in r and kind == "ideal":
            r["expect"] = [_unhex(v) for v in r["expect"]]
    return recs


@functools.lru_cache(maxsize=None)
def _ragged_arrays(name: str) -> dict:
    with np.load(GOLDEN / f"random_{name}.npz") as d:  # NpzFile re-inflates on every d[key]
        return {k: d[k] for k in d.files}


def iter_ragged(name: str):
    """Yield (x, h, params, y) from random_{fixed,ideal}.npz."""
    d = _ragged_arrays(name)
    xo, ho, yo = d["x_off"], d["h_off"], d["y_off"]
    for i in range(len(xo) - 1):
        params = tuple(int(v) for v in d["params"][i]) if d["params"].shape[1] else ()
        yield d["x"][xo[i]:xo[i + 1]], d["h"][ho[i]:ho[i + 1]], params, d["y"][yo[i]:yo[i + 1]]


def load_images() -> dict[str, np.ndarray]:
    d = np.load(IMAGES)
    return {k: d[k] for k in d.files}


def load_image_outputs() -> dict:
    return json.loads((GOLDEN / "image_outputs.json").read_text())


def load_metrics_dtypes():
    """[(name, ideal, fixed, reference metrics)] of metrics_dtypes.{npz,json}; floats decoded from
    hex, NaN as float('nan')."""
    recs = json.loads((GOLDEN / "metrics_dtypes.json").read_text())
    with np.load(GOLDEN / "metrics_dtypes.npz") as d:
        out = []
        for r in recs:
            m = {k: (v if isinstance(v, int) else (float("nan") if v == "nan" else float.fromhex(v)))
                 for k, v in r["metrics"].items()}
            out.append((r["name"], d[r["name"] + "__ideal"], d[r["name"] + "__fixed"], m))
    return out


def same_metrics(got: dict, want: dict) -> list[str]:
    """Keys whose values differ bit for bit (NaN equals NaN)."""
    import math

    bad = []
    for k, w in want.items():
        g = got[k]
        if isinstance(w, float) and math.isnan(w):
            if not (isinstance(g, float) and math.isnan(g)):
                bad.append(k)
        elif g != w or (isinstance(w, float) and math.copysign(1.0, g) != math.copysign(1.0, w)):
            bad.append(k)
    return bad


@pytest.fixture(scope="session")
def images():
    return load_images()


@pytest.fixture(scope="session")
def image_outputs():
    return load_image_outputs()

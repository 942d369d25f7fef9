#!/usr/bin/env python3
"""Run the REFERENCE's own test suite (fir_1d/sim/tests under /root/reference) against this repo's
package, in the build container (the reference never travels to the GPU box, and its test files
are not copied into this repo).

The reference's test modules import ``fir_1d.model.python.*`` and ``fir_1d.sim.vector.*``; with this
repo's package first on the path those resolve to the GPU-backed mirrors, and only the test helpers
(``fir_1d.sim.tests.output_test_common``) come from the reference.  There is no GPU here, so the
device calls are stood in for by the oracle exactly as in tests/test_stage_contract.py (the host
layer -- validation, quantisation, input preparation, the stage drivers, files -- is this repo's).
Nothing is written under /root/reference (no bytecode, no pytest cache; tmp_path is under /tmp).

Usage:  python tools/run_reference_tests.py [pytest args]
"""
import os
import sys
from pathlib import Path

sys.dont_write_bytecode = True
ROOT = Path(__file__).resolve().parents[1]
REF = Path(os.environ.get("FIR_REFERENCE", "/root/reference"))
sys.path[:0] = [str(ROOT / "warmup-fir-filter_amd"), str(ROOT), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import pytest  # noqa: E402

import fir_1d.sim  # noqa: E402  (this repo's)

fir_1d.sim.__path__.append(str(REF / "fir_1d" / "sim"))  # fir_1d.sim.tests -> the reference's helpers


class _Patch:
    def setattr(self, obj, name, value):
        setattr(obj, name, value)


def _oracle() -> None:
    import fir_hip
    from oracle import fir_oracle as fo
    from test_stage_contract import _oracle_batches

    _oracle_batches(_Patch())

    def rows(x, hq, frac_bits=12, acc_bits=32, out_stage=0, channels=1, device=0, out=None):
        x = np.asarray(x)
        y = fo.fir1d_rows(x.reshape(1, -1) if x.ndim == 1 else x, np.asarray(hq, np.int64), frac_bits, acc_bits,
                          out_stage)
        return y.reshape(x.shape)

    def ideal_rows(x, h, device=0, out=None):
        x = np.asarray(x)
        y = fo.fir1d_ideal_rows(x.reshape(1, -1) if x.ndim == 1 else x, np.asarray(h, np.float64))
        return y.reshape(x.shape)

    fir_hip.fir1d_fixed_rows = rows
    fir_hip.fir1d_ideal_rows = ideal_rows


def main() -> int:
    _oracle()
    import fir_1d.model.python.fir_1d_fixed_ref as m
    import fir_1d.model.python.fir_1d_ref as mi
    import fir_1d.sim.vector.gen_fixed_output as gf
    import fir_1d.sim.vector.gen_ideal_output as gi

    for mod in (m, mi, gf, gi):  # the modules under test are this repo's
        assert Path(mod.__file__).resolve().is_relative_to(ROOT), mod.__file__
        print("under test:", Path(mod.__file__).resolve().relative_to(ROOT))
    args = [str(REF / "fir_1d" / "sim" / "tests"), "-q", "-p", "no:cacheprovider", "--import-mode=importlib",
            "--rootdir", "/tmp", "-o", "python_files=test_*.py", *sys.argv[1:]]
    return pytest.main(args)


if __name__ == "__main__":
    raise SystemExit(main())

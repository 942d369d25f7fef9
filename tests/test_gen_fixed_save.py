"""The fixed-output stage writes a bank's files concurrently (gen_fixed_output._save_all): every
file is attempted, the outputs are the arrays given, and the first failure (in bank order) is
raised after the others were written."""
import numpy as np
import pytest

from fir_1d.sim.vector.gen_fixed_output import _save_all


def test_saves_every_file(tmp_path):
    ys = [np.full((3, 5), i, np.uint8) for i in range(4)]
    paths = [tmp_path / f"y{i}.npy" for i in range(4)]
    assert _save_all(list(zip(paths, ys))) == 4
    for p, y in zip(paths, ys):
        assert np.array_equal(np.load(p), y)
    assert _save_all([]) == 0
    assert _save_all([(tmp_path / "one.npy", ys[0])]) == 1


def test_first_failure_is_raised_after_the_others_are_written(tmp_path):
    ys = [np.full((2, 2), i, np.uint8) for i in range(3)]
    bad = tmp_path / "missing_dir" / "y1.npy"  # parent does not exist
    items = [(tmp_path / "y0.npy", ys[0]), (bad, ys[1]), (tmp_path / "y2.npy", ys[2])]
    with pytest.raises(FileNotFoundError):
        _save_all(items)
    assert np.array_equal(np.load(tmp_path / "y0.npy"), ys[0])
    assert np.array_equal(np.load(tmp_path / "y2.npy"), ys[2])

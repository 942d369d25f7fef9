"""The stages' ordered writer (stage_io.OrderedSaver, used by gen_fixed_output._save_all and the
batched stages): files are written concurrently but put in place in the stage's order, and the
first failure is the reference's own np.save error, raised after the files before it, with none
of the files after it written (the reference's one-file-at-a-time loop,
gen_fixed_output.py:92-105, stops there)."""
import os

import numpy as np
import pytest

from fir_1d.sim.vector import stage_io
from fir_1d.sim.vector.gen_fixed_output import _save_all


def test_saves_every_file(tmp_path):
    ys = [np.full((3, 5), i, np.uint8) for i in range(4)]
    paths = [tmp_path / f"y{i}.npy" for i in range(4)]
    assert _save_all(list(zip(paths, ys))) == 4
    for p, y in zip(paths, ys):
        assert np.array_equal(np.load(p), y)
        assert p.read_bytes() == _npy_bytes(tmp_path, y)  # byte-identical to np.save(path, y)
    assert _save_all([]) == 0
    assert _save_all([(tmp_path / "one.npy", ys[0])]) == 1
    assert not list(tmp_path.glob(".*.part"))


def _npy_bytes(tmp_path, y):
    p = tmp_path / "ref_np_save.npy"
    np.save(p, y)
    b = p.read_bytes()
    p.unlink()
    return b


def test_first_failure_stops_the_group_like_the_reference(tmp_path):
    ys = [np.full((2, 2), i, np.uint8) for i in range(3)]
    bad = tmp_path / "missing_dir" / "y1.npy"  # parent does not exist
    items = [(tmp_path / "y0.npy", ys[0]), (bad, ys[1]), (tmp_path / "y2.npy", ys[2])]
    with pytest.raises(FileNotFoundError) as ei:
        _save_all(items)
    with pytest.raises(FileNotFoundError) as ref:  # the reference's call, for the error text
        np.save(bad, ys[1])
    assert str(ei.value) == str(ref.value)
    assert np.array_equal(np.load(tmp_path / "y0.npy"), ys[0])
    assert not (tmp_path / "y2.npy").exists()  # the reference never reached it
    assert sorted(p.name for p in tmp_path.iterdir()) == ["y0.npy"]  # no temporary files left


def test_later_existing_files_keep_their_contents(tmp_path):
    old = np.full((2, 2), 9, np.uint8)
    np.save(tmp_path / "y2.npy", old)
    (tmp_path / "y1.npy").mkdir()  # np.save(dir) fails: IsADirectoryError
    ys = [np.full((2, 2), i, np.uint8) for i in range(3)]
    with pytest.raises(IsADirectoryError):
        _save_all([(tmp_path / f"y{i}.npy", y) for i, y in enumerate(ys)])
    assert np.array_equal(np.load(tmp_path / "y0.npy"), ys[0])
    assert np.array_equal(np.load(tmp_path / "y2.npy"), old)  # not overwritten


@pytest.mark.skipif(os.geteuid() == 0, reason="root ignores file permissions")
def test_read_only_target_raises_the_reference_permission_error(tmp_path):
    p = tmp_path / "y0.npy"
    np.save(p, np.zeros(3, np.uint8))
    p.chmod(0o444)
    with pytest.raises(PermissionError):
        _save_all([(p, np.ones(3, np.uint8))])


def test_npy_header_fast_path_accepts_only_2d_c_order_u8(tmp_path):
    a = np.arange(12, dtype=np.uint8).reshape(3, 4)
    np.save(tmp_path / "a.npy", a)
    r, c, off = stage_io.npy_u8_2d_shape(tmp_path / "a.npy")
    assert (r, c) == (3, 4)
    out = np.empty(12, np.uint8)
    assert stage_io.read_u8_2d_into(tmp_path / "a.npy", r, c, off, out)
    assert np.array_equal(out.reshape(3, 4), a)
    for name, arr in (("f", np.asfortranarray(a)), ("i16", a.astype(np.int16)), ("d1", a.reshape(-1)),
                      ("d3", a.reshape(1, 3, 4))):
        np.save(tmp_path / f"{name}.npy", arr)
        assert stage_io.npy_u8_2d_shape(tmp_path / f"{name}.npy") is None
    (tmp_path / "trunc.npy").write_bytes((tmp_path / "a.npy").read_bytes()[:-2])  # short data
    assert stage_io.npy_u8_2d_shape(tmp_path / "trunc.npy") is None
    (tmp_path / "junk.npy").write_bytes(b"not an npy file")
    assert stage_io.npy_u8_2d_shape(tmp_path / "junk.npy") is None


def test_links_are_written_through_like_np_save(tmp_path):
    """np.save writes through a symlink and into a file other names share; the ordered writer
    does the same for such targets (it does not replace the link by a new file)."""
    target = tmp_path / "target.npy"
    np.save(target, np.zeros(3, np.uint8))
    (tmp_path / "y0.npy").symlink_to(target)
    other = tmp_path / "other_name.npy"
    np.save(other, np.zeros(2, np.uint8))
    os.link(other, tmp_path / "y1.npy")
    ys = [np.full(3, 5, np.uint8), np.full(2, 6, np.uint8)]
    assert _save_all([(tmp_path / "y0.npy", ys[0]), (tmp_path / "y1.npy", ys[1])]) == 2
    assert (tmp_path / "y0.npy").is_symlink() and np.array_equal(np.load(target), ys[0])
    assert np.array_equal(np.load(other), ys[1])  # the shared file itself was rewritten


def test_largest_first_pool_runs_the_largest_pending_job_first():
    """LargestFirstPool (the restore stage's PNG writers): with its one worker held, the queued jobs
    run largest first; results and exceptions come back through the futures."""
    import threading

    pool = stage_io.LargestFirstPool(1)
    gate, started, order = threading.Event(), threading.Event(), []

    def hold():
        started.set()
        return gate.wait()
    held = pool.submit(hold, size=0)
    assert started.wait(10)  # the one worker is busy before the others are queued
    futs = [pool.submit(order.append, s, size=s) for s in (3, 50, 7, 50, 1)]
    bad = pool.submit(lambda: 1 / 0, size=2)
    gate.set()
    assert held.result(timeout=10) is True
    for f in futs:
        f.result(timeout=10)
    with pytest.raises(ZeroDivisionError):
        bad.result(timeout=10)
    assert order == [50, 50, 7, 3, 1]  # equal sizes in submission order
    pool.shutdown()
    with pytest.raises(RuntimeError):
        pool.submit(print)


def test_largest_first_pool_uses_its_workers():
    import threading

    pool = stage_io.LargestFirstPool(4)
    barrier = threading.Barrier(4, timeout=10)
    futs = [pool.submit(barrier.wait, size=i) for i in range(4)]  # only completes with 4 threads at once
    assert sorted(f.result(timeout=10) for f in futs) == [0, 1, 2, 3]
    pool.shutdown()


def test_ordered_saver_with_another_writer(tmp_path):
    """OrderedSaver with a writer / redo pair (the PNG restore): bytes are the writer's, the first
    failing item is redone by ``redo`` and raises, later items are not left behind."""
    def writer(f, y):
        if y == b"boom":
            raise OSError("writer failed")
        f.write(y)

    def redo(path, y):
        raise ValueError(f"redo {path.name}")

    saver = stage_io.OrderedSaver(workers=2, writer=writer, redo=redo, largest_first=True)
    paths = [tmp_path / f"f{i}.bin" for i in range(4)]
    for i, (p, y) in enumerate(zip(paths, [b"a", b"bb", b"boom", b"dddd"])):
        saver.submit(i, p, y, size=len(y))
    with pytest.raises(ValueError, match="redo f2.bin"):
        saver.commit()
    assert saver.failed_index == 2
    saver.close()
    assert paths[0].read_bytes() == b"a" and paths[1].read_bytes() == b"bb"
    assert not paths[2].exists() and not paths[3].exists()
    assert not list(tmp_path.glob(".*.part"))

"""The C-ABI library: it loads, exports exactly what include/fir_hip.h declares, and rejects
structurally invalid calls with FIR_EINVAL and a message — all without a GPU (no compute
call is made here)."""
from __future__ import annotations

import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

import fir_hip

HEADER = Path(__file__).resolve().parents[1] / "include" / "fir_hip.h"


def _declared() -> set[str]:
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return set(re.findall(r"^\s*(?!typedef\b)(?:const\s+)?\w+\s*\*?\s*(\w+)\s*\(", text, flags=re.M))


@pytest.fixture(scope="module")
def lib():
    if not fir_hip.lib_path().exists():
        pytest.fail(f"{fir_hip.lib_path()} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    return fir_hip.lib()


def test_header_declares_the_binding_table():
    assert _declared() == set(fir_hip.EXPORTS), "include/fir_hip.h and fir_hip.EXPORTS disagree"


def test_library_exports_every_declared_symbol(lib):
    raw = ctypes.CDLL(str(fir_hip.lib_path()))
    for name in _declared():
        assert hasattr(raw, name), name


def test_abi_version(lib):
    assert lib.fir_abi_version() == fir_hip.ABI_VERSION == 6


def test_invalid_arguments_are_rejected_without_device(lib):
    h = (ctypes.c_int32 * 3)(1, 2, 1)
    rc = lib.fir1d_fixed_rows_dev(None, 7, 1, 16, 1, h, 3, 12, 32, 0, None, None)
    assert rc == 1 and b"in_dtype" in lib.fir_last_error()
    rc = lib.fir1d_fixed_rows_dev(None, 0, 1, 16, 1, h, 0, 12, 32, 0, None, None)
    assert rc == 1 and b"taps" in lib.fir_last_error()
    rc = lib.fir1d_fixed_rows_dev(None, 0, 1, 16, 1, h, 3, 0, 32, 0, None, None)
    assert rc == 1 and b"frac_bits" in lib.fir_last_error()
    rc = lib.fir1d_fixed_rows_dev(None, 0, 1, 16, 1, h, 3, 12, 32, 0, None, None)
    assert rc == 1 and b"NULL" in lib.fir_last_error()
    rc = lib.fir2d_fixed_dev(None, 4, 4, h, 0, 3, 12, 32, 0, None, None)
    assert rc == 1
    # empty problems are valid no-ops
    assert lib.fir1d_fixed_rows_dev(None, 0, 0, 16, 1, h, 3, 12, 32, 0, None, None) == 0


def test_images_batch_argument_checks_without_device(lib):
    """fir1d_fixed_images_multi_dev refuses the whole call before anything launches, naming the
    image at fault; no images is a no-op."""
    h = (ctypes.c_int32 * 3)(1, 2, 1)
    i64x2 = ctypes.c_int64 * 2
    vpx2 = ctypes.c_void_p * 2
    xs, ys = vpx2(16, 32), vpx2(48, 64)  # never dereferenced: every call below is refused first
    assert lib.fir1d_fixed_images_multi_dev(0, None, None, None, 0, 1, h, 3, 1, 12, 32, 0, None, None) == 0
    assert lib.fir1d_fixed_images_multi_dev(-1, None, None, None, 0, 1, h, 3, 1, 12, 32, 0, None, None) == 1
    assert b"images" in lib.fir_last_error()
    assert lib.fir1d_fixed_images_multi_dev(2, None, i64x2(4, 4), i64x2(64, 64), 0, 1, h, 3, 1, 12, 32, 0, ys,
                                            None) == 1
    assert b"NULL" in lib.fir_last_error()
    assert lib.fir1d_fixed_images_multi_dev(2, xs, i64x2(4, -4), i64x2(64, 64), 0, 1, h, 3, 1, 12, 32, 0, ys,
                                            None) == 1
    assert b"image 1" in lib.fir_last_error()
    assert lib.fir1d_fixed_images_multi_dev(2, xs, i64x2(4, 4), i64x2(64, 64), 0, 1, h, 3, 0, 12, 32, 0, ys,
                                            None) == 1
    assert b"filters" in lib.fir_last_error()
    assert lib.fir1d_fixed_images_multi_dev(2, xs, i64x2(4, 4), i64x2(64, 64), 5, 1, h, 3, 1, 12, 32, 0, ys,
                                            None) == 1
    assert b"image 0" in lib.fir_last_error() and b"in_dtype" in lib.fir_last_error()


def test_errors_surface_as_firhiperror():
    with pytest.raises(fir_hip.FirHipError):
        fir_hip._taps_i32([])
    with pytest.raises(fir_hip.FirHipError):
        fir_hip._taps_i32(np.broadcast_to(np.int64(1), (fir_hip.MAX_TAPS + 1,)))  # refused before any copy
    assert fir_hip._taps_i32(np.ones(4099, np.int64)).size == 4099  # long filters are legal


def test_sharded_and_restore_argument_checks_without_device(lib):
    h = (ctypes.c_int32 * 3)(1, 2, 1)
    devs = (ctypes.c_int32 * 1)(0)
    assert lib.fir1d_fixed_rows_sharded(None, 0, 1, 16, 1, h, 3, 12, 32, 0, None, devs, 0) == 1
    assert b"ndev" in lib.fir_last_error()
    assert lib.fir1d_fixed_rows_sharded(None, 5, 1, 16, 1, h, 3, 12, 32, 0, None, devs, 1) == 1
    assert b"in_dtype" in lib.fir_last_error()
    assert lib.fir1d_fixed_rows_sharded(None, 0, 0, 16, 1, h, 3, 12, 32, 0, None, devs, 1) == 0  # empty no-op
    assert lib.fir_restore_u8_dev(None, 8, 7, None, None, None) == 1
    assert b"policy" in lib.fir_last_error()
    assert lib.fir_restore_u8_dev(None, 0, 1, None, None, None) == 0
    assert lib.fir_restore_u8_dev(None, 8, 1, None, None, None) == 1
    assert lib.fir_restore_work_bytes() >= 256
    # the metrics work buffer: fixed part + 3 float64 sums per 8192-sample block (NumPy's order)
    w0 = lib.fir_metrics_work_bytes(0)
    assert w0 > 0 and lib.fir_metrics_work_bytes(1) == w0 + 24 == lib.fir_metrics_work_bytes(8192)
    assert lib.fir_metrics_work_bytes(1 << 28) == w0 + 24 * (1 << 15)


def test_ipc_argument_checks_without_device(lib):
    off = ctypes.c_int64(0)
    handle = ctypes.create_string_buffer(64)
    p = ctypes.c_void_p(0)
    assert lib.fir_ipc_export(None, handle, ctypes.byref(off)) == 1 and b"NULL" in lib.fir_last_error()
    assert lib.fir_ipc_import(None, 0, 0, ctypes.byref(p)) == 1
    assert lib.fir_ipc_import(handle, -1, 0, ctypes.byref(p)) == 1
    assert lib.fir_ipc_close(ctypes.c_void_p(1234)) == 1 and b"fir_ipc_import" in lib.fir_last_error()
    assert lib.fir_peek(None, None, 0) == 0  # empty no-op
    assert lib.fir_peek(None, None, 8) == 1
    assert lib.fir_peek(None, None, -1) == 1
    can = ctypes.c_int32(7)
    assert lib.fir_device_bus_id(0, None, 64) == 1 and b"16 bytes" in lib.fir_last_error()
    assert lib.fir_device_bus_id(0, ctypes.create_string_buffer(8), 8) == 1
    assert lib.fir_peer_access(0, None, ctypes.byref(can)) == 1 and b"NULL" in lib.fir_last_error()
    assert lib.fir_peer_access(0, b"0000:00:00.0", None) == 1


def test_out_argument_is_checked_before_any_call():
    """``out=`` (reused host output): wrong dtype/shape/layout or an overlap with
    the input is refused in the host layer, before the library is called."""
    x = np.zeros((4, 64), np.uint8)
    h = [1, 2, 1]
    bad = [np.zeros((4, 64), np.int32), np.zeros((4, 63), np.uint8), np.zeros((64, 4), np.uint8).T,
           [[0] * 64] * 4]
    ro = np.zeros((4, 64), np.uint8)
    ro.flags.writeable = False
    for out in bad + [ro]:
        with pytest.raises(fir_hip.FirHipError):
            fir_hip.fir1d_fixed_rows(x, h, out=out)
    with pytest.raises(fir_hip.FirHipError, match="overlap"):
        fir_hip.fir2d_fixed(x, [[0, 1, 0]], out=x)
    with pytest.raises(fir_hip.FirHipError, match="overlap"):
        fir_hip.fir1d_fixed_rows_multi(x, [h], out=x[None])
    with pytest.raises(fir_hip.FirHipError, match="overlap"):
        fir_hip.fir1d_fixed_rows_sharded(x, h, out=x)
    x16 = np.zeros(128, np.int16)
    with pytest.raises(fir_hip.FirHipError, match="overlap"):  # partial overlap via a view
        fir_hip.fir1d_fixed_rows(x16[:64].view(np.uint8), h, out=x16.view(np.uint8)[64:192])


def test_stale_library_is_refused(tmp_path):
    """The library carries the id of the sources it was built from (fir_build_id); the loader
    refuses it when the sources beside it differ — one flipped source byte, no rebuild."""
    import os
    import shutil
    import subprocess
    import sys

    pkg = Path(fir_hip.__file__).resolve().parents[1]  # warmup-fir-filter_amd/
    dst = tmp_path / "tree" / pkg.name
    shutil.copytree(pkg / "fir_hip", dst / "fir_hip", ignore=shutil.ignore_patterns("__pycache__"))
    shutil.copytree(pkg / "csrc", dst / "csrc", ignore=shutil.ignore_patterns("build"))
    (dst.parent / "include").mkdir()
    shutil.copy(HEADER, dst.parent / "include" / HEADER.name)
    env = {k: v for k, v in os.environ.items() if k != "FIR_HIP_LIB"}
    probe = f"import sys; sys.path.insert(0, {str(dst)!r}); import fir_hip; fir_hip.lib(); print(fir_hip.build_id())"

    ok = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr
    assert ok.stdout.strip() == fir_hip.build_id()

    src = dst / "csrc" / "fir1d.hip"
    data = bytearray(src.read_bytes())
    i = data.index(b"gfx950")
    data[i] ^= 0x20  # 'g' -> 'G' inside a comment: the compiled code would not even change
    src.write_bytes(bytes(data))
    bad = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True)
    assert bad.returncode != 0
    assert "built from other sources" in bad.stderr


def test_torch_runtime_shared_only_when_sonames_match(tmp_path):
    """fir_hip loads PyTorch's bundled HIP/HSA runtime first only when its DT_SONAME majors equal
    those of the ROCm the library was built with: the decision reads the ELF headers of
    the real files, and a runtime of another major (here: a copy whose soname says .so.6) or a
    missing one keeps /opt/rocm's."""
    import shutil

    import fir_hip

    rocm = Path("/opt/rocm/lib")
    if not (rocm / "libamdhip64.so").exists():
        pytest.skip("no /opt/rocm here")
    assert fir_hip._elf_soname(rocm / "libamdhip64.so").startswith("libamdhip64.so.")
    same = tmp_path / "same"
    same.mkdir()
    for stem in ("libamdhip64.so", "libhsa-runtime64.so"):
        shutil.copy(rocm / stem, same / stem)
    assert fir_hip._runtime_compatible(same, rocm)
    other = tmp_path / "other"
    other.mkdir()
    shutil.copy(rocm / "libhsa-runtime64.so", other / "libhsa-runtime64.so")
    data = bytearray((rocm / "libamdhip64.so").read_bytes())
    name = fir_hip._elf_soname(rocm / "libamdhip64.so").encode()
    i = data.index(name + b"\0")
    data[i:i + len(name)] = name.replace(b".so.7", b".so.6") if b".so.7" in name else name[:-1] + b"9"
    (other / "libamdhip64.so").write_bytes(bytes(data))
    assert not fir_hip._runtime_compatible(other, rocm)
    assert not fir_hip._runtime_compatible(tmp_path / "empty", rocm)

"""ctypes binding of ``libfir_hip.so`` — the MI355X (gfx950) fixed-point FIR path.

The C ABI is declared in ``include/fir_hip.h``.  This module is the only place that
loads the library; it raises :class:`FirHipError` (a ``RuntimeError``) when the
library is missing, no gfx950 device is present, or a HIP call fails.  There is no
CPU fallback: the product path fails loudly rather than computing elsewhere.

Host-array entry points (NumPy in, NumPy out, synchronous):
    fir1d_fixed_rows, fir1d_fixed_rows_multi, fir1d_fixed_rows_sharded, fir2d_fixed,
    fir1d_ideal_rows, compare_metrics, restore_u8, and the stage drivers' image batches
    fir1d_fixed_images_multi / fir1d_ideal_images_multi (page-locked staging: host_empty)
Device entry points (torch tensors on a HIP device, enqueued on the current stream):
    see :mod:`fir_hip.torch_ops`.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import numpy as np

__all__ = [
    "FirHipError", "lib", "lib_path", "device_count", "fir1d_fixed_rows", "fir1d_fixed_rows_multi",
    "fir1d_fixed_rows_sharded", "fir2d_fixed", "fir1d_ideal_rows", "compare_metrics", "restore_u8", "IN_U8", "IN_I16",
    "OUT_U8_SAT", "OUT_I32", "RESTORE_CLIP", "RESTORE_NORMALIZE", "MAX_TAPS", "EXPORTS", "ipc_export", "ipc_import",
    "ipc_close", "peek", "IPC_HANDLE_BYTES", "device_bus_id", "peer_access", "peer_atomics", "halo_mailbox_bytes",
    "GATE_TIMEOUT", "GATE_LAYOUT", "build_id", "parse_devices", "METRIC_DTYPES", "fir1d_fixed_images_multi",
    "fir1d_ideal_images_multi", "host_empty", "TIMING_KEYS",
]

IN_U8, IN_I16 = 0, 1
OUT_U8_SAT, OUT_I32 = 0, 1
RESTORE_CLIP, RESTORE_NORMALIZE = 0, 1
MAX_TAPS = 1 << 30  # FIR_MAX_TAPS: any practical length (the reference has no limit)
IPC_HANDLE_BYTES = 64
ABI_VERSION = 6
GATE_TIMEOUT = 1  # FIR_GATE_TIMEOUT
GATE_LAYOUT = 2  # FIR_GATE_LAYOUT

_HERE = Path(__file__).resolve().parent


def lib_path() -> Path:
    return Path(os.environ.get("FIR_HIP_LIB", _HERE / "libfir_hip.so"))


class FirHipError(RuntimeError):
    """A failure inside libfir_hip (missing library, no device, HIP error, bad call)."""


_i32, _i64, _vp = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p

# symbol -> (restype, argtypes); mirrors include/fir_hip.h one to one
EXPORTS = {
    "fir_abi_version": (_i32, []),
    "fir_build_id": (ctypes.c_char_p, []),
    "fir_last_error": (ctypes.c_char_p, []),
    "fir_device_count": (_i32, [ctypes.POINTER(_i32)]),
    "fir1d_fixed_rows": (_i32, [_vp, _i32, _i64, _i64, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _i32]),
    "fir1d_fixed_rows_dev": (_i32, [_vp, _i32, _i64, _i64, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp]),
    "fir1d_fixed_rows_multi": (_i32, [_vp, _i32, _i64, _i64, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _i32]),
    "fir1d_fixed_rows_multi_dev": (_i32, [_vp, _i32, _i64, _i64, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp]),
    "fir1d_fixed_images_multi_dev": (_i32, [_i32, _vp, _vp, _vp, _i32, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _vp,
                                            _vp]),
    "fir1d_fixed_images_multi": (_i32, [_i32, _vp, _vp, _vp, _i32, _i32, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _i32,
                                        _vp, _vp, _vp]),
    "fir1d_ideal_images_multi": (_i32, [_i32, _vp, _vp, _vp, _vp, _i32, _i32, _vp, _i32, _vp, _vp, _vp]),
    "fir_host_alloc": (_i32, [_i64, ctypes.POINTER(_vp)]),
    "fir_host_free": (_i32, [_vp]),
    "fir1d_fixed_edges_dev": (_i32, [_vp, _i32, _i64, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    "fir1d_fixed_segment_dev": (_i32, [_vp, _i32, _i64, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    "fir2d_fixed": (_i32, [_vp, _i64, _i64, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _i32]),
    "fir2d_fixed_dev": (_i32, [_vp, _i64, _i64, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp]),
    "fir2d_fixed_frames": (_i32, [_vp, _i64, _i64, _i64, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _i32]),
    "fir2d_fixed_frames_dev": (_i32, [_vp, _i64, _i64, _i64, _vp, _i32, _i32, _i32, _i32, _i32, _vp, _vp]),
    "fir1d_ideal_rows": (_i32, [_vp, _i64, _i64, _vp, _i32, _vp, _i32]),
    "fir1d_ideal_rows_dev": (_i32, [_vp, _i64, _i64, _vp, _i32, _vp, _vp]),
    "fir_metrics_work_bytes": (_i64, [_i64]),
    "fir_compare_metrics": (_i32, [_vp, _vp, _i32, _i64, _vp, _i32]),
    "fir_compare_metrics_dev": (_i32, [_vp, _vp, _i32, _i64, _vp, _vp, _vp]),
    "fir1d_fixed_rows_sharded": (_i32, [_vp, _i32, _i64, _i64, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _i32]),
    "fir_restore_work_bytes": (_i64, []),
    "fir_restore_u8": (_i32, [_vp, _i64, _i32, _vp, _i32]),
    "fir_restore_u8_dev": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp]),
    "fir_ipc_export": (_i32, [_vp, _vp, ctypes.POINTER(_i64)]),
    "fir_ipc_import": (_i32, [_vp, _i64, _i32, ctypes.POINTER(_vp)]),
    "fir_ipc_close": (_i32, [_vp]),
    "fir_peek": (_i32, [_vp, _vp, _i64]),
    "fir_device_bus_id": (_i32, [_i32, ctypes.c_char_p, _i32]),
    "fir_peer_access": (_i32, [_i32, ctypes.c_char_p, ctypes.POINTER(_i32)]),
    "fir_peer_atomics": (_i32, [_i32, ctypes.c_char_p, ctypes.POINTER(_i32)]),
    "fir_halo_mailbox_bytes": (_i64, [_i64, _i64]),
    "fir_halo_mailbox_init_dev": (_i32, [_vp, _i64, _i64, _i64, _vp]),
    "fir_halo_gate_dev": (_i32, [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_double, _vp]),
}

_lib = None
_lock = threading.Lock()


def _elf_soname(path: Path) -> str | None:
    """DT_SONAME of a 64-bit little-endian ELF shared object (None if it is not one); reads the
    headers, the dynamic section and its string table only."""
    import struct

    try:
        with open(path, "rb") as f:
            hdr = f.read(64)
            if len(hdr) < 64 or hdr[:4] != b"\x7fELF" or hdr[4] != 2 or hdr[5] != 1:
                return None
            shoff, = struct.unpack_from("<Q", hdr, 0x28)
            shentsize, shnum = struct.unpack_from("<HH", hdr, 0x3A)
            f.seek(shoff)
            raw = f.read(shentsize * shnum)
            secs = [struct.unpack_from("<IIQQQQIIQQ", raw, i * shentsize) for i in range(shnum)]
            for sh in secs:
                if sh[1] != 6:  # SHT_DYNAMIC; sh_link = its string table
                    continue
                f.seek(sh[4])
                dyn = f.read(sh[5])
                strtab = secs[sh[6]]
                for off in range(0, len(dyn) - 15, 16):
                    tag, val = struct.unpack_from("<qQ", dyn, off)
                    if tag == 0:
                        break
                    if tag == 14:  # DT_SONAME
                        f.seek(strtab[4] + val)
                        return f.read(256).split(b"\0", 1)[0].decode()
    except (OSError, struct.error, IndexError, UnicodeDecodeError):
        return None
    return None


def _soname_majors(libdir: Path, stem: str) -> set[int]:
    """Major versions in the DT_SONAME (``stem.so.<major>``) of ``stem.so*`` files in ``libdir``."""
    majors = set()
    for p in {q.resolve() for q in libdir.glob(stem + ".so*")}:
        name = _elf_soname(p) if p.is_file() else None
        if name and name.startswith(stem + ".so."):
            head = name[len(stem) + 4:].split(".")[0]
            if head.isdigit():
                majors.add(int(head))
    return majors


def _runtime_compatible(torch_lib: Path, rocm_lib: Path = Path("/opt/rocm/lib")) -> bool:
    """True when torch's bundled HIP / HSA runtimes carry the same soname majors as the ROCm this
    library was built against (or that ROCm is not installed to compare with): only then may the
    library run on torch's copies.  An older or newer major keeps /opt/rocm's runtime."""
    for stem in ("libamdhip64", "libhsa-runtime64"):
        mine = _soname_majors(rocm_lib, stem)
        theirs = _soname_majors(torch_lib, stem)
        if not theirs or (mine and not (mine & theirs)):
            return False
    return True


def _share_torch_hip_runtime() -> None:
    """Make this library and PyTorch use ONE HIP runtime in a process that has both.

    PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 with the same sonames as
    /opt/rocm's.  Loaded after torch, libfir_hip binds to torch's copies (the soname is already
    loaded); loaded first, it pulls in /opt/rocm's, torch later loads its own by path, and the
    second HSA runtime in the process finds no device ("No HIP GPUs are available").  So when
    torch is installed and its runtime has the sonames of the ROCm the library was built with
    (_runtime_compatible), its runtime is loaded first, whichever of the two is imported first.
    FIR_HIP_OWN_RUNTIME=1 keeps /opt/rocm's (a process without torch uses it anyway)."""
    if os.environ.get("FIR_HIP_OWN_RUNTIME") == "1":
        return
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    tlib = Path(spec.origin).parent / "lib"
    if not _runtime_compatible(tlib):
        return
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        p = tlib / name
        if p.exists():
            try:
                ctypes.CDLL(str(p), mode=ctypes.RTLD_GLOBAL)
            except OSError:
                return


def lib() -> ctypes.CDLL:
    """Load libfir_hip.so once; raise FirHipError if it is missing or mismatched."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = lib_path()
        if not path.exists():
            raise FirHipError(
                f"{path} is not built: run `make -C warmup-fir-filter_amd/csrc` or "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
        _share_torch_hip_runtime()
        try:
            handle = ctypes.CDLL(str(path))
        except OSError as exc:
            raise FirHipError(f"cannot load {path}: {exc}") from exc
        for name, (res, args) in EXPORTS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        ver = handle.fir_abi_version()
        if ver != ABI_VERSION:
            raise FirHipError(f"{path}: ABI version {ver}, expected {ABI_VERSION}")
        from ._srcid import source_id

        built, want = handle.fir_build_id().decode(), source_id()
        if want is not None and built != want:
            raise FirHipError(f"{path} was built from other sources (build id {built}, the sources beside it hash "
                              f"to {want}): rebuild with `make -C warmup-fir-filter_amd/csrc`")
        _lib = handle
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().fir_last_error().decode(errors="replace")
        raise FirHipError(f"{what} failed (status {rc}): {msg}")


def device_count() -> int:
    n = _i32(0)
    _check(lib().fir_device_count(ctypes.byref(n)), "fir_device_count")
    return n.value


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_vp)


def _taps_i32(hq) -> np.ndarray:
    h = np.asarray(hq)
    if h.ndim != 1 or h.size == 0:
        raise FirHipError("hq must be a non-empty 1-D array")
    if h.size > MAX_TAPS:  # before any copy
        raise FirHipError(f"{h.size} taps exceed the library limit of {MAX_TAPS}")
    h = np.ascontiguousarray(h, dtype=np.int64)
    if h.min() < -(1 << 31) or h.max() >= (1 << 31):
        raise FirHipError("quantized taps must fit in int32")
    return h.astype(np.int32)


def _out_buf(out, shape, dtype, x, same_ok: bool = False) -> np.ndarray:
    """The output array: a fresh one, or the caller's ``out`` (reused buffers skip the
    first-touch page faults a fresh host array pays).  ``out`` must match
    exactly and must not overlap the input ``x``, except that ``same_ok`` lets it BE the input
    buffer (u8 in place: fir1d_fixed_rows' C entry stages the input on the device before any
    write to the output, tested aliased)."""
    if out is None:
        return np.empty(shape, dtype=dtype)
    if not isinstance(out, np.ndarray):
        raise FirHipError("out must be a numpy array")
    if out.dtype != np.dtype(dtype) or out.shape != tuple(shape):
        raise FirHipError(f"out must be {np.dtype(dtype)} of shape {tuple(shape)}, "
                          f"got {out.dtype} of shape {out.shape}")
    if not out.flags.c_contiguous or not out.flags.writeable:
        raise FirHipError("out must be C-contiguous and writeable")
    if same_ok and out.ctypes.data == x.ctypes.data and out.nbytes == x.nbytes:
        return out
    if np.shares_memory(out, x):
        raise FirHipError("out must not overlap the input")
    return out


def fir1d_fixed_rows(x: np.ndarray, hq, frac_bits: int = 12, acc_bits: int = 32,
                     out_stage: int = OUT_U8_SAT, channels: int = 1, device: int = 0,
                     out: np.ndarray | None = None) -> np.ndarray:
    """Row-wise same-mode fixed FIR of a uint8/int16 array (last axis = row of
    width*channels interleaved samples).  Returns uint8 (OUT_U8_SAT) or int32 (OUT_I32)."""
    x = np.ascontiguousarray(x)
    if x.dtype == np.uint8:
        in_dtype = IN_U8
    elif x.dtype == np.int16:
        in_dtype = IN_I16
    else:
        raise FirHipError(f"x dtype must be uint8 or int16, got {x.dtype}")
    h = _taps_i32(hq)
    if x.ndim == 0:
        x = x.reshape(1)
    rowlen = x.shape[-1]
    rows = x.size // rowlen if rowlen else 0
    if rowlen % channels:
        raise FirHipError("row length must be a multiple of channels")
    y = _out_buf(out, x.shape, np.uint8 if out_stage == OUT_U8_SAT else np.int32, x, same_ok=True)
    _check(lib().fir1d_fixed_rows(_ptr(x), in_dtype, rows, rowlen // channels, channels, _ptr(h), h.size,
                                  int(frac_bits), int(acc_bits), int(out_stage), _ptr(y), int(device)),
           "fir1d_fixed_rows")
    return y


def fir1d_fixed_rows_sharded(x: np.ndarray, hq, frac_bits: int = 12, acc_bits: int = 32,
                             out_stage: int = OUT_U8_SAT, channels: int = 1, devices=(0,),
                             out: np.ndarray | None = None) -> np.ndarray:
    """fir1d_fixed_rows spread over several devices of this process (``devices`` may repeat
    an id): row blocks for images, halo-widened segments for one long row."""
    x = np.ascontiguousarray(x)
    if x.dtype == np.uint8:
        in_dtype = IN_U8
    elif x.dtype == np.int16:
        in_dtype = IN_I16
    else:
        raise FirHipError(f"x dtype must be uint8 or int16, got {x.dtype}")
    h = _taps_i32(hq)
    devs = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32).reshape(-1))
    if devs.size == 0:
        raise FirHipError("devices must not be empty")
    if x.ndim == 0:
        x = x.reshape(1)
    rowlen = x.shape[-1]
    rows = x.size // rowlen if rowlen else 0
    if rowlen % channels:
        raise FirHipError("row length must be a multiple of channels")
    y = _out_buf(out, x.shape, np.uint8 if out_stage == OUT_U8_SAT else np.int32, x)
    _check(lib().fir1d_fixed_rows_sharded(_ptr(x), in_dtype, rows, rowlen // channels, channels, _ptr(h), h.size,
                                          int(frac_bits), int(acc_bits), int(out_stage), _ptr(y), _ptr(devs),
                                          devs.size), "fir1d_fixed_rows_sharded")
    return y


def parse_devices(spec) -> list[int]:
    """A ``--devices`` value: N (devices 0..N-1), a comma list of ids (repeats allowed: a
    device then takes several row blocks in turn; a trailing comma makes one id a list, so
    "3," is device 3 alone), or a sequence of ids; None = [0]."""
    if spec is None:
        return [0]
    if isinstance(spec, str):
        spec = [int(v) for v in spec.split(",") if v.strip()] if "," in spec else int(spec)
    if isinstance(spec, (int, np.integer)):
        if spec < 1:
            raise ValueError("--devices N needs N >= 1")
        return list(range(int(spec)))
    devs = [int(v) for v in spec]
    if not devs or min(devs) < 0:
        raise ValueError("devices must be a non-empty list of ids >= 0")
    return devs


def _over_devices(nrows: int, devices, run) -> None:
    """run(r0, r1, device) over contiguous row blocks, one block per entry of ``devices``; each
    distinct device on its own host thread (the C ABI is reentrant across devices and serialises
    calls on one device; ctypes releases the GIL).  Rows are independent: no exchange."""
    devs = list(devices)
    by_dev: dict[int, list] = {}
    for i, d in enumerate(devs):
        r0, r1 = nrows * i // len(devs), nrows * (i + 1) // len(devs)
        if r1 > r0:
            by_dev.setdefault(d, []).append((r0, r1))
    if len(by_dev) <= 1:
        for d, blocks in by_dev.items():
            for r0, r1 in blocks:
                run(r0, r1, d)
        return
    errors = []

    def worker(d, blocks):
        try:
            for r0, r1 in blocks:
                run(r0, r1, d)
        except BaseException as exc:  # noqa: BLE001 - re-raised in the caller
            errors.append(exc)

    threads = [threading.Thread(target=worker, args=(d, b)) for d, b in by_dev.items()]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]


def fir1d_fixed_rows_multi(x: np.ndarray, hq2, frac_bits: int = 12, acc_bits: int = 32,
                           out_stage: int = OUT_U8_SAT, channels: int = 1, device: int = 0,
                           out: np.ndarray | None = None, devices=None) -> np.ndarray:
    """F filters (rows of the F x L array hq2) over the same x in one call; returns an
    array of shape (F, *x.shape).  u8 input is read once per 4 filters on the GPU.
    ``devices`` (a list, see parse_devices) spreads the rows over several devices."""
    if devices is not None and len(parse_devices(devices)) == 1:
        device = parse_devices(devices)[0]  # one id: that device (as fir1d_ideal_rows does)
    elif devices is not None and np.ndim(x) >= 2:
        x = np.ascontiguousarray(x)
        rowlen = x.shape[-1]
        x2 = x.reshape(-1, rowlen)
        nf = np.asarray(hq2).shape[0]
        y = _out_buf(out, (nf,) + x.shape, np.uint8 if out_stage == OUT_U8_SAT else np.int32, x)
        y2 = y.reshape(nf, -1, rowlen)

        def run(r0, r1, d):
            y2[:, r0:r1] = fir1d_fixed_rows_multi(x2[r0:r1], hq2, frac_bits, acc_bits, out_stage, channels, d)

        _over_devices(x2.shape[0], parse_devices(devices), run)
        return y
    x = np.ascontiguousarray(x)
    if x.dtype == np.uint8:
        in_dtype = IN_U8
    elif x.dtype == np.int16:
        in_dtype = IN_I16
    else:
        raise FirHipError(f"x dtype must be uint8 or int16, got {x.dtype}")
    h2 = np.asarray(hq2, dtype=np.int64)
    if h2.ndim != 2 or h2.shape[0] < 1:
        raise FirHipError("hq2 must be a non-empty (filters, taps) array")
    nf, L = h2.shape
    if L > MAX_TAPS:
        raise FirHipError(f"{L} taps exceed the library limit of {MAX_TAPS}")
    h = np.concatenate([_taps_i32(row) for row in h2])
    if x.ndim == 0:
        x = x.reshape(1)
    rowlen = x.shape[-1]
    rows = x.size // rowlen if rowlen else 0
    if rowlen % channels:
        raise FirHipError("row length must be a multiple of channels")
    y = _out_buf(out, (nf,) + x.shape, np.uint8 if out_stage == OUT_U8_SAT else np.int32, x)
    _check(lib().fir1d_fixed_rows_multi(_ptr(x), in_dtype, rows, rowlen // channels, channels, _ptr(h), L, nf,
                                        int(frac_bits), int(acc_bits), int(out_stage), _ptr(y), int(device)),
           "fir1d_fixed_rows_multi")
    return y


# ---- host image batches (the stage drivers' entries, fir_hip.h ABI 6) -------------------
_PLANE_READY = ctypes.CFUNCTYPE(None, _vp, ctypes.c_int)  # fir_plane_ready_fn
TIMING_KEYS = ("h2d_ms", "kernel_ms", "d2h_ms", "call_ms")  # FIR_TIMING_SLOTS, in order


class _Pinned:
    """One fir_host_alloc block; freed when the last array over it is gone."""

    def __init__(self, nbytes: int):
        p = _vp(0)
        _check(lib().fir_host_alloc(int(nbytes), ctypes.byref(p)), "fir_host_alloc")
        self.ptr, self.nbytes = p.value, int(nbytes)

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.fir_host_free(_vp(self.ptr))
            self.ptr = None


def host_empty(nbytes: int) -> np.ndarray:
    """A uint8 array of ``nbytes`` in page-locked host memory (fir_host_alloc): the copies of the
    image-batch entries run as DMA straight from / into it.  The block is released when the array
    (and every view of it) is garbage."""
    if nbytes <= 0:
        return np.empty(0, dtype=np.uint8)
    owner = _Pinned(nbytes)
    raw = (ctypes.c_uint8 * owner.nbytes).from_address(owner.ptr)
    raw._owner = owner  # the ctypes array keeps the block alive; NumPy's base chain keeps the array
    return np.frombuffer(raw, dtype=np.uint8)


def _host_planes(xs: list, nf: int, dtype, outs):
    """The output planes of an image batch: the caller's ``outs`` (per image, F arrays shaped like
    the image, C-contiguous, writeable, of ``dtype``) or fresh arrays."""
    if outs is None:
        return [[np.empty(x.shape, dtype=dtype) for _ in range(nf)] for x in xs]
    outs = [list(o) for o in outs]
    if len(outs) != len(xs):
        raise FirHipError("outs must hold one entry per image")
    for i, (x, ps) in enumerate(zip(xs, outs)):
        if len(ps) != nf:
            raise FirHipError(f"outs[{i}] must hold {nf} planes")
        for f, p in enumerate(ps):
            if not isinstance(p, np.ndarray) or p.dtype != np.dtype(dtype) or p.shape != x.shape:
                raise FirHipError(f"outs[{i}][{f}] must be a {np.dtype(dtype)} array of shape {x.shape}")
            if not p.flags.c_contiguous or not p.flags.writeable:
                raise FirHipError(f"outs[{i}][{f}] must be C-contiguous and writeable")
    return outs


def _run_images(fn, what: str, args_head: list, planes: list, device: int, ready, timing):
    """Call an image-batch entry: planes flattened image-major, ``ready(i, f)`` per landed plane
    (exceptions it raises are re-raised after the call), ``timing`` (dict) filled from the
    entry's FIR_TIMING_SLOTS."""
    nf = len(planes[0]) if planes else 1
    flat = [p for ps in planes for p in ps]
    yp = (_vp * max(1, len(flat)))(*[p.ctypes.data for p in flat])
    errors = []

    def on_ready(_ctx, p):
        try:
            ready(p // nf, p % nf)
        except BaseException as exc:  # noqa: BLE001 - re-raised after the C call returns
            errors.append(exc)

    cb = _PLANE_READY(on_ready) if ready is not None else None
    t = (ctypes.c_double * 4)() if timing is not None else None
    _check(fn(*args_head, yp, int(device), ctypes.cast(cb, _vp) if cb is not None else None, None, t), what)
    if timing is not None:
        timing.update({k: float(v) for k, v in zip(TIMING_KEYS, t)})
    if errors:
        raise errors[0]
    return planes


def _image_geometry(xs: list, dtype_ok) -> tuple:
    xs = [np.ascontiguousarray(x) for x in xs]
    for i, x in enumerate(xs):
        if x.ndim != 2:
            raise FirHipError(f"xs[{i}] must be a 2-D (rows, width) image, got shape {x.shape}")
        if not dtype_ok(x.dtype):
            raise FirHipError(f"xs[{i}] has dtype {x.dtype}")
    n = len(xs)
    ptrs = (_vp * max(1, n))(*[x.ctypes.data for x in xs])
    rows = (_i64 * max(1, n))(*[x.shape[0] for x in xs])
    return xs, ptrs, rows


def fir1d_fixed_images_multi(xs, hq2, frac_bits: int = 12, acc_bits: int = 32, out_stage: int = OUT_U8_SAT,
                             channels: int = 1, device: int = 0, outs=None, ready=None, timing: dict | None = None):
    """The F filters (rows of hq2) over every 2-D image of ``xs`` (all uint8 or all int16; row =
    width*channels interleaved samples) in one device call: the images uploaded once, one batch
    launch, each plane downloaded into ``outs[i][f]`` (fresh arrays when None; page-locked ones from
    host_empty make every copy a DMA).  ``ready(i, f)`` runs on this thread as soon as plane (i, f)
    is in host memory, while later planes are still in flight.  Returns outs.  Replaces the loop
    over images x coefficient sets of fir_1d/sim/vector/gen_fixed_output.py:88-107 (reference root)."""
    xs = list(xs)
    dt = xs[0].dtype if xs else np.dtype(np.uint8)
    xs, ptrs, rows = _image_geometry(xs, lambda d: d == dt and d in (np.uint8, np.int16))
    h2 = np.asarray(hq2, dtype=np.int64)
    if h2.ndim != 2 or h2.shape[0] < 1:
        raise FirHipError("hq2 must be a non-empty (filters, taps) array")
    nf, L = h2.shape
    h = np.concatenate([_taps_i32(row) for row in h2])
    for i, x in enumerate(xs):
        if x.shape[1] % channels:
            raise FirHipError(f"xs[{i}]: row length must be a multiple of channels")
    widths = (_i64 * max(1, len(xs)))(*[x.shape[1] // channels for x in xs])
    planes = _host_planes(xs, nf, np.uint8 if out_stage == OUT_U8_SAT else np.int32, outs)
    head = [len(xs), ptrs, rows, widths, IN_U8 if dt == np.uint8 else IN_I16, int(channels), _ptr(h), L, nf,
            int(frac_bits), int(acc_bits), int(out_stage)]
    return _run_images(lib().fir1d_fixed_images_multi, "fir1d_fixed_images_multi", head, planes, device, ready, timing)


def fir1d_ideal_images_multi(xs, hs, device: int = 0, outs=None, ready=None, timing: dict | None = None):
    """The float64 ideal model with each coefficient set of ``hs`` (F x taps floats) over every 2-D
    uint8 image of ``xs``, one upload per image for all F sets; planes, ``ready`` and ``timing`` as
    fir1d_fixed_images_multi.  Replaces the loop of fir_1d/sim/vector/gen_ideal_output.py:75-86."""
    xs, ptrs, rows = _image_geometry(list(xs), lambda d: d == np.uint8)
    h2 = np.ascontiguousarray(np.asarray(hs, dtype=np.float64))
    if h2.ndim != 2 or h2.shape[0] < 1 or h2.shape[1] < 1 or h2.shape[1] > MAX_TAPS:
        raise FirHipError(f"hs must be a (filters, taps) array with 1 <= taps <= {MAX_TAPS}")
    nf, L = h2.shape
    widths = (_i64 * max(1, len(xs)))(*[x.shape[1] for x in xs])
    planes = _host_planes(xs, nf, np.float64, outs)
    head = [len(xs), ptrs, rows, widths, _ptr(h2), L, nf]
    return _run_images(lib().fir1d_ideal_images_multi, "fir1d_ideal_images_multi", head, planes, device, ready, timing)


def fir2d_fixed(x: np.ndarray, hq2, frac_bits: int = 12, acc_bits: int = 32, out_stage: int = OUT_U8_SAT,
                device: int = 0, out: np.ndarray | None = None) -> np.ndarray:
    """2-D same-mode fixed FIR of a uint8 frame (H, W), or of a batch of frames (F, H, W) each
    filtered on its own in one launch, with a (R, C) quantized kernel."""
    x = np.ascontiguousarray(x, dtype=np.uint8)
    if x.ndim not in (2, 3):
        raise FirHipError("x must be 2-D (a frame) or 3-D (frames, height, width)")
    h2 = np.asarray(hq2, dtype=np.int64)
    if h2.ndim != 2:
        raise FirHipError("hq2 must be 2-D")
    R, C = h2.shape
    h = _taps_i32(h2.reshape(-1))
    y = _out_buf(out, x.shape, np.uint8 if out_stage == OUT_U8_SAT else np.int32, x)
    frames = x.shape[0] if x.ndim == 3 else 1
    _check(lib().fir2d_fixed_frames(_ptr(x), frames, x.shape[-2], x.shape[-1], _ptr(h), R, C, int(frac_bits),
                                    int(acc_bits), int(out_stage), _ptr(y), int(device)), "fir2d_fixed_frames")
    return y


def fir1d_ideal_rows(x_u8: np.ndarray, h, device: int = 0, devices=None) -> np.ndarray:
    """float64 ideal model over uint8 rows (last axis); ``devices`` spreads the rows over
    several devices (see parse_devices)."""
    x = np.ascontiguousarray(x_u8, dtype=np.uint8)
    hh = np.ascontiguousarray(np.asarray(h, dtype=np.float64).reshape(-1))
    if hh.size == 0 or hh.size > MAX_TAPS:
        raise FirHipError(f"tap count must be in [1, {MAX_TAPS}]")
    if x.ndim == 0:
        x = x.reshape(1)
    width = x.shape[-1]
    rows = x.size // width if width else 0
    y = np.empty(x.shape, dtype=np.float64)
    x2, y2 = x.reshape(rows, width), y.reshape(rows, width)

    def run(r0, r1, d):
        _check(lib().fir1d_ideal_rows(_ptr(x2[r0:r1]), r1 - r0, width, _ptr(hh), hh.size, _ptr(y2[r0:r1]), int(d)),
               "fir1d_ideal_rows")

    if rows == 0:
        run(0, 0, device)
    else:
        _over_devices(rows, [device] if devices is None else parse_devices(devices), run)
    return y


def metrics_from_sums(s, n: int) -> dict:
    """The report's metric dict (gen_3tap_compare_report.py:102-112) from the 9 sums (s[8]: the
    kernel's status, non-zero when its in-kernel hand-off timed out)."""
    if len(s) > 8 and float(s[8]) != 0.0:
        raise FirHipError("metrics: the in-kernel hand-off timed out (status in out[8])")
    if n == 0:
        return {"num_samples": 0, "max_abs_err": 0.0, "mae": 0.0, "rmse": 0.0, "mean_err": 0.0,
                "sat_low_ratio": 0.0, "sat_high_ratio": 0.0, "sat_ratio": 0.0, "clip_needed_ratio": 0.0}
    lo, hi = float(s[4]) / n, float(s[5]) / n
    return {"num_samples": int(n), "max_abs_err": float(s[0]), "mae": float(s[1]) / n,
            "rmse": float(np.sqrt(float(s[2]) / n)), "mean_err": float(s[3]) / n, "sat_low_ratio": lo,
            "sat_high_ratio": hi, "sat_ratio": lo + hi, "clip_needed_ratio": float(s[6]) / n}


# fixed-array dtypes of the metrics kernel (fir_num_dtype); bool goes as its uint8 bytes (0/1)
METRIC_DTYPES = {np.dtype(np.uint8): 0, np.dtype(np.int8): 1, np.dtype(np.uint16): 2, np.dtype(np.int16): 3,
                 np.dtype(np.uint32): 4, np.dtype(np.int32): 5, np.dtype(np.uint64): 6, np.dtype(np.int64): 7,
                 np.dtype(np.float16): 8, np.dtype(np.float32): 9, np.dtype(np.float64): 10}


def metrics_fixed_view(y_fixed: np.ndarray):
    """(flat contiguous array, fir_num_dtype code) of a fixed output for the metrics kernel: its
    own values in native byte order, as the reference's y_fixed.astype(np.float64) reads them."""
    yf = np.asarray(y_fixed)
    if yf.dtype == np.bool_:
        yf = yf.view(np.uint8)
    dt = yf.dtype.newbyteorder("=") if yf.dtype.byteorder not in ("=", "|") else yf.dtype
    if dt not in METRIC_DTYPES:
        raise FirHipError(f"fixed dtype {yf.dtype} is not supported (integer, bool or float16/32/64)")
    yf = np.ascontiguousarray(yf, dtype=dt).reshape(-1)
    return yf, METRIC_DTYPES[dt]


def compare_metrics(y_ideal: np.ndarray, y_fixed: np.ndarray, device: int = 0) -> dict:
    """_compute_metrics (gen_3tap_compare_report.py:67-112) in one GPU pass, for a fixed array of
    any integer / bool / float dtype (the reference converts it with astype(np.float64), :85)."""
    if y_ideal.shape != y_fixed.shape:
        raise ValueError(f"Shape mismatch: ideal={y_ideal.shape}, fixed={y_fixed.shape}")
    yi = np.ascontiguousarray(y_ideal, dtype=np.float64).reshape(-1)
    yf, code = metrics_fixed_view(y_fixed)
    out = np.zeros(9, dtype=np.float64)
    _check(lib().fir_compare_metrics(_ptr(yi), _ptr(yf), code, yi.size, _ptr(out), int(device)),
           "fir_compare_metrics")
    return metrics_from_sums(out, yi.size)


def restore_u8(a: np.ndarray, policy: int = RESTORE_CLIP, device: int = 0) -> np.ndarray:
    """restore_images._to_u8_clip / _to_u8_normalized (restore_images.py:51-64) on the GPU;
    same shape, uint8."""
    arr = np.ascontiguousarray(a, dtype=np.float64)
    if policy == RESTORE_NORMALIZE and arr.size == 0:
        raise ValueError("zero-size array to reduction operation minimum which has no identity")
    out = np.empty(arr.shape, dtype=np.uint8)
    _check(lib().fir_restore_u8(_ptr(arr), arr.size, int(policy), _ptr(out), int(device)), "fir_restore_u8")
    return out


# ---- xGMI peer halos (fir_hip.h; used by fir_hip.sharded.XgmiHalo) ---------------------
def ipc_export(dev_ptr: int) -> tuple[bytes, int]:
    """(handle, byte offset) of the device allocation holding ``dev_ptr``, for another process."""
    h = ctypes.create_string_buffer(IPC_HANDLE_BYTES)
    off = ctypes.c_int64(0)
    _check(lib().fir_ipc_export(ctypes.c_void_p(dev_ptr), h, ctypes.byref(off)), "fir_ipc_export")
    return h.raw, int(off.value)


def ipc_import(handle: bytes, offset: int, device: int) -> int:
    """Map a peer process's exported allocation on ``device``; returns base + ``offset``."""
    if len(handle) != IPC_HANDLE_BYTES:
        raise FirHipError(f"IPC handle must be {IPC_HANDLE_BYTES} bytes")
    p = ctypes.c_void_p(0)
    _check(lib().fir_ipc_import(handle, int(offset), int(device), ctypes.byref(p)), "fir_ipc_import")
    return int(p.value)


def ipc_close(dev_ptr: int) -> None:
    _check(lib().fir_ipc_close(ctypes.c_void_p(dev_ptr)), "fir_ipc_close")


def device_bus_id(device: int) -> str:
    """PCI bus id of ``device`` (names the GPU across processes with different device orders)."""
    buf = ctypes.create_string_buffer(64)
    _check(lib().fir_device_bus_id(int(device), buf, 64), "fir_device_bus_id")
    return buf.value.decode()


def peer_access(device: int, peer_bus_id: str) -> bool:
    """Whether kernels on ``device`` may read the HBM of the GPU at ``peer_bus_id``."""
    can = _i32(0)
    _check(lib().fir_peer_access(int(device), peer_bus_id.encode(), ctypes.byref(can)), "fir_peer_access")
    return bool(can.value)


def peer_atomics(device: int, peer_bus_id: str) -> bool:
    """Whether kernels on ``device`` may perform atomics on the HBM of the GPU at ``peer_bus_id``
    (the halo gate's mailbox protocol needs it)."""
    can = _i32(0)
    _check(lib().fir_peer_atomics(int(device), peer_bus_id.encode(), ctypes.byref(can)), "fir_peer_atomics")
    return bool(can.value)


def halo_mailbox_bytes(halo_left_bytes: int, halo_right_bytes: int) -> int:
    """Bytes of one rank's halo-gate mailbox (fir_hip.h, fir_halo_gate_dev)."""
    n = int(lib().fir_halo_mailbox_bytes(int(halo_left_bytes), int(halo_right_bytes)))
    if n < 0:
        raise FirHipError("halo byte counts must be >= 0")
    return n


def build_id() -> str:
    """The source id the loaded library was built from (see fir_hip._srcid)."""
    return lib().fir_build_id().decode()


def peek(dev_ptr: int, nbytes: int) -> bytes:
    """Synchronous copy of ``nbytes`` device bytes (own or imported) to the host."""
    buf = ctypes.create_string_buffer(max(1, nbytes))
    _check(lib().fir_peek(ctypes.c_void_p(dev_ptr), buf, int(nbytes)), "fir_peek")
    return buf.raw[:nbytes]

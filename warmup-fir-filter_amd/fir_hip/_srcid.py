"""The source id of libfir_hip.so: a hash of the sources it is built from.

``make -C warmup-fir-filter_amd/csrc`` embeds it (``-DFIR_BUILD_ID``, exported as
``fir_build_id()``); :func:`fir_hip.lib` recomputes it from the sources beside the package and
refuses a library built from other sources, so a stale ``.so`` cannot pass as the tree's.
Standalone on purpose (no NumPy): the Makefile runs it as ``python3 _srcid.py``.
"""
from __future__ import annotations

import hashlib
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parents[1]  # warmup-fir-filter_amd/


def source_files(pkg: Path = PKG) -> list[Path]:
    csrc = pkg / "csrc"
    files = sorted(p for p in csrc.iterdir() if p.is_file() and p.suffix in (".hip", ".h")) if csrc.is_dir() else []
    files += [csrc / "Makefile", pkg.parent / "include" / "fir_hip.h"]
    return files


def source_id(pkg: Path = PKG) -> str | None:
    """sha256 over (path relative to the repo root, contents) of every source; None when the
    sources are not present (a library used without its tree)."""
    files = source_files(pkg)
    if not all(p.is_file() for p in files):
        return None
    h = hashlib.sha256()
    for p in files:
        h.update(p.relative_to(pkg.parent).as_posix().encode() + b"\0")
        h.update(p.read_bytes() + b"\0")
    return h.hexdigest()[:32]


if __name__ == "__main__":
    sid = source_id()
    if sid is None:
        sys.exit("libfir_hip sources not found")
    print(sid)

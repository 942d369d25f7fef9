"""End-to-end FIR 1-D pipeline on MI355X: vectors -> ideal/fixed outputs -> reports -> images.

Mirror of the reference driver ``pipeline_fir_1d.py`` (``run_pipeline`` :34-98, CLI
:102-175, ``[OK]``/``[FAIL]`` status line :224-241): same stage order, flags and return
dict.  Stages 2-4 run on the GPU (ideal and fixed models one launch per image -- the fixed
bank fused into one read of each image -- and the report metrics as one reduction per
case); input decoding and PNG restore stay host I/O.  Extra keyword arguments (``image_dir``,
``vector_dir``, ``image_out_dir``) relocate the reference's fixed directories; by default
the golden inputs come from ``fir_1d/sim/img`` next to this package if present (the reference's
image files, ``pipeline_fir_1d.py:204-205``), else from the package's own decoded copy of them,
``fir_1d/sim/img_u8.npz`` (the 7 images as the reference's Pillow decode gives them; SHA-256s in
SURVEY Appendix A).

    python warmup-fir-filter_amd/pipeline_fir_1d.py --tap all --overwrite-vectors
"""
from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path
from time import perf_counter
from typing import Any

_HERE = Path(__file__).resolve().parent
if str(_HERE) not in sys.path:
    sys.path.insert(0, str(_HERE))

from fir_1d.sim.vector.gen_3tap_compare_report import generate_3tap_compare_report  # noqa: E402
from fir_1d.sim.vector.gen_5tap_compare_report import generate_5tap_compare_report  # noqa: E402
from fir_1d.sim.vector.gen_fixed_output import (generate_fixed_3tap_output_vector,  # noqa: E402
                                                generate_fixed_5tap_output_vector)
from fir_1d.sim.vector.gen_ideal_output import (generate_ideal_3tap_output_vector,  # noqa: E402
                                                generate_ideal_5tap_output_vector)
from fir_1d.sim.vector.gen_input_vectors import generate_input_vector_jsons  # noqa: E402
from fir_1d.sim.vector.restore_images import restore_images  # noqa: E402

SIM_DIR = _HERE / "fir_1d" / "sim"
DEFAULT_VECTOR_DIR = SIM_DIR / "vector"
DEFAULT_IMAGE_OUT_DIR = SIM_DIR / "output_img"


def default_image_source() -> Path:
    img = SIM_DIR / "img"
    if img.exists():
        return img
    return SIM_DIR / "img_u8.npz"


def _selected_taps(tap: str) -> list[str]:
    return ["3", "5"] if tap == "all" else [tap]


def _log_stage(message: str) -> None:
    print(f"[pipeline] {message}")


def _start_devices(devices):
    """Bring the devices the vector stages will use up on a side thread (the HIP runtime, the
    library's per-device state, its code objects: about 0.16 s per process) while the input stage
    decodes on this one.  Best effort: a failure here is left for the stage itself to report."""
    import threading

    def warm():
        try:
            import numpy as np

            import fir_hip

            for d in dict.fromkeys(fir_hip.parse_devices(devices)):
                fir_hip.fir1d_fixed_rows(np.zeros((1, 64), np.uint8), [1], device=d)
        except Exception:  # noqa: BLE001 - the stages raise the real error
            pass

    t = threading.Thread(target=warm, name="fir-device-start", daemon=True)
    t.start()
    return t


def run_pipeline(*, tap: str, overwrite_vectors: bool, skip_input: bool, skip_ideal: bool, skip_fixed: bool,
                 skip_report: bool, skip_restore: bool, restore_kind: str, ideal_policy: str, overwrite_images: bool,
                 strict_report: bool, strict_restore: bool, top_k: int, image_dir: Path | None = None,
                 vector_dir: Path = DEFAULT_VECTOR_DIR, image_out_dir: Path = DEFAULT_IMAGE_OUT_DIR,
                 devices=None) -> dict[str, Any]:
    taps = _selected_taps(tap)
    vector_dir = Path(vector_dir)
    in_dir, out_dir = vector_dir / "input", vector_dir / "output"
    results: dict[str, Any] = {"selected_taps": taps}
    starting = None
    if not skip_input:
        if not (skip_ideal and skip_fixed and skip_report and skip_restore) and \
                os.environ.get("FIR_PIPELINE_START_DEVICES", "1") != "0":
            starting = _start_devices(devices)
        _log_stage("Generate input vectors")
        try:
            results["input_manifest"] = generate_input_vector_jsons(image_dir or default_image_source(), in_dir,
                                                                    overwrite=overwrite_vectors)
        finally:
            if starting is not None:
                starting.join()
    if not skip_ideal:
        _log_stage("Generate ideal outputs")
        gen = {"3": generate_ideal_3tap_output_vector, "5": generate_ideal_5tap_output_vector}
        results["ideal_counts"] = {f"ideal_{t}tap": gen[t](in_dir, out_dir, overwrite=overwrite_vectors, devices=devices)
                                   for t in taps}
    if not skip_fixed:
        _log_stage("Generate fixed outputs")
        gen = {"3": generate_fixed_3tap_output_vector, "5": generate_fixed_5tap_output_vector}
        results["fixed_counts"] = {f"fixed_{t}tap": gen[t](in_dir, out_dir, overwrite=overwrite_vectors, devices=devices)
                                   for t in taps}
    if not skip_report:
        _log_stage("Generate compare reports")
        gen = {"3": generate_3tap_compare_report, "5": generate_5tap_compare_report}
        results["report_results"] = {
            f"report_{t}tap": gen[t](ideal_dir=out_dir / f"ideal_{t}tap", fixed_dir=out_dir / f"fixed_{t}tap",
                                     report_dir=out_dir / f"report_{t}tap", top_k=top_k, strict=strict_report)
            for t in taps}
    if not skip_restore:
        _log_stage("Restore output images")
        summary = restore_images(vector_output_dir=out_dir, output_img_dir=image_out_dir, kind=restore_kind, tap=tap,
                                 ideal_policy=ideal_policy, overwrite=overwrite_images, strict=strict_restore)
        results["restore_summary"] = {"num_converted": summary["num_converted"], "num_skipped": summary["num_skipped"]}
    return results


def _build_argparser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Run FIR 1D end-to-end pipeline on MI355X: vectors, ideal/fixed "
                                             "outputs, compare reports, and image restore.")
    ap.add_argument("--tap", choices=("all", "3", "5"), default="all")
    for flag in ("overwrite-vectors", "skip-input", "skip-ideal", "skip-fixed", "skip-report", "skip-restore",
                 "overwrite-images", "strict-report", "strict-restore"):
        ap.add_argument(f"--{flag}", action="store_true")
    ap.add_argument("--restore-kind", choices=("all", "ideal", "fixed"), default="all")
    ap.add_argument("--ideal-policy", choices=("clip", "normalize"), default="clip")
    ap.add_argument("--top-k", type=int, default=5)
    ap.add_argument("--image-dir", type=Path, default=None, help="image folder or .npz of decoded uint8 images")
    ap.add_argument("--vector-dir", type=Path, default=DEFAULT_VECTOR_DIR)
    ap.add_argument("--image-out-dir", type=Path, default=DEFAULT_IMAGE_OUT_DIR)
    ap.add_argument("--devices", default=None,
                    help="GPUs the ideal / fixed stages spread each image's rows over: N (devices 0..N-1) or a "
                         "comma list of ids (default: device 0)")
    return ap


def main(argv=None) -> int:
    args = _build_argparser().parse_args(argv)
    t0 = perf_counter()
    skipped = sum(int(v) for v in (args.skip_input, args.skip_ideal, args.skip_fixed, args.skip_report,
                                   args.skip_restore))
    outs = f"{(args.vector_dir / 'output').resolve()}|{args.image_out_dir.resolve()}"
    try:
        summary = run_pipeline(tap=args.tap, overwrite_vectors=args.overwrite_vectors, skip_input=args.skip_input,
                               skip_ideal=args.skip_ideal, skip_fixed=args.skip_fixed, skip_report=args.skip_report,
                               skip_restore=args.skip_restore, restore_kind=args.restore_kind,
                               ideal_policy=args.ideal_policy, overwrite_images=args.overwrite_images,
                               strict_report=args.strict_report, strict_restore=args.strict_restore,
                               top_k=args.top_k, image_dir=args.image_dir, vector_dir=args.vector_dir,
                               image_out_dir=args.image_out_dir, devices=args.devices)
    except Exception as exc:
        print(f"[FAIL] pipeline_fir_1d file=pipeline_fir_1d.py generated=0 skipped={skipped} failed=1 "
              f"elapsed={perf_counter() - t0:.2f}s out={outs} error=\"{exc}\"")
        raise
    generated = len([k for k in summary if k != "selected_taps"])
    print(f"[OK] pipeline_fir_1d file=pipeline_fir_1d.py generated={generated} skipped={skipped} failed=0 "
          f"elapsed={perf_counter() - t0:.2f}s out={outs}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

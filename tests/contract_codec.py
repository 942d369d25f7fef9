"""JSON codec for the input-contract fixtures (tests/golden/input_contract.json).

The cases are inputs of every Python / NumPy kind a caller can hand to the fir_1d API
(str, complex, None, Decimal, Fraction, big ints, bytes, ranges, dicts, generators, 0-d /
1-D / 2-D / 3-D arrays of every dtype, masked arrays ...).  ``enc`` turns one into plain
JSON data and ``dec`` rebuilds an equal object (fresh generator included), so the generator
script (tests/golden/make_golden.py) calls the reference on ``dec(enc(case))`` — exactly
what the tests later rebuild — and stores the reference's result with ``enc`` as well.

Data only: nothing here executes anything read from the file.
"""
from __future__ import annotations

from decimal import Decimal
from fractions import Fraction

import numpy as np


class Gen:
    """A generator input: ``dec`` gives a fresh one-shot generator over ``items``."""

    def __init__(self, items):
        self.items = list(items)


def enc(v):
    if v is None:
        return {"t": "none"}
    if isinstance(v, Gen):
        return {"t": "gen", "v": [enc(i) for i in v.items]}
    if isinstance(v, np.ma.MaskedArray):
        return {"t": "masked", "data": enc(np.asarray(v.data)), "mask": enc(np.asarray(np.ma.getmaskarray(v)))}
    if isinstance(v, np.ndarray):
        if v.dtype == object:
            return {"t": "ndarray_obj", "shape": list(v.shape), "v": [enc(i) for i in v.reshape(-1).tolist()]}
        return {"t": "ndarray", "dtype": v.dtype.str, "shape": list(v.shape),
                "v": np.ascontiguousarray(v).tobytes().hex()}
    if isinstance(v, np.generic):
        return {"t": "npscalar", "dtype": v.dtype.str, "v": v.tobytes().hex()}
    if isinstance(v, bool):
        return {"t": "bool", "v": v}
    if isinstance(v, int):
        return {"t": "int", "v": str(v)}
    if isinstance(v, float):
        return {"t": "float", "v": v.hex()}
    if isinstance(v, complex):
        return {"t": "complex", "v": [v.real.hex(), v.imag.hex()]}
    if isinstance(v, str):
        return {"t": "str", "v": v}
    if isinstance(v, bytes):
        return {"t": "bytes", "v": v.hex()}
    if isinstance(v, bytearray):
        return {"t": "bytearray", "v": bytes(v).hex()}
    if isinstance(v, Decimal):
        return {"t": "decimal", "v": str(v)}
    if isinstance(v, Fraction):
        return {"t": "fraction", "v": [v.numerator, v.denominator]}
    if isinstance(v, range):
        return {"t": "range", "v": [v.start, v.stop, v.step]}
    if isinstance(v, dict):
        return {"t": "dict", "v": [[enc(k), enc(i)] for k, i in v.items()]}
    if isinstance(v, (list, tuple)):
        return {"t": type(v).__name__, "v": [enc(i) for i in v]}
    raise TypeError(f"contract_codec: cannot encode {type(v).__name__}")


def dec(d):
    t = d["t"]
    if t == "none":
        return None
    if t == "gen":
        return (dec(i) for i in d["v"])
    if t == "masked":
        return np.ma.MaskedArray(dec(d["data"]), mask=dec(d["mask"]))
    if t == "ndarray_obj":
        a = np.empty(len(d["v"]), dtype=object)
        for i, item in enumerate(d["v"]):
            a[i] = dec(item)
        return a.reshape(d["shape"])
    if t == "ndarray":
        return np.frombuffer(bytes.fromhex(d["v"]), dtype=np.dtype(d["dtype"])).reshape(d["shape"]).copy()
    if t == "npscalar":
        return np.frombuffer(bytes.fromhex(d["v"]), dtype=np.dtype(d["dtype"]))[0]
    if t == "bool":
        return bool(d["v"])
    if t == "int":
        return int(d["v"])
    if t == "float":
        return float.fromhex(d["v"])
    if t == "complex":
        return complex(float.fromhex(d["v"][0]), float.fromhex(d["v"][1]))
    if t == "str":
        return d["v"]
    if t == "bytes":
        return bytes.fromhex(d["v"])
    if t == "bytearray":
        return bytearray.fromhex(d["v"])
    if t == "decimal":
        return Decimal(d["v"])
    if t == "fraction":
        return Fraction(*d["v"])
    if t == "range":
        return range(*d["v"])
    if t == "dict":
        return {dec(k): dec(i) for k, i in d["v"]}
    if t == "list":
        return [dec(i) for i in d["v"]]
    if t == "tuple":
        return tuple(dec(i) for i in d["v"])
    raise ValueError(f"contract_codec: unknown tag {t!r}")


def same(a, b) -> bool:
    """Bit-level equality of two decoded results: type, dtype, shape and bytes for arrays,
    element type and float bits for lists."""
    if type(a) is not type(b):
        return False
    if isinstance(a, np.ndarray):
        return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()
    if isinstance(a, (list, tuple)):
        return len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
    if isinstance(a, float):
        return a.hex() == b.hex() or (a != a and b != b)
    return a == b

"""The drop-in input contract on the GPU: every input the reference accepts in
tests/golden/input_contract.json (non-list inputs to the models, non-u8 images to the row
drivers) computes through libfir_hip.so to the reference's own output, bit for bit (type,
dtype, shape, float bits).  The rejected inputs are checked on the CPU in
test_input_contract.py.
"""
from __future__ import annotations

import pytest

from contract_codec import dec, same
from test_input_contract import RECORDS, _empty, _rid, call


@pytest.mark.parametrize("rec", [r for r in RECORDS if "result" in r and not _empty(r)], ids=_rid)
def test_accepted_inputs_compute_the_reference_output(rec):
    got = call(rec)
    want = dec(rec["result"])
    assert same(got, want), (rec["fn"], rec["id"], got, want)

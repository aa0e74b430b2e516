"""The Quantity restatement (csrc/quantity.cpp: ParseQuantity + AsInt64 of apimachinery
v0.22.2, which the reference does not vendor) against every Quantity literal the reference
holds (tests/golden/quantity_literals.json, written by make_quantity_golden.py with the
values written out from each literal's suffix).  Inputs beyond these are parity unpinned."""
import json
import os

import numpy as np
import pytest

import pas_amd
from pas_amd import wire

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "quantity_literals.json")) as f:
    Q = json.load(f)


@pytest.mark.parametrize("case", Q["literals"], ids=lambda c: f"{c['literal']}@{c['source']}")
def test_literal_milli_and_as_int64(case):
    assert pas_amd.quantity_to_milli(case["literal"]) == case["milli"]
    assert pas_amd.quantity_as_int64(case["literal"]) == case["as_int64"]


def test_bb_example_pod_requests():
    c = Q["bb_example_pod"]
    req, mask, nc, unknown = wire.decode_pod_requests(json.dumps(c["pod"]).encode(), c["kinds"])
    assert nc[0] == 1 and unknown == 0 and mask[0, 0] == 0b111
    np.testing.assert_array_equal(req[0], np.array(c["want_requests"], np.int64))

"""Reservation oracle (oracle/reservation.c) pinned by the reference's own test tables (tests/golden/reservation.json,
made by tests/golden/make_golden_resv.py from reservation/scoring_test.go and plugin_test.go)."""
import json
import os

import numpy as np
import pytest

from koordinator_amd import abi
from oracle import oracle

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reservation.json")))["cases"]


def rsv_row(slots):
    r = np.zeros(1, dtype=abi.NODE_RSV_DTYPE)[0]
    r["n"] = len(slots)
    for s, d in enumerate(slots):
        for k, v in d.items():
            r[k][s] = v
        r["owner"][s] = 0
        r["available"][s] = 1
    return r


@pytest.mark.parametrize("case", CASES, ids=[c["ref"] for c in CASES])
def test_reservation_golden(case):
    pod = np.zeros(1, dtype=abi.POD_DTYPE)[0]
    pod["requests"][0], pod["requests"][1] = case["pod"]
    pod["reservation_owner_mask"] = 1
    pod["reservation_flags"] = abi.POD_RSV_AFFINITY if case.get("affinity") else 0
    if case.get("reserve"):
        pod["flags"] |= abi.POD_RESERVE
    ok, nom, score = oracle.rsv_case(pod, case["allowed_pods"], case["alloc"], case["num_pods"],
                                     case["pod_requested"], case["r_allocated"], case["has_state"],
                                     rsv_row(case["slots"]))
    if "want_score" in case:
        assert score == case["want_score"]
    if "want_nominated" in case:
        assert nom == case["want_nominated"]
    if "want_pass" in case:
        assert ok == case["want_pass"]

"""(r6) The committed oracle fixtures of the C4 and shipped bench queues (tests/golden/c4_queue.npz, shipped_queue.npz,
written by tests/golden/make_bench_fixture.py) checked on the CPU: the queue they were made from is the one bench.py
draws (segment digests of synth.make_stream), their first placements are the oracle's live schedule, and every
placement is a valid node.  bench.py's fixture_check compares the device's placements of every timed pod with them."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from koordinator_amd import framework  # noqa: E402

LIVE = {"c4": 200, "shipped": 60}  # pods re-run through the live oracle (seconds on the CPU)


def _load(wl):
    path = os.path.join(ROOT, "tests", "golden", f"{wl}_queue.npz")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated")
    z = np.load(path)
    return z, json.loads(str(z["meta"]))


def _work(wl, meta):
    profile, la = bench.workload_profile(wl)
    cfg = framework.build_config(profile=profile, la=la)
    return bench.Work(wl, meta["nodes"], cfg)


@pytest.mark.parametrize("wl", ["c4", "shipped"])
def test_bench_fixture(wl):
    z, meta = _load(wl)
    assert meta["workload"] == wl and meta["nodes"] == bench.WORKLOADS[wl][0]
    assert meta["queue"] == "synth.make_stream" and meta["pods"] % meta["segment"] == 0
    assert len(z["node"]) == meta["pods"] and len(z["seg_sha"]) == meta["pods"] // meta["segment"]
    assert ((z["node"] >= -1) & (z["node"] < meta["nodes"])).all()
    work = _work(wl, meta)
    assert work.seed == meta["cluster_seed"]
    pods = work.make_pods(meta["pods"], seed=meta["pods_seed"])
    work.set_queue(pods)
    for s in (0, len(z["seg_sha"]) - 1):  # first and last segment of the queue
        seg = np.ascontiguousarray(pods[s * meta["segment"]:(s + 1) * meta["segment"]])
        assert hashlib.sha256(seg.tobytes()).hexdigest() == str(z["seg_sha"][s])
    n = LIVE[wl]
    on, _ = work.oracle_run(pods[:n], 8)
    np.testing.assert_array_equal(z["node"][:n], on)
    assert (z["node"] >= 0).mean() > 0.5  # most of the queue is placed

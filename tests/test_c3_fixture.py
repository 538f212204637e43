"""(r6) The committed oracle fixture of config 3's whole queue (tests/golden/c3_queue.npz, written by
tests/golden/make_c3_fixture.py) checked on the CPU: its queue is the one synth.make_pods_stream draws (segment digests),
its first pods are the oracle's live schedule, and its 1M-pod node state is conserved (initial requests + every placed
pod's).  The GPU side (tests/test_parity_gpu.py::test_c3_full_size) compares the engine with it pod by pod."""
import hashlib
import json
import os

import numpy as np
import pytest

from koordinator_amd import abi, framework, synth
from oracle import oracle

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c3_queue.npz")


@pytest.fixture(scope="module")
def fx():
    z = np.load(PATH)
    return z, json.loads(str(z["meta"]))


def test_fixture_meta(fx):
    z, meta = fx
    assert meta["nodes"] == 100_000 and meta["pods"] >= 1_000_000 and meta["state_at"] == 1_000_000
    assert meta["queue"] == "synth.make_pods_stream" and meta["segment"] == 100_000
    assert len(z["node"]) == meta["pods"] == len(z["score"]) and len(z["seg_sha"]) == meta["pods"] // meta["segment"]
    assert ((z["node"] >= -1) & (z["node"] < 100_000)).all()


def test_fixture_queue_digests(fx):
    """The first two segments of the queue the fixture was made from are synth.make_pods_stream's (prefix-stable)."""
    z, meta = fx
    pods = synth.make_pods_stream(2 * meta["segment"], seed=meta["pods_seed"])
    for s in range(2):
        seg = np.ascontiguousarray(pods[s * meta["segment"]:(s + 1) * meta["segment"]])
        assert hashlib.sha256(seg.tobytes()).hexdigest() == str(z["seg_sha"][s])


def test_fixture_is_the_oracle_schedule(fx):
    z, meta = fx
    cfg = framework.build_config()
    cl = synth.make_cluster(meta["nodes"], seed=meta["cluster_seed"])
    pods = synth.make_pods_stream(1500, seed=meta["pods_seed"])
    on, sc, _ = oracle.schedule_cluster(cfg, cl, pods, n_threads=8)
    np.testing.assert_array_equal(z["node"][:1500], on)
    np.testing.assert_array_equal(z["score"][:1500].astype(np.int64), sc)


def test_fixture_state_conserved(fx):
    """Requested cpu / memory and the pod count after 1M pods = the initial bound pods' + every placed pod's."""
    z, meta = fx
    n = meta["state_at"]
    cl = synth.make_cluster(meta["nodes"], seed=meta["cluster_seed"])
    pods = synth.make_pods_stream(n, seed=meta["pods_seed"])
    g = z["node"][:n]
    placed = g >= 0
    for r, col in ((abi.RES_CPU, "st1m_requested_cpu"), (abi.RES_MEMORY, "st1m_requested_mem")):
        base = np.bincount(cl.existing_node, weights=cl.existing_pods["requests"][:, r].astype(np.float64),
                           minlength=cl.n)
        add = np.bincount(g[placed], weights=pods["requests"][placed, r].astype(np.float64), minlength=cl.n)
        np.testing.assert_array_equal(z[col], (base + add).astype(np.int64))
        assert (z[col] <= cl.nodes["allocatable"][:, r]).all()
    np.testing.assert_array_equal(z["st1m_num_pods"], np.bincount(cl.existing_node, minlength=cl.n) +
                                  np.bincount(g[placed], minlength=cl.n))

"""Topology-manager policies: mergeFilteredHints + the best-effort / restricted / single-numa-node
Merge and canAdmitPodResult (frameworkext/topologymanager/policy*.go), pinned by the reference's own tables
(tests/golden/topology_policy.json, written by tests/golden/make_golden_topology.py).

The oracle's general merge (any number of provider lists, hints in list order) runs every case.  The device runs
the same cases through kg_debug_numa_merge, i.e. policy_merge — the code NodeNUMAResource Filter calls, including
the r2 "preferred permutations first" shortcut — with each provider list encoded as the device holds it (a set of
IterateBitMasks positions with a preferred subset, or one "don't care" hint).  Every merge case of the tables has ≤ 2
such lists; TestPolicySingleNumaNodeFilterHints mixes nil and mask hints in one list and has 3 lists, shapes
generateResourceHints never produces, so that table pins the oracle only (the device's filter runs inside every
single-numa-node merge case).  A randomized differential test then compares the device merge with the oracle's on
hint lists shaped like NodeNUMAResource's (1-4 NUMA nodes, per-mask scores, arbitrary preferred flags)."""
import numpy as np
import pytest

import golden_cases as G
from koordinator_amd import Engine, abi, framework as F
from oracle import oracle

GOLD = G.load("topology_policy.json")
ORDER = (1, 2, 4, 8, 3, 5, 9, 6, 10, 12, 7, 11, 13, 14, 15)  # IterateBitMasks over 4 NUMA nodes
POLICY = {"best-effort": abi.NUMA_POLICY["BestEffort"], "restricted": abi.NUMA_POLICY["Restricted"],
          "single-numa-node": abi.NUMA_POLICY["SingleNUMANode"]}


def provider_lists(providers):
    """filterProvidersHints (policy.go:94-125): one list per resource; a provider without hints (nil / empty map)
    contributes one preferred "don't care" hint, a nil resource slice the same, an empty one a non-preferred one.
    Resources in sorted-name order (the tables' results do not depend on the Go map order)."""
    lists = []
    for hints in providers:
        if not hints:
            lists.append([[None, True]])
            continue
        for res in sorted(hints):
            h = hints[res]
            lists.append([[None, True]] if h is None else ([[None, False]] if len(h) == 0 else h))
    return lists


def bits(mask):
    return sum(1 << b for b in mask)


def device_case(policy, num_numa, lists, scores=None):
    """One kg_debug_numa_merge case, or None when a list is not representable on the device."""
    if len(lists) == 0:
        lists = [[[None, True]]]  # no provider: mergeFilteredHints folds the empty permutation = one preferred nil
    if len(lists) > 2:
        return None
    c = np.zeros(abi.DBG_MERGE_WORDS, dtype=np.int64)
    c[0], c[1], c[2] = POLICY[policy], num_numa, len(lists)
    for l, hints in enumerate(lists):
        w = 3 + 5 * l
        if len(hints) == 0:
            c[w + 4] = 1  # empty
        elif any(h[0] is None for h in hints):
            if len(hints) != 1:
                return None
            c[w + 2], c[w + 3] = 1, int(hints[0][1])
        else:
            for m, pref in hints:
                k = ORDER.index(bits(m))
                c[w] |= 1 << k
                if pref:
                    c[w + 1] |= 1 << k
    if scores is not None:
        c[13:29] = scores
    return c


def _unpack(row):
    admit, nil, mask, pref = (int(x) for x in row[:4])
    return bool(admit), None if nil else [b for b in range(8) if (mask >> b) & 1], bool(pref)


@pytest.mark.parametrize("c", GOLD["merge"], ids=lambda c: f"{c['policy']}:{c['source_line'].split(':')[-1]}")
def test_policy_merge_oracle(c):
    admit, mask, pref, _ = oracle.policy_merge(c["policy"], 2, provider_lists(c["providers"]))
    assert [mask, pref] == c["want"], c["source_line"]
    assert admit == (True if c["policy"] == "best-effort" else pref)


@pytest.mark.parametrize("c", GOLD["single_numa_filter"], ids=lambda c: c["source_line"].split(":")[-1])
def test_single_numa_filter_oracle(c):
    assert oracle.single_numa_filter(c["lists"]) == c["want"], c["source_line"]


def test_can_admit_tables():
    """canAdmitPodResult: best-effort always admits, restricted and single-numa-node admit a preferred hint."""
    for policy, rows in GOLD["admit"].items():
        for r in rows:
            # a one-list merge of a single nil hint returns exactly {nil / default, preferred}
            admit, _, pref, _ = oracle.policy_merge(policy, 2, [[[None, r["preferred"]]]])
            assert pref == r["preferred"] and admit == r["want"], r["source_line"]


def test_every_merge_case_is_device_representable():
    assert all(device_case(c["policy"], 2, provider_lists(c["providers"])) is not None for c in GOLD["merge"])


@pytest.mark.gpu
def test_policy_merge_device():
    cases = [c for c in GOLD["merge"]]
    enc = np.stack([device_case(c["policy"], 2, provider_lists(c["providers"])) for c in cases])
    with Engine(F.build_config(), 1) as e:
        out = e.debug_numa_merge(enc)
    for c, row in zip(cases, out):
        admit, mask, pref = _unpack(row)
        assert [mask, pref] == c["want"], c["source_line"]
        assert admit == (True if c["policy"] == "best-effort" else pref), c["source_line"]


@pytest.mark.gpu
def test_can_admit_device():
    rows = [(policy, r) for policy, rs in GOLD["admit"].items() for r in rs]
    enc = np.stack([device_case(policy, 2, [[[None, r["preferred"]]]]) for policy, r in rows])
    with Engine(F.build_config(), 1) as e:
        out = e.debug_numa_merge(enc)
    for (policy, r), row in zip(rows, out):
        admit, _, pref = _unpack(row)
        assert pref == r["preferred"] and admit == r["want"], r["source_line"]


def _random_lists(rng, nn):
    """≤ 2 lists shaped like generateResourceHints: masks within the node's NUMA set in IterateBitMasks order,
    random preferred flags; sometimes a "don't care" or an empty list."""
    lists = []
    for _ in range(int(rng.integers(1, 3))):
        r = rng.random()
        if r < 0.1:
            lists.append([[None, bool(rng.random() < 0.5)]])
        elif r < 0.15:
            lists.append([])
        else:
            masks = [m for m in ORDER if m < (1 << nn) and rng.random() < 0.5]
            lists.append([[[b for b in range(4) if (m >> b) & 1], bool(rng.random() < 0.5)] for m in masks] or
                         [[None, True]])
    return lists


@pytest.mark.gpu
def test_policy_merge_device_matches_oracle_random():
    rng = np.random.default_rng(20250117)
    cases, want = [], []
    for _ in range(4000):
        nn = int(rng.integers(1, 5))
        policy = ("best-effort", "restricted", "single-numa-node")[int(rng.integers(0, 3))]
        lists = _random_lists(rng, nn)
        scores = rng.integers(0, 101, 16)
        scored = [[h + [int(scores[bits(h[0])]) if h[0] is not None else 0] for h in l] for l in lists]
        cases.append(device_case(policy, nn, lists, scores))
        want.append(oracle.policy_merge(policy, nn, scored))
    with Engine(F.build_config(), 1) as e:
        out = e.debug_numa_merge(np.stack(cases))
    for k, (row, w) in enumerate(zip(out, want)):
        assert _unpack(row) == w[:3] and int(row[4]) == w[3], (k, w)

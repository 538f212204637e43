"""(r6) NodeNUMAResource with reservations that hold cpusets: the oracle restatement (oracle/numa.c)
against the reference's own test tables (tests/golden/numa_reservation.json, transcribed by
tests/golden/make_golden_numa_rsv.py with source lines).  The device runs the same cases in
tests/test_numa_rsv_gpu.py."""
import numpy as np
import pytest

import golden_cases as G
from koordinator_amd import abi, framework
from oracle import oracle

DOC = G.load("numa_reservation.json")
NUMA_PROFILE = framework.Profile(filter=(framework.NODE_NUMA_RESOURCE,), score={framework.NODE_NUMA_RESOURCE: 1})


def words(cpus):
    w = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
    for c in cpus:
        w[c // 64] |= np.uint64(1) << np.uint64(c % 64)
    return w


def rsv_row(reservation_cpus, assigned_cpus):
    """One node's reservation slots: slot 0 holds `reservation_cpus`, its assigned pods `assigned_cpus`."""
    r = np.zeros(1, dtype=abi.NODE_RSV_DTYPE)
    r["n"] = 1
    r["available"][0, 0] = 1
    r["allocatable_cpu"][0, 0] = 1000 * len(reservation_cpus)
    r["cpus"][0, 0] = words(reservation_cpus)
    for a in assigned_cpus:
        r["cpus_assigned"][0, 0] |= words(a)
    r["assigned"][0, 0] = len(assigned_cpus)
    return r


@pytest.mark.parametrize("c", DOC["restore"], ids=lambda c: c["name"].replace(" ", "_"))
def test_restore_reserved_cpus(c):
    """TestRestoreReservation: the reservation's cpus minus its assigned pods'."""
    assert oracle.numa_rsv_reserved(rsv_row(c["reservation_cpus"], c["assigned_cpus"])[0], 0) == c["want"], \
        c["source_line"]


@pytest.mark.parametrize("c", DOC["available"], ids=lambda c: c["name"].replace(" ", "_"))
def test_available_with_preferred(c):
    nn = framework.make_node_numa(*c["topo"], allocated_cpus=c["allocated"])
    assert oracle.numa_available_pref(nn[0], c["preferred"]) == c["want"], c["source_line"]


@pytest.mark.parametrize("c", DOC["take_preferred"], ids=lambda c: c["name"].replace(" ", "_"))
def test_take_preferred(c):
    pol = DOC["take_preferred_policy"]
    got = oracle.take_preferred(tuple(c["topo"]), c["available"], c["preferred"], c["need"], pol["bind"],
                                pol["strategy"])
    assert got == c["want"], c["source_line"]


def reserve_case(c):
    cfg = framework.build_config(profile=NUMA_PROFILE)
    # the reservation's cpus are in NodeAllocation (addCPUs), with its assigned pods' on top
    alloc = sorted(set(c["reservation_cpus"]).union(*[set(a) for a in c["assigned_cpus"]]))
    nn = framework.make_node_numa(*c["topo"], allocated_cpus=alloc)
    pod = framework.make_pod({"cpu": str(c["cpus"])}, priority_class="koord-prod", qos="LSR",
                             preferred_cpu_bind_policy=c["preferred"])
    return cfg, nn, rsv_row(c["reservation_cpus"], c["assigned_cpus"]), pod


@pytest.mark.parametrize("c", DOC["reserve"], ids=lambda c: c["name"].replace(" ", "_"))
def test_reserve_from_reservation(c):
    cfg, nn, rsv, pod = reserve_case(c)
    rc, cpus = oracle.numa_reserve_rsv(cfg, nn[0], rsv[0], pod[0])
    assert rc == 0 and cpus == c["want"], c["source_line"]


def test_reserve_without_nomination_takes_free_cpus():
    """Without the reservation (a pod that may not use cpusets from it, AllowUseCPUSet false) the reservation's cpus
    stay allocated: the same request lands outside them."""
    c = DOC["reserve"][0]
    cfg, nn, rsv, _ = reserve_case(c)
    rc, cpus = oracle.numa_reserve(cfg, nn[0], framework.make_pod({"cpu": "4"}, priority_class="koord-prod",
                                                                   qos="LSR", preferred_cpu_bind_policy="FullPCPUs")[0])
    assert rc == 0 and not set(cpus) & set(c["reservation_cpus"])

"""(r6) NodeNUMAResource with reservations that hold cpusets: RestoreReservation's reserved cpus
(nodenumaresource/reservation.go:76-113) offered to the pod nominated into the reservation as preferredCPUs and reusable
NUMA cpu at Score and Reserve (plugin.go:465-535, node_allocation.go:133-177, cpu_accumulator.go:33-85), the RefCount-2
cpus an assigned pod shares with its reservation (node_allocation.go:76-131), and Unreserve.

* The reference's test tables (tests/golden/numa_reservation.json) run through the engine's Reserve on a one-node
  cluster with one reservation slot (device) and through the oracle's scheduling loop: restore, getAvailableCPUs with
  preferred cpus, takePreferredCPUs, and the plugin_test.go Reserve case.
* The shipped profile (LoadAware + NodeNUMAResource + DeviceShare + Reservation + ElasticQuota) with 30 % of the
  whole-core cpu reservations holding cpusets: device vs oracle bit-exact on placements, totals, slots, cpusets,
  minors, NUMA state and the reservations' assigned cpus, with Unreserve interleaved, at 1.5k and 50k nodes.

Known deviation (both sides alike): k8s v1.24 skips PreScore / Score when one node is feasible, so the reference's
NodeNUMAResource / DeviceShare Reserve then see no nominated reservation; the engine and the oracle always nominate."""
import numpy as np
import pytest

import golden_cases as G
import test_shipped_profile as SP
from koordinator_amd import Engine, abi, framework as F, synth
from oracle import oracle

DOC = G.load("numa_reservation.json")
RSV_NUMA = F.Profile(filter=(F.NODE_NUMA_RESOURCE, F.RESERVATION), score={F.NODE_NUMA_RESOURCE: 1, F.RESERVATION: 1})


def words(cpus):
    w = np.zeros(abi.MAX_CPUS // 64, dtype=np.uint64)
    for c in cpus:
        w[c // 64] |= np.uint64(1) << np.uint64(c % 64)
    return w


def one_node_case(topo, rsv_cpus, assigned, other, pod_cpus, bind, strategy=None):
    """(cfg, nodes, metrics, numa, rsv, existing pods, their nodes, pod): one node of `topo`; one Available reservation
    (owner group 0, cpu-only, allocatable = |rsv_cpus| cores, or 1 core without a cpuset) holding `rsv_cpus`, its
    assigned pods holding the cpu lists `assigned` (RefCount 2); other bound pods holding `other`; the pod (LSR
    koord-prod, owner group 0) requests `pod_cpus` cpus preferring `bind`."""
    cfg = F.build_config(profile=RSV_NUMA)
    total = topo[0] * topo[1] * topo[2] * topo[3]
    nodes = F.make_node({"cpu": f"{total * 1000}m", "memory": str(1 << 40)})
    metrics = np.zeros(1, dtype=abi.METRIC_DTYPE)
    alloc = sorted(set(rsv_cpus) | set(other).union(*[set(a) for a in assigned]))
    numa = F.make_node_numa(*topo, numa_allocate_strategy=strategy, allocated_cpus=alloc)
    rsv = np.zeros(1, dtype=abi.NODE_RSV_DTYPE)
    rc = 1000 * max(len(rsv_cpus), 1)
    rsv["n"] = 1
    rsv["available"][0, 0] = 1
    rsv["allocatable_cpu"][0, 0] = rc
    rsv["cpus"][0, 0] = words(rsv_cpus)
    for a in assigned:
        rsv["cpus_assigned"][0, 0] |= words(a)
    rsv["assigned"][0, 0] = len(assigned)
    rsv["allocated_cpu"][0, 0] = 1000 * sum(len(a) for a in assigned)
    ex = [F.make_pod({"cpu": f"{rc}m"})]  # the reserve pod in NodeInfo
    ex[0]["flags"] |= abi.POD_RESERVE
    ex += [F.make_pod({"cpu": str(len(a))}, priority_class="koord-prod", qos="LSR") for a in assigned]
    if other:
        ex.append(F.make_pod({"cpu": str(len(other))}, priority_class="koord-prod", qos="LSR"))
    ex = np.concatenate(ex)
    pod = F.make_pod({"cpu": str(pod_cpus)}, priority_class="koord-prod", qos="LSR", preferred_cpu_bind_policy=bind)
    pod["reservation_owner_mask"] = 1
    return cfg, nodes, metrics, numa, rsv, ex, np.zeros(len(ex), np.int32), pod


def run_oracle(cfg, nodes, metrics, numa, rsv, ex, ex_node, pod):
    st = oracle.states(1)
    oracle.add_pods(cfg, st, ex, ex_node)
    r = rsv.copy()
    node, _, slot, cpus, _ = oracle.schedule_resv(cfg, nodes, metrics, st, r, pod, 0, numa_buf=oracle.numa_states(numa),
                                                  with_numa=True)
    return int(node[0]), int(slot[0]), F.cpuset_of(cpus[0]), r


def run_engine(cfg, nodes, metrics, numa, rsv, ex, ex_node, pod):
    with Engine(cfg, 1) as e:
        e.upsert_nodes(nodes)
        e.update_metrics(metrics, 0)
        e.add_pods(ex, ex_node)
        e.upsert_numa(numa)
        e.upsert_reservations(rsv)
        e.stage(pod)
        e.schedule_staged(0, 1)
        node, _ = e.fetch(0, 1)
        return (int(node[0]), int(e.fetch_reservations(0, 1)[0]), F.cpuset_of(e.fetch_cpusets(0, 1)[0]),
                e.read_reservation_cpus())


def golden_cases():
    """Every table row as a one-node scheduling case: (id, case args, want cpus, reservation cpus, source line)."""
    out = []
    for c in DOC["reserve"]:
        out.append(("reserve-" + c["name"], (c["topo"], c["reservation_cpus"], c["assigned_cpus"], [], c["cpus"],
                                             c["preferred"]), c["want"], c["source_line"]))
    for c in DOC["restore"]:
        # the pod takes 2 cpus FullPCPUs: the reserved cpus when some are left (TestRestoreReservation's {8,9})
        out.append(("restore-" + c["name"], (c["topo"], c["reservation_cpus"], c["assigned_cpus"], [], 2, "FullPCPUs"),
                    c["want"] if c["want"] else None, c["source_line"]))
    for c in DOC["available"]:
        # the reservation holds the preferred cpus, a bound pod the rest of the allocated ones; a pod needing every
        # available cpu (FullPCPUs preferred, not required) takes exactly getAvailableCPUs' set
        other = [x for x in c["allocated"] if x not in c["preferred"]]
        out.append(("available-" + c["name"], (c["topo"], c["preferred"], [], other, len(c["want"]), "FullPCPUs"),
                    c["want"], c["source_line"]))
    pol = DOC["take_preferred_policy"]
    for c in DOC["take_preferred"]:
        total = c["topo"][0] * c["topo"][1] * c["topo"][2] * c["topo"][3]
        other = [x for x in range(total) if x not in c["available"]]
        out.append(("take-" + c["name"], (c["topo"], c["preferred"], [], other, c["need"], pol["bind"], pol["strategy"]),
                    c["want"], c["source_line"]))
    return out


CASES = golden_cases()


@pytest.mark.parametrize("case", CASES, ids=[c[0].replace(" ", "_") for c in CASES])
def test_golden_oracle_loop(case):
    """The oracle's scheduling loop (nomination, RestoreReservation, preferred cpus at Reserve) reproduces the tables."""
    _, args, want, src = case
    node, slot, cpus, r = run_oracle(*one_node_case(*args))
    assert node == 0 and slot == 0, src
    if want is None:  # nothing reserved: the pod's cpus come from the free ones
        assert not set(cpus) & set(args[1]) and len(cpus) == args[4], src
    else:
        assert cpus == sorted(want), src
    if args[1]:  # the reservation's assigned cpus now hold the pod's
        assert set(F.cpuset_of(r["cpus_assigned"][0, 0])) >= set(cpus) & set(args[1]), src


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0].replace(" ", "_") for c in CASES])
def test_golden_device(case):
    _, args, want, src = case
    a = one_node_case(*args)
    node, slot, cpus, assigned = run_engine(*a)
    w = run_oracle(*a)
    assert (node, slot, cpus) == w[:3], src
    if want is None:
        assert not set(cpus) & set(args[1]) and len(cpus) == args[4], src
    else:
        assert cpus == sorted(want), src
    assert np.array_equal(assigned[0], w[3]["cpus_assigned"][0]), src


# ---------------------------------------------------------------------------------------------------------------
# the shipped profile with cpuset reservations
# ---------------------------------------------------------------------------------------------------------------
def cpuset_workload(n_nodes, n_pods, seed, frac=0.3):
    cluster, numa, dev, rsv, pods, quotas = SP.workload(n_nodes, n_pods, seed)
    made = synth.add_cpuset_reservations(numa, rsv, frac, seed=seed + 9)
    assert made > 0
    return cluster, numa, dev, rsv, pods, quotas


def test_oracle_cpuset_reservations_used():
    """The oracle places owned cpuset pods into cpuset reservations and takes their reserved cpus."""
    cluster, numa, dev, rsv, pods, quotas = cpuset_workload(400, 1500, 181, frac=0.6)
    w = SP.oracle_run(SP.config(), cluster, numa, dev, rsv, pods, quotas)
    took = 0
    for j in np.flatnonzero(w["slot"] >= 0):
        i, s = int(w["node"][j]), int(w["slot"][j])
        r = set(F.cpuset_of(rsv["cpus"][i, s])) - set(F.cpuset_of(rsv["cpus_assigned"][i, s]))
        took += bool(r & set(F.cpuset_of(w["cpus"][j])))
    assert took > 0
    assert (w["rsv"]["cpus_assigned"] != rsv["cpus_assigned"]).any()


def check_cpusets(cluster, numa, dev, rsv, pods, quotas, chunks):
    cfg = SP.config()
    g, w = SP.check(cfg, cluster, numa, dev, rsv, pods, quotas, chunks)
    with Engine(cfg, cluster.n) as e:  # the assigned cpus after the same queue
        synth.load_shipped_into(e, cluster, numa, dev, rsv, quotas)
        e.stage(pods)
        e.schedule_staged(0, len(pods))
        got = e.read_reservation_cpus()
    on = np.arange(abi.MAX_RSV_SLOTS)[None, :] < rsv["n"][:, None]
    holds = (rsv["cpus"] != 0).any(axis=2) & on
    assert np.array_equal(got[holds], w["rsv"]["cpus_assigned"][holds])
    return g, w


@pytest.mark.gpu
@pytest.mark.parametrize("n_nodes,n_pods,seed,chunks", [(1500, 1500, 191, 2), (120, 900, 192, 1)])
def test_shipped_cpuset_reservations_parity(n_nodes, n_pods, seed, chunks):
    cluster, numa, dev, rsv, pods, quotas = cpuset_workload(n_nodes, n_pods, seed, frac=0.6)
    g, w = check_cpusets(cluster, numa, dev, rsv, pods, quotas, chunks)
    assert (w["rsv"]["cpus_assigned"] != rsv["cpus_assigned"]).any()  # some pod took reserved cpus


@pytest.mark.gpu
def test_shipped_cpuset_reservations_parity_50k_nodes():
    """The verdict's bar: the shipped profile with 30 % cpuset reservations, 50k nodes, device vs oracle bit-exact."""
    cluster, numa, dev, rsv, pods, quotas = cpuset_workload(50_000, 2000, 193, frac=0.3)
    check_cpusets(cluster, numa, dev, rsv, pods, quotas, 1)


@pytest.mark.gpu
def test_cpuset_reservations_unreserve():
    """Unreserve of half the placed pods returns their cpus to the reservations' reserved cpus (a cpu a reservation
    holds keeps RefCount 1 and stays allocated); the next batch places alike on both sides."""
    cfg = SP.config()
    cluster, numa, dev, rsv, pods, quotas = cpuset_workload(300, 900, 195, frac=0.8)
    first, second = pods[:600], pods[600:]
    w = SP.oracle_run(cfg, cluster, numa, dev, rsv, first, quotas)
    mask = (np.arange(len(first)) % 2 == 0) & (w["node"] >= 0)
    for j in np.flatnonzero(mask):
        oracle.unreserve(cfg, w["st"], first[j], int(w["node"][j]), numa_buf=w["numa"], devices=w["dev"], rsv=w["rsv"],
                         quotas=w["quotas"], cpus=w["cpus"][j], numa_alloc=w["nalloc"][j], minors=int(w["minors"][j]),
                         slot=int(w["slot"][j]))
    after_numa = oracle.numa_state_read(w["numa"], cluster.n)
    node2, score2, slot2, minors2, cpus2, _ = oracle.schedule_resv(cfg, cluster.nodes, cluster.metrics, w["st"], w["rsv"],
                                                                  second, cluster.now_ns, devices=w["dev"],
                                                                  quotas=w["quotas"], n_threads=8, with_minors=True,
                                                                  numa_buf=w["numa"], with_numa=True)
    with Engine(cfg, cluster.n) as e:
        synth.load_shipped_into(e, cluster, numa, dev, rsv, quotas)
        e.stage(first)
        e.schedule_staged(0, len(first))
        e.unreserve(0, len(first), mask.astype(np.uint8))
        ga, gc, gm = e.read_numa()
        wa, wc, wm = after_numa
        assert np.array_equal(ga, wa) and np.array_equal(gc, wc) and np.array_equal(gm, wm)
        e.stage(second)
        e.schedule_staged(0, len(second))
        node, score = e.fetch(0, len(second))
        assert np.array_equal(node, node2) and np.array_equal(score, score2)
        assert np.array_equal(e.fetch_reservations(0, len(second)), slot2)
        assert np.array_equal(e.fetch_devices(0, len(second)), minors2)
        assert np.array_equal(e.fetch_cpusets(0, len(second)), cpus2)
        on = (rsv["cpus"] != 0).any(axis=2) & (np.arange(abi.MAX_RSV_SLOTS)[None, :] < rsv["n"][:, None])
        assert np.array_equal(e.read_reservation_cpus()[on], w["rsv"]["cpus_assigned"][on])

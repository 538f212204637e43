"""(r6) Oracle fixtures of the C4 and shipped bench queues: tests/golden/c4_queue.npz, shipped_queue.npz.

TEST INFRASTRUCTURE.  Builds the workload exactly as bench.py does (bench.Work: the same cluster, the prefix-stable
queue synth.make_stream draws, the shipped ElasticQuota groups sized on the queue's first 25k pods) and runs the
oracle's sequential FIFO schedule (bench.Work.oracle_run: oracle/oracle.c or_schedule_numa for C4,
oracle/reservation.c or_schedule_resv_full for shipped) over the first --pods pods.  Writes every placement, the
per-segment SHA-256 of the queue (so a consumer proves it generated the same pods) and the metadata.  bench.py's
fixture_check compares the device's placements of every timed pod with it; tests/test_bench_fixtures.py re-checks it
on the CPU.

    python tests/golden/make_bench_fixture.py --workload c4 --pods 100000 --threads 4
    python tests/golden/make_bench_fixture.py --workload shipped --pods 50000 --threads 4
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=("c4", "shipped"), required=True)
    ap.add_argument("--pods", type=int, required=True)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--seg", type=int, default=5000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import bench
    from koordinator_amd import framework

    wl = a.workload
    nodes = bench.WORKLOADS[wl][0]
    profile, la = bench.workload_profile(wl)
    cfg = framework.build_config(profile=profile, la=la)
    work = bench.Work(wl, nodes, cfg)
    pods = work.make_pods(a.pods, seed=work.seed + 1)
    work.set_queue(pods)
    assert a.pods % a.seg == 0
    t0 = time.time()
    node, desc = work.oracle_run(pods, a.threads)
    dt = time.time() - t0
    seg_sha = np.array([hashlib.sha256(np.ascontiguousarray(pods[s * a.seg:(s + 1) * a.seg]).tobytes()).hexdigest()
                        for s in range(a.pods // a.seg)])
    meta = {"workload": wl, "nodes": nodes, "pods": a.pods, "cluster_seed": work.seed, "pods_seed": work.seed + 1,
            "queue": "synth.make_stream", "segment": a.seg, "oracle": desc, "threads": a.threads,
            "quota_basis": bench.Work.QUOTA_BASIS if wl == "shipped" else None, "seconds": round(dt, 1)}
    out = a.out or os.path.join(ROOT, "tests", "golden", f"{wl}_queue.npz")
    np.savez_compressed(out, node=np.asarray(node, dtype=np.int32), seg_sha=seg_sha, meta=json.dumps(meta))
    print(f"[{wl} fixture] {a.pods} pods in {dt:.0f} s, placed {(np.asarray(node) >= 0).sum()}, wrote {out}",
          flush=True)


if __name__ == "__main__":
    main()

"""Model of the C3 resolver's slow paths (analysis, not a test): which pods re-score modified rows, and how many of
those re-scores a resolver would still need if the rows modified by EARLIER rounds came pre-scored (exact keys per
pod computed wave-parallel before the chain starts), leaving only rows modified within the round itself.

Sequential oracle schedule (the ground truth) + the round protocol's snapshots at depth D: round r's records come
from the table after rounds <= r - D; pod j's slow path (today) = some node listed above its first candidate that no
earlier pod since the snapshot modified.  Usage: python scripts/r05/slowpath_model.py [nodes] [pods] [depth...]"""
import sys

import numpy as np

sys.path.insert(0, ".")
from koordinator_amd import framework as F, synth  # noqa: E402
from oracle import oracle  # noqa: E402

KC, B = 64, 32


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    npods = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    depths = [int(x) for x in sys.argv[3:]] or [2, 3, 4]
    cfg = F.build_config()
    cluster = synth.make_cluster(n, seed=7)
    pods = synth.make_pods(npods, seed=8)
    st0 = oracle.states(n)
    oracle.add_pods(cfg, st0, cluster.existing_pods, cluster.existing_node)
    st = st0.copy()
    win, _ = oracle.schedule(cfg, cluster.nodes, cluster.metrics, st, pods, cluster.now_ns, 8)
    nr = (npods + B - 1) // B
    snaps = [st0.copy()]  # table after rounds < r
    s = st0.copy()
    for r in range(nr):
        for j in range(r * B, min((r + 1) * B, npods)):
            if win[j] >= 0:
                oracle.apply_pod(cfg, s, pods[j], int(win[j]))
        snaps.append(s.copy())
    K = 4
    for D in depths:
        slow = slow_round = slow_pre = 0
        for r in range(nr):
            snap = snaps[max(r - D + 1, 0)]  # after rounds <= r - D
            cur = snaps[r]                   # after rounds <= r - 1: the state the pre-scoring sees
            prev = sorted(set(int(w) for w in win[max(r - D + 1, 0) * B:r * B] if w >= 0))
            this = set()
            for j in range(r * B, min((r + 1) * B, npods)):
                keys = oracle.node_keys(cfg, cluster.nodes, cluster.metrics, snap, pods[j], cluster.now_ns, 0, n)
                top = np.sort(keys[keys != 0])[::-1][:KC]
                nodes = [0xFFFFFFFF - (int(k) & 0xFFFFFFFF) for k in top]
                pos = next((i for i, x in enumerate(nodes) if x not in prev and x not in this), len(nodes))
                c1 = int(top[pos]) if pos < len(top) else 0
                if pos > 0:
                    slow += 1
                    if any(x in this for x in nodes[:pos]):
                        slow_round += 1
                # the pre-scored design: exact round-start keys of the earlier rounds' rows, top K per pod
                pk = []
                for w in prev:
                    k = int(oracle.node_keys(cfg, cluster.nodes, cluster.metrics, cur, pods[j], cluster.now_ns, w,
                                             w + 1)[0])
                    if k:
                        pk.append(k)
                pk = sorted(pk, reverse=True)[:K]
                pn = [0xFFFFFFFF - (k & 0xFFFFFFFF) for k in pk]
                c2i = next((i for i, x in enumerate(pn) if x not in this), None)
                if c2i is None and len(prev) > len(pk) - 0 and len(pk) == K:
                    slow_pre += 1  # every pre-scored candidate was re-modified in this round: full re-score
                else:
                    c2 = pk[c2i] if c2i is not None else 0
                    best = max(c1, c2)
                    s1 = any(x in this and int(top[i]) > best for i, x in enumerate(nodes[:pos]))
                    s2 = any(pk[i] > best for i in range(c2i if c2i is not None else len(pk)))
                    slow_pre += 1 if (s1 or s2) else 0
                if win[j] >= 0:
                    this.add(int(win[j]))
        print(f"D={D}: pods {npods}, slow paths today {slow} ({slow / npods:.1%}), this-round rows only "
              f"{slow_round} ({slow_round / npods:.1%}), pre-scored design (K={K}) {slow_pre} "
              f"({slow_pre / npods:.1%})", flush=True)


if __name__ == "__main__":
    main()

"""Executable model of the engine's round protocol — TEST INFRASTRUCTURE.

The HIP engine schedules a FIFO pod queue in rounds of B pods:
  eval    — every pod of the round scored on every node of this rank's shard against a table snapshot; per
            (pod, tile) only the top-kR packed keys survive;
  merge   — per pod: the top-kC keys of the union + a strict upper bound `ub` on every key left out;
  [ranks] — the per-rank records are all-gathered and merged again (same rule);
  resolve — pods replayed in queue order: best unmodified listed candidate vs the exact re-score of every row
            modified since the snapshot; valid iff ≥ ub, else the round stops and the pod is retried.
With `pipelined=True` the snapshot a round is evaluated on is the table as it was BEFORE the previous round
was resolved (the engine overlaps eval(r+1) with resolve(r)), and the previous round's rows count as modified.

This model runs the protocol with the oracle as the per-node scoring function (oracle.node_keys) so that its
placements can be compared with the oracle's sequential schedule (oracle.schedule) on the same inputs, in one
process or sharded over torch.distributed ranks (gloo) — the multi-GPU exchange path without a GPU.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle


def _node(k: int) -> int:
    return 0xFFFFFFFF - (k & 0xFFFFFFFF)


def _top_with_ub(keys, kc: int, ub_in: int):
    """Top-kc non-zero keys (descending) of `keys` + a strict upper bound on the rest (merge_round)."""
    nz = sorted((int(k) for k in keys if k), reverse=True)
    top = nz[:kc]
    ub = ub_in
    if len(nz) > kc:
        ub = max(ub, nz[kc] + 1)
    return top, ub


def tile_record(keys: np.ndarray, tile: int, kr: int, kc: int):
    """eval_round + merge_round<false> for one pod on one rank's shard (keys in node order)."""
    union, ub = [], 0
    for t0 in range(0, len(keys), tile):
        t = keys[t0:t0 + tile]
        feas = [int(k) for k in t if k]
        if len(feas) <= kr:
            lst = feas
        else:
            lst = sorted(feas, reverse=True)[:kr]
        if len(lst) == kr:  # full list: the tile's unseen nodes score below its minimum
            ub = max(ub, min(lst))
        union.extend(lst)
    return _top_with_ub(union, kc, ub)


def merge_ranks(records, kc: int):
    """merge_round<true>: the per-rank records of one pod → the final record."""
    union = [k for top, _ in records for k in top]
    return _top_with_ub(union, kc, max(ub for _, ub in records))


class RoundModel:
    def __init__(self, cfg, cluster, B=32, tile=256, kr=8, kc=64, rank=0, world=1, allgather=None,
                 pipelined=False):
        self.cfg, self.cl = cfg, cluster
        self.B, self.tile, self.kr, self.kc = B, tile, kr, kc
        self.rank, self.world = rank, world
        self.allgather = allgather  # callable(list_of_records) -> list over ranks of lists of records
        self.pipelined = pipelined
        n = cluster.n
        shard = -(-n // world) if n else 0
        self.lo = min(n, rank * shard)
        self.hi = min(n, self.lo + shard)
        self.st = oracle.states(n)
        if len(cluster.existing_pods):
            oracle.add_pods(cfg, self.st, cluster.existing_pods, cluster.existing_node)
        self.stats = {"rounds": 0, "breaks": 0, "slow_path": 0, "resyncs": 0}

    def _records(self, pods, state):
        cl = self.cl
        recs = []
        for p in pods:
            keys = oracle.node_keys(self.cfg, cl.nodes, cl.metrics, state, p, cl.now_ns, self.lo, self.hi)
            recs.append(tile_record(keys, self.tile, self.kr, self.kc))
        if self.world > 1:
            per_rank = self.allgather(recs)
            recs = [merge_ranks([per_rank[r][j] for r in range(self.world)], self.kc) for j in range(len(pods))]
        return recs

    def _key_now(self, pod, node: int) -> int:
        cl = self.cl
        return int(oracle.node_keys(self.cfg, cl.nodes, cl.metrics, self.st, pod, cl.now_ns, node, node + 1)[0])

    def schedule(self, pods):
        out_node = np.full(len(pods), -1, dtype=np.int32)
        out_score = np.zeros(len(pods), dtype=np.int64)
        cursor = 0
        snap = self.st.copy()  # the table the next round is evaluated on
        prev_mod: set = set()  # rows modified after `snap` was taken, before this round (pipelined)
        while cursor < len(pods):
            rp = pods[cursor:cursor + self.B]
            eval_state = snap if self.pipelined else self.st
            recs = self._records(rp, eval_state)
            if self.pipelined:
                snap = self.st.copy()  # eval(r+1) overlaps resolve(r): it sees the table before this round
            mod = set(prev_mod) if self.pipelined else set()
            cur: set = set()  # rows this round modifies (may repeat rows of the previous round)
            consumed = 0
            for j, p in enumerate(rp):
                top, ub = recs[j]
                pos = next((i for i, k in enumerate(top) if _node(k) not in mod), None)
                e = top[pos] if pos is not None else 0
                mbest = max((self._key_now(p, m) for m in mod), default=0)
                if pos == 0 and mbest > e:
                    raise AssertionError("monotone shortcut violated: a modified row beats the top candidate")
                self.stats["slow_path"] += int(bool(mod) and pos != 0)
                best = max(e, mbest)
                if best < ub:
                    self.stats["breaks"] += 1
                    break
                consumed += 1
                if best:
                    w = _node(best)
                    out_node[cursor + j] = w
                    out_score[cursor + j] = best >> 32
                    oracle.apply_pod(self.cfg, self.st, p, w, +1)
                    mod.add(w)
                    cur.add(w)
            self.stats["rounds"] += 1
            cursor += consumed
            if self.pipelined:
                if consumed < len(rp):
                    # the engine's speculative next round started at the wrong pod: the host re-syncs and
                    # restarts the pipeline from the fully written table
                    self.stats["resyncs"] += 1
                    snap = self.st.copy()
                    prev_mod = set()
                else:
                    prev_mod = cur
        return out_node, out_score

"""The engine's round protocol (tile top-k → merge with upper bound → [rank all-gather + merge] → FIFO resolve),
run on CPU through tests/round_model.py with the oracle as the per-node scorer, must place every pod exactly
where the sequential oracle does — single rank, pipelined (eval of round r+1 on the table before round r's
resolve), and sharded over a world_size-2 gloo process group (the multi-GPU exchange path)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from koordinator_amd import framework, synth
from oracle import oracle
from round_model import RoundModel

# (nodes, pods, B, tile, kR, kC): the engine's geometry, and shrunken tiles/lists that force truncated tile
# lists, upper-bound breaks and resyncs at small N
GEOMS = [
    (300, 400, 32, 256, 8, 64),
    (500, 600, 32, 32, 2, 64),
    (257, 300, 8, 16, 2, 16),
    (120, 400, 1, 64, 8, 64),
]


def _case(n, npods, seed=7):
    cfg = framework.build_config()
    cl = synth.make_cluster(n, seed=seed)
    pods = synth.make_pods(npods, seed=seed + 1)
    return cfg, cl, pods


@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("n,npods,B,tile,kr,kc", GEOMS)
def test_round_protocol_matches_sequential_oracle(n, npods, B, tile, kr, kc, pipelined):
    cfg, cl, pods = _case(n, npods)
    on, os_, st = oracle.schedule_cluster(cfg, cl, pods)
    m = RoundModel(cfg, cl, B=B, tile=tile, kr=kr, kc=kc, pipelined=pipelined)
    gn, gs = m.schedule(pods)
    np.testing.assert_array_equal(gn, on)
    np.testing.assert_array_equal(gs, os_)
    np.testing.assert_array_equal(m.st, st)  # final NodeInfo / assign-cache state too


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, geom, pipelined, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, npods, B, tile, kr, kc = geom
        cfg, cl, pods = _case(n, npods, seed=11)

        def allgather(recs):
            out = [None] * world
            dist.all_gather_object(out, recs)
            return out

        m = RoundModel(cfg, cl, B=B, tile=tile, kr=kr, kc=kc, rank=rank, world=world, allgather=allgather,
                       pipelined=pipelined)
        node, score = m.schedule(pods)
        np.save(os.path.join(out_dir, f"node{rank}.npy"), node)
        np.save(os.path.join(out_dir, f"score{rank}.npy"), score)
        np.save(os.path.join(out_dir, f"range{rank}.npy"), np.array([m.lo, m.hi]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("geom", [GEOMS[0], GEOMS[2]])
def test_two_rank_gloo_sharded_protocol(tmp_path, geom, pipelined):
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), geom, pipelined, str(tmp_path)), nprocs=world, join=True)
    n, npods = geom[0], geom[1]
    cfg, cl, pods = _case(n, npods, seed=11)
    on, os_, _ = oracle.schedule_cluster(cfg, cl, pods)
    ranges = [tuple(np.load(tmp_path / f"range{r}.npy")) for r in range(world)]
    # contiguous shards covering [0, N): global index = snapshot index
    assert ranges[0][0] == 0 and ranges[-1][1] == n and ranges[0][1] == ranges[1][0]
    for r in range(world):  # every rank resolves identically on its replica
        np.testing.assert_array_equal(np.load(tmp_path / f"node{r}.npy"), on)
        np.testing.assert_array_equal(np.load(tmp_path / f"score{r}.npy"), os_)

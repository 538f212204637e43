"""The RCCL library path of the multi-rank engine (ncclGetUniqueId → ncclCommInitRank → ncclCommSplit →
ncclAllGather on a HIP stream) on a one-rank communicator.  A one-GPU box cannot hold two RCCL ranks (RCCL refuses two
ranks on one device), so the multi-rank logic itself is covered by the loopback and gloo-hosted tests
(test_multirank_loopback.py, test_dist_engine_gloo.py); this checks the collective library the driver's 8-GPU run
uses, through the C ABI."""
import pytest

from koordinator_amd import abi


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 4096, 1 << 20])
def test_rccl_one_rank_allgather(n):
    lib = abi.load_library()
    abi.check(lib, lib.kg_debug_rccl_selftest(0, n))


@pytest.mark.gpu
def test_rccl_selftest_rejects_bad_size():
    lib = abi.load_library()
    assert lib.kg_debug_rccl_selftest(0, 0) != 0

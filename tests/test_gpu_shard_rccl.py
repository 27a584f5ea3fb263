"""lx_shard_comm (include/lachesis_hip.h): the column-shard collectives issued
by the library over RCCL, the path a Go caller binds without PyTorch.

A one-GPU box can only form a one-rank communicator (RCCL refuses two ranks
on one device), so this checks the RCCL load / communicator / stream-ordered
ForklessCause plumbing at nranks = 1 against the oracle, and the argument
checks.  The multi-rank protocol itself (block offsets, uint16 wire, partial
sums + all-reduce) is the one tests/test_gpu_shards.py and
tests/test_gpu_shard_dist.py check bit-exactly through ShardedIndex."""

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


def test_shard_comm_single_rank_fc_matches_oracle():
    import torch
    import lachesis_hip as lx
    d = lx.tools.gen_dag(12, 25, 4, 3, 4, 13)
    w = [5, 4, 4, 3, 3, 2, 2, 1, 1, 1, 1, 1]
    ix = lx.Index(device=0)
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    uid = lx.shard_comm_unique_id()
    assert len(uid) == 128
    comm = lx.ShardComm(ix, uid, 1, 0)
    comm.exchange()                       # one rank: whole rows already local
    qa, qb = lx.tools.fc_queries(d.lamport, 30_000, window=20, seed=13)
    dev = torch.device("cuda", 0)
    a = torch.from_numpy(qa.view(np.int32)).to(dev)
    b = torch.from_numpy(qb.view(np.int32)).to(dev)
    out = torch.empty(len(qa), dtype=torch.uint8, device=dev)
    comm.forkless_cause_dev(len(qa), a.data_ptr(), b.data_ptr(), out.data_ptr())
    ix.sync()
    np.testing.assert_array_equal(out.cpu().numpy(), o.forkless_cause_batch(qa, qb))
    comm.close()


def test_shard_comm_rejects_mismatched_rank():
    import lachesis_hip as lx
    ix = lx.Index(device=0, shard_rank=1, shard_count=2)
    ix.reset([1, 1, 1, 1])
    assert ix.shard_of() == (1, 2)
    uid = lx.shard_comm_unique_id()
    with pytest.raises(lx.LxError):
        lx.ShardComm(ix, uid, 2, 0)       # handle is shard 1 of 2
    with pytest.raises(lx.LxError):
        lx.ShardComm(ix, uid, 3, 1)       # handle has 2 shards

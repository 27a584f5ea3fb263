"""The column-sharded index end to end through torch.distributed: G processes
(gloo, all on cuda:0 -- the driver's N-GPU runs use RCCL, one GPU per rank)
each hold a shard handle, index the same fork DAG, run
lachesis_hip.shard.ShardedIndex.exchange (all-to-all of LowestAfter blocks)
and forkless_cause_dev (partial stake sums + all-reduce); every rank's answers
must equal the C oracle."""

import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lachesis_hip as lx
        from lachesis_hip.shard import ShardedIndex
        from oracle import corc
        d = lx.tools.gen_dag(28, 40, 6, 5, 6, 3)
        rng = np.random.default_rng(3)
        weights = sorted((int(x) for x in rng.integers(1, 40, 28)), reverse=True)
        ix = lx.Index(device=0, shard_rank=rank, shard_count=world)
        ix.reset(weights)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        dev = torch.device("cuda", 0)
        si = ShardedIndex(ix, device=dev)
        si.exchange()
        qa, qb = lx.tools.fc_queries(d.lamport, 30_000, window=30, seed=5)
        out = si.forkless_cause_dev(torch.from_numpy(qa.view(np.int32)).to(dev),
                                    torch.from_numpy(qb.view(np.int32)).to(dev)).cpu().numpy()
        o = corc.OracleIndex(weights)
        assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
        q.put((rank, bool(np.array_equal(out, o.forkless_cause_batch(qa, qb))), int(out.sum())))
    except Exception as e:   # report instead of hanging the other ranks' queue reads
        q.put((rank, False, repr(e)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_index_over_torch_distributed(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    assert len({n for *_, n in res}) == 1          # every rank holds the same answers

"""The column-sharded index as a drop-in abft.DagIndexer.

G processes (gloo, all on cuda:0 -- RCCL with one GPU per rank is the
product path; lx_shard_get_rows / lx_forkless_cause_sharded_dev are its C
form) each hold a shard handle behind lachesis_hip.shard.ShardedDagIndexer
and run the unchanged caller -- abft.IndexedLachesis restated in
oracle/abft_oracle.py (abft/indexed_lachesis.go:17-99: Build = Add +
DropNotFlushed, Process = Add + ForklessCause per pair + Flush, and
abft/lachesis.go:56-57: GetMergedHighestBefore(atropos) for the cheaters) --
over a fork DAG (tdag.ForEachRandFork shape with double-signers).  Every
rank's blocks (frame, Atropos, cheaters, confirmed events) must equal the
caller's over the C oracle index; the whole getter rows of every event
(HighestBefore, LowestAfter, merged HighestBefore) must equal an unsharded
handle's byte for byte."""

import multiprocessing as mp
import os
import socket

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_caller(index, weights, cheaters, events_per_node):
    """testConfirmBlocks' driver (frame_decide_test.go:57-124): Build + Process
    of every event of a fork DAG, the blocks recorded."""
    from abft_harness import FakeLachesis, node_ids
    from oracle import tdag
    from oracle.tdag import SplitMix64
    nodes = node_ids(len(weights), seed=len(weights) + cheaters)
    t = FakeLachesis(dict(zip(nodes, weights)), index)
    evs = []

    def build(e):
        e.epoch = 1
        t.build(e)                      # Add + DropNotFlushed (a real rollback)
        assert t.process(e) is None     # Add + ForklessCause + Flush
        evs.append(e)
        return True
    tdag.rand_fork_dag(len(nodes), events_per_node, min(5, len(nodes)), cheaters=cheaters, forks_count=6,
                       node_ids=nodes, rng=SplitMix64(len(nodes) + cheaters), build=build)
    return t, evs


def _worker(rank, world, port, q, weights, cheaters, epn):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd"), os.path.join(ROOT, "tests")]
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lachesis_hip as lx
        from lachesis_hip.shard import ShardedDagIndexer, ShardedIndex
        from oracle import abft_oracle as ao
        dev = torch.device("cuda", 0)
        ix = lx.Index(device=0, shard_rank=rank, shard_count=world)
        sdi = ShardedDagIndexer(ShardedIndex(ix, device=dev))
        t, evs = _run_caller(sdi, weights, cheaters, epn)
        want, _ = _run_caller(ao.DenseOracleIndex(), weights, cheaters, epn)
        blocks_ok = t.block_list == want.block_list and len(t.block_list) >= 3
        n_cheaters = max((len(b[3]) for b in t.block_list), default=0)
        # whole rows of every event, joined over the shards, against one unsharded handle
        sdi._fresh()
        n = len(sdi.ids)
        full = lx.Index(device=0)
        full.reset(list(sdi.validators.weights))
        pos = sdi.pos
        by_id = {e.id: e for e in evs}
        for eid in sdi.ids:
            e = by_id[eid]
            full.add(sdi.validators.idxs[e.creator], e.seq, [pos[p] for p in e.parents])
        rows_ok = True
        for mode in (0, 1, 2):
            got = sdi.sx.get_rows(mode, np.arange(n, dtype=np.uint32))
            off, raw = full.rows_np(mode, np.arange(n, dtype=np.uint32))
            for i in range(n):
                if got[i] != bytes(raw[off[i]:off[i + 1]]):
                    rows_ok = False
                    break
        full.close()
        q.put((rank, blocks_ok, rows_ok, len(t.block_list), n_cheaters))
    except Exception as e:   # report instead of hanging the other ranks' queue reads
        import traceback
        q.put((rank, False, False, repr(e) + traceback.format_exc()[-1500:], -1))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,weights,cheaters,epn", [
    (2, [1, 2, 1, 2, 1, 2, 1, 2, 1, 2], 3, 30),
    (3, [5, 9, 1, 3, 7, 2, 8, 4, 6, 1, 2, 9, 3, 5, 7, 4], 4, 20),
])
def test_sharded_dag_indexer_drives_the_caller(world, weights, cheaters, epn):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, weights, cheaters, epn)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(b and r for _, b, r, *_ in res), res
    assert max(c for *_, c in res) >= 1, res     # the forks were detected: cheaters in some block

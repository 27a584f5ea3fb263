"""Multi-process protocol of the column-sharded index (lachesis_hip/shard.py)
on CPU with gloo, world sizes 2 and 3.

The GPU kernels behind the provider interface are covered by
tests/test_gpu_shards.py; here a numpy provider with the same semantics
stands in for them so the collective plumbing (block sizes, all-to-all
placement, partial-sum all-reduce, combine) runs without a GPU:

* rank r initially knows LowestAfter rows of events on its own branches, all
  columns (what its walker fills), and must end with every row of its own
  columns (what its FC kernel reads);
* the partial for (a, b) is the stake of own creators c with
  0 < LA[b][c] <= HB[a][c]; the combine is ``sum >= quorum``.
"""

import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _bounds(V, G, q):
    return V if q >= G else (V * q // G) & ~3


class FakeShard:
    def __init__(self, rank, G, la, hb, owner, weights):
        self.r, self.G = rank, G
        self.la_full, self.hb, self.owner, self.w = la, hb, owner, np.asarray(weights, np.int64)
        V = la.shape[1]
        self.cols = [np.arange(_bounds(V, G, q), _bounds(V, G, q + 1)) for q in range(G)]
        self.rows = [np.nonzero(np.isin(owner, self.cols[q]))[0] for q in range(G)]
        self.la = np.zeros_like(la)                 # this rank's view
        self.la[self.rows[rank]] = la[self.rows[rank]]
        self.quorum = int(self.w.sum()) * 2 // 3 + 1

    @staticmethod
    def _view(ptr, n):
        return np.ctypeslib.as_array((ctypes.c_int32 * n).from_address(ptr))

    def shard_block(self, src, dst):
        return len(self.rows[src]) * len(self.cols[dst])

    def la_pack_dev(self, dst, ptr):
        blk = self.la[np.ix_(self.rows[self.r], self.cols[dst])]
        self._view(ptr, blk.size)[:] = blk.reshape(-1)

    def la_unpack_dev(self, src, ptr):
        n = self.shard_block(src, self.r)
        blk = self._view(ptr, n).reshape(len(self.rows[src]), len(self.cols[self.r]))
        self.la[np.ix_(self.rows[src], self.cols[self.r])] = blk

    def la_own_dev(self):
        pass                                        # own block already in self.la

    def forkless_cause_partial_dev(self, n, pa, pb, pout):
        a, b = self._view(pa, n), self._view(pb, n)
        c = self.cols[self.r]
        lab, hba = self.la[b][:, c], self.hb[a][:, c]
        hit = (lab > 0) & (lab <= hba)
        self._view(pout, n)[:] = (hit * self.w[c]).sum(axis=1).astype(np.int32)

    def fc_combine_dev(self, n, psum, pout):
        s = self._view(psum, n).astype(np.int64)
        out = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(pout))
        out[:] = (s >= self.quorum).astype(np.uint8)

    def sync(self):
        pass


def _case(seed, V=13, N=200, Q=500):
    rng = np.random.default_rng(seed)
    la = rng.integers(0, 6, (N, V)).astype(np.int32)
    hb = rng.integers(0, 6, (N, V)).astype(np.int32)
    owner = rng.integers(0, V, N)
    weights = rng.integers(1, 9, V)
    qa = rng.integers(0, N, Q).astype(np.int32)
    qb = rng.integers(0, N, Q).astype(np.int32)
    return la, hb, owner, weights, qa, qb


def _expected(la, hb, weights, qa, qb):
    lab, hba = la[qb], hb[qa]
    s = (((lab > 0) & (lab <= hba)) * np.asarray(weights)).sum(axis=1)
    return (s >= int(np.sum(weights)) * 2 // 3 + 1).astype(np.uint8)


def _worker(rank, world, port, seed, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lachesis-base_amd"))
        from lachesis_hip.shard import ShardedIndex
        la, hb, owner, weights, qa, qb = _case(seed)
        fake = FakeShard(rank, world, la, hb, owner, weights)
        si = ShardedIndex(fake, device=torch.device("cpu"))
        sent = si.exchange()
        c = fake.cols[rank]
        ok_la = bool(np.array_equal(fake.la[:, c], la[:, c]))
        out = si.forkless_cause_dev(torch.from_numpy(qa), torch.from_numpy(qb)).numpy()
        ok_fc = bool(np.array_equal(out, _expected(la, hb, weights, qa, qb)))
        q.put((rank, ok_la, ok_fc, sum(sent)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_shard_protocol_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 7 + world, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok_la and ok_fc for _, ok_la, ok_fc, _ in res), res
    assert sum(s for *_, s in res) > 0


def test_single_rank_no_collective():
    """world 1: exchange sends nothing, FC equals the unsharded rule."""
    la, hb, owner, weights, qa, qb = _case(3)
    if not dist.is_initialized():
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        from lachesis_hip.shard import ShardedIndex
        fake = FakeShard(0, 1, la, hb, owner, weights)
        si = ShardedIndex(fake, device=torch.device("cpu"))
        assert sum(si.exchange()) == 0
        out = si.forkless_cause_dev(torch.from_numpy(qa), torch.from_numpy(qb)).numpy()
        np.testing.assert_array_equal(out, _expected(la, hb, weights, qa, qb))
    finally:
        dist.destroy_process_group()

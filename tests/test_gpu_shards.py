"""Column-sharded index on one GPU: G handles, each
owning a creator range, exchange LowestAfter blocks (what the all-to-all does
between GPUs), compute ForklessCause partial stake sums, add them (what the
all-reduce does) and combine.  Must equal the unsharded index and the oracle."""

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


def exchange(shards):
    """What ShardedIndex.exchange's all-to-all does between GPUs."""
    import torch
    dev = torch.device("cuda", 0)
    G = len(shards)
    wb = shards[0].shard_wire_bytes()
    assert all(ix.shard_wire_bytes() == wb for ix in shards)   # every shard picks the same width
    widths = {}
    for s in range(G):
        for t in range(G):
            if s == t:
                continue
            n = shards[s].shard_block(s, t)
            assert n == shards[t].shard_block(s, t)
            w = shards[s].shard_block_wire(t)          # the sender picks, the receiver is told
            assert w in (1, wb)
            widths[(s, t)] = w
            # torch fills on its own stream and the library runs on its own:
            # no fill kernel may still be in flight when the pack writes
            buf = torch.empty(max(n * w, 1), dtype=torch.uint8, device=dev)
            shards[s].la_pack_wire_dev(t, buf.data_ptr(), w)
            shards[t].la_unpack_wire_dev(s, buf.data_ptr(), w)
    for ix in shards:
        ix.la_own_dev()
    return widths


def fc(lx, shards, qa, qb):
    """Partial stake sums per shard, added (the all-reduce), combined."""
    import torch
    dev = torch.device("cuda", 0)
    a = torch.from_numpy(qa.view(np.int32)).to(dev)
    b = torch.from_numpy(qb.view(np.int32)).to(dev)
    total = torch.zeros(len(qa), dtype=torch.int64, device=dev)
    for ix in shards:
        part = torch.empty(len(qa), dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)      # inputs and `total` ready before the library stream runs
        ix.forkless_cause_partial_dev(len(qa), a.data_ptr(), b.data_ptr(), part.data_ptr())
        ix.sync()
        total += part.to(torch.int64) & 0xFFFFFFFF
    s32 = (total & 0xFFFFFFFF).to(torch.int64)
    s32 = torch.where(s32 >= 2 ** 31, s32 - 2 ** 32, s32).to(torch.int32)
    out = torch.empty(len(qa), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)          # s32 is computed on torch's stream
    shards[0].fc_combine_dev(len(qa), s32.data_ptr(), out.data_ptr())
    shards[0].sync()
    return out.cpu().numpy()


def sharded_fc(lx, d, weights, G, qa, qb, options=None):
    shards = []
    for r in range(G):
        ix = lx.Index(shard_rank=r, shard_count=G, options=options)
        ix.reset(weights)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        shards.append(ix)
    exchange.last = exchange(shards)
    return fc(lx, shards, qa, qb), shards


@pytest.mark.parametrize("G", [2, 3, 4])
@pytest.mark.parametrize("shape", [(16, 40, 5, 0, 0, 1), (24, 30, 6, 5, 6, 2)])
def test_sharded_fc_matches_oracle(G, shape):
    import lachesis_hip as lx
    n, ev, p, ch, fk, seed = shape
    d = lx.tools.gen_dag(n, ev, p, ch, fk, seed)
    rng = np.random.default_rng(seed)
    weights = sorted((int(x) for x in rng.integers(1, 20, n)), reverse=True)
    o = corc.OracleIndex(weights)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    qa, qb = lx.tools.fc_queries(d.lamport, 50_000, window=24, seed=seed)
    got, shards = sharded_fc(lx, d, weights, G, qa, qb)
    np.testing.assert_array_equal(got, o.forkless_cause_batch(qa, qb))
    # the shard ranges partition the creators
    ranges = [shards[0].shard_range(r) for r in range(G)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    assert all(ranges[i][1] == ranges[i + 1][0] for i in range(G - 1))


@pytest.mark.parametrize("cpw", [8, 12])
def test_sharded_wide_slices_fall_back(cpw):
    """Option cpw 8 / 12 on column shards (their column lists are not the
    identity: 12-column slices walk as 8) on a fork-free DAG whose seqs fit
    16 bits: ForklessCause equals the oracle."""
    import lachesis_hip as lx
    d = lx.tools.gen_dag(40, 60, 6, 0, 0, 3)
    weights = [1 + (i % 5) for i in range(40)]
    o = corc.OracleIndex(weights)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    qa, qb = lx.tools.fc_queries(d.lamport, 50_000, window=24, seed=3)
    got, _ = sharded_fc(lx, d, weights, 3, qa, qb, options={"cpw": cpw, "small_max": 0, "dbl": 0})
    np.testing.assert_array_equal(got, o.forkless_cause_batch(qa, qb))


@pytest.mark.parametrize("force", [None, "4"])
def test_sharded_wire_width(force, monkeypatch):
    """LowestAfter blocks travel as uint16 while every seq < 2^16, else (or
    with option shard_wire=4) as uint32; FC equals the oracle either way."""
    import lachesis_hip as lx
    if force:
        monkeypatch.setitem(lx.capi.DEFAULT_OPTIONS, "shard_wire", int(force))
    d = lx.tools.gen_dag(12, 30, 4, 3, 4, 9)
    weights = [3, 3, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1]
    o = corc.OracleIndex(weights)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    qa, qb = lx.tools.fc_queries(d.lamport, 20_000, window=24, seed=9)
    got, shards = sharded_fc(lx, d, weights, 3, qa, qb)
    assert shards[0].shard_wire_bytes() == (4 if force else 2)
    if force:
        assert set(exchange.last.values()) == {4}
    np.testing.assert_array_equal(got, o.forkless_cause_batch(qa, qb))


def test_sharded_wire_long_branches():
    """Seqs past 2^16 switch the wire to uint32 (bit-exact FC vs the oracle)."""
    import lachesis_hip as lx
    d = lx.tools.gen_dag(3, 66_000, 3, 0, 0, 4)
    assert int(d.seq.max()) > 0xFFFF
    weights = [1, 1, 1]
    o = corc.OracleIndex(weights)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    qa, qb = lx.tools.fc_queries(d.lamport, 50_000, window=8, seed=4)
    got, shards = sharded_fc(lx, d, weights, 2, qa, qb)
    assert shards[0].shard_wire_bytes() == 4
    np.testing.assert_array_equal(got, o.forkless_cause_batch(qa, qb))


def test_sharded_byte_wire():
    """Balanced DAG: every LowestAfter entry is within 127 of its row's seq, so
    every block travels as one byte per entry; FC equals the oracle."""
    import lachesis_hip as lx
    d = lx.tools.gen_dag(16, 300, 5, 0, 0, 71)
    w = [2] * 16
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    qa, qb = lx.tools.fc_queries(d.lamport, 50_000, window=24, seed=71)
    got, shards = sharded_fc(lx, d, w, 4, qa, qb)
    assert set(exchange.last.values()) == {1}
    np.testing.assert_array_equal(got, o.forkless_cause_batch(qa, qb))


def test_sharded_byte_wire_fallback_on_skewed_progress():
    """Validator 0 runs 300 events alone, then validators 1..7 join with their
    first event on top of it, and 0's next event observes them: LowestAfter
    entries lie far from their rows' seqs in both directions, so both blocks
    fall back to the wider wire; all-pairs FC equals the oracle."""
    import types
    import lachesis_hip as lx
    n0 = 300
    creator = [0] * n0 + list(range(1, 8)) + [0]
    seq = list(range(1, n0 + 1)) + [1] * 7 + [n0 + 1]
    pars = [[]] + [[i - 1] for i in range(1, n0)] + [[n0 - 1]] * 7 + [[n0 - 1] + list(range(n0, n0 + 7))]
    poff = np.cumsum([0] + [len(p) for p in pars]).astype(np.uint32)
    d = types.SimpleNamespace(creator=np.array(creator, dtype=np.uint32), seq=np.array(seq, dtype=np.uint32),
                              poff=poff, par=np.array([x for p in pars for x in p], dtype=np.uint32))
    w = [1] * 8
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    N = len(creator)
    qa = np.repeat(np.arange(N, dtype=np.uint32), N)
    qb = np.tile(np.arange(N, dtype=np.uint32), N)
    got, shards = sharded_fc(lx, d, w, 2, qa, qb)
    import torch
    buf = torch.empty(shards[0].shard_block(0, 1), dtype=torch.uint8, device=torch.device("cuda", 0))
    with pytest.raises(lx.LxError) as ei:
        shards[0].la_pack_wire_dev(1, buf.data_ptr(), 1)   # the pack itself reports the misfit
    assert ei.value.code == -7
    # (0 -> 1): LA(0, s)[j >= 4] = 1 for s up to 300; (1 -> 0): LA(k, 1)[0] = 301
    assert exchange.last == {(0, 1): 2, (1, 0): 2}
    np.testing.assert_array_equal(got, o.forkless_cause_batch(qa, qb))
    assert got.sum() > 0


def test_shard_planes_hold_own_columns():
    """Memory per GPU ~ 1/G: a shard's plane rows are its own columns only."""
    import lachesis_hip as lx
    d = lx.tools.gen_dag(64, 10, 5, 0, 0, 3)
    w = [1] * 64
    full = lx.Index()
    full.reset(w)
    full.add_batch(d.creator, d.seq, d.poff, d.par)
    stride = full.device_planes()[2]
    for G in (2, 4):
        for r in range(G):
            ix = lx.Index(shard_rank=r, shard_count=G)
            ix.reset(w)
            ix.add_batch(d.creator, d.seq, d.poff, d.par)
            lo, hi = ix.shard_range(r)
            p = ix.device_planes()[2]
            assert hi - lo <= p < stride // G + 32, (G, r, p, stride)
            with pytest.raises(lx.LxError):
                ix.highest_before(0)          # shards hold partial rows


@pytest.mark.parametrize("G", [2, 3])
def test_sharded_drop_and_reexchange(G):
    """DropNotFlushed on every shard (incl. fork branches created after the
    flush), exchange again, FC equals the oracle of the flushed prefix; then
    re-add and compare with the full oracle."""
    import lachesis_hip as lx
    d = lx.tools.gen_dag(20, 30, 5, 4, 6, 5)
    rng = np.random.default_rng(5)
    weights = sorted((int(x) for x in rng.integers(1, 30, 20)), reverse=True)
    cut = 80                   # 26 branches here, 37 at the end: forks after the flush
    shards = []
    for r in range(G):
        ix = lx.Index(shard_rank=r, shard_count=G)
        ix.reset(weights)
        ix.add_batch(d.creator[:cut], d.seq[:cut], d.poff[:cut + 1], d.par)
        ix.flush()
        ix.add_batch(d.creator[cut:], d.seq[cut:], d.poff[cut:] , d.par)
        shards.append(ix)
    assert shards[0].num_branches() == 37
    o = corc.OracleIndex(weights)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    qa, qb = lx.tools.fc_queries(d.lamport, 20_000, window=30, seed=1)
    exchange(shards)
    np.testing.assert_array_equal(fc(lx, shards, qa, qb), o.forkless_cause_batch(qa, qb))
    for ix in shards:
        ix.drop_not_flushed()
        assert ix.num_branches() == 26
    o1 = corc.OracleIndex(weights)
    assert o1.add_batch(d.creator[:cut], d.seq[:cut], d.poff[:cut + 1], d.par) == -1
    qa1, qb1 = lx.tools.fc_queries(d.lamport[:cut], 20_000, window=30, seed=2)
    exchange(shards)
    np.testing.assert_array_equal(fc(lx, shards, qa1, qb1), o1.forkless_cause_batch(qa1, qb1))
    for ix in shards:
        ix.add_batch(d.creator[cut:], d.seq[cut:], d.poff[cut:], d.par)
    exchange(shards)
    np.testing.assert_array_equal(fc(lx, shards, qa, qb), o.forkless_cause_batch(qa, qb))


@pytest.mark.parametrize("G", [5, 7, 8])
def test_sharded_config3_shape_zipf_cheaters(G):
    """BASELINE configs[2]'s split (V = 1000, Zipf stakes floor(2^20/(i+1)),
    P = 10) at G = 8 and the uneven G = 5 / 7, with 20 double-signers: the
    column shards' ForklessCause equals the oracle's; the shard ranges
    partition the creators (multiples of 4)."""
    import lachesis_hip as lx
    V = 1000
    w = [(1 << 20) // (i + 1) for i in range(V)]
    d = lx.tools.gen_dag(V, 5, 10, cheaters=20, forks=3, seed=G)
    o = corc.OracleIndex(w)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    assert o.num_branches() > V
    qa, qb = lx.tools.fc_queries(d.lamport, 100_000, window=24, seed=G)
    got, shards = sharded_fc(lx, d, w, G, qa, qb)
    np.testing.assert_array_equal(got, o.forkless_cause_batch(qa, qb))
    ranges = [shards[0].shard_range(r) for r in range(G)]
    assert ranges[0][0] == 0 and ranges[-1][1] == V
    assert all(ranges[i][1] == ranges[i + 1][0] and ranges[i][1] % 4 == 0 for i in range(G - 1))
    for ix in shards:
        ix.close()

"""The native row-segment exchange (lx_rowseg_exchange: the driver of
csrc/lx_rowseg_exchange.h, which the Go shim runs over RCCL) with G ranks in
one process on one GPU: tests/csrc/rowseg_fake.cpp runs the same driver, one
thread per rank, over an in-process transport (RCCL refuses two ranks on one
device).  Every rank's own HighestBefore / LowestAfter rows must equal an
ordinary single index's rows byte for byte, its ForklessCause answers between
own events must equal the C oracle's, and the exchange statistics must equal
those of the torch.distributed protocol (lachesis_hip/rowseg.py) on the same
epoch, which tests/test_gpu_rowseg.py checks the same way."""

import ctypes
import os

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SHAPES = {
    "forks": (28, 60, 6, 5, 6, 3),       # fork branches, cheaters' marks
    "parents": (20, 80, 16, 0, 0, 4),    # parents beyond the inline twelve
    "short": (200, 6, 3, 0, 0, 5),       # segments shorter than a level: several row rounds
    "wide": (300, 40, 10, 0, 0, 6),
}


@pytest.fixture(scope="module")
def lx():
    import lachesis_hip
    return lachesis_hip


@pytest.fixture(scope="module")
def fake(lx):
    lx.load_library()
    L = ctypes.CDLL(os.path.join(ROOT, "lachesis-base_amd", "build", "librowseg_fake.so"))
    L.lx_fake_rowseg_exchange.restype = ctypes.c_int
    L.lx_fake_rowseg_exchange.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.c_char_p, ctypes.c_uint32]
    vpp = ctypes.POINTER(ctypes.c_void_p)
    L.lx_fake_rowseg_fc.restype = ctypes.c_int
    L.lx_fake_rowseg_fc.argtypes = [vpp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), vpp, vpp, vpp,
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.c_char_p, ctypes.c_uint32]
    L.lx_fake_rowseg_get_rows.restype = ctypes.c_int
    L.lx_fake_rowseg_get_rows.argtypes = [vpp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), vpp,
                                          vpp, ctypes.c_uint64, vpp, ctypes.c_char_p, ctypes.c_uint32]
    return L


def _planes(ix, lo, hi):
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    ix.sync()
    hb, la, stride, _ = ix.device_planes()
    out = []
    for p in (hb, la):
        a = np.empty((hi - lo, stride), dtype=np.uint32)
        assert hip.hipMemcpy(a.ctypes.data, p + 4 * lo * stride, a.nbytes, 2) == 0
        out.append(a)
    return out


@pytest.mark.parametrize("world,shape,sub", [(2, "forks", 0), (3, "forks", 0), (4, "parents", 0), (4, "short", 0),
                                             (3, "wide", 0), (8, "wide", 0),
                                             (2, "forks", 2), (3, "wide", 3), (4, "parents", 2), (2, "wide", 5)])
def test_native_row_segment_exchange(lx, fake, world, shape, sub):
    """sub > 1: every rank walks its own segment as `sub` side-by-side
    sub-segments (option seg_sub; auto picks it for large epochs), fixed up in
    order after the rows of the other ranks arrive."""
    V, epv, P, ch, fk, seed = SHAPES[shape]
    d = lx.tools.gen_dag(V, epv, P, ch, fk, seed)
    rng = np.random.default_rng(seed)
    weights = [int(x) for x in rng.integers(1, 40, V)]
    ranks = []
    for r in range(world):
        ix = lx.Index(device=0, options={"seg_count": world, "seg_rank": r, "small_max": 0, "seg_sub": sub})
        ix.reset(weights)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        ranks.append(ix)
    hs = (ctypes.c_void_p * world)(*[ix.h for ix in ranks])
    stats = (ctypes.c_uint64 * (4 * world))()
    err = ctypes.create_string_buffer(512)
    rc = fake.lx_fake_rowseg_exchange(hs, world, stats, err, 512)
    assert rc == 0, err.value.decode()
    ref = lx.Index(device=0, options={"small_max": 0})
    ref.reset(weights)
    ref.add_batch(d.creator, d.seq, d.poff, d.par)
    B = ref.num_branches()
    o = corc.OracleIndex(weights)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    for r, ix in enumerate(ranks):
        lo, hi = ix.rowseg_range()
        mine, theirs = _planes(ix, lo, hi), _planes(ref, lo, hi)
        assert np.array_equal(mine[0][:, :B], theirs[0][:, :B]), ("hb", r)
        assert np.array_equal(mine[1][:, :B], theirs[1][:, :B]), ("la", r)
        n = hi - lo
        qa = (lo + rng.integers(0, n, 20_000)).astype(np.uint32)
        qb = np.clip(qa.astype(np.int64) - rng.integers(0, 300, 20_000), lo, hi - 1).astype(np.uint32)
        np.testing.assert_array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb))
    st = np.array(stats[:], dtype=np.uint64).reshape(world, 4)
    assert st[:, 2].sum() == st[:, 3].sum()               # every LowestAfter triple sent was received
    if shape == "short":
        assert st[:, 0].max() >= 2, st                    # not-ready rows asked again
    for ix in ranks:
        ix.close()
    ref.close()


@pytest.mark.parametrize("world,shape,sub", [(2, "forks", 0), (3, "forks", 0), (4, "parents", 0), (8, "wide", 0),
                                             (3, "wide", 2)])
def test_native_row_segment_forkless_cause_any_pair(lx, fake, world, shape, sub):
    """ForklessCause of ANY pair of the epoch across row-segment ranks
    (lx_rowseg_forkless_cause's driver, csrc/lx_rowseg_exchange.h
    rowseg_fc_run, over the in-process transport): every rank asks queries
    with a uniform over the whole epoch and b up to 300 events before it --
    most pairs leave the asking rank, many cross a segment boundary -- and
    gets the C oracle's answers in its own order (vecfc/forkless_cause.go:40-82)."""
    import torch
    V, epv, P, ch, fk, seed = SHAPES[shape]
    d = lx.tools.gen_dag(V, epv, P, ch, fk, seed)
    N = len(d)
    rng = np.random.default_rng(seed + 100)
    weights = [int(x) for x in rng.integers(1, 40, V)]
    ranks = []
    for r in range(world):
        ix = lx.Index(device=0, options={"seg_count": world, "seg_rank": r, "small_max": 0, "seg_sub": sub})
        ix.reset(weights)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        ranks.append(ix)
    hs = (ctypes.c_void_p * world)(*[ix.h for ix in ranks])
    stats = (ctypes.c_uint64 * (4 * world))()
    err = ctypes.create_string_buffer(512)
    assert fake.lx_fake_rowseg_exchange(hs, world, stats, err, 512) == 0, err.value.decode()
    o = corc.OracleIndex(weights)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    dev = torch.device("cuda", 0)
    qs, bufs = [], []
    for r in range(world):
        k = 30_000 + 1000 * r                          # ranks ask different numbers of queries
        qa = rng.integers(0, N, k).astype(np.uint32)
        qb = np.clip(qa.astype(np.int64) - rng.integers(0, 300, k), 0, N - 1).astype(np.uint32)
        qs.append((qa, qb))
        t = lambda x: torch.from_numpy(x.view(np.int32)).to(dev)
        bufs.append((t(qa), t(qb), torch.full((k,), 7, dtype=torch.uint8, device=dev)))
    torch.cuda.synchronize()
    ns = (ctypes.c_uint64 * world)(*[len(q[0]) for q in qs])
    P_ = lambda i: (ctypes.c_void_p * world)(*[b[i].data_ptr() for b in bufs])
    fst = (ctypes.c_uint64 * (4 * world))()
    for rep in range(2):                               # a second batch re-asks (and re-ships) its rows
        rc = fake.lx_fake_rowseg_fc(hs, world, ns, P_(0), P_(1), P_(2), fst, err, 512)
        assert rc == 0, err.value.decode()
        for r in range(world):
            qa, qb = qs[r]
            np.testing.assert_array_equal(bufs[r][2].cpu().numpy(), o.forkless_cause_batch(qa, qb), err_msg=str(r))
    st = np.array(fst[:], dtype=np.uint64).reshape(world, 4)
    assert st[:, 0].sum() > 0 and st[:, 2].sum() > 0, st      # pairs left their rank, rows crossed
    assert st[:, 1].sum() == sum(len(q[0]) for q in qs)        # every query answered exactly once
    assert st[:, 2].sum() == st[:, 3].sum()                    # every LA row sent was received
    for ix in ranks:
        ix.close()


def test_rowseg_comm_one_rank_and_mismatch(lx):
    """lx_rowseg_comm_create over real RCCL with one rank (the 1-GPU box): a
    whole index has nothing to join; a handle whose seg_rank / seg_count do not
    match the communicator's rank is refused before RCCL is touched."""
    d = lx.tools.gen_dag(10, 20, 4, 0, 0, 9)
    ix = lx.Index(device=0)
    ix.reset([1] * 10)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    assert ix.rowseg_of() == (0, 1)
    c = lx.RowsegComm(ix, lx.shard_comm_unique_id(), 1, 0)
    assert c.exchange() == {"row_rounds": 0, "rows_received": 0, "la_sent": 0, "la_received": 0}
    # one rank: lx_rowseg_forkless_cause is the whole index's batch call
    import torch
    N = len(d)
    qa, qb = lx.tools.fc_queries(d.lamport, 5000, seed=3)
    dev = torch.device("cuda", 0)
    ta = torch.from_numpy(qa.view(np.int32)).to(dev)
    tb = torch.from_numpy(qb.view(np.int32)).to(dev)
    out = torch.empty(len(qa), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    c.forkless_cause_dev(len(qa), ta.data_ptr(), tb.data_ptr(), out.data_ptr())
    np.testing.assert_array_equal(out.cpu().numpy(), ix.forkless_cause_batch(qa, qb))
    assert N > 0
    c.close()
    seg = lx.Index(device=0, options={"seg_count": 2, "seg_rank": 1, "small_max": 0})
    assert seg.rowseg_of() == (1, 2)
    with pytest.raises(lx.LxError, match="row segment 1 of 2"):
        lx.RowsegComm(seg, bytes(128), 1, 0)
    with pytest.raises(lx.LxError):
        lx.ShardComm(seg, bytes(128), 2, 1)   # not a column-shard handle
    seg.close()
    ix.close()


def _planes_equal(ix, ref, lo, hi, B, chunk=50_000):
    for r0 in range(lo, hi, chunk):
        r1 = min(hi, r0 + chunk)
        mine, theirs = _planes(ix, r0, r1), _planes(ref, r0, r1)
        for k in range(2):
            if not np.array_equal(mine[k][:, :B], theirs[k][:, :B]):
                bad = np.argwhere(mine[k][:, :B] != theirs[k][:, :B])[:5]
                return ("hb", "la")[k], r0, bad.tolist()
    return None


@pytest.mark.parametrize("world", [2, 4])
def test_native_row_segments_c3_shape_auto_sub(lx, fake, world):
    """The multi-GPU default at the headline shape (V = 1000, Zipf stakes, 10
    parents; 1M events here): every rank walks its segment as the side-by-side
    sub-segments it picks on its own (seg_sub auto, 12-column slices, one
    launch), and every own HB / LA row equals the single walk's byte for byte;
    ForklessCause of pairs across the rank boundaries equals the whole index's."""
    import torch
    V = 1000
    d = lx.tools.gen_dag(V, 1000, 10, seed=1)
    N = len(d)
    w = [(1 << 20) // (i + 1) for i in range(V)]
    ranks = []
    for r in range(world):
        ix = lx.Index(device=0, event_capacity=N, options={"seg_count": world, "seg_rank": r, "small_max": 0})
        ix.reset(w)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        st = ix.segment_stats()
        assert st["one_launch"], st            # sub-segments side by side in one launch
        ranks.append(ix)
    hs = (ctypes.c_void_p * world)(*[ix.h for ix in ranks])
    stats = (ctypes.c_uint64 * (4 * world))()
    err = ctypes.create_string_buffer(512)
    assert fake.lx_fake_rowseg_exchange(hs, world, stats, err, 512) == 0, err.value.decode()
    ref = lx.Index(device=0, event_capacity=N, options={"small_max": 0, "seg_auto": 0})
    ref.reset(w)
    ref.add_batch(d.creator, d.seq, d.poff, d.par)
    B = ref.num_branches()
    for r, ix in enumerate(ranks):
        lo, hi = ix.rowseg_range()
        assert _planes_equal(ix, ref, lo, hi, B) is None, r
    # pairs that cross every rank boundary: a just after it, b up to 3000 before
    rng = np.random.default_rng(5)
    dev = torch.device("cuda", 0)
    bounds = [ix.rowseg_range()[0] for ix in ranks[1:]]
    qs, bufs = [], []
    for r in range(world):
        k = 40_000
        at = np.array(bounds, dtype=np.int64)[rng.integers(0, len(bounds), k)]
        qa = (at + rng.integers(0, 20_000, k)).astype(np.uint32)
        qb = np.clip(qa.astype(np.int64) - rng.integers(1, 23_000, k), 0, N - 1).astype(np.uint32)
        qs.append((qa, qb))
        t = lambda x: torch.from_numpy(x.view(np.int32)).to(dev)
        bufs.append((t(qa), t(qb), torch.full((k,), 7, dtype=torch.uint8, device=dev)))
    torch.cuda.synchronize()
    ns = (ctypes.c_uint64 * world)(*[len(q[0]) for q in qs])
    P_ = lambda i: (ctypes.c_void_p * world)(*[b[i].data_ptr() for b in bufs])
    fst = (ctypes.c_uint64 * (4 * world))()
    assert fake.lx_fake_rowseg_fc(hs, world, ns, P_(0), P_(1), P_(2), fst, err, 512) == 0, err.value.decode()
    crossing = 0
    for r in range(world):
        qa, qb = qs[r]
        np.testing.assert_array_equal(bufs[r][2].cpu().numpy(), ref.forkless_cause_batch(qa, qb), err_msg=str(r))
        crossing += int(sum(((qb < b) & (qa >= b)).sum() for b in bounds))
    assert crossing > 10_000, crossing
    for ix in ranks:
        ix.close()
    ref.close()


@pytest.mark.parametrize("world,shape", [(2, "forks"), (3, "forks"), (4, "wide")])
def test_native_row_segment_getters_any_rank(lx, fake, world, shape):
    """The vector getters of events on every rank through the native driver
    (csrc/lx_rowseg_exchange.h rowseg_get_run, which lx_rowseg_get_rows runs
    over RCCL): each rank asks for rows of events anywhere in the epoch (and
    one past it), in every mode, and gets the oracle's bytes in its own order
    (vecfc/store_vectors.go:26-51, vecengine/index.go:235-250)."""
    import torch
    V, epv, P, ch, fk, seed = SHAPES[shape]
    d = lx.tools.gen_dag(V, epv, P, ch, fk, seed)
    N = len(d)
    rng = np.random.default_rng(seed + 7)
    weights = [int(x) for x in rng.integers(1, 40, V)]
    ranks = []
    for r in range(world):
        ix = lx.Index(device=0, options={"seg_count": world, "seg_rank": r, "small_max": 0})
        ix.reset(weights)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        ranks.append(ix)
    hs = (ctypes.c_void_p * world)(*[ix.h for ix in ranks])
    stats = (ctypes.c_uint64 * (4 * world))()
    err = ctypes.create_string_buffer(512)
    assert fake.lx_fake_rowseg_exchange(hs, world, stats, err, 512) == 0, err.value.decode()
    o = corc.OracleIndex(weights)
    assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
    dev = torch.device("cuda", 0)
    slot = (ranks[0].row_bytes_max() + 15) // 16 * 16
    evs = [np.concatenate([rng.integers(0, N, 200 + 13 * r), [N + 3]]).astype(np.uint32) for r in range(world)]
    n = (ctypes.c_uint64 * world)(*[len(e) for e in evs])
    t_ev = [torch.from_numpy(e.view(np.int32)).to(dev) for e in evs]
    for mode, want in ((0, o.hb), (1, o.la), (2, o.merged_hb)):
        t_out = [torch.zeros(len(e) * slot, dtype=torch.uint8, device=dev) for e in evs]
        t_len = [torch.zeros(len(e), dtype=torch.int32, device=dev) for e in evs]
        pv = lambda ts: (ctypes.c_void_p * world)(*[t.data_ptr() for t in ts])
        rc = fake.lx_fake_rowseg_get_rows(hs, world, mode, n, pv(t_ev), pv(t_out), slot, pv(t_len), err, 512)
        assert rc == 0, err.value.decode()
        for r in range(world):
            rows = t_out[r].cpu().numpy().reshape(len(evs[r]), slot)
            lens = t_len[r].cpu().numpy().view(np.uint32)
            for i, e in enumerate(evs[r]):
                if e >= N:
                    assert lens[i] == 0xFFFFFFFF
                else:
                    assert bytes(rows[i, :lens[i]]) == want(int(e)), (mode, r, int(e))
    for ix in ranks:
        ix.close()


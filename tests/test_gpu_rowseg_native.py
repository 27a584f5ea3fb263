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


@pytest.mark.parametrize("world,shape", [(2, "forks"), (3, "forks"), (4, "parents"), (4, "short"), (3, "wide"),
                                         (8, "wide")])
def test_native_row_segment_exchange(lx, fake, world, shape):
    V, epv, P, ch, fk, seed = SHAPES[shape]
    d = lx.tools.gen_dag(V, epv, P, ch, fk, seed)
    rng = np.random.default_rng(seed)
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
    with pytest.raises(lx.LxError):
        c.forkless_cause_dev(0, 0, 0, 0)
    c.close()
    seg = lx.Index(device=0, options={"seg_count": 2, "seg_rank": 1, "small_max": 0})
    assert seg.rowseg_of() == (1, 2)
    with pytest.raises(lx.LxError, match="row segment 1 of 2"):
        lx.RowsegComm(seg, bytes(128), 1, 0)
    with pytest.raises(lx.LxError):
        lx.ShardComm(seg, bytes(128), 2, 1)   # not a column-shard handle
    seg.close()
    ix.close()

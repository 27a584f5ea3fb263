"""Row segments end to end through torch.distributed (lachesis_hip.rowseg):
G processes (gloo, all on cuda:0 -- the driver's N-GPU runs use RCCL, one GPU
per rank) each add the same epoch with options seg_count = G, seg_rank = r,
walk only their own Add-order segment and run RowSegments.exchange (row
requests in rounds, LowestAfter triples to their owners).  Every rank's own
HighestBefore / LowestAfter rows must equal an ordinary single index's rows,
byte for byte (that index is pinned to the oracle by the parity tests), and
its ForklessCause answers between own events must equal the C oracle's, and
so must ForklessCause of any pair and the vector getters of events on any
rank, routed to their owners.  A rank's planes hold only its own rows."""

import ctypes
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SHAPES = {
    "forks": (28, 60, 6, 5, 6, 3),       # fork branches, cheaters' marks
    "parents": (20, 80, 16, 0, 0, 4),    # parents beyond the inline twelve
    "short": (200, 6, 3, 0, 0, 5),       # segments shorter than a level: several row rounds
    "wide": (300, 40, 10, 0, 0, 6),
}


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


def _worker(rank, world, port, q, shape, sub=0):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lachesis_hip as lx
        from lachesis_hip.rowseg import RowSegments
        from oracle import corc
        V, epv, P, ch, fk, seed = SHAPES[shape]
        d = lx.tools.gen_dag(V, epv, P, ch, fk, seed)
        rng = np.random.default_rng(seed)
        weights = [int(x) for x in rng.integers(1, 40, V)]
        ix = lx.Index(device=0, options={"seg_count": world, "seg_rank": rank, "small_max": 0, "seg_sub": sub})
        ix.reset(weights)
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        dev = torch.device("cuda", 0)
        rs = RowSegments(ix, device=dev)
        info = rs.exchange()
        lo, hi = ix.rowseg_range()
        assert ix.rowseg_bounds(world)[rank] == lo
        ref = lx.Index(device=0, options={"small_max": 0})
        ref.reset(weights)
        ref.add_batch(d.creator, d.seq, d.poff, d.par)
        B = ref.num_branches()
        mine, theirs = _planes(ix, lo, hi), _planes(ref, lo, hi)
        ok = bool(np.array_equal(mine[0][:, :B], theirs[0][:, :B]) and np.array_equal(mine[1][:, :B], theirs[1][:, :B]))
        n = hi - lo
        qa = (lo + rng.integers(0, n, 40_000)).astype(np.uint32)
        qb = np.clip(qa.astype(np.int64) - rng.integers(0, 300, 40_000), lo, hi - 1).astype(np.uint32)
        o = corc.OracleIndex(weights)
        assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
        ok = ok and bool(np.array_equal(ix.forkless_cause_batch(qa, qb), o.forkless_cause_batch(qa, qb)))
        # a query outside the own rows is refused, not answered
        try:
            ix.forkless_cause_batch(np.array([lo - 1 if lo else hi], dtype=np.uint32), np.array([lo], dtype=np.uint32))
            ok = False
        except Exception:
            pass
        # ForklessCause of ANY pair across ranks (RowSegments.forkless_cause_dev):
        # a uniform over the epoch, b up to 300 events before it
        N = len(d)
        k = 20_000 + 500 * rank
        qa2 = rng.integers(0, N, k).astype(np.uint32)
        qb2 = np.clip(qa2.astype(np.int64) - rng.integers(0, 300, k), 0, N - 1).astype(np.uint32)
        ta = torch.from_numpy(qa2.view(np.int32)).to(dev)
        tb = torch.from_numpy(qb2.view(np.int32)).to(dev)
        out = torch.full((k,), 7, dtype=torch.uint8, device=dev)
        fc = rs.forkless_cause_dev(k, ta, tb, out)
        ok = ok and bool(np.array_equal(out.cpu().numpy(), o.forkless_cause_batch(qa2, qb2)))
        info = dict(info, fc=fc)
        # the vector getters of events on EVERY rank (RowSegments.get_rows:
        # ids to their owners, encoded rows back) and of own events directly
        ev = [int(x) for x in rng.integers(0, N, 150)] + [0, N - 1]
        for mode, want in ((0, o.hb), (1, o.la), (2, o.merged_hb)):
            rows = rs.get_rows(mode, ev)
            ok = ok and all(r == want(e) for r, e in zip(rows, ev))
        ok = ok and rs.get_rows(0, [N + 5])[0] is None
        own = [int(x) for x in rng.integers(lo, hi, 20)]
        ok = ok and all(ix.highest_before(e) == o.hb(e) and ix.lowest_after(e) == o.la(e) and
                        ix.merged_highest_before(e) == o.merged_hb(e) for e in own)
        try:
            ix.highest_before(lo - 1 if lo else hi)      # another rank's row: routed, not answered here
            ok = False
        except Exception:
            pass
        # the planes hold the own rows only
        mem = ix.device_bytes()
        info = dict(info, planes=mem["planes"], plane_rows=(hi - lo), stride=ix.device_planes()[2])
        ok = ok and mem["planes"] == 2 * 4 * (hi - lo) * ix.device_planes()[2]
        q.put((rank, ok, info))
    except Exception as e:   # report instead of hanging the other ranks' queue reads
        q.put((rank, False, repr(e)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,shape,sub", [(2, "forks", 0), (3, "forks", 0), (4, "parents", 0), (4, "short", 0),
                                             (3, "wide", 0), (2, "forks", 3)])
def test_row_segments_over_torch_distributed(world, shape, sub):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, shape, sub)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    assert sum(r[2]["fc"]["rows_received"] for r in res) > 0, res     # LA rows crossed ranks
    if shape == "short":
        assert max(r[2]["row_rounds"] for r in res) >= 2, res    # not-ready rows asked again

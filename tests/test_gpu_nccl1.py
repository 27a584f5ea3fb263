"""The device-tensor collective paths of the multi-GPU wrappers, run once on
the 1-GPU box: a world_size-1 process group over RCCL (backend "nccl"), so
RowSegments' and ShardedIndex's non-staged branches (device tensors straight
into all_to_all_single / all_reduce) execute exactly as on the driver's 8-GPU
node, and the library's own RCCL transports with one rank:

* RowSegments on a one-rank row-segment handle (seg_count = 1: the whole
  epoch is the rank's segment; every exchange, route and getter route runs
  with nothing to move): planes, ForklessCause of any pair and the routed
  getters equal the C oracle;
* ShardedIndex on a whole handle: its exchange and FC collectives run on
  device tensors (zero-length blocks), FC equals the oracle;
* lx_rowseg_comm_create / lx_rowseg_exchange / lx_rowseg_forkless_cause over
  RCCL with one rank equal the oracle.

Each case runs in a spawned process (one RCCL communicator, torn down at exit)."""

import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(case, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        import lachesis_hip as lx
        from oracle import corc
        d = lx.tools.gen_dag(40, 50, 6, 4, 4, 21)
        rng = np.random.default_rng(3)
        w = [int(x) for x in rng.integers(1, 30, 40)]
        o = corc.OracleIndex(w)
        assert o.add_batch(d.creator, d.seq, d.poff, d.par) == -1
        N = len(d)
        qa = rng.integers(0, N, 30_000).astype(np.uint32)
        qb = np.clip(qa.astype(np.int64) - rng.integers(0, 400, 30_000), 0, N - 1).astype(np.uint32)
        want = o.forkless_cause_batch(qa, qb)
        ta = torch.from_numpy(qa.view(np.int32)).to(dev)
        tb = torch.from_numpy(qb.view(np.int32)).to(dev)
        out = torch.full((len(qa),), 7, dtype=torch.uint8, device=dev)
        ok = True
        info = {}
        if case == "rowseg":
            from lachesis_hip.rowseg import RowSegments
            ix = lx.Index(device=0, options={"seg_count": 1, "seg_rank": 0, "small_max": 0, "seg_sub": 2})
            ix.reset(w)
            ix.add_batch(d.creator, d.seq, d.poff, d.par)
            rs = RowSegments(ix, device=dev)
            assert not rs.stage                      # device tensors into the collectives
            info["exchange"] = rs.exchange()
            assert ix.rowseg_range() == (0, N)
            fc = rs.forkless_cause_dev(len(qa), ta, tb, out, timing=True)
            ok = ok and bool(np.array_equal(out.cpu().numpy(), want)) and fc["answered"] == len(qa)
            ev = [int(x) for x in rng.integers(0, N, 120)]
            for mode, f in ((0, o.hb), (1, o.la), (2, o.merged_hb)):
                ok = ok and all(r == f(e) for r, e in zip(rs.get_rows(mode, ev), ev))
            info["fc"] = fc
            ix.close()
        elif case == "shard":
            from lachesis_hip.shard import ShardedIndex
            ix = lx.Index(device=0)
            ix.reset(w)
            ix.add_batch(d.creator, d.seq, d.poff, d.par)
            sx = ShardedIndex(ix, device=dev)
            assert not sx.stage
            assert sx.exchange() == [0]
            res = sx.forkless_cause_dev(ta, tb)
            ok = ok and bool(np.array_equal(res.cpu().numpy(), want))
            ix.close()
        else:   # the library's RCCL transport, one rank
            ix = lx.Index(device=0, options={"seg_count": 1, "seg_rank": 0, "small_max": 0})
            ix.reset(w)
            ix.add_batch(d.creator, d.seq, d.poff, d.par)
            comm = lx.RowsegComm(ix, lx.shard_comm_unique_id(), 1, 0)
            info["exchange"] = comm.exchange()
            comm.forkless_cause_dev(len(qa), ta.data_ptr(), tb.data_ptr(), out.data_ptr())
            ix.sync()
            ok = ok and bool(np.array_equal(out.cpu().numpy(), want))
            ev = np.array([int(x) for x in rng.integers(0, N, 100)] + [N + 1], dtype=np.uint32)
            slot = (ix.row_bytes_max() + 15) // 16 * 16
            te = torch.from_numpy(ev.view(np.int32)).to(dev)
            for mode, f in ((0, o.hb), (1, o.la), (2, o.merged_hb)):
                rows = torch.zeros(len(ev) * slot, dtype=torch.uint8, device=dev)
                lens = torch.zeros(len(ev), dtype=torch.int32, device=dev)
                comm.get_rows_dev(mode, len(ev), te.data_ptr(), rows.data_ptr(), slot, lens.data_ptr())
                rr, ll = rows.cpu().numpy().reshape(len(ev), slot), lens.cpu().numpy().view(np.uint32)
                ok = ok and ll[-1] == 0xFFFFFFFF and all(bytes(rr[i, :ll[i]]) == f(int(e))
                                                         for i, e in enumerate(ev[:-1]))
            comm.close()
            ix.close()
        q.put((ok, repr(info)))
    except Exception as e:
        q.put((False, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["rowseg", "shard", "rccl_rowseg"])
def test_world1_nccl(case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(case, _free_port(), q))
    p.start()
    ok, info = q.get(timeout=170)
    p.join(timeout=60)
    assert p.exitcode == 0 and ok, info

"""Probe: can two processes form an RCCL communicator on ONE GPU (lx_shard_comm)?
If so, run the full 2-shard exchange + ForklessCause and compare with the oracle."""
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "lachesis-base_amd")):
    sys.path.insert(0, p)


def worker(rank, G, uid_q, res_q):
    import numpy as np
    import torch
    import lachesis_hip as lx
    d = lx.tools.gen_dag(16, 30, 5, 3, 4, 21)
    w = [6, 5, 5, 4, 4, 3, 3, 2, 2, 2, 1, 1, 1, 1, 1, 1]
    ix = lx.Index(device=0, shard_rank=rank, shard_count=G)
    ix.reset(w)
    ix.add_batch(d.creator, d.seq, d.poff, d.par)
    if rank == 0:
        uid = lx.shard_comm_unique_id()
        for _ in range(G - 1):
            uid_q.put(uid)
    else:
        uid = uid_q.get()
    try:
        comm = lx.ShardComm(ix, uid, G, rank)
    except Exception as e:
        res_q.put((rank, "create failed: %s" % e))
        return
    comm.exchange()
    qa, qb = lx.tools.fc_queries(d.lamport, 20000, window=20, seed=21)
    dev = torch.device("cuda", 0)
    a = torch.from_numpy(qa.view(np.int32)).to(dev)
    b = torch.from_numpy(qb.view(np.int32)).to(dev)
    out = torch.empty(len(qa), dtype=torch.uint8, device=dev)
    comm.forkless_cause_dev(len(qa), a.data_ptr(), b.data_ptr(), out.data_ptr())
    ix.sync()
    from oracle import corc
    o = corc.OracleIndex(w)
    o.add_batch(d.creator, d.seq, d.poff, d.par)
    ok = bool(np.array_equal(out.cpu().numpy(), o.forkless_cause_batch(qa, qb)))
    comm.close()
    res_q.put((rank, "fc equal to oracle: %s" % ok))


if __name__ == "__main__":
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = mp.get_context("spawn")
    uq, rq = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, G, uq, rq)) for r in range(G)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(80)
    res = []
    while not rq.empty():
        res.append(rq.get())
    print("results:", sorted(res))
    bad = [p for p in ps if p.exitcode != 0]
    for p in ps:
        if p.is_alive():
            p.kill()
    sys.exit(1 if bad or len(res) < G else 0)

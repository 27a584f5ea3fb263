"""k_fc on the bench's 2^24 queries in their own order and reordered by a
(fully sorted, or bucketed by a >> k): do HB(a) duplicates and the LA(b)
window of nearby a's hit L2 / MALL?  Timed with HIP events on the library
stream, 5 launches each, after an untimed one."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402

V = 1000
d = lx.tools.gen_dag(V, 10_000, 10, seed=1)
N = len(d)
w = [(1 << 20) // (i + 1) for i in range(V)]
dev = torch.device("cuda", 0)
to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
ix = lx.Index(event_capacity=N)
ix.reset(w)
keep = [to_dev(d.creator), to_dev(d.seq), to_dev(d.poff.astype(np.uint32)), to_dev(d.par)]   # alive until the add
ix.add_batch_dev(N, *[t.data_ptr() for t in keep])
ix.sync()
nq = 1 << 24
qa, qb = lx.tools.fc_queries(d.lamport, nq, window=64, seed=7)
_, _, _, sp = ix.device_planes()
st = torch.cuda.ExternalStream(sp, device=dev)
res = {}
ref = None
for name in ("given", "sorted_a", "bucket_a>>10", "bucket_a>>14", "bucket_a>>17"):
    if name == "given":
        perm = np.arange(nq)
    elif name == "sorted_a":
        perm = np.argsort(qa, kind="stable")
    else:
        sh = int(name.split(">>")[1])
        perm = np.argsort(qa >> sh, kind="stable")
    a, b = to_dev(qa[perm]), to_dev(qb[perm])
    out = torch.empty(nq, dtype=torch.uint8, device=dev)
    ix.forkless_cause_batch_dev(nq, a.data_ptr(), b.data_ptr(), out.data_ptr())
    ix.sync()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        ix.forkless_cause_batch_dev(nq, a.data_ptr(), b.data_ptr(), out.data_ptr())
        e1.record(st)
        ix.sync()
        ts.append(e0.elapsed_time(e1))
    got = np.empty(nq, dtype=np.uint8)
    got[perm] = out.cpu().numpy()
    if ref is None:
        ref = got
    res[name] = {"ms": float(np.median(ts)), "same_answers": bool(np.array_equal(got, ref)),
                 "tb_per_s_algorithmic": 8.0 * V * nq / (np.median(ts) * 1e-3) / 1e12}
    print(json.dumps(res), flush=True)

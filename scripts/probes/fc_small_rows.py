"""ForklessCause on configs[0] / [1] (20-B / 400-B rows): k_fc time per 2^22
queries (HIP events, median of 7) and a checksum of the answers, with the
library LX_LIB names (A/B of lane counts per query)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402

out = {"lib": os.environ.get("LX_LIB", "build")}
for name, (V, epv, P) in {"c1": (5, 1000, 5), "c2": (100, 10000, 10)}.items():
    d = lx.tools.gen_dag(V, epv, P, seed=1)
    N = len(d)
    dev = torch.device("cuda", 0)
    to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    ix = lx.Index(event_capacity=N)
    ix.reset([1] * V)
    keep = [to_dev(d.creator), to_dev(d.seq), to_dev(d.poff.astype(np.uint32)), to_dev(d.par)]
    ix.add_batch_dev(N, *[t.data_ptr() for t in keep])
    ix.sync()
    n = 1 << 22
    qa, qb = lx.tools.fc_queries(d.lamport, n, window=64, seed=7)
    da, db = to_dev(qa), to_dev(qb)
    o = torch.empty(n, dtype=torch.uint8, device=dev)
    st = torch.cuda.ExternalStream(ix.device_planes()[3], device=dev)
    ms = []
    for r in range(8):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        ix.forkless_cause_batch_dev(n, da.data_ptr(), db.data_ptr(), o.data_ptr())
        e1.record(st)
        ix.sync()
        ms.append(e0.elapsed_time(e1))
    out[name] = {"kernel_ms_median": float(np.median(ms[1:])), "true": int(o.sum().item()),
                 "checksum": int((o.to(torch.int64) * torch.arange(n, device=dev)).sum().item())}
    ix.close()
print(json.dumps(out))

"""k_fc_early with one or two queries' first round in flight beside the
current one (option fc_early_depth) on the headline config: C3 (V = 1000,
Zipf stakes, 10M events), 2^24 queries of the bench's shape; median of 5
launches each, alternating, answers compared byte for byte with the
whole-row kernel.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402

d = lx.tools.gen_dag(1000, 10000, 10, seed=1)
N = len(d)
w = [(1 << 20) // (i + 1) for i in range(1000)]
dev = torch.device("cuda", 0)
to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
dc, ds, dp, do = to_dev(d.creator), to_dev(d.seq), to_dev(d.par), to_dev(d.poff.astype(np.uint32))
ix = lx.Index(event_capacity=N)
ix.reset(w)
ix.add_batch_dev(N, dc.data_ptr(), ds.data_ptr(), do.data_ptr(), dp.data_ptr())
ix.sync()
qa, qb = lx.tools.fc_queries(d.lamport, 1 << 24, window=64, seed=7)
ta, tb = to_dev(qa), to_dev(qb)
res = {"queries": len(qa)}
outs = {}
for var in ("d1", "d2", "whole", "d1", "d2", "d1", "d2"):
    ix.set_option("fc_early", 0 if var == "whole" else 1)
    if var != "whole":
        ix.set_option("fc_early_depth", int(var[1]))
    out = torch.empty(len(qa), dtype=torch.uint8, device=dev)
    ts = []
    for rep in range(6):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ix.forkless_cause_batch_dev(len(qa), ta.data_ptr(), tb.data_ptr(), out.data_ptr())
        ix.sync()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    outs[var] = out.cpu().numpy()
    res.setdefault("ms_" + var, []).append(float(np.median(ts[1:])))
res["identical"] = bool(np.array_equal(outs["whole"], outs["d1"]) and np.array_equal(outs["whole"], outs["d2"]))
print(json.dumps(res))

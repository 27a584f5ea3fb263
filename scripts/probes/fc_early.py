"""k_fc with and without the early exit (option fc_early) on the headline
config: C3 (V = 1000, Zipf stakes, 10M events), 2^24 queries of the bench's
shape (b within 64 Lamport of a), device arrays; median of 5 launches each,
answers compared byte for byte.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402

V, epv = int(os.environ.get("FE_V", "1000")), int(os.environ.get("FE_EPV", "10000"))
zipf = os.environ.get("FE_W", "zipf") == "zipf"
d = lx.tools.gen_dag(V, epv, 10, seed=1)
N = len(d)
w = [(1 << 20) // (i + 1) for i in range(V)] if zipf else [1] * V
dev = torch.device("cuda", 0)
to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
dc, ds, dp, do = to_dev(d.creator), to_dev(d.seq), to_dev(d.par), to_dev(d.poff.astype(np.uint32))
ix = lx.Index(event_capacity=N)
ix.reset(w)
ix.add_batch_dev(N, dc.data_ptr(), ds.data_ptr(), do.data_ptr(), dp.data_ptr())
ix.sync()
qa, qb = lx.tools.fc_queries(d.lamport, 1 << 24, window=64, seed=7)
ta, tb = to_dev(qa), to_dev(qb)
res = {"V": V, "events": N, "zipf": zipf, "queries": len(qa)}
outs = {}
# variants: 0 = whole rows, 32 / 16 = the early exit with that many lanes per query
for early in (32, 0, 16, 32, 0, 16):
    ix.set_option("fc_early", 1 if early else 0)
    if early:
        ix.set_option("fc_early_lanes", early)
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
        ms = e0.elapsed_time(e1)
        ts.append(ms)
    outs[early] = out.cpu().numpy()
    res.setdefault("ms_early%d" % early, []).append(float(np.median(ts[1:])))
res["identical"] = bool(np.array_equal(outs[0], outs[32]) and np.array_equal(outs[0], outs[16]))
res["true_frac"] = float(outs[0].mean())
for L in (32, 16):
    ix.set_option("fc_early", 1)
    ix.set_option("fc_early_lanes", L)
    ix.fc_early_rounds()
    ix.forkless_cause_batch_dev(len(qa), ta.data_ptr(), tb.data_ptr(), out.data_ptr())
    res["rounds_L%d" % L] = ix.fc_early_rounds()
print(json.dumps(res))

"""k_fc_early with one or two queries in flight ahead per half-wave (option
fc_early_depth, removed after this A/B), interleaved in one process on the headline config (C3, 2^24
queries of the bench's shape, device arrays): per setting and round the
median of 5 launches; answers compared byte for byte.  One JSON line."""
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
ix.set_option("fc_early", 1)
res, outs = {}, {}
for rnd in range(4):
    for depth in (1, 2):
        for lanes in (32, 16):
            ix.set_option("fc_early_depth", depth)
            ix.set_option("fc_early_lanes", lanes)
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
            outs[(depth, lanes)] = out.cpu().numpy()
            res.setdefault("ms_d%d_L%d" % (depth, lanes), []).append(round(float(np.median(ts[1:])), 3))
ref = outs[(1, 32)]
res["identical"] = all(bool(np.array_equal(ref, o)) for o in outs.values())
print(json.dumps(res))

"""Per-rank walk of the row-segment mode at C3 (V = 1000, 10M events), one
rank at a time on one GPU: a handle with seg_count = G, seg_rank = r adds the
whole epoch (assignment of every event + the walk of its own segment) -- the
part of a rank's index step before the exchanges.  seg_sub = 1 (one walk of
the rank's segment) against the default (side-by-side sub-segments)."""
import json
import os
import sys
import time

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
keep = [to_dev(d.creator), to_dev(d.seq), to_dev(d.poff.astype(np.uint32)), to_dev(d.par)]
res = {}
for G in (2, 4, 8):
    for r in (0, G - 1):
        for sub in (1, 0):
            ix = lx.Index(event_capacity=N, options={"seg_count": G, "seg_rank": r, "seg_sub": sub})
            ts = []
            for rep in range(3):
                ix.reset(w)
                ix.sync()
                t0 = time.perf_counter()
                ix.add_batch_dev(N, *[t.data_ptr() for t in keep])
                ix.sync()
                ts.append((time.perf_counter() - t0) * 1e3)
            st = ix.segment_stats()
            res["G%d r%d sub%d" % (G, r, sub)] = {"add_ms": float(np.median(ts[1:])), "walk_ms": st["walk_ms"][r],
                                                  "one_launch": st["one_launch"], "partial": st["partial"][r]}
            ix.close()
            print(json.dumps(res), flush=True)

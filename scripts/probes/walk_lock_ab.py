"""Option A/B inside one process: the C3 walk (V = 1000, Zipf stakes, 10M
events, one batch, default options: three side-by-side walks of 12-column
slices) with each setting of WL_OPT (default lockstep) in WL_VALUES taken in
turn, WL_ROUNDS rounds.  Boxes run whole processes in a fast or a slow mode
(profiles/r05/walker), so the settings are interleaved walk by
walk in one process.  One JSON line per walk: setting, walk ms (the slowest
segment), the shader clock and its per-XCD slowest workgroup."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402

opt = os.environ.get("WL_OPT", "lockstep")
values = [int(x) for x in os.environ.get("WL_VALUES", "0,16,4").split(",")]
d = lx.tools.gen_dag(1000, 10000, 10, seed=1)
N = len(d)
w = [(1 << 20) // (i + 1) for i in range(1000)]
dev = torch.device("cuda", 0)
to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
dc, ds, dp, do = to_dev(d.creator), to_dev(d.seq), to_dev(d.par), to_dev(d.poff.astype(np.uint32))
ix = lx.Index(event_capacity=N)
ix.reset(w)
ix.add_batch_dev(N, dc.data_ptr(), ds.data_ptr(), do.data_ptr(), dp.data_ptr())   # first touches
for r in range(int(os.environ.get("WL_ROUNDS", "4"))):
    for v in values:
        ix.set_option(opt, v)
        ix.reset(w)
        ix.add_batch_dev(N, dc.data_ptr(), ds.data_ptr(), do.data_ptr(), dp.data_ptr())
        ix.sync()
        st = ix.segment_stats()
        c = ix.walk_clock()
        print(json.dumps({"pid": os.getpid(), "round": r, opt: v, "walk_ms": round(max(st["walk_ms"]), 2),
                          "ms_index": round(ix.last_stats()["ms_index"], 2), "partial": st["partial"],
                          "mhz": round(c["mhz_median"], 1), "xcd_walk_ms_max": c["xcd_walk_ms_max"]}), flush=True)

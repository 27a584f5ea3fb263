"""Walk time of the headline config (C3: V = 1000, Zipf stakes, 10M events,
one batch, default options = three side-by-side segments of 12-column slices)
with whichever library LX_LIB names: median of 5 index steps (ms_index and
the segment walk from lx_last_segment_stats).  scripts/probes/walk_ab.sh runs
it alternately on the shipped build and an A/B baseline build."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402

V, epv = int(os.environ.get("WT_V", "1000")), int(os.environ.get("WT_EPV", "10000"))
d = lx.tools.gen_dag(V, epv, 10, seed=1)
N = len(d)
w = [(1 << 20) // (i + 1) for i in range(V)]
dev = torch.device("cuda", 0)
to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
dc, ds, dp, do = to_dev(d.creator), to_dev(d.seq), to_dev(d.par), to_dev(d.poff.astype(np.uint32))
# WT_OPTS: index options as JSON, e.g. '{"cpw": 8}'
ix = lx.Index(event_capacity=N, options=json.loads(os.environ.get("WT_OPTS", "{}")))
ks, walks = [], []
for r in range(6):
    ix.reset(w)
    ix.add_batch_dev(N, dc.data_ptr(), ds.data_ptr(), do.data_ptr(), dp.data_ptr())
    ix.sync()
    ks.append(ix.last_stats()["ms_index"])
    st = ix.segment_stats()
    walks.append(max(st["walk_ms"]) if st["segments"] else None)
print(json.dumps({"lib": os.environ.get("LX_LIB", "build/liblachesis_hip.so"), "opts": os.environ.get("WT_OPTS", "{}"), "events": N,
                  "ms_index_median": float(np.median(ks[1:])), "ms_index": ks[1:],
                  "walk_ms": walks[1:], "segments": ix.segment_stats()["segments"],
                  # partial events per segment: a walk that publishes wrong rows shows up here
                  "partial": ix.segment_stats()["partial"]}))

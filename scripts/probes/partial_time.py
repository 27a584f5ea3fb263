"""C3 default walk (two side-by-side segments): the partial-event fix-up
(k_seg_partial) and the whole index step, median of 5 after a warmup."""
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
keep = [to_dev(d.creator), to_dev(d.seq), to_dev(d.poff.astype(np.uint32)), to_dev(d.par)]
ix = lx.Index(event_capacity=N)
pm, ms = [], []
for r in range(6):
    ix.reset(w)
    ix.add_batch_dev(N, *[t.data_ptr() for t in keep])
    ix.sync()
    st = ix.segment_stats()
    pm.append(st["partial_ms"])
    ms.append(ix.last_stats()["ms_index"])
print(json.dumps({"lib": os.environ.get("LX_LIB", "build"), "partial": st["partial"], "partial_ms": float(np.median(pm[1:])),
                  "ms_index": float(np.median(ms[1:]))}))

"""configs[1] (V = 100, 1M events) index step with the batch split into
concurrent Add-order segments on idle CUs (seg_auto = 1, the default) and as
one walk (seg_auto = 0): step time, k_index time, segment stats."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import lachesis_hip as lx  # noqa: E402

V = int(os.environ.get("V", "100"))
EPV = int(os.environ.get("EPV", str(1_000_000 // V)))
CH, FK = int(os.environ.get("CH", "0")), int(os.environ.get("FK", "0"))
d = lx.tools.gen_dag(V, EPV, 10, CH, FK, seed=1)
w = [1] * V
res = {}
for auto in (1, 0):
    ix = lx.Index(options={"seg_auto": auto}, event_capacity=len(d))
    ts = []
    for r in range(5):
        ix.reset(w)
        ix.sync()
        t0 = time.perf_counter()
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        ix.sync()
        ts.append((time.perf_counter() - t0) * 1e3)
    r = {"step_ms_med": float(np.median(ts[1:])), "index_ms": ix.last_stats()["ms_index"]}
    if auto:
        try:
            r["segments"] = ix.segment_stats()
        except Exception as e:  # not segmented
            r["segments"] = repr(e)
    res["seg_auto%d" % auto] = r
    ix.close()
print(json.dumps(res))

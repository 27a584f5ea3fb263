"""Walk time on 8-column slices: C3 (V = 1000) as one walk at 4 and 8
columns per slice and as 2 side-by-side segments of 8-column slices; C2
(V = 100) as 8 segments of 4-column and 16 of 8-column slices."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import lachesis_hip as lx  # noqa: E402

CASES = {
    "c3": (1000, 10000, [{}, {"cpw": 8, "seg_auto": 0}, {"cpw": 8, "segments": 2}, {"cpw": 4, "segments": 2}]),
    "c2": (100, 10000, [{"cpw": 4, "segments": 8}, {"cpw": 8, "segments": 16}, {"cpw": 8, "segments": 8}]),
}
res = {}
for name in sys.argv[1:] or list(CASES):
    V, epv, variants = CASES[name]
    d = lx.tools.gen_dag(V, epv, 10, seed=1)
    w = [(1 << 20) // (i + 1) for i in range(V)]
    for opts in variants:
        ix = lx.Index(options=dict(opts), event_capacity=len(d))
        ts, ks = [], []
        for r in range(3):
            ix.reset(w)
            ix.sync()
            t0 = time.perf_counter()
            ix.add_batch(d.creator, d.seq, d.poff, d.par)
            ix.sync()
            ts.append((time.perf_counter() - t0) * 1e3)
            ks.append(ix.last_stats()["ms_index"])
        r = {"step_ms": float(np.median(ts[1:])), "index_ms": float(np.median(ks[1:]))}
        if opts.get("segments"):
            st = ix.segment_stats()
            r.update(walk_ms=st["walk_ms"][:1], partial=int(sum(st["partial"])), partial_ms=st["partial_ms"], la_ms=st["la_ms"])
        res["%s %s" % (name, json.dumps(opts, sort_keys=True))] = r
        ix.close()
        print(json.dumps(res), flush=True)

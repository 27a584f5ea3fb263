import sys, os, json, time
sys.path[:0] = ["/root/repo", "/root/repo/lachesis-base_amd"]
import numpy as np, lachesis_hip as lx
d = lx.tools.gen_dag(5, 1000, 5, seed=1)
w = [1]*5
res = {}
for dbl in (1, 0):
    ix = lx.Index(options={"dbl": dbl})
    ts, ks = [], []
    for r in range(12):
        ix.reset(w)
        ix.sync()
        t0 = time.perf_counter()
        ix.add_batch(d.creator, d.seq, d.poff, d.par)
        ix.sync()
        ts.append((time.perf_counter() - t0) * 1e3)
        ks.append(ix.last_stats()["ms_index"])
    res["dbl%d" % dbl] = {"step_ms_med": float(np.median(ts[2:])), "index_ms_med": float(np.median(ks[2:]))}
    ix.close()
print(json.dumps(res))

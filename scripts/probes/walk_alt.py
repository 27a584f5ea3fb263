"""Does the walk's slow mode follow the index handle (its planes and record
buffers) or the moment?  Two handles alive at once (C3: V = 1000, Zipf
stakes, 10M events, one batch, default options), walks alternating A, B, A,
B, ... (WA_MOVE=1: handle A's record buffers moved to a fresh allocation
before every odd round); one JSON line per walk: handle, walk ms, the slowest XCD's walk ms
and the KFD eviction time of this process over the walk."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd"), os.path.dirname(os.path.abspath(__file__))]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402
from kfd_stats import kfd_self  # noqa: E402

d = lx.tools.gen_dag(1000, 10000, 10, seed=1)
N = len(d)
w = [(1 << 20) // (i + 1) for i in range(1000)]
dev = torch.device("cuda", 0)
to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
dc, ds, dp, do = to_dev(d.creator), to_dev(d.seq), to_dev(d.par), to_dev(d.poff.astype(np.uint32))
hs = [lx.Index(event_capacity=N) for _ in range(int(os.environ.get("WA_HANDLES", "2")))]
move = os.environ.get("WA_MOVE") == "1"   # handle 0's record buffers moved before every other round
for r in range(int(os.environ.get("WA_ROUNDS", "4"))):
    if move and r % 2 == 1:
        hs[0].set_option("realloc_records", 1)
    for k, ix in enumerate(hs):
        k0 = kfd_self()
        ix.reset(w)
        ix.add_batch_dev(N, dc.data_ptr(), ds.data_ptr(), do.data_ptr(), dp.data_ptr())
        ix.sync()
        k1 = kfd_self()
        st = ix.segment_stats()
        c = ix.walk_clock()
        ev = None
        if k0 and k1:
            ev = {p: [k1[p]["evicted_ms"] - k0.get(p, k1[p])["evicted_ms"], round(k1[p]["vram_gib"])]
                  for p in k1 if k1[p]["vram_gib"] >= 60}
        print(json.dumps({"pid": os.getpid(), "round": r, "handle": k, "moved": bool(move and k == 0 and r % 2 == 1), "walk_ms": round(max(st["walk_ms"]), 2),
                          "walk_ms_by_segment": [round(x, 2) for x in st["walk_ms"]],
                          "mhz": round(c["mhz_median"], 1), "xcd_walk_ms_max": c["xcd_walk_ms_max"],
                          "evicted_ms": ev}), flush=True)

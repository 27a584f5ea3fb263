"""Is the walk's slow mode a property of the process or of the allocation?

One process, WM_INST fresh Index handles one after the other (each allocates
its own HB / LA planes and record buffers, and frees them before the next),
WM_WALKS walks of the headline config (C3: V = 1000, Zipf stakes, 10M events,
one batch, default options) on each.  One JSON line per handle: walk ms per
step.  LX_LIB picks the library (probe builds: make build_pNOLA/... or
build_pNOHB/..., the LowestAfter range-fill or HB row stores compiled out).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kfd_stats import kfd_self  # noqa: E402

V, epv = int(os.environ.get("WT_V", "1000")), int(os.environ.get("WT_EPV", "10000"))
n_inst, n_walk = int(os.environ.get("WM_INST", "3")), int(os.environ.get("WM_WALKS", "4"))
d = lx.tools.gen_dag(V, epv, 10, seed=1)
N = len(d)
w = [(1 << 20) // (i + 1) for i in range(V)]
dev = torch.device("cuda", 0)
to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
dc, ds, dp, do = to_dev(d.creator), to_dev(d.seq), to_dev(d.par), to_dev(d.poff.astype(np.uint32))
lib = os.path.basename(os.path.dirname(os.environ.get("LX_LIB", "build/x")))
clk = None
if os.environ.get("WM_CLK") == "1":
    # probe build build_pCLK: per workgroup of the last walk, shader cycles and
    # 100 MHz ticks of compute wave 0 and its XCD (lx_probe_clk_read)
    import ctypes
    clk = ctypes.CDLL(os.environ["LX_LIB"])
    buf = (ctypes.c_ulonglong * (1024 * 3))()


def clocks():
    n = clk.lx_probe_clk_read(buf, 1024)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 3)[:n].astype(np.float64)
    a = a[a[:, 1] > 0]
    mhz = a[:, 0] / a[:, 1] * 100.0
    per_xcd = {int(x): round(float(np.median(mhz[a[:, 2] == x])), 1) for x in sorted(set(a[:, 2]))}
    return {"mhz_median": round(float(np.median(mhz)), 1), "mhz_min": round(float(mhz.min()), 1),
            "mhz_max": round(float(mhz.max()), 1), "wave0_ms_max": round(float(a[:, 1].max()) / 1e5, 2),
            "mhz_by_xcd": per_xcd}


for inst in range(n_inst):
    ix = lx.Index(event_capacity=N, options=json.loads(os.environ.get("WT_OPTS", "{}")))
    hb_ptr, la_ptr, stride, _ = ix.device_planes()
    walks, clks, kfd = [], [], []
    for r in range(n_walk):
        k0 = kfd_self()
        ix.reset(w)
        ix.add_batch_dev(N, dc.data_ptr(), ds.data_ptr(), do.data_ptr(), dp.data_ptr())
        ix.sync()
        st = ix.segment_stats()
        walks.append(round(max(st["walk_ms"]), 2) if st["segments"] else round(ix.last_stats()["ms_index"], 2))
        k1 = kfd_self()
        if k0 and k1:
            # the process holding >= 60 GiB (this one's planes), its changes over the walk
            mine = [p for p in k1 if k1[p]["vram_gib"] >= 60]
            kfd.append({p: {"evicted_ms": k1[p]["evicted_ms"] - k0.get(p, k1[p])["evicted_ms"],
                            "page_in": k1[p]["page_in"] - k0.get(p, k1[p])["page_in"],
                            "page_out": k1[p]["page_out"] - k0.get(p, k1[p])["page_out"],
                            "vram_gib": round(k1[p]["vram_gib"], 1)} for p in mine})
        if clk is not None:
            clks.append(clocks())
        elif os.environ.get("WM_SHIPCLK") == "1":
            # the shipped walker's own clock record (lx_last_walk_clock)
            c = ix.walk_clock()
            clks.append({k: (round(v, 2) if isinstance(v, float) else v) for k, v in c.items()} | {"t": round(time.time(), 3)})
    print(json.dumps({"lib": lib, "pid": os.getpid(), "inst": inst, "walk_ms": walks,
                      "hb": hex(hb_ptr or 0), "la": hex(la_ptr or 0), "partial": st["partial"],
                      **({"clk": clks} if clks else {}), **({"kfd_delta": kfd} if kfd else {})}), flush=True)
    ix.close()
    del ix

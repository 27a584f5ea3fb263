"""How far the slices of one walk drift apart (probe build build_pSKEW: the
drain of every 32nd round stamps the wall clock per workgroup).  C3 (V =
1000, Zipf stakes, 10M events, one batch, default options: three side-by-side
walks of 84 twelve-column slices).  Per walk: the spread (max - min over the
84 slices) of the time each 2048-event mark was drained, and the same between
neighbouring slices (which share 128-B HB lines), in microseconds and in
events of the walk's average rate.  One JSON line per walk."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lachesis_hip as lx  # noqa: E402

SLOTS = 2048
d = lx.tools.gen_dag(1000, 10000, 10, seed=1)
N = len(d)
w = [(1 << 20) // (i + 1) for i in range(1000)]
dev = torch.device("cuda", 0)
to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
dc, ds, dp, do = to_dev(d.creator), to_dev(d.seq), to_dev(d.par), to_dev(d.poff.astype(np.uint32))
L = ctypes.CDLL(os.environ["LX_LIB"])
stamps = np.zeros(1024 * SLOTS, dtype=np.uint64)
wmap = np.zeros(1024, dtype=np.uint32)
ix = lx.Index(event_capacity=N, options=json.loads(os.environ.get("WT_OPTS", "{}")))
for r in range(int(os.environ.get("WS_WALKS", "3"))):
    ix.reset(w)
    ix.add_batch_dev(N, dc.data_ptr(), ds.data_ptr(), do.data_ptr(), dp.data_ptr())
    ix.sync()
    st = ix.segment_stats()
    assert L.lx_probe_skew_read(stamps.ctypes.data_as(ctypes.c_void_p), wmap.ctypes.data_as(ctypes.c_void_p)) == 0
    S = stamps.reshape(1024, SLOTS).astype(np.float64) / 100.0   # 100 MHz ticks -> us
    out = {"walk_ms": [round(x, 2) for x in st["walk_ms"]], "clock": ix.walk_clock(), "walks": []}
    for k in range(st["segments"]):
        n_k = st["first_event"][k + 1] - st["first_event"][k]
        marks = n_k // 2048
        rows, xcd_of = {}, {}
        for g in range(1024):
            if S[g, 0] > 0 and (wmap[g] >> 16) == k:
                rows[int(wmap[g] & 0xFFFF)] = S[g, :marks]
                xcd_of[int(wmap[g] & 0xFFFF)] = g % 8        # blocks g, g + 8, ... share an XCD
        sl = sorted(rows)
        M = np.stack([rows[s] for s in sl])                 # slices x marks
        M = M - M[:, :1].min()                              # from the walk's first mark
        rate = n_k / (M[:, -1].max() - M[:, 0].min())       # events per us
        spread = M.max(axis=0) - M.min(axis=0)
        nb = np.abs(np.diff(M, axis=0))                     # neighbouring slices
        q = lambda a, p: round(float(np.percentile(a, p)), 1)
        out["walks"].append({
            "slices": len(sl), "marks": int(marks), "events_per_us": round(float(rate), 1),
            "spread_us": {"p50": q(spread, 50), "p90": q(spread, 90), "max": q(spread, 100), "end": q(spread[-1:], 50)},
            "neighbour_us": {"p50": q(nb, 50), "p90": q(nb, 90), "p99": q(nb, 99), "max": q(nb, 100)},
            "neighbour_events_p90": round(float(np.percentile(nb, 90)) * rate, 0),
            "slowest_slice_at_end": int(sl[int(np.argmax(M[:, -1]))]),
            # where the slowest slice lost its time: marks (x 2048 events into the
            # walk) at which its lag behind the median slice grew by > 200 us
            "lag_jumps": [(int(t), round(float(dl), 0)) for t, dl in enumerate(np.diff(
                M[int(np.argmax(M[:, -1]))] - np.median(M, axis=0))) if dl > 200.0][:40],
            # each XCD group's (g % 8) slowest slice end, ms after the walk's first mark
            "end_ms_by_block_group": {x: round(float(max(M[i, -1] for i, s_ in enumerate(sl) if xcd_of[s_] == x)) / 1e3, 2)
                                      for x in sorted(set(xcd_of.values()))}})
    print(json.dumps(out), flush=True)

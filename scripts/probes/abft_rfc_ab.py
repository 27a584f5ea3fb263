"""A/B of the root ForklessCause early exit (lx_abft option rfc_early) on
BASELINE configs[4] (C5: V = 1000, Zipf stakes, 50 events per validator,
claimed frames), settings interleaved epoch by epoch in one process: per
epoch the wall time and the phase split (lx_abft_last_stats)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import lachesis_hip as lx  # noqa: E402

V, epv, P = 1000, 50, 10
w = [(1 << 20) // (i + 1) for i in range(V)]
dag = lx.tools.gen_dag(V, epv, P, 0, 0, seed=1)
N = len(dag)
lch = lx.abft.DenseLachesis(w, event_capacity=N, apply_events=False)
rc, consumed, frames = lch.process_batch(dag.creator, dag.seq, dag.poff, dag.par)
claimed = frames.copy()
for r in range(int(os.environ.get("AB_ROUNDS", "4"))):
    for v in (0, 1):
        lch.set_option("rfc_early", v)
        lch.L.lx_abft_reset(lch.h, 1, V, np.ascontiguousarray(w, dtype=np.uint32).ctypes.data_as(
            lx.capi.u32p))
        t = time.perf_counter()
        rc, consumed, out = lch.process_batch(dag.creator, dag.seq, dag.poff, dag.par, claimed)
        dt = (time.perf_counter() - t) * 1e3
        assert rc == 0 and consumed == N and np.array_equal(out, claimed)
        st = lch.last_stats()
        print(json.dumps({"rfc_early": v, "ms": round(dt, 2), "ms_frames": round(st["ms_frames"], 2),
                          "ms_root_fc_gpu": round(st["ms_root_fc_gpu"], 2), "fc_launches": st["fc_launches"],
                          "frame_steps": st["frame_steps"],
                          "tiled": st["fc_pair_cols_tiled"] / max(1, st["fc_pair_cols"])}), flush=True)

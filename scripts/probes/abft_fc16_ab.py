"""abft option A/B inside one process (default option fc16: the packed
root-FC kernel k_root_fc16 against the 32-bit k_root_fc) on bench.py's abft
leg workload (BASELINE configs[4], C5: V = 1000, Zipf stakes, 50k events, one
epoch per step, claimed frames).  Settings are interleaved step by step; one
JSON line per step: setting, step ms, phase ms, root-FC GPU ms and launches."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import numpy as np  # noqa: E402
import bench  # noqa: E402
import lachesis_hip as lx  # noqa: E402

opt = os.environ.get("AB_OPT", "fc16")
values = [int(x) for x in os.environ.get("AB_VALUES", "1,0").split(",")]
name, V, epv, P, wkind = bench.ABFT_CONFIG
weights = bench.weights_for(V, wkind)
dag = lx.tools.gen_dag(V, epv, P, 0, 0, seed=1)
N = len(dag)
lch = lx.abft.DenseLachesis(weights, device=0, event_capacity=N, apply_events=False)
rc, consumed, frames = lch.process_batch(dag.creator, dag.seq, dag.poff, dag.par)
assert rc == 0 and consumed == N
claimed = frames.copy()
n_blocks = len(lch.blocks)
w32 = np.ascontiguousarray(weights, dtype=np.uint32)
for r in range(int(os.environ.get("AB_ROUNDS", "6"))):
    for v in values:
        lch.set_option(opt, v)
        lch.L.lx_abft_reset(lch.h, 1, V, w32.ctypes.data_as(lx.capi.u32p))
        lch.blocks = []
        t0 = time.perf_counter()
        rc, consumed, out = lch.process_batch(dag.creator, dag.seq, dag.poff, dag.par, claimed)
        dt = (time.perf_counter() - t0) * 1e3
        assert rc == 0 and consumed == N and len(lch.blocks) == n_blocks and np.array_equal(out, claimed)
        st = lch.last_stats()
        print(json.dumps({"round": r, opt: v, "ms_step": round(dt, 3),
                          "ms_frames": round(st["ms_frames"], 3), "ms_election": round(st["ms_election"], 3),
                          "ms_root_fc_gpu": round(st["ms_root_fc_gpu"], 3), "fc_launches": st["fc_launches"],
                          "ops_per_pair_col": round(st["fc_lane_ops"] / max(st["fc_pair_cols"], 1), 3),
                          "frame_steps": st["frame_steps"], "vote_launches": st["vote_launches"],
                          "elections_ahead": st["elections_ahead"]}), flush=True)
lch.close()

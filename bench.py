"""Benchmark: events indexed/sec + ForklessCause queries/sec at 1000 validators.

Workload (BASELINE.json configs[2], the config the metric is quoted on; it fits
one MI355X): V = 1000 validators with skewed stakes w_i = floor(2^20/(i+1)),
10M events (10k per validator), P = 10 parents, tdag-structured synthetic DAG
(lachesis-base_amd/tools/dag_gen.cpp, seed 1).  Inputs are uploaded to HBM
before timing.

  index step : lx_reset + lx_add_batch_dev over the whole epoch (branch
               assignment, HB max-join, fork marks, LA range fill) -- the
               reference's Reset + Add x N (vecfc/index.go:98-105,
               vecengine/index.go:71-233)
  fc step    : 2^24 ForklessCause queries (a uniform, b within 64 Lamport of a,
               SURVEY 8d) -- vecfc/forkless_cause.go:28-82

value = events indexed/sec (whole job, all ranks); fc_queries_per_sec is
reported beside it.  Multi-GPU: one process per GPU.
  --mode rowseg (default for N > 1): the epoch's Add order split into N row
      segments, one per rank: each rank walks its segment
      and holds its own rows, the row / LowestAfter exchange is inside the
      index step; FC routes every rank's 2^24 queries to owner(a) (6c).  The
      same run then measures BASELINE configs[2] as it names it -- "column-
      sharded across 8xMI355X" -- in the line's `colshard` block (skip with
      --no-colshard): each rank indexes its creator columns, the index step
      ends with the all-to-all of LowestAfter blocks, FC sums per-rank partial
      stakes with an all-reduce (strong scaling: value = the epoch's events /
      time, both modes).
  --mode shard: column shards as the line's primary measurement.
  --mode replica: each rank indexes its own copy of the workload (independent
      epochs; no data-path collective; weak scaling).
LX_DIST_BACKEND=gloo (rehearsal only) lets several ranks share one GPU.
"""

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "lachesis-base_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

CONFIGS = {
    # name: (V, events per validator, parents, cheaters, forks, weights)
    "c1": (5, 1000, 5, 0, 0, "equal"),
    "c2": (100, 10_000, 10, 0, 0, "equal"),
    "c3": (1000, 10_000, 10, 0, 0, "zipf"),
    "c4": (100, 1000, 10, 10, 10, "equal"),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec


def measured_traffic(config, fc_queries):
    """HBM bytes per launch from the newest committed PMC profile of this
    workload (profiles/r*/traffic_<config>.json; round 2: scripts/prof_round.sh,
    reads from the L2's memory-side read requests by size, writes from
    WRITE_SIZE, separate passes), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic_%s.json" % config)))
    if not files:
        return None, None
    with open(files[-1]) as f:
        t = json.load(f)
    if t.get("fc_queries") != fc_queries:
        return None, None
    return t["kernels"], os.path.relpath(files[-1], ROOT)


def weights_for(V, kind):
    if kind == "zipf":
        return [(1 << 20) // (i + 1) for i in range(V)]
    return [1] * V


def cpu_baseline(dag, weights, n_events_max, fc_n, budget_s):
    """Single-threaded C restatement of the reference algorithm (oracle/,
    kind 'port'): per-event Add with DFS LowestAfter, byte rows; then FC."""
    import numpy as np
    from oracle import corc
    o = corc.OracleIndex(weights)
    t0 = time.perf_counter()
    done = 0
    chunk = 200
    while done < n_events_max and time.perf_counter() - t0 < budget_s:
        hi = min(n_events_max, done + chunk)
        r = o.add_batch(dag.creator[done:hi], dag.seq[done:hi], dag.poff[done:hi + 1], dag.par)
        assert r == -1
        done = hi
    t_add = time.perf_counter() - t0
    from lachesis_hip import tools
    qa, qb = tools.fc_queries(dag.lamport[:done], fc_n, seed=3)
    t1 = time.perf_counter()
    o.forkless_cause_batch(qa, qb)
    t_fc = time.perf_counter() - t1
    # FC over all host cores given to this job (OpenMP)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)   # the job's CPU share
    qa2, qb2 = tools.fc_queries(dag.lamport[:done], fc_n * threads, seed=4)
    t2 = time.perf_counter()
    o.forkless_cause_batch_mt(qa2, qb2, threads)
    t_mt = time.perf_counter() - t2
    return done, t_add, fc_n, t_fc, (len(qa2), t_mt, threads)


LAT_KINDS = ["add1_async", "add1_sync", "build1_add_drop_sync", "antichain_add_sync", "add1024_sync", "fc1", "fc667",
             "get_hb", "get_la", "get_merged_hb", "get_merged_hb_x64"]


def latency_leg(lx, dag, weights, device, history=200_000, reps=2000, feed=1_000_000):
    """Per-call latency of the drop-in boundary at the granularity the
    reference's callers use it (abft/indexed_lachesis.go:53-82 one Add per
    event, Build = Add + DropNotFlushed; abft/event_processing.go:149-161 one
    ForklessCause per (event, root); abft/lachesis.go:57 GetMergedHighestBefore
    per event), timed from native code over the C ABI (tools/lx_latency.cpp:
    wall clock around each call, p50/p99/mean in us) on an epoch of the bench
    DAG with `history` events already indexed; then C3 events/s when the DAG is
    fed antichain by antichain (events re-ordered by topological level, one
    lx_add_batch + lx_flush per level), directly and through the level batcher."""
    import ctypes
    import numpy as np
    path = os.path.join(PKG, "build", "liblx_bench.so")
    L = ctypes.CDLL(path)
    f = L.lx_bench_latency
    f.restype = ctypes.c_int
    u32p, u64p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)
    f.argtypes = [ctypes.c_int, ctypes.c_uint32, u32p, ctypes.c_uint64, u32p, u32p, u64p, u32p, ctypes.c_uint64,
                  ctypes.c_uint32, ctypes.c_uint64, ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, ctypes.c_uint32]
    n = min(len(dag), history + 2 * feed + 600_000)
    w = np.ascontiguousarray(weights, dtype=np.uint32)
    cr = np.ascontiguousarray(dag.creator[:n])
    sq = np.ascontiguousarray(dag.seq[:n])
    po = np.ascontiguousarray(dag.poff[:n + 1])
    out = (ctypes.c_double * 128)()
    err = ctypes.create_string_buffer(512)
    rc = f(device, len(w), w.ctypes.data_as(u32p), n, cr.ctypes.data_as(u32p), sq.ctypes.data_as(u32p),
           po.ctypes.data_as(u64p), dag.par.ctypes.data_as(u32p), history, reps, feed, out, err, 512)
    if rc != 0:
        raise RuntimeError("lx_bench_latency: " + err.value.decode())
    res = {"unit": "us", "history_events": history, "reps": reps,
           "calls": {k: {"p50": out[3 * i], "p99": out[3 * i + 1], "mean": out[3 * i + 2], "p999": out[48 + 4 * i],
                         "max": out[48 + 4 * i + 1], "first_call": out[48 + 4 * i + 2], "n": int(out[48 + 4 * i + 3])}
                     for i, k in enumerate(LAT_KINDS)},
           "add1024_split": {"add_call_p50": out[96], "add_call_p99": out[97], "sync_p50": out[98], "sync_p99": out[99]},
           "antichain_fed_events_per_sec": out[33], "batcher_fed_events_per_sec": out[36],
           "fc_pair_cached": {"first_call_miss": {"p50": out[40], "p99": out[41], "mean": out[42]},
                              "next_calls_hit": {"p50": out[43], "p99": out[44], "mean": out[45]}},
           "fed_events": int(out[34]), "fed_levels": int(out[35]), "mean_events_per_level": out[37],
           "note": "add1_async = host time of lx_add_batch(n=1) + lx_flush (the launch is not waited for); "
                   "*_sync include lx_sync (completion); fc/getters are synchronous calls; fc1 / fc667 = "
                   "lx_forkless_cause_batch (no cache); fc_pair_cached = lx_forkless_cause (the drop-in path); "
                   "each kind's first call (one-time setup: pinned buffers, the row server's stream, a kernel's "
                   "first launch) is first_call, then 3 untimed calls, then the timed ones"}
    return res


def _bench_lib():
    import ctypes
    L = ctypes.CDLL(os.path.join(PKG, "build", "liblx_bench.so"))
    u32p, u64p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)
    L.lx_bench_feed.restype = ctypes.c_int
    L.lx_bench_feed.argtypes = [ctypes.c_int, ctypes.c_uint32, u32p, ctypes.c_uint64, u32p, u32p, u64p, u32p,
                                ctypes.c_uint32, ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, ctypes.c_uint32]
    L.lx_bench_feed_levels.restype = ctypes.c_int
    L.lx_bench_feed_levels.argtypes = [ctypes.c_int, ctypes.c_uint32, u32p, ctypes.c_uint64, u32p, u32p, u64p, u32p,
                                       ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                       ctypes.c_char_p, ctypes.c_uint32]
    return L


def feed_levels(dag, weights, device, history=200_000, feed=1_000_000):
    """C3 fed antichain by antichain (the DAG renumbered by topological level,
    one lx_add_batch + lx_flush per level; or each level pushed into and popped
    from lx_batcher first), after 100 untimed levels; one lx_sync at the end
    (tools/lx_latency.cpp lx_bench_feed_levels).  Host seconds split between
    the Adds and the batcher."""
    import ctypes
    import numpy as np
    L = _bench_lib()
    u32p, u64p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)
    w = np.ascontiguousarray(weights, dtype=np.uint32)
    res = {}
    for mode, name in ((0, "direct"), (1, "batcher")):
        out = (ctypes.c_double * 8)()
        err = ctypes.create_string_buffer(512)
        rc = L.lx_bench_feed_levels(device, len(w), w.ctypes.data_as(u32p), len(dag), dag.creator.ctypes.data_as(u32p),
                                    dag.seq.ctypes.data_as(u32p), dag.poff.ctypes.data_as(u64p),
                                    dag.par.ctypes.data_as(u32p), history, feed, mode, out, err, 512)
        if rc != 0:
            raise RuntimeError("lx_bench_feed_levels: " + err.value.decode())
        res[name] = {"events_per_sec": out[0], "events": int(out[1]), "levels": int(out[2]), "add_s": out[3],
                     "batcher_s": out[4], "final_sync_s": out[5]}
    return res


def qi_leg(dag, weights, device, want_cpu, history=20_000, reps=2000, every=50, cands=64):
    """The emitter's QuorumIndexer at V=1000 (emitter/ancestor/quorum_indexer.go:
    86-136) on the HIP index, per call as the emitter makes them
    (tools/lx_latency.cpp lx_bench_qi): after `history` events, each next event
    is Added and handed to ProcessEvent alone; every `every`-th event
    GetMetricOf for `cands` candidate parents (medians recomputed lazily, as
    recacheState does).  The CPU line is the numpy port
    (oracle/emitter_oracle.DenseQuorumIndexerNp over the C restatement's
    merged rows) making the same calls; the last metric batch must agree."""
    import ctypes
    import numpy as np
    L = _bench_lib()
    u32p, u64p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)
    L.lx_bench_qi.restype = ctypes.c_int
    L.lx_bench_qi.argtypes = [ctypes.c_int, ctypes.c_uint32, u32p, ctypes.c_uint64, u32p, u32p, u64p, u32p,
                              ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                              ctypes.POINTER(ctypes.c_double), u64p, ctypes.c_char_p, ctypes.c_uint32]
    w = np.ascontiguousarray(weights, dtype=np.uint32)
    out = (ctypes.c_double * 8)()
    mo = np.zeros(cands, dtype=np.uint64)
    err = ctypes.create_string_buffer(512)
    rc = L.lx_bench_qi(device, len(w), w.ctypes.data_as(u32p), len(dag), dag.creator.ctypes.data_as(u32p),
                       dag.seq.ctypes.data_as(u32p), dag.poff.ctypes.data_as(u64p), dag.par.ctypes.data_as(u32p),
                       history, reps, every, cands, out, mo.ctypes.data_as(u64p), err, 512)
    if rc != 0:
        raise RuntimeError("lx_bench_qi: " + err.value.decode())
    nlast = int(out[6])
    res = {"unit": "us", "validators": len(w), "history_events": history, "events": reps, "metric_every": every,
           "candidates": cands,
           "process_event": {"p50": out[0], "p99": out[1], "mean": out[2]},
           "metric_batch": {"p50": out[3], "p99": out[4], "mean": out[5]}}
    if want_cpu:
        from oracle import corc
        from oracle.emitter_oracle import DenseQuorumIndexerNp
        n = history + reps
        ix = corc.OracleIndex(weights)
        assert ix.add_batch(dag.creator[:n], dag.seq[:n], dag.poff[:n + 1], dag.par) == -1
        ix.flush()
        qi = DenseQuorumIndexerNp(weights, ix, cap=2)
        for e in range(history):
            qi.process_event(e, int(dag.creator[e]), dag.creator[e] == 0)
        last = {}
        for e in range(history):
            last[int(dag.creator[e])] = e
        tp, tm, got = [], [], None
        for r in range(reps):
            e = history + r
            last[int(dag.creator[e])] = e
            t0 = time.perf_counter()
            qi.process_event(e, int(dag.creator[e]), dag.creator[e] == 0)
            tp.append(time.perf_counter() - t0)
            if every and r % every == every - 1:
                cv = [last[c] for c in range(len(w)) if c in last][:cands]
                t1 = time.perf_counter()
                got = qi.metric_of(cv)
                tm.append(time.perf_counter() - t1)
        assert got is not None and np.array_equal(got, mo[:nlast]), "QuorumIndexer metric mismatch vs the CPU port"
        res["metrics_checked"] = nlast
        res["cpu_baseline"] = {"kind": "port", "cores": 1,
                               "process_event_mean_us": float(np.mean(tp)) * 1e6,
                               "metric_batch_mean_us": float(np.mean(tm)) * 1e6,
                               "sample": "the same %d ProcessEvent and %d GetMetricOf batches on the numpy port "
                                         "over oracle.c merged rows (same DAG prefix, already indexed)"
                                         % (len(tp), len(tm))}
    return res


def feed_rate(dag, weights, device, batch):
    """Events/s adding the DAG in its Add order in batches of `batch` events
    (lx_add_batch + lx_flush each; 1 = per-event Add), tools/lx_latency.cpp."""
    import ctypes
    import numpy as np
    L = _bench_lib()
    u32p, u64p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64)
    w = np.ascontiguousarray(weights, dtype=np.uint32)
    out = (ctypes.c_double * 4)()
    err = ctypes.create_string_buffer(512)
    rc = L.lx_bench_feed(device, len(w), w.ctypes.data_as(u32p), len(dag), dag.creator.ctypes.data_as(u32p),
                         dag.seq.ctypes.data_as(u32p), dag.poff.ctypes.data_as(u64p), dag.par.ctypes.data_as(u32p),
                         batch, out, err, 512)
    if rc != 0:
        raise RuntimeError("lx_bench_feed: " + err.value.decode())
    return out[0], {"seconds": out[1], "host_calls_s": out[2], "final_sync_s": out[3]}


def config_leg(lx, name, steps, warmup, device, want_cpu, cpu_budget, fc_n=1 << 22):
    """Secondary line for another BASELINE config: the same
    index step (reset + one lx_add_batch_dev of the epoch) and FC step as the
    headline, with the k_fc roofline (8 B per branch per query) and the C
    restatement's CPU baseline on a bounded sample; C1 also adds its events
    one at a time (the reference's per-event Add)."""
    import numpy as np
    import torch
    V, epv, P, ch, fk, wkind = CONFIGS[name]
    weights = weights_for(V, wkind)
    dag = lx.tools.gen_dag(V, epv, P, ch, fk, seed=1)
    N = len(dag)
    dev = torch.device("cuda", device)
    to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)
    d_c, d_s, d_p = to_dev(dag.creator), to_dev(dag.seq), to_dev(dag.par)
    d_o = to_dev(dag.poff.astype(np.uint32))
    qa, qb = lx.tools.fc_queries(dag.lamport, fc_n, window=64, seed=7)
    d_qa, d_qb = to_dev(qa), to_dev(qb)
    d_out = torch.empty(fc_n, dtype=torch.uint8, device=dev)
    ix = lx.Index(device=device, event_capacity=N)

    def step():
        ix.reset(weights)
        ix.add_batch_dev(N, d_c.data_ptr(), d_s.data_ptr(), d_o.data_ptr(), d_p.data_ptr())
        return ix.last_stats()["ms_index"]

    for _ in range(warmup):
        step()
    ix.sync()
    t0 = time.perf_counter()
    kms = [step() for _ in range(steps)]
    ix.sync()
    t_idx = (time.perf_counter() - t0) / steps
    _, _, _, sp = ix.device_planes()
    st = torch.cuda.ExternalStream(sp, device=dev)
    for _ in range(warmup):
        ix.forkless_cause_batch_dev(fc_n, d_qa.data_ptr(), d_qb.data_ptr(), d_out.data_ptr())
    ix.sync()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t1 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(st)
        ix.forkless_cause_batch_dev(fc_n, d_qa.data_ptr(), d_qb.data_ptr(), d_out.data_ptr())
        e1.record(st)
    ix.sync()
    t_fc = (time.perf_counter() - t1) / steps
    fc_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    B = ix.num_branches()
    o = None
    if want_cpu:
        from oracle import corc
        o = corc.OracleIndex(weights)
    got = d_out[:4096].cpu().numpy()
    ix.close()
    fc_bytes = 8.0 * B * fc_n
    p_mean = float(len(dag.par)) / N
    res = {"workload": "%s: V=%d, %d events (%d/validator), P=%d, %s stakes, cheaters=%d x %d forks; FC 2^%d queries"
                       % (name, V, N, epv, P, wkind, ch, fk, int(np.log2(fc_n))),
           "events": N, "branches": B, "events_per_sec": N / t_idx, "ms_per_step": t_idx * 1e3,
           "index_kernel_ms": float(np.mean(kms)), "fc_queries_per_sec": fc_n / t_fc,
           "roofline": {"bound": "hbm", "kernel": "k_fc<%s>" % ("forks" if B > V else "no forks"),
                        "achieved": fc_bytes / (fc_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": fc_bytes / (fc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                        "algorithmic_bytes_per_launch": fc_bytes, "kernel_ms": fc_ms},
           "roofline_index": {"kernel": "k_index", "algorithmic_bytes_per_launch":
                              ((p_mean + 1) * 4 * B + 4 * B + 8) * N, "kernel_ms": float(np.mean(kms))}}
    if name == "c1":
        res["per_event_add_events_per_sec"], res["per_event_add_split"] = feed_rate(dag, weights, device, 1)
    if o is not None:
        t2 = time.perf_counter()
        done = 0
        while done < N and time.perf_counter() - t2 < cpu_budget:
            hi = min(N, done + 500)
            assert o.add_batch(dag.creator[done:hi], dag.seq[done:hi], dag.poff[done:hi + 1], dag.par) == -1
            done = hi
        t_add = time.perf_counter() - t2
        nq = 100_000
        qa2, qb2 = lx.tools.fc_queries(dag.lamport[:done], nq, seed=3)
        t3 = time.perf_counter()
        want = o.forkless_cause_batch(qa2, qb2)
        t_q = time.perf_counter() - t3
        if done == N:   # whole epoch indexed on the CPU: this run's GPU answers must match
            assert np.array_equal(got, o.forkless_cause_batch(qa[:4096], qb[:4096]))
        res["cpu_baseline"] = {"value": done / t_add, "unit": "events/s", "cores": 1, "kind": "port",
                               "sample": "first %d events indexed by the C restatement in %.1fs; FC %d queries in %.2fs"
                                         % (done, t_add, nq, t_q), "fc_value": nq / t_q}
        assert want.max() <= 1
    return res


ABFT_CONFIG = ("c5", 1000, 50, 10, "zipf")   # BASELINE configs[4]: V, events/validator, parents, stakes


VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # 78.6 T lane-ops/s (2-cycle wave64 VALU ops)
# k_root_fc16 issues only v_pk_sub_u16, v_pk_min_u16 and v_dot2_u32_u16, each 4
# shader cycles per wave-instruction on a SIMD (scripts/probes/valu_rate.hip,
# profiles/r06/abft/valu_rate.json: 4.19-4.22 measured against 2.31 for
# v_add_u32 / v_fma_f32 in the same harness), so its issue peak is half
VALU_PEAK_4CYC_TOPS = 256 * 4 * 64 / 4 * 2.4e9 / 1e12   # 39.3 T lane-ops/s


def abft_leg(lx, steps, warmup, device, cpu_budget, want_cpu):
    """BASELINE configs[4]: full abft.IndexedLachesis.Process over one epoch --
    index Add, frames and roots (batched root ForklessCause tiles), election
    (vote kernels), blocks (cheaters, confirmation DFS) -- through
    lx_abft_process_batch with the events' claimed frames.  A step = reset +
    the whole 50k-event epoch in one batch (host arrays in, so the PCIe copy
    of the batch, ~44 B/event, is inside the step)."""
    import numpy as np
    name, V, epv, P, wkind = ABFT_CONFIG
    weights = weights_for(V, wkind)
    dag = lx.tools.gen_dag(V, epv, P, 0, 0, seed=1)
    N = len(dag)
    # the blocks come back through the library's block log (the confirmation
    # DFS runs as under a BeginBlock callback; no Python callback per block)
    lch = lx.abft.DenseLachesis(weights, device=device, event_capacity=N, apply_events=False, block_log=True)
    rc, consumed, frames = lch.process_batch(dag.creator, dag.seq, dag.poff, dag.par)   # Build-path frames
    assert rc == 0 and consumed == N
    claimed = frames.copy()
    n_blocks = len(lch.blocks)

    def step():
        lch.L.lx_abft_reset(lch.h, 1, V, np.ascontiguousarray(weights, dtype=np.uint32).ctypes.data_as(
            lx.capi.u32p))
        lch.blocks = []
        rc, consumed, out = lch.process_batch(dag.creator, dag.seq, dag.poff, dag.par, claimed)
        assert rc == 0 and consumed == N and len(lch.blocks) == n_blocks
        return lch.last_stats()

    for _ in range(warmup):
        step()
    t0 = time.perf_counter()
    stats = [step() for _ in range(steps)]
    dt = (time.perf_counter() - t0) / steps
    st = {k: float(np.mean([s[k] for s in stats])) for k in stats[0]}
    res = {"workload": "%s: V=%d, %d events (%d/validator), P=%d, %s stakes, no cheaters; one epoch per step, "
                       "claimed frames checked" % (name, V, N, epv, P, wkind),
           "events": N, "events_per_sec": N / dt, "ms_per_step": dt * 1e3, "blocks_decided": n_blocks,
           "max_frame": int(claimed.max()), "phase_ms": {k: st[k] for k in ("ms_index", "ms_frames", "ms_election", "ms_blocks")},
           "frame_steps": st["frame_steps"], "fc_launches": st["fc_launches"], "vote_launches": st["vote_launches"],
           "root_fc_pairs": st["fc_pairs"]}
    # The root-FC kernels are VALU-bound integer work.  k_root_fc (32-bit):
    # per (pair, column) one compare and one select, and one 3-input add per
    # two columns (gfx950 ISA of the inner loop: v_cmp_lt_u32 + v_cndmask_b32
    # per column, v_add3_u32 per two) = 2.5 lane-ops.  k_root_fc16 (fork-free
    # epochs with 16-bit seqs, the C5 case): per pair and two columns one
    # v_pk_sub_u16 (clamp), one v_pk_min_u16 and one v_dot2_u32_u16 per weight
    # half = 1.5 lane-ops per column, 2 in 32-column chunks holding a weight >=
    # 2^16.  fc_lane_ops counts what the launches issued (padded columns);
    # peak = 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md:
    # wave64 VALU op = 2 cycles on a SIMD) for k_root_fc; half that for
    # k_root_fc16, whose three instructions all take 4 cycles (measured).
    if st["ms_root_fc_gpu"] > 0:
        sec = st["ms_root_fc_gpu"] * 1e-3
        pc = st["fc_pair_cols"] / sec
        ach = st["fc_lane_ops"] / sec / 1e12
        opc = st["fc_lane_ops"] / max(st["fc_pair_cols"], 1)
        packed = opc < 2.4   # 1.5-2 lane-ops per pair-column: k_root_fc16 ran
        peak = VALU_PEAK_4CYC_TOPS if packed else VALU_PEAK_TOPS
        res["roofline_root_fc"] = {"bound": "valu", "kernel": "k_root_fc16" if packed else "k_root_fc",
                                   "achieved": ach, "peak": peak,
                                   "unit": "T int32 lane-ops/s", "frac": ach / peak,
                                   "pair_cols_per_s": pc,
                                   "ops_per_pair_col": st["fc_lane_ops"] / max(st["fc_pair_cols"], 1),
                                   "ms_per_epoch": st["ms_root_fc_gpu"]}
    lch.close()
    if want_cpu:
        from oracle import corc
        n = min(N, 3000)
        o = corc.AbftOracle(weights)
        t1 = time.perf_counter()
        done = 0
        while done < n and time.perf_counter() - t1 < cpu_budget:
            hi = min(n, done + 250)
            rc, c, _ = o.process_batch(dag.creator[done:hi], dag.seq[done:hi], dag.poff[done:hi + 1], dag.par,
                                       claimed[done:hi])
            assert rc == 0 and c == hi - done
            done = hi
        t_cpu = time.perf_counter() - t1
        res["cpu_baseline"] = {
            "value": done / t_cpu, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": "first %d events of the same epoch through the C abft restatement (oracle/csrc/abft_oracle.c "
                      "over oracle.c: per-event Add with DFS LowestAfter, calcFrameIdx with early exit, per-root "
                      "election) in %.1fs" % (done, t_cpu)}
    return res


def dropin_leg(lx, device, want_cpu, cpu_events=4000):
    """BASELINE configs[4] through the UNCHANGED caller: IndexedLachesis.Process
    restated in C++ (tools/lx_dropin.cpp) makes the reference's index calls one
    by one -- Add per event, ForklessCause per (event, root) pair from
    calcFrameIdx, the election and processKnownRoots, Flush, DropNotFlushed,
    GetMergedHighestBefore per decided frame (abft/indexed_lachesis.go:69-82,
    abft/event_processing.go:102-189, abft/election/election.go:101-123) --
    on the HIP library's C ABI (lx_forkless_cause and its result cache, the
    path a cgo shim binds).  The same driver replaying the recorded answers
    gives the caller's own time; the CPU baseline is the same driver over the
    C restatement of the index behind the reference's ForklessCause LRU
    (20000 pairs, vecfc/index.go:52-61) on a prefix of the epoch."""
    import numpy as np
    from lachesis_hip import dropin
    name, V, epv, P, wkind = ABFT_CONFIG
    weights = weights_for(V, wkind)
    dag = lx.tools.gen_dag(V, epv, P, 0, 0, seed=1)
    N = len(dag)
    lch = lx.abft.DenseLachesis(weights, device=device, event_capacity=N, apply_events=False)
    rc, consumed, claimed = lch.process_batch(dag.creator, dag.seq, dag.poff, dag.par)   # claimed frames (Build)
    assert rc == 0 and consumed == N
    blocks = [(int(b[1]), int(b[2])) for b in lch.blocks]
    lch.close()
    rec = dropin.Recording(60_000_000, V)
    r = dropin.replay(dag, weights, claimed, kind="hip", device=device, record=rec)
    assert np.array_equal(r["frames"], claimed)
    assert [(int(f), int(a)) for f, a in zip(r["block_frame"], r["block_atropos"])] == blocks
    q = dropin.replay(dag, weights, claimed, kind="recorded", record=rec)
    assert q["trace_hash"] == r["trace_hash"]
    st = r["fc_cache"]
    t_idx = r["seconds"] - q["seconds"]
    res = {"workload": "%s: V=%d, %d events, P=%d, %s stakes; IndexedLachesis.Process per event with the claimed "
                       "frames, every index call made one at a time as the reference's caller makes it" % (
                           name, V, N, P, wkind),
           "events": N, "events_per_sec": N / r["seconds"], "ms_per_epoch": r["seconds"] * 1e3,
           "caller_ms": q["seconds"] * 1e3, "index_ms": t_idx * 1e3, "index_events_per_sec": N / t_idx,
           "add_ms": r["add_seconds"] * 1e3,
           "fc_calls": r["fc_calls"], "fc_calls_per_sec": r["fc_calls"] / r["seconds"],
           "fc_cache_hit_rate": st["hits"] / max(1, st["calls"]), "fc_row_fills": st["row_fills"],
           "fc_tile_fills": st["tile_fills"], "fc_pairs_evaluated": st["pairs"], "fc_cache_slots": st["slots"],
           "blocks": len(blocks), "trace_hash": str(r["trace_hash"]),
           "note": "caller_ms = the same driver replaying the recorded answers without an index; "
                   "index_ms = the rest (Add, ForklessCause incl. cache hits, Flush, DropNotFlushed, merged HB)"}
    if want_cpu:
        from oracle import corc
        ix = corc.OracleIndex(weights)
        c = dropin.replay(dag, weights, claimed, kind="cpu", cpu=ix.c_funcs(), lru_pairs=20000, max_events=cpu_events)
        assert np.array_equal(c["frames"], claimed[:cpu_events])
        g = float(r["checkpoint_s"][cpu_events // 1000 - 1])
        res["cpu_baseline"] = {
            "value": c["events"] / c["seconds"], "unit": "events/s", "cores": 1, "kind": "port",
            "sample": "first %d events of the epoch through the same caller driver over the C restatement of the "
                      "index (oracle/csrc/oracle.c: per-event Add with DFS LowestAfter) behind the reference's "
                      "ForklessCause LRU of 20000 pairs, in %.1fs (%d ForklessCause calls, %d LRU hits)"
                      % (c["events"], c["seconds"], c["fc_calls"], c["lru_hits"]),
            "gpu_seconds_same_prefix": g, "speedup_same_prefix": c["seconds"] / g}
    return res


def smi_json(argv, timeout=10):
    """amd-smi (read-only queries) as JSON, or None when it is absent or fails."""
    import subprocess
    try:
        r = subprocess.run(["amd-smi"] + argv + ["--json"], capture_output=True, text=True, timeout=timeout)
        return json.loads(r.stdout)
    except Exception:
        return None


def power_probe(step, seconds=2.5):
    """The board's socket power, GFX clocks and hotspot / HBM temperatures (amd-smi metric, sampled by a
    host thread) while the index step runs back to back for ~`seconds`,
    untimed, after the timed steps; and the socket power limit.  The walk's
    time is a fixed number of shader cycles over the clock the box gives it
    (walk_clock), and the walk draws within ~15 % of the limit:
    these samples say what the box did with its power budget."""
    import threading

    import numpy as np
    lim = smi_json(["static", "--limit"])
    samples, stop = [], threading.Event()

    def gpu0(d):
        return d["gpu_data"][0] if isinstance(d, dict) else d[0]

    def sampler():
        while not stop.is_set():
            d = smi_json(["metric", "-p", "-c", "-t"])
            try:
                g = gpu0(d)
                clk = [g["clock"][k]["clk"]["value"] for k in g["clock"] if k.startswith("gfx")]
                t = g.get("temperature", {})
                tv = lambda k: float(t[k]["value"]) if isinstance(t.get(k), dict) else float("nan")
                samples.append((time.time(), float(g["power"]["socket_power"]["value"]), float(np.mean(clk)),
                                tv("hotspot"), tv("mem")))
            except Exception:
                time.sleep(0.2)

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    t_start = time.time()
    steps = 0
    while time.time() < t_start + seconds:
        step()
        steps += 1
    t_end = time.time()
    stop.set()
    th.join(timeout=15)
    s = [x for x in samples if t_start + 0.3 <= x[0] <= t_end]
    try:
        limit_w = float(gpu0(lim)["limit"]["ppt0"]["socket_power_limit"]["value"])
    except Exception:
        limit_w = None
    if not s:
        return {"samples": 0, "socket_power_limit_w": limit_w, "note": "amd-smi gave no samples"}
    return {"samples": len(s), "steps": steps, "socket_power_w_mean": float(np.mean([x[1] for x in s])),
            "socket_power_w_max": float(max(x[1] for x in s)), "smi_gfx_mhz_mean": float(np.mean([x[2] for x in s])),
            "hotspot_c_max": max((x[3] for x in s if x[3] == x[3]), default=None),
            "hbm_c_max": max((x[4] for x in s if x[4] == x[4]), default=None),
            "socket_power_limit_w": limit_w,
            "source": "amd-smi metric -p -c (read-only) sampled during back-to-back index steps after the timed ones"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--fc-queries", type=int, default=1 << 24)
    ap.add_argument("--batch", type=int, default=0, help="events per lx_add_batch_dev call (0 = whole epoch)")
    ap.add_argument("--order", default="add", choices=["add", "level"],
                    help="event order of the batch: generator (Add) order, or level order as a "
                         "level-synchronous batcher releases the epoch (same DAG, renumbered)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-power", action="store_true",
                    help="skip the untimed amd-smi power / clock samples beside back-to-back index steps")
    ap.add_argument("--mode", default="rowseg", choices=["replica", "shard", "rowseg"],
                    help="N > 1: rowseg = the epoch split into N Add-order row segments, one walk per rank "
                         "(DESIGN.md 6b, the default); shard = column shards; replica = independent epochs")
    ap.add_argument("--no-abft", action="store_true", help="skip the configs[4] abft leg")
    ap.add_argument("--no-dropin", action="store_true", help="skip the configs[4] drop-in (unchanged caller) leg")
    ap.add_argument("--no-latency", action="store_true", help="skip the per-call latency / antichain-fed leg")
    ap.add_argument("--no-configs", action="store_true", help="skip the secondary C1/C2/C4 lines")
    ap.add_argument("--no-colshard", action="store_true",
                    help="N > 1 row segments: skip the column-shard leg of the same run (BASELINE configs[2])")
    ap.add_argument("--segments", type=int, default=0,
                    help="single GPU: walk the epoch as G Add-order segments + fix-up (option segments, the "
                         "per-rank work of the row-segment multi-GPU mode timed segment by segment)")
    ap.add_argument("--shard-solo", type=int, default=0,
                    help="diagnostic: time rank 0 of a G-way column shard alone on this GPU (its index walk, "
                         "the packing of its outgoing LowestAfter blocks, its partial FC); no collectives")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("LX_DIST_BACKEND", "nccl")
    rowseg = args.mode == "rowseg" and world > 1
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())   # rehearsal: ranks may share a GPU
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import lachesis_hip as lx

    V, epv, P_, cheaters, forks, wkind = CONFIGS[args.config]
    weights = weights_for(V, wkind)
    t_gen = time.perf_counter()
    dag = lx.tools.gen_dag(V, epv, P_, cheaters, forks, seed=1)
    if args.order == "level":
        dag = lx.tools.level_order(dag)
    # every rank asks 2^k queries of the same shape (a uniform over the epoch, b
    # within 64 Lamport of a); rank 0's are the N=1 set, the others draw their own
    qa, qb = lx.tools.fc_queries(dag.lamport, args.fc_queries, window=64, seed=7 + rank)
    t_gen = time.perf_counter() - t_gen
    N = len(dag)
    batch = args.batch if args.batch > 0 else N

    # inputs resident in HBM before timing
    def to_dev(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)

    d_creator = to_dev(dag.creator)
    d_seq = to_dev(dag.seq)
    d_par = to_dev(dag.par)
    batches = []
    for lo in range(0, N, batch):
        hi = min(N, lo + batch)
        off = (dag.poff[lo:hi + 1] - dag.poff[lo]).astype(np.uint32)
        batches.append((lo, hi, to_dev(off), int(dag.poff[lo])))
    d_qa, d_qb = to_dev(qa), to_dev(qb)
    d_out = torch.empty(args.fc_queries, dtype=torch.uint8, device=dev)

    shard = args.mode == "shard" and world > 1
    solo = args.shard_solo if world == 1 and args.shard_solo > 1 else 0

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def reduce_over_ranks(x, op):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=op)
        return float(t.item())

    def max_over_ranks(x):
        return reduce_over_ranks(x, dist.ReduceOp.MAX) if world > 1 else x

    def sum_over_ranks(x):
        return reduce_over_ranks(x, dist.ReduceOp.SUM) if world > 1 else x

    early_lanes = 32   # k_fc_early's lanes per query (lx_capi.cpp: option fc_early_lanes)

    def fc_bytes_read(nq, B, early):
        """Bytes k_fc reads for nq queries over rows of B branches: whole rows
        (8 B per branch: HB(a) 4 B + LA(b) 4 B) without the early exit; with it
        (k_fc_early, device counters: queries on the early path, of them the
        ones that read round 2, round 3, the rest; rounds of 4 x L columns, 4 x L
        more, 8 x L more, the rest, L = lanes per query) 2 x 4 x L x 4 B per
        query, as much again past round 1, twice that past round 2, the rest
        of both rows past round 3."""
        qe, q2, q3, qw = early
        row16 = ((B + 3) // 4) * 16
        r1 = 32.0 * early_lanes                       # bytes of round 1, both rows
        return (qe * r1 + q2 * r1 + q3 * 2 * r1 + qw * 2.0 * max(0, row16 - 64 * early_lanes) +
                (nq - qe) * 8.0 * B)

    def leg(kind):
        """One index + ForklessCause measurement: kind 'single' (one GPU, or
        one independent epoch per rank), 'solo' (rank 0 of a column shard
        alone), 'rowseg' (the epoch as Add-order row segments, one per rank),
        'shard' (the epoch's creator columns split over the ranks).  Warmup +
        K timed steps each, barrier + device sync on both sides, the max over
        ranks; k_fc timed by HIP events on the library's stream."""
        if kind == "solo":
            ix = lx.Index(device=local, event_capacity=N, shard_rank=0, shard_count=solo)
            d_part = torch.empty(args.fc_queries, dtype=torch.int32, device=dev)
        elif kind == "rowseg":
            ix = lx.Index(device=local, event_capacity=N, options={"seg_count": world, "seg_rank": rank})
            from lachesis_hip.rowseg import RowSegments
            rsx = RowSegments(ix, device=dev)
        elif kind == "shard":
            ix = lx.Index(device=local, event_capacity=N, shard_rank=rank, shard_count=world)
            from lachesis_hip.shard import ShardedIndex
            sx = ShardedIndex(ix, device=dev)
            d_part = torch.empty(args.fc_queries, dtype=torch.int32, device=dev)
        else:
            ix = lx.Index(device=local, event_capacity=N,
                          options={"segments": args.segments} if args.segments > 1 else None)
        st_x = []   # shard / rowseg: the exchange of each step, ms
        clk_log = []   # shader clock of each step's walk (lx_last_walk_clock)
        d_blk = None

        def index_step():
            nonlocal d_blk
            ix.reset(weights)
            st_idx = 0.0
            st_asg = 0.0
            for lo, hi, off, pbase in batches:
                ix.add_batch_dev(hi - lo, d_creator.data_ptr() + 4 * lo, d_seq.data_ptr() + 4 * lo,
                                 off.data_ptr(), d_par.data_ptr() + 4 * pbase)
                s = ix.last_stats()
                st_idx += s["ms_index"]
                st_asg += s["ms_assign"] + s["ms_marks"]
            clk_log.append(ix.walk_clock())
            if kind == "shard":
                tx = time.perf_counter()
                sx.exchange()
                st_x.append((time.perf_counter() - tx) * 1e3)
            if kind == "rowseg":
                tx = time.perf_counter()
                rsx.exchange()
                st_x.append((time.perf_counter() - tx) * 1e3)
            if kind == "solo":
                sizes = [ix.shard_block(0, t) for t in range(1, solo)]
                if d_blk is None:
                    d_blk = torch.empty(max(sizes + [1]), dtype=torch.int32, device=dev)
                for t in range(1, solo):
                    ix.la_pack_dev(t, d_blk.data_ptr())
                ix.la_own_dev()
            return st_idx, st_asg

        _, _, _, stream_ptr = ix.device_planes()
        lib_stream = torch.cuda.ExternalStream(stream_ptr, device=dev)
        kern_ms = []
        shard_q = []   # column shards: queries this rank's partial-sum launch summed per step
        proto_split = []   # row segments: (device steps, collectives) of the FC protocol per step, ms

        def fc_step(evs=None):
            if evs is not None:
                evs[0].record(lib_stream)
            if kind == "shard":
                # partial stake sums + all-reduce; shard 0 decides most queries
                # alone when the epoch allows (the early exit), the
                # other ranks sum the undecided ones only; the partial-sum
                # launches timed inside
                sx.forkless_cause_dev(d_qa, d_qb, d_out, timing=evs is not None)
            elif kind == "solo":
                ix.forkless_cause_partial_dev(args.fc_queries, d_qa.data_ptr(), d_qb.data_ptr(), d_part.data_ptr())
            elif kind == "rowseg":
                # any pair: queries to owner(a), remote LowestAfter rows to it,
                # answers back; k_fc itself timed inside
                rsx.forkless_cause_dev(args.fc_queries, d_qa, d_qb, d_out, timing=evs is not None)
            else:
                ix.forkless_cause_batch_dev(args.fc_queries, d_qa.data_ptr(), d_qb.data_ptr(), d_out.data_ptr())
            if evs is not None:
                evs[1].record(lib_stream)
            if evs is not None and kind == "rowseg":
                kern_ms.append(rsx.last_fc["kernel_ms"])
                proto_split.append((rsx.last_fc["device_ms"], rsx.last_fc["collective_ms"]))
            if evs is not None and kind == "shard":
                kern_ms.append(sx.last_fc["kernel_ms"])
                shard_q.append(sx.last_fc["partial_queries"])

        # ---- index: warmup + K timed steps
        for _ in range(args.warmup):
            index_step()
        barrier()
        t0 = time.perf_counter()
        k_index_ms, k_assign_ms = [], []
        for _ in range(args.steps):
            a, b = index_step()
            k_index_ms.append(a)
            k_assign_ms.append(b)
        barrier()
        t_index = max_over_ranks(time.perf_counter() - t0)
        clk_timed = list(clk_log[-args.steps:])
        power = None
        # (not under rocprofv3: its tool library would load into the amd-smi child too)
        profiled = any(k.startswith("ROCPROF") for k in os.environ)
        if kind == "single" and rank == 0 and world == 1 and not args.no_power and not profiled:
            power = power_probe(index_step)   # untimed, after the timed steps

        # ---- FC: warmup + K timed steps
        for _ in range(args.warmup):
            fc_step()
        ix.sync()
        barrier()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        ix.fc_early_rounds()            # reset (the warmup's launches)
        t1 = time.perf_counter()
        for k in range(args.steps):
            fc_step(evs[k])
        ix.sync()
        barrier()
        t_fc = max_over_ranks(time.perf_counter() - t1)
        step_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
        # k_fc's own time on this rank: the launch (single / shard partial), or
        # the launch inside the row-segment protocol (the rest is routing)
        fc_kernel_ms = float(np.mean(kern_ms)) if kind in ("rowseg", "shard") else step_ms
        early = ix.fc_early_rounds()
        # the queries this rank's k_fc answered per step: its own, or (row
        # segments) the ones routed to it as owner(a)
        nq = rsx.last_fc["answered"] if kind == "rowseg" else args.fc_queries
        if kind == "shard":
            # shard 0 sums every query, the others the undecided ones (early exit)
            nq = float(np.mean(shard_q))
        B = ix.num_branches()
        if kind in ("shard", "solo"):
            lo_c, hi_c = ix.shard_range(rank if kind == "shard" else 0)
            B = hi_c - lo_c                 # columns this rank streams (no forks in the bench DAG)
        fc_read = fc_bytes_read(nq * args.steps, B, early) / args.steps
        # per-GPU bandwidth over all ranks: sum of the ranks' bytes over the sum
        # of their k_fc times (equal to the rank's own at N = 1)
        fc_read_all = sum_over_ranks(fc_read)
        fc_ms_all = sum_over_ranks(fc_kernel_ms)
        early_all = [sum_over_ranks(float(x)) for x in early]
        nq_all = sum_over_ranks(float(nq))
        out = {"ix": ix, "kind": kind, "t_index": t_index, "t_fc": t_fc, "k_index_ms": k_index_ms,
               "k_assign_ms": k_assign_ms, "fc_kernel_ms": fc_kernel_ms, "fc_step_ms": step_ms, "B": B,
               "fc_read": fc_read, "fc_read_all": fc_read_all, "fc_achieved": fc_read_all / (fc_ms_all * 1e-3) / 1e9,
               "fc_kernel_ms_max": max_over_ranks(fc_kernel_ms),
               "early": {"queries": int(early_all[0]), "round2": int(early_all[1]), "round3": int(early_all[2]),
                         "whole_rows": int(early_all[3]), "answered": int(nq_all) * args.steps}
               if early_all[0] else None,
               "whole_row_bytes": 8.0 * B * nq, "st_x": st_x,
               "mem": ix.device_bytes(), "clk": clk_timed, "power": power}
        if kind == "rowseg":
            out["rsx"] = rsx
            out["proto_split"] = proto_split
        if kind == "shard":
            out["sx"] = sx
        return out

    def walk_clock_summary(clk):
        """The shader clock each timed step's walk ran at (lx_last_walk_clock:
        s_memtime cycles over s_memrealtime ticks of every workgroup's compute
        wave 0), and the walk's cycle count: the walk's time is a fixed number
        of cycles over the clock the box gives it."""
        c = [x for x in clk if x["mhz_median"] > 0]
        if not c:
            return None
        mhz = [x["mhz_median"] for x in c]
        mcyc = [x["mhz_median"] * x["walk_ms"] / 1e3 for x in c]
        xcd = [float(np.median([x["xcd_mhz"][k] for x in c])) for k in range(8)] if "xcd_mhz" in c[0] else None
        return {"mhz_median": float(np.median(mhz)), "mhz_min_step": float(min(mhz)), "mhz_max_step": float(max(mhz)),
                "mhz_by_xcd": xcd,
                "mhz_min_workgroup": float(min(x["mhz_min"] for x in c)),
                "walk_mcycles_median": float(np.median(mcyc)), "steps": len(c),
                "source": "lx_last_walk_clock after each timed step (median over workgroups per step)"}

    primary = "solo" if solo else "rowseg" if rowseg else "shard" if shard else "single"
    P = leg(primary)
    ix = P["ix"]
    k_index_ms, k_assign_ms, t_index, t_fc = P["k_index_ms"], P["k_assign_ms"], P["t_index"], P["t_fc"]
    fc_kernel_ms = P["fc_kernel_ms"]
    B = P["B"]

    # correctness spot check: this run's first 4096 ForklessCause answers
    # recomputed on the host from the index's own HighestBefore / LowestAfter
    # rows (reference byte layouts through the batched getters; row segments:
    # routed to their owners): sum of stakes over branches j with
    # 0 < LA(b)[j] <= HB(a)[j].Seq >= quorum (vecfc/forkless_cause.go:63-82;
    # the bench DAG has no forks)
    spot_n = 0
    if primary in ("single", "rowseg"):
        qa_s, qb_s = qa[:4096], qb[:4096]
        got = d_out[:4096].cpu().numpy()
        if primary == "rowseg":
            hb_rows = P["rsx"].get_rows(0, qa_s)
            la_rows = P["rsx"].get_rows(1, qb_s)
            hbs = np.stack([np.frombuffer(r, dtype=np.uint32)[0::2][:V] for r in hb_rows]).astype(np.int64)
            las = np.stack([np.frombuffer(r, dtype=np.uint32)[:V] for r in la_rows]).astype(np.int64)
        else:
            _, hbb = ix.rows_np(0, qa_s)
            _, lab = ix.rows_np(1, qb_s)
            hbs = hbb.view(np.uint32).reshape(len(qa_s), -1, 2)[:, :V, 0].astype(np.int64)
            las = lab.view(np.uint32).reshape(len(qb_s), -1)[:, :V].astype(np.int64)
        wv = np.asarray(weights, dtype=np.int64)
        stake = (((las > 0) & (las <= hbs)) * wv).sum(axis=1)
        want = (stake >= ix.quorum()).astype(np.uint8)
        assert np.array_equal(got, want), "ForklessCause spot check failed"
        spot_n = int(sum_over_ranks(float(len(got))))

    units = 1 if (shard or rowseg) else world          # shard / rowseg: the ranks share one epoch
    fc_units = 1 if shard else world                   # rowseg / replica: every rank asks its own 2^k queries
    events_per_s = N * args.steps * units / t_index
    fc_per_s = args.fc_queries * args.steps * fc_units / t_fc
    fc_bytes = P["whole_row_bytes"]
    # the ForklessCause kernel this run timed (its traffic figure must be its own)
    fc_kernel_name = "k_fc_early" if P["early"] else "k_fc"
    fc_read = P["fc_read"]
    fc_achieved = P["fc_achieved"]
    kidx = float(np.mean(k_index_ms))
    # index algorithmic bytes/event: (P+1)*4*B parent+own HB + 4*B LA + 8 B metadata
    p_mean = float(len(dag.par)) / N
    idx_bytes = ((p_mean + 1) * 4 * B + 4 * B + 8) * N
    idx_achieved = idx_bytes / (kidx * 1e-3) / 1e9

    traffic, traffic_src = measured_traffic(args.config, args.fc_queries)
    if shard or rowseg or solo or args.segments > 1 or args.batch:
        traffic = None   # the committed profile is of the default single-GPU run
    # the walk kernel this run timed: one k_index_segs launch when the batch was
    # walked as side-by-side segments, else k_index; the traffic
    # figure must be that kernel's own, or null
    walk_kernel = "k_index"
    if primary in ("single", "rowseg"):
        sg0 = ix.segment_stats()
        if primary == "rowseg" or (sg0["segments"] >= 2 and sg0["one_launch"]):
            walk_kernel = "k_index_segs"
    idx_traffic = traffic.get(walk_kernel) if traffic else None
    # compulsory HBM bytes of the walk: every HB and LA row this rank walks
    # written once at the plane's row stride (8 * stride bytes per event)
    plane_stride = ix.device_planes()[2]
    walked = N
    if primary == "rowseg":
        r0, r1 = ix.rowseg_range()
        walked = r1 - r0
    # (the row stride's padding columns are never written: 8 x B bytes per event
    # is the algorithmic write, 8 x stride the planes' footprint)
    idx_compulsory = 8.0 * B * walked
    idx_footprint = 8.0 * plane_stride * walked
    result = {
        "metric": "events indexed/sec + ForklessCause queries/sec at 1000 validators, 1/2/4/8 GPU",
        "value": events_per_s,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_index / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if (shard or rowseg) else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic tdag-structured DAG (splitmix64 seed 1), no forks",
        "config": {"workload": "%s: V=%d, %d events (%d/validator), P=%d, %s stakes, cheaters=%d; FC 2^%d queries, b within 64 Lamport of a"
                   % (args.config, V, N, epv, P_, wkind, cheaters, int(np.log2(args.fc_queries)), ),
                   "validators": V, "events": N, "parents": P_, "fc_queries": args.fc_queries,
                   "parallelism": ("solo-shard0-of-%d" % solo) if solo else
                                  ("colshard%d" if shard else "rowseg%d" if rowseg else "replica%d") % world,
                   "batch": batch},
        "fc_queries_per_sec": fc_per_s,
        "fc_ms_per_step": t_fc / args.steps * 1e3,
        "index_kernel_ms": kidx,
        "walk_clock": walk_clock_summary(P["clk"]),
        "walk_power": P["power"],
        "assign_and_marks_ms": float(np.mean(k_assign_ms)),
        "roofline": {"bound": "hbm", "kernel": fc_kernel_name, "achieved": fc_achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": fc_achieved / HBM_PEAK_GBS,
                     "bytes_read_per_launch": fc_read,
                     "early_exit": dict(P["early"], note="k_fc_early, device counters summed over the ranks: every "
                                        "query reads columns 0-127 of both rows (2 x 512 B), round2 of them 128-255 "
                                        "(2 x 512 B more), round3 256-511 (2 x 1 KB), whole_rows the rest; achieved = "
                                        "the ranks' bytes read / the sum of their k_fc times (per-GPU bandwidth); "
                                        "algorithmic_bytes_per_launch is SURVEY 8d's whole-row figure") if P["early"] else None,
                     "traffic": traffic[fc_kernel_name]["hbm_bytes"] if traffic and fc_kernel_name in traffic else None,
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": fc_bytes, "kernel_ms": fc_kernel_ms,
                     "kernel_ms_max_over_ranks": P["fc_kernel_ms_max"],
                     "whole_row_equiv_frac": fc_bytes / (fc_kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "whole_row_equiv_note": "SURVEY 8d's whole-row bytes (8 B per branch per query) over the kernel "
                                             "time: above 1 when the early exit skips most of the rows -- a rate of "
                                             "answered queries, not HBM use"},
        "roofline_index": {"bound": "latency (DAG depth x pass latency); hbm ceiling", "kernel": walk_kernel,
                           "achieved": idx_compulsory / (kidx * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": idx_compulsory / (kidx * 1e-3) / 1e9 / HBM_PEAK_GBS,
                           "traffic": idx_traffic["hbm_bytes"] if idx_traffic else None,
                           "traffic_kernel_names": idx_traffic.get("kernel_names") if idx_traffic else None,
                           "traffic_source": traffic_src if idx_traffic else None,
                           "compulsory_bytes_per_launch": idx_compulsory,
                           "plane_footprint_bytes_per_launch": idx_footprint, "kernel_ms": kidx,
                           "traffic_over_compulsory": (idx_traffic["hbm_bytes"] / idx_compulsory) if idx_traffic else None,
                           "compulsory_frac": idx_compulsory / (kidx * 1e-3) / 1e9 / HBM_PEAK_GBS,
                           "algorithmic_bytes_per_launch": idx_bytes,
                           "survey_formula_achieved": idx_achieved,
                           "survey_formula_frac": idx_achieved / HBM_PEAK_GBS,
                           "note": "achieved / frac: the compulsory HBM bytes (every HB and LA entry of the rows "
                                   "this rank walks written once, 8 x B bytes per event; the planes' padded stride "
                                   "in plane_footprint_bytes_per_launch) over the kernel time; "
                                   "survey_formula_* follow SURVEY 8d's per-event formula, which also counts every "
                                   "parent-row read -- the walker serves those from LDS, so it can exceed the HBM "
                                   "peak: the walk is latency-bound (DAG depth x pass latency)"},
        "device_bytes_per_rank": P["mem"],
        "host_gen_s": t_gen,
        "fc_spot_checked": spot_n,
    }
    if args.segments > 1 and world == 1:
        sg = ix.segment_stats()
        rest = sg["partial_ms"] + sg["la_ms"]
        sg["per_rank_estimate_ms"] = {"walk_max": max(sg["walk_ms"]), "fixup_share": rest / sg["segments"],
                                      "assign_and_marks": float(np.mean(k_assign_ms))}
        sg["note"] = ("one GPU, the segments walked one after another; a rank of the row-segment mode walks one "
                      "segment and does 1/G of the fix-up and LowestAfter passes")
        result["segments"] = sg
    if rowseg:
        sg = ix.segment_stats()
        rsx = P["rsx"]
        result["rowseg"] = {"rows": [int(x) for x in ix.rowseg_range()], "walk_ms": sg["walk_ms"][rank],
                            "partial_events": sg["partial"][rank], "partial_ms": sg["partial_ms"], "la_ms": sg["la_ms"],
                            "exchange_ms": float(np.mean(P["st_x"][-args.steps:])) if P["st_x"] else None,
                            "exchange": rsx.last, "fc": rsx.last_fc,
                            "fc_kernel_ms": fc_kernel_ms, "fc_protocol_ms": P["fc_step_ms"] - fc_kernel_ms,
                            "fc_step_ms": P["fc_step_ms"],
                            # the routing protocol split (rank 0, mean per step): the library's
                            # device steps (route, need, serve, store, unroute -- each completed
                            # on return) and the collectives between them (gloo staging on a
                            # shared-GPU rehearsal, RCCL over xGMI on the driver's node)
                            "fc_protocol_device_ms": float(np.mean([d for d, _ in P["proto_split"]]))
                            if P["proto_split"] else None,
                            "fc_protocol_collective_ms": float(np.mean([c for _, c in P["proto_split"]]))
                            if P["proto_split"] else None,
                            "device_bytes": P["mem"],
                            "note": "index step = assignment of every event + walk of the own segment + row "
                                    "requests, partial fix-up, LowestAfter pass and triples (exchange_ms), timed "
                                    "inside value; FC: every rank asks 2^k queries of the N=1 shape over the whole "
                                    "epoch, routed to owner(a) with the LowestAfter rows of remote b shipped to it "
                                    "(DESIGN.md 6c), timed inside fc_queries_per_sec; fc_kernel_ms = k_fc alone, "
                                    "fc_protocol_ms = the routing around it (rank 0)"}
    if shard or solo:
        sx = P.get("sx")
        wire = sorted(set(w for w in sx.last_wire[0] if w)) if shard and getattr(sx, "last_wire", None) else \
            [ix.shard_wire_bytes()]
        result["shard"] = {"columns": B, "wire_bytes_per_entry": wire,
                           "exchange_ms": float(np.mean(P["st_x"][-args.steps:])) if P["st_x"] else None,
                           "note": "index step = walk of own columns + LowestAfter all-to-all (timed inside value)"}
    if rowseg and not args.no_colshard:
        # BASELINE configs[2] as it names it: the same epoch column-sharded over
        # the same ranks (north_star (5)); the row-segment handle is freed first
        ix.close()
        C = leg("shard")
        cx = C["ix"]
        sx = C["sx"]
        result["colshard"] = {
            "events_per_sec": N * args.steps / C["t_index"], "ms_per_step": C["t_index"] / args.steps * 1e3,
            "fc_queries_per_sec": args.fc_queries * args.steps / C["t_fc"],
            "fc_ms_per_step": C["t_fc"] / args.steps * 1e3,
            "index_kernel_ms": float(np.mean(C["k_index_ms"])),
            "exchange_ms": float(np.mean(C["st_x"][-args.steps:])) if C["st_x"] else None,
            "columns": C["B"], "wire_bytes_per_entry": sorted(set(w for w in sx.last_wire[0] if w))
            if getattr(sx, "last_wire", None) else None,
            "roofline": {"bound": "hbm", "kernel": "k_fc partial (own columns)", "achieved": C["fc_achieved"],
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": C["fc_achieved"] / HBM_PEAK_GBS,
                         # summed over the ranks (as the row-segment leg counts), rank 0's own beside it
                         "bytes_read_per_launch": C["fc_read_all"], "bytes_read_per_launch_rank0": C["fc_read"],
                         "algorithmic_bytes_per_launch": C["whole_row_bytes"] * world,
                         "kernel_ms": C["fc_kernel_ms"], "kernel_ms_max_over_ranks": C["fc_kernel_ms_max"]},
            "device_bytes": C["mem"],
            "fc_early": {k: v for k, v in getattr(sx, "last_fc", {}).items() if k != "kernel_ms"},
            "scaling": "strong",
            "note": "the epoch's creator columns split over the ranks (DESIGN.md 6): each rank walks its columns of "
                    "every event, the LowestAfter all-to-all makes the shards FC-ready (inside events_per_sec), FC "
                    "sums the ranks' partial stakes with an all-reduce (inside fc_queries_per_sec); every rank "
                    "answers the same 2^k queries; shard 0 decides most of them alone on Zipf stakes (DESIGN.md 6f: the "
                    "others sum and all-reduce the undecided ones only), so bytes_read_per_launch sums rank 0's whole "
                    "pass and the others' undecided queries"}
        cx.close()
        ix = cx

    if not args.no_latency and world == 1 and not solo:
        ix.close()   # free the bench epoch's planes first
        result["latency"] = latency_leg(lx, dag, weights, local)
        fl = feed_levels(dag, weights, local)
        result["latency"]["antichain_fed_events_per_sec"] = fl["direct"]["events_per_sec"]
        result["latency"]["batcher_fed_events_per_sec"] = fl["batcher"]["events_per_sec"]
        result["latency"]["fed"] = fl
        result["quorum_indexer"] = qi_leg(dag, weights, local, rank == 0 and not args.no_cpu)

    if not args.no_configs and world == 1 and not solo:
        ix.close()
        want_cpu = rank == 0 and not args.no_cpu
        result["configs"] = {c: config_leg(lx, c, args.steps, args.warmup, local, want_cpu, min(args.cpu_budget, 4.0))
                             for c in ("c2", "c4", "c1")}

    if not args.no_abft:
        ab = abft_leg(lx, args.steps, args.warmup, local, args.cpu_budget, rank == 0 and world == 1 and not args.no_cpu)
        barrier()
        ab["ms_per_step"] = max_over_ranks(ab["ms_per_step"])   # replicas: one epoch per rank
        ab["events_per_sec"] = ab["events"] * world / (ab["ms_per_step"] * 1e-3)
        ab["parallelism"] = "replica%d" % world
        result["abft"] = ab

    if not args.no_dropin and world == 1 and not solo:
        result["dropin_c5"] = dropin_leg(lx, local, rank == 0 and not args.no_cpu)

    if rank == 0 and world == 1 and not args.no_cpu:     # the CPU baseline is an N=1 figure
        sample_max = N
        done, t_add, nq, t_q, (nq_mt, t_mt, thr) = cpu_baseline(dag, weights, sample_max, 200_000, args.cpu_budget)
        result["cpu_baseline"] = {
            "value": done / t_add, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": "first %d events of the same DAG indexed by the C restatement (oracle/csrc/oracle.c, -O2, "
                      "DFS LowestAfter, byte rows) in %.1fs; FC: %d queries over them in %.2fs" % (done, t_add, nq, t_q),
            "fc_value": nq / t_q, "fc_unit": "queries/s",
            "fc_value_mt": nq_mt / t_mt, "fc_threads": thr,
            "fc_sample_mt": "%d queries over the same prefix, OpenMP over queries, in %.2fs" % (nq_mt, t_mt),
            "fc_mt_note": "timed on the job's CPU share (OMP_NUM_THREADS=%d of %d logical CPUs on the box; the "
                          "pool's rule is to stay within the share)" % (thr, os.cpu_count() or 1),
            "host": "%s, %d logical cpus" % (platform.processor() or platform.machine(), os.cpu_count()),
        }
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""bench.py runs only on a GPU box: catch names a leg uses but never binds
(a NameError there costs a whole GPU call) with a static scan on the CPU."""

import ast
import builtins
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bound(node):
    out = set()
    for n in ast.walk(node):
        if isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            out.add(n.id)
        elif isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out.add(n.name)
        elif isinstance(n, ast.arg):
            out.add(n.arg)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            out.update((a.asname or a.name).split(".")[0] for a in n.names)
        elif isinstance(n, ast.ExceptHandler) and n.name:
            out.add(n.name)
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            out.update(n.names)
    return out


def test_bench_functions_bind_every_name_they_use():
    tree = ast.parse(open(os.path.join(ROOT, "bench.py"), encoding="utf-8").read())
    module = set(dir(builtins)) | {"__file__", "__name__"}
    for n in tree.body:
        module |= _bound(n) if not isinstance(n, (ast.FunctionDef, ast.ClassDef)) else {n.name}
    bad = []
    for f in tree.body:
        if not isinstance(f, ast.FunctionDef):
            continue
        known = module | _bound(f)
        for n in ast.walk(f):
            if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load) and n.id not in known:
                bad.append((f.name, n.id, n.lineno))
    assert not bad, bad


def test_multi_gpu_line_keys():
    """The committed N = 2 rehearsal line (two ranks over gloo on one GPU,
    scripts/rowseg_rehearsal.sh; the driver's N > 1 runs use RCCL) carries what
    the N > 1 bench line must: the k_fc roofline computed the N = 1 way from
    the early-exit counters summed over the ranks (frac < 1), k_fc timed
    apart from the routing protocol, per-rank device bytes, and both the
    row-segment block and the column-shard block of BASELINE configs[2]."""
    import glob
    import json
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "rehearsal", "rowseg_colshard_g2*.json")))
    assert files, "no committed N=2 rehearsal line"
    r = json.loads(open(files[-1]).read().strip().splitlines()[-1])
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "rowseg2"
    roof = r["roofline"]
    assert roof["early_exit"] is not None and roof["early_exit"]["queries"] > 0
    assert roof["early_exit"]["answered"] == 2 * r["steps"] * r["config"]["fc_queries"]
    assert 0 < roof["frac"] < 1 and roof["bytes_read_per_launch"] < roof["algorithmic_bytes_per_launch"]
    assert "whole_row_equiv_frac" in roof
    rs = r["rowseg"]
    assert rs["fc_kernel_ms"] > 0 and rs["fc_protocol_ms"] > 0
    # the protocol split into the library's device steps and the collectives (round 6)
    assert rs["fc_protocol_device_ms"] > 0 and rs["fc_protocol_collective_ms"] > 0
    assert rs["fc_protocol_device_ms"] + rs["fc_protocol_collective_ms"] <= rs["fc_protocol_ms"] * 1.05
    assert abs(rs["fc_kernel_ms"] + rs["fc_protocol_ms"] - rs["fc_step_ms"]) < 1e-6 * rs["fc_step_ms"] + 1e-9
    cs = r["colshard"]
    assert cs["events_per_sec"] > 0 and cs["fc_queries_per_sec"] > 0 and cs["exchange_ms"] is not None
    assert 0 < cs["roofline"]["frac"] < 1
    # a rank's planes hold its own rows: half of the epoch's at N = 2
    rows = rs["rows"][1] - rs["rows"][0]
    assert r["device_bytes_per_rank"]["planes"] <= 8 * rows * 1088 + 1

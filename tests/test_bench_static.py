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

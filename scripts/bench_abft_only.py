"""Runs only bench.py's abft leg (BASELINE configs[4]) -- for profiling."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lachesis-base_amd")]
import bench  # noqa: E402
import lachesis_hip as lx  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
print(json.dumps(bench.abft_leg(lx, steps, 1, 0, 0, False)))

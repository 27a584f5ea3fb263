"""Summarise scripts/probes/power_ab_r06.sh: per library, the socket power and
GFX clocks amd-smi sampled while the walks ran, beside the walks' own clock
record (lx_last_walk_clock) and cycle counts.  Usage: power_ab.py DIR [LIB...]"""
import json
import re
import sys

import numpy as np


def samples(path):
    txt = open(path).read()
    parts = re.split(r"^T (\d+\.\d+)\s*$", txt, flags=re.M)
    out = []
    for i in range(1, len(parts), 2):
        try:
            d = json.loads(parts[i + 1].strip())
        except ValueError:
            continue
        g = d["gpu_data"][0] if isinstance(d, dict) else d[0]
        p = g["power"]["socket_power"]["value"]
        clk = [g["clock"][k]["clk"]["value"] for k in g["clock"] if k.startswith("gfx")]
        out.append((float(parts[i]), float(p), float(np.mean(clk))))
    return out


def summary(d, lib):
    walks = [json.loads(x) for x in open("%s/walks_%s.jsonl" % (d, lib)) if x.strip()]
    w = walks[0]
    clk = w["clk"][1:]                      # the first walk of a handle pays first touches
    ms = w["walk_ms"][1:]
    t0, t1 = clk[0]["t"] - 0.05, clk[-1]["t"]
    s = [x for x in samples("%s/trace_%s.txt" % (d, lib)) if t0 <= x[0] <= t1]
    mhz = [c["mhz_median"] for c in clk]
    mcyc = [c["mhz_median"] * c["walk_ms"] / 1e3 for c in clk]
    return {"lib": lib, "walks": len(ms), "walk_ms_median": float(np.median(ms)), "walk_ms_max": float(max(ms)),
            "clock_mhz_median": float(np.median(mhz)), "wave0_mcycles_median": float(np.median(mcyc)),
            "power_w_samples": [x[1] for x in s], "power_w_mean": float(np.mean([x[1] for x in s])) if s else None,
            "smi_gfx_mhz_mean": float(np.mean([x[2] for x in s])) if s else None}


if __name__ == "__main__":
    d = sys.argv[1]
    libs = sys.argv[2:] or ["build", "build_pNOLA", "build_pNOHB"]
    for lib in libs:
        print(json.dumps(summary(d, lib)))

"""Durations of the headline launches in a rocprofv3 kernel trace of the
default bench run: k_index of configs[2] (the 10M-event C3 walk, the longest
k_index launches) and k_fc of the 2^24-query FC steps (the longest k_fc
launches), separated from the many small launches of the latency, level-fed
and drop-in legs that share the kernel names.

    python3 scripts/headline_kernels.py <dir with *kernel_trace.csv> > headline_kernels.json
"""
import csv
import glob
import json
import os
import sys


def main():
    root = sys.argv[1]
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    out = {"source": "rocprofv3 --kernel-trace of `python3 bench.py --no-cpu` (scripts/prof_round.sh)", "kernels": {}}
    # the C3 walk: one 4-column k_index, or (side-by-side segments)
    # one 8-column k_index_segs launch
    # (the C3 ForklessCause steps run the early-exit kernel since round 5)
    for key, match, min_ms in (("k_index_c3", "k_index", 20.0), ("k_fc_c3", "k_fc_early<false", 2.0)):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
             if match in r["Kernel_Name"]]
        big = sorted(x for x in d if x >= min_ms)
        out["kernels"][key] = {"launches": len(big), "avg_ms": sum(big) / len(big) if big else None,
                               "min_ms": big[0] if big else None, "max_ms": big[-1] if big else None,
                               "rule": "launches of %s* lasting >= %.0f ms" % (match, min_ms),
                               "all_launches_of_the_name": len(d)}
    # without the trace (deleted after a run): the statistics, for a name whose
    # every launch is a headline one (k_fc_early runs only for >= 2^14 queries:
    # the C3 FC steps of the bench)
    if not out["kernels"]["k_fc_c3"]["launches"]:
        for f in glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if "k_fc_early<false" in r["Name"]:
                        out["kernels"]["k_fc_c3"] = {
                            "launches": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                            "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6,
                            "rule": "every launch of %s (kernel statistics)" % r["Name"]}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()

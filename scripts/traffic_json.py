"""Per-launch HBM bytes of k_index and k_fc from the --pmc passes of
scripts/prof_round.sh (mean over dispatches, summed over TCC instances).

Reads: the L2's memory-side read requests by size, TCC_EA0_RDREQ_{32B,64B,128B}
(bytes = 32 n32 + 64 n64 + 128 n128), which needs no assumption about the
access pattern.  FETCH_SIZE, the older figure, is kept for reference: gfx950
tallies a 128-B request at 64 B (MI355X_MICROARCH.md), so it undercounts wide
streaming reads by 2x and is exact for narrow ones.  Writes: WRITE_SIZE (KiB)
and the request counts TCC_EA0_WRREQ / _64B.
"""
import csv
import glob
import json
import os
import sys


names = {}   # key -> full kernel names seen (template arguments included)


def per_kernel(root, counters):
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    acc = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                c = row.get("Counter_Name")
                if c not in counters:
                    continue
                name = row["Kernel_Name"]
                # keyed by the kernel's own name (k_fc, k_index, k_index_segs):
                # bench.py takes the figure of the kernel it timed, never a
                # neighbour's
                key = next((k for k in ("k_index_segs", "k_index", "k_fc_early", "k_fc") if name.startswith("void lx::" + k + "<")
                            or name.startswith(k + "<") or ("lx::" + k + "<") in name), None)
                if key is None:
                    continue
                names.setdefault(key, set()).add(name.split("(")[0])
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                d = acc.setdefault(key, {}).setdefault(c, {})
                d[disp] = d.get(disp, 0.0) + float(row["Counter_Value"])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    root = sys.argv[1]
    rd = per_kernel(os.path.join(root, "rdreq"), {"TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_64B", "TCC_EA0_RDREQ_128B",
                                                   "TCC_EA0_RDREQ"})
    wr = per_kernel(os.path.join(root, "write"), {"WRITE_SIZE", "TCC_EA0_WRREQ", "TCC_EA0_WRREQ_64B"})
    fe = per_kernel(os.path.join(root, "fetch"), {"FETCH_SIZE"})
    out = {"workload": os.environ.get("CFG", "c3"), "fc_queries": 1 << 24,
           "method": "rocprofv3 --pmc passes of scripts/prof_round.sh (one TCC group per pass): reads = "
                     "32*TCC_EA0_RDREQ_32B + 64*TCC_EA0_RDREQ_64B + 128*TCC_EA0_RDREQ_128B, writes = WRITE_SIZE "
                     "(KiB); mean over dispatches, summed over TCC instances",
           "kernels": {}}
    for k in sorted(set(rd) | set(wr)):
        r = rd.get(k, {})
        w = wr.get(k, {})
        rb = 32 * r.get("TCC_EA0_RDREQ_32B", 0) + 64 * r.get("TCC_EA0_RDREQ_64B", 0) + 128 * r.get("TCC_EA0_RDREQ_128B", 0)
        wb = 1024 * w.get("WRITE_SIZE", 0)
        out["kernels"][k] = {"hbm_read_bytes": rb, "hbm_write_bytes": wb, "hbm_bytes": rb + wb, "counters": {**r, **w},
                             "FETCH_SIZE_KiB_mean": fe.get(k, {}).get("FETCH_SIZE"),
                             "kernel_names": sorted(names.get(k, ()))}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()

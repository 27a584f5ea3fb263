"""k_root_fc VALU evidence from scripts/prof_abft.sh's two --pmc passes:
per launch shape, executed VALU instructions per pair-column and the share of
the SIMDs' VALU issue slots used (a wave64 VALU instruction holds its SIMD for
2 cycles; 1024 SIMDs; clock from GRBM_GUI_ACTIVE / 8 XCDs / duration)."""
import collections
import csv
import json
import sys

d = collections.defaultdict(dict)
out = sys.argv[1]
for p in ("pmc1", "pmc2"):
    for r in csv.DictReader(open("%s/%s/%s_counter_collection.csv" % (out, p, p))):
        k = (p, int(r["Dispatch_Id"]))
        d[k][r["Counter_Name"]] = float(r["Counter_Value"])
        d[k]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        d[k]["grid"] = int(r["Grid_Size"]) // 256
shapes = collections.defaultdict(lambda: collections.defaultdict(list))
for (p, _), v in d.items():
    for c, x in v.items():
        shapes[v["grid"]][c].append(x)
res = {}
for g, s in sorted(shapes.items()):
    m = {c: sum(x) / len(x) for c, x in s.items()}
    if "SQ_INSTS_VALU" not in m or "GRBM_GUI_ACTIVE" not in m:
        continue
    cyc = m["GRBM_GUI_ACTIVE"] / 8
    res[g] = {"launches": len(s["SQ_INSTS_VALU"]), "us": m["dur"] * 1e6, "clock_ghz": cyc / m["dur"] / 1e9,
              "valu_per_wave": m["SQ_INSTS_VALU"] / m["SQ_WAVES"],
              "valu_issue_frac": m["SQ_INSTS_VALU"] * 2 / (1024 * cyc),
              "lds_per_valu": m["SQ_INSTS_LDS"] / m["SQ_INSTS_VALU"],
              "busy_frac": m["SQ_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"])}
print(json.dumps(res, indent=1))

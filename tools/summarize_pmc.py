#!/usr/bin/env python3
"""Summarise tools/pmc_ab.sh: per variant, median per-dispatch SQ counters of
the verify kernel and derived ratios (cycle counters are quad-cycles)."""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
res = {}
for path in sorted(glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True)):
    variant = os.path.relpath(path, d).split(os.sep)[0]
    agg = {}
    for r in csv.DictReader(open(path)):
        if "verify_kernel" not in r["Kernel_Name"]:
            continue
        key = (r["Dispatch_Id"], r["Counter_Name"])
        agg[key] = agg.get(key, 0.0) + float(r["Counter_Value"])
    per = {}
    for (_, c), v in agg.items():
        per.setdefault(c, []).append(v)
    med = {c: statistics.median(v) for c, v in per.items()}
    wc = med.get("SQ_WAVE_CYCLES", 0) or 1
    med["frac_wait_any"] = med.get("SQ_WAIT_ANY", 0) / wc
    med["frac_wait_inst_any"] = med.get("SQ_WAIT_INST_ANY", 0) / wc
    med["frac_active_inst_any"] = med.get("SQ_ACTIVE_INST_ANY", 0) / wc
    res[variant] = med
json.dump(res, open(os.path.join(d, "summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))

#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc_ab.sh): per variant and per
kernel, median per-dispatch counter values and derived ratios (SQ cycle
counters are quad-cycles; FETCH_SIZE / WRITE_SIZE are KiB)."""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
kfilter = sys.argv[2] if len(sys.argv) > 2 else "verify"
res = {}
for path in sorted(glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True)):
    variant = os.path.relpath(path, d).split(os.sep)[0]
    agg = {}
    for r in csv.DictReader(open(path)):
        kname = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if kfilter not in kname:
            continue
        key = (kname, r["Dispatch_Id"], r["Counter_Name"])
        agg[key] = agg.get(key, 0.0) + float(r["Counter_Value"])
    per = {}
    for (k, _, c), v in agg.items():
        per.setdefault(k, {}).setdefault(c, []).append(v)
    out = {}
    for k, cs in per.items():
        med = {c: statistics.median(v) for c, v in cs.items()}
        wc = med.get("SQ_WAVE_CYCLES", 0)
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in med:
                    med["frac_" + c[3:].lower()] = med[c] / wc
        out[k] = med
    res.setdefault(variant, {}).update(out)
json.dump(res, open(os.path.join(d, "summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))

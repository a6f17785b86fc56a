#!/usr/bin/env python3
"""Summarise a tools/profile.sh run.  Per verify kernel (scalar / point / main /
fallback): kernel-trace average duration, FETCH_SIZE / WRITE_SIZE per launch
(KiB x 1024; FETCH raw and with the gfx950 x2 wide-read correction of
MI355X_MICROARCH.md 'HBM' as an upper bound) and SQ counters; totals per
verify launch sequence (one stl_ed25519_verify_batch_device call = the three
kernels on one stream).  Writes <dir>/summary.json; with --traffic also
profiles/traffic_latest.json, which bench.py reports as roofline.traffic."""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kname(s):
    return s.split("(")[0].replace("void ", "").strip()


def pmc(sub):
    out = {}
    for path in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        agg = {}
        for r in csv.DictReader(open(path)):
            k = kname(r["Kernel_Name"])
            if "verify" not in k:
                continue
            key = (k, r["Dispatch_Id"], r["Counter_Name"])
            agg[key] = agg.get(key, 0.0) + float(r["Counter_Value"])
        for (k, _, c), v in agg.items():
            out.setdefault(k, {}).setdefault(c, []).append(v)
    return {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in out.items()}


stats = {}
for path in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        stats[kname(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                   "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
f, w, sq = pmc("pmc_fetch"), pmc("pmc_write"), pmc("pmc_sq")
kernels = sorted(set(f) | set(w) | set(sq) | {k for k in stats if "verify" in k})
per = {}
tot = {"fetch_bytes_raw": 0.0, "write_bytes": 0.0, "avg_ns": 0.0}
for k in kernels:
    fb = f.get(k, {}).get("FETCH_SIZE", 0.0) * 1024
    wb = w.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
    e = {"fetch_bytes_raw": fb, "write_bytes": wb, "sq": sq.get(k, {}), "trace": stats.get(k)}
    s = sq.get(k, {})
    if s.get("GRBM_GUI_ACTIVE") and stats.get(k):
        e["effective_clock_ghz"] = s["GRBM_GUI_ACTIVE"] / 8 / (stats[k]["avg_ns"] * 1e-9) / 1e9
    if s.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            e["frac_" + c[3:].lower()] = s.get(c, 0.0) / s["SQ_WAVE_CYCLES"]
    per[k] = e
    tot["fetch_bytes_raw"] += fb
    tot["write_bytes"] += wb
    tot["avg_ns"] += stats.get(k, {}).get("avg_ns", 0.0)
tot["hbm_bytes_per_launch"] = tot["fetch_bytes_raw"] + tot["write_bytes"]
tot["hbm_bytes_per_launch_fetch_x2_upper"] = 2 * tot["fetch_bytes_raw"] + tot["write_bytes"]
summary = {"kernels": per, "verify_launch_sequence": tot,
           "other_kernels": {k: v for k, v in stats.items() if "verify" not in k}}
json.dump(summary, open(os.path.join(d, "summary.json"), "w"), indent=1)
if "--traffic" in sys.argv:
    traffic = {"source": f"{d}/summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, summed "
                         "over the verify_scalar/point/main/fallback kernels, one verify launch sequence of the bench batch)",
               "hbm_bytes_per_launch": tot["hbm_bytes_per_launch"],
               "hbm_bytes_per_launch_fetch_x2_upper": tot["hbm_bytes_per_launch_fetch_x2_upper"],
               "note": "FETCH_SIZE+WRITE_SIZE KiB x 1024, raw; FETCH x2 (gfx950 wide-read correction) upper bound"}
    sys.path.insert(0, ROOT)
    from stellard_amd.build import source_digest
    traffic["build"] = {"sources_sha256": source_digest(), "git_head": os.environ.get("GIT_HEAD"),
                        "execution": os.environ.get("STL_EXEC_NOTE")}
    # the dominant kernel, as bench.py's roofline reports it (verify_main_kernel<JOINT>)
    mk = [k for k in summary["kernels"] if k.startswith("stl::verify_main_kernel")]
    m = summary["kernels"][mk[0]] if len(mk) == 1 else None
    if m:
        traffic["main_kernel"] = {
            "kernel": mk[0],
            "fetch_size_bytes_raw": m["fetch_bytes_raw"], "write_size_bytes": m["write_bytes"],
            "hbm_bytes_per_launch": 2 * m["fetch_bytes_raw"] + m["write_bytes"],
            "correction": "MI355X_MICROARCH.md HBM section: FETCH_SIZE reports half the bytes of 16-B/lane reads "
                          "on gfx950 (all of this kernel's global reads are 16-B/lane uint4 table loads and "
                          "global_load_lds rows), so 2 x FETCH_SIZE + WRITE_SIZE",
            "avg_ns_rocprof": m["trace"]["avg_ns"]}
    for path in (os.path.join(ROOT, "profiles", "traffic_latest.json"), os.path.join(d, "traffic_latest.json")):
        with open(path, "w") as f:
            json.dump(traffic, f, indent=1)
print(json.dumps(summary, indent=1))

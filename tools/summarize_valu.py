#!/usr/bin/env python3
"""Summarise tools/valu_pmc.sh output into profiles/valu_latest.json.

Per verify kernel (mean over the profiled launches): VALUBusy and
VALUUtilization (rocprofv3 derived metrics), OccupancyPercent, VALU
instruction counts (SQ_INSTS_VALU / _INT32 / _INT64 / _IOPS) and the kernel's
GPU-active cycles; plus the launch-level VALUBusy weighted by each kernel's
GRBM_GUI_ACTIVE cycles.  Also the kernel's issue-cost bound:
the time its VALU instruction stream needs at the measured per-instruction
costs (tools/microbench) -- 64-bit ops 4.61 SIMD-cycles
per wave instruction, every other VALU op 2.5 (the VOP2 cost; VOP3 ops cost
more, so this is a lower bound) -- spread over 256 CUs x 4 SIMDs at the
effective clock of the same dispatches (GRBM_GUI_ACTIVE / 8 XCDs / duration).
usage: summarize_valu.py gpurun_out/<dir> [--out F]"""
import collections
import csv
import glob
import json
import os
import sys

MEAN = {"VALUBusy", "VALUUtilization", "OccupancyPercent", "MeanOccupancyPerActiveCU"}
CYC_INT64, CYC_OTHER = 4.61, 2.5  # SIMD-cycles per wave instruction at 2 waves/SIMD
SIMDS, XCDS = 256 * 4, 8


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)  # kernel -> dispatch -> ns (the pass with GRBM_GUI_ACTIVE)
    for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "verify" not in k:
                continue
            # one row per (dispatch, counter): sum over dimensions per dispatch
            per[k][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r.get("Start_Timestamp"):
                dur[k][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = {}
    for k, v in per.items():
        acc = collections.defaultdict(list)
        for (c, _), xs in v.items():
            acc[c].append(sum(xs) / len(xs) if c in MEAN else sum(xs))
        out[k] = {c: sum(xs) / len(xs) for c, xs in acc.items()}
        if dur[k]:
            ns = sum(dur[k].values()) / len(dur[k])
            o = out[k]
            o["duration_ns_pmc_pass"] = ns
            if o.get("GRBM_GUI_ACTIVE") and o.get("SQ_INSTS_VALU") and "SQ_INSTS_VALU_INT64" in o:
                ghz = o["GRBM_GUI_ACTIVE"] / XCDS / ns
                cyc = CYC_INT64 * o["SQ_INSTS_VALU_INT64"] + CYC_OTHER * (o["SQ_INSTS_VALU"] - o["SQ_INSTS_VALU_INT64"])
                o["effective_clock_ghz"] = ghz
                o["issue_bound_ms"] = cyc / SIMDS / ghz / 1e6
                o["issue_bound_ms_at_2p4ghz"] = cyc / SIMDS / 2.4 / 1e6
                o["issue_bound_model"] = (f"{CYC_INT64} SIMD-cycles x SQ_INSTS_VALU_INT64 + {CYC_OTHER} x the other "
                                          f"VALU instructions, / {SIMDS} SIMDs / effective clock")
    return out


def main():
    d = sys.argv[1]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "valu_latest.json")
    k = load(d)
    w = sum(v.get("GRBM_GUI_ACTIVE", 0) for v in k.values())
    busy = sum(v.get("VALUBusy", 0) * v.get("GRBM_GUI_ACTIVE", 0) for v in k.values()) / w if w else None
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from stellard_amd.build import source_digest
    doc = {"source": d + " (rocprofv3 --pmc, one pass per counter group: tools/valu_pmc.sh)",
           "build": {"sources_sha256": source_digest(), "git_head": os.environ.get("GIT_HEAD"),
                     "execution": os.environ.get("STL_EXEC_NOTE")},
           "launch_valu_busy_pct": busy, "kernels": k}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()

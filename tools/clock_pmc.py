#!/usr/bin/env python3
"""Effective clock of one kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE,GRBM_COUNT
--kernel-trace run (csv output): GRBM_GUI_ACTIVE / 8 XCDs / kernel duration,
per dispatch, joined on the dispatch id (MI355X_MICROARCH.md: GRBM counts sum
over the 8 XCDs).

    python tools/clock_pmc.py <out_dir> <kernel-substring> [--last N]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("kernel")
    ap.add_argument("--last", type=int, default=40)
    a = ap.parse_args()
    cc = glob.glob(os.path.join(a.out_dir, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(a.out_dir, "**", "*kernel_trace.csv"), recursive=True)
    grbm = {}
    for p in cc:
        for r in csv.DictReader(open(p)):
            if a.kernel in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                grbm[r["Dispatch_Id"]] = grbm.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    dur = {}
    for p in kt:
        for r in csv.DictReader(open(p)):
            if a.kernel in r["Kernel_Name"]:
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ids = sorted(set(grbm) & set(dur), key=int)[-a.last:]
    ghz = [grbm[i] / 8 / dur[i] / 1e9 for i in ids]
    us = [dur[i] * 1e6 for i in ids]
    print(json.dumps({"kernel": a.kernel, "dispatches": len(ids), "clock_ghz_median": statistics.median(ghz) if ghz else None,
                      "clock_ghz_min": min(ghz) if ghz else None, "clock_ghz_max": max(ghz) if ghz else None,
                      "us_median": statistics.median(us) if us else None}))


if __name__ == "__main__":
    main()

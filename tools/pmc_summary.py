#!/usr/bin/env python3
"""Summarise the rocprofv3 PMC passes of tools/gpu_pmc.sh for one kernel.

    python tools/pmc_summary.py gpurun_out/pmc_TAG <kernel-substring> --K 128 --N 1048576 \
        [--out profiles/round1_pmc_estep.json]

Per-launch values (each pass averages the kernel's dispatches):
  * hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).  The x2 is
    the gfx950 correction of MI355X_MICROARCH.md (HBM section): FETCH_SIZE tallies
    128-B requests at 64 B; WRITE_SIZE counts streaming stores exactly;
  * VALU instructions, VALU-active cycles (SQ_ACTIVE_INST_VALU is in quad-cycles)
    and their ratio, the wave-cycle split (active / issue-wait / waitcnt-parked).
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(pmc_dir, sub):
    vals = collections.defaultdict(list)
    for p in sorted(glob.glob(os.path.join(pmc_dir, "p*", "run_counter_collection.csv"))):
        per_dispatch = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(p)):
            if sub not in r["Kernel_Name"]:
                continue
            per_dispatch[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for d in per_dispatch.values():
            for c, v in d.items():
                vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items()}, {c: len(v) for c, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("kernel")
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--N", type=int, default=1 << 20)
    ap.add_argument("--out")
    a = ap.parse_args()
    v, n = load(a.pmc_dir, a.kernel)
    out = {"kernel": a.kernel, "K": a.K, "N": a.N, "dispatches": max(n.values()) if n else 0,
           "source": a.pmc_dir, "counters_per_launch": v}
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        fetch = 2.0 * v["FETCH_SIZE"] * 1024
        write = v["WRITE_SIZE"] * 1024
        out["hbm_read_bytes_per_launch"] = fetch
        out["hbm_write_bytes_per_launch"] = write
        out["hbm_bytes_per_launch"] = fetch + write
        out["algorithmic_bytes_per_launch"] = a.N * (28 + 4 * a.K)
    if "SQ_INSTS_VALU" in v and "SQ_ACTIVE_INST_VALU" in v:
        out["valu_insts"] = v["SQ_INSTS_VALU"]
        out["valu_active_cycles"] = 4 * v["SQ_ACTIVE_INST_VALU"]
        out["valu_cycles_per_inst"] = 4 * v["SQ_ACTIVE_INST_VALU"] / v["SQ_INSTS_VALU"]
    if "SQ_WAVE_CYCLES" in v:
        wc = v["SQ_WAVE_CYCLES"]
        out["wave_cycle_split"] = {k: v.get(c, 0.0) / wc for k, c in
                                   (("active", "SQ_ACTIVE_INST_ANY"), ("issue_wait", "SQ_WAIT_INST_ANY"),
                                    ("parked", "SQ_WAIT_ANY"))}
    js = json.dumps(out, indent=1, sort_keys=True)
    print(js)
    if a.out:
        open(a.out, "w").write(js + "\n")


if __name__ == "__main__":
    main()

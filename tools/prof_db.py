#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace SQLite database
(ROCm 7.x writes <name>_results.db by default): calls, average / total
duration, and optionally grid sizes.  Usage:
    python tools/prof_db.py gpurun_out/<dir>/<name>_results.db [--grid] [--filter SUBSTR]"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--grid", action="store_true")
    ap.add_argument("--filter", default="")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--timeline", type=int, default=0, help="also print the last N dispatches: start gap, duration")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    names = {r[0]: r[1] for r in c.execute("select id, display_name from rocpd_info_kernel_symbol")}
    rows = c.execute("select kernel_id, start, end, grid_size_x, workgroup_size_x from rocpd_kernel_dispatch").fetchall()
    agg = collections.defaultdict(list)
    for kid, s, e, gx, wx in rows:
        key = names.get(kid, str(kid))
        if a.grid:
            key = f"[grid {gx}/{wx}] {key}"
        if a.filter in key:
            agg[key].append(e - s)
    if a.timeline:
        prev = None
        for kid, s, e, gx, wx in sorted(rows, key=lambda r: r[1])[-a.timeline:]:
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"gap {gap:8.2f} us  dur {(e - s) / 1e3:8.2f} us  grid {gx}/{wx}  {names.get(kid, kid)[:70]}")
            prev = e
    total = sum(sum(v) for v in agg.values())
    print(f"{'kernel':90s} {'calls':>6s} {'avg_us':>9s} {'total_us':>10s} {'%':>5s}")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        print(f"{k[:90]:90s} {len(v):6d} {sum(v) / len(v) / 1e3:9.2f} {sum(v) / 1e3:10.1f} {100 * sum(v) / total:5.1f}")


if __name__ == "__main__":
    main()

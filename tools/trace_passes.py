#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of tools/cornell_bench.py into render passes
(one per li_camera_kernel) and print, per pass, the wall span, the summed
kernel time, the idle gaps and the top kernels.

    python tools/trace_passes.py gpurun_out/prof_corn/run_kernel_trace.csv [first_pass] [n_passes]
"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    starts = [i for i, k in enumerate(ks) if "li_camera_kernel" in k[2]]
    for p in range(first, min(first + count, len(starts))):
        a = starts[p]
        b = starts[p + 1] if p + 1 < len(starts) else len(ks)
        seg = ks[a:b]
        # the pass ends at the last kernel before the next camera kernel
        t0, t1 = seg[0][0], max(e for _, e, _ in seg)
        busy = 0
        cur = t0
        for s, e, _ in seg:
            if e > cur:
                busy += e - max(s, cur)
                cur = e
        by = collections.defaultdict(lambda: [0, 0])
        for s, e, n in seg:
            short = n.split("(")[0].replace("void ", "")[:70]
            by[short][0] += e - s
            by[short][1] += 1
        print(f"pass {p}: span {(t1 - t0) / 1e6:.2f} ms, kernels busy {busy / 1e6:.2f} ms, "
              f"idle {(t1 - t0 - busy) / 1e6:.2f} ms, launches {len(seg)}")
        for n, (d, c) in sorted(by.items(), key=lambda x: -x[1][0])[:14]:
            print(f"   {d / 1e6:8.3f} ms  x{c:5d}  {n}")


if __name__ == "__main__":
    main()


def gaps(path, p, thresh_us=150):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    starts = [i for i, k in enumerate(ks) if "li_camera_kernel" in k[2]]
    a = starts[p]
    b = starts[p + 1] if p + 1 < len(starts) else len(ks)
    seg = ks[a:b]
    t0 = seg[0][0]
    cur = seg[0][1]
    for i in range(1, len(seg)):
        s, e, n = seg[i]
        if s - cur > thresh_us * 1000:
            prev = seg[i - 1][2].split("(")[0].replace("void ", "")[:50]
            print(f"  t={((cur - t0) / 1e6):7.2f} ms gap {(s - cur) / 1e3:8.1f} us  after {prev:50s} before {n.split('(')[0].replace('void ', '')[:50]}")
        cur = max(cur, e)

#!/usr/bin/env python3
"""Summarise tools/cornell_bench.py output (stdin): per run its total and the
guided (non-training) passes' times and fallback counts."""
import json
import sys

for line in sys.stdin:
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "workload" in d:
        print(d["workload"][:48], "total", round(d["total_ms"], 1), "ms")
    elif not d["train"]:
        print("   pass", round(d["ms"], 2), "ms  fallback", d["fallback_queries"])
    else:
        print("   train", round(d["ms"], 2), "ms")

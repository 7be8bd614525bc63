#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace (rocpd .db or kernel_trace.csv) into a
per-kernel table: calls, total/avg time, share.  Usage:
    python scripts/prof_summary.py <db-or-csv-or-dir> [--steps N] [--top K]
"""
import argparse
import glob
import os
import sqlite3
from collections import defaultdict


def load(path):
    rows = []
    if os.path.isdir(path):
        cands = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) + \
            glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = cands[0]
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = """select ks.kernel_name, kd.start, kd.end from rocpd_kernel_dispatch kd
               join rocpd_info_kernel_symbol ks on kd.kernel_id = ks.id"""
        for name, s, e in c.execute(q):
            rows.append((name, s, e))
    else:
        import csv
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = load(a.path)
    agg = defaultdict(lambda: [0, 0.0])
    for name, s, e in rows:
        short = name.split("(")[0][:90]
        agg[short][0] += 1
        agg[short][1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"| kernel | calls | total us | avg us | share |" + (" us/step |" if a.steps else ""))
    print("|---|---|---|---|---|" + ("---|" if a.steps else ""))
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        extra = f" {t / a.steps:.1f} |" if a.steps else ""
        print(f"| `{k}` | {n} | {t:.1f} | {t / n:.2f} | {100 * t / tot:.1f}% |" + extra)
    print(f"\nTOTAL kernel time: {tot:.1f} us over {len(rows)} dispatches")


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Per-kernel averages of rocprofv3 counter CSVs (one or more run dirs) as a
markdown table, with derived VALU/MFMA and L2 hit-rate columns."""
import collections
import csv
import glob
import os
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(collections.Counter)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0][:60]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[k][r["Counter_Name"]] += 1
    cols = sorted({c for v in agg.values() for c in v})
    print("| kernel | " + " | ".join(cols) + " | VALU/MFMA | L2 hit % |")
    print("|---" * (len(cols) + 3) + "|")
    for k, v in sorted(agg.items()):
        avg = {c: v[c] / max(cnt[k][c], 1) for c in cols}
        mf = avg.get("SQ_INSTS_MFMA", 0.0)
        ratio = f"{avg.get('SQ_INSTS_VALU', 0.0) / mf:.2f}" if mf else "-"
        h, m = avg.get("TCC_HIT_sum", 0.0), avg.get("TCC_MISS_sum", 0.0)
        hit = f"{100 * h / (h + m):.0f}" if h + m else "-"
        print(f"| `{k}` | " + " | ".join(f"{avg[c]:.4g}" for c in cols) + f" | {ratio} | {hit} |")


if __name__ == "__main__":
    main()

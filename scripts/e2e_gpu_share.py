#!/usr/bin/env python
"""Where the GPU time of an end-to-end run goes: a rocprofv3 kernel trace of
``main.py --mode gpu`` (learner thread replaying its step graphs, actor thread running
batched inference + inserts) split by the host thread that dispatched each kernel.

Per thread over the steady-state window (the last ``--tail`` fraction of the trace):
kernel count, summed kernel time, busy time (union of its kernels' intervals), the time
it is busy while the other thread's kernels are also resident, and its top kernels.

    python scripts/e2e_gpu_share.py gpurun_out/e2e_trace/run_kernel_trace.csv [--tail 0.6]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json


def union(iv):
    out, s, e = 0, None, None
    for a, b in sorted(iv):
        if s is None or a > e:
            if s is not None:
                out += e - s
            s, e = a, b
        else:
            e = max(e, b)
    return out + (e - s if s is not None else 0)


def merged(iv):
    res = []
    for a, b in sorted(iv):
        if res and a <= res[-1][1]:
            res[-1][1] = max(res[-1][1], b)
        else:
            res.append([a, b])
    return res


def overlap(a, b):
    """Total length of the intersection of two merged interval lists."""
    i = j = tot = 0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if hi > lo:
            tot += hi - lo
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--tail", type=float, default=0.6)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    w0 = t1 - a.tail * (t1 - t0)
    by = collections.defaultdict(list)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= w0:
            by[r["Thread_Id"]].append((s, e, r["Kernel_Name"][:60]))
    window = t1 - w0
    iv = {t: merged([(s, e) for s, e, _ in k]) for t, k in by.items()}
    out = {"window_ms": round(window / 1e6, 2), "threads": {}}
    all_busy = union([(s, e) for k in by.values() for s, e, _ in k])
    out["gpu_busy_share"] = round(all_busy / window, 3)
    for t, ks in sorted(by.items(), key=lambda kv: -len(kv[1])):
        tot = collections.Counter()
        for s, e, n in ks:
            tot[n] += e - s
        others = merged([x for u, v in iv.items() if u != t for x in v])
        busy = union([(s, e) for s, e, _ in ks])
        out["threads"][t] = {
            "kernels": len(ks), "kernel_ms": round(sum(tot.values()) / 1e6, 2),
            "busy_ms": round(busy / 1e6, 2), "busy_share": round(busy / window, 3),
            "busy_beside_other_threads_ms": round(overlap(iv[t], others) / 1e6, 2),
            "top": [(n, round(v / 1e6, 2)) for n, v in tot.most_common(8)]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Per-kernel durations of the CU-steal proxy (scripts/bench_cu_steal.py) from a rocprofv3
kernel trace: the learner kernels that run while the spinner holds K CUs against the
same kernels with K = 0 (phases split at the spinner's launches)."""
import collections
import csv
import json
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    phases, cur = [], None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0][:60]
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "spin" in name:
            cur = {"k": int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0), "t0": t0, "t1": t1,
                   "k_durs": collections.defaultdict(list)}
            phases.append(cur)
            continue
        if cur is not None and cur["t0"] <= t0 and t1 <= cur["t1"]:
            cur["k_durs"][name].append((t1 - t0) / 1e3)
    for p in phases:
        agg = {k: round(sum(v) / len(v), 2) for k, v in p["k_durs"].items() if len(v) >= 5}
        print(json.dumps({"spinner_grid": p["k"], "kernels_us": dict(sorted(agg.items(), key=lambda kv: -kv[1]))}))


if __name__ == "__main__":
    main()

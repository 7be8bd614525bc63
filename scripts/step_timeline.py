"""Per-kernel timeline of one learner step from a rocprofv3 kernel trace:
start / end (us, relative to the step's first kernel), duration, HW queue, grid.
Usage: python scripts/step_timeline.py <run_kernel_trace.csv> [first-kernel-prefix]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# find last occurrences of tree_sample_kernel as step starts
first = sys.argv[2] if len(sys.argv) > 2 else "void conv12_fused_kernel"
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(first)]
i0, i1 = starts[-6], starts[-5]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1000; e = (int(r["End_Timestamp"]) - t0) / 1000
    print("%7.1f %7.1f %6.1f q%s grid=%s wg=%s  %s" % (s, e, e - s, r["Queue_Id"], r["Grid_Size_X"], r["Workgroup_Size_X"], r["Kernel_Name"][:60]))

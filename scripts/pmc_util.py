"""Per-kernel LDS bank-conflict share and approximate MFMA busy share from a
scripts/pmc_step.sh counter pass (rocprofv3 CSV).  conflict % = SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE; MFMA busy % ~ SQ_VALU_MFMA_BUSY_CYCLES / (kernel ns x clock GHz x
1024 SIMDs) (the counter sums over every SIMD; the shader clock under load is taken as
--ghz, default 2.4, so the percentage is approximate)."""
import argparse
import collections
import csv
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--ghz", type=float, default=2.4)
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(os.path.join(a.dir, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"].split("(")[0][:60]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            acc[k]["_ns"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    print("| kernel | calls | mean us | LDS conflict % | MFMA busy % (approx) |")
    print("|---|---|---|---|---|")
    rows = []
    for k, c in acc.items():
        if not c.get("SQ_VALU_MFMA_BUSY_CYCLES") and not c.get("SQ_LDS_IDX_ACTIVE"):
            continue
        n = len(c["SQ_BUSY_CYCLES"])
        ns = sum(c["_ns"]) / len(c["_ns"])
        lds = sum(c["SQ_LDS_IDX_ACTIVE"]) / n
        conf = sum(c["SQ_LDS_BANK_CONFLICT"]) / n
        mf = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / n
        util = 100.0 * mf / (ns * a.ghz * 1024) if ns > 0 else 0.0
        rows.append((ns, k, n, conf, lds, util))
    for ns, k, n, conf, lds, util in sorted(rows, reverse=True):
        if ns < 3000:
            continue
        print(f"| `{k}` | {n} | {ns / 1e3:.1f} | {100 * conf / lds if lds else 0:.1f} | {util:.1f} |")


if __name__ == "__main__":
    main()

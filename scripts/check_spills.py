#!/usr/bin/env python
"""Register / scratch / occupancy report of every gfx950 kernel (hipcc
-Rpass-analysis=kernel-resource-usage), failing when a kernel of the learner's or the
actors' path spills to scratch.  The split conv2 data gradient once spilled 396 B per lane
(44 -> 36 us once fixed, docs/PERF_NOTES.md): run this after touching a kernel.
    python scripts/check_spills.py [--all]
"""
import argparse
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "apex_dqn_amd", "csrc")
# kernels on the default learner / actor paths (substring of the mangled name)
HOT = ["conv12_fused_kernel", "conv2_dgrad_img", "conv3_dgrad_img", "igemm_dma_kernel", "igemm_wgrad_kernel",
       "fc_gemm128_kernel", "conv1_wgrad_img_kernel", "fc_wgrad_head_prio_kernel", "rmsprop_sample_kernel",
       "grad_finalize_kernel", "actor_head_kernel", "sconv_", "resblock_", "maxpool_bwd"]


def usage(path):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{CSRC}", "-c", path, "-o",
           os.devnull, "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\S+)",
                      line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k.split()[0]] = int(v)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--all", action="store_true", help="print every kernel, not only the hot ones")
    a = ap.parse_args()
    bad = []
    for f in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        for r in usage(f):
            hot = any(h in r["name"] for h in HOT)
            if a.all or hot or r.get("ScratchSize", 0):
                print(f"{os.path.basename(f):22s} {r['name'][:70]:70s} V {r.get('VGPRs', 0):3d} A {r.get('AGPRs', 0):3d} "
                      f"scratch {r.get('ScratchSize', 0):4d} occ {r.get('Occupancy', 0)}")
            if hot and r.get("ScratchSize", 0):
                bad.append(r["name"])
    if bad:
        print("SPILLS on the hot path:", *bad, sep="\n  ")
        sys.exit(1)
    print("no scratch on the hot path")


if __name__ == "__main__":
    main()

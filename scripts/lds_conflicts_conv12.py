#!/usr/bin/env python
"""Per-phase attribution of the fused conv1 -> conv2 kernel's LDS bank conflicts
(csrc/conv12_fused.hip, split mode, C = 4), from the kernel's own address arithmetic and
the gfx950 LDS banking rules (/opt/skills/guides/MI355X_MICROARCH.md §LDS):

  ds_read_b64    2 groups of 32 lanes, bank (a/4) mod 64
  ds_read_b128   4 groups of 16 lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, (+32), bank (a/4) mod 64
  ds_write_b64   4 groups of 16 contiguous lanes, bank (a/4) mod 32
  ds_write_b128  8 groups of 8 contiguous lanes, bank (a/4) mod 32

A group takes max over banks of (distinct dword addresses on the bank) LDS-array cycles;
the cycles above one per group are the conflict cycles (SQ_LDS_BANK_CONFLICT), all of them
SQ_LDS_IDX_ACTIVE.  Every LDS instruction of one image is enumerated (4 waves), per phase:

  conv1_frag   conv1's 8-byte s2d fragment reads (13 tiles x 2C K steps per wave)
  conv1_epi    conv1's epilogue stores of y1 hi / lo into conv2's class-major layout
  y1_copy      the S_t rows' y1 copy-out reads (1 image in 3)
  conv2_A      conv2's A-fragment reads of y1 hi / lo (32 K steps x 3 row tiles)
  reduce       the kernel-row-pair partial sums through LDS (writes + reads)

The LDS-DMA of the frames is not an LDS instruction of the waves and is left out.  Prints
one JSON line per phase and the total conflict share, to compare with the measured
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (profiles/r4_pmc_fp32_step_lds_mfma.md)."""
from __future__ import annotations

import collections
import json

C = 4
CF_FRAME = 7056
CF_PLANE = 52224
B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[x + 32 for x in gr] for gr in B128_GROUPS]


def cf_pix(ih, iw):
    return ((ih & 1) * 2 + (iw & 1)) * 100 + (ih >> 1) * 10 + (iw >> 1)


def cf_off(P, c):
    return (P << 7) + ((c ^ ((P >> 1) & 7)) << 4)


def cycles(addrs, groups, nbanks, width):
    """(LDS-array cycles, conflict cycles) of one wave-instruction: addrs[lane] = byte
    address (None: lane idle), width = bytes per lane."""
    tot = ext = 0
    for gr in groups:
        per_bank = collections.defaultdict(set)
        for ln in gr:
            a = addrs[ln]
            if a is None:
                continue
            for d in range(width // 4):
                dw = a // 4 + d
                per_bank[dw % nbanks].add(dw)
        c = max((len(v) for v in per_bank.values()), default=1)
        tot += c
        ext += c - 1
    return tot, ext


G_B64 = [list(range(0, 32)), list(range(32, 64))]
G_W64 = [list(range(16 * i, 16 * i + 16)) for i in range(4)]
G_W128 = [list(range(8 * i, 8 * i + 8)) for i in range(8)]


def phases():
    out = collections.defaultdict(lambda: [0, 0, 0])   # tot, ext, instructions

    def add(name, addrs, groups, nb, width):
        t, e = cycles(addrs, groups, nb, width)
        out[name][0] += t
        out[name][1] += e
        out[name][2] += 1

    for wv in range(4):
        cp, th = wv & 1, wv >> 1
        nh, kp = wv & 1, wv >> 1
        # ---- conv1 fragment reads: tile T = th + 2 j, step s2 (ds_read_b64)
        for j in range(13):
            for s2 in range(2 * C):
                addrs = []
                for lane in range(64):
                    g, pl = lane >> 4, lane & 15
                    p = 16 * (th + 2 * j) + pl
                    if j == 12:
                        p = min(p, 399)
                    oh, ow = divmod(p, 20)
                    q = 2 * s2 + (g >> 1)
                    tap, c = divmod(q, C)
                    aoff = c * CF_FRAME + ((((tap >> 1) * 21 + (tap & 1))) << 4) + ((g & 1) << 3)
                    addrs.append(((oh * 21 + ow) << 4) + aoff)
                add("conv1_frag", addrs, G_B64, 64, 8)
        # ---- conv1 epilogue stores (ds_write_b64, hi and lo planes)
        for j in range(13):
            for nt in range(2):
                for plane in range(2):
                    addrs = []
                    for lane in range(64):
                        g, pl = lane >> 4, lane & 15
                        p = 16 * (th + 2 * j) + pl
                        oh, ow = divmod(p, 20)
                        P = 400 + (pl & 7) if (j == 12 and p >= 400) else cf_pix(oh, ow)
                        ch = 32 * cp + 16 * nt + 4 * g
                        addrs.append(cf_off(P, ch >> 3) + (ch & 7) * 2 + plane * CF_PLANE)
                    add("conv1_epi", addrs, G_W64, 32, 8)
        # ---- conv2 A reads (ds_read_b128), 32 K steps x 3 row tiles x 2 planes
        q0 = []
        for mt in range(3):
            pass
        for s in range(32):
            for mt in range(3):
                for plane in range(2):
                    addrs = []
                    for lane in range(64):
                        rr, kg = lane & 31, lane >> 5
                        r = mt * 32 + rr
                        oh, ow = divmod(r, 10)
                        q0 = (oh + kp) * 10 + ow
                        P_ = ((s >> 4) * 2 + ((s >> 2) & 1)) * 100 + q0 + ((s >> 3) & 1)
                        addrs.append(cf_off(P_, ((s & 3) << 1) | kg) + plane * CF_PLANE)
                    add("conv2_A", addrs, B128_GROUPS, 64, 16)
        # ---- reduction: 6 float4 writes + 6 float4 reads per wave, lane-contiguous
        for _ in range(6):
            addrs = [16 * lane for lane in range(64)]
            add("reduce", addrs, G_W128, 32, 16)
            add("reduce", addrs, B128_GROUPS, 64, 16)
    # ---- y1 copy-out (S_t rows: 1 image in 3): 25 ds_read_b128 per thread, 256 threads
    for wv in range(4):
        for r in range(25):
            addrs = [r * 4096 + (64 * wv + lane) * 16 for lane in range(64)]
            t, e = cycles(addrs, B128_GROUPS, 64, 16)
            out["y1_copy"][0] += t / 3
            out["y1_copy"][1] += e / 3
            out["y1_copy"][2] += 1 / 3
    return out


def main():
    out = phases()
    T = sum(v[0] for v in out.values())
    E = sum(v[1] for v in out.values())
    for k, (t, e, n) in sorted(out.items(), key=lambda kv: -kv[1][1]):
        print(json.dumps({"phase": k, "wave_instructions_per_image": round(n, 1), "lds_cycles": round(t),
                          "conflict_cycles": round(e), "conflict_pct_of_phase": round(100 * e / t, 1) if t else 0,
                          "share_of_all_conflicts_pct": round(100 * e / E, 1) if E else 0}))
    print(json.dumps({"phase": "total", "lds_cycles": round(T), "conflict_cycles": round(E),
                      "conflict_pct": round(100 * E / T, 1), "measured_conflict_pct": 45.4}))


if __name__ == "__main__":
    main()

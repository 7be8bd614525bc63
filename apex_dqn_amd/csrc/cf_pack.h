// Weight-fragment pack of the fused conv1 -> conv2 forward (csrc/conv12_fused.hip): the
// pack launch's block bodies (cf_pack_kernel).
#pragma once
#include "mfma_common.h"
#include "conv2_wfrag.h"

#define CF_LO_SCALE 4096.f

// conv1 fragments per (set, cp, nt, K step s, hi / lo) as 64 lanes x 16 B
#define CF_W1FRAG(C_) (2 * 2 * 2 * 2 * (C_) * 2 * 64)
#define CF_W1FRAG_U4 CF_W1FRAG(4)

// The pack: blocks [0, nc2f) pack the requested conv2 weight sets into C2F fragment order
// (csrc/conv2_wfrag.h), the next 4 per requested set the conv1 operands exactly as the MFMA
// lanes consume them: block (set, cp, nt), lane (g, pl), K step s holds channel
// 32 cp + 16 nt + pl, K 32 s + 8 g .. + 7 (s2d K order k = (tap C + c) 16 + r4 4 + c4,
// tap = 2 a + b) as f16 hi + lo * 2^-12 of w * in_scale.
// The fused kernel's weight-set switch is then 34 coalesced loads instead of ~13k cycles of
// gathers and conversions.  The target set changes only at a target sync: the learner
// repacks it then (pack_sets bit 1).
struct CfPack {
  C2fPack c2f;
  int nc2f;                // C2F blocks (of 256 threads)
  C3fPack c3f;             // fused conv3's fragments (out null: none)
  int nc3f;                // C3F blocks, after the C2F ones
  int sets;                // bit 0: online, bit 1: target
  const float* w1[2];      // fp32 OIHW [64][C][8][8]
  const float* b1[2];
  float in_scale;
  uint4* w1frag;
};

// conv1 operand of weight w (fp32) with the input scale folded in: f16 hi and lo * 2^12
__device__ __forceinline__ void cf_w1_split(float w, float sc, _Float16& hi, _Float16& lo) {
  const float x = w * sc;
  hi = (_Float16)x;
  lo = (_Float16)((x - (float)hi) * CF_LO_SCALE);
}

// The optimizer launch writes the fused forward's ONLINE operands itself (csrc/rmsprop_common.h
// rmsprop_body): every fragment element is one updated weight, so a thread that has just
// computed 4 consecutive weights of w1 or w2 also stores them in fragment order -- no
// pack launch, and no hand-off between workgroups (the folded conv1 bias is summed by the
// fused kernel from the fragments it loads).  Offsets are flat parameter indices.
struct CfFragOut {
  uint4* w1frag;           // conv1 fragments (set 0 half), or null: off
  uint4* c2f;              // conv2 C2F fragments (set 0 hi plane; lo at + C2F_FRAGS)
  int64_t w1_off, w2_off;  // flat offsets of w1 (OIHW [64][C][8][8]) and w2 (OHWI [64][4][4][64])
  int C;
  float in_scale;
  uint4* c3f;              // fused conv3's C3F fragments (set 0 hi; lo at + C3F_FRAGS), or null
  int64_t w3_off;          // flat offset of w3 (OHWI [64][3][3][64])
};

// 4 consecutive updated weights e .. e + 3 (e % 4 == 0): fp32 values px, bf16 hi / lo words
__device__ __forceinline__ void cf_frag_store(const CfFragOut& fo, int64_t e, const float* px, uint2 hi, uint2 lo) {
  const int64_t n1 = 64LL * fo.C * 64;
  if (e >= fo.w1_off && e < fo.w1_off + n1) {
    // (n, c, y, x0 .. x0 + 3) of OIHW -> K step s, lane (g, pl), half r of the 8 K values
    const int k = (int)(e - fo.w1_off);
    const int x0 = k & 7, y = (k >> 3) & 7, nc = k >> 6;
    const int c = nc % fo.C, n = nc / fo.C;
    const int tap = 2 * (y >> 2) + (x0 >> 2), h = (y >> 1) & 1, r = y & 1;
    const int q = tap * fo.C + c, sstep = q >> 1, g = 2 * (q & 1) + h;
    const int cp = n >> 5, nt = (n >> 4) & 1, lane = g * 16 + (n & 15);
    f16x2v a, b;
    _Float16 h0, l0, h1, l1, h2, l2, h3, l3;
    cf_w1_split(px[0], fo.in_scale, h0, l0);
    cf_w1_split(px[1], fo.in_scale, h1, l1);
    cf_w1_split(px[2], fo.in_scale, h2, l2);
    cf_w1_split(px[3], fo.in_scale, h3, l3);
    uint8_t* base = reinterpret_cast<uint8_t*>(fo.w1frag + (((cp * 2 + nt) * 2 * fo.C + sstep) * 2) * 64 + lane) + r * 8;
    a = (f16x2v){h0, h1}; b = (f16x2v){h2, h3};
    *reinterpret_cast<uint2*>(base) = make_uint2(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b));
    a = (f16x2v){l0, l1}; b = (f16x2v){l2, l3};
    *reinterpret_cast<uint2*>(base + 64 * 16) = make_uint2(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b));
    return;
  }
  if (fo.c3f != nullptr && e >= fo.w3_off && e < fo.w3_off + 36864) {
    // 4 of the 8 K values of fragment (nt, s, lane) (csrc/conv2_wfrag.h c3f_src_off)
    const int k = (int)(e - fo.w3_off);
    const int ci = k & 63, tap = (k >> 6) % 9, co = k / 576;
    const int t = ((co >> 5) * 36 + tap * 4 + (ci >> 4)) * 64 + ((ci >> 3) & 1) * 32 + (co & 31);
    uint8_t* base = reinterpret_cast<uint8_t*>(fo.c3f + t) + (ci & 4) * 2;
    *reinterpret_cast<uint2*>(base) = hi;
    *reinterpret_cast<uint2*>(base + C3F_FRAGS * 16) = lo;
    return;
  }
  if (e >= fo.w2_off && e < fo.w2_off + 65536) {
    // 8-element chunk ((co kh) kw) ci0 of OHWI -> fragment t (csrc/conv2_wfrag.h c2f_src_off)
    const int k = (int)(e - fo.w2_off);
    const int ci = k & 63, kw = (k >> 6) & 3, kh = (k >> 8) & 3, co = k >> 10;
    const int nh = co >> 5, rr = co & 31, kp = kh >> 1, st = (kh & 1) * 16 + kw * 4 + (ci >> 4);
    const int kg = (ci >> 3) & 1, t = (kp * 2 + nh) * 2048 + st * 64 + kg * 32 + rr;
    uint8_t* base = reinterpret_cast<uint8_t*>(fo.c2f + t) + (ci & 4) * 2;
    *reinterpret_cast<uint2*>(base) = hi;
    *reinterpret_cast<uint2*>(base + C2F_FRAGS * 16) = lo;
  }
}

// conv1 operands of pack block jb (set, cp, nt) (256 threads; the fused kernel folds the
// 1024-offset bias from the fragments it loads).
__device__ __forceinline__ void cf_pack_w1_block(const CfPack& p, int C, int jb, int t) {
  const int set = p.sets == 2 ? 1 : jb >> 2, cp = (jb >> 1) & 1, nt = jb & 1;
  const int lane = t & 63, sq = t >> 6, g = lane >> 4, pl = lane & 15;
  const float* W1 = p.w1[set];
  const int n = 32 * cp + 16 * nt + pl;
  if (t >= 256) return;
  for (int s = sq; s < 2 * C; s += 4) {
    const int q = 2 * s + (g >> 1), tap = q / C, c = q - tap * C, h = g & 1;
    const int kh = 4 * (tap >> 1) + 2 * h, kw = 4 * (tap & 1);
    const float4 r0 = *reinterpret_cast<const float4*>(W1 + ((n * C + c) * 8 + kh) * 8 + kw);
    const float4 r1 = *reinterpret_cast<const float4*>(W1 + ((n * C + c) * 8 + kh + 1) * 8 + kw);
    const float w8[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    f16x8 hv, lv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      _Float16 hi, lo;
      cf_w1_split(w8[j], p.in_scale, hi, lo);    // the input scale rides in the weights
      hv[j] = hi;
      lv[j] = lo;
    }
    uint4* o = p.w1frag + ((((set * 2 + cp) * 2 + nt) * 2 * C + s) * 2) * 64 + lane;
    o[0] = __builtin_bit_cast(uint4, hv);
    o[64] = __builtin_bit_cast(uint4, lv);
  }
}

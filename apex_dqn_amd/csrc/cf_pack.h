// Weight-fragment pack of the fused conv1 -> conv2 forward (csrc/conv12_fused.hip): the
// pack launch's block bodies (cf_pack_kernel).
#pragma once
#include "mfma_common.h"
#include "conv2_wfrag.h"

#define CF_LO_SCALE 4096.f

// conv1 fragments per (set, cp, nt, K step s, hi / lo) as 64 lanes x 16 B, then the folded
// biases per (set, cp, nt) x 64 lanes (float4)
#define CF_W1FRAG(C_) (2 * 2 * 2 * 2 * (C_) * 2 * 64)
#define CF_W1FRAG_U4 (CF_W1FRAG(4) + 2 * 2 * 2 * 64)

// The pack: blocks [0, nc2f) pack the requested conv2 weight sets into C2F fragment order
// (csrc/conv2_wfrag.h), the next 4 per requested set the conv1 operands exactly as the MFMA
// lanes consume them: block (set, cp, nt), lane (g, pl), K step s holds channel
// 32 cp + 16 nt + pl, K 32 s + 8 g .. + 7 (s2d K order k = (tap C + c) 16 + r4 4 + c4,
// tap = 2 a + b) as f16 hi + lo * 2^-12 of w * in_scale, and the bias the hi accumulation
// chain starts from: bias - 1024 * sum_k w16[n][k] (pixels enter the MFMAs as 1024 + x).
// The fused kernel's weight-set switch is then 34 coalesced loads instead of ~13k cycles of
// gathers and conversions.  The target set changes only at a target sync: the learner
// repacks it then (pack_sets bit 1).
struct CfPack {
  C2fPack c2f;
  int nc2f;                // C2F blocks (of 256 threads)
  int sets;                // bit 0: online, bit 1: target
  const float* w1[2];      // fp32 OIHW [64][C][8][8]
  const float* b1[2];
  float in_scale;
  uint4* w1frag;
};

// conv1 operands of pack block jb (set, cp, nt).  Threads t < 256 work (four K-step
// groups summed in a fixed order: the folded bias is bit-identical whichever launch
// packs); threads >= 256 of a larger block only meet the barriers.
__device__ __forceinline__ void cf_pack_w1_block(const CfPack& p, int C, int jb, int t) {
  __shared__ float part[4][64];
  __shared__ float tot[64];
  const int set = p.sets == 2 ? 1 : jb >> 2, cp = (jb >> 1) & 1, nt = jb & 1;
  const int lane = t & 63, sq = t >> 6, g = lane >> 4, pl = lane & 15;
  const float* W1 = p.w1[set];
  const float sc = p.in_scale;
  const int n = 32 * cp + 16 * nt + pl;
  float ws = 0.f;
  if (t < 256) {
    for (int s = sq; s < 2 * C; s += 4) {
      const int q = 2 * s + (g >> 1), tap = q / C, c = q - tap * C, h = g & 1;
      const int kh = 4 * (tap >> 1) + 2 * h, kw = 4 * (tap & 1);
      const float4 r0 = *reinterpret_cast<const float4*>(W1 + ((n * C + c) * 8 + kh) * 8 + kw);
      const float4 r1 = *reinterpret_cast<const float4*>(W1 + ((n * C + c) * 8 + kh + 1) * 8 + kw);
      const float w8[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
      f16x8 hv, lv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float w = w8[j] * sc;                      // the input scale rides in the weights
        const _Float16 hi = (_Float16)w;
        const _Float16 lo = (_Float16)((w - (float)hi) * CF_LO_SCALE);
        hv[j] = hi;
        lv[j] = lo;
        ws += (float)hi + (float)lo * (1.f / CF_LO_SCALE);
      }
      uint4* o = p.w1frag + ((((set * 2 + cp) * 2 + nt) * 2 * C + s) * 2) * 64 + lane;
      o[0] = __builtin_bit_cast(uint4, hv);
      o[64] = __builtin_bit_cast(uint4, lv);
    }
    part[sq][lane] = ws;
  }
  __syncthreads();
  if (t < 64) tot[t] = ((part[0][t] + part[1][t]) + part[2][t]) + part[3][t];
  __syncthreads();
  if (t < 64) {
    // channel 4 g + i: its sum over the four K-group lanes (fixed order)
    float c4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = 4 * g + i;
      c4[i] = ((tot[ch] + tot[16 + ch]) + tot[32 + ch]) + tot[48 + ch];
    }
    const float4 bb = *reinterpret_cast<const float4*>(p.b1[set] + 32 * cp + 16 * nt + 4 * g);
    reinterpret_cast<float4*>(p.w1frag + CF_W1FRAG(4))[((set * 2 + cp) * 2 + nt) * 64 + t] =
        make_float4(bb.x - 1024.f * c4[0], bb.y - 1024.f * c4[1], bb.z - 1024.f * c4[2], bb.w - 1024.f * c4[3]);
  }
}

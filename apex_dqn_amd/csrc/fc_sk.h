// Stream-K work split of the 128x128-tile fc forward (csrc/conv_mfma.hip
// fc_gemm128_kernel) and the tile -> partial-plane map its consumers share
// (fc_splitk_epilogue_kernel, the DDQN head's load_row_part).
//
// The fc forward has few output tiles (96 at the learner's 1,536 x 1,024; 24 at a
// 74-row per-rank batch) and a 49-step K loop.  A fixed K split leaves CUs idle (2
// splits: 192 of 256) or multiplies the fp32 partial traffic.  Stream-K instead gives
// each of `nblk` workgroups an equal contiguous range of the T = tiles x KT (tile,
// K-step) iterations, tiles in order, K fastest.  A workgroup writes one partial per
// tile its range touches, into plane z = (its index) - (the first workgroup touching
// the tile); a tile's partials are planes 0 .. count - 1, summed in z order, so the
// result is deterministic.  Iteration x belongs to workgroup floor(((x+1) nblk - 1) / T).
#pragma once
#include <stdint.h>

struct FcSK {
  int nblk;       // workgroups; 0: off (plain K split over gridDim.z)
  int kt;         // K steps of 64 per tile
  int ntm, ntn;   // row tiles, 128-column tiles (tile t = bx * ntn + by)
  int m_switch;   // first row of the second weight set (segment-aligned row tiles), or -1
};

__host__ __device__ inline int64_t fc_sk_total(const FcSK& s) { return (int64_t)s.ntm * s.ntn * s.kt; }

// the workgroup that runs iteration x
__host__ __device__ inline int fc_sk_owner(const FcSK& s, int64_t x) {
  return (int)(((x + 1) * (int64_t)s.nblk - 1) / fc_sk_total(s));
}

// first iteration of workgroup b (b = nblk: the end)
__host__ __device__ inline int64_t fc_sk_start(const FcSK& s, int b) {
  return (int64_t)b * fc_sk_total(s) / s.nblk;
}

// partial planes of tile t
__host__ __device__ inline int fc_sk_count(const FcSK& s, int t) {
  const int64_t x0 = (int64_t)t * s.kt;
  return fc_sk_owner(s, x0 + s.kt - 1) - fc_sk_owner(s, x0) + 1;
}

// tile of output element (m, n): the 128-row tiles restart at m_switch
__host__ __device__ inline int fc_sk_tile(const FcSK& s, int m, int n) {
  int bx = m >> 7;
  if (s.m_switch >= 0 && m >= s.m_switch) bx = ((s.m_switch + 127) >> 7) + ((m - s.m_switch) >> 7);
  return bx * s.ntn + (n >> 7);
}

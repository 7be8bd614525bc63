// conv2 weights in the per-lane MFMA fragment order of the conv2 data-gradient
// kernels (csrc/conv2_img.hip): shared by their own launcher and by the fc forward's
// split-K epilogue launch (csrc/conv_mfma.hip), which packs them in spare blocks.
#pragma once
#include "apex_common.h"

#define C2D_FRAGS 8192   // (class, channel half, K step, lane)

// The data-gradient kernels hold the conv2 weights as MFMA A fragments: wave (class,
// channel half), K step s, lane -> 8 bf16 of input channel nh*32 + (lane & 31) over
// output channels co0 .. co0 + 7 at one kernel tap, i.e. 8 two-byte gathers strided by
// 2 KB.  Done in every workgroup that is 256 x 512 (split: 1024) such gathers per lane,
// ~10 us of the launch; here one pass writes the fragments once per step and each
// workgroup reads them back as coalesced 16-B loads.
// a pack riding on another launch (fc_splitk_epilogue_kernel / ddqn_head_kernel spare blocks)
struct C2dPackJob {
  const bf16_t* w;
  const bf16_t* w_lo;
  uint32_t* out;
};
#define C2D_PACK_THREADS (2 * 4 * C2D_FRAGS)   // one per 4-byte word of both planes
__device__ __forceinline__ void pack_c2d_wfrag_word(int i, const bf16_t* __restrict__ w,
                                                   const bf16_t* __restrict__ w_lo, uint32_t* __restrict__ out) {
  // one thread per 4-byte word (two output channels) of one plane: 64 K threads.  As a
  // launch of its own this takes ~5.8 us of the step (the launch, not the work), so
  // the step runs it in spare blocks of the fc forward's epilogue launch.
  if (i >= C2D_PACK_THREADS) return;
  const int pl = i / (4 * C2D_FRAGS), j = i - pl * 4 * C2D_FRAGS;
  const int t = j >> 2, e = j & 3;
  const int lane = t & 63, s = (t >> 6) & 15, nh = (t >> 10) & 1, cls = t >> 11;
  const int p = cls >> 1, q = cls & 1, rr = lane & 31, kg = lane >> 5;
  const int a = (s >> 3) & 1, b = (s >> 2) & 1, co0 = ((s & 3) << 4) + kg * 8;
  const int kh = p + 2 * a, kw = q + 2 * b, ci = nh * 32 + rr;
  const bf16_t* __restrict__ src = pl ? w_lo : w;
  if (src == nullptr) return;
  const int o0 = ((co0 + 2 * e) * 16 + kh * 4 + kw) * 64 + ci, o1 = o0 + 16 * 64;
  out[i] = (uint32_t)src[o0] | ((uint32_t)src[o1] << 16);
}


// Split conv2 forward weights in fragment order (csrc/conv2_img.hip
// conv2_img_fwd_split_kernel): fragment t = (wave (nh, kp), K step s, lane) holds the 16 B
// of w[co = nh*32 + (lane & 31)][kh = 2 kp + (s >> 4)][kw = (s >> 2) & 3][ci0 ..]; four
// planes (set 0 hi, lo, set 1 hi, lo) of C2F_FRAGS uint4.  Packed by the conv2 launcher or
// at the start of the step's conv1 launch (csrc/conv1_s2d.hip).
#define C2F_FRAGS 8192
__device__ __forceinline__ int c2f_src_off(int t) {
  const int lane = t & 63, s = (t >> 6) & 31, wv = t >> 11;
  const int nh = wv & 1, kp = wv >> 1, rr = lane & 31, kg = lane >> 5;
  const int co = nh * 32 + rr, kh = 2 * kp + (s >> 4), kw = (s >> 2) & 3, ci0 = ((s & 3) << 4) + kg * 8;
  return ((co * 4 + kh) * 4 + kw) * 64 + ci0;
}
// bf16 forward (conv2_img_fwd_kernel, 8 waves): fragment t = (wave (nh, kq), K step s <
// 16, lane) holds w[co = nh*32 + (lane & 31)][kh = kq][kw = s >> 2][ci0 ..]; planes: set 0, set 1
__device__ __forceinline__ int c2b_src_off(int t) {
  const int lane = t & 63, s = (t >> 6) & 15, wv = t >> 10;
  const int nh = wv & 1, kq = wv >> 1, rr = lane & 31, kg = lane >> 5;
  const int co = nh * 32 + rr, kw = s >> 2, ci0 = ((s & 3) << 4) + kg * 8;
  return ((co * 4 + kq) * 4 + kw) * 64 + ci0;
}
// Fused conv3 forward weights in fragment order (csrc/conv12_fused.hip conv3_image):
// fragment t = (nt, K step s < 36, lane) holds the 16 B of w[co = 32 nt + (lane & 31)][tap =
// s >> 2][ci0 = 16 (s & 3) + 8 (lane >> 5) ..] of OHWI [64][3][3][64]; four planes (set 0 hi,
// lo, set 1 hi, lo) of C3F_FRAGS uint4 -- one coalesced 1-KB load per wave and K step
// instead of 32 scattered rows.
#define C3F_FRAGS 4608
__device__ __forceinline__ int c3f_src_off(int t) {
  const int lane = t & 63, s = (t >> 6) % 36, nt = t / 2304;
  return (32 * nt + (lane & 31)) * 576 + (s >> 2) * 64 + 16 * (s & 3) + 8 * (lane >> 5);
}
struct C3fPack {
  const bf16_t* src[4];   // set 0 hi, lo, set 1 hi, lo (null planes are skipped)
  uint4* out;             // 4 * C3F_FRAGS, or null: no pack
};
__device__ __forceinline__ void c3f_pack_range(const C3fPack& p, int i0, int stride) {
  for (int i = i0; i < 4 * C3F_FRAGS; i += stride) {
    const int q = i / C3F_FRAGS;
    const bf16_t* src = p.src[q];
    if (src != nullptr) p.out[i] = *reinterpret_cast<const uint4*>(src + c3f_src_off(i - q * C3F_FRAGS));
  }
}

struct C2fPack {
  const bf16_t* src[4];   // set 0 hi, lo, set 1 hi, lo (null planes are skipped)
  uint4* out;             // 4 * C2F_FRAGS, or null: no pack
  int bf16;               // bf16 forward layout: two planes (set 0, set 1 = src[0], src[2])
};
__device__ __forceinline__ void c2f_pack_range(const C2fPack& p, int i0, int stride) {
  for (int i = i0; i < 4 * C2F_FRAGS; i += stride) {
    if (p.bf16) {
      if (i >= 2 * C2F_FRAGS) break;
      const int q = i / C2F_FRAGS;
      const bf16_t* src = p.src[2 * q];
      if (src != nullptr) p.out[i] = *reinterpret_cast<const uint4*>(src + c2b_src_off(i - q * C2F_FRAGS));
      continue;
    }
    const int q = i / C2F_FRAGS;
    const bf16_t* src = p.src[q];
    if (src != nullptr) p.out[i] = *reinterpret_cast<const uint4*>(src + c2f_src_off(i - q * C2F_FRAGS));
  }
}

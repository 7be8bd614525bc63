// MFMA weight-gradient GEMM (igemm_wgrad_body) as a block-level device body, shared
// by csrc/conv_mfma.hip (igemm_wgrad_kernel) and csrc/sumtree.hip
// (fc_wgrad_head_prio_kernel: the fc weight gradient, the head weight gradient and
// the priority write-back in one launch).
#pragma once
#include "mfma_common.h"

struct WgradDesc {
  const bf16_t* dy;           // [Mred][ldd] rows = output pixels / samples
  const void* x;              // mode 0: bf16 [Mred][ldx]; 1: NHWC bf16; 2: u8 frame ring
  const int32_t* frame_slots;
  float* slab;                // [nsplit][Co][Kc] fp32 partial sums
  float* bias_slab;           // [nsplit][Co] (optional)
  int N, H, W, Cin;
  int OH, OW, KH, KW;
  int stride, pad_h, pad_w, mode;
  int Co, Kc, ldd, ldx;
  int rows_per_split, Mred;
  double* norm_part;          // optional: per-wave sum of squares of this (final) gradient tile
  int norm_slot0;             // first slot; slot = norm_slot0 + 4 * linear block + wave
  int pad0;
  // fp32-accurate ("split") mode: lo planes of dY and X (x_lo null for the exact
  // uint8 frames of mode 2); see igemm_wgrad_body's SP
  const bf16_t* dy_lo;
  const void* x_lo;
};

// =====================================================================================
// weight gradient: dW[Co][Kc] partial over a slice of the reduction rows
// =====================================================================================

// Design: a block owns CT x NT 64x64 output tiles (CT along Co, NT along Kc) of
// one split-K slice; wave w owns tile (w / NT, w % NT), and all waves walk the
// slice's reduction rows in 64-row steps.  Each step stages CT dY images and NT
// X images (64 rows x 128 B each) in LDS once, so dY is read from L2 / Infinity
// Cache Kc/(64 NT) times instead of Kc/64 times -- the wgrad GEMMs are bound by
// those bytes (measured: 64x64 blocks re-read dY per Kc tile, ~170 MB for conv2),
// not by MFMA or VALU.  All global reads are buffer loads: dY and dense X rows
// are affine in the row index; im2col / s2d-ring X rows come from a per-block
// LDS table of pixel byte offsets built in the prologue (rows past the split end
// hold BUF_OOB -> zeros).  The bias gradient is 2 extra MFMAs per k-step against
// an all-ones fragment, done by the waves owning Kc tile 0 -- no VALU sums.
#define WG_ROWS 64
#define WG_IMG 8192                     // one 64-row x 128-B operand image
#define WG_TBL 1024                     // u32 row-offset table entries (4 KB; dense mode: none)

// MODE: X-operand source (0 dense rows, 1 NHWC im2col (pad 0), 2 s2d uint8 ring).
// OWC/OHWC: output width / pixels per image as compile-time constants (0 = runtime);
// only the prologue divides.  CT x NT (<= 4) output tiles per block; the block
// always has 4 waves (all stage; waves past CT * NT do not compute).
// SP: fp32-accurate operands.  0: bf16; 1: dY and X both hi + lo (three MFMAs per
// fragment pair: hi.hi + lo.hi + hi.lo); 2: dY hi + lo, X exact in bf16 (uint8
// frames: two MFMAs).  The lo images sit after the hi images of each stage.
// Two-tile blocks (CT * NT == 2, split mode's conv2 shape: the hi + lo images of a
// 4-tile block do not fit two stages) pair the waves instead of idling two: waves w
// and w + 2 own the same tile and take the two 32-row halves of every 64-row step,
// and the pair's accumulators are summed through LDS at the end (fixed order).
// NSW: LDS stages.  Split-mode MODE 0 / 1 operands go global -> LDS by buffer LDS-DMA
// (lane sources chosen so the fixed slots receive the swz_tr image; rows past the split
// end read zeros through the buffer range check) into an NSW-deep ring (conv2 / conv3 /
// fc weight gradients 36 / 19 / 29 -> 34 / 15 / 26 us); MODE 2's uint8 frames are
// converted on the way, so it stays register-staged (two stages), as does bf16.
template <int MODE, int OWC, int OHWC, int CT, int NT, int SP = 0, int NSW = 2>
__device__ __forceinline__ void igemm_wgrad_body(const WgradDesc& d, int lin, int gx, int gy, int gz) {
  static_assert(CT * NT <= 4, "at most 4 output tiles per block");
  static_assert(SP != 1 || MODE != 2, "mode 2 X is exact: SP = 2");
  constexpr int NLO = SP == 0 ? 0 : (SP == 1 ? CT + NT : CT);
  constexpr int NIMG = CT + NT + NLO;
  constexpr int STAGE = NIMG * WG_IMG;
  constexpr int NTHR = 256;
  // dense rows (MODE 0) need no row table: 80 KB for a 4-tile block, two blocks per CU
  constexpr int TBL = MODE == 0 ? 0 : WG_TBL;
  // bf16 (SP 0) stays register-staged too: measured tie / 1-5 % slower with the ring
  constexpr bool DMA = MODE != 2 && SP != 0;
  constexpr int NS = DMA ? NSW : 2;
  static_assert(NS * STAGE + TBL * 4 <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NS * STAGE + TBL * 4];
  uint32_t* tbl = reinterpret_cast<uint32_t*>(smem + NS * STAGE);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // XCD-contiguous order: the Kc / Co blocks of one split (same dY rows, overlapping
  // input pixels) and neighbouring splits run on one XCD's L2
  const int wg = xcd_swizzle(lin, gx * gy * gz);
  const int bx = wg % gx, byz = wg / gx;
  const int kcb = bx * NT;               // first 64-wide Kc tile of the block
  const int cob = (byz % gy) * CT; // first 64-wide Co tile
  const int split = byz / gy;
  const int r_begin = split * d.rows_per_split;
  const int r_end = min(d.Mred, r_begin + d.rows_per_split);
  const int nst = (r_end - r_begin + WG_ROWS - 1) / WG_ROWS;
  const int trows = nst * WG_ROWS;
  const uint32_t OW = OWC ? OWC : d.OW;
  const uint32_t OHW = OHWC ? OHWC : d.OH * d.OW;

  // ---------------- prologue: per-row X pixel byte offsets (MODE 1 / 2)
  if (MODE == 1) {
    for (int r = tid; r < trows; r += NTHR) {
      const uint32_t m = r_begin + r;
      uint32_t e = BUF_OOB;
      if ((int)m < r_end) {
        const uint32_t img = udiv<OHWC>(m, OHW), rem = m - img * OHW;
        const uint32_t oh = udiv<OWC>(rem, OW), ow = rem - oh * OW;
        e = (uint32_t)(((img * d.H + oh * d.stride) * d.W + ow * d.stride) * d.Cin) * 2u;
      }
      tbl[r] = e;
    }
  } else if (MODE == 2) {
    for (int i = tid; i < d.Cin * trows; i += NTHR) {
      const int c = i / trows, r = i - c * trows;
      const uint32_t m = r_begin + r;
      uint32_t e = BUF_OOB;
      if ((int)m < r_end) {
        const uint32_t img = udiv<OHWC>(m, OHW), rem = m - img * OHW;
        const uint32_t oh = udiv<OWC>(rem, OW), ow = rem - oh * OW;
        e = (uint32_t)d.frame_slots[img * d.Cin + c] * 7056u + ((oh * 21 + ow) << 4);
      }
      tbl[i] = e;
    }
  }
  __syncthreads();

  // ---------------- staging geometry (each image: 64 rows; thread rows srow, srow + 32;
  // chunk sc -- with DMA, the chunk that lands in the thread's fixed slot tid & 7 of
  // the swz_tr image: (tid & 7) ^ (s(srow) << 1), the same for srow + 32)
  const int srow = tid >> 3;
  const int sc = DMA ? ((tid & 7) ^ ((((srow >> 1) & 1) | (((srow >> 3) & 1) << 1)) << 1)) : (tid & 7);
  const __amdgpu_buffer_rsrc_t dy_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(d.dy), (short)0, r_end * d.ldd * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t x_rs = MODE == 0
      ? __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(d.x), (short)0, r_end * d.ldx * 2, 0x00020000)
      : buf_rsrc(d.x);
  const __amdgpu_buffer_rsrc_t dyl_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(SP ? d.dy_lo : d.dy), (short)0, r_end * d.ldd * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t xl_rs = MODE == 0
      ? __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(SP == 1 ? d.x_lo : d.x), (short)0, r_end * d.ldx * 2,
                                          0x00020000)
      : buf_rsrc(SP == 1 ? d.x_lo : d.x);
  const uint32_t dy_off = (uint32_t)(((r_begin + srow) * d.ldd + cob * 64 + sc * 8) * 2);
  const uint32_t dy_r32 = (uint32_t)(32 * d.ldd * 2), dy_step = (uint32_t)(WG_ROWS * d.ldd * 2);
  const uint32_t x_off = (uint32_t)(((r_begin + srow) * d.ldx + kcb * 64 + sc * 8) * 2);
  const uint32_t x_r32 = (uint32_t)(32 * d.ldx * 2), x_step = (uint32_t)(WG_ROWS * d.ldx * 2);
  // MODE 1: Kc tile t = (tap, channel block); tap shifts the pixel by (kh W + kw) Cin
  uint32_t x_tap[NT];
  // MODE 2: lane = row, wave = s2d block b of every Kc tile; frame c / tap per tile
  int x2_tb[NT];
  const int x2_row = lane, x2_b = wv;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    x_tap[t] = 0;
    x2_tb[t] = 0;
    if (MODE == 1) {
      const int cpb = d.Cin >> 6, kt = kcb + t;
      const int tap = kt / cpb, cb = kt - tap * cpb;
      const int kh = tap / d.KW, kw = tap - kh * d.KW;
      x_tap[t] = (uint32_t)(((kh * d.W + kw) * d.Cin + (cb << 6) + sc * 8) * 2);
    } else if (MODE == 2) {
      const int q = 4 * (kcb + t) + x2_b, tap = q / d.Cin, c = q - tap * d.Cin;
      x2_tb[t] = c * trows;
      x_tap[t] = (uint32_t)(((tap >> 1) * 21 + (tap & 1)) << 4);
    }
  }

  struct Regs {
    uint4 dy[CT][2];
    uint4 x[NT][2];
    uint4 dyl[CT][2];
    uint4 xl[NT][2];
  };

  auto load_step = [&](int st, Regs& R) {
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const uint32_t o = dy_off + st * dy_step + c * 128;
      R.dy[c][0] = buf_ld16(dy_rs, o, 0);
      R.dy[c][1] = buf_ld16(dy_rs, o + dy_r32, 0);
      if (SP) {
        R.dyl[c][0] = buf_ld16(dyl_rs, o, 0);
        R.dyl[c][1] = buf_ld16(dyl_rs, o + dy_r32, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (MODE == 0) {
        const uint32_t o = x_off + st * x_step + t * 128;
        R.x[t][0] = buf_ld16(x_rs, o, 0);
        R.x[t][1] = buf_ld16(x_rs, o + x_r32, 0);
        if (SP == 1) {
          R.xl[t][0] = buf_ld16(xl_rs, o, 0);
          R.xl[t][1] = buf_ld16(xl_rs, o + x_r32, 0);
        }
      } else if (MODE == 1) {
        const uint32_t* tb = tbl + st * WG_ROWS + srow;
        R.x[t][0] = buf_ld16(x_rs, tb[0] + x_tap[t], 0);
        R.x[t][1] = buf_ld16(x_rs, tb[32] + x_tap[t], 0);
        if (SP == 1) {
          R.xl[t][0] = buf_ld16(xl_rs, tb[0] + x_tap[t], 0);
          R.xl[t][1] = buf_ld16(xl_rs, tb[32] + x_tap[t], 0);
        }
      } else {
        R.x[t][0] = buf_ld16(x_rs, tbl[x2_tb[t] + st * WG_ROWS + x2_row] + x_tap[t], 0);
      }
    }
  };

  // image i of stage stg: i < CT: dY co tile i; i >= CT: X kc tile i - CT; then the
  // lo planes: CT + NT + c = dY lo tile c, 2 CT + NT + t = X lo tile t
  auto img = [&](int stg, int i) -> uint8_t* { return smem + stg * STAGE + i * WG_IMG; };

  auto write_step = [&](int stg, const Regs& R) {
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      *reinterpret_cast<uint4*>(img(stg, c) + swz_tr(srow, sc)) = R.dy[c][0];
      *reinterpret_cast<uint4*>(img(stg, c) + swz_tr(srow + 32, sc)) = R.dy[c][1];
      if (SP) {
        *reinterpret_cast<uint4*>(img(stg, CT + NT + c) + swz_tr(srow, sc)) = R.dyl[c][0];
        *reinterpret_cast<uint4*>(img(stg, CT + NT + c) + swz_tr(srow + 32, sc)) = R.dyl[c][1];
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      uint8_t* X = img(stg, CT + t);
      if (MODE != 2) {
        *reinterpret_cast<uint4*>(X + swz_tr(srow, sc)) = R.x[t][0];
        *reinterpret_cast<uint4*>(X + swz_tr(srow + 32, sc)) = R.x[t][1];
        if (SP == 1) {
          uint8_t* XL = img(stg, 2 * CT + NT + t);
          *reinterpret_cast<uint4*>(XL + swz_tr(srow, sc)) = R.xl[t][0];
          *reinterpret_cast<uint4*>(XL + swz_tr(srow + 32, sc)) = R.xl[t][1];
        }
      } else {
        // 16 uint8 of s2d block x2_b -> bf16 chunks 2 x2_b, 2 x2_b + 1 of row x2_row
        *reinterpret_cast<uint4*>(X + swz_tr(x2_row, 2 * x2_b)) = u8x8_to_bf16x8(R.x[t][0].x, R.x[t][0].y);
        *reinterpret_cast<uint4*>(X + swz_tr(x2_row, 2 * x2_b + 1)) = u8x8_to_bf16x8(R.x[t][0].z, R.x[t][0].w);
      }
    }
  };

  constexpr bool PAIR = CT * NT == 2;
  const int tw = PAIR ? (wv & 1) : wv;
  const bool active = PAIR || wv < CT * NT;
  const int wc = active ? tw / NT : 0, wn = active ? tw - (tw / NT) * NT : 0;   // this wave's (co, kc) tile
  const int kk0 = PAIR ? (wv >> 1) : 0, kk1 = PAIR ? kk0 + 1 : 2;              // 32-row halves of a step
  const bool do_bias = active && d.bias_slab != nullptr && kcb + wn == 0;
  // acc[i][j] = D[kc][co] (swapped operands): lane holds kc 16j + 4g + {0..3} of co 16i + (lane&15)
  f32x4 acc[4][4], accb[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    accb[a] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u));

  auto compute = [&](int stg) {
    if (!active) return;
    const uint8_t* D = img(stg, wc);
    const uint8_t* X = img(stg, CT + wn);
    const uint8_t* DL = img(stg, CT + NT + wc);
    const uint8_t* XL = img(stg, 2 * CT + NT + wn);
#pragma unroll
    for (int kk = kk0; kk < kk1; ++kk) {
      bf16x8 a[4], b[4], al[4], bl[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = tr_frag8(D, kk, 16 * t, lane);
        if (SP) al[t] = tr_frag8(DL, kk, 16 * t, lane);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        b[t] = tr_frag8(X, kk, 16 * t, lane);
        if (SP == 1) bl[t] = tr_frag8(XL, kk, 16 * t, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (SP) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], al[i], acc[i][j], 0, 0, 0);
          if (SP == 1) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j], a[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
        }
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (SP) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, al[i], accb[i], 0, 0, 0);
          accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, a[i], accb[i], 0, 0, 0);
        }
      }
    }
  };

  // DMA: step st's images into stage st % NS, NS - 1 steps ahead; one barrier per step
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem;
  auto issue_step = [&](int st) {
    const uint32_t base = lds0 + (uint32_t)(st % NS) * STAGE + (uint32_t)wv * 1024u;
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const uint32_t o = dy_off + st * dy_step + c * 128;
      const uint32_t l = __builtin_amdgcn_readfirstlane(base + c * WG_IMG);
      bdma16(dy_rs, o, l);
      bdma16(dy_rs, o + dy_r32, l + 4096);
      if (SP) {
        const uint32_t ll = __builtin_amdgcn_readfirstlane(base + (CT + NT + c) * WG_IMG);
        bdma16(dyl_rs, o, ll);
        bdma16(dyl_rs, o + dy_r32, ll + 4096);
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      uint32_t o0, o1;
      if (MODE == 0) {
        o0 = x_off + st * x_step + t * 128;
        o1 = o0 + x_r32;
      } else {
        const uint32_t* tb = tbl + st * WG_ROWS + srow;
        o0 = tb[0] + x_tap[t];
        o1 = tb[32] + x_tap[t];
      }
      const uint32_t l = __builtin_amdgcn_readfirstlane(base + (CT + t) * WG_IMG);
      bdma16(x_rs, o0, l);
      bdma16(x_rs, o1, l + 4096);
      if (SP == 1) {
        const uint32_t ll = __builtin_amdgcn_readfirstlane(base + (2 * CT + NT + t) * WG_IMG);
        bdma16(xl_rs, o0, ll);
        bdma16(xl_rs, o1, ll + 4096);
      }
    }
  };
  constexpr int DPW = 2 * (CT + NT + NLO);   // DMAs per wave per step
  if (DMA && nst > 0) {
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
      if (p < nst) issue_step(p);
    for (int st = 0; st < nst; ++st) {
      vmcnt_le(min(NS - 2, nst - 1 - st) * DPW);
      __syncthreads();
      if (st + NS - 1 < nst) issue_step(st + NS - 1);
      compute(st % NS);
    }
  }

  // MODE 2: two register stages + two LDS stages, straight-line (loads past the end
  // re-read the last step -- never computed)
  Regs RA, RB;
  const int SL = nst - 1;
  if (!DMA && nst > 0) {
    load_step(0, RA);
    load_step(min(1, SL), RB);
    write_step(0, RA);
    __syncthreads();
    load_step(min(2, SL), RA);
    int st = 0;
    for (; st + 1 < nst; st += 2) {
      compute(0);
      write_step(1, RB);
      __syncthreads();
      load_step(min(st + 3, SL), RB);
      compute(1);
      write_step(0, RA);
      __syncthreads();
      load_step(min(st + 4, SL), RA);
    }
    if (st < nst) compute(0);
  }

  // ---------------- this wave's fp32 partial tile -> slab[split][co][kc] (float4 along kc)
  const int lin_blk = lin;
  if (PAIR) {
    // waves 2, 3 hand their half-step sums to waves 0, 1 (acc then accb, lane-major)
    __syncthreads();                       // every wave is done reading the stages
    f32x4* red = reinterpret_cast<f32x4*>(smem) + (wv & 1) * (20 * 64) + lane;
    if (wv >= 2) {
#pragma unroll
      for (int q = 0; q < 16; ++q) red[q * 64] = acc[q >> 2][q & 3];
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(16 + i) * 64] = accb[i];
    }
    __syncthreads();
    if (wv >= 2) {
      if (d.norm_part != nullptr && lane == 0) d.norm_part[d.norm_slot0 + 4 * lin_blk + wv] = 0.0;
      return;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q >> 2][q & 3] += red[q * 64];
#pragma unroll
    for (int i = 0; i < 4; ++i) accb[i] += red[(16 + i) * 64];
  }
  if (!active) {
    if (d.norm_part != nullptr && lane == 0) d.norm_part[d.norm_slot0 + 4 * lin_blk + wv] = 0.0;
    return;
  }
  const int g = lane >> 4, pl = lane & 15;
  if (d.norm_part != nullptr) {
    // the tile is the FINAL gradient (single split): its squared norm feeds the clip
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ss += acc[i][j][r] * acc[i][j][r];
    if (do_bias && g == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) ss += accb[i][0] * accb[i][0];
    }
    ss = wave_sum_dpp(ss);
    if (lane == 0) d.norm_part[d.norm_slot0 + 4 * lin_blk + wv] = (double)ss;
  }
  float* slab = d.slab + (int64_t)split * d.Co * d.Kc;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = (cob + wc) * 64 + 16 * i + pl;
      *reinterpret_cast<f32x4*>(slab + (int64_t)co * d.Kc + (kcb + wn) * 64 + 16 * j + 4 * g) = acc[i][j];
    }
  if (do_bias && g == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) d.bias_slab[(int64_t)split * d.Co + (cob + wc) * 64 + 16 * i + pl] = accb[i][0];
  }
}

// Block shape choice (host): fewest re-read bytes -- X is read once per Co group
// (ct / CT times), dY once per Kc group (kt / NT times); 4-tile shapes keep every
// wave busy.  Index into {CT,NT} = {1,4} {2,2} {4,1} {1,3} {1,1} {1,2} {2,1}.
// Split mode doubles the images per stage, so only shapes with CT + NT <= 4
// (2 CT + NT <= 6 with SP = 2's exact X) fit two stages in LDS next to the row table.
struct WgShape { int c, n; };
#define WG_NSHAPES 7
static inline int wgrad_shape(int kt, int ct, int Kc, int Co, int sp = 0) {
  const WgShape cands[WG_NSHAPES] = {{1, 4}, {2, 2}, {4, 1}, {1, 3}, {1, 1}, {1, 2}, {2, 1}};
  int best = 4;
  double bc = 1e300;
  for (int i = 0; i < WG_NSHAPES; ++i) {
    const WgShape c = cands[i];
    if (kt % c.n || ct % c.c) continue;
    if (sp == 1 && c.c + c.n > 4) continue;
    if (sp == 2 && 2 * c.c + c.n > 6) continue;
    if (sp == 0 && i >= 5) continue;     // the 3-tile shapes are for split mode only
    const double cost = (double)(ct / c.c) * (double)Kc + (double)(kt / c.n) * (double)Co;
    if (cost < bc) { bc = cost; best = i; }
  }
  return best;
}

// fp32-class ("split") trunk kernels of the IMPALA-deep ResNet dueling Q-net
// (BASELINE.json config 5 at Runtime.dtype = fp32; the bf16-operand kernels are
// csrc/impala.hip, whose layouts and tilings these follow).
//
// Storage: activations and gradients are fp32 planar-16 tensors ((N, C/16, H, W, 16)
// floats, 64-byte pixel rows).  Staging into LDS splits every value v into bf16
// hi = bf16(v) and lo = bf16(v - hi) (v = hi + lo to 2^-17, csrc/mfma_common.h
// split_pk_bf16) held as TWO plane sets of the bf16 kernels' 32-byte-row layout, so
// every fragment read is the conflict-free read of csrc/impala.hip, issued once per
// plane.  Weights arrive as packed hi + lo MFMA fragments (sconv_pack of the hi and
// the lo plane of the bf16 weight copy).  Each product is hi*hi + lo*hi + hi*lo on
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation (the lo*lo term is below 2^-16
// relative); the uint8 frame inputs of stack 1 are exact in bf16, so those convs
// issue hi*x + lo*x only.  Epilogues, the max pool and its backward run in fp32.
//
//   sconv_fwd_split     3x3 correlation (+ bias, mask, add, ReLU epilogue; or the
//                       fused 3x3 / s2 max pool with argmax codes: conv tile in LDS
//                       as fp32) -- forward convs and data gradients
//   resblock_fwd_split  x + conv1(relu(conv0(relu(x)))) with conv0's output in LDS
//                       (hi / lo); conv0's output saved for the training rows; the
//                       last block may write its output as bf16 hi / lo planes
//                       straight into the fc GEMM's operand rows
//   sconv_wgrad_split   weight / bias gradient partials (same slab format as
//                       sconv_wgrad: reduced by sconv_wgrad_reduce, csrc/impala.hip)
//   maxpool_bwd_split   the pool backward as a gather (fp32)
//   merge_split         fp32 = hi + lo (the fc data gradient into the trunk)
#include "mfma_common.h"

struct SconvSDesc {
  const void* x;              // fp32 planar input, or (mode 3) the uint8 s2d frame ring
  const int32_t* slots;       // mode 3: [N][4] frame-ring slots
  const bf16_t* wf;           // packed weight fragments, hi / lo
  const bf16_t* wf_lo;
  const bf16_t* wf2;          // second weight set (images >= n_switch), or null
  const bf16_t* wf2_lo;
  const float* bias;
  const float* bias2;
  const float* add;           // fp32, output layout, or null
  const float* mask;          // output multiplied by (mask > 0), fp32 output layout, or null
  float* y;                   // fp32 planar output (pooled output when POOL)
  uint8_t* mask_out;          // POOL: argmax codes [N][planes][Ho][Wo][16], or null
  int64_t x_img, y_img, add_img, mask_img;
  int N, n_switch, relu_in, relu_out;
  float scale;
  int pad0;                   // POOL: argmax codes for images < pad0 only (0 = all)
};

// ---- split helpers
__device__ __forceinline__ void split8s(const float4 a, const float4 b, uint4& hi, uint4& lo) {
  split_pk_bf16(a.x, a.y, hi.x, lo.x);
  split_pk_bf16(a.z, a.w, hi.y, lo.y);
  split_pk_bf16(b.x, b.y, hi.z, lo.z);
  split_pk_bf16(b.z, b.w, hi.w, lo.w);
}
__device__ __forceinline__ float4 relu4s(float4 v) {
  return make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
}
// ReLU of v = hi + lo on packed planes: sign(v) = sign(hi) (|lo| <= ulp(hi) / 2, and hi
// is 0 only when v is), so lo survives exactly where hi > 0
__device__ __forceinline__ void relu_split(uint4& h, uint4& l) {
  l = make_uint4(mask_bf16x2(l.x, h.x), mask_bf16x2(l.y, h.y), mask_bf16x2(l.z, h.z), mask_bf16x2(l.w, h.w));
  h = make_uint4(relu_pk16(h.x), relu_pk16(h.y), relu_pk16(h.z), relu_pk16(h.w));
}
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Stage SROWS fp32 input rows starting at global row row0 (cols [-1, W], zero outside
// the image) of image n as hi planes at xs and lo planes at xs + P * plane_pix * 32;
// pixels past the SROWS x (W+2) block up to plane_pix are zeroed in both sets.
// One item = 8 channels (two float4 loads), BATCH items in flight per thread.
// ROLLED keeps the batch loop rolled (a caller holding many live accumulators).
template <int P, int H, int W, int SROWS, int NTHR, int BATCH, bool ROLLED = false>
__device__ __forceinline__ void stage_rows_split(uint8_t* xs, int plane_pix, const float* x, int64_t x_img, int n,
                                                 int row0, int relu, int tid) {
  constexpr int WP = W + 2, BLK = SROWS * WP;
  constexpr int NCK = P * BLK * 2;
  const float* xi = x + (int64_t)n * x_img;
  uint8_t* xl = xs + P * plane_pix * 32;
  auto batch = [&](int base) {
    float4 va[BATCH], vb[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int i = base + k * NTHR + tid;
      const int hf = i & 1, pix = i >> 1;
      const int p = pix / BLK, rem = pix - (pix / BLK) * BLK;
      const int lr = rem / WP, c = rem - (rem / WP) * WP;
      const int h = row0 + lr, w = c - 1;
      va[k] = vb[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < NCK && h >= 0 && h < H && w >= 0 && w < W) {
        const float* s = xi + ((int64_t)(p * H + h) * W + w) * 16 + hf * 8;
        va[k] = ld4(s);
        vb[k] = ld4(s + 4);
      }
    }
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      const int i = base + k * NTHR + tid;
      const int hf = i & 1, pix = i >> 1;
      const int p = pix / BLK, rem = pix - (pix / BLK) * BLK;
      if (i < NCK) {
        uint4 hi, lo;
        split8s(relu ? relu4s(va[k]) : va[k], relu ? relu4s(vb[k]) : vb[k], hi, lo);
        const int o = (p * plane_pix + rem) * 32 + hf * 16;
        *reinterpret_cast<uint4*>(xs + o) = hi;
        *reinterpret_cast<uint4*>(xl + o) = lo;
      }
    }
  };
  if constexpr (ROLLED) {
#pragma unroll 1
    for (int base = 0; base < NCK; base += NTHR * BATCH) batch(base);
  } else {
    for (int base = 0; base < NCK; base += NTHR * BATCH) batch(base);
  }
  const int slack = plane_pix - BLK;
  for (int i = tid; i < 2 * P * slack * 2; i += NTHR) {
    const int set = i / (P * slack * 2), r0 = i - set * (P * slack * 2);
    const int p = r0 / (slack * 2), r = r0 - p * slack * 2;
    *reinterpret_cast<uint4*>(xs + set * P * plane_pix * 32 + (p * plane_pix + BLK) * 32 + r * 16) =
        make_uint4(0, 0, 0, 0);
  }
}

// stage_rows_split in two halves, every load of the block in flight at once: load()
// issues them into registers, the caller zero-fills what it needs meanwhile (zero_slack:
// the plane slack past the SROWS x (W+2) block), store() splits them into the hi / lo
// planes (resblock 16 ch x 42²: 171 -> 158 µs against the batched stage_rows_split).
template <int P, int H, int W, int SROWS, int NTHR>
struct RowLoads {
  static constexpr int WP = W + 2, BLK = SROWS * WP, NCK = P * BLK * 2, K = (NCK + NTHR - 1) / NTHR;
  float4 va[K], vb[K];
  __device__ __forceinline__ void load(const float* x, int64_t x_img, int n, int row0, int tid) {
    const float* xi = x + (int64_t)n * x_img;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = k * NTHR + tid;
      const int hf = i & 1, pix = i >> 1;
      const int p = pix / BLK, rem = pix - (pix / BLK) * BLK;
      const int lr = rem / WP, c = rem - (rem / WP) * WP;
      const int h = row0 + lr, w = c - 1;
      va[k] = vb[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < NCK && h >= 0 && h < H && w >= 0 && w < W) {
        const float* s = xi + ((int64_t)(p * H + h) * W + w) * 16 + hf * 8;
        va[k] = ld4(s);
        vb[k] = ld4(s + 4);
      }
    }
  }
  __device__ __forceinline__ void store(uint8_t* xs, int plane_pix, int relu, int tid) const {
    uint8_t* xl = xs + P * plane_pix * 32;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = k * NTHR + tid;
      const int hf = i & 1, pix = i >> 1;
      const int p = pix / BLK, rem = pix - (pix / BLK) * BLK;
      if (i < NCK) {
        uint4 hi, lo;
        split8s(relu ? relu4s(va[k]) : va[k], relu ? relu4s(vb[k]) : vb[k], hi, lo);
        const int o = (p * plane_pix + rem) * 32 + hf * 16;
        *reinterpret_cast<uint4*>(xs + o) = hi;
        *reinterpret_cast<uint4*>(xl + o) = lo;
      }
    }
  }
  static __device__ __forceinline__ void zero_slack(uint8_t* xs, int plane_pix, int tid) {
    const int slack = plane_pix - BLK;
    for (int i = tid; i < 2 * P * slack * 2; i += NTHR) {
      const int set = i / (P * slack * 2), r0 = i - set * (P * slack * 2);
      const int p = r0 / (slack * 2), r = r0 - p * slack * 2;
      *reinterpret_cast<uint4*>(xs + set * P * plane_pix * 32 + (p * plane_pix + BLK) * 32 + r * 16) =
          make_uint4(0, 0, 0, 0);
    }
  }
};

// The 4 stacked uint8 frames as 4-channel bf16 pixels (8 bytes; exact), rows [row0,
// row0 + SROWS) x cols [-1, W] of image n (csrc/impala.hip stage_ring4).
template <int H, int W, int SROWS, int NTHR>
__device__ __forceinline__ void stage_ring4_split(uint8_t* xs, int plane_pix, const uint8_t* ring,
                                                  const int32_t* slots, int n, int row0, int tid) {
  constexpr int WP = W + 2, G4 = W / 4;
  static_assert(W % 4 == 0, "ring rows are s2d blocks of 4 pixels");
  const int32_t* sl = slots + (int64_t)n * 4;
  const int64_t f0 = (int64_t)sl[0] * 7056, f1 = (int64_t)sl[1] * 7056;
  const int64_t f2 = (int64_t)sl[2] * 7056, f3 = (int64_t)sl[3] * 7056;
  for (int i = tid; i < SROWS * G4; i += NTHR) {
    const int lr = i / G4, g = i - (i / G4) * G4;
    const int h = row0 + lr;
    uint32_t u0 = 0, u1 = 0, u2 = 0, u3 = 0;
    if (h >= 0 && h < H) {
      const int o = ((h >> 2) * 21 + g) * 16 + (h & 3) * 4;
      u0 = *reinterpret_cast<const uint32_t*>(ring + f0 + o);
      u1 = *reinterpret_cast<const uint32_t*>(ring + f1 + o);
      u2 = *reinterpret_cast<const uint32_t*>(ring + f2 + o);
      u3 = *reinterpret_cast<const uint32_t*>(ring + f3 + o);
    }
    uint8_t* dst = xs + (lr * WP + 4 * g + 1) * 8;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      *reinterpret_cast<uint2*>(dst + 8 * k) = make_uint2(cvt_pk_bf16(ubyte(u0, k), ubyte(u1, k)),
                                                          cvt_pk_bf16(ubyte(u2, k), ubyte(u3, k)));
  }
  for (int i = tid; i < SROWS * 2; i += NTHR) {
    const int lr = i >> 1, c = (i & 1) ? WP - 1 : 0;
    *reinterpret_cast<uint2*>(xs + (lr * WP + c) * 8) = make_uint2(0, 0);
  }
  for (int i = SROWS * WP + tid; i < plane_pix; i += NTHR) *reinterpret_cast<uint2*>(xs + i * 8) = make_uint2(0, 0);
}

// 4 uint8 frames of the s2d ring as channels 0..3 of a 16-channel bf16 plane (exact),
// rows [row0, row0 + SROWS) x cols [-1, W] (the weight gradient's mode-2 staging)
template <int H, int W, int SROWS, int NTHR>
__device__ __forceinline__ void stage_ring16_split(uint8_t* xs, int plane_pix, const uint8_t* ring,
                                                   const int32_t* slots, int n, int row0, int tid) {
  constexpr int WP = W + 2, BLK = SROWS * WP;
  const int32_t* sl = slots + (int64_t)n * 4;
  const int64_t f0 = (int64_t)sl[0] * 7056, f1 = (int64_t)sl[1] * 7056;
  const int64_t f2 = (int64_t)sl[2] * 7056, f3 = (int64_t)sl[3] * 7056;
  for (int i = tid; i < BLK; i += NTHR) {
    const int lr = i / WP, c = i - (i / WP) * WP;
    const int h = row0 + lr, w = c - 1;
    uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0;
    if (h >= 0 && h < H && w >= 0 && w < W) {
      const int o = ((h >> 2) * 21 + (w >> 2)) * 16 + (h & 3) * 4 + (w & 3);
      b0 = ring[f0 + o]; b1 = ring[f1 + o]; b2 = ring[f2 + o]; b3 = ring[f3 + o];
    }
    *reinterpret_cast<uint4*>(xs + i * 32) =
        make_uint4(cvt_pk_bf16((float)b0, (float)b1), cvt_pk_bf16((float)b2, (float)b3), 0, 0);
    *reinterpret_cast<uint4*>(xs + i * 32 + 16) = make_uint4(0, 0, 0, 0);
  }
  for (int i = BLK + tid; i < plane_pix; i += NTHR) {
    *reinterpret_cast<uint4*>(xs + i * 32) = make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(xs + i * 32 + 16) = make_uint4(0, 0, 0, 0);
  }
}

// =====================================================================================
// forward / data-gradient correlation (+ fused 3x3/s2 max pool), split operands
// =====================================================================================
template <int CIN, int COUT, int H, int W, int R, int MODE, int POOL>
__global__ void __launch_bounds__(512) sconv_fwd_split_kernel(SconvSDesc d) {
  constexpr int NTHR = 512, NW = NTHR / 64;
  constexpr int P = CIN / 16, NT = COUT / 16;
  constexpr int WP = W + 2;
  constexpr int OROWS = POOL ? R + 1 : R;
  constexpr int SROWS = OROWS + 2;
  constexpr int PLANE = SROWS * WP + 24;
  constexpr int PIXB = MODE == 3 ? 8 : 32;
  constexpr int NSET = MODE == 3 ? 1 : 2;                // exact frames: no lo set
  constexpr int NCH = MODE == 3 ? 2 : (9 * P + 1) / 2;
  constexpr int MROWS = OROWS * WP;
  constexpr int NTILE = (MROWS + 15) / 16;
  constexpr int OPIX = POOL ? OROWS * W : 0;
  constexpr int XB = NSET * P * PLANE * PIXB;
  constexpr int LO = P * PLANE * PIXB;                   // byte offset of the lo set
  static_assert(!POOL || (R % 2) == 0, "pooled bands need an even row count");
  __shared__ __attribute__((aligned(16))) uint8_t xs[XB + NT * OPIX * 64];
  float* ot = reinterpret_cast<float*>(xs + XB);        // POOL: fp32 conv tile [NT][OROWS][W][16]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int band = blockIdx.x, n = blockIdx.y;
  const int o0 = POOL ? band * R - 1 : band * R;
  const bool second = d.wf2 != nullptr && n >= d.n_switch;
  const bf16_t* __restrict__ wf = second ? d.wf2 : d.wf;
  const bf16_t* __restrict__ wfl = second ? d.wf2_lo : d.wf_lo;
  const float* __restrict__ bias = second ? d.bias2 : d.bias;

  // fp32 input rows: every load in flight before the weight loads when they fit in 5
  // float4 pairs per thread (RowLoads; 5 vs 4: +0.4 % on the IMPALA step), batched through
  // stage_rows_split otherwise
  using Rows = RowLoads<P, H, W, SROWS, NTHR>;
  constexpr bool ONE_BATCH = MODE != 3 && Rows::K <= 5;
  Rows rows;
  if constexpr (ONE_BATCH) rows.load(reinterpret_cast<const float*>(d.x), d.x_img, n, o0 - 1, tid);

  bf16x8 wh[NCH][NT], wl[NCH][NT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      wh[c][nt] = *reinterpret_cast<const bf16x8*>(wf + ((int64_t)(c * NT + nt) * 64 + lane) * 8);
      wl[c][nt] = *reinterpret_cast<const bf16x8*>(wfl + ((int64_t)(c * NT + nt) * 64 + lane) * 8);
    }

  if constexpr (MODE == 3) {
    stage_ring4_split<H, W, SROWS, NTHR>(xs, PLANE, reinterpret_cast<const uint8_t*>(d.x), d.slots, n, o0 - 1, tid);
  } else if constexpr (ONE_BATCH) {
    Rows::zero_slack(xs, PLANE, tid);
    rows.store(xs, PLANE, d.relu_in, tid);
  } else {
    stage_rows_split<P, H, W, SROWS, NTHR, 4>(xs, PLANE, reinterpret_cast<const float*>(d.x), d.x_img, n, o0 - 1,
                                              d.relu_in, tid);
  }
  __syncthreads();

  const int kg = lane >> 4;
  int aoff[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (MODE == 3) {
      const int kh = c == 0 ? (kg >> 1) : 2;
      aoff[c] = (kh * WP + 2 * (kg & 1) + (lane & 15)) * 8;
      continue;
    }
    int pair = 2 * c + (kg >> 1);
    if (pair >= 9 * P) pair = 9 * P - 1;
    const int t = pair / P, p = pair - (pair / P) * P;
    aoff[c] = (p * PLANE + (t / 3) * WP + (t % 3) + (lane & 15)) * 32 + (kg & 1) * 16;
  }
  float* __restrict__ yi = d.y + (int64_t)n * d.y_img;
  const float* __restrict__ addi = d.add ? d.add + (int64_t)n * d.add_img : nullptr;
  const float* __restrict__ mski = d.mask ? d.mask + (int64_t)n * d.mask_img : nullptr;
  float4 bv[NT];                                                // bias: loaded once, not per tile
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) bv[nt] = bias ? ld4(bias + nt * 16 + 4 * kg) : make_float4(0.f, 0.f, 0.f, 0.f);

  for (int tile = wv; tile < NTILE; tile += NW) {
    const int q0 = tile * 16;
    const int q = q0 + (lane & 15);
    const int lh = q / WP, w = q - (q / WP) * WP;
    const int h = o0 + lh;
    const bool valid = lh < OROWS && w < W && (POOL || h < H);
    float4 am[NT], mm[NT];
    if (!POOL && valid) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int64_t off = ((int64_t)(nt * H + h) * W + w) * 16 + 4 * kg;
        if (addi) am[nt] = ld4(addi + off);
        if (mski) mm[nt] = ld4(mski + off);
      }
    }
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      bf16x8 xh, xl;
      if (MODE == 3) {
        const uint2 a = *reinterpret_cast<const uint2*>(xs + aoff[c] + q0 * 8);
        const uint2 b = *reinterpret_cast<const uint2*>(xs + aoff[c] + q0 * 8 + 8);
        xh = __builtin_bit_cast(bf16x8, make_uint4(a.x, a.y, b.x, b.y));
      } else {
        xh = *reinterpret_cast<const bf16x8*>(xs + aoff[c] + q0 * 32);
        xl = *reinterpret_cast<const bf16x8*>(xs + LO + aoff[c] + q0 * 32);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[c][nt], xh, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[c][nt], xh, acc[nt], 0, 0, 0);
        if (MODE != 3) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[c][nt], xl, acc[nt], 0, 0, 0);
      }
    }
    if (!valid) continue;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[nt][r] * d.scale;
      if (bias) {
        const float4 b = bv[nt];
        v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
      }
      if (POOL) {
        if (h < 0 || h >= H) v[0] = v[1] = v[2] = v[3] = -INFINITY;
        *reinterpret_cast<float4*>(ot + ((nt * OROWS + lh) * W + w) * 16 + 4 * kg) = make_float4(v[0], v[1], v[2], v[3]);
        continue;
      }
      if (mski) {
        const float4 m = mm[nt];
        v[0] = m.x > 0.f ? v[0] : 0.f;
        v[1] = m.y > 0.f ? v[1] : 0.f;
        v[2] = m.z > 0.f ? v[2] : 0.f;
        v[3] = m.w > 0.f ? v[3] : 0.f;
      }
      if (addi) {
        const float4 a = am[nt];
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      }
      if (d.relu_out) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      *reinterpret_cast<float4*>(yi + ((int64_t)(nt * H + h) * W + w) * 16 + 4 * kg) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  if constexpr (POOL) {
    // 3x3 / s2 / pad 1 max pool of the fp32 tile; one item per (plane, pooled pixel,
    // 4-channel quad); argmax code = kh*3 + kw of the first maximum in window order
    constexpr int HO = (H + 1) / 2, WO = (W + 1) / 2, PR = R / 2;
    __syncthreads();
    uint8_t* __restrict__ am_out = d.mask_out;
    const bool track = am_out != nullptr && (d.pad0 <= 0 || n < d.pad0);
    for (int it = tid; it < NT * PR * WO * 4; it += NTHR) {
      const int qd = it & 3, r1 = it >> 2;
      const int ow = r1 % WO, r2 = r1 / WO;
      const int pr = r2 % PR, nt = r2 / PR;
      const int oh = band * PR + pr;
      if (oh >= HO) continue;
      float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      int code[4] = {0, 0, 0, 0};
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int lr = 2 * pr + kh;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int wc = 2 * ow - 1 + kw;
          if (wc < 0 || wc >= W) continue;
          const float4 v = ld4(ot + ((nt * OROWS + lr) * W + wc) * 16 + 4 * qd);
          const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (f[c] > best[c]) { best[c] = f[c]; code[c] = kh * 3 + kw; }
        }
      }
      const int64_t po = (((int64_t)nt * HO + oh) * WO + ow) * 16 + 4 * qd;
      *reinterpret_cast<float4*>(yi + po) = make_float4(best[0], best[1], best[2], best[3]);
      if (track)
        *reinterpret_cast<uint32_t*>(am_out + (int64_t)n * NT * HO * WO * 16 + po) =
            code[0] | (code[1] << 8) | (code[2] << 16) | (code[3] << 24);
    }
  }
}

// =====================================================================================
// fused residual block forward (split): out = x + conv1(relu(conv0(relu(x))))
// =====================================================================================
struct ResSDesc {
  const float* x;
  const bf16_t* wf0; const bf16_t* wf0_lo; const bf16_t* wf0b; const bf16_t* wf0b_lo;
  const float* b0; const float* b0b;
  const bf16_t* wf1; const bf16_t* wf1_lo; const bf16_t* wf1b; const bf16_t* wf1b_lo;
  const float* b1; const float* b1b;
  float* ysave;                 // conv0 output (fp32) for images < n_save, or null
  void* out;                    // fp32 planar output, or (out_lo set) the bf16 hi plane
  bf16_t* out_lo;               // bf16 lo plane of the output (the fc operand rows), or null
  int64_t x_img, ysave_img, out_img;
  int N, n_switch, n_save, relu_out;
};

// All M tiles of an OROWS x WP output grid from the hi / lo LDS plane sets at img
// (lo set at img + lo_off bytes), relu on the fragments; epi(lh, w, nt, kg, acc)
// (RELU: apply relu to the staged planes per fragment; false when they were stored
// relu'd already)
// Per-tile operand of an epilogue loaded before the tile's MFMA chain (none by default)
struct NoPrefetch {
  struct T {};
  __device__ __forceinline__ T operator()(int, int, int) const { return T{}; }
};

// All M tiles of an OROWS x WP output grid from the hi / lo LDS plane sets at img (lo set
// at img + lo_off bytes); pf(lh, w, kg) is issued before each tile's MFMAs (its global
// loads overlap them instead of stalling the epilogue), epi(lh, w, nt, kg, acc, pf value).
// RELU: apply relu to the staged planes per fragment (false when stored relu'd already).
// A convolution's hi / lo weight fragments in registers (loaded by the caller, so their
// latency can hide behind other work)
template <int P, int NT>
struct WFrags {
  static constexpr int NCH = (9 * P + 1) / 2;
  bf16x8 h[NCH][NT], l[NCH][NT];
  __device__ __forceinline__ void load(const bf16_t* __restrict__ wf, const bf16_t* __restrict__ wfl, int lane) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        h[c][nt] = *reinterpret_cast<const bf16x8*>(wf + ((int64_t)(c * NT + nt) * 64 + lane) * 8);
        l[c][nt] = *reinterpret_cast<const bf16x8*>(wfl + ((int64_t)(c * NT + nt) * 64 + lane) * 8);
      }
  }
};

template <int P, int NT, int WP, int OROWS, int PLANE, int NTHR, bool RELU = true, typename Epi,
          typename Pf = NoPrefetch>
__device__ __forceinline__ void conv_grid_split(const uint8_t* img, int lo_off, const WFrags<P, NT>& wfr, int lane,
                                                int wv, Epi epi, Pf pf = Pf()) {
  constexpr int NCH = WFrags<P, NT>::NCH, NW = NTHR / 64;
  constexpr int NTILE = (OROWS * WP + 15) / 16;
  const auto& wh = wfr.h;
  const auto& wl = wfr.l;
  const int kg = lane >> 4;
  int aoff[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    int pair = 2 * c + (kg >> 1);
    if (pair >= 9 * P) pair = 9 * P - 1;
    const int t = pair / P, p = pair - (pair / P) * P;
    aoff[c] = (p * PLANE + (t / 3) * WP + (t % 3) + (lane & 15)) * 32 + (kg & 1) * 16;
  }
  for (int tile = wv; tile < NTILE; tile += NW) {
    const int q0 = tile * 16;
    const int q = q0 + (lane & 15);
    const int lh = q / WP, w = q - (q / WP) * WP;
    const auto pre = pf(lh, w, kg);
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      uint4 h = *reinterpret_cast<const uint4*>(img + aoff[c] + q0 * 32);
      uint4 l = *reinterpret_cast<const uint4*>(img + lo_off + aoff[c] + q0 * 32);
      if (RELU) relu_split(h, l);
      const bf16x8 xh = __builtin_bit_cast(bf16x8, h), xl = __builtin_bit_cast(bf16x8, l);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[c][nt], xh, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[c][nt], xh, acc[nt], 0, 0, 0);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[c][nt], xl, acc[nt], 0, 0, 0);
      }
    }
    if (lh < OROWS) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) epi(lh, w, nt, kg, acc[nt], pre);
    }
  }
}

// conv0 -> ys, barrier, conv1 (+ x, ReLU) -> out for image n, row band `band`, from the
// staged x rows (LDS x row 0 = image row band R - 2)
template <int C, int HW, int R>
__device__ __forceinline__ void resblock_item_split(const ResSDesc& d, const uint8_t* xs, uint8_t* ys, int n, int band,
                                                    int lane, int wv) {
  constexpr int NTHR = 512, P = C / 16, NT = C / 16, WP = HW + 2;
  constexpr int XROWS = R + 4, YROWS = R + 2;
  constexpr int XPL = XROWS * WP + 24, YPL = YROWS * WP + 24;
  constexpr int XLO = P * XPL * 32, YLO = P * YPL * 32;      // lo set offsets
  const int r0 = band * R;
  const bool second = d.wf0b != nullptr && n >= d.n_switch;
  {  // conv0 on rows r0 - 1 + lh, lh in [0, R + 2): LDS x row 0 = image row r0 - 2
    const float* __restrict__ b0 = second ? d.b0b : d.b0;
    const bool save = d.ysave != nullptr && n < d.n_save;
    float* __restrict__ ysv = save ? d.ysave + (int64_t)n * d.ysave_img : nullptr;
    // (x was staged relu'd; conv1's input -- this conv's output -- is stored relu'd: neither
    // convolution re-applies relu per fragment read, 9 reads per pixel)
    float4 bias[NT];                                            // loaded once, not per tile
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bias[nt] = ld4(b0 + nt * 16 + 4 * (lane >> 4));
    WFrags<P, NT> w0;
    w0.load(second ? d.wf0b : d.wf0, second ? d.wf0b_lo : d.wf0_lo, lane);
    conv_grid_split<P, NT, WP, YROWS, XPL, NTHR, false>(xs, XLO, w0, lane, wv, [&](int lh, int w, int nt, int kg,
                                                                                  f32x4 a, NoPrefetch::T) {
      if (w >= HW) return;
      const int h = r0 - 1 + lh;
      const bool inside = h >= 0 && h < HW;
      const float4 b = bias[nt];
      const float v0 = a[0] + b.x, v1 = a[1] + b.y, v2 = a[2] + b.z, v3 = a[3] + b.w;
      uint2 hi = make_uint2(0, 0), lo = make_uint2(0, 0);
      if (inside) {
        split_pk_bf16(fmaxf(v0, 0.f), fmaxf(v1, 0.f), hi.x, lo.x);
        split_pk_bf16(fmaxf(v2, 0.f), fmaxf(v3, 0.f), hi.y, lo.y);
      }
      const int o = (nt * YPL + lh * WP + w + 1) * 32 + 8 * kg;
      *reinterpret_cast<uint2*>(ys + o) = hi;
      *reinterpret_cast<uint2*>(ys + YLO + o) = lo;
      if (ysv != nullptr && lh >= 1 && lh <= R && h < HW)
        // (read back only by the backward, after the rest of the forward: a non-temporal
        // store keeps it out of the caches the forward is using -- +0.7 %)
        __builtin_nontemporal_store((f32x4){v0, v1, v2, v3},
                                    reinterpret_cast<f32x4*>(ysv + ((int64_t)(nt * HW + h) * HW + w) * 16 + 4 * kg));
    });
  }
  __syncthreads();
  {  // conv1 on rows r0 + lh, lh in [0, R): LDS y row 0 = image row r0 - 1; + x, (ReLU)
    const float* __restrict__ b1 = second ? d.b1b : d.b1;
    const int relu_out = d.relu_out;
    const bool planes = d.out_lo != nullptr;
    float4 bias[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bias[nt] = ld4(b1 + nt * 16 + 4 * (lane >> 4));
    // the residual -- the block's fp32 input itself (the staged planes hold relu(x)) --
    // loaded before each tile's MFMAs
    struct Res {
      float4 v[NT];
    };
    const float* __restrict__ xn = d.x + (int64_t)n * d.x_img;
    auto residual = [&](int lh, int w, int kg) {
      Res r;
      const int h = r0 + lh;
      const bool ok = lh < R && w < HW && h < HW;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        r.v[nt] = ok ? ld4(xn + ((int64_t)(nt * HW + h) * HW + w) * 16 + 4 * kg) : make_float4(0.f, 0.f, 0.f, 0.f);
      return r;
    };
    WFrags<P, NT> w1;
    w1.load(second ? d.wf1b : d.wf1, second ? d.wf1b_lo : d.wf1_lo, lane);
    conv_grid_split<P, NT, WP, R, YPL, NTHR, false>(ys, YLO, w1, lane, wv, [&](int lh, int w, int nt, int kg, f32x4 a,
                                                                              const Res& res) {
      const int h = r0 + lh;
      if (w >= HW || h >= HW) return;
      const float4 b = bias[nt];
      const float4 xr = res.v[nt];
      float v0 = a[0] + b.x + xr.x;
      float v1 = a[1] + b.y + xr.y;
      float v2 = a[2] + b.z + xr.z;
      float v3 = a[3] + b.w + xr.w;
      if (relu_out) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f); }
      const int64_t off = (int64_t)n * d.out_img + ((int64_t)(nt * HW + h) * HW + w) * 16 + 4 * kg;
      if (planes) {
        uint2 hi, lo;
        split_pk_bf16(v0, v1, hi.x, lo.x);
        split_pk_bf16(v2, v3, hi.y, lo.y);
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(d.out) + off) = hi;
        *reinterpret_cast<uint2*>(d.out_lo + off) = lo;
      } else {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(d.out) + off) = make_float4(v0, v1, v2, v3);
      }
    }, residual);
  }
}

// conv1's zero padding in both y sets: halo columns of every row + the slack past the rows
// (conv0's epilogue never writes them)
template <int P, int WP, int YROWS, int YPL, int YLO, int NTHR>
__device__ __forceinline__ void zero_y_halo(uint8_t* ys, int tid) {
  for (int i = tid; i < 2 * P * YROWS * 2; i += NTHR) {
    const int set = i / (P * YROWS * 2), i1 = i - set * (P * YROWS * 2);
    const int p = i1 / (YROWS * 2), r = i1 - p * YROWS * 2;
    const int c = (r & 1) ? WP - 1 : 0;
    uint8_t* q = ys + set * YLO + (p * YPL + (r >> 1) * WP + c) * 32;
    *reinterpret_cast<uint4*>(q) = make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(q + 16) = make_uint4(0, 0, 0, 0);
  }
  for (int i = tid; i < 2 * P * 24 * 2; i += NTHR) {
    const int set = i / (P * 48), i1 = i - set * (P * 48);
    const int p = i1 / 48, r = i1 - p * 48;
    *reinterpret_cast<uint4*>(ys + set * YLO + (p * YPL + YROWS * WP) * 32 + r * 16) = make_uint4(0, 0, 0, 0);
  }
}

template <int C, int HW, int R>
__global__ void __launch_bounds__(512) resblock_fwd_split_kernel(ResSDesc d) {
  constexpr int NTHR = 512, P = C / 16, WP = HW + 2;
  constexpr int XROWS = R + 4, YROWS = R + 2;
  constexpr int XPL = XROWS * WP + 24, YPL = YROWS * WP + 24;
  constexpr int XLO = P * XPL * 32, YLO = P * YPL * 32;      // lo set offsets
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * (XLO + YLO)];
  uint8_t* xs = smem;
  uint8_t* ys = smem + 2 * XLO;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int band = blockIdx.x, n = blockIdx.y;
  using Rows = RowLoads<P, HW, HW, XROWS, NTHR>;
  Rows rows;
  rows.load(d.x, d.x_img, n, band * R - 2, tid);
  Rows::zero_slack(xs, XPL, tid);
  zero_y_halo<P, WP, YROWS, YPL, YLO, NTHR>(ys, tid);
  rows.store(xs, XPL, 1, tid);                                  // relu(x)
  __syncthreads();
  resblock_item_split<C, HW, R>(d, xs, ys, n, band, lane, wv);
}

// =====================================================================================
// weight gradient (split): same partial-slab format as csrc/impala.hip sconv_wgrad
// =====================================================================================
struct SconvWgSDesc {
  const float* dy;            // fp32 planar gradient of the conv output
  const void* x;              // fp32 planar conv input, or (mode 2) the frame ring
  const int32_t* slots;
  float* slab;
  int64_t dy_img, x_img;
  int N, relu_in;
  int imgs_per_group, cin_real;
  // mode 2 with amax set: dy is the gradient of the 3x3/s2 max pool that follows this conv
  // ([HO][WO][16] per plane, dy_img its image stride) and amax its argmax codes; the conv
  // output gradient is formed while staging (maxpool_bwd_split_kernel's sums, same order)
  const uint8_t* amax;
};

// csrc/impala.hip tr_pix_frag: channel (lane & 15) of pixels 16h + 4(lane >> 4) + {0..3}
__device__ __forceinline__ bf16x8 tr_pix_frag_s(const uint8_t* plane, int pix0, int lane) {
  const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
  const lds_s16x4* pa = (const lds_s16x4*)(plane + (pix0 + 4 * g + qq) * 32 + 8 * pp);
  const lds_s16x4* pb = (const lds_s16x4*)(plane + (pix0 + 16 + 4 * g + qq) * 32 + 8 * pp);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(pa));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(pb));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = (s16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int CIN, int COUT, int H, int W, int R, int MODE, int NTHR>
__global__ void __launch_bounds__(NTHR) sconv_wgrad_split_kernel(SconvWgSDesc d) {
  // NTHR = 512: 8 waves (2 per SIMD), the per-image staging one batch of loads per thread
  // and the other wave of a SIMD covering the LDS-read latency of the MFMA chain (the
  // 4-wave form ran one wave per SIMD at 13 % MFMA busy, profiles/r5_pmc_impala_step.md)
  constexpr int NW = NTHR / 64;
  constexpr int P = CIN / 16, NT = COUT / 16;
  constexpr int WP = W + 2;
  constexpr int NQ = (R * WP + 31) / 32;
  constexpr int DPIX = NQ * 32;
  constexpr int XPIX = DPIX + 2 * WP + 2;
  static_assert(XPIX >= (R + 2) * WP, "x plane too small");
  constexpr int XSETS = MODE == 2 ? 1 : 2;           // the frames are exact: no lo set
  constexpr int DLO = NT * DPIX * 32, XLO = P * XPIX * 32;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * DLO + XSETS * XLO];
  uint8_t* dys = smem;
  uint8_t* xs = smem + 2 * DLO;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int band = blockIdx.x, group = blockIdx.y;
  const int r0 = band * R;
  const int n_begin = group * d.imgs_per_group;
  const int n_end = min(d.N, n_begin + d.imgs_per_group);

  f32x4 acc[NT][9 * P], accb[NT];
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    accb[a] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < 9 * P; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u));

  // fused max-pool backward (mode 2): the band's 2 x 2 pixel blocks, one per (block,
  // 8-channel half); the pad pixels of the dy planes (columns W, W+1 of each row, rows past
  // the band / image, the tail) are never written by it: zeroed once here
  constexpr bool POOLED = MODE == 2 && NT == 1 && (R % 2) == 0 && (H % 2) == 0 && (W % 2) == 0;
  const bool pooled = POOLED && d.amax != nullptr;
  if (POOLED && pooled) {
    for (int q = tid; q < DPIX; q += NTHR) {
      const int lh = q / WP, w = q - (q / WP) * WP;
      if (lh < R && w < W && r0 + lh < H) continue;
#pragma unroll
      for (int set = 0; set < 2; ++set) {
        *reinterpret_cast<uint4*>(dys + set * DLO + q * 32) = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(dys + set * DLO + q * 32 + 16) = make_uint4(0, 0, 0, 0);
      }
    }
  }

  for (int n = n_begin; n < n_end; ++n) {
    const float* dyi = d.dy + (int64_t)n * d.dy_img;
    constexpr int NDC = NT * DPIX * 2, DB = NT * P >= 4 ? 2 : 4;   // 32 x 32: 144 accumulator VGPRs live
    if constexpr (POOLED) {
      if (pooled) {
        constexpr int HO = H / 2, WO = W / 2, NBLK = (R / 2) * WO * 2;
        const uint8_t* ami = d.amax + (int64_t)n * HO * WO * 16;
        for (int it = tid; it < NBLK; it += NTHR) {
          const int hf = it & 1, rest = it >> 1;
          const int al = rest / WO, b = rest - (rest / WO) * WO;
          const int a = (r0 >> 1) + al;
          if (2 * a >= H) continue;
          const bool i1 = a + 1 < HO, j1 = b + 1 < WO;
          float4 g0[4], g1[4];
          uint2 cv[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int oh = (k >> 1) && i1 ? a + 1 : a, ow = (k & 1) && j1 ? b + 1 : b;
            const int64_t po = ((int64_t)oh * WO + ow) * 16 + 8 * hf;
            g0[k] = ld4(dyi + po);
            g1[k] = ld4(dyi + po + 4);
            cv[k] = *reinterpret_cast<const uint2*>(ami + po);
          }
#pragma unroll
          for (int dh = 0; dh < 2; ++dh)
#pragma unroll
            for (int dw = 0; dw < 2; ++dw) {
              const int khs[2] = {1 + dh, (dh && i1) ? 0 : -16}, kws[2] = {1 + dw, (dw && j1) ? 0 : -16};
              float acc8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const int want = khs[k >> 1] * 3 + kws[k & 1];
                const float gv[8] = {g0[k].x, g0[k].y, g0[k].z, g0[k].w, g1[k].x, g1[k].y, g1[k].z, g1[k].w};
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                  const uint32_t word = c < 4 ? cv[k].x : cv[k].y;
                  acc8[c] += (int)((word >> (8 * (c & 3))) & 0xffu) == want ? gv[c] : 0.f;
                }
              }
              uint4 hi, lo;
              split8s(make_float4(acc8[0], acc8[1], acc8[2], acc8[3]), make_float4(acc8[4], acc8[5], acc8[6], acc8[7]),
                      hi, lo);
              const int q = (2 * al + dh) * WP + 2 * b + dw;
              *reinterpret_cast<uint4*>(dys + q * 32 + hf * 16) = hi;
              *reinterpret_cast<uint4*>(dys + DLO + q * 32 + hf * 16) = lo;
            }
        }
      }
    }
#pragma unroll 1
    for (int base = 0; base < (pooled ? 0 : NDC); base += NTHR * DB) {
      float4 va[DB], vb[DB];
#pragma unroll
      for (int k = 0; k < DB; ++k) {
        const int i = base + k * NTHR + tid;
        const int hf = i & 1, pix = i >> 1;
        const int p = pix / DPIX, q = pix - (pix / DPIX) * DPIX;
        const int lh = q / WP, w = q - (q / WP) * WP;
        const int h = r0 + lh;
        va[k] = vb[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < NDC && lh < R && w < W && h < H) {
          const float* s = dyi + ((int64_t)(p * H + h) * W + w) * 16 + hf * 8;
          va[k] = ld4(s);
          vb[k] = ld4(s + 4);
        }
      }
#pragma unroll
      for (int k = 0; k < DB; ++k) {
        const int i = base + k * NTHR + tid;
        if (i < NDC) {
          uint4 hi, lo;
          split8s(va[k], vb[k], hi, lo);
          *reinterpret_cast<uint4*>(dys + (i >> 1) * 32 + (i & 1) * 16) = hi;
          *reinterpret_cast<uint4*>(dys + DLO + (i >> 1) * 32 + (i & 1) * 16) = lo;
        }
      }
    }
    if constexpr (MODE == 2)
      stage_ring16_split<H, W, R + 2, NTHR>(xs, XPIX, reinterpret_cast<const uint8_t*>(d.x), d.slots, n, r0 - 1, tid);
    else
      stage_rows_split<P, H, W, R + 2, NTHR, 4, (NT * P >= 4)>(xs, XPIX, reinterpret_cast<const float*>(d.x), d.x_img, n, r0 - 1,
                                               d.relu_in, tid);
    __syncthreads();
#pragma unroll 1
    for (int j = wv; j < NQ; j += NW) {
      const int qb = 32 * j;
      bf16x8 ah[NT], al[NT];
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        ah[ct] = tr_pix_frag_s(dys + ct * DPIX * 32, qb, lane);
        al[ct] = tr_pix_frag_s(dys + DLO + ct * DPIX * 32, qb, lane);
        accb[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ct], ones, accb[ct], 0, 0, 0);
        accb[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[ct], ones, accb[ct], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int toff = (t / 3) * WP + (t % 3);
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const bf16x8 bh = tr_pix_frag_s(xs + p * XPIX * 32, qb + toff, lane);
          bf16x8 bl;
          if (MODE != 2) bl = tr_pix_frag_s(xs + XLO + p * XPIX * 32, qb + toff, lane);
#pragma unroll
          for (int ct = 0; ct < NT; ++ct) {
            f32x4& A = acc[ct][t * P + p];
            A = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ct], bh, A, 0, 0, 0);
            A = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[ct], bh, A, 0, 0, 0);
            if (MODE != 2) A = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ct], bl, A, 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();
  }

  // cross-wave sum through LDS, one coalesced fp32 partial per workgroup (slab[split][tile][lane][4])
  constexpr int T = NT * 9 * P, TT = T + NT;
  const int split = group * gridDim.x + band;
  f32x4* __restrict__ slab = reinterpret_cast<f32x4*>(d.slab) + (int64_t)split * TT * 64;
  f32x4* red = reinterpret_cast<f32x4*>(smem);
  static_assert(sizeof(smem) >= NW * 4 * 64 * sizeof(f32x4), "reduction slab exceeds the staging LDS");
#pragma unroll
  for (int base = 0; base < TT; base += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int tt = base + u;
      if (tt < T) red[(wv * 4 + u) * 64 + lane] = acc[tt / (9 * P)][tt % (9 * P)];
      else if (tt < TT) red[(wv * 4 + u) * 64 + lane] = accb[tt - T];
    }
    __syncthreads();
    if (tid < 256) {
      const int u = tid >> 6, l = tid & 63, tt = base + u;
      if (tt < TT) {
        f32x4 v = red[u * 64 + l];
#pragma unroll
        for (int w = 1; w < NW; ++w) v += red[(w * 4 + u) * 64 + l];
        slab[tt * 64 + l] = v;
      }
    }
    __syncthreads();
  }
}

// =====================================================================================
// max-pool backward (split storage: fp32 gather), merge of hi / lo planes
// =====================================================================================
template <int H, int W>
__global__ void __launch_bounds__(256) maxpool_bwd_split_kernel(const float* __restrict__ dy, int64_t dy_img,
                                                                const uint8_t* __restrict__ amax, int P,
                                                                float* __restrict__ dx, int64_t dx_img, int N) {
  // one thread per (image, plane, pooled pixel (a, b), 4-channel quad): the input pixels
  // (2a + dh, 2b + dw) of its 2 x 2 block see only the windows (a + i, b + j), i, j in
  // {0, 1} (i = 1 only for dh = 1: kernel row 0), so each window's gradient and argmax
  // codes are loaded once for four outputs (the per-pixel form loaded four windows per
  // output pixel).  Per output the windows are summed in the same (i, j) order as before.
  constexpr int HO = (H + 1) / 2, WO = (W + 1) / 2;
  constexpr int64_t PIMG = (int64_t)HO * WO * 16;
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  const uint32_t total = (uint32_t)N * (uint32_t)P * (uint32_t)(HO * WO * 4);
  if (idx >= total) return;
  const int qd = (int)(idx & 3u);
  uint32_t r = idx >> 2;
  const uint32_t rb = r / (uint32_t)WO;
  const int b = (int)(r - rb * (uint32_t)WO);
  const uint32_t ra = rb / (uint32_t)HO;
  const int a = (int)(rb - ra * (uint32_t)HO);
  const uint32_t rp = ra / (uint32_t)P;
  const int p = (int)(ra - rp * (uint32_t)P);
  const int n = (int)rp;
  const float* dp = dy + (int64_t)n * dy_img;
  const uint8_t* am = amax + (int64_t)n * P * PIMG;
  const bool i1 = a + 1 < HO, j1 = b + 1 < WO;
  float4 g[4];
  uint32_t cv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int oh = (k >> 1) && i1 ? a + 1 : a, ow = (k & 1) && j1 ? b + 1 : b;
    const int64_t po = (((int64_t)p * HO + oh) * WO + ow) * 16 + 4 * qd;
    g[k] = ld4(dp + po);
    cv[k] = *reinterpret_cast<const uint32_t*>(am + po);
  }
  float* dxi = dx + (int64_t)n * dx_img;
#pragma unroll
  for (int dh = 0; dh < 2; ++dh) {
    const int h = 2 * a + dh;
    if (h >= H) continue;
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      const int w = 2 * b + dw;
      if (w >= W) continue;
      // window (a + i, b + j) holds this pixel at kernel (kh, kw); absent windows never match
      const int khs[2] = {1 + dh, (dh && i1) ? 0 : -16}, kws[2] = {1 + dw, (dw && j1) ? 0 : -16};
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int want = khs[k >> 1] * 3 + kws[k & 1];
        const float gv[4] = {g[k].x, g[k].y, g[k].z, g[k].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] += (int)((cv[k] >> (8 * c)) & 0xffu) == want ? gv[c] : 0.f;
      }
      *reinterpret_cast<float4*>(dxi + (((int64_t)p * H + h) * W + w) * 16 + 4 * qd) =
          make_float4(acc[0], acc[1], acc[2], acc[3]);
    }
  }
}

// out[r][c] = hi[r][c] + lo[r][c] (fp32) for c < cols, rows of ld elements
__global__ void __launch_bounds__(256) merge_split_kernel(const bf16_t* __restrict__ hi, const bf16_t* __restrict__ lo,
                                                          float* __restrict__ out, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const uint2 h = reinterpret_cast<const uint2*>(hi)[i];
    const uint2 l = reinterpret_cast<const uint2*>(lo)[i];
    reinterpret_cast<float4*>(out)[i] =
        make_float4(bf16_to_f32(h.x & 0xffff) + bf16_to_f32(l.x & 0xffff), bf16_to_f32(h.x >> 16) + bf16_to_f32(l.x >> 16),
                    bf16_to_f32(h.y & 0xffff) + bf16_to_f32(l.y & 0xffff), bf16_to_f32(h.y >> 16) + bf16_to_f32(l.y >> 16));
  }
}

// ------------------------------------------------------------------ launchers
// (shapes and row bands of csrc/impala.hip; the pooled stack-2 entry uses R = 22)
// (row bands R: the first listed per shape is the default; the others are LDS-occupancy
// variants -- fewer staged rows per workgroup, more workgroups per CU -- chosen by the
// host, ops/impala.py SPLIT_BANDS)
#define SCONV_S_SHAPES(X)       \
  X(16, 16, 84, 84, 6, 3, 1)    \
  X(16, 16, 84, 84, 10, 3, 1)   \
  X(16, 32, 42, 42, 14, 0, 1)   \
  X(16, 32, 42, 42, 6, 0, 1)    \
  X(32, 32, 21, 21, 22, 0, 1)   \
  X(32, 32, 21, 21, 8, 0, 1)    \
  X(16, 16, 84, 84, 21, 3, 0)   \
  X(16, 16, 42, 42, 42, 0, 0)   \
  X(16, 16, 42, 42, 21, 0, 0)   \
  X(16, 16, 42, 42, 14, 0, 0)   \
  X(16, 32, 42, 42, 42, 0, 0)   \
  X(32, 16, 42, 42, 21, 0, 0)   \
  X(32, 16, 42, 42, 11, 0, 0)   \
  X(32, 32, 21, 21, 21, 0, 0)   \
  X(32, 32, 21, 21, 11, 0, 0)   \
  X(32, 32, 21, 21, 7, 0, 0)    \
  X(32, 32, 11, 11, 11, 0, 0)

APEX_EXPORT int apex_sconv_fwd_split(SconvSDesc d, int cin, int cout, int H, int W, int mode, int pool, int R,
                                     hipStream_t st) {
  if (d.N <= 0) return 0;
  if (d.wf == nullptr || d.wf_lo == nullptr || (d.wf2 != nullptr && d.wf2_lo == nullptr)) return (int)hipErrorInvalidValue;
  if (pool && (d.add || d.mask || d.relu_out)) return (int)hipErrorInvalidValue;
#define SCONV_S_FWD_CASE(CI, CO, HH, WW, RR, MM, PP)                                                     \
  if (cin == CI && cout == CO && H == HH && W == WW && mode == MM && pool == PP && (R == 0 || R == RR)) { \
    const int bands = PP ? ((HH + 1) / 2 + RR / 2 - 1) / (RR / 2) : (HH + RR - 1) / RR;                  \
    sconv_fwd_split_kernel<CI, CO, HH, WW, RR, MM, PP><<<dim3(bands, d.N), 512, 0, st>>>(d);             \
    APEX_CHECK_LAUNCH();                                                                                 \
  }
  SCONV_S_SHAPES(SCONV_S_FWD_CASE)
#undef SCONV_S_FWD_CASE
  return (int)hipErrorInvalidValue;
}

#define RESBLOCK_S_SHAPES(X) \
  X(16, 42, 14)              \
  X(16, 42, 10)              \
  X(16, 42, 7)               \
  X(32, 21, 21)              \
  X(32, 21, 11)              \
  X(32, 21, 7)               \
  X(32, 11, 11)              \
  X(32, 11, 6)

APEX_EXPORT int apex_resblock_fwd_split(ResSDesc d, int C, int HW, int R, hipStream_t st) {
  if (d.N <= 0) return 0;
  if (d.wf0_lo == nullptr || d.wf1_lo == nullptr || (d.wf0b != nullptr && (d.wf0b_lo == nullptr || d.wf1b_lo == nullptr)))
    return (int)hipErrorInvalidValue;
#define RESBLOCK_S_CASE(CC, HH, RR)                                                           \
  if (C == CC && HW == HH && (R == 0 || R == RR)) {                                          \
    resblock_fwd_split_kernel<CC, HH, RR><<<dim3((HH + RR - 1) / RR, d.N), 512, 0, st>>>(d);  \
    APEX_CHECK_LAUNCH();                                                                      \
  }
  RESBLOCK_S_SHAPES(RESBLOCK_S_CASE)
#undef RESBLOCK_S_CASE
  return (int)hipErrorInvalidValue;
}

// weight-gradient shapes (cin, cout, H, W, rows per band, mode, threads); the launcher
// takes the first match of the requested (rows, threads), 0 = any (ops/impala.py
// SPLIT_BANDS "wg" keys).  Swept on the fp32 IMPALA step (PERF_NOTES round 5): 11-row
// bands (2 workgroups per CU where the LDS allows) beat the 21-row single-workgroup form
// by 3.4 % together; 8 waves per workgroup except where 256 VGPRs need 4.
#define SCONV_WG_S_SHAPES(X)      \
  X(16, 16, 84, 84, 12, 2, 512)   \
  X(16, 16, 42, 42, 11, 0, 512)   \
  X(16, 32, 42, 42, 7, 0, 256)    \
  X(32, 32, 21, 21, 11, 0, 512)   \
  X(32, 32, 11, 11, 11, 0, 256)

APEX_EXPORT int apex_sconv_wgrad_split_rows(int cin, int cout, int H, int W, int mode, int R, int nthr) {
#define SCONV_WG_S_ROWS(CI, CO, HH, WW, RR, MM, NT)                                                        \
  if (cin == CI && cout == CO && H == HH && W == WW && mode == MM && (R == 0 || R == RR) && (nthr == 0 || nthr == NT)) \
    return RR;
  SCONV_WG_S_SHAPES(SCONV_WG_S_ROWS)
#undef SCONV_WG_S_ROWS
  return 0;
}

APEX_EXPORT int apex_sconv_wgrad_split(SconvWgSDesc d, int cin, int cout, int H, int W, int mode, int R, int nthr,
                                       int groups, hipStream_t st) {
  if (d.N <= 0 || groups <= 0) return (int)hipErrorInvalidValue;
#define SCONV_WG_S_CASE(CI, CO, HH, WW, RR, MM, NT)                                                            \
  if (cin == CI && cout == CO && H == HH && W == WW && mode == MM && (R == 0 || R == RR) && (nthr == 0 || nthr == NT)) { \
    sconv_wgrad_split_kernel<CI, CO, HH, WW, RR, MM, NT><<<dim3((HH + RR - 1) / RR, groups), NT, 0, st>>>(d);    \
    APEX_CHECK_LAUNCH();                                                                                        \
  }
  SCONV_WG_S_SHAPES(SCONV_WG_S_CASE)
#undef SCONV_WG_S_CASE
  return (int)hipErrorInvalidValue;
}

APEX_EXPORT int apex_maxpool_bwd_split(const float* dy, int64_t dy_img, const uint8_t* amax, int P, int H, int W,
                                       float* dx, int64_t dx_img, int N, hipStream_t st) {
  const int64_t total = (int64_t)N * P * ((H + 1) / 2) * ((W + 1) / 2) * 4;   // threads: pooled pixels x quads
  if (total <= 0 || (int64_t)N * P * H * W * 4 >= 0x7fffff00LL) return (int)hipErrorInvalidValue;
  const int blocks = (int)((total + 255) / 256);
  if (H == 84 && W == 84) maxpool_bwd_split_kernel<84, 84><<<blocks, 256, 0, st>>>(dy, dy_img, amax, P, dx, dx_img, N);
  else if (H == 42 && W == 42) maxpool_bwd_split_kernel<42, 42><<<blocks, 256, 0, st>>>(dy, dy_img, amax, P, dx, dx_img, N);
  else if (H == 21 && W == 21) maxpool_bwd_split_kernel<21, 21><<<blocks, 256, 0, st>>>(dy, dy_img, amax, P, dx, dx_img, N);
  else return (int)hipErrorInvalidValue;
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_merge_split(const bf16_t* hi, const bf16_t* lo, float* out, int64_t n, hipStream_t st) {
  if (n <= 0 || (n & 3) || (((uintptr_t)hi | (uintptr_t)lo) & 7) || ((uintptr_t)out & 15)) return (int)hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  int nb = (int)((n4 + 255) / 256);
  nb = nb > 2048 ? 2048 : nb;
  merge_split_kernel<<<nb, 256, 0, st>>>(hi, lo, out, n4);
  APEX_CHECK_LAUNCH();
}

// Small-channel 3x3 convolutions for the IMPALA-deep ResNet dueling Q-net
// (BASELINE.json config 5; not in the reference, whose only network is the
// NatureCNN of duelling_network.py:8-19).  gfx950, wave64, MFMA 16x16x32 bf16.
//
// Activation layout ("planar-16"): an activation of C channels is stored per
// image as C/16 planes of [H][W][16] bf16, i.e. 32-byte pixel rows.  That row
// width makes BOTH LDS reads the kernels need conflict-free without swizzles:
//   * the im2col row fragment (ds_read_b128, 16 pixels x 16 B): pixel p's two
//     16-B halves land on bank quads 2p, 2p+1 -- distinct for 16 consecutive
//     pixels in every ds_read_b128 lane group;
//   * the transposed fragment (ds_read_b64_tr_b16, 4 pixel rows x 16 channels
//     per 16-lane group): a 32-lane half reads 8 consecutive pixel rows = 256
//     contiguous bytes = all 64 banks once.
//
// sconv_fwd   one workgroup per (image, row band): the band's input rows (+1-row
//             halo, zero-padded to (R+2) x (W+2)) are staged in LDS once (ReLU
//             applied on the way in when the conv consumes relu(x)); outputs are
//             computed on the flattened padded-width grid q = h (W+2) + w, so
//             tap (kh, kw) of a 16-pixel M tile is the LDS row block at
//             q + kh (W+2) + kw: a plain ds_read_b128 per K chunk, no index math.
//             K = 9 taps x C_in in 32-wide chunks of two (tap, 16-ch plane)
//             pairs; weights live in VGPRs as pre-packed MFMA fragments
//             (sconv_pack).  Swapped operands (weights as A) give each lane 4
//             consecutive output channels of one pixel -> one 8-byte store.
//             Epilogue: *scale + bias, optional (* (mask > 0)), optional + add,
//             optional ReLU -- covers the forward (bias, residual add) and the
//             data gradient (mask = forward activation, add = skip gradient),
//             which is the same correlation with transposed + flipped weights.
// sconv_wgrad dW[co][ci][t] = sum over pixels dY[p][co] x[p + toff(t)][ci]: both
//             operands through the transposed LDS read, reduction over 32-pixel
//             chunks split across the 4 waves, summed in LDS; each workgroup writes
//             one fp32 partial to a split-K slab, reduced by grad_finalize (conv_mfma.hip).
// maxpool3s2  3x3 / stride 2 / pad 1 max pool (+ argmax codes for the backward);
//             its backward is a gather (each input pixel sums the <= 4 window
//             gradients whose argmax it is): no atomics.
#include "mfma_common.h"

struct SconvDesc {
  const void* x;              // bf16 planar input, or (mode 2) the uint8 s2d frame ring
  const int32_t* slots;       // mode 2: [N][4] frame-ring slots of each image
  const bf16_t* wf;           // packed weight fragments (sconv_pack)
  const bf16_t* wf2;          // second weight set for images >= n_switch (target net), or null
  const float* bias;          // [C_out] or null
  const float* bias2;
  const bf16_t* add;          // added after the mask (output layout), or null
  const bf16_t* mask;         // output multiplied by (mask > 0) (output layout), or null
  bf16_t* y;                  // bf16 planar output (pooled output when POOL)
  void* mask_out;             // POOL: uint8 argmax codes [N][planes][Ho][Wo][16], or null
  int64_t x_img, y_img;       // image strides (elements)
  int64_t add_img, mask_img;
  int N, n_switch;
  int relu_in, relu_out;
  float scale;                // applied to the accumulator before the bias
  int pad0;                   // POOL: argmax codes for images < pad0 only (0 = all)
};

struct SconvWgDesc {
  const bf16_t* dy;           // planar gradient of the conv output
  const void* x;              // planar conv input (or mode 2: the frame ring)
  const int32_t* slots;
  float* slab;                // [nsplit][(C_out/16)(9 C_in/16) + C_out/16 tiles][64 lanes][4] fp32 partials
  float* bslab;               // unused (bias partials are the slab's last tiles)
  int64_t dy_img, x_img;
  int N, relu_in;
  int imgs_per_group, cin_real;
  // mode 2 with amax set: dy is the gradient of the 3x3/s2 max pool after this conv (its
  // argmax codes here); the conv output gradient is gathered while staging (pool_grad8,
  // maxpool_bwd_kernel's arithmetic: bit-identical)
  const uint8_t* amax;
};

__device__ __forceinline__ uint4 relu_u4(uint4 v) {
  return make_uint4(relu_pk16(v.x), relu_pk16(v.y), relu_pk16(v.z), relu_pk16(v.w));
}

// Gradient of a pre-pool conv output (h, w), channels 8 hf .. 8 hf + 7 of plane p,
// from the pooled gradient dp and argmax codes am of one image (3x3 / s2 / pad 1):
// the sum over the <= 4 windows whose argmax is (h, w): the max-pool backward as a
// gather, one output element per thread, no atomics (maxpool_bwd_kernel).
template <int H, int W>
__device__ __forceinline__ uint4 pool_grad8(const bf16_t* __restrict__ dp, const uint8_t* __restrict__ am, int p,
                                            int h, int w, int hf) {
  // windows containing row h: oh = h >> 1 (tap row kh = 1 + (h & 1)) and, for odd h,
  // oh + 1 (kh = 0); same for columns.  All four candidates are loaded up front
  // (clamped address, masked out when absent): independent loads, no branches.
  constexpr int HO = (H + 1) / 2, WO = (W + 1) / 2;
  const int oha = h >> 1, owa = w >> 1;
  const bool hb = (h & 1) && oha + 1 < HO, wb = (w & 1) && owa + 1 < WO;
  const int kha = 1 + (h & 1), kwa = 1 + (w & 1);
  const int ohs[2] = {oha, hb ? oha + 1 : oha}, ows[2] = {owa, wb ? owa + 1 : owa};
  const int khs[2] = {kha, hb ? 0 : -16}, kws[2] = {kwa, wb ? 0 : -16};   // -16: never matches
  uint4 g[4];
  uint2 cv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t po = (((int64_t)p * HO + ohs[i >> 1]) * WO + ows[i & 1]) * 16 + hf * 8;
    g[i] = *reinterpret_cast<const uint4*>(dp + po);
    cv[i] = *reinterpret_cast<const uint2*>(am + po);
  }
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int want = khs[i >> 1] * 3 + kws[i & 1];
    const uint32_t gu[4] = {g[i].x, g[i].y, g[i].z, g[i].w};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int cd = (int)(((c < 4 ? cv[i].x : cv[i].y) >> (8 * (c & 3))) & 0xff);
      const float gv = bf16_to_f32((bf16_t)((gu[c >> 1] >> (16 * (c & 1))) & 0xffff));
      acc[c] += cd == want ? gv : 0.f;
    }
  }
  return make_uint4(cvt_pk_bf16(acc[0], acc[1]), cvt_pk_bf16(acc[2], acc[3]), cvt_pk_bf16(acc[4], acc[5]),
                    cvt_pk_bf16(acc[6], acc[7]));
}

// Stage SROWS input rows starting at global row `row0` (x cols [-1, W]; zero
// outside the image) into P LDS planes of `plane_pix` 32-byte pixel rows; pixels
// past the SROWS x (W+2) block up to plane_pix are zeroed (M-tile overrun reads).
// MODE 0: planar bf16; MODE 2: 4 uint8 frames from the space-to-depth ring
// (csrc/conv1_s2d.hip layout) as channels 0..3 of a 16-channel plane.
// Loads are issued in batches of BATCH per thread before any LDS store, so each
// thread has BATCH global loads in flight instead of one load-use round trip.
template <int P, int H, int W, int SROWS, int MODE, int NTHR, int BATCH>
__device__ __forceinline__ void stage_rows(uint8_t* xs, int plane_pix, const void* x, int64_t x_img,
                                           const int32_t* slots, int n, int row0, int relu, int tid) {
  constexpr int WP = W + 2, BLK = SROWS * WP;
  if constexpr (MODE == 2) {
    const uint8_t* ring = reinterpret_cast<const uint8_t*>(x);
    const int32_t* sl = slots + (int64_t)n * 4;
    const int64_t f0 = (int64_t)sl[0] * 7056, f1 = (int64_t)sl[1] * 7056;
    const int64_t f2 = (int64_t)sl[2] * 7056, f3 = (int64_t)sl[3] * 7056;
    for (int base = 0; base < BLK; base += NTHR * BATCH) {
      uint32_t b[BATCH][4];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int i = base + k * NTHR + tid;
        const int lr = i / WP, c = i - (i / WP) * WP;
        const int h = row0 + lr, w = c - 1;
        b[k][0] = b[k][1] = b[k][2] = b[k][3] = 0;
        if (i < BLK && h >= 0 && h < H && w >= 0 && w < W) {
          const int o = ((h >> 2) * 21 + (w >> 2)) * 16 + (h & 3) * 4 + (w & 3);
          b[k][0] = ring[f0 + o]; b[k][1] = ring[f1 + o]; b[k][2] = ring[f2 + o]; b[k][3] = ring[f3 + o];
        }
      }
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int i = base + k * NTHR + tid;
        if (i < BLK) {
          const uint4 lo = make_uint4(cvt_pk_bf16((float)b[k][0], (float)b[k][1]),
                                      cvt_pk_bf16((float)b[k][2], (float)b[k][3]), 0, 0);
          *reinterpret_cast<uint4*>(xs + i * 32) = lo;
          *reinterpret_cast<uint4*>(xs + i * 32 + 16) = make_uint4(0, 0, 0, 0);
        }
      }
    }
  } else {
    const bf16_t* xi = reinterpret_cast<const bf16_t*>(x) + (int64_t)n * x_img;
    constexpr int NCK = P * BLK * 2;
    for (int base = 0; base < NCK; base += NTHR * BATCH) {
      uint4 v[BATCH];
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int i = base + k * NTHR + tid;
        const int hf = i & 1, pix = i >> 1;
        const int p = pix / BLK, rem = pix - (pix / BLK) * BLK;
        const int lr = rem / WP, c = rem - (rem / WP) * WP;
        const int h = row0 + lr, w = c - 1;
        v[k] = make_uint4(0, 0, 0, 0);
        if (i < NCK && h >= 0 && h < H && w >= 0 && w < W)
          v[k] = *reinterpret_cast<const uint4*>(xi + ((int64_t)(p * H + h) * W + w) * 16 + hf * 8);
      }
#pragma unroll
      for (int k = 0; k < BATCH; ++k) {
        const int i = base + k * NTHR + tid;
        const int hf = i & 1, pix = i >> 1;
        const int p = pix / BLK, rem = pix - (pix / BLK) * BLK;
        if (i < NCK) *reinterpret_cast<uint4*>(xs + (p * plane_pix + rem) * 32 + hf * 16) = relu ? relu_u4(v[k]) : v[k];
      }
    }
  }
  const int slack = plane_pix - BLK;
  for (int i = tid; i < P * slack * 2; i += NTHR) {
    const int p = i / (slack * 2), r = i - p * slack * 2;
    *reinterpret_cast<uint4*>(xs + (p * plane_pix + BLK) * 32 + r * 16) = make_uint4(0, 0, 0, 0);
  }
}

// MODE 3 staging: the 4 stacked uint8 frames as 4-channel bf16 pixels (8 bytes),
// rows [row0, row0 + SROWS) x cols [-1, W] of image n, zero outside the image.
// One item = 4 image pixels of one row: a dword per frame from the s2d ring
// (4 horizontally adjacent pixels are 4 contiguous bytes), transposed in VGPRs.
template <int H, int W, int SROWS, int NTHR>
__device__ __forceinline__ void stage_ring4(uint8_t* xs, int plane_pix, const uint8_t* ring, const int32_t* slots,
                                            int n, int row0, int tid) {
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
  for (int i = tid; i < SROWS * 2; i += NTHR) {     // halo columns -1 and W
    const int lr = i >> 1, c = (i & 1) ? WP - 1 : 0;
    *reinterpret_cast<uint2*>(xs + (lr * WP + c) * 8) = make_uint2(0, 0);
  }
  for (int i = SROWS * WP + tid; i < plane_pix; i += NTHR) *reinterpret_cast<uint2*>(xs + i * 8) = make_uint2(0, 0);
}

// =====================================================================================
// forward / data-gradient correlation (+ fused 3x3/s2 max pool)
// =====================================================================================
// POOL = 0: one workgroup computes output rows [R band, R band + R) and applies the
//           bias / mask / add / ReLU epilogue straight to global memory.
// POOL = 1: (R even) the workgroup computes conv rows [R band - 1, R band + R) into
//           an LDS tile (rows outside the image = -inf), then max-pools them into
//           pooled rows [R band / 2, R band / 2 + R / 2) + argmax codes: the
//           full-resolution conv output never reaches HBM.
// MODE 3 (stack-1 input, 4 frames): K = 9 taps x 4 channels packed as tap PAIRS --
//           lane group kg reads 16 B = pixels (kw0, kw0 + 1) x 4 channels of tap
//           row kh (two ds_read_b64 on 8-byte pixels), so 2 K chunks cover the
//           3x3 window (kw = 3 and the last half-chunk have zero weights) instead
//           of 5 chunks of a 16-channel zero-padded image.
template <int CIN, int COUT, int H, int W, int R, int MODE, int POOL>
__global__ void __launch_bounds__(512) sconv_fwd_kernel(SconvDesc d) {
  constexpr int NTHR = 512, NW = NTHR / 64;
  constexpr int P = CIN / 16, NT = COUT / 16;
  constexpr int WP = W + 2;
  constexpr int OROWS = POOL ? R + 1 : R;      // conv rows computed
  constexpr int SROWS = OROWS + 2;             // staged input rows (1-row halo each side)
  constexpr int PLANE = SROWS * WP + 24;       // + overrun of the last M tile's taps
  constexpr int PIXB = MODE == 3 ? 8 : 32;     // LDS bytes per staged pixel
  constexpr int NCH = MODE == 3 ? 2 : (9 * P + 1) / 2;   // 32-wide K chunks
  constexpr int MROWS = OROWS * WP;
  constexpr int NTILE = (MROWS + 15) / 16;
  constexpr int OPIX = POOL ? OROWS * W : 0;   // pool tile: conv pixels per output plane
  static_assert(!POOL || (R % 2) == 0, "pooled bands need an even row count");
  __shared__ __attribute__((aligned(16))) uint8_t xs[P * PLANE * PIXB + NT * OPIX * 32];
  uint8_t* ot = xs + P * PLANE * PIXB;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int band = blockIdx.x, n = blockIdx.y;
  const int o0 = POOL ? band * R - 1 : band * R;   // first conv output row of the band
  const bool second = d.wf2 != nullptr && n >= d.n_switch;
  const bf16_t* __restrict__ wf = second ? d.wf2 : d.wf;
  const float* __restrict__ bias = second ? d.bias2 : d.bias;

  // weight fragments first (L2-resident; overlap the staging loads)
  bf16x8 wfr[NCH][NT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      wfr[c][nt] = *reinterpret_cast<const bf16x8*>(wf + ((int64_t)(c * NT + nt) * 64 + lane) * 8);

  if constexpr (MODE == 3)
    stage_ring4<H, W, SROWS, NTHR>(xs, PLANE, reinterpret_cast<const uint8_t*>(d.x), d.slots, n, o0 - 1, tid);
  else
    stage_rows<P, H, W, SROWS, MODE, NTHR, 8>(xs, PLANE, d.x, d.x_img, d.slots, n, o0 - 1, d.relu_in, tid);
  __syncthreads();

  // per-lane LDS byte offset of each K chunk: lane group kg = lane >> 4 reads
  // pair 2c + (kg >> 1) (tap-major: pair = t * P + p), 16-B half (kg & 1)
  const int kg = lane >> 4;
  int aoff[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (MODE == 3) {
      // chunk 0: tap rows 0 (kg 0, 1) and 1 (kg 2, 3); chunk 1: row 2 (kg 0, 1), kg 2, 3 zero
      const int kh = c == 0 ? (kg >> 1) : 2;
      aoff[c] = (kh * WP + 2 * (kg & 1) + (lane & 15)) * 8;
      continue;
    }
    int pair = 2 * c + (kg >> 1);
    if (pair >= 9 * P) pair = 9 * P - 1;       // zero-weight K slot: any in-bounds read
    const int t = pair / P, p = pair - (pair / P) * P;
    const int toff = (t / 3) * WP + (t % 3);
    aoff[c] = (p * PLANE + toff + (lane & 15)) * 32 + (kg & 1) * 16;
  }
  bf16_t* __restrict__ yi = d.y + (int64_t)n * d.y_img;
  const bf16_t* __restrict__ addi = d.add ? d.add + (int64_t)n * d.add_img : nullptr;
  const bf16_t* __restrict__ mski = d.mask ? d.mask + (int64_t)n * d.mask_img : nullptr;
  float4 bv[NT];                                   // bias: loaded once, not per tile epilogue
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) bv[nt] = bias ? *reinterpret_cast<const float4*>(bias + nt * 16 + 4 * kg)
                                               : make_float4(0.f, 0.f, 0.f, 0.f);

  for (int tile = wv; tile < NTILE; tile += NW) {
    const int q0 = tile * 16;
    // lane: pixel q0 + (lane & 15), output channels nt*16 + 4 kg + {0..3}
    const int q = q0 + (lane & 15);
    const int lh = q / WP, w = q - (q / WP) * WP;
    const int h = o0 + lh;
    const bool valid = lh < OROWS && w < W && (POOL || h < H);
    // epilogue operands first: their latency hides under the fragment reads + MFMAs
    uint2 am[NT], mm[NT];
    if (!POOL && valid) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int64_t off = ((int64_t)(nt * H + h) * W + w) * 16 + 4 * kg;
        if (addi) am[nt] = *reinterpret_cast<const uint2*>(addi + off);
        if (mski) mm[nt] = *reinterpret_cast<const uint2*>(mski + off);
      }
    }
    bf16x8 xf[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (MODE == 3) {
        const uint2 lo = *reinterpret_cast<const uint2*>(xs + aoff[c] + q0 * 8);
        const uint2 hi = *reinterpret_cast<const uint2*>(xs + aoff[c] + q0 * 8 + 8);
        xf[c] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      } else {
        xf[c] = *reinterpret_cast<const bf16x8*>(xs + aoff[c] + q0 * 32);
      }
    }
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[c][nt], xf[c], acc[nt], 0, 0, 0);
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
        if (h < 0 || h >= H) v[0] = v[1] = v[2] = v[3] = -INFINITY;   // max-pool padding row
        *reinterpret_cast<uint2*>(ot + ((nt * OROWS + lh) * W + w) * 32 + 8 * kg) =
            make_uint2(cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3]));
        continue;
      }
      if (mski) {
        const uint2 m = mm[nt];
        v[0] = bf16_to_f32(m.x & 0xffff) > 0.f ? v[0] : 0.f;
        v[1] = bf16_to_f32(m.x >> 16) > 0.f ? v[1] : 0.f;
        v[2] = bf16_to_f32(m.y & 0xffff) > 0.f ? v[2] : 0.f;
        v[3] = bf16_to_f32(m.y >> 16) > 0.f ? v[3] : 0.f;
      }
      if (addi) {
        const uint2 a = am[nt];
        v[0] += bf16_to_f32(a.x & 0xffff);
        v[1] += bf16_to_f32(a.x >> 16);
        v[2] += bf16_to_f32(a.y & 0xffff);
        v[3] += bf16_to_f32(a.y >> 16);
      }
      if (d.relu_out) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      const int64_t off = ((int64_t)(nt * H + h) * W + w) * 16 + 4 * kg;
      *reinterpret_cast<uint2*>(yi + off) = make_uint2(cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3]));
    }
  }
  if constexpr (POOL) {
    // 3x3 / s2 / pad 1 max pool of the LDS conv tile: pooled rows band*R/2 + [0, R/2),
    // one item per (plane, pooled pixel, 8-channel half); argmax code = kh*3 + kw of
    // the first maximum in window order (torch.max_pool2d's rule)
    constexpr int HO = (H + 1) / 2, WO = (W + 1) / 2, PR = R / 2;
    __syncthreads();
    uint8_t* __restrict__ am_out = reinterpret_cast<uint8_t*>(d.mask_out);
    // argmax codes only where a backward follows: images < pad0 (all when pad0 == 0)
    const bool track = am_out != nullptr && (d.pad0 <= 0 || n < d.pad0);
    for (int it = tid; it < NT * PR * WO * 2; it += NTHR) {
      const int hf = it & 1, r1 = it >> 1;
      const int ow = r1 % WO, r2 = r1 / WO;
      const int pr = r2 % PR, nt = r2 / PR;
      const int oh = band * PR + pr;
      if (oh >= HO) continue;
      float best[8];
      int code[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) { best[c] = -INFINITY; code[c] = 0; }
      if (track) {
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const int lr = 2 * pr + kh;            // conv row 2 oh - 1 + kh relative to o0
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int wc = 2 * ow - 1 + kw;
            if (wc < 0 || wc >= W) continue;
            const uint4 v = *reinterpret_cast<const uint4*>(ot + ((nt * OROWS + lr) * W + wc) * 32 + hf * 16);
            const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int c = 0; c < 8; ++c) {
              const float f = bf16_to_f32((bf16_t)((u[c >> 1] >> (16 * (c & 1))) & 0xffff));
              if (f > best[c]) { best[c] = f; code[c] = kh * 3 + kw; }
            }
          }
        }
      } else {
        // no backward through these images: plain max, two channels per dword
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const int lr = 2 * pr + kh;
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int wc = 2 * ow - 1 + kw;
            if (wc < 0 || wc >= W) continue;
            const uint4 v = *reinterpret_cast<const uint4*>(ot + ((nt * OROWS + lr) * W + wc) * 32 + hf * 16);
            const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              best[2 * c] = fmaxf(best[2 * c], __uint_as_float(u[c] << 16));
              best[2 * c + 1] = fmaxf(best[2 * c + 1], __uint_as_float(u[c] & 0xffff0000u));
            }
          }
        }
      }
      const int64_t po = (((int64_t)nt * HO + oh) * WO + ow) * 16 + hf * 8;
      *reinterpret_cast<uint4*>(yi + po) = make_uint4(cvt_pk_bf16(best[0], best[1]), cvt_pk_bf16(best[2], best[3]),
                                                      cvt_pk_bf16(best[4], best[5]), cvt_pk_bf16(best[6], best[7]));
      if (track) {
        uint2 cv;
        cv.x = code[0] | (code[1] << 8) | (code[2] << 16) | (code[3] << 24);
        cv.y = code[4] | (code[5] << 8) | (code[6] << 16) | (code[7] << 24);
        *reinterpret_cast<uint2*>(am_out + (int64_t)n * NT * HO * WO * 16 + po) = cv;
      }
    }
  }
}

// =====================================================================================
// fused residual block forward: out = x + conv1(relu(conv0(relu(x))))
// =====================================================================================
// One workgroup per (image, row band [r0, r0 + R)).  x rows [r0 - 2, r0 + R + 2)
// are staged once; conv0 is evaluated on rows [r0 - 1, r0 + R + 1) into an LDS
// image (rows outside the image stored as the zero padding conv1 reads); conv1
// reads it, adds x from LDS and stores the block output.  The intermediate y =
// conv0(.) goes to HBM only for the rows the backward needs (images < n_save,
// own band rows) -- the unfused pair moved x, y, y, x, out through HBM.
struct ResDesc {
  const bf16_t* x;
  const bf16_t* wf0; const bf16_t* wf0b;    // conv0 fragments (online, target)
  const float* b0; const float* b0b;
  const bf16_t* wf1; const bf16_t* wf1b;    // conv1 fragments
  const float* b1; const float* b1b;
  bf16_t* ysave;                            // conv0 output for images < n_save (or null)
  bf16_t* out;
  int64_t x_img, ysave_img, out_img;
  int N, n_switch, n_save, relu_out;
};

// All M tiles of an OROWS x WP output grid from an LDS image of P planes (plane
// stride PLANE pixels, LDS row 0 = output row -1), ReLU on the fragments when
// `relu`; epi(lh, w, nt, kg, acc) for every lane-pixel of the grid.
template <int P, int NT, int WP, int OROWS, int PLANE, int NTHR, typename Epi>
__device__ __forceinline__ void conv_grid(const uint8_t* img, const bf16_t* __restrict__ wf, bool relu, int lane,
                                          int wv, Epi epi) {
  constexpr int NCH = (9 * P + 1) / 2, NW = NTHR / 64;
  constexpr int NTILE = (OROWS * WP + 15) / 16;
  bf16x8 wfr[NCH][NT];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      wfr[c][nt] = *reinterpret_cast<const bf16x8*>(wf + ((int64_t)(c * NT + nt) * 64 + lane) * 8);
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
    bf16x8 xf[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      uint4 v = *reinterpret_cast<const uint4*>(img + aoff[c] + q0 * 32);
      if (relu) v = relu_u4(v);
      xf[c] = __builtin_bit_cast(bf16x8, v);
    }
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[c][nt], xf[c], acc[nt], 0, 0, 0);
    const int q = q0 + (lane & 15);
    const int lh = q / WP, w = q - (q / WP) * WP;
    if (lh < OROWS) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) epi(lh, w, nt, kg, acc[nt]);
    }
  }
}

template <int C, int HW, int R>
__global__ void __launch_bounds__(512) resblock_fwd_kernel(ResDesc d) {
  constexpr int NTHR = 512, P = C / 16, NT = C / 16, WP = HW + 2;
  constexpr int XROWS = R + 4, YROWS = R + 2;
  constexpr int XPL = XROWS * WP + 24, YPL = YROWS * WP + 24;
  __shared__ __attribute__((aligned(16))) uint8_t smem[(P * XPL + P * YPL) * 32];
  uint8_t* xs = smem;
  uint8_t* ys = smem + P * XPL * 32;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int band = blockIdx.x, n = blockIdx.y;
  const int r0 = band * R;
  const bool second = d.wf0b != nullptr && n >= d.n_switch;
  stage_rows<P, HW, HW, XROWS, 0, NTHR, 8>(xs, XPL, d.x, d.x_img, nullptr, n, r0 - 2, 0, tid);
  // conv1's zero padding: halo columns of every y row + the slack past the rows
  for (int i = tid; i < P * YROWS * 2; i += NTHR) {
    const int p = i / (YROWS * 2), r = i - p * YROWS * 2;
    const int c = (r & 1) ? WP - 1 : 0;
    *reinterpret_cast<uint4*>(ys + (p * YPL + (r >> 1) * WP + c) * 32) = make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(ys + (p * YPL + (r >> 1) * WP + c) * 32 + 16) = make_uint4(0, 0, 0, 0);
  }
  for (int i = tid; i < P * 24 * 2; i += NTHR) {
    const int p = i / 48, r = i - p * 48;
    *reinterpret_cast<uint4*>(ys + (p * YPL + YROWS * WP) * 32 + r * 16) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  // conv0 on rows r0 - 1 + lh, lh in [0, R + 2): LDS x row 0 = image row r0 - 2
  {
    const float* __restrict__ b0 = second ? d.b0b : d.b0;
    const bool save = d.ysave != nullptr && n < d.n_save;
    bf16_t* __restrict__ ysv = save ? d.ysave + (int64_t)n * d.ysave_img : nullptr;
    float4 bias[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bias[nt] = *reinterpret_cast<const float4*>(b0 + nt * 16 + 4 * (lane >> 4));
    conv_grid<P, NT, WP, YROWS, XPL, NTHR>(xs, second ? d.wf0b : d.wf0, true, lane, wv,
      [&](int lh, int w, int nt, int kg, f32x4 a) {
        if (w >= HW) return;                   // padded-width garbage columns
        const int h = r0 - 1 + lh;
        const bool inside = h >= 0 && h < HW;
        const float4 b = bias[nt];
        const uint2 v = inside ? make_uint2(cvt_pk_bf16(a[0] + b.x, a[1] + b.y), cvt_pk_bf16(a[2] + b.z, a[3] + b.w))
                               : make_uint2(0, 0);
        *reinterpret_cast<uint2*>(ys + (nt * YPL + lh * WP + w + 1) * 32 + 8 * kg) = v;
        if (ysv != nullptr && lh >= 1 && lh <= R && h < HW)
          *reinterpret_cast<uint2*>(ysv + ((int64_t)(nt * HW + h) * HW + w) * 16 + 4 * kg) = v;
      });
  }
  __syncthreads();
  // conv1 on rows r0 + lh, lh in [0, R): LDS y row 0 = image row r0 - 1; + x, (ReLU)
  {
    const float* __restrict__ b1 = second ? d.b1b : d.b1;
    bf16_t* __restrict__ oi = d.out + (int64_t)n * d.out_img;
    const int relu_out = d.relu_out;
    float4 bias[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bias[nt] = *reinterpret_cast<const float4*>(b1 + nt * 16 + 4 * (lane >> 4));
    conv_grid<P, NT, WP, R, YPL, NTHR>(ys, second ? d.wf1b : d.wf1, true, lane, wv,
      [&](int lh, int w, int nt, int kg, f32x4 a) {
        const int h = r0 + lh;
        if (w >= HW || h >= HW) return;
        const float4 b = bias[nt];
        const uint2 xv = *reinterpret_cast<const uint2*>(xs + (nt * XPL + (lh + 2) * WP + w + 1) * 32 + 8 * kg);
        float v0 = a[0] + b.x + bf16_to_f32(xv.x & 0xffff), v1 = a[1] + b.y + bf16_to_f32(xv.x >> 16);
        float v2 = a[2] + b.z + bf16_to_f32(xv.y & 0xffff), v3 = a[3] + b.w + bf16_to_f32(xv.y >> 16);
        if (relu_out) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f); }
        *reinterpret_cast<uint2*>(oi + ((int64_t)(nt * HW + h) * HW + w) * 16 + 4 * kg) =
            make_uint2(cvt_pk_bf16(v0, v1), cvt_pk_bf16(v2, v3));
      });
  }
}

#define RESBLOCK_SHAPES(X) \
  X(16, 42, 21)            \
  X(16, 42, 14)            \
  X(16, 42, 11)            \
  X(32, 21, 21)            \
  X(32, 11, 11)

// band rows R: 0 = default (the first listed for the shape)
APEX_EXPORT int apex_resblock_fwd(ResDesc d, int C, int HW, int R, hipStream_t st) {
  if (d.N <= 0) return 0;
#define RESBLOCK_CASE(CC, HH, RR)                                                           \
  if (C == CC && HW == HH && (R == 0 || R == RR)) {                                         \
    resblock_fwd_kernel<CC, HH, RR><<<dim3((HH + RR - 1) / RR, d.N), 512, 0, st>>>(d);      \
    APEX_CHECK_LAUNCH();                                                                    \
  }
  RESBLOCK_SHAPES(RESBLOCK_CASE)
#undef RESBLOCK_CASE
  return (int)hipErrorInvalidValue;
}

// =====================================================================================
// weight gradient
// =====================================================================================
// MFMA operand from a transposed read of 32-byte pixel rows: lane (g = lane>>4,
// i = lane&15) receives channel i of pixels 16h + 4g + {0..3} for h = 0, 1 --
// the K order (k = 8g + 4h + r <-> pixel 16h + 4g + r) is the same for both
// operands, and each 32-lane half reads 8 consecutive pixel rows per instruction.
__device__ __forceinline__ bf16x8 tr_pix_frag(const uint8_t* plane, int pix0, int lane) {
  const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
  const lds_s16x4* pa = (const lds_s16x4*)(plane + (pix0 + 4 * g + qq) * 32 + 8 * pp);
  const lds_s16x4* pb = (const lds_s16x4*)(plane + (pix0 + 16 + 4 * g + qq) * 32 + 8 * pp);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(pa));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(pb));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = (s16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int CIN, int COUT, int H, int W, int R, int MODE>
__global__ void __launch_bounds__(256) sconv_wgrad_kernel(SconvWgDesc d) {
  constexpr int P = CIN / 16, NT = COUT / 16;
  constexpr int WP = W + 2;
  constexpr int NQ = (R * WP + 31) / 32;             // 32-pixel reduction chunks per band
  constexpr int DPIX = NQ * 32;                      // dY plane (zero past R x WP)
  constexpr int XPIX = DPIX + 2 * WP + 2;            // x plane: covers every tap of every chunk
  static_assert(XPIX >= (R + 2) * WP, "x plane too small");
  __shared__ __attribute__((aligned(16))) uint8_t smem[(NT * DPIX + P * XPIX) * 32];
  uint8_t* dys = smem;
  uint8_t* xs = smem + NT * DPIX * 32;
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

  for (int n = n_begin; n < n_end; ++n) {
    // dY band: pixel q = lh * WP + w, zero for w >= W, rows past H / R, and q >= R * WP
    const bf16_t* dyi = d.dy + (int64_t)n * d.dy_img;
    constexpr int NDC = NT * DPIX * 2, DB = 4;
    for (int base = 0; base < NDC; base += 256 * DB) {
      uint4 v[DB];
#pragma unroll
      for (int k = 0; k < DB; ++k) {
        const int i = base + k * 256 + tid;
        const int hf = i & 1, pix = i >> 1;
        const int p = pix / DPIX, q = pix - (pix / DPIX) * DPIX;
        const int lh = q / WP, w = q - (q / WP) * WP;
        const int h = r0 + lh;
        v[k] = make_uint4(0, 0, 0, 0);
        if (i < NDC && lh < R && w < W && h < H) {
          if (MODE == 2 && d.amax != nullptr)
            v[k] = pool_grad8<H, W>(dyi, d.amax + (int64_t)n * NT * ((H + 1) / 2) * ((W + 1) / 2) * 16, p, h, w, hf);
          else
            v[k] = *reinterpret_cast<const uint4*>(dyi + ((int64_t)(p * H + h) * W + w) * 16 + hf * 8);
        }
      }
#pragma unroll
      for (int k = 0; k < DB; ++k) {
        const int i = base + k * 256 + tid;
        if (i < NDC) *reinterpret_cast<uint4*>(dys + (i >> 1) * 32 + (i & 1) * 16) = v[k];
      }
    }
    stage_rows<P, H, W, R + 2, MODE, 256, 4>(xs, XPIX, d.x, d.x_img, d.slots, n, r0 - 1, d.relu_in, tid);
    __syncthreads();
    for (int j = wv; j < NQ; j += 4) {
      const int qb = 32 * j;
      bf16x8 a[NT];
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        a[ct] = tr_pix_frag(dys + ct * DPIX * 32, qb, lane);
        accb[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ct], ones, accb[ct], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int toff = (t / 3) * WP + (t % 3);
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const bf16x8 b = tr_pix_frag(xs + p * XPIX * 32, qb + toff, lane);
#pragma unroll
          for (int ct = 0; ct < NT; ++ct)
            acc[ct][t * P + p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ct], b, acc[ct][t * P + p], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }

  // the 4 waves' partials are summed through LDS (4 tiles per round) and the
  // workgroup writes ONE partial in accumulator order -- slab[split][tile][lane][4],
  // tiles = the T weight tiles then NT bias tiles -- as coalesced 16-byte stores;
  // sconv_wgrad_reduce sums the splits and scatters to OIHW.
  constexpr int T = NT * 9 * P, TT = T + NT;
  const int split = group * gridDim.x + band;
  f32x4* __restrict__ slab = reinterpret_cast<f32x4*>(d.slab) + (int64_t)split * TT * 64;
  f32x4* red = reinterpret_cast<f32x4*>(smem);          // [wave][4 tiles][64 lanes]
#pragma unroll
  for (int base = 0; base < TT; base += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int tt = base + u;
      if (tt < T) red[(wv * 4 + u) * 64 + lane] = acc[tt / (9 * P)][tt % (9 * P)];
      else if (tt < TT) red[(wv * 4 + u) * 64 + lane] = accb[tt - T];
    }
    __syncthreads();
    {
      const int u = tid >> 6, l = tid & 63, tt = base + u;
      if (tt < TT) {
        f32x4 v = red[u * 64 + l];
#pragma unroll
        for (int w = 1; w < 4; ++w) v += red[(w * 4 + u) * 64 + l];
        slab[tt * 64 + l] = v;
      }
    }
    __syncthreads();
  }
}

// Sum the split partials of every IMPALA conv weight gradient (one launch for
// all jobs) and scatter them to the OIHW fp32 gradient (x scale) + bias.  A block
// owns 16 float4 columns of one job's slab; 16 thread groups stride the splits.
struct WgRedJob {
  const float* slab;
  float* out;
  float* bout;
  int nsplit, NT, P, cin_real;
  float scale;
  int blk0;
};
struct WgRedDesc {
  WgRedJob job[16];
  int njobs, nblocks;
};

__global__ void __launch_bounds__(256) sconv_wgrad_reduce_kernel(WgRedDesc d) {
  __shared__ f32x4 red[16][16];
  const int b = blockIdx.x;
  int j = 0;
#pragma unroll
  for (int k = 1; k < 16; ++k)
    if (k < d.njobs && b >= d.job[k].blk0) j = k;
  const WgRedJob& J = d.job[j];
  const int T = J.NT * 9 * J.P, TT = T + J.NT;
  const int lc = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int col = (b - J.blk0) * 16 + lc;               // float4 column = tile * 64 + lane
  const f32x4* __restrict__ src = reinterpret_cast<const f32x4*>(J.slab);
  const int64_t stride = (int64_t)TT * 64;
  f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (col < TT * 64) {
#pragma unroll 8
    for (int k = grp; k < J.nsplit; k += 16) v += src[(int64_t)k * stride + col];
  }
  red[grp][lc] = v;
  __syncthreads();
  if (grp != 0 || col >= TT * 64) return;
#pragma unroll
  for (int g2 = 1; g2 < 16; ++g2) v += red[g2][lc];
  const int tt = col >> 6, l = col & 63, g = l >> 4, i = l & 15;
  if (tt < T) {
    const int ct = tt / (9 * J.P), k = tt - ct * (9 * J.P);
    const int t = k / J.P, p = k - (k / J.P) * J.P;
    const int ci = p * 16 + i;
    if (ci < J.cin_real) {
#pragma unroll
      for (int r = 0; r < 4; ++r) J.out[((int64_t)(ct * 16 + 4 * g + r) * J.cin_real + ci) * 9 + t] = v[r] * J.scale;
    }
  } else if (i == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) J.bout[(tt - T) * 16 + 4 * g + r] = v[r];
  }
}

APEX_EXPORT int apex_sconv_wgrad_reduce(WgRedDesc d, hipStream_t st) {
  if (d.njobs <= 0 || d.njobs > 16 || d.nblocks <= 0) return (int)hipErrorInvalidValue;
  sconv_wgrad_reduce_kernel<<<d.nblocks, 256, 0, st>>>(d);
  APEX_CHECK_LAUNCH();
}

// =====================================================================================
// 3x3 / stride 2 / pad 1 max pool on planar-16 tensors (+ backward)
// =====================================================================================
// one thread per (image, plane, output pixel, 8-channel half); argmax code = kh * 3 + kw
// of the first maximum in window order (torch.max_pool2d's tie rule)
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const bf16_t* __restrict__ x, int64_t x_img, int P, int H,
                                                          int W, int Ho, int Wo, bf16_t* __restrict__ y,
                                                          int64_t y_img, uint8_t* __restrict__ amax, int N) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)N * P * Ho * Wo * 2;
  if (idx >= total) return;
  const int hf = (int)(idx & 1);
  int64_t r = idx >> 1;
  const int ow = (int)(r % Wo); r /= Wo;
  const int oh = (int)(r % Ho); r /= Ho;
  const int p = (int)(r % P);
  const int n = (int)(r / P);
  const bf16_t* xp = x + (int64_t)n * x_img + (int64_t)p * H * W * 16 + hf * 8;
  float best[8];
  int code[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) { best[c] = -INFINITY; code[c] = 0; }
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int h = 2 * oh - 1 + kh;
    if (h < 0 || h >= H) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int w = 2 * ow - 1 + kw;
      if (w < 0 || w >= W) continue;
      const uint4 v = *reinterpret_cast<const uint4*>(xp + ((int64_t)h * W + w) * 16);
      const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float f = bf16_to_f32((bf16_t)((u[c >> 1] >> (16 * (c & 1))) & 0xffff));
        if (f > best[c]) { best[c] = f; code[c] = kh * 3 + kw; }
      }
    }
  }
  const int64_t o = (int64_t)n * y_img + (((int64_t)p * Ho + oh) * Wo + ow) * 16 + hf * 8;
  // the max is one of the inputs: bf16 -> f32 -> bf16 is exact
  *reinterpret_cast<uint4*>(y + o) = make_uint4(cvt_pk_bf16(best[0], best[1]), cvt_pk_bf16(best[2], best[3]),
                                                cvt_pk_bf16(best[4], best[5]), cvt_pk_bf16(best[6], best[7]));
  if (amax) {
    const int64_t ao = ((((int64_t)n * P + p) * Ho + oh) * Wo + ow) * 16 + hf * 8;
    uint2 cv;
    cv.x = code[0] | (code[1] << 8) | (code[2] << 16) | (code[3] << 24);
    cv.y = code[4] | (code[5] << 8) | (code[6] << 16) | (code[7] << 24);
    *reinterpret_cast<uint2*>(amax + ao) = cv;
  }
}

template <int H, int W>
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const bf16_t* __restrict__ dy, int64_t dy_img,
                                                          const uint8_t* __restrict__ amax, int P,
                                                          bf16_t* __restrict__ dx, int64_t dx_img, int N) {
  // 32-bit index math (the launcher checks N * P * H * W * 2 < 2^31): compile-time
  // H / W divide by multiply-shift, no 64-bit division sequences
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  const uint32_t total = (uint32_t)N * (uint32_t)P * (uint32_t)(H * W * 2);
  if (idx >= total) return;
  const int hf = (int)(idx & 1u);
  uint32_t r = idx >> 1;
  const uint32_t rw = r / (uint32_t)W;
  const int w = (int)(r - rw * (uint32_t)W);
  const uint32_t rh = rw / (uint32_t)H;
  const int h = (int)(rw - rh * (uint32_t)H);
  const uint32_t rp = rh / (uint32_t)P;
  const int p = (int)(rh - rp * (uint32_t)P);
  const int n = (int)rp;
  constexpr int64_t PIMG = (int64_t)((H + 1) / 2) * ((W + 1) / 2) * 16;
  const uint4 v = pool_grad8<H, W>(dy + (int64_t)n * dy_img, amax + (int64_t)n * P * PIMG, p, h, w, hf);
  *reinterpret_cast<uint4*>(dx + (int64_t)n * dx_img + (((int64_t)p * H + h) * W + w) * 16 + hf * 8) = v;
}

// =====================================================================================
// weight fragment packing (OIHW bf16 master copy -> per-lane MFMA A fragments)
// =====================================================================================
// frag[c][nt][lane][j] = W'[co = nt*16 + (lane&15)][ci][t] for K chunk c, lane group
// kg = lane>>4: pair = 2c + (kg>>1) = t * P + p, ci = p*16 + (kg&1)*8 + j (0 past 9P).
// transpose = 1 packs the data-gradient correlation: W'[co'][ci'][t] = W[ci'][co'][8-t].
struct PackJob {
  const bf16_t* w;            // OIHW [cout][cin_real][3][3]
  bf16_t* out;
  int cin, cout;              // logical (multiples of 16; cin >= cin_real)
  int cin_real, transpose;
};
struct PackDesc {
  PackJob job[32];
  int njobs;
};

__global__ void __launch_bounds__(256) sconv_pack_kernel(PackDesc d) {
  const PackJob J = d.job[blockIdx.y];
  const bool tr = J.transpose == 1, ring = J.transpose == 2;
  const int Ci = tr ? J.cout : J.cin, Co = tr ? J.cin : J.cout;
  const int P = Ci / 16, NT = Co / 16, NCH = ring ? 2 : (9 * P + 1) / 2;
  const int total = NCH * NT * 512;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int j = e & 7, lane = (e >> 3) & 63, cn = e >> 9;
    const int nt = cn % NT, c = cn / NT;
    const int kg = lane >> 4, pair = 2 * c + (kg >> 1);
    const int co = nt * 16 + (lane & 15);
    bf16_t v = 0;
    if (ring) {
      // tap-pair K (sconv_fwd MODE 3): kh from (chunk, kg), kw = 2 (kg & 1) + j / 4, channel j % 4
      const int kh = c == 0 ? (kg >> 1) : (kg < 2 ? 2 : 3);
      const int kw = 2 * (kg & 1) + (j >> 2), ch = j & 3;
      if (kh < 3 && kw < 3 && ch < J.cin_real) v = J.w[((int64_t)co * J.cin_real + ch) * 9 + kh * 3 + kw];
    } else if (pair < 9 * P) {
      const int t = pair / P, p = pair - (pair / P) * P;
      const int ci = p * 16 + (kg & 1) * 8 + j;
      if (tr) {
        if (co < J.cin_real) v = J.w[((int64_t)ci * J.cin_real + co) * 9 + (8 - t)];
      } else if (ci < J.cin_real) {
        v = J.w[((int64_t)co * J.cin_real + ci) * 9 + t];
      }
    }
    J.out[e] = v;
  }
}

// ------------------------------------------------------------------ launchers
#define SCONV_SHAPES(X)         \
  X(16, 16, 84, 84, 10, 3, 1)   \
  X(16, 32, 42, 42, 14, 0, 1)   \
  X(32, 32, 21, 21, 22, 0, 1)   \
  X(16, 16, 84, 84, 21, 3, 0)   \
  X(16, 16, 42, 42, 42, 0, 0)   \
  X(16, 32, 42, 42, 42, 0, 0)   \
  X(32, 16, 42, 42, 21, 0, 0)   \
  X(32, 32, 21, 21, 21, 0, 0)   \
  X(32, 32, 11, 11, 11, 0, 0)

// pool = 1: fused conv + 3x3/s2 max pool (d.y = pooled output, d.mask_out = argmax)
APEX_EXPORT int apex_sconv_fwd(SconvDesc d, int cin, int cout, int H, int W, int mode, int pool, hipStream_t st) {
  if (d.N <= 0) return 0;
  if (pool && (d.add || d.mask || d.relu_out)) return (int)hipErrorInvalidValue;
#define SCONV_FWD_CASE(CI, CO, HH, WW, RR, MM, PP)                                                      \
  if (cin == CI && cout == CO && H == HH && W == WW && mode == MM && pool == PP) {                      \
    const int bands = PP ? ((HH + 1) / 2 + RR / 2 - 1) / (RR / 2) : (HH + RR - 1) / RR;                 \
    sconv_fwd_kernel<CI, CO, HH, WW, RR, MM, PP><<<dim3(bands, d.N), 512, 0, st>>>(d);                  \
    APEX_CHECK_LAUNCH();                                                                                \
  }
  SCONV_SHAPES(SCONV_FWD_CASE)
#undef SCONV_FWD_CASE
  return (int)hipErrorInvalidValue;
}

// wgrad bands (LDS: dY band + x band with halo; 2 workgroups per CU)
#define SCONV_WG_SHAPES(X)   \
  X(16, 16, 84, 84, 12, 2)   \
  X(16, 16, 42, 42, 21, 0)   \
  X(16, 32, 42, 42, 14, 0)   \
  X(32, 32, 21, 21, 21, 0)   \
  X(32, 32, 11, 11, 11, 0)

APEX_EXPORT int apex_sconv_wgrad_bands(int cin, int cout, int H, int W, int mode) {
#define SCONV_WG_BANDS(CI, CO, HH, WW, RR, MM) \
  if (cin == CI && cout == CO && H == HH && W == WW && mode == MM) return (HH + RR - 1) / RR;
  SCONV_WG_SHAPES(SCONV_WG_BANDS)
#undef SCONV_WG_BANDS
  return 0;
}

APEX_EXPORT int apex_sconv_wgrad(SconvWgDesc d, int cin, int cout, int H, int W, int mode, int groups,
                                 hipStream_t st) {
  if (d.N <= 0 || groups <= 0) return (int)hipErrorInvalidValue;
#define SCONV_WG_CASE(CI, CO, HH, WW, RR, MM)                                                          \
  if (cin == CI && cout == CO && H == HH && W == WW && mode == MM) {                                   \
    sconv_wgrad_kernel<CI, CO, HH, WW, RR, MM><<<dim3((HH + RR - 1) / RR, groups), 256, 0, st>>>(d);     \
    APEX_CHECK_LAUNCH();                                                                                \
  }
  SCONV_WG_SHAPES(SCONV_WG_CASE)
#undef SCONV_WG_CASE
  return (int)hipErrorInvalidValue;
}

APEX_EXPORT int apex_maxpool_fwd(const bf16_t* x, int64_t x_img, int P, int H, int W, bf16_t* y, int64_t y_img,
                                 uint8_t* amax, int N, hipStream_t st) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int64_t total = (int64_t)N * P * Ho * Wo * 2;
  maxpool_fwd_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>(x, x_img, P, H, W, Ho, Wo, y, y_img, amax, N);
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_maxpool_bwd(const bf16_t* dy, int64_t dy_img, const uint8_t* amax, int P, int H, int W,
                                 bf16_t* dx, int64_t dx_img, int N, hipStream_t st) {
  const int64_t total = (int64_t)N * P * H * W * 2;
  if (total <= 0 || total >= 0x7fffff00LL) return (int)hipErrorInvalidValue;   // 32-bit kernel indexing
  const int blocks = (int)((total + 255) / 256);
  if (H == 84 && W == 84) maxpool_bwd_kernel<84, 84><<<blocks, 256, 0, st>>>(dy, dy_img, amax, P, dx, dx_img, N);
  else if (H == 42 && W == 42) maxpool_bwd_kernel<42, 42><<<blocks, 256, 0, st>>>(dy, dy_img, amax, P, dx, dx_img, N);
  else if (H == 21 && W == 21) maxpool_bwd_kernel<21, 21><<<blocks, 256, 0, st>>>(dy, dy_img, amax, P, dx, dx_img, N);
  else return (int)hipErrorInvalidValue;
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_sconv_pack(PackDesc d, hipStream_t st) {
  if (d.njobs <= 0 || d.njobs > 32) return (int)hipErrorInvalidValue;
  sconv_pack_kernel<<<dim3(8, d.njobs), 256, 0, st>>>(d);
  APEX_CHECK_LAUNCH();
}

// packed fragment elements of one conv (for buffer sizing on the host)
APEX_EXPORT int64_t apex_sconv_frag_elems(int cin, int cout) {
  const int P = cin / 16, NT = cout / 16, NCH = (9 * P + 1) / 2;
  return (int64_t)NCH * NT * 512;
}

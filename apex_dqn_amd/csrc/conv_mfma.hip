// MFMA implicit-GEMM kernels for the dueling NatureCNN (gfx950, wave64).
//
// Reference compute: duelling_network.py:8-28 (3 convs + 2 stream FCs, run by
// PyTorch-0.4 on the CPU) and learner.py:56 (autograd backward).  Here every
// GEMM-shaped op of the learner step is one of two hand-written kernels:
//
//  igemm_fwd   C[M,N] = A[M,K] . B[N,K]^T  (+bias, *scale, ReLU | *mask)
//              A-operand modes: 0 dense bf16 rows (fc fwd / fc dgrad),
//                               1 NHWC bf16 implicit im2col (conv2/conv3 fwd,
//                                 conv3 dgrad, conv2 dgrad per stride-parity class),
//              (conv1 forward runs on the space-to-depth ring: csrc/conv1_s2d.hip);
//              B operand row-major [N][K] or K-major (dgrad reads natural weights).
//  igemm_wgrad dW[Co,Kc] = sum_m dY[m,Co] . X[m,Kc]   (split over m, fp32 slabs),
//              both operands read column-wise from LDS with ds_read_b64_tr_b16
//              (the hardware transpose read); conv1 gathers uint8 s2d frame blocks.
//
// Tiles: fwd 128x64x64 (4 waves, 32x64 per wave, v_mfma_f32_16x16x32_bf16);
// wgrad 64x64 per block over 64-row reduction steps.  LDS images are XOR
// swizzled so both the row reads (ds_read_b128) and the transposed reads are
// bank-conflict free.  Global->LDS staging is register double-buffered: the
// next tile's loads are issued before the current tile's MFMAs.
#include "mfma_common.h"
#include "igemm_wgrad.h"
#include "conv2_wfrag.h"

struct ConvDesc {
  const void* x;              // mode 0: bf16 [M][K]; mode 1: bf16 NHWC [N][H][W][Cin]
  const int32_t* frame_slots; // unused (conv1 runs in csrc/conv1_s2d.hip)
  const bf16_t* w;            // B operand [Cout][K] (K contiguous), + cls * w_cls_stride
  const float* bias;          // [Cout] or null
  bf16_t* y;                  // output rows of ldy elements
  const bf16_t* mask;         // optional ReLU mask source (same addressing as y): y = acc * (mask > 0)
  int N, H, W, Cin;
  int OH, OW, Cout, KH;
  int KW, stride, pad_h, pad_w;
  int mode, relu, ldy, ncls;
  int ostride_h, ostride_w, OHfull, OWfull;
  int K;
  float in_scale;
  int64_t w_cls_stride;
  const bf16_t* w2;           // weights for output rows >= m_switch (target network), or null
  const float* bias2;
  int m_switch;               // first output row of the second weight set (any row: row_tile)
  // B operand stored K-major (bt != 0): element (k, n) at w + koff(cls, k/64) + (k%64)*ldb + n.
  // Lets the dgrad GEMMs read the natural weight tensors (no transposed / flipped copies):
  // bt = 1: koff from the table koff[cls * KT + kt]; bt = 2: koff = kt * 64 * ldb.
  int bt;
  int ldb;
  int koff[16];
  int tile_hint;              // 0 auto, 1 / 2 register-staged BM=128 / 64, 3-5 LDS-DMA (apex_conv_fwd)
  int order_hint;             // 0 auto, 1 M tiles fastest per XCD, 2 N tiles fastest
  // fp32-accurate ("split") mode, all four set: the lo planes of A, B (both weight
  // sets) and the output; every operand is hi + lo (csrc/mfma_common.h split_pk_bf16)
  const bf16_t* x_lo;
  const bf16_t* w_lo;
  const bf16_t* w2_lo;
  bf16_t* y_lo;
};


// =====================================================================================
// forward / dgrad implicit GEMM
// =====================================================================================
#define FWD_BN 64

struct FwdRegs {
  uint4 a[4];
  uint4 b0, b1;
  uint4 al[4];                // SPLIT: lo planes of the same rows
  uint4 bl0, bl1;
};



// MODE: A-operand source (0 dense rows, 1 NHWC implicit im2col).
// PAD: im2col taps may fall outside the input (padding / dgrad): per-row tap
//      validity bitmask, invalid taps read zeros through the buffer range check.
// BT: B operand K-major (d.bt), read through the LDS transpose path.
// OWC / OHWC: output width / pixels per image as compile-time constants for the
// learner's layers (0 = runtime), so the per-row div/mod is multiply-shift.
// BM: rows per block (128: 32 per wave; 64: 16 per wave, for grids that would
// otherwise leave CUs idle -- fc fwd/dgrad and the 7x7 / 9x9 layers).
// SPLIT: fp32-accurate mode.  Every stage holds the hi AND lo planes of both
// operand tiles (the same staging addresses, a second buffer resource), each
// fragment pair takes three MFMAs (hi.hi + lo.hi + hi.lo into one fp32
// accumulator), and the epilogue writes the fp32 result as hi / lo bf16 planes
// (ReLU applied in fp32 before the split: a ReLU on the lo plane alone would be
// wrong; the dgrad mask zeroes both planes).
// Row tiles of a launch whose rows >= m_switch use a second weight set (online /
// target networks in one launch): [0, m_switch) and [m_switch, M) are tiled from their
// own starts, so no tile straddles the switch and the weight set stays block-uniform;
// rows past a segment's end read row 0 and are never stored.  With m_switch a
// multiple of BM this is the plain tiling.  row_tiles() is the host-side tile count.
struct RowTile {
  int m0, mend;
  bool second;
};

__device__ __forceinline__ RowTile row_tile(const ConvDesc& d, int bx, int BM, int M) {
  if (d.w2 == nullptr) return RowTile{bx * BM, M, false};
  const int t1 = (d.m_switch + BM - 1) / BM;
  if (bx < t1) return RowTile{bx * BM, d.m_switch, false};
  return RowTile{d.m_switch + (bx - t1) * BM, M, true};
}

static inline int row_tiles(const ConvDesc& d, int M, int BM) {
  if (d.w2 == nullptr) return (M + BM - 1) / BM;
  return (d.m_switch + BM - 1) / BM + (M - d.m_switch + BM - 1) / BM;
}

template <int MODE, bool PAD, bool BT, int OWC, int OHWC, int BM, bool SPLIT>
__global__ void __launch_bounds__(256) igemm_fwd_kernel(ConvDesc d) {
  constexpr int AR = BM / 32;            // A rows staged per thread
  constexpr int MT = BM / 64;            // 16-row MFMA tiles per wave
  constexpr int WR = BM / 4;             // output rows per wave
  constexpr int HALF = BM * 128 + FWD_BN * 128;   // one precision plane of a stage
  constexpr int STAGE = SPLIT ? 2 * HALF : HALF;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // XCD-contiguous tile order: adjacent M tiles (overlapping im2col input rows) share an L2
  const int wg = xcd_swizzle(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                             gridDim.x * gridDim.y * gridDim.z);
  // order_hint 2 (set by the launcher): N tiles fastest, so an XCD keeps its few A
  // panels in L2 and streams B (fc forward: A re-read once per N tile otherwise)
  int bx, by, bz;
  if (d.order_hint == 2) {
    by = wg % gridDim.y;
    const int r = wg / gridDim.y;
    bx = r % gridDim.x;
    bz = r / gridDim.x;
  } else {
    bx = wg % gridDim.x;
    const int r = wg / gridDim.x;
    by = r % gridDim.y;
    bz = r / gridDim.y;
  }
  const int cls = bz;
  const uint32_t OHW = OHWC ? OHWC : d.OH * d.OW;
  const uint32_t OWv = OWC ? OWC : d.OW;
  const int M = d.N * OHW;
  const RowTile rt = row_tile(d, bx, BM, M);
  const int m0 = rt.m0, mend = rt.mend;
  const int n0 = by * FWD_BN;
  // online / target weight sets in one launch: the switch row is block-uniform
  const bool second = rt.second;
  const bf16_t* __restrict__ wb = (second ? d.w2 : d.w) + (int64_t)cls * d.w_cls_stride;
  const float* __restrict__ bias = second ? d.bias2 : d.bias;
  const int KT = d.K >> 6;
  const int sc = tid & 7;
  const int srow = tid >> 3;
  const __amdgpu_buffer_rsrc_t ra_rs = buf_rsrc(d.x);
  const __amdgpu_buffer_rsrc_t rb_rs = buf_rsrc(wb);
  const __amdgpu_buffer_rsrc_t ra_lo = buf_rsrc(SPLIT ? d.x_lo : d.x);
  const __amdgpu_buffer_rsrc_t rb_lo =
      buf_rsrc(SPLIT ? (second ? d.w2_lo : d.w_lo) + (int64_t)cls * d.w_cls_stride : wb);

  // per-thread staging rows (4 A rows, 2 B rows): loop-invariant byte offsets.
  // Rows past M are clamped to row 0 (their outputs are never stored).
  uint32_t a_off[AR], vmask[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + srow + 32 * i;
    const int mm = m < mend ? m : 0;
    if (MODE == 0) {
      a_off[i] = ((uint32_t)mm * d.K + sc * 8) * 2u;
      vmask[i] = 0;
    } else {
      const int img = udiv<OHWC>(mm, OHW), rem = mm - img * OHW;
      const int oh = udiv<OWC>(rem, OWv), ow = rem - oh * OWv;
      const int ih0 = oh * d.stride - d.pad_h, iw0 = ow * d.stride - d.pad_w;
      // PAD: offset of the (possibly out-of-range) tap (0,0) pixel; taps add to it in VALU
      a_off[i] = (uint32_t)(((img * d.H + ih0) * d.W + iw0) * d.Cin + sc * 8) * 2u;
      uint32_t vm = 0;
      if (PAD) {
        // valid taps form a rectangle [kh0, kh1) x [kw0, kw1): one row mask per kh
        const int kh0 = max(0, -ih0), kh1 = min(d.KH, d.H - ih0);
        const int kw0 = max(0, -iw0), kw1 = min(d.KW, d.W - iw0);
        const uint32_t colbits = kw1 > kw0 ? ((1u << kw1) - 1u) & ~((1u << kw0) - 1u) : 0u;
        for (int kh = kh0; kh < kh1; ++kh) vm |= colbits << (kh * d.KW);
      }
      vmask[i] = vm;
    }
  }
  const uint32_t b_off0 = BT ? (uint32_t)((srow * d.ldb + n0 + sc * 8) * 2)
                             : (uint32_t)(((n0 + srow) * d.K + sc * 8) * 2);
  const uint32_t b_off1 = b_off0 + (BT ? 64u * d.ldb : 64u * d.K);
  const int cpb = d.Cin >> 6;

  // Tiles are loaded strictly in order (0, 1, 2, ... then KT-1 repeated), so the
  // im2col tap decode is a scalar cursor advanced once per load: no integer
  // division (which lowers to VALU and would make the offsets look divergent).
  int lt = 0, c_cb = 0, c_kw = 0, c_kh = 0;
  auto load_next = [&](FwdRegs& R) {
    const int kt = lt;
    const uint32_t bso = BT ? (uint32_t)(d.bt == 2 ? kt * 128 * d.ldb : 2 * d.koff[cls * KT + kt]) : (uint32_t)kt * 128u;
    R.b0 = buf_ld16(rb_rs, b_off0, bso);
    R.b1 = buf_ld16(rb_rs, b_off1, bso);
    if (SPLIT) {
      R.bl0 = buf_ld16(rb_lo, b_off0, bso);
      R.bl1 = buf_ld16(rb_lo, b_off1, bso);
    }
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        R.a[i] = buf_ld16(ra_rs, a_off[i], (uint32_t)kt * 128u);
        if (SPLIT) R.al[i] = buf_ld16(ra_lo, a_off[i], (uint32_t)kt * 128u);
      }
    } else {
      const int tap = c_kh * d.KW + c_kw;
      const uint32_t toff = (uint32_t)(((c_kh * d.W + c_kw) * d.Cin + (c_cb << 6)) * 2);
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        if (PAD) {
          const uint32_t vo = ((vmask[i] >> tap) & 1u) ? a_off[i] + toff : BUF_OOB;
          R.a[i] = buf_ld16(ra_rs, vo, 0);
          if (SPLIT) R.al[i] = buf_ld16(ra_lo, vo, 0);
        } else {
          R.a[i] = buf_ld16(ra_rs, a_off[i], toff);
          if (SPLIT) R.al[i] = buf_ld16(ra_lo, a_off[i], toff);
        }
      }
    }
    if (lt < KT - 1) {
      ++lt;
      if (MODE == 1 && ++c_cb == cpb) {
        c_cb = 0;
        if (++c_kw == d.KW) { c_kw = 0; ++c_kh; }
      }
    }
  };

  auto write_tile = [&](int buf, const FwdRegs& R) {
    uint8_t* As = smem + buf * STAGE;
    uint8_t* Bs = As + BM * 128;
#pragma unroll
    for (int i = 0; i < AR; ++i) *reinterpret_cast<uint4*>(As + swz_row(srow + 32 * i, sc)) = R.a[i];
    *reinterpret_cast<uint4*>(Bs + (BT ? swz_tr(srow, sc) : swz_row(srow, sc))) = R.b0;
    *reinterpret_cast<uint4*>(Bs + (BT ? swz_tr(srow + 32, sc) : swz_row(srow + 32, sc))) = R.b1;
    if (SPLIT) {
      uint8_t* Al = As + HALF;
      uint8_t* Bl = Bs + HALF;
#pragma unroll
      for (int i = 0; i < AR; ++i) *reinterpret_cast<uint4*>(Al + swz_row(srow + 32 * i, sc)) = R.al[i];
      *reinterpret_cast<uint4*>(Bl + (BT ? swz_tr(srow, sc) : swz_row(srow, sc))) = R.bl0;
      *reinterpret_cast<uint4*>(Bl + (BT ? swz_tr(srow + 32, sc) : swz_row(srow + 32, sc))) = R.bl1;
    }
  };

  // acc[mt][nt] holds C^T (channels x pixels): lane (g = lane>>4, p = lane&15) owns
  // channels 16nt + 4g + {0..3} of pixel 16mt + p -- 4 consecutive channels, so the
  // epilogue packs them with v_cvt_pk_bf16_f32 into one 8-byte LDS write.
  f32x4 acc[MT][4];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const uint8_t* As = smem + buf * STAGE;
    const uint8_t* Bs = As + BM * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + (lane >> 4);
      bf16x8 a[MT], b[4], al[MT], bl[4];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        a[mt] = *reinterpret_cast<const bf16x8*>(As + swz_row(WR * wv + 16 * mt + (lane & 15), c));
        if (SPLIT) al[mt] = *reinterpret_cast<const bf16x8*>(As + HALF + swz_row(WR * wv + 16 * mt + (lane & 15), c));
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        b[nt] = BT ? tr_frag8(Bs, s, 16 * nt, lane)
                   : *reinterpret_cast<const bf16x8*>(Bs + swz_row(16 * nt + (lane & 15), c));
        if (SPLIT)
          bl[nt] = BT ? tr_frag8(Bs + HALF, s, 16 * nt, lane)
                      : *reinterpret_cast<const bf16x8*>(Bs + HALF + swz_row(16 * nt + (lane & 15), c));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          if (SPLIT) {
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[nt], a[mt], acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], al[mt], acc[mt][nt], 0, 0, 0);
          }
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], a[mt], acc[mt][nt], 0, 0, 0);
        }
    }
  };

  // Software pipeline: two register stages + two LDS stages, straight-line body.
  // Tile t's global loads are issued two half-iterations before its MFMAs
  // (prefetch distance 2); loads past the last tile re-read tile KT-1 (cache
  // hits) so the body has no branches and the vmcnt waits stay partial.
  FwdRegs RA, RB;
  load_next(RA);                        // tile 0
  load_next(RB);                        // tile 1
  write_tile(0, RA);
  __syncthreads();
  load_next(RA);                        // tile 2
  int kt = 0;
  for (; kt + 1 < KT; kt += 2) {
    compute(0);
    write_tile(1, RB);                  // tile kt+1
    __syncthreads();
    load_next(RB);                      // tile kt+3
    compute(1);
    write_tile(0, RA);                  // tile kt+2 (or a harmless duplicate)
    __syncthreads();
    load_next(RA);                      // tile kt+4
  }
  if (kt < KT) compute(0);              // odd KT: last tile sits in buffer 0
  __syncthreads();

  // ---- epilogue: (acc*scale + bias) -> bf16x4 per lane -> swizzled LDS image -> 16-B row stores
  // (SPLIT: a second image for the lo plane right after the BM-row hi image)
  uint8_t* Es = smem + wv * (WR * 128);
  uint8_t* El = smem + BM * 128 + wv * (WR * 128);
  const int g = lane >> 4, pl = lane & 15;
  const bool relu32 = SPLIT && d.relu && d.mask == nullptr;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int ch = 16 * nt + 4 * g;
    float b4[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
      const float4 bb = *reinterpret_cast<const float4*>(bias + n0 + ch);
      b4[0] = bb.x; b4[1] = bb.y; b4[2] = bb.z; b4[3] = bb.w;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row = 16 * mt + pl;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[mt][nt][r] * d.in_scale + b4[r];
        if (relu32) v[r] = fmaxf(v[r], 0.f);
      }
      if (SPLIT) {
        uint32_t h01, l01, h23, l23;
        split_pk_bf16(v[0], v[1], h01, l01);
        split_pk_bf16(v[2], v[3], h23, l23);
        *reinterpret_cast<uint2*>(Es + epi_off(row, ch * 2)) = make_uint2(h01, h23);
        *reinterpret_cast<uint2*>(El + epi_off(row, ch * 2)) = make_uint2(l01, l23);
      } else {
        *reinterpret_cast<uint2*>(Es + epi_off(row, ch * 2)) =
            make_uint2(cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3]));
      }
    }
  }
  __syncthreads();
  const int ooh = (d.ncls == 4) ? (cls >> 1) : 0;
  const int oow = (d.ncls == 4) ? (cls & 1) : 0;
#pragma unroll
  for (int p = 0; p < WR / 8; ++p) {
    const int row = 8 * p + (lane >> 3), ch = lane & 7;
    const int m = m0 + WR * wv + row;
    if (m >= mend) continue;
    uint4 v = *reinterpret_cast<const uint4*>(Es + epi_off(row, ch * 16));
    uint4 vl = make_uint4(0, 0, 0, 0);
    if (SPLIT) vl = *reinterpret_cast<const uint4*>(El + epi_off(row, ch * 16));
    const int img = udiv<OHWC>(m, OHW), rem = m - img * OHW;
    const int oh = udiv<OWC>(rem, OWv), ow = rem - oh * OWv;
    const int64_t orow = ((int64_t)img * d.OHfull + oh * d.ostride_h + ooh) * d.OWfull + ow * d.ostride_w + oow;
    const int64_t off = orow * d.ldy + n0 + ch * 8;
    if (d.mask) {
      const uint4 mk = *reinterpret_cast<const uint4*>(d.mask + off);
      v = make_uint4(mask_bf16x2(v.x, mk.x), mask_bf16x2(v.y, mk.y), mask_bf16x2(v.z, mk.z),
                     mask_bf16x2(v.w, mk.w));
      if (SPLIT)
        vl = make_uint4(mask_bf16x2(vl.x, mk.x), mask_bf16x2(vl.y, mk.y), mask_bf16x2(vl.z, mk.z),
                        mask_bf16x2(vl.w, mk.w));
    } else if (d.relu && !SPLIT) {
      v = make_uint4(relu_bf16x2(v.x), relu_bf16x2(v.y), relu_bf16x2(v.z), relu_bf16x2(v.w));
    }
    *reinterpret_cast<uint4*>(d.y + off) = v;
    if (SPLIT) *reinterpret_cast<uint4*>(d.y_lo + off) = vl;
  }
}

// =====================================================================================
// forward / dgrad implicit GEMM, LDS-DMA staged (the default for 128-row tiles)
// =====================================================================================
// The same GEMM, LDS images, fragments and epilogue as igemm_fwd_kernel at BM = 128
// (4 waves x 32 rows x 64 channels), but the operand tiles travel global -> LDS by
// global_load_lds_dwordx4 into an NS-deep ring of stages.  The register-staged
// kernel moves every operand byte through VGPRs and a ds_write_b128 (13 LDS-path
// cycles per wave-instruction, under 80 B/clk/CU): at 64-row tiles that costs more
// LDS cycles than the fragment reads, and it needs the 64-row tiles to fill the
// chip with a 2-deep pipeline.  Here no VALU or ds_write touches the staging: each
// lane's DMA source is chosen so its fixed LDS slot (M0 + 16 lane) receives the
// chunk that the swizzled image (swz_row / swz_tr) wants there, and the tile a wave
// computes on was issued NS - 1 tiles earlier (one barrier per K tile).
//   slot p of 128-B row r holds chunk p ^ ((r >> 1) & 7)   (swz_row: A, and B rows)
//   slot p of K-major row k holds chunk p ^ (s(k) << 1)     (swz_tr: K-major B)
// Padding taps (dgrad) read a zero row instead of predicating the load.
__device__ __attribute__((aligned(16))) uint8_t apex_zero_row[128];

template <int MODE, bool PAD, bool BT, int OWC, int OHWC, bool SPLIT, int NS, int BM = 128>
__global__ void __launch_bounds__(256) igemm_dma_kernel(ConvDesc d) {
  constexpr int MT = BM / 64, WR = BM / 4;
  constexpr int HALF = BM * 128 + FWD_BN * 128;   // one precision plane of a stage
  constexpr int STAGE = SPLIT ? 2 * HALF : HALF;
  constexpr int NA = BM / 32;                     // A DMA instructions per wave per plane
  constexpr int NB = FWD_BN / 32;                 // B DMA instructions per wave per plane
  constexpr int DPT = (NA + NB) * (SPLIT ? 2 : 1);   // DMAs per wave per K tile
  static_assert(NS >= 2 && NS * STAGE <= 163840, "LDS ring");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wg = xcd_swizzle(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                             gridDim.x * gridDim.y * gridDim.z);
  int bx, by, bz;
  if (d.order_hint == 2) {
    by = wg % gridDim.y;
    const int r = wg / gridDim.y;
    bx = r % gridDim.x;
    bz = r / gridDim.x;
  } else {
    bx = wg % gridDim.x;
    const int r = wg / gridDim.x;
    by = r % gridDim.y;
    bz = r / gridDim.y;
  }
  const int cls = bz;
  const uint32_t OHW = OHWC ? OHWC : d.OH * d.OW;
  const uint32_t OWv = OWC ? OWC : d.OW;
  const int M = d.N * OHW;
  const RowTile rt = row_tile(d, bx, BM, M);
  const int m0 = rt.m0, mend = rt.mend;
  const int n0 = by * FWD_BN;
  const bool second = rt.second;
  const uint8_t* wb = reinterpret_cast<const uint8_t*>((second ? d.w2 : d.w) + (int64_t)cls * d.w_cls_stride);
  const uint8_t* wl = SPLIT ? reinterpret_cast<const uint8_t*>((second ? d.w2_lo : d.w_lo) + (int64_t)cls * d.w_cls_stride)
                            : wb;
  const uint8_t* xa = reinterpret_cast<const uint8_t*>(d.x);
  const uint8_t* xl = SPLIT ? reinterpret_cast<const uint8_t*>(d.x_lo) : xa;
  const float* __restrict__ bias = second ? d.bias2 : d.bias;
  const int KT = d.K >> 6;
  const int cpb = d.Cin >> 6;

  // per-lane DMA sources: A instruction i of this wave fills rows 8 (wv + 4 i) .. +7
  // (lane >> 3 picks the row, lane & 7 the LDS slot), B likewise with 64 rows
  uint32_t a_off[NA], vmask[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int r = 8 * (wv + 4 * i) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int m = m0 + r;
    const int mm = m < mend ? m : 0;
    if (MODE == 0) {
      a_off[i] = ((uint32_t)mm * d.K + c * 8) * 2u;
      vmask[i] = 0;
    } else {
      const int img = udiv<OHWC>(mm, OHW), rem = mm - img * OHW;
      const int oh = udiv<OWC>(rem, OWv), ow = rem - oh * OWv;
      const int ih0 = oh * d.stride - d.pad_h, iw0 = ow * d.stride - d.pad_w;
      a_off[i] = (uint32_t)(((img * d.H + ih0) * d.W + iw0) * d.Cin + c * 8) * 2u;
      uint32_t vm = 0;
      if (PAD) {
        const int kh0 = max(0, -ih0), kh1 = min(d.KH, d.H - ih0);
        const int kw0 = max(0, -iw0), kw1 = min(d.KW, d.W - iw0);
        const uint32_t colbits = kw1 > kw0 ? ((1u << kw1) - 1u) & ~((1u << kw0) - 1u) : 0u;
        for (int kh = kh0; kh < kh1; ++kh) vm |= colbits << (kh * d.KW);
      }
      vmask[i] = vm;
    }
  }
  uint32_t b_off[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int r = 8 * (wv + 4 * i) + (lane >> 3);
    if (BT) {
      const int s = ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
      const int c = (lane & 7) ^ (s << 1);
      b_off[i] = (uint32_t)((r * d.ldb + n0 + c * 8) * 2);
    } else {
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      b_off[i] = (uint32_t)(((n0 + r) * d.K + c * 8) * 2);
    }
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem;
  // tiles are issued strictly in order: the im2col tap is a scalar cursor
  int lt = 0, c_cb = 0, c_kw = 0, c_kh = 0;
  auto issue = [&]() {
    const int kt = lt;
    const uint32_t dst = lds0 + (uint32_t)(kt % NS) * STAGE;
    const uint32_t bso = BT ? (uint32_t)(d.bt == 2 ? kt * 128 * d.ldb : 2 * d.koff[cls * KT + kt]) : (uint32_t)kt * 128u;
    uint32_t toff;
    int tap = 0;
    if (MODE == 0) {
      toff = (uint32_t)kt * 128u;
    } else {
      tap = c_kh * d.KW + c_kw;
      toff = (uint32_t)(((c_kh * d.W + c_kw) * d.Cin + (c_cb << 6)) * 2);
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const uint32_t ldsa = __builtin_amdgcn_readfirstlane(dst + (wv + 4 * i) * 1024);
      const bool ok = !PAD || ((vmask[i] >> tap) & 1u);
      const uint32_t ao = a_off[i] + toff;   // 32-bit: a padded row's tap-(0,0) offset wraps
      dma16(ok ? (const void*)(xa + ao) : (const void*)apex_zero_row, ldsa);
      if (SPLIT) dma16(ok ? (const void*)(xl + ao) : (const void*)apex_zero_row, ldsa + HALF);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const uint32_t ldsb = __builtin_amdgcn_readfirstlane(dst + BM * 128 + (wv + 4 * i) * 1024);
      const uint32_t bo = b_off[i] + bso;
      dma16(wb + bo, ldsb);
      if (SPLIT) dma16(wl + bo, ldsb + HALF);
    }
    ++lt;
    if (MODE == 1 && ++c_cb == cpb) {
      c_cb = 0;
      if (++c_kw == d.KW) { c_kw = 0; ++c_kh; }
    }
  };

  f32x4 acc[MT][4];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const uint8_t* As = smem + buf * STAGE;
    const uint8_t* Bs = As + BM * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + (lane >> 4);
      bf16x8 a[MT], b[4], al[MT], bl[4];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        a[mt] = *reinterpret_cast<const bf16x8*>(As + swz_row(WR * wv + 16 * mt + (lane & 15), c));
        if (SPLIT) al[mt] = *reinterpret_cast<const bf16x8*>(As + HALF + swz_row(WR * wv + 16 * mt + (lane & 15), c));
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        b[nt] = BT ? tr_frag8(Bs, s, 16 * nt, lane)
                   : *reinterpret_cast<const bf16x8*>(Bs + swz_row(16 * nt + (lane & 15), c));
        if (SPLIT)
          bl[nt] = BT ? tr_frag8(Bs + HALF, s, 16 * nt, lane)
                      : *reinterpret_cast<const bf16x8*>(Bs + HALF + swz_row(16 * nt + (lane & 15), c));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          if (SPLIT) {
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[nt], a[mt], acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], al[mt], acc[mt][nt], 0, 0, 0);
          }
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], a[mt], acc[mt][nt], 0, 0, 0);
        }
    }
  };

  // ring: tiles 0 .. NS-2 in flight before the loop; iteration kt waits for its own
  // DMAs of tile kt (later tiles may stay in flight: completions are in order), the
  // barrier publishes everyone's, and frees stage (kt - 1) % NS for tile kt + NS - 1
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < KT) issue();
  for (int kt = 0; kt < KT; ++kt) {
    const int ahead = min(NS - 2, KT - 1 - kt);
    vmcnt_le(ahead * DPT);
    __syncthreads();
    if (kt + NS - 1 < KT) issue();
    compute(kt % NS);
  }
  __syncthreads();

  // ---- epilogue (as igemm_fwd_kernel)
  uint8_t* Es = smem + wv * (WR * 128);
  uint8_t* El = smem + BM * 128 + wv * (WR * 128);
  const int g = lane >> 4, pl = lane & 15;
  const bool relu32 = SPLIT && d.relu && d.mask == nullptr;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int ch = 16 * nt + 4 * g;
    float b4[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
      const float4 bb = *reinterpret_cast<const float4*>(bias + n0 + ch);
      b4[0] = bb.x; b4[1] = bb.y; b4[2] = bb.z; b4[3] = bb.w;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row = 16 * mt + pl;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[mt][nt][r] * d.in_scale + b4[r];
        if (relu32) v[r] = fmaxf(v[r], 0.f);
      }
      if (SPLIT) {
        uint32_t h01, l01, h23, l23;
        split_pk_bf16(v[0], v[1], h01, l01);
        split_pk_bf16(v[2], v[3], h23, l23);
        *reinterpret_cast<uint2*>(Es + epi_off(row, ch * 2)) = make_uint2(h01, h23);
        *reinterpret_cast<uint2*>(El + epi_off(row, ch * 2)) = make_uint2(l01, l23);
      } else {
        *reinterpret_cast<uint2*>(Es + epi_off(row, ch * 2)) =
            make_uint2(cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3]));
      }
    }
  }
  __syncthreads();
  const int ooh = (d.ncls == 4) ? (cls >> 1) : 0;
  const int oow = (d.ncls == 4) ? (cls & 1) : 0;
#pragma unroll
  for (int p = 0; p < WR / 8; ++p) {
    const int row = 8 * p + (lane >> 3), ch = lane & 7;
    const int m = m0 + WR * wv + row;
    if (m >= mend) continue;
    uint4 v = *reinterpret_cast<const uint4*>(Es + epi_off(row, ch * 16));
    uint4 vl = make_uint4(0, 0, 0, 0);
    if (SPLIT) vl = *reinterpret_cast<const uint4*>(El + epi_off(row, ch * 16));
    const int img = udiv<OHWC>(m, OHW), rem = m - img * OHW;
    const int oh = udiv<OWC>(rem, OWv), ow = rem - oh * OWv;
    const int64_t orow = ((int64_t)img * d.OHfull + oh * d.ostride_h + ooh) * d.OWfull + ow * d.ostride_w + oow;
    const int64_t off = orow * d.ldy + n0 + ch * 8;
    if (d.mask) {
      const uint4 mk = *reinterpret_cast<const uint4*>(d.mask + off);
      v = make_uint4(mask_bf16x2(v.x, mk.x), mask_bf16x2(v.y, mk.y), mask_bf16x2(v.z, mk.z),
                     mask_bf16x2(v.w, mk.w));
      if (SPLIT)
        vl = make_uint4(mask_bf16x2(vl.x, mk.x), mask_bf16x2(vl.y, mk.y), mask_bf16x2(vl.z, mk.z),
                        mask_bf16x2(vl.w, mk.w));
    } else if (d.relu && !SPLIT) {
      v = make_uint4(relu_bf16x2(v.x), relu_bf16x2(v.y), relu_bf16x2(v.z), relu_bf16x2(v.w));
    }
    *reinterpret_cast<uint4*>(d.y + off) = v;
    if (SPLIT) *reinterpret_cast<uint4*>(d.y_lo + off) = vl;
  }
}

// =====================================================================================
// dense GEMM on 128x128 tiles with split K (the fc forward)
// =====================================================================================
// igemm_dma_kernel's 64x64 tiles stream every activation row once per 64 output
// columns and every weight row once per 64 batch rows: for the split fc forward
// (1536 x 3136 -> 1024, hi + lo planes) that is ~616 MB of L2/MALL -> LDS traffic,
// and the traffic bounds it (a DMA-only variant takes 32 of its ~40 us).  Here a
// block owns a 128x128 output tile: four waves in 2x2, each 64x64 (4x4 MFMA tiles,
// every A and B fragment feeds four MFMAs per product), so the traffic halves and
// the LDS fragment reads per MFMA drop 2.5x.  The K range is split over gridDim.z so
// the 96 tiles of the fc still cover the chip; partials go to an fp32 workspace
// [z][M][N] and fc_splitk_epilogue_kernel sums them in fixed z order (deterministic),
// adds the bias, applies ReLU (or the dgrad mask) and writes the output planes.
// Staging is the LDS-DMA ring of igemm_dma_kernel (same swizzled images, same
// lane-source trick); A rows past M read row 0 and are dropped at the store.
// LW: four extra loader waves issue every DMA (the compute waves then carry only
// MFMAs and fragment reads; an LDS-DMA issue costs ~60 cycles of the issuing wave).
template <bool SPLIT, int NS, bool LW>
__global__ void __launch_bounds__(LW ? 512 : 256) fc_gemm128_kernel(ConvDesc d, float* __restrict__ ws, int kt_per) {
  constexpr int BM = 128, BN = 128;
  constexpr int HALF = (BM + BN) * 128;           // one precision plane of a stage
  constexpr int STAGE = SPLIT ? 2 * HALF : HALF;
  constexpr int NA = BM / 32, NB = BN / 32;       // DMA instructions per wave per plane
  constexpr int DPT = (NA + NB) * (SPLIT ? 2 : 1);
  static_assert(NS >= 2 && NS * STAGE <= 163840, "LDS ring");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = LW ? (tid >> 6) & 3 : tid >> 6;
  const bool loader = !LW || tid >= 256, computer = !LW || tid < 256;
  const int ntm = gridDim.x, ntn = gridDim.y;
  // N tiles fastest, then M tiles, then K splits: the blocks of one XCD share A rows
  // and a K range (consecutive logical ids land on one XCD)
  const int wg = xcd_swizzle(blockIdx.x + ntm * (blockIdx.y + ntn * blockIdx.z), ntm * ntn * gridDim.z);
  const int M = d.N, Nc = d.Cout;
  const int KT = d.K >> 6;
  const uint8_t* xa = reinterpret_cast<const uint8_t*>(d.x);
  const uint8_t* xl = SPLIT ? reinterpret_cast<const uint8_t*>(d.x_lo) : xa;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)smem;
  const int wm = wv >> 1, wn = wv & 1;

  // one (tile, K range) per workgroup
  {
    const int tile = wg % (ntn * ntm);
    const int bz = wg / (ntn * ntm);
    const int kt0 = bz * kt_per;
    const int nk = min(KT, kt0 + kt_per) - kt0;      // >= 1 (host sizes the grid)
    const int by = tile % ntn;
    const int bx = tile / ntn;
    const RowTile rt = row_tile(d, bx, BM, M);
    const int m0 = rt.m0, mend = rt.mend, n0 = by * BN;
    const bool second = rt.second;
    const uint8_t* wb = reinterpret_cast<const uint8_t*>(second ? d.w2 : d.w);
    const uint8_t* wl = SPLIT ? reinterpret_cast<const uint8_t*>(second ? d.w2_lo : d.w_lo) : wb;

    // instruction i of wave wv fills tile rows 8 (wv + 4 i) .. +7: lane >> 3 picks the
    // row, lane & 7 the LDS slot, and the source chunk is the one swz_row puts there
    uint32_t a_off[NA], b_off[NB];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int r = 8 * (wv + 4 * i) + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int m = m0 + r < mend ? m0 + r : 0;
      a_off[i] = ((uint32_t)m * d.K + c * 8) * 2u;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int r = 8 * (wv + 4 * i) + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      b_off[i] = ((uint32_t)(n0 + r) * d.K + c * 8) * 2u;
    }
    int lt = 0;
    auto issue = [&]() {
      const uint32_t dst = lds0 + (uint32_t)(lt % NS) * STAGE;
      const uint32_t toff = (uint32_t)(kt0 + lt) * 128u;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const uint32_t l = __builtin_amdgcn_readfirstlane(dst + (wv + 4 * i) * 1024);
        dma16(xa + a_off[i] + toff, l);
        if (SPLIT) dma16(xl + a_off[i] + toff, l + HALF);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const uint32_t l = __builtin_amdgcn_readfirstlane(dst + BM * 128 + (wv + 4 * i) * 1024);
        dma16(wb + b_off[i] + toff, l);
        if (SPLIT) dma16(wl + b_off[i] + toff, l + HALF);
      }
      ++lt;
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int buf) {
      const uint8_t* As = smem + buf * STAGE;
      const uint8_t* Bs = As + BM * 128;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int c = 4 * s + (lane >> 4);
        bf16x8 a[4], b[4], al[4], bl[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          a[t] = *reinterpret_cast<const bf16x8*>(As + swz_row(64 * wm + 16 * t + (lane & 15), c));
          b[t] = *reinterpret_cast<const bf16x8*>(Bs + swz_row(64 * wn + 16 * t + (lane & 15), c));
          if (SPLIT) {
            al[t] = *reinterpret_cast<const bf16x8*>(As + HALF + swz_row(64 * wm + 16 * t + (lane & 15), c));
            bl[t] = *reinterpret_cast<const bf16x8*>(Bs + HALF + swz_row(64 * wn + 16 * t + (lane & 15), c));
          }
        }
        // product-major order: 16 independent accumulators between dependent MFMAs
        if (SPLIT) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[nt], a[mt], acc[mt][nt], 0, 0, 0);
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], al[mt], acc[mt][nt], 0, 0, 0);
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nt], a[mt], acc[mt][nt], 0, 0, 0);
      }
    };

    if (loader) {
#pragma unroll
      for (int p = 0; p < NS - 1; ++p)
        if (p < nk) issue();
    }
    for (int j = 0; j < nk; ++j) {
      if (loader) vmcnt_le(min(NS - 2, nk - 1 - j) * DPT);
      __syncthreads();
      if (loader && j + NS - 1 < nk) issue();
      if (computer) compute(j % NS);
    }

    // partial tile -> ws[bz][m][n]: lane (g = lane >> 4, pl = lane & 15) of MFMA tile
    // (mt, nt) holds row 16 mt + pl, columns 16 nt + 4 g .. +3
    if (computer) {
      float* wz = ws + (int64_t)bz * M * Nc;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int m = m0 + 64 * wm + 16 * mt + (lane & 15);
        if (m >= mend) continue;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int n = n0 + 64 * wn + 16 * nt + 4 * (lane >> 4);
          *reinterpret_cast<f32x4*>(wz + (int64_t)m * Nc + n) = acc[mt][nt];
        }
      }
    }
  }
}

// y[m][n] = act(sum_z ws[z][m][n] * in_scale + bias[n]): 8 outputs per thread, the
// z partials summed in fixed order.  act = ReLU (fp32, before the hi / lo split) or
// the dgrad mask (both planes, from the producer's bf16 activation).
// Side job (pk.out != null): blocks past the epilogue's grid pack the conv2 weights
// for the step's conv2 data gradient (csrc/conv2_wfrag.h) -- a launch of its own costs
// ~5 us in the step's graph; here it rides on an elementwise pass.

template <bool SPLIT>
__global__ void __launch_bounds__(256) fc_splitk_epilogue_kernel(ConvDesc d, const float* __restrict__ ws,
                                                                 int nz, int eb, C2dPackJob pk) {
  if ((int)blockIdx.x >= eb) {
    pack_c2d_wfrag_word(((int)blockIdx.x - eb) * 256 + threadIdx.x, pk.w, pk.w_lo, pk.out);
    return;
  }
  const int Nc = d.Cout;
  const int64_t MN = (int64_t)d.N * Nc;
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (e >= MN) return;
  const int m = (int)(e / Nc), n = (int)(e - (int64_t)m * Nc);
  float v[8];
  {
    const float4 p0 = *reinterpret_cast<const float4*>(ws + e);
    const float4 p1 = *reinterpret_cast<const float4*>(ws + e + 4);
    v[0] = p0.x; v[1] = p0.y; v[2] = p0.z; v[3] = p0.w;
    v[4] = p1.x; v[5] = p1.y; v[6] = p1.z; v[7] = p1.w;
  }
  for (int z = 1; z < nz; ++z) {
    const float4 p0 = *reinterpret_cast<const float4*>(ws + z * MN + e);
    const float4 p1 = *reinterpret_cast<const float4*>(ws + z * MN + e + 4);
    v[0] += p0.x; v[1] += p0.y; v[2] += p0.z; v[3] += p0.w;
    v[4] += p1.x; v[5] += p1.y; v[6] += p1.z; v[7] += p1.w;
  }
  const float* __restrict__ bias = (d.w2 != nullptr && m >= d.m_switch) ? d.bias2 : d.bias;
  float b8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(bias + n);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + n + 4);
    b8[0] = b0.x; b8[1] = b0.y; b8[2] = b0.z; b8[3] = b0.w;
    b8[4] = b1.x; b8[5] = b1.y; b8[6] = b1.z; b8[7] = b1.w;
  }
  const bool relu = d.relu && d.mask == nullptr;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    v[r] = v[r] * d.in_scale + b8[r];
    if (relu) v[r] = fmaxf(v[r], 0.f);
  }
  const int64_t off = (int64_t)m * d.ldy + n;
  uint32_t h[4], l[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (SPLIT) split_pk_bf16(v[2 * q], v[2 * q + 1], h[q], l[q]);
    else h[q] = cvt_pk_bf16(v[2 * q], v[2 * q + 1]);
  }
  if (d.mask) {
    const uint4 mk = *reinterpret_cast<const uint4*>(d.mask + off);
    const uint32_t mm[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      h[q] = mask_bf16x2(h[q], mm[q]);
      if (SPLIT) l[q] = mask_bf16x2(l[q], mm[q]);
    }
  }
  *reinterpret_cast<uint4*>(d.y + off) = make_uint4(h[0], h[1], h[2], h[3]);
  if (SPLIT) *reinterpret_cast<uint4*>(d.y_lo + off) = make_uint4(l[0], l[1], l[2], l[3]);
}

// weight gradient: csrc/igemm_wgrad.h (igemm_wgrad_body)
// three-stage LDS-DMA ring where it fits next to the row table (else two)
template <int MODE, int CT, int NT, int SP>
constexpr int wgrad_stages() {
  constexpr int nimg = CT + NT + (SP == 0 ? 0 : (SP == 1 ? CT + NT : CT));
  return SP != 0 && 3 * nimg * WG_IMG + (MODE == 0 ? 0 : WG_TBL * 4) <= 163840 ? 3 : 2;
}

template <int MODE, int OWC, int OHWC, int CT, int NT, int SP>
__global__ void __launch_bounds__(256) igemm_wgrad_kernel(WgradDesc d) {
  igemm_wgrad_body<MODE, OWC, OHWC, CT, NT, SP, wgrad_stages<MODE, CT, NT, SP>()>(d, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                                                gridDim.x, gridDim.y, gridDim.z);
}

// Sum the fp32 split-K slabs -> fp32 gradient (scaled) and the bias partials.
// Block = 16 float4 columns x 16 split groups (256 threads): every thread keeps
// its loads independent (nsplit/16 in flight), an LDS tree finishes, and the
// grid has n/64 blocks so even the 16K-element conv1 gradient fills the chip.
// The last ceil(nb/64) blocks reduce the bias slab the same way.
// s2dC > 0: the slab is in conv1's space-to-depth K order (csrc/conv1_s2d.hip);
// the store permutes it back to OIHW (each float4 = 4 consecutive kw: contiguous).
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab, int nsplit, int64_t n,
                                                          float scale, float* __restrict__ out,
                                                          const float* __restrict__ bslab, int nb,
                                                          float* __restrict__ bout, int s2dC, int Kc) {
  __shared__ float4 red[16][16];
  const int lc = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t nwb = (n / 4 + 15) / 16;
  const bool bias = blockIdx.x >= nwb;
  const float* src = bias ? bslab : slab;
  const int64_t stride = bias ? nb : n;
  const int64_t n4 = bias ? nb / 4 : n / 4;
  const int64_t c4 = (bias ? (int64_t)(blockIdx.x - nwb) : (int64_t)blockIdx.x) * 16 + lc;
  float4 s = make_float4(0, 0, 0, 0);
  if (c4 < n4) {
#pragma unroll 4
    for (int k = grp; k < nsplit; k += 16) {
      const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)k * stride + c4 * 4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[grp][lc] = s;
  __syncthreads();
  if (grp == 0 && c4 < n4) {
    float4 a = red[0][lc];
#pragma unroll
    for (int g = 1; g < 16; ++g) {
      const float4 b = red[g][lc];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    if (bias) {
      *reinterpret_cast<float4*>(bout + c4 * 4) = a;
      return;
    }
    a.x *= scale; a.y *= scale; a.z *= scale; a.w *= scale;
    int64_t o = c4 * 4;
    if (s2dC > 0) {
      const int64_t row = o / Kc;
      const int k = (int)(o - row * Kc);
      const int q = k >> 4, r4 = (k >> 2) & 3;
      const int tap = q / s2dC, c = q - tap * s2dC;
      o = row * Kc + (c * 8 + 4 * (tap >> 1) + r4) * 8 + 4 * (tap & 1);
    }
    *reinterpret_cast<float4*>(out + o) = a;
  }
}

// Pack the bf16 weight copies the dgrad GEMMs read as their B operand:
//  WfcT[n][k] = Wfc[k][n]                              (3136 x 1024, LDS-tiled transpose)
//  W3TF[ci][kh][kw][co] = W3[co][2-kh][2-kw][ci]        (flipped + transposed; 64 x 576)
//  W2T[cls=(p,q)][ci][a][b][co] = W2[co][p+2(1-a)][q+2(1-b)][ci]   (4 x 64 x 256)
__global__ void __launch_bounds__(256) transpose_bf16_kernel(const bf16_t* __restrict__ src, int R, int C,
                                                             bf16_t* __restrict__ dst) {
  __shared__ bf16_t t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, c = i & 63;
    if (r0 + r < R && c0 + c < C) t[r][c] = src[(int64_t)(r0 + r) * C + c0 + c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int c = i >> 6, r = i & 63;
    if (r0 + r < R && c0 + c < C) dst[(int64_t)(c0 + c) * R + r0 + r] = t[r][c];
  }
}

__global__ void pack_conv_dgrad_weights_kernel(const bf16_t* __restrict__ w3, const bf16_t* __restrict__ w2,
                                               bf16_t* __restrict__ w3tf, bf16_t* __restrict__ w2t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n1 = 64LL * 576, n2 = 4LL * 64 * 256;
  if (i < n1) {
    const int ci = (int)(i / 576), r = (int)(i - (int64_t)ci * 576);
    const int kh = r / 192, kw = (r / 64) % 3, co = r & 63;
    w3tf[i] = w3[((co * 3 + (2 - kh)) * 3 + (2 - kw)) * 64 + ci];
  } else if (i < n1 + n2) {
    const int64_t j = i - n1;
    const int cls = (int)(j / (64 * 256)), r = (int)(j - (int64_t)cls * 64 * 256);
    const int ci = r / 256, r2 = r & 255;
    const int a = r2 / 128, b = (r2 / 64) & 1, co = r2 & 63;
    const int p = cls >> 1, qq = cls & 1;
    const int kh = p + 2 * (1 - a), kw = qq + 2 * (1 - b);
    w2t[j] = w2[((co * 4 + kh) * 4 + kw) * 64 + ci];
  }
}

// ------------------------------------------------------------------ launchers
template <int BM, bool SPLIT>
static void launch_fwd(const ConvDesc& d, dim3 grid, hipStream_t st) {
  const bool pad = d.pad_h > 0 || d.pad_w > 0;
  const bool g9 = d.OH == 9 && d.OW == 9, g7 = d.OH == 7 && d.OW == 7, g10 = d.OH == 10 && d.OW == 10;
  if (d.mode == 0 && d.bt) igemm_fwd_kernel<0, false, true, 1, 1, BM, SPLIT><<<grid, 256, 0, st>>>(d);
  else if (d.mode == 0) igemm_fwd_kernel<0, false, false, 1, 1, BM, SPLIT><<<grid, 256, 0, st>>>(d);
  else if (pad && d.bt) {
    // dgrad: conv3 (9x9 out), conv2 per parity class (10x10 out)
    if (g9) igemm_fwd_kernel<1, true, true, 9, 81, BM, SPLIT><<<grid, 256, 0, st>>>(d);
    else if (g10) igemm_fwd_kernel<1, true, true, 10, 100, BM, SPLIT><<<grid, 256, 0, st>>>(d);
    else igemm_fwd_kernel<1, true, true, 0, 0, BM, SPLIT><<<grid, 256, 0, st>>>(d);
  } else if (pad) igemm_fwd_kernel<1, true, false, 0, 0, BM, SPLIT><<<grid, 256, 0, st>>>(d);
  else if (d.bt) igemm_fwd_kernel<1, false, true, 0, 0, BM, SPLIT><<<grid, 256, 0, st>>>(d);
  else if (g9) igemm_fwd_kernel<1, false, false, 9, 81, BM, SPLIT><<<grid, 256, 0, st>>>(d);   // conv2 fwd
  else if (g7) igemm_fwd_kernel<1, false, false, 7, 49, BM, SPLIT><<<grid, 256, 0, st>>>(d);   // conv3 fwd
  else igemm_fwd_kernel<1, false, false, 0, 0, BM, SPLIT><<<grid, 256, 0, st>>>(d);
}

template <bool SPLIT, int NS, int BM>
static void launch_dma(const ConvDesc& d, dim3 grid, hipStream_t st) {
  const bool pad = d.pad_h > 0 || d.pad_w > 0;
  const bool g9 = d.OH == 9 && d.OW == 9, g7 = d.OH == 7 && d.OW == 7, g10 = d.OH == 10 && d.OW == 10;
  if (d.mode == 0 && d.bt) igemm_dma_kernel<0, false, true, 1, 1, SPLIT, NS, BM><<<grid, 256, 0, st>>>(d);
  else if (d.mode == 0) igemm_dma_kernel<0, false, false, 1, 1, SPLIT, NS, BM><<<grid, 256, 0, st>>>(d);
  else if (pad && d.bt) {
    if (g9) igemm_dma_kernel<1, true, true, 9, 81, SPLIT, NS, BM><<<grid, 256, 0, st>>>(d);
    else if (g10) igemm_dma_kernel<1, true, true, 10, 100, SPLIT, NS, BM><<<grid, 256, 0, st>>>(d);
    else igemm_dma_kernel<1, true, true, 0, 0, SPLIT, NS, BM><<<grid, 256, 0, st>>>(d);
  } else if (pad) igemm_dma_kernel<1, true, false, 0, 0, SPLIT, NS, BM><<<grid, 256, 0, st>>>(d);
  else if (d.bt) igemm_dma_kernel<1, false, true, 0, 0, SPLIT, NS, BM><<<grid, 256, 0, st>>>(d);
  else if (g9) igemm_dma_kernel<1, false, false, 9, 81, SPLIT, NS, BM><<<grid, 256, 0, st>>>(d);
  else if (g7) igemm_dma_kernel<1, false, false, 7, 49, SPLIT, NS, BM><<<grid, 256, 0, st>>>(d);
  else igemm_dma_kernel<1, false, false, 0, 0, SPLIT, NS, BM><<<grid, 256, 0, st>>>(d);
}

// Dense C[M,N] = act(A[M,K] . B[N,K]^T + b) on 128x128 tiles, K split `ksplit` ways
// (fc_gemm128_kernel + fc_splitk_epilogue_kernel).  ws: fp32 workspace of at least
// ksplit * M * N elements.  Row-major B only (d.bt == 0), N % 128 == 0.  pk: optional
// conv2 weight-fragment pack riding on the epilogue launch (fc_splitk_epilogue_kernel).
// no_epilogue: only the GEMM runs; the caller consumes the ws partials.
// (A stream-K split was measured slower -- fc 43.1 vs 40.5 us at 512 rows, 18.8 vs
// 12.6 at 74, profiles/r4_ab_fc_stream_k_rejected.txt -- and removed.)
APEX_EXPORT int apex_fc_gemm128(ConvDesc d, float* ws, int64_t ws_elems, int ksplit, int loader_waves,
                                int no_epilogue, C2dPackJob pk, hipStream_t st) {
  if (d.mode != 0 || d.bt != 0 || (d.K & 63) || d.K <= 0 || (d.Cout & 127) || d.N <= 0 || ksplit < 1)
    return (int)hipErrorInvalidValue;
  if ((d.ldy & 7) || d.ldy < d.Cout) return (int)hipErrorInvalidValue;
  if ((int64_t)d.N * d.K * 2 >= 0x7ffffff0LL || (int64_t)d.Cout * d.K * 2 >= 0x7ffffff0LL)
    return (int)hipErrorInvalidValue;
  if (d.w2 != nullptr && (d.m_switch < 0 || d.m_switch > d.N)) return (int)hipErrorInvalidValue;
  const bool split = d.x_lo != nullptr;
  if (split && (d.w_lo == nullptr || d.y_lo == nullptr || (d.w2 != nullptr && d.w2_lo == nullptr)))
    return (int)hipErrorInvalidValue;
  const int KT = d.K >> 6;
  const int kt_per = (KT + ksplit - 1) / ksplit;
  const int nz = (KT + kt_per - 1) / kt_per;
  const dim3 grid(row_tiles(d, d.N, 128), d.Cout / 128, nz);
  if (ws == nullptr || nz < 1 || ws_elems < (int64_t)nz * d.N * d.Cout) return (int)hipErrorInvalidValue;
  if (loader_waves) {
    if (split) fc_gemm128_kernel<true, 2, true><<<grid, 512, 0, st>>>(d, ws, kt_per);
    else fc_gemm128_kernel<false, 4, true><<<grid, 512, 0, st>>>(d, ws, kt_per);
  } else {
    if (split) fc_gemm128_kernel<true, 2, false><<<grid, 256, 0, st>>>(d, ws, kt_per);
    else fc_gemm128_kernel<false, 4, false><<<grid, 256, 0, st>>>(d, ws, kt_per);
  }
  const int64_t nthr = (int64_t)d.N * d.Cout / 8;
  const int eb = (int)((nthr + 255) / 256);
  // no_epilogue: the partials stay in ws for the consumer (csrc/head_common.h
  // load_row_part: the DDQN head sums them itself)
  if (no_epilogue) {
    if (pk.out != nullptr) return (int)hipErrorInvalidValue;
    APEX_CHECK_LAUNCH();
  }
  if (pk.out != nullptr && (pk.w == nullptr || ((uintptr_t)pk.out & 15))) return (int)hipErrorInvalidValue;
  const int pb = pk.out != nullptr ? C2D_PACK_THREADS / 256 : 0;
  if (split) fc_splitk_epilogue_kernel<true><<<eb + pb, 256, 0, st>>>(d, ws, nz, eb, pk);
  else fc_splitk_epilogue_kernel<false><<<eb + pb, 256, 0, st>>>(d, ws, nz, eb, pk);
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_conv_fwd(ConvDesc d, hipStream_t st) {
  if ((d.K & 63) || (d.Cout & 63) || d.K <= 0) return (int)hipErrorInvalidValue;
  if (d.mode == 1 && (d.Cin & 63)) return (int)hipErrorInvalidValue;
  if (d.mode != 0 && d.mode != 1) return (int)hipErrorInvalidValue;
  // buffer addressing: 32-bit byte offsets
  const int64_t xbytes = d.mode == 0 ? (int64_t)d.N * d.K * 2 : (int64_t)d.N * d.H * d.W * d.Cin * 2;
  if (xbytes >= 0x7ffffff0LL) return (int)hipErrorInvalidValue;
  if (d.mode == 1 && (d.pad_h > 0 || d.pad_w > 0) && d.KH * d.KW > 32) return (int)hipErrorInvalidValue;
  if (d.w2 != nullptr && (d.m_switch < 0 || d.m_switch > d.N * d.OH * d.OW)) return (int)hipErrorInvalidValue;
  if (d.bt == 1 && (d.K >> 6) * (d.ncls > 0 ? d.ncls : 1) > 16) return (int)hipErrorInvalidValue;
  // split mode: every lo plane present (and the target set's when there is one)
  const bool split = d.x_lo != nullptr;
  if (split && (d.w_lo == nullptr || d.y_lo == nullptr || (d.w2 != nullptr && d.w2_lo == nullptr)))
    return (int)hipErrorInvalidValue;
  const int M = d.N * d.OH * d.OW;
  const int ncls = d.ncls > 0 ? d.ncls : 1;
  // 128-row tiles unless that leaves the chip under ~2.5 blocks per CU
  const int64_t blocks128 = (int64_t)((M + 127) / 128) * (d.Cout / FWD_BN) * ncls;
  const bool pad = d.pad_h > 0 || d.pad_w > 0;
  // measured (scripts/bench_kernels.py sweep): 64-row tiles pay off for the dgrad
  // GEMMs (K-major B): conv3/conv2 dgrad and fc dgrad; 128 for the conv forward
  // GEMMs; 64 for a forward grid of < 1 block per CU (the fc: 192 -> 384 blocks,
  // 3446 -> 3491 steps/s end to end).  Split mode doubles the LDS stages (96 KB
  // at 128 rows: one block per CU), so it takes 64-row tiles throughout.
  bool bm64 = split ? true : (d.bt != 0 ? (pad || blocks128 < 640) : blocks128 < 256);
  if (d.tile_hint == 1) bm64 = false;
  if (d.tile_hint == 2) bm64 = true;
  if (d.order_hint == 0) d.order_hint = (d.mode == 0 && !d.bt && d.Cout >= 512) ? 2 : 1;
  const dim3 g64(row_tiles(d, M, 64), d.Cout / FWD_BN, ncls), g128(row_tiles(d, M, 128), d.Cout / FWD_BN, ncls);
  // LDS-DMA kernel (scripts/bench_dma_gemm.py, learner shapes at batch 512, us):
  //   split: 64-row tiles, 2 stages (two blocks per CU) win everywhere -- fc fwd 39.6
  //     (register-staged 51.5), fc dgrad 17.9 (22.7), conv3 fwd 27.9 (32.0), conv3
  //     dgrad 20.4 (22.3), generic conv2 dgrad 46.1 (52.8; the image-resident kernel
  //     ties at 45.9 and stays);
  //   bf16: fc fwd 64-row, 3 stages 22.4 (26.6), fc dgrad 64-row, 2 stages 10.3 (11.5);
  //     the conv GEMMs tie or lose and stay register-staged.
  // tile_hint 3 / 4 / 5 force 128-row 3-stage / 64-row 2-stage / 64-row 3-stage.
  // (Loader waves -- 4 extra waves issuing the DMAs -- measured no gain on these
  // 64-row tiles: split fc fwd 40.7 vs 40.1, conv3 fwd 29.3 vs 28.9 us,
  // profiles/r2_dma_gemm_loader_waves.json; they pay on the 128x128 fc tiles.)
  const int dma = d.tile_hint >= 3 ? d.tile_hint
                : d.tile_hint != 0 ? 0
                : split ? 4 : (d.mode == 0 ? (d.bt ? 4 : 5) : 0);
  if (dma == 3) {
    if (split) launch_dma<true, 3, 128>(d, g128, st);
    else launch_dma<false, 3, 128>(d, g128, st);
  } else if (dma == 4) {
    if (split) launch_dma<true, 2, 64>(d, g64, st);
    else launch_dma<false, 2, 64>(d, g64, st);
  } else if (dma == 5) {
    if (split) launch_dma<true, 3, 64>(d, g64, st);
    else launch_dma<false, 3, 64>(d, g64, st);
  } else if (split) {
    if (bm64) launch_fwd<64, true>(d, g64, st);
    else launch_fwd<128, true>(d, g128, st);
  } else {
    if (bm64) launch_fwd<64, false>(d, g64, st);
    else launch_fwd<128, false>(d, g128, st);
  }
  APEX_CHECK_LAUNCH();
}

// Block shape: fewest re-read bytes -- X is read once per Co group (ct / CT
// times), dY once per Kc group (kt / NT times); 4-tile shapes keep every wave busy.
template <int MODE, int OWC, int OHWC, int SP>
static void launch_wgrad(const WgradDesc& d, int nsplit, hipStream_t st) {
  const int kt = d.Kc / 64, ct = d.Co / 64;
  const int best = wgrad_shape(kt, ct, d.Kc, d.Co, SP);
  const WgShape cands[WG_NSHAPES] = {{1, 4}, {2, 2}, {4, 1}, {1, 3}, {1, 1}, {1, 2}, {2, 1}};
  const dim3 grid(kt / cands[best].n, ct / cands[best].c, nsplit);
  if constexpr (SP == 0) {
    switch (best) {
      case 0: igemm_wgrad_kernel<MODE, OWC, OHWC, 1, 4, 0><<<grid, 256, 0, st>>>(d); break;
      case 1: igemm_wgrad_kernel<MODE, OWC, OHWC, 2, 2, 0><<<grid, 256, 0, st>>>(d); break;
      case 2: igemm_wgrad_kernel<MODE, OWC, OHWC, 4, 1, 0><<<grid, 256, 0, st>>>(d); break;
      case 3: igemm_wgrad_kernel<MODE, OWC, OHWC, 1, 3, 0><<<grid, 256, 0, st>>>(d); break;
      default: igemm_wgrad_kernel<MODE, OWC, OHWC, 1, 1, 0><<<grid, 256, 0, st>>>(d); break;
    }
  } else {
    switch (best) {
      case 1: igemm_wgrad_kernel<MODE, OWC, OHWC, 2, 2, SP><<<grid, 256, 0, st>>>(d); break;
      case 3: igemm_wgrad_kernel<MODE, OWC, OHWC, 1, 3, SP><<<grid, 256, 0, st>>>(d); break;
      case 5: igemm_wgrad_kernel<MODE, OWC, OHWC, 1, 2, SP><<<grid, 256, 0, st>>>(d); break;
      case 6: igemm_wgrad_kernel<MODE, OWC, OHWC, 2, 1, SP><<<grid, 256, 0, st>>>(d); break;
      default: igemm_wgrad_kernel<MODE, OWC, OHWC, 1, 1, SP><<<grid, 256, 0, st>>>(d); break;
    }
  }
}

APEX_EXPORT int apex_conv_wgrad(WgradDesc d, float* out, float* bout, int nsplit, float scale, hipStream_t st) {
  if ((d.Kc & 63) || (d.Co & 63)) return (int)hipErrorInvalidValue;
  if (d.mode == 1 && ((d.Cin & 63) || d.pad_h || d.pad_w)) return (int)hipErrorInvalidValue;
  // per-block row-offset table capacity (rounded up to 64-row steps)
  const int trows = (d.rows_per_split + WG_ROWS - 1) / WG_ROWS * WG_ROWS;
  if (d.mode == 1 && trows > WG_TBL) return (int)hipErrorInvalidValue;
  if (d.mode == 2 && (d.Cin * trows > WG_TBL || d.Cin > 4)) return (int)hipErrorInvalidValue;
  if ((int64_t)d.Mred * d.ldd * 2 >= 0x7ffffff0LL) return (int)hipErrorInvalidValue;
  if (d.mode == 0 && (int64_t)d.Mred * d.ldx * 2 >= 0x7ffffff0LL) return (int)hipErrorInvalidValue;
  // split mode: dY lo plane; X lo plane too except for the exact uint8 frames (mode 2)
  const bool split = d.dy_lo != nullptr;
  if (split && d.mode != 2 && d.x_lo == nullptr) return (int)hipErrorInvalidValue;
  // learner shapes get compile-time output geometry (conv3 7x7, conv2 9x9, conv1 20x20)
  if (d.mode == 0) {
    if (split) launch_wgrad<0, 1, 1, 1>(d, nsplit, st);
    else launch_wgrad<0, 1, 1, 0>(d, nsplit, st);
  } else if (d.mode == 1 && d.OH == 7 && d.OW == 7) {
    if (split) launch_wgrad<1, 7, 49, 1>(d, nsplit, st);
    else launch_wgrad<1, 7, 49, 0>(d, nsplit, st);
  } else if (d.mode == 1 && d.OH == 9 && d.OW == 9) {
    if (split) launch_wgrad<1, 9, 81, 1>(d, nsplit, st);
    else launch_wgrad<1, 9, 81, 0>(d, nsplit, st);
  } else if (d.mode == 1) {
    if (split) launch_wgrad<1, 0, 0, 1>(d, nsplit, st);
    else launch_wgrad<1, 0, 0, 0>(d, nsplit, st);
  } else if (split) {
    // conv1 in split mode: dY hi + lo against the exact frames (20 x 20 output only)
    const int kt = d.Kc / 64;
    const dim3 grid(1, d.Co / 64, nsplit);
    if (d.OH != 20 || d.OW != 20) return (int)hipErrorInvalidValue;
    if (kt == 4) igemm_wgrad_kernel<2, 20, 400, 1, 4, 2><<<grid, 256, 0, st>>>(d);
    else if (kt == 2) igemm_wgrad_kernel<2, 20, 400, 1, 2, 2><<<grid, 256, 0, st>>>(d);
    else if (kt == 1) igemm_wgrad_kernel<2, 20, 400, 1, 1, 2><<<grid, 256, 0, st>>>(d);
    else return (int)hipErrorInvalidValue;
  } else {
    // conv1: Kc = 64 C (C = 1, 2, 4 stacked frames) -> all Kc tiles in one block
    const int kt = d.Kc / 64;
    const dim3 grid(1, d.Co / 64, nsplit);
    const bool fixed = d.OH == 20 && d.OW == 20;
    if (kt == 4 && fixed) igemm_wgrad_kernel<2, 20, 400, 1, 4, 0><<<grid, 256, 0, st>>>(d);
    else if (kt == 2 && fixed) igemm_wgrad_kernel<2, 20, 400, 1, 2, 0><<<grid, 256, 0, st>>>(d);
    else if (kt == 1 && fixed) igemm_wgrad_kernel<2, 20, 400, 1, 1, 0><<<grid, 256, 0, st>>>(d);
    else if (kt == 4) igemm_wgrad_kernel<2, 0, 0, 1, 4, 0><<<grid, 256, 0, st>>>(d);
    else if (kt == 2) igemm_wgrad_kernel<2, 0, 0, 1, 2, 0><<<grid, 256, 0, st>>>(d);
    else if (kt == 1) igemm_wgrad_kernel<2, 0, 0, 1, 1, 0><<<grid, 256, 0, st>>>(d);
    else return (int)hipErrorInvalidValue;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  if (out != nullptr) {
    const int64_t n = (int64_t)d.Co * d.Kc;
    const int nb = d.bias_slab ? d.Co : 0;
    const int64_t blocks = (n / 4 + 15) / 16 + (nb / 4 + 15) / 16;
    slab_reduce_kernel<<<(int)blocks, 256, 0, st>>>(d.slab, nsplit, n, scale, out, d.bias_slab, nb, bout,
                                                    d.mode == 2 ? d.Cin : 0, d.Kc);
  }
  APEX_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// One launch that finalises every split-K gradient of the step (conv3, conv2,
// conv1 slabs + their bias slabs) and, optionally, writes one squared-norm
// partial per block of the values it stores plus one for an extra plain range
// (the head gradients): with the fc wgrad's epilogue partials these cover the
// whole flat gradient, so the clip norm needs no separate pass over 13 MB.
struct RedJob {
  const float* slab;
  const float* bslab;
  float* out;
  float* bout;
  int64_t n;                 // weight elements (multiple of 4)
  int nsplit, nb, s2dC, Kc;
  float scale;
  int blk0;                  // first block of this job
  int cpb;                   // 16-float4 column chunks per block (>= 1: wide jobs, fewer blocks);
                             // < 0: direct mode (few splits): one float4 column per thread,
                             // -cpb passes of 256 columns per block, splits summed in order
  double* jnorm;             // null, or this job's own squared-norm partials: jnorm[block - blk0]
};

struct FinalizeDesc {
  RedJob job[4];
  int njobs;
  int nrm_n;                 // plain range [nrm_ptr, nrm_ptr + nrm_n): norm only (last block)
  const float* nrm_ptr;
  double* norm_part;         // null: no norm partials
  int norm_slot0;
  int nblocks;
};

__global__ void __launch_bounds__(256) grad_finalize_kernel(FinalizeDesc d) {
  __shared__ float4 red[16][16];
  __shared__ float nred[4];
  const int lc = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int b = blockIdx.x;
  float ss = 0.f;
  int j = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (k < d.njobs && b >= d.job[k].blk0) j = k;
  const int last_blk = d.nblocks - 1;
  double* jn = nullptr;                // the block's slot in its job's own partials (RedJob.jnorm)
  if (d.nrm_n > 0 && b == last_blk) {
    for (int i = threadIdx.x; i < d.nrm_n; i += 256) ss += d.nrm_ptr[i] * d.nrm_ptr[i];
  } else if (j >= 0 && d.job[j].cpb < 0) {
    // direct mode: thread = float4 column, the splits summed in order 0, 1, ... (the same
    // values as the 16-group reduction when nsplit <= 16)
    const RedJob& J = d.job[j];
    const int lb = b - J.blk0, np = -J.cpb;
    const int64_t nwb = (J.n / 4 + 256 * np - 1) / (256 * np);
    const bool bias = lb >= nwb;
    const float* src = bias ? J.bslab : J.slab;
    const int64_t stride = bias ? J.nb : J.n;
    const int64_t n4 = bias ? J.nb / 4 : J.n / 4;
    for (int q = 0; q < np; ++q) {
      const int64_t c4 = ((bias ? (int64_t)(lb - nwb) : (int64_t)lb) * np + q) * 256 + threadIdx.x;
      if (c4 >= n4) break;
      float4 a = *reinterpret_cast<const float4*>(src + c4 * 4);
      for (int k = 1; k < J.nsplit; ++k) {
        const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)k * stride + c4 * 4);
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
      if (bias) {
        *reinterpret_cast<float4*>(J.bout + c4 * 4) = a;
      } else {
        a.x *= J.scale; a.y *= J.scale; a.z *= J.scale; a.w *= J.scale;
        *reinterpret_cast<float4*>(J.out + c4 * 4) = a;
      }
      ss += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
    }
    jn = J.jnorm != nullptr ? J.jnorm + lb : nullptr;
  } else if (j >= 0) {
    const RedJob& J = d.job[j];
    const int lb = b - J.blk0;
    const int cpb = J.cpb > 1 ? J.cpb : 1;
    const int64_t nwb = (J.n / 4 + 16 * cpb - 1) / (16 * cpb);
    const bool bias = lb >= nwb;
    const float* src = bias ? J.bslab : J.slab;
    const int64_t stride = bias ? J.nb : J.n;
    const int64_t n4 = bias ? J.nb / 4 : J.n / 4;
    // (block-uniform trip count: every thread reaches the barriers)
    for (int q = 0; q < cpb; ++q) {
      const int64_t c4 = ((bias ? (int64_t)(lb - nwb) : (int64_t)lb) * cpb + q) * 16 + lc;
      float4 s = make_float4(0, 0, 0, 0);
      if (c4 < n4) {
#pragma unroll 4
        for (int k = grp; k < J.nsplit; k += 16) {
          const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)k * stride + c4 * 4);
          s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
      }
      if (q > 0) __syncthreads();          // the previous chunk's red[] reads are done
      red[grp][lc] = s;
      __syncthreads();
      if (grp == 0 && c4 < n4) {
        float4 a = red[0][lc];
#pragma unroll
        for (int g = 1; g < 16; ++g) {
          const float4 v = red[g][lc];
          a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
        }
        if (bias) {
          *reinterpret_cast<float4*>(J.bout + c4 * 4) = a;
        } else {
          a.x *= J.scale; a.y *= J.scale; a.z *= J.scale; a.w *= J.scale;
          int64_t o = c4 * 4;
          if (J.s2dC > 0) {
            const int64_t row = o / J.Kc;
            const int k = (int)(o - row * J.Kc);
            const int qq = k >> 4, r4 = (k >> 2) & 3;
            const int tap = qq / J.s2dC, c = qq - tap * J.s2dC;
            o = row * J.Kc + (c * 8 + 4 * (tap >> 1) + r4) * 8 + 4 * (tap & 1);
          }
          *reinterpret_cast<float4*>(J.out + o) = a;
        }
        ss += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
      }
    }
    jn = J.jnorm != nullptr ? J.jnorm + lb : nullptr;
  }
  if (d.norm_part == nullptr && jn == nullptr) return;
  ss = wave_sum_dpp(ss);
  if ((threadIdx.x & 63) == 0) nred[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = (double)nred[0] + nred[1] + nred[2] + nred[3];
    if (d.norm_part != nullptr) d.norm_part[d.norm_slot0 + b] = t;
    if (jn != nullptr) jn[0] = t;
  }
}

// Sum of the squared-norm partials of the step (fc wgrad epilogue + grad_finalize
// blocks) into one value for the optimizer: one small block, deterministic order.
// (A last-arriving-block total inside grad_finalize serialises ~1,900 returning
// atomics on one word: measured 10 % slower end to end.)
__global__ void __launch_bounds__(1024) norm_total_kernel(const double* __restrict__ part, int n,
                                                          double* __restrict__ total) {
  __shared__ double red[16];
  double t = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) t += part[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < 16; ++w) s += red[w];
    total[0] = s;
  }
}

APEX_EXPORT int apex_norm_total(const double* part, int n, double* total, hipStream_t st) {
  norm_total_kernel<<<1, 1024, 0, st>>>(part, n, total);
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_grad_finalize(FinalizeDesc d, hipStream_t st) {
  if (d.njobs < 0 || d.njobs > 4 || d.nblocks < 1) return (int)hipErrorInvalidValue;
  grad_finalize_kernel<<<d.nblocks, 256, 0, st>>>(d);
  APEX_CHECK_LAUNCH();
}

// standalone split-K finalisation (used by csrc/conv1_wgrad.hip's per-block partials)
APEX_EXPORT int apex_slab_reduce(const float* slab, int nsplit, int64_t n, float scale, float* out, const float* bslab,
                                 int nb, float* bout, int s2dC, int Kc, hipStream_t st) {
  const int64_t blocks = (n / 4 + 15) / 16 + (bslab ? (nb / 4 + 15) / 16 : 0);
  slab_reduce_kernel<<<(int)blocks, 256, 0, st>>>(slab, nsplit, n, scale, out, bslab, bslab ? nb : 0, bout, s2dC, Kc);
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_pack_dgrad_weights(const bf16_t* wfc, const bf16_t* w3, const bf16_t* w2, bf16_t* wfcT,
                                        bf16_t* w3tf, bf16_t* w2t, hipStream_t st) {
  transpose_bf16_kernel<<<dim3(3136 / 64, 1024 / 64), 256, 0, st>>>(wfc, 1024, 3136, wfcT);
  const int64_t n = 64LL * 576 + 4LL * 64 * 256;
  pack_conv_dgrad_weights_kernel<<<(int)((n + 255) / 256), 256, 0, st>>>(w3, w2, w3tf, w2t);
  APEX_CHECK_LAUNCH();
}

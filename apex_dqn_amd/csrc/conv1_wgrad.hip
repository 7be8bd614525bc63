// conv1 weight gradient on the space-to-depth frame ring, image-resident.
//
// Reference: the conv1 part of loss.backward() (learner.py:56) --
//   dW1[co][k] = sum_{img, pixel p} dY1[img][p][co] * X[img][p][k],  dB1[co] = sum dY1
// with X the 8x8/s4 im2col of the uint8 frame stack (K = 64 C in the s2d order
// k = ((tap*C + c)*16 + r4*4 + c4) of csrc/conv1_s2d.hip).
//
// A persistent workgroup (8 waves) walks whole images.  Per image, LDS holds
//   * the C frames as bf16 planes (frame c, half h) of 441 x 16 B, converted ONCE
//     from an LDS-DMA'd uint8 staging copy (the next image's frames stream in
//     while this one computes);
//   * the image's 400 x 64 dY1 rows (+16 zero rows), LDS-DMA'd with the
//     transposed-read swizzle applied through the SOURCE addresses.
// Work items: item i (< gridDim.x) is the image group {i, i + G, i + 2G, ...}; its
// partial goes to slab slot i.  Statically workgroup i does item i; with the work
// queue (d.wq, the data-parallel step, where RCCL's kernels can hold CUs) a resident
// workgroup takes the items of workgroups that have no CU yet.  Either way every slot
// holds the same image group's sum, so the reduction is bit-identical.
// The reduction runs over pixels (MFMA K = 32 pixels): dY fragments come from
// ds_read_b64_tr_b16 on the dY image, X fragments from ds_read_b64_tr_b16 with
// per-lane plane addresses (4 consecutive k of one pixel are 8 contiguous bytes).
// Wave w owns co half (w & 1) x K quarter (w >> 1): acc 2 x C tiles.  The bias
// gradient is 2 extra MFMAs per k-step against an all-ones fragment (K-quarter 0
// waves).  dW is read from L2/HBM exactly once per image (vs once per 64-wide
// K tile in the generic wgrad); each block writes one fp32 partial to the slab.
//
// SPLIT (fp32-accurate mode, dy_lo set): the frames are exact in bf16 and dY comes
// as hi + lo planes -- two MFMAs per fragment pair.  Both dY planes do not fit in
// LDS next to the frame planes, so an image's pixels run in two halves (224 + 192
// rows, the last 16 zero): per half both dY planes are LDS-DMA'd (rows past pixel
// 399 read the zero block), and the next image's frames stream in under half 1.
#include "mfma_common.h"

#define C1W_PLANE 7168
#define C1W_THREADS 512

struct Conv1WgDesc {
  const uint8_t* ring;        // s2d frame ring [F][21][21][16]
  const int32_t* slots;       // [N][C]
  const bf16_t* dy;           // [N][400][64]
  float* slab;                // [gridDim.x][64][64 C] partials (s2d K order)
  float* bias_slab;           // [gridDim.x][64]
  const uint8_t* zero16;      // 16 zero bytes (DMA filler)
  int N, C;
  const bf16_t* dy_lo;        // split mode: lo plane of dY (else null)
  unsigned long long* wq;     // item work queue counter (csrc/mfma_common.h wq_next); null: static order
};

template <int C, bool SPLIT>
__global__ void __launch_bounds__(C1W_THREADS, 1) conv1_wgrad_img_kernel(Conv1WgDesc d) {
  constexpr int K = 64 * C;
  constexpr int IMG = 2 * C * C1W_PLANE;
  constexpr int NCHUNK = C * 441;
  constexpr int NDMA = (NCHUNK + 63) / 64;
  constexpr int NW = C1W_THREADS / 64;
  constexpr int NDW = (NDMA + NW - 1) / NW;
  constexpr int STG = NDMA * 1024;
  // dY rows per LDS plane: 400 + 16 zero rows (13 k-steps of 32); SPLIT: one half
  // (224 rows = 7 k-steps, the second half 192) per plane, two planes
  constexpr int DYR = SPLIT ? 224 : 416;
  constexpr int NDY = 400 * 128 / 1024;  // dY DMA wave-instructions (8 rows each)
  constexpr int NDYW = (NDY + NW - 1) / NW;
  __shared__ __attribute__((aligned(16))) uint8_t smem[IMG + STG + (SPLIT ? 2 : 1) * DYR * 128];
  uint8_t* Pl = smem;
  uint8_t* Sg = Pl + IMG;
  uint8_t* Dy = Sg + STG;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, q = (lane >> 2) & 3, pcol = lane & 3;
  const int wc = wv & 1, wk = wv >> 1;   // co tiles 2wc, 2wc+1; K tiles C*wk .. C*wk + C-1

  // zero dY rows 400..415 once (never written by the DMA)
  if (!SPLIT) {
    for (int i = tid; i < 16 * 128 / 16; i += C1W_THREADS)
      *reinterpret_cast<uint4*>(Dy + 400 * 128 + i * 16) = make_uint4(0, 0, 0, 0);
  }

  // per-lane constant part of the X fragment address of each of this wave's K tiles:
  // tile t = (tap, frame c) block; lane reads k = 4 pcol .. +3 -> half pcol >> 1, +8 B for pcol & 1
  int xoff[C];
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const int t = C * wk + j, tap = t / C, c = t - tap * C;
    xoff[j] = (2 * c + (pcol >> 1)) * C1W_PLANE + (((tap >> 1) * 21 + (tap & 1)) << 4) + ((pcol & 1) << 3);
  }

  auto issue_frames = [&](int img) {
    int sl[4];
    sload_slots<C>(d.slots + img * C, sl);
#pragma unroll
    for (int i = 0; i < NDW; ++i) {
      const int k = wv * NDW + i;
      if (k < NDMA) {
        const int j = 64 * k + lane;
        const uint8_t* src = d.zero16;
        if (j < NCHUNK) {
          const int c = j / 441, blk = j - c * 441;
          int slot = sl[0];
#pragma unroll
          for (int cc = 1; cc < C; ++cc)
            if (c == cc) slot = sl[cc];
          src = d.ring + (int64_t)slot * 7056 + (blk << 4);
        }
        const uint32_t off = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(Sg + k * 1024);
        dma16(src, __builtin_amdgcn_readfirstlane(off));
      }
    }
  };
  // dY rows of one image -> swizzled transposed-read image: LDS chunk (r, pc) holds
  // logical chunk c = pc ^ (s(r) << 1) (swz_tr is an involution on the chunk index)
  auto issue_dy = [&](int img) {
#pragma unroll
    for (int i = 0; i < NDYW; ++i) {
      const int k = wv * NDYW + i;
      if (k < NDY) {
        const int r = 8 * k + (lane >> 3), pc = lane & 7;
        const int s = ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
        const int c = pc ^ (s << 1);
        const bf16_t* src = d.dy + ((int64_t)img * 400 + r) * 64 + c * 8;
        const uint32_t off = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(Dy + k * 1024);
        dma16(src, __builtin_amdgcn_readfirstlane(off));
      }
    }
  };
  // SPLIT: rows [224 h, 224 h + 224) of both dY planes (28 + 28 DMA instructions over
  // the 8 waves; local row = global row - 224 h keeps swz_tr's row bits, 224 % 16 == 0)
  constexpr int NDYS = 2 * DYR * 128 / 1024;
  constexpr int NDYSW = (NDYS + NW - 1) / NW;
  auto issue_dy_half = [&](int img, int h) {
#pragma unroll
    for (int i = 0; i < NDYSW; ++i) {
      const int k = wv * NDYSW + i;
      if (k < NDYS) {
        const int pln = k / (NDYS / 2), kk = k - pln * (NDYS / 2);
        const int r = 8 * kk + (lane >> 3), pc = lane & 7;
        const int s = ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
        const int c = pc ^ (s << 1);
        const int gr = DYR * h + r;
        const uint8_t* src = d.zero16;
        if (gr < 400) src = reinterpret_cast<const uint8_t*>((pln ? d.dy_lo : d.dy) + ((int64_t)img * 400 + gr) * 64 + c * 8);
        const uint32_t off =
            (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(Dy + pln * DYR * 128 + kk * 1024);
        dma16(src, __builtin_amdgcn_readfirstlane(off));
      }
    }
  };
  // frame-DMA instructions this wave issues per image (vmcnt accounting of SPLIT)
  const int nfr_w = NDMA > wv * NDW ? min(NDW, NDMA - wv * NDW) : 0;

  f32x4 acc[2][C], accb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    accb[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < C; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u));

  // k-steps [ks0, ks1) of the image, dY rows from plane `DyH` (row 32 ks - rbase)
  auto compute_steps = [&](int ks0, int ks1, int rbase) {
#pragma unroll 1
    for (int ks = ks0; ks < ks1; ++ks) {
      const int p0 = min(32 * ks + 8 * g + q, 399), p1 = min(32 * ks + 8 * g + q + 4, 399);
      const int oh0 = p0 / 20, oh1 = p1 / 20;
      const int b0 = ((oh0 * 21 + p0 - 20 * oh0) << 4), b1 = ((oh1 * 21 + p1 - 20 * oh1) << 4);
      const int lk = ks - rbase / 32;
      bf16x8 a[2], al[2], b[C];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = tr_frag8(Dy, lk, 16 * (2 * wc + i), lane);
        if (SPLIT) al[i] = tr_frag8(Dy + DYR * 128, lk, 16 * (2 * wc + i), lane);
      }
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const lds_s16x4* pa = (const lds_s16x4*)(Pl + b0 + xoff[j]);
        const lds_s16x4* pb = (const lds_s16x4*)(Pl + b1 + xoff[j]);
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(pa));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(pb));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        b[j] = __builtin_bit_cast(bf16x8, (s16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
      }
      // D[k][co] (swapped operands): lane holds k 16 j' + 4 g + {0..3} of co 16 i' + (lane & 15)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < C; ++j) {
          if (SPLIT) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], al[i], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
        }
      if (wk == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (SPLIT) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, al[i], accb[i], 0, 0, 0);
          accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, a[i], accb[i], 0, 0, 0);
        }
      }
    }
  };
  auto convert_frames = [&]() {
    for (int j = tid; j < NCHUNK; j += C1W_THREADS) {
      const uint4 v = *reinterpret_cast<const uint4*>(Sg + j * 16);
      const int c = j / 441, blk = j - c * 441;
      *reinterpret_cast<uint4*>(Pl + (2 * c) * C1W_PLANE + blk * 16) = u8x8_to_bf16x8(v.x, v.y);
      *reinterpret_cast<uint4*>(Pl + (2 * c + 1) * C1W_PLANE + blk * 16) = u8x8_to_bf16x8(v.z, v.w);
    }
  };

  const int G = gridDim.x;
  __shared__ int q_item;
  int wq_seq = 0;
  if (tid == 0) reinterpret_cast<volatile int*>(&q_item)[0] = wq_next(d.wq, wq_seq, G);
  __syncthreads();
  int item = __builtin_amdgcn_readfirstlane(reinterpret_cast<volatile int*>(&q_item)[0]);
  while (item < G) {
    int img = item;
    if (img < d.N) issue_frames(img);
    if constexpr (SPLIT) {
      for (; img < d.N; img += G) {
        issue_dy_half(img, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // frames(img) + dY half 0 of this wave
        __builtin_amdgcn_s_barrier();
        convert_frames();
        __syncthreads();
        compute_steps(0, DYR / 32, 0);
        __syncthreads();                                    // dY planes and staging free
        issue_dy_half(img, 1);
        if (img + G < d.N) issue_frames(img + G);           // lands under half 1
        vmcnt_le(img + G < d.N ? nfr_w : 0);                // dY half 1 of this wave
        __builtin_amdgcn_s_barrier();
        compute_steps(DYR / 32, 13, DYR);
        __syncthreads();                                    // planes and dY may be overwritten
      }
    }
    for (; !SPLIT && img < d.N; img += G) {
      issue_dy(img);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // frames(img) + dY(img) of this wave
      __builtin_amdgcn_s_barrier();
      convert_frames();
      __syncthreads();
      if (img + G < d.N) issue_frames(img + G);            // staging is free again
      compute_steps(0, DYR / 32, 0);
      __syncthreads();   // planes and dY image may be overwritten
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the next item (static order: none -- item + G), fetched before this one's stores
    if (tid == 0) reinterpret_cast<volatile int*>(&q_item)[0] = wq_next(d.wq, wq_seq, G);

    // ---- this item's partial: slab[item][co][k] (s2d K order), float4 along k
    float* slab = d.slab + (int64_t)item * 64 * K;
    const int pl = lane & 15;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const int co = 16 * (2 * wc + i) + pl;
        *reinterpret_cast<f32x4*>(slab + (int64_t)co * K + 16 * (C * wk + j) + 4 * g) = acc[i][j];
        acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    if (wk == 0 && g == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i) d.bias_slab[(int64_t)item * 64 + 16 * (2 * wc + i) + pl] = accb[i][0];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) accb[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    item = __builtin_amdgcn_readfirstlane(reinterpret_cast<volatile int*>(&q_item)[0]);
    __syncthreads();   // every wave has read q_item before thread 0 overwrites it
  }
}

APEX_EXPORT int apex_conv1_wgrad_img(Conv1WgDesc d, int grid, hipStream_t st) {
  if (d.N < 1) return 0;
  if (grid <= 0) return (int)hipErrorInvalidValue;
  if (d.dy_lo != nullptr) {
    switch (d.C) {
      case 1: conv1_wgrad_img_kernel<1, true><<<grid, C1W_THREADS, 0, st>>>(d); break;
      case 2: conv1_wgrad_img_kernel<2, true><<<grid, C1W_THREADS, 0, st>>>(d); break;
      case 4: conv1_wgrad_img_kernel<4, true><<<grid, C1W_THREADS, 0, st>>>(d); break;
      default: return (int)hipErrorInvalidValue;
    }
  } else {
    switch (d.C) {
      case 1: conv1_wgrad_img_kernel<1, false><<<grid, C1W_THREADS, 0, st>>>(d); break;
      case 2: conv1_wgrad_img_kernel<2, false><<<grid, C1W_THREADS, 0, st>>>(d); break;
      case 4: conv1_wgrad_img_kernel<4, false><<<grid, C1W_THREADS, 0, st>>>(d); break;
      default: return (int)hipErrorInvalidValue;
    }
  }
  APEX_CHECK_LAUNCH();
}

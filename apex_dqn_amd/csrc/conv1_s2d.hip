// conv1 (8x8 stride 4, C stacked uint8 frames -> 64) on a space-to-depth frame ring.
//
// Frames live in the replay ring as s2d(4): frame[84][84] -> [21][21][4][4]
// (each 4x4 pixel block = 16 contiguous bytes).  The 8x8/s4 convolution is then
// a 2x2/s1 convolution whose implicit-GEMM A row for output pixel (oh,ow) is
// 4 taps x C frames x one 16-byte block: every A element arrives through a
// 16-byte LDS-DMA (global_load_lds_dwordx4) straight from the replay ring --
// the frame stack is never materialised in HBM, and no VGPR staging or
// ds_write is spent on it.  K order: k = ((tap*C + c)*16 + r4*4 + c4),
// tap = 2a+b: the kernel gathers that permutation of OIHW w1 into LDS itself.
//
// Forward: persistent workgroups (one per CU) keep both weight sets (online and
// target network, 2 x 64 x 64C bf16) resident in LDS and stream 128-row A tiles
// (uint8, double-buffered, DMA of tile i+1 in flight under the MFMAs of tile i);
// uint8 -> bf16 conversion happens at fragment-read time (values 0..255 are
// exact in bf16; the 1/255 input scale is applied in the epilogue).
#include "mfma_common.h"

#define S2D_FRAME 7056

struct Conv1S2DDesc {
  const uint8_t* ring;        // s2d frame ring [F][21][21][16]
  const int32_t* slots;       // [N][C]
  const bf16_t* w;            // [64][C][8][8] OIHW (online)
  const bf16_t* w2;           // second set (target), or null
  const float* bias;
  const float* bias2;
  bf16_t* y;                  // [N][20][20][64]
  const uint8_t* zero16;      // 16 zero bytes (padding rows)
  uint8_t* scratch;           // >= 1 KB dummy store target (rows past the end)
  int N, C, m_switch;
  float in_scale;
};

// ---------------------------------------------------------------------------
// Image-resident forward.  A persistent workgroup (8 waves, one per CU)
// walks whole images.  Per image:
//   * its C uint8 frames (C x 7056 contiguous bytes in the ring) arrive in an
//     LDS staging area by LDS-DMA, issued while the previous image computes;
//   * every 16-byte s2d block is converted to bf16 ONCE, into 2C planes
//     (frame c, half h) of 441 x 16 B (plane stride 7168 = 28 x 256 B, so the
//     two halves read by one ds_read_b128 lane group never share banks);
//   * the A fragment of (pixel p, tap (a,b), frame c, half h) is then a single
//     ds_read_b128 at base(p) + lane-constant offset -- no conversion or address
//     VALU per MFMA; the B fragments (weights, 2C x 4 per lane) live in VGPRs;
//   * 25 row tiles of 16 pixels; wave pair (2p, 2p+1) takes tiles p, p+4, ...,
//     each wave one half of the 64 output channels (half the B fragments per
//     wave, so two waves fit per SIMD); the epilogue stages each tile through
//     a wave-private LDS tile for 64-B row-half stores.
// The 1/255 scale, bias and ReLU are applied in the epilogue; online/target
// weights switch per image (m_switch is a multiple of 400 rows).
#define C1_PLANE 7168
#define C1_TILES 25
#define C1_THREADS 512

template <int C>
__global__ void __launch_bounds__(C1_THREADS, 1) conv1_s2d_fwd_kernel(Conv1S2DDesc d) {
  constexpr int NW = C1_THREADS / 64;    // 8 waves: 2 per SIMD hide each other's epilogue / LDS latency
  constexpr int IMG = 2 * C * C1_PLANE;
  constexpr int NCHUNK = C * 441;        // 16-B s2d blocks per image
  constexpr int NDMA = (NCHUNK + 63) / 64;
  constexpr int NDW = (NDMA + NW - 1) / NW;   // DMA wave-instructions per wave
  constexpr int STG = NDMA * 1024;       // u8 staging (lane-linear DMA pieces)
  __shared__ __attribute__((aligned(16))) uint8_t smem[IMG + STG + NW * 1024];
  uint8_t* Pl = smem;
  uint8_t* Sg = Pl + IMG;
  uint8_t* Ep = Sg + STG;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, pl = lane & 15;
  const bool two = d.w2 != nullptr;
  const int img_switch = two ? d.m_switch / 400 : 1 << 30;

  // wave pair (2 p, 2 p + 1) shares row tiles p, p+4, ...; wave w owns channels
  // [32 (w & 1), 32 (w & 1) + 32) = n-tiles nt0, nt0 + 1: half the B fragments per wave
  const int nt0 = 2 * (wv & 1);
  float4 bv[2];                          // bias of the current weight set (channels 16 (nt0+j) + 4 g ..)
  // lane-constant A offsets per k-step s: block q = 2s + (g >> 1) = (tap, frame c), half g & 1
  int aoff[2 * C];
#pragma unroll
  for (int s = 0; s < 2 * C; ++s) {
    const int q = 2 * s + (g >> 1), tap = q / C, c = q - tap * C;
    aoff[s] = (2 * c + (g & 1)) * C1_PLANE + (((tap >> 1) * 21 + (tap & 1)) << 4);
  }
  // ---- B fragments of the current weight set in VGPRs (swapped-operand MFMA: lane
  // (g, pl) supplies output channel n = 16 nt + pl, s2d K 32 s + 8 g .. +7), gathered
  // from OIHW w1: 16-B K chunk c = 4 s + g is (tap, frame) block q = c >> 1, kernel
  // rows r4 = 2 (c & 1) + {0, 1}, each 4 contiguous kw taps (8 B)
  bf16x8 bfr[2 * C][2];
  int cur_set = -1;
  auto load_b = [&](int set) {
    const bf16_t* W = set ? d.w2 : d.w;
    const float* bsrc = set ? d.bias2 : d.bias;
#pragma unroll
    for (int j = 0; j < 2; ++j) bv[j] = *reinterpret_cast<const float4*>(bsrc + 16 * (nt0 + j) + 4 * g);
#pragma unroll
    for (int s = 0; s < 2 * C; ++s)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int n = 16 * (nt0 + nt) + pl, c = 4 * s + g;
        const int q = c >> 1, tap = q / C, ch = q - tap * C;
        const int kh = 4 * (tap >> 1) + 2 * (c & 1), kw = 4 * (tap & 1);
        const bf16_t* p = W + ((n * C + ch) * 8 + kh) * 8 + kw;
        const uint2 lo = *reinterpret_cast<const uint2*>(p);
        const uint2 hi = *reinterpret_cast<const uint2*>(p + 8);
        bfr[s][nt] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
    cur_set = set;
  };

  // ---- LDS-DMA of one image's frames: chunk j = frame j / 441, block j % 441
  auto issue_dma = [&](int img) {
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
          src = d.ring + (int64_t)slot * S2D_FRAME + (blk << 4);
        }
        const uint32_t off = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(Sg + k * 1024);
        dma16(src, __builtin_amdgcn_readfirstlane(off));
      }
    }
  };

  const int G = gridDim.x;
  int img = blockIdx.x;
  if (img < d.N) {
    load_b(img >= img_switch ? 1 : 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    issue_dma(img);
  }
  uint8_t* E = Ep + wv * 1024;
  for (int it = 0; img < d.N; img += G, ++it) {
    // this wave's DMA(img) landed: younger VMEM ops are the previous image's
    // epilogue stores (1 per row tile: 7 tiles for waves 0-1, 6 for the others)
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (wv < 2) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- u8 staging -> bf16 planes (each block converted once)
    for (int j = tid; j < NCHUNK; j += C1_THREADS) {
      const uint4 v = *reinterpret_cast<const uint4*>(Sg + j * 16);
      const int c = j / 441, blk = j - c * 441;
      const uint4 lo = make_uint4(bf16pair_from_f32(ubyte(v.x, 0), ubyte(v.x, 1)), bf16pair_from_f32(ubyte(v.x, 2), ubyte(v.x, 3)),
                                  bf16pair_from_f32(ubyte(v.y, 0), ubyte(v.y, 1)), bf16pair_from_f32(ubyte(v.y, 2), ubyte(v.y, 3)));
      const uint4 hi = make_uint4(bf16pair_from_f32(ubyte(v.z, 0), ubyte(v.z, 1)), bf16pair_from_f32(ubyte(v.z, 2), ubyte(v.z, 3)),
                                  bf16pair_from_f32(ubyte(v.w, 0), ubyte(v.w, 1)), bf16pair_from_f32(ubyte(v.w, 2), ubyte(v.w, 3)));
      *reinterpret_cast<uint4*>(Pl + (2 * c) * C1_PLANE + blk * 16) = lo;
      *reinterpret_cast<uint4*>(Pl + (2 * c + 1) * C1_PLANE + blk * 16) = hi;
    }
    __syncthreads();
    // staging is free: prefetch the next image under this one's MFMAs
    if (img + G < d.N) issue_dma(img + G);
    const int set = img >= img_switch ? 1 : 0;
    if (set != cur_set) {
      // weight-set switch (once per block): reload, then restore the vmcnt invariant
      load_b(set);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    for (int t = wv >> 1; t < C1_TILES; t += NW / 2) {
      const int p = 16 * t + pl;
      const int oh = p / 20, ow = p - 20 * oh;
      const uint8_t* A = Pl + ((oh * 21 + ow) << 4);
      f32x4 acc[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2 * C; ++s) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + aoff[s]);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[s][nt], a, acc[nt], 0, 0, 0);
      }
      // epilogue: lane holds channels 16 (nt0+nt) + 4 g .. +3 of pixel pl -> wave tile
      // (16 rows x 64 B: 4 chunks, chunk c of row r at c ^ ((r >> 1) & 3)) -> one
      // 16-B store per lane (rows of the output are 128 B: this wave writes one half)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const f32x4 v = acc[nt];
        const uint2 o = make_uint2(relu2(cvt_pk_bf16(v[0] * d.in_scale + bv[nt].x, v[1] * d.in_scale + bv[nt].y)),
                                   relu2(cvt_pk_bf16(v[2] * d.in_scale + bv[nt].z, v[3] * d.in_scale + bv[nt].w)));
        const int byte = 2 * (16 * nt + 4 * g);
        *reinterpret_cast<uint2*>(E + pl * 64 + ((((byte >> 4) ^ ((pl >> 1) & 3))) << 4) + (byte & 15)) = o;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      {
        const int row = lane >> 2, ch = lane & 3;
        const uint4 v = *reinterpret_cast<const uint4*>(E + row * 64 + ((ch ^ ((row >> 1) & 3)) << 4));
        *reinterpret_cast<uint4*>(d.y + ((int64_t)img * 400 + 16 * t + row) * 64 + 32 * (wv & 1) + ch * 8) = v;
      }
    }
    __syncthreads();   // planes may be overwritten by the next conversion
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// w1 [64][C][8][8] (OIHW) -> s2d K order [64][(tap*C + c)*16 + r4*4 + c4], tap = 2a + b,
// kh = 4a + r4, kw = 4b + c4.  Optionally a second set (target network).
__global__ void s2d_pack_w1_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ ws, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = 64 * C;
  if (i >= 64 * K) return;
  const int n = i / K, k = i - n * K;
  const int q = k >> 4, r4 = (k >> 2) & 3, c4 = k & 3;
  const int tap = q / C, c = q - tap * C;
  const int kh = 4 * (tap >> 1) + r4, kw = 4 * (tap & 1) + c4;
  ws[i] = w[((n * C + c) * 8 + kh) * 8 + kw];
}

// inverse for gradients: dW in s2d K order (fp32) -> OIHW (fp32), optional scale
__global__ void s2d_unpack_w1_grad_kernel(const float* __restrict__ gs, float* __restrict__ g, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = 64 * C;
  if (i >= 64 * K) return;
  const int n = i / K, k = i - n * K;
  const int q = k >> 4, r4 = (k >> 2) & 3, c4 = k & 3;
  const int tap = q / C, c = q - tap * C;
  const int kh = 4 * (tap >> 1) + r4, kw = 4 * (tap & 1) + c4;
  g[((n * C + c) * 8 + kh) * 8 + kw] = gs[i];
}

// frames [n][84][84] -> s2d [n][21][21][4][4]  (one thread per 16-byte block)
__global__ void s2d_frames_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int64_t n,
                                  int64_t F, int64_t start) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // block index
  if (i >= n * 441) return;
  const int64_t f = i / 441;
  const int blk = (int)(i - f * 441);
  const int R = blk / 21, Q = blk - R * 21;
  const uint8_t* s = src + f * 7056 + (4 * R) * 84 + 4 * Q;
  uint32_t w[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) w[r] = *reinterpret_cast<const uint32_t*>(s + r * 84);
  uint8_t* o = dst + ((start + f) % F) * 7056 + blk * 16;
  *reinterpret_cast<uint4*>(o) = make_uint4(w[0], w[1], w[2], w[3]);
}

APEX_EXPORT int apex_conv1_s2d_fwd(Conv1S2DDesc d, int grid, hipStream_t st) {
  if (d.w2 != nullptr && (d.m_switch % 400)) return (int)hipErrorInvalidValue;
  if (d.N < 1) return 0;
  if (grid <= 0 || grid > d.N) grid = d.N < 256 ? d.N : 256;
  switch (d.C) {
    case 1: conv1_s2d_fwd_kernel<1><<<grid, C1_THREADS, 0, st>>>(d); break;
    case 2: conv1_s2d_fwd_kernel<2><<<grid, C1_THREADS, 0, st>>>(d); break;
    case 4: conv1_s2d_fwd_kernel<4><<<grid, C1_THREADS, 0, st>>>(d); break;
    default: return (int)hipErrorInvalidValue;
  }
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_s2d_pack_w1(const bf16_t* w, bf16_t* ws, int C, hipStream_t st) {
  const int n = 64 * 64 * C;
  s2d_pack_w1_kernel<<<(n + 255) / 256, 256, 0, st>>>(w, ws, C);
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_s2d_unpack_w1_grad(const float* gs, float* g, int C, hipStream_t st) {
  const int n = 64 * 64 * C;
  s2d_unpack_w1_grad_kernel<<<(n + 255) / 256, 256, 0, st>>>(gs, g, C);
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_s2d_frames(const uint8_t* src, uint8_t* dst, int64_t n, int64_t F, int64_t start,
                                hipStream_t st) {
  if (n <= 0) return 0;
  const int64_t t = n * 441;
  s2d_frames_kernel<<<(int)((t + 255) / 256), 256, 0, st>>>(src, dst, n, F, start);
  APEX_CHECK_LAUNCH();
}

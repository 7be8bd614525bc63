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
#include "apex_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define S2D_ROWS 128
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

// 8 uint8 (two dwords) -> 8 bf16: v_cvt_f32_ubyte{0..3} then one v_perm per pair
// picks the high halves of two exact f32 integers (their low halves are zero).
__device__ __forceinline__ uint32_t bf16pair_from_f32(float lo, float hi) {
  return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);
}

// (float)(byte k of v): hipcc lowers this pattern to one v_cvt_f32_ubyte{k}
__device__ __forceinline__ float ubyte(uint32_t v, int k) { return (float)((v >> (8 * k)) & 0xffu); }

__device__ __forceinline__ bf16x8 u8x8_frag(uint2 v) {
  const uint4 r = make_uint4(bf16pair_from_f32(ubyte(v.x, 0), ubyte(v.x, 1)), bf16pair_from_f32(ubyte(v.x, 2), ubyte(v.x, 3)),
                             bf16pair_from_f32(ubyte(v.y, 0), ubyte(v.y, 1)), bf16pair_from_f32(ubyte(v.y, 2), ubyte(v.y, 3)));
  return __builtin_bit_cast(bf16x8, r);
}

// ReLU on two packed bf16 (sign bits spread over their halves, then cleared)
__device__ __forceinline__ uint32_t relu2(uint32_t v) {
  const uint32_t neg = ((v & 0x80008000u) >> 15) * 0xffffu;
  return v & ~neg;
}

#define S2D_STAGES 3

// 16-byte LDS-DMA issued from inline asm: hipcc does not track it, so it emits no
// conservative vmcnt(0) before later ds_reads; completion is counted by hand with
// explicit s_waitcnt vmcnt(N) + s_barrier (M0 is written inside the statement).
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_off) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_off)
               : "memory");
}

// Scalar (SMEM) load of the C frame slots of one image: counted by lgkmcnt, so it
// never forces a vmcnt drain of the LDS-DMA in flight.  `p` must be wave-uniform.
template <int C>
__device__ __forceinline__ void sload_slots(const int32_t* p, int (&out)[4]) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int32_t* q = (const int32_t*)(((uint64_t)hi << 32) | lo);
  if constexpr (C == 4) {
    int __attribute__((ext_vector_type(4))) v;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(q) : "memory");
    out[0] = v[0]; out[1] = v[1]; out[2] = v[2]; out[3] = v[3];
  } else if constexpr (C == 2) {
    int __attribute__((ext_vector_type(2))) v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(q) : "memory");
    out[0] = v[0]; out[1] = v[1]; out[2] = 0; out[3] = 0;
  } else {
    int v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(q) : "memory");
    out[0] = v; out[1] = 0; out[2] = 0; out[3] = 0;
  }
}

typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){lo, hi}, bf16x2v));
}

template <int C>
__global__ void __launch_bounds__(256, 1) conv1_s2d_fwd_kernel(Conv1S2DDesc d) {
  constexpr int NCH = 4 * C;             // 16-byte chunks (tap, frame) per A row
  constexpr int K = 64 * C;
  constexpr int WROW = 2 * K;            // bytes per weight row (bf16)
  constexpr int WCH = WROW / 16;         // 16-byte chunks per weight row
  constexpr int PLANE = S2D_ROWS * 16;   // one chunk for all 128 rows
  constexpr int ATILE = NCH * PLANE;
  constexpr int WSET = 64 * WROW;
  constexpr int NDMA = 2 * NCH / 4;      // DMA wave-instructions per wave per tile (64 rows each)
  // A tile is CHUNK-MAJOR: plane j holds chunk j of all 128 rows.  One DMA
  // wave-instruction = one (tap, frame) chunk of 64 consecutive output pixels,
  // which are consecutive 16-B s2d blocks of one frame row: contiguous reads.
  // (A row-major image would gather 64 scattered 16-B pieces per instruction.)
  constexpr bool EPI_IN_A = NCH >= 8;    // wave's rows in 8 planes = 8 x 512 B = its 4 KB epilogue image
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * WSET + S2D_STAGES * ATILE + (EPI_IN_A ? 0 : 4 * 4096)];
  uint8_t* Wl = smem;
  uint8_t* Al = smem + 2 * WSET;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int M = d.N * 400;
  const int ntiles = (M + S2D_ROWS - 1) / S2D_ROWS;
  const bool two = d.w2 != nullptr;

  // ---- weights (both sets) -> LDS, chunk c of row n stored at c ^ (n & mask).
  // Gathered straight from OIHW w1: s2d chunk c = (tap, frame) block q = c >> 1, kernel
  // rows r4 = 2(c & 1) + {0, 1}; each is 4 contiguous kw taps (8 B) of the OIHW tensor.
  constexpr int WMASK = WCH >= 16 ? 15 : WCH - 1;
  for (int s = 0; s < (two ? 2 : 1); ++s) {
    const bf16_t* src = s ? d.w2 : d.w;
    for (int i = tid; i < 64 * WCH; i += 256) {
      const int n = i / WCH, c = i - n * WCH;
      const int q = c >> 1, tap = q / C, ch = q - tap * C;
      const int kh = 4 * (tap >> 1) + 2 * (c & 1), kw = 4 * (tap & 1);
      const bf16_t* p = src + ((n * C + ch) * 8 + kh) * 8 + kw;
      const uint2 lo = *reinterpret_cast<const uint2*>(p);
      const uint2 hi = *reinterpret_cast<const uint2*>(p + 8);
      *reinterpret_cast<uint4*>(Wl + s * WSET + n * WROW + ((c ^ (n & WMASK)) << 4)) =
          make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
  }
  // lane (g, p) owns output channels 16nt + 4g + {0..3} (swapped-operand MFMA below)
  float4 bias4[2][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    bias4[0][nt] = *reinterpret_cast<const float4*>(d.bias + 16 * nt + 4 * (lane >> 4));
    bias4[1][nt] = two ? *reinterpret_cast<const float4*>(d.bias2 + 16 * nt + 4 * (lane >> 4))
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- A-tile DMA: wave wv issues instructions q = NDMA*wv .. +NDMA-1, each one
  // (chunk j = q >> 1, half = q & 1) for rows 64*half + lane.  A tile spans at most
  // two images; their C slots come from SCALAR loads (lgkmcnt, not vmcnt).
  auto issue_dma = [&](int tile, int buf) {
    const int img0 = __builtin_amdgcn_readfirstlane((tile * S2D_ROWS) / 400);
    int s0[4], s1[4];
    sload_slots<C>(d.slots + img0 * C, s0);
    if (img0 + 1 < d.N) sload_slots<C>(d.slots + (img0 + 1) * C, s1);
    else { s1[0] = s0[0]; s1[1] = s0[1]; s1[2] = s0[2]; s1[3] = s0[3]; }
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int q = NDMA * wv + i;
      const int j = q >> 1, half = q & 1;
      const int tap = j / C, c = j - tap * C;
      const int r = 64 * half + lane;
      const int m = tile * S2D_ROWS + r;
      const uint8_t* src = d.zero16;
      if (m < M) {
        const int img = m / 400;
        const int rem = m - img * 400;
        const int oh = rem / 20, ow = rem - oh * 20;
        int slot = s0[0];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc)
          if (cc == c) slot = (img == img0) ? s0[cc] : s1[cc];
        src = d.ring + (int64_t)slot * S2D_FRAME + (((oh + (tap >> 1)) * 21 + ow + (tap & 1)) << 4);
      }
      uint8_t* dst = Al + buf * ATILE + j * PLANE + half * 64 * 16;  // wave-uniform base
      const uint32_t off = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)dst;
      dma16(src, __builtin_amdgcn_readfirstlane(off));
    }
  };

  const int G = gridDim.x;
  // XCD-contiguous tile order: the ~3 tiles of one frame stack run on one L2
  int tile = xcd_swizzle(blockIdx.x, G);
  if (tile < ntiles) issue_dma(tile, 0);
  if (tile + G < ntiles) issue_dma(tile + G, 1);
  int buf = 0;
  for (int it = 0; tile < ntiles; tile += G, ++it) {
    // Wait until this tile's DMA group has landed.  Issue order per iteration is
    // [DMA(tile+2G)][4 epilogue stores], so the VMEM ops younger than DMA(tile)
    // are: only DMA(tile+G) at it=0, +4 stores at it=1, +8 after.
    if (tile + G >= ntiles) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (it == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
    else if (it == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA + 4) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA + 8) : "memory");
    __builtin_amdgcn_s_barrier();
    // stage (buf+2)%3 was consumed two iterations ago by every wave: refill it
    const int far = tile + 2 * G;
    if (far < ntiles) issue_dma(far, buf == 0 ? 2 : buf - 1);
    const bool second = two && tile * S2D_ROWS >= d.m_switch;
    const uint8_t* W = Wl + (second ? WSET : 0);
    uint8_t* A = Al + buf * ATILE;
    f32x4 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int g = lane >> 4;
#pragma unroll
    for (int s = 0; s < 2 * C; ++s) {
      const int j = 2 * s + (g >> 1), h = g & 1;
      bf16x8 af[2], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int r = 32 * wv + 16 * mt + (lane & 15);
        const uint2 v = *reinterpret_cast<const uint2*>(A + j * PLANE + r * 16 + h * 8);
        af[mt] = u8x8_frag(v);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int n = 16 * nt + (lane & 15);
        const int c = 4 * s + g;
        bfr[nt] = *reinterpret_cast<const bf16x8*>(W + n * WROW + ((c ^ (n & WMASK)) << 4));
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nt], af[mt], acc[mt][nt], 0, 0, 0);
    }
    // ---- epilogue: the wave's 32x64 bf16 output image (rows rho = 0..31, 128 B each)
    // lives in its own consumed A rows: piece rho/4 = plane rho/4, rows [32wv, 32wv+32).
    // 16-B chunk c of row rho sits at c ^ ((rho >> 1) & 7) (conflict-free 8-B writes).
    auto eaddr = [&](int rho) -> uint8_t* {
      return EPI_IN_A ? A + (rho >> 2) * PLANE + 32 * wv * 16 + (rho & 3) * 128
                      : Al + S2D_STAGES * ATILE + wv * 4096 + rho * 128;
    };
    auto eswz = [&](int rho, int byte) -> int { return (((byte >> 4) ^ ((rho >> 1) & 7)) << 4) + (byte & 15); };
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const float4 bv = second ? bias4[1][nt] : bias4[0][nt];
      const int cb = 2 * (16 * nt + 4 * (lane >> 4));
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int row = 16 * mt + (lane & 15);
        const f32x4 a = acc[mt][nt];
        const uint2 v = make_uint2(cvt_pk_bf16(a[0] * d.in_scale + bv.x, a[1] * d.in_scale + bv.y),
                                   cvt_pk_bf16(a[2] * d.in_scale + bv.z, a[3] * d.in_scale + bv.w));
        *reinterpret_cast<uint2*>(eaddr(row) + eswz(row, cb)) = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = 8 * p + (lane >> 3), ch = lane & 7;
      const int m = tile * S2D_ROWS + 32 * wv + row;
      uint4 v = *reinterpret_cast<const uint4*>(eaddr(row) + eswz(row, ch * 16));
      v = make_uint4(relu2(v.x), relu2(v.y), relu2(v.z), relu2(v.w));
      // out-of-range rows store into a dummy (keeps the per-iteration store count fixed)
      bf16_t* dst = (m < M) ? d.y + (int64_t)m * 64 + ch * 8 : (bf16_t*)d.scratch + lane * 8;
      *reinterpret_cast<uint4*>(dst) = v;
    }
    buf = (buf == S2D_STAGES - 1) ? 0 : buf + 1;
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
  if (d.w2 != nullptr && (d.m_switch % S2D_ROWS)) return (int)hipErrorInvalidValue;
  const int M = d.N * 400;
  const int ntiles = (M + S2D_ROWS - 1) / S2D_ROWS;
  if (grid <= 0 || grid > ntiles) grid = ntiles < 256 ? ntiles : 256;
  switch (d.C) {
    case 1: conv1_s2d_fwd_kernel<1><<<grid, 256, 0, st>>>(d); break;
    case 2: conv1_s2d_fwd_kernel<2><<<grid, 256, 0, st>>>(d); break;
    case 4: conv1_s2d_fwd_kernel<4><<<grid, 256, 0, st>>>(d); break;
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

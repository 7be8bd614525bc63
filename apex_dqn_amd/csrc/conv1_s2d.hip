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
#include "conv2_wfrag.h"

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
  uint64_t* probe;            // optional phase timestamps (blocks < PROBE_BLOCKS), see mfma_common.h
  // fp32-accurate ("split") mode when y_lo is set: the fp32 master weights (OIHW)
  // are read instead of w / w2 and the output leaves as hi / lo bf16 planes
  const float* w32;
  const float* w2_32;
  bf16_t* y_lo;
  // side job: pack the split conv2 forward's weights for this step (csrc/conv2_wfrag.h)
  // at the start of the workgroups -- behind their first frame DMAs' latency instead of
  // a launch of its own (~5 us in the step)
  C2fPack c2f;
};

// ---------------------------------------------------------------------------
// Image-resident forward.  A persistent workgroup (8 waves, one per CU)
// walks whole images.  Per image:
//   * its C uint8 frames (C x 7056 contiguous bytes in the ring) arrive in an
//     LDS staging area by LDS-DMA;
//   * every 16-byte s2d block is converted ONCE into 2C planes (frame c, half h)
//     of 441 x 16 B (plane stride 7168 = 28 x 256 B) as f16 (1024 + x): one
//     v_perm_b32 per two pixels (u8x8_to_f16off), exact; the offset adds
//     1024 * sum_k w[n][k] to output channel n, folded into the epilogue bias;
//   * the A fragment of (pixel p, tap (a,b), frame c, half h) is then a single
//     ds_read_b128 at base(p) + lane-constant offset; the B fragments (weights
//     converted to f16, 2C x 2 per lane) live in VGPRs; v_mfma_f32_16x16x32_f16;
//   * 25 row tiles of 16 pixels; wave pair (2p, 2p+1) takes tiles p, p+4, ...,
//     each wave one half of the 64 output channels (two waves fit per SIMD).
// Pipelining (tuned with the PROBE phase stamps, scripts/probe_kernels.py):
//   * planes are double-buffered: image i+1 is converted while image i computes;
//   * each wave converts exactly the staging chunks its own LDS-DMA brought in,
//     so the DMA -> convert hand-off is a per-wave vmcnt wait, no barrier, and
//     no wait ever covers the epilogue stores (store acks cost microseconds);
//   * waves 0-3 convert first and then compute, waves 4-7 compute first: every
//     SIMD overlaps one wave's conversion with the other's MFMAs; the staging
//     chunks are dealt so that the two waves with 7 tiles convert fewer chunks;
//   * the epilogue is packed fp32 FMA (scale, bias), cvt_pk_bf16 and a packed
//     int16 max (ReLU), stored straight from registers (two 8-byte stores).
//   * weight sets are fetched with contiguous 16-B loads one image ahead, then
//     installed through a swizzled LDS copy (a conflict-free fragment gather).
// Online/target weights switch per image (m_switch is a multiple of 400 rows;
// strided images make it at most one switch per block).
// SPLIT (fp32-accurate): the pixels are exact in f16, the fp32 weights become
// w = hi + lo * 2^-12 with hi = f16(w) and lo = f16((w - hi) * 2^12) (22
// significant bits; the 2^12 keeps lo out of the f16 subnormals), gathered in two
// install rounds; every fragment takes two MFMAs into two accumulators, combined
// in fp32 in the epilogue, which writes the result as hi / lo bf16 planes.
#define C1_PLANE 7168
#define C1_TILES 25
#define C1_THREADS 512
#define C1_MAXIMG 256   // images per workgroup (slot table in LDS)

// staging instruction k (1 KB, 64 lanes x 16 B) belongs to the wave at position
// k % 8 of the order 2,3,4,5,6,7,0,1: waves 0-1 (7 tiles) take the fewest
__device__ __forceinline__ constexpr int c1_owner_pos(int w) { return (w + 6) & 7; }

// LDS byte offset of the 8-byte piece (chunk q, half h) of the installed OIHW
// weight copy: chunk low bits XOR the output channel, halves swapped on q bit 1,
// so the per-lane fragment gather (16 channels x 4 K-chunks) is conflict-free.
template <int C>
__device__ __forceinline__ int c1_wswz(int q, int h) {
  constexpr int NSH = 3 + (C == 4 ? 2 : (C == 2 ? 1 : 0));   // chunk -> output channel shift
  return (((q & ~15) | ((q ^ (q >> NSH)) & 15)) << 4) + ((h ^ ((q >> 1) & 1)) << 3);
}

#define C1_LO_SCALE 4096.f

template <int C, bool SPLIT>
__global__ void __launch_bounds__(C1_THREADS, 1) conv1_s2d_fwd_kernel(Conv1S2DDesc d) {
  constexpr int NST = SPLIT ? 4 : 2;     // epilogue stores per row tile (vmcnt accounting)
  constexpr int NW = C1_THREADS / 64;
  constexpr int IMG = 2 * C * C1_PLANE;
  constexpr int NCHUNK = C * 441;        // 16-B s2d blocks per image
  constexpr int NDMA = (NCHUNK + 63) / 64;
  constexpr int NDW = (NDMA + NW - 1) / NW;   // max staging instructions per wave
  constexpr int STG = NDMA * 1024;
  static_assert(IMG >= 64 * 64 * C * 2 + 256, "weight install needs one plane buffer");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * IMG + STG];
  __shared__ int32_t slot_tbl[C1_MAXIMG * C];   // this block's frame slots (prologue)
  uint8_t* Sg = smem + 2 * IMG;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (d.c2f.out != nullptr) c2f_pack_range(d.c2f, blockIdx.x * C1_THREADS + tid, gridDim.x * C1_THREADS);
  const int g = lane >> 4, pl = lane & 15;
  const bool two = d.w2 != nullptr;
  const int img_switch = two ? d.m_switch / 400 : 1 << 30;
  const int pos = c1_owner_pos(wv);
  const bool conv_first = wv < 4;        // group A: convert, then compute
  const int ntiles = (wv >> 1) == 0 ? 7 : 6;
  const int nt0 = 2 * (wv & 1);
  const int ndma_w = NDMA > pos ? (NDMA - pos + NW - 1) / NW : 0;   // this wave's DMA instructions / image
  f32x2v bv[2][2];                       // epilogue bias (offset-corrected), channel pairs
  int aoff[2 * C];
#pragma unroll
  for (int s = 0; s < 2 * C; ++s) {
    const int q = 2 * s + (g >> 1), tap = q / C, c = q - tap * C;
    aoff[s] = (2 * c + (g & 1)) * C1_PLANE + (((tap >> 1) * 21 + (tap & 1)) << 4);
  }
  // ---- B fragments of the current weight set in VGPRs (swapped-operand MFMA: lane
  // (g, pl) supplies output channel n = 16 nt + pl, s2d K 32 s + 8 g .. +7), gathered
  // from OIHW w1: 16-B K chunk c = 4 s + g is (tap, frame) block q = c >> 1, kernel
  // rows r4 = 2 (c & 1) + {0, 1}, each 4 contiguous kw taps (8 B).
  f16x8 bfr[2 * C][2], bfl[2 * C][2];
  uint4 wpf[C];
  uint4 wpf32[SPLIT ? 2 * C : 1];        // SPLIT: the 8 fp32 weights of chunk q in two uint4
  float4 bpf = make_float4(0.f, 0.f, 0.f, 0.f);
  int cur_set = -1;
  auto prefetch_w = [&](int set) {
    if constexpr (SPLIT) {
      const uint4* W = reinterpret_cast<const uint4*>(set ? d.w2_32 : d.w32);
#pragma unroll
      for (int j = 0; j < C; ++j) {
        wpf32[2 * j] = W[2 * (tid + C1_THREADS * j)];
        wpf32[2 * j + 1] = W[2 * (tid + C1_THREADS * j) + 1];
      }
    } else {
      const uint4* W = reinterpret_cast<const uint4*>(set ? d.w2 : d.w);
#pragma unroll
      for (int j = 0; j < C; ++j) wpf[j] = W[tid + C1_THREADS * j];
    }
    if (tid < 16) bpf = reinterpret_cast<const float4*>(set ? d.bias2 : d.bias)[tid];
  };
  // SPLIT: f16 pair (hi or scaled lo part) of two fp32 weights, packed
  auto f16pair = [&](uint32_t a, uint32_t b, int round) -> uint32_t {
    const float fa = __uint_as_float(a), fb = __uint_as_float(b);
    const _Float16 ha = (_Float16)fa, hb = (_Float16)fb;
    f16x2v r;
    if (round == 0) {
      r = (f16x2v){ha, hb};
    } else {
      r = (f16x2v){(_Float16)((fa - (float)ha) * C1_LO_SCALE), (_Float16)((fb - (float)hb) * C1_LO_SCALE)};
    }
    return __builtin_bit_cast(uint32_t, r);
  };
  // `younger`: VMEM ops this wave issued after the prefetch that need not finish
  auto install_w = [&](uint8_t* L, int set, int younger) {   // every wave; L: a free plane buffer
    // SPLIT: the fp32 weights are fetched here, not one image ahead (their 8 C
    // prefetch VGPRs would stay live across the loop and spill the 4-frame kernel)
    if (SPLIT) prefetch_w(set);
    vmcnt_le(SPLIT ? 0 : younger);
    float* Lb = reinterpret_cast<float*>(L + 64 * 64 * C * 2);
    float ws[2] = {0.f, 0.f};
#pragma unroll
    for (int round = 0; round < (SPLIT ? 2 : 1); ++round) {
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const int q = tid + C1_THREADS * j;
        uint4 v = wpf[j];
        if constexpr (SPLIT) {
          const uint4 a = wpf32[2 * j], b = wpf32[2 * j + 1];
          v = make_uint4(f16pair(a.x, a.y, round), f16pair(a.z, a.w, round), f16pair(b.x, b.y, round),
                         f16pair(b.z, b.w, round));
        }
        *reinterpret_cast<uint2*>(L + c1_wswz<C>(q, 0)) = make_uint2(v.x, v.y);
        *reinterpret_cast<uint2*>(L + c1_wswz<C>(q, 1)) = make_uint2(v.z, v.w);
      }
      if (round == 0 && tid < 16) reinterpret_cast<float4*>(Lb)[tid] = bpf;
      __syncthreads();
#pragma unroll
      for (int s = 0; s < 2 * C; ++s)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int n = 16 * (nt0 + nt) + pl, c = 4 * s + g;
          const int q = c >> 1, tap = q / C, ch = q - tap * C;
          const int kh = 4 * (tap >> 1) + 2 * (c & 1), kw = 4 * (tap & 1);
          const int p = ((n * C + ch) * 8 + kh) * 8 + kw;     // element offset, multiple of 4
          const uint2 lo = *reinterpret_cast<const uint2*>(L + c1_wswz<C>(p >> 3, (p >> 2) & 1));
          const uint2 hi = *reinterpret_cast<const uint2*>(L + c1_wswz<C>((p >> 3) + 1, (p >> 2) & 1));
          const uint32_t wd[4] = {lo.x, lo.y, hi.x, hi.y};
          f16x8 f;
          if constexpr (SPLIT) {
            // the LDS copy already holds f16 (hi, or lo * 2^12 in round 1)
            f = __builtin_bit_cast(f16x8, make_uint4(wd[0], wd[1], wd[2], wd[3]));
            const float sc = round == 0 ? 1.f : 1.f / C1_LO_SCALE;
#pragma unroll
            for (int i = 0; i < 8; ++i) ws[nt] += (float)f[i] * sc;
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float a0 = __uint_as_float(wd[i] << 16), a1 = __uint_as_float(wd[i] & 0xffff0000u);
              f[2 * i] = (_Float16)a0;
              f[2 * i + 1] = (_Float16)a1;
              ws[nt] += (float)f[2 * i] + (float)f[2 * i + 1];
            }
          }
          if (round == 0) bfr[s][nt] = f;
          else bfl[s][nt] = f;
        }
      if (SPLIT && round == 0) __syncthreads();   // every gather done before round 1 rewrites L
    }
    // channel sums over the 4 K-chunk lanes, then the epilogue's channels 4 g + i
    // fetch theirs: bias' = bias - 1024 * scale * sum_k w16[n][k]
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      float t = ws[nt];
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      float c4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) c4[i] = __shfl(t, 4 * g + i, 64);
      const float4 bb = *reinterpret_cast<const float4*>(Lb + 16 * (nt0 + nt) + 4 * g);
      const float k = 1024.f * d.in_scale;
      bv[nt][0] = (f32x2v){bb.x - k * c4[0], bb.y - k * c4[1]};
      bv[nt][1] = (f32x2v){bb.z - k * c4[2], bb.w - k * c4[3]};
    }
    cur_set = set;
    __syncthreads();   // L is a plane buffer: free it for the next conversion
  };

  // ---- this wave's LDS-DMA share of one image: instructions k = pos + 8 j
  auto issue_dma = [&](int img, int it_img) {
    // slots from the LDS table: a scalar load here would expose its full memory
    // latency (s_waitcnt lgkmcnt(0)) every image (~1400 clocks, PROBE-measured)
    int sl[4] = {0, 0, 0, 0};
#pragma unroll
    for (int cc = 0; cc < C; ++cc) sl[cc] = slot_tbl[it_img * C + cc];
#pragma unroll
    for (int j = 0; j < NDW; ++j) {
      const int k = pos + NW * j;
      if (k < NDMA) {
        const int ch = 64 * k + lane;
        const uint8_t* src = d.zero16;
        if (ch < NCHUNK) {
          const int c = ch / 441, blk = ch - c * 441;
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
  // ---- convert this wave's own staging chunks into planes `P` (u8 -> f16 1024+x)
  auto convert = [&](uint8_t* P) {
#pragma unroll
    for (int j = 0; j < NDW; ++j) {
      const int k = pos + NW * j;
      const int ch = 64 * k + lane;
      if (k < NDMA && ch < NCHUNK) {
        const uint4 v = *reinterpret_cast<const uint4*>(Sg + ch * 16);
        const int c = ch / 441, blk = ch - c * 441;
        *reinterpret_cast<uint4*>(P + (2 * c) * C1_PLANE + blk * 16) = u8x8_to_f16off(v.x, v.y);
        *reinterpret_cast<uint4*>(P + (2 * c + 1) * C1_PLANE + blk * 16) = u8x8_to_f16off(v.z, v.w);
      }
    }
    // staging reads retired before the next DMA may overwrite them
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  // ---- this wave's row tiles of image `img` from planes `P`; 2 stores per tile
  auto compute = [&](const uint8_t* P, int img) {
    for (int t = wv >> 1; t < C1_TILES; t += NW / 2) {
      const int p = 16 * t + pl;
      const int oh = p / 20, ow = p - 20 * oh;
      const uint8_t* A = P + ((oh * 21 + ow) << 4);
      // (SPLIT: the fragments are read per K step -- all 2 C of them up front next to
      // both weight sets would exceed the 256 VGPRs of two waves per SIMD)
      constexpr int NA = SPLIT ? 1 : 2 * C;
      f16x8 a[NA];
      if (!SPLIT) {
#pragma unroll
        for (int s = 0; s < NA; ++s) a[s] = *reinterpret_cast<const f16x8*>(A + aoff[s]);
      }
      f32x4 acc[2], accl[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[nt] = accl[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2 * C; ++s) {
        const f16x8 as = SPLIT ? *reinterpret_cast<const f16x8*>(A + aoff[s]) : a[SPLIT ? 0 : s];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bfr[s][nt], as, acc[nt], 0, 0, 0);
          if (SPLIT) accl[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bfl[s][nt], as, accl[nt], 0, 0, 0);
        }
      }
      // lane holds channels 16 (nt0+nt) + 4 g .. +3 of pixel p: one 8-byte store each
      const int64_t yo = ((int64_t)img * 400 + p) * 64 + 16 * nt0 + 4 * g;
      const f32x2v sc = {d.in_scale, d.in_scale};
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        if constexpr (SPLIT) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[r] = fmaxf((acc[nt][r] + accl[nt][r] * (1.f / C1_LO_SCALE)) * d.in_scale + bv[nt][r >> 1][r & 1], 0.f);
          uint32_t h01, l01, h23, l23;
          split_pk_bf16(v[0], v[1], h01, l01);
          split_pk_bf16(v[2], v[3], h23, l23);
          *reinterpret_cast<uint2*>(d.y + yo + 16 * nt) = make_uint2(h01, h23);
          *reinterpret_cast<uint2*>(d.y_lo + yo + 16 * nt) = make_uint2(l01, l23);
        } else {
          const f32x2v v0 = (f32x2v){acc[nt][0], acc[nt][1]} * sc + bv[nt][0];
          const f32x2v v1 = (f32x2v){acc[nt][2], acc[nt][3]} * sc + bv[nt][1];
          const uint2 o = make_uint2(relu_pk16(cvt_pk_bf16(v0[0], v0[1])), relu_pk16(cvt_pk_bf16(v1[0], v1[1])));
          *reinterpret_cast<uint2*>(d.y + yo + 16 * nt) = o;
        }
      }
    }
  };
  // wait for this wave's DMA(next): younger VMEM ops are the stores of one compute()
  auto wait_dma = [&](bool exact0) {
    if (exact0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (ntiles == 7) {
      if (SPLIT) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
    } else {
      if (SPLIT) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    }
  };

  const int G = gridDim.x;
  int img = blockIdx.x;
  if (img >= d.N) return;
  // this block's frame slots -> LDS (host guarantees ceil(N / G) <= C1_MAXIMG)
  for (int i = tid; i < C1_MAXIMG * C; i += C1_THREADS) {
    const int im = blockIdx.x + (i / C) * G;
    slot_tbl[i] = im < d.N ? d.slots[im * C + (i % C)] : 0;
  }
  __syncthreads();
  // prologue: weights installed (via planes[1]), image 0 converted into planes[0],
  // DMA of image 1 in flight
  if (!SPLIT) prefetch_w(img >= img_switch ? 1 : 0);
  issue_dma(img, 0);
  install_w(smem + IMG, img >= img_switch ? 1 : 0, 0);   // vmcnt(0): DMA(img) landed too
  convert(smem);
  if (img + G < d.N) issue_dma(img + G, 1);
  __syncthreads();
  for (int it = 0; img < d.N; img += G, ++it) {
    PROBE(d.probe, NW, it, 0);
    uint8_t* Pc = smem + (it & 1) * IMG;
    uint8_t* Pn = smem + ((it & 1) ^ 1) * IMG;
    const bool has_next = img + G < d.N;
    const int set = img >= img_switch ? 1 : 0;
    if (set != cur_set) install_w(Pn, set, NST * ntiles + ndma_w);   // prefetched last iteration
    // next image switches sets: fetch them now, hidden under this image's work
    // (extra loads only make the vmcnt waits below more conservative)
    if (!SPLIT && has_next && (img + G >= img_switch ? 1 : 0) != set) prefetch_w(set ^ 1);
    if (conv_first) {
      if (has_next) wait_dma(it == 0);
      PROBE(d.probe, NW, it, 1);
      if (has_next) {
        convert(Pn);
        if (img + 2 * G < d.N) issue_dma(img + 2 * G, it + 2);
      }
      PROBE(d.probe, NW, it, 2);
      compute(Pc, img);
      PROBE(d.probe, NW, it, 3);
    } else {
      compute(Pc, img);
      PROBE(d.probe, NW, it, 1);
      if (has_next) wait_dma(false);
      PROBE(d.probe, NW, it, 2);
      if (has_next) {
        convert(Pn);
        if (img + 2 * G < d.N) issue_dma(img + 2 * G, it + 2);
      }
      PROBE(d.probe, NW, it, 3);
    }
    __syncthreads();   // planes[next] complete, planes[cur] free
  }
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
  if ((d.N + grid - 1) / grid > C1_MAXIMG) grid = (d.N + C1_MAXIMG - 1) / C1_MAXIMG;
  const bool split = d.y_lo != nullptr;
  if (split && (d.w32 == nullptr || (d.w2 != nullptr && d.w2_32 == nullptr))) return (int)hipErrorInvalidValue;
  if (split) {
    switch (d.C) {
      case 1: conv1_s2d_fwd_kernel<1, true><<<grid, C1_THREADS, 0, st>>>(d); break;
      case 2: conv1_s2d_fwd_kernel<2, true><<<grid, C1_THREADS, 0, st>>>(d); break;
      case 4: conv1_s2d_fwd_kernel<4, true><<<grid, C1_THREADS, 0, st>>>(d); break;
      default: return (int)hipErrorInvalidValue;
    }
  } else {
    switch (d.C) {
      case 1: conv1_s2d_fwd_kernel<1, false><<<grid, C1_THREADS, 0, st>>>(d); break;
      case 2: conv1_s2d_fwd_kernel<2, false><<<grid, C1_THREADS, 0, st>>>(d); break;
      case 4: conv1_s2d_fwd_kernel<4, false><<<grid, C1_THREADS, 0, st>>>(d); break;
      default: return (int)hipErrorInvalidValue;
    }
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

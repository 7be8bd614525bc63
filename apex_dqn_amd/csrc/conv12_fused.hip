// conv1 -> conv2 of the dueling NatureCNN fused in one persistent kernel, fp32-accurate
// ("split") operands (duelling_network.py:8-11: Conv(C->64, 8, s4) + ReLU ->
// Conv(64->64, 4, s2) + ReLU; learner.py:43-46 runs it on S_t, S_{t+n} online and
// S_{t+n} target).
//
// Why: the separate kernels (csrc/conv1_s2d.hip + csrc/conv2_img.hip) write conv1's
// output y1 -- 20 x 20 x 64 as hi + lo bf16 planes, 102 KB per image, 157 MB per fp32
// learner step -- to HBM and read it back for conv2, and the conv1 kernel is bound by
// those 8-byte epilogue stores (~10.7 us per image per CU against 2.7 us of MFMA).  Two
// thirds of the rows (S_{t+n}, online and target) feed only conv2 and are never used by
// the backward.  Here a workgroup (4 waves, one per SIMD, one workgroup per CU) walks
// whole images and keeps y1 in LDS:
//   * the image's C uint8 frames arrive by LDS-DMA straight from the space-to-depth
//     replay ring (two staging buffers: image i + 1 lands while image i computes);
//   * conv1: wave w owns output channels 16 w .. 16 w + 15 over all 25 pixel tiles
//     (v_mfma_f32_16x16x32_f16, swapped operands: the weights are A).  The pixel
//     fragment of a K step is 8 bytes of one s2d block, read with ds_read_b64 and turned
//     into f16 (1024 + x) with four v_perm (exact; the offset is folded into the bias).
//     The fp32 weights become f16 hi + lo * 2^-12 (22 significant bits) in registers, two
//     MFMAs per fragment.  The epilogue writes y1's hi / lo planes into LDS in conv2's
//     class-major, chunk-swizzled pixel layout;
//   * rows < copy_n (S_t: the backward needs them) also leave for HBM as coalesced
//     16-byte chunks of the LDS image;
//   * conv2 as the split image-resident kernel (wave (nh, kp) = channel half x
//     kernel-row pair, products x_hi w_hi + x_hi w_lo + x_lo w_hi, 32x32x16 bf16 MFMAs)
//     but with its weights STREAMED: conv1's weights (64 registers) and conv2's hi + lo
//     fragments (256) do not fit one wave's 512 registers together (148 spilled
//     registers), so the conv2 fragments come from L2 in per-lane fragment order
//     (csrc/conv2_wfrag.h C2F layout, 1 KB per wave and K step, every CU reads the same
//     256 KB) three K steps ahead of their MFMAs, 32 GB/s per CU against ~70 available.
//     One pass over K reads both planes and issues all three products.  Operands are
//     swapped so a lane holds 4 consecutive output channels of a pixel; the two
//     kernel-row pairs meet in a 24 KB fp32 LDS buffer (the image's spent staging
//     buffer), summed in fixed order by the kp = 0 waves, which apply bias + ReLU and
//     store y2 as hi / lo planes.
// LDS: y1 hi + lo planes 2 x 52224 B + staging 2 x 28 KB (C = 4) + slot table = 159 KB.
//
// Online / target weights switch at image img_switch; each workgroup takes a contiguous
// image range, so at most one workgroup reloads its weights.
#include "mfma_common.h"
#include "conv2_wfrag.h"

#define CF_THREADS 256
#define CF_PLANE 52224       // y1 plane: 408 class-major pixel slots of 128 B (conv2's padding rows read past 400)
#define CF_MAXIMG 64         // images per workgroup (slot table)
#define CF_FRAME 7056        // s2d frame: 441 blocks of 16 B
#define CF_LO_SCALE 4096.f
#define CF_NY2 12            // y2 epilogue store instructions per wave and image (3 mt x 2 jq x 2 planes)
#define CF_WAHEAD 3          // conv2 weight fragments in flight ahead of their MFMAs (K steps)

// both conv2 weight sets -> C2F fragment order (csrc/conv2_wfrag.h), when not packed yet
__global__ void __launch_bounds__(256) cf_pack_c2f_kernel(C2fPack p) {
  c2f_pack_range(p, blockIdx.x * 256 + threadIdx.x, 4 * C2F_FRAGS);
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct Conv12Desc {
  const uint8_t* ring;     // s2d frame ring [F][441][16]
  const int32_t* slots;    // [N][C] frame slots
  const float* w1;         // conv1 fp32 OIHW [64][C][8][8], online
  const float* w1b;        //   target (images >= img_switch), or null
  const float* b1;
  const float* b1b;
  const bf16_t* w2;        // conv2 OHWI [64][4][4][64] bf16 hi / lo planes, online
  const bf16_t* w2_lo;
  const bf16_t* w2b;       //   target, or null
  const bf16_t* w2b_lo;
  uint4* wfrag;            // both sets in C2F fragment order (4 x C2F_FRAGS uint4: set 0 hi, lo, set 1 hi, lo)
  int wfrag_ready;         // packed earlier in the step; else the launcher packs them first
  const float* b2;
  const float* b2b;
  bf16_t* y1;              // [copy_n][20][20][64] hi / lo (rows < copy_n only)
  bf16_t* y1_lo;
  bf16_t* y2;              // [N][9][9][64] hi / lo
  bf16_t* y2_lo;
  const uint8_t* zero16;   // >= 16 zero bytes (DMA source of the staging tail)
  uint8_t* scratch;        // >= 512 B: target of the y2 stores of padding pixels
  int N, C, img_switch, copy_n;
  float in_scale;
  uint64_t* probe;         // phase stamps (diagnostic build, csrc/mfma_common.h PROBE), or null
};

// class-major y1 pixel slot of input pixel (ih, iw) and the byte offset of its 16-B chunk c
__device__ __forceinline__ int cf_pix(int ih, int iw) { return ((ih & 1) * 2 + (iw & 1)) * 100 + (ih >> 1) * 10 + (iw >> 1); }
__device__ __forceinline__ int cf_off(int P, int c) { return (P << 7) + ((c ^ ((P >> 1) & 7)) << 4); }

template <int C>
__global__ void __launch_bounds__(CF_THREADS, 1) conv12_fused_split_kernel(Conv12Desc d) {
  constexpr int NCHUNK = C * 441;                 // 16-B s2d blocks per image
  constexpr int NDMA = (NCHUNK + 63) / 64;        // 1-KB LDS-DMA instructions per image
  constexpr int NDW = (NDMA + 3) / 4;             // per wave (max)
  // staging buffer (also the conv2 reduction's 24 KB of partials once its image is read)
  constexpr int STGB = NDMA * 1024 > 2 * 3 * 4 * 64 * 16 ? NDMA * 1024 : 2 * 3 * 4 * 64 * 16;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * CF_PLANE + 2 * STGB];
  __shared__ int32_t slot_tbl[CF_MAXIMG * C];
  uint8_t* Y1 = smem;                              // hi plane; lo plane at + CF_PLANE
  uint8_t* STG = smem + 2 * CF_PLANE;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, pl = lane & 15;         // conv1 (16x16 MFMA) lane roles
  const int rr = lane & 31, kg = lane >> 5;        // conv2 (32x32 MFMA) lane roles
  const int nh = wv & 1, kp = wv >> 1;             // conv2 wave roles
  const int per = (d.N + (int)gridDim.x - 1) / (int)gridDim.x;
  const int img0 = blockIdx.x * per, img1 = min(d.N, img0 + per);
  if (img0 >= img1) return;
  const int nimg = img1 - img0;
  for (int i = tid; i < nimg * C; i += CF_THREADS) slot_tbl[i] = d.slots[(int64_t)img0 * C + i];
  __syncthreads();

  // ---- LDS-DMA of image `li` (local index) into staging buffer `buf`: this wave's
  // instructions k = wv + 4 j (1 KB each; lanes past the frames read zeros)
  auto issue_dma = [&](int li, int buf) {
    int sl[4] = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < C; ++c) sl[c] = slot_tbl[li * C + c];
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(STG + buf * STGB);
#pragma unroll
    for (int j = 0; j < NDW; ++j) {
      const int k = wv + 4 * j;
      if (k < NDMA) {
        const int ch = 64 * k + lane;
        const uint8_t* src = d.zero16;
        if (ch < NCHUNK) {
          const int c = ch / 441, blk = ch - c * 441;
          int s = sl[0];
#pragma unroll
          for (int cc = 1; cc < C; ++cc)
            if (c == cc) s = sl[cc];
          src = d.ring + (int64_t)s * CF_FRAME + (blk << 4);
        }
        dma16(src, __builtin_amdgcn_readfirstlane(base + (uint32_t)k * 1024u));
      }
    }
  };

  // ---- conv1: wave w owns output channels 32 cp .. 32 cp + 31 (cp = w & 1; two 16-channel
  // MFMA tiles nt) for the pixel tiles of parity th = w >> 1, so each staged fragment is
  // converted by two waves instead of four.  Weights of channel 32 cp + 16 nt + pl, K
  // 32 s + 8 g .. + 7 (s2d K order k = (tap C + c) 16 + r4 4 + c4, tap = 2 a + b): f16
  // hi + lo * 2^-12
  const int cp = wv & 1, th = wv >> 1;
  f16x8 w1h[2][2 * C], w1l[2][2 * C];
  f32x2v bias1[2][2];                                // [nt]: channels 32 cp + 16 nt + 4 g + {0..3}
  int aoff[2 * C];                                   // staging byte offset of step s's 8-B fragment
#pragma unroll
  for (int s = 0; s < 2 * C; ++s) {
    const int q = 2 * s + (g >> 1), tap = q / C, c = q - tap * C;
    aoff[s] = c * CF_FRAME + (((tap >> 1) * 21 + (tap & 1)) << 4) + ((g & 1) << 3);
  }
  float4 bias2[2];                                   // conv2 bias of the quads this wave finishes:
                                                     // channels 32 nh + 8 (2 kp + jh) + 4 kg .. + 3
  const uint4* wf = nullptr;                         // this wave's conv2 fragments (hi; lo at + C2F_FRAGS)
  auto load_weights = [&](int set) {
    const float* W1 = set ? d.w1b : d.w1;
    const float* B1 = set ? d.b1b : d.b1;
    const float k = 1024.f * d.in_scale;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int n = 32 * cp + 16 * nt + pl;
      float ws = 0.f;
#pragma unroll
      for (int s = 0; s < 2 * C; ++s) {
        const int q = 2 * s + (g >> 1), tap = q / C, c = q - tap * C, h = g & 1;
        const int kh = 4 * (tap >> 1) + 2 * h, kw = 4 * (tap & 1);
        const float4 r0 = *reinterpret_cast<const float4*>(W1 + ((n * C + c) * 8 + kh) * 8 + kw);
        const float4 r1 = *reinterpret_cast<const float4*>(W1 + ((n * C + c) * 8 + kh + 1) * 8 + kw);
        const float w8[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const _Float16 hi = (_Float16)w8[j];
          const _Float16 lo = (_Float16)((w8[j] - (float)hi) * CF_LO_SCALE);
          w1h[nt][s][j] = hi;
          w1l[nt][s][j] = lo;
          ws += (float)hi + (float)lo * (1.f / CF_LO_SCALE);
        }
      }
      // channel sums over the four K-group lanes; the epilogue's channels 4 g + i take
      // theirs: bias' = bias - 1024 * in_scale * sum_k w16[n][k] (pixels enter as 1024 + x)
      ws += __shfl_xor(ws, 16, 64);
      ws += __shfl_xor(ws, 32, 64);
      float c4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) c4[i] = __shfl(ws, 4 * g + i, 64);
      const float4 bb = *reinterpret_cast<const float4*>(B1 + 32 * cp + 16 * nt + 4 * g);
      bias1[nt][0] = (f32x2v){bb.x - k * c4[0], bb.y - k * c4[1]};
      bias1[nt][1] = (f32x2v){bb.z - k * c4[2], bb.w - k * c4[3]};
    }
    wf = d.wfrag + set * 2 * C2F_FRAGS + wv * 32 * 64 + lane;
    const float* B2 = set ? d.b2b : d.b2;
#pragma unroll
    for (int jh = 0; jh < 2; ++jh)
      bias2[jh] = *reinterpret_cast<const float4*>(B2 + nh * 32 + 8 * (2 * kp + jh) + 4 * kg);
    // drained here, once per weight set (the compiler does not count the asm DMAs)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  // conv2 M rows (output pixels on a 10-wide grid, 96 = 3 tiles of 32): class-major
  // pixel slot of this lane's row at kernel-row pair kp, column 0
  int q0[3];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) {
    const int r = mt * 32 + rr, oh = r / 10, ow = r - oh * 10;
    q0[mt] = (oh + kp) * 10 + ow;
  }

  const bool two = d.w1b != nullptr;
  int cur_set = -1;
  issue_dma(0, 0);
  if (nimg > 1) issue_dma(1, 1);
  for (int i = 0; i < nimg; ++i) {
    const int img = img0 + i;
    const int set = (two && img >= d.img_switch) ? 1 : 0;
    if (set != cur_set) {
      load_weights(set);      // vmcnt(0): every DMA issued so far has landed as well
      cur_set = set;
      __syncthreads();
    }
    PROBE(d.probe, 4, i, 0);
    const uint8_t* S = STG + (i & 1) * STGB;
    // ================= conv1: this wave's pixel tiles T = th, th + 2, .. (16 pixels each)
    // x 32 channels.  Software-pipelined over tiles (one wave per SIMD hides nothing by
    // itself): the 2C fragment reads of the next tile are in flight while this tile's
    // MFMAs issue, and the previous tile's epilogue runs behind them.
    {
      const int nT = th == 0 ? 13 : 12;
      auto load_tile = [&](int j, uint2* u) {
        const int p = 16 * (th + 2 * j) + pl, oh = p / 20, ow = p - 20 * oh;
        const uint8_t* A = S + ((oh * 21 + ow) << 4);
#pragma unroll
        for (int s2 = 0; s2 < 2 * C; ++s2) u[s2] = *reinterpret_cast<const uint2*>(A + aoff[s2]);
      };
      auto mfma_tile = [&](const uint2* u, f32x4* acc, f32x4* accl) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[nt] = accl[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 2 * C; ++s2) {
          const f16x8 a = __builtin_bit_cast(f16x8, u8x8_to_f16off(u[s2].x, u[s2].y));
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1h[nt][s2], a, acc[nt], 0, 0, 0);
            accl[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1l[nt][s2], a, accl[nt], 0, 0, 0);
          }
        }
      };
      // lane: channels 32 cp + 16 nt + 4 g .. + 3 of pixel (oh, ow) -> y1 hi / lo planes
      auto epi = [&](int j, const f32x4* acc, const f32x4* accl) {
        const int p = 16 * (th + 2 * j) + pl, oh = p / 20, ow = p - 20 * oh;
        const int P = cf_pix(oh, ow);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[r] = fmaxf((acc[nt][r] + accl[nt][r] * (1.f / CF_LO_SCALE)) * d.in_scale + bias1[nt][r >> 1][r & 1],
                         0.f);
          uint32_t h01, l01, h23, l23;
          split_pk_bf16(v[0], v[1], h01, l01);
          split_pk_bf16(v[2], v[3], h23, l23);
          const int ch = 32 * cp + 16 * nt + 4 * g;
          const int off = cf_off(P, ch >> 3) + (ch & 7) * 2;
          *reinterpret_cast<uint2*>(Y1 + off) = make_uint2(h01, h23);
          *reinterpret_cast<uint2*>(Y1 + CF_PLANE + off) = make_uint2(l01, l23);
        }
      };
      uint2 uA[2 * C], uB[2 * C];
      f32x4 aA[2], aAl[2], aB[2], aBl[2];
      load_tile(0, uA);
      load_tile(1, uB);
      __builtin_amdgcn_sched_barrier(0);
      mfma_tile(uA, aA, aAl);                    // tile 0
      for (int j = 1; j < nT; j += 2) {          // uA: tile j - 1 (consumed), uB: tile j
        if (j + 1 < nT) load_tile(j + 1, uA);
        __builtin_amdgcn_sched_barrier(0);
        mfma_tile(uB, aB, aBl);                  // tile j
        epi(j - 1, aA, aAl);
        __builtin_amdgcn_sched_barrier(0);
        if (j + 1 < nT) {
          if (j + 2 < nT) load_tile(j + 2, uB);
          __builtin_amdgcn_sched_barrier(0);
          mfma_tile(uA, aA, aAl);                // tile j + 1
        }
        epi(j, aB, aBl);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (nT & 1) epi(nT - 1, aA, aAl);
    }
    PROBE(d.probe, 4, i, 1);
    // image i + 1's frames (issued during image i - 1) have landed: only the CF_NY2 y2
    // stores of image i - 1 are younger (their acks are not waited for)
    static_assert(CF_NY2 == 12, "the vmcnt below counts the y2 epilogue stores");
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    __syncthreads();          // y1 complete; staging(i) read; staging(i + 1) visible
    const bool copy = img < d.copy_n;
    // S_t rows: y1 (hi, lo) leaves for HBM (the backward's input).  Thread tid copies LDS
    // chunks k = tid + 256 r in LDS order (pixel slot P = k >> 3, stored chunk k & 7):
    // the LDS reads are immediate offsets, and 8 consecutive lanes write one pixel's full
    // 128-B NHWC row.  Reads go out in batches of 5 (20 registers), stores are not waited.
    if (copy) {
      // (opaque copy of tid: keeps the compiler from hoisting the 25 per-thread addresses
      // out of the image loop into registers it does not have)
      int tq = tid;
      asm volatile("" : "+v"(tq));
      const int cst = tq & 7;
#pragma unroll
      for (int r0 = 0; r0 < 25; r0 += 5) {
        uint4 v[5];
#pragma unroll
        for (int r = 0; r < 5; ++r)
          v[r] = *reinterpret_cast<const uint4*>(
              Y1 + (r0 + r) * 4096 + tq * 16 +
              ((r0 + r > 12 || (r0 + r == 12 && tq >= 128)) ? CF_PLANE - 51200 : 0));    // lo plane
#pragma unroll
        for (int r = 0; r < 5; ++r) {
          const int k = tq + CF_THREADS * (r0 + r);
          const int plane = k >= 3200 ? 1 : 0, kk = k - plane * 3200;
          const int P = kk >> 3, c = cst ^ ((P >> 1) & 7);      // the chunk stored at slot cst
          const int cls = P / 100, q = P - cls * 100, a = q / 10, b = q - a * 10;
          const int ih = 2 * a + (cls >> 1), iw = 2 * b + (cls & 1);
          *reinterpret_cast<uint4*>((plane ? d.y1_lo : d.y1) + (int64_t)img * 25600 + (ih * 20 + iw) * 64 + c * 8) =
              v[r];
        }
      }
    }
    PROBE(d.probe, 4, i, 2);
    // ================= conv2 over the resident hi / lo planes, weights streamed from L2
    // K step s: kernel row kh = 2 kp + (s >> 4), column kw = (s >> 2) & 3, channels
    // 16 (s & 3) + 8 kg .. + 7; fragments of step s + CF_WAHEAD are in flight
    f32x16 acc2[3];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc2[mt][j] = 0.f;
    {
      bf16x8 wh[CF_WAHEAD + 1], wl[CF_WAHEAD + 1];
#pragma unroll
      for (int s = 0; s < CF_WAHEAD; ++s) {
        wh[s] = __builtin_bit_cast(bf16x8, wf[s * 64]);
        wl[s] = __builtin_bit_cast(bf16x8, wf[C2F_FRAGS + s * 64]);
      }
      bf16x8 ah[2][3], al[2][3];
#define CF_LDA(s_, buf_)                                                                     \
      _Pragma("unroll") for (int mt = 0; mt < 3; ++mt) {                                     \
        const int P_ = (((s_) >> 4) * 2 + (((s_) >> 2) & 1)) * 100 + q0[mt] + (((s_) >> 3) & 1); \
        const int o_ = cf_off(P_, (((s_) & 3) << 1) | kg);                                   \
        ah[buf_][mt] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(Y1 + o_)); \
        al[buf_][mt] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(Y1 + CF_PLANE + o_)); \
      }
      CF_LDA(0, 0)
#pragma unroll
      for (int s = 0; s < 32; ++s) {
        if (s + CF_WAHEAD < 32) {
          wh[(s + CF_WAHEAD) % (CF_WAHEAD + 1)] = __builtin_bit_cast(bf16x8, wf[(s + CF_WAHEAD) * 64]);
          wl[(s + CF_WAHEAD) % (CF_WAHEAD + 1)] = __builtin_bit_cast(bf16x8, wf[C2F_FRAGS + (s + CF_WAHEAD) * 64]);
        }
        if (s + 1 < 32) CF_LDA(s + 1, (s + 1) & 1)
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 bh = wh[s % (CF_WAHEAD + 1)], bl = wl[s % (CF_WAHEAD + 1)];
#pragma unroll
        for (int mt = 0; mt < 3; ++mt) {
          acc2[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bl, ah[s & 1][mt], acc2[mt], 0, 0, 0);
          acc2[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh, al[s & 1][mt], acc2[mt], 0, 0, 0);
          acc2[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh, ah[s & 1][mt], acc2[mt], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#undef CF_LDA
    }
    PROBE(d.probe, 4, i, 3);
    __syncthreads();          // every read of y1 is done: its LDS takes the partial sums
    // the two kernel-row pairs meet in LDS: wave (nh, kp) finishes output channels
    // 32 nh + 16 kp .. + 15 (jq = 2 kp, 2 kp + 1) and hands the other half of its partial
    // sums to its partner; sum = (bias + pair 0) + pair 1 in both waves (fixed order)
    float4* red = reinterpret_cast<float4*>(Y1);
    // (kp is wave-uniform: both branches index the accumulators with constants)
    auto give = [&](const int jq0) {
#pragma unroll
      for (int mt = 0; mt < 3; ++mt)
#pragma unroll
        for (int jh = 0; jh < 2; ++jh)
          red[(((kp * 2 + nh) * 3 + mt) * 2 + jh) * 64 + lane] =
              make_float4(acc2[mt][4 * (jq0 + jh)], acc2[mt][4 * (jq0 + jh) + 1], acc2[mt][4 * (jq0 + jh) + 2],
                          acc2[mt][4 * (jq0 + jh) + 3]);
    };
    if (kp == 0) give(2);
    else give(0);
    // staging(i) is free (read by conv1(i)): image i + 2's frames go there now, ahead of
    // this image's epilogue stores (the wait after the next conv1 counts only those)
    if (i + 2 < nimg) issue_dma(i + 2, i & 1);
    __syncthreads();          // partials visible
    // acc2[mt][4 jq + i] = D[channel 32 nh + 8 jq + 4 kg + i][pixel mt * 32 + rr]
    auto finish = [&](const int jq0, const bool own_first) {
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) {
        const int r = mt * 32 + rr, oh = r / 10, ow = r - oh * 10;
        const bool valid = oh < 9 && ow < 9;
#pragma unroll
        for (int jh = 0; jh < 2; ++jh) {
          const int jq = jq0 + jh;
          const float4 o = red[((((kp ^ 1) * 2 + nh) * 3 + mt) * 2 + jh) * 64 + lane];
          const float4 own = make_float4(acc2[mt][4 * jq], acc2[mt][4 * jq + 1], acc2[mt][4 * jq + 2],
                                         acc2[mt][4 * jq + 3]);
          const float4 p0 = own_first ? own : o, p1 = own_first ? o : own;
          const float4 bb = bias2[jh];
          const float v0 = fmaxf((bb.x + p0.x) + p1.x, 0.f);
          const float v1 = fmaxf((bb.y + p0.y) + p1.y, 0.f);
          const float v2 = fmaxf((bb.z + p0.z) + p1.z, 0.f);
          const float v3 = fmaxf((bb.w + p0.w) + p1.w, 0.f);
          uint32_t h01, l01, h23, l23;
          split_pk_bf16(v0, v1, h01, l01);
          split_pk_bf16(v2, v3, h23, l23);
          // every lane stores (padding pixels into scratch): a fixed count of CF_NY2 store
          // instructions per wave keeps the vmcnt wait of the next image exact
          const int64_t o2 = ((int64_t)img * 81 + oh * 9 + ow) * 64 + nh * 32 + 8 * jq + 4 * kg;
          bf16_t* dh = valid ? d.y2 + o2 : reinterpret_cast<bf16_t*>(d.scratch + lane * 8);
          bf16_t* dl = valid ? d.y2_lo + o2 : reinterpret_cast<bf16_t*>(d.scratch + lane * 8);
          *reinterpret_cast<uint2*>(dh) = make_uint2(h01, h23);
          *reinterpret_cast<uint2*>(dl) = make_uint2(l01, l23);
        }
      }
    };
    if (kp == 0) finish(0, true);        // (bias + own pair 0) + pair 1
    else finish(2, false);               // (bias + pair 0) + own pair 1
    __syncthreads();          // the partials are read: y1's LDS is free for the next conv1
  }
}

APEX_EXPORT int apex_conv12_fused_fwd(Conv12Desc d, int grid, hipStream_t st) {
  if (d.N < 1) return 0;
  if (d.ring == nullptr || d.slots == nullptr || d.w1 == nullptr || d.b1 == nullptr || d.w2 == nullptr ||
      d.w2_lo == nullptr || d.b2 == nullptr || d.y2 == nullptr || d.y2_lo == nullptr || d.zero16 == nullptr ||
      d.wfrag == nullptr || d.scratch == nullptr)
    return (int)hipErrorInvalidValue;
  const bool two = d.w1b != nullptr;
  if (two && (d.b1b == nullptr || d.w2b == nullptr || d.w2b_lo == nullptr || d.b2b == nullptr))
    return (int)hipErrorInvalidValue;
  if (d.copy_n > 0 && (d.y1 == nullptr || d.y1_lo == nullptr || d.copy_n > d.N)) return (int)hipErrorInvalidValue;
  if ((((uintptr_t)d.w1 | (uintptr_t)(two ? d.w1b : d.w1) | (uintptr_t)d.b1 | (uintptr_t)(two ? d.b1b : d.b1) |
        (uintptr_t)d.w2 | (uintptr_t)d.w2_lo | (uintptr_t)d.b2 | (uintptr_t)d.y1 | (uintptr_t)d.y1_lo) & 15) ||
      (((uintptr_t)d.y2 | (uintptr_t)d.y2_lo | (uintptr_t)d.scratch) & 7) || ((uintptr_t)d.wfrag & 15))
    return (int)hipErrorInvalidValue;
  int G = grid > 0 ? grid : 256;
  if (G > d.N) G = d.N;
  if ((d.N + G - 1) / G > CF_MAXIMG) G = (d.N + CF_MAXIMG - 1) / CF_MAXIMG;
  if (!d.wfrag_ready)
    cf_pack_c2f_kernel<<<4 * C2F_FRAGS / 256, 256, 0, st>>>(C2fPack{{d.w2, d.w2_lo, d.w2b, d.w2b_lo}, d.wfrag, 0});
  switch (d.C) {
    case 1: conv12_fused_split_kernel<1><<<G, CF_THREADS, 0, st>>>(d); break;
    case 2: conv12_fused_split_kernel<2><<<G, CF_THREADS, 0, st>>>(d); break;
    case 4: conv12_fused_split_kernel<4><<<G, CF_THREADS, 0, st>>>(d); break;
    default: return (int)hipErrorInvalidValue;
  }
  APEX_CHECK_LAUNCH();
}

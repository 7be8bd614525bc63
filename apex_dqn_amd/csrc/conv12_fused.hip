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
//
// bf16 learner (SPLIT = false, d.bf16): the same pipeline with one operand plane -- conv1
// runs the f16 hi chain only (w * in_scale rounded to f16: at least bf16's precision), y1
// is one bf16 plane in LDS (and in HBM for the S_t rows), conv2 issues one product per
// fragment (x w, the bf16 weights) and y2 is one bf16 plane.
#include "mfma_common.h"
#include "conv2_wfrag.h"
#include "cf_pack.h"

#define CF_THREADS 256
#define CF_PLANE 52224       // y1 plane: 408 class-major pixel slots of 128 B (conv2's padding rows read past 400)
#define CF_MAXIMG 64         // images per workgroup (slot table)
#define CF_FRAME 7056        // s2d frame: 441 blocks of 16 B
#define CF_NY2 12            // y2 store instructions per wave and image (3 mt x 2 jh x 2 planes)
#define CF_WAHEAD 3          // conv2 weight fragments in flight ahead of their MFMAs (K steps)
#define CF_W3AHEAD 5         // fused conv3: weight fragments in flight ahead of their MFMAs
#define CF_W3EARLY 0         // 1: the first ones issued before conv2's epilogue (spills at C = 4)

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
  int pack_sets;           // weight sets the launcher (re)packs first (wfrag, w1frag): bit 0 online,
                           // bit 1 target; the others' fragments are current (cf_pack_kernel)
  const float* b2;
  const float* b2b;
  bf16_t* y1;              // [copy_n][20][20][64] hi / lo (rows < copy_n only)
  bf16_t* y1_lo;
  bf16_t* y2;              // [N][9][9][64] hi / lo
  bf16_t* y2_lo;
  uint4* w1frag;           // conv1 f16 hi / lo fragments of both sets (CF_W1FRAG_U4 uint4), written
                           // by cf_pack_kernel or (online set) by the previous optimizer launch
  uint8_t* scratch;        // >= 512 B: target of the y2 stores of padding pixels
  int N, C, img_switch, copy_n;
  float in_scale;
  uint64_t* probe;         // phase stamps (diagnostic build, csrc/mfma_common.h PROBE), or null
  unsigned long long* wq;  // image work queue counter (mfma_common.h wq_next), or null: static
                           // strided image order
  int bf16;                // 1: one bf16 plane everywhere (w2_lo, y1_lo, y2_lo unused)
  int probe_split;         // diagnostic build: bit 0 = wait for the first image's frames before
                           // the weight loads (prologue split); 0 otherwise
  // conv3 fused (w3 non-null): 3x3 / s1, OHWI [64][3][3][64] bf16 hi / lo planes per set,
  // fp32 biases; y3 [N][7][7][64] hi / lo (ReLU'd) -- conv3 reads y2 from LDS
  const bf16_t* w3;
  const bf16_t* w3_lo;
  const bf16_t* w3b;
  const bf16_t* w3b_lo;
  const float* b3;
  const float* b3b;
  bf16_t* y3;
  bf16_t* y3_lo;
  uint4* w3frag;           // both sets' conv3 weights in C3F fragment order (csrc/conv2_wfrag.h:
                           // set 0 hi, lo, set 1 hi, lo), packed with the other fragments
};

template <int C>
__global__ void __launch_bounds__(256) cf_pack_kernel(CfPack p) {
  if ((int)blockIdx.x < p.nc2f) {
    c2f_pack_range(p.c2f, blockIdx.x * 256 + threadIdx.x, p.nc2f * 256);
    return;
  }
  if ((int)blockIdx.x < p.nc2f + p.nc3f) {
    c3f_pack_range(p.c3f, (blockIdx.x - p.nc2f) * 256 + threadIdx.x, p.nc3f * 256);
    return;
  }
  cf_pack_w1_block(p, C, (int)blockIdx.x - p.nc2f - p.nc3f, threadIdx.x);
}

// class-major y1 pixel slot of input pixel (ih, iw) and the byte offset of its 16-B chunk c
__device__ __forceinline__ int cf_pix(int ih, int iw) { return ((ih & 1) * 2 + (iw & 1)) * 100 + (ih >> 1) * 10 + (iw >> 1); }
__device__ __forceinline__ int cf_off(int P, int c) { return (P << 7) + ((c ^ ((P >> 1) & 7)) << 4); }

// y2 stores younger than the last frame DMA piece after conv1 (store of tile q = j - 1 at
// tile j >= 1, after that tile's piece; the bf16 kernel stores plane 0 only: even q)
__host__ __device__ constexpr int cf_young_stores(int ndw, bool split) {
  int n = 0;
  for (int q = ndw - 1; q < 12; ++q) n += (split || (q & 1) == 0) ? 1 : 0;
  return n;
}

template <int C, bool SPLIT>
__global__ void __launch_bounds__(CF_THREADS, 1) conv12_fused_kernel(Conv12Desc d) {
  // staging buffer: an image's C frames (s2d, 7056 B each), then the conv2 reduction's
  // 24 KB of partials once conv1 has read them
  constexpr int STGB = C * CF_FRAME > 2 * 3 * 4 * 64 * 16 ? C * CF_FRAME : 2 * 3 * 4 * 64 * 16;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * CF_PLANE + 2 * STGB];
  __shared__ int q_img;                            // the work queue's next-but-one image
  uint8_t* Y1 = smem;                              // hi plane; lo plane at + CF_PLANE
  uint8_t* STG = smem + 2 * CF_PLANE;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: branches on wave
                                                             // roles stay scalar
  const int g = lane >> 4, pl = lane & 15;         // conv1 (16x16 MFMA) lane roles
  const int rr = lane & 31, kg = lane >> 5;        // conv2 (32x32 MFMA) lane roles
  const int nh = wv & 1, kp = wv >> 1;             // conv2 wave roles
  // Images come from a device-side work queue (d.wq, csrc/mfma_common.h wq_*), two ahead
  // of the one in flight: a workgroup that starts late -- its CU held by another kernel,
  // e.g. RCCL's beside a data-parallel step -- takes fewer images instead of holding the
  // launch up (scripts/bench_cu_steal.py).  Every image is computed whole by one
  // workgroup, so the outputs do not depend on the assignment.  Images leave the queue in
  // order: the S_t rows (y1 also copied out) spread over all workgroups first.
  PROBE(d.probe, 4, PROBE_ITERS - 1, 0);          // kernel entry (diagnostic build)
#ifdef APEX_PROBE
  if (d.probe != nullptr && blockIdx.x < PROBE_BLOCKS && (threadIdx.x & 63) == 0)
    d.probe[((blockIdx.x * 4 + (threadIdx.x >> 6)) * PROBE_ITERS + PROBE_ITERS - 1) * 4 + 2] =
        __builtin_amdgcn_s_memrealtime();
#endif
  int wq_seq = 0;                                  // (thread 0: static order, d.wq null)
  if (tid == 0) {
    // (the second fetch only after an item: each workgroup stops at its first value >= N)
    const int a = wq_next(d.wq, wq_seq, d.N), b = a < d.N ? wq_next(d.wq, wq_seq, d.N) : d.N;
    reinterpret_cast<volatile int*>(&q_img)[0] = a;
    reinterpret_cast<volatile int*>(Y1)[0] = b;     // (y1 is free until the first conv1)
  }
  __syncthreads();
  int cur = __builtin_amdgcn_readfirstlane(reinterpret_cast<volatile int*>(&q_img)[0]);
  int nxt = __builtin_amdgcn_readfirstlane(reinterpret_cast<volatile int*>(Y1)[0]);
  __syncthreads();

  // ---- LDS-DMA of image `li` into staging buffer `buf`: piece k = wv + 4 j (1 KB) copies
  // bytes 1024 r .. of frame c = k / 7 (r = k % 7; the frame's 7056 bytes end 48 lanes into
  // piece 6).  Frame slots of the image in SGPRs (`sl`), the address a scalar base plus
  // the lane's 16 B: a piece is a handful of scalar instructions and one DMA.
  constexpr int NPF = (CF_FRAME + 1023) / 1024;   // pieces per frame (7)
  constexpr int NDMA = C * NPF;
  constexpr int NDW = (NDMA + 3) / 4;             // per wave (max)
  // (the slots travel as a vector VALUE: an int[4] whose element was picked by a runtime
  // frame index became a scratch array, and each scratch load's vmcnt(0) waited for every
  // DMA piece and y2 store in flight)
  typedef int sl4_t __attribute__((ext_vector_type(4)));
  auto image_slots = [&](int img) -> sl4_t {
    int a[4];
    sload_slots<C>(d.slots + (int64_t)img * C, a);
    return (sl4_t){a[0], a[1], a[2], a[3]};
  };
  auto issue_dma_piece = [&](const sl4_t sl, int buf, int j) {
    const int k = wv + 4 * j;
    if (k < NDMA) {
      const int c = k / NPF, r = k - c * NPF;
      const int s = __builtin_amdgcn_readfirstlane(c == 0 ? sl.x : c == 1 ? sl.y : c == 2 ? sl.z : sl.w);
      const uint8_t* src = d.ring + (int64_t)s * CF_FRAME + r * 1024;
      const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(STG + buf * STGB) +
                           (uint32_t)(c * CF_FRAME + r * 1024);
      if (r * 1024 + lane * 16 < CF_FRAME) dma16_s(src, (uint32_t)lane * 16u, dst);
    }
  };
  auto issue_dma = [&](int img, int buf) {
    const sl4_t sl = image_slots(img);
#pragma unroll
    for (int j = 0; j < NDW; ++j) issue_dma_piece(sl, buf, j);
  };

  // ---- conv1: wave w owns output channels 32 cp .. 32 cp + 31 (cp = w & 1; two 16-channel
  // MFMA tiles nt) for the pixel tiles of parity th = w >> 1, so each staged fragment is
  // converted by two waves instead of four.  Weights of channel 32 cp + 16 nt + pl, K
  // 32 s + 8 g .. + 7 (s2d K order k = (tap C + c) 16 + r4 4 + c4, tap = 2 a + b): f16
  // hi + lo * 2^-12
  const int cp = wv & 1, th = wv >> 1;
  f16x8 w1h[2][2 * C], w1l[2][2 * C];
  f32x4 bias1[2];                                    // [nt]: channels 32 cp + 16 nt + 4 g + {0..3}
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
    const uint4* F = d.w1frag + (((set * 2 + cp) * 2) * 2 * C * 2) * 64 + lane;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
      for (int s = 0; s < 2 * C; ++s) {
        w1h[nt][s] = __builtin_bit_cast(f16x8, F[((nt * 2 * C + s) * 2) * 64]);
        if (SPLIT) w1l[nt][s] = __builtin_bit_cast(f16x8, F[((nt * 2 * C + s) * 2 + 1) * 64]);
      }
      // the bias the hi chain starts from: b - 1024 * sum_k w16[n][k] (pixels enter as
      // 1024 + x): this lane's 2C x 8 K values of channel 32 cp + 16 nt + pl, summed over
      // the four K-group lanes (fixed order), then gathered into the accumulator layout
      // (lane (g, pl) holds channels 4 g .. 4 g + 3 of its pixel)
      float ws = 0.f;
#pragma unroll
      for (int s = 0; s < 2 * C; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) ws += (float)w1h[nt][s][j] + (SPLIT ? (float)w1l[nt][s][j] * (1.f / CF_LO_SCALE) : 0.f);
      ws += __shfl_xor(ws, 16, 64);
      ws += __shfl_xor(ws, 32, 64);
      const float* B1 = set ? d.b1b : d.b1;
      const float4 bb = *reinterpret_cast<const float4*>(B1 + 32 * cp + 16 * nt + 4 * g);
      const float s0 = __shfl(ws, 4 * g, 64), s1 = __shfl(ws, 4 * g + 1, 64);
      const float s2 = __shfl(ws, 4 * g + 2, 64), s3 = __shfl(ws, 4 * g + 3, 64);
      bias1[nt] = (f32x4){bb.x - 1024.f * s0, bb.y - 1024.f * s1, bb.z - 1024.f * s2, bb.w - 1024.f * s3};
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
  // y2 of the previous image waits in registers (hi, lo of channels .. + 3 per (mt, jh)) and
  // leaves during the next conv1, one store per tile among the MFMAs: a wave's store issue
  // moves ~7-25 B per cycle, so 12 stores in a row after the reduction cost ~3k cycles
  uint4 pend[3][2];
  int pend_img = -1;
  // byte offset of this lane's y2 quad at (mt, jq = 0) within an image, -1 for padding
  // rows (their lanes skip; every wave has valid lanes in each mt, so the 12 store
  // instructions per wave and image that the vmcnt wait after conv1 counts always issue)
  int yoff[3];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) {
    const int r = mt * 32 + rr, oh = r / 10, ow = r - oh * 10;
    yoff[mt] = (oh < 9 && ow < 9) ? ((oh * 9 + ow) * 64 + nh * 32 + 4 * kg) * 2 : -1;
  }
  auto store_y2 = [&](int q) {       // q = 2 (2 mt + jh) + plane, 0 .. 11
    const int mt = q >> 2, jh = (q >> 1) & 1, plane = q & 1;
    const int jq = 2 * kp + jh;
    // uniform base (image) + 32-bit lane offset: the saddr store form, no 64-bit math
    if (!SPLIT && plane) return;
    const uint8_t* base = reinterpret_cast<const uint8_t*>((plane ? d.y2_lo : d.y2) + (int64_t)pend_img * 5184);
    if (yoff[mt] >= 0) {
      const uint4 v = pend[mt][jh];
      *reinterpret_cast<uint2*>(const_cast<uint8_t*>(base) + (uint32_t)(yoff[mt] + 16 * jq)) =
          plane ? make_uint2(v.z, v.w) : make_uint2(v.x, v.y);
    }
  };
  // ---- conv3 (fused, d.w3 != null): after image img's conv2 epilogue, its y2 (this wave's
  // quads in `pend`) goes into the image's spent staging buffer as hi / lo planes of 96
  // pixel slots (slot oh * 9 + ow; conv2's class swizzle cf_off), then conv3 runs from
  // there: wave (nt = wv & 1, kh3 = wv >> 1) takes output channels 32 nt .. + 31 over all
  // 64 rows r = 32 mt + rr (output pixel (r / 9, r % 9), valid < 7 x 7: the input slot of
  // tap (kh, kw) is r + 9 kh + kw) and K steps 18 kh3 .. + 17 of 36 (tap s >> 2, 16
  // channels 16 (s & 3) ..); weights straight from OHWI (L2-resident, CF_WAHEAD steps
  // ahead).  The two K halves meet in the (free) y1 planes; kh3 = 0 sums them in fixed
  // order, + bias, ReLU, hi / lo split, stores y3.  Padding slots and invalid rows only
  // feed output columns that are never stored (MFMA columns are independent).
  // conv3 weights: lane's row = output channel 32 nt + rr (nt = wv & 1), K chunk kg of each
  // 16-channel step; step s of this wave's 18 (kh3 = wv >> 1: steps 18 kh3 ..) lives in
  // slot s % (CF_W3AHEAD + 1) (6 in flight spill at C = 4; issued before conv2 s epilogue, 4 do).
  bf16x8 wh3[CF_W3AHEAD + 1], wl3[CF_W3AHEAD + 1];
  // (the C3F fragments: one coalesced 1-KB load per wave and K step; the OHWI rows were 32
  // scattered 32-B pieces per load)
  auto w3row = [&](const int set3, const bool lo) -> const uint4* {
    return d.w3frag + (2 * set3 + (lo ? 1 : 0)) * C3F_FRAGS + (wv & 1) * 36 * 64 + lane;
  };
  auto wofs3 = [](int s) { return s * 64; };
  auto conv3_prefetch = [&](const int set3) {
    const uint4* wr = w3row(set3, false);
    const uint4* wrl = SPLIT ? w3row(set3, true) : wr;
    const int s0 = 18 * (wv >> 1);
#pragma unroll
    for (int q = 0; q < CF_W3AHEAD; ++q) {
      wh3[q] = *reinterpret_cast<const bf16x8*>(wr + wofs3(s0 + q));
      if (SPLIT) wl3[q] = *reinterpret_cast<const bf16x8*>(wrl + wofs3(s0 + q));
    }
  };
  auto conv3_image = [&](const int img, const int set3, uint8_t* Y2S, const int it) {
    const int nt = wv & 1, kh3 = wv >> 1;
    if (it == 0) PROBE(d.probe, 4, PROBE_ITERS - 3, 0);   // (diagnostic build: conv3 phases, image 0)
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
#pragma unroll
      for (int jh = 0; jh < 2; ++jh) {
        const int r = mt * 32 + rr, oh = r / 10, ow = r - oh * 10;
        if (oh < 9 && ow < 9) {
          const int jq = 2 * kp + jh;
          const int off = cf_off(oh * 9 + ow, 4 * nh + jq) + 8 * kg;
          const uint4 v = pend[mt][jh];
          *reinterpret_cast<uint2*>(Y2S + off) = make_uint2(v.x, v.y);
          if (SPLIT) *reinterpret_cast<uint2*>(Y2S + 12288 + off) = make_uint2(v.z, v.w);
        }
      }
    }
    __syncthreads();          // y2 of the image complete in LDS
    if (it == 0) PROBE(d.probe, 4, PROBE_ITERS - 3, 1);
    const uint4* wr = w3row(set3, false);
    const uint4* wrl = SPLIT ? w3row(set3, true) : wr;
    f32x16 acc3[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc3[mt][j] = 0.f;
    const int s0 = 18 * kh3;
    if (!CF_W3EARLY) conv3_prefetch(set3);
    // the biases of the two channel quads this wave finishes, loaded ahead of the MFMA loop
    // (an epilogue load is one exposed L2 round trip)
    const float* B3 = set3 ? d.b3b : d.b3;
    float4 bias3[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) bias3[jj] = *reinterpret_cast<const float4*>(B3 + 32 * nt + 8 * ((kh3 ? 2 : 0) + jj) + 4 * kg);
    bf16x8 bh3[2][2], bl3[2][2];
    auto lda3 = [&](int s, int buf) {
      const int tap = s >> 2, kh = tap / 3, kw = tap - 3 * kh;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int o = cf_off(mt * 32 + rr + 9 * kh + kw, ((s & 3) << 1) | kg);
        bh3[buf][mt] = *reinterpret_cast<const bf16x8*>(Y2S + o);
        if (SPLIT) bl3[buf][mt] = *reinterpret_cast<const bf16x8*>(Y2S + 12288 + o);
      }
    };
    lda3(s0, 0);
#pragma unroll
    for (int q = 0; q < 18; ++q) {
      const int s = s0 + q;
      if (q + CF_W3AHEAD < 18) {
        wh3[(q + CF_W3AHEAD) % (CF_W3AHEAD + 1)] = *reinterpret_cast<const bf16x8*>(wr + wofs3(s + CF_W3AHEAD));
        if (SPLIT)
          wl3[(q + CF_W3AHEAD) % (CF_W3AHEAD + 1)] = *reinterpret_cast<const bf16x8*>(wrl + wofs3(s + CF_W3AHEAD));
      }
      if (q + 1 < 18) lda3(s + 1, (q + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 ah = wh3[q % (CF_W3AHEAD + 1)], al = wl3[q % (CF_W3AHEAD + 1)];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        if (SPLIT) {
          acc3[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh3[q & 1][mt], acc3[mt], 0, 0, 0);
          acc3[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl3[q & 1][mt], acc3[mt], 0, 0, 0);
        }
        acc3[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh3[q & 1][mt], acc3[mt], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (it == 0) PROBE(d.probe, 4, PROBE_ITERS - 3, 2);
    // K halves meet in the y1 planes (conv2 has read them; conv1 of the next image writes
    // them only after the barrier that closes this image)
    // each wave hands the other K half the channel quads it does not finish: kh3 = 0
    // finishes jq 0, 1 and kh3 = 1 jq 2, 3 of its nt; sum = (bias + half 0) + half 1
    float4* red3 = reinterpret_cast<float4*>(Y1);
    const int jgive = kh3 ? 0 : 2;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int jq = jgive + jj;
        red3[((nt * 2 + mt) * 4 + jq) * 64 + lane] =
            make_float4(acc3[mt][4 * jq], acc3[mt][4 * jq + 1], acc3[mt][4 * jq + 2], acc3[mt][4 * jq + 3]);
      }
    __syncthreads();
    {
      uint8_t* y3h = reinterpret_cast<uint8_t*>(d.y3) + (int64_t)img * 6272;
      uint8_t* y3l = SPLIT ? reinterpret_cast<uint8_t*>(d.y3_lo) + (int64_t)img * 6272 : y3h;
      const int jown = kh3 ? 2 : 0;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int jq = jown + jj;
        // acc3[mt][4 jq + e] = D[channel 32 nt + 8 jq + 4 kg + e][pixel 32 mt + rr]
        const int c0 = 32 * nt + 8 * jq + 4 * kg;
        const float4 bb = bias3[jj];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int r = mt * 32 + rr, oh = r / 9, ow = r - oh * 9;
          const float4 o = red3[((nt * 2 + mt) * 4 + jq) * 64 + lane];
          const float4 own = make_float4(acc3[mt][4 * jq], acc3[mt][4 * jq + 1], acc3[mt][4 * jq + 2],
                                         acc3[mt][4 * jq + 3]);
          const float4 p0 = kh3 ? o : own, p1 = kh3 ? own : o;
          const float v0 = fmaxf((bb.x + p0.x) + p1.x, 0.f);
          const float v1 = fmaxf((bb.y + p0.y) + p1.y, 0.f);
          const float v2 = fmaxf((bb.z + p0.z) + p1.z, 0.f);
          const float v3 = fmaxf((bb.w + p0.w) + p1.w, 0.f);
          uint32_t h01, l01 = 0, h23, l23 = 0;
          if (SPLIT) {
            split_pk_bf16(v0, v1, h01, l01);
            split_pk_bf16(v2, v3, h23, l23);
          } else {
            h01 = cvt_pk_bf16(v0, v1);
            h23 = cvt_pk_bf16(v2, v3);
          }
          if (oh < 7 && ow < 7) {
            const uint32_t off = (uint32_t)(((oh * 7 + ow) * 64 + c0) * 2);
            *reinterpret_cast<uint2*>(y3h + off) = make_uint2(h01, h23);
            if (SPLIT) *reinterpret_cast<uint2*>(y3l + off) = make_uint2(l01, l23);
          }
        }
      }
    }
    __syncthreads();          // staging(i) and the y1 planes are free again
    if (it == 0) PROBE(d.probe, 4, PROBE_ITERS - 3, 3);
  };

  // image i's frames land in staging(i & 1): image 0's here, image i + 1's during conv1(i)
  PROBE(d.probe, 4, PROBE_ITERS - 2, 0);          // (diagnostic build: prologue split)
  if (cur < d.N) issue_dma(cur, 0);
  PROBE(d.probe, 4, PROBE_ITERS - 2, 1);
  for (int i = 0; cur < d.N; ++i) {
    const int img = cur;
    const bool more = nxt < d.N;
    const int set = (two && img >= d.img_switch) ? 1 : 0;
    if (set != cur_set) {
#ifdef APEX_PROBE
      if (i == 0 && (d.probe_split & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (i == 0) PROBE(d.probe, 4, PROBE_ITERS - 2, 2);
#endif
      load_weights(set);      // vmcnt(0): every DMA issued so far has landed as well
      cur_set = set;
      if (i == 0) PROBE(d.probe, 4, PROBE_ITERS - 2, 3);
      __syncthreads();
    }
    sl4_t nsl = (sl4_t){0, 0, 0, 0};                  // image i + 1's frame slots
    if (more) nsl = image_slots(nxt);
    // the image after next (read after this image's last barrier).  The fetch's return is
    // waited for here, before any DMA is in flight: ~0.5 us of one wave per image (the
    // compiler moves the value into a register of its choosing at once, so a later use
    // does not hide the atomic's latency)
    if (tid == 0) reinterpret_cast<volatile int*>(&q_img)[0] = more ? wq_next(d.wq, wq_seq, d.N) : d.N;
    PROBE(d.probe, 4, i, 0);
    const uint8_t* S = STG + (i & 1) * STGB;
    // ================= conv1: this wave's pixel tiles T = th + 2 j, j = 0 .. 12 (16 pixels
    // each; th = 1's 13th tile lies past pixel 399: it reads pixel 399 and writes the
    // spare slots 400..407, which only conv2's invalid rows read) x 32 channels.
    // Software-pipelined: tile j + 1's fragment reads are in flight while tile j's MFMAs
    // issue with tile j - 1's epilogue between them -- every epilogue shares its tile with
    // MFMAs (one wave per SIMD: the vector issue slots an MFMA leaves free are the only
    // free ones).
    {
      auto load_tile = [&](int j, uint2* u) {
        int p = 16 * (th + 2 * j) + pl;
        if (j == 12) p = min(p, 399);
        const int oh = p / 20, ow = p - 20 * oh;
        const uint8_t* A = S + ((oh * 21 + ow) << 4);
#pragma unroll
        for (int s2 = 0; s2 < 2 * C; ++s2) u[s2] = *reinterpret_cast<const uint2*>(A + aoff[s2]);
      };
      // tile j - 1's epilogue in 8 pieces (per 16-channel half nt: combine + ReLU of
      // rows 0-1, of rows 2-3, bf16 hi / lo split, LDS stores); lane: channels
      // 32 cp + 16 nt + 4 g .. + 3 of pixel p -> y1 hi / lo planes
      float ev[2][4];
      uint32_t eh[2][2], el[2][2];
      auto epi_piece = [&](int k, int j, const f32x4* acc, const f32x4* accl) {
        const int nt = k >> 2, part = k & 3;
        if (part < 2) {
#pragma unroll
          for (int r = 2 * part; r < 2 * part + 2; ++r)
            ev[nt][r] = SPLIT ? fmaxf(fmaf(accl[nt][r], 1.f / CF_LO_SCALE, acc[nt][r]), 0.f) : fmaxf(acc[nt][r], 0.f);
        } else if (part == 2) {
          if (SPLIT) {
            split_pk_bf16_s(ev[nt][0], ev[nt][1], eh[nt][0], el[nt][0]);
            split_pk_bf16_s(ev[nt][2], ev[nt][3], eh[nt][1], el[nt][1]);
          } else {
            eh[nt][0] = cvt_pk_bf16(ev[nt][0], ev[nt][1]);
            eh[nt][1] = cvt_pk_bf16(ev[nt][2], ev[nt][3]);
          }
        } else {
          const int p = 16 * (th + 2 * j) + pl, oh = p / 20, ow = p - 20 * oh;
          const int P = (j == 12 && p >= 400) ? 400 + (pl & 7) : cf_pix(oh, ow);
          const int ch = 32 * cp + 16 * nt + 4 * g;
          const int off = cf_off(P, ch >> 3) + (ch & 7) * 2;
          *reinterpret_cast<uint2*>(Y1 + off) = make_uint2(eh[nt][0], eh[nt][1]);
          if (SPLIT) *reinterpret_cast<uint2*>(Y1 + CF_PLANE + off) = make_uint2(el[nt][0], el[nt][1]);
        }
      };
      auto cvt = [&](const uint2 v) {
        return __builtin_bit_cast(f16x8, u8x8_to_f16off(v.x, v.y));
      };
      // tile j's 2C K steps (4 MFMAs each); step s2 + 1's fragment conversion and 8 / 2C
      // epilogue pieces of tile j - 1 (pj >= 0) go between them, one scheduling region
      // per step, so the vector work rides in the MFMAs' free issue slots
      auto mfma_tile = [&](const uint2* u, f32x4* acc, f32x4* accl, int pj, const f32x4* pacc,
                           const f32x4* paccl) {
        f16x8 av[2];
        av[0] = cvt(u[0]);
#pragma unroll
        for (int s2 = 0; s2 < 2 * C; ++s2) {
          if (s2 + 1 < 2 * C) av[(s2 + 1) & 1] = cvt(u[s2 + 1]);
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1h[nt][s2], av[s2 & 1], s2 ? acc[nt] : bias1[nt], 0, 0, 0);
            if (SPLIT)
              accl[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1l[nt][s2], av[s2 & 1],
                                                                s2 ? accl[nt] : (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          }
          if (pj >= 0) {
#pragma unroll
            for (int k = s2 * 8 / (2 * C); k < (s2 + 1) * 8 / (2 * C); ++k) epi_piece(k, pj, pacc, paccl);
          }
#pragma unroll
          for (int q = 0; q < (SPLIT ? 4 : 2); ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, SPLIT ? 3 : 5, 0);    // VALU
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      uint2 u[2][2 * C];
      f32x4 a[2][2], al[2][2];
      load_tile(0, u[0]);
      load_tile(1, u[1]);
      __builtin_amdgcn_sched_barrier(0);
      mfma_tile(u[0], a[0], al[0], -1, nullptr, nullptr);
#pragma unroll
      for (int j = 1; j < 13; ++j) {
        if (j + 1 < 13) load_tile(j + 1, u[(j + 1) & 1]);     // tile j - 1's registers
        // image i + 1's frames -> staging((i + 1) & 1), one 1-KB DMA per tile among the
        // MFMAs (that buffer's last readers -- conv1(i - 1), the reduction of image i - 1
        // -- finished before the barrier that closed image i - 1)
        if (j - 1 < NDW && more) issue_dma_piece(nsl, (i + 1) & 1, j - 1);
        if (i > 0) store_y2(j - 1);                           // image i - 1's y2
        __builtin_amdgcn_sched_barrier(0);
        mfma_tile(u[j & 1], a[j & 1], al[j & 1], j - 1, a[(j - 1) & 1], al[(j - 1) & 1]);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) epi_piece(k, 12, a[0], al[0]);
    }
    PROBE(d.probe, 4, i, 1);
    // image i + 1's frames (DMA pieces at tiles 1 .. NDW, each before that tile's y2 store)
    // have landed: only the y2 stores of tiles NDW .. 12 are younger than the last piece
    static_assert(NDW <= 7, "the vmcnt below assumes the last DMA piece at tile <= 7");
    if (i > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(cf_young_stores(NDW, SPLIT)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();          // y1 complete; staging(i) read (free: the reduction's); staging(i + 1) visible
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
      auto store_chunk = [&](const int r, const uint4 v) {
        const int k = tq + CF_THREADS * r;
        const int plane = k >= 3200 ? 1 : 0, kk = k - plane * 3200;
        const int P = kk >> 3, c = cst ^ ((P >> 1) & 7);      // the chunk stored at slot cst
        const int cls = P / 100, q = P - cls * 100, a = q / 10, b = q - a * 10;
        const int ih = 2 * a + (cls >> 1), iw = 2 * b + (cls & 1);
        *reinterpret_cast<uint4*>((plane ? d.y1_lo : d.y1) + (int64_t)img * 25600 + (ih * 20 + iw) * 64 + c * 8) = v;
      };
      // (bf16: 3200 chunks of one plane = 12 full rounds + half a round)
      constexpr int NR = SPLIT ? 25 : 12, NB = SPLIT ? 5 : 4;
#pragma unroll
      for (int r0 = 0; r0 < NR; r0 += NB) {
        uint4 v[NB];
#pragma unroll
        for (int r = 0; r < NB; ++r)
          v[r] = *reinterpret_cast<const uint4*>(
              Y1 + (r0 + r) * 4096 + tq * 16 +
              ((SPLIT && (r0 + r > 12 || (r0 + r == 12 && tq >= 128))) ? CF_PLANE - 51200 : 0));    // lo plane
#pragma unroll
        for (int r = 0; r < NB; ++r) store_chunk(r0 + r, v[r]);
      }
      if (!SPLIT && tq < 128) store_chunk(12, *reinterpret_cast<const uint4*>(Y1 + 12 * 4096 + tq * 16));
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
        if (SPLIT) wl[s] = __builtin_bit_cast(bf16x8, wf[C2F_FRAGS + s * 64]);
      }
      bf16x8 ah[2][3], al[2][3];
#define CF_LDA(s_, buf_)                                                                     \
      _Pragma("unroll") for (int mt = 0; mt < 3; ++mt) {                                     \
        const int P_ = (((s_) >> 4) * 2 + (((s_) >> 2) & 1)) * 100 + q0[mt] + (((s_) >> 3) & 1); \
        const int o_ = cf_off(P_, (((s_) & 3) << 1) | kg);                                   \
        ah[buf_][mt] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(Y1 + o_)); \
        if (SPLIT) al[buf_][mt] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(Y1 + CF_PLANE + o_)); \
      }
      CF_LDA(0, 0)
#pragma unroll
      for (int s = 0; s < 32; ++s) {
        if (s + CF_WAHEAD < 32) {
          wh[(s + CF_WAHEAD) % (CF_WAHEAD + 1)] = __builtin_bit_cast(bf16x8, wf[(s + CF_WAHEAD) * 64]);
          if (SPLIT)
            wl[(s + CF_WAHEAD) % (CF_WAHEAD + 1)] = __builtin_bit_cast(bf16x8, wf[C2F_FRAGS + (s + CF_WAHEAD) * 64]);
        }
        if (s + 1 < 32) CF_LDA(s + 1, (s + 1) & 1)
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 bh = wh[s % (CF_WAHEAD + 1)], bl = wl[s % (CF_WAHEAD + 1)];
#pragma unroll
        for (int mt = 0; mt < 3; ++mt) {
          if (SPLIT) {
            acc2[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bl, ah[s & 1][mt], acc2[mt], 0, 0, 0);
            acc2[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh, al[s & 1][mt], acc2[mt], 0, 0, 0);
          }
          acc2[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh, ah[s & 1][mt], acc2[mt], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#undef CF_LDA
    }
    PROBE(d.probe, 4, i, 3);
    if (d.w3 != nullptr && CF_W3EARLY) conv3_prefetch(set);   // (latency hidden behind conv2's epilogue)
    // the two kernel-row pairs meet in LDS (staging(i), read by conv1(i) before the barrier
    // above): wave (nh, kp) finishes output channels 32 nh + 16 kp .. + 15 (jq = 2 kp,
    // 2 kp + 1) and hands the other half of its partial sums to its partner;
    // sum = (bias + pair 0) + pair 1 in both waves (fixed order)
    float4* red = reinterpret_cast<float4*>(STG + (i & 1) * STGB);
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
    __syncthreads();          // partials visible; every read of y1 is done
    // (read before the closing barrier: thread 0 rewrites it at the next image's start)
    const int nn = __builtin_amdgcn_readfirstlane(reinterpret_cast<volatile int*>(&q_img)[0]);
    // acc2[mt][4 jq + i] = D[channel 32 nh + 8 jq + 4 kg + i][pixel mt * 32 + rr]
    auto finish = [&](const int jq0, const bool own_first) {
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) {
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
          uint32_t h01, l01 = 0, h23, l23 = 0;
          if (SPLIT) {
            split_pk_bf16(v0, v1, h01, l01);
            split_pk_bf16(v2, v3, h23, l23);
          } else {
            h01 = cvt_pk_bf16(v0, v1);
            h23 = cvt_pk_bf16(v2, v3);
          }
          pend[mt][jh] = make_uint4(h01, h23, l01, l23);
        }
      }
    };
    if (kp == 0) finish(0, true);        // (bias + own pair 0) + pair 1
    else finish(2, false);               // (bias + pair 0) + own pair 1
    pend_img = img;
    __syncthreads();          // the partials are read: staging(i) may take image i + 2's frames
    if (d.w3 != nullptr) conv3_image(img, set, STG + (i & 1) * STGB, i);
    cur = nxt;
    nxt = nn;
  }
  if (pend_img >= 0) {
#pragma unroll
    for (int q = 0; q < 12; ++q) store_y2(q);   // the last image's y2
  }
  PROBE(d.probe, 4, PROBE_ITERS - 1, 1);          // every store issued (diagnostic build)
#ifdef APEX_PROBE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (d.probe != nullptr && blockIdx.x < PROBE_BLOCKS && (threadIdx.x & 63) == 0)
    d.probe[((blockIdx.x * 4 + (threadIdx.x >> 6)) * PROBE_ITERS + PROBE_ITERS - 1) * 4 + 3] =
        __builtin_amdgcn_s_memrealtime();
#endif
}

static int cf_launch_pack(const Conv12Desc& d, hipStream_t st) {
  const int sets = d.pack_sets & ((d.w1b != nullptr) ? 3 : 1);
  if (sets == 0) return 0;
  const bool s0 = sets & 1, s1 = (sets & 2) != 0;
  const bool c3 = d.w3 != nullptr && d.w3frag != nullptr;
  CfPack pk{C2fPack{{s0 ? d.w2 : nullptr, s0 ? d.w2_lo : nullptr, s1 ? d.w2b : nullptr, s1 ? d.w2b_lo : nullptr},
                    d.wfrag, 0},
            (s1 ? 4 : 2) * C2F_FRAGS / 256,
            C3fPack{{c3 && s0 ? d.w3 : nullptr, c3 && s0 ? d.w3_lo : nullptr, c3 && s1 ? d.w3b : nullptr,
                     c3 && s1 ? d.w3b_lo : nullptr}, d.w3frag},
            c3 ? (s1 ? 4 : 2) * C3F_FRAGS / 256 : 0,
            sets, {d.w1, d.w1b}, {d.b1, d.b1b}, d.in_scale, d.w1frag};
  const int nb = pk.nc2f + pk.nc3f + 4 * (s0 + s1);
  switch (d.C) {
    case 1: cf_pack_kernel<1><<<nb, 256, 0, st>>>(pk); break;
    case 2: cf_pack_kernel<2><<<nb, 256, 0, st>>>(pk); break;
    case 4: cf_pack_kernel<4><<<nb, 256, 0, st>>>(pk); break;
    default: return (int)hipErrorInvalidValue;
  }
  return 0;
}

// pack only (the learner's target sync): d.pack_sets of d's weights
APEX_EXPORT int apex_conv12_pack(Conv12Desc d, hipStream_t st) {
  const bool sp = d.bf16 == 0;
  if (d.w1 == nullptr || d.b1 == nullptr || d.w2 == nullptr || (sp && d.w2_lo == nullptr) || d.wfrag == nullptr ||
      d.w1frag == nullptr || ((d.pack_sets & 2) && (d.w1b == nullptr || d.b1b == nullptr || d.w2b == nullptr ||
                                                   (sp && d.w2b_lo == nullptr))))
    return (int)hipErrorInvalidValue;
  return cf_launch_pack(d, st);
}

APEX_EXPORT int apex_conv12_fused_fwd(Conv12Desc d, int grid, hipStream_t st) {
  if (d.N < 1) return 0;
  const bool sp = d.bf16 == 0;
  if (d.ring == nullptr || d.slots == nullptr || d.w1 == nullptr || d.b1 == nullptr || d.w2 == nullptr ||
      (sp && d.w2_lo == nullptr) || d.b2 == nullptr || d.y2 == nullptr || (sp && d.y2_lo == nullptr) ||
      d.wfrag == nullptr || d.scratch == nullptr || d.w1frag == nullptr)
    return (int)hipErrorInvalidValue;
  const bool two = d.w1b != nullptr;
  if (two && (d.b1b == nullptr || d.w2b == nullptr || (sp && d.w2b_lo == nullptr) || d.b2b == nullptr))
    return (int)hipErrorInvalidValue;
  if (d.copy_n > 0 && (d.y1 == nullptr || (sp && d.y1_lo == nullptr) || d.copy_n > d.N))
    return (int)hipErrorInvalidValue;
  if (d.w3 != nullptr &&
      (d.b3 == nullptr || d.y3 == nullptr || d.w3frag == nullptr || ((uintptr_t)d.w3frag & 15) || (sp && (d.w3_lo == nullptr || d.y3_lo == nullptr)) ||
       (two && (d.w3b == nullptr || d.b3b == nullptr || (sp && d.w3b_lo == nullptr))) ||
       (((uintptr_t)d.w3 | (uintptr_t)(sp ? d.w3_lo : d.w3) | (uintptr_t)(two ? d.w3b : d.w3) |
         (uintptr_t)(two && sp ? d.w3b_lo : d.w3) | (uintptr_t)d.b3 | (uintptr_t)(two ? d.b3b : d.b3)) & 15) ||
       (((uintptr_t)d.y3 | (uintptr_t)(sp ? d.y3_lo : d.y3)) & 7)))
    return (int)hipErrorInvalidValue;
  if ((((uintptr_t)d.w1 | (uintptr_t)(two ? d.w1b : d.w1) | (uintptr_t)d.b1 | (uintptr_t)(two ? d.b1b : d.b1) |
        (uintptr_t)d.w2 | (uintptr_t)d.w2_lo | (uintptr_t)d.b2 | (uintptr_t)d.y1 | (uintptr_t)d.y1_lo) & 15) ||
      (((uintptr_t)d.y2 | (uintptr_t)d.y2_lo | (uintptr_t)d.scratch) & 7) || ((uintptr_t)d.wfrag & 15))
    return (int)hipErrorInvalidValue;
  int G = grid > 0 ? grid : 256;
  if (G > d.N) G = d.N;
  if ((d.N + G - 1) / G > CF_MAXIMG) G = (d.N + CF_MAXIMG - 1) / CF_MAXIMG;
  const int err = cf_launch_pack(d, st);
  if (err) return err;
  switch (d.C * 2 + (sp ? 1 : 0)) {
    case 3: conv12_fused_kernel<1, true><<<G, CF_THREADS, 0, st>>>(d); break;
    case 5: conv12_fused_kernel<2, true><<<G, CF_THREADS, 0, st>>>(d); break;
    case 9: conv12_fused_kernel<4, true><<<G, CF_THREADS, 0, st>>>(d); break;
    case 2: conv12_fused_kernel<1, false><<<G, CF_THREADS, 0, st>>>(d); break;
    case 4: conv12_fused_kernel<2, false><<<G, CF_THREADS, 0, st>>>(d); break;
    case 8: conv12_fused_kernel<4, false><<<G, CF_THREADS, 0, st>>>(d); break;
    default: return (int)hipErrorInvalidValue;
  }
  APEX_CHECK_LAUNCH();
}

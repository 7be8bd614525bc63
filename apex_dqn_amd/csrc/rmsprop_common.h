// Centered RMSprop + global-norm clip + bf16 pack as a block-level device body
// (rmsprop_body), shared by csrc/optimizer.hip (rmsprop_kernel) and by
// csrc/sumtree.hip (rmsprop_sample_kernel: the optimizer launch also draws the
// next step's prioritized batch in its first blocks).
#pragma once
#include "apex_common.h"
#include "cf_pack.h"

// Batch-max IS-weight normalisation (Runtime.is_normalise = "batch_max"): the head
// kernel leaves m = max_j (p_j / p_min)^-beta over the batch (DP: one per rank, in the
// all-gathered shard statistics, stride `wstride`); the loss used the global-min
// weights w_j, so the batch-max weights w_j / m give the gradient g / m -- one scalar
// applied here, before the clip, instead of a second pass over the weights.
__device__ __forceinline__ float is_grad_scale(const double* wnorm, int wn, int wstride) {
  if (wnorm == nullptr) return 1.0f;
  double m = 0.0;
  for (int k = 0; k < wn; ++k) m = fmax(m, wnorm[(int64_t)k * wstride]);
  return m > 0.0 ? (float)(1.0 / m) : 1.0f;
}

// Clip coefficient from the squared-norm partials: every thread of the block sums a
// fixed strided subset, then a fixed-order wave / LDS reduction -- deterministic.
// `gscale` multiplies the gradient first (is_grad_scale); the returned coefficient
// includes it and sh[1] is the norm of the scaled gradient.
// `gpre` (n_pre floats, 16-B aligned, or null): a short gradient range whose squares every
// block sums itself, in the same fixed thread-strided order (the data-parallel step's conv1
// bucket, all-reduced right before this launch: no separate norm launch on the critical
// path, learner/dp_step.py).
__device__ __forceinline__ float clip_coef_from_partials(const double* partials, int npart, float clip,
                                                         float* sh, float gscale = 1.0f,
                                                         const float* gpre = nullptr, int64_t npre = 0) {
  __shared__ double red[16];
  double s = 0.0;
  if (gpre != nullptr) {
    const float4* g4 = reinterpret_cast<const float4*>(gpre);
    const int64_t n4 = npre / 4;
    for (int64_t i = threadIdx.x; i < n4; i += blockDim.x) {
      const float4 v = g4[i];
      s += (double)(v.x * v.x + v.y * v.y) + (double)(v.z * v.z + v.w * v.w);
    }
    for (int64_t i = n4 * 4 + threadIdx.x; i < npre; i += blockDim.x) s += (double)gpre[i] * gpre[i];
  }
  for (int i = threadIdx.x; i < npart; i += blockDim.x) s += partials[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    const float norm = (float)sqrt(t) * gscale;
    sh[0] = gscale * ((clip > 0.f) ? fminf(1.0f, clip / (norm + 1e-6f)) : 1.0f);
    sh[1] = norm;
  }
  __syncthreads();
  return sh[0];
}

struct RmspropArgs {
  float* p;
  const float* g;
  float* v;
  float* m;
  bf16_t* pb;
  int64_t n;
  const double* partials;
  int npart;
  float lr, alpha, eps, clip;
  int centered;
  float* norm_out;
  bf16_t* pb_lo;     // fp32-accurate mode: lo plane of the bf16 copy (p = pb + pb_lo), else null
  const double* wnorm;  // batch-max IS normalisation (is_grad_scale), or null
  int wn, wstride;
  CfFragOut fo;         // the fused forward's online operands in fragment order (w1frag null: off)
  const float* gpre;    // clip norm: a gradient range summed in every block (clip_coef_from_partials), or null
  int64_t npre;
};

// one block `bid` of `nblk` (grid-stride over float4 chunks)
__device__ __forceinline__ void rmsprop_body(const RmspropArgs& A_, int bid, int nblk) {
  // no FMA contraction: every inlined copy of the update (steady loop, peeled chunk, the
  // other launches) rounds identically
#pragma clang fp contract(off)
  float* __restrict__ p = A_.p;
  const float* __restrict__ g = A_.g;
  float* __restrict__ v = A_.v;
  float* __restrict__ m = A_.m;
  bf16_t* __restrict__ pb = A_.pb;
  bf16_t* __restrict__ pbl = A_.pb_lo;
  const int64_t n = A_.n;
  const float lr = A_.lr, alpha = A_.alpha, eps = A_.eps;
  const int centered = A_.centered;
  __shared__ float sh[2];
  const int64_t n4 = n / 4;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* v4 = reinterpret_cast<float4*>(v);
  float4* m4 = reinterpret_cast<float4*>(m);
  uint2* pb4 = reinterpret_cast<uint2*>(pb);
  uint2* pbl4 = reinterpret_cast<uint2*>(pbl);
  const int64_t stride = (int64_t)nblk * blockDim.x;
  int64_t i = (int64_t)bid * blockDim.x + threadIdx.x;
  // the first chunk's loads are in flight while the block sums the clip-norm
  // partials, and every iteration prefetches the next chunk (one-deep pipeline)
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 gg = z4, pp = z4, vv = z4, mm = z4;
  if (i < n4) {
    gg = g4[i]; pp = p4[i]; vv = v4[i];
    if (centered) mm = m4[i];
  }
  const float coef = clip_coef_from_partials(A_.partials, A_.npart, A_.clip, sh,
                                             is_grad_scale(A_.wnorm, A_.wn, A_.wstride), A_.gpre, A_.npre);
  if (bid == 0 && threadIdx.x == 0 && A_.norm_out) A_.norm_out[0] = sh[1];
  const float a1 = 1.0f - alpha;
  auto update = [&](int64_t i, const float4 gg, const float4 pp, const float4 vv, const float4 mm, const bool frag) {
    float gx[4] = {gg.x * coef, gg.y * coef, gg.z * coef, gg.w * coef};
    float px[4] = {pp.x, pp.y, pp.z, pp.w};
    float vx[4] = {vv.x, vv.y, vv.z, vv.w};
    float mx[4] = {mm.x, mm.y, mm.z, mm.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      vx[j] = alpha * vx[j] + a1 * gx[j] * gx[j];
      float var = vx[j];
      if (centered) {
        mx[j] = alpha * mx[j] + a1 * gx[j];
        var = vx[j] - mx[j] * mx[j];
      }
      px[j] -= lr * gx[j] / (sqrtf(fmaxf(var, 0.f)) + eps);
    }
    p4[i] = make_float4(px[0], px[1], px[2], px[3]);
    v4[i] = make_float4(vx[0], vx[1], vx[2], vx[3]);
    if (centered) m4[i] = make_float4(mx[0], mx[1], mx[2], mx[3]);
    if (pbl != nullptr) {
      uint32_t h01, l01, h23, l23;
      split_pk_bf16_h(px[0], px[1], h01, l01);
      split_pk_bf16_h(px[2], px[3], h23, l23);
      pb4[i] = make_uint2(h01, h23);
      pbl4[i] = make_uint2(l01, l23);
      if (frag) cf_frag_store(A_.fo, 4 * i, px, make_uint2(h01, h23), make_uint2(l01, l23));
    } else {
      const uint2 hb = make_uint2(pack_bf16x2(px[0], px[1]), pack_bf16x2(px[2], px[3]));
      pb4[i] = hb;
      if (frag) cf_frag_store(A_.fo, 4 * i, px, hb, make_uint2(0u, 0u));
    }
  };
  // The first chunk is peeled: the fused forward's operand stores (A_.fo, the launcher
  // checks that w1 / w2 lie within every thread's first chunk) run before the next
  // chunk's loads are issued, so the steady loop keeps 6 waves per SIMD (every block of
  // the launch resident at once; with the stores inside the loop it held 85 VGPRs)
  if (i < n4) {
    update(i, gg, pp, vv, mm, A_.fo.w1frag != nullptr);
    i += stride;
    if (i < n4) {
      gg = g4[i]; pp = p4[i]; vv = v4[i];
      if (centered) mm = m4[i];
    }
  }
  for (; i < n4; i += stride) {
    const int64_t inx = i + stride;
    float4 gn = z4, pn = z4, vn = z4, mn = z4;
    if (inx < n4) {
      gn = g4[inx]; pn = p4[inx]; vn = v4[inx];
      if (centered) mn = m4[inx];
    }
    update(i, gg, pp, vv, mm, false);
    gg = gn; pp = pn; vv = vn; mm = mn;
  }
  for (int64_t i = n4 * 4 + (int64_t)bid * blockDim.x + threadIdx.x; i < n; i += (int64_t)nblk * blockDim.x) {
    float gg = g[i] * coef;
    float vv = alpha * v[i] + a1 * gg * gg, var = vv;
    v[i] = vv;
    if (centered) {
      float mm = alpha * m[i] + a1 * gg;
      m[i] = mm;
      var = vv - mm * mm;
    }
    float pp = p[i] - lr * gg / (sqrtf(fmaxf(var, 0.f)) + eps);
    p[i] = pp;
    pb[i] = f32_to_bf16(pp);
    if (pbl != nullptr) pbl[i] = f32_to_bf16(pp - bf16_to_f32(pb[i]));
  }
}

// Fused dueling heads + n-step double-DQN target + Huber/IS loss + priorities
// + head backward.  One block of three waves per sample: each wave evaluates
// one 2*HS-wide activation row (online S_t, online S_t+n, target S_t+n; HS =
// stream width, 512 for the NatureCNN, 256 for IMPALA) and
// the q-values meet in LDS; wave 0 finishes loss, priority and backward.
//
// Covers reference duelling_network.py:18-19,25-27 (value/advantage heads and
// the dueling combine, with the per-sample advantage mean instead of the
// batch-global sum, defect A15) and learner.py:43-50 (DDQN target from the
// online argmax and the target net's value, TD error, loss, priorities) plus
// the loss gradient back to the 1024-wide stream activations -- work that the
// reference spreads over ~20 separate torch ops.
//
// Inputs (per sample b of the local batch B):
//   Hon  [2B,1024] bf16  online stream activations (post-ReLU): rows [0,B) = S_t,
//                        rows [B,2B) = S_{t+n}; cols [0,512) value, [512,1024) adv
//   Htg  [B,1024]  bf16  target-network stream activations for S_{t+n}
//   head params fp32: wv[512] bv[1] wa[A,512] ba[A] (online, target)
//   act int32, rew/gam/isw fp32
// Outputs: td_abs[B], loss[B], q_t[B,A] (optional), dH[B,1024] bf16 (gradient
// at the pre-ReLU stream outputs), dhead[B,1+A] fp32 (d value, d advantage).
#include "apex_common.h"

#define HEAD_MAXA 32

struct HeadParams {
  const float* wv;
  const float* bv;
  const float* wa;
  const float* ba;
};

// NPL consecutive fp32 weights (16-B aligned: NPL is 4 or 8) as float4 loads
template <int NPL>
__device__ __forceinline__ void load_w(const float* __restrict__ p, float* w) {
#pragma unroll
  for (int k = 0; k < NPL; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(p + k);
    w[k] = v.x; w[k + 1] = v.y; w[k + 2] = v.z; w[k + 3] = v.w;
  }
}

// bf16 elements k of a packed row chunk (k < 2 * dwords)
__device__ __forceinline__ float bf16_at(const uint32_t* u, int k) {
  return __uint_as_float((k & 1) ? (u[k >> 1] & 0xffff0000u) : (u[k >> 1] << 16));
}

// q-values of one 2*HS-wide activation row (HS = stream width: 512 NatureCNN, 256
// IMPALA): lane holds cols lane*NPL..+NPL-1 of each stream, NPL = HS / 64
template <int HS>
__device__ __forceinline__ void head_row(const bf16_t* __restrict__ row, const HeadParams& P, int A,
                                         int lane, float* q, float* hv, float* ha) {
  constexpr int NPL = HS / 64;
  uint32_t wv_[NPL / 2], wa_[NPL / 2];
  if constexpr (NPL == 8) {
    const uint4 rv = *reinterpret_cast<const uint4*>(row + lane * 8);
    const uint4 ra = *reinterpret_cast<const uint4*>(row + HS + lane * 8);
    wv_[0] = rv.x; wv_[1] = rv.y; wv_[2] = rv.z; wv_[3] = rv.w;
    wa_[0] = ra.x; wa_[1] = ra.y; wa_[2] = ra.z; wa_[3] = ra.w;
  } else {
    const uint2 rv = *reinterpret_cast<const uint2*>(row + lane * 4);
    const uint2 ra = *reinterpret_cast<const uint2*>(row + HS + lane * 4);
    wv_[0] = rv.x; wv_[1] = rv.y;
    wa_[0] = ra.x; wa_[1] = ra.y;
  }
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    hv[k] = bf16_at(wv_, k);
    ha[k] = bf16_at(wa_, k);
  }
  float part[HEAD_MAXA + 1];
  {
    float w[NPL], s = 0.f;
    load_w<NPL>(P.wv + lane * NPL, w);
#pragma unroll
    for (int k = 0; k < NPL; ++k) s += hv[k] * w[k];
    part[0] = s;
  }
#pragma unroll
  for (int j = 0; j < HEAD_MAXA; ++j) {
    if (j < A) {
      float w[NPL], s = 0.f;
      load_w<NPL>(P.wa + j * HS + lane * NPL, w);
#pragma unroll
      for (int k = 0; k < NPL; ++k) s += ha[k] * w[k];
      part[j + 1] = s;
    } else {
      part[j + 1] = 0.f;
    }
  }
  float v = wave_sum_dpp(part[0]) + P.bv[0];
  float amean = 0.f;
#pragma unroll
  for (int j = 0; j < HEAD_MAXA; ++j) {
    if (j < A) {
      float a = wave_sum_dpp(part[j + 1]) + P.ba[j];
      part[j + 1] = a;
      amean += a;
    }
  }
  amean /= (float)A;
#pragma unroll
  for (int j = 0; j < HEAD_MAXA; ++j)
    if (j < A) q[j] = v + part[j + 1] - amean;
}

template <int HS>
__global__ void __launch_bounds__(192) ddqn_head_kernel(
    const bf16_t* __restrict__ Hon, const bf16_t* __restrict__ Htg, HeadParams Pon, HeadParams Ptg,
    const int32_t* __restrict__ act, const float* __restrict__ rew, const float* __restrict__ gam,
    const float* __restrict__ isw, int B, int A, int huber, float kappa, float grad_scale,
    float* __restrict__ td_abs, float* __restrict__ loss, float* __restrict__ q_out,
    bf16_t* __restrict__ dH, float* __restrict__ dhead, float* __restrict__ zero_ptr, int zero_n) {
  __shared__ float qs[2][HEAD_MAXA];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.x;
  // zero the head-gradient region that head_wgrad accumulates into (stream-ordered)
  if (zero_ptr != nullptr) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < zero_n; i += gridDim.x * blockDim.x) zero_ptr[i] = 0.f;
  }
  constexpr int NPL = HS / 64, ROW = 2 * HS;
  float q_t[HEAD_MAXA], q_n[HEAD_MAXA], q_g[HEAD_MAXA];
  float hv_t[NPL], ha_t[NPL];
  if (wv == 0) {
    head_row<HS>(Hon + (int64_t)b * ROW, Pon, A, lane, q_t, hv_t, ha_t);
  } else {
    float hv_x[NPL], ha_x[NPL], q[HEAD_MAXA];
    if (wv == 1) head_row<HS>(Hon + (int64_t)(B + b) * ROW, Pon, A, lane, q, hv_x, ha_x);
    else head_row<HS>(Htg + (int64_t)b * ROW, Ptg, A, lane, q, hv_x, ha_x);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < HEAD_MAXA; ++j)
        if (j < A) qs[wv - 1][j] = q[j];
    }
  }
  __syncthreads();
  if (wv != 0) return;
#pragma unroll
  for (int j = 0; j < HEAD_MAXA; ++j) {
    q_n[j] = j < A ? qs[0][j] : 0.f;
    q_g[j] = j < A ? qs[1][j] : 0.f;
  }
  // double DQN: argmax from the online net, value from the target net
  int astar = 0;
  float best = -3.4e38f, qg_star = 0.f, q_sa = 0.f;
  const int a_b = act[b];
#pragma unroll
  for (int j = 0; j < HEAD_MAXA; ++j) {
    if (j < A) {
      if (q_n[j] > best) { best = q_n[j]; astar = j; qg_star = q_g[j]; }
      if (j == a_b) q_sa = q_t[j];
    }
  }
  (void)astar;
  const float G = rew[b] + gam[b] * qg_star;
  const float delta = G - q_sa;
  const float ad = fabsf(delta);
  float l, dl;
  if (huber && ad > kappa) {
    l = kappa * (ad - 0.5f * kappa);
    dl = delta > 0.f ? kappa : -kappa;
  } else {
    l = 0.5f * delta * delta;
    dl = delta;
  }
  const float w = isw ? isw[b] : 1.0f;
  // d loss_mean / d q(S_t, a_b) = -w * dl / B  (grad_scale = 1/B)
  const float dq = -w * dl * grad_scale;
  if (lane == 0) {
    td_abs[b] = ad;
    loss[b] = w * l;
    dhead[(int64_t)b * (A + 1)] = dq;
  }
  if (q_out != nullptr && lane < A) {
    float qv = 0.f;
#pragma unroll
    for (int j = 0; j < HEAD_MAXA; ++j)
      if (j == lane) qv = q_t[j];
    q_out[(int64_t)b * A + lane] = qv;
  }
  const float invA = 1.0f / (float)A;
  if (lane < A) dhead[(int64_t)b * (A + 1) + 1 + lane] = dq * ((lane == a_b ? 1.f : 0.f) - invA);
  // back through the heads and the stream ReLUs
  float dv[NPL], da[NPL], wvv[NPL];
  load_w<NPL>(Pon.wv + lane * NPL, wvv);
#pragma unroll
  for (int k = 0; k < NPL; ++k) dv[k] = hv_t[k] > 0.f ? dq * wvv[k] : 0.f;
  float colsum[NPL], wsel[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) { colsum[k] = 0.f; wsel[k] = 0.f; }
  for (int j = 0; j < A; ++j) {
    float wr[NPL];
    load_w<NPL>(Pon.wa + j * HS + lane * NPL, wr);
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const float ww = wr[k];
      colsum[k] += ww;
      if (j == a_b) wsel[k] = ww;
    }
  }
#pragma unroll
  for (int k = 0; k < NPL; ++k) da[k] = ha_t[k] > 0.f ? dq * (wsel[k] - colsum[k] * invA) : 0.f;
  if constexpr (NPL == 8) {
    const uint4 ov = make_uint4(pack_bf16x2(dv[0], dv[1]), pack_bf16x2(dv[2], dv[3]), pack_bf16x2(dv[4], dv[5]),
                                pack_bf16x2(dv[6], dv[7]));
    const uint4 oa = make_uint4(pack_bf16x2(da[0], da[1]), pack_bf16x2(da[2], da[3]), pack_bf16x2(da[4], da[5]),
                                pack_bf16x2(da[6], da[7]));
    *reinterpret_cast<uint4*>(dH + (int64_t)b * ROW + lane * 8) = ov;
    *reinterpret_cast<uint4*>(dH + (int64_t)b * ROW + HS + lane * 8) = oa;
  } else {
    *reinterpret_cast<uint2*>(dH + (int64_t)b * ROW + lane * 4) =
        make_uint2(pack_bf16x2(dv[0], dv[1]), pack_bf16x2(dv[2], dv[3]));
    *reinterpret_cast<uint2*>(dH + (int64_t)b * ROW + HS + lane * 4) =
        make_uint2(pack_bf16x2(da[0], da[1]), pack_bf16x2(da[2], da[3]));
  }
}

// head weight/bias gradients: dW[j][k] += sum_b dhead[b][j] * h[b][stream(j)][k]
// grid: (A+1) rows x HS/256 column blocks x batch slices of 16; fp32 atomics into a
// region zeroed by ddqn_head_kernel.  Output layout = flat param layout:
//   gwv[HS] gbv[1] gwa[A*HS] gba[A]
__global__ void __launch_bounds__(256) head_wgrad_kernel(const bf16_t* __restrict__ Hon,
                                                         const float* __restrict__ dhead, int B, int A,
                                                         float* __restrict__ gwv, float* __restrict__ gbv,
                                                         float* __restrict__ gwa, float* __restrict__ gba, int HS) {
  const int j = blockIdx.x;            // 0 = value, 1..A = advantage j-1
  const int k = blockIdx.y * 256 + threadIdx.x;  // 0..HS-1
  const int b0 = blockIdx.z * 16;
  const int b1 = min(B, b0 + 16);
  const int col = (j == 0 ? 0 : HS) + k;
  float acc = 0.f, accb = 0.f;
  for (int b = b0; b < b1; ++b) {
    const float d = dhead[(int64_t)b * (A + 1) + j];
    acc += d * bf16_to_f32(Hon[(int64_t)b * 2 * HS + col]);
    accb += d;
  }
  if (j == 0) {
    atomicAdd(&gwv[k], acc);
    if (k == 0 && blockIdx.y == 0) atomicAdd(gbv, accb);
  } else {
    atomicAdd(&gwa[(j - 1) * HS + k], acc);
    if (k == 0 && blockIdx.y == 0) atomicAdd(&gba[j - 1], accb);
  }
}

APEX_EXPORT int apex_ddqn_head(const bf16_t* Hon, const bf16_t* Htg, HeadParams Pon, HeadParams Ptg,
                               const int32_t* act, const float* rew, const float* gam, const float* isw,
                               int B, int A, int huber, float kappa, float grad_scale, float* td_abs,
                               float* loss, float* q_out, bf16_t* dH, float* dhead, float* zero_ptr,
                               int zero_n, int hidden, hipStream_t st) {
  if (A < 1 || A > HEAD_MAXA || B < 1) return (int)hipErrorInvalidValue;
  if (hidden == 512)
    ddqn_head_kernel<512><<<B, 192, 0, st>>>(Hon, Htg, Pon, Ptg, act, rew, gam, isw, B, A, huber, kappa, grad_scale,
                                             td_abs, loss, q_out, dH, dhead, zero_ptr, zero_n);
  else if (hidden == 256)
    ddqn_head_kernel<256><<<B, 192, 0, st>>>(Hon, Htg, Pon, Ptg, act, rew, gam, isw, B, A, huber, kappa, grad_scale,
                                             td_abs, loss, q_out, dH, dhead, zero_ptr, zero_n);
  else
    return (int)hipErrorInvalidValue;
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_head_wgrad(const bf16_t* Hon, const float* dhead, int B, int A, float* gwv, float* gbv,
                                float* gwa, float* gba, int hidden, hipStream_t st) {
  if (hidden != 512 && hidden != 256) return (int)hipErrorInvalidValue;
  dim3 grid(A + 1, hidden / 256, (B + 15) / 16);
  head_wgrad_kernel<<<grid, 256, 0, st>>>(Hon, dhead, B, A, gwv, gbv, gwa, gba, hidden);
  APEX_CHECK_LAUNCH();
}

// Actor-side: dueling q from stream activations + epsilon-greedy selection.
// One wave per env row. eps per row; uniform draws from the counter RNG.
template <int HS>
__global__ void __launch_bounds__(256) actor_head_kernel(const bf16_t* __restrict__ H, HeadParams P, int E,
                                                         int A, const float* __restrict__ eps, uint64_t seed,
                                                         const uint64_t* __restrict__ ctr,
                                                         float* __restrict__ q_out, int32_t* __restrict__ a_out) {
  const int lane = threadIdx.x & 63;
  const int e = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (e >= E) return;
  float q[HEAD_MAXA], hv[HS / 64], ha[HS / 64];
  head_row<HS>(H + (int64_t)e * 2 * HS, P, A, lane, q, hv, ha);
  int best = 0;
  float bq = -3.4e38f;
#pragma unroll
  for (int j = 0; j < HEAD_MAXA; ++j)
    if (j < A && q[j] > bq) { bq = q[j]; best = j; }
  if (lane < A) {
    float qv = 0.f;
#pragma unroll
    for (int j = 0; j < HEAD_MAXA; ++j)
      if (j == lane) qv = q[j];
    q_out[(int64_t)e * A + lane] = qv;
  }
  if (lane == 0) {
    const uint64_t c = ctr ? ctr[0] : 0;
    float u = apex_uniform(seed, c, 2 * (uint64_t)e);
    float r = apex_uniform(seed, c, 2 * (uint64_t)e + 1);
    int a = best;
    if (u < eps[e]) a = min((int)(r * (float)A), A - 1);
    a_out[e] = a;
  }
}

APEX_EXPORT int apex_actor_head(const bf16_t* H, HeadParams P, int E, int A, const float* eps, uint64_t seed,
                                const uint64_t* ctr, float* q_out, int32_t* a_out, int hidden, hipStream_t st) {
  if (A < 1 || A > HEAD_MAXA || E < 1) return (int)hipErrorInvalidValue;
  if (hidden == 512) actor_head_kernel<512><<<(E + 3) / 4, 256, 0, st>>>(H, P, E, A, eps, seed, ctr, q_out, a_out);
  else if (hidden == 256) actor_head_kernel<256><<<(E + 3) / 4, 256, 0, st>>>(H, P, E, A, eps, seed, ctr, q_out, a_out);
  else return (int)hipErrorInvalidValue;
  APEX_CHECK_LAUNCH();
}

// Fused dueling heads + n-step double-DQN target + Huber/IS loss + priorities
// + head backward.  One block of three waves per sample: each wave evaluates
// one 1024-wide activation row (online S_t, online S_t+n, target S_t+n) and
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

// q-values of one 1024-wide activation row: lane holds cols lane*8..+7 of each stream
__device__ __forceinline__ void head_row(const bf16_t* __restrict__ row, const HeadParams& P, int A,
                                         int lane, float* q, float hv[8], float ha[8]) {
  const uint4 rv = *reinterpret_cast<const uint4*>(row + lane * 8);
  const uint4 ra = *reinterpret_cast<const uint4*>(row + 512 + lane * 8);
  const uint32_t wv_[4] = {rv.x, rv.y, rv.z, rv.w};
  const uint32_t wa_[4] = {ra.x, ra.y, ra.z, ra.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    hv[2 * j] = __uint_as_float(wv_[j] << 16);
    hv[2 * j + 1] = __uint_as_float(wv_[j] & 0xffff0000u);
    ha[2 * j] = __uint_as_float(wa_[j] << 16);
    ha[2 * j + 1] = __uint_as_float(wa_[j] & 0xffff0000u);
  }
  float part[HEAD_MAXA + 1];
  {
    const float4 w0 = *reinterpret_cast<const float4*>(P.wv + lane * 8);
    const float4 w1 = *reinterpret_cast<const float4*>(P.wv + lane * 8 + 4);
    part[0] = hv[0] * w0.x + hv[1] * w0.y + hv[2] * w0.z + hv[3] * w0.w + hv[4] * w1.x + hv[5] * w1.y +
              hv[6] * w1.z + hv[7] * w1.w;
  }
#pragma unroll
  for (int j = 0; j < HEAD_MAXA; ++j) {
    if (j < A) {
      const float* w = P.wa + j * 512 + lane * 8;
      const float4 w0 = *reinterpret_cast<const float4*>(w);
      const float4 w1 = *reinterpret_cast<const float4*>(w + 4);
      part[j + 1] = ha[0] * w0.x + ha[1] * w0.y + ha[2] * w0.z + ha[3] * w0.w + ha[4] * w1.x +
                    ha[5] * w1.y + ha[6] * w1.z + ha[7] * w1.w;
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
  float q_t[HEAD_MAXA], q_n[HEAD_MAXA], q_g[HEAD_MAXA];
  float hv_t[8], ha_t[8];
  if (wv == 0) {
    head_row(Hon + (int64_t)b * 1024, Pon, A, lane, q_t, hv_t, ha_t);
  } else {
    float hv_x[8], ha_x[8], q[HEAD_MAXA];
    if (wv == 1) head_row(Hon + (int64_t)(B + b) * 1024, Pon, A, lane, q, hv_x, ha_x);
    else head_row(Htg + (int64_t)b * 1024, Ptg, A, lane, q, hv_x, ha_x);
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
  float dv[8], da[8];
  {
    const float4 w0 = *reinterpret_cast<const float4*>(Pon.wv + lane * 8);
    const float4 w1 = *reinterpret_cast<const float4*>(Pon.wv + lane * 8 + 4);
    const float wvv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) dv[k] = hv_t[k] > 0.f ? dq * wvv[k] : 0.f;
  }
  float colsum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, wsel[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < A; ++j) {
    const float* wr = Pon.wa + j * 512 + lane * 8;
    const float4 w0 = *reinterpret_cast<const float4*>(wr);
    const float4 w1 = *reinterpret_cast<const float4*>(wr + 4);
    const float ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      colsum[k] += ww[k];
      if (j == a_b) wsel[k] = ww[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) da[k] = ha_t[k] > 0.f ? dq * (wsel[k] - colsum[k] * invA) : 0.f;
  uint4 ov = make_uint4(pack_bf16x2(dv[0], dv[1]), pack_bf16x2(dv[2], dv[3]), pack_bf16x2(dv[4], dv[5]),
                        pack_bf16x2(dv[6], dv[7]));
  uint4 oa = make_uint4(pack_bf16x2(da[0], da[1]), pack_bf16x2(da[2], da[3]), pack_bf16x2(da[4], da[5]),
                        pack_bf16x2(da[6], da[7]));
  *reinterpret_cast<uint4*>(dH + (int64_t)b * 1024 + lane * 8) = ov;
  *reinterpret_cast<uint4*>(dH + (int64_t)b * 1024 + 512 + lane * 8) = oa;
}

// head weight/bias gradients: dW[j][k] += sum_b dhead[b][j] * h[b][stream(j)][k]
// grid: (A+1) rows x 2 column halves x batch slices of 16; fp32 atomics into a
// region zeroed by ddqn_head_kernel.  Output layout = flat param layout:
//   gwv[512] gbv[1] gwa[A*512] gba[A]
__global__ void __launch_bounds__(256) head_wgrad_kernel(const bf16_t* __restrict__ Hon,
                                                         const float* __restrict__ dhead, int B, int A,
                                                         float* __restrict__ gwv, float* __restrict__ gbv,
                                                         float* __restrict__ gwa, float* __restrict__ gba) {
  const int j = blockIdx.x;            // 0 = value, 1..A = advantage j-1
  const int k = blockIdx.y * 256 + threadIdx.x;  // 0..511
  const int b0 = blockIdx.z * 16;
  const int b1 = min(B, b0 + 16);
  const int col = (j == 0 ? 0 : 512) + k;
  float acc = 0.f, accb = 0.f;
  for (int b = b0; b < b1; ++b) {
    const float d = dhead[(int64_t)b * (A + 1) + j];
    acc += d * bf16_to_f32(Hon[(int64_t)b * 1024 + col]);
    accb += d;
  }
  if (j == 0) {
    atomicAdd(&gwv[k], acc);
    if (k == 0 && blockIdx.y == 0) atomicAdd(gbv, accb);
  } else {
    atomicAdd(&gwa[(j - 1) * 512 + k], acc);
    if (k == 0 && blockIdx.y == 0) atomicAdd(&gba[j - 1], accb);
  }
}

APEX_EXPORT int apex_ddqn_head(const bf16_t* Hon, const bf16_t* Htg, HeadParams Pon, HeadParams Ptg,
                               const int32_t* act, const float* rew, const float* gam, const float* isw,
                               int B, int A, int huber, float kappa, float grad_scale, float* td_abs,
                               float* loss, float* q_out, bf16_t* dH, float* dhead, float* zero_ptr,
                               int zero_n, hipStream_t st) {
  if (A < 1 || A > HEAD_MAXA || B < 1) return (int)hipErrorInvalidValue;
  ddqn_head_kernel<<<B, 192, 0, st>>>(Hon, Htg, Pon, Ptg, act, rew, gam, isw, B, A,
                                                            huber, kappa, grad_scale, td_abs, loss, q_out,
                                                            dH, dhead, zero_ptr, zero_n);
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_head_wgrad(const bf16_t* Hon, const float* dhead, int B, int A, float* gwv, float* gbv,
                                float* gwa, float* gba, hipStream_t st) {
  dim3 grid(A + 1, 2, (B + 15) / 16);
  head_wgrad_kernel<<<grid, 256, 0, st>>>(Hon, dhead, B, A, gwv, gbv, gwa, gba);
  APEX_CHECK_LAUNCH();
}

// Actor-side: dueling q from stream activations + epsilon-greedy selection.
// One wave per env row. eps per row; uniform draws from the counter RNG.
__global__ void __launch_bounds__(256) actor_head_kernel(const bf16_t* __restrict__ H, HeadParams P, int E,
                                                         int A, const float* __restrict__ eps, uint64_t seed,
                                                         const uint64_t* __restrict__ ctr,
                                                         float* __restrict__ q_out, int32_t* __restrict__ a_out) {
  const int lane = threadIdx.x & 63;
  const int e = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (e >= E) return;
  float q[HEAD_MAXA], hv[8], ha[8];
  head_row(H + (int64_t)e * 1024, P, A, lane, q, hv, ha);
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
                                const uint64_t* ctr, float* q_out, int32_t* a_out, hipStream_t st) {
  if (A < 1 || A > HEAD_MAXA || E < 1) return (int)hipErrorInvalidValue;
  actor_head_kernel<<<(E + 3) / 4, 256, 0, st>>>(H, P, E, A, eps, seed, ctr, q_out, a_out);
  APEX_CHECK_LAUNCH();
}

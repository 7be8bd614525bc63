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
#include "head_common.h"
#include "conv2_wfrag.h"

// Batch-max IS normalisation (Runtime.is_normalise = "batch_max"): block 0's second
// wave also leaves m = max_b isw[b] / wscale -- the largest (p / p_min)^-beta of the
// batch, the sampler's W B / M factor taken out -- for the optimizer, which scales the
// gradient by 1 / m (csrc/rmsprop_common.h is_grad_scale).  With DP `out` is this
// rank's slot of the shard statistics that are all-gathered later in the step.
struct IsNorm {
  const float* wscale;   // sampler's W B / M (null: 1)
  double* out;           // null: off
  unsigned long long* valid_count;   // DP: += rows of this batch the rank drew (weight > 0); or null
};

// hp.part != null: the fc forward's split-K epilogue runs inside (head_common.h
// load_row_part); blocks >= B run the conv2 weight-fragment pack job (pk.out != null)
// that otherwise rides on that epilogue's launch.
template <int HS, int MAXA>
__global__ void __launch_bounds__(192) ddqn_head_kernel(
    const bf16_t* __restrict__ Hon, const bf16_t* __restrict__ Htg, HeadParams Pon, HeadParams Ptg,
    const int32_t* __restrict__ act, const float* __restrict__ rew, const float* __restrict__ gam,
    const float* __restrict__ isw, int B, int A, int huber, float kappa, float grad_scale,
    float* __restrict__ td_abs, float* __restrict__ loss, float* __restrict__ q_out,
    bf16_t* __restrict__ dH, float* __restrict__ dhead, float* __restrict__ zero_ptr, int zero_n, HeadLo lo,
    HeadPart hp, C2dPackJob pk, IsNorm isn) {
  if ((int)blockIdx.x >= B) {
    for (int i = ((int)blockIdx.x - B) * 192 + (int)threadIdx.x; i < C2D_PACK_THREADS; i += ((int)gridDim.x - B) * 192)
      pack_c2d_wfrag_word(i, pk.w, pk.w_lo, pk.out);
    return;
  }
  float ad;
  const bool w0 = ddqn_head_body<HS, MAXA>(Hon, Htg, Pon, Ptg, act, rew, gam, isw, B, A, huber, kappa, grad_scale, td_abs,
                                     loss, q_out, dH, dhead, zero_ptr, zero_n, &ad, lo, hp);
  if (!w0 && (isn.out != nullptr || isn.valid_count != nullptr) && blockIdx.x == 0 && (threadIdx.x >> 6) == 1) {
    float m = 0.f;
    int nv = 0;
    for (int i = threadIdx.x & 63; i < B; i += 64) {
      m = fmaxf(m, isw[i]);
      nv += isw[i] > 0.f ? 1 : 0;
    }
    m = wave_max(m);
    nv = wave_sum(nv);
    if ((threadIdx.x & 63) == 0) {
      const float ws = isn.wscale != nullptr ? isn.wscale[0] : 1.f;
      if (isn.out != nullptr) isn.out[0] = ws > 0.f ? (double)m / (double)ws : 0.0;
      if (isn.valid_count != nullptr) atomicAdd(isn.valid_count, (unsigned long long)nv);
    }
  }
}

__global__ void __launch_bounds__(512) head_wgrad_kernel(HeadWgArgs h) { head_wgrad_body(h, blockIdx.x, blockIdx.y); }

APEX_EXPORT int apex_ddqn_head(const bf16_t* Hon, const bf16_t* Htg, HeadParams Pon, HeadParams Ptg,
                               const int32_t* act, const float* rew, const float* gam, const float* isw,
                               int B, int A, int huber, float kappa, float grad_scale, float* td_abs,
                               float* loss, float* q_out, bf16_t* dH, float* dhead, float* zero_ptr,
                               int zero_n, int hidden, HeadLo lo, HeadPart hp, C2dPackJob pk, IsNorm isn,
                               hipStream_t st) {
  if (A < 1 || A > HEAD_MAXA || B < 1) return (int)hipErrorInvalidValue;
  if ((isn.out != nullptr || isn.valid_count != nullptr) && isw == nullptr) return (int)hipErrorInvalidValue;
  if (lo.Hon != nullptr && (lo.Htg == nullptr || lo.dH == nullptr)) return (int)hipErrorInvalidValue;
  if (hp.part != nullptr) {   // split-K partials [nz][3B][2 hidden]; rows [0, B) of h written to hp.hon
    if (hp.nz < 1 || hp.hon == nullptr || hp.bias_on == nullptr || hp.bias_tg == nullptr || hp.two_b != 2 * B ||
        (lo.Hon != nullptr) != (hp.hon_lo != nullptr) || (((uintptr_t)hp.part | (uintptr_t)hp.hon) & 15))
      return (int)hipErrorInvalidValue;
  }
  if (pk.out != nullptr && (pk.w == nullptr || ((uintptr_t)pk.out & 15))) return (int)hipErrorInvalidValue;
  const int grid = B + (pk.out != nullptr ? 128 : 0);
#define APEX_HEAD_LAUNCH(HS_, MA_)                                                                              \
  ddqn_head_kernel<HS_, MA_><<<grid, 192, 0, st>>>(Hon, Htg, Pon, Ptg, act, rew, gam, isw, B, A, huber, kappa,     \
                                                   grad_scale, td_abs, loss, q_out, dH, dhead, zero_ptr, zero_n, lo, \
                                                   hp, pk, isn)
  // the q arrays in registers: 8 actions (every ALE minimal action set but the full
  // 18) keep the kernel free of scratch
  if (hidden == 512 && A <= 8) APEX_HEAD_LAUNCH(512, 8);
  else if (hidden == 512) APEX_HEAD_LAUNCH(512, HEAD_MAXA);
  else if (hidden == 256 && A <= 8) APEX_HEAD_LAUNCH(256, 8);
  else if (hidden == 256) APEX_HEAD_LAUNCH(256, HEAD_MAXA);
  else
    return (int)hipErrorInvalidValue;
#undef APEX_HEAD_LAUNCH
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_head_wgrad(const bf16_t* Hon, const float* dhead, int B, int A, float* gwv, float* gbv,
                                float* gwa, float* gba, int hidden, const bf16_t* Hon_lo, hipStream_t st) {
  if (hidden != 512 && hidden != 256) return (int)hipErrorInvalidValue;
  dim3 grid(A + 1, hidden / 64);
  head_wgrad_kernel<<<grid, 512, 0, st>>>(HeadWgArgs{Hon, dhead, B, A, gwv, gbv, gwa, gba, hidden, Hon_lo});
  APEX_CHECK_LAUNCH();
}

// Actor-side: dueling q from stream activations + epsilon-greedy selection.
// One wave per env row. eps per row; uniform draws from the counter RNG.
// H_lo (fp32 learner, split mode): the lo plane of the stream activations, so the
// actor's q-values (and the initial priorities built from them) are fp32-accurate.
template <int HS, int MAXA>
__global__ void __launch_bounds__(256) actor_head_kernel(const bf16_t* __restrict__ H, HeadParams P, int E,
                                                         int A, const float* __restrict__ eps, uint64_t seed,
                                                         const uint64_t* __restrict__ ctr,
                                                         float* __restrict__ q_out, int32_t* __restrict__ a_out,
                                                         const bf16_t* __restrict__ H_lo) {
  const int lane = threadIdx.x & 63;
  const int e = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (e >= E) return;
  float q[MAXA], hv[HS / 64], ha[HS / 64];
  head_row<HS, MAXA>(H + (int64_t)e * 2 * HS, H_lo != nullptr ? H_lo + (int64_t)e * 2 * HS : nullptr, P, A, lane, q,
                     hv, ha);
  int best = 0;
  float bq = -3.4e38f;
#pragma unroll
  for (int j = 0; j < MAXA; ++j)
    if (j < A && q[j] > bq) { bq = q[j]; best = j; }
  if (lane < A) {
    float qv = 0.f;
#pragma unroll
    for (int j = 0; j < MAXA; ++j)
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
                                const uint64_t* ctr, float* q_out, int32_t* a_out, int hidden, const bf16_t* H_lo,
                                hipStream_t st) {
  if (A < 1 || A > HEAD_MAXA || E < 1) return (int)hipErrorInvalidValue;
#define APEX_ACTOR_HEAD(HS_, MA_) \
  actor_head_kernel<HS_, MA_><<<(E + 3) / 4, 256, 0, st>>>(H, P, E, A, eps, seed, ctr, q_out, a_out, H_lo)
  if (hidden == 512 && A <= 8) APEX_ACTOR_HEAD(512, 8);
  else if (hidden == 512) APEX_ACTOR_HEAD(512, HEAD_MAXA);
  else if (hidden == 256 && A <= 8) APEX_ACTOR_HEAD(256, 8);
  else if (hidden == 256) APEX_ACTOR_HEAD(256, HEAD_MAXA);
  else return (int)hipErrorInvalidValue;
#undef APEX_ACTOR_HEAD
  APEX_CHECK_LAUNCH();
}

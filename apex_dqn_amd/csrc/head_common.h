// Device code shared by the dueling-head kernels: the q-values of one activation
// row (head_row) and the fused DDQN loss / priority / head-backward body
// (ddqn_head_body), used by csrc/ddqn_head.hip (ddqn_head_kernel), and the head
// weight gradient (head_wgrad_body, run by csrc/sumtree.hip head_wgrad_prio_kernel
// and fc_wgrad_head_prio_kernel beside the priority write-back).
#pragma once
#include "apex_common.h"

#define HEAD_MAXA 32

struct HeadParams {
  const float* wv;
  const float* bv;
  const float* wa;
  const float* ba;
};

// fp32-accurate ("split") mode: lo planes of the stream activations (online,
// target) and of the stream gradient dH; all null in bf16 mode
struct HeadLo {
  const bf16_t* Hon;
  const bf16_t* Htg;
  bf16_t* dH;
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
// NPL bf16 of each stream of one row -> fp32 (lane's columns)
template <int HS>
__device__ __forceinline__ void load_row_streams(const bf16_t* __restrict__ row, int lane, float* hv, float* ha) {
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
}

// q-values of one row; `row_lo` (split mode, else null) adds the lo plane: the
// activations are then fp32-accurate (hi + lo)
// MAXA: compile-time bound on the action count (the q arrays live in registers; the
// launchers pick 8 when A <= 8, else HEAD_MAXA).  KEEP: also leave the weights the head
// backward needs (wave 0 of ddqn_head_body) -- wv, the column sums of wa and wa's row
// for action a_sel -- so the backward issues no second round of weight loads.
template <int HS, int MAXA = HEAD_MAXA, bool KEEP = false>
__device__ __forceinline__ void head_q(const HeadParams& P, int A, int lane, float* q, const float* hv,
                                       const float* ha, float* kwv = nullptr, float* kcs = nullptr,
                                       float* kws = nullptr, int a_sel = 0);

template <int HS, int MAXA = HEAD_MAXA>
__device__ __forceinline__ void head_row(const bf16_t* __restrict__ row, const bf16_t* __restrict__ row_lo,
                                         const HeadParams& P, int A, int lane, float* q, float* hv, float* ha) {
  constexpr int NPL = HS / 64;
  load_row_streams<HS>(row, lane, hv, ha);
  if (row_lo != nullptr) {
    float lv[NPL], la[NPL];
    load_row_streams<HS>(row_lo, lane, lv, la);
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      hv[k] += lv[k];
      ha[k] += la[k];
    }
  }
  head_q<HS, MAXA>(P, A, lane, q, hv, ha);
}

// The fc forward's split-K epilogue fused into the head (csrc/conv_mfma.hip
// fc_gemm128_kernel leaves fp32 partials [nz][3B][2 HS]): a wave builds its row from
// the partials exactly as fc_splitk_epilogue_kernel would (z-ordered sum, + bias,
// ReLU, bf16 or hi / lo rounding) and uses the rounded values, so the step is
// bit-identical to the two-launch path; wave 0 stores its S_t row for the head
// weight gradient.  Saves the epilogue launch and its 19 MB pass over h.
struct HeadPart {
  const float* part;      // null: the head reads h (Hon / Htg) as usual
  int64_t zstride;        // floats between partial planes
  int nz;
  const float* bias_on;   // fc bias of rows < two_b (online), of rows >= two_b (target)
  const float* bias_tg;
  int two_b;
  bf16_t* hon;            // rows [0, B) of h written back (hi plane / bf16)
  bf16_t* hon_lo;         // split mode: lo plane (else null)
};

template <int HS>
__device__ __forceinline__ void load_row_part(const HeadPart& hp, int row, int lane, float* hv, float* ha,
                                              bool store) {
  // Every load of a group of ZU partial planes (both streams) is issued before any of
  // them is summed -- at a small per-rank batch the fc forward runs ~10 K splits and a
  // plane-by-plane loop paid one memory round trip per plane -- and the sum keeps the
  // z order of fc_splitk_epilogue_kernel (bit-identical).
  constexpr int NPL = HS / 64, ROW = 2 * HS, ZU = 4;
  const bool split = hp.hon_lo != nullptr;
  const float* __restrict__ bias = row < hp.two_b ? hp.bias_on : hp.bias_tg;
  float v[2][NPL], bs[2][NPL];
  const float* p0 = hp.part + (int64_t)row * ROW + lane * NPL;
  const int nzs[2] = {hp.nz, hp.nz};
  const int nzmax = hp.nz;
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int k = 0; k < NPL; k += 4) {
      const float4 a = *reinterpret_cast<const float4*>(p0 + st * HS + k);
      const float4 b = *reinterpret_cast<const float4*>(bias + st * HS + lane * NPL + k);
      v[st][k] = a.x; v[st][k + 1] = a.y; v[st][k + 2] = a.z; v[st][k + 3] = a.w;
      bs[st][k] = b.x; bs[st][k + 1] = b.y; bs[st][k + 2] = b.z; bs[st][k + 3] = b.w;
    }
  for (int z0 = 1; z0 < nzmax; z0 += ZU) {
    float4 t[ZU][2][NPL / 4];
#pragma unroll
    for (int u = 0; u < ZU; ++u)
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int k = 0; k < NPL / 4; ++k)
          t[u][st][k] = z0 + u < nzs[st]
                            ? *reinterpret_cast<const float4*>(p0 + (int64_t)(z0 + u) * hp.zstride + st * HS + 4 * k)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < ZU; ++u)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        if (z0 + u >= nzs[st]) continue;      // (no +0.0: keeps a -0.0 sum bit-exact)
#pragma unroll
        for (int k = 0; k < NPL / 4; ++k) {
          v[st][4 * k] += t[u][st][k].x; v[st][4 * k + 1] += t[u][st][k].y;
          v[st][4 * k + 2] += t[u][st][k].z; v[st][4 * k + 3] += t[u][st][k].w;
        }
      }
  }
#pragma unroll
  for (int st = 0; st < 2; ++st) {       // value stream, advantage stream
    const int c0 = st * HS + lane * NPL;
    uint32_t hh[NPL / 2], ll[NPL / 2];
#pragma unroll
    for (int k = 0; k < NPL; ++k) v[st][k] = v[st][k] * 1.0f + bs[st][k];
#pragma unroll
    for (int k = 0; k < NPL / 2; ++k) {
      // fc_splitk_epilogue_kernel: ReLU in fp32, then the (hi / lo) bf16 rounding
      if (split) {
        split_pk_bf16_h(fmaxf(v[st][2 * k], 0.f), fmaxf(v[st][2 * k + 1], 0.f), hh[k], ll[k]);
      } else {
        hh[k] = pack_bf16x2(fmaxf(v[st][2 * k], 0.f), fmaxf(v[st][2 * k + 1], 0.f));
        ll[k] = 0;
      }
    }
    // (no pointer select between hv / ha: that put both arrays in scratch)
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const float x = bf16_at(hh, k) + (split ? bf16_at(ll, k) : 0.f);
      if (st) ha[k] = x;
      else hv[k] = x;
    }
    if (store) {
      bf16_t* o = hp.hon + (int64_t)row * ROW + c0;
      if constexpr (NPL == 8) {
        *reinterpret_cast<uint4*>(o) = make_uint4(hh[0], hh[1], hh[2], hh[3]);
        if (split) *reinterpret_cast<uint4*>(hp.hon_lo + (int64_t)row * ROW + c0) = make_uint4(ll[0], ll[1], ll[2], ll[3]);
      } else {
        *reinterpret_cast<uint2*>(o) = make_uint2(hh[0], hh[1]);
        if (split) *reinterpret_cast<uint2*>(hp.hon_lo + (int64_t)row * ROW + c0) = make_uint2(ll[0], ll[1]);
      }
    }
  }
}

template <int HS, int MAXA, bool KEEP>
__device__ __forceinline__ void head_q(const HeadParams& P, int A, int lane, float* q, const float* hv,
                                       const float* ha, float* kwv, float* kcs, float* kws, int a_sel) {
  constexpr int NPL = HS / 64;
  float part[MAXA + 1];
  // every weight row of the heads is loaded before the first product (MAXA <= 8: 9 x NPL
  // registers): issued one row at a time, each row's load waited for before the next --
  // one memory round trip per action
  constexpr bool PRE = MAXA <= 8;
  float wpre[PRE ? MAXA : 1][NPL];
  float bpre[PRE ? MAXA : 1];           // the advantage biases, with the weights
  float w0[NPL];
  load_w<NPL>(P.wv + lane * NPL, w0);
  const float bv = P.bv[0];
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < MAXA; ++j) {
      if (j < A) {
        load_w<NPL>(P.wa + j * HS + lane * NPL, wpre[j]);
        bpre[j] = P.ba[j];
      } else {
        bpre[j] = 0.f;
#pragma unroll
        for (int k = 0; k < NPL; ++k) wpre[j][k] = 0.f;
      }
    }
  }
  {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NPL; ++k) s += hv[k] * w0[k];
    part[0] = s;
    if constexpr (KEEP) {
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        kwv[k] = w0[k];
        kcs[k] = 0.f;
        kws[k] = 0.f;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < MAXA; ++j) {
    if (j < A) {
      float w[NPL], s = 0.f;
      if constexpr (PRE) {
#pragma unroll
        for (int k = 0; k < NPL; ++k) w[k] = wpre[j][k];
      } else {
        load_w<NPL>(P.wa + j * HS + lane * NPL, w);
      }
#pragma unroll
      for (int k = 0; k < NPL; ++k) s += ha[k] * w[k];
      part[j + 1] = s;
      if constexpr (KEEP) {
#pragma unroll
        for (int k = 0; k < NPL; ++k) {
          kcs[k] += w[k];
          if (j == a_sel) kws[k] = w[k];
        }
      }
    } else {
      part[j + 1] = 0.f;
    }
  }
  float v = wave_sum_dpp(part[0]) + bv;
  float amean = 0.f;
#pragma unroll
  for (int j = 0; j < MAXA; ++j) {
    if (j < A) {
      float a = wave_sum_dpp(part[j + 1]) + (PRE ? bpre[PRE ? j : 0] : P.ba[j]);
      part[j + 1] = a;
      amean += a;
    }
  }
  amean /= (float)A;
#pragma unroll
  for (int j = 0; j < MAXA; ++j)
    if (j < A) q[j] = v + part[j + 1] - amean;
}

// One block of three waves per sample (blockIdx.x = b).  Returns true in wave 0,
// which finishes the sample and holds |delta| (wave-uniform) in *ad_out.
template <int HS, int MAXA = HEAD_MAXA>
__device__ __forceinline__ bool ddqn_head_body(
    const bf16_t* __restrict__ Hon, const bf16_t* __restrict__ Htg, HeadParams Pon, HeadParams Ptg,
    const int32_t* __restrict__ act, const float* __restrict__ rew, const float* __restrict__ gam,
    const float* __restrict__ isw, int B, int A, int huber, float kappa, float grad_scale,
    float* __restrict__ td_abs, float* __restrict__ loss, float* __restrict__ q_out,
    bf16_t* __restrict__ dH, float* __restrict__ dhead, float* __restrict__ zero_ptr, int zero_n,
    float* ad_out, HeadLo lo, const HeadPart& hp) {
  __shared__ float qs[2][MAXA];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.x;
  // zero the head-gradient region that head_wgrad accumulates into (stream-ordered)
  if (zero_ptr != nullptr) {   // B blocks (a launch may carry extra side-job blocks)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < zero_n; i += B * blockDim.x) zero_ptr[i] = 0.f;
  }
  constexpr int NPL = HS / 64, ROW = 2 * HS;
  float q_t[MAXA], q_n[MAXA], q_g[MAXA];
  float hv_t[NPL], ha_t[NPL];
  const bool split = lo.Hon != nullptr;
  // the sample's scalars are loaded up front (wave 0 consumes them after the barrier)
  float kwv[NPL], kcs[NPL], kws[NPL];     // kept by head_q for the backward
  int a_b = 0;
  float rew_b = 0.f, gam_b = 0.f, w_b = 1.f;
  if (wv == 0) {
    a_b = act[b];
    rew_b = rew[b];
    gam_b = gam[b];
    if (isw) w_b = isw[b];
    if (hp.part != nullptr) {
      load_row_part<HS>(hp, b, lane, hv_t, ha_t, true);
      head_q<HS, MAXA, true>(Pon, A, lane, q_t, hv_t, ha_t, kwv, kcs, kws, a_b);
    } else {
      const bf16_t* row = Hon + (int64_t)b * ROW;
      load_row_streams<HS>(row, lane, hv_t, ha_t);
      if (split) {
        float lv[NPL], la[NPL];
        load_row_streams<HS>(lo.Hon + (int64_t)b * ROW, lane, lv, la);
#pragma unroll
        for (int k = 0; k < NPL; ++k) {
          hv_t[k] += lv[k];
          ha_t[k] += la[k];
        }
      }
      head_q<HS, MAXA, true>(Pon, A, lane, q_t, hv_t, ha_t, kwv, kcs, kws, a_b);
    }
  } else {
    float hv_x[NPL], ha_x[NPL], q[MAXA];
    if (hp.part != nullptr) {
      load_row_part<HS>(hp, wv == 1 ? B + b : hp.two_b + b, lane, hv_x, ha_x, false);
      head_q<HS, MAXA>(wv == 1 ? Pon : Ptg, A, lane, q, hv_x, ha_x);
    } else if (wv == 1)
      head_row<HS, MAXA>(Hon + (int64_t)(B + b) * ROW, split ? lo.Hon + (int64_t)(B + b) * ROW : nullptr, Pon, A, lane, q,
                   hv_x, ha_x);
    else
      head_row<HS, MAXA>(Htg + (int64_t)b * ROW, split ? lo.Htg + (int64_t)b * ROW : nullptr, Ptg, A, lane, q, hv_x, ha_x);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < MAXA; ++j)
        if (j < A) qs[wv - 1][j] = q[j];
    }
  }
  __syncthreads();
  if (wv != 0) return false;
#pragma unroll
  for (int j = 0; j < MAXA; ++j) {
    q_n[j] = j < A ? qs[0][j] : 0.f;
    q_g[j] = j < A ? qs[1][j] : 0.f;
  }
  // double DQN: argmax from the online net, value from the target net
  int astar = 0;
  float best = -3.4e38f, qg_star = 0.f, q_sa = 0.f;
#pragma unroll
  for (int j = 0; j < MAXA; ++j) {
    if (j < A) {
      if (q_n[j] > best) { best = q_n[j]; astar = j; qg_star = q_g[j]; }
      if (j == a_b) q_sa = q_t[j];
    }
  }
  (void)astar;
  const float G = rew_b + gam_b * qg_star;
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
  const float w = w_b;
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
    for (int j = 0; j < MAXA; ++j)
      if (j == lane) qv = q_t[j];
    q_out[(int64_t)b * A + lane] = qv;
  }
  const float invA = 1.0f / (float)A;
  if (lane < A) dhead[(int64_t)b * (A + 1) + 1 + lane] = dq * ((lane == a_b ? 1.f : 0.f) - invA);
  // back through the heads and the stream ReLUs
  // (wv, wa's column sums and the taken action's row: kept by head_q)
  float dv[NPL], da[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) dv[k] = hv_t[k] > 0.f ? dq * kwv[k] : 0.f;
#pragma unroll
  for (int k = 0; k < NPL; ++k) da[k] = ha_t[k] > 0.f ? dq * (kws[k] - kcs[k] * invA) : 0.f;
  if (split) {
    // fp32 dH -> hi / lo planes (NPL consecutive columns per stream: 2 per dword)
    uint32_t vh[NPL / 2], vl[NPL / 2], ah[NPL / 2], al[NPL / 2];
#pragma unroll
    for (int k = 0; k < NPL / 2; ++k) {
      split_pk_bf16_h(dv[2 * k], dv[2 * k + 1], vh[k], vl[k]);
      split_pk_bf16_h(da[2 * k], da[2 * k + 1], ah[k], al[k]);
    }
    bf16_t* o[2] = {dH + (int64_t)b * ROW, lo.dH + (int64_t)b * ROW};
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
      const uint32_t* V = pl ? vl : vh;
      const uint32_t* Av = pl ? al : ah;
      if constexpr (NPL == 8) {
        *reinterpret_cast<uint4*>(o[pl] + lane * 8) = make_uint4(V[0], V[1], V[2], V[3]);
        *reinterpret_cast<uint4*>(o[pl] + HS + lane * 8) = make_uint4(Av[0], Av[1], Av[2], Av[3]);
      } else {
        *reinterpret_cast<uint2*>(o[pl] + lane * 4) = make_uint2(V[0], V[1]);
        *reinterpret_cast<uint2*>(o[pl] + HS + lane * 4) = make_uint2(Av[0], Av[1]);
      }
    }
  } else if constexpr (NPL == 8) {
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
  *ad_out = ad;
  return true;
}

// head weight/bias gradients: dW[j][k] += sum_b dhead[b][j] * h[b][stream(j)][k]
// grid: (A+1) rows x HS/64 column chunks; block = 8 waves, lane = column, wave w
// sums rows w, w+8, ...; the 8 wave partials meet in LDS and are added in a fixed
// order -- no atomics, so the step is bitwise reproducible.  Output layout = flat
// param layout: gwv[HS] gbv[1] gwa[A*HS] gba[A] (accumulated into, the region is
// zeroed by ddqn_head_kernel).
struct HeadWgArgs {
  const bf16_t* Hon;
  const float* dhead;
  int B, A;
  float* gwv;
  float* gbv;
  float* gwa;
  float* gba;
  int HS;
  const bf16_t* Hon_lo;      // split mode: lo plane of Hon (else null)
};

// block (j, chunk): any multiple of 64 threads up to 1024 (waves split the rows)
__device__ __forceinline__ void head_wgrad_body(const HeadWgArgs& h, int j, int chunk) {
  const bf16_t* __restrict__ Hon = h.Hon;
  const float* __restrict__ dhead = h.dhead;
  const int B = h.B, A = h.A, HS = h.HS;
  __shared__ float red[16][65];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int k = chunk * 64 + lane;  // 0..HS-1
  const int col = (j == 0 ? 0 : HS) + k;
  float acc = 0.f, accb = 0.f;
  const bf16_t* __restrict__ Hlo = h.Hon_lo;
  if (Hlo != nullptr) {
#pragma unroll 8
    for (int b = w; b < B; b += nw) {
      const float d = dhead[(int64_t)b * (A + 1) + j];
      const int64_t o = (int64_t)b * 2 * HS + col;
      acc += d * (bf16_to_f32(Hon[o]) + bf16_to_f32(Hlo[o]));
      accb += d;
    }
  } else {
#pragma unroll 8
    for (int b = w; b < B; b += nw) {
      const float d = dhead[(int64_t)b * (A + 1) + j];
      acc += d * bf16_to_f32(Hon[(int64_t)b * 2 * HS + col]);
      accb += d;
    }
  }
  red[w][lane] = acc;
  if (lane == 0) red[w][64] = accb;
  __syncthreads();
  if (w != 0) return;
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q)
    if (q < nw) s += red[q][lane];
  if (j == 0) h.gwv[k] += s;
  else h.gwa[(j - 1) * HS + k] += s;
  if (lane == 0 && chunk == 0) {
    float sb = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (q < nw) sb += red[q][64];
    if (j == 0) h.gbv[0] += sb;
    else h.gba[j - 1] += sb;
  }
}

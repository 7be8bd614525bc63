// Native host runtime: see host_runtime.h.
#include "host_runtime.h"

#include <cmath>
#include <cstring>
#include <limits>
#include <thread>

APEX_RT_API int apex_rt_version() { return 1; }

// ------------------------------------------------------------------ sum-tree
// Binary sum-tree + min-tree (min over POSITIVE leaves; +inf when none).  The
// updates of one call are applied in order, so a duplicated index keeps its
// LAST value (the rule the HIP 64-ary tree implements with its LDS dedupe).
APEX_RT_API int apex_rt_st_update(double* sum, double* mn, int64_t size2, int64_t capacity, const int64_t* idx,
                                  const double* val, int64_t n) {
  const double inf = std::numeric_limits<double>::infinity();
  for (int64_t i = 0; i < n; ++i)
    if (idx[i] < 0 || idx[i] >= capacity) return -1;
  for (int64_t i = 0; i < n; ++i) {
    int64_t node = size2 + idx[i];
    const double v = val[i];
    sum[node] = v;
    mn[node] = v > 0.0 ? v : inf;
    node >>= 1;
    while (node >= 1) {
      sum[node] = sum[2 * node] + sum[2 * node + 1];
      const double a = mn[2 * node], b = mn[2 * node + 1];
      mn[node] = a < b ? a : b;
      node >>= 1;
    }
  }
  return 0;
}

// smallest leaf i with prefix(i) > u; never descends into an empty subtree
static inline int64_t st_find_one(const double* sum, int64_t size2, int64_t capacity, double u) {
  int64_t node = 1;
  while (node < size2) {
    const int64_t left = 2 * node;
    const double lv = sum[left];
    if (u >= lv && sum[left + 1] > 0.0) {
      u -= lv;
      node = left + 1;
    } else {
      node = left;
    }
  }
  const int64_t leaf = node - size2;
  return leaf < capacity ? leaf : capacity - 1;
}

APEX_RT_API int apex_rt_st_find(const double* sum, int64_t size2, int64_t capacity, const double* u, int64_t n,
                                int64_t* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = st_find_one(sum, size2, capacity, u[i]);
  return 0;
}

// stratified proportional sampling: draw i targets (i + r_i) / batch of the mass
APEX_RT_API int apex_rt_st_sample_stratified(const double* sum, int64_t size2, int64_t capacity, int64_t batch,
                                             const double* r01, int64_t* out) {
  const double total = sum[1];
  if (!(total > 0.0) || batch <= 0) return -1;
  const double seg = total / (double)batch;
  const double top = std::nextafter(total, 0.0);
  for (int64_t i = 0; i < batch; ++i) {
    double u = ((double)i + r01[i]) * seg;
    if (u > top) u = top;
    out[i] = st_find_one(sum, size2, capacity, u);
  }
  return 0;
}

// ------------------------------------------------------------------ CartPole-v1
// Barto, Sutton & Anderson cart-pole with the gym v1 constants and 500-step
// truncation -- the same dynamics as apex_dqn_amd/envs/vector_envs.py:CartPoleVec.
namespace {
constexpr double kGravity = 9.8, kMassCart = 1.0, kMassPole = 0.1, kTotalMass = kMassCart + kMassPole;
constexpr double kLength = 0.5, kPoleMassLength = kMassPole * kLength, kForce = 10.0, kTau = 0.02;
constexpr double kThetaThreshold = 12.0 * 2.0 * M_PI / 360.0, kXThreshold = 2.4;
constexpr int64_t kMaxSteps = 500;

inline uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
inline double uniform(uint64_t& s, double lo, double hi) {
  return lo + (hi - lo) * ((double)(splitmix(s) >> 11) * (1.0 / 9007199254740992.0));
}
inline void reset_one(double* st, int64_t* t, double* ret, uint64_t* rng, int e) {
  for (int k = 0; k < 4; ++k) st[4 * e + k] = uniform(rng[e], -0.05, 0.05);
  t[e] = 0;
  ret[e] = 0.0;
}
}  // namespace

APEX_RT_API void apex_rt_cp_reset(double* state, int64_t* t, double* ep_ret, uint64_t* rng, int E,
                                  const int32_t* mask, float* obs) {
  for (int e = 0; e < E; ++e) {
    if (mask == nullptr || mask[e]) reset_one(state, t, ep_ret, rng, e);
    for (int k = 0; k < 4; ++k) obs[4 * e + k] = (float)state[4 * e + k];
  }
}

APEX_RT_API void apex_rt_cp_step(double* state, int64_t* t, double* ep_ret, uint64_t* rng, int E,
                                 const int64_t* actions, float* obs, float* rew, uint8_t* done, uint8_t* trunc,
                                 double* info_ret, int64_t* info_len) {
  for (int e = 0; e < E; ++e) {
    double* s = state + 4 * e;
    const double x = s[0], x_dot = s[1], th = s[2], th_dot = s[3];
    const double force = actions[e] == 1 ? kForce : -kForce;
    const double c = std::cos(th), sn = std::sin(th);
    const double temp = (force + kPoleMassLength * th_dot * th_dot * sn) / kTotalMass;
    const double th_acc = (kGravity * sn - c * temp) / (kLength * (4.0 / 3.0 - kMassPole * c * c / kTotalMass));
    const double x_acc = temp - kPoleMassLength * th_acc * c / kTotalMass;
    s[0] = x + kTau * x_dot;
    s[1] = x_dot + kTau * x_acc;
    s[2] = th + kTau * th_dot;
    s[3] = th_dot + kTau * th_acc;
    t[e] += 1;
    const bool term = std::fabs(s[0]) > kXThreshold || std::fabs(s[2]) > kThetaThreshold;
    const bool tr = t[e] >= kMaxSteps;
    rew[e] = 1.0f;
    ep_ret[e] += 1.0;
    done[e] = (uint8_t)(term || tr);
    trunc[e] = (uint8_t)(tr && !term);
    if (term || tr) {
      info_ret[e] = ep_ret[e];
      info_len[e] = t[e];
      reset_one(state, t, ep_ret, rng, e);
    } else {
      info_ret[e] = std::numeric_limits<double>::quiet_NaN();
      info_len[e] = -1;
    }
    for (int k = 0; k < 4; ++k) obs[4 * e + k] = (float)s[k];
  }
}

// ------------------------------------------------------------------ seqlock
// Writer: seq -> odd (relaxed) + release fence, copy, seq -> even (release).
// Reader: even seq (acquire), copy, acquire fence, seq unchanged -> consistent.
APEX_RT_API int64_t apex_rt_seqlock_write(uint64_t* seq, void* dst, const void* src, int64_t nbytes) {
  const uint64_t s = __atomic_load_n(seq, __ATOMIC_RELAXED);
  __atomic_store_n(seq, s + 1, __ATOMIC_RELAXED);
  __atomic_thread_fence(__ATOMIC_RELEASE);
  std::memcpy(dst, src, (size_t)nbytes);
  __atomic_store_n(seq, s + 2, __ATOMIC_RELEASE);
  return (int64_t)(s + 2);
}

APEX_RT_API int64_t apex_rt_seqlock_read(const uint64_t* seq, void* dst, const void* src, int64_t nbytes,
                                         int64_t last, int max_tries) {
  for (int i = 0; i < max_tries; ++i) {
    const uint64_t s0 = __atomic_load_n(seq, __ATOMIC_ACQUIRE);
    if ((int64_t)s0 == last) return -2;          // unchanged since the caller's copy
    if (s0 & 1u) {                               // writer active
      std::this_thread::yield();
      continue;
    }
    std::memcpy(dst, src, (size_t)nbytes);
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    if (__atomic_load_n(seq, __ATOMIC_RELAXED) == s0) return (int64_t)s0;
  }
  return -1;
}

// Self-test of the native host runtime, built with -fsanitize=address,undefined
// by tests/test_native_runtime.py (host-side sanitizers; GPU ASan is not
// available on the MI355X pool).  Exercises every entry point, including a
// two-thread seqlock stress that checks no torn snapshot is ever accepted.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../host_runtime.h"

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                    \
    }                                                              \
  } while (0)

static int test_sumtree() {
  const int64_t cap = 1000, size2 = 1024;
  std::vector<double> sum(2 * size2, 0.0), mn(2 * size2, INFINITY);
  std::vector<int64_t> idx(cap);
  std::vector<double> val(cap);
  double ref = 0.0;
  for (int64_t i = 0; i < cap; ++i) {
    idx[i] = i;
    val[i] = 1.0 + (double)(i % 17);
    ref += val[i];
  }
  CHECK(apex_rt_st_update(sum.data(), mn.data(), size2, cap, idx.data(), val.data(), cap) == 0);
  CHECK(std::fabs(sum[1] - ref) < 1e-9);
  CHECK(mn[1] == 1.0);
  // duplicate index: last writer wins
  int64_t di[3] = {5, 5, 5};
  double dv[3] = {100.0, 0.0, 7.0};
  CHECK(apex_rt_st_update(sum.data(), mn.data(), size2, cap, di, dv, 3) == 0);
  CHECK(sum[size2 + 5] == 7.0);
  int64_t bad = cap;
  double bv = 1.0;
  CHECK(apex_rt_st_update(sum.data(), mn.data(), size2, cap, &bad, &bv, 1) == -1);
  std::vector<double> r(256);
  std::vector<int64_t> out(256);
  for (int i = 0; i < 256; ++i) r[i] = (i * 0.618033988749895) - std::floor(i * 0.618033988749895);
  CHECK(apex_rt_st_sample_stratified(sum.data(), size2, cap, 256, r.data(), out.data()) == 0);
  for (int i = 0; i < 256; ++i) CHECK(out[i] >= 0 && out[i] < cap && sum[size2 + out[i]] > 0);
  return 0;
}

static int test_cartpole() {
  const int E = 64;
  std::vector<double> st(4 * E);
  std::vector<int64_t> t(E), act(E), ilen(E);
  std::vector<double> ret(E), iret(E);
  std::vector<uint64_t> rng(E);
  for (int e = 0; e < E; ++e) rng[e] = 12345 + e;
  std::vector<float> obs(4 * E), rew(E);
  std::vector<uint8_t> done(E), trunc(E);
  apex_rt_cp_reset(st.data(), t.data(), ret.data(), rng.data(), E, nullptr, obs.data());
  int episodes = 0;
  for (int k = 0; k < 2000; ++k) {
    for (int e = 0; e < E; ++e) act[e] = (k + e) & 1;
    apex_rt_cp_step(st.data(), t.data(), ret.data(), rng.data(), E, act.data(), obs.data(), rew.data(), done.data(),
                    trunc.data(), iret.data(), ilen.data());
    for (int e = 0; e < E; ++e) {
      CHECK(rew[e] == 1.0f);
      if (done[e]) {
        ++episodes;
        CHECK(ilen[e] >= 1 && ilen[e] <= 500 && iret[e] == (double)ilen[e]);
        CHECK(t[e] == 0);
      }
    }
  }
  CHECK(episodes > 0);
  return 0;
}

static int test_seqlock() {
  const int n = 4096;
  std::vector<float> shared(n, 0.0f), src(n), dst(n);
  uint64_t seq = 0;
  std::atomic<bool> stop{false};
  std::thread writer([&] {
    for (int v = 1; v <= 3000; ++v) {
      for (int i = 0; i < n; ++i) src[i] = (float)v;
      apex_rt_seqlock_write(&seq, shared.data(), src.data(), n * sizeof(float));
    }
    stop = true;
  });
  int64_t last = -1;
  int reads = 0;
  while (!stop.load()) {
    const int64_t v = apex_rt_seqlock_read(&seq, dst.data(), shared.data(), n * sizeof(float), last, 64);
    if (v >= 0) {
      for (int i = 1; i < n; ++i) CHECK(dst[i] == dst[0]);   // never a torn snapshot
      CHECK(v % 2 == 0);
      last = v;
      ++reads;
    }
  }
  writer.join();
  CHECK(apex_rt_seqlock_read(&seq, dst.data(), shared.data(), n * sizeof(float), -1, 4) == 6000);
  CHECK(dst[0] == 3000.0f && dst[n - 1] == 3000.0f);
  CHECK(apex_rt_seqlock_read(&seq, dst.data(), shared.data(), n * sizeof(float), 6000, 4) == -2);
  (void)reads;
  return 0;
}

// n-step builder: random episode ends, partial and full takes; every emitted
// transition's discount is gamma^n or 0 and the buffers drain to empty
static int test_nstep() {
  const int E = 9, A = 4, n = 3;
  void* h = apex_rt_ns_create(E, n, 0.99, 4 * sizeof(int64_t), 5);
  CHECK(h != nullptr);
  CHECK(apex_rt_ns_create(0, n, 0.99, 8, 0) == nullptr);
  std::vector<int64_t> obs(E * 4), nxt(E * 4), act(E);
  std::vector<float> q(E * A), rew(E);
  std::vector<uint8_t> done(E);
  uint64_t x = 0x1234567ull;
  auto rnd = [&]() { x = x * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(x >> 33); };
  int64_t total = 0;
  for (int t = 0; t < 500; ++t) {
    for (int e = 0; e < E; ++e) {
      for (int c = 0; c < 4; ++c) nxt[e * 4 + c] = rnd();
      for (int a = 0; a < A; ++a) q[e * A + a] = (float)(rnd() % 100) * 0.01f;
      act[e] = rnd() % A;
      rew[e] = (float)(rnd() % 7) - 3.0f;
      done[e] = (rnd() % 13) == 0;
    }
    CHECK(apex_rt_ns_step(h, obs.data(), q.data(), A, act.data(), rew.data(), done.data(), nxt.data()) == 0);
    obs = nxt;
    const int64_t sz = apex_rt_ns_size(h);
    if (t % 5 == 4 && sz > 0) {
      const int64_t k = (t % 10 == 9) ? -1 : sz / 2 + 1;
      const int64_t m = k < 0 ? sz : k;
      std::vector<int64_t> o(m * 4), nx(m * 4), a(m), key(m), env(m);
      std::vector<float> R(m), G(m), pr(m);
      const int64_t got = apex_rt_ns_take(h, k, o.data(), nx.data(), a.data(), R.data(), G.data(), pr.data(),
                                          key.data(), env.data());
      CHECK(got == m);
      for (int64_t i = 0; i < got; ++i) {
        CHECK(G[i] == 0.0f || std::fabs(G[i] - 0.970299f) < 1e-6f);
        CHECK(env[i] >= 5 && env[i] < 5 + E && a[i] >= 0 && a[i] < A && pr[i] >= 0.0f);
      }
      total += got;
    }
  }
  act[0] = A;  // out of range: rejected
  CHECK(apex_rt_ns_step(h, obs.data(), q.data(), A, act.data(), rew.data(), done.data(), nxt.data()) == 1);
  CHECK(total > 1000);
  apex_rt_ns_destroy(h);
  return 0;
}

int main() {
  CHECK(apex_rt_version() == 1);
  if (test_sumtree()) return 1;
  if (test_cartpole()) return 1;
  if (test_seqlock()) return 1;
  if (test_nstep()) return 1;
  std::puts("runtime selftest OK");
  return 0;
}

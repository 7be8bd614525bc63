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

int main() {
  CHECK(apex_rt_version() == 1);
  if (test_sumtree()) return 1;
  if (test_cartpole()) return 1;
  if (test_seqlock()) return 1;
  std::puts("runtime selftest OK");
  return 0;
}

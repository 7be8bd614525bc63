// HBM-resident prioritized-replay shard: 64-ary sum-tree + record ring.
//
// Replaces the reference ReplayMemory (replay.py:8-84: dict priorities with an
// O(N^2) recompute per add/update, O(B*N) sampling, FIFO list eviction) with a
// tree whose fan-out equals the wavefront width: one wave descends one level
// per coalesced 64-child load + wave prefix scan, so a 2^21-leaf shard is 4
// dependent loads deep instead of 21 (binary tree).
//
// Layout: leaves = p^alpha (fp32, [cap]); internal levels k=1..L in one fp64
// array (level k has ceil(n_{k-1}/64) nodes, root at level L).  Leaf writes
// propagate fp64 deltas up with hardware fp64 atomics (no level-synchronous
// passes, one launch); tree_rebuild re-derives every internal node exactly
// from the leaves (run at the eviction cadence) so fp drift never accumulates.
// Duplicate indices in one update batch: last occurrence wins (deterministic).
#include "apex_common.h"
#include <stdlib.h>
#include "head_common.h"
#include "igemm_wgrad.h"
#include "rmsprop_common.h"
#include "pack_rows.h"

// Bounds-checking debug build (SURVEY §5.2 "race / bounds detection"): built as a
// separate library with -DAPEX_DEBUG_BOUNDS and selected by APEX_DEBUG_BOUNDS=1.
// Every leaf / ring-slot / frame index a replay kernel dereferences is checked;
// a violation bumps a per-site device counter, records the first bad index and
// is clamped into range (or dropped) -- nothing traps, so a corrupt index shows
// up as a readable error report instead of a GPU fault that resets the node.
// Sites: 0 tree_update leaf, 1 replay_insert slot, 2 tree_sample leaf/record,
// 3 gather_frames ring slot, 4 replay_insert frame-slot value, 5 zero_range slot.
#define APEX_DBG_SITES 8
#ifdef APEX_DEBUG_BOUNDS
__device__ int apex_dbg_count[APEX_DBG_SITES];
__device__ long long apex_dbg_first[APEX_DBG_SITES];
__device__ __forceinline__ bool apex_dbg_ok(int64_t i, int64_t n, int site) {
  if (i >= 0 && i < n) return true;
  if (atomicAdd(&apex_dbg_count[site], 1) == 0) apex_dbg_first[site] = (long long)i;
  return false;
}
#define APEX_DBG_OK(i, n, site) apex_dbg_ok((int64_t)(i), (int64_t)(n), site)
#define APEX_DBG_CLAMP(i, n, site) (APEX_DBG_OK(i, n, site) ? (i) : ((i) < 0 ? 0 : (n) - 1))
#else
#define APEX_DBG_OK(i, n, site) true
#define APEX_DBG_CLAMP(i, n, site) (i)
#endif

struct TreeDesc {
  float* leaf;
  double* nodes;
  int64_t off[8];
  int64_t n[8];
  int L;
  uint32_t* min_bits;  // running min over positive leaves (float bits)
};

struct RecordDesc {
  int32_t* obs;   // [cap, C] frame-ring slots of S_t's stack
  int32_t* nxt;   // [cap, C] frame-ring slots of S_{t+n}'s stack
  int32_t* act;   // [cap]
  float* rew;     // [cap]
  float* gam;     // [cap]
  int32_t* gen;   // [cap] slot generation (bumped on every insert)
  int C;
  int64_t cap;
  int64_t nframes;  // frame-ring size (debug bounds checks of stored slots; 0 = unchecked)
};

// Write leaf values and propagate the deltas up the tree, block-cooperatively
// (every thread of the block must call; contains __syncthreads):
//  * levels with many nodes (k < kfirst): one fp64 global atomic per updated
//    leaf -- random leaves rarely share a parent there;
//  * the small top levels (k >= kfirst, <= TREE_LACC nodes in total): deltas are
//    summed in LDS with ds_add_f64 first, then each touched node gets ONE global
//    atomic per block -- the root sees #blocks atomics instead of #leaves.
// The running min of positive leaves is reduced the same way.
#define TREE_LACC 4096

__device__ __forceinline__ void tree_block_update(const TreeDesc& t, bool act, int64_t i, float v,
                                                  double* lacc, uint32_t* lmin, int kfirst) {
  double d = 0.0;
  if (act) {
    const float old = t.leaf[i];
    t.leaf[i] = v;
    d = (double)v - (double)old;
  }
  int nsmall = 0;
  for (int k = kfirst; k <= t.L; ++k) nsmall += (int)t.n[k];
  for (int j = threadIdx.x; j < nsmall; j += blockDim.x) lacc[j] = 0.0;
  if (threadIdx.x == 0) *lmin = 0x7f800000u;
  __syncthreads();
  if (act && d != 0.0) {
    int64_t node = i;
    int loff = 0;
    for (int k = 1; k <= t.L; ++k) {
      node >>= 6;
      if (k < kfirst) {
        atomicAdd(&t.nodes[t.off[k] + node], d);
      } else {
        atomicAdd(&lacc[loff + node], d);
        loff += (int)t.n[k];
      }
    }
  }
  if (act && v > 0.f) atomicMin(lmin, __float_as_uint(v));
  __syncthreads();
  int loff = 0;
  for (int k = kfirst; k <= t.L; ++k) {
    for (int j = threadIdx.x; j < t.n[k]; j += blockDim.x) {
      const double a = lacc[loff + j];
      if (a != 0.0) atomicAdd(&t.nodes[t.off[k] + j], a);
    }
    loff += (int)t.n[k];
  }
  if (threadIdx.x == 0 && *lmin != 0x7f800000u) atomicMin(t.min_bits, *lmin);
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// mode 0: values are leaf values; mode 1: values are |td| -> (|td|+eps)^alpha,
// skipping evicted leaves (leaf == 0) and slots re-used since sampling (gen).
// dedupe (single block, n <= 1024): last occurrence of an index wins, found with
// an LDS hash table (atomicCAS insert + atomicMax of the position).
__global__ void __launch_bounds__(1024) tree_update_kernel(TreeDesc t, const int64_t* __restrict__ idx,
                                                           const float* __restrict__ values, int n, int mode,
                                                           float alpha, float eps,
                                                           const int32_t* __restrict__ gen_expect,
                                                           const int32_t* __restrict__ gen, int dedupe,
                                                           uint64_t* ctr_to_bump, int kfirst) {
  __shared__ uint32_t hkey[2048];
  __shared__ int32_t hval[2048];
  __shared__ double lacc[TREE_LACC];
  __shared__ uint32_t lmin;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (ctr_to_bump != nullptr && i == 0) ctr_to_bump[0] += 1;
  bool act = i < n;
  int64_t s = 0;
  if (act) {
    s = idx[i];
    act = APEX_DBG_OK(s, t.n[0], 0);
    // rows of a sharded draw that landed in another shard (generation -1) write
    // nothing, so they must not take part in the dedupe either: a foreign row on
    // the same leaf as a valid row would otherwise win and then be dropped
    if (gen_expect != nullptr && gen_expect[i] < 0) act = false;
  }
  if (dedupe) {  // host guarantees gridDim.x == 1 and n <= 1024
    for (int j = threadIdx.x; j < 2048; j += blockDim.x) {
      hkey[j] = 0u;
      hval[j] = -1;
    }
    __syncthreads();
    int h = 0;
    const uint32_t key = (uint32_t)s + 1u;
    if (act) {
      h = (int)(hash32(key) & 2047u);
      while (true) {
        const uint32_t old = atomicCAS(&hkey[h], 0u, key);
        if (old == 0u || old == key) {
          atomicMax(&hval[h], i);
          break;
        }
        h = (h + 1) & 2047;
      }
    }
    __syncthreads();
    if (act && hval[h] != i) act = false;  // a later write to the same leaf wins
  }
  float v = 0.f;
  if (act) {
    v = values[i];
    if (mode == 1) {
      if (t.leaf[s] <= 0.f) act = false;
      else if (gen_expect != nullptr && gen[s] != gen_expect[i]) act = false;
      v = powf(fabsf(v) + eps, alpha);
    }
  }
  tree_block_update(t, act, s, v, lacc, &lmin, kfirst);
}

// zero `count` leaves starting at ring slot `start` (FIFO eviction)
__global__ void __launch_bounds__(256) tree_zero_range_kernel(TreeDesc t, int64_t start, int64_t count,
                                                              int kfirst) {
  __shared__ double lacc[TREE_LACC];
  __shared__ uint32_t lmin;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool act = i < count;
  int64_t s = act ? (start + i) % t.n[0] : 0;
  s = APEX_DBG_CLAMP(s, t.n[0], 5);
  if (act && t.leaf[s] == 0.f) act = false;
  tree_block_update(t, act, s, 0.f, lacc, &lmin, kfirst);
}

// scatter K staged records into ring slots start..start+K-1 (mod cap) and set
// their leaves to (prio+eps)^alpha
__global__ void __launch_bounds__(256) replay_insert_kernel(TreeDesc t, RecordDesc r, int64_t start, int K,
                                                            const int32_t* __restrict__ s_obs,
                                                            const int32_t* __restrict__ s_nxt,
                                                            const int32_t* __restrict__ s_act,
                                                            const float* __restrict__ s_rew,
                                                            const float* __restrict__ s_gam,
                                                            const float* __restrict__ s_prio, float alpha,
                                                            float eps, int kfirst) {
  __shared__ double lacc[TREE_LACC];
  __shared__ uint32_t lmin;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < K;
  int64_t s = act ? (start + i) % r.cap : 0;
  s = APEX_DBG_CLAMP(s, r.cap < t.n[0] ? r.cap : t.n[0], 1);
  float v = 0.f;
  if (act) {
    for (int c = 0; c < r.C; ++c) {
      const int32_t so = s_obs[(int64_t)i * r.C + c], sn = s_nxt[(int64_t)i * r.C + c];
#ifdef APEX_DEBUG_BOUNDS
      if (r.nframes > 0) {
        APEX_DBG_OK(so, r.nframes, 4);
        APEX_DBG_OK(sn, r.nframes, 4);
      }
#endif
      r.obs[s * r.C + c] = so;
      r.nxt[s * r.C + c] = sn;
    }
    r.act[s] = s_act[i];
    r.rew[s] = s_rew[i];
    r.gam[s] = s_gam[i];
    r.gen[s] += 1;
    v = powf(fabsf(s_prio[i]) + eps, alpha);
  }
  tree_block_update(t, act, s, v, lacc, &lmin, kfirst);
}

// first level whose node count, summed with all levels above it, fits TREE_LACC
static int tree_kfirst(const TreeDesc& t) {
  int k = t.L;
  int64_t sum = t.n[t.L];
  while (k > 1 && sum + t.n[k - 1] <= TREE_LACC) {
    sum += t.n[k - 1];
    --k;
  }
  return k;
}

// Stratified proportional sampling: one wave per sample, 64-ary descent.
// Also gathers the sampled records and the IS weight
//   w_i = (N P(i) / max_j N P(j))^-beta = (p_i / min_j p_j)^-beta   (max-normalised).
//
// Sharded mode (`shard_stats` set: the all-gathered (total, min p) of the W shards,
// fp64 [W][2]): ONE global stratified draw over the concatenation of the shards'
// mass intervals, identical on every rank (same seed, same counter, same gathered
// totals summed in the same order), so every global draw lands in exactly one
// shard and an item's sampling probability is p_i / sum_all p -- the single
// prioritized replay of the reference (replay.py:44-57) spread over W GPUs.
// Rank r takes the draws in its interval [c_{r-1}, c_r): slot b of the local batch
// holds the b-th of them.  The global batch is M = min(W B, floor((B - 2) sum / max
// T_r)) draws, so no interval catches more than B (an interval of length T spans at
// most floor(T M / sum) + 2 strata); unused slots get weight 0 and generation -1
// (their priority write-back is dropped).  IS weights use the global minimum:
// w = (p / p_min)^-beta * (W B / M), the last factor turning the head's 1/(W B)
// gradient scale into the 1/M mean over the draws actually taken.
// all-gathered per-shard statistics: (sum p^alpha, min p^alpha, max IS weight of the
// shard's rows in the current batch -- written by the head kernel, read by the optimizer)
#define SHARD_STATS 3
struct SampleArgs {
  TreeDesc t;
  RecordDesc r;
  int B;
  uint64_t seed;
  const uint64_t* ctr;
  float beta;
  int64_t* out_idx;
  float* out_w;
  int32_t* out_gen;
  int32_t* out_obs;
  int32_t* out_nxt;
  int32_t* out_act;
  float* out_rew;
  float* out_gam;
  int32_t* out_nxt2;
  const double* shard_stats;   // sharded mode: [W][SHARD_STATS] (total, min p, batch IS max) per shard, or null
  int shard_rank, shard_world;
  uint64_t shard_seed;         // common to all ranks (the local `seed` is per shard)
  float* out_wscale;           // the batch's W B / M factor (1 unsharded), for the IS batch-max; or null
  int64_t mcap;                // sharded: cap on the global batch M (W B: per-rank batches; the
                               // configured global batch: Runtime.batch_scope = "global")
};

// block `bid` of 4 waves: samples 4 bid .. 4 bid + 3
__device__ __forceinline__ void tree_sample_body(const SampleArgs& S, int bid) {
  const TreeDesc& t = S.t;
  const RecordDesc& r = S.r;
  const int B = S.B;
  const uint64_t seed = S.seed;
  const uint64_t* __restrict__ ctr = S.ctr;
  const float beta = S.beta;
  int64_t* __restrict__ out_idx = S.out_idx;
  float* __restrict__ out_w = S.out_w;
  int32_t* __restrict__ out_gen = S.out_gen;
  int32_t* __restrict__ out_obs = S.out_obs;
  int32_t* __restrict__ out_nxt = S.out_nxt;
  int32_t* __restrict__ out_act = S.out_act;
  float* __restrict__ out_rew = S.out_rew;
  float* __restrict__ out_gam = S.out_gam;
  int32_t* __restrict__ out_nxt2 = S.out_nxt2;
  const int lane = threadIdx.x & 63;
  const int b = (bid * blockDim.x + threadIdx.x) >> 6;
  if (b >= B) return;
  const double total = t.nodes[t.off[t.L]];
  double u;
  bool valid = true;
  float wscale = 1.f, pmin_g = 0.f;
  if (S.shard_stats != nullptr) {
    const int W = S.shard_world, r = S.shard_rank;
    double sum = 0.0, c0 = 0.0, tmax = 0.0;
    float pm = __uint_as_float(0x7f800000u);
    for (int q = 0; q < W; ++q) {
      const double Tq = S.shard_stats[SHARD_STATS * q];
      if (q < r) c0 += Tq;
      sum += Tq;
      tmax = fmax(tmax, Tq);
      const float mq = (float)S.shard_stats[SHARD_STATS * q + 1];
      if (Tq > 0.0 && mq > 0.f) pm = fminf(pm, mq);
    }
    const double Tr = S.shard_stats[SHARD_STATS * r];
    const double c1 = c0 + Tr;
    int64_t M = 0;
    if (tmax > 0.0) {
      // one shard holds every stratum: B rows suffice; otherwise an interval of mass T
      // catches at most floor(T M / sum) + 2 strata
      const double mb = W == 1 ? (double)B : floor((double)(B - 2) * sum / tmax);
      M = (int64_t)fmin((double)S.mcap, fmax(mb, 0.0));
    }
    const uint64_t cc = ctr[0];
    double ul = 0.0;
    if (M > 0 && Tr > 0.0) {
      const double delta = sum / (double)M;
      int64_t j0 = (int64_t)floor(c0 / delta);
      if (((double)j0 + (double)apex_uniform(S.shard_seed, cc, (uint64_t)j0)) * delta < c0) ++j0;
      const int64_t j = j0 + b;
      const double uj = ((double)j + (double)apex_uniform(S.shard_seed, cc, (uint64_t)j)) * delta;
      // (the last interval ends at the total: strata rounded past it are still its own)
      valid = j < M && (r == W - 1 || uj < c1);
      ul = uj - c0;
      wscale = (float)((double)W * (double)B / (double)M);
    } else {
      valid = false;
    }
    u = valid ? fmin(fmax(ul, 0.0), total) : 0.0;
    pmin_g = pm;
  } else {
    const float uu = apex_uniform(seed, ctr[0], (uint64_t)b);
    u = ((double)b + (double)uu) * (total / (double)B);
  }
  int64_t node = 0;
  for (int k = t.L - 1; k >= 0; --k) {
    int64_t child = node * 64 + lane;
    double v = 0.0;
    if (child < t.n[k]) v = (k == 0) ? (double)t.leaf[child] : t.nodes[t.off[k] + child];
    double incl = wave_inclusive_scan(v, lane);
    // first child whose inclusive prefix exceeds u; fall back to the last
    // non-empty child when round-off pushes u past the subtree mass
    uint64_t pass = __ballot(incl > u && v > 0.0);
    uint64_t nonempty = __ballot(v > 0.0);
    int sel;
    if (pass) sel = __ffsll((unsigned long long)pass) - 1;
    else sel = nonempty ? 63 - __clzll((long long)nonempty) : 0;
    double excl = __shfl(incl - v, sel, 64);
    u -= excl;
    node = node * 64 + sel;
  }
  int64_t s = node < t.n[0] ? node : t.n[0] - 1;
  s = APEX_DBG_CLAMP(s, r.cap < t.n[0] ? r.cap : t.n[0], 2);
  if (lane == 0) {
    float p = t.leaf[s];
    // (p / p_min)^-beta <= 1 (p_min global over the shards in sharded mode), times
    // the global-batch correction
    const float pmin = S.shard_stats != nullptr ? pmin_g : __uint_as_float(t.min_bits[0]);
    const float w = (valid && p > 0.f && pmin > 0.f) ? fminf(powf(p / pmin, -beta), 1.0f) * wscale : 0.f;
    out_idx[b] = s;
    out_w[b] = w;
    if (b == 0 && S.out_wscale != nullptr) S.out_wscale[0] = wscale;
    out_gen[b] = valid ? r.gen[s] : -1;
    out_act[b] = r.act[s];
    out_rew[b] = r.rew[s];
    out_gam[b] = r.gam[s];
  }
  for (int c = lane; c < r.C; c += 64) {
    out_obs[(int64_t)b * r.C + c] = r.obs[s * r.C + c];
    const int32_t nv = r.nxt[s * r.C + c];
    out_nxt[(int64_t)b * r.C + c] = nv;
    if (out_nxt2) out_nxt2[(int64_t)b * r.C + c] = nv;
  }
}

__global__ void __launch_bounds__(256) tree_sample_kernel(SampleArgs s) { tree_sample_body(s, blockIdx.x); }

// Exact rebuild of one internal level from its children (wave per parent);
// the leaf pass also recomputes the min over positive leaves.
__global__ void tree_reduce_level_kernel(const float* __restrict__ leaf, const double* __restrict__ src,
                                         int64_t nsrc, double* __restrict__ dst, int64_t ndst,
                                         uint32_t* min_bits) {
  const int lane = threadIdx.x & 63;
  const int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (p >= ndst) return;
  int64_t c = p * 64 + lane;
  double v = 0.0;
  float mn = __uint_as_float(0x7f800000u);
  if (c < nsrc) {
    if (leaf) {
      float f = leaf[c];
      v = (double)f;
      if (f > 0.f) mn = f;
    } else {
      v = src[c];
    }
  }
  v = wave_sum(v);
  if (leaf) mn = wave_min(mn);
  if (lane == 0) {
    dst[p] = v;
    if (leaf && mn < __uint_as_float(0x7f800000u)) atomicMin(min_bits, __float_as_uint(mn));
  }
}

// The leaf level of the exact rebuild: parents grid-strided over a bounded grid, the
// min over positive leaves kept per lane and reduced once per block -- one atomicMin per
// block instead of one per parent (at 2.5 M leaves the per-parent atomics on the single
// min word serialised the rebuild: 0.38 ms, profiles/r5_replay_2m.json).
__global__ void __launch_bounds__(256) tree_reduce_leaf_kernel(const float* __restrict__ leaf, int64_t nsrc,
                                                               double* __restrict__ dst, int64_t ndst,
                                                               uint32_t* min_bits) {
  __shared__ float wmin[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nw = (int64_t)gridDim.x * 4;
  float mn = __uint_as_float(0x7f800000u);
  for (int64_t p = (int64_t)blockIdx.x * 4 + w; p < ndst; p += nw) {
    const int64_t c = p * 64 + lane;
    double v = 0.0;
    if (c < nsrc) {
      const float f = leaf[c];
      v = (double)f;
      if (f > 0.f) mn = fminf(mn, f);
    }
    v = wave_sum(v);
    if (lane == 0) dst[p] = v;
  }
  mn = wave_min(mn);
  if (lane == 0) wmin[w] = mn;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fminf(fminf(wmin[0], wmin[1]), fminf(wmin[2], wmin[3]));
    if (m < __uint_as_float(0x7f800000u)) atomicMin(min_bits, __float_as_uint(m));
  }
}

__global__ void fill_u32_kernel(uint32_t* p, uint32_t v, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// gather stacked frames: out[b, c] = ring[slots[b, c]]  (uint8, frame_bytes each)
__global__ void gather_frames_kernel(const uint8_t* __restrict__ ring, const int32_t* __restrict__ slots,
                                     int64_t nframes, int64_t frame_bytes, uint8_t* __restrict__ out) {
  const int bc = blockIdx.x;  // one block per (sample, channel)
  int32_t s = slots[bc];
#ifdef APEX_DEBUG_BOUNDS
  if (!(s >= 0 && s < nframes)) {
    if (threadIdx.x == 0) (void)APEX_DBG_OK(s, nframes, 3);
    s = s < 0 ? 0 : (int32_t)(nframes - 1);
  }
#endif
  const uint4* src = reinterpret_cast<const uint4*>(ring + (int64_t)s * frame_bytes);
  uint4* dst = reinterpret_cast<uint4*>(out + (int64_t)bc * frame_bytes);
  const int64_t nv = frame_bytes / 16;
  for (int64_t i = threadIdx.x; i < nv; i += blockDim.x) dst[i] = src[i];
}

// ------------------------------------------------- fused learner-step kernels
// The priority write-back and the next batch's draw ride in launches that run
// anyway, so the learner step has no separate latency-bound tree kernels on its
// critical path (a lone tree_update / tree_sample launch is a few waves running
// dependent global loads while the rest of the chip idles).

// Single-block priority write-back (tree_update mode 1 with dedupe) for n <= 1024
// leaves and n <= TU_MAXR * blockDim (the launchers check both): items tid,
// tid + blockDim, ...; the LDS hash keeps the last occurrence of a duplicated leaf;
// every item's delta goes through the block-aggregated tree_block_update (the root
// sees ONE atomic per item round).
#define TU_MAXR 4
struct TreeUpdArgs {
  TreeDesc t;
  const int64_t* idx;
  const float* td;           // |delta| per sample
  const int32_t* gen_expect;
  const int32_t* gen;
  uint64_t* ctr_to_bump;
  float alpha, eps;
  int n, kfirst;
  double* stats_out;         // sharded replay: (sum p^alpha, min p^alpha) after the update, or null
};

__device__ __forceinline__ void tree_update_block(const TreeUpdArgs& a) {
  __shared__ uint32_t hkey[2048];
  __shared__ int32_t hval[2048];
  __shared__ double lacc[TREE_LACC];
  __shared__ uint32_t lmin;
  const TreeDesc& t = a.t;
  const int nt = blockDim.x, R = (a.n + nt - 1) / nt;
  if (a.ctr_to_bump != nullptr && threadIdx.x == 0) a.ctr_to_bump[0] += 1;
  for (int j = threadIdx.x; j < 2048; j += nt) {
    hkey[j] = 0u;
    hval[j] = -1;
  }
  __syncthreads();
  int64_t s[TU_MAXR];
  int h[TU_MAXR];
#pragma unroll
  for (int r = 0; r < TU_MAXR; ++r) {
    if (r >= R) break;
    const int i = threadIdx.x + r * nt;
    s[r] = 0;
    h[r] = -1;
    if (i < a.n) {
      s[r] = a.idx[i];
      // foreign rows of a sharded draw (generation -1) stay out of the dedupe
      if (APEX_DBG_OK(s[r], t.n[0], 0) && (a.gen_expect == nullptr || a.gen_expect[i] >= 0)) {
        const uint32_t key = (uint32_t)s[r] + 1u;
        int hh = (int)(hash32(key) & 2047u);
        while (true) {
          const uint32_t old = atomicCAS(&hkey[hh], 0u, key);
          if (old == 0u || old == key) {
            atomicMax(&hval[hh], i);
            break;
          }
          hh = (hh + 1) & 2047;
        }
        h[r] = hh;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < TU_MAXR; ++r) {
    if (r >= R) break;
    const int i = threadIdx.x + r * nt;
    bool act = h[r] >= 0 && hval[h[r]] == i;   // a later write to the same leaf wins
    float v = 0.f;
    if (act) {
      if (t.leaf[s[r]] <= 0.f) act = false;
      else if (a.gen_expect != nullptr && a.gen[s[r]] != a.gen_expect[i]) act = false;
      v = powf(fabsf(a.td[i]) + a.eps, a.alpha);
    }
    tree_block_update(t, act, s[r], v, lacc, &lmin, a.kfirst);
    __syncthreads();
  }
  if (a.stats_out != nullptr) {
    // this shard's statistics for the step's all-gather (replay/gpu_replay.py
    // gather_shard_stats): the root and the min after every update above -- read by
    // L2 atomics, which see this block's own atomic updates
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
      a.stats_out[0] = atomicAdd(t.nodes + t.off[t.L], 0.0);
      a.stats_out[1] = (double)__uint_as_float(atomicOr(t.min_bits, 0u));
    }
  }
}

// head weight gradient + priority write-back in one launch: block 0 runs the
// single-block tree update (dispatched first, it is the long pole), blocks 1..
// the (A+1) x HS/64 head_wgrad blocks.  Both only need the head kernel's outputs.
// (DP step: blocks past 1 + nhw pack the factored exchange's send rows, csrc/pack_rows.h)
__global__ void __launch_bounds__(512) head_wgrad_prio_kernel(HeadWgArgs hw, TreeUpdArgs tu, PackRows pk, int nhw,
                                                             int npk) {
  if (blockIdx.x == 0) {
    tree_update_block(tu);
    return;
  }
  if ((int)blockIdx.x > nhw) {
    pack_rows_body(pk, blockIdx.x - 1 - nhw, npk);
    return;
  }
  const int b = blockIdx.x - 1, nch = hw.HS / 64;
  head_wgrad_body(hw, b / nch, b - (b / nch) * nch);
}

// fc weight gradient + head weight gradient + priority write-back in ONE launch
// (all three only need the head kernel's outputs).  Block 0: the single-block tree
// update (the latency-bound long pole, dispatched first); blocks 1..nhw: head
// wgrad (4 waves each); from blk0 (a multiple of 8, so the XCD-contiguous tile
// order of the GEMM part is preserved): the fc wgrad GEMM tiles (one split, the
// shape launch_wgrad picks for the 1024 x 3136 fc: CT=4, NT=1 in bf16; CT=2, NT=1
// in split mode, whose doubled images leave room for the tree update's LDS).  The
// fc wgrad takes one block per CU and leaves CUs idle; the other two fill them.
template <int SP>
__global__ void __launch_bounds__(256) fc_wgrad_head_prio_kernel(WgradDesc d, int gx, int gy, HeadWgArgs hw,
                                                                 TreeUpdArgs tu, int nhw, int blk0) {
  const int b = blockIdx.x;
  if (b == 0) {
    tree_update_block(tu);
  } else if (b <= nhw) {
    const int nch = hw.HS / 64, q = b - 1;
    head_wgrad_body(hw, q / nch, q - (q / nch) * nch);
  } else if (b >= blk0) {
    igemm_wgrad_body<0, 1, 1, SP ? 2 : 4, 1, SP>(d, b - blk0, gx, gy, 1);
  }
}

// optimizer + the next step's prioritized draw: blocks [0, nsb) sample, the rest
// run the clip + centered RMSprop + bf16 pack over the flat parameters.  The tree
// already holds this step's priorities (written by fc_wgrad_head_prio_kernel), so the
// draw equals the one a sample launch at the head of the next step would make.
//
// SEG: the update covers only the listed ranges of the flat arrays (RmsSegs): the
// data-parallel step with a sharded optimizer (learner/dp_step.py) updates the conv +
// head range and the rank's own fc rows.  Every element's update is the same
// arithmetic as in the whole-range launch (the clip coefficient comes from the same
// partials), so a sharded update equals the unsharded one element for element.
struct RmsSegs {
  int nseg;            // 1..3
  int blk0[4];         // first optimizer block of segment k; blk0[nseg] = the total
  int64_t off[3];      // element offset of segment k (a multiple of 4)
  int64_t len[3];
};

template <int NT, bool SEG>
__global__ void __launch_bounds__(NT) rmsprop_sample_kernel(RmspropArgs a, SampleArgs s, int nsb, RmsSegs sg) {
  if ((int)blockIdx.x < nsb) {
    tree_sample_body(s, blockIdx.x);
    return;
  }
  const int b = blockIdx.x - nsb;
  if constexpr (!SEG) {
    rmsprop_body(a, b, gridDim.x - nsb);
  } else {
    int k = 0;
    while (k + 1 < sg.nseg && b >= sg.blk0[k + 1]) ++k;
    RmspropArgs t = a;
    const int64_t o = sg.off[k];
    t.p += o;
    t.g += o;
    t.v += o;
    t.m += o;
    t.pb += o;
    if (t.pb_lo != nullptr) t.pb_lo += o;
    t.n = sg.len[k];
    if (k != 0) {                 // the fused-forward operand stores and the norm live in segment 0
      t.fo = CfFragOut{};
      t.norm_out = nullptr;
    }
    rmsprop_body(t, b - sg.blk0[k], sg.blk0[k + 1] - sg.blk0[k]);
  }
}

// ---------------------------------------------------------------- launchers
static inline int blocks_for(int64_t n, int t) { return (int)((n + t - 1) / t); }

APEX_EXPORT int apex_tree_update(TreeDesc t, const int64_t* idx, const float* values, int n, int mode,
                                 float alpha, float eps, const int32_t* gen_expect, const int32_t* gen,
                                 int dedupe, uint64_t* ctr_to_bump, hipStream_t st) {
  if (n <= 0 && ctr_to_bump == nullptr) return 0;
  if (dedupe && n > 1024) return (int)hipErrorInvalidValue;
  const int threads = n <= 1024 ? ((n + 63) / 64) * 64 : 1024;
  const int nb = n > 0 ? blocks_for(n, threads) : 1;
  tree_update_kernel<<<nb, threads > 0 ? threads : 64, 0, st>>>(t, idx, values, n, mode, alpha, eps, gen_expect,
                                                               gen, dedupe, ctr_to_bump, tree_kfirst(t));
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_tree_zero_range(TreeDesc t, int64_t start, int64_t count, hipStream_t st) {
  if (count <= 0) return 0;
  tree_zero_range_kernel<<<blocks_for(count, 256), 256, 0, st>>>(t, start, count, tree_kfirst(t));
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_replay_insert(TreeDesc t, RecordDesc r, int64_t start, int K, const int32_t* s_obs,
                                   const int32_t* s_nxt, const int32_t* s_act, const float* s_rew,
                                   const float* s_gam, const float* s_prio, float alpha, float eps,
                                   hipStream_t st) {
  if (K <= 0) return 0;
  replay_insert_kernel<<<blocks_for(K, 256), 256, 0, st>>>(t, r, start, K, s_obs, s_nxt, s_act, s_rew,
                                                           s_gam, s_prio, alpha, eps, tree_kfirst(t));
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_tree_sample(TreeDesc t, RecordDesc r, int B, uint64_t seed, const uint64_t* ctr,
                                 float beta, int64_t* out_idx, float* out_w,
                                 int32_t* out_gen, int32_t* out_obs, int32_t* out_nxt, int32_t* out_act,
                                 float* out_rew, float* out_gam, int32_t* out_nxt2, const double* shard_stats,
                                 int shard_rank, int shard_world, uint64_t shard_seed, float* out_wscale,
                                 int64_t mcap, hipStream_t st) {
  if (B <= 0) return 0;
  if (mcap <= 0) mcap = (int64_t)shard_world * B;
  if (shard_stats != nullptr && (B < 3 || shard_world < 1 || shard_rank < 0 || shard_rank >= shard_world))
    return (int)hipErrorInvalidValue;
  const int waves_per_block = 4;
  tree_sample_kernel<<<blocks_for(B, waves_per_block), 64 * waves_per_block, 0, st>>>(
      SampleArgs{t, r, B, seed, ctr, beta, out_idx, out_w, out_gen, out_obs, out_nxt, out_act,
                 out_rew, out_gam, out_nxt2, shard_stats, shard_rank, shard_world, shard_seed, out_wscale,
                 mcap});
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_tree_rebuild(TreeDesc t, hipStream_t st) {
  fill_u32_kernel<<<1, 64, 0, st>>>(t.min_bits, 0x7f800000u, 1);
  for (int k = 1; k <= t.L; ++k) {
    int64_t nd = t.n[k];
    const int wpb = 4;
    if (k == 1) {
      const int nb = blocks_for(nd, wpb);
      tree_reduce_leaf_kernel<<<nb < 512 ? nb : 512, 64 * wpb, 0, st>>>(t.leaf, t.n[0], t.nodes + t.off[1], nd,
                                                                       t.min_bits);
      continue;
    }
    tree_reduce_level_kernel<<<blocks_for(nd, wpb), 64 * wpb, 0, st>>>(
        nullptr, t.nodes + t.off[k - 1], t.n[k - 1], t.nodes + t.off[k], nd, t.min_bits);
  }
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_gather_frames(const uint8_t* ring, const int32_t* slots, int n_slots, int64_t nframes,
                                   int64_t frame_bytes, uint8_t* out, hipStream_t st) {
  if (n_slots <= 0) return 0;
  if (frame_bytes % 16) return (int)hipErrorInvalidValue;
  gather_frames_kernel<<<n_slots, 256, 0, st>>>(ring, slots, nframes, frame_bytes, out);
  APEX_CHECK_LAUNCH();
}

// Cache-policy probe (scripts/bench_cold_mall.py): fill n 16-B words with plain or
// non-temporal stores -- does a streaming write evict the Infinity Cache?
__global__ void fill16_kernel(uint4* p, int64_t n, int nt) {
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  const uint4 v = make_uint4(1u, 1u, 1u, 1u);
  const u32x4v vv = {1u, 1u, 1u, 1u};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (nt) __builtin_nontemporal_store(vv, reinterpret_cast<u32x4v*>(p + i));
    else p[i] = v;
  }
}

APEX_EXPORT int apex_fill16(void* p, int64_t n, int nt, hipStream_t st) {
  fill16_kernel<<<2048, 256, 0, st>>>(reinterpret_cast<uint4*>(p), n, nt);
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_abi_version() { return 8; }

// 1 if this library was built with -DAPEX_DEBUG_BOUNDS
APEX_EXPORT int apex_debug_bounds_enabled() {
#ifdef APEX_DEBUG_BOUNDS
  return 1;
#else
  return 0;
#endif
}

// copy (and optionally reset) the per-site violation counters + first bad index
APEX_EXPORT int apex_debug_errors(int* counts, long long* first, int reset) {
#ifdef APEX_DEBUG_BOUNDS
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(counts, HIP_SYMBOL(apex_dbg_count), sizeof(int) * APEX_DBG_SITES);
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(first, HIP_SYMBOL(apex_dbg_first), sizeof(long long) * APEX_DBG_SITES);
  if (e != hipSuccess) return (int)e;
  if (reset) {
    int zc[APEX_DBG_SITES] = {0};
    long long zf[APEX_DBG_SITES] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(apex_dbg_count), zc, sizeof(zc));
    e = hipMemcpyToSymbol(HIP_SYMBOL(apex_dbg_first), zf, sizeof(zf));
  }
  return (int)e;
#else
  for (int i = 0; i < APEX_DBG_SITES; ++i) {
    counts[i] = 0;
    first[i] = 0;
  }
  return 0;
#endif
}

// rmsprop (clip norm from `npart` partials, as apex_rmsprop_step_np) + tree_sample of B.
// `seg` (nullable): update only those ranges (offsets relative to p / g / v / m / pb);
// blk0 is filled in here.
APEX_EXPORT int apex_rmsprop_sample(float* p, const float* g, float* v, float* m, bf16_t* pb, int64_t n,
                                    const double* partials, int npart, float lr, float alpha, float eps_opt,
                                    float clip, int centered, float* norm_out, TreeDesc t, RecordDesc r, int B,
                                    uint64_t seed, const uint64_t* ctr, float beta,
                                    int64_t* out_idx, float* out_w, int32_t* out_gen, int32_t* out_obs,
                                    int32_t* out_nxt, int32_t* out_act, float* out_rew, float* out_gam,
                                    int32_t* out_nxt2, const double* shard_stats, int shard_rank, int shard_world,
                                    uint64_t shard_seed, float* out_wscale, int64_t mcap, bf16_t* pb_lo,
                                    const double* wnorm, int wn, int wstride, CfFragOut fo, const RmsSegs* seg,
                                    const float* gpre, int64_t npre, hipStream_t st) {
  if (mcap <= 0) mcap = (int64_t)shard_world * B;
  if (shard_stats != nullptr && (B < 3 || shard_world < 1 || shard_rank < 0 || shard_rank >= shard_world))
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)v | (uintptr_t)m) & 15) return (int)hipErrorInvalidValue;
  if ((((uintptr_t)pb | (uintptr_t)pb_lo) & 7) || B < 0) return (int)hipErrorInvalidValue;
  // 512-thread blocks, grid capped at 256: every block first sums the ~2.6 K clip-norm
  // partials, so fewer, fatter blocks cut those L2 reads (256 x 512 measured 2,540 / 4,175
  // fp32 / bf16 steps/s vs 2,528 / 4,107 at 512 x 512 and 3497-3520 vs 3543-3576 at
  // 256 x 2048 before; profiles/r3_ab_optimizer_blocks_512_384_256.txt)
  constexpr int nt = 512, maxb = 256;
  int nb = (int)((n / 4 + nt - 1) / nt);
  nb = nb < 1 ? 1 : (nb > maxb ? maxb : nb);
  RmsSegs sg{};
  if (seg != nullptr) {
    sg = *seg;
    if (sg.nseg < 1 || sg.nseg > 3) return (int)hipErrorInvalidValue;
    int64_t tot = 0;
    for (int k = 0; k < sg.nseg; ++k) {
      if ((sg.off[k] & 3) || sg.len[k] <= 0 || sg.off[k] < 0 || sg.off[k] + sg.len[k] > n)
        return (int)hipErrorInvalidValue;
      tot += sg.len[k];
    }
    // blocks in proportion to the segment sizes (at least one each, at most one float4
    // per thread), segment 0 enough for the fragment stores' first-chunk rule below
    const int64_t fend = fo.c3f != nullptr && fo.w3_off + 36864 > fo.w2_off + 65536 ? fo.w3_off + 36864
                                                                                     : fo.w2_off + 65536;
    const int64_t need0 = fo.w1frag != nullptr ? fend / 4 / nt + 1 : 1;
    int b0 = 0;
    for (int k = 0; k < sg.nseg; ++k) {
      const int64_t full = (sg.len[k] / 4 + nt - 1) / nt;
      int64_t nbk = (int64_t)maxb * sg.len[k] / tot;
      if (k == 0 && nbk < need0) nbk = need0;
      if (nbk > full) nbk = full;
      if (nbk < 1) nbk = 1;
      sg.blk0[k] = b0;
      b0 += (int)nbk;
    }
    sg.blk0[sg.nseg] = b0;
    nb = sg.blk0[1];              // segment 0's blocks: the fragment-store check below
  }
  const int nsb = B > 0 ? blocks_for(B, nt / 64) : 0;
  const int64_t n0 = seg != nullptr ? sg.len[0] : n;
  if (fo.w1frag != nullptr && (seg != nullptr && sg.off[0] != 0)) return (int)hipErrorInvalidValue;
  if (fo.w1frag != nullptr && (fo.c2f == nullptr || (fo.C != 1 && fo.C != 2 && fo.C != 4) ||
                               (fo.w1_off & 3) || (fo.w2_off & 7) || fo.w1_off + 4096LL * fo.C > n0 ||
                               fo.w2_off + 65536 > n0 ||
                               // (stored in each thread's first chunk: rmsprop_body's peel)
                               (fo.w1_off + 4096LL * fo.C) / 4 > (int64_t)nb * nt || (fo.w2_off + 65536) / 4 > (int64_t)nb * nt))
    return (int)hipErrorInvalidValue;
  if (fo.w1frag != nullptr && fo.c3f != nullptr &&
      ((fo.w3_off & 3) || fo.w3_off + 36864 > n0 || (fo.w3_off + 36864) / 4 > (int64_t)nb * nt || ((uintptr_t)fo.c3f & 15)))
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)gpre & 15) || npre < 0 || (npre > 0 && gpre == nullptr)) return (int)hipErrorInvalidValue;
  const RmspropArgs ra{p, g, v, m, pb, n, partials, npart, lr, alpha, eps_opt, clip, centered, norm_out, pb_lo,
                      wnorm, wn, wstride, fo, npre > 0 ? gpre : nullptr, npre};
  const SampleArgs sa{t, r, B, seed, ctr, beta, out_idx, out_w, out_gen, out_obs, out_nxt,
                      out_act, out_rew, out_gam, out_nxt2, shard_stats, shard_rank, shard_world, shard_seed,
                      out_wscale, mcap};
  if (seg != nullptr) rmsprop_sample_kernel<nt, true><<<sg.blk0[sg.nseg] + nsb, nt, 0, st>>>(ra, sa, nsb, sg);
  else rmsprop_sample_kernel<nt, false><<<nb + nsb, nt, 0, st>>>(ra, sa, nsb, sg);
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_head_wgrad_prio(const bf16_t* Hon, const float* dhead, int B, int A, float* gwv, float* gbv,
                                     float* gwa, float* gba, int hidden, TreeDesc t, const int64_t* idx,
                                     const float* td, const int32_t* gen_expect, const int32_t* gen,
                                     float alpha, float eps, uint64_t* ctr_to_bump, const bf16_t* Hon_lo,
                                     double* stats_out, const uint16_t* const* psrc, const int64_t* pld,
                                     const int* pcols, int pnseg, int prows, uint16_t* pdst, int64_t pdld,
                                     hipStream_t st) {
  // the single-block tree update holds TU_MAXR items per thread
  if ((hidden != 512 && hidden != 256) || B < 1 || B > 1024 || B > TU_MAXR * 512 || idx == nullptr)
    return (int)hipErrorInvalidValue;
  const int nhw = (A + 1) * (hidden / 64);
  // optional row pack in the same launch (pnseg > 0): up to 256 tail blocks
  PackRows pk{};
  int npk = 0;
  if (pnseg > 0) {
    int64_t nchunks = 0;
    const int err = make_pack_rows(psrc, pld, pcols, pnseg, prows, pdst, pdld, pk, nchunks);
    if (err) return err;
    npk = (int)((nchunks + 511) / 512);
    npk = npk > 256 ? 256 : npk;
  }
  head_wgrad_prio_kernel<<<1 + nhw + npk, 512, 0, st>>>(
      HeadWgArgs{Hon, dhead, B, A, gwv, gbv, gwa, gba, hidden, Hon_lo},
      TreeUpdArgs{t, idx, td, gen_expect, gen, ctr_to_bump, alpha, eps, B, tree_kfirst(t), stats_out}, pk, nhw, npk);
  APEX_CHECK_LAUNCH();
}

// the fused launch above; returns hipErrorInvalidValue when the fc problem is not
// the (CT=4, NT=1, single split, dense) shape it is compiled for -- the caller then
// issues the three launches separately
APEX_EXPORT int apex_fc_wgrad_head_prio(WgradDesc d, const bf16_t* Hon, const float* dhead, int B, int A,
                                        float* gwv, float* gbv, float* gwa, float* gba, int hidden, TreeDesc t,
                                        const int64_t* idx, const float* td, const int32_t* gen_expect,
                                        const int32_t* gen, float alpha, float eps, uint64_t* ctr_to_bump,
                                        const bf16_t* Hon_lo, double* stats_out, hipStream_t st) {
  // 256-thread blocks: the single-block tree update holds TU_MAXR items per thread
  if ((hidden != 512 && hidden != 256) || B < 1 || B > 1024 || B > TU_MAXR * 256 || idx == nullptr)
    return (int)hipErrorInvalidValue;
  if (d.mode != 0 || (d.Kc & 63) || (d.Co & 63) || d.rows_per_split < d.Mred) return (int)hipErrorInvalidValue;
  if ((int64_t)d.Mred * d.ldd * 2 >= 0x7ffffff0LL || (int64_t)d.Mred * d.ldx * 2 >= 0x7ffffff0LL)
    return (int)hipErrorInvalidValue;
  const bool split = d.dy_lo != nullptr;
  if (split && (d.x_lo == nullptr || Hon_lo == nullptr)) return (int)hipErrorInvalidValue;
  const int kt = d.Kc / 64, ct = d.Co / 64;
  // the compiled shape: {CT,NT} = {4,1} (index 2) in bf16, {2,1} (index 6) in split mode
  if (wgrad_shape(kt, ct, d.Kc, d.Co, split ? 1 : 0) != (split ? 6 : 2)) return (int)hipErrorInvalidValue;
  const int gx = kt, gy = ct / (split ? 2 : 4);
  const int nhw = (A + 1) * (hidden / 64);
  const int blk0 = (1 + nhw + 7) & ~7;
  const HeadWgArgs hw{Hon, dhead, B, A, gwv, gbv, gwa, gba, hidden, Hon_lo};
  const TreeUpdArgs tu{t, idx, td, gen_expect, gen, ctr_to_bump, alpha, eps, B, tree_kfirst(t), stats_out};
  if (split) fc_wgrad_head_prio_kernel<1><<<blk0 + gx * gy, 256, 0, st>>>(d, gx, gy, hw, tu, nhw, blk0);
  else fc_wgrad_head_prio_kernel<0><<<blk0 + gx * gy, 256, 0, st>>>(d, gx, gy, hw, tu, nhw, blk0);
  APEX_CHECK_LAUNCH();
}

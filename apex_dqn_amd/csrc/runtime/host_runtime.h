// Native host runtime for the CPU side of the framework (C ABI, loaded with
// ctypes by apex_dqn_amd/runtime/native.py).
//
//  * sum-tree / min-tree over caller-owned arrays (the CPU prioritized replay,
//    apex_dqn_amd/replay/host_replay.py) -- replaces the reference's dict of
//    priorities with an O(N^2) probability recompute (replay.py:18-30) and its
//    O(B*N) sampling scan (replay.py:44-57);
//  * vectorised CartPole-v1 stepping with auto-reset (the CPU actor hot loop,
//    reference actor.py:146-191 steps one gym env per process);
//  * a seqlock for learner -> actor parameter publication through shared
//    memory (reference: a 13.3 MB pickle through a Manager dict every step,
//    learner.py:74 / actor.py:189-191).
#pragma once
#include <cstdint>

#define APEX_RT_API extern "C" __attribute__((visibility("default")))

APEX_RT_API int apex_rt_version();

// ---- sum-tree: sum[2*size2], mn[2*size2], leaves at [size2, size2 + capacity)
APEX_RT_API int apex_rt_st_update(double* sum, double* mn, int64_t size2, int64_t capacity, const int64_t* idx,
                                  const double* val, int64_t n);
APEX_RT_API int apex_rt_st_find(const double* sum, int64_t size2, int64_t capacity, const double* u, int64_t n,
                                int64_t* out);
APEX_RT_API int apex_rt_st_sample_stratified(const double* sum, int64_t size2, int64_t capacity, int64_t batch,
                                             const double* r01, int64_t* out);

// ---- CartPole-v1, E environments; state[E][4] (double), t[E], ep_ret[E], rng[E]
APEX_RT_API void apex_rt_cp_reset(double* state, int64_t* t, double* ep_ret, uint64_t* rng, int E,
                                  const int32_t* mask, float* obs);
APEX_RT_API void apex_rt_cp_step(double* state, int64_t* t, double* ep_ret, uint64_t* rng, int E,
                                 const int64_t* actions, float* obs, float* rew, uint8_t* done, uint8_t* trunc,
                                 double* info_ret, int64_t* info_len);

// ---- seqlock over shared memory: *seq even = stable, odd = write in progress
APEX_RT_API int64_t apex_rt_seqlock_write(uint64_t* seq, void* dst, const void* src, int64_t nbytes);
APEX_RT_API int64_t apex_rt_seqlock_read(const uint64_t* seq, void* dst, const void* src, int64_t nbytes,
                                         int64_t last, int max_tries);

// ---- sliding-window n-step transition builder (csrc/runtime/nstep.cpp)
APEX_RT_API void* apex_rt_ns_create(int E, int n, double gamma, int obs_bytes, int64_t env_id_offset);
APEX_RT_API void apex_rt_ns_destroy(void* h);
APEX_RT_API int apex_rt_ns_step(void* h, const void* obs, const float* q, int A, const int64_t* actions,
                                const float* rewards, const uint8_t* dones, const void* next_obs);
APEX_RT_API int64_t apex_rt_ns_size(void* h);
APEX_RT_API int64_t apex_rt_ns_take(void* h, int64_t max_items, void* obs, void* nxt, int64_t* act, float* R,
                                    float* G, float* prio, int64_t* key, int64_t* env);

// Common helpers for the apex_dqn_amd CDNA4 (gfx950) kernels.
// Written directly for HIP on gfx950: wave64 everywhere, no CUDA shims.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define APEX_EXPORT extern "C" __attribute__((visibility("default")))
#define APEX_WAVE 64

typedef uint16_t bf16_t;  // raw bf16 bits

__device__ __forceinline__ float bf16_to_f32(bf16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

// round-to-nearest-even f32 -> bf16 (NaN preserved)
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (bf16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

// fp32 pair -> hi / lo packed bf16 planes (v = hi + lo; see mfma_common.h split_pk_bf16)
__device__ __forceinline__ void split_pk_bf16_h(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = pack_bf16x2(a, b);
  lo = pack_bf16x2(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xffff0000u));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// XCD-aware workgroup remap (bijective for any nwg): the dispatcher sends
// workgroup i to XCD i % 8, each XCD with a private 4 MB L2.  Returned ids are
// contiguous per XCD, so tiles that share operand rows (adjacent GEMM tiles,
// the Kc blocks of one wgrad split, the tiles of one frame stack) hit one L2.
__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// full-wave float sum without the LDS crossbar: DPP quad / row rotations reduce each
// 16-lane row, four v_readlane finish.  Result is wave-uniform.
#define APEX_DPP_ADD(v, ctrl)                                                                          \
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, false))
__device__ __forceinline__ float wave_sum_dpp(float v) {
  APEX_DPP_ADD(v, 0xB1);   // quad_perm(1,0,3,2)
  APEX_DPP_ADD(v, 0x4E);   // quad_perm(2,3,0,1)
  APEX_DPP_ADD(v, 0x124);  // row_ror:4
  APEX_DPP_ADD(v, 0x128);  // row_ror:8
  return (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
          __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32)) +
          __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48)));
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_xor(v, o, 64);
    v = v > w ? v : w;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_xor(v, o, 64);
    v = v < w ? v : w;
  }
  return v;
}

// inclusive prefix sum across the 64 lanes of a wave
template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T w = __shfl_up(v, o, 64);
    if (lane >= o) v += w;
  }
  return v;
}

// counter-based RNG (splitmix64 finaliser over (seed, counter, index))
__device__ __forceinline__ uint64_t apex_mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float apex_uniform(uint64_t seed, uint64_t ctr, uint64_t i) {
  uint64_t r = apex_mix64(seed ^ apex_mix64(ctr * 0x100000001b3ull + i));
  return (float)(r >> 40) * (1.0f / 16777216.0f);  // [0,1)
}

#define APEX_CHECK_LAUNCH() return (int)hipGetLastError()

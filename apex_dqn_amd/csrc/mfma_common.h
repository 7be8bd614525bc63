// Shared MFMA / LDS / memory helpers of the CDNA4 (gfx950) GEMM kernels:
// conv_mfma.hip, conv1_s2d.hip, conv1_wgrad.hip.
#pragma once
#include "apex_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));

// uint8 pixels -> f16 (1024 + x), exact for x <= 1023: the f16 with exponent 2^10
// and mantissa x.  Two bytes of `v` (b_i, b_{i+1}) become one f16 pair with a
// single v_perm_b32 (bytes [b_i, 0x64, b_{i+1}, 0x64]); the +1024 offset is a
// per-output-channel constant (1024 * sum of the channel's weights) removed in
// the GEMM epilogue.  3x fewer VALU than cvt_f32_ubyte + cvt_pk_bf16.
__device__ __forceinline__ uint32_t u8pair_f16off(uint32_t v, int hi) {
  return __builtin_amdgcn_perm(0x64646464u, v, hi ? 0x04030402u : 0x04010400u);
}
__device__ __forceinline__ uint4 u8x8_to_f16off(uint32_t lo, uint32_t hi) {
  return make_uint4(u8pair_f16off(lo, 0), u8pair_f16off(lo, 1), u8pair_f16off(hi, 0), u8pair_f16off(hi, 1));
}
// relu on two packed 16-bit floats (bf16 or f16): signed-int16 max with 0
__device__ __forceinline__ uint32_t relu_pk16(uint32_t v) {
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  const s16x2 x = __builtin_bit_cast(s16x2, v);
  const s16x2 z = {0, 0};
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, z));
}

// 128-byte LDS rows, 16-byte chunk c of row r stored at chunk c ^ ((r >> 1) & 7):
// a 16-lane ds_read_b128 group (16 rows, one chunk) hits 16 distinct 16-B slots.
__device__ __forceinline__ int swz_row(int r, int c) { return (r << 7) + ((c ^ ((r >> 1) & 7)) << 4); }
// GEMM epilogue image: 128-B rows, 16-B chunk of byte `byte` in row r at chunk ^ ((r>>1)&7)
__device__ __forceinline__ int epi_off(int r, int byte) {
  return (r << 7) + ((((byte >> 4) ^ ((r >> 1) & 7))) << 4) + (byte & 15);
}
// transposed-read image: chunk16 c of row r at c ^ (s(r) << 1), s(r) = bit1(r) | bit3(r)<<1;
// both ds_read_b64_tr_b16 halves (rows 8g+q, 8(g+1)+q) then cover 64 distinct banks.
__device__ __forceinline__ int swz_tr(int r, int c) {
  const int s = ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
  return (r << 7) + ((c ^ (s << 1)) << 4);
}

// two floats -> packed bf16x2 (one v_cvt_pk_bf16_f32, round-to-nearest-even)
__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){lo, hi}, bf16x2v));
}

// fp32-accurate ("split") operands: v = hi + lo with hi = bf16(v), lo = bf16(v - hi),
// both round-to-nearest-even (v - hi is exact in fp32).  A product of two split
// operands is hi*hi + hi*lo + lo*hi (the lo*lo term is below 2^-16 relative):
// three bf16 MFMAs with fp32 accumulation instead of one fp32 MFMA at 1/16 the rate.
__device__ __forceinline__ void split_pk_bf16(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = cvt_pk_bf16(a, b);
  lo = cvt_pk_bf16(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xffff0000u));
}

// The same split with two scalar v_sub_f32 (asm keeps the compiler from pairing them into
// a v_pk_add_f32, which costs ~13 extra cycles each beside MFMAs: MI355X_MICROARCH.md).
__device__ __forceinline__ void split_pk_bf16_s(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = cvt_pk_bf16(a, b);
  float ra, rb;
  asm("v_sub_f32 %0, %1, %2" : "=v"(ra) : "v"(a), "v"(__uint_as_float(hi << 16)));
  asm("v_sub_f32 %0, %1, %2" : "=v"(rb) : "v"(b), "v"(__uint_as_float(hi & 0xffff0000u)));
  lo = cvt_pk_bf16(ra, rb);
}

__device__ __forceinline__ uint32_t u8pair_bf16(uint32_t v, int sh) {
  // two consecutive bytes of v (starting at byte sh) -> two bf16 (exact: integers <= 255):
  // v_cvt_f32_ubyteN x2 + v_cvt_pk_bf16_f32
  return cvt_pk_bf16((float)((v >> (8 * sh)) & 0xffu), (float)((v >> (8 * sh + 8)) & 0xffu));
}

__device__ __forceinline__ uint4 u8x8_to_bf16x8(uint32_t lo, uint32_t hi) {
  return make_uint4(u8pair_bf16(lo, 0), u8pair_bf16(lo, 2), u8pair_bf16(hi, 0), u8pair_bf16(hi, 2));
}

// ReLU on two packed bf16: zero the halves whose sign bit is set.
// (v & 0x80008000) >> 15 marks negative halves with a 1 in their low bit; x 0xffff
// spreads it over the half (v_mul_u32_u24, no carry between halves); v_bfi clears.
__device__ __forceinline__ uint32_t relu_bf16x2(uint32_t v) {
  const uint32_t neg = ((v & 0x80008000u) >> 15) * 0xffffu;
  return v & ~neg;
}

// dgrad ReLU mask: keep v's half where the producer activation m's half is > 0
// (exact for any bf16 m): |m| + 0x7fff sets bit 15 of a half exactly when its
// magnitude is non-zero (max 0xfffe: no carry into the next half); AND with the
// inverted sign bits drops negative halves (and -0).  (A NaN half of m keeps v;
// torch's m > 0 would drop it -- only reachable after the activations diverged.)
__device__ __forceinline__ uint32_t mask_bf16x2(uint32_t v, uint32_t m) {
  const uint32_t pos = ((m & 0x7fff7fffu) + 0x7fff7fffu) & ~m & 0x80008000u;
  return v & ((pos >> 15) * 0xffffu);
}

// MFMA fragment of 8 consecutive K rows (32kk + 8(lane>>4) .. +7) of column col0 + (lane&15)
// from a K-major 64x64 bf16 image stored with swz_tr (two ds_read_b64_tr_b16).
__device__ __forceinline__ bf16x8 tr_frag8(const uint8_t* img, int kk, int col0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pcol = lane & 3;
  const int rA = 32 * kk + 8 * g + q;
  const int cbyte = (col0 + 4 * pcol) * 2;  // byte offset of 4 columns inside the 128-B row
  const int c16 = cbyte >> 4, within = cbyte & 15;
  const lds_s16x4* pa = (const lds_s16x4*)(img + swz_tr(rA, c16) + within);
  const lds_s16x4* pb = (const lds_s16x4*)(img + swz_tr(rA + 4, c16) + within);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(pa));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4*>(pb));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = (s16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Raw buffer resource over a tensor (< 2 GB): loads with a 32-bit per-lane byte
// offset (loop-invariant VGPR) + a scalar k-tile offset (SGPR), and an offset of
// BUF_OOB reads zeros (hardware range check) -- no per-element selects or branches.
#define BUF_OOB 0x80000000u
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ uint4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// a / D with D a compile-time constant when DC != 0 (multiply-shift), else runtime
template <int DC>
__device__ __forceinline__ uint32_t udiv(uint32_t a, uint32_t d) {
  return DC ? a / (uint32_t)DC : a / d;
}

// 8 uint8 (two dwords) -> 8 bf16: v_cvt_f32_ubyte{0..3} then one v_perm per pair
// picks the high halves of two exact f32 integers (their low halves are zero).
__device__ __forceinline__ uint32_t bf16pair_from_f32(float lo, float hi) {
  return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);
}

// (float)(byte k of v): hipcc lowers this pattern to one v_cvt_f32_ubyte{k}
__device__ __forceinline__ float ubyte(uint32_t v, int k) { return (float)((v >> (8 * k)) & 0xffu); }


// ReLU on two packed bf16 (sign bits spread over their halves, then cleared)
__device__ __forceinline__ uint32_t relu2(uint32_t v) {
  const uint32_t neg = ((v & 0x80008000u) >> 15) * 0xffffu;
  return v & ~neg;
}


// 16-byte LDS-DMA issued from inline asm: hipcc does not track it, so it emits no
// conservative vmcnt(0) before later ds_reads; completion is counted by hand with
// explicit s_waitcnt vmcnt(N) + s_barrier (M0 is written inside the statement).
// the same with a wave-uniform 64-bit base (SGPR pair) and a per-lane 32-bit offset:
// no per-lane address arithmetic
__device__ __forceinline__ void dma16_s(const void* base, uint32_t voff, uint32_t lds_off) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  // (readfirstlane returns int: through uint32_t, or bit 31 of the low half sign-extends)
  const uint64_t sbase = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b) |
                         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_off)
               : "memory");
}

__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_off) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_off)
               : "memory");
}

// 16-byte LDS-DMA through a buffer resource (buffer_load_dwordx4 ... lds): like dma16,
// but offsets past the resource's range read zeros (rows past a GEMM's end).
__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t lds_off) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(r), "s"(lds_off)
               : "memory");
}

// s_waitcnt vmcnt(n) for a run-time n (immediate operand: one branch per value;
// n is wave-uniform, values >= 63 = no wait)
__device__ __forceinline__ void vmcnt_le(int n) {
#define APEX_VMCNT_CASE(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n) {
    APEX_VMCNT_CASE(0) APEX_VMCNT_CASE(1) APEX_VMCNT_CASE(2) APEX_VMCNT_CASE(3) APEX_VMCNT_CASE(4)
    APEX_VMCNT_CASE(5) APEX_VMCNT_CASE(6) APEX_VMCNT_CASE(7) APEX_VMCNT_CASE(8) APEX_VMCNT_CASE(9)
    APEX_VMCNT_CASE(10) APEX_VMCNT_CASE(11) APEX_VMCNT_CASE(12) APEX_VMCNT_CASE(13) APEX_VMCNT_CASE(14)
    APEX_VMCNT_CASE(15) APEX_VMCNT_CASE(16) APEX_VMCNT_CASE(17) APEX_VMCNT_CASE(18) APEX_VMCNT_CASE(19)
    APEX_VMCNT_CASE(20) APEX_VMCNT_CASE(21) APEX_VMCNT_CASE(22) APEX_VMCNT_CASE(23) APEX_VMCNT_CASE(24)
    APEX_VMCNT_CASE(25) APEX_VMCNT_CASE(26) APEX_VMCNT_CASE(27) APEX_VMCNT_CASE(28) APEX_VMCNT_CASE(29)
    APEX_VMCNT_CASE(30) APEX_VMCNT_CASE(31) APEX_VMCNT_CASE(32) APEX_VMCNT_CASE(33) APEX_VMCNT_CASE(34)
    APEX_VMCNT_CASE(35) APEX_VMCNT_CASE(36) APEX_VMCNT_CASE(37) APEX_VMCNT_CASE(38) APEX_VMCNT_CASE(39)
    APEX_VMCNT_CASE(40) APEX_VMCNT_CASE(41) APEX_VMCNT_CASE(42) APEX_VMCNT_CASE(43) APEX_VMCNT_CASE(44)
    APEX_VMCNT_CASE(45) APEX_VMCNT_CASE(46) APEX_VMCNT_CASE(47) APEX_VMCNT_CASE(48) APEX_VMCNT_CASE(49)
    APEX_VMCNT_CASE(50) APEX_VMCNT_CASE(51) APEX_VMCNT_CASE(52) APEX_VMCNT_CASE(53) APEX_VMCNT_CASE(54)
    APEX_VMCNT_CASE(55) APEX_VMCNT_CASE(56) APEX_VMCNT_CASE(57) APEX_VMCNT_CASE(58) APEX_VMCNT_CASE(59)
    APEX_VMCNT_CASE(60) APEX_VMCNT_CASE(61) APEX_VMCNT_CASE(62)
    default: break;
  }
#undef APEX_VMCNT_CASE
}

// ---- device-side work queue of a persistent kernel.  One thread per workgroup fetches
// (vector atomics: one lane's global_atomic_add_x2 with return) from a 64-bit counter
// that is never reset: a launch over n items with G workgroups consumes exactly n + G
// values -- every workgroup fetches until its first value >= n and then stops -- so
// value v means item v mod (n + G) in every launch (no end-of-launch atomics, no memset
// node).  The counter belongs to one (call site, n, G).  Items leave in increasing order.
// (the address goes through an opaque zero in a VGPR: with a uniform address the
// compiler's atomic optimizer broadcasts the result with a readfirstlane right after the
// atomic, i.e. waits for its return there; this way the wait lands where the value is
// first used, after work that hides it)
__device__ __forceinline__ int wq_fetch(unsigned long long* ctr, int n_items) {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  const unsigned long long v = atomicAdd(ctr + z, 1ull);
  return (int)(v % (unsigned long long)(n_items + (int)gridDim.x));
}
// Item source of a persistent kernel: ctr == nullptr gives the static strided order
// (the k-th item of workgroup b is b + k * gridDim.x; `seq` counts k, no atomics); else
// the work queue.  A queue item costs a device-scope atomic round trip, so the learner
// enables the queue only where another kernel can hold CUs during the launch (the conv
// backward beside the data-parallel step's RCCL collectives).
__device__ __forceinline__ int wq_next(unsigned long long* ctr, int& seq, int n_items) {
  if (ctr == nullptr) return (int)blockIdx.x + (seq++) * (int)gridDim.x;
  return wq_fetch(ctr, n_items);
}

// Scalar (SMEM) load of the C frame slots of one image: counted by lgkmcnt, so it
// never forces a vmcnt drain of the LDS-DMA in flight.  `p` must be wave-uniform.
template <int C>
__device__ __forceinline__ void sload_slots(const int32_t* p, int (&out)[4]) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int32_t* q = (const int32_t*)(((uint64_t)hi << 32) | lo);
  if constexpr (C == 4) {
    int __attribute__((ext_vector_type(4))) v;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(q) : "memory");
    out[0] = v[0]; out[1] = v[1]; out[2] = v[2]; out[3] = v[3];
  } else if constexpr (C == 2) {
    int __attribute__((ext_vector_type(2))) v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(q) : "memory");
    out[0] = v[0]; out[1] = v[1]; out[2] = 0; out[3] = 0;
  } else {
    int v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(q) : "memory");
    out[0] = v; out[1] = 0; out[2] = 0; out[3] = 0;
  }
}

// Phase probes for persistent kernels (diagnostic build only: compiled in with
// -DAPEX_PROBE, i.e. in libapex_kernels_debug.so, selected by APEX_DEBUG_BOUNDS=1;
// the release kernels carry no stamps, so their waits are unaffected).  With a
// non-null buffer, lane 0 of every wave of the first PROBE_BLOCKS workgroups
// stores s_memtime (shader clock) at point `pt` of iteration `it` ->
// buf[((block * NW + wave) * PROBE_ITERS + it) * 4 + pt].  scripts/probe_kernels.py.
#define PROBE_BLOCKS 4
#define PROBE_ITERS 16
#ifdef APEX_PROBE
#define PROBE(buf, NW, it, pt)                                                                          \
  do {                                                                                                  \
    if ((buf) != nullptr && blockIdx.x < PROBE_BLOCKS && (it) < PROBE_ITERS && (threadIdx.x & 63) == 0) \
      (buf)[((blockIdx.x * (NW) + (threadIdx.x >> 6)) * PROBE_ITERS + (it)) * 4 + (pt)] =                \
          __builtin_amdgcn_s_memtime();                                                                 \
  } while (0)
#else
#define PROBE(buf, NW, it, pt) \
  do {                         \
  } while (0)
#endif

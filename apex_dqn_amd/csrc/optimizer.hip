// Fused multi-tensor centered RMSprop + global grad-norm clip + bf16 pack.
//
// Reference learner.py:26 builds torch RMSprop(lr=0.00025/4, weight_decay=0.95,
// eps=1.5e-7) (decay passed as L2 weight decay, defect A16) and steps 14
// parameter tensors one by one.  Here the whole 3.3 M-parameter model lives in
// one flat fp32 buffer: one pass computes the squared-norm partials, a second
// applies clip coefficient + centered RMSprop (torch semantics:
//   v = a v + (1-a) g^2;  m = a m + (1-a) g;  p -= lr g / (sqrt(v - m^2) + eps))
// and writes the bf16 compute copy that the MFMA kernels read, so no separate
// cast kernel runs.  Memory-bound: 16 B read + 14 B written per parameter.
#include "rmsprop_common.h"
#include "pack_rows.h"

#define NPART 1024

__global__ void __launch_bounds__(256) sqnorm_partial_kernel(const float* __restrict__ g, int64_t n,
                                                             double* __restrict__ partials) {
  __shared__ double red[4];
  double acc = 0.0;
  const int64_t n4 = n / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = g4[i];
    acc += (double)(v.x * v.x + v.y * v.y) + (double)(v.z * v.z + v.w * v.w);
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc += (double)g[i] * g[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) rmsprop_kernel(RmspropArgs a) { rmsprop_body(a, blockIdx.x, gridDim.x); }

// fp32 -> bf16 copy; with `lo` also the residual plane (x = y + lo: fp32-accurate mode)
__global__ void cast_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, bf16_t* __restrict__ lo,
                                 int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bf16_t h = f32_to_bf16(x[i]);
    y[i] = h;
    if (lo != nullptr) lo[i] = f32_to_bf16(x[i] - bf16_to_f32(h));
  }
}

APEX_EXPORT int apex_grad_sqnorm_partials(const float* g, int64_t n, double* partials, hipStream_t st) {
  sqnorm_partial_kernel<<<NPART, 256, 0, st>>>(g, n, partials);
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_rmsprop_step(float* p, const float* g, float* v, float* m, bf16_t* pb, int64_t n,
                                  const double* partials, float lr, float alpha, float eps, float clip,
                                  int centered, float* norm_out, bf16_t* pb_lo, const double* wnorm, int wn,
                                  int wstride, hipStream_t st) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)v | (uintptr_t)m) & 15) return (int)hipErrorInvalidValue;
  if (((uintptr_t)pb | (uintptr_t)pb_lo) & 7) return (int)hipErrorInvalidValue;
  int nb = (int)((n / 4 + 255) / 256);
  nb = nb < 1 ? 1 : (nb > 2048 ? 2048 : nb);
  rmsprop_kernel<<<nb, 256, 0, st>>>(RmspropArgs{p, g, v, m, pb, n, partials, NPART, lr, alpha, eps, clip, centered,
                                                 norm_out, pb_lo, wnorm, wn, wstride, CfFragOut{}});
  APEX_CHECK_LAUNCH();
}

// the same step with the clip norm taken from ``npart`` producer-written partials
// (fc wgrad epilogue + grad_finalize blocks): no separate squared-norm pass
APEX_EXPORT int apex_rmsprop_step_np(float* p, const float* g, float* v, float* m, bf16_t* pb, int64_t n,
                                     const double* partials, int npart, float lr, float alpha, float eps, float clip,
                                     int centered, float* norm_out, bf16_t* pb_lo, const double* wnorm, int wn,
                                  int wstride, hipStream_t st) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)v | (uintptr_t)m) & 15) return (int)hipErrorInvalidValue;
  if (((uintptr_t)pb | (uintptr_t)pb_lo) & 7) return (int)hipErrorInvalidValue;
  int nb = (int)((n / 4 + 255) / 256);
  nb = nb < 1 ? 1 : (nb > 2048 ? 2048 : nb);
  rmsprop_kernel<<<nb, 256, 0, st>>>(RmspropArgs{p, g, v, m, pb, n, partials, npart, lr, alpha, eps, clip, centered,
                                                 norm_out, pb_lo, wnorm, wn, wstride, CfFragOut{}});
  APEX_CHECK_LAUNCH();
}

APEX_EXPORT int apex_cast_bf16(const float* x, bf16_t* y, int64_t n, bf16_t* lo, hipStream_t st) {
  int nb = (int)((n + 255) / 256);
  nb = nb > 2048 ? 2048 : (nb < 1 ? 1 : nb);
  cast_bf16_kernel<<<nb, 256, 0, st>>>(x, y, lo, n);
  APEX_CHECK_LAUNCH();
}

// ------------------------------------------------ data-parallel fc-gradient factors
// (csrc/pack_rows.h)
__global__ void __launch_bounds__(256) pack_rows_kernel(PackRows p) { pack_rows_body(p, blockIdx.x, gridDim.x); }

APEX_EXPORT int apex_pack_rows(const uint16_t* const* src, const int64_t* ld, const int* cols, int nseg, int rows,
                               uint16_t* dst, int64_t dld, hipStream_t st) {
  PackRows p;
  int64_t nchunks = 0;
  const int err = make_pack_rows(src, ld, cols, nseg, rows, dst, dld, p, nchunks);
  if (err) return err;
  if (rows == 0) return 0;
  int nb = (int)((nchunks + 255) / 256);
  nb = nb > 1024 ? 1024 : nb;
  pack_rows_kernel<<<nb, 256, 0, st>>>(p);
  APEX_CHECK_LAUNCH();
}

// Squared-norm partials of two fp32 ranges (the all-reduced conv + head gradient
// regions of the factored DP step; the fc part's partials come from its wgrad
// epilogue): `nblk` partials into `partials`.
__global__ void __launch_bounds__(256) sqnorm_ranges_kernel(const float* __restrict__ p0, int64_t n0,
                                                            const float* __restrict__ p1, int64_t n1,
                                                            double* __restrict__ partials) {
  __shared__ double red[4];
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int r = 0; r < 2; ++r) {
    const float* g = r ? p1 : p0;
    const int64_t n = r ? n1 : n0;
    if (g == nullptr) continue;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const float v = g[i];
      acc += (double)v * v;
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

APEX_EXPORT int apex_sqnorm_ranges(const float* p0, int64_t n0, const float* p1, int64_t n1, double* partials,
                                   int nblk, hipStream_t st) {
  if (nblk < 1 || nblk > 1024) return (int)hipErrorInvalidValue;
  sqnorm_ranges_kernel<<<nblk, 256, 0, st>>>(p0, n0, p1, n1, partials);
  APEX_CHECK_LAUNCH();
}

// Several device copies in ONE launch (grid.y = segment): the emulated world's stand-in
// for an RCCL group (parallel/rccl.py EmulatedCollectives.fused) -- RCCL launches a
// group's collectives as one kernel, so the emulation issues one copy kernel per group
// instead of one per member.  16-B chunks where both ends are 16-B aligned, bytes else.
#define COPY_SEGS 32
struct CopySegs {
  const uint8_t* src[COPY_SEGS];
  uint8_t* dst[COPY_SEGS];
  int64_t bytes[COPY_SEGS];
};

__global__ void __launch_bounds__(256) copy_segments_kernel(CopySegs c) {
  const int s = blockIdx.y;
  const uint8_t* src = c.src[s];
  uint8_t* dst = c.dst[s];
  const int64_t nb = c.bytes[s];
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int64_t n16 = nb >> 4;
    for (int64_t i = t0; i < n16; i += stride)
      reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    for (int64_t i = (n16 << 4) + t0; i < nb; i += stride) dst[i] = src[i];
  } else {
    for (int64_t i = t0; i < nb; i += stride) dst[i] = src[i];
  }
}

APEX_EXPORT int apex_copy_segments(int n, const int64_t* src, const int64_t* dst, const int64_t* bytes,
                                   hipStream_t st) {
  if (n < 1 || n > COPY_SEGS) return (int)hipErrorInvalidValue;
  CopySegs c{};
  int64_t mx = 0;
  for (int i = 0; i < n; ++i) {
    if (bytes[i] < 0 || (bytes[i] > 0 && (src[i] == 0 || dst[i] == 0))) return (int)hipErrorInvalidValue;
    c.src[i] = reinterpret_cast<const uint8_t*>(src[i]);
    c.dst[i] = reinterpret_cast<uint8_t*>(dst[i]);
    c.bytes[i] = bytes[i];
    mx = bytes[i] > mx ? bytes[i] : mx;
  }
  int64_t bx = (mx / 16 + 255) / 256;
  bx = bx < 1 ? 1 : (bx > 1024 ? 1024 : bx);
  copy_segments_kernel<<<dim3((unsigned)bx, (unsigned)n), 256, 0, st>>>(c);
  APEX_CHECK_LAUNCH();
}

// Row pack of up to 4 (src, src row stride, cols) segments of 16-bit values into one
// [rows][ld] buffer: the send rows of the factored fc-gradient exchange
// (learner/dp_step.py: [dH | dH lo | y3 | y3 lo] per sample, one all-gather instead of
// an all-reduce of the 1024 x 3136 gradient).  16-B chunks, every column count and
// stride a multiple of 8.  Run by csrc/optimizer.hip pack_rows_kernel and by the tail
// blocks of csrc/sumtree.hip head_wgrad_prio_kernel (the DP step's head launch).
#pragma once
#include "apex_common.h"

struct PackRows {
  const uint16_t* src[4];
  int64_t ld[4];
  int cols[4];
  int nseg, rows;
  uint16_t* dst;
  int64_t dld;
};

// block `bid` of `nblk` (grid-stride over the 16-B chunks)
__device__ __forceinline__ void pack_rows_body(const PackRows& p, int bid, int nblk) {
  int tot = 0;
  for (int s = 0; s < p.nseg; ++s) tot += p.cols[s] >> 3;
  const int64_t nchunks = (int64_t)p.rows * tot;
  for (int64_t c = (int64_t)bid * blockDim.x + threadIdx.x; c < nchunks; c += (int64_t)nblk * blockDim.x) {
    const int r = (int)(c / tot);
    int k = (int)(c - (int64_t)r * tot), s = 0, col0 = 0;
    while (k >= (p.cols[s] >> 3)) {
      k -= p.cols[s] >> 3;
      col0 += p.cols[s];
      ++s;
    }
    const uint4 v = *reinterpret_cast<const uint4*>(p.src[s] + (int64_t)r * p.ld[s] + 8 * k);
    *reinterpret_cast<uint4*>(p.dst + (int64_t)r * p.dld + col0 + 8 * k) = v;
  }
}

// host: validated PackRows from the segment arrays (hipErrorInvalidValue on a bad shape)
static inline int make_pack_rows(const uint16_t* const* src, const int64_t* ld, const int* cols, int nseg, int rows,
                                 uint16_t* dst, int64_t dld, PackRows& p, int64_t& nchunks) {
  if (nseg < 1 || nseg > 4 || rows < 0 || (dld & 7) || ((uintptr_t)dst & 15)) return (int)hipErrorInvalidValue;
  p = PackRows{};
  int tot = 0;
  for (int s = 0; s < nseg; ++s) {
    if ((cols[s] & 7) || (ld[s] & 7) || ((uintptr_t)src[s] & 15)) return (int)hipErrorInvalidValue;
    p.src[s] = src[s];
    p.ld[s] = ld[s];
    p.cols[s] = cols[s];
    tot += cols[s];
  }
  if (tot > dld) return (int)hipErrorInvalidValue;
  p.nseg = nseg;
  p.rows = rows;
  p.dst = dst;
  p.dld = dld;
  nchunks = (int64_t)rows * (tot >> 3);
  return 0;
}

// seed.h — the serial seeding step of StandardNLSFitter._fit_parallel
// (fitters.py:403-410): buffer 0 of every record is demodulated and fitted from
// the default guess; its result seeds every other buffer of that record.
//
// One workgroup (one wavefront) per record: the wave demodulates the record's
// buffer 0 (fold_segment / direct_segment, basis table read through the cache),
// then lane 0 runs the per-segment LM. The host launches this kernel on a
// SIDE stream, concurrently with the bulk demodulation on the main stream, and
// the bulk LM waits on an event: the seed costs no wall time as long as it is
// shorter than the bulk demodulation.
#pragma once
#include "demod.h"
#include "lm.h"

namespace dfmi {

template <int NDMAX>
__global__ __launch_bounds__(64, 4) void seed_kernel(const double* __restrict__ x, int64_t rec_stride, int R, int L,
                                                  int ndata, double w0, const double* __restrict__ tab,
                                                  double* __restrict__ qis, double* __restrict__ dcs, int64_t nrec,
                                                  const double* __restrict__ guess, GuessInline ginl, int use_inline,
                                                  const double* __restrict__ jtab, LMConst c,
                                                  double* __restrict__ out, int64_t out_ld, int64_t nbuf,
                                                  int32_t* __restrict__ status) {
  const int64_t r = blockIdx.x;
  const int lane = threadIdx.x;
  const double* __restrict__ xs = x + r * rec_stride;
  if (L > 0) fold_segment<1, 16>(xs, R, L, ndata, tab, lane, qis, nrec, r, dcs);
  else direct_segment(xs, R, ndata, w0, lane, qis, nrec, r, dcs);
  __syncthreads();  // QI of this record (global, same workgroup) visible to lane 0
  if (lane != 0) return;
  double p[4] = {0.0, 0.0, 0.0, 0.0};
  if (use_inline) {
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      if (r == rr) {
#pragma unroll
        for (int i = 0; i < 4; ++i) p[i] = ginl.v[rr][i];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = guess[r * 4 + i];
  }
  double ssq;
  const int st = fit_segment<NDMAX>(qis + r, nrec, ndata, jtab, c, p, ssq);
  const int64_t sidx = r * nbuf;
  out[0 * out_ld + sidx] = p[0];
  out[1 * out_ld + sidx] = p[1];
  out[2 * out_ld + sidx] = p[2];
  out[3 * out_ld + sidx] = p[3];
  out[5 * out_ld + sidx] = ssq;
  status[sidx] = st;
}

}  // namespace dfmi

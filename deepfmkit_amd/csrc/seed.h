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

// The seed fit runs the GENERAL LM path (literal coeffs + pivoting msolve, two-pass
// Bessel walk: no stored Bessel / trig state) in every seed kernel: in the fused
// kernel the seed shares the bulk demodulation's 168-VGPR budget (3 waves per SIMD),
// which the register path's trial state would exceed; one lane's fit beside a
// ~0.5 ms demodulation costs no wall time either way. Same path in every variant,
// so the seed (and with it every chunk's start) does not depend on the scheduling.
constexpr int kSeedPath = 0;

// The seed's fit is run by a WHOLE wave: the lambda ladder of every LM iteration is tried
// 8 rungs at a time by 8-lane groups (lm_descend_ladder, FLAT = 2: bit-identical to the
// one-lane descent, tests/test_gpu_numerics.py::test_lm_ladder_bit_identical); every group
// of the wave runs the same fit and lane 0 writes it. A seed whose descent walks the whole
// ladder at many iterations (records whose phase the default guess does not reach, e.g.
// phi = 1.3, psi = 0.4: ~27 ms one lane at a time) then costs ~1/8 of the
// passes, so it stays hidden under (or close to) the bulk demodulation.
constexpr int kSeedFlat = 2;

// tabT (not null): the many-harmonic demodulation (demod.h wide_seed_segment, basis_table_wide
// with `no` output slices; dynamic LDS L + 4 doubles): the record's buffer 0 gets the QI the
// bulk demod_wide_kernel would give it.
// SFLAT: the seed's descent — kSeedFlat (8 rungs by 8-lane groups, every group the same fit) or,
// beyond 16 harmonics (tuning seed_wave_split), 3: the wave's 64 lanes as 8 rungs x 8 harmonic
// shares (lm.h PartFullEval), one fit.
template <int NDMAX, int SFLAT = kSeedFlat>
__global__ __launch_bounds__(64) void seed_kernel(const double* __restrict__ x, int64_t rec_stride, int R, int L,
                                                  int ndata, double w0, const double* __restrict__ tab,
                                                  double* __restrict__ qis, double* __restrict__ dcs, int64_t nrec,
                                                  const double* __restrict__ guess, GuessInline ginl, int use_inline,
                                                  const double* __restrict__ jtab, LMConst c,
                                                  double* __restrict__ out, int64_t out_ld, int64_t nbuf,
                                                  int32_t* __restrict__ status, const double* __restrict__ tabT,
                                                  int no) {
  extern __shared__ __attribute__((aligned(16))) double ybin_dyn[];
  const int64_t r = blockIdx.x;
  const int lane = threadIdx.x;
  const double* __restrict__ xs = x + r * rec_stride;
  if (tabT) wide_seed_segment(xs, R, L, ndata, tabT, no, ybin_dyn, lane, qis, nrec, r, dcs);
  else if (L > 0) fold_segment<1, 16>(xs, R, L, ndata, tab, lane, qis, nrec, r, dcs);
  else direct_segment(xs, R, ndata, w0, lane, qis, nrec, r, dcs);
  __syncthreads();  // QI of this record (global, same workgroup) visible to the wave
  // ... and into LDS for the fit: its evaluations read every QI value once per harmonic, and
  // from global memory each read waited a round trip under the bulk demodulation's load
  // (the kernel took 0.36 / 0.47 / 0.61 ms at ndata 20 / 30 / 62, longer than the bulk
  // demodulation at 62; profiles/r05/ndata_sweep_kernel_stats.csv). Same values: same fit.
  __shared__ double qsh[2 * 128];
  for (int i = lane; i < 2 * ndata && i < 2 * 128; i += 64) qsh[i] = qis[(int64_t)i * nrec + r];
  __syncthreads();
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
  const QGlobal qs{ndata <= 128 ? qsh : qis + r, ndata <= 128 ? 1 : nrec, ndata};
  // NDMAX == kWideNd / kWideNdF (more than 16 harmonics, lm_wide / lm_wide_fused): the
  // many-harmonic evaluation, as the bulk LM that this seed's result seeds
  const int st = fit_segment_q<(wide_nd(NDMAX) ? NDMAX : kSeedPath), QGlobal, SFLAT>(qs, ndata, jtab, c, p, ssq);
  if (lane != 0) return;
  const int64_t sidx = r * nbuf;
  out[0 * out_ld + sidx] = p[0];
  out[1 * out_ld + sidx] = p[1];
  out[2 * out_ld + sidx] = p[2];
  out[3 * out_ld + sidx] = p[3];
  out[5 * out_ld + sidx] = ssq;
  status[sidx] = st;
}

// Seed step for inputs the bin kernel handles (16-B rows, even L in [128, 1024]):
// the wave folds its record's buffer 0 with 16 chunk loads in flight into LDS bins,
// contracts it into an LDS row (the demodulation row layout, dfmi_row_stride), and
// lane 0 fits it reading QI from LDS — no memory traffic inside the LM and no
// register cap, so the fit runs at its own instruction latency even while the bulk
// demodulation saturates HBM (seed_kernel, with QI in global memory and a
// 128-VGPR cap, took as long as the whole demodulation beside it:
// profiles/r01b_seed_timeline.txt). Same QI, dc and fit as the bulk path.
template <int NDMAX, int MAXSLOT>
__global__ __launch_bounds__(64) void seed_bins_kernel(const double* __restrict__ x, int64_t rec_stride, int R, int L,
                                                       int ndata, const double* __restrict__ tab,
                                                       const double* __restrict__ guess, GuessInline ginl,
                                                       int use_inline, const double* __restrict__ jtab, LMConst c,
                                                       double* __restrict__ out, int64_t out_ld, int64_t nbuf,
                                                       int32_t* __restrict__ status, uint64_t* __restrict__ probe,
                                                       int write_dc) {
  // probe (diagnostics, may be null): s_memrealtime (100 MHz) at entry, after the
  // fold, after the fit, written by record 0. write_dc = 0: the bulk demodulation beside this
  // kernel writes buffer 0's dc itself (component-major QI + dc), so this kernel leaves it
  // alone — one writer, the same bits every run
  const uint64_t t_in = __builtin_amdgcn_s_memrealtime();
  extern __shared__ __attribute__((aligned(16))) double sh[];  // basis | bins [L] | row
  const int64_t r = blockIdx.x;
  const int lane = threadIdx.x;
  __builtin_amdgcn_s_setprio(3);  // ahead of the demodulation waves sharing this SIMD
  const int ntab = 2 * ndata * L;  // even (L even)
  {
    // basis table -> LDS with every load in flight at once (a load-then-store loop
    // pays one memory round trip per iteration, which under the bulk
    // demodulation's HBM saturation is several microseconds each)
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v* __restrict__ src = reinterpret_cast<const d2v*>(tab);
    d2v* dst = reinterpret_cast<d2v*>(sh);
    const int n2 = ntab / 2;
    for (int base = 0; base < n2; base += 64 * 32) {
      d2v v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const int i = base + u * 64 + lane;
        v[u] = i < n2 ? src[i] : d2v{0.0, 0.0};
      }
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const int i = base + u * 64 + lane;
        if (i < n2) dst[i] = v[u];
      }
    }
  }
  __syncthreads();
  double* ybin = sh + ntab;
  double* row = ybin + L;
  const int nslot = (L + 127) / 128;
  int pbase[MAXSLOT];
  bool pval[MAXSLOT];
#pragma unroll
  for (int j = 0; j < MAXSLOT; ++j) {
    pbase[j] = 2 * (lane + 64 * j);
    pval[j] = (j < nslot) && (pbase[j] < L);
  }
  bins_segment<MAXSLOT, 32, false, kHarmBlock, true, 0, true>(x + r * rec_stride, R, L, ndata, sh, ybin, lane, pval, pbase,
                                                        row, 0, 0, nullptr);
  __syncthreads();
  const uint64_t t_fold = __builtin_amdgcn_s_memrealtime();
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
  const QRow<1> q{row};
  const int st = fit_segment_q<kSeedPath, QRow<1>, kSeedFlat>(q, ndata, jtab, c, p, ssq);
  if (lane != 0) return;
  const int64_t sidx = r * nbuf;
  out[0 * out_ld + sidx] = p[0];
  out[1 * out_ld + sidx] = p[1];
  out[2 * out_ld + sidx] = p[2];
  out[3 * out_ld + sidx] = p[3];
  if (write_dc) out[4 * out_ld + sidx] = q.at(dfmi_row_dc(ndata));
  out[5 * out_ld + sidx] = ssq;
  status[sidx] = st;
  if (probe && r == 0) {
    probe[0] = t_in;
    probe[1] = t_fold;
    probe[2] = __builtin_amdgcn_s_memrealtime();
  }
}

}  // namespace dfmi

namespace dfmi {

// Seed + bulk demodulation in ONE launch (record pipeline, row layout): workgroups
// 0..nrec-1 are the seed step of record blockIdx.x (wave 0 folds buffer 0 into LDS
// bins and contracts it into an LDS row, lane 0 fits it — seed_bins_kernel's work),
// the others are the persistent bin demodulation of all nseg segments
// (demod_bins_kernel's work). Lower block indices dispatch first, so the seeds are
// resident from the start without a second queue, an event, or idle "spacer"
// workgroups; the LM follows on the same stream. Records are contiguous (segment s
// at x + s*R). The kernel is held to the bin kernel's 3-waves-per-SIMD register budget
// (168 VGPRs): the seed's whole-wave ladder fit (round 4) wants 223, which cost the BULK
// demodulation a third of its occupancy (0.497 -> 0.530 ms, r04q); capped, the seed's
// overflow goes to scratch in the one wave that fits (DFMI_SEED_WAVES 0: no cap, A/B builds).
#ifndef DFMI_SEED_WAVES
#define DFMI_SEED_WAVES 3
#endif
#if DFMI_SEED_WAVES > 0
#define DFMI_SEED_BOUNDS __launch_bounds__(kBlockThreads, DFMI_SEED_WAVES)
#else
#define DFMI_SEED_BOUNDS __launch_bounds__(kBlockThreads)
#endif
template <int MAXSLOT, int NDMAX, int PFN = 0, int LOADS = 8>
__global__ DFMI_SEED_BOUNDS void demod_seed_bins_kernel(
    const double* __restrict__ x, int64_t nseg, int64_t rec_stride, int64_t nrec, int R, int L, int ndata,
    const double* __restrict__ tab, double* __restrict__ rows, int64_t row_ld, const double* __restrict__ guess,
    GuessInline ginl, int use_inline, const double* __restrict__ jtab, LMConst c, double* __restrict__ out,
    int64_t out_ld, int64_t nbuf, int32_t* __restrict__ status, uint64_t* __restrict__ probe) {
  if ((int64_t)blockIdx.x >= nrec) {
    bins_kernel_body<MAXSLOT, LOADS, true, PFN>(x, nseg, (int64_t)R, R, L, ndata, tab, rows, row_ld, nullptr, probe,
                                                (int)nrec);
    return;
  }
  const uint64_t t_in = __builtin_amdgcn_s_memrealtime();
  extern __shared__ __attribute__((aligned(16))) double sh[];  // basis | bins [L] | row
  const int64_t r = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_amdgcn_s_setprio(3);
  const int ntab = 2 * ndata * L;
  {
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v* __restrict__ src = reinterpret_cast<const d2v*>(tab);
    d2v* dst = reinterpret_cast<d2v*>(sh);
    const int n2 = ntab / 2;
    for (int base = 0; base < n2; base += kBlockThreads * 8) {
      d2v v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * kBlockThreads + (int)threadIdx.x;
        v[u] = i < n2 ? src[i] : d2v{0.0, 0.0};
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * kBlockThreads + (int)threadIdx.x;
        if (i < n2) dst[i] = v[u];
      }
    }
  }
  __syncthreads();
  double* ybin = sh + ntab;
  double* row = ybin + L;
  if (wave == 0) {
    const int nslot = (L + 127) / 128;
    int pbase[MAXSLOT];
    bool pval[MAXSLOT];
#pragma unroll
    for (int j = 0; j < MAXSLOT; ++j) {
      pbase[j] = 2 * (lane + 64 * j);
      pval[j] = (j < nslot) && (pbase[j] < L);
    }
    bins_segment<MAXSLOT, 32, false, kHarmBlock, true, 0, true>(x + r * rec_stride, R, L, ndata, sh, ybin, lane, pval, pbase,
                                                          row, 0, 0, nullptr);
  }
  __syncthreads();
  const uint64_t t_fold = __builtin_amdgcn_s_memrealtime();
  if (wave != 0) return;
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
  const QRow<1> q{row};
  const int st = fit_segment_q<kSeedPath, QRow<1>, kSeedFlat>(q, ndata, jtab, c, p, ssq);
  if (lane != 0) return;
  const int64_t sidx = r * nbuf;
  out[0 * out_ld + sidx] = p[0];
  out[1 * out_ld + sidx] = p[1];
  out[2 * out_ld + sidx] = p[2];
  out[3 * out_ld + sidx] = p[3];
  out[4 * out_ld + sidx] = q.at(dfmi_row_dc(ndata));
  out[5 * out_ld + sidx] = ssq;
  status[sidx] = st;
  if (probe && r == 0) {
    probe[0] = t_in;
    probe[1] = t_fold;
    probe[2] = __builtin_amdgcn_s_memrealtime();
  }
}

}  // namespace dfmi

// demod.h — harmonic pick-off (demodulation) kernels for gfx950.
//
// Reference: fit.py:18-66 (calculate_quadratures) + fitters.py:45-49,57 (the
// per-buffer mean of x·cos((n+1)·w0·t), x·sin(...), t = 0..R-1, and dc = mean(x)).
//
// Fold kernel (the hot one). When the demodulation basis is periodic with an
// integer period of L samples (L·w0 = 2π·integer; L = f_samp/f_mod = 200 at the
// BASELINE configs) the correlation is computed as
//     Q_h = (1/R) Σ_{p<L} cos(h·w0·p) · y[p],   y[p] = Σ_k x[p + k·L]
// i.e. every sample is ADDED once into its phase bin (1 flop/sample) and the
// tiny L × 2·ndata contraction runs once per segment. The kernel is then a
// pure HBM stream: algorithmic bytes per segment = 8·R (read) + 8·(2·ndata+1)
// (write), no per-sample transcendental and no per-sample basis read.
//
// Layout: one wavefront owns one segment at a time (persistent grid-stride over
// segments). Lane l owns the phase bins p = VEC·(l + 64·j) + e (j < nslot,
// e < VEC); a cycle of L samples is then read as nslot coalesced wave loads of
// 64·VEC contiguous doubles (16 B per lane when VEC = 2). The basis table
// (2·ndata × L doubles: cos rows then sin rows, built on the host with
// angle = fl(h·w0)·p exactly as the reference forms it) lives in LDS, shared by
// the 4 waves of the workgroup. The 2·ndata lane-partial sums are reduced with
// a reduce-scatter butterfly over the 64 lanes (16 values → 17 shuffles per
// block of 8 harmonics, instead of 16×6).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfmi {

constexpr int kWavesPerBlock = 4;
constexpr int kBlockThreads = 64 * kWavesPerBlock;
constexpr int kHarmBlock = 8;  // harmonics per contraction block (16 partial sums)

// Reduce-scatter of 16 per-lane partial sums over a wavefront. On return lane l
// holds, in v[0], the wave-wide sum of value index (l >> 2) & 15.
__device__ __forceinline__ void butterfly16(double (&v)[16], int lane) {
  {
    const bool hi = lane & 32;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const double send = hi ? v[i] : v[i + 8];
      const double keep = hi ? v[i + 8] : v[i];
      v[i] = keep + __shfl_xor(send, 32);
    }
  }
  {
    const bool hi = lane & 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const double send = hi ? v[i] : v[i + 4];
      const double keep = hi ? v[i + 4] : v[i];
      v[i] = keep + __shfl_xor(send, 16);
    }
  }
  {
    const bool hi = lane & 8;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const double send = hi ? v[i] : v[i + 2];
      const double keep = hi ? v[i + 2] : v[i];
      v[i] = keep + __shfl_xor(send, 8);
    }
  }
  {
    const bool hi = lane & 4;
    const double send = hi ? v[0] : v[1];
    const double keep = hi ? v[1] : v[0];
    v[0] = keep + __shfl_xor(send, 4);
  }
  v[0] += __shfl_xor(v[0], 2);
  v[0] += __shfl_xor(v[0], 1);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <int VEC>
struct VecT;
template <>
struct VecT<1> {
  using T = double;
  __device__ static __forceinline__ void load(const double* p, double (&o)[1]) { o[0] = *p; }
  __device__ static __forceinline__ void load_nt(const double* p, double (&o)[1]) {
    o[0] = __builtin_nontemporal_load(p);
  }
};
template <>
struct VecT<2> {
  using T = double2;
  __device__ static __forceinline__ void load(const double* p, double (&o)[2]) {
    const double2 v = *reinterpret_cast<const double2*>(p);
    o[0] = v.x;
    o[1] = v.y;
  }
  __device__ static __forceinline__ void load_nt(const double* p, double (&o)[2]) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    o[0] = v.x;
    o[1] = v.y;
  }
};

// Write one block of 8 harmonics (16 sums) of segment s.
__device__ __forceinline__ void store_block(const double (&v)[16], int lane, int hb, int ndata,
                                            double* __restrict__ qi, int64_t qi_ld, int64_t s, int R) {
  if ((lane & 3) == 0) {
    const int vi = lane >> 2;
    const int h = hb * kHarmBlock + (vi & 7);
    if (h < ndata) {
      const int c = (vi >> 3) ? (ndata + h) : h;
      qi[(int64_t)c * qi_ld + s] = v[0] / (double)R;  // numpy mean: sum / count
    }
  }
}

// One segment, one wavefront: fold + dc + contraction (see the header comment).
// T: basis table (LDS or global), col: the segment's column in qi / dc.
// MAXSLOT: compile-time bound on nslot = ceil(L / (64·VEC)); LOADS: vector loads
// kept in flight per lane in the fold loop; NT: non-temporal (streaming) loads.
template <int VEC, int MAXSLOT, int LOADS = 8, bool NT = true>
__device__ __forceinline__ void fold_segment(const double* __restrict__ xs, int R, int L, int ndata,
                                             const double* __restrict__ T, int lane, double* __restrict__ qi,
                                             int64_t qi_ld, int64_t col, double* __restrict__ dc) {
  const int nslot = (L + 64 * VEC - 1) / (64 * VEC);
  const int ncyc = R / L;
  const int rem = R - ncyc * L;
  constexpr int UNR = (MAXSLOT >= LOADS) ? 1 : (LOADS / MAXSLOT);
  const int nblk = (ndata + kHarmBlock - 1) / kHarmBlock;
  int pbase[MAXSLOT];
  bool pval[MAXSLOT];
#pragma unroll
  for (int j = 0; j < MAXSLOT; ++j) {
    pbase[j] = VEC * (lane + 64 * j);
    pval[j] = (j < nslot) && (pbase[j] < L);
  }
  double y[MAXSLOT][VEC];
#pragma unroll
  for (int j = 0; j < MAXSLOT; ++j)
#pragma unroll
    for (int e = 0; e < VEC; ++e) y[j][e] = 0.0;

  // ---- fold: y[p] += x[p + k L] over the full cycles ----
  int k = 0;
  for (; k + UNR <= ncyc; k += UNR) {
    double v[UNR][MAXSLOT][VEC];
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int j = 0; j < MAXSLOT; ++j) {
        if (pval[j]) {
          if constexpr (NT) VecT<VEC>::load_nt(xs + (int64_t)(k + u) * L + pbase[j], v[u][j]);
          else VecT<VEC>::load(xs + (int64_t)(k + u) * L + pbase[j], v[u][j]);
        }
        else {
#pragma unroll
          for (int e = 0; e < VEC; ++e) v[u][j][e] = 0.0;
        }
      }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int j = 0; j < MAXSLOT; ++j)
#pragma unroll
        for (int e = 0; e < VEC; ++e) y[j][e] += v[u][j][e];
  }
  for (; k < ncyc; ++k) {
#pragma unroll
    for (int j = 0; j < MAXSLOT; ++j) {
      if (pval[j]) {
        double v[VEC];
        VecT<VEC>::load(xs + (int64_t)k * L + pbase[j], v);
#pragma unroll
        for (int e = 0; e < VEC; ++e) y[j][e] += v[e];
      }
    }
  }
  if (rem) {  // ragged last cycle: element-wise bounds
    const double* xr = xs + (int64_t)ncyc * L;
#pragma unroll
    for (int j = 0; j < MAXSLOT; ++j)
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        if (pval[j] && pbase[j] + e < rem) y[j][e] += xr[pbase[j] + e];
  }

  // ---- dc = mean(x) ----
  double tot = 0.0;
#pragma unroll
  for (int j = 0; j < MAXSLOT; ++j)
#pragma unroll
    for (int e = 0; e < VEC; ++e) tot += y[j][e];
  tot = wave_sum(tot);
  if (lane == 0) dc[col] = tot / (double)R;

  // ---- contraction with the basis, 8 harmonics per block ----
  for (int hb = 0; hb < nblk; ++hb) {
    double acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0;
#pragma unroll
    for (int j = 0; j < MAXSLOT; ++j) {
      if (!pval[j]) continue;
#pragma unroll
      for (int h = 0; h < kHarmBlock; ++h) {
        const int hh = hb * kHarmBlock + h;
        if (hh < ndata) {
          double bc[VEC], bs[VEC];
          VecT<VEC>::load(T + (int64_t)hh * L + pbase[j], bc);
          VecT<VEC>::load(T + (int64_t)(ndata + hh) * L + pbase[j], bs);
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            acc[h] = fma(y[j][e], bc[e], acc[h]);
            acc[8 + h] = fma(y[j][e], bs[e], acc[8 + h]);
          }
        }
      }
    }
    butterfly16(acc, lane);
    store_block(acc, lane, hb, ndata, qi, qi_ld, col, R);
  }
}

template <int VEC, int MAXSLOT, bool LDS_TAB, int LOADS = 8, bool NT = true>
__global__ __launch_bounds__(kBlockThreads) void demod_fold_kernel(
    const double* __restrict__ x, int64_t nseg, int64_t seg_stride, int R, int L, int ndata,
    const double* __restrict__ tab, double* __restrict__ qi, int64_t qi_ld, double* __restrict__ dc) {
  extern __shared__ __attribute__((aligned(16))) double lds_tab[];
  if constexpr (LDS_TAB) {
    const int n = 2 * ndata * L;
    for (int i = threadIdx.x; i < n; i += kBlockThreads) lds_tab[i] = tab[i];
    __syncthreads();
  }
  const double* __restrict__ T = LDS_TAB ? lds_tab : tab;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  for (int64_t s = (int64_t)blockIdx.x * kWavesPerBlock + wave; s < nseg;
       s += (int64_t)gridDim.x * kWavesPerBlock) {
    fold_segment<VEC, MAXSLOT, LOADS, NT>(x + s * seg_stride, R, L, ndata, T, lane, qi, qi_ld, s, dc);
  }
}

// Fallback when no short integer period exists: per-sample angles
// fl(fl(h·w0)·t) exactly as fit.py:55-64 forms them, sincos on the device.
// VALU-bound; only used for unusual f_samp/f_mod ratios.
__device__ __forceinline__ void direct_segment(const double* __restrict__ xs, int R, int ndata, double w0, int lane,
                                               double* __restrict__ qi, int64_t qi_ld, int64_t col,
                                               double* __restrict__ dc) {
  const int nblk = (ndata + kHarmBlock - 1) / kHarmBlock;
  double tot = 0.0;
  for (int t = lane; t < R; t += 64) tot += xs[t];
  tot = wave_sum(tot);
  if (lane == 0) dc[col] = tot / (double)R;
  for (int hb = 0; hb < nblk; ++hb) {
    double acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0;
    double wh[kHarmBlock];
#pragma unroll
    for (int h = 0; h < kHarmBlock; ++h) wh[h] = (double)(hb * kHarmBlock + h + 1) * w0;
    for (int t = lane; t < R; t += 64) {
      const double xv = xs[t];
      const double tt = (double)t;
#pragma unroll
      for (int h = 0; h < kHarmBlock; ++h) {
        if (hb * kHarmBlock + h < ndata) {
          double sn, cs;
          sincos(wh[h] * tt, &sn, &cs);
          acc[h] = fma(xv, cs, acc[h]);
          acc[8 + h] = fma(xv, sn, acc[8 + h]);
        }
      }
    }
    butterfly16(acc, lane);
    store_block(acc, lane, hb, ndata, qi, qi_ld, col, R);
  }
}

__global__ __launch_bounds__(kBlockThreads) void demod_direct_kernel(
    const double* __restrict__ x, int64_t nseg, int64_t seg_stride, int R, int ndata, double w0,
    double* __restrict__ qi, int64_t qi_ld, double* __restrict__ dc) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  for (int64_t s = (int64_t)blockIdx.x * kWavesPerBlock + wave; s < nseg;
       s += (int64_t)gridDim.x * kWavesPerBlock) {
    direct_segment(x + s * seg_stride, R, ndata, w0, lane, qi, qi_ld, s, dc);
  }
}

}  // namespace dfmi

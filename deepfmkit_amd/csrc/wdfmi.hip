// wdfmi.hip — witness-based W-DFMI / HW-DFMI fitters on gfx950 (fp64).
//
// Reference (file:line in /root/reference/fitters.py):
//   _get_phase_modulation_basis ... 88-122   -> wdfmi_template_kernel (W-DFMI)
//   _get_total_laser_phase ........ 124-162  -> wdfmi_template_kernel (HW-DFMI)
//   WDFMI_NLSFitter.fit ........... 481-570  -> fit_nls   (MINPACK lmdif, as least_squares(method='lm'))
//   WDFMI_OrthogonalFitter.fit .... 572-648  -> fit_ortho (Nelder-Mead over (tau, psi), VarPro inner solve)
//   WDFMI_SequentialFitter.fit .... 650-776  -> fit_seq   (Brent tau, bounded-Brent psi, linear fit)
//   HWDFMI_Fitter.fit ............. 778-891  -> fit_hw    (Brent tau, VarPro)
// The optimisers follow scipy 1.15.3 (third-party, not in the reference), restated
// line by line from oracle/wdfmi_oracle.py, which is pinned bit-exactly to the
// reference's outputs (tests/golden/wdfmi.npz).
//
// Mapping: ONE WORKGROUP OWNS ONE RECORD CHAIN (nls / ortho / hw: buffer b starts
// from buffer b-1's answer, as the reference's loops do) or ONE BUFFER (seq: its
// buffers are independent). Every thread runs the optimiser's scalar control
// flow redundantly — the values it branches on come out of block reductions
// that hand every thread the same bits — and a cost evaluation is spread over the
// workgroup: thread t owns samples k = t + T*s. Per evaluation:
//   shifted[k] = interp(t_k + psi/omega)           np.interp(period=t[-1]), LDS table -> LDS
//   delta[k]   = interp_{shifted}(t_k - tau) - shifted[k]
//   VarPro     = lstsq([cos delta, sin delta], v)  (QR by two reductions + a residual pass)
//   harmonics  = (2/R) sum v cos/sin(h w0 k)       fold into L phase bins + L-term contraction
// The witness template (R doubles), the shifted phase and the model live in LDS;
// the time axis t_k = k / f_samp (numpy's arange(R)/f_samp, bit-exact) in L1/L2.
//
// Numerics: this translation unit is compiled without FMA contraction, so the
// interpolation, lstsq and optimiser arithmetic rounds operation by operation like
// numpy/MINPACK. Bit-exact with the reference: time axis, template (cumsum /
// cumulative_trapezoid order), the numpy pairwise means. Not bit-exact: lstsq
// (LAPACK dgelsd SVD there, QR + direct residual here), sums over samples, cos/sin.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <cmath>
#include <type_traits>

#include "dfmi_math.h"
#include "np_sum.h"
#include "wdfmi.h"

#pragma clang fp contract(off)

namespace dfmi {
namespace {

constexpr int MMAX = 64;     // lmdif residuals (2 * ndata <= 64)
constexpr int NHMAX = 64;    // harmonics per evaluation (ndata, ndata_psi <= 64)
constexpr int LEAFMAX = 512; // numpy pairwise tree nodes (<= 256 leaves: R <= 16384)
constexpr double kEps = 2.220446049250313e-16;
constexpr double kPi = 3.141592653589793;

__device__ __forceinline__ double inf_d() { return __builtin_huge_val(); }

// Diagnostics (dfmi_set_tuning("probe", 1)): workgroup 0, thread 0 accumulates
// s_memrealtime ticks (100 MHz) per phase into probe[slot]; results are unaffected.
struct Probe {
  uint64_t* p;
  uint64_t acc[8];
  uint64_t last;
  __device__ void init(uint64_t* ptr) {
    p = (ptr && blockIdx.x == 0 && threadIdx.x == 0) ? ptr : nullptr;
    for (int i = 0; i < 8; ++i) acc[i] = 0;
    last = p ? __builtin_amdgcn_s_memrealtime() : 0;
  }
  __device__ __forceinline__ void mark(int slot) {
    if (p) {
      const uint64_t t = __builtin_amdgcn_s_memrealtime();
      acc[slot] += t - last;
      last = t;
    }
  }
  __device__ void flush() {
    if (p)
      for (int i = 0; i < 8; ++i) p[i] = acc[i];
  }
};

// np.sum of an LDS vector following a host-built plan of numpy's tree
// (wdfmi_pairwise_plan): leaves summed in parallel, then the internal nodes level
// by level (children before parents), every addition exactly numpy's.
//   plan[0] = leaves nl, plan[1] = levels H, plan[2 .. 2+nl] = leaf offsets,
//   then H+1 level starts into the node triples (dst, a, b) that follow.
template <int T>
__device__ double block_np_sum(const double* a, const int* __restrict__ plan, double* nodes) {
  const int nl = plan[0], H = plan[1];
  const int* off = plan + 2;
  const int* lvl = off + nl + 1;
  const int* tri = lvl + H + 1;
  for (int t = threadIdx.x; t < nl; t += T) nodes[t] = dfmi_np_leaf_sum(a + off[t], off[t + 1] - off[t]);
  __syncthreads();
  for (int h = 0; h < H; ++h) {
    for (int j = lvl[h] + threadIdx.x; j < lvl[h + 1]; j += T) {
      const int* q = tri + 3 * j;
      nodes[q[0]] = nodes[q[1]] + nodes[q[2]];
    }
    __syncthreads();
  }
  const double s = nodes[nl > 1 ? 2 * nl - 2 : 0];
  __syncthreads();
  return s;
}

// ---------------------------------------------------------------------------
// Block reductions. The xor butterfly gives every lane the same bits (IEEE + and
// max/min are commutative); the cross-wave pass reads the partials in one fixed
// order, so every thread of the workgroup holds an identical result.
// ---------------------------------------------------------------------------
struct OpAdd {
  __device__ double operator()(double a, double b) const { return a + b; }
};
struct OpMax {  // np.max: NaN propagates
  __device__ double operator()(double a, double b) const { return (a != a || b != b) ? __builtin_nan("") : fmax(a, b); }
};
struct OpMin {
  __device__ double operator()(double a, double b) const { return (a != a || b != b) ? __builtin_nan("") : fmin(a, b); }
};

template <int T, int N, typename Op>
__device__ void block_reduce(double (&v)[N], double* red, Op op) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v[i] = op(v[i], __shfl_xor(v[i], o, 64));
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) red[w * N + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double s = red[i];
    for (int k = 1; k < T / 64; ++k) s = op(s, red[k * N + i]);
    v[i] = s;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// np.interp on the buffer's time axis t_k = k / f_samp.
// ---------------------------------------------------------------------------
struct Geo {
  int R;
  bool fast;  // WdfmiLaunch::t_fast
  double fs, rfs, period, omega;
  const double* slp;  // LDS: the template's interval slopes (null: divide per sample)
  // t_k = k / f_samp, formed in registers, rounded exactly like numpy's
  // np.arange(R) / f_samp: q = k * (1/f_samp) corrected by one fma of its residual
  // (Markstein) where the host verified that this equals the IEEE quotient for every
  // k in [0, R], else the division itself (~12 fp64 instructions).
  template <bool FAST>
  __device__ __forceinline__ double tt(int k) const {
    const double kd = (double)k;
    if constexpr (FAST) {
      const double q = kd * rfs;
      return fma(fma(-q, fs, kd), rfs, q);
    } else {
      return kd / fs;
    }
  }
  // runtime choice (prologues, the rare exact search); the per-sample loops take the
  // compile-time form, dispatched once per evaluation, so they stay straight-line
  __device__ __forceinline__ double t(int k) const { return fast ? tt<true>(k) : tt<false>(k); }
};

// Largest i <= hi with t_i <= x (caller guarantees t_0 <= x); also returns t_i, t_{i+1}.
__device__ __forceinline__ int seek(const Geo& g, double x, int hi, double& ti, double& tn) {
  int i = (int)(x * g.fs);
  if (i > hi) i = hi;
  if (i < 0) i = 0;
  ti = g.t(i);
  tn = g.t(i + 1);
  while (i < hi && tn <= x) {
    ++i;
    ti = tn;
    tn = g.t(i + 1);
  }
  while (i > 0 && ti > x) {
    --i;
    tn = ti;
    ti = g.t(i);
  }
  return i;
}

// ---- np.interp, batched and branch-free (one thread's SPT samples at once) ----
// The straight-line bodies let the compiler interleave the samples' dependent
// chains; the exact sequential search only runs when the first guess
// i = (int)(x * f_samp) does not bracket x (rounding at a grid point: rare).

// numpy's x % period, branch-free for -period <= x < 2*period (exact there).
__device__ __forceinline__ double pmod_fast(double x, double period, bool& slow) {
  double r = x;
  r = (x >= period) ? (x == period ? 0.0 : x - period) : r;
  r = (x < 0.0) ? x + period : r;
  r = (x == 0.0) ? 0.0 : r;
  slow = !(x >= -period && x < 2.0 * period);
  return r;
}

// x[s] in [0, period] (numpy's reduced abscissae) -> np.interp(x, t, f, period=t[-1]).
// numpy sorts xp = t % period: t[R-1] % period = 0 ties with t[0]; argsort places
// index 0 first, so the sorted/padded table is
//   xp = [t_{R-2}-P, 0, 0, t_1 .. t_{R-2}, P],  fp = [f_{R-2}, f_0, f_{R-1}, f_1 .. f_{R-2}, f_0]
// and x in [0, t_1) interpolates from the second zero (value f_{R-1}).
// SLP: take the slopes from g.slp (the template's table) instead of dividing per sample.
template <int SPT, bool FAST, bool SLP>
__device__ __forceinline__ void interp_per_batch(const Geo& g, const double (&x)[SPT], const double* f,
                                                 double (&out)[SPT], int nvalid) {
  const int R = g.R;
  int idx[SPT];
  double ti[SPT], tn[SPT];
  bool bad = false;
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const double xs = (x[s] == x[s]) ? x[s] : 0.0;
    int i = (int)(xs * g.fs);
    i = i < 0 ? 0 : (i > R - 2 ? R - 2 : i);
    ti[s] = g.tt<FAST>(i);
    tn[s] = g.tt<FAST>(i + 1);
    const bool ok = (ti[s] <= xs) && (xs < tn[s] || i == R - 2);
    bad = bad || (s < nvalid && !ok);
    idx[s] = i;
  }
  if (bad) {
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      const double xs = (x[s] == x[s]) ? x[s] : 0.0;
      if (s < nvalid && !((ti[s] <= xs) && (xs < tn[s] || idx[s] == R - 2))) idx[s] = seek(g, xs, R - 2, ti[s], tn[s]);
    }
  }
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const int i = idx[s];
    const double fl = (i == 0) ? f[R - 1] : f[i];
    const double fr = (i == R - 2) ? f[0] : f[i + 1];
    const double slope = SLP ? g.slp[i] : (fr - fl) / (tn[s] - ti[s]);
    double r = slope * (x[s] - ti[s]) + fl;
    r = (x[s] == ti[s]) ? fl : r;
    r = (x[s] >= g.period) ? f[0] : r;
    out[s] = (x[s] != x[s]) ? x[s] : r;
  }
}

// np.interp(x, t, f) (no period; left = f[0], right = f[R-1]) for a batch
template <int SPT, bool FAST, bool SLP>
__device__ __forceinline__ void interp_lin_batch(const Geo& g, const double (&x)[SPT], const double* f,
                                                 double (&out)[SPT], int nvalid) {
  const int R = g.R;
  int idx[SPT];
  double ti[SPT], tn[SPT];
  bool bad = false;
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const double xs = (x[s] >= 0.0 && x[s] <= g.period) ? x[s] : 0.0;  // out of range / NaN: selected below
    int i = (int)(xs * g.fs);
    i = i < 0 ? 0 : (i > R - 2 ? R - 2 : i);
    ti[s] = g.tt<FAST>(i);
    tn[s] = g.tt<FAST>(i + 1);
    const bool ok = (ti[s] <= xs) && (xs < tn[s] || i == R - 2);
    bad = bad || (s < nvalid && !ok);
    idx[s] = i;
  }
  if (bad) {
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      const double xs = (x[s] >= 0.0 && x[s] <= g.period) ? x[s] : 0.0;
      if (s < nvalid && !((ti[s] <= xs) && (xs < tn[s] || idx[s] == R - 2))) {
        idx[s] = seek(g, xs, R - 2, ti[s], tn[s]);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const int i = idx[s];
    const double fl = f[i], fr = f[i + 1];
    const double slope = SLP ? g.slp[i] : (fr - fl) / (tn[s] - ti[s]);
    double r = slope * (x[s] - ti[s]) + fl;
    r = (x[s] == ti[s]) ? fl : r;
    r = (x[s] >= g.period) ? f[R - 1] : r;  // x == t[R-1] and beyond: right value
    r = (x[s] < 0.0) ? f[0] : r;
    out[s] = (x[s] != x[s]) ? x[s] : r;
  }
}

// W-DFMI phase difference (fitters.py:533-539 / 611-617 / 688-694):
//   shifted = interp(t - (-psi/omega), t, tab, period), delayed = interp(t - tau, t, shifted, period)
template <int T, int SPT, bool FAST, bool SLP>
__device__ __forceinline__ void wdfmi_delta(const Geo& g, const double* tab, double* sh, double tau, double psi,
                                            double (&d)[SPT]) {
  const double c = (-psi) / g.omega;
  const int nvalid = (g.R - (int)threadIdx.x + T - 1) / T;
  double x[SPT], y[SPT];
  bool slow = false;
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    bool sl;
    x[s] = pmod_fast(g.tt<FAST>(threadIdx.x + T * s) - c, g.period, sl);
    slow = slow || sl;
  }
  if (slow) {
#pragma unroll
    for (int s = 0; s < SPT; ++s) x[s] = dfmi_pymod(g.tt<FAST>(threadIdx.x + T * s) - c, g.period);
  }
  interp_per_batch<SPT, FAST, SLP>(g, x, tab, y, nvalid);
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const int k = threadIdx.x + T * s;
    if (k < g.R) sh[k] = y[s];
  }
  __syncthreads();
  slow = false;
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    bool sl;
    x[s] = pmod_fast(g.tt<FAST>(threadIdx.x + T * s) - tau, g.period, sl);
    slow = slow || sl;
  }
  if (slow) {
#pragma unroll
    for (int s = 0; s < SPT; ++s) x[s] = dfmi_pymod(g.tt<FAST>(threadIdx.x + T * s) - tau, g.period);
  }
  interp_per_batch<SPT, FAST, false>(g, x, sh, d, nvalid);
#pragma unroll
  for (int s = 0; s < SPT; ++s) d[s] = d[s] - y[s];
  __syncthreads();
}

// HW-DFMI (fitters.py:848-852): delta = tmpl - interp(t - tau, t, tmpl)
template <int T, int SPT, bool FAST, bool SLP>
__device__ __forceinline__ void hw_delta(const Geo& g, const double* tab, double tau, double (&d)[SPT]) {
  const int nvalid = (g.R - (int)threadIdx.x + T - 1) / T;
  double x[SPT];
#pragma unroll
  for (int s = 0; s < SPT; ++s) x[s] = g.tt<FAST>(threadIdx.x + T * s) - tau;
  interp_lin_batch<SPT, FAST, SLP>(g, x, tab, d, nvalid);
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const int k = threadIdx.x + T * s;
    d[s] = (k < g.R) ? tab[k] - d[s] : 0.0;
  }
}

// ---------------------------------------------------------------------------
// VarPro inner solve: np.linalg.lstsq([cos d, sin d], v, rcond=None).
// full  = rank 2 (sigma_min > eps*max(R,2)*sigma_max, numpy's rcond=None);
// res   = sum of squared residuals (numpy returns it only at full rank);
// p     = solution (minimum-norm at rank < 2, like dgelsd).
// ---------------------------------------------------------------------------
struct VP {
  double p0, p1, res;
  bool full;
};

template <int T, int SPT>
__device__ __forceinline__ VP varpro(const Geo& g, double* red, const double (&d)[SPT], const double (&v)[SPT], double (&bi)[SPT],
                     double (&bq)[SPT], bool want_res) {
  double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  bool big = false;
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    dfmi_sincos_fast(d[q], &bq[q], &bi[q]);
    big = big || !(fabs(d[q]) < 524288.0);
  }
  if (big) {
#pragma unroll
    for (int q = 0; q < SPT; ++q)
      if (!(fabs(d[q]) < 524288.0)) sincos(d[q], &bq[q], &bi[q]);
  }
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    const int k = threadIdx.x + T * q;
    if (k < g.R) {
      const double cs = bi[q], sn = bq[q];
      s[0] += cs * cs;
      s[1] += cs * sn;
      s[2] += sn * sn;
      s[3] += cs * v[q];
      s[4] += sn * v[q];
    } else {
      bi[q] = bq[q] = 0.0;
    }
  }
  block_reduce<T, 5>(s, red, OpAdd());
  const double a = s[0], b = s[1], c = s[2];
  VP r;
  r.res = 0.0;
  bool full = false;
  double r22sq = 0.0, wv = 0.0;
  if (a > 0.0) {
    // second column orthogonalised against the first: w = bq - (b/a) bi
    const double mu = b / a;
    double t2[2] = {0.0, 0.0};
#pragma unroll
    for (int q = 0; q < SPT; ++q) {
      const int k = threadIdx.x + T * q;
      if (k < g.R) {
        const double w = bq[q] - mu * bi[q];
        t2[0] += w * w;
        t2[1] += w * v[q];
      }
    }
      block_reduce<T, 2>(t2, red, OpAdd());
      r22sq = t2[0];
    wv = t2[1];
    // singular values of [[r11, r12], [0, r22]]
    const double r12sq = (b * b) / a;
    const double S = a + r12sq + r22sq, P = sqrt(a) * sqrt(r22sq);
    const double disc = S * S - 4.0 * P * P;
    const double smax = sqrt(0.5 * (S + sqrt(disc > 0.0 ? disc : 0.0)));
    const double smin = smax > 0.0 ? P / smax : 0.0;
    const double rcond = kEps * (double)(g.R > 2 ? g.R : 2);
    full = smin > rcond * smax;
  }
  r.full = full;
  if (full) {
    r.p1 = wv / r22sq;
    r.p0 = (s[3] - b * r.p1) / a;
    if (want_res) {
      double t1[1] = {0.0};
#pragma unroll
      for (int q = 0; q < SPT; ++q) {
        const int k = threadIdx.x + T * q;
        if (k < g.R) {
          const double e = v[q] - r.p0 * bi[q] - r.p1 * bq[q];
          t1[0] += e * e;
        }
      }
          block_reduce<T, 1>(t1, red, OpAdd());
          r.res = t1[0];
    }
  } else {
    // rank <= 1: minimum-norm solution on the dominant right singular vector
    const double h = 0.5 * (a - c);
    const double lam = 0.5 * (a + c) + sqrt(h * h + b * b);
    double u0 = b, u1 = lam - a;
    const double w0 = lam - c, w1 = b;
    if (w0 * w0 + w1 * w1 > u0 * u0 + u1 * u1) {
      u0 = w0;
      u1 = w1;
    }
    const double nu = sqrt(u0 * u0 + u1 * u1);
    if (lam > 0.0 && nu > 0.0) {
      u0 /= nu;
      u1 /= nu;
      const double coef = (u0 * s[3] + u1 * s[4]) / lam;
      r.p0 = coef * u0;
      r.p1 = coef * u1;
    } else {
      r.p0 = r.p1 = 0.0;
    }
  }
  return r;
}

// ---------------------------------------------------------------------------
// Harmonic sums (2/R) * sum_k m[k] * cos/sin(fl(h*w0) * k), h = 1..nh, of an LDS
// vector (fitters.py:545-548, 553-556, 706-710, 721-724). With a basis period L
// (L*w0 = 2*pi*integer) the samples are folded into L phase bins and contracted
// with the host-built table; otherwise the angles are formed per sample.
// out[c]: c < nh cos harmonics, c >= nh sin harmonics. Caller: m written, any state.
// ---------------------------------------------------------------------------
template <int T>
__device__ void harmonics(const Geo& g, int nh, int L, const double* __restrict__ btab, double w0, const double* m,
                          double* bins, double* out) {
  __syncthreads();
  const int R = g.R;
  const double scale = 2.0 / (double)R;
  if (L > 0) {
    for (int p = threadIdx.x; p < L; p += T) {
      double s = 0.0;
      for (int k = p; k < R; k += L) s += m[k];
      bins[p] = s;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * nh; c += T) {
      const double* __restrict__ row = btab + (int64_t)c * L;
      double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
      int p = 0;
      for (; p + 4 <= L; p += 4) {
        s0 += bins[p] * row[p];
        s1 += bins[p + 1] * row[p + 1];
        s2 += bins[p + 2] * row[p + 2];
        s3 += bins[p + 3] * row[p + 3];
      }
      for (; p < L; ++p) s0 += bins[p] * row[p];
      out[c] = scale * ((s0 + s1) + (s2 + s3));
    }
  } else {
    for (int c = threadIdx.x; c < 2 * nh; c += T) {
      const bool is_sin = c >= nh;
      const double wh = (double)((is_sin ? c - nh : c) + 1) * w0;
      double s = 0.0;
      for (int k = 0; k < R; ++k) {
        const double ang = wh * (double)k;
        s += m[k] * (is_sin ? sin(ang) : cos(ang));
      }
      out[c] = scale * s;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// scipy optimisers (restated from oracle/wdfmi_oracle.py; scipy 1.15.3)
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool np_less(double a, double b) { return a < b || (b != b && a == a); }
__device__ __forceinline__ double nanmax(double a, double b) { return OpMax()(a, b); }

// _minimize_neldermead (N = 2, adaptive=False, no bounds). Returns success.
template <typename F>
__device__ bool nelder_mead2(F&& f, const double (&x0)[2], double (&xout)[2]) {
  const int maxfun = 400, maxiter = 400;
  const double xatol = 1e-4, fatol = 1e-4;
  double sim[3][2], fsim[3];
  sim[0][0] = x0[0];
  sim[0][1] = x0[1];
  for (int k = 0; k < 2; ++k) {
    double y[2] = {x0[0], x0[1]};
    y[k] = (y[k] != 0.0) ? (1.0 + 0.05) * y[k] : 0.00025;
    sim[k + 1][0] = y[0];
    sim[k + 1][1] = y[1];
  }
  int calls = 0;
  auto fun = [&](const double* x, double& out) -> bool {
    if (calls >= maxfun) return false;  // _MaxFun
    ++calls;
    out = f(x[0], x[1]);
    return true;
  };
  auto order = [&]() {  // np.argsort(fsim, kind="stable")
    for (int i = 1; i < 3; ++i) {
      const double kf = fsim[i], k0 = sim[i][0], k1 = sim[i][1];
      int j = i - 1;
      while (j >= 0 && np_less(kf, fsim[j])) {
        fsim[j + 1] = fsim[j];
        sim[j + 1][0] = sim[j][0];
        sim[j + 1][1] = sim[j][1];
        --j;
      }
      fsim[j + 1] = kf;
      sim[j + 1][0] = k0;
      sim[j + 1][1] = k1;
    }
  };
  fsim[0] = fsim[1] = fsim[2] = inf_d();
  for (int k = 0; k < 3; ++k)
    if (!fun(sim[k], fsim[k])) break;
  order();
  int it = 1;
  while (calls < maxfun && it < maxiter) {
    double mx = 0.0, mf = 0.0;
    for (int j = 1; j < 3; ++j) {
      mx = nanmax(nanmax(mx, fabs(sim[j][0] - sim[0][0])), fabs(sim[j][1] - sim[0][1]));
      mf = nanmax(mf, fabs(fsim[0] - fsim[j]));
    }
    if (mx <= xatol && mf <= fatol) {
      order();
      break;
    }
    do {
      double xbar[2], xr[2];
      for (int i = 0; i < 2; ++i) {
        xbar[i] = (sim[0][i] + sim[1][i]) / 2.0;
        xr[i] = 2.0 * xbar[i] - sim[2][i];
      }
      double fxr;
      if (!fun(xr, fxr)) break;
      bool shrink = false;
      if (fxr < fsim[0]) {
        double xe[2] = {3.0 * xbar[0] - 2.0 * sim[2][0], 3.0 * xbar[1] - 2.0 * sim[2][1]};
        double fxe;
        if (!fun(xe, fxe)) break;
        if (fxe < fxr) {
          sim[2][0] = xe[0];
          sim[2][1] = xe[1];
          fsim[2] = fxe;
        } else {
          sim[2][0] = xr[0];
          sim[2][1] = xr[1];
          fsim[2] = fxr;
        }
      } else if (fxr < fsim[1]) {
        sim[2][0] = xr[0];
        sim[2][1] = xr[1];
        fsim[2] = fxr;
      } else if (fxr < fsim[2]) {
        double xc[2] = {1.5 * xbar[0] - 0.5 * sim[2][0], 1.5 * xbar[1] - 0.5 * sim[2][1]};
        double fxc;
        if (!fun(xc, fxc)) break;
        if (fxc <= fxr) {
          sim[2][0] = xc[0];
          sim[2][1] = xc[1];
          fsim[2] = fxc;
        } else {
          shrink = true;
        }
      } else {
        double xcc[2] = {0.5 * xbar[0] + 0.5 * sim[2][0], 0.5 * xbar[1] + 0.5 * sim[2][1]};
        double fxcc;
        if (!fun(xcc, fxcc)) break;
        if (fxcc < fsim[2]) {
          sim[2][0] = xcc[0];
          sim[2][1] = xcc[1];
          fsim[2] = fxcc;
        } else {
          shrink = true;
        }
      }
      if (shrink) {
        bool aborted = false;
        for (int j = 1; j < 3 && !aborted; ++j) {
          sim[j][0] = sim[0][0] + 0.5 * (sim[j][0] - sim[0][0]);
          sim[j][1] = sim[0][1] + 0.5 * (sim[j][1] - sim[0][1]);
          aborted = !fun(sim[j], fsim[j]);
        }
        if (aborted) break;
      }
      ++it;
    } while (false);
    order();
  }
  xout[0] = sim[0][0];
  xout[1] = sim[0][1];
  return !(calls >= maxfun || it >= maxiter);
}

// scipy.optimize.bracket (grow_limit 110, maxiter 1000). Returns true on a valid
// bracket; on failure (xa, xb, xc, fa, fb, fc) hold the last points.
template <typename F>
__device__ bool bracket(F&& f, double xa, double xb, double (&o)[6]) {
  const double gold = 1.618034, small = 1e-21, grow_limit = 110.0;
  const int maxiter = 1000;
  double fa = f(xa), fb = f(xb);
  if (fa < fb) {
    double t = xa;
    xa = xb;
    xb = t;
    t = fa;
    fa = fb;
    fb = t;
  }
  double xc = xb + gold * (xb - xa);
  double fc = f(xc);
  int it = 0;
  bool fail = false;
  while (fc < fb) {
    const double tmp1 = (xb - xa) * (fb - fc);
    const double tmp2 = (xb - xc) * (fb - fa);
    const double val = tmp2 - tmp1;
    const double denom = fabs(val) < small ? 2.0 * small : 2.0 * val;
    double w = xb - ((xb - xc) * tmp2 - (xb - xa) * tmp1) / denom;
    const double wlim = xb + grow_limit * (xc - xb);
    if (it > maxiter) {
      fail = true;
      break;
    }
    ++it;
    double fw;
    if ((w - xc) * (xb - w) > 0.0) {
      fw = f(w);
      if (fw < fc) {
        xa = xb;
        xb = w;
        fa = fb;
        fb = fw;
        break;
      } else if (fw > fb) {
        xc = w;
        fc = fw;
        break;
      }
      w = xc + gold * (xc - xb);
      fw = f(w);
    } else if ((w - wlim) * (wlim - xc) >= 0.0) {
      w = wlim;
      fw = f(w);
    } else if ((w - wlim) * (xc - w) > 0.0) {
      fw = f(w);
      if (fw < fc) {
        xb = xc;
        xc = w;
        w = xc + gold * (xc - xb);
        fb = fc;
        fc = fw;
        fw = f(w);
      }
    } else {
      w = xc + gold * (xc - xb);
      fw = f(w);
    }
    xa = xb;
    xb = xc;
    xc = w;
    fa = fb;
    fb = fc;
    fc = fw;
  }
  o[0] = xa;
  o[1] = xb;
  o[2] = xc;
  o[3] = fa;
  o[4] = fb;
  o[5] = fc;
  if (fail) return false;
  const bool c1 = (fb < fc && fb <= fa) || (fb < fa && fb <= fc);
  const bool c2 = (xa < xb && xb < xc) || (xc < xb && xb < xa);
  const bool c3 = isfinite(xa) && isfinite(xb) && isfinite(xc);
  return c1 && c2 && c3;
}

// minimize_scalar(method='brent', bracket=(x0, x1)) incl. the BracketError recovery.
template <typename F>
__device__ double brent(F&& f, double b0, double b1, bool* ok_out) {
  double br[6];
  if (!bracket(f, b0, b1, br)) {
    const double xs[3] = {br[0], br[1], br[2]}, fs[3] = {br[3], br[4], br[5]};
    for (int i = 0; i < 3; ++i)
      if (xs[i] != xs[i] || fs[i] != fs[i]) {
        *ok_out = false;
        return __builtin_nan("");
      }
    int i = 0;
    for (int j = 1; j < 3; ++j)
      if (fs[j] < fs[i]) i = j;
    *ok_out = false;
    return xs[i];
  }
  const double tol = 1.48e-8, mintol = 1.0e-11, cg = 0.3819660;
  const int maxiter = 500;
  double x = br[1], w = br[1], v = br[1];
  double fw = br[4], fv = br[4], fx = br[4];
  double a = br[0] < br[2] ? br[0] : br[2];
  double b = br[0] < br[2] ? br[2] : br[0];
  double deltax = 0.0, rat = 0.0;
  int it = 0;
  while (it < maxiter) {
    const double tol1 = tol * fabs(x) + mintol;
    const double tol2 = 2.0 * tol1;
    const double xmid = 0.5 * (a + b);
    if (fabs(x - xmid) < (tol2 - 0.5 * (b - a))) break;
    if (fabs(deltax) <= tol1) {
      deltax = (x >= xmid) ? (a - x) : (b - x);
      rat = cg * deltax;
    } else {
      double tmp1 = (x - w) * (fx - fv);
      double tmp2 = (x - v) * (fx - fw);
      double p = (x - v) * tmp2 - (x - w) * tmp1;
      tmp2 = 2.0 * (tmp2 - tmp1);
      if (tmp2 > 0.0) p = -p;
      tmp2 = fabs(tmp2);
      const double dx_temp = deltax;
      deltax = rat;
      if ((p > tmp2 * (a - x)) && (p < tmp2 * (b - x)) && (fabs(p) < fabs(0.5 * tmp2 * dx_temp))) {
        rat = p * 1.0 / tmp2;
        const double u = x + rat;
        if ((u - a) < tol2 || (b - u) < tol2) rat = (xmid - x >= 0) ? tol1 : -tol1;
      } else {
        deltax = (x >= xmid) ? (a - x) : (b - x);
        rat = cg * deltax;
      }
    }
    const double u = (fabs(rat) < tol1) ? ((rat >= 0) ? x + tol1 : x - tol1) : x + rat;
    const double fu = f(u);
    if (fu > fx) {
      if (u < x) a = u;
      else b = u;
      if (fu <= fw || w == x) {
        v = w;
        w = u;
        fv = fw;
        fw = fu;
      } else if (fu <= fv || v == x || v == w) {
        v = u;
        fv = fu;
      }
    } else {
      if (u >= x) a = x;
      else b = x;
      v = w;
      w = x;
      x = u;
      fv = fw;
      fw = fx;
      fx = fu;
    }
    ++it;
  }
  *ok_out = it < maxiter && !(x != x || fx != fx);
  return x;
}

// minimize_scalar(method='bounded', bounds=(x1, x2)) (xatol 1e-5, maxfun 500).
template <typename F>
__device__ double fminbound(F&& f, double x1, double x2) {
  const double xatol = 1e-5;
  const int maxfun = 500;
  const double sqrt_eps = sqrt(2.2e-16);
  const double golden_mean = 0.5 * (3.0 - sqrt(5.0));
  double a = x1, b = x2;
  double fulc = a + golden_mean * (b - a);
  double nfc = fulc, xf = fulc;
  double rat = 0.0, e = 0.0;
  double x = xf;
  double fx = f(x);
  int num = 1;
  double ffulc = fx, fnfc = fx;
  double xm = 0.5 * (a + b);
  double tol1 = sqrt_eps * fabs(xf) + xatol / 3.0;
  double tol2 = 2.0 * tol1;
  while (fabs(xf - xm) > (tol2 - 0.5 * (b - a))) {
    bool golden = true;
    if (fabs(e) > tol1) {
      golden = false;
      double r = (xf - nfc) * (fx - ffulc);
      double q = (xf - fulc) * (fx - fnfc);
      double p = (xf - fulc) * q - (xf - nfc) * r;
      q = 2.0 * (q - r);
      if (q > 0.0) p = -p;
      q = fabs(q);
      r = e;
      e = rat;
      if ((fabs(p) < fabs(0.5 * q * r)) && (p > q * (a - xf)) && (p < q * (b - xf))) {
        rat = (p + 0.0) / q;
        x = xf + rat;
        if (((x - a) < tol2) || ((b - x) < tol2)) {
          const double d = xm - xf;
          const double si = (d > 0.0 ? 1.0 : (d < 0.0 ? -1.0 : 0.0)) + (d == 0.0 ? 1.0 : 0.0);
          rat = tol1 * si;
        }
      } else {
        golden = true;
      }
    }
    if (golden) {
      e = (xf >= xm) ? (a - xf) : (b - xf);
      rat = golden_mean * e;
    }
    const double si = (rat > 0.0 ? 1.0 : (rat < 0.0 ? -1.0 : 0.0)) + (rat == 0.0 ? 1.0 : 0.0);
    x = xf + si * fmax(fabs(rat), tol1);
    const double fu = f(x);
    ++num;
    if (fu <= fx) {
      if (x >= xf) a = xf;
      else b = xf;
      fulc = nfc;
      ffulc = fnfc;
      nfc = xf;
      fnfc = fx;
      xf = x;
      fx = fu;
    } else {
      if (x < xf) a = x;
      else b = x;
      if ((fu <= fnfc) || (nfc == xf)) {
        fulc = nfc;
        ffulc = fnfc;
        nfc = x;
        fnfc = fu;
      } else if ((fu <= ffulc) || (fulc == xf) || (fulc == nfc)) {
        fulc = x;
        ffulc = fu;
      }
    }
    xm = 0.5 * (a + b);
    tol1 = sqrt_eps * fabs(xf) + xatol / 3.0;
    tol2 = 2.0 * tol1;
    if (num >= maxfun) break;
  }
  return xf;
}

// ---- MINPACK lmdif (Moré, Garbow, Hillstrom 1980) as least_squares(method='lm')
// calls it: n = 4, diag = 1 (mode 2), factor 100, epsfcn = eps, ftol = xtol = gtol =
// 1e-8, maxfev = 100*n*(n+1).
constexpr int NP = 4;

__device__ double enorm(int n, const double* x) {
  const double rdwarf = 3.834e-20, rgiant = 1.304e19;
  double s1 = 0.0, s2 = 0.0, s3 = 0.0, x1max = 0.0, x3max = 0.0;
  const double agiant = rgiant / (double)n;
  for (int i = 0; i < n; ++i) {
    const double xabs = fabs(x[i]);
    if (xabs > rdwarf && xabs < agiant) {
      s2 += xabs * xabs;
    } else if (xabs <= rdwarf) {
      if (xabs > x3max) {
        const double r = x3max / xabs;
        s3 = 1.0 + s3 * (r * r);
        x3max = xabs;
      } else if (xabs != 0.0) {
        const double r = xabs / x3max;
        s3 += r * r;
      }
    } else {
      if (xabs > x1max) {
        const double r = x1max / xabs;
        s1 = 1.0 + s1 * (r * r);
        x1max = xabs;
      } else {
        const double r = xabs / x1max;
        s1 += r * r;
      }
    }
  }
  if (s1 != 0.0) return x1max * sqrt(s1 + (s2 / x1max) / x1max);
  if (s2 != 0.0) {
    if (s2 >= x3max) return sqrt(s2 * (1.0 + (x3max / s2) * (x3max * s3)));
    return sqrt(x3max * ((s2 / x3max) + (x3max * s3)));
  }
  return x3max * sqrt(s3);
}

__device__ void qrfac(int m, double (&a)[NP][MMAX], int (&ipvt)[NP], double (&rdiag)[NP], double (&acnorm)[NP]) {
  double wa[NP];
  for (int j = 0; j < NP; ++j) {
    acnorm[j] = enorm(m, a[j]);
    rdiag[j] = acnorm[j];
    wa[j] = rdiag[j];
    ipvt[j] = j;
  }
  const int mn = m < NP ? m : NP;
  for (int j = 0; j < mn; ++j) {
    int kmax = j;
    for (int k = j; k < NP; ++k)
      if (rdiag[k] > rdiag[kmax]) kmax = k;
    if (kmax != j) {
      for (int i = 0; i < m; ++i) {
        const double t = a[j][i];
        a[j][i] = a[kmax][i];
        a[kmax][i] = t;
      }
      rdiag[kmax] = rdiag[j];
      wa[kmax] = wa[j];
      const int t = ipvt[j];
      ipvt[j] = ipvt[kmax];
      ipvt[kmax] = t;
    }
    double ajnorm = enorm(m - j, a[j] + j);
    if (ajnorm != 0.0) {
      if (a[j][j] < 0.0) ajnorm = -ajnorm;
      for (int i = j; i < m; ++i) a[j][i] = a[j][i] / ajnorm;
      a[j][j] = a[j][j] + 1.0;
      for (int k = j + 1; k < NP; ++k) {
        double s = 0.0;
        for (int i = j; i < m; ++i) s = s + a[j][i] * a[k][i];
        const double temp = s / a[j][j];
        for (int i = j; i < m; ++i) a[k][i] = a[k][i] - temp * a[j][i];
        if (rdiag[k] != 0.0) {
          const double t = a[k][j] / rdiag[k];
          const double q = 1.0 - t * t;
          rdiag[k] = rdiag[k] * sqrt(q > 0.0 ? q : 0.0);
          const double r = rdiag[k] / wa[k];
          if (0.05 * (r * r) <= kEps) {
            rdiag[k] = enorm(m - (j + 1), a[k] + j + 1);
            wa[k] = rdiag[k];
          }
        }
      }
    }
    rdiag[j] = -ajnorm;
  }
}

// r[j][i] = R(i, j); the strict lower part is overwritten.
__device__ void qrsolv(double (&r)[NP][NP], const int (&ipvt)[NP], const double (&diag)[NP], const double (&qtb)[NP],
                       double (&out)[NP], double (&sdiag)[NP]) {
  double x[NP], wa[NP];
  for (int j = 0; j < NP; ++j) {
    for (int i = j; i < NP; ++i) r[j][i] = r[i][j];
    x[j] = r[j][j];
    wa[j] = qtb[j];
  }
  for (int j = 0; j < NP; ++j) {
    const int l = ipvt[j];
    if (diag[l] != 0.0) {
      for (int k = j; k < NP; ++k) sdiag[k] = 0.0;
      sdiag[j] = diag[l];
      double qtbpj = 0.0;
      for (int k = j; k < NP; ++k) {
        if (sdiag[k] == 0.0) continue;
        double sn, cs;
        if (fabs(r[k][k]) < fabs(sdiag[k])) {
          const double cotan = r[k][k] / sdiag[k];
          sn = 0.5 / sqrt(0.25 + 0.25 * cotan * cotan);
          cs = sn * cotan;
        } else {
          const double tn = sdiag[k] / r[k][k];
          cs = 0.5 / sqrt(0.25 + 0.25 * tn * tn);
          sn = cs * tn;
        }
        r[k][k] = cs * r[k][k] + sn * sdiag[k];
        const double temp = cs * wa[k] + sn * qtbpj;
        qtbpj = -sn * wa[k] + cs * qtbpj;
        wa[k] = temp;
        for (int i = k + 1; i < NP; ++i) {
          const double t2 = cs * r[k][i] + sn * sdiag[i];
          sdiag[i] = -sn * r[k][i] + cs * sdiag[i];
          r[k][i] = t2;
        }
      }
    }
    sdiag[j] = r[j][j];
    r[j][j] = x[j];
  }
  int nsing = NP;
  for (int j = 0; j < NP; ++j) {
    if (sdiag[j] == 0.0 && nsing == NP) nsing = j;
    if (nsing < NP) wa[j] = 0.0;
  }
  for (int k = 0; k < nsing; ++k) {
    const int j = nsing - k - 1;
    double s = 0.0;
    for (int i = j + 1; i < nsing; ++i) s = s + r[j][i] * wa[i];
    wa[j] = (wa[j] - s) / sdiag[j];
  }
  for (int j = 0; j < NP; ++j) out[ipvt[j]] = wa[j];
}

__device__ double lmpar(double (&r)[NP][NP], const int (&ipvt)[NP], const double (&diag)[NP], const double (&qtb)[NP],
                        double delta, double par, double (&x)[NP]) {
  const double dwarf = 2.2250738585072014e-308;
  double wa1[NP], wa2[NP], sdiag[NP];
  int nsing = NP;
  for (int j = 0; j < NP; ++j) {
    wa1[j] = qtb[j];
    if (r[j][j] == 0.0 && nsing == NP) nsing = j;
    if (nsing < NP) wa1[j] = 0.0;
  }
  for (int k = 0; k < nsing; ++k) {
    const int j = nsing - k - 1;
    wa1[j] = wa1[j] / r[j][j];
    const double temp = wa1[j];
    for (int i = 0; i < j; ++i) wa1[i] = wa1[i] - r[j][i] * temp;
  }
  for (int j = 0; j < NP; ++j) x[ipvt[j]] = wa1[j];
  int it = 0;
  for (int j = 0; j < NP; ++j) wa2[j] = diag[j] * x[j];
  double dxnorm = enorm(NP, wa2);
  double fp = dxnorm - delta;
  if (fp <= 0.1 * delta) return 0.0;
  double parl = 0.0;
  if (nsing >= NP) {
    for (int j = 0; j < NP; ++j) {
      const int l = ipvt[j];
      wa1[j] = diag[l] * (wa2[l] / dxnorm);
    }
    for (int j = 0; j < NP; ++j) {
      double s = 0.0;
      for (int i = 0; i < j; ++i) s = s + r[j][i] * wa1[i];
      wa1[j] = (wa1[j] - s) / r[j][j];
    }
    const double temp = enorm(NP, wa1);
    parl = ((fp / delta) / temp) / temp;
  }
  for (int j = 0; j < NP; ++j) {
    double s = 0.0;
    for (int i = 0; i <= j; ++i) s = s + r[j][i] * qtb[i];
    wa1[j] = s / diag[ipvt[j]];
  }
  const double gnorm = enorm(NP, wa1);
  double paru = gnorm / delta;
  if (paru == 0.0) paru = dwarf / (delta < 0.1 ? delta : 0.1);
  par = par > parl ? par : parl;
  par = par < paru ? par : paru;
  if (par == 0.0) par = gnorm / dxnorm;
  for (;;) {
    ++it;
    if (par == 0.0) par = (dwarf > 0.001 * paru) ? dwarf : 0.001 * paru;
    const double temp = sqrt(par);
    for (int j = 0; j < NP; ++j) wa1[j] = temp * diag[j];
    qrsolv(r, ipvt, wa1, qtb, x, sdiag);
    for (int j = 0; j < NP; ++j) wa2[j] = diag[j] * x[j];
    dxnorm = enorm(NP, wa2);
    const double fp_old = fp;
    fp = dxnorm - delta;
    if (fabs(fp) <= 0.1 * delta || (parl == 0.0 && fp <= fp_old && fp_old < 0.0) || it == 10) break;
    for (int j = 0; j < NP; ++j) {
      const int l = ipvt[j];
      wa1[j] = diag[l] * (wa2[l] / dxnorm);
    }
    for (int j = 0; j < NP; ++j) {
      wa1[j] = wa1[j] / sdiag[j];
      const double t = wa1[j];
      for (int i = j + 1; i < NP; ++i) wa1[i] = wa1[i] - r[j][i] * t;
    }
    const double t = enorm(NP, wa1);
    const double parc = ((fp / delta) / t) / t;
    if (fp > 0.0) parl = parl > par ? parl : par;
    if (fp < 0.0) paru = paru < par ? paru : par;
    par = (parl > par + parc) ? parl : par + parc;
  }
  return par;
}

// fcn(const double (&x)[NP], double* fvec) evaluates the m residuals (collective).
// Returns MINPACK's info; x, fvec hold the final point and its residuals.
template <typename F>
__device__ int lmdif(F&& fcn, int m, double (&x)[NP], double (&fvec)[MMAX]) {
  const double ftol = 1e-8, xtol = 1e-8, gtol = 1e-8, factor = 100.0;
  const int maxfev = 100 * NP * (NP + 1);
  double diag[NP] = {1.0, 1.0, 1.0, 1.0};
  fcn(x, fvec);
  int nfev = 1;
  double fnorm = enorm(m, fvec);
  double par = 0.0;
  int it = 1, info = 0;
  const double eps = sqrt(kEps);
  double xnorm = 0.0, delta = 0.0;
  double cols[NP][MMAX], wa[MMAX], wa4[MMAX];
  double r[NP][NP];
  int ipvt[NP];
  double rdiag[NP], acnorm[NP], qtf[NP];
  for (;;) {
    // fdjac2: forward differences, h = eps*|x_j| (eps if zero)
    for (int j = 0; j < NP; ++j) {
      const double temp = x[j];
      double h = eps * fabs(temp);
      if (h == 0.0) h = eps;
      double xp[NP] = {x[0], x[1], x[2], x[3]};
      xp[j] = temp + h;
      fcn(xp, wa);
      for (int i = 0; i < m; ++i) cols[j][i] = (wa[i] - fvec[i]) / h;
    }
    nfev += NP;
    qrfac(m, cols, ipvt, rdiag, acnorm);
    if (it == 1) {
      double wa3[NP];
      for (int j = 0; j < NP; ++j) wa3[j] = diag[j] * x[j];
      xnorm = enorm(NP, wa3);
      delta = factor * xnorm;
      if (delta == 0.0) delta = factor;
    }
    for (int i = 0; i < m; ++i) wa4[i] = fvec[i];
    for (int j = 0; j < NP; ++j) {
      if (cols[j][j] != 0.0) {
        double s = 0.0;
        for (int i = j; i < m; ++i) s = s + cols[j][i] * wa4[i];
        const double temp = -s / cols[j][j];
        for (int i = j; i < m; ++i) wa4[i] = wa4[i] + cols[j][i] * temp;
      }
      cols[j][j] = rdiag[j];
      qtf[j] = wa4[j];
    }
    double gnorm = 0.0;
    if (fnorm != 0.0) {
      for (int j = 0; j < NP; ++j) {
        const int l = ipvt[j];
        if (acnorm[l] != 0.0) {
          double s = 0.0;
          for (int i = 0; i <= j; ++i) s = s + cols[j][i] * (qtf[i] / fnorm);
          const double g = fabs(s / acnorm[l]);
          gnorm = gnorm > g ? gnorm : g;
        }
      }
    }
    if (gnorm <= gtol) info = 4;
    if (info != 0) break;
    for (int j = 0; j < NP; ++j)
      for (int i = 0; i < NP; ++i) r[j][i] = cols[j][i];
    for (;;) {
      double pstep[NP];
      par = lmpar(r, ipvt, diag, qtf, delta, par, pstep);
      double wa1[NP], wa2[NP], wa3[NP];
      for (int j = 0; j < NP; ++j) {
        wa1[j] = -pstep[j];
        wa2[j] = x[j] + wa1[j];
        wa3[j] = diag[j] * wa1[j];
      }
      const double pnorm = enorm(NP, wa3);
      if (it == 1) delta = delta < pnorm ? delta : pnorm;
      fcn(wa2, wa4);
      ++nfev;
      const double fnorm1 = enorm(m, wa4);
      double actred = -1.0;
      if (0.1 * fnorm1 < fnorm) {
        const double q = fnorm1 / fnorm;
        actred = 1.0 - q * q;
      }
      for (int j = 0; j < NP; ++j) wa3[j] = 0.0;
      for (int j = 0; j < NP; ++j) {
        const double temp = wa1[ipvt[j]];
        for (int i = 0; i <= j; ++i) wa3[i] = wa3[i] + r[j][i] * temp;
      }
      const double temp1 = enorm(NP, wa3) / fnorm;
      const double temp2 = (sqrt(par) * pnorm) / fnorm;
      const double prered = temp1 * temp1 + temp2 * temp2 / 0.5;
      const double dirder = -(temp1 * temp1 + temp2 * temp2);
      double ratio = 0.0;
      if (prered != 0.0) ratio = actred / prered;
      if (ratio <= 0.25) {
        double temp = (actred >= 0.0) ? 0.5 : 0.5 * dirder / (dirder + 0.5 * actred);
        if (0.1 * fnorm1 >= fnorm || temp < 0.1) temp = 0.1;
        const double dl = pnorm / 0.1;
        delta = temp * (delta < dl ? delta : dl);
        par = par / temp;
      } else if (par == 0.0 || ratio >= 0.75) {
        delta = pnorm / 0.5;
        par = 0.5 * par;
      }
      if (ratio >= 1e-4) {
        for (int j = 0; j < NP; ++j) {
          x[j] = wa2[j];
          wa2[j] = diag[j] * x[j];
        }
        for (int i = 0; i < m; ++i) fvec[i] = wa4[i];
        xnorm = enorm(NP, wa2);
        fnorm = fnorm1;
        ++it;
      }
      if (fabs(actred) <= ftol && prered <= ftol && 0.5 * ratio <= 1.0) info = 1;
      if (delta <= xtol * xnorm) info = 2;
      if (fabs(actred) <= ftol && prered <= ftol && 0.5 * ratio <= 1.0 && info == 2) info = 3;
      if (info != 0) break;
      if (nfev >= maxfev) info = 5;
      if (fabs(actred) <= kEps && prered <= kEps && 0.5 * ratio <= 1.0) info = 6;
      if (delta <= kEps * xnorm) info = 7;
      if (gnorm <= kEps) info = 8;
      if (info != 0) break;
      if (ratio >= 1e-4) break;
    }
    if (info != 0) break;
  }
  return info;
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------

// Witness template per record (fitters.py:88-162), written to a.tmpl[r*R + k].
//  W-DFMI: v = w - mean(w); f = -v / max|v|; (2 pi df) * (cumsum(f) * dt)
//  HW:     2 pi * cumulative_trapezoid(w + f_ref, dx=dt, initial=0)
template <int T>
__global__ __launch_bounds__(T) void wdfmi_template_kernel(WdfmiLaunch a) {
  extern __shared__ double lds[];
  const int R = a.R;
  double* buf = lds;
  double* inc = lds + R;
  double* leafv = inc + R;
  double* red = leafv + LEAFMAX;
  const int64_t rec = blockIdx.x;
  const double* __restrict__ w = a.wit + rec * a.wit_stride;
  double* __restrict__ out = a.tmpl + rec * R;
  for (int k = threadIdx.x; k < R; k += T) buf[k] = w[k];
  __syncthreads();
  const double dt = 1.0 / a.f_samp - 0.0 / a.f_samp;  // t[1] - t[0]
  if (a.method != kHwdfmi) {
    const double mean = block_np_sum<T>(buf, a.pw_plan, leafv) / (double)R;
    double mx[1] = {0.0};
    for (int k = threadIdx.x; k < R; k += T) {
      const double v = buf[k] - mean;
      buf[k] = v;
      mx[0] = OpMax()(mx[0], fabs(v));
    }
    block_reduce<T, 1>(mx, red, OpMax());
    for (int k = threadIdx.x; k < R; k += T) inc[k] = (-buf[k]) / mx[0];
    __syncthreads();
    if (threadIdx.x == 0) {
      const double scale = (2.0 * kPi) * a.df;
      double c = inc[0];
      out[0] = scale * (c * dt);
      for (int k = 1; k < R; ++k) {
        c = c + inc[k];
        out[k] = scale * (c * dt);
      }
    }
  } else {
    for (int k = threadIdx.x; k < R - 1; k += T) {
      const double y1 = buf[k + 1] + a.f_ref, y0 = buf[k] + a.f_ref;
      inc[k] = (dt * (y1 + y0)) / 2.0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const double tp = 2.0 * kPi;
      out[0] = tp * 0.0;
      double c = 0.0;
      for (int k = 0; k < R - 1; ++k) {
        c = (k == 0) ? inc[0] : c + inc[k];
        out[k + 1] = tp * c;
      }
    }
  }
}

struct LdsMap {
  double *tab, *sh, *vac, *mv, *bins, *hout, *hmeas, *red, *leafv, *slp;
};

// All methods: tab (witness template) | sh (shifted phase / scratch) | vac (the
// buffer minus its mean) | red | leafv; nls / seq add the model vector, the phase
// bins and the harmonic vectors.
__host__ __device__ inline bool needs_harmonics(int method) { return method == kWdfmiNLS || method == kWdfmiSeq; }

__host__ __device__ inline size_t lds_doubles_base(int method, int R, int L, int threads) {
  const int Lp = ((L > 0 ? L : 1) + 1) & ~1;
  size_t n = 3 * (size_t)R + (threads / 64) * 8 + LEAFMAX;
  if (needs_harmonics(method)) n += (size_t)R + Lp + 4 * NHMAX;
  return n;
}

// The template's slope table (R - 1 doubles) rides along where the workgroup's LDS
// still has room for it (ortho / hw at R = 4000; not nls / seq).
constexpr size_t kLdsDoubles = 160 * 1024 / 8;
__host__ __device__ inline bool slopes_in_lds(const WdfmiLaunch& a) {
  return (a.accel & 2) && lds_doubles_base(a.method, a.R, a.L, a.threads) + (size_t)a.R <= kLdsDoubles;
}

__host__ __device__ inline size_t lds_doubles(const WdfmiLaunch& a) {
  return lds_doubles_base(a.method, a.R, a.L, a.threads) + (slopes_in_lds(a) ? (size_t)a.R : 0);
}

template <int T>
__device__ LdsMap lds_map(double* lds, const WdfmiLaunch& a) {
  const int method = a.method, R = a.R, L = a.L;
  LdsMap m;
  const int Lp = ((L > 0 ? L : 1) + 1) & ~1;
  m.tab = lds;
  m.sh = m.tab + R;
  m.vac = m.sh + R;
  m.red = m.vac + R;
  m.leafv = m.red + (T / 64) * 8;
  m.mv = m.bins = m.hout = m.hmeas = nullptr;
  double* end = m.leafv + LEAFMAX;
  if (needs_harmonics(method)) {
    m.mv = end;
    m.bins = m.mv + R;
    m.hout = m.bins + Lp;
    m.hmeas = m.hout + 2 * NHMAX;
    end = m.hmeas + 2 * NHMAX;
  }
  m.slp = slopes_in_lds(a) ? end : nullptr;
  return m;
}

template <int T>
__device__ void put_row(const WdfmiLaunch& a, int64_t idx, double amp, double m, double phi, double psi, double tau,
                        double dc, double ssq, int ok) {
  if (threadIdx.x == 0) {
    const int64_t n = a.nrec * a.nbuf;
    a.out[0 * n + idx] = amp;
    a.out[1 * n + idx] = m;
    a.out[2 * n + idx] = phi;
    a.out[3 * n + idx] = psi;
    a.out[4 * n + idx] = tau;
    a.out[5 * n + idx] = dc;
    a.out[6 * n + idx] = ssq;
    a.fitok[idx] = ok;
  }
}

// Buffer prologue: raw samples into registers and LDS, dc = np.mean(buffer).
// Buffer prologue: dc = np.mean(buffer) (raw samples staged in sh), vac = buffer - dc;
// with keep_raw the raw samples are also left in mv (WDFMI_NLS demodulates them).
template <int T>
__device__ double load_buffer(const WdfmiLaunch& a, const LdsMap& L, const double* __restrict__ xb, bool keep_raw) {
  for (int k = threadIdx.x; k < a.R; k += T) {
    const double v = xb[k];
    L.sh[k] = v;
    if (keep_raw) L.mv[k] = v;
  }
  __syncthreads();
  const double dc = block_np_sum<T>(L.sh, a.pw_plan, L.leafv) / (double)a.R;
  for (int k = threadIdx.x; k < a.R; k += T) L.vac[k] = L.sh[k] - dc;
  __syncthreads();
  return dc;
}

// One cost evaluation, shared by every optimiser call site (a single out-of-line
// copy keeps the kernels small; the per-sample arrays live in its registers).
enum : int {
  kEvHW = 1,      // HW-DFMI delta (non-periodic), else the W-DFMI shifted/delayed delta
  kEvRes = 2,     // VarPro residual sum of squares
  kEvModel = 4,   // mv[k] = p0 cos(d) - p1 sin(d) (WDFMI_SequentialFitter stage 2)
  kEvPtp = 8,     // max / min of delta (HWDFMI m)
  kEvNls = 16,    // mv[k] = amp cos(phi + d), no VarPro (WDFMI_NLSFitter residual)
};

struct EvalOut {
  double p0, p1, res, dmax, dmin;
  bool full;
};

template <int T, int SPT>
__device__ __attribute__((noinline)) EvalOut evaluate(const Geo g, const LdsMap L, double tau, double psi, int flags,
                                                      double amp, double phi) {
  double d[SPT], v[SPT], bi[SPT], bq[SPT];
  auto delta = [&](auto fast, auto slp) {
    constexpr bool F = decltype(fast)::value, S = decltype(slp)::value;
    if (flags & kEvHW) hw_delta<T, SPT, F, S>(g, L.tab, tau, d);
    else wdfmi_delta<T, SPT, F, S>(g, L.tab, L.sh, tau, psi, d);
  };
  using yes = std::true_type;
  using no = std::false_type;
  if (g.fast && g.slp) delta(yes(), yes());
  else if (g.fast) delta(yes(), no());
  else delta(no(), no());  // the slope table without the fast time axis: not worth a variant
  EvalOut o;
  o.p0 = o.p1 = o.res = o.dmax = o.dmin = 0.0;
  o.full = false;
  if (flags & kEvNls) {
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      const int k = threadIdx.x + T * s;
      if (k < g.R) L.mv[k] = amp * cos(phi + d[s]);
    }
    return o;
  }
#pragma unroll
  for (int s = 0; s < SPT; ++s) {
    const int k = threadIdx.x + T * s;
    v[s] = (k < g.R) ? L.vac[k] : 0.0;
  }
  const VP r = varpro<T, SPT>(g, L.red, d, v, bi, bq, (flags & kEvRes) != 0);
  o.p0 = r.p0;
  o.p1 = r.p1;
  o.res = r.res;
  o.full = r.full;
  if (flags & kEvModel) {
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      const int k = threadIdx.x + T * s;
      if (k < g.R) L.mv[k] = r.p0 * bi[s] - r.p1 * bq[s];
    }
  }
  if (flags & kEvPtp) {
    double mx[1] = {-inf_d()}, mn[1] = {inf_d()};
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      const int k = threadIdx.x + T * s;
      if (k < g.R) {
        mx[0] = OpMax()(mx[0], d[s]);
        mn[0] = OpMin()(mn[0], d[s]);
      }
    }
    block_reduce<T, 1>(mx, L.red, OpMax());
    block_reduce<T, 1>(mn, L.red, OpMin());
    o.dmax = mx[0];
    o.dmin = mn[0];
  }
  return o;
}

template <int T, int SPT, int METHOD>
__global__ __launch_bounds__(T) void wdfmi_fit_kernel(WdfmiLaunch a) {
  extern __shared__ double lds[];
  const int R = a.R;
  const LdsMap L = lds_map<T>(lds, a);
  Geo g;
  g.R = R;
  g.fast = a.t_fast != 0;
  g.fs = a.f_samp;
  g.rfs = a.t_rcp;
  g.slp = nullptr;
  g.period = g.t(R - 1);  // t[-1]
  g.omega = (2.0 * kPi) * a.f_mod;
  const double m_scale = (2.0 * kPi) * a.df;

  int64_t rec, b0, b1;
  if (METHOD == kWdfmiSeq) {
    rec = blockIdx.x / a.nbuf;
    b0 = blockIdx.x - rec * a.nbuf;
    b1 = b0 + 1;
  } else {
    rec = blockIdx.x;
    b0 = 0;
    b1 = a.nbuf;
  }
  const double* __restrict__ tsrc = a.tmpl + (a.wit_stride == 0 ? 0 : rec) * (int64_t)R;
  for (int k = threadIdx.x; k < R; k += T) L.tab[k] = tsrc[k];
  __syncthreads();
  if (L.slp) {
    // np.interp's interval slopes (fp[j+1] - fp[j]) / (xp[j+1] - xp[j]) of the template
    // table, formed once per record: HW-DFMI's clamped table, else the periodic one
    // (interp_per_batch's sorted/padded layout: interval 0 starts at the second zero
    // with f_{R-1}, interval R-2 ends at the period with f_0).
    const bool per = METHOD != kHwdfmi;
    for (int i = threadIdx.x; i < R - 1; i += T) {
      const double fl = (per && i == 0) ? L.tab[R - 1] : L.tab[i];
      const double fr = (per && i == R - 2) ? L.tab[0] : L.tab[i + 1];
      L.slp[i] = (fr - fl) / (g.t(i + 1) - g.t(i));
    }
    __syncthreads();
    g.slp = L.slp;
  }
  Probe pr;
  pr.init(a.probe);
  auto ev = [&](double tau, double psi, int flags, double amp = 0.0, double phi = 0.0) -> EvalOut {
    pr.mark(5);
    const EvalOut o = evaluate<T, SPT>(g, L, tau, psi, flags, amp, phi);
    pr.mark(1);
    if (pr.p) ++pr.acc[7];
    return o;
  };

  if constexpr (METHOD == kWdfmiOrtho) {
    double guess[2] = {a.tau_init, a.init_psi};
    for (int64_t b = b0; b < b1; ++b) {
      const double dc = load_buffer<T>(a, L, a.x + rec * a.rec_stride + b * R, false);
      pr.mark(0);
      auto cost = [&](double tau, double psi) -> double {
        const EvalOut o = ev(tau, psi, kEvRes);
        return o.full ? o.res : inf_d();
      };
      double x[2];
      const bool ok = nelder_mead2(cost, guess, x);
      const EvalOut r = ev(x[0], x[1], kEvRes);
      const double amp = sqrt(r.p0 * r.p0 + r.p1 * r.p1);
      put_row<T>(a, rec * a.nbuf + b, amp, m_scale * x[0], atan2(-r.p1, r.p0), x[1], x[0], dc,
                 r.full ? r.res : 0.0, ok ? 1 : 0);
      guess[0] = x[0];
      guess[1] = x[1];
    }
  } else if constexpr (METHOD == kHwdfmi) {
    double guess = a.tau_init;
    for (int64_t b = b0; b < b1; ++b) {
      const double dc = load_buffer<T>(a, L, a.x + rec * a.rec_stride + b * R, false);
      pr.mark(0);
      auto cost = [&](double tau) -> double {
        const EvalOut o = ev(tau, 0.0, kEvHW | kEvRes);
        return o.full ? o.res : inf_d();
      };
      const double lo = guess != 0.0 ? guess * 0.8 : -1e-9;
      const double hi = guess != 0.0 ? guess * 1.2 : 1e-9;
      bool bok;
      const double tau = brent(cost, lo, hi, &bok);
      const EvalOut r = ev(tau, 0.0, kEvHW | kEvRes | kEvPtp);
      const double amp = sqrt(r.p0 * r.p0 + r.p1 * r.p1);
      put_row<T>(a, rec * a.nbuf + b, amp, (r.dmax - r.dmin) / 2.0, atan2(-r.p1, r.p0), 0.0, tau, dc,
                 r.full ? r.res : 0.0, 1);
      guess = tau;
    }
  } else if constexpr (METHOD == kWdfmiSeq) {
    const int nh = a.ndata_psi;
    for (int64_t b = b0; b < b1; ++b) {
      const double dc = load_buffer<T>(a, L, a.x + rec * a.rec_stride + b * R, false);
      pr.mark(0);
      // stage 1: tau by Brent on the VarPro cost at psi = init_psi
      auto cost_tau = [&](double tau) -> double {
        const EvalOut o = ev(tau, a.init_psi, kEvRes);
        return o.full ? o.res : inf_d();
      };
      const double lo = a.tau_init > 0.0 ? a.tau_init * 0.9 : -1e-9;
      const double hi = a.tau_init > 0.0 ? a.tau_init * 1.1 : 1e-9;
      bool bok;
      const double tau_fit = brent(cost_tau, lo, hi, &bok);
      // stage 2: psi by bounded Brent on the variance of the unwrapped harmonic phase error
      harmonics<T>(g, nh, a.L, a.btab_psi, a.w0, L.vac, L.bins, L.hmeas);
      auto cost_psi = [&](double dpsi) -> double {
        ev(tau_fit, a.init_psi + dpsi, kEvModel);
        harmonics<T>(g, nh, a.L, a.btab_psi, a.w0, L.mv, L.bins, L.hout);
        // np.angle(alpha_meas * conj(alpha_model)), np.unwrap, np.var (every thread)
        double pe[NHMAX];
        for (int i = 0; i < nh; ++i) {
          const double ar = L.hmeas[i], ai = L.hmeas[nh + i];
          const double br = L.hout[i], bim = -L.hout[nh + i];
          pe[i] = atan2(ar * bim + ai * br, ar * br - ai * bim);
        }
        const double two_pi = 2.0 * kPi;
        double cum = 0.0;
        double up[NHMAX];
        up[0] = pe[0];
        for (int i = 1; i < nh; ++i) {
          const double dd = pe[i] - pe[i - 1];
          double ddmod = dfmi_pymod(dd - (-kPi), two_pi) + (-kPi);
          if (ddmod == -kPi && dd > 0.0) ddmod = kPi;
          double corr = ddmod - dd;
          if (fabs(dd) < kPi) corr = 0.0;
          cum = (i == 1) ? corr : cum + corr;
          up[i] = pe[i] + cum;
        }
        const double mean = dfmi_np_leaf_sum(up, nh) / (double)nh;
        for (int i = 0; i < nh; ++i) {
          const double x = up[i] - mean;
          up[i] = x * x;
        }
        return dfmi_np_leaf_sum(up, nh) / (double)nh;
      };
      const double dpsi = fminbound(cost_psi, -kPi / 2.0, kPi / 2.0);
      const double psi_fit = a.init_psi + dpsi;
      // stage 3: linear fit at (tau, psi)
      const EvalOut r = ev(tau_fit, psi_fit, kEvRes);
      const double amp = sqrt(r.p0 * r.p0 + r.p1 * r.p1);
      put_row<T>(a, rec * a.nbuf + b, amp, m_scale * tau_fit, atan2(-r.p1, r.p0), psi_fit, tau_fit, dc,
                 r.full ? r.res : 0.0, 1);
    }
  } else {  // kWdfmiNLS
    const int nd = a.ndata, m = 2 * a.ndata;
    double guess[NP] = {a.init_a, a.tau_init, a.init_phi, a.init_psi};
    for (int64_t b = b0; b < b1; ++b) {
      const double dc = load_buffer<T>(a, L, a.x + rec * a.rec_stride + b * R, true);
      pr.mark(0);
      // QI of the raw buffer (fitters.py:551-556)
      harmonics<T>(g, nd, a.L, a.btab_nls, a.w0, L.mv, L.bins, L.hmeas);
      auto fcn = [&](const double (&p)[NP], double* fv) {
        ev(p[1], p[3], kEvNls, p[0], p[2]);
        harmonics<T>(g, nd, a.L, a.btab_nls, a.w0, L.mv, L.bins, L.hout);
        for (int i = 0; i < m; ++i) fv[i] = L.hout[i] - L.hmeas[i];
      };
      double x[NP] = {guess[0], guess[1], guess[2], guess[3]};
      double fvec[MMAX];
      const int info = lmdif(fcn, m, x, fvec);
      for (int i = 0; i < m; ++i) fvec[i] = fvec[i] * fvec[i];
      const double ssq = dfmi_np_leaf_sum(fvec, m);
      put_row<T>(a, rec * a.nbuf + b, x[0], m_scale * x[1], x[2], x[3], x[1], dc, ssq,
                 (info >= 1 && info <= 4) ? 1 : 0);
      for (int i = 0; i < NP; ++i) guess[i] = x[i];
    }
  }
  pr.flush();
}

template <int T, int SPT>
hipError_t launch_t(const WdfmiLaunch& a, hipStream_t st) {
  const int64_t ntmpl = a.wit_stride == 0 ? 1 : a.nrec;
  const size_t tl = (size_t)(2 * a.R + LEAFMAX + (T / 64) * 8) * 8;
  hipLaunchKernelGGL(wdfmi_template_kernel<T>, dim3((unsigned)ntmpl), dim3(T), tl, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t fl = wdfmi_lds_bytes(a);
  const int64_t grid = a.method == kWdfmiSeq ? a.nrec * a.nbuf : a.nrec;
  switch (a.method) {
    case kWdfmiNLS:
      hipLaunchKernelGGL((wdfmi_fit_kernel<T, SPT, kWdfmiNLS>), dim3((unsigned)grid), dim3(T), fl, st, a);
      break;
    case kWdfmiOrtho:
      hipLaunchKernelGGL((wdfmi_fit_kernel<T, SPT, kWdfmiOrtho>), dim3((unsigned)grid), dim3(T), fl, st, a);
      break;
    case kWdfmiSeq:
      hipLaunchKernelGGL((wdfmi_fit_kernel<T, SPT, kWdfmiSeq>), dim3((unsigned)grid), dim3(T), fl, st, a);
      break;
    default:
      hipLaunchKernelGGL((wdfmi_fit_kernel<T, SPT, kHwdfmi>), dim3((unsigned)grid), dim3(T), fl, st, a);
      break;
  }
  return hipGetLastError();
}

}  // namespace

size_t wdfmi_lds_bytes(const WdfmiLaunch& a) { return lds_doubles(a) * 8; }

hipError_t wdfmi_launch(const WdfmiLaunch& in, hipStream_t st) {
  if (in.nrec == 0 || in.nbuf == 0) return hipSuccess;
  WdfmiLaunch a = in;
  a.t_rcp = 1.0 / a.f_samp;
  a.t_fast = (a.accel & 1) ? 1 : 0;
  for (int k = 0; k <= a.R && a.t_fast; ++k) {
    const double kd = (double)k, q = kd * a.t_rcp;
    if (std::fma(std::fma(-q, a.f_samp, kd), a.t_rcp, q) != kd / a.f_samp) a.t_fast = 0;
  }
  // one wave per SIMD and 16 samples per thread measured fastest at R = 4000 (256 vs
  // 512 vs 1024 threads: scripts/bench_wdfmi.py --threads); larger R widens the group
  if (a.R <= 16 * 256) return launch_t<256, 16>(a, st);
  return launch_t<1024, 16>(a, st);
}

}  // namespace dfmi

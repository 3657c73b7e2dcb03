// lm_phase.h — the row-layout LM (chunk size 1: _fit_parallel, fitters.py:395-428 ->
// fit.fit per buffer, fit.py:322-361) in two phases with compaction between them.
//
// Why: the LM is VALU-issue bound (fp64: 8 cycles per wave instruction) and a wave runs
// its lanes' passes in lock step, so a wave costs (its slowest lane's passes) x (one
// pass). At m = 6, 40 dB half the segments finish their descent in 3 passes (3
// acceptances, the last below the 1e-9 step); the rest need up to 10 (two acceptances,
// then 8 lambdas that no longer lower ssq, fit.py:246-247), so most waves run ~10
// passes for ~6.8 useful per lane (scripts/lm_refill_probe.py, r02f).
//
// Phase A (lm_phase_a_kernel): every segment, one lane each (the lm_chunks_kernel
// layout: the wave's 64 rows staged into LDS), runs the first evaluation and at most
// `pa` passes of the flattened descent (lm_descend_flat's loop, lm.h). A lane whose
// descent ends with ssq < FITOK_THRESHOLD writes its result (status 0). Every other lane
// appends its state (p, the current J^T J / J^T r / ssq, iteration and lambda index, or
// "descent done, m-grid retry pending") to a compact list (one atomic per wave).
// Phase B (lm_phase_b_kernel): a persistent grid over the list, one lane per item:
// the item's row is gathered into LDS, its descent resumes where phase A left it, then
// fit.py:334-361 (m-grid retry, status, normalisation) as fit_segment_t does.
// Per lane the sequence of solves, trials and acceptances is exactly the one-phase
// kernel's: same bits (tests/test_gpu_numerics.py::test_lm_phase_bit_identical).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lm.h"

namespace dfmi {

// State of one flattened descent (lm_descend_flat): point, evaluation at the point,
// accepted steps so far, position on the lambda ladder.
struct FlatState {
  double p[4];
  Eval e;
  int it, li;
};

// Passes of lm_descend_flat's loop from state s, at most max_pass (< 0: no cap).
// Returns true when the descent has ended (converged, no lambda improved, MAX_LMA_STEPS).
template <typename Ev>
DFMI_HDI bool lm_flat_passes(Ev& ev, FlatState& s, const LMConst& c, int max_pass) {
  if (!(c.max_steps > 0 && c.n_lambda > 0)) return true;
  for (int pass = 0; max_pass < 0 || pass < max_pass; ++pass) {
    double dp[4];
    ev.solve(s.e, c.lambdas[s.li], dp);
    bool accepted = false;
    if (!norm_below(sumsq4(dp[0], dp[1], dp[2], dp[3]), c.min_step_norm)) {
      double pt[4] = {s.p[0] + dp[0], s.p[1] + dp[1], s.p[2] + dp[2], s.p[3] + dp[3]};
      typename std::decay_t<Ev>::Trial tt;
      const double ssq_try = ev.trial(pt, tt);
      if (ssq_try < s.e.ssq) {
        accepted = true;
        const double change2 = sumsq4(pt[0] - s.p[0], pt[1] - s.p[1], pt[2] - s.p[2], pt[3] - s.p[3]);
        s.p[0] = pt[0];
        s.p[1] = pt[1];
        s.p[2] = pt[2];
        s.p[3] = pt[3];
        const double best_ssq = ssq_try;
        ev.accept(s.p, tt, s.e);
        ++s.it;
        s.li = 0;
        if (((s.e.ssq - best_ssq) < c.conv_improve && norm_below(change2, c.conv_param_change)) ||
            s.it >= c.max_steps)
          return true;
      }
    }
    if (!accepted && ++s.li >= c.n_lambda) return true;
  }
  return false;
}

// fit.py:341-361 after the first descent ended at (p, ssq) with ssq >= the threshold:
// m-grid guess, second descent, keep the better, status 1 / 2 (fit_segment_t).
template <typename Ev, typename QF>
DFMI_HDI int lm_retry_and_status(Ev& ev, const QF& q, int ndata, const double* __restrict__ jtab, const LMConst& c,
                                 double (&p)[4], double& ssq) {
  double g[4];
  m_grid_seed(q, ndata, jtab, c, g);
  if (!(g[0] == 0.0) || !(g[1] == 0.0) || !(g[2] == 0.0) || !(g[3] == 0.0)) {  // np.any
    const double ssq2 = lm_descend_flat(ev, g, c);
    if (ssq2 < ssq) {
      ssq = ssq2;
      p[0] = g[0];
      p[1] = g[1];
      p[2] = g[2];
      p[3] = g[3];
    }
  }
  return (ssq < c.fitok_threshold) ? 1 : 2;
}

// fit.py:350-357: a < 0 -> (-a, phi + pi), m < 0 -> (-m, phi + pi), phi wrapped to [-pi, pi)
DFMI_HDI void lm_normalise(double (&p)[4]) {
  const double pi = 3.141592653589793;
  if (p[0] < 0.0) {
    p[0] = -p[0];
    p[2] += pi;
  }
  if (p[1] < 0.0) {
    p[1] = -p[1];
    p[2] += pi;
  }
  p[2] = dfmi_pymod(p[2] + pi, 2.0 * pi) - pi;
}

// The compact list between the phases (SoA, cap entries): kLmSt doubles per item
// [p0..p3, ssq, a00, a01, a02, a11, a12, a22, a33, g0, g1, g2, g3] and an int4
// (segment low / high 32 bits, it, li | flags).
constexpr int kLmSt = 16;
constexpr int kLmRetry = 1 << 16;  // li field flag: descent done, m-grid retry pending

// Stage row `s` of a lane into column `lane` of a [pos][65] LDS tile (QS positions).
DFMI_HDI void lm_stage_row(const double* __restrict__ qi, int64_t qi_ld, int64_t s, int QS, double* lds, int lane) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  const double* __restrict__ r = qi + s * qi_ld;
#pragma unroll 4
  for (int pos = 0; pos < QS; pos += 2) {
    const d2v v = *reinterpret_cast<const d2v*>(r + pos);
    lds[pos * 65 + lane] = v.x;
    lds[(pos + 1) * 65 + lane] = v.y;
  }
}

// Phase A: items u in [0, nrec * nitems): record r = u / nitems, segment
// r * nbuf + first + u % nitems; guess[r * g_rec + i * g_comp] seeds record r.
// Also writes every item's dc (out[4]) and the seed buffers' dc (segments before first).
// WPE: waves per SIMD the register allocation must allow (2: <= 256 VGPRs).
template <int V, int WPE = 1>
__global__ __launch_bounds__(64, WPE) void lm_phase_a_kernel(const double* __restrict__ qi, int64_t qi_ld, int ndata,
                                                        int64_t nrec, int64_t nbuf, int64_t first, int64_t nitems,
                                                        int pa, const double* __restrict__ guess, int64_t g_rec,
                                                        int64_t g_comp, const double* __restrict__ jtab, LMConst c,
                                                        double* __restrict__ out, int64_t out_ld,
                                                        int32_t* __restrict__ status, double* __restrict__ lst,
                                                        int4* __restrict__ lmeta, int64_t cap,
                                                        unsigned long long* __restrict__ lcount) {
  extern __shared__ double lds_q[];  // [qi_ld][65]
  const int lane = threadIdx.x;
  const int QS = (int)qi_ld;
  const int64_t total = nrec * nitems;
  const int64_t u = (int64_t)blockIdx.x * 64 + lane;
  const bool valid = u < total;
  const int64_t uc = valid ? u : 0;
  const int64_t r = uc / nitems;
  const int64_t s = r * nbuf + first + (uc - r * nitems);
  {  // stage: contiguous rows with coalesced 16-B loads, else per lane
    const int64_t s0 = __shfl(s, 0);
    const int nv = (int)((total - (int64_t)blockIdx.x * 64) < 64 ? (total - (int64_t)blockIdx.x * 64) : 64);
    const bool contiguous = __all(!valid || s == s0 + lane);
    if (contiguous) {
      typedef double d2v __attribute__((ext_vector_type(2)));
      const double* __restrict__ base = qi + s0 * qi_ld;
      const int tot = nv * QS;
      for (int e = 2 * lane; e < tot; e += 128) {
        const d2v v = *reinterpret_cast<const d2v*>(base + e);
        const int row = e / QS, pos = e - row * QS;
        lds_q[pos * 65 + row] = v.x;
        lds_q[(pos + 1) * 65 + row] = v.y;
      }
    } else if (valid) {
      lm_stage_row(qi, qi_ld, s, QS, lds_q, lane);
    }
    __syncthreads();
  }
  if (!valid) return;
  const QRow<65> q{lds_q + lane};
  {
    out[4 * out_ld + s] = q.at(dfmi_row_dc(ndata));
    if (uc - r * nitems == 0)  // the record's seed buffers (fitted elsewhere): carry their dc
      for (int64_t t = r * nbuf; t < r * nbuf + first; ++t) out[4 * out_ld + t] = qi[t * qi_ld + dfmi_row_dc(ndata)];
  }
  SplitEval<V, QRow<65>> ev{q, ndata, c.trig};
  FlatState st;
#pragma unroll
  for (int i = 0; i < 4; ++i) st.p[i] = guess[r * g_rec + i * g_comp];
  {
    typename SplitEval<V, QRow<65>>::Trial t0;
    ev.trial(st.p, t0);
    ev.accept(st.p, t0, st.e);
  }
  st.it = 0;
  st.li = 0;
  const bool ended = lm_flat_passes(ev, st, c, pa);
  const bool finished = ended && (st.e.ssq < c.fitok_threshold);
  if (valid && finished) {
    lm_normalise(st.p);
    out[0 * out_ld + s] = st.p[0];
    out[1 * out_ld + s] = st.p[1];
    out[2 * out_ld + s] = st.p[2];
    out[3 * out_ld + s] = st.p[3];
    out[5 * out_ld + s] = st.e.ssq;
    status[s] = 0;
  }
  // the rest to the compact list: one atomic per wave
  const bool pend = valid && !finished;
  const uint64_t bal = __ballot(pend);
  if (bal == 0) return;
  const int leader = __ffsll((unsigned long long)bal) - 1;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(lcount, (unsigned long long)__popcll(bal));
  base = __shfl(base, leader);
  if (pend) {
    const int64_t k = (int64_t)base + __popcll(bal & ((1ull << lane) - 1ull));
    if (k < cap) {
      const double v[kLmSt] = {st.p[0], st.p[1], st.p[2], st.p[3], st.e.ssq, st.e.a00, st.e.a01, st.e.a02,
                               st.e.a11, st.e.a12, st.e.a22, st.e.a33, st.e.g0, st.e.g1, st.e.g2, st.e.g3};
#pragma unroll
      for (int i = 0; i < kLmSt; ++i) lst[(int64_t)i * cap + k] = v[i];
      lmeta[k] = make_int4((int)(s & 0xffffffff), (int)(s >> 32), st.it, st.li | (ended ? kLmRetry : 0));
    }
  }
}

// Phase B: a persistent grid over the *lcount items of the list (cap bounds it).
template <int V>
__global__ __launch_bounds__(64) void lm_phase_b_kernel(const double* __restrict__ qi, int64_t qi_ld, int ndata,
                                                        const double* __restrict__ jtab, LMConst c,
                                                        double* __restrict__ out, int64_t out_ld,
                                                        int32_t* __restrict__ status, const double* __restrict__ lst,
                                                        const int4* __restrict__ lmeta, int64_t cap,
                                                        const unsigned long long* __restrict__ lcount) {
  extern __shared__ double lds_q[];  // [qi_ld][65]
  const int lane = threadIdx.x;
  const int QS = (int)qi_ld;
  int64_t n = (int64_t)*lcount;
  if (n > cap) n = cap;
  for (int64_t k0 = (int64_t)blockIdx.x * 64; k0 < n; k0 += (int64_t)gridDim.x * 64) {
    const int64_t k = k0 + lane;
    const bool valid = k < n;
    const int64_t kc = valid ? k : k0;
    const int4 m = lmeta[kc];
    const int64_t s = (int64_t)(uint32_t)m.x | ((int64_t)m.y << 32);
    lm_stage_row(qi, qi_ld, s, QS, lds_q, lane);
    __syncthreads();
    const QRow<65> q{lds_q + lane};
    SplitEval<V, QRow<65>> ev{q, ndata, c.trig};
    FlatState st;
    double v[kLmSt];
#pragma unroll
    for (int i = 0; i < kLmSt; ++i) v[i] = lst[(int64_t)i * cap + kc];
#pragma unroll
    for (int i = 0; i < 4; ++i) st.p[i] = v[i];
    st.e = Eval{v[4], v[5], v[6], v[7], 0.0, v[8], v[9], 0.0, v[10], 0.0, v[11], v[12], v[13], v[14], v[15]};
    st.it = m.z;
    st.li = m.w & (kLmRetry - 1);
    if (!(m.w & kLmRetry)) lm_flat_passes(ev, st, c, -1);  // resume the first descent
    double ssq = st.e.ssq;
    int stt = 0;
    if (!(ssq < c.fitok_threshold)) stt = lm_retry_and_status(ev, q, ndata, jtab, c, st.p, ssq);
    lm_normalise(st.p);
    if (valid) {
      out[0 * out_ld + s] = st.p[0];
      out[1 * out_ld + s] = st.p[1];
      out[2 * out_ld + s] = st.p[2];
      out[3 * out_ld + s] = st.p[3];
      out[5 * out_ld + s] = ssq;
      status[s] = stt;
    }
    __syncthreads();  // the tile is restaged for the next round
  }
}

}  // namespace dfmi

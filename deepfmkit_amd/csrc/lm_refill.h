// lm_refill.h — the LM over demodulation rows with lane refill (chunk size 1, the
// _fit_parallel path of the record pipeline; fitters.py:395-428 -> fit.fit per buffer,
// fit.py:322-361).
//
// Why: with one lane per segment and one segment per lane (lm_chunks_kernel), a wave
// runs until its slowest lane is done: at m = 6, 40 dB a lane needs ~6.8 LM passes
// (solve + trial) on average while its wave runs ~9-10, and every pass in which any
// lane accepts also runs the accept (Jacobian) evaluation. The LM is VALU-issue bound
// (scripts/lm_scaling.py: time grows linearly with waves per SIMD), so the idle lanes
// of those passes are the cost.
//
// Here ONE WAVE OWNS A TILE of up to TMAX segments, staged once into LDS (transposed,
// [pos][T+1]), and every lane runs a per-lane state machine of the flattened descent
// (lm_descend_flat, lm.h): each pass is ONE damped solve + ONE full evaluation (ssqf and
// coeffs fused: eval_reg_full) for every lane, wherever it stands on its lambda ladder;
// a lane whose fit ends writes its segment's result and takes the tile's next segment in
// the same pass. The wave runs ~sum(passes) / 64 + a tail instead of 64 x max(passes).
// Per lane the sequence of solves, trials and acceptances is exactly the reference's
// nested loop (fit.py:208-258), and the m-grid retry of fit.py:334-349 runs as a second
// descent of the same lane (its first result parked in LDS).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lm.h"

namespace dfmi {

// QI of one lane's segment in the wave's transposed LDS tile: pos -> p[pos * ld]
struct QRowT {
  const double* __restrict__ p;
  int ld;
  DFMI_HDI double qc(int h) const { return p[((h >> 3) * 16 + (h & 7)) * ld]; }
  DFMI_HDI double qs(int h) const { return p[((h >> 3) * 16 + 8 + (h & 7)) * ld]; }
  DFMI_HDI double at(int pos) const { return p[pos * ld]; }
};

constexpr int kRefillTmax = 128;  // segments per wave tile (32 x 129 doubles = 33 KB LDS at ndata <= 16)

// LDS bytes of one refill workgroup (one wave): the tile + the parked first descents
inline size_t lm_refill_lds(int qs, int tile) {
  return ((size_t)qs * (tile + 1) + 64 * 5 + kMaxLambda) * sizeof(double);
}

// Items u in [0, nrec * nitems): record r = u / nitems, segment r * nbuf + first + u % nitems
// (the record's segments after the seed buffers). Wave b owns items [b * tile, ...).
// guess[r * g_rec + i * g_comp]: record r's seed (the fitted buffer 0 on the device).
// ROWS = true: qi holds demodulation rows (qi + s * qi_ld, dfmi_qi_row_stride); the
// kernel also writes each segment's dc (out[4]) and carries the seed buffers' dc.
// ROWS = false: qi is component-major (qi[c * qi_ld + s], dfmi_demod's layout), staged
// into the same row positions; dc is the caller's.
// WPE: waves per SIMD the register allocation must allow (1, or 2 = at most 256 VGPRs).
template <int V, bool ROWS = true, int WPE = 1>
__global__ __launch_bounds__(64, WPE) void lm_refill_kernel(const double* __restrict__ qi, int64_t qi_ld, int ndata,
                                                       int64_t nrec, int64_t nbuf, int64_t first, int64_t nitems,
                                                       int tile, const double* __restrict__ guess, int64_t g_rec,
                                                       int64_t g_comp, const double* __restrict__ jtab, LMConst c,
                                                       double* __restrict__ out, int64_t out_ld,
                                                       int32_t* __restrict__ status,
                                                       unsigned long long* __restrict__ probe) {
  // probe (diagnostics, may be null): [8] passes, [9] lane-passes with an item,
  // [10] wave cycles (s_memtime), [11] waves, [12] cycles in the evaluations
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
  uint64_t n_pass = 0, n_busy = 0, t_eval = 0, t_solve = 0, t_done = 0, t_stage = 0;
  extern __shared__ double lds[];
  const int lane = threadIdx.x;
  const int QS = ROWS ? (int)qi_ld : dfmi_row_stride(ndata);  // LDS positions per segment
  const int TP = tile + 1;                // odd row pitch of the transposed tile
  double* __restrict__ park = lds + (size_t)QS * TP;  // [5][64]: p, ssq of a lane's first descent
  // the lambda ladder (fit.py:222) in LDS: a lane-indexed read of the kernel-argument
  // copy would be a vector memory load, and on gfx9 a wait for it also waits for every
  // result store still in flight (one counter for loads and stores)
  double* __restrict__ lam = park + 5 * 64;
  if (lane < kMaxLambda) lam[lane] = c.lambdas[lane < c.n_lambda ? lane : 0];
  const int64_t total = nrec * nitems;
  const int64_t u0 = (int64_t)blockIdx.x * tile;
  if (u0 >= total) return;
  const int nt = (int)((total - u0) < tile ? (total - u0) : tile);
  auto seg_of = [&](int64_t u) {
    const int64_t r = u / nitems;
    return r * nbuf + first + (u - r * nitems);
  };

  // ---- stage the tile's rows, transposed into [pos][TP]: every load of a group of
  // kStageLoads issued before the first LDS write (one memory round trip per group) ----
  constexpr int kStageLoads = 8;
  if constexpr (!ROWS) {  // component c of the tile's segments: coalesced along segments
    const int tot = 2 * ndata * nt;
    for (int e0 = 0; e0 < tot; e0 += 64 * kStageLoads) {
      double v[kStageLoads];
#pragma unroll
      for (int k = 0; k < kStageLoads; ++k) {
        const int e = e0 + 64 * k + lane;
        const int ec = e < tot ? e : 0;
        const int cc = ec / nt, row = ec - cc * nt;
        v[k] = qi[(int64_t)cc * qi_ld + seg_of(u0 + row)];
      }
#pragma unroll
      for (int k = 0; k < kStageLoads; ++k) {
        const int e = e0 + 64 * k + lane;
        if (e < tot) {
          const int cc = e / nt, row = e - cc * nt;
          const int h = cc < ndata ? cc : cc - ndata;
          const int pos = (h >> 3) * 16 + (cc < ndata ? 0 : 8) + (h & 7);
          lds[pos * TP + row] = v[k];
        }
      }
    }
  } else {
    typedef double d2v __attribute__((ext_vector_type(2)));
    const int tot = nt * QS;  // doubles (QS even)
    const bool contiguous = (nrec == 1) || (seg_of(u0 + nt - 1) - seg_of(u0) == nt - 1);
    const double* __restrict__ base = qi + seg_of(u0) * qi_ld;
    for (int e0 = 0; e0 < tot; e0 += 128 * kStageLoads) {
      d2v v[kStageLoads];
#pragma unroll
      for (int k = 0; k < kStageLoads; ++k) {
        const int e = e0 + 128 * k + 2 * lane;
        const int ec = e < tot ? e : 0;
        const int row = ec / QS, pos = ec - row * QS;
        v[k] = contiguous ? *reinterpret_cast<const d2v*>(base + ec)
                          : *reinterpret_cast<const d2v*>(qi + seg_of(u0 + row) * qi_ld + pos);
      }
#pragma unroll
      for (int k = 0; k < kStageLoads; ++k) {
        const int e = e0 + 128 * k + 2 * lane;
        if (e < tot) {
          const int row = e / QS, pos = e - row * QS;
          lds[pos * TP + row] = v[k].x;
          lds[(pos + 1) * TP + row] = v[k].y;
        }
      }
    }
    // dc of the seed buffers (segments before `first`, fitted elsewhere) rides with the
    // tile holding the record's first item
    for (int e = lane; e < nt; e += 64) {
      const int64_t u = u0 + e;
      if (u % nitems == 0) {
        const int64_t r = u / nitems;
        for (int64_t t = r * nbuf; t < r * nbuf + first; ++t)
          out[4 * out_ld + t] = qi[t * qi_ld + dfmi_row_dc(ndata)];
      }
    }
  }
  __syncthreads();

  if (probe) t_stage = __builtin_amdgcn_s_memtime() - t_start;
  // ---- per-lane state ----
  int slot = lane < nt ? lane : -1;  // the lane's item within the tile (-1: none)
  int next = nt < 64 ? nt : 64;      // wave-uniform: the tile's next unassigned item
  double p[4];
  // the seed of the tile's first record stays in registers: a refill then needs no
  // global load (a tile spans two records only at a record boundary)
  const int64_t r0 = u0 / nitems;
  const int64_t r0_end = (r0 + 1) * nitems;  // first item of the next record
  double g0[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) g0[i] = guess[r0 * g_rec + i * g_comp];
  auto load_guess = [&](int sl) {
    const int64_t u = u0 + sl;
    if (u < r0_end) {
#pragma unroll
      for (int i = 0; i < 4; ++i) p[i] = g0[i];
    } else {
      const int64_t r = u / nitems;
#pragma unroll
      for (int i = 0; i < 4; ++i) p[i] = guess[r * g_rec + i * g_comp];
    }
  };
  if (slot >= 0) load_guess(slot);
  else p[0] = p[1] = p[2] = p[3] = 1.0;  // finite, never used: keeps idle lanes off slow paths
  Eval e;
  eval_zero(e);
  int it = 0, li = 0;
  bool init = true;   // next pass evaluates p itself (the descent's first coeffs, fit.py:215)
  int phase = 0;      // 0: first descent, 1: the descent from the m-grid guess
  const bool ladder = c.max_steps > 0 && c.n_lambda > 0;

  while (__any(slot >= 0)) {
    const int sl = slot >= 0 ? slot : 0;
    const QRowT q{lds + sl, TP};
    // one damped solve (skipped in effect for init lanes) ...
    double dp[4];
    const uint64_t ts0 = probe ? __builtin_amdgcn_s_memtime() : 0;
    damped_solve_block(e, lam[li], dp);
    const bool tiny = norm_below(sumsq4(dp[0], dp[1], dp[2], dp[3]), c.min_step_norm);
    double pt[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) pt[i] = init ? p[i] : p[i] + dp[i];
    // ... and one full evaluation for every lane
    Eval et;
    const uint64_t te0 = probe ? __builtin_amdgcn_s_memtime() : 0;
    if (probe) t_solve += te0 - ts0;
    eval_reg_full<V>(q, ndata, pt, et, c.trig);
    if (probe) {
      t_eval += __builtin_amdgcn_s_memtime() - te0;
      ++n_pass;
      n_busy += __popcll(__ballot(slot >= 0));
    }
    bool done = false;
    if (slot >= 0) {
      if (init) {
        e = et;
        it = 0;
        li = 0;
        init = false;
        done = !ladder;
      } else if (!tiny && et.ssq < e.ssq) {  // fit.py:240-243: first improving lambda wins
        const double change2 = sumsq4(pt[0] - p[0], pt[1] - p[1], pt[2] - p[2], pt[3] - p[3]);
        const double best_ssq = et.ssq;
#pragma unroll
        for (int i = 0; i < 4; ++i) p[i] = pt[i];
        e = et;  // coeffs at the accepted point (fit.py:250-251)
        ++it;
        li = 0;
        if (((e.ssq - best_ssq) < c.conv_improve && norm_below(change2, c.conv_param_change)) ||
            it >= c.max_steps)
          done = true;
      } else if (++li >= c.n_lambda) {  // no lambda improved (fit.py:246-247)
        done = true;
      }
    }
    const uint64_t td0 = probe ? __builtin_amdgcn_s_memtime() : 0;
    if (done) {  // fit.py:334-361 for this lane's descent
      double ssq = e.ssq;
      bool finished = true;
      int st = 0;
      if (phase == 0) {
        if (!(ssq < c.fitok_threshold)) {
          double g[4];
          m_grid_seed(q, ndata, jtab, c, g);
          if (!(g[0] == 0.0) || !(g[1] == 0.0) || !(g[2] == 0.0) || !(g[3] == 0.0)) {  // np.any
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              park[i * 64 + lane] = p[i];
              p[i] = g[i];
            }
            park[4 * 64 + lane] = ssq;
            phase = 1;
            init = true;
            finished = false;
          } else {
            st = 2;  // ssq >= threshold and no grid guess: status 2 (fit.py:349)
          }
        }
      } else {
        const double ssq1 = park[4 * 64 + lane];
        if (!(ssq < ssq1)) {  // keep the first descent unless the retry is better (fit.py:341-345)
          ssq = ssq1;
#pragma unroll
          for (int i = 0; i < 4; ++i) p[i] = park[i * 64 + lane];
        }
        st = (ssq < c.fitok_threshold) ? 1 : 2;
      }
      if (finished) {
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
        // the result goes into the item's own (now dead) LDS column, positions 0..6; the
        // wave stores the tile's results coalesced after the loop: a store in the loop
        // would make every later wait on vector memory also wait for it (gfx9 counts
        // loads and stores together)
        double* col = lds + slot;
        const double dcv = ROWS ? q.at(dfmi_row_dc(ndata)) : 0.0;
        col[0 * TP] = p[0];
        col[1 * TP] = p[1];
        col[2 * TP] = p[2];
        col[3 * TP] = p[3];
        col[4 * TP] = dcv;
        col[5 * TP] = ssq;
        col[6 * TP] = (double)st;
        slot = -1;
      }
    }
    if (probe) t_done += __builtin_amdgcn_s_memtime() - td0;
    // refill: lanes without an item take the tile's next ones, in lane order
    const bool need = slot < 0;
    const uint64_t bal = __ballot(need);
    if (next < nt && bal) {
      const int rank = __popcll(bal & ((1ull << lane) - 1ull));
      if (need && next + rank < nt) {
        slot = next + rank;
        load_guess(slot);
        init = true;
        phase = 0;
      }
      next += __popcll(bal);
    }
  }
  // ---- the tile's results, coalesced ----
  for (int e = lane; e < nt; e += 64) {
    const int64_t sg = seg_of(u0 + e);
    out[0 * out_ld + sg] = lds[0 * TP + e];
    out[1 * out_ld + sg] = lds[1 * TP + e];
    out[2 * out_ld + sg] = lds[2 * TP + e];
    out[3 * out_ld + sg] = lds[3 * TP + e];
    if constexpr (ROWS) out[4 * out_ld + sg] = lds[4 * TP + e];
    out[5 * out_ld + sg] = lds[5 * TP + e];
    status[sg] = (int32_t)lds[6 * TP + e];
  }
  if (probe && lane == 0) {
    atomicAdd(probe + 8, (unsigned long long)n_pass);
    atomicAdd(probe + 9, (unsigned long long)n_busy);
    atomicAdd(probe + 10, (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
    atomicAdd(probe + 11, 1ull);
    atomicAdd(probe + 12, (unsigned long long)t_eval);
    atomicAdd(probe + 13, (unsigned long long)t_solve);
    atomicAdd(probe + 14, (unsigned long long)t_done);
    atomicAdd(probe + 15, (unsigned long long)t_stage);
  }
}

}  // namespace dfmi

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

#include "dfmi_math.h"

namespace dfmi {

constexpr int kWavesPerBlock = 4;
constexpr int kBlockThreads = 64 * kWavesPerBlock;
constexpr int kHarmBlock = 8;  // harmonics per contraction block (16 partial sums)

// One exchange stage of the reduce-scatter: lanes with the mask bit set keep
// the upper HALF of their live values, the others the lower half, and each adds
// its partner's copy of the half it keeps.
template <int HALF, int MASK, int NV>
__device__ __forceinline__ void bfly_stage(double (&v)[NV], int lane) {
  const bool hi = lane & MASK;
#pragma unroll
  for (int i = 0; i < HALF; ++i) {
    const double send = hi ? v[i] : v[i + HALF];
    const double keep = hi ? v[i + HALF] : v[i];
    v[i] = keep + __shfl_xor(send, MASK);
  }
}

// Reduce-scatter of NV (4, 8 or 16) per-lane partial sums over a wavefront: the
// exchange stages (masks 32, 16, ...) halve the live values, the remaining
// stages are plain butterfly sums. On return lane l holds, in v[0], the
// wave-wide sum of value index (l >> (6 - log2 NV)) & (NV - 1).
// (NV = 16: 15 exchange-adds + 2 sums = 17 shuffles instead of 16 x 6.)
template <int NV>
__device__ __forceinline__ void butterfly(double (&v)[NV], int lane) {
  static_assert(NV == 4 || NV == 8 || NV == 16, "NV");
  if constexpr (NV == 16) {
    bfly_stage<8, 32>(v, lane);
    bfly_stage<4, 16>(v, lane);
    bfly_stage<2, 8>(v, lane);
    bfly_stage<1, 4>(v, lane);
    v[0] += __shfl_xor(v[0], 2);
    v[0] += __shfl_xor(v[0], 1);
  } else if constexpr (NV == 8) {
    bfly_stage<4, 32>(v, lane);
    bfly_stage<2, 16>(v, lane);
    bfly_stage<1, 8>(v, lane);
    v[0] += __shfl_xor(v[0], 4);
    v[0] += __shfl_xor(v[0], 2);
    v[0] += __shfl_xor(v[0], 1);
  } else {
    bfly_stage<2, 32>(v, lane);
    bfly_stage<1, 16>(v, lane);
    v[0] += __shfl_xor(v[0], 8);
    v[0] += __shfl_xor(v[0], 4);
    v[0] += __shfl_xor(v[0], 2);
    v[0] += __shfl_xor(v[0], 1);
  }
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

// Write one block of HB harmonics (2·HB sums, after butterfly<2·HB>) of segment s.
template <int HB>
__device__ __forceinline__ void store_block(const double (&v)[2 * HB], int lane, int hb, int ndata,
                                            double* __restrict__ qi, int64_t qi_ld, int64_t s, int R) {
  constexpr int SH = (HB == 8) ? 2 : (HB == 4) ? 3 : 4;  // 6 - log2(2·HB)
  if ((lane & ((1 << SH) - 1)) == 0) {
    const int vi = lane >> SH;
    const int h = hb * HB + (vi % HB);
    if (h < ndata) {
      const int c = (vi / HB) ? (ndata + h) : h;
      qi[(int64_t)c * qi_ld + s] = v[0] / (double)R;  // numpy mean: sum / count
    }
  }
}

// One value of a demodulation row. The row lives in global memory (the record pipeline's
// rows, written once and read once by the LM: non-temporal) or in LDS (the seed step's row,
// seed.h, fitted in place): ROW_LDS says which, statically, and each case stores through a
// pointer of its own address space — a global-only store instruction aimed at an LDS
// address faults (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION, seen in round 3 with an A/B
// variant that sent both rows through one global `sc1 nt` store). Built with
// -DDFMI_DEBUG_ROWS, every store also checks the pointer's aperture against ROW_LDS
// (__graft_entry__.build() builds it as ab/libdfmi_dbg.so; tests/test_gpu_debug_build.py runs
// the record pipeline through it once).
template <bool ROW_LDS>
__device__ __forceinline__ void row_put(double* p, double v) {
#if defined(DFMI_DEBUG_ROWS) && defined(__HIP_DEVICE_COMPILE__)
  if (__builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)p) != ROW_LDS) __builtin_trap();
#endif
  if constexpr (ROW_LDS) {
    typedef __attribute__((address_space(3))) double lds_double;
    *(lds_double*)p = v;  // ds_write_b64
  } else {
    typedef __attribute__((address_space(1))) double global_double;
    __builtin_nontemporal_store(v, (global_double*)p);  // global_store_dwordx2 ... nt
  }
}

// dc part of fold_finish: the lane's partial sum of its bins (returned), and dc itself
// (wave sum / R) unless the row layout carries it in a spare Q slot.
template <int VEC, int MAXSLOT, int HB, bool ROWS, bool ROW_LDS = false>
__device__ __forceinline__ double finish_dc(const double (&y)[MAXSLOT][VEC], int R, int ndata, int lane,
                                            double* __restrict__ qi, int64_t qi_ld, int64_t col,
                                            double* __restrict__ dc) {
  double tot = 0.0;
#pragma unroll
  for (int j = 0; j < MAXSLOT; ++j)
#pragma unroll
    for (int e = 0; e < VEC; ++e) tot += y[j][e];
  static_assert(!ROWS || HB == 8, "row layout uses 8-harmonic blocks");
  const int spare = ndata % HB;  // ROWS: dc slot in the last block (0: no spare slot)
  if (!ROWS || spare == 0) {
    const double all = wave_sum(tot);
    if (lane == 0) {
      if constexpr (ROWS) row_put<ROW_LDS>(qi + col * qi_ld + dfmi_row_dc(ndata), all / (double)R);
      else dc[col] = all / (double)R;
    }
  }
  return tot;
}

// Harmonic block hb of fold_finish: HB harmonics contracted with the basis, reduced by
// the butterfly and stored (tot: finish_dc's partial sum, for the rows' dc slot).
template <int VEC, int MAXSLOT, int HB, bool ROWS, bool ROW_LDS = false>
__device__ __forceinline__ void finish_block(const double (&y)[MAXSLOT][VEC], const bool (&pval)[MAXSLOT],
                                             const int (&pbase)[MAXSLOT], double tot, int hb, int R, int L,
                                             int ndata, const double* __restrict__ T, int lane,
                                             double* __restrict__ qi, int64_t qi_ld, int64_t col) {
  const int nblk = (ndata + HB - 1) / HB;
  const int spare = ndata % HB;
  double acc[2 * HB];
#pragma unroll
  for (int i = 0; i < 2 * HB; ++i) acc[i] = 0.0;
  if constexpr (ROWS) {
    if (spare && hb == nblk - 1) {
#pragma unroll
      for (int i = 0; i < HB; ++i)
        if (i == spare) acc[i] = tot;  // Q slot of harmonic >= ndata: no basis term lands here
    }
  }
#pragma unroll
  for (int j = 0; j < MAXSLOT; ++j) {
    if (!pval[j]) continue;
#pragma unroll
    for (int h = 0; h < HB; ++h) {
      const int hh = hb * HB + h;
      if (hh < ndata) {
        double bc[VEC], bs[VEC];
        VecT<VEC>::load(T + (int64_t)hh * L + pbase[j], bc);
        VecT<VEC>::load(T + (int64_t)(ndata + hh) * L + pbase[j], bs);
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          acc[h] = fma(y[j][e], bc[e], acc[h]);
          acc[HB + h] = fma(y[j][e], bs[e], acc[HB + h]);
        }
      }
    }
  }
  butterfly<2 * HB>(acc, lane);
  if constexpr (ROWS) {
    // one 128-B line, non-temporal: plain row stores cost the bin kernel 3.5 % (0.520 vs
    // 0.502 ms per 100k segments, profiles/r02l_ab_store.log)
    if ((lane & 3) == 0) row_put<ROW_LDS>(qi + col * qi_ld + hb * 16 + (lane >> 2), acc[0] / (double)R);
  } else {
    store_block<HB>(acc, lane, hb, ndata, qi, qi_ld, col, R);
  }
}

// dc + contraction of the folded phase bins y (lane-owned, see fold_segment)
// with the basis table T, 8 harmonics per block; writes qi[:, col] and dc[col].
// ROWS = false: qi[c·qi_ld + col] (component-major) and dc[col].
// ROWS = true : the row layout of dfmi_qi_row_stride — qi + col·qi_ld holds the
// segment's row; with HB = 8 every block is one 128-B line written by one store
// instruction (16 lanes x 8 B), and dc rides in the last block's first spare Q
// slot: its per-lane partial sum enters the same reduce-scatter, whose pairing
// tree is wave_sum's, so dc is bit-identical to the ROWS = false value. (Scattered
// 8-B stores into 21 component rows cost 13 % of the demodulation time:
// profiles/r01_tune_demod_probe.json.)
template <int VEC, int MAXSLOT, int HB = kHarmBlock, bool ROWS = false, bool ROW_LDS = false>
__device__ __forceinline__ void fold_finish(const double (&y)[MAXSLOT][VEC], const bool (&pval)[MAXSLOT],
                                            const int (&pbase)[MAXSLOT], int R, int L, int ndata,
                                            const double* __restrict__ T, int lane, double* __restrict__ qi,
                                            int64_t qi_ld, int64_t col, double* __restrict__ dc) {
  const int nblk = (ndata + HB - 1) / HB;
  const double tot = finish_dc<VEC, MAXSLOT, HB, ROWS, ROW_LDS>(y, R, ndata, lane, qi, qi_ld, col, dc);
  for (int hb = 0; hb < nblk; ++hb)
    finish_block<VEC, MAXSLOT, HB, ROWS, ROW_LDS>(y, pval, pbase, tot, hb, R, L, ndata, T, lane, qi, qi_ld, col);
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

  fold_finish<VEC, MAXSLOT>(y, pval, pbase, R, L, ndata, T, lane, qi, qi_ld, col, dc);
}

// Basis table (n doubles, 16-B aligned) -> LDS at kernel start, each thread's loads all
// in flight before its first LDS write: a plain load-then-store loop waits one memory
// round trip per iteration (~19 at ndata 10, L 200), while every workgroup of the
// persistent grid starts at once and HBM is already saturated by the first segments.
__device__ __forceinline__ void stage_table(const double* __restrict__ tab, double* lds, int n, int tid,
                                            int nthreads) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  const d2v* __restrict__ src = reinterpret_cast<const d2v*>(tab);
  d2v* dst = reinterpret_cast<d2v*>(lds);
  const int n2 = n / 2;
  for (int base = 0; base < n2; base += nthreads * 16) {
    d2v v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = base + u * nthreads + tid;
      v[u] = i < n2 ? src[i] : d2v{0.0, 0.0};
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = base + u * nthreads + tid;
      if (i < n2) dst[i] = v[u];
    }
  }
  if ((n & 1) && tid == 0) lds[n - 1] = tab[n - 1];
}

template <int VEC, int MAXSLOT, bool LDS_TAB, int LOADS = 8, bool NT = true>
__global__ __launch_bounds__(kBlockThreads) void demod_fold_kernel(
    const double* __restrict__ x, int64_t nseg, int64_t seg_stride, int R, int L, int ndata,
    const double* __restrict__ tab, double* __restrict__ qi, int64_t qi_ld, double* __restrict__ dc) {
  extern __shared__ __attribute__((aligned(16))) double lds_tab[];
  if constexpr (LDS_TAB) {
    stage_table(tab, lds_tab, 2 * ndata * L, threadIdx.x, kBlockThreads);
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

// Bin-in-LDS fold: the same fold + contraction as demod_fold_kernel, but the
// segment is read the way HBM likes it — as flat, 1-KB-aligned wave loads
// (lane l reads x[128c + 2l .. +1] of chunk c), not cycle by cycle. A cycle of
// L = 200 doubles is 1600 B, so cycle-aligned wave loads start 64 B off a
// 128-B line every other cycle and the second slot is a 576-B partial load:
// measured 5.5 TB/s against 6.7 TB/s for the flat pattern
// (profiles/r01_readbw.jsonl, segwave_l8_nt_g4). The phase bins then cannot
// live in fixed lanes, so each wave keeps its L bins in LDS and adds every
// chunk into them with a ds_read_b128 / add / ds_write_b128 per lane (the 128
// consecutive samples of a chunk fall in 128 distinct bins when L >= 128, and a
// wave's LDS operations execute in order, so no atomics are needed). Every bin
// still receives its samples in ascending t from 0.0, exactly as in
// fold_segment, and the contraction is fold_finish on the same lane-owned
// bins: results are bit-identical to demod_fold_kernel.
// Preconditions (host-checked): 16-B aligned rows (x and seg_stride even),
// L even, 128 <= L <= 128·MAXSLOT.
// Measured and dropped (profiles/r01_tune_demod_stream.json, r01b_*): software
// pipelining the next batch across the contraction (slower for both load
// patterns: the 8-chunk bursts per wave stream better), 6-8 waves per SIMD with
// leaner contractions (no gain), LDS-DMA rings (readbw.hip: no gain over register
// loads), and dynamic segment queues on padded atomic counters (10 % slower).
// One segment of the bin-in-LDS fold: the wave's L bins (ybin, LDS) are zeroed,
// every 1-KB chunk is added into them, and fold_finish contracts the lane-owned
// bins with the basis T (LDS or global) into column / row `col` of qi (and dc).
// PFN > 0: the segment's first PFN chunks arrive prefetched in pf (nch >= PFN), and
// the next segment's first PFN chunks (at `next`, if not null) are issued into pf
// before this segment's contraction, so the wave has loads in flight while it
// contracts.
template <int MAXSLOT, int LOADS, bool NT, int HB, bool ROWS, int PFN = 0, bool ROW_LDS = false>
__device__ __forceinline__ void bins_segment(const double* __restrict__ xs0, int R, int L, int ndata,
                                             const double* __restrict__ T, double* __restrict__ ybin, int lane,
                                             const bool (&pval)[MAXSLOT], const int (&pbase)[MAXSLOT],
                                             double* __restrict__ qi, int64_t qi_ld, int64_t col,
                                             double* __restrict__ dc, double (*pf)[2] = nullptr,
                                             const double* __restrict__ next = nullptr) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  const int nch = R >> 7;           // full 128-sample chunks
  const int tail = R - (nch << 7);  // samples of the last, partial chunk
  auto add_chunk = [&](int p0, const double (&v)[2]) {
    int p = p0 + 2 * lane;
    if (p >= L) p -= L;
    d2v* yp = reinterpret_cast<d2v*>(ybin + p);
    d2v t = *yp;
    t.x += v[0];
    t.y += v[1];
    *yp = t;
  };
#pragma unroll
  for (int j = 0; j < MAXSLOT; ++j)
    if (pval[j]) *reinterpret_cast<d2v*>(ybin + pbase[j]) = d2v{0.0, 0.0};
  const double* __restrict__ xs = xs0 + 2 * lane;
  int p0 = 0;  // bin of the chunk's first sample: (128 c) mod L
  int c = 0;
  if constexpr (PFN > 0) {
#pragma unroll
    for (int u = 0; u < PFN; ++u) {
      add_chunk(p0, pf[u]);
      p0 += 128;
      if (p0 >= L) p0 -= L;
    }
    c = PFN;
  }
  for (; c + LOADS <= nch; c += LOADS) {
    double v[LOADS][2];
#pragma unroll
    for (int u = 0; u < LOADS; ++u) {
      if constexpr (NT) VecT<2>::load_nt(xs + (c + u) * 128, v[u]);
      else VecT<2>::load(xs + (c + u) * 128, v[u]);
    }
#pragma unroll
    for (int u = 0; u < LOADS; ++u) {
      add_chunk(p0, v[u]);
      p0 += 128;
      if (p0 >= L) p0 -= L;
    }
  }
  {
    // the remaining (< LOADS) full chunks and the partial tail chunk as ONE more load
    // group (issued together, then added in chunk order as before: same bits); one
    // HBM round trip instead of one per chunk
    const int rem = nch - c;
    double v[LOADS][2];
#pragma unroll
    for (int u = 0; u < LOADS; ++u) {
      if (u < rem) {
        if constexpr (NT) VecT<2>::load_nt(xs + (c + u) * 128, v[u]);
        else VecT<2>::load(xs + (c + u) * 128, v[u]);
      }
    }
    const int t0 = 2 * lane;
    double tv0 = 0.0, tv1 = 0.0;
    if (t0 < tail) tv0 = xs[nch * 128];  // partial chunk: element-wise (R may be odd)
    if (t0 + 1 < tail) tv1 = xs[nch * 128 + 1];
#pragma unroll
    for (int u = 0; u < LOADS; ++u) {
      if (u < rem) {
        add_chunk(p0, v[u]);
        p0 += 128;
        if (p0 >= L) p0 -= L;
      }
    }
    if (tail) {
      int p = p0 + t0;
      if (p >= L) p -= L;
      if (t0 < tail) ybin[p] += tv0;
      if (t0 + 1 < tail) ybin[p + 1] += tv1;
    }
  }
  if constexpr (PFN > 0) {
    if (next) {
      const double* __restrict__ xn = next + 2 * lane;
#pragma unroll
      for (int u = 0; u < PFN; ++u) {
        if constexpr (NT) VecT<2>::load_nt(xn + u * 128, pf[u]);
        else VecT<2>::load(xn + u * 128, pf[u]);
      }
    }
  }
  double y[MAXSLOT][2];
#pragma unroll
  for (int j = 0; j < MAXSLOT; ++j) {
    if (pval[j]) {
      const d2v t = *reinterpret_cast<const d2v*>(ybin + pbase[j]);
      y[j][0] = t.x;
      y[j][1] = t.y;
    } else {
      y[j][0] = y[j][1] = 0.0;
    }
  }
  fold_finish<2, MAXSLOT, HB, ROWS, ROW_LDS>(y, pval, pbase, R, L, ndata, T, lane, qi, qi_ld, col, dc);
}

// One wavefront per segment (grid-stride over 4-wave workgroups that share one LDS
// copy of the basis); each wave's L bins follow the basis in LDS. LOADS 1-KB chunk
// loads per lane in flight (non-temporal: the input is read once). ROWS selects the
// output layout (fold_finish). PFN > 0 (and R >= 128·PFN): the next segment's first
// PFN chunks are in flight during a segment's contraction (bins_segment).
// probe (diagnostics, may be null): s_memrealtime at the entry of workgroups 0 and
// gridDim-1 and at the exit of workgroup 0's wave 0 ([3], [4], [5]).
constexpr int kProbeWaves = 16384;  // per-wave slots of the diagnostics probe buffer
template <int MAXSLOT, int LOADS, bool ROWS, int PFN = 0>
__device__ __forceinline__ void bins_kernel_body(
    const double* __restrict__ x, int64_t nseg, int64_t seg_stride, int R, int L, int ndata,
    const double* __restrict__ tab, double* __restrict__ qi, int64_t qi_ld, double* __restrict__ dc,
    uint64_t* __restrict__ probe, int block0 = 0) {
  // block0: leading workgroups that play another role (the fused seed kernel, seed.h)
  const int bid = (int)blockIdx.x - block0;
  if (probe && threadIdx.x == 0) {
    if (bid == 0) probe[3] = __builtin_amdgcn_s_memrealtime();
    if ((int)blockIdx.x == (int)gridDim.x - 1) probe[4] = __builtin_amdgcn_s_memrealtime();
  }
  const int nwork = (int)gridDim.x - block0;
  if (bid < 0) return;
  extern __shared__ __attribute__((aligned(16))) double lds_dyn[];
  const int ntab = 2 * ndata * L;
  stage_table(tab, lds_dyn, ntab, threadIdx.x, kBlockThreads);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double* __restrict__ ybin = lds_dyn + ntab + wave * L;  // this wave's L phase bins
  const int nslot = (L + 127) / 128;
  int pbase[MAXSLOT];
  bool pval[MAXSLOT];
#pragma unroll
  for (int j = 0; j < MAXSLOT; ++j) {
    pbase[j] = 2 * (lane + 64 * j);
    pval[j] = (j < nslot) && (pbase[j] < L);
  }
  const int64_t s0 = (int64_t)bid * kWavesPerBlock + wave, ds = (int64_t)nwork * kWavesPerBlock;
  if (PFN > 0 && (R >> 7) >= PFN) {
    // software pipeline across this wave's segments (see bins_segment PFN)
    double pf[PFN > 0 ? PFN : 1][2];
    if (s0 < nseg) {
      const double* __restrict__ x0 = x + s0 * seg_stride + 2 * lane;
#pragma unroll
      for (int u = 0; u < PFN; ++u) VecT<2>::load_nt(x0 + u * 128, pf[u]);
    }
    for (int64_t s = s0; s < nseg; s += ds)
      bins_segment<MAXSLOT, LOADS, true, kHarmBlock, ROWS, PFN>(x + s * seg_stride, R, L, ndata, lds_dyn, ybin, lane,
                                                                pval, pbase, qi, qi_ld, s, dc, pf,
                                                                s + ds < nseg ? x + (s + ds) * seg_stride : nullptr);
  } else {
    for (int64_t s = s0; s < nseg; s += ds)
      bins_segment<MAXSLOT, LOADS, true, kHarmBlock, ROWS>(x + s * seg_stride, R, L, ndata, lds_dyn, ybin, lane, pval,
                                                           pbase, qi, qi_ld, s, dc);
  }
  if (probe && threadIdx.x == 0 && bid == 0) probe[5] = __builtin_amdgcn_s_memrealtime();
  // per-wave exit times (probe[16 + global wave], up to kProbeWaves waves) and the
  // hardware XCC of the wave ([16 + kProbeWaves + wave])
  if (probe && lane == 0) {
    const int64_t gw = (int64_t)bid * kWavesPerBlock + wave;
    if (gw < kProbeWaves) {
      probe[16 + gw] = __builtin_amdgcn_s_memrealtime();
      unsigned xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      probe[16 + kProbeWaves + gw] = (uint64_t)(xcc & 0xf);
    }
  }
}

template <int MAXSLOT, int LOADS, bool ROWS, int PFN = 0>
__global__ __launch_bounds__(kBlockThreads) void demod_bins_kernel(
    const double* __restrict__ x, int64_t nseg, int64_t seg_stride, int R, int L, int ndata,
    const double* __restrict__ tab, double* __restrict__ qi, int64_t qi_ld, double* __restrict__ dc,
    uint64_t* __restrict__ probe) {
  bins_kernel_body<MAXSLOT, LOADS, ROWS, PFN>(x, nseg, seg_stride, R, L, ndata, tab, qi, qi_ld, dc, probe);
}

// Many harmonics (the bin kernel's LDS basis, 2·ndata·L doubles, no longer fits beside the
// bins: ndata > 16 at L = 200). The fold is the bin kernel's (bins in LDS, flat 1-KB wave
// loads); each wave folds KSEG consecutive segments into KSEG bin sets and then contracts
// them together, with the lanes over the OUTPUTS instead of over the bins: lane l accumulates
// outputs o = l + 64·i (i < NO) of [Q_1..Q_nd, I_1..I_nd, dc] (2·ndata + 1), with no cross-lane
// reduction (the bin kernel's butterfly costs 17 shuffles per 16 sums).
// Half-period symmetry: with L·w0 = 2π·k, cos(h w0 (L-p)) = cos(h w0 p) and sin(h w0 (L-p)) =
// -sin(h w0 p), so each segment's bins are first paired in place, y+[p] = y[p] + y[L-p] and
// y-[p] = y[p] - y[L-p] for 0 < p < L/2 (y±[0] = y[0], y±[L/2] = y[L/2]), and the cos / dc
// lanes contract y+ and the sin lanes y- over p = 0..L/2 only: half the LDS reads and FMAs.
// The basis values at L-p are taken equal to those at p: the host's cos / sin of the
// reference's angles fl(fl(h w0) p) differ from them by the angle rounding, ~h·L·w0·eps
// (4e-14 at h = 62, L = 200), inside the periodicity error the fold itself accepts
// (dfmi_detect_period: 1e-11 rad over the record); so QI agree with the bin / fold kernels to
// ~1e-14 relative, not bit for bit (tests/test_gpu_demod_wide.py).
// Basis: tabT[pp·64·NO + o] = (T[o][2pp], T[o][2pp+1]) for p <= L/2 (zero beyond), o over
// [cos rows | sin rows | ones | zeros], global (L2-resident: 51 KB at ndata 62), TD pairs
// in flight.
// Work: workgroup b owns segments [b·4·KSEG, +4·KSEG), its wave w the KSEG from b·4·KSEG +
// w·KSEG (one group per wave: the dispatcher balances the tail). The waves' results meet in
// LDS and the workgroup stores each output row's 4·KSEG consecutive segments as one run
// (8-B stores one line per lane cost 0.09 ms of 0.65 at ndata 30, r05s).
// Preconditions (host-checked): 16-B aligned rows, L even, 128 <= L <= 256, 2·ndata + 1 <=
// 64·NO; dynamic LDS 4·KSEG·wide_set(L, NO, KSEG) doubles.
__host__ __device__ constexpr int wide_set(int L, int NO, int KSEG) {
  // per-set doubles: the bins (L) + 4 for the paired layout (ym + 2·npair <= L + 4), or this wave's share of the
  // result tile (64·NO rows x (KSEG + 1) pitch), whichever is larger
  // (even: the sets' pair loads / stores stay 16-B aligned)
  return (((L + 4 > (64 * NO * (KSEG + 1) + KSEG - 1) / KSEG) ? L + 4 : (64 * NO * (KSEG + 1) + KSEG - 1) / KSEG) + 1) & ~1;
}
template <int LOADS, int PFN>
__device__ __forceinline__ void wide_fold(const double* __restrict__ xs0, int R, int L, double* ybin, int lane,
                                          double (*pf)[2], const double* __restrict__ next) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  const int nch = R >> 7;
  const int tail = R - (nch << 7);
  auto add_chunk = [&](int p0, const double (&v)[2]) {
    int p = p0 + 2 * lane;
    if (p >= L) p -= L;
    d2v* yp = reinterpret_cast<d2v*>(ybin + p);
    d2v t = *yp;
    t.x += v[0];
    t.y += v[1];
    *yp = t;
  };
#pragma unroll
  for (int j = 0; j < 2; ++j)
    if (2 * (lane + 64 * j) < L) *reinterpret_cast<d2v*>(ybin + 2 * (lane + 64 * j)) = d2v{0.0, 0.0};
  const double* __restrict__ xs = xs0 + 2 * lane;
  int p0 = 0;
  int c = 0;
  if constexpr (PFN > 0) {
#pragma unroll
    for (int u = 0; u < PFN; ++u) {
      add_chunk(p0, pf[u]);
      p0 += 128;
      if (p0 >= L) p0 -= L;
    }
    c = PFN;
  }
  for (; c + LOADS <= nch; c += LOADS) {
    double v[LOADS][2];
#pragma unroll
    for (int u = 0; u < LOADS; ++u) VecT<2>::load_nt(xs + (c + u) * 128, v[u]);
#pragma unroll
    for (int u = 0; u < LOADS; ++u) {
      add_chunk(p0, v[u]);
      p0 += 128;
      if (p0 >= L) p0 -= L;
    }
  }
  {
    const int rem = nch - c;
    double v[LOADS][2];
#pragma unroll
    for (int u = 0; u < LOADS; ++u)
      if (u < rem) VecT<2>::load_nt(xs + (c + u) * 128, v[u]);
    const int t0 = 2 * lane;
    double tv0 = 0.0, tv1 = 0.0;
    if (t0 < tail) tv0 = xs[nch * 128];
    if (t0 + 1 < tail) tv1 = xs[nch * 128 + 1];
#pragma unroll
    for (int u = 0; u < LOADS; ++u) {
      if (u < rem) {
        add_chunk(p0, v[u]);
        p0 += 128;
        if (p0 >= L) p0 -= L;
      }
    }
    if (tail) {
      int p = p0 + t0;
      if (p >= L) p -= L;
      if (t0 < tail) ybin[p] += tv0;
      if (t0 + 1 < tail) ybin[p + 1] += tv1;
    }
  }
  if constexpr (PFN > 0) {
    if (next) {
      const double* __restrict__ xn = next + 2 * lane;
#pragma unroll
      for (int u = 0; u < PFN; ++u) VecT<2>::load_nt(xn + u * 128, pf[u]);
    }
  }
}

// The fold of a workgroup-wave's nk CONTIGUOUS segments (seg_stride == R) as one flat stream of
// nk·R samples: 1-KB chunk loads, LOADS in flight, with no restart at segment boundaries (a
// short segment, R = 200, is otherwise one exposed memory round trip of 1.6 KB: 0.1 of peak,
// r05ad). Lane l's two samples of a chunk sit in one segment (R even), at position t, bin p;
// (k, t, p) advance by 128 samples a chunk (p -= R mod L at each segment wrap).
template <int LOADS>
__device__ __forceinline__ void wide_fold_flat(const double* __restrict__ xg, int nk, int R, int L, double* ybase,
                                               int ws, int lane) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  for (int k = 0; k < nk; ++k)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (2 * (lane + 64 * j) < L) *reinterpret_cast<d2v*>(ybase + k * ws + 2 * (lane + 64 * j)) = d2v{0.0, 0.0};
  const int64_t total = (int64_t)nk * R;
  const int64_t nch = total >> 7;
  const int tail = (int)(total - (nch << 7));
  const int rL = R % L;
  int k = (2 * lane) / R, t = 2 * lane - k * R, p = t % L;
  auto add = [&](const d2v v) {
    d2v* yp = reinterpret_cast<d2v*>(ybase + k * ws + p);
    d2v y = *yp;
    y.x += v.x;
    y.y += v.y;
    *yp = y;
    t += 128;
    p += 128;
    if (p >= L) p -= L;
    while (t >= R) {
      t -= R;
      ++k;
      p -= rL;
      if (p < 0) p += L;
    }
  };
  const d2v* __restrict__ xv = reinterpret_cast<const d2v*>(xg) + lane;
  int64_t c = 0;
  for (; c + LOADS <= nch; c += LOADS) {
    d2v v[LOADS];
#pragma unroll
    for (int u = 0; u < LOADS; ++u) v[u] = __builtin_nontemporal_load(xv + (c + u) * 64);
#pragma unroll
    for (int u = 0; u < LOADS; ++u) add(v[u]);
  }
  {
    const int rem = (int)(nch - c);
    d2v v[LOADS];
#pragma unroll
    for (int u = 0; u < LOADS; ++u)
      if (u < rem) v[u] = __builtin_nontemporal_load(xv + (c + u) * 64);
    d2v tv = d2v{0.0, 0.0};
    if (2 * lane < tail) tv = xv[nch * 64];  // partial last chunk (tail even: both samples or none)
#pragma unroll
    for (int u = 0; u < LOADS; ++u)
      if (u < rem) add(v[u]);
    if (2 * lane < tail) add(tv);
  }
}

// HALF (NO = 1, 2·ndata + 1 <= 32): the two half-waves contract different segments (lanes
// 0..31 the even k, 32..63 the odd), halving the contraction's instructions per segment.
template <int NO, int KSEG, int LOADS, int PFN, int HALF = 0, int TD = (NO >= 4 ? 2 : 8 / NO)>
__global__ __launch_bounds__(kBlockThreads, 3) void demod_wide_kernel(  // 3 waves per SIMD: <= 168 VGPRs
    const double* __restrict__ x, int64_t nseg, int64_t seg_stride, int R, int L, int ndata,
    const double* __restrict__ tabT, double* __restrict__ qi, int64_t qi_ld, double* __restrict__ dc, int dbg) {
  // dbg (diagnostics, demod_wide_dbg): bit 0 skips the contraction (acc = one bin), bit 1
  // the stores (kept alive by a never-true NaN test) — fold / contraction / store split;
  // bit 2 folds contiguous segments one by one (the strided-record path) instead of flat
  typedef double d2v __attribute__((ext_vector_type(2)));
  extern __shared__ __attribute__((aligned(16))) double lds_dyn[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ws = wide_set(L, NO, KSEG);
  double* ybase = lds_dyn + (size_t)wave * KSEG * ws;  // this wave's KSEG bin sets
  const int64_t b0 = (int64_t)blockIdx.x * kWavesPerBlock * KSEG;
  const int64_t sbeg = b0 + (int64_t)wave * KSEG;
  const int64_t send = sbeg + KSEG < nseg ? sbeg + KSEG : nseg;
  const int nk = sbeg < send ? (int)(send - sbeg) : 0;
  const int nout = 2 * ndata + 1;
  const int half = L >> 1;
  const int npair = (half + 2) >> 1;  // basis pairs covering p = 0..half
  const int ym = (half + 2) & ~1;     // start of y- in a set
  const bool pfok = PFN > 0 && (R >> 7) >= PFN;
  double pf[PFN > 0 ? PFN : 1][2];
  if (pfok && nk > 0 && !(seg_stride == R && !(dbg & 4))) {
    const double* __restrict__ x0 = x + sbeg * seg_stride + 2 * lane;
#pragma unroll
    for (int u = 0; u < (PFN > 0 ? PFN : 1); ++u) VecT<2>::load_nt(x0 + u * 128, pf[u]);
  }
  const bool flat = seg_stride == R && !(dbg & 4);  // contiguous segments: one flat stream per wave
  if (flat && nk > 0) wide_fold_flat<LOADS>(x + sbeg * seg_stride, nk, R, L, ybase, ws, lane);
  for (int k = 0; k < nk; ++k) {
    const int64_t s = sbeg + k;
    double* yb = ybase + k * ws;
    const double* nx = s + 1 < send ? x + (s + 1) * seg_stride : nullptr;
    if (flat) {
    } else if (pfok) {
      wide_fold<LOADS, PFN>(x + s * seg_stride, R, L, yb, lane, pf, nx);
    } else {
      wide_fold<LOADS, 0>(x + s * seg_stride, R, L, yb, lane, pf, nullptr);
    }
    // pair the bins in place: y+ at [0, 2 npp), y- at [ym, ym + 2 npp) (ym even: 16-B aligned
    // pair reads), zero past half; every lane reads all its inputs before any lane writes
    // (one wave: its LDS operations execute in order)
    double a[3], bb[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int p = lane + 64 * u;
      a[u] = p <= half ? yb[p] : 0.0;
      bb[u] = (p > 0 && p < half) ? yb[L - p] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int p = lane + 64 * u;
      if (p < 2 * npair) {
        const bool self = p == 0 || p == half;
        yb[p] = self ? a[u] : a[u] + bb[u];
        yb[ym + p] = self ? a[u] : a[u] - bb[u];
      }
    }
  }
  static_assert(!HALF || (NO == 1 && KSEG % 2 == 0), "half-wave contraction: one output slice, even KSEG");
  constexpr int KH = HALF ? KSEG / 2 : KSEG;  // segments contracted per lane
  const int grp = HALF ? lane >> 5 : 0;       // half-wave: which segments (k = 2 j + grp)
  const int ol = HALF ? lane & 31 : lane;     // output lane
  double acc[KH][NO];
#pragma unroll
  for (int j = 0; j < KH; ++j)
#pragma unroll
    for (int i = 0; i < NO; ++i) acc[j][i] = 0.0;
  // lanes of sin rows read y-, the others y+ (two addresses per lane group: no conflict)
  int yoff[NO];
#pragma unroll
  for (int i = 0; i < NO; ++i) {
    const int o = ol + 64 * i;
    yoff[i] = (o >= ndata && o < 2 * ndata) ? ym : 0;
  }
  const int npp = (dbg & 1) || nk == 0 ? 0 : npair;
  if (dbg & 1)
#pragma unroll
    for (int j = 0; j < KH; ++j) acc[j][0] = ybase[(HALF ? 2 * j + grp : j) * ws + lane];
  const d2v* __restrict__ T2 = reinterpret_cast<const d2v*>(tabT);
  d2v tb[TD][NO];
#pragma unroll
  for (int u = 0; u < TD; ++u)
#pragma unroll
    for (int i = 0; i < NO; ++i)
      if (u < npp) tb[u][i] = T2[(size_t)u * 64 * NO + ol + 64 * i];
  for (int pp0 = 0; pp0 < npp; pp0 += TD) {
#pragma unroll
    for (int u = 0; u < TD; ++u) {
      const int pp = pp0 + u;
      if (pp < npp) {
        d2v t[NO];
#pragma unroll
        for (int i = 0; i < NO; ++i) {
          t[i] = tb[u][i];
          if (pp + TD < npp) tb[u][i] = T2[(size_t)(pp + TD) * 64 * NO + ol + 64 * i];
        }
#pragma unroll
        for (int j = 0; j < KH; ++j) {
          const int k = HALF ? 2 * j + grp : j;
#pragma unroll
          for (int i = 0; i < NO; ++i) {
            const d2v y = *reinterpret_cast<const d2v*>(ybase + k * ws + yoff[i] + 2 * pp);
            acc[j][i] = fma(y.x, t[i].x, acc[j][i]);
            acc[j][i] = fma(y.y, t[i].y, acc[j][i]);
          }
        }
      }
    }
  }
  // results to LDS (this wave's share of the tile: [o][KSEG + 1] in its own sets), then the
  // workgroup writes each output row's 4·KSEG consecutive segments as one run. The stores
  // are what this kernel pays beyond its fold (0.463 ms at config 2): +0.087 ms at ndata 30
  // for 48.8 MB (TCC_EA0_WRREQ_64B: exactly the bytes), the same for a segment-major order
  // (one contiguous run per workgroup), with plain stores, or with XCD-contiguous ranges,
  // and +0.008 ms for one store per wave — the write bytes themselves, in a saturated read
  // stream (profiles/r05/wide_demod_ab.jsonl)
  constexpr int KP = KSEG + 1;
#pragma unroll
  for (int j = 0; j < KH; ++j)
#pragma unroll
    for (int i = 0; i < NO; ++i)  // mean: sum / count
      ybase[(ol + 64 * i) * KP + (HALF ? 2 * j + grp : j)] = acc[j][i] / (double)R;
  __syncthreads();
  constexpr int SEGS = kWavesPerBlock * KSEG;  // consecutive segments per output row
  for (int e = threadIdx.x; e < nout * SEGS; e += kBlockThreads) {
    const int o = e / SEGS, c = e - o * SEGS;
    const int64_t s = b0 + c;
    if (s < nseg) {
      const double v = lds_dyn[(size_t)(c / KSEG) * KSEG * ws + o * KP + (c % KSEG)];
      if ((dbg & 2) && v == v) continue;
      __builtin_nontemporal_store(v, o < nout - 1 ? qi + (int64_t)o * qi_ld + s : dc + s);
    }
  }
}

// One segment the many-harmonic way, by one wave (the seed step beyond the bin kernel's LDS
// basis, seed.h seed_kernel): wide_fold into the wave's LDS bins (ybin, L + 4 doubles), the
// half-period pairing and the lanes-over-outputs contraction of demod_wide_kernel, the same
// operations in the same order — the segment's QI and dc are bit-identical to what the bulk
// demod_wide_kernel gives it; written component-major to qi[o * qi_ld + col] / dc[col].
__device__ __forceinline__ void wide_seed_segment(const double* __restrict__ xs, int R, int L, int ndata,
                                                  const double* __restrict__ tabT, int no, double* ybin, int lane,
                                                  double* __restrict__ qi, int64_t qi_ld, int64_t col,
                                                  double* __restrict__ dc) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  double pf[1][2];
  wide_fold<10, 0>(xs, R, L, ybin, lane, pf, nullptr);
  const int half = L >> 1;
  const int npair = (half + 2) >> 1;
  const int ym = (half + 2) & ~1;
  double a[3], bb[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int p = lane + 64 * u;
    a[u] = p <= half ? ybin[p] : 0.0;
    bb[u] = (p > 0 && p < half) ? ybin[L - p] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int p = lane + 64 * u;
    if (p < 2 * npair) {
      const bool self = p == 0 || p == half;
      ybin[p] = self ? a[u] : a[u] + bb[u];
      ybin[ym + p] = self ? a[u] : a[u] - bb[u];
    }
  }
  const d2v* __restrict__ T2 = reinterpret_cast<const d2v*>(tabT);
  const int nout = 2 * ndata + 1;
  for (int i = 0; i < no; ++i) {
    const int o = lane + 64 * i;
    const int yoff = (o >= ndata && o < 2 * ndata) ? ym : 0;
    double acc = 0.0;
    for (int pp = 0; pp < npair; ++pp) {
      const d2v t = T2[(size_t)pp * 64 * no + o];
      const d2v y = *reinterpret_cast<const d2v*>(ybin + yoff + 2 * pp);
      acc = fma(y.x, t.x, acc);
      acc = fma(y.y, t.y, acc);
    }
    const double v = acc / (double)R;
    if (o < nout - 1) qi[(int64_t)o * qi_ld + col] = v;
    else if (o == nout - 1) dc[col] = v;
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
    butterfly<16>(acc, lane);
    store_block<kHarmBlock>(acc, lane, hb, ndata, qi, qi_ld, col, R);
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

// readbw.hip — read-bandwidth microbenchmark of the access patterns the demod
// kernel can use (measurement tool, not product code). 3.2 GB of fp64 is read
// once per launch; every kernel reduces what it reads so nothing is elided.
//   contig   : grid-stride 16-B loads over the whole buffer (torch-sum-like)
//   segwave  : one wavefront per 4000-double segment (the demod mapping)
//   segblock : one 4-wave workgroup per segment (waves interleave 1-KB chunks)
//   glds     : one wavefront per segment, 1-KB chunks by LDS-DMA into a per-wave ring
// Build: hipcc --offload-arch=gfx950 -O3 -o readbw scripts/readbw.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#include "../deepfmkit_amd/csrc/demod.h"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ d2v ld2(const double* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
  else return *reinterpret_cast<const d2v*>(p);
}

template <int LOADS, bool NT>
__global__ __launch_bounds__(256) void contig(const double* __restrict__ x, int64_t n2, double* out) {
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t T = (int64_t)gridDim.x * 256;
  double s = 0.0;
  int64_t i = tid;
  for (; i + (LOADS - 1) * T < n2; i += LOADS * T) {
    d2v v[LOADS];
#pragma unroll
    for (int u = 0; u < LOADS; ++u) v[u] = ld2<NT>(x + 2 * (i + u * T));
#pragma unroll
    for (int u = 0; u < LOADS; ++u) s += v[u].x + v[u].y;
  }
  for (; i < n2; i += T) {
    d2v v = ld2<NT>(x + 2 * i);
    s += v.x + v.y;
  }
  out[tid] = s;
}

// S doubles per segment; chunk = 128 doubles (1 KB per wave instruction)
template <int LOADS, bool NT>
__global__ __launch_bounds__(256) void segwave(const double* __restrict__ x, int64_t nseg, int S, double* out) {
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t W = (int64_t)gridDim.x * 4;
  double s = 0.0;
  const int nch = S / 128;  // full chunks
  for (int64_t seg = gw; seg < nseg; seg += W) {
    const double* xs = x + seg * S + 2 * lane;
    int c = 0;
    for (; c + LOADS <= nch; c += LOADS) {
      d2v v[LOADS];
#pragma unroll
      for (int u = 0; u < LOADS; ++u) v[u] = ld2<NT>(xs + (c + u) * 128);
#pragma unroll
      for (int u = 0; u < LOADS; ++u) s += v[u].x + v[u].y;
    }
    for (; c < nch; ++c) {
      d2v v = ld2<NT>(xs + c * 128);
      s += v.x + v.y;
    }
    const int tail = S - nch * 128;
    if (2 * lane < tail) {
      d2v v = ld2<NT>(xs + nch * 128);
      s += v.x + v.y;
    }
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

template <int LOADS, bool NT>
__global__ __launch_bounds__(256) void segblock(const double* __restrict__ x, int64_t nseg, int S, double* out) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double s = 0.0;
  const int nch = S / 128;
  for (int64_t seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    const double* xs = x + seg * S + 2 * lane;
    int c = wave;
    for (; c + 4 * (LOADS - 1) < nch; c += 4 * LOADS) {
      d2v v[LOADS];
#pragma unroll
      for (int u = 0; u < LOADS; ++u) v[u] = ld2<NT>(xs + (c + 4 * u) * 128);
#pragma unroll
      for (int u = 0; u < LOADS; ++u) s += v[u].x + v[u].y;
    }
    for (; c < nch; c += 4) {
      d2v v = ld2<NT>(xs + c * 128);
      s += v.x + v.y;
    }
    const int tail = S - nch * 128;
    if (wave == 0 && 2 * lane < tail) {
      d2v v = ld2<NT>(xs + nch * 128);
      s += v.x + v.y;
    }
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// LDS-DMA ring: D slots of 1 KB per wave; chunk c lands in slot c % D.
template <int D, int AUX>
__global__ __launch_bounds__(256) void glds(const double* __restrict__ x, int64_t nseg, int S, double* out) {
  __shared__ __attribute__((aligned(16))) double ring[4][D][128];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  const int64_t W = (int64_t)gridDim.x * 4;
  double s = 0.0;
  const int nch = S / 128;  // full chunks only (tail read directly)
  for (int64_t seg = gw; seg < nseg; seg += W) {
    const double* xs = x + seg * S;
#pragma unroll
    for (int c = 0; c < D; ++c)
      __builtin_amdgcn_global_load_lds((const void*)(xs + c * 128 + 2 * lane), (void*)&ring[wave][c][0], 16, 0, AUX);
    for (int c = 0; c < nch; ++c) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
      const int slot = c % D;
      const d2v v = *reinterpret_cast<const d2v*>(&ring[wave][slot][2 * lane]);
      s += v.x + v.y;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int cn = c + D < nch ? c + D : c;  // keep the count: re-read the same chunk at the end
      __builtin_amdgcn_global_load_lds((const void*)(xs + cn * 128 + 2 * lane), (void*)&ring[wave][slot][0], 16, 0,
                                       AUX);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int tail = S - nch * 128;
    if (2 * lane < tail) {
      d2v v = ld2<true>(xs + nch * 128 + 2 * lane);
      s += v.x + v.y;
    }
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// segwave + the bins kernel's per-chunk LDS read-modify-write (no contraction)
template <int LOADS>
__global__ __launch_bounds__(256) void segwave_rmw(const double* __restrict__ x, int64_t nseg, int S, double* out) {
  __shared__ __attribute__((aligned(16))) double bins[4][200];
  const int L = 200;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  const int64_t W = (int64_t)gridDim.x * 4;
  double* yb = bins[wave];
  double s = 0.0;
  const int nch = S / 128;
  for (int64_t seg = gw; seg < nseg; seg += W) {
    const double* xs = x + seg * S + 2 * lane;
    int p0 = 0;
    for (int c = 0; c + LOADS <= nch; c += LOADS) {
      d2v v[LOADS];
#pragma unroll
      for (int u = 0; u < LOADS; ++u) v[u] = ld2<true>(xs + (c + u) * 128);
#pragma unroll
      for (int u = 0; u < LOADS; ++u) {
        int p = p0 + 2 * lane;
        if (p >= L) p -= L;
        d2v* yp = reinterpret_cast<d2v*>(yb + p);
        d2v t = *yp;
        t += v[u];
        *yp = t;
        p0 += 128;
        if (p0 >= L) p0 -= L;
      }
    }
    for (int c = (nch / LOADS) * LOADS; c < nch; ++c) {
      const d2v v = ld2<true>(xs + c * 128);
      int p = p0 + 2 * lane;
      if (p >= L) p -= L;
      d2v* yp = reinterpret_cast<d2v*>(yb + p);
      d2v t = *yp;
      t += v;
      *yp = t;
      p0 += 128;
      if (p0 >= L) p0 -= L;
    }
    const d2v t = *reinterpret_cast<const d2v*>(yb + (2 * lane) % L);
    s += t.x + t.y;
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// segwave + the demod contraction (fold_finish on register bins, basis in LDS), no RMW
// STORE: 0 = QI component-major (the demod layout), 1 = no stores (sums folded into
// one value per wave), 2 = segment-major (each segment's 21 values contiguous)
template <int LOADS, int HB, int STORE>
__global__ __launch_bounds__(256) void segwave_con(const double* __restrict__ x, int64_t nseg, int S,
                                                   const double* __restrict__ tab, double* qi, double* dcv) {
  __shared__ __attribute__((aligned(16))) double T[20 * 200];
  const int L = 200, ndata = 10;
  for (int i = threadIdx.x; i < 20 * L; i += 256) T[i] = tab[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t W = (int64_t)gridDim.x * 4;
  const int nch = S / 128;
  int pbase[2] = {2 * lane, 2 * (lane + 64)};
  bool pval[2] = {true, 2 * (lane + 64) < L};
  for (int64_t seg = gw; seg < nseg; seg += W) {
    const double* xs = x + seg * S + 2 * lane;
    double y[2][2] = {{0, 0}, {0, 0}};
    for (int c = 0; c + LOADS <= nch; c += LOADS) {
      d2v v[LOADS];
#pragma unroll
      for (int u = 0; u < LOADS; ++u) v[u] = ld2<true>(xs + (c + u) * 128);
#pragma unroll
      for (int u = 0; u < LOADS; ++u) {
        y[u & 1][0] += v[u].x;
        y[u & 1][1] += v[u].y;
      }
    }
    for (int c = (nch / LOADS) * LOADS; c < nch; ++c) {
      const d2v v = ld2<true>(xs + c * 128);
      y[c & 1][0] += v.x;
      y[c & 1][1] += v.y;
    }
    if constexpr (STORE == 0) {
      dfmi::fold_finish<2, 2, HB>(y, pval, pbase, S, L, ndata, T, lane, qi, nseg, seg, dcv);
    } else if constexpr (STORE == 1) {
      double acc[2 * HB] = {};
      for (int hb = 0; hb < 2; ++hb) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int h = 0; h < HB; ++h) {
            const d2v bc = *reinterpret_cast<const d2v*>(T + (hb * HB + h) * L + pbase[j]);
            const d2v bs = *reinterpret_cast<const d2v*>(T + (10 + hb * HB + h) * L + pbase[j]);
            acc[h] = fma(y[j][0], bc.x, fma(y[j][1], bc.y, acc[h]));
            acc[HB + h] = fma(y[j][0], bs.x, fma(y[j][1], bs.y, acc[HB + h]));
          }
        dfmi::butterfly<2 * HB>(acc, lane);
      }
      if (acc[0] == 12345.0) dcv[seg] = acc[0];  // never true: keeps the work, drops the stores
    } else {
      double acc[2 * HB] = {};
      for (int hb = 0; hb < 2; ++hb) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int h = 0; h < HB; ++h) {
            const d2v bc = *reinterpret_cast<const d2v*>(T + (hb * HB + h) * L + pbase[j]);
            const d2v bs = *reinterpret_cast<const d2v*>(T + (10 + hb * HB + h) * L + pbase[j]);
            acc[h] = fma(y[j][0], bc.x, fma(y[j][1], bc.y, acc[h]));
            acc[HB + h] = fma(y[j][0], bs.x, fma(y[j][1], bs.y, acc[HB + h]));
          }
        dfmi::butterfly<2 * HB>(acc, lane);
        constexpr int SH = (HB == 8) ? 2 : 3;
        if ((lane & ((1 << SH) - 1)) == 0) qi[seg * 21 + hb * 2 * HB + (lane >> SH)] = acc[0];
      }
    }
  }
}

int main(int argc, char** argv) {
  const int S = 4000;
  const int64_t nseg = argc > 1 ? atoll(argv[1]) : 100000;
  const int64_t n = nseg * S;
  int ncu = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  ncu = prop.multiProcessorCount;
  double *x, *out;
  CK(hipMalloc(&x, n * 8));
  CK(hipMalloc(&out, (size_t)ncu * 64 * 256 * 8));
  CK(hipMemset(x, 0, n * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 7; ++r) {
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < 5; ++k) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms / 5);
    }
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, med, n * 8.0 / med / 1e6);
    fflush(stdout);
  };
  char nm[128];
  for (int occ : {8}) {
    snprintf(nm, sizeof nm, "contig_l8_nt_g%d", occ);
    run(nm, [&] { contig<8, true><<<ncu * occ, 256>>>(x, n / 2, out); });
    snprintf(nm, sizeof nm, "contig_l8_g%d", occ);
    run(nm, [&] { contig<8, false><<<ncu * occ, 256>>>(x, n / 2, out); });
  }
  for (int occ : {4}) {
    snprintf(nm, sizeof nm, "segwave_l8_nt_g%d", occ);
    run(nm, [&] { segwave<8, true><<<ncu * occ, 256>>>(x, nseg, S, out); });
    snprintf(nm, sizeof nm, "segwave_l16_nt_g%d", occ);
    run(nm, [&] { segwave<16, true><<<ncu * occ, 256>>>(x, nseg, S, out); });
    snprintf(nm, sizeof nm, "segwave_l8_g%d", occ);
    run(nm, [&] { segwave<8, false><<<ncu * occ, 256>>>(x, nseg, S, out); });
    snprintf(nm, sizeof nm, "segblock_l4_nt_g%d", occ);
    run(nm, [&] { segblock<4, true><<<ncu * occ, 256>>>(x, nseg, S, out); });
    snprintf(nm, sizeof nm, "segblock_l8_nt_g%d", occ);
    run(nm, [&] { segblock<8, true><<<ncu * occ, 256>>>(x, nseg, S, out); });
    snprintf(nm, sizeof nm, "glds_d8_nt_g%d", occ);
    run(nm, [&] { glds<8, 2><<<ncu * occ, 256>>>(x, nseg, S, out); });
    snprintf(nm, sizeof nm, "glds_d8_g%d", occ);
    run(nm, [&] { glds<8, 0><<<ncu * occ, 256>>>(x, nseg, S, out); });
    snprintf(nm, sizeof nm, "glds_d16_nt_g%d", occ);
    run(nm, [&] { glds<16, 2><<<ncu * occ, 256>>>(x, nseg, S, out); });
  }
  double *tab, *qi, *dcv;
  CK(hipMalloc(&tab, 20 * 200 * 8));
  CK(hipMemset(tab, 0, 20 * 200 * 8));
  CK(hipMalloc(&qi, (size_t)nseg * 21 * 8));
  CK(hipMalloc(&dcv, (size_t)nseg * 8));
  for (int occ : {4}) {
    snprintf(nm, sizeof nm, "segwave_rmw_l8_g%d", occ);
    run(nm, [&] { segwave_rmw<8><<<ncu * occ, 256>>>(x, nseg, S, out); });
    snprintf(nm, sizeof nm, "segwave_con_hb8_l8_g%d", occ);
    run(nm, [&] { segwave_con<8, 8, 0><<<ncu * occ, 256>>>(x, nseg, S, tab, qi, dcv); });
    snprintf(nm, sizeof nm, "segwave_con_hb4_l8_g%d", occ);
    run(nm, [&] { segwave_con<8, 4, 0><<<ncu * occ, 256>>>(x, nseg, S, tab, qi, dcv); });
    snprintf(nm, sizeof nm, "segwave_con_nostore_hb8_l8_g%d", occ);
    run(nm, [&] { segwave_con<8, 8, 1><<<ncu * occ, 256>>>(x, nseg, S, tab, qi, dcv); });
    snprintf(nm, sizeof nm, "segwave_con_segmajor_hb8_l8_g%d", occ);
    run(nm, [&] { segwave_con<8, 8, 2><<<ncu * occ, 256>>>(x, nseg, S, tab, qi, dcv); });
    snprintf(nm, sizeof nm, "segwave_l8_nt_g%d(again)", occ);
    run(nm, [&] { segwave<8, true><<<ncu * occ, 256>>>(x, nseg, S, out); });
  }
  CK(hipFree(x));
  CK(hipFree(out));
  return 0;
}

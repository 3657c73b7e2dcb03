// synth.hip — dfmi_synth_asd's kernel: ONE WAVE PER TRIAL runs synth.h's generator.
//
//   seeding      lane 0 (624 serial multiply-xors), state in LDS
//   twist        the 624-word MT19937 twist in three parallel phases: words
//                [0, 227) read only old words, [227, 454) and [454, 623) the new words
//                227 below them, word 623 the new words 0 and 396
//   gaussians    the polar method's candidates, 156 per twisted block (4 words each),
//                64 at a time across the lanes; a ballot + prefix count gives every
//                accepted candidate its place in numpy's output order (f*x2, then the
//                cached f*x1), so the stream is exactly RandomState's
//   physics      max|g|, the cumsum summands and the signal in parallel over samples;
//                the cumsum itself (numpy's order: one running sum) by lane 0
// Scratch per trial (global, contiguous): 2n + 2 gaussians, n phi_mod values.
// Built without FMA contraction (synth.h also pins it per function).
#include <hip/hip_runtime.h>

#include "synth.h"

namespace dfmi {
namespace {

constexpr int kLanes = 64;
constexpr int kWordsPerLane = (kMtN + kLanes - 1) / kLanes;  // 10
constexpr int kCandidates = kMtN / 4;                        // 156 per twisted block

struct GVec {
  const double* p;
  __device__ __forceinline__ double operator()(int64_t k) const { return p[k]; }
};

__global__ __launch_bounds__(kLanes) void synth_wave_kernel(const dfmi_synth_trial* __restrict__ trials, int64_t n,
                                                             double f_samp, double* scratch, double* out) {
#pragma clang fp contract(off)
  __shared__ uint32_t mt[kMtN];
  const int64_t r = blockIdx.x;
  const int lane = threadIdx.x;
  const dfmi_synth_trial p = trials[r];
  double* gauss = scratch + r * (3 * n + 2);
  double* phi = gauss + 2 * n + 2;
  const bool amp_on = p.s_amp != 0.0, df_on = p.s_df != 0.0;
  const int64_t need = (amp_on ? n : 0) + (df_on ? n : 0);

  // numpy mt19937_seed
  if (lane == 0) {
    uint32_t s = p.seed;
    for (int i = 0; i < kMtN; ++i) {
      mt[i] = s;
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
    }
  }
  __syncthreads();

  int64_t have = 0;
  while (have < need) {
    // twist: old operands into registers first, then the three phases
    uint32_t o0[kWordsPerLane], o1[kWordsPerLane];
#pragma unroll
    for (int j = 0; j < kWordsPerLane; ++j) {
      const int i = lane + kLanes * j;
      o0[j] = i < kMtN ? mt[i] : 0u;
      o1[j] = i < kMtN - 1 ? mt[i + 1] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kWordsPerLane; ++j) {
      const int i = lane + kLanes * j;
      if (i < kMtN - kMtM) mt[i] = mt_twist_word(o0[j], o1[j], mt[i + kMtM]);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kWordsPerLane; ++j) {
      const int i = lane + kLanes * j;
      if (i >= kMtN - kMtM && i < 2 * (kMtN - kMtM)) mt[i] = mt_twist_word(o0[j], o1[j], mt[i + (kMtM - kMtN)]);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kWordsPerLane; ++j) {
      const int i = lane + kLanes * j;
      if (i >= 2 * (kMtN - kMtM) && i < kMtN - 1) mt[i] = mt_twist_word(o0[j], o1[j], mt[i + (kMtM - kMtN)]);
    }
    __syncthreads();
    if (lane == (kMtN - 1) % kLanes) mt[kMtN - 1] = mt_twist_word(o0[(kMtN - 1) / kLanes], mt[0], mt[kMtM - 1]);
    __syncthreads();
    // the block's 156 candidates in stream order
    for (int c0 = 0; c0 < kCandidates && have < need; c0 += kLanes) {
      const int c = c0 + lane;
      double x1 = 0.0, x2 = 0.0, r2 = 0.0;
      bool ok = false;
      if (c < kCandidates)
        ok = polar_candidate(mt_temper(mt[4 * c]), mt_temper(mt[4 * c + 1]), mt_temper(mt[4 * c + 2]),
                             mt_temper(mt[4 * c + 3]), &x1, &x2, &r2);
      const uint64_t bal = __ballot(ok);
      const int rank = __popcll(bal & ((1ull << lane) - 1ull));
      const int64_t idx = have + 2 * (int64_t)rank;
      if (ok && idx < need) {
        const double f = polar_scale(r2);
        gauss[idx] = f * x2;
        gauss[idx + 1] = f * x1;
      }
      have += 2 * (int64_t)__popcll(bal);
    }
    __syncthreads();
  }
  const double* n_amp = amp_on ? gauss : nullptr;
  const double* n_df = df_on ? gauss + (amp_on ? n : 0) : nullptr;

  // max |g_t| (exact in any order), every lane gets the result
  double gm = 0.0;
  for (int64_t k = lane; k < n; k += kLanes) gm = synth_gmax_step(gm, fabs(synth_g(p, k, f_samp)));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) gm = synth_gmax_step(gm, __shfl_xor(gm, off));
  // cumsum summands, then the running sum in numpy's order
  for (int64_t k = lane; k < n; k += kLanes)
    phi[k] = synth_v(p, k, f_samp, gm, n_df ? 0.0 + p.s_df * n_df[k] : 0.0);
  __syncthreads();
  if (lane == 0) {
    double acc = 0.0;
    int64_t k = 0;
    for (; k + 8 <= n; k += 8) {
      double v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = phi[k + j];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc = (k + j == 0) ? v[j] : acc + v[j];
        phi[k + j] = p.cphi * acc;
      }
    }
    for (; k < n; ++k) {
      const double v = phi[k];
      acc = k == 0 ? v : acc + v;
      phi[k] = p.cphi * acc;
    }
  }
  __syncthreads();
  const GVec ph{phi};
  double* o = out + r * n;
  for (int64_t k = lane; k < n; k += kLanes)
    o[k] = synth_signal(p, k, n, f_samp, ph, n_amp ? 0.0 + p.s_amp * n_amp[k] : 0.0);
}

}  // namespace

size_t synth_scratch_bytes(int64_t ntrial, int64_t n) { return (size_t)ntrial * (3 * n + 2) * 8; }

hipError_t synth_launch(const dfmi_synth_trial* d_trials, int64_t ntrial, int64_t n, double f_samp, void* scratch,
                        double* out, hipStream_t st) {
  if (ntrial == 0) return hipSuccess;
  hipLaunchKernelGGL(synth_wave_kernel, dim3((unsigned)ntrial), dim3(kLanes), 0, st, d_trials, n, f_samp,
                     (double*)scratch, out);
  return hipGetLastError();
}

}  // namespace dfmi

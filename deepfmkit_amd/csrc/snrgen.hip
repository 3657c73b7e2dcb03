// snrgen.hip — dfmi_synth_snr's kernel: the snr-mode DFMI signal of
// SignalGenerator._generate_with_snr (reference physics.py:475-530,
// ideal signal physics.py:493-518 with is_dynamic=False) for ANY range of sample
// indices of an unbounded record, generated on the device.
//
// Why a counter-based generator: the bench's 8-GPU configuration (BASELINE config
// 4, 10 M segments) shards one long record over ranks; every rank must be able to
// regenerate every segment — in particular buffer 0, whose fit seeds all others
// (fitters.py:403-410) — bit-identically, whatever the world size. So sample i is a
// pure function of (seed, stream, i):
//   noise  Philox4x32-10 (Salmon et al., SC'11) keyed by the 64-bit seed, counter
//          (i >> 1, stream, 0): 4 words -> two 53-bit uniforms u1 in (0, 1], u2 in
//          [0, 1) -> Box-Muller -> the normal pair of samples 2j (cos) and 2j+1 (sin)
//   signal amp * (1 + vis * cos(phi + m * cos(w_mod * t + psi))), t = (i mod P) / f_samp
//          with P = period (samples per modulation cycle; 0 = no wrap), so the phase
//          stays exact for 1e10-sample records instead of rounding w_mod * t at 1e9 rad
// The reference draws its noise from RandomState(trial_num).randn (legacy MT19937);
// that stream cannot be split over ranks, so this generator is a synthetic-input
// substitute of the same distribution (parity of the FITS is checked on the bytes it
// produces, tests/test_gpu_config4.py).
//
// Mapping: one lane per sample PAIR (one Philox call), 16-B stores; grid-stride.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dfmi.h"

namespace dfmi {

struct Philox {
  uint32_t c[4];
};

__device__ __forceinline__ void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += W0;
      k1 += W1;
    }
    const uint64_t p0 = (uint64_t)M0 * c[0];
    const uint64_t p1 = (uint64_t)M1 * c[2];
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
  }
}

// 53 random bits from two words: (a >> 5) * 2^26 + (b >> 6)
__device__ __forceinline__ uint64_t bits53(uint32_t a, uint32_t b) {
  return ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
}

__device__ __forceinline__ double snr_clean(const dfmi_snr_params& p, int64_t i) {
  const int64_t ti = p.period > 0 ? i % (int64_t)p.period : i;
  const double t = (double)ti / p.f_samp;
  const double w = 2.0 * 3.141592653589793 * p.f_mod;
  return p.amp * (1.0 + p.visibility * cos(p.phi + p.m * cos(w * t + p.psi)));
}

__global__ __launch_bounds__(256) void snr_gen_kernel(dfmi_snr_params p, int64_t idx0, int64_t n,
                                                      double* __restrict__ out) {
  // pairs j cover samples [2j, 2j+1]; the output window is [idx0, idx0 + n)
  const int64_t j0 = idx0 >> 1, j1 = (idx0 + n + 1) >> 1;
  const uint32_t k0 = (uint32_t)p.seed, k1 = (uint32_t)(p.seed >> 32);
  for (int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < j1;
       j += (int64_t)gridDim.x * blockDim.x) {
    uint32_t c[4] = {(uint32_t)j, (uint32_t)((uint64_t)j >> 32), p.stream, 0u};
    philox4x32_10(c, k0, k1);
    const double u1 = ((double)bits53(c[0], c[1]) + 1.0) * 0x1.0p-53;  // (0, 1]
    const double u2 = (double)bits53(c[2], c[3]) * 0x1.0p-53;          // [0, 1)
    const double rr = sqrt(-2.0 * log(u1));
    double s, co;
    sincospi(2.0 * u2, &s, &co);
    const int64_t i = 2 * j;
    const double y0 = snr_clean(p, i) + p.noise_std * (rr * co);
    const double y1 = snr_clean(p, i + 1) + p.noise_std * (rr * s);
    const int64_t o = i - idx0;  // position of sample i in out
    if (o >= 0 && o + 1 < n && (((uintptr_t)(out + o)) & 15) == 0) {
      typedef double d2v __attribute__((ext_vector_type(2)));
      *reinterpret_cast<d2v*>(out + o) = d2v{y0, y1};
    } else {
      if (o >= 0 && o < n) out[o] = y0;
      if (o + 1 >= 0 && o + 1 < n) out[o + 1] = y1;
    }
  }
}

hipError_t snr_gen_launch(const dfmi_snr_params& p, int64_t idx0, int64_t n, double* out, int n_cu,
                          hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t pairs = ((idx0 + n + 1) >> 1) - (idx0 >> 1);
  int64_t grid = (pairs + 255) / 256;
  const int64_t cap = (int64_t)n_cu * 32;
  if (grid > cap) grid = cap;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(snr_gen_kernel, dim3((unsigned)grid), dim3(256), 0, st, p, idx0, n, out);
  return hipGetLastError();
}

}  // namespace dfmi

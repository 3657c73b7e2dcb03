// cumask_probe.hip — what hipExtStreamCreateWithCUMask does on this GPU
// (measurement tool). Launches 4096 one-wave workgroups on a default stream and on
// streams whose CU mask excludes bit 0 / keeps only bit 0, and reports the distinct
// (XCC, SE, CU) hardware slots the workgroups ran on (HW_ID / XCC_ID registers).
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/cumask_probe scripts/cumask_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <set>
#include <vector>

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

__global__ void where(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));     // HW_REG_HW_ID (gfx9: id 4)
    unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));   // HW_REG_XCC_ID (id 20), low 16 bits
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    // spin a little so workgroups spread over the machine
    long t0 = clock64();
    while (clock64() - t0 < 20000) {
    }
  }
}

static void report(const char* name, hipStream_t s, unsigned* d, int nblk) {
  CK(hipMemsetAsync(d, 0xff, nblk * 8, s));
  hipLaunchKernelGGL(where, dim3(nblk), dim3(64), 0, s, d);
  CK(hipStreamSynchronize(s));
  std::vector<unsigned> h(2 * nblk);
  CK(hipMemcpy(h.data(), d, nblk * 8, hipMemcpyDeviceToHost));
  std::set<unsigned> cus, xccs;
  for (int b = 0; b < nblk; ++b) {
    const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
    const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
    cus.insert((xcc << 16) | (se << 8) | (sh << 4) | cu);
    xccs.insert(xcc);
  }
  printf("{\"stream\": \"%s\", \"distinct_cus\": %zu, \"distinct_xcc\": %zu}\n", name, cus.size(), xccs.size());
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount, words = (ncu + 31) / 32, nblk = 4096;
  unsigned* d;
  CK(hipMalloc(&d, nblk * 8));
  hipStream_t s0;
  CK(hipStreamCreate(&s0));
  report("default", s0, d, nblk);
  std::vector<uint32_t> all_but0(words, 0xffffffffu), only0(words, 0);
  if (ncu % 32) all_but0[words - 1] = (1u << (ncu % 32)) - 1;
  all_but0[0] &= ~1u;
  only0[0] = 1u;
  hipStream_t sa, sb;
  CK(hipExtStreamCreateWithCUMask(&sa, words, all_but0.data()));
  CK(hipExtStreamCreateWithCUMask(&sb, words, only0.data()));
  std::vector<uint32_t> got(words);
  CK(hipExtStreamGetCUMask(sa, words, got.data()));
  int bits = 0;
  for (auto w : got) bits += __builtin_popcount(w);
  printf("{\"mask_all_but_bit0_bits\": %d, \"ncu\": %d}\n", bits, ncu);
  report("all_but_bit0", sa, d, nblk);
  report("only_bit0", sb, d, nblk);
  return 0;
}

// lm_probe.hip — DIAGNOSTIC build (not part of libdfmi.so): the register-path LM
// (lm.h building blocks: eval_reg_trial / eval_reg_accept / damped_solve_block and
// lm_descend_flat's control flow, restated here with s_memtime stamps) so that the
// cycles of one wave's fit split into solve / trial / accept / other, and passes are
// counted. Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o lm_probe.so lm_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../deepfmkit_amd/csrc/lm.h"

using namespace dfmi;

template <int NDMAX>
__global__ __launch_bounds__(64) void lm_probe_kernel(const double* __restrict__ qi, int64_t ld, int64_t nseg,
                                                      const double* __restrict__ guess, LMConst c,
                                                      double* __restrict__ pout, uint64_t* __restrict__ cyc) {
  const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (s >= nseg) return;
  const QGlobal q{qi + s, ld, 10};
  const int nd = 10;
  double p[4] = {guess[0], guess[1], guess[2], guess[3]};
  uint64_t t_solve = 0, t_trial = 0, t_acc = 0, n_pass = 0, n_acc = 0;
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
  Eval e;
  {
    TrialReg<NDMAX> t0;
    uint64_t a = __builtin_amdgcn_s_memtime();
    eval_reg_trial<NDMAX>(q, nd, p, t0);
    uint64_t b = __builtin_amdgcn_s_memtime();
    eval_reg_accept<NDMAX>(q, nd, p, t0, e);
    uint64_t d = __builtin_amdgcn_s_memtime();
    t_trial += b - a;
    t_acc += d - b;
  }
  int it = 0, li = 0;
  bool active = true;
  while (active) {
    ++n_pass;
    double dp[4];
    uint64_t a = __builtin_amdgcn_s_memtime();
    damped_solve_block(e, c.lambdas[li], dp);
    uint64_t b = __builtin_amdgcn_s_memtime();
    t_solve += b - a;
    bool accepted = false;
    if (!norm_below(sumsq4(dp[0], dp[1], dp[2], dp[3]), c.min_step_norm)) {
      double pt[4] = {p[0] + dp[0], p[1] + dp[1], p[2] + dp[2], p[3] + dp[3]};
      TrialReg<NDMAX> tt;
      uint64_t a2 = __builtin_amdgcn_s_memtime();
      const double ssq_try = eval_reg_trial<NDMAX>(q, nd, pt, tt);
      uint64_t b2 = __builtin_amdgcn_s_memtime();
      t_trial += b2 - a2;
      if (ssq_try < e.ssq) {
        accepted = true;
        const double change2 = sumsq4(pt[0] - p[0], pt[1] - p[1], pt[2] - p[2], pt[3] - p[3]);
        p[0] = pt[0];
        p[1] = pt[1];
        p[2] = pt[2];
        p[3] = pt[3];
        uint64_t a3 = __builtin_amdgcn_s_memtime();
        eval_reg_accept<NDMAX>(q, nd, p, tt, e);
        uint64_t b3 = __builtin_amdgcn_s_memtime();
        t_acc += b3 - a3;
        ++n_acc;
        ++it;
        li = 0;
        if ((norm_below(change2, c.conv_param_change)) || it >= c.max_steps) active = false;
      }
    }
    if (!accepted && ++li >= c.n_lambda) active = false;
  }
  const uint64_t t_end = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 4; ++i) pout[s * 4 + i] = p[i];
  uint64_t* o = cyc + s * 8;
  o[0] = t_end - t_start;
  o[1] = t_solve;
  o[2] = t_trial;
  o[3] = t_acc;
  o[4] = n_pass;
  o[5] = n_acc;
}

extern "C" int lm_probe(const double* qi_host, int64_t nseg, const double* guess_host, double* p_host,
                        uint64_t* cyc_host, int reps, double* ms_out) {
  LMConst c{};
  c.max_steps = 100;
  c.n_lambda = 8;
  const double lam[8] = {0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0};
  for (int i = 0; i < 8; ++i) c.lambdas[i] = lam[i];
  c.min_step_norm = 1e-15;
  c.conv_improve = 1e-9;
  c.conv_param_change = 1e-9;
  c.fitok_threshold = 1e-3;
  double *dq, *dg, *dp;
  uint64_t* dc;
  hipMalloc(&dq, (size_t)nseg * 20 * 8);
  hipMalloc(&dg, 32);
  hipMalloc(&dp, (size_t)nseg * 32);
  hipMalloc(&dc, (size_t)nseg * 64);
  hipMemcpy(dq, qi_host, (size_t)nseg * 20 * 8, hipMemcpyHostToDevice);
  hipMemcpy(dg, guess_host, 32, hipMemcpyHostToDevice);
  const unsigned grid = (unsigned)((nseg + 63) / 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(lm_probe_kernel<12>, dim3(grid), dim3(64), 0, 0, dq, nseg, nseg, dg, c, dp, dc);
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(lm_probe_kernel<12>, dim3(grid), dim3(64), 0, 0, dq, nseg, nseg, dg, c, dp, dc);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  *ms_out = ms / reps;
  hipMemcpy(p_host, dp, (size_t)nseg * 32, hipMemcpyDeviceToHost);
  hipMemcpy(cyc_host, dc, (size_t)nseg * 64, hipMemcpyDeviceToHost);
  hipFree(dq);
  hipFree(dg);
  hipFree(dp);
  hipFree(dc);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    fprintf(stderr, "%s\n", hipGetErrorString(err));
    return -1;
  }
  return 0;
}

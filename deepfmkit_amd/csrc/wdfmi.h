// wdfmi.h — launcher interface of the witness-based fitters (wdfmi.hip), used by
// the C ABI in dfmi_capi.hip. Internal: the public surface is dfmi_wdfmi_fit in
// include/dfmi.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfmi {

enum WdfmiMethod : int32_t { kWdfmiNLS = 0, kWdfmiOrtho = 1, kWdfmiSeq = 2, kHwdfmi = 3 };

// Everything a launch needs (passed to the kernels by value).
struct WdfmiLaunch {
  int32_t method;
  int32_t R;          // samples per buffer
  int32_t ndata;      // WDFMI_NLSFitter harmonics (fitters.py:492)
  int32_t ndata_psi;  // WDFMI_SequentialFitter stage-2 harmonics (fitters.py:705)
  int32_t L;          // basis period of the harmonic tables (0: per-sample sincos)
  int32_t threads;    // workgroup size (256 / 512 / 1024)
  int64_t nrec, nbuf, rec_stride, wit_stride;
  double f_samp, f_mod, df, f_ref, tau_init, init_a, init_phi, init_psi;
  double w0;                     // (2 pi f_mod) / f_samp
  const double* x;               // main records x[r*rec_stride + b*R + k]
  const double* wit;             // witness records wit[r*wit_stride + k], k < R
  const double* btab_nls;        // 2*ndata x L basis (cos rows, then sin rows), or null
  const double* btab_psi;        // 2*ndata_psi x L basis, or null
  double* tmpl;                  // workspace: nrec_t x R witness templates
  double* out;                   // 7 x (nrec*nbuf): amp, m, phi, psi, tau, dc, ssq
  int32_t* fitok;                // nrec*nbuf
  uint64_t* probe;               // diagnostics timestamps (null: off)
  const int* pw_plan;            // numpy summation plan over R (np_sum.h dfmi_pairwise_plan)
  // bit 0: time axis by multiply + fma correction (when exact), bit 1: the template's
  // slope table in LDS (when it fits); dfmi_set_tuning("wdfmi_accel"), default 3
  int32_t accel;
  // set by wdfmi_launch: the time axis k / f_samp formed as q = k * t_rcp plus one
  // fma correction when that reproduces the division for every k in [0, R] (t_fast)
  int32_t t_fast;
  double t_rcp;
};

// Dynamic LDS bytes the fit kernel of this launch needs.
size_t wdfmi_lds_bytes(const WdfmiLaunch& a);

// Enqueue the template kernel and the fit kernel on `st`.
hipError_t wdfmi_launch(const WdfmiLaunch& a, hipStream_t st);

}  // namespace dfmi

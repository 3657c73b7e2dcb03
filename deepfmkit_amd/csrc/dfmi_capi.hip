// dfmi_capi.hip — host side of libdfmi.so: the C ABI declared in include/dfmi.h.
//
// Owns: lazy HIP initialisation, per-device grow-only workspaces, the cached
// demodulation basis tables and m-grid Bessel tables, kernel selection and
// launch geometry. No torch, no Python.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/dfmi.h"
#include "demod.h"
#include "dfmi_math.h"
#include "ekf.h"
#include "lm.h"
#include "seed.h"

namespace {

thread_local std::string g_err;
std::mutex g_mu;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                       \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      return fail(DFMI_ERR_HIP, std::string(#expr " failed: ") + hipGetErrorString(_e));   \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
};

struct DeviceState {
  bool init = false;
  int n_cu = 0;
  size_t lds_per_block = 0;
  std::map<std::string, DevBuf> ws;                                  // named workspaces
  std::map<std::tuple<int, int, uint64_t>, DevBuf> basis;            // (L, ndata, w0 bits)
  std::map<std::tuple<int, uint64_t, uint64_t, uint64_t>, DevBuf> gridtab;  // (ndata, min, max, step)
  hipStream_t side = nullptr;  // seed step runs here, concurrently with the bulk demod
  hipEvent_t ev_in = nullptr, ev_seed = nullptr;
  uint64_t* seed_ctr = nullptr;  // seed -> bulk LM hand-off: [0] monotonic counter, [8..] seeds (lm.h)
  uint64_t seed_total = 0;       // seeds issued so far (the LM's wait target)
};

std::map<int, DeviceState> g_dev;
int g_ndev = -1;

int ensure_init(int* dev_out) {
  if (g_ndev < 0) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
      g_ndev = 0;
      return fail(DFMI_ERR_NODEV, "no HIP device visible (hipGetDeviceCount: " +
                                      std::string(hipGetErrorString(e)) + ")");
    }
    g_ndev = n;
  }
  if (g_ndev == 0) return fail(DFMI_ERR_NODEV, "no HIP device visible");
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  DeviceState& ds = g_dev[dev];
  if (!ds.init) {
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, dev));
    ds.n_cu = prop.multiProcessorCount;
    ds.lds_per_block = prop.sharedMemPerBlock;
    int prio_lo = 0, prio_hi = 0;  // the seed stream dispatches ahead of the bulk demodulation
    HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    HIPCHK(hipStreamCreateWithPriority(&ds.side, hipStreamNonBlocking, prio_hi));
    HIPCHK(hipEventCreateWithFlags(&ds.ev_in, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ds.ev_seed, hipEventDisableTiming));
    HIPCHK(hipMalloc(&ds.seed_ctr, 512));
    HIPCHK(hipMemset(ds.seed_ctr, 0, 512));
    ds.init = true;
  }
  *dev_out = dev;
  return DFMI_OK;
}

int workspace(int dev, const char* name, size_t bytes, void** out) {
  DevBuf& b = g_dev[dev].ws[name];
  if (b.n < bytes) {
    if (b.p) HIPCHK(hipFree(b.p));
    b.p = nullptr;
    b.n = 0;
    HIPCHK(hipMalloc(&b.p, bytes));
    b.n = bytes;
  }
  *out = b.p;
  return DFMI_OK;
}

uint64_t bits(double v) {
  uint64_t u;
  memcpy(&u, &v, 8);
  return u;
}

// Basis table for the fold kernel: row c < ndata = cos(fl((c+1) w0) p), row
// ndata + c = sin(...), p < L. fit.py:55-64 forms the angle as ((n+1)*w0)*t.
int basis_table(int dev, int L, int ndata, double w0, hipStream_t st, const double** out) {
  auto key = std::make_tuple(L, ndata, bits(w0));
  DevBuf& b = g_dev[dev].basis[key];
  if (!b.p) {
    std::vector<double> h((size_t)2 * ndata * L);
    for (int c = 0; c < ndata; ++c) {
      const double wh = (double)(c + 1) * w0;
      for (int p = 0; p < L; ++p) {
        const double ang = wh * (double)p;
        h[(size_t)c * L + p] = cos(ang);
        h[(size_t)(ndata + c) * L + p] = sin(ang);
      }
    }
    HIPCHK(hipMalloc(&b.p, h.size() * 8));
    b.n = h.size() * 8;
    HIPCHK(hipMemcpy(b.p, h.data(), b.n, hipMemcpyHostToDevice));
  }
  (void)st;
  *out = (const double*)b.p;
  return DFMI_OK;
}

// numpy.arange(min, max + step, step): length ceil((stop - start)/step),
// values start + i*((start + step) - start).
void grid_geometry(const dfmi_lm_config& c, int* n, double* delta) {
  const double stop = c.m_grid_max + c.m_grid_step;
  const double len = ceil((stop - c.m_grid_min) / c.m_grid_step);
  *n = len > 0 ? (int)len : 0;
  *delta = (c.m_grid_min + c.m_grid_step) - c.m_grid_min;
}

int grid_table(int dev, int ndata, const dfmi_lm_config& c, const double** out) {
  auto key = std::make_tuple(ndata, bits(c.m_grid_min), bits(c.m_grid_max), bits(c.m_grid_step));
  DevBuf& b = g_dev[dev].gridtab[key];
  if (!b.p) {
    int n;
    double delta;
    grid_geometry(c, &n, &delta);
    std::vector<double> h((size_t)(n > 0 ? n : 1) * ndata, 0.0);
    std::vector<double> row(ndata + 2);
    for (int g = 0; g < n; ++g) {
      const double mtry = c.m_grid_min + (double)g * delta;
      dfmi_bessel_table(mtry, ndata, row.data());
      for (int i = 0; i < ndata; ++i) h[(size_t)g * ndata + i] = row[i + 1];
    }
    HIPCHK(hipMalloc(&b.p, h.size() * 8));
    b.n = h.size() * 8;
    HIPCHK(hipMemcpy(b.p, h.data(), b.n, hipMemcpyHostToDevice));
  }
  *out = (const double*)b.p;
  return DFMI_OK;
}

int to_lmconst(const dfmi_lm_config* cfg, dfmi::LMConst* c) {
  dfmi_lm_config d;
  if (!cfg) {
    dfmi_lm_config_default(&d);
    cfg = &d;
  }
  if (cfg->n_lambda < 0 || cfg->n_lambda > DFMI_MAX_LAMBDA) return fail(DFMI_ERR_ARG, "n_lambda out of range");
  if (cfg->max_lma_steps < 0) return fail(DFMI_ERR_ARG, "max_lma_steps < 0");
  if (!(cfg->m_grid_step > 0)) return fail(DFMI_ERR_ARG, "m_grid_step must be > 0");
  memset(c, 0, sizeof(*c));
  c->max_steps = cfg->max_lma_steps;
  c->n_lambda = cfg->n_lambda;
  for (int i = 0; i < cfg->n_lambda; ++i) c->lambdas[i] = cfg->lambdas[i];
  c->min_step_norm = cfg->min_step_norm;
  c->conv_improve = cfg->conv_improve;
  c->conv_param_change = cfg->conv_param_change;
  c->fitok_threshold = cfg->fitok_threshold;
  c->bessel_amp_thr = cfg->bessel_amp_threshold;
  c->sincos_amp_thr = cfg->sincos_amp_threshold;
  grid_geometry(*cfg, &c->n_grid, &c->grid_delta);
  c->grid_min = cfg->m_grid_min;
  return DFMI_OK;
}

constexpr int kMaxSlotCap = 8;

// Tuning knobs (dfmi_set_tuning): measured, then frozen as defaults.
struct Tuning {
  int demod_loads = 8;         // vector loads in flight per lane (8 or 16)
  int demod_nt = 1;            // non-temporal stream loads (measured +14 %, profiles/r01_tune_demod.json)
  int demod_blocks_per_cu = 0; // 0 = occupancy limit
  int lm_general = 0;          // 1: force the two-pass (general) LM path for every ndata
  int demod_kernel = 2;        // 0: cycle-aligned fold, 1: software-pipelined cycle-aligned fold
                               // (measured slower: profiles/r01_tune_demod_stream.json), 2: bins in LDS,
                               // 3: bins in LDS, pipelined
  int demod_unr = 4;           // cycles per batch of the streaming fold (1, 2, 4, 5)
  int seed_reserve = 0;        // 1: the bulk demodulation grid leaves slots free for the seed waves
  int demod_dyn = 0;           // 1: dynamic segment scheduling in the bin kernel (demod.h SegQueue;
                               // measured 10 % slower: profiles/r01b_tune_step_dyn_seed.json)
  int seed_spacer = 0;         // 1: bulk demodulation leaves a slot for the seed wave (g_spacer; measured
                               // slower: the 8-wave workgroups cost more than the seed gains)
  int seed_handoff = 1;        // 1: seed -> bulk LM hand-off through a device counter (lm.h seed_ctr)
  int seed_handoff_unreachable = 0;  // test hook: a target the counter never reaches (LM fallback path)
  int seed_bins = 1;           // 1: seed step with the LDS fold + LDS-resident QI (seed.h seed_bins_kernel)
  int demod_bins_cfg = 0;      // bins kernel shape: 0 = 4-wave blocks, LDS basis, 8 harmonics per
                               // reduction block; 1..6 = higher-occupancy shapes (launch_bins_t);
                               // 7, 8 = timing probes (no QI stores / no contraction: results invalid)
};
Tuning g_tune;
std::string g_last_demod;
int g_spacer = 0;
uint64_t* g_probe = nullptr;  // diagnostics timestamps (dfmi_set_tuning("probe", 1), dfmi_probe_read)  // bin kernel: 8-wave workgroups + an idle last workgroup (seed co-scheduling)
// Workgroup slots a persistent demodulation grid leaves free (set by the record
// pipeline for the concurrent seed waves; every launcher subtracts it).
int64_t g_grid_reserve = 0;

int64_t persistent_grid(int n_cu, int per_cu, int64_t need) {
  int64_t grid = (int64_t)n_cu * per_cu - g_grid_reserve;
  if (grid > need) grid = need;
  if (grid < 1) grid = 1;
  return grid;
}  // kernel variant of the last demodulation launch (dfmi_last_demod_kernel)



int32_t detect_period_impl(double w0, int32_t R, int32_t ndata) {
  if (!(w0 > 0) || R <= 0 || ndata <= 0) return 0;
  const double two_pi = 6.283185307179586;
  const int Lmax = 64 * 2 * kMaxSlotCap;
  for (int L = 1; L <= Lmax; ++L) {
    const double v = (double)L * w0 / two_pi;
    const double n = nearbyint(v);
    if (n < 1) continue;
    // periodicity error of the basis, accumulated over R/L cycles at the top harmonic
    const double err = two_pi * fabs(v - n) * (double)ndata * ((double)R / (double)L + 1.0);
    if (err <= 1e-11) return L;
  }
  return 0;
}

template <int VEC, int MS, bool LDS, int LOADS = 8, bool NT = true>
int launch_fold_t(const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata, const double* tab,
                  double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu) {
  if constexpr (VEC == 2 && MS == 2 && LDS && LOADS == 8 && NT) {  // the BASELINE shape: tunable
    if (g_tune.demod_loads == 16 && g_tune.demod_nt)
      return launch_fold_t<2, 2, true, 16, true>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
    if (g_tune.demod_loads == 16)
      return launch_fold_t<2, 2, true, 16, false>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
    if (!g_tune.demod_nt)
      return launch_fold_t<2, 2, true, 8, false>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
  }
  const size_t lds = LDS ? (size_t)2 * ndata * L * sizeof(double) : 0;
  auto kern = dfmi::demod_fold_kernel<VEC, MS, LDS, LOADS, NT>;
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, dfmi::kBlockThreads, lds));
  if (per_cu < 1) per_cu = 1;
  if (g_tune.demod_blocks_per_cu > 0 && g_tune.demod_blocks_per_cu < per_cu) per_cu = g_tune.demod_blocks_per_cu;
  const int64_t grid = persistent_grid(n_cu, per_cu, (nseg + dfmi::kWavesPerBlock - 1) / dfmi::kWavesPerBlock);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(dfmi::kBlockThreads), lds, st, x, nseg, stride, R, L, ndata,
                     tab, qi, qi_ld, dc);
  HIPCHK(hipGetLastError());
  g_last_demod = "demod_fold_kernel<" + std::to_string(VEC) + "," + std::to_string(MS) + "," +
                 std::to_string((int)LDS) + "," + std::to_string(LOADS) + "," + std::to_string((int)NT) + ">";
  return DFMI_OK;
}

template <int VEC, bool LDS>
int launch_fold_ms(int ms, const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata, const double* tab,
                   double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu) {
  switch (ms) {
    case 1: return launch_fold_t<VEC, 1, LDS>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
    case 2: return launch_fold_t<VEC, 2, LDS>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
    case 4: return launch_fold_t<VEC, 4, LDS>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
    default: return launch_fold_t<VEC, 8, LDS>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
  }
}

template <int UNR>
int launch_stream_t(int dev, const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata,
                    const double* tab, double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu) {
  constexpr int MINB = UNR <= 2 ? 4 : 3;
  const size_t lds = (size_t)2 * ndata * L * sizeof(double);
  auto kern = dfmi::demod_stream_kernel<2, UNR, true, MINB>;
  void* pad = nullptr;
  int rc = workspace(dev, "stream_pad", ((size_t)UNR * L + 256) * sizeof(double), &pad);
  if (rc) return rc;
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, dfmi::kBlockThreads, lds));
  if (per_cu < 1) per_cu = 1;
  if (g_tune.demod_blocks_per_cu > 0 && g_tune.demod_blocks_per_cu < per_cu) per_cu = g_tune.demod_blocks_per_cu;
  const int64_t grid = persistent_grid(n_cu, per_cu, (nseg + dfmi::kWavesPerBlock - 1) / dfmi::kWavesPerBlock);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(dfmi::kBlockThreads), lds, st, x, nseg, stride, R, L, ndata,
                     tab, (const double*)pad, qi, qi_ld, dc);
  HIPCHK(hipGetLastError());
  g_last_demod = "demod_stream_kernel<2," + std::to_string(UNR) + ",1," + std::to_string(MINB) + ">";
  return DFMI_OK;
}

// Streaming fold (demod.h demod_stream_kernel) when its preconditions hold:
// 16-B rows, 128 < L <= 256 (two 16-B slots per lane), R % L == 0, basis in LDS,
// and a batch size dividing R / L. Returns 1 if it does not apply.
int try_stream(int dev, const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata, const double* tab,
               double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu, bool vec2, bool use_lds) {
  if (g_tune.demod_kernel != 1 || !vec2 || !use_lds || L <= 128 || L > 256 || R % L) return 1;
  const int ncyc = R / L;
  int unr = g_tune.demod_unr;
  const int prefs[4] = {unr, 4, 2, 1};
  for (int u : prefs) {
    if (ncyc % u) continue;
    switch (u) {
      case 1: return launch_stream_t<1>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
      case 2: return launch_stream_t<2>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
      case 4: return launch_stream_t<4>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
      case 5: return launch_stream_t<5>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
      default: break;
    }
  }
  return 1;
}

template <int MS, int LOADS, bool NT, int WPB = 4, int WPEU = 1, bool TAB_LDS = true, int HB = 8, int PROBE = 0,
          bool ROWS = false, bool DYN = false>
int launch_bins_t(int dev, const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata, const double* tab,
                  double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu, size_t lds_cap) {
  if constexpr (!DYN) {  // dynamic segment scheduling (demod.h SegQueue) unless tuned off
    if (g_tune.demod_dyn)
      return launch_bins_t<MS, LOADS, NT, WPB, WPEU, TAB_LDS, HB, PROBE, ROWS, true>(dev, x, nseg, stride, R, L, ndata,
                                                                                     tab, qi, qi_ld, dc, st, n_cu,
                                                                                     lds_cap);
  }
  if constexpr (MS == 2 && LOADS == 8 && NT && WPB == 4 && WPEU == 1 && TAB_LDS && HB == 8 && PROBE == 0 && !ROWS &&
                !DYN) {
    switch (g_tune.demod_bins_cfg) {  // tunable shape
      case 7: return launch_bins_t<2, 8, true, 4, 1, true, 8, 1>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
      case 8: return launch_bins_t<2, 8, true, 4, 1, true, 8, 2>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
      case 1: return launch_bins_t<2, 8, true, 8, 6, true, 4>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
      case 2: return launch_bins_t<2, 4, true, 8, 6, true, 4>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
      case 3: return launch_bins_t<2, 8, true, 16, 8, true, 2>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
      case 4: return launch_bins_t<2, 4, true, 16, 8, true, 2>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
      case 5: return launch_bins_t<2, 8, true, 4, 6, false, 4>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
      case 6: return launch_bins_t<2, 8, true, 4, 8, false, 2>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
      default: break;
    }
    if (g_tune.demod_loads == 16)
      return launch_bins_t<2, 16, true>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
    if (!g_tune.demod_nt)
      return launch_bins_t<2, 8, false>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
  }
  if constexpr (ROWS && !DYN && WPB == 4 && MS == 2 && LOADS == 8 && NT && WPEU == 1 && TAB_LDS && HB == 8 &&
                PROBE == 0) {
    // With a seed wave co-scheduled (nls_record_device), 8-wave workgroups (2 waves
    // per SIMD, 2 per CU): the spacer's slot is 2 x 128 VGPRs per SIMD + 45 KB LDS,
    // enough for the seed kernel (161 VGPRs, 34 KB); a 4-wave workgroup's is not.
    if (g_spacer)
      return launch_bins_t<2, 8, true, 8, 1, true, 8, 0, true>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc,
                                                               st, n_cu, lds_cap);
  }
  const size_t lds = ((TAB_LDS ? (size_t)2 * ndata * L : 0) + (size_t)WPB * L) * sizeof(double);
  if (lds > lds_cap) return fail(DFMI_ERR_UNSUPPORTED, "demod_bins_kernel: LDS footprint exceeds the workgroup limit");
  auto kern = dfmi::demod_bins_kernel<MS, LOADS, NT, WPB, WPEU, TAB_LDS, HB, PROBE, ROWS, DYN>;
  unsigned* ctr = nullptr;
  if constexpr (DYN) {
    void* cw = nullptr;
    int rc = workspace(dev, "seg_queue", 8 * 64 * sizeof(unsigned), &cw);
    if (rc) return rc;
    ctr = (unsigned*)cw;
    HIPCHK(hipMemsetAsync(ctr, 0, 8 * 64 * sizeof(unsigned), st));
  }
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * WPB, lds));
  if (per_cu < 1) per_cu = 1;
  if (g_tune.demod_blocks_per_cu > 0 && g_tune.demod_blocks_per_cu < per_cu) per_cu = g_tune.demod_blocks_per_cu;
  const int spacer = (g_spacer && !DYN) ? 8 : 0;
  const int64_t grid = persistent_grid(n_cu, per_cu, (nseg + WPB - 1) / WPB + spacer);  // spacer: one of the slots
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * WPB), lds, st, x, nseg, stride, R, L, ndata, tab, qi,
                     qi_ld, dc, ctr, spacer, g_probe);
  HIPCHK(hipGetLastError());
  g_last_demod = "demod_bins_kernel<" + std::to_string(MS) + "," + std::to_string(LOADS) + "," +
                 std::to_string((int)NT) + "," + std::to_string(WPB) + "," + std::to_string(WPEU) + "," +
                 std::to_string((int)TAB_LDS) + "," + std::to_string(HB) + (ROWS ? ",rows" : "") +
                 (DYN ? ",dyn" : "") + (spacer ? ",spacer" : "") + ">";
  return DFMI_OK;
}

template <int MS, int UNR>
int launch_bins_pipe_t(int dev, const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata,
                       const double* tab, double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu,
                       size_t lds) {
  auto kern = g_tune.demod_nt ? dfmi::demod_bins_pipe_kernel<MS, UNR, true> : dfmi::demod_bins_pipe_kernel<MS, UNR, false>;
  void* pad = nullptr;
  int rc = workspace(dev, "bins_pad", 256 * sizeof(double), &pad);
  if (rc) return rc;
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, dfmi::kBlockThreads, lds));
  if (per_cu < 1) per_cu = 1;
  if (g_tune.demod_blocks_per_cu > 0 && g_tune.demod_blocks_per_cu < per_cu) per_cu = g_tune.demod_blocks_per_cu;
  const int64_t grid = persistent_grid(n_cu, per_cu, (nseg + dfmi::kWavesPerBlock - 1) / dfmi::kWavesPerBlock);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(dfmi::kBlockThreads), lds, st, x, nseg, stride, R, L, ndata,
                     tab, (const double*)pad, qi, qi_ld, dc);
  HIPCHK(hipGetLastError());
  g_last_demod = "demod_bins_pipe_kernel<" + std::to_string(MS) + "," + std::to_string(UNR) + "," +
                 std::to_string(g_tune.demod_nt) + ">";
  return DFMI_OK;
}

// Bin-in-LDS fold (demod.h demod_bins_kernel) when its preconditions hold:
// 16-B rows, even L with 128 <= L <= 1024, basis + 4 waves' bins in LDS.
// Returns 1 if it does not apply.
bool bins_applicable(bool vec2, int R, int L, int ndata, size_t lds_cap) {
  (void)R;
  if ((g_tune.demod_kernel != 2 && g_tune.demod_kernel != 3) || !vec2 || (L & 1) || L < 128 || L > 1024) return false;
  const size_t lds = ((size_t)2 * ndata * L + (size_t)dfmi::kWavesPerBlock * L) * sizeof(double);
  return lds <= lds_cap && lds <= 64 * 1024;
}

int try_bins(int dev, const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata, const double* tab,
             double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu, bool vec2, size_t lds_cap,
             bool rows) {
  if (!bins_applicable(vec2, R, L, ndata, lds_cap)) return 1;
  const size_t lds = ((size_t)2 * ndata * L + (size_t)dfmi::kWavesPerBlock * L) * sizeof(double);
  const int nslot = (L + 127) / 128;
  if (rows) {
    if (nslot <= 2)
      return launch_bins_t<2, 8, true, 4, 1, true, 8, 0, true>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st,
                                                               n_cu, lds_cap);
    if (nslot <= 4)
      return launch_bins_t<4, 8, true, 4, 1, true, 8, 0, true>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st,
                                                               n_cu, lds_cap);
    return launch_bins_t<8, 8, true, 4, 1, true, 8, 0, true>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st,
                                                             n_cu, lds_cap);
  }
  if (g_tune.demod_kernel == 3 && (R % 2) == 0) {
    if (nslot <= 2)
      return g_tune.demod_unr == 8
                 ? launch_bins_pipe_t<2, 8>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds)
                 : launch_bins_pipe_t<2, 4>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds);
    if (nslot <= 4) return launch_bins_pipe_t<4, 4>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds);
    return launch_bins_pipe_t<8, 4>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds);
  }
  if (nslot <= 2) return launch_bins_t<2, 8, true>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
  if (nslot <= 4) return launch_bins_t<4, 8, true>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
  return launch_bins_t<8, 8, true>(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds_cap);
}

// Whether demod_device can write the row layout (dfmi_qi_row_stride) for this
// input: only the bin-in-LDS kernel implements it.
bool rows_supported(int dev, const double* x, int64_t stride, int R, int ndata, double w0, int period) {
  int L = period;
  if (L == 0) L = detect_period_impl(w0, R, ndata);
  if (L <= 0) return false;
  const bool vec2 = (L % 2 == 0) && (stride % 2 == 0) && (((uintptr_t)x & 15) == 0);
  return bins_applicable(vec2, R, L, ndata, g_dev[dev].lds_per_block);
}

// Device-pointer demodulation (all pointers on the current device).
// rows = true: write the row layout (qi + s·qi_ld, dfmi_qi_row_stride; dc inside
// the row, `dc` unused) — callers check rows_supported() first.
int demod_device(int dev, const double* x, int64_t nseg, int64_t stride, int R, int ndata, double w0, int period,
                 double* qi, int64_t qi_ld, double* dc, hipStream_t st, bool rows = false) {
  if (nseg == 0) return DFMI_OK;
  int L = period;
  if (L == 0) L = detect_period_impl(w0, R, ndata);
  struct {
    int n_cu;
    size_t lds_per_block;
  } ds = {g_dev[dev].n_cu, g_dev[dev].lds_per_block};
  if (L > 0) {
    const bool vec2 = (L % 2 == 0) && (stride % 2 == 0) && (((uintptr_t)x & 15) == 0);
    const int VEC = vec2 ? 2 : 1;
    int nslot = (L + 64 * VEC - 1) / (64 * VEC);
    if (nslot <= kMaxSlotCap) {
      int ms = 1;
      while (ms < nslot) ms <<= 1;
      const double* tab = nullptr;
      int rc = basis_table(dev, L, ndata, w0, st, &tab);
      if (rc) return rc;
      const size_t lds = (size_t)2 * ndata * L * sizeof(double);
      const bool use_lds = lds <= 64 * 1024 && lds <= ds.lds_per_block;
      rc = try_bins(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, ds.n_cu, vec2, ds.lds_per_block,
                    rows);
      if (rc <= 0) return rc;
      if (rows) return fail(DFMI_ERR_UNSUPPORTED, "row layout needs the bin-in-LDS demodulation kernel");
      rc = try_stream(dev, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, ds.n_cu, vec2, use_lds);
      if (rc <= 0) return rc;
      if (vec2) {
        return use_lds ? launch_fold_ms<2, true>(ms, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, ds.n_cu)
                       : launch_fold_ms<2, false>(ms, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, ds.n_cu);
      }
      return use_lds ? launch_fold_ms<1, true>(ms, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, ds.n_cu)
                     : launch_fold_ms<1, false>(ms, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, ds.n_cu);
    }
  }
  if (rows) return fail(DFMI_ERR_UNSUPPORTED, "row layout needs the bin-in-LDS demodulation kernel");
  // direct kernel
  int64_t need = (nseg + dfmi::kWavesPerBlock - 1) / dfmi::kWavesPerBlock;
  int64_t grid = (int64_t)ds.n_cu * 8;
  if (grid > need) grid = need;
  hipLaunchKernelGGL(dfmi::demod_direct_kernel, dim3((unsigned)grid), dim3(dfmi::kBlockThreads), 0, st, x, nseg,
                     stride, R, ndata, w0, qi, qi_ld, dc);
  HIPCHK(hipGetLastError());
  g_last_demod = "demod_direct_kernel";
  return DFMI_OK;
}

int lm_device(int dev, const double* qi, int64_t qi_ld, int ndata, int64_t nrec, int64_t nbuf, int64_t first,
              int64_t nitems, int64_t nchunk, const double* guess_dev, int64_t g_rec, int64_t g_comp,
              const double* guess_host /* nrec*4, used when nrec <= 8 and guess_dev == null */,
              const dfmi::LMConst& c, const double* jtab, double* out, int64_t out_ld, int32_t* status,
              hipStream_t st, bool rows = false, const uint64_t* seed_ctr = nullptr, uint64_t seed_target = 0,
              const double* seed_init_host = nullptr) {
  if (nrec == 0 || nitems == 0) return DFMI_OK;
  if (nchunk < 1) nchunk = 1;
  if (nchunk > nitems) nchunk = nitems;  // np.array_split chunks beyond nitems are empty
  dfmi::GuessInline ginl;
  memset(&ginl, 0, sizeof(ginl));
  int use_inline = 0;
  if (!guess_dev) {
    if (nrec > 8) return fail(DFMI_ERR_ARG, "inline guesses support at most 8 records");
    for (int64_t r = 0; r < nrec; ++r)
      for (int i = 0; i < 4; ++i) ginl.v[r][i] = guess_host[r * 4 + i];
    use_inline = 1;
  }
  if (seed_ctr) {  // fallback seeds (lm.h): the records' initial guesses
    if (nrec > 8) return fail(DFMI_ERR_ARG, "device seed hand-off supports at most 8 records");
    for (int64_t r = 0; r < nrec; ++r)
      for (int i = 0; i < 4; ++i) ginl.v[r][i] = seed_init_host[r * 4 + i];
  }
  const int64_t lanes = nrec * nchunk;
  const int block = 64;
  const int64_t grid = (lanes + block - 1) / block;
  // register path for ndata <= 16 (QI/Bessel in registers), general path above
  const bool chain = nitems > nchunk;
  const int nd_sel = g_tune.lm_general ? 1000 : ndata;
  if (rows && chain) return fail(DFMI_ERR_ARG, "row layout: chunk size 1 only");
  size_t lds = 0;
  auto kern = chain ? (nd_sel <= 12   ? dfmi::lm_chunks_kernel<12, true>
                       : nd_sel <= 16 ? dfmi::lm_chunks_kernel<16, true>
                                     : dfmi::lm_chunks_kernel<0, true>)
                    : (nd_sel <= 12   ? dfmi::lm_chunks_kernel<12, false>
                       : nd_sel <= 16 ? dfmi::lm_chunks_kernel<16, false>
                                     : dfmi::lm_chunks_kernel<0, false>);
  if (rows) {
    kern = nd_sel <= 12   ? dfmi::lm_chunks_kernel<12, false, true>
           : nd_sel <= 16 ? dfmi::lm_chunks_kernel<16, false, true>
                          : dfmi::lm_chunks_kernel<0, false, true>;
    if (nd_sel <= 16) lds = (size_t)qi_ld * 65 * sizeof(double);  // the wave's rows, transposed
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(block), lds, st, qi, qi_ld, ndata, nrec, nbuf, first, nitems,
                     nchunk, guess_dev, g_rec, g_comp, ginl, use_inline, jtab, c, out, out_ld, status, seed_ctr,
                     seed_target);
  HIPCHK(hipGetLastError());
  return DFMI_OK;
}

// Whole record pipeline on device pointers (fitters.py:370-428).
int nls_record_device(int dev, const double* x, int64_t nrec, int64_t rec_stride, int64_t nbuf, int R, int ndata,
                      double w0, int period, const double* init_guess_host, int parallel, int64_t nchunk,
                      const dfmi_lm_config& cfg, const dfmi::LMConst& c, double* out, int32_t* fitok,
                      hipStream_t st) {
  const int64_t nseg = nrec * nbuf;
  if (nseg == 0) return DFMI_OK;
  DeviceState& ds = g_dev[dev];
  void* qiw = nullptr;
  int rc = workspace(dev, "qi", (size_t)2 * ndata * nseg * sizeof(double), &qiw);
  if (rc) return rc;
  double* qi = (double*)qiw;
  const double* jtab = nullptr;
  rc = grid_table(dev, ndata, cfg, &jtab);
  if (rc) return rc;
  const int64_t out_ld = nseg;
  double* dc = out + 4 * out_ld;
  // guesses: inline kernel arguments for up to 8 records, a device table otherwise
  const double* gdev = nullptr;
  if (nrec > 8) {
    void* gw = nullptr;
    rc = workspace(dev, "guess", (size_t)nrec * 4 * sizeof(double), &gw);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(gw, init_guess_host, (size_t)nrec * 4 * sizeof(double), hipMemcpyHostToDevice, st));
    gdev = (const double*)gw;
  }
  dfmi::GuessInline ginl;
  memset(&ginl, 0, sizeof(ginl));
  if (nrec <= 8)
    for (int64_t r = 0; r < nrec; ++r)
      for (int i = 0; i < 4; ++i) ginl.v[r][i] = init_guess_host[r * 4 + i];

  int64_t reserve = 0;  // persistent-grid slots left free for the seed waves
  bool spacer = false;  // bin kernel with an idle workgroup slot for the seed wave
  bool handoff = false; // seed -> LM through ds.seed_ctr (no stream event)
  if (parallel) {
    // seed step (buffer 0 of every record) on the side stream, concurrently with the
    // bulk demodulation. The bulk grid leaves one workgroup slot (one wave slot on
    // each of a CU's 4 SIMDs) per 4 seed waves, so the seed is resident from the start
    // instead of waiting for the whole demodulation to drain (seed dispatched second)
    // or holding back demod blocks (seed dispatched first): profiles/r01b_seed_timeline.txt.
    int L = period;
    if (L == 0) L = detect_period_impl(w0, R, ndata);
    if (L > 64 * 16) L = 0;
    const double* tab = nullptr;
    if (L > 0 && (rc = basis_table(dev, L, ndata, w0, st, &tab))) return rc;
    void *qs, *ds_;
    if ((rc = workspace(dev, "qi_seed", (size_t)2 * ndata * nrec * 8, &qs))) return rc;
    if ((rc = workspace(dev, "dc_seed", (size_t)nrec * 8, &ds_))) return rc;
    HIPCHK(hipEventRecord(ds.ev_in, st));
    HIPCHK(hipStreamWaitEvent(ds.side, ds.ev_in, 0));
    const bool seed_bins = L > 0 && g_tune.seed_bins && rows_supported(dev, x, R, R, ndata, w0, period) &&
                           (nrec == 1 || (rec_stride % 2) == 0);
    // device-side seed hand-off to the bulk LM (lm.h seed_ctr) instead of ev_seed
    handoff = seed_bins && g_tune.seed_handoff && nrec <= 8 && nbuf > 1 && nchunk >= nbuf - 1;
    if (handoff) ds.seed_total += (uint64_t)nrec;
    if (seed_bins) {  // fold into LDS, QI from LDS in the fit (seed.h seed_bins_kernel)
      const int nslot = (L + 127) / 128;
      const size_t lds = ((size_t)2 * ndata * L + L + dfmi_row_stride(ndata)) * sizeof(double);
      auto sk = ndata <= 12 ? (nslot <= 2 ? dfmi::seed_bins_kernel<12, 2> : nslot <= 4 ? dfmi::seed_bins_kernel<12, 4>
                                                                                     : dfmi::seed_bins_kernel<12, 8>)
              : ndata <= 16 ? (nslot <= 2 ? dfmi::seed_bins_kernel<16, 2> : nslot <= 4 ? dfmi::seed_bins_kernel<16, 4>
                                                                                     : dfmi::seed_bins_kernel<16, 8>)
                            : (nslot <= 2 ? dfmi::seed_bins_kernel<0, 2> : nslot <= 4 ? dfmi::seed_bins_kernel<0, 4>
                                                                                    : dfmi::seed_bins_kernel<0, 8>);
      hipLaunchKernelGGL(sk, dim3((unsigned)nrec), dim3(64), lds, ds.side, x, rec_stride, R, L, ndata, tab, gdev, ginl,
                         gdev ? 0 : 1, jtab, c, out, out_ld, nbuf, fitok, handoff ? ds.seed_ctr : nullptr, g_probe);
    } else {
      auto sk = ndata <= 12 ? dfmi::seed_kernel<12> : ndata <= 16 ? dfmi::seed_kernel<16> : dfmi::seed_kernel<0>;
      hipLaunchKernelGGL(sk, dim3((unsigned)nrec), dim3(64), 0, ds.side, x, rec_stride, R, L, ndata, w0, tab,
                         (double*)qs, (double*)ds_, nrec, gdev, ginl, gdev ? 0 : 1, jtab, c, out, out_ld, nbuf, fitok,
                         nullptr);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ds.ev_seed, ds.side));
    if (g_tune.seed_reserve) reserve = (nrec + 3) / 4 < 64 ? (nrec + 3) / 4 : 64;
    spacer = seed_bins && nrec == 1 && g_tune.seed_spacer;
  }
  // Row layout (one 128-B line per 8 harmonics, dc inside the row: full-line
  // stores) for the chunk-size-1 parallel path when the bin kernel applies;
  // component-major QI otherwise (warm-start chains read QI component-major).
  const bool rows = parallel && (nbuf <= 1 || nchunk >= nbuf - 1) &&
                    (nrec == 1 || (rec_stride % 2) == 0) && rows_supported(dev, x, R, R, ndata, w0, period);
  const int64_t qs = rows ? dfmi_row_stride(ndata) : 0;
  if (rows) {
    void* rw = nullptr;
    if ((rc = workspace(dev, "qrow", (size_t)qs * nseg * sizeof(double), &rw))) return rc;
    qi = (double*)rw;
  }
  g_grid_reserve = reserve;
  g_spacer = spacer ? 1 : 0;
  if (rec_stride == nbuf * (int64_t)R) {
    rc = rows ? demod_device(dev, x, nseg, R, R, ndata, w0, period, qi, qs, nullptr, st, true)
              : demod_device(dev, x, nseg, R, R, ndata, w0, period, qi, nseg, dc, st);
  } else {
    for (int64_t r = 0; r < nrec && rc == 0; ++r) {
      rc = rows ? demod_device(dev, x + r * rec_stride, nbuf, R, R, ndata, w0, period, qi + r * nbuf * qs, qs,
                               nullptr, st, true)
                : demod_device(dev, x + r * rec_stride, nbuf, R, R, ndata, w0, period, qi + r * nbuf, nseg,
                               dc + r * nbuf, st);
    }
  }
  g_grid_reserve = 0;
  g_spacer = 0;
  if (rc) return rc;
  if (!parallel) {
    return lm_device(dev, qi, nseg, ndata, nrec, nbuf, 0, nbuf, 1, gdev, 4, 1, init_guess_host, c, jtab, out, out_ld,
                     fitok, st);
  }
  if (!(handoff && rows)) HIPCHK(hipStreamWaitEvent(st, ds.ev_seed, 0));
  if (nbuf <= 1) {
    if (rows)  // dc of the seed buffers (the LM kernel carries it otherwise)
      HIPCHK(hipMemcpy2DAsync(dc, nbuf * sizeof(double), qi + dfmi_row_dc(ndata), qs * nbuf * sizeof(double),
                              sizeof(double), nrec, hipMemcpyDeviceToDevice, st));
    return DFMI_OK;
  }
  // the rest, seeded with each record's buffer-0 result (read on device: no host sync)
  if (handoff && rows)
    return lm_device(dev, qi, qs, ndata, nrec, nbuf, 1, nbuf - 1, nchunk, out, nbuf, out_ld, nullptr, c, jtab, out,
                     out_ld, fitok, st, true, ds.seed_ctr,
                     ds.seed_total + (g_tune.seed_handoff_unreachable ? (uint64_t)1 << 40 : 0), init_guess_host);
  return lm_device(dev, qi, rows ? qs : nseg, ndata, nrec, nbuf, 1, nbuf - 1, nchunk, out, nbuf, out_ld, nullptr, c,
                   jtab, out, out_ld, fitok, st, rows);
}

}  // namespace

extern "C" {

void dfmi_lm_config_default(dfmi_lm_config* cfg) {
  if (!cfg) return;
  memset(cfg, 0, sizeof(*cfg));
  cfg->max_lma_steps = 100;
  const double lam[8] = {0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0};
  cfg->n_lambda = 8;
  for (int i = 0; i < 8; ++i) cfg->lambdas[i] = lam[i];
  cfg->min_step_norm = 1e-15;
  cfg->conv_improve = 1e-9;
  cfg->conv_param_change = 1e-9;
  cfg->fitok_threshold = 1e-3;
  cfg->m_grid_min = 5.0;
  cfg->m_grid_max = 30.0;
  cfg->m_grid_step = 0.5;
  cfg->bessel_amp_threshold = 0.05;
  cfg->sincos_amp_threshold = 0.1;
}

int32_t dfmi_detect_period(double w0, int32_t R, int32_t ndata) { return detect_period_impl(w0, R, ndata); }

int dfmi_device_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return 0;
  return g_ndev;
}

const char* dfmi_last_error(void) { return g_err.c_str(); }

const char* dfmi_version(void) { return "dfmi 0.2 gfx950"; }

const char* dfmi_last_demod_kernel(void) { return g_last_demod.c_str(); }

int dfmi_probe_read(int64_t* out, int32_t n) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_err.clear();
  if (!g_probe) return fail(DFMI_ERR_ARG, "probe not enabled (dfmi_set_tuning(\"probe\", 1))");
  if (n < 0 || n > 16 || (n && !out)) return fail(DFMI_ERR_ARG, "bad probe read");
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, g_probe, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return DFMI_OK;
}

int dfmi_set_tuning(const char* key, int64_t value) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_err.clear();
  if (!key) return fail(DFMI_ERR_ARG, "null key");
  const std::string k(key);
  if (k == "demod_loads") {
    if (value != 8 && value != 16) return fail(DFMI_ERR_ARG, "demod_loads must be 8 or 16");
    g_tune.demod_loads = (int)value;
  } else if (k == "demod_kernel") {
    if (value < 0 || value > 3) return fail(DFMI_ERR_ARG, "demod_kernel must be 0..3");
    g_tune.demod_kernel = (int)value;
  } else if (k == "seed_bins") {
    g_tune.seed_bins = value ? 1 : 0;
  } else if (k == "probe") {
    if (value && !g_probe) {
      int dev;
      int rc = ensure_init(&dev);
      if (rc) return rc;
      void* p = nullptr;
      if ((rc = workspace(dev, "probe", 16 * sizeof(uint64_t), &p))) return rc;
      HIPCHK(hipMemset(p, 0, 16 * sizeof(uint64_t)));
      g_probe = (uint64_t*)p;
    } else if (!value) {
      g_probe = nullptr;
    }
  } else if (k == "seed_handoff_unreachable") {
    g_tune.seed_handoff_unreachable = value ? 1 : 0;
  } else if (k == "seed_handoff") {
    g_tune.seed_handoff = value ? 1 : 0;
  } else if (k == "seed_spacer") {
    g_tune.seed_spacer = value ? 1 : 0;
  } else if (k == "demod_dyn") {
    g_tune.demod_dyn = value ? 1 : 0;
  } else if (k == "seed_reserve") {
    g_tune.seed_reserve = value ? 1 : 0;
  } else if (k == "demod_bins_cfg") {
    if (value < 0 || value > 8) return fail(DFMI_ERR_ARG, "demod_bins_cfg must be 0..8 (7, 8: timing probes)");
    g_tune.demod_bins_cfg = (int)value;
  } else if (k == "demod_unr") {
    if (value != 1 && value != 2 && value != 4 && value != 5 && value != 8)
      return fail(DFMI_ERR_ARG, "demod_unr must be 1, 2, 4, 5 or 8");
    g_tune.demod_unr = (int)value;
  } else if (k == "demod_nt") {
    g_tune.demod_nt = value ? 1 : 0;
  } else if (k == "lm_general") {
    g_tune.lm_general = value ? 1 : 0;
  } else if (k == "demod_blocks_per_cu") {
    if (value < 0) return fail(DFMI_ERR_ARG, "demod_blocks_per_cu < 0");
    g_tune.demod_blocks_per_cu = (int)value;
  } else {
    return fail(DFMI_ERR_ARG, "unknown tuning key " + k);
  }
  return DFMI_OK;
}

int dfmi_demod(const double* x, int64_t nseg, int64_t seg_stride, int32_t R, int32_t ndata, double w0,
               int32_t period, double* qi, double* dc, int32_t mem, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_err.clear();
  if (nseg < 0 || R <= 0 || ndata <= 0 || seg_stride < R) return fail(DFMI_ERR_ARG, "bad demod geometry");
  if (nseg > 0 && (!x || !qi || !dc)) return fail(DFMI_ERR_ARG, "null pointer");
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (mem == DFMI_MEM_DEVICE) return demod_device(dev, x, nseg, seg_stride, R, ndata, w0, period, qi, nseg, dc, st);
  if (nseg == 0) return DFMI_OK;
  const size_t xb = (size_t)((nseg - 1) * seg_stride + R) * sizeof(double);
  void *dx, *dq, *dd;
  if ((rc = workspace(dev, "h_x", xb, &dx))) return rc;
  if ((rc = workspace(dev, "h_qi", (size_t)2 * ndata * nseg * 8, &dq))) return rc;
  if ((rc = workspace(dev, "h_dc", (size_t)nseg * 8, &dd))) return rc;
  HIPCHK(hipMemcpyAsync(dx, x, xb, hipMemcpyHostToDevice, st));
  rc = demod_device(dev, (const double*)dx, nseg, seg_stride, R, ndata, w0, period, (double*)dq, nseg, (double*)dd, st);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(qi, dq, (size_t)2 * ndata * nseg * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(dc, dd, (size_t)nseg * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return DFMI_OK;
}

int32_t dfmi_qi_row_stride(int32_t ndata) { return ndata > 0 ? dfmi_row_stride((int)ndata) : 0; }

int32_t dfmi_qi_row_dc(int32_t ndata) { return ndata > 0 ? dfmi_row_dc((int)ndata) : 0; }

int dfmi_demod_rows(const double* x, int64_t nseg, int64_t seg_stride, int32_t R, int32_t ndata, double w0,
                    int32_t period, double* rows, int32_t mem, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_err.clear();
  if (nseg < 0 || R <= 0 || ndata <= 0 || seg_stride < R) return fail(DFMI_ERR_ARG, "bad demod geometry");
  if (nseg > 0 && (!x || !rows)) return fail(DFMI_ERR_ARG, "null pointer");
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  if (nseg == 0) return DFMI_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t qs = dfmi_row_stride((int)ndata);
  if (mem == DFMI_MEM_DEVICE) {
    if (!rows_supported(dev, x, seg_stride, R, ndata, w0, period))
      return fail(DFMI_ERR_UNSUPPORTED, "row layout needs 16-B rows and an even basis period 128 <= L <= 1024");
    return demod_device(dev, x, nseg, seg_stride, R, ndata, w0, period, rows, qs, nullptr, st, true);
  }
  const size_t xb = (size_t)((nseg - 1) * seg_stride + R) * sizeof(double);
  void *dx, *dq;
  if ((rc = workspace(dev, "h_x", xb, &dx))) return rc;
  if ((rc = workspace(dev, "h_rows", (size_t)qs * nseg * 8, &dq))) return rc;
  if (!rows_supported(dev, (const double*)dx, seg_stride, R, ndata, w0, period))
    return fail(DFMI_ERR_UNSUPPORTED, "row layout needs 16-B rows and an even basis period 128 <= L <= 1024");
  HIPCHK(hipMemcpyAsync(dx, x, xb, hipMemcpyHostToDevice, st));
  rc = demod_device(dev, (const double*)dx, nseg, seg_stride, R, ndata, w0, period, (double*)dq, qs, nullptr, st, true);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(rows, dq, (size_t)qs * nseg * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return DFMI_OK;
}

int dfmi_lm(const double* qi, int64_t nseg, int32_t ndata, const double* guess, int32_t guess_per_segment,
            int64_t nchunk, const dfmi_lm_config* cfg, double* params, double* ssq, int32_t* status, int32_t mem,
            void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_err.clear();
  if (nseg < 0 || ndata <= 0) return fail(DFMI_ERR_ARG, "bad lm geometry");
  if (nseg > 0 && (!qi || !guess || !params || !ssq || !status)) return fail(DFMI_ERR_ARG, "null pointer");
  dfmi_lm_config dcfg;
  if (!cfg) {
    dfmi_lm_config_default(&dcfg);
    cfg = &dcfg;
  }
  dfmi::LMConst c;
  int rc = to_lmconst(cfg, &c);
  if (rc) return rc;
  int dev;
  if ((rc = ensure_init(&dev))) return rc;
  if (nseg == 0) return DFMI_OK;
  hipStream_t st = (hipStream_t)stream;
  const double* jtab = nullptr;
  if ((rc = grid_table(dev, ndata, *cfg, &jtab))) return rc;
  // the kernel writes 6 columns (col 4 = dc is untouched); stage through a workspace
  void *dq = nullptr, *dg = nullptr, *dout = nullptr, *dst = nullptr;
  const size_t qib = (size_t)2 * ndata * nseg * 8;
  const size_t gb = (size_t)(guess_per_segment ? nseg : 1) * 4 * 8;
  if ((rc = workspace(dev, "lm_out", (size_t)6 * nseg * 8, &dout))) return rc;
  if ((rc = workspace(dev, "lm_status", (size_t)nseg * 4, &dst))) return rc;
  if (mem == DFMI_MEM_DEVICE) {
    dq = (void*)qi;
    dg = (void*)guess;
  } else {
    if ((rc = workspace(dev, "h_qi", qib, &dq))) return rc;
    if ((rc = workspace(dev, "h_guess", gb, &dg))) return rc;
    HIPCHK(hipMemcpyAsync(dq, qi, qib, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dg, guess, gb, hipMemcpyHostToDevice, st));
  }
  double* o = (double*)dout;
  if (guess_per_segment) {
    rc = lm_device(dev, (const double*)dq, nseg, ndata, nseg, 1, 0, 1, 1, (const double*)dg, 4, 1, nullptr, c, jtab, o,
                   nseg, (int32_t*)dst, st);
  } else {
    rc = lm_device(dev, (const double*)dq, nseg, ndata, 1, nseg, 0, nseg, nchunk, (const double*)dg, 4, 1, nullptr,
                   c, jtab, o, nseg, (int32_t*)dst, st);
  }
  if (rc) return rc;
  const hipMemcpyKind kind = (mem == DFMI_MEM_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  HIPCHK(hipMemcpyAsync(params, o, (size_t)4 * nseg * 8, kind, st));
  HIPCHK(hipMemcpyAsync(ssq, o + 5 * nseg, (size_t)nseg * 8, kind, st));
  HIPCHK(hipMemcpyAsync(status, dst, (size_t)nseg * 4, kind, st));
  if (mem != DFMI_MEM_DEVICE) HIPCHK(hipStreamSynchronize(st));
  return DFMI_OK;
}

int dfmi_nls_record(const double* x, int64_t nrec, int64_t rec_stride, int64_t nbuf, int32_t R, int32_t ndata,
                    double w0, int32_t period, const double* init_guess, int32_t parallel, int64_t nchunk,
                    const dfmi_lm_config* cfg, double* out, int32_t* fitok, int32_t mem, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_err.clear();
  if (nrec < 0 || nbuf < 0 || R <= 0 || ndata <= 0) return fail(DFMI_ERR_ARG, "bad record geometry");
  if (nrec > 1 && rec_stride < nbuf * (int64_t)R) return fail(DFMI_ERR_ARG, "rec_stride < nbuf*R");
  if (nrec * nbuf > 0 && (!x || !init_guess || !out || !fitok)) return fail(DFMI_ERR_ARG, "null pointer");
  dfmi_lm_config dcfg;
  if (!cfg) {
    dfmi_lm_config_default(&dcfg);
    cfg = &dcfg;
  }
  dfmi::LMConst c;
  int rc = to_lmconst(cfg, &c);
  if (rc) return rc;
  int dev;
  if ((rc = ensure_init(&dev))) return rc;
  const int64_t nseg = nrec * nbuf;
  if (nseg == 0) return DFMI_OK;
  hipStream_t st = (hipStream_t)stream;
  if (mem == DFMI_MEM_DEVICE)
    return nls_record_device(dev, x, nrec, rec_stride, nbuf, R, ndata, w0, period, init_guess, parallel, nchunk, *cfg,
                             c, out, fitok, st);
  const int64_t rs = (nrec > 1) ? rec_stride : nbuf * (int64_t)R;
  const size_t xb = (size_t)((nrec - 1) * rs + nbuf * (int64_t)R) * 8;
  void *dx, *dout, *dst;
  if ((rc = workspace(dev, "h_x", xb, &dx))) return rc;
  if ((rc = workspace(dev, "h_out", (size_t)6 * nseg * 8, &dout))) return rc;
  if ((rc = workspace(dev, "h_status", (size_t)nseg * 4, &dst))) return rc;
  HIPCHK(hipMemcpyAsync(dx, x, xb, hipMemcpyHostToDevice, st));
  rc = nls_record_device(dev, (const double*)dx, nrec, rs, nbuf, R, ndata, w0, period, init_guess, parallel, nchunk,
                         *cfg, c, (double*)dout, (int32_t*)dst, st);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(out, dout, (size_t)6 * nseg * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(fitok, dst, (size_t)nseg * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return DFMI_OK;
}

int dfmi_ekf(const double* x, int64_t nrec, int64_t rec_stride, int64_t n_samp, const double* x0,
             const double* p0_diag, const double* q_diag, const double* r_val, double w_m, double f_samp, int32_t R,
             int64_t nbuf, double* states, int32_t mem, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_err.clear();
  if (nrec < 0 || n_samp < 0 || R <= 0 || nbuf < 0) return fail(DFMI_ERR_ARG, "bad ekf geometry");
  if (nrec > 1 && rec_stride < n_samp) return fail(DFMI_ERR_ARG, "rec_stride < n_samp");
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  if (nrec == 0) return DFMI_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t rs = nrec > 1 ? rec_stride : n_samp;
  const double *dx = x, *dx0 = x0, *dp0 = p0_diag, *dq = q_diag, *dr = r_val;
  double* dstates = states;
  const size_t sb = (size_t)nrec * nbuf * 5 * 8;
  if (mem != DFMI_MEM_DEVICE) {
    void *a, *b, *c2, *d, *e, *f;
    const size_t xb = (size_t)((nrec - 1) * rs + n_samp) * 8;
    if ((rc = workspace(dev, "e_x", xb > 0 ? xb : 8, &a))) return rc;
    if ((rc = workspace(dev, "e_x0", (size_t)nrec * 5 * 8, &b))) return rc;
    if ((rc = workspace(dev, "e_p0", 5 * 8, &c2))) return rc;
    if ((rc = workspace(dev, "e_q", 5 * 8, &d))) return rc;
    if ((rc = workspace(dev, "e_r", (size_t)nrec * 8, &e))) return rc;
    if ((rc = workspace(dev, "e_st", sb > 0 ? sb : 8, &f))) return rc;
    if (xb) HIPCHK(hipMemcpyAsync(a, x, xb, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(b, x0, (size_t)nrec * 5 * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c2, p0_diag, 5 * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d, q_diag, 5 * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e, r_val, (size_t)nrec * 8, hipMemcpyHostToDevice, st));
    dx = (const double*)a;
    dx0 = (const double*)b;
    dp0 = (const double*)c2;
    dq = (const double*)d;
    dr = (const double*)e;
    dstates = (double*)f;
  }
  if (sb) HIPCHK(hipMemsetAsync(dstates, 0, sb, st));
  const int block = 64;
  const int64_t grid = (nrec + block - 1) / block;
  hipLaunchKernelGGL(dfmi::ekf_kernel, dim3((unsigned)grid), dim3(block), 0, st, dx, nrec, rs, n_samp, dx0, dp0, dq,
                     dr, w_m, f_samp, (int)R, nbuf, dstates);
  HIPCHK(hipGetLastError());
  if (mem != DFMI_MEM_DEVICE) {
    if (sb) HIPCHK(hipMemcpyAsync(states, dstates, sb, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  return DFMI_OK;
}

}  // extern "C"

// dfmi_capi.hip — host side of libdfmi.so: the C ABI declared in include/dfmi.h.
//
// Owns: lazy HIP initialisation, per-device grow-only workspaces, the cached
// demodulation basis tables and m-grid Bessel tables, kernel selection and
// launch geometry. No torch, no Python.
#include <hip/hip_runtime.h>
#include <math.h>
#include <unistd.h>
#include <stdio.h>
#include <string.h>

#include <array>
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
#include "ekf_pit.h"
#include "lm.h"
#include "seed.h"
#include "np_sum.h"
#include "fork_guard.h"
#include "moments.h"
#include "synth.h"
#include "wdfmi.h"

namespace dfmi {
hipError_t snr_gen_launch(const dfmi_snr_params& p, int64_t idx0, int64_t n, double* out, int n_cu, hipStream_t st);
hipError_t bessel_eval_launch(const double* x, int64_t nx, int nmax, int method, double* out, hipStream_t st);
}

namespace {

thread_local std::string g_err;
std::mutex g_mu;  // the device map, HIP initialisation and the tuning knobs

// Tuning knobs (dfmi_set_tuning): every knob selects a path some input can need or a
// measured schedule; results do not depend on them. Set under g_mu; each C-ABI call
// works on its own snapshot (CallScope), so a concurrent dfmi_set_tuning never races
// a launch. Variants measured slower and removed in round 3 (numbers in DESIGN.md §4;
// code in git history before commit "remove measured-slower variants"): lm_refill,
// lm_phase, lm_spec 1/2, bins_roll, bins_ilv, bins_loads 16, demod_occ4, demod_loads /
// demod_nt, seed_fused 0 / seed_order.
struct Tuning {
  int demod_kernel = 1;  // 1: bin-in-LDS kernel where it applies, 0: cycle-aligned fold kernel
  int lm_general = 0;    // 1: force the two-pass (general) LM path for every ndata
  int demod_spw = 2;     // bin kernels: grid sized for ~this many segments per wave (0: one persistent
                         // wave per slot); later workgroups go to the slots that free first
  int demod_wide = 1;    // component-major QI where the bin kernel's LDS basis does not fit: 1 the
                         // many-harmonic kernel (demod_wide_kernel), 0 the fold kernel; 2 (A/B) the
                         // many-harmonic kernel wherever its geometry applies
  int demod_wide_from = 13;  // ndata from which demod_wide_kernel (component-major) goes ahead of the bin
                             // kernel, and the record pipeline leaves the row layout for it
  int lm_wide = 1;              // ndata > 16: the many-harmonic LM path (lm.h kWideNd: closed-form sums over a
                                // lean Miller walk); 0 = the literal general path (lm_general = 1 forces it too)
  int lm_wide_fused = 1;        // many-harmonic LM with QI from L2 (ndata > lm_wide_lds), the ladder and the seed:
                                // each trial walks once for ssqf AND coeffs (lm.h wide_full, same bits); 0:
                                // ssqf-only trials + a second walk at accepted points
  int lm_ladder_split = 4;      // the ladder beyond 16 harmonics for at most this many items per CU: one wave per
                                // item as 8 rungs x 8 harmonic shares (lm.h PartFullEval); 0 = 8 lanes per item
  int seed_wave_split = 1;      // the seed beyond 16 harmonics: the wave as 8 rungs x 8 harmonic shares (seed.h
                                // SFLAT 3); 0: 8 rungs, every 8-lane group the same whole fit
  int lm_wide_lds = 20;         // many-harmonic LM: QI staged in LDS per lane up to this ndata (0: never): while 8
                                // waves per CU still fit (20 KB per wave); ndata 20 0.076 vs 0.088 ms per 100k
                                // segments, but 30 / 40 0.151 / 0.179 vs 0.118 / 0.149 at 5 / 3 waves per CU (r06g)
  int lm_split = 0;             // many-harmonic LM with this many lanes per segment (2 / 4; 0 = one lane): measured
  int lm_split_from = 41;       // slower everywhere (ndata 30 / 62: 0.195 / 0.432 ms at 2 lanes, 0.260 / 0.420 at 4,
                                // against 0.118 / 0.215 for one lane; r06g), kept for A/B
  int lm_onepass = 1;           // LM general path: one Bessel walk per evaluation with the values in LDS
                                // (1: where 7 waves per CU still fit, 2: always, 0: never)
  int demod_wide_rmax = 2000;  // segments shorter than this go through demod_wide_kernel too
  int demod_wide_half = 1;  // demod_wide_kernel: half-wave contraction at 2·ndata + 1 <= 32 (0: off, A/B)
  int demod_wide_dbg = 0;   // diagnostics: demod_wide_kernel without its contraction (1) / stores (2)
  int demod_wide_k = 0;     // demod_wide_kernel segments per wave (KSEG): 0 = 8; 2 / 4 / 8 (A/B)
  int ekf_row = 1;       // EKF: ekf_row_kernel (4 channels per wave) up to ekf_row x 4 x 4 x CUs channels
                         // (past one wave per SIMD the issue-bound rows share a SIMD, and one lane per
                         // channel carries 16x the channels per instruction); 0 = ekf_kernel only
  int ekf_rot = 1;       // EKF row kernel: sincos by rotation between anchors (ekf_rot_kernel) where R % 4 == 0
  int wdfmi_accel = 3;   // W-DFMI: bit 0 time axis without division, bit 1 template slopes in LDS
  int lm_ladder = 32;    // LM launches of at most lm_ladder x CUs chains / segments (latency-bound: warm-start
                         // chains, small batches) run the parallel lambda ladder (lm.h lm_ladder_kernel);
                         // 0 = always one lane per chain / segment
  int ws_streams = 4;    // caller streams whose workspaces are kept; a call from one more stream first
                         // drains the DEVICE (hipDeviceSynchronize) and frees the least recently used set
  int ekf_pit = 1024;    // EKF parallel in time (ekf_pit.h) for up to this many channels of at least
                         // ekf_pit_min samples (1,024 channels at 400k samples: 48 vs 71 ms for the row
                         // kernel, r04z); 0 = the sequential kernels always
  int ekf_pit_min = 4096;     // samples per channel below which the sequential kernels run (crossover
                              // ~3,000 samples: 2,000 0.8x, 4,000 1.45x the row kernel, r04r)
  int ekf_pit_block = 0;      // samples per block (0: ~n nrec^(2/3) / 16384, at least 16)
  int ekf_pit_passes = 0;     // pass cap: a channel still passing then goes to the sequential kernel; 0 = by
                              // length, n / 1600 within [48, 256] (a pass of one 400k-sample channel costs
                              // ~0.1 ms against ~68 ms for the sequential kernel; 48 passes of a
                              // 4,096-sample one cost about its ~0.7-ms sequential run)
  int ekf_pit_first = 5;      // passes enqueued before the host first reads how many channels still pass
                              // (then every ekf_pit_every); config 5's record converges in 5
  int ekf_pit_every = 2;
  int ekf_pit_topfix = 1;     // the scan's top level (<= 4 elements, above level 1) folded by the fix-up below it
  int ekf_pit_tol = 13;       // stop rule: distance from the fixed point bounded by 10^-ekf_pit_tol (pit_decide)
  int ekf_pit_overlap = 0;    // sequential re-runs of handed-over channels: 0 all in one launch after the passes;
                              // 3 at each host check on the next of kEkfPool high-priority streams beside the
                              // passes, 2 on one high-priority stream, 1 on one default-priority stream
  int ekf_pit_slow_from = 16; // pass from which "too slow to meet the bound within the cap" counts (pit_decide)
  int ekf_pit_stall = 3;      // passes in a row not contracting fast enough to meet the bound within the cap
                              // before the sequential kernel (pit_decide)
  int ekf_pit_trace = 0;      // 1: record every pass's move per channel (dfmi_ekf_pit_trace)
  int ekf_pit_seq = 1;        // 0 (diagnostics only): leave an unconverged channel's last pass in place
  int ekf_pit_measure = 0;    // the stop rule's move: 0 the output snapshots, 1 (diagnostics) the block entries
  int ekf_pit_head = 256;     // samples the sequential EKF runs first to seed the trajectory (ekf_pit_head_kernel)
  int ekf_pit_fused = 1;      // 1: EKF + fold in one kernel per pass (ekf_pit_pass_kernel); 0: separate kernels
};
Tuning g_tune;

// One C-ABI call on this thread: clears the error, snapshots the tuning knobs,
// remembers the caller's stream (workspaces are per stream: two DFMI_MEM_DEVICE calls
// in flight on different streams never share scratch) and, once ensure_init has picked
// the device, holds that DEVICE's lock — calls on different devices from different
// host threads run concurrently; calls on one device are serialised while they enqueue.
struct CallScope;
thread_local CallScope* t_call = nullptr;
thread_local Tuning t_tune;
struct CallScope {
  std::unique_lock<std::mutex> dev_lk;
  hipStream_t stream;
  explicit CallScope(void* s = nullptr) : stream((hipStream_t)s) {
    g_err.clear();
    {
      std::lock_guard<std::mutex> g(g_mu);
      t_tune = g_tune;
    }
    t_call = this;
  }
  ~CallScope() { t_call = nullptr; }
  CallScope(const CallScope&) = delete;
  CallScope& operator=(const CallScope&) = delete;
};

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
  int64_t aux = 0;  // pwplan: leaves of the plan
};

// Workspaces of one caller stream (name -> buffer) and when that stream last used them.
struct StreamWs {
  std::map<std::string, DevBuf> bufs;
  uint64_t last_use = 0;
};

struct DeviceState {
  bool init = false;
  int n_cu = 0;
  size_t lds_per_block = 0;
  std::map<uintptr_t, StreamWs> ws;                                  // caller stream -> workspaces
  uint64_t ws_clock = 0;
  std::map<std::tuple<int, int, uint64_t>, DevBuf> basis;            // (L, ndata, w0 bits); (L, -(8 ndata + no), w0 bits): wide
  std::map<std::tuple<int, uint64_t, uint64_t, uint64_t>, DevBuf> gridtab;  // (ndata, min, max, step)
  std::map<int64_t, DevBuf> pwplan;                                 // n -> numpy pairwise-sum plan
  std::map<std::pair<const void*, int>, int> occupancy;              // (kernel, LDS bytes) -> blocks per CU
  std::mutex mu;               // held by the call that drives this device (CallScope)
  hipStream_t side = nullptr;  // seed step runs here, concurrently with the bulk demod (unfused layouts)
  hipEvent_t ev_in = nullptr, ev_seed = nullptr;
  uint64_t* probe = nullptr;   // diagnostics timestamps of this device (dfmi_set_tuning("probe", 1))
  // dfmi_step_timing: timing events around the record pipeline's kernels, per call
  // [start, after the demodulation launch, after the LM launch]
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::array<hipEvent_t, 3>> ev_steps;
  void* pin = nullptr;  // pinned host scratch for the EKF's pass control read-backs
  size_t pin_n = 0;
  // the EKF parallel in time's hand-over stream: sequential re-runs of channels that stopped
  // contracting run here beside the remaining passes (created on first use)
  hipStream_t ekf_side = nullptr, ekf_side_lo = nullptr;  // high / default priority (ekf_pit_overlap 2 / 1)
  hipStream_t ekf_pool[3] = {};                           // ekf_pit_overlap 3: one per hand-over, round robin
  hipEvent_t ev_ekf_in = nullptr, ev_ekf_out = nullptr;
};

std::map<int, DeviceState> g_dev;
int g_ndev = -1;
long g_init_pid = 0;  // the process that first initialised HIP through this library (fork_guard.h)

thread_local DeviceState* t_ds = nullptr;  // the device of the current call

int ensure_init_locked(int* dev_out);

// Picks (and on first use initialises) the current HIP device and takes its lock
// for the rest of the current CallScope.
int ensure_init(int* dev_out) {
  DeviceState* ds = nullptr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    int rc = ensure_init_locked(dev_out);
    if (rc) return rc;
    ds = &g_dev[*dev_out];
  }
  if (t_call && !t_call->dev_lk.owns_lock()) t_call->dev_lk = std::unique_lock<std::mutex>(ds->mu);
  t_ds = ds;
  return DFMI_OK;
}

int ensure_init_locked(int* dev_out) {
  // fork_guard.h: a process forked after this library initialised HIP gets an error
  // before any runtime call (the pid is recorded at the first initialisation attempt)
  const std::string forked = dfmi_fork_guard(g_init_pid, (long)getpid());
  if (!forked.empty()) return fail(DFMI_ERR_HIP, forked);
  if (g_ndev < 0) {
    g_init_pid = (long)getpid();
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
    ds.init = true;
  }
  *dev_out = dev;
  return DFMI_OK;
}

// Step-timing marks (dfmi_step_timing): mark(i) records event i of the current step's
// triple on st when timing is on. The triple joins ds.ev_steps only by commit(), after
// its last mark: a call that fails (or turns out not to be fused) half-way hands its
// events back to the pool in the destructor, so dfmi_step_timing_read never meets an
// event that was not recorded. At most kMaxMarkedSteps triples wait to be read; further
// calls are not marked (dfmi_step_timing_read reports how many were).
constexpr size_t kMaxMarkedSteps = 1 << 16;
struct StepMarks {
  std::array<hipEvent_t, 3> ev{};
  DeviceState* ds = nullptr;
  bool on = false, committed = false;
  int begin(DeviceState& d) {
    ds = &d;
    on = d.timing && d.ev_steps.size() < kMaxMarkedSteps;
    if (!on) return DFMI_OK;
    int got = 0;
    for (auto& e : ev) {
      if (d.ev_pool.empty()) {
        if (hipEventCreate(&e) != hipSuccess) {
          for (int i = 0; i < got; ++i) d.ev_pool.push_back(ev[i]);
          on = false;
          return fail(DFMI_ERR_HIP, "hipEventCreate (step timing)");
        }
      } else {
        e = d.ev_pool.back();
        d.ev_pool.pop_back();
      }
      ++got;
    }
    return DFMI_OK;
  }
  int mark(int i, hipStream_t st) {
    if (on) HIPCHK(hipEventRecord(ev[i], st));
    return DFMI_OK;
  }
  void commit() {
    if (!on) return;
    ds->ev_steps.push_back(ev);
    committed = true;
  }
  ~StepMarks() {
    if (on && !committed) ds->ev_pool.insert(ds->ev_pool.end(), ev.begin(), ev.end());
  }
};

int free_stream_ws(StreamWs& s) {
  for (auto& kv : s.bufs)
    if (kv.second.p) HIPCHK(hipFree(kv.second.p));
  s.bufs.clear();
  return DFMI_OK;
}

// Grow-only scratch buffer `name` of the current caller stream. Workspaces of at most
// ws_streams (tuning key, default 4) caller streams are kept: a call from a further stream
// first waits for the device to drain and frees the least recently used stream's set
// (include/dfmi.h: a caller cycling over more streams than that serialises on the device,
// and such a call cannot be captured into a graph).
int workspace(int dev, const char* name, size_t bytes, void** out) {
  (void)dev;
  const uintptr_t key = t_call ? (uintptr_t)t_call->stream : 0;
  DeviceState& ds = *t_ds;
  auto it = ds.ws.find(key);
  if (it == ds.ws.end()) {
    if (ds.ws.size() >= (size_t)(t_tune.ws_streams > 0 ? t_tune.ws_streams : 1)) {
      auto lru = ds.ws.begin();
      for (auto jt = ds.ws.begin(); jt != ds.ws.end(); ++jt)
        if (jt->second.last_use < lru->second.last_use) lru = jt;
      HIPCHK(hipDeviceSynchronize());  // its buffers may still be read by queued work
      if (int rc = free_stream_ws(lru->second)) return rc;
      ds.ws.erase(lru);
    }
    it = ds.ws.emplace(key, StreamWs{}).first;
  }
  it->second.last_use = ++ds.ws_clock;
  DevBuf& b = it->second.bufs[std::string(name)];
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

// Device copy of numpy's summation plan over n elements (np_sum.h), cached per n;
// n_leaves (optional) = plan[0].
int pairwise_plan(int dev, int64_t n, const int** out, int64_t* n_leaves) {
  DevBuf& pb = t_ds->pwplan[n];
  if (!pb.p) {
    const std::vector<int> plan = dfmi_pairwise_plan((int)n);
    HIPCHK(hipMalloc(&pb.p, plan.size() * sizeof(int)));
    pb.n = plan.size() * sizeof(int);
    HIPCHK(hipMemcpy(pb.p, plan.data(), pb.n, hipMemcpyHostToDevice));
    pb.aux = plan[0];
  }
  *out = (const int*)pb.p;
  if (n_leaves) *n_leaves = pb.aux;
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
  DevBuf& b = t_ds->basis[key];
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

// The basis for demod_wide_kernel: pairs (T[o][p], T[o][p+1]) at [(p/2)·64·no + o] for
// p = 0..L/2 (zero beyond), o over [cos rows | sin rows | ones (dc) | zeros up to 64·no]; the
// values are basis_table's.
int basis_table_wide(int dev, int L, int ndata, double w0, int no, const double** out) {
  auto key = std::make_tuple(L, -(ndata * 8 + no), bits(w0));
  DevBuf& b = t_ds->basis[key];
  if (!b.p) {
    const int w = 64 * no;
    const int npp = (L / 2 + 2) / 2;
    std::vector<double> h((size_t)npp * w * 2, 0.0);
    auto put = [&](int o, int p, double v) { h[((size_t)(p / 2) * w + o) * 2 + (p & 1)] = v; };
    for (int c = 0; c < ndata; ++c) {
      const double wh = (double)(c + 1) * w0;
      for (int p = 0; p <= L / 2; ++p) {
        const double ang = wh * (double)p;
        put(c, p, cos(ang));
        put(ndata + c, p, sin(ang));
      }
    }
    for (int p = 0; p <= L / 2; ++p) put(2 * ndata, p, 1.0);
    HIPCHK(hipMalloc(&b.p, h.size() * 8));
    b.n = h.size() * 8;
    HIPCHK(hipMemcpy(b.p, h.data(), b.n, hipMemcpyHostToDevice));
  }
  (void)dev;
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
  DevBuf& b = t_ds->gridtab[key];
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
  c->trig = dfmi_trig_k();
  return DFMI_OK;
}

constexpr int kMaxSlotCap = 8;

// A/B build switches of the bin kernel (defaults = the shipped configuration)
#ifndef DFMI_EKF_SPLIT
#define DFMI_EKF_SPLIT 1      // EKF row kernel: lane-split sincos (ekf.h ekf_sincos_row); 0 for A/B builds
#endif
#ifndef DFMI_BINS_LOADS
#define DFMI_BINS_LOADS 10    // 1-KB chunk loads in flight per wave (10: the step 0.7-1.0 % shorter than 8, r03x)
#endif
#ifndef DFMI_BINS_PFN
#define DFMI_BINS_PFN 4       // next segment's chunks prefetched during the contraction (L <= 256)
#endif
#ifndef DFMI_WIDE_LOADS
#define DFMI_WIDE_LOADS 10    // demod_wide_kernel: 1-KB chunk loads in flight per wave
#endif
#ifndef DFMI_BINS_LDS_PAD
#define DFMI_BINS_LDS_PAD 0   // extra dynamic LDS bytes per workgroup (occupancy experiments)
#endif

thread_local std::string g_last_demod;  // kernel variant of the last demodulation launch (dfmi_last_demod_kernel)

// hipOccupancyMaxActiveBlocksPerMultiprocessor, cached per (kernel, LDS bytes): the
// query costs host time on every call otherwise.
template <typename K>
int occupancy(K kern, int threads, size_t lds, int* per_cu) {
  const auto key = std::make_pair((const void*)kern, (int)lds * 4096 + threads);
  auto it = t_ds->occupancy.find(key);
  if (it == t_ds->occupancy.end()) {
    int v = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kern, threads, lds));
    it = t_ds->occupancy.emplace(key, v).first;
  }
  *per_cu = it->second;
  return DFMI_OK;
}

int64_t persistent_grid(int n_cu, int per_cu, int64_t need) {
  int64_t grid = (int64_t)n_cu * per_cu;
  if (grid > need) grid = need;
  if (grid < 1) grid = 1;
  return grid;
}

// Bin-kernel grid (4-wave workgroups, grid-stride over segments): at least the resident
// slots; with demod_spw > 0 enough workgroups for ~demod_spw segments per wave, so the
// hardware dispatcher hands the later workgroups to the slots that free first. With one
// persistent wave per slot and a static segment list, waves finished between 448 and
// 548 us (XCC and HBM-path dependent, profiles/r02j_demod_wave_finish.jsonl) and the
// launch ended with the slowest; ~2 segments per wave measured best (0.513-0.516 vs
// 0.533-0.535 ms, profiles/r02k_tune_spw.json).
int64_t bins_grid(int n_cu, int per_cu, int64_t nseg) {
  const int64_t need = (nseg + dfmi::kWavesPerBlock - 1) / dfmi::kWavesPerBlock;
  int64_t grid = persistent_grid(n_cu, per_cu, need);
  if (t_tune.demod_spw > 0) {
    const int64_t per = (int64_t)dfmi::kWavesPerBlock * t_tune.demod_spw;
    const int64_t want = (nseg + per - 1) / per;
    if (want > grid) grid = want;
  }
  return grid;
}

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

// Cycle-aligned fold kernel (lane-owned bins in registers): the fallback for periods the
// bin kernel does not take (L < 128, odd L, unaligned rows). 8 vector loads in flight per
// lane, non-temporal (+14 %, profiles/r01_tune_demod.json; 16 in flight measured level).
template <int VEC, int MS, bool LDS>
int launch_fold_t(const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata, const double* tab,
                  double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu) {
  const size_t lds = LDS ? (size_t)2 * ndata * L * sizeof(double) : 0;
  auto kern = dfmi::demod_fold_kernel<VEC, MS, LDS, 8, true>;
  int per_cu = 0;
  if (int orc = occupancy(kern, dfmi::kBlockThreads, lds, &per_cu)) return orc;
  if (per_cu < 1) per_cu = 1;
  const int64_t grid = persistent_grid(n_cu, per_cu, (nseg + dfmi::kWavesPerBlock - 1) / dfmi::kWavesPerBlock);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(dfmi::kBlockThreads), lds, st, x, nseg, stride, R, L, ndata,
                     tab, qi, qi_ld, dc);
  HIPCHK(hipGetLastError());
  g_last_demod = "demod_fold_kernel<" + std::to_string(VEC) + "," + std::to_string(MS) + "," +
                 std::to_string((int)LDS) + ",8,1>";
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

// The bin kernel: 8 chunk loads in flight per wave; with L <= 256 (MS 2) the next
// segment's first 4 chunks are prefetched during the contraction (+1.4 % on the step,
// profiles/r01g_ab_prefetch.jsonl; 6 chunks tied, 16 loads per group -1.7 %, a rolling
// pipeline -0.7 %, the contraction interleaved with the next segment's loads level).
template <int MS, bool ROWS>
int launch_bins_t(const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata, const double* tab,
                  double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu, size_t lds) {
  constexpr int PFN = MS == 2 ? DFMI_BINS_PFN : 0;
  auto kern = dfmi::demod_bins_kernel<MS, DFMI_BINS_LOADS, ROWS, PFN>;
  lds += DFMI_BINS_LDS_PAD;
  int per_cu = 0;
  if (int orc = occupancy(kern, dfmi::kBlockThreads, lds, &per_cu)) return orc;
  if (per_cu < 1) per_cu = 1;
  const int64_t grid = bins_grid(n_cu, per_cu, nseg);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(dfmi::kBlockThreads), lds, st, x, nseg, stride, R, L, ndata,
                     tab, qi, qi_ld, dc, t_ds->probe);
  HIPCHK(hipGetLastError());
  g_last_demod = std::string("demod_bins_kernel<") + std::to_string(MS) + "," + std::to_string(DFMI_BINS_LOADS) +
                 (ROWS ? ",rows" : "") + "," + std::to_string(PFN) + ">" +
                 (PFN && (R >> 7) >= PFN ? " (prefetch " + std::to_string(PFN) + ")" : "");
  return DFMI_OK;
}

// Component-major QI through demod_wide_kernel ahead of the bin kernel: from
// demod_wide_from harmonics on (the bin kernel's LDS basis costs it occupancy from 13: 0.624
// vs ~0.55 ms at ndata 16, bench r05z), for segments shorter than demod_wide_rmax samples
// (the bin kernel's per-segment contraction and butterfly dominate there: the record step at
// R = 200 / 400 / 1000, ndata 10, 1.69 / 0.96 / 0.43 ms against 0.95 / 0.58 / 0.34 through
// demod_wide_kernel, 0.233 against 0.265 at R = 4000: profiles/r05/short_segments.jsonl), or
// everywhere with demod_wide = 2 (A/B).
bool wide_first(int ndata, int R) {
  return t_tune.demod_kernel == 1 &&
         (t_tune.demod_wide == 2 ||
          (t_tune.demod_wide == 1 && (ndata >= t_tune.demod_wide_from || R < t_tune.demod_wide_rmax)));
}

int wide_no(int ndata) { return 2 * ndata + 1 <= 64 ? 1 : 2 * ndata + 1 <= 128 ? 2 : 4; }

// Segments per wave demod_wide_kernel runs with: the requested KSEG (demod_wide_k, 0 = 8),
// halved until the workgroup's dynamic LDS (kWavesPerBlock·KSEG·wide_set doubles: 66,560 B at
// L = 256, KSEG 8) fits this device's LDS per workgroup; 0 when not even KSEG 2 fits.
int wide_kseg(int L, int ndata) {
  const int no = wide_no(ndata);
  for (int k = t_tune.demod_wide_k ? t_tune.demod_wide_k : 8; k >= 2; k >>= 1)
    if ((size_t)dfmi::kWavesPerBlock * k * dfmi::wide_set(L, no, k) * sizeof(double) <= t_ds->lds_per_block) return k;
  return 0;
}

// demod_wide_kernel (component-major QI at many harmonics): its geometry (16-B rows, an even
// basis period 128..256, at most 127 harmonics) and an LDS footprint this device holds
// (otherwise the bin / fold kernels run).
bool wide_geometry(bool vec2, int L, int ndata) {
  return vec2 && !(L & 1) && L >= 128 && L <= 256 && 2 * ndata + 1 <= 64 * 4 && wide_kseg(L, ndata) > 0;
}

template <int NO, int KSEG>
int launch_wide_t(const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata, const double* tabT,
                  double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu) {
  // half-wave contraction where the outputs fit 32 lanes (2·ndata + 1 <= 32)
  const bool half = NO == 1 && 2 * ndata + 1 <= 32 && t_tune.demod_wide_half;
  auto kern = half ? dfmi::demod_wide_kernel<NO, KSEG, DFMI_WIDE_LOADS, 4, (NO == 1 && KSEG % 2 == 0) ? 1 : 0>
                   : dfmi::demod_wide_kernel<NO, KSEG, DFMI_WIDE_LOADS, 4, 0>;
  const size_t lds = (size_t)dfmi::kWavesPerBlock * KSEG * dfmi::wide_set(L, NO, KSEG) * sizeof(double);
  (void)n_cu;
  const int64_t per_block = (int64_t)dfmi::kWavesPerBlock * KSEG;
  const int64_t grid = (nseg + per_block - 1) / per_block;  // one group of KSEG segments per wave
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(dfmi::kBlockThreads), lds, st, x, nseg, stride, R, L, ndata,
                     tabT, qi, qi_ld, dc, t_tune.demod_wide_dbg);
  HIPCHK(hipGetLastError());
  g_last_demod = "demod_wide_kernel<" + std::to_string(NO) + "," + std::to_string(KSEG) + "," +
                 std::to_string(DFMI_WIDE_LOADS) + ",4," + (half && KSEG % 2 == 0 ? "1" : "0") + ">";
  return DFMI_OK;
}

int launch_wide(int dev, const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata, double w0,
                double* qi, int64_t qi_ld, double* dc, hipStream_t st, int n_cu) {
  const int no = wide_no(ndata);
  const double* tabT = nullptr;
  if (int rc = basis_table_wide(dev, L, ndata, w0, no, &tabT)) return rc;
  // KSEG 8: level with 4 at R = 4000 (0.578 / 0.576 ms at ndata 30, r05t-x), ahead at 62 (0.631 /
  // 0.617) and for short segments, where the contraction dominates (R = 200, ndata 10: 0.768 /
  // 0.684 ms; R = 400: 0.471 / 0.423; profiles/r05/short_segments_split.jsonl); fewer where the
  // device's LDS per workgroup cannot hold 8 (wide_kseg; callers checked wide_geometry)
  const int k = wide_kseg(L, ndata);
  if (k == 0) return fail(DFMI_ERR_UNSUPPORTED, "demod_wide_kernel: LDS per workgroup too small");
#define DFMI_WIDE(NO_)                                                                                   \
  return k == 8 ? launch_wide_t<NO_, 8>(x, nseg, stride, R, L, ndata, tabT, qi, qi_ld, dc, st, n_cu)      \
         : k == 4 ? launch_wide_t<NO_, 4>(x, nseg, stride, R, L, ndata, tabT, qi, qi_ld, dc, st, n_cu)    \
                  : launch_wide_t<NO_, 2>(x, nseg, stride, R, L, ndata, tabT, qi, qi_ld, dc, st, n_cu)
  if (no == 1) DFMI_WIDE(1);
  if (no == 2) DFMI_WIDE(2);
  DFMI_WIDE(4);
#undef DFMI_WIDE
}

// Geometry the LDS bin fold needs (bin kernels, seed kernels): 16-B rows, an even basis
// period 128 <= L <= 1024, and a basis + `nbins` bin sets that fit in LDS.
bool bins_geometry(bool vec2, int L, int ndata, size_t lds_cap, int nbins) {
  if (!vec2 || (L & 1) || L < 128 || L > 1024) return false;
  const size_t lds = ((size_t)2 * ndata * L + (size_t)nbins * L) * sizeof(double);
  return lds <= lds_cap && lds <= 64 * 1024;
}

bool bins_applicable(bool vec2, int L, int ndata, size_t lds_cap) {
  return t_tune.demod_kernel == 1 && bins_geometry(vec2, L, ndata, lds_cap, dfmi::kWavesPerBlock);
}

// Returns 1 if the bin kernel does not apply.
int try_bins(const double* x, int64_t nseg, int64_t stride, int R, int L, int ndata, const double* tab, double* qi,
             int64_t qi_ld, double* dc, hipStream_t st, int n_cu, bool vec2, size_t lds_cap, bool rows) {
  if (!bins_applicable(vec2, L, ndata, lds_cap)) return 1;
  const size_t lds = ((size_t)2 * ndata * L + (size_t)dfmi::kWavesPerBlock * L) * sizeof(double);
  const int nslot = (L + 127) / 128;
  if (rows) {
    if (nslot <= 2) return launch_bins_t<2, true>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds);
    if (nslot <= 4) return launch_bins_t<4, true>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds);
    return launch_bins_t<8, true>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds);
  }
  if (nslot <= 2) return launch_bins_t<2, false>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds);
  if (nslot <= 4) return launch_bins_t<4, false>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds);
  return launch_bins_t<8, false>(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, lds);
}

bool vec2_ok(const double* x, int64_t stride, int L) {
  return (L % 2 == 0) && (stride % 2 == 0) && (((uintptr_t)x & 15) == 0);
}

// Whether demod_device can write the row layout (dfmi_qi_row_stride) for this
// input: only the bin-in-LDS kernel implements it.
bool rows_supported(int dev, const double* x, int64_t stride, int R, int ndata, double w0, int period) {
  int L = period;
  if (L == 0) L = detect_period_impl(w0, R, ndata);
  if (L <= 0) return false;
  return bins_applicable(vec2_ok(x, stride, L), L, ndata, t_ds->lds_per_block);
}

// Device-pointer demodulation (all pointers on the current device).
// rows = true: write the row layout (qi + s·qi_ld, dfmi_qi_row_stride; dc inside
// the row, `dc` unused) — callers check rows_supported() first.
int demod_device(int dev, const double* x, int64_t nseg, int64_t stride, int R, int ndata, double w0, int period,
                 double* qi, int64_t qi_ld, double* dc, hipStream_t st, bool rows = false) {
  if (nseg == 0) return DFMI_OK;
  int L = period;
  if (L == 0) L = detect_period_impl(w0, R, ndata);
  const int n_cu = t_ds->n_cu;
  const size_t lds_cap = t_ds->lds_per_block;
  if (L > 0) {
    const bool vec2 = vec2_ok(x, stride, L);
    const int VEC = vec2 ? 2 : 1;
    int nslot = (L + 64 * VEC - 1) / (64 * VEC);
    if (nslot <= kMaxSlotCap) {
      int ms = 1;
      while (ms < nslot) ms <<= 1;
      const double* tab = nullptr;
      int rc = basis_table(dev, L, ndata, w0, st, &tab);
      if (rc) return rc;
      const size_t lds = (size_t)2 * ndata * L * sizeof(double);
      const bool use_lds = lds <= 64 * 1024 && lds <= lds_cap;
      if (!rows && wide_first(ndata, R) && wide_geometry(vec2, L, ndata))
        return launch_wide(dev, x, nseg, stride, R, L, ndata, w0, qi, qi_ld, dc, st, n_cu);
      rc = try_bins(x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu, vec2, lds_cap, rows);
      if (rc <= 0) return rc;
      if (rows) return fail(DFMI_ERR_UNSUPPORTED, "row layout needs the bin-in-LDS demodulation kernel");
      if (t_tune.demod_wide && t_tune.demod_kernel == 1 && wide_geometry(vec2, L, ndata))
        return launch_wide(dev, x, nseg, stride, R, L, ndata, w0, qi, qi_ld, dc, st, n_cu);
      if (vec2) {
        return use_lds ? launch_fold_ms<2, true>(ms, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu)
                       : launch_fold_ms<2, false>(ms, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
      }
      return use_lds ? launch_fold_ms<1, true>(ms, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu)
                     : launch_fold_ms<1, false>(ms, x, nseg, stride, R, L, ndata, tab, qi, qi_ld, dc, st, n_cu);
    }
  }
  if (rows) return fail(DFMI_ERR_UNSUPPORTED, "row layout needs the bin-in-LDS demodulation kernel");
  // direct kernel
  int64_t need = (nseg + dfmi::kWavesPerBlock - 1) / dfmi::kWavesPerBlock;
  int64_t grid = (int64_t)n_cu * 8;
  if (grid > need) grid = need;
  hipLaunchKernelGGL(dfmi::demod_direct_kernel, dim3((unsigned)grid), dim3(dfmi::kBlockThreads), 0, st, x, nseg,
                     stride, R, ndata, w0, qi, qi_ld, dc);
  HIPCHK(hipGetLastError());
  g_last_demod = "demod_direct_kernel";
  return DFMI_OK;
}

// LM kernel selection: the register path (ndata <= 16; the exact-ndata variant with QI
// in registers for the reference default ndata = 10) or the general path (any ndata,
// or lm_general = 1). CHAIN: warm-start chains (sequential / n_cores chunks).
// nd_sel: ndata, or 1000 for the literal general path (lm_general = 1); beyond 16 harmonics
// the many-harmonic path (lm.h kWideNd) on component-major QI, "lm_wide" = 0 the literal one.
template <bool CHAIN, bool ROWS>
auto lm_kernel(int nd_sel) {
  constexpr int kNd10 = dfmi::kExactNd | 10;
  const bool wide = nd_sel > 16 && nd_sel < 1000 && t_tune.lm_wide && !ROWS;
  if constexpr (CHAIN) {
    return nd_sel == 10   ? dfmi::lm_chunks_kernel<kNd10, true>
           : nd_sel <= 12 ? dfmi::lm_chunks_kernel<12, true>
           : nd_sel <= 16 ? dfmi::lm_chunks_kernel<16, true>
           : wide         ? dfmi::lm_chunks_kernel<dfmi::kWideNd, true>
                          : dfmi::lm_chunks_kernel<0, true>;
  } else {
    return nd_sel == 10   ? dfmi::lm_chunks_kernel<kNd10, false, ROWS, true>
           : nd_sel <= 12 ? dfmi::lm_chunks_kernel<12, false, ROWS>
           : nd_sel <= 16 ? dfmi::lm_chunks_kernel<16, false, ROWS>
           : wide && t_tune.lm_wide_fused ? dfmi::lm_chunks_kernel<dfmi::kWideNdF, false, false>
           : wide                         ? dfmi::lm_chunks_kernel<dfmi::kWideNd, false, false>
                                          : dfmi::lm_chunks_kernel<0, false, ROWS>;
  }
}

int lm_device(int dev, const double* qi, int64_t qi_ld, int ndata, int64_t nrec, int64_t nbuf, int64_t first,
              int64_t nitems, int64_t nchunk, const double* guess_dev, int64_t g_rec, int64_t g_comp,
              const double* guess_host /* nrec*4, used when nrec <= 8 and guess_dev == null */,
              const dfmi::LMConst& c, const double* jtab, double* out, int64_t out_ld, int32_t* status,
              hipStream_t st, bool rows = false) {
  (void)dev;
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
  const int64_t lanes = nrec * nchunk;
  const int block = 64;
  const int64_t grid = (lanes + block - 1) / block;
  const bool chain = nitems > nchunk;
  const int nd_sel = t_tune.lm_general ? 1000 : ndata;
  if (rows && chain) return fail(DFMI_ERR_ARG, "row layout: chunk size 1 only");
  // latency-bound launches (few chains or segments: at most ~2 ladder waves per SIMD):
  // the parallel lambda ladder, kLadderLanes lanes per item (lm.h lm_ladder_kernel)
  if (t_tune.lm_ladder && lanes <= (int64_t)t_tune.lm_ladder * t_ds->n_cu) {
    constexpr int kNd10 = dfmi::kExactNd | 10;
    using LK = void (*)(const double*, int64_t, int, int64_t, int64_t, int64_t, int64_t, int64_t, const double*,
                        int64_t, int64_t, dfmi::GuessInline, int, const double*, dfmi::LMConst, double*, int64_t,
                        int32_t*);
    LK lk;
    // beyond 16 harmonics the many-harmonic evaluation as in the one-lane kernels (same bits as
    // lm_chunks_kernel<kWideNd / kWideNdF>: the ladder only tries the rungs in parallel)
    const bool wide = nd_sel > 16 && nd_sel < 1000 && t_tune.lm_wide;
    if (rows)
      lk = nd_sel == 10 ? dfmi::lm_ladder_kernel<kNd10, false, true> : nd_sel <= 12 ? dfmi::lm_ladder_kernel<12, false, true>
           : nd_sel <= 16 ? dfmi::lm_ladder_kernel<16, false, true> : dfmi::lm_ladder_kernel<0, false, true>;
    else if (chain)
      lk = nd_sel == 10 ? dfmi::lm_ladder_kernel<kNd10, true, false> : nd_sel <= 12 ? dfmi::lm_ladder_kernel<12, true, false>
           : nd_sel <= 16 ? dfmi::lm_ladder_kernel<16, true, false>
           : wide && t_tune.lm_wide_fused ? dfmi::lm_ladder_kernel<dfmi::kWideNdF, true, false>
           : wide ? dfmi::lm_ladder_kernel<dfmi::kWideNd, true, false> : dfmi::lm_ladder_kernel<0, true, false>;
    else
      lk = nd_sel == 10 ? dfmi::lm_ladder_kernel<kNd10, false, false> : nd_sel <= 12 ? dfmi::lm_ladder_kernel<12, false, false>
           : nd_sel <= 16 ? dfmi::lm_ladder_kernel<16, false, false>
           : wide && t_tune.lm_wide_fused ? dfmi::lm_ladder_kernel<dfmi::kWideNdF, false, false>
           : wide ? dfmi::lm_ladder_kernel<dfmi::kWideNd, false, false> : dfmi::lm_ladder_kernel<0, false, false>;
    // beyond 16 harmonics, while at most lm_ladder_split x CUs items: one wave per item, its 64
    // lanes 8 rungs x 8 harmonic shares (lm.h PartFullEval, as the seed)
    const bool wsplit = !rows && wide && t_tune.lm_wide_fused && t_tune.lm_ladder_split &&
                        lanes <= (int64_t)t_tune.lm_ladder_split * t_ds->n_cu;
    if (wsplit) lk = chain ? dfmi::lm_ladder_kernel<dfmi::kWideNdF, true, false, 64>
                           : dfmi::lm_ladder_kernel<dfmi::kWideNdF, false, false, 64>;
    const int64_t lgrid = (lanes * (wsplit ? 64 : dfmi::kLadderLanes) + block - 1) / block;
    hipLaunchKernelGGL(lk, dim3((unsigned)lgrid), dim3(block), 0, st, qi, qi_ld, ndata, nrec, nbuf, first, nitems,
                       nchunk, guess_dev, g_rec, g_comp, ginl, use_inline, jtab, c, out, out_ld, status);
    HIPCHK(hipGetLastError());
    return DFMI_OK;
  }
  size_t lds = 0;
  auto kern = chain ? lm_kernel<true, false>(nd_sel) : rows ? lm_kernel<false, true>(nd_sel)
                                                            : lm_kernel<false, false>(nd_sel);
  if (rows && nd_sel <= 16) lds = (size_t)qi_ld * 65 * sizeof(double);  // the wave's rows, transposed
  // the general path's one-pass Bessel walk: the lane's recurrence values in LDS, while 7
  // waves per CU still fit (ndata + 2 <= 45): ndata 40 0.276 -> 0.264 ms per 100k; at 62 (5
  // waves per CU) 0.384 -> 0.663, r05ax
  // many harmonics, P lanes per segment (lm.h lm_split_kernel: QI in a per-wave LDS tile of
  // 64 / P segments) from "lm_split_from" harmonics on ("lm_split" = P, 0 = never)
  const int sp = t_tune.lm_split;
  if (!chain && !rows && nd_sel > 16 && nd_sel < 1000 && t_tune.lm_wide && sp > 1 && ndata >= t_tune.lm_split_from &&
      (size_t)2 * ndata * (64 / sp) * sizeof(double) <= t_ds->lds_per_block) {
    const size_t slds = (size_t)2 * ndata * (64 / sp) * sizeof(double);
    const int64_t sgrid = (nrec * nitems + 64 / sp - 1) / (64 / sp);
    auto sk = sp == 4 ? dfmi::lm_split_kernel<4> : dfmi::lm_split_kernel<2>;
    hipLaunchKernelGGL(sk, dim3((unsigned)sgrid), dim3(64), slds, st, qi, qi_ld, ndata, nrec, nbuf, first, nitems,
                       guess_dev, g_rec, g_comp, ginl, use_inline, jtab, c, out, out_ld, status);
    HIPCHK(hipGetLastError());
    return DFMI_OK;
  }
  // many harmonics with QI staged in LDS per lane (lm.h QLds) while 2 ndata x 64 x 8 B per wave
  // leaves 8 waves per CU ("lm_wide_lds": the largest ndata staged, default 20 = 20 KB)
  if (!chain && !rows && nd_sel > 16 && nd_sel < 1000 && t_tune.lm_wide && ndata <= t_tune.lm_wide_lds &&
      (size_t)2 * ndata * 64 * sizeof(double) <= t_ds->lds_per_block) {
    // (split trials here: the one-walk form measured slower with the QI in LDS, 0.078 against
    // 0.073 ms at ndata 20, profiles/r06/ndata_sweep_fused.jsonl)
    kern = dfmi::lm_chunks_kernel<dfmi::kWideNd, false, false, true>;
    lds = (size_t)2 * ndata * 64 * sizeof(double);
  }
  if (!chain && !rows && nd_sel > 16 && !(t_tune.lm_wide && nd_sel < 1000) && t_tune.lm_onepass &&
      (t_tune.lm_onepass == 2 || (size_t)64 * (ndata + 2) * 8 * 7 <= t_ds->lds_per_block)) {
    kern = dfmi::lm_chunks_kernel<0, false, false, false, true>;
    lds = (size_t)64 * (ndata + 2) * sizeof(double);
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(block), lds, st, qi, qi_ld, ndata, nrec, nbuf, first, nitems,
                     nchunk, guess_dev, g_rec, g_comp, ginl, use_inline, jtab, c, out, out_ld, status);
  HIPCHK(hipGetLastError());
  return DFMI_OK;
}

// Whole record pipeline on device pointers (fitters.py:370-428).
// Fused seed + bulk demodulation (seed.h demod_seed_bins_kernel) on one stream.
// Returns 1 when it does not apply (caller uses the two-kernel path).
int fused_seed_demod(int dev, const double* x, int64_t nrec, int64_t nbuf, int R, int ndata, int L,
                     const double* tab, double* rows, int64_t qs, const double* gdev, const dfmi::GuessInline& ginl,
                     const double* jtab, const dfmi::LMConst& c, double* out, int64_t out_ld, int32_t* fitok,
                     hipStream_t st) {
  if (ndata > 16 || L <= 0) return 1;
  const int nslot = (L + 127) / 128;
  if (nslot > 8) return 1;
  using K = void (*)(const double*, int64_t, int64_t, int64_t, int, int, int, const double*, double*, int64_t,
                     const double*, dfmi::GuessInline, int, const double*, dfmi::LMConst, double*, int64_t, int64_t,
                     int32_t*, uint64_t*);
  const bool pf = nslot <= 2 && ndata <= 12;  // bins_segment's prefetch (bulk path, MS 2)
  K kern;
  const size_t lds = ((size_t)2 * ndata * L + (size_t)dfmi::kWavesPerBlock * L) * sizeof(double) +
                     (nslot <= 2 && ndata <= 12 ? DFMI_BINS_LDS_PAD : 0);
  if (ndata <= 12)
    kern = nslot <= 2 ? dfmi::demod_seed_bins_kernel<2, 12, DFMI_BINS_PFN, DFMI_BINS_LOADS>
           : nslot <= 4 ? dfmi::demod_seed_bins_kernel<4, 12>
                                                                          : dfmi::demod_seed_bins_kernel<8, 12>;
  else
    kern = nslot <= 2 ? dfmi::demod_seed_bins_kernel<2, 16> : nslot <= 4 ? dfmi::demod_seed_bins_kernel<4, 16>
                                                                       : dfmi::demod_seed_bins_kernel<8, 16>;
  int per_cu = 0;
  if (int orc = occupancy(kern, dfmi::kBlockThreads, lds, &per_cu)) return orc;
  if (per_cu < 1) per_cu = 1;
  const int64_t slots = (int64_t)t_ds->n_cu * per_cu;
  const int64_t nseg = nrec * nbuf;
  if (nrec + 1 > slots / 2) return 1;  // every seed and most of the bulk must be resident at once
  int64_t bulk = slots - nrec;
  const int64_t need = (nseg + dfmi::kWavesPerBlock - 1) / dfmi::kWavesPerBlock;
  if (bulk > need) bulk = need;
  if (t_tune.demod_spw > 0) {  // as bins_grid: later workgroups to the slots that free first
    const int64_t per = (int64_t)dfmi::kWavesPerBlock * t_tune.demod_spw;
    if ((nseg + per - 1) / per > bulk) bulk = (nseg + per - 1) / per;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(nrec + bulk)), dim3(dfmi::kBlockThreads), lds, st, x, nseg,
                     nbuf * (int64_t)R, nrec, R, L, ndata, tab, rows, qs, gdev, ginl, gdev ? 0 : 1, jtab, c, out,
                     out_ld, nbuf, fitok, t_ds->probe);
  HIPCHK(hipGetLastError());
  // the template arguments of the instance launched (loads in flight / prefetched chunks
  // from the build's macros, so A/B builds report their own geometry)
  const bool geo = nslot <= 2 && ndata <= 12;
  g_last_demod = "demod_seed_bins_kernel<" + std::to_string(nslot <= 2 ? 2 : nslot <= 4 ? 4 : 8) + "," +
                 std::to_string(ndata <= 12 ? 12 : 16) + "," + std::to_string(geo ? DFMI_BINS_PFN : 0) + "," +
                 std::to_string(geo ? DFMI_BINS_LOADS : 8) + ">" +
                 (pf && (R >> 7) >= DFMI_BINS_PFN ? " (prefetch " + std::to_string(DFMI_BINS_PFN) + ")" : "");
  return DFMI_OK;
}

// Seed step of the unfused layouts (fitters.py:403-410): buffer 0 of every record
// demodulated and fitted by one wave per record on the side stream, concurrently with
// the bulk demodulation on the caller's stream; the LM waits on its event. The LDS bin
// fold (seed_bins_kernel) wherever its geometry applies — the fused kernel's seed fold,
// so both paths give the same bits — the global fold / direct kernel otherwise.
int seed_launch(int dev, const double* x, int64_t nrec, int64_t rec_stride, int R, int ndata, double w0, int L,
                const double* gdev, const dfmi::GuessInline& ginl, const double* jtab, const dfmi::LMConst& c,
                double* out, int64_t out_ld, int64_t nbuf, int32_t* fitok, hipStream_t sst, bool seed_dc) {
  int rc;
  if (L > 64 * 16) L = 0;  // no table: the direct kernel's per-sample sincos
  const double* tab = nullptr;
  if (L > 0 && (rc = basis_table(dev, L, ndata, w0, sst, &tab))) return rc;
  const bool vec2 = L > 0 && vec2_ok(x, nrec > 1 ? rec_stride : 0, L);
  const size_t blds = ((size_t)2 * ndata * L + L + dfmi_row_stride(ndata)) * sizeof(double);
  if (L > 0 && bins_geometry(vec2, L, ndata, t_ds->lds_per_block, 1) && blds <= t_ds->lds_per_block) {
    const int nslot = (L + 127) / 128;
    auto sk = ndata <= 12 ? (nslot <= 2 ? dfmi::seed_bins_kernel<12, 2> : nslot <= 4 ? dfmi::seed_bins_kernel<12, 4>
                                                                                   : dfmi::seed_bins_kernel<12, 8>)
            : ndata <= 16 ? (nslot <= 2 ? dfmi::seed_bins_kernel<16, 2> : nslot <= 4 ? dfmi::seed_bins_kernel<16, 4>
                                                                                   : dfmi::seed_bins_kernel<16, 8>)
                          : (nslot <= 2 ? dfmi::seed_bins_kernel<0, 2> : nslot <= 4 ? dfmi::seed_bins_kernel<0, 4>
                                                                                  : dfmi::seed_bins_kernel<0, 8>);
    hipLaunchKernelGGL(sk, dim3((unsigned)nrec), dim3(64), blds, sst, x, rec_stride, R, L, ndata, tab, gdev, ginl,
                       gdev ? 0 : 1, jtab, c, out, out_ld, nbuf, fitok, t_ds->probe, seed_dc ? 1 : 0);
  } else {
    void *qs, *ds_;
    if ((rc = workspace(dev, "qi_seed", (size_t)2 * ndata * nrec * 8, &qs))) return rc;
    if ((rc = workspace(dev, "dc_seed", (size_t)nrec * 8, &ds_))) return rc;
    auto sk = ndata <= 12 ? dfmi::seed_kernel<12> : ndata <= 16 ? dfmi::seed_kernel<16>
              : t_tune.lm_wide ? (t_tune.seed_wave_split ? dfmi::seed_kernel<dfmi::kWideNdF, 3>
                                  : t_tune.lm_wide_fused ? dfmi::seed_kernel<dfmi::kWideNdF>
                                                         : dfmi::seed_kernel<dfmi::kWideNd>)
                               : dfmi::seed_kernel<0>;
    // the many-harmonic demodulation where its geometry holds (16-B rows, 128 <= L <= 256):
    // the bulk's own QI for buffer 0, and a fold with 10 wave loads in flight instead of the
    // cycle-aligned scalar fold against a global basis
    const double* tabT = nullptr;
    int no = 0;
    if (L > 0 && wide_geometry(vec2, L, ndata)) {
      no = wide_no(ndata);
      if ((rc = basis_table_wide(dev, L, ndata, w0, no, &tabT))) return rc;
    }
    const size_t lds = tabT ? (size_t)(L + 4) * sizeof(double) : 0;
    hipLaunchKernelGGL(sk, dim3((unsigned)nrec), dim3(64), lds, sst, x, rec_stride, R, L, ndata, w0, tab,
                       (double*)qs, (double*)ds_, nrec, gdev, ginl, gdev ? 0 : 1, jtab, c, out, out_ld, nbuf, fitok,
                       tabT, no);
  }
  HIPCHK(hipGetLastError());
  return DFMI_OK;
}

int nls_record_device(int dev, const double* x, int64_t nrec, int64_t rec_stride, int64_t nbuf, int R, int ndata,
                      double w0, int period, const double* init_guess_host, int parallel, int64_t nchunk,
                      const dfmi_lm_config& cfg, const dfmi::LMConst& c, double* out, int32_t* fitok,
                      hipStream_t st) {
  const int64_t nseg = nrec * nbuf;
  if (nseg == 0) return DFMI_OK;
  DeviceState& ds = *t_ds;
  const double* jtab = nullptr;
  int rc = grid_table(dev, ndata, cfg, &jtab);
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

  // Row layout (one 128-B line per 8 harmonics, dc inside the row: full-line
  // stores) for the chunk-size-1 parallel path when the bin kernel applies and
  // demod_wide_kernel does not go ahead of it (wide_first); component-major QI
  // otherwise (warm-start chains read QI component-major).
  int L = period;
  if (L == 0) L = detect_period_impl(w0, R, ndata);
  const bool even_recs = nrec == 1 || (rec_stride % 2) == 0;
  const bool wide = L > 0 && even_recs && wide_first(ndata, R) && wide_geometry(vec2_ok(x, R, L), L, ndata);
  const bool rows = parallel && (nbuf <= 1 || nchunk >= nbuf - 1) && even_recs && !wide &&
                    rows_supported(dev, x, R, R, ndata, w0, period);
  const int64_t qs = rows ? dfmi_row_stride(ndata) : 0;
  if (parallel && rows && (nrec == 1 || rec_stride == nbuf * (int64_t)R) && nbuf > 1) {
    // ONE launch: the seeds (buffer 0 of every record) + the bulk demodulation; the LM
    // follows in stream order
    const double* tab = nullptr;
    if ((rc = basis_table(dev, L, ndata, w0, st, &tab))) return rc;
    void* rw = nullptr;
    if ((rc = workspace(dev, "qrow", (size_t)qs * nseg * sizeof(double), &rw))) return rc;
    StepMarks sm;
    if ((rc = sm.begin(ds)) || (rc = sm.mark(0, st))) return rc;
    rc = fused_seed_demod(dev, x, nrec, nbuf, R, ndata, L, tab, (double*)rw, qs, gdev, ginl, jtab, c, out, out_ld,
                          fitok, st);
    if (rc < 0) return rc;
    if (rc == 0) {
      if ((rc = sm.mark(1, st))) return rc;
      rc = lm_device(dev, (double*)rw, qs, ndata, nrec, nbuf, 1, nbuf - 1, nchunk, out, nbuf, out_ld, nullptr, c,
                     jtab, out, out_ld, fitok, st, true);
      if (rc) return rc;
      if ((rc = sm.mark(2, st))) return rc;
      sm.commit();
      return DFMI_OK;
    }
    // not fused after all: no marks for this call (sm hands its events back)
  }
  if (parallel) {  // the seed beside the bulk demodulation (side stream, event)
    HIPCHK(hipEventRecord(ds.ev_in, st));
    HIPCHK(hipStreamWaitEvent(ds.side, ds.ev_in, 0));
    // buffer 0's dc: the bulk demodulation writes it on the component-major path (beside the
    // seed, unordered: one writer only); on the row path the LM skips buffer 0, so the seed does
    if ((rc = seed_launch(dev, x, nrec, rec_stride, R, ndata, w0, L, gdev, ginl, jtab, c, out, out_ld, nbuf, fitok,
                          ds.side, rows)))
      return rc;
    HIPCHK(hipEventRecord(ds.ev_seed, ds.side));
  }
  double* qi = nullptr;
  {
    void* w = nullptr;
    if (rows) rc = workspace(dev, "qrow", (size_t)qs * nseg * sizeof(double), &w);
    else rc = workspace(dev, "qi", (size_t)2 * ndata * nseg * sizeof(double), &w);
    if (rc) return rc;
    qi = (double*)w;
  }
  if (rec_stride == nbuf * (int64_t)R || nrec == 1) {
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
  if (rc) return rc;
  if (!parallel) {
    return lm_device(dev, qi, nseg, ndata, nrec, nbuf, 0, nbuf, 1, gdev, 4, 1, init_guess_host, c, jtab, out, out_ld,
                     fitok, st);
  }
  HIPCHK(hipStreamWaitEvent(st, ds.ev_seed, 0));
  if (nbuf <= 1) {
    if (rows)  // dc of the seed buffers (the LM kernel carries it otherwise)
      HIPCHK(hipMemcpy2DAsync(dc, nbuf * sizeof(double), qi + dfmi_row_dc(ndata), qs * nbuf * sizeof(double),
                              sizeof(double), nrec, hipMemcpyDeviceToDevice, st));
    return DFMI_OK;
  }
  // the rest, seeded with each record's buffer-0 result (read on device: no host sync)
  return lm_device(dev, qi, rows ? qs : nseg, ndata, nrec, nbuf, 1, nbuf - 1, nchunk, out, nbuf, out_ld, nullptr, c,
                   jtab, out, out_ld, fitok, st, rows);
}

}  // namespace

namespace {
// key -> (knob, allowed values or empty = any value >= 0)
struct Knob {
  int Tuning::*v;
  std::vector<int> allowed;
};
const std::map<std::string, Knob>& knobs() {
  static const std::map<std::string, Knob> k = {
      {"demod_kernel", {&Tuning::demod_kernel, {0, 1}}},
      {"lm_general", {&Tuning::lm_general, {0, 1}}},
      {"demod_spw", {&Tuning::demod_spw, {}}},
      {"demod_wide", {&Tuning::demod_wide, {0, 1, 2}}},
      {"demod_wide_k", {&Tuning::demod_wide_k, {0, 2, 4, 8}}},
      {"demod_wide_from", {&Tuning::demod_wide_from, {}}},
      {"demod_wide_rmax", {&Tuning::demod_wide_rmax, {}}},
      {"lm_onepass", {&Tuning::lm_onepass, {0, 1, 2}}},
      {"lm_wide", {&Tuning::lm_wide, {0, 1}}},
      {"lm_wide_lds", {&Tuning::lm_wide_lds, {}}},
      {"lm_wide_fused", {&Tuning::lm_wide_fused, {0, 1}}},
      {"seed_wave_split", {&Tuning::seed_wave_split, {0, 1}}},
      {"lm_ladder_split", {&Tuning::lm_ladder_split, {}}},
      {"lm_split", {&Tuning::lm_split, {0, 2, 4}}},
      {"lm_split_from", {&Tuning::lm_split_from, {}}},
      {"demod_wide_half", {&Tuning::demod_wide_half, {0, 1}}},
      {"demod_wide_dbg", {&Tuning::demod_wide_dbg, {0, 1, 2, 3, 4, 5, 6, 7}}},
      {"ekf_row", {&Tuning::ekf_row, {}}},
      {"ekf_rot", {&Tuning::ekf_rot, {0, 1}}},
      {"wdfmi_accel", {&Tuning::wdfmi_accel, {0, 1, 2, 3}}},
      {"lm_ladder", {&Tuning::lm_ladder, {}}},
      {"ws_streams", {&Tuning::ws_streams, {}}},
      {"ekf_pit", {&Tuning::ekf_pit, {}}},
      {"ekf_pit_min", {&Tuning::ekf_pit_min, {}}},
      {"ekf_pit_block", {&Tuning::ekf_pit_block, {}}},
      {"ekf_pit_passes", {&Tuning::ekf_pit_passes, {}}},
      {"ekf_pit_first", {&Tuning::ekf_pit_first, {}}},
      {"ekf_pit_every", {&Tuning::ekf_pit_every, {}}},
      {"ekf_pit_topfix", {&Tuning::ekf_pit_topfix, {0, 1}}},
      {"ekf_pit_tol", {&Tuning::ekf_pit_tol, {}}},
      {"ekf_pit_stall", {&Tuning::ekf_pit_stall, {}}},
      {"ekf_pit_slow_from", {&Tuning::ekf_pit_slow_from, {}}},
      {"ekf_pit_overlap", {&Tuning::ekf_pit_overlap, {0, 1, 2, 3}}},
      {"ekf_pit_trace", {&Tuning::ekf_pit_trace, {0, 1}}},
      {"ekf_pit_seq", {&Tuning::ekf_pit_seq, {0, 1}}},
      {"ekf_pit_measure", {&Tuning::ekf_pit_measure, {0, 1}}},
      {"ekf_pit_head", {&Tuning::ekf_pit_head, {}}},
      {"ekf_pit_fused", {&Tuning::ekf_pit_fused, {0, 1}}}};
  return k;
}
// np.mean / np.var of nrec device records on st (moments.hip), numpy-exact.
int moments_dev(int dev, const double* dx, int64_t nrec, int64_t rs, int64_t n, double* mean, int64_t mean_stride,
                double* var, int64_t var_stride, hipStream_t st) {
  const int* plan;
  int64_t nl;
  int rc = pairwise_plan(dev, n, &plan, &nl);
  if (rc) return rc;
  void* nodes;
  if ((rc = workspace(dev, "m_nodes", (size_t)nrec * 2 * nl * 8, &nodes))) return rc;
  HIPCHK(dfmi::moments_launch(dx, nrec, rs, n, plan, nl, (double*)nodes, mean, mean_stride, var, var_stride, st));
  return DFMI_OK;
}

// Pass counts (and, with ekf_pit_trace, every pass's move) of the last EKF call on this
// thread, copied to the host at the end of that call: dfmi_ekf_pit_passes /
// dfmi_ekf_pit_trace read these, never a device workspace.
thread_local std::vector<int32_t> g_pit_passes;
thread_local std::vector<double> g_pit_hist;
thread_local int g_pit_hist_n = 0;
constexpr int kPitNoMem = 1;  // ekf_pit_run: a workspace could not be allocated (nothing launched)
// Hand-over streams of ekf_pit_overlap 3: successive hand-overs run concurrently on up to this many
// streams (a process has GPU_MAX_HW_QUEUES = 4 hardware queues by default, the caller's stream holds
// one). A sequential re-run lasts as long as the record whatever its channel count (63 ms for the
// 1,024-channel bench batch), so every extra launch costs that again: the batch took 143 ms with one
// launch after the 80 ms of passes (mode 0, the default), 194 ms over this pool (mode 3) and 432 ms
// queued in one stream (modes 1 and 2), profiles/r06/ekf_handover_probe.jsonl
constexpr int kEkfPool = 3;

// Pinned host scratch of the current device (grow-only).
int pinned(size_t bytes, void** out) {
  DeviceState& ds = *t_ds;
  if (ds.pin_n < bytes) {
    if (ds.pin) HIPCHK(hipHostFree(ds.pin));
    ds.pin = nullptr;
    ds.pin_n = 0;
    HIPCHK(hipHostMalloc(&ds.pin, bytes, hipHostMallocDefault));
    ds.pin_n = bytes;
  }
  *out = ds.pin;
  return DFMI_OK;
}

// The sequential EKF kernels over nrec channels (device pointers): few channels one 16-lane
// row each (ekf_rot_kernel with sin / cos by rotation between anchors when R % 4 == 0, else
// ekf_row_kernel, ~1.7x the per-channel rate), many one lane each (ekf_lane_rot_kernel /
// ekf_kernel, 16x the channels per instruction). Returns the variant's name in *name.
int ekf_seq_launch(const double* dx, int64_t nrec, int64_t rs, int64_t n, const double* dx0, const double* dp0,
                   const double* dq, const double* dr, const double* wt, int32_t R, int64_t nbuf, double* dstates,
                   hipStream_t st, const char** name, const int* idx = nullptr) {
  const int block = 64;
  const bool row = t_tune.ekf_row && nrec <= (int64_t)t_tune.ekf_row * t_ds->n_cu * 16;
  const int64_t grid = row ? (nrec + 3) / 4 : (nrec + block - 1) / block;
  // rotation between anchors: groups of 16 (8, 4) samples whose ends carry the snapshots
  const bool rot = t_tune.ekf_rot && R % 4 == 0;
  using EK = void (*)(const double*, int64_t, int64_t, int64_t, const double*, const double*, const double*,
                      const double*, const double*, int, int64_t, double*, DfmiTrigK, const int*);
  EK ek;
  if (row)
    ek = !rot ? dfmi::ekf_row_kernel<DFMI_EKF_SPLIT != 0>
         : R % DFMI_EKF_ROT_G == 0 ? dfmi::ekf_rot_kernel<DFMI_EKF_ROT_G>
         : R % 8 == 0              ? dfmi::ekf_rot_kernel<8>
                                   : dfmi::ekf_rot_kernel<4>;
  else
    ek = !rot ? dfmi::ekf_kernel : R % 8 == 0 ? dfmi::ekf_lane_rot_kernel<8> : dfmi::ekf_lane_rot_kernel<4>;
  hipLaunchKernelGGL(ek, dim3((unsigned)grid), dim3(block), 0, st, dx, nrec, rs, n, dx0, dp0, dq, dr, wt, (int)R, nbuf,
                     dstates, dfmi_trig_k(), idx);
  HIPCHK(hipGetLastError());
  *name = row ? (rot ? "ekf_rot_kernel" : "ekf_row_kernel") : (rot ? "ekf_lane_rot_kernel" : "ekf_kernel");
  return DFMI_OK;
}

// The EKF parallel in time (ekf_pit.h) for nrec long channels: head, gather, the first
// aggregates and their scan, then passes (pass kernel + scan hierarchy), a converged
// channel's kernels returning at once. The host reads the number of channels still passing
// after ekf_pit_first passes and then every ekf_pit_every (one stream sync each) and stops at
// zero or at the cap ekf_pit_passes; the channels that stopped contracting or hit the cap are
// re-run by the sequential kernel. wt: ekf_phase_kernel's table (the sequential kernel's).
// Returns kPitNoMem, with nothing launched, when a workspace cannot be allocated.
int ekf_pit_run(int dev, const double* dx, int64_t nrec, int64_t rs, int64_t n, const double* dx0, const double* dp0,
                const double* dq, const double* dr, const double* wt, double w_m, double f_samp, int32_t R,
                int64_t nbuf, double* dstates, hipStream_t st) {
  // samples per block: the measured best keeps ~16k x nrec^(1/3) blocks in flight over all
  // channels (1 channel: B = 25 at 400k samples; 4: 64; 16: 128; 64: 512; 256: 1024,
  // profiles/r04w..y): one channel is latency-bound (many short blocks), many channels fill
  // the GPU anyway and fewer, longer blocks cut the scan's work
  int64_t B = t_tune.ekf_pit_block;
  if (B <= 0) B = (int64_t)std::ceil((double)n * std::pow((double)nrec, 2.0 / 3.0) / 16384.0);
  if (B < 16) B = 16;
  const int64_t nb = (n + B - 1) / B, slots = B * nb;
  // the scan hierarchy: level 0 = the block aggregates, level l+1 = the workgroup totals of
  // level l, up to the first level that fits one workgroup
  std::vector<int64_t> lsz = {nb};
  while (lsz.back() > dfmi::kPitWg) lsz.push_back((lsz.back() + dfmi::kPitWg - 1) / dfmi::kPitWg);
  const int L = (int)lsz.size() - 1;
  const int64_t T0 = std::min<int64_t>(std::max(t_tune.ekf_pit_head, 0), n);
  const int cap = t_tune.ekf_pit_passes > 0 ? t_tune.ekf_pit_passes
                                            : (int)std::min<int64_t>(256, std::max<int64_t>(48, n / 1600));
  const int hist_n = t_tune.ekf_pit_trace ? cap : 0;
  void *xt, *wtt, *xbar, *conv, *chan, *hst, *done, *hs, *ent = nullptr, *hist = nullptr, *pin;
  void *sidx = nullptr, *handed = nullptr;
  std::vector<double*> lv[2];  // per aggregate buffer: level arrays [r][65][lsz[l]]
  // every allocation before the first launch: a failure leaves the sequential kernels to run
  {
    int rc = 0;
    auto ws = [&](const char* name, size_t bytes, void** p) {
      if (!rc) rc = workspace(dev, name, bytes, p);
    };
    ws("p_xt", (size_t)(nrec * slots) * 8, &xt);
    ws("p_wt", (size_t)slots * 8, &wtt);
    xbar = nullptr;  // the unfused path's trajectory; the fused first pass reads the head directly
    if (!t_tune.ekf_pit_fused) ws("p_xbar", (size_t)(nrec * 5 * slots) * 8, &xbar);
    for (int bf = 0; bf < 2 && !rc; ++bf)
      for (int l = 0; l <= L && !rc; ++l) {
        void* a = nullptr;
        const std::string name = "p_lv" + std::to_string(bf) + "_" + std::to_string(l);
        ws(name.c_str(), (size_t)(nrec * dfmi::kPitEl * lsz[l]) * 8, &a);
        lv[bf].push_back((double*)a);
      }
    ws("p_conv", (size_t)nrec * 8, &conv);
    ws("p_chan", (size_t)nrec * sizeof(dfmi::PitChan), &chan);
    ws("p_hst", (size_t)(nrec * 5) * 8, &hst);
    ws("p_done", (size_t)nrec * sizeof(unsigned), &done);
    ws("p_hs", (size_t)(nrec * (T0 > 0 ? T0 : 1) * 5) * 8, &hs);
    if (t_tune.ekf_pit_fused && t_tune.ekf_pit_measure == 1) ws("p_ent", (size_t)(nrec * 5 * nb) * 8, &ent);
    if (hist_n) ws("p_hist", (size_t)nrec * hist_n * 8, &hist);
    if (t_tune.ekf_pit_seq) {  // the hand-over list (sequential re-runs read the records in place)
      ws("p_sidx", (size_t)nrec * sizeof(int), &sidx);
      ws("p_handed", (size_t)nrec * sizeof(unsigned), &handed);
    }
    if (!rc) rc = pinned((size_t)nrec * sizeof(dfmi::PitChan) + 64, &pin);
    if (rc) {
      (void)hipGetLastError();  // clear the failed allocation
      g_err.clear();
      return kPitNoMem;
    }
  }
  dfmi::PitChan* ch = (dfmi::PitChan*)chan;
  const DfmiTrigK tk = dfmi_trig_k();
  const unsigned nr = (unsigned)nrec;
  dfmi::PitRule rule;
  rule.tol = std::pow(10.0, -(double)t_tune.ekf_pit_tol);
  rule.noise = rule.tol;
  rule.stall_max = std::max(t_tune.ekf_pit_stall, 1);
  rule.cap = cap;
  rule.slow_from = t_tune.ekf_pit_slow_from;
  rule.hist_n = hist_n;
  rule.measure = t_tune.ekf_pit_measure;
  if (hist_n) HIPCHK(hipMemsetAsync(hist, 0xFF, (size_t)nrec * hist_n * 8, st));  // NaN: pass not run
  hipLaunchKernelGGL(dfmi::ekf_pit_head_kernel, dim3((unsigned)((nrec + 3) / 4)), dim3(64), 0, st, dx, nrec, rs, T0,
                     dx0, dp0, dq, dr, wt, (double*)hs, (double*)hst, tk);
  if (xbar)  // the unfused path: the trajectory buffer too
    hipLaunchKernelGGL(dfmi::ekf_pit_gather_kernel, dim3((unsigned)((slots + 255) / 256), nr), dim3(256), 0, st, dx,
                       rs, n, (const double*)hs, (const double*)hst, T0, B, nb, w_m, f_samp, (double*)xt,
                       (double*)wtt, (double*)xbar, ch, (double*)conv, (unsigned*)done);
  else
    hipLaunchKernelGGL(dfmi::ekf_pit_gather_tiled_kernel, dim3((unsigned)((B + 31) / 32), (unsigned)((nb + 63) / 64), nr),
                       dim3(256), 0, st, dx, rs, n, B, nb, w_m, f_samp, (double*)xt, (double*)wtt, ch,
                       (double*)conv, (unsigned*)done);
  const dim3 lanes((unsigned)((nb + 63) / 64), nr);
  // scan of one buffer's hierarchy: every level bottom-up, then the fix-ups top-down; the
  // pass kernels read level 0 (prefixes within workgroups) and level 1 (true prefixes)
  // (ekf_pit_topfix: a top level of at most 4 elements above level 1 is not scanned; the
  // fix-up of the level below folds its prefix itself, ekf_pit_fixup_top_kernel)
  const bool topfix = t_tune.ekf_pit_topfix && L >= 2 && lsz[L] <= 4;
  auto scan = [&](std::vector<double*>& a) {
    for (int l = 0; l <= L - (topfix ? 1 : 0); ++l)
      hipLaunchKernelGGL(dfmi::ekf_pit_scan_kernel<dfmi::kPitWg>,
                         dim3((unsigned)((lsz[l] + dfmi::kPitWg - 1) / dfmi::kPitWg), nr), dim3(4 * dfmi::kPitWg), 0,
                         st, a[l], lsz[l], lsz[l], l < L ? a[l + 1] : nullptr, (const dfmi::PitChan*)ch);
    for (int l = L - 1; l >= 1; --l)
      if (lsz[l] > dfmi::kPitWg)
        hipLaunchKernelGGL(topfix && l == L - 1 ? dfmi::ekf_pit_fixup_top_kernel : dfmi::ekf_pit_fixup_kernel,
                           dim3((unsigned)((lsz[l] - dfmi::kPitWg + 63) / 64), nr), dim3(64), 0, st, a[l], lsz[l],
                           (const double*)a[l + 1], lsz[l + 1], (const dfmi::PitChan*)ch);
  };
  const double* tops[2] = {L >= 1 ? lv[0][1] : nullptr, L >= 1 ? lv[1][1] : nullptr};
  const int every = std::max(t_tune.ekf_pit_every, 1);
  int next_check = std::min(std::max(t_tune.ekf_pit_first, 1), cap);
  if (t_tune.ekf_pit_fused) {
    // first aggregates at the seeded trajectory, then per pass: EKF + fold (ekf_pit_pass_kernel,
    // aggregates into the other buffer, the stop rule by its last workgroup per channel), scan
    // of the new aggregates
    if (ent) HIPCHK(hipMemsetAsync(ent, 0xFF, (size_t)(nrec * 5 * nb) * 8, st));  // NaN: no previous entry
    hipLaunchKernelGGL(dfmi::ekf_pit_aggregate_kernel, lanes, dim3(64), 0, st, (const double*)xt, (const double*)wtt,
                       (const double*)nullptr, n, B, nb, dx0, dp0, dq, dr, (const dfmi::PitChan*)ch, lv[0][0], tk,
                       (const double*)hs, (const double*)hst, T0);
    scan(lv[0]);
  }
  // Hand-over: channels the stop rule gave up on (status 2; at the end every channel not
  // converged) are re-run by the sequential kernel as soon as a host check sees them, on the
  // device's hand-over stream beside the passes the other channels still run (a pass kernel
  // returns at once for a channel whose status is set, so the two never write the same
  // states). The list is built on the device (ekf_pit_handover_kernel); the host only counts.
  std::vector<char> host_handed((size_t)nrec, 0);
  int64_t nh = 0;
  bool side_used = false;
  hipStream_t side_stream = nullptr;
  int n_batches = 0;                     // hand-over launches so far
  hipStream_t used_streams[kEkfPool] = {};  // the streams they went to (pool mode)
  std::string seq_name;
  if (handed) HIPCHK(hipMemsetAsync(handed, 0, (size_t)nrec * sizeof(unsigned), st));
  const int overlap = t_tune.ekf_pit_overlap;
  auto hand_over = [&](const dfmi::PitChan* hc, bool final_) -> int {
    if (!t_tune.ekf_pit_seq) return DFMI_OK;
    if (!overlap && !final_) return DFMI_OK;  // ekf_pit_overlap 0: every re-run after the passes, on st
    int64_t cnt = 0;
    for (int64_t r = 0; r < nrec; ++r)
      if (!host_handed[r] && (hc[r].status == 2 || (final_ && hc[r].status != 1))) {
        host_handed[r] = 1;
        ++cnt;
      }
    if (cnt == 0) return DFMI_OK;
    DeviceState& d = *t_ds;
    hipStream_t side = st;
    if (overlap == 3) {  // a pool of streams: successive hand-overs run concurrently, not queued in one stream
      hipStream_t& sref = d.ekf_pool[n_batches % kEkfPool];
      if (!sref) {
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&sref, hipStreamNonBlocking, hi));
      }
      if (!d.ev_ekf_in) {
        HIPCHK(hipEventCreateWithFlags(&d.ev_ekf_in, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.ev_ekf_out, hipEventDisableTiming));
      }
      side = sref;
    } else if (overlap) {
      hipStream_t& sref = overlap == 2 ? d.ekf_side : d.ekf_side_lo;
      if (!sref) {
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&sref, hipStreamNonBlocking, overlap == 2 ? hi : lo));
      }
      if (!d.ev_ekf_in) {
        HIPCHK(hipEventCreateWithFlags(&d.ev_ekf_in, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.ev_ekf_out, hipEventDisableTiming));
      }
      side = sref;
    }
    hipLaunchKernelGGL(dfmi::ekf_pit_handover_kernel, dim3(1), dim3(64), 0, st, (const dfmi::PitChan*)ch, nrec,
                       (unsigned*)handed, (int*)sidx + nh, final_ ? 1 : 0);
    HIPCHK(hipGetLastError());
    if (side != st) {
      HIPCHK(hipEventRecord(d.ev_ekf_in, st));
      HIPCHK(hipStreamWaitEvent(side, d.ev_ekf_in, 0));
      side_stream = side;
      side_used = true;
      if (n_batches < kEkfPool) used_streams[n_batches] = side;
    }
    ++n_batches;
    const char* kname;
    if (int rc = ekf_seq_launch(dx, cnt, rs, n, dx0, dp0, dq, dr, wt, R, nbuf, dstates, side, &kname,
                                (const int*)sidx + nh))
      return rc;
    seq_name = kname;
    nh += cnt;
    return DFMI_OK;
  };
  int cur = 0;
  bool fresh = false;  // pin holds the channels' final control blocks
  for (int pass = 1;; ++pass) {
    if (t_tune.ekf_pit_fused) {
      hipLaunchKernelGGL(dfmi::ekf_pit_pass_kernel, lanes, dim3(64), 0, st, (const double*)xt, (const double*)wtt, n,
                         B, nb, dx0, dp0, dq, dr, (const double*)lv[cur][0], tops[cur], lv[cur ^ 1][0], (double*)ent,
                         ch, (double*)conv, (unsigned*)done, rule, (double*)hist, (int)R, nbuf,
                         dstates, tk);
    } else {
      hipLaunchKernelGGL(dfmi::ekf_pit_aggregate_kernel, lanes, dim3(64), 0, st, (const double*)xt,
                         (const double*)wtt, (const double*)xbar, n, B, nb, dx0, dp0, dq, dr,
                         (const dfmi::PitChan*)ch, lv[0][0], tk, (const double*)nullptr, (const double*)nullptr,
                         (int64_t)0);
      scan(lv[0]);
      hipLaunchKernelGGL(dfmi::ekf_pit_blocks_kernel, lanes, dim3(64), 0, st, (const double*)xt, (const double*)wtt,
                         (double*)xbar, n, B, nb, dx0, dp0, dq, dr, (const double*)lv[0][0], tops[0],
                         (const dfmi::PitChan*)ch, (double*)conv, (int)R, nbuf, dstates, rule.measure, tk);
      hipLaunchKernelGGL(dfmi::ekf_pit_check_kernel, dim3((unsigned)((nrec + 63) / 64)), dim3(64), 0, st,
                         (double*)conv, nrec, rule, ch, (double*)hist);
    }
    HIPCHK(hipGetLastError());
    if (pass >= cap) break;
    if (pass == next_check) {
      // the channels' control blocks to the host (one copy, one stream sync): the check and,
      // when no channel is left passing, the outcome below
      HIPCHK(hipMemcpyAsync(pin, ch, (size_t)nrec * sizeof(dfmi::PitChan), hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      const dfmi::PitChan* hc = (const dfmi::PitChan*)pin;
      bool any = false;
      for (int64_t r = 0; r < nrec && !any; ++r) any = hc[r].status == 0;
      if (!any) {
        fresh = true;
        break;
      }
      if (int rc = hand_over(hc, false)) return rc;  // beside the passes still to come
      next_check = std::min(pass + every, cap);
    }
    if (t_tune.ekf_pit_fused) {
      scan(lv[cur ^ 1]);
      cur ^= 1;
    }
  }
  // the channels' outcomes on the host; the ones not converged go to the sequential kernel
  if (!fresh) HIPCHK(hipMemcpyAsync(pin, ch, (size_t)nrec * sizeof(dfmi::PitChan), hipMemcpyDeviceToHost, st));
  if (hist_n) {
    g_pit_hist.assign((size_t)nrec * hist_n, 0.0);
    HIPCHK(hipMemcpyAsync(g_pit_hist.data(), hist, g_pit_hist.size() * 8, hipMemcpyDeviceToHost, st));
    g_pit_hist_n = hist_n;
  }
  if (!fresh || hist_n) HIPCHK(hipStreamSynchronize(st));
  const dfmi::PitChan* hc = (const dfmi::PitChan*)pin;
  g_pit_passes.assign((size_t)nrec, 0);
  for (int64_t r = 0; r < nrec; ++r) g_pit_passes[r] = hc[r].status == 1 ? hc[r].passes : -hc[r].passes;
  g_last_demod = "ekf_pit (B=" + std::to_string(B) + ", nb=" + std::to_string(nb) + ")";
  if (int rc = hand_over(hc, true)) return rc;  // every channel still not converged
  if (side_used) {  // join: the caller's stream sees the re-run states
    for (int i = 0; i < kEkfPool; ++i) {
      hipStream_t w = overlap == 3 ? used_streams[i] : (i == 0 ? side_stream : nullptr);
      if (!w) continue;
      HIPCHK(hipEventRecord(t_ds->ev_ekf_out, w));
      HIPCHK(hipStreamWaitEvent(st, t_ds->ev_ekf_out, 0));
    }
  }
  if (nh) g_last_demod += std::string(" + ") + seq_name + " x" + std::to_string(nh);
  return DFMI_OK;
}

// EKFFitter.fit (fitters.py:214-320) for nrec channels. Either x0 (nrec x 5, dc
// included) and r_val (nrec) come from the caller (dfmi_ekf), or init4 (a, m, phi,
// psi for every record) does and the pre-reductions run on the device (dfmi_ekf_fit):
// x0[4] = np.mean(data) (fitters.py:253), R_val = np.var(data) unless given (:256).
int ekf_impl(const double* x, int64_t nrec, int64_t rec_stride, int64_t n_samp, const double* x0, const double* init4,
             const double* p0_diag, const double* q_diag, const double* r_val, double w_m, double f_samp, int32_t R,
             int64_t nbuf, double* states, int32_t mem, void* stream) {
  if (nrec < 0 || n_samp < 0 || R <= 0 || nbuf < 0) return fail(DFMI_ERR_ARG, "bad ekf geometry");
  if (nrec > 1 && rec_stride < n_samp) return fail(DFMI_ERR_ARG, "rec_stride < n_samp");
  if (init4 && n_samp > INT32_MAX) return fail(DFMI_ERR_ARG, "n_samp >= 2^31");
  g_pit_passes.clear();  // this call's outcome replaces the last one's, whatever path it takes
  g_pit_hist.clear();
  g_pit_hist_n = 0;
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  if (nrec == 0) return DFMI_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t rs = nrec > 1 ? rec_stride : n_samp;
  const double *dx = x, *dx0 = x0, *dp0 = p0_diag, *dq = q_diag, *dr = r_val;
  double* dstates = states;
  const size_t sb = (size_t)nrec * nbuf * 5 * 8;
  const bool host = mem != DFMI_MEM_DEVICE;
  if (host) {
    void *a, *c2, *d, *f;
    const size_t xb = (size_t)((nrec - 1) * rs + n_samp) * 8;
    if ((rc = workspace(dev, "e_x", xb > 0 ? xb : 8, &a))) return rc;
    if ((rc = workspace(dev, "e_p0", 5 * 8, &c2))) return rc;
    if ((rc = workspace(dev, "e_q", 5 * 8, &d))) return rc;
    if ((rc = workspace(dev, "e_st", sb > 0 ? sb : 8, &f))) return rc;
    if (xb) HIPCHK(hipMemcpyAsync(a, x, xb, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c2, p0_diag, 5 * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d, q_diag, 5 * 8, hipMemcpyHostToDevice, st));
    dx = (const double*)a;
    dp0 = (const double*)c2;
    dq = (const double*)d;
    dstates = (double*)f;
  }
  if (init4) {
    // x0 = [init4, mean] and r_val (given or np.var) formed on the device
    void *b, *e;
    if ((rc = workspace(dev, "e_x0", (size_t)nrec * 5 * 8, &b))) return rc;
    if ((rc = workspace(dev, "e_r", (size_t)nrec * 8, &e))) return rc;
    // init4 in every row (from the device copy when it lives there: no host round trip),
    // then the moments kernels fill x0[r*5+4] and r (an empty record keeps numpy's NaN
    // mean / variance)
    dfmi::EkfInit hv{};
    if (host) {
      memcpy(hv.i4, init4, sizeof(hv.i4));
      if (r_val) hv.rv = *r_val;
    }
    hipLaunchKernelGGL(dfmi::ekf_x0_kernel, dim3((unsigned)((nrec + 63) / 64)), dim3(64), 0, st, (double*)b, (double*)e,
                       nrec, host ? (const double*)nullptr : init4, host ? (const double*)nullptr : r_val,
                       r_val != nullptr, hv);
    if (n_samp >= 1) {
      if ((rc = moments_dev(dev, dx, nrec, rs, n_samp, (double*)b + 4, 5, r_val ? nullptr : (double*)e, 1, st)))
        return rc;
    }
    dx0 = (const double*)b;
    dr = (const double*)e;
  } else if (host) {
    void *b, *e;
    if ((rc = workspace(dev, "e_x0", (size_t)nrec * 5 * 8, &b))) return rc;
    if ((rc = workspace(dev, "e_r", (size_t)nrec * 8, &e))) return rc;
    HIPCHK(hipMemcpyAsync(b, x0, (size_t)nrec * 5 * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e, r_val, (size_t)nrec * 8, hipMemcpyHostToDevice, st));
    dx0 = (const double*)b;
    dr = (const double*)e;
  }
  if (sb) HIPCHK(hipMemsetAsync(dstates, 0, sb, st));
  void* wtw = nullptr;
  if ((rc = workspace(dev, "e_wt", (size_t)(n_samp > 0 ? n_samp : 1) * 8, &wtw))) return rc;
  if (n_samp > 0)
    hipLaunchKernelGGL(dfmi::ekf_phase_kernel, dim3((unsigned)((n_samp + 255) / 256)), dim3(256), 0, st,
                       (double*)wtw, n_samp, w_m, f_samp);
  // the parallel form by channel count and length alone (the same input always takes the same
  // path); only when its scratch (~6 x 8 B per sample + 2 x 65 doubles per block per channel,
  // ~37 MB for 400k samples) cannot be allocated do the sequential kernels run instead
  bool pit = t_tune.ekf_pit > 0 && nrec <= t_tune.ekf_pit && n_samp >= t_tune.ekf_pit_min && n_samp >= 2;
  if (pit) {
    rc = ekf_pit_run(dev, dx, nrec, rs, n_samp, dx0, dp0, dq, dr, (const double*)wtw, w_m, f_samp, R, nbuf, dstates,
                     st);
    if (rc == kPitNoMem) pit = false;
    else if (rc) return rc;
  }
  if (!pit) {
    const char* kname;
    if ((rc = ekf_seq_launch(dx, nrec, rs, n_samp, dx0, dp0, dq, dr, (const double*)wtw, R, nbuf, dstates, st, &kname)))
      return rc;
    g_last_demod = kname;  // also reports the EKF variant
  }
  if (host) {
    if (sb) HIPCHK(hipMemcpyAsync(states, dstates, sb, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  return DFMI_OK;
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
  CallScope cs;
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return 0;
  return g_ndev;
}

const char* dfmi_last_error(void) { return g_err.c_str(); }

const char* dfmi_version(void) { return "dfmi 0.3 gfx950"; }

const char* dfmi_last_demod_kernel(void) { return g_last_demod.c_str(); }

int dfmi_probe_read(int64_t* out, int32_t n) {
  CallScope cs;
  int dev;
  if (int rc = ensure_init(&dev)) return rc;
  if (!t_ds->probe) return fail(DFMI_ERR_ARG, "probe not enabled on this device (dfmi_set_tuning(\"probe\", 1))");
  if (n < 0 || n > 16 + 2 * dfmi::kProbeWaves || (n && !out)) return fail(DFMI_ERR_ARG, "bad probe read");
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, t_ds->probe, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return DFMI_OK;
}

int dfmi_get_tuning(const char* key, int64_t* value) {
  CallScope cs;
  if (!key || !value) return fail(DFMI_ERR_ARG, "null argument");
  const std::string k(key);
  if (k == "probe") {
    int dev;
    if (int rc = ensure_init(&dev)) return rc;
    *value = t_ds->probe ? 1 : 0;
    return DFMI_OK;
  }
  auto it = knobs().find(k);
  if (it == knobs().end()) return fail(DFMI_ERR_ARG, "unknown tuning key " + k);
  *value = t_tune.*(it->second.v);
  return DFMI_OK;
}

int dfmi_set_tuning(const char* key, int64_t value) {
  CallScope cs;
  if (!key) return fail(DFMI_ERR_ARG, "null key");
  const std::string k(key);
  if (k == "probe") {  // per device: a timestamp buffer in this device's memory
    int dev;
    if (int rc = ensure_init(&dev)) return rc;
    if (value && !t_ds->probe) {
      void* p = nullptr;
      const size_t pb = (16 + 2 * (size_t)dfmi::kProbeWaves) * sizeof(uint64_t);
      HIPCHK(hipMalloc(&p, pb));
      HIPCHK(hipMemset(p, 0, pb));
      t_ds->probe = (uint64_t*)p;
    } else if (!value && t_ds->probe) {
      HIPCHK(hipDeviceSynchronize());
      HIPCHK(hipFree(t_ds->probe));
      t_ds->probe = nullptr;
    }
    return DFMI_OK;
  }
  auto it = knobs().find(k);
  if (it == knobs().end()) return fail(DFMI_ERR_ARG, "unknown tuning key " + k);
  const Knob& kn = it->second;
  if (value < 0 || value > (1 << 20)) return fail(DFMI_ERR_ARG, "tuning value out of range for " + k);
  if (!kn.allowed.empty()) {
    bool ok = false;
    for (int a : kn.allowed) ok = ok || (a == value);
    if (!ok) return fail(DFMI_ERR_ARG, "value not allowed for " + k);
  }
  std::lock_guard<std::mutex> g(g_mu);
  g_tune.*(kn.v) = (int)value;
  return DFMI_OK;
}

int dfmi_step_timing(int32_t enable) {
  CallScope cs;
  int dev;
  if (int rc = ensure_init(&dev)) return rc;
  t_ds->timing = enable != 0;
  return DFMI_OK;
}

int dfmi_step_timing_read(double* demod_ms, double* lm_ms, int64_t* nsteps) {
  CallScope cs;
  if (!demod_ms || !lm_ms || !nsteps) return fail(DFMI_ERR_ARG, "null pointer");
  int dev;
  if (int rc = ensure_init(&dev)) return rc;
  DeviceState& ds = *t_ds;
  double d = 0.0, l = 0.0;
  hipError_t err = hipSuccess;
  for (auto& tr : ds.ev_steps) {  // every triple goes back to the pool, read or not
    float a = 0.f, b = 0.f;
    if (err == hipSuccess) err = hipEventSynchronize(tr[2]);
    if (err == hipSuccess) err = hipEventElapsedTime(&a, tr[0], tr[1]);
    if (err == hipSuccess) err = hipEventElapsedTime(&b, tr[1], tr[2]);
    d += a;
    l += b;
    ds.ev_pool.insert(ds.ev_pool.end(), tr.begin(), tr.end());
  }
  *nsteps = (int64_t)ds.ev_steps.size();
  *demod_ms = d;
  *lm_ms = l;
  ds.ev_steps.clear();
  if (err != hipSuccess) return fail(DFMI_ERR_HIP, std::string("step timing read: ") + hipGetErrorString(err));
  return DFMI_OK;
}

// Frees every workspace of the current device (waits for the device first). The next
// call re-allocates what it needs.
int dfmi_release_workspaces(void) {
  CallScope cs;
  int dev;
  if (int rc = ensure_init(&dev)) return rc;
  HIPCHK(hipDeviceSynchronize());
  for (auto& kv : t_ds->ws)
    if (int rc = free_stream_ws(kv.second)) return rc;
  t_ds->ws.clear();
  if (t_ds->pin) HIPCHK(hipHostFree(t_ds->pin));
  t_ds->pin = nullptr;
  t_ds->pin_n = 0;
  return DFMI_OK;
}

int dfmi_demod(const double* x, int64_t nseg, int64_t seg_stride, int32_t R, int32_t ndata, double w0,
               int32_t period, double* qi, double* dc, int32_t mem, void* stream) {
  CallScope cs(stream);
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
  CallScope cs(stream);
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
  CallScope cs(stream);
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
  CallScope cs(stream);
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

int dfmi_wdfmi_fit(const double* x, int64_t nrec, int64_t rec_stride, int64_t nbuf, int32_t R,
                   const double* witness, int64_t wit_stride, const dfmi_wdfmi_config* cfg, double* out,
                   int32_t* fitok, int32_t mem, void* stream) {
  CallScope cs(stream);
  if (!cfg) return fail(DFMI_ERR_ARG, "null config");
  if (cfg->method < DFMI_WDFMI_NLS || cfg->method > DFMI_HWDFMI) return fail(DFMI_ERR_ARG, "unknown W-DFMI method");
  if (nrec < 0 || nbuf < 0 || R < 4) return fail(DFMI_ERR_ARG, "bad record geometry (R >= 4)");
  if (R > 16384) return fail(DFMI_ERR_UNSUPPORTED, "W-DFMI fitters support R <= 16384");
  if (nrec > 1 && rec_stride < nbuf * (int64_t)R) return fail(DFMI_ERR_ARG, "rec_stride < nbuf*R");
  if (nrec > 1 && wit_stride != 0 && wit_stride < R) return fail(DFMI_ERR_ARG, "wit_stride < R");
  if (!(cfg->f_samp > 0.0)) return fail(DFMI_ERR_ARG, "f_samp must be > 0");
  if (cfg->method == DFMI_WDFMI_NLS && (cfg->ndata < 1 || cfg->ndata > 32))
    return fail(DFMI_ERR_UNSUPPORTED, "W-DFMI NLS: 1 <= ndata <= 32");
  if (cfg->method == DFMI_WDFMI_SEQ && (cfg->ndata_psi < 1 || cfg->ndata_psi > 64))
    return fail(DFMI_ERR_UNSUPPORTED, "W-DFMI SEQ: 1 <= ndata_psi <= 64");
  if (nrec * nbuf > 0 && (!x || !witness || !out || !fitok)) return fail(DFMI_ERR_ARG, "null pointer");
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  const int64_t nseg = nrec * nbuf;
  if (nseg == 0) return DFMI_OK;
  hipStream_t st = (hipStream_t)stream;
  dfmi::WdfmiLaunch a;
  memset(&a, 0, sizeof(a));
  a.method = cfg->method;
  a.R = R;
  a.ndata = cfg->ndata;
  a.ndata_psi = cfg->ndata_psi;
  a.threads = R <= 4096 ? 256 : 1024;
  a.accel = t_tune.wdfmi_accel;
  a.probe = t_ds->probe;
  a.nrec = nrec;
  a.nbuf = nbuf;
  a.f_samp = cfg->f_samp;
  a.f_mod = cfg->f_mod;
  a.df = cfg->df;
  a.f_ref = cfg->f_ref;
  a.tau_init = cfg->tau_init;
  a.init_a = cfg->init_a;
  a.init_phi = cfg->init_phi;
  a.init_psi = cfg->init_psi;
  a.w0 = (2.0 * M_PI * cfg->f_mod) / cfg->f_samp;  // omega_mod / f_samp (fitters.py:506-507)
  const int nh = cfg->method == DFMI_WDFMI_NLS ? cfg->ndata : (cfg->method == DFMI_WDFMI_SEQ ? cfg->ndata_psi : 0);
  a.L = 0;
  if (nh > 0 && cfg->period >= 0) a.L = cfg->period > 0 ? cfg->period : detect_period_impl(a.w0, R, nh);
  if (a.L > R) a.L = 0;
  if ((rc = pairwise_plan(dev, R, &a.pw_plan, nullptr))) return rc;
  const size_t lds = dfmi::wdfmi_lds_bytes(a);
  if (lds > t_ds->lds_per_block)
    return fail(DFMI_ERR_UNSUPPORTED, "W-DFMI: R too large for the LDS budget (" + std::to_string(lds) + " B)");
  if (nh > 0 && a.L > 0) {
    const double* bt;
    if ((rc = basis_table(dev, a.L, nh, a.w0, st, &bt))) return rc;
    if (cfg->method == DFMI_WDFMI_NLS) a.btab_nls = bt;
    else a.btab_psi = bt;
  }
  const int64_t rs = nrec > 1 ? rec_stride : nbuf * (int64_t)R;
  const int64_t ws = nrec > 1 ? wit_stride : 0;
  const int64_t ntmpl = ws == 0 ? 1 : nrec;
  void* tm;
  if ((rc = workspace(dev, "w_tmpl", (size_t)ntmpl * R * 8, &tm))) return rc;
  a.tmpl = (double*)tm;
  a.rec_stride = rs;
  a.wit_stride = ws;
  a.x = x;
  a.wit = witness;
  a.out = out;
  a.fitok = fitok;
  if (mem != DFMI_MEM_DEVICE) {
    void *dx, *dw, *dout, *dok;
    const size_t xb = (size_t)((nrec - 1) * rs + nbuf * (int64_t)R) * 8;
    const size_t wb = (size_t)((ntmpl - 1) * ws + R) * 8;
    if ((rc = workspace(dev, "w_x", xb, &dx))) return rc;
    if ((rc = workspace(dev, "w_wit", wb, &dw))) return rc;
    if ((rc = workspace(dev, "w_out", (size_t)7 * nseg * 8, &dout))) return rc;
    if ((rc = workspace(dev, "w_ok", (size_t)nseg * 4, &dok))) return rc;
    HIPCHK(hipMemcpyAsync(dx, x, xb, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dw, witness, wb, hipMemcpyHostToDevice, st));
    a.x = (const double*)dx;
    a.wit = (const double*)dw;
    a.out = (double*)dout;
    a.fitok = (int32_t*)dok;
  }
  HIPCHK(dfmi::wdfmi_launch(a, st));
  if (mem != DFMI_MEM_DEVICE) {
    HIPCHK(hipMemcpyAsync(out, a.out, (size_t)7 * nseg * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(fitok, a.fitok, (size_t)nseg * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  return DFMI_OK;
}

int dfmi_ekf(const double* x, int64_t nrec, int64_t rec_stride, int64_t n_samp, const double* x0,
             const double* p0_diag, const double* q_diag, const double* r_val, double w_m, double f_samp, int32_t R,
             int64_t nbuf, double* states, int32_t mem, void* stream) {
  CallScope cs(stream);
  return ekf_impl(x, nrec, rec_stride, n_samp, x0, nullptr, p0_diag, q_diag, r_val, w_m, f_samp, R, nbuf, states, mem,
                  stream);
}

int dfmi_ekf_fit(const double* x, int64_t nrec, int64_t rec_stride, int64_t n_samp, const double* init4,
                 const double* p0_diag, const double* q_diag, const double* r_val, double w_m, double f_samp,
                 int32_t R, int64_t nbuf, double* states, int32_t mem, void* stream) {
  CallScope cs(stream);
  if (!init4) return fail(DFMI_ERR_ARG, "null init4");
  return ekf_impl(x, nrec, rec_stride, n_samp, nullptr, init4, p0_diag, q_diag, r_val, w_m, f_samp, R, nbuf, states,
                  mem, stream);
}

int dfmi_ekf_pit_passes(int32_t* passes, int64_t nrec) {
  CallScope cs;
  if (!passes || nrec < 0) return fail(DFMI_ERR_ARG, "bad pass buffer");
  if (g_pit_passes.empty()) {
    for (int64_t r = 0; r < nrec; ++r) passes[r] = 0;
    return DFMI_OK;
  }
  if (nrec != (int64_t)g_pit_passes.size()) return fail(DFMI_ERR_ARG, "nrec differs from the last EKF call's");
  memcpy(passes, g_pit_passes.data(), (size_t)nrec * sizeof(int32_t));
  return DFMI_OK;
}

int dfmi_ekf_pit_trace(double* moves, int64_t nrec, int32_t max_pass) {
  CallScope cs;
  if (!moves || nrec < 0 || max_pass < 0) return fail(DFMI_ERR_ARG, "bad trace buffer");
  if (g_pit_hist_n == 0) return fail(DFMI_ERR_ARG, "no trace: set ekf_pit_trace to 1 before a parallel-in-time EKF call");
  if ((size_t)nrec * g_pit_hist_n != g_pit_hist.size()) return fail(DFMI_ERR_ARG, "nrec differs from the last EKF call's");
  for (int64_t r = 0; r < nrec; ++r)
    for (int32_t p = 0; p < max_pass; ++p)
      moves[r * max_pass + p] = p < g_pit_hist_n ? g_pit_hist[(size_t)r * g_pit_hist_n + p] : __builtin_nan("");
  return DFMI_OK;
}

int dfmi_synth_asd(const dfmi_synth_trial* trials, int64_t ntrial, int64_t n_samp, double f_samp, double* out,
                   int32_t mem, void* stream) {
  CallScope cs(stream);
  if (ntrial < 0 || n_samp < 2 || !(f_samp > 0.0)) return fail(DFMI_ERR_ARG, "bad synthesis geometry (n_samp >= 2)");
  if (ntrial > 0 && (!trials || !out)) return fail(DFMI_ERR_ARG, "null pointer");
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  if (ntrial == 0) return DFMI_OK;
  hipStream_t st = (hipStream_t)stream;
  void *dt, *scr, *dout = out;
  const size_t ob = (size_t)ntrial * n_samp * 8;
  if ((rc = workspace(dev, "s_trials", (size_t)ntrial * sizeof(dfmi_synth_trial), &dt))) return rc;
  if ((rc = workspace(dev, "s_scratch", dfmi::synth_scratch_bytes(ntrial, n_samp), &scr))) return rc;
  if (mem != DFMI_MEM_DEVICE && (rc = workspace(dev, "s_out", ob, &dout))) return rc;
  HIPCHK(hipMemcpyAsync(dt, trials, (size_t)ntrial * sizeof(dfmi_synth_trial), hipMemcpyHostToDevice, st));
  HIPCHK(dfmi::synth_launch((const dfmi_synth_trial*)dt, ntrial, n_samp, f_samp, scr, (double*)dout, st));
  if (mem != DFMI_MEM_DEVICE) HIPCHK(hipMemcpyAsync(out, dout, ob, hipMemcpyDeviceToHost, st));
  // the trial table is a caller (host) array: done with it only once the copy ran
  HIPCHK(hipStreamSynchronize(st));
  return DFMI_OK;
}

int dfmi_synth_snr(const dfmi_snr_params* prm, int64_t idx0, int64_t n, double* out, int32_t mem, void* stream) {
  CallScope cs(stream);
  if (!prm || n < 0 || idx0 < 0) return fail(DFMI_ERR_ARG, "bad snr synthesis arguments");
  if (!(prm->f_samp > 0.0) || prm->period < 0) return fail(DFMI_ERR_ARG, "f_samp must be > 0, period >= 0");
  if (n > 0 && !out) return fail(DFMI_ERR_ARG, "null pointer");
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  if (n == 0) return DFMI_OK;
  hipStream_t st = (hipStream_t)stream;
  double* dout = out;
  if (mem != DFMI_MEM_DEVICE && (rc = workspace(dev, "g_out", (size_t)n * 8, (void**)&dout))) return rc;
  HIPCHK(dfmi::snr_gen_launch(*prm, idx0, n, dout, t_ds->n_cu, st));
  if (mem != DFMI_MEM_DEVICE) {
    HIPCHK(hipMemcpyAsync(out, dout, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  return DFMI_OK;
}

int dfmi_bessel_eval(const double* x, int64_t nx, int32_t nmax, int32_t method, double* out, int32_t mem,
                     void* stream) {
  CallScope cs(stream);
  if (nx < 0 || nmax < 0 || method < 0 || method > 2) return fail(DFMI_ERR_ARG, "bad bessel_eval arguments");
  if ((method == 1 && nmax > 13) || (method == 2 && nmax > 17))
    return fail(DFMI_ERR_ARG, "register path: nmax <= 13 (method 1) / 17 (method 2)");
  if (nx > 0 && (!x || !out)) return fail(DFMI_ERR_ARG, "null pointer");
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  if (nx == 0) return DFMI_OK;
  hipStream_t st = (hipStream_t)stream;
  const size_t ob = (size_t)nx * (nmax + 1) * 8;
  const double* dx = x;
  double* dout = out;
  if (mem != DFMI_MEM_DEVICE) {
    void *a, *b;
    if ((rc = workspace(dev, "b_x", (size_t)nx * 8, &a))) return rc;
    if ((rc = workspace(dev, "b_out", ob, &b))) return rc;
    HIPCHK(hipMemcpyAsync(a, x, (size_t)nx * 8, hipMemcpyHostToDevice, st));
    dx = (const double*)a;
    dout = (double*)b;
  }
  HIPCHK(dfmi::bessel_eval_launch(dx, nx, nmax, method, dout, st));
  if (mem != DFMI_MEM_DEVICE) {
    HIPCHK(hipMemcpyAsync(out, dout, ob, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  return DFMI_OK;
}

int dfmi_record_moments(const double* x, int64_t nrec, int64_t rec_stride, int64_t n, double* mean, double* var,
                        int32_t mem, void* stream) {
  CallScope cs(stream);
  if (nrec < 0 || n < 1 || n > INT32_MAX) return fail(DFMI_ERR_ARG, "bad moments geometry (1 <= n < 2^31)");
  if (nrec > 1 && rec_stride < n) return fail(DFMI_ERR_ARG, "rec_stride < n");
  if (nrec > 0 && (!x || !mean)) return fail(DFMI_ERR_ARG, "null pointer");
  int dev;
  int rc = ensure_init(&dev);
  if (rc) return rc;
  if (nrec == 0) return DFMI_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t rs = nrec > 1 ? rec_stride : n;
  const double* dx = x;
  double *dm = mean, *dv = var;
  if (mem != DFMI_MEM_DEVICE) {
    void *a, *b;
    if ((rc = workspace(dev, "m_x", (size_t)((nrec - 1) * rs + n) * 8, &a))) return rc;
    if ((rc = workspace(dev, "m_out", (size_t)nrec * 16, &b))) return rc;
    HIPCHK(hipMemcpyAsync(a, x, (size_t)((nrec - 1) * rs + n) * 8, hipMemcpyHostToDevice, st));
    dx = (const double*)a;
    dm = (double*)b;
    dv = var ? dm + nrec : nullptr;
  }
  if ((rc = moments_dev(dev, dx, nrec, rs, n, dm, 1, dv, 1, st))) return rc;
  if (mem != DFMI_MEM_DEVICE) {
    HIPCHK(hipMemcpyAsync(mean, dm, (size_t)nrec * 8, hipMemcpyDeviceToHost, st));
    if (var) HIPCHK(hipMemcpyAsync(var, dv, (size_t)nrec * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  return DFMI_OK;
}

}  // extern "C"

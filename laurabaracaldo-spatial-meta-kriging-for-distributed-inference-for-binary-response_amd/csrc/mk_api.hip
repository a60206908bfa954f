// C ABI (include/mk.h) and the per-iteration launch schedule.
//
// One mk_session = one GPU's shard of subsets resident in HBM.  The shard is split into
// contiguous subset groups, each advanced by its own HIP stream: a group's iteration is a
// fixed sequence of stream-ordered launches with no host synchronisation (data-dependent
// control -- which factors changed -- lives in device work lists), and the groups' streams
// overlap on the GPU, so one group's latency-bound steps (diagonal-tile factorisations,
// the MH decisions, launch tails) run beside another group's MFMA panel updates.  A group
// is a pointer view into the shard's arrays (every array is [subset][...]); the chains do
// not depend on the grouping (RNG streams are keyed by global subset index).
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <unistd.h>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <utility>
#include <memory>
#include <mutex>
#include <string>
#include <vector>
#include "../../include/mk.h"
#include "mk_kernels.hpp"
#include "mk_gemm.hpp"
#include "mk_internal.hpp"

using namespace mk;

static thread_local std::string g_err;

static int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return set_err(MK_E_HIP, std::string(#x " -> ") + hipGetErrorString(e_)); \
  } while (0)

// Entry of a C-ABI call that works on `dev`: registered with the stall watchdog, the caller's
// current device restored on every return path (an R or torch host keeps its own device).
#define MK_ENTRY_DEVICE(dev) \
  ApiCall mk_call_(__func__); \
  DeviceGuard mk_dg_;         \
  HIPCHK(hipSetDevice(dev))

extern "C" const char* mk_last_error(void) { return g_err.c_str(); }
namespace mk {
int host_error(int code, const char* msg) { return set_err(code, msg); }   // for host-only sources
}

extern "C" int mk_hip_initialized(void) {
  DIR* d = opendir("/proc/self/fd");
  if (!d) return 0;
  int found = 0;
  char path[64], target[256];
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    std::snprintf(path, sizeof path, "/proc/self/fd/%s", e->d_name);
    const ssize_t n = readlink(path, target, sizeof target - 1);
    if (n <= 0) continue;
    target[n] = 0;
    if (std::strcmp(target, "/dev/kfd") == 0) {
      found = 1;
      break;
    }
  }
  closedir(d);
  return found;
}

extern "C" int mk_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" int mk_device_memory(int32_t device, int64_t* free_bytes, int64_t* total_bytes) {
  MK_ENTRY_DEVICE(device);
  size_t f = 0, t = 0;
  HIPCHK(hipMemGetInfo(&f, &t));
  if (free_bytes) *free_bytes = (int64_t)f;
  if (total_bytes) *total_bytes = (int64_t)t;
  return 0;
}

namespace {

constexpr int NKSTAT = 14;
// KS_CHOL_UPDATE: the 128-tile panel-update launches (k_chol_update<128>); KS_CHOL_UPDATE_SUB:
// the 64- / 32-sub-tile ones (small grids).  Together: the roofline kernel k_chol_update.
// KS_UPDATE_BUSY: both, with the time of launches that overlap (the split schedule's bulk and
// critical streams) counted once -- the union of their event intervals.
// KS_PRED_VAR: the kriging GEMM k_pred_var; its flops assume every pair is refreshed (an upper
// bound: only the pairs whose factor changed are in the list -- bench_kriging counts exactly).
// KS_COV: the candidates' covariance assembly (k_cov_candidate, with k_matern_table for Matern).
enum { KS_CHOL_UPDATE = 0, KS_CHOL_DIAG, KS_CHOL_TRSM, KS_SWEEP, KS_LAUUM, KS_ITER, KS_INV, KS_CHOL_UPDATE_SUB,
       KS_UPDATE_BUSY, KS_PRED_VAR, KS_COV, KS_SWEEP_FALLBACK, KS_KRIG_CHEB, KS_KRIG_FALLBACK };
// KS_KRIG_CHEB: tiles kriged by phi interpolation (predict_tile_cheb): launches = tiles, flops = exact
// s evaluations ((subset, node or check point) pairs), total_ms = the largest check difference seen
// (not a time).  KS_KRIG_FALLBACK: tiles whose check failed and were replayed exactly (launches), and
// total_ms the largest failing difference.
// KS_SWEEP_FALLBACK: launches = (subset, iteration) sweeps k_sweep_mg refused admission and its
// k_sweep fallback ran (counted on the device, read at the end of every mk_session_run; no timing).

struct Stat {
  long launches = 0;
  double ms = 0.0, flops = 0.0;
};

struct Timed {
  int which;
  hipEvent_t a, b;
  double flops;
  int cnt = -1;   // >= 0: flops are per listed factor, times the device-side count copied to inv_cnt[cnt]
};

// One stream's share of the shard: views of the shard arrays starting at subset s0.
struct Group {
  Model md{};
  MatSet ms{};
  hipStream_t stream = nullptr;
  int S = 0, s0 = 0;
  int* d_list = nullptr;   // pairs whose factor changed (inverse work list)
  int* d_count = nullptr;
  int* d_plist = nullptr;  // pairs needing a kriging refresh
  int* d_pcount = nullptr;
  hipEvent_t done = nullptr;         // fork-join sweep: this group's pre-sweep work is queued
  hipStream_t bulk = nullptr;        // split Cholesky (launch_cholesky): CU-masked bulk-update stream
  std::vector<hipEvent_t> ev;        // 2 nt + 1 events reused every factorisation
};

Model model_view(const Model& m, int s0, int S) {
  Model v = m;
  v.S = S;
  v.subset_base = m.subset_base + s0;
  const long q = m.q, np = m.n_pad, Np = m.Np, s = s0;
  v.n_s = m.n_s + s;
  v.coords = m.coords + s * 2 * np;
  v.y = m.y + s * Np;
  v.wt = m.wt + s * Np;
  v.X = m.X + s * m.p * Np;
  v.beta = m.beta + s * m.p;
  v.theta = m.theta + s * m.n_theta;
  v.w = m.w + s * Np;
  v.eta = m.eta + s * Np;
  v.tune = m.tune + s * m.n_mh_max;
  v.acc = m.acc + s * m.n_mh_max;
  v.u = m.u + s * q * np;
  v.z = m.z + s * q * np;
  v.Z = m.Z + s * q * q * np;
  v.logdetR = m.logdetR + s * q;
  v.quad = m.quad + s * q;
  v.A_full = m.A_full + s * q * q;
  v.Ainv = m.Ainv + s * q * q;
  v.dirty = m.dirty + s * q;
  v.ld_part = m.ld_part + (long)s * m.q * m.nt;   // per (subset, outcome) pair
  v.quad_c = m.quad_c + (long)s * m.q;
  v.info = m.info + (long)s * m.q;
  v.sw_delta = m.sw_delta + s * Np;
  v.sw_dll = m.sw_dll + s * Np;
  v.sw_logu = m.sw_logu + s * Np;
  v.sw_acc = m.sw_acc + s * Np;
  v.samples = m.samples + s * m.n_samples * m.P;
  v.acc_hist = m.acc_hist + s * m.n_batch * (m.o_w + 1);
  if (m.w_samples) v.w_samples = m.w_samples + s * m.n_samples * Np;
  v.s_pred = m.s_pred + s * q * m.n_test_pad;
  v.s_part = m.s_part + s * q * m.nt * m.n_test_pad;
  if (m.PT) v.PT = m.PT + s * q * np * m.n_test_pad;
  if (m.XK) v.XK = m.XK + s * q * np * m.n_test_pad;
  v.w_pred = m.w_pred + s * m.n_kept * q * (long)std::max(m.n_test, 1);
  if (m.kz) v.kz = m.kz + s * q * np;
  if (m.kth) v.kth = m.kth + s * m.n_theta;
  if (m.kA) v.kA = m.kA + s * q * q;
  if (m.bacc) v.bacc = m.bacc + s * q * np;
  if (m.zc) v.zc = m.zc + s * q * np;
  if (m.la_nu) v.la_nu = m.la_nu + s * q;
  if (m.span) v.span = m.span + s;
  if (m.span_pt) v.span_pt = m.span_pt + s;
  if (m.chtab) v.chtab = m.chtab + s * q * MK_CH_TAB;
  if (m.chtab_p) v.chtab_p = m.chtab_p + s * q * MK_CH_TAB;
  return v;
}

MatSet matset_view(const MatSet& m, int s0) {
  MatSet v = m;
  const long sq = (long)s0 * m.q, e = (long)m.ld * m.ld, wt = (long)m.nt * MK_NB * MK_NB;
  v.L = m.L + sq * 2 * e;
  v.Winv = m.Winv + sq * 2 * wt;
  v.W = m.W + sq * e;
  if (m.Q) v.Q = m.Q + sq * e;
  if (m.QB) v.QB = m.QB + sq * wt;
  v.cur = m.cur + sq;
  if (m.Y) v.Y = m.Y + sq * e;
  return v;
}

}  // namespace

static std::atomic<int> g_live_sessions{0};

// ------------------------------------------------------------------ stream pool
// HIP streams outlive the sessions that use them: a session takes its streams from a per-process
// pool keyed by device and kind (plain, high priority, CU-masked with a given mask) and hands them
// back drained when it is destroyed.  A process that runs many sessions (the GPU test suite
// creates a few hundred) then creates its queues once instead of creating and destroying HIP
// queues -- CU-masked and priority ones included -- per session, the common factor of the
// intermittent stalls DESIGN.md 4.2 records (in session create / destroy).
enum { SK_PLAIN = 0, SK_PRIO = 1, SK_CUMASK = 2 };
struct PoolKey {
  int device = -1, kind = SK_PLAIN, prio = 0;
  std::vector<uint32_t> mask;
  bool operator==(const PoolKey& o) const {
    return device == o.device && kind == o.kind && prio == o.prio && mask == o.mask;
  }
};
typedef std::vector<std::pair<PoolKey, hipStream_t>> StreamList;
static std::mutex g_pool_mu;
static StreamList g_pool;        // idle streams
static bool g_pool_closed = false;   // mk_shutdown ran: returned streams are destroyed, not pooled
static std::vector<int> g_pool_count;   // streams of the pool in existence per device (idle or owned)
static int hw_queues();
static int tile_env(const char* name, int dflt);
static int krig_tables(mk_session* s);
static void kt_wait(mk_session* s, hipStream_t st);

static int& pool_count(int device) {   // g_pool_mu held
  if ((int)g_pool_count.size() <= device) g_pool_count.resize(device + 1, 0);
  return g_pool_count[device];
}

// Drain and destroy one stream on its device (the calling thread's device is restored).
static void stream_destroy(const PoolKey& k, hipStream_t st) {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    --pool_count(k.device);
  }
  DeviceGuard dg;
  if (hipSetDevice(k.device) == hipSuccess) {
    (void)hipStreamSynchronize(st);
    wd_forget(st);
    (void)hipStreamDestroy(st);
  }
  (void)hipGetLastError();
}

// Every idle pooled stream is destroyed while the HIP runtime is still alive.  Before this, the
// pool's CU-masked and priority queues stayed alive into the runtime's own static teardown, which
// crashed in __cxa_finalize after a profiler had finalised (rocprofv3, profiles/r03/final3/prof32.log:
// the 32-subset shard's lookahead schedule is the path that creates CU-masked queues).  Registered
// with atexit at the first stream the pool creates -- after HIP initialised, so it runs before HIP's
// own exit handlers -- and called by the hosts' exit hooks (Python atexit, the R package's
// .onUnload / exit finalizer).  Idempotent; sessions still alive keep their streams, which are then
// destroyed when the session is.
extern "C" void mk_shutdown(void) {
  StreamList idle;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool_closed = true;
    idle.swap(g_pool);
  }
  for (auto& o : idle) stream_destroy(o.first, o.second);
}
static void shutdown_at_exit() { mk_shutdown(); }

// A stream of this kind on the current device (hipSetDevice(device) done by the caller), recorded
// in `owned` for the session's destructor.
static hipError_t pool_stream(StreamList& owned, hipStream_t* st, int device, int kind, int prio = 0,
                              const std::vector<uint32_t>& mask = {}) {
  PoolKey k;
  k.device = device;
  k.kind = kind;
  k.prio = prio;
  k.mask = mask;
  StreamList evict;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_pool.size(); ++i)
      if (g_pool[i].first == k) {
        *st = g_pool[i].second;
        g_pool.erase(g_pool.begin() + (long)i);
        owned.push_back({k, *st});
        return hipSuccess;
      }
    // No exact match: a session of another configuration (another shard size needs another CU mask).
    // Idle streams left by earlier sessions still hold hardware queues, and a new queue among them
    // ends up sharing one with another stream (serialising the split Cholesky's streams: 5,427 ->
    // 4,087 subset-iters/s at 32 subsets) -- well before GPU_MAX_HW_QUEUES streams exist: configs[1]
    // after the 32-subset shard in one process ran 15,045-15,356 -> 12,659-13,189 subset-iters/s,
    // configs[3]'s share 1,666-1,701 -> 1,092.  So the idle streams on the device go (oldest first)
    // until at most MK_POOL_CAP - 1 streams remain besides the new one (default 1: every idle one;
    // measured cap 8 / 5 / 1: 12,659 / 15,261 / 15,532 and 1,092 / 1,678 / 1,714,
    // profiles/r04/pool/).  Repeated sessions of one configuration still reuse their queues.
    static const int cap_env = tile_env("MK_POOL_CAP", 1);
    int over = pool_count(device) + 1 - std::max(1, cap_env);
    for (size_t i = 0; i < g_pool.size() && over > 0;) {
      if (g_pool[i].first.device == device) {
        evict.push_back(g_pool[i]);
        g_pool.erase(g_pool.begin() + (long)i);
        --over;
      } else {
        ++i;
      }
    }
  }
  for (auto& o : evict) stream_destroy(o.first, o.second);
  hipError_t e;
  if (kind == SK_CUMASK) {
    // cuMaskSize = the device's CU count (as before the pool); the array is padded to that many
    // words so the runtime never reads past it, whichever unit it counts in (the words past the
    // CU count are ignored)
    const uint32_t size = (uint32_t)(mask.size() * 32);
    std::vector<uint32_t> padded(size, 0xffffffffu);
    for (size_t i = 0; i < mask.size(); ++i) padded[i] = mask[i];
    e = hipExtStreamCreateWithCUMask(st, size, padded.data());
  } else {
    e = kind == SK_PRIO ? hipStreamCreateWithPriority(st, hipStreamNonBlocking, prio)
                        : hipStreamCreateWithFlags(st, hipStreamNonBlocking);
  }
  if (e == hipSuccess) {
    owned.push_back({k, *st});
    {
      std::lock_guard<std::mutex> lk(g_pool_mu);
      ++pool_count(device);
    }
    static std::once_flag at_exit;
    std::call_once(at_exit, [] { std::atexit(shutdown_at_exit); });
  }
  return e;
}
static void pool_return(StreamList& owned) {
  StreamList gone;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (auto& o : owned) (g_pool_closed ? gone : g_pool).push_back(o);
  }
  owned.clear();
  for (auto& o : gone) stream_destroy(o.first, o.second);
}
namespace mk {
hipError_t stream_acquire(int device, hipStream_t* st) {
  StreamList one;
  return pool_stream(one, st, device, SK_PLAIN);
}
void stream_release(int device, hipStream_t st) {
  StreamList one;
  PoolKey k;
  k.device = device;
  k.kind = SK_PLAIN;
  one.push_back({k, st});
  pool_return(one);
}
}  // namespace mk
// Hardware queues of this process's HIP runtime (mk_set_hw_queues; -1: GPU_MAX_HW_QUEUES as set in
// the environment, HIP's default 4 when unset).
static std::atomic<int> g_hw_queues{-1};
static int hw_queues() {
  const int n = g_hw_queues.load();
  if (n >= 0) return n;
  const char* v = std::getenv("GPU_MAX_HW_QUEUES");
  return (v && *v) ? std::atoi(v) : 4;
}
extern "C" int mk_set_hw_queues(int32_t n) {
  g_hw_queues.store(n < 0 ? -1 : n);
  return 0;
}

struct mk_session {
  mk_session() { g_live_sessions.fetch_add(1); }
  int device = 0;
  hipStream_t stream = nullptr;   // set-up, outputs and the one-group paths
  StreamList owned;               // every stream of the session (pool_stream), back to the pool at the end
  Model md{};
  MatSet ms{};
  int S = 0, q = 1, p = 0, n_pad = 0, nt = 0, P = 0;
  int iter = 0;
  bool matern = false, record_samples = true, record_w = false;
  bool pred_gen = false;          // kriging P^T generated inside k_pred_var (exponential; no P^T buffer)
  Group all;                      // the whole shard on `stream`
  bool tiled = false;             // kriging after the fit over test-site tiles (predict_tile)
  int pred_tile = 0, n_test_all = 0, n_test_pad_all = 0;
  int tile_req = 0;               // predict_tile as configured
  int win_lo = 0, win_n = -1;     // tiled kriging: kept states [win_lo, win_lo + win_n) (-1: all)
  // phi-interpolated tiled kriging (predict_tile_cheb): the window's g_k = W_k' z_k and phi_k, kept
  // across tiles (made at the first tile after a run or a window change)
  double* cg_G = nullptr;         // [S][n_pad][nkp]: g of the window's states (nkp = window rounded up to 8)
  double* cg_phi = nullptr;       // [win][S]
  double* cg_phit = nullptr;      // [S][nkp]: phi per state, padded with the last
  std::vector<double> cg_phi_h;
  int cg_iter = -1, cg_lo = -1, cg_n = -1;
  std::vector<double> span_pt_h;  // [S] bound on the subset-site to test-site distances (host copy)
  // fused kriging from phi tables (krig_tables; exponential, q = 1, one group): s(t; phi) at Chebyshev
  // nodes of the prior's phi range, made at session creation; kept iterations interpolate them
  bool kt_on = false;
  int kt_fail = 0;                // set-up checks that failed (the session then refreshes X exactly)
  double kt_check = 0.0, kt_evals = 0.0;
  ChebK kt{};
  double* kt_g = nullptr;         // [S][n_pad] g = W' z of the current kept iteration
  double* kt_z = nullptr;         // [S][n_pad + 2]: its z, then phi and A per subset (k_kt_snap)
  hipEvent_t kt_ev[2] = {nullptr, nullptr};   // [0] snapshot taken, [1] draws done (side stream)
  bool kt_pending = false;        // draws queued on the side stream, not yet waited for
  std::vector<void*> kbufs;       // the kriging buffers (re-sized by mk_session_set_test_sites)
  std::vector<double> bbox;       // [S][4] xmin xmax ymin ymax of each subset's sites (Matern table ranges)
  double* d_ct_all = nullptr;     // all test sites [2][n_test_pad_all] (tiled mode)
  int* d_slist = nullptr;         // tiled replay: per-outcome subset lists [q][S] + counts [q]
  int* d_run_start = nullptr;     // tiled replay, q = 1: first window state of each subset's pending draws
  int* d_scount = nullptr;
  std::vector<Group> groups;      // the run-time split, one stream each
  // The latent sweep (launch_sweep).  sweep_site: the one-pass site sweep (default; row pairs per
  // thread, 0: off) with its LDS and lean form; else, for multi-outcome small shards, the split-launch
  // multi-workgroup kernel behind its admission consensus, k_sweep sweeping the subsets it did not
  // admit (sweep_coop), or the split-launch sweep (sweep_split: no inter-workgroup waits);
  // else the 64-site-block kernel (k_sweep, one workgroup per subset).
  int sweep_site = 0;
  size_t sweep_site_lds = 0;
  int sweep_lean = 0;             // q = 1: 1 border row by factor, 2 every n_s even (sweep_site_kernel)
  bool sweep_split = false;       // k_sweep_step, one launch per 64-site block
  bool sweep_coop = false;        // k_sweep_mg (admission consensus) + k_sweep for the subsets not admitted
  size_t sweep_mg_lds = 0;
  double* sp_part = nullptr;
  hipEvent_t swept = nullptr;     // fork-join sweep (several groups): the whole-shard sweep is queued
  double* sw_part = nullptr;
  int* sw_cnt = nullptr;           // [S][n_pad / 64] block counters, then [S] admission words (sw_adm)
  int* sw_adm = nullptr;
  int adm_spins = MK_ADM_SPINS;
  int* sw_xcc = nullptr;
  int* sw_err = nullptr;
  double* d_probs = nullptr;
  // Lookahead schedule (exponential model, one group; run_iteration_la): iteration t+1's phi
  // candidates are factored on la_c while iteration t's inverse and sweep run on the main stream,
  // and their z' = L'^-1 u is solved on la_x trailing the factorisation panel by panel.
  int la_mode = -1;               // mk_session_set_lookahead: -1 auto, 0 off, 1 on
  bool la_ok = false;             // eligible (buffers allocated)
  bool la = false;                // in use
  int la_next = -1;               // iteration whose candidates are queued on la_c (-1: none)
  // Sequential schedule, one group (MK_EARLY_COV, default on): iteration t+1's phi candidates are
  // assembled (without the bordered row) on cov_st beside iteration t's sweep; iteration t+1 writes
  // the row once its A step has produced u (k_cand_border) and factors as usual -- the same matrices.
  int cov_pre = -1;               // iteration whose candidates cov_st has assembled (-1: none)
  hipStream_t cov_st = nullptr;
  hipEvent_t cov_ev[2] = {nullptr, nullptr};   // [0] main stream ready for it, [1] assembled
  int la_enq = 0;                 // panels of those candidates enqueued so far
  hipStream_t la_m = nullptr;     // MK_LA_MASK: CU-masked main stream of the lookahead iterations
  hipStream_t la_c = nullptr;     // created at the first lookahead run (an unused stream still takes a
                                  // hardware queue, GPU_MAX_HW_QUEUES = 4, and slows the split Cholesky)
  hipStream_t la_k = nullptr;     // kept iterations' kriging refresh beside the sweep (MK_LA_KRIG)
  std::vector<hipEvent_t> la_ev;  // [nt] panel k final | decided (or adapted) | join | W ready | kriged
  hipError_t launch_err = hipSuccess;   // first failed kernel launch of a run
  const char* poisoned = nullptr;       // set when a run left the chain in a state that is not the sampler's
  std::vector<int> n_part;
  std::vector<void*> allocs;
  bool prof = false;
  uint32_t prof_kinds = ~0u;   // kernel kinds bracketed by events while prof (bit per KS_ kind)
  int prof_every = 1;          // bracket the launches of every prof_every-th iteration only
  bool prof_iter = true;       // this iteration's launches are bracketed (mk_session_run)
  std::vector<Timed> pending;
  // KS_INV timing: the inverse's work list length lives on the device, so each timed inverse copies
  // its count into a pinned slot in stream order; drain_timers prices the launches with it
  static constexpr int INV_CNT_CAP = 65536;
  int* inv_cnt = nullptr;
  int inv_cnt_used = 0;
  Stat stats[NKSTAT];

  // Free one buffer allocated by alloc().
  void release(void* ptr) {
    if (!ptr) return;
    for (size_t i = 0; i < allocs.size(); ++i)
      if (allocs[i] == ptr) {
        hipFree(ptr);
        allocs.erase(allocs.begin() + (long)i);
        return;
      }
  }
  template <typename T>
  int alloc(T** p_, size_t n) {
    void* ptr = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&ptr, n * sizeof(T));
    if (e != hipSuccess) {
      (void)hipGetLastError();   // the failed malloc is sticky in hipGetLastError: clear it for later calls
      return set_err(MK_E_NOMEM, std::string("hipMalloc ") + std::to_string(n * sizeof(T)) + " B");
    }
    allocs.push_back(ptr);
    *p_ = (T*)ptr;
    return 0;
  }
  // Teardown order: drain every stream first (no queued work may still reference an event or a
  // buffer), then destroy the events the streams recorded, then the streams (CU-masked and
  // priority queues included), then free the memory.
  ~mk_session() {
    g_live_sessions.fetch_sub(1);
    if (device >= 0) hipSetDevice(device);
    for (auto& o : owned) hipStreamSynchronize(o.second);
    for (auto& t : pending) { hipEventDestroy(t.a); hipEventDestroy(t.b); }
    if (inv_cnt) hipHostFree(inv_cnt);
    for (auto& g : groups) {
      if (g.done) hipEventDestroy(g.done);
      for (hipEvent_t e : g.ev) hipEventDestroy(e);
    }
    if (swept) hipEventDestroy(swept);
    for (hipEvent_t e : cov_ev)
      if (e) hipEventDestroy(e);
    for (hipEvent_t e : kt_ev)
      if (e) hipEventDestroy(e);
    for (hipEvent_t e : la_ev) hipEventDestroy(e);
    pool_return(owned);   // drained above; their waits on the destroyed events are satisfied
    for (void* p_ : allocs) hipFree(p_);
    (void)hipGetLastError();   // teardown errors are not the next call's
  }
};

static hipEvent_t ev_new() {
  hipEvent_t e;
  hipEventCreate(&e);
  return e;
}

// Launch helper that optionally brackets a kernel with events on its stream.
template <typename F>
static void timed(mk_session* s, hipStream_t st, int which, double flops, F&& launch, int cnt = -1) {
  if (!s->prof || !s->prof_iter || !((s->prof_kinds >> which) & 1u)) {
    launch();
    return;
  }
  Timed t{which, ev_new(), ev_new(), flops, cnt};
  hipEventRecord(t.a, st);
  launch();
  hipEventRecord(t.b, st);
  s->pending.push_back(t);
}

static void drain_timers(mk_session* s) {
  std::vector<std::pair<float, float>> upd;   // update launches: [start, end] relative to the first event
  for (auto& t : s->pending) {
    hipEventSynchronize(t.b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, t.a, t.b);
    if (t.cnt >= 0) t.flops *= (double)s->inv_cnt[t.cnt];
    s->stats[t.which].launches += 1;
    s->stats[t.which].ms += ms;
    s->stats[t.which].flops += t.flops;
    if (t.which == KS_CHOL_UPDATE || t.which == KS_CHOL_UPDATE_SUB) {
      float t0 = 0.f;
      hipEventElapsedTime(&t0, s->pending.front().a, t.a);
      upd.push_back({t0, t0 + ms});
      s->stats[KS_UPDATE_BUSY].launches += 1;
      s->stats[KS_UPDATE_BUSY].flops += t.flops;
    }
  }
  std::sort(upd.begin(), upd.end());
  double busy = 0.0, lo = 0.0, hi = -1.0;
  for (auto& iv : upd) {
    if (iv.first > hi) {
      if (hi > lo) busy += hi - lo;
      lo = iv.first;
      hi = iv.second;
    } else {
      hi = std::max(hi, (double)iv.second);
    }
  }
  if (hi > lo) busy += hi - lo;
  s->stats[KS_UPDATE_BUSY].ms += busy;
  for (auto& t : s->pending) {
    hipEventDestroy(t.a);
    hipEventDestroy(t.b);
  }
  s->pending.clear();
  s->inv_cnt_used = 0;
}

static inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

// Every tile-GEMM kernel takes gb_lds_bytes(TM, TN) of dynamic LDS: two DMA stages (> 64 KiB at 128 x 128).
static constexpr size_t LDS_128 = gb_lds_bytes(128, 128), LDS_64 = gb_lds_bytes(64, 64),
                        LDS_64x128 = gb_lds_bytes(64, 128), LDS_32 = gb_lds_bytes(32, 32),
                        LDS_32x128 = gb_lds_bytes(32, 128);
static bool set_gemm_lds() {
  const std::pair<const void*, size_t> fns[] = {
      {(const void*)k_chol_update<128>, LDS_128}, {(const void*)k_chol_update<64>, LDS_64},
      {(const void*)k_chol_trsm<128>, LDS_128},   {(const void*)k_chol_trsm<64>, LDS_64x128},
      {(const void*)k_inv_level<128>, LDS_128},   {(const void*)k_inv_level<64>, LDS_64},
      {(const void*)k_chol_update<32>, LDS_32},   {(const void*)k_chol_trsm<32>, LDS_32x128},
      {(const void*)k_chol_update_trsm<128>, LDS_128}, {(const void*)k_chol_update_trsm<64>, LDS_128},
      {(const void*)k_inv_level<32>, LDS_32},
      {(const void*)k_qblocks, LDS_64},           {(const void*)k_lauum, LDS_128},
      {(const void*)k_pred_var<true>, LDS_128},   {(const void*)k_pred_var<false>, LDS_128}};
  for (const auto& f : fns)
    if (hipFuncSetAttribute(f.first, hipFuncAttributeMaxDynamicSharedMemorySize, (int)f.second) != hipSuccess)
      return false;
  return true;
}

// Type-7 quantiles of n_rows kept values per (subset, column) (k_quantiles): the bitonic sort takes
// the next power of two >= n_rows doubles of dynamic LDS (n_rows <= MK_QUANT_MAX).
static int launch_quantiles(unsigned grid, hipStream_t st, const double* data, long subset_stride, long row_stride,
                            int n_rows, int n_cols, const double* probs, int n_probs, double* out) {
  HIPCHK(hipFuncSetAttribute((const void*)k_quantiles, hipFuncAttributeMaxDynamicSharedMemorySize, MK_QUANT_MAX * 8));
  if (n_rows < 1 || n_rows > MK_QUANT_MAX)
    return set_err(MK_E_ARG, "quantile summaries take 1 .. " + std::to_string(MK_QUANT_MAX) + " kept samples");
  size_t n2 = 1;
  while (n2 < (size_t)n_rows) n2 <<= 1;
  MK_LAUNCH(k_quantiles, dim3(grid), dim3(256), n2 * 8, st, data, subset_stride, row_stride, n_rows, n_cols,
                     probs, n_probs, out);
  HIPCHK(hipGetLastError());
  return 0;
}

// Tile shape of a GEMM launch: 64-sub-tiles (bit-identical, mk_gemm.hpp) when the 128-tile grid
// would leave the chip short of work -- fewer than MK_TILE_THRESH workgroups (default 256, one per
// CU; 512 before the lookahead schedule, whose concurrent chain fills the rest: 32 subsets
// 6,360 -> 6,546 subset-iters/s, 250 subsets unchanged).  MK_TILE=128 / 64 / 32 forces one shape (tests compare them; 32-sub-tiles were measured no
// faster than 64 on the last, single-tile panels of small shards, so the policy does not pick them).
static int tile_env(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}
static int tile_size(long wg128) {
  static const int force = tile_env("MK_TILE", 0);
  static const int thresh = tile_env("MK_TILE_THRESH", 256);
  if (force == 32 || force == 64 || force == 128) return force;
  return wg128 >= thresh ? 128 : 64;
}

// ------------------------------------------------------------------ candidate assembly
// Candidate matrices of n_entries (subset, outcome) entries (k_cov_candidate); Matern sessions
// first store each entry's Chebyshev table (k_matern_table, one workgroup per entry), which the
// tile workgroups then load.
static void launch_candidates(const Model& md, const MatSet& ms, hipStream_t st, int n_entries, int h0, int hc,
                              int which, int iter, const int* slist = nullptr, const int* scount = nullptr) {
  if (md.cov_model == MK_COV_MATERN && md.chtab)
    MK_LAUNCH(k_matern_table, dim3(n_entries), dim3(256), 0, st, md, h0, hc, which, iter, slist, scount);
  const int ntiles = ms.nt * (ms.nt + 1) / 2;
  MK_LAUNCH(cov_candidate_kernel(md.cov_model), dim3(xcd_grid_h(n_entries, ntiles)),
                     dim3(256), 0, st, md, ms, h0, hc, which, iter, slist, scount);
}

// ------------------------------------------------------------------ Cholesky of all candidates of outcome h
// Candidate tiles are in the free slot (k_cov_candidate, or k_load_plain for the test entry).
// One launch per step covers outcomes h0 .. h0+hc-1 of every subset (hc = q in the sampler).
// Launch pieces of the blocked Cholesky for panel k, tiles [ia, ib), on stream st.

static void chol_update(mk_session* s, Group& g, hipStream_t st, int h0, int hc, int k, int ia, int ib, int j0, int j1,
                        const int* slist, const int* scount, double flops) {
  const int E = g.S * hc, nti = ib - ia;
  if (nti <= 0) return;
  const int tm = tile_size((long)E * nti);
  if (tm == 32) {
    timed(s, st, KS_CHOL_UPDATE_SUB, flops, [&] {
      MK_LAUNCH(k_chol_update<32>, dim3(xcd_grid_h(E, nti * 16)), dim3(256), LDS_32, st, g.ms, g.S, h0, hc, k, ia,
                         ib, j0, j1, slist, scount);
    });
  } else if (tm == 64) {
    timed(s, st, KS_CHOL_UPDATE_SUB, flops, [&] {
      MK_LAUNCH(k_chol_update<64>, dim3(xcd_grid_h(E, nti * 4)), dim3(256), LDS_64, st, g.ms, g.S, h0, hc, k, ia,
                         ib, j0, j1, slist, scount);
    });
  } else {
    timed(s, st, KS_CHOL_UPDATE, flops, [&] {
      MK_LAUNCH(k_chol_update<128>, dim3(xcd_grid_h(E, nti)), dim3(256), LDS_128, st, g.ms, g.S, h0, hc, k, ia,
                         ib, j0, j1, slist, scount);
    });
  }
}
static void chol_trsm(mk_session* s, Group& g, hipStream_t st, int h0, int hc, int k, int ia, int ib, const int* slist,
                      const int* scount, double flops) {
  const int E = g.S * hc, nti = ib - ia;
  if (nti <= 0) return;
  const int tm = tile_size((long)E * nti);
  timed(s, st, KS_CHOL_TRSM, flops, [&] {
    if (tm == 32)
      MK_LAUNCH(k_chol_trsm<32>, dim3(xcd_grid_h(E, nti * 4)), dim3(256), LDS_32x128, st, g.ms, g.S, h0, hc, k,
                         ia, ib, slist, scount);
    else if (tm == 64)
      MK_LAUNCH(k_chol_trsm<64>, dim3(xcd_grid_h(E, nti * 2)), dim3(256), LDS_64x128, st, g.ms, g.S, h0, hc, k,
                         ia, ib, slist, scount);
    else
      MK_LAUNCH(k_chol_trsm<128>, dim3(xcd_grid_h(E, nti)), dim3(256), LDS_128, st, g.ms, g.S, h0, hc, k, ia, ib,
                         slist, scount);
  });
}
// F(k): column k's update of tiles k+1.. by panels [j0, k) with the panel solve in the epilogue
// (k_chol_update_trsm, 1 <= k < nt - 1), plus (extra) the next diagonal tile's update by panels [0, k).
static void chol_update_trsm(mk_session* s, Group& g, hipStream_t st, int h0, int hc, int k, int j0, int extra,
                             const int* slist, const int* scount, double flops) {
  const int E = g.S * hc, nt = s->nt, nti = nt - (k + 1);
  const int tm = tile_size((long)E * (nti + extra));
  timed(s, st, tm == 128 ? KS_CHOL_UPDATE : KS_CHOL_UPDATE_SUB, flops, [&] {
    if (tm == 128)
      MK_LAUNCH(k_chol_update_trsm<128>, dim3(xcd_grid_h(E, nti + extra)), dim3(256), LDS_128, st, g.ms, g.S, h0, hc,
                k, k + 1, nt, j0, extra, slist, scount);
    else
      MK_LAUNCH(k_chol_update_trsm<64>, dim3(xcd_grid_h(E, 2 * nti + extra)), dim3(256), LDS_128, st, g.ms, g.S, h0,
                hc, k, k + 1, nt, j0, extra, slist, scount);
  });
}
// cj0 < cj1: the diagonal tile's update by panels [cj0, cj1) first, in the same launch (fused form).
static void chol_diag(mk_session* s, Group& g, hipStream_t st, int h0, int hc, int k, const int* slist,
                      const int* scount, int cj0 = 0, int cj1 = 0, double flops = 0.0) {
  timed(s, st, KS_CHOL_DIAG, flops, [&] {
    MK_LAUNCH(k_chol_diag, dim3(g.S * hc), dim3(256), (size_t)MK_DIAG_LDS_BYTES, st, g.ms, g.md.n_s, h0, hc, k,
                       g.md.ld_part, g.md.quad_c, g.md.info, slist, scount, cj0, cj1);
  });
}

// Algorithmic flops of the column-k update over panels [j0, j1) (trsm: of panel k) of tiles
// [ia, ib): every (subset, outcome) factor counted over its own valid extent n_s + 1 (the
// bordered row; padding excluded), so ragged subsets (MK.R:18: the last takes the remainder) are
// priced exactly.  Algorithmic, not executed: an off-diagonal tile's update is a GEMM,
// 2 rows cols depth; the diagonal tile's (tile k of column k) a SYRK, cols (cols + 1) depth; the
// panel solve L(i,k) = C(i,k) L(k,k)^-T a triangular solve, rows cols^2 (the kernels skip most of the
// triangle's zero MFMA blocks but not all of them: what they execute is more than this).  With a
// subset list (tiled kriging replay) the active subsets live on the device: the count is then an
// upper bound (every subset).
static double panel_flops(mk_session* s, Group& g, int hc, int k, int ia, int ib, bool trsm, int j0 = 0, int j1 = -1) {
  if (j1 < 0) j1 = k;
  double fl = 0.0;
  for (int i = g.s0; i < g.s0 + g.S; ++i) {
    const double nv = (double)s->n_part[i] + 1.0;
    const double cols = std::fmin((double)MK_NB, std::fmax(0.0, nv - (double)k * MK_NB));
    const double depth = std::fmax(0.0, std::fmin((double)j1 * MK_NB, nv) - (double)j0 * MK_NB);
    const bool diag = ia <= k && k < ib;   // tile k of column k is in [ia, ib)
    const double lo = (double)(diag ? k + 1 : ia) * MK_NB;
    const double rows = std::fmax(0.0, std::fmin(nv, (double)ib * MK_NB) - lo);   // off-diagonal rows
    if (trsm)
      fl += rows * cols * cols;
    else
      fl += 2.0 * rows * cols * depth + (diag ? cols * (cols + 1.0) * depth : 0.0);
  }
  return fl * hc;
}

// Algorithmic flops of one factor's inverse level (k_inv_level, level sz, phase): over the pairs of
// blocks T = tiles [T0, T0+sz), B = [T0+sz, T0+2sz) clipped to the extent n, phase 0 Y = L_BT W_TT is
// a full-by-triangular product (|B| |T|^2), phase 1 W_BT = -W_BB Y a triangular-by-full one (|B|^2 |T|).
// Summed over the levels with the diagonal tiles' inverses (k_chol_diag's) this is n^3 / 3.
static double inv_level_flops(int n, int nt, int sz, int phase) {
  double fl = 0.0;
  for (int T0 = 0; T0 < nt; T0 += 2 * sz) {
    const double t0 = (double)T0 * MK_NB, b0 = (double)(T0 + sz) * MK_NB, b1 = (double)(T0 + 2 * sz) * MK_NB;
    const double bt = std::fmax(0.0, std::fmin((double)n, b0) - t0), bb = std::fmax(0.0, std::fmin((double)n, b1) - b0);
    fl += phase == 0 ? bb * bt * bt : bb * bb * bt;
  }
  return fl;
}

// Cholesky of all candidates of outcomes h0 .. h0+hc-1 (candidate tiles in the free slot), left-
// looking by 128-panels: per column k the update by panels < k, the diagonal tile, the trsm of
// tiles k+1.. .
//
// Sequential form (one stream): U(k; panels 0..k-1), D(k), T(k).  Fused (MK_CHOL_FUSED, default on;
// 0 restores U, D, T): D(0), T(0), then per k >= 1
//   D(k)  the diagonal tile's last panel k-1 (its panels [0, k-1) came with F(k-1); k = 1: panel 0)
//         applied inside the diagonal launch, then the factor,
//   F(k)  tiles k+1.. of column k, update and solve in one launch (C(i,k) stays in registers), plus
//         the next diagonal tile by panels [0, k)
// -- no C(i,k) round trip through HBM between the update and the solve; same bits.  (The split form
// below stays unfused: there F(k) would put the off-diagonal tiles' critical correction after the
// diagonal factor instead of beside the diagonal tile's -- a longer chain; 32 subsets 7,479-7,597 vs
// 8,059-8,078 subset-iters/s)
//
// Split form (small shards, g.bulk set): the update of column c by panels 0..c-2 only needs
// panels that are final two steps earlier, so it runs on the CU-masked bulk stream beside the
// critical chain, which keeps only the rank-128 correction by panel c-1:
//   critical (g.stream, all CUs):  U(k; k-1) [after bulk U(k; 0..k-2)], D(k), T(k)
//   bulk (g.bulk, CUs minus the first `reserve`): U(k+2; 0..k) after T(k)
// The diagonal kernel (one 149 KB-LDS workgroup per matrix) then finds idle CUs at once instead
// of waiting for update workgroups to drain.  Same kernels, same per-element MFMA sequence (the
// accumulator passes through fp64 memory between the two updates): same bits.  (An earlier
// lookahead that moved the full-depth update of the next diagonal tile onto a second stream was
// slower: that update's long K chain sat on the critical path)
//
// crit: the critical stream (default g.stream; the lookahead schedule factors on its own stream).
// evP (optional, nt events): evP[k] is recorded on it once panel k is final (after T(k); the last
// after D(nt-1)), for the border solve that trails the factorisation.
// [k_lo, k_hi): the panels to enqueue (the lookahead schedule enqueues a factorisation in two
// pieces around the main stream's work, so the host does not hold back either stream).
static void launch_cholesky(mk_session* s, Group& g, int h0, int hc, const int* slist = nullptr,
                            const int* scount = nullptr, hipStream_t crit = nullptr, hipEvent_t* evP = nullptr,
                            int k_lo = 0, int k_hi = -1) {
  const int nt = s->nt;
  if (k_hi < 0) k_hi = nt;
  hipStream_t A = crit ? crit : g.stream;
  static const int fused = tile_env("MK_CHOL_FUSED", 1);
  if ((slist || !g.bulk) && fused) {
    for (int k = k_lo; k < k_hi; ++k) {
      // X(k) inside D(k): the diagonal tile's last panel (k = 1: panel 0) before it factors
      const int j0 = k >= 2 ? k - 1 : 0;
      chol_diag(s, g, A, h0, hc, k, slist, scount, j0, k, k > 0 ? panel_flops(s, g, hc, k, k, k + 1, false, j0, k) : 0.0);
      if (k == 0 && nt > 1)
        chol_trsm(s, g, A, h0, hc, 0, 1, nt, slist, scount, panel_flops(s, g, hc, 0, 1, nt, true));
      else if (k > 0 && k < nt - 1)
        chol_update_trsm(s, g, A, h0, hc, k, 0, 1, slist, scount,
                         panel_flops(s, g, hc, k, k + 1, nt, false) + panel_flops(s, g, hc, k, k + 1, nt, true) +
                             panel_flops(s, g, hc, k + 1, k + 1, k + 2, false, 0, k));
      if (evP) hipEventRecord(evP[k], A);
    }
    return;
  }
  if (slist || !g.bulk) {
    for (int k = k_lo; k < k_hi; ++k) {
      if (k > 0)
        chol_update(s, g, A, h0, hc, k, k, nt, 0, k, slist, scount, panel_flops(s, g, hc, k, k, nt, false));
      chol_diag(s, g, A, h0, hc, k, slist, scount);
      if (k < nt - 1)
        chol_trsm(s, g, A, h0, hc, k, k + 1, nt, slist, scount, panel_flops(s, g, hc, k, k + 1, nt, true));
      if (evP) hipEventRecord(evP[k], A);
    }
    return;
  }
  // depth d (MK_CHOL_DEPTH, default 2): the bulk update of column c covers panels [0, c-d) and is
  // launched after T(c-d-1), so it has d critical steps to finish; the critical correction is
  // then rank-128d, U(k; k-d..k-1).  Same per-element MFMA sequence for any d (same bits).
  static const int depth_env = tile_env("MK_CHOL_DEPTH", 2);
  const int d = std::max(1, std::min(depth_env, 4));
  hipStream_t B = g.bulk;
  hipEvent_t* eT = g.ev.data();                  // eT[k]: T(k) done (critical)
  hipEvent_t* eU = g.ev.data() + nt;             // eU[c]: bulk U(c; 0..c-d-1) done, c = d+1 .. nt-1
  if (k_lo == 0) {
    hipEventRecord(g.ev[2 * nt], A);             // the candidates are on A
    hipStreamWaitEvent(B, g.ev[2 * nt], 0);
  }
  for (int k = k_lo; k < k_hi; ++k) {
    if (k > d) hipStreamWaitEvent(A, eU[k], 0);
    if (k >= 1) {
      const int j0 = std::max(0, k - d);
      chol_update(s, g, A, h0, hc, k, k, nt, j0, k, nullptr, nullptr, panel_flops(s, g, hc, k, k, nt, false, j0, k));
    }
    chol_diag(s, g, A, h0, hc, k, nullptr, nullptr);
    if (k < nt - 1)
      chol_trsm(s, g, A, h0, hc, k, k + 1, nt, nullptr, nullptr, panel_flops(s, g, hc, k, k + 1, nt, true));
    if (evP) hipEventRecord(evP[k], A);
    if (k + d + 1 < nt) {
      const int c = k + d + 1;
      hipEventRecord(eT[k], A);
      hipStreamWaitEvent(B, eT[k], 0);
      chol_update(s, g, B, h0, hc, c, c, nt, 0, c - d, nullptr, nullptr, panel_flops(s, g, hc, c, c, nt, false, 0, c - d));
      hipEventRecord(eU[c], B);
    }
  }
}

// W = L^-1 of the listed pairs: diagonal tiles, then recursive doubling.
static void launch_trinv(mk_session* s, Group& g, int max_entries, const int* list, const int* count) {
  const int nt = s->nt;
  MK_LAUNCH(k_inv_copydiag, dim3(max_entries * nt * MK_CD_SPLIT), dim3(256), 0, g.stream, g.ms, list, count);
  // profiled: the listed count in stream order into a pinned slot (drain_timers multiplies the
  // per-factor flops below by it); no slot left -> the launches run untimed
  int cnt = -1;
  if (s->prof && s->prof_iter && ((s->prof_kinds >> KS_INV) & 1u)) {
    if (!s->inv_cnt && hipHostMalloc((void**)&s->inv_cnt, mk_session::INV_CNT_CAP * sizeof(int)) != hipSuccess) {
      (void)hipGetLastError();
      s->inv_cnt = nullptr;
    }
    if (s->inv_cnt && s->inv_cnt_used < mk_session::INV_CNT_CAP) {
      cnt = s->inv_cnt_used++;
      hipMemcpyAsync(s->inv_cnt + cnt, count, sizeof(int), hipMemcpyDeviceToHost, g.stream);
    }
  }
  for (int sz = 1; sz < nt; sz *= 2) {
    const int npairs = (nt + 2 * sz - 1) / (2 * sz);
    // the grid is sized for every pair, but only the accepted candidates' factors are in the
    // list (about 40% at the amcmc target rate) and the level's K ranges are uneven: price the
    // launch at an eighth of its 128-tile grid (measured: 32 subsets 1.33 -> 1.16 ms per iteration)
    const int tm = tile_size((long)max_entries * npairs * sz * sz / 8);
    for (int phase = 0; phase < 2; ++phase) {
      // per listed factor: the mean over the group's subsets (exact for equal subset sizes)
      double per = 0.0;
      if (cnt >= 0) {
        for (int i = g.s0; i < g.s0 + g.S; ++i) per += inv_level_flops(s->n_part[i], nt, sz, phase);
        per /= std::max(1, g.S);
      }
      auto launch = [&] {
        if (tm == 32)
          MK_LAUNCH(k_inv_level<32>, dim3(xcd_grid_h(max_entries, npairs * sz * sz * 16)), dim3(256), LDS_32,
                             g.stream, g.ms, list, count, sz, phase);
        else if (tm == 64)
          MK_LAUNCH(k_inv_level<64>, dim3(xcd_grid_h(max_entries, npairs * sz * sz * 4)), dim3(256), LDS_64,
                             g.stream, g.ms, list, count, sz, phase);
        else
          MK_LAUNCH(k_inv_level<128>, dim3(xcd_grid_h(max_entries, npairs * sz * sz)), dim3(256), LDS_128,
                             g.stream, g.ms, list, count, sz, phase);
      };
      if (cnt >= 0)
        timed(s, g.stream, KS_INV, per, launch, cnt);
      else
        launch();     // not profiled, or no count slot (untimed: the stats' ms and flops stay paired)
    }
  }
}

// W = L^-1 for the changed factors, diagonal tiles of R^-1, z from the bordered row.
static void launch_inverse(mk_session* s, Group& g, bool from_zc = false) {
  const int nt = s->nt, max_entries = g.S * s->q;
  launch_trinv(s, g, max_entries, g.d_list, g.d_count);
  // the diagonal tiles of R^-1 feed the 64-site-block sweeps only; the site sweep reads W alone
  if (!s->sweep_site)
    timed(s, g.stream, KS_LAUUM, 0.0, [&] {
      MK_LAUNCH(k_qblocks, dim3(xcd_grid_h(max_entries, nt * 2)), dim3(256), LDS_64, g.stream, g.ms, g.md.n_s,
                g.d_list, g.d_count);
    });
  MK_LAUNCH(k_take_border, dim3(max_entries * ((s->n_pad + 255) / 256)), dim3(256), 0, g.stream, g.md, g.ms,
                     g.d_list, g.d_count, from_zc ? (const double*)g.md.zc : nullptr);
}

// Algorithmic flops of k_pred_var over every pair of the group: 2 n_s^2 / 2 per test site (W
// lower-triangular) -- an upper bound, the list holds the pairs whose factor changed.
static double pred_flops(mk_session* s, Group& g) {
  double fl = 0.0;
  for (int i = g.s0; i < g.s0 + g.S; ++i) fl += (double)s->n_part[i] * s->n_part[i] * g.md.n_test;
  return fl * s->q;
}

// Kriging refresh (kept iterations): X = W P^T and s = |X_t|^2 for the pairs in the pred list
// (P^T generated in the GEMM for the exponential model, else stored first by k_pred_PT).
static void launch_pred_refresh(mk_session* s, Group& g, hipStream_t st = nullptr) {
  Model& md = g.md;
  if (md.n_test <= 0) return;
  if (!st) st = g.stream;
  const int nt = s->nt, max_entries = g.S * s->q;
  if (md.cov_model == MK_COV_MATERN && md.chtab_p)
    MK_LAUNCH(k_matern_table_list, dim3(max_entries), dim3(256), 0, st, md, g.d_plist, g.d_pcount);
  if (md.cov_model == MK_COV_MATERN)
    MK_LAUNCH(k_pred_PT_matern, dim3(max_entries * (md.n_pad / MK_PT_RB)), dim3(256), 0, st, md, g.d_plist,
                       g.d_pcount);
  else if (!s->pred_gen)
    MK_LAUNCH(pred_PT_kernel(md.cov_model), dim3(max_entries * md.n_pad), dim3(256), 0, st, md, g.d_plist,
                       g.d_pcount);
  timed(s, st, KS_PRED_VAR, pred_flops(s, g), [&] {
    MK_LAUNCH(s->pred_gen ? k_pred_var<true> : k_pred_var<false>, dim3(pv_grid(max_entries, nt, md.ntt)),
              dim3(256), LDS_128, st, md, g.ms, g.d_plist, g.d_pcount);
  });
  MK_LAUNCH(k_pred_var_reduce, dim3(max_entries * (md.n_test_pad / 256)), dim3(256), 0, st, md, nt,
                     g.d_plist, g.d_pcount);
}

// The latent-w sweep: the multi-workgroup kernel when the session chose it (small shard; g is then
// the whole-shard view), else the site sweep or one workgroup per subset; the block sweeps give the
// same bits (mk_mcmc.hip).
// Default schedule: lookahead for shards of up to 224 (subset, outcome) pairs, where the chains
// leave the chip room to overlap (measured vs sequential: 32 subsets 5,427 -> 6,972, 63 6,174 ->
// 7,719, 125 7,486 -> 8,303, 188 8,071 -> 8,486 subset-iters/s); at 250 subsets both saturate the
// chip and the sequential schedule is as fast (8,572 vs 8,553-8,565) while its panel-update
// launches run alone (roofline timing 0.71 of peak vs 0.52-0.57 beside the main stream's kernels).
// Round 4 (lean sweep): at 250 subsets the lookahead schedule gains 0.9 % (10,574-10,579 sequential vs
// 10,660-10,686, three interleaved 40-step windows each, profiles/r04/la250/) but its update launches
// share the chip, so each launch's own rate reads ~0.55 instead of ~0.70 of peak; the sequential
// schedule stays the default there (MK_LOOKAHEAD=1 takes the 0.9 %).
static bool la_auto(const mk_session* s) { return (long)s->S * s->q <= 224; }

// The multi-workgroup sweep is a plain launch on either schedule: its admission consensus
// (k_sweep_mg) sweeps a subset only once all its workgroups are resident, and the k_sweep launch
// queued behind it sweeps the rest -- no wait depends on co-residency the hardware does not give.
// (Round 4 had relied on the workgroups becoming resident eventually; round 5's first answer ran the
// kernel only as a cooperative launch, i.e. not beside the lookahead schedule's other streams.)
static bool use_sweep_mg(const mk_session* s) { return s->sweep_coop; }

static void launch_sweep(mk_session* s, Group& g, int it) {
  const int q = s->q;
  Model md = g.md;
  MatSet ms = g.ms;
  int iter = it;
  hipError_t e = hipSuccess;
  if (s->sweep_site) {
    void* args[] = {&md, &ms, &iter};
    e = hipLaunchKernel(sweep_site_kernel(q, s->sweep_site, s->sweep_lean), dim3(g.S), dim3(MK_SS_T), args,
                        s->sweep_site_lds, g.stream);
    wd_trace(g.stream, "k_sweep_site");
  } else if (use_sweep_mg(s)) {
    hipMemsetAsync(s->sw_cnt, 0, (size_t)s->S * (s->n_pad / 64 + 1) * sizeof(int), g.stream);   // g: the whole shard
    double* part = s->sw_part;
    int* cnt = s->sw_cnt;
    int* xcc = s->sw_xcc;
    int* err = s->sw_err;
    int* adm = s->sw_adm;
    int spins = s->adm_spins;
    void* args[] = {&md, &ms, &iter, &part, &cnt, &xcc, &err, &adm, &spins};
    e = hipLaunchKernel(sweep_kernel(q, true), dim3(xcd_grid(g.S, s->nt)), dim3(256), args, s->sweep_mg_lds,
                        g.stream);
    wd_trace(g.stream, "k_sweep_mg");
    if (e == hipSuccess) {   // the subsets k_sweep_mg did not admit (normally none: every workgroup returns at once)
      const size_t sw_lds = (size_t)q * (64 * 64 + 2 * 64) * sizeof(double);
      const int* cadm = adm;
      int* fb = s->sw_err + 1;
      void* fa[] = {&md, &ms, &iter, &cadm, &fb};
      e = hipLaunchKernel(sweep_kernel(q, false), dim3(g.S), dim3(MK_SW_T), fa, sw_lds, g.stream);
      wd_trace(g.stream, "k_sweep(fallback)");
    }
  } else if (s->sweep_split) {   // one launch per 64-site block, ordered by the stream (no waits on the device)
    int nmax = 1;
    for (int i = g.s0; i < g.s0 + g.S; ++i) nmax = std::max(nmax, s->n_part[i]);
    const int nblk = (nmax + 63) / 64, nt = s->nt;
    double* part = s->sp_part + (long)g.s0 * 2 * nt * q * 64;
    const size_t lds = (size_t)q * (64 * 64 + 2 * 64) * sizeof(double) + 4 * MK_NB * sizeof(double);
    for (int B = 0; B <= nblk && e == hipSuccess; ++B) {
      void* ta[] = {&md, &ms, &iter, &B, &part};
      e = hipLaunchKernel(sweep_step_kernel(q), dim3(g.S * nt), dim3(256), ta, lds, g.stream);
      wd_trace(g.stream, "k_sweep_step");
    }
  } else {
    const size_t sw_lds = (size_t)q * (64 * 64 + 2 * 64) * sizeof(double);
    const int* adm = nullptr;
    int* fb = nullptr;
    void* args[] = {&md, &ms, &iter, &adm, &fb};
    e = hipLaunchKernel(sweep_kernel(q, false), dim3(g.S), dim3(MK_SW_T), args, sw_lds, g.stream);
    wd_trace(g.stream, "k_sweep");
  }
  if (e != hipSuccess && s->launch_err == hipSuccess) s->launch_err = e;
}

// The stream st waits for the table draws queued on the side stream (iteration_post_sweep).
static void kt_wait(mk_session* s, hipStream_t st) {
  if (!s->kt_pending) return;
  hipStreamWaitEvent(st, s->kt_ev[1], 0);
  s->kt_pending = false;
}

// One MCMC iteration of a group, in two halves around the latent sweep (run_iterations).
static void iteration_pre_sweep(mk_session* s, Group& g, int it) {
  Model& md = g.md;
  const int S = g.S, q = s->q;
  const bool kept = it >= md.kept0;
  hipStream_t st = g.stream;
  MK_LAUNCH(k_beta, dim3(S), dim3(256), 0, st, md, it);
  if (q > 1) MK_LAUNCH(k_trmv_Z, dim3(S * q * ((s->n_pad + 255) / 256)), dim3(256), 0, st, md, g.ms);
  MK_LAUNCH(k_Aphase, dim3(S), dim3(256), 0, st, md, it);
  const int nkinds = s->matern ? 2 : 1;
  // the q outcomes' (phi_h, nu_h) steps are independent given u: one batched pass per kind
  for (int which = 0; which < nkinds; ++which) {
    if (which == 0 && s->cov_pre == it) {   // assembled beside the previous sweep: the bordered row now
      hipStreamWaitEvent(st, s->cov_ev[1], 0);
      MK_LAUNCH(k_cand_border, dim3(S * q * ((s->n_pad + 255) / 256)), dim3(256), 0, st, md, g.ms, 0, q);
      s->cov_pre = -1;
    } else {
      timed(s, st, KS_COV, 0.0, [&] { launch_candidates(md, g.ms, st, S * q, 0, q, which, it); });
    }
    launch_cholesky(s, g, 0, q);
    MK_LAUNCH(k_theta_mh, dim3((S * q + 63) / 64), dim3(64), 0, st, md, g.ms, 0, q, which, it);
  }
  MK_LAUNCH(k_dirty_list, dim3(1), dim3(256), 0, st, md, (int)(it == md.kept0), g.d_list, g.d_count,
                     g.d_plist, g.d_pcount);
  kt_wait(s, st);   // the previous kept iteration's draws read W
  launch_inverse(s, g);
  if (kept && !s->tiled && !s->kt_on) launch_pred_refresh(s, g);
  // the next iteration's phi candidates depend only on this iteration's decisions (and on the proposal
  // scale, which adapts after a batch's last iteration): assemble them on cov_st beside the sweep into
  // the free factor slots, which nothing reads from here to the next iteration's Cholesky (the
  // inverse's scratch is Y).  250 subsets, 40-step windows interleaved: 11,075-11,120 vs 11,034-11,063
  // in line (profiles/r06/earlycov; both VALU-heavy, the sweep slows 0.95 -> 1.2 ms, the assembly
  // stretches to 1.9 ms beside it); started at the decision instead, beside the inverse, 11,011-11,029
  // (the inverse 4.65 -> 5.69 ms).
  if (s->cov_st && it + 1 < md.n_samples && (it + 1) % md.batch_length != 0) {
    hipEventRecord(s->cov_ev[0], st);
    hipStreamWaitEvent(s->cov_st, s->cov_ev[0], 0);
    timed(s, s->cov_st, KS_COV, 0.0,
          [&] { launch_candidates(md, g.ms, s->cov_st, S * q, 0, q, MK_CAND_NOBORDER, it + 1); });
    hipEventRecord(s->cov_ev[1], s->cov_st);
    s->cov_pre = it + 1;
  }
}

static void iteration_post_sweep(mk_session* s, Group& g, int it) {
  Model& md = g.md;
  const int S = g.S;
  const bool kept = it >= md.kept0;
  hipStream_t st = g.stream;
  if (s->record_samples) MK_LAUNCH(k_record, dim3((S + 63) / 64), dim3(64), 0, st, md, it);
  if (s->record_w) MK_LAUNCH(k_record_w, dim3((md.Np + 255) / 256, S), dim3(256), 0, st, md, it);
  if (kept && md.n_test > 0 && !s->tiled && s->kt_on) {
    // from the phi tables (krig_tables): z, phi and A captured now, then g = W' z and the draws on a
    // side stream -- the lookahead schedule's kriging stream, else the early assembly's stream after its
    // assembly -- beside the next iteration's beta, A and decision steps (W is rewritten only by the next
    // inverse, which waits for them: kt_wait).  At 250 subsets they then overlap the next Cholesky's first
    // columns and slow its diagonal launches (a kept iteration 22.0 ms against 20.0 for a burn-in one,
    // profiles/r06/zg/), but in line costs as much: 40-step windows 11,971-11,988 vs 11,957-11,976, and
    // 8,690-8,730 vs 8,601-8,642 at 32 subsets (profiles/r06/kside/).  MK_KT_SIDE=0: in line.
    double* zs = s->kt_z;
    double* ph = zs + (size_t)S * md.n_pad;
    double* As = ph + S;
    MK_LAUNCH(k_kt_snap, dim3(S), dim3(256), 0, st, md, zs, ph, As);
    static const int side_env = tile_env("MK_KT_SIDE", 1);
    hipStream_t side = st;
    if (side_env) side = s->la_k ? s->la_k : (s->cov_st ? s->cov_st : st);
    if (side != st) {
      hipEventRecord(s->kt_ev[0], st);
      hipStreamWaitEvent(side, s->kt_ev[0], 0);
    }
    MK_LAUNCH(k_krig_g, dim3(S * (md.n_pad / 4)), dim3(256), 0, side, md, g.ms, (const double*)zs, s->kt_g, 0, 1);
    MK_LAUNCH(k_pred_tab_draw, dim3(S * ((md.n_test + 255) / 256)), dim3(256), 0, side, md, s->kt, s->kt_g,
              md.coords, (const double*)ph, (const double*)As, it, it - md.kept0);
    if (side != st) {
      hipEventRecord(s->kt_ev[1], side);
      s->kt_pending = true;
    }
    s->stats[KS_KRIG_CHEB].launches += 1;
  } else if (kept && md.n_test > 0 && !s->tiled) {
    const int per = (md.n_test + 3) / 4;
    MK_LAUNCH(k_pred_draw, dim3(S * per), dim3(256), 0, st, md, it, it - md.kept0);
  }
  if (kept && s->tiled) MK_LAUNCH(k_record_kept, dim3(S), dim3(256), 0, st, md, it - md.kept0);
  if ((it + 1) % md.batch_length == 0) MK_LAUNCH(k_adapt, dim3(S), dim3(256), 0, st, md, it / md.batch_length);
}

// Lookahead schedule (exponential model, one group).  The phi proposal of iteration t+1 is known
// once iteration t's phi step has decided (and, at a batch end, adapted), so its candidates
// R(phi'_{t+1}) are assembled and factored on la_c while the main stream runs iteration t's
// inverse, kriging and sweep -- at small shards both chains are latency-bound and overlap.  The
// candidates carry no bordered row (u_{t+1} = A_{t+1}^-1 w_t does not exist yet): after the A step
// the main stream solves z' = L'^-1 u one tile column per launch, each behind the factorisation's
// panel (k_border_step), and |z'|^2 completes the phi ratio (k_border_quad).  The chain is the
// sequential schedule's (same draws, same decisions); z' differs from the bordered factor's row
// by rounding only (tests compare both schedules and the oracle).
// Panels [0, k_hi) of iteration it's candidates (the assembly with the first piece); the rest by
// enqueue_candidates_rest.  MK_LA_HEAD sets the first piece (default 3 panels: the GPU needs
// ~0.2 ms per panel at small shards, the host ~10 us per launch for the main stream's ~30).
static int la_head(mk_session* s) {
  static const int head = tile_env("MK_LA_HEAD", 3);
  return std::max(1, std::min(head, s->nt));
}
static void enqueue_candidates(mk_session* s, Group& g, int it, hipEvent_t after, int k_hi) {
  const int S = g.S, q = s->q, nt = s->nt;
  hipStreamWaitEvent(s->la_c, after, 0);
  timed(s, s->la_c, KS_COV, 0.0,
        [&] { launch_candidates(g.md, g.ms, s->la_c, S * q, 0, q, MK_CAND_NOBORDER, it); });
  launch_cholesky(s, g, 0, q, nullptr, nullptr, s->la_c, s->la_ev.data(), 0, k_hi);
  s->la_next = it;
  s->la_enq = k_hi;
}
static void enqueue_candidates_rest(mk_session* s, Group& g) {
  if (s->la_enq < s->nt) launch_cholesky(s, g, 0, s->q, nullptr, nullptr, s->la_c, s->la_ev.data(), s->la_enq, s->nt);
  s->la_enq = s->nt;
}

static void run_iteration_la(mk_session* s, int it) {
  Group& g = s->groups[0];
  Model& md = g.md;
  const int S = g.S, q = s->q, nt = s->nt;
  hipStream_t M = g.stream;
  hipEvent_t* evP = s->la_ev.data();
  hipEvent_t ev_d = evP[nt];
  if (s->la_next != it) {   // first iteration of the session (or after a tiled replay reused the slots)
    hipEventRecord(ev_d, M);
    enqueue_candidates(s, g, it, ev_d, nt);
  }
  enqueue_candidates_rest(s, g);
  MK_LAUNCH(k_beta, dim3(S), dim3(256), 0, M, md, it);
  if (q > 1) MK_LAUNCH(k_trmv_Z, dim3(S * q * ((s->n_pad + 255) / 256)), dim3(256), 0, M, md, g.ms);
  MK_LAUNCH(k_Aphase, dim3(S), dim3(256), 0, M, md, it);
  for (int k = 0; k < nt; ++k) {   // z' = L'^-1 u, trailing the candidates' panels
    hipStreamWaitEvent(M, evP[k], 0);
    MK_LAUNCH(k_border_step, dim3(xcd_grid_h(S * q, std::max(1, nt - 1 - k))), dim3(256), 0, M, md, g.ms, k);
  }
  MK_LAUNCH(k_border_quad, dim3(S * q), dim3(256), 0, M, md);
  MK_LAUNCH(k_theta_mh, dim3((S * q + 63) / 64), dim3(64), 0, M, md, g.ms, 0, q, 0, it);
  if (s->matern) {
    // the nu step: its candidate R(phi_t, nu') needs this phi decision, so it is factored now, as in
    // the sequential schedule (bordered row: u is known), on the idle high-priority candidate stream
    // (all CUs; the main stream is CU-masked); where it is accepted its border row becomes z
    // (k_nu_border into zc).  The next phi candidates follow on the same stream (they need nu_t).
    hipEventRecord(ev_d, M);
    hipStreamWaitEvent(s->la_c, ev_d, 0);
    timed(s, s->la_c, KS_COV, 0.0, [&] { launch_candidates(md, g.ms, s->la_c, S * q, 0, q, 1, it); });
    launch_cholesky(s, g, 0, q, nullptr, nullptr, s->la_c);
    MK_LAUNCH(k_theta_mh, dim3((S * q + 63) / 64), dim3(64), 0, s->la_c, md, g.ms, 0, q, 1, it);
    MK_LAUNCH(k_nu_border, dim3(S * q * ((s->n_pad + 255) / 256)), dim3(256), 0, s->la_c, md, g.ms);
    hipEventRecord(evP[nt + 4], s->la_c);
    hipStreamWaitEvent(M, evP[nt + 4], 0);
  }
  const bool more = it + 1 < md.n_samples, batch_end = (it + 1) % md.batch_length == 0;
  if (more && !batch_end) {   // the head now; the rest after the main stream's launches
    hipEventRecord(ev_d, M);
    enqueue_candidates(s, g, it + 1, ev_d, la_head(s));
  }
  MK_LAUNCH(k_dirty_list, dim3(1), dim3(256), 0, M, md, (int)(it == md.kept0), g.d_list, g.d_count, g.d_plist,
                     g.d_pcount);
  kt_wait(s, M);   // the previous kept iteration's draws read W
  launch_inverse(s, g, true);
  const bool kept = it >= md.kept0;
  // kept iterations: the kriging refresh (X = W P^T of the changed pairs) only reads W, as the sweep
  // does, and the draws after the sweep are its only consumer -- it runs on la_k beside the sweep
  const bool side = kept && !s->tiled && !s->kt_on && md.n_test > 0 && s->la_k;
  if (side) {
    hipEventRecord(evP[nt + 2], M);
    hipStreamWaitEvent(s->la_k, evP[nt + 2], 0);
    launch_pred_refresh(s, g, s->la_k);
    hipEventRecord(evP[nt + 3], s->la_k);
  } else if (kept && !s->tiled && !s->kt_on) {
    launch_pred_refresh(s, g);
  }
  timed(s, M, KS_SWEEP, 0.0, [&] { launch_sweep(s, g, it); });
  if (side) hipStreamWaitEvent(M, evP[nt + 3], 0);
  iteration_post_sweep(s, g, it);
  if (more && batch_end) {   // the next proposal's scale is the adapted one
    hipEventRecord(ev_d, M);
    enqueue_candidates(s, g, it + 1, ev_d, nt);
  }
  enqueue_candidates_rest(s, g);
  if (!more) s->la_next = -1;
}

// One iteration of the shard.  Each group (stream) runs its own chain of launches; with the
// multi-workgroup sweep and several groups, the groups join for one whole-shard sweep on the
// session stream and fork again (the groups' Cholesky chains overlap each other's latency-bound
// diagonal steps; the sweep is one multi-workgroup launch).  Same kernels, same operands, same bits.
static void run_iteration(mk_session* s, int it) {
  if (s->la) {
    run_iteration_la(s, it);
    return;
  }
  if (use_sweep_mg(s) && s->groups.size() > 1) {
    for (auto& g : s->groups) {
      hipStreamWaitEvent(g.stream, s->swept, 0);
      iteration_pre_sweep(s, g, it);
      hipEventRecord(g.done, g.stream);
      hipStreamWaitEvent(s->stream, g.done, 0);
    }
    timed(s, s->stream, KS_SWEEP, 0.0, [&] { launch_sweep(s, s->all, it); });
    hipEventRecord(s->swept, s->stream);
    for (auto& g : s->groups) {
      hipStreamWaitEvent(g.stream, s->swept, 0);
      iteration_post_sweep(s, g, it);
    }
    return;
  }
  for (auto& g : s->groups) {
    iteration_pre_sweep(s, g, it);
    timed(s, g.stream, KS_SWEEP, 0.0, [&] { launch_sweep(s, g, it); });
    iteration_post_sweep(s, g, it);
  }
}

static int check_cfg(const mk_problem* pr, const mk_config* c) {
  if (!pr || !c) return set_err(MK_E_ARG, "null problem/config");
  if (pr->n_subsets < 1) return set_err(MK_E_ARG, "n_subsets must be >= 1");
  if (pr->q < 1 || pr->q > MK_QMAX) return set_err(MK_E_ARG, "q must be in [1, 4]");
  if (pr->p < 1) return set_err(MK_E_ARG, "p must be >= 1");
  if (!pr->n_part || !pr->coords || !pr->y || !pr->weights || !pr->x) return set_err(MK_E_ARG, "null data pointer");
  if (pr->n_test < 0 || (pr->n_test > 0 && !pr->coords_test)) return set_err(MK_E_ARG, "bad coords_test");
  if (c->cov_model != MK_COV_EXPONENTIAL && c->cov_model != MK_COV_MATERN) return set_err(MK_E_ARG, "cov.model must be exponential or matern");
  if (c->n_batch < 1 || c->batch_length < 1) return set_err(MK_E_ARG, "n.batch and batch.length must be >= 1");
  const int n_samples = c->n_batch * c->batch_length;
  if (c->burn_in < 1 || c->burn_in > n_samples) return set_err(MK_E_ARG, "burn_in must be in [1, n.samples]");
  if (n_samples - c->burn_in + 1 > MK_QUANT_MAX)
    return set_err(MK_E_ARG, "at most " + std::to_string(MK_QUANT_MAX) + " kept samples supported");
  if (c->n_streams < 0 || c->n_streams > 8) return set_err(MK_E_ARG, "n_streams must be in [0, 8]");
  if (c->predict_tile < 0) return set_err(MK_E_ARG, "predict_tile must be >= 0");
  if (c->link != MK_LINK_LOGIT && c->link != MK_LINK_PROBIT) return set_err(MK_E_ARG, "link must be logit or probit");
  if (!c->beta_starting || !c->beta_tuning || !c->phi_starting || !c->phi_tuning || !c->A_starting || !c->A_tuning ||
      !c->phi_unif_a || !c->phi_unif_b || !c->K_IW_S)
    return set_err(MK_E_ARG, "null starting/tuning/prior array");
  if (c->cov_model == MK_COV_MATERN && (!c->nu_starting || !c->nu_tuning || !c->nu_unif_a || !c->nu_unif_b))
    return set_err(MK_E_ARG, "matern needs nu starting/tuning/prior");
  for (int i = 0; i < pr->n_subsets; ++i)
    if (pr->n_part[i] < 1) return set_err(MK_E_ARG, "every subset needs >= 1 site");
  for (int h = 0; h < pr->q; ++h) {
    if (!(c->phi_unif_a[h] < c->phi_starting[h] && c->phi_starting[h] < c->phi_unif_b[h]))
      return set_err(MK_E_ARG, "phi starting value outside phi.Unif support");
  }
  return 0;
}

// Work lists for `ng` run groups + the whole-shard view (last): list/plist per pair, 2 counts per view.
static int setup_groups(mk_session* s, int n_groups) {
  const int S = s->S, q = s->q;
  const int G = std::max(1, std::min(n_groups, S));
  int *lists = nullptr, *counts = nullptr;
  int rc;
  if ((rc = s->alloc(&lists, (size_t)4 * S * q)) || (rc = s->alloc(&counts, (size_t)2 * (G + 1)))) return rc;
  s->all.md = s->md;
  s->all.ms = s->ms;
  s->all.stream = s->stream;
  s->all.S = S;
  s->all.s0 = 0;
  s->all.d_list = lists;
  s->all.d_plist = lists + S * q;
  s->all.d_count = counts + 2 * G;
  s->all.d_pcount = counts + 2 * G + 1;
  const int per = (S + G - 1) / G;
  for (int gi = 0; gi < G; ++gi) {
    const int s0 = gi * per, Sg = std::min(per, S - s0);
    if (Sg <= 0) break;
    Group g;
    g.S = Sg;
    g.s0 = s0;
    g.md = model_view(s->md, s0, Sg);
    g.ms = matset_view(s->ms, s0);
    g.d_list = lists + 2 * S * q + s0 * q;
    g.d_plist = lists + 3 * S * q + s0 * q;
    g.d_count = counts + 2 * gi;
    g.d_pcount = counts + 2 * gi + 1;
    if (G == 1) {
      g.stream = s->stream;
    } else if (pool_stream(s->owned, &g.stream, s->device, SK_PLAIN) != hipSuccess) {
      return set_err(MK_E_HIP, "group stream");
    }
    s->groups.push_back(g);
  }
  if (G > 1) {
    for (auto& g : s->groups)
      if (hipEventCreateWithFlags(&g.done, hipEventDisableTiming) != hipSuccess) return set_err(MK_E_HIP, "group event");
    if (hipEventCreateWithFlags(&s->swept, hipEventDisableTiming) != hipSuccess) return set_err(MK_E_HIP, "sweep event");
  }
  // Split Cholesky (launch_cholesky) for small shards on one stream: a bulk-update stream that
  // leaves the first `reserve` CUs (mask bits 0..reserve-1 = reserve/8 CUs on each XCD, measured
  // by tools/cumask_probe.hip) to the diagonal kernels.  MK_CHOL_SPLIT=0 / 1 forces it off / on;
  // MK_RESERVE_CU sets the reserve (default: one CU per diagonal workgroup, 8..64).
  static const int split_env = tile_env("MK_CHOL_SPLIT", -1);
  int n_cu = 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, s->device) != hipSuccess)
    return set_err(MK_E_HIP, "device attribute");
  const bool split = G == 1 && s->nt > 2 && (split_env == 1 || (split_env < 0 && (long)S * q * 4 <= n_cu));
  if (split) {
    const int reserve = std::max(8, std::min(64, round_up(tile_env("MK_RESERVE_CU", S * q), 8)));
    std::vector<uint32_t> mask((n_cu + 31) / 32, 0xffffffffu);
    for (int b = 0; b < reserve && b < n_cu; ++b) mask[b / 32] &= ~(1u << (b % 32));
    Group& g = s->groups[0];
    if (pool_stream(s->owned, &g.bulk, s->device, SK_CUMASK, 0, mask) != hipSuccess)
      return set_err(MK_E_HIP, "bulk stream");
    g.ev.assign(2 * s->nt + 1, nullptr);
    for (auto& e : g.ev)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return set_err(MK_E_HIP, "cholesky event");
  }
  return 0;
}

// (Re)allocate the kriging buffers for n_test_all test sites (coords_test: n_test_all x 2
// column-major) and upload the sites: all of them in d_ct_all, the fused path's copy in the tile
// buffer d_ct.  Tiled sessions size the buffers for one tile.  Refreshes the group views.
static int kriging_buffers(mk_session* s, int n_test_all, const double* coords_test) {
  Model& md = s->md;
  for (void* b : s->kbufs) s->release(b);
  s->kbufs.clear();
  md.PT = md.XK = md.s_pred = md.s_part = md.w_pred = nullptr;
  md.span_pt = nullptr;
  const int S = s->S, q = s->q, nt = s->nt, n_pad = s->n_pad;
  s->n_test_all = n_test_all;
  s->n_test_pad_all = round_up(std::max(n_test_all, 1), 256);
  s->pred_tile = s->tiled ? std::min(s->tile_req, std::max(n_test_all, 1)) : n_test_all;
  double* d_ct = nullptr;
  double* d_spt = nullptr;
  int rc;
  // Tiled sessions whose buffers for the requested tile do not fit in HBM (X and P^T are n_pad x tile
  // per pair, the draws n_kept x tile per subset: configs[4]'s 250 subsets at 65,536 sites on one GPU
  // would need ~700 GB) take the largest tile that fits, halving it (in 256-site steps) until the
  // allocations succeed.  The draws do not depend on the tile (keyed by the global site index);
  // mk_session_predict_tile reports the tile in use.
  // MK_KRIG_MEM_GB (optional): a budget for the tile's kriging buffers (tests; hosts sharing the GPU)
  const char* cap_env = std::getenv("MK_KRIG_MEM_GB");
  const double cap = (cap_env && *cap_env) ? std::atof(cap_env) * 1e9 : 0.0;
  for (;;) {
    const int n_test = n_test_all > 0 ? s->pred_tile : 0;
    const int n_test_pad = round_up(std::max(n_test, 1), 256);
    const double bytes = 8.0 * ((double)S * q * n_test_pad * (1.0 + nt + (n_test > 0 ? (s->pred_gen ? 1 : 2) * n_pad : 0)) +
                                (double)S * md.n_kept * q * std::max(n_test, 1));
    if (cap > 0.0 && bytes > cap && s->tiled && s->pred_tile > 256) {
      s->pred_tile = std::max(256, round_up(s->pred_tile / 2, 256));
      continue;
    }
    md.n_test = n_test;
    md.n_test_pad = n_test_pad;
    md.ntt = n_test_pad / MK_NB;
    d_ct = d_spt = nullptr;
    md.PT = md.XK = md.s_pred = md.s_part = md.w_pred = nullptr;
    s->d_ct_all = nullptr;
    if ((rc = s->alloc(&d_ct, (size_t)2 * n_test_pad)) || (rc = s->alloc(&s->d_ct_all, (size_t)2 * s->n_test_pad_all)) ||
        (rc = s->alloc(&d_spt, (size_t)S)) ||
        (rc = s->alloc(&md.s_pred, (size_t)S * q * n_test_pad)) ||
        (rc = s->alloc(&md.s_part, (size_t)S * q * nt * n_test_pad)) ||
        (n_test > 0 && !s->pred_gen && (rc = s->alloc(&md.PT, (size_t)S * q * n_pad * n_test_pad))) ||
        (n_test > 0 && (rc = s->alloc(&md.XK, (size_t)S * q * n_pad * n_test_pad))) ||
        (rc = s->alloc(&md.w_pred, (size_t)S * md.n_kept * q * std::max(n_test, 1)))) {
      for (void* b : {(void*)d_ct, (void*)s->d_ct_all, (void*)d_spt, (void*)md.s_pred, (void*)md.s_part, (void*)md.PT,
                      (void*)md.XK, (void*)md.w_pred})
        s->release(b);
      md.PT = md.XK = md.s_pred = md.s_part = md.w_pred = nullptr;
      s->d_ct_all = nullptr;
      if (rc == MK_E_NOMEM && s->tiled && s->pred_tile > 256) {
        s->pred_tile = std::max(256, round_up(s->pred_tile / 2, 256));
        continue;
      }
      return rc;
    }
    break;
  }
  md.coords_test = d_ct;
  s->kbufs = {d_ct, s->d_ct_all, md.s_pred, md.s_part, md.PT, md.XK, md.w_pred, d_spt};
  {   // Matern kriging tables (k_pred_PT_matern): a bound on every subset-site to test-site distance
    double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
    for (int t = 0; t < n_test_all; ++t) {
      const double x = coords_test[t], y = coords_test[n_test_all + t];
      if (t == 0 || x < t0) t0 = x;
      if (t == 0 || x > t1) t1 = x;
      if (t == 0 || y < t2) t2 = y;
      if (t == 0 || y > t3) t3 = y;
    }
    std::vector<double> hs(S);
    for (int i = 0; i < S; ++i) {
      const double* b = s->bbox.data() + 4 * i;
      hs[i] = n_test_all > 0 ? std::hypot(std::fmax(std::fabs(b[1] - t0), std::fabs(t1 - b[0])),
                                          std::fmax(std::fabs(b[3] - t2), std::fabs(t3 - b[2])))
                             : 0.0;
    }
    HIPCHK(hipMemcpy(d_spt, hs.data(), (size_t)S * 8, hipMemcpyHostToDevice));
    md.span_pt = d_spt;
    s->span_pt_h = hs;
  }
  HIPCHK(hipMemset(md.s_pred, 0, (size_t)S * q * md.n_test_pad * 8));
  const int npa = s->n_test_pad_all;
  std::vector<double> hct((size_t)2 * npa, 0.0);
  for (int t = 0; t < n_test_all; ++t) {
    hct[t] = coords_test[t];
    hct[npa + t] = coords_test[n_test_all + t];
  }
  HIPCHK(hipMemcpy(s->d_ct_all, hct.data(), hct.size() * 8, hipMemcpyHostToDevice));
  // fused kriging reads every site from d_ct ([2][n_test_pad]); tiled mode fills it per tile
  if (!s->tiled) HIPCHK(hipMemcpy(d_ct, hct.data(), hct.size() * 8, hipMemcpyHostToDevice));
  s->all.md = s->md;
  for (auto& g : s->groups) g.md = model_view(s->md, g.s0, g.S);
  return 0;
}

extern "C" int mk_session_set_test_sites(mk_session* s, int32_t n_test, const double* coords_test) {
  if (!s) return set_err(MK_E_ARG, "null session");
  if (!s->tiled)
    return set_err(MK_E_ARG, "the session keeps no chain states: create it with predict_tile > 0 (and no test sites)");
  if (n_test < 1 || !coords_test) return set_err(MK_E_ARG, "n_test must be >= 1 with coordinates");
  MK_ENTRY_DEVICE(s->device);
  HIPCHK(hipStreamSynchronize(s->stream));
  return kriging_buffers(s, n_test, coords_test);
}

extern "C" int mk_session_set_kept_window(mk_session* s, int32_t first, int32_t last) {
  if (!s) return set_err(MK_E_ARG, "null session");
  if (!s->tiled) return set_err(MK_E_ARG, "kept windows need a session created with predict_tile > 0");
  const int lo = s->md.kept0 + 1, hi = s->md.n_samples;
  if (first < lo || last < first || last > hi)
    return set_err(MK_E_ARG, "kept window must satisfy burn_in <= first <= last <= n.samples");
  s->win_lo = first - lo;
  s->win_n = last - first + 1;
  return 0;
}

extern "C" int mk_session_create(const mk_problem* pr, const mk_config* c, mk_session** out) {
  if (!out) return set_err(MK_E_ARG, "null out");
  *out = nullptr;
  int rc = check_cfg(pr, c);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return set_err(MK_E_NODEV, "no HIP device");
  if (c->device < 0 || c->device >= ndev) return set_err(MK_E_ARG, "bad device ordinal");
  MK_ENTRY_DEVICE(c->device);
  // the guard owns the session until it is handed out: every early return (allocation failure,
  // HIPCHK, argument error) frees the session and every device buffer allocated so far
  std::unique_ptr<mk_session> hold(new mk_session());
  mk_session* s = hold.get();
  s->device = c->device;
  if (pool_stream(s->owned, &s->stream, s->device, SK_PLAIN) != hipSuccess) return set_err(MK_E_HIP, "stream");

  const int S = pr->n_subsets, q = pr->q, p = pr->p;
  s->S = S; s->q = q; s->p = p;
  s->matern = c->cov_model == MK_COV_MATERN;
  // MK_PRED_GEN=1: P^T generated inside the kriging GEMM (exponential; no P^T buffer, half the
  // kriging memory, but 0.52 vs 0.74 of fp64 peak: the exp/sqrt per element are recomputed for
  // every row panel).  Default: stored P^T.
  s->pred_gen = !s->matern && tile_env("MK_PRED_GEN", 0) != 0;
  s->n_part.assign(pr->n_part, pr->n_part + S);
  s->bbox.assign((size_t)4 * S, 0.0);
  {
    long off = 0;
    for (int i = 0; i < S; ++i) {
      const int ns = pr->n_part[i];
      const double* cs = pr->coords + 2 * off;
      double* b = s->bbox.data() + 4 * i;
      for (int r = 0; r < ns; ++r) {
        if (r == 0 || cs[r] < b[0]) b[0] = cs[r];
        if (r == 0 || cs[r] > b[1]) b[1] = cs[r];
        if (r == 0 || cs[ns + r] < b[2]) b[2] = cs[ns + r];
        if (r == 0 || cs[ns + r] > b[3]) b[3] = cs[ns + r];
      }
      off += ns;
    }
  }
  int nmax = 0;
  for (int i = 0; i < S; ++i) nmax = std::max(nmax, (int)pr->n_part[i]);
  const int n_pad = round_up(nmax + 1, MK_NB);
  const int nt = n_pad / MK_NB;
  s->n_pad = n_pad; s->nt = nt;
  const int Np = n_pad * q;
  const int ntri = q * (q + 1) / 2;
  const int n_theta = ntri + q * (s->matern ? 2 : 1);
  const int P = p + n_theta;
  s->P = P;
  const int o_w = p + n_theta;
  const int n_mh_max = o_w + Np;
  const int n_samples = c->n_batch * c->batch_length;
  const int kept0 = c->burn_in - 1;
  const int n_kept = n_samples - kept0;
  // tiled kriging: device kriging buffers hold one tile of test sites; all sites stay in HBM.
  // predict_tile > 0 without test sites records the kept states for a later
  // mk_session_set_test_sites (spPredict after spMvGLM without refitting).
  s->tiled = c->predict_tile > 0 && (pr->n_test == 0 || c->predict_tile < pr->n_test);
  s->tile_req = c->predict_tile;

  Model& md = s->md;
  md.S = S; md.q = q; md.p = p; md.n_pad = n_pad; md.Np = Np; md.nt = nt; md.ntri = ntri; md.n_theta = n_theta;
  md.cov_model = c->cov_model;
  md.link = c->link;
  md.o_A = p; md.o_phi = p + ntri; md.o_nu = p + ntri + q; md.o_w = o_w; md.n_mh_max = n_mh_max;
  md.n_batch = c->n_batch; md.batch_length = c->batch_length; md.n_samples = n_samples;
  md.kept0 = kept0; md.n_kept = n_kept;
  md.subset_base = pr->subset_base;
  md.S_all = S;
  md.t_off = 0;
  md.seed = c->seed;
  md.accept_rate = c->accept_rate;
  md.P = P;
  for (int h = 0; h < q; ++h) {
    md.phi_a[h] = c->phi_unif_a[h]; md.phi_b[h] = c->phi_unif_b[h];
    md.nu_a[h] = s->matern ? c->nu_unif_a[h] : 0.0;
    md.nu_b[h] = s->matern ? c->nu_unif_b[h] : 1.0;
  }
  md.iw_df = c->K_IW_df;
  for (int i = 0; i < q * q; ++i) md.iw_S[i] = c->K_IW_S[i];
  s->record_samples = true;   // needed on device for the parameter quantiles
  s->record_w = c->record_w != 0;

  // ---------------- allocations
  int* d_ns; double *d_coords, *d_y, *d_wt, *d_X;
  if ((rc = s->alloc(&d_ns, S)) || (rc = s->alloc(&d_coords, (size_t)S * 2 * n_pad)) ||
      (rc = s->alloc(&d_y, (size_t)S * Np)) || (rc = s->alloc(&d_wt, (size_t)S * Np)) ||
      (rc = s->alloc(&d_X, (size_t)S * p * Np)))
    return rc;
  md.n_s = d_ns; md.coords = d_coords; md.y = d_y; md.wt = d_wt; md.X = d_X;
  if ((rc = s->alloc(&md.beta, (size_t)S * p)) || (rc = s->alloc(&md.theta, (size_t)S * n_theta)) ||
      (rc = s->alloc(&md.w, (size_t)S * Np)) || (rc = s->alloc(&md.eta, (size_t)S * Np)) ||
      (rc = s->alloc(&md.tune, (size_t)S * n_mh_max)) || (rc = s->alloc(&md.acc, (size_t)S * n_mh_max)) ||
      (rc = s->alloc(&md.u, (size_t)S * q * n_pad)) || (rc = s->alloc(&md.z, (size_t)S * q * n_pad)) ||
      (rc = s->alloc(&md.Z, (size_t)S * q * q * n_pad)) || (rc = s->alloc(&md.logdetR, (size_t)S * q)) ||
      (rc = s->alloc(&md.quad, (size_t)S * q)) || (rc = s->alloc(&md.A_full, (size_t)S * q * q)) ||
      (rc = s->alloc(&md.Ainv, (size_t)S * q * q)) || (rc = s->alloc(&md.dirty, (size_t)S * q)) ||
      (rc = s->alloc(&md.ld_part, (size_t)S * q * nt)) || (rc = s->alloc(&md.quad_c, (size_t)S * q)) ||
      (rc = s->alloc(&md.info, (size_t)S * q)) || (rc = s->alloc(&md.sw_delta, (size_t)S * Np)) ||
      (rc = s->alloc(&md.sw_dll, (size_t)S * Np)) || (rc = s->alloc(&md.sw_logu, (size_t)S * Np)) ||
      (rc = s->alloc(&md.sw_acc, (size_t)S * Np)) || (rc = s->alloc(&md.samples, (size_t)S * n_samples * P)) ||
      (rc = s->alloc(&md.acc_hist, (size_t)S * c->n_batch * (o_w + 1))))
    return rc;
  if (s->record_w && (rc = s->alloc(&md.w_samples, (size_t)S * n_samples * Np))) return rc;
  if (s->tiled && ((rc = s->alloc(&md.kz, (size_t)n_kept * S * q * n_pad)) ||
                   (rc = s->alloc(&md.kth, (size_t)n_kept * S * n_theta)) ||
                   (rc = s->alloc(&md.kA, (size_t)n_kept * S * q * q)) ||
                   (rc = s->alloc(&s->d_slist, (size_t)q * S)) || (rc = s->alloc(&s->d_scount, (size_t)q))))
    return rc;
  if ((rc = kriging_buffers(s, pr->n_test, pr->coords_test))) return rc;
  {   // Matern candidate tables (k_cov_candidate): bounding-box diagonal of every subset
    double* d_span = nullptr;
    if ((rc = s->alloc(&d_span, (size_t)S))) return rc;
    std::vector<double> hs(S);
    for (int i = 0; i < S; ++i)
      hs[i] = std::hypot(s->bbox[4 * i + 1] - s->bbox[4 * i], s->bbox[4 * i + 3] - s->bbox[4 * i + 2]);
    HIPCHK(hipMemcpy(d_span, hs.data(), (size_t)S * 8, hipMemcpyHostToDevice));
    md.span = d_span;
    if (s->matern && ((rc = s->alloc(&md.chtab, (size_t)S * q * MK_CH_TAB)) ||
                      (rc = s->alloc(&md.chtab_p, (size_t)S * q * MK_CH_TAB))))
      return rc;
  }
  // ---------------- the latent sweep (launch_sweep)
  // MK_SWEEP (tests and measurements): 1 the 64-site-block kernel (k_sweep: the fallback for subsets
  // too large for the site sweep), 2 the multi-workgroup kernel (k_sweep_mg + the k_sweep fallback;
  // where its grid fits the chip at once, else split launches), 3 split launches.
  // 0 (default): the one-pass site sweep (k_sweep_site; W read once, no Q_BB tiles, no inter-workgroup
  // waits) wherever it fits -- n_pad <= 4096 (q = 4: not instantiated) and the sites' data in LDS
  // (configs[3]: n_s = 2,000, q = 3 takes 152 KB) -- except multi-outcome small shards (q >= 2, <= 16
  // subsets: one workgroup per subset is the iteration's longest chain there), which take the
  // multi-workgroup kernel on either schedule.
  // Measured (subset-iters/s, 40-step windows, profiles/r04/knobs, r04e): configs[2] 250 subsets block
  // sweep 10,143 / site pair 10,527; configs[1] 15,198 / 15,626; configs[3] (q = 3, 50 subsets) block
  // 3,016 / site 3,106; configs[3]'s 7-subset share split launches 1,476 / site 1,340 / block 1,107
  // (lookahead schedule).  q = 1 runs the lean pair form (k_sweep_site LN > 0: 250 subsets 10,452 ->
  // 10,567-10,622, 32 subsets 7,832 -> 7,957-8,067).
  {
    HIPCHK(hipFuncSetAttribute(sweep_kernel(q, false), hipFuncAttributeMaxDynamicSharedMemorySize,
                               q * (64 * 64 + 2 * 64) * 8));
    s->sweep_mg_lds = (size_t)q * (64 * 64 + 2 * 64) * 8 + 4 * MK_NB * 8;
    const void* fn = sweep_kernel(q, true);
    HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)s->sweep_mg_lds));
    int per_cu = 0, n_cu = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, s->sweep_mg_lds));
    HIPCHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device));
    const int mode = tile_env("MK_SWEEP", 0);
    // the whole grid fits at once (else admission would mostly fall back) -- on the CUs the sweep's
    // stream may use: a one-group session can run the lookahead schedule, whose main stream leaves
    // MK_LA_MASK CUs (default 32 with 8 hardware queues) to the candidates' chain
    const bool one_group = (c->n_streams > 0 ? std::min((int)c->n_streams, S) : 1) <= 1;
    const int mask_env = tile_env("MK_LA_MASK", -1);
    const int la_mask = one_group ? (mask_env >= 0 ? mask_env : (hw_queues() >= 8 ? 32 : 0)) : 0;
    const bool coop_fits = (long)xcd_grid(S, nt) <= (long)per_cu * std::max(1, n_cu - la_mask) && nt <= 32;
    const bool small_multi = q >= 2 && S <= 16;
    const bool site_fits = sweep_site_kernel(q, n_pad <= 8 * MK_SS_T ? 1 : 2) != nullptr && n_pad <= 16 * MK_SS_T &&
                           sweep_site_lds_bytes(nmax, q, q == 1) <= 156 * 1024;
    const bool site = mode == 0 && !small_multi && site_fits;
    const bool multi = (mode == 0 && !site && small_multi) || mode == 2 || mode == 3;
    s->sweep_coop = multi && mode != 3 && coop_fits;
    s->sweep_split = multi && !s->sweep_coop && nt <= 32;   // k_sweep_step sums <= 32 tile partials
    if (site) {
      s->sweep_site = n_pad <= 8 * MK_SS_T ? 1 : 2;
      bool all_even = true;
      for (int i = 0; i < S; ++i) all_even = all_even && (s->n_part[i] % 2 == 0);
      s->sweep_lean = q == 1 ? (all_even ? 2 : 1) : 0;
      s->sweep_site_lds = sweep_site_lds_bytes(nmax, q, s->sweep_lean);
      HIPCHK(hipFuncSetAttribute(sweep_site_kernel(q, s->sweep_site, s->sweep_lean),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)s->sweep_site_lds));
    }
    if (s->sweep_split) {
      HIPCHK(hipFuncSetAttribute(sweep_step_kernel(q), hipFuncAttributeMaxDynamicSharedMemorySize,
                                 q * (64 * 64 + 2 * 64) * 8 + 4 * MK_NB * 8));
      if ((rc = s->alloc(&s->sp_part, (size_t)S * 2 * nt * q * 64))) return rc;
    }
    if (s->sweep_coop) {
      if ((rc = s->alloc(&s->sw_part, (size_t)S * 2 * nt * q * 64)) ||
          (rc = s->alloc(&s->sw_cnt, (size_t)S * (n_pad / 64 + 1))) || (rc = s->alloc(&s->sw_xcc, (size_t)S * nt)) ||
          (rc = s->alloc(&s->sw_err, 2)))
        return rc;
      s->sw_adm = s->sw_cnt + (size_t)S * (n_pad / 64);
      s->adm_spins = tile_env("MK_ADM_SPINS", MK_ADM_SPINS);
      HIPCHK(hipMemsetAsync(s->sw_err, 0, 2 * sizeof(int), s->stream));
    }
  }
  MatSet& ms = s->ms;
  ms.ld = n_pad; ms.nt = nt; ms.q = q;
  if ((rc = s->alloc(&ms.L, (size_t)S * q * 2 * n_pad * n_pad)) ||
      (rc = s->alloc(&ms.Winv, (size_t)S * q * 2 * nt * MK_NB * MK_NB)) ||
      (rc = s->alloc(&ms.W, (size_t)S * q * n_pad * n_pad)) ||
      (!s->sweep_site && (rc = s->alloc(&ms.QB, (size_t)S * q * nt * MK_NB * MK_NB))) ||   // Q_BB: block sweeps only
      (rc = s->alloc(&ms.cur, (size_t)S * q)) ||
      (rc = s->alloc(&s->d_probs, MK_N_LEVELS)))
    return rc;
  // lookahead schedule buffers (run_iteration_la): one stream group (either covariance model)
  {
    const int G = std::max(1, std::min(c->n_streams > 0 ? (int)c->n_streams : 1, S));
    s->la_ok = G == 1;
    if (s->la_ok) {
      if ((rc = s->alloc(&md.bacc, (size_t)S * q * n_pad)) || (rc = s->alloc(&md.zc, (size_t)S * q * n_pad)) ||
          (rc = s->alloc(&ms.Y, (size_t)S * q * n_pad * n_pad)) || (rc = s->alloc(&md.la_nu, (size_t)S * q)))
        return rc;
      HIPCHK(hipMemset(md.la_nu, 0, (size_t)S * q * sizeof(int)));
      s->la_ev.assign(nt + 5, nullptr);
      for (auto& e : s->la_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return set_err(MK_E_HIP, "lookahead event");
    }
  }
  if ((rc = setup_groups(s, c->n_streams > 0 ? c->n_streams : 1))) return rc;

  // ---------------- host staging (R layout -> padded device layout)
  std::vector<double> hc((size_t)S * 2 * n_pad, 0.0), hy((size_t)S * Np, 0.0), hw((size_t)S * Np, 0.0),
      hX((size_t)S * p * Np, 0.0);
  {
    long off_site = 0;
    for (int i = 0; i < S; ++i) {
      const int ns = pr->n_part[i];
      const double* cs = pr->coords + 2 * off_site;
      for (int r = 0; r < ns; ++r) {
        hc[(size_t)i * 2 * n_pad + r] = cs[r];
        hc[(size_t)i * 2 * n_pad + n_pad + r] = cs[ns + r];
      }
      const double* ys = pr->y + off_site * q;
      const double* ws = pr->weights + off_site * q;
      for (int k = 0; k < ns * q; ++k) {
        hy[(size_t)i * Np + k] = ys[k];
        hw[(size_t)i * Np + k] = ws[k];
      }
      const double* xs = pr->x + off_site * q * p;
      for (int j = 0; j < p; ++j)
        for (int k = 0; k < ns * q; ++k) hX[((size_t)i * p + j) * Np + k] = xs[(size_t)j * ns * q + k];
      off_site += ns;
    }
  }
  HIPCHK(hipMemcpy(d_ns, pr->n_part, S * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_coords, hc.data(), hc.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_y, hy.data(), hy.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_wt, hw.data(), hw.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_X, hX.data(), hX.size() * 8, hipMemcpyHostToDevice));

  // ---------------- starting values (identical for every subset, MK.R:54-62)
  std::vector<double> hb((size_t)S * p), hth((size_t)S * n_theta), hwv((size_t)S * Np, 0.0),
      htune((size_t)S * n_mh_max, 0.0), hA((size_t)S * q * q), hAi((size_t)S * q * q);
  std::vector<double> th0(n_theta), A0(q * q, 0.0), Ai0(q * q, 0.0), tune0(o_w);
  {
    int k = 0;
    for (int j = 0; j < q; ++j)
      for (int i = j; i < q; ++i, ++k) {
        const double a = c->A_starting[k];
        if (i == j && !(a > 0.0)) { return set_err(MK_E_ARG, "A starting diagonal must be > 0"); }
        th0[k] = (i == j) ? std::log(a) : a;
        A0[i + j * q] = a;
      }
    for (int h = 0; h < q; ++h) {
      const double ph = c->phi_starting[h];
      th0[ntri + h] = std::log((ph - md.phi_a[h]) / (md.phi_b[h] - ph));
      if (s->matern) {
        const double nv = c->nu_starting[h];
        if (!(md.nu_a[h] < nv && nv < md.nu_b[h])) { return set_err(MK_E_ARG, "nu starting value outside nu.Unif support"); }
        th0[ntri + q + h] = std::log((nv - md.nu_a[h]) / (md.nu_b[h] - nv));
      }
    }
    for (int cc = 0; cc < q; ++cc)
      for (int r = 0; r < q; ++r) {
        if (r < cc) continue;
        double sum = (r == cc) ? 1.0 : 0.0;
        for (int m = cc; m < r; ++m) sum -= A0[r + m * q] * Ai0[m + cc * q];
        Ai0[r + cc * q] = sum / A0[r + r * q];
      }
    for (int j = 0; j < p; ++j) {
      if (!(c->beta_tuning[j] > 0.0)) { return set_err(MK_E_ARG, "beta tuning must be > 0"); }
      tune0[j] = std::log(std::sqrt(c->beta_tuning[j]));
    }
    for (int k2 = 0; k2 < ntri; ++k2) tune0[p + k2] = std::log(std::sqrt(c->A_tuning[k2]));
    for (int h = 0; h < q; ++h) {
      tune0[p + ntri + h] = std::log(std::sqrt(c->phi_tuning[h]));
      if (s->matern) tune0[p + ntri + q + h] = std::log(std::sqrt(c->nu_tuning[h]));
    }
  }
  const double tw = std::log(std::sqrt(c->w_tuning));
  for (int i = 0; i < S; ++i) {
    for (int j = 0; j < p; ++j) hb[(size_t)i * p + j] = c->beta_starting[j];
    for (int k = 0; k < n_theta; ++k) hth[(size_t)i * n_theta + k] = th0[k];
    for (int k = 0; k < pr->n_part[i] * q; ++k) {
      hwv[(size_t)i * Np + k] = c->w_starting;
      htune[(size_t)i * n_mh_max + o_w + k] = tw;
    }
    for (int k = 0; k < o_w; ++k) htune[(size_t)i * n_mh_max + k] = tune0[k];
    for (int k = 0; k < q * q; ++k) { hA[(size_t)i * q * q + k] = A0[k]; hAi[(size_t)i * q * q + k] = Ai0[k]; }
  }
  HIPCHK(hipMemcpy(md.beta, hb.data(), hb.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(md.theta, hth.data(), hth.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(md.w, hwv.data(), hwv.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(md.tune, htune.data(), htune.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(md.A_full, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(md.Ainv, hAi.data(), hAi.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemsetAsync(md.acc, 0, (size_t)S * n_mh_max * 8, s->stream));
  HIPCHK(hipMemsetAsync(md.dirty, 0, (size_t)S * q * 4, s->stream));
  HIPCHK(hipMemsetAsync(md.info, 0, (size_t)S * q * 4, s->stream));
  HIPCHK(hipMemsetAsync(ms.cur, 0, (size_t)S * q * 4, s->stream));
  HIPCHK(hipMemsetAsync(md.u, 0, (size_t)S * q * n_pad * 8, s->stream));
  HIPCHK(hipMemsetAsync(md.z, 0, (size_t)S * q * n_pad * 8, s->stream));
  HIPCHK(hipMemsetAsync(md.Z, 0, (size_t)S * q * q * n_pad * 8, s->stream));
  HIPCHK(hipMemsetAsync(ms.W, 0, (size_t)S * q * n_pad * n_pad * 8, s->stream));
  // upper triangles of the Winv tiles stay zero (k_chol_diag writes the lower triangles only)
  HIPCHK(hipMemsetAsync(ms.Winv, 0, (size_t)S * q * 2 * nt * MK_NB * MK_NB * 8, s->stream));
  {
    std::vector<double> probs(MK_N_LEVELS);
    // seq(0.005, 1, 0.005): from + (0:n)*by, pmin(x, to)  (MK.R:88)
    for (int i = 0; i < MK_N_LEVELS; ++i) probs[i] = std::fmin(0.005 + (double)i * 0.005, 1.0);
    HIPCHK(hipMemcpy(s->d_probs, probs.data(), MK_N_LEVELS * 8, hipMemcpyHostToDevice));
  }
  HIPCHK(hipFuncSetAttribute((const void*)k_chol_diag, hipFuncAttributeMaxDynamicSharedMemorySize,
                             MK_DIAG_LDS_BYTES));
  if (!set_gemm_lds()) return set_err(MK_E_HIP, "gemm lds attribute");
  HIPCHK(hipFuncSetAttribute(sweep_kernel(q, false), hipFuncAttributeMaxDynamicSharedMemorySize,
                             q * (64 * 64 + 2 * 64) * 8));
  // fused kriging tables (before the initial factorisation: their evaluation uses the factor slots and
  // W as scratch), then the slots, W and the diagonal inverses as the initial state expects them
  if ((rc = krig_tables(s))) return rc;
  HIPCHK(hipMemsetAsync(ms.cur, 0, (size_t)S * q * 4, s->stream));
  HIPCHK(hipMemsetAsync(md.info, 0, (size_t)S * q * 4, s->stream));
  HIPCHK(hipMemsetAsync(ms.W, 0, (size_t)S * q * n_pad * n_pad * 8, s->stream));
  HIPCHK(hipMemsetAsync(ms.Winv, 0, (size_t)S * q * 2 * nt * MK_NB * MK_NB * 8, s->stream));
  // ---------------- initial state: eta, u, factor every R_h at the starting values, W, z (whole shard)
  Group& a = s->all;
  MK_LAUNCH(k_init_state, dim3(S), dim3(256), 0, s->stream, md);
  launch_candidates(md, ms, s->stream, S * q, 0, q, 2, 0);
  launch_cholesky(s, a, 0, q);
  MK_LAUNCH(k_theta_init, dim3((S * q + 63) / 64), dim3(64), 0, s->stream, md, ms, 0, q);
  MK_LAUNCH(k_dirty_list, dim3(1), dim3(256), 0, s->stream, md, 0, a.d_list, a.d_count, a.d_plist, a.d_pcount);
  launch_inverse(s, a);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s->stream));
  drain_timers(s);
  for (auto& st : s->stats) st = Stat();
  if (s->kt_on) {   // the tables: exact evaluations and the largest set-up check difference
    s->stats[KS_KRIG_CHEB].flops = s->kt_evals;
    s->stats[KS_KRIG_CHEB].ms = s->kt_check;
  } else if (s->kt_fail) {
    s->stats[KS_KRIG_FALLBACK].launches = s->kt_fail;
    s->stats[KS_KRIG_FALLBACK].ms = s->kt_check;
  }
  // default schedule: lookahead where eligible; MK_LOOKAHEAD=0 / 1 overrides (mk_session_set_lookahead too)
  static const int la_env = tile_env("MK_LOOKAHEAD", -1);
  s->la = s->la_ok && (la_env == 1 || (la_env < 0 && la_auto(s)));
  *out = hold.release();
  return 0;
}

extern "C" int mk_session_run(mk_session* s, int32_t n_iter) {
  if (!s) return set_err(MK_E_ARG, "null session");
  if (s->poisoned) return set_err(MK_E_HIP, std::string("session unusable after an earlier failure: ") + s->poisoned);
  MK_ENTRY_DEVICE(s->device);
  if (n_iter < 0 || s->iter + n_iter > s->md.n_samples) return set_err(MK_E_ARG, "n_iter beyond n.samples");
  if (s->la && !s->la_c) {
    // the candidates' factorisation is the critical chain: its stream gets the device's highest
    // priority, so its small diagonal / trsm grids are dispatched ahead of the main stream's
    // inverse and sweep workgroups as CUs free up (MK_LA_PRIO=0: default priority)
    static const int prio_env = tile_env("MK_LA_PRIO", 1);
    int lo = 0, hi = 0;
    if (prio_env && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess) {
      if (pool_stream(s->owned, &s->la_c, s->device, SK_PRIO, hi) != hipSuccess)
        return set_err(MK_E_HIP, "lookahead stream");
    } else if (pool_stream(s->owned, &s->la_c, s->device, SK_PLAIN) != hipSuccess) {
      return set_err(MK_E_HIP, "lookahead stream");
    }
    // Two more streams when the process has the hardware queues for them (HIP maps streams onto
    // GPU_MAX_HW_QUEUES queues, default 4, shared round-robin beyond that -- a shared queue
    // serialises the split Cholesky's streams: measured 5,427 -> 4,087 subset-iters/s at 32
    // subsets; the package and bench.py set 8 before HIP starts):
    //  * la_k: the kept iterations' kriging refresh beside the sweep (MK_LA_KRIG=0: off);
    //  * la_m: the iterations' main-stream work on a stream that leaves the first MK_LA_MASK CUs
    //    (default 32: 4 per XCD, the split Cholesky's reserve) to the candidates' critical chain --
    //    its diagonal-tile workgroups take a whole CU's LDS and otherwise wait behind the inverse
    //    and kriging GEMMs (32 / 63 / 125 subsets: 6,669 -> 6,921, 7,550 -> 7,645, 8,062 -> 8,211).
    const bool queues = hw_queues() >= 8;
    static const int krig_env = tile_env("MK_LA_KRIG", -1);
    if ((krig_env == 1 || (krig_env < 0 && queues)) && s->md.n_test > 0 && !s->tiled &&
        pool_stream(s->owned, &s->la_k, s->device, SK_PLAIN) != hipSuccess)
      return set_err(MK_E_HIP, "lookahead kriging stream");
    static const int mask_env = tile_env("MK_LA_MASK", -1);
    const int mask_cu = mask_env >= 0 ? mask_env : (queues ? 32 : 0);
    int n_cu = 0;
    if (mask_cu > 0 && hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, s->device) == hipSuccess) {
      std::vector<uint32_t> mask((n_cu + 31) / 32, 0xffffffffu);
      for (int b = 0; b < mask_cu && b < n_cu; ++b) mask[b / 32] &= ~(1u << (b % 32));
      if (pool_stream(s->owned, &s->la_m, s->device, SK_CUMASK, 0, mask) != hipSuccess)
        return set_err(MK_E_HIP, "lookahead main stream");
    }
  }
  static const int early_cov = tile_env("MK_EARLY_COV", 1);
  // (the inverse must have its own scratch Y: without it, it works in the free factor slots)
  if (early_cov && !s->la && s->groups.size() == 1 && s->ms.Y && !s->cov_st) {
    if (pool_stream(s->owned, &s->cov_st, s->device, SK_PLAIN) != hipSuccess) return set_err(MK_E_HIP, "covariance stream");
    for (auto& e : s->cov_ev)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return set_err(MK_E_HIP, "covariance event");
  }
  const bool swap_m = s->la && s->la_m;
  if (swap_m) {   // the iterations' main-stream work on la_m, after everything queued on the session stream
    hipEventRecord(s->la_ev[s->nt + 1], s->stream);
    hipStreamWaitEvent(s->la_m, s->la_ev[s->nt + 1], 0);
    s->groups[0].stream = s->la_m;
  }
  const auto t0 = std::chrono::steady_clock::now();
  s->launch_err = hipSuccess;
  hipError_t le = hipSuccess;
  for (int i = 0; i < n_iter; ++i) {
    s->prof_iter = s->prof_every <= 1 || s->iter % s->prof_every == 0;
    run_iteration(s, s->iter);
    s->iter++;
    le = hipGetLastError();
    if (le == hipSuccess) le = s->launch_err;
    if (le != hipSuccess) break;
  }
  s->prof_iter = true;   // launches outside the iterations (the tiled replay) follow prof alone
  if (swap_m) s->groups[0].stream = s->stream;
  // every stream is drained before an error returns: nothing of this run is left queued
  if (le != hipSuccess) {
    for (hipStream_t st : {s->la_m, s->la_c, s->la_k, s->cov_st}) if (st) (void)hipStreamSynchronize(st);
    s->kt_pending = false;
    for (auto& g : s->groups) (void)hipStreamSynchronize(g.stream);
    return set_err(MK_E_HIP, std::string("kernel launch in iteration ") + std::to_string(s->iter - 1) + ": " +
                                 hipGetErrorString(le));
  }
  if (swap_m) HIPCHK(hipStreamSynchronize(s->la_m));
  for (auto& g : s->groups) HIPCHK(hipStreamSynchronize(g.stream));
  if (s->la_c) HIPCHK(hipStreamSynchronize(s->la_c));   // the next iteration's candidates
  if (s->la_k) HIPCHK(hipStreamSynchronize(s->la_k));
  if (s->kt_pending) {   // the last kept iteration's table draws (side stream)
    HIPCHK(hipEventSynchronize(s->kt_ev[1]));
    s->kt_pending = false;
  }
  if (s->sweep_coop) {
    // the multi-workgroup sweep's barrier time-out (after admission every wait completes: this is the
    // net under that argument): its chain state is then not the sampler's -- the session is
    // poisoned, every later call on it fails
    int e[2] = {0, 0};
    HIPCHK(hipMemcpy(e, s->sw_err, 2 * sizeof(int), hipMemcpyDeviceToHost));
    if (e[1]) {
      s->stats[KS_SWEEP_FALLBACK].launches += e[1];
      HIPCHK(hipMemset(s->sw_err + 1, 0, sizeof(int)));
    }
    if (e[0]) {
      s->poisoned = "latent sweep: workgroup barrier timed out (MK_SWEEP=3 avoids the kernel)";
      return set_err(MK_E_HIP, s->poisoned);
    }
  }
  if (s->prof) {
    s->stats[KS_ITER].launches += n_iter;
    s->stats[KS_ITER].ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    drain_timers(s);
  }
  return 0;
}

extern "C" int32_t mk_session_iteration(const mk_session* s) { return s ? s->iter : -1; }

extern "C" int32_t mk_session_predict_tile(const mk_session* s) { return (s && s->tiled) ? s->pred_tile : 0; }

// The chain state of one subset after the iterations run so far, in spMvGLM's MH order: beta (p),
// theta (n_theta: A lower-tri col-major with log diagonal | logit phi | logit nu), w (n_s q,
// location-major), tune (p + n_theta + n_s q log proposal sds) and accept (the same, accept counts
// of the current amcmc batch).  Any pointer may be NULL.  A host can resume the chain elsewhere from
// it -- bench.py's CPU baseline times the oracle over the very window the device timed.
extern "C" int mk_session_chain_state(mk_session* s, int32_t subset, double* beta, double* theta, double* w,
                                      double* tune, double* accept) {
  if (!s) return set_err(MK_E_ARG, "null session");
  if (s->poisoned) return set_err(MK_E_HIP, std::string("session unusable after an earlier failure: ") + s->poisoned);
  if (subset < 0 || subset >= s->S) return set_err(MK_E_ARG, "subset out of range");
  MK_ENTRY_DEVICE(s->device);
  const Model& md = s->md;
  const long i = subset, nq = (long)s->n_part[subset] * s->q, nmh = md.o_w + nq;
  HIPCHK(hipStreamSynchronize(s->stream));
  if (beta) HIPCHK(hipMemcpy(beta, md.beta + i * md.p, (size_t)md.p * 8, hipMemcpyDeviceToHost));
  if (theta) HIPCHK(hipMemcpy(theta, md.theta + i * md.n_theta, (size_t)md.n_theta * 8, hipMemcpyDeviceToHost));
  if (w) HIPCHK(hipMemcpy(w, md.w + i * md.Np, (size_t)nq * 8, hipMemcpyDeviceToHost));
  if (tune) HIPCHK(hipMemcpy(tune, md.tune + i * md.n_mh_max, (size_t)nmh * 8, hipMemcpyDeviceToHost));
  if (accept) HIPCHK(hipMemcpy(accept, md.acc + i * md.n_mh_max, (size_t)nmh * 8, hipMemcpyDeviceToHost));
  return 0;
}


extern "C" int mk_session_set_lookahead(mk_session* s, int32_t mode) {
  if (!s) return set_err(MK_E_ARG, "null session");
  if (mode < -1 || mode > 1) return set_err(MK_E_ARG, "lookahead mode must be -1 (auto), 0 or 1");
  if (s->iter > 0) return set_err(MK_E_ARG, "the schedule is fixed once the chain has started");
  if (mode == 1 && !s->la_ok)
    return set_err(MK_E_ARG, "lookahead needs the exponential model on one stream group");
  s->la_mode = mode;
  s->la = s->la_ok && (mode == 1 || (mode == -1 && la_auto(s)));
  return 0;
}

extern "C" int32_t mk_session_lookahead(const mk_session* s) { return (s && s->la) ? 1 : 0; }

extern "C" int mk_session_profile(mk_session* s, int32_t enable) {
  if (!s) return set_err(MK_E_ARG, "null session");
  s->prof = enable != 0;
  s->prof_kinds = (enable == 1) ? ~0u : ((uint32_t)enable >> 1);
  return 0;
}

extern "C" int mk_session_profile_every(mk_session* s, int32_t every) {
  if (!s) return set_err(MK_E_ARG, "null session");
  if (every < 1) return set_err(MK_E_ARG, "every must be >= 1");
  s->prof_every = every;
  return 0;
}

extern "C" int mk_session_kernel_stats(const mk_session* s, int32_t which, int64_t* launches, double* total_ms,
                                       double* flops) {
  if (!s || which < 0 || which >= NKSTAT) return set_err(MK_E_ARG, "bad stats query");
  if (launches) *launches = s->stats[which].launches;
  if (total_ms) *total_ms = s->stats[which].ms;
  if (flops) *flops = s->stats[which].flops;
  return 0;
}

// ------------------------------------------------------------------ scoped device scratch (freed on every return path)
namespace {
struct DevBufs {
  std::vector<void*> p;
  ~DevBufs() {
    for (void* x : p) hipFree(x);
  }
  template <typename T>
  T* get(size_t n) {
    void* x = nullptr;
    if (hipMalloc(&x, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) {
      (void)hipGetLastError();   // not sticky for the caller's later launch checks
      return nullptr;
    }
    p.push_back(x);
    return (T*)x;
  }
};

}  // namespace

// A tile's draws are in md.w_pred ([S][n_kept][Ct]): its 200-level grids into dq and, if
// o->w_pred_samples, the draws to the host.  Returns after the stream is idle.
static int tile_outputs(mk_session* s, int t0, double* dq, mk_outputs* o, int n_kept, int Ct) {
  Model& md = s->md;
  const int S = s->S, q = s->q;
  const long C = (long)q * s->n_test_all;
  hipStream_t st = s->stream;
  if (dq) {
    const int rq = launch_quantiles(S * Ct, st, md.w_pred, (long)n_kept * Ct, (long)Ct, n_kept, Ct, s->d_probs,
                                    MK_N_LEVELS, dq);
    if (rq) return rq;
  }
  if (o && o->w_pred_samples)   // per subset (C x kept) column-major
    for (int i = 0; i < S; ++i)
      HIPCHK(hipMemcpy2DAsync(o->w_pred_samples + (size_t)i * n_kept * C + (size_t)t0 * q, (size_t)C * 8,
                              md.w_pred + (size_t)i * n_kept * Ct, (size_t)Ct * 8, (size_t)Ct * 8, n_kept,
                              hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

// ------------------------------------------------------------------ kriging variance by phi interpolation
// (exponential, q = 1; DESIGN.md 4.7, mk_mcmc.hip section 11).  s(t; phi) = rho_t' R(phi)^-1 rho_t is
// analytic in phi: it is computed exactly (the replay's own kernels: candidate, Cholesky, inverse,
// X = W P^T) at nc Chebyshev nodes (first kind) of a phi range per subset and interpolated (barycentric)
// wherever a draw needs it.  nc = 6 + ceil((phi_hi - phi_lo) * d_max), at least 10, at most 32 (d_max:
// the subset's largest site-to-site or site-to-test-site distance, so the rule counts the range in units
// of the correlation decay; measured in float64 on 2,000-site subsets with clustered sites and test
// sites 1e-6 from a site, d_max 1.41: |error| 2e-14 over phi in [3.3, 11.8] with the rule's 18 nodes,
// 1e-14 over [4.5, 10.5] with 15, 1e-14 over [6, 8] with 10; on the GPU at configs[4] 4 + ceil(.), at
// least 8, left 6.5e-12 and 8 + ceil(.), at least 12, 2.6e-14).  The
// exact values at nchk check points (the range's ends, then interior points) bound the interpolant's
// error before any draw uses it.

// The φ-interpolated paths return 0 when done, this when the exact path must run instead (not
// applicable, scratch memory short, a check failed), and an MK_E_* code (< 0) on an error.
constexpr int MK_CHEB_EXACT = 1;

// Nodes of [lo, hi] for each subset: nc[i], the slots' phi (nodes, then nchk check points) and the
// barycentric weights.  Returns the slot count E (the largest nc + nchk).
static int cheb_plan(mk_session* s, const std::vector<double>& lo, const std::vector<double>& hi, int force_n, int nchk,
                     std::vector<int>& nc, std::vector<std::vector<double>>& sphi, std::vector<double>& wts) {
  const int S = s->S;
  nc.assign(S, 0);
  sphi.assign(S, {});
  wts.assign((size_t)S * MK_CHEB_MAX, 0.0);
  int E = 0;
  for (int i = 0; i < S; ++i) {
    const double* bb = s->bbox.data() + 4 * i;
    const double dmax = std::fmax(s->span_pt_h[i], std::hypot(bb[1] - bb[0], bb[3] - bb[2]));
    const int n = force_n > 1 ? std::min(force_n, MK_CHEB_MAX)
                              : std::max(10, std::min(MK_CHEB_MAX, 6 + (int)std::ceil((hi[i] - lo[i]) * dmax)));
    nc[i] = n;
    const double c = 0.5 * (lo[i] + hi[i]), h = 0.5 * (hi[i] - lo[i]);
    for (int m = 0; m < n; ++m) {
      const double ang = M_PI * (2.0 * m + 1.0) / (2.0 * n);
      sphi[i].push_back(c + h * std::cos(ang));
      wts[(size_t)i * MK_CHEB_MAX + m] = ((m & 1) ? -1.0 : 1.0) * std::sin(ang);
    }
    static const double frac[5] = {0.0, 1.0, 0.5, 0.25, 0.75};
    for (int k = 0; k < nchk; ++k) sphi[i].push_back(lo[i] + frac[k] * (hi[i] - lo[i]));
    E = std::max(E, n + nchk);
  }
  return E;
}

// Exact s of every planned slot into Sn ([slot][S][n_test_pad] of mt's sites) and the slots' device phi
// into nphi; then the interpolant against the check points (largest difference into *emax).  The factor
// slots, cur and W serve as scratch: callers are the tiled replay (the chain is finished) and session
// set-up (before the initial factorisation).  The host stays at most four slots ahead of the device.
static int cheb_eval(mk_session* s, Model mt, const std::vector<int>& nc, const std::vector<std::vector<double>>& sphi,
                     const std::vector<double>& wts, int E, int nchk, DevBufs& scratch, ChebK* ck, double* emax) {
  Model& md = s->md;
  const int S = s->S, nth = md.n_theta, T_pad = md.n_test_pad;
  const double pa = md.phi_a[0], pb = md.phi_b[0];
  hipStream_t st = s->stream;
  Group g = s->all;
  // slot e's theta (phi in the candidate's logit form; the device's phi of it is what counts) and its
  // subset list (the subsets with that many slots)
  std::vector<double> thn((size_t)E * S * nth, 0.0);
  std::vector<int> lists((size_t)E * (S + 1), 0);
  for (int e = 0; e < E; ++e) {
    int cnt = 0;
    for (int i = 0; i < S; ++i) {
      const double ph = e < (int)sphi[i].size() ? sphi[i][e] : sphi[i][0];
      thn[((size_t)e * S + i) * nth + md.ntri] = std::log((ph - pa) / (pb - ph));
      if (e < (int)sphi[i].size()) lists[(size_t)e * (S + 1) + cnt++] = i;
    }
    lists[(size_t)e * (S + 1) + S] = cnt;
  }
  double* d_thn = scratch.get<double>(thn.size());
  double* d_nphi = scratch.get<double>((size_t)E * S);
  double* d_wts = scratch.get<double>(wts.size());
  int* d_nc = scratch.get<int>((size_t)S);
  int* d_lists = scratch.get<int>(lists.size());
  double* d_Sn = scratch.get<double>((size_t)E * S * T_pad);
  unsigned long long* d_err = scratch.get<unsigned long long>(1);
  if (!d_thn || !d_nphi || !d_wts || !d_nc || !d_lists || !d_Sn || !d_err) return MK_CHEB_EXACT;
  HIPCHK(hipMemcpyAsync(d_thn, thn.data(), thn.size() * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_wts, wts.data(), wts.size() * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_nc, nc.data(), (size_t)S * sizeof(int), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(d_lists, lists.data(), lists.size() * sizeof(int), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemsetAsync(d_Sn, 0, (size_t)E * S * T_pad * 8, st));
  HIPCHK(hipMemsetAsync(d_err, 0, 8, st));
  MK_LAUNCH(k_kept_phi, dim3((unsigned)(((long)E * S + 255) / 256)), dim3(256), 0, st, md, d_thn, E, d_nphi);
  for (int e = 0; e < E; ++e) {
    int* L = d_lists + (size_t)e * (S + 1);
    int* C = L + S;
    mt.theta = d_thn + (size_t)e * S * nth;
    mt.s_pred = d_Sn + (size_t)e * S * T_pad;
    launch_candidates(mt, g.ms, st, S, 0, 1, 2, 0, L, C);
    launch_cholesky(s, g, 0, 1, L, C);
    MK_LAUNCH(k_flip_pairs, dim3((S + 255) / 256), dim3(256), 0, st, g.ms, L, C);
    launch_trinv(s, g, S, L, C);
    Group gp = g;
    gp.md = mt;
    gp.d_plist = L;
    gp.d_pcount = C;
    launch_pred_refresh(s, gp);
    HIPCHK(hipGetLastError());
    if (e % 4 == 3) HIPCHK(hipStreamSynchronize(st));   // four slots are ~0.6 s of GEMMs at configs[4]
  }
  ck->Sn = d_Sn;
  ck->nphi = d_nphi;
  ck->wts = d_wts;
  ck->nc = d_nc;
  ck->nchk = nchk;
  ck->T_pad = T_pad;
  MK_LAUNCH(k_cheb_check, dim3(S * ((mt.n_test + 255) / 256)), dim3(256), 0, st, mt, *ck, d_err);
  unsigned long long eb = 0;
  HIPCHK(hipMemcpyAsync(&eb, d_err, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  std::memcpy(emax, &eb, 8);
  return 0;
}

static double cheb_tol() {
  const char* tenv = std::getenv("MK_KRIG_CHEB_TOL");
  return (tenv && *tenv) ? std::atof(tenv) : 1e-10;
}

// Fused kriging by phi tables (called by mk_session_create before the initial factorisation; exponential,
// q = 1, one group).  The fused path refreshes X = W P^T at every kept iteration for the pairs whose phi
// changed (~0.4 of them at configs[2]: 6.9 ms of a kept iteration at 250 subsets).  Instead, s(t; phi)
// is computed once over the prior's whole phi range [a, b] (MK.R:63 phi.Unif), so it holds wherever the
// chain goes: Chebyshev nodes of [a, b] per subset, checked at a, b, the middle and the quarters (5
// points); a difference above MK_KRIG_CHEB_TOL keeps the exact refresh for the session (KS_KRIG_FALLBACK).
// Kept iterations then draw with g = W' z (one W pass) and the interpolated s (k_pred_tab_draw).
// MK_KRIG_CHEB: 1 (default) where the kept window's expected refreshes (0.25 n_kept per subset, below
// the amcmc target's 0.43) exceed the nodes and checks, -1 always, n > 1 always with n nodes, 0 never.
static int krig_tables(mk_session* s) {
  Model& md = s->md;
  s->kt_on = false;
  const char* env = std::getenv("MK_KRIG_CHEB");
  const int force_n = (env && *env) ? std::atoi(env) : 1;
  const int S = s->S;
  if (force_n == 0 || s->tiled || md.n_test <= 0 || s->q != 1 || md.cov_model != MK_COV_EXPONENTIAL ||
      s->groups.size() != 1 || (int)s->span_pt_h.size() != S)
    return 0;
  const double pa = md.phi_a[0], pb = md.phi_b[0], eps = (pb - pa) * 1e-9;
  std::vector<double> lo(S, pa + eps), hi(S, pb - eps);
  std::vector<int> nc;
  std::vector<std::vector<double>> sphi;
  std::vector<double> wts;
  const int nchk = MK_CHEB_CHECKS_MAX;
  const int E = cheb_plan(s, lo, hi, force_n, nchk, nc, sphi, wts);
  double evals = 0.0;
  for (int i = 0; i < S; ++i) evals += nc[i] + nchk;
  if (force_n == 1 && 0.25 * md.n_kept * S <= evals) return 0;
  Model mt = md;   // every test site (the fused path's buffers hold them all)
  DevBufs scratch;
  ChebK ck;
  double emax = 0.0;
  const int rc = cheb_eval(s, mt, nc, sphi, wts, E, nchk, scratch, &ck, &emax);
  if (rc < 0) return rc;
  if (rc == MK_CHEB_EXACT) return 0;   // scratch memory short: exact refreshes
  s->kt_check = emax;
  if (!(emax <= cheb_tol())) {          // the check failed: exact refreshes
    s->kt_fail += 1;
    return 0;
  }
  // keep the node slots (the checks are not needed past this point)
  int nmax = 0;
  for (int i = 0; i < S; ++i) nmax = std::max(nmax, nc[i]);
  const size_t sn = (size_t)nmax * S * md.n_test_pad;
  double *Sn = nullptr, *nphi = nullptr, *w = nullptr;
  int* n = nullptr;
  if (s->alloc(&Sn, sn) || s->alloc(&nphi, (size_t)nmax * S) || s->alloc(&w, wts.size()) || s->alloc(&n, (size_t)S) ||
      s->alloc(&s->kt_g, (size_t)S * md.n_pad) || s->alloc(&s->kt_z, (size_t)S * (md.n_pad + 2))) {
    // HBM short: the session keeps the exact refresh (the tables are an optimisation, not a requirement)
    for (void* b : {(void*)Sn, (void*)nphi, (void*)w, (void*)n, (void*)s->kt_g, (void*)s->kt_z}) s->release(b);
    s->kt_g = s->kt_z = nullptr;
    set_err(0, "");
    return 0;
  }
  for (auto& e : s->kt_ev)
    if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return set_err(MK_E_HIP, "table event");
  HIPCHK(hipMemcpyAsync(Sn, ck.Sn, sn * 8, hipMemcpyDeviceToDevice, s->stream));
  HIPCHK(hipMemcpyAsync(nphi, ck.nphi, (size_t)nmax * S * 8, hipMemcpyDeviceToDevice, s->stream));
  HIPCHK(hipMemcpyAsync(w, ck.wts, wts.size() * 8, hipMemcpyDeviceToDevice, s->stream));
  HIPCHK(hipMemcpyAsync(n, ck.nc, (size_t)S * sizeof(int), hipMemcpyDeviceToDevice, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  s->kt.Sn = Sn;
  s->kt.nphi = nphi;
  s->kt.wts = w;
  s->kt.nc = n;
  s->kt.nchk = 0;
  s->kt.T_pad = md.n_test_pad;
  s->kt_evals = evals;
  s->kt_on = true;
  return 0;
}

// Tile [t0, t0 + Tc) of the tiled replay by phi interpolation: nodes over each subset's kept phi range,
// checked at its ends and middle (a difference above MK_KRIG_CHEB_TOL, default 1e-10, sends the tile
// to the exact replay: KS_KRIG_FALLBACK); the mean m_k(t) = rho_t(phi_k)' g_k with g_k = W_k' z_k made
// once per kept window (the exact replay's factorisations where phi changed, one W' z per state).  At
// configs[4]: ~490 X refreshes per subset and tile become 13-21 nodes + 3 checks.  MK_KRIG_CHEB: 1
// (default) where the nodes and checks cost fewer exact evaluations than the exact replay's refreshes,
// -1 always, n > 1 always with n nodes, 0 never (the exact replay); read at every tile.
// Returns 0, MK_CHEB_EXACT (the exact replay must run) or an error (< 0).
static int predict_tile_cheb(mk_session* s, int t0, double* dq, mk_outputs* o) {
  Model& md = s->md;
  const char* env = std::getenv("MK_KRIG_CHEB");
  const int force_n = (env && *env) ? std::atoi(env) : 1;   // 0 exact, 1 auto, -1 always, n > 1 always, n nodes
  if (force_n == 0 || s->q != 1 || md.cov_model != MK_COV_EXPONENTIAL) return MK_CHEB_EXACT;
  const int S = s->S, nth = md.n_theta, n_pad = md.n_pad;
  const int k_lo = s->win_lo, n_kept = s->win_n < 0 ? md.n_kept : s->win_n;
  if (n_kept < 1 || (int)s->span_pt_h.size() != S) return MK_CHEB_EXACT;
  const int T_pad = md.n_test_pad, Tc = std::min(s->pred_tile, s->n_test_all - t0);
  hipStream_t st = s->stream;
  Group g = s->all;
  s->la_next = -1;   // the replay factors into the free slots
  s->cov_pre = -1;
  // 1. phi_k of the window's kept states (once per window)
  if (s->cg_iter != s->iter || s->cg_lo != k_lo || s->cg_n != n_kept) {
    s->release(s->cg_G);
    s->release(s->cg_phi);
    s->release(s->cg_phit);
    s->cg_G = s->cg_phi = s->cg_phit = nullptr;
    s->cg_iter = -1;
    if (s->alloc(&s->cg_phi, (size_t)n_kept * S)) return MK_CHEB_EXACT;
    MK_LAUNCH(k_kept_phi, dim3((unsigned)(((long)n_kept * S + 255) / 256)), dim3(256), 0, st, md,
              md.kth + (long)k_lo * S * nth, n_kept, s->cg_phi);
    s->cg_phi_h.assign((size_t)n_kept * S, 0.0);
    HIPCHK(hipMemcpyAsync(s->cg_phi_h.data(), s->cg_phi, (size_t)n_kept * S * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    s->cg_iter = s->iter;
    s->cg_lo = k_lo;
    s->cg_n = n_kept;
  }
  // 2. per subset: nodes over its kept phi range (a nearly fixed phi: a short interval around it)
  const double pa = md.phi_a[0], pb = md.phi_b[0];
  std::vector<double> lo(S), hi(S);
  long refreshes = 0;
  for (int i = 0; i < S; ++i) {
    double l = s->cg_phi_h[i], h = l;
    refreshes += 1;
    for (int j = 1; j < n_kept; ++j) {
      const double v = s->cg_phi_h[(size_t)j * S + i];
      refreshes += v != s->cg_phi_h[(size_t)(j - 1) * S + i];
      l = std::fmin(l, v);
      h = std::fmax(h, v);
    }
    const double mag = std::fmax(1.0, std::fabs(l));
    if (h - l < 1e-6 * mag) {
      const double c = 0.5 * (l + h);
      l = c - 5e-7 * mag;
      h = c + 5e-7 * mag;
    }
    const double eps = (pb - pa) * 1e-9;
    lo[i] = std::fmax(l, pa + eps);
    hi[i] = std::fmin(h, pb - eps);
  }
  std::vector<int> nc;
  std::vector<std::vector<double>> sphi;
  std::vector<double> wts;
  const int E = cheb_plan(s, lo, hi, force_n, MK_CHEB_CHECKS, nc, sphi, wts);
  long evals = 0;
  for (int i = 0; i < S; ++i) evals += nc[i] + MK_CHEB_CHECKS;
  // auto: only where it saves exact evaluations -- the exact replay refreshes X at each subset's first
  // state and wherever phi changed (a short window, e.g. the bench's 6-state kriging sample, refreshes
  // less often than a range needs nodes)
  if (force_n == 1 && evals >= refreshes) return MK_CHEB_EXACT;
  // 3. g_k = W_k' z_k of the window's kept states (once per window): the exact replay's
  //    factorisations where phi changed, then one W' z per state
  const int nkp = (n_kept + 7) / 8 * 8;
  if (!s->cg_G) {
    if (s->alloc(&s->cg_G, (size_t)S * n_pad * nkp)) return MK_CHEB_EXACT;
    if (s->alloc(&s->cg_phit, (size_t)S * nkp)) {
      s->release(s->cg_G);
      s->cg_G = nullptr;
      return MK_CHEB_EXACT;
    }
    std::vector<double> pt((size_t)S * nkp);
    for (int i = 0; i < S; ++i)
      for (int j = 0; j < nkp; ++j) pt[(size_t)i * nkp + j] = s->cg_phi_h[(size_t)std::min(j, n_kept - 1) * S + i];
    HIPCHK(hipMemcpyAsync(s->cg_phit, pt.data(), pt.size() * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(s->cg_G, 0, (size_t)S * n_pad * nkp * 8, st));
    Model mt = md;
    for (int j = 0; j < n_kept; ++j) {
      const int k = k_lo + j;
      mt.theta = md.kth + (long)k * S * nth;
      const double* prev = j ? md.kth + (long)(k - 1) * S * nth : nullptr;
      MK_LAUNCH(k_kept_dirty, dim3(1), dim3(256), 0, st, mt, prev, s->d_slist, s->d_scount, g.d_plist, g.d_pcount);
      launch_candidates(mt, g.ms, st, S, 0, 1, 2, 0, s->d_slist, s->d_scount);
      launch_cholesky(s, g, 0, 1, s->d_slist, s->d_scount);
      MK_LAUNCH(k_flip_pairs, dim3((S + 255) / 256), dim3(256), 0, st, g.ms, g.d_plist, g.d_pcount);
      launch_trinv(s, g, S, g.d_plist, g.d_pcount);
      MK_LAUNCH(k_krig_g, dim3(S * (n_pad / 4)), dim3(256), 0, st, mt, g.ms, md.kz + (long)k * S * n_pad, s->cg_G,
                j, nkp);
      HIPCHK(hipGetLastError());
      // the host stays at most 32 states (~2,000 launches) ahead: rocprofv3's queue intercept read
      // past its packet buffer with tens of thousands queued
      if (j % 32 == 31) HIPCHK(hipStreamSynchronize(st));
    }
  }
  // 4. the tile's sites (as predict_tile), exact s at every slot, the check
  HIPCHK(hipMemsetAsync((void*)md.coords_test, 0, (size_t)2 * T_pad * 8, st));
  HIPCHK(hipMemcpyAsync((void*)md.coords_test, s->d_ct_all + t0, (size_t)Tc * 8, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemcpyAsync((void*)(md.coords_test + T_pad), s->d_ct_all + s->n_test_pad_all + t0, (size_t)Tc * 8,
                        hipMemcpyDeviceToDevice, st));
  Model mt = md;
  mt.n_kept = n_kept;
  mt.n_test = Tc;
  mt.t_off = t0;
  mt.ntt = (Tc + MK_NB - 1) / MK_NB;
  DevBufs scratch;
  ChebK ck;
  double emax = 0.0;
  const int rc = cheb_eval(s, mt, nc, sphi, wts, E, MK_CHEB_CHECKS, scratch, &ck, &emax);
  if (rc) return rc;
  if (!(emax <= cheb_tol())) {
    Stat& f = s->stats[KS_KRIG_FALLBACK];
    f.launches += 1;
    f.ms = std::fmax(f.ms, std::isfinite(emax) ? emax : 1e300);
    return MK_CHEB_EXACT;
  }
  // 5. the draws
  MK_LAUNCH(k_pred_cheb_draw, dim3(S * ((Tc + 255) / 256)), dim3(256), 0, st, mt, ck, s->cg_G, s->cg_phit, md.coords,
            md.kA, k_lo, nkp);
  HIPCHK(hipGetLastError());
  Stat& c = s->stats[KS_KRIG_CHEB];
  c.launches += 1;
  c.flops += (double)evals;
  c.ms = std::fmax(c.ms, emax);
  return tile_outputs(s, t0, dq, o, n_kept, s->q * Tc);
}

// spPredict after the fit (MK.R:87-89) over test-site tiles: replays the kriging of every kept
// iteration from the recorded chain states (z, theta, A).  A factor is recomputed only where
// (phi, nu) changed since the previous kept sample, with the same kernels and inputs as in the
// fit (rows < n_s of a factor do not depend on its border row), so the draws, the quantiles and
// their sum are bit-identical to the fused path.  Per tile the device holds q*T x kept draws
// per subset instead of q*n_test x kept.
// One tile [t0, t0 + Tc): the replay, then the tile's 200-level grids into dq ([S][q*Tc][200] in
// HBM, on s->stream) and, if o->w_pred_samples, its draws to the host.  Returns after the stream
// is idle.
static int predict_tile(mk_session* s, int t0, double* dq, mk_outputs* o) {
  const int rc_cheb = predict_tile_cheb(s, t0, dq, o);
  if (rc_cheb != MK_CHEB_EXACT) return rc_cheb;
  Model& md = s->md;
  const int S = s->S, q = s->q;
  const int k_lo = s->win_lo, n_kept = s->win_n < 0 ? md.n_kept : s->win_n;   // kept states replayed
  const int T = s->pred_tile, T_pad = md.n_test_pad, n_test = s->n_test_all;
  const long C = (long)q * n_test;
  const int Tc = std::min(T, n_test - t0);
  const int Ct = q * Tc;
  hipStream_t st = s->stream;
  Group g = s->all;
  s->la_next = -1;   // the replay factors into the free slots: a lookahead candidate is gone
  s->cov_pre = -1;   // and so is an early-assembled one
  HIPCHK(hipMemsetAsync((void*)md.coords_test, 0, (size_t)2 * T_pad * 8, st));
  HIPCHK(hipMemcpyAsync((void*)md.coords_test, s->d_ct_all + t0, (size_t)Tc * 8, hipMemcpyDeviceToDevice, st));
  HIPCHK(hipMemcpyAsync((void*)(md.coords_test + T_pad), s->d_ct_all + s->n_test_pad_all + t0, (size_t)Tc * 8,
                        hipMemcpyDeviceToDevice, st));
  Model mt = md;
  mt.n_kept = n_kept;   // w_pred holds the window's draws
  mt.n_test = Tc;
  mt.t_off = t0;
  mt.ntt = (Tc + MK_NB - 1) / MK_NB;   // a short last tile: only its valid 128-site column blocks
                                        // (strides stay those of the full tile, n_test_pad)
  // q = 1 (MK_DRAW_RUNS, default on): a subset's draws wait until its X is about to change, and the
  // states of one phi run then read X once per 4 (k_pred_draw_runs; the same bits as per state)
  static const int runs_env = tile_env("MK_DRAW_RUNS", 1);
  const bool runs = q == 1 && runs_env;
  const int per = (Tc + 3) / 4;
  if (runs) {
    int rc;
    if (!s->d_run_start && (rc = s->alloc(&s->d_run_start, (size_t)S))) return rc;
    HIPCHK(hipMemsetAsync(s->d_run_start, 0, (size_t)S * sizeof(int), st));
  }
  for (int j = 0; j < n_kept; ++j) {
    const int k = k_lo + j;   // kept state k = iteration kept0 + k
    mt.theta = md.kth + (long)k * S * md.n_theta;
    mt.z = md.kz + (long)k * S * q * md.n_pad;
    mt.A_full = md.kA + (long)k * S * q * q;
    const double* prev = j ? md.kth + (long)(k - 1) * S * md.n_theta : nullptr;
    MK_LAUNCH(k_kept_dirty, dim3(1), dim3(256), 0, st, mt, prev, s->d_slist, s->d_scount, g.d_plist,
                       g.d_pcount);
    if (runs && j > 0) {   // the listed subsets' X changes now: their pending states first
      MK_LAUNCH(k_pred_draw_runs, dim3(S * per), dim3(256), 0, st, mt, md.kz, md.kA, k_lo, g.d_plist, g.d_pcount,
                s->d_run_start, j);
      MK_LAUNCH(k_run_start, dim3((S + 255) / 256), dim3(256), 0, st, g.d_plist, g.d_pcount, s->d_run_start, j);
    }
    for (int h = 0; h < q; ++h) {
      launch_candidates(mt, g.ms, st, S, h, 1, 2, 0, s->d_slist + h * S, s->d_scount + h);
      launch_cholesky(s, g, h, 1, s->d_slist + h * S, s->d_scount + h);
    }
    MK_LAUNCH(k_flip_pairs, dim3((S * q + 255) / 256), dim3(256), 0, st, g.ms, g.d_plist, g.d_pcount);
    launch_trinv(s, g, S * q, g.d_plist, g.d_pcount);
    g.md = mt;
    launch_pred_refresh(s, g);
    if (!runs) MK_LAUNCH(k_pred_draw, dim3(S * per), dim3(256), 0, st, mt, md.kept0 + k, j);
    HIPCHK(hipGetLastError());
  }
  if (runs && n_kept > 0) {   // every subset's last run
    MK_LAUNCH(k_pred_draw_runs, dim3(S * per), dim3(256), 0, st, mt, md.kz, md.kA, k_lo, (const int*)nullptr,
              (const int*)nullptr, s->d_run_start, n_kept);
    HIPCHK(hipGetLastError());
  }
  return tile_outputs(s, t0, dq, o, n_kept, Ct);
}

static int predict_tiled(mk_session* s, mk_outputs* o) {
  const int S = s->S, q = s->q;
  const int T = s->pred_tile, n_test = s->n_test_all;
  const long C = (long)q * n_test;
  hipStream_t st = s->stream;
  DevBufs scratch;
  double* dq = scratch.get<double>((size_t)S * q * T * MK_N_LEVELS);
  double* dsum = scratch.get<double>((size_t)q * T * MK_N_LEVELS);
  if (!dq || !dsum) return set_err(MK_E_NOMEM, "tiled kriging scratch");
  const bool grids = o->w_predict || o->w_predict_sum;
  for (int t0 = 0; t0 < n_test; t0 += T) {
    const int Ct = q * std::min(T, n_test - t0);
    int rc = predict_tile(s, t0, grids ? dq : nullptr, o);
    if (rc) return rc;
    if (o->w_predict)   // per subset [C][200]: this tile's columns
      HIPCHK(hipMemcpy2DAsync(o->w_predict + (size_t)t0 * q * MK_N_LEVELS, (size_t)C * MK_N_LEVELS * 8, dq,
                              (size_t)Ct * MK_N_LEVELS * 8, (size_t)Ct * MK_N_LEVELS * 8, S, hipMemcpyDeviceToHost, st));
    if (o->w_predict_sum) {
      MK_LAUNCH(k_combine, dim3((unsigned)(((long)Ct * MK_N_LEVELS + 255) / 256)), dim3(256), 0, st, dq, S,
                         (long)Ct * MK_N_LEVELS, dsum, 0);
      HIPCHK(hipMemcpyAsync(o->w_predict_sum + (size_t)t0 * q * MK_N_LEVELS, dsum, (size_t)Ct * MK_N_LEVELS * 8,
                            hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipStreamSynchronize(st));
  }
  return 0;
}

// ------------------------------------------------------------------ shard interface (mk_multi.hip)
namespace mk {
int session_info(const mk_session* s, ShardInfo* in) {
  in->device = s->device;
  in->S = s->S;
  in->P = s->P;
  in->q = s->q;
  in->n_test = s->n_test_all;
  in->tiled = s->tiled ? 1 : 0;
  in->pred_tile = s->tiled ? s->pred_tile : s->n_test_all;
  in->n_kept = s->md.n_kept;
  in->stream = s->stream;
  return 0;
}
// [S][P][200] parameter grids (obj[[i]]$parameters, MK.R:89) into d_out (HBM), on the session stream.
int session_param_grids(mk_session* s, double* d_out) {
  MK_ENTRY_DEVICE(s->device);
  Model& md = s->md;
  if (s->iter < md.n_samples) return set_err(MK_E_ARG, "quantile outputs need all n.samples iterations");
  const int rq = launch_quantiles(s->S * s->P, s->stream, md.samples + (long)md.kept0 * s->P, (long)md.n_samples * s->P,
                                  (long)s->P, md.n_kept, s->P, s->d_probs, MK_N_LEVELS, d_out);
  if (rq) return rq;
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}
// [S][q n_test][200] w.predict grids of a fused session into d_out.
int session_wpred_grids(mk_session* s, double* d_out) {
  MK_ENTRY_DEVICE(s->device);
  Model& md = s->md;
  if (s->tiled) return set_err(MK_E_ARG, "tiled sessions produce their grids per tile");
  if (s->iter < md.n_samples) return set_err(MK_E_ARG, "quantile outputs need all n.samples iterations");
  const int C = s->q * md.n_test;
  const int rq = launch_quantiles(s->S * C, s->stream, md.w_pred, (long)md.n_kept * C, (long)C, md.n_kept, C, s->d_probs,
                                  MK_N_LEVELS, d_out);
  if (rq) return rq;
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}
// Tiled session: the grids [S][q Tc][200] of test-site tile [t0, t0 + Tc) into d_out (and the
// tile's draws into o->w_pred_samples when set).
int session_tile_grids(mk_session* s, int t0, double* d_out, mk_outputs* o) {
  MK_ENTRY_DEVICE(s->device);
  if (!s->tiled) return set_err(MK_E_ARG, "not a tiled session");
  if (s->iter < s->md.n_samples) return set_err(MK_E_ARG, "quantile outputs need all n.samples iterations");
  if (t0 < 0 || t0 >= s->n_test_all || t0 % s->pred_tile) return set_err(MK_E_ARG, "bad tile offset");
  return predict_tile(s, t0, d_out, o);
}
}  // namespace mk

extern "C" int mk_session_grids(mk_session* s, int32_t which, double* out, int32_t device_out) {
  if (!s || !out) return set_err(MK_E_ARG, "null session/output");
  if (s->poisoned) return set_err(MK_E_HIP, std::string("session unusable after an earlier failure: ") + s->poisoned);
  if (which != 0 && which != 1) return set_err(MK_E_ARG, "which must be 0 (parameters) or 1 (w.predict)");
  if (which == 1 && s->tiled) return set_err(MK_E_ARG, "tiled sessions give w.predict grids per tile (mk_session_tile_grids)");
  if (which == 1 && s->md.n_test < 1) return set_err(MK_E_ARG, "the session has no test sites");
  const long C = which == 0 ? (long)s->P : (long)s->q * s->md.n_test;
  MK_ENTRY_DEVICE(s->device);
  DevBufs scratch;
  double* d = out;
  if (!device_out && !(d = scratch.get<double>((size_t)s->S * C * MK_N_LEVELS))) return set_err(MK_E_NOMEM, "grid scratch");
  const int rc = which == 0 ? session_param_grids(s, d) : session_wpred_grids(s, d);
  if (rc) return rc;
  if (!device_out) HIPCHK(hipMemcpy(out, d, (size_t)s->S * C * MK_N_LEVELS * 8, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int mk_session_tile_grids(mk_session* s, int32_t t0, double* out, int32_t device_out) {
  if (!s || !out) return set_err(MK_E_ARG, "null session/output");
  if (s->poisoned) return set_err(MK_E_HIP, std::string("session unusable after an earlier failure: ") + s->poisoned);
  if (!s->tiled) return set_err(MK_E_ARG, "tile grids need a session created with predict_tile > 0");
  if (device_out) return session_tile_grids(s, t0, out, nullptr);
  const long Tc = std::min(s->pred_tile, s->n_test_all - t0);
  MK_ENTRY_DEVICE(s->device);
  DevBufs scratch;
  double* dq = scratch.get<double>((size_t)s->S * s->q * std::max(Tc, 1L) * MK_N_LEVELS);
  if (!dq) return set_err(MK_E_NOMEM, "tile grid scratch");
  const int rc = session_tile_grids(s, t0, dq, nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpy(out, dq, (size_t)s->S * s->q * Tc * MK_N_LEVELS * 8, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int mk_session_outputs(mk_session* s, mk_outputs* o) {
  if (!s || !o) return set_err(MK_E_ARG, "null session/outputs");
  if (s->poisoned) return set_err(MK_E_HIP, std::string("session unusable after an earlier failure: ") + s->poisoned);
  MK_ENTRY_DEVICE(s->device);
  Model& md = s->md;
  const int S = s->S, P = s->P, q = s->q;
  const int n_test = md.n_test;
  const bool done = s->iter >= md.n_samples;
  if ((o->parameters || o->w_predict || o->w_pred_samples) && !done)
    return set_err(MK_E_ARG, "quantile/predictive outputs need all n.samples iterations");
  DevBufs scratch;
  if (o->parameters) {
    double* dq = scratch.get<double>((size_t)S * P * MK_N_LEVELS);
    if (!dq) return set_err(MK_E_NOMEM, "quantile scratch");
    int rq = launch_quantiles(S * P, s->stream, md.samples + (long)md.kept0 * P, (long)md.n_samples * P, (long)P,
                              md.n_kept, P, s->d_probs, MK_N_LEVELS, dq);
    if (rq) return rq;
    // device layout [S][P][200] == R's 200 x P column-major per subset
    HIPCHK(hipMemcpyAsync(o->parameters, dq, (size_t)S * P * MK_N_LEVELS * 8, hipMemcpyDeviceToHost, s->stream));
  }
  if (s->tiled && (o->w_predict || o->w_pred_samples || o->w_predict_sum)) {
    HIPCHK(hipStreamSynchronize(s->stream));
    int rc = predict_tiled(s, o);
    if (rc) return rc;
    if (s->prof) drain_timers(s);
  } else if ((o->w_predict || o->w_predict_sum) && n_test > 0) {
    const int C = q * n_test;
    double* dq = scratch.get<double>((size_t)S * C * MK_N_LEVELS);
    if (!dq) return set_err(MK_E_NOMEM, "quantile scratch");
    int rq = launch_quantiles(S * C, s->stream, md.w_pred, (long)md.n_kept * C, (long)C, md.n_kept, C, s->d_probs,
                              MK_N_LEVELS, dq);
    if (rq) return rq;
    if (o->w_predict)
      HIPCHK(hipMemcpyAsync(o->w_predict, dq, (size_t)S * C * MK_N_LEVELS * 8, hipMemcpyDeviceToHost, s->stream));
    if (o->w_predict_sum) {   // this shard's term of the combine: sequential sum over its subsets
      double* dsum = scratch.get<double>((size_t)C * MK_N_LEVELS);
      if (!dsum) return set_err(MK_E_NOMEM, "combine scratch");
      MK_LAUNCH(k_combine, dim3((unsigned)(((long)C * MK_N_LEVELS + 255) / 256)), dim3(256), 0, s->stream, dq,
                         S, (long)C * MK_N_LEVELS, dsum, 0);
      HIPCHK(hipMemcpyAsync(o->w_predict_sum, dsum, (size_t)C * MK_N_LEVELS * 8, hipMemcpyDeviceToHost, s->stream));
    }
  }
  HIPCHK(hipStreamSynchronize(s->stream));
  const int it = s->iter;
  if (o->samples) {
    std::vector<double> h((size_t)S * md.n_samples * P);
    HIPCHK(hipMemcpy(h.data(), md.samples, h.size() * 8, hipMemcpyDeviceToHost));
    // [S][iter][P] -> per subset n_samples x P column-major (rows beyond `it` are zero)
    for (int i = 0; i < S; ++i)
      for (int r = 0; r < md.n_samples; ++r)
        for (int cc = 0; cc < P; ++cc)
          o->samples[(size_t)i * md.n_samples * P + r + (size_t)cc * md.n_samples] =
              (r < it) ? h[((size_t)i * md.n_samples + r) * P + cc] : 0.0;
  }
  if (o->w_samples) {
    if (!md.w_samples) return set_err(MK_E_ARG, "w samples were not recorded (record_w = 0)");
    std::vector<double> h((size_t)S * md.n_samples * md.Np);
    HIPCHK(hipMemcpy(h.data(), md.w_samples, h.size() * 8, hipMemcpyDeviceToHost));
    size_t off = 0;
    for (int i = 0; i < S; ++i) {
      const int N = s->n_part[i] * q;
      for (int r = 0; r < md.n_samples; ++r)
        for (int k = 0; k < N; ++k)
          o->w_samples[off + k + (size_t)r * N] = (r < it) ? h[((size_t)i * md.n_samples + r) * md.Np + k] : 0.0;
      off += (size_t)N * md.n_samples;
    }
  }
  if (o->w_pred_samples && n_test > 0 && !s->tiled) {
    const int C = q * n_test;
    std::vector<double> h((size_t)S * md.n_kept * C);
    HIPCHK(hipMemcpy(h.data(), md.w_pred, h.size() * 8, hipMemcpyDeviceToHost));
    // [S][kept][C] -> per subset C x kept column-major (p.w.predictive.samples)
    for (int i = 0; i < S; ++i)
      for (int k = 0; k < md.n_kept; ++k)
        for (int cc = 0; cc < C; ++cc)
          o->w_pred_samples[(size_t)i * md.n_kept * C + cc + (size_t)k * C] = h[((size_t)i * md.n_kept + k) * C + cc];
  }
  if (o->acceptance) {
    const int nrep = md.o_w + 1;
    std::vector<double> h((size_t)S * md.n_batch * nrep);
    HIPCHK(hipMemcpy(h.data(), md.acc_hist, h.size() * 8, hipMemcpyDeviceToHost));
    for (int i = 0; i < S; ++i)
      for (int b = 0; b < md.n_batch; ++b)
        for (int j = 0; j < nrep; ++j)
          o->acceptance[(size_t)i * md.n_batch * nrep + b + (size_t)j * md.n_batch] =
              h[((size_t)i * md.n_batch + b) * nrep + j];
  }
  return 0;
}

extern "C" void mk_session_destroy(mk_session* s) {
  ApiCall call(__func__);
  DeviceGuard dg;
  delete s;
}

extern "C" int32_t mk_session_count(void) { return g_live_sessions.load(); }

extern "C" int mk_fit_predict_batched(const mk_problem* pr, const mk_config* c, mk_outputs* o) {
  mk_session* s = nullptr;
  int rc = mk_session_create(pr, c, &s);
  if (rc) return rc;
  rc = mk_session_run(s, c->n_batch * c->batch_length);
  if (!rc) rc = mk_session_outputs(s, o);
  mk_session_destroy(s);
  return rc;
}

namespace {
// R's seq.default(from, to, by) for by > 0: from + (0:n)*by, n = as.integer(del/by + 1e-10), pmin(x, to).
std::vector<double> r_seq(double from, double to, double by) {
  const int n = (int)((to - from) / by + 1e-10);
  std::vector<double> x(n + 1);
  for (int i = 0; i <= n; ++i) x[i] = std::fmin(from + (double)i * by, to);
  return x;
}
}  // namespace

// ------------------------------------------------------------------ combine
static int combine_host(const double* grids, int32_t K, int64_t G, double* out, int mean, int32_t device) {
  if (!grids || !out || K < 1 || G < 1) return set_err(MK_E_ARG, "bad combine arguments");
  MK_ENTRY_DEVICE(device);
  DevBufs b;
  double* dg = b.get<double>((size_t)K * G);
  double* dout = b.get<double>((size_t)G);
  if (!dg || !dout) return set_err(MK_E_NOMEM, "combine alloc");
  HIPCHK(hipMemcpy(dg, grids, (size_t)K * G * 8, hipMemcpyHostToDevice));
  MK_LAUNCH(k_combine, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, 0, dg, K, (long)G, dout, mean);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, (size_t)G * 8, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int mk_combine(const double* grids, int32_t K, int64_t G, double* out, int32_t device) {
  return combine_host(grids, K, G, out, 1, device);
}

extern "C" int mk_combine_sum(const double* grids, int32_t K, int64_t G, double* out, int32_t device) {
  return combine_host(grids, K, G, out, 0, device);
}

extern "C" int mk_combine_device(const double* d_grids, int32_t K, int64_t G, double* d_out, int32_t mean,
                                 int32_t device, void* stream) {
  if (!d_grids || !d_out || K < 1 || G < 1) return set_err(MK_E_ARG, "bad combine arguments");
  MK_ENTRY_DEVICE(device);
  MK_LAUNCH(k_combine, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_grids, K, (long)G,
                     d_out, mean ? 1 : 0);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int mk_combine_median(const double* grids, int32_t K, int32_t L, int64_t C, int32_t max_iter, double tol,
                                 double* out, int32_t* iters, int32_t device) {
  if (!grids || !out || K < 1 || L < 1 || L > 256 || C < 1 || max_iter < 1 || !(tol >= 0.0))
    return set_err(MK_E_ARG, "bad combine_median arguments (1 <= n_levels <= 256, max_iter >= 1, tol >= 0)");
  MK_ENTRY_DEVICE(device);
  DevBufs b;
  const size_t G = (size_t)L * C;
  double* dg = b.get<double>((size_t)K * G);
  double* dout = b.get<double>(G);
  int* dit = b.get<int>((size_t)C);
  if (!dg || !dout || !dit) return set_err(MK_E_NOMEM, "combine_median alloc");
  HIPCHK(hipMemcpy(dg, grids, (size_t)K * G * 8, hipMemcpyHostToDevice));
  MK_LAUNCH(k_weiszfeld, dim3((unsigned)((C + 3) / 4)), dim3(256), 0, 0, dg, K, L, (long)C, max_iter, tol, dout,
                     dit);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, G * 8, hipMemcpyDeviceToHost));
  if (iters) HIPCHK(hipMemcpy(iters, dit, (size_t)C * 4, hipMemcpyDeviceToHost));
  return 0;
}

// ------------------------------------------------------------------ post-combine steps (MK.R:136-165)
extern "C" int mk_combine_median_device(const double* d_grids, int32_t K, int32_t L, int64_t C, int32_t max_iter,
                                        double tol, double* d_out, int32_t* d_iters, int32_t device, void* stream) {
  if (!d_grids || !d_out || K < 1 || L < 1 || L > 256 || C < 1 || max_iter < 1 || !(tol >= 0.0))
    return set_err(MK_E_ARG, "bad combine_median arguments (1 <= n_levels <= 256, max_iter >= 1, tol >= 0)");
  MK_ENTRY_DEVICE(device);
  MK_LAUNCH(k_weiszfeld, dim3((unsigned)((C + 3) / 4)), dim3(256), 0, (hipStream_t)stream, d_grids, K, L, (long)C,
                     max_iter, tol, d_out, d_iters);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int mk_posterior_summary_ex(const double* result, int32_t P, const double* result2, int64_t C,
                                       const double* x_test, int32_t p, int32_t S, uint64_t seed,
                                       const int32_t* index, int32_t link, mk_summary* o, int32_t device) {
  if (!result || !o || P < 1 || C < 0 || p < 0 || p > P || S < 1 || S > MK_QUANT_MAX)
    return set_err(MK_E_ARG, "bad posterior_summary arguments (P >= 1, 0 <= p <= P, 1 <= samplesize <= 16384)");
  if (C > 0 && (!result2 || (p > 0 && !x_test))) return set_err(MK_E_ARG, "result2 / x_test missing");
  if (link != MK_LINK_LOGIT && link != MK_LINK_PROBIT) return set_err(MK_E_ARG, "link must be logit or probit");
  MK_ENTRY_DEVICE(device);
  const int L = MK_N_LEVELS;
  const std::vector<double> xg = r_seq(0.005, 1.0, 0.005);   // allquant levels (MK.R:88)
  const std::vector<double> xo = r_seq(0.005, 1.0, 0.001);   // Xout (MK.R:140)
  const int n = (int)xg.size(), NL = (int)xo.size();
  if (n != L) return set_err(MK_E_ARG, "internal: probs grid");
  // stats/src/approx.c approx1: bisection to x[i] <= v <= x[j], exact hits return y
  std::vector<int> lo(NL), hi(NL), mode(NL);
  std::vector<double> tt(NL, 0.0);
  for (int k = 0; k < NL; ++k) {
    const double v = xo[k];
    int i = 0, j = n - 1;
    while (i < j - 1) {
      const int ij = (i + j) / 2;
      if (v < xg[ij]) j = ij; else i = ij;
    }
    lo[k] = i;
    hi[k] = j;
    if (v == xg[j]) mode[k] = 0;
    else if (v == xg[i]) mode[k] = 1;
    else { mode[k] = 2; tt[k] = (v - xg[i]) / (xg[j] - xg[i]); }
  }
  const double probs3[3] = {0.5, 0.025, 0.975};   // quant.pred (MK.R:163)
  DevBufs b;
  const size_t Cs = (size_t)std::max<int64_t>(C, 1);
  double* d_res = b.get<double>((size_t)L * P);
  double* d_res2 = b.get<double>((size_t)L * Cs);
  double* d_xt = b.get<double>(Cs * std::max(p, 1));
  int* d_idx = b.get<int>(S);
  int* d_lo = b.get<int>(NL);
  int* d_hi = b.get<int>(NL);
  int* d_mode = b.get<int>(NL);
  double* d_t = b.get<double>(NL);
  double* d_spar = b.get<double>((size_t)S * P);
  double* d_sw = b.get<double>((size_t)S * Cs);
  double* d_p = b.get<double>((size_t)S * Cs);
  double* d_q = b.get<double>((size_t)3 * std::max<size_t>(Cs, P));
  double* d_pr = b.get<double>(3);
  if (!d_res || !d_res2 || !d_xt || !d_idx || !d_lo || !d_hi || !d_mode || !d_t || !d_spar || !d_sw || !d_p || !d_q ||
      !d_pr)
    return set_err(MK_E_NOMEM, "posterior_summary alloc");
  hipStream_t st = 0;
  HIPCHK(hipMemcpy(d_res, result, (size_t)L * P * 8, hipMemcpyHostToDevice));
  if (C > 0) HIPCHK(hipMemcpy(d_res2, result2, (size_t)L * C * 8, hipMemcpyHostToDevice));
  if (C > 0 && p > 0) HIPCHK(hipMemcpy(d_xt, x_test, (size_t)C * p * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_lo, lo.data(), NL * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_hi, hi.data(), NL * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_mode, mode.data(), NL * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_t, tt.data(), NL * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_pr, probs3, 3 * 8, hipMemcpyHostToDevice));
  if (index) {   // sampleparIndex drawn by the caller (R: sample(seq(1, length(Xout), 1), ...)), 1-based
    std::vector<int> hidx(S);
    for (int j = 0; j < S; ++j) {
      if (index[j] < 1 || index[j] > NL) return set_err(MK_E_ARG, "index entries must be in 1..length(Xout)");
      hidx[j] = index[j] - 1;
    }
    HIPCHK(hipMemcpy(d_idx, hidx.data(), (size_t)S * 4, hipMemcpyHostToDevice));
  } else {
    MK_LAUNCH(k_post_index, dim3((S + 255) / 256), dim3(256), 0, st, seed, S, NL, d_idx);
  }
  MK_LAUNCH(k_post_interp, dim3((unsigned)(((long)S * P + 255) / 256)), dim3(256), 0, st, d_res, L, (long)P,
                     d_idx, S, d_lo, d_hi, d_mode, d_t, d_spar);
  if (C > 0) {
    const unsigned nb = (unsigned)(((long)S * C + 255) / 256);
    MK_LAUNCH(k_post_interp, dim3(nb), dim3(256), 0, st, d_res2, L, (long)C, d_idx, S, d_lo, d_hi, d_mode, d_t,
                       d_sw);
    MK_LAUNCH(k_post_prob, dim3(nb), dim3(256), 0, st, d_spar, S, d_xt, (long)C, p, d_sw, link, d_p);
  }
  HIPCHK(hipGetLastError());
  if (o->index) HIPCHK(hipMemcpy(o->index, d_idx, (size_t)S * 4, hipMemcpyDeviceToHost));
  if (o->sample_par) HIPCHK(hipMemcpy(o->sample_par, d_spar, (size_t)S * P * 8, hipMemcpyDeviceToHost));
  if (C > 0 && o->sample_w) HIPCHK(hipMemcpy(o->sample_w, d_sw, (size_t)S * C * 8, hipMemcpyDeviceToHost));
  if (C > 0 && o->p_sample) HIPCHK(hipMemcpy(o->p_sample, d_p, (size_t)S * C * 8, hipMemcpyDeviceToHost));
  // type-7 (0.5, 0.025, 0.975) per column: each column is S contiguous rows -> 3 x ncol column-major
  auto quant = [&](const double* src, long ncol, double* dst) -> int {
    const int rq = launch_quantiles((unsigned)ncol, st, src, (long)S, 1L, S, 1, d_pr, 3, d_q);
    if (rq) return rq;
    HIPCHK(hipMemcpy(dst, d_q, (size_t)ncol * 3 * 8, hipMemcpyDeviceToHost));
    return 0;
  };
  int rc;
  if (o->param_quant && (rc = quant(d_spar, P, o->param_quant))) return rc;
  if (C > 0 && o->w_quant && (rc = quant(d_sw, C, o->w_quant))) return rc;
  if (C > 0 && o->p_quant && (rc = quant(d_p, C, o->p_quant))) return rc;
  return 0;
}

extern "C" int mk_posterior_summary(const double* result, int32_t P, const double* result2, int64_t C,
                                    const double* x_test, int32_t p, int32_t S, uint64_t seed, mk_summary* o,
                                    int32_t device) {
  return mk_posterior_summary_ex(result, P, result2, C, x_test, p, S, seed, nullptr, MK_LINK_LOGIT, o, device);
}

// ------------------------------------------------------------------ glm start values (MK.R:53-55)
// p x p symmetric positive definite solve / inverse through a host Cholesky (p <= 8).
static bool chol_small(const std::vector<double>& A, int p, std::vector<double>& Lc) {
  Lc.assign((size_t)p * p, 0.0);
  for (int j = 0; j < p; ++j) {
    double d = A[j + j * p];
    for (int k = 0; k < j; ++k) d -= Lc[j + k * p] * Lc[j + k * p];
    if (!(d > 0.0)) return false;
    d = std::sqrt(d);
    Lc[j + j * p] = d;
    for (int i = j + 1; i < p; ++i) {
      double v = A[i + j * p];
      for (int k = 0; k < j; ++k) v -= Lc[i + k * p] * Lc[j + k * p];
      Lc[i + j * p] = v / d;
    }
  }
  return true;
}
static void chol_solve_small(const std::vector<double>& Lc, int p, const double* b, double* x) {
  std::vector<double> y(p);
  for (int i = 0; i < p; ++i) {
    double v = b[i];
    for (int k = 0; k < i; ++k) v -= Lc[i + k * p] * y[k];
    y[i] = v / Lc[i + i * p];
  }
  for (int i = p - 1; i >= 0; --i) {
    double v = y[i];
    for (int k = i + 1; k < p; ++k) v -= Lc[k + i * p] * x[k];
    x[i] = v / Lc[i + i * p];
  }
}

extern "C" int mk_glm_binomial_link(const double* y, const double* weights, const double* x, int64_t n, int32_t p,
                                    int32_t link, double epsilon, int32_t maxit, double* coef, double* vcov,
                                    int32_t* iters, int32_t device) {
  if (!y || !weights || !x || !coef || n < 1 || p < 1 || p > 8 || maxit < 1)
    return set_err(MK_E_ARG, "bad glm arguments (n >= 1, 1 <= p <= 8, maxit >= 1)");
  if (link != MK_LINK_LOGIT && link != MK_LINK_PROBIT) return set_err(MK_E_ARG, "link must be logit or probit");
  MK_ENTRY_DEVICE(device);
  std::vector<double> yp((size_t)n);
  for (int64_t i = 0; i < n; ++i) yp[i] = y[i] / weights[i];     // glm((y/weight) ~ x - 1, ...)  MK.R:53
  const int ntri = p * (p + 1) / 2, NP = 1 + ntri + p;
  const int nblk = (int)std::min<int64_t>(1024, (n + 255) / 256);
  DevBufs b;
  double* d_y = b.get<double>((size_t)n);
  double* d_w = b.get<double>((size_t)n);
  double* d_x = b.get<double>((size_t)n * p);
  double* d_c = b.get<double>(p);
  double* d_part = b.get<double>((size_t)nblk * NP);
  if (!d_y || !d_w || !d_x || !d_c || !d_part) return set_err(MK_E_NOMEM, "glm alloc");
  HIPCHK(hipMemcpy(d_y, yp.data(), (size_t)n * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_w, weights, (size_t)n * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d_x, x, (size_t)n * p * 8, hipMemcpyHostToDevice));
  std::vector<double> part((size_t)nblk * NP), A((size_t)p * p), rhs(p), Lc, c(p, 0.0), A_used;
  double dev = 0.0;
  auto pass = [&](int mode) -> int {
    if (mode == 1) HIPCHK(hipMemcpy(d_c, c.data(), (size_t)p * 8, hipMemcpyHostToDevice));
    MK_LAUNCH(k_glm_pass, dim3(nblk), dim3(256), 0, 0, d_y, d_w, d_x, (long)n, p, d_c, mode, link, d_part);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(part.data(), d_part, part.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> tot(NP, 0.0);
    for (int bk = 0; bk < nblk; ++bk)
      for (int i = 0; i < NP; ++i) tot[i] += part[(size_t)bk * NP + i];
    dev = tot[0];
    int k = 1;
    for (int a = 0; a < p; ++a)
      for (int bb = a; bb < p; ++bb, ++k) A[a + bb * p] = A[bb + a * p] = tot[k];
    for (int a = 0; a < p; ++a) rhs[a] = tot[1 + ntri + a];
    return 0;
  };
  int rc = pass(0);
  if (rc) return rc;
  double devold = dev;
  int it = 0;
  for (it = 1; it <= maxit; ++it) {
    if (!chol_small(A, p, Lc)) return set_err(MK_E_ARG, "glm: singular weighted design");
    A_used = A;
    chol_solve_small(Lc, p, rhs.data(), c.data());
    if ((rc = pass(1))) return rc;
    if (std::fabs(dev - devold) / (std::fabs(dev) + 0.1) < epsilon) break;
    devold = dev;
  }
  if (it > maxit) it = maxit;
  for (int j = 0; j < p; ++j) coef[j] = c[j];
  if (vcov) {   // chol2inv of the final fit's weighted design = (X'WX)^-1 at the weights that produced coef
    if (!chol_small(A_used, p, Lc)) return set_err(MK_E_ARG, "glm: singular weighted design");
    std::vector<double> e(p), col(p);
    for (int j = 0; j < p; ++j) {
      std::fill(e.begin(), e.end(), 0.0);
      e[j] = 1.0;
      chol_solve_small(Lc, p, e.data(), col.data());
      for (int i = 0; i < p; ++i) vcov[i + j * p] = col[i];
    }
  }
  if (iters) *iters = it;
  return 0;
}

extern "C" int mk_glm_binomial(const double* y, const double* weights, const double* x, int64_t n, int32_t p,
                               double epsilon, int32_t maxit, double* coef, double* vcov, int32_t* iters,
                               int32_t device) {
  return mk_glm_binomial_link(y, weights, x, n, p, MK_LINK_LOGIT, epsilon, maxit, coef, vcov, iters, device);
}

// ------------------------------------------------------------------ parity-test entry points
extern "C" int mk_correlation_batched(const double* coords, int32_t S, int32_t n, const double* phi, const double* nu,
                                      int32_t cov_model, double* R_out, int32_t device) {
  if (!coords || !phi || !R_out || S < 1 || n < 1) return set_err(MK_E_ARG, "bad correlation arguments");
  if (cov_model != MK_COV_EXPONENTIAL && cov_model != MK_COV_MATERN) return set_err(MK_E_ARG, "bad cov_model");
  if (cov_model == MK_COV_MATERN && !nu) return set_err(MK_E_ARG, "matern needs nu");
  for (int s = 0; s < S; ++s)
    if (!(phi[s] > 0.0) || (nu && cov_model == MK_COV_MATERN && !(nu[s] > 0.0)))
      return set_err(MK_E_ARG, "phi and nu must be > 0");
  MK_ENTRY_DEVICE(device);
  // The sampler's own candidate kernel (k_cov_candidate, which = 2: the current theta) on a
  // one-outcome model per point set: theta = 0 with Unif(0, 2 phi) / Unif(0, 2 nu) supports gives
  // exactly phi and nu (logitInv(0, 0, b) = b - b/2).  The border row is u = 0.
  const int n_pad = round_up(n + 1, MK_NB), nt = n_pad / MK_NB;
  const bool matern = cov_model == MK_COV_MATERN;
  const int n_theta = matern ? 3 : 2;
  DevBufs b;
  double* dc = b.get<double>((size_t)S * 2 * n_pad);
  double* dth = b.get<double>((size_t)S * n_theta);
  double* du = b.get<double>((size_t)S * n_pad);
  int* dns = b.get<int>(S);
  int* dcur = b.get<int>(S);
  double* dL = b.get<double>((size_t)S * 2 * n_pad * n_pad);
  double* dr = b.get<double>((size_t)S * n * n);
  if (!dc || !dth || !du || !dns || !dcur || !dL || !dr) return set_err(MK_E_NOMEM, "correlation alloc");
  std::vector<double> hc((size_t)S * 2 * n_pad, 0.0);
  for (int s = 0; s < S; ++s)
    for (int r = 0; r < n; ++r) {
      hc[(size_t)s * 2 * n_pad + r] = coords[(size_t)s * 2 * n + r];
      hc[(size_t)s * 2 * n_pad + n_pad + r] = coords[(size_t)s * 2 * n + n + r];
    }
  std::vector<int> hn(S, n);
  HIPCHK(hipMemcpy(dc, hc.data(), hc.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dns, hn.data(), (size_t)S * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(dth, 0, (size_t)S * n_theta * 8));
  HIPCHK(hipMemset(du, 0, (size_t)S * n_pad * 8));
  HIPCHK(hipMemset(dcur, 0, (size_t)S * 4));
  MatSet ms{};
  ms.L = dL; ms.cur = dcur; ms.ld = n_pad; ms.nt = nt; ms.q = 1;
  const int ntri_tiles = nt * (nt + 1) / 2;
  for (int s = 0; s < S; ++s) {
    Model md{};
    md.S = 1; md.q = 1; md.p = 0; md.n_pad = n_pad; md.Np = n_pad; md.nt = nt; md.ntri = 1; md.n_theta = n_theta;
    md.cov_model = cov_model;
    md.o_A = 0; md.o_phi = 1; md.o_nu = 2; md.o_w = n_theta; md.n_mh_max = n_theta;
    md.phi_a[0] = 0.0; md.phi_b[0] = 2.0 * phi[s];
    md.nu_a[0] = 0.0; md.nu_b[0] = matern ? 2.0 * nu[s] : 1.0;
    md.n_s = dns + s;
    md.coords = dc + (size_t)s * 2 * n_pad;
    md.theta = dth + (size_t)s * n_theta;
    md.u = du + (size_t)s * n_pad;
    MatSet mv = ms;
    mv.L = dL + (size_t)s * 2 * n_pad * n_pad;
    mv.cur = dcur + s;
    MK_LAUNCH(cov_candidate_kernel(cov_model), dim3(xcd_grid_h(1, ntri_tiles)), dim3(256), 0, 0, md, mv, 0, 1,
                       2, 0, nullptr, nullptr);
  }
  MK_LAUNCH(k_extract_candidate, dim3(2048), dim3(256), 0, 0, ms, n, S, dr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(R_out, dr, (size_t)S * n * n * 8, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int mk_cholesky_batched(const double* A, int32_t S, int32_t n, double* L_out, double* logdet_out,
                                   double* inv_out, int32_t device) {
  if (!A || S < 1 || n < 1) return set_err(MK_E_ARG, "bad cholesky arguments");
  MK_ENTRY_DEVICE(device);
  mk_session* s = new mk_session();
  s->device = device;
  auto fail = [&](int code) { delete s; return code; };
  if (pool_stream(s->owned, &s->stream, device, SK_PLAIN) != hipSuccess) return fail(set_err(MK_E_HIP, "stream"));
  const int n_pad = round_up(n + 1, MK_NB), nt = n_pad / MK_NB;
  s->S = S; s->q = 1; s->n_pad = n_pad; s->nt = nt;
  s->n_part.assign(S, n);
  Model& md = s->md;
  md.S = S; md.q = 1; md.nt = nt; md.n_pad = n_pad;
  MatSet& ms = s->ms;
  ms.ld = n_pad; ms.nt = nt; ms.q = 1;
  int rc;
  int* d_ns;
  double* dA;
  if ((rc = s->alloc(&d_ns, S)) || (rc = s->alloc(&md.ld_part, (size_t)S * nt)) || (rc = s->alloc(&md.quad_c, S)) ||
      (rc = s->alloc(&md.info, S)) || (rc = s->alloc(&md.dirty, S)) || (rc = s->alloc(&ms.cur, S)) ||
      (rc = s->alloc(&md.logdetR, S)) || (rc = s->alloc(&md.quad, S)) ||
      (rc = s->alloc(&ms.L, (size_t)S * 2 * n_pad * n_pad)) || (rc = s->alloc(&ms.Winv, (size_t)S * 2 * nt * MK_NB * MK_NB)) ||
      (rc = s->alloc(&ms.Q, (size_t)S * n_pad * n_pad)) || (rc = s->alloc(&ms.W, (size_t)S * n_pad * n_pad)) ||
      (rc = s->alloc(&dA, (size_t)S * n * n)))
    return fail(rc);
  md.n_s = d_ns;
  if ((rc = setup_groups(s, 1))) return fail(rc);
  Group& a = s->all;
  std::vector<int> hn(S, n);
  if (hipMemcpy(d_ns, hn.data(), S * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dA, A, (size_t)S * n * n * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(ms.cur, 0, S * 4) != hipSuccess || hipMemset(md.info, 0, S * 4) != hipSuccess ||
      hipMemset(ms.Winv, 0, (size_t)S * 2 * nt * MK_NB * MK_NB * 8) != hipSuccess)
    return fail(set_err(MK_E_HIP, "cholesky upload"));
  if (hipFuncSetAttribute((const void*)k_chol_diag, hipFuncAttributeMaxDynamicSharedMemorySize,
                          MK_DIAG_LDS_BYTES) != hipSuccess || !set_gemm_lds())
    return fail(set_err(MK_E_HIP, "lds attribute"));
  MK_LAUNCH(k_load_plain, dim3(2048), dim3(256), 0, s->stream, ms, dA, n, S);
  launch_cholesky(s, a, 0, 1);
  std::vector<double> part((size_t)S * nt);
  std::vector<int> info(S);
  if (hipStreamSynchronize(s->stream) != hipSuccess) return fail(set_err(MK_E_HIP, "cholesky run"));
  if (hipMemcpy(info.data(), md.info, S * 4, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(set_err(MK_E_HIP, "info download"));
  for (int i = 0; i < S; ++i)
    if (info[i]) return fail(set_err(MK_E_ARG, "matrix " + std::to_string(i) + " is not positive definite"));
  MK_LAUNCH(k_theta_init, dim3((S + 63) / 64), dim3(64), 0, s->stream, md, ms, 0, 1);
  double* dL = nullptr;
  if ((rc = s->alloc(&dL, (size_t)S * n * n))) return fail(rc);
  if (L_out) {
    MK_LAUNCH(k_extract_L, dim3(2048), dim3(256), 0, s->stream, ms, n, S, dL, 0);
    if (hipMemcpyAsync(L_out, dL, (size_t)S * n * n * 8, hipMemcpyDeviceToHost, s->stream) != hipSuccess)
      return fail(set_err(MK_E_HIP, "L download"));
  }
  if (logdet_out) {
    if (hipMemcpy(part.data(), md.ld_part, part.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
      return fail(set_err(MK_E_HIP, "logdet download"));
    for (int i = 0; i < S; ++i) {
      double v = 0.0;
      for (int k = 0; k < nt; ++k) v += part[(size_t)i * nt + k];
      logdet_out[i] = v;
    }
  }
  if (inv_out) {
    MK_LAUNCH(k_dirty_list, dim3(1), dim3(256), 0, s->stream, md, 1, a.d_plist, a.d_pcount, a.d_list,
                       a.d_count);
    const int ntiles = nt * (nt + 1) / 2;
    launch_trinv(s, a, S, a.d_list, a.d_count);
    MK_LAUNCH(k_lauum, dim3(S * ntiles), dim3(256), LDS_128, s->stream, ms, md.n_s, a.d_list, a.d_count);
    MK_LAUNCH(k_extract_L, dim3(2048), dim3(256), 0, s->stream, ms, n, S, dL, 1);
    if (hipMemcpyAsync(inv_out, dL, (size_t)S * n * n * 8, hipMemcpyDeviceToHost, s->stream) != hipSuccess)
      return fail(set_err(MK_E_HIP, "inverse download"));
  }
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess) return fail(set_err(MK_E_HIP, std::string("cholesky: ") + hipGetErrorString(e)));
  delete s;
  return 0;
}

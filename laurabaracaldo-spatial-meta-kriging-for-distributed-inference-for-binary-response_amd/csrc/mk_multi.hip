// mk_meta_fit: the whole node in one call (include/mk.h) -- the subsets sharded over the GPUs of
// one host, one host thread per shard, and the combine device to device.
//
// Replaces MK.R:100-114 (makeCluster(n.core) + foreach(i = 1:n.core) %dopar% partitioned_spMvGLM)
// and the combine loop MK.R:119-133.  The fits exchange nothing: shard r is the
// balanced contiguous block [floor(rK/G), floor((r+1)K/G)) of subsets with its global subset
// indices, so its chains are the one-device chains.  The one exchange is the combine:
//
//   grids_r [S_r][C][200]  (HBM of device r; C = P parameter columns, or q*n_test kriging columns,
//                           or q*tile per test-site tile)
//   pack    send_r [G][S_r][per][200]  (column block j of each of its subsets; per = ceil(C/G))
//   all-to-all: recv_j [K][per][200] <- send_r block j, at subset offset lo_r (global order)
//   combine on device j: k_combine (sequential mean / sum over k = 0..K-1) or k_weiszfeld
//   columns [a_j, a_j + c_j) of the combined grid -> host
//
// The all-to-all is RCCL send/recv in one group (xGMI) when the devices are distinct, and device
// copies (hipMemcpyPeerAsync; same-device copies) when a device appears more than once -- RCCL
// refuses two ranks on one GPU.  RCCL is loaded at run time (dlopen), so libmk has no link-time
// dependency on it and a host that already loaded one (torch) shares it.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <algorithm>
#include <cstdio>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>
#include "../../include/mk.h"
#include "mk_internal.hpp"
#include "mk_kernels.hpp"

using namespace mk;

namespace {

int fail(int code, const std::string& msg) { return host_error(code, msg.c_str()); }

#define MHIP(x)                                                                                     \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return fail(MK_E_HIP, std::string(#x " -> ") + hipGetErrorString(e_));    \
  } while (0)

// ------------------------------------------------------------------ RCCL, resolved at run time
struct Rccl {
  bool ok = false;
  std::string why;
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  const char* (*last_error)(ncclComm_t) = nullptr;   // optional: RCCL's last WARN text
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;   // optional: ranks a communicator holds
};

// RCCL must run on the HIP runtime libmk runs on.  A process can hold two: a host that loads torch
// after libmk (torch's CPU ops, e.g. the synthetic generator) maps torch's bundled libamdhip64 and
// librccl beside the system's, and a dlopen("librccl.so.1") by soname then returns torch's RCCL,
// bound to the second runtime -- which reported "no ROCm-capable device is detected" from
// ncclCommInitAll (the round-3 "unhandled cuda error", reproduced in round 4 by the GPU suite).  So
// the library is opened by path from the directory of the libamdhip64 libmk is bound to (dladdr).
std::string hip_runtime_dir() {
  Dl_info info{};
  if (dladdr((const void*)&hipGetDeviceCount, &info) && info.dli_fname) {
    std::string f = info.dli_fname;
    const size_t slash = f.rfind('/');
    if (slash != std::string::npos) return f.substr(0, slash);
  }
  return "";
}

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    const std::string dir = hip_runtime_dir();
    void* h = nullptr;
    std::string tried;
    for (const char* name : {"librccl.so.1", "librccl.so"}) {
      if (h || dir.empty()) break;
      const std::string path = dir + "/" + name;
      tried += path + " ";
      h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    }
    if (!h && dir.empty()) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);   // no path known: by soname
    if (!h) {
      const char* e = dlerror();
      x.why = std::string("librccl not loadable beside libmk's HIP runtime (") + tried + "): " + (e ? e : "?");
      return x;
    }
    x.comm_init_all = (decltype(x.comm_init_all))dlsym(h, "ncclCommInitAll");
    x.comm_destroy = (decltype(x.comm_destroy))dlsym(h, "ncclCommDestroy");
    x.comm_abort = (decltype(x.comm_abort))dlsym(h, "ncclCommAbort");
    x.last_error = (decltype(x.last_error))dlsym(h, "ncclGetLastError");
    x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
    x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
    x.send = (decltype(x.send))dlsym(h, "ncclSend");
    x.recv = (decltype(x.recv))dlsym(h, "ncclRecv");
    x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
    x.comm_count = (decltype(x.comm_count))dlsym(h, "ncclCommCount");
    x.ok = x.comm_init_all && x.comm_destroy && x.comm_abort && x.group_start && x.group_end && x.send && x.recv && x.error_string;
    if (!x.ok) x.why = "librccl lacks a symbol";
    return x;
  }();
  return r;
}

#define MNCCL(x)                                                                                    \
  do {                                                                                              \
    ncclResult_t e_ = (x);                                                                          \
    if (e_ != ncclSuccess) return fail(MK_E_HIP, std::string(#x " -> ") + rccl().error_string(e_)); \
  } while (0)

// One persistent host thread per device block for the whole call (HIP's per-thread state stays
// warm: a fresh thread per amcmc batch measured 2-4x slower chains on small shards, whose
// iterations are bound by the host's launch rate).  run(f) executes f(r) on worker r for every r
// and returns the first failure with its message (the library's error text is thread-local: it
// is carried back to the calling thread).
class Pool {
 public:
  explicit Pool(int n) : n_(n), rc_(n, 0), msg_(n) {
    for (int r = 0; r < n; ++r) th_.emplace_back([this, r] { loop(r); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int run(const std::function<int(int)>& f) {
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = &f;
      pending_ = n_;
      ++gen_;
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return pending_ == 0; });
    for (int r = 0; r < n_; ++r)
      if (rc_[r]) return fail(rc_[r], "device block " + std::to_string(r) + ": " + msg_[r]);
    return 0;
  }

 private:
  void loop(int r) {
    long seen = 0;
    for (;;) {
      const std::function<int(int)>* job;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        job = job_;
      }
      const int rc = (*job)(r);
      std::string msg = rc ? mk_last_error() : "";
      std::lock_guard<std::mutex> lk(m_);
      rc_[r] = rc;
      msg_[r] = std::move(msg);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  int n_;
  std::vector<int> rc_;
  std::vector<std::string> msg_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<int(int)>* job_ = nullptr;
  long gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

// Device buffer that grows on demand (freed on its device).
struct DBuf {
  int dev = 0;
  double* p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return 0;
    MHIP(hipSetDevice(dev));
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(double)) != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      return fail(MK_E_NOMEM, "combine buffer of " + std::to_string(n * 8) + " B");
    }
    cap = n;
    return 0;
  }
  ~DBuf() {
    if (p) {
      (void)hipSetDevice(dev);
      (void)hipFree(p);
    }
  }
};

// One device block: its session and its share of the exchange.
struct Block {
  int dev = 0, lo = 0, S = 0;
  mk_session* ses = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t packed = nullptr;
  DBuf grids, send, recv, comb, sum, iters;   // iters: Weiszfeld iteration counts (as int)
  ~Block() {
    (void)hipSetDevice(dev);
    if (st) (void)hipStreamSynchronize(st);
    if (ses) mk_session_destroy(ses);
    if (packed) (void)hipEventDestroy(packed);
    if (st) stream_release(dev, st);   // drained above
  }
};

// Teardown order: every block's stream is drained before the communicators go (a send/recv still
// queued on a stream must not outlive its communicator); after a failed exchange the communicators
// are aborted instead of destroyed, since a recv whose matching send was never issued would never
// complete and a drain would wait on it forever.  Then the blocks (sessions, buffers), then the
// host threads.
struct Node {
  std::unique_ptr<Pool> pool;   // first member: its threads are joined after the blocks are freed
  int G = 0, K = 0;
  std::vector<std::unique_ptr<Block>> b;
  bool use_rccl = false;
  bool exchange_failed = false;
  std::vector<ncclComm_t> comms;
  ~Node() {
    if (exchange_failed) {
      for (ncclComm_t c : comms)
        if (c) rccl().comm_abort(c);
      comms.clear();
    }
    for (auto& x : b)
      if (x && x->st) {
        (void)hipSetDevice(x->dev);
        (void)hipStreamSynchronize(x->st);
      }
    for (ncclComm_t c : comms)
      if (c) rccl().comm_destroy(c);
    comms.clear();
  }
};

std::string rccl_detail(ncclResult_t e) {
  std::string m = rccl().error_string(e);
  if (rccl().last_error) {
    const char* d = rccl().last_error(nullptr);
    if (d && *d) m += std::string(" [") + d + "]";
  }
  return m;
}

constexpr int L = MK_N_LEVELS;

// The exchange + combine of one grid set: every block's grids [S_r][C][200] are in b.grids.
// Writes (when not NULL) the combined columns: mean (or median) -> h_comb, sum -> h_sum, both
// 200 x C column-major with column c at c*200.
int exchange_combine(Node& nd, long C, const mk_combined* comb, double* h_comb, double* h_sum) {
  if (!h_comb && !h_sum) return 0;
  const int G = nd.G, K = nd.K;
  const long per = std::max(1L, (C + G - 1) / G);
  auto col0 = [&](int j) { return std::min(C, (long)j * per); };
  auto ncol = [&](int j) { return std::min(C, (long)(j + 1) * per) - col0(j); };
  const bool median = comb && comb->method == MK_COMBINE_MEDIAN;
  // pack: column block j of every subset of block r
  int rc = nd.pool->run([&](int r) -> int {
    Block& x = *nd.b[r];
    MHIP(hipSetDevice(x.dev));
    int e;
    if ((e = x.send.ensure((size_t)G * x.S * per * L)) || (e = x.recv.ensure((size_t)K * per * L)) ||
        (e = x.comb.ensure((size_t)per * L)) || (e = x.sum.ensure((size_t)per * L)) || (e = x.iters.ensure((size_t)per)))
      return e;
    MHIP(hipMemsetAsync(x.recv.p, 0, (size_t)K * per * L * 8, x.st));
    if (x.S > 0) {
      MHIP(hipMemsetAsync(x.send.p, 0, (size_t)G * x.S * per * L * 8, x.st));
      for (int j = 0; j < G; ++j)
        if (ncol(j) > 0)
          MHIP(hipMemcpy2DAsync(x.send.p + (size_t)j * x.S * per * L, (size_t)per * L * 8, x.grids.p + col0(j) * L,
                                (size_t)C * L * 8, (size_t)ncol(j) * L * 8, x.S, hipMemcpyDeviceToDevice, x.st));
    }
    MHIP(hipEventRecord(x.packed, x.st));
    return 0;
  });
  if (rc) return rc;
  // all-to-all: recv_j[lo_r ..] <- send_r[j]
  if (nd.use_rccl) {
    const Rccl& R = rccl();
    MNCCL(R.group_start());
    ncclResult_t first = ncclSuccess;
    for (int r = 0; r < G; ++r)
      for (int j = 0; j < G; ++j) {
        Block &xr = *nd.b[r], &xj = *nd.b[j];
        if (xr.S == 0 || ncol(j) == 0) continue;
        const size_t cnt = (size_t)xr.S * per * L;
        ncclResult_t e1 = R.send(xr.send.p + (size_t)j * xr.S * per * L, cnt, ncclFloat64, j, nd.comms[r], xr.st);
        ncclResult_t e2 = R.recv(xj.recv.p + (size_t)xr.lo * per * L, cnt, ncclFloat64, r, nd.comms[j], xj.st);
        if (first == ncclSuccess) first = e1 != ncclSuccess ? e1 : e2;
      }
    const ncclResult_t eg = R.group_end();
    if (first != ncclSuccess || eg != ncclSuccess) nd.exchange_failed = true;
    if (first != ncclSuccess) return fail(MK_E_HIP, std::string("ncclSend/ncclRecv -> ") + rccl_detail(first));
    if (eg != ncclSuccess) return fail(MK_E_HIP, std::string("ncclGroupEnd -> ") + rccl_detail(eg));
  } else {
    for (int j = 0; j < G; ++j) {
      Block& xj = *nd.b[j];
      if (ncol(j) == 0) continue;
      MHIP(hipSetDevice(xj.dev));
      for (int r = 0; r < G; ++r) {
        Block& xr = *nd.b[r];
        if (xr.S == 0) continue;
        MHIP(hipStreamWaitEvent(xj.st, xr.packed, 0));
        const size_t bytes = (size_t)xr.S * per * L * 8;
        const double* src = xr.send.p + (size_t)j * xr.S * per * L;
        double* dst = xj.recv.p + (size_t)xr.lo * per * L;
        if (xr.dev == xj.dev)
          MHIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, xj.st));
        else
          MHIP(hipMemcpyPeerAsync(dst, xj.dev, src, xr.dev, bytes, xj.st));
      }
    }
  }
  // combine on the owner of each column block, in global subset order; columns to the host
  return nd.pool->run([&](int j) -> int {
    Block& x = *nd.b[j];
    MHIP(hipSetDevice(x.dev));
    const long a = col0(j), cj = ncol(j);
    if (cj > 0) {
      const long g = per * L;
      const unsigned nb = (unsigned)((g + 255) / 256);
      if (h_comb) {
        if (median) {
          const int it = comb->max_iter > 0 ? comb->max_iter : 100;
          const double tol = comb->tol >= 0.0 ? comb->tol : 1e-12;
          MK_LAUNCH(k_weiszfeld, dim3((unsigned)((per + 3) / 4)), dim3(256), 0, x.st, x.recv.p, K, L, per, it,
                             tol, x.comb.p, (int*)x.iters.p);
        } else {
          MK_LAUNCH(k_combine, dim3(nb), dim3(256), 0, x.st, x.recv.p, K, g, x.comb.p, 1);
        }
        MHIP(hipGetLastError());
        MHIP(hipMemcpyAsync(h_comb + a * L, x.comb.p, (size_t)cj * L * 8, hipMemcpyDeviceToHost, x.st));
      }
      if (h_sum) {
        MK_LAUNCH(k_combine, dim3(nb), dim3(256), 0, x.st, x.recv.p, K, g, x.sum.p, 0);
        MHIP(hipGetLastError());
        MHIP(hipMemcpyAsync(h_sum + a * L, x.sum.p, (size_t)cj * L * 8, hipMemcpyDeviceToHost, x.st));
      }
    }
    MHIP(hipStreamSynchronize(x.st));
    return 0;
  });
}

}  // namespace

extern "C" int mk_meta_fit(const mk_problem* pr, const mk_config* c, const int32_t* devices, int32_t G,
                           mk_progress_fn progress, void* user, mk_outputs* out, mk_combined* comb) {
  if (!pr || !c) return fail(MK_E_ARG, "null problem/config");
  if (!devices || G < 1) return fail(MK_E_ARG, "n_devices must be >= 1 with a device list");
  const int K = pr->n_subsets;
  if (K < 1) return fail(MK_E_ARG, "n_subsets must be >= 1");
  if (pr->q < 1 || pr->q > 4 || pr->p < 1 || !pr->n_part) return fail(MK_E_ARG, "bad q / p / n_part");
  if (comb && comb->method != MK_COMBINE_MEAN && comb->method != MK_COMBINE_MEDIAN)
    return fail(MK_E_ARG, "combine method must be MK_COMBINE_MEAN or MK_COMBINE_MEDIAN");
  ApiCall call(__func__);
  DeviceGuard dg;   // the caller's current device is restored on every return path
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MK_E_NODEV, "no HIP device");
  for (int r = 0; r < G; ++r)
    if (devices[r] < 0 || devices[r] >= ndev) return fail(MK_E_ARG, "bad device ordinal in the device list");
  for (int i = 0; i < K; ++i)
    if (pr->n_part[i] < 1) return fail(MK_E_ARG, "every subset needs >= 1 site");
  const int q = pr->q, p = pr->p, n_samples = c->n_batch * c->batch_length;
  if (c->n_batch < 1 || c->batch_length < 1) return fail(MK_E_ARG, "n.batch and batch.length must be >= 1");

  Node nd;
  nd.G = G;
  nd.K = K;
  nd.pool = std::make_unique<Pool>(G);
  bool distinct = true;
  for (int r = 0; r < G; ++r)
    for (int j = 0; j < r; ++j) distinct = distinct && devices[r] != devices[j];
  const char* xenv = std::getenv("MK_EXCHANGE");   // "copy": device copies even on distinct devices (opt-in)
  nd.use_rccl = distinct && !(xenv && std::strcmp(xenv, "copy") == 0);
  if (nd.use_rccl && !rccl().ok) return fail(MK_E_HIP, rccl().why);

  // ---- blocks: balanced contiguous subset ranges, data pointers offset into the caller's arrays
  std::vector<long> site0(K + 1, 0);
  for (int i = 0; i < K; ++i) site0[i + 1] = site0[i] + pr->n_part[i];
  for (int r = 0; r < G; ++r) {
    auto x = std::make_unique<Block>();
    x->dev = devices[r];
    x->lo = (int)(((long)r * K) / G);
    x->S = (int)(((long)(r + 1) * K) / G) - x->lo;
    x->grids.dev = x->send.dev = x->recv.dev = x->comb.dev = x->sum.dev = x->iters.dev = x->dev;
    nd.b.push_back(std::move(x));
  }
  int rc = nd.pool->run([&](int r) -> int {
    Block& x = *nd.b[r];
    MHIP(hipSetDevice(x.dev));
    MHIP(stream_acquire(x.dev, &x.st));
    MHIP(hipEventCreateWithFlags(&x.packed, hipEventDisableTiming));
    if (x.S == 0) return 0;
    mk_problem sp = *pr;
    const long s0 = site0[x.lo];
    sp.n_subsets = x.S;
    sp.subset_base = pr->subset_base + x.lo;
    sp.n_part = pr->n_part + x.lo;
    sp.coords = pr->coords + 2 * s0;
    sp.y = pr->y + s0 * q;
    sp.weights = pr->weights + s0 * q;
    sp.x = pr->x + s0 * q * p;
    mk_config sc = *c;
    sc.device = x.dev;
    return mk_session_create(&sp, &sc, &x.ses);
  });
  if (rc) return rc;
  if (nd.use_rccl) {
    // A communicator that cannot be created is an error (MK_E_HIP), never a silent switch to the
    // device-copy exchange (MK_EXCHANGE=copy asks for that explicitly).  The message carries RCCL's
    // own last warning and any HIP error this thread held before the call (RCCL reports a pending
    // one as "unhandled cuda error"; seen once in a long round-3 test process), so a repeat names
    // the failing call.
    const hipError_t pending = hipGetLastError();
    nd.comms.assign(G, nullptr);
    const ncclResult_t e = rccl().comm_init_all(nd.comms.data(), G, devices);
    if (e != ncclSuccess) {
      nd.comms.clear();
      const hipError_t after = hipGetLastError();
      return fail(MK_E_HIP, std::string("ncclCommInitAll -> ") + rccl_detail(e) + "; HIP error pending before: " +
                                hipGetErrorName(pending) + ", after: " + hipGetErrorName(after) +
                                " (MK_EXCHANGE=copy selects the device-copy exchange)");
    }
  }
  if (comb) {
    comb->exchange = nd.use_rccl ? 1 : 0;
    // the ranks the exchange spans, as RCCL itself counts them (communicator 0); copies: the blocks
    int nr = G;
    if (nd.use_rccl && rccl().comm_count && rccl().comm_count(nd.comms[0], &nr) != ncclSuccess) nr = -1;
    comb->comm_ranks = nr;
  }

  // ---- the chains, one amcmc batch at a time on every device; progress between batches
  for (int it = 0; it < n_samples; it += c->batch_length) {
    rc = nd.pool->run([&](int r) -> int {
      Block& x = *nd.b[r];
      return x.ses ? mk_session_run(x.ses, c->batch_length) : 0;
    });
    if (rc) return rc;
    if (progress && progress(user, it + c->batch_length, n_samples))
      return fail(MK_E_INTERRUPT, "interrupted after " + std::to_string(it + c->batch_length) + " of " +
                                      std::to_string(n_samples) + " iterations");
  }

  // ---- per-subset outputs other than the grids (samples, w, draws, acceptance): each block
  // writes its subsets' slice of the caller's arrays
  ShardInfo info0{};
  for (auto& x : nd.b)
    if (x->ses) {
      session_info(x->ses, &info0);
      break;
    }
  const int P = info0.P, n_test = info0.n_test, n_kept = info0.n_kept;
  const long C = (long)q * n_test;
  const int n_theta = P - p;
  const bool tiled = info0.tiled != 0;
  auto shard_out = [&](const Block& x) {
    mk_outputs o{};
    if (!out) return o;
    const long s0 = site0[x.lo];
    if (out->samples) o.samples = out->samples + (size_t)x.lo * n_samples * P;
    if (out->w_samples) o.w_samples = out->w_samples + (size_t)s0 * q * n_samples;
    if (out->w_pred_samples) o.w_pred_samples = out->w_pred_samples + (size_t)x.lo * C * n_kept;
    if (out->acceptance) o.acceptance = out->acceptance + (size_t)x.lo * c->n_batch * (p + n_theta + 1);
    return o;
  };
  rc = nd.pool->run([&](int r) -> int {
    Block& x = *nd.b[r];
    if (!x.ses) return 0;
    mk_outputs o = shard_out(x);
    if (tiled) o.w_pred_samples = nullptr;   // written per tile below
    if (!o.samples && !o.w_samples && !o.w_pred_samples && !o.acceptance) return 0;
    return mk_session_outputs(x.ses, &o);
  });
  if (rc) return rc;

  // ---- parameter grids (MK.R:89) -> out->parameters, combine -> comb->result (MK.R:127)
  const bool want_par = (out && out->parameters) || (comb && comb->result);
  if (want_par) {
    rc = nd.pool->run([&](int r) -> int {
      Block& x = *nd.b[r];
      if (!x.ses) return 0;
      int e = x.grids.ensure((size_t)x.S * P * L);
      if (e || (e = session_param_grids(x.ses, x.grids.p))) return e;
      if (out && out->parameters)
        MHIP(hipMemcpy(out->parameters + (size_t)x.lo * P * L, x.grids.p, (size_t)x.S * P * L * 8, hipMemcpyDeviceToHost));
      return 0;
    });
    if (rc) return rc;
    if (comb && comb->result && (rc = exchange_combine(nd, P, comb, comb->result, nullptr))) return rc;
  }

  // ---- w.predict grids (MK.R:87-89) -> out->w_predict; combine -> comb->result2 (MK.R:133) and
  // the sequential sum -> out->w_predict_sum
  if (n_test > 0) {
    double* h_w = out ? out->w_predict : nullptr;
    double* h_sum = out ? out->w_predict_sum : nullptr;
    double* h_comb = comb ? comb->result2 : nullptr;
    const bool want_w = h_w || h_sum || h_comb || (tiled && out && out->w_pred_samples);
    if (want_w && !tiled) {
      rc = nd.pool->run([&](int r) -> int {
        Block& x = *nd.b[r];
        if (!x.ses) return 0;
        int e = x.grids.ensure((size_t)x.S * C * L);
        if (e || (e = session_wpred_grids(x.ses, x.grids.p))) return e;
        if (h_w) MHIP(hipMemcpy(h_w + (size_t)x.lo * C * L, x.grids.p, (size_t)x.S * C * L * 8, hipMemcpyDeviceToHost));
        return 0;
      });
      if (rc) return rc;
      if ((rc = exchange_combine(nd, C, comb, h_comb, h_sum))) return rc;
    } else if (want_w) {
      const int T = info0.pred_tile;
      // every shard replays the same tiles (the exchange combines tile by tile): a shard whose HBM
      // made it take a smaller kriging tile than the others (mk_session_predict_tile) cannot follow
      for (auto& x : nd.b)
        if (x->ses) {
          ShardInfo in{};
          session_info(x->ses, &in);
          if (in.pred_tile != T)
            return fail(MK_E_NOMEM, "the shards took different kriging tiles (" + std::to_string(T) + " and " +
                                           std::to_string(in.pred_tile) +
                                           " test sites: HBM limits differ); pass predict_tile <= the smaller");
        }
      for (int t0 = 0; t0 < n_test; t0 += T) {
        const long Ct = (long)q * std::min(T, n_test - t0);
        rc = nd.pool->run([&](int r) -> int {
          Block& x = *nd.b[r];
          if (!x.ses) return 0;
          mk_outputs o = shard_out(x);
          int e = x.grids.ensure((size_t)x.S * Ct * L);
          if (e || (e = session_tile_grids(x.ses, t0, x.grids.p, &o))) return e;
          if (h_w)   // per subset [C][200]: this tile's columns
            MHIP(hipMemcpy2D(h_w + (size_t)x.lo * C * L + (size_t)t0 * q * L, (size_t)C * L * 8, x.grids.p,
                             (size_t)Ct * L * 8, (size_t)Ct * L * 8, x.S, hipMemcpyDeviceToHost));
          return 0;
        });
        if (rc) return rc;
        if ((rc = exchange_combine(nd, Ct, comb, h_comb ? h_comb + (size_t)t0 * q * L : nullptr,
                                   h_sum ? h_sum + (size_t)t0 * q * L : nullptr)))
          return rc;
      }
    }
  }
  return 0;
}

// Stall watchdog (MK_WATCHDOG=<seconds>, or mk_set_watchdog): names the kernel a stuck stream is on.
//
// When enabled, every launch of the library is followed on its stream by a one-thread kernel that
// stores the launch's sequence number into a word of host-pinned memory (vector store, system
// scope), and the host keeps the launched kernels' names per stream in a ring.  Every C-ABI entry
// that can wait on the device registers itself (ApiCall).  A host thread checks once a second; when
// an entry has been running for longer than the limit it prints, once per entry, every stream with
// work outstanding: launches completed / enqueued, the last kernel that completed and the one the
// stream is on (or queued behind).  The report goes to stderr and, with MK_WATCHDOG_LOG=<path>, is
// appended to that file (a test runner that captures stderr still leaves it on disk).
//
// Off by default (the bench and the R package run without it): with it on, every launch costs a
// second dispatch.  The device-side waits that exist (the multi-workgroup sweep, after its admission
// consensus) have their own bounded spins and error flag (mk_mcmc.hip); this names the launch when a
// stream stops moving.
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include "../../include/mk.h"
#include "mk_internal.hpp"

namespace mk {

__global__ void k_progress(unsigned* word, unsigned seq) {
  if (threadIdx.x == 0) __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

namespace {

constexpr int RING = 256;
constexpr int MAX_STREAMS = 512;

struct Traced {
  hipStream_t st = nullptr;
  int device = -1;
  unsigned enq = 0;                 // launches enqueued (the last one's sequence number)
  unsigned slot = 0;                // index of its progress word
  const char* names[RING] = {};
};

struct Call {
  long id;
  const char* name;
  std::chrono::steady_clock::time_point t0;
  bool reported;
};

std::atomic<int> g_limit{-2};       // seconds; -2: not read from the environment yet, 0: off
std::mutex g_mu;
std::vector<Traced> g_streams;
std::vector<Call> g_calls;
unsigned* g_words = nullptr;        // [MAX_STREAMS] host-pinned progress words
unsigned* g_words_dev = nullptr;
long g_next_call = 0;
std::thread* g_thread = nullptr;

int limit() {
  int v = g_limit.load();
  if (v == -2) {
    const char* e = std::getenv("MK_WATCHDOG");
    const int x = (e && *e) ? std::atoi(e) : 0;
    int expect = -2;
    g_limit.compare_exchange_strong(expect, x > 0 ? x : 0);
    v = g_limit.load();
  }
  return v;
}

void emit(const std::string& text) {
  std::fputs(text.c_str(), stderr);
  std::fflush(stderr);
  const char* path = std::getenv("MK_WATCHDOG_LOG");
  if (path && *path) {
    if (FILE* f = std::fopen(path, "a")) {
      std::fputs(text.c_str(), f);
      std::fclose(f);
    }
  }
}

// Caller holds g_mu.
std::string report(const Call& c, double secs) {
  char line[512];
  std::snprintf(line, sizeof line, "libmk watchdog: %s (call %ld) still running after %.0f s\n", c.name, c.id, secs);
  std::string out = line;
  int pending = 0;
  for (const Traced& t : g_streams) {
    if (!t.st) continue;   // a free slot
    const unsigned done = __atomic_load_n(g_words + t.slot, __ATOMIC_ACQUIRE);
    if (done == t.enq) continue;
    ++pending;
    const char* last = done ? t.names[done % RING] : "(none)";
    const char* next = t.names[(done + 1) % RING];
    std::snprintf(line, sizeof line,
                  "  device %d stream %p: %u of %u launches done; last done %s; running or next: %s (launch %u)\n",
                  t.device, (void*)t.st, done, t.enq, last ? last : "?", next ? next : "?", done + 1);
    out += line;
  }
  if (!pending) out += "  no traced stream has work outstanding (a host-side wait, or untraced work)\n";
  return out;
}

void watch_loop() {
  for (;;) {
    std::this_thread::sleep_for(std::chrono::seconds(1));
    const int lim = g_limit.load();
    if (lim <= 0) continue;
    std::string text;
    {
      std::lock_guard<std::mutex> lk(g_mu);
      const auto now = std::chrono::steady_clock::now();
      for (Call& c : g_calls) {
        const double secs = std::chrono::duration<double>(now - c.t0).count();
        if (!c.reported && secs > lim) {
          c.reported = true;
          text += report(c, secs);
        }
      }
    }
    if (!text.empty()) emit(text);
  }
}

// Caller holds g_mu.  The pinned words and the thread come with the first traced launch.
bool ensure_started() {
  if (!g_words) {
    void* p = nullptr;
    if (hipHostMalloc(&p, MAX_STREAMS * sizeof(unsigned), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
      (void)hipGetLastError();
      d = p;
    }
    g_words = (unsigned*)p;
    g_words_dev = (unsigned*)d;
    for (int i = 0; i < MAX_STREAMS; ++i) g_words[i] = 0;
  }
  if (!g_thread) {
    g_thread = new std::thread(watch_loop);
    g_thread->detach();   // sleeps between checks; never joined (it holds nothing at exit)
  }
  return true;
}

}  // namespace

bool wd_enabled() { return limit() > 0; }

void wd_trace(hipStream_t st, const char* name) {
  if (limit() <= 0) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!ensure_started()) return;
  Traced* t = nullptr;
  for (Traced& x : g_streams)
    if (x.st == st) t = &x;
  if (!t) {
    // a destroyed stream's entry (wd_forget) is reused first: the stream pool destroys and recreates
    // streams when the shard configuration changes, so a long process would otherwise run out of slots
    for (Traced& x : g_streams)
      if (!x.st) {
        t = &x;
        break;
      }
    if (!t && (int)g_streams.size() < MAX_STREAMS) {
      g_streams.push_back(Traced{});
      t = &g_streams.back();
      t->slot = (unsigned)(g_streams.size() - 1);
    }
    if (!t) {
      static bool warned = false;
      if (!warned) emit("libmk watchdog: stream table full; new streams are not traced\n");
      warned = true;
      return;
    }
    const unsigned slot = t->slot;
    *t = Traced{};
    t->slot = slot;
    t->st = st;
    (void)hipGetDevice(&t->device);
    __atomic_store_n(g_words + slot, 0u, __ATOMIC_RELEASE);
  }
  const unsigned seq = ++t->enq;
  t->names[seq % RING] = name;
  hipLaunchKernelGGL(k_progress, dim3(1), dim3(64), 0, st, g_words_dev + t->slot, seq);
}

void wd_forget(hipStream_t st) {
  if (limit() <= 0) return;
  std::lock_guard<std::mutex> lk(g_mu);
  for (Traced& x : g_streams)
    if (x.st == st) {   // the slot becomes free for the next new stream (wd_trace resets it)
      __atomic_store_n(g_words + x.slot, x.enq, __ATOMIC_RELEASE);
      x.st = nullptr;
    }
}

ApiCall::ApiCall(const char* name) : id(-1) {
  if (limit() <= 0) return;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_thread) {
    g_thread = new std::thread(watch_loop);
    g_thread->detach();
  }
  id = ++g_next_call;
  g_calls.push_back(Call{id, name, std::chrono::steady_clock::now(), false});
}

ApiCall::~ApiCall() {
  if (id < 0) return;
  std::lock_guard<std::mutex> lk(g_mu);
  for (size_t i = 0; i < g_calls.size(); ++i)
    if (g_calls[i].id == id) {
      if (g_calls[i].reported) {
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - g_calls[i].t0).count();
        char line[160];
        std::snprintf(line, sizeof line, "libmk watchdog: %s (call %ld) returned after %.1f s\n", g_calls[i].name, id,
                      secs);
        emit(line);
      }
      g_calls.erase(g_calls.begin() + (long)i);
      break;
    }
}

}  // namespace mk

extern "C" int mk_set_watchdog(int32_t seconds) {
  mk::g_limit.store(seconds > 0 ? seconds : 0);
  return 0;
}

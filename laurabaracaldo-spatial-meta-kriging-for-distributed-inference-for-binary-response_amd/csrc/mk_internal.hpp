// Library-internal interface between the session (mk_api.hip) and the multi-device driver
// (mk_multi.hip): a shard's quantile grids stay in HBM for the device-to-device combine.
#pragma once
#include <hip/hip_runtime.h>
#include <string>
#include "../../include/mk.h"

namespace mk {
struct ShardInfo {
  int device, S, P, q, n_test, tiled, pred_tile, n_kept;
  hipStream_t stream;
};
int host_error(int code, const char* msg);   // sets mk_last_error()
int session_info(const mk_session* s, ShardInfo* info);
int session_param_grids(mk_session* s, double* d_out);                   // [S][P][200]
int session_wpred_grids(mk_session* s, double* d_out);                   // fused: [S][q n_test][200]
int session_tile_grids(mk_session* s, int t0, double* d_out, mk_outputs* o);   // tiled: [S][q Tc][200]
// A plain non-blocking stream of the current device from libmk's stream pool, and its return
// (drained by the caller): the node driver's per-block streams live as long as the sessions' do.
hipError_t stream_acquire(int device, hipStream_t* st);
void stream_release(int device, hipStream_t st);

// Saves the calling thread's current device and restores it at scope exit.
struct DeviceGuard {
  int saved = -1;
  DeviceGuard() {
    if (hipGetDevice(&saved) != hipSuccess) {
      saved = -1;
      (void)hipGetLastError();
    }
  }
  ~DeviceGuard() {
    if (saved >= 0) (void)hipSetDevice(saved);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// Stall watchdog (mk_watch.hip; MK_WATCHDOG=<seconds>): wd_trace after every launch records the
// kernel's name for its stream and enqueues the progress-word store; ApiCall registers a C-ABI
// entry that may wait on the device, for the watchdog thread to report when it overruns.
bool wd_enabled();
void wd_trace(hipStream_t st, const char* name);
void wd_forget(hipStream_t st);
struct ApiCall {
  explicit ApiCall(const char* name);
  ~ApiCall();
  ApiCall(const ApiCall&) = delete;
  ApiCall& operator=(const ApiCall&) = delete;
  long id;
};
}  // namespace mk

// A kernel launch followed by its watchdog trace (a no-op unless the watchdog is on).
#define MK_LAUNCH(kernel, grid, block, lds, st, ...)                      \
  do {                                                                    \
    hipLaunchKernelGGL(kernel, grid, block, lds, st, __VA_ARGS__);        \
    ::mk::wd_trace(st, #kernel);                                          \
  } while (0)

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
}  // namespace mk

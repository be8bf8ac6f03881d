// Shared helpers for the gfx950 kernels of libtt_mi355x.so (wave64, CDNA4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string>
#include "tt_mi355x.h"

// Experiment hooks (environment switches, s_memrealtime phase stamps, T1 debug bits used by
// scripts/*_stamps.py): compiled out of release builds. The experiment library is built by
// `python -m two_tower_recommender_model_amd.build --experiments` into lib_exp/ (never over the
// release lib/) and loaded with TT_EXPERIMENT_LIB=1
#ifndef TT_EXPERIMENTS
#define TT_EXPERIMENTS 0
#endif

#define TT_WAVE 64

typedef __attribute__((ext_vector_type(4))) float f32x4v;

namespace tt {

// thread-local last error, set by the host-side launch functions
void set_error(const std::string& msg);

inline int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return (int)e;
  }
  return TT_OK;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// workgroups are dealt round-robin over the 8 XCDs (bid % 8): logical index of workgroup bid
// among n so that each XCD runs one contiguous 1/8 of [0, n) (any n)
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int x = bid & 7, loc = bid >> 3, q = n >> 3, r = n & 7;
  return x * q + min(x, r) + loc;
}

// a consumer launch's in-launch signal / wait of a device-initiated exchange (tt_peer_wait_t),
// by value in the kernel arguments; W = 0: none
struct PxWait {
  int32_t W, sys;
  int32_t* flag[TT_PEER_MAXW];
  const int32_t* flags;
  const int32_t* epoch;
  int32_t* err;
  int64_t ticks;
};
// workgroup 0, threads [0, W): store the epoch into every peer's flag word for this source
__device__ __forceinline__ void px_signal(const PxWait& w) {
  const int s = (int)threadIdx.x;
  if (s < w.W) {
    const int e = __hip_atomic_load(w.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w.sys)
      __hip_atomic_store(w.flag[s], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      __hip_atomic_store(w.flag[s], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// every thread of the workgroup: threads [0, W) poll (relaxed) until source s's flag holds the
// epoch, then acquire; the workgroup's barrier releases the others. A wait past the timeout sets
// *err (sticky) and goes on (the data is then invalid).
__device__ __forceinline__ void px_wait(const PxWait& w) {
  const int s = (int)threadIdx.x;
  if (s < w.W) {
    // the epoch and the first poll of the flag in flight together (one round trip, not two)
    const int e = __hip_atomic_load(w.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int f = __hip_atomic_load(w.flags + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
    bool late = false;
    while (f < e) {
      if ((int64_t)__builtin_amdgcn_s_memrealtime() - t0 > w.ticks) {
        late = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      f = __hip_atomic_load(w.flags + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (late) __hip_atomic_fetch_or(w.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w.sys)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    else
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// host: a tt_peer_wait_t into kernel arguments (W = 0 for none)
inline int peer_wait_args(const tt_peer_wait_t* p, PxWait& w, const char* who) {
  w = PxWait{};
  if (!p) return TT_OK;
  const std::string s(who);
  if (p->W < 1 || p->W > TT_PEER_MAXW || !p->flags || !p->epoch || !p->err || p->timeout_ticks <= 0)
    return fail(TT_EINVAL, s + ": wait.W 1..TT_PEER_MAXW, flags, epoch, err and a timeout");
  w.W = p->W;
  w.sys = p->sys ? 1 : 0;
  for (int d = 0; d < p->W; ++d) {
    if (!p->flag[d]) return fail(TT_EINVAL, s + ": wait.flag[d] is null");
    w.flag[d] = p->flag[d];
  }
  w.flags = p->flags;
  w.epoch = p->epoch;
  w.err = p->err;
  w.ticks = p->timeout_ticks;
  return TT_OK;
}

// host: a direct-exchange descriptor (tt_peer_direct_t) the kernels can follow blindly
inline int peer_direct_check(const tt_peer_direct_t& x, const char* who) {
  const std::string w(who);
  if (x.W < 1 || x.W > TT_PEER_MAXW) return fail(TT_EINVAL, w + ": direct.W must be 1..TT_PEER_MAXW");
  if (x.first_row[0] != 0) return fail(TT_EINVAL, w + ": direct.first_row[0] must be 0");
  for (int d = 0; d < x.W; ++d) {
    if (!x.row0[d]) return fail(TT_EINVAL, w + ": direct.row0[d] is null");
    if (d && x.first_row[d] < x.first_row[d - 1]) return fail(TT_EINVAL, w + ": direct.first_row not ascending");
    if (x.copy_len[d] < 0 || (x.copy_len[d] & 15) ||
        (x.copy_len[d] && (!x.copy_src[d] || !x.copy_dst[d] || (reinterpret_cast<uintptr_t>(x.copy_src[d]) & 15) ||
                           (reinterpret_cast<uintptr_t>(x.copy_dst[d]) & 15))))
      return fail(TT_EINVAL, w + ": direct copies must be 16-B aligned multiples of 16 B");
  }
  return TT_OK;
}

// Kernel-argument bundle of the table / feature metadata (passed by value: graph-capturable, no
// host->device copy per call). 64 tables x 32 B + 64 features x 8 B + 16 = 2.6 KB < 4 KB limit.
struct EmbMeta {
  tt_table_meta_t tables[TT_MAX_TABLES];
  tt_feature_meta_t features[TT_MAX_FEATURES];
  int32_t T;
  int32_t F;
  int64_t B;
};

int pack_meta(EmbMeta& m, const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features,
              int F, int64_t B);

// --- device helpers -------------------------------------------------------------------------

__device__ __forceinline__ int64_t load_id(const void* values, int id_dtype, int64_t i) {
  return id_dtype == TT_I64 ? reinterpret_cast<const int64_t*>(values)[i]
                            : (int64_t)reinterpret_cast<const int32_t*>(values)[i];
}

// Python's a % n (result takes the divisor's sign): transform_to_torchrec_batch's `id % N`,
// 03_model_training.py:361, on tensors of either sign
__device__ __forceinline__ int64_t py_mod64(int64_t a, int64_t n) {
  // ids already in [0, n) (what a well-formed dataset holds): no division at all
  if ((uint64_t)a < (uint64_t)n) return a;
  // 32-bit fast path (ids and table sizes below 2^32: the usual case): a 64-bit remainder is a
  // long emulated sequence on CDNA, a 32-bit one a short float-reciprocal sequence
  if ((uint64_t)a <= 0xffffffffull && (uint64_t)n <= 0xffffffffull && n > 0) return (int64_t)((uint32_t)a % (uint32_t)n);
  int64_t r = a % n;
  return (r != 0 && ((r < 0) != (n < 0))) ? r + n : r;
}

// a / b for 0 <= a, 0 < b (32-bit fast path as py_mod64)
__device__ __forceinline__ int64_t udiv64(int64_t a, int64_t b) {
  if ((uint64_t)a <= 0xffffffffull && (uint64_t)b <= 0xffffffffull) return (int64_t)((uint32_t)a / (uint32_t)b);
  return a / b;
}

// Row-wise Adagrad arithmetic (torchrec RowWiseAdagrad, 03_model_training.py:791-795) of one
// 4-wide chunk of a row, shared by the update paths so that each computes bitwise-identical
// results for the same gradient row: s += mean_d(G^2); w -= lr * G / (sqrt(s) + eps).
// rw_step is the row's factor -lr / (sqrt(s) + eps), divided once per row; rw_apply is one fma
// per element (a precise division per element was ~10 VALU instructions each)
__device__ __forceinline__ float rw_sq4(const f32x4v& g) { return g[0] * g[0] + g[1] * g[1] + g[2] * g[2] + g[3] * g[3]; }
__device__ __forceinline__ float rw_state(float s_old, float sq, int D) { return s_old + sq / (float)D; }
__device__ __forceinline__ float rw_step(float snew, float lr, float eps) { return -lr / (sqrtf(snew) + eps); }
__device__ __forceinline__ f32x4v rw_apply(f32x4v w, const f32x4v& g, float step) {
#pragma unroll
  for (int v = 0; v < 4; ++v) w[v] = fmaf(g[v], step, w[v]);
  return w;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace tt

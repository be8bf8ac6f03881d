// Device-initiated fixed-block exchange: the sharded step's two all-to-alls (exchange A: gradient
// rows | tower gradient | next ids; exchange B: next rows) as this rank's own kernels storing
// straight into every peer's receive buffer, mapped into this process with hipIpcOpenMemHandle.
// Replaces dist.all_to_all_single (the RCCL kernel, ~10 us of fixed latency per exchange even as a
// local copy at world 1) on the sharded step's data path; opt-in (sharded.PeerComm).
//
// Protocol, per registered receive buffer (one per exchange), W ranks in lockstep:
//   put  (grid chunks x W): block d of the send buffer -> peer d's buffer at this rank's slot; each
//        workgroup releases its stores at system scope and counts in; the last one of destination
//        d stores the epoch into peer d's flag word for this source (release, system scope).
//   wait (one wave): spins until every source's flag word holds the epoch (acquire, system scope),
//        bounded by a timeout (sticky error word, no hang), then advances the local epoch.
// Reuse of a receive buffer is ordered by the exchanges themselves: a rank puts exchange A of step
// s + 1 only after its wait on exchange B of step s, which every peer signals after consuming its
// exchange-A block of step s (and symmetrically for B), so one buffer per exchange suffices.
#include <algorithm>
#include <cstring>

#include "tt_common.h"

namespace tt {
namespace {

constexpr int PX_THREADS = 256;
constexpr int PX_UNROLL = 8;
constexpr int64_t PX_CHUNK = (int64_t)PX_THREADS * 16 * PX_UNROLL;  // bytes per workgroup (32 KB)

struct PxArgs {
  int32_t W, rank;
  const char* src;
  int64_t src_off[TT_PEER_MAXW];
  int64_t len[TT_PEER_MAXW];
  char* dst[TT_PEER_MAXW];
  int32_t* flag[TT_PEER_MAXW];
  int32_t* state;  // [0] epoch, [1 + d] workgroups done for destination d
};

__global__ void __launch_bounds__(PX_THREADS) peer_put_kernel(PxArgs a) {
  const int d = blockIdx.y;
  const int tid = threadIdx.x;
  const int64_t len = a.len[d];
  const int64_t c0 = (int64_t)blockIdx.x * PX_CHUNK;
  if (c0 < len) {
    const char* s = a.src + a.src_off[d];
    char* t = a.dst[d];
    uint4 v[PX_UNROLL];
#pragma unroll
    for (int u = 0; u < PX_UNROLL; ++u) {
      const int64_t i = c0 + ((int64_t)u * PX_THREADS + tid) * 16;
      if (i < len) v[u] = *reinterpret_cast<const uint4*>(s + i);
    }
#pragma unroll
    for (int u = 0; u < PX_UNROLL; ++u) {
      const int64_t i = c0 + ((int64_t)u * PX_THREADS + tid) * 16;
      if (i < len) *reinterpret_cast<uint4*>(t + i) = v[u];
    }
  }
  // every wave's stores done and past this agent's caches before the count
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (tid == 0) {
    int32_t* done = a.state + 1 + d;
    const int prev = __hip_atomic_fetch_add(done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (int)gridDim.x - 1) {
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int e = __hip_atomic_load(a.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
      __hip_atomic_store(a.flag[d], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ void __launch_bounds__(64) peer_wait_kernel(const int32_t* flags, int W, int32_t* state, int32_t* err,
                                                       int64_t timeout_ticks) {
  const int s = threadIdx.x;
  const int e = __hip_atomic_load(state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  int late = 0;
  if (s < W) {
    const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flags + s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if ((int64_t)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        late = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  if (late) __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the peers' blocks visible to the kernels after this one
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (s == 0) __hip_atomic_store(state, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" {

int tt_peer_alloc(size_t bytes, void** out) {
  if (!out || bytes == 0) return fail(TT_EINVAL, "peer_alloc: null output or zero bytes");
  *out = nullptr;
  hipError_t e = hipExtMallocWithFlags(out, bytes, hipDeviceMallocFinegrained);
  if (e != hipSuccess) return fail((int)e, std::string("peer_alloc: ") + hipGetErrorString(e));
  e = hipMemset(*out, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    (void)hipFree(*out);
    *out = nullptr;
    return fail((int)e, std::string("peer_alloc: ") + hipGetErrorString(e));
  }
  return TT_OK;
}

int tt_peer_free(void* p) {
  hipError_t e = hipFree(p);
  return e == hipSuccess ? TT_OK : fail((int)e, std::string("peer_free: ") + hipGetErrorString(e));
}

int tt_peer_export(const void* p, void* handle, int64_t* offset) {
  if (!p || !handle || !offset) return fail(TT_EINVAL, "peer_export: null argument");
  static_assert(sizeof(hipIpcMemHandle_t) <= TT_PEER_HANDLE_BYTES, "IPC handle size");
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, const_cast<void*>(p));
  hipIpcMemHandle_t h;
  if (e == hipSuccess) e = hipIpcGetMemHandle(&h, base);
  if (e != hipSuccess) return fail((int)e, std::string("peer_export: ") + hipGetErrorString(e));
  std::memset(handle, 0, TT_PEER_HANDLE_BYTES);
  std::memcpy(handle, &h, sizeof(h));
  *offset = (int64_t)(reinterpret_cast<const char*>(p) - reinterpret_cast<const char*>(base));
  return TT_OK;
}

int tt_peer_import(const void* handle, void** base) {
  if (!handle || !base) return fail(TT_EINVAL, "peer_import: null argument");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  *base = nullptr;
  hipError_t e = hipIpcOpenMemHandle(base, h, hipIpcMemLazyEnablePeerAccess);
  return e == hipSuccess ? TT_OK : fail((int)e, std::string("peer_import: ") + hipGetErrorString(e));
}

int tt_peer_unimport(void* base) {
  hipError_t e = hipIpcCloseMemHandle(base);
  return e == hipSuccess ? TT_OK : fail((int)e, std::string("peer_unimport: ") + hipGetErrorString(e));
}

int tt_peer_put(const tt_peer_put_t* p, void* stream) {
  if (!p || p->W < 1 || p->W > TT_PEER_MAXW || p->rank < 0 || p->rank >= p->W || !p->src || !p->state)
    return fail(TT_EINVAL, "peer_put: 1 <= W <= TT_PEER_MAXW, 0 <= rank < W, src and state set");
  PxArgs a;
  a.W = p->W;
  a.rank = p->rank;
  a.src = reinterpret_cast<const char*>(p->src);
  a.state = p->state;
  int64_t most = 0;
  for (int d = 0; d < TT_PEER_MAXW; ++d) {
    const bool live = d < p->W;
    a.src_off[d] = live ? p->src_off[d] : 0;
    a.len[d] = live ? p->len[d] : 0;
    a.dst[d] = live ? reinterpret_cast<char*>(p->dst[d]) : nullptr;
    a.flag[d] = live ? p->flag[d] : nullptr;
    if (!live) continue;
    const uintptr_t s = reinterpret_cast<uintptr_t>(a.src) + (uintptr_t)a.src_off[d];
    if (a.len[d] < 0 || a.src_off[d] < 0 || (a.len[d] & 15) || (s & 15) ||
        (reinterpret_cast<uintptr_t>(a.dst[d]) & 15) || (a.len[d] && !a.dst[d]) || !a.flag[d] ||
        (reinterpret_cast<uintptr_t>(a.flag[d]) & 3))
      return fail(TT_EINVAL, "peer_put: blocks must be 16-B aligned multiples of 16 B, every flag word set");
    most = std::max(most, a.len[d]);
  }
  const int64_t nchunk = std::max<int64_t>(1, ceil_div(most, PX_CHUNK));
  if (nchunk > INT32_MAX) return fail(TT_EINVAL, "peer_put: block too large");
  peer_put_kernel<<<dim3((unsigned)nchunk, (unsigned)p->W), dim3(PX_THREADS), 0, as_stream(stream)>>>(a);
  return check_launch("peer_put");
}

int tt_peer_wait(const int32_t* flags, int W, int32_t* state, int32_t* err, double timeout_s, void* stream) {
  if (!flags || !state || !err || W < 1 || W > TT_PEER_MAXW || !(timeout_s > 0))
    return fail(TT_EINVAL, "peer_wait: flags, state, err set, 1 <= W <= TT_PEER_MAXW, timeout > 0");
  // s_memrealtime counts at 100 MHz on MI355X
  const int64_t ticks = (int64_t)std::min(timeout_s * 1e8, 9e17);
  peer_wait_kernel<<<dim3(1), dim3(64), 0, as_stream(stream)>>>(flags, W, state, err, ticks);
  return check_launch("peer_wait");
}

}  // extern "C"

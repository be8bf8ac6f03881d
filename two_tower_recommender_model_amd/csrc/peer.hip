// Device-initiated fixed-block exchange: the sharded step's two all-to-alls (exchange A: gradient
// rows | tower gradient | next ids; exchange B: next rows) as this rank's own kernels storing
// straight into every peer's receive buffer, mapped into this process with hipIpcOpenMemHandle.
// Replaces dist.all_to_all_single (the RCCL kernel, ~10 us of fixed latency per exchange even as a
// local copy at world 1) on the sharded step's data path; opt-in (sharded.PeerComm).
//
// Protocol, per registered receive buffer (one per exchange), W ranks in lockstep:
//   put  (grid chunks x W): block d of the send buffer -> peer d's buffer at this rank's slot.
//   signal / wait (one wave, after the put's kernel boundary): lane d stores the epoch into peer
//        d's flag word for this source (release, system scope), then spins until source d's word
//        in this rank's buffer holds the epoch (acquire, system scope), bounded by a timeout
//        (sticky error word, no hang); the local epoch then advances.
// Reuse of a receive buffer is ordered by the exchanges themselves: a rank puts exchange A of step
// s + 1 only after its wait on exchange B of step s, which every peer signals after consuming its
// exchange-A block of step s (and symmetrically for B), so one buffer per exchange suffices.
#include <algorithm>
#include <cstring>

#include "tt_common.h"

namespace tt {
namespace {

constexpr int PX_THREADS = 256;
constexpr int PX_UNROLL = 4;  // 16-B units per lane
constexpr int64_t PX_CHUNK = (int64_t)PX_THREADS * 16 * PX_UNROLL;  // bytes per workgroup (16 KB; 4 KB narrow)

struct PxArgs {
  int32_t W, rank, sys;
  const char* src;
  int64_t src_off[TT_PEER_MAXW];
  int64_t len[TT_PEER_MAXW];
  char* dst[TT_PEER_MAXW];
  int32_t* flag[TT_PEER_MAXW];
  int32_t* state;  // [0] epoch
};

// V = uint4 (every block 16-B aligned, the sharded steps' usual layout) or uint32_t (4-B blocks)
template <typename V>
__global__ void __launch_bounds__(PX_THREADS) peer_put_kernel(PxArgs a) {
  const int d = blockIdx.y;
  const int64_t n = a.len[d] / (int64_t)sizeof(V);
  const int64_t i0 = (int64_t)blockIdx.x * (PX_THREADS * PX_UNROLL) + threadIdx.x;
  if (i0 >= n) return;
  const V* s = reinterpret_cast<const V*>(a.src + a.src_off[d]);
  V* t = reinterpret_cast<V*>(a.dst[d]);
  // four independent loads per lane in flight, then their stores; scalars, not a local array:
  // the array form was promoted to LDS with every load waited on alone (3.8 against 28.6 us per put
  // of 8.5 MB, profiles/r05_peer_exchange_notes.log)
  const int64_t i1 = i0 + PX_THREADS, i2 = i0 + 2 * PX_THREADS, i3 = i0 + 3 * PX_THREADS;
  V v0 = s[i0], v1, v2, v3;
  if (i1 < n) v1 = s[i1];
  if (i2 < n) v2 = s[i2];
  if (i3 < n) v3 = s[i3];
  t[i0] = v0;
  if (i1 < n) t[i1] = v1;
  if (i2 < n) t[i2] = v2;
  if (i3 < n) t[i3] = v3;
}

// One wave, after the put kernel (whose end made its stores visible): lane d signals peer d, then
// waits for source d's signal. A release fence + arrival count in every put workgroup instead (the
// last one signalling) cost 25.6 against 8.8 us per put of that form (profiles/r05_peer_exchange_notes.log).
__global__ void __launch_bounds__(64) peer_signal_wait_kernel(PxArgs a, const int32_t* flags, int32_t* err,
                                                              int64_t timeout_ticks) {
  const int s = threadIdx.x;
  const int e = __hip_atomic_load(a.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  int late = 0;
  if (s < a.W) {
    // peers on other devices: a release at system scope (the L2 write-back of the put's data). All
    // on this device: the put's kernel boundary already published its stores at agent scope, so a
    // relaxed store of the flag is enough (the release cost 4.5 us, most of this kernel)
    if (a.sys)
      __hip_atomic_store(a.flag[s], e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      __hip_atomic_store(a.flag[s], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
    while ((a.sys ? __hip_atomic_load(flags + s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)
                  : __hip_atomic_load(flags + s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) < e) {
      if ((int64_t)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        late = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  if (late) __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the peers' blocks visible to the kernels after this one
  if (a.sys)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (s == 0) __hip_atomic_store(a.state, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

int tt_peer_exchange(const tt_peer_put_t* p, const int32_t* flags, int32_t* err, double timeout_s, void* stream) {
  if (!p || p->W < 1 || p->W > TT_PEER_MAXW || p->rank < 0 || p->rank >= p->W || !p->src || !p->state || !flags ||
      !err || !(timeout_s > 0))
    return fail(TT_EINVAL, "peer_exchange: 1 <= W <= TT_PEER_MAXW, 0 <= rank < W, src, state, flags, err set, "
                           "timeout > 0");
  PxArgs a;
  a.W = p->W;
  a.rank = p->rank;
  a.sys = p->same_device ? 0 : 1;
  a.src = reinterpret_cast<const char*>(p->src);
  a.state = p->state;
  int64_t most = 0;
  bool wide = true;
  for (int d = 0; d < TT_PEER_MAXW; ++d) {
    const bool live = d < p->W;
    a.src_off[d] = live ? p->src_off[d] : 0;
    a.len[d] = live ? p->len[d] : 0;
    a.dst[d] = live ? reinterpret_cast<char*>(p->dst[d]) : nullptr;
    a.flag[d] = live ? p->flag[d] : nullptr;
    if (!live) continue;
    const uintptr_t s = reinterpret_cast<uintptr_t>(a.src) + (uintptr_t)a.src_off[d];
    const uintptr_t t = reinterpret_cast<uintptr_t>(a.dst[d]);
    if (a.len[d] < 0 || a.src_off[d] < 0 || (a.len[d] & 3) || (s & 3) || (t & 3) || (a.len[d] && !a.dst[d]) ||
        !a.flag[d] || (reinterpret_cast<uintptr_t>(a.flag[d]) & 3))
      return fail(TT_EINVAL, "peer_exchange: blocks must be 4-B aligned multiples of 4 B, every flag word set");
    if ((a.len[d] & 15) || (s & 15) || (t & 15)) wide = false;
    most = std::max(most, a.len[d]);
  }
  const int64_t nchunk = ceil_div(most, wide ? PX_CHUNK : PX_CHUNK / 4);
  if (nchunk > INT32_MAX) return fail(TT_EINVAL, "peer_exchange: block too large");
  if (nchunk > 0) {
    const dim3 grid((unsigned)nchunk, (unsigned)p->W);
    if (wide)
      peer_put_kernel<uint4><<<grid, dim3(PX_THREADS), 0, as_stream(stream)>>>(a);
    else
      peer_put_kernel<uint32_t><<<grid, dim3(PX_THREADS), 0, as_stream(stream)>>>(a);
    if (int rc = check_launch("peer_exchange (put)")) return rc;
  }
  // s_memrealtime counts at 100 MHz on MI355X
  const int64_t ticks = (int64_t)std::min(timeout_s * 1e8, 9e17);
  peer_signal_wait_kernel<<<dim3(1), dim3(64), 0, as_stream(stream)>>>(a, flags, err, ticks);
  return check_launch("peer_exchange (signal / wait)");
}

}  // extern "C"

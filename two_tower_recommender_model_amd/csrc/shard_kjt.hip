// Multi-hot sharded step (BASELINE config 5: bags of ~20 ids, users table-wise + items row-wise) with
// FIXED-SIZE exchanges, so the whole step is capturable into HIP graphs (TorchRec's KJTAllToAll
// host-synchronises its split sizes every batch, torchrec/distributed/embeddingbag.py:337-339 in this
// repo's shim). Requester -> owner: per destination a fixed block [lengths F*B | ids cap] (int32);
// owner -> requester: one pooled row per (bag, owner) (row-wise: partial sums, TorchRec's
// reduce-scatter semantics); requester -> owner: the bag gradients. Integer routing + row copies:
// HBM / latency bound, no MFMA. Device code here; orchestration in sharded_kjt.py.
#include "tt_common.h"

namespace tt {

constexpr int KR_MAXW = 16;

struct KjtRouteArgs {
  const void* values;
  int id_dtype;
  const int32_t* offsets;  // [F*B + 1]
  int64_t num_emb[TT_MAX_FEATURES];
  int64_t block[TT_MAX_FEATURES];  // row-wise block (> 0) or 0: table-wise
  int32_t owner[TT_MAX_FEATURES];
  int F, W;
  int64_t B, cap, stride;  // ids per destination block, elements per destination block
  int32_t* send;           // [W][stride]: lengths [F*B] then ids [cap]
  int32_t* flags;          // {overflow, bad key}
  int32_t* lens;           // workspace [W][F*B]: the lengths, contiguous
  int32_t* base;           // workspace [W*F*B + 1]: their complete cumsum (prefix within d = base - base[d*F*B])
};

__device__ __forceinline__ int64_t kr_id(const KjtRouteArgs& a, int64_t i) {
  return a.id_dtype == TT_I64 ? reinterpret_cast<const int64_t*>(a.values)[i]
                              : (int64_t)reinterpret_cast<const int32_t*>(a.values)[i];
}

// owner of id (in range) of feature f, and its row in the owner's shard
__device__ __forceinline__ int kr_owner(const KjtRouteArgs& a, int f, int64_t id, int64_t& local) {
  if (a.block[f] > 0) {
    const int d = (int)(id / a.block[f]);
    local = id - (int64_t)d * a.block[f];
    return d;
  }
  local = id;
  return a.owner[f];
}

// the ids of bag i in chunks of KR_CHUNK loads issued together (a thread-per-bag loop of dependent
// loads waited ~1 us per id): fn(k, id) for each id in bag order
constexpr int KR_CHUNK = 8;
template <typename Fn>
__device__ __forceinline__ void kr_bag_ids(const KjtRouteArgs& a, int32_t o0, int32_t o1, Fn&& fn) {
  for (int32_t k0 = o0; k0 < o1; k0 += KR_CHUNK) {
    int64_t v[KR_CHUNK];
#pragma unroll
    for (int u = 0; u < KR_CHUNK; ++u) v[u] = k0 + u < o1 ? kr_id(a, k0 + u) : 0;
#pragma unroll
    for (int u = 0; u < KR_CHUNK; ++u)
      if (k0 + u < o1) fn(k0 + u, v[u]);
  }
}

// pass 1 (thread per bag): ids per owner of the bag -> each destination's lengths region and the
// contiguous [W][F*B] copy the scan reads
__global__ void __launch_bounds__(256) kjt_route_count_kernel(KjtRouteArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = (int64_t)a.F * a.B;
  if (i >= n) return;
  const int f = (int)(i / a.B);
  const int32_t o0 = a.offsets[i], o1 = a.offsets[i + 1];
  int c[KR_MAXW];
#pragma unroll
  for (int w = 0; w < KR_MAXW; ++w) c[w] = 0;
  int bad = 0;
  kr_bag_ids(a, o0, o1, [&](int32_t, int64_t id) {
    if (id < 0 || id >= a.num_emb[f]) {
      bad = 1;
      return;
    }
    int64_t lr;
    const int d = kr_owner(a, f, id, lr);
#pragma unroll
    for (int w = 0; w < KR_MAXW; ++w) c[w] += d == w;
  });
  if (bad) a.flags[1] = 1;
#pragma unroll
  for (int w = 0; w < KR_MAXW; ++w)
    if (w < a.W) {
      a.send[(int64_t)w * a.stride + i] = c[w];
      a.lens[(int64_t)w * n + i] = c[w];
    }
}

// pass 3 (thread per bag): each kept id -> its destination's id region at (the destination's
// exclusive prefix of its lengths) + rank in the bag; the block totals against cap (overflow flag)
__global__ void __launch_bounds__(256) kjt_route_place_kernel(KjtRouteArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = (int64_t)a.F * a.B;
  if (i < a.W) {
    const int32_t tot = a.base[(i + 1) * n] - a.base[i * n];
    if (tot > a.cap) a.flags[0] = 1;
  }
  if (i >= n) return;
  const int f = (int)(i / a.B);
  const int32_t o0 = a.offsets[i], o1 = a.offsets[i + 1];
  int c[KR_MAXW];
#pragma unroll
  for (int w = 0; w < KR_MAXW; ++w) {
    c[w] = 0;
    if (w < a.W) {
      const int32_t lo = a.base[(int64_t)w * n + i], hi = a.base[(int64_t)w * n + i + 1];
      c[w] = lo - a.base[(int64_t)w * n];
      // a block over cap keeps the ids that fit (positions < cap) and the lengths it sends say so:
      // the owner's offsets then never pass cap per source, whatever the flag says later
      const int64_t room = a.cap - (int64_t)c[w];
      const int32_t keep = (int32_t)(room <= 0 ? 0 : (room < hi - lo ? room : hi - lo));
      if (keep != hi - lo) a.send[(int64_t)w * a.stride + i] = keep;
    }
  }
  kr_bag_ids(a, o0, o1, [&](int32_t, int64_t id) {
    if (id < 0 || id >= a.num_emb[f]) return;
    int64_t lr;
    const int d = kr_owner(a, f, id, lr);
    int pos = 0;
#pragma unroll
    for (int w = 0; w < KR_MAXW; ++w)
      if (d == w) pos = c[w]++;
    if (pos < a.cap) a.send[(int64_t)d * a.stride + n + pos] = (int32_t)lr;
  });
}

// ---- owner side: received blocks -> one contiguous KJT over (source s, served feature k) keys ----
struct KjtUnpackArgs {
  const int32_t* recv;  // [W][stride]
  int64_t stride, FB, cap, B;
  int W, Fr;
  int32_t feats[TT_MAX_FEATURES];  // served features, ascending
  int32_t* lengths;  // [W * Fr * B]
  const int32_t* offsets;  // [W * Fr * B + 1] (complete cumsum of lengths)
  int32_t* values;
};

__global__ void __launch_bounds__(256) kjt_unpack_lengths_kernel(KjtUnpackArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (s, k, b)
  const int64_t per = (int64_t)a.Fr * a.B;
  if (i >= (int64_t)a.W * per) return;
  const int s = (int)(i / per);
  const int64_t r = i - (int64_t)s * per;
  const int k = (int)(r / a.B);
  const int64_t b = r - (int64_t)k * a.B;
  a.lengths[i] = a.recv[(int64_t)s * a.stride + (int64_t)a.feats[k] * a.B + b];
}

__global__ void __launch_bounds__(256) kjt_unpack_values_kernel(KjtUnpackArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (s, j < cap)
  if (i >= (int64_t)a.W * a.cap) return;
  const int s = (int)(i / a.cap);
  const int64_t j = i - (int64_t)s * a.cap;
  const int64_t per = (int64_t)a.Fr * a.B;
  const int32_t lo = a.offsets[(int64_t)s * per], hi = a.offsets[(int64_t)(s + 1) * per];
  if (j < hi - lo) a.values[lo + j] = a.recv[(int64_t)s * a.stride + a.FB + j];
}

// ---- requester side: pooled partials of every owner -> the tower input; the bag gradients -> every
// owner's block (owner_col[d][f] = column of feature f in owner d's block rows, -1: d does not serve f)
struct PartialArgs {
  int W, F, D;
  int64_t B, blk_stride, ld_blk, ldo;
  int32_t col[KR_MAXW][TT_MAX_FEATURES];
};

__global__ void __launch_bounds__(256) pooled_partials_sum_kernel(PartialArgs a, const float* __restrict__ recv,
                                                                  float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (b, f, 4-float chunk)
  const int q = a.D / 4;
  if (i >= a.B * a.F * q) return;
  const int64_t b = i / ((int64_t)a.F * q);
  const int r = (int)(i - b * a.F * q);
  const int f = r / q, c = 4 * (r - f * q);
  f32x4v acc = (f32x4v)(0.f);
  for (int d = 0; d < a.W; ++d) {  // ascending owner: the same sum on every rank and run
    const int col = a.col[d][f];
    if (col >= 0) acc += *reinterpret_cast<const f32x4v*>(recv + d * a.blk_stride + b * a.ld_blk + col + c);
  }
  *reinterpret_cast<f32x4v*>(out + b * a.ldo + (int64_t)f * a.D + c) = acc;
}

__global__ void __launch_bounds__(256) pooled_grad_pack_kernel(PartialArgs a, const float* __restrict__ g,
                                                               float* __restrict__ send) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int q = a.D / 4;
  if (i >= a.B * a.F * q) return;
  const int64_t b = i / ((int64_t)a.F * q);
  const int r = (int)(i - b * a.F * q);
  const int f = r / q, c = 4 * (r - f * q);
  const f32x4v v = *reinterpret_cast<const f32x4v*>(g + b * a.ldo + (int64_t)f * a.D + c);
  for (int d = 0; d < a.W; ++d) {
    const int col = a.col[d][f];
    if (col >= 0) *reinterpret_cast<f32x4v*>(send + d * a.blk_stride + b * a.ld_blk + col + c) = v;
  }
}

static int partial_args(int W, int F, int64_t B, int D, const int32_t* owner_col, int64_t blk_stride, int64_t ld_blk,
                        int64_t ldo, PartialArgs& p) {
  if (W < 1 || W > KR_MAXW || F < 1 || F > TT_MAX_FEATURES || B < 1 || D < 4 || D % 4 || !owner_col)
    return fail(TT_EINVAL, "pooled partials: W in [1, 16], F in [1, 64], D % 4 == 0");
  if (ldo % 4 || ld_blk % 4 || blk_stride % 4 || ldo < (int64_t)F * D)
    return fail(TT_EINVAL, "pooled partials: strides must be multiples of 4 floats");
  p.W = W;
  p.F = F;
  p.D = D;
  p.B = B;
  p.blk_stride = blk_stride;
  p.ld_blk = ld_blk;
  p.ldo = ldo;
  for (int d = 0; d < W; ++d)
    for (int f = 0; f < F; ++f) {
      const int c = owner_col[d * F + f];
      if (c >= 0 && (c % 4 || c + D > ld_blk)) return fail(TT_EINVAL, "pooled partials: column outside the block row");
      p.col[d][f] = c;
    }
  return TT_OK;
}

}  // namespace tt

using namespace tt;

extern "C" {

int tt_complete_cumsum(const int32_t* lengths, int64_t n, int32_t* offsets, void* workspace, size_t ws_bytes,
                       void* stream);
size_t tt_complete_cumsum_workspace_bytes(int64_t n);

size_t tt_kjt_route_workspace_bytes(int F, int64_t B, int W) {
  const int64_t n = (int64_t)W * F * B;
  return align_up((size_t)n * 4, 256) + align_up((size_t)(n + 1) * 4, 256) + tt_complete_cumsum_workspace_bytes(n);
}

int tt_kjt_route(int F, int64_t B, const void* values, int id_dtype, const int32_t* offsets,
                 const int64_t* num_embeddings, const int64_t* block_sizes, const int32_t* owners, int W, int64_t cap,
                 int64_t blk_stride, int32_t* send, int32_t* flags, void* workspace, size_t ws_bytes, void* stream) {
  if (F < 1 || F > TT_MAX_FEATURES || W < 1 || W > KR_MAXW || B < 1 || cap < 0)
    return fail(TT_EINVAL, "kjt_route: F in [1, 64], W in [1, 16], B >= 1");
  if ((int64_t)F * B + cap > blk_stride || cap >= INT32_MAX)
    return fail(TT_EINVAL, "kjt_route: a destination block holds F*B lengths + cap ids");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "kjt_route: ids must be int32/int64");
  if (!offsets || !num_embeddings || !block_sizes || !owners || !send || !flags)
    return fail(TT_EINVAL, "kjt_route: null pointer");
  if (!workspace || ws_bytes < tt_kjt_route_workspace_bytes(F, B, W))
    return fail(TT_ECAPACITY, "kjt_route: workspace too small");
  KjtRouteArgs a{};
  a.values = values;
  a.id_dtype = id_dtype;
  a.offsets = offsets;
  for (int f = 0; f < F; ++f) {
    if (num_embeddings[f] < 1 || num_embeddings[f] > INT32_MAX || block_sizes[f] < 0 ||
        (block_sizes[f] == 0 && (owners[f] < 0 || owners[f] >= W)) ||
        (block_sizes[f] > 0 && ceil_div(num_embeddings[f], block_sizes[f]) > W))
      return fail(TT_EINVAL, "kjt_route: bad table / block / owner (rows < 2^31, blocks cover W ranks)");
    a.num_emb[f] = num_embeddings[f];
    a.block[f] = block_sizes[f];
    a.owner[f] = owners[f];
  }
  a.F = F;
  a.W = W;
  a.B = B;
  a.cap = cap;
  a.stride = blk_stride;
  a.send = send;
  a.flags = flags;
  const int64_t n = (int64_t)W * F * B;
  char* ws = reinterpret_cast<char*>(workspace);
  a.lens = reinterpret_cast<int32_t*>(ws);
  a.base = reinterpret_cast<int32_t*>(ws + align_up((size_t)n * 4, 256));
  char* cws = ws + align_up((size_t)n * 4, 256) + align_up((size_t)(n + 1) * 4, 256);
  hipStream_t st = as_stream(stream);
  const unsigned g = (unsigned)ceil_div((int64_t)F * B, 256);
  kjt_route_count_kernel<<<dim3(g), dim3(256), 0, st>>>(a);
  int rc = check_launch("kjt_route count");
  if (rc) return rc;
  rc = tt_complete_cumsum(a.lens, n, a.base, cws, tt_complete_cumsum_workspace_bytes(n), stream);
  if (rc) return rc;
  kjt_route_place_kernel<<<dim3(g), dim3(256), 0, st>>>(a);
  return check_launch("kjt_route place");
}

size_t tt_kjt_unpack_workspace_bytes(int W, int Fr, int64_t B) {
  return tt_complete_cumsum_workspace_bytes((int64_t)W * Fr * B);
}

int tt_kjt_unpack(int W, int F, int64_t B, const int32_t* recv, int64_t blk_stride, int64_t cap, const int32_t* feats,
                  int Fr, int32_t* lengths_out, int32_t* offsets_out, int32_t* values_out, void* workspace,
                  size_t ws_bytes, void* stream) {
  if (W < 1 || W > KR_MAXW || F < 1 || F > TT_MAX_FEATURES || Fr < 1 || Fr > F || B < 1 || cap < 0)
    return fail(TT_EINVAL, "kjt_unpack: W in [1, 16], 1 <= Fr <= F <= 64");
  if ((int64_t)F * B + cap > blk_stride || (int64_t)W * Fr * B >= INT32_MAX)
    return fail(TT_EINVAL, "kjt_unpack: bad block layout");
  if (!recv || !feats || !lengths_out || !offsets_out || !values_out) return fail(TT_EINVAL, "kjt_unpack: null pointer");
  if (!workspace || ws_bytes < tt_kjt_unpack_workspace_bytes(W, Fr, B))
    return fail(TT_ECAPACITY, "kjt_unpack: workspace too small");
  KjtUnpackArgs a{};
  a.recv = recv;
  a.stride = blk_stride;
  a.FB = (int64_t)F * B;
  a.cap = cap;
  a.B = B;
  a.W = W;
  a.Fr = Fr;
  for (int k = 0; k < Fr; ++k) {
    if (feats[k] < 0 || feats[k] >= F || (k && feats[k] <= feats[k - 1]))
      return fail(TT_EINVAL, "kjt_unpack: served features must be ascending feature indices");
    a.feats[k] = feats[k];
  }
  a.lengths = lengths_out;
  a.offsets = offsets_out;
  a.values = values_out;
  hipStream_t st = as_stream(stream);
  const int64_t n = (int64_t)W * Fr * B;
  kjt_unpack_lengths_kernel<<<dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st>>>(a);
  int rc = check_launch("kjt_unpack lengths");
  if (rc) return rc;
  rc = tt_complete_cumsum(lengths_out, n, offsets_out, workspace, ws_bytes, stream);
  if (rc) return rc;
  kjt_unpack_values_kernel<<<dim3((unsigned)ceil_div((int64_t)W * cap, 256)), dim3(256), 0, st>>>(a);
  return check_launch("kjt_unpack values");
}

int tt_pooled_partials_sum(int W, int F, int64_t B, int D, const float* recv, int64_t blk_stride, int64_t ld_blk,
                           const int32_t* owner_col, float* out, int64_t ldo, void* stream) {
  PartialArgs p{};
  int rc = partial_args(W, F, B, D, owner_col, blk_stride, ld_blk, ldo, p);
  if (rc) return rc;
  if (!recv || !out) return fail(TT_EINVAL, "pooled_partials_sum: null pointer");
  const int64_t n = B * F * (D / 4);
  pooled_partials_sum_kernel<<<dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream)>>>(p, recv, out);
  return check_launch("pooled_partials_sum");
}

int tt_pooled_grad_pack(int W, int F, int64_t B, int D, const float* grad, int64_t ldg, const int32_t* owner_col,
                        float* send, int64_t blk_stride, int64_t ld_blk, void* stream) {
  PartialArgs p{};
  int rc = partial_args(W, F, B, D, owner_col, blk_stride, ld_blk, ldg, p);
  if (rc) return rc;
  if (!grad || !send) return fail(TT_EINVAL, "pooled_grad_pack: null pointer");
  const int64_t n = B * F * (D / 4);
  pooled_grad_pack_kernel<<<dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream)>>>(p, grad, send);
  return check_launch("pooled_grad_pack");
}

}  // extern "C"

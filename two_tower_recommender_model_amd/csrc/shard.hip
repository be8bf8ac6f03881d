// Sharded single-hot lookups on gfx950: input_dist / output_dist of the sharded two-tower step.
//
// Replaces, for single-hot bags, what DistributedModelParallel's ShardedEmbeddingBagCollection does
// around the local lookups (03_model_training.py:798-815, torchrec input_dist: KJT permute +
// block_bucketize_sparse_features + lengths/values all-to-all; output_dist: pooled all-to-all
// (table-wise) or reduce-scatter (row-wise)) with an id-level exchange whose buffers have a FIXED
// size, so the whole sharded step is one HIP graph with RCCL collectives inside:
//
//   route (requester)   lookup (f, b): id 0 dropped, row = id mod N_f (transform_to_torchrec_batch,
//                       03:356-365); owner d = row / block (row-wise, torchrec block_bucketize
//                       semantics: block = ceil(N / W)) or the table's rank (table-wise); local
//                       row = row - d * block. Lookups are filed into segment (d, f) in ascending
//                       bag order (slot k), capacity C per segment; send[d] = {count(d, f) for f,
//                       then the F segments of C keys (f << 40 | local row)}; pos[f][b] =
//                       (d * F + f) * C + k, the row of this lookup in the returned-rows buffer
//                       (-1: dropped). More than C lookups for one segment set the sticky overflow
//                       flag (the step's results are then invalid: the host checks it).
//   all-to-all          send -> recv, W equal blocks of F + F * C int64.
//   gather (owner)      slot i = (s * F + f) * C + k < count: rows_out[i] = table_f[local row]; the
//                       slot is also inserted into the dedup table (dedup.h) as lookup i, so the
//                       owner's fused row-wise Adagrad after the gradient all-to-all reads it.
//   all-to-all          rows_out -> rows_in ([W * F * C][D]); T1 reads rows_in[pos] (tower.hip,
//                       indexed mode) and writes its input gradient to grad_out[pos]; the reverse
//                       all-to-all takes grad_out to the owners, whose gradient row of lookup i is
//                       row i: tt_dedup_rowwise_adagrad(flat) sums a row's lookups in ascending i =
//                       (source rank, bag) order — the order of the single-process batch
//                       concatenated over ranks.
#include "shard.h"

namespace tt {

__global__ void __launch_bounds__(RT_BLOCK) shard_route_count_kernel(RouteArgs a) {
  __shared__ int wc[RT_BLOCK / 64][RT_MAXW];
  route_count_block(a, (int)blockIdx.x, (int)blockIdx.y, wc);
}

template <bool SEGS>
__global__ void __launch_bounds__(RT_BLOCK) shard_route_place_kernel(RouteArgs a) {
  __shared__ int base[RT_MAXW];
  __shared__ int wc[RT_BLOCK / 64][RT_MAXW];
  route_place_block<SEGS>(a, (int)blockIdx.x, (int)blockIdx.y, base, wc);
}

struct GatherArgs {
  const float* weights;
  tt_table_meta_t tables[TT_MAX_TABLES];
  int T;
  int F;
  int W;
  int64_t C;
  int D;
  const int64_t* recv;  // [W][F + F * C]
  float* rows_out;      // [W * F * C][D] fp32, or bf16 when out_bf16
  int out_bf16;
  DedupWs dd;
  int dd_on;
  int32_t* bad;         // sticky: a received key outside the local shard
};

// owner side: a half-wave per received slot: copy the row, file the lookup for the Adagrad update
__global__ void __launch_bounds__(256) shard_gather_rows_kernel(GatherArgs a) {
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int64_t n = (int64_t)a.W * a.F * a.C;
  const int64_t i = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  if (i >= n) return;
  const int64_t fc = (int64_t)a.F * a.C;
  const int64_t s = i / fc, f = (i / a.C) % a.F, k = i % a.C;
  const int64_t* blk = a.recv + s * (a.F + fc);
  const int64_t cnt = blk[f];
  uint64_t key = DD_EMPTY;
  const float* src = nullptr;
  if (k < cnt) {
    key = (uint64_t)blk[a.F + f * a.C + k];
    const int t = (int)(key >> DD_TABLE_SHIFT);
    const int64_t r = (int64_t)(key & ((1ull << DD_TABLE_SHIFT) - 1));
    if (t < a.T && r < a.tables[t].num_rows && a.tables[t].dim == a.D) {
      src = a.weights + a.tables[t].weight_offset + r * a.D;
    } else {
      key = DD_EMPTY;
      if (hl == 0) atomicOr(a.bad, 1);
    }
  }
  DdPend pend;
  if (a.dd_on && hl == 0) dd_insert_begin(a.dd, key, (int32_t)i, pend);
  if (src && a.out_bf16) {  // the rows T1 rounds to bf16 anyway: half the all-to-all bytes
    __bf16* dst = reinterpret_cast<__bf16*>(a.rows_out) + i * a.D;
    for (int c = hl * 4; c < a.D; c += 128) {
      const f32x4v v = *reinterpret_cast<const f32x4v*>(src + c);
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4v;
      bf16x4v o;
      o[0] = (__bf16)v[0];
      o[1] = (__bf16)v[1];
      o[2] = (__bf16)v[2];
      o[3] = (__bf16)v[3];
      *reinterpret_cast<bf16x4v*>(dst + c) = o;
    }
  } else if (src) {
    float* dst = a.rows_out + i * a.D;
    for (int c = hl * 4; c < a.D; c += 128)
      *reinterpret_cast<f32x4v*>(dst + c) = *reinterpret_cast<const f32x4v*>(src + c);
  }
  if (a.dd_on && hl == 0) dd_insert_finish(a.dd, pend, (int32_t)i);
}


__global__ void __launch_bounds__(256) shard_gather_segs_kernel(GatherSegArgs a) { shard_gather_block(a, (int)blockIdx.x); }

// host: the owner-side gather's arguments (tt_shard_gather_segs_bf16 and the pipelined step's
// combined launch in csrc/tower.hip)
int gather_segs_args(const float* weights, const tt_table_meta_t* tables, int T, int F, int W, const int64_t* recv,
                     int64_t block_i64, int64_t counts_i64, const int64_t* seg_off, int64_t slots, void* rows_out,
                     int64_t out_stride, int32_t* bad, void* dedup_ws, size_t dedup_ws_bytes,
                     int64_t dedup_max_lookups, GatherSegArgs& a) {
  if (T < 1 || T > TT_MAX_TABLES || F < 1 || F > TT_MAX_FEATURES || F > T || W < 1 || slots < 0 ||
      (int64_t)W * slots >= (1ll << 31))
    return fail(TT_EINVAL, "shard_gather_segs: bad sizes");
  if (!weights || !tables || !recv || !rows_out || !bad || !seg_off)
    return fail(TT_EINVAL, "shard_gather_segs: null pointer");
  a = GatherSegArgs{};
  a.D = tables[0].dim;
  for (int t = 0; t < T; ++t) {
    if (tables[t].dim != a.D) return fail(TT_EINVAL, "shard_gather_segs: tables must share one dim");
    if (tables[t].weight_offset % 4) return fail(TT_EINVAL, "shard_gather_segs: rows must be 16-B aligned");
    a.tables[t] = tables[t];
  }
  if (a.D % 4 || (reinterpret_cast<uintptr_t>(weights) & 15) || (reinterpret_cast<uintptr_t>(rows_out) & 7))
    return fail(TT_EINVAL, "shard_gather_segs: D % 4 == 0 and aligned buffers required");
  for (int f = 0; f <= F; ++f) {
    a.seg_off[f] = f < F ? seg_off[f] : slots;
    if (a.seg_off[f] < 0 || a.seg_off[f] > slots || (f && a.seg_off[f] < a.seg_off[f - 1]))
      return fail(TT_EINVAL, "shard_gather_segs: segment offsets must ascend within [0, slots]");
  }
  if (block_i64 < counts_i64 + F + slots || counts_i64 < 0) return fail(TT_EINVAL, "shard_gather_segs: bad block layout");
  const int64_t n = (int64_t)W * slots;
  if (n > INT32_MAX) return fail(TT_EINVAL, "shard_gather_segs: too many slots");
  a.weights = weights;
  a.T = T;
  a.F = F;
  a.W = W;
  a.S = slots;
  if (out_stride < slots) return fail(TT_EINVAL, "shard_gather_segs: out_stride < slots");
  a.out_stride = out_stride;
  a.blk64 = block_i64;
  a.cnt64 = counts_i64;
  a.recv = recv;
  a.rows_out = reinterpret_cast<__bf16*>(rows_out);
  a.bad = bad;
  if (dedup_ws) {
    if (dedup_max_lookups < n || dedup_max_lookups >= (int64_t)DD_CNT_MASK ||
        dedup_ws_bytes < dedup_layout(nullptr, dedup_max_lookups, nullptr) ||
        (reinterpret_cast<uintptr_t>(dedup_ws) & 63))
      return fail(TT_ECAPACITY, "shard_gather_segs: dedup workspace too small / misaligned");
    dedup_layout(dedup_ws, dedup_max_lookups, &a.dd);
    a.dd_on = 1;
  }
  return TT_OK;
}

// Admission counts of one KJT batch (tt_kjt_admit, the N > 1 drop-in): the bags longer than one id,
// the values outside [0, N), and the ids each (owner, feature) segment would receive. Workgroups
// [0, nbw) check 2048 bags each (lengths from the offsets), the rest 2048 values each; every
// workgroup reduces in LDS and adds to the zeroed output with one atomic per word.
constexpr int ADM_PT = 8;  // bags / values per thread
struct AdmArgs {
  int F, W, id_dtype, nbw;
  int64_t B, nnz;
  const void* values;
  const int32_t* offsets;
  int32_t* out;
  int64_t ne[TT_MAX_FEATURES], blk[TT_MAX_FEATURES];
  int32_t own[TT_MAX_FEATURES];
};
__global__ void __launch_bounds__(256) kjt_admit_kernel(AdmArgs a) {
  const int F = a.F, W = a.W, id_dtype = a.id_dtype, nbw = a.nbw;
  const int64_t B = a.B, nnz = a.nnz;
  const void* values = a.values;
  const int32_t* offsets = a.offsets;
  int32_t* out = a.out;
  __shared__ int cnt[TT_PEER_MAXW * TT_MAX_FEATURES];
  __shared__ int flags[2];
  const int tid = threadIdx.x;
  for (int u = tid; u < W * F; u += 256) cnt[u] = 0;
  if (tid < 2) flags[tid] = 0;
  __syncthreads();
  int multi = 0, bad = 0;
  if ((int)blockIdx.x < nbw) {
    const int64_t nb = (int64_t)F * B;
#pragma unroll
    for (int k = 0; k < ADM_PT; ++k) {
      const int64_t b = ((int64_t)blockIdx.x * ADM_PT + k) * 256 + tid;
      if (b < nb && offsets[b + 1] - offsets[b] > 1) multi = 1;
    }
  } else {
    // feature boundaries: a uniform loop over the F segment starts (scalar loads)
#pragma unroll
    for (int k = 0; k < ADM_PT; ++k) {
      const int64_t i = ((int64_t)(blockIdx.x - nbw) * ADM_PT + k) * 256 + tid;
      if (i >= nnz) break;
      int f = 0;
      int64_t nef = a.ne[0], bf = a.blk[0];
      int of = a.own[0];
      for (int q = 1; q < F; ++q)
        if (i >= (int64_t)offsets[(int64_t)q * B]) {
          f = q;
          nef = a.ne[q];
          bf = a.blk[q];
          of = a.own[q];
        }
      const int64_t id = load_id(values, id_dtype, i);
      if (id < 0 || id >= nef) {
        bad = 1;
        continue;
      }
      const int d = bf > 0 ? (int)udiv64(id, bf) : of;
      if (d >= 0 && d < W) atomicAdd(&cnt[d * F + f], 1);
    }
  }
  if (multi) flags[0] = 1;
  if (bad) flags[1] = 2;
  __syncthreads();
  if (tid < 2 && flags[tid]) atomicOr(&out[tid], flags[tid]);
  for (int u = tid; u < W * F; u += 256)
    if (cnt[u]) atomicAdd(&out[2 + u], cnt[u]);
}

}  // namespace tt

using namespace tt;

extern "C" {

size_t tt_shard_route_workspace_bytes(int F, int64_t B) {
  const int64_t nblk = ceil_div(std::max<int64_t>(B, 1), RT_BLOCK);
  return align_up(sizeof(int64_t) * (size_t)F * (size_t)std::max<int64_t>(B, 1), 256) +
         align_up(sizeof(int32_t) * (size_t)F * (size_t)nblk * RT_MAXW, 256);
}

int tt_shard_route_cols(int F, int64_t B, const void* const* cols, int id_dtype, const int64_t* num_embeddings,
                        const int64_t* block_sizes, const int32_t* owners, int W, int64_t seg_capacity,
                        int64_t* send, int32_t* pos, int32_t* overflow, void* workspace, size_t ws_bytes,
                        void* stream) {
  if (F < 1 || F > TT_MAX_FEATURES) return fail(TT_EINVAL, "shard_route: feature count out of range");
  if (W < 1 || W > RT_MAXW) return fail(TT_EINVAL, "shard_route: 1..16 ranks supported");
  if (B < 0 || seg_capacity < 1 || seg_capacity > INT32_MAX / ((int64_t)W * F))
    return fail(TT_EINVAL, "shard_route: bad batch / segment capacity");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "shard_route: ids must be int32/int64");
  if (!cols || !num_embeddings || !block_sizes || !owners || !send || !pos || !overflow)
    return fail(TT_EINVAL, "shard_route: null pointer");
  if (!workspace || ws_bytes < tt_shard_route_workspace_bytes(F, B))
    return fail(TT_ECAPACITY, "shard_route: workspace too small");
  RouteArgs a{};
  for (int f = 0; f < F; ++f) {
    if (!cols[f] || num_embeddings[f] < 1) return fail(TT_EINVAL, "shard_route: bad column");
    if (block_sizes[f] < 0 || (block_sizes[f] == 0 && (owners[f] < 0 || owners[f] >= W)))
      return fail(TT_EINVAL, "shard_route: bad sharding of a feature");
    if (block_sizes[f] > 0 && (num_embeddings[f] + block_sizes[f] - 1) / block_sizes[f] > W)
      return fail(TT_EINVAL, "shard_route: row blocks exceed the rank count");
    if ((block_sizes[f] > 0 ? block_sizes[f] : num_embeddings[f]) >= (1ll << DD_TABLE_SHIFT))
      return fail(TT_EINVAL, "shard_route: local rows >= 2^40");
    a.col[f] = cols[f];
    a.num_emb[f] = num_embeddings[f];
    a.block[f] = block_sizes[f];
    a.owner[f] = owners[f];
  }
  if (B == 0) return TT_OK;
  a.id_dtype = id_dtype;
  a.F = F;
  a.W = W;
  a.B = B;
  a.C = seg_capacity;
  a.nblk = (int)ceil_div(B, RT_BLOCK);
  a.send = send;
  a.pos = pos;
  a.overflow = overflow;
  char* ws = reinterpret_cast<char*>(workspace);
  a.dl = reinterpret_cast<int64_t*>(ws);
  a.cnt = reinterpret_cast<int32_t*>(ws + align_up(sizeof(int64_t) * (size_t)F * (size_t)B, 256));
  const dim3 grid(a.nblk, F);
  shard_route_count_kernel<<<grid, dim3(RT_BLOCK), 0, as_stream(stream)>>>(a);
  shard_route_place_kernel<false><<<grid, dim3(RT_BLOCK), 0, as_stream(stream)>>>(a);
  return check_launch("shard_route");
}

static int gather_rows(const float* weights, const tt_table_meta_t* tables, int T, int F, int W,
                       int64_t seg_capacity, const int64_t* recv, float* rows_out, int32_t* bad, void* dedup_ws,
                       size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream, int out_bf16) {
  if (T < 1 || T > TT_MAX_TABLES || F < 1 || F > TT_MAX_FEATURES || W < 1 || seg_capacity < 1)
    return fail(TT_EINVAL, "shard_gather_rows: bad sizes");
  if (!weights || !tables || !recv || !rows_out || !bad) return fail(TT_EINVAL, "shard_gather_rows: null pointer");
  GatherArgs a{};
  a.D = tables[0].dim;
  for (int t = 0; t < T; ++t) {
    if (tables[t].dim != a.D) return fail(TT_EINVAL, "shard_gather_rows: tables must share one dim");
    if (tables[t].weight_offset % 4) return fail(TT_EINVAL, "shard_gather_rows: rows must be 16-B aligned");
    a.tables[t] = tables[t];
  }
  if (a.D % 4 || (reinterpret_cast<uintptr_t>(weights) & 15) || (reinterpret_cast<uintptr_t>(rows_out) & 15))
    return fail(TT_EINVAL, "shard_gather_rows: D % 4 == 0 and 16-B aligned buffers required");
  const int64_t n = (int64_t)W * F * seg_capacity;
  if (n > INT32_MAX) return fail(TT_EINVAL, "shard_gather_rows: too many slots");
  a.weights = weights;
  a.T = T;
  a.F = F;
  a.W = W;
  a.C = seg_capacity;
  a.recv = recv;
  a.rows_out = rows_out;
  a.out_bf16 = out_bf16;
  a.bad = bad;
  if (dedup_ws) {
    if (dedup_max_lookups < n || dedup_max_lookups >= (int64_t)DD_CNT_MASK ||
        dedup_ws_bytes < dedup_layout(nullptr, dedup_max_lookups, nullptr) ||
        (reinterpret_cast<uintptr_t>(dedup_ws) & 63))
      return fail(TT_ECAPACITY, "shard_gather_rows: dedup workspace too small / misaligned");
    dedup_layout(dedup_ws, dedup_max_lookups, &a.dd);
    a.dd_on = 1;
  }
  const int64_t grid = ceil_div(n, 8);
  shard_gather_rows_kernel<<<dim3((unsigned)grid), dim3(256), 0, as_stream(stream)>>>(a);
  return check_launch("shard_gather_rows");
}

int tt_shard_gather_rows(const float* weights, const tt_table_meta_t* tables, int T, int F, int W,
                         int64_t seg_capacity, const int64_t* recv, float* rows_out, int32_t* bad, void* dedup_ws,
                         size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream) {
  return gather_rows(weights, tables, T, F, W, seg_capacity, recv, rows_out, bad, dedup_ws, dedup_ws_bytes,
                     dedup_max_lookups, stream, 0);
}

int tt_shard_gather_rows_bf16(const float* weights, const tt_table_meta_t* tables, int T, int F, int W,
                              int64_t seg_capacity, const int64_t* recv, void* rows_out, int32_t* bad, void* dedup_ws,
                              size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream) {
  return gather_rows(weights, tables, T, F, W, seg_capacity, recv, reinterpret_cast<float*>(rows_out), bad, dedup_ws,
                     dedup_ws_bytes, dedup_max_lookups, stream, 1);
}

int tt_shard_route_segs(int F, int64_t B, const void* const* cols, int id_dtype, const int64_t* num_embeddings,
                        const int64_t* block_sizes, const int32_t* owners, int W, const tt_shard_seg_t* segs,
                        int64_t* send, int32_t* pos_in, int32_t* pos_out, int32_t* overflow, void* workspace,
                        size_t ws_bytes, void* stream) {
  if (F < 1 || F > TT_MAX_FEATURES) return fail(TT_EINVAL, "shard_route_segs: feature count out of range");
  if (W < 1 || W > RT_MAXW) return fail(TT_EINVAL, "shard_route_segs: 1..16 ranks supported");
  if (B < 0) return fail(TT_EINVAL, "shard_route_segs: negative batch");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "shard_route_segs: ids must be int32/int64");
  if (!cols || !num_embeddings || !block_sizes || !owners || !segs || !send || !pos_in || !pos_out || !overflow)
    return fail(TT_EINVAL, "shard_route_segs: null pointer");
  if (!workspace || ws_bytes < tt_shard_route_workspace_bytes(F, B))
    return fail(TT_ECAPACITY, "shard_route_segs: workspace too small");
  RouteArgs a{};
  for (int f = 0; f < F; ++f) {
    if (!cols[f] || num_embeddings[f] < 1) return fail(TT_EINVAL, "shard_route_segs: bad column");
    if (block_sizes[f] < 0 || (block_sizes[f] == 0 && (owners[f] < 0 || owners[f] >= W)))
      return fail(TT_EINVAL, "shard_route_segs: bad sharding of a feature");
    if (block_sizes[f] > 0 && (num_embeddings[f] + block_sizes[f] - 1) / block_sizes[f] > W)
      return fail(TT_EINVAL, "shard_route_segs: row blocks exceed the rank count");
    if ((block_sizes[f] > 0 ? block_sizes[f] : num_embeddings[f]) >= (1ll << DD_TABLE_SHIFT))
      return fail(TT_EINVAL, "shard_route_segs: local rows >= 2^40");
    a.col[f] = cols[f];
    a.num_emb[f] = num_embeddings[f];
    a.block[f] = block_sizes[f];
    a.owner[f] = owners[f];
  }
  if (B == 0) return TT_OK;
  a.id_dtype = id_dtype;
  a.F = F;
  a.W = W;
  a.B = B;
  a.C = 1;
  a.nblk = (int)ceil_div(B, RT_BLOCK);
  a.send = send;
  a.pos = pos_in;
  a.pos_out = pos_out;
  a.segs = segs;
  a.overflow = overflow;
  char* ws = reinterpret_cast<char*>(workspace);
  a.dl = reinterpret_cast<int64_t*>(ws);
  a.cnt = reinterpret_cast<int32_t*>(ws + align_up(sizeof(int64_t) * (size_t)F * (size_t)B, 256));
  const dim3 grid(a.nblk, F);
  shard_route_count_kernel<<<grid, dim3(RT_BLOCK), 0, as_stream(stream)>>>(a);
  shard_route_place_kernel<true><<<grid, dim3(RT_BLOCK), 0, as_stream(stream)>>>(a);
  return check_launch("shard_route_segs");
}

int tt_shard_gather_segs_bf16(const float* weights, const tt_table_meta_t* tables, int T, int F, int W,
                              const int64_t* recv, int64_t block_i64, int64_t counts_i64, const int64_t* seg_off,
                              int64_t slots, void* rows_out, int64_t out_stride, int32_t* bad, void* dedup_ws,
                              size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream) {
  GatherSegArgs a{};
  int rc = gather_segs_args(weights, tables, T, F, W, recv, block_i64, counts_i64, seg_off, slots, rows_out, out_stride,
                            bad, dedup_ws, dedup_ws_bytes, dedup_max_lookups, a);
  if (rc) return rc;
  const int64_t n = (int64_t)W * slots;
  if (n == 0) return TT_OK;
  shard_gather_segs_kernel<<<dim3((unsigned)ceil_div(ceil_div(n, GS_SL), 8)), dim3(256), 0, as_stream(stream)>>>(a);
  return check_launch("shard_gather_segs");
}

int tt_kjt_admit(int F, int64_t B, const void* values, int id_dtype, int64_t nnz, const int32_t* offsets,
                 const int64_t* num_embeddings, const int64_t* block_sizes, const int32_t* owners, int W, int32_t* out,
                 void* stream) {
  if (F < 1 || F > TT_MAX_FEATURES || B < 1 || W < 1 || W > TT_PEER_MAXW || nnz < 0)
    return fail(TT_EINVAL, "kjt_admit: 1 <= F <= 64, B >= 1, 1 <= W <= 16, nnz >= 0");
  if (!offsets || !num_embeddings || !block_sizes || !owners || !out || (nnz && !values))
    return fail(TT_EINVAL, "kjt_admit: null pointer");
  if (nnz && id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "kjt_admit: ids must be int32/int64");
  AdmArgs a{};
  a.F = F;
  a.W = W;
  a.id_dtype = id_dtype;
  a.B = B;
  a.nnz = nnz;
  a.values = values;
  a.offsets = offsets;
  a.out = out;
  for (int f = 0; f < F; ++f) {
    if (num_embeddings[f] < 1 || block_sizes[f] < 0 || (block_sizes[f] == 0 && (owners[f] < 0 || owners[f] >= W)))
      return fail(TT_EINVAL, "kjt_admit: bad table size or sharding of a feature");
    a.ne[f] = num_embeddings[f];
    a.blk[f] = block_sizes[f];
    a.own[f] = owners[f];
  }
  hipError_t e = hipMemsetAsync(out, 0, sizeof(int32_t) * (size_t)(2 + W * F), as_stream(stream));
  if (e != hipSuccess) return fail((int)e, std::string("kjt_admit: ") + hipGetErrorString(e));
  const int64_t per = 256 * ADM_PT;
  const int64_t nbw = ceil_div((int64_t)F * B, per), nvw = ceil_div(nnz, per);
  if (nbw + nvw > INT32_MAX) return fail(TT_EINVAL, "kjt_admit: grid too large");
  a.nbw = (int)nbw;
  kjt_admit_kernel<<<dim3((unsigned)(nbw + nvw)), dim3(256), 0, as_stream(stream)>>>(a);
  return check_launch("kjt_admit");
}

}  // extern "C"

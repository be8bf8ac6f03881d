// KeyedJaggedTensor kernels: the vectorised KJT builder (replaces the reference's per-element host
// loop, 03_model_training.py:356-371), complete-cumsum offsets, key permute and row-wise
// block-bucketize. All integer work: HBM/latency bound, one pass each, coalesced, no MFMA.
//
// Scans use a two-launch reduce-then-scan over 1024-element tiles (no inter-workgroup hand-off
// inside a launch, so nothing depends on dispatch order or XCD placement).
#include "tt_common.h"

namespace tt {

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 4;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;  // 1024 elements per workgroup

// Block-wide exclusive scan of one int per thread (256 threads = 4 waves). Returns the exclusive
// prefix of this thread; *total receives the block total.
__device__ __forceinline__ int block_exclusive_scan(int v, int* lds /*[4]*/, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) lds[wid] = incl;
  __syncthreads();
  int wbase = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < SCAN_THREADS / 64; ++w) {
    int s = lds[w];
    if (w < wid) wbase += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return wbase + incl - v;
}

// Sum of bsum[0 .. nb) computed by the whole block (nb = number of preceding tiles).
__device__ __forceinline__ int block_prefix_of_tiles(const int* bsum, int nb, int* lds) {
  int s = 0;
  for (int i = threadIdx.x; i < nb; i += SCAN_THREADS) s += bsum[i];
  s = (int)wave_sum_i(s);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = s;
  __syncthreads();
  int tot = 0;
#pragma unroll
  for (int w = 0; w < SCAN_THREADS / 64; ++w) tot += lds[w];
  __syncthreads();
  return tot;
}

// ---- complete cumsum --------------------------------------------------------------------------

__global__ void __launch_bounds__(SCAN_THREADS) cumsum_reduce_kernel(const int32_t* __restrict__ x,
                                                                     int64_t n, int* __restrict__ bsum) {
  __shared__ int lds[4];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  int s = 0;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    int64_t i = base + threadIdx.x * SCAN_ITEMS + j;
    if (i < n) s += x[i];
  }
  s = wave_sum_i(s);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = lds[0] + lds[1] + lds[2] + lds[3];
}

__global__ void __launch_bounds__(SCAN_THREADS) cumsum_scan_kernel(const int32_t* __restrict__ x,
                                                                   int64_t n, const int* __restrict__ bsum,
                                                                   int32_t* __restrict__ out) {
  __shared__ int lds[4];
  __shared__ int lds2[4];
  const int prefix = block_prefix_of_tiles(bsum, blockIdx.x, lds2);
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  int v[SCAN_ITEMS];
  int local = 0;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    v[j] = (base + j < n) ? x[base + j] : 0;
    local += v[j];
  }
  int total;
  int excl = block_exclusive_scan(local, lds, &total) + prefix;
  if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = 0;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    excl += v[j];
    if (base + j < n) out[base + j + 1] = excl;
  }
}

static int launch_cumsum(const int32_t* x, int64_t n, int32_t* out, int* bsum, hipStream_t st) {
  if (n == 0) {
    return hipMemsetAsync(out, 0, sizeof(int32_t), st) == hipSuccess
               ? TT_OK
               : fail(TT_EINVAL, "hipMemsetAsync failed");
  }
  const int64_t nb = ceil_div(n, SCAN_TILE);
  cumsum_reduce_kernel<<<dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st>>>(x, n, bsum);
  cumsum_scan_kernel<<<dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st>>>(x, n, bsum, out);
  return check_launch("complete_cumsum");
}

// ---- KJT builder: mod + drop-zero + compaction (03_model_training.py:356-371) ------------------

struct KjtCols {
  const void* col[TT_MAX_FEATURES];
  int64_t num_emb[TT_MAX_FEATURES];
};

__device__ __forceinline__ int64_t py_mod(int64_t a, int64_t n) {
  int64_t r = a % n;  // C remainder: sign of a
  return (r != 0 && ((r < 0) != (n < 0))) ? r + n : r;  // Python/torch floor-mod: sign of n
}

__global__ void __launch_bounds__(SCAN_THREADS) kjt_flags_kernel(KjtCols cols, int id_dtype, int F,
                                                                 int64_t B, int32_t* __restrict__ lengths,
                                                                 int* __restrict__ bsum,
                                                                 int64_t* __restrict__ lpk) {
  __shared__ int lds[4];
  const int64_t n = (int64_t)F * B;
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  if (lpk && blockIdx.x == 0 && threadIdx.x < F) lpk[threadIdx.x] = 0;
  int s = 0;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    // element-major over threads so consecutive lanes read consecutive ids (coalesced)
    int64_t i = base + j * SCAN_THREADS + threadIdx.x;
    if (i < n) {
      const int f = (int)(i / B);
      const int64_t b = i - (int64_t)f * B;
      const int64_t id = load_id(cols.col[f], id_dtype, b);
      const int flag = id != 0;
      lengths[i] = flag;
      s += flag;
    }
  }
  s = wave_sum_i(s);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = lds[0] + lds[1] + lds[2] + lds[3];
}

__global__ void __launch_bounds__(SCAN_THREADS) kjt_scatter_kernel(
    KjtCols cols, int id_dtype, int F, int64_t B, const int32_t* __restrict__ lengths,
    const int* __restrict__ bsum, void* __restrict__ values, int32_t* __restrict__ offsets,
    int64_t* __restrict__ lpk) {
  __shared__ int lds[4];
  __shared__ int lds2[4];
  __shared__ int key_cnt[TT_MAX_FEATURES];
  const int64_t n = (int64_t)F * B;
  const int prefix = block_prefix_of_tiles(bsum, blockIdx.x, lds2);
  if (lpk && threadIdx.x < TT_MAX_FEATURES) key_cnt[threadIdx.x] = 0;
  // this pass needs the tile in thread-contiguous order for the scan
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  int v[SCAN_ITEMS];
  int local = 0;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    v[j] = (base + j < n) ? lengths[base + j] : 0;
    local += v[j];
  }
  int total;
  int excl = block_exclusive_scan(local, lds, &total) + prefix;
  if (blockIdx.x == 0 && threadIdx.x == 0) offsets[0] = 0;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    const int64_t i = base + j;
    if (i < n) {
      if (v[j]) {
        const int f = (int)(i / B);
        const int64_t b = i - (int64_t)f * B;
        const int64_t id = load_id(cols.col[f], id_dtype, b);
        const int64_t m = py_mod(id, cols.num_emb[f]);
        if (id_dtype == TT_I64)
          reinterpret_cast<int64_t*>(values)[excl] = m;
        else
          reinterpret_cast<int32_t*>(values)[excl] = (int32_t)m;
        if (lpk) atomicAdd(&key_cnt[f], 1);
      }
      excl += v[j];
      offsets[i + 1] = excl;
    }
  }
  if (lpk) {
    __syncthreads();
    if (threadIdx.x < F && key_cnt[threadIdx.x] != 0)
      atomicAdd(reinterpret_cast<unsigned long long*>(&lpk[threadIdx.x]),
                (unsigned long long)key_cnt[threadIdx.x]);
  }
}

}  // namespace tt

using namespace tt;

extern "C" {

size_t tt_complete_cumsum_workspace_bytes(int64_t n) {
  return align_up((size_t)std::max<int64_t>(1, ceil_div(n, SCAN_TILE)) * sizeof(int), 256);
}

int tt_complete_cumsum(const int32_t* lengths, int64_t n, int32_t* offsets, void* workspace,
                       size_t ws_bytes, void* stream) {
  if (n < 0 || !offsets || (n > 0 && !lengths)) return fail(TT_EINVAL, "complete_cumsum: bad args");
  if (n > INT32_MAX) return fail(TT_EINVAL, "complete_cumsum: n exceeds int32 offsets");
  if (ws_bytes < tt_complete_cumsum_workspace_bytes(n) || !workspace)
    return fail(TT_ECAPACITY, "complete_cumsum: workspace too small");
  return launch_cumsum(lengths, n, offsets, reinterpret_cast<int*>(workspace), as_stream(stream));
}

size_t tt_kjt_build_workspace_bytes(int64_t n) { return tt_complete_cumsum_workspace_bytes(n); }

int tt_kjt_build_mod_dropzero(int F, int64_t B, const void* const* cols, int id_dtype,
                              const int64_t* num_embeddings, void* values_out,
                              int32_t* lengths_out, int32_t* offsets_out,
                              int64_t* length_per_key_out, void* workspace, size_t ws_bytes,
                              void* stream) {
  if (F < 1 || F > TT_MAX_FEATURES) return fail(TT_EINVAL, "kjt_build: F out of range [1,64]");
  if (B < 0 || (int64_t)F * B > INT32_MAX) return fail(TT_EINVAL, "kjt_build: bad B");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "kjt_build: ids must be int32/int64");
  if (!cols || !num_embeddings || !lengths_out || !offsets_out || (B > 0 && !values_out))
    return fail(TT_EINVAL, "kjt_build: null pointer");
  const int64_t n = (int64_t)F * B;
  if (ws_bytes < tt_kjt_build_workspace_bytes(n) || !workspace)
    return fail(TT_ECAPACITY, "kjt_build: workspace too small");
  KjtCols c{};
  for (int f = 0; f < F; ++f) {
    if (num_embeddings[f] < 1) return fail(TT_EINVAL, "kjt_build: num_embeddings must be >= 1");
    if (B > 0 && !cols[f]) return fail(TT_EINVAL, "kjt_build: null column");
    c.col[f] = cols[f];
    c.num_emb[f] = num_embeddings[f];
  }
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    if (hipMemsetAsync(offsets_out, 0, sizeof(int32_t), st) != hipSuccess)
      return fail(TT_EINVAL, "kjt_build: memset failed");
    if (length_per_key_out &&
        hipMemsetAsync(length_per_key_out, 0, sizeof(int64_t) * F, st) != hipSuccess)
      return fail(TT_EINVAL, "kjt_build: memset failed");
    return TT_OK;
  }
  const int64_t nb = ceil_div(n, SCAN_TILE);
  int* bsum = reinterpret_cast<int*>(workspace);
  kjt_flags_kernel<<<dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st>>>(c, id_dtype, F, B, lengths_out,
                                                                      bsum, length_per_key_out);
  kjt_scatter_kernel<<<dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st>>>(
      c, id_dtype, F, B, lengths_out, bsum, values_out, offsets_out, length_per_key_out);
  return check_launch("kjt_build_mod_dropzero");
}

// ---- single-hot KJT -> id columns (the drop-in pipeline's input to the fused step) -----------
// For key f, bag b of a KJT whose bags hold at most one id: col_f[b] = 0 for an empty bag (the
// fused kernels' "dropped id"), else the bag's value v, or N_f for v == 0 (py_mod(N_f, N_f) = row 0:
// the fused kernels read row py_mod(id, N) for every non-zero id). A bag with more than one id or
// a value outside [0, N_f) sets bit 0 / bit 1 of the sticky err word (TorchRec's EBC would index
// out of range there); its column entry is 0.
}  // extern "C"

namespace tt {
__global__ void __launch_bounds__(256) kjt_single_hot_cols_kernel(KjtCols c, int id_dtype, int F, int64_t B,
                                                                  const void* __restrict__ values,
                                                                  const int32_t* __restrict__ offsets,
                                                                  int32_t* __restrict__ err, const void* labels,
                                                                  int label_dtype, int32_t* __restrict__ labels_out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)F * B) return;
  if (labels_out && i < B)
    labels_out[i] = label_dtype == TT_I64 ? (int32_t)reinterpret_cast<const int64_t*>(labels)[i]
                                          : reinterpret_cast<const int32_t*>(labels)[i];
  const int f = (int)(i / B);
  const int64_t b = i - (int64_t)f * B;
  const int32_t o0 = offsets[i], o1 = offsets[i + 1];
  const int64_t N = c.num_emb[f];
  int64_t out = 0;
  int bad = 0;
  if (o1 - o0 == 1) {
    const int64_t v = id_dtype == TT_I64 ? reinterpret_cast<const int64_t*>(values)[o0]
                                         : (int64_t)reinterpret_cast<const int32_t*>(values)[o0];
    if (v < 0 || v >= N) bad = 2;
    else out = v == 0 ? N : v;
  } else if (o1 - o0 != 0) {
    bad = 1;
  }
  if (bad) atomicOr(err, bad);
  if (id_dtype == TT_I64) reinterpret_cast<int64_t*>(const_cast<void*>(c.col[f]))[b] = out;
  else reinterpret_cast<int32_t*>(const_cast<void*>(c.col[f]))[b] = (int32_t)out;
}
}  // namespace tt

extern "C" {
int tt_kjt_single_hot_cols(int F, int64_t B, const void* values, int id_dtype, const int32_t* offsets,
                           const int64_t* num_embeddings, void* const* cols_out, int32_t* err, const void* labels,
                           int label_dtype, int32_t* labels_out, void* stream) {
  if (labels_out && (!labels || (label_dtype != TT_I32 && label_dtype != TT_I64)))
    return fail(TT_EINVAL, "kjt_single_hot_cols: labels must be int32/int64");
  if (F < 1 || F > TT_MAX_FEATURES) return fail(TT_EINVAL, "kjt_single_hot_cols: F out of range [1,64]");
  if (B < 1 || (int64_t)F * B > INT32_MAX) return fail(TT_EINVAL, "kjt_single_hot_cols: bad B");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "kjt_single_hot_cols: ids must be int32/int64");
  if (!offsets || !num_embeddings || !cols_out || !err) return fail(TT_EINVAL, "kjt_single_hot_cols: null pointer");
  KjtCols c{};
  for (int f = 0; f < F; ++f) {
    if (num_embeddings[f] < 1 || (id_dtype == TT_I32 && num_embeddings[f] > INT32_MAX))
      return fail(TT_EINVAL, "kjt_single_hot_cols: num_embeddings out of range for the id dtype");
    if (!cols_out[f]) return fail(TT_EINVAL, "kjt_single_hot_cols: null column");
    c.col[f] = cols_out[f];
    c.num_emb[f] = num_embeddings[f];
  }
  const int64_t n = (int64_t)F * B;
  kjt_single_hot_cols_kernel<<<dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, as_stream(stream)>>>(
      c, id_dtype, F, B, values, offsets, err, labels, label_dtype, labels_out);
  return check_launch("kjt_single_hot_cols");
}
}  // extern "C"

// ---- permute_2D_sparse_data -------------------------------------------------------------------

namespace tt {

struct PermArgs {
  int32_t perm[TT_MAX_FEATURES];
};

// One kernel, grid-stride: every workgroup first derives the output key starts from the input
// key boundaries (F_out <= 64 loads), then writes lengths/offsets and copies value segments.
__global__ void __launch_bounds__(256) kjt_permute_kernel(
    int64_t B, const int32_t* __restrict__ lengths, const int32_t* __restrict__ offsets,
    const void* __restrict__ values, int id_dtype, const float* __restrict__ weights, PermArgs pa,
    int F_out, int32_t* __restrict__ out_lengths, int32_t* __restrict__ out_offsets,
    void* __restrict__ out_values, float* __restrict__ out_weights) {
  __shared__ int64_t key_start[TT_MAX_FEATURES + 1];
  __shared__ int64_t key_src[TT_MAX_FEATURES];
  if (threadIdx.x == 0) {
    int64_t acc = 0;
    for (int k = 0; k < F_out; ++k) {
      const int p = pa.perm[k];
      const int64_t s = offsets[(int64_t)p * B], e = offsets[(int64_t)(p + 1) * B];
      key_start[k] = acc;
      key_src[k] = s;
      acc += e - s;
    }
    key_start[F_out] = acc;
  }
  __syncthreads();
  const int64_t nb = (int64_t)F_out * B;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = tid; i < nb; i += stride) {
    const int k = (int)(i / B);
    const int64_t b = i - (int64_t)k * B;
    const int p = pa.perm[k];
    const int64_t src = (int64_t)p * B + b;
    out_lengths[i] = lengths[src];
    out_offsets[i + 1] = (int32_t)(key_start[k] + offsets[src + 1] - key_src[k]);
  }
  if (tid == 0) out_offsets[0] = 0;
  const int64_t total = key_start[F_out];
  for (int64_t j = tid; j < total; j += stride) {
    int k = 0;
    while (key_start[k + 1] <= j) ++k;  // F_out <= 64, keys with empty segments are skipped
    const int64_t s = key_src[k] + (j - key_start[k]);
    if (id_dtype == TT_I64)
      reinterpret_cast<int64_t*>(out_values)[j] = reinterpret_cast<const int64_t*>(values)[s];
    else
      reinterpret_cast<int32_t*>(out_values)[j] = reinterpret_cast<const int32_t*>(values)[s];
    if (out_weights) out_weights[j] = weights[s];
  }
}

// ---- block_bucketize_sparse_features (row-wise sharding input_dist) ---------------------------

struct BucketArgs {
  int64_t block_size[TT_MAX_FEATURES];
};

__device__ __forceinline__ void bucket_of(int64_t id, int64_t bs, int W, int* p, int64_t* local) {
  if (id < bs * (int64_t)W) {
    *p = (int)(id / bs);
    *local = id - (int64_t)(*p) * bs;
  } else {
    *p = (int)(id % W);
    *local = id / W;
  }
}

// thread per input bag: count ids per bucket into new_lengths[p][f][b]
__global__ void __launch_bounds__(256) bucketize_count_kernel(
    int F, int64_t B, const int32_t* __restrict__ offsets, const void* __restrict__ values,
    int id_dtype, BucketArgs ba, int W, int32_t* __restrict__ new_lengths) {
  const int64_t nb = (int64_t)F * B;
  const int64_t FB = nb;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(i / B);
    for (int p = 0; p < W; ++p) new_lengths[(int64_t)p * FB + i] = 0;
    const int64_t s = offsets[i], e = offsets[i + 1];
    for (int64_t j = s; j < e; ++j) {
      int p;
      int64_t loc;
      bucket_of(load_id(values, id_dtype, j), ba.block_size[f], W, &p, &loc);
      new_lengths[(int64_t)p * FB + i] += 1;
    }
  }
}

// thread per input bag: write local ids at new_offsets[p][f][b] + running count (input order)
__global__ void __launch_bounds__(256) bucketize_scatter_kernel(
    int F, int64_t B, const int32_t* __restrict__ offsets, const void* __restrict__ values,
    int id_dtype, BucketArgs ba, int W, const int32_t* __restrict__ new_offsets,
    int32_t* __restrict__ cursor, void* __restrict__ new_values) {
  const int64_t nb = (int64_t)F * B;
  const int64_t FB = nb;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(i / B);
    for (int p = 0; p < W; ++p) cursor[(int64_t)p * FB + i] = new_offsets[(int64_t)p * FB + i];
    const int64_t s = offsets[i], e = offsets[i + 1];
    for (int64_t j = s; j < e; ++j) {
      int p;
      int64_t loc;
      bucket_of(load_id(values, id_dtype, j), ba.block_size[f], W, &p, &loc);
      const int64_t pos = cursor[(int64_t)p * FB + i]++;
      if (id_dtype == TT_I64)
        reinterpret_cast<int64_t*>(new_values)[pos] = loc;
      else
        reinterpret_cast<int32_t*>(new_values)[pos] = (int32_t)loc;
    }
  }
}

}  // namespace tt

extern "C" {

int tt_kjt_permute(int F, int64_t B, const int32_t* lengths, const int32_t* offsets,
                   const void* values, int id_dtype, const float* weights, const int32_t* perm,
                   int F_out, int32_t* out_lengths, int32_t* out_offsets, void* out_values,
                   float* out_weights, void* stream) {
  if (F < 1 || F > TT_MAX_FEATURES || F_out < 0 || F_out > TT_MAX_FEATURES || B < 0)
    return fail(TT_EINVAL, "kjt_permute: F/F_out/B out of range");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "kjt_permute: bad id dtype");
  if (!perm || !lengths || !offsets || !out_lengths || !out_offsets)
    return fail(TT_EINVAL, "kjt_permute: null pointer");
  if ((weights == nullptr) != (out_weights == nullptr))
    return fail(TT_EINVAL, "kjt_permute: weights and out_weights must both be set or both null");
  PermArgs pa{};
  for (int k = 0; k < F_out; ++k) {
    if (perm[k] < 0 || perm[k] >= F) return fail(TT_EINVAL, "kjt_permute: perm index out of range");
    pa.perm[k] = perm[k];
  }
  hipStream_t st = as_stream(stream);
  if (F_out == 0 || B == 0) {
    if (hipMemsetAsync(out_offsets, 0, sizeof(int32_t), st) != hipSuccess)
      return fail(TT_EINVAL, "kjt_permute: memset failed");
    return TT_OK;
  }
  const int64_t nb = (int64_t)F_out * B;
  const int grid = (int)std::min<int64_t>(2048, std::max<int64_t>(1, ceil_div(nb, 256)));
  kjt_permute_kernel<<<dim3(grid), dim3(256), 0, st>>>(B, lengths, offsets, values, id_dtype, weights,
                                                       pa, F_out, out_lengths, out_offsets,
                                                       out_values, out_weights);
  return check_launch("kjt_permute");
}

size_t tt_block_bucketize_workspace_bytes(int F, int64_t B, int W) {
  const int64_t n = (int64_t)F * B * W;
  return align_up((size_t)n * sizeof(int32_t), 256) + tt_complete_cumsum_workspace_bytes(n);
}

int tt_block_bucketize(int F, int64_t B, const int32_t* lengths, const int32_t* offsets,
                       const void* values, int id_dtype, const int64_t* block_sizes, int W,
                       int32_t* new_lengths, int32_t* new_offsets, void* new_values,
                       void* workspace, size_t ws_bytes, void* stream) {
  (void)lengths;
  if (F < 1 || F > TT_MAX_FEATURES || B < 0 || W < 1)
    return fail(TT_EINVAL, "block_bucketize: F/B/W out of range");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "block_bucketize: bad id dtype");
  if (!offsets || !block_sizes || !new_lengths || !new_offsets)
    return fail(TT_EINVAL, "block_bucketize: null pointer");
  if ((int64_t)F * B * W > INT32_MAX) return fail(TT_EINVAL, "block_bucketize: too many bags");
  if (ws_bytes < tt_block_bucketize_workspace_bytes(F, B, W) || !workspace)
    return fail(TT_ECAPACITY, "block_bucketize: workspace too small");
  BucketArgs ba{};
  for (int f = 0; f < F; ++f) {
    if (block_sizes[f] < 1) return fail(TT_EINVAL, "block_bucketize: block size must be >= 1");
    ba.block_size[f] = block_sizes[f];
  }
  hipStream_t st = as_stream(stream);
  const int64_t nb = (int64_t)F * B;
  const int64_t n = nb * W;
  if (nb == 0) {
    if (hipMemsetAsync(new_offsets, 0, sizeof(int32_t), st) != hipSuccess)
      return fail(TT_EINVAL, "block_bucketize: memset failed");
    return TT_OK;
  }
  int32_t* cursor = reinterpret_cast<int32_t*>(workspace);
  int* bsum = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) +
                                     align_up((size_t)n * sizeof(int32_t), 256));
  const int grid = (int)std::min<int64_t>(4096, std::max<int64_t>(1, ceil_div(nb, 256)));
  bucketize_count_kernel<<<dim3(grid), dim3(256), 0, st>>>(F, B, offsets, values, id_dtype, ba, W,
                                                           new_lengths);
  int rc = launch_cumsum(new_lengths, n, new_offsets, bsum, st);
  if (rc) return rc;
  bucketize_scatter_kernel<<<dim3(grid), dim3(256), 0, st>>>(F, B, offsets, values, id_dtype, ba, W,
                                                             new_offsets, cursor, new_values);
  return check_launch("block_bucketize");
}

}  // extern "C"

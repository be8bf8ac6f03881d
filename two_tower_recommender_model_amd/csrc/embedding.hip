// Embedding-bag hot path for gfx950: pooled (segmented gather + sum) forward and the
// deduplicated backward with exact row-wise Adagrad fused in (no weight .grad is materialised).
//
// Forward (k1): a group of G lanes owns one bag; each lane owns a 16-B column slice (float4) of the
// row, so one D=128 fp32 row is one 512-B coalesced read by 32 lanes and a wave pools 2 bags at
// once. Ids of a bag are read 4 at a time so 4 independent rows are in flight per group.
// Algorithmic bytes per lookup: 4*D (row) + id bytes; per bag 4*D write + 4 (offset).
// A column variant (k1c) reads single-hot ids straight from the loader's columns and applies the
// reference transform inline (drop id 0, id mod N: transform_to_torchrec_batch semantics).
//
// Backward: lookups are grouped by unique (table,row) with an open-addressing hash (k2a), a
// reduce-then-scan over the hash slots gives every unique row a segment and a 16-B record
// {key, start, count} and leaves the hash table clean for the next step (k2b), the bag ids are
// scattered into their segments (k2c), then per unique row the pooled-gradient rows of its
// segment are summed and the row-wise Adagrad update is applied in place (k2d). k2a-k2c read only
// ids, so they run beside the forward and the towers.
// k2d "narrow" (D <= 128, D % 4 == 0): a half-wave per unique row (32 lanes x float4 = one
// 512-B row), two rows per wave; segments of <= 32 lookups are summed in ascending bag order
// (bitwise reproducible). k2d "generic": a wave per row for other dims. Longer segments ("hot"
// rows) go to a workgroup-per-row kernel that sorts their bag ids in LDS: same canonical order.
#include "tt_common.h"

namespace tt {

struct ColArgs {
  const void* col[TT_MAX_FEATURES];
  int64_t num_emb[TT_MAX_FEATURES];  // the transform's divisor (id mod N)
};

// ============================== forward =======================================================

struct FwdArgs {
  EmbMeta m;
  int32_t block_start[TT_MAX_FEATURES + 1];  // first workgroup of each feature
  int8_t group[TT_MAX_FEATURES];             // lanes per bag (power of two <= 64)
  int8_t vec[TT_MAX_FEATURES];               // 4 = float4 path, 1 = scalar path
};

template <int VEC>
__device__ __forceinline__ void pool_bag_cols(const float* __restrict__ w, const void* __restrict__ values,
                                              int id_dtype, int64_t s, int64_t e, int64_t rows, int D,
                                              int lane_g, int G, float scale, float* __restrict__ out,
                                              int bounds_check, int32_t* err) {
  typedef __attribute__((ext_vector_type(VEC))) float vf;
  const int ncol = D / VEC;
  for (int c = lane_g; c < ncol; c += G) {
    vf acc0 = (vf)(0.f);
    int64_t j = s;
    for (; j + 4 <= e; j += 4) {
      int64_t id0 = load_id(values, id_dtype, j), id1 = load_id(values, id_dtype, j + 1);
      int64_t id2 = load_id(values, id_dtype, j + 2), id3 = load_id(values, id_dtype, j + 3);
      if (bounds_check) {
        if ((uint64_t)id0 >= (uint64_t)rows) { if (c == lane_g && lane_g == 0) atomicAdd(err, 1); id0 = 0; }
        if ((uint64_t)id1 >= (uint64_t)rows) { if (c == lane_g && lane_g == 0) atomicAdd(err, 1); id1 = 0; }
        if ((uint64_t)id2 >= (uint64_t)rows) { if (c == lane_g && lane_g == 0) atomicAdd(err, 1); id2 = 0; }
        if ((uint64_t)id3 >= (uint64_t)rows) { if (c == lane_g && lane_g == 0) atomicAdd(err, 1); id3 = 0; }
      }
      const vf r0 = *reinterpret_cast<const vf*>(w + id0 * D + c * VEC);
      const vf r1 = *reinterpret_cast<const vf*>(w + id1 * D + c * VEC);
      const vf r2 = *reinterpret_cast<const vf*>(w + id2 * D + c * VEC);
      const vf r3 = *reinterpret_cast<const vf*>(w + id3 * D + c * VEC);
      // fixed left-to-right order within the bag, like a sequential fp32 sum
      acc0 += r0;
      acc0 += r1;
      acc0 += r2;
      acc0 += r3;
    }
    for (; j < e; ++j) {
      int64_t id = load_id(values, id_dtype, j);
      if (bounds_check && (uint64_t)id >= (uint64_t)rows) {
        if (c == lane_g && lane_g == 0) atomicAdd(err, 1);
        id = 0;
      }
      acc0 += *reinterpret_cast<const vf*>(w + id * D + c * VEC);
    }
    acc0 *= scale;
    *reinterpret_cast<vf*>(out + c * VEC) = acc0;
  }
}

__device__ __forceinline__ int feature_of_block(const FwdArgs& a) {
  int f = 0;
  while (f + 1 < a.m.F && (int)blockIdx.x >= a.block_start[f + 1]) ++f;
  return f;
}

__global__ void __launch_bounds__(256) pooled_fwd_kernel(const float* __restrict__ weights, FwdArgs a,
                                                         const void* __restrict__ values, int id_dtype,
                                                         const int32_t* __restrict__ offsets, int pooling,
                                                         float* __restrict__ out, int64_t ldo,
                                                         int bounds_check, int32_t* __restrict__ err) {
  const int f = feature_of_block(a);  // wave-uniform scalar search (F <= 64)
  const tt_feature_meta_t fm = a.m.features[f];
  const tt_table_meta_t tm = a.m.tables[fm.table];
  const int G = a.group[f];
  const int bags_per_block = 256 / G;
  const int64_t B = a.m.B;
  const int64_t b = (int64_t)(blockIdx.x - a.block_start[f]) * bags_per_block + threadIdx.x / G;
  if (b >= B) return;
  const int lane_g = threadIdx.x & (G - 1);
  const int64_t bag = (int64_t)f * B + b;
  const int64_t s = offsets[bag], e = offsets[bag + 1];
  const float scale = (pooling == TT_POOL_MEAN && e > s) ? 1.0f / (float)(e - s) : 1.0f;
  const float* w = weights + tm.weight_offset;
  float* o = out + (fm.out_row + b) * ldo + fm.out_offset;
  if (a.vec[f] == 4)
    pool_bag_cols<4>(w, values, id_dtype, s, e, tm.num_rows, tm.dim, lane_g, G, scale, o, bounds_check, err);
  else
    pool_bag_cols<1>(w, values, id_dtype, s, e, tm.num_rows, tm.dim, lane_g, G, scale, o, bounds_check, err);
}

// k1c: single-hot columns -> pooled rows, transform applied inline (id 0 -> empty bag -> zeros)
template <int VEC>
__device__ __forceinline__ void copy_row(const float* __restrict__ src, float* __restrict__ dst, int D, int lane_g,
                                         int G) {
  typedef __attribute__((ext_vector_type(VEC))) float vf;
  for (int c = lane_g; c < D / VEC; c += G) {
    vf v = src ? *reinterpret_cast<const vf*>(src + c * VEC) : (vf)(0.f);
    *reinterpret_cast<vf*>(dst + c * VEC) = v;
  }
}

__global__ void __launch_bounds__(256) pooled_fwd_cols_kernel(const float* __restrict__ weights, FwdArgs a, ColArgs ca,
                                                              int id_dtype, float* __restrict__ out, int64_t ldo) {
  const int f = feature_of_block(a);
  const tt_feature_meta_t fm = a.m.features[f];
  const tt_table_meta_t tm = a.m.tables[fm.table];
  const int G = a.group[f];
  const int64_t B = a.m.B;
  const int64_t b = (int64_t)(blockIdx.x - a.block_start[f]) * (256 / G) + threadIdx.x / G;
  if (b >= B) return;
  const int lane_g = threadIdx.x & (G - 1);
  const int64_t id = load_id(ca.col[f], id_dtype, b);
  const float* src = nullptr;
  if (id != 0) src = weights + tm.weight_offset + py_mod64(id, ca.num_emb[f]) * tm.dim;
  float* o = out + (fm.out_row + b) * ldo + fm.out_offset;
  if (a.vec[f] == 4)
    copy_row<4>(src, o, tm.dim, lane_g, G);
  else
    copy_row<1>(src, o, tm.dim, lane_g, G);
}

// ============================== backward ======================================================

constexpr uint64_t EMPTY_KEY = ~0ull;
constexpr int KEY_TABLE_SHIFT = 40;  // key = table << 40 | row  (rows < 2^40 per shard)

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

struct URec {
  uint64_t key;
  int32_t seg;
  int32_t len;
};

// Rows looked up more than HOT_MIN - 1 times in a step are "hot": the per-row kernels (which sort
// a segment of <= 32 bag ids in registers) skip them and bwd_adagrad_hot_kernel sums them in
// ascending bag order through LDS, so every row's gradient is summed in one canonical order.
constexpr int HOT_MIN = 33;
constexpr int HOT_CAP = 4096;  // bag ids sorted in LDS per pass of the hot kernel

struct BwdWs {
  uint64_t* keys;   // [cap] hash keys (EMPTY when free; cleaned by k2b)
  int32_t* cnt;     // [cap] lookups per slot (cleaned by k2b)
  int32_t* cur;     // [cap] scatter cursor per slot (set by k2b)
  int32_t* slot_of; // [L]   slot of each lookup (-1: none)
  int32_t* perm;    // [L]   bag ids grouped by unique row
  URec* urec;       // [L]   per unique row
  int32_t* bsum_u;  // [nb]  scan partials (unique count)
  int32_t* bsum_c;  // [nb]  scan partials (lookup count)
  int32_t* hot;     // [L/HOT_MIN] unique indices whose segment is longer than HOT_MIN - 1
  int32_t* U;       // [4]   {unique rows, -, hot rows, -}
  int64_t cap;
  int64_t L;
};

static int64_t bwd_cap(int64_t L) {
  int64_t c = 1024;
  while (c < 2 * L) c <<= 1;
  return c;
}

static size_t bwd_layout(void* base, int64_t L, BwdWs* w) {
  const int64_t cap = bwd_cap(L);
  const int64_t nb = ceil_div(cap, 1024);
  char* p = reinterpret_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = p ? p + off : nullptr;
    off += align_up(bytes, 256);
    return r;
  };
  BwdWs t;
  t.keys = reinterpret_cast<uint64_t*>(take(sizeof(uint64_t) * cap));
  t.cnt = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * cap));
  t.cur = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * cap));
  t.slot_of = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.perm = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.urec = reinterpret_cast<URec*>(take(sizeof(URec) * L));
  t.bsum_u = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * nb));
  t.bsum_c = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * nb));
  t.hot = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (L / HOT_MIN + 1)));
  t.U =reinterpret_cast<int32_t*>(take(sizeof(int32_t) * 4));
  t.cap = cap;
  t.L = L;
  if (w) *w = t;
  return off;
}

__device__ __forceinline__ int32_t hash_insert(BwdWs& ws, uint64_t key) {
  // one returning CAS per probe: it claims an empty slot or reports who holds it
  const uint64_t mask = (uint64_t)ws.cap - 1;
  uint64_t h = mix64(key) & mask;
  while (true) {
    const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&ws.keys[h]),
                                    (unsigned long long)EMPTY_KEY, (unsigned long long)key);
    if (prev == EMPTY_KEY || prev == key) break;
    h = (h + 1) & mask;
  }
  atomicAdd(&ws.cnt[h], 1);
  return (int32_t)h;
}

// k2a: thread per bag: hash-insert every lookup's (table,row), count per slot
__global__ void __launch_bounds__(256) bwd_hash_kernel(EmbMeta m, const void* __restrict__ values, int id_dtype,
                                                       const int32_t* __restrict__ offsets, int bounds_check,
                                                       BwdWs ws) {
  const int64_t nbag = (int64_t)m.F * m.B;
  for (int64_t bag = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; bag < nbag;
       bag += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(bag / m.B);
    const int t = m.features[f].table;
    const int64_t rows = m.tables[t].num_rows;
    const int64_t s = offsets[bag], e = offsets[bag + 1];
    for (int64_t j = s; j < e; ++j) {
      int64_t id = load_id(values, id_dtype, j);
      if (bounds_check && (uint64_t)id >= (uint64_t)rows) id = 0;
      ws.slot_of[j] = hash_insert(ws, ((uint64_t)t << KEY_TABLE_SHIFT) | (uint64_t)id);
    }
  }
}

// k2a (columns): lookup index = bag index; dropped ids get slot -1
__global__ void __launch_bounds__(256) bwd_hash_cols_kernel(EmbMeta m, ColArgs ca, int id_dtype, BwdWs ws) {
  const int64_t nbag = (int64_t)m.F * m.B;
  for (int64_t bag = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; bag < nbag;
       bag += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(bag / m.B);
    const int64_t b = bag - (int64_t)f * m.B;
    const int64_t id = load_id(ca.col[f], id_dtype, b);
    int32_t h = -1;
    if (id != 0) {
      const int t = m.features[f].table;
      h = hash_insert(ws, ((uint64_t)t << KEY_TABLE_SHIFT) | (uint64_t)py_mod64(id, ca.num_emb[f]));
    }
    ws.slot_of[bag] = h;
  }
}

// k2b-1: per 1024-slot tile: number of occupied slots and of lookups
__global__ void __launch_bounds__(256) bwd_scan_reduce_kernel(BwdWs ws) {
  __shared__ int lu[4], lc[4];
  const int64_t base = (int64_t)blockIdx.x * 1024;
  int su = 0, sc = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = ws.cnt[base + j * 256 + threadIdx.x];
    su += c > 0;
    sc += c;
  }
  su = wave_sum_i(su);
  sc = wave_sum_i(sc);
  if ((threadIdx.x & 63) == 0) {
    lu[threadIdx.x >> 6] = su;
    lc[threadIdx.x >> 6] = sc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ws.bsum_u[blockIdx.x] = lu[0] + lu[1] + lu[2] + lu[3];
    ws.bsum_c[blockIdx.x] = lc[0] + lc[1] + lc[2] + lc[3];
    if (blockIdx.x == 0) ws.U[2] = 0;  // hot list, filled by k2b-2
  }
}

// k2b-2: exclusive scans -> record {key, segment start, count} per unique row; cursor per slot;
// the slot's key and count are reset here, so the table is clean for the next step's k2a.
__global__ void __launch_bounds__(256) bwd_scan_kernel(BwdWs ws) {
  __shared__ int lds[8];
  int pu = 0, pc = 0;
  for (int i = threadIdx.x; i < (int)blockIdx.x; i += 256) {
    pu += ws.bsum_u[i];
    pc += ws.bsum_c[i];
  }
  pu = wave_sum_i(pu);
  pc = wave_sum_i(pc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    lds[wid] = pu;
    lds[4 + wid] = pc;
  }
  __syncthreads();
  pu = lds[0] + lds[1] + lds[2] + lds[3];
  pc = lds[4] + lds[5] + lds[6] + lds[7];
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  int c[4], lu = 0, lcnt = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = ws.cnt[base + j];
    lu += c[j] > 0;
    lcnt += c[j];
  }
  int iu = lu, ic = lcnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int yu = __shfl_up(iu, o, 64), yc = __shfl_up(ic, o, 64);
    if (lane >= o) {
      iu += yu;
      ic += yc;
    }
  }
  if (lane == 63) {
    lds[wid] = iu;
    lds[4 + wid] = ic;
  }
  __syncthreads();
  int wu = 0, wc = 0, tu = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    if (w < wid) {
      wu += lds[w];
      wc += lds[4 + w];
    }
    tu += lds[w];
  }
  int eu = pu + wu + iu - lu, ec = pc + wc + ic - lcnt;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (c[j] > 0) {
      const int64_t h = base + j;
      URec rec;
      rec.key = ws.keys[h];
      rec.seg = ec;
      rec.len = c[j];
      ws.urec[eu] = rec;
      if (c[j] >= HOT_MIN) ws.hot[atomicAdd(&ws.U[2], 1)] = eu;
      ws.cur[h] = ec;
      ws.keys[h] = EMPTY_KEY;
      ws.cnt[h] = 0;
      eu += 1;
      ec += c[j];
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) ws.U[0] = pu + tu;
}

// k2c: thread per bag: scatter bag ids into their unique row's segment
__global__ void __launch_bounds__(256) bwd_scatter_kernel(EmbMeta m, const int32_t* __restrict__ offsets, BwdWs ws) {
  const int64_t nbag = (int64_t)m.F * m.B;
  for (int64_t bag = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; bag < nbag;
       bag += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = offsets ? offsets[bag] : bag, e = offsets ? offsets[bag + 1] : bag + 1;
    for (int64_t j = s; j < e; ++j) {
      const int h = ws.slot_of[j];
      if (h < 0) continue;
      const int pos = atomicAdd(&ws.cur[h], 1);
      ws.perm[pos] = (int32_t)bag;
    }
  }
}

// ascending bitonic sort of one int per lane over groups of W lanes (W = 32 or 64)
template <int W>
__device__ __forceinline__ int bitonic_sort(int v) {
  const int lane = threadIdx.x & (W - 1);
#pragma unroll
  for (int k = 2; k <= W; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int o = __shfl_xor(v, j, 64);
      const bool up = (lane & k) == 0;
      const bool lower = (lane & j) == 0;
      const int mn = v < o ? v : o, mx = v < o ? o : v;
      v = (lower == up) ? mn : mx;
    }
  }
  return v;
}

struct BagRow {
  const float* g;
  int64_t B;
  int64_t ldg;
  const tt_feature_meta_t* feats;
  __device__ __forceinline__ const float* row(int bag) const {
    const int f = (int)(bag / B);
    const int64_t b = bag - (int64_t)f * B;
    return g + (feats[f].out_row + b) * ldg + feats[f].out_offset;
  }
};

// ---- k2d narrow: half-wave per unique row, D <= 128, D % 4 == 0 ----------------------------
__global__ void __launch_bounds__(256) bwd_adagrad_narrow_kernel(EmbMeta m, const float* __restrict__ grad_out,
                                                                 int64_t ldg, const int32_t* __restrict__ offsets,
                                                                 int pooling, float* __restrict__ weights,
                                                                 float* __restrict__ state, float lr, float eps,
                                                                 BwdWs ws) {
  const int U = ws.U[0];
  const int lane = threadIdx.x & 63;
  const int hl = lane & 31, half = lane >> 5;
  const BagRow br{grad_out, m.B, ldg, m.features};
  const int64_t nhalf = (int64_t)gridDim.x * 8;
  for (int64_t u = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + half; u - half < U; u += nhalf) {
    URec rec{0, 0, 0};
    if (u < U) rec = ws.urec[u];
    const bool active = u < U && rec.len < HOT_MIN;  // hot rows: bwd_adagrad_hot_kernel
    if (!active) rec = URec{0, 0, 0};
    const int t = (int)(rec.key >> KEY_TABLE_SHIFT);
    const int64_t r = (int64_t)(rec.key & ((1ull << KEY_TABLE_SHIFT) - 1));
    const tt_table_meta_t tm = m.tables[active ? t : 0];
    const int D = tm.dim;
    const bool col_ok = active && hl * 4 < D;
    // independent of the gradient: fetch the row and its state early
    float* wrow = weights + tm.weight_offset + r * D;
    float* srow = state + tm.state_offset + r;
    f32x4v wv = col_ok ? *reinterpret_cast<const f32x4v*>(wrow + hl * 4) : (f32x4v)(0.f);
    const float s_old = active ? *srow : 0.f;
    const int n = rec.len;
    f32x4v g = (f32x4v)(0.f);
    // ascending bag order (bitonic over the half-wave), fp32: bitwise reproducible
    const int nmax = max(n, __shfl_xor(n, 32, 64));
    int mine = (active && hl < n) ? ws.perm[rec.seg + hl] : 0x7fffffff;
    mine = bitonic_sort<32>(mine);
    for (int i = 0; i < nmax; i += 2) {
      const int b0 = __shfl(mine, (lane & 32) + i, 64);
      const int b1 = __shfl(mine, (lane & 32) + min(i + 1, 31), 64);
      const bool v0 = i < n, v1 = i + 1 < n;
      f32x4v x0 = (f32x4v)(0.f), x1 = (f32x4v)(0.f);
      if (col_ok && v0) x0 = *reinterpret_cast<const f32x4v*>(br.row(b0) + hl * 4);
      if (col_ok && v1) x1 = *reinterpret_cast<const f32x4v*>(br.row(b1) + hl * 4);
      if (pooling == TT_POOL_MEAN) {
        if (v0) x0 *= 1.f / (float)max(1, offsets[b0 + 1] - offsets[b0]);
        if (v1) x1 *= 1.f / (float)max(1, offsets[b1 + 1] - offsets[b1]);
      }
      if (v0) g += x0;
      if (v1) g += x1;
    }
    // row-wise Adagrad: s += mean(G^2); w += (-lr * G) / (sqrt(s) + eps)
    float sq = g[0] * g[0] + g[1] * g[1] + g[2] * g[2] + g[3] * g[3];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
    if (active) {
      const float snew = s_old + sq / (float)D;
      const float stdv = sqrtf(snew) + eps;
      if (col_ok) {
#pragma unroll
        for (int v = 0; v < 4; ++v) wv[v] = wv[v] + (-lr * g[v]) / stdv;
        *reinterpret_cast<f32x4v*>(wrow + hl * 4) = wv;
      }
      if (hl == 0) *srow = snew;
    }
  }
}

// ---- k2d generic: a wave per unique row, any D <= 1024 ------------------------------------
constexpr int ADA_KMAX = 4;  // up to 4 x 64 x VEC columns per row

template <int VEC>
__device__ __forceinline__ void adagrad_row(const EmbMeta& m, const BagRow& br, const int32_t* __restrict__ offsets,
                                            int pooling, float* __restrict__ weights, float* __restrict__ state,
                                            float lr, float eps, const BwdWs& ws, int t, int64_t r, int s, int n) {
  typedef __attribute__((ext_vector_type(VEC))) float vf;
  const int lane = threadIdx.x & 63;
  const tt_table_meta_t tm = m.tables[t];
  const int D = tm.dim;
  const int ncol = D / VEC;
  float* w = weights + tm.weight_offset + r * D;
  float* srow = state + tm.state_offset + r;
  float sq = 0.f;
  float gsave[ADA_KMAX][VEC];
  // n < HOT_MIN (hot rows go to bwd_adagrad_hot_kernel): ascending bag order, fp32
  int sorted = lane < n ? ws.perm[s + lane] : 0x7fffffff;
  sorted = bitonic_sort<64>(sorted);
#pragma unroll
  for (int k = 0; k < ADA_KMAX; ++k) {
    const int c = lane + k * 64;
    float accf[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) accf[v] = 0.f;
    for (int i = 0; i < n; ++i) {
      const int b = __shfl(sorted, i, 64);
      if (c < ncol) {
        vf x = *reinterpret_cast<const vf*>(br.row(b) + c * VEC);
        const float sc = pooling == TT_POOL_MEAN ? 1.f / (float)max(1, offsets[b + 1] - offsets[b]) : 1.f;
#pragma unroll
        for (int v = 0; v < VEC; ++v) accf[v] += x[v] * sc;
      }
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      gsave[k][v] = accf[v];
      sq += accf[v] * accf[v];
    }
  }
  sq = wave_sum(sq);
  const float snew = *srow + sq / (float)D;
  const float stdv = sqrtf(snew) + eps;
#pragma unroll
  for (int k = 0; k < ADA_KMAX; ++k) {
    const int c = lane + k * 64;
    if (c < ncol) {
      vf x = *reinterpret_cast<vf*>(w + c * VEC);
#pragma unroll
      for (int v = 0; v < VEC; ++v) x[v] = x[v] + (-lr * gsave[k][v]) / stdv;
      *reinterpret_cast<vf*>(w + c * VEC) = x;
    }
  }
  if (lane == 0) *srow = snew;
}

__global__ void __launch_bounds__(256) bwd_adagrad_kernel(EmbMeta m, const float* __restrict__ grad_out, int64_t ldg,
                                                          const int32_t* __restrict__ offsets, int pooling,
                                                          float* __restrict__ weights, float* __restrict__ state,
                                                          float lr, float eps, BwdWs ws, int vec4_ok) {
  const int U = ws.U[0];
  const BagRow br{grad_out, m.B, ldg, m.features};
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); u < U; u += nwaves) {
    const URec rec = ws.urec[u];
    if (rec.len >= HOT_MIN) continue;  // bwd_adagrad_hot_kernel
    const int t = (int)(rec.key >> KEY_TABLE_SHIFT);
    const int64_t r = (int64_t)(rec.key & ((1ull << KEY_TABLE_SHIFT) - 1));
    const int D = m.tables[t].dim;
    if (vec4_ok && (D & 3) == 0 && D >= 256)
      adagrad_row<4>(m, br, offsets, pooling, weights, state, lr, eps, ws, t, r, rec.seg, rec.len);
    else if (vec4_ok && (D & 1) == 0)
      adagrad_row<2>(m, br, offsets, pooling, weights, state, lr, eps, ws, t, r, rec.seg, rec.len);
    else
      adagrad_row<1>(m, br, offsets, pooling, weights, state, lr, eps, ws, t, r, rec.seg, rec.len);
  }
}

// ---- k2d hot rows: a workgroup per row looked up >= HOT_MIN times --------------------------
// The segment's bag ids are summed in ascending order whatever order the scatter left them in:
// passes over bag-id ranges [lo, hi) holding <= HOT_CAP ids each (hi found by halving, so the
// ranges depend on the id multiset only), each range sorted in LDS; inside a range, group g of
// HOT_G sums sorted positions g, g + HOT_G, ..., and the group partials are added in group order.
// Every step of that is a function of the multiset of bag ids: bitwise reproducible.
constexpr int HOT_TPR = 64;                 // threads per gradient row (columns strided by 64)
constexpr int HOT_G = 256 / HOT_TPR;        // row groups
constexpr int HOT_KC = 1024 / HOT_TPR;      // columns per thread at D = 1024

__device__ __forceinline__ int block_sum_i(int v, int* red) {
  v = wave_sum_i(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) bwd_adagrad_hot_kernel(EmbMeta m, const float* __restrict__ grad_out,
                                                              int64_t ldg, const int32_t* __restrict__ offsets,
                                                              int pooling, float* __restrict__ weights,
                                                              float* __restrict__ state, float lr, float eps,
                                                              BwdWs ws) {
  __shared__ int ids[HOT_CAP];
  __shared__ float part[HOT_G][1024];
  __shared__ int redi[4];
  __shared__ float redf[4];
  __shared__ int fill;
  const int tid = threadIdx.x;
  const int cg = tid % HOT_TPR, gi = tid / HOT_TPR;
  const int nhot = ws.U[2];
  const BagRow br{grad_out, m.B, ldg, m.features};
  for (int h = blockIdx.x; h < nhot; h += gridDim.x) {
    const URec rec = ws.urec[ws.hot[h]];
    const int t = (int)(rec.key >> KEY_TABLE_SHIFT);
    const int64_t r = (int64_t)(rec.key & ((1ull << KEY_TABLE_SHIFT) - 1));
    const tt_table_meta_t tm = m.tables[t];
    const int D = tm.dim;
    const int32_t* seg = ws.perm + rec.seg;
    const int n = rec.len;
    float tot[4] = {0.f, 0.f, 0.f, 0.f};  // column tid + 256 k (D <= 1024)
    const int64_t NB = (int64_t)m.F * m.B;  // bag ids are < F * B
    int64_t lo = 0, width = 1;
    while (width < NB) width <<= 1;
    while (lo < NB) {
      int64_t hi;
      int c;
      while (true) {  // shrink [lo, hi) until it holds <= HOT_CAP ids (or a single bag id)
        hi = lo + width < NB ? lo + width : NB;
        int k = 0;
        for (int i = tid; i < n; i += 256) {
          const int b = seg[i];
          k += (b >= lo && b < hi);
        }
        c = block_sum_i(k, redi);
        if (c <= HOT_CAP || hi - lo == 1) break;
        width >>= 1;
      }
      if (c == 0) {
        lo = hi;
        width <<= 1;
        continue;
      }
      const bool single = c > HOT_CAP;  // one bag id repeated c times: every position holds lo
      if (!single) {
        if (tid == 0) fill = 0;
        __syncthreads();
        for (int i = tid; i < n; i += 256) {
          const int b = seg[i];
          if (b >= lo && b < hi) ids[atomicAdd(&fill, 1)] = b;
        }
        int P = 1;
        while (P < c) P <<= 1;
        for (int i = c + tid; i < P; i += 256) ids[i] = 0x7fffffff;
        __syncthreads();
        for (int k = 2; k <= P; k <<= 1)
          for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P; i += 256) {
              const int x = i ^ j;
              if (x > i) {
                const int a = ids[i], b = ids[x];
                if ((a > b) == ((i & k) == 0)) {
                  ids[i] = b;
                  ids[x] = a;
                }
              }
            }
            __syncthreads();
          }
      }
      float acc[HOT_KC];
#pragma unroll
      for (int k = 0; k < HOT_KC; ++k) acc[k] = 0.f;
      for (int i = gi; i < c; i += HOT_G) {
        const int b = single ? (int)lo : ids[i];
        const float* g = br.row(b);
        const float sc = pooling == TT_POOL_MEAN ? 1.f / (float)max(1, offsets[b + 1] - offsets[b]) : 1.f;
#pragma unroll
        for (int k = 0; k < HOT_KC; ++k) {
          const int col = cg + k * HOT_TPR;
          if (col < D) acc[k] += g[col] * sc;
        }
      }
#pragma unroll
      for (int k = 0; k < HOT_KC; ++k) {
        const int col = cg + k * HOT_TPR;
        if (col < D) part[gi][col] = acc[k];
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int col = tid + 256 * k;
        if (col < D) {
          float s = 0.f;
#pragma unroll
          for (int g = 0; g < HOT_G; ++g) s += part[g][col];
          tot[k] += s;
        }
      }
      __syncthreads();
      lo = hi;
      width <<= 1;  // the next range starts wider (still a function of the id multiset only)
    }
    // row-wise Adagrad on the summed row
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (tid + 256 * k < D) sq += tot[k] * tot[k];
    sq = wave_sum(sq);
    __syncthreads();
    if ((tid & 63) == 0) redf[tid >> 6] = sq;
    __syncthreads();
    sq = (redf[0] + redf[1]) + (redf[2] + redf[3]);
    float* srow = state + tm.state_offset + r;
    const float snew = *srow + sq / (float)D;
    const float stdv = sqrtf(snew) + eps;
    float* wrow = weights + tm.weight_offset + r * D;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int col = tid + 256 * k;
      if (col < D) wrow[col] = wrow[col] + (-lr * tot[k]) / stdv;
    }
    __syncthreads();
    if (tid == 0) *srow = snew;
  }
}

// unfused dense backward: grad_weights[row] += grad_out[bag] (fp32 atomics)
__global__ void __launch_bounds__(256) bwd_dense_kernel(EmbMeta m, const float* __restrict__ grad_out, int64_t ldg,
                                                        const void* __restrict__ values, int id_dtype,
                                                        const int32_t* __restrict__ offsets, int pooling,
                                                        float* __restrict__ gw, int bounds_check) {
  const int64_t nbag = (int64_t)m.F * m.B;
  const int lane = threadIdx.x & 63;
  for (int64_t bag = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); bag < nbag; bag += (int64_t)gridDim.x * 4) {
    const int f = (int)(bag / m.B);
    const int64_t b = bag - (int64_t)f * m.B;
    const tt_table_meta_t tm = m.tables[m.features[f].table];
    const int64_t s = offsets[bag], e = offsets[bag + 1];
    const float sc = (pooling == TT_POOL_MEAN && e > s) ? 1.f / (float)(e - s) : 1.f;
    const float* g = grad_out + (m.features[f].out_row + b) * ldg + m.features[f].out_offset;
    for (int64_t j = s; j < e; ++j) {
      int64_t id = load_id(values, id_dtype, j);
      if (bounds_check && (uint64_t)id >= (uint64_t)tm.num_rows) id = 0;
      float* dst = gw + tm.weight_offset + id * tm.dim;
      for (int c = lane; c < tm.dim; c += 64) atomicAdd(dst + c, g[c] * sc);
    }
  }
}

// ---- host helpers ---------------------------------------------------------------------------

static int fwd_geometry(FwdArgs& a, const float* weights, const float* out, int64_t ldo, int64_t B, int64_t* blocks) {
  int64_t nb = 0;
  for (int f = 0; f < a.m.F; ++f) {
    const tt_table_meta_t& tm = a.m.tables[a.m.features[f].table];
    if (a.m.features[f].out_offset + tm.dim > ldo) return fail(TT_EINVAL, "pooled_fwd: output row too short");
    const bool v4 = (tm.dim % 4 == 0) && (tm.weight_offset % 4 == 0) && (a.m.features[f].out_offset % 4 == 0) &&
                    (ldo % 4 == 0) && ((reinterpret_cast<uintptr_t>(weights) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
    a.vec[f] = v4 ? 4 : 1;
    const int cols = tm.dim / a.vec[f];
    int g = 1;
    while (g < cols && g < 64) g <<= 1;
    a.group[f] = (int8_t)g;
    a.block_start[f] = (int32_t)nb;
    nb += ceil_div(B, 256 / g);
  }
  a.block_start[a.m.F] = (int32_t)nb;
  if (nb > INT32_MAX) return fail(TT_EINVAL, "pooled_fwd: grid too large");
  *blocks = nb;
  return TT_OK;
}

static int pack_cols(ColArgs& ca, int F, const void* const* cols, const int64_t* num_emb, int id_dtype) {
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "cols: ids must be int32/int64");
  if (!cols || !num_emb) return fail(TT_EINVAL, "cols: null pointer");
  for (int f = 0; f < F; ++f) {
    if (!cols[f] || num_emb[f] < 1) return fail(TT_EINVAL, "cols: null column or num_embeddings < 1");
    ca.col[f] = cols[f];
    ca.num_emb[f] = num_emb[f];
  }
  return TT_OK;
}

static int check_ws(void* workspace, size_t ws_bytes, int64_t max_lookups, const char* what);

}  // namespace tt

using namespace tt;

extern "C" {

int tt_pooled_fwd(const float* weights, const tt_table_meta_t* tables, int T,
                  const tt_feature_meta_t* features, int F, int64_t B, const void* values,
                  int id_dtype, const int32_t* offsets, int pooling, float* out, int64_t ldo,
                  int bounds_check, int32_t* err_count, void* stream) {
  FwdArgs a{};
  int rc = pack_meta(a.m, tables, T, features, F, B);
  if (rc) return rc;
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "pooled_fwd: ids must be int32/int64");
  if (pooling != TT_POOL_SUM && pooling != TT_POOL_MEAN) return fail(TT_EINVAL, "pooled_fwd: bad pooling");
  if (B == 0) return TT_OK;
  if (!weights || !offsets || !out) return fail(TT_EINVAL, "pooled_fwd: null pointer");
  if (bounds_check && !err_count) return fail(TT_EINVAL, "pooled_fwd: bounds_check needs err_count");
  int64_t blocks;
  rc = fwd_geometry(a, weights, out, ldo, B, &blocks);
  if (rc) return rc;
  pooled_fwd_kernel<<<dim3((unsigned)blocks), dim3(256), 0, as_stream(stream)>>>(
      weights, a, values, id_dtype, offsets, pooling, out, ldo, bounds_check, err_count);
  return check_launch("pooled_fwd");
}

int tt_pooled_fwd_cols(const float* weights, const tt_table_meta_t* tables, int T,
                       const tt_feature_meta_t* features, int F, int64_t B, const void* const* cols,
                       int id_dtype, const int64_t* num_embeddings, float* out, int64_t ldo, void* stream) {
  FwdArgs a{};
  int rc = pack_meta(a.m, tables, T, features, F, B);
  if (rc) return rc;
  ColArgs ca{};
  rc = pack_cols(ca, F, cols, num_embeddings, id_dtype);
  if (rc) return rc;
  for (int f = 0; f < F; ++f)
    if (num_embeddings[f] > tables[features[f].table].num_rows)
      return fail(TT_EINVAL, "pooled_fwd_cols: num_embeddings exceeds the table's rows");
  if (B == 0) return TT_OK;
  if (!weights || !out) return fail(TT_EINVAL, "pooled_fwd_cols: null pointer");
  int64_t blocks;
  rc = fwd_geometry(a, weights, out, ldo, B, &blocks);
  if (rc) return rc;
  pooled_fwd_cols_kernel<<<dim3((unsigned)blocks), dim3(256), 0, as_stream(stream)>>>(weights, a, ca, id_dtype,
                                                                                       out, ldo);
  return check_launch("pooled_fwd_cols");
}

size_t tt_bwd_workspace_bytes(int64_t max_lookups) {
  return bwd_layout(nullptr, std::max<int64_t>(1, max_lookups), nullptr);
}

int tt_bwd_workspace_init(void* workspace, size_t ws_bytes, int64_t max_lookups, void* stream) {
  if (max_lookups < 1) max_lookups = 1;
  if (!workspace || ws_bytes < tt_bwd_workspace_bytes(max_lookups))
    return fail(TT_ECAPACITY, "bwd_workspace_init: workspace too small");
  BwdWs w;
  bwd_layout(workspace, max_lookups, &w);
  hipStream_t st = as_stream(stream);
  if (hipMemsetAsync(w.keys, 0xff, sizeof(uint64_t) * w.cap, st) != hipSuccess ||
      hipMemsetAsync(w.cnt, 0, sizeof(int32_t) * w.cap, st) != hipSuccess ||
      hipMemsetAsync(w.U, 0, sizeof(int32_t) * 4, st) != hipSuccess)
    return fail(TT_EINVAL, "bwd_workspace_init: memset failed");
  return TT_OK;
}

static int launch_scan_scatter(const EmbMeta& m, const int32_t* offsets, BwdWs& w, hipStream_t st, int gb) {
  const int nb = (int)ceil_div(w.cap, 1024);
  bwd_scan_reduce_kernel<<<dim3(nb), dim3(256), 0, st>>>(w);
  bwd_scan_kernel<<<dim3(nb), dim3(256), 0, st>>>(w);
  if ((int64_t)m.F * m.B > 0) bwd_scatter_kernel<<<dim3(gb), dim3(256), 0, st>>>(m, offsets, w);
  return check_launch("bwd_prepare");
}

int tt_bwd_prepare(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F,
                   int64_t B, const void* values, int id_dtype, const int32_t* offsets,
                   int bounds_check, void* workspace, size_t ws_bytes, int64_t max_lookups,
                   void* stream) {
  EmbMeta m{};
  int rc = pack_meta(m, tables, T, features, F, B);
  if (rc) return rc;
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "bwd_prepare: ids must be int32/int64");
  if (max_lookups < 1) max_lookups = 1;
  rc = check_ws(workspace, ws_bytes, max_lookups, "bwd_prepare");
  if (rc) return rc;
  if (!offsets) return fail(TT_EINVAL, "bwd_prepare: null offsets");
  for (int t = 0; t < T; ++t)
    if (tables[t].num_rows >= (1ll << KEY_TABLE_SHIFT)) return fail(TT_EINVAL, "bwd_prepare: table rows >= 2^40");
  BwdWs w;
  bwd_layout(workspace, max_lookups, &w);
  hipStream_t st = as_stream(stream);
  const int64_t nbag = (int64_t)F * B;
  const int gb = (int)std::min<int64_t>(8192, std::max<int64_t>(1, ceil_div(nbag, 256)));
  if (nbag > 0) bwd_hash_kernel<<<dim3(gb), dim3(256), 0, st>>>(m, values, id_dtype, offsets, bounds_check, w);
  return launch_scan_scatter(m, offsets, w, st, gb);
}

int tt_bwd_prepare_cols(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F, int64_t B,
                        const void* const* cols, int id_dtype, const int64_t* num_embeddings, void* workspace,
                        size_t ws_bytes, int64_t max_lookups, void* stream) {
  EmbMeta m{};
  int rc = pack_meta(m, tables, T, features, F, B);
  if (rc) return rc;
  ColArgs ca{};
  rc = pack_cols(ca, F, cols, num_embeddings, id_dtype);
  if (rc) return rc;
  if (max_lookups < (int64_t)F * B) return fail(TT_ECAPACITY, "bwd_prepare_cols: max_lookups < F*B");
  rc = check_ws(workspace, ws_bytes, max_lookups, "bwd_prepare_cols");
  if (rc) return rc;
  for (int f = 0; f < F; ++f)
    if (num_embeddings[f] > tables[features[f].table].num_rows)
      return fail(TT_EINVAL, "bwd_prepare_cols: num_embeddings exceeds the table's rows");
  BwdWs w;
  bwd_layout(workspace, max_lookups, &w);
  hipStream_t st = as_stream(stream);
  const int64_t nbag = (int64_t)F * B;
  const int gb = (int)std::min<int64_t>(8192, std::max<int64_t>(1, ceil_div(nbag, 256)));
  // one wave per workgroup: the inserts are latency-bound round trips, spread them over all CUs
  const int gh = (int)std::min<int64_t>(32768, std::max<int64_t>(1, ceil_div(nbag, 64)));
  if (nbag > 0) bwd_hash_cols_kernel<<<dim3(gh), dim3(64), 0, st>>>(m, ca, id_dtype, w);
  return launch_scan_scatter(m, nullptr, w, st, gb);
}

int tt_bwd_rowwise_adagrad(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features,
                           int F, int64_t B, const float* grad_out, int64_t ldg,
                           const int32_t* offsets, int pooling, float* weights, float* state,
                           float lr, float eps, void* workspace, size_t ws_bytes,
                           int64_t max_lookups, void* stream) {
  EmbMeta m{};
  int rc = pack_meta(m, tables, T, features, F, B);
  if (rc) return rc;
  if (max_lookups < 1) max_lookups = 1;
  rc = check_ws(workspace, ws_bytes, max_lookups, "bwd_rowwise_adagrad");
  if (rc) return rc;
  if (pooling != TT_POOL_SUM && pooling != TT_POOL_MEAN) return fail(TT_EINVAL, "bwd_rowwise_adagrad: bad pooling");
  if (!grad_out || !weights || !state) return fail(TT_EINVAL, "bwd_rowwise_adagrad: null pointer");
  if (pooling == TT_POOL_MEAN && !offsets) return fail(TT_EINVAL, "bwd_rowwise_adagrad: MEAN pooling needs offsets");
  bool vec_ok = (ldg % 4 == 0) && ((reinterpret_cast<uintptr_t>(grad_out) & 15) == 0) &&
                ((reinterpret_cast<uintptr_t>(weights) & 15) == 0);
  for (int t = 0; t < T; ++t)
    if (tables[t].weight_offset % 4) vec_ok = false;
  for (int f = 0; f < F; ++f)
    if (features[f].out_offset % 4) vec_ok = false;
  bool narrow = vec_ok;
  for (int t = 0; t < T; ++t) {
    const int D = tables[t].dim;
    if (D > 128 || D % 4) narrow = false;
    // generic path's per-row choice: float4 (D%4==0, D>=256, D<=1024), float2 (D even, D<=512),
    // scalar (D<=256)
    const bool v4 = vec_ok && D % 4 == 0 && D >= 256;
    const bool v2 = vec_ok && D % 2 == 0 && !v4;
    const int cap = v4 ? 1024 : (v2 ? 512 : 256);
    if (D > cap) return fail(TT_EINVAL, "bwd_rowwise_adagrad: unaligned dim > 256 unsupported");
  }
  BwdWs w;
  bwd_layout(workspace, max_lookups, &w);
  hipStream_t st = as_stream(stream);
  if (narrow) {
    const int grid = (int)std::min<int64_t>(8192, std::max<int64_t>(1, ceil_div(max_lookups, 8)));
    bwd_adagrad_narrow_kernel<<<dim3(grid), dim3(256), 0, st>>>(m, grad_out, ldg, offsets, pooling, weights, state,
                                                                lr, eps, w);
  } else {
    const int grid = (int)std::min<int64_t>(16384, std::max<int64_t>(1, ceil_div(max_lookups, 4)));
    bwd_adagrad_kernel<<<dim3(grid), dim3(256), 0, st>>>(m, grad_out, ldg, offsets, pooling, weights, state, lr, eps,
                                                         w, vec_ok ? 1 : 0);
  }
  if (max_lookups >= HOT_MIN) {
    const int hgrid = (int)std::min<int64_t>(512, max_lookups / HOT_MIN);
    bwd_adagrad_hot_kernel<<<dim3(hgrid), dim3(256), 0, st>>>(m, grad_out, ldg, offsets, pooling, weights, state,
                                                              lr, eps, w);
  }
  return check_launch("bwd_rowwise_adagrad");
}

int tt_pooled_bwd_dense(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features,
                        int F, int64_t B, const float* grad_out, int64_t ldg, const void* values,
                        int id_dtype, const int32_t* offsets, int pooling, float* grad_weights,
                        int bounds_check, void* stream) {
  EmbMeta m{};
  int rc = pack_meta(m, tables, T, features, F, B);
  if (rc) return rc;
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "pooled_bwd_dense: bad id dtype");
  if ((int64_t)F * B == 0) return TT_OK;
  if (!grad_out || !grad_weights || !offsets) return fail(TT_EINVAL, "pooled_bwd_dense: null pointer");
  const int grid = (int)std::min<int64_t>(16384, std::max<int64_t>(1, ceil_div((int64_t)F * B, 4)));
  bwd_dense_kernel<<<dim3(grid), dim3(256), 0, as_stream(stream)>>>(m, grad_out, ldg, values, id_dtype, offsets,
                                                                    pooling, grad_weights, bounds_check);
  return check_launch("pooled_bwd_dense");
}

}  // extern "C"

namespace tt {
static int check_ws(void* workspace, size_t ws_bytes, int64_t max_lookups, const char* what) {
  if (max_lookups > INT32_MAX / 2) return fail(TT_EINVAL, std::string(what) + ": max_lookups too large");
  if (!workspace || ws_bytes < tt_bwd_workspace_bytes(max_lookups))
    return fail(TT_ECAPACITY, std::string(what) + ": workspace too small");
  return TT_OK;
}
}  // namespace tt

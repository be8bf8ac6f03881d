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

// Fast path (float4 columns, the whole row in one pass of the group: D <= 4 G): the group's lanes
// load up to G ids of the bag at once (one coalesced read), broadcast them by lane shuffles, and
// keep FWD_INFLIGHT rows in flight per lane; rows are still added in bag order.
constexpr int FWD_INFLIGHT = 8;

__device__ __forceinline__ void pool_bag_row4(const float* __restrict__ w, const void* __restrict__ values,
                                              int id_dtype, int64_t s, int64_t e, int64_t rows, int D,
                                              int lane_g, int G, float scale, float* __restrict__ out,
                                              int bounds_check, int32_t* err) {
  const int gbase = (threadIdx.x & 63) & ~(G - 1);
  const bool col_ok = lane_g * 4 < D;
  f32x4v acc = (f32x4v)(0.f);
  for (int64_t j0 = s; j0 < e; j0 += G) {
    const int cnt = (int)min((int64_t)G, e - j0);
    int64_t myid = 0;
    if (lane_g < cnt) {
      myid = load_id(values, id_dtype, j0 + lane_g);
      if (bounds_check && (uint64_t)myid >= (uint64_t)rows) {
        atomicAdd(err, 1);
        myid = 0;
      }
    }
    for (int k = 0; k < cnt; k += FWD_INFLIGHT) {
      f32x4v r[FWD_INFLIGHT];
#pragma unroll
      for (int u = 0; u < FWD_INFLIGHT; ++u) {
        const int64_t id = __shfl(myid, gbase + min(k + u, G - 1), 64);
        r[u] = (col_ok && k + u < cnt) ? *reinterpret_cast<const f32x4v*>(w + id * D + lane_g * 4) : (f32x4v)(0.f);
      }
#pragma unroll
      for (int u = 0; u < FWD_INFLIGHT; ++u)
        if (k + u < cnt) acc += r[u];
    }
  }
  if (col_ok) *reinterpret_cast<f32x4v*>(out + lane_g * 4) = acc * scale;
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
  if (a.vec[f] == 4 && tm.dim <= 4 * G)
    pool_bag_row4(w, values, id_dtype, s, e, tm.num_rows, tm.dim, lane_g, G, scale, o, bounds_check, err);
  else if (a.vec[f] == 4)
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
// Global hash slot word of the KJT-form grouping: (table << 34 | row) << 24 | lookup count, so ONE
// CAS claims a free slot with its count and a repeat key adds to the same word (rows < 2^34 - 1,
// < 2^24 lookups per step; checked on the host).
constexpr int PK_CNT_BITS = 24;
constexpr int PK_ROW_BITS = 34;
constexpr uint64_t PK_CNT_MASK = (1ull << PK_CNT_BITS) - 1;
__device__ __forceinline__ uint64_t pk_key(int t, uint64_t row) { return ((uint64_t)t << PK_ROW_BITS) | row; }
__device__ __forceinline__ uint64_t pk_to_key(uint64_t word) {  // slot word -> table << 40 | row
  const uint64_t k = word >> PK_CNT_BITS;
  return ((k >> PK_ROW_BITS) << KEY_TABLE_SHIFT) | (k & ((1ull << PK_ROW_BITS) - 1));
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// Rows looked up more than HOT_MIN - 1 times in a step are "hot": the per-row kernels (which sort
// a segment of <= 32 bag ids in registers) skip them; bwd_hot_partial_kernel / bwd_hot_final_kernel
// sum them in a canonical order (bag-id ranges, ascending bag id inside a range, see below).
constexpr int HOT_MIN = 33;
// A hot row is split into NR bag-id ranges summed by separate workgroups (NR = 1 up to HOT_SPLIT
// lookups, at most HOT_NR_MAX); range r of NB bags is [r*NB/NR, (r+1)*NB/NR), so the split depends
// on the lookup count and the batch shape only.
constexpr int HOT_SPLIT = 512;
constexpr int HOT_NR_MAX = 64;
constexpr int HOT_WIN = 8192;   // bags counted per LDS pass of bwd_hot_partial_kernel
constexpr int HOT_DMAX = 1024;  // partial row stride (floats)
// Tiled grouping of KJT lookups (bwd_tile_hash_kernel / bwd_tile_scatter_kernel): a workgroup owns
// TILE_BAGS bags and walks their lookups in chunks of TILE_CH; a chunk's duplicate ids are merged in
// an LDS hash first, so the global hash and the segment cursors see one atomic per (chunk, row)
// instead of one per lookup (a Zipf-hot row costs a few hundred same-address atomics, not 10^5).
constexpr int TILE_BAGS = 16;
constexpr int TILE_CH = 1024;
constexpr int TILE_HS = 2048;  // LDS hash slots per chunk (load <= 1/2)

struct URec {
  uint64_t key;
  int32_t seg;  // first position of the row's bag ids in perm; the bag id itself when len == 1
  int32_t len;
};

struct HotRec {
  int32_t u;      // unique-row index
  int32_t pbase;  // first work item (bwd_hot_partial_kernel) / partial row of this hot row
  int32_t nr;     // bag-id ranges
  int32_t pad;
};

struct BwdWs {
  uint64_t* keys;   // [cap] hash keys (EMPTY when free; cleaned by k2b)
  int32_t* cnt;     // [cap] lookups of the slot's row this step (written by k2b)
  int32_t* cur;     // [cap] scatter cursor per slot (set by k2b)
  int32_t* slot_of; // [L]   slot of each lookup (-1: none; column form)
  int32_t* perm;    // [L]   bag ids grouped by unique row
  URec* urec;       // [L]   per unique row
  int32_t* lk;      // [L]   tiled form: chunk entry | rank in entry << 16, per lookup
  int32_t* ent_h;   // [L]   tiled form: global slot of chunk entry d, at [chunk start + d]
  int32_t* ent_c;   // [L]   tiled form: lookups of chunk entry d
  int32_t* ent_n;   // [L]   tiled form: entries of the chunk starting at this lookup
  int32_t* bsum_u;  // [nb]  scan partials (unique count)
  int32_t* bsum_c;  // [nb]  scan partials (lookup count)
  int32_t* bsum_m;  // [nb]  scan partials (rows looked up more than once)
  HotRec* hot;      // [L/HOT_MIN + 1] hot rows
  float* hotp;      // [hot items][HOT_DMAX] partial sums of split hot rows
  int32_t* U;       // [8]   {unique rows, KJT-form flag, hot work items, hot rows (U[2..3]: one 64-bit word),
                    //        rows looked up more than once (their records come first), -, -, -}
  int64_t* vmeta;   // [2]   KJT form: the step's values pointer and id dtype (for the direct update)
  int64_t cap;
  int64_t L;
};

constexpr int SCAN_TILE = 4096;  // hash slots per workgroup of k2b

static int64_t bwd_cap(int64_t L) {
  int64_t c = SCAN_TILE;
  while (c < 2 * L) c <<= 1;
  return c;
}

// hot work items <= hot rows + sum over split rows of ceil(c / HOT_SPLIT) <= L/HOT_MIN + 2L/HOT_SPLIT
static int64_t hot_items_max(int64_t L) { return L / HOT_MIN + 2 * ceil_div(L, HOT_SPLIT) + 1; }

__host__ __device__ __forceinline__ int hot_nr(int c) {
  if (c <= HOT_SPLIT) return 1;
  const int n = (c + HOT_SPLIT - 1) / HOT_SPLIT;
  return n < HOT_NR_MAX ? n : HOT_NR_MAX;
}

static size_t bwd_layout(void* base, int64_t L, BwdWs* w) {
  const int64_t cap = bwd_cap(L);
  const int64_t nb = ceil_div(cap, SCAN_TILE);
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
  t.lk = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.ent_h = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.ent_c = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.ent_n = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.bsum_u = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * nb));
  t.bsum_c = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * nb));
  t.bsum_m = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * nb));
  t.hot = reinterpret_cast<HotRec*>(take(sizeof(HotRec) * (L / HOT_MIN + 1)));
  t.hotp = reinterpret_cast<float*>(take(sizeof(float) * HOT_DMAX * hot_items_max(L)));
  t.U = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * 8));
  t.vmeta = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * 2));
  t.cap = cap;
  t.L = L;
  if (w) *w = t;
  return off;
}

__device__ __forceinline__ int32_t hash_insert(BwdWs& ws, uint64_t pk) {
  // one returning CAS per probe: it claims an empty slot (count 1) or reports who holds it
  const uint64_t mask = (uint64_t)ws.cap - 1;
  uint64_t h = mix64(pk) & mask;
  while (true) {
    const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&ws.keys[h]),
                                    (unsigned long long)EMPTY_KEY, (unsigned long long)((pk << PK_CNT_BITS) | 1));
    if (prev == EMPTY_KEY) break;
    if ((prev >> PK_CNT_BITS) == pk) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&ws.keys[h]), 1ull);
      break;
    }
    h = (h + 1) & mask;
  }
  return (int32_t)h;
}

// Block-wide exclusive scan of one int per thread (256 threads); *total = the block's sum.
__device__ __forceinline__ int block_excl_scan(int v, int* red, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  __syncthreads();
  if (lane == 63) red[wid] = inc;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    base += w < wid ? red[w] : 0;
    tot += red[w];
  }
  *total = tot;
  return base + inc - v;
}

// local bag of lookup j: the largest i < nb with off[i] <= j (off[0] <= j < off[nb])
__device__ __forceinline__ int lds_bag_of(const int32_t* off, int nb, int64_t j) {
  int lo = 0, hi = nb;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)off[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// k2a (KJT form): workgroup per TILE_BAGS bags, their lookups in chunks of TILE_CH. Per chunk:
// (1) every lookup joins its (table,row) entry of an LDS hash (rank = its LDS count ticket);
// (2) the entries are compacted (dense index d, ascending LDS slot) and each is inserted ONCE into
//     the global hash with its count: all of a thread's first-probe CASes are issued together,
//     collisions retried in rounds;
// (3) per lookup lk = d | rank << 16; per entry ent_h / ent_c at [chunk start + d], ent_n at the
//     chunk start. k2c turns (entry base + rank) into the lookup's position in its row's segment.
constexpr int TILE_EPT = TILE_CH / 256;  // lookups (and at most entries) per thread
constexpr int TILE_SPT = TILE_HS / 256;  // LDS hash slots per thread in the compaction

__global__ void __launch_bounds__(256) bwd_tile_hash_kernel(EmbMeta m, const void* __restrict__ values, int id_dtype,
                                                            const int32_t* __restrict__ offsets, int bounds_check,
                                                            BwdWs ws) {
  __shared__ unsigned long long hkey[TILE_HS];
  __shared__ int hcnt[TILE_HS];
  __shared__ int16_t hmap[TILE_HS];
  __shared__ int32_t off[TILE_BAGS + 1];
  __shared__ int red[4];
  const int tid = threadIdx.x;
  const int64_t NB = (int64_t)m.F * m.B;
  const int64_t b0 = (int64_t)xcd_remap((int)blockIdx.x, (int)gridDim.x) * TILE_BAGS;  // a contiguous 1/8 per XCD
  const int nb = (int)min((int64_t)TILE_BAGS, NB - b0);
  if (tid <= nb) off[tid] = offsets[b0 + tid];
  for (int i = tid; i < TILE_HS; i += 256) {
    hkey[i] = EMPTY_KEY;
    hcnt[i] = 0;
  }
  __syncthreads();
  const int64_t s0 = off[0], e0 = off[nb];
  const uint64_t gmask = (uint64_t)ws.cap - 1;
  if (blockIdx.x == 0 && tid == 0) {
    ws.vmeta[0] = reinterpret_cast<int64_t>(values);
    ws.vmeta[1] = id_dtype;
  }
  for (int64_t j0 = s0; j0 < e0; j0 += TILE_CH) {
    const int n = (int)min((int64_t)TILE_CH, e0 - j0);
    int pos[TILE_EPT], rk[TILE_EPT];
    int64_t idv[TILE_EPT];
    int tv[TILE_EPT];
#pragma unroll
    for (int q = 0; q < TILE_EPT; ++q) {  // all id loads first
      const int i = q * 256 + tid;
      tv[q] = -1;
      if (i < n) {
        const int64_t j = j0 + i;
        const int f = (int)((b0 + lds_bag_of(off, nb, j)) / m.B);
        tv[q] = m.features[f].table;
        idv[q] = load_id(values, id_dtype, j);
      }
    }
#pragma unroll
    for (int q = 0; q < TILE_EPT; ++q) {
      pos[q] = -1;
      if (tv[q] >= 0) {
        int64_t id = idv[q];
        if (bounds_check && (uint64_t)id >= (uint64_t)m.tables[tv[q]].num_rows) id = 0;
        const unsigned long long key = pk_key(tv[q], (uint64_t)id);
        unsigned h = (unsigned)mix64(key) & (TILE_HS - 1);
        while (true) {
          const unsigned long long prev = atomicCAS(&hkey[h], (unsigned long long)EMPTY_KEY, key);
          if (prev == EMPTY_KEY || prev == key) break;
          h = (h + 1) & (TILE_HS - 1);
        }
        pos[q] = (int)h;
        rk[q] = atomicAdd(&hcnt[h], 1);
      }
    }
    __syncthreads();
    // (2) compaction: thread owns slots [tid*SPT, tid*SPT+SPT)
    unsigned long long ck[TILE_SPT];
    int cc[TILE_SPT], k = 0;
#pragma unroll
    for (int v = 0; v < TILE_SPT; ++v) {
      cc[v] = hcnt[tid * TILE_SPT + v];
      ck[v] = hkey[tid * TILE_SPT + v];
      k += cc[v] > 0;
    }
    int tot;
    int d = block_excl_scan(k, red, &tot);  // its barriers order the reads above before the writes below
#pragma unroll
    for (int v = 0; v < TILE_SPT; ++v) {
      if (cc[v] > 0) {
        hmap[tid * TILE_SPT + v] = (int16_t)d;
        hkey[d] = ck[v];  // compacted in place (d <= slot index)
        hcnt[d] = cc[v];
        ++d;
      }
    }
    __syncthreads();
    // global insert: entries tid, tid+256, ... (<= TILE_EPT per thread); first probes issued together
    unsigned long long ekey[TILE_EPT];
    uint32_t eh[TILE_EPT];
    bool todo[TILE_EPT];
#pragma unroll
    for (int q = 0; q < TILE_EPT; ++q) {
      const int e = q * 256 + tid;
      todo[q] = e < tot;
      ekey[q] = todo[q] ? hkey[e] : 0ull;
      eh[q] = (uint32_t)(mix64(ekey[q]) & gmask);
    }
    int ecnt[TILE_EPT];
#pragma unroll
    for (int q = 0; q < TILE_EPT; ++q) ecnt[q] = todo[q] ? hcnt[q * 256 + tid] : 0;
    bool any = true;
    while (any) {
      unsigned long long prev[TILE_EPT];
#pragma unroll
      for (int q = 0; q < TILE_EPT; ++q)
        if (todo[q])
          prev[q] = atomicCAS(reinterpret_cast<unsigned long long*>(&ws.keys[eh[q]]), (unsigned long long)EMPTY_KEY,
                              (ekey[q] << PK_CNT_BITS) | (unsigned long long)ecnt[q]);
      any = false;
#pragma unroll
      for (int q = 0; q < TILE_EPT; ++q) {
        if (!todo[q]) continue;
        const bool mine = prev[q] == EMPTY_KEY;
        if (mine || (prev[q] >> PK_CNT_BITS) == ekey[q]) {
          const int e = q * 256 + tid;
          const int c = ecnt[q];
          if (!mine) atomicAdd(reinterpret_cast<unsigned long long*>(&ws.keys[eh[q]]), (unsigned long long)c);
          ws.ent_h[j0 + e] = (int32_t)eh[q];
          ws.ent_c[j0 + e] = c;
          todo[q] = false;
        } else {
          eh[q] = (uint32_t)((eh[q] + 1) & gmask);
          any = true;
        }
      }
    }
    if (tid == 0) ws.ent_n[j0] = tot;
#pragma unroll
    for (int q = 0; q < TILE_EPT; ++q)
      if (pos[q] >= 0) ws.lk[j0 + q * 256 + tid] = (int32_t)hmap[pos[q]] | (rk[q] << 16);
    __syncthreads();
    if (j0 + TILE_CH < e0) {
      for (int i = tid; i < TILE_HS; i += 256) {
        hkey[i] = EMPTY_KEY;
        hcnt[i] = 0;
      }
      __syncthreads();
    }
  }
}

constexpr int SINGLE_MARK = (int)0x80000000;  // lk sign bit: the lookup's row is looked up once

// k2c (KJT form): per chunk, one cursor atomic per entry reserves its run in the row's segment,
// then every lookup writes its bag id at (run base + rank).
__global__ void __launch_bounds__(256) bwd_tile_scatter_kernel(EmbMeta m, const int32_t* __restrict__ offsets,
                                                               BwdWs ws) {
  __shared__ int32_t off[TILE_BAGS + 1];
  __shared__ int lbase[TILE_CH];
  const int tid = threadIdx.x;
  const int64_t NB = (int64_t)m.F * m.B;
  const int64_t b0 = (int64_t)xcd_remap((int)blockIdx.x, (int)gridDim.x) * TILE_BAGS;  // as the hash kernel
  const int nb = (int)min((int64_t)TILE_BAGS, NB - b0);
  if (tid <= nb) off[tid] = offsets[b0 + tid];
  __syncthreads();
  const int64_t s0 = off[0], e0 = off[nb];
  for (int64_t j0 = s0; j0 < e0; j0 += TILE_CH) {
    const int n = (int)min((int64_t)TILE_CH, e0 - j0);
    const int ne = ws.ent_n[j0];
    int hb[TILE_EPT], cb[TILE_EPT];
#pragma unroll
    for (int q = 0; q < TILE_EPT; ++q) {
      const int e = q * 256 + tid;
      hb[q] = e < ne ? ws.ent_h[j0 + e] : -1;
      cb[q] = e < ne ? ws.ent_c[j0 + e] : 0;
    }
    int ln[TILE_EPT];
#pragma unroll
    for (int q = 0; q < TILE_EPT; ++q) ln[q] = hb[q] >= 0 ? ws.cnt[hb[q]] : 0;
    // a row whose lookups all sit in this chunk owns its whole segment: no cursor atomic; a row
    // looked up once gets no segment at all: its lookup is marked (lk sign bit) and updated in
    // lookup order by bwd_adagrad_direct_kernel
#pragma unroll
    for (int q = 0; q < TILE_EPT; ++q)
      if (hb[q] >= 0)
        lbase[q * 256 + tid] = ln[q] == cb[q] ? (ln[q] == 1 ? SINGLE_MARK : ws.cur[hb[q]])
                                              : atomicAdd(&ws.cur[hb[q]], cb[q]);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < TILE_EPT; ++q) {
      const int i = q * 256 + tid;
      if (i < n) {
        const int v = ws.lk[j0 + i];
        const int lb = lbase[v & 0xffff];
        if (lb == SINGLE_MARK) ws.lk[j0 + i] = v | SINGLE_MARK;
        else ws.perm[lb + (v >> 16)] = (int32_t)(b0 + lds_bag_of(off, nb, j0 + i));
      }
    }
    __syncthreads();
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
      h = hash_insert(ws, pk_key(t, (uint64_t)py_mod64(id, ca.num_emb[f])));
    }
    ws.slot_of[bag] = h;
  }
}

__device__ __forceinline__ int slot_count(uint64_t w) { return w == EMPTY_KEY ? 0 : (int)(w & PK_CNT_MASK); }

// k2b-1: per SCAN_TILE-slot tile: number of occupied slots and of lookups
__global__ void __launch_bounds__(256) bwd_scan_reduce_kernel(BwdWs ws, int tiled) {
  __shared__ int lu[4], lc[4], lm[4];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  int su = 0, sc = 0, sm = 0;
#pragma unroll
  for (int j = 0; j < SCAN_TILE / 256; ++j) {
    const int c = slot_count(ws.keys[base + j * 256 + threadIdx.x]);
    su += c > 0;
    sc += c;
    sm += c > 1;
  }
  su = wave_sum_i(su);
  sc = wave_sum_i(sc);
  sm = wave_sum_i(sm);
  if ((threadIdx.x & 63) == 0) {
    lu[threadIdx.x >> 6] = su;
    lc[threadIdx.x >> 6] = sc;
    lm[threadIdx.x >> 6] = sm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ws.bsum_u[blockIdx.x] = lu[0] + lu[1] + lu[2] + lu[3];
    ws.bsum_c[blockIdx.x] = lc[0] + lc[1] + lc[2] + lc[3];
    ws.bsum_m[blockIdx.x] = lm[0] + lm[1] + lm[2] + lm[3];
    if (blockIdx.x == 0) {
      *reinterpret_cast<unsigned long long*>(ws.U + 2) = 0ull;  // hot list, filled by k2b-2
      ws.U[1] = tiled;  // 1: KJT-form grouping (once-looked-up lookups marked in lk, see k2c)
    }
  }
}

// k2b-2: exclusive scans -> record {key, segment start, count} per unique row; cursor per slot;
// the slot's key and count are reset here, so the table is clean for the next step's k2a.
__global__ void __launch_bounds__(256) bwd_scan_kernel(BwdWs ws) {
  __shared__ int lds[20];
  __shared__ uint64_t tile[SCAN_TILE + SCAN_TILE / 16];  // the block's slot words (padded: no bank conflicts)
  // prefixes over the previous blocks (unique rows, lookups, multi rows) and the totals (U, M)
  int pu = 0, pc = 0, pm = 0, tU = 0, tM = 0;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += 256) {
    const int bu = ws.bsum_u[i], bm = ws.bsum_m[i];
    if (i < (int)blockIdx.x) {
      pu += bu;
      pc += ws.bsum_c[i];
      pm += bm;
    }
    tU += bu;
    tM += bm;
  }
  pu = wave_sum_i(pu);
  pc = wave_sum_i(pc);
  pm = wave_sum_i(pm);
  tU = wave_sum_i(tU);
  tM = wave_sum_i(tM);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    lds[wid] = pu;
    lds[4 + wid] = pc;
    lds[8 + wid] = pm;
    lds[12 + wid] = tU;
    lds[16 + wid] = tM;
  }
  __syncthreads();
  pu = lds[0] + lds[1] + lds[2] + lds[3];
  pc = lds[4] + lds[5] + lds[6] + lds[7];
  pm = lds[8] + lds[9] + lds[10] + lds[11];
  tU = lds[12] + lds[13] + lds[14] + lds[15];
  tM = lds[16] + lds[17] + lds[18] + lds[19];
  __syncthreads();
  constexpr int SPT = SCAN_TILE / 256;
  const int64_t tbase = (int64_t)blockIdx.x * SCAN_TILE;
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int idx = j * 256 + threadIdx.x;
    tile[idx + idx / 16] = ws.keys[tbase + idx];
    ws.keys[tbase + j * 256 + threadIdx.x] = EMPTY_KEY;  // clean for the next step's k2a
  }
  __syncthreads();
  const int64_t base = tbase + threadIdx.x * SPT;
  int c[SPT], lu = 0, lcnt = 0;
  uint64_t wd[SPT];
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    wd[j] = tile[threadIdx.x * (SPT + 1) + j];
    c[j] = slot_count(wd[j]);
    lu += c[j] > 0;
    lcnt += c[j];
  }
  int lmul = 0;
#pragma unroll
  for (int j = 0; j < SPT; ++j) lmul += c[j] > 1;
  int iu = lu, ic = lcnt, im = lmul;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int yu = __shfl_up(iu, o, 64), yc = __shfl_up(ic, o, 64), ym = __shfl_up(im, o, 64);
    if (lane >= o) {
      iu += yu;
      ic += yc;
      im += ym;
    }
  }
  if (lane == 63) {
    lds[wid] = iu;
    lds[4 + wid] = ic;
    lds[8 + wid] = im;
  }
  __syncthreads();
  int wu = 0, wc = 0, wm = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    if (w < wid) {
      wu += lds[w];
      wc += lds[4 + w];
      wm += lds[8 + w];
    }
  }
  // records: rows looked up more than once first (in slot order), then the once-looked-up rows
  // from the end of the record array (in reverse slot order), so the per-row kernels of the KJT
  // form visit only the first M records
  int em = pm + wm + im - lmul;                                   // multi rows before this thread's
  int es = (pu - pm) + (wu - wm) + (iu - lu) - (im - lmul);      // single rows before this thread's
  int ec = pc + wc + ic - lcnt;
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    if (c[j] > 0) {
      const int64_t h = base + j;
      const int eu = c[j] > 1 ? em++ : tU - 1 - es++;
      URec rec;
      rec.key = pk_to_key(wd[j]);
      rec.seg = ec;
      rec.len = c[j];
      ws.urec[eu] = rec;
      if (c[j] >= HOT_MIN) {  // one 64-bit atomic: hot-row index (high word) and first work item (low)
        const int nr = hot_nr(c[j]);
        const unsigned long long pk =
            atomicAdd(reinterpret_cast<unsigned long long*>(ws.U + 2), (1ull << 32) | (unsigned long long)nr);
        ws.hot[(int)(pk >> 32)] = HotRec{eu, (int32_t)(pk & 0xffffffffull), nr, 0};
      }
      ws.cur[h] = c[j] == 1 ? eu : ec;  // a single lookup's bag goes into its record (k2c)
      ws.cnt[h] = c[j];
      ec += c[j];
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    ws.U[0] = tU;
    ws.U[4] = tM;
  }
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
      if (ws.cnt[h] == 1) {
        ws.urec[ws.cur[h]].seg = (int32_t)bag;
      } else {
        const int pos = atomicAdd(&ws.cur[h], 1);
        ws.perm[pos] = (int32_t)bag;
      }
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

// Table / feature metadata staged in LDS at block start: indexing the kernel-argument copy with a
// per-lane index is a vector load from the kernarg segment (one more dependent hop per row).
struct LdsMeta {
  tt_table_meta_t tab[TT_MAX_TABLES];
  tt_feature_meta_t feat[TT_MAX_FEATURES];
};

__device__ __forceinline__ void stage_meta(const EmbMeta& m, LdsMeta& lm) {
  for (int i = threadIdx.x; i < m.T; i += blockDim.x) lm.tab[i] = m.tables[i];
  for (int i = threadIdx.x; i < m.F; i += blockDim.x) lm.feat[i] = m.features[i];
  __syncthreads();
}

struct BagRow {
  const float* g;
  int64_t B;
  int64_t ldg;
  const tt_feature_meta_t* feats;
  __device__ __forceinline__ const float* row(int bag) const {
    const int f = (int)((uint32_t)bag / (uint32_t)B);  // bag ids < F * B < 2^31: 32-bit division
    const int64_t b = bag - (int64_t)f * B;
    return g + (feats[f].out_row + b) * ldg + feats[f].out_offset;
  }
};

// ---- k2d narrow: half-wave per unique row, D <= 128, D % 4 == 0 ----------------------------
// 32 lanes x float4 = one 512-B row; two rows per wave, many waves (the update is bound by the
// number of independent row chains in flight: measured, a deeper per-wave pipeline with fewer
// waves was slower). A row looked up once has its bag in its record (no perm hop); segments of
// 2..32 lookups are summed in ascending bag order (bitonic over the half-wave): bitwise reproducible.
__global__ void __launch_bounds__(256) bwd_adagrad_narrow_kernel(EmbMeta m, const float* __restrict__ grad_out,
                                                                 int64_t ldg, const int32_t* __restrict__ offsets,
                                                                 int pooling, float* __restrict__ weights,
                                                                 float* __restrict__ state, float lr, float eps,
                                                                 BwdWs ws) {
  __shared__ LdsMeta lm;
  stage_meta(m, lm);
  const int lane = threadIdx.x & 63;
  const int hl = lane & 31, half = lane >> 5;
  const BagRow br{grad_out, m.B, ldg, lm.feat};
  const bool direct = ws.U[1] != 0;
  const int U = direct ? ws.U[4] : ws.U[0];  // direct: the once-looked-up rows are not visited at all
  const int64_t nhalf = (int64_t)gridDim.x * 8;
  for (int64_t u = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + half; u - half < U; u += nhalf) {
    URec rec{0, 0, 0};
    if (u < U) rec = ws.urec[u];
    // hot rows: bwd_hot_partial_kernel; once-looked-up rows of the KJT form: bwd_adagrad_direct_kernel
    const bool active = u < U && rec.len < HOT_MIN && !(direct && rec.len == 1);
    if (!active) rec = URec{0, 0, 0};
    const int t = (int)(rec.key >> KEY_TABLE_SHIFT);
    const int64_t r = (int64_t)(rec.key & ((1ull << KEY_TABLE_SHIFT) - 1));
    const tt_table_meta_t tm = lm.tab[active ? t : 0];
    const int D = tm.dim;
    const bool col_ok = active && hl * 4 < D;
    float* wrow = weights + tm.weight_offset + r * D;
    float* srow = state + tm.state_offset + r;
    const int n = rec.len;
    // once-looked-up row: its gradient row is known now, fetched with the weight row and state
    const int b1 = n == 1 ? rec.seg : 0;
    f32x4v g = (col_ok && n == 1) ? *reinterpret_cast<const f32x4v*>(br.row(b1) + hl * 4) : (f32x4v)(0.f);
    f32x4v wv = col_ok ? *reinterpret_cast<const f32x4v*>(wrow + hl * 4) : (f32x4v)(0.f);
    const float s_old = active ? *srow : 0.f;
    if (pooling == TT_POOL_MEAN && n == 1) g *= 1.f / (float)max(1, offsets[b1 + 1] - offsets[b1]);
    const int nmax = max(n, __shfl_xor(n, 32, 64));
    if (nmax > 1) {  // ascending bag order (bitonic over the half-wave), fp32: bitwise reproducible
      const bool many = n > 1;
      int mine = (many && hl < n) ? ws.perm[rec.seg + hl] : 0x7fffffff;
      mine = bitonic_sort<32>(mine);
      for (int i = 0; i < nmax; i += 2) {
        const int b0 = __shfl(mine, (lane & 32) + i, 64);
        const int bb = __shfl(mine, (lane & 32) + min(i + 1, 31), 64);
        const bool v0 = many && i < n, v1 = many && i + 1 < n;
        f32x4v x0 = (f32x4v)(0.f), x1 = (f32x4v)(0.f);
        if (col_ok && v0) x0 = *reinterpret_cast<const f32x4v*>(br.row(b0) + hl * 4);
        if (col_ok && v1) x1 = *reinterpret_cast<const f32x4v*>(br.row(bb) + hl * 4);
        if (pooling == TT_POOL_MEAN) {
          if (v0) x0 *= 1.f / (float)max(1, offsets[b0 + 1] - offsets[b0]);
          if (v1) x1 *= 1.f / (float)max(1, offsets[bb + 1] - offsets[bb]);
        }
        if (v0) g += x0;
        if (v1) g += x1;
      }
    }
    // row-wise Adagrad: s += mean(G^2); w += G * (-lr / (sqrt(s) + eps)) (rw_step, tt_common.h)
    float sq = g[0] * g[0] + g[1] * g[1] + g[2] * g[2] + g[3] * g[3];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
    if (active) {
      const float snew = s_old + sq / (float)D;
      const float step = rw_step(snew, lr, eps);
      if (col_ok) {
#pragma unroll
        for (int v = 0; v < 4; ++v) wv[v] = fmaf(g[v], step, wv[v]);
        *reinterpret_cast<f32x4v*>(wrow + hl * 4) = wv;
      }
      if (hl == 0) *srow = snew;
    }
  }
}

// ---- k2d direct (KJT form, D <= 128): once-looked-up rows in lookup order --------------------
// Most rows of a uniform multi-hot batch are looked up once. Their lookups (marked by k2c) are
// updated straight from the bag walk: half-wave per lookup, consecutive lookups share their bag's
// gradient row (cache hits instead of a random gradient-row read per row), no record / segment
// indirection. Four lookups per half-wave in flight. The row is the hash's row: ids >= rows -> 0.
__global__ void __launch_bounds__(256) bwd_adagrad_direct_kernel(EmbMeta m, const float* __restrict__ grad_out,
                                                                 int64_t ldg, const int32_t* __restrict__ offsets,
                                                                 int pooling, float* __restrict__ weights,
                                                                 float* __restrict__ state, float lr, float eps,
                                                                 BwdWs ws) {
  if (ws.U[1] == 0) return;
  __shared__ int32_t off[TILE_BAGS + 1];
  __shared__ LdsMeta lm;
  const int tid = threadIdx.x;
  const int64_t NB = (int64_t)m.F * m.B;
  // bag tiles a contiguous 1/8 per XCD (xcd_remap): every tile's lookups are independent
  const int64_t b0 = (int64_t)xcd_remap((int)blockIdx.x, (int)gridDim.x) * TILE_BAGS;
  const int nb = (int)min((int64_t)TILE_BAGS, NB - b0);
  if (tid <= nb) off[tid] = offsets[b0 + tid];
  stage_meta(m, lm);
  const void* values = reinterpret_cast<const void*>(ws.vmeta[0]);
  const int id_dtype = (int)ws.vmeta[1];
  __syncthreads();
  const int64_t s0 = off[0], e0 = off[nb];
  const int hw = tid >> 5, hl = tid & 31;
  const BagRow br{grad_out, m.B, ldg, lm.feat};
  constexpr int UN = 4;
  for (int64_t j0 = s0 + hw; j0 < e0; j0 += 8 * UN) {
    bool on[UN];
    int lb[UN];
    int64_t id[UN];
    f32x4v wv[UN], g[UN];
    float s_old[UN];
    float* wrow[UN];
    float* srow[UN];
    int D[UN];
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const int64_t j = j0 + 8 * k;
      on[k] = j < e0 && ws.lk[j] < 0;
      id[k] = j < e0 ? load_id(values, id_dtype, j) : 0;
    }
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      const int64_t j = j0 + 8 * k;
      lb[k] = on[k] ? lds_bag_of(off, nb, j) : 0;
      const int64_t bag = b0 + lb[k];
      const tt_table_meta_t tm = lm.tab[lm.feat[on[k] ? (int)((uint32_t)bag / (uint32_t)m.B) : 0].table];
      if ((uint64_t)id[k] >= (uint64_t)tm.num_rows) id[k] = 0;
      D[k] = tm.dim;
      const bool col = on[k] && hl * 4 < D[k];
      wrow[k] = weights + tm.weight_offset + id[k] * D[k];
      srow[k] = state + tm.state_offset + id[k];
      wv[k] = col ? *reinterpret_cast<const f32x4v*>(wrow[k] + hl * 4) : (f32x4v)(0.f);
      s_old[k] = on[k] ? *srow[k] : 0.f;
      g[k] = col ? *reinterpret_cast<const f32x4v*>(br.row((int)bag) + hl * 4) : (f32x4v)(0.f);
    }
#pragma unroll
    for (int k = 0; k < UN; ++k) {
      if (pooling == TT_POOL_MEAN && on[k]) g[k] *= 1.f / (float)max(1, off[lb[k] + 1] - off[lb[k]]);
      float sq = g[k][0] * g[k][0] + g[k][1] * g[k][1] + g[k][2] * g[k][2] + g[k][3] * g[k][3];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
      if (on[k]) {
        const float snew = s_old[k] + sq / (float)D[k];
        const float step = rw_step(snew, lr, eps);
        if (hl * 4 < D[k]) {
          f32x4v w = wv[k];
#pragma unroll
          for (int v = 0; v < 4; ++v) w[v] = fmaf(g[k][v], step, w[v]);
          *reinterpret_cast<f32x4v*>(wrow[k] + hl * 4) = w;
        }
        if (hl == 0) *srow[k] = snew;
      }
    }
  }
}

// generic-width tables (no direct kernel): the once-looked-up rows of the KJT form get their bag
// written into their record (seg), as the per-row kernels expect
__global__ void __launch_bounds__(256) bwd_single_fix_kernel(EmbMeta m, const int32_t* __restrict__ offsets, BwdWs ws) {
  if (ws.U[1] == 0) return;
  __shared__ int32_t off[TILE_BAGS + 1];
  const int tid = threadIdx.x;
  const int64_t NB = (int64_t)m.F * m.B;
  const int64_t b0 = (int64_t)blockIdx.x * TILE_BAGS;
  const int nb = (int)min((int64_t)TILE_BAGS, NB - b0);
  if (tid <= nb) off[tid] = offsets[b0 + tid];
  __syncthreads();
  const int64_t s0 = off[0], e0 = off[nb];
  for (int64_t j0 = s0; j0 < e0; j0 += TILE_CH)
    for (int i = tid; i < (int)min((int64_t)TILE_CH, e0 - j0); i += 256) {
      const int v = ws.lk[j0 + i];
      if (v < 0) ws.urec[ws.cur[ws.ent_h[j0 + (v & 0xffff)]]].seg = (int32_t)(b0 + lds_bag_of(off, nb, j0 + i));
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
  int sorted = lane < n ? (n == 1 ? s : ws.perm[s + lane]) : 0x7fffffff;  // n == 1: s is the bag
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
  const float step = rw_step(snew, lr, eps);
#pragma unroll
  for (int k = 0; k < ADA_KMAX; ++k) {
    const int c = lane + k * 64;
    if (c < ncol) {
      vf x = *reinterpret_cast<vf*>(w + c * VEC);
#pragma unroll
      for (int v = 0; v < VEC; ++v) x[v] = fmaf(gsave[k][v], step, x[v]);
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

// ---- k2d hot rows (looked up >= HOT_MIN times) -----------------------------------------------
// A hot row with c lookups is split into NR = hot_nr(c) bag-id ranges (one work item each; bwd_
// hot_partial_kernel, persistent grid). An item counts its row's lookups per bag of its range in LDS
// (HOT_WIN bags per pass; passes start at the smallest bag not yet counted, so empty windows cost
// nothing), compacts the non-zero bags in ascending order, and 8 half-wave groups sum
// count x grad_out[bag] over positions g, g+8, ...; the group partials are added in group order.
// NR = 1: the item applies row-wise Adagrad itself; NR > 1: it writes a partial row and
// bwd_hot_final_kernel adds the NR partials in range order and applies Adagrad. Every step is a
// function of the multiset of (row, bag) lookups: bitwise reproducible, no sort, no same-address
// atomics beyond LDS, and the hottest row is spread over up to HOT_NR_MAX workgroups.
__device__ __forceinline__ int block_min_i(int v, int* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return min(min(red[0], red[1]), min(red[2], red[3]));
}

template <int VEC, int KC>
__device__ __forceinline__ void hot_accumulate(const BagRow& br, const int32_t* __restrict__ offsets, int pooling,
                                               int D, const int* wcnt, const int16_t* wb, int64_t wlo, int mtot,
                                               float (&acc)[KC][VEC]) {
  typedef __attribute__((ext_vector_type(VEC))) float vf;
  const int g = threadIdx.x >> 5, l = threadIdx.x & 31;
  constexpr int U4 = KC == 1 ? 4 : 1;  // rows in flight per group (KC loads each)
  for (int e0 = g; e0 < mtot; e0 += 8 * U4) {
    vf x[U4][KC];
    float sc[U4];
#pragma unroll
    for (int u = 0; u < U4; ++u) {
      const int e = e0 + 8 * u;
      sc[u] = 0.f;
      if (e < mtot) {
        const int b = (int)(wlo + wb[e]);
        float s = (float)wcnt[e];
        if (pooling == TT_POOL_MEAN) s *= 1.f / (float)max(1, offsets[b + 1] - offsets[b]);
        sc[u] = s;
        const float* row = br.row(b);
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const int c = l + 32 * k;
          x[u][k] = c * VEC < D ? *reinterpret_cast<const vf*>(row + c * VEC) : (vf)(0.f);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U4; ++u) {
      if (e0 + 8 * u < mtot) {
#pragma unroll
        for (int k = 0; k < KC; ++k)
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[k][v] += sc[u] == 1.f ? x[u][k][v] : x[u][k][v] * sc[u];
      }
    }
  }
}

template <int VEC, int KC>
__device__ __forceinline__ void hot_item(const EmbMeta& m, const BagRow& br, const int32_t* __restrict__ offsets,
                                         int pooling, float* __restrict__ weights, float* __restrict__ state,
                                         float lr, float eps, const BwdWs& ws, const HotRec& hr, int item,
                                         int* wcnt, int16_t* wb, int* red, float* redf) {
  const int tid = threadIdx.x;
  const URec rec = ws.urec[hr.u];
  const int t = (int)(rec.key >> KEY_TABLE_SHIFT);
  const int64_t row = (int64_t)(rec.key & ((1ull << KEY_TABLE_SHIFT) - 1));
  const tt_table_meta_t tm = m.tables[t];
  const int D = tm.dim;
  const int32_t* seg = ws.perm + rec.seg;
  const int n = rec.len;
  const int64_t NB = (int64_t)m.F * m.B;
  const int r = item - hr.pbase;
  const int64_t rlo = r * NB / hr.nr, rhi = (r + 1) * NB / hr.nr;
  float acc[KC][VEC];
#pragma unroll
  for (int k = 0; k < KC; ++k)
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[k][v] = 0.f;
  int64_t wlo = rlo;
  while (wlo < rhi) {
    int mn = 0x7fffffff;
    for (int i = tid; i < n; i += 256) {
      const int b = seg[i];
      if (b >= wlo && b < rhi) mn = min(mn, b);
    }
    mn = block_min_i(mn, red);
    if (mn == 0x7fffffff) break;
    wlo = mn;
    const int64_t whi = min(rhi, wlo + HOT_WIN);
    for (int i = tid; i < HOT_WIN; i += 256) wcnt[i] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 256) {
      const int b = seg[i];
      if (b >= wlo && b < whi) atomicAdd(&wcnt[b - wlo], 1);
    }
    __syncthreads();
    constexpr int BPT = HOT_WIN / 256;
    int cc[BPT], k = 0;
#pragma unroll
    for (int v = 0; v < BPT; ++v) {
      cc[v] = wcnt[tid * BPT + v];
      k += cc[v] > 0;
    }
    int mtot;
    int d = block_excl_scan(k, red, &mtot);
#pragma unroll
    for (int v = 0; v < BPT; ++v)
      if (cc[v] > 0) {
        wcnt[d] = cc[v];
        wb[d] = (int16_t)(tid * BPT + v);
        ++d;
      }
    __syncthreads();
    hot_accumulate<VEC, KC>(br, offsets, pooling, D, wcnt, wb, wlo, mtot, acc);
    __syncthreads();
    wlo = whi;
  }
  // group partials -> LDS (wcnt reused as float[8][HOT_DMAX]) -> summed in group order
  float* part = reinterpret_cast<float*>(wcnt);
  const int g = tid >> 5, l = tid & 31;
#pragma unroll
  for (int k = 0; k < KC; ++k)
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const int c = (l + 32 * k) * VEC + v;
      if (c < D) part[g * HOT_DMAX + c] = acc[k][v];
    }
  __syncthreads();
  float tot[HOT_DMAX / 256];
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < HOT_DMAX / 256; ++k) {
    const int c = tid + 256 * k;
    float s = 0.f;
    if (c < D) {
#pragma unroll
      for (int gg = 0; gg < 8; ++gg) s += part[gg * HOT_DMAX + c];
    }
    tot[k] = s;
    sq += s * s;
  }
  if (hr.nr == 1) {
    sq = wave_sum(sq);
    if ((tid & 63) == 0) redf[tid >> 6] = sq;
    __syncthreads();
    sq = (redf[0] + redf[1]) + (redf[2] + redf[3]);
    float* srow = state + tm.state_offset + row;
    const float snew = *srow + sq / (float)D;
    const float step = rw_step(snew, lr, eps);
    float* wrow = weights + tm.weight_offset + row * D;
#pragma unroll
    for (int k = 0; k < HOT_DMAX / 256; ++k) {
      const int c = tid + 256 * k;
      if (c < D) wrow[c] = fmaf(tot[k], step, wrow[c]);
    }
    __syncthreads();
    if (tid == 0) *srow = snew;
  } else {
    float* p = ws.hotp + (int64_t)item * HOT_DMAX;
#pragma unroll
    for (int k = 0; k < HOT_DMAX / 256; ++k) {
      const int c = tid + 256 * k;
      if (c < D) p[c] = tot[k];
    }
  }
  __syncthreads();  // LDS reuse by the next item
}

__global__ void __launch_bounds__(256) bwd_hot_partial_kernel(EmbMeta m, const float* __restrict__ grad_out,
                                                              int64_t ldg, const int32_t* __restrict__ offsets,
                                                              int pooling, float* __restrict__ weights,
                                                              float* __restrict__ state, float lr, float eps,
                                                              BwdWs ws, int vec4_ok) {
  __shared__ int wcnt[HOT_WIN];  // per-bag counts of a window / compacted counts / group partials
  __shared__ int16_t wb[HOT_WIN];
  __shared__ int red[4];
  __shared__ float redf[4];
  const unsigned long long hw = *reinterpret_cast<const unsigned long long*>(ws.U + 2);
  const int items = (int)(hw & 0xffffffffull), nhot = (int)(hw >> 32);
  const BagRow br{grad_out, m.B, ldg, m.features};
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    int lo = 0, hi = nhot;  // hot row of the item: the largest h with pbase <= it (pbase ascends with h)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (ws.hot[mid].pbase <= it) lo = mid;
      else hi = mid;
    }
    const HotRec hr = ws.hot[lo];
    const int D = m.tables[(int)(ws.urec[hr.u].key >> KEY_TABLE_SHIFT)].dim;
    if (vec4_ok && (D & 3) == 0 && D <= 128)
      hot_item<4, 1>(m, br, offsets, pooling, weights, state, lr, eps, ws, hr, it, wcnt, wb, red, redf);
    else if (vec4_ok && (D & 3) == 0)
      hot_item<4, 8>(m, br, offsets, pooling, weights, state, lr, eps, ws, hr, it, wcnt, wb, red, redf);
    else
      hot_item<1, 32>(m, br, offsets, pooling, weights, state, lr, eps, ws, hr, it, wcnt, wb, red, redf);
  }
}

// rows split over NR > 1 ranges: a wave per row adds the partials in range order, then Adagrad
__global__ void __launch_bounds__(256) bwd_hot_final_kernel(EmbMeta m, float* __restrict__ weights,
                                                            float* __restrict__ state, float lr, float eps,
                                                            BwdWs ws) {
  const int nhot = ws.U[3];
  const int lane = threadIdx.x & 63;
  for (int h = blockIdx.x * 4 + (threadIdx.x >> 6); h < nhot; h += gridDim.x * 4) {
    const HotRec hr = ws.hot[h];
    if (hr.nr == 1) continue;
    const URec rec = ws.urec[hr.u];
    const int t = (int)(rec.key >> KEY_TABLE_SHIFT);
    const int64_t row = (int64_t)(rec.key & ((1ull << KEY_TABLE_SHIFT) - 1));
    const tt_table_meta_t tm = m.tables[t];
    const int D = tm.dim;
    const float* p = ws.hotp + (int64_t)hr.pbase * HOT_DMAX;
    float tot[HOT_DMAX / 64];
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < HOT_DMAX / 64; ++k) {
      const int c = lane + 64 * k;
      float s = 0.f;
      if (c < D)
        for (int r = 0; r < hr.nr; ++r) s += p[(int64_t)r * HOT_DMAX + c];
      tot[k] = s;
      sq += s * s;
    }
    sq = wave_sum(sq);
    float* srow = state + tm.state_offset + row;
    const float snew = *srow + sq / (float)D;
    const float step = rw_step(snew, lr, eps);
    float* wrow = weights + tm.weight_offset + row * D;
#pragma unroll
    for (int k = 0; k < HOT_DMAX / 64; ++k) {
      const int c = lane + 64 * k;
      if (c < D) wrow[c] = fmaf(tot[k], step, wrow[c]);
    }
    if (lane == 0) *srow = snew;
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

// One 4-byte load per page of the tables (tt_table_prefault): the address translations of every
// page walked once at setup, so the first training steps do not pay the page-table misses a cold
// process otherwise takes ~30 steps to absorb (profiles/r06dr_overhead4.log). The loads are
// XOR-folded and stored only if the fold equals one fixed value, so they cannot be dropped; in
// practice the sink is never written (and if so, by a vector store).
__global__ void __launch_bounds__(256) table_prefault_kernel(const uint32_t* __restrict__ base, int64_t words,
                                                             int64_t stride, uint32_t* sink) {
  const int64_t n = (words + stride - 1) / stride;
  uint32_t acc = 0;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x)
    acc ^= base[p * stride];
  if (acc == 0x7fc0dead) sink[0] = acc;
}

}  // namespace tt

using namespace tt;

extern "C" {

int tt_table_prefault(const void* base, size_t bytes, size_t page_bytes, uint32_t* sink, void* stream) {
  if (bytes == 0) return TT_OK;
  if (!base || !sink) return fail(TT_EINVAL, "table_prefault: null pointer");
  if (page_bytes < 4 || page_bytes % 4 || reinterpret_cast<uintptr_t>(base) % 4)
    return fail(TT_EINVAL, "table_prefault: page_bytes must be a multiple of 4 and base 4-byte aligned");
  const int64_t words = (int64_t)(bytes / 4), stride = (int64_t)(page_bytes / 4);
  const int64_t pages = (words + stride - 1) / stride;
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(4096, ceil_div(pages, 256)));
  table_prefault_kernel<<<dim3((unsigned)grid), dim3(256), 0, as_stream(stream)>>>(
      reinterpret_cast<const uint32_t*>(base), words, stride, sink);
  return check_launch("table_prefault");
}

int tt_table_alloc(size_t bytes, void** out, int* contiguous) {
  if (!out || bytes == 0) return fail(TT_EINVAL, "table_alloc: null output or zero bytes");
  *out = nullptr;
  // one physically contiguous range when the driver has it: the largest page fragments, so the
  // random row gathers walk fewer translation levels (profiles/r06al_alloc.log)
  hipError_t e = hipExtMallocWithFlags(out, bytes, hipDeviceMallocContiguous);
  int contig = 1;
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    contig = 0;
    e = hipMalloc(out, bytes);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return fail((int)e, std::string("table_alloc: ") + hipGetErrorString(e));
  }
  if (contiguous) *contiguous = contig;
  return TT_OK;
}

int tt_table_free(void* p) {
  if (!p) return TT_OK;
  hipError_t e = hipFree(p);
  return e == hipSuccess ? TT_OK : fail((int)e, std::string("table_free: ") + hipGetErrorString(e));
}

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
      hipMemsetAsync(w.U, 0, sizeof(int32_t) * 8, st) != hipSuccess)
    return fail(TT_EINVAL, "bwd_workspace_init: memset failed");
  return TT_OK;
}

static int launch_scan_scatter(const EmbMeta& m, const int32_t* offsets, BwdWs& w, hipStream_t st, int gb) {
  const int nb = (int)ceil_div(w.cap, SCAN_TILE);
  bwd_scan_reduce_kernel<<<dim3(nb), dim3(256), 0, st>>>(w, 0);
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
    if (tables[t].num_rows >= (1ll << PK_ROW_BITS) - 1) return fail(TT_EINVAL, "bwd_prepare: table rows >= 2^34 - 1");
  BwdWs w;
  bwd_layout(workspace, max_lookups, &w);
  hipStream_t st = as_stream(stream);
  const int64_t nbag = (int64_t)F * B;
  const int64_t tiles = ceil_div(nbag, TILE_BAGS);
  if (tiles > INT32_MAX) return fail(TT_EINVAL, "bwd_prepare: too many bags");
  if (nbag > 0)
    bwd_tile_hash_kernel<<<dim3((unsigned)tiles), dim3(256), 0, st>>>(m, values, id_dtype, offsets, bounds_check, w);
  const int nb = (int)ceil_div(w.cap, SCAN_TILE);
  bwd_scan_reduce_kernel<<<dim3(nb), dim3(256), 0, st>>>(w, 1);
  bwd_scan_kernel<<<dim3(nb), dim3(256), 0, st>>>(w);
  if (nbag > 0) bwd_tile_scatter_kernel<<<dim3((unsigned)tiles), dim3(256), 0, st>>>(m, offsets, w);
  return check_launch("bwd_prepare");
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
  for (int t = 0; t < T; ++t)
    if (tables[t].num_rows >= (1ll << PK_ROW_BITS) - 1) return fail(TT_EINVAL, "bwd_prepare_cols: table rows >= 2^34 - 1");
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

static int bwd_rowwise_adagrad(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F,
                               int64_t B, const float* grad_out, int64_t ldg, const int32_t* offsets, int pooling,
                               float* weights, float* state, float lr, float eps, void* workspace, size_t ws_bytes,
                               int64_t max_lookups, void* stream, int part) {
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
  if (part && !narrow)  // the generic path's single-row fix feeds its update: one stream only
    return fail(TT_EINVAL, "bwd_rowwise_adagrad_part: parts need 16-B aligned rows of D <= 128 (the narrow path)");
  BwdWs w;
  bwd_layout(workspace, max_lookups, &w);
  hipStream_t st = as_stream(stream);
  const int64_t tiles = ceil_div((int64_t)F * B, TILE_BAGS);
  if (part != 2 && offsets && F * B > 0 && tiles <= INT32_MAX) {  // once-looked-up rows of a KJT-form prepare
    if (narrow)
      bwd_adagrad_direct_kernel<<<dim3((unsigned)tiles), dim3(256), 0, st>>>(m, grad_out, ldg, offsets, pooling, weights,
                                                                            state, lr, eps, w);
    else
      bwd_single_fix_kernel<<<dim3((unsigned)tiles), dim3(256), 0, st>>>(m, offsets, w);
  }
  if (part == 1) return check_launch("bwd_rowwise_adagrad_direct");
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
    const int hgrid = (int)std::min<int64_t>(2048, hot_items_max(max_lookups));
    bwd_hot_partial_kernel<<<dim3(hgrid), dim3(256), 0, st>>>(m, grad_out, ldg, offsets, pooling, weights, state,
                                                              lr, eps, w, vec_ok ? 1 : 0);
    const int fgrid = (int)std::min<int64_t>(1024, max_lookups / HOT_SPLIT / 4 + 1);
    bwd_hot_final_kernel<<<dim3(fgrid), dim3(256), 0, st>>>(m, weights, state, lr, eps, w);
  }
  return check_launch("bwd_rowwise_adagrad");
}

int tt_bwd_rowwise_adagrad(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features,
                           int F, int64_t B, const float* grad_out, int64_t ldg,
                           const int32_t* offsets, int pooling, float* weights, float* state,
                           float lr, float eps, void* workspace, size_t ws_bytes,
                           int64_t max_lookups, void* stream) {
  return bwd_rowwise_adagrad(tables, T, features, F, B, grad_out, ldg, offsets, pooling, weights, state, lr, eps,
                             workspace, ws_bytes, max_lookups, stream, 0);
}

int tt_bwd_rowwise_adagrad_part(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F,
                                int64_t B, const float* grad_out, int64_t ldg, const int32_t* offsets, int pooling,
                                float* weights, float* state, float lr, float eps, void* workspace, size_t ws_bytes,
                                int64_t max_lookups, int part, void* stream) {
  if (part < 0 || part > 2) return fail(TT_EINVAL, "bwd_rowwise_adagrad_part: part must be 0, 1 or 2");
  if (part == 1 && !offsets) return fail(TT_EINVAL, "bwd_rowwise_adagrad_part: part 1 needs the KJT offsets");
  return bwd_rowwise_adagrad(tables, T, features, F, B, grad_out, ldg, offsets, pooling, weights, state, lr, eps,
                             workspace, ws_bytes, max_lookups, stream, part);
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
  if (max_lookups >= (1ll << PK_CNT_BITS)) return fail(TT_EINVAL, std::string(what) + ": max_lookups >= 2^24");
  if (!workspace || ws_bytes < tt_bwd_workspace_bytes(max_lookups))
    return fail(TT_ECAPACITY, std::string(what) + ": workspace too small");
  return TT_OK;
}
}  // namespace tt

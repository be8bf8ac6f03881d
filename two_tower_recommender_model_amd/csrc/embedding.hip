// Embedding-bag hot path for gfx950: pooled (segmented gather + sum) forward and the
// deduplicated backward with exact row-wise Adagrad fused in (no weight .grad is materialised).
//
// Forward (k1): a group of G lanes owns one bag; each lane owns a 16-B column slice (float4) of the
// row, so one D=128 fp32 row is one 512-B coalesced read by 32 lanes and a wave pools 2 bags at
// once. Ids of a bag are read 4 at a time so 4 independent rows are in flight per group.
// Algorithmic bytes per lookup: 4*D (row) + id bytes; per bag 4*D write + 4 (offset).
//
// Backward (k2a..k2d): lookups are grouped by unique (table,row) with an open-addressing hash in
// the workspace (k2a), a reduce-then-scan over the hash slots assigns each unique row a segment
// (k2b), the bag ids are scattered into their segments (k2c), and one wave per unique row sums the
// pooled-output gradient rows of its segment and applies the row-wise Adagrad update in place
// (k2d). k2a-k2c read only ids, so they can run concurrently with the forward and the towers.
// k2d leaves the hash table clean for the next step (no per-step memset).
#include "tt_common.h"

namespace tt {

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
    vf acc0 = (vf)(0.f), acc1 = (vf)(0.f);
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
    (void)acc1;
    acc0 *= scale;
    *reinterpret_cast<vf*>(out + c * VEC) = acc0;
  }
}

__global__ void __launch_bounds__(256) pooled_fwd_kernel(const float* __restrict__ weights, FwdArgs a,
                                                         const void* __restrict__ values, int id_dtype,
                                                         const int32_t* __restrict__ offsets, int pooling,
                                                         float* __restrict__ out, int64_t ldo,
                                                         int bounds_check, int32_t* __restrict__ err) {
  // which feature does this workgroup serve (F <= 64, wave-uniform scalar search)
  int f = 0;
  while (f + 1 < a.m.F && (int)blockIdx.x >= a.block_start[f + 1]) ++f;
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

struct BwdWs {
  uint64_t* keys;   // [cap] hash keys (EMPTY when free)
  int32_t* cnt;     // [cap] lookups per slot / scatter cursor
  int32_t* seg;     // [cap] segment start per slot
  int32_t* slot_of; // [L]   slot of each lookup
  int32_t* perm;    // [L]   bag ids grouped by unique row
  int32_t* useg;    // [L]   segment start per unique
  int32_t* ulen;    // [L]   segment length per unique
  int32_t* uslot;   // [L]   slot per unique
  int32_t* bsum_u;  // [nb]  scan partials (unique count)
  int32_t* bsum_c;  // [nb]  scan partials (lookup count)
  int32_t* U;       // [1]   number of unique rows this step
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
  t.seg = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * cap));
  t.slot_of = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.perm = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.useg = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.ulen = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.uslot = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.bsum_u = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * nb));
  t.bsum_c = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * nb));
  t.U = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * 4));
  t.cap = cap;
  t.L = L;
  if (w) *w = t;
  return off;
}

// k2a: thread per bag: hash-insert every lookup's (table,row), count per slot
__global__ void __launch_bounds__(256) bwd_hash_kernel(EmbMeta m, const void* __restrict__ values, int id_dtype,
                                                       const int32_t* __restrict__ offsets, int bounds_check,
                                                       BwdWs ws) {
  const int64_t nbag = (int64_t)m.F * m.B;
  const uint64_t mask = (uint64_t)ws.cap - 1;
  for (int64_t bag = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; bag < nbag;
       bag += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(bag / m.B);
    const int t = m.features[f].table;
    const int64_t rows = m.tables[t].num_rows;
    const int64_t s = offsets[bag], e = offsets[bag + 1];
    for (int64_t j = s; j < e; ++j) {
      int64_t id = load_id(values, id_dtype, j);
      if (bounds_check && (uint64_t)id >= (uint64_t)rows) id = 0;
      const uint64_t key = ((uint64_t)t << KEY_TABLE_SHIFT) | (uint64_t)id;
      uint64_t h = mix64(key) & mask;
      while (true) {
        uint64_t cur = __hip_atomic_load(&ws.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == key) break;
        if (cur == EMPTY_KEY) {
          uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(&ws.keys[h]),
                                    (unsigned long long)EMPTY_KEY, (unsigned long long)key);
          if (prev == EMPTY_KEY || prev == key) break;
        }
        h = (h + 1) & mask;
      }
      ws.slot_of[j] = (int32_t)h;
      atomicAdd(&ws.cnt[h], 1);
    }
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
  }
}

// k2b-2: exclusive scans -> unique index and segment start per occupied slot
__global__ void __launch_bounds__(256) bwd_scan_kernel(BwdWs ws) {
  __shared__ int lds[8];
  // prefixes of the preceding tiles
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
  // two block scans at once (wave shuffles, then 4 wave totals)
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
      ws.useg[eu] = ec;
      ws.ulen[eu] = c[j];
      ws.uslot[eu] = (int32_t)h;
      ws.seg[h] = ec;
      ws.cnt[h] = 0;  // becomes the scatter cursor
      eu += 1;
      ec += c[j];
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) ws.U[0] = pu + tu;
}

// k2c: thread per bag: scatter bag ids into their unique row's segment
__global__ void __launch_bounds__(256) bwd_scatter_kernel(EmbMeta m, const int32_t* __restrict__ offsets,
                                                          BwdWs ws) {
  const int64_t nbag = (int64_t)m.F * m.B;
  for (int64_t bag = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; bag < nbag;
       bag += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = offsets[bag], e = offsets[bag + 1];
    for (int64_t j = s; j < e; ++j) {
      const int h = ws.slot_of[j];
      const int pos = ws.seg[h] + atomicAdd(&ws.cnt[h], 1);
      ws.perm[pos] = (int32_t)bag;
    }
  }
}

// 64-lane bitonic sort (ascending) of one int per lane
__device__ __forceinline__ int wave_bitonic_sort(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
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

constexpr int ADA_KMAX = 4;  // up to 4 x 64 x VEC columns per row (D <= 1024 with float4)

template <int VEC>
__device__ __forceinline__ void adagrad_row(const EmbMeta& m, const float* __restrict__ grad_out, int64_t ldg,
                                            const int32_t* __restrict__ offsets, int pooling,
                                            float* __restrict__ weights, float* __restrict__ state, float lr,
                                            float eps, const BwdWs& ws, int t, int64_t r, int s, int n) {
  typedef __attribute__((ext_vector_type(VEC))) float vf;
  const int lane = threadIdx.x & 63;
  const tt_table_meta_t tm = m.tables[t];
  const int D = tm.dim;
  const int ncol = D / VEC;  // VEC divides D
  const int64_t B = m.B;
  float g[ADA_KMAX][VEC];
#pragma unroll
  for (int k = 0; k < ADA_KMAX; ++k)
#pragma unroll
    for (int v = 0; v < VEC; ++v) g[k][v] = 0.f;

  auto row_ptr = [&](int bag) -> const float* {
    const int f = bag / (int)B;
    const int64_t b = bag - (int64_t)f * B;
    return grad_out + (m.features[f].out_row + b) * ldg + m.features[f].out_offset;
  };
  auto bag_scale = [&](int bag) -> float {
    if (pooling != TT_POOL_MEAN) return 1.f;
    const int len = offsets[bag + 1] - offsets[bag];
    return len > 0 ? 1.f / (float)len : 1.f;
  };

  if (n <= 64) {
    // deterministic: sum in ascending bag order
    int mine = lane < n ? ws.perm[s + lane] : 0x7fffffff;
    mine = wave_bitonic_sort(mine);
    int i = 0;
    for (; i + 2 <= n; i += 2) {
      const int b0 = __shfl(mine, i, 64), b1 = __shfl(mine, i + 1, 64);
      const float* p0 = row_ptr(b0);
      const float* p1 = row_ptr(b1);
      const float s0 = bag_scale(b0), s1 = bag_scale(b1);
#pragma unroll
      for (int k = 0; k < ADA_KMAX; ++k) {
        const int c = lane + k * 64;
        if (c < ncol) {
          const vf x0 = *reinterpret_cast<const vf*>(p0 + c * VEC);
          const vf x1 = *reinterpret_cast<const vf*>(p1 + c * VEC);
#pragma unroll
          for (int v = 0; v < VEC; ++v) {
            g[k][v] += x0[v] * s0;
            g[k][v] += x1[v] * s1;
          }
        }
      }
    }
    if (i < n) {
      const int b0 = __shfl(mine, i, 64);
      const float* p0 = row_ptr(b0);
      const float s0 = bag_scale(b0);
#pragma unroll
      for (int k = 0; k < ADA_KMAX; ++k) {
        const int c = lane + k * 64;
        if (c < ncol) {
          const vf x0 = *reinterpret_cast<const vf*>(p0 + c * VEC);
#pragma unroll
          for (int v = 0; v < VEC; ++v) g[k][v] += x0[v] * s0;
        }
      }
    }
  } else {
    // hot row: fp64 accumulation (order-independent in practice), 64 bag ids per chunk
    double gd[ADA_KMAX][VEC];
#pragma unroll
    for (int k = 0; k < ADA_KMAX; ++k)
#pragma unroll
      for (int v = 0; v < VEC; ++v) gd[k][v] = 0.0;
    for (int base = 0; base < n; base += 64) {
      const int cnt = min(64, n - base);
      const int mine = lane < cnt ? ws.perm[s + base + lane] : 0;
      int i = 0;
      for (; i + 4 <= cnt; i += 4) {
        const int bb[4] = {__shfl(mine, i, 64), __shfl(mine, i + 1, 64), __shfl(mine, i + 2, 64),
                           __shfl(mine, i + 3, 64)};
#pragma unroll
        for (int k = 0; k < ADA_KMAX; ++k) {
          const int c = lane + k * 64;
          if (c < ncol) {
            vf x[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) x[q] = *reinterpret_cast<const vf*>(row_ptr(bb[q]) + c * VEC);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float sc = bag_scale(bb[q]);
#pragma unroll
              for (int v = 0; v < VEC; ++v) gd[k][v] += (double)(x[q][v] * sc);
            }
          }
        }
      }
      for (; i < cnt; ++i) {
        const int b0 = __shfl(mine, i, 64);
        const float* p0 = row_ptr(b0);
        const float s0 = bag_scale(b0);
#pragma unroll
        for (int k = 0; k < ADA_KMAX; ++k) {
          const int c = lane + k * 64;
          if (c < ncol) {
            const vf x0 = *reinterpret_cast<const vf*>(p0 + c * VEC);
#pragma unroll
            for (int v = 0; v < VEC; ++v) gd[k][v] += (double)(x0[v] * s0);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < ADA_KMAX; ++k)
#pragma unroll
      for (int v = 0; v < VEC; ++v) g[k][v] = (float)gd[k][v];
  }

  // row-wise Adagrad: s += mean(G^2); w += (-lr * G) / (sqrt(s) + eps)
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < ADA_KMAX; ++k)
#pragma unroll
    for (int v = 0; v < VEC; ++v) sq += g[k][v] * g[k][v];
  sq = wave_sum(sq);
  float* srow = state + tm.state_offset + r;
  const float snew = *srow + sq / (float)D;
  const float stdv = sqrtf(snew) + eps;
  float* w = weights + tm.weight_offset + r * D;
#pragma unroll
  for (int k = 0; k < ADA_KMAX; ++k) {
    const int c = lane + k * 64;
    if (c < ncol) {
      vf x = *reinterpret_cast<vf*>(w + c * VEC);
#pragma unroll
      for (int v = 0; v < VEC; ++v) x[v] = x[v] + (-lr * g[k][v]) / stdv;
      *reinterpret_cast<vf*>(w + c * VEC) = x;
    }
  }
  if (lane == 0) *srow = snew;
}

// k2d: one wave per unique row (grid-stride over the device-side unique count)
__global__ void __launch_bounds__(256) bwd_adagrad_kernel(EmbMeta m, const float* __restrict__ grad_out,
                                                          int64_t ldg, const int32_t* __restrict__ offsets,
                                                          int pooling, float* __restrict__ weights,
                                                          float* __restrict__ state, float lr, float eps,
                                                          BwdWs ws, int vec4_ok) {
  const int U = ws.U[0];
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); u < U; u += nwaves) {
    const int h = ws.uslot[u];
    const int s = ws.useg[u];
    const int n = ws.ulen[u];
    const uint64_t key = ws.keys[h];
    const int t = (int)(key >> KEY_TABLE_SHIFT);
    const int64_t r = (int64_t)(key & ((1ull << KEY_TABLE_SHIFT) - 1));
    const int D = m.tables[t].dim;
    if (vec4_ok && (D & 3) == 0 && D >= 256)
      adagrad_row<4>(m, grad_out, ldg, offsets, pooling, weights, state, lr, eps, ws, t, r, s, n);
    else if (vec4_ok && (D & 1) == 0)
      adagrad_row<2>(m, grad_out, ldg, offsets, pooling, weights, state, lr, eps, ws, t, r, s, n);
    else
      adagrad_row<1>(m, grad_out, ldg, offsets, pooling, weights, state, lr, eps, ws, t, r, s, n);
    if (lane == 0) {
      ws.keys[h] = EMPTY_KEY;  // leave the hash table clean for the next step
      ws.cnt[h] = 0;
    }
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
  int64_t blocks = 0;
  for (int f = 0; f < F; ++f) {
    const tt_table_meta_t& tm = tables[features[f].table];
    if (features[f].out_offset + tm.dim > ldo) return fail(TT_EINVAL, "pooled_fwd: output row too short");
    const bool v4 = (tm.dim % 4 == 0) && (tm.weight_offset % 4 == 0) && (features[f].out_offset % 4 == 0) &&
                    (ldo % 4 == 0) && ((reinterpret_cast<uintptr_t>(weights) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
    a.vec[f] = v4 ? 4 : 1;
    const int cols = tm.dim / a.vec[f];
    int g = 1;
    while (g < cols && g < 64) g <<= 1;
    a.group[f] = g;
    a.block_start[f] = (int32_t)blocks;
    blocks += ceil_div(B, 256 / g);
  }
  a.block_start[F] = (int32_t)blocks;
  if (blocks > INT32_MAX) return fail(TT_EINVAL, "pooled_fwd: grid too large");
  pooled_fwd_kernel<<<dim3((unsigned)blocks), dim3(256), 0, as_stream(stream)>>>(
      weights, a, values, id_dtype, offsets, pooling, out, ldo, bounds_check, err_count);
  return check_launch("pooled_fwd");
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

int tt_bwd_prepare(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F,
                   int64_t B, const void* values, int id_dtype, const int32_t* offsets,
                   int bounds_check, void* workspace, size_t ws_bytes, int64_t max_lookups,
                   void* stream) {
  EmbMeta m{};
  int rc = pack_meta(m, tables, T, features, F, B);
  if (rc) return rc;
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "bwd_prepare: ids must be int32/int64");
  if (max_lookups < 1) max_lookups = 1;
  if (max_lookups > INT32_MAX / 2) return fail(TT_EINVAL, "bwd_prepare: max_lookups too large");
  if (!workspace || ws_bytes < tt_bwd_workspace_bytes(max_lookups))
    return fail(TT_ECAPACITY, "bwd_prepare: workspace too small");
  for (int t = 0; t < T; ++t)
    if (tables[t].num_rows >= (1ll << KEY_TABLE_SHIFT)) return fail(TT_EINVAL, "bwd_prepare: table rows >= 2^40");
  BwdWs w;
  bwd_layout(workspace, max_lookups, &w);
  hipStream_t st = as_stream(stream);
  const int64_t nbag = (int64_t)F * B;
  const int gb = (int)std::min<int64_t>(8192, std::max<int64_t>(1, ceil_div(nbag, 256)));
  if (nbag > 0) bwd_hash_kernel<<<dim3(gb), dim3(256), 0, st>>>(m, values, id_dtype, offsets, bounds_check, w);
  const int nb = (int)ceil_div(w.cap, 1024);
  bwd_scan_reduce_kernel<<<dim3(nb), dim3(256), 0, st>>>(w);
  bwd_scan_kernel<<<dim3(nb), dim3(256), 0, st>>>(w);
  if (nbag > 0) bwd_scatter_kernel<<<dim3(gb), dim3(256), 0, st>>>(m, offsets, w);
  return check_launch("bwd_prepare");
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
  if (!workspace || ws_bytes < tt_bwd_workspace_bytes(max_lookups))
    return fail(TT_ECAPACITY, "bwd_rowwise_adagrad: workspace too small");
  if (pooling != TT_POOL_SUM && pooling != TT_POOL_MEAN) return fail(TT_EINVAL, "bwd_rowwise_adagrad: bad pooling");
  if (!grad_out || !weights || !state || !offsets) return fail(TT_EINVAL, "bwd_rowwise_adagrad: null pointer");
  bool vec_ok = (ldg % 4 == 0) && ((reinterpret_cast<uintptr_t>(grad_out) & 15) == 0) &&
                ((reinterpret_cast<uintptr_t>(weights) & 15) == 0);
  for (int t = 0; t < T; ++t)
    if (tables[t].weight_offset % 4) vec_ok = false;
  for (int f = 0; f < F; ++f)
    if (features[f].out_offset % 4) vec_ok = false;
  // the kernel's per-row choice: float4 (D%4==0, D>=256, D<=1024), float2 (D even, D<=512),
  // scalar (D<=256)
  for (int t = 0; t < T; ++t) {
    const int D = tables[t].dim;
    const bool v4 = vec_ok && D % 4 == 0 && D >= 256;
    const bool v2 = vec_ok && D % 2 == 0 && !v4;
    const int cap = v4 ? 1024 : (v2 ? 512 : 256);
    if (D > cap) return fail(TT_EINVAL, "bwd_rowwise_adagrad: unaligned dim > 256 unsupported");
  }
  BwdWs w;
  bwd_layout(workspace, max_lookups, &w);
  const int grid = (int)std::min<int64_t>(16384, std::max<int64_t>(1, ceil_div(max_lookups, 4)));
  bwd_adagrad_kernel<<<dim3(grid), dim3(256), 0, as_stream(stream)>>>(m, grad_out, ldg, offsets, pooling, weights,
                                                                      state, lr, eps, w, vec_ok ? 1 : 0);
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

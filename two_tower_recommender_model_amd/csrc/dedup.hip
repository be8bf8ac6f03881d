// Two-launch deduplicated backward + exact row-wise Adagrad for single-hot lookups (gfx950).
//
// Replaces, for single-hot bags (the fused step's columns and the sharded step's received ids),
// the FBGEMM TBE backward with EXACT_ROWWISE_ADAGRAD fused in (reached from
// _apply_optimizer_in_backward(RowWiseAdagrad, ...), 03_model_training.py:791-795):
//
//   insert  (dd_insert_*_kernel, or fused into the tower kernel T1): every lookup claims/joins its
//           (table, row) slot — see dedup.h.
//   update  (dd_adagrad_kernel): one launch, two roles.
//           * a half-wave per hash slot (32 lanes x float4 = one 512-B row): one 64-B read of the
//             slot gives key, count and the <= 14 lookup indices; the lookups are sorted ascending
//             (register bitonic), their pooled-gradient rows summed in that order in fp32 (the
//             order of the dense index_add the CPU oracle uses: bitwise equal), then
//             s += mean(G^2); w -= lr * G / (sqrt(s) + eps); the slot is reset for the next step.
//           * the first `hot_wgs` workgroups take the hot rows (> 14 lookups): the row's lookups
//             are found by scanning the per-lookup keys in index order (4096 per pass, compacted
//             in LDS), 8 lane groups sum positions j = g (mod 8) in ascending order and the 8
//             partials are added in group order: deterministic; the last hot workgroup to finish
//             resets the hot-row counter (the hot list is final before this launch starts).
// Algorithmic bytes per unique row (count c): 64 (slot) + c * (4 D grad row) + 8 D (row r/w) + 8
// (state r/w); per lookup 8 (key) written by the insert.
#include "dedup.h"

namespace tt {

struct ColArgsD {
  const void* col[TT_MAX_FEATURES];
  int64_t num_emb[TT_MAX_FEATURES];
};

// slots: a power of two >= 16 x the lookups (load factor <= 1/16 even if every lookup is unique): a
// first CAS rarely collides and probe chains stay short; the update walks the claiming lookups,
// so the table's size costs only memory (128 B a slot)
static int64_t dedup_cap(int64_t L) {
  int64_t c = 1024;
  while (c < 16 * L) c <<= 1;
  return c;
}

size_t dedup_layout(void* base, int64_t L, DedupWs* w) {
  const int64_t cap = dedup_cap(L);
  char* p = reinterpret_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = p ? p + off : nullptr;
    off += align_up(bytes, 256);
    return r;
  };
  DedupWs t;
  t.slots = reinterpret_cast<DSlot*>(take(sizeof(DSlot) * cap));
  t.lkey = reinterpret_cast<uint64_t*>(take(sizeof(uint64_t) * L));
  t.hot = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (L / (DD_INL + 1) + 1)));
  t.ctr = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * 4));
  t.claim = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * L));
  t.ovf_groups = (int32_t)((L + 63) / 64);
  t.ovf = reinterpret_cast<DedupWs::Ovf*>(take(sizeof(DedupWs::Ovf) * 64 * (size_t)t.ovf_groups));
  int64_t* dbg = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * 8 * (L / (8 * DD_SPH) + 64)));
#if TT_EXPERIMENTS
  t.stamps = getenv("TT_DD_STAMPS") ? dbg : nullptr;
#else
  (void)dbg;
#endif
  const int64_t hot_cap = L / (DD_INL + 1) + 1;
  t.hotp = reinterpret_cast<float*>(take(sizeof(float) * 128 * DD_HOT_TEAM * hot_cap));
  t.hcnt = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * hot_cap));
  t.nseg = (int32_t)((L + 15) / 16);
  t.multi = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * DD_SEGW * (size_t)t.nseg));
  t.hkey = reinterpret_cast<uint64_t*>(take(sizeof(uint64_t) * (L / (DD_INL + 1) + 1)));  // (last: the
  // layout before it is what tests/test_gpu_dedup.py inspects)
  t.cap = cap;
  t.L = L;
  t.hot_cap = (int32_t)(L / (DD_INL + 1) + 1);
  if (w) *w = t;
  return off;
}

// ---- insert ----------------------------------------------------------------------------------
// single-hot columns: lookup i = f * B + b; transform_to_torchrec_batch semantics (id 0 dropped,
// id mod N), 03_model_training.py:356-365
__global__ void __launch_bounds__(64) dd_insert_cols_kernel(EmbMeta m, ColArgsD ca, int id_dtype, DedupWs ws) {
  const int64_t n = (int64_t)m.F * m.B;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(i / m.B);
    const int64_t b = i - (int64_t)f * m.B;
    const int64_t id = load_id(ca.col[f], id_dtype, b);
    uint64_t key = DD_EMPTY;
    if (id != 0)
      key = ((uint64_t)m.features[f].table << DD_TABLE_SHIFT) | (uint64_t)py_mod64(id, ca.num_emb[f]);
    dd_insert(ws, key, (int32_t)i);
  }
}

// received segments (sharded owner side): lookup i = seg * C + k holds keys[i] when k < counts[seg]
__global__ void __launch_bounds__(64) dd_insert_segments_kernel(const int64_t* __restrict__ keys,
                                                                const int32_t* __restrict__ counts, int64_t C,
                                                                int64_t n, DedupWs ws) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t seg = i / C, k = i - seg * C;
    const uint64_t key = k < counts[seg] ? (uint64_t)keys[i] : DD_EMPTY;
    dd_insert(ws, key, (int32_t)i);
  }
}

// ---- deferred inserts: dd_resolve_block (dedup.h) ------------------------------------------------
constexpr int DD_RES_WGS = 64;
__global__ void __launch_bounds__(256) dd_resolve_kernel(DedupWs ws) { dd_resolve_block(ws, (int)blockIdx.x, DD_RES_WGS); }

// ---- update: dd_update_block (dedup.h) ----------------------------------------------------------
__global__ void __launch_bounds__(256) dd_adagrad_kernel(DdUpdateArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[DD_SMEM];
  dd_update_block(a, (int)blockIdx.x, smem);
}

static int check_dd_ws(void* workspace, size_t ws_bytes, int64_t max_lookups, const char* what) {
  if (max_lookups < 1 || max_lookups >= (int64_t)DD_CNT_MASK)
    return fail(TT_EINVAL, std::string(what) + ": max_lookups out of range");
  if (!workspace || ws_bytes < dedup_layout(nullptr, max_lookups, nullptr))
    return fail(TT_ECAPACITY, std::string(what) + ": workspace too small");
  if (reinterpret_cast<uintptr_t>(workspace) & 63) return fail(TT_EINVAL, std::string(what) + ": workspace not 64-B aligned");
  return TT_OK;
}


int dedup_update_args(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F, int64_t B,
                      const float* grad, int64_t ldg, float* weights, float* state, float lr, float eps,
                      void* workspace, size_t ws_bytes, int64_t max_lookups, DdUpdateArgs& a, int64_t* grid) {
  int rc = pack_meta(a.m, tables, T, features, F, B);
  if (rc) return rc;
  rc = check_dd_ws(workspace, ws_bytes, max_lookups, "dedup_rowwise_adagrad");
  if (rc) return rc;
  const int64_t n = (int64_t)F * B;
  if (n > max_lookups) return fail(TT_ECAPACITY, "dedup_rowwise_adagrad: F*B > max_lookups");
  if (!grad || !weights || !state) return fail(TT_EINVAL, "dedup_rowwise_adagrad: null pointer");
  if ((ldg % 4) || (reinterpret_cast<uintptr_t>(grad) & 15) || (reinterpret_cast<uintptr_t>(weights) & 15))
    return fail(TT_EINVAL, "dedup_rowwise_adagrad: grad/weights must be 16-B aligned with ldg % 4 == 0");
  for (int t = 0; t < T; ++t)
    if (tables[t].dim > 128 || tables[t].dim % 4 || tables[t].weight_offset % 4)
      return fail(TT_EINVAL, "dedup_rowwise_adagrad: needs D % 4 == 0, D <= 128 (16-B rows)");
  for (int f = 0; f < F; ++f)
    if (features[f].out_offset % 4) return fail(TT_EINVAL, "dedup_rowwise_adagrad: out_offset % 4 != 0");
  dedup_layout(workspace, max_lookups, &a.ws);
  a.grad = grad;
  a.ldg = ldg;
  a.n = n;
  a.weights = weights;
  a.state = state;
  a.lr = lr;
  a.eps = eps;
  // a hot row takes a team of up to DD_HOT_TEAM workgroups (dd_hot_role, dd_hot_team)
  // 64 hot workgroups: every one that finds no hot row still checks in, and at uniform ids (no hot
  // rows) 128 cost the ring's tail launch ~0.3 us on MI355X while halving the Zipf tail's hot rows
  int64_t hot_max = 64;
#if TT_EXPERIMENTS
  if (const char* e = getenv("TT_DD_HOT_WGS")) hot_max = std::max(8, atoi(e));  // EXPERIMENT (A/B)
#endif
  a.hot_wgs = (int)std::min<int64_t>(hot_max, std::max<int64_t>(1, max_lookups / (DD_INL + 1)));
  a.slot_hw = ceil_div(ceil_div(max_lookups, DD_SPH), 8) * 8;
  *grid = a.hot_wgs + a.slot_hw / 8;
  return TT_OK;
}

}  // namespace tt

using namespace tt;

extern "C" {

size_t tt_dedup_workspace_bytes(int64_t max_lookups) {
  return dedup_layout(nullptr, std::max<int64_t>(1, max_lookups), nullptr);
}

int tt_dedup_workspace_init(void* workspace, size_t ws_bytes, int64_t max_lookups, void* stream) {
  int rc = check_dd_ws(workspace, ws_bytes, max_lookups, "dedup_workspace_init");
  if (rc) return rc;
  DedupWs w;
  dedup_layout(workspace, max_lookups, &w);
  hipStream_t st = as_stream(stream);
  // every slot word EMPTY (all ones; items unused), counters 0
  if (hipMemsetAsync(w.slots, 0xff, sizeof(DSlot) * w.cap, st) != hipSuccess ||
      hipMemsetAsync(w.ctr, 0, sizeof(int32_t) * 4, st) != hipSuccess ||
      hipMemsetAsync(w.hcnt, 0, sizeof(int32_t) * w.hot_cap, st) != hipSuccess ||
      hipMemsetAsync(w.ovf, 0xff, sizeof(DedupWs::Ovf) * 64 * w.ovf_groups, st) != hipSuccess)
    return fail(TT_EINVAL, "dedup_workspace_init: memset failed");
  if (hipStreamSynchronize(st) != hipSuccess) return fail(TT_EINVAL, "dedup_workspace_init: sync failed");
  return TT_OK;
}

int tt_dedup_resolve(void* workspace, size_t ws_bytes, int64_t max_lookups, void* stream) {
  int rc = check_dd_ws(workspace, ws_bytes, max_lookups, "dedup_resolve");
  if (rc) return rc;
  DedupWs w;
  dedup_layout(workspace, max_lookups, &w);
  dd_resolve_kernel<<<dim3(DD_RES_WGS), dim3(256), 0, as_stream(stream)>>>(w);
  return check_launch("dedup_resolve");
}

int tt_dedup_insert_cols(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F, int64_t B,
                         const void* const* cols, int id_dtype, const int64_t* num_embeddings, void* workspace,
                         size_t ws_bytes, int64_t max_lookups, void* stream) {
  EmbMeta m{};
  int rc = pack_meta(m, tables, T, features, F, B);
  if (rc) return rc;
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "dedup_insert_cols: ids must be int32/int64");
  if (!cols || !num_embeddings) return fail(TT_EINVAL, "dedup_insert_cols: null pointer");
  ColArgsD ca{};
  for (int f = 0; f < F; ++f) {
    if (!cols[f] || num_embeddings[f] < 1) return fail(TT_EINVAL, "dedup_insert_cols: null column or N < 1");
    if (num_embeddings[f] > tables[features[f].table].num_rows)
      return fail(TT_EINVAL, "dedup_insert_cols: num_embeddings exceeds the table's rows");
    if (tables[features[f].table].num_rows >= (1ll << DD_TABLE_SHIFT))
      return fail(TT_EINVAL, "dedup_insert_cols: table rows >= 2^40");
    ca.col[f] = cols[f];
    ca.num_emb[f] = num_embeddings[f];
  }
  if (max_lookups < (int64_t)F * B) return fail(TT_ECAPACITY, "dedup_insert_cols: max_lookups < F*B");
  rc = check_dd_ws(workspace, ws_bytes, max_lookups, "dedup_insert_cols");
  if (rc) return rc;
  const int64_t n = (int64_t)F * B;
  if (n == 0) return TT_OK;
  DedupWs w;
  dedup_layout(workspace, max_lookups, &w);
  const int grid = (int)std::min<int64_t>(32768, ceil_div(n, 64));
  dd_insert_cols_kernel<<<dim3(grid), dim3(64), 0, as_stream(stream)>>>(m, ca, id_dtype, w);
  return check_launch("dedup_insert_cols");
}

int tt_dedup_insert_segments(const int64_t* keys, const int32_t* counts, int64_t num_segments, int64_t seg_capacity,
                             void* workspace, size_t ws_bytes, int64_t max_lookups, void* stream) {
  if (num_segments < 0 || seg_capacity < 0) return fail(TT_EINVAL, "dedup_insert_segments: negative size");
  const int64_t n = num_segments * seg_capacity;
  if (max_lookups < n) return fail(TT_ECAPACITY, "dedup_insert_segments: max_lookups < segments x capacity");
  int rc = check_dd_ws(workspace, ws_bytes, max_lookups, "dedup_insert_segments");
  if (rc) return rc;
  if (n == 0) return TT_OK;
  if (!keys || !counts) return fail(TT_EINVAL, "dedup_insert_segments: null pointer");
  DedupWs w;
  dedup_layout(workspace, max_lookups, &w);
  const int grid = (int)std::min<int64_t>(32768, ceil_div(n, 64));
  dd_insert_segments_kernel<<<dim3(grid), dim3(64), 0, as_stream(stream)>>>(keys, counts, seg_capacity, n, w);
  return check_launch("dedup_insert_segments");
}

int tt_dedup_rowwise_adagrad(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F,
                             int64_t B, const float* grad, int64_t ldg, float* weights, float* state, float lr,
                             float eps, void* workspace, size_t ws_bytes, int64_t max_lookups, void* stream) {
  DdUpdateArgs a{};
  int64_t grid = 0;
  int rc = dedup_update_args(tables, T, features, F, B, grad, ldg, weights, state, lr, eps, workspace, ws_bytes,
                             max_lookups, a, &grid);
  if (rc) return rc;
  dd_adagrad_kernel<<<dim3((unsigned)grid), dim3(256), 0, as_stream(stream)>>>(a);
  return check_launch("dedup_rowwise_adagrad");
}

}  // extern "C"

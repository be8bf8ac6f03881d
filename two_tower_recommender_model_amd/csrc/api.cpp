// Error plumbing and small host helpers of the C ABI (no kernels here).
#include <hip/hip_runtime.h>
#include <string>
#include "tt_common.h"

namespace tt {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int pack_meta(EmbMeta& m, const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features,
              int F, int64_t B) {
  if (T < 1 || T > TT_MAX_TABLES) return fail(TT_EINVAL, "table count out of range [1, 64]");
  if (F < 1 || F > TT_MAX_FEATURES) return fail(TT_EINVAL, "feature count out of range [1, 64]");
  if (B < 0) return fail(TT_EINVAL, "negative batch size");
  if (!tables || !features) return fail(TT_EINVAL, "null table/feature metadata");
  for (int t = 0; t < T; ++t) {
    if (tables[t].dim < 1) return fail(TT_EINVAL, "table dim must be >= 1");
    if (tables[t].num_rows < 0) return fail(TT_EINVAL, "negative table rows");
    m.tables[t] = tables[t];
  }
  for (int f = 0; f < F; ++f) {
    if (features[f].table < 0 || features[f].table >= T)
      return fail(TT_EINVAL, "feature references a table index out of range");
    if (features[f].out_offset < 0 || features[f].out_row < 0) return fail(TT_EINVAL, "negative feature output offset/row");
    m.features[f] = features[f];
  }
  m.T = T;
  m.F = F;
  m.B = B;
  return TT_OK;
}

}  // namespace tt

extern "C" {

const char* tt_last_error_string(void) { return tt::g_last_error.c_str(); }

int tt_abi_version(void) { return TT_ABI_VERSION; }

// tt_kjt_build_mod_dropzero, tt_complete_cumsum, tt_kjt_permute, tt_block_bucketize, tt_pooled_fwd,
// tt_bwd_workspace_init, tt_bwd_prepare, tt_bwd_rowwise_adagrad, tt_pooled_bwd_dense,
// tt_linear_fwd, tt_linear_bwd_data, tt_linear_bwd_weight, tt_dot_bce_workspace_init,
// tt_dot_bce_fwd_bwd, tt_adam_step, tt_tower_workspace_init, tt_tower_fwd_bwd, tt_tower_wgrad,
// tt_tower_update
// tt_pooled_fwd_cols, tt_bwd_prepare_cols
// tt_dedup_workspace_init, tt_dedup_insert_cols, tt_dedup_insert_segments, tt_dedup_rowwise_adagrad
// tt_tower_fwd_bwd_indexed, tt_shard_route_cols, tt_shard_gather_rows, tt_shard_gather_rows_bf16,
// tt_tower_fwd_bwd_indexed_bf16, tt_tower_adam_grads, tt_tower_update_pre, tt_tower_wgrad_pre,
// tt_dedup_resolve
// tt_shard_route_segs, tt_shard_gather_segs_bf16, tt_tower_fwd_bwd_indexed2_bf16, tt_tower_grads_replicated,
// tt_tower_fwd_bwd_gather_update, tt_tower_adam_pre_grads_sum
// tt_tower_fwd_bwd_kjt, tt_tower_fwd_bwd_gather, tt_tower_fwd_bwd_indexed_multi_bf16
// tt_launch (every multi-role fused launch, by plan)
// tt_kjt_single_hot_cols
// tt_kjt_route, tt_kjt_unpack, tt_pooled_partials_sum, tt_pooled_grad_pack
// tt_bwd_rowwise_adagrad_part
// tt_peer_exchange
// tt_kjt_admit
// tt_table_prefault
int tt_num_entry_points(void) { return 53; }

}  // extern "C"

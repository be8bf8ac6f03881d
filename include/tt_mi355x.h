/*
 * tt_mi355x.h — C ABI of libtt_mi355x.so, the MI355X-native (gfx950) sparse + tower hot path of
 * the two-tower training step of alexmillerdb/two_tower_recommender_model.
 *
 * Every entry point takes raw device pointers, sizes and a hipStream_t (passed as void*), is
 * asynchronous on that stream, never allocates, frees or synchronises (the one exception: the
 * device-initiated exchange's SETUP calls tt_peer_alloc / _free / _export / _import / _unimport,
 * which allocate, map and synchronise; called once per buffer at setup, never per step), and returns 0 on success
 * or a non-zero status (a hipError_t value, or one of the TT_E* codes below). The message of the
 * last failure on the calling thread is returned by tt_last_error_string(). No C++ exception
 * crosses this boundary. The caller owns every buffer, including workspaces (size queries first).
 *
 * What each entry point replaces (reference call site -> the pinned third-party op it reaches):
 *   tt_kjt_build_mod_dropzero  <- transform_to_torchrec_batch, 03_model_training.py:353-382
 *                                 (host loop :356-365 + KeyedJaggedTensor.from_lengths_sync :367-371)
 *   tt_complete_cumsum         <- torch.ops.fbgemm.asynchronous_complete_cumsum (KJT offsets,
 *                                 KeyedJaggedTensor built at 03_model_training.py:367-371)
 *   tt_kjt_permute             <- torch.ops.fbgemm.permute_2D_sparse_data (KJT.permute inside
 *                                 ShardedEmbeddingBagCollection.input_dist, reached from
 *                                 DistributedModelParallel at 03_model_training.py:812-815)
 *   tt_block_bucketize         <- torch.ops.fbgemm.block_bucketize_sparse_features (row-wise
 *                                 input_dist, same call site)
 *   tt_pooled_fwd              <- EmbeddingBagCollection.forward / FBGEMM TBE forward
 *                                 (self.ebc(kjt), 03_model_training.py:417)
 *   tt_bwd_prepare +
 *   tt_bwd_rowwise_adagrad     <- TBE backward with EXACT_ROWWISE_ADAGRAD fused in backward
 *                                 (_apply_optimizer_in_backward(RowWiseAdagrad, ...),
 *                                 03_model_training.py:791-795)
 *   tt_pooled_bwd_dense        <- nn.EmbeddingBag dense backward (unfused EBC, no optimizer in bwd)
 *   tt_linear_fwd / _bwd_data /
 *   tt_linear_bwd_weight       <- torchrec.modules.mlp.MLP / Perceptron (Linear + ReLU every layer),
 *                                 query_proj / candidate_proj, 03_model_training.py:411-412,:420-436
 *   tt_dot_bce_fwd_bwd         <- TwoTowerTrainTask.forward, 03_model_training.py:447-455
 *                                 ((q*c).sum(1).squeeze() + BCEWithLogitsLoss(mean) + its backward)
 *   tt_adam_step               <- KeyedOptimizerWrapper(torch.optim.Adam), 03_model_training.py:826-829
 *   tt_pooled_fwd_cols +
 *   tt_bwd_prepare_cols        <- transform_to_torchrec_batch (03:353-380) + EBC forward (03:417) +
 *                                 the fused backward, for single-hot columns: the KJT is never built
 *   tt_tower_fwd_bwd / tt_tower_wgrad / tt_tower_update
 *                              <- both MLP towers (03:411-412, :420-436) + TwoTowerTrainTask
 *                                 (03:447-455) + loss.backward() through the towers + the dense
 *                                 Adam step (03:826-829), as three fused kernels
 *   tt_launch (a launch plan)  <- the same backward work with several roles in one launch: the
 *                                 weight gradients beside the embedding update / next-batch insert /
 *                                 shard route and gather ("launch plans" below)
 */
#ifndef TT_MI355X_H
#define TT_MI355X_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: tt_tower_shape_t._pad became `flags`; the 12 role-combination exports became tt_launch
 * 3: the measured-and-rejected fused-T3 forms removed (tt_tower_fwd_bwd_gather_update_t3,
 *    tt_tower_fwd_bwd_indexed2_bf16_t3, tt_tower_update_lazy, tt_tower_t3_fuse_supported,
 *    tt_tower_counter_offset; the WGRAD | INSERT | ADAGRAD | UPDATE launch plan)
 * 4: direct stores into the peers' receive buffers (tt_peer_direct_t): tt_tower_fwd_bwd_indexed2_bf16
 *    gained its `direct` argument, tt_gather_role_t its `direct` field (last) */
#define TT_ABI_VERSION 4

/* ---- device-initiated exchange: the producer stores straight into the peers' buffers ------------
 * A producer of an all-to-all's send buffer (the sharded step's T1 for exchange A, the owner's
 * gather for exchange B) given a tt_peer_direct_t writes each unit (row) of destination block d at
 * row0[d] + (row - first_row[d]) * row_bytes — destination d's receive buffer as mapped into this
 * process (tt_peer_import) — instead of into the send buffer; block d holds rows [first_row[d],
 * first_row[d + 1]). The copy fields name further bytes (the exchange's non-row region) that the
 * producer copies to each destination beside its rows. Only the exchange's signal / wait then runs
 * (tt_peer_exchange with every len 0). NULL: the send buffer is written as before. */
#define TT_PEER_MAXW 16
typedef struct {
  int32_t W;                             /* destination blocks, 1..TT_PEER_MAXW */
  int32_t _pad;
  int64_t first_row[TT_PEER_MAXW];       /* ascending; first_row[0] = 0 */
  void* row0[TT_PEER_MAXW];              /* mapped address of row first_row[d] at destination d */
  const void* copy_src[TT_PEER_MAXW];    /* 16-B aligned; NULL / copy_len 0: nothing to copy */
  void* copy_dst[TT_PEER_MAXW];          /* 16-B aligned mapped address at destination d */
  int64_t copy_len[TT_PEER_MAXW];        /* bytes, a multiple of 16 */
  int32_t* epoch;                        /* nullable: the exchange's epoch word (this rank's), advanced
                                            by one by the producer (a tt_peer_wait_t consumer follows) */
} tt_peer_direct_t;

/* The consumer of such an exchange signals and waits INSIDE its own launch instead of a separate
 * signal / wait kernel: workgroup 0's first W threads store the epoch into the peers' flag words
 * for this source (release: system scope when sys, else a relaxed agent-scope store after the
 * producer's kernel boundary), and every workgroup that reads the received blocks polls this
 * rank's W flag words (relaxed, bounded by timeout_ticks of s_memrealtime, 100 MHz; a wait that
 * gives up sets *err, sticky) and then acquires (system scope when sys) before its reads — the
 * consumer's other roles start at once. The epoch is the one the producer advanced
 * (tt_peer_direct_t.epoch). Only for ranks on different devices or a single rank: ranks sharing a
 * device could fill every CU with spinning workgroups (the caller uses the signal / wait kernel
 * there). */
typedef struct {
  int32_t W;                             /* ranks, 1..TT_PEER_MAXW */
  int32_t sys;                           /* 1: system-scope release / acquire */
  int32_t* flag[TT_PEER_MAXW];           /* mapped: peer d's flag word for this source */
  const int32_t* flags;                  /* this rank's W flag words */
  const int32_t* epoch;                  /* this rank's epoch word of the exchange */
  int32_t* err;                          /* sticky: a wait gave up */
  int64_t timeout_ticks;
} tt_peer_wait_t;

/* status codes (besides hipError_t values, which are all < 1000) */
#define TT_OK 0
#define TT_EINVAL 1001      /* bad argument (shape, dtype, null pointer, limit exceeded) */
#define TT_ECAPACITY 1002   /* workspace too small for the requested lookups */

/* dtypes used at the boundary */
#define TT_I32 0
#define TT_I64 1
#define TT_F32 2
#define TT_BF16 3

/* pooling modes (torchrec PoolingType) */
#define TT_POOL_SUM 0
#define TT_POOL_MEAN 1

#define TT_MAX_FEATURES 64
#define TT_MAX_TABLES 64

/* One embedding table resident in a flat fp32 weight buffer (FBGEMM-TBE style "weights" +
 * "weights_offsets"), with its row-wise optimizer state in a flat fp32 buffer. */
typedef struct {
  int64_t weight_offset; /* element offset of row 0 in the flat weight buffer */
  int64_t state_offset;  /* element offset of row 0 in the flat row-wise state buffer */
  int64_t num_rows;      /* rows held by this shard (local rows) */
  int32_t dim;           /* embedding dim D (any value >= 1; D % 4 == 0 is the fast path) */
  int32_t _pad;
} tt_table_meta_t;

/* One KJT key (feature) -> its table and where its bags land in the pooled output: bag b of this
 * key is row (out_row + b), columns [out_offset, out_offset + D). out_row = 0 for an ordinary
 * [B, sum D] KeyedTensor; sharded lookups stack source ranks as row blocks (out_row = s * B). */
typedef struct {
  int32_t table;      /* index into the table array */
  int32_t out_offset; /* first column of this feature in the pooled output row */
  int64_t out_row;    /* first output row of this feature's bags */
} tt_feature_meta_t;

const char* tt_last_error_string(void);
int tt_abi_version(void);
/* number of exported compute entry points (used by the loader to check the symbol table) */
int tt_num_entry_points(void);

/* ---- a1/a2: KeyedJaggedTensor build + offsets --------------------------------------------- */

/* Workspace bytes needed by tt_kjt_build_mod_dropzero for n = F*B elements. */
size_t tt_kjt_build_workspace_bytes(int64_t n);

/* For key f in [0,F) and row b in [0,B): id = cols[f][b]. If id != 0 ("if value:",
 * 03_model_training.py:358) the element contributes value id mod num_embeddings[f] (Python/torch
 * floor-mod: result in [0, N)) and length 1, else length 0. Values are compacted key-major in
 * (f, b) order, exactly like the reference's host loop. cols is a HOST array of F device pointers
 * of dtype id_dtype; values_out (capacity F*B, dtype id_dtype), lengths_out [F*B] int32,
 * offsets_out [F*B+1] int32 (complete cumsum), length_per_key_out [F] int64 (nullable). */
int tt_kjt_build_mod_dropzero(int F, int64_t B, const void* const* cols, int id_dtype,
                              const int64_t* num_embeddings, void* values_out,
                              int32_t* lengths_out, int32_t* offsets_out,
                              int64_t* length_per_key_out, void* workspace, size_t ws_bytes,
                              void* stream);

/* Single-hot KJT (every bag 0 or 1 ids, e.g. the reference's transform_to_torchrec_batch output,
 * 03_model_training.py:353-380) -> the F id columns the fused single-hot kernels take (the inverse
 * of tt_kjt_build_mod_dropzero on its output): cols_out[f][b] = 0 for an empty bag, else its value
 * v, or num_embeddings[f] for v == 0 (row 0 through the kernels' id mod N). offsets [F*B+1] int32;
 * cols_out is a HOST array of F device pointers of dtype id_dtype (capacity B each). A bag of more
 * than one id sets bit 0 of *err, a value outside [0, N) bit 1 (sticky: the caller zeroes it and
 * checks it when it wants; such bags get column entry 0). labels_out (nullable): the batch's B
 * labels (int32 / int64, label_dtype) copied as int32 in the same launch. Replaces nothing in
 * TorchRec: the glue between TrainPipelineSparseDist's KJT batches and the fused step (dropin.py). */
int tt_kjt_single_hot_cols(int F, int64_t B, const void* values, int id_dtype, const int32_t* offsets,
                           const int64_t* num_embeddings, void* const* cols_out, int32_t* err, const void* labels,
                           int label_dtype, int32_t* labels_out, void* stream);

size_t tt_complete_cumsum_workspace_bytes(int64_t n);
/* offsets[0] = 0, offsets[i+1] = sum(lengths[0..i]); n may be 0. */
int tt_complete_cumsum(const int32_t* lengths, int64_t n, int32_t* offsets, void* workspace,
                       size_t ws_bytes, void* stream);

/* permute_2D_sparse_data: keys of a [F][B] jagged tensor reordered by perm (HOST array of F_out
 * key indices, repeats allowed). out_offsets [F_out*B+1]. values may carry optional fp32
 * per-value weights (weights/out_weights nullable). out_values capacity must be >= the permuted
 * total, which the caller bounds (e.g. by the input total when perm is a permutation). */
int tt_kjt_permute(int F, int64_t B, const int32_t* lengths, const int32_t* offsets,
                   const void* values, int id_dtype, const float* weights, const int32_t* perm,
                   int F_out, int32_t* out_lengths, int32_t* out_offsets, void* out_values,
                   float* out_weights, void* stream);

size_t tt_block_bucketize_workspace_bytes(int F, int64_t B, int W);
/* block_bucketize_sparse_features (row-wise input_dist), keep_orig_idx = false:
 * for id in bag (f,b): bs = block_sizes[f] (host); p = id < bs*W ? id / bs : id % W;
 * local = id < bs*W ? id % bs : id / W. Output is bucket-major [W][F][B]: new_lengths
 * [W*F*B], new_offsets [W*F*B+1], new_values (capacity = input total), order inside a
 * (bucket, bag) = input order. */
int tt_block_bucketize(int F, int64_t B, const int32_t* lengths, const int32_t* offsets,
                       const void* values, int id_dtype, const int64_t* block_sizes, int W,
                       int32_t* new_lengths, int32_t* new_offsets, void* new_values,
                       void* workspace, size_t ws_bytes, void* stream);

/* ---- a4: pooled (segmented gather + sum) forward ------------------------------------------- */

/* out[b, features[f].out_offset + d] = pool_{i in bag(f,b)} W_t[values[i], d] for every key f and
 * row b; empty bags give 0. offsets [F*B+1] int32 (key-major KJT offsets). ldo = row stride of out
 * in elements. bounds_check: 0 = trust ids; 1 = ids outside [0, num_rows) read row 0 (FBGEMM
 * BoundsCheckMode.WARNING) and are counted into *err_count (device int32, nullable). */
int tt_pooled_fwd(const float* weights, const tt_table_meta_t* tables, int T,
                  const tt_feature_meta_t* features, int F, int64_t B, const void* values,
                  int id_dtype, const int32_t* offsets, int pooling, float* out, int64_t ldo,
                  int bounds_check, int32_t* err_count, void* stream);

/* Single-hot column form of the reference's batch (one [B] id column per key, the loader's
 * dict at 03_model_training.py:356-357): the transform of transform_to_torchrec_batch is applied
 * inline (id 0 -> empty bag -> zero row; otherwise row = id mod num_embeddings[f], Python
 * floor-mod), so the result equals tt_kjt_build_mod_dropzero followed by tt_pooled_fwd (SUM),
 * without materialising the KJT. cols: HOST array of F device pointers. */
int tt_pooled_fwd_cols(const float* weights, const tt_table_meta_t* tables, int T,
                       const tt_feature_meta_t* features, int F, int64_t B, const void* const* cols,
                       int id_dtype, const int64_t* num_embeddings, float* out, int64_t ldo,
                       void* stream);

/* ---- a8: deduplicated backward + fused exact row-wise Adagrad -------------------------------- */

/* Workspace for up to max_lookups ids per step (max_lookups < 2^24; table rows < 2^34 - 1). Must be
 * initialised once by tt_bwd_workspace_init; every prepare leaves the hash clean again for the next
 * step. */
size_t tt_bwd_workspace_bytes(int64_t max_lookups);
int tt_bwd_workspace_init(void* workspace, size_t ws_bytes, int64_t max_lookups, void* stream);

/* Group the step's lookups by unique (table,row) (FBGEMM's linearize + radix sort + run-length
 * encode, done as a hash): per chunk of 1024 lookups the duplicates are merged in an LDS hash, each
 * (chunk, row) pair pays ONE global CAS (key and count share a 64-bit slot word), a scan assigns
 * segments (rows looked up more than once first), and a chunk scatter fills them (one cursor
 * atomic per (chunk, row), none for a row whose lookups sit in one chunk); a row looked up once
 * gets no segment, its lookup is marked for the direct update. Depends only on the ids, so it may
 * run concurrently with the forward and the towers. values must stay valid until the matching
 * tt_bwd_rowwise_adagrad, which must be given the same offsets. */
int tt_bwd_prepare(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F,
                   int64_t B, const void* values, int id_dtype, const int32_t* offsets,
                   int bounds_check, void* workspace, size_t ws_bytes, int64_t max_lookups,
                   void* stream);

/* The same grouping for the single-hot column form (see tt_pooled_fwd_cols); lookup index =
 * bag index, max_lookups >= F*B. Follow with tt_bwd_rowwise_adagrad (pooling SUM, offsets may
 * be NULL). */
int tt_bwd_prepare_cols(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features,
                        int F, int64_t B, const void* const* cols, int id_dtype,
                        const int64_t* num_embeddings, void* workspace, size_t ws_bytes,
                        int64_t max_lookups, void* stream);

/* For every unique row r of table t touched this step:
 *   G[r]   = sum over its lookups of grad_out[b, out_offset(f) : +D]  (x 1/len for MEAN pooling)
 *   s[r]  += mean_d G[r,d]^2
 *   W[r,d] = W[r,d] + (-lr * G[r,d]) / (sqrt(s[r]) + eps)
 * (torchrec RowWiseAdagrad, lr_decay = weight_decay = 0). Bitwise reproducible: rows of 2..32
 * lookups are summed in ascending bag order, hotter rows over fixed bag-id ranges (ascending inside
 * a range, ranges in order); rows looked up once (KJT form) are updated in lookup order. */
int tt_bwd_rowwise_adagrad(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features,
                           int F, int64_t B, const float* grad_out, int64_t ldg,
                           const int32_t* offsets, int pooling, float* weights, float* state,
                           float lr, float eps, void* workspace, size_t ws_bytes,
                           int64_t max_lookups, void* stream);
/* The same update in two parts that touch disjoint rows, for two streams: part 1 the rows looked up
 * once (KJT form: offsets required), part 2 every other row (2..32 lookups and the hot rows); part 0
 * is tt_bwd_rowwise_adagrad. Both parts read the same completed grouping and gradient. Parts 1 / 2
 * need the narrow path (rows of D <= 128, 16-B aligned: TT_EINVAL otherwise). */
int tt_bwd_rowwise_adagrad_part(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F,
                                int64_t B, const float* grad_out, int64_t ldg, const int32_t* offsets, int pooling,
                                float* weights, float* state, float lr, float eps, void* workspace, size_t ws_bytes,
                                int64_t max_lookups, int part, void* stream);

/* Unfused backward: grad_weights (flat, same layout as weights) += scatter of grad_out rows.
 * Uses fp32 atomics (summation order not fixed). */
int tt_pooled_bwd_dense(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features,
                        int F, int64_t B, const float* grad_out, int64_t ldg, const void* values,
                        int id_dtype, const int32_t* offsets, int pooling, float* grad_weights,
                        int bounds_check, void* stream);

/* ---- a6: tower GEMMs on MFMA (fp32 accumulate) ------------------------------------------------ */

/* A grouped launch runs `groups` (1 or 2: the two towers) independent problems of equal shape.
 * Pointer arrays are HOST arrays of `groups` device pointers. compute = TT_BF16 (operands rounded
 * to bf16, v_mfma_f32_16x16x32_bf16: the production mode) or TT_F32 (exact fp32 operands,
 * v_mfma_f32_16x16x4_f32: the fp32 parity mode). */

/* Y[m,n] = act(sum_k X[m,k] W[n,k] + bias[n]); X fp32 or bf16 (x_dtype), W [N,K] fp32 row-major
 * (nn.Linear layout), bias nullable, act = relu if relu != 0. Y fp32 with row stride ldy. */
int tt_linear_fwd(int groups, const void* const* X, int x_dtype, int64_t ldx,
                  const float* const* W, const float* const* bias, int64_t M, int N, int K,
                  float* const* Y, int64_t ldy, int relu, int compute, void* stream);

/* dX[m,k] = sum_n dZ[m,n] W[n,k], dZ = dY * (Y > 0) if relu (Y nullable when relu == 0). */
int tt_linear_bwd_data(int groups, const float* const* dY, const float* const* Y, int64_t ldy,
                       const float* const* W, int64_t M, int N, int K, float* const* dX,
                       int64_t ldx, int relu, int compute, void* stream);

size_t tt_linear_bwd_weight_workspace_bytes(int groups, int64_t M, int N, int K);
/* dW[n,k] = sum_m dZ[m,n] X[m,k]; db[n] = sum_m dZ[m,n] (db nullable). Split over M with fp32
 * slabs in the workspace, summed in a fixed order (bitwise reproducible). */
int tt_linear_bwd_weight(int groups, const float* const* dY, const float* const* Y, int64_t ldy,
                         const void* const* X, int x_dtype, int64_t ldx, int64_t M, int N, int K,
                         float* const* dW, float* const* db, int relu, int compute,
                         void* workspace, size_t ws_bytes, void* stream);

/* ---- a7: logits = sum_d q*c ; loss = mean BCEWithLogits ; dlogit = (sigmoid - y) / B ---------- */

size_t tt_dot_bce_workspace_bytes(int64_t B);
/* Must be zeroed once (tt_dot_bce_workspace_init); each call leaves it clean. labels: TT_I32,
 * TT_I64 or TT_F32. logits [B] fp32; loss scalar fp32 (mean); dq/dc (nullable: forward only)
 * receive dlogit*c and dlogit*q, scaled by grad_scale (d loss_total / d loss). */
int tt_dot_bce_workspace_init(void* workspace, size_t ws_bytes, int64_t B, void* stream);
int tt_dot_bce_fwd_bwd(const float* q, int64_t ldq, const float* c, int64_t ldc, int64_t B,
                       int dim, const void* labels, int label_dtype, float* logits, float* loss,
                       float* dq, int64_t lddq, float* dc, int64_t lddc, float grad_scale,
                       void* workspace, size_t ws_bytes, void* stream);

/* ---- a6+a7+a9 fused: both towers' MLP step, dot + BCE, Adam (3 launches) --------------------- */

/* Two towers of L layers each (Linear + ReLU on every layer); tower t reads pooled columns
 * [in_col[t], in_col[t] + in_dim[t]). Flat fp32 parameter layout: for t in (query, candidate),
 * for l < L: W_(t,l) [width[l]][in_l] row-major, then b_(t,l) [width[l]]; in_0 = in_dim[t],
 * in_l = width[l-1]. Limits: L <= 4; widths multiples of 32 in [32, 128]; in_dim multiples of
 * 32 in [32, 1024]; in_col % 4 == 0; B % 8 == 0. bf16 MFMA operands, fp32 accumulation. */
typedef struct {
  int32_t L;
  int32_t width[4];
  int32_t in_dim[2];
  int32_t in_col[2];
  int32_t flags; /* TT_TOWER_GENERAL_T1: T1 is always the general kernel (several features per tower,
                    tt_tower_fwd_bwd_indexed_multi_bf16), so T3 keeps its plain bf16 weight copies
                    even for 2-layer shapes <= 128 wide; every other T1 entry point returns TT_EINVAL
                    for such a shape. 0 otherwise; any other bit is TT_EINVAL. (ABI 2: this field
                    was `_pad` in ABI 1 — zero it.) */
} tt_tower_shape_t;
#define TT_TOWER_GENERAL_T1 1

int64_t tt_tower_num_params(const tt_tower_shape_t* shape);
size_t tt_tower_workspace_bytes(const tt_tower_shape_t* shape, int64_t B);
/* Zero the workspace and upload the T2 tile list (synchronises `stream`: call at setup only).
 * The workspace also holds the bf16 weight copies: run tt_tower_update(do_adam = 0) after
 * (re)loading parameters. */
int tt_tower_workspace_init(const tt_tower_shape_t* shape, int64_t B, void* workspace, size_t ws_bytes,
                            void* stream);
/* T1: forward of both towers, logits, BCE and its gradient back through every layer; dX written
 * into gpooled's tower-input columns (ld = ldp; pooled and gpooled 16-B aligned). Leaves, in the
 * workspace, what T2 needs (transposed operands, bias and loss partials). */
int tt_tower_fwd_bwd(const tt_tower_shape_t* shape, int64_t B, const float* pooled, int64_t ldp,
                     float* gpooled, const float* params, const void* labels, int label_dtype,
                     float grad_scale, float* logits, void* workspace, size_t ws_bytes, void* stream);
/* T1 with the EBC forward fused in, for single-hot columns (one key per tower, L = 2, inputs
 * <= 128 wide): tower t's input row m is row (cols[t][m] mod num_embeddings[t]) of the table
 * starting at table_rows[t] ([rows][in_dim[t]] fp32, 16-B aligned), zeros when the id is 0
 * (transform_to_torchrec_batch semantics, 03_model_training.py:356-365); the pooled rows are
 * never materialised unless pooled_out (nullable, ld = ldp, columns in_col[t]) is given.
 * With dedup_ws (nullable; a tt_dedup workspace) every kept lookup (tower t, row m) is also
 * inserted as lookup t * B + m with key dedup_tables[t] << 40 | row, ready for
 * tt_dedup_rowwise_adagrad over gpooled (features t -> columns in_col[t]). */
int tt_tower_fwd_bwd_gather(const tt_tower_shape_t* shape, int64_t B, const void* const* cols, int id_dtype,
                            const int64_t* num_embeddings, const float* const* table_rows,
                            float* pooled_out, int64_t ldp, float* gpooled, const float* params,
                            const void* labels, int label_dtype, float grad_scale, float* logits,
                            const int32_t* dedup_tables, void* dedup_ws, size_t dedup_ws_bytes,
                            int64_t dedup_max_lookups, void* workspace, size_t ws_bytes, void* stream);
/* T1 with the multi-hot EBC forward fused in (KeyedJaggedTensor input, one key per tower, L = 2,
 * towers [128, 64], inputs 64 or 128 wide): tower t's input row m is the SUM pool of bag (t, m),
 * i.e. rows values[offsets[t*B + m] .. offsets[t*B + m + 1]) of table_rows[t] (num_rows[t] rows;
 * ids are taken as the EBC takes them, an id >= num_rows[t] reads row 0) — bit-identical to
 * tt_pooled_fwd (SUM) followed by tt_tower_fwd_bwd, without materialising the pooled rows unless
 * pooled_out (nullable) is given. Replaces self.ebc(kjt) + the towers' forward/backward of
 * 03_model_training.py:417-455 for the config-5 multi-hot shape. offsets: complete, key-major
 * [2B + 1] int32. dX goes to gpooled's columns in_col[t] (ld = ldp) for tt_bwd_rowwise_adagrad. */
int tt_tower_fwd_bwd_kjt(const tt_tower_shape_t* shape, int64_t B, const void* values, int id_dtype,
                         const int32_t* offsets, const int64_t* num_rows, const float* const* table_rows,
                         float* pooled_out, int64_t ldp, float* gpooled, const float* params,
                         const void* labels, int label_dtype, float grad_scale, float* logits,
                         void* workspace, size_t ws_bytes, void* stream);
/* ---- the pipelined fused step: dedup one step ahead, single-lookup rows updated inside T1 ----------
 * Step i (the production ring): T1 (gather + towers + in-place row-wise Adagrad of batch i's rows
 * looked up ONCE, from batch i's dedup table completed by step i-1) -> the tail (tt_launch roles
 * WGRAD | INSERT | ADAGRAD: weight gradients + the complete insert of batch i+1 into the other
 * table + the rows looked up more than once) -> T3 (tt_tower_update_pre). The first batch's table
 * is built by tt_dedup_insert_cols. */
/* T1 as tt_tower_fwd_bwd_gather, plus: a kept lookup (t, m) whose slot in dedup_ws (its claim, count
 * 1) says its row is looked up once in the step updates table_rows[t] / table_state[t] in place
 * (lr, eps: torchrec RowWiseAdagrad, 03_model_training.py:791-795); dX goes to gpooled for the
 * others (for every lookup with pooled_out). Shapes: in_dim in {64, 128}, widths [128, 64].
 * It also hands dedup_ws over to the update that follows (a role with ADAGRAD.multi_only = 1): the
 * table's hot-row count moves to the update's word (the insert count is zeroed for the table's next
 * fill), and with the row-owned T1 (the default for these shapes) the slots of the rows it updated
 * are freed and the slots of rows looked up 2..30 times are listed per wave for the tail. */
int tt_tower_fwd_bwd_gather_update(const tt_tower_shape_t* shape, int64_t B, const void* const* cols, int id_dtype,
                                   const int64_t* num_embeddings, float* const* table_rows, float* const* table_state,
                                   float* pooled_out, int64_t ldp, float* gpooled, const float* params,
                                   const void* labels, int label_dtype, float grad_scale, float* logits, float lr,
                                   float eps, void* dedup_ws, size_t dedup_ws_bytes, int64_t dedup_max_lookups,
                                   const void* const* next_cols, void* workspace, size_t ws_bytes, void* stream);
/* T1 for the sharded step (row-wise / table-wise shards, single-hot): tower t's input row m is row
 * pos[t][m] of rows_in[t] ([*][in_dim[t]] fp32: the rows returned by the owners' all-to-all; -1
 * -> zeros, a dropped id), and its gradient row dX is written to row pos[t][m] of grad_rows_out[t]
 * (the buffer the gradient all-to-all sends back to the owners). Replaces the EBC lookup's output
 * KeyedTensor + the towers (03_model_training.py:417-455) on the sharded path. */
int tt_tower_fwd_bwd_indexed(const tt_tower_shape_t* shape, int64_t B, const int32_t* const* pos,
                             const float* const* rows_in, float* const* grad_rows_out, const float* params,
                             const void* labels, int label_dtype, float grad_scale, float* logits,
                             void* workspace, size_t ws_bytes, void* stream);
/* The same with bf16 rows_in (from tt_shard_gather_rows_bf16): T1 computes on bf16 inputs anyway,
 * so the result is bit-identical to the fp32-row form, and the rows all-to-all moves half the bytes. */
int tt_tower_fwd_bwd_indexed_bf16(const tt_tower_shape_t* shape, int64_t B, const int32_t* const* pos,
                                  const void* const* rows_in, float* const* grad_rows_out, const float* params,
                                  const void* labels, int label_dtype, float grad_scale, float* logits,
                                  void* workspace, size_t ws_bytes, void* stream);
/* T2: weight/bias gradients of every layer into the workspace (fixed-order partial slabs), and
 * the mean BCE of the preceding T1 into loss[0] (nullable; fixed-order sum of T1's partials). */
int tt_tower_wgrad(const tt_tower_shape_t* shape, int64_t B, float* loss, void* workspace, size_t ws_bytes,
                   void* stream);
/* T2 alone (tt_tower_wgrad) that also advances the Adam step and precomputes the step's
 * bias-correction scalars for tt_tower_update_pre (or a tt_launch plan's UPDATE role) (the fused
 * single-GPU step: T1 -> this -> T3 + embedding update). With dedup_ws (nullable) the same launch
 * finishes the dedup inserts T1 deferred (as tt_dedup_resolve). Replaces the towers' autograd
 * weight gradients (03_model_training.py:455) and the step-count part of Adam (:826-829). */
int tt_tower_wgrad_pre(const tt_tower_shape_t* shape, int64_t B, float* loss, void* workspace, size_t ws_bytes,
                       int64_t* adam_step_state, float adam_lr, float adam_beta1, float adam_beta2, void* dedup_ws,
                       size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream);
/* T3 after tt_tower_wgrad_pre or a tt_launch WGRAD role (adam_step_state != NULL): reduction
 * + Adam with the precomputed scalars + bf16 copies. */
int tt_tower_update_pre(const tt_tower_shape_t* shape, int64_t B, float* params, float* exp_avg, float* exp_avg_sq,
                        float eps, float beta1, float beta2, float weight_decay, float* grads_out, void* workspace,
                        size_t ws_bytes, void* stream);
/* T3: fixed-order reduction of T2's partials, Adam (when do_adam; step_state as tt_adam_step),
 * and the bf16 weight copies for the next T1. grads_out (nullable) receives the gradient. */
int tt_tower_update(const tt_tower_shape_t* shape, int64_t B, float* params, float* exp_avg,
                    float* exp_avg_sq, float lr, float beta1, float beta2, float eps,
                    float weight_decay, int64_t* step_state, int do_adam, float* grads_out,
                    void* workspace, size_t ws_bytes, void* stream);

/* ---- a8 (single-hot): two-launch dedup + fused row-wise Adagrad --------------------------------
 * For single-hot lookups (the fused step's id columns; the sharded step's received ids) this
 * replaces tt_bwd_prepare(_cols) + tt_bwd_rowwise_adagrad (TBE backward with EXACT_ROWWISE_ADAGRAD,
 * _apply_optimizer_in_backward(RowWiseAdagrad, ...), 03_model_training.py:791-795) with one insert
 * launch and one update launch. Lookup i of the step maps to pooled-gradient row
 * (features[f].out_row + b) * ldg + features[f].out_offset with f = i / B, b = i % B.
 * The workspace is clean between steps (the update resets what the insert wrote); initialise it
 * once with tt_dedup_workspace_init (synchronises `stream`). 64-B aligned. */
size_t tt_dedup_workspace_bytes(int64_t max_lookups);
int tt_dedup_workspace_init(void* workspace, size_t ws_bytes, int64_t max_lookups, void* stream);
/* Finishes the inserts that tt_tower_fwd_bwd_gather (dedup on) deferred: a lookup whose first CAS
 * did not claim a free slot is listed by T1 and filed here (probe / count). Run it between T1 and
 * the update (tt_tower_wgrad_pre with the dedup workspace does the same inside its launch). */
int tt_dedup_resolve(void* workspace, size_t ws_bytes, int64_t max_lookups, void* stream);
/* lookups i = f * B + b: key (table of feature f, cols[f][b] mod num_embeddings[f]); id 0 dropped */
int tt_dedup_insert_cols(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F, int64_t B,
                         const void* const* cols, int id_dtype, const int64_t* num_embeddings, void* workspace,
                         size_t ws_bytes, int64_t max_lookups, void* stream);
/* lookups i = s * seg_capacity + k, k < counts[s]: keys[i] = local table << 40 | local row */
int tt_dedup_insert_segments(const int64_t* keys, const int32_t* counts, int64_t num_segments, int64_t seg_capacity,
                             void* workspace, size_t ws_bytes, int64_t max_lookups, void* stream);
/* sum every unique row's gradient rows (ascending lookup order; rows with > 30 lookups: fixed
 * 8-way interleave), then s += mean(G^2), w -= lr * G / (sqrt(s) + eps). D % 4 == 0, D <= 128. */
int tt_dedup_rowwise_adagrad(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F,
                             int64_t B, const float* grad, int64_t ldg, float* weights, float* state, float lr,
                             float eps, void* workspace, size_t ws_bytes, int64_t max_lookups, void* stream);

/* ---- a10 (single-hot): sharded lookups with fixed-size exchanges (csrc/shard.hip) ------------------
 * Replace ShardedEmbeddingBagCollection's input_dist (KJT permute + block_bucketize_sparse_features
 * + lengths/values all-to-all) and output_dist (pooled all-to-all / reduce-scatter), reached from
 * DistributedModelParallel at 03_model_training.py:812-815, for single-hot features, with an id
 * exchange (ids out, rows back, gradient rows out) whose buffers have a fixed size, so RCCL
 * all-to-alls sit inside one HIP graph. Segment (d, f) of capacity C holds the lookups of feature f
 * owned by rank d, in ascending bag order. */
/* requester: send[d] = {count(d, f) for f < F; keys (f << 40 | local row) of segment (d, f) at
 * F + f * C + k}; pos[f * B + b] = (d * F + f) * C + k, or -1 (id 0). block_sizes[f] > 0: row-wise
 * (owner = (id mod N) / block); 0: table-wise (owner = owners[f]). W <= 16. A segment over capacity
 * sets *overflow (sticky; results invalid). */
size_t tt_shard_route_workspace_bytes(int F, int64_t B);
int tt_shard_route_cols(int F, int64_t B, const void* const* cols, int id_dtype, const int64_t* num_embeddings,
                        const int64_t* block_sizes, const int32_t* owners, int W, int64_t seg_capacity,
                        int64_t* send, int32_t* pos, int32_t* overflow, void* workspace, size_t ws_bytes,
                        void* stream);
/* owner: rows_out[(s * F + f) * C + k] = local table f's row of the received key (all tables one
 * dim D, D % 4 == 0), and, with dedup_ws, that slot inserted as lookup (s * F + f) * C + k (then
 * tt_dedup_rowwise_adagrad(F = 1, B = W * F * C) on the received gradient rows). A key outside the
 * local shard sets *bad (sticky). */
int tt_shard_gather_rows(const float* weights, const tt_table_meta_t* tables, int T, int F, int W,
                         int64_t seg_capacity, const int64_t* recv, float* rows_out, int32_t* bad, void* dedup_ws,
                         size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream);
/* The same with rows_out in bf16 (round to nearest even), for tt_tower_fwd_bwd_indexed_bf16. */
int tt_shard_gather_rows_bf16(const float* weights, const tt_table_meta_t* tables, int T, int F, int W,
                              int64_t seg_capacity, const int64_t* recv, void* rows_out, int32_t* bad, void* dedup_ws,
                              size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream);

/* ---- a10 (single-hot), pipelined: TWO collectives per step ------------------------------------
 * Exchange A (requester -> owner, one all-to-all with fixed per-destination sizes) carries, in the
 * block for destination d: [gradient rows of step i: S_d x D fp32 | tower gradient of step i: P fp32
 * (padded to a multiple of D) | counts: F int64 | keys of step i+1: S_d int64 | pad], S_d = sum over f
 * of the capacity of segment (d, f). Exchange B (owner -> requester) returns the rows (bf16) of the
 * received keys. Replaces ShardedEmbeddingBagCollection's input_dist (KJT all-to-all), output_dist
 * (pooled all-to-all / reduce-scatter) and their adjoints, and DDP's all-reduce of the towers'
 * gradients (03_model_training.py:812-815): the next batch's ids travel with this batch's gradients.
 * Segment (d, f) = the lookups of feature f owned by rank d, ascending bag order. */
typedef struct {
  int64_t cap;        /* slots of segment (d, f); 0 when rank d holds no rows of feature f */
  int64_t key_index;  /* int64 index (send buffer viewed as int64) of slot 0's key */
  int64_t cnt_index;  /* int64 index of the segment's count */
  int32_t pos_in;     /* row of slot 0 in the requester's returned-rows buffer (exchange B output) */
  int32_t pos_out;    /* row (units of D floats) of slot 0's gradient row in the send buffer */
} tt_shard_seg_t;

/* requester: every kept lookup (id 0 dropped, row = id mod N, 03_model_training.py:356-365) of
 * feature f owned by d (row-wise: (row / block_sizes[f]); table-wise: owners[f]) takes slot k of
 * segment (d, f): send[key_index + k] = f << 40 | local row, send[cnt_index] = count (<= cap),
 * pos_in[f * B + b] = pos_in + k, pos_out[f * B + b] = pos_out + k (both -1 for id 0). segs: DEVICE
 * array [W][F]. A segment over capacity sets *overflow (sticky; the step's results are invalid). */
int tt_shard_route_segs(int F, int64_t B, const void* const* cols, int id_dtype, const int64_t* num_embeddings,
                        const int64_t* block_sizes, const int32_t* owners, int W, const tt_shard_seg_t* segs,
                        int64_t* send, int32_t* pos_in, int32_t* pos_out, int32_t* overflow, void* workspace,
                        size_t ws_bytes, void* stream);
/* owner: source s's block of the received buffer starts at recv + s * block_i64 (int64 units), its
 * counts at + counts_i64, feature f's keys at + counts_i64 + F + seg_off[f] (seg_off: host [F],
 * ascending, slots = S). Slot j of source s: rows_out[s * out_stride + j] (out_stride >= S rows) =
 * the local row (bf16, round to nearest even) and, with dedup_ws, lookup s * S + j inserted for
 * tt_dedup_rowwise_adagrad (one pseudo-feature per source: B = S, out_row = the row of source s's
 * gradient block). Tables: one per feature (table f = feature f), one dim. A key outside the shard
 * sets *bad (sticky). */
int tt_shard_gather_segs_bf16(const float* weights, const tt_table_meta_t* tables, int T, int F, int W,
                              const int64_t* recv, int64_t block_i64, int64_t counts_i64, const int64_t* seg_off,
                              int64_t slots, void* rows_out, int64_t out_stride, int32_t* bad, void* dedup_ws,
                              size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream);
/* T1 of the pipelined sharded step: tt_tower_fwd_bwd_indexed_bf16 with the dX row of (tower t,
 * bag m) written at row pos_out[t][m] (units of in_dim floats) of grad_rows_out[t] — the gradient
 * region of exchange A's send buffer — instead of at its input row. direct (nullable, ABI 4): that
 * row goes to its destination's receive buffer instead (row units of in_dim floats, rows counted
 * from grad_rows_out[0] == grad_rows_out[1]), and the copy fields' bytes (exchange A's key region)
 * travel beside them. */
int tt_tower_fwd_bwd_indexed2_bf16(const tt_tower_shape_t* shape, int64_t B, const int32_t* const* pos_in,
                                   const int32_t* const* pos_out, const void* const* rows_in,
                                   float* const* grad_rows_out, const float* params, const void* labels,
                                   int label_dtype, float grad_scale, float* logits, void* workspace, size_t ws_bytes,
                                   const tt_peer_direct_t* direct, void* stream);
/* T1 of the pipelined sharded step with SEVERAL single-hot features per tower (BASELINE configs 3
 * and 4: 8 table-wise features per tower, 1024-wide tower inputs; TorchRec KeyedTensor slices
 * concatenated per tower, 03_model_training.py:420-436, generalised as in
 * ray_tune_optuna_tuning_alex_test.py:270-306): features are numbered query first
 * (f < in_dim[0] / D), then candidate; column k of tower t is column k % D of bf16 row
 * pos_in[f * B + m] of rows_in (f = tower t's first feature + k / D; -1 -> zeros, a dropped id),
 * and its dX column goes to column k % D of row pos_out[f * B + m] of grad_rows_out (-1: none).
 * Any tower width the general T1 takes (inputs up to 1024); D in {16, 32, 64, 128}. */
int tt_tower_fwd_bwd_indexed_multi_bf16(const tt_tower_shape_t* shape, int64_t B, int D, const int32_t* pos_in,
                                        const int32_t* pos_out, const void* rows_in, float* grad_rows_out,
                                        const float* params, const void* labels, int label_dtype, float grad_scale,
                                        float* logits, void* workspace, size_t ws_bytes, void* stream);
/* T3 without Adam: the reduced tower gradient, times `scale`, written at base + offsets[q] for
 * q < copies <= 16 (offsets: host array, floats) — the tower region of every destination block of
 * exchange A: DDP's mean all-reduce becomes a fixed-order sum on the receivers. */
int tt_tower_grads_replicated(const tt_tower_shape_t* shape, int64_t B, float* params, float* base, int copies,
                              const int64_t* offsets, float scale, void* workspace, size_t ws_bytes, void* stream);
/* T3 with Adam on the gradient sum_{s < nsrc} grads[s * src_stride + i] (ascending s: identical on
 * every rank) + the bf16 weight copies, with the step scalars a preceding WGRAD role (tt_tower_wgrad_pre,
 * or launch U of the pipelined sharded step) wrote into the workspace: no pow() per thread. */
int tt_tower_adam_pre_grads_sum(const tt_tower_shape_t* shape, int64_t B, float* params, const float* grads, int nsrc,
                                int64_t src_stride, float* exp_avg, float* exp_avg_sq, float eps, float beta1,
                                float beta2, float weight_decay, void* workspace, size_t ws_bytes,
                                const tt_peer_wait_t* wait, void* stream);
/* (wait, nullable, ABI 4: every workgroup waits for the exchange that brought the W gradients;
 * workgroup 0 signals it first — tt_peer_wait_t) */

/* T3 with the gradient taken from `grads` (data-parallel towers: the all-reduced gradient) instead
 * of T2's partials: Adam + the bf16 weight copies. */
int tt_tower_adam_grads(const tt_tower_shape_t* shape, int64_t B, float* params, const float* grads,
                        float* exp_avg, float* exp_avg_sq, float lr, float beta1, float beta2, float eps,
                        float weight_decay, int64_t* step_state, void* workspace, size_t ws_bytes, void* stream);

/* Admission counts of one KJT batch for the N > 1 drop-in (dropin.FusedShardedDropin; what TorchRec's
 * input_dist learns from its host-read split sizes, torchrec/distributed/embeddingbag.py, reached
 * from 03_model_training.py:648, :812-815): out[0] = 1 if a bag holds more than one id, out[1] = 2
 * if a value lies outside [0, num_embeddings[f]), out[2 + d * F + f] = the ids of feature f that
 * owner d would receive (row-wise: id / block_sizes[f]; table-wise: owners[f]). out (int32
 * [2 + W * F]) is zeroed by the call (memset + one kernel, asynchronous). offsets: int32
 * [F * B + 1] of the key-major KJT, nnz = offsets[F * B]. W <= 16. */
int tt_kjt_admit(int F, int64_t B, const void* values, int id_dtype, int64_t nnz, const int32_t* offsets,
                 const int64_t* num_embeddings, const int64_t* block_sizes, const int32_t* owners, int W, int32_t* out,
                 void* stream);

/* Setup helper, no reference counterpart (TorchRec's tables pay the same cold page-table walks in
 * their first training iterations, 03_model_training.py:648's loop): one 4-byte load per page_bytes
 * of [base, base + bytes) (bytes / 4 words, the tail page included), asynchronous on `stream`. It
 * warms the address translations of the embedding tables before the first step; nothing is
 * written except, never in practice, one word of `sink` (device, 4 bytes). page_bytes: a multiple
 * of 4 (4096 = the GPU page). ABI 4. */
int tt_table_prefault(const void* base, size_t bytes, size_t page_bytes, uint32_t* sink, void* stream);

/* SETUP ONLY (allocating, synchronising): device memory for embedding tables on the current
 * device, physically contiguous when the driver can give it (hipDeviceMallocContiguous: the largest
 * page fragments for the random row gathers; *contiguous = 1), plain device memory otherwise
 * (*contiguous = 0; contiguous may be NULL). Uninitialised. Free with tt_table_free (NULL is a
 * no-op). No reference counterpart: FBGEMM's TBE allocates its weights through the caching
 * allocator (torchrec, reached from 03_model_training.py:812-815). ABI 4. */
int tt_table_alloc(size_t bytes, void** out, int* contiguous);
int tt_table_free(void* p);

/* ---- multi-hot sharded step (config 5, sharded_kjt.py): fixed-size exchanges ------------------------
 * TorchRec's KJTAllToAll / PooledEmbeddingsAllToAll / reduce-scatter (torchrec/distributed/embeddingbag.py,
 * reached from 03_model_training.py:812-815) exchange variable split sizes the host reads every batch;
 * here every exchange block has a fixed size, so the step is capturable. Requester -> owner block d
 * (int32, blk_stride elements): [lengths [F][B] of the ids d owns | those ids (row in d's shard) in
 * (feature, bag, position) order, capacity cap]. A row-wise feature's owner is id / block_sizes[f]
 * (block_sizes[f] > 0), a table-wise one's owners[f]. flags[0] (sticky): some destination got more
 * than cap ids; flags[1]: an id outside [0, num_embeddings[f]) (skipped). W <= 16. */
size_t tt_kjt_route_workspace_bytes(int F, int64_t B, int W);
int tt_kjt_route(int F, int64_t B, const void* values, int id_dtype, const int32_t* offsets,
                 const int64_t* num_embeddings, const int64_t* block_sizes, const int32_t* owners, int W, int64_t cap,
                 int64_t blk_stride, int32_t* send, int32_t* flags, void* workspace, size_t ws_bytes, void* stream);
/* Owner side: the W received blocks -> one KJT whose keys are (source s, served feature k) (feats[k],
 * ascending; Fr of them): lengths_out [W*Fr*B], offsets_out [W*Fr*B + 1] (complete cumsum), the ids
 * compacted into values_out (capacity W*cap). */
size_t tt_kjt_unpack_workspace_bytes(int W, int Fr, int64_t B);
int tt_kjt_unpack(int W, int F, int64_t B, const int32_t* recv, int64_t blk_stride, int64_t cap, const int32_t* feats,
                  int Fr, int32_t* lengths_out, int32_t* offsets_out, int32_t* values_out, void* workspace,
                  size_t ws_bytes, void* stream);
/* Requester side of the pooled exchange: owner d's block (blk_stride floats) holds rows of ld_blk floats, bag b
 * of feature f at row b, column owner_col[d*F + f] (-1: d does not serve f). partials_sum: out[b][f*D ..] =
 * the sum over d (ascending) of those rows (row-wise: TorchRec's reduce-scatter; table-wise: one term).
 * grad_pack: the inverse copy of the bag gradients grad[b][f*D ..] into every serving owner's block. */
int tt_pooled_partials_sum(int W, int F, int64_t B, int D, const float* recv, int64_t blk_stride, int64_t ld_blk,
                           const int32_t* owner_col, float* out, int64_t ldo, void* stream);
int tt_pooled_grad_pack(int W, int F, int64_t B, int D, const float* grad, int64_t ldg, const int32_t* owner_col,
                        float* send, int64_t blk_stride, int64_t ld_blk, void* stream);

/* ---- launch plans: the step's multi-role fused launches through ONE entry point ------------------
 * A fused launch runs several ROLES side by side in one grid (each role a range of workgroups): the
 * towers' weight gradients beside the embedding update, the next batch's dedup insert or route
 * beside both, so the work after T1 shares the CUs behind one launch boundary. Instead of an export
 * per combination the caller names the roles (tt_launch_plan_t.roles) and fills each named role's
 * arguments; tt_launch checks the set against the fused launches the library implements:
 *
 *   roles                          the launch (reference work it replaces)
 *   WGRAD | INSERT | ADAGRAD       single-GPU ring tail: T2 + the next batch's complete insert + the
 *                                  rows looked up more than once (ADAGRAD.multi_only = 1); T1 updated
 *                                  the others (03:455 backward + 03:791-795 RowWiseAdagrad)
 *   WGRAD | INSERT                 T2 + the next batch's insert, first CAS only (the rest deferred
 *                                  to the RESOLVE role of the following launch)
 *   UPDATE | ADAGRAD | RESOLVE     T3 + rows looked up more than once (multi_only = 1) + the
 *                                  deferred inserts of RESOLVE.dedup_ws (03:826-829, :791-795)
 *   WGRAD | ADAGRAD                T2 + every row's update (multi_only = 0)
 *   UPDATE | ADAGRAD               T3 + every row's update (multi_only = 0)
 *   WGRAD | ROUTE_COUNT | ADAGRAD  sharded launch U: T2 + a later batch's route count pass + the
 *                                  owner's update of the received gradient rows (multi_only = 0)
 *   ROUTE_COUNT | ADAGRAD          launch U without T2 (T2 on a parallel graph branch)
 *   UPDATE | ROUTE_PLACE | GATHER  sharded launch G: the tower gradient x scale into every
 *                                  destination block (UPDATE.replicated = 1, no Adam) + the route's
 *                                  place pass + the owner's gather of the next batch's rows (bf16)
 *
 * and fails with TT_EINVAL for any other set. A role's fields mean what the single-role entry
 * point's arguments of the same name mean (tt_tower_wgrad_pre, tt_tower_update_pre /
 * tt_tower_grads_replicated, tt_dedup_insert_cols, tt_dedup_resolve, tt_dedup_rowwise_adagrad,
 * tt_shard_route_segs, tt_shard_gather_segs_bf16). The towers' shape / B / workspace are the plan's. */
#define TT_ROLE_WGRAD 0x01u       /* T2: weight-gradient tiles, bias / loss sums, Adam step scalars */
#define TT_ROLE_UPDATE 0x02u      /* T3: gradient reduction + Adam + bf16 weight copies */
#define TT_ROLE_INSERT 0x04u      /* the next batch's dedup insert from its single-hot id columns */
#define TT_ROLE_RESOLVE 0x08u     /* finish deferred dedup inserts */
#define TT_ROLE_ADAGRAD 0x10u     /* row-wise Adagrad of the dedup workspace's rows */
#define TT_ROLE_ROUTE_COUNT 0x20u /* sharded route, count pass (tt_shard_route_segs' first half) */
#define TT_ROLE_ROUTE_PLACE 0x40u /* sharded route, place pass (its second half) */
#define TT_ROLE_GATHER 0x80u      /* the owner's gather of the received keys' rows (bf16) */

typedef struct {
  float* loss;               /* nullable: mean BCE of the preceding T1 */
  int64_t* adam_step_state;  /* advanced; the step scalars go to the workspace for UPDATE */
  float adam_lr, adam_beta1, adam_beta2;
} tt_wgrad_role_t;

typedef struct {
  float* params;
  float* exp_avg;
  float* exp_avg_sq;
  float eps, beta1, beta2, weight_decay;
  float* grads_out;        /* nullable: the reduced gradient */
  int32_t replicated;      /* 1: no Adam; gradient x scale to base + offsets[q], q < copies <= 16 */
  int32_t copies;
  float* base;
  const int64_t* offsets;  /* host array, floats (any flat address: a direct exchange points copy q
                              into destination q's mapped receive buffer) */
  float scale;
} tt_update_role_t;

typedef struct {
  const void* const* next_cols;  /* host array of 2 device id columns (towers 0, 1) */
  int32_t id_dtype;
  const int64_t* num_embeddings; /* host [2] */
  const int32_t* dedup_tables;   /* host [2]: key table index of each tower */
  void* next_dedup_ws;
  size_t dedup_ws_bytes;
  int64_t dedup_max_lookups;
} tt_insert_role_t;

typedef struct {
  void* dedup_ws;  /* bytes / max lookups: the ADAGRAD role's */
} tt_resolve_role_t;

typedef struct {
  const tt_table_meta_t* tables;
  int32_t T;
  int32_t F;
  const tt_feature_meta_t* features;
  int64_t B;               /* lookups per feature (WGRAD | INSERT | ADAGRAD, the ring tail: 0 or the plan's B) */
  const float* grad;
  int64_t ldg;
  float* weights;
  float* state;
  float lr, eps;
  void* dedup_ws;
  size_t dedup_ws_bytes;
  int64_t dedup_max_lookups;
  int32_t multi_only;      /* 1: only rows looked up more than once (T1 updated the others) */
} tt_adagrad_role_t;

typedef struct {
  int32_t F;
  int32_t id_dtype;
  const void* const* cols;
  const int64_t* num_embeddings;
  const int64_t* block_sizes;
  const int32_t* owners;
  int32_t W;
  const tt_shard_seg_t* segs;
  int64_t* send;
  int32_t* pos_in;
  int32_t* pos_out;
  int32_t* overflow;
  void* route_ws;
  size_t route_ws_bytes;
} tt_route_role_t;

typedef struct {
  const float* weights;
  const tt_table_meta_t* tables;
  int32_t T;
  const int64_t* recv;
  int64_t block_i64, counts_i64;
  const int64_t* seg_off;
  int64_t slots;
  void* rows_out;
  int64_t out_stride;
  int32_t* bad;
  void* dedup_ws;
  size_t dedup_ws_bytes;
  int64_t dedup_max_lookups;
  const tt_peer_direct_t* direct; /* nullable (ABI 4): source s's rows to row0[s] + j rows (first_row[s] =
                                     s * out_stride); the copy fields are not used */
} tt_gather_role_t;

typedef struct {
  uint32_t roles;                 /* TT_ROLE_* bits */
  const tt_tower_shape_t* shape;  /* the towers (WGRAD, UPDATE; the batch size B for the others) */
  int64_t B;
  void* workspace;
  size_t ws_bytes;
  tt_wgrad_role_t wgrad;
  tt_update_role_t update;
  tt_insert_role_t insert;
  tt_resolve_role_t resolve;
  tt_adagrad_role_t adagrad;
  tt_route_role_t route;          /* ROUTE_COUNT / ROUTE_PLACE */
  tt_gather_role_t gather;        /* F and W: the route's */
  const tt_peer_wait_t* wait;     /* nullable (ABI 4): the ADAGRAD role's workgroups of launch U wait for
                                     the exchange that brought their gradient rows (the others start
                                     at once); workgroup 0 signals it first */
} tt_launch_plan_t;

int tt_launch(const tt_launch_plan_t* plan, void* stream);

/* ---- a9: Adam on the flat dense-parameter buffer (torch.optim.Adam, amsgrad=False) ------------ */

/* step_state: device int64[2] = {steps taken so far, arrival counter (0)}; the kernel uses
 * t = step_state[0] + 1 and advances it, so the call is graph-replayable. */
int tt_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n,
                 float lr, float beta1, float beta2, float eps, float weight_decay,
                 int64_t* step_state, void* stream);

/* ---- device-initiated fixed-block exchange (sharded.PeerComm; the sharded steps' N > 1 default) -----
 * Replaces dist.all_to_all_single on the sharded step's data path: the all-to-alls TorchRec's
 * ShardedEmbeddingBagCollection input_dist / output_dist issue under DistributedModelParallel
 * (03_model_training.py:812-815) and DDP's gradient all-reduce of the towers (:812), both reached
 * through TrainPipelineSparseDist.progress (:648). Each rank stores its blocks straight into every
 * peer's receive buffer (mapped with hipIpcOpenMemHandle) and signals one flag word per (peer,
 * source); the receiver waits on its W flag words.
 * SETUP ONLY: tt_peer_alloc / tt_peer_free / tt_peer_export / tt_peer_import / tt_peer_unimport
 * allocate (hipExtMallocWithFlags), map (hipIpcOpenMemHandle) and synchronise — the only entry
 * points of this library that do; the caller runs them once per receive buffer, before any step,
 * never inside a graph capture. tt_peer_exchange is asynchronous like every compute entry point. */
#define TT_PEER_HANDLE_BYTES 64

typedef struct {
  int32_t W, rank;
  const void* src;                 /* this rank's send buffer */
  int64_t src_off[TT_PEER_MAXW];   /* bytes: where destination d's block starts in src */
  int64_t len[TT_PEER_MAXW];       /* bytes sent to d (multiple of 4, 4-B aligned; 16 B: wide copy) */
  void* dst[TT_PEER_MAXW];         /* d's receive buffer at this rank's slot (mapped address) */
  int32_t* flag[TT_PEER_MAXW];     /* d's flag word for this source (mapped address) */
  int32_t* state;                  /* this rank's epoch word for the exchange (int32) */
  int32_t same_device;             /* every rank on this device: agent-scope signals (else system) */
  int32_t _pad;
} tt_peer_put_t;

/* SETUP: fine-grained device memory, zeroed (hipExtMallocWithFlags(hipDeviceMallocFinegrained),
 * hipMemset, hipDeviceSynchronize) */
int tt_peer_alloc(size_t bytes, void** out);
int tt_peer_free(void* p);
/* IPC handle (TT_PEER_HANDLE_BYTES) of the allocation holding p, and p's offset in it */
int tt_peer_export(const void* p, void* handle, int64_t* offset);
int tt_peer_import(const void* handle, void** base);
int tt_peer_unimport(void* base);
/* block d of src -> dst[d]; then flag[d] = epoch + 1 (release, system scope) and a wait until
 * flags[0..W) >= epoch + 1 (acquire, system scope), then epoch += 1. A wait longer than timeout_s
 * gives up and sets *err = 1 (sticky; the exchange's data is then invalid). Two kernels; one (the
 * signal / wait) when every len is 0 — the producers stored the data (tt_peer_direct_t). */
int tt_peer_exchange(const tt_peer_put_t* p, const int32_t* flags, int32_t* err, double timeout_s, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TT_MI355X_H */

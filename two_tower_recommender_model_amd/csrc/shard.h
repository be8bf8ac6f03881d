// Device code of the sharded route (requester side of input_dist), shared by csrc/shard.hip (its
// own launches) and csrc/tower.hip (the route of the next batch as extra workgroups of the towers'
// T2 / T3 launches in the pipelined sharded step). See shard.hip for the exchange's layout.
#pragma once

#include "dedup.h"

namespace tt {

constexpr int RT_BLOCK = 256;  // bags per workgroup of the two route kernels
constexpr int RT_MAXW = 16;

struct RouteArgs {
  const void* col[TT_MAX_FEATURES];
  int64_t num_emb[TT_MAX_FEATURES];  // id mod N divisor
  int64_t block[TT_MAX_FEATURES];    // row-wise block size (> 0), or 0: table-wise
  int32_t owner[TT_MAX_FEATURES];    // table-wise owner rank
  int id_dtype;
  int F;
  int W;
  int64_t B;
  int64_t C;
  int nblk;           // workgroups per feature = ceil(B / RT_BLOCK)
  int64_t* send;      // [W][F + F * C]
  int32_t* pos;       // [F][B]
  int32_t* overflow;  // sticky flag
  int64_t* dl;        // [F][B] workspace: owner << 48 | local row, -1 = dropped
  int32_t* cnt;       // [F][nblk][RT_MAXW] workspace: lookups per (block, owner)
  // segment-table form (tt_shard_route_segs): per (owner d, feature f) capacity and addresses in
  // the packed send buffer; pos_out (nullable) = the lookup's gradient row in that buffer
  const tt_shard_seg_t* segs;
  int32_t* pos_out;
};

// route pass 1 (thread per bag, coalesced): owner + local row of every lookup, and per-workgroup
// per-owner counts (wave ballots, summed in wave order)
// one 256-thread workgroup (bags blk * 256 .. of feature f); wc: RT_BLOCK / 64 x RT_MAXW ints of LDS
__device__ __forceinline__ void route_count_block(const RouteArgs& a, int blk, int f, int (*wc)[RT_MAXW]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t b = (int64_t)blk * RT_BLOCK + threadIdx.x;
  int d = -1;
  int64_t lr = 0;
  if (b < a.B) {
    const int64_t id = load_id(a.col[f], a.id_dtype, b);
    if (id != 0) {
      const int64_t row = py_mod64(id, a.num_emb[f]);
      if (a.block[f] > 0) {
        d = (int)udiv64(row, a.block[f]);
        lr = row - (int64_t)d * a.block[f];
      } else {
        d = a.owner[f];
        lr = row;
      }
    }
    a.dl[(int64_t)f * a.B + b] = d >= 0 ? (int64_t)(((uint64_t)d << 48) | (uint64_t)lr) : -1;
  }
  for (int w = 0; w < a.W; ++w) {
    const uint64_t m = __ballot(d == w);
    if (lane == 0) wc[wid][w] = __popcll(m);
  }
  __syncthreads();
  if (threadIdx.x < a.W) {
    int t = 0;
    for (int v = 0; v < RT_BLOCK / 64; ++v) t += wc[v][threadIdx.x];
    a.cnt[((int64_t)f * a.nblk + blk) * RT_MAXW + threadIdx.x] = t;
  }
}

// route pass 2: slot k = (lookups of the same owner in earlier workgroups) + (earlier waves) +
// (earlier lanes): ascending bag order inside each (owner, feature) segment. SEGS: per-(owner,
// feature) capacities and addresses from the segment table (tt_shard_route_segs), else the
// uniform layout of tt_shard_route_cols.
template <bool SEGS>
__device__ __forceinline__ void route_place_block(const RouteArgs& a, int blk, int f, int* base, int (*wc)[RT_MAXW]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t seg_stride = (int64_t)a.F + (int64_t)a.F * a.C;
  const int32_t* cf = a.cnt + (int64_t)f * a.nblk * RT_MAXW;
  if (threadIdx.x < a.W) {
    int t = 0, all = 0;
    for (int q = 0; q < a.nblk; ++q) {
      const int c = cf[q * RT_MAXW + threadIdx.x];
      if (q < blk) t += c;
      all += c;
    }
    base[threadIdx.x] = t;
    if (blk == 0) {  // the segment header: lookups kept for this (owner, feature)
      if (SEGS) {
        const tt_shard_seg_t sg = a.segs[(int64_t)threadIdx.x * a.F + f];
        if (all > sg.cap) atomicOr(a.overflow, 1);
        a.send[sg.cnt_index] = all < sg.cap ? all : sg.cap;
      } else {
        if (all > a.C) atomicOr(a.overflow, 1);
        a.send[(int64_t)threadIdx.x * seg_stride + f] = all < a.C ? all : a.C;
      }
    }
  }
  const int64_t b = (int64_t)blk * RT_BLOCK + threadIdx.x;
  int64_t v = -1;
  if (b < a.B) v = a.dl[(int64_t)f * a.B + b];
  const int d = v >= 0 ? (int)(v >> 48) : -1;
  int rank = 0;
  for (int w = 0; w < a.W; ++w) {
    const uint64_t m = __ballot(d == w);
    if (d == w) rank = __popcll(m & ((1ull << lane) - 1));
    if (lane == 0) wc[wid][w] = __popcll(m);
  }
  __syncthreads();
  if (b >= a.B) return;
  int32_t p = -1, po = -1;
  if (d >= 0) {
    int k = base[d] + rank;
    for (int v2 = 0; v2 < wid; ++v2) k += wc[v2][d];
    const int64_t key = (int64_t)(((uint64_t)f << DD_TABLE_SHIFT) | ((uint64_t)v & ((1ull << 48) - 1)));
    if (SEGS) {
      const tt_shard_seg_t sg = a.segs[(int64_t)d * a.F + f];
      if (k < sg.cap) {
        a.send[sg.key_index + k] = key;
        p = sg.pos_in + k;
        po = sg.pos_out + k;
      } else {
        atomicOr(a.overflow, 1);
      }
    } else if (k < a.C) {
      a.send[(int64_t)d * seg_stride + a.F + (int64_t)f * a.C + k] = key;
      p = (int32_t)(((int64_t)d * a.F + f) * a.C + k);
    } else {
      atomicOr(a.overflow, 1);
    }
  }
  a.pos[(int64_t)f * a.B + b] = p;
  if (SEGS) a.pos_out[(int64_t)f * a.B + b] = po;
}

// Owner side of the pipelined exchange (tt_shard_gather_segs_bf16, and the pipelined step's
// combined launch in csrc/tower.hip): the keys of source s sit in source block s of the received
// buffer (int64 view: block s at s * blk64, counts at + cnt64, the slots of feature f at + cnt64 + F
// + seg_off[f]); slot j of source s (j < S) -> rows_out[s * out_stride + j] (bf16) and, with the
// dedup on, lookup s * S + j. A half-wave per slot.
struct GatherSegArgs {
  const float* weights;
  tt_table_meta_t tables[TT_MAX_TABLES];
  int T;
  int F;
  int W;
  int D;
  int64_t S;
  int64_t out_stride;  // rows between source blocks of rows_out (>= S)
  int64_t blk64, cnt64;
  int64_t seg_off[TT_MAX_FEATURES + 1];
  const int64_t* recv;
  __bf16* rows_out;
  DedupWs dd;
  int dd_on;
  int32_t* bad;
  // direct exchange (dW > 0): source s's slot j -> dblk[s] + j * D (s's mapped receive buffer)
  int dW;
  int32_t* epoch;  // nullable: exchange B's epoch word, advanced by launch G's workgroup 0
  __bf16* dblk[TT_PEER_MAXW];
};

// SL slots per half-wave (slot hw + u * nhw, u < SL, nhw = ceil(W S / SL)), their loads, claiming
// CASes and row gathers interleaved: the launch's grid then fits one round of residency (one slot per
// half-wave was 2048 workgroups at 16k lookups, past the 8 per CU the combined launch G holds)
constexpr int GS_SL = 2;
__device__ __forceinline__ void shard_gather_block(const GatherSegArgs& a, int blk) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4v;
  typedef __attribute__((ext_vector_type(4))) float f32x4g;
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int64_t n = (int64_t)a.W * a.S;
  const int64_t hw = ((int64_t)blk * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const int64_t nhw = (n + GS_SL - 1) / GS_SL;
  if (hw >= nhw) return;
  int64_t iu[GS_SL], s[GS_SL], j[GS_SL], kk[GS_SL], cnt[GS_SL];
  uint64_t kraw[GS_SL];
  int fu[GS_SL];
#pragma unroll
  for (int u = 0; u < GS_SL; ++u) {
    const int64_t i = hw + u * nhw;
    iu[u] = i;
    const int64_t ic = i < n ? i : 0;
    s[u] = (int64_t)((uint32_t)ic / (uint32_t)a.S);  // W * S < 2^31 (host-checked)
    j[u] = ic - s[u] * a.S;
    // feature of slot j and its segment start: a loop over the (uniform) feature list with scalar
    // kernarg loads (a per-lane index into the kernarg arrays is a dependent vector load)
    int f = 0;
    int64_t so = a.seg_off[0];
    for (int q = 1; q < a.F; ++q)
      if (j[u] >= a.seg_off[q]) {
        f = q;
        so = a.seg_off[q];
      }
    fu[u] = f;
    kk[u] = j[u] - so;
    const int64_t* blkp = a.recv + s[u] * a.blk64 + a.cnt64;
    // the slot's key is loaded beside its segment's count (slot j lies inside the block: a stale
    // value past the count is never used), not after it: one dependent round trip fewer
    cnt[u] = blkp[f];
    kraw[u] = (uint64_t)blkp[a.F + j[u]];
  }
  uint64_t key[GS_SL];
  const float* src[GS_SL];
#pragma unroll
  for (int u = 0; u < GS_SL; ++u) {
    key[u] = DD_EMPTY;
    src[u] = nullptr;
    if (iu[u] < n && kk[u] < cnt[u]) {
      key[u] = kraw[u];
      const int t = (int)(key[u] >> DD_TABLE_SHIFT);
      const int64_t r = (int64_t)(key[u] & ((1ull << DD_TABLE_SHIFT) - 1));
      int64_t woff = 0, nrows = 0;
      int dim = 0;
      for (int q = 0; q < a.T; ++q)
        if (q == t) {
          woff = a.tables[q].weight_offset;
          nrows = a.tables[q].num_rows;
          dim = a.tables[q].dim;
        }
      if (t == fu[u] && t < a.T && r < nrows && dim == a.D) {
        src[u] = a.weights + woff + r * a.D;
      } else {
        key[u] = DD_EMPTY;
        if (hl == 0) atomicOr(a.bad, 1);
      }
    }
  }
  DdPend pend[GS_SL];
#pragma unroll
  for (int u = 0; u < GS_SL; ++u)
    if (a.dd_on && hl == 0 && iu[u] < n) dd_insert_begin(a.dd, key[u], (int32_t)iu[u], pend[u]);
  f32x4g v[GS_SL][1];
#pragma unroll
  for (int u = 0; u < GS_SL; ++u)
    v[u][0] = src[u] && hl * 4 < a.D ? *reinterpret_cast<const f32x4g*>(src[u] + hl * 4) : (f32x4g)(0.f);
#pragma unroll
  for (int u = 0; u < GS_SL; ++u) {
    if (!src[u]) continue;
    __bf16* dst = a.rows_out + (s[u] * a.out_stride + j[u]) * a.D;
    if (a.dW) {  // uniform loop, scalar kernarg loads (s differs per half-wave)
      __bf16* b0 = a.dblk[0];
#pragma unroll
      for (int q = 1; q < TT_PEER_MAXW; ++q)
        if (q < a.dW && s[u] == q) b0 = a.dblk[q];
      dst = b0 + j[u] * a.D;
    }
    for (int c = hl * 4; c < a.D; c += 128) {
      const f32x4g x = c == hl * 4 ? v[u][0] : *reinterpret_cast<const f32x4g*>(src[u] + c);
      bf16x4v o;
      o[0] = (__bf16)x[0];
      o[1] = (__bf16)x[1];
      o[2] = (__bf16)x[2];
      o[3] = (__bf16)x[3];
      *reinterpret_cast<bf16x4v*>(dst + c) = o;
    }
  }
#pragma unroll
  for (int u = 0; u < GS_SL; ++u)
    if (a.dd_on && hl == 0 && iu[u] < n) dd_insert_finish(a.dd, pend[u], (int32_t)iu[u]);
}

int gather_segs_args(const float* weights, const tt_table_meta_t* tables, int T, int F, int W, const int64_t* recv,
                     int64_t block_i64, int64_t counts_i64, const int64_t* seg_off, int64_t slots, void* rows_out,
                     int64_t out_stride, int32_t* bad, void* dedup_ws, size_t dedup_ws_bytes,
                     int64_t dedup_max_lookups, GatherSegArgs& a);

}  // namespace tt

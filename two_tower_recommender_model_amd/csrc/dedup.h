// Single-pass dedup of single-hot lookups for the fused row-wise Adagrad (gfx950).
//
// A lookup i (one id of a single-hot bag) is inserted into an open-addressing table of 128-B slots
// (one cache line) {word = key << 18 | count, items[30]}: a first-time key claims a free slot with ONE returning
// 64-bit CAS that also sets its count to 1 (the common case: a single atomic round trip); a
// repeated key finds its slot and takes a position with one atomicAdd on the same word. Positions
// < 30 store the lookup index inline, so after the insert pass every unique (table, row) owns ONE
// cache line holding everything its update needs, read in one hop by a half-wave. Rows looked up
// more than 30 times in a step ("hot") are listed by the lookup that takes position 30 and are summed by a
// workgroup that finds their lookups by scanning the per-lookup key array in index order.
#pragma once

#include "tt_common.h"

namespace tt {

constexpr uint64_t DD_EMPTY = ~0ull;
constexpr int DD_TABLE_SHIFT = 40;  // key = table << 40 | row (table < 64, rows < 2^40 per shard)
constexpr int DD_CNT_BITS = 18;     // slot word = key << 18 | count; a step has < 2^18 lookups
constexpr uint64_t DD_CNT_MASK = (1ull << DD_CNT_BITS) - 1;
constexpr int DD_INL = 30;          // lookups stored inline per slot (128-B slot: word + 30 items)
constexpr int DD_SPH = 4;           // slots per half-wave in the update launch
constexpr int DD_SEGW = 20;         // ints per T1 list segment: [0] count, [1 .. 16] slots (80 B: one
                                    // 16-B load reads the count and the first three entries)
#ifndef DD_MR
#define DD_MR 4                     // gradient rows of a multi-lookup slot in flight per half-wave
#endif

struct __attribute__((aligned(128))) DSlot {
  uint64_t word;  // DD_EMPTY when free, else key << 18 | lookups of this key in the step
  int32_t item[DD_INL];
};

struct DedupWs {
  DSlot* slots;    // [cap], clean (key EMPTY, cnt 0) between steps
  uint64_t* lkey;  // [L] key of each lookup (DD_EMPTY: dropped / padding)
  int32_t* hot;    // [L / (DD_INL + 1) + 1] slots with cnt > DD_INL
  uint64_t* hkey;  // [same] their keys, filed beside them (the hot role's first hop is the key)
  int32_t* ctr;    // [4] {hot rows, hot-workgroup ticket, hot rows as the row-owned T1 found them, -}
  int64_t cap;
  int64_t L;
  int32_t hot_cap;  // entries of `hot` (a step inserts <= L lookups: <= L / 14 hot rows)
  // deferred inserts (dd_insert_defer): lookups whose first CAS did not claim a free slot, per
  // group of 64 (one T1 workgroup), finished later by dd_resolve_block
  struct Ovf {
    uint64_t key;
    int32_t i;
    int32_t pad;
  };
  int32_t* claim;    // [L] slot claimed by lookup i (position 0 of its key), else -1: the update
                     // walks the claimers instead of all cap slots
  Ovf* ovf;          // [groups][64], key EMPTY between steps (the resolver clears what it filed)
  int32_t ovf_groups;
#if TT_EXPERIMENTS
  int64_t* stamps;  // EXPERIMENT (TT_DD_STAMPS): [update workgroups][8] s_memrealtime per phase
#endif
  // hot rows split over a team of workgroups (dd_hot_role): partial sums [hot_cap][DD_HOT_TEAM][128]
  // and per hot row the team's arrival counter (zero between launches: reset by the last arriver)
  float* hotp;
  int32_t* hcnt;
  // the ring's rows looked up 2..DD_INL times, listed by the row-owned T1 (which updates the rows
  // looked up once and frees their slots): per T1 wave (segment) of 16 lookups, its count at
  // multi[DD_SEGW seg] and its slots behind it, written every step (no reset); the tail's list role
  // updates them
  int32_t* multi;  // [nseg * DD_SEGW]
  int32_t nseg;    // capacity in segments: ceil(L / 16)
};
#if TT_EXPERIMENTS
#define DD_STAMP(k) \
  do { if (ws.stamps && threadIdx.x == 0) ws.stamps[(int64_t)bid * 8 + (k)] = (int64_t)__builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define DD_STAMP(k) do { } while (0)
#endif

__device__ __forceinline__ uint64_t dd_mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// Insert in two halves so a kernel can issue the claiming CAS early and finish late (the tower
// kernel overlaps the CAS round trip with its MFMA chain): begin stores the lookup's key and
// issues one returning CAS on the key's home slot; finish resolves the result (claimed -> position
// 0; same key -> atomicAdd for a position; other key -> linear probing) and files the lookup.
struct DdPend {
  uint64_t key;
  uint64_t prev;
  uint64_t h;
};

__device__ __forceinline__ void dd_insert_begin(const DedupWs& ws, uint64_t key, int32_t i, DdPend& p) {
  ws.lkey[i] = key;
  p.key = key;
  p.prev = 0;
  p.h = 0;
  if (key == DD_EMPTY) {
    ws.claim[i] = -1;
    return;
  }
  p.h = dd_mix64(key) & ((uint64_t)ws.cap - 1);
  p.prev = atomicCAS(reinterpret_cast<unsigned long long*>(&ws.slots[p.h].word), (unsigned long long)DD_EMPTY,
                     (unsigned long long)((key << DD_CNT_BITS) | 1ull));
}

__device__ __forceinline__ void dd_insert_finish(const DedupWs& ws, const DdPend& p, int32_t i) {
  if (p.key == DD_EMPTY) return;
  const uint64_t mask = (uint64_t)ws.cap - 1;
  const uint64_t mine = (p.key << DD_CNT_BITS) | 1ull;
  uint64_t h = p.h, prev = p.prev;
  int k;
  while (true) {
    unsigned long long* w = reinterpret_cast<unsigned long long*>(&ws.slots[h].word);
    if (prev == DD_EMPTY) {
      k = 0;
      break;
    }
    if ((prev >> DD_CNT_BITS) == p.key) {
      k = (int)(atomicAdd(w, 1ull) & DD_CNT_MASK);
      break;
    }
    h = (h + 1) & mask;
    prev = atomicCAS(reinterpret_cast<unsigned long long*>(&ws.slots[h].word), (unsigned long long)DD_EMPTY,
                     (unsigned long long)mine);
  }
  ws.claim[i] = k == 0 ? (int32_t)h : -1;
  if (k < DD_INL) {
    ws.slots[h].item[k] = i;
  } else if (k == DD_INL) {
    const int q = atomicAdd(&ws.ctr[0], 1);
    if (q < ws.hot_cap) {  // bound holds unless inserts skip an update
      ws.hot[q] = (int32_t)h;
      ws.hkey[q] = p.key;
    }
  }
}

// lookup i of the step has key `key` (DD_EMPTY: the lookup contributes nothing)
__device__ __forceinline__ void dd_insert(const DedupWs& ws, uint64_t key, int32_t i) {
  DdPend p;
  dd_insert_begin(ws, key, i, p);
  dd_insert_finish(ws, p, i);
}

// Deferred finish, for a whole wave (group `group` of <= 64 lookups, lane l holding entry l): a
// lookup whose first CAS claimed a free slot files itself (position 0: no further round trip);
// every other one (home slot held by its key or by another key) leaves its key in the group's
// overflow entry for dd_resolve_block, which runs in a later launch. Every lane writes its entry
// (EMPTY when there is nothing to resolve): no counts, no compaction. The wave's tail is then ONE
// atomic round trip, not a probe chain (the slowest of 64 lanes decides when a wave ends).
__device__ __forceinline__ void dd_insert_defer_finish_at(const DedupWs& ws, const DdPend& p, int32_t i, int group,
                                                          int entry);
__device__ __forceinline__ void dd_insert_defer_finish(const DedupWs& ws, const DdPend& p, int32_t i, int group) {
  dd_insert_defer_finish_at(ws, p, i, group, threadIdx.x & 63);
}
// the same with the entry (< 64) of the group given explicitly (the row-owned T1: 16 lookups per wave)
__device__ __forceinline__ void dd_insert_defer_finish_at(const DedupWs& ws, const DdPend& p, int32_t i, int group,
                                                          int entry) {
  const int lane = entry;
  const bool live = p.key != DD_EMPTY;
  const bool claimed = live && p.prev == DD_EMPTY;
  if (claimed) ws.slots[p.h].item[0] = i;
  if (live) ws.claim[i] = claimed ? (int32_t)p.h : -1;  // deferred: the resolver rewrites it
  DedupWs::Ovf o;
  o.key = live && !claimed ? p.key : DD_EMPTY;
  o.i = i;
  o.pad = 0;
  ws.ovf[(int64_t)group * 64 + lane] = o;
}

// finishes the deferred inserts of groups [rb * gpw, (rb + 1) * gpw), gpw = ceil(groups / nres):
// one thread per overflow entry; the entry is cleared for the next step
__device__ __forceinline__ void dd_resolve_block(const DedupWs& ws, int rb, int nres) {
  const int G = ws.ovf_groups;
  const int gpw = (G + nres - 1) / nres;
  for (int e = threadIdx.x; e < gpw * 64; e += blockDim.x) {
    const int64_t g = (int64_t)rb * gpw + e / 64;
    if (g >= G) break;
    DedupWs::Ovf* op = ws.ovf + g * 64 + e % 64;
    const DedupWs::Ovf o = *op;
    if (o.key != DD_EMPTY) {
      op->key = DD_EMPTY;
      dd_insert(ws, o.key, o.i);
    }
  }
}

size_t dedup_layout(void* base, int64_t L, DedupWs* w);

// arguments of the update launch (dd_adagrad_kernel, or a role of a combined launch)
struct DdUpdateArgs {
  EmbMeta m;           // tables; features map lookup i = f * B + b to its gradient row
  const float* grad;   // pooled gradient, row (features[f].out_row + b), cols features[f].out_offset..
  int64_t ldg;
  int64_t n;           // lookups inserted this step (F * B)
  float* weights;
  float* state;
  float lr, eps;
  DedupWs ws;
  int hot_wgs;         // workgroups of the hot role; the slot role has slot_hw / 8 more
  int64_t slot_hw;     // half-waves of the slot role: ceil(L / DD_SPH), a multiple of 8
  int skip_single;     // rows looked up once were updated by T1 (dd_mode 2): only free their slots
  int xcd;             // 1: the slot role's workgroups start at a multiple of 8 in their launch: they
                       // take the claiming lookups a contiguous 1/8 per XCD (xcd_remap)
  int multi_nseg;      // > 0: the slot role walks the T1 list of multi-lookup rows (DedupWs::multi, this
                       // many segments) instead of every claiming lookup; T1 freed the single slots
#if TT_EXPERIMENTS
  int exp_skip;        // EXPERIMENT (TT_EXP_SKIP, timing only, wrong results): 1 hot role, 2 slot role
#endif
};

// Per-lane table / feature meta from LDS: indexing the kernel-argument arrays by a per-lane value
// compiles to a vector load from the kernarg segment — one more dependent memory hop (and an
// in-order vmcnt wait) in front of every row access. The update workgroup copies the meta of its
// T tables and F features into LDS once (overlapping its first slot load) and reads it per lane.
struct DdMeta {
  int64_t woff[TT_MAX_TABLES];
  int64_t soff[TT_MAX_TABLES];
  int64_t frow[TT_MAX_FEATURES];
  int64_t foff[TT_MAX_FEATURES];
  int32_t dim[TT_MAX_TABLES];
};

__device__ __forceinline__ void dd_meta_fill(const EmbMeta& m, DdMeta* lm) {
  for (int u = threadIdx.x; u < m.T; u += blockDim.x) {
    lm->woff[u] = m.tables[u].weight_offset;
    lm->soff[u] = m.tables[u].state_offset;
    lm->dim[u] = m.tables[u].dim;
  }
  for (int u = threadIdx.x; u < m.F; u += blockDim.x) {
    lm->frow[u] = m.features[u].out_row;
    lm->foff[u] = m.features[u].out_offset;
  }
}

// lookup i = f * B + b -> its gradient row (features[f].out_row + b), column features[f].out_offset
struct GradMap {
  const float* g;
  int64_t ldg;
  uint32_t B;  // lookups < 2^18 (DD_CNT_BITS): 32-bit division
  const DdMeta* lm;
  __device__ __forceinline__ const float* row(int i) const {
    const uint32_t f = (uint32_t)i / B;
    return g + (lm->frow[f] + (int64_t)((uint32_t)i - f * B)) * ldg + lm->foff[f];
  }
};

template <int W>
__device__ __forceinline__ int dd_bitonic(int v) {
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

constexpr int DD_HOT_PT = 16;                // lookups per thread per scan pass (4096 a pass)
constexpr int DD_HOT_CH = 256 * DD_HOT_PT;  // lookups scanned per pass of a hot workgroup (LDS list)
constexpr int DD_HOT_TEAM = 8;              // at most this many workgroups share one hot row
#ifndef DD_HOT_STAMPS
// EXPERIMENT (scripts/hot_stamps.py): TT_EXTRA_CFLAGS=-DDD_HOT_STAMPS=1 python -m
// two_tower_recommender_model_amd.build --experiments, run with TT_EXPERIMENT_LIB=1
#define DD_HOT_STAMPS 0
#endif
#if DD_HOT_STAMPS && !TT_EXPERIMENTS
#error "DD_HOT_STAMPS needs the experiment build (DD_STAMP records nothing without TT_EXPERIMENTS): build --experiments"
#endif
// LDS of the hot role (list + per (pass slice, wave) match counts and their prefix + group
// partials), provided by the launching kernel so a combined launch can overlay it on its other
// roles' LDS
constexpr int DD_SMEM_HOT = DD_HOT_CH * 4 + 2 * DD_HOT_PT * 4 * 4 + 16 + 8 * 32 * 16;
constexpr int DD_SMEM = DD_SMEM_HOT + (int)sizeof(DdMeta);  // + the per-workgroup meta copy

// members per hot row: as many as the hot workgroups allow in one round (at least 1), at most one
// per scan pass and DD_HOT_TEAM (every workgroup computes it from the same nh)
__device__ __forceinline__ int dd_hot_team(int nh, int64_t n, int hot_wgs) {
  const int npass = (int)((n + DD_HOT_CH - 1) / DD_HOT_CH);
  return max(1, min(min(DD_HOT_TEAM, npass), hot_wgs / max(1, nh)));
}

// every hot workgroup checks in once; the last one resets the hot-row count and the ticket
__device__ __forceinline__ void dd_hot_ticket(const DedupWs& ws, int hot_wgs) {
  if (threadIdx.x == 0) {
    const int tk = atomicAdd(&ws.ctr[1], 1);
    if (tk == hot_wgs - 1) {
      atomicExch(&ws.ctr[0], 0);
      atomicExch(&ws.ctr[1], 0);
    }
  }
}

// Rows looked up more than DD_INL times in the step. A row is split over a team of K workgroups
// (dd_hot_team): member k scans passes k, k + K, ... of the step's keys (4096
// a pass, the next pass's keys in flight beside this pass's matching), its 8 groups add the pass's
// matches at positions == group (mod 8) in ascending order (8 rows in flight), and the group sums
// are added in group order: the member's partial. Members publish their partial write-through
// (relaxed agent-scope stores: sc1) and add to the row's counter; the member whose add returns
// K - 1 reads the K partials (sc1 loads, after its add returned) and adds them in member order —
// the same sum whichever member arrives last — then applies the row-wise Adagrad step. No member
// waits on another (cdna_hip_programming.md Guideline 16: counter form, the last arriver combines).
// nh: the step's hot rows; ticket: check in at the end (the last resets the count)
__device__ __forceinline__ void dd_hot_role(const GradMap& gm, int64_t n,
                                            float* __restrict__ weights, float* __restrict__ state, float lr,
                                            float eps, const DedupWs& ws, int hot_wgs, int bid, char* smem, int nh,
                                            bool ticket, int32_t hc, uint64_t hk,
                                            const uint64_t (&kspec)[DD_HOT_PT], int ks) {
  f32x4v (*part)[32] = reinterpret_cast<f32x4v (*)[32]>(smem);       // [8][32], 16-B aligned
  int* list = reinterpret_cast<int*>(smem + 8 * 32 * 16);             // [DD_HOT_CH]
  int* qc = reinterpret_cast<int*>(smem + 8 * 32 * 16 + DD_HOT_CH * 4);  // [PT][4] matches per (q, wave)
  int* qoff = qc + DD_HOT_PT * 4;                                          // [PT][4] their prefix, + total
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = tid >> 5, hl = tid & 31;
  const int nn = (int)n;  // lookups < 2^18 (DD_CNT_BITS): 32-bit indices
  const int npass = (nn + DD_HOT_CH - 1) / DD_HOT_CH;
  const int K = dd_hot_team(nh, n, hot_wgs);
  for (int w = bid; w < nh * K; w += hot_wgs) {
    const int j = w / K, k = w - j * K;
    // hc / hk: lane l holds hot[bid / (l + 1)] and its key, loaded beside the count (the first item
    // for team size K): the key scan starts one round trip after the launch, not two
    const int32_t h = w == bid ? __shfl(hc, K - 1, 64) : ws.hot[j];
    const uint64_t key = w == bid ? (uint64_t)__shfl((long long)hk, K - 1, 64) : ws.hkey[j];
    const int t = (int)(key >> DD_TABLE_SHIFT);
    const int64_t r = (int64_t)(key & ((1ull << DD_TABLE_SHIFT) - 1));
    const int D = gm.lm->dim[t];
    const bool col_ok = hl * 4 < D;
    // the row and its state, loaded now for whichever member applies the update (nothing else in
    // the launch writes a hot row): off the chain's end
    float* wrow = weights + gm.lm->woff[t] + r * D;
    float* srow = state + gm.lm->soff[t] + r;
    const f32x4v wpre = col_ok && wid == 0 && lane < 32 ? *reinterpret_cast<const f32x4v*>(wrow + hl * 4) : (f32x4v)(0.f);
    const float spre = wid == 0 ? *srow : 0.f;
    f32x4v acc = (f32x4v)(0.f);
    uint64_t kc[DD_HOT_PT], kn[DD_HOT_PT];
    // thread tid holds lookups pass * CH + 256 q + tid (q < PT): every key load instruction reads
    // 512 contiguous bytes (16 consecutive keys per thread made each instruction touch 64 lines).
    // The first pass of the first item comes from kspec when the speculation held (pass ks)
    if (w == bid && k == ks) {
#pragma unroll
      for (int q = 0; q < DD_HOT_PT; ++q) kc[q] = kspec[q];
    } else {
#pragma unroll
      for (int q = 0; q < DD_HOT_PT; ++q) {
        const int i = k * DD_HOT_CH + 256 * q + tid;
        kc[q] = i < nn ? ws.lkey[i] : DD_EMPTY;
      }
    }
    const uint64_t lt = (1ull << lane) - 1;
    for (int p = k; p < npass; p += K) {
      const int pb = p * DD_HOT_CH;
#pragma unroll
      for (int q = 0; q < DD_HOT_PT; ++q) {
        const int i = pb + K * DD_HOT_CH + 256 * q + tid;
        kn[q] = i < nn ? ws.lkey[i] : DD_EMPTY;
      }
      // matches per (q, wave) by ballot; their exclusive prefix in (q, wave) order is the
      // ascending lookup order (lookup pb + 256 q + 64 wave + lane): the list is the same as before
      uint64_t bq[DD_HOT_PT];
#pragma unroll
      for (int q = 0; q < DD_HOT_PT; ++q) {
        bq[q] = __ballot(kc[q] == key);
        if (lane == 0) qc[q * 4 + wid] = __popcll(bq[q]);
      }
      __syncthreads();
      if (wid == 0) {  // 64 counts, one per lane: inclusive scan
        const int v = qc[lane];
        int inc = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(inc, o, 64);
          if (lane >= o) inc += y;
        }
        qoff[lane] = inc - v;
        if (lane == 63) qoff[DD_HOT_PT * 4] = inc;
      }
      __syncthreads();
#if DD_HOT_STAMPS
      if (p == k) DD_STAMP(4);  // first pass: keys matched, scanned
#endif
      const int total = qoff[DD_HOT_PT * 4];
#pragma unroll
      for (int q = 0; q < DD_HOT_PT; ++q)
        if ((bq[q] >> lane) & 1) list[qoff[q * 4 + wid] + __popcll(bq[q] & lt)] = pb + 256 * q + tid;
      __syncthreads();
      // 8 matched rows in flight per group, the pass's last partial round included (a one-row-per-
      // iteration remainder was up to 7 dependent round trips per pass); added in position order
      for (int pp = grp; pp < total; pp += 64) {
        f32x4v x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const bool on = col_ok && pp + 8 * u < total;
          x[u] = on ? *reinterpret_cast<const f32x4v*>(gm.row(list[pp + 8 * u]) + hl * 4) : (f32x4v)(0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (pp + 8 * u < total) acc += x[u];
      }
      __syncthreads();  // the list and the counts are rewritten by the next pass
#pragma unroll
      for (int q = 0; q < DD_HOT_PT; ++q) kc[q] = kn[q];
    }
    part[grp][hl] = acc;
    __syncthreads();
#if DD_HOT_STAMPS
    DD_STAMP(5);  // the member's passes summed
#endif
    if (wid == 0) {
      f32x4v g = part[0][hl];
#pragma unroll
      for (int q = 1; q < 8; ++q) g += part[q][hl];
      bool last = true;
      if (K > 1) {
        float* mine = ws.hotp + ((int64_t)j * DD_HOT_TEAM + k) * 128 + hl * 4;
        if (lane < 32) {
#pragma unroll
          for (int v = 0; v < 4; ++v) __hip_atomic_store(mine + v, g[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial has left this CU
        int prev = 0;
        if (lane == 0) prev = __hip_atomic_fetch_add(&ws.hcnt[j], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        prev = __shfl(prev, 0, 64);
        last = prev == K - 1;
#if DD_HOT_STAMPS
        DD_STAMP(6);  // partial published, counter added
#endif
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the add
          const float* all = ws.hotp + (int64_t)j * DD_HOT_TEAM * 128 + hl * 4;
          f32x4v pk[DD_HOT_TEAM];
#pragma unroll
          for (int q = 0; q < DD_HOT_TEAM; ++q)
#pragma unroll
            for (int v = 0; v < 4; ++v)
              pk[q][v] = q < K ? __hip_atomic_load(all + q * 128 + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
          g = pk[0];
#pragma unroll
          for (int q = 1; q < DD_HOT_TEAM; ++q)
            if (q < K) g += pk[q];
          if (lane == 0) __hip_atomic_store(&ws.hcnt[j], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (last) {
        float sq = col_ok ? rw_sq4(g) : 0.f;
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
        if (lane < 32) {
          const float snew = rw_state(spre, sq, D);
          const float step = rw_step(snew, lr, eps);
          if (col_ok) *reinterpret_cast<f32x4v*>(wrow + hl * 4) = rw_apply(wpre, g, step);
          __builtin_amdgcn_wave_barrier();
          if (lane == 0) {
            *srow = snew;
            ws.slots[h].word = DD_EMPTY;
          }
#if DD_HOT_STAMPS
          DD_STAMP(7);  // row update issued
#endif
        }
      }
    }
    __syncthreads();
  }
  if (ticket) dd_hot_ticket(ws, hot_wgs);
}

// host: validate + fill the update launch's arguments; *grid = its workgroup count
int dedup_update_args(const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F, int64_t B,
                      const float* grad, int64_t ldg, float* weights, float* state, float lr, float eps,
                      void* workspace, size_t ws_bytes, int64_t max_lookups, DdUpdateArgs& a, int64_t* grid);

// the slot part of the update: DD_SPH slots per half-wave (sp, their first 128 B in dw, hq >= 0
// for a slot to take), gradient rows summed in ascending lookup order, row-wise Adagrad, the slot
// freed. spec: the claimer's key is lk[q] (its row, state and own gradient row loaded beside the slot)
__device__ __forceinline__ void dd_slots_finish(const DdUpdateArgs& a, const GradMap& gm, const DdMeta* lm, bool spec,
                                                const int (&hq)[DD_SPH], const uint64_t (&lk)[DD_SPH],
                                                DSlot* const (&sp)[DD_SPH], const int (&dw)[DD_SPH], int64_t hw,
                                                int64_t nhw, int bid) {
  const DedupWs& ws = a.ws;
  (void)ws;
  (void)bid;
  float* __restrict__ weights = a.weights;
  float* __restrict__ state = a.state;
  const float lr = a.lr, eps = a.eps;
  const int lane = threadIdx.x & 63;
  const int hl = lane & 31, hb = lane & 32;
  bool active[DD_SPH], col_ok[DD_SPH];
  int c[DD_SPH], cmax[DD_SPH], mine[DD_SPH], D[DD_SPH];
  float* wrow[DD_SPH];
  float* srow[DD_SPH];
  f32x4v wv[DD_SPH], g[DD_SPH], gown[DD_SPH];
  float s_old[DD_SPH];
  if (spec) {
#pragma unroll
    for (int q = 0; q < DD_SPH; ++q) {
      const bool cl = hq[q] >= 0;
      const int t = cl ? (int)(lk[q] >> DD_TABLE_SHIFT) : 0;
      const int64_t r = cl ? (int64_t)(lk[q] & ((1ull << DD_TABLE_SHIFT) - 1)) : 0;
      D[q] = lm->dim[t];
      col_ok[q] = cl && hl * 4 < D[q];
      wrow[q] = weights + lm->woff[t] + r * D[q];
      srow[q] = state + lm->soff[t] + r;
      wv[q] = col_ok[q] ? *reinterpret_cast<const f32x4v*>(wrow[q] + hl * 4) : (f32x4v)(0.f);
      s_old[q] = cl ? *srow[q] : 0.f;
      const int64_t i = hw + q * nhw;
      gown[q] = col_ok[q] ? *reinterpret_cast<const f32x4v*>(gm.row((int)i) + hl * 4) : (f32x4v)(0.f);
    }
  }
#pragma unroll
  for (int q = 0; q < DD_SPH; ++q) {
    const uint64_t word = ((uint64_t)(uint32_t)__shfl(dw[q], hb + 1, 64) << 32) | (uint32_t)__shfl(dw[q], hb, 64);
    const uint64_t key = word >> DD_CNT_BITS;
    const int cnt = (int)(word & DD_CNT_MASK);
    const int item = __shfl(dw[q], hb + 2 + (hl < DD_INL ? hl : 0), 64);
    // hot slots (reset by the hot role, one 8-B store) are never taken here
    active[q] = word != DD_EMPTY && cnt <= DD_INL;
    // skip_single: a row looked up once was updated in place by T1; its slot is only freed here
    const bool upd = active[q] && !(a.skip_single && cnt == 1);
    if (!spec) {
      const int t = upd ? (int)(key >> DD_TABLE_SHIFT) : 0;
      const int64_t r = upd ? (int64_t)(key & ((1ull << DD_TABLE_SHIFT) - 1)) : 0;
      D[q] = lm->dim[t];
      col_ok[q] = upd && hl * 4 < D[q];
      wrow[q] = weights + lm->woff[t] + r * D[q];
      srow[q] = state + lm->soff[t] + r;
      wv[q] = col_ok[q] ? *reinterpret_cast<const f32x4v*>(wrow[q] + hl * 4) : (f32x4v)(0.f);
      s_old[q] = upd ? *srow[q] : 0.f;
    } else {
      col_ok[q] = col_ok[q] && upd;  // the claimer's key is the slot's: the loads above are its row's
    }
    c[q] = upd ? cnt : 0;
    cmax[q] = max(c[q], __shfl_xor(c[q], 32, 64));
    mine[q] = hl < c[q] ? item : 0x7fffffff;
    g[q] = (f32x4v)(0.f);
  }
  bool single = true;  // wave-uniform: every slot of the wave has at most one lookup
#pragma unroll
  for (int q = 0; q < DD_SPH; ++q) single = single && cmax[q] <= 1;
  if (single) {
    // the common case (uniform ids): one gradient row per slot, all loads in flight together (spec:
    // the claimer's own row, already loaded — the slot's one lookup IS the claimer)
#pragma unroll
    for (int q = 0; q < DD_SPH; ++q) {
      const int b0 = __shfl(mine[q], hb, 64);  // the slot's one lookup, held by lane 0 of the half
      if (col_ok[q] && c[q] == 1) g[q] += spec ? gown[q] : *reinterpret_cast<const f32x4v*>(gm.row(b0) + hl * 4);
    }
  } else {
#pragma unroll
    for (int q = 0; q < DD_SPH; ++q) {
      if (cmax[q] > 1) mine[q] = dd_bitonic<32>(mine[q]);
      // DD_MR gradient rows in flight, added in ascending order (12 measured: Zipf -0.8 / +0.5 µs
      // in two A/Bs, uniform +0.3 — code-layout noise, not a gain; scripts/r04_mr.sh)
      for (int i = 0; i < cmax[q]; i += DD_MR) {
        f32x4v x[DD_MR];
#pragma unroll
        for (int u = 0; u < DD_MR; ++u) {
          const int b = __shfl(mine[q], hb + min(i + u, 31), 64);
          x[u] = col_ok[q] && i + u < c[q] ? *reinterpret_cast<const f32x4v*>(gm.row(b) + hl * 4) : (f32x4v)(0.f);
        }
#pragma unroll
        for (int u = 0; u < DD_MR; ++u)
          if (i + u < c[q]) g[q] += x[u];
      }
    }
  }
  DD_STAMP(2);
#pragma unroll
  for (int q = 0; q < DD_SPH; ++q) {
    float sq = rw_sq4(g[q]);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
    if (c[q] > 0) {
      const float snew = rw_state(s_old[q], sq, D[q]);
      const float step = rw_step(snew, lr, eps);
      if (col_ok[q]) *reinterpret_cast<f32x4v*>(wrow[q] + hl * 4) = rw_apply(wv[q], g[q], step);
      if (hl == 0) *srow[q] = snew;
    }
    if (active[q] && hl == 0) sp[q]->word = DD_EMPTY;
  }
  DD_STAMP(3);
}

// the list role (DdUpdateArgs::multi_nseg): every workgroup reads the head of every T1 segment
// (thread t owns segments t, t + 256, ...: one 16-B load = the segment's count and its first three
// slots), takes the equal share [lb per, (lb + 1) per) of the listed slots in that order (per <= 256:
// the host sizes nlb >= lookups / 512), files their slot indices into LDS (an entry past a head's
// three is loaded then: rare, a segment is one T1 wave of 16 lookups) and updates those slots,
// DD_SPH per half-wave per round. Counts and first entries in one round trip: the slot words follow
// at the second, not the third. Each slot's update is the same whichever half-wave takes it.
__device__ __forceinline__ void dd_multi_block(const DdUpdateArgs& a, const GradMap& gm, DdMeta* lm, int lb, int nlb,
                                               char* smem, int bid) {
  const DedupWs& ws = a.ws;
  int* lst = reinterpret_cast<int*>(smem);  // [256]
  int* wsum = lst + 256;                    // [4] wave totals
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nseg = a.multi_nseg;
  constexpr int SPT = 8;  // segments per thread (nseg <= 2048)
  int4 hd[SPT];
#pragma unroll
  for (int k = 0; k < SPT; ++k)
    hd[k] = tid + 256 * k < nseg ? *reinterpret_cast<const int4*>(ws.multi + (int64_t)(tid + 256 * k) * DD_SEGW)
                                 : make_int4(0, -1, -1, -1);
  dd_meta_fill(a.m, lm);
  int mine = 0;
#pragma unroll
  for (int k = 0; k < SPT; ++k) mine += hd[k].x;
  int inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  int base = inc - mine, total = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    base += w < wid ? wsum[w] : 0;
    total += wsum[w];
  }
  const int per = (total + nlb - 1) / nlb;
  const int r0 = lb * per, r1 = min(total, r0 + per);
  int p = base;
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int seg = tid + 256 * k;
    for (int e = 0; e < hd[k].x; ++e, ++p)
      if (p >= r0 && p < r1)
        lst[p - r0] = e == 0 ? hd[k].y : e == 1 ? hd[k].z : e == 2 ? hd[k].w : ws.multi[(int64_t)seg * DD_SEGW + 1 + e];
  }
  const int len = max(0, r1 - r0);
  __syncthreads();
  const int hl = lane & 31;
  const int hw = wid * 2 + ((lane & 32) >> 5);  // half-wave of the workgroup (8)
  for (int j0 = 0; j0 < len; j0 += 8 * DD_SPH) {
    int hq[DD_SPH];
    uint64_t lk[DD_SPH];
    DSlot* sp[DD_SPH];
    int dw[DD_SPH];
#pragma unroll
    for (int q = 0; q < DD_SPH; ++q) {
      const int j = j0 + hw + 8 * q;
      hq[q] = j < len ? lst[j] : -1;
      lk[q] = DD_EMPTY;
      sp[q] = ws.slots + (hq[q] >= 0 ? hq[q] : 0);
      dw[q] = hq[q] >= 0 ? reinterpret_cast<const int32_t*>(sp[q])[hl] : (hl < 2 ? -1 : 0);
    }
    dd_slots_finish(a, gm, lm, false, hq, lk, sp, dw, 0, 0, bid);
  }
}

// One workgroup (256 threads) of the update launch: bid < hot_wgs -> hot role, else 8 slots.
// smem: DD_SMEM bytes of 16-B aligned LDS.
template <bool LIST_ONLY = false>
__device__ __forceinline__ void dd_update_block(const DdUpdateArgs& a, int bid, char* smem) {
  const EmbMeta& m = a.m;
  const DedupWs& ws = a.ws;
  float* __restrict__ weights = a.weights;
  float* __restrict__ state = a.state;
  const float lr = a.lr, eps = a.eps;
  DD_STAMP(0);
  DdMeta* lm = reinterpret_cast<DdMeta*>(smem + DD_SMEM_HOT);
  const GradMap gm{a.grad, a.ldg, (uint32_t)m.B, lm};
#if TT_EXPERIMENTS
  if ((a.exp_skip & 1) && bid < a.hot_wgs) return;
  if ((a.exp_skip & 2) && bid >= a.hot_wgs) return;
#endif
  if (bid < a.hot_wgs) {
    // speculative: the keys of the first pass a member of a two-workgroup team scans (teams of two
    // are the skewed steps' usual case: 17..32 hot rows over 64 hot workgroups), issued beside the
    // count instead of a round trip after it; any other team size loads its own
    const int ks = bid & 1;
    uint64_t kspec[DD_HOT_PT];
#pragma unroll
    for (int q = 0; q < DD_HOT_PT; ++q) {
      const int64_t i = (int64_t)ks * DD_HOT_CH + 256 * q + threadIdx.x;
      kspec[q] = i < a.n ? ws.lkey[i] : DD_EMPTY;
    }
    // a workgroup with no hot work item (most of them at uniform ids) only checks in: the ticket
    // that resets the hot-row count once every hot workgroup has read it. skip_single: the row-owned
    // T1 moved the count to ctr[2] and zeroed ctr[0] (no ticket: 64 returning atomics on one word
    // serialise, the last check-in ended the ring's tail ~3 us after its other roles)
    const bool ticket = !a.skip_single;
    // beside the count: the hot-list entry this workgroup takes first for each team size it can get
    // (lane l: team size l + 1), so the slot word is the next hop, not the list entry
    const int hi = min(bid / (min((int)(threadIdx.x & 63), DD_HOT_TEAM - 1) + 1), ws.hot_cap - 1);
    const int32_t hc = ws.hot[hi];
    const uint64_t hk = ws.hkey[hi];
    const int nh = min(ticket ? __hip_atomic_load(&ws.ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ws.ctr[2],
                       ws.hot_cap);
    if (bid >= nh * dd_hot_team(nh, a.n, a.hot_wgs)) {
      if (ticket) dd_hot_ticket(ws, a.hot_wgs);
      return;
    }
    dd_meta_fill(m, lm);
    __syncthreads();
    dd_hot_role(gm, a.n, weights, state, lr, eps, ws, a.hot_wgs, bid, smem, nh, ticket, hc, hk, kspec, ks);
    return;
  }
  if (LIST_ONLY || a.multi_nseg > 0) {
    dd_multi_block(a, gm, lm, bid - a.hot_wgs, (int)(a.slot_hw / 8), smem, bid);
    return;
  }
  const int lane = threadIdx.x & 63;
  const int hl = lane & 31, hb = lane & 32;
  // DD_SPH claiming lookups per half-wave (i and i + nhw, ...), their dependent loads interleaved:
  // the slot a lookup claimed (claim[i] >= 0) is updated by that lookup's half-wave; the grid covers
  // the step's lookups (not the cap slots) in one round of resident waves
  int sb = bid - a.hot_wgs;
  if (a.xcd) {  // (a uniform remap of the slot workgroups: which workgroup takes a lookup is free)
    const int ns = (int)(a.slot_hw / 8), x = sb & 7, loc = sb >> 3, q = ns >> 3, r = ns & 7;
    sb = x * q + min(x, r) + loc;
  }
  const int64_t hw = ((int64_t)sb * 4 + (threadIdx.x >> 6)) * 2 + (hb >> 5);
  const int64_t nhw = a.slot_hw;
  int hq[DD_SPH];
  uint64_t lk[DD_SPH];
  // spec (every mode but skip_single): the claiming lookup's own key is its slot's key, so its row,
  // row state and own gradient row are loaded beside the slot (from lkey[i]) instead of after it —
  // the update of a row looked up once (the common case) waits two dependent round trips, not three
  const bool spec = !a.skip_single;
#pragma unroll
  for (int q = 0; q < DD_SPH; ++q) {
    const int64_t i = hw + q * nhw;
    hq[q] = i < a.n ? ws.claim[i] : -1;
    lk[q] = spec && i < a.n ? ws.lkey[i] : DD_EMPTY;
  }
  DSlot* sp[DD_SPH];
  int dw[DD_SPH];
#pragma unroll
  for (int q = 0; q < DD_SPH; ++q) {
    sp[q] = ws.slots + (hq[q] >= 0 ? hq[q] : 0);
    // an idle half-wave reads nothing and sees an EMPTY word
    dw[q] = hq[q] >= 0 ? reinterpret_cast<const int32_t*>(sp[q])[hl] : (hl < 2 ? -1 : 0);  // 32 lanes: 128 B
  }
  dd_meta_fill(m, lm);  // beside the slot loads
  __syncthreads();
  DD_STAMP(1);
  dd_slots_finish(a, gm, lm, spec, hq, lk, sp, dw, hw, nhw, bid);
}



}  // namespace tt

// Fused two-tower MLP step on gfx950 bf16 MFMA (v_mfma_f32_16x16x32_bf16, fp32 accumulate).
//
// Replaces ~9 per-layer launches of the towers (torchrec MLP = Linear + ReLU on every layer,
// 03_model_training.py:411-412), the dot + BCE head (:452-453) and Adam (:826-829) with three:
//
//  T1 tower_fwd_bwd   one 256-thread workgroup per 32 rows: both towers' forward through all layers
//                     (activations stay in LDS), logits + BCE + dlogit, the backward through all
//                     layers down to dX, written straight into the pooled-embedding gradient
//                     [B, sum D] that the fused row-wise Adagrad consumes. It also stores, for T2,
//                     the layer inputs and the dZ of every layer TRANSPOSED ([feature][row], bf16),
//                     and per-workgroup bias-gradient partials (fp32).
//  T2 tower_wgrad     dW = dZ^T A over all rows: one wave per (32x32 tile, row slice), fragments
//                     loaded straight from the transposed bf16 buffers (16 B per lane, no LDS),
//                     partial tiles into fp32 slabs.
//  T3 tower_update    per parameter: fixed-order sum of the slabs / bias partials, Adam
//                     (torch.optim.Adam formula), and the bf16 weight copies T1 reads next step
//                     (W [out][in] for the forward, W^T [in][out] for the backward).
// Every reduction is in a fixed order: bitwise reproducible, independent of XCD placement.
//
// MFMA 16x16x32 operand maps (lane l, element j < 8): A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15];
// result C[4(l>>4)+r][l&15], r < 4.
#include <vector>

#include "tt_common.h"
#include "dedup.h"
#include "shard.h"

namespace tt {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;

constexpr int TR = 32;                // rows per workgroup
constexpr int MAXW = 128;             // max layer width
constexpr int XCH = 128;              // input columns per chunk
constexpr int LSTR = MAXW + 8;        // bf16 LDS row stride (272 B: conflict-light ds_read_b128)
constexpr int FSTR = MAXW + 4;        // fp32 LDS row stride
constexpr int MAXL = 4;

// T1 -> T2 operand strips (X^T, activations, dZ^T; bf16), tile-major: element (feature f, batch
// row m) of a strip block with nf features sits at ((m / 32) * nf + f) * 32 + m % 32, blocks of
// nf x Bp elements (Bp = B rounded up to 32). One T1 workgroup's 32-row tile of a block is one
// contiguous run (whole cache lines written once), and a T2 chunk of 32 rows x 16 features is 1 KB
// contiguous (a full-rate load per wave instruction) instead of 16 scattered 64-B pieces.
__device__ __forceinline__ int64_t strip_at(int64_t f, int64_t m, int64_t nf) {
  return (((m >> 5) * nf + f) << 5) + (m & 31);
}

struct TowerArgs {
  tt_tower_shape_t s;
  int64_t B;
  const float* pooled;  // [B, ldp]
  int64_t ldp;
  float* gpooled;       // [B, ldp] (tower-input columns written)
  const float* params;  // flat fp32 (bias read from here)
  const __bf16* wb;     // bf16 W  [out][in] per (t,l), flat like params' W blocks
  const __bf16* wtb;    // bf16 W^T [in][out]
  const __bf16* wbf;    // the same two copies in MFMA B-fragment order (frag_off): every fragment
  const __bf16* wtbf;   //   load of a wave is 1 KB contiguous (full 128-B lines, one request each)
  int64_t woff[2][MAXL];  // element offset of W_(t,l) in params
  int64_t boff[2][MAXL];  // element offset of b_(t,l) in params
  int64_t wcoff[2][MAXL]; // element offset of W_(t,l) in the bf16 copies
  const void* labels;
  int label_dtype;
  float grad_scale;
  float* logits;
  // T1 -> T2 buffers
  __bf16* xt;           // [2] blocks of in_max x Bp (strip_at)
  __bf16* act;          // [2][MAXL][MAXW][B]  (layer-l OUTPUT, transposed; layers 0..L-2 used)
  __bf16* dzt;          // [2][MAXL][MAXW][B]
  float* dbpart;        // [2][MAXL][nwg][MAXW]
  float* loss_part;     // [nwg]
  int64_t in_max;
  int64_t Bp;           // strip rows per block (B rounded up to 32)
  int nwg;
  // fused single-hot gather (tt_tower_fwd_bwd_gather): tower t's input row m is table row
  // (gcol[t][m] mod gmod[t]) of gtab[t] (zeros for id 0) instead of pooled row m
  const void* gcol[2];
  const float* gtab[2];
  int64_t gmod[2];
  int gid_dtype;
  float* pooled_out;    // nullable: the gathered rows are also written here (ld = ldp)
  // dedup insert of the gathered lookups (lookup i = t * B + m, key = dd_table[t] << 40 | row)
  DedupWs dd;
  int dd_on;
  int dd_table[2];
  // indexed gather (sharded step, tt_tower_fwd_bwd_indexed): tower t's input row m is row
  // gpos[t][m] of gsrc[t] ([*][in_dim[t]] fp32; -1 -> zeros) and its dX row goes to row gpos[t][m]
  // of gdst[t] instead of gpooled
  const int32_t* gpos[2];
  const float* gsrc[2];  // fp32 rows, or bf16 rows when gsrc_bf16 (the same bf16 values T1 computes on)
  float* gdst[2];
  const int32_t* gpos_out[2];  // nullable: dX row index in gdst (units of in_dim floats) when it differs
                               // from the input row (the pipelined sharded step's packed send buffer)
  int gsrc_bf16;
  // in-place row-wise Adagrad of the rows looked up ONCE in the step (the pipelined fused step,
  // tower_l2_kernel<..., UPD = true>): `dd` is this batch's dedup table, completed before T1 (by the
  // previous step's T2 / K3); a kept lookup whose slot count is 1 updates its row and state here from
  // its dX (the same arithmetic as the K3 update: rw_* helpers); the others leave dX for K3
  float* uw[2];  // tower t's table rows (writable; == gtab[t])
  float* us[2];  // tower t's table row-wise state
  float ulr, ueps;
  // UPD, nullable: the NEXT batch's id columns; the dedup wave touches every 64-B segment of this
  // tile's next rows and their state (a prefetch into the memory-side cache and this XCD's TLB;
  // the values are discarded)
  const void* pcol[2];
  // multi-hot EBC forward fused in (tt_tower_fwd_bwd_kjt, tower_l2_kernel<..., MH = true>): tower
  // t's input row m is the SUM of rows values[moff[t][m] .. moff[t][m + 1]) of gtab[t] (gmod[t]
  // rows: an id >= gmod[t] reads row 0, never out of bounds)
  const void* mval;
  const int32_t* moff[2];
  // multi-feature indexed rows (sharded step with several single-hot features per tower,
  // tt_tower_fwd_bwd_indexed_multi_bf16; the general kernel): input column k of tower t is column
  // k % iD of bf16 row ipos[(ifeat0[t] + k / iD) * B + m] of isrc (-1 -> zeros), and dX column k
  // goes to column k % iD of row ipos_out[same] of idst (-1: not written)
  const int32_t* ipos;
  const int32_t* ipos_out;
  const __bf16* isrc;
  float* idst;
  int ifeat0[2];
  int iD;
  // the row-owned T1 (tower_rows_kernel): both towers' bf16 weight image, the LDS layout (rk_off)
  const char* wimg;
  // indexed2 with a direct exchange (W > 0): dX rows go to the destinations' mapped receive buffers
  // (px_row) and the copy fields' bytes travel beside them (px_copy_*); W = 0: gdst as above
  tt_peer_direct_t xd;
#if TT_EXPERIMENTS
  int dbg;  // EXPERIMENT: 1 skip T2 operand stores, 2 skip dX stores, 4 gather row 0 only, 8 stamps
  int64_t* stamps;  // EXPERIMENT: [nwg][16] s_memrealtime per phase (thread 0)
#endif
};
#if TT_EXPERIMENTS
#define TDBG(bit) ((a.dbg & (bit)) != 0)
#else
#define TDBG(bit) false
#endif
// EXPERIMENT (TT_T1_DEBUG bit 64 with 8): lane 0 of every wave at its arrival at barrier k (1..7),
// at its start (0) and its end (8): [nwg][16][9] after the 8192 stamps of the other launches
#if TT_EXPERIMENTS
#define T1_WSTAMP(k) \
  do { if (a.stamps && (a.dbg & 64) && lane == 0) a.stamps[8192 + ((int64_t)blockIdx.x * 16 + (k)) * 9 + wid] = (int64_t)__builtin_amdgcn_s_memrealtime(); } while (0)
#define T1_STAMP(k) \
  do { if (a.stamps && threadIdx.x == 0) a.stamps[(int64_t)blockIdx.x * 16 + (k)] = (int64_t)__builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define T1_WSTAMP(k) do { } while (0)
#define T1_STAMP(k) do { } while (0)
#endif

__device__ __forceinline__ float lbl(const void* p, int dt, int64_t i) {
  if (dt == TT_I32) return (float)reinterpret_cast<const int32_t*>(p)[i];
  if (dt == TT_I64) return (float)reinterpret_cast<const int64_t*>(p)[i];
  return reinterpret_cast<const float*>(p)[i];
}

// acc[mt][j] += A(lds, rows 16*mt..) x B(global bf16, k-major rows) over K (multiple of 32)
// B fragment: lane reads 8 consecutive k of "column" n from a [n][k]-layout matrix (ldb elems).
__device__ __forceinline__ void mma_lds_global(f32x4 (&acc)[2][2], const __bf16* As, int lda_s,
                                               const __bf16* Bg, int64_t ldb, int K, int n0a, int n0b,
                                               bool has_b) {
  // K <= 128 (4 k-steps): every B fragment (weights, L2-resident) is issued before the first
  // MFMA so the GEMM pays one L2 round trip, not one per k-step.
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int nk = K >> 5;
  bf16x8 b0[4], b1[4];
  const __bf16* p0 = Bg + (int64_t)(n0a + r) * ldb + q * 8;
  const __bf16* p1 = Bg + (int64_t)(n0b + r) * ldb + q * 8;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s < nk) {
      b0[s] = *reinterpret_cast<const bf16x8*>(p0 + s * 32);
      if (has_b) b1[s] = *reinterpret_cast<const bf16x8*>(p1 + s * 32);
    }
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s < nk) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(As + r * lda_s + s * 32 + q * 8);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(As + (16 + r) * lda_s + s * 32 + q * 8);
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0[s], acc[0][0], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0[s], acc[1][0], 0, 0, 0);
      if (has_b) {
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1[s], acc[0][1], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1[s], acc[1][1], 0, 0, 0);
      }
    }
  }
}

__global__ void __launch_bounds__(256) tower_fwd_bwd_kernel(TowerArgs a) {
  // LDS: X chunk, activations per (tower, layer) bf16, last-layer outputs fp32, dZ ping-pong
  __shared__ __attribute__((aligned(16))) __bf16 xs[TR * LSTR];
  __shared__ __attribute__((aligned(16))) __bf16 acts[2][MAXL][TR * LSTR];
  __shared__ __attribute__((aligned(16))) float outf[2][TR * FSTR];
  __shared__ __attribute__((aligned(16))) __bf16 dz[2][TR * LSTR];
  __shared__ float dlog[TR];
  __shared__ float lpart[TR];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r16 = lane & 15, q4 = lane >> 4;
  const int64_t B = a.B;
  const int64_t m0 = (int64_t)blockIdx.x * TR;
  const int L = a.s.L;

  // ================= forward, both towers =================
  for (int t = 0; t < 2; ++t) {
    const int in = a.s.in_dim[t];
    for (int l = 0; l < L; ++l) {
      const int N = a.s.width[l];
      const int K = l == 0 ? in : a.s.width[l - 1];
      const int ntile = N / 16;
      // this wave's n-tiles: wid and wid + 4
      const bool h0 = wid < ntile, h1 = wid + 4 < ntile;
      f32x4 acc[2][2];
      for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4)(0.f);
      const __bf16* Wg = a.wb + a.wcoff[t][l];
      if (l == 0) {
        for (int k0 = 0; k0 < K; k0 += XCH) {
          const int kc = min(XCH, K - k0);
          // stage X[m0.., in_col + k0 ..] fp32 -> bf16 LDS, and X^T to global for T2
          for (int e = threadIdx.x; e < TR * (kc / 4); e += 256) {
            const int row = e / (kc / 4), c4 = (e % (kc / 4)) * 4;
            const int64_t gm = m0 + row;
            bf16x4 bv;
            if (a.ipos) {  // the feature's row as returned by its owner (bf16, what T1 computes on)
              const int kk = k0 + c4, f = a.ifeat0[t] + kk / a.iD;
              const int32_t p = gm < B ? a.ipos[(int64_t)f * B + gm] : -1;
              bv = p >= 0 ? *reinterpret_cast<const bf16x4*>(a.isrc + (int64_t)p * a.iD + kk % a.iD)
                          : (bf16x4)(__bf16)0.f;
            } else {
              f32x4 v = (f32x4)(0.f);
              if (gm < B) v = *reinterpret_cast<const f32x4*>(a.pooled + gm * a.ldp + a.s.in_col[t] + k0 + c4);
              bv[0] = (__bf16)v[0]; bv[1] = (__bf16)v[1]; bv[2] = (__bf16)v[2]; bv[3] = (__bf16)v[3];
            }
            *reinterpret_cast<bf16x4*>(xs + row * LSTR + c4) = bv;
          }
          __syncthreads();
          // X^T [t][k][B]: thread -> (k, 8 consecutive rows)
          for (int e = threadIdx.x; e < kc * (TR / 8); e += 256) {
            const int k = e / (TR / 8), rb = (e % (TR / 8)) * 8;
            bf16x8 v;
            for (int j = 0; j < 8; ++j) v[j] = xs[(rb + j) * LSTR + k];
            const int64_t gm = m0 + rb;
            __bf16* dst = a.xt + (int64_t)t * a.in_max * a.Bp + strip_at(k0 + k, gm, a.in_max);
            if (gm + 8 <= B) {
              *reinterpret_cast<bf16x8*>(dst) = v;
            } else {
              for (int j = 0; j < 8; ++j)
                if (gm + j < B) dst[j] = v[j];
            }
          }
          if (h0) mma_lds_global(acc, xs, LSTR, Wg + k0, K, kc, wid * 16, (wid + 4) * 16, h1);
          __syncthreads();
        }
      } else {
        if (h0) mma_lds_global(acc, acts[t][l - 1], LSTR, Wg, K, K, wid * 16, (wid + 4) * 16, h1);
      }
      // epilogue: bias + relu -> LDS (bf16; fp32 too for the last layer), act^T -> global
      const float* bias = a.params + a.boff[t][l];
      for (int j = 0; j < 2; ++j) {
        if (!(j == 0 ? h0 : h1)) continue;
        const int col = (wid + 4 * j) * 16 + r16;
        const float bv = bias[col];
        for (int i = 0; i < 2; ++i) {
          bf16x4 pk;
          for (int rr = 0; rr < 4; ++rr) {
            const int row = i * 16 + q4 * 4 + rr;
            const float v = fmaxf(acc[i][j][rr] + bv, 0.f);
            acts[t][l][row * LSTR + col] = (__bf16)v;
            pk[rr] = (__bf16)v;
            if (l == L - 1) outf[t][row * FSTR + col] = v;
          }
          if (l < L - 1) {
            const int64_t gm = m0 + i * 16 + q4 * 4;
            __bf16* dst = a.act + ((int64_t)t * MAXL + l) * MAXW * a.Bp + strip_at(col, gm, MAXW);
            if (gm + 4 <= B) {
              *reinterpret_cast<bf16x4*>(dst) = pk;
            } else {
              for (int rr = 0; rr < 4; ++rr)
                if (gm + rr < B) dst[rr] = pk[rr];
            }
          }
        }
      }
      __syncthreads();
    }
  }

  // ================= logits, BCE, dlogit =================
  const int NL = a.s.width[L - 1];
  {
    // 8 threads per row
    const int row = threadIdx.x >> 3, sub = threadIdx.x & 7;
    float d = 0.f;
    for (int c = sub; c < NL; c += 8) d += outf[0][row * FSTR + c] * outf[1][row * FSTR + c];
    d += __shfl_xor(d, 1, 64);
    d += __shfl_xor(d, 2, 64);
    d += __shfl_xor(d, 4, 64);
    const int64_t gm = m0 + row;
    float lo = 0.f, dl = 0.f;
    if (gm < B) {
      const float x = d, y = lbl(a.labels, a.label_dtype, gm);
      const float lsig = fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
      lo = (1.f - y) * x - lsig;
      dl = (1.f / (1.f + expf(-x)) - y) / (float)B * a.grad_scale;
      if (sub == 0) a.logits[gm] = x;
    }
    if (sub == 0) {
      dlog[row] = dl;
      lpart[row] = lo;
    }
  }
  __syncthreads();

  // ================= backward, tower by tower =================
  for (int t = 0; t < 2; ++t) {
    // dZ_{L-1} = dlogit * other * (self > 0): thread -> (8 consecutive rows, column), fp32
    {
      const float* self_ = outf[t];
      const float* other = outf[1 - t];
      float* dbp = a.dbpart + (((int64_t)t * MAXL + (L - 1)) * a.nwg + blockIdx.x) * MAXW;
      for (int c = threadIdx.x >> 2; c < NL; c += 64) {
        const int rb = (threadIdx.x & 3) * 8;
        bf16x8 v;
        float s = 0.f;
        for (int j = 0; j < 8; ++j) {
          const int row = rb + j;
          float z = self_[row * FSTR + c] > 0.f ? dlog[row] * other[row * FSTR + c] : 0.f;
          if (m0 + row >= B) z = 0.f;
          s += z;
          v[j] = (__bf16)z;
          dz[0][row * LSTR + c] = (__bf16)z;
        }
        // bias-grad partial: 4 threads per column, fixed order
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        if ((threadIdx.x & 3) == 0) dbp[c] = s;
        const int64_t gm = m0 + rb;
        __bf16* dst = a.dzt + ((int64_t)t * MAXL + (L - 1)) * MAXW * a.Bp + strip_at(c, gm, MAXW);
        if (gm + 8 <= B) {
          *reinterpret_cast<bf16x8*>(dst) = v;
        } else {
          for (int j = 0; j < 8; ++j)
            if (gm + j < B) dst[j] = v[j];
        }
      }
    }
    __syncthreads();
    int cur = 0;
    for (int l = L - 1; l >= 1; --l) {
      // dA_{l-1} = dZ_l W_l : [TR, K=width[l]] x [width[l], width[l-1]], B from W^T [in][out]
      const int Kd = a.s.width[l];
      const int N = a.s.width[l - 1];
      const int ntile = N / 16;
      const bool h0 = wid < ntile, h1 = wid + 4 < ntile;
      f32x4 acc[2][2];
      for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4)(0.f);
      if (h0) mma_lds_global(acc, dz[cur], LSTR, a.wtb + a.wcoff[t][l], Kd, Kd, wid * 16, (wid + 4) * 16, h1);
      // dZ_{l-1} = dA * (act_{l-1} > 0)
      float* dbp = a.dbpart + (((int64_t)t * MAXL + (l - 1)) * a.nwg + blockIdx.x) * MAXW;
      for (int j = 0; j < 2; ++j) {
        if (!(j == 0 ? h0 : h1)) continue;
        const int col = (wid + 4 * j) * 16 + r16;
        float s = 0.f;
        for (int i = 0; i < 2; ++i) {
          bf16x4 pk;
          for (int rr = 0; rr < 4; ++rr) {
            const int row = i * 16 + q4 * 4 + rr;
            float z = (float)acts[t][l - 1][row * LSTR + col] > 0.f ? acc[i][j][rr] : 0.f;
            if (m0 + row >= B) z = 0.f;
            s += z;
            pk[rr] = (__bf16)z;
            dz[cur ^ 1][row * LSTR + col] = (__bf16)z;
          }
          const int64_t gm = m0 + i * 16 + q4 * 4;
          __bf16* dst = a.dzt + ((int64_t)t * MAXL + (l - 1)) * MAXW * a.Bp + strip_at(col, gm, MAXW);
          if (gm + 4 <= B) {
            *reinterpret_cast<bf16x4*>(dst) = pk;
          } else {
            for (int rr = 0; rr < 4; ++rr)
              if (gm + rr < B) dst[rr] = pk[rr];
          }
        }
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        if (q4 == 0) dbp[col] = s;
      }
      __syncthreads();
      cur ^= 1;
    }
    // dX = dZ_0 W_0 : [TR, width[0]] x [width[0], in] -> fp32 into the pooled gradient
    {
      const int in = a.s.in_dim[t];
      const int Kd = a.s.width[0];
      const __bf16* WT = a.wtb + a.wcoff[t][0];  // [in][width0]
      for (int c0 = 0; c0 < in; c0 += XCH) {
        const int nc = min(XCH, in - c0);
        const int ntile = nc / 16;
        const bool h0 = wid < ntile, h1 = wid + 4 < ntile;
        f32x4 acc[2][2];
        for (int i = 0; i < 2; ++i)
          for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4)(0.f);
        if (h0) mma_lds_global(acc, dz[cur], LSTR, WT, Kd, Kd, c0 + wid * 16, c0 + (wid + 4) * 16, h1);
        for (int j = 0; j < 2; ++j) {
          if (!(j == 0 ? h0 : h1)) continue;
          const int col = c0 + (wid + 4 * j) * 16 + r16;
          if (a.ipos) {  // dX column -> the lookup's gradient row in the exchange buffer
            const int f = a.ifeat0[t] + col / a.iD, cc = col % a.iD;
            for (int i = 0; i < 2; ++i)
              for (int rr = 0; rr < 4; ++rr) {
                const int64_t gm = m0 + i * 16 + q4 * 4 + rr;
                const int32_t p = gm < B ? a.ipos_out[(int64_t)f * B + gm] : -1;
                if (p >= 0) a.idst[(int64_t)p * a.iD + cc] = acc[i][j][rr];
              }
            continue;
          }
          for (int i = 0; i < 2; ++i)
            for (int rr = 0; rr < 4; ++rr) {
              const int64_t gm = m0 + i * 16 + q4 * 4 + rr;
              if (gm < B) a.gpooled[gm * a.ldp + a.s.in_col[t] + col] = acc[i][j][rr];
            }
        }
      }
    }
    __syncthreads();
  }

  // loss: per-workgroup partial; T2 sums the partials in a fixed order (no cross-workgroup
  // hand-off inside T1: a release fence here costs more than the rest of the epilogue)
  if (threadIdx.x == 0) {
    float p = 0.f;
    for (int i = 0; i < TR; ++i) p += lpart[i];
    a.loss_part[blockIdx.x] = p;
  }
}

// ---------------------------------------------------------------------------------------------
// T1 fast path: two layers per tower, every width <= 128. 512 threads: waves 0-3 run the query
// tower, waves 4-7 the candidate tower, in lockstep. Every weight fragment a wave needs for the
// whole step (fwd L0, fwd L1, bwd L1, bwd L0: up to 32 x 16 B per lane) is issued at kernel
// entry together with the X rows, so the only global round trip on the chain is X itself; the rest
// is LDS + MFMA.

struct Frags {
  bf16x8 f[4][2];
};

// B-fragment order of a [N][K] matrix (K % 32 == 0): the 16 x 32 fragment (n-tile nt, k-step s) is
// 64 lanes x 8 contiguous elements, lane q * 16 + r holding row nt * 16 + r, columns s * 32 + q * 8 ..
__host__ __device__ __forceinline__ int64_t frag_off(int n, int k, int K) {
  return ((int64_t)((n >> 4) * (K >> 5) + (k >> 5)) * 64 + ((k & 31) >> 3) * 16 + (n & 15)) * 8 + (k & 7);
}

// fragments of W (fragment-major copy, see frag_off): one 1-KB contiguous load per (tile, k-step)
__device__ __forceinline__ void load_frags(Frags& fr, const __bf16* Wf, int ld, int K, int N, int w4) {
  const int lane = threadIdx.x & 63;
  const int nk = K >> 5, nt = N >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int tile = w4 + 4 * j;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (tile < nt && s < nk)
        fr.f[s][j] = *reinterpret_cast<const bf16x8*>(Wf + ((int64_t)(tile * nk + s) * 64 + lane) * 8);
  }
}

__device__ __forceinline__ void mma_frags(f32x4 (&acc)[2][2], const __bf16* As, const Frags& fr, int K, int N,
                                          int w4) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int nk = K >> 5, nt = N >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4)(0.f);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s < nk) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(As + r * LSTR + s * 32 + q * 8);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(As + (16 + r) * LSTR + s * 32 + q * 8);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (w4 + 4 * j < nt) {
          acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, fr.f[s][j], acc[0][j], 0, 0, 0);
          acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, fr.f[s][j], acc[1][j], 0, 0, 0);
        }
    }
  }
}

// T1's W0 image in LDS: [hidden unit][input column] bf16 in 256-B rows whose 16-B chunks are
// XOR-swizzled by row (CDNA4 guide T10, layout (b)). Layer 0 takes its W0 fragments from global
// memory and files them here; the dX product reads the SAME image transposed
// (ds_read_b64_tr_b16) instead of loading a second, transposed copy of W0 from global memory.
__device__ __forceinline__ int w0_off(int row, int ch) {  // byte offset of 16-B chunk ch of row
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// f0 (B fragments of W0 as layer 0 reads it: lane r + 16 q of fragment (k-step s, tile j) holds
// W0[tile * 16 + r][s * 32 + 8 q .. + 7], one 16-B chunk) -> the image
__device__ __forceinline__ void w0_image_store(char* img, const Frags& f0, int K, int N, int w4) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int nk = K >> 5, nt = N >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (w4 + 4 * j < nt && s < nk)
        *reinterpret_cast<bf16x8*>(img + w0_off((w4 + 4 * j) * 16 + r, 4 * s + q)) = f0.f[s][j];
}

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// acc = A (LDS rows, K = W0 columns) x W0 (the image, [K = hidden][N = input]): the B fragment of
// (k-step s, n-tile nt) is B[s * 32 + 8 q + e][nt * 16 + r] = image[row s * 32 + 8 q + e][col nt * 16 + r],
// two transposed reads of 4 image rows x 16 columns each (lane 4 q' + p of a 16-lane group
// addresses row q', columns 4 p .. 4 p + 3; lane i receives column i). Every lane of the wave
// executes the reads (wave-uniform conditions only: the read needs a full EXEC mask).
__device__ __forceinline__ void mma_w0_tr(f32x4 (&acc)[2][2], const __bf16* As, const char* img, int K, int N,
                                          int w4) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int qq = (lane & 15) >> 2, p = lane & 3;
  const int nk = K >> 5, nt = N >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4)(0.f);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s < nk) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(As + r * LSTR + s * 32 + q * 8);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(As + (16 + r) * LSTR + s * 32 + q * 8);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (w4 + 4 * j < nt) {
          const int row = s * 32 + 8 * q + qq, ch = 2 * (w4 + 4 * j) + (p >> 1);
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(img + w0_off(row, ch) + 8 * (p & 1)));
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_bf16x4*)(img + w0_off(row + 4, ch) + 8 * (p & 1)));
          const bf16x8 b = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b, acc[0][j], 0, 0, 0);
          acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b, acc[1][j], 0, 0, 0);
        }
    }
  }
}

// lane value from another lane of its 16-lane row by DPP (no LDS round trip: ds_bpermute is one)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// sum over each 16-lane row, every lane of the row receives it: quad_perm [1,0,3,2], quad_perm
// [2,3,0,1], row_half_mirror, row_mirror (each step adds the mirrored partner's partial sum, so
// partners compute identical values)
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}

// 4 consecutive rows r0.. of one strip feature (tile-local row r0, nval valid rows in the tile)
__device__ __forceinline__ void store_t4(__bf16* dst, const bf16x4& pk, int r0, int nval) {
  if (r0 + 4 <= nval) {
    *reinterpret_cast<bf16x4*>(dst) = pk;
  } else {
    for (int rr = 0; rr < 4; ++rr)
      if (r0 + rr < nval) dst[rr] = pk[rr];
  }
}

// Multi-hot EBC forward inside T1 (MH): thread tt of tower t's 256-thread group owns the float4
// column c4 of rows (tt + 256 i) / LPR, i < NXV, as the single-hot gather does. The LPR lanes of a
// row group walk the concatenation of their NXV bags (bag order kept inside each bag) in chunks of
// LPR ids, one coalesced id read per chunk (the next chunk's ids in flight beside this chunk's
// rows), ids broadcast by lane shuffles, R rows in flight per lane whatever the bag lengths. Each
// bag's rows are added in bag order starting from zero: the fp32 sums are bit-identical to
// tt_pooled_fwd (SUM) of the same bag.
template <int IN_>
__device__ __forceinline__ void mh_gather(const TowerArgs& a, int t, int tt, int64_t m0, int64_t B,
                                          f32x4 (&xv)[4]) {
  constexpr int LPR = IN_ / 4;   // lanes per row: 32 (D 128) or 16 (D 64)
  constexpr int NXV = IN_ / 32;  // rows (bags) per thread: 4 or 2
  constexpr int R = IN_ == 128 ? 16 : 8;  // rows in flight per lane (D 64: 8, no spills)
  static_assert(LPR % R == 0, "a chunk is a whole number of rounds");
  const int lane = threadIdx.x & 63;
  const int lg = lane & (LPR - 1), gb = lane & ~(LPR - 1);
  const float* tab = t ? a.gtab[1] : a.gtab[0];
  const int32_t* off = t ? a.moff[1] : a.moff[0];
  const uint64_t nrows = (uint64_t)(t ? a.gmod[1] : a.gmod[0]);
  const float* colp = tab + lg * 4;
  int s[NXV], p[NXV + 1];
  p[0] = 0;
#pragma unroll
  for (int i = 0; i < NXV; ++i) {
    const int64_t gm = m0 + (tt + 256 * i) / LPR;
    s[i] = 0;
    int n = 0;
    if (gm < B) {
      s[i] = off[gm];
      n = off[gm + 1] - s[i];
    }
    p[i + 1] = p[i] + n;
    xv[i] = (f32x4)(0.f);
  }
  const int total = p[NXV];
  // combined position k (< total) -> element offset of its table row (an id >= rows reads row 0)
  auto row_at = [&](int k) -> int64_t {
    int si = s[0], pi = 0;
#pragma unroll
    for (int i = 1; i < NXV; ++i)
      if (k >= p[i]) {
        si = s[i];
        pi = p[i];
      }
    const int64_t id = load_id(a.mval, a.gid_dtype, (int64_t)si + (k - pi));
    return (uint64_t)id < nrows ? id * IN_ : 0;
  };
  int64_t nxt = lg < total ? row_at(lg) : 0;
  for (int k0 = 0; __ballot(k0 < total) != 0; k0 += LPR) {
    const int64_t cur = nxt;
    if (k0 + LPR + lg < total) nxt = row_at(k0 + LPR + lg);
#pragma unroll
    for (int k = 0; k < LPR; k += R) {
      if (__ballot(k0 + k < total) == 0) break;
      f32x4 r[R];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int64_t o = __shfl((long long)cur, gb + k + u, 64);
        r[u] = k0 + k + u < total ? *reinterpret_cast<const f32x4*>(colp + o) : (f32x4)(0.f);
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int kk = k0 + k + u;
#pragma unroll
        for (int i = 0; i < NXV; ++i)
          if (kk >= p[i] && kk < p[i + 1]) xv[i] += r[u];
      }
    }
  }
}

// IN_/W0_/W1_: compile-time tower input width and layer widths (0 = read from the shape at run
// time). With them fixed every fragment load is unconditional, so the waitcnt that guards X (issued
// first) does not also wait for the weight fragments issued behind it.
// 8 compute waves + 1 dedup wave; the compute path has exactly T1_BARRIERS __syncthreads
constexpr int T1_THREADS = 576;
constexpr int T1_BARRIERS = 7;

// R16: indexed rows arrive as bf16 (sharded step, tt_tower_fwd_bwd_indexed_bf16); its own
// instantiation, so the other modes' code and registers are untouched. UPD: the in-place update of
// single-lookup rows (TowerArgs::uw); gather mode only.
template <int IN_, int W0_, int W1_, bool R16 = false, bool UPD = false, bool MH = false>
__global__ void __launch_bounds__(T1_THREADS) tower_l2_kernel(TowerArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 xs[2][TR * LSTR];   // X, later dZ0
  __shared__ __attribute__((aligned(16))) __bf16 hs[2][TR * LSTR];   // hidden activation (bf16)
  __shared__ __attribute__((aligned(16))) __bf16 dzs[2][TR * LSTR];  // dZ1
  __shared__ __attribute__((aligned(16))) float outf[2][TR * FSTR];  // tower outputs, later dX (fp32)
  __shared__ float dlog[TR];
  __shared__ float lpart[TR];
  __shared__ __attribute__((aligned(16))) char w0img[2][128 * 256];  // W0 image (w0_off), per tower
  // UPD: per (tower, row) the lookup's table row (-1: not updated here) and its row-wise state,
  // filed by the dedup wave (the fp32 rows as gathered stay in the compute waves' registers)
  __shared__ int64_t urow[2][TR];
  __shared__ float ustate[2][TR];

  // wid via readfirstlane: the compiler then knows t (below) is wave-uniform and reads a.gcol[t],
  // a.gtab[t], ... with scalar loads (a per-lane index into the kernarg arrays is a vector load from
  // the kernarg segment: one more dependent memory hop in front of the row gather)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the [128, 64] towers over 64- or 128-wide inputs write ROW-MAJOR operand strips ([Bp][features], as the
  // row-owned T1 does; the tail reads them with wgrad_lds_block_rm): copies of the LDS tiles
  constexpr bool RM = (IN_ == 128 || IN_ == 64) && W0_ == 128 && W1_ == 64;
  auto rm_copy = [&](const __bf16* tile, __bf16* dst, int nchunk, int ld, int nval_) {
    // tile: TR rows at LSTR; dst: row 0 of the tile in a [Bp][ld] strip; nchunk 16-B pieces per row
    const int tt_ = threadIdx.x & 255;
    for (int idx = tt_; idx < TR * nchunk; idx += 256) {
      const int row = idx / nchunk, ch = idx % nchunk;
      if (row < nval_)
        *reinterpret_cast<bf16x8*>(dst + (int64_t)row * ld + ch * 8) = *reinterpret_cast<const bf16x8*>(tile + row * LSTR + ch * 8);
    }
  };
  if (UPD && wid == 8) {
    T1_WSTAMP(0);
    // ---- the dedup wave (UPD): for each of the 2 x TR lookups, is its row looked up once in this
    // step? (claim >= 0 and slot count 1 in the batch's completed table) -> row and state to LDS
    // All of this wave's dependent global round trips (id -> claim / state -> slot word; the next
    // batch's id) finish before barrier 1: the compute waves spend ~5 us gathering there, while a
    // round trip after barrier 1 made this wave the last arrival at barrier 2 (by 0.8-1.2 us).
    const int tq = lane / TR, row = lane % TR;
    const int64_t gm = (int64_t)xcd_remap((int)blockIdx.x, (int)gridDim.x) * TR + row;
    const bool pref = a.pcol[0] != nullptr;
    int64_t r = -1;
    int32_t cl = -1;
    float st = 0.f;
    int64_t idn = 0;
    if (gm < a.B) {
      const int64_t id = load_id(tq ? a.gcol[1] : a.gcol[0], a.gid_dtype, gm);
      if (pref) idn = load_id(tq ? a.pcol[1] : a.pcol[0], a.gid_dtype, gm);
      if (id != 0) {
        r = py_mod64(id, tq ? a.gmod[1] : a.gmod[0]);
        cl = a.dd.claim[tq * a.B + gm];
        st = (tq ? a.us[1] : a.us[0])[r];  // speculative: used only for a single-lookup row
      }
    }
    const uint64_t word = cl >= 0 ? a.dd.slots[cl].word : DD_EMPTY;
    const bool single = r >= 0 && cl >= 0 && (word & (uint32_t)DD_CNT_MASK) == 1u;
    urow[tq][row] = single ? r : -1;
    ustate[tq][row] = st;
    if (blockIdx.x == 0 && lane == 0) {  // the table's hot-row count for the update launch (dd_update_block)
      const int32_t nh = a.dd.ctr[0];
      a.dd.ctr[2] = nh;
      a.dd.ctr[0] = 0;
    }
    T1_WSTAMP(1);
    __syncthreads();
    // the next batch's rows of this tile, after the compute waves' gather has landed (barrier 1):
    // 64-B segment k = j * 64 + lane of row k / SEG, all loads in flight across the remaining
    // barriers (a barrier waits only on LDS counters), consumed once after the last one
    constexpr int SEG = (IN_ ? IN_ : 128) * 4 / 64;  // 64-B segments per row (UPD: IN_ is 64 or 128)
    constexpr int NPF = 2 * TR * SEG / 64;
    uint32_t pv[NPF];
    uint32_t pf = 0;
    auto issue_prefetch = [&]() {
      const float* base = nullptr;
      if (gm < a.B) {
        if (idn != 0) {
          const int64_t rn = py_mod64(idn, tq ? a.gmod[1] : a.gmod[0]);
          base = (tq ? a.gtab[1] : a.gtab[0]) + rn * IN_;
          pf = __float_as_uint((tq ? a.us[1] : a.us[0])[rn]);
        }
      }
      const uint64_t b64 = reinterpret_cast<uint64_t>(base);
#pragma unroll
      for (int j = 0; j < NPF; ++j) {
        const int k = j * 64 + lane, lk = k / SEG;  // lookup lk = tq * TR + row of the wave's lane order
        const uint64_t p = (uint64_t)__shfl((long long)b64, lk, 64);
        pv[j] = p ? *reinterpret_cast<const uint32_t*>(p + (k % SEG) * 64) : 0u;
      }
    };
    const bool late = TDBG(256);  // experiment: prefetch after the last barrier
    if (pref && !late) issue_prefetch();
    uint32_t touch = 0;
#pragma unroll 1
    for (int k = 1; k < T1_BARRIERS; ++k) {
      if (k == 5 && TDBG(512) && r >= 0) {
        // experiment: re-touch this lookup's row and state (translation) ahead of the in-place update
        touch = *reinterpret_cast<const uint32_t*>((tq ? a.gtab[1] : a.gtab[0]) + r * IN_) ^
                __float_as_uint((tq ? a.us[1] : a.us[0])[r]);
      }
      T1_WSTAMP(k + 1);
      __syncthreads();
    }
    if (pref && late) issue_prefetch();
    if (pref || touch) {
      pf ^= touch;
#pragma unroll
      for (int j = 0; j < NPF; ++j) pf ^= pref ? pv[j] : 0u;
      if (pf == 0x7fc00123u && a.B < 0) a.logits[0] = 0.f;  // never taken: keeps the loads
    }
    T1_WSTAMP(8);
    return;
  }
  if (wid == 8) {
    // ---- the dedup wave: files this workgroup's 2 x TR lookups (gather + dedup) into the hash
    // table; its CAS round trips count only in ITS vmcnt, so the 8 compute waves never wait on
    // them. It passes the compute waves' barriers (T1_BARRIERS, all unconditional) in step.
    const int tq = lane / TR, row = lane % TR;
    const int64_t gm = (int64_t)xcd_remap((int)blockIdx.x, (int)gridDim.x) * TR + row;
    const bool own = a.dd_on && gm < a.B;
    DdPend p;
    if (own) {
      // per-lane tower: select between the two towers' kernel arguments (no dynamic kernarg index)
      const int64_t id = load_id(tq ? a.gcol[1] : a.gcol[0], a.gid_dtype, gm);
      const int64_t mod = tq ? a.gmod[1] : a.gmod[0];
      const uint64_t tab = (uint64_t)(tq ? a.dd_table[1] : a.dd_table[0]);
      const uint64_t key = id != 0 ? ((tab << DD_TABLE_SHIFT) | (uint64_t)py_mod64(id, mod)) : DD_EMPTY;
      dd_insert_begin(a.dd, key, (int32_t)(tq * a.B + gm), p);
    } else {
      p.key = DD_EMPTY;
    }
    // the CAS results are needed only after two barriers (about half the compute chain later); a
    // lookup that did not claim a free slot is deferred to the next launch's resolver instead of
    // probing here (dd_insert_defer_finish): this wave's tail is one atomic round trip
    __syncthreads();
    __syncthreads();
    if (a.dd_on) dd_insert_defer_finish(a.dd, p, (int32_t)(tq * a.B + gm), xcd_remap((int)blockIdx.x, (int)gridDim.x));
#if TT_EXPERIMENTS
    if (a.stamps && lane == 0) a.stamps[(int64_t)blockIdx.x * 16 + 8] = (int64_t)__builtin_amdgcn_s_memrealtime();
#endif
#pragma unroll 1
    for (int k = 2; k < T1_BARRIERS; ++k) __syncthreads();
    return;
  }
  const int t = wid >> 2, w4 = wid & 3;
  T1_STAMP(0);
  T1_WSTAMP(0);
  const int tt = threadIdx.x & 255;  // thread index inside the tower group
  const int r16 = lane & 15, q4 = lane >> 4;
  const int64_t B = a.B;
  // the tile: a contiguous 1/8 per XCD (xcd_remap), as tower_rows_body; per-tile partials by tile
  const int tl2 = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int64_t m0 = (int64_t)tl2 * TR;
  const int nval = (int)min((int64_t)TR, B - m0);  // valid rows of this tile (32-bit row tests)
  // this tile's run of each T1 -> T2 strip (tile-major, strip_at): wave-uniform bases, so a
  // store's address is base + (feature * TR + row) in 32 bits
  const int64_t tile_el = (int64_t)tl2 * TR;
  __bf16* const xt_tile = a.xt + (int64_t)t * a.in_max * a.Bp + tile_el * a.in_max;
  __bf16* const act_tile = a.act + ((int64_t)t * MAXL + 0) * MAXW * a.Bp + tile_el * MAXW;
  __bf16* const dz0_tile = a.dzt + ((int64_t)t * MAXL + 0) * MAXW * a.Bp + tile_el * MAXW;
  __bf16* const dz1_tile = a.dzt + ((int64_t)t * MAXL + 1) * MAXW * a.Bp + tile_el * MAXW;
  float* const db0 = a.dbpart + (((int64_t)t * MAXL + 0) * a.nwg + tl2) * MAXW;
  float* const db1 = a.dbpart + (((int64_t)t * MAXL + 1) * a.nwg + tl2) * MAXW;
  const int in = IN_ ? IN_ : a.s.in_dim[t];
  const int W0 = W0_ ? W0_ : a.s.width[0];
  const int W1 = W1_ ? W1_ : a.s.width[1];

  // ---- 0. everything this wave will read from global: X rows first (the chain waits on them),
  // then every weight fragment of the step in order of use, then the biases
  f32x4 xv[4];
  bf16x4 xb[4];  // R16: the bf16 rows as loaded (T1 stores bf16 to LDS anyway: no widening)
  const int nxv = in / 32;  // f32x4 loads per thread: TR rows x in/4 vectors over 256 threads
  const bool gather = a.gcol[t] != nullptr;
  const bool indexed = a.gpos[t] != nullptr;
  const int incol = a.s.in_col[t];  // read once, before any store (no vmcnt waits mid-chain)
  int32_t rpos[4];                   // indexed: the dX row of each xv (gpos_out, else its input row)
#pragma unroll
  for (int i = 0; i < 4; ++i) rpos[i] = -1;
  if constexpr (MH) {
    mh_gather<IN_>(a, t, tt, m0, B, xv);
  } else if (gather || indexed) {
    // single-hot: the embedding row itself (EBC forward fused in); id 0 -> empty bag -> zeros.
    // Indexed rows may be bf16 (tt_tower_fwd_bwd_indexed_bf16): byte offsets with the element size
    const bool r16 = R16;
    const char* src[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      src[i] = nullptr;
      rpos[i] = -1;
      if (i < nxv) {
        const int e = tt + 256 * i;
        const int row = e / (in / 4), c4 = (e % (in / 4)) * 4;
        const int64_t gm = m0 + row;
        if (gm < B) {
          if (indexed) {
            const int32_t pin = a.gpos[t][gm];
            rpos[i] = pin >= 0 && a.gpos_out[t] ? a.gpos_out[t][gm] : pin;
            if (pin >= 0)
              src[i] = reinterpret_cast<const char*>(a.gsrc[t]) + ((int64_t)pin * in + c4) * (r16 ? 2 : 4);
          } else {
            const int64_t id = TDBG(32) ? 1 : load_id(a.gcol[t], a.gid_dtype, gm);
            if (id != 0)
              src[i] = reinterpret_cast<const char*>(a.gtab[t] + (TDBG(4) ? 0 : py_mod64(id, a.gmod[t])) * in + c4);
          }
        }
      }
    }
    if (r16) {
#pragma unroll
      for (int i = 0; i < 4; ++i) xb[i] = src[i] ? *reinterpret_cast<const bf16x4*>(src[i]) : (bf16x4)(__bf16)0.f;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) xv[i] = src[i] ? *reinterpret_cast<const f32x4*>(src[i]) : (f32x4)(0.f);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xv[i] = (f32x4)(0.f);
      if (i < nxv) {
        const int e = tt + 256 * i;
        const int row = e / (in / 4), c4 = (e % (in / 4)) * 4;
        const int64_t gm = m0 + row;
        if (gm < B) xv[i] = *reinterpret_cast<const f32x4*>(a.pooled + gm * a.ldp + incol + c4);
      }
    }
  }
  Frags f0, f1, g1;
  if (TDBG(16)) {
    for (int s_ = 0; s_ < 4; ++s_) for (int j_ = 0; j_ < 2; ++j_) { f0.f[s_][j_] = (bf16x8)(__bf16)0.f; f1.f[s_][j_] = f0.f[s_][j_]; g1.f[s_][j_] = f0.f[s_][j_]; }
  } else {
  load_frags(f0, a.wbf + a.wcoff[t][0], in, in, W0, w4);      // W0 [W0][in]
  load_frags(f1, a.wbf + a.wcoff[t][1], W0, W0, W1, w4);      // W1 [W1][W0]
  load_frags(g1, a.wtbf + a.wcoff[t][1], W1, W1, W0, w4);     // W1^T [W0][W1]
  }
  float bias0[2], bias1[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = (w4 + 4 * j) * 16 + r16;
    bias0[j] = c < W0 ? a.params[a.boff[t][0] + c] : 0.f;
    bias1[j] = c < W1 ? a.params[a.boff[t][1] + c] : 0.f;
  }
  // the label of the row this thread scores in phase 3 (loaded now: no global load after the CAS)
  const int64_t lrow = m0 + (threadIdx.x >> 4);
  const float ylab = lrow < B ? lbl(a.labels, a.label_dtype, lrow) : 0.f;
  const float gscale = a.grad_scale / (float)B;

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < nxv) {
      const int e = tt + 256 * i;
      const int row = e / (in / 4), c4 = (e % (in / 4)) * 4;
      bf16x4 bv;
      if (R16) {
        bv = xb[i];
      } else {
        bv[0] = (__bf16)xv[i][0]; bv[1] = (__bf16)xv[i][1]; bv[2] = (__bf16)xv[i][2]; bv[3] = (__bf16)xv[i][3];
      }
      *reinterpret_cast<bf16x4*>(xs[t] + row * LSTR + c4) = bv;
      const int64_t gm = m0 + row;
      if (!R16 && a.pooled_out && gm < B)
        *reinterpret_cast<f32x4*>(a.pooled_out + gm * a.ldp + incol + c4) = xv[i];
    }
  }
  // vmcnt(0) while only this wave's loads are outstanding (X, weight fragments, biases, label; the
  // fragments and biases come from L2 right behind X). Without it the compiler's merge of the
  // label-dtype branches leaves the biases "pending", and their first use in phase 1 becomes a
  // vmcnt(0) issued AFTER phase 1's strip stores: a wait for HBM store acknowledgements mid-chain.
  __builtin_amdgcn_s_waitcnt(0x0F70);
  T1_WSTAMP(1);
  __syncthreads();
  T1_STAMP(1);
  // X^T for T2's dW0 (fire-and-forget stores). A 16-lane group takes a block of 16 columns x 8
  // rows of X with two transposed LDS reads (ds_read_b64_tr_b16: lane 4 q' + p addresses row q',
  // columns 4 p .. 4 p + 3 of a 4-row block; lane i receives column i): lane i then holds rows
  // r0 .. r0 + 7 of column c0 + i, one 16-B strip store. Every lane executes the reads (full EXEC):
  // groups past the last block read block 0 and store nothing.
  if (RM) {
    rm_copy(xs[t], a.xt + (int64_t)t * a.in_max * a.Bp + m0 * a.in_max, IN_ / 8, (int)a.in_max, nval);
  } else if (!TDBG(1)) {
    const int g16 = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
    const int nblk = (in / 16) * (TR / 8);  // blocks of 16 columns x 8 rows
    for (int b0 = w4 * 4; b0 < nblk; b0 += 16) {  // wave-uniform
      const int b = b0 + g16;
      const bool own = b < nblk;
      const int cb = own ? b % (in / 16) : 0, r0 = own ? (b / (in / 16)) * 8 : 0;
      const __bf16* src = xs[t] + (r0 + qq) * LSTR + cb * 16 + 4 * pp;
      const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)src);
      const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(src + 4 * LSTR));
      const bf16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      if (own) {
        __bf16* dst = xt_tile + (cb * 16 + i16) * TR + r0;
        if (r0 + 8 <= nval) {
          *reinterpret_cast<bf16x8*>(dst) = v;
        } else {
          for (int j = 0; j < 8; ++j)
            if (r0 + j < nval) dst[j] = v[j];
        }
      }
    }
  }
  T1_WSTAMP(11);
  f32x4 acc[2][2];
  // ---- 1. layer 0: h = relu(X W0^T + b0)
  mma_frags(acc, xs[t], f0, in, W0, w4);
  T1_WSTAMP(12);
  w0_image_store(w0img[t], f0, in, W0, w4);  // read back transposed by the dX product (phase 6)
  T1_WSTAMP(13);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (w4 + 4 * j >= W0 / 16) continue;
    const int col = (w4 + 4 * j) * 16 + r16;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bf16x4 pk;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = i * 16 + q4 * 4 + rr;
        const float v = fmaxf(acc[i][j][rr] + bias0[j], 0.f);
        pk[rr] = (__bf16)v;
        hs[t][row * LSTR + col] = pk[rr];
      }
      const int r0 = i * 16 + q4 * 4;
      if (!RM && !TDBG(1)) store_t4(act_tile + col * TR + r0, pk, r0, nval);
    }
  }
  T1_WSTAMP(2);
  __syncthreads();
  T1_STAMP(2);
  if (RM) rm_copy(hs[t], a.act + ((int64_t)t * MAXL + 0) * MAXW * a.Bp + m0 * MAXW, W0_ / 8, MAXW, nval);
  // ---- 2. layer 1: out = relu(h W1^T + b1) (fp32)
  mma_frags(acc, hs[t], f1, W0, W1, w4);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (w4 + 4 * j >= W1 / 16) continue;
    const int col = (w4 + 4 * j) * 16 + r16;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = i * 16 + q4 * 4 + rr;
        outf[t][row * FSTR + col] = fmaxf(acc[i][j][rr] + bias1[j], 0.f);
      }
  }
  T1_WSTAMP(3);
  __syncthreads();
  T1_STAMP(3);
  // ---- 3. logits, BCE, dlogit: 16 threads per row
  {
    // 16 lanes per row, 4 consecutive columns per lane (one 16-B LDS read per tower), DPP sum
    // over the row's lanes; BCE from one exp, one log and one reciprocal (hardware
    // transcendentals, ~1 ulp) — the phase is one dependent chain per wave, so its length is its
    // instruction count
    const int row = threadIdx.x >> 4, sub = threadIdx.x & 15;
    float d = 0.f;
    for (int c = sub * 4; c < W1; c += 64) {
      const f32x4 u = *reinterpret_cast<const f32x4*>(&outf[0][row * FSTR + c]);
      const f32x4 v = *reinterpret_cast<const f32x4*>(&outf[1][row * FSTR + c]);
      d = fmaf(u[0], v[0], d);
      d = fmaf(u[1], v[1], d);
      d = fmaf(u[2], v[2], d);
      d = fmaf(u[3], v[3], d);
    }
    d = row16_sum(d);
    const int64_t gm = m0 + row;
    float lo = 0.f, dl = 0.f;
    if (gm < B) {
      const float x = d, y = ylab;
      const float e = __expf(-fabsf(x));  // exp(-|x|) in (0, 1]
      const float l1p = e < 1e-4f ? e * (1.f - 0.5f * e) : __logf(1.f + e);
      const float lsig = fminf(x, 0.f) - l1p;  // log(sigmoid(x))
      lo = (1.f - y) * x - lsig;
      const float rc = __builtin_amdgcn_rcpf(1.f + e);
      dl = ((x >= 0.f ? rc : e * rc) - y) * gscale;  // (sigmoid(x) - y) * grad_scale / B
      if (sub == 0) a.logits[gm] = x;
    }
    if (sub == 0) {
      dlog[row] = dl;
      lpart[row] = lo;
    }
  }
  T1_WSTAMP(4);
  __syncthreads();
  T1_STAMP(4);
  // ---- 4. dZ1 = dlogit * other * (self > 0): thread -> (column, 8 consecutive rows)
  for (int c = tt >> 2; c < W1; c += 64) {
    const int rb = (tt & 3) * 8;
    bf16x8 v;
    float s = 0.f, zz[8];
    for (int j = 0; j < 8; ++j) {
      const int row = rb + j;
      float z = outf[t][row * FSTR + c] > 0.f ? dlog[row] * outf[1 - t][row * FSTR + c] : 0.f;
      if (row >= nval) z = 0.f;
      zz[j] = z;
      s += z;
      v[j] = (__bf16)z;
      dzs[t][row * LSTR + c] = v[j];
    }
    if (RM) {
      // the row-owned T1's tree (rk_colsum, then the two 16-row halves): rows paired at row bits
      // 3 (the quad partner ^ 1), 2, 1, 0 (in thread), then the halves (quad partner ^ 2)
#pragma unroll
      for (int j = 0; j < 8; ++j) zz[j] += dpp_f<0xB1>(zz[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) zz[j] += zz[j + 4];
      zz[0] += zz[2];
      zz[1] += zz[3];
      s = zz[0] + zz[1];
      s += dpp_f<0x4E>(s);
    } else {
      s += dpp_f<0xB1>(s);  // the 4 lanes of a column are one quad: xor 1, then xor 2
      s += dpp_f<0x4E>(s);
    }
    if ((tt & 3) == 0) db1[c] = s;
    __bf16* dst = dz1_tile + c * TR + rb;
    if (RM || TDBG(1)) {
    } else if (rb + 8 <= nval) {
      *reinterpret_cast<bf16x8*>(dst) = v;
    } else {
      for (int j = 0; j < 8; ++j)
        if (rb + j < nval) dst[j] = v[j];
    }
  }
  T1_WSTAMP(5);
  __syncthreads();
  T1_STAMP(5);
  if (RM) rm_copy(dzs[t], a.dzt + ((int64_t)t * MAXL + 1) * MAXW * a.Bp + m0 * MAXW, W1_ / 8, MAXW, nval);
  // ---- 5. dZ0 = (dZ1 W1) * (h > 0)  -> xs (X is no longer needed)
  mma_frags(acc, dzs[t], g1, W1, W0, w4);
  T1_WSTAMP(14);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (w4 + 4 * j >= W0 / 16) continue;
    const int col = (w4 + 4 * j) * 16 + r16;
    float s = 0.f, hsum[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bf16x4 pk;
      float zz[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = i * 16 + q4 * 4 + rr;
        float z = (float)hs[t][row * LSTR + col] > 0.f ? acc[i][j][rr] : 0.f;
        if (row >= nval) z = 0.f;
        zz[rr] = z;
        s += z;
        pk[rr] = (__bf16)z;
        xs[t][row * LSTR + col] = pk[rr];
      }
      if (RM) {
        // the row-owned T1's tree over the 16-row half i: row bits 3 (lanes ^ 32), 2 (^ 16), 1, 0
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) zz[rr] += __shfl_xor(zz[rr], 32, 64);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) zz[rr] += __shfl_xor(zz[rr], 16, 64);
        hsum[i] = (zz[0] + zz[2]) + (zz[1] + zz[3]);
      }
      const int r0 = i * 16 + q4 * 4;
      if (!RM && !TDBG(1)) store_t4(dz0_tile + col * TR + r0, pk, r0, nval);
    }
    if (RM) {
      s = hsum[0] + hsum[1];
    } else {
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
    }
    if (q4 == 0) db0[col] = s;
  }
  T1_WSTAMP(6);
  __syncthreads();
  T1_STAMP(6);
  if (RM) rm_copy(xs[t], a.dzt + ((int64_t)t * MAXL + 0) * MAXW * a.Bp + m0 * MAXW, W0_ / 8, MAXW, nval);
  // ---- 6. dX = dZ0 W0 -> LDS (outf is free since phase 4) -> pooled gradient, whole rows
  mma_w0_tr(acc, xs[t], w0img[t], W0, in, w4);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (w4 + 4 * j >= in / 16) continue;
    const int col = (w4 + 4 * j) * 16 + r16;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) outf[t][(i * 16 + q4 * 4 + rr) * FSTR + col] = acc[i][j][rr];
  }
  // ---- 7. loss: per-workgroup partial (T2 sums the partials in a fixed order)
  if (threadIdx.x == 0) {
    float p = 0.f;
    for (int i = 0; i < TR; ++i) p += lpart[i];
    a.loss_part[tl2] = p;
  }
  T1_WSTAMP(7);
  __syncthreads();
  T1_STAMP(7);
  T1_WSTAMP(9);
  // ---- 8. dX from LDS; UPD: the in-place row-wise Adagrad of the rows looked up once. A thread's
  // rows go through each step together — their shuffle reductions and sqrt / division chains
  // interleave instead of running row after row; each row's arithmetic is the K3 update's (sum(G^2)
  // over the row's lanes by xor 16, 8, 4, 2, 1, then rw_state / rw_step / rw_apply)
  f32x4 gq[4];
  float* dstq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dstq[i] = nullptr;
    gq[i] = (f32x4)(0.f);
    if (i < nxv) {
      const int e = tt + 256 * i;
      const int row = e / (in / 4), c4 = (e % (in / 4)) * 4;
      const int64_t gm = m0 + row;
      if (gm < B) {
        if (indexed)
          dstq[i] = rpos[i] >= 0 ? a.gdst[t] + (int64_t)rpos[i] * in + c4 : nullptr;
        else
          dstq[i] = a.gpooled + gm * a.ldp + incol + c4;
      }
      gq[i] = *reinterpret_cast<const f32x4*>(&outf[t][row * FSTR + c4]);
    }
  }
  if (UPD) {
    const int lpr = in / 4;  // the lanes of one row are consecutive (a power of two <= 32)
    float sq[4], s_old[4], snew[4], step[4];
    int64_t ur[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ur[i] = -1;
      sq[i] = 0.f;
      s_old[i] = 0.f;
      if (i < nxv) {
        const int row = (tt + 256 * i) / (in / 4);
        ur[i] = urow[t][row];
        s_old[i] = ustate[t][row];
        sq[i] = rw_sq4(gq[i]);
      }
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1)
      if (o < lpr)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i < nxv) sq[i] += __shfl_xor(sq[i], o, 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      snew[i] = rw_state(s_old[i], sq[i], in);
      step[i] = rw_step(snew[i], a.ulr, a.ueps);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < nxv && ur[i] >= 0) {
        const int c4 = ((tt + 256 * i) % (in / 4)) * 4;
        if (!TDBG(128)) {
          *reinterpret_cast<f32x4*>(a.uw[t] + ur[i] * in + c4) = rw_apply(xv[i], gq[i], step[i]);
          if (c4 == 0) a.us[t][ur[i]] = snew[i];
        }
        if (!a.pooled_out) dstq[i] = nullptr;  // dX is needed only for inspection (pooled_out mode)
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (i < nxv && dstq[i] && !TDBG(2)) *reinterpret_cast<f32x4*>(dstq[i]) = gq[i];
  T1_WSTAMP(8);
  T1_STAMP(15);
}

// ---------------------------------------------------------------------------------------------
// T1, row-owned form (tower_rows_kernel): the production shape — both towers over 128-wide
// single-hot rows gathered from the tables, layers [128, 64]. One workgroup of 4 waves per 32
// batch rows; wave w runs tower t = w >> 1 over rows 16 (w & 1) .. + 15 of the tile through the
// whole chain (gather, both layers, logit, dZ1, dZ0, dX, the in-place row-wise Adagrad) with every
// activation in registers: three barriers (the weight image landed; the towers' outputs exchanged
// for the logit; the workgroup's bias / loss partials combined), no LDS round trip between layers.
//
// Every product is computed transposed, Z^T = W A^T: the weights are the MFMA A operand (M = the
// layer's output features, from an LDS image of both towers' bf16 weights, 96 KB, copied whole by
// LDS-DMA), the wave's 16 batch rows are N. The M rows of every tile are PERMUTED (rk_perm): row
// rho of M-tile mt is feature 32 (mt >> 1) + 8 (rho >> 2) + 4 (mt & 1) + (rho & 3), so a lane's
// result values of the tile pair (2 s, 2 s + 1) are features 32 s + 8 q .. + 7 of its batch row n
// (q = lane >> 4, n = lane & 15) — exactly the B operand of the next product's k-step s, and two
// 16-B pieces of the row (the gathered fp32 row is loaded straight into that layout, and dX comes
// out in it: the row-wise Adagrad updates the row from registers). Forward A fragments are one
// ds_read_b128 per lane (W [out][in] image, conflict-free under rk_swz); backward ones (W^T) two
// ds_read_b64_tr_b16 from the same image (2-way: the minimum with a fixed 8-B half per read).
// The T1 -> T2 operand strips (tile-major, strip_at) go through a per-wave LDS transpose; the bias
// partials are fp32 column sums (a DPP transpose-reduce over the wave's 16 rows, then the two row
// halves in order): the tail launch and T3 read the same buffers as with tower_l2_kernel.
constexpr int RK_IN = 128, RK_W0 = 128, RK_W1 = 64;
constexpr int RK_IMG_T = (RK_W0 + RK_W1) * 256;  // bytes per tower: W0 [128][128], then W1 [64][128]
constexpr int RK_IMG = 2 * RK_IMG_T;             // 98,304 B
// 16-B chunk swizzle of image row `row` (256-B rows): b128 reads of 16 permuted rows x one chunk
// and transposed reads of 8 rows x 4 chunks (two 16-lane groups) hit distinct banks
__host__ __device__ __forceinline__ int rk_swz(int row) {
  return (row & 3) | (((row & 1) | (((row >> 3) & 1) << 1)) << 2);
}
__host__ __device__ __forceinline__ int rk_off(int row, int col) {  // byte offset of bf16 element (row, col)
  return row * 256 + (((col >> 3) ^ rk_swz(row)) << 4) + ((col & 7) << 1);
}
__device__ __forceinline__ int rk_perm(int mt, int rho) {
  return 32 * (mt >> 1) + 8 * (rho >> 2) + 4 * (mt & 1) + (rho & 3);
}
// A fragment (M-tile mt, k-step s) of W from its image ([M][K] rows): lane (rho, q) holds
// W[rk_perm(mt, rho)][32 s + 8 q .. + 7]
__device__ __forceinline__ bf16x8 rk_afwd(const char* img, int mt, int s, int rho, int q) {
  return *reinterpret_cast<const bf16x8*>(img + rk_off(rk_perm(mt, rho), 32 * s + 8 * q));
}
// A fragment (M-tile mt, k-step s) of W^T from the image of W ([K][M] rows): lane 4 q' + p of the
// 16-lane group q addresses image row 32 s + 8 q + q' (+ 4) at the 4 contiguous features
// rk_perm(mt, 4 p .. 4 p + 3); lane rho receives feature rk_perm(mt, rho) at those rows
__device__ __forceinline__ bf16x8 rk_abwd(const char* img, int mt, int s, int lane) {
  const int q = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
  const int row = 32 * s + 8 * q + qq;
  const int col = 32 * (mt >> 1) + 8 * p + 4 * (mt & 1);
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + rk_off(row, col)));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + rk_off(row + 4, col)));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 rk_pack(const f32x4& a, const f32x4& b) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = (__bf16)a[j];
    v[4 + j] = (__bf16)b[j];
  }
  return v;
}
// acc[mt] (mt < MT) = sum over k-steps s < S of A(mt, s) x b[s]: the A fragments of k-step s + 1
// are read (into the other of two register sets) before k-step s's MFMAs issue, so with one wave
// per SIMD each k-step's LDS latency hides behind the previous step's MFMAs
template <int MT, int S, bool BWD>
__device__ __forceinline__ void rk_gemm(f32x4 (&acc)[8], const char* img, const bf16x8 (&b)[4], int lane) {
  const int n = lane & 15, q = lane >> 4;
  bf16x8 fa[2][MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    acc[mt] = (f32x4)(0.f);
    fa[0][mt] = BWD ? rk_abwd(img, mt, 0, lane) : rk_afwd(img, mt, 0, n, q);
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (s + 1 < S) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        fa[(s + 1) & 1][mt] = BWD ? rk_abwd(img, mt, s + 1, lane) : rk_afwd(img, mt, s + 1, n, q);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s & 1][mt], b[s], acc[mt], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}
// lane value from lane ^ X of its 16-lane row (X in {1, 2, 4, 8}) by DPP
template <int X>
__device__ __forceinline__ float rk_xor(float v) {
  if constexpr (X == 1) return dpp_f<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  if constexpr (X == 2) return dpp_f<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  if constexpr (X == 4) return dpp_f<0x1B>(dpp_f<0x141>(v));  // row_half_mirror, then quad reversal
  return dpp_f<0x128>(v);                        // row_ror 8
}
// column sums over the 16 lanes of each 16-lane row: NV values per lane in, NV / 16 out; after it,
// lane n holds the sums of values k = (NV / 16) n + i, i < NV / 16 (halving at lane bits 3, 2, 1, 0)
template <int X, int H>  // the live values v[0, 2 H) -> v[0, H)
__device__ __forceinline__ void rk_halve(float* v, int n) {
  const bool up = (n & X) != 0;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const float keep = up ? v[H + i] : v[i], send = up ? v[i] : v[H + i];
    v[i] = keep + rk_xor<X>(send);
  }
}
template <int NV>
__device__ __forceinline__ void rk_colsum(float (&v)[NV], int n) {
  static_assert(NV == 32 || NV == 16, "column sum of 32 or 16 values per lane");
  rk_halve<8, NV / 2>(v, n);
  rk_halve<4, NV / 4>(v, n);
  rk_halve<2, NV / 8>(v, n);
  rk_halve<1, NV / 16>(v, n);
}
// row-major operand strip ([Bp][nf] bf16, what the tail's wgrad_lds_block_rm reads): lane (q, n)
// stores its 16-B pieces (features 32 s + 8 q .. + 7) of batch row m; a wave instruction writes 16
// whole 64-B row segments
// (every row of the tile, dead rows of a ragged tile included: the strips hold Bp rows, the tail
// reads the first B; no branch around the stores, which would make later load waits count
// conservatively)
template <int NS>
__device__ __forceinline__ void rk_strip(const bf16x8 (&v)[4], __bf16* row, int q) {
#pragma unroll
  for (int s = 0; s < NS; ++s) *reinterpret_cast<bf16x8*>(row + 32 * s + 8 * q) = v[s];
}


// direct exchange (tt_peer_direct_t): where send-buffer row `row` lands (the destination block's
// mapped receive buffer); a uniform loop with scalar kernarg loads selects the block
__device__ __forceinline__ char* px_row(const tt_peer_direct_t& x, int64_t row, int64_t row_bytes) {
  char* base = reinterpret_cast<char*>(x.row0[0]);
  int64_t f0 = 0;
#pragma unroll
  for (int q = 1; q < TT_PEER_MAXW; ++q) {
    if (q < x.W && row >= x.first_row[q]) {
      base = reinterpret_cast<char*>(x.row0[q]);
      f0 = x.first_row[q];
    }
  }
  return base + (row - f0) * row_bytes;
}
// the copy fields split over the grid: workgroup b takes 16-B units [b per, (b + 1) per) of their
// concatenation (d ascending); unit u of this thread -> (src, dst), or false past the end
__device__ __forceinline__ bool px_copy_unit(const tt_peer_direct_t& x, int64_t u, const uint4*& src, uint4*& dst) {
  int64_t pre = 0;
  bool hit = false;
#pragma unroll
  for (int q = 0; q < TT_PEER_MAXW; ++q) {
    const int64_t n = q < x.W ? x.copy_len[q] >> 4 : 0;
    if (!hit && u >= pre && u < pre + n) {
      src = reinterpret_cast<const uint4*>(x.copy_src[q]) + (u - pre);
      dst = reinterpret_cast<uint4*>(x.copy_dst[q]) + (u - pre);
      hit = true;
    }
    pre += n;
  }
  return hit;
}
__device__ __forceinline__ int64_t px_copy_units(const tt_peer_direct_t& x) {
  int64_t n = 0;
#pragma unroll
  for (int q = 0; q < TT_PEER_MAXW; ++q) n += q < x.W ? x.copy_len[q] >> 4 : 0;
  return n;
}

// raw 4- or 8-byte element i of an id / label column: the conversion is left to the caller, so a
// dtype branch does not put a wait for the load right behind it (the loads of a prologue all issue
// before the first wait)
struct RkRaw {
  uint32_t lo, hi;
};
__device__ __forceinline__ RkRaw rk_raw(const void* p, bool wide, int64_t i) {
  RkRaw r;
  if (wide) {
    const uint2 v = reinterpret_cast<const uint2*>(p)[i];
    r.lo = v.x;
    r.hi = v.y;
  } else {
    r.lo = reinterpret_cast<const uint32_t*>(p)[i];
    r.hi = 0u;
  }
  return r;
}
__device__ __forceinline__ int64_t rk_id(RkRaw r, bool wide) {
  return wide ? (int64_t)(((uint64_t)r.hi << 32) | r.lo) : (int64_t)(int32_t)r.lo;
}
__device__ __forceinline__ float rk_label(RkRaw r, int dt) {
  if (dt == TT_I32) return (float)(int32_t)r.lo;
  if (dt == TT_I64) return (float)(int64_t)(((uint64_t)r.hi << 32) | r.lo);
  return __uint_as_float(r.lo);
}
// EXPERIMENT (TT_T1_DEBUG bit 8): lane 0 of each wave at point k: stamps[8192 + (wg * 16 + k) * 9 + wave]
#if TT_EXPERIMENTS
#define RK_STAMP(k) \
  do { if (a.stamps && lane == 0) a.stamps[8192 + ((int64_t)blockIdx.x * 16 + (k)) * 9 + wid] = (int64_t)__builtin_amdgcn_s_memrealtime(); } while (0)
// extra points in wave slots 4 .. 7
#define RK_STAMP2(k) \
  do { if (a.stamps && lane == 0) a.stamps[8192 + ((int64_t)blockIdx.x * 16 + (k)) * 9 + 4 + wid] = (int64_t)__builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define RK_STAMP(k) do { } while (0)
#define RK_STAMP2(k) do { } while (0)
#endif
// ---------------------------------------------------------------------------------------------
// T3: reduce + Adam + bf16 weight copies

struct UpdateArgs {
  float* params;
  float* exp_avg;
  float* exp_avg_sq;
  const float* slab;
  const float* dbpart;
  int64_t P;
  int S;
  int nwg;
  int nseg;
  // segments of the flat parameter vector: W or b of (t, l)
  int64_t seg_off[2 * 2 * MAXL + 1];
  int32_t seg_t[2 * 2 * MAXL], seg_l[2 * 2 * MAXL], seg_isw[2 * 2 * MAXL], seg_n[2 * 2 * MAXL], seg_k[2 * 2 * MAXL];
  int64_t seg_wc[2 * 2 * MAXL];  // bf16 copy offset for W segments
  __bf16* wb;
  __bf16* wtb;
  __bf16* wbf;
  __bf16* wtbf;
  int skip_plain;  // wb / wtb unused by this shape's T1 (tower_l2_kernel): not written
  float lr, beta1, beta2, eps, wd;
  int64_t* step_state;
  int do_adam;
  float* grads_out;  // nullable: the reduced gradient (tests / inspection)
  const float* grads_in;  // nullable: take the gradient from here (data-parallel: all-reduced)
  const float* adam_pre;  // nullable: step size / sqrt(bias correction 2) precomputed by T2 (which
                          // also advanced step_state): no pow() and no arrival ticket here
  // data-parallel towers without an all-reduce launch (pipelined sharded step): grads_out is
  // written out_copies times (stride out_stride, scaled by out_scale: one copy per destination
  // rank of the exchange), and grads_in is the fixed-order sum of in_srcs vectors (stride in_stride)
  int out_copies;
  int64_t out_stride;
  int64_t out_off[16];  // with out_copies > 1: element offset of copy q (explicit, out_stride unused)
  float out_scale;
  int in_srcs;
  int64_t in_stride;
  char* wimg;  // nullable: the row-owned T1's weight image (rk_off), written beside the other copies
  PxWait wt;   // W > 0: every workgroup waits for the exchange that brought grads_in (workgroup 0 signals)
#if TT_EXPERIMENTS
  int64_t* stamps;  // EXPERIMENT (TT_RING_STAMPS): [workgroups][4] s_memrealtime per phase
#endif
};
#if TT_EXPERIMENTS
#define T3_STAMP(k) \
  do { if (a.stamps && threadIdx.x == 0 && bid < 512) a.stamps[(int64_t)bid * 4 + (k)] = (int64_t)__builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define T3_STAMP(k) do { } while (0)
#endif

// one parameter's segment (W or b of tower t, layer l): a loop over the (wave-uniform) segment list
// with scalar kernarg loads and per-lane selects — a per-lane index into the kernarg arrays would be
// a chain of dependent vector loads from the kernarg segment (several us per launch)
struct T3Seg {
  int64_t soff = 0, swc = 0;
  int sisw = 0, sk = 1, sn = 1, st_ = 0, sl_ = 0;
};
__device__ __forceinline__ T3Seg t3_seg(const UpdateArgs& a, int64_t i) {
  T3Seg g;
#pragma unroll
  for (int q = 0; q < 2 * 2 * MAXL; ++q) {
    if (q < a.nseg && i >= a.seg_off[q]) {
      g.soff = a.seg_off[q];
      g.sisw = a.seg_isw[q];
      g.sk = a.seg_k[q];
      g.sn = a.seg_n[q];
      g.swc = a.seg_wc[q];
      g.st_ = a.seg_t[q];
      g.sl_ = a.seg_l[q];
    }
  }
  return g;
}

// after the gradient g of parameter i (value p): gradient copies, Adam, the bf16 copies T1 reads
__device__ __forceinline__ void t3_apply(const UpdateArgs& a, int64_t i, const T3Seg& sg, float p, float m,
                                         float v0, float g, float step_size, float bc2_sqrt, bool adam) {
  // no fma contraction: the contraction choice would otherwise depend on the inlining context (T3,
  // the sharded step's launch G), and every form must give the same bits
#pragma clang fp contract(off)
  const int64_t e = i - sg.soff;
  if (a.grads_out) {
    if (a.out_copies <= 1) {
      a.grads_out[i] = g;
    } else {
      const float gs = g * a.out_scale;
      for (int q = 0; q < a.out_copies; ++q) a.grads_out[a.out_off[q] + i] = gs;
    }
  }
  if (adam) {
    if (a.wd != 0.f) g = g + a.wd * p;
    m = m + (1.f - a.beta1) * (g - m);
    const float v = v0 * a.beta2 + (1.f - a.beta2) * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + a.eps;
    p = p + (-step_size) * m / denom;
    a.exp_avg[i] = m;
    a.exp_avg_sq[i] = v;
    a.params[i] = p;
  }
  if (sg.sisw) {
    const int K = sg.sk, N = sg.sn;
    const int64_t n = e / K, k = e - n * K;
    if (!a.skip_plain) {
      a.wb[sg.swc + e] = (__bf16)p;
      a.wtb[sg.swc + k * N + n] = (__bf16)p;
    }
    a.wbf[sg.swc + frag_off((int)n, (int)k, K)] = (__bf16)p;   // W as [N][K]
    a.wtbf[sg.swc + frag_off((int)k, (int)n, N)] = (__bf16)p;  // W^T as [K][N]
    if (a.wimg)  // the row-owned T1's image: W [out][in], 256-B swizzled rows, W1 after W0
      *reinterpret_cast<__bf16*>(a.wimg + sg.st_ * RK_IMG_T + sg.sl_ * (RK_W0 * 256) + rk_off((int)n, (int)k)) = (__bf16)p;
  }
}

// IDX: the sharded step's form (tt_tower_fwd_bwd_indexed2_bf16): tower t's input row m is bf16 row
// gpos[t][m] of gsrc[t] (-1: zeros; the rows an owner returned, dense), its dX goes to fp32 row
// gpos_out[t][m] of gdst[t]; no in-place update, no insert
// IN: the input width (128 or 64: config 2's D = 64; the first layer then has 2 k-steps and dX 4
// M-tiles, the rows are 256 B)
// POOL: the input rows are the pooled matrix's (tower t's row m at a.pooled + m ldp + in_col[t]:
// the multi-hot path's T1 after tt_pooled_fwd), no ids, no dedup
template <bool UPD, bool IDX, int IN, bool POOL = false>
__device__ __forceinline__ void tower_rows_body(const TowerArgs& a) {
  static_assert(IN == 128 || IN == 64, "row-owned T1: inputs of 128 or 64");
  static_assert(!POOL || (!UPD && !IDX), "pooled input: the plain T1 only");
  constexpr int NI = IN / 32;   // layer-0 k-steps (B-operand pieces xb[s], s < NI)
  constexpr int MTI = IN / 16;  // dX M-tiles (row pieces xv[mt], mt < MTI)
  __shared__ __attribute__((aligned(16))) char wimg[RK_IMG];         // both towers' W0, W1 (rk_off)
  __shared__ __attribute__((aligned(16))) float xo[2][2][16 * 64];  // tower outputs per (tower, row half)
  __shared__ float bsum[2][RK_W0 + RK_W1];                          // row half 1's bias partials
  __shared__ float lrow[TR];                                        // row losses
  __shared__ __attribute__((aligned(16))) float xr[4][16 * IN];     // per wave: its 16 gathered rows
                                                                    // (fp32, 16-B chunk c of row n at c ^ n)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = wid >> 1, h = wid & 1, q = lane >> 4, n = lane & 15;
  // the tile: XCD x runs tiles [x n / 8, (x + 1) n / 8) (xcd_remap), so the 256-row slices the
  // tail's T2 tiles read (also placed a contiguous 1/8 per XCD) were written through that XCD's L2
  const int tile = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int64_t B = a.B, m0 = (int64_t)tile * TR, m = m0 + 16 * h + n;
  const bool live = m < B;
  RK_STAMP(0);
  // ---- 0. loads in dependency order (vmcnt retires in issue order: a wait for a load also waits
  // for everything issued before it): the ids, the label, the biases (raw: no conversion between
  // them); the weight image -> LDS (LDS-DMA, 1 KB per wave instruction); the row
  const bool wide = a.gid_dtype == TT_I64;
  const int64_t mc = live ? m : 0;  // dead rows of a ragged tile read row 0 of every column
  RkRaw id_raw{0u, 0u}, pout_raw{0u, 0u};
  if (IDX) {
    id_raw.lo = (uint32_t)(t ? a.gpos[1] : a.gpos[0])[mc];
    pout_raw.lo = a.gpos_out[0] ? (uint32_t)(t ? a.gpos_out[1] : a.gpos_out[0])[mc] : id_raw.lo;
  } else if (!POOL) {
    id_raw = rk_raw(t ? a.gcol[1] : a.gcol[0], wide, mc);
  }
  // UPD: the claim of this row's lookup in the batch's completed dedup table (no dependency: issued
  // beside the id, so the slot word's load can follow the row DMA instead of stalling the chain after
  // layer 1 for a whole memory round trip)
  int32_t cl = -1;
  if (UPD) cl = a.dd.claim[live ? t * B + m : 0];
  const RkRaw lab_raw = rk_raw(a.labels, a.label_dtype == TT_I64, mc);
  f32x4 b0v[8], b1v[4];
  auto load_biases = [&]() {
    const float* b0p = a.params + a.boff[t][0];
    const float* b1p = a.params + a.boff[t][1];
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) b0v[mt] = *reinterpret_cast<const f32x4*>(b0p + 32 * (mt >> 1) + 8 * q + 4 * (mt & 1));
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) b1v[mt] = *reinterpret_cast<const f32x4*>(b1p + 32 * (mt >> 1) + 8 * q + 4 * (mt & 1));
  };
  // the weight image (no dependency): 24 16-B loads per lane into registers, issued while the ids
  // come back (plain loads: with an LDS-DMA in flight the compiler waits vmcnt(0) at the first use
  // of any load, so the ids must land before the first DMA is issued), written to LDS below
  bf16x8 wreg[RK_IMG / 1024 / 4];
  auto load_image = [&]() {
#pragma unroll
    for (int k = 0; k < RK_IMG / 1024 / 4; ++k)
      wreg[k] = TDBG(16) ? (bf16x8)(__bf16)0.f  // EXPERIMENT (timing only): no image fill
                         : *reinterpret_cast<const bf16x8*>(a.wimg + (wid + 4 * k) * 1024 + lane * 16);
  };
  load_biases();
  __builtin_amdgcn_sched_barrier(0);
  load_image();
  __builtin_amdgcn_sched_barrier(0);
  // direct exchange: this workgroup's first share of the copy region (exchange A's keys), loaded
  // now beside the prologue's loads, stored at the end (the rest of a large share there too)
  uint4 cpv = make_uint4(0u, 0u, 0u, 0u);
  uint4* cpd = nullptr;
  int64_t cp_per = 0, cp_end = 0;
  if constexpr (IDX) {
    if (a.xd.W) {
      const int64_t tot = px_copy_units(a.xd);
      cp_per = (tot + gridDim.x - 1) / gridDim.x;
      cp_end = min(tot, ((int64_t)blockIdx.x + 1) * cp_per);
      const int64_t u = (int64_t)blockIdx.x * cp_per + threadIdx.x;
      const uint4* cps;
      if (u < cp_end && px_copy_unit(a.xd, u, cps, cpd)) cpv = *cps;
      else cpd = nullptr;
    }
  }
  int64_t r;  // the row's index in its source (table row / returned-rows buffer row), -1: zeros
  if (POOL) {
    r = live ? m : -1;
  } else if (IDX) {
    r = live ? (int64_t)(int32_t)id_raw.lo : -1;
  } else {
    const int64_t id = live ? rk_id(id_raw, wide) : 0;
    r = id != 0 ? py_mod64(id, t ? a.gmod[1] : a.gmod[0]) : -1;
  }
  const float* tab = POOL ? a.pooled + a.s.in_col[t] : (t ? a.gtab[1] : a.gtab[0]);
  const int64_t rstride = POOL ? a.ldp : IN;  // floats between consecutive source rows
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) void glb_void;
  // the wave's 16 rows -> LDS by LDS-DMA, two whole 512-B rows per wave instruction (two TLB pages
  // per instruction, full lines; a lane-per-row-piece register gather touches 16 rows per
  // instruction): lane l of instruction i carries 16-B chunk (l & 31) ^ row of row 2 i + (l >> 5),
  // so that the B-layout reads below are conflict-free; rows without an id read table row 0
  // (ignored)
  float* xw = xr[wid];
  // (IN = 64: four 256-B rows per instruction)
  constexpr int CPR = IDX ? IN / 8 : IN / 4;  // 16-B chunks per row (chunk swizzle: c ^ (row & (CPR - 1)))
  constexpr int RPI = 64 / CPR;               // rows per wave instruction
  if (IDX) {
    // bf16 rows (2 IN bytes): lane l carries 16-B chunk (l % CPR) ^ row of row RPI i + l / CPR
    const int rr0 = lane / CPR, pc = lane % CPR;
    const char* src0 = reinterpret_cast<const char*>(t ? a.gsrc[1] : a.gsrc[0]);
#pragma unroll
    for (int i = 0; i < 16 / RPI; ++i) {
      const int row = RPI * i + rr0;
      const int64_t rid = __shfl((long long)r, row, 64);
      const char* src = src0 + (rid >= 0 ? rid : 0) * (IN * 2) + 16 * (pc ^ (row & (CPR - 1)));
      __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)(reinterpret_cast<char*>(xw) + i * 1024), 16, 0, 0);
    }
  } else {
    const int rr0 = lane / CPR, pc = lane % CPR;
#pragma unroll
    for (int i = 0; i < 16 / RPI; ++i) {
      const int row = RPI * i + rr0;
      const int64_t rid = __shfl((long long)r, row, 64);
      const float* src = tab + (rid >= 0 ? rid : 0) * rstride + 4 * (pc ^ row);
      if (!TDBG(32))  // EXPERIMENT (timing only, garbage rows): no row gather
        __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)(xw + i * 256), 16, 0, 0);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // the classic step's insert of this batch's lookups (T1 with a dedup workspace): the claiming
  // CAS now, the deferred finish at the end (lane q == 0 of each row)
  DdPend pend;
  pend.key = DD_EMPTY;
  const int32_t li = (int32_t)(t * B + m);
  if (!UPD && a.dd_on && q == 0 && live) {
    const uint64_t key = r >= 0 ? (((uint64_t)(t ? a.dd_table[1] : a.dd_table[0]) << DD_TABLE_SHIFT) | (uint64_t)r)
                                : DD_EMPTY;
    dd_insert_begin(a.dd, key, li, pend);
  }
  RK_STAMP(1);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the rows (LDS-DMA) and the image registers
  RK_STAMP(2);
#pragma unroll
  for (int k = 0; k < RK_IMG / 1024 / 4; ++k)
    *reinterpret_cast<bf16x8*>(wimg + (wid + 4 * k) * 1024 + lane * 16) = wreg[k];
  __syncthreads();
  RK_STAMP(3);
  // this lane's row in the B layout: xv[mt] = features 32 (mt >> 1) + 8 q + 4 (mt & 1) .. + 3 (fp32)
  f32x4 xv[8];
  bf16x8 xb[4];
  if (IDX) {  // the bf16 B operand straight from the returned rows
#pragma unroll
    for (int s2 = 0; s2 < NI; ++s2) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(xw) + n * (IN * 2) +
                                                         16 * ((4 * s2 + q) ^ (n & (CPR - 1))));
      xb[s2] = r >= 0 ? v : (bf16x8)(__bf16)0.f;
    }
  } else {
#pragma unroll
    for (int mt = 0; mt < MTI; ++mt) {
      const int c = 8 * (mt >> 1) + 2 * q + (mt & 1);
      const f32x4 v = *reinterpret_cast<const f32x4*>(xw + n * IN + 4 * (c ^ n));
      xv[mt] = r >= 0 ? v : (f32x4)(0.f);
    }
#pragma unroll
    for (int s2 = 0; s2 < NI; ++s2) xb[s2] = rk_pack(xv[2 * s2], xv[2 * s2 + 1]);
  }
  // UPD, past barrier 1 (nothing waits on these until the row update; the claim landed with the id,
  // so neither waits for a round trip here): the slot word (its low half holds the lookup count:
  // DD_CNT_BITS < 32, little-endian) and the row's state — unconditional loads at clamped indices
  // (a branch around a load pulls its first use, and the wait for it, into the branch); the state
  // is used only for a single-lookup row. Issued before the row DMA, the two random loads held the
  // DMA's issue back 1.4 us (profiles/r05_t1_claim_ab.log)
  uint32_t word = 0u;
  float s_old = 0.f;
  if (UPD) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the table's hot-row count for the tail (dd_update_block)
      const int32_t nh = a.dd.ctr[0];
      a.dd.ctr[2] = nh;
      a.dd.ctr[0] = 0;
    }
    word = reinterpret_cast<const uint32_t*>(&a.dd.slots[cl >= 0 ? cl : 0].word)[0];
    s_old = (t ? a.us[1] : a.us[0])[r >= 0 ? r : 0];
  }
  __builtin_amdgcn_sched_barrier(0);
  const char* img0 = wimg + t * RK_IMG_T;
  const char* img1 = img0 + RK_W0 * 256;
  // ---- 1. layer 0: h^T = relu(W0 X^T + b0), 8 M-tiles x 4 k-steps
  f32x4 acc[8];
  // the T1 -> T2 strip of X (row-major), fire-and-forget: issued before the layer's MFMAs so the
  // stores drain under them (likewise h's after layer 0, the dZ strips before dX)
  if (!TDBG(512)) rk_strip<NI>(xb, a.xt + (int64_t)t * a.in_max * a.Bp + m * a.in_max, q);  // (TDBG: timing only)
  rk_gemm<8, NI, false>(acc, img0, xb, lane);
  RK_STAMP(4);
  bf16x8 hb[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    f32x4 u0, u1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      u0[j] = fmaxf(acc[2 * s][j] + b0v[2 * s][j], 0.f);
      u1[j] = fmaxf(acc[2 * s + 1][j] + b0v[2 * s + 1][j], 0.f);
    }
    hb[s] = rk_pack(u0, u1);
  }
  if (!TDBG(256)) rk_strip<4>(hb, a.act + ((int64_t)t * MAXL + 0) * MAXW * a.Bp + m * MAXW, q);
  // ---- 2. layer 1: out^T = relu(W1 h^T + b1) (fp32), 4 M-tiles x 4 k-steps; exchanged in LDS
  f32x4 uo[4];
  rk_gemm<4, 4, false>(acc, img1, hb, lane);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) uo[mt] = acc[mt];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int j = 0; j < 4; ++j) uo[mt][j] = fmaxf(uo[mt][j] + b1v[mt][j], 0.f);
    const int c = 8 * (mt >> 1) + 2 * q + (mt & 1);  // 16-B chunk of the 64-float row
    *reinterpret_cast<f32x4*>(&xo[t][h][n * 64 + ((c ^ n) << 2)]) = uo[mt];
  }
  RK_STAMP(5);
  RK_STAMP(6);
  __syncthreads();
  RK_STAMP(7);
  // ---- 3. logit (both towers compute it: the same products in the same order), BCE, dlogit
  f32x4 vo[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int c = 8 * (mt >> 1) + 2 * q + (mt & 1);
    vo[mt] = *reinterpret_cast<const f32x4*>(&xo[t ^ 1][h][n * 64 + ((c ^ n) << 2)]);
  }
  // the summation tree of tower_l2_kernel's logit (bit-identical logits): per group of 4 columns
  // an fma chain from 0, groups g = 16 s' + ... combined at group bits 0 (in lane), 1 (lanes ^ 16),
  // 2 (lanes ^ 32), 3 (in lane); uo[mt] holds group 8 (mt >> 1) + 2 q + (mt & 1)
  float gs[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    float e = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) e = fmaf(uo[mt][j], vo[mt][j], e);
    gs[mt] = e;
  }
  float c0 = gs[0] + gs[1], c1 = gs[2] + gs[3];
  c0 += __shfl_xor(c0, 16, 64);
  c1 += __shfl_xor(c1, 16, 64);
  c0 += __shfl_xor(c0, 32, 64);
  c1 += __shfl_xor(c1, 32, 64);
  const float d = c0 + c1;
  float lo = 0.f, dl = 0.f;
  if (live) {
    const float x = d, y = rk_label(lab_raw, a.label_dtype);
    const float e = __expf(-fabsf(x));
    const float l1p = e < 1e-4f ? e * (1.f - 0.5f * e) : __logf(1.f + e);
    const float lsig = fminf(x, 0.f) - l1p;
    lo = (1.f - y) * x - lsig;
    const float rc = __builtin_amdgcn_rcpf(1.f + e);
    dl = ((x >= 0.f ? rc : e * rc) - y) * (a.grad_scale / (float)B);
  }
  if (t == 0 && q == 0) lrow[16 * h + n] = lo;
  // ---- 4. dZ1 = dlogit * other * (self > 0) (fp32: bias sums; bf16: the next product, the strip)
  float z1[16];
  bf16x8 z1b[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) z1[4 * mt + j] = live && uo[mt][j] > 0.f ? dl * vo[mt][j] : 0.f;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)z1[8 * s + j];
    z1b[s] = v;
  }
  // ---- 5. dZ0^T = (W1^T dZ1^T) * (h > 0): 8 M-tiles x 2 k-steps
  RK_STAMP(8);
  rk_gemm<8, 2, true>(acc, img1, z1b, lane);
  float z0[32];
  bf16x8 z0b[4];
#pragma unroll
  for (int mt = 0; mt < 8; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      z0[4 * mt + j] = live && (float)hb[mt >> 1][4 * (mt & 1) + j] > 0.f ? acc[mt][j] : 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)z0[8 * s + j];
    z0b[s] = v;
  }
  // the dZ strips (T1 -> T2), issued here so they drain beside dX and the row update instead of at
  // the kernel's end
  if (!TDBG(512)) rk_strip<2>(z1b, a.dzt + ((int64_t)t * MAXL + 1) * MAXW * a.Bp + m * MAXW, q);
  if (!TDBG(128)) rk_strip<4>(z0b, a.dzt + ((int64_t)t * MAXL + 0) * MAXW * a.Bp + m * MAXW, q);
  // ---- 6. dX^T = W0^T dZ0^T: 8 M-tiles x 4 k-steps; acc[mt] = dX features of xv[mt]
  RK_STAMP(9);
  rk_gemm<MTI, 4, true>(acc, img0, z0b, lane);
  RK_STAMP(10);
  // ---- 7. the row: UPD + looked up once -> row-wise Adagrad in place (the K3 update's arithmetic and
  // summation tree: feature groups of 4 combined at group bits 4, 3 (in lane), 2, 1 (lanes ^ 32,
  // ^ 16), 0 (in lane)); otherwise dX -> the pooled gradient (and the gathered row, pooled_out)
  float* grow;
  bool store_dx;
  if (IDX) {  // dX -> the requester's gradient row in the send buffer (none for a zero row)
    const int32_t po = (int32_t)pout_raw.lo;
    store_dx = r >= 0 && po >= 0;
    grow = (t ? a.gdst[1] : a.gdst[0]) + (int64_t)(store_dx ? po : 0) * IN;
    if (a.xd.W) grow = reinterpret_cast<float*>(px_row(a.xd, store_dx ? po : 0, IN * 4));
  } else {
    grow = live ? a.gpooled + m * a.ldp + a.s.in_col[t] : nullptr;
    store_dx = live;
  }
  if (UPD) {
    float e2[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      // IN = 64: K3's first level (group bit 4) adds zeros, which is exact: only bit 3 remains
      const float s0 = rw_sq4(acc[0 + hh]), s1 = rw_sq4(acc[2 + hh]);
      float c2;
      if constexpr (IN == 128) {
        const float s2 = rw_sq4(acc[4 + hh]), s3 = rw_sq4(acc[6 + hh]);
        c2 = (s0 + s2) + (s1 + s3);
      } else {
        c2 = s0 + s1;
      }
      c2 += __shfl_xor(c2, 32, 64);
      c2 += __shfl_xor(c2, 16, 64);
      e2[hh] = c2;
    }
    RK_STAMP2(0);
    const float sq = e2[0] + e2[1];
    const float snew = rw_state(s_old, sq, IN);
    const float step = rw_step(snew, a.ulr, a.ueps);
    const uint32_t cnt = word & (uint32_t)DD_CNT_MASK;
    const bool single = r >= 0 && cl >= 0 && cnt == 1u;
    {
      // this wave's rows looked up 2..DD_INL times (their claiming lookups): the tail's list role
      // updates them (segment = the wave; plain stores, the count written every step)
      const bool mul = q == 0 && r >= 0 && cl >= 0 && cnt >= 2u && cnt <= (uint32_t)DD_INL;
      const uint64_t bal = __ballot(mul);
      const int seg = tile * 4 + wid;
      if (seg < a.dd.nseg) {  // [count, slots...] (DD_SEGW): the list role reads count + 3 slots at once
        if (mul) a.dd.multi[(int64_t)seg * DD_SEGW + 1 + __popcll(bal & ((1ull << lane) - 1))] = cl;
        if (lane == 0) a.dd.multi[(int64_t)seg * DD_SEGW] = __popcll(bal);
      }
    }
    // the updated rows go back through the wave's LDS rows (same chunk swizzle) and out as two
    // whole rows per store instruction, as they came in
#pragma unroll
    for (int mt = 0; mt < MTI; ++mt) {
      const int c = 8 * (mt >> 1) + 2 * q + (mt & 1);
      *reinterpret_cast<f32x4*>(xw + n * IN + 4 * (c ^ n)) = rw_apply(xv[mt], acc[mt], step);
    }
    RK_STAMP2(1);
    asm volatile("" ::: "memory");  // LDS is in order per wave: only the compiler must not reorder
    {
      const int rr0 = lane / CPR, pc = lane % CPR;
      float* wtab = t ? a.uw[1] : a.uw[0];
#pragma unroll
      for (int i = 0; i < 16 / RPI; ++i) {
        const int row = RPI * i + rr0;
        const int64_t rid = __shfl((long long)r, row, 64);
        const int sg = __shfl((int)single, row, 64);
        const f32x4 w = *reinterpret_cast<const f32x4*>(xw + row * IN + 4 * pc);
        if (sg) *reinterpret_cast<f32x4*>(wtab + rid * IN + 4 * (pc ^ row)) = w;
      }
    }
    RK_STAMP2(2);
    if (single) {
      if (q == 0) {
        (t ? a.us[1] : a.us[0])[r] = snew;
        a.dd.slots[cl].word = DD_EMPTY;  // free: nothing else of the step reads a single slot
      }
      store_dx = a.pooled_out != nullptr;  // dX only for inspection
    }
  }
  if (store_dx) {
#pragma unroll
    for (int mt = 0; mt < MTI; ++mt)
      *reinterpret_cast<f32x4*>(grow + 32 * (mt >> 1) + 8 * q + 4 * (mt & 1)) = acc[mt];
  }
  RK_STAMP2(3);
  if (t == 0 && q == 0 && live) a.logits[m] = d;  // after the row update (see rk_strip)
  if (!IDX && !POOL && a.pooled_out && live) {
    float* prow = a.pooled_out + m * a.ldp + a.s.in_col[t];
#pragma unroll
    for (int mt = 0; mt < MTI; ++mt) *reinterpret_cast<f32x4*>(prow + 32 * (mt >> 1) + 8 * q + 4 * (mt & 1)) = xv[mt];
  }
  RK_STAMP(11);
  // ---- 8. bias partials (fp32 column sums over the wave's rows, then row half 0 +
  // row half 1); the loss partial (the tile's 32 row losses in order)
  RK_STAMP(12);
  rk_colsum<32>(z0, n);  // lane n: k = 2 n + i, i < 2 (k = 4 mt + j)
  rk_colsum<16>(z1, n);  // lane n: k = n
  // feature of value k = 4 mt + j: 32 (mt >> 1) + 8 q + 4 (mt & 1) + j
  auto feat = [&](int k) { return 32 * ((k >> 2) >> 1) + 8 * q + 4 * ((k >> 2) & 1) + (k & 3); };
  if (h == 1) {
    bsum[t][feat(2 * n)] = z0[0];
    bsum[t][feat(2 * n + 1)] = z0[1];
    bsum[t][RK_W0 + feat(n)] = z1[0];
  }
  RK_STAMP(13);
  __syncthreads();
  RK_STAMP(14);
  if (h == 0) {
    float* db0 = a.dbpart + (((int64_t)t * MAXL + 0) * a.nwg + tile) * MAXW;  // by tile: T2 sums them in tile order
    float* db1 = a.dbpart + (((int64_t)t * MAXL + 1) * a.nwg + tile) * MAXW;
    db0[feat(2 * n)] = z0[0] + bsum[t][feat(2 * n)];
    db0[feat(2 * n + 1)] = z0[1] + bsum[t][feat(2 * n + 1)];
    db1[feat(n)] = z1[0] + bsum[t][RK_W0 + feat(n)];
    if (t == 0 && lane == 0) {
      float p = 0.f;
      for (int i = 0; i < TR; ++i) p += lrow[i];
      a.loss_part[tile] = p;
    }
  }
  // every row's overflow entry is written (EMPTY for a dropped id or a dead row of a ragged tile):
  // the resolver reads all 64 entries of the group
  if (!UPD && a.dd_on && q == 0) dd_insert_defer_finish_at(a.dd, pend, li, tile, 16 * wid + n);
  if constexpr (IDX) {
    if (cpd) *cpd = cpv;
    if (a.xd.W) {  // a share past 256 units (not at the sharded steps' sizes)
      for (int64_t u = (int64_t)blockIdx.x * cp_per + threadIdx.x + 256; u < cp_end; u += 256) {
        const uint4* s2;
        uint4* d2;
        if (px_copy_unit(a.xd, u, s2, d2)) *d2 = *s2;
      }
    }
    // the exchange's epoch advances with its producer (a consumer that signals / waits in-launch
    // reads it after this kernel's boundary)
    if (a.xd.epoch && blockIdx.x == 0 && threadIdx.x == 0)
      __hip_atomic_fetch_add(a.xd.epoch, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  RK_STAMP(15);
}
template <bool UPD, bool IDX = false, int IN = 128, bool POOL = false>
__global__ void __launch_bounds__(256) tower_rows_kernel(TowerArgs a) {
  tower_rows_body<UPD, IDX, IN, POOL>(a);
}

// ---------------------------------------------------------------------------------------------
// T2: dW_(t,l)[n][k] = sum_m dZ_(t,l)[m][n] * A_(t,l)[m][k], A = X (l=0) or act_(t,l-1)

struct WgradTile {
  int32_t t, l, n0, k0;
};


struct WgradArgs {
  const __bf16* xt;
  const __bf16* act;
  const __bf16* dzt;
  float* slab;  // [S][P]
  int64_t P;
  int64_t B;
  int64_t in_max;
  int64_t Bp;      // strip rows per block (strip_at)
  int S;
  int64_t mslice;  // rows per slice (multiple of 32)
  int ntiles;
  int64_t woff[2][MAXL];
  int64_t boff[2][MAXL];
  int32_t K[2][MAXL];  // layer input width
  int32_t width[MAXL];
  int L;
  const float* dbpart;
  int nwg;
  const float* loss_part;  // [nwg] T1 partials
  float* loss;             // nullable
  int nbias;
  int64_t tiles_off;       // byte offset of the tile list in the workspace (host side)
  // Adam's per-step scalars for the T3 that follows (nullable): t = ++step_state[0];
  // adam_pre = {lr / (1 - beta1^t), sqrt(1 - beta2^t)} — one thread, once, instead of every T3
  // thread evaluating pow() and an arrival ticket advancing the counter
  int64_t* step_state;
  float* adam_pre;
  float lr, beta1, beta2;
  // staged path (every K <= 128): tiles of T2_NT dW rows x the whole K, (t, l, n0) per tile
  int lds;
  int rm;  // row-major operand strips ([Bp][features], the row-owned T1's shape): wgrad_lds_block_rm
  int32_t t2_code[16];  // t | l << 4 | n0 << 8
#if TT_EXPERIMENTS
  int64_t* stamps;      // EXPERIMENT (TT_T2_STAMPS): [workgroups][8] s_memrealtime per phase
#endif
  DedupWs dd;           // tt_tower_wgrad_pre with a dedup workspace: the first n_res workgroups
  int n_res;            //   finish T1's deferred inserts (dd_resolve_block)
};

#if TT_EXPERIMENTS
#define T2_STAMP(k) \
  do { if (a.stamps && threadIdx.x == 0) a.stamps[(int64_t)blockIdx.x * 8 + (k)] = (int64_t)__builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define T2_STAMP(k) do { } while (0)
#endif

// staged T2 (wgrad_lds_block): a workgroup owns T2_NT rows x all K columns of one dW over a batch
// slice. The slice is read in passes of T2_PF chunks of T2_MB rows; ALL loads of a pass are issued
// up front (T2_PF x 3 x 16 B per thread in flight: one memory latency per pass, not one per chunk),
// then each chunk (T2_NT rows of dZ^T + K rows of A^T, bf16) goes through LDS (double-buffered, one
// barrier per chunk) where the 4 waves share it
constexpr int T2_NT = 64;
constexpr int T2_MB = 32;                              // batch rows per staged chunk (one k-step)
constexpr int T2_PF = 8;                               // chunks per pass (256 rows)
constexpr int T2_STR = T2_MB + 8;                      // bf16 LDS row stride (80 B: conflict-free b128)
constexpr int T2_ROWS = T2_NT + MAXW;                  // Z rows [0, 64) + A rows [64, 64 + K)
constexpr int T2_LDS = 2 * T2_ROWS * T2_STR * 2;       // bytes (30,720)
constexpr int T2_RED = 3 * 64 * 16 * 4;                // bytes of the register-path reduction
constexpr int T2_SMEM0 = T2_LDS > T2_RED ? T2_LDS : T2_RED;
constexpr int T2_SMEM = T2_SMEM0 > DD_SMEM ? T2_SMEM0 : DD_SMEM;  // the combined launch shares it with dedup.h


__device__ __forceinline__ void wgrad_lds_block(const WgradArgs& a, int lb, char* smem) {
  __bf16* buf = reinterpret_cast<__bf16*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  // lb is workgroup-uniform: readfirstlane keeps the tile lookup a scalar kernarg load (a VGPR index
  // would be a vector load from the kernarg segment, a dependent hop before the first operand load)
  const int s = __builtin_amdgcn_readfirstlane(lb / a.ntiles), ti = __builtin_amdgcn_readfirstlane(lb % a.ntiles);
  T2_STAMP(0);
  const int code = a.t2_code[ti];
  const int t = code & 15, l = (code >> 4) & 15, n0 = code >> 8;
  const int K = a.K[t][l];
  const int NT = min(T2_NT, a.width[l] - n0);  // 64, or 32 for the last tile of a width % 64 layer
  const int64_t B = a.B;
  const __bf16* Z = a.dzt + ((int64_t)t * MAXL + l) * MAXW * a.Bp;  // strip blocks (strip_at)
  const __bf16* A = l == 0 ? a.xt + (int64_t)t * a.in_max * a.Bp : a.act + ((int64_t)t * MAXL + l - 1) * MAXW * a.Bp;
  const int64_t anf = l == 0 ? a.in_max : MAXW;
  const int64_t mb = (int64_t)s * a.mslice;
  const int64_t me = min(mb + a.mslice, B);
  // loader: 4 threads per 64-B operand row segment (32 batch rows), 64 rows per pass; row i's
  // chunk at batch row m (a multiple of 32) starts at src[i] + (m / 32) * tstr[i]
  const int seg = (tid & 3) * 8, frow = tid >> 2;
  const __bf16* src[3];
  int64_t tstr[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int f = frow + 64 * i;
    src[i] = f < T2_NT ? (f < NT ? Z + ((int64_t)(n0 + f) << 5) : nullptr)
                       : (f - T2_NT < K ? A + ((int64_t)(f - T2_NT) << 5) : nullptr);
    tstr[i] = (f < T2_NT ? (int64_t)MAXW : anf) << 5;
  }
  const int nh = wid >> 1, kh = wid & 1;  // wave: dW rows [32 nh, +32) x columns [64 kh, +64)
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4)(0.f);
  for (int64_t p0 = mb; p0 < me; p0 += T2_PF * T2_MB) {
    bf16x8 ld[T2_PF][3];
#pragma unroll
    for (int c = 0; c < T2_PF; ++c) {
      const int64_t m = p0 + c * T2_MB + seg;  // B % 8 == 0: a segment is wholly in or out
#pragma unroll
      for (int i = 0; i < 3; ++i)
        ld[c][i] = (src[i] && m < me) ? *reinterpret_cast<const bf16x8*>(src[i] + (m >> 5) * tstr[i] + seg)
                                      : (bf16x8)(__bf16)0.f;
    }
#pragma unroll
    for (int c = 0; c < T2_PF; ++c) {
      if (p0 + c * T2_MB >= me) break;  // uniform: the slice's tail
      __bf16* d = buf + (c & 1) * T2_ROWS * T2_STR;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (src[i]) *reinterpret_cast<bf16x8*>(d + (frow + 64 * i) * T2_STR + seg) = ld[c][i];
      __syncthreads();  // one barrier per chunk: buffer c & 1 was last read two chunks ago
      if (c == 0 && p0 == mb) T2_STAMP(1);
      bf16x8 fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(d + (nh * 32 + i * 16 + r) * T2_STR + q * 8);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(d + (T2_NT + kh * 64 + j * 16 + r) * T2_STR + q * 8);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (nh * 32 + i * 16 < NT && kh * 64 + j * 16 < K)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  T2_STAMP(2);
  // C[n][k]: row n = 4q + rr, column k = r of each 16 x 16 block
  float* dst = a.slab + (int64_t)s * a.P + a.woff[t][l];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (nh * 32 + i * 16 < NT && kh * 64 + j * 16 < K)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int n = n0 + nh * 32 + i * 16 + q * 4 + rr;
          const int k = kh * 64 + j * 16 + r;
          dst[(int64_t)n * K + k] = acc[i][j][rr];
        }
  T2_STAMP(3);
}

// staged T2 over ROW-MAJOR operand strips ([Bp][features] bf16: what the row-owned T1 and the
// fixed-shape tower_l2_kernel write for the [128, 64] towers over 128-wide inputs): a chunk of 32 batch
// rows x [T2_NT dZ features | K layer-input features] goes to LDS as 32 rows at a 416-B stride
// (whole 16-B pieces of rows, three loads per thread as in wgrad_lds_block), and the fragments are
// transposed reads (ds_read_b64_tr_b16). K-slot (q, j) of every fragment is chunk row
// 4 q + (j & 3) + 16 (j >> 2): the 32 lanes of a read then address 8 consecutive rows, which the
// 416-B stride (= 160 mod 256) spreads over all 64 banks
constexpr int T2R_STR = 208;  // bf16 per LDS row
static_assert(2 * TR * T2R_STR * 2 <= T2_SMEM, "the row-major staged chunks fit the tail's LDS");
__device__ __forceinline__ bf16x8 t2r_frag(const __bf16* d, int col0, int lane) {
  const int q = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
  const __bf16* base = d + (4 * q + qq) * T2R_STR + col0 + 4 * p;
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)base);
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + 16 * T2R_STR));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ void wgrad_lds_block_rm(const WgradArgs& a, int lb, char* smem) {
  __bf16* buf = reinterpret_cast<__bf16*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int s = __builtin_amdgcn_readfirstlane(lb / a.ntiles), ti = __builtin_amdgcn_readfirstlane(lb % a.ntiles);
  T2_STAMP(0);
  const int code = a.t2_code[ti];
  const int t = code & 15, l = (code >> 4) & 15, n0 = code >> 8;
  const int K = a.K[t][l];
  const int NT = min(T2_NT, a.width[l] - n0);
  const int64_t B = a.B;
  const __bf16* Z = a.dzt + ((int64_t)t * MAXL + l) * MAXW * a.Bp;  // [Bp][MAXW]
  const __bf16* A = l == 0 ? a.xt + (int64_t)t * a.in_max * a.Bp : a.act + ((int64_t)t * MAXL + l - 1) * MAXW * a.Bp;
  const int64_t anf = l == 0 ? a.in_max : MAXW;
  const int64_t mb = (int64_t)s * a.mslice;
  const int64_t me = min(mb + a.mslice, B);
  // loader: piece 0 = dZ row tid >> 3, features n0 + 8 (tid & 7); pieces 1, 2 = layer-input row
  // idx >> 4, features 8 (idx & 15), idx = tid + 256 (i - 1); LDS column of a piece: dZ at 0, layer
  // input at T2_NT. Uniform block bases + 32-bit per-thread byte offsets (one address VGPR per load
  // of the 24 in flight: the tail kernel's roles share its register allocation)
  const char* zb = reinterpret_cast<const char*>(Z);
  const char* ab = reinterpret_cast<const char*>(A);
  const int prow0 = tid >> 3, prow1 = tid >> 4, prow2 = (tid + 256) >> 4;
  const bool ok0 = 8 * (tid & 7) < NT, ok1 = 8 * (tid & 15) < K, ok2 = 8 * ((tid + 256) & 15) < K;
  const uint32_t zstr = MAXW * 2, astr = (uint32_t)anf * 2;  // bytes per strip row
  const uint32_t zo = (uint32_t)(mb + prow0) * zstr + (uint32_t)(n0 + 8 * (tid & 7)) * 2;
  const uint32_t ao1 = (uint32_t)(mb + prow1) * astr + (uint32_t)(8 * (tid & 15)) * 2;
  const uint32_t ao2 = (uint32_t)(mb + prow2) * astr + (uint32_t)(8 * ((tid + 256) & 15)) * 2;
  const int lw0 = prow0 * T2R_STR + 8 * (tid & 7);
  const int lw1 = prow1 * T2R_STR + T2_NT + 8 * (tid & 15);
  const int lw2 = prow2 * T2R_STR + T2_NT + 8 * ((tid + 256) & 15);
  const int nh = wid >> 1, kh = wid & 1;  // wave: dW rows [32 nh, +32) x columns [64 kh, +64)
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4)(0.f);
  for (int64_t p0 = mb; p0 < me; p0 += T2_PF * T2_MB) {
    bf16x8 ld[T2_PF][3];
    const uint32_t dr = (uint32_t)(p0 - mb);  // rows into the slice
    // every load unconditional (an invalid piece reads the slice's first row and is zeroed after):
    // loads behind branches make the compiler wait for ALL of them (vmcnt(0)) before chunk 0's
    // LDS write; straight-line loads let chunk c wait for its own three only
    bool okc[T2_PF][3];
#pragma unroll
    for (int c = 0; c < T2_PF; ++c) {
      const uint32_t rc = dr + c * T2_MB;
      const int64_t mrow = p0 + c * T2_MB;
      okc[c][0] = ok0 && mrow + prow0 < me;
      okc[c][1] = ok1 && mrow + prow1 < me;
      okc[c][2] = ok2 && mrow + prow2 < me;
      ld[c][0] = *reinterpret_cast<const bf16x8*>(zb + zo + (okc[c][0] ? rc * zstr : 0u));
      ld[c][1] = *reinterpret_cast<const bf16x8*>(ab + ao1 + (okc[c][1] ? rc * astr : 0u));
      ld[c][2] = *reinterpret_cast<const bf16x8*>(ab + ao2 + (okc[c][2] ? rc * astr : 0u));
    }
#pragma unroll
    for (int c = 0; c < T2_PF; ++c) {
      if (p0 + c * T2_MB >= me) break;  // uniform: the slice's tail
      __bf16* d = buf + (c & 1) * TR * T2R_STR;
      // pieces outside the tile's features land in LDS columns no fragment of this tile reads
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (!okc[c][i]) ld[c][i] = (bf16x8)(__bf16)0.f;
      *reinterpret_cast<bf16x8*>(d + lw0) = ld[c][0];
      *reinterpret_cast<bf16x8*>(d + lw1) = ld[c][1];
      *reinterpret_cast<bf16x8*>(d + lw2) = ld[c][2];
      __syncthreads();  // one barrier per chunk: buffer c & 1 was last read two chunks ago
      if (c == 0 && p0 == mb) T2_STAMP(1);
      bf16x8 fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = t2r_frag(d, nh * 32 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = t2r_frag(d, T2_NT + kh * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (nh * 32 + i * 16 < NT && kh * 64 + j * 16 < K)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  T2_STAMP(2);
  float* dst = a.slab + (int64_t)s * a.P + a.woff[t][l];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (nh * 32 + i * 16 < NT && kh * 64 + j * 16 < K)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int n = n0 + nh * 32 + i * 16 + q * 4 + rr;
          const int k = kh * 64 + j * 16 + r;
          dst[(int64_t)n * K + k] = acc[i][j][rr];
        }
  T2_STAMP(3);
}

__device__ __forceinline__ void wgrad_block(const WgradArgs& a, const WgradTile* __restrict__ tiles, int bid,
                                            char* smem) {
  // workgroups [0, ntiles * S): one (32x32 tile of dW, batch slice) each, its 4 waves on 4
  // consecutive quarters of the slice, reduced through LDS in wave order -> one slab row.
  // Workgroups beyond: one wave per bias output (+ one for the loss).
  float (*red)[64 * 16] = reinterpret_cast<float (*)[64 * 16]>(smem);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int64_t nwg_tiles = (int64_t)a.ntiles * a.S;
  if ((int64_t)bid >= nwg_tiles) {
    T2_STAMP(0);
    // bias gradient of one output n of (t, l): sum of the T1 workgroups' partials, lanes strided
    // over workgroups, then a fixed butterfly -> slab[0]
    int64_t b = ((int64_t)bid - nwg_tiles) * 4 + wid;
    if (b == a.nbias) {  // the scalar loss: T1's per-workgroup partials in a fixed order
      b = -1;            // (no bias output below)
      if (a.loss) {
        float s = 0.f;
        for (int w0 = 0; w0 < a.nwg; w0 += 512) {
          float v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = w0 + k * 64 + lane < a.nwg ? a.loss_part[w0 + k * 64 + lane] : 0.f;
#pragma unroll
          for (int k = 0; k < 8; ++k) s += v[k];
        }
        s = wave_sum(s);
        if (lane == 0) a.loss[0] = s / (float)a.B;
      }
      if (a.adam_pre && lane == 0) {
        const int64_t t_step = a.step_state[0] + 1;
        a.step_state[0] = t_step;
        const double bc1 = 1.0 - pow((double)a.beta1, (double)t_step);
        const double bc2 = 1.0 - pow((double)a.beta2, (double)t_step);
        a.adam_pre[0] = (float)((double)a.lr / bc1);
        a.adam_pre[1] = (float)sqrt(bc2);
      }
    }
    for (int t = 0; t < 2; ++t)
      for (int l = 0; l < a.L; ++l) {
        if (b >= 0 && b < a.width[l]) {
          const float* dbp = a.dbpart + ((int64_t)t * MAXL + l) * a.nwg * MAXW + b;
          // 8 independent loads per lane in flight per round (not one dependent load per add)
          float s = 0.f;
          for (int w0 = 0; w0 < a.nwg; w0 += 512) {
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const int w = w0 + k * 64 + lane;
              v[k] = w < a.nwg ? dbp[(int64_t)w * MAXW] : 0.f;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) s += v[k];
          }
          s = wave_sum(s);
          if (lane == 0) a.slab[a.boff[t][l] + b] = s;
        }
        if (b >= 0) b -= a.width[l];
      }
    T2_STAMP(3);
    return;
  }
  // XCD-aware placement: a contiguous 1/8 of the (slice, tile) list — whole slices, whose tiles
  // re-read the same operand strips — on one XCD and its L2
  const int lb = xcd_remap(bid, (int)nwg_tiles);
  if (a.lds && a.rm) {
    wgrad_lds_block_rm(a, lb, smem);
    return;
  }
  if (a.lds) {
    wgrad_lds_block(a, lb, smem);
    return;
  }
  const int s = (int)(lb / a.ntiles);
  const WgradTile tl = tiles[lb % a.ntiles];
  const int64_t B = a.B;
  const __bf16* Z = a.dzt + ((int64_t)tl.t * MAXL + tl.l) * MAXW * a.Bp;  // strip blocks (strip_at)
  const __bf16* A = tl.l == 0 ? a.xt + (int64_t)tl.t * a.in_max * a.Bp
                              : a.act + ((int64_t)tl.t * MAXL + tl.l - 1) * MAXW * a.Bp;
  const int64_t anf = tl.l == 0 ? a.in_max : MAXW;
  const int64_t mw = a.mslice / 4;
  int64_t mb = (int64_t)s * a.mslice + wid * mw;
  int64_t me = mb + mw;
  if (mb > B) mb = B;
  if (me > B) me = B;
  f32x4 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4)(0.f);
  // feature row bases in the tile-major strips; batch row o of a row: + (o / 32) * nf * 32 + o % 32
  const __bf16* z0 = Z + ((int64_t)(tl.n0 + r) << 5);
  const __bf16* z1 = Z + ((int64_t)(tl.n0 + 16 + r) << 5);
  const __bf16* a0 = A + ((int64_t)(tl.k0 + r) << 5);
  const __bf16* a1 = A + ((int64_t)(tl.k0 + 16 + r) << 5);
  auto zo = [&](int64_t o) { return (((o >> 5) * MAXW) << 5) + (o & 31); };
  auto ao = [&](int64_t o) { return (((o >> 5) * anf) << 5) + (o & 31); };
  int64_t m = mb;
  // 4 k-steps per iteration: their 16 fragment loads are issued before the first MFMA
  for (; m + 128 <= me; m += 128) {
    bf16x8 fa0[4], fa1[4], fb0[4], fb1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t o = m + 32 * u + q * 8;
      fa0[u] = *reinterpret_cast<const bf16x8*>(z0 + zo(o));
      fa1[u] = *reinterpret_cast<const bf16x8*>(z1 + zo(o));
      fb0[u] = *reinterpret_cast<const bf16x8*>(a0 + ao(o));
      fb1[u] = *reinterpret_cast<const bf16x8*>(a1 + ao(o));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0[u], fb0[u], acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0[u], fb1[u], acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[u], fb0[u], acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[u], fb1[u], acc[1][1], 0, 0, 0);
    }
  }
  for (; m + 32 <= me; m += 32) {
    const int64_t o = m + q * 8;
    const bf16x8 fa0 = *reinterpret_cast<const bf16x8*>(z0 + zo(o));
    const bf16x8 fa1 = *reinterpret_cast<const bf16x8*>(z1 + zo(o));
    const bf16x8 fb0 = *reinterpret_cast<const bf16x8*>(a0 + ao(o));
    const bf16x8 fb1 = *reinterpret_cast<const bf16x8*>(a1 + ao(o));
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0, fb0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0, fb1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1, fb0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1, fb1, acc[1][1], 0, 0, 0);
  }
  if (m < me) {  // ragged tail (B % 32 != 0): zero-padded fragments
    bf16x8 fa0, fa1, fb0, fb1;
    for (int j = 0; j < 8; ++j) {
      const int64_t mm = m + q * 8 + j;
      const bool ok = mm < me;
      fa0[j] = ok ? z0[zo(mm)] : (__bf16)0.f;
      fa1[j] = ok ? z1[zo(mm)] : (__bf16)0.f;
      fb0[j] = ok ? a0[ao(mm)] : (__bf16)0.f;
      fb1[j] = ok ? a1[ao(mm)] : (__bf16)0.f;
    }
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0, fb0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0, fb1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1, fb0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1, fb1, acc[1][1], 0, 0, 0);
  }
  // fixed-order reduction of the 4 waves' tiles: wave 0 adds waves 1, 2, 3 in that order
  if (wid > 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) red[wid - 1][((i * 2 + j) * 4 + rr) * 64 + lane] = acc[i][j][rr];
  }
  __syncthreads();
  if (wid > 0) return;
#pragma unroll
  for (int w = 0; w < 3; ++w)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[i][j][rr] += red[w][((i * 2 + j) * 4 + rr) * 64 + lane];
  // C[n][k]: row = n (4q + rr), col = k (r)
  const int K = a.K[tl.t][tl.l];
  float* dst = a.slab + (int64_t)s * a.P + a.woff[tl.t][tl.l];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int rr = 0; rr < 4; ++rr) {
        const int n = tl.n0 + i * 16 + q * 4 + rr;
        const int k = tl.k0 + j * 16 + r;
        dst[(int64_t)n * K + k] = acc[i][j][rr];
      }
}

__global__ void __launch_bounds__(256) tower_wgrad_kernel(WgradArgs a, const WgradTile* __restrict__ tiles) {
  __shared__ __attribute__((aligned(16))) char smem[T2_SMEM];
  // resolver workgroups first (their probe chains are the longest dependent work of the launch);
  // n_res % 8 == 0 keeps the tiles' XCD placement
  if ((int)blockIdx.x < a.n_res)
    dd_resolve_block(a.dd, (int)blockIdx.x, a.n_res);
  else
    wgrad_block(a, tiles, (int)blockIdx.x - a.n_res, smem);
}

// T2 + the embedding path's fused row-wise Adagrad (dedup.h) in ONE launch: workgroups
// [0, n_t2) are T2's, the rest run dd_update_block. Both read only what T1 wrote, so one launch
// boundary (and no cross-stream join) separates them from T1, and the MFMA/L2-bound tiles overlap
// the HBM-bound row updates on the same CUs.
__global__ void __launch_bounds__(256) tower_wgrad_dedup_kernel(WgradArgs a, const WgradTile* __restrict__ tiles,
                                                                DdUpdateArgs d, int n_t2) {
  __shared__ __attribute__((aligned(16))) char smem[T2_SMEM];
  if ((int)blockIdx.x < n_t2)
    wgrad_block(a, tiles, (int)blockIdx.x, smem);
  else
    dd_update_block(d, (int)blockIdx.x - n_t2, smem);
}

// Pipelined fused step: T2 with the NEXT batch's dedup insert as extra workgroups (one wave per
// 64 lookups i = t * B + m: one returning CAS each, lookups that lost it deferred to the next
// launch's resolver), so T1 of the next step finds a complete table and updates the rows looked up
// once in place (tower_l2_kernel<..., UPD>).
struct InsertArgs {
  const void* col[2];
  int64_t mod[2];
  int32_t tab[2];
  int id_dtype;
  int64_t B;
  DedupWs dd;
  int xcd_wpt;  // > 0: insert_next_full_block files by T1 tile class (ins_lookup), this many workgroups
                // per (XCD class, tower); 0: 256 consecutive lookups per workgroup
};
// lookup of thread tid in insert workgroup blk (blk < 2B / 256). xcd_wpt > 0 (B % 2048 == 0): the
// workgroup takes only rows of the T1 tiles (32 rows each) that run on its own XCD (blk % 8): T1
// places tiles [c B / 256, (c + 1) B / 256) on XCD c (xcd_remap), so the next batch's ids and the
// claims T1 reads first are in that XCD's L2 when its T1 tile starts (plain loads and stores keep
// their lines there). Lookup order is irrelevant to the results: every row's lookups are summed in
// ascending lookup order whatever their slot positions.
__device__ __forceinline__ int64_t ins_lookup(const InsertArgs& ins, int blk, int tid) {
  if (ins.xcd_wpt <= 0) return (int64_t)blk * 256 + tid;
  const int c = blk & 7, j = blk >> 3;
  const int t = j / ins.xcd_wpt, qi = j - t * ins.xcd_wpt;
  // T1 tile b runs on XCD c for b in [c B / 256, (c + 1) B / 256) (tower_rows_body's xcd_remap)
  const int64_t b = (int64_t)c * (ins.B / 256) + 8 * qi + (tid >> 5);
  return (int64_t)t * ins.B + 32 * b + (tid & 31);
}

__device__ __forceinline__ void insert_next_block(const InsertArgs& ins, int blk) {
  const int lane = threadIdx.x & 63;
  const int64_t grp = (int64_t)blk * 4 + (threadIdx.x >> 6);
  const int64_t i = grp * 64 + lane;
  DdPend p;
  p.key = DD_EMPTY;
  if (i < 2 * ins.B) {
    const int t = i >= ins.B;
    const int64_t m = i - (t ? ins.B : 0);
    const int64_t id = load_id(t ? ins.col[1] : ins.col[0], ins.id_dtype, m);
    const uint64_t key = id != 0 ? (((uint64_t)(t ? ins.tab[1] : ins.tab[0]) << DD_TABLE_SHIFT) |
                                    (uint64_t)py_mod64(id, t ? ins.mod[1] : ins.mod[0]))
                                 : DD_EMPTY;
    dd_insert_begin(ins.dd, key, (int32_t)i, p);
  }
  if (grp < ins.dd.ovf_groups) dd_insert_defer_finish(ins.dd, p, (int32_t)(i < 2 * ins.B ? i : 0), (int)grp);
}

// EXPERIMENT (TT_RING_STAMPS): s_memrealtime of wave 0 at the start / end of each workgroup's role
#if TT_EXPERIMENTS
#define RING_STAMP(p, k) \
  do { if ((p) && threadIdx.x == 0 && blockIdx.x < 2048) (p)[(int64_t)blockIdx.x * 2 + (k)] = (int64_t)__builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define RING_STAMP(p, k) do { (void)(p); } while (0)
#endif

__global__ void __launch_bounds__(256) tower_wgrad_insert_kernel(WgradArgs a, const WgradTile* __restrict__ tiles,
                                                                 InsertArgs ins, int n_t2, int64_t* stamps) {
  __shared__ __attribute__((aligned(16))) char smem[T2_SMEM];
  RING_STAMP(stamps, 0);
  if ((int)blockIdx.x < n_t2)
    wgrad_block(a, tiles, (int)blockIdx.x, smem);
  else
    insert_next_block(ins, (int)blockIdx.x - n_t2);
  RING_STAMP(stamps, 1);
}

// Pipelined sharded step, launch U (after exchange A brought the gradient rows of batch i and the
// ids of batch i+1): T2 of batch i (weight-gradient tiles, bias sums, loss) beside the owner's
// row-wise Adagrad of batch i's rows and the count pass of batch i+2's route — all three read only
// what T1 and the exchange wrote, so the tower weight gradients overlap the embedding update.
// n_dd > 0: the owner's update workgroups come FIRST in the grid (they carry the launch's longest
// chain, claim -> slot -> rows -> stores; dispatched behind the T2 tiles, the last of them started
// ~4.5 us late), then the T2 tiles, then the route count
__global__ void __launch_bounds__(256, 3) tower_wgrad_route_rowwise_kernel(WgradArgs a, const WgradTile* __restrict__ tiles,
                                                                        RouteArgs r, DdUpdateArgs d, int n_t2,
                                                                        int n_cnt, int n_dd, PxWait w) {
  __shared__ __attribute__((aligned(16))) char smem[T2_SMEM];
  int b = (int)blockIdx.x;
  if (w.W) {
    // in-launch exchange A: workgroup 0 signals; it and the owner's update workgroups (the only
    // readers of the received blocks) wait — workgroup 0 always, so a rank with no update
    // workgroups still holds launch G back until every peer consumed its exchange-B buffer
    if (b == 0) px_signal(w);
    if (b == 0 || (n_dd > 0 ? b < n_dd : b >= n_t2 + n_cnt)) px_wait(w);
  }
  if (n_dd > 0) {
    if (b < n_dd) {
      dd_update_block(d, b, smem);
      return;
    }
    b -= n_dd;
    if (b >= n_t2 + n_cnt) return;
  }
  if (b < n_t2) {
    wgrad_block(a, tiles, b, smem);
  } else if (b < n_t2 + n_cnt) {
    const int j = b - n_t2;
    route_count_block(r, j % r.nblk, j / r.nblk, reinterpret_cast<int (*)[RT_MAXW]>(smem));
  } else {
    dd_update_block(d, b - n_t2 - n_cnt, smem);
  }
}

__device__ __forceinline__ void update_block(const UpdateArgs& a, int bid, int nblocks) {
  T3_STAMP(0);
  if (a.wt.W) {
    if (bid == 0) px_signal(a.wt);
    px_wait(a.wt);
  }
  const int64_t i = (int64_t)bid * blockDim.x + threadIdx.x;
  int64_t t_step = 0;
  float step_size = 0.f, bc2_sqrt = 1.f;
  if (a.do_adam && a.adam_pre) {
    step_size = a.adam_pre[0];
    bc2_sqrt = a.adam_pre[1];
  } else if (a.do_adam) {
    t_step = a.step_state[0] + 1;
    const double bc1 = 1.0 - pow((double)a.beta1, (double)t_step);
    const double bc2 = 1.0 - pow((double)a.beta2, (double)t_step);
    step_size = (float)((double)a.lr / bc1);
    bc2_sqrt = (float)sqrt(bc2);
  }
  if (i < a.P) {
    const T3Seg sg = t3_seg(a, i);
    const float p = a.params[i];
    const float m = a.do_adam ? a.exp_avg[i] : 0.f, v = a.do_adam ? a.exp_avg_sq[i] : 0.f;
    float g = 0.f;
    if (a.grads_in) {
      g = a.grads_in[i];
      for (int q = 1; q < a.in_srcs; ++q) g += a.grads_in[(int64_t)q * a.in_stride + i];
    } else if (a.do_adam || a.grads_out) {
      if (sg.sisw) {
        // a round's 32 slab loads all in flight (one memory latency per 32 slabs, not per load);
        // the sum keeps the sequential order s = 0, 1, ...
        for (int s0 = 0; s0 < a.S; s0 += 32) {
          float v[32];
#pragma unroll
          for (int u = 0; u < 32; ++u) {
            v[u] = s0 + u < a.S ? a.slab[(int64_t)(s0 + u) * a.P + i] : 0.f;
          }
#pragma unroll
          for (int u = 0; u < 32; ++u)
            if (s0 + u < a.S) g += v[u];
        }
      } else {
        // bias gradient, reduced over the T1 workgroups by T2's bias waves
        g = a.slab[i];
      }
    }
    T3_STAMP(1);
    t3_apply(a, i, sg, p, m, v, g, step_size, bc2_sqrt, a.do_adam);
    T3_STAMP(2);
  }
  if (a.do_adam && !a.adam_pre) {
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned* counter = reinterpret_cast<unsigned*>(a.step_state + 1);
      const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == (unsigned)nblocks - 1) {
        __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.step_state), (unsigned long long)t_step,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// the parameter blocks a contiguous 1/8 per XCD (xcd_remap; every parameter's update is independent
// of its workgroup): -0.45 us a step at the north star against blockIdx order, same box
// (profiles/r06y2_ab_t3_by_xcd.log)
__global__ void __launch_bounds__(256) tower_update_kernel(UpdateArgs a) {
  update_block(a, xcd_remap((int)blockIdx.x, (int)gridDim.x), (int)gridDim.x);
}

// Pipelined sharded step, launch G (after launch U updated this rank's rows): the owner's gather of
// batch i+1's rows (bf16, into exchange B's row blocks, filing batch i+1's dedup table), the tower
// gradient of batch i x 1/W into exchange B's tower block of every destination (slab reduction, no
// Adam), and the place pass of batch i+2's route.
__global__ void __launch_bounds__(256) tower_grads_place_gather_kernel(UpdateArgs a, RouteArgs r, GatherSegArgs g,
                                                                       int n_upd, int n_place) {
  __shared__ int base[RT_MAXW];
  __shared__ int wc[RT_BLOCK / 64][RT_MAXW];
  const int b = (int)blockIdx.x;
  if (g.epoch && b == 0 && threadIdx.x == 0)  // exchange B's epoch advances with its producer
    __hip_atomic_fetch_add(g.epoch, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (b < n_upd) {
    update_block(a, xcd_remap(b, n_upd), n_upd);  // a contiguous 1/8 per XCD, as T3
  } else if (b < n_upd + n_place) {
    const int j = b - n_upd;
    route_place_block<true>(r, j % r.nblk, j / r.nblk, base, wc);
  } else {
    shard_gather_block(g, b - n_upd - n_place);
  }
}

// K3 of the pipelined fused step: resolver workgroups for the NEXT batch's deferred inserts, then
// the update of this batch's rows looked up more than once (skip_single), then T3
constexpr int K3_RES_WGS = 32;
__global__ void __launch_bounds__(256) tower_update_dedup_resolve_kernel(UpdateArgs a, DdUpdateArgs d, DedupWs next,
                                                                         int n_dd, int64_t* stamps) {
  __shared__ __attribute__((aligned(16))) char smem[DD_SMEM];
  const int bid = (int)blockIdx.x;
  RING_STAMP(stamps, 0);
  if (bid < K3_RES_WGS)
    dd_resolve_block(next, bid, K3_RES_WGS);
  else if (bid < K3_RES_WGS + n_dd)
    dd_update_block(d, bid - K3_RES_WGS, smem);
  else
    update_block(a, bid - K3_RES_WGS - n_dd, (int)gridDim.x - K3_RES_WGS - n_dd);
  RING_STAMP(stamps, 1);
}

// The pipelined fused step's backward tail, one launch: T2 (weight gradients, bias sums, loss,
// Adam scalars) + the NEXT batch's complete insert (probing in place: its latency hides behind the
// tiles, so no deferral and no resolver launch) + the update of this batch's rows looked up more
// than once. The three roles read only what T1 (or the previous step) wrote; T3 follows as its own
// launch (it needs every T2 slab: in-launch, that hand-off across the 8 XCDs' L2s cost more than
// the launch boundary it saves — DESIGN.md section 5).
// the NEXT batch's lookups, INS_PT per thread, inserted completely (probing in place). The
// workgroup's repeated keys are merged in LDS first: one leader per key claims or joins the key's
// slot with the group's count in ONE global atomic and hands each member its position (base +
// rank in the group) — at skewed ids a hot row costs one atomic per workgroup, not one per lookup
// (the update sums a row's lookups in lookup order whatever the positions: the same results).
#ifndef TT_INS_PT
#define TT_INS_PT 1
#endif
constexpr int INS_PT = TT_INS_PT;  // lookups per thread (1: 256 per workgroup, 64 workgroups at the
                                   // north star; 2 measured 0.3-0.4 µs slower per step, scripts/r04_inspt.sh)
constexpr int INS_HS = 1024;  // LDS hash slots per 512 lookups
static_assert(INS_HS * (8 + 3 * 4) <= T2_SMEM, "the insert role's LDS hash fits the tail's LDS");
__device__ __forceinline__ void insert_next_full_block(const InsertArgs& ins, int blk, char* smem) {
  unsigned long long* hk = reinterpret_cast<unsigned long long*>(smem);  // [INS_HS] keys
  int* hc = reinterpret_cast<int*>(smem + 8 * INS_HS);                   // [INS_HS] group counts
  int* hb = hc + INS_HS;                                                 // [INS_HS] group base position
  int* hg = hb + INS_HS;                                                 // [INS_HS] global slot
  const DedupWs& ws = ins.dd;
  for (int q = threadIdx.x; q < INS_HS; q += 256) {
    hk[q] = DD_EMPTY;
    hc[q] = 0;
  }
  int64_t iv[INS_PT];
  uint64_t key[INS_PT];
#pragma unroll
  for (int u = 0; u < INS_PT; ++u) {
    const int64_t i = INS_PT == 1 ? ins_lookup(ins, blk, (int)threadIdx.x)
                                  : ((int64_t)blk * INS_PT + u) * 256 + threadIdx.x;
    iv[u] = i;
    key[u] = DD_EMPTY;
    if (i < 2 * ins.B) {
      const int t = i >= ins.B;
      const int64_t m = i - (t ? ins.B : 0);
      const int64_t id = load_id(t ? ins.col[1] : ins.col[0], ins.id_dtype, m);
      if (id != 0)
        key[u] = ((uint64_t)(t ? ins.tab[1] : ins.tab[0]) << DD_TABLE_SHIFT) |
                 (uint64_t)py_mod64(id, t ? ins.mod[1] : ins.mod[0]);
      ws.lkey[i] = key[u];
    }
  }
  __syncthreads();
  int hl[INS_PT], rank[INS_PT];
#pragma unroll
  for (int u = 0; u < INS_PT; ++u) {
    hl[u] = -1;
    rank[u] = 0;
    if (key[u] != DD_EMPTY) {
      unsigned h = (unsigned)dd_mix64(key[u]) & (INS_HS - 1);
      while (true) {
        const unsigned long long prev = atomicCAS(&hk[h], (unsigned long long)DD_EMPTY, (unsigned long long)key[u]);
        if (prev == DD_EMPTY || prev == key[u]) break;
        h = (h + 1) & (INS_HS - 1);
      }
      hl[u] = (int)h;
      rank[u] = atomicAdd(&hc[h], 1);
    }
  }
  __syncthreads();
  // each group's leader: one claiming CAS (with the group's count) or one add of it
  const uint64_t mask = (uint64_t)ws.cap - 1;
#pragma unroll
  for (int u = 0; u < INS_PT; ++u) {
    if (hl[u] >= 0 && rank[u] == 0) {
      const uint64_t c = (uint64_t)hc[hl[u]];
      uint64_t g = dd_mix64(key[u]) & mask;
      int base;
      while (true) {
        unsigned long long* w = reinterpret_cast<unsigned long long*>(&ws.slots[g].word);
        const unsigned long long prev =
            atomicCAS(w, (unsigned long long)DD_EMPTY, (unsigned long long)((key[u] << DD_CNT_BITS) | c));
        if (prev == DD_EMPTY) {
          base = 0;
          break;
        }
        if ((prev >> DD_CNT_BITS) == key[u]) {
          base = (int)(atomicAdd(w, (unsigned long long)c) & DD_CNT_MASK);
          break;
        }
        g = (g + 1) & mask;
      }
      hb[hl[u]] = base;
      hg[hl[u]] = (int)g;
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < INS_PT; ++u) {
    const int64_t i = iv[u];
    if (i >= 2 * ins.B) continue;
    if (hl[u] < 0) {
      ws.claim[i] = -1;
      continue;
    }
    const int k = hb[hl[u]] + rank[u], h = hg[hl[u]];
    ws.claim[i] = k == 0 ? h : -1;
    if (k < DD_INL) {
      ws.slots[h].item[k] = (int32_t)i;
    } else if (k == DD_INL) {
      const int q = atomicAdd(&ws.ctr[0], 1);
      if (q < ws.hot_cap) {
        ws.hot[q] = h;
        ws.hkey[q] = key[u];
      }
    }
  }
}

template <bool LIST>
__global__ void __launch_bounds__(256, 3) tower_tail_kernel(WgradArgs a2, const WgradTile* __restrict__ tiles,
                                                         InsertArgs ins, DdUpdateArgs d, int n_ins, int n_t2,
                                                         int64_t* stamps) {
  __shared__ __attribute__((aligned(16))) char smem[T2_SMEM];
  int b = (int)blockIdx.x;
  RING_STAMP(stamps, 0);
  if (b < n_ins)
    insert_next_full_block(ins, b, smem);
  else if ((b -= n_ins) < n_t2)
    wgrad_block(a2, tiles, b, smem);  // n_ins % 8 == 0: b keeps the XCD placement of wgrad_block
  else
    dd_update_block<LIST>(d, b - n_t2, smem);
  RING_STAMP(stamps, 1);
}

// T3 + the embedding path's fused row-wise Adagrad (dedup.h) in ONE launch: workgroups [0, n_dd)
// run dd_update_block (its slot workgroups fit one round of resident waves), the rest T3 (Adam with
// T2's precomputed scalars). T2 runs alone before it with the registers and LDS it needs.
__global__ void __launch_bounds__(256) tower_update_dedup_kernel(UpdateArgs a, DdUpdateArgs d, int n_dd) {
  __shared__ __attribute__((aligned(16))) char smem[DD_SMEM];
  if ((int)blockIdx.x < n_dd)
    dd_update_block(d, (int)blockIdx.x, smem);
  else
    update_block(a, (int)blockIdx.x - n_dd, (int)gridDim.x - n_dd);
}

// ---------------------------------------------------------------------------------------------

struct TowerLayout {
  int64_t P;         // dense params
  int64_t PW;        // weight elements (bf16 copies)
  int64_t woff[2][MAXL], boff[2][MAXL], wcoff[2][MAXL];
  int32_t K[2][MAXL];
  int64_t in_max;
  int64_t Bp;        // strip rows per block (B rounded up to 32)
  int nwg;
  int S;
  int64_t mslice;
  int ntiles;
  int lds;  // staged T2 (wgrad_lds_block)
  int32_t t2_code[16];
  int rows;  // the row-owned T1 (tower_rows_kernel) serves this shape's single-hot gather launches
  // workspace carve (bytes)
  size_t o_xt, o_act, o_dzt, o_dbpart, o_slab, o_losspart, o_counter, o_wb, o_wtb, o_wbf, o_wtbf, o_wimg, o_tiles, o_dbg, total;
};

static int tower_layout(const tt_tower_shape_t* s, int64_t B, TowerLayout* lay) {
  if (!s) return fail(TT_EINVAL, "tower: null shape");
  if (s->L < 1 || s->L > MAXL) return fail(TT_EINVAL, "tower: 1..4 layers supported");
  if (B < 8 || B % 8) return fail(TT_EINVAL, "tower: B must be a positive multiple of 8");
  if (s->flags & ~TT_TOWER_GENERAL_T1) return fail(TT_EINVAL, "tower: unknown shape flags");
  for (int l = 0; l < s->L; ++l)
    if (s->width[l] < 16 || s->width[l] > MAXW || s->width[l] % 32)
      return fail(TT_EINVAL, "tower: layer widths must be multiples of 32 in [32, 128]");
  for (int t = 0; t < 2; ++t) {
    if (s->in_dim[t] < 32 || s->in_dim[t] > 1024 || s->in_dim[t] % 32)
      return fail(TT_EINVAL, "tower: input widths must be multiples of 32 in [32, 1024]");
    if (s->in_col[t] < 0 || s->in_col[t] % 4) return fail(TT_EINVAL, "tower: input column must be >= 0, % 4 == 0");
  }
  TowerLayout L{};
  int64_t o = 0, w = 0;
  for (int t = 0; t < 2; ++t) {
    int k = s->in_dim[t];
    for (int l = 0; l < s->L; ++l) {
      L.woff[t][l] = o;
      L.wcoff[t][l] = w;
      L.K[t][l] = k;
      o += (int64_t)s->width[l] * k;
      w += (int64_t)s->width[l] * k;
      L.boff[t][l] = o;
      o += s->width[l];
      k = s->width[l];
    }
  }
  L.P = o;
  L.PW = w;
  L.in_max = std::max(s->in_dim[0], s->in_dim[1]);
  L.nwg = (int)ceil_div(B, TR);
  int nt = 0;
  L.lds = L.in_max <= MAXW;
  if (L.lds) {
    // staged T2: tiles of 64 dW rows x all K
    for (int t = 0; t < 2; ++t)
      for (int l = 0; l < s->L; ++l)
        for (int n0 = 0; n0 < s->width[l]; n0 += T2_NT) {
          L.t2_code[nt] = t | l << 4 | n0 << 8;
          ++nt;
        }
    // slices of whole passes (256 rows), at most 64 (the slab depth T3 reduces over)
    const int64_t pass = T2_PF * T2_MB;
    int64_t passes = 1;  // per slice
#if TT_EXPERIMENTS
    if (const char* e = getenv("TT_T2_SLICE_PASSES")) passes = std::max(1, atoi(e));  // EXPERIMENT
#endif
    const int64_t S = std::min<int64_t>(64, ceil_div(B, pass * passes));
    L.mslice = ceil_div(ceil_div(B, S), pass) * pass;
    L.S = (int)ceil_div(B, L.mslice);
  } else {
    for (int t = 0; t < 2; ++t)
      for (int l = 0; l < s->L; ++l) nt += (s->width[l] / 32) * (L.K[t][l] / 32);
    // slices (one T2 workgroup each per tile, 4 waves of mslice/4 rows): aim for ~400 workgroups,
    // >= 512 rows per slice; the slice count is also the slab depth T3 reduces over
    int64_t S = std::max<int64_t>(1, 400 / std::max(1, nt));
    S = std::min<int64_t>(S, std::max<int64_t>(1, ceil_div(B, 512)));
    S = std::min<int64_t>(S, 64);
    L.S = (int)S;
    L.mslice = ceil_div(ceil_div(B, S), 128) * 128;
  }
  L.ntiles = nt;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t r = off;
    off += align_up(bytes, 256);
    return r;
  };
  L.Bp = ceil_div(B, 32) * 32;
  L.o_xt = take(2 * (size_t)L.in_max * L.Bp * 2);
  L.o_act = take(2 * (size_t)MAXL * MAXW * L.Bp * 2);
  L.o_dzt = take(2 * (size_t)MAXL * MAXW * L.Bp * 2);
  L.o_dbpart = take(2 * (size_t)MAXL * L.nwg * MAXW * 4);
  L.o_slab = take((size_t)L.S * L.P * 4);
  L.o_losspart = take((size_t)L.nwg * 4);
  L.o_counter = take(64);
  L.o_wb = take((size_t)L.PW * 2);
  L.o_wtb = take((size_t)L.PW * 2);
  L.o_wbf = take((size_t)L.PW * 2);
  L.o_wtbf = take((size_t)L.PW * 2);
  L.rows = s->L == 2 && s->in_dim[0] == s->in_dim[1] && (s->in_dim[0] == RK_IN || s->in_dim[0] == 64) &&
           s->width[0] == RK_W0 && s->width[1] == RK_W1 && !(s->flags & TT_TOWER_GENERAL_T1);
  L.o_wimg = take(L.rows ? (size_t)RK_IMG : 0);
  L.o_tiles = take((size_t)nt * sizeof(WgradTile));
  L.o_dbg = take((size_t)(std::max<int64_t>(L.nwg * 2, 1024) * 8 + L.nwg * 16 * 9) * sizeof(int64_t));
  L.total = off;
  *lay = L;
  return TT_OK;
}

}  // namespace tt

using namespace tt;

extern "C" {

int64_t tt_tower_num_params(const tt_tower_shape_t* shape) {
  TowerLayout L;
  if (tower_layout(shape, 8, &L)) return -1;
  return L.P;
}

size_t tt_tower_workspace_bytes(const tt_tower_shape_t* shape, int64_t B) {
  TowerLayout L;
  if (tower_layout(shape, B, &L)) return 0;
  return L.total;
}

int tt_tower_workspace_init(const tt_tower_shape_t* shape, int64_t B, void* workspace, size_t ws_bytes,
                            void* stream) {
  TowerLayout L;
  int rc = tower_layout(shape, B, &L);
  if (rc) return rc;
  if (!workspace || ws_bytes < L.total) return fail(TT_ECAPACITY, "tower: workspace too small");
  hipStream_t st = as_stream(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  if (hipMemsetAsync(ws, 0, L.total, st) != hipSuccess) return fail(TT_EINVAL, "tower: memset failed");
  if (L.lds) return hipStreamSynchronize(st) == hipSuccess ? TT_OK : fail(TT_EINVAL, "tower: init sync failed");
  // the tile list of the register-path T2 (host-built, copied once)
  std::vector<WgradTile> tiles;
  for (int t = 0; t < 2; ++t)
    for (int l = 0; l < shape->L; ++l)
      for (int n0 = 0; n0 < shape->width[l]; n0 += 32)
        for (int k0 = 0; k0 < L.K[t][l]; k0 += 32) tiles.push_back({t, l, n0, k0});
  if (hipMemcpyAsync(ws + L.o_tiles, tiles.data(), tiles.size() * sizeof(WgradTile), hipMemcpyHostToDevice, st) !=
      hipSuccess)
    return fail(TT_EINVAL, "tower: tile upload failed");
  return hipStreamSynchronize(st) == hipSuccess ? TT_OK : fail(TT_EINVAL, "tower: init sync failed");
}

}  // extern "C"

namespace tt {
// the NEXT batch's insert role (tt_tower_wgrad_pre_insert, tt_tower_tail_rowwise_adagrad_insert)
static int insert_args(int64_t B, const void* const* next_cols, int id_dtype, const int64_t* num_embeddings,
                       const int32_t* dedup_tables, void* next_dedup_ws, int64_t dedup_max_lookups, InsertArgs& ins) {
  for (int t = 0; t < 2; ++t) {
    if (!next_cols[t] || num_embeddings[t] < 1 || num_embeddings[t] >= (1ll << DD_TABLE_SHIFT) ||
        dedup_tables[t] < 0 || dedup_tables[t] >= TT_MAX_TABLES)
      return fail(TT_EINVAL, "tower insert: bad column / table");
    ins.col[t] = next_cols[t];
    ins.mod[t] = num_embeddings[t];
    ins.tab[t] = dedup_tables[t];
  }
  ins.id_dtype = id_dtype;
  ins.B = B;
  // tile-class filing (ins_lookup): 2B / 256 workgroups, B / 2048 of them per (class, tower)
  ins.xcd_wpt = (INS_PT == 1 && B % 2048 == 0) ? (int)(B / 2048) : 0;
  dedup_layout(next_dedup_ws, dedup_max_lookups, &ins.dd);
  return TT_OK;
}

}  // namespace tt

namespace tt {
// shared by tt_tower_fwd_bwd / tt_tower_fwd_bwd_gather: checks, T1 arguments, launch
static int launch_t1(const tt_tower_shape_t* shape, int64_t B, TowerArgs& a, const float* pooled, int64_t ldp,
                     float* gpooled, const float* params, const void* labels, int label_dtype, float grad_scale,
                     float* logits, void* workspace, size_t ws_bytes, void* stream) {
  TowerLayout L;
  int rc = tower_layout(shape, B, &L);
  if (rc) return rc;
  if (!workspace || ws_bytes < L.total) return fail(TT_ECAPACITY, "tower: workspace too small");
  if ((!pooled && !a.gcol[0] && !a.gpos[0] && !a.mval && !a.ipos) || (!gpooled && !a.gpos[0] && !a.ipos) || !params ||
      !labels || !logits)
    return fail(TT_EINVAL, "tower: null pointer");
  if (label_dtype != TT_I32 && label_dtype != TT_I64 && label_dtype != TT_F32)
    return fail(TT_EINVAL, "tower: labels must be int32/int64/float32");
  if (ldp % 4 || (reinterpret_cast<uintptr_t>(pooled) & 15) || (reinterpret_cast<uintptr_t>(gpooled) & 15) ||
      (reinterpret_cast<uintptr_t>(a.pooled_out) & 15))
    return fail(TT_EINVAL, "tower: pooled rows and their gradient must be 16-B aligned");
  for (int t = 0; t < 2; ++t)
    if (shape->in_col[t] + shape->in_dim[t] > ldp) return fail(TT_EINVAL, "tower: input columns exceed the pooled row");
  char* ws = reinterpret_cast<char*>(workspace);
  a.s = *shape;
  a.B = B;
  a.pooled = pooled;
  a.ldp = ldp;
  a.gpooled = gpooled;
  a.params = params;
  a.wb = reinterpret_cast<const __bf16*>(ws + L.o_wb);
  a.wtb = reinterpret_cast<const __bf16*>(ws + L.o_wtb);
  a.wbf = reinterpret_cast<const __bf16*>(ws + L.o_wbf);
  a.wtbf = reinterpret_cast<const __bf16*>(ws + L.o_wtbf);
  for (int t = 0; t < 2; ++t)
    for (int l = 0; l < MAXL; ++l) {
      a.woff[t][l] = L.woff[t][l];
      a.boff[t][l] = L.boff[t][l];
      a.wcoff[t][l] = L.wcoff[t][l];
    }
  a.labels = labels;
  a.label_dtype = label_dtype;
  a.grad_scale = grad_scale;
  a.logits = logits;
  a.xt = reinterpret_cast<__bf16*>(ws + L.o_xt);
  a.act = reinterpret_cast<__bf16*>(ws + L.o_act);
  a.dzt = reinterpret_cast<__bf16*>(ws + L.o_dzt);
  a.dbpart = reinterpret_cast<float*>(ws + L.o_dbpart);
  a.loss_part = reinterpret_cast<float*>(ws + L.o_losspart);
  a.in_max = L.in_max;
  a.Bp = L.Bp;
  a.nwg = L.nwg;
#if TT_EXPERIMENTS
  if (const char* e = getenv("TT_T1_DEBUG")) a.dbg = atoi(e);
  if (a.dbg & 8) a.stamps = reinterpret_cast<int64_t*>(ws + L.o_dbg);
#endif
  const int i0 = shape->in_dim[0], i1 = shape->in_dim[1], w0 = shape->width[0], w1 = shape->width[1];
  const dim3 g(L.nwg), b512(T1_THREADS);
  const bool two = shape->L == 2 && i0 <= 128 && i1 <= 128;
  if ((a.gcol[0] || a.gpos[0]) && !two)
    return fail(TT_EINVAL, "tower: the fused gather needs 2 layers and inputs <= 128 wide");
  // TT_TOWER_GENERAL_T1 shapes keep tile-major operand strips for T2 (a.rm = L.rows is false for
  // them): only the general indexed kernel writes that layout for every shape, so every other T1
  // entry point refuses the flag rather than hand T2 strips in a layout it does not read
  if ((shape->flags & TT_TOWER_GENERAL_T1) && !a.ipos)
    return fail(TT_EINVAL, "tower: TT_TOWER_GENERAL_T1 shapes run T1 through tt_tower_fwd_bwd_indexed_multi only");
  if (a.ipos) {  // several features per tower: the general kernel (any width, chunks of 128 columns)
    tower_fwd_bwd_kernel<<<dim3(L.nwg), dim3(256), 0, as_stream(stream)>>>(a);
    return check_launch("tower_fwd_bwd_indexed_multi");
  }
  if (a.mval) {  // multi-hot EBC forward fused in: compile-time shapes only
    if (two && i0 == 128 && i1 == 128 && w0 == 128 && w1 == 64)
      tower_l2_kernel<128, 128, 64, false, false, true><<<g, b512, 0, as_stream(stream)>>>(a);
    else if (two && i0 == 64 && i1 == 64 && w0 == 128 && w1 == 64)
      tower_l2_kernel<64, 128, 64, false, false, true><<<g, b512, 0, as_stream(stream)>>>(a);
    else
      return fail(TT_EINVAL, "tower_fwd_bwd_kjt: shapes in {64, 128} x [128, 64] only");
    return check_launch("tower_fwd_bwd_kjt");
  }
  // single-hot rows gathered from the tables (not indexed / multi-hot / pooled input): the row-owned T1
  bool rows_t1 = L.rows && !a.ipos && !a.mval && ((a.gcol[0] && !a.gpos[0]) || (a.gpos[0] && a.gsrc_bf16));
  // pooled input (the multi-hot path after tt_pooled_fwd): the row-owned T1 reads the pooled rows
  const bool rows_pool = L.rows && !a.ipos && !a.mval && !a.gcol[0] && !a.gpos[0] && pooled &&
                         !(reinterpret_cast<uintptr_t>(pooled) & 15);
  bool rows_pool_ok = true;
#if TT_EXPERIMENTS
  if (getenv("TT_T1_CLASSIC")) rows_t1 = false;  // EXPERIMENT (A/B): tower_l2_kernel instead
#endif
  if (rows_t1) {
    a.wimg = ws + L.o_wimg;
    if (a.gpos[0])
      i0 == 64 ? tower_rows_kernel<false, true, 64><<<g, dim3(256), 0, as_stream(stream)>>>(a)
               : tower_rows_kernel<false, true, 128><<<g, dim3(256), 0, as_stream(stream)>>>(a);
    else if (a.uw[0])
      i0 == 64 ? tower_rows_kernel<true, false, 64><<<g, dim3(256), 0, as_stream(stream)>>>(a)
               : tower_rows_kernel<true, false, 128><<<g, dim3(256), 0, as_stream(stream)>>>(a);
    else
      i0 == 64 ? tower_rows_kernel<false, false, 64><<<g, dim3(256), 0, as_stream(stream)>>>(a)
               : tower_rows_kernel<false, false, 128><<<g, dim3(256), 0, as_stream(stream)>>>(a);
    return check_launch(a.uw[0] ? "tower_rows_gather_update" : "tower_rows_gather");
  }
#if TT_EXPERIMENTS
  if (getenv("TT_T1_CLASSIC")) rows_pool_ok = false;
#endif
  if (rows_pool && rows_pool_ok) {
    a.wimg = ws + L.o_wimg;
    i0 == 64 ? tower_rows_kernel<false, false, 64, true><<<g, dim3(256), 0, as_stream(stream)>>>(a)
             : tower_rows_kernel<false, false, 128, true><<<g, dim3(256), 0, as_stream(stream)>>>(a);
    return check_launch("tower_rows_pooled");
  }
  if (a.uw[0]) {  // in-place update of single-lookup rows: compile-time shapes only
    if (two && i0 == 128 && i1 == 128 && w0 == 128 && w1 == 64)
      tower_l2_kernel<128, 128, 64, false, true><<<g, b512, 0, as_stream(stream)>>>(a);
    else if (two && i0 == 64 && i1 == 64 && w0 == 128 && w1 == 64)
      tower_l2_kernel<64, 128, 64, false, true><<<g, b512, 0, as_stream(stream)>>>(a);
    else
      return fail(TT_EINVAL, "tower_gather_update: shapes in {64, 128} x [128, 64] only");
    return check_launch("tower_fwd_bwd_gather_update");
  }
  if (two && i0 == 128 && i1 == 128 && w0 == 128 && w1 == 64 && a.gsrc_bf16)
    tower_l2_kernel<128, 128, 64, true><<<g, b512, 0, as_stream(stream)>>>(a);
  else if (two && a.gsrc_bf16)
    tower_l2_kernel<0, 0, 0, true><<<g, b512, 0, as_stream(stream)>>>(a);
  else if (two && i0 == 128 && i1 == 128 && w0 == 128 && w1 == 64)
    tower_l2_kernel<128, 128, 64><<<g, b512, 0, as_stream(stream)>>>(a);
  else if (two && i0 == 64 && i1 == 64 && w0 == 128 && w1 == 64)
    tower_l2_kernel<64, 128, 64><<<g, b512, 0, as_stream(stream)>>>(a);
  else if (two)
    tower_l2_kernel<0, 0, 0><<<g, b512, 0, as_stream(stream)>>>(a);
  else
    tower_fwd_bwd_kernel<<<dim3(L.nwg), dim3(256), 0, as_stream(stream)>>>(a);
  return check_launch("tower_fwd_bwd");
}

// T2 arguments from the shape + workspace (shared by tt_tower_wgrad and the combined launch)
static int wgrad_args(const tt_tower_shape_t* shape, int64_t B, float* loss, void* workspace, size_t ws_bytes,
                      WgradArgs& a, int64_t* wgs) {
  TowerLayout L;
  int rc = tower_layout(shape, B, &L);
  if (rc) return rc;
  if (!workspace || ws_bytes < L.total) return fail(TT_ECAPACITY, "tower: workspace too small");
  char* ws = reinterpret_cast<char*>(workspace);
  a.xt = reinterpret_cast<const __bf16*>(ws + L.o_xt);
  a.act = reinterpret_cast<const __bf16*>(ws + L.o_act);
  a.dzt = reinterpret_cast<const __bf16*>(ws + L.o_dzt);
  a.slab = reinterpret_cast<float*>(ws + L.o_slab);
  a.P = L.P;
  a.B = B;
  a.in_max = L.in_max;
  a.Bp = L.Bp;
  a.S = L.S;
  a.mslice = L.mslice;
  a.ntiles = L.ntiles;
  for (int t = 0; t < 2; ++t)
    for (int l = 0; l < MAXL; ++l) {
      a.woff[t][l] = L.woff[t][l];
      a.boff[t][l] = L.boff[t][l];
      a.K[t][l] = L.K[t][l];
    }
  int nbias = 0;
  for (int l = 0; l < shape->L; ++l) {
    a.width[l] = shape->width[l];
    nbias += 2 * shape->width[l];
  }
  a.L = shape->L;
  a.dbpart = reinterpret_cast<const float*>(ws + L.o_dbpart);
  a.nwg = L.nwg;
  a.loss_part = reinterpret_cast<const float*>(ws + L.o_losspart);
  a.loss = loss;
  a.nbias = nbias;
  a.tiles_off = (int64_t)L.o_tiles;
#if TT_EXPERIMENTS
  if (getenv("TT_T2_STAMPS")) a.stamps = reinterpret_cast<int64_t*>(ws + L.o_dbg);
#endif
  a.lds = L.lds;
  a.rm = L.rows;
  for (int i = 0; i < 16; ++i) {
    a.t2_code[i] = L.t2_code[i];
  }
  *wgs =(int64_t)L.ntiles * L.S + ceil_div(nbias + 1, 4);
  return TT_OK;
}
}  // namespace tt

extern "C" {

int tt_tower_fwd_bwd(const tt_tower_shape_t* shape, int64_t B, const float* pooled, int64_t ldp, float* gpooled,
                     const float* params, const void* labels, int label_dtype, float grad_scale, float* logits,
                     void* workspace, size_t ws_bytes, void* stream) {
  TowerArgs a{};
  return launch_t1(shape, B, a, pooled, ldp, gpooled, params, labels, label_dtype, grad_scale, logits, workspace,
                   ws_bytes, stream);
}

int tt_tower_fwd_bwd_gather(const tt_tower_shape_t* shape, int64_t B, const void* const* cols, int id_dtype,
                            const int64_t* num_embeddings, const float* const* table_rows, float* pooled_out,
                            int64_t ldp, float* gpooled, const float* params, const void* labels, int label_dtype,
                            float grad_scale, float* logits, const int32_t* dedup_tables, void* dedup_ws,
                            size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* workspace, size_t ws_bytes,
                            void* stream) {
  if (!cols || !num_embeddings || !table_rows) return fail(TT_EINVAL, "tower_gather: null pointer");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "tower_gather: ids must be int32/int64");
  TowerArgs a{};
  for (int t = 0; t < 2; ++t) {
    if (!cols[t] || !table_rows[t] || num_embeddings[t] < 1) return fail(TT_EINVAL, "tower_gather: bad column");
    if (reinterpret_cast<uintptr_t>(table_rows[t]) & 15) return fail(TT_EINVAL, "tower_gather: rows not 16-B aligned");
    a.gcol[t] = cols[t];
    a.gtab[t] = table_rows[t];
    a.gmod[t] = num_embeddings[t];
  }
  a.gid_dtype = id_dtype;
  a.pooled_out = pooled_out;
  if (dedup_ws) {
    if (!dedup_tables) return fail(TT_EINVAL, "tower_gather: dedup needs the key table of each tower");
    if (dedup_max_lookups < 2 * B || dedup_max_lookups >= (int64_t)DD_CNT_MASK ||
        dedup_ws_bytes < dedup_layout(nullptr, dedup_max_lookups, nullptr) ||
        (reinterpret_cast<uintptr_t>(dedup_ws) & 63))
      return fail(TT_ECAPACITY, "tower_gather: dedup workspace too small / misaligned");
    for (int t = 0; t < 2; ++t) {
      if (dedup_tables[t] < 0 || dedup_tables[t] >= TT_MAX_TABLES || num_embeddings[t] >= (1ll << DD_TABLE_SHIFT))
        return fail(TT_EINVAL, "tower_gather: bad dedup table");
      a.dd_table[t] = dedup_tables[t];
    }
    dedup_layout(dedup_ws, dedup_max_lookups, &a.dd);
    a.dd_on = 1;
  }
  return launch_t1(shape, B, a, nullptr, ldp, gpooled, params, labels, label_dtype, grad_scale, logits, workspace,
                   ws_bytes, stream);
}

int tt_tower_fwd_bwd_kjt(const tt_tower_shape_t* shape, int64_t B, const void* values, int id_dtype,
                         const int32_t* offsets, const int64_t* num_rows, const float* const* table_rows,
                         float* pooled_out, int64_t ldp, float* gpooled, const float* params, const void* labels,
                         int label_dtype, float grad_scale, float* logits, void* workspace, size_t ws_bytes,
                         void* stream) {
  if (!values || !offsets || !num_rows || !table_rows) return fail(TT_EINVAL, "tower_fwd_bwd_kjt: null pointer");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "tower_fwd_bwd_kjt: ids must be int32/int64");
  TowerArgs a{};
  for (int t = 0; t < 2; ++t) {
    if (!table_rows[t] || num_rows[t] < 1) return fail(TT_EINVAL, "tower_fwd_bwd_kjt: bad table");
    if (reinterpret_cast<uintptr_t>(table_rows[t]) & 15)
      return fail(TT_EINVAL, "tower_fwd_bwd_kjt: rows not 16-B aligned");
    a.gtab[t] = table_rows[t];
    a.gmod[t] = num_rows[t];
    a.moff[t] = offsets + (int64_t)t * B;  // key-major: tower t's bags follow the previous key's B
  }
  a.mval = values;
  a.gid_dtype = id_dtype;
  a.pooled_out = pooled_out;
  return launch_t1(shape, B, a, nullptr, ldp, gpooled, params, labels, label_dtype, grad_scale, logits, workspace,
                   ws_bytes, stream);
}

static int tower_indexed(const tt_tower_shape_t* shape, int64_t B, const int32_t* const* pos,
                         const float* const* rows_in, float* const* grad_rows_out, const float* params,
                         const void* labels, int label_dtype, float grad_scale, float* logits, void* workspace,
                         size_t ws_bytes, void* stream, int bf16_rows) {
  if (!pos || !rows_in || !grad_rows_out) return fail(TT_EINVAL, "tower_indexed: null pointer");
  TowerArgs a{};
  a.gsrc_bf16 = bf16_rows;
  for (int t = 0; t < 2; ++t) {
    if (!pos[t] || !rows_in[t] || !grad_rows_out[t]) return fail(TT_EINVAL, "tower_indexed: null pointer");
    if ((reinterpret_cast<uintptr_t>(rows_in[t]) & 15) || (reinterpret_cast<uintptr_t>(grad_rows_out[t]) & 15))
      return fail(TT_EINVAL, "tower_indexed: rows not 16-B aligned");
    a.gpos[t] = pos[t];
    a.gsrc[t] = rows_in[t];
    a.gdst[t] = grad_rows_out[t];
  }
  return launch_t1(shape, B, a, nullptr,
                   std::max(shape->in_col[0] + shape->in_dim[0], shape->in_col[1] + shape->in_dim[1]), nullptr, params, labels, label_dtype,
                   grad_scale, logits, workspace, ws_bytes, stream);
}

int tt_tower_fwd_bwd_indexed(const tt_tower_shape_t* shape, int64_t B, const int32_t* const* pos,
                             const float* const* rows_in, float* const* grad_rows_out, const float* params,
                             const void* labels, int label_dtype, float grad_scale, float* logits, void* workspace,
                             size_t ws_bytes, void* stream) {
  return tower_indexed(shape, B, pos, rows_in, grad_rows_out, params, labels, label_dtype, grad_scale, logits,
                       workspace, ws_bytes, stream, 0);
}

int tt_tower_fwd_bwd_indexed_bf16(const tt_tower_shape_t* shape, int64_t B, const int32_t* const* pos,
                                  const void* const* rows_in, float* const* grad_rows_out, const float* params,
                                  const void* labels, int label_dtype, float grad_scale, float* logits,
                                  void* workspace, size_t ws_bytes, void* stream) {
  return tower_indexed(shape, B, pos, reinterpret_cast<const float* const*>(rows_in), grad_rows_out, params, labels,
                       label_dtype, grad_scale, logits, workspace, ws_bytes, stream, 1);
}

int tt_tower_wgrad(const tt_tower_shape_t* shape, int64_t B, float* loss, void* workspace, size_t ws_bytes,
                   void* stream) {
  WgradArgs a{};
  int64_t wgs = 0;
  int rc = wgrad_args(shape, B, loss, workspace, ws_bytes, a, &wgs);
  if (rc) return rc;
  tower_wgrad_kernel<<<dim3((unsigned)wgs), dim3(256), 0, as_stream(stream)>>>(
      a, reinterpret_cast<const WgradTile*>(reinterpret_cast<char*>(workspace) + a.tiles_off));
  return check_launch("tower_wgrad");
}

int tt_tower_wgrad_pre(const tt_tower_shape_t* shape, int64_t B, float* loss, void* workspace, size_t ws_bytes,
                       int64_t* adam_step_state, float adam_lr, float adam_beta1, float adam_beta2, void* dedup_ws,
                       size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream) {
  if (!adam_step_state) return fail(TT_EINVAL, "tower_wgrad_pre: null Adam step state");
  WgradArgs a{};
  int64_t wgs = 0;
  int rc = wgrad_args(shape, B, loss, workspace, ws_bytes, a, &wgs);
  if (rc) return rc;
  if (dedup_ws) {
    if (dedup_max_lookups < 1 || dedup_max_lookups >= (int64_t)DD_CNT_MASK ||
        dedup_ws_bytes < dedup_layout(nullptr, dedup_max_lookups, nullptr) ||
        (reinterpret_cast<uintptr_t>(dedup_ws) & 63))
      return fail(TT_ECAPACITY, "tower_wgrad_pre: dedup workspace too small / misaligned");
    dedup_layout(dedup_ws, dedup_max_lookups, &a.dd);
    a.n_res = 64;
    wgs += a.n_res;
  }
  TowerLayout L;
  tower_layout(shape, B, &L);
  a.step_state = adam_step_state;
  a.adam_pre = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + L.o_counter);
  a.lr = adam_lr;
  a.beta1 = adam_beta1;
  a.beta2 = adam_beta2;
  tower_wgrad_kernel<<<dim3((unsigned)wgs), dim3(256), 0, as_stream(stream)>>>(
      a, reinterpret_cast<const WgradTile*>(reinterpret_cast<char*>(workspace) + a.tiles_off));
  return check_launch("tower_wgrad_pre");
}

static int fused_wgrad_adagrad(const tt_tower_shape_t* shape, int64_t B, float* loss, void* workspace,
                               size_t ws_bytes, const tt_table_meta_t* tables, int T,
                               const tt_feature_meta_t* features, int F, int64_t emb_B, const float* grad,
                               int64_t ldg, float* weights, float* state, float lr, float eps, void* dedup_ws,
                               size_t dedup_ws_bytes, int64_t dedup_max_lookups, int64_t* adam_step_state,
                               float adam_lr, float adam_beta1, float adam_beta2, void* stream) {
  WgradArgs a{};
  int64_t wgs = 0;
  int rc = wgrad_args(shape, B, loss, workspace, ws_bytes, a, &wgs);
  if (rc) return rc;
  if (adam_step_state) {  // T2 advances the Adam step and precomputes its scalars for T3
    TowerLayout L;
    tower_layout(shape, B, &L);
    a.step_state = adam_step_state;
    a.adam_pre = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + L.o_counter);
    a.lr = adam_lr;
    a.beta1 = adam_beta1;
    a.beta2 = adam_beta2;
  }
  DdUpdateArgs d{};
  int64_t dd_grid = 0;
  rc = dedup_update_args(tables, T, features, F, emb_B, grad, ldg, weights, state, lr, eps, dedup_ws, dedup_ws_bytes,
                         dedup_max_lookups, d, &dd_grid);
  if (rc) return rc;
  if (wgs + dd_grid > INT32_MAX) return fail(TT_EINVAL, "tower_wgrad_rowwise_adagrad: grid too large");
  tower_wgrad_dedup_kernel<<<dim3((unsigned)(wgs + dd_grid)), dim3(256), 0, as_stream(stream)>>>(
      a, reinterpret_cast<const WgradTile*>(reinterpret_cast<char*>(workspace) + a.tiles_off), d, (int)wgs);
  return check_launch("tower_wgrad_rowwise_adagrad");
}

// T3 arguments (shared by every T3 launch form)
static int t3_args(const tt_tower_shape_t* shape, int64_t B, float* params, float* exp_avg, float* exp_avg_sq,
                   float lr, float beta1, float beta2, float eps, float weight_decay, int64_t* step_state, int do_adam,
                   float* grads_out, const float* grads_in, void* workspace, size_t ws_bytes, const float* adam_pre,
                   int out_copies, const int64_t* out_off, float out_scale, int in_srcs, int64_t in_stride,
                   UpdateArgs& a, int64_t* grid) {
  TowerLayout L;
  int rc = tower_layout(shape, B, &L);
  if (rc) return rc;
  if (!workspace || ws_bytes < L.total) return fail(TT_ECAPACITY, "tower: workspace too small");
  if (!params || (do_adam && (!exp_avg || !exp_avg_sq || (!step_state && !adam_pre))))
    return fail(TT_EINVAL, "tower: null pointer");
  if (out_copies > 16) return fail(TT_EINVAL, "tower: at most 16 gradient copies");
  char* ws = reinterpret_cast<char*>(workspace);
  a = UpdateArgs{};
  a.params = params;
  a.exp_avg = exp_avg;
  a.exp_avg_sq = exp_avg_sq;
  a.slab = reinterpret_cast<const float*>(ws + L.o_slab);
  a.dbpart = reinterpret_cast<const float*>(ws + L.o_dbpart);
  a.P = L.P;
  a.S = L.S;
  a.nwg = L.nwg;
  int sg = 0;
  for (int t = 0; t < 2; ++t)
    for (int l = 0; l < shape->L; ++l) {
      a.seg_off[sg] = L.woff[t][l];
      a.seg_t[sg] = t; a.seg_l[sg] = l; a.seg_isw[sg] = 1;
      a.seg_n[sg] = shape->width[l]; a.seg_k[sg] = L.K[t][l];
      a.seg_wc[sg] = L.wcoff[t][l];
      ++sg;
      a.seg_off[sg] = L.boff[t][l];
      a.seg_t[sg] = t; a.seg_l[sg] = l; a.seg_isw[sg] = 0;
      a.seg_n[sg] = shape->width[l]; a.seg_k[sg] = 1;
      a.seg_wc[sg] = 0;
      ++sg;
    }
  a.nseg = sg;
  a.seg_off[sg] = L.P;
  a.wb = reinterpret_cast<__bf16*>(ws + L.o_wb);
  a.wtb = reinterpret_cast<__bf16*>(ws + L.o_wtb);
  a.wbf = reinterpret_cast<__bf16*>(ws + L.o_wbf);
  a.wtbf = reinterpret_cast<__bf16*>(ws + L.o_wtbf);
  a.wimg = L.rows ? ws + L.o_wimg : nullptr;
  // the plain [out][in] / [in][out] bf16 copies are read only by tower_fwd_bwd_kernel, which
  // launch_t1 uses for shapes other than two layers over inputs <= 128 wide
  a.skip_plain = shape->L == 2 && shape->in_dim[0] <= 128 && shape->in_dim[1] <= 128 &&
                 !(shape->flags & TT_TOWER_GENERAL_T1);
  a.lr = lr; a.beta1 = beta1; a.beta2 = beta2; a.eps = eps; a.wd = weight_decay;
  a.step_state = step_state;
  a.do_adam = do_adam;
  a.grads_out = grads_out;
  a.grads_in = grads_in;
  a.adam_pre = adam_pre;
  a.out_copies = out_copies;
  for (int q = 0; q < out_copies && out_off; ++q) a.out_off[q] = out_off[q];
  a.out_scale = out_scale;
  a.in_srcs = in_srcs;
  a.in_stride = in_stride;
  *grid = ceil_div(L.P, 256);
  return TT_OK;
}

static int launch_t3(const tt_tower_shape_t* shape, int64_t B, float* params, float* exp_avg, float* exp_avg_sq,
                     float lr, float beta1, float beta2, float eps, float weight_decay, int64_t* step_state,
                     int do_adam, float* grads_out, const float* grads_in, void* workspace, size_t ws_bytes,
                     void* stream, const float* adam_pre = nullptr, const DdUpdateArgs* dd = nullptr,
                     int64_t dd_grid = 0, int out_copies = 1, const int64_t* out_off = nullptr,
                     float out_scale = 1.f, int in_srcs = 1, int64_t in_stride = 0,
                     const tt_peer_wait_t* wait = nullptr) {
  UpdateArgs a;
  int64_t g3 = 0;
  int rc = t3_args(shape, B, params, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step_state, do_adam,
                   grads_out, grads_in, workspace, ws_bytes, adam_pre, out_copies, out_off, out_scale, in_srcs,
                   in_stride, a, &g3);
  if (rc) return rc;
  if ((rc = peer_wait_args(wait, a.wt, "tower_update"))) return rc;
  if (dd) {
    if (dd_grid + g3 > INT32_MAX) return fail(TT_EINVAL, "tower_update_rowwise_adagrad: grid too large");
    tower_update_dedup_kernel<<<dim3((unsigned)(dd_grid + g3)), dim3(256), 0, as_stream(stream)>>>(a, *dd, (int)dd_grid);
    return check_launch("tower_update_rowwise_adagrad");
  }
#if TT_EXPERIMENTS
  if (getenv("TT_RING_STAMPS")) {  // workgroups [0, 512) stamp
    TowerLayout L;
    tower_layout(shape, B, &L);
    a.stamps = reinterpret_cast<int64_t*>(reinterpret_cast<char*>(workspace) + L.o_dbg) + 6144;
  }
#endif
  int bs = 256;
#if TT_EXPERIMENTS
  if (const char* e = getenv("TT_T3_BLOCK")) bs = atoi(e) == 128 ? 128 : 256;  // EXPERIMENT
#endif
  tower_update_kernel<<<dim3((unsigned)ceil_div(a.P, (int64_t)bs)), dim3(bs), 0, as_stream(stream)>>>(a);
  return check_launch("tower_update");
}

int tt_tower_update(const tt_tower_shape_t* shape, int64_t B, float* params, float* exp_avg, float* exp_avg_sq,
                    float lr, float beta1, float beta2, float eps, float weight_decay, int64_t* step_state,
                    int do_adam, float* grads_out, void* workspace, size_t ws_bytes, void* stream) {
  return launch_t3(shape, B, params, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step_state, do_adam,
                   grads_out, nullptr, workspace, ws_bytes, stream);
}

int tt_tower_update_pre(const tt_tower_shape_t* shape, int64_t B, float* params, float* exp_avg, float* exp_avg_sq,
                        float eps, float beta1, float beta2, float weight_decay, float* grads_out, void* workspace,
                        size_t ws_bytes, void* stream) {
  TowerLayout L;
  int rc = tower_layout(shape, B, &L);
  if (rc) return rc;
  if (!workspace || ws_bytes < L.total) return fail(TT_ECAPACITY, "tower: workspace too small");
  const float* pre = reinterpret_cast<const float*>(reinterpret_cast<const char*>(workspace) + L.o_counter);
  return launch_t3(shape, B, params, exp_avg, exp_avg_sq, 0.f, beta1, beta2, eps, weight_decay, nullptr, 1, grads_out,
                   nullptr, workspace, ws_bytes, stream, pre);
}

static int fused_update_adagrad(const tt_tower_shape_t* shape, int64_t B, float* params, float* exp_avg,
                                float* exp_avg_sq, float eps, float beta1, float beta2, float weight_decay,
                                float* grads_out, void* workspace, size_t ws_bytes,
                                const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features, int F,
                                int64_t emb_B, const float* grad, int64_t ldg, float* weights, float* state,
                                float lr, float emb_eps, void* dedup_ws, size_t dedup_ws_bytes,
                                int64_t dedup_max_lookups, void* stream) {
  TowerLayout L;
  int rc = tower_layout(shape, B, &L);
  if (rc) return rc;
  if (!workspace || ws_bytes < L.total) return fail(TT_ECAPACITY, "tower: workspace too small");
  DdUpdateArgs d{};
  int64_t dd_grid = 0;
  rc = dedup_update_args(tables, T, features, F, emb_B, grad, ldg, weights, state, lr, emb_eps, dedup_ws,
                         dedup_ws_bytes, dedup_max_lookups, d, &dd_grid);
  if (rc) return rc;
  const float* pre = reinterpret_cast<const float*>(reinterpret_cast<const char*>(workspace) + L.o_counter);
  return launch_t3(shape, B, params, exp_avg, exp_avg_sq, 0.f, beta1, beta2, eps, weight_decay, nullptr, 1, grads_out,
                   nullptr, workspace, ws_bytes, stream, pre, &d, dd_grid);
}

int tt_tower_adam_grads(const tt_tower_shape_t* shape, int64_t B, float* params, const float* grads,
                        float* exp_avg, float* exp_avg_sq, float lr, float beta1, float beta2, float eps,
                        float weight_decay, int64_t* step_state, void* workspace, size_t ws_bytes, void* stream) {
  if (!grads) return fail(TT_EINVAL, "tower_adam_grads: null gradient");
  return launch_t3(shape, B, params, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step_state, 1,
                   nullptr, grads, workspace, ws_bytes, stream);
}

int tt_tower_grads_replicated(const tt_tower_shape_t* shape, int64_t B, float* params, float* base, int copies,
                              const int64_t* offsets, float scale, void* workspace, size_t ws_bytes, void* stream) {
  TowerLayout L;
  int rc = tower_layout(shape, B, &L);
  if (rc) return rc;
  if (!base || !offsets || copies < 1 || copies > 16) return fail(TT_EINVAL, "tower_grads_replicated: bad output");
  for (int q = 0; q < copies; ++q)
    if (offsets[q] < 0) return fail(TT_EINVAL, "tower_grads_replicated: negative offset");
  int64_t off[16];
  for (int q = 0; q < copies; ++q) off[q] = offsets[q];
  if (copies == 1) off[1] = off[0];
  // copies == 1 takes the multi-copy path too (scale applied): give it two identical copies
  return launch_t3(shape, B, params, nullptr, nullptr, 0.f, 0.9f, 0.999f, 1e-8f, 0.f, nullptr, 0, base, nullptr,
                   workspace, ws_bytes, stream, nullptr, nullptr, 0, copies == 1 ? 2 : copies, off, scale);
}

int tt_tower_adam_pre_grads_sum(const tt_tower_shape_t* shape, int64_t B, float* params, const float* grads, int nsrc,
                                int64_t src_stride, float* exp_avg, float* exp_avg_sq, float eps, float beta1,
                                float beta2, float weight_decay, void* workspace, size_t ws_bytes,
                                const tt_peer_wait_t* wait, void* stream) {
  TowerLayout L;
  int rc = tower_layout(shape, B, &L);
  if (rc) return rc;
  if (!workspace || ws_bytes < L.total) return fail(TT_ECAPACITY, "tower: workspace too small");
  if (!grads || nsrc < 1 || (nsrc > 1 && src_stride < L.P)) return fail(TT_EINVAL, "tower_adam_pre_grads_sum: bad gradient");
  if (wait && wait->W != nsrc) return fail(TT_EINVAL, "tower_adam_pre_grads_sum: wait.W must be nsrc");
  const float* pre = reinterpret_cast<const float*>(reinterpret_cast<const char*>(workspace) + L.o_counter);
  return launch_t3(shape, B, params, exp_avg, exp_avg_sq, 0.f, beta1, beta2, eps, weight_decay, nullptr, 1, nullptr,
                   grads, workspace, ws_bytes, stream, pre, nullptr, 0, 1, nullptr, 1.f, nsrc, src_stride, wait);
}

}  // extern "C"

namespace tt {
// shared by the two fused entry points: the next batch's route arguments (as tt_shard_route_segs)
static int route_segs_args(int F, int64_t B, const void* const* cols, int id_dtype, const int64_t* num_embeddings,
                           const int64_t* block_sizes, const int32_t* owners, int W, const tt_shard_seg_t* segs,
                           int64_t* send, int32_t* pos_in, int32_t* pos_out, int32_t* overflow, void* route_ws,
                           size_t route_ws_bytes, RouteArgs& a) {
  if (F < 1 || F > TT_MAX_FEATURES || W < 1 || W > RT_MAXW || B < 1) return fail(TT_EINVAL, "route: bad sizes");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "route: ids must be int32/int64");
  if (!cols || !num_embeddings || !block_sizes || !owners || !segs || !send || !pos_in || !pos_out || !overflow)
    return fail(TT_EINVAL, "route: null pointer");
  if (!route_ws || route_ws_bytes < tt_shard_route_workspace_bytes(F, B))
    return fail(TT_ECAPACITY, "route: workspace too small");
  for (int f = 0; f < F; ++f) {
    if (!cols[f] || num_embeddings[f] < 1) return fail(TT_EINVAL, "route: bad column");
    if (block_sizes[f] < 0 || (block_sizes[f] == 0 && (owners[f] < 0 || owners[f] >= W)))
      return fail(TT_EINVAL, "route: bad sharding of a feature");
    if (block_sizes[f] > 0 && (num_embeddings[f] + block_sizes[f] - 1) / block_sizes[f] > W)
      return fail(TT_EINVAL, "route: row blocks exceed the rank count");
    if ((block_sizes[f] > 0 ? block_sizes[f] : num_embeddings[f]) >= (1ll << DD_TABLE_SHIFT))
      return fail(TT_EINVAL, "route: local rows >= 2^40");
    a.col[f] = cols[f];
    a.num_emb[f] = num_embeddings[f];
    a.block[f] = block_sizes[f];
    a.owner[f] = owners[f];
  }
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
  char* ws = reinterpret_cast<char*>(route_ws);
  a.dl = reinterpret_cast<int64_t*>(ws);
  a.cnt = reinterpret_cast<int32_t*>(ws + align_up(sizeof(int64_t) * (size_t)F * (size_t)B, 256));
  return TT_OK;
}
}  // namespace tt

extern "C" {

static int fused_wgrad_route_count_adagrad(const tt_tower_shape_t* shape, int64_t B, float* loss, void* workspace,
                                           size_t ws_bytes, int64_t* adam_step_state, float adam_lr,
                                           float adam_beta1, float adam_beta2, int F, const void* const* cols,
                                           int id_dtype,
                                           const int64_t* num_embeddings, const int64_t* block_sizes,
                                           const int32_t* owners, int W, const tt_shard_seg_t* segs, int64_t* send,
                                           int32_t* pos_in, int32_t* pos_out, int32_t* overflow, void* route_ws,
                                           size_t route_ws_bytes, const tt_table_meta_t* tables, int T,
                                           const tt_feature_meta_t* features, int Fsrc, int64_t emb_B,
                                           const float* emb_grad, int64_t ldg, float* weights, float* state,
                                           float emb_lr, float emb_eps, void* dedup_ws, size_t dedup_ws_bytes,
                                           int64_t dedup_max_lookups, const tt_peer_wait_t* wait, void* stream) {
  if (!adam_step_state) return fail(TT_EINVAL, "tower_wgrad_route_rowwise: null Adam step state");
  PxWait pw;
  if (int rc = peer_wait_args(wait, pw, "tower_wgrad_route_rowwise")) return rc;
  WgradArgs a{};
  int64_t wgs = 0;
  int rc = wgrad_args(shape, B, loss, workspace, ws_bytes, a, &wgs);
  if (rc) return rc;
  TowerLayout L;
  tower_layout(shape, B, &L);
  a.step_state = adam_step_state;  // the loss wave advances Adam's step and writes its scalars
  a.adam_pre = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + L.o_counter);
  a.lr = adam_lr;
  a.beta1 = adam_beta1;
  a.beta2 = adam_beta2;
  RouteArgs r{};
  rc = route_segs_args(F, B, cols, id_dtype, num_embeddings, block_sizes, owners, W, segs, send, pos_in, pos_out,
                       overflow, route_ws, route_ws_bytes, r);
  if (rc) return rc;
  DdUpdateArgs d{};
  int64_t dd_grid = 0;
  rc = dedup_update_args(tables, T, features, Fsrc, emb_B, emb_grad, ldg, weights, state, emb_lr, emb_eps, dedup_ws,
                         dedup_ws_bytes, dedup_max_lookups, d, &dd_grid);
  if (rc) return rc;
  const int64_t n_cnt = (int64_t)r.nblk * F;
  if (wgs + n_cnt + dd_grid > INT32_MAX) return fail(TT_EINVAL, "tower_wgrad_route_rowwise: grid too large");
  d.xcd = d.hot_wgs % 8 == 0 ? 1 : 0;  // the owner's update workgroups first (dd_first): slot role aligned
#if TT_EXPERIMENTS
  static const bool dd_first = !getenv("TT_U_DD_FIRST") || atoi(getenv("TT_U_DD_FIRST")) != 0;  // A/B switch
#else
  constexpr bool dd_first = true;
#endif
  tower_wgrad_route_rowwise_kernel<<<dim3((unsigned)(wgs + n_cnt + dd_grid)), dim3(256), 0, as_stream(stream)>>>(
      a, reinterpret_cast<const WgradTile*>(reinterpret_cast<char*>(workspace) + a.tiles_off), r, d, (int)wgs,
      (int)n_cnt, dd_first ? (int)dd_grid : 0, pw);
  return check_launch("tower_wgrad_route_count_rowwise_adagrad");
}

static int fused_route_count_adagrad(int F, int64_t B, const void* const* cols, int id_dtype,
                                     const int64_t* num_embeddings, const int64_t* block_sizes,
                                     const int32_t* owners, int W, const tt_shard_seg_t* segs, int64_t* send,
                                     int32_t* pos_in, int32_t* pos_out, int32_t* overflow, void* route_ws,
                                     size_t route_ws_bytes, const tt_table_meta_t* tables, int T,
                                     const tt_feature_meta_t* features, int Fsrc, int64_t emb_B,
                                     const float* emb_grad, int64_t ldg, float* weights, float* state,
                                     float emb_lr, float emb_eps, void* dedup_ws, size_t dedup_ws_bytes,
                                     int64_t dedup_max_lookups, const tt_peer_wait_t* wait, void* stream) {
  PxWait pw;
  if (int rc = peer_wait_args(wait, pw, "shard_route_count_rowwise_adagrad")) return rc;
  // launch U of the pipelined sharded step without its T2 tiles (those run on a parallel branch of
  // the step graph, beside exchange A): the owner's update workgroups first, then the route count
  RouteArgs r{};
  int rc = route_segs_args(F, B, cols, id_dtype, num_embeddings, block_sizes, owners, W, segs, send, pos_in, pos_out,
                           overflow, route_ws, route_ws_bytes, r);
  if (rc) return rc;
  DdUpdateArgs d{};
  int64_t dd_grid = 0;
  rc = dedup_update_args(tables, T, features, Fsrc, emb_B, emb_grad, ldg, weights, state, emb_lr, emb_eps, dedup_ws,
                         dedup_ws_bytes, dedup_max_lookups, d, &dd_grid);
  if (rc) return rc;
  const int64_t n_cnt = (int64_t)r.nblk * F;
  if (n_cnt + dd_grid > INT32_MAX) return fail(TT_EINVAL, "shard_route_count_rowwise_adagrad: grid too large");
  d.xcd = d.hot_wgs % 8 == 0 ? 1 : 0;  // the owner's update workgroups first: slot role aligned
  WgradArgs a{};
  tower_wgrad_route_rowwise_kernel<<<dim3((unsigned)(n_cnt + dd_grid)), dim3(256), 0, as_stream(stream)>>>(
      a, nullptr, r, d, 0, (int)n_cnt, (int)dd_grid, pw);
  return check_launch("shard_route_count_rowwise_adagrad");
}

static int fused_grads_route_place_gather(const tt_tower_shape_t* shape, int64_t B, float* params, float* base,
                                          int copies, const int64_t* offsets, float scale, void* workspace,
                                          size_t ws_bytes, int F, const void* const* cols, int id_dtype,
                                          const int64_t* num_embeddings, const int64_t* block_sizes,
                                          const int32_t* owners, int W, const tt_shard_seg_t* segs,
                                          int64_t* send, int32_t* pos_in, int32_t* pos_out, int32_t* overflow,
                                          void* route_ws, size_t route_ws_bytes, const float* weights,
                                          const tt_table_meta_t* tables, int T, const int64_t* recv,
                                          int64_t block_i64, int64_t counts_i64, const int64_t* seg_off,
                                          int64_t slots, void* rows_out, int64_t out_stride, int32_t* bad,
                                          void* dedup_ws, size_t dedup_ws_bytes, int64_t dedup_max_lookups,
                                          const tt_peer_direct_t* direct, void* stream) {
  if (!params || !base || !offsets || copies < 1 || copies > 16) return fail(TT_EINVAL, "tower_grads_replicated: bad output");
  RouteArgs r{};
  int rc = route_segs_args(F, B, cols, id_dtype, num_embeddings, block_sizes, owners, W, segs, send, pos_in, pos_out,
                           overflow, route_ws, route_ws_bytes, r);
  if (rc) return rc;
  GatherSegArgs g{};
  rc = gather_segs_args(weights, tables, T, F, W, recv, block_i64, counts_i64, seg_off, slots, rows_out, out_stride,
                        bad, dedup_ws, dedup_ws_bytes, dedup_max_lookups, g);
  if (rc) return rc;
  if (direct) {
    if ((rc = peer_direct_check(*direct, "tower_grads_place_gather"))) return rc;
    if (direct->W != W) return fail(TT_EINVAL, "tower_grads_place_gather: direct.W must be the route's W");
    for (int s = 0; s < W; ++s) {
      if (direct->first_row[s] != (int64_t)s * out_stride)
        return fail(TT_EINVAL, "tower_grads_place_gather: direct.first_row[s] must be s * out_stride");
      g.dblk[s] = reinterpret_cast<__bf16*>(direct->row0[s]);
    }
    g.dW = W;
    g.epoch = direct->epoch;
  }
  int64_t off[16];
  for (int q = 0; q < copies; ++q) off[q] = offsets[q];
  if (copies == 1) off[1] = off[0];  // one copy takes the multi-copy path too (scale applied)
  UpdateArgs a;
  int64_t g3 = 0;
  rc = t3_args(shape, B, params, nullptr, nullptr, 0.f, 0.9f, 0.999f, 1e-8f, 0.f, nullptr, 0, base, nullptr, workspace,
               ws_bytes, nullptr, copies == 1 ? 2 : copies, off, scale, 1, 0, a, &g3);
  if (rc) return rc;
  const int64_t n_place = (int64_t)r.nblk * F, n_gather = ceil_div(ceil_div((int64_t)W * slots, GS_SL), 8);
  if (g3 + n_place + n_gather > INT32_MAX) return fail(TT_EINVAL, "tower_grads_place_gather: grid too large");
  tower_grads_place_gather_kernel<<<dim3((unsigned)(g3 + n_place + n_gather)), dim3(256), 0, as_stream(stream)>>>(
      a, r, g, (int)g3, (int)n_place);
  return check_launch("tower_grads_replicated_route_place_gather");
}

int tt_tower_fwd_bwd_gather_update(const tt_tower_shape_t* shape, int64_t B, const void* const* cols, int id_dtype,
                                   const int64_t* num_embeddings, float* const* table_rows, float* const* table_state,
                                   float* pooled_out, int64_t ldp, float* gpooled, const float* params,
                                   const void* labels, int label_dtype, float grad_scale, float* logits, float lr,
                                   float eps, void* dedup_ws, size_t dedup_ws_bytes, int64_t dedup_max_lookups,
                                   const void* const* next_cols, void* workspace, size_t ws_bytes, void* stream) {
  if (!cols || !num_embeddings || !table_rows || !table_state || !dedup_ws)
    return fail(TT_EINVAL, "tower_gather_update: null pointer");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "tower_gather_update: ids must be int32/int64");
  if (dedup_max_lookups < 2 * B || dedup_max_lookups >= (int64_t)DD_CNT_MASK ||
      dedup_ws_bytes < dedup_layout(nullptr, dedup_max_lookups, nullptr) || (reinterpret_cast<uintptr_t>(dedup_ws) & 63))
    return fail(TT_ECAPACITY, "tower_gather_update: dedup workspace too small / misaligned");
  TowerArgs a{};
  for (int t = 0; t < 2; ++t) {
    if (!cols[t] || !table_rows[t] || !table_state[t] || num_embeddings[t] < 1)
      return fail(TT_EINVAL, "tower_gather_update: bad column");
    if (reinterpret_cast<uintptr_t>(table_rows[t]) & 15) return fail(TT_EINVAL, "tower_gather_update: rows not 16-B aligned");
    a.gcol[t] = cols[t];
    a.gtab[t] = table_rows[t];
    a.gmod[t] = num_embeddings[t];
    a.uw[t] = table_rows[t];
    a.us[t] = table_state[t];
    if (next_cols) {
      if (!next_cols[t]) return fail(TT_EINVAL, "tower_gather_update: null next column");
      a.pcol[t] = next_cols[t];
    }
  }
  a.gid_dtype = id_dtype;
  a.pooled_out = pooled_out;
  a.ulr = lr;
  a.ueps = eps;
  dedup_layout(dedup_ws, dedup_max_lookups, &a.dd);
  return launch_t1(shape, B, a, nullptr, ldp, gpooled, params, labels, label_dtype, grad_scale, logits, workspace,
                   ws_bytes, stream);
}

static int fused_wgrad_insert(const tt_tower_shape_t* shape, int64_t B, float* loss, void* workspace, size_t ws_bytes,
                              int64_t* adam_step_state, float adam_lr, float adam_beta1, float adam_beta2,
                              const void* const* next_cols, int id_dtype, const int64_t* num_embeddings,
                              const int32_t* dedup_tables, void* next_dedup_ws, size_t dedup_ws_bytes,
                              int64_t dedup_max_lookups, void* stream) {
  if (!adam_step_state || !next_cols || !num_embeddings || !dedup_tables || !next_dedup_ws)
    return fail(TT_EINVAL, "tower_wgrad_pre_insert: null pointer");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "tower_wgrad_pre_insert: ids must be int32/int64");
  if (dedup_max_lookups < 2 * B || dedup_max_lookups >= (int64_t)DD_CNT_MASK ||
      dedup_ws_bytes < dedup_layout(nullptr, dedup_max_lookups, nullptr) ||
      (reinterpret_cast<uintptr_t>(next_dedup_ws) & 63))
    return fail(TT_ECAPACITY, "tower_wgrad_pre_insert: dedup workspace too small / misaligned");
  WgradArgs a{};
  int64_t wgs = 0;
  int rc = wgrad_args(shape, B, loss, workspace, ws_bytes, a, &wgs);
  if (rc) return rc;
  TowerLayout L;
  tower_layout(shape, B, &L);
  a.step_state = adam_step_state;
  a.adam_pre = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + L.o_counter);
  a.lr = adam_lr;
  a.beta1 = adam_beta1;
  a.beta2 = adam_beta2;
  InsertArgs ins{};
  rc = insert_args(B, next_cols, id_dtype, num_embeddings, dedup_tables, next_dedup_ws, dedup_max_lookups, ins);
  if (rc) return rc;
  const int64_t n_ins = ceil_div(ceil_div(2 * B, 64), 4);  // 4 waves of 64 lookups per workgroup
  int64_t* stamps = TT_EXPERIMENTS && getenv("TT_RING_STAMPS") ? reinterpret_cast<int64_t*>(reinterpret_cast<char*>(workspace) + L.o_dbg) + 4096 : nullptr;
  tower_wgrad_insert_kernel<<<dim3((unsigned)(wgs + n_ins)), dim3(256), 0, as_stream(stream)>>>(
      a, reinterpret_cast<const WgradTile*>(reinterpret_cast<char*>(workspace) + a.tiles_off), ins, (int)wgs, stamps);
  return check_launch("tower_wgrad_pre_insert");
}

static int fused_update_adagrad_resolve(const tt_tower_shape_t* shape, int64_t B, float* params,
                                        float* exp_avg, float* exp_avg_sq, float eps, float beta1,
                                        float beta2, float weight_decay, float* grads_out, void* workspace,
                                        size_t ws_bytes, const tt_table_meta_t* tables, int T,
                                        const tt_feature_meta_t* features, int F, int64_t emb_B,
                                        const float* grad, int64_t ldg, float* weights, float* state,
                                        float lr, float emb_eps, void* dedup_ws, void* next_dedup_ws,
                                        size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream) {
  if (!next_dedup_ws || (reinterpret_cast<uintptr_t>(next_dedup_ws) & 63))
    return fail(TT_EINVAL, "tower_update_resolve: next dedup workspace null / misaligned");
  DdUpdateArgs d{};
  int64_t dd_grid = 0;
  int rc = dedup_update_args(tables, T, features, F, emb_B, grad, ldg, weights, state, lr, emb_eps, dedup_ws,
                             dedup_ws_bytes, dedup_max_lookups, d, &dd_grid);
  if (rc) return rc;
  d.skip_single = 1;
  DedupWs next;
  dedup_layout(next_dedup_ws, dedup_max_lookups, &next);
  TowerLayout L;
  rc = tower_layout(shape, B, &L);
  if (rc) return rc;
  const float* pre = reinterpret_cast<const float*>(reinterpret_cast<const char*>(workspace) + L.o_counter);
  UpdateArgs a;
  int64_t g3 = 0;
  rc = t3_args(shape, B, params, exp_avg, exp_avg_sq, 0.f, beta1, beta2, eps, weight_decay, nullptr, 1, grads_out,
               nullptr, workspace, ws_bytes, pre, 1, nullptr, 1.f, 1, 0, a, &g3);
  if (rc) return rc;
  int64_t* stamps = TT_EXPERIMENTS && getenv("TT_RING_STAMPS") ? reinterpret_cast<int64_t*>(reinterpret_cast<char*>(workspace) + L.o_dbg) + 6144 : nullptr;
  if (stamps && (K3_RES_WGS + dd_grid + g3 > 1024 || L.nwg > 256)) stamps = nullptr;
  tower_update_dedup_resolve_kernel<<<dim3((unsigned)(K3_RES_WGS + dd_grid + g3)), dim3(256), 0,
                                      as_stream(stream)>>>(a, d, next, (int)dd_grid, stamps);
  return check_launch("tower_update_pre_rowwise_adagrad_resolve");
}

static int fused_wgrad_insert_adagrad(const tt_tower_shape_t* shape, int64_t B, float* loss, void* workspace,
                                      size_t ws_bytes, int64_t* adam_step_state, float adam_lr,
                                      float adam_beta1, float adam_beta2, const void* const* next_cols,
                                      int id_dtype, const int64_t* num_embeddings, const int32_t* dedup_tables,
                                      const tt_table_meta_t* tables, int T, const tt_feature_meta_t* features,
                                      int F, const float* grad, int64_t ldg, float* weights, float* state,
                                      float lr, float emb_eps, void* dedup_ws, void* next_dedup_ws,
                                      size_t dedup_ws_bytes, int64_t dedup_max_lookups, void* stream) {
  if (!adam_step_state || !next_cols || !num_embeddings || !dedup_tables || !next_dedup_ws)
    return fail(TT_EINVAL, "tower_tail: null pointer");
  if (id_dtype != TT_I32 && id_dtype != TT_I64) return fail(TT_EINVAL, "tower_tail: ids must be int32/int64");
  if (dedup_max_lookups < 2 * B || dedup_max_lookups >= (int64_t)DD_CNT_MASK ||
      dedup_ws_bytes < dedup_layout(nullptr, dedup_max_lookups, nullptr) ||
      (reinterpret_cast<uintptr_t>(next_dedup_ws) & 63))
    return fail(TT_ECAPACITY, "tower_tail: dedup workspace too small / misaligned");
  WgradArgs a2{};
  int64_t wgs = 0;
  int rc = wgrad_args(shape, B, loss, workspace, ws_bytes, a2, &wgs);
  if (rc) return rc;
  TowerLayout L;
  tower_layout(shape, B, &L);
  char* ws = reinterpret_cast<char*>(workspace);
  a2.step_state = adam_step_state;
  a2.adam_pre = reinterpret_cast<float*>(ws + L.o_counter);
  a2.lr = adam_lr;
  a2.beta1 = adam_beta1;
  a2.beta2 = adam_beta2;
  InsertArgs ins{};
  rc = insert_args(B, next_cols, id_dtype, num_embeddings, dedup_tables, next_dedup_ws, dedup_max_lookups, ins);
  if (rc) return rc;
  DdUpdateArgs d{};
  int64_t dd_grid = 0;
  rc = dedup_update_args(tables, T, features, F, B, grad, ldg, weights, state, lr, emb_eps, dedup_ws, dedup_ws_bytes,
                         dedup_max_lookups, d, &dd_grid);
  if (rc) return rc;
  d.skip_single = 1;
  bool list = L.rows && L.lds;  // the row-owned T1 listed the multi-lookup rows and freed the single slots
#if TT_EXPERIMENTS
  if (const char* e = getenv("TT_MULTI_LIST")) list = list && e[0] != '0';  // EXPERIMENT: A/B
  if (getenv("TT_T1_CLASSIC")) list = false;  // EXPERIMENT: tower_l2_kernel T1 writes no list
  if (const char* e = getenv("TT_EXP_SKIP")) d.exp_skip = atoi(e);
#endif
  // the list role scans at most 2048 segments (B <= 16384); past that the slot role walks every
  // claiming lookup (T1 still freed the single slots: their words read EMPTY there)
  list = list && L.nwg * 4 <= std::min<int64_t>(d.ws.nseg, 2048);
  if (list) {
    d.multi_nseg = (int)(L.nwg * 4);
    // a workgroup's share of the listed slots <= 256 (at most lookups / 2 slots are listed)
    int64_t nlb = std::max<int64_t>(8, ceil_div(2 * B, 512) * 4);
#if TT_EXPERIMENTS
    if (const char* e = getenv("TT_LIST_WGS")) nlb = std::max(nlb, (int64_t)atoi(e));  // EXPERIMENT
#endif
    d.slot_hw = nlb * 8;
    dd_grid = d.hot_wgs + nlb;
  }
  const int64_t n_ins = ceil_div(ceil_div(2 * B, 256 * INS_PT), 8) * 8;  // INS_PT lookups per thread; % 8 == 0
  int64_t* stamps = TT_EXPERIMENTS && getenv("TT_RING_STAMPS") ? reinterpret_cast<int64_t*>(ws + L.o_dbg) + 4096 : nullptr;
  if (stamps && L.nwg > 256) stamps = nullptr;
  // the list role (the ring) in a kernel of its own code: no slot-role instructions in its footprint
  auto kern = list ? tower_tail_kernel<true> : tower_tail_kernel<false>;
  kern<<<dim3((unsigned)(n_ins + wgs + dd_grid)), dim3(256), 0, as_stream(stream)>>>(
      a2, reinterpret_cast<const WgradTile*>(ws + a2.tiles_off), ins, d, (int)n_ins, (int)wgs, stamps);
  return check_launch("tower_wgrad_pre_insert_rowwise_adagrad");
}

int tt_tower_fwd_bwd_indexed_multi_bf16(const tt_tower_shape_t* shape, int64_t B, int D, const int32_t* pos_in,
                                        const int32_t* pos_out, const void* rows_in, float* grad_rows_out,
                                        const float* params, const void* labels, int label_dtype, float grad_scale,
                                        float* logits, void* workspace, size_t ws_bytes, void* stream) {
  if (!shape || !pos_in || !pos_out || !rows_in || !grad_rows_out)
    return fail(TT_EINVAL, "tower_indexed_multi: null pointer");
  if (D < 16 || D > 128 || D % 16 || XCH % D)
    return fail(TT_EINVAL, "tower_indexed_multi: feature dim must be 16..128, a multiple of 16 dividing 128");
  for (int t = 0; t < 2; ++t)
    if (shape->in_dim[t] % D) return fail(TT_EINVAL, "tower_indexed_multi: tower input not a multiple of D");
  if (shape->in_col[0] != 0 || shape->in_col[1] != shape->in_dim[0])
    return fail(TT_EINVAL, "tower_indexed_multi: query features first, then candidate features");
  if ((reinterpret_cast<uintptr_t>(rows_in) & 7) || (reinterpret_cast<uintptr_t>(grad_rows_out) & 3))
    return fail(TT_EINVAL, "tower_indexed_multi: rows not aligned");
  if (shape->L == 2 && shape->in_dim[0] <= 128 && shape->in_dim[1] <= 128 && !(shape->flags & TT_TOWER_GENERAL_T1))
    return fail(TT_EINVAL, "tower_indexed_multi: set TT_TOWER_GENERAL_T1 in the shape (T3 must keep the general "
                           "T1's weight copies)");
  TowerArgs a{};
  a.ipos = pos_in;
  a.ipos_out = pos_out;
  a.isrc = reinterpret_cast<const __bf16*>(rows_in);
  a.idst = grad_rows_out;
  a.ifeat0[0] = 0;
  a.ifeat0[1] = shape->in_dim[0] / D;
  a.iD = D;
  return launch_t1(shape, B, a, nullptr, shape->in_dim[0] + shape->in_dim[1], nullptr, params, labels, label_dtype,
                   grad_scale, logits, workspace, ws_bytes, stream);
}

static int tower_indexed2(const tt_tower_shape_t* shape, int64_t B, const int32_t* const* pos_in,
                          const int32_t* const* pos_out, const void* const* rows_in, float* const* grad_rows_out,
                          const float* params, const void* labels, int label_dtype, float grad_scale, float* logits,
                          void* workspace, size_t ws_bytes, const tt_peer_direct_t* direct, void* stream) {
  if (!pos_in || !pos_out || !rows_in || !grad_rows_out) return fail(TT_EINVAL, "tower_indexed2: null pointer");
  TowerArgs a{};
  if (direct) {
    if (int rc = peer_direct_check(*direct, "tower_indexed2")) return rc;
    if (grad_rows_out[0] != grad_rows_out[1])
      return fail(TT_EINVAL, "tower_indexed2: a direct exchange takes one send buffer (grad_rows_out[0] == [1])");
    a.xd = *direct;
  }
  a.gsrc_bf16 = 1;
  for (int t = 0; t < 2; ++t) {
    if (!pos_in[t] || !pos_out[t] || !rows_in[t] || !grad_rows_out[t]) return fail(TT_EINVAL, "tower_indexed2: null pointer");
    if ((reinterpret_cast<uintptr_t>(rows_in[t]) & 15) || (reinterpret_cast<uintptr_t>(grad_rows_out[t]) & 15))
      return fail(TT_EINVAL, "tower_indexed2: rows not 16-B aligned");
    a.gpos[t] = pos_in[t];
    a.gpos_out[t] = pos_out[t];
    a.gsrc[t] = reinterpret_cast<const float*>(rows_in[t]);
    a.gdst[t] = grad_rows_out[t];
  }
  return launch_t1(shape, B, a, nullptr,
                   std::max(shape->in_col[0] + shape->in_dim[0], shape->in_col[1] + shape->in_dim[1]), nullptr, params,
                   labels, label_dtype, grad_scale, logits, workspace, ws_bytes, stream);
}

int tt_tower_fwd_bwd_indexed2_bf16(const tt_tower_shape_t* shape, int64_t B, const int32_t* const* pos_in,
                                   const int32_t* const* pos_out, const void* const* rows_in,
                                   float* const* grad_rows_out, const float* params, const void* labels,
                                   int label_dtype, float grad_scale, float* logits, void* workspace, size_t ws_bytes,
                                   const tt_peer_direct_t* direct, void* stream) {
  return tower_indexed2(shape, B, pos_in, pos_out, rows_in, grad_rows_out, params, labels, label_dtype, grad_scale,
                        logits, workspace, ws_bytes, direct, stream);
}

// ---- launch plans (include/tt_mi355x.h): the multi-role fused launches behind one entry point ----
int tt_launch(const tt_launch_plan_t* p, void* stream) {
  if (!p) return fail(TT_EINVAL, "launch: null plan");
  const tt_wgrad_role_t& w = p->wgrad;
  const tt_update_role_t& u = p->update;
  const tt_insert_role_t& in = p->insert;
  const tt_adagrad_role_t& g = p->adagrad;
  const tt_route_role_t& r = p->route;
  const tt_gather_role_t& ga = p->gather;
  const int64_t B = p->B;
  auto need_multi = [&](int want) {
    return g.multi_only == want ? TT_OK
                                : fail(TT_EINVAL, want ? "launch: this plan updates only rows looked up more than once "
                                                         "(adagrad.multi_only = 1)"
                                                       : "launch: this plan updates every row (adagrad.multi_only = 0)");
  };
  // the in-launch exchange wait is launch U's alone
  if (p->wait && p->roles != (TT_ROLE_WGRAD | TT_ROLE_ROUTE_COUNT | TT_ROLE_ADAGRAD) &&
      p->roles != (TT_ROLE_ROUTE_COUNT | TT_ROLE_ADAGRAD))
    return fail(TT_EINVAL, "launch: only launch U (ROUTE_COUNT | ADAGRAD [| WGRAD]) takes a wait");
  auto adam_mode = [&]() {
    return u.replicated ? fail(TT_EINVAL, "launch: this plan's UPDATE role runs Adam (update.replicated = 0)") : TT_OK;
  };
  int rc = TT_OK;
  switch (p->roles) {
    case TT_ROLE_WGRAD | TT_ROLE_INSERT | TT_ROLE_ADAGRAD:
      if ((rc = need_multi(1))) return rc;
      // the ring tail's lookups per feature are the plan's B (the tower batch): a different
      // adagrad.B is a caller error, not something to ignore
      if (g.B && g.B != B) return fail(TT_EINVAL, "launch: this plan's ADAGRAD role uses the plan's B (adagrad.B = 0 or B)");
      if ((in.dedup_ws_bytes && in.dedup_ws_bytes != g.dedup_ws_bytes) ||
          (in.dedup_max_lookups && in.dedup_max_lookups != g.dedup_max_lookups))
        return fail(TT_EINVAL, "launch: the ring's two dedup workspaces have one size (the ADAGRAD role's)");
      return fused_wgrad_insert_adagrad(p->shape, B, w.loss, p->workspace, p->ws_bytes, w.adam_step_state, w.adam_lr,
                                        w.adam_beta1, w.adam_beta2, in.next_cols, in.id_dtype, in.num_embeddings,
                                        in.dedup_tables, g.tables, g.T, g.features, g.F, g.grad, g.ldg, g.weights,
                                        g.state, g.lr, g.eps, g.dedup_ws, in.next_dedup_ws, g.dedup_ws_bytes,
                                        g.dedup_max_lookups, stream);
    case TT_ROLE_WGRAD | TT_ROLE_INSERT:
      return fused_wgrad_insert(p->shape, B, w.loss, p->workspace, p->ws_bytes, w.adam_step_state, w.adam_lr,
                                w.adam_beta1, w.adam_beta2, in.next_cols, in.id_dtype, in.num_embeddings,
                                in.dedup_tables, in.next_dedup_ws, in.dedup_ws_bytes, in.dedup_max_lookups, stream);
    case TT_ROLE_UPDATE | TT_ROLE_ADAGRAD | TT_ROLE_RESOLVE:
      if ((rc = need_multi(1)) || (rc = adam_mode())) return rc;
      return fused_update_adagrad_resolve(p->shape, B, u.params, u.exp_avg, u.exp_avg_sq, u.eps, u.beta1, u.beta2,
                                          u.weight_decay, u.grads_out, p->workspace, p->ws_bytes, g.tables, g.T,
                                          g.features, g.F, g.B, g.grad, g.ldg, g.weights, g.state, g.lr, g.eps,
                                          g.dedup_ws, p->resolve.dedup_ws, g.dedup_ws_bytes, g.dedup_max_lookups,
                                          stream);
    case TT_ROLE_WGRAD | TT_ROLE_ADAGRAD:
      if ((rc = need_multi(0))) return rc;
      return fused_wgrad_adagrad(p->shape, B, w.loss, p->workspace, p->ws_bytes, g.tables, g.T, g.features, g.F, g.B,
                                 g.grad, g.ldg, g.weights, g.state, g.lr, g.eps, g.dedup_ws, g.dedup_ws_bytes,
                                 g.dedup_max_lookups, w.adam_step_state, w.adam_lr, w.adam_beta1, w.adam_beta2,
                                 stream);
    case TT_ROLE_UPDATE | TT_ROLE_ADAGRAD:
      if ((rc = need_multi(0)) || (rc = adam_mode())) return rc;
      return fused_update_adagrad(p->shape, B, u.params, u.exp_avg, u.exp_avg_sq, u.eps, u.beta1, u.beta2,
                                  u.weight_decay, u.grads_out, p->workspace, p->ws_bytes, g.tables, g.T, g.features,
                                  g.F, g.B, g.grad, g.ldg, g.weights, g.state, g.lr, g.eps, g.dedup_ws,
                                  g.dedup_ws_bytes, g.dedup_max_lookups, stream);
    case TT_ROLE_WGRAD | TT_ROLE_ROUTE_COUNT | TT_ROLE_ADAGRAD:
      if ((rc = need_multi(0))) return rc;
      return fused_wgrad_route_count_adagrad(p->shape, B, w.loss, p->workspace, p->ws_bytes, w.adam_step_state,
                                             w.adam_lr, w.adam_beta1, w.adam_beta2, r.F, r.cols, r.id_dtype,
                                             r.num_embeddings, r.block_sizes, r.owners, r.W, r.segs, r.send, r.pos_in,
                                             r.pos_out, r.overflow, r.route_ws, r.route_ws_bytes, g.tables, g.T,
                                             g.features, g.F, g.B, g.grad, g.ldg, g.weights, g.state, g.lr, g.eps,
                                             g.dedup_ws, g.dedup_ws_bytes, g.dedup_max_lookups, p->wait, stream);
    case TT_ROLE_ROUTE_COUNT | TT_ROLE_ADAGRAD:
      if ((rc = need_multi(0))) return rc;
      return fused_route_count_adagrad(r.F, B, r.cols, r.id_dtype, r.num_embeddings, r.block_sizes, r.owners, r.W,
                                       r.segs, r.send, r.pos_in, r.pos_out, r.overflow, r.route_ws, r.route_ws_bytes,
                                       g.tables, g.T, g.features, g.F, g.B, g.grad, g.ldg, g.weights, g.state, g.lr,
                                       g.eps, g.dedup_ws, g.dedup_ws_bytes, g.dedup_max_lookups, p->wait, stream);
    case TT_ROLE_UPDATE | TT_ROLE_ROUTE_PLACE | TT_ROLE_GATHER:
      if (!u.replicated) return fail(TT_EINVAL, "launch: launch G's UPDATE role writes the replicated gradient "
                                                "(update.replicated = 1)");
      return fused_grads_route_place_gather(p->shape, B, u.params, u.base, u.copies, u.offsets, u.scale, p->workspace,
                                            p->ws_bytes, r.F, r.cols, r.id_dtype, r.num_embeddings, r.block_sizes,
                                            r.owners, r.W, r.segs, r.send, r.pos_in, r.pos_out, r.overflow, r.route_ws,
                                            r.route_ws_bytes, ga.weights, ga.tables, ga.T, ga.recv, ga.block_i64,
                                            ga.counts_i64, ga.seg_off, ga.slots, ga.rows_out, ga.out_stride, ga.bad,
                                            ga.dedup_ws, ga.dedup_ws_bytes, ga.dedup_max_lookups, ga.direct, stream);
    default:
      return fail(TT_EINVAL, "launch: no fused launch runs this set of roles (see tt_launch_plan_t)");
  }
}

}  // extern "C"

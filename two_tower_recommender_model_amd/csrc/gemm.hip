// Tower GEMMs on gfx950 MFMA: bf16 operands (v_mfma_f32_16x16x32_bf16) or exact fp32 operands
// (v_mfma_f32_16x16x4_f32, the fp32 parity mode), fp32 accumulation in both.
//
// One template covers the three products of an MLP layer (torchrec Perceptron = Linear + ReLU on
// every layer, 03_model_training.py:411-412):
//   FWD         Y  = relu(X W^T + b)            A = X   [M,K] row-major,  B_c[n][k] = W[n][k]
//   BWD_DATA    dX = (dY * (Y>0)) W             A = dZ  [M,N] row-major,  B_c[j][n] = W[n][j]
//   BWD_WEIGHT  dW = (dY * (Y>0))^T X, db       A = dZ^T (transposed),    B_c[j][m] = X[m][j]
// Operands are staged global -> registers (fp32 or bf16 source, ReLU mask applied, converted to
// the compute type) -> LDS in the canonical [row][k] layout with k contiguous, so a bf16 MFMA
// fragment is one 16-B ds_read. 64x64 output tile per 256-thread workgroup (4 waves, 2x2 of 32x32),
// BK = 32. BWD_WEIGHT splits the M reduction over workgroups into fp32 slabs summed in a fixed
// order by a second kernel (bitwise reproducible; no float atomics).
#include "tt_common.h"

namespace tt {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 64, BN = 64, BK = 32;

enum { MODE_FWD = 0, MODE_BWD_DATA = 1, MODE_BWD_WEIGHT = 2 };

template <bool F32>
struct Tile {
  typedef typename std::conditional<F32, float, __bf16>::type T;
  static constexpr int STRIDE = F32 ? BK + 4 : BK + 8;  // 144-B / 80-B rows
};

struct GemmProblem {
  const void* a;       // X (FWD), dY (BWD_DATA, BWD_WEIGHT)
  const float* amask;  // Y for the relu mask (BWD_*), else null
  const void* b;       // W (FWD, BWD_DATA), X (BWD_WEIGHT)
  const float* bias;   // FWD only, nullable
  float* c;            // Y (FWD), dX (BWD_DATA), slab base (BWD_WEIGHT)
  float* dbslab;       // BWD_WEIGHT: [S][N] partial bias grads (nullable)
};

struct GemmArgs {
  GemmProblem p[2];
  int64_t M;  // canonical rows of C
  int64_t N;  // canonical cols of C
  int64_t K;  // canonical reduction length
  int64_t lda, ldb, ldc, ldmask;
  int a_bf16, b_bf16;
  int relu;
  int splits;      // BWD_WEIGHT: slices of K
  int64_t kslice;  // BWD_WEIGHT: K per slice (multiple of BK)
};

__device__ __forceinline__ float ld_elem(const void* p, int bf, int64_t i) {
  if (bf) {
    const unsigned short u = reinterpret_cast<const unsigned short*>(p)[i];
    return __uint_as_float(((unsigned)u) << 16);
  }
  return reinterpret_cast<const float*>(p)[i];
}

template <typename T>
__device__ __forceinline__ void store8(T* dst, const float (&v)[8]) {
  if constexpr (std::is_same<T, float>::value) {
    reinterpret_cast<f32x4*>(dst)[0] = f32x4{v[0], v[1], v[2], v[3]};
    reinterpret_cast<f32x4*>(dst)[1] = f32x4{v[4], v[5], v[6], v[7]};
  } else {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (__bf16)v[j];
    *reinterpret_cast<bf16x8*>(dst) = o;
  }
}

// Row-major source: tile element (r, k) = src[(r0 + r) * ld + k0 + k]. Thread t stages row t/4,
// k-chunk (t%4)*8 .. +8 (8 consecutive elements: 32 B fp32 / 16 B bf16).
template <typename T, int STRIDE>
__device__ __forceinline__ void stage_rowmajor(T* lds, const void* src, int bf, int64_t ld, const float* mask,
                                               int64_t ldm, int64_t rows, int64_t cols, int64_t r0, int64_t k0) {
  const int t = threadIdx.x;
  const int r = t >> 2, kc = (t & 3) * 8;
  const int64_t gr = r0 + r, gk = k0 + kc;
  float v[8];
  if (gr < rows && gk + 8 <= cols && !bf && mask == nullptr && ((ld & 3) == 0) &&
      ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
    const f32x4* s4 = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(src) + gr * ld + gk);
    const f32x4 x0 = s4[0], x1 = s4[1];
    v[0] = x0[0]; v[1] = x0[1]; v[2] = x0[2]; v[3] = x0[3];
    v[4] = x1[0]; v[5] = x1[1]; v[6] = x1[2]; v[7] = x1[3];
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = 0.f;
      if (gr < rows && gk + j < cols) {
        x = ld_elem(src, bf, gr * ld + gk + j);
        if (mask && !(mask[gr * ldm + gk + j] > 0.f)) x = 0.f;
      }
      v[j] = x;
    }
  }
  store8(lds + r * STRIDE + kc, v);
}

// Transposed source: tile element (r, k) = src[(k0 + k) * ld + r0 + r]. Thread t stages row t%64,
// k = (t/64)*8 .. +8; consecutive lanes read consecutive r (coalesced). Returns the fp32 sum of
// the 8 staged values (before any rounding) for the fused bias gradient.
template <typename T, int STRIDE>
__device__ __forceinline__ float stage_transposed(T* lds, const void* src, int bf, int64_t ld, const float* mask,
                                                  int64_t ldm, int64_t rows, int64_t ks, int64_t r0, int64_t k0) {
  const int t = threadIdx.x;
  const int r = t & 63, kc = (t >> 6) * 8;
  const int64_t gr = r0 + r;
  float v[8];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t gk = k0 + kc + j;
    float x = 0.f;
    if (gr < rows && gk < ks) {
      x = ld_elem(src, bf, gk * ld + gr);
      if (mask && !(mask[gk * ldm + gr] > 0.f)) x = 0.f;
    }
    sum += x;
    v[j] = x;
  }
  store8(lds + r * STRIDE + kc, v);
  return sum;
}

template <int MODE, bool F32>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs a) {
  typedef typename Tile<F32>::T T;
  constexpr int STRIDE = Tile<F32>::STRIDE;
  __shared__ __attribute__((aligned(16))) T As[BM * STRIDE];
  __shared__ __attribute__((aligned(16))) T Bs[BN * STRIDE];
  __shared__ float dbred[4][BM];

  int g, split = 0;
  if (MODE == MODE_BWD_WEIGHT) {
    g = blockIdx.z / a.splits;
    split = blockIdx.z - g * a.splits;
  } else {
    g = blockIdx.z;
  }
  const GemmProblem P = a.p[g];
  const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
  int64_t kbeg = 0, kend = a.K;
  if (MODE == MODE_BWD_WEIGHT) {
    kbeg = (int64_t)split * a.kslice;
    kend = kbeg + a.kslice < a.K ? kbeg + a.kslice : a.K;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4)(0.f);
  float dbacc = 0.f;
  const bool do_db = MODE == MODE_BWD_WEIGHT && P.dbslab != nullptr && blockIdx.y == 0;

  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    if (MODE == MODE_FWD) {
      stage_rowmajor<T, STRIDE>(As, P.a, a.a_bf16, a.lda, nullptr, 0, a.M, a.K, m0, k0);
      stage_rowmajor<T, STRIDE>(Bs, P.b, a.b_bf16, a.ldb, nullptr, 0, a.N, a.K, n0, k0);
    } else if (MODE == MODE_BWD_DATA) {
      stage_rowmajor<T, STRIDE>(As, P.a, 0, a.lda, a.relu ? P.amask : nullptr, a.ldmask, a.M, a.K, m0, k0);
      stage_transposed<T, STRIDE>(Bs, P.b, 0, a.ldb, nullptr, 0, a.N, a.K, n0, k0);
    } else {
      const float s =
          stage_transposed<T, STRIDE>(As, P.a, 0, a.lda, a.relu ? P.amask : nullptr, a.ldmask, a.M, kend, m0, k0);
      dbacc += s;
      stage_transposed<T, STRIDE>(Bs, P.b, a.b_bf16, a.ldb, nullptr, 0, a.N, kend, n0, k0);
    }
    __syncthreads();
    if constexpr (F32) {
      // v_mfma_f32_16x16x4_f32: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15]; 8 steps of K=4
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        float af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = As[(wm * 32 + i * 16 + (lane & 15)) * STRIDE + kk + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bfr[j] = Bs[(wn * 32 + j * 16 + (lane & 15)) * STRIDE + kk + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 32 + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(As + row * STRIDE + (lane >> 4) * 8);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wn * 32 + j * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + col * STRIDE + (lane >> 4) * 8);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // epilogue: C/D layout of the 16x16 MFMAs: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (row < a.M && col < a.N) {
          float x = acc[i][j][r];
          if (MODE == MODE_FWD) {
            if (P.bias) x += P.bias[col];
            if (a.relu) x = fmaxf(x, 0.f);
            P.c[row * a.ldc + col] = x;
          } else if (MODE == MODE_BWD_DATA) {
            P.c[row * a.ldc + col] = x;
          } else {
            P.c[((int64_t)split * a.M + row) * a.N + col] = x;
          }
        }
      }
    }
  if (do_db) {
    // 4 threads per canonical row (t/64 = 0..3) combine in a fixed order
    dbred[threadIdx.x >> 6][threadIdx.x & 63] = dbacc;
    __syncthreads();
    if (threadIdx.x < 64) {
      const int64_t row = m0 + threadIdx.x;
      const float s = ((dbred[0][threadIdx.x] + dbred[1][threadIdx.x]) + dbred[2][threadIdx.x]) + dbred[3][threadIdx.x];
      if (row < a.M) P.dbslab[(int64_t)split * a.M + row] = s;
    }
  }
}

// dW[n][k] = sum_s slab[s][n][k]; db[n] = sum_s dbslab[s][n] (fixed order)
struct ReduceArgs {
  const float* slab[2];
  const float* dbslab[2];
  float* dw[2];
  float* db[2];
  int64_t MN;  // elements of dW
  int64_t Mrows;
  int splits;
};

__global__ void __launch_bounds__(256) slab_reduce_kernel(ReduceArgs r) {
  const int g = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < r.MN) {
    float s = 0.f;
    for (int k = 0; k < r.splits; ++k) s += r.slab[g][(int64_t)k * r.MN + i];
    r.dw[g][i] = s;
  }
  if (r.db[g] && i < r.Mrows) {
    float s = 0.f;
    for (int k = 0; k < r.splits; ++k) s += r.dbslab[g][(int64_t)k * r.Mrows + i];
    r.db[g][i] = s;
  }
}

static int check_common(int groups, int compute) {
  if (groups < 1 || groups > 2) return fail(TT_EINVAL, "gemm: groups must be 1 or 2");
  if (compute != TT_BF16 && compute != TT_F32) return fail(TT_EINVAL, "gemm: compute dtype must be TT_BF16 or TT_F32");
  return TT_OK;
}

static int bwd_weight_splits(int groups, int64_t M, int N, int K) {
  const int64_t tiles = ceil_div(N, BM) * ceil_div(K, BN) * groups;
  int64_t s = std::max<int64_t>(1, 512 / std::max<int64_t>(1, tiles));
  s = std::min<int64_t>(s, std::max<int64_t>(1, ceil_div(M, BK)));
  return (int)std::min<int64_t>(s, 256);
}

template <int MODE>
static void launch(dim3 grid, const GemmArgs& a, int compute, hipStream_t st) {
  if (compute == TT_F32)
    gemm_kernel<MODE, true><<<grid, dim3(256), 0, st>>>(a);
  else
    gemm_kernel<MODE, false><<<grid, dim3(256), 0, st>>>(a);
}

}  // namespace tt

using namespace tt;

extern "C" {

int tt_linear_fwd(int groups, const void* const* X, int x_dtype, int64_t ldx, const float* const* W,
                  const float* const* bias, int64_t M, int N, int K, float* const* Y, int64_t ldy, int relu,
                  int compute, void* stream) {
  int rc = check_common(groups, compute);
  if (rc) return rc;
  if (M < 0 || N < 1 || K < 1) return fail(TT_EINVAL, "linear_fwd: bad shape");
  if (x_dtype != TT_F32 && x_dtype != TT_BF16) return fail(TT_EINVAL, "linear_fwd: X must be fp32 or bf16");
  if (!X || !W || !Y) return fail(TT_EINVAL, "linear_fwd: null pointer array");
  if (M == 0) return TT_OK;
  GemmArgs a{};
  for (int g = 0; g < groups; ++g) {
    if (!X[g] || !W[g] || !Y[g]) return fail(TT_EINVAL, "linear_fwd: null pointer");
    a.p[g].a = X[g];
    a.p[g].b = W[g];
    a.p[g].bias = bias ? bias[g] : nullptr;
    a.p[g].c = Y[g];
  }
  a.M = M; a.N = N; a.K = K;
  a.lda = ldx; a.ldb = K; a.ldc = ldy;
  a.a_bf16 = x_dtype == TT_BF16; a.b_bf16 = 0; a.relu = relu;
  launch<MODE_FWD>(dim3((unsigned)ceil_div(M, BM), (unsigned)ceil_div(N, BN), (unsigned)groups), a, compute,
                   as_stream(stream));
  return check_launch("linear_fwd");
}

int tt_linear_bwd_data(int groups, const float* const* dY, const float* const* Y, int64_t ldy,
                       const float* const* W, int64_t M, int N, int K, float* const* dX, int64_t ldx, int relu,
                       int compute, void* stream) {
  int rc = check_common(groups, compute);
  if (rc) return rc;
  if (M < 0 || N < 1 || K < 1) return fail(TT_EINVAL, "linear_bwd_data: bad shape");
  if (!dY || !W || !dX || (relu && !Y)) return fail(TT_EINVAL, "linear_bwd_data: null pointer array");
  if (M == 0) return TT_OK;
  GemmArgs a{};
  for (int g = 0; g < groups; ++g) {
    if (!dY[g] || !W[g] || !dX[g] || (relu && !Y[g])) return fail(TT_EINVAL, "linear_bwd_data: null pointer");
    a.p[g].a = dY[g];
    a.p[g].amask = relu ? Y[g] : nullptr;
    a.p[g].b = W[g];
    a.p[g].c = dX[g];
  }
  // canonical: C[M, K] = A[M, N] * B, B_c[j][n] = W[n][j]
  a.M = M; a.N = K; a.K = N;
  a.lda = ldy; a.ldmask = ldy; a.ldb = K; a.ldc = ldx;
  a.relu = relu;
  launch<MODE_BWD_DATA>(dim3((unsigned)ceil_div(M, BM), (unsigned)ceil_div(K, BN), (unsigned)groups), a, compute,
                        as_stream(stream));
  return check_launch("linear_bwd_data");
}

size_t tt_linear_bwd_weight_workspace_bytes(int groups, int64_t M, int N, int K) {
  if (groups < 1 || groups > 2 || N < 1 || K < 1) return 0;
  const int s = bwd_weight_splits(groups, M, N, K);
  return (size_t)groups * (align_up(sizeof(float) * (size_t)s * N * K, 256) + align_up(sizeof(float) * (size_t)s * N, 256));
}

int tt_linear_bwd_weight(int groups, const float* const* dY, const float* const* Y, int64_t ldy,
                         const void* const* X, int x_dtype, int64_t ldx, int64_t M, int N, int K,
                         float* const* dW, float* const* db, int relu, int compute, void* workspace,
                         size_t ws_bytes, void* stream) {
  int rc = check_common(groups, compute);
  if (rc) return rc;
  if (M < 0 || N < 1 || K < 1) return fail(TT_EINVAL, "linear_bwd_weight: bad shape");
  if (x_dtype != TT_F32 && x_dtype != TT_BF16) return fail(TT_EINVAL, "linear_bwd_weight: X must be fp32 or bf16");
  if (!dY || !X || !dW || (relu && !Y)) return fail(TT_EINVAL, "linear_bwd_weight: null pointer array");
  if (!workspace || ws_bytes < tt_linear_bwd_weight_workspace_bytes(groups, M, N, K))
    return fail(TT_ECAPACITY, "linear_bwd_weight: workspace too small");
  const int S = bwd_weight_splits(groups, M, N, K);
  GemmArgs a{};
  ReduceArgs r{};
  char* ws = reinterpret_cast<char*>(workspace);
  const size_t slab_bytes = align_up(sizeof(float) * (size_t)S * N * K, 256);
  const size_t dbs_bytes = align_up(sizeof(float) * (size_t)S * N, 256);
  for (int g = 0; g < groups; ++g) {
    if (!dY[g] || !X[g] || !dW[g] || (relu && !Y[g])) return fail(TT_EINVAL, "linear_bwd_weight: null pointer");
    float* slab = reinterpret_cast<float*>(ws + g * (slab_bytes + dbs_bytes));
    float* dbslab = reinterpret_cast<float*>(ws + g * (slab_bytes + dbs_bytes) + slab_bytes);
    a.p[g].a = dY[g];
    a.p[g].amask = relu ? Y[g] : nullptr;
    a.p[g].b = X[g];
    a.p[g].c = slab;
    a.p[g].dbslab = (db && db[g]) ? dbslab : nullptr;
    r.slab[g] = slab;
    r.dbslab[g] = dbslab;
    r.dw[g] = dW[g];
    r.db[g] = (db && db[g]) ? db[g] : nullptr;
  }
  hipStream_t st = as_stream(stream);
  if (M == 0) {
    for (int g = 0; g < groups; ++g) {
      if (hipMemsetAsync(dW[g], 0, sizeof(float) * (size_t)N * K, st) != hipSuccess) return fail(TT_EINVAL, "memset");
      if (r.db[g] && hipMemsetAsync(r.db[g], 0, sizeof(float) * (size_t)N, st) != hipSuccess)
        return fail(TT_EINVAL, "memset");
    }
    return TT_OK;
  }
  // canonical: C[N, K] = A[N, M] * B, A_c[n][m] = dZ[m][n], B_c[j][m] = X[m][j]
  a.M = N; a.N = K; a.K = M;
  a.lda = ldy; a.ldmask = ldy; a.ldb = ldx; a.ldc = K;
  a.b_bf16 = x_dtype == TT_BF16;
  a.relu = relu;
  a.splits = S;
  a.kslice = ceil_div(ceil_div(M, S), BK) * BK;
  launch<MODE_BWD_WEIGHT>(dim3((unsigned)ceil_div(N, BM), (unsigned)ceil_div(K, BN), (unsigned)(groups * S)), a,
                          compute, st);
  r.MN = (int64_t)N * K;
  r.Mrows = N;
  r.splits = S;
  dim3 rgrid((unsigned)ceil_div(std::max<int64_t>(r.MN, N), 256), (unsigned)groups);
  slab_reduce_kernel<<<rgrid, dim3(256), 0, st>>>(r);
  return check_launch("linear_bwd_weight");
}

}  // extern "C"

// Small fused kernels of the step: logits + BCEWithLogits(mean) + its gradient (k5), and Adam on
// the flat dense-parameter buffer. Both reduce across workgroups with the agent-scope
// release -> arrival counter -> acquire recipe (last arriver combines the partials in block
// order, so the loss is bitwise reproducible and independent of XCD placement).
#include "tt_common.h"

namespace tt {

// Every workgroup: thread 0 publishes `partial` and arrives; returns true (block-uniform) in the
// last arriving workgroup, after an agent-scope acquire, with the counter reset for the next call.
__device__ __forceinline__ bool arrive_last(float* partials, unsigned* counter, float partial, int* lds_flag) {
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = partial;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *lds_flag = last;
  }
  __syncthreads();
  return *lds_flag != 0;
}

__device__ __forceinline__ float load_label(const void* labels, int dt, int64_t i) {
  if (dt == TT_I32) return (float)reinterpret_cast<const int32_t*>(labels)[i];
  if (dt == TT_I64) return (float)reinterpret_cast<const int64_t*>(labels)[i];
  return reinterpret_cast<const float*>(labels)[i];
}

// G lanes per row, each lane 4 consecutive dims (float4 when aligned).
__global__ void __launch_bounds__(256) dot_bce_kernel(const float* __restrict__ q, int64_t ldq,
                                                      const float* __restrict__ c, int64_t ldc, int64_t B, int dim,
                                                      int G, const void* __restrict__ labels, int ldt,
                                                      float* __restrict__ logits, float* __restrict__ loss,
                                                      float* __restrict__ dq, int64_t lddq, float* __restrict__ dc,
                                                      int64_t lddc, float grad_scale, float* __restrict__ partials,
                                                      unsigned* __restrict__ counter) {
  __shared__ float row_loss[256];
  __shared__ int flag;
  const int rows_per_block = 256 / G;
  const int lr = threadIdx.x / G, lg = threadIdx.x & (G - 1);
  const int64_t row = (int64_t)blockIdx.x * rows_per_block + lr;
  float dot = 0.f;
  float qv[4][4], cv[4][4];  // up to 4 chunks of 4 dims per lane (dim <= 16*G)
  const int nchunk = (dim + 4 * G - 1) / (4 * G);
  if (row < B) {
    for (int k = 0; k < 4; ++k) {
      if (k >= nchunk) break;
      const int d0 = (lg + k * G) * 4;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int d = d0 + v;
        qv[k][v] = d < dim ? q[row * ldq + d] : 0.f;
        cv[k][v] = d < dim ? c[row * ldc + d] : 0.f;
        dot += qv[k][v] * cv[k][v];
      }
    }
  }
  for (int o = G >> 1; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
  float l = 0.f, dlogit = 0.f;
  if (row < B) {
    const float x = dot, y = load_label(labels, ldt, row);
    // BCEWithLogits: (1 - y) * x - logsigmoid(x), logsigmoid(x) = min(x,0) - log1p(exp(-|x|))
    const float lsig = fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
    l = (1.f - y) * x - lsig;
    const float sig = 1.f / (1.f + expf(-x));
    dlogit = (sig - y) / (float)B * grad_scale;
    if (lg == 0) logits[row] = x;
    if (dq) {
      for (int k = 0; k < 4; ++k) {
        if (k >= nchunk) break;
        const int d0 = (lg + k * G) * 4;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int d = d0 + v;
          if (d < dim) {
            dq[row * lddq + d] = dlogit * cv[k][v];
            dc[row * lddc + d] = dlogit * qv[k][v];
          }
        }
      }
    }
  }
  if (lg == 0) row_loss[lr] = l;
  __syncthreads();
  float part = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < rows_per_block; ++i) part += row_loss[i];
  if (arrive_last(partials, counter, part, &flag)) {
    // deterministic: thread i sums partials i, i+256, ... then a fixed-order LDS combine
    float s = 0.f;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += 256) s += partials[i];
    row_loss[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      float tot = 0.f;
      for (int i = 0; i < 256; ++i) tot += row_loss[i];
      loss[0] = tot / (float)B;
    }
  }
}

__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n, float lr,
                                                   float beta1, float beta2, float eps, float wd,
                                                   int64_t* __restrict__ step_state) {
  __shared__ int flag;
  const int64_t t = step_state[0] + 1;
  const double bc1 = 1.0 - pow((double)beta1, (double)t);
  const double bc2 = 1.0 - pow((double)beta2, (double)t);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i];
    float pi = p[i];
    if (wd != 0.f) gi = gi + wd * pi;
    float mi = m[i];
    mi = mi + (1.f - beta1) * (gi - mi);  // exp_avg.lerp_(grad, 1 - beta1)
    float vi = v[i] * beta2 + (1.f - beta2) * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi + (-step_size) * mi / denom;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
  // last arriver advances the step counter (every workgroup read it before arriving)
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* counter = reinterpret_cast<unsigned*>(step_state + 1);
    const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(step_state), (unsigned long long)t,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  (void)flag;
}

}  // namespace tt

using namespace tt;

extern "C" {

size_t tt_dot_bce_workspace_bytes(int64_t B) {
  const int64_t blocks = std::max<int64_t>(1, ceil_div(B, 1));  // upper bound (G >= 1)
  return align_up(sizeof(float) * (size_t)blocks, 256) + 256;
}

int tt_dot_bce_workspace_init(void* workspace, size_t ws_bytes, int64_t B, void* stream) {
  if (!workspace || ws_bytes < tt_dot_bce_workspace_bytes(B)) return fail(TT_ECAPACITY, "dot_bce: workspace too small");
  if (hipMemsetAsync(workspace, 0, tt_dot_bce_workspace_bytes(B), as_stream(stream)) != hipSuccess)
    return fail(TT_EINVAL, "dot_bce: memset failed");
  return TT_OK;
}

int tt_dot_bce_fwd_bwd(const float* q, int64_t ldq, const float* c, int64_t ldc, int64_t B, int dim,
                       const void* labels, int label_dtype, float* logits, float* loss, float* dq, int64_t lddq,
                       float* dc, int64_t lddc, float grad_scale, void* workspace, size_t ws_bytes,
                       void* stream) {
  if (B < 1 || dim < 1 || dim > 1024) return fail(TT_EINVAL, "dot_bce: B >= 1 and 1 <= dim <= 1024 required");
  if (!q || !c || !labels || !logits || !loss) return fail(TT_EINVAL, "dot_bce: null pointer");
  if ((dq == nullptr) != (dc == nullptr)) return fail(TT_EINVAL, "dot_bce: dq and dc must both be set or null");
  if (label_dtype != TT_I32 && label_dtype != TT_I64 && label_dtype != TT_F32)
    return fail(TT_EINVAL, "dot_bce: labels must be int32/int64/float32");
  if (!workspace || ws_bytes < tt_dot_bce_workspace_bytes(B)) return fail(TT_ECAPACITY, "dot_bce: workspace too small");
  int G = 1;
  while (G * 4 < dim && G < 64) G <<= 1;
  const int64_t blocks = ceil_div(B, 256 / G);
  float* partials = reinterpret_cast<float*>(workspace);
  unsigned* counter =
      reinterpret_cast<unsigned*>(reinterpret_cast<char*>(workspace) + align_up(sizeof(float) * (size_t)B, 256));
  dot_bce_kernel<<<dim3((unsigned)blocks), dim3(256), 0, as_stream(stream)>>>(
      q, ldq, c, ldc, B, dim, G, labels, label_dtype, logits, loss, dq, lddq, dc, lddc, grad_scale, partials,
      counter);
  return check_launch("dot_bce_fwd_bwd");
}

int tt_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, int64_t n, float lr,
                 float beta1, float beta2, float eps, float weight_decay, int64_t* step_state, void* stream) {
  if (n < 1) return TT_OK;
  if (!params || !grads || !exp_avg || !exp_avg_sq || !step_state) return fail(TT_EINVAL, "adam: null pointer");
  const int grid = (int)std::min<int64_t>(1024, ceil_div(n, 256));
  adam_kernel<<<dim3(grid), dim3(256), 0, as_stream(stream)>>>(params, grads, exp_avg, exp_avg_sq, n, lr, beta1,
                                                               beta2, eps, weight_decay, step_state);
  return check_launch("adam_step");
}

}  // extern "C"

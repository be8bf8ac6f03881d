// EXPERIMENT: the row-wise Adagrad's random read-modify-write ceiling at config 5's shape (~653k
// distinct 512-B fp32 rows of a 76.8 GB table + their fp32 state, each updated once from a gradient
// row read in lookup order), against bwd_adagrad_direct_kernel (202 us in the sharded world-1 step,
// profiles/r04_config5_sharded_w1_kernel_stats.csv). A half-wave per row, R rows in flight per
// half-wave (all loads of a round issued before the first use), grid-stride over the rows.
// Reported: us and GB/s of table bytes (512 B read + 512 B written per row) and of all bytes
// (+ 8 B state + 512 B gradient read).
// Build + run: hipcc --offload-arch=gfx950 -O3 scripts/micro_rmw.hip -o scripts/micro_rmw.bin && scripts/micro_rmw.bin
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

template <int R, bool IDS_AHEAD>
__global__ void __launch_bounds__(256) k_rmw(float* __restrict__ tab, float* __restrict__ st,
                                             const int32_t* __restrict__ ids, const float* __restrict__ g, int n,
                                             float lr) {
  const int lane = threadIdx.x & 63, pc = lane & 31;
  const int hw0 = (blockIdx.x * 256 + threadIdx.x) >> 5, nhw = gridDim.x * 8;
  int64_t idn[R];
  if (IDS_AHEAD) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int j = hw0 + nhw * u;
      idn[u] = j < n ? ids[j] : 0;
    }
  }
  for (int j0 = hw0; j0 < n; j0 += nhw * R) {
    int64_t id[R];
    f4 w[R], gv[R];
    float s[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int j = j0 + nhw * u;
      id[u] = IDS_AHEAD ? idn[u] : (j < n ? ids[j] : 0);
    }
    if (IDS_AHEAD) {  // the next round's ids in flight beside this round's rows
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int j = j0 + nhw * (R + u);
        idn[u] = j < n ? ids[j] : 0;
      }
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int j = j0 + nhw * u;
      const bool on = j < n;
      w[u] = on ? *reinterpret_cast<const f4*>(tab + id[u] * 128 + pc * 4) : (f4)(0.f);
      s[u] = on ? st[id[u]] : 0.f;
      gv[u] = on ? *reinterpret_cast<const f4*>(g + (int64_t)j * 128 + pc * 4) : (f4)(0.f);
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int j = j0 + nhw * u;
      float sq = gv[u][0] * gv[u][0] + gv[u][1] * gv[u][1] + gv[u][2] * gv[u][2] + gv[u][3] * gv[u][3];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
      const float sn = s[u] + sq / 128.f;
      const float step = -lr / (sqrtf(sn) + 1e-10f);
      if (j < n) {
        f4 x = w[u];
#pragma unroll
        for (int v = 0; v < 4; ++v) x[v] = fmaf(gv[u][v], step, x[v]);
        *reinterpret_cast<f4*>(tab + id[u] * 128 + pc * 4) = x;
        if (pc == 0) st[id[u]] = sn;
      }
    }
  }
}

int main() {
  const int64_t rows = 150000000ll;
  const int n = 653000, NSET = 4;
  float *tab, *st, *g;
  CHECK(hipMalloc(&tab, (size_t)rows * 512));
  CHECK(hipMemset(tab, 0, (size_t)rows * 512));
  CHECK(hipMalloc(&st, (size_t)rows * 4));
  CHECK(hipMemset(st, 0, (size_t)rows * 4));
  CHECK(hipMalloc(&g, (size_t)n * 512));
  CHECK(hipMemset(g, 0, (size_t)n * 512));
  std::mt19937_64 rng(5);
  std::vector<int32_t*> sets(NSET);
  for (auto& d : sets) {
    std::vector<int32_t> h(n);
    for (auto& x : h) x = (int32_t)(rng() % (uint64_t)rows);  // ~distinct at this density
    CHECK(hipMalloc(&d, (size_t)n * 4));
    CHECK(hipMemcpy(d, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  }
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) -> int {
    launch(0);
    CHECK(hipDeviceSynchronize());
    const int reps = 12;
    CHECK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) launch(i);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-28s %8.2f us  table r+w %6.0f GB/s  all bytes %6.0f GB/s\n", name, ms * 1e3, (double)n * 1024 / ms / 1e6,
           (double)n * (1024 + 8 + 512) / ms / 1e6);
    return 0;
  };
#define RMW(R_, AHEAD_, WGS_)                                                                              \
  if (run("rmw R=" #R_ " ahead=" #AHEAD_ " wgs=" #WGS_,                                                    \
          [&](int i) { k_rmw<R_, AHEAD_><<<WGS_, 256>>>(tab, st, sets[i % NSET], g, n, 0.01f); }))          \
    return 1;
  RMW(1, false, 20408)
  RMW(2, false, 10204)
  RMW(4, false, 5102)
  RMW(4, false, 2048)
  RMW(8, false, 2551)
  RMW(8, false, 1024)
  RMW(4, true, 2048)
  RMW(8, true, 1024)
  RMW(4, true, 4096)
  return 0;
}

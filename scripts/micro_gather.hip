// EXPERIMENT: random 512-B row gather (16,384 rows, one half-wave per row, like the embedding
// update) from tables of different sizes — isolates the cost of address translation on random rows.
// Build + run on the box: hipcc --offload-arch=gfx950 -O3 scripts/micro_gather.hip -o /tmp/mg && rocprofv3 --kernel-trace ... -- /tmp/mg
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_gather(const float* __restrict__ tab, const int64_t* __restrict__ rows, float* __restrict__ out, int n) {
  const int hw = (blockIdx.x * blockDim.x + threadIdx.x) >> 5, hl = threadIdx.x & 31;
  if (hw < n) {
    const int64_t r = rows[hw];
    const f4 v = *reinterpret_cast<const f4*>(tab + r * 128 + hl * 4);
    *reinterpret_cast<f4*>(out + (int64_t)hw * 128 + hl * 4) = v;
  }
}

// read-modify-write of the random rows (the update's weight row pattern)
__global__ void k_rmw(float* __restrict__ tab, const int64_t* __restrict__ rows, const float* __restrict__ g, int n) {
  const int hw = (blockIdx.x * blockDim.x + threadIdx.x) >> 5, hl = threadIdx.x & 31;
  if (hw < n) {
    const int64_t r = rows[hw];
    f4 v = *reinterpret_cast<const f4*>(tab + r * 128 + hl * 4);
    v += *reinterpret_cast<const f4*>(g + (int64_t)hw * 128 + hl * 4);
    *reinterpret_cast<f4*>(tab + r * 128 + hl * 4) = v;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 16384;  // rows per launch (654342: config 5 multi-hot scale)
  const int64_t sizes_rows[] = {1ll << 17, 1ll << 21, 1ll << 24, 1ll << 26, 150000000ll};  // 64 MB .. 76.8 GB
  float* out;
  int64_t* rows;
  hipMalloc(&out, (size_t)n * 512);
  hipMalloc(&rows, (size_t)n * 8);
  hipEvent_t e0, e1, e2;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventCreate(&e2);
  std::mt19937_64 rng(1);
  for (int64_t R : sizes_rows) {
    float* tab = nullptr;
    if (hipMalloc(&tab, (size_t)R * 512) != hipSuccess) {
      printf("alloc %lld rows failed\n", (long long)R);
      continue;
    }
    hipMemset(tab, 0, (size_t)R * 512);
    std::vector<int64_t> h(n);
    for (auto& x : h) x = (int64_t)(rng() % (uint64_t)R);
    hipMemcpy(rows, h.data(), (size_t)n * 8, hipMemcpyHostToDevice);
    float tg = 0.f, tr = 0.f;
    const int reps = 20;
    for (int rep = 0; rep < reps + 2; ++rep) {
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k_gather, dim3((unsigned)((int64_t)n * 32 / 256)), dim3(256), 0, 0, tab, rows, out, n);
      hipEventRecord(e1, 0);
      hipLaunchKernelGGL(k_rmw, dim3((unsigned)((int64_t)n * 32 / 256)), dim3(256), 0, 0, tab, rows, out, n);
      hipEventRecord(e2, 0);
      hipEventSynchronize(e2);
      float a = 0.f, b = 0.f;
      hipEventElapsedTime(&a, e0, e1);
      hipEventElapsedTime(&b, e1, e2);
      if (rep >= 2) {
        tg += a;
        tr += b;
      }
    }
    tg /= reps;
    tr /= reps;
    printf("rows %lld n %d: gather %.1f us (%.0f GB/s of rows), rmw %.1f us (%.0f GB/s of rows r+w)\n", (long long)R, n,
           tg * 1e3, (double)n * 512 / tg / 1e6, tr * 1e3, (double)n * 1024 / tr / 1e6);
    hipFree(tab);
  }
  return 0;
}

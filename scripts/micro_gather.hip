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

int main() {
  const int n = 16384;
  const int64_t sizes_rows[] = {1ll << 17, 1ll << 21, 1ll << 24, 1ll << 26, 150000000ll};  // 64 MB .. 76.8 GB
  float* out;
  int64_t* rows;
  hipMalloc(&out, (size_t)n * 512);
  hipMalloc(&rows, (size_t)n * 8);
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
    hipMemcpy(rows, h.data(), n * 8, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 20; ++rep) {
      hipLaunchKernelGGL(k_gather, dim3(n * 32 / 256), dim3(256), 0, 0, tab, rows, out, n);
      hipLaunchKernelGGL(k_rmw, dim3(n * 32 / 256), dim3(256), 0, 0, tab, rows, out, n);
    }
    hipDeviceSynchronize();
    printf("rows %lld done\n", (long long)R);
    hipFree(tab);
  }
  return 0;
}

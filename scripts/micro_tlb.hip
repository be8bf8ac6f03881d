// Random 512-B row gather (16,384 rows per launch, the north-star step's lookups) from tables of
// growing size: how much of the gather latency is the table's size (TLB reach) rather than HBM.
// One wave per 4 rows, all loads of a wave in flight, rows summed into a per-wave output.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void __launch_bounds__(256) gather(const float* __restrict__ tab, const int64_t* __restrict__ rows,
                                              float* __restrict__ out, int n) {
  const int lane = threadIdx.x & 63, w = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int r0 = w * 4;
  float4 v[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // 2 instructions x 2 rows (32 lanes x 16 B per row)
    const int r = r0 + k * 2 + (lane >> 5);
    v[k] = r < n ? *reinterpret_cast<const float4*>(tab + rows[r] * 128 + (lane & 31) * 4) : make_float4(0, 0, 0, 0);
  }
  float4 s = make_float4(v[0].x + v[1].x, v[0].y + v[1].y, v[0].z + v[1].z, v[0].w + v[1].w);
  if (r0 < n) *reinterpret_cast<float4*>(out + (size_t)w * 256 + lane * 4) = s;
}

int main() {
  const int n = 16384;
  const size_t max_rows = 150000000ull;  // 76.8 GB
  float* tab = nullptr;
  if (hipMalloc(&tab, max_rows * 128 * 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMemset(tab, 0, max_rows * 128 * 4);
  int64_t* rows; float* out;
  hipMalloc(&rows, n * 8 * 64);
  hipMalloc(&out, (size_t)n / 4 * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const size_t sizes[] = {250000, 2000000, 8000000, 32000000, 64000000, 150000000};  // rows: 128 MB .. 76.8 GB
  for (size_t R : sizes) {
    std::vector<int64_t> h(n * 64);
    uint64_t x = 88172645463325252ull;
    for (auto& e : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; e = (int64_t)(x % R); }
    hipMemcpy(rows, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    // 64 different batches, cycled (as the bench's 64 resident batches)
    for (int w = 0; w < 64; ++w) hipLaunchKernelGGL(gather, dim3(n / 16), dim3(256), 0, 0, tab, rows + w * n, out, n);
    hipDeviceSynchronize();
    hipEventRecord(a);
    const int iters = 256;
    for (int it = 0; it < iters; ++it)
      hipLaunchKernelGGL(gather, dim3(n / 16), dim3(256), 0, 0, tab, rows + (it % 64) * n, out, n);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / iters;
    printf("table %9zu rows (%6.1f GB): %.2f us per 16384-row gather = %.2f TB/s of rows\n", R, R * 512.0 / 1e9, us,
           n * 512.0 / us / 1e6);
  }
  return 0;
}

// EXPERIMENT: workgroup start spread (s_memrealtime of each workgroup's first wave) for 256
// workgroups of various shapes: threads x LDS bytes x VGPR pressure. Prints p50/p90/max start
// relative to the earliest workgroup, in us (100 MHz counter).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int THREADS, int LDS, int NV>
__global__ void __launch_bounds__(THREADS) k_probe(int64_t* st, float* sink) {
  if (threadIdx.x == 0) st[blockIdx.x] = (int64_t)__builtin_amdgcn_s_memrealtime();
  __shared__ float lds[LDS / 4];
  float v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = sink[(threadIdx.x + i * 64) & 1023];
  lds[threadIdx.x % (LDS / 4)] = v[0];
  __syncthreads();
  float s = lds[(threadIdx.x + 1) % (LDS / 4)];
#pragma unroll
  for (int i = 0; i < NV; ++i) s += v[i] * v[(i + 1) % NV];
  if (s == 12345.f) sink[0] = s;
}

template <int THREADS, int LDS, int NV>
void run(const char* name, int64_t* st, float* sink, int grid) {
  std::vector<int64_t> h(grid);
  std::vector<double> rel;
  for (int rep = 0; rep < 6; ++rep) {
    hipLaunchKernelGGL((k_probe<THREADS, LDS, NV>), dim3(grid), dim3(THREADS), 0, 0, st, sink);
    hipDeviceSynchronize();
  }
  hipMemcpy(h.data(), st, grid * 8, hipMemcpyDeviceToHost);
  const int64_t t0 = *std::min_element(h.begin(), h.end());
  for (auto x : h) rel.push_back((x - t0) * 0.01);
  std::sort(rel.begin(), rel.end());
  printf("%-28s grid %4d: start p50 %.2f p90 %.2f max %.2f us\n", name, grid, rel[grid / 2], rel[grid * 9 / 10], rel[grid - 1]);
}

int main() {
  int64_t* st;
  float* sink;
  hipMalloc(&st, 8 * 4096);
  hipMalloc(&sink, 4096 * 4);
  hipMemset(sink, 0, 4096 * 4);
  run<576, 86272, 8>("576 thr, 86 KB LDS, low vgpr", st, sink, 256);
  run<576, 86272, 128>("576 thr, 86 KB LDS, 128 vgpr", st, sink, 256);
  run<512, 86272, 128>("512 thr, 86 KB LDS, 128 vgpr", st, sink, 256);
  run<576, 1024, 128>("576 thr, 1 KB LDS, 128 vgpr", st, sink, 256);
  run<576, 1024, 8>("576 thr, 1 KB LDS, low vgpr", st, sink, 256);
  run<256, 1024, 8>("256 thr, 1 KB LDS, low vgpr", st, sink, 256);
  run<256, 1024, 8>("256 thr, 1 KB LDS, low vgpr", st, sink, 2048);
  run<256, 30720, 64>("256 thr, 30 KB LDS, 64 vgpr", st, sink, 1024);
  return 0;
}

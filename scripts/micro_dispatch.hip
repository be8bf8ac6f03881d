// EXPERIMENT: workgroup dispatch floor on MI355X — near-empty kernels of various grids, timed by
// rocprofv3 --kernel-trace. Build: hipcc --offload-arch=gfx950 -O3 scripts/micro_dispatch.hip -o build/micro_dispatch
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1;
}

// one dependent global load per thread (latency probe), then a store
__global__ void k_load(const float* __restrict__ x, float* __restrict__ y, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = x[i] * 2.f;
}

int main() {
  int* p;
  float *x, *y;
  hipMalloc(&p, 64);
  hipMalloc(&x, 64 << 20);
  hipMalloc(&y, 64 << 20);
  hipMemset(x, 0, 64 << 20);
  const int grids[] = {256, 512, 1024, 2048, 4096};
  for (int rep = 0; rep < 20; ++rep)
    for (int g : grids) {
      hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, 0, p);
      hipLaunchKernelGGL(k_load, dim3(g), dim3(256), 0, 0, x, y, g * 256);
    }
  for (int rep = 0; rep < 20; ++rep) {
    hipLaunchKernelGGL(k_empty, dim3(256), dim3(576), 0, 0, p);
    hipLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, 0, p);
    hipLaunchKernelGGL(k_empty, dim3(2048), dim3(64), 0, 0, p);
  }
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}

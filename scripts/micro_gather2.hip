// Random-row gather ceiling on MI355X for the north-star step's shapes:
// 512-B fp32 rows (D = 128) from a 76.8 GB table (150M rows, the north star's two tables) and from a
// 128 MB one (Infinity-Cache resident) for contrast; 16,384 rows per launch (one north-star step's
// lookups), 65,536 and 654,336 (config 5's per-step lookups).
//
// Forms (MI355X_MICROARCH.md "Indexed rows: gather into LDS"):
//   reg  : a wave owns R rows; its R ids come in one coalesced load (lane j < R), broadcast by
//          readlane; R / 2 instructions of 16 B per lane (a half-wave per 512-B row) are issued back to
//          back, then consumed (summed) — R rows in flight per wave
//   lds  : the same, each instruction an LDS-DMA (global_load_lds_dwordx4) into a per-wave LDS tile
//   hash : as reg, the row index computed from the lookup's position (no id load: isolates the rows)
// Waves per CU follow from the grid: n / R waves over 256 CUs, 256-thread workgroups.
// Every launch reads a different random id set (64 sets: 64 x 8.4 MB > the 256 MB Infinity Cache at
// n = 16,384), so rows are HBM reads (plus L2/IC hits the table size allows).
// Reported per launch: device time (HIP events around each launch, median of the set) and row GB/s,
// and the back-to-back rate (64 launches between two events: launch gaps hidden).
//
// Build + run on the box:
//   hipcc --offload-arch=gfx950 -O3 scripts/micro_gather2.hip -o /tmp/mg2 && /tmp/mg2
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);      \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// MODE 0 = reg, 1 = lds, 2 = hash
template <int R, int MODE>
__global__ void __launch_bounds__(256) k_gather(const float* __restrict__ tab, int64_t nrows,
                                                const int64_t* __restrict__ ids, int n, uint64_t salt,
                                                float* __restrict__ out) {
  static_assert(R % 2 == 0 && R <= 64, "rows per wave");
  __shared__ __attribute__((aligned(16))) char tile[MODE == 1 ? 4 * R * 512 : 16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * 4 + wid;
  const int64_t r0 = wave * R;
  if (r0 >= n) return;
  int64_t myid = 0;
  if (MODE == 2) {
    myid = (int64_t)(mix((uint64_t)(r0 + (lane % R)) ^ salt) % (uint64_t)nrows);
  } else {
    myid = lane < R && r0 + lane < n ? ids[r0 + lane] : 0;
  }
  const int half = lane >> 5, pc = lane & 31;
  f4 acc = (f4)(0.f);
  if (MODE == 1) {
    char* t = tile + wid * R * 512;
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {
      const int64_t row = __shfl((long long)myid, 2 * i + half, 64);
      __builtin_amdgcn_global_load_lds((glb_void*)(tab + row * 128 + 4 * pc), (lds_void*)(t + i * 1024), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's DMAs landed (it reads only its own rows)
#pragma unroll
    for (int i = 0; i < R / 2; ++i) acc += *reinterpret_cast<const f4*>(t + i * 1024 + lane * 16);
  } else {
    f4 v[R / 2];
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {
      const int64_t row = __shfl((long long)myid, 2 * i + half, 64);
      v[i] = *reinterpret_cast<const f4*>(tab + row * 128 + 4 * pc);
    }
#pragma unroll
    for (int i = 0; i < R / 2; ++i) acc += v[i];
  }
  const float s = acc[0] + acc[1] + acc[2] + acc[3];
  if (s == 12345.f) out[wave] = s;  // keeps the loads; never true (table is zero)
}

template <int R, int MODE>
static int run(const char* name, const float* tab, int64_t nrows, const std::vector<int64_t*>& sets, int n,
               float* out, hipEvent_t* ev, int nev) {
  const int64_t waves = (n + R - 1) / R;
  const dim3 grid((unsigned)((waves + 3) / 4)), blk(256);
  // warm (code, TLB of the index arrays)
  for (int i = 0; i < 4; ++i) k_gather<R, MODE><<<grid, blk>>>(tab, nrows, sets[i % sets.size()], n, i, out);
  CHECK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int i = 0; i < nev - 1 && i < (int)sets.size(); ++i) {
    CHECK(hipEventRecord(ev[i], 0));
    k_gather<R, MODE><<<grid, blk>>>(tab, nrows, sets[i], n, 1000 + i, out);
    CHECK(hipEventRecord(ev[i + 1], 0));
    CHECK(hipEventSynchronize(ev[i + 1]));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const float med = t[t.size() / 2];
  // back to back
  CHECK(hipEventRecord(ev[0], 0));
  for (size_t i = 0; i < sets.size(); ++i)
    k_gather<R, MODE><<<grid, blk>>>(tab, nrows, sets[i], n, 5000 + i, out);
  CHECK(hipEventRecord(ev[1], 0));
  CHECK(hipEventSynchronize(ev[1]));
  float tot = 0.f;
  CHECK(hipEventElapsedTime(&tot, ev[0], ev[1]));
  const float b2b = tot / sets.size();
  const double bytes = (double)n * 512;
  printf("%-5s R=%2d waves/CU=%5.1f n=%7d table=%6.1f GB: launch %7.2f us (%5.0f GB/s)  back-to-back %7.2f us (%5.0f GB/s)\n",
         name, R, (double)waves / 256, n, nrows * 512.0 / 1e9, med * 1e3, bytes / med / 1e6, b2b * 1e3,
         bytes / b2b / 1e6);
  return 0;
}

int main(int argc, char** argv) {
  const int64_t big = 150000000ll, small = 1ll << 18;  // 76.8 GB (north star), 134 MB
  const int ns[] = {16384, 65536, 654336};
  float* tab = nullptr;
  CHECK(hipMalloc(&tab, (size_t)big * 512));
  CHECK(hipMemset(tab, 0, (size_t)big * 512));
  float* out;
  CHECK(hipMalloc(&out, 1 << 24));
  hipEvent_t ev[80];
  for (auto& e : ev) CHECK(hipEventCreate(&e));
  std::mt19937_64 rng(1);
  for (int64_t nrows : {big, small}) {
    for (int n : ns) {
      const int nsets = n >= 654336 ? 8 : 64;
      std::vector<int64_t*> sets(nsets);
      std::vector<int64_t> h(n);
      for (auto& s : sets) {
        for (auto& x : h) x = (int64_t)(rng() % (uint64_t)nrows);
        CHECK(hipMalloc(&s, (size_t)n * 8));
        CHECK(hipMemcpy(s, h.data(), (size_t)n * 8, hipMemcpyHostToDevice));
      }
      const float* tb = tab;  // the small table is the first 134 MB of the big one
      if (run<2, 0>("reg", tb, nrows, sets, n, out, ev, 80)) return 1;
      if (run<4, 0>("reg", tb, nrows, sets, n, out, ev, 80)) return 1;
      if (run<8, 0>("reg", tb, nrows, sets, n, out, ev, 80)) return 1;
      if (run<16, 0>("reg", tb, nrows, sets, n, out, ev, 80)) return 1;
      if (run<4, 1>("lds", tb, nrows, sets, n, out, ev, 80)) return 1;
      if (run<8, 1>("lds", tb, nrows, sets, n, out, ev, 80)) return 1;
      if (run<16, 1>("lds", tb, nrows, sets, n, out, ev, 80)) return 1;
      if (run<4, 2>("hash", tb, nrows, sets, n, out, ev, 80)) return 1;
      if (run<8, 2>("hash", tb, nrows, sets, n, out, ev, 80)) return 1;
      for (auto s : sets) CHECK(hipFree(s));
      fflush(stdout);
    }
  }
  return 0;
}

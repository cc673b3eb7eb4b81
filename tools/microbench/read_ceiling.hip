// Microbenchmark: the HBM read ceiling for the statistics kernels' byte count.
//
// The C2 statistics read 262144 padded rows of 8192 B (2.15 GB; 2000 of 2048
// floats per row are data) at 0.30 ms = 0.87 of 8 TB/s.  What does a kernel
// that only reads (a float sum, nothing written but one value per block) reach
// on the same bytes?
//   gs<U>/<B>   grid-stride, 16-B loads, U loads in flight per lane, B blocks per CU
//   blk<U>      one block per 64-KiB slice, U loads in flight per lane
//   row         one wave per 8192-B row, 8 x 16-B loads per lane (the rows
//               kernel's access shape, data part of the row only: 8000 B)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench/readc.bin tools/microbench/read_ceiling.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef __attribute__((ext_vector_type(4))) float f4;

__device__ __forceinline__ float hsum(f4 v) { return (v.x + v.y) + (v.z + v.w); }

template <int U>
__global__ void __launch_bounds__(256) k_gs(const f4* __restrict__ s, uint64_t n, float* out) {
  f4 acc = {0, 0, 0, 0};
  const uint64_t step = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n; i += step) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = (i + u * 256 < n) ? __builtin_nontemporal_load(s + i + u * 256) : f4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  const float r = hsum(acc);
  if (r == 123.456f) out[blockIdx.x] = r;  // keeps the loads, writes nothing in practice
}

template <int U>
__global__ void __launch_bounds__(256) k_blk(const f4* __restrict__ s, uint64_t n, float* out) {
  // 64 KiB = 4096 vectors per block: 16 per lane, in U-deep batches
  const uint64_t base = (uint64_t)blockIdx.x * 4096;
  f4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 16; k += U) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (uint64_t)(k + u) * 256 + threadIdx.x;
      v[u] = i < n ? __builtin_nontemporal_load(s + i) : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  const float r = hsum(acc);
  if (r == 123.456f) out[blockIdx.x] = r;
}

// one wave per 8192-B row (512 vectors, 500 of them data), 4 waves per block
__global__ void __launch_bounds__(256) k_row(const f4* __restrict__ s, uint64_t rows, float* out) {
  const uint64_t row = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const int lane = threadIdx.x % 64;
  if (row >= rows) return;
  const f4* p = s + row * 512;
  f4 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int j = k * 64 + lane;
    v[k] = j < 500 ? __builtin_nontemporal_load(p + j) : f4{0, 0, 0, 0};
  }
  f4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 8; ++k) acc += v[k];
  const float r = hsum(acc);
  if (r == 123.456f) out[row] = r;
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t rows = 262144, nbytes = rows * 8192, n = nbytes / 16;
  f4* src;
  float* out;
  CK(hipMalloc(&src, nbytes));
  CK(hipMalloc(&out, rows * 4));
  CK(hipMemset(src, 0, nbytes));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct Var { const char* name; int kind; int a; };
  std::vector<Var> vars = {{"gs1/8", 1, 8}, {"gs4/8", 4, 8}, {"gs4/16", 4, 16}, {"gs8/8", 8, 8},
                           {"gs8/4", 8, 4}, {"gs4/32", 4, 32}, {"blk4", 14, 0}, {"blk8", 18, 0},
                           {"blk16", 116, 0}, {"row", 20, 0}};
  for (int rep = 0; rep < 3; ++rep) {
    for (const Var& v : vars) {
      auto launch = [&]() {
        switch (v.kind) {
          case 1: k_gs<1><<<ncu * v.a, 256>>>(src, n, out); break;
          case 4: k_gs<4><<<ncu * v.a, 256>>>(src, n, out); break;
          case 8: k_gs<8><<<ncu * v.a, 256>>>(src, n, out); break;
          case 14: k_blk<4><<<(int)(n / 4096), 256>>>(src, n, out); break;
          case 18: k_blk<8><<<(int)(n / 4096), 256>>>(src, n, out); break;
          case 116: k_blk<16><<<(int)(n / 4096), 256>>>(src, n, out); break;
          default: k_row<<<(int)(rows / 4), 256>>>(src, rows, out); break;
        }
      };
      launch();
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      std::vector<float> ms;
      for (int i = 0; i < 9; ++i) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float m; CK(hipEventElapsedTime(&m, e0, e1)); ms.push_back(m);
      }
      std::sort(ms.begin(), ms.end());
      const double med = ms[ms.size() / 2];
      const double bytes = v.kind == 20 ? rows * 8000.0 : (double)nbytes;
      printf("rep %d  %-7s median %7.4f ms  min %7.4f  %7.1f GB/s (%.3f of 8 TB/s)\n", rep, v.name, med, ms[0],
             bytes / med / 1e6, bytes / med / 1e6 / 8000.0);
      fflush(stdout);
    }
  }
  return 0;
}

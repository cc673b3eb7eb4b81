// Microbenchmark: C5's .T (float64 64^5, every axis reversed) as a 32 (e) x
// 64 (a) tile transpose, the product's k_transpose<u64,32,64> layout.  Source
// rows (a) and destination rows (e) are 128 MiB apart; a tile touches 64
// source and 32 destination 2-MiB pages, and the r02 counters show two thirds
// of its read requests missing the UTCL1 (profiles/r02_kernel_counters.md).
// Variants:
//   base/O0   one tile per block, tiles in the product's order (ta, then the
//             batch dim b -- 2 MiB in the source -- fastest)
//   base/O1   one tile per block, batch dim c fastest (32 KiB on both sides:
//             consecutive tiles share all their pages)
//   pipe/M    persistent blocks, each walking M consecutive O1 tiles (the same
//             pages) with the next tile's loads in flight during the current
//             tile's stores (register prefetch, as k_transpose_pkp)
//   pipe/gs   the same prefetching block, grid-stride over O0 tiles
//   copy      a float4 copy of the same bytes (the box's ceiling)
// Outputs compared with base/O0's on the device (whole array).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench/tc5t.bin tools/microbench/transpose_c5t.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
#include <dlfcn.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef __attribute__((ext_vector_type(2))) double d2;
typedef __attribute__((ext_vector_type(4))) float f4;

constexpr int64_t S4 = 1LL << 24, S3 = 1LL << 18, S2 = 1LL << 12, S1 = 1LL << 6;
constexpr uint64_t NT = 2ull << 18;  // 2 tiles per batch element, 64^3 batch elements

template <int ORDER>
__device__ __forceinline__ void coords(uint64_t t, int64_t& so, int64_t& dof) {
  const int ta = (int)(t & 1);
  const uint64_t r = t >> 1;
  int64_t b, c, d;
  if (ORDER == 0) { b = r & 63; c = (r >> 6) & 63; d = r >> 12; }
  else { c = r & 63; b = (r >> 6) & 63; d = r >> 12; }
  so = b * S3 + c * S2 + d * S1 + ta * 32;          // + a * S4
  dof = d * S3 + c * S2 + b * S1 + ta * 32 * S4;    // + e_local * S4
}

struct Tile {
  d2 v[4];
};

__device__ __forceinline__ void tload(const double* __restrict__ src, int64_t so, Tile& T) {
  const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    T.v[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(src + so + (int64_t)(ty + 16 * j) * S4 + tx * 2));
}

__device__ __forceinline__ void twrite(double (*tile)[33], const Tile& T) {
  const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    tile[ty + 16 * j][tx * 2] = T.v[j].x;
    tile[ty + 16 * j][tx * 2 + 1] = T.v[j].y;
  }
}

__device__ __forceinline__ void tstore(double (*tile)[33], double* __restrict__ dst, int64_t dof) {
  const int ux = threadIdx.x % 32, uy = threadIdx.x / 32;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i = uy + 8 * it;
    d2 w;
    w.x = tile[ux * 2][i];
    w.y = tile[ux * 2 + 1][i];
    __builtin_nontemporal_store(w, reinterpret_cast<d2*>(dst + dof + (int64_t)i * S4 + ux * 2));
  }
}

template <int ORDER>
__global__ void __launch_bounds__(256) k_base(const double* __restrict__ src, double* __restrict__ dst) {
  __shared__ double tile[64][33];
  int64_t so, dof;
  coords<ORDER>(blockIdx.x, so, dof);
  Tile T;
  tload(src, so, T);
  twrite(tile, T);
  __syncthreads();
  tstore(tile, dst, dof);
}

// M > 0: block k walks O1 tiles [k*M, k*M + M); M == 0: grid-stride over O0 tiles.
template <int ORDER>
__global__ void __launch_bounds__(256) k_pipe(const double* __restrict__ src, double* __restrict__ dst, int M) {
  __shared__ double tile[64][33];
  uint64_t t, end, step;
  if (M > 0) { t = (uint64_t)blockIdx.x * M; end = t + M; step = 1; }
  else { t = blockIdx.x; end = NT; step = gridDim.x; }
  if (end > NT) end = NT;
  if (t >= end) return;
  Tile T;
  int64_t so, dof;
  coords<ORDER>(t, so, dof);
  tload(src, so, T);
  for (; t < end; t += step) {
    twrite(tile, T);
    __syncthreads();
    int64_t dcur;
    coords<ORDER>(t, so, dcur);
    const uint64_t tn = t + step;
    if (tn < end) {
      coords<ORDER>(tn, so, dof);
      tload(src, so, T);  // in flight during this tile's stores
    }
    tstore(tile, dst, dcur);
    __syncthreads();
  }
}

__global__ void k_copy(const f4* __restrict__ s, f4* __restrict__ d, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

__global__ void k_cmp(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint64_t n,
                      unsigned long long* bad) {
  unsigned long long m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    m += a[i] != b[i];
  if (m) atomicAdd(bad, m);
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = i * 0x9E3779B97F4A7C15ull;
}

int main(int argc, char** argv) {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t n = 1ull << 30;  // 64^5 elements
  double *src, *ref, *dst;
  CK(hipMalloc(&src, n * 8)); CK(hipMalloc(&ref, n * 8)); CK(hipMalloc(&dst, n * 8));
  unsigned long long* bad;
  CK(hipMalloc(&bad, 8));
  k_fill<<<8192, 256>>>((uint64_t*)src, n);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  k_base<0><<<(int)NT, 256>>>(src, ref);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());

  // the product library's bm_permute on the same buffers (argv[1]: path to libbolt_mi355x.so)
  typedef int (*permute_fn)(const void*, void*, int, const int64_t*, const int32_t*, int, void*);
  permute_fn prod = nullptr;
  if (argc > 1) {
    void* h = dlopen(argv[1], RTLD_NOW);
    if (!h) { printf("dlopen %s: %s\n", argv[1], dlerror()); return 1; }
    prod = (permute_fn)dlsym(h, "bm_permute");
  }
  const int64_t shp[5] = {64, 64, 64, 64, 64};
  const int32_t prm[5] = {4, 3, 2, 1, 0};
  struct Var { const char* name; int kind; int M; };
  std::vector<Var> vars = {{"base/O0", 0, 0}, {"base/O1", 1, 0}, {"pipe/gs", 2, 0}, {"pipe/8", 3, 8},
                           {"pipe/32", 3, 32}, {"pipe/128", 3, 128}, {"pipe/512", 3, 512}, {"copy", 4, 0}};
  if (prod) vars.insert(vars.begin() + 1, Var{"product", 5, 0});
  for (int rep = 0; rep < 3; ++rep) {
    for (const Var& v : vars) {
      auto launch = [&]() {
        switch (v.kind) {
          case 0: k_base<0><<<(int)NT, 256>>>(src, dst); break;
          case 1: k_base<1><<<(int)NT, 256>>>(src, dst); break;
          case 2: k_pipe<0><<<ncu * 8, 256>>>(src, dst, 0); break;
          case 3: k_pipe<1><<<(int)((NT + v.M - 1) / v.M), 256>>>(src, dst, v.M); break;
          case 4: k_copy<<<ncu * 64, 256>>>((const f4*)src, (f4*)dst, n * 8 / 16); break;
          default:
            if (prod(src, dst, 5, shp, prm, 8, nullptr)) { printf("bm_permute failed\n"); exit(1); }
            break;
        }
      };
      CK(hipMemset(dst, 0, n * 8));
      launch();
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      unsigned long long nb = 0;
      if (v.kind != 4) {
        CK(hipMemset(bad, 0, 8));
        k_cmp<<<8192, 256>>>((const uint64_t*)ref, (const uint64_t*)dst, n, bad);
        CK(hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost));
      }
      std::vector<float> ms;
      for (int i = 0; i < 7; ++i) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float m; CK(hipEventElapsedTime(&m, e0, e1)); ms.push_back(m);
      }
      std::sort(ms.begin(), ms.end());
      const double med = ms[ms.size() / 2];
      printf("rep %d  %-9s median %7.4f ms  min %7.4f  %7.1f GB/s  %s\n", rep, v.name, med, ms[0],
             2.0 * n * 8 / med / 1e6, v.kind == 4 ? "-" : (nb ? "MISMATCH" : "bit-exact"));
      fflush(stdout);
    }
  }
  return 0;
}

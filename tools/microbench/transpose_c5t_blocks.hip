// Microbenchmark: C5's .T (float64 64^5, every axis reversed) with the batch
// walk blocked over the two batch dims that are contiguous on ONE side each.
//
// Tile: 32 (e) x 64 (a), the product's k_transpose<u64,32,64> layout.  The
// batch dims are b, c, d (source [a][b][c][d][e], destination
// [e][d][c][b][a]).  d continues e in the source, b continues a in the
// destination.  The product walks b fastest: the tiles in flight write whole
// 32-KiB (b, a) planes per (e, d, c) but read only 512 B per (a, b, c, d).
// Walking d fastest is the mirror image.  A block of 2^LB b's x 2^LD d's in
// flight gives both sides contiguous runs: 2^LD * 512 B read per (a, b, c) and
// 2^LB * 512 B written per (e, d, c).
//   O0        the product's order (b, then c, then d)
//   B<LB>x<LD> ta fastest, then 2^LB b's, 2^LD d's, the rest of b, of d, then c
//   copy      a float4 copy of the same bytes (the box's ceiling)
// Outputs compared with O0's on the device (whole array).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench/tc5b.bin tools/microbench/transpose_c5t_blocks.hip
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

template <int LB, int LD>
__device__ __forceinline__ void coords(uint64_t t, int64_t& so, int64_t& dof) {
  const int ta = (int)(t & 1);
  uint64_t r = t >> 1;
  int64_t b, c, d;
  if (LB < 0) {  // the product's order
    b = r & 63; c = (r >> 6) & 63; d = r >> 12;
  } else {
    const int64_t blo = r & ((1 << LB) - 1); r >>= LB;
    const int64_t dlo = r & ((1 << LD) - 1); r >>= LD;
    const int64_t bhi = r & ((64 >> LB) - 1); r >>= (6 - LB);
    const int64_t dhi = r & ((64 >> LD) - 1); r >>= (6 - LD);
    c = r & 63;
    b = (bhi << LB) | blo;
    d = (dhi << LD) | dlo;
  }
  so = b * S3 + c * S2 + d * S1 + ta * 32;          // + a * S4
  dof = d * S3 + c * S2 + b * S1 + ta * 32 * S4;    // + e_local * S4
}

template <int LB, int LD>
__global__ void __launch_bounds__(256) k_tile(const double* __restrict__ src, double* __restrict__ dst) {
  __shared__ double tile[64][33];
  int64_t so, dof;
  coords<LB, LD>(blockIdx.x, so, dof);
  const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
  d2 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    v[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(src + so + (int64_t)(ty + 16 * j) * S4 + tx * 2));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    tile[ty + 16 * j][tx * 2] = v[j].x;
    tile[ty + 16 * j][tx * 2 + 1] = v[j].y;
  }
  __syncthreads();
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

typedef void (*launch_fn)(const double*, double*);
template <int LB, int LD>
void launch_tile(const double* s, double* d) { k_tile<LB, LD><<<(int)NT, 256>>>(s, d); }

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
  launch_tile<-1, 0>(src, ref);
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
  struct Var { const char* name; int kind; launch_fn f; };
  std::vector<Var> vars = {
      {"O0", 0, launch_tile<-1, 0>}, {"B6x0", 0, launch_tile<6, 0>}, {"B0x6", 0, launch_tile<0, 6>},
      {"B1x1", 0, launch_tile<1, 1>}, {"B2x2", 0, launch_tile<2, 2>}, {"B3x3", 0, launch_tile<3, 3>},
      {"B4x4", 0, launch_tile<4, 4>}, {"B4x2", 0, launch_tile<4, 2>}, {"B2x4", 0, launch_tile<2, 4>},
      {"B5x1", 0, launch_tile<5, 1>}, {"B3x1", 0, launch_tile<3, 1>}, {"copy", 1, nullptr}};
  if (prod) vars.insert(vars.begin() + 1, Var{"product", 2, nullptr});
  for (int rep = 0; rep < 3; ++rep) {
    for (const Var& v : vars) {
      auto launch = [&]() {
        if (v.kind == 0) v.f(src, dst);
        else if (v.kind == 1) k_copy<<<ncu * 64, 256>>>((const f4*)src, (f4*)dst, n * 8 / 16);
        else if (prod(src, dst, 5, shp, prm, 8, nullptr)) { printf("bm_permute failed\n"); exit(1); }
      };
      CK(hipMemset(dst, 0, n * 8));
      launch();
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      unsigned long long nb = 0;
      if (v.kind != 1) {
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
      printf("rep %d  %-8s median %7.4f ms  min %7.4f  %7.1f GB/s  %s\n", rep, v.name, med, ms[0],
             2.0 * n * 8 / med / 1e6, v.kind == 1 ? "-" : (nb ? "MISMATCH" : "bit-exact"));
      fflush(stdout);
    }
  }
  return 0;
}

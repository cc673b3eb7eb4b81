// Microbenchmark: the row-permuting copy of the C4 swap, uint16
// (10000, 1024, 1024) -> (1024, 10000, 1024) (perm (1, 0, 2): 2-KiB rows kept).
// Variants: the product's grid-stride form at several grid caps, one 16-B
// vector per lane with a grid of all vectors (2-D: x = vectors of a row
// group, y = destination row groups), and XCD-grouped row ranges.  Sampled
// rows are checked against the source.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/rc.bin tools/microbench/rowcopy_c4.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef __attribute__((ext_vector_type(4))) uint32_t u4;

constexpr int64_t K0 = 10000, K1 = 1024, V = 1024;  // uint16
constexpr int64_t VPR = V * 2 / 16;                  // 16-B vectors per row (128)

// product form: grid-stride over all vectors, row = g / VPR, (d1, d0) = row decomposed
__global__ void __launch_bounds__(256) k_gs(const u4* __restrict__ src, u4* __restrict__ dst, uint64_t total) {
  const uint64_t step = (uint64_t)gridDim.x * 256;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += step) {
    const uint64_t row = g / VPR, v = g % VPR;         // destination row (k1, k0)
    const uint64_t k1 = row / K0, k0 = row % K0;
    const u4 x = __builtin_nontemporal_load(src + (k0 * K1 + k1) * VPR + v);
    __builtin_nontemporal_store(x, dst + g);
  }
}

// one vector per lane: block b covers 256 vectors = 2 destination rows
template <int XCD>
__global__ void __launch_bounds__(256) k_one(const u4* __restrict__ src, u4* __restrict__ dst, uint64_t total) {
  uint64_t b = blockIdx.x;
  if (XCD) {
    const uint64_t per = gridDim.x / 8;
    b = (blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  const uint64_t g = b * 256 + threadIdx.x;
  if (g >= total) return;
  const uint64_t row = g / VPR, v = g % VPR;
  const uint64_t k1 = row / K0, k0 = row % K0;
  const u4 x = __builtin_nontemporal_load(src + (k0 * K1 + k1) * VPR + v);
  __builtin_nontemporal_store(x, dst + g);
}

// one vector per lane, source-ordered: consecutive blocks read consecutive source rows
__global__ void __launch_bounds__(256) k_src(const u4* __restrict__ src, u4* __restrict__ dst, uint64_t total) {
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;  // source vector index
  if (g >= total) return;
  const uint64_t row = g / VPR, v = g % VPR;  // source row (k0, k1)
  const uint64_t k0 = row / K1, k1 = row % K1;
  const u4 x = __builtin_nontemporal_load(src + g);
  __builtin_nontemporal_store(x, dst + (k1 * K0 + k0) * VPR + v);
}

// 4 vectors per lane in flight, block covers 1024 vectors (8 rows)
__global__ void __launch_bounds__(256) k_four(const u4* __restrict__ src, u4* __restrict__ dst, uint64_t total) {
  u4 x[4];
  uint64_t gg[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint64_t g = (uint64_t)blockIdx.x * 1024 + u * 256 + threadIdx.x;
    gg[u] = g;
    if (g < total) {
      const uint64_t row = g / VPR, v = g % VPR;
      const uint64_t k1 = row / K0, k0 = row % K0;
      x[u] = __builtin_nontemporal_load(src + (k0 * K1 + k1) * VPR + v);
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (gg[u] < total) __builtin_nontemporal_store(x[u], dst + gg[u]);
}

int main() {
  const uint64_t total = (uint64_t)K0 * K1 * VPR;  // vectors
  const size_t bytes = total * 16;
  u4 *src, *dst;
  CK(hipMalloc(&src, bytes)); CK(hipMalloc(&dst, bytes));
  {
    std::vector<uint16_t> row(V);
    std::vector<uint16_t> h((size_t)K1 * V);
    for (int64_t k0 = 0; k0 < K0; ++k0) {  // row (k0, k1) filled with a pattern of (k0, k1, i)
      for (int64_t k1 = 0; k1 < K1; ++k1)
        for (int64_t i = 0; i < V; ++i) h[k1 * V + i] = (uint16_t)(k0 * 7919 + k1 * 104729 + i * 31);
      CK(hipMemcpy((char*)src + k0 * K1 * V * 2, h.data(), K1 * V * 2, hipMemcpyHostToDevice));
    }
  }
  auto check = [&](const char* name) {
    std::vector<uint16_t> r(V);
    bool ok = true;
    for (int s = 0; s < 64 && ok; ++s) {
      const int64_t k1 = (s * 131) % K1, k0 = (s * 7877) % K0;
      CK(hipMemcpy(r.data(), (char*)dst + (k1 * K0 + k0) * V * 2, V * 2, hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < V; ++i)
        if (r[i] != (uint16_t)(k0 * 7919 + k1 * 104729 + i * 31)) { ok = false; break; }
    }
    if (!ok) printf("%s MISMATCH\n", name);
    return ok;
  };
  struct Var { const char* name; int kind; int grid; std::vector<float> ms; };
  std::vector<Var> vs = {
      {"grid-stride cap 1M (product)", 0, 1 << 20, {}},
      {"grid-stride cap 256K", 0, 1 << 18, {}},
      {"grid-stride cap 4M", 0, 1 << 22, {}},
      {"one vec/lane, all blocks", 1, 0, {}},
      {"one vec/lane, XCD-grouped", 2, 0, {}},
      {"one vec/lane, source order", 3, 0, {}},
      {"four vec/lane", 4, 0, {}},
  };
  auto launch = [&](Var& v) {
    const uint64_t nb1 = (total + 255) / 256;
    switch (v.kind) {
      case 0: k_gs<<<v.grid, 256>>>(src, dst, total); break;
      case 1: k_one<0><<<(unsigned)nb1, 256>>>(src, dst, total); break;
      case 2: k_one<1><<<(unsigned)((nb1 + 7) / 8 * 8), 256>>>(src, dst, total); break;
      case 3: k_src<<<(unsigned)nb1, 256>>>(src, dst, total); break;
      default: k_four<<<(unsigned)((total + 1023) / 1024), 256>>>(src, dst, total); break;
    }
  };
  for (auto& v : vs) {
    CK(hipMemset(dst, 0, bytes));
    launch(v);
    CK(hipDeviceSynchronize());
    check(v.name);
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < 4; ++r)
    for (auto& v : vs) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 3; ++i) launch(v);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / 3);
    }
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    printf("%-34s median %7.3f ms  %7.1f GB/s\n", v.name, med, 2.0 * bytes / (med * 1e-3) / 1e9);
  }
  return 0;
}

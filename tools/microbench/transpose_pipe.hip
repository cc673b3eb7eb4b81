// Microbenchmark: persistent / pipelined / XCD-grouped variants of the f32
// tile transpose on the C2 swap shape [B=2000][A=262144] -> [A][B].
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/tp.bin tools/microbench/transpose_pipe.hip
// Every variant is checked bit-exactly against a host transpose.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef __attribute__((ext_vector_type(4))) uint32_t u4;

// TA along the source-contiguous dim a, TB along the destination-contiguous dim b.
// MODE 0: one tile per block (grid = ntiles), tiles b-fast.
// MODE 1: persistent (grid-stride), register prefetch of the next tile during the store phase.
// MODE 2: like 0 but the block -> tile map groups consecutive tiles on one XCD
//         (block g runs on XCD g % 8 under round-robin dispatch).
// MODE 3: persistent + prefetch + XCD grouping (each XCD walks its own contiguous tile range).
__constant__ int64_t g_chunk;

template <int TA, int TB, int THREADS, int MODE>
__global__ void __launch_bounds__(THREADS) ktp(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                               int64_t La, int64_t Lb, int64_t ntB, int64_t ntiles) {
  __shared__ uint32_t tile[TB][TA + 1];
  constexpr int NVA = TA / 4, RPA = THREADS / NVA, NL = TB / RPA;
  constexpr int NVB = TB / 4, RPB = THREADS / NVB, NS = TA / RPB;
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
  u4 v[NL];
  auto load = [&](int64_t t) {
    const int64_t tb = t % ntB, ta = t / ntB;
    const int64_t a0 = ta * TA, b0 = tb * TB;
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int rb = ty + it * RPA;
      if (b0 + rb < Lb && a0 + tx * 4 < La)
        v[it] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(src + (b0 + rb) * La + a0 + tx * 4));
    }
  };
  auto to_lds = [&]() {
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int rb = ty + it * RPA;
      uint32_t f[4]; __builtin_memcpy(f, &v[it], 16);
#pragma unroll
      for (int k = 0; k < 4; ++k) tile[rb][tx * 4 + k] = f[k];
    }
  };
  auto store = [&](int64_t t) {
    const int64_t tb = t % ntB, ta = t / ntB;
    const int64_t a0 = ta * TA, b0 = tb * TB;
#pragma unroll
    for (int it = 0; it < NS; ++it) {
      const int ra = uy + it * RPB;
      if (a0 + ra < La && b0 + ux * 4 + 3 < Lb) {
        uint32_t f[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) f[k] = tile[ux * 4 + k][ra];
        u4 w; __builtin_memcpy(&w, f, 16);
        __builtin_nontemporal_store(w, reinterpret_cast<u4*>(dst + (a0 + ra) * Lb + b0 + ux * 4));
      } else if (a0 + ra < La) {
        for (int k = 0; k < 4; ++k) if (b0 + ux * 4 + k < Lb) dst[(a0 + ra) * Lb + b0 + ux * 4 + k] = tile[ux * 4 + k][ra];
      }
    }
  };
  if (MODE == 0 || MODE == 2 || MODE == 4) {
    int64_t t = blockIdx.x;
    if (MODE == 2) {  // XCD x gets tiles [x*per, (x+1)*per)
      const int64_t G = gridDim.x, per = (G + 7) / 8;
      const int64_t x = blockIdx.x % 8, k = blockIdx.x / 8;
      t = x * per + k;
      if (t >= ntiles) return;
    }
    if (MODE == 4) {  // chunks of g_chunk tiles dealt to XCDs round-robin
      const int64_t x = blockIdx.x % 8, k = blockIdx.x / 8;
      const int64_t c = k / g_chunk, w = k % g_chunk;
      t = (c * 8 + x) * g_chunk + w;
      if (t >= ntiles) return;
    }
    load(t); to_lds(); __syncthreads(); store(t);
    return;
  }
  // persistent
  int64_t t, step;
  if (MODE == 3) {
    const int64_t G = gridDim.x;            // multiple of 8
    const int64_t x = blockIdx.x % 8, k = blockIdx.x / 8, per = G / 8;
    const int64_t span = (ntiles + 7) / 8;  // XCD x walks tiles [x*span, (x+1)*span)
    t = x * span + k;
    step = per;
    const int64_t end = min(ntiles, (x + 1) * span);
    if (t >= end) return;
    load(t);
    for (; t < end; t += step) {
      to_lds(); __syncthreads();
      if (t + step < end) load(t + step);
      store(t); __syncthreads();
    }
    return;
  }
  t = blockIdx.x; step = gridDim.x;
  if (t >= ntiles) return;
  load(t);
  for (; t < ntiles; t += step) {
    to_lds(); __syncthreads();
    if (t + step < ntiles) load(t + step);
    store(t); __syncthreads();
  }
}

struct Variant {
  const char* name;
  void (*launch)(const uint32_t*, uint32_t*, int64_t, int64_t);
  std::vector<float> ms;
  bool ok;
};

template <int TA, int TB, int THREADS, int MODE>
void launch_v(const uint32_t* src, uint32_t* dst, int64_t La, int64_t Lb) {
  const int64_t ntA = (La + TA - 1) / TA, ntB = (Lb + TB - 1) / TB, ntiles = ntA * ntB;
  int grid = (int)ntiles;
  if (MODE == 2) grid = (int)(((ntiles + 7) / 8) * 8);
  ktp<TA, TB, THREADS, MODE><<<grid, THREADS>>>(src, dst, La, Lb, ntB, ntiles);
}

template <int TA, int TB, int THREADS, int MODE>
Variant V(const char* name) { return Variant{name, &launch_v<TA, TB, THREADS, MODE>, {}, false}; }

__global__ void kcopy4(const u4* __restrict__ s, u4* __restrict__ d, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

__global__ void kcopy1(const u4* __restrict__ s, u4* __restrict__ d, int64_t n, int xcd) {
  int64_t b = blockIdx.x;
  if (xcd) {
    const int64_t per = gridDim.x / 8;
    b = (blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  const int64_t i = b * blockDim.x + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

int main() {
  const int64_t Lb = 2000, La = 262144;
  const int64_t n = La * Lb;
  uint32_t *src, *dst;
  CK(hipMalloc(&src, n * 4)); CK(hipMalloc(&dst, n * 4));
  std::vector<uint32_t> h(n);
  for (int64_t i = 0; i < n; ++i) h[i] = (uint32_t)(i * 2654435761u);
  CK(hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> ref(n);
  for (int64_t b = 0; b < Lb; ++b) for (int64_t a = 0; a < La; ++a) ref[a * Lb + b] = h[b * La + a];
  const int reps = 20;
  {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int g : {4096, 16384, 65536}) {
      kcopy4<<<g, 256>>>((const u4*)src, (u4*)dst, n / 4);
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) kcopy4<<<g, 256>>>((const u4*)src, (u4*)dst, n / 4);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
      printf("copy NT grid %-6d                                         %8.3f ms  %8.1f GB/s\n", g, ms,
             2.0 * n * 4 / (ms * 1e-3) / 1e9);
    }
    for (int x = 0; x < 2; ++x) {
      const int g = (int)(n / 4 / 256);  // multiple of 8
      kcopy1<<<g, 256>>>((const u4*)src, (u4*)dst, n / 4, x);
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) kcopy1<<<g, 256>>>((const u4*)src, (u4*)dst, n / 4, x);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
      printf("copy NT 1 vec/thread %s grid %-7d                     %8.3f ms  %8.1f GB/s\n", x ? "XCD" : "   ", g, ms,
             2.0 * n * 4 / (ms * 1e-3) / 1e9);
    }
  }
  std::vector<Variant> vs = {
      V<64, 64, 256, 0>("64x64 t256 (product)"),
      V<64, 256, 256, 0>("64x256 t256"),
      V<32, 256, 256, 0>("32x256 t256"),
      V<32, 256, 128, 0>("32x256 t128"),
      V<16, 256, 256, 0>("16x256 t256"),
      V<32, 512, 256, 0>("32x512 t256"),
      V<32, 512, 512, 0>("32x512 t512"),
      V<16, 512, 256, 0>("16x512 t256"),
      V<64, 512, 512, 0>("64x512 t512"),
  };
  std::vector<uint32_t> hh(n);
  for (auto& v : vs) {
    CK(hipMemset(dst, 0, n * 4));
    v.launch(src, dst, La, Lb);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hh.data(), dst, n * 4, hipMemcpyDeviceToHost));
    v.ok = memcmp(hh.data(), ref.data(), n * 4) == 0;
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int rounds = 7, rr = 10;
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vs) {
      v.launch(src, dst, La, Lb);
      CK(hipEventRecord(e0));
      for (int i = 0; i < rr; ++i) v.launch(src, dst, La, Lb);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / rr);
    }
  }
  for (auto& v : vs) {
    std::vector<float> m = v.ms;
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2], best = m[0];
    printf("%-30s median %7.4f ms %7.1f GB/s  best %7.4f ms %7.1f GB/s  %s\n", v.name, med,
           2.0 * n * 4 / (med * 1e-3) / 1e9, best, 2.0 * n * 4 / (best * 1e-3) / 1e9, v.ok ? "ok" : "MISMATCH");
  }
  return 0;
}

// Microbenchmark: tile order of the f32 LDS transpose (64 x 256 tiles,
// loads-first) against the source row stride.  [Lb][La] -> [La][Lb] with
// La * 4 B = 512 KiB .. 4 MiB rows; orders: b-fast (product), a-fast, and a
// diagonal walk (tb fast, ta skewed by tb) that spreads concurrent tiles over
// source columns.  Bit-exact check per variant (sampled).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/to.bin tools/microbench/transpose_order.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef __attribute__((ext_vector_type(4))) uint32_t u4;

template <int ORDER>
__global__ void __launch_bounds__(256) kto(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int64_t La,
                                           int64_t Lb, int64_t ntA, int64_t ntB) {
  constexpr int TA = 64, TB = 256, NVA = 16, RPA = 16, NL = 16, NVB = 64, RPB = 4, NS = 16;
  __shared__ uint32_t tile[TB][TA + 1];
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
  const int64_t t = blockIdx.x;
  int64_t ta, tb;
  if (ORDER == 0) { tb = t % ntB; ta = t / ntB; }
  else if (ORDER == 1) { ta = t % ntA; tb = t / ntA; }
  else { tb = t % ntB; ta = (t / ntB + tb * (ntA / ntB + 1)) % ntA; }  // diagonal
  const int64_t a0 = ta * TA, b0 = tb * TB;
  u4 v[NL];
#pragma unroll
  for (int it = 0; it < NL; ++it) {
    const int rb = ty + it * RPA;
    if (b0 + rb < Lb) v[it] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(src + (b0 + rb) * La + a0 + tx * 4));
  }
#pragma unroll
  for (int it = 0; it < NL; ++it) {
    const int rb = ty + it * RPA;
    uint32_t f[4]; __builtin_memcpy(f, &v[it], 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) tile[rb][tx * 4 + k] = f[k];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NS; ++it) {
    const int ra = uy + it * RPB;
    if (b0 + ux * 4 + 3 < Lb) {
      uint32_t f[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) f[k] = tile[ux * 4 + k][ra];
      u4 w; __builtin_memcpy(&w, f, 16);
      __builtin_nontemporal_store(w, reinterpret_cast<u4*>(dst + (a0 + ra) * Lb + b0 + ux * 4));
    } else {
      for (int k = 0; k < 4; ++k) if (b0 + ux * 4 + k < Lb) dst[(a0 + ra) * Lb + b0 + ux * 4 + k] = tile[ux * 4 + k][ra];
    }
  }
}

int main() {
  const int64_t maxn = 2000LL * 524288;
  uint32_t *src, *dst;
  CK(hipMalloc(&src, maxn * 4)); CK(hipMalloc(&dst, maxn * 4));
  std::vector<uint32_t> h(maxn);
  for (int64_t i = 0; i < maxn; ++i) h[i] = (uint32_t)(i * 2654435761u);
  CK(hipMemcpy(src, h.data(), maxn * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct Shape { int64_t Lb, La; };
  for (Shape sh : {Shape{4000, 131072}, Shape{2000, 262144}, Shape{2000, 524288}, Shape{1000, 1048576}}) {
    const int64_t La = sh.La, Lb = sh.Lb, n = La * Lb;
    const int64_t ntA = La / 64, ntB = (Lb + 255) / 256, nt = ntA * ntB;
    float best[3] = {0, 0, 0};
    for (int order = 0; order < 3; ++order) {
      auto launch = [&]() {
        if (order == 0) kto<0><<<(int)nt, 256>>>(src, dst, La, Lb, ntA, ntB);
        else if (order == 1) kto<1><<<(int)nt, 256>>>(src, dst, La, Lb, ntA, ntB);
        else kto<2><<<(int)nt, 256>>>(src, dst, La, Lb, ntA, ntB);
      };
      CK(hipMemset(dst, 0, n * 4));
      launch();
      CK(hipDeviceSynchronize());
      bool ok = true;
      for (int s = 0; s < 200 && ok; ++s) {
        const int64_t a = (s * 7919LL) % La, b = (s * 104729LL) % Lb;
        uint32_t got;
        CK(hipMemcpy(&got, dst + a * Lb + b, 4, hipMemcpyDeviceToHost));
        ok = got == h[b * La + a];
      }
      std::vector<float> ms;
      for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0));
        for (int i = 0; i < 5; ++i) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float m; CK(hipEventElapsedTime(&m, e0, e1));
        ms.push_back(m / 5);
      }
      std::sort(ms.begin(), ms.end());
      printf("rows %5lld KiB  Lb %5lld  order %-8s  median %7.4f ms  %7.1f GB/s  %s\n", (long long)(La * 4 / 1024),
             (long long)Lb, order == 0 ? "b-fast" : order == 1 ? "a-fast" : "diagonal", ms[2],
             2.0 * n * 4 / (ms[2] * 1e-3) / 1e9, ok ? "ok" : "MISMATCH");
      fflush(stdout);
    }
  }
  return 0;
}

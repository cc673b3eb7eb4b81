// Microbenchmark: tile shapes of the LDS transpose per element size.
// [Lb=2000][La] -> [La][Lb] with La*es = 1 MiB rows (2 GB arrays), element
// sizes 1/2/4/8 B; tile TA (source-contiguous) x TB (destination-contiguous),
// 16-B non-temporal loads along a and stores along b, one tile per block.
// Variants run interleaved over rounds (median reported), each checked
// bit-exactly against a host transpose.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/tt.bin tools/microbench/transpose_tiles.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef __attribute__((ext_vector_type(4))) uint32_t u4;

template <typename T, int TA, int TB, int THREADS>
__global__ void __launch_bounds__(THREADS) ktt(const T* __restrict__ src, T* __restrict__ dst, int64_t La, int64_t Lb,
                                               int64_t ntB) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ T tile[TB][TA + 1];
  constexpr int NVA = TA / VEC, RPA = THREADS / NVA, NL = TB / RPA;
  constexpr int NVB = TB / VEC, RPB = THREADS / NVB, NS = TA / RPB;
  static_assert(NL >= 1 && NS >= 1, "tile too small");
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
  const int64_t t = blockIdx.x;
  const int64_t tb = t % ntB, ta = t / ntB;
  const int64_t a0 = ta * TA, b0 = tb * TB;
  u4 v[NL];
#pragma unroll
  for (int it = 0; it < NL; ++it) {  // every load in flight before the first LDS write
    const int rb = ty + it * RPA;
    if (b0 + rb < Lb) v[it] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(src + (b0 + rb) * La + a0 + tx * VEC));
  }
#pragma unroll
  for (int it = 0; it < NL; ++it) {
    const int rb = ty + it * RPA;
    T f[VEC]; __builtin_memcpy(f, &v[it], 16);
#pragma unroll
    for (int k = 0; k < VEC; ++k) tile[rb][tx * VEC + k] = f[k];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NS; ++it) {
    const int ra = uy + it * RPB;
    if (b0 + ux * VEC + VEC - 1 < Lb) {
      T f[VEC];
#pragma unroll
      for (int k = 0; k < VEC; ++k) f[k] = tile[ux * VEC + k][ra];
      u4 w; __builtin_memcpy(&w, f, 16);
      __builtin_nontemporal_store(w, reinterpret_cast<u4*>(dst + (a0 + ra) * Lb + b0 + ux * VEC));
    } else {
      for (int k = 0; k < VEC; ++k) if (b0 + ux * VEC + k < Lb) dst[(a0 + ra) * Lb + b0 + ux * VEC + k] = tile[ux * VEC + k][ra];
    }
  }
}

struct Variant {
  char name[64];
  int es;
  void (*launch)(const void*, void*, int64_t, int64_t);
  std::vector<float> ms;
  bool ok;
};

template <typename T, int TA, int TB, int THREADS>
void launch_v(const void* src, void* dst, int64_t La, int64_t Lb) {
  const int64_t ntB = (Lb + TB - 1) / TB, ntiles = (La / TA) * ntB;
  ktt<T, TA, TB, THREADS><<<(int)ntiles, THREADS>>>((const T*)src, (T*)dst, La, Lb, ntB);
}

template <typename T, int TA, int TB, int THREADS>
Variant V() {
  Variant v;
  snprintf(v.name, sizeof v.name, "es%d %3dx%-4d t%-4d (%4dB rd, %4dB wr, %2dKB)", (int)sizeof(T), TA, TB, THREADS,
           TA * (int)sizeof(T), TB * (int)sizeof(T), (int)(TA * TB * sizeof(T) / 1024));
  v.es = sizeof(T);
  v.launch = &launch_v<T, TA, TB, THREADS>;
  v.ok = false;
  return v;
}

int main() {
  const int64_t Lb = 2000, rowbytes = 1 << 20;
  const int64_t nbytes = Lb * rowbytes;
  char *src, *dst;
  CK(hipMalloc(&src, nbytes)); CK(hipMalloc(&dst, nbytes));
  std::vector<uint8_t> h(nbytes), hh(nbytes), ref(nbytes);
  for (int64_t i = 0; i < nbytes; ++i) h[i] = (uint8_t)((i * 2654435761ull) >> 13);
  CK(hipMemcpy(src, h.data(), nbytes, hipMemcpyHostToDevice));
  std::vector<Variant> vs = {
      V<uint32_t, 64, 256, 256>(),
      V<uint16_t, 128, 256, 256>(), V<uint16_t, 128, 512, 1024>(), V<uint16_t, 128, 512, 512>(),
      V<uint8_t, 128, 256, 256>(),  V<uint8_t, 256, 512, 1024>(),  V<uint8_t, 128, 512, 512>(),
      V<uint8_t, 256, 256, 512>(),
  };
  int cur_es = 0;
  for (auto& v : vs) {
    const int64_t La = rowbytes / v.es;
    if (v.es != cur_es) {  // host reference for this element size
      cur_es = v.es;
      for (int64_t b = 0; b < Lb; ++b)
        for (int64_t a = 0; a < La; ++a) memcpy(&ref[(a * Lb + b) * v.es], &h[(b * La + a) * v.es], v.es);
    }
    CK(hipMemset(dst, 0, nbytes));
    v.launch(src, dst, La, Lb);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hh.data(), dst, nbytes, hipMemcpyDeviceToHost));
    v.ok = memcmp(hh.data(), ref.data(), nbytes) == 0;
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int rounds = 5, rr = 8;
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vs) {
      const int64_t La = rowbytes / v.es;
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
    const double med = m[m.size() / 2];
    printf("%-48s median %7.4f ms %7.1f GB/s  %s\n", v.name, med, 2.0 * nbytes / (med * 1e-3) / 1e9,
           v.ok ? "ok" : "MISMATCH");
  }
  return 0;
}

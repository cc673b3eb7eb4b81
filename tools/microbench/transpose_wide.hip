// Microbenchmark: 2-KiB destination segments for the float32 C2 transpose.
// [Lb=2000][La=262144] f32 -> [La][Lb] (the C2 swap's shape, 8000-B destination
// rows).  The round-1 sweep (profiles/r01_tt2.log) put every float64 tile with
// 2-KiB write segments ahead of the float32 64x256 tile (1-KiB writes) by
// 1.4-2.8%; float32 never had a 2-KiB-write tile because 256 threads cap the
// tile at 64 KiB.  Variants: the shipped 64x256/256 threads, 32x512/256 (128-B
// reads, 2-KiB writes, 2 blocks per CU), 64x512/512 and /1024 (one 133-KB tile
// per CU), 128x256/512; each checked bit-exactly, interleaved over rounds,
// median reported.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/tw.bin tools/microbench/transpose_wide.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef __attribute__((ext_vector_type(4))) uint32_t u4;

template <typename T, int TA, int TB, int THREADS>
__global__ void __launch_bounds__(THREADS) ktw(const T* __restrict__ src, T* __restrict__ dst, int64_t La, int64_t Lb,
                                               int64_t ntB) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ T tile[TB][TA + 1];
  constexpr int NVA = TA / VEC, RPA = THREADS / NVA, NL = TB / RPA;
  constexpr int NVB = TB / VEC, RPB = THREADS / NVB, NS = TA / RPB;
  static_assert(NL >= 1 && NS >= 1 && NVB <= THREADS, "tile too small");
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
  ktw<T, TA, TB, THREADS><<<(int)ntiles, THREADS>>>((const T*)src, (T*)dst, La, Lb, ntB);
}

template <typename T, int TA, int TB, int THREADS>
Variant V() {
  Variant v;
  snprintf(v.name, sizeof v.name, "es%d %3dx%-4d t%-4d (%4dB rd, %4dB wr, %3dKB)", (int)sizeof(T), TA, TB, THREADS,
           TA * (int)sizeof(T), TB * (int)sizeof(T), (int)(TA * TB * sizeof(T) / 1024));
  v.es = sizeof(T);
  v.launch = &launch_v<T, TA, TB, THREADS>;
  v.ok = false;
  return v;
}

int main(int argc, char** argv) {
  const int64_t Lb = 2000, rowbytes = 1 << 20;
  const int64_t nbytes = Lb * rowbytes;
  const int nbuf = argc > 1 ? atoi(argv[1]) : 1;  // source buffers (placements) to cycle through
  std::vector<char*> srcs(nbuf);
  char* dst;
  for (auto& s : srcs) CK(hipMalloc(&s, nbytes));
  CK(hipMalloc(&dst, nbytes));
  std::vector<uint8_t> h(nbytes), hh(nbytes), ref(nbytes);
  for (int64_t i = 0; i < nbytes; ++i) h[i] = (uint8_t)((i * 2654435761ull) >> 13);
  for (auto& s : srcs) CK(hipMemcpy(s, h.data(), nbytes, hipMemcpyHostToDevice));
  std::vector<Variant> vs = {
      V<uint32_t, 64, 256, 256>(), V<uint32_t, 32, 512, 256>(), V<uint32_t, 64, 512, 512>(),
      V<uint32_t, 64, 512, 1024>(), V<uint32_t, 128, 256, 512>(), V<uint64_t, 32, 256, 256>(),
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
    v.launch(srcs[0], dst, La, Lb);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hh.data(), dst, nbytes, hipMemcpyDeviceToHost));
    v.ok = memcmp(hh.data(), ref.data(), nbytes) == 0;
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int rounds = 7, rr = 8;
  for (int b = 0; b < nbuf; ++b) {
    for (auto& v : vs) v.ms.clear();
    for (int r = 0; r < rounds; ++r) {
      for (auto& v : vs) {
        const int64_t La = rowbytes / v.es;
        v.launch(srcs[b], dst, La, Lb);
        CK(hipEventRecord(e0));
        for (int i = 0; i < rr; ++i) v.launch(srcs[b], dst, La, Lb);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        v.ms.push_back(ms / rr);
      }
    }
    printf("source buffer %d\n", b);
    for (auto& v : vs) {
      std::vector<float> m = v.ms;
      std::sort(m.begin(), m.end());
      const double med = m[m.size() / 2];
      printf("  %-50s median %7.4f ms %7.1f GB/s  %s\n", v.name, med, 2.0 * nbytes / (med * 1e-3) / 1e9,
             v.ok ? "ok" : "MISMATCH");
    }
    fflush(stdout);
  }
  return 0;
}

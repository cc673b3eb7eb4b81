// Microbenchmark: variants of the 2-D f32 tile transpose on the C2 swap shape
// [B=2000][A=262144] -> [A][B], against a contiguous copy of the same bytes.
// Build: hipcc -O3 --offload-arch=gfx950 -o tv transpose_variants.hip
// Each variant is checked bit-exactly against the first.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef __attribute__((ext_vector_type(4))) uint32_t u4;

template <int TA, int TB, int THREADS, bool NT, bool BFAST, bool NTL = false>
__global__ void __launch_bounds__(THREADS) ktr(const float* __restrict__ src, float* __restrict__ dst,
                                               int64_t La, int64_t Lb, int64_t ntA, int64_t ntB) {
  __shared__ float tile[TB][TA + 1];
  constexpr int NVA = TA / 4, RPA = THREADS / NVA;
  constexpr int NVB = TB / 4, RPB = THREADS / NVB;
  const int64_t t = blockIdx.x;
  int64_t ta, tb;
  if (BFAST) { tb = t % ntB; ta = t / ntB; } else { ta = t % ntA; tb = t / ntA; }
  const int64_t a0 = ta * TA, b0 = tb * TB;
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
  u4 v[TB / RPA];
#pragma unroll
  for (int it = 0; it < TB / RPA; ++it) {
    const int rb = ty + it * RPA;
    if (b0 + rb < Lb && a0 + tx * 4 < La)
      v[it] = NTL ? __builtin_nontemporal_load(reinterpret_cast<const u4*>(src + (b0 + rb) * La + a0 + tx * 4))
                  : *reinterpret_cast<const u4*>(src + (b0 + rb) * La + a0 + tx * 4);
  }
#pragma unroll
  for (int it = 0; it < TB / RPA; ++it) {
    const int rb = ty + it * RPA;
    float f[4]; __builtin_memcpy(f, &v[it], 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) tile[rb][tx * 4 + k] = f[k];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < TA / RPB; ++it) {
    const int ra = uy + it * RPB;
    if (a0 + ra < La && b0 + ux * 4 + 3 < Lb) {
      float f[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) f[k] = tile[ux * 4 + k][ra];
      u4 w; __builtin_memcpy(&w, f, 16);
      u4* p = reinterpret_cast<u4*>(dst + (a0 + ra) * Lb + b0 + ux * 4);
      if (NT) __builtin_nontemporal_store(w, p); else *p = w;
    } else if (a0 + ra < La) {
      for (int k = 0; k < 4; ++k) if (b0 + ux * 4 + k < Lb) dst[(a0 + ra) * Lb + b0 + ux * 4 + k] = tile[ux * 4 + k][ra];
    }
  }
}

__global__ void kcopy(const u4* __restrict__ s, u4* __restrict__ d, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) d[i] = s[i];
}
__global__ void kcopynt(const u4* __restrict__ s, u4* __restrict__ d, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) __builtin_nontemporal_store(s[i], d + i);
}
__global__ void kcopynt4(const u4* __restrict__ s, u4* __restrict__ d, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    u4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
    __builtin_nontemporal_store(a, d + i); __builtin_nontemporal_store(b, d + i + stride);
    __builtin_nontemporal_store(c, d + i + 2 * stride); __builtin_nontemporal_store(e, d + i + 3 * stride);
  }
  for (; i < n; i += stride) __builtin_nontemporal_store(s[i], d + i);
}

__global__ void kread(const u4* __restrict__ s, int64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) { u4 x = s[i]; acc ^= x.x ^ x.y ^ x.z ^ x.w; }
  if (acc == 0x12345678) out[0] = acc;
}

template <int TA, int TB, int THREADS, bool NT, bool BFAST, bool NTL = false>
float run(const char* name, const float* src, float* dst, int64_t La, int64_t Lb, int reps, const std::vector<uint32_t>* ref) {
  int64_t ntA = (La + TA - 1) / TA, ntB = (Lb + TB - 1) / TB;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 2; ++i) ktr<TA, TB, THREADS, NT, BFAST, NTL><<<ntA * ntB, THREADS>>>(src, dst, La, Lb, ntA, ntB);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) ktr<TA, TB, THREADS, NT, BFAST, NTL><<<ntA * ntB, THREADS>>>(src, dst, La, Lb, ntA, ntB);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
  double gbs = 2.0 * La * Lb * 4 / (ms * 1e-3) / 1e9;
  bool ok = true;
  if (ref) {
    std::vector<uint32_t> h(La * Lb);
    CK(hipMemcpy(h.data(), dst, La * Lb * 4, hipMemcpyDeviceToHost));
    ok = memcmp(h.data(), ref->data(), La * Lb * 4) == 0;
  }
  printf("%-40s %8.3f ms  %8.1f GB/s  %5.1f%% of 8 TB/s  %s\n", name, ms, gbs, gbs / 80.0, ok ? "ok" : "MISMATCH");
  return ms;
}

int main() {
  const int64_t Lb = 2000, La = 262144;  // src [Lb][La] -> dst [La][Lb]
  const int64_t n = La * Lb;
  float *src, *dst, *dst2;
  CK(hipMalloc(&src, n * 4)); CK(hipMalloc(&dst, n * 4)); CK(hipMalloc(&dst2, n * 4));
  std::vector<uint32_t> h(n);
  for (int64_t i = 0; i < n; ++i) h[i] = (uint32_t)(i * 2654435761u);
  CK(hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> ref(n);
  for (int64_t b = 0; b < Lb; ++b) for (int64_t a = 0; a < La; ++a) ref[a * Lb + b] = h[b * La + a];
  const int reps = 20;
  // copy / read ceilings
  {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    int64_t nv = n / 4;
    for (int g : {2048, 4096, 8192, 16384}) {
      kcopy<<<g, 256>>>((const u4*)src, (u4*)dst2, nv);
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) kcopy<<<g, 256>>>((const u4*)src, (u4*)dst2, nv);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
      printf("copy grid %-6d                           %8.3f ms  %8.1f GB/s\n", g, ms, 2.0 * n * 4 / (ms * 1e-3) / 1e9);
    }
    for (int g : {2048, 8192, 16384}) {
      for (int v = 0; v < 2; ++v) {
        if (v == 0) kcopynt<<<g, 256>>>((const u4*)src, (u4*)dst2, nv); else kcopynt4<<<g, 256>>>((const u4*)src, (u4*)dst2, nv);
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) { if (v == 0) kcopynt<<<g, 256>>>((const u4*)src, (u4*)dst2, nv); else kcopynt4<<<g, 256>>>((const u4*)src, (u4*)dst2, nv); }
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("copy NT%s grid %-6d                       %8.3f ms  %8.1f GB/s\n", v ? "x4" : "  ", g, ms, 2.0 * n * 4 / (ms * 1e-3) / 1e9);
      }
    }
    uint32_t* o; CK(hipMalloc(&o, 4));
    kread<<<8192, 256>>>((const u4*)src, nv, o);
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) kread<<<8192, 256>>>((const u4*)src, nv, o);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
    printf("read-only                                %8.3f ms  %8.1f GB/s\n", ms, 1.0 * n * 4 / (ms * 1e-3) / 1e9);
  }
  run<64, 64, 256, true, true>("64x64 t256 NT bfast", src, dst, La, Lb, reps, &ref);
  run<64, 64, 256, true, true, true>("64x64 t256 NT bfast NTL", src, dst, La, Lb, reps, &ref);
  run<64, 128, 256, true, true>("64x128 t256 NT bfast", src, dst, La, Lb, reps, &ref);
  run<64, 128, 256, true, true, true>("64x128 t256 NT bfast NTL", src, dst, La, Lb, reps, &ref);
  run<128, 64, 256, true, true>("128x64 t256 NT bfast", src, dst, La, Lb, reps, &ref);
  run<128, 128, 256, true, true>("128x128 t256 NT bfast", src, dst, La, Lb, reps, &ref);
  run<128, 128, 512, true, true>("128x128 t512 NT bfast", src, dst, La, Lb, reps, &ref);
  run<128, 128, 512, true, true, true>("128x128 t512 NT bfast NTL", src, dst, La, Lb, reps, &ref);
  run<64, 256, 256, true, true>("64x256 t256 NT bfast", src, dst, La, Lb, reps, &ref);
  run<64, 256, 512, true, true>("64x256 t512 NT bfast", src, dst, La, Lb, reps, &ref);
  run<32, 256, 256, true, true>("32x256 t256 NT bfast", src, dst, La, Lb, reps, &ref);
  run<64, 64, 128, true, true>("64x64 t128 NT bfast", src, dst, La, Lb, reps, &ref);
  run<64, 64, 512, true, true>("64x64 t512 NT bfast", src, dst, La, Lb, reps, &ref);
  return 0;
}

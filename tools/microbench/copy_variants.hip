// Streaming copy recipes on MI355X (2.1 GB -> 2.1 GB), to find the copy
// ceiling the permute kernels should be measured against.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef __attribute__((ext_vector_type(4))) uint32_t u4;

// grid-stride, U vectors per thread per iteration, interleaved by blockDim
template <int U, bool NTL, bool NTS>
__global__ void kgs(const u4* __restrict__ s, u4* __restrict__ d, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < n; base += stride) {
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { int64_t i = base + (int64_t)u * blockDim.x; if (i < n) v[u] = NTL ? __builtin_nontemporal_load(s + i) : s[i]; }
#pragma unroll
    for (int u = 0; u < U; ++u) { int64_t i = base + (int64_t)u * blockDim.x; if (i < n) { if (NTS) __builtin_nontemporal_store(v[u], d + i); else d[i] = v[u]; } }
  }
}

// each block copies one contiguous chunk of CH vectors (no grid-stride)
template <int U, bool NTL, bool NTS>
__global__ void kchunk(const u4* __restrict__ s, u4* __restrict__ d, int64_t n, int64_t ch) {
  const int64_t lo = (int64_t)blockIdx.x * ch, hi = lo + ch < n ? lo + ch : n;
  for (int64_t base = lo + threadIdx.x; base < hi; base += (int64_t)blockDim.x * U) {
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { int64_t i = base + (int64_t)u * blockDim.x; if (i < hi) v[u] = NTL ? __builtin_nontemporal_load(s + i) : s[i]; }
#pragma unroll
    for (int u = 0; u < U; ++u) { int64_t i = base + (int64_t)u * blockDim.x; if (i < hi) { if (NTS) __builtin_nontemporal_store(v[u], d + i); else d[i] = v[u]; } }
  }
}

int main() {
  const int64_t bytes = 2097152000;  // C2 array
  const int64_t n = bytes / 16;
  u4 *s, *d;
  CK(hipMalloc(&s, bytes)); CK(hipMalloc(&d, bytes));
  CK(hipMemset(s, 1, bytes));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) launch();
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 10; if (ms < best) best = ms;
    }
    printf("%-44s %8.4f ms %8.1f GB/s\n", name, best, 2.0 * bytes / (best * 1e-3) / 1e9);
  };
  char nm[128];
#define GS(U, NTL, NTS, G, B) snprintf(nm, 128, "gs U%d ntl%d nts%d grid %d blk %d", U, NTL, NTS, G, B); \
  time(nm, [&] { kgs<U, NTL, NTS><<<G, B>>>(s, d, n); });
  GS(1, 0, 0, 8192, 256) GS(1, 1, 1, 8192, 256) GS(4, 1, 1, 4096, 256) GS(4, 1, 1, 2048, 256)
  GS(8, 1, 1, 2048, 256) GS(4, 0, 1, 4096, 256) GS(4, 1, 0, 4096, 256) GS(2, 1, 1, 16384, 256)
  GS(4, 1, 1, 1024, 512) GS(4, 1, 1, 2048, 512) GS(4, 1, 1, 512, 1024) GS(8, 1, 1, 1024, 1024)
  GS(1, 1, 1, 65536, 256) GS(1, 0, 1, 65536, 256)
#define CH(U, NTL, NTS, CHV, B) snprintf(nm, 128, "chunk U%d ntl%d nts%d ch %dKiB blk %d", U, NTL, NTS, (int)(CHV * 16 / 1024), B); \
  time(nm, [&] { kchunk<U, NTL, NTS><<<(int)((n + CHV - 1) / CHV), B>>>(s, d, n, CHV); });
  CH(4, 1, 1, 4096, 256) CH(4, 1, 1, 16384, 256) CH(4, 1, 1, 65536, 256) CH(8, 1, 1, 16384, 256)
  CH(4, 1, 1, 16384, 512) CH(2, 1, 1, 4096, 256) CH(4, 0, 0, 16384, 256)
  printf("hipMemcpyAsync D2D: ");
  time("hipMemcpyAsync", [&] { CK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0)); });
  return 0;
}

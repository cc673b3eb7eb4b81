// Microbenchmark: the row-permuting copy of the C3 swap, float32
// (4096, 256, 256, 32) -> (256, 256, 4096, 32) (perm (1, 2, 0, 3): 128-B rows
// kept).  Source row (c, a, b) -> destination row (a, b, c).
// Variants (all 16-B non-temporal loads/stores, 256 threads, 4 vectors in
// flight per lane):
//   dst   destination order: a wave reads 8 rows at 8-MiB source stride and
//         writes 1 KiB contiguous (the product's order);
//   src   source order: a wave reads 1 KiB contiguous and writes 8 rows at
//         512-KiB destination stride;
//   dstwW destination order within c-windows of W rows (W source pages in
//         flight instead of C);
//   tileN 2-D tiles of 8 b x N c rows per wave: each load instruction reads
//         1 KiB contiguous (8 b of one c), the N loads of a lane cover N
//         consecutive c, so each destination row (a, b) receives an N*128-B
//         contiguous run from one wave.
// Sampled rows are checked against the source.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/rc3.bin tools/microbench/rowcopy_c3.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef __attribute__((ext_vector_type(4))) uint32_t u4;

constexpr uint64_t C = 4096, A = 256, B = 256;  // rows of 32 f32 = 128 B = 8 vectors
constexpr uint64_t ROWS = C * A * B;
constexpr uint64_t TOTAL = ROWS * 8;             // 16-B vectors

template <int U>
__global__ void __launch_bounds__(256) k_dst(const u4* __restrict__ src, u4* __restrict__ dst) {
  const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
  u4 r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t g = base + (uint64_t)u * 256;
    const uint64_t row = g >> 3, v = g & 7;       // destination row (a, b, c)
    const uint64_t c = row % C, ab = row / C;
    const uint64_t a = ab / B, b = ab % B;
    r[u] = __builtin_nontemporal_load(src + ((c * A + a) * B + b) * 8 + v);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], dst + base + (uint64_t)u * 256);
}

template <int U>
__global__ void __launch_bounds__(256) k_src(const u4* __restrict__ src, u4* __restrict__ dst) {
  const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
  u4 r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load(src + base + (uint64_t)u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t g = base + (uint64_t)u * 256;
    const uint64_t row = g >> 3, v = g & 7;       // source row (c, a, b)
    const uint64_t b = row % B, ca = row / B;
    const uint64_t a = ca % A, c = ca / A;
    __builtin_nontemporal_store(r[u], dst + ((a * B + b) * C + c) * 8 + v);
  }
}

// a wave = 8 b (lanes / 8) x N c (unrolled); a block = 4 waves along b
// (32 b); blocks walk b fastest, then c groups, then a.
template <int N>
__global__ void __launch_bounds__(256) k_tile(const u4* __restrict__ src, u4* __restrict__ dst) {
  const uint64_t nbB = B / 32, ncG = C / N;
  uint64_t blk = blockIdx.x;
  const uint64_t bb = blk % nbB; blk /= nbB;
  const uint64_t cg = blk % ncG;
  const uint64_t a = blk / ncG;
  const uint64_t b = bb * 32 + (threadIdx.x >> 3);
  const uint64_t v = threadIdx.x & 7;
  const uint64_t c0 = cg * N;
  u4 r[N];
#pragma unroll
  for (int u = 0; u < N; ++u) r[u] = __builtin_nontemporal_load(src + (((c0 + u) * A + a) * B + b) * 8 + v);
#pragma unroll
  for (int u = 0; u < N; ++u) __builtin_nontemporal_store(r[u], dst + ((a * B + b) * C + c0 + u) * 8 + v);
}

// destination order inside c-windows of W: for each a, for each window, the
// rows (b, c) with c in the window, c fastest -- a window touches W source
// pages (one per c) instead of all C.
template <int U, int W>
__global__ void __launch_bounds__(256) k_dstw(const u4* __restrict__ src, u4* __restrict__ dst) {
  const uint64_t base = (uint64_t)blockIdx.x * 256 * U + threadIdx.x;
  u4 r[U];
  uint64_t dof[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t g = base + (uint64_t)u * 256;
    const uint64_t row = g >> 3, v = g & 7;       // traversal index (a, cw, b, ci)
    const uint64_t ci = row % W;
    const uint64_t t1 = row / W;
    const uint64_t b = t1 % B;
    const uint64_t t2 = t1 / B;
    const uint64_t cw = t2 % (C / W), a = t2 / (C / W);
    const uint64_t c = cw * W + ci;
    r[u] = __builtin_nontemporal_load(src + ((c * A + a) * B + b) * 8 + v);
    dof[u] = ((a * B + b) * C + c) * 8 + v;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], dst + dof[u]);
}

static bool check(const u4* dsrc, const u4* ddst) {
  for (int t = 0; t < 64; ++t) {
    const uint64_t c = (t * 977) % C, a = (t * 131) % A, b = (t * 37 + 5) % B;
    u4 s[8], d[8];
    CK(hipMemcpy(s, dsrc + ((c * A + a) * B + b) * 8, 128, hipMemcpyDeviceToHost));
    CK(hipMemcpy(d, ddst + ((a * B + b) * C + c) * 8, 128, hipMemcpyDeviceToHost));
    if (memcmp(s, d, 128)) return false;
  }
  return true;
}

template <typename F>
static void run(const char* name, F launch, const u4* src, u4* dst) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipMemset(dst, 0, TOTAL * 16));
  launch(); CK(hipGetLastError()); CK(hipDeviceSynchronize());
  const bool ok = check(src, dst);
  std::vector<float> ms;
  for (int i = 0; i < 8; ++i) {
    CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float t; CK(hipEventElapsedTime(&t, e0, e1)); ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  printf("%-10s median %8.3f ms  %7.1f GB/s  (min %.3f)  %s\n", name, ms[4], 2.0 * TOTAL * 16 / (ms[4] * 1e-3) / 1e9,
         ms[0], ok ? "ok" : "MISMATCH");
  fflush(stdout);
}

int main() {
  u4 *src, *dst;
  CK(hipMalloc(&src, TOTAL * 16)); CK(hipMalloc(&dst, TOTAL * 16));
  // fill: every 32-bit word with a hash of its index (a device-side loop via memset patterns is too regular)
  {
    std::vector<uint32_t> h(1 << 24);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u);
    const size_t chunk = h.size() * 4;
    for (uint64_t off = 0; off < TOTAL * 16; off += chunk) {
      for (size_t i = 0; i < 16; ++i) h[i] = (uint32_t)(off / chunk) * 16 + i;
      CK(hipMemcpy((char*)src + off, h.data(), std::min<uint64_t>(chunk, TOTAL * 16 - off), hipMemcpyHostToDevice));
    }
  }
  constexpr int U = 4;
  const uint64_t g4 = TOTAL / (256 * U);
  run("dst", [&] { k_dst<U><<<g4, 256>>>(src, dst); }, src, dst);
  run("src", [&] { k_src<U><<<g4, 256>>>(src, dst); }, src, dst);
  run("tile4", [&] { k_tile<4><<<(B / 32) * (C / 4) * A, 256>>>(src, dst); }, src, dst);
  run("tile8", [&] { k_tile<8><<<(B / 32) * (C / 8) * A, 256>>>(src, dst); }, src, dst);
  run("tile16", [&] { k_tile<16><<<(B / 32) * (C / 16) * A, 256>>>(src, dst); }, src, dst);
  run("dst", [&] { k_dst<U><<<g4, 256>>>(src, dst); }, src, dst);
  run("src", [&] { k_src<U><<<g4, 256>>>(src, dst); }, src, dst);
  run("dstw64", [&] { k_dstw<U, 64><<<g4, 256>>>(src, dst); }, src, dst);
  run("dstw256", [&] { k_dstw<U, 256><<<g4, 256>>>(src, dst); }, src, dst);
  run("dstw1024", [&] { k_dstw<U, 1024><<<g4, 256>>>(src, dst); }, src, dst);
  run("dst", [&] { k_dst<U><<<g4, 256>>>(src, dst); }, src, dst);
  run("dstw256", [&] { k_dstw<U, 256><<<g4, 256>>>(src, dst); }, src, dst);
  return 0;
}

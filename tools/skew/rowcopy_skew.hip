// Microbenchmark: skewed (diagonal) traversals of the C3 swap's row copy,
// float32 (4096, 256, 256, 32) -> (256, 256, 4096, 32): source row (c, h),
// h = a*256 + b, goes to destination row (h, c); rows are 128 B.
// Counters (profiles/r02_kernel_counters.md) put the product's destination-
// order copy at 10-15x the L2 tag stalls per byte of the other copies: a
// block's 32 rows are one c-run, i.e. 32 source lines at an 8-MiB stride.
// Variants (16-B non-temporal loads/stores, 256 threads, 4 slots of 32 rows
// per block):
//   dst     destination order (the product's order; baseline)
//   diagT   T x T super-tiles of (h, c) walked by diagonals: slot row k of
//           diagonal j is (h0 + k, c0 + (k + j) mod T), so the 32 rows of a
//           slot have distinct h AND distinct c -- distinct low address bits
//           on both the source and the destination side; super-tiles walk c
//           fastest.  T = 16, 32, 64.
//   diagTg  the same with runs of g rows contiguous along c (g = 4: 512-B
//           destination runs, 4 source lines per h)
//   ldsT    T x T record tiles transposed through LDS: T*128-B contiguous
//           runs on both the source and the destination side
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/rcs.bin tools/skew/rowcopy_skew.hip
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


template <int U, int T, int G>
__global__ void __launch_bounds__(256) k_diag(const u4* __restrict__ src, u4* __restrict__ dst) {
  constexpr uint64_t H = A * B;
  constexpr uint64_t PER_TILE = (uint64_t)T * T;        // rows per super-tile
  constexpr uint64_t SLOTS = PER_TILE / 32;              // 32-row slots per super-tile
  const uint64_t v = threadIdx.x & 7;
  const uint64_t k32 = threadIdx.x >> 3;                 // row within the slot
  u4 r[U];
  uint64_t dof[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t slot = (uint64_t)blockIdx.x * U + u;
    const uint64_t S = slot / SLOTS;
    const uint64_t q = (slot % SLOTS) * 32 + k32;        // row index within the super-tile
    // runs of G rows along c: diagonal over (h, c-run) of a T x (T/G) grid
    const uint64_t runs = T / G;
    const uint64_t qr = q / G, gi = q % G;
    const uint64_t j = qr / T, kk = qr % T;              // diagonal j (0..runs-1), position kk (h)
    const uint64_t cb = S % (C / T), hb = S / (C / T);
    const uint64_t h = hb * T + kk;
    const uint64_t c = cb * T + ((kk + j) % runs) * G + gi;
    r[u] = __builtin_nontemporal_load(src + (c * H + h) * 8 + v);
    dof[u] = (h * C + c) * 8 + v;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], dst + dof[u]);
}


// Record-tile transpose through LDS: a T x T tile of 128-B records (T h by
// T c) is read as T source runs of T*128 B (one c each) and written as T
// destination runs of T*128 B (one h each): long contiguous runs on BOTH
// sides, the records re-ordered in LDS (row pitch padded by one 16-B vector).
template <int T>
__global__ void __launch_bounds__(256) k_ldsT(const u4* __restrict__ src, u4* __restrict__ dst) {
  constexpr uint64_t H = A * B;
  constexpr int RV = T * 8;                 // 16-B vectors per tile row (T records)
  constexpr int NV = T * RV;                // vectors per tile
  constexpr int PER = NV / 256;             // vectors per thread
  __shared__ u4 tile[T][RV + 1];
  const uint64_t ntc = C / T;
  for (uint64_t t = blockIdx.x; t < (H / T) * ntc; t += gridDim.x) {
    const uint64_t c0 = (t % ntc) * T, h0 = (t / ntc) * T;
    u4 r[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = threadIdx.x + 256 * i;
      const int cl = q / RV, w = q % RV;    // tile row = one c; w = h_local * 8 + v
      r[i] = __builtin_nontemporal_load(src + ((c0 + cl) * H + h0) * 8 + w);
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = threadIdx.x + 256 * i;
      tile[q / RV][q % RV] = r[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = threadIdx.x + 256 * i;
      const int hl = q / RV, w = q % RV;    // output row = one h; w = c_local * 8 + v
      const int cl = w / 8, v = w % 8;
      __builtin_nontemporal_store(tile[cl][hl * 8 + v], dst + ((h0 + hl) * C + c0) * 8 + w);
    }
    __syncthreads();
  }
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
  for (int rep = 0; rep < 2; ++rep) {
    run("dst", [&] { k_dst<U><<<g4, 256>>>(src, dst); }, src, dst);
    run("diag16", [&] { k_diag<U, 16, 1><<<g4, 256>>>(src, dst); }, src, dst);
    run("diag32", [&] { k_diag<U, 32, 1><<<g4, 256>>>(src, dst); }, src, dst);
    run("diag64", [&] { k_diag<U, 64, 1><<<g4, 256>>>(src, dst); }, src, dst);
    run("diag32g4", [&] { k_diag<U, 32, 4><<<g4, 256>>>(src, dst); }, src, dst);
    run("diag64g4", [&] { k_diag<U, 64, 4><<<g4, 256>>>(src, dst); }, src, dst);
    run("diag64g8", [&] { k_diag<U, 64, 8><<<g4, 256>>>(src, dst); }, src, dst);
    run("lds8", [&] { k_ldsT<8><<<262144, 256>>>(src, dst); }, src, dst);
    run("lds16", [&] { k_ldsT<16><<<262144, 256>>>(src, dst); }, src, dst);
  }
  return 0;
}

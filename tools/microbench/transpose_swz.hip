// Microbenchmark: LDS layout of the 32-bit tile transpose (C2's swap:
// [2000][262144] float32 -> [262144][2000]).
//   pad  : tile[TB][TA+1], ds_write/ds_read of single dwords (the product kernel
//          before this test); reads of 4 rows 1 apart per lane are 4-way bank
//          conflicts (SQ_LDS_BANK_CONFLICT = 66% of LDS cycles).
//   swz  : tile[TB][TA] unpadded, 16-B chunks XOR-swizzled by (row / 4) % 16;
//          ds_write_b128 of each loaded vector, ds_read_b128 of a 4x4 block
//          (4 rows x one chunk) per lane, rearranged in registers into four
//          16-B stores.  Conflict-free on both sides.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/tsw.bin tools/microbench/transpose_swz.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef __attribute__((ext_vector_type(4))) uint32_t u4;

template <int TA, int TB, int THREADS>
__global__ void __launch_bounds__(THREADS) k_pad(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                 int64_t La, int64_t Lb, int64_t ntB) {
  constexpr int VEC = 4;
  __shared__ uint32_t tile[TB][TA + 1];
  constexpr int NVA = TA / VEC, RPA = THREADS / NVA, NL = TB / RPA;
  constexpr int NVB = TB / VEC, RPB = THREADS / NVB, NS = TA / RPB;
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
  const int64_t t = blockIdx.x;
  const int64_t tb = t % ntB, ta = t / ntB;
  const int64_t a0 = ta * TA, b0 = tb * TB;
  u4 v[NL];
#pragma unroll
  for (int it = 0; it < NL; ++it) {
    const int rb = ty + it * RPA;
    if (b0 + rb < Lb) v[it] = __builtin_nontemporal_load(reinterpret_cast<const u4*>(src + (b0 + rb) * La + a0 + tx * VEC));
  }
#pragma unroll
  for (int it = 0; it < NL; ++it) {
    const int rb = ty + it * RPA;
#pragma unroll
    for (int k = 0; k < VEC; ++k) tile[rb][tx * VEC + k] = v[it][k];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NS; ++it) {
    const int ra = uy + it * RPB;
    if (b0 + ux * VEC + VEC - 1 < Lb) {
      u4 w;
#pragma unroll
      for (int k = 0; k < VEC; ++k) w[k] = tile[ux * VEC + k][ra];
      __builtin_nontemporal_store(w, reinterpret_cast<u4*>(dst + (a0 + ra) * Lb + b0 + ux * VEC));
    } else {
      for (int k = 0; k < VEC; ++k)
        if (b0 + ux * VEC + k < Lb) dst[(a0 + ra) * Lb + b0 + ux * VEC + k] = tile[ux * VEC + k][ra];
    }
  }
}

// cache policy variants of the padded kernel: NTL / NTS = non-temporal loads / stores
template <int TA, int TB, int THREADS, bool NTL, bool NTS>
__global__ void __launch_bounds__(THREADS) k_pol(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                 int64_t La, int64_t Lb, int64_t ntB) {
  constexpr int VEC = 4;
  __shared__ uint32_t tile[TB][TA + 1];
  constexpr int NVA = TA / VEC, RPA = THREADS / NVA, NL = TB / RPA;
  constexpr int NVB = TB / VEC, RPB = THREADS / NVB, NS = TA / RPB;
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
  const int64_t t = blockIdx.x;
  const int64_t tb = t % ntB, ta = t / ntB;
  const int64_t a0 = ta * TA, b0 = tb * TB;
  u4 v[NL];
#pragma unroll
  for (int it = 0; it < NL; ++it) {
    const int rb = ty + it * RPA;
    const u4* p = reinterpret_cast<const u4*>(src + (b0 + rb) * La + a0 + tx * VEC);
    if (b0 + rb < Lb) v[it] = NTL ? __builtin_nontemporal_load(p) : *p;
  }
#pragma unroll
  for (int it = 0; it < NL; ++it) {
    const int rb = ty + it * RPA;
#pragma unroll
    for (int k = 0; k < VEC; ++k) tile[rb][tx * VEC + k] = v[it][k];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NS; ++it) {
    const int ra = uy + it * RPB;
    if (b0 + ux * VEC + VEC - 1 < Lb) {
      u4 w;
#pragma unroll
      for (int k = 0; k < VEC; ++k) w[k] = tile[ux * VEC + k][ra];
      u4* q = reinterpret_cast<u4*>(dst + (a0 + ra) * Lb + b0 + ux * VEC);
      if (NTS) __builtin_nontemporal_store(w, q); else *q = w;
    } else {
      for (int k = 0; k < VEC; ++k)
        if (b0 + ux * VEC + k < Lb) dst[(a0 + ra) * Lb + b0 + ux * VEC + k] = tile[ux * VEC + k][ra];
    }
  }
}

template <int TA, int TB, int THREADS, bool NTL, bool NTS>
void launch_pol(const void* src, void* dst, int64_t La, int64_t Lb) {
  const int64_t ntB = (Lb + TB - 1) / TB, ntiles = (La / TA) * ntB;
  k_pol<TA, TB, THREADS, NTL, NTS><<<(int)ntiles, THREADS>>>((const uint32_t*)src, (uint32_t*)dst, La, Lb, ntB);
}

// TA = 64 words (16 chunks of 16 B per row), TB = 4 * 64 rows per reading wave
// pass: lanes along b, 4 rows each.
template <int TA, int TB, int THREADS>
__global__ void __launch_bounds__(THREADS) k_swz(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                 int64_t La, int64_t Lb, int64_t ntB) {
  constexpr int NCH = TA / 4;            // 16-B chunks per tile row
  static_assert(NCH == 16, "swizzle spans 16 chunks");
  constexpr int NVA = NCH, RPA = THREADS / NVA, NL = TB / RPA;
  constexpr int LB = TB / 4;             // lanes along b on the read side (4 rows each)
  constexpr int CPP = THREADS / LB;      // chunk columns per pass
  constexpr int NR = NCH / CPP;          // read passes
  static_assert(LB <= THREADS && NCH % CPP == 0, "layout");
  __shared__ u4 tile[TB * NCH];
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % LB, uy = threadIdx.x / LB;
  const int64_t t = blockIdx.x;
  const int64_t tb = t % ntB, ta = t / ntB;
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
    tile[rb * NCH + (tx ^ ((rb >> 2) & 15))] = v[it];
  }
  __syncthreads();
  const int b = ux * 4;
  const bool full = b0 + b + 4 <= Lb;
#pragma unroll
  for (int p = 0; p < NR; ++p) {
    const int c = uy + p * CPP;
    u4 r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = tile[(b + i) * NCH + (c ^ (ux & 15))];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t a = a0 + c * 4 + j;
      u4 w = {r[0][j], r[1][j], r[2][j], r[3][j]};
      uint32_t* q = dst + a * Lb + b0 + b;
      if (full) {
        __builtin_nontemporal_store(w, reinterpret_cast<u4*>(q));
      } else {
        for (int i = 0; i < 4; ++i)
          if (b0 + b + i < Lb) q[i] = w[i];
      }
    }
  }
}

struct Variant {
  const char* name;
  void (*launch)(const void*, void*, int64_t, int64_t);
  std::vector<float> ms;
  bool ok;
};

// XK: extra dynamic LDS (KiB) per block, to cap blocks per CU
template <int TA, int TB, int THREADS, bool SWZ, int XK = 0>
void launch_v(const void* src, void* dst, int64_t La, int64_t Lb) {
  const int64_t ntB = (Lb + TB - 1) / TB, ntiles = (La / TA) * ntB;
  if constexpr (SWZ)
    k_swz<TA, TB, THREADS><<<(int)ntiles, THREADS, XK * 1024>>>((const uint32_t*)src, (uint32_t*)dst, La, Lb, ntB);
  else
    k_pad<TA, TB, THREADS><<<(int)ntiles, THREADS, XK * 1024>>>((const uint32_t*)src, (uint32_t*)dst, La, Lb, ntB);
}

int main() {
  const int64_t Lb = 2000, La = 512 * 512;
  const int64_t n = Lb * La, nbytes = n * 4;
  uint32_t *src, *dst;
  CK(hipMalloc(&src, nbytes)); CK(hipMalloc(&dst, nbytes));
  std::vector<uint32_t> h(n), hh(n), ref(n);
  for (int64_t i = 0; i < n; ++i) h[i] = (uint32_t)(i * 2654435761ull >> 7);
  for (int64_t b = 0; b < Lb; ++b)
    for (int64_t a = 0; a < La; ++a) ref[a * Lb + b] = h[b * La + a];
  CK(hipMemcpy(src, h.data(), nbytes, hipMemcpyHostToDevice));
  std::vector<Variant> vs = {
      {"pad 32x256 t256", &launch_v<32, 256, 256, false>, {}, false},
      {"pad 64x128 t256", &launch_v<64, 128, 256, false>, {}, false},
      {"pad 64x256 t256", &launch_v<64, 256, 256, false>, {}, false},
      {"pad 32x256 t256 (again)", &launch_v<32, 256, 256, false>, {}, false},
      {"pad 64x128 t256 (again)", &launch_v<64, 128, 256, false>, {}, false},
  };
  for (auto& v : vs) {
    CK(hipMemset(dst, 0, nbytes));
    v.launch(src, dst, La, Lb);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hh.data(), dst, nbytes, hipMemcpyDeviceToHost));
    v.ok = memcmp(hh.data(), ref.data(), nbytes) == 0;
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int rounds = 7, rr = 8;
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
    const double med = m[m.size() / 2];
    printf("%-26s median %7.4f ms %7.1f GB/s  best %7.4f  %s\n", v.name, med, 2.0 * nbytes / (med * 1e-3) / 1e9, m[0],
           v.ok ? "ok" : "MISMATCH");
  }
  return 0;
}

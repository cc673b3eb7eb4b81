// Destination-row alignment probe for the f32 tile transpose (register staging,
// 64x256 tiles): is a 128-B-misaligned destination row pitch (C2: 8000 B)
// slower per byte than an aligned one?
// tile transpose.  [Lb][La] -> [La][Lb], 64 (a) x 256 (b) tiles as in the
// product's k_transpose<u32,64,256>:
//   reg     the product's register staging: 16 x 16-B nt loads per lane in
//           flight, then ds_write, barrier, column reads, 16-B nt stores.
//   glds    global_load_lds_dwordx4 straight into an unpadded LDS image (one
//           wave-instruction = 1 KiB = 4 source rows of 256 B); the image is
//           XOR-swizzled through the per-lane SOURCE address (LDS stays
//           lane-linear), and the store side reads 4 columns x 64 rows per
//           wave-instruction, conflict-free.  One tile per block (64 KiB of
//           LDS: 2 blocks per CU, as reg).
//   glds2   the same tiles in a persistent block with two LDS buffers: tile
//           i+1's DMA is in flight while tile i is stored (512 threads, 128
//           KiB, one block per CU).
//   glds2h  two buffers of 64 x 128 tiles (32 KiB each), 256 threads, two
//           blocks per CU.
// Every variant's output is compared with reg's, byte for byte (whole array).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench/tglds.bin tools/microbench/transpose_glds.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef __attribute__((ext_vector_type(4))) uint32_t u4;
typedef __attribute__((address_space(3))) void lds_void;

// ---- register staging (product structure) ----
__global__ void __launch_bounds__(256) k_reg(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int64_t La,
                                             int64_t Lb, int64_t ntB) {
  constexpr int TA = 64, TB = 256, NVA = 16, RPA = 16, NL = 16, NVB = 64, RPB = 4, NS = 16;
  __shared__ uint32_t tile[TB][TA + 1];
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
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

// ---- direct-to-LDS staging ----
// LDS image: TB rows of 64 floats (256 B), unpadded; row r holds source chunk c
// (4 floats) at position c ^ sw(r), sw(r) = (r >> 2) & 15.
__device__ __forceinline__ int sw(int r) { return (r >> 2) & 15; }

// DMA one TB x 64 tile into `img` (wave w of NW issues rows [4*(w + NW*j), +4)).
template <int TB, int NW>
__device__ __forceinline__ void tile_dma(const uint32_t* __restrict__ src, uint32_t* img, int64_t La, int64_t Lb,
                                         int64_t a0, int64_t b0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int J = TB / 4 / NW;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int r0 = 4 * (w + NW * j);
    const int r = r0 + (lane >> 4), p = lane & 15;
    const int c = p ^ sw(r);
    if (b0 + r < Lb)
      __builtin_amdgcn_global_load_lds((const void*)(src + (b0 + r) * La + a0 + 4 * c), (lds_void*)(img + r0 * 64), 16,
                                       0, 0);
  }
}

// Store the tile in `img`: a wave-instruction covers 4 columns x 64 rows.
template <int TB, int NW>
__device__ __forceinline__ void tile_store(const uint32_t* img, uint32_t* __restrict__ dst, int64_t Lb, int64_t a0,
                                           int64_t b0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cj = lane >> 4, bq = lane & 15;
  constexpr int NB64 = TB / 64;          // 64-row groups
  constexpr int J = 16 * NB64 / NW;      // wave-instructions per wave
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int q = w + NW * j;
    const int ca = 4 * (q % 16), bb = 64 * (q / 16);
    const int a = ca + cj;
    const int b = bb + 4 * bq;
    uint32_t f[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = b + k;
      f[k] = img[r * 64 + 4 * ((a >> 2) ^ sw(r)) + (a & 3)];
    }
    uint32_t* p = dst + (a0 + a) * Lb + b0 + b;
    if (b0 + b + 3 < Lb) {
      u4 wv; __builtin_memcpy(&wv, f, 16);
      __builtin_nontemporal_store(wv, reinterpret_cast<u4*>(p));
    } else {
      for (int k = 0; k < 4; ++k) if (b0 + b + k < Lb) p[k] = f[k];
    }
  }
}

__global__ void __launch_bounds__(256) k_glds(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int64_t La,
                                              int64_t Lb, int64_t ntB) {
  __shared__ uint32_t img[256 * 64];
  const int64_t t = blockIdx.x;
  const int64_t tb = t % ntB, ta = t / ntB;
  const int64_t a0 = ta * 64, b0 = tb * 256;
  tile_dma<256, 4>(src, img, La, Lb, a0, b0);
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0) expcnt(0)
  __syncthreads();
  tile_store<256, 4>(img, dst, Lb, a0, b0);
}

template <int TB, int NT>
__global__ void __launch_bounds__(NT) k_glds2(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int64_t La,
                                              int64_t Lb, int64_t ntB, int64_t nt) {
  constexpr int NW = NT / 64;
  __shared__ uint32_t img[2][TB * 64];
  int64_t t = blockIdx.x;
  if (t >= nt) return;
  tile_dma<TB, NW>(src, img[0], La, Lb, (t / ntB) * 64, (t % ntB) * TB);
  for (int buf = 0; t < nt; t += gridDim.x, buf ^= 1) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const int64_t tn = t + gridDim.x;
    if (tn < nt) tile_dma<TB, NW>(src, img[buf ^ 1], La, Lb, (tn / ntB) * 64, (tn % ntB) * TB);
    tile_store<TB, NW>(img[buf], dst, Lb, (t / ntB) * 64, (t % ntB) * TB);
  }
}

int main(int argc, char** argv) {
  // dest-row alignment probe: reg kernel on [Lb][La] -> [La][Lb] for several Lb
  // (Lb * 4 B = destination row pitch: 7936 and 8192 are 128-B multiples, 8000 is not)
  const int64_t La = 262144;
  const int64_t lbs[] = {2048, 2000, 1792, 2304, 1536, 2040, 1024, 1000};
  const int64_t maxn = 2304LL * La;
  uint32_t *src, *dst;
  CK(hipMalloc(&src, maxn * 4)); CK(hipMalloc(&dst, maxn * 4));
  CK(hipMemset(src, 1, maxn * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    for (int64_t Lb : lbs) {
      const int64_t n = La * Lb, ntB = (Lb + 255) / 256, nt = (La / 64) * ntB;
      k_reg<<<(int)nt, 256>>>(src, dst, La, Lb, ntB);
      CK(hipDeviceSynchronize());
      std::vector<float> ms;
      for (int i = 0; i < 15; ++i) {
        CK(hipEventRecord(e0));
        k_reg<<<(int)nt, 256>>>(src, dst, La, Lb, ntB);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float m; CK(hipEventElapsedTime(&m, e0, e1)); ms.push_back(m);
      }
      std::sort(ms.begin(), ms.end());
      const double med = ms[ms.size() / 2];
      printf("rep %d Lb %5lld (dest row %5lld B, %s)  median %7.4f ms  %7.1f GB/s\n", rep, (long long)Lb,
             (long long)(Lb * 4), (Lb * 4) % 128 ? "misaligned" : "128-B aligned", med, 2.0 * n * 4 / med / 1e6);
      fflush(stdout);
    }
  }
  return 0;
}

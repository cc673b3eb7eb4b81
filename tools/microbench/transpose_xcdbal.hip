// Microbenchmark: XCD-balanced tile order for the C2 transpose.
// [Lb][262144] f32 -> [262144][Lb], the product's 64x256 register-staged
// tiles.  With 8 b-tiles per a-tile and consecutive blocks walking b, block i
// runs b-tile i % 8, and blocks are dealt round-robin over the 8 XCDs: XCD
// slot s runs every (a, s) tile.  At Lb = 2000 the last b-tile holds 208 of
// 256 rows, so slot 7 carries 0.8125 of the others' work, and
// profiles/r02_rowalign.log suggests slots 0-6 set the time (Lb 1920 ran no
// faster than 2048).  Variants:
//   base      tile t = blockIdx: (t / 8, t % 8) (the product's walk)
//   grpG_D    per group of G a-tiles, slots 0-6 give their last D a-tiles of
//             the group to slot 7 (which runs its G partial tiles, then the
//             7*D donated ones); slots 0-6 fill with empty blocks
//   end_D     slots 0-6 give their last D a-tiles of the whole array
//   xcda      the 8 b-tiles of an a-tile on one XCD slot, the same 64 tiles
//             in flight as base (the half lines an odd destination row's
//             neighbouring segments share then meet in one L2)
// Every variant's output is compared with base's, byte for byte.  Lb 2048
// (no partial tile) is timed as the balanced ceiling.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/txb.bin tools/microbench/transpose_xcdbal.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef __attribute__((ext_vector_type(4))) uint32_t u4;

constexpr int TA = 64, TB = 256, NT = 256;

// mode 0: base; 1: groups of G a-tiles, D donated per slot per group; 2: D donated at the end;
// 3: an a-tile's b-tiles on one XCD slot (needs ntA % 8 == 0)
__global__ void __launch_bounds__(NT) kxb(const float* __restrict__ src, float* __restrict__ dst, int64_t La, int64_t Lb,
                                          int64_t ntA, int mode, int G, int D) {
  __shared__ float tile[TB][TA + 1];
  constexpr int VEC = 4;
  constexpr int NVA = TA / VEC, RPA = NT / NVA, NL = TB / RPA;
  constexpr int NVB = TB / VEC, RPB = NT / NVB, NS = TA / RPB;
  const int64_t i = blockIdx.x;
  int64_t ta, tb;
  if (mode == 0) {
    tb = i % 8; ta = i / 8;
  } else if (mode == 1) {
    const int64_t s = i & 7, j = i >> 3;
    const int64_t per = G + 7 * D;         // blocks per slot per group
    const int64_t grp = j / per, k = j - grp * per;
    if (s < 7) {
      if (k >= G - D) return;
      tb = s; ta = grp * G + k;
    } else if (k < G) {
      tb = 7; ta = grp * G + k;
    } else {
      const int64_t q = k - G;
      tb = q / D; ta = grp * G + (G - D) + q % D;
    }
  } else if (mode == 3) {
    // the 8 b-tiles of an a-tile on one XCD slot (a % 8 == i % 8), so the
    // half lines two neighbouring b-tiles share meet in one L2
    ta = (i >> 6) * 8 + (i & 7); tb = (i >> 3) & 7;
  } else {
    const int64_t s = i & 7, j = i >> 3;
    if (s < 7) {
      if (j >= ntA - D) return;
      tb = s; ta = j;
    } else if (j < ntA) {
      tb = 7; ta = j;
    } else {
      const int64_t q = j - ntA;
      tb = q / D; ta = ntA - D + q % D;
    }
  }
  if (ta >= ntA) return;
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
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
    float f[VEC]; __builtin_memcpy(f, &v[it], 16);
#pragma unroll
    for (int k = 0; k < VEC; ++k) tile[rb][tx * VEC + k] = f[k];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NS; ++it) {
    const int ra = uy + it * RPB;
    if (b0 + ux * VEC + VEC - 1 < Lb) {
      float f[VEC];
#pragma unroll
      for (int k = 0; k < VEC; ++k) f[k] = tile[ux * VEC + k][ra];
      u4 w; __builtin_memcpy(&w, f, 16);
      __builtin_nontemporal_store(w, reinterpret_cast<u4*>(dst + (a0 + ra) * Lb + b0 + ux * VEC));
    } else {
      for (int k = 0; k < VEC; ++k) if (b0 + ux * VEC + k < Lb) dst[(a0 + ra) * Lb + b0 + ux * VEC + k] = tile[ux * VEC + k][ra];
    }
  }
}

struct Variant { char name[48]; int64_t Lb; int mode, G, D; std::vector<float> ms; bool ok; };

static int64_t grid_of(const Variant& v, int64_t ntA) {
  if (v.mode == 0 || v.mode == 3) return ntA * 8;
  if (v.mode == 1) return 8 * ((ntA + v.G - 1) / v.G) * (v.G + 7 * v.D);
  return 8 * (ntA + 7 * v.D);
}

int main(int argc, char** argv) {
  const int64_t La = 262144, maxLb = 2048;
  const int64_t nbytes = maxLb * La * 4;
  const int nbuf = argc > 1 ? atoi(argv[1]) : 1;
  std::vector<char*> srcs(nbuf);
  char *dst, *ref;
  for (auto& s : srcs) CK(hipMalloc(&s, nbytes));
  CK(hipMalloc(&dst, nbytes)); CK(hipMalloc(&ref, nbytes));
  std::vector<uint8_t> h(nbytes), a(nbytes), b(nbytes);
  for (int64_t i = 0; i < nbytes; ++i) h[i] = (uint8_t)((i * 2654435761ull) >> 13);
  for (auto& s : srcs) CK(hipMemcpy(s, h.data(), nbytes, hipMemcpyHostToDevice));
  const int64_t ntA = La / TA;
  std::vector<Variant> vs = {
      {"base Lb2000", 2000, 0, 0, 0},       {"xcda Lb2000", 2000, 3, 0, 0},
      {"grp256_6 Lb2000", 2000, 1, 256, 6}, {"end96 Lb2000", 2000, 2, 0, 96},
      {"base Lb2048", 2048, 0, 0, 0},       {"xcda Lb2048", 2048, 3, 0, 0},
      {"base Lb2016", 2016, 0, 0, 0},       {"xcda Lb2016", 2016, 3, 0, 0},
  };
  for (auto& v : vs) {
    snprintf(v.name + strlen(v.name), 8, "");
    // reference: base of the same Lb
    kxb<<<(int)(ntA * 8), NT>>>((const float*)srcs[0], (float*)ref, La, v.Lb, ntA, 0, 0, 0);
    CK(hipMemset(dst, 0, nbytes));
    kxb<<<(int)grid_of(v, ntA), NT>>>((const float*)srcs[0], (float*)dst, La, v.Lb, ntA, v.mode, v.G, v.D);
    CK(hipDeviceSynchronize());
    const int64_t nb = v.Lb * La * 4;
    CK(hipMemcpy(a.data(), ref, nb, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), dst, nb, hipMemcpyDeviceToHost));
    v.ok = memcmp(a.data(), b.data(), nb) == 0;
    // spot check base against the host transpose
    bool hok = true;
    for (int64_t k = 0; k < 100000 && hok; ++k) {
      const int64_t e = (k * 7919 * 104729) % (v.Lb * La);
      const int64_t ai = e / v.Lb, bi = e % v.Lb;
      hok = memcmp(&a[e * 4], &h[(bi * La + ai) * 4], 4) == 0;
    }
    v.ok = v.ok && hok;
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int rounds = 7, rr = 8;
  for (int bu = 0; bu < nbuf; ++bu) {
    for (auto& v : vs) v.ms.clear();
    for (int r = 0; r < rounds; ++r)
      for (auto& v : vs) {
        const int g = (int)grid_of(v, ntA);
        kxb<<<g, NT>>>((const float*)srcs[bu], (float*)dst, La, v.Lb, ntA, v.mode, v.G, v.D);
        CK(hipEventRecord(e0));
        for (int i = 0; i < rr; ++i) kxb<<<g, NT>>>((const float*)srcs[bu], (float*)dst, La, v.Lb, ntA, v.mode, v.G, v.D);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        v.ms.push_back(ms / rr);
      }
    printf("source buffer %d\n", bu);
    for (auto& v : vs) {
      std::vector<float> m = v.ms;
      std::sort(m.begin(), m.end());
      const double med = m[m.size() / 2];
      printf("  %-20s grid %6lld  median %7.4f ms  %7.1f GB/s  %s\n", v.name, (long long)grid_of(v, ntA), med,
             2.0 * v.Lb * La * 4 / (med * 1e-3) / 1e9, v.ok ? "ok" : "MISMATCH");
    }
    fflush(stdout);
  }
  return 0;
}

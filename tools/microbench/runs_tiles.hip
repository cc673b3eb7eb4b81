// Microbenchmark: the runs transpose (permutations that keep a short inner
// run) on the C3 swap shape, float32 (K0, 256, 256, 32) -> (256, 256, K0, 32)
// with K0 = 512 (4.3 GB), i.e. perm (1, 2, 0, 3): 128-B runs (W = 8 16-B
// units), source-contiguous run axis A = axis 2, destination-contiguous run
// axis B = axis 0, batch = axis 1.  Tile = TB rows (along B) x TAU units
// (TAU / W runs along A).  Variants run interleaved (median of rounds) and are
// checked bit-exactly against a host permute.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/rt.bin tools/microbench/runs_tiles.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef __attribute__((ext_vector_type(4))) uint32_t u4;

struct Desc {
  int64_t La, Lb;   // runs along A / rows along B
  int64_t sb, da;   // source stride of B, destination stride of A (units)
  int64_t sbt, dbt; // batch strides (units)
  int64_t ntB, ntAB, ntiles;
};

template <int W, int TAU, int TB, int THREADS, bool LF>
__global__ void __launch_bounds__(THREADS) krt(const u4* __restrict__ src, u4* __restrict__ dst, Desc d) {
  constexpr int TA = TAU / W;
  constexpr int PAD = W < 16 ? W : 0;
  constexpr int ROW = TAU + PAD;
  constexpr int NL = TB * TAU / THREADS;
  static_assert(NL >= 1 && (TB * TAU) % THREADS == 0, "tile");
  __shared__ u4 tile[TB * ROW];
  const int64_t t = blockIdx.x;
  const int64_t bt = t / d.ntAB, rem = t % d.ntAB;
  const int64_t ta = rem / d.ntB, tb = rem % d.ntB;
  const int64_t a0 = ta * TA, b0 = tb * TB;
  const int64_t na = min((int64_t)TA, d.La - a0), nb = min((int64_t)TB, d.Lb - b0);
  const u4* s = src + bt * d.sbt + a0 * W + b0 * d.sb;
  if (LF) {
    u4 v[NL];
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int idx = it * THREADS + threadIdx.x;
      const int rb = idx / TAU, u = idx % TAU;
      if (rb < nb && u < na * W) v[it] = __builtin_nontemporal_load(s + (int64_t)rb * d.sb + u);
    }
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int idx = it * THREADS + threadIdx.x;
      const int rb = idx / TAU, u = idx % TAU;
      tile[rb * ROW + u] = v[it];
    }
  } else {
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int idx = it * THREADS + threadIdx.x;
      const int rb = idx / TAU, u = idx % TAU;
      if (rb < nb && u < na * W) tile[rb * ROW + u] = __builtin_nontemporal_load(s + (int64_t)rb * d.sb + u);
    }
  }
  __syncthreads();
  u4* q = dst + bt * d.dbt + b0 * W + a0 * d.da;
#pragma unroll
  for (int it = 0; it < NL; ++it) {
    const int idx = it * THREADS + threadIdx.x;
    const int ra = idx / (TB * W), m = idx % (TB * W);
    const int b = m / W, w = m % W;
    if (ra < na && b < nb) __builtin_nontemporal_store(tile[b * ROW + ra * W + w], q + (int64_t)ra * d.da + m);
  }
}

struct Variant {
  char name[64];
  void (*launch)(const u4*, u4*, int64_t K0);
  std::vector<float> ms;
  bool ok;
};

template <int W, int TAU, int TB, int THREADS, bool LF>
void launch_v(const u4* src, u4* dst, int64_t K0) {
  Desc d;
  d.La = 256; d.Lb = K0;
  d.sb = 256LL * 256 * W; d.da = K0 * W;
  d.sbt = 256LL * W; d.dbt = 256LL * K0 * W;
  constexpr int TA = TAU / W;
  d.ntB = (d.Lb + TB - 1) / TB;
  d.ntAB = ((d.La + TA - 1) / TA) * d.ntB;
  d.ntiles = d.ntAB * 256;
  krt<W, TAU, TB, THREADS, LF><<<(int)d.ntiles, THREADS>>>(src, dst, d);
}

template <int W, int TAU, int TB, int THREADS, bool LF>
Variant V() {
  Variant v;
  snprintf(v.name, sizeof v.name, "TAU %3d (%5dB) x TB %3d t%d %s (%3dKB)", TAU, TAU * 16, TB, THREADS, LF ? "LF" : "  ",
           TAU * TB * 16 / 1024);
  v.launch = &launch_v<W, TAU, TB, THREADS, LF>;
  v.ok = false;
  return v;
}

int main() {
  const int64_t K0 = 512, K1 = 256, V0 = 256, R = 32;
  const int64_t n = K0 * K1 * V0 * R;  // float32 elements
  uint32_t *src, *dst;
  CK(hipMalloc(&src, n * 4)); CK(hipMalloc(&dst, n * 4));
  std::vector<uint32_t> h(n), hh(n), ref(n);
  for (int64_t i = 0; i < n; ++i) h[i] = (uint32_t)(i * 2654435761u);
  CK(hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice));
  // ref[k1][v0][k0][r] = h[k0][k1][v0][r]
  for (int64_t k0 = 0; k0 < K0; ++k0)
    for (int64_t k1 = 0; k1 < K1; ++k1)
      for (int64_t v0 = 0; v0 < V0; ++v0)
        memcpy(&ref[((k1 * V0 + v0) * K0 + k0) * R], &h[((k0 * K1 + k1) * V0 + v0) * R], R * 4);
  std::vector<Variant> vs = {
      V<8, 128, 16, 256, false>(),  // product
      V<8, 128, 16, 256, true>(),
      V<8, 128, 32, 256, true>(),
      V<8, 64, 32, 256, true>(),
      V<8, 64, 16, 256, true>(),
      V<8, 256, 8, 256, true>(),
      V<8, 64, 64, 256, true>(),
      V<8, 32, 64, 256, true>(),
      V<8, 128, 32, 512, true>(),
  };
  for (auto& v : vs) {
    CK(hipMemset(dst, 0, n * 4));
    v.launch((const u4*)src, (u4*)dst, K0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hh.data(), dst, n * 4, hipMemcpyDeviceToHost));
    v.ok = memcmp(hh.data(), ref.data(), n * 4) == 0;
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int rounds = 5, rr = 5;
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      v.launch((const u4*)src, (u4*)dst, K0);
      CK(hipEventRecord(e0));
      for (int i = 0; i < rr; ++i) v.launch((const u4*)src, (u4*)dst, K0);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / rr);
    }
  for (auto& v : vs) {
    std::vector<float> m = v.ms;
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    printf("%-48s median %7.4f ms %7.1f GB/s  %s\n", v.name, med, 2.0 * n * 4 / (med * 1e-3) / 1e9, v.ok ? "ok" : "MISMATCH");
  }
  return 0;
}

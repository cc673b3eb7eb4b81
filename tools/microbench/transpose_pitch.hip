// Microbenchmark: a padded destination pitch for the C2 transpose.
// [2000][262144] f32 -> [262144][P] with 2000 valid elements per destination
// row: P = 2000 (C2's dense 8000-B rows, every other one 64 B off a line),
// 2016 / 2048 (line-aligned padded rows).  profiles/r02_rowalign.log varied
// the row length itself (Lb 2048: 7.7% more bytes per us than 2000); here the
// data is C2's and only where the rows start changes.  The shipped 64x256
// register-staged tiles.  Every variant's valid bytes are compared with P =
// 2000's.  Also the rows reduction's input side: a sum over each 2000-element
// row at each pitch (one wave per row, 16-B loads), the read pattern of the
// C2 mean / std.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/tpitch.bin tools/microbench/transpose_pitch.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef __attribute__((ext_vector_type(4))) uint32_t u4;
typedef __attribute__((ext_vector_type(4))) float f4;

__global__ void __launch_bounds__(256) kt(const float* __restrict__ src, float* __restrict__ dst, int64_t La,
                                          int64_t Lb, int64_t P, int64_t ntB) {
  constexpr int TA = 64, TB = 256, NT = 256, VEC = 4;
  __shared__ float tile[TB][TA + 1];
  constexpr int NVA = TA / VEC, RPA = NT / NVA, NL = TB / RPA;
  constexpr int NVB = TB / VEC, RPB = NT / NVB, NS = TA / RPB;
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
  const int64_t t = blockIdx.x, tb = t % ntB, ta = t / ntB;
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
      __builtin_nontemporal_store(w, reinterpret_cast<u4*>(dst + (a0 + ra) * P + b0 + ux * VEC));
    }
  }
}

// one wave per row: sum of the row's n floats at pitch P (16-B loads, 2 in flight)
__global__ void __launch_bounds__(256) krows(const float* __restrict__ src, float* __restrict__ out, int64_t rows,
                                             int n, int64_t P) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* r = src + row * P;
  double acc = 0.0;
  for (int j = lane * 4; j < n; j += 512) {
    f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(r + j));
    acc += (double)a.x + a.y + a.z + a.w;
    if (j + 256 < n) {
      f4 b = __builtin_nontemporal_load(reinterpret_cast<const f4*>(r + j + 256));
      acc += (double)b.x + b.y + b.z + b.w;
    }
  }
  for (int o = 32; o; o >>= 1) acc += __shfl_down(acc, o);
  if (lane == 0) out[row] = (float)acc;
}

int main(int argc, char** argv) {
  const int64_t Lb = 2000, La = 262144;
  const int64_t sbytes = Lb * La * 4;
  const int pitches[] = {2000, 2016, 2048};
  const int nbuf = argc > 1 ? atoi(argv[1]) : 1;
  std::vector<float*> srcs(nbuf);
  for (auto& s : srcs) CK(hipMalloc(&s, sbytes));
  float *dst, *red;
  CK(hipMalloc(&dst, La * 2048 * 4));
  CK(hipMalloc(&red, La * 4));
  std::vector<uint8_t> h(sbytes);
  for (int64_t i = 0; i < sbytes; ++i) h[i] = (uint8_t)((i * 2654435761ull) >> 13);
  for (int64_t i = 3; i < sbytes; i += 4) h[i] = 0x3f;  // sane floats for the sums
  for (auto& s : srcs) CK(hipMemcpy(s, h.data(), sbytes, hipMemcpyHostToDevice));
  const int64_t ntB = (Lb + 255) / 256;
  // correctness: every pitch's valid bytes equal the dense result
  std::vector<float> dense(La * Lb), got(La * 2048);
  kt<<<(int)(La / 64 * ntB), 256>>>(srcs[0], dst, La, Lb, 2000, ntB);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(dense.data(), dst, La * Lb * 4, hipMemcpyDeviceToHost));
  bool ok[3] = {true, true, true};
  for (int pi = 1; pi < 3; ++pi) {
    const int P = pitches[pi];
    kt<<<(int)(La / 64 * ntB), 256>>>(srcs[0], dst, La, Lb, P, ntB);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), dst, La * P * 4, hipMemcpyDeviceToHost));
    for (int64_t a = 0; a < La && ok[pi]; ++a)
      ok[pi] = memcmp(&got[a * P], &dense[a * Lb], Lb * 4) == 0;
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int rounds = 7, rr = 8;
  for (int bu = 0; bu < nbuf; ++bu) {
    std::vector<float> tm[3], rm[3];
    for (int r = 0; r < rounds; ++r)
      for (int pi = 0; pi < 3; ++pi) {
        const int P = pitches[pi];
        kt<<<(int)(La / 64 * ntB), 256>>>(srcs[bu], dst, La, Lb, P, ntB);
        CK(hipEventRecord(e0));
        for (int i = 0; i < rr; ++i) kt<<<(int)(La / 64 * ntB), 256>>>(srcs[bu], dst, La, Lb, P, ntB);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        tm[pi].push_back(ms / rr);
        krows<<<(int)(La / 4), 256>>>(dst, red, La, (int)Lb, P);
        CK(hipEventRecord(e0));
        for (int i = 0; i < rr; ++i) krows<<<(int)(La / 4), 256>>>(dst, red, La, (int)Lb, P);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        rm[pi].push_back(ms / rr);
      }
    printf("source buffer %d\n", bu);
    for (int pi = 0; pi < 3; ++pi) {
      std::sort(tm[pi].begin(), tm[pi].end());
      std::sort(rm[pi].begin(), rm[pi].end());
      const double t = tm[pi][rounds / 2], q = rm[pi][rounds / 2];
      printf("  pitch %4d  transpose %7.4f ms %7.1f GB/s  rows-sum %7.4f ms %7.1f GB/s  %s\n", pitches[pi], t,
             2.0 * sbytes / (t * 1e-3) / 1e9, q, 1.0 * sbytes / (q * 1e-3) / 1e9, ok[pi] ? "ok" : "MISMATCH");
    }
    fflush(stdout);
  }
  return 0;
}

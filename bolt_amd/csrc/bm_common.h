// bm_common.h -- shared helpers for libbolt_mi355x (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>

#define BM_MAXD 16

// ---------------------------------------------------------------------------
// FastDiv: 64-bit division by a runtime-invariant divisor with one mul-hi.
// "Round-up" magic (Hacker's Delight 10-9 / libdivide branchfree u64):
//   l = ceil(log2 d), m = floor(2^64 (2^l - d) / d) + 1,
//   q = (t + ((n - t) >> 1)) >> (l - 1),  t = mulhi(m, n)
// exact for every n < 2^64 and 2 <= d < 2^63; d == 1 is flagged.
// Host and device share the code so the host test can check it exhaustively.
// ---------------------------------------------------------------------------
struct FastDiv {
  uint64_t d;
  uint64_t m;
  uint32_t s;
  uint32_t is1;
};

static inline FastDiv make_fastdiv(uint64_t d) {
  FastDiv f;
  f.d = d;
  f.is1 = (d <= 1) ? 1u : 0u;
  f.m = 0;
  f.s = 0;
  if (d <= 1) return f;
  int l = 64 - __builtin_clzll(d - 1);  // ceil(log2 d), 1..63
  unsigned __int128 num = ((unsigned __int128)((1ull << l) - d)) << 64;
  f.m = (uint64_t)(num / d) + 1;
  f.s = (uint32_t)(l - 1);
  return f;
}

__host__ __device__ __forceinline__ uint64_t bm_mulhi(uint64_t a, uint64_t b) {
  return (uint64_t)(((unsigned __int128)a * (unsigned __int128)b) >> 64);
}

__host__ __device__ __forceinline__ uint64_t fd_div(uint64_t n, const FastDiv &f) {
  if (f.is1) return n;
  uint64_t t = bm_mulhi(f.m, n);
  return (t + ((n - t) >> 1)) >> f.s;
}

// Mixed-radix decomposition of a linear index over up to BM_MAXD dims,
// stored innermost first; accumulates source and destination offsets.
struct Decomp {
  int32_t n;
  int32_t pad_;
  FastDiv div[BM_MAXD];
  int64_t ss[BM_MAXD];
  int64_t ds[BM_MAXD];
};

__device__ __forceinline__ void decomp2(uint64_t idx, const Decomp &d, int64_t &so,
                                        int64_t &dof) {
  so = 0;
  dof = 0;
  const int n = d.n;
  for (int k = 0; k + 1 < n; ++k) {
    const uint64_t q = fd_div(idx, d.div[k]);
    const uint64_t r = idx - q * d.div[k].d;
    so += (int64_t)r * d.ss[k];
    dof += (int64_t)r * d.ds[k];
    idx = q;
  }
  if (n > 0) {  // outermost: the remaining index is the coordinate
    so += (int64_t)idx * d.ss[n - 1];
    dof += (int64_t)idx * d.ds[n - 1];
  }
}

// decomp2 with the dim count known at compile time (ND >= 1): the loop
// unrolls, so every divisor and stride is loaded into scalar registers once
// per wave instead of once per dim per work item (the runtime loop indexes
// the kernel-argument arrays with a loop counter, and each iteration waits
// for its scalar loads).  ND = 0: the runtime loop.
template <int ND>
__device__ __forceinline__ void decomp_n(uint64_t idx, const Decomp &d, int64_t &so, int64_t &dof) {
  if constexpr (ND == 0) {
    decomp2(idx, d, so, dof);
  } else {
    so = 0;
    dof = 0;
#pragma unroll
    for (int k = 0; k + 1 < ND; ++k) {
      const uint64_t q = fd_div(idx, d.div[k]);
      const uint64_t r = idx - q * d.div[k].d;
      so += (int64_t)r * d.ss[k];
      dof += (int64_t)r * d.ds[k];
      idx = q;
    }
    so += (int64_t)idx * d.ss[ND - 1];
    dof += (int64_t)idx * d.ds[ND - 1];
  }
}

// decomp2 for up to 4 dims with every divisor and stride read at a constant
// kernel-argument offset (an unrolled, predicated loop: the scalar loads are
// hoisted to the kernel's start instead of one dependent load + wait per dim
// and call); more dims take decomp2.  For kernels that decompose once per tile.
__device__ __forceinline__ void decomp_le4(uint64_t idx, const Decomp &d, int64_t &so, int64_t &dof) {
  const int n = d.n;
  if (n > 4) {
    decomp2(idx, d, so, dof);
    return;
  }
  so = 0;
  dof = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < n) {
      uint64_t q = 0, r = idx;
      if (k + 1 < n) {
        q = fd_div(idx, d.div[k]);
        r = idx - q * d.div[k].d;
      }
      so += (int64_t)r * d.ss[k];
      dof += (int64_t)r * d.ds[k];
      idx = q;
    }
  }
}

// Byte vectors for wide global accesses.
template <int NB> struct VecB;
template <> struct VecB<1> { typedef uint8_t t; };
template <> struct VecB<2> { typedef uint16_t t; };
template <> struct VecB<4> { typedef uint32_t t; };
template <> struct VecB<8> { typedef __attribute__((ext_vector_type(2))) uint32_t t; };
template <> struct VecB<16> { typedef __attribute__((ext_vector_type(4))) uint32_t t; };

template <typename T, int N>
__device__ __forceinline__ void vload(const T *p, T (&out)[N]) {
  typedef typename VecB<N * sizeof(T)>::t V;
  V v = *reinterpret_cast<const V *>(p);
  __builtin_memcpy(out, &v, sizeof(V));
}

template <typename T, int N>
__device__ __forceinline__ void vstore(T *p, const T (&in)[N]) {
  typedef typename VecB<N * sizeof(T)>::t V;
  V v;
  __builtin_memcpy(&v, in, sizeof(V));
  *reinterpret_cast<V *>(p) = v;
}

// Streaming (non-temporal) variants: data that is read or written once per
// launch bypasses cache residency (measured on the C2 swap: NT stores +15%,
// NT loads +8% on top -- tools/microbench/transpose_variants.hip).
template <typename T, int N>
__device__ __forceinline__ void vload_nt(const T *p, T (&out)[N]) {
  typedef typename VecB<N * sizeof(T)>::t V;
  V v = __builtin_nontemporal_load(reinterpret_cast<const V *>(p));
  __builtin_memcpy(out, &v, sizeof(V));
}

template <typename T, int N>
__device__ __forceinline__ void vstore_nt(T *p, const T (&in)[N]) {
  typedef typename VecB<N * sizeof(T)>::t V;
  V v;
  __builtin_memcpy(&v, in, sizeof(V));
  __builtin_nontemporal_store(v, reinterpret_cast<V *>(p));
}

// thread-local error channel (bm_last_error)
void bm_set_error(const char *fmt, ...);

// bm_reduce.hip -- sum / mean / var / std reductions of libbolt_mi355x (gfx950).
//
// Replaces the Spark path's per-partition StatCounter (bolt/spark/
// statcounter.py:38-59, driven by array.py:321-322), its treeReduce of
// StatCounter.combine (statcounter.py:67-99, array.py:323) and the
// treeReduce(add) of reduce/sum (array.py:243-282).
//
// Layout: a C-contiguous array viewed as [O][R][I]; R is reduced.
//   cols kernel (I > 1): lanes own VEC adjacent columns, 16-B loads along I,
//     row phases stride R; phases are Chan-combined through LDS.
//   rows kernel (I == 1): one wave per (row, chunk), 16-B loads along R,
//     Chan combination across the 64 lanes by __shfl_xor.
//   Long R is split into chunks over blocks (enough waves to fill 256 CUs);
//   chunk states go to a workspace and a combine kernel merges them in chunk
//   order (deterministic) and finalises.
// Numerics: float64 pivot-shifted sums per lane (pivot = the lane's first
// element: S1 = sum(x-K), S2 = sum((x-K)^2), mean = K + S1/n,
// M2 = S2 - S1^2/n), Chan combination everywhere else.  SUM over integers is
// a uint64 modular sum truncated to the input width; SUM over bool is OR.
// All are HBM-bound: algorithmic bytes = N*elem_bytes + nout*out_bytes.
#include "bm_common.h"
#include "../../include/bolt_mi355x.h"

#include <cmath>

namespace {

constexpr int kThreads = 256;
constexpr int64_t kMaxBlocks = 0xffffffffLL / kThreads;  // HIP launch limit: grid * block threads < 2^32
#ifndef BM_COLS_UNROLL
#define BM_COLS_UNROLL 4  // rows in flight per lane in the column reductions (A/B knob)
#endif
#ifndef BM_COLS_BLOCKS
#define BM_COLS_BLOCKS 2048  // split R over blocks below this many column tiles (A/B knob)
#endif
constexpr int kColsUnroll = BM_COLS_UNROLL;
#ifndef BM_ROWS_UNROLL
#define BM_ROWS_UNROLL 2  // A/B on C2 rows: 2 beats 4 by 4%, 8 by 25% (profiles/r01_ab1.log)
#endif
constexpr int kRowsUnroll = BM_ROWS_UNROLL;  // 16-B vectors in flight per lane (rows kernel)

enum Mode { M_MEAN = 0, M_MOM = 1, M_FSUM = 2, M_ISUM = 3, M_OR = 4, M_MAX = 5, M_MIN = 6 };

// "bit modes" keep a uint64 accumulator: modular integer sum, OR (bool sum),
// and max / min holding the element's own bits (typed compares below).
template <int MODE> constexpr bool bit_mode() {
  return MODE == M_ISUM || MODE == M_OR || MODE == M_MAX || MODE == M_MIN;
}

template <typename T> __device__ __forceinline__ double to_f64(T x) { return (double)x; }
template <> __device__ __forceinline__ double to_f64<_Float16>(_Float16 x) { return (double)(float)x; }

template <typename T> __device__ __forceinline__ uint64_t to_u64(T x) {
  return (uint64_t)(int64_t)x;  // sign-extends signed types: modular sums stay exact
}
template <> __device__ __forceinline__ uint64_t to_u64<uint64_t>(uint64_t x) { return x; }
template <> __device__ __forceinline__ uint64_t to_u64<uint8_t>(uint8_t x) { return x; }
template <> __device__ __forceinline__ uint64_t to_u64<uint16_t>(uint16_t x) { return x; }
template <> __device__ __forceinline__ uint64_t to_u64<uint32_t>(uint32_t x) { return x; }

template <typename T> __device__ __forceinline__ uint64_t bits_of(T x) {
  uint64_t u = 0;
  __builtin_memcpy(&u, &x, sizeof(T));
  return u;
}
template <typename T> __device__ __forceinline__ T from_bits(uint64_t u) {
  T x;
  __builtin_memcpy(&x, &u, sizeof(T));
  return x;
}
template <typename T> __device__ __forceinline__ bool is_nan(T x) { return x != x; }

// numpy.maximum / numpy.minimum: a NaN operand wins (NaNs propagate)
template <typename T, bool MAX> __device__ __forceinline__ T pick(T a, T b) {
  if (is_nan(a)) return a;
  if (is_nan(b)) return b;
  return MAX ? (b > a ? b : a) : (b < a ? b : a);
}

template <typename T> struct Lim;
template <> struct Lim<uint8_t> { static __device__ uint8_t lo() { return 0; } static __device__ uint8_t hi() { return 0xff; } };
template <> struct Lim<int8_t> { static __device__ int8_t lo() { return -128; } static __device__ int8_t hi() { return 127; } };
template <> struct Lim<uint16_t> { static __device__ uint16_t lo() { return 0; } static __device__ uint16_t hi() { return 0xffff; } };
template <> struct Lim<int16_t> { static __device__ int16_t lo() { return -32768; } static __device__ int16_t hi() { return 32767; } };
template <> struct Lim<uint32_t> { static __device__ uint32_t lo() { return 0; } static __device__ uint32_t hi() { return 0xffffffffu; } };
template <> struct Lim<int32_t> { static __device__ int32_t lo() { return (-2147483647 - 1); } static __device__ int32_t hi() { return 2147483647; } };
template <> struct Lim<uint64_t> { static __device__ uint64_t lo() { return 0; } static __device__ uint64_t hi() { return ~0ull; } };
template <> struct Lim<int64_t> { static __device__ int64_t lo() { return (-9223372036854775807ll - 1); } static __device__ int64_t hi() { return 9223372036854775807ll; } };
template <> struct Lim<_Float16> { static __device__ _Float16 lo() { return -__builtin_inff16(); } static __device__ _Float16 hi() { return __builtin_inff16(); } };
template <> struct Lim<float> { static __device__ float lo() { return -__builtin_inff(); } static __device__ float hi() { return __builtin_inff(); } };
template <> struct Lim<double> { static __device__ double lo() { return -__builtin_inf(); } static __device__ double hi() { return __builtin_inf(); } };

// identity, element conversion and combination of the bit modes
template <typename T, int MODE> __device__ __forceinline__ uint64_t bident() {
  if (MODE == M_MAX) return bits_of<T>(Lim<T>::lo());
  if (MODE == M_MIN) return bits_of<T>(Lim<T>::hi());
  return 0;
}
template <typename T, int MODE> __device__ __forceinline__ uint64_t belem(T x) {
  if (MODE == M_ISUM) return to_u64(x);
  if (MODE == M_OR) return (uint64_t)(x != 0);
  return bits_of<T>(x);
}
template <typename T, int MODE> __device__ __forceinline__ uint64_t bop(uint64_t a, uint64_t b) {
  if (MODE == M_ISUM) return a + b;
  if (MODE == M_OR) return a | b;
  return bits_of<T>(pick<T, MODE == M_MAX>(from_bits<T>(a), from_bits<T>(b)));
}

// Per-lane accumulator for one output column.
template <int MODE> struct Acc;

template <> struct Acc<M_MEAN> {
  // two interleaved partial sums share the pivot: halves the add chain
  double K, S1, S1b;
  int64_t n;
  __device__ void init() { K = 0; S1 = 0; S1b = 0; n = 0; }
  __device__ void first(double x) { K = x; S1 = 0; S1b = 0; n = 1; }
  __device__ void pivot(double k) { K = k; S1 = 0; S1b = 0; n = 0; }
  __device__ double s1() const { return S1 + S1b; }
  __device__ double s2() const { return 0.0; }
  __device__ void add(double x) { S1 += x - K; ++n; }
  __device__ void add2(double x, double y) { S1 += x - K; S1b += y - K; n += 2; }
  __device__ double mean() const { return n ? K + (S1 + S1b) / (double)n : 0.0; }
  __device__ double m2() const { return 0.0; }
};

template <> struct Acc<M_MOM> {
  double K, S1, S2, S1b, S2b;
  int64_t n;
  __device__ void init() { K = 0; S1 = 0; S2 = 0; S1b = 0; S2b = 0; n = 0; }
  __device__ void first(double x) { K = x; S1 = 0; S2 = 0; S1b = 0; S2b = 0; n = 1; }
  __device__ void pivot(double k) { K = k; S1 = 0; S2 = 0; S1b = 0; S2b = 0; n = 0; }
  __device__ double s1() const { return S1 + S1b; }
  __device__ double s2() const { return S2 + S2b; }
  __device__ void add(double x) {
    const double dx = x - K;
    S1 += dx;
    S2 = fma(dx, dx, S2);
    ++n;
  }
  __device__ void add2(double x, double y) {
    const double dx = x - K, dy = y - K;
    S1 += dx;
    S2 = fma(dx, dx, S2);
    S1b += dy;
    S2b = fma(dy, dy, S2b);
    n += 2;
  }
  __device__ double mean() const { return n ? K + (S1 + S1b) / (double)n : 0.0; }
  __device__ double m2() const {
    if (!n) return 0.0;
    const double s1 = S1 + S1b;
    const double v = (S2 + S2b) - s1 * (s1 / (double)n);
    return v > 0.0 ? v : 0.0;
  }
};

// (n, K, S1, S2) of pivot-shifted sums -> mean, M2
__device__ __forceinline__ void from_sums(double n, double K, double s1, double s2, double &mean,
                                          double &m2) {
  mean = n > 0.0 ? K + s1 / n : 0.0;
  const double v = n > 0.0 ? s2 - s1 * (s1 / n) : 0.0;
  m2 = v > 0.0 ? v : 0.0;
}

// Chan et al. pairwise combination of (n, mean, M2) -- statcounter.py:85-96
// in its exact form (no 10x heuristic needed in float64).
__device__ __forceinline__ void chan(double &na, double &ma, double &qa, double nb, double mb,
                                     double qb, bool need_m2) {
  if (nb == 0.0) return;
  if (na == 0.0) {
    na = nb; ma = mb; qa = qb;
    return;
  }
  const double n = na + nb;
  const double delta = mb - ma;
  ma = ma + delta * (nb / n);
  if (need_m2) qa = qa + qb + delta * delta * (na * (nb / n));
  na = n;
}

__device__ __forceinline__ void store_out(void *out, int64_t idx, double v, int dt) {
  switch (dt) {
    case BM_F16: ((_Float16 *)out)[idx] = (_Float16)v; break;
    case BM_F32: ((float *)out)[idx] = (float)v; break;
    default: ((double *)out)[idx] = v; break;
  }
}

__device__ __forceinline__ void store_int(void *out, int64_t idx, uint64_t v, int dt) {
  switch (dt) {  // the low bytes of v, by the element width
    case BM_BOOL:
    case BM_U8:
    case BM_I8: ((uint8_t *)out)[idx] = (uint8_t)v; break;
    case BM_U16:
    case BM_I16:
    case BM_F16: ((uint16_t *)out)[idx] = (uint16_t)v; break;
    case BM_U32:
    case BM_I32:
    case BM_F32: ((uint32_t *)out)[idx] = (uint32_t)v; break;
    default: ((uint64_t *)out)[idx] = v; break;
  }
}

__device__ __forceinline__ double finish(int stat, double mean, double m2, double n) {
  if (stat == BM_STAT_MEAN) return mean;
  const double var = n > 0.0 ? m2 / n : __builtin_nan("");
  return stat == BM_STAT_VAR ? var : sqrt(var);
}

// Output sink: either final values or state planes (p0, p1) at index e.
struct Sink {
  void *out;        // final output (final_out != 0)
  int out_dtype;
  int stat;
  int final_out;
  double *p0;       // state plane 0 (mean / fsum) or uint64 plane (isum / or)
  double *p1;       // state plane 1 (M2)
};

template <int MODE>
__device__ __forceinline__ void emit(const Sink &sk, int64_t e, double n, double mean, double m2,
                                     uint64_t u) {
  if (bit_mode<MODE>()) {
    if (sk.final_out) store_int(sk.out, e, u, sk.out_dtype);
    else ((uint64_t *)sk.p0)[e] = u;
  } else if (MODE == M_FSUM) {
    if (sk.final_out) store_out(sk.out, e, mean, sk.out_dtype);
    else sk.p0[e] = mean;
  } else {
    if (sk.final_out) store_out(sk.out, e, finish(sk.stat, mean, m2, n), sk.out_dtype);
    else {
      sk.p0[e] = mean;
      if (MODE == M_MOM) sk.p1[e] = m2;
    }
  }
}

// ------------------------------------------------------------------ cols --
struct ColsDesc {
  int64_t O, R, I;
  int64_t rchunk;
  int64_t nchunks;
  int32_t tcv;  // threads across columns (power of two <= 256)
  int32_t nph;  // row phases = 256 / tcv
  FastDiv ntc;  // column tiles per O
  int64_t tile0;  // first (o, column tile) of this launch (launches split at the grid limit)
};

template <typename T, int VEC, int MODE>
__global__ void __launch_bounds__(kThreads)
    k_red_cols(const T *__restrict__ src, ColsDesc d, Sink sk) {
  __shared__ double sm0[kThreads * VEC];
  __shared__ double sm1[(MODE == M_MOM) ? kThreads * VEC : 1];
  const uint64_t ot = (uint64_t)d.tile0 + blockIdx.x;
  const uint64_t o = fd_div(ot, d.ntc);
  const uint64_t tc = ot - o * d.ntc.d;
  const int64_t c = blockIdx.y;
  const int64_t r_lo = c * d.rchunk;
  const int64_t r_hi = min(d.R, r_lo + d.rchunk);
  const int cv = threadIdx.x % d.tcv;
  const int ph = threadIdx.x / d.tcv;
  const int64_t col0 = ((int64_t)tc * d.tcv + cv) * VEC;
  const bool active = col0 < d.I;
  const int64_t nph = d.nph;

  Acc<(MODE == M_MOM) ? M_MOM : M_MEAN> acc[VEC];
  double fs[VEC];
  uint64_t us[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) { acc[k].init(); fs[k] = 0.0; us[k] = bident<T, MODE>(); }

  if (active) {
    const T *base = src + ((int64_t)o * d.R) * d.I + col0;
    int64_t r = r_lo + ph;
    if (MODE == M_MEAN || MODE == M_MOM) {
      // one pivot per column for every row phase of the block (the chunk's
      // first row): the phases then combine by plain sums, no divisions
      T k0[VEC];
      vload<T, VEC>(base + r_lo * d.I, k0);
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k].pivot(to_f64(k0[k]));
    }
    if constexpr (MODE == M_MEAN || MODE == M_MOM || MODE == M_FSUM) {
      // kColsUnroll rows in flight per lane; the adds stay in row order
      for (; r + (kColsUnroll - 1) * nph < r_hi; r += kColsUnroll * nph) {
        T v[kColsUnroll][VEC];
#pragma unroll
        for (int u = 0; u < kColsUnroll; ++u) vload_nt<T, VEC>(base + (r + u * nph) * d.I, v[u]);
#pragma unroll
        for (int u = 0; u < kColsUnroll; ++u) {
#pragma unroll
          for (int k = 0; k < VEC; ++k) {
            if (MODE == M_FSUM) fs[k] += to_f64(v[u][k]);
            else acc[k].add(to_f64(v[u][k]));
          }
        }
      }
    }
    for (; r + 3 * nph < r_hi; r += 4 * nph) {
      T v0[VEC], v1[VEC], v2[VEC], v3[VEC];
      vload_nt<T, VEC>(base + r * d.I, v0);
      vload_nt<T, VEC>(base + (r + nph) * d.I, v1);
      vload_nt<T, VEC>(base + (r + 2 * nph) * d.I, v2);
      vload_nt<T, VEC>(base + (r + 3 * nph) * d.I, v3);
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        if (MODE == M_MEAN || MODE == M_MOM) {
          acc[k].add(to_f64(v0[k])); acc[k].add(to_f64(v1[k]));
          acc[k].add(to_f64(v2[k])); acc[k].add(to_f64(v3[k]));
        } else if (MODE == M_FSUM) {
          fs[k] += to_f64(v0[k]); fs[k] += to_f64(v1[k]);
          fs[k] += to_f64(v2[k]); fs[k] += to_f64(v3[k]);
        } else {
          us[k] = bop<T, MODE>(us[k], bop<T, MODE>(bop<T, MODE>(belem<T, MODE>(v0[k]), belem<T, MODE>(v1[k])),
                                                   bop<T, MODE>(belem<T, MODE>(v2[k]), belem<T, MODE>(v3[k]))));
        }
      }
    }
    for (; r < r_hi; r += nph) {
      T v[VEC];
      vload_nt<T, VEC>(base + r * d.I, v);
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        if (MODE == M_MEAN || MODE == M_MOM) acc[k].add(to_f64(v[k]));
        else if (MODE == M_FSUM) fs[k] += to_f64(v[k]);
        else us[k] = bop<T, MODE>(us[k], belem<T, MODE>(v[k]));
      }
    }
  }

  // combine the row phases of each column through LDS (phase order)
  double n_own = 0.0;
  {
    const int64_t span = r_hi - r_lo - ph;
    n_own = span > 0 ? (double)((span + nph - 1) / nph) : 0.0;
  }
  // mean / moment modes carry the shared-pivot sums (S1, S2) until the end
  double m_[VEC], q_[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    if (MODE == M_MEAN || MODE == M_MOM) { m_[k] = acc[k].s1(); q_[k] = acc[k].s2(); }
    else if (MODE == M_FSUM) { m_[k] = fs[k]; q_[k] = 0.0; }
    else { m_[k] = __builtin_bit_cast(double, us[k]); q_[k] = 0.0; }
  }
  if (nph > 1) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      sm0[threadIdx.x * VEC + k] = m_[k];
      if (MODE == M_MOM) sm1[threadIdx.x * VEC + k] = q_[k];
    }
    __syncthreads();
    if (ph == 0) {
      double n0 = n_own;
      for (int p = 1; p < nph; ++p) {
        const int other = p * d.tcv + cv;
        const int64_t span = r_hi - r_lo - p;
        const double nb = span > 0 ? (double)((span + nph - 1) / nph) : 0.0;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const double mb = sm0[other * VEC + k];
          if (MODE == M_MEAN || MODE == M_MOM) {
            m_[k] += mb;
            if (MODE == M_MOM) q_[k] += sm1[other * VEC + k];
          } else if (MODE == M_FSUM) {
            m_[k] += mb;
          } else {
            m_[k] = __builtin_bit_cast(double, bop<T, MODE>(__builtin_bit_cast(uint64_t, m_[k]),
                                                            __builtin_bit_cast(uint64_t, mb)));
          }
        }
        n0 += nb;
      }
      n_own = n0;
    }
  }
  if (ph != 0 || !active) return;
  const double ntot = (double)(r_hi - r_lo);
  const int64_t plane = d.O * d.I;
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    if (MODE == M_MEAN || MODE == M_MOM) from_sums(ntot, acc[k].K, m_[k], q_[k], m_[k], q_[k]);
    const int64_t e = (int64_t)o * d.I + col0 + k;
    const int64_t idx = sk.final_out ? e : (c * plane + e);
    emit<MODE>(sk, idx, ntot, m_[k], q_[k], __builtin_bit_cast(uint64_t, m_[k]));
  }
}

// ------------------------------------------------------------------ rows --
struct RowsDesc {
  int64_t O, R;
  int64_t rchunk;
  FastDiv nchunks;
  int64_t nitems;  // O * nchunks
  int64_t item0;   // first item of this launch (launches split at the grid limit)
};

template <typename T, int VEC, int MODE>
__global__ void __launch_bounds__(kThreads)
    k_red_rows(const T *__restrict__ src, RowsDesc d, Sink sk) {
  const int lane = threadIdx.x & 63;
  const int64_t item = d.item0 + (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (item >= d.nitems) return;  // whole wave exits; no block barrier below
  const uint64_t o = fd_div((uint64_t)item, d.nchunks);
  const int64_t c = item - (int64_t)o * (int64_t)d.nchunks.d;
  const int64_t r_lo = c * d.rchunk;
  const int64_t r_hi = min(d.R, r_lo + d.rchunk);
  const T *row = src + (int64_t)o * d.R;

  Acc<(MODE == M_MOM) ? M_MOM : M_MEAN> acc;
  acc.init();
  double fs = 0.0;
  uint64_t us = bident<T, MODE>();
  int64_t j = r_lo + (int64_t)lane * VEC;
  const int64_t stride = 64 * VEC;
  // one pivot for the whole (row, chunk) -- its first element -- so the
  // 64 lanes combine by plain sums (no per-step division, see butterfly)
  if (MODE == M_MEAN || MODE == M_MOM) acc.pivot(to_f64(row[r_lo]));
  // kRowsUnroll 16-B vectors in flight per lane (HBM latency cover)
  for (; j + VEC + (kRowsUnroll - 1) * stride <= r_hi; j += kRowsUnroll * stride) {
    T v[kRowsUnroll][VEC];
#pragma unroll
    for (int u = 0; u < kRowsUnroll; ++u) vload_nt<T, VEC>(row + j + u * stride, v[u]);
#pragma unroll
    for (int u = 0; u < kRowsUnroll; ++u) {
      if constexpr ((MODE == M_MEAN || MODE == M_MOM) && VEC % 2 == 0) {
#pragma unroll
        for (int k = 0; k < VEC; k += 2) acc.add2(to_f64(v[u][k]), to_f64(v[u][k + 1]));
        continue;
      }
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        if (MODE == M_MEAN || MODE == M_MOM) acc.add(to_f64(v[u][k]));
        else if (MODE == M_FSUM) fs += to_f64(v[u][k]);
        else us = bop<T, MODE>(us, belem<T, MODE>(v[u][k]));
      }
    }
  }
  for (; j < r_hi; j += stride) {
    if (j + VEC <= r_hi) {
      T v[VEC];
      vload_nt<T, VEC>(row + j, v);
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        if (MODE == M_MEAN || MODE == M_MOM) acc.add(to_f64(v[k]));
        else if (MODE == M_FSUM) fs += to_f64(v[k]);
        else us = bop<T, MODE>(us, belem<T, MODE>(v[k]));
      }
    } else {
      for (int64_t k = j; k < r_hi; ++k) {
        if (MODE == M_MEAN || MODE == M_MOM) acc.add(to_f64(row[k]));
        else if (MODE == M_FSUM) fs += to_f64(row[k]);
        else us = bop<T, MODE>(us, belem<T, MODE>(row[k]));
      }
    }
  }

  // wave combination (butterfly, fixed order -> deterministic): shared
  // pivot, so the lanes' (S1, S2) simply add; the element count is known
  double m = acc.s1(), q = acc.s2();
  if (MODE == M_FSUM) m = fs;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    if (MODE == M_MEAN || MODE == M_MOM) {
      const double mb = __shfl_xor(m, off);
      const double qb = (MODE == M_MOM) ? __shfl_xor(q, off) : 0.0;
      // lower lane adds (self + partner), upper lane (partner + self):
      // the same ordered sum on both sides of every butterfly step
      m = (lane & off) ? (mb + m) : (m + mb);
      if (MODE == M_MOM) q = (lane & off) ? (qb + q) : (q + qb);
    } else if (MODE == M_FSUM) {
      const double mb = __shfl_xor(m, off);
      m = (lane & off) ? (mb + m) : (m + mb);
    } else {
      const uint64_t ub = (uint64_t)__shfl_xor((long long)us, off);
      us = (lane & off) ? bop<T, MODE>(ub, us) : bop<T, MODE>(us, ub);
    }
  }
  if (lane != 0) return;
  const double ntot = (double)(r_hi - r_lo);
  if (MODE == M_MEAN || MODE == M_MOM) from_sums(ntot, acc.K, m, q, m, q);
  const int64_t e = (int64_t)o;
  const int64_t idx = sk.final_out ? e : (c * d.O + e);
  emit<MODE>(sk, idx, ntot, m, q, us);
}

// --------------------------------------------------------------- combine --
struct CombDesc {
  int64_t nout;
  int64_t nparts;
  int64_t part_stride;  // elements between parts in a plane
  int64_t R, rchunk;    // uniform chunk counts when explicit == 0
  int32_t explicit_counts;
  int32_t pad_;
  int64_t counts[64];
};

template <int MODE, typename T>
__global__ void __launch_bounds__(kThreads)
    k_red_combine(const double *__restrict__ p0, const double *__restrict__ p1, CombDesc d, Sink sk) {
  const int64_t step = (int64_t)gridDim.x * kThreads;
  for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < d.nout; e += step) {
    double n = 0.0, m = 0.0, q = 0.0;
    uint64_t u = 0;
    bool first = true;
    for (int64_t p = 0; p < d.nparts; ++p) {
      const double nb = d.explicit_counts
                            ? (double)d.counts[p]
                            : (double)(min(d.R, (p + 1) * d.rchunk) - p * d.rchunk);
      if (nb <= 0.0) continue;
      const int64_t at = p * d.part_stride + e;
      if (MODE == M_MEAN || MODE == M_MOM) {
        chan(n, m, q, nb, p0[at], (MODE == M_MOM) ? p1[at] : 0.0, MODE == M_MOM);
      } else if (MODE == M_FSUM) {
        m += p0[at];
        n += nb;
      } else {
        const uint64_t b = ((const uint64_t *)p0)[at];
        u = first ? b : bop<T, MODE>(u, b);
      }
      first = false;
    }
    emit<MODE>(sk, e, n, m, q, u);
  }
}

// ------------------------------------------------------------------ host --
int dtype_size(int dt) {
  switch (dt) {
    case BM_BOOL: case BM_U8: case BM_I8: return 1;
    case BM_U16: case BM_I16: case BM_F16: return 2;
    case BM_U32: case BM_I32: case BM_F32: return 4;
    case BM_U64: case BM_I64: case BM_F64: return 8;
    default: return 0;
  }
}
bool is_float(int dt) { return dt == BM_F16 || dt == BM_F32 || dt == BM_F64; }

int mode_of(int stat, int dt) {
  if (stat == BM_STAT_MEAN) return M_MEAN;
  if (stat == BM_STAT_VAR || stat == BM_STAT_STD) return M_MOM;
  if (stat == BM_STAT_MAX) return M_MAX;
  if (stat == BM_STAT_MIN) return M_MIN;
  if (is_float(dt)) return M_FSUM;
  if (dt == BM_BOOL) return M_OR;
  return M_ISUM;
}
int planes_of(int mode) { return mode == M_MOM ? 2 : 1; }
bool bit_mode_host(int mode) { return mode == M_ISUM || mode == M_OR || mode == M_MAX || mode == M_MIN; }

struct RedPlan {
  bool rows;
  int vec;
  int64_t rchunk, nchunks;
  int32_t tcv, nph;
  int64_t ntc;
};

int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

RedPlan plan_reduce(int dt, int64_t O, int64_t R, int64_t I, const void *src) {
  RedPlan p{};
  const int es = dtype_size(dt);
  const bool al16 = src == nullptr || ((uintptr_t)src % 16) == 0;
  if (I == 1) {
    p.rows = true;
    int vec = 16 / es;
    while (vec > 1 && !(R % vec == 0 && (src == nullptr || ((uintptr_t)src % (vec * es)) == 0))) vec >>= 1;
    p.vec = vec;
    const int64_t target_waves = 8192;
    int64_t nch = 1;
    if (O < target_waves) {
      nch = cdiv(target_waves, O);
      const int64_t maxch = std::max<int64_t>(1, R / (64 * vec * 4));
      nch = std::min(nch, maxch);
    }
    int64_t rc = cdiv(R, nch);
    rc = cdiv(rc, vec) * vec;
    p.rchunk = rc;
    p.nchunks = cdiv(R, rc);
  } else {
    p.rows = false;
    int vec = std::min(16 / es, 8);
    (void)al16;
    while (vec > 1 && !(I % vec == 0 && (src == nullptr || ((uintptr_t)src % (vec * es)) == 0))) vec >>= 1;
    p.vec = vec;
    const int64_t ncolv = cdiv(I, vec);
    int tcv = 1;
    while (tcv < 256 && tcv < ncolv) tcv <<= 1;
    p.tcv = tcv;
    p.nph = 256 / tcv;
    p.ntc = cdiv(ncolv, tcv);
    const int64_t blocks = O * p.ntc;
    int64_t nch = 1;
    if (blocks < BM_COLS_BLOCKS) {
      nch = cdiv(BM_COLS_BLOCKS, blocks);
      const int64_t maxch = std::max<int64_t>(1, R / ((int64_t)p.nph * 8));
      nch = std::min(nch, maxch);
    }
    nch = std::min<int64_t>(nch, 65535);
    p.rchunk = cdiv(R, nch);
    p.nchunks = cdiv(R, p.rchunk);
  }
  return p;
}

template <typename T, int MODE>
int launch_main_t(const RedPlan &p, const void *src, int64_t O, int64_t R, int64_t I, Sink sk,
                  hipStream_t st) {
  const T *s = (const T *)src;
  if (p.rows) {
    RowsDesc d;
    d.O = O; d.R = R; d.rchunk = p.rchunk;
    d.nchunks = make_fastdiv((uint64_t)p.nchunks);
    d.nitems = O * p.nchunks;
    const int64_t blocks = cdiv(d.nitems, kThreads / 64);
    // one launch per kMaxBlocks blocks (HIP: grid * block threads < 2^32)
    for (int64_t b0 = 0; b0 < blocks; b0 += kMaxBlocks) {
      const int g = (int)std::min<int64_t>(kMaxBlocks, blocks - b0);
      d.item0 = b0 * (kThreads / 64);
      switch (p.vec) {
#define BM_ROWS_CASE(V) \
  case V: if constexpr (V * sizeof(T) <= 16) { k_red_rows<T, V, MODE><<<g, kThreads, 0, st>>>(s, d, sk); } break;
        BM_ROWS_CASE(16) BM_ROWS_CASE(8) BM_ROWS_CASE(4) BM_ROWS_CASE(2)
        default: k_red_rows<T, 1, MODE><<<g, kThreads, 0, st>>>(s, d, sk); break;
#undef BM_ROWS_CASE
      }
    }
  } else {
    ColsDesc d;
    d.O = O; d.R = R; d.I = I;
    d.rchunk = p.rchunk; d.nchunks = p.nchunks;
    d.tcv = p.tcv; d.nph = p.nph;
    d.ntc = make_fastdiv((uint64_t)p.ntc);
    const int64_t bx = O * p.ntc;
    const int64_t per = std::max<int64_t>(1, kMaxBlocks / p.nchunks);
    for (int64_t t0 = 0; t0 < bx; t0 += per) {
      d.tile0 = t0;
      dim3 grid((unsigned)std::min<int64_t>(per, bx - t0), (unsigned)p.nchunks);
      switch (p.vec) {
#define BM_COLS_CASE(V) \
  case V: if constexpr (V * sizeof(T) <= 16) { k_red_cols<T, V, MODE><<<grid, kThreads, 0, st>>>(s, d, sk); } break;
        BM_COLS_CASE(8) BM_COLS_CASE(4) BM_COLS_CASE(2)
        default: k_red_cols<T, 1, MODE><<<grid, kThreads, 0, st>>>(s, d, sk); break;
#undef BM_COLS_CASE
      }
    }
  }
  return BM_OK;
}

template <int MODE>
int launch_main_m(int dt, const RedPlan &p, const void *src, int64_t O, int64_t R, int64_t I,
                  Sink sk, hipStream_t st) {
  switch (dt) {
    case BM_BOOL:
    case BM_U8: return launch_main_t<uint8_t, MODE>(p, src, O, R, I, sk, st);
    case BM_I8: return launch_main_t<int8_t, MODE>(p, src, O, R, I, sk, st);
    case BM_U16: return launch_main_t<uint16_t, MODE>(p, src, O, R, I, sk, st);
    case BM_I16: return launch_main_t<int16_t, MODE>(p, src, O, R, I, sk, st);
    case BM_U32: return launch_main_t<uint32_t, MODE>(p, src, O, R, I, sk, st);
    case BM_I32: return launch_main_t<int32_t, MODE>(p, src, O, R, I, sk, st);
    case BM_U64: return launch_main_t<uint64_t, MODE>(p, src, O, R, I, sk, st);
    case BM_I64: return launch_main_t<int64_t, MODE>(p, src, O, R, I, sk, st);
    case BM_F16:
      if constexpr (MODE != M_ISUM && MODE != M_OR) return launch_main_t<_Float16, MODE>(p, src, O, R, I, sk, st);
      break;
    case BM_F32:
      if constexpr (MODE != M_ISUM && MODE != M_OR) return launch_main_t<float, MODE>(p, src, O, R, I, sk, st);
      break;
    case BM_F64:
      if constexpr (MODE != M_ISUM && MODE != M_OR) return launch_main_t<double, MODE>(p, src, O, R, I, sk, st);
      break;
    default: break;
  }
  bm_set_error("bm_reduce: unsupported dtype %d for this statistic", dt);
  return BM_E_ARG;
}

int launch_main(int mode, int dt, const RedPlan &p, const void *src, int64_t O, int64_t R,
                int64_t I, Sink sk, hipStream_t st) {
  switch (mode) {
    case M_MEAN: return launch_main_m<M_MEAN>(dt, p, src, O, R, I, sk, st);
    case M_MOM: return launch_main_m<M_MOM>(dt, p, src, O, R, I, sk, st);
    case M_FSUM: return launch_main_m<M_FSUM>(dt, p, src, O, R, I, sk, st);
    case M_ISUM: return launch_main_m<M_ISUM>(dt, p, src, O, R, I, sk, st);
    case M_MAX: return launch_main_m<M_MAX>(dt, p, src, O, R, I, sk, st);
    case M_MIN: return launch_main_m<M_MIN>(dt, p, src, O, R, I, sk, st);
    default: return launch_main_m<M_OR>(dt, p, src, O, R, I, sk, st);
  }
}

template <int MODE>
void launch_combine_m(int dt, int g, const double *p0, const double *p1, const CombDesc &cd, Sink sk,
                      hipStream_t st) {
  switch (dt) {  // only max/min look at the element type
    case BM_BOOL: case BM_U8: k_red_combine<MODE, uint8_t><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case BM_I8: k_red_combine<MODE, int8_t><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case BM_U16: k_red_combine<MODE, uint16_t><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case BM_I16: k_red_combine<MODE, int16_t><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case BM_U32: k_red_combine<MODE, uint32_t><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case BM_I32: k_red_combine<MODE, int32_t><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case BM_U64: k_red_combine<MODE, uint64_t><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case BM_I64: k_red_combine<MODE, int64_t><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case BM_F16: k_red_combine<MODE, _Float16><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case BM_F32: k_red_combine<MODE, float><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    default: k_red_combine<MODE, double><<<g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
  }
}

int launch_combine(int mode, int dt, const double *p0, const double *p1, const CombDesc &cd, Sink sk,
                   hipStream_t st) {
  int64_t g = cdiv(cd.nout, kThreads);
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  switch (mode) {
    case M_MEAN: k_red_combine<M_MEAN, double><<<(int)g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case M_MOM: k_red_combine<M_MOM, double><<<(int)g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case M_FSUM: k_red_combine<M_FSUM, double><<<(int)g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case M_ISUM: k_red_combine<M_ISUM, uint64_t><<<(int)g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case M_OR: k_red_combine<M_OR, uint64_t><<<(int)g, kThreads, 0, st>>>(p0, p1, cd, sk); break;
    case M_MAX: launch_combine_m<M_MAX>(dt, (int)g, p0, p1, cd, sk, st); break;
    default: launch_combine_m<M_MIN>(dt, (int)g, p0, p1, cd, sk, st); break;
  }
  return BM_OK;
}

int check_args(int stat, int dt, int64_t O, int64_t R, int64_t I, const char *who) {
  if (stat < BM_STAT_MEAN || stat > BM_STAT_MIN || dtype_size(dt) == 0) {
    bm_set_error("%s: bad stat %d / dtype %d", who, stat, dt);
    return BM_E_ARG;
  }
  if (O < 1 || R < 1 || I < 1) {
    bm_set_error("%s: empty reduction (O=%lld R=%lld I=%lld)", who, (long long)O, (long long)R,
                 (long long)I);
    return BM_E_ARG;
  }
  return BM_OK;
}

int check_launch(const char *who) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    bm_set_error("%s: launch failed: %s", who, hipGetErrorString(e));
    return BM_E_HIP;
  }
  return BM_OK;
}

size_t ws_bytes_for(int mode, const RedPlan &p, int64_t nout) {
  if (p.nchunks <= 1) return 0;
  return (size_t)planes_of(mode) * (size_t)p.nchunks * (size_t)nout * 8;
}

// Shared body of bm_reduce / bm_reduce_state.
int run_reduce(int stat, const void *src, int dt, int64_t O, int64_t R, int64_t I, Sink sk,
               void *ws, size_t ws_bytes, hipStream_t st, const char *who) {
  const int mode = mode_of(stat, dt);
  const RedPlan p = plan_reduce(dt, O, R, I, src);
  const int64_t nout = O * I;
  if (p.nchunks <= 1) {
    int rc = launch_main(mode, dt, p, src, O, R, I, sk, st);
    if (rc) return rc;
    return check_launch(who);
  }
  const size_t need = ws_bytes_for(mode, p, nout);
  if (!ws || ws_bytes < need) {
    bm_set_error("%s: workspace too small (%zu < %zu)", who, ws_bytes, need);
    return BM_E_WS;
  }
  double *w0 = (double *)ws;
  double *w1 = w0 + (size_t)p.nchunks * nout;
  Sink part = sk;
  part.final_out = 0;
  part.p0 = w0;
  part.p1 = w1;
  int rc = launch_main(mode, dt, p, src, O, R, I, part, st);
  if (rc) return rc;
  CombDesc cd{};
  cd.nout = nout;
  cd.nparts = p.nchunks;
  cd.part_stride = nout;
  cd.R = R;
  cd.rchunk = p.rchunk;
  cd.explicit_counts = 0;
  rc = launch_combine(mode, dt, w0, w1, cd, sk, st);
  if (rc) return rc;
  return check_launch(who);
}

}  // namespace

extern "C" int bm_reduce_workspace_bytes(int stat, int in_dtype, int64_t O, int64_t R, int64_t I,
                                         size_t *bytes) {
  if (!bytes) { bm_set_error("bm_reduce_workspace_bytes: null out"); return BM_E_ARG; }
  int rc = check_args(stat, in_dtype, O, R, I, "bm_reduce_workspace_bytes");
  if (rc) return rc;
  // The plan depends on the pointer only through the vector width; reserve
  // for both the 16-B-aligned plan and the scalar (unaligned) plan.
  const int mode = mode_of(stat, in_dtype);
  const size_t a = ws_bytes_for(mode, plan_reduce(in_dtype, O, R, I, nullptr), O * I);
  const size_t b = ws_bytes_for(mode, plan_reduce(in_dtype, O, R, I, (const void *)1), O * I);
  *bytes = a > b ? a : b;
  return BM_OK;
}

extern "C" int bm_reduce(int stat, const void *src, int in_dtype, int64_t O, int64_t R, int64_t I,
                         void *out, int out_dtype, void *workspace, size_t workspace_bytes,
                         void *stream) {
  int rc = check_args(stat, in_dtype, O, R, I, "bm_reduce");
  if (rc) return rc;
  if (!src || !out) { bm_set_error("bm_reduce: null pointer"); return BM_E_ARG; }
  const int mode = mode_of(stat, in_dtype);
  if (bit_mode_host(mode)) {
    if (out_dtype != in_dtype) { bm_set_error("bm_reduce: integer sum / max / min keep the input dtype"); return BM_E_ARG; }
  } else if (!is_float(out_dtype)) {
    bm_set_error("bm_reduce: out_dtype must be a float dtype");
    return BM_E_ARG;
  }
  Sink sk{};
  sk.out = out;
  sk.out_dtype = out_dtype;
  sk.stat = stat;
  sk.final_out = 1;
  return run_reduce(stat, src, in_dtype, O, R, I, sk, workspace, workspace_bytes,
                    (hipStream_t)stream, "bm_reduce");
}

extern "C" int bm_reduce_state_bytes(int stat, int in_dtype, int64_t nout, size_t *bytes) {
  if (!bytes || nout < 0 || stat < BM_STAT_MEAN || stat > BM_STAT_MIN || dtype_size(in_dtype) == 0) {
    bm_set_error("bm_reduce_state_bytes: bad arguments");
    return BM_E_ARG;
  }
  *bytes = (size_t)planes_of(mode_of(stat, in_dtype)) * (size_t)nout * 8;
  return BM_OK;
}

extern "C" int bm_reduce_state(int stat, const void *src, int in_dtype, int64_t O, int64_t R,
                               int64_t I, void *state, void *workspace, size_t workspace_bytes,
                               void *stream) {
  int rc = check_args(stat, in_dtype, O, R, I, "bm_reduce_state");
  if (rc) return rc;
  if (!src || !state) { bm_set_error("bm_reduce_state: null pointer"); return BM_E_ARG; }
  const int64_t nout = O * I;
  Sink sk{};
  sk.out = nullptr;
  sk.out_dtype = BM_F64;
  sk.stat = stat;
  sk.final_out = 0;
  sk.p0 = (double *)state;
  sk.p1 = (double *)state + nout;
  return run_reduce(stat, src, in_dtype, O, R, I, sk, workspace, workspace_bytes,
                    (hipStream_t)stream, "bm_reduce_state");
}

extern "C" int bm_reduce_combine(int stat, int in_dtype, const void *states, const int64_t *counts,
                                 int nparts, int64_t nout, void *out, int out_dtype, void *stream) {
  if (stat < BM_STAT_MEAN || stat > BM_STAT_MIN || dtype_size(in_dtype) == 0 || nparts < 1 ||
      nparts > 64 || nout < 1 || !states || !counts || !out) {
    bm_set_error("bm_reduce_combine: bad arguments");
    return BM_E_ARG;
  }
  const int mode = mode_of(stat, in_dtype);
  if (bit_mode_host(mode)) {
    if (out_dtype != in_dtype) { bm_set_error("bm_reduce_combine: integer sum / max / min keep the input dtype"); return BM_E_ARG; }
  } else if (!is_float(out_dtype)) {
    bm_set_error("bm_reduce_combine: out_dtype must be a float dtype");
    return BM_E_ARG;
  }
  CombDesc cd{};
  cd.nout = nout;
  cd.nparts = nparts;
  cd.part_stride = (int64_t)planes_of(mode) * nout;
  cd.explicit_counts = 1;
  for (int p = 0; p < nparts; ++p) cd.counts[p] = counts[p];
  Sink sk{};
  sk.out = out;
  sk.out_dtype = out_dtype;
  sk.stat = stat;
  sk.final_out = 1;
  const double *p0 = (const double *)states;
  int rc = launch_combine(mode, in_dtype, p0, p0 + nout, cd, sk, (hipStream_t)stream);
  if (rc) return rc;
  return check_launch("bm_reduce_combine");
}

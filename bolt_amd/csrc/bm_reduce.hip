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
//     lane states folded across the 64 lanes through DPP moves (wave_fold).
//   Long R is split into chunks over blocks (enough waves to fill 256 CUs);
//   chunk states go to a workspace and a combine kernel merges them in chunk
//   order (deterministic) and finalises.
// Numerics (all float64):
//   var / std: batched Welford.  Each lane reduces the B values of one load
//     batch (B = vectors in flight x vector width, 1..32) around a pivot that
//     is one of those values, so the batch's M2 = S2 - S1^2/B carries at most
//     O(B eps) relative error whatever the data's offset or outliers; the
//     batch state (B, mean_b, M2_b) is then merged into the lane's running
//     (n, mean, M2) by Chan's formula (statcounter.py:85-96), as are lanes,
//     row phases, chunks and ranks, always in a fixed order (deterministic).
//   mean: pivot-shifted sums around the (row, chunk)'s first element,
//     mean = K + S1/n (no cancellation: the error is eps-relative to max|x|).
//   SUM over floats is a float64 sum; over integers a uint64 modular sum
//   truncated to the input width; over bool an OR.
// All are HBM-bound: algorithmic bytes = N*elem_bytes + nout*out_bytes.
#include "bm_common.h"
#include "../../include/bolt_mi355x.h"

#include <cmath>

namespace {

constexpr int kThreads = 256;
constexpr int64_t kMaxBlocks = 0xffffffffLL / kThreads;  // HIP launch limit: grid * block threads < 2^32
// Shipped parameters (the A/B runs that chose them are cited; the rejected
// values live in git history and tools/microbench/):
// rows in flight per lane in the column reductions: 8 over 4 +1.2-1.4% on the
// 64 GiB target mean / std and C2-shape columns, 2 -4-8% (profiles/r02_ab_cols.log);
// on round 6's 64-vector tiles 16 is within +0.2..+1.4% of 8 (two placements,
// profiles/r06l_ab_cols_unroll.log): 8 stays (half the load registers)
constexpr int kColsUnroll = 8;
// split R over blocks below this many column tiles; column vectors per block
// at most (the rest of the 256 lanes are row phases); the narrowest tile taken
// to reach kColsBlocks before chunking R (profiles/r03zb_ab_tcv.log, r03zc_ab_tcv_rule.log).
// Round 6: 64-vector tiles (four row phases per block) for every shape, not
// only the few-tile ones: the 64 GiB target's mean / std over axis 0
// +0.8..+1.8% on two placements, 128-vector tiles +0.7..+1.7%, C2 / C4
// columns +-0.3% (profiles/r06j_ab_cols_tiles.log, r06k_ab_cols_tiles.log; the
// column kernels had 4x the rows kernel's DRAM read-credit stalls per byte,
// r06i_cols_vs_rows_counters.md); 32 B per lane lost 6-12%
constexpr int64_t kColsBlocks = 2048;
constexpr int64_t kColsTcv = 64;
constexpr int64_t kColsTcvMin = 64;
// 16-B vectors in flight per lane in the rows kernel: 2 beats 4 by 4%, 8 by 25%
// (profiles/r01_ab1.log; 3: equal, 4: -5% again on padded rows, r05z_rows_unroll.txt)
constexpr int kRowsUnroll = 2;
// exact-integer column var: rows in flight per lane (C4 var 3.76 -> 3.47 ms over 4, profiles/r02_ab_int.log)
constexpr int kIntUnroll = 8;
// rows kernel: blocks dealt to one XCD take consecutive rows (C2 mean / std
// +3-4%, profiles/r02_ab_redxcd.log); column kernels: blocks dealt to one XCD
// take consecutive column tiles (C4 var +1.1%, 64 GiB-target-shaped mean / std
// over axis 0 +2.2% / +1.6%, profiles/r05h_ab_cols_xcd.log)

enum Mode {
  M_MEAN = 0, M_MOM = 1, M_FSUM = 2, M_ISUM = 3, M_OR = 4, M_MAX = 5, M_MIN = 6,
  M_FPROD = 7, M_IPROD = 8, M_LAND = 9, M_BAND = 10, M_BOR = 11, M_BXOR = 12, M_FMAX = 13, M_FMIN = 14
};

// "bit modes" keep a uint64 accumulator: modular integer sum / product,
// logical OR (bool sum, logical_or) / AND, bitwise and / or / xor, and
// max / min / fmax / fmin holding the element's own bits (typed compares).
template <int MODE> constexpr bool bit_mode() {
  return MODE == M_ISUM || MODE == M_OR || MODE == M_MAX || MODE == M_MIN || MODE == M_IPROD ||
         MODE == M_LAND || MODE == M_BAND || MODE == M_BOR || MODE == M_BXOR || MODE == M_FMAX ||
         MODE == M_FMIN;
}
// float-accumulating modes: a float64 sum or product
template <int MODE> constexpr bool facc_mode() { return MODE == M_FSUM || MODE == M_FPROD; }
template <int MODE> __device__ __forceinline__ double fident() { return MODE == M_FPROD ? 1.0 : 0.0; }
template <int MODE> __device__ __forceinline__ double fop(double a, double b) {
  return MODE == M_FPROD ? a * b : a + b;
}
// modes meaningless for floating inputs (numpy raises for bitwise ufuncs)
template <int MODE> constexpr bool int_only_mode() {
  return MODE == M_ISUM || MODE == M_IPROD || MODE == M_BAND || MODE == M_BOR || MODE == M_BXOR;
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

// ---- wave fold through DPP ----
// A 64-bit lane value moved by a DPP modifier of v_mov (two 32-bit halves, the
// same source lane): the cross-lane read stays in the VALU, no LDS round trip
// as __shfl_xor's ds_bpermute takes.  Controls (GFX9 DPP): quad_perm [1,0,3,2]
// = 0xB1 (lane ^ 1), [2,3,0,1] = 0x4E (lane ^ 2), row_half_mirror 0x141
// (lane 7-i of its 8), row_mirror 0x140 (lane 15-i of its row), row_bcast15
// 0x142 (lane 15 of row r -> row r+1), row_bcast31 0x143 (lane 31 -> rows 2, 3).
template <int CTRL, typename V> __device__ __forceinline__ V dpp_mov(V v) {
  static_assert(sizeof(V) == 8, "64-bit lane values");
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(V, ((uint64_t)hi << 32) | lo);
}
// Lane 63 receives op over all 64 lanes, combined in lane order: every step
// combines (lower lanes, upper lanes), so the result equals a left fold over
// lanes 0..63 for any associative op (first NaN / first of equal values wins,
// as in a sequential scan).  Steps 1-4 leave identical bits in the lanes that
// feed the next step (both lanes of a pair form op(lower, upper)); steps 5-6
// fold the four 16-lane rows.  Requires all 64 lanes active.
template <typename V, typename F> __device__ __forceinline__ V wave_fold(V v, int lane, F op) {
  V p = dpp_mov<0xB1>(v);
  v = (lane & 1) ? op(p, v) : op(v, p);
  p = dpp_mov<0x4E>(v);
  v = (lane & 2) ? op(p, v) : op(v, p);
  p = dpp_mov<0x141>(v);
  v = (lane & 4) ? op(p, v) : op(v, p);
  p = dpp_mov<0x140>(v);
  v = (lane & 8) ? op(p, v) : op(v, p);
  p = dpp_mov<0x142>(v);
  if (lane & 16) v = op(p, v);  // lane 31 = rows 0+1, lane 63 = rows 2+3
  p = dpp_mov<0x143>(v);
  if (lane & 32) v = op(p, v);  // lane 63 = (rows 0+1) + (rows 2+3)
  return v;
}
constexpr int kFoldLane = 63;
// lane 0's value in every lane (v_readlane into a scalar register)
__device__ __forceinline__ double lane0_of(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, 0);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 0);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// numpy.maximum / numpy.minimum: a NaN operand wins (NaNs propagate)
template <typename T, bool MAX> __device__ __forceinline__ T pick(T a, T b) {
  if (is_nan(a)) return a;
  if (is_nan(b)) return b;
  return MAX ? (b > a ? b : a) : (b < a ? b : a);
}
// numpy.fmax / numpy.fmin: a NaN operand loses (NaN only if both are NaN)
template <typename T, bool MAX> __device__ __forceinline__ T pickf(T a, T b) {
  if (is_nan(a)) return b;
  if (is_nan(b)) return a;
  return MAX ? (b > a ? b : a) : (b < a ? b : a);
}
template <typename T> __device__ __forceinline__ T qnan() { return T(0); }
template <> __device__ __forceinline__ _Float16 qnan<_Float16>() { return (_Float16)__builtin_nanf(""); }
template <> __device__ __forceinline__ float qnan<float>() { return __builtin_nanf(""); }
template <> __device__ __forceinline__ double qnan<double>() { return __builtin_nan(""); }
template <typename T> constexpr bool is_float_t() {
  return std::is_same<T, _Float16>::value || std::is_same<T, float>::value || std::is_same<T, double>::value;
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
  // fmax / fmin: NaN is the identity of floats (all-NaN -> NaN)
  if (MODE == M_FMAX) return bits_of<T>(is_float_t<T>() ? qnan<T>() : Lim<T>::lo());
  if (MODE == M_FMIN) return bits_of<T>(is_float_t<T>() ? qnan<T>() : Lim<T>::hi());
  if (MODE == M_IPROD || MODE == M_LAND) return 1;
  if (MODE == M_BAND) return ~0ull;
  return 0;
}
template <typename T, int MODE> __device__ __forceinline__ uint64_t belem(T x) {
  if (MODE == M_ISUM || MODE == M_IPROD) return to_u64(x);
  if (MODE == M_OR || MODE == M_LAND) return (uint64_t)(x != 0);
  return bits_of<T>(x);
}
template <typename T, int MODE> __device__ __forceinline__ uint64_t bop(uint64_t a, uint64_t b) {
  if (MODE == M_ISUM) return a + b;
  if (MODE == M_IPROD) return a * b;  // modular: the low bits depend only on the low bits
  if (MODE == M_OR || MODE == M_BOR) return a | b;
  if (MODE == M_LAND || MODE == M_BAND) return a & b;
  if (MODE == M_BXOR) return a ^ b;
  if (MODE == M_FMAX || MODE == M_FMIN)
    return bits_of<T>(pickf<T, MODE == M_FMAX>(from_bits<T>(a), from_bits<T>(b)));
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

// (n, K, S1) of pivot-shifted sums -> mean
__device__ __forceinline__ double mean_from_sums(double n, double K, double s1) {
  return n > 0.0 ? K + s1 / n : 0.0;
}

// Batch moments of B values around the pivot K = x[0] (one of the values, so
// S2 <= (1 + B) M2_b and the subtraction loses at most log2(B+1) bits),
// returned in the frame shifted by the row's pivot P: mb = mean_b - P.
// K - P is exact for values within a factor of two of P (offset data) and
// otherwise rounds once, at the data's own scale.
template <int B>
__device__ __forceinline__ void batch_moments(const double (&x)[B], double P, double &mb, double &qb) {
  const double K = x[0];
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int i = 1; i < B; ++i) {
    const double d = x[i] - K;
    s1 += d;
    s2 = fma(d, d, s2);
  }
  constexpr double inv = 1.0 / (double)B;  // B is a power of two: exact
  mb = fma(s1, inv, K - P);
  const double q = fma(-s1, s1 * inv, s2);
  qb = q > 0.0 ? q : 0.0;
}

// Chan merge of a batch (nb values, mean mb, M2 qb) into (mean, m2) holding
// na values, with f = nb / (na + nb) and nf = na * f precomputed by the caller
// (shared by the VEC columns of a lane).  na == 0 gives f = 1, nf = 0: the
// batch is taken as is.
__device__ __forceinline__ void merge_batch(double &mean, double &m2, double mb, double qb, double f,
                                            double nf) {
  const double delta = mb - mean;
  mean = fma(delta, f, mean);
  m2 = m2 + qb + delta * delta * nf;
}

__device__ __forceinline__ void batch_weights(double na, double nb, double &f, double &nf) {
  if (na == nb) {
    f = 0.5;  // equal halves (the butterfly and phase trees): no division
  } else {
    f = nb / (na + nb);
  }
  nf = na * f;
}

// 1/k for the k-th equal batch of a lane's main loop: f = B / ((k+1) B) =
// 1/(k+1), the same correctly rounded value the division gives, from a table.
constexpr int kInvN = 512;
struct InvTab {
  double v[kInvN];
  constexpr InvTab() : v() {
    for (int i = 1; i < kInvN; ++i) v[i] = 1.0 / (double)i;
  }
};
__device__ constexpr InvTab kInvTab{};

__device__ __forceinline__ void uniform_weights(int64_t kb, double B, double &f, double &nf) {
  f = kb + 1 < kInvN ? kInvTab.v[kb + 1] : 1.0 / (double)(kb + 1);
  nf = ((double)kb * B) * f;
}

// Running Welford state of one output (rows kernel), in the frame shifted by
// the row's pivot P.
struct Wel {
  double n, mean, m2;
  int64_t kb;  // equal main-loop batches merged so far
  __device__ void init() { n = 0.0; mean = 0.0; m2 = 0.0; kb = 0; }
  template <int B> __device__ void add_main(const double (&x)[B], double P) {
    double mb, qb, f, nf;
    batch_moments<B>(x, P, mb, qb);
    uniform_weights(kb, (double)B, f, nf);
    merge_batch(mean, m2, mb, qb, f, nf);
    ++kb;
    n += (double)B;
  }
  template <int B> __device__ void add_batch(const double (&x)[B], double P) {
    double mb, qb, f, nf;
    batch_moments<B>(x, P, mb, qb);
    batch_weights(n, (double)B, f, nf);
    merge_batch(mean, m2, mb, qb, f, nf);
    n += (double)B;
  }
  __device__ void add1(double y) {  // Welford's own update (statcounter.py:51-59), y = x - P
    n += 1.0;
    const double delta = y - mean;
    mean += delta / n;
    m2 = fma(delta, y - mean, m2);
  }
};

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
  double f;
  if (na == nb) {
    f = 0.5;
  } else {
    f = nb / n;
  }
  ma = fma(delta, f, ma);
  if (need_m2) qa = qa + qb + delta * delta * (na * f);
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
  double *p2;       // var / std chunk partials: the row's pivot P per output
  int shifted;      // var / std: p0 holds mean - P (chunk partials in the workspace)
};

// var / std output of one (output, chunk): the Welford state is kept around
// the pivot P (an element of the output's first row), mean_y = mean - P.
// Final: var / std (M2 only); state: mean, M2 -- shifted for the workspace
// partials (chunk 0 records P), absolute for bm_reduce_state.
__device__ __forceinline__ void emit_mom(const Sink &sk, int64_t idx, int64_t e, int64_t c, double n,
                                         double mean_y, double m2, double P) {
  m2 = m2 > 0.0 ? m2 : 0.0;
  if (sk.final_out) {
    store_out(sk.out, idx, finish(sk.stat, 0.0, m2, n), sk.out_dtype);
    return;
  }
  sk.p0[idx] = sk.shifted ? mean_y : P + mean_y;
  sk.p1[idx] = m2;
  if (sk.shifted && c == 0) sk.p2[e] = P;
}

template <int MODE>
__device__ __forceinline__ void emit(const Sink &sk, int64_t e, double n, double mean, double m2,
                                     uint64_t u) {
  if (bit_mode<MODE>()) {
    if (sk.final_out) store_int(sk.out, e, u, sk.out_dtype);
    else ((uint64_t *)sk.p0)[e] = u;
  } else if (facc_mode<MODE>()) {
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
// blockIdx.x, with the blocks the hardware deals to one XCD (every 8th)
// remapped to consecutive indices (a bijection of the grid):
// each XCD then reads one contiguous range of every row
// (the rows kernel's rotated start, rows_block, does not help the columns:
// -0.1...-0.6% on the 64 GiB target / C4 / C2 column statistics,
// profiles/r05zf_ab_colskew.log)
__device__ __forceinline__ uint64_t xcd_block() {
  uint64_t bid = blockIdx.x;
  const uint64_t g8 = gridDim.x / 8 * 8;
  if (bid < g8) bid = (bid % 8) * (g8 / 8) + bid / 8;
  return bid;
}

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
  // row-phase merge buffers, dynamic: sized only when the block has more
  // than one row phase (cols_lds_bytes), so the wide-output case (C4's var,
  // one phase) keeps the occupancy of an LDS-free kernel
  extern __shared__ double smem[];
  double *sm0 = smem;
  double *sm1 = smem + kThreads * VEC;
  double *smn = smem + 2 * kThreads * VEC;
  const uint64_t ot = (uint64_t)d.tile0 + xcd_block();
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

  Acc<M_MEAN> acc[VEC];
  double fs[VEC];
  uint64_t us[VEC];
  // var / std: the lane's Welford state per column; the VEC columns share n
  double wm[VEC], wq[VEC];
  double wn = 0.0;
  int64_t wkb = 0;  // equal main-loop batches merged
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    acc[k].init(); fs[k] = fident<MODE>(); us[k] = bident<T, MODE>(); wm[k] = 0.0; wq[k] = 0.0;
  }

  double P[VEC];  // var / std: pivot per column, the column's element in row 0
#pragma unroll
  for (int k = 0; k < VEC; ++k) P[k] = 0.0;
  if (active) {
    const T *base = src + ((int64_t)o * d.R) * d.I + col0;
    int64_t r = r_lo + ph;
    if (MODE == M_MOM) {
      T p0v[VEC];
      vload<T, VEC>(base, p0v);
#pragma unroll
      for (int k = 0; k < VEC; ++k) P[k] = to_f64(p0v[k]);
    }
    if (MODE == M_MEAN) {
      // one pivot per column for every row phase of the block (the chunk's
      // first row): the phases then combine by plain sums, no divisions
      T k0[VEC];
      vload<T, VEC>(base + r_lo * d.I, k0);
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k].pivot(to_f64(k0[k]));
    }
    if constexpr (MODE == M_MEAN || MODE == M_MOM || facc_mode<MODE>()) {
      // kColsUnroll rows in flight per lane; the adds stay in row order
      for (; r + (kColsUnroll - 1) * nph < r_hi; r += kColsUnroll * nph) {
        T v[kColsUnroll][VEC];
#pragma unroll
        for (int u = 0; u < kColsUnroll; ++u) vload_nt<T, VEC>(base + (r + u * nph) * d.I, v[u]);
        if constexpr (MODE == M_MOM) {
          // one Welford batch of kColsUnroll rows per column
          double f, nf;
          uniform_weights(wkb, (double)kColsUnroll, f, nf);
#pragma unroll
          for (int k = 0; k < VEC; ++k) {
            double x[kColsUnroll];
#pragma unroll
            for (int u = 0; u < kColsUnroll; ++u) x[u] = to_f64(v[u][k]);
            double mb, qb;
            batch_moments<kColsUnroll>(x, P[k], mb, qb);
            merge_batch(wm[k], wq[k], mb, qb, f, nf);
          }
          ++wkb;
          wn += (double)kColsUnroll;
          continue;
        }
#pragma unroll
        for (int u = 0; u < kColsUnroll; ++u) {
#pragma unroll
          for (int k = 0; k < VEC; ++k) {
            if (facc_mode<MODE>()) fs[k] = fop<MODE>(fs[k], to_f64(v[u][k]));
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
      double f = 0.0, nf = 0.0;
      if (MODE == M_MOM) batch_weights(wn, 4.0, f, nf);
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        if (MODE == M_MOM) {
          const double x[4] = {to_f64(v0[k]), to_f64(v1[k]), to_f64(v2[k]), to_f64(v3[k])};
          double mb, qb;
          batch_moments<4>(x, P[k], mb, qb);
          merge_batch(wm[k], wq[k], mb, qb, f, nf);
        } else if (MODE == M_MEAN) {
          acc[k].add(to_f64(v0[k])); acc[k].add(to_f64(v1[k]));
          acc[k].add(to_f64(v2[k])); acc[k].add(to_f64(v3[k]));
        } else if (facc_mode<MODE>()) {
          fs[k] = fop<MODE>(fs[k], to_f64(v0[k])); fs[k] = fop<MODE>(fs[k], to_f64(v1[k]));
          fs[k] = fop<MODE>(fs[k], to_f64(v2[k])); fs[k] = fop<MODE>(fs[k], to_f64(v3[k]));
        } else {
          us[k] = bop<T, MODE>(us[k], bop<T, MODE>(bop<T, MODE>(belem<T, MODE>(v0[k]), belem<T, MODE>(v1[k])),
                                                   bop<T, MODE>(belem<T, MODE>(v2[k]), belem<T, MODE>(v3[k]))));
        }
      }
      if (MODE == M_MOM) wn += 4.0;
    }
    for (; r < r_hi; r += nph) {
      T v[VEC];
      vload_nt<T, VEC>(base + r * d.I, v);
      if (MODE == M_MOM) wn += 1.0;
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        if (MODE == M_MOM) {  // Welford's single-value update
          const double x = to_f64(v[k]) - P[k];
          const double delta = x - wm[k];
          wm[k] += delta / wn;
          wq[k] = fma(delta, x - wm[k], wq[k]);
        } else if (MODE == M_MEAN) acc[k].add(to_f64(v[k]));
        else if (facc_mode<MODE>()) fs[k] = fop<MODE>(fs[k], to_f64(v[k]));
        else us[k] = bop<T, MODE>(us[k], belem<T, MODE>(v[k]));
      }
    }
  }

  if constexpr (MODE == M_MOM) {
    // row phases: Chan merges in a fixed binary tree over the phases (phase
    // p absorbs p + s at stride s), through LDS
    for (int s = 1; s < nph; s <<= 1) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        sm0[threadIdx.x * VEC + k] = wm[k];
        sm1[threadIdx.x * VEC + k] = wq[k];
      }
      smn[threadIdx.x] = wn;
      __syncthreads();
      if ((ph & (2 * s - 1)) == 0 && ph + s < nph) {
        const int other = (ph + s) * d.tcv + cv;
        const double nb = smn[other];
        if (nb > 0.0) {
          double f, nf;
          batch_weights(wn, nb, f, nf);
#pragma unroll
          for (int k = 0; k < VEC; ++k)
            merge_batch(wm[k], wq[k], sm0[other * VEC + k], sm1[other * VEC + k], f, nf);
          wn += nb;
        }
      }
    }
    if (ph != 0 || !active) return;
    const double ntot = (double)(r_hi - r_lo);
    const int64_t plane = d.O * d.I;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const int64_t e = (int64_t)o * d.I + col0 + k;
      const int64_t idx = sk.final_out ? e : (c * plane + e);
      emit_mom(sk, idx, e, c, ntot, wm[k], wq[k], P[k]);
    }
    return;
  }

  // other modes: combine the row phases of each column through LDS (phase
  // order); mean carries the shared-pivot sum S1 until the end
  double m_[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    if (MODE == M_MEAN) m_[k] = acc[k].s1();
    else if (facc_mode<MODE>()) m_[k] = fs[k];
    else m_[k] = __builtin_bit_cast(double, us[k]);
  }
  if (nph > 1) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) sm0[threadIdx.x * VEC + k] = m_[k];
    __syncthreads();
    if (ph == 0) {
      for (int p = 1; p < nph; ++p) {
        const int other = p * d.tcv + cv;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const double mb = sm0[other * VEC + k];
          if (MODE == M_MEAN || facc_mode<MODE>()) {
            m_[k] = fop<MODE>(m_[k], mb);
          } else {
            m_[k] = __builtin_bit_cast(double, bop<T, MODE>(__builtin_bit_cast(uint64_t, m_[k]),
                                                            __builtin_bit_cast(uint64_t, mb)));
          }
        }
      }
    }
  }
  if (ph != 0 || !active) return;
  const double ntot = (double)(r_hi - r_lo);
  const int64_t plane = d.O * d.I;
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    if (MODE == M_MEAN) m_[k] = mean_from_sums(ntot, acc[k].K, m_[k]);
    const int64_t e = (int64_t)o * d.I + col0 + k;
    const int64_t idx = sk.final_out ? e : (c * plane + e);
    emit<MODE>(sk, idx, ntot, m_[k], 0.0, __builtin_bit_cast(uint64_t, m_[k]));
  }
}

// ------------------------------------------------------------------ rows --
// Round-robin dispatch puts block b on XCD b % 8: give XCD x the x-th
// contiguous eighth of the rows, so the 128-B lines two neighbouring rows
// share are fetched into one L2 instead of two (runs of 16 / 128 / 1024
// blocks per XCD in turn: no better, padded rows 5% worse at 16,
// profiles/r05w_xcd_runs.txt).  XCD x starts its eighth x * SKEW blocks in
// and wraps, so the eight XCDs are never a power-of-two distance apart: on
// C2's padded rows (8192-B pitch, eighths 256 MiB apart) mean / std
// -1.2% / -1.0% over 3 alternating rounds (profiles/r05zd_xcd_skew.txt)
constexpr uint64_t kRedXcdSkew = 37;
__device__ __forceinline__ uint64_t rows_block() {
  uint64_t bid = blockIdx.x;
  const uint64_t g8 = gridDim.x / 8 * 8;
  if (bid < g8) {
    const uint64_t E = g8 / 8;
    bid = (bid % 8) * E + (bid / 8 + (bid % 8) * kRedXcdSkew) % E;
  }
  return bid;
}

struct RowsDesc {
  int64_t O, R;
  int64_t P;       // elements between row starts (R, or a padded row pitch >= R)
  int64_t rchunk;
  FastDiv nchunks;
  int64_t nitems;  // O * nchunks
  int64_t item0;   // first item of this launch (launches split at the grid limit)
};

template <typename T, int VEC, int MODE>
__global__ void __launch_bounds__(kThreads)
    k_red_rows(const T *__restrict__ src, RowsDesc d, Sink sk) {
  const int lane = threadIdx.x & 63;
  const uint64_t bid = rows_block();
  const int64_t item = d.item0 + (int64_t)bid * (kThreads / 64) + (threadIdx.x >> 6);
  if (item >= d.nitems) return;  // whole wave exits; no block barrier below
  const uint64_t o = fd_div((uint64_t)item, d.nchunks);
  const int64_t c = item - (int64_t)o * (int64_t)d.nchunks.d;
  const int64_t r_lo = c * d.rchunk;
  const int64_t r_hi = min(d.R, r_lo + d.rchunk);
  const T *row = src + (int64_t)o * d.P;

  Acc<M_MEAN> acc;
  acc.init();
  Wel w;  // var / std
  w.init();
  double fs = fident<MODE>();
  uint64_t us = bident<T, MODE>();
  int64_t j = r_lo + (int64_t)lane * VEC;
  const int64_t stride = 64 * VEC;
  // mean: one pivot for the whole (row, chunk) -- its first element -- so the
  // 64 lanes combine by plain sums (no per-step division, see butterfly).
  // var / std: every value is shifted by the row's first element P (shared
  // by all chunks of the row), so the Welford means stay near zero and keep
  // their digits on offset data (1e6 + N(0,1)); batches bound outliers.
  if (MODE == M_MEAN) acc.pivot(to_f64(row[r_lo]));
  const double P = (MODE == M_MOM) ? to_f64(row[0]) : 0.0;
  // kRowsUnroll 16-B vectors in flight per lane (HBM latency cover), over
  // whole wave-wide steps only: every lane runs the same iterations, so a
  // step ends on a line boundary of a line-aligned row and no 128-B line is
  // split between a main-loop load and a tail load issued later (padded C2
  // rows: the split line was fetched from HBM twice about 60% of the time,
  // 1.018x read traffic)
  // (chunks shorter than one step keep the per-lane bound, so the Welford
  // batches still cover most of them)
  const int64_t step = kRowsUnroll * stride;
  const int64_t main_end = r_hi - r_lo >= step ? r_lo + (r_hi - r_lo) / step * step
                                               : r_hi - VEC - (kRowsUnroll - 1) * stride + 1;
  for (; j < main_end; j += step) {
    T v[kRowsUnroll][VEC];
#pragma unroll
    for (int u = 0; u < kRowsUnroll; ++u) vload_nt<T, VEC>(row + j + u * stride, v[u]);
    if constexpr (MODE == M_MOM) {
      // the kRowsUnroll * VEC values in hand form one Welford batch
      double x[kRowsUnroll * VEC];
#pragma unroll
      for (int u = 0; u < kRowsUnroll; ++u)
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[u * VEC + k] = to_f64(v[u][k]);
      w.add_main<kRowsUnroll * VEC>(x, P);
      continue;
    }
#pragma unroll
    for (int u = 0; u < kRowsUnroll; ++u) {
      if constexpr (MODE == M_MEAN && VEC % 2 == 0) {
#pragma unroll
        for (int k = 0; k < VEC; k += 2) acc.add2(to_f64(v[u][k]), to_f64(v[u][k + 1]));
        continue;
      }
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        if (MODE == M_MEAN) acc.add(to_f64(v[u][k]));
        else if (facc_mode<MODE>()) fs = fop<MODE>(fs, to_f64(v[u][k]));
        else us = bop<T, MODE>(us, belem<T, MODE>(v[u][k]));
      }
    }
  }
  // var / std: the rest of the row and the cross-lane merge run as sums
  // around one wave-wide pivot C = lane 0's Welford mean (lane 0 holds 1/64
  // of the main-loop data, so n (mean - C)^2 <= 64 M2 and S2 - S1^2/n loses
  // at most ~6 bits): plain adds, no division per lane or per butterfly step
  const double C = (MODE == M_MOM) ? lane0_of(w.mean) : 0.0;
  double t1 = 0.0, t2 = 0.0;
  for (; j < r_hi; j += stride) {
    if (j + VEC <= r_hi) {
      T v[VEC];
      vload_nt<T, VEC>(row + j, v);
      if constexpr (MODE == M_MOM) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const double y = (to_f64(v[k]) - P) - C;
          t1 += y;
          t2 = fma(y, y, t2);
        }
        continue;
      }
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        if (MODE == M_MEAN) acc.add(to_f64(v[k]));
        else if (facc_mode<MODE>()) fs = fop<MODE>(fs, to_f64(v[k]));
        else us = bop<T, MODE>(us, belem<T, MODE>(v[k]));
      }
    } else {
      for (int64_t k = j; k < r_hi; ++k) {
        if (MODE == M_MOM) {
          const double y = (to_f64(row[k]) - P) - C;
          t1 += y;
          t2 = fma(y, y, t2);
        } else if (MODE == M_MEAN) acc.add(to_f64(row[k]));
        else if (facc_mode<MODE>()) fs = fop<MODE>(fs, to_f64(row[k]));
        else us = bop<T, MODE>(us, belem<T, MODE>(row[k]));
      }
    }
  }

  // wave combination: DPP fold into lane 63 in lane order (deterministic).
  // mean: shared pivot, the S1 sums simply add; var / std: each lane's
  // Welford state as sums around C, which add.
  double m = facc_mode<MODE>() ? fs : acc.s1();
  double wq = 0.0;
  if constexpr (MODE == M_MOM) {
    const double dm = w.mean - C;
    const double s1 = w.n * dm;
    m = s1 + t1;
    wq = fma(s1, dm, w.m2) + t2;
    const auto add = [](double a, double b) { return a + b; };
    m = wave_fold(m, lane, add);
    wq = wave_fold(wq, lane, add);
  } else if constexpr (MODE == M_MEAN || facc_mode<MODE>()) {
    m = wave_fold(m, lane, [](double a, double b) { return fop<MODE>(a, b); });
  } else {
    us = wave_fold(us, lane, [](uint64_t a, uint64_t b) { return bop<T, MODE>(a, b); });
  }
  if (lane != kFoldLane) return;
  const double ntot = (double)(r_hi - r_lo);
  const int64_t e = (int64_t)o;
  const int64_t idx = sk.final_out ? e : (c * d.O + e);
  if constexpr (MODE == M_MOM) {
    // (S1, S2) around C -> mean - P and M2
    const double q = fma(-m, m / ntot, wq);
    emit_mom(sk, idx, e, c, ntot, C + m / ntot, q, P);
    return;
  }
  if (MODE == M_MEAN) m = mean_from_sums(ntot, acc.K, m);
  emit<MODE>(sk, idx, ntot, m, 0.0, us);
}

// ----------------------------------------------- exact integer var / std --
// 1- and 2-byte integer (and bool) inputs: var / std from exact integer sums.
// Each lane keeps S1 = sum x (int64) and S2 = sum x^2 (uint64; x^2 < 2^32);
// lanes, row phases and waves add exactly (any order gives the same bits),
// and M2 = (n S2 - S1^2) / n is formed in 128-bit integers and rounded once
// -- exact up to that rounding, cheaper than the float64 Welford path (no
// conversions, one multiply-add per element) and deterministic by
// construction.  (statcounter.py:51-59 computes the same M2 in float64.)
template <typename T> constexpr bool small_int() {
  return std::is_integral<T>::value && sizeof(T) <= 2;
}

// x^2 of a value of a 1- or 2-byte type, in 32-bit unsigned arithmetic (< 2^32)
__device__ __forceinline__ uint64_t sq32(int32_t x) {
  const uint32_t a = (uint32_t)(x < 0 ? -x : x);
  return (uint64_t)(a * a);
}

// (n, S1, S2) -> (mean, M2) with the n S2 - S1^2 difference in 128 bits.  S2
// arrives as a 128-bit (hi, lo) pair: one chunk's S2 fits 64 bits (the host
// caps a chunk at 2^31 rows, x^2 < 2^32), but the sum over chunks does not
// once an output covers 2^32 values of magnitude ~2^16 (an 8 GiB uint16
// var(axis=None)).  n < 2^38 and S2 < 2^70, so n S2 < 2^108; |S1| < 2^54.
__device__ __forceinline__ void int_moments(uint64_t n, int64_t s1, uint64_t s2, uint64_t s2_hi, double &mean,
                                            double &m2) {
  mean = n ? (double)s1 / (double)n : 0.0;
  const uint64_t a1 = (uint64_t)(s1 < 0 ? -s1 : s1);
  // n * s2 and a1 * a1 as (hi, lo)
  const uint64_t p_lo = n * s2, p_hi = __umul64hi(n, s2) + n * s2_hi;
  const uint64_t q_lo = a1 * a1, q_hi = __umul64hi(a1, a1);
  const uint64_t lo = p_lo - q_lo;
  const uint64_t hi = p_hi - q_hi - (p_lo < q_lo ? 1 : 0);
  const double num = (double)hi * 18446744073709551616.0 + (double)lo;  // >= 0 (Cauchy-Schwarz)
  m2 = n ? num / (double)n : 0.0;
}

// 128-bit running S2: (hi, lo) += v
__device__ __forceinline__ void add128(uint64_t &lo, uint64_t &hi, uint64_t v_lo, uint64_t v_hi) {
  const uint64_t t = lo + v_lo;
  hi += v_hi + (t < lo ? 1 : 0);
  lo = t;
}

// chunk partials (workspace) stay exact integer sums, merged by the combine
// kernel's integer branch; final outputs and rank states get (mean, M2)
__device__ __forceinline__ void emit_int_mom(const Sink &sk, int64_t idx, int64_t e, int64_t c, int64_t n,
                                             int64_t s1, uint64_t s2) {
  if (!sk.final_out && sk.shifted) {
    reinterpret_cast<int64_t *>(sk.p0)[idx] = s1;
    reinterpret_cast<uint64_t *>(sk.p1)[idx] = s2;
    return;
  }
  double mean, m2;
  int_moments((uint64_t)n, s1, s2, 0, mean, m2);
  emit_mom(sk, idx, e, c, (double)n, mean, m2, 0.0);
}

template <typename T, int VEC>
__global__ void __launch_bounds__(kThreads)
    k_red_cols_int(const T *__restrict__ src, ColsDesc d, Sink sk) {
  extern __shared__ double smem[];
  uint64_t *l1 = reinterpret_cast<uint64_t *>(smem);
  uint64_t *l2 = l1 + kThreads * VEC;
  const uint64_t ot = (uint64_t)d.tile0 + xcd_block();
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
  int64_t s1[VEC];
  uint64_t s2[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) { s1[k] = 0; s2[k] = 0; }
  if (active) {
    const T *base = src + ((int64_t)o * d.R) * d.I + col0;
    int64_t r = r_lo + ph;
    constexpr int U = kIntUnroll;  // rows in flight per lane
    for (; r + (U - 1) * nph < r_hi; r += U * nph) {
      T v[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) vload_nt<T, VEC>(base + (r + u * nph) * d.I, v[u]);
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        int32_t t1 = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int32_t x = (int32_t)v[u][k];
          t1 += x;
          s2[k] += sq32(x);
        }
        s1[k] += t1;
      }
    }
    for (; r < r_hi; r += nph) {
      T v[VEC];
      vload_nt<T, VEC>(base + r * d.I, v);
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const int32_t x = (int32_t)v[k];
        s1[k] += x;
        s2[k] += sq32(x);
      }
    }
  }
  if (nph > 1) {  // row phases: exact integer sums
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      l1[threadIdx.x * VEC + k] = (uint64_t)s1[k];
      l2[threadIdx.x * VEC + k] = s2[k];
    }
    __syncthreads();
    if (ph == 0) {
      for (int p = 1; p < nph; ++p) {
        const int other = p * d.tcv + cv;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          s1[k] += (int64_t)l1[other * VEC + k];
          s2[k] += l2[other * VEC + k];
        }
      }
    }
  }
  if (ph != 0 || !active) return;
  const int64_t n = r_hi - r_lo;
  const int64_t plane = d.O * d.I;
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    const int64_t e = (int64_t)o * d.I + col0 + k;
    const int64_t idx = sk.final_out ? e : (c * plane + e);
    emit_int_mom(sk, idx, e, c, n, s1[k], s2[k]);
  }
}

template <typename T, int VEC>
__global__ void __launch_bounds__(kThreads)
    k_red_rows_int(const T *__restrict__ src, RowsDesc d, Sink sk) {
  const int lane = threadIdx.x & 63;
  const uint64_t bid = rows_block();
  const int64_t item = d.item0 + (int64_t)bid * (kThreads / 64) + (threadIdx.x >> 6);
  if (item >= d.nitems) return;  // whole wave exits
  const uint64_t o = fd_div((uint64_t)item, d.nchunks);
  const int64_t c = item - (int64_t)o * (int64_t)d.nchunks.d;
  const int64_t r_lo = c * d.rchunk;
  const int64_t r_hi = min(d.R, r_lo + d.rchunk);
  const T *row = src + (int64_t)o * d.P;
  int64_t s1 = 0;
  uint64_t s2 = 0;
  const int64_t stride = 64 * VEC;
  for (int64_t j = r_lo + (int64_t)lane * VEC; j < r_hi; j += stride) {
    if (j + VEC <= r_hi) {
      T v[VEC];
      vload_nt<T, VEC>(row + j, v);
      int32_t t1 = 0;
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const int32_t x = (int32_t)v[k];
        t1 += x;
        s2 += sq32(x);
      }
      s1 += t1;
    } else {
      for (int64_t k = j; k < r_hi; ++k) {
        const int32_t x = (int32_t)row[k];
        s1 += x;
        s2 += sq32(x);
      }
    }
  }
  // exact integer sums: any order gives the same bits
  s1 = wave_fold(s1, lane, [](int64_t a, int64_t b) { return a + b; });
  s2 = wave_fold(s2, lane, [](uint64_t a, uint64_t b) { return a + b; });
  if (lane != kFoldLane) return;
  const int64_t n = r_hi - r_lo;
  const int64_t e = (int64_t)o;
  const int64_t idx = sk.final_out ? e : (c * d.O + e);
  emit_int_mom(sk, idx, e, c, n, s1, s2);
}

// --------------------------------------------------------------- combine --
constexpr int kMaxParts = 256;  // parts per bm_reduce_combine (ranks of a merge); kernarg-resident counts
struct CombDesc {
  int64_t nout;
  int64_t nparts;
  int64_t part_stride;  // elements between parts in a plane
  int64_t R, rchunk;    // uniform chunk counts when explicit == 0
  int32_t explicit_counts;
  int32_t pivots;       // var / std chunk partials: p0 is mean - P, P in the plane after M2
  int32_t int_sums;     // var / std of 1-2 byte integers: partials are exact (S1, S2) sums
  int32_t pad_;
  int64_t counts[kMaxParts];
};

template <int MODE, typename T>
__global__ void __launch_bounds__(kThreads)
    k_red_combine(const double *__restrict__ p0, const double *__restrict__ p1, CombDesc d, Sink sk) {
  const int64_t step = (int64_t)gridDim.x * kThreads;
  for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < d.nout; e += step) {
    double n = 0.0, m = 0.0, q = 0.0;
    uint64_t u = 0;
    bool first = true;
    if constexpr (MODE == M_MOM) {
      if (d.int_sums) {  // exact: add the chunks' integer sums
        int64_t s1 = 0, cnt = 0;
        uint64_t s2 = 0, s2_hi = 0;
        for (int64_t p = 0; p < d.nparts; ++p) {
          const int64_t nb = min(d.R, (p + 1) * d.rchunk) - p * d.rchunk;
          if (nb <= 0) continue;
          const int64_t at = p * d.part_stride + e;
          s1 += reinterpret_cast<const int64_t *>(p0)[at];
          add128(s2, s2_hi, reinterpret_cast<const uint64_t *>(p1)[at], 0);
          cnt += nb;
        }
        double mean, m2;
        int_moments((uint64_t)cnt, s1, s2, s2_hi, mean, m2);
        emit_mom(sk, e, e, 1, (double)cnt, mean, m2, 0.0);
        continue;
      }
    }
    for (int64_t p = 0; p < d.nparts; ++p) {
      const double nb = d.explicit_counts
                            ? (double)d.counts[p]
                            : (double)(min(d.R, (p + 1) * d.rchunk) - p * d.rchunk);
      if (nb <= 0.0) continue;
      const int64_t at = p * d.part_stride + e;
      if (MODE == M_MEAN || MODE == M_MOM) {
        // chunk partials of var / std are all around the same pivot P
        chan(n, m, q, nb, p0[at], (MODE == M_MOM) ? p1[at] : 0.0, MODE == M_MOM);
      } else if (facc_mode<MODE>()) {
        m = first ? p0[at] : fop<MODE>(m, p0[at]);
        n += nb;
      } else {
        const uint64_t b = ((const uint64_t *)p0)[at];
        u = first ? b : bop<T, MODE>(u, b);
      }
      first = false;
    }
    if constexpr (MODE == M_MOM) {
      const double P = d.pivots ? p1[d.nparts * d.part_stride + e] : 0.0;
      emit_mom(sk, e, e, 1, n, m, q, P);
    } else {
      emit<MODE>(sk, e, n, m, q, u);
    }
  }
}

// Few outputs, many parts (axis=None statistics: one output from hundreds of
// chunk states): one block per output.  Thread t merges the contiguous run of
// parts [t*L, (t+1)*L) in order, then the 256 partial states merge in a fixed
// binary tree through LDS (thread j absorbs j + s): deterministic, and a
// serial chain of hundreds of dependent loads and divisions becomes ~L + 8.
struct PartState {
  double n, m, q;
  uint64_t u;
  int64_t s1, cnt;
  uint64_t s2, s2_hi;  // 128-bit sum of the chunks' S2
  int any;
};

template <int MODE, typename T>
__device__ __forceinline__ void merge_state(PartState &a, const PartState &b, bool int_sums) {
  if (!b.any) return;
  if (!a.any) {
    a = b;
    return;
  }
  if (MODE == M_MOM && int_sums) {
    a.s1 += b.s1; a.cnt += b.cnt;
    add128(a.s2, a.s2_hi, b.s2, b.s2_hi);
  } else if (MODE == M_MEAN || MODE == M_MOM) {
    chan(a.n, a.m, a.q, b.n, b.m, b.q, MODE == M_MOM);
  } else if (facc_mode<MODE>()) {
    a.m = fop<MODE>(a.m, b.m);
    a.n += b.n;
  } else {
    a.u = bop<T, MODE>(a.u, b.u);
  }
}

template <int MODE, typename T>
__global__ void __launch_bounds__(kThreads)
    k_red_combine_blk(const double *__restrict__ p0, const double *__restrict__ p1, CombDesc d, Sink sk) {
  __shared__ PartState sm[kThreads];
  const int64_t e = blockIdx.x;
  const bool int_sums = MODE == M_MOM && d.int_sums;
  const int64_t L = (d.nparts + kThreads - 1) / kThreads;
  const int64_t p_lo = (int64_t)threadIdx.x * L, p_hi = min(d.nparts, p_lo + L);
  PartState st{};
  for (int64_t p = p_lo; p < p_hi; ++p) {
    const int64_t cnt = d.explicit_counts ? d.counts[p] : min(d.R, (p + 1) * d.rchunk) - p * d.rchunk;
    if (cnt <= 0) continue;
    const int64_t at = p * d.part_stride + e;
    PartState b{};
    b.any = 1;
    b.n = (double)cnt;
    if (int_sums) {
      b.s1 = reinterpret_cast<const int64_t *>(p0)[at];
      b.s2 = reinterpret_cast<const uint64_t *>(p1)[at];
      b.cnt = cnt;
    } else if (MODE == M_MEAN || MODE == M_MOM) {
      b.m = p0[at];
      b.q = (MODE == M_MOM) ? p1[at] : 0.0;
    } else if (facc_mode<MODE>()) {
      b.m = p0[at];
    } else {
      b.u = ((const uint64_t *)p0)[at];
    }
    merge_state<MODE, T>(st, b, int_sums);
  }
  sm[threadIdx.x] = st;
  for (int s = 1; s < kThreads; s <<= 1) {
    __syncthreads();
    if ((threadIdx.x & (2 * s - 1)) == 0) {
      PartState a = sm[threadIdx.x];
      merge_state<MODE, T>(a, sm[threadIdx.x + s], int_sums);
      sm[threadIdx.x] = a;
    }
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const PartState r = sm[0];
  if constexpr (MODE == M_MOM) {
    if (int_sums) {
      double mean, m2;
      int_moments((uint64_t)r.cnt, r.s1, r.s2, r.s2_hi, mean, m2);
      emit_mom(sk, e, e, 1, (double)r.cnt, mean, m2, 0.0);
      return;
    }
    const double P = d.pivots ? p1[d.nparts * d.part_stride + e] : 0.0;
    emit_mom(sk, e, e, 1, r.n, r.m, r.q, P);
  } else {
    emit<MODE>(sk, e, r.n, r.m, r.q, r.u);
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
  if (stat == BM_STAT_PROD) return is_float(dt) ? M_FPROD : (dt == BM_BOOL ? M_LAND : M_IPROD);
  if (stat == BM_STAT_LAND) return M_LAND;
  if (stat == BM_STAT_LOR) return M_OR;
  if (stat == BM_STAT_BAND) return M_BAND;
  if (stat == BM_STAT_BOR) return M_BOR;
  if (stat == BM_STAT_BXOR) return M_BXOR;
  if (stat == BM_STAT_FMAX) return is_float(dt) ? M_FMAX : M_MAX;
  if (stat == BM_STAT_FMIN) return is_float(dt) ? M_FMIN : M_MIN;
  if (is_float(dt)) return M_FSUM;
  if (dt == BM_BOOL) return M_OR;
  return M_ISUM;
}
int planes_of(int mode) { return mode == M_MOM ? 2 : 1; }
bool bit_mode_host(int mode) {
  return mode == M_ISUM || mode == M_OR || mode == M_MAX || mode == M_MIN || mode == M_IPROD ||
         mode == M_LAND || mode == M_BAND || mode == M_BOR || mode == M_BXOR || mode == M_FMAX ||
         mode == M_FMIN;
}
// the dtype a reduction writes: logical and / or give bool (numpy's
// logical_* ufuncs; bool sum is OR, bool product AND), the other bit modes
// and float sums / products keep the input dtype, statistics are float
int out_dtype_ok(int stat, int mode, int in_dt, int out_dt) {
  if (stat == BM_STAT_LAND || stat == BM_STAT_LOR) return out_dt == BM_BOOL;
  if (bit_mode_host(mode)) return out_dt == in_dt;
  return is_float(out_dt);
}

struct RedPlan {
  bool rows;
  int vec;
  int64_t rchunk, nchunks;
  int32_t tcv, nph;
  int64_t ntc;
};

int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

RedPlan plan_reduce(int dt, int64_t O, int64_t R, int64_t I, const void *src, int64_t P) {
  RedPlan p{};
  const int es = dtype_size(dt);
  const bool al16 = src == nullptr || ((uintptr_t)src % 16) == 0;
  if (I == 1) {
    p.rows = true;
    int vec = 16 / es;
    while (vec > 1 && !(R % vec == 0 && P % vec == 0 && (src == nullptr || ((uintptr_t)src % (vec * es)) == 0)))
      vec >>= 1;
    p.vec = vec;
    const int64_t target_waves = 8192;
    int64_t nch = 1;
    if (O < target_waves) {
      nch = cdiv(target_waves, O);
      const int64_t maxch = std::max<int64_t>(1, R / (64 * vec * 4));
      nch = std::min(nch, maxch);
    }
    // one chunk's exact integer S2 (x^2 < 2^32 per value) must fit 64 bits:
    // at most 2^31 values per chunk (a no-op below 4 GiB per output row)
    nch = std::max<int64_t>(nch, cdiv(R, (int64_t)1 << 31));
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
    while (tcv < kColsTcv && tcv < ncolv) tcv <<= 1;
    // narrower column tiles (more row phases merged in LDS) before splitting
    // R into chunks that need a workspace and a combine launch: C4's uint16
    // var over axis 0 3.50 -> 3.17 ms with 64-vector tiles and no chunks
    // (profiles/r03zb_ab_tcv.log); the float C2 column statistics move +-2%
    while (tcv > kColsTcvMin && O * cdiv(ncolv, tcv) < kColsBlocks) tcv >>= 1;
    p.tcv = tcv;
    p.nph = 256 / tcv;
    p.ntc = cdiv(ncolv, tcv);
    const int64_t blocks = O * p.ntc;
    int64_t nch = 1;
    if (blocks < kColsBlocks) {
      nch = cdiv(kColsBlocks, blocks);
      const int64_t maxch = std::max<int64_t>(1, R / ((int64_t)p.nph * 8));
      nch = std::min(nch, maxch);
    }
    nch = std::min<int64_t>(nch, 65535);
    nch = std::max<int64_t>(nch, cdiv(R, (int64_t)1 << 31));  // exact integer S2 per chunk < 2^63
    p.rchunk = cdiv(R, nch);
    p.nchunks = cdiv(R, p.rchunk);
  }
  return p;
}

// exact integer var / std: the same grids as the float kernels
template <typename T>
int launch_int_mom(const RedPlan &p, const T *s, int64_t O, int64_t R, int64_t P, int64_t I, Sink sk,
                   hipStream_t st) {
  if (p.rows) {
    RowsDesc d;
    d.O = O; d.R = R; d.P = P; d.rchunk = p.rchunk;
    d.nchunks = make_fastdiv((uint64_t)p.nchunks);
    d.nitems = O * p.nchunks;
    const int64_t blocks = cdiv(d.nitems, kThreads / 64);
    for (int64_t b0 = 0; b0 < blocks; b0 += kMaxBlocks) {
      const int g = (int)std::min<int64_t>(kMaxBlocks, blocks - b0);
      d.item0 = b0 * (kThreads / 64);
      switch (p.vec) {
        case 16: if constexpr (sizeof(T) == 1) { k_red_rows_int<T, 16><<<g, kThreads, 0, st>>>(s, d, sk); } break;
        case 8: k_red_rows_int<T, 8><<<g, kThreads, 0, st>>>(s, d, sk); break;
        case 4: k_red_rows_int<T, 4><<<g, kThreads, 0, st>>>(s, d, sk); break;
        case 2: k_red_rows_int<T, 2><<<g, kThreads, 0, st>>>(s, d, sk); break;
        default: k_red_rows_int<T, 1><<<g, kThreads, 0, st>>>(s, d, sk); break;
      }
    }
    return BM_OK;
  }
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
    const size_t lds = p.nph > 1 ? 2 * (size_t)kThreads * p.vec * sizeof(uint64_t) : 0;
    switch (p.vec) {
      case 8: k_red_cols_int<T, 8><<<grid, kThreads, lds, st>>>(s, d, sk); break;
      case 4: k_red_cols_int<T, 4><<<grid, kThreads, lds, st>>>(s, d, sk); break;
      case 2: k_red_cols_int<T, 2><<<grid, kThreads, lds, st>>>(s, d, sk); break;
      default: k_red_cols_int<T, 1><<<grid, kThreads, lds, st>>>(s, d, sk); break;
    }
  }
  return BM_OK;
}

// dynamic LDS of a k_red_cols launch: the row-phase buffers when nph > 1
template <int MODE> size_t cols_lds_bytes(int nph, int vec) {
  if (nph <= 1) return 0;
  return (MODE == M_MOM ? (2 * (size_t)kThreads * vec + kThreads) : (size_t)kThreads * vec) * sizeof(double);
}

template <typename T, int MODE>
int launch_main_t(const RedPlan &p, const void *src, int64_t O, int64_t R, int64_t P, int64_t I, Sink sk,
                  hipStream_t st) {
  const T *s = (const T *)src;
  if constexpr (MODE == M_MOM && small_int<T>()) {
    return launch_int_mom<T>(p, s, O, R, P, I, sk, st);
  }
  if (p.rows) {
    RowsDesc d;
    d.O = O; d.R = R; d.P = P; d.rchunk = p.rchunk;
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
  case V: if constexpr (V * sizeof(T) <= 16) { k_red_cols<T, V, MODE><<<grid, kThreads, cols_lds_bytes<MODE>(p.nph, V), st>>>(s, d, sk); } break;
        BM_COLS_CASE(8) BM_COLS_CASE(4) BM_COLS_CASE(2)
        default: k_red_cols<T, 1, MODE><<<grid, kThreads, cols_lds_bytes<MODE>(p.nph, 1), st>>>(s, d, sk); break;
#undef BM_COLS_CASE
      }
    }
  }
  return BM_OK;
}

template <int MODE>
int launch_main_m(int dt, const RedPlan &p, const void *src, int64_t O, int64_t R, int64_t P, int64_t I,
                  Sink sk, hipStream_t st) {
  switch (dt) {
    case BM_BOOL:
    case BM_U8: return launch_main_t<uint8_t, MODE>(p, src, O, R, P, I, sk, st);
    case BM_I8: return launch_main_t<int8_t, MODE>(p, src, O, R, P, I, sk, st);
    case BM_U16: return launch_main_t<uint16_t, MODE>(p, src, O, R, P, I, sk, st);
    case BM_I16: return launch_main_t<int16_t, MODE>(p, src, O, R, P, I, sk, st);
    case BM_U32: return launch_main_t<uint32_t, MODE>(p, src, O, R, P, I, sk, st);
    case BM_I32: return launch_main_t<int32_t, MODE>(p, src, O, R, P, I, sk, st);
    case BM_U64: return launch_main_t<uint64_t, MODE>(p, src, O, R, P, I, sk, st);
    case BM_I64: return launch_main_t<int64_t, MODE>(p, src, O, R, P, I, sk, st);
    case BM_F16:
      if constexpr (!int_only_mode<MODE>()) return launch_main_t<_Float16, MODE>(p, src, O, R, P, I, sk, st);
      break;
    case BM_F32:
      if constexpr (!int_only_mode<MODE>()) return launch_main_t<float, MODE>(p, src, O, R, P, I, sk, st);
      break;
    case BM_F64:
      if constexpr (!int_only_mode<MODE>()) return launch_main_t<double, MODE>(p, src, O, R, P, I, sk, st);
      break;
    default: break;
  }
  bm_set_error("bm_reduce: unsupported dtype %d for this statistic", dt);
  return BM_E_ARG;
}

int launch_main(int mode, int dt, const RedPlan &p, const void *src, int64_t O, int64_t R,
                int64_t P, int64_t I, Sink sk, hipStream_t st) {
  switch (mode) {
    case M_MEAN: return launch_main_m<M_MEAN>(dt, p, src, O, R, P, I, sk, st);
    case M_MOM: return launch_main_m<M_MOM>(dt, p, src, O, R, P, I, sk, st);
    case M_FSUM: return launch_main_m<M_FSUM>(dt, p, src, O, R, P, I, sk, st);
    case M_ISUM: return launch_main_m<M_ISUM>(dt, p, src, O, R, P, I, sk, st);
    case M_MAX: return launch_main_m<M_MAX>(dt, p, src, O, R, P, I, sk, st);
    case M_MIN: return launch_main_m<M_MIN>(dt, p, src, O, R, P, I, sk, st);
    case M_FPROD: return launch_main_m<M_FPROD>(dt, p, src, O, R, P, I, sk, st);
    case M_IPROD: return launch_main_m<M_IPROD>(dt, p, src, O, R, P, I, sk, st);
    case M_LAND: return launch_main_m<M_LAND>(dt, p, src, O, R, P, I, sk, st);
    case M_BAND: return launch_main_m<M_BAND>(dt, p, src, O, R, P, I, sk, st);
    case M_BOR: return launch_main_m<M_BOR>(dt, p, src, O, R, P, I, sk, st);
    case M_BXOR: return launch_main_m<M_BXOR>(dt, p, src, O, R, P, I, sk, st);
    case M_FMAX: return launch_main_m<M_FMAX>(dt, p, src, O, R, P, I, sk, st);
    case M_FMIN: return launch_main_m<M_FMIN>(dt, p, src, O, R, P, I, sk, st);
    default: return launch_main_m<M_OR>(dt, p, src, O, R, P, I, sk, st);
  }
}

// block-per-output combine for few outputs from many parts
bool comb_blk(const CombDesc &cd) { return cd.nout <= 1024 && cd.nparts >= 8; }

template <int MODE, typename T>
void launch_combine_k(int g, const double *p0, const double *p1, const CombDesc &cd, Sink sk, hipStream_t st) {
  if (comb_blk(cd))
    k_red_combine_blk<MODE, T><<<(int)cd.nout, kThreads, 0, st>>>(p0, p1, cd, sk);
  else
    k_red_combine<MODE, T><<<g, kThreads, 0, st>>>(p0, p1, cd, sk);
}

template <int MODE>
void launch_combine_m(int dt, int g, const double *p0, const double *p1, const CombDesc &cd, Sink sk,
                      hipStream_t st) {
  switch (dt) {  // only max/min look at the element type
    case BM_BOOL: case BM_U8: launch_combine_k<MODE, uint8_t>(g, p0, p1, cd, sk, st); break;
    case BM_I8: launch_combine_k<MODE, int8_t>(g, p0, p1, cd, sk, st); break;
    case BM_U16: launch_combine_k<MODE, uint16_t>(g, p0, p1, cd, sk, st); break;
    case BM_I16: launch_combine_k<MODE, int16_t>(g, p0, p1, cd, sk, st); break;
    case BM_U32: launch_combine_k<MODE, uint32_t>(g, p0, p1, cd, sk, st); break;
    case BM_I32: launch_combine_k<MODE, int32_t>(g, p0, p1, cd, sk, st); break;
    case BM_U64: launch_combine_k<MODE, uint64_t>(g, p0, p1, cd, sk, st); break;
    case BM_I64: launch_combine_k<MODE, int64_t>(g, p0, p1, cd, sk, st); break;
    case BM_F16: launch_combine_k<MODE, _Float16>(g, p0, p1, cd, sk, st); break;
    case BM_F32: launch_combine_k<MODE, float>(g, p0, p1, cd, sk, st); break;
    default: launch_combine_k<MODE, double>(g, p0, p1, cd, sk, st); break;
  }
}

int launch_combine(int mode, int dt, const double *p0, const double *p1, const CombDesc &cd, Sink sk,
                   hipStream_t st) {
  int64_t g = cdiv(cd.nout, kThreads);
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  switch (mode) {
    case M_MEAN: launch_combine_k<M_MEAN, double>((int)g, p0, p1, cd, sk, st); break;
    case M_MOM: launch_combine_k<M_MOM, double>((int)g, p0, p1, cd, sk, st); break;
    case M_FSUM: launch_combine_k<M_FSUM, double>((int)g, p0, p1, cd, sk, st); break;
    case M_FPROD: launch_combine_k<M_FPROD, double>((int)g, p0, p1, cd, sk, st); break;
    case M_ISUM: launch_combine_k<M_ISUM, uint64_t>((int)g, p0, p1, cd, sk, st); break;
    case M_IPROD: launch_combine_k<M_IPROD, uint64_t>((int)g, p0, p1, cd, sk, st); break;
    case M_OR: launch_combine_k<M_OR, uint64_t>((int)g, p0, p1, cd, sk, st); break;
    case M_LAND: launch_combine_k<M_LAND, uint64_t>((int)g, p0, p1, cd, sk, st); break;
    case M_BAND: launch_combine_k<M_BAND, uint64_t>((int)g, p0, p1, cd, sk, st); break;
    case M_BOR: launch_combine_k<M_BOR, uint64_t>((int)g, p0, p1, cd, sk, st); break;
    case M_BXOR: launch_combine_k<M_BXOR, uint64_t>((int)g, p0, p1, cd, sk, st); break;
    case M_MAX: launch_combine_m<M_MAX>(dt, (int)g, p0, p1, cd, sk, st); break;
    case M_FMAX: launch_combine_m<M_FMAX>(dt, (int)g, p0, p1, cd, sk, st); break;
    case M_FMIN: launch_combine_m<M_FMIN>(dt, (int)g, p0, p1, cd, sk, st); break;
    default: launch_combine_m<M_MIN>(dt, (int)g, p0, p1, cd, sk, st); break;
  }
  return BM_OK;
}

int check_args(int stat, int dt, int64_t O, int64_t R, int64_t I, const char *who) {
  if (stat < BM_STAT_MEAN || stat > BM_STAT_FMIN || dtype_size(dt) == 0) {
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
  // var / std: + one plane of pivots
  return ((size_t)planes_of(mode) * (size_t)p.nchunks + (mode == M_MOM ? 1 : 0)) * (size_t)nout * 8;
}

// Shared body of bm_reduce / bm_reduce_state.
// P: row pitch in elements (rows reductions, I == 1); R for a dense input.
int run_reduce(int stat, const void *src, int dt, int64_t O, int64_t R, int64_t I, Sink sk,
               void *ws, size_t ws_bytes, hipStream_t st, const char *who, int64_t P) {
  const int mode = mode_of(stat, dt);
  const RedPlan p = plan_reduce(dt, O, R, I, src, P);
  const int64_t nout = O * I;
  if (p.nchunks <= 1) {
    int rc = launch_main(mode, dt, p, src, O, R, P, I, sk, st);
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
  part.p2 = w1 + (size_t)p.nchunks * nout;  // var / std pivots (ws_bytes_for reserves the plane)
  part.shifted = mode == M_MOM;
  int rc = launch_main(mode, dt, p, src, O, R, P, I, part, st);
  if (rc) return rc;
  CombDesc cd{};
  cd.nout = nout;
  cd.nparts = p.nchunks;
  cd.part_stride = nout;
  cd.R = R;
  cd.rchunk = p.rchunk;
  cd.explicit_counts = 0;
  cd.int_sums = mode == M_MOM && !is_float(dt) && dtype_size(dt) <= 2;
  cd.pivots = mode == M_MOM && !cd.int_sums;
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
  const size_t a = ws_bytes_for(mode, plan_reduce(in_dtype, O, R, I, nullptr, R), O * I);
  const size_t b = ws_bytes_for(mode, plan_reduce(in_dtype, O, R, I, (const void *)1, R), O * I);
  *bytes = a > b ? a : b;
  return BM_OK;
}

namespace {
// bm_reduce / bm_reduce_rows: validation, then run_reduce into `out`.
int reduce_to_out(int stat, const void *src, int in_dtype, int64_t O, int64_t R, int64_t I, int64_t P,
                  void *out, int out_dtype, void *workspace, size_t workspace_bytes, void *stream,
                  const char *who) {
  int rc = check_args(stat, in_dtype, O, R, I, who);
  if (rc) return rc;
  if (!src || !out) { bm_set_error("%s: null pointer", who); return BM_E_ARG; }
  const int mode = mode_of(stat, in_dtype);
  if (!out_dtype_ok(stat, mode, in_dtype, out_dtype)) {
    bm_set_error("%s: out_dtype %d does not fit stat %d on dtype %d (float for statistics and "
                 "float sums / products, bool for logical and / or, else the input dtype)",
                 who, out_dtype, stat, in_dtype);
    return BM_E_ARG;
  }
  if (is_float(in_dtype) && (mode == M_BAND || mode == M_BOR || mode == M_BXOR)) {
    bm_set_error("%s: bitwise reductions need an integer or bool dtype", who);
    return BM_E_ARG;
  }
  Sink sk{};
  sk.out = out;
  sk.out_dtype = out_dtype;
  sk.stat = stat;
  sk.final_out = 1;
  return run_reduce(stat, src, in_dtype, O, R, I, sk, workspace, workspace_bytes,
                    (hipStream_t)stream, who, P);
}
}  // namespace

extern "C" int bm_reduce(int stat, const void *src, int in_dtype, int64_t O, int64_t R, int64_t I,
                         void *out, int out_dtype, void *workspace, size_t workspace_bytes,
                         void *stream) {
  return reduce_to_out(stat, src, in_dtype, O, R, I, R, out, out_dtype, workspace, workspace_bytes,
                       stream, "bm_reduce");
}

extern "C" int bm_reduce_rows(int stat, const void *src, int in_dtype, int64_t O, int64_t R,
                              int64_t row_pitch, void *out, int out_dtype, void *workspace,
                              size_t workspace_bytes, void *stream) {
  if (row_pitch < R) {
    bm_set_error("bm_reduce_rows: row_pitch %lld < row length %lld", (long long)row_pitch, (long long)R);
    return BM_E_ARG;
  }
  return reduce_to_out(stat, src, in_dtype, O, R, 1, row_pitch, out, out_dtype, workspace, workspace_bytes,
                       stream, "bm_reduce_rows");
}

extern "C" int bm_reduce_state_bytes(int stat, int in_dtype, int64_t nout, size_t *bytes) {
  if (!bytes || nout < 0 || stat < BM_STAT_MEAN || stat > BM_STAT_FMIN || dtype_size(in_dtype) == 0) {
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
                    (hipStream_t)stream, "bm_reduce_state", R);
}

extern "C" int bm_reduce_combine(int stat, int in_dtype, const void *states, const int64_t *counts,
                                 int nparts, int64_t nout, void *out, int out_dtype, void *stream) {
  if (stat < BM_STAT_MEAN || stat > BM_STAT_FMIN || dtype_size(in_dtype) == 0 || nparts < 1 ||
      nparts > kMaxParts || nout < 1 || !states || !counts || !out) {
    bm_set_error("bm_reduce_combine: bad arguments");
    return BM_E_ARG;
  }
  const int mode = mode_of(stat, in_dtype);
  if (!out_dtype_ok(stat, mode, in_dtype, out_dtype)) {
    bm_set_error("bm_reduce_combine: out_dtype %d does not fit stat %d on dtype %d (float for statistics and "
                 "float sums / products, bool for logical and / or, else the input dtype)",
                 out_dtype, stat, in_dtype);
    return BM_E_ARG;
  }
  if (is_float(in_dtype) && (mode == M_BAND || mode == M_BOR || mode == M_BXOR)) {
    bm_set_error("bm_reduce_combine: bitwise reductions need an integer or bool dtype");
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

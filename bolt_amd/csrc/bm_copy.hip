// bm_copy.hip -- the data-movement kernels of libbolt_mi355x (gfx950).
//
// One primitive, bm_copy_strided, serves every record-moving call site of
// bolt's Spark path (see include/bolt_mi355x.h).  The host side reduces an
// arbitrary N-d strided copy to a canonical form (unit dims dropped, dims
// ordered by destination stride, mergeable neighbours fused) and picks:
//
//   rowcopy    innermost dim contiguous on both sides (a permutation that
//              keeps the last axis, chunk pack/unpack of row bands): one 16-B
//              vector per lane, a block per 256 vectors.
//   runs       a kept inner run of 32-64 B with the two axes around it
//              swapped: a tile transpose of 16-B-unit "super elements".
//   transpose  the destination-contiguous dim differs from the source-
//              contiguous one (swap / .T on the innermost axis): TA x TB
//              tiles staged through LDS (row pad of one element breaks the
//              power-of-two bank stride), 16-B global loads along the source
//              axis and 16-B stores along the destination axis; the tile
//              shape is picked per element size and extents (pick_tile);
//              1- and 2-byte elements pack 4 / 2 rows per 32-bit LDS word.
//   generic    anything else (no unit stride): one element per lane.
//
// All are HBM-bound; algorithmic bytes = 2 * N * elem_bytes.
#include "bm_common.h"
#include "../../include/bolt_mi355x.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace {

constexpr int kThreads = 256;
// Shipped parameters (the A/B runs that chose them are in docs/HISTORY.md;
// the rejected variants live in git history and tools/microbench/).
// rowcopy: one 16-B vector per lane, a block per 256 vectors, up to the 2^32
// thread launch limit (profiles/r01_ab3..ab5: many blocks +15-25% on C3/C4 swaps)
constexpr int kRcThreads = 256;
constexpr int kUnroll = 1;
constexpr uint64_t kRcGridCap = 16777208;
// rowcopy diagonal tiles (Diag16 below) when the fastest row dim steps the
// source by >= kDiagMinStep bytes (C3 +8-9%, 64 GiB target +13-15%,
// profiles/r02_ab_diag.log) and rows are at most kDiagMaxRow bytes: round 3
// extended them from 256-B to 4-KiB rows (C4 swap, 2-KiB rows, +8.5-9.4%;
// 4-KiB rows +10-11%; 16-KiB rows lose 2-9%, a 16x16 tile then spans 4 MiB
// per side; profiles/r03k_ab_diag_c4.log, r03l_ab_diag_rows.log)
constexpr int64_t kDiagMinStep = 65536;
constexpr int64_t kDiagMaxRow = 4096;
// packed-word tiles for 1-/2-byte transposes (profiles/r01_ab_pk2.log: u16
// 128x256 +9%, u8 +11% over element-wise LDS tiles; 128x512 with 1024 threads,
// 128 KiB of LDS, +6-8% more, r01_ab_pk3.log).  uint8 runs software-pipelined
// (k_transpose_pkp, one block per CU): +9.8% on .T; uint16 gains 1-2% on .T
// but loses 3% on a 2-D transpose, so it stays unpipelined (r02_ab_pkpipe.log)
constexpr int kPkTA = 128, kPkTB = 512, kPkThreads = 1024;
// generic copies: grid-stride (uncapped measured -20% on reversed slices, r01_index2)
constexpr int kGenGridCap = 4096;
// fused transposes (a short source-contiguous axis fused with its
// continuation, C3's .T): the a-tiles of consecutive tiles are spread S ways
// over the fused source rows (ta -> (ta % S) * (ntA / S) + ta / S) when
// ntA >= 2 S: C3 .T +0.7..+2.0% at full size, +4.2..+5.5% at 1024 rows on six
// placements (profiles/r03q_ab_asp_c3full.log); the unfused C2 swap loses
// 12-23% with any S (its tiles in flight share DRAM pages of one window)
constexpr int kASpread = 32;
// runs transpose for kept inner runs of 32..kRunsMaxBytes bytes
// (profiles/r01_ab5: +35% at 32-B runs, +4% at 64 B, even at 128 B)
constexpr int64_t kRunsMaxBytes = 64;
// HIP launch limit: grid * block threads < 2^32
constexpr uint64_t kMaxGrid = 0xffffffffull / 1024;

// ---------------------------------------------------------------- rowcopy --
// 16x16 diagonal tiles over the two fastest row dims (c fastest, g next, in
// destination order): the 16 rows of a diagonal have distinct g AND distinct c,
// so neither side of a block's rows shares the low address bits of a large
// power-of-two stride, while a 16x16 tile keeps both sides' pages local
// (tools/skew/rowcopy_skew.hip "diag16").  A bijection inside each tile.
struct Diag16 {
  int on;
  int lg;        // log2 of the (square) tile side (3: 8, 4: 16)
  FastDiv grp;   // Ng * Nc rows per (outer) group
  FastDiv ntc;   // Nc / D tiles along c
  uint64_t nc;   // Nc
};

__device__ __forceinline__ uint64_t diag16_row(uint64_t row, const Diag16 &t) {
  const uint64_t outer = fd_div(row, t.grp);
  const uint64_t q = row - outer * t.grp.d;
  const int L = t.lg;
  const uint64_t D = 1ull << L;
  const uint64_t tile = q >> (2 * L), w = q & (D * D - 1);
  // c-tiles vary fastest between consecutive tiles (g-fastest measured
  // -6..-11% on the C3 / 64 GiB target swaps, profiles/r03b_ab_diag.log)
  const uint64_t gt = fd_div(tile, t.ntc);
  const uint64_t ct = tile - gt * t.ntc.d;
  // diagonal j, position k along g: a bijection of the D x D tile
  const uint64_t j = w >> L, k = w & (D - 1);
  const uint64_t g = gt * D + k, c = ct * D + ((k + j) & (D - 1));
  return outer * t.grp.d + g * t.nc + c;
}

// One VB-byte vector per lane: vector v of row `row` (rows in destination
// order, through the diagonal tiles when dg.on).  ND: the outer dims, known
// at compile time for 1..kRcMaxND (0: a runtime loop); d's strides are in
// BYTES; vpr_lg >= 0: vectors per row is 2^vpr_lg (a shift, not a division).
constexpr int kRcMaxND = 6;
template <int VB, int ND>
__global__ void __launch_bounds__(kRcThreads)
    k_rowcopy(const char *__restrict__ src, char *__restrict__ dst, Decomp d,
              FastDiv vpr, int vpr_lg, uint64_t total, Diag16 dg) {
  typedef typename VecB<VB>::t V;
  const uint64_t step = (uint64_t)gridDim.x * kRcThreads * kUnroll;
  for (uint64_t base = (uint64_t)blockIdx.x * kRcThreads * kUnroll + threadIdx.x;
       base < total; base += step) {
    V reg[kUnroll];
    int64_t doff[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t g = base + (uint64_t)u * kRcThreads;
      doff[u] = -1;
      if (g < total) {
        const uint64_t row = vpr_lg >= 0 ? g >> vpr_lg : fd_div(g, vpr);
        const uint64_t v = g - row * vpr.d;
        int64_t so, dof;
        decomp_n<ND>(dg.on ? diag16_row(row, dg) : row, d, so, dof);
        reg[u] = __builtin_nontemporal_load(reinterpret_cast<const V *>(src + so + (int64_t)v * VB));
        doff[u] = dof + (int64_t)v * VB;
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      if (doff[u] >= 0) __builtin_nontemporal_store(reg[u], reinterpret_cast<V *>(dst + doff[u]));
    }
  }
}

// -------------------------------------------------------------- transpose --
struct TransDesc {
  int64_t La;      // extent of the source-contiguous dim a
  int64_t Lb;      // extent of the destination-contiguous dim b
  int64_t sb;      // source stride of dim b (elements)
  int64_t da;      // destination stride of dim a (elements)
  FastDiv ntB;     // tiles along b
  FastDiv ntAB;    // tiles per batch element
  uint64_t ntiles; // total tiles
  Decomp batch;    // remaining dims
  // fused pairs (FUSED kernels): b = b_hi * Lb1 + b_lo is contiguous in the
  // destination but reads source rows at b_lo * sb + b_hi * sb2; a = a_hi *
  // La1 + a_lo is contiguous in the source and writes destination rows at
  // a_lo * da + a_hi * da2.  Short extents (C5's 64-wide axes) then still get
  // long tile rows.
  FastDiv Lb1, La1;
  int64_t sb2, da2;
  FastDiv asp;     // a-tile spread S (kASpread; 1 = off)
  uint64_t aspq;   // ntA / S
};

// TA x TB tile (TA along a, the source-contiguous dim; TB along b, the
// destination-contiguous dim), chosen on the host per element size and
// extents (pick_tile).  VA / VB: elements per lane for the global load
// (along a) / store (along b).  Every load of a tile is issued before the
// first LDS write, so a block keeps TB*TA*sizeof(T) bytes in flight
// (tools/microbench/transpose_tiles.hip: +6% at 64x256 f32 over writing
// each load to LDS as it lands).
template <bool FUSED>
__device__ __forceinline__ int64_t brow(const TransDesc &d, int64_t b) {
  if (!FUSED) return b * d.sb;
  const int64_t hi = (int64_t)fd_div((uint64_t)b, d.Lb1);
  return (b - hi * (int64_t)d.Lb1.d) * d.sb + hi * d.sb2;
}

template <bool FUSED>
__device__ __forceinline__ int64_t arow(const TransDesc &d, int64_t a) {
  if (!FUSED) return a * d.da;
  const int64_t hi = (int64_t)fd_div((uint64_t)a, d.La1);
  return (a - hi * (int64_t)d.La1.d) * d.da + hi * d.da2;
}

template <typename T, int TA, int TB, int VA, int VB, bool FUSED = false>
__global__ void __launch_bounds__(kThreads)
    k_transpose(const T *__restrict__ src, T *__restrict__ dst, TransDesc d) {
  __shared__ T tile[TB][TA + 1];
  constexpr int NVA = TA / VA;
  constexpr int RPA = kThreads / NVA;
  constexpr int NVB = TB / VB;
  constexpr int RPB = kThreads / NVB;
  static_assert(NVA <= kThreads && NVB <= kThreads, "tile row wider than the block");
  static_assert(RPA <= TB && RPB <= TA && TB % RPA == 0 && TA % RPB == 0, "tile too small for the thread layout");
  constexpr int NL = TB / RPA;
  constexpr int NS = TA / RPB;
  // loads in flight per lane: all of them, up to 16 registers' worth (unaligned
  // element-wise loads go in batches instead of spilling)
  constexpr int RPL = (VA * (int)sizeof(T) + 3) / 4;  // VGPRs per load
  constexpr int NLB = (NL * RPL <= 64) ? NL : (16 / RPL > 0 ? 16 / RPL : 1);
  static_assert(NL % NLB == 0, "load batch must divide the loads");
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
  const int ia = tx * VA;
  const int ib = ux * VB;

  for (uint64_t t = blockIdx.x; t < d.ntiles; t += gridDim.x) {
    // consecutive blocks walk dim b (the destination-contiguous one): their
    // stores land side by side in the same destination rows (+9% measured)
    const uint64_t bt = fd_div(t, d.ntAB);
    const uint64_t rem = t - bt * d.ntAB.d;
    uint64_t ta = fd_div(rem, d.ntB);
    uint64_t tb = rem - ta * d.ntB.d;
    if (d.asp.d > 1) {
      const uint64_t hi = fd_div(ta, d.asp);
      ta = (ta - hi * d.asp.d) * d.aspq + hi;
    }
    int64_t so, dof;
    decomp_le4(bt, d.batch, so, dof);
    const int64_t a0 = (int64_t)ta * TA, b0 = (int64_t)tb * TB;

    // load: lanes walk dim a (source-contiguous); all loads in flight first
    const T *s = src + so + a0;
    const bool fullA = (a0 + ia + VA <= d.La);
#pragma unroll
    for (int i0 = 0; i0 < NL; i0 += NLB) {
      T v[NLB][VA];
#pragma unroll
      for (int j = 0; j < NLB; ++j) {
        const int rb = ty + (i0 + j) * RPA;
        if (b0 + rb < d.Lb) {
          const T *p = s + ia + brow<FUSED>(d, b0 + rb);
          if (fullA) {
            vload_nt<T, VA>(p, v[j]);
          } else {
#pragma unroll
            for (int k = 0; k < VA; ++k) v[j][k] = (a0 + ia + k < d.La) ? p[k] : T(0);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < NLB; ++j) {
        const int rb = ty + (i0 + j) * RPA;
#pragma unroll
        for (int k = 0; k < VA; ++k) tile[rb][ia + k] = v[j][k];
      }
    }
    __syncthreads();

    // store: lanes walk dim b (destination-contiguous)
    T *q = dst + dof + b0;
    const bool fullB = (b0 + ib + VB <= d.Lb);
#pragma unroll
    for (int it = 0; it < NS; ++it) {
      const int ra = uy + it * RPB;
      if (a0 + ra < d.La) {
        T w[VB];
#pragma unroll
        for (int k = 0; k < VB; ++k) w[k] = tile[ib + k][ra];
        T *p = q + arow<FUSED>(d, a0 + ra) + ib;
        if (fullB) {
          vstore_nt<T, VB>(p, w);
        } else {
#pragma unroll
          for (int k = 0; k < VB; ++k)
            if (b0 + ib + k < d.Lb) p[k] = w[k];
        }
      }
    }
    __syncthreads();
  }
}


// ------------------------------------------------------ packed transpose --
// 1- and 2-byte elements: P = 4 / sizeof(T) consecutive source rows (along b)
// are packed into 32-bit words, one word per column a, so the LDS tile is a
// 32-bit transpose of TA x (TB / P) words -- no 8-/16-bit LDS traffic.  A
// lane loads P 16-B rows, writes VA words; the store side reads 4 words along
// b (4 * P consecutive elements = 16 B) and stores them as one vector.
// Requires 16-B aligned source and destination rows (the caller checks).
// (tile sweep: element-wise LDS tiles move u16 / u8 at 4.6 / 3.0 TB/s,
// profiles/r01_tt2.log)
template <typename T, int TA, int TB, int NT = kThreads>
__global__ void __launch_bounds__(NT)
    k_transpose_pk(const T *__restrict__ src, T *__restrict__ dst, TransDesc d) {
  constexpr int P = 4 / (int)sizeof(T);  // rows per word
  constexpr int VA = 16 / (int)sizeof(T);
  constexpr int TBW = TB / P;            // word rows in the tile
  constexpr int NVA = TA / VA;           // lanes per word row (load)
  constexpr int RGA = NT / NVA;    // word rows per pass
  constexpr int NL = TBW / RGA;
  constexpr int NVB = TBW / 4;           // lanes per destination row (4 words each)
  constexpr int RPB = NT / NVB;
  constexpr int NS = TA / RPB;
  constexpr int BITS = 8 * (int)sizeof(T);
  static_assert(NL >= 1 && TBW % RGA == 0 && NS >= 1 && TA % RPB == 0, "tile too small for the thread layout");
  static_assert(NL * P * 4 <= 64, "loads in flight exceed the register budget");
  __shared__ uint32_t tile[TBW][TA + 1];
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
  const int ia = tx * VA;

  for (uint64_t t = blockIdx.x; t < d.ntiles; t += gridDim.x) {
    const uint64_t bt = fd_div(t, d.ntAB);
    const uint64_t rem = t - bt * d.ntAB.d;
    const uint64_t ta = fd_div(rem, d.ntB);
    uint64_t tb = rem - ta * d.ntB.d;
    int64_t so, dof;
    decomp_le4(bt, d.batch, so, dof);
    const int64_t a0 = (int64_t)ta * TA, b0 = (int64_t)tb * TB;

    const T *s = src + so + a0 + b0 * d.sb;
    const bool fullA = (a0 + ia + VA <= d.La);
    T v[NL][P][VA];
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int wr = ty + it * RGA;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int rb = wr * P + j;
        const T *p = s + ia + (int64_t)rb * d.sb;
        if (b0 + rb < d.Lb && fullA) {
          vload_nt<T, VA>(p, v[it][j]);
        } else {
#pragma unroll
          for (int k = 0; k < VA; ++k) v[it][j][k] = (b0 + rb < d.Lb && a0 + ia + k < d.La) ? p[k] : T(0);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int wr = ty + it * RGA;
#pragma unroll
      for (int k = 0; k < VA; ++k) {
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < P; ++j) w |= (uint32_t)v[it][j][k] << (j * BITS);
        tile[wr][ia + k] = w;
      }
    }
    __syncthreads();

    T *q = dst + dof + b0 + a0 * d.da;
    const int ib = ux * 4 * P;  // first element of this lane's 16 B along b
    const bool fullB = (b0 + ib + 4 * P <= d.Lb);
#pragma unroll
    for (int it = 0; it < NS; ++it) {
      const int ra = uy + it * RPB;
      if (a0 + ra < d.La) {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = tile[ux * 4 + k][ra];
        T *p = q + (int64_t)ra * d.da + ib;
        if (fullB) {
          typedef typename VecB<16>::t V16;
          V16 x;
          __builtin_memcpy(&x, w, 16);
          __builtin_nontemporal_store(x, reinterpret_cast<V16 *>(p));
        } else {
#pragma unroll
          for (int e = 0; e < 4 * P; ++e)
            if (b0 + ib + e < d.Lb) p[e] = (T)(w[e / P] >> ((e % P) * BITS));
        }
      }
    }
    __syncthreads();
  }
}

// Software-pipelined packed transpose: a block walks tiles t, t + grid, ... and
// issues the global loads of its next tile before the LDS reads and global
// stores of the current one, so HBM reads stay in flight through the store
// phase (the 128-KiB u16 tile leaves room for one block per CU, whose load and
// store phases would otherwise alternate).  Same tile layout as k_transpose_pk.
template <typename T, int TA, int TB, int NT = kThreads>
__global__ void __launch_bounds__(NT)
    k_transpose_pkp(const T *__restrict__ src, T *__restrict__ dst, TransDesc d) {
  constexpr int P = 4 / (int)sizeof(T);
  constexpr int VA = 16 / (int)sizeof(T);
  constexpr int TBW = TB / P;
  constexpr int NVA = TA / VA;
  constexpr int RGA = NT / NVA;
  constexpr int NL = TBW / RGA;
  constexpr int NVB = TBW / 4;
  constexpr int RPB = NT / NVB;
  constexpr int NS = TA / RPB;
  constexpr int BITS = 8 * (int)sizeof(T);
  static_assert(NL >= 1 && TBW % RGA == 0 && NS >= 1 && TA % RPB == 0, "tile too small for the thread layout");
  static_assert(NL * P * 4 <= 64, "loads in flight exceed the register budget");
  __shared__ uint32_t tile[TBW][TA + 1];
  const int tx = threadIdx.x % NVA, ty = threadIdx.x / NVA;
  const int ux = threadIdx.x % NVB, uy = threadIdx.x / NVB;
  const int ia = tx * VA;

  T v[NL][P][VA];
  auto coords = [&](uint64_t t, int64_t &a0, int64_t &b0, int64_t &so, int64_t &dof) {
    const uint64_t bt = fd_div(t, d.ntAB);
    const uint64_t rem = t - bt * d.ntAB.d;
    const uint64_t ta = fd_div(rem, d.ntB);
    const uint64_t tb = rem - ta * d.ntB.d;
    decomp_le4(bt, d.batch, so, dof);
    a0 = (int64_t)ta * TA;
    b0 = (int64_t)tb * TB;
  };
  auto load = [&](uint64_t t) {
    int64_t a0, b0, so, dof;
    coords(t, a0, b0, so, dof);
    const T *s = src + so + a0 + b0 * d.sb;
    const bool fullA = (a0 + ia + VA <= d.La);
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int wr = ty + it * RGA;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int rb = wr * P + j;
        const T *p = s + ia + (int64_t)rb * d.sb;
        if (b0 + rb < d.Lb && fullA) {
          vload_nt<T, VA>(p, v[it][j]);
        } else {
#pragma unroll
          for (int k = 0; k < VA; ++k) v[it][j][k] = (b0 + rb < d.Lb && a0 + ia + k < d.La) ? p[k] : T(0);
        }
      }
    }
  };

  uint64_t t = blockIdx.x;
  if (t < d.ntiles) load(t);
  for (; t < d.ntiles; t += gridDim.x) {
#pragma unroll
    for (int it = 0; it < NL; ++it) {
      const int wr = ty + it * RGA;
#pragma unroll
      for (int k = 0; k < VA; ++k) {
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < P; ++j) w |= (uint32_t)v[it][j][k] << (j * BITS);
        tile[wr][ia + k] = w;
      }
    }
    __syncthreads();
    const uint64_t tn = t + gridDim.x;
    if (tn < d.ntiles) load(tn);  // in flight during this tile's stores

    int64_t a0, b0, so, dof;
    coords(t, a0, b0, so, dof);
    T *q = dst + dof + b0 + a0 * d.da;
    const int ib = ux * 4 * P;
    const bool fullB = (b0 + ib + 4 * P <= d.Lb);
#pragma unroll
    for (int it = 0; it < NS; ++it) {
      const int ra = uy + it * RPB;
      if (a0 + ra < d.La) {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = tile[ux * 4 + k][ra];
        T *p = q + (int64_t)ra * d.da + ib;
        if (fullB) {
          typedef typename VecB<16>::t V16;
          V16 x;
          __builtin_memcpy(&x, w, 16);
          __builtin_nontemporal_store(x, reinterpret_cast<V16 *>(p));
        } else {
#pragma unroll
          for (int e = 0; e < 4 * P; ++e)
            if (b0 + ib + e < d.Lb) p[e] = (T)(w[e / P] >> ((e % P) * BITS));
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------ runs transpose --
// A permutation that keeps a short innermost run (W 16-B units, 32-256 B) but
// swaps the two axes around it (C3 / the 64 GiB target: swap((0,),(0,)) on
// (K0, K1, V0, 32) float32) is a transpose of W-unit "super elements".  Moving
// runs one by one reads 128-B pieces megabytes apart; tiling TA x TB runs
// through LDS reads TA*W units (2 KiB) contiguously per source row and writes
// TB*W units contiguously per destination row.
struct RunsDesc {
  int64_t La, Lb;    // extents of dims A (source-contiguous runs) and B (destination-contiguous runs)
  int64_t sb;        // source stride of B, in 16-B units
  int64_t da;        // destination stride of A, in 16-B units
  FastDiv ntB;       // tiles along B
  FastDiv ntAB;      // tiles per batch element
  uint64_t ntiles;
  Decomp batch;      // remaining dims (strides in 16-B units)
};

constexpr int kRunUnits = 128;  // units per tile row along A (2 KiB)
constexpr int kRunTB = 16;      // tile rows along B

template <int W>
__global__ void __launch_bounds__(kThreads)
    k_transpose_runs(const uint4 *__restrict__ src, uint4 *__restrict__ dst, RunsDesc d) {
  constexpr int TA = kRunUnits / W;
  constexpr int PAD = W < 16 ? W : 0;  // spreads 16-lane read groups over both bank halves
  constexpr int ROW = kRunUnits + PAD;
  __shared__ uint4 tile[kRunTB * ROW];
  typedef typename VecB<16>::t V;
  for (uint64_t t = blockIdx.x; t < d.ntiles; t += gridDim.x) {
    const uint64_t bt = fd_div(t, d.ntAB);
    const uint64_t rem = t - bt * d.ntAB.d;
    const uint64_t ta = fd_div(rem, d.ntB);
    uint64_t tb = rem - ta * d.ntB.d;
    int64_t so, dof;
    decomp_le4(bt, d.batch, so, dof);
    const int64_t a0 = (int64_t)ta * TA, b0 = (int64_t)tb * kRunTB;
    const int64_t na = min((int64_t)TA, d.La - a0);   // runs in this tile along A
    const int64_t nb = min((int64_t)kRunTB, d.Lb - b0);
    // load: source row b holds na*W contiguous units starting at run a0
    const uint4 *s = src + so + a0 * W + b0 * d.sb;
#pragma unroll
    for (int it = 0; it < kRunTB * kRunUnits / kThreads; ++it) {
      const int idx = it * kThreads + threadIdx.x;
      const int rb = idx / kRunUnits, u = idx % kRunUnits;
      if (rb < nb && u < na * W) {
        V v = __builtin_nontemporal_load(reinterpret_cast<const V *>(s + (int64_t)rb * d.sb + u));
        *reinterpret_cast<V *>(&tile[rb * ROW + u]) = v;
      }
    }
    __syncthreads();
    // store: destination row a holds nb*W contiguous units starting at run b0
    uint4 *q = dst + dof + b0 * W + a0 * d.da;
#pragma unroll
    for (int it = 0; it < kRunTB * kRunUnits / kThreads; ++it) {
      const int idx = it * kThreads + threadIdx.x;
      const int ra = idx / (kRunTB * W), m = idx % (kRunTB * W);
      const int b = m / W, w = m % W;
      if (ra < na && b < nb) {
        V v = *reinterpret_cast<const V *>(&tile[b * ROW + ra * W + w]);
        __builtin_nontemporal_store(v, reinterpret_cast<V *>(q + (int64_t)ra * d.da + m));
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- generic --
template <int ES>
__global__ void __launch_bounds__(kThreads)
    k_generic(const char *__restrict__ src, char *__restrict__ dst, Decomp d,
              uint64_t total) {
  typedef typename VecB<ES>::t V;
  const uint64_t step = (uint64_t)gridDim.x * kThreads;
  for (uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x; g < total; g += step) {
    int64_t so, dof;
    decomp2(g, d, so, dof);
    *reinterpret_cast<V *>(dst + dof * ES) = *reinterpret_cast<const V *>(src + so * ES);
  }
}

// ------------------------------------------------------------------- host --
struct Dim {
  int64_t n, ss, ds;
};

bool fill_decomp(Decomp &d, const std::vector<Dim> &outer_to_inner) {
  const int n = (int)outer_to_inner.size();
  if (n > BM_MAXD) return false;
  d.n = n;
  d.pad_ = 0;
  for (int k = 0; k < n; ++k) {  // store innermost first
    const Dim &x = outer_to_inner[n - 1 - k];
    d.div[k] = make_fastdiv((uint64_t)x.n);
    d.ss[k] = x.ss;
    d.ds[k] = x.ds;
  }
  for (int k = n; k < BM_MAXD; ++k) {
    d.div[k] = make_fastdiv(1);
    d.ss[k] = 0;
    d.ds[k] = 0;
  }
  return true;
}

int grid_for(uint64_t work_items, uint64_t per_block, uint64_t cap = 256ull * 16) {
  uint64_t g = (work_items + per_block - 1) / per_block;
  // default cap: 256 CUs x 16 resident-ish blocks, then grid-stride
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

bool aligned(const void *p, int64_t a) { return ((uintptr_t)p % (uintptr_t)a) == 0; }

template <int VB>
void launch_rowcopy_nd(const char *src, char *dst, const Decomp &d, FastDiv fv, int vpr_lg, uint64_t total,
                       const Diag16 &dg, int grid, hipStream_t st) {
  switch (d.n) {
    case 1: k_rowcopy<VB, 1><<<grid, kRcThreads, 0, st>>>(src, dst, d, fv, vpr_lg, total, dg); break;
    case 2: k_rowcopy<VB, 2><<<grid, kRcThreads, 0, st>>>(src, dst, d, fv, vpr_lg, total, dg); break;
    case 3: k_rowcopy<VB, 3><<<grid, kRcThreads, 0, st>>>(src, dst, d, fv, vpr_lg, total, dg); break;
    case 4: k_rowcopy<VB, 4><<<grid, kRcThreads, 0, st>>>(src, dst, d, fv, vpr_lg, total, dg); break;
    case 5: k_rowcopy<VB, 5><<<grid, kRcThreads, 0, st>>>(src, dst, d, fv, vpr_lg, total, dg); break;
    case 6: k_rowcopy<VB, 6><<<grid, kRcThreads, 0, st>>>(src, dst, d, fv, vpr_lg, total, dg); break;
    default: k_rowcopy<VB, 0><<<grid, kRcThreads, 0, st>>>(src, dst, d, fv, vpr_lg, total, dg); break;
  }
  static_assert(kRcMaxND == 6, "launch_rowcopy_nd covers 1..kRcMaxND");
}

int launch_rowcopy(const char *src, char *dst, const std::vector<Dim> &dims, int es,
                   hipStream_t st) {
  const Dim inner = dims.back();
  std::vector<Dim> outer(dims.begin(), dims.end() - 1);
  const int64_t row_bytes = inner.n * es;
  int VB = 16;
  for (; VB > 1; VB >>= 1) {
    if (row_bytes % VB) continue;
    if (!aligned(src, VB) || !aligned(dst, VB)) continue;
    bool ok = true;
    for (const Dim &x : outer)
      if ((x.ss * es) % VB || (x.ds * es) % VB) ok = false;
    if (ok) break;
  }
  Decomp d;
  {
    std::vector<Dim> bytes(outer);  // the kernel's offsets are in bytes
    for (Dim &x : bytes) { x.ss *= es; x.ds *= es; }
    if (!fill_decomp(d, bytes)) {
      bm_set_error("bm_copy_strided: too many dims after fusion (%d)", (int)outer.size());
      return BM_E_ARG;
    }
  }
  Diag16 dg{};
  {
    // 16x16 diagonal tiles when the fastest row dim steps the source by a
    // large stride and the next one by less (C3 / 64 GiB swaps: c then b)
    const int n = (int)outer.size();
    if (row_bytes <= kDiagMaxRow && n >= 2) {
      const Dim &f = outer[n - 1], &g = outer[n - 2];
      // 8x8 tiles for rows up to 1 KiB, 16x16 above (profiles/r03n_ab_diagsize.log,
      // r03o_ab_diag8_*.log: 8x8 on C3's 128-B rows +4.3-6.1% on three
      // placements, 1-KiB rows +2%, the 64 GiB target -0.4..-1.8%; on 2-4-KiB
      // rows 16x16 is equal or +1%; 32x32 loses everywhere)
      const int lg = row_bytes <= 1024 ? 3 : 4;
      const int64_t D = (int64_t)1 << lg;
      if (f.n % D == 0 && g.n % D == 0 && std::llabs(f.ss) * es >= kDiagMinStep &&
          std::llabs(g.ss) < std::llabs(f.ss)) {
        dg.on = 1;
        dg.lg = lg;
        dg.grp = make_fastdiv((uint64_t)(f.n * g.n));
        dg.ntc = make_fastdiv((uint64_t)(f.n / D));
        dg.nc = (uint64_t)f.n;
      }
    }
  }
  uint64_t rows = 1;
  for (const Dim &x : outer) rows *= (uint64_t)x.n;
  const uint64_t vpr = (uint64_t)(row_bytes / VB);
  const uint64_t total = rows * vpr;
  const FastDiv fv = make_fastdiv(vpr);
  const int vpr_lg = (vpr & (vpr - 1)) == 0 ? __builtin_ctzll(vpr) : -1;
  const uint64_t per = (uint64_t)kRcThreads * kUnroll;
  const uint64_t need = (total + per - 1) / per;
  // one vector per lane (an XCD-grouped covering grid measured +5% in a C4
  // microbench but -3..-20% in the product A/B, profiles/r01_ab_rc)
  const int grid = need <= kRcGridCap ? (int)std::max<uint64_t>(need, 1) : grid_for(total, per, kRcGridCap);
  switch (VB) {
    case 16: launch_rowcopy_nd<16>(src, dst, d, fv, vpr_lg, total, dg, grid, st); break;
    case 8: launch_rowcopy_nd<8>(src, dst, d, fv, vpr_lg, total, dg, grid, st); break;
    case 4: launch_rowcopy_nd<4>(src, dst, d, fv, vpr_lg, total, dg, grid, st); break;
    case 2: launch_rowcopy_nd<2>(src, dst, d, fv, vpr_lg, total, dg, grid, st); break;
    default: launch_rowcopy_nd<1>(src, dst, d, fv, vpr_lg, total, dg, grid, st); break;
  }
  return BM_OK;
}

template <typename T, int TA, int TB>
void launch_transpose_tile(const T *src, T *dst, const TransDesc &td, bool va_vec, bool vb_vec, int grid,
                           bool fused, hipStream_t st) {
  constexpr int W = 16 / (int)sizeof(T);
  if constexpr (sizeof(T) >= 4) {
    if (fused) {  // fused axis pairs: vectorised only (the host fuses aligned layouts)
      k_transpose<T, TA, TB, W, W, true><<<grid, kThreads, 0, st>>>(src, dst, td);
      return;
    }
  }
  if (va_vec && vb_vec)
    k_transpose<T, TA, TB, W, W><<<grid, kThreads, 0, st>>>(src, dst, td);
  else if (va_vec)
    k_transpose<T, TA, TB, W, 1><<<grid, kThreads, 0, st>>>(src, dst, td);
  else if (vb_vec)
    k_transpose<T, TA, TB, 1, W><<<grid, kThreads, 0, st>>>(src, dst, td);
  else
    k_transpose<T, TA, TB, 1, 1><<<grid, kThreads, 0, st>>>(src, dst, td);
}

// Tile shapes per element size (TA x TB elements).  Measured on the C2 swap
// shape with 1 MiB source rows (tools/microbench/transpose_tiles.hip,
// profiles/r01_tt2.log): 128-256-B source segments and ~1-2 KiB destination
// segments per tile row are fastest; the others serve short extents.
struct Tile { int ta, tb; };
constexpr Tile kTiles1[] = {{128, 256}, {128, 128}, {64, 64}, {256, 64}, {64, 256}};
constexpr Tile kTiles2[] = {{128, 256}, {64, 256}, {64, 64}, {128, 64}, {256, 32}, {32, 256}};
constexpr Tile kTiles4[] = {{64, 256}, {32, 256}, {64, 64}, {64, 128}, {128, 32}, {256, 16}, {16, 256}, {32, 64}};
// f64 with 512-B destination rows whose source rows are at most
// kT8Fuse512 bytes apart (C5 transpose(2,0,4,1,3)): fuse b with its
// continuation and use 32 x 128 tiles, 1-KiB write segments: +5% (2.798 ->
// 2.657 ms); with far-apart source rows (C5 .T) fusing loses 5-20%
// (profiles/r02_ab_f512.log)
constexpr int64_t kT8Fuse512 = 4096;
constexpr Tile kT8FusedTile = {32, 128};
constexpr Tile kTiles8[] = {{32, 256}, {16, 256}, {32, 64}, {64, 64}, {64, 32}, {128, 16}, {16, 128}};

template <typename T>
int launch_transpose_t(const T *src, T *dst, const TransDesc &td, Tile tl, bool va_vec, bool vb_vec,
                       bool fused, hipStream_t st) {
  uint64_t g = td.ntiles;
  if (g > kMaxGrid) g = kMaxGrid;  // grid-stride beyond the launch limit
  const int grid = (int)g;
#define BM_TILE(A, B) \
  if (tl.ta == A && tl.tb == B) { launch_transpose_tile<T, A, B>(src, dst, td, va_vec, vb_vec, grid, fused, st); return BM_OK; }
  if constexpr (sizeof(T) == 1) {
    BM_TILE(128, 256) BM_TILE(128, 128) BM_TILE(64, 64) BM_TILE(256, 64) BM_TILE(64, 256)
  } else if constexpr (sizeof(T) == 2) {
    BM_TILE(128, 256) BM_TILE(64, 256) BM_TILE(64, 64) BM_TILE(128, 64) BM_TILE(256, 32) BM_TILE(32, 256)
  } else if constexpr (sizeof(T) == 4) {
    BM_TILE(64, 256) BM_TILE(32, 256) BM_TILE(64, 64) BM_TILE(64, 128) BM_TILE(128, 32) BM_TILE(256, 16)
    BM_TILE(16, 256) BM_TILE(32, 64)
  } else {
    BM_TILE(32, 256) BM_TILE(16, 256) BM_TILE(32, 64) BM_TILE(64, 64) BM_TILE(64, 32) BM_TILE(128, 16)
    BM_TILE(16, 128)
    BM_TILE(kT8FusedTile.ta, kT8FusedTile.tb)
  }
#undef BM_TILE
  bm_set_error("bm_copy_strided: no transpose tile %dx%d for %d-byte elements", tl.ta, tl.tb, (int)sizeof(T));
  return BM_E_ARG;
}

// Relative cost of a tile row segment of n bytes (1.0 = the fastest shape),
// from the same sweep: short segments waste DRAM bursts.
double seg_cost_read(int64_t n) { return n >= 256 ? 1.0 : n >= 128 ? 1.02 : n >= 64 ? 1.25 : 1.6; }
double seg_cost_write(int64_t n) { return n >= 1024 ? 1.0 : n >= 512 ? 1.05 : n >= 256 ? 1.06 : n >= 128 ? 1.3 : 1.6; }

// The tile with the least estimated time for extents (La, Lb): padded tile
// traffic x segment costs.
Tile pick_tile(int64_t La, int64_t Lb, int es) {
  const Tile *c;
  int n;
  switch (es) {
    case 1: c = kTiles1; n = sizeof(kTiles1) / sizeof(Tile); break;
    case 2: c = kTiles2; n = sizeof(kTiles2) / sizeof(Tile); break;
    case 4: c = kTiles4; n = sizeof(kTiles4) / sizeof(Tile); break;
    default: c = kTiles8; n = sizeof(kTiles8) / sizeof(Tile); break;
  }
  Tile best = c[0];
  double best_w = 1e300;
  for (int i = 0; i < n; ++i) {
    const int64_t ta = c[i].ta, tb = c[i].tb;
    const double pa = (double)(((La + ta - 1) / ta) * ta), pb = (double)(((Lb + tb - 1) / tb) * tb);
    const double w = pa * pb * seg_cost_read(std::min(ta, La) * es) * seg_cost_write(std::min(tb, Lb) * es);
    if (w < best_w * 0.999) {
      best_w = w;
      best = c[i];
    }
  }
  return best;
}

int launch_transpose(const char *src, char *dst, const std::vector<Dim> &dims, int a, int es,
                     hipStream_t st, bool allow_fuse = true) {
  const int b = (int)dims.size() - 1;
  std::vector<Dim> batch;
  for (int k = 0; k < (int)dims.size(); ++k)
    if (k != a && k != b) batch.push_back(dims[k]);
  TransDesc td;
  td.La = dims[a].n;
  td.Lb = dims[b].n;
  td.sb = dims[b].ss;
  td.da = dims[a].ds;
  td.Lb1 = make_fastdiv((uint64_t)td.Lb);
  td.La1 = make_fastdiv((uint64_t)td.La);
  td.sb2 = 0;
  td.da2 = 0;
  // Short contiguous axes: fuse b with the dim that continues it in the
  // destination (ds == Lb) and a with the dim that continues it in the source
  // (ss == La), so tile rows stay >= 512 B / 256 B (C3 .T: 128-B source rows,
  // +21%, profiles/r01_ab_fuse.log).
  bool fused = false, fused512 = false;
  if (allow_fuse && es >= 4 && aligned(src, 16) && aligned(dst, 16)) {
    auto take = [&](bool want_b) -> int {
      for (int k = 0; k < (int)batch.size(); ++k)
        if (want_b ? batch[k].ds == td.Lb : batch[k].ss == td.La) return k;
      return -1;
    };
    const bool f512 = es == 8 && td.Lb * es == 512 && std::llabs(td.sb) * es <= kT8Fuse512;
    if (td.Lb * es < 512 || f512) {
      const int k = take(true);
      if (k >= 0) {
        fused512 = f512;
        td.sb2 = batch[k].ss;
        td.Lb *= batch[k].n;
        batch.erase(batch.begin() + k);
        fused = true;
      }
    }
    if (td.La * es < 256) {
      const int k = take(false);
      if (k >= 0) {
        td.da2 = batch[k].ds;
        td.La *= batch[k].n;
        batch.erase(batch.begin() + k);
        fused = true;
      }
    }
  }
  Tile tl = pick_tile(td.La, td.Lb, es);
  if (fused512) tl = kT8FusedTile;
  const int TA = tl.ta, TB = tl.tb;
  const uint64_t ntA = (uint64_t)((td.La + TA - 1) / TA);
  const uint64_t ntB = (uint64_t)((td.Lb + TB - 1) / TB);
  uint64_t nb = 1;
  for (const Dim &x : batch) nb *= (uint64_t)x.n;
  if (!fill_decomp(td.batch, batch)) {
    bm_set_error("bm_copy_strided: too many dims after fusion (%d)", (int)batch.size());
    return BM_E_ARG;
  }
  td.ntB = make_fastdiv(ntB);
  td.ntAB = make_fastdiv(ntA * ntB);
  td.ntiles = ntA * ntB * nb;
  td.asp = make_fastdiv(1);
  td.aspq = ntA;
  if (fused && ntA % kASpread == 0 && ntA >= 2 * kASpread) {
    td.asp = make_fastdiv(kASpread);
    td.aspq = ntA / kASpread;
  }
  // 16-B vectors when every source row start (dims other than a) and every
  // destination row start (dims other than b) is 16-B aligned.
  bool va = aligned(src, 16), vb = aligned(dst, 16);
  for (int k = 0; k < (int)dims.size(); ++k) {
    if (k != a && (dims[k].ss * es) % 16) va = false;
    if (k != b && (dims[k].ds * es) % 16) vb = false;
  }
  if (fused && !(va && vb && (td.Lb1.d * es) % 16 == 0 && (td.La1.d * es) % 16 == 0)) {
    // the fused kernels are vectorised only: the plain tiles handle it
    return launch_transpose(src, dst, dims, a, es, st, false);
  }
  if (va && vb && (es == 1 || es == 2)) {
    // packed-word tiles: 256-B (u16) / 128-B (u8) source and 1-KiB destination segments
    TransDesc tp = td;
    const uint64_t pA = (uint64_t)((td.La + kPkTA - 1) / kPkTA), pB = (uint64_t)((td.Lb + kPkTB - 1) / kPkTB);
    tp.ntB = make_fastdiv(pB);
    tp.ntAB = make_fastdiv(pA * pB);
    tp.ntiles = pA * pB * nb;
    uint64_t g = tp.ntiles;
    if (g > kMaxGrid) g = kMaxGrid;
    if (es == 2) {
      k_transpose_pk<uint16_t, kPkTA, kPkTB, kPkThreads><<<(int)g, kPkThreads, 0, st>>>((const uint16_t *)src,
                                                                                     (uint16_t *)dst, tp);
    } else {
      if (g > 256) g = 256;  // pipelined: one block per CU (MI355X: 256 CUs)
      k_transpose_pkp<uint8_t, kPkTA, kPkTB, kPkThreads><<<(int)g, kPkThreads, 0, st>>>((const uint8_t *)src,
                                                                                      (uint8_t *)dst, tp);
    }
    return BM_OK;
  }
  int rc = BM_E_ARG;
  switch (es) {
    case 1: rc = launch_transpose_t<uint8_t>((const uint8_t *)src, (uint8_t *)dst, td, tl, va, vb, false, st); break;
    case 2: rc = launch_transpose_t<uint16_t>((const uint16_t *)src, (uint16_t *)dst, td, tl, va, vb, false, st); break;
    case 4: rc = launch_transpose_t<uint32_t>((const uint32_t *)src, (uint32_t *)dst, td, tl, va, vb, fused, st); break;
    case 8: rc = launch_transpose_t<uint64_t>((const uint64_t *)src, (uint64_t *)dst, td, tl, va, vb, fused, st); break;
    default: bm_set_error("bm_copy_strided: transpose with elem_bytes %d", es);
  }
  return rc;
}

int launch_generic(const char *src, char *dst, const std::vector<Dim> &dims, int es,
                   hipStream_t st) {
  Decomp d;
  if (!fill_decomp(d, dims)) {
    bm_set_error("bm_copy_strided: too many dims after fusion (%d)", (int)dims.size());
    return BM_E_ARG;
  }
  uint64_t total = 1;
  for (const Dim &x : dims) total *= (uint64_t)x.n;
  const int grid = grid_for(total, kThreads, kGenGridCap);
  switch (es) {
    case 1: k_generic<1><<<grid, kThreads, 0, st>>>(src, dst, d, total); break;
    case 2: k_generic<2><<<grid, kThreads, 0, st>>>(src, dst, d, total); break;
    case 4: k_generic<4><<<grid, kThreads, 0, st>>>(src, dst, d, total); break;
    case 8: k_generic<8><<<grid, kThreads, 0, st>>>(src, dst, d, total); break;
    case 16: k_generic<16><<<grid, kThreads, 0, st>>>(src, dst, d, total); break;
    default:
      bm_set_error("bm_copy_strided: generic with elem_bytes %d", es);
      return BM_E_ARG;
  }
  return BM_OK;
}


// Runs transpose applies when the innermost (both-contiguous) run is W 16-B
// units with 2 <= W <= 16, dim B (next in destination order) continues the
// destination run and some other dim A continues the source run.
int try_transpose_runs(const char *src, char *dst, const std::vector<Dim> &dims, int es,
                       hipStream_t st) {
  const int n = (int)dims.size();
  if (n < 3) return 1;
  const Dim &in = dims.back();
  const int64_t rb = in.n * es;
  if (rb % 16 || rb < 32 || rb > kRunsMaxBytes) return 1;
  if (!aligned(src, 16) || !aligned(dst, 16)) return 1;
  const int B = n - 2;
  if (dims[B].ds != in.n) return 1;
  int A = -1;
  for (int k = 0; k < n - 1; ++k)
    if (k != B && dims[k].ss == in.n) A = k;
  if (A < 0) return 1;
  for (int k = 0; k < n - 1; ++k)
    if ((dims[k].ss * es) % 16 || (dims[k].ds * es) % 16) return 1;
  const int W = (int)(rb / 16);
  const int64_t u = 16 / es;  // elements per unit
  RunsDesc d;
  d.La = dims[A].n;
  d.Lb = dims[B].n;
  d.sb = dims[B].ss / u;
  d.da = dims[A].ds / u;
  std::vector<Dim> batch;
  for (int k = 0; k < n - 1; ++k)
    if (k != A && k != B) batch.push_back({dims[k].n, dims[k].ss / u, dims[k].ds / u});
  if (!fill_decomp(d.batch, batch)) return 1;
  const int TA = kRunUnits / W;
  const uint64_t ntA = (uint64_t)((d.La + TA - 1) / TA);
  const uint64_t ntB = (uint64_t)((d.Lb + kRunTB - 1) / kRunTB);
  uint64_t nbatch = 1;
  for (const Dim &x : batch) nbatch *= (uint64_t)x.n;
  d.ntB = make_fastdiv(ntB);
  d.ntAB = make_fastdiv(ntA * ntB);
  d.ntiles = ntA * ntB * nbatch;
  uint64_t g = d.ntiles;
  if (g > kMaxGrid) g = kMaxGrid;
  const uint4 *s = (const uint4 *)src;
  uint4 *t = (uint4 *)dst;
  switch (W) {
    case 2: k_transpose_runs<2><<<(int)g, kThreads, 0, st>>>(s, t, d); break;
    case 4: k_transpose_runs<4><<<(int)g, kThreads, 0, st>>>(s, t, d); break;
    case 8: k_transpose_runs<8><<<(int)g, kThreads, 0, st>>>(s, t, d); break;
    case 16: k_transpose_runs<16><<<(int)g, kThreads, 0, st>>>(s, t, d); break;
    default: return 1;  // other widths: rowcopy
  }
  return 0;
}

// Canonical form: unit dims dropped, dims ordered by destination stride
// (outermost first), mergeable neighbours fused.
std::vector<Dim> canonicalize(std::vector<Dim> dims) {
  std::vector<Dim> v;
  for (const Dim &x : dims)
    if (x.n != 1) v.push_back(x);
  std::stable_sort(v.begin(), v.end(), [](const Dim &p, const Dim &q) {
    if (p.ds != q.ds) return p.ds > q.ds;
    return p.ss > q.ss;
  });
  std::vector<Dim> out;
  for (const Dim &x : v) {
    if (!out.empty() && out.back().ss == x.n * x.ss && out.back().ds == x.n * x.ds) {
      out.back().n *= x.n;
      out.back().ss = x.ss;
      out.back().ds = x.ds;
    } else {
      out.push_back(x);
    }
  }
  return out;
}

}  // namespace

extern "C" int bm_copy_strided(const void *src_, void *dst_, int ndim, const int64_t *shape,
                               const int64_t *src_strides, const int64_t *dst_strides,
                               int elem_bytes, void *stream) {
  if (ndim < 0 || ndim > 24 || elem_bytes <= 0 || (ndim > 0 && (!shape || !src_strides || !dst_strides))) {
    bm_set_error("bm_copy_strided: bad arguments (ndim=%d elem_bytes=%d)", ndim, elem_bytes);
    return BM_E_ARG;
  }
  std::vector<Dim> dims;
  for (int k = 0; k < ndim; ++k) {
    if (shape[k] < 0 || dst_strides[k] < 0) {  // source strides may be negative (reversed slices)
      bm_set_error("bm_copy_strided: negative shape / destination stride at dim %d", k);
      return BM_E_ARG;
    }
    if (shape[k] == 0) return BM_OK;  // empty: nothing to move
    dims.push_back({shape[k], src_strides[k], dst_strides[k]});
  }
  if (!src_ || !dst_) {
    bm_set_error("bm_copy_strided: null pointer");
    return BM_E_ARG;
  }
  int es = elem_bytes;
  // Element sizes without a native path move as bytes (extra inner dim).
  if (es != 1 && es != 2 && es != 4 && es != 8 && es != 16) {
    for (Dim &x : dims) { x.ss *= es; x.ds *= es; }
    dims.push_back({es, 1, 1});
    es = 1;
  }
  std::vector<Dim> c = canonicalize(dims);
  if (c.empty()) c.push_back({1, 1, 1});
  hipStream_t st = (hipStream_t)stream;
  const char *src = (const char *)src_;
  char *dst = (char *)dst_;
  int rc;
  const Dim &in = c.back();
  if (in.ss == 1 && in.ds == 1) {
    rc = try_transpose_runs(src, dst, c, es, st) == 0 ? BM_OK : launch_rowcopy(src, dst, c, es, st);
  } else {
    int a = -1;
    if (in.ds == 1 && es <= 8)
      for (int k = (int)c.size() - 2; k >= 0; --k)
        if (c[k].ss == 1) { a = k; break; }
    if (a >= 0) {
      rc = launch_transpose(src, dst, c, a, es, st);
    } else if (es == 16 && in.ds == 1) {
      // 16-B elements that need a transpose: move as pairs of 8-B words
      for (Dim &x : c) { x.ss *= 2; x.ds *= 2; }
      c.push_back({2, 1, 1});
      rc = launch_rowcopy(src, dst, canonicalize(c), 8, st);
    } else {
      rc = launch_generic(src, dst, c, es, st);
    }
  }
  if (rc != BM_OK) return rc;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    bm_set_error("bm_copy_strided: launch failed: %s", hipGetErrorString(e));
    return BM_E_HIP;
  }
  return BM_OK;
}

extern "C" int bm_permute(const void *src, void *dst, int ndim, const int64_t *shape,
                          const int32_t *perm, int elem_bytes, void *stream) {
  if (ndim < 0 || ndim > 24 || (ndim > 0 && (!shape || !perm))) {
    bm_set_error("bm_permute: bad arguments (ndim=%d)", ndim);
    return BM_E_ARG;
  }
  int64_t sstr[24], oshape[24], dstr[24];
  bool seen[24] = {false};
  int64_t acc = 1;
  for (int k = ndim - 1; k >= 0; --k) {
    sstr[k] = acc;
    acc *= shape[k];
  }
  for (int k = 0; k < ndim; ++k) {
    const int p = perm[k];
    if (p < 0 || p >= ndim || seen[p]) {
      bm_set_error("bm_permute: invalid permutation");
      return BM_E_ARG;
    }
    seen[p] = true;
    oshape[k] = shape[p];
  }
  acc = 1;
  for (int k = ndim - 1; k >= 0; --k) {
    dstr[k] = acc;
    acc *= oshape[k];
  }
  int64_t srcs[24];
  for (int k = 0; k < ndim; ++k) srcs[k] = sstr[perm[k]];
  return bm_copy_strided(src, dst, ndim, oshape, srcs, dstr, elem_bytes, stream);
}


// bm_chunk.hip -- record-map gather of libbolt_mi355x (gfx950): chunk pack /
// unpack of small records.
//
// ChunkedArray._chunk (bolt/spark/chunk.py:87-144) cuts every record's value
// block into the same set of (padded) chunks, and unchunk/removepad
// (chunk.py:146-200, :514-550) stitches them back; the layout change is the
// same for every record.  The host turns it into one int32 map per
// direction (plan.ChunkGeometry.record_map):
//
//     dst[r * dst_rec + o] = src[r * src_rec + map[o]]      o < dst_rec
//
// When a source record fits in LDS (C5: 64x64 float64 = 32 KiB; padded
// 16x16 chunks with 2-cell halos are 160-B rows that a strided copy reads
// badly), a block stages whole records with 16-B loads (records are
// contiguous, so a tile of RB records is one contiguous read), then writes
// the destination records contiguously, VEC elements per lane, picking each
// element out of LDS through the map (int32, L2-resident, shared by all
// records).  HBM traffic = the algorithmic bytes: src_rec + dst_rec element
// bytes per record, each byte moved once; the halo re-reads come from LDS.
//
// Parts: the host may split a record's destination into up to 8 ranges
// [dlo, dhi), each reading only the source range [slo, shi) it needs (chunks
// are laid out band by band, so these ranges are short); a tile is then one
// (record, part) and stages (shi - slo) elements -- a smaller LDS footprint,
// more blocks per CU.
// Larger records use the direct form (map lookups straight from HBM/L2).
#include "bm_common.h"
#include "../../include/bolt_mi355x.h"

#include <algorithm>

namespace {

constexpr int kCThreads = 256;
constexpr int64_t kStageBytes = 32768;   // LDS per tile when records are small (5 blocks / CU)
constexpr int64_t kMaxStageBytes = 65536;
constexpr int kMaxParts = 8;
constexpr int kRecmapGridCap = 16384;  // blocks per launch, then grid-stride over tiles

template <int ES> struct Elem;
template <> struct Elem<1> { typedef uint8_t t; };
template <> struct Elem<2> { typedef uint16_t t; };
template <> struct Elem<4> { typedef uint32_t t; };
template <> struct Elem<8> { typedef uint64_t t; };

struct Parts {
  int32_t n;
  int32_t pad_;
  int64_t dlo[kMaxParts], dhi[kMaxParts], slo[kMaxParts], shi[kMaxParts];
};

// Stage n L-vectors of a contiguous source range into LDS, kStageU loads in
// flight per lane (a one-load-then-wait loop left the kernel latency-bound;
// 4 or 16 in flight measured +-0.5%, profiles/r04i_pack_knobs.log).  Records
// are read and written once: non-temporal loads and stores.
template <typename V> __device__ __forceinline__ V ld_src(const V *p) { return __builtin_nontemporal_load(p); }
template <typename V> __device__ __forceinline__ void st_dst(V v, V *p) { __builtin_nontemporal_store(v, p); }
constexpr int kStageU = 8;
template <typename L>
__device__ __forceinline__ void stage_lds(L *sl, const L *s, int64_t n) {
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += (int64_t)kStageU * kCThreads) {
    L v[kStageU];
#pragma unroll
    for (int u = 0; u < kStageU; ++u) {
      const int64_t i = i0 + (int64_t)u * kCThreads;
      if (i < n) v[u] = ld_src(s + i);
    }
#pragma unroll
    for (int u = 0; u < kStageU; ++u) {
      const int64_t i = i0 + (int64_t)u * kCThreads;
      if (i < n) sl[i] = v[u];
    }
  }
}

// stage_lds over the units a bitmask marks (bit k: the 16-B unit k of the
// range), skipping the rest: halo rows the gather never reads stay in HBM.
template <typename L>
__device__ __forceinline__ void stage_lds_masked(L *sl, const L *s, int64_t n, const uint32_t *m) {
  constexpr int kLPU = 16 / (int)sizeof(L) > 0 ? 16 / (int)sizeof(L) : 1;  // L-vectors per 16-B unit
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += (int64_t)kStageU * kCThreads) {
    L v[kStageU];
    bool use[kStageU];
#pragma unroll
    for (int u = 0; u < kStageU; ++u) {
      const int64_t i = i0 + (int64_t)u * kCThreads;
      const int64_t k = i / kLPU;
      use[u] = i < n && ((m[k >> 5] >> (k & 31)) & 1u);
      if (use[u]) v[u] = ld_src(s + i);
    }
#pragma unroll
    for (int u = 0; u < kStageU; ++u) {
      const int64_t i = i0 + (int64_t)u * kCThreads;
      if (use[u]) sl[i] = v[u];
    }
  }
}

// destination vectors per lane per gather round (16 B of map per lane): their
// map reads go out together
template <int VEC>
struct GatherU {
  static constexpr int v = VEC >= 8 ? 2 : 16 / VEC;
};

// LB: staging load width in bytes (16 when the tile's bytes are 16-B aligned)
template <int ES, int VEC, int LB>
__global__ void __launch_bounds__(kCThreads)
    k_recmap_lds(const char *__restrict__ src, char *__restrict__ dst, const int32_t *__restrict__ map,
                 int64_t src_rec, int64_t dst_rec, int64_t nrec, int64_t rb, FastDiv fdst) {
  typedef typename Elem<ES>::t T;
  typedef typename VecB<LB>::t L;
  typedef typename VecB<ES * VEC>::t V;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const T *lds = reinterpret_cast<const T *>(smem);
  const int64_t ntiles = (nrec + rb - 1) / rb;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t r0 = t * rb;
    const int64_t nr = min(rb, nrec - r0);
    // stage nr contiguous source records
    stage_lds(reinterpret_cast<L *>(smem), reinterpret_cast<const L *>(src + r0 * src_rec * ES),
              nr * src_rec * ES / LB);
    __syncthreads();
    // gather nr destination records, VEC elements per lane, GU vectors per round
    constexpr int GU = GatherU<VEC>::v;
    const int64_t nout = nr * dst_rec / VEC;
    V *d = reinterpret_cast<V *>(dst + r0 * dst_rec * ES);
    for (int64_t i0 = threadIdx.x; i0 < nout; i0 += (int64_t)GU * kCThreads) {
      int32_t m[GU][VEC];
      int64_t rb_[GU];
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int64_t i = i0 + (int64_t)u * kCThreads;
        if (i < nout) {
          const uint64_t e = (uint64_t)i * VEC;
          const uint64_t r = fd_div(e, fdst);
          const int64_t o = (int64_t)(e - r * fdst.d);
          rb_[u] = (int64_t)r * src_rec;
#pragma unroll
          for (int k = 0; k < VEC; ++k) m[u][k] = map[o + k];
        }
      }
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int64_t i = i0 + (int64_t)u * kCThreads;
        if (i < nout) {
          T v[VEC];
#pragma unroll
          for (int k = 0; k < VEC; ++k) v[k] = lds[rb_[u] + m[u][k]];
          V w;
          __builtin_memcpy(&w, v, sizeof(V));
          st_dst(w, d + i);
        }
      }
    }
    __syncthreads();
  }
}

// one (record, part) per tile: stage src[slo, shi) of the record, write dst[dlo, dhi)
template <int ES, int VEC, int LB>
__global__ void __launch_bounds__(kCThreads)
    k_recmap_parts(const char *__restrict__ src, char *__restrict__ dst, const int32_t *__restrict__ map,
                   Parts P, int64_t src_rec, int64_t dst_rec, int64_t nrec, const uint32_t *__restrict__ mask,
                   int mask_words, int64_t mask_off) {
  typedef typename Elem<ES>::t T;
  typedef typename VecB<LB>::t L;
  typedef typename VecB<ES * VEC>::t V;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const T *lds = reinterpret_cast<const T *>(smem);
  const int64_t ntiles = nrec * P.n;
  uint32_t *lmask = reinterpret_cast<uint32_t *>(smem + mask_off);
  if (mask) {  // every part's unit mask, once per block
    for (int i = threadIdx.x; i < P.n * mask_words; i += kCThreads) lmask[i] = mask[i];
    __syncthreads();
  }
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t r = t / P.n;
    const int p = (int)(t - r * P.n);
    const int64_t slo = P.slo[p], dlo = P.dlo[p];
    if (mask)
      stage_lds_masked(reinterpret_cast<L *>(smem), reinterpret_cast<const L *>(src + (r * src_rec + slo) * ES),
                       (P.shi[p] - slo) * ES / LB, lmask + p * mask_words);
    else
      stage_lds(reinterpret_cast<L *>(smem), reinterpret_cast<const L *>(src + (r * src_rec + slo) * ES),
                (P.shi[p] - slo) * ES / LB);
    __syncthreads();
    constexpr int GU = GatherU<VEC>::v;
    const int64_t nout = (P.dhi[p] - dlo) / VEC;
    V *d = reinterpret_cast<V *>(dst + (r * dst_rec + dlo) * ES);
    const int32_t *mp = map + dlo;
    for (int64_t i0 = threadIdx.x; i0 < nout; i0 += (int64_t)GU * kCThreads) {
      int32_t m[GU][VEC];
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int64_t i = i0 + (int64_t)u * kCThreads;
        if (i < nout) {
#pragma unroll
          for (int k = 0; k < VEC; ++k) m[u][k] = mp[i * VEC + k];
        }
      }
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int64_t i = i0 + (int64_t)u * kCThreads;
        if (i < nout) {
          T v[VEC];
#pragma unroll
          for (int k = 0; k < VEC; ++k) v[k] = lds[m[u][k] - slo];
          V w;
          __builtin_memcpy(&w, v, sizeof(V));
          st_dst(w, d + i);
        }
      }
    }
    __syncthreads();
  }
}

template <int ES>
__global__ void __launch_bounds__(kCThreads)
    k_recmap_direct(const char *__restrict__ src, char *__restrict__ dst, const int32_t *__restrict__ map,
                    int64_t src_rec, uint64_t total, FastDiv fdst) {
  typedef typename Elem<ES>::t T;
  const T *s = reinterpret_cast<const T *>(src);
  T *d = reinterpret_cast<T *>(dst);
  const uint64_t step = (uint64_t)gridDim.x * kCThreads;
  for (uint64_t g = (uint64_t)blockIdx.x * kCThreads + threadIdx.x; g < total; g += step) {
    const uint64_t r = fd_div(g, fdst);
    const int64_t o = (int64_t)(g - r * fdst.d);
    d[g] = s[(int64_t)r * src_rec + map[o]];
  }
}

// Record scatter: source records are read front to back, VEC elements per
// lane, and every element p of record r goes to
//     dst[(r / group) * gstride + map_a[p] + (r % group) * map_b[p]]
// (map_a[p] < 0: dropped).  For the packed -> packed moves whose source record
// is read whole and whose destination runs are chunk boxes: keys_to_values of
// the trailing keys (group = their extent, map_b = box sizes), values_to_keys
// and unchunk (group 1).  Reads are one contiguous stream; writes are
// contiguous runs of whole boxes, adjacent across consecutive records.
// One source vector per lane per round (U = 2..8 in flight measured
// -4..-17%: a wave's vectors then sit 4 KiB apart; a speculative source load
// before the map entry arrives -1.5%, profiles/r04b_scatter_u.log).
constexpr int kScatterU = 1;
template <int ES, int VEC>
__global__ void __launch_bounds__(kCThreads)
    k_recmap_scatter(const char *__restrict__ src, char *__restrict__ dst, const int32_t *__restrict__ ma,
                     const int32_t *__restrict__ mb, uint64_t total, FastDiv fvpr, FastDiv fgroup,
                     int64_t gstride) {
  typedef typename VecB<ES * VEC>::t V;
  constexpr int U = kScatterU;
  const uint64_t step = (uint64_t)gridDim.x * kCThreads * U;
  for (uint64_t i0 = (uint64_t)blockIdx.x * kCThreads * U + threadIdx.x; i0 < total; i0 += step) {
    V x[U];
    int64_t d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = i0 + (uint64_t)u * kCThreads;
      d[u] = -1;
      if (i < total) {
        const uint64_t r = fd_div(i, fvpr);
        const int64_t p = (int64_t)(i - r * fvpr.d) * VEC;
        const int32_t a = ma[p];
        if (a >= 0) {
          const uint64_t hi = fd_div(r, fgroup);
          d[u] = (int64_t)hi * gstride + a;
          if (mb) d[u] += (int64_t)(r - hi * fgroup.d) * mb[p];
          x[u] = ld_src(reinterpret_cast<const V *>(src) + i);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (d[u] >= 0) st_dst(x[u], reinterpret_cast<V *>(dst + d[u] * ES));
  }
}

template <int ES>
void launch_scatter(const char *src, char *dst, const int32_t *ma, const int32_t *mb, int64_t nrec,
                    int64_t src_rec, int64_t group, int64_t gstride, int vec, hipStream_t st) {
  const uint64_t vpr = (uint64_t)(src_rec / vec);
  const uint64_t total = (uint64_t)nrec * vpr;
  uint64_t g = (total + (uint64_t)kCThreads * kScatterU - 1) / ((uint64_t)kCThreads * kScatterU);
  if (g > 16777215ull) g = 16777215ull;  // HIP launch limit, then grid-stride
  const FastDiv fv = make_fastdiv(vpr), fg = make_fastdiv((uint64_t)group);
  constexpr int V16 = 16 / ES;
  if (vec == V16)
    k_recmap_scatter<ES, V16><<<(int)g, kCThreads, 0, st>>>(src, dst, ma, mb, total, fv, fg, gstride);
  else if (ES <= 4 && vec == (8 / ES > 0 ? 8 / ES : 1))
    k_recmap_scatter<ES, (8 / ES > 0 ? 8 / ES : 1)><<<(int)g, kCThreads, 0, st>>>(src, dst, ma, mb, total, fv, fg,
                                                                                gstride);
  else if (ES <= 2 && vec == (4 / ES > 0 ? 4 / ES : 1))
    k_recmap_scatter<ES, (4 / ES > 0 ? 4 / ES : 1)><<<(int)g, kCThreads, 0, st>>>(src, dst, ma, mb, total, fv, fg,
                                                                                gstride);
  else if (ES == 1 && vec == 2)
    k_recmap_scatter<ES, 2><<<(int)g, kCThreads, 0, st>>>(src, dst, ma, mb, total, fv, fg, gstride);
  else
    k_recmap_scatter<ES, 1><<<(int)g, kCThreads, 0, st>>>(src, dst, ma, mb, total, fv, fg, gstride);
}

// Record runs: the same moves as the record scatter when a source record is a
// handful of long runs (C5 keys_to_values((2,)): 16 chunk boxes of 2.6-3.2 KB,
// each contiguous in the source record and in its new record).  Run b of
// record r (r = g * group + k):
//     dst[g * gstride + a_b + k * m_b + j] = src[r * src_rec + s_b + j],  j < len_b
// One wave per (record, run) unit, ordered by source (u = r * nruns + b), no
// maps: every lane's loads issue at once, kRunsU vectors in flight per lane,
// and a wave writes one contiguous run.  (Destination-major unit order ran
// within 0.6% of it, profiles/r04b_runs.log; runs that tile the new records
// take the destination walk below instead.)
// Runs table: DEVICE int64 [s, len, a, m] x nruns, in VB-byte vectors.
constexpr int kRunsU = 4;
template <int VB>
__global__ void __launch_bounds__(kCThreads)
    k_record_runs(const char *__restrict__ src, char *__restrict__ dst, const int64_t *__restrict__ runs,
                  int nruns, uint64_t nunits, int64_t src_rec, int64_t gstride, FastDiv fruns, FastDiv fgroup) {
  typedef typename VecB<VB>::t V;
  constexpr int U = kRunsU;
  const V *s = reinterpret_cast<const V *>(src);
  V *d = reinterpret_cast<V *>(dst);
  const int lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * (kCThreads / 64);
  for (uint64_t u = (uint64_t)blockIdx.x * (kCThreads / 64) + (threadIdx.x >> 6); u < nunits; u += nw) {
    const uint64_t r = fd_div(u, fruns);
    const int b = (int)(u - r * fruns.d);
    const uint64_t g = fd_div(r, fgroup);
    const uint64_t k = r - g * fgroup.d;
    const int64_t *e = runs + 4 * b;
    const int64_t len = e[1];
    const V *sp = s + (int64_t)r * src_rec + e[0];
    V *dp = d + (int64_t)g * gstride + e[2] + (int64_t)k * e[3];
    for (int64_t v0 = lane; v0 < len; v0 += 64 * U) {
      V x[U];
#pragma unroll
      for (int t = 0; t < U; ++t)
        if (v0 + 64 * t < len) x[t] = ld_src(sp + v0 + 64 * t);
#pragma unroll
      for (int t = 0; t < U; ++t)
        if (v0 + 64 * t < len) st_dst(x[t], dp + v0 + 64 * t);
    }
  }
}

// Destination walk (runs tile each new record: m_b = len_b, regions
// [a_b, a_b + group * len_b) back to back): lanes take the destination vectors
// in order -- every wave writes 64 * U consecutive vectors, whole lines -- and
// each finds its source: run b by binary search over the runs (sorted by a,
// staged in LDS), k = (o - a_b) / len_b, then the source record g * group + k.
// kWalkU = 2 vectors per lane beats 1 (-1.7%) and 4 (-2.5%); the blocks of
// one XCD walk one contiguous eighth of the destination, and the source loads
// are temporal: a source line two chunk boxes of a record share is then read
// again a region later from the same XCD's L2 (PMC traffic 1.0375x ->
// 1.0000x, +0.7..+2.5% on C5's keys_to_values, profiles/r04o_runs_xcd.log).
constexpr int kWalkU = 2;
constexpr int kMaxWalkRuns = 64;
template <int VB, int U>
__global__ void __launch_bounds__(kCThreads)
    k_record_runs_dst(const char *__restrict__ src, char *__restrict__ dst, const int64_t *__restrict__ runs,
                      int nruns, uint64_t total, int64_t src_rec, int64_t group, FastDiv fgs) {
  typedef typename VecB<VB>::t V;
  __shared__ int64_t tab[4 * kMaxWalkRuns];
  __shared__ double inv[kMaxWalkRuns];
  for (int i = threadIdx.x; i < 4 * nruns; i += kCThreads) tab[i] = runs[i];
  for (int i = threadIdx.x; i < nruns; i += kCThreads) inv[i] = 1.0 / (double)runs[4 * i + 1];
  __syncthreads();
  const V *s = reinterpret_cast<const V *>(src);
  V *d = reinterpret_cast<V *>(dst);
  const int lane = threadIdx.x & 63;
  const uint64_t per_block = (uint64_t)kCThreads * U;
  const uint64_t wave0 = (uint64_t)(threadIdx.x >> 6) * 64 * U;
  const uint64_t nwork = (total + per_block - 1) / per_block;
  // the blocks of one XCD (w % 8 under round-robin dispatch; the grid is a
  // multiple of 8) take one contiguous eighth of the destination (affinity
  // only: any block-to-XCD mapping is correct)
  const bool xcd = nwork % 8 == 0 && gridDim.x % 8 == 0;
  for (uint64_t w = blockIdx.x; w < nwork; w += gridDim.x) {
    const uint64_t base = (xcd ? (w % 8) * (nwork / 8) + w / 8 : w) * per_block;
    V x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = base + wave0 + (uint64_t)u * 64 + lane;
      if (j < total) {
        const uint64_t g = fd_div(j, fgs);
        const int64_t o = (int64_t)(j - g * fgs.d);
        int lo = 0, hi = nruns - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (tab[4 * mid + 2] <= o) lo = mid;
          else hi = mid - 1;
        }
        const int64_t off = o - tab[4 * lo + 2], len = tab[4 * lo + 1];
        int64_t k = (int64_t)((double)off * inv[lo]);
        if (k * len > off) --k;
        else if ((k + 1) * len <= off) ++k;
        // a table that does not tile the records (a wrong BM_RUNS_TILED) gives
        // wrong bytes, never an access outside run b of a source record of
        // this group: k in [0, group), the offset in [0, len)
        k = k < 0 ? 0 : (k >= group ? group - 1 : k);
        int64_t pos = off - k * len;
        pos = pos < 0 ? 0 : (pos >= len ? len - 1 : pos);
        const V *sp = s + ((int64_t)g * group + k) * src_rec + tab[4 * lo] + pos;
        x[u] = *sp;  // temporal: the shared line's second read hits L2
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = base + wave0 + (uint64_t)u * 64 + lane;
      if (j < total) st_dst(x[u], d + j);
    }
  }
}

template <int VB>
void launch_runs(const char *src, char *dst, const int64_t *runs, int nruns, int64_t nrec, int64_t src_rec,
                 int64_t group, int64_t gstride, bool tiled, hipStream_t st) {
  if (tiled) {
    const uint64_t total = (uint64_t)(nrec / group) * (uint64_t)gstride;
    const uint64_t per_block = (uint64_t)kCThreads * kWalkU;
    uint64_t g = (total + per_block - 1) / per_block;
    if (g > 1048576) g = 1048576;
    k_record_runs_dst<VB, kWalkU><<<(int)g, kCThreads, 0, st>>>(src, dst, runs, nruns, total, src_rec, group,
                                                               make_fastdiv((uint64_t)gstride));
    return;
  }
  const uint64_t nunits = (uint64_t)nrec * (uint64_t)nruns;
  uint64_t g = (nunits + kCThreads / 64 - 1) / (kCThreads / 64);
  if (g > 1048576) g = 1048576;  // then grid-stride over units
  const FastDiv fr = make_fastdiv((uint64_t)nruns), fg = make_fastdiv((uint64_t)group);
  k_record_runs<VB><<<(int)g, kCThreads, 0, st>>>(src, dst, runs, nruns, nunits, src_rec, gstride, fr, fg);
}

struct Launch {
  const char *src;
  char *dst;
  const int32_t *map;
  int64_t src_rec, dst_rec, nrec, rb;
  const Parts *parts;  // null: whole records, rb per tile
  const uint32_t *mask;  // parts only: 16-B unit masks of the staged ranges (null: stage all)
  int mask_words;
  int64_t mask_off;
  int grid;
  size_t shmem;
  hipStream_t st;
};

template <int ES, int VEC, int LB>
void launch_one(const Launch &L) {
  if (L.parts)
    k_recmap_parts<ES, VEC, LB><<<L.grid, kCThreads, L.shmem, L.st>>>(L.src, L.dst, L.map, *L.parts, L.src_rec,
                                                                       L.dst_rec, L.nrec, L.mask, L.mask_words,
                                                                       L.mask_off);
  else
    k_recmap_lds<ES, VEC, LB><<<L.grid, kCThreads, L.shmem, L.st>>>(L.src, L.dst, L.map, L.src_rec, L.dst_rec,
                                                                     L.nrec, L.rb, make_fastdiv((uint64_t)L.dst_rec));
}

template <int ES, int VEC>
void launch_lb(const Launch &L, int lb) {
  switch (lb) {
    case 16: launch_one<ES, VEC, 16>(L); break;
    case 8: launch_one<ES, VEC, 8>(L); break;
    case 4: launch_one<ES, VEC, 4>(L); break;
    case 2: launch_one<ES, VEC, 2>(L); break;
    default: launch_one<ES, VEC, 1>(L); break;
  }
}

template <int ES>
void launch_lds(const Launch &L, int lb, int vec) {
  constexpr int V16 = 16 / ES;
  if (vec >= V16) return launch_lb<ES, V16>(L, lb);
  if (ES <= 4 && vec >= 8 / ES) return launch_lb<ES, (8 / ES > 0 ? 8 / ES : 1)>(L, lb);
  if (ES <= 2 && vec >= 4 / ES) return launch_lb<ES, (4 / ES > 0 ? 4 / ES : 1)>(L, lb);
  if (ES == 1 && vec >= 2) return launch_lb<ES, 2>(L, lb);
  launch_lb<ES, 1>(L, lb);
}

int pow2_align(uintptr_t a, int64_t bytes, int cap) {
  int w = cap;
  while (w > 1 && (((a % (uintptr_t)w) != 0) || (bytes % w) != 0)) w >>= 1;
  return w;
}

}  // namespace

extern "C" int bm_record_gather_masked(const void *src_, void *dst_, int64_t nrec, int64_t src_rec,
                                       int64_t dst_rec, const int32_t *map, int nparts, const int64_t *parts,
                                       const uint32_t *stage_mask, int mask_words, int elem_bytes, void *stream);

extern "C" int bm_record_gather(const void *src_, void *dst_, int64_t nrec, int64_t src_rec, int64_t dst_rec,
                                const int32_t *map, int nparts, const int64_t *parts, int elem_bytes,
                                void *stream) {
  return bm_record_gather_masked(src_, dst_, nrec, src_rec, dst_rec, map, nparts, parts, nullptr, 0, elem_bytes,
                                 stream);
}

extern "C" int bm_record_gather_masked(const void *src_, void *dst_, int64_t nrec, int64_t src_rec,
                                       int64_t dst_rec, const int32_t *map, int nparts, const int64_t *parts,
                                       const uint32_t *stage_mask, int mask_words, int elem_bytes, void *stream) {
  if (nrec < 0 || src_rec <= 0 || dst_rec <= 0 || src_rec > 0x7fffffffLL || nparts < 0 || nparts > kMaxParts ||
      (nparts > 1 && !parts) || (elem_bytes != 1 && elem_bytes != 2 && elem_bytes != 4 && elem_bytes != 8)) {
    bm_set_error("bm_record_gather: bad arguments (nrec %lld, src_rec %lld, dst_rec %lld, nparts %d, elem_bytes %d)",
                 (long long)nrec, (long long)src_rec, (long long)dst_rec, nparts, elem_bytes);
    return BM_E_ARG;
  }
  const int es = elem_bytes;
  Parts P;
  P.n = nparts > 1 ? nparts : 1;
  P.pad_ = 0;
  int64_t span = src_rec;
  if (nparts > 1) {  // the ranges must tile [0, dst_rec) in order, sources inside the record
    int64_t at = 0;
    span = 0;
    for (int p = 0; p < nparts; ++p) {
      const int64_t dlo = parts[4 * p], dhi = parts[4 * p + 1], slo = parts[4 * p + 2], shi = parts[4 * p + 3];
      if (dlo != at || dhi <= dlo || slo < 0 || shi <= slo || shi > src_rec) {
        bm_set_error("bm_record_gather: part %d [%lld, %lld) <- [%lld, %lld) does not tile the record", p,
                     (long long)dlo, (long long)dhi, (long long)slo, (long long)shi);
        return BM_E_ARG;
      }
      P.dlo[p] = dlo; P.dhi[p] = dhi; P.slo[p] = slo; P.shi[p] = shi;
      span = std::max(span, shi - slo);
      at = dhi;
    }
    if (at != dst_rec || span * es > kMaxStageBytes) {
      bm_set_error("bm_record_gather: parts cover %lld of %lld elements, widest source range %lld B",
                   (long long)at, (long long)dst_rec, (long long)(span * es));
      return BM_E_ARG;
    }
  }
  if (nrec == 0) return BM_OK;
  if (!src_ || !dst_ || !map) {
    bm_set_error("bm_record_gather: null pointer");
    return BM_E_ARG;
  }
  const char *src = static_cast<const char *>(src_);
  char *dst = static_cast<char *>(dst_);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t rec_bytes = src_rec * es;
  if (span * es <= kMaxStageBytes) {
    Launch L;
    L.src = src; L.dst = dst; L.map = map;
    L.src_rec = src_rec; L.dst_rec = dst_rec; L.nrec = nrec; L.st = st;
    int lb = pow2_align((uintptr_t)src, rec_bytes, 16);     // every tile start aligned
    int vb = pow2_align((uintptr_t)dst, dst_rec * es, 16);  // bytes per store
    int64_t ntiles;
    if (nparts > 1) {
      for (int p = 0; p < nparts; ++p) {
        lb = std::min(lb, pow2_align((uintptr_t)(P.slo[p] * es), (P.shi[p] - P.slo[p]) * es, 16));
        vb = std::min(vb, pow2_align((uintptr_t)(P.dlo[p] * es), (P.dhi[p] - P.dlo[p]) * es, 16));
      }
      L.rb = 1;
      L.parts = &P;
      L.shmem = (size_t)(span * es + 15) / 16 * 16;
      L.mask = nullptr;
      L.mask_words = 0;
      L.mask_off = (int64_t)L.shmem;
      if (stage_mask && mask_words > 0) {
        // one bit per 16-B unit of the widest range (checked against it), all parts' masks in LDS
        if ((int64_t)mask_words * 32 * 16 < span * es) {
          bm_set_error("bm_record_gather: %d mask words cannot cover %lld-B ranges", mask_words,
                       (long long)(span * es));
          return BM_E_ARG;
        }
        L.mask = stage_mask;
        L.mask_words = mask_words;
        L.shmem += (size_t)nparts * mask_words * 4;
      }
      ntiles = nrec * nparts;
    } else {
      int64_t rb = rec_bytes >= kStageBytes ? 1 : kStageBytes / rec_bytes;
      if (rb > nrec) rb = nrec;
      L.rb = rb;
      L.parts = nullptr;
      L.mask = nullptr;
      L.mask_words = 0;
      L.mask_off = 0;
      L.shmem = (size_t)(rb * rec_bytes + 15) / 16 * 16;
      ntiles = (nrec + rb - 1) / rb;
    }
    L.grid = (int)(ntiles < kRecmapGridCap ? ntiles : kRecmapGridCap);
    const int vec = std::max(1, vb / es);
    switch (es) {
      case 1: launch_lds<1>(L, lb, vec); break;
      case 2: launch_lds<2>(L, lb, vec); break;
      case 4: launch_lds<4>(L, lb, vec); break;
      default: launch_lds<8>(L, lb, vec); break;
    }
  } else {
    const uint64_t total = (uint64_t)nrec * (uint64_t)dst_rec;
    uint64_t g = (total + kCThreads - 1) / kCThreads;
    if (g > 1048576) g = 1048576;
    const FastDiv f = make_fastdiv((uint64_t)dst_rec);
    switch (es) {
      case 1: k_recmap_direct<1><<<(int)g, kCThreads, 0, st>>>(src, dst, map, src_rec, total, f); break;
      case 2: k_recmap_direct<2><<<(int)g, kCThreads, 0, st>>>(src, dst, map, src_rec, total, f); break;
      case 4: k_recmap_direct<4><<<(int)g, kCThreads, 0, st>>>(src, dst, map, src_rec, total, f); break;
      default: k_recmap_direct<8><<<(int)g, kCThreads, 0, st>>>(src, dst, map, src_rec, total, f); break;
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    bm_set_error("bm_record_gather: launch failed: %s", hipGetErrorString(e));
    return BM_E_HIP;
  }
  return BM_OK;
}

extern "C" int bm_record_scatter(const void *src_, void *dst_, int64_t nrec, int64_t src_rec, int64_t group,
                                 int64_t dst_group_stride, const int32_t *map_a, const int32_t *map_b, int vec,
                                 int elem_bytes, void *stream) {
  const int es = elem_bytes;
  if (nrec < 0 || src_rec <= 0 || group < 1 || dst_group_stride < 0 || vec < 1 || (vec & (vec - 1)) ||
      (es != 1 && es != 2 && es != 4 && es != 8) || vec * es > 16 || src_rec % vec || dst_group_stride % vec ||
      src_rec > 0x7fffffffLL) {
    bm_set_error("bm_record_scatter: bad arguments (nrec %lld, src_rec %lld, group %lld, stride %lld, vec %d, "
                 "elem_bytes %d)", (long long)nrec, (long long)src_rec, (long long)group,
                 (long long)dst_group_stride, vec, es);
    return BM_E_ARG;
  }
  if (nrec == 0) return BM_OK;
  if (!src_ || !dst_ || !map_a) {
    bm_set_error("bm_record_scatter: null pointer");
    return BM_E_ARG;
  }
  if ((uintptr_t)src_ % (uintptr_t)(vec * es) || (uintptr_t)dst_ % (uintptr_t)(vec * es)) {
    bm_set_error("bm_record_scatter: buffers not aligned to %d-element vectors", vec);
    return BM_E_ARG;
  }
  const char *src = static_cast<const char *>(src_);
  char *dst = static_cast<char *>(dst_);
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (es) {
    case 1: launch_scatter<1>(src, dst, map_a, map_b, nrec, src_rec, group, dst_group_stride, vec, st); break;
    case 2: launch_scatter<2>(src, dst, map_a, map_b, nrec, src_rec, group, dst_group_stride, vec, st); break;
    case 4: launch_scatter<4>(src, dst, map_a, map_b, nrec, src_rec, group, dst_group_stride, vec, st); break;
    default: launch_scatter<8>(src, dst, map_a, map_b, nrec, src_rec, group, dst_group_stride, vec, st); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    bm_set_error("bm_record_scatter: launch failed: %s", hipGetErrorString(e));
    return BM_E_HIP;
  }
  return BM_OK;
}

extern "C" int bm_record_runs(const void *src_, void *dst_, int64_t nrec, int64_t src_rec, int64_t group,
                              int64_t dst_group_stride, int nruns, const int64_t *runs, int vec_bytes, int flags,
                              int elem_bytes, void *stream) {
  const int es = elem_bytes, vb = vec_bytes;
  const bool tiled = (flags & BM_RUNS_TILED) != 0;
  if (nrec < 0 || src_rec <= 0 || group < 1 || nrec % group || dst_group_stride < 0 || nruns < 1 ||
      nruns > 4096 || (tiled && nruns > kMaxWalkRuns) || (flags & ~BM_RUNS_TILED) ||
      (es != 1 && es != 2 && es != 4 && es != 8) || vb < es || vb > 16 || (vb & (vb - 1)) ||
      (src_rec * es) % vb || (dst_group_stride * es) % vb) {
    bm_set_error("bm_record_runs: bad arguments (nrec %lld, src_rec %lld, group %lld, stride %lld, nruns %d, "
                 "vec_bytes %d, flags %d, elem_bytes %d)", (long long)nrec, (long long)src_rec, (long long)group,
                 (long long)dst_group_stride, nruns, vb, flags, es);
    return BM_E_ARG;
  }
  if (nrec == 0) return BM_OK;
  if (!src_ || !dst_ || !runs) {
    bm_set_error("bm_record_runs: null pointer");
    return BM_E_ARG;
  }
  if ((uintptr_t)src_ % (uintptr_t)vb || (uintptr_t)dst_ % (uintptr_t)vb) {
    bm_set_error("bm_record_runs: buffers not aligned to %d-byte vectors", vb);
    return BM_E_ARG;
  }
  const char *src = static_cast<const char *>(src_);
  char *dst = static_cast<char *>(dst_);
  hipStream_t st = static_cast<hipStream_t>(stream);
  // record size and group stride in vectors; the table is in vectors already
  const int64_t sv = src_rec * es / vb, gv = dst_group_stride * es / vb;
  switch (vb) {
    case 16: launch_runs<16>(src, dst, runs, nruns, nrec, sv, group, gv, tiled, st); break;
    case 8: launch_runs<8>(src, dst, runs, nruns, nrec, sv, group, gv, tiled, st); break;
    case 4: launch_runs<4>(src, dst, runs, nruns, nrec, sv, group, gv, tiled, st); break;
    case 2: launch_runs<2>(src, dst, runs, nruns, nrec, sv, group, gv, tiled, st); break;
    default: launch_runs<1>(src, dst, runs, nruns, nrec, sv, group, gv, tiled, st); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    bm_set_error("bm_record_runs: launch failed: %s", hipGetErrorString(e));
    return BM_E_HIP;
  }
  return BM_OK;
}

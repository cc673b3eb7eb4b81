// bm_gather.hip -- row gather of libbolt_mi355x (gfx950): advanced indexing.
//
// dst[a, j, :] = src[a, idx[j], :] over a (n_outer, src_rows, row_bytes) view
// of the source.  Serves the two non-strided selections of
// BoltArraySpark.__getitem__ (bolt/spark/array.py:514-593):
//   mixed     one index list on one axis: n_outer = product of the axes in
//             front of it, row = the axes behind it (x.take(idx, axis));
//   advanced  one index list per axis: n_outer = 1, row = one element (a
//             point gather, out[j] = x.flat[idx[j]]).
// Every lane moves one vector of the widest size (16/8/4/2/1 B) that divides
// the row and both base pointers; HBM-bound, algorithmic bytes =
// 2 * n_outer * n_idx * row_bytes (+ 8 B per index, read once per row).
#include "bm_common.h"
#include "../../include/bolt_mi355x.h"

namespace {

constexpr int kGThreads = 256;

template <int VB>
__global__ __launch_bounds__(kGThreads) void k_gather_rows(const char *__restrict__ src, char *__restrict__ dst,
                                                          const int64_t *__restrict__ idx, FastDiv upr,
                                                          FastDiv nidx, int64_t src_rows, uint64_t total) {
  typedef typename VecB<VB>::t V;
  const uint64_t step = (uint64_t)gridDim.x * kGThreads;
  for (uint64_t g = (uint64_t)blockIdx.x * kGThreads + threadIdx.x; g < total; g += step) {
    const uint64_t row = fd_div(g, upr);       // output row (a, j)
    const uint64_t u = g - row * upr.d;        // vector within the row
    const uint64_t a = fd_div(row, nidx);
    const uint64_t j = row - a * nidx.d;
    const int64_t srow = (int64_t)a * src_rows + idx[j];
    const V v = __builtin_nontemporal_load(reinterpret_cast<const V *>(src) + srow * (int64_t)upr.d + u);
    __builtin_nontemporal_store(v, reinterpret_cast<V *>(dst) + g);
  }
}

template <int VB>
void launch(const char *src, char *dst, const int64_t *idx, int64_t n_outer, int64_t src_rows,
            int64_t row_bytes, int64_t n_idx, hipStream_t st) {
  const uint64_t upr = (uint64_t)(row_bytes / VB);
  const uint64_t total = (uint64_t)n_outer * (uint64_t)n_idx * upr;
  uint64_t g = (total + kGThreads - 1) / kGThreads;
  if (g > 1048576) g = 1048576;
  k_gather_rows<VB><<<(int)g, kGThreads, 0, st>>>(src, dst, idx, make_fastdiv(upr), make_fastdiv((uint64_t)n_idx),
                                                  src_rows, total);
}

}  // namespace

extern "C" int bm_gather_rows(const void *src, void *dst, int64_t n_outer, int64_t src_rows, int64_t row_bytes,
                              const int64_t *idx, int64_t n_idx, void *stream) {
  if (n_outer < 0 || src_rows < 0 || row_bytes <= 0 || n_idx < 0) {
    bm_set_error("bm_gather_rows: bad sizes (n_outer %lld, src_rows %lld, row_bytes %lld, n_idx %lld)",
                 (long long)n_outer, (long long)src_rows, (long long)row_bytes, (long long)n_idx);
    return BM_E_ARG;
  }
  if (n_outer == 0 || n_idx == 0) return BM_OK;
  if (!src || !dst || !idx || src_rows == 0) {
    bm_set_error("bm_gather_rows: null pointer or empty source");
    return BM_E_ARG;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const char *s = static_cast<const char *>(src);
  char *d = static_cast<char *>(dst);
  const uintptr_t al = (uintptr_t)s | (uintptr_t)d;
  int vb = 16;
  while (vb > 1 && ((row_bytes % vb) != 0 || (al % vb) != 0)) vb >>= 1;
  switch (vb) {
    case 16: launch<16>(s, d, idx, n_outer, src_rows, row_bytes, n_idx, st); break;
    case 8: launch<8>(s, d, idx, n_outer, src_rows, row_bytes, n_idx, st); break;
    case 4: launch<4>(s, d, idx, n_outer, src_rows, row_bytes, n_idx, st); break;
    case 2: launch<2>(s, d, idx, n_outer, src_rows, row_bytes, n_idx, st); break;
    default: launch<1>(s, d, idx, n_outer, src_rows, row_bytes, n_idx, st); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    bm_set_error("bm_gather_rows: launch failed: %s", hipGetErrorString(e));
    return BM_E_HIP;
  }
  return BM_OK;
}

/*
 * bolt_mi355x.h -- C ABI of libbolt_mi355x.so, the MI355X (gfx950) execution
 * backend for bolt's Spark-mode data-parallel hot path.
 *
 * The reference (beautifulNow1992/bolt v0.7.1) is pure Python; its "FFI" for
 * this path is the pyspark RDD API that the bolt/spark modules call.  Every entry
 * point below replaces one of those call sites; the ctypes binding a bolt
 * maintainer would add is bolt_amd/_lib.py.
 *
 * Conventions
 *   - Plain pointers and sizes only; no torch / numpy types cross this ABI.
 *   - Device buffers are owned by the caller (PyTorch allocations passed as
 *     tensor.data_ptr()).  The library allocates no device memory: scratch
 *     comes from a caller-provided workspace.
 *   - All work is stream-ordered on the caller's HIP stream (`stream` is a
 *     hipStream_t; NULL = the legacy default stream).  No call synchronises
 *     the device.
 *   - Every function returns 0 on success and a negative BM_E* code on
 *     failure; the message is available from bm_last_error() (thread-local).
 *     Nothing throws or aborts across this boundary.
 *   - Strides and shapes are in ELEMENTS, int64, C order (outermost first).
 */
#ifndef BOLT_MI355X_H
#define BOLT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BM_ABI_VERSION 1

/* status codes */
#define BM_OK 0
#define BM_E_ARG (-1)    /* invalid argument (shape, stride, dtype, ...)   */
#define BM_E_HIP (-2)    /* a HIP runtime call failed (launch, ...)       */
#define BM_E_WS (-3)     /* workspace too small                            */

/* element dtypes understood by the reductions (numpy kinds) */
#define BM_BOOL 0
#define BM_U8 1
#define BM_I8 2
#define BM_U16 3
#define BM_I16 4
#define BM_U32 5
#define BM_I32 6
#define BM_U64 7
#define BM_I64 8
#define BM_F16 9
#define BM_F32 10
#define BM_F64 11

/* statistics (bolt/spark/array.py:_stat names + reduce(add)) */
#define BM_STAT_MEAN 0   /* StatCounter.mean      statcounter.py:109-112 */
#define BM_STAT_VAR 1    /* StatCounter.variance  statcounter.py:119-125 */
#define BM_STAT_STD 2    /* StatCounter.stdev     statcounter.py:127-130 */
#define BM_STAT_SUM 3    /* reduce(operator.add)  array.py:243-282, :381-395 */
#define BM_STAT_MAX 4    /* reduce(numpy.maximum) array.py:397-411 (NaN propagates) */
#define BM_STAT_MIN 5    /* reduce(numpy.minimum) array.py:413-427 (NaN propagates) */

/* Version of this ABI (BM_ABI_VERSION).  Host code refuses a mismatch. */
int bm_abi_version(void);

/* Last error message of the calling thread ("" if none). */
const char *bm_last_error(void);

/* Number of compute units of the current device (for sizing), or <0. */
int bm_device_cus(void);

/*
 * bm_host_writable -- *ok = 1 if [p, p + bytes) is page-locked host memory that
 * the current device addresses at the same pointer, else 0.  Statistics with
 * small results (mean/var/std/sum over most axes, array.py:284-395) pass such
 * a buffer as bm_reduce's `out`: the kernel stores the result into host
 * memory and the separate device-to-host copy (collect, array.py:1012-1014)
 * disappears.
 */
int bm_host_writable(const void *p, size_t bytes, int *ok);

/*
 * bm_copy_strided -- dst[i] = src[i] over an N-d index space.
 *
 * The single data-movement primitive of the backend.  It replaces every
 * record-moving call site of the Spark path:
 *   - the ingest transpose + parallelize    bolt/spark/construct.py:55-69
 *   - ChunkedArray._chunk flatMap (pack)    bolt/spark/chunk.py:131-142
 *   - ChunkedArray.unchunk / removepad      bolt/spark/chunk.py:146-200, :514-550
 *   - keys_to_values partitionBy+_rebuild   bolt/spark/chunk.py:202-289
 *   - values_to_keys flatMap(_extract)      bolt/spark/chunk.py:291-347
 *   - Keys.transpose / Values.transpose     bolt/spark/shapes.py:66-89, :136-159
 *   - the multi-GPU swap's pack and unpack around the all-to-all
 *   - basic indexing, BoltArraySpark._getbasic  bolt/spark/array.py:480-512
 * Element i = (i_0..i_{n-1}) is read at src + sum(i_k*src_strides[k]) and
 * written at dst + sum(i_k*dst_strides[k]) (strides in elements; source
 * strides may be negative -- a reversed slice, BoltArraySpark.__getitem__
 * array.py:480-676 -- destination strides are >= 0; dst must not overlap
 * itself or src).
 * elem_bytes: any positive size (1/2/4/8/16 are native; others are moved
 * as bytes).  Data is moved bit-exactly.  ndim <= 24.
 */
int bm_copy_strided(const void *src, void *dst, int ndim, const int64_t *shape,
                    const int64_t *src_strides, const int64_t *dst_strides,
                    int elem_bytes, void *stream);

/*
 * bm_permute -- dst = ascontiguousarray(src.transpose(perm)) for a
 * C-contiguous src of `shape`.  This is BoltArraySpark.swap
 * (bolt/spark/array.py:716-763) and .transpose / .T / .swapaxes
 * (array.py:765-833) collapsed into their net permutation; one kernel,
 * bit-exact for every dtype.
 */
int bm_permute(const void *src, void *dst, int ndim, const int64_t *shape,
               const int32_t *perm, int elem_bytes, void *stream);

/*
 * bm_gather_rows -- dst[a, j, :] = src[a, idx[j], :] for a C-contiguous src
 * viewed as [n_outer][src_rows][row_bytes]; dst is [n_outer][n_idx][row_bytes].
 * idx is a DEVICE array of n_idx int64 row numbers in [0, src_rows) (the host
 * checks bounds, as BoltArraySpark.__getitem__ does, array.py:652-659).
 * The non-strided selections of __getitem__ (bolt/spark/array.py:514-593):
 *   _getmixed    one index list on one axis (x.take(idx, axis)),
 *   _getadvanced one list per axis -> a point gather (row = one element).
 * Bit-exact for every dtype.
 */
int bm_gather_rows(const void *src, void *dst, int64_t n_outer, int64_t src_rows,
                   int64_t row_bytes, const int64_t *idx, int64_t n_idx, void *stream);

/*
 * bm_record_gather -- dst[r*dst_rec + o] = src[r*src_rec + map[o]] for
 * r < nrec, o < dst_rec (sizes in elements of elem_bytes = 1/2/4/8).
 * map is a DEVICE array of dst_rec int32 indices in [0, src_rec), shared by
 * every record.  The pack and unpack of ChunkedArray for small records:
 *   pack   ChunkedArray._chunk flatMap     bolt/spark/chunk.py:131-142
 *          (map: packed chunk element -> dense value index, halos included)
 *   unpack ChunkedArray.unchunk/removepad  bolt/spark/chunk.py:146-200, :514-550
 *          (map: dense value index -> packed element of its chunk's core)
 * A source record of <= 64 KiB is staged whole in LDS; bit-exact.
 * parts (HOST array, nparts <= 8; nparts 0 or 1 = the whole record): the
 * destination record split into ranges, part p = {dlo, dhi, slo, shi}:
 * dst[dlo, dhi) reads only src[slo, shi) (every map entry of the range lies
 * there; the caller guarantees it), staged alone -- a smaller LDS tile.  The
 * ranges must tile [0, dst_rec) in order.
 */
int bm_record_gather(const void *src, void *dst, int64_t nrec, int64_t src_rec,
                     int64_t dst_rec, const int32_t *map, int nparts,
                     const int64_t *parts, int elem_bytes, void *stream);

/*
 * Reductions over a C-contiguous array viewed as [O][R][I]: the middle axis
 * (R records) is reduced, O*I outputs are produced in [O][I] order.  This is
 * the aligned layout that BoltArraySpark._align (array.py:85-115) builds
 * before StatCounter / treeReduce run (array.py:269, :321-323).
 *
 * Arithmetic: floating inputs and every mean/var/std accumulate in float64
 * (pivot-shifted sums per lane, Chan combination across lanes, waves,
 * blocks and chunks in a fixed order: deterministic) and round once to
 * out_dtype.  SUM over integer dtypes is modular in the input width
 * (numpy add of same-dtype arrays wraps: the reference's treeReduce(add));
 * SUM over BM_BOOL is logical OR (numpy bool add).  MAX / MIN compare in the
 * input dtype with numpy.maximum / numpy.minimum semantics (a NaN wins).
 * out_dtype: BM_F16/BM_F32/BM_F64 for MEAN/VAR/STD; in_dtype for SUM/MAX/MIN.
 * Population variance (M2/n), std = sqrt(var), as statcounter.py:119-130.
 */
int bm_reduce_workspace_bytes(int stat, int in_dtype, int64_t O, int64_t R,
                              int64_t I, size_t *bytes);

int bm_reduce(int stat, const void *src, int in_dtype, int64_t O, int64_t R,
              int64_t I, void *out, int out_dtype, void *workspace,
              size_t workspace_bytes, void *stream);

/*
 * Partial reduction state for the multi-GPU merge (the per-partition
 * StatCounter of array.py:321-322).  `state` receives, for O*I outputs:
 *   MEAN/VAR/STD: two float64 planes, mean[O*I] then M2[O*I] (count = R);
 *   SUM float:    one float64 plane (the sum);
 *   SUM int/bool: one uint64 plane (modular sum / OR);
 *   MAX / MIN:    one uint64 plane holding the element's bits.
 * bm_reduce_state_bytes gives the state size in bytes.
 */
int bm_reduce_state_bytes(int stat, int in_dtype, int64_t nout, size_t *bytes);

int bm_reduce_state(int stat, const void *src, int in_dtype, int64_t O,
                    int64_t R, int64_t I, void *state, void *workspace,
                    size_t workspace_bytes, void *stream);

/*
 * Combine nparts states (laid out back to back, part-major) in part order
 * -- the StatCounter.combine tree of statcounter.py:67-99 / treeReduce of
 * array.py:323, made deterministic -- and finalise into out[nout].
 * counts: host array of nparts record counts (parts with count 0 are
 * skipped).  nparts <= 64.
 */
int bm_reduce_combine(int stat, int in_dtype, const void *states,
                      const int64_t *counts, int nparts, int64_t nout,
                      void *out, int out_dtype, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* BOLT_MI355X_H */

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
#define BM_E_COMM (-4)   /* communicator failed: async RCCL error, timeout or abort */

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
/* reduce(func) with a numpy ufunc, array.py:243-282 (treeReduce(func)) */
#define BM_STAT_PROD 6   /* numpy.multiply / operator.mul (bool: logical and)   */
#define BM_STAT_LAND 7   /* numpy.logical_and -> bool                           */
#define BM_STAT_LOR 8    /* numpy.logical_or  -> bool                           */
#define BM_STAT_BAND 9   /* numpy.bitwise_and / operator.and_ (int, bool)       */
#define BM_STAT_BOR 10   /* numpy.bitwise_or  / operator.or_  (int, bool)       */
#define BM_STAT_BXOR 11  /* numpy.bitwise_xor / operator.xor  (int, bool)       */
#define BM_STAT_FMAX 12  /* numpy.fmax (NaN ignored unless all NaN)             */
#define BM_STAT_FMIN 13  /* numpy.fmin                                          */

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
 * (combined across lanes, waves, blocks and chunks in a fixed order:
 * deterministic) and round once to out_dtype.  SUM over integer dtypes is modular in the input width
 * (numpy add of same-dtype arrays wraps: the reference's treeReduce(add));
 * SUM over BM_BOOL is logical OR (numpy bool add).  MAX / MIN compare in the
 * input dtype with numpy.maximum / numpy.minimum semantics (a NaN wins),
 * FMAX / FMIN with numpy.fmax / numpy.fmin (a NaN loses).  PROD over floats
 * accumulates in float64, over integers is modular in the input width, over
 * BM_BOOL is logical AND.  LAND / LOR test x != 0 and write BM_BOOL;
 * BAND / BOR / BXOR act on the element bits (integer and bool dtypes only).
 * out_dtype: BM_F16/BM_F32/BM_F64 for MEAN/VAR/STD and float SUM/PROD;
 * BM_BOOL for LAND/LOR; in_dtype otherwise.
 * var / std: batched Welford -- each lane reduces a batch of up to 32 values
 * around a pivot drawn from the batch, merged by Chan's formula
 * (statcounter.py:51-59, :85-96) -- so the relative error of M2 stays
 * O(32 eps) whatever the offset or outliers of the data.
 * Population variance (M2/n), std = sqrt(var), as statcounter.py:119-130.
 */
/*
 * bm_record_gather_masked -- bm_record_gather whose (record, part) tiles
 * stage only the 16-B units of their source range that the map reads:
 * stage_mask (DEVICE, nparts x mask_words uint32) has bit k of part p set
 * when unit k (bytes [16k, 16k + 16) from the part's slo) holds an element
 * the part's map entries name.  values_to_keys drops the moved axis' halo
 * rows, which then stay in HBM (bolt/spark/chunk.py:291-347, removepad
 * :514-550).  A NULL mask stages everything (= bm_record_gather).
 */
int bm_record_gather_masked(const void *src, void *dst, int64_t nrec, int64_t src_rec,
                            int64_t dst_rec, const int32_t *map, int nparts,
                            const int64_t *parts, const uint32_t *stage_mask,
                            int mask_words, int elem_bytes, void *stream);

/*
 * bm_record_scatter -- the packed -> packed moves whose source record is read
 * whole, as one stream: for record r < nrec (src_rec elements each, records
 * contiguous) and element p,
 *     dst[(r / group) * dst_group_stride + map_a[p] + (r % group) * map_b[p]]
 *         = src[r * src_rec + p]                    (map_a[p] < 0: dropped)
 * map_a / map_b: DEVICE int32 arrays of src_rec entries (map_b may be NULL:
 * 0).  Replaces, for small records,
 *   - keys_to_values of the trailing keys (group = their extent, map_b = the
 *     chunk box sizes)                     bolt/spark/chunk.py:202-289
 *   - values_to_keys (group 1)             bolt/spark/chunk.py:291-347
 *   - unchunk, padding dropped (group 1)   bolt/spark/chunk.py:146-200
 * vec: elements per vector (power of two, vec * elem_bytes <= 16); the caller
 * guarantees every aligned vec-group of source elements is dropped whole or
 * lands on vec consecutive, vec-aligned destinations.  Bit-exact.
 */
int bm_record_scatter(const void *src, void *dst, int64_t nrec, int64_t src_rec,
                      int64_t group, int64_t dst_group_stride, const int32_t *map_a,
                      const int32_t *map_b, int vec, int elem_bytes, void *stream);

/*
 * bm_record_runs -- bm_record_scatter's moves when every source record is a
 * few long runs (no maps): run b of record r = g * group + k is copied whole,
 *     dst[g * dst_group_stride + a_b + k * m_b + j] = src[r * src_rec + s_b + j]
 * for j < len_b.  runs: DEVICE int64 array [s_b, len_b, a_b, m_b] x nruns,
 * in units of vec_bytes-byte vectors (vec_bytes a power of two in
 * [elem_bytes, 16] dividing every record, stride and run; the caller checks
 * the runs lie inside the records and the destination).  src_rec and
 * dst_group_stride are in elements; nrec must be a multiple of group.
 * flags: BM_RUNS_TILED when the runs tile every new record (m_b = len_b and
 * the regions [a_b, a_b + group * len_b), sorted by a_b, lie back to back
 * from 0 to dst_group_stride; at most 64 runs): the kernel then walks the
 * destination in order, whole lines per wave, each lane finding its source;
 * the flag on runs that do not tile gives wrong bytes (every read stays inside
 * a run of a source record of the group, the runs themselves inside the
 * records as above).  Without the flag: one wave per (record, run).
 * C5's keys_to_values((2,)): 16 chunk boxes of 2.6-3.2 KB per record
 * (bolt/spark/chunk.py:202-289).  Bit-exact.
 */
#define BM_RUNS_TILED 1
int bm_record_runs(const void *src, void *dst, int64_t nrec, int64_t src_rec,
                   int64_t group, int64_t dst_group_stride, int nruns,
                   const int64_t *runs, int vec_bytes, int flags, int elem_bytes,
                   void *stream);

int bm_reduce_workspace_bytes(int stat, int in_dtype, int64_t O, int64_t R,
                              int64_t I, size_t *bytes);

int bm_reduce(int stat, const void *src, int in_dtype, int64_t O, int64_t R,
              int64_t I, void *out, int out_dtype, void *workspace,
              size_t workspace_bytes, void *stream);

/*
 * bm_reduce over rows of a padded layout (I = 1): row o is the R elements at
 * src + o * row_pitch (row_pitch >= R, in elements; the pad is never read).
 * The per-record statistics of a transposed result -- mean / std over the
 * time axis after swap((0,),(0,1)), bolt/spark/array.py:284-334 over
 * statcounter.py -- when the swap wrote its rows at a line-aligned pitch
 * (a row of 2000 float32 at 8000 B starts 64 B into a line every other row;
 * padded to 8192 B the transpose and this read both run whole lines).
 * Results identical to bm_reduce on the compacted rows when row_pitch keeps
 * the rows' 16-B vector width (a pitch in whole vectors: every padded layout
 * the array makes; other pitches read narrower vectors, another summation
 * order); the same workspace (bm_reduce_workspace_bytes with I = 1 covers
 * every pitch).
 */
int bm_reduce_rows(int stat, const void *src, int in_dtype, int64_t O, int64_t R,
                   int64_t row_pitch, void *out, int out_dtype, void *workspace,
                   size_t workspace_bytes, void *stream);

/*
 * Partial reduction state for the multi-GPU merge (the per-partition
 * StatCounter of array.py:321-322).  `state` receives, for O*I outputs:
 *   MEAN/VAR/STD: two float64 planes, mean[O*I] then M2[O*I] (count = R);
 *   SUM / PROD float: one float64 plane (the sum / product);
 *   SUM / PROD int/bool, LAND / LOR / BAND / BOR / BXOR: one uint64 plane;
 *   MAX / MIN / FMAX / FMIN: one uint64 plane holding the element's bits.
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
 * skipped).  nparts <= 256.
 */
int bm_reduce_combine(int stat, int in_dtype, const void *states,
                      const int64_t *counts, int nparts, int64_t nout,
                      void *out, int out_dtype, void *stream);

/*
 * ---------------------------------------------------------------------------
 * Multi-GPU record exchange over RCCL (xGMI), one process per GPU.
 *
 * These replace the Spark shuffles that move records between executors:
 *   keys_to_values' partitionBy + _rebuild   bolt/spark/chunk.py:251-261
 *   unchunk's partitionBy (shuffle #2)       bolt/spark/chunk.py:179-191
 * (and so the swap / transpose that run through them, array.py:716-808), and
 * the driver-side merge of per-partition statistics partials
 * (treeReduce of StatCounter.combine, array.py:321-323).
 * RCCL is bound at run time (dlopen): the librccl already in the process
 * (PyTorch-ROCm's) is reused, else the system librccl.so.1.  All transfers
 * are stream-ordered on `stream`; no call blocks the host on the transfer.
 * Buffers are device memory owned by the caller; sizes and offsets in BYTES.
 */
#define BM_COMM_ID_BYTES 128   /* sizeof(ncclUniqueId) */

/* Rank 0 creates the communicator id (BM_COMM_ID_BYTES) and sends it to the
 * other ranks out of band (bolt_amd sends it through the torch.distributed
 * rendezvous store). */
int bm_comm_unique_id(void *id, size_t bytes);

/* Collective over `world` ranks: every rank calls it with the same id and
 * its own rank, with its GPU current.  *comm receives an opaque handle. */
int bm_comm_init(void **comm, int world, const void *id, int rank);

/* Release a communicator (NULL is a no-op). */
int bm_comm_destroy(void *comm);

/* rank / world of a communicator and the path of the RCCL library in use
 * (lib may be NULL). */
int bm_comm_info(void *comm, int *rank, int *world, char *lib, size_t lib_bytes);

/*
 * bm_alltoallv -- block q of send (send_bytes[q] bytes at send_offs[q]) goes
 * to rank q; block s of recv (recv_bytes[s] at recv_offs[s]) arrives from rank
 * s.  The self block is a local device copy on `stream` (send_bytes[rank]
 * must equal recv_bytes[rank], else BM_E_ARG); the peers are one RCCL group of
 * ncclSend / ncclRecv pairs, every peer at once (each ordered GPU pair has its
 * own xGMI link).  The multi-GPU swap's exchange step (pack -> bm_alltoallv ->
 * unpack).  Arrays have `world` entries; send_bytes[q] must equal what rank q
 * expects (a mismatch across ranks is caught by bm_comm_wait's timeout).
 * BM_E_COMM if the communicator has failed or been aborted.
 */
int bm_alltoallv(void *comm, const void *send, const int64_t *send_bytes,
                 const int64_t *send_offs, void *recv, const int64_t *recv_bytes,
                 const int64_t *recv_offs, void *stream);

/*
 * bm_allgatherv -- rank s's send_bytes (its `send`) land at recv_offs[s] of
 * every rank's recv (recv_bytes[s] = rank s's send_bytes).  Uniform sizes at
 * packed offsets use ncclAllGather, others one group of point-to-point pairs.
 * Statistics states before bm_reduce_combine, and output slabs of reductions
 * that keep the sharded axis.
 */
int bm_allgatherv(void *comm, const void *send, int64_t send_bytes, void *recv,
                  const int64_t *recv_bytes, const int64_t *recv_offs, void *stream);

/*
 * bm_comm_wait -- block the host until all work queued on `stream` is done,
 * polling RCCL's asynchronous error meanwhile.  On an RCCL error, or when the
 * work is not done after timeout_s seconds (<= 0: no limit), the communicator
 * is aborted (ncclCommAbort: its kernels exit and the stream drains) and
 * BM_E_COMM is returned with the reason in bm_last_error() -- a lost or
 * mismatched peer becomes an error, not a hang.  This is how a failed Spark
 * shuffle (chunk.py:251-261) surfaces: as an exception on the driver.
 */
int bm_comm_wait(void *comm, void *stream, double timeout_s);

/* Non-blocking: BM_OK, or BM_E_COMM (communicator aborted) after an
 * asynchronous RCCL error or an earlier abort. */
int bm_comm_check(void *comm);

/* Abort now: pending exchanges stop, later calls return BM_E_COMM.
 * bm_comm_destroy still releases the handle. */
int bm_comm_abort(void *comm);

#ifdef __cplusplus
}
#endif

#endif /* BOLT_MI355X_H */

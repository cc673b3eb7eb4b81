// bm_comm.hip -- RCCL communicators and the record exchanges of libbolt_mi355x.
//
// Replaces the Spark shuffles that move records between executors:
//   keys_to_values partitionBy          bolt/spark/chunk.py:251-261 (shuffle #1)
//   unchunk partitionBy                 bolt/spark/chunk.py:179-191 (shuffle #2)
//   collect of statistics partials      bolt/spark/array.py:321-323 (treeReduce)
// with RCCL point-to-point transfers over xGMI, one process per GPU.  Every
// ordered GPU pair of an MI355X node has its own xGMI link, so the exchange is
// a group of ncclSend / ncclRecv, one pair per peer, which RCCL runs
// concurrently on all links (no ring).
//
// RCCL is bound at run time: the library already in the process is used
// (PyTorch-ROCm loads its own librccl, and one RCCL instance per process keeps
// a single view of the devices); otherwise the system librccl.so.1.  Nothing
// links RCCL at build time, so the rest of the library loads without it.
#include "bm_common.h"
#include "../../include/bolt_mi355x.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>

namespace {

struct Rccl {
  void *handle = nullptr;
  decltype(&ncclGetUniqueId) getUniqueId = nullptr;
  decltype(&ncclCommInitRank) commInitRank = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclCommAbort) commAbort = nullptr;
  decltype(&ncclCommGetAsyncError) commGetAsyncError = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclAllGather) allGather = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  decltype(&ncclGetVersion) getVersion = nullptr;
  char where[512] = "";
};

Rccl g_rccl;
std::once_flag g_rccl_once;
int g_rccl_rc = BM_E_HIP;

template <typename F> bool bind(void *h, const char *name, F &f) {
  f = reinterpret_cast<F>(dlsym(h, name));
  return f != nullptr;
}

void load_rccl() {
  // 1) an RCCL already loaded in this process (PyTorch's), 2) an explicit
  // override, 3) the system library.
  const char *env = std::getenv("BOLT_AMD_RCCL");
  const char *resident[] = {"librccl.so", "librccl.so.1"};
  void *h = nullptr;
  const char *name = nullptr;
  if (env && *env) {
    h = dlopen(env, RTLD_NOW | RTLD_LOCAL);
    name = env;
  }
  for (const char *n : resident) {
    if (h) break;
    h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
    name = n;
  }
  if (!h) {
    h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    name = "librccl.so.1";
  }
  if (!h) {
    h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    name = "/opt/rocm/lib/librccl.so.1";
  }
  if (!h) {
    bm_set_error("RCCL not found (librccl.so / librccl.so.1): %s", dlerror());
    g_rccl_rc = BM_E_HIP;
    return;
  }
  Rccl r;
  r.handle = h;
  const bool ok = bind(h, "ncclGetUniqueId", r.getUniqueId) && bind(h, "ncclCommInitRank", r.commInitRank) &&
                  bind(h, "ncclCommDestroy", r.commDestroy) && bind(h, "ncclCommAbort", r.commAbort) &&
                  bind(h, "ncclCommGetAsyncError", r.commGetAsyncError) &&
                  bind(h, "ncclGroupStart", r.groupStart) && bind(h, "ncclGroupEnd", r.groupEnd) &&
                  bind(h, "ncclSend", r.send) && bind(h, "ncclRecv", r.recv) &&
                  bind(h, "ncclAllGather", r.allGather) && bind(h, "ncclGetErrorString", r.errorString) &&
                  bind(h, "ncclGetVersion", r.getVersion);
  if (!ok) {
    bm_set_error("RCCL at %s lacks a required symbol", name);
    g_rccl_rc = BM_E_HIP;
    return;
  }
  Dl_info info;
  if (dladdr(reinterpret_cast<void *>(r.getUniqueId), &info) && info.dli_fname)
    std::snprintf(r.where, sizeof(r.where), "%s", info.dli_fname);
  g_rccl = r;
  g_rccl_rc = BM_OK;
}

int rccl(const char *who) {
  std::call_once(g_rccl_once, load_rccl);
  if (g_rccl_rc != BM_OK) {
    const std::string msg = bm_last_error();
    bm_set_error("%s: %s", who, msg.c_str());
  }
  return g_rccl_rc;
}

int nccl_check(ncclResult_t r, const char *who, const char *what) {
  if (r == ncclSuccess) return BM_OK;
  bm_set_error("%s: %s failed: %s", who, what, g_rccl.errorString ? g_rccl.errorString(r) : "?");
  return BM_E_HIP;
}

struct Comm {
  ncclComm_t comm;
  int rank, world;
  bool aborted;      // ncclCommAbort has run: the handle is gone, every call fails
  char why[256];     // what aborted it
};

// The communicator after a failure: abort it once (RCCL kernels still in
// flight see the abort flag and exit, so streams drain instead of hanging)
// and remember why.
int comm_fail(Comm *c, const char *who, const char *why) {
  if (!c->aborted) {
    c->aborted = true;
    std::snprintf(c->why, sizeof(c->why), "%s", why);
    if (g_rccl.commAbort) g_rccl.commAbort(c->comm);
  }
  bm_set_error("%s: communicator aborted: %s", who, c->why);
  return BM_E_COMM;
}

// BM_OK, or abort + BM_E_COMM when the communicator is already aborted or
// RCCL reports an asynchronous error (a peer that died, a transport failure).
int comm_health(Comm *c, const char *who) {
  if (c->aborted) {
    bm_set_error("%s: communicator aborted earlier: %s", who, c->why);
    return BM_E_COMM;
  }
  ncclResult_t async = ncclSuccess;
  const ncclResult_t r = g_rccl.commGetAsyncError(c->comm, &async);
  if (r != ncclSuccess || (async != ncclSuccess && async != ncclInProgress)) {
    char why[200];
    std::snprintf(why, sizeof(why), "RCCL asynchronous error: %s",
                  g_rccl.errorString(r != ncclSuccess ? r : async));
    return comm_fail(c, who, why);
  }
  return BM_OK;
}

}  // namespace

extern "C" int bm_comm_unique_id(void *id, size_t bytes) {
  if (!id || bytes < BM_COMM_ID_BYTES) {
    bm_set_error("bm_comm_unique_id: need a %d-byte buffer", BM_COMM_ID_BYTES);
    return BM_E_ARG;
  }
  if (int rc = rccl("bm_comm_unique_id")) return rc;
  static_assert(sizeof(ncclUniqueId) == BM_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId uid;
  if (int rc = nccl_check(g_rccl.getUniqueId(&uid), "bm_comm_unique_id", "ncclGetUniqueId")) return rc;
  std::memcpy(id, &uid, sizeof(uid));
  return BM_OK;
}

extern "C" int bm_comm_init(void **comm, int world, const void *id, int rank) {
  if (!comm || !id || world < 1 || rank < 0 || rank >= world) {
    bm_set_error("bm_comm_init: bad arguments (world %d, rank %d)", world, rank);
    return BM_E_ARG;
  }
  *comm = nullptr;
  if (int rc = rccl("bm_comm_init")) return rc;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  Comm *c = new (std::nothrow) Comm{};
  if (!c) {
    bm_set_error("bm_comm_init: out of host memory");
    return BM_E_ARG;
  }
  c->rank = rank;
  c->world = world;
  if (int rc = nccl_check(g_rccl.commInitRank(&c->comm, world, uid, rank), "bm_comm_init", "ncclCommInitRank")) {
    delete c;
    return rc;
  }
  *comm = c;
  return BM_OK;
}

extern "C" int bm_comm_destroy(void *comm) {
  if (!comm) return BM_OK;
  Comm *c = static_cast<Comm *>(comm);
  int rc = BM_OK;
  if (!c->aborted && rccl("bm_comm_destroy") == BM_OK)  // (an aborted handle is already released)
    rc = nccl_check(g_rccl.commDestroy(c->comm), "bm_comm_destroy", "ncclCommDestroy");
  delete c;
  return rc;
}

extern "C" int bm_comm_info(void *comm, int *rank, int *world, char *lib, size_t lib_bytes) {
  if (!comm) {
    bm_set_error("bm_comm_info: null communicator");
    return BM_E_ARG;
  }
  const Comm *c = static_cast<const Comm *>(comm);
  if (rank) *rank = c->rank;
  if (world) *world = c->world;
  if (lib && lib_bytes) std::snprintf(lib, lib_bytes, "%s", g_rccl.where);
  return BM_OK;
}

// Variable-size all-to-all of byte blocks: block q of `send` (send_bytes[q]
// at send_offs[q]) goes to rank q; block s of `recv` (recv_bytes[s] at
// recv_offs[s]) comes from rank s.  The self block is a local device copy on
// `stream`; the peers are one RCCL group of point-to-point pairs, all
// stream-ordered on `stream`.
extern "C" int bm_alltoallv(void *comm, const void *send, const int64_t *send_bytes,
                            const int64_t *send_offs, void *recv, const int64_t *recv_bytes,
                            const int64_t *recv_offs, void *stream) {
  if (!comm || !send_bytes || !send_offs || !recv_bytes || !recv_offs) {
    bm_set_error("bm_alltoallv: null argument");
    return BM_E_ARG;
  }
  Comm *c = static_cast<Comm *>(comm);
  for (int q = 0; q < c->world; ++q) {
    if (send_bytes[q] < 0 || recv_bytes[q] < 0 || send_offs[q] < 0 || recv_offs[q] < 0 ||
        (send_bytes[q] && !send) || (recv_bytes[q] && !recv)) {
      bm_set_error("bm_alltoallv: bad block %d (send %lld at %lld, recv %lld at %lld)", q,
                   (long long)send_bytes[q], (long long)send_offs[q], (long long)recv_bytes[q],
                   (long long)recv_offs[q]);
      return BM_E_ARG;
    }
  }
  const int me = c->rank;
  if (send_bytes[me] != recv_bytes[me]) {  // the one pairing this rank can check alone
    bm_set_error("bm_alltoallv: self block mismatch (sends %lld bytes to itself, expects %lld)",
                 (long long)send_bytes[me], (long long)recv_bytes[me]);
    return BM_E_ARG;
  }
  if (int rc = rccl("bm_alltoallv")) return rc;
  if (int rc = comm_health(c, "bm_alltoallv")) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (send_bytes[me]) {
    const hipError_t e = hipMemcpyAsync(static_cast<char *>(recv) + recv_offs[me],
                                        static_cast<const char *>(send) + send_offs[me], (size_t)send_bytes[me],
                                        hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) {
      bm_set_error("bm_alltoallv: self-block copy failed: %s", hipGetErrorString(e));
      return BM_E_HIP;
    }
  }
  if (c->world == 1) return BM_OK;
  if (int rc = nccl_check(g_rccl.groupStart(), "bm_alltoallv", "ncclGroupStart")) return rc;
  int rc = BM_OK;
  for (int k = 1; k < c->world && rc == BM_OK; ++k) {
    // rank r pairs with r+k (send) and r-k (recv): every link busy at once
    const int to = (me + k) % c->world;
    const int from = (me - k + c->world) % c->world;
    if (send_bytes[to])
      rc = nccl_check(g_rccl.send(static_cast<const char *>(send) + send_offs[to], (size_t)send_bytes[to],
                                  ncclUint8, to, c->comm, st),
                      "bm_alltoallv", "ncclSend");
    if (rc == BM_OK && recv_bytes[from])
      rc = nccl_check(g_rccl.recv(static_cast<char *>(recv) + recv_offs[from], (size_t)recv_bytes[from],
                                  ncclUint8, from, c->comm, st),
                      "bm_alltoallv", "ncclRecv");
  }
  const int rc_end = nccl_check(g_rccl.groupEnd(), "bm_alltoallv", "ncclGroupEnd");
  return rc != BM_OK ? rc : rc_end;
}

// Every rank's block on every rank: rank s contributes recv_bytes[s] bytes
// (this rank's are `send`), landing at recv_offs[s].  Equal sizes at packed
// offsets take ncclAllGather; otherwise one group of point-to-point pairs.
extern "C" int bm_allgatherv(void *comm, const void *send, int64_t send_bytes, void *recv,
                             const int64_t *recv_bytes, const int64_t *recv_offs, void *stream) {
  if (!comm || !recv_bytes || !recv_offs || send_bytes < 0 || (send_bytes && !send)) {
    bm_set_error("bm_allgatherv: bad arguments");
    return BM_E_ARG;
  }
  Comm *c = static_cast<Comm *>(comm);
  if (recv_bytes[c->rank] != send_bytes) {
    bm_set_error("bm_allgatherv: send_bytes %lld != recv_bytes[rank] %lld", (long long)send_bytes,
                 (long long)recv_bytes[c->rank]);
    return BM_E_ARG;
  }
  bool uniform = true;
  for (int s = 0; s < c->world; ++s) {
    if (recv_bytes[s] < 0 || recv_offs[s] < 0 || (recv_bytes[s] && !recv)) {
      bm_set_error("bm_allgatherv: bad block %d", s);
      return BM_E_ARG;
    }
    uniform = uniform && recv_bytes[s] == send_bytes && recv_offs[s] == (int64_t)s * send_bytes;
  }
  if (int rc = rccl("bm_allgatherv")) return rc;
  if (int rc = comm_health(c, "bm_allgatherv")) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (uniform) {
    if (send_bytes == 0) return BM_OK;
    return nccl_check(g_rccl.allGather(send, recv, (size_t)send_bytes, ncclUint8, c->comm, st), "bm_allgatherv",
                      "ncclAllGather");
  }
  if (send_bytes) {  // own block: a local device copy
    const hipError_t e = hipMemcpyAsync(static_cast<char *>(recv) + recv_offs[c->rank], send, (size_t)send_bytes,
                                        hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) {
      bm_set_error("bm_allgatherv: own-block copy failed: %s", hipGetErrorString(e));
      return BM_E_HIP;
    }
  }
  if (c->world == 1) return BM_OK;
  if (int rc = nccl_check(g_rccl.groupStart(), "bm_allgatherv", "ncclGroupStart")) return rc;
  int rc = BM_OK;
  for (int k = 1; k < c->world && rc == BM_OK; ++k) {
    const int to = (c->rank + k) % c->world;
    const int from = (c->rank - k + c->world) % c->world;
    if (send_bytes)
      rc = nccl_check(g_rccl.send(send, (size_t)send_bytes, ncclUint8, to, c->comm, st), "bm_allgatherv", "ncclSend");
    if (rc == BM_OK && recv_bytes[from])
      rc = nccl_check(g_rccl.recv(static_cast<char *>(recv) + recv_offs[from], (size_t)recv_bytes[from], ncclUint8,
                                  from, c->comm, st),
                      "bm_allgatherv", "ncclRecv");
  }
  const int rc_end = nccl_check(g_rccl.groupEnd(), "bm_allgatherv", "ncclGroupEnd");
  return rc != BM_OK ? rc : rc_end;
}

// Host wait for everything queued on `stream` (the exchanges of this
// communicator and whatever precedes them), bounded: RCCL's asynchronous
// error is polled while waiting, and on an error or after timeout_s seconds
// the communicator is aborted -- its kernels exit, the stream drains -- and
// BM_E_COMM comes back instead of a hang (a peer that died or posted a
// mismatched exchange; the Spark shuffle it replaces, chunk.py:251-261,
// surfaces a lost executor as an exception the same way).
extern "C" int bm_comm_wait(void *comm, void *stream, double timeout_s) {
  if (!comm) {
    bm_set_error("bm_comm_wait: null communicator");
    return BM_E_ARG;
  }
  Comm *c = static_cast<Comm *>(comm);
  if (int rc = rccl("bm_comm_wait")) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  for (;;) {
    const hipError_t q = hipStreamQuery(st);
    if (q == hipSuccess) return c->aborted ? comm_health(c, "bm_comm_wait") : BM_OK;
    if (q != hipErrorNotReady) {
      bm_set_error("bm_comm_wait: hipStreamQuery: %s", hipGetErrorString(q));
      return BM_E_HIP;
    }
    if (int rc = comm_health(c, "bm_comm_wait")) {
      // aborted: RCCL's kernels exit; give the stream a bounded time to drain
      const auto ta = std::chrono::steady_clock::now();
      while (hipStreamQuery(st) == hipErrorNotReady &&
             std::chrono::steady_clock::now() - ta < std::chrono::seconds(10))
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      return rc;
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_s > 0 && el > timeout_s) {
      char why[200];
      std::snprintf(why, sizeof(why),
                    "exchange not complete after %.1f s (a peer rank failed, stalled or posted a mismatched "
                    "exchange)", el);
      comm_fail(c, "bm_comm_wait", why);
      const auto ta = std::chrono::steady_clock::now();
      while (hipStreamQuery(st) == hipErrorNotReady &&
             std::chrono::steady_clock::now() - ta < std::chrono::seconds(10))
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      return BM_E_COMM;
    }
    // spin briefly (exchanges of a few ms), then back off to 200 us polls
    if (++spins > 2000) std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

// Non-blocking health check: BM_OK, or BM_E_COMM (and the communicator
// aborted) after an asynchronous RCCL error or an earlier abort.
extern "C" int bm_comm_check(void *comm) {
  if (!comm) {
    bm_set_error("bm_comm_check: null communicator");
    return BM_E_ARG;
  }
  if (int rc = rccl("bm_comm_check")) return rc;
  return comm_health(static_cast<Comm *>(comm), "bm_comm_check");
}

// Abort a communicator now (ncclCommAbort): pending exchanges stop, every
// later call on it returns BM_E_COMM.  bm_comm_destroy still frees the handle.
extern "C" int bm_comm_abort(void *comm) {
  if (!comm) return BM_OK;
  if (int rc = rccl("bm_comm_abort")) return rc;
  comm_fail(static_cast<Comm *>(comm), "bm_comm_abort", "aborted by the caller");
  return BM_OK;
}

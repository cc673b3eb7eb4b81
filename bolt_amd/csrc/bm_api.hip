// bm_api.hip -- version, error channel and device queries of libbolt_mi355x.
#include "bm_common.h"
#include "../../include/bolt_mi355x.h"

#include <cstdarg>
#include <cstdio>

static thread_local char g_bm_err[1024] = "";

void bm_set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_bm_err, sizeof(g_bm_err), fmt, ap);
  va_end(ap);
}

extern "C" int bm_abi_version(void) { return BM_ABI_VERSION; }

extern "C" const char *bm_last_error(void) { return g_bm_err; }

extern "C" int bm_device_cus(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    bm_set_error("bm_device_cus: hipGetDevice failed");
    return BM_E_HIP;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    bm_set_error("bm_device_cus: hipDeviceGetAttribute failed");
    return BM_E_HIP;
  }
  return cus;
}

// 1 if [p, p + bytes) is page-locked host memory the current device can store
// to at the same address (ROCm maps hipHostMalloc'd memory into every GPU's
// address space), so a kernel can write a small result straight into it.
extern "C" int bm_host_writable(const void *p, size_t bytes, int *ok) {
  if (!ok) {
    bm_set_error("bm_host_writable: null result pointer");
    return BM_E_ARG;
  }
  *ok = 0;
  if (!p || bytes == 0) return BM_OK;
  const char *lo = static_cast<const char *>(p);
  for (const char *q : {lo, lo + bytes - 1}) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, q) != hipSuccess) {
      (void)hipGetLastError();  // unknown (pageable) memory: not writable, not an error
      return BM_OK;
    }
    if (a.type != hipMemoryTypeHost || a.devicePointer != (void *)q) return BM_OK;
  }
  *ok = 1;
  return BM_OK;
}

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

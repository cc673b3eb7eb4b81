// Dispatch-offset probe: an empty kernel of n blocks advances the dispatcher's
// round-robin over the 8 XCDs by n; block 0 of every launch records the XCD it
// ran on (HW_REG_XCC_ID), so a caller can steer which XCD the NEXT kernel's
// block 0 lands on and check that it did.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

__global__ void k_shift(int *out) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && out) out[0] = (int)xcc_id();
}

// every block writes its XCD id: out[b] for b < n
__global__ void k_xcd_map(int *out, int n) {
  if (threadIdx.x == 0 && (int)blockIdx.x < n) out[blockIdx.x] = (int)xcc_id();
}

extern "C" int xcd_shift(int blocks, int *out, hipStream_t st) {
  if (blocks <= 0) return 0;
  k_shift<<<blocks, 64, 0, st>>>(out);
  return (int)hipGetLastError();
}

extern "C" int xcd_map(int blocks, int *out, hipStream_t st) {
  if (blocks <= 0) return 0;
  k_xcd_map<<<blocks, 64, 0, st>>>(out, blocks);
  return (int)hipGetLastError();
}

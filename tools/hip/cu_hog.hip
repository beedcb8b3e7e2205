// Co-residency probe (tools/coresidency_probe.py; not part of the library): workgroups that sit
// on their CUs the way a persistent decode grid does -- resident, holding registers and LDS,
// mostly asleep -- until a release flag is set.  WAVES x 64 threads, every wave holding 256
// VGPRs (the clobber below), `lds` bytes of dynamic LDS; one workgroup per grid slot.
#include <hip/hip_runtime.h>

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void cu_hog_kernel(const int* flag, int* out) {
  extern __shared__ int s[];
  asm volatile("" ::: "v255");                      // the wave holds 256 VGPRs
  if (threadIdx.x == 0) s[0] = blockIdx.x;
  int seen = 0;
  for (int it = 0; it < (1 << 22); ++it) {         // exit after ~15 s whatever the flag
    seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (seen) break;
    __builtin_amdgcn_s_sleep(127);
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = seen + s[0];
}

extern "C" int cu_hog_launch(int waves, int blocks, int lds, const int* flag, int* out,
                             void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (waves == 8)
    hipLaunchKernelGGL(cu_hog_kernel<8>, dim3(blocks), dim3(512), lds, st, flag, out);
  else if (waves == 4)
    hipLaunchKernelGGL(cu_hog_kernel<4>, dim3(blocks), dim3(256), lds, st, flag, out);
  else
    return 1;
  return (int)hipGetLastError();
}

// XCC_ID of the XCD each workgroup runs on (hardware register), per workgroup
__global__ void xcc_probe_kernel(int* out) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) out[blockIdx.x] = (int)x;
}

extern "C" int xcc_probe(int blocks, int* out, void* stream) {
  hipLaunchKernelGGL(xcc_probe_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, out);
  return (int)hipGetLastError();
}

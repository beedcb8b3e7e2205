// Dispatch-cost probe: back-to-back dependent kernels on one stream, eager and hipGraph-captured,
// at several grid sizes, with an empty body and with a 1-KB-per-block read + write body.
// Build: hipcc --offload-arch=gfx950 -O3 launch_bench.hip -o launch_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void empty_kernel(float* p) {
  if (p == nullptr && threadIdx.x == 1234567) p[0] = 0.f;
}
__global__ void touch_kernel(float* __restrict__ p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 1.0001f + 1.f;
}

int main() {
  float* buf;
  CK(hipMalloc(&buf, 64 << 20));
  CK(hipMemset(buf, 0, 64 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 200;
  for (int body = 0; body < 2; ++body) {
    for (int grid : {1, 16, 256, 1024}) {
      auto enqueue = [&]() {
        for (int i = 0; i < reps; ++i) {
          if (body == 0) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, s, buf);
          else hipLaunchKernelGGL(touch_kernel, dim3(grid), dim3(256), 0, s, buf, grid * 256);
        }
      };
      // eager
      enqueue();
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      enqueue();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms_e;
      CK(hipEventElapsedTime(&ms_e, e0, e1));
      // graph
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      enqueue();
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms_g;
      CK(hipEventElapsedTime(&ms_g, e0, e1));
      printf("%s grid %5d: eager %6.2f us/kernel, graph %6.2f us/kernel\n",
             body ? "touch" : "empty", grid, ms_e * 1e3 / reps, ms_g * 1e3 / (5 * reps));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}

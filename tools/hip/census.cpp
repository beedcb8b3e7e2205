// Residency census for persistent grids: K concurrent launches (one per stream) of G workgroups
// of 512 threads with ~110 KB of LDS and 256 VGPRs (the decode_persist_kernel footprint).  Every
// workgroup records its XCC / SE / CU (s_getreg HW_ID) and spins (bounded) until all K x G have
// arrived; prints how many became co-resident and the per-(XCC, SE) histogram.
//   census G K
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <map>

__global__ __launch_bounds__(512) void census(unsigned* cnt, int* ids, int total, int base) {
  __shared__ char pad[110 * 1024];
  volatile char* vp = pad;
  if (threadIdx.x == 0) {
    vp[blockIdx.x] = 1;
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    ids[base + blockIdx.x] = (int)((xcc & 0xf) << 16 | hw >> 8);
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned i = 0; i < (1u << 20); ++i) {
      if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)total) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (threadIdx.x == 1 && vp[blockIdx.x] != 1) ids[0] = -1;
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 48, K = argc > 2 ? atoi(argv[2]) : 5;
  unsigned* cnt; int* ids;
  hipMalloc(&cnt, 4); hipMalloc(&ids, 4 * G * K);
  hipMemset(cnt, 0, 4); hipMemset(ids, 0xff, 4 * G * K);
  std::vector<hipStream_t> st(K);
  for (auto& s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int k = 0; k < K; ++k) hipLaunchKernelGGL(census, dim3(G), dim3(512), 0, st[k], cnt, ids, G * K, G * k);
  hipDeviceSynchronize();
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<int> h(G * K); unsigned c;
  hipMemcpy(h.data(), ids, 4 * G * K, hipMemcpyDeviceToHost); hipMemcpy(&c, cnt, 4, hipMemcpyDeviceToHost);
  std::map<int, int> xse; std::map<int, int> cu;
  for (int v : h) { int xcc = v >> 16, se = (v >> 5) & 3, cuid = v & 0x1f; xse[xcc * 10 + se]++; cu[v]++; }
  int dup = 0; for (auto& p : cu) if (p.second > 1) dup++;
  printf("G=%d K=%d: %.2f ms (all co-resident would be ~ms; serialised ~%d x spin)  distinct CUs %zu, CUs with >1 WG %d\n",
         G, K, ms, K, cu.size(), dup);
  for (auto& p : xse) printf("xcc%d.se%d:%d ", p.first / 10, p.first % 10, p.second);
  printf("\n");
  return 0;
}

// Diagnostic: where a row-group GEMM launch (csrc/gemm_rows.hip built with -DZS_STAMPS) spends
// its time.  Each workgroup's thread 0 stamps s_memrealtime (100 MHz) at: entry (0), all loads
// issued (1), all loads landed (2), LN done + barrier (3), MFMAs + partials in LDS (4), partials
// barrier (5), output stored (6).  The stamped build waits for every load before phase 2, so its
// run time is not the real kernel's: read the shares, not the length.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DZS_STAMPS \
//     zero-shot-aac_amd/csrc/gemm_rows.hip zero-shot-aac_amd/csrc/runtime.cpp \
//     tools/hip/rows_stamps.cpp -o tools/hip/rows_stamps
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

extern "C" int zs_set_stamp_buf(void* p);

extern "C" int zs_gemm_ln(int M, int N, int K, const float* x, int ldx, const float* ln_w,
                          const float* ln_b, float eps, const void* W, int ldw, const float* bias,
                          const float* residual, int ldr, void* out, int ldo, int out_dtype,
                          int act, void* stream);
extern "C" int zs_gemm_rows_internal(int M, int N, int K, const void* A, int lda, const void* W,
                                     int ldw, const float* bias, const float* residual, int ldr,
                                     void* out, int ldo, int out_dtype, int act, void* stream);

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[v.size() / 2];
}

int main() {
  const int M = 64, K = 768;
  const int ncopy = 64;
  float *x, *lw, *lb, *bias, *outf;
  void *W, *out, *A;
  unsigned long long* st;
  CK(hipMalloc(&x, M * 3072 * 4));
  CK(hipMalloc(&lw, 3072 * 4));
  CK(hipMalloc(&lb, 3072 * 4));
  CK(hipMalloc(&bias, 3072 * 4));
  CK(hipMalloc(&outf, M * 3072 * 4));
  CK(hipMalloc(&out, M * 3072 * 2));
  CK(hipMalloc(&A, M * 3072 * 2));
  const size_t wbytes = (size_t)3072 * 768 * 2;
  CK(hipMalloc(&W, wbytes * ncopy));
  CK(hipMemset(x, 0, M * 3072 * 4));
  CK(hipMemset(lw, 0, 3072 * 4));
  CK(hipMemset(lb, 0, 3072 * 4));
  CK(hipMemset(bias, 0, 3072 * 4));
  CK(hipMemset(A, 0, M * 3072 * 2));
  CK(hipMemset(W, 0, wbytes * ncopy));
  CK(hipMalloc(&st, 4096 * 8 * 8));
  if (zs_set_stamp_buf(st)) { printf("stamp buffer\n"); return 1; }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  struct Case { const char* name; int ln, N, K, out_bf16, act; };
  const Case cases[] = {{"ln  c_fc  64x768x3072 gelu", 1, 3072, 768, 1, 2},
                        {"ln  c_attn 64x768x2304", 1, 2304, 768, 1, 0},
                        {"    proj  64x768x768 +res", 0, 768, 768, 0, 0},
                        {"    mproj 64x3072x768 +res", 0, 768, 3072, 0, 0}};
  for (const Case& c : cases) {
    std::vector<double> d[7], span, skew;
    for (int it = 0; it < 40; ++it) {
      const void* w = (const char*)W + (size_t)(it % ncopy) * wbytes;   // cold weights
      CK(hipMemsetAsync(st, 0, 4096 * 8 * 8, s));
      int rc = c.ln ? zs_gemm_ln(M, c.N, c.K, x, c.K, lw, lb, 1e-5f, w, c.K, bias, nullptr, 0,
                                 out, c.N, 1, c.act, s)
                    : zs_gemm_rows_internal(M, c.N, c.K, A, c.K, w, c.K, bias, outf, c.N, outf,
                                            c.N, 0, 0, s);
      if (rc) { printf("launch rc %d\n", rc); return 1; }
      CK(hipStreamSynchronize(s));
      if (it < 5) continue;
      std::vector<unsigned long long> h(4096 * 8);
      CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
      unsigned long long t0 = ~0ull, t1 = 0;
      int nwg = 0;
      for (int b = 0; b < 4096; ++b) {
        const unsigned long long* t = &h[b * 8];
        if (!t[0]) continue;
        ++nwg;
        t0 = std::min(t0, t[0]);
        t1 = std::max(t1, t[6] ? t[6] : t[5]);
        for (int k = 1; k < 7; ++k)
          if (t[k] && t[k - 1]) d[k].push_back((t[k] - t[k - 1]) * 10.0 / 1000.0);   // us
      }
      std::vector<double> starts;
      for (int b = 0; b < 4096; ++b) if (h[b * 8]) starts.push_back((h[b * 8] - t0) * 0.01);
      span.push_back((t1 - t0) * 0.01);
      skew.push_back(*std::max_element(starts.begin(), starts.end()));
      if (it == 39) printf("%s: %d workgroups\n", c.name, nwg);
    }
    printf("  span first start -> last store %.2f us, last WG starts +%.2f us\n", med(span), med(skew));
    const char* nm[7] = {"", "issue", "loads land", "LN+barrier", "MFMA+LDS", "barrier", "epilogue"};
    for (int k = 1; k < 7; ++k) printf("  %-11s median %.2f us\n", nm[k], med(d[k]));
  }
  return 0;
}

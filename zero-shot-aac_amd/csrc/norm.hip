// Row-wise normalisation kernels: LayerNorm (GPT-2 ln_1/ln_2/ln_f, HTSAT norm1/norm2, mapper
// norm1/norm2), PatchMerging gather + LayerNorm, final LayerNorm + mean-pool, L2 normalisation.
// One wave per row, two-pass mean/variance in f32 (matches torch's LayerNorm numerics closely).
#include "common.h"

namespace zs {

template <typename TO>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int M, int C,
                                                        int ldx, const int* __restrict__ rows,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ b, float eps,
                                                        TO* __restrict__ y, int ldy) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + (long)(rows ? rows[row] : row) * ldx;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[c];
  const float mean = wave_sum(s) / C;
  float v = 0.f;
  for (int c = lane; c < C; c += 64) {
    float d = xr[c] - mean;
    v += d * d;
  }
  const float rstd = rsqrtf(wave_sum(v) / C + eps);
  TO* yr = y + (long)row * ldy;
  for (int c = lane; c < C; c += 64) stf(yr + c, (xr[c] - mean) * rstd * w[c] + b[c]);
}

// Single-pass variant for C % 4 == 0, C <= 256*NV: one wave per row, the row held in registers
// as float4 (one 16-byte load per lane per 256 elements), mean and variance from registers.
template <typename TO, int NV>
__global__ __launch_bounds__(256) void layernorm_reg_kernel(const float* __restrict__ x, int M,
                                                            int C, int ldx,
                                                            const int* __restrict__ rows,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ b, float eps,
                                                            TO* __restrict__ y, int ldy) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float4* xr = reinterpret_cast<const float4*>(x + (long)(rows ? rows[row] : row) * ldx);
  const int C4 = C >> 2;
  float4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < C4 ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (lane + 64 * i < C4) {
      const float a = v[i].x - mean, bb = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
      q += (a * a + bb * bb) + (c * c + d * d);
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / C + eps);
  TO* yr = y + (long)row * ldy;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < C4) {
      const float4 ww = reinterpret_cast<const float4*>(w)[c];
      const float4 bv = reinterpret_cast<const float4*>(b)[c];
      const float o0 = (v[i].x - mean) * rstd * ww.x + bv.x, o1 = (v[i].y - mean) * rstd * ww.y + bv.y;
      const float o2 = (v[i].z - mean) * rstd * ww.z + bv.z, o3 = (v[i].w - mean) * rstd * ww.w + bv.w;
      // one 8-byte (bf16) / 16-byte (f32) store per lane: the caller guarantees the alignment
      if constexpr (sizeof(TO) == 2) {
        uint2 u;
        u.x = pk2bf(o0, o1);
        u.y = pk2bf(o2, o3);
        *reinterpret_cast<uint2*>(yr + 4 * c) = u;
      } else {
        *reinterpret_cast<float4*>(yr + 4 * c) = make_float4(o0, o1, o2, o3);
      }
    }
  }
}

// PatchMerging (htsat.py:492-511): out token (i,j) = LN([x(2i,2j), x(2i+1,2j), x(2i,2j+1),
// x(2i+1,2j+1)]) over 4C.  One 256-thread block per output token.
template <typename TO>
__global__ __launch_bounds__(256) void patch_merge_ln_kernel(const float* __restrict__ x, int H,
                                                             int W, int C,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ b,
                                                             TO* __restrict__ y) {
  __shared__ float red[4];
  const int Ho = H / 2, Wo = W / 2;
  const int tok = blockIdx.x;
  const int bb = tok / (Ho * Wo), ij = tok % (Ho * Wo), i = ij / Wo, j = ij % Wo;
  const int C4 = 4 * C;
  auto src = [&](int c) -> float {
    const int part = c / C, cc = c % C;
    const int hh = 2 * i + (part & 1), ww = 2 * j + (part >> 1);
    return x[(((long)bb * H + hh) * W + ww) * C + cc];
  };
  float s = 0.f;
  for (int c = threadIdx.x; c < C4; c += 256) s += src(c);
  const float mean = block_sum(s, red) / C4;
  float v = 0.f;
  for (int c = threadIdx.x; c < C4; c += 256) {
    float d = src(c) - mean;
    v += d * d;
  }
  const float rstd = rsqrtf(block_sum(v, red) / C4 + 1e-5f);
  TO* yr = y + (long)tok * C4;
  for (int c = threadIdx.x; c < C4; c += 256) stf(yr + c, (src(c) - mean) * rstd * w[c] + b[c]);
}

// The same, one wave per output token with the 4C-wide row in registers (VPL values per lane):
// one read of x, wave reductions, no block barriers (the block version above read x three times
// and synchronised 256 threads twice per token).  Stores move 64 consecutive elements per
// instruction.
template <int VPL, typename TO>
__global__ __launch_bounds__(256) void patch_merge_ln_wave_kernel(const float* __restrict__ x,
                                                                  int H, int W, int C,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ b,
                                                                  TO* __restrict__ y, long ntok) {
  const int lane = threadIdx.x & 63;
  const long tok = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= ntok) return;
  const int Ho = H / 2, Wo = W / 2;
  const int bb = (int)(tok / (Ho * Wo)), ij = (int)(tok % (Ho * Wo)), i = ij / Wo, j = ij % Wo;
  const int C4 = 4 * C;
  float v[VPL];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < VPL; ++q) {
    const int c = lane + 64 * q;
    v[q] = 0.f;
    if (c < C4) {
      const int part = c / C, cc = c - part * C;
      const int hh = 2 * i + (part & 1), ww = 2 * j + (part >> 1);
      v[q] = x[(((long)bb * H + hh) * W + ww) * C + cc];
      s += v[q];
    }
  }
  const float mean = wave_sum(s) / C4;
  float var = 0.f;
#pragma unroll
  for (int q = 0; q < VPL; ++q)
    if (lane + 64 * q < C4) { const float d = v[q] - mean; var += d * d; }
  const float rstd = rsqrtf(wave_sum(var) / C4 + 1e-5f);
  TO* yr = y + tok * C4;
#pragma unroll
  for (int q = 0; q < VPL; ++q) {
    const int c = lane + 64 * q;
    if (c < C4) stf(yr + c, (v[q] - mean) * rstd * w[c] + b[c]);
  }
}

// final LayerNorm + mean over N tokens (htsat.py:830,838-847): one 1024-thread block per clip,
// wave w normalises tokens w, w+16, ... with the row held in registers (CPL values per lane);
// the 16 per-wave partial sums are added in wave order (deterministic).
template <int CPL>
__global__ __launch_bounds__(1024) void ln_meanpool_kernel(const float* __restrict__ x, int N,
                                                           int C, const float* __restrict__ w,
                                                           const float* __restrict__ b,
                                                           float* __restrict__ out) {
  extern __shared__ float part[];  // [16 waves][C]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float acc[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) acc[q] = 0.f;
  const float* xb = x + (long)blockIdx.x * N * C;
  for (int t = wid; t < N; t += 16) {
    const float* xr = xb + (long)t * C;
    float v[CPL], s = 0.f;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int c = lane + 64 * q;
      v[q] = c < C ? xr[c] : 0.f;
      s += v[q];
    }
    const float mean = wave_sum(s) / C;
    float d2 = 0.f;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int c = lane + 64 * q;
      const float d = c < C ? v[q] - mean : 0.f;
      d2 += d * d;
    }
    const float rstd = rsqrtf(wave_sum(d2) / C + 1e-5f);
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int c = lane + 64 * q;
      if (c < C) acc[q] += (v[q] - mean) * rstd * w[c] + b[c];
    }
  }
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = lane + 64 * q;
    if (c < C) part[wid * C + c] = acc[q];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 1024) {
    float s = 0.f;
    for (int k = 0; k < 16; ++k) s += part[k * C + c];
    out[(long)blockIdx.x * C + c] = s / N;
  }
}

__global__ __launch_bounds__(256) void l2norm_kernel(const float* __restrict__ x, int M, int C,
                                                     float eps, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + (long)row * C;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[c] * xr[c];
  const float inv = 1.0f / fmaxf(sqrtf(wave_sum(s)), eps);
  for (int c = lane; c < C; c += 64) y[(long)row * C + c] = xr[c] * inv;
}

template <typename TO>
__global__ void cast_kernel(const float* __restrict__ x, long n, TO* __restrict__ y) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) stf(y + i, x[i]);
}

}  // namespace zs

using namespace zs;

extern "C" int zs_layernorm(const float* x, int M, int C, int ldx, const int* rows, const float* w,
                            const float* b, float eps, void* y, int ldy, int ydtype,
                            void* stream) {
  ZS_REQUIRE(M >= 0 && C > 0 && ldx >= C && ldy >= C, "zs_layernorm: bad shape");
  if (M == 0) return 0;
  dim3 grid(cdiv(M, 4));
  const int yal = ydtype == ZS_BF16 ? 8 : 16;
  if (C % 4 == 0 && ldx % 4 == 0 && C <= 1024 && ldy % 4 == 0 && ((uintptr_t)x & 15) == 0 &&
      ((uintptr_t)y & (yal - 1)) == 0) {
    const int nv = cdiv(C / 4, 64);
#define LNR(TO, NV_)                                                                           \
  hipLaunchKernelGGL((layernorm_reg_kernel<TO, NV_>), grid, dim3(256), 0, S(stream), x, M, C,    \
                     ldx, rows, w, b, eps, (TO*)y, ldy)
#define LNR_T(TO) do { if (nv == 1) LNR(TO, 1); else if (nv == 2) LNR(TO, 2); \
                       else if (nv == 3) LNR(TO, 3); else LNR(TO, 4); } while (0)
    if (ydtype == ZS_BF16) LNR_T(bf16_t); else LNR_T(float);
#undef LNR_T
#undef LNR
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (ydtype == ZS_BF16)
    hipLaunchKernelGGL(layernorm_kernel<bf16_t>, grid, dim3(256), 0, S(stream), x, M, C, ldx, rows, w,
                       b, eps, (bf16_t*)y, ldy);
  else
    hipLaunchKernelGGL(layernorm_kernel<float>, grid, dim3(256), 0, S(stream), x, M, C, ldx, rows, w,
                       b, eps, (float*)y, ldy);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_patch_merge_ln(const float* x, int B, int H, int W, int C, const float* ln_w,
                                 const float* ln_b, void* y, int dtype, void* stream) {
  ZS_REQUIRE(B > 0 && H % 2 == 0 && W % 2 == 0 && C > 0, "zs_patch_merge_ln: bad shape");
  const long ntok = (long)B * (H / 2) * (W / 2);
  const int C4 = 4 * C;
  if (C4 <= 64 * 24) {
    const dim3 grid((unsigned)cdiv(ntok, 4));
#define PMW(VPL_)                                                                               \
    do {                                                                                        \
      if (dtype == ZS_BF16)                                                                     \
        hipLaunchKernelGGL((patch_merge_ln_wave_kernel<VPL_, bf16_t>), grid, dim3(256), 0,       \
                           S(stream), x, H, W, C, ln_w, ln_b, (bf16_t*)y, ntok);                \
      else                                                                                      \
        hipLaunchKernelGGL((patch_merge_ln_wave_kernel<VPL_, float>), grid, dim3(256), 0,        \
                           S(stream), x, H, W, C, ln_w, ln_b, (float*)y, ntok);                 \
    } while (0)
    if (C4 <= 64 * 6) PMW(6); else if (C4 <= 64 * 12) PMW(12); else PMW(24);
#undef PMW
    ZS_LAUNCH_CHECK();
    return 0;
  }
  dim3 grid(B * (H / 2) * (W / 2));
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(patch_merge_ln_kernel<bf16_t>, grid, dim3(256), 0, S(stream), x, H, W, C,
                       ln_w, ln_b, (bf16_t*)y);
  else
    hipLaunchKernelGGL(patch_merge_ln_kernel<float>, grid, dim3(256), 0, S(stream), x, H, W, C,
                       ln_w, ln_b, (float*)y);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_ln_meanpool(const float* x, int B, int N, int C, const float* ln_w,
                              const float* ln_b, float* out, void* stream) {
  ZS_REQUIRE(B > 0 && N > 0 && C > 0 && C <= 2048, "zs_ln_meanpool: bad shape (C <= 2048)");
  const size_t smem = 16 * C * sizeof(float);
#define LMP(CPL_)                                                                              \
  hipLaunchKernelGGL(ln_meanpool_kernel<CPL_>, dim3(B), dim3(1024), smem, S(stream), x, N, C,   \
                     ln_w, ln_b, out)
  if (C <= 256) LMP(4); else if (C <= 768) LMP(12); else LMP(32);
#undef LMP
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_l2norm_rows(const float* x, int M, int C, float eps, float* y, void* stream) {
  ZS_REQUIRE(M >= 0 && C > 0, "zs_l2norm_rows: bad shape");
  if (M == 0) return 0;
  hipLaunchKernelGGL(l2norm_kernel, dim3(cdiv(M, 4)), dim3(256), 0, S(stream), x, M, C, eps, y);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_cast(const float* x, long n, void* y, int dtype, void* stream) {
  ZS_REQUIRE(n >= 0, "zs_cast: n");
  if (n == 0) return 0;
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(cast_kernel<bf16_t>, dim3(cdiv(n, 256)), dim3(256), 0, S(stream), x, n,
                       (bf16_t*)y);
  else
    hipLaunchKernelGGL(cast_kernel<float>, dim3(cdiv(n, 256)), dim3(256), 0, S(stream), x, n,
                       (float*)y);
  ZS_LAUNCH_CHECK();
  return 0;
}

// CNN14 (retrieval/models/cnns.py:36-78 ConvBlock, 171-201 forward) on the MFMA GEMM core:
// conv3x3 (pad 1, no bias) as an implicit GEMM over NHWC activations,
//   M = B*H*W output pixels, N = Cout, K = 9*Cin (k = (ky*3+kx)*Cin + ci),
// with eval-BN folded to a per-channel scale/shift and ReLU in the epilogue; then 2x2 average
// pooling and the head (mean over mel, max + mean over time).  For Cin % 32 == 0 every 32-deep
// k-tile is one tap's contiguous channel slice, so the A loader issues 16-byte loads of
// x[b][h+ky-1][w+kx-1][ci0..ci0+31] (zero outside the image).  The first conv (Cin = 1) gathers
// its 9 taps into a K padded to 32.
#include "gemm_core.h"

namespace zs {

template <typename T, int BM>
struct ConvA {
  const T* x;
  int H, W, Cin, M, m0;
  static constexpr int EPC = GemmTraits<T>::EPC;
  static constexpr int CPR = BK / EPC;
  static constexpr int CHUNKS = BM * CPR;
  static constexpr int PER_T = (CHUNKS + 255) / 256;
  uint4 r[PER_T];
  __device__ __forceinline__ void load(int k0) {
    if (Cin % BK == 0) {
      const int tap = k0 / Cin, ci0 = k0 % Cin, ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int c = threadIdx.x + i * 256;
        const int row = c / CPR, col = (c % CPR) * EPC;
        uint4 v = make_uint4(0, 0, 0, 0);
        const int m = m0 + row;
        if (c < CHUNKS && m < M) {
          const int w = m % W, h = (m / W) % H, b = m / (W * H);
          const int hh = h + ky - 1, ww = w + kx - 1;
          if (hh >= 0 && hh < H && ww >= 0 && ww < W)
            v = *reinterpret_cast<const uint4*>(x + (((long)b * H + hh) * W + ww) * Cin + ci0 + col);
        }
        r[i] = v;
      }
    } else {  // Cin == 1: k in [0, 9) are the taps, the rest zero padding
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int c = threadIdx.x + i * 256;
        const int row = c / CPR, col = (c % CPR) * EPC;
        T vals[EPC];
        const int m = m0 + row;
        const int w = m % W, h = (m / W) % H, b = m / (W * H);
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const int k = k0 + col + e;
          float v = 0.f;
          if (c < CHUNKS && m < M && k < 9) {
            const int hh = h + k / 3 - 1, ww = w + k % 3 - 1;
            if (hh >= 0 && hh < H && ww >= 0 && ww < W) v = ldf(x + ((long)b * H + hh) * W + ww);
          }
          vals[e] = Cvt<T>::from_f(v);
        }
        r[i] = *reinterpret_cast<uint4*>(vals);
      }
    }
  }
  __device__ __forceinline__ void store(T* lds) {
    constexpr int LDW = BK + GemmTraits<T>::PAD;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = threadIdx.x + i * 256;
      if (c < CHUNKS) {
        const int row = c / CPR, col = (c % CPR) * EPC;
        *reinterpret_cast<uint4*>(lds + row * LDW + col) = r[i];
      }
    }
  }
};

template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void conv3x3_kernel(const T* x, int H, int W, int Cin, int M,
                                                      const T* w, int Cout, int Kp,
                                                      const float* scale, const float* shift,
                                                      T* out) {
  constexpr int LDW = BK + GemmTraits<T>::PAD;
  __shared__ __attribute__((aligned(16))) T smem[2 * (BM + BN) * LDW];
  constexpr int TM = BM / 64, TN = BN / 64;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  f32x16_t acc[TM][TN];
  ConvA<T, BM> la{x, H, W, Cin, M, m0};
  gemm_mainloop<T, BM, BN>(la, w, Kp, Cout, n0, 0, Kp, smem, acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr0 = (wid >> 1) * (BM / 2), wc0 = (wid & 1) * (BN / 2);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wc0 + j * 32 + (lane & 31);
      if (n >= Cout) continue;
      const float sc = scale[n], sh = shift[n];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wr0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (m < M) stf(out + (long)m * Cout + n, fmaxf(acc[i][j][e] * sc + sh, 0.f));
      }
    }
}

template <typename T>
__global__ void avgpool2_kernel(const T* __restrict__ x, int H, int W, int C, long total,
                                T* __restrict__ y) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int Ho = H / 2, Wo = W / 2;
  const int c = e % C;
  const long p = e / C;
  const int wo = p % Wo, ho = (p / Wo) % Ho, b = p / ((long)Wo * Ho);
  const T* base = x + (((long)b * H + 2 * ho) * W + 2 * wo) * C + c;
  // F.avg_pool2d: (x00 + x01 + x10 + x11) / 4 in f32
  const float s = ldf(base) + ldf(base + C) + ldf(base + (long)W * C) + ldf(base + (long)W * C + C);
  stf(y + e, s / 4.0f);
}

// x [B][H=time][W=mel][C]: mean over mel, then max + mean over time (cnns.py:195-199)
template <typename T>
__global__ void cnn_head_kernel(const T* __restrict__ x, int H, int W, int C,
                                float* __restrict__ out) {
  const int b = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mx = -INFINITY, sum = 0.f;
  for (int h = 0; h < H; ++h) {
    float s = 0.f;
    for (int w = 0; w < W; ++w) s += ldf(x + (((long)b * H + h) * W + w) * C + c);
    s /= W;
    mx = fmaxf(mx, s);
    sum += s;
  }
  out[(long)b * C + c] = mx + sum / H;
}

}  // namespace zs

using namespace zs;

extern "C" int zs_conv3x3_bn_relu(const void* x, int B, int H, int W, int Cin, const void* w,
                                  int Cout, const float* scale, const float* shift, void* out,
                                  int dtype, void* stream) {
  ZS_REQUIRE(B > 0 && H > 0 && W > 0 && Cout > 0, "zs_conv3x3: bad shape");
  ZS_REQUIRE(Cin == 1 || Cin % BK == 0, "zs_conv3x3: Cin must be 1 or a multiple of 32");
  const int M = B * H * W;
  const int Kp = Cin == 1 ? BK : 9 * Cin;   // weights packed [Cout][Kp] (Cin==1: 9 taps + 0 pad)
  hipStream_t st = S(stream);
#define CV(T, BM_, BN_)                                                                          \
  hipLaunchKernelGGL((conv3x3_kernel<T, BM_, BN_>), dim3(cdiv(Cout, BN_), cdiv(M, BM_)), dim3(256), \
                     0, st, (const T*)x, H, W, Cin, M, (const T*)w, Cout, Kp, scale, shift, (T*)out)
  if (Cout >= 128) {
    if (dtype == ZS_BF16) CV(bf16_t, 128, 128); else CV(float, 128, 128);
  } else {
    if (dtype == ZS_BF16) CV(bf16_t, 128, 64); else CV(float, 128, 64);
  }
#undef CV
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_avgpool2(const void* x, int B, int H, int W, int C, void* out, int dtype,
                           void* stream) {
  ZS_REQUIRE(B > 0 && H >= 2 && W >= 2 && C > 0, "zs_avgpool2: bad shape");
  const long total = (long)B * (H / 2) * (W / 2) * C;
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(avgpool2_kernel<bf16_t>, dim3(cdiv(total, 256)), dim3(256), 0, S(stream),
                       (const bf16_t*)x, H, W, C, total, (bf16_t*)out);
  else
    hipLaunchKernelGGL(avgpool2_kernel<float>, dim3(cdiv(total, 256)), dim3(256), 0, S(stream),
                       (const float*)x, H, W, C, total, (float*)out);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_cnn_head(const void* x, int B, int H, int W, int C, float* out, int dtype,
                           void* stream) {
  ZS_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0, "zs_cnn_head: bad shape");
  dim3 grid(cdiv(C, 256), B);
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(cnn_head_kernel<bf16_t>, grid, dim3(256), 0, S(stream), (const bf16_t*)x, H,
                       W, C, out);
  else
    hipLaunchKernelGGL(cnn_head_kernel<float>, grid, dim3(256), 0, S(stream), (const float*)x, H, W,
                       C, out);
  ZS_LAUNCH_CHECK();
  return 0;
}

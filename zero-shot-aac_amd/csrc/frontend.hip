// Audio front end: fused STFT power -> Slaney mel -> 10*log10 -> bn0 (torchlibrosa Spectrogram +
// LogmelFilterBank, retrieval/models/feature_extractor.py:16-38; bn0 htsat.py:949-951), the
// HTSAT bicubic resize + fold (htsat.py:908-923) and PatchEmbed + LayerNorm (htsat.py:115-125).
//
// STFT: one 256-thread block per frame; the reflect-padded, Hann-windowed 1024-sample frame is
// loaded (coalesced) into LDS in bit-reversed order, transformed with a radix-2 complex FFT
// (10 stages, 2 butterflies/thread/stage, twiddles from a host table), |X_k|^2 for k <= 512, then
// 64 threads contract the power spectrum with their mel filter's nonzero band.
#include "common.h"

namespace zs {

constexpr int NFFT = 1024, HOP = 320, NMEL = 64, NBIN = NFFT / 2 + 1;

__global__ __launch_bounds__(256) void logmel_kernel(
    const float* __restrict__ wav, int T, int n_frames, const float* __restrict__ window,
    const float* __restrict__ twiddle, const float* __restrict__ melW,
    const int* __restrict__ mel_lo, const int* __restrict__ mel_hi,
    const float* __restrict__ bn_mean, const float* __restrict__ bn_var,
    const float* __restrict__ bn_w, const float* __restrict__ bn_b, float* __restrict__ out) {
  __shared__ float re[NFFT], im[NFFT];
  __shared__ float pw[NBIN];
  const int f = blockIdx.x % n_frames, b = blockIdx.x / n_frames;
  const float* x = wav + (long)b * T;
  const int start = f * HOP - NFFT / 2;
  for (int n = threadIdx.x; n < NFFT; n += 256) {
    int o = start + n;
    if (o < 0) o = -o;                       // reflect (no edge repeat), torch F.pad 'reflect'
    if (o >= T) o = 2 * (T - 1) - o;
    const float v = x[o] * window[n];
    const int rev = __brev(n) >> (32 - 10);
    re[rev] = v;
    im[rev] = 0.f;
  }
  __syncthreads();
  // iterative radix-2 DIT: stage with half-size `half`, twiddle stride NFFT/(2*half)
  for (int half = 1; half < NFFT; half <<= 1) {
    const int tstride = NFFT / (2 * half);
    for (int bf = threadIdx.x; bf < NFFT / 2; bf += 256) {
      const int grp = bf / half, j = bf % half;
      const int i0 = grp * 2 * half + j, i1 = i0 + half;
      const float wr = twiddle[2 * (j * tstride)], wi = twiddle[2 * (j * tstride) + 1];
      const float xr = re[i1], xi = im[i1];
      const float tr = xr * wr - xi * wi, ti = xr * wi + xi * wr;
      const float ur = re[i0], ui = im[i0];
      re[i0] = ur + tr; im[i0] = ui + ti;
      re[i1] = ur - tr; im[i1] = ui - ti;
    }
    __syncthreads();
  }
  for (int k = threadIdx.x; k < NBIN; k += 256) pw[k] = re[k] * re[k] + im[k] * im[k];
  __syncthreads();
  if (threadIdx.x < NMEL) {
    const int m = threadIdx.x;
    const float* wrow = melW + m * NBIN;
    float acc = 0.f;
    for (int k = mel_lo[m]; k < mel_hi[m]; ++k) acc += pw[k] * wrow[k];
    float v = 10.0f * log10f(fmaxf(acc, 1e-10f));   // power_to_db, ref 1.0 -> offset 0
    if (bn_mean) v = (v - bn_mean[m]) / sqrtf(bn_var[m] + 1e-5f) * bn_w[m] + bn_b[m];
    out[((long)b * n_frames + f) * NMEL + m] = v;
  }
}

// bicubic (A = -0.75, align_corners = True) along time T_in -> 1024, identity along the 64 mels,
// then fold: img[r = chunk*64 + mel][c] = resized[t = chunk*256 + c][mel]
__global__ void wav2img_kernel(const float* __restrict__ in, int T_in, float* __restrict__ img) {
#pragma clang fp contract(off)   // torch rounds scale*t before `- floor` and each weight term
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c = e % 256, r = (e / 256) % 256, b = e / 65536;
  const int chunk = r / 64, mel = r % 64;
  const int t = chunk * 256 + c;
  const float scale = (float)(T_in - 1) / (float)(1024 - 1);
  // rounded product (no FMA contraction into `src - i0`): torch's area_pixel_compute_source_index
  const float src = __fmul_rn(scale, (float)t);
  const int i0 = (int)floorf(src);
  const float x1 = src - (float)i0;
  const float A = -0.75f;
  auto cc1 = [&](float x) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; };
  auto cc2 = [&](float x) { return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; };
  const float w0 = cc2(x1 + 1.f), w1 = cc1(x1), x2 = 1.f - x1, w2 = cc1(x2), w3 = cc2(x2 + 1.f);
  const float* col = in + (long)b * T_in * 64 + mel;
  auto at = [&](int i) { i = i < 0 ? 0 : (i >= T_in ? T_in - 1 : i); return col[(long)i * 64]; };
  float v = at(i0 - 1) * w0;
  v += at(i0) * w1;
  v += at(i0 + 1) * w2;
  v += at(i0 + 2) * w3;
  img[e] = v;
}

// PatchEmbed: one wave per token; lanes own channels c = lane and lane+64 (< 96)
__global__ __launch_bounds__(256) void patch_embed_kernel(const float* __restrict__ img,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ lnw,
                                                          const float* __restrict__ lnb,
                                                          float* __restrict__ x, long ntok) {
  constexpr int C = 96;
  const int lane = threadIdx.x & 63;
  const long tok = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= ntok) return;
  const int b = tok / 4096, t = tok % 4096, ph = t / 64, pwc = t % 64;
  const float* base = img + (long)b * 65536 + (ph * 4) * 256 + pwc * 4;
  float px[16];
#pragma unroll
  for (int ky = 0; ky < 4; ++ky)
#pragma unroll
    for (int kx = 0; kx < 4; ++kx) px[ky * 4 + kx] = base[ky * 256 + kx];
  float v0 = 0.f, v1 = 0.f;
  {
    const float* wr = w + lane * 16;
    float a = bias[lane];
#pragma unroll
    for (int q = 0; q < 16; ++q) a += wr[q] * px[q];
    v0 = a;
  }
  const bool has1 = lane + 64 < C;
  if (has1) {
    const float* wr = w + (lane + 64) * 16;
    float a = bias[lane + 64];
#pragma unroll
    for (int q = 0; q < 16; ++q) a += wr[q] * px[q];
    v1 = a;
  }
  const float mean = wave_sum(v0 + (has1 ? v1 : 0.f)) / C;
  const float d0 = v0 - mean, d1 = has1 ? v1 - mean : 0.f;
  const float rstd = rsqrtf(wave_sum(d0 * d0 + d1 * d1) / C + 1e-5f);
  float* xr = x + tok * C;
  xr[lane] = d0 * rstd * lnw[lane] + lnb[lane];
  if (has1) xr[lane + 64] = d1 * rstd * lnw[lane + 64] + lnb[lane + 64];
}

}  // namespace zs

using namespace zs;

extern "C" int zs_logmel(const float* wav, int B, int T, const float* window, const float* twiddle,
                         const float* melW, const int* mel_lo, const int* mel_hi,
                         const float* bn_mean, const float* bn_var, const float* bn_weight,
                         const float* bn_bias, float* out, void* stream) {
  ZS_REQUIRE(B > 0 && T > NFFT / 2, "zs_logmel: need T > 512 samples for reflect padding");
  const int n_frames = T / HOP + 1;
  hipLaunchKernelGGL(logmel_kernel, dim3((long)B * n_frames), dim3(256), 0, S(stream), wav, T,
                     n_frames, window, twiddle, melW, mel_lo, mel_hi, bn_mean, bn_var, bn_weight,
                     bn_bias, out);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_wav2img(const float* in, int B, int T_in, float* img, void* stream) {
  ZS_REQUIRE(B > 0 && T_in > 1 && T_in <= 1024, "zs_wav2img: 1 < T_in <= 1024");
  const long total = (long)B * 65536;
  hipLaunchKernelGGL(wav2img_kernel, dim3(cdiv(total, 256)), dim3(256), 0, S(stream), in, T_in, img);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_patch_embed(const float* img, int B, const float* w, const float* b,
                              const float* ln_w, const float* ln_b, float* x, void* stream) {
  ZS_REQUIRE(B > 0, "zs_patch_embed: B");
  const long ntok = (long)B * 4096;
  hipLaunchKernelGGL(patch_embed_kernel, dim3(cdiv(ntok, 4)), dim3(256), 0, S(stream), img, w, b,
                     ln_w, ln_b, x, ntok);
  ZS_LAUNCH_CHECK();
  return 0;
}

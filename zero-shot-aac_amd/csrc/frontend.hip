// Audio front end: fused STFT power -> Slaney mel -> 10*log10 -> bn0 (torchlibrosa Spectrogram +
// LogmelFilterBank, retrieval/models/feature_extractor.py:16-38; bn0 htsat.py:949-951), the
// HTSAT bicubic resize + fold (htsat.py:908-923) and PatchEmbed + LayerNorm (htsat.py:115-125).
//
// STFT: one 256-thread block per LM_PAIRS pairs of frames: two real, reflect-padded,
// Hann-windowed 1024-sample frames are packed as z = a + i*b, loaded (coalesced) into padded LDS
// rows in natural order and transformed with a radix-4 decimation-in-frequency complex FFT (5
// stages, one radix-4 butterfly per thread per pair per stage, twiddles from a host table staged
// in LDS; the output lands in base-4 digit-reversed order); the two spectra are
// separated as A_k = (Z_k + conj Z_{N-k})/2, B_k = (Z_k - conj Z_{N-k})/2i, |.|^2 for k <= 512,
// then 64 threads per frame contract the power spectrum with their mel filter's nonzero band.
#include "common.h"

namespace zs {

constexpr int NFFT = 1024, HOP = 320, NMEL = 64, NBIN = NFFT / 2 + 1;

__device__ __forceinline__ int digrev4(int n) {   // reverse the 5 base-4 digits of n < 1024
  int r = 0;
#pragma unroll
  for (int d = 0; d < 5; ++d) { r = (r << 2) | (n & 3); n >>= 2; }
  return r;
}

constexpr int LM_PAIRS = 2;               // frame pairs (complex FFTs) per 256-thread block
constexpr int LPAD = NFFT + NFFT / 16;     // padded LDS row: element i lives at i + i/16
__device__ __forceinline__ int lp(int i) { return i + (i >> 4); }

__global__ __launch_bounds__(256) void logmel_kernel(
    const float* __restrict__ wav, int T, int n_frames, int total_frames,
    const float* __restrict__ window, const float* __restrict__ twiddle,
    const float* __restrict__ melW, const int* __restrict__ mel_lo, const int* __restrict__ mel_hi,
    const float* __restrict__ bn_mean, const float* __restrict__ bn_var,
    const float* __restrict__ bn_w, const float* __restrict__ bn_b, float* __restrict__ out) {
  constexpr int NP = LM_PAIRS;
  __shared__ float re[NP][LPAD], im[NP][LPAD];
  __shared__ float tw[NFFT];              // (cos, sin)(-2 pi k / 1024), k < 512
  __shared__ float mw[2 * NBIN];          // the mel filters' nonzero bands, packed
  __shared__ float pw[2 * NP][NBIN];
  __shared__ int moff[NMEL + 1], mlo[NMEL];
  for (int n = threadIdx.x; n < NFFT; n += 256) tw[n] = twiddle[n];
  if (threadIdx.x < 64) {                 // band offsets: wave-wide inclusive scan of the widths
    const int m = threadIdx.x;
    const int lo = mel_lo[m], len = mel_hi[m] - lo;
    int inc = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int o = __shfl_up(inc, d, 64);
      if (m >= d) inc += o;
    }
    mlo[m] = lo;
    moff[m + 1] = inc;
    if (m == 0) moff[0] = 0;
  }
  __syncthreads();
  {   // pack the bands: 4 threads per mel filter
    const int m = threadIdx.x >> 2, s0 = threadIdx.x & 3;
    const int lo = mlo[m], len = moff[m + 1] - moff[m];
    for (int k = s0; k < len; k += 4) mw[moff[m] + k] = melW[m * NBIN + lo + k];
  }
  // persistent over frame groups: the twiddles and the packed mel bands are staged once per block
  for (int g0 = 2 * NP * blockIdx.x; g0 < total_frames; g0 += 2 * NP * gridDim.x) {
  // natural-order load (coalesced global reads, conflict-free LDS writes)
  for (int n = threadIdx.x; n < NP * NFFT; n += 256) {
    const int p = n / NFFT, k = n % NFFT;
    float v[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int g = g0 + 2 * p + q;
      v[q] = 0.f;
      if (g < total_frames) {
        const int b = g / n_frames, f = g % n_frames;
        int o = f * HOP - NFFT / 2 + k;
        if (o < 0) o = -o;                       // reflect (no edge repeat), torch F.pad 'reflect'
        if (o >= T) o = 2 * (T - 1) - o;
        v[q] = wav[(long)b * T + o] * window[k];
      }
    }
    re[p][lp(k)] = v[0];
    im[p][lp(k)] = v[1];
  }
  __syncthreads();
  // radix-4 DIF (natural-order in, base-4 digit-reversed out):
  // y0 = x0+x1+x2+x3, y1 = (x0-x2) - i(x1-x3), y2 = (x0+x2) - (x1+x3), y3 = (x0-x2) + i(x1-x3),
  // then y_p *= W_{4L}^{p j} = W_1024^{p j S}
  for (int L = NFFT / 4, S = 1; L >= 1; L >>= 2, S <<= 2) {
    const int bf = threadIdx.x, grp = bf / L, j = bf % L;
    const int i0 = grp * 4 * L + j;
    float wr[4], wi[4];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const int e = j * q * S;                   // < 768
      if (e < 512) { wr[q] = tw[2 * e]; wi[q] = tw[2 * e + 1]; }
      else { wr[q] = -tw[2 * (e - 512)]; wi[q] = -tw[2 * (e - 512) + 1]; }
    }
    float xr[NP][4], xi[NP][4];
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) { xr[p][q] = re[p][lp(i0 + q * L)]; xi[p][q] = im[p][lp(i0 + q * L)]; }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const float s02r = xr[p][0] + xr[p][2], s02i = xi[p][0] + xi[p][2];
      const float d02r = xr[p][0] - xr[p][2], d02i = xi[p][0] - xi[p][2];
      const float s13r = xr[p][1] + xr[p][3], s13i = xi[p][1] + xi[p][3];
      const float d13r = xr[p][1] - xr[p][3], d13i = xi[p][1] - xi[p][3];
      float yr[4], yi[4];
      yr[0] = s02r + s13r; yi[0] = s02i + s13i;
      yr[1] = d02r + d13i; yi[1] = d02i - d13r;
      yr[2] = s02r - s13r; yi[2] = s02i - s13i;
      yr[3] = d02r - d13i; yi[3] = d02i + d13r;
      re[p][lp(i0)] = yr[0];
      im[p][lp(i0)] = yi[0];
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        re[p][lp(i0 + q * L)] = yr[q] * wr[q] - yi[q] * wi[q];
        im[p][lp(i0 + q * L)] = yr[q] * wi[q] + yi[q] * wr[q];
      }
    }
    __syncthreads();
  }
  // X[k] sits at digrev4(k); separate the two real spectra, |.|^2 for k <= 512
  for (int n = threadIdx.x; n < NP * NBIN; n += 256) {
    const int p = n / NBIN, k = n % NBIN;
    const int a = lp(digrev4(k)), c = lp(digrev4((NFFT - k) & (NFFT - 1)));
    const float zr = re[p][a], zi = im[p][a], cr = re[p][c], ci = -im[p][c];   // conj Z_{N-k}
    const float ar = zr + cr, ai = zi + ci;        // 2 A_k
    const float br = zi - ci, bi = cr - zr;        // 2 B_k = (Z - conj Z_{N-k}) / i
    pw[2 * p][k] = 0.25f * (ar * ar + ai * ai);
    pw[2 * p + 1][k] = 0.25f * (br * br + bi * bi);
  }
  __syncthreads();
  for (int o = threadIdx.x; o < 2 * NP * NMEL; o += 256) {
    const int fr = o / NMEL, m = o % NMEL;
    const int g = g0 + fr;
    if (g >= total_frames) continue;
    const int lo = mlo[m], base = moff[m], len = moff[m + 1] - base;
    float acc = 0.f;
    for (int k = 0; k < len; ++k) acc += pw[fr][lo + k] * mw[base + k];
    float v = 10.0f * log10f(fmaxf(acc, 1e-10f));   // power_to_db, ref 1.0 -> offset 0
    if (bn_mean) v = (v - bn_mean[m]) / sqrtf(bn_var[m] + 1e-5f) * bn_w[m] + bn_b[m];
    out[(long)g * NMEL + m] = v;
  }
  __syncthreads();   // re/im/pw are refilled by the next group
  }
}

// ------------------------------------------------------------------ wave-per-FFT front end
// One wave per frame pair (complex 1024-point FFT), 4 independent waves per block, no block
// barriers in the frame loop.  The same radix-4 DIF as logmel_kernel (same twiddles, same
// butterfly arithmetic), but with the 16 points a lane holds two stages run in registers between
// LDS exchanges (3 exchanges instead of 5 block-wide stage round trips):
//   phase 1: lane l holds n = 256a + 64b + l            -> stages over a, b
//   phase 2: lane (p1, p2, e) holds 256p1+64p2+16c+4d+e -> stages over c, d
//   phase 3: lane l holds 16l + 4r + e (r = 0..3)        -> the last stage over e
// Every exchange is conflict-free in the padded row (i + i/16).  The wave's row then holds the
// spectrum in base-4 digit-reversed order; the two real spectra are separated into power rows
// (aliasing the row: each lane's reads finish before its writes, LDS ops of a wave are in
// order) and lane m contracts mel band m for both frames.
__device__ __forceinline__ float2 twd(const float* tw, int e) {   // W_1024^e, e < 1024
  if (e < 512) return make_float2(tw[2 * e], tw[2 * e + 1]);
  return make_float2(-tw[2 * (e - 512)], -tw[2 * (e - 512) + 1]);
}
__device__ __forceinline__ void bfly4(float (&xr)[4], float (&xi)[4]) {
  const float s02r = xr[0] + xr[2], s02i = xi[0] + xi[2];
  const float d02r = xr[0] - xr[2], d02i = xi[0] - xi[2];
  const float s13r = xr[1] + xr[3], s13i = xi[1] + xi[3];
  const float d13r = xr[1] - xr[3], d13i = xi[1] - xi[3];
  xr[0] = s02r + s13r; xi[0] = s02i + s13i;
  xr[1] = d02r + d13i; xi[1] = d02i - d13r;
  xr[2] = s02r - s13r; xi[2] = s02i - s13i;
  xr[3] = d02r - d13i; xi[3] = d02i + d13r;
}
__device__ __forceinline__ void twmul(float& r, float& i, float2 w) {
  const float t = r * w.x - i * w.y;
  i = r * w.y + i * w.x;
  r = t;
}
// W_1024^{64 m} = W_16^m (m < 16): exact-rounded constants, folded after unrolling
__device__ __forceinline__ float2 w16(int m) {
  constexpr float C[16] = {1.f, 0.92387953f, 0.70710678f, 0.38268343f, 0.f, -0.38268343f,
                           -0.70710678f, -0.92387953f, -1.f, -0.92387953f, -0.70710678f,
                           -0.38268343f, 0.f, 0.38268343f, 0.70710678f, 0.92387953f};
  return make_float2(C[m & 15], C[(m + 4) & 15]);   // (cos, -sin)(2 pi m / 16)
}
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// orders this wave's LDS accesses for the compiler (the hardware keeps a wave's LDS ops in order)
__device__ __forceinline__ void wave_lds_order() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

int g_logmel_wave = 1;   // zs_tune_set("logmel_wave", 0): the block-per-4-frames kernel

__global__ __launch_bounds__(256, 3) void logmel_wave_kernel(
    const float* __restrict__ wav, int T, int n_frames, int total_frames,
    const float* __restrict__ window, const float* __restrict__ twiddle,
    const float* __restrict__ melW, const int* __restrict__ mel_lo, const int* __restrict__ mel_hi,
    const float* __restrict__ bn_mean, const float* __restrict__ bn_var,
    const float* __restrict__ bn_w, const float* __restrict__ bn_b, float* __restrict__ out) {
  __shared__ float rows[4][2][LPAD];      // per wave: re, im (later: the two power rows)
  __shared__ float tw[NFFT];
  __shared__ float swin[NFFT];
  __shared__ float mw[2 * NBIN];
  __shared__ int moff[NMEL + 1], mlo[NMEL];
  for (int n = threadIdx.x; n < NFFT; n += 256) { tw[n] = twiddle[n]; swin[n] = window[n]; }
  if (threadIdx.x < 64) {
    const int m = threadIdx.x;
    const int lo = mel_lo[m], len = mel_hi[m] - lo;
    int inc = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int o = __shfl_up(inc, d, 64);
      if (m >= d) inc += o;
    }
    mlo[m] = lo;
    moff[m + 1] = inc;
    if (m == 0) moff[0] = 0;
  }
  __syncthreads();
  {
    const int m = threadIdx.x >> 2, s0 = threadIdx.x & 3;
    const int lo = mlo[m], len = moff[m + 1] - moff[m];
    for (int k = s0; k < len; k += 4) mw[moff[m] + k] = melW[m * NBIN + lo + k];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* re = rows[wid][0];
  float* im = rows[wid][1];
  const int npairs = (total_frames + 1) >> 1;
  // raw samples of a pair (zero for a missing second frame); the next pair's are fetched before
  // the current pair's FFT so their HBM latency overlaps it
  auto fetch = [&](int gp, float (&sr)[16], float (&si)[16]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int g = 2 * gp + q;
      const bool valid = g < total_frames;
      const int gb = valid ? g / n_frames : 0, f = valid ? g % n_frames : 0;
      const float* src = wav + (long)gb * T;
      const int base = f * HOP - NFFT / 2;
      if (valid && base >= 0 && base + NFFT <= T) {   // interior frame (wave-uniform): one
        const float* p = src + base + lane;            // pointer, immediate offsets
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if (q == 0) sr[i] = p[64 * i]; else si[i] = p[64 * i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          int o = base + 64 * i + lane;
          if (o < 0) o = -o;                       // reflect (no edge repeat), torch F.pad 'reflect'
          if (o >= T) o = 2 * (T - 1) - o;
          const float v = valid ? src[o] : 0.f;
          if (q == 0) sr[i] = v; else si[i] = v;
        }
      }
    }
  };
  const int stride = gridDim.x * 4;
  float cr_[16], ci_[16];
  int gp = blockIdx.x * 4 + wid;
  if (gp < npairs) fetch(gp, cr_, ci_);
  for (; gp < npairs; gp += stride) {
    float zr[4][4], zi[4][4];             // phase 1: [a][b], n = 256a + 64b + lane
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float wv = swin[256 * a + 64 * b + lane];
        zr[a][b] = cr_[4 * a + b] * wv;
        zi[a][b] = ci_[4 * a + b] * wv;
      }
    if (gp + stride < npairs) fetch(gp + stride, cr_, ci_);
    // stage 1 (over a), twiddle W_1024^{p (64b + lane)} = W_1024^{p lane} W_16^{p b} (three
    // table twiddles per lane instead of twelve: they stay in registers across the frame loop)
    const float2 t1[4] = {make_float2(1.f, 0.f), twd(tw, lane), twd(tw, 2 * lane), twd(tw, 3 * lane)};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      float xr[4] = {zr[0][b], zr[1][b], zr[2][b], zr[3][b]};
      float xi[4] = {zi[0][b], zi[1][b], zi[2][b], zi[3][b]};
      bfly4(xr, xi);
#pragma unroll
      for (int p = 1; p < 4; ++p) twmul(xr[p], xi[p], b == 0 ? t1[p] : cmul(t1[p], w16(p * b)));
#pragma unroll
      for (int p = 0; p < 4; ++p) { zr[p][b] = xr[p]; zi[p][b] = xi[p]; }
    }
    // stage 2 (over b), twiddle W_1024^{4 p lane}
    {
      const float2 w1 = twd(tw, 4 * lane), w2 = twd(tw, 8 * lane), w3 = twd(tw, 12 * lane);
#pragma unroll
      for (int p1 = 0; p1 < 4; ++p1) {
        float xr[4] = {zr[p1][0], zr[p1][1], zr[p1][2], zr[p1][3]};
        float xi[4] = {zi[p1][0], zi[p1][1], zi[p1][2], zi[p1][3]};
        bfly4(xr, xi);
        twmul(xr[1], xi[1], w1);
        twmul(xr[2], xi[2], w2);
        twmul(xr[3], xi[3], w3);
#pragma unroll
        for (int p = 0; p < 4; ++p) { zr[p1][p] = xr[p]; zi[p1][p] = xi[p]; }
      }
    }
    wave_lds_order();                      // previous pair's mel reads of this row are done
#pragma unroll
    for (int p1 = 0; p1 < 4; ++p1)
#pragma unroll
      for (int p2 = 0; p2 < 4; ++p2) {
        re[lp(256 * p1 + 64 * p2 + lane)] = zr[p1][p2];
        im[lp(256 * p1 + 64 * p2 + lane)] = zi[p1][p2];
      }
    wave_lds_order();
    // phase 2: lane = 16 p1 + 4 p2 + e holds pb + 16c + 4d
    const int E = lane & 3;
    const int pb = 256 * (lane >> 4) + 64 * ((lane >> 2) & 3) + E;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        zr[c][d] = re[lp(pb + 16 * c + 4 * d)];
        zi[c][d] = im[lp(pb + 16 * c + 4 * d)];
      }
    // stage 3 (over c), twiddle W_1024^{16 p (4d + e)} = W_1024^{16 p e} W_16^{p d}
    const float2 t3[4] = {make_float2(1.f, 0.f), twd(tw, 16 * E), twd(tw, 32 * E), twd(tw, 48 * E)};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      float xr[4] = {zr[0][d], zr[1][d], zr[2][d], zr[3][d]};
      float xi[4] = {zi[0][d], zi[1][d], zi[2][d], zi[3][d]};
      bfly4(xr, xi);
#pragma unroll
      for (int p = 1; p < 4; ++p) twmul(xr[p], xi[p], d == 0 ? t3[p] : cmul(t3[p], w16(p * d)));
#pragma unroll
      for (int p = 0; p < 4; ++p) { zr[p][d] = xr[p]; zi[p][d] = xi[p]; }
    }
    // stage 4 (over d), twiddle W_1024^{64 p e}
    {
      const float2 w1 = twd(tw, 64 * E), w2 = twd(tw, 128 * E), w3 = twd(tw, 192 * E);
#pragma unroll
      for (int p3 = 0; p3 < 4; ++p3) {
        float xr[4] = {zr[p3][0], zr[p3][1], zr[p3][2], zr[p3][3]};
        float xi[4] = {zi[p3][0], zi[p3][1], zi[p3][2], zi[p3][3]};
        bfly4(xr, xi);
        twmul(xr[1], xi[1], w1);
        twmul(xr[2], xi[2], w2);
        twmul(xr[3], xi[3], w3);
#pragma unroll
        for (int p = 0; p < 4; ++p) { zr[p3][p] = xr[p]; zi[p3][p] = xi[p]; }
      }
    }
    wave_lds_order();
#pragma unroll
    for (int p3 = 0; p3 < 4; ++p3)
#pragma unroll
      for (int p4 = 0; p4 < 4; ++p4) {
        re[lp(pb + 16 * p3 + 4 * p4)] = zr[p3][p4];
        im[lp(pb + 16 * p3 + 4 * p4)] = zi[p3][p4];
      }
    wave_lds_order();
    // phase 3: lane holds 16 lane + 4r + e; the last stage (twiddle 1), written back in place
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float xr[4], xi[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) { xr[e] = re[lp(16 * lane + 4 * r + e)]; xi[e] = im[lp(16 * lane + 4 * r + e)]; }
      bfly4(xr, xi);
#pragma unroll
      for (int e = 0; e < 4; ++e) { re[lp(16 * lane + 4 * r + e)] = xr[e]; im[lp(16 * lane + 4 * r + e)] = xi[e]; }
    }
    wave_lds_order();
    // X[k] sits at digrev4(k): separate the two real spectra, |.|^2 for k <= 512
    float pa[9], pq[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int k = min(lane + 64 * t, NBIN - 1);
      const int a = lp(digrev4(k)), c = lp(digrev4((NFFT - k) & (NFFT - 1)));
      const float zr_ = re[a], zi_ = im[a], cr = re[c], ci = -im[c];
      const float ar = zr_ + cr, ai = zi_ + ci;
      const float br = zi_ - ci, bi = cr - zr_;
      pa[t] = 0.25f * (ar * ar + ai * ai);
      pq[t] = 0.25f * (br * br + bi * bi);
    }
    wave_lds_order();
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int k = lane + 64 * t;
      if (k < NBIN) { re[k] = pa[t]; im[k] = pq[t]; }
    }
    wave_lds_order();
    {
      const int m = lane;
      const int lo = mlo[m], base = moff[m], len = moff[m + 1] - base;
      float acc0 = 0.f, acc1 = 0.f;
      for (int k = 0; k < len; ++k) {
        const float wv = mw[base + k];
        acc0 += re[lo + k] * wv;
        acc1 += im[lo + k] * wv;
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int g = 2 * gp + q;
        if (g >= total_frames) continue;
        float v = 10.0f * log10f(fmaxf(q ? acc1 : acc0, 1e-10f));   // power_to_db, ref 1.0
        if (bn_mean) v = (v - bn_mean[m]) / sqrtf(bn_var[m] + 1e-5f) * bn_w[m] + bn_b[m];
        out[(long)g * NMEL + m] = v;
      }
    }
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

// PatchEmbed: 4 lanes per token (a 4x4 patch -> 96 channels, 24 per lane, LayerNorm reduced over
// the lane quad); 256 threads = 64 tokens = one row of the 64x64 patch grid, weights / bias / LN
// params broadcast from LDS.  Lane g of a quad owns channels 16i + 4g .. 16i + 4g + 3 (i < 6), so
// each 16-byte store instruction writes 64 contiguous bytes per token.  (One thread per token held
// 96 values, ran at one wave per SIMD and stored 64 scattered lines per instruction.)
__global__ __launch_bounds__(256) void patch_embed_kernel(const float* __restrict__ img,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ lnw,
                                                          const float* __restrict__ lnb,
                                                          float* __restrict__ x, long ntok) {
  constexpr int C = 96, CPL = C / 4, WS = 20;   // weight row stride: 16 + 4 pad (16-B aligned)
  // 20-float rows: the quad's 4 lanes read channels 4 apart, whose rows then start 16 banks apart
  // (a 16-float stride put all four on the same banks: 4-way conflicts on every weight read)
  __shared__ __attribute__((aligned(16))) float sw[C * WS];
  __shared__ float sb[C], sg[C], sbeta[C];
  for (int i = threadIdx.x; i < C * 16; i += 256) sw[(i / 16) * WS + (i % 16)] = w[i];
  if (threadIdx.x < C) {
    sb[threadIdx.x] = bias[threadIdx.x];
    sg[threadIdx.x] = lnw[threadIdx.x];
    sbeta[threadIdx.x] = lnb[threadIdx.x];
  }
  __syncthreads();
  const long tok = (long)blockIdx.x * 64 + (threadIdx.x >> 2);
  const int g = threadIdx.x & 3;
  const bool valid = tok < ntok;          // whole quads (ntok is a multiple of 4096)
  const long tk = valid ? tok : 0;
  const int b = (int)(tk / 4096), t = (int)(tk % 4096), ph = t / 64, pwc = t % 64;
  const float* base = img + (long)b * 65536 + (ph * 4) * 256 + pwc * 4;
  float px[16];
#pragma unroll
  for (int ky = 0; ky < 4; ++ky) {
    const float4 r = *reinterpret_cast<const float4*>(base + ky * 256);
    px[ky * 4 + 0] = r.x; px[ky * 4 + 1] = r.y; px[ky * 4 + 2] = r.z; px[ky * 4 + 3] = r.w;
  }
  float v[CPL];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < CPL / 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 16 * i + 4 * g + j;
      float a = sb[c];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const float4 wq = *reinterpret_cast<const float4*>(sw + c * WS + 4 * q4);
        a += wq.x * px[4 * q4];
        a += wq.y * px[4 * q4 + 1];
        a += wq.z * px[4 * q4 + 2];
        a += wq.w * px[4 * q4 + 3];
      }
      v[4 * i + j] = a;
      sum += a;
    }
  sum += __shfl_xor(sum, 1, 64);
  sum += __shfl_xor(sum, 2, 64);
  const float mean = sum / C;
  float var = 0.f;
#pragma unroll
  for (int k = 0; k < CPL; ++k) { const float d = v[k] - mean; var += d * d; }
  var += __shfl_xor(var, 1, 64);
  var += __shfl_xor(var, 2, 64);
  const float rstd = rsqrtf(var / C + 1e-5f);
  if (!valid) return;
#pragma unroll
  for (int i = 0; i < CPL / 4; ++i) {
    const int c = 16 * i + 4 * g;
    *reinterpret_cast<float4*>(x + tok * C + c) =
        make_float4((v[4 * i] - mean) * rstd * sg[c] + sbeta[c],
                    (v[4 * i + 1] - mean) * rstd * sg[c + 1] + sbeta[c + 1],
                    (v[4 * i + 2] - mean) * rstd * sg[c + 2] + sbeta[c + 2],
                    (v[4 * i + 3] - mean) * rstd * sg[c + 3] + sbeta[c + 3]);
  }
}

// Ragged clips -> [B][T] fixed-length rows (data_handing/embeddings_generator.py:53-59): clip b
// (length len[b], starting at off[b] of one flat buffer) is cropped to its first T samples or
// zero-padded at the end.  float4 stores; the source is read with scalar loads (clip offsets
// need not be 16-byte aligned).
__global__ __launch_bounds__(256) void pack_clips_kernel(const float* __restrict__ flat,
                                                         const long* __restrict__ off,
                                                         const int* __restrict__ len, int T,
                                                         float* __restrict__ out) {
  const int b = blockIdx.y;
  const long o = off[b];
  const int n = min(len[b], T);
  for (int i = 4 * (blockIdx.x * 256 + threadIdx.x); i < T; i += 4 * 256 * gridDim.x) {
    float4 v;
    v.x = i < n ? flat[o + i] : 0.f;
    v.y = i + 1 < n ? flat[o + i + 1] : 0.f;
    v.z = i + 2 < n ? flat[o + i + 2] : 0.f;
    v.w = i + 3 < n ? flat[o + i + 3] : 0.f;
    *reinterpret_cast<float4*>(out + (long)b * T + i) = v;
  }
}

}  // namespace zs

using namespace zs;

extern "C" int zs_pack_clips(const float* flat, const long* offsets, const int* lengths, int B,
                             int T, float* out, void* stream) {
  ZS_REQUIRE(B > 0 && T > 0 && T % 4 == 0, "zs_pack_clips: B > 0, T > 0, T %% 4 == 0");
  ZS_REQUIRE(flat && offsets && lengths && out && ((uintptr_t)out & 15) == 0,
             "zs_pack_clips: pointers (out 16-byte aligned)");
  hipLaunchKernelGGL(pack_clips_kernel, dim3(std::min(cdiv(T, 1024), 64), B), dim3(256), 0,
                     S(stream), flat, offsets, lengths, T, out);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_logmel(const float* wav, int B, int T, const float* window, const float* twiddle,
                         const float* melW, const int* mel_lo, const int* mel_hi,
                         const float* bn_mean, const float* bn_var, const float* bn_weight,
                         const float* bn_bias, float* out, void* stream) {
  ZS_REQUIRE(B > 0 && T > NFFT / 2, "zs_logmel: need T > 512 samples for reflect padding");
  const int n_frames = T / HOP + 1;
  const int total = B * n_frames;
  if (g_logmel_wave) {
    const int npairs = cdiv(total, 2);
    // 3 blocks per CU fit the LDS (47.6 KB each): one resident wave of blocks, no tail round
    hipLaunchKernelGGL(logmel_wave_kernel, dim3(std::min(cdiv(npairs, 4), 256 * 3)), dim3(256), 0,
                       S(stream), wav, T, n_frames, total, window, twiddle, melW, mel_lo, mel_hi,
                       bn_mean, bn_var, bn_weight, bn_bias, out);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  const int groups = cdiv(total, 2 * LM_PAIRS);
  hipLaunchKernelGGL(logmel_kernel, dim3(std::min(groups, 256 * 8)), dim3(256), 0, S(stream), wav, T,
                     n_frames, total, window, twiddle, melW, mel_lo, mel_hi, bn_mean, bn_var,
                     bn_weight, bn_bias, out);
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
  hipLaunchKernelGGL(patch_embed_kernel, dim3(cdiv(ntok, 64)), dim3(256), 0, S(stream), img, w, b,
                     ln_w, ln_b, x, ntok);
  ZS_LAUNCH_CHECK();
  return 0;
}

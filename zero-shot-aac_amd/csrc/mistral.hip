// Mistral-7B caption decoder (BASELINE.json config C5): fp8 weight streaming for the batch-32
// greedy decode of predict_mistralai_multilingual.py:105-111 (MistralForCausalLM.generate over
// inputs_embeds = clap_to_gpt(prefix, hard prompt, language tag), models/caption_model.py:340-413).
//
// Design (MI355X): at 32 rows a decode step streams the 7.2 B weights once; bf16 would move
// 14.5 GB per token step, fp8 e4m3 (OCP) with one f32 scale per output channel 7.2 GB.  The
// weight-only fp8 GEMM converts each weight fragment to bf16 in registers
// (v_cvt_scalef32_pk_bf16_fp8, exact) and runs bf16 MFMA with f32 accumulation against bf16
// activations, so activations keep bf16 precision.  RMSNorm weights are folded into the GEMM that
// follows them at load time (W'[n,k] = W[n,k] g[k], before quantisation), so the norms only
// normalise.
//
// Split-K without atomics: a GEMM writes f32 partial slabs [split][M][N]; the kernel that consumes
// its output (RoPE + KV append, SiLU * up, residual add + RMSNorm) sums the slabs in a fixed order,
// so results are deterministic and no extra reduction launch exists.  The f32 / bf16 weight modes
// reuse the same consumers with one slab written by zs_gemm.
#include "common.h"

namespace zs {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8m_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2m_t;
typedef __attribute__((ext_vector_type(4))) float f32x4m_t;

constexpr int F8_NT = 64;     // columns per workgroup (4 waves x 16)
constexpr int F8_KC = 1024;   // k per workgroup (one split)
constexpr int F8_MAXM = 64;

// out[split][m][n] = scale[n] * sum_{k in split} A[m][k] * W8[n][k]   (M <= 64)
// Lane l of a wave covers column n = l & 15 of the wave's 16; in each 64-deep k block lane group
// g = l >> 4 loads the 16 consecutive fp8 at k = 64 j + 16 g (one 16-byte load) and feeds them as
// two MFMA k-slices of 8; A is read from LDS with the same k assignment, so the products pair up
// (the sum runs over a permuted k order).
__global__ __launch_bounds__(256) void fp8_gemm_rows_kernel(const bf16_t* __restrict__ A, int lda,
                                                            const uint8_t* __restrict__ W8,
                                                            const float* __restrict__ scale, int M,
                                                            int N, int K, float* __restrict__ out,
                                                            long split_stride, int ldo) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* as = reinterpret_cast<bf16_t*>(smem);      // [M][F8_KC + 8]
  constexpr int LDA_S = F8_KC + 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * F8_NT + wid * 16;
  const int split = blockIdx.y, k0 = split * F8_KC;
  const int kc = min(F8_KC, K - k0);                 // multiple of 64
  const int fr = lane & 15, g = lane >> 4;
  // weight loads first (independent of A): kc / 64 blocks of 16 bytes per lane
  const int nrow = min(n0 + fr, N - 1);
  const uint8_t* wr = W8 + (long)nrow * K + k0 + 16 * g;
  uint4 wv[F8_KC / 64];
#pragma unroll
  for (int j = 0; j < F8_KC / 64; ++j)
    if (64 * j < kc) wv[j] = *reinterpret_cast<const uint4*>(wr + 64 * j);
  // A chunk -> LDS (16 bytes per thread per step)
  const int per_row = kc / 8;
  for (int i = threadIdx.x; i < M * per_row; i += 256) {
    const int m = i / per_row, c = (i % per_row) * 8;
    *reinterpret_cast<uint4*>(as + m * LDA_S + c) =
        *reinterpret_cast<const uint4*>(A + (long)m * lda + k0 + c);
  }
  __syncthreads();
  const int nrb = (M + 15) / 16;
  f32x4m_t acc[F8_MAXM / 16];
#pragma unroll
  for (int rb = 0; rb < F8_MAXM / 16; ++rb) acc[rb] = f32x4m_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < F8_KC / 64; ++j) {
    if (64 * j >= kc) break;
    const uint4 w = wv[j];
    bf16x8m_t b0, b1;
    {
      const bf16x2m_t p0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.x, 1.0f, false);
      const bf16x2m_t p1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.x, 1.0f, true);
      const bf16x2m_t p2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.y, 1.0f, false);
      const bf16x2m_t p3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.y, 1.0f, true);
      b0 = bf16x8m_t{p0[0], p0[1], p1[0], p1[1], p2[0], p2[1], p3[0], p3[1]};
      const bf16x2m_t q0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.z, 1.0f, false);
      const bf16x2m_t q1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.z, 1.0f, true);
      const bf16x2m_t q2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.w, 1.0f, false);
      const bf16x2m_t q3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.w, 1.0f, true);
      b1 = bf16x8m_t{q0[0], q0[1], q1[0], q1[1], q2[0], q2[1], q3[0], q3[1]};
    }
    const int ka = 64 * j + 16 * g;
#pragma unroll
    for (int rb = 0; rb < F8_MAXM / 16; ++rb) {
      if (rb >= nrb) break;
      const int m = min(rb * 16 + fr, M - 1);
      const bf16x8m_t a0 = *reinterpret_cast<const bf16x8m_t*>(as + m * LDA_S + ka);
      const bf16x8m_t a1 = *reinterpret_cast<const bf16x8m_t*>(as + m * LDA_S + ka + 8);
      acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc[rb], 0, 0, 0);
      acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc[rb], 0, 0, 0);
    }
  }
  // C layout: lane -> column n0 + (lane & 15), rows 16 rb + 4 (lane >> 4) + i
  const int n = n0 + fr;
  if (n >= N) return;
  const float s = scale[n];
  float* o = out + split * split_stride;
#pragma unroll
  for (int rb = 0; rb < F8_MAXM / 16; ++rb) {
    if (rb >= nrb) break;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = rb * 16 + 4 * g + i;
      if (m < M) o[(long)m * ldo + n] = acc[rb][i] * s;
    }
  }
}

// ---------------------------------------------------------------- consumers of the slabs
__device__ __forceinline__ float slab_sum(const float* __restrict__ p, int nsplit, long ss) {
  float v = p[0];
  for (int s = 1; s < nsplit; ++s) v += p[s * ss];
  return v;
}

// x[m] += sum_s y[s][m]  (skipped when y == nullptr), then h[m] = w * (x[m] * rsqrt(mean(x^2) +
// eps)) (MistralRMSNorm; w == nullptr: the weight is folded into the next GEMM), one block per row
template <typename T>
__global__ __launch_bounds__(256) void mistral_add_rmsnorm_kernel(
    float* __restrict__ x, const float* __restrict__ y, int nsplit, long ss, int D, float eps,
    const float* __restrict__ w, T* __restrict__ h) {
  __shared__ float red[4];
  const int m = blockIdx.x;
  float* xr = x + (long)m * D;
  float q = 0.f;
  for (int c = threadIdx.x; c < D; c += 256) {
    float v = xr[c];
    if (y) {
      v += slab_sum(y + (long)m * D + c, nsplit, ss);
      xr[c] = v;
    }
    q += v * v;
  }
  const float r = rsqrtf(block_sum(q, red) / D + eps);
  for (int c = threadIdx.x; c < D; c += 256)
    stf(h + (long)m * D + c, w ? w[c] * (xr[c] * r) : xr[c] * r);
}

// prefill input rows (predict_mistralai_multilingual.py:97-107 clap_to_gpt): row b*P + i is
// embed[hard[b][i]] for i < H (pads included: the reference attends to them), soft[b][i-H] for
// the next ns rows, embed[tail[i-H-ns]] (the language tag's ids) after; decode rows embed[tok[m]]
template <typename T>
__global__ __launch_bounds__(256) void mistral_embed_kernel(
    const int* __restrict__ hard, int H, const float* __restrict__ soft, int ns,
    const int* __restrict__ tail, int nt, const int* __restrict__ tok, const T* __restrict__ emb,
    int D, float* __restrict__ x) {
  const int m = blockIdx.x;
  const float* src = nullptr;
  int id = -1;
  if (tok) {
    id = tok[m];
  } else {
    const int P = H + ns + nt, b = m / P, i = m % P;
    if (i < H) id = hard[(long)b * H + i];
    else if (i < H + ns) src = soft + ((long)b * ns + (i - H)) * D;
    else id = tail[i - H - ns];
  }
  for (int c = threadIdx.x; c < D; c += 256)
    x[(long)m * D + c] = src ? src[c] : ldf(emb + (long)id * D + c);
}

// qkv slabs [split][M][(H + 2 KVH) * 128] -> RoPE(q) into q [M][H*128] (T), RoPE(k) and v into
// the caches [row][KVH][Lmax][128] at position pos[m] (row = m / rows_per_seq for the prefill's
// P rows per sequence); cos / sin tables [Lmax][64] from the host (HF's rotary embedding).
template <typename T>
__global__ __launch_bounds__(128) void mistral_rope_kv_kernel(
    const float* __restrict__ qkv, int nsplit, long ss, int H, int KVH, const int* __restrict__ pos,
    int rows_per_seq, const float* __restrict__ cosb, const float* __restrict__ sinb,
    T* __restrict__ q, T* __restrict__ kc, T* __restrict__ vc, int Lmax) {
  constexpr int HD = 128, HALF = 64;
  const int m = blockIdx.x, hh = blockIdx.y, i = threadIdx.x;   // hh < H + 2 KVH
  const int NQKV = (H + 2 * KVH) * HD;
  const float* src = qkv + (long)m * NQKV + hh * HD;
  const int p = pos[m];
  const int seq = m / rows_per_seq;
  if (hh < H + KVH) {                                           // q or k head: RoPE
    if (i >= HALF) return;
    const float a = slab_sum(src + i, nsplit, ss), b = slab_sum(src + i + HALF, nsplit, ss);
    const float c = cosb[(long)p * HALF + i], s = sinb[(long)p * HALF + i];
    const float lo = a * c - b * s, hi = b * c + a * s;
    if (hh < H) {
      T* qr = q + (long)m * H * HD + hh * HD;
      stf(qr + i, lo);
      stf(qr + i + HALF, hi);
    } else {
      T* kr = kc + (((long)seq * KVH + (hh - H)) * Lmax + p) * HD;
      stf(kr + i, lo);
      stf(kr + i + HALF, hi);
    }
  } else {                                                      // v head: copy
    T* vr = vc + (((long)seq * KVH + (hh - H - KVH)) * Lmax + p) * HD;
    stf(vr + i, slab_sum(src + i, nsplit, ss));
  }
}

// act[m][f] = silu(gate) * up from the gate|up slabs [split][M][2F] (T out)
template <typename T>
__global__ __launch_bounds__(256) void mistral_silu_mul_kernel(const float* __restrict__ gu,
                                                               int nsplit, long ss, int M, int F,
                                                               T* __restrict__ act) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)M * F) return;
  const int m = idx / F, f = idx % F;
  const float gt = slab_sum(gu + (long)m * 2 * F + f, nsplit, ss);
  const float up = slab_sum(gu + (long)m * 2 * F + F + f, nsplit, ss);
  stf(act + idx, gt / (1.0f + expf(-gt)) * up);     // F.silu(gate) * up
}

// causal GQA attention, one wave per (query row m, q head h): keys 0..pos[m] of the sequence
// m / rows_per_seq from kv head h / (H / KVH); softmax(q k^T / sqrt(128)) v, f32 math
template <typename T>
__global__ __launch_bounds__(256) void mistral_attn_kernel(const T* __restrict__ q, int M, int H,
                                                           int KVH, const int* __restrict__ pos,
                                                           int rows_per_seq,
                                                           const T* __restrict__ kc,
                                                           const T* __restrict__ vc, int Lmax,
                                                           T* __restrict__ out) {
  constexpr int HD = 128;
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= M * H) return;
  const int m = w / H, h = w % H, kvh = h / (H / KVH), seq = m / rows_per_seq;
  const int p = pos[m];
  const T* qr = q + (long)m * H * HD + h * HD;
  const float scale = 0.08838834764831845f;                      // 128^-0.5 (HF: (q k^T) * s)
  const float q0 = ldf(qr + lane), q1 = ldf(qr + lane + 64);
  const long base = ((long)seq * KVH + kvh) * Lmax;
  float mx = -INFINITY, l = 0.f, o0 = 0.f, o1 = 0.f;
  for (int j = 0; j <= p; ++j) {
    const T* kr = kc + (base + j) * HD;
    const float s = wave_sum(q0 * ldf(kr + lane) + q1 * ldf(kr + lane + 64)) * scale;
    const float mn = fmaxf(mx, s);
    float corr, e;
    if constexpr (sizeof(T) == 4) { corr = expf(mx - mn); e = expf(s - mn); }   // parity mode
    else { corr = __expf(mx - mn); e = __expf(s - mn); }
    const T* vr = vc + (base + j) * HD;
    l = l * corr + e;
    o0 = o0 * corr + e * ldf(vr + lane);
    o1 = o1 * corr + e * ldf(vr + lane + 64);
    mx = mn;
  }
  const float inv = 1.0f / l;
  T* orow = out + (long)m * H * HD + h * HD;
  stf(orow + lane, o0 * inv);
  stf(orow + lane + 64, o1 * inv);
}

}  // namespace zs

using namespace zs;

extern "C" int zs_fp8_gemm_rows(const void* A, int lda, const void* W8, const float* scale, int M,
                                int N, int K, float* out, long split_stride, int ldo,
                                void* stream) {
  ZS_REQUIRE(M > 0 && M <= F8_MAXM && N > 0 && K > 0 && K % 64 == 0,
             "zs_fp8_gemm_rows: 1 <= M <= %d, K %% 64 == 0 (M=%d N=%d K=%d)", F8_MAXM, M, N, K);
  ZS_REQUIRE(lda % 8 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)W8 & 15) == 0 && K % 16 == 0,
             "zs_fp8_gemm_rows: 16-byte aligned A / W rows");
  ZS_REQUIRE(split_stride >= (long)(M - 1) * ldo + N && ldo >= N, "zs_fp8_gemm_rows: out layout");
  const dim3 grid(cdiv(N, F8_NT), cdiv(K, F8_KC));
  const size_t lds = (size_t)M * (F8_KC + 8) * 2;
  hipLaunchKernelGGL(fp8_gemm_rows_kernel, grid, dim3(256), lds, S(stream), (const bf16_t*)A, lda,
                     (const uint8_t*)W8, scale, M, N, K, out, split_stride, ldo);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_fp8_splits(int K) { return K > 0 ? cdiv(K, F8_KC) : 0; }

extern "C" int zs_mistral_embed(const int* hard, int H, const float* soft, int ns, const int* tail,
                                int nt, const int* tok, const void* emb, int D, int M, float* x,
                                int dtype, void* stream) {
  ZS_REQUIRE(M > 0 && D > 0 && emb && x && (tok || (H + ns + nt > 0 && (ns == 0 || soft))),
             "zs_mistral_embed: bad arguments");
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(mistral_embed_kernel<bf16_t>, dim3(M), dim3(256), 0, S(stream), hard, H,
                       soft, ns, tail, nt, tok, (const bf16_t*)emb, D, x);
  else
    hipLaunchKernelGGL(mistral_embed_kernel<float>, dim3(M), dim3(256), 0, S(stream), hard, H,
                       soft, ns, tail, nt, tok, (const float*)emb, D, x);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_mistral_add_rmsnorm(float* x, const float* y, int nsplit, long ss, int M, int D,
                                      float eps, const float* w, void* h, int hdtype,
                                      void* stream) {
  ZS_REQUIRE(M > 0 && D > 0 && x && h && (y == nullptr || nsplit >= 1),
             "zs_mistral_add_rmsnorm: bad arguments");
  if (hdtype == ZS_BF16)
    hipLaunchKernelGGL(mistral_add_rmsnorm_kernel<bf16_t>, dim3(M), dim3(256), 0, S(stream), x, y,
                       nsplit, ss, D, eps, w, (bf16_t*)h);
  else
    hipLaunchKernelGGL(mistral_add_rmsnorm_kernel<float>, dim3(M), dim3(256), 0, S(stream), x, y,
                       nsplit, ss, D, eps, w, (float*)h);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_mistral_rope_kv(const float* qkv, int nsplit, long ss, int M, int H, int KVH,
                                  const int* pos, int rows_per_seq, const float* cosb,
                                  const float* sinb, void* q, void* kc, void* vc, int Lmax,
                                  int dtype, void* stream) {
  ZS_REQUIRE(M > 0 && H > 0 && KVH > 0 && H % KVH == 0 && rows_per_seq > 0 && nsplit >= 1,
             "zs_mistral_rope_kv: bad shape");
  const dim3 grid(M, H + 2 * KVH);
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(mistral_rope_kv_kernel<bf16_t>, grid, dim3(128), 0, S(stream), qkv, nsplit,
                       ss, H, KVH, pos, rows_per_seq, cosb, sinb, (bf16_t*)q, (bf16_t*)kc,
                       (bf16_t*)vc, Lmax);
  else
    hipLaunchKernelGGL(mistral_rope_kv_kernel<float>, grid, dim3(128), 0, S(stream), qkv, nsplit,
                       ss, H, KVH, pos, rows_per_seq, cosb, sinb, (float*)q, (float*)kc,
                       (float*)vc, Lmax);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_mistral_silu_mul(const float* gu, int nsplit, long ss, int M, int F, void* act,
                                   int dtype, void* stream) {
  ZS_REQUIRE(M > 0 && F > 0 && nsplit >= 1, "zs_mistral_silu_mul: bad shape");
  const int nb = cdiv((long)M * F, 256);
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(mistral_silu_mul_kernel<bf16_t>, dim3(nb), dim3(256), 0, S(stream), gu,
                       nsplit, ss, M, F, (bf16_t*)act);
  else
    hipLaunchKernelGGL(mistral_silu_mul_kernel<float>, dim3(nb), dim3(256), 0, S(stream), gu,
                       nsplit, ss, M, F, (float*)act);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_mistral_attention(const void* q, int M, int H, int KVH, const int* pos,
                                    int rows_per_seq, const void* kc, const void* vc, int Lmax,
                                    void* out, int dtype, void* stream) {
  ZS_REQUIRE(M > 0 && H > 0 && KVH > 0 && H % KVH == 0 && rows_per_seq > 0 && Lmax > 0,
             "zs_mistral_attention: bad shape");
  const dim3 grid(cdiv((long)M * H, 4));
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(mistral_attn_kernel<bf16_t>, grid, dim3(256), 0, S(stream),
                       (const bf16_t*)q, M, H, KVH, pos, rows_per_seq, (const bf16_t*)kc,
                       (const bf16_t*)vc, Lmax, (bf16_t*)out);
  else
    hipLaunchKernelGGL(mistral_attn_kernel<float>, grid, dim3(256), 0, S(stream), (const float*)q,
                       M, H, KVH, pos, rows_per_seq, (const float*)kc, (const float*)vc, Lmax,
                       (float*)out);
  ZS_LAUNCH_CHECK();
  return 0;
}

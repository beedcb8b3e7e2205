// Fused attention half of a GPT-2 decode step at small batch (R <= 64 rows, bf16): for one
// (16-row group, head) per workgroup
//
//   h = LayerNorm(x) (ln_1)  ->  q, k, v = h @ W_{q,k,v; head}^T + b  ->  k, v appended to the
//   KV cache at each row's position  ->  softmax(q k^T / 8) v over the row's cached keys + itself
//
// which replaces the ln_1 -> attn.c_attn launch and the decode attention launch of one
// transformers GPT2Block step (GPT2Attention with a KV cache: past keys/values concatenated with
// the new token's, causal, scale 1/sqrt(64)).  At 64 rows those two launches were dependency
// chains of ~9 us and ~8 us; here the q/k/v of a head never leave the workgroup.
//
// Layout: 1024 threads = 16 waves.  LN: wave w normalises row w (full row in registers, wave
// reductions) into a bf16 LDS image.  QKV: the head's 192 output columns are 12 tiles of 16
// (q 0-3, k 4-7, v 8-11); wave w = (column group w & 3: tiles 3(w&3)..+2, K quarter w >> 2),
// v_mfma_f32_16x16x32_bf16 with A from LDS and the weight fragments loaded straight to
// registers (all issued before the LN); the 4 K-quarter partials are summed through LDS in
// order.  Attention: wave w = row w, lanes = 8 key slots x 8 dims, keys in phases of 64 loaded
// branch-free (decode_attn6's arithmetic: q, k, v rounded to bf16 as the unfused path stores
// them, online softmax across phases, f32 statistics).
#include "common.h"

namespace zs {

typedef __attribute__((ext_vector_type(8))) __bf16 df_bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float df_f32x4_t;

constexpr int DF_D = 768, DF_HEADS = 12, DF_HD = 64, DF_RG = 16, DF_NCOL = 3 * DF_HD;
constexpr int DF_LDH = DF_D + 8;                 // padded bf16 LN row (conflict-free b128 reads)
constexpr int DF_KPP = 64, DF_NG = DF_KPP / 8;   // keys per phase, key groups per lane

struct QkvAttnArgs {
  int R, Lmax, rgroups;
  const float* x;                  // [R][768] f32 residual stream
  const float* ln_w; const float* ln_b; float eps;
  const bf16_t* W;                 // c_attn weight [2304][768] (out x in), rows q | k | v
  const float* bias;               // [2304]
  bf16_t* kc; bf16_t* vc;          // [R][12][Lmax][64]
  const int* pos;                  // [R] position of the new token
  bf16_t* out;                     // [R][768] attention output (heads concatenated)
};

__device__ __forceinline__ void df_unpack8(const uint4& u, float (&f)[8]) {
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
  f[4] = __uint_as_float(u.z << 16); f[5] = __uint_as_float(u.z & 0xffff0000u);
  f[6] = __uint_as_float(u.w << 16); f[7] = __uint_as_float(u.w & 0xffff0000u);
}
__device__ __forceinline__ uint32_t df_pack2(float a, float b) {
  return pk2bf(a, b);
}
__device__ __forceinline__ uint4 df_sel(bool c, const uint4& a, const uint4& b) {
  return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

__global__ __launch_bounds__(1024) void decode_qkv_attn_kernel(QkvAttnArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* hs = reinterpret_cast<bf16_t*>(smem);                              // [16][776]
  float* red = reinterpret_cast<float*>(smem + DF_RG * DF_LDH * 2);         // [4][16][192]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // units (head, row group), the row groups of a head consecutive -> one XCD (bijective remap)
  const int nwg = gridDim.x, id = blockIdx.x, xcd = id & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
  const int h = u / g.rgroups, m0 = (u % g.rgroups) * DF_RG;

  // ---- loads, all issued before any is used
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const int cg = wid & 3, kq = wid >> 2;            // column group (3 tiles), K quarter
  constexpr int S = DF_D / 4 / 32;                  // 6 k-steps of 32 per K quarter
  df_bf16x8_t b[S][3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int t = 3 * cg + j;                       // tile: q 0-3, k 4-7, v 8-11
    const bf16_t* wr = g.W + (long)((t >> 2) * DF_D + h * DF_HD + (t & 3) * 16 + fr) * DF_D;
#pragma unroll
    for (int s = 0; s < S; ++s)
      b[s][j] = *reinterpret_cast<const df_bf16x8_t*>(wr + kq * (DF_D / 4) + 32 * s + fk);
  }
  const int row = m0 + wid;                         // this wave's row (LN, KV append, attention)
  const bool rowv = row < g.R;
  const int rr = min(row, g.R - 1);
  const float4* xr = reinterpret_cast<const float4*>(g.x + (long)rr * DF_D);
  float4 xv[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) xv[i] = xr[lane + 64 * i];
  const int p = __builtin_amdgcn_readfirstlane(min(g.pos[rr], g.Lmax - 1));
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // ---- ln_1: wave w normalises row w
  {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) s += (xv[i].x + xv[i].y) + (xv[i].z + xv[i].w);
    const float mean = wave_sum(s) * (1.0f / DF_D);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float a0 = xv[i].x - mean, a1 = xv[i].y - mean, a2 = xv[i].z - mean, a3 = xv[i].w - mean;
      q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
    const float rstd = rsqrtf(wave_sum(q) * (1.0f / DF_D) + g.eps);
    // LN parameters (L2-resident) fetched here: holding them with the weight fragments and x
    // from the start exceeds the 128 VGPRs of a 1024-thread workgroup
    float4 lw[3], lb[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      lw[i] = reinterpret_cast<const float4*>(g.ln_w)[lane + 64 * i];
      lb[i] = reinterpret_cast<const float4*>(g.ln_b)[lane + 64 * i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int c = lane + 64 * i;
      uint2 pk;
      pk.x = df_pack2((xv[i].x - mean) * rstd * lw[i].x + lb[i].x,
                      (xv[i].y - mean) * rstd * lw[i].y + lb[i].y);
      pk.y = df_pack2((xv[i].z - mean) * rstd * lw[i].z + lb[i].z,
                      (xv[i].w - mean) * rstd * lw[i].w + lb[i].w);
      *reinterpret_cast<uint2*>(hs + wid * DF_LDH + 4 * c) = pk;
    }
  }
  __syncthreads();

  // ---- q, k, v of this head for the 16 rows: K-quarter partials -> LDS
  {
    df_f32x4_t acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[j] = df_f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const df_bf16x8_t af =
          *reinterpret_cast<const df_bf16x8_t*>(hs + fr * DF_LDH + kq * (DF_D / 4) + 32 * s + fk);
#pragma unroll
      for (int j = 0; j < 3; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b[s][j], acc[j], 0, 0, 0);
    }
    float* mine = red + kq * DF_RG * DF_NCOL;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        mine[(4 * (lane >> 4) + i) * DF_NCOL + 16 * (3 * cg + j) + fr] = acc[j][i];
  }
  __syncthreads();
  // sum the K quarters in order + bias, round to bf16 (the unfused path stores qkv as bf16);
  // the result overwrites quarter 0 (each element is read and written by one thread)
  for (int e = threadIdx.x; e < DF_RG * DF_NCOL; e += 1024) {
    const int r = e / DF_NCOL, c = e % DF_NCOL;
    const float v = ((red[e] + red[DF_RG * DF_NCOL + e]) + red[2 * DF_RG * DF_NCOL + e]) +
                    red[3 * DF_RG * DF_NCOL + e];
    const int n = (c >> 6) * DF_D + h * DF_HD + (c & 63);
    red[e] = bf2f(f2bf(v + g.bias[n]));
    (void)r;
  }
  __syncthreads();
  if (!rowv) return;                                // no barrier below

  // ---- this wave's row: append k, v; attention over keys 0..p
  const float* qkvr = red + wid * DF_NCOL;          // q | k | v of (row, head), bf16 values
  const int grp = lane >> 3, sub = lane & 7;
  const long rh = ((long)row * DF_HEADS + h) * g.Lmax;
  const float4 k0 = *reinterpret_cast<const float4*>(qkvr + DF_HD + 8 * sub);
  const float4 k1 = *reinterpret_cast<const float4*>(qkvr + DF_HD + 8 * sub + 4);
  const float4 v0 = *reinterpret_cast<const float4*>(qkvr + 2 * DF_HD + 8 * sub);
  const float4 v1 = *reinterpret_cast<const float4*>(qkvr + 2 * DF_HD + 8 * sub + 4);
  const uint4 knu = make_uint4(df_pack2(k0.x, k0.y), df_pack2(k0.z, k0.w), df_pack2(k1.x, k1.y),
                               df_pack2(k1.z, k1.w));
  const uint4 vnu = make_uint4(df_pack2(v0.x, v0.y), df_pack2(v0.z, v0.w), df_pack2(v1.x, v1.y),
                               df_pack2(v1.z, v1.w));
  if (grp == 0) {
    *reinterpret_cast<uint4*>(g.kc + (rh + p) * DF_HD + sub * 8) = knu;
    *reinterpret_cast<uint4*>(g.vc + (rh + p) * DF_HD + sub * 8) = vnu;
  }
  float q[8];
  {
    const float4 q0 = *reinterpret_cast<const float4*>(qkvr + 8 * sub);
    const float4 q1 = *reinterpret_cast<const float4*>(qkvr + 8 * sub + 4);
    q[0] = q0.x * 0.125f; q[1] = q0.y * 0.125f; q[2] = q0.z * 0.125f; q[3] = q0.w * 0.125f;
    q[4] = q1.x * 0.125f; q[5] = q1.y * 0.125f; q[6] = q1.z * 0.125f; q[7] = q1.w * 0.125f;
  }
  float m = -INFINITY, sum = 0.f, o[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) o[t] = 0.f;
  for (int base = 0; base <= p; base += DF_KPP) {
    uint4 kr[DF_NG], vr[DF_NG];
#pragma unroll
    for (int i = 0; i < DF_NG; ++i) {            // branch-free: cached slots < p only
      const int jc = max(min(base + i * 8 + grp, p - 1), 0);
      kr[i] = *reinterpret_cast<const uint4*>(g.kc + (rh + jc) * DF_HD + sub * 8);
      vr[i] = *reinterpret_cast<const uint4*>(g.vc + (rh + jc) * DF_HD + sub * 8);
    }
    float sc[DF_NG];
    float pm = -INFINITY;
#pragma unroll
    for (int i = 0; i < DF_NG; ++i) {
      const int j = base + i * 8 + grp;
      const uint4 z = make_uint4(0, 0, 0, 0);
      kr[i] = df_sel(j < p, kr[i], df_sel(j == p, knu, z));
      vr[i] = df_sel(j < p, vr[i], df_sel(j == p, vnu, z));
      float kf[8];
      df_unpack8(kr[i], kf);
      float sv = 0.f;
#pragma unroll
      for (int t = 0; t < 8; ++t) sv += q[t] * kf[t];
      sv += __shfl_xor(sv, 1, 64);
      sv += __shfl_xor(sv, 2, 64);
      sv += __shfl_xor(sv, 4, 64);
      sc[i] = j <= p ? sv : -INFINITY;
      pm = fmaxf(pm, sc[i]);
    }
    pm = fmaxf(pm, __shfl_xor(pm, 8, 64));
    pm = fmaxf(pm, __shfl_xor(pm, 16, 64));
    pm = fmaxf(pm, __shfl_xor(pm, 32, 64));
    const float mn = fmaxf(m, pm);
    const float scale = expf(m - mn);              // 0 on the first phase (m = -inf)
    sum *= scale;
#pragma unroll
    for (int t = 0; t < 8; ++t) o[t] *= scale;
    m = mn;
#pragma unroll
    for (int i = 0; i < DF_NG; ++i) {
      const float e = (base + i * 8 + grp <= p) ? expf(sc[i] - m) : 0.f;
      sum += e;
      float vf[8];
      df_unpack8(vr[i], vf);
#pragma unroll
      for (int t = 0; t < 8; ++t) o[t] += e * vf[t];
    }
  }
#pragma unroll
  for (int d = 8; d < 64; d <<= 1) {
    sum += __shfl_xor(sum, d, 64);
#pragma unroll
    for (int t = 0; t < 8; ++t) o[t] += __shfl_xor(o[t], d, 64);
  }
  if (grp == 0) {
    const float inv = 1.0f / sum;
    *reinterpret_cast<uint4*>(g.out + (long)row * DF_D + h * DF_HD + sub * 8) =
        make_uint4(df_pack2(o[0] * inv, o[1] * inv), df_pack2(o[2] * inv, o[3] * inv),
                   df_pack2(o[4] * inv, o[5] * inv), df_pack2(o[6] * inv, o[7] * inv));
  }
}

}  // namespace zs

using namespace zs;

extern "C" int zs_decode_qkv_attention(int R, const float* x, const float* ln_w,
                                       const float* ln_b, float eps, const void* w_qkv,
                                       const float* b_qkv, void* kc, void* vc, int Lmax,
                                       const int* pos, void* out, void* stream) {
  ZS_REQUIRE(R > 0 && R <= 64, "zs_decode_qkv_attention: R in 1..64 (got %d)", R);
  ZS_REQUIRE(Lmax > 0 && Lmax <= 4096, "zs_decode_qkv_attention: Lmax");
  ZS_REQUIRE(x && ln_w && ln_b && w_qkv && b_qkv && kc && vc && pos && out,
             "zs_decode_qkv_attention: null pointer");
  ZS_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)ln_w & 15) == 0 &&
             ((uintptr_t)ln_b & 15) == 0 && ((uintptr_t)w_qkv & 15) == 0 &&
             ((uintptr_t)kc & 15) == 0 && ((uintptr_t)vc & 15) == 0 && ((uintptr_t)out & 15) == 0,
             "zs_decode_qkv_attention: 16-byte aligned operands");
  QkvAttnArgs g{R, Lmax, cdiv(R, DF_RG), x, ln_w, ln_b, eps, (const bf16_t*)w_qkv, b_qkv,
                (bf16_t*)kc, (bf16_t*)vc, pos, (bf16_t*)out};
  const size_t lds = (size_t)DF_RG * DF_LDH * 2 + (size_t)4 * DF_RG * DF_NCOL * 4;   // 74 KB
  static bool attr = false;
  if (!attr) {      // dynamic LDS above 64 KB (gfx950 has 160 KB per CU)
    ZS_CHECK_HIP(hipFuncSetAttribute((const void*)decode_qkv_attn_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL(decode_qkv_attn_kernel, dim3(g.rgroups * DF_HEADS), dim3(1024), lds,
                     S(stream), g);
  ZS_LAUNCH_CHECK();
  return 0;
}

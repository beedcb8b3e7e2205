// Fused HTSAT Swin block (bf16 operands, f32 residual stream): one workgroup per 8x8 window.
//
//   SwinTransformerBlock.forward, eval (ref:retrieval/models/htsat.py:427-474):
//     x = x + proj(W-MSA / SW-MSA(LN1(x)))        (htsat.py:269-350, roll 443-463, mask 406-425)
//     x = x + fc2(GELU(fc1(LN2(x))))              (Mlp htsat.py:129-148)
//
// The unfused path (LayerNorm -> qkv GEMM -> window attention -> proj GEMM -> LayerNorm -> fc1 ->
// fc2) moves every intermediate through HBM: at stage 1 (C = 96, 262144 tokens per 64-clip
// batch) that is ~1.45 GB per block against 200 MB for the residual stream alone.  Every token
// belongs to exactly one (shifted) window and both MLP and LayerNorm are per token, so the whole
// block runs window-locally: the workgroup reads its 64 tokens' residual rows once (roll folded
// into the row index), keeps LN outputs, q/k/v, attention output and the MLP hidden chunk in LDS
// and the proj output in registers, and writes the 64 rows back in place.
//
// GEMMs (qkv, proj, fc1, fc2) use v_mfma_f32_16x16x32_bf16 with the activations (64 tokens x K,
// bf16) in LDS and the weights streamed straight from global memory (L2-resident: 0.2-3.5 MB per
// block) in a fragment-packed layout, so every weight fragment is ONE contiguous 1 KiB
// wave-load (16 B per lane) that feeds 4 MFMAs (the 4 token tiles of 16).  Waves split the
// output columns: wave w owns n-tiles w, w+4, w+8, ...  Most products are computed TRANSPOSED
// (weights as the A operand, tokens on the accumulator's lane axis), so a lane ends up with 4
// consecutive output columns of one token: LayerNorm row sums need 2 cross-lane steps, and
// LDS / global writes of q, k, the MLP hidden chunk and the residual rows are 8-16 bytes wide.
// Only V is produced in the natural orientation (4 consecutive tokens of one dim per lane),
// which is exactly the V^T layout the attention's PV product reads.
//
// Packed weights (prepared once on the host, zsaac/encoder.py):
//   frag(nt, ks)[lane][j] = W[16 nt + (lane & 15)][32 ks + 8 (lane >> 4) + j]   (W is [N][K])
//   stored frag-major [N/16][K/32][64][8] bf16.
//   qkv: per group of G heads (G = waves / 2: 2 for C <= 192, 4 for C = 384), rows
//   [q h0..h(G-1), k h0.., v h0..] x 32 (head dim 24 zero-padded to 32), i.e. [NH/G][96 G][C]
//   before fragment packing; bias [NH/G][96 G] f32.
//
// Attention per (head, 32 queries) wave, as window_attn_mfma_kernel (attn.hip): S^T = K Q^T and
// O^T = V^T P^T on v_mfma_f32_32x32x16_bf16, rel-pos bias + shift mask, f32 softmax.
#include "common.h"

namespace zs {

typedef __attribute__((ext_vector_type(8))) __bf16 sw_bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 sw_bf16x4;
typedef __attribute__((ext_vector_type(4))) float sw_f32x4;
typedef __attribute__((ext_vector_type(16))) float sw_f32x16;

struct SwinArgs {
  float* x;                       // [B*H*W][C] f32, updated in place
  int H, W, shift;
  const float* ln1_w;
  const float* ln1_b;
  const uint4* wqkv;              // packed, see above
  const float* bqkv;              // [NH/2][192]
  const float* rel;               // [225][NH]
  const uint4* wproj;             // [C/16][C/32][64] fragments
  const float* bproj;
  const float* ln2_w;
  const float* ln2_b;
  const uint4* w1;                // [4C/16][C/32][64]
  const float* b1;
  const uint4* w2;                // [C/16][4C/32][64]
  const float* b2;
  int dbg;                        // experiment knob (zs_tune_set "swin_dbg"): 1 = GELU -> identity,
                                  // 2 = no rel-pos bias / mask lookups, 4 = skip the MLP
};

int g_swin_dbg = 0;
int g_swin_occ3 = 1;              // zs_tune_set "swin_occ3": C = 96 at 3 workgroups per CU

__device__ __forceinline__ sw_bf16x8 as_bf8(uint4 u) { return __builtin_bit_cast(sw_bf16x8, u); }

// Weight fragments in flight: D k-steps x NTW n-tile slots (1 KiB wave-loads from L2).  A GEMM
// consumes slot ks % D and immediately refills it with k-step ks + D, and the NEXT GEMM's first D
// k-steps are issued (wp_prefetch) as soon as the current GEMM has consumed its pipe — before
// the epilogue / attention / LayerNorm work in between — so the L2 latency of a phase's first
// k-steps hides behind the previous phase instead of stalling it.
template <int NTW, int D>
struct WPipe {
  uint4 b[D][NTW];
};

template <int NTW, int NTOT, int D, int NW>
__device__ __forceinline__ void wp_load(WPipe<NTW, D>& p, int slot, const uint4* __restrict__ Wp,
                                        int kstot, int ks, int nt0) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < NTW; ++j)
    if (NTOT % NW == 0 || nt0 + NW * j < NTOT)
      p.b[slot][j] = Wp[((long)(nt0 + NW * j) * kstot + ks) * 64 + l];
}

template <int NTW, int NTOT, int D, int NW>
__device__ __forceinline__ void wp_prefetch(WPipe<NTW, D>& p, const uint4* __restrict__ Wp,
                                            int kstot, int ks0, int nt0) {
#pragma unroll
  for (int s = 0; s < D; ++s) wp_load<NTW, NTOT, D, NW>(p, s, Wp, kstot, ks0 + s, nt0);
}

// acc[mi][j] += A[16 mi .. +16][k] * W[n-tile nt0 + NW j][k] over KS k-steps of 32 starting at
// global k-step ks0 of a packed matrix with kstot k-steps per n-tile; the pipe must hold k-steps
// ks0 .. ks0 + D - 1 (wp_prefetch).  A: LDS, row stride lda (elements).  Slots j with
// nt0 + NW j >= NTOT are skipped (wave-uniform; NW = waves per workgroup).
//   TRMASK bit j set: slot j is computed transposed (acc = W . A^T): lane -> token 16 mi + (l & 15),
//   registers i -> columns 16 nt + 4 (l >> 4) + i.  Clear: lane -> column 16 nt + (l & 15),
//   registers i -> tokens 16 mi + 4 (l >> 4) + i.
template <int NTW, int KS, int NTOT, int D, int NW, int TRMASK = (1 << NTW) - 1>
__device__ __forceinline__ void win_gemm(const bf16_t* A, int lda, WPipe<NTW, D>& p,
                                         const uint4* __restrict__ Wp, int kstot, int ks0, int nt0,
                                         sw_f32x4 (&acc)[4][NTW]) {
  static_assert(KS >= D, "pipe deeper than the GEMM");
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    sw_bf16x8 a[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
      a[mi] = *reinterpret_cast<const sw_bf16x8*>(A + (16 * mi + (l & 15)) * lda + 32 * ks +
                                                  8 * (l >> 4));
    const int slot = ks % D;
#pragma unroll
    for (int j = 0; j < NTW; ++j)
      if (NTOT % NW == 0 || nt0 + NW * j < NTOT) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          acc[mi][j] = ((TRMASK >> j) & 1)
                           ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(p.b[slot][j]), a[mi],
                                                                     acc[mi][j], 0, 0, 0)
                           : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mi], as_bf8(p.b[slot][j]),
                                                                     acc[mi][j], 0, 0, 0);
      }
    if (ks + D < KS) wp_load<NTW, NTOT, D, NW>(p, slot, Wp, kstot, ks0 + ks + D, nt0);
  }
}

// OCC: workgroups per CU.  C = 96 runs 3 (53 KB of LDS, <= 168 VGPRs: two-deep weight pipes and
// fc2 accumulated straight onto the residual registers), the wider blocks 2 (1 at C = 384).
template <int C, int OCC = 2>
struct SwinCfg {
  static constexpr int NW = C >= 384 ? 8 : 4;  // waves per workgroup
  static constexpr int G = NW / 2;           // heads per q/k/v group: one (head, 32 queries) per wave
  static constexpr int NH = C / 24;          // heads (head dim 24)
  static constexpr int NG = NH / G;          // head groups
  static constexpr int LD = OCC >= 3 ? C + 8 : C + 16;   // H / ATT row stride (elements): conflict-free reads
  static constexpr int HC = 48 * NW;         // MLP hidden chunk (3 n-tiles per wave)
  static constexpr int LDH = HC + 16;
  static constexpr int NCH = 4 * C / HC;
  static constexpr int NTP = C / 16;         // n-tiles of proj / fc2
  static constexpr int NTW = (NTP + NW - 1) / NW;   // per wave (max)
  static constexpr int DA = OCC >= 3 ? 2 : (C <= 96 || C >= 384) ? 3 : 2;   // weight pipe depth (k-steps): qkv / fc1
  static constexpr int DB = OCC >= 3 ? 2 : (C <= 96 || C >= 384) ? 3 : 2;   // proj / fc2
  static constexpr int SZ_H = 64 * LD * 2;
  static constexpr int OFF_H = 0, OFF_ATT = SZ_H, OFF_QKV = 2 * SZ_H;
  static constexpr int SZ_QKV = 3 * G * 64 * 32 * 2;   // Qs[G][64][32], Ks[G][64][32], Vt[G][32][64]
  static constexpr int OFF_BT = OFF_QKV + SZ_QKV;      // [G][225] f32
  static constexpr int OFF_ROW = OFF_BT + ((G * 225 * 4 + 15) & ~15);  // [64] int token rows
  static constexpr int LDS = OFF_ROW + 256;
  static constexpr int LDX = C + 4;                    // final f32 staging [64][C+4]
  static_assert(64 * LDX * 4 <= LDS, "output staging fits");
  static_assert(64 * LDH * 2 <= SZ_H + SZ_QKV, "hidden chunk fits ATT + QKV");
  static_assert(2 * NW * 64 * 4 <= SZ_QKV, "LN2 reduction fits QKV");
  static_assert(LDS * OCC <= 160 * 1024 || (OCC == 2 && LDS <= 160 * 1024), "LDS");
  static_assert(C % 96 == 0 && NH % G == 0 && (4 * C) % HC == 0 && C % (16 * NW / 4) == 0, "C");
};

template <int C, bool SH, int OCC>   // SH: shifted windows (shift = ws / 2 = 4, odd blocks)
__global__ __launch_bounds__((64 * SwinCfg<C, OCC>::NW), OCC) void swin_block_kernel(SwinArgs g) {
  using CF = SwinCfg<C, OCC>;
  constexpr int LD = CF::LD, NTW = CF::NTW, NTP = CF::NTP, KS = C / 32, NW = CF::NW, G = CF::G;
  constexpr int NT = 64 * NW, TPT = NW;      // threads; threads per token in the row passes
  __shared__ __attribute__((aligned(16))) char lds[CF::LDS];
  bf16_t* sH = reinterpret_cast<bf16_t*>(lds + CF::OFF_H);
  bf16_t* sATT = reinterpret_cast<bf16_t*>(lds + CF::OFF_ATT);
  bf16_t* sQ = reinterpret_cast<bf16_t*>(lds + CF::OFF_QKV);
  bf16_t* sK = sQ + G * 64 * 32;
  bf16_t* sVt = sK + G * 64 * 32;
  float* sBt = reinterpret_cast<float*>(lds + CF::OFF_BT);
  int* sRow = reinterpret_cast<int*>(lds + CF::OFF_ROW);

  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  constexpr int DA = CF::DA, DB = CF::DB, KH = CF::HC / 32;
  WPipe<3, DA> pa;        // qkv / fc1 weight fragments in flight
  WPipe<NTW, DB> pb;      // proj / fc2
  wp_prefetch<3, 3 * NW, DA, NW>(pa, g.wqkv, KS, 0, w);
  const int H = g.H, W = g.W;
  constexpr int shift = SH ? 4 : 0;
  const int nWw = W / 8, nWh = H / 8;
  const int win = blockIdx.x;
  const int b = win / (nWh * nWw), wyx = win % (nWh * nWw), wy = wyx / nWw, wx = wyx % nWw;

  // ---- P1: LN1.  thread = (token t = tid / TPT, part q = tid % TPT); the row is read as float4
  // chunks q, q+TPT, ... so the TPT threads of a token cover 16 TPT contiguous bytes per load.
  {
    constexpr int NQ = C / (4 * TPT);               // float4 chunks per thread
    const int t = tid / TPT, q = tid % TPT;
    const int sy = wy * 8 + (t >> 3), sx = wx * 8 + (t & 7);     // rolled coords
    const int hh = (sy + shift) % H, ww = (sx + shift) % W;      // natural (roll(-shift))
    const int row = (b * H + hh) * W + ww;
    if (q == 0) sRow[t] = row;
    const float4* xr = reinterpret_cast<const float4*>(g.x + (long)row * C);
    float4 v[NQ];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      v[j] = xr[TPT * j + q];
      s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    }
#pragma unroll
    for (int o = 1; o < TPT; o <<= 1) s += __shfl_xor(s, o, 64);
    const float mean = s * (1.0f / C);
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const float a0 = v[j].x - mean, a1 = v[j].y - mean, a2 = v[j].z - mean, a3 = v[j].w - mean;
      ss += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
#pragma unroll
    for (int o = 1; o < TPT; o <<= 1) ss += __shfl_xor(ss, o, 64);
    const float rstd = rsqrtf(ss * (1.0f / C) + 1e-5f);
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int c0 = (TPT * j + q) * 4;
      const float4 gw = *reinterpret_cast<const float4*>(g.ln1_w + c0);
      const float4 gb = *reinterpret_cast<const float4*>(g.ln1_b + c0);
      uint2 u;
      u.x = pk2bf((v[j].x - mean) * rstd * gw.x + gb.x, (v[j].y - mean) * rstd * gw.y + gb.y);
      u.y = pk2bf((v[j].z - mean) * rstd * gw.z + gb.z, (v[j].w - mean) * rstd * gw.w + gb.w);
      *reinterpret_cast<uint2*>(sH + t * LD + c0) = u;
    }
  }
  __syncthreads();

  // ---- P2: per group of 2 heads: qkv GEMM -> Q/K/V^T in LDS -> attention -> ATT
  const int r32 = l & 31, h2 = l >> 5;
  for (int grp = 0; grp < CF::NG; ++grp) {
    {
      sw_f32x4 acc[4][3];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[mi][j] = sw_f32x4{0.f, 0.f, 0.f, 0.f};
      // slot j of wave w is n-tile w + NW j = part j (q, k, v) of head w / 2, dims 16 (w & 1)..+16;
      // q and k transposed (token rows for the attention fragments), v natural (V^T rows)
      constexpr long GS = 3L * NW * KS * 64;       // fragments per head group
      win_gemm<3, KS, 3 * NW, DA, NW, 3>(sH, LD, pa, g.wqkv + grp * GS, KS, 0, w, acc);
      if (grp + 1 < CF::NG) wp_prefetch<3, 3 * NW, DA, NW>(pa, g.wqkv + (grp + 1) * GS, KS, 0, w);
      else wp_prefetch<NTW, NTP, DB, NW>(pb, g.wproj, KS, 0, w);
      for (int i = tid; i < G * 225; i += NT)
        sBt[i] = g.rel[(i % 225) * CF::NH + G * grp + i / 225];
      const int hh = w >> 1;
      const float* bq = g.bqkv + grp * 48 * NW;
#pragma unroll
      for (int j = 0; j < 2; ++j) {                      // q, k: lane = token, 4 dims
        const int d0 = (w & 1) * 16 + 4 * (l >> 4);
        const float4 bias = *reinterpret_cast<const float4*>(bq + (w + NW * j) * 16 + 4 * (l >> 4));
        bf16_t* base = (j == 0 ? sQ : sK) + hh * 2048;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const int t = 16 * mi + (l & 15);
          uint2 u;
          u.x = pk2bf(acc[mi][j][0] + bias.x, acc[mi][j][1] + bias.y);
          u.y = pk2bf(acc[mi][j][2] + bias.z, acc[mi][j][3] + bias.w);
          *reinterpret_cast<uint2*>(base + t * 32 + 8 * ((d0 >> 3) ^ ((t >> 2) & 3)) + (d0 & 7)) = u;
        }
      }
      {                                                  // v: lane = dim, 4 tokens -> V^T
        const int d = (w & 1) * 16 + (l & 15);
        const float bias = bq[(w + 2 * NW) * 16 + (l & 15)];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const int t0 = 16 * mi + 4 * (l >> 4);
          uint2 u;
          u.x = pk2bf(acc[mi][2][0] + bias, acc[mi][2][1] + bias);
          u.y = pk2bf(acc[mi][2][2] + bias, acc[mi][2][3] + bias);
          *reinterpret_cast<uint2*>(sVt + hh * 2048 + d * 64 + 4 * ((t0 >> 2) ^ (d & 15))) = u;
        }
      }
    }
    __syncthreads();
    {
      // wave = (head hh of the group, query block qb)
      const int hh = w >> 1, qb = w & 1;
      const bf16_t* Q = sQ + hh * 2048;
      const bf16_t* K = sK + hh * 2048;
      const bf16_t* Vt = sVt + hh * 2048;
      const float* Bt = sBt + hh * 225;
      sw_f32x16 st[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int e = 0; e < 16; ++e) st[kb][e] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = 2 * ks + h2;
        const int qrow = 32 * qb + r32;
        const sw_bf16x8 bq =
            *reinterpret_cast<const sw_bf16x8*>(Q + qrow * 32 + 8 * (c ^ ((qrow >> 2) & 3)));
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int krow = 32 * kb + r32;
          const sw_bf16x8 a =
              *reinterpret_cast<const sw_bf16x8*>(K + krow * 32 + 8 * (c ^ ((krow >> 2) & 3)));
          st[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bq, st[kb], 0, 0, 0);
        }
      }
      const float scale = 0.20412414523193148f;    // 24 ** -0.5 (htsat.py:285, 320)
      const int qi = 32 * qb + r32, qy = qi >> 3, qx = qi & 7;
      // key of register e of block kb: kj = 32 kb + (e & 3) + 8 (e >> 2) + 4 h2, i.e. key row
      // ky = 4 kb + (e >> 2), key column kx = 4 h2 + (e & 3): the bias index
      // (qy - ky + 7) * 15 + (qx - kx + 7) is a per-lane base minus a compile-time constant, so
      // every lookup is one ds_read with an immediate offset
      const float* bt0 = Bt + (qy + 7) * 15 + qx - 4 * h2 + 7 - 108;
      // shift-mask (htsat.py:406-425): only windows in the last window row / column have more
      // than one region; with shift 4 (= ws/2, the only shift HTSAT uses) a key's region row is
      // (ky >= 4) == kb and its region column (kx >= 4) == h2, so the mask is per (lane, kb)
      const bool lastr = wy == nWh - 1, lastc = wx == nWw - 1;
      float mk[2] = {0.f, 0.f};
      if (SH) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
          mk[kb] = ((lastr && kb != (qy >= 4)) || (lastc && h2 != (qx >= 4))) ? -100.0f : 0.f;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float v = st[kb][e] * scale;
          if (!(g.dbg & 2)) {
            v += bt0[108 - 15 * (4 * kb + (e >> 2)) - (e & 3)] + mk[kb];
          }
          st[kb][e] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float sum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float p = __expf(st[kb][e] - mx);
          st[kb][e] = p;
          sum += p;
        }
      sum += __shfl_xor(sum, 32, 64);
      sw_f32x16 ot;
#pragma unroll
      for (int e = 0; e < 16; ++e) ot[e] = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          sw_bf16x8 pb;
#pragma unroll
          for (int u = 0; u < 8; ++u) pb[u] = (__bf16)st[kb][8 * t + u];
          const int k0 = 32 * kb + 16 * t + 4 * h2, d = r32;
          const sw_bf16x4 lo = *reinterpret_cast<const sw_bf16x4*>(Vt + d * 64 + 4 * ((k0 >> 2) ^ (d & 15)));
          const sw_bf16x4 hi = *reinterpret_cast<const sw_bf16x4*>(Vt + d * 64 + 4 * (((k0 + 8) >> 2) ^ (d & 15)));
          sw_bf16x8 va;
#pragma unroll
          for (int u = 0; u < 4; ++u) { va[u] = lo[u]; va[4 + u] = hi[u]; }
          ot = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb, ot, 0, 0, 0);
        }
      const float inv = 1.0f / sum;
      bf16_t* orow = sATT + qi * LD + (G * grp + hh) * 24;
#pragma unroll
      for (int gq = 0; gq < 3; ++gq) {       // dims 8 gq + 4 h2 .. +3 (< 24)
        const int d0 = 8 * gq + 4 * h2;
        uint2 u;
        u.x = pk2bf(ot[4 * gq] * inv, ot[4 * gq + 1] * inv);
        u.y = pk2bf(ot[4 * gq + 2] * inv, ot[4 * gq + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d0) = u;
      }
    }
    __syncthreads();
  }

  // ---- P3: proj (transposed) + bias + residual -> x1 (registers: lane = token 16 mi + (l & 15),
  // x1[mi][j][i] = column 16 (w + NW j) + 4 (l >> 4) + i)
  sw_f32x4 x1[4][NTW];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int j = 0; j < NTW; ++j) x1[mi][j] = sw_f32x4{0.f, 0.f, 0.f, 0.f};
  win_gemm<NTW, KS, NTP, DB, NW>(sATT, LD, pb, g.wproj, KS, 0, w, x1);
  wp_prefetch<3, 3 * NW, DA, NW>(pa, g.w1, KS, 0, w);
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    if (NTP % NW == 0 || w + NW * j < NTP) {
      const int c0 = (w + NW * j) * 16 + 4 * (l >> 4);
      const float4 bias = *reinterpret_cast<const float4*>(g.bproj + c0);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const float4 xv =
            *reinterpret_cast<const float4*>(g.x + (long)sRow[16 * mi + (l & 15)] * C + c0);
        x1[mi][j][0] += bias.x + xv.x;
        x1[mi][j][1] += bias.y + xv.y;
        x1[mi][j][2] += bias.z + xv.z;
        x1[mi][j][3] += bias.w + xv.w;
      }
    }
  }

  // ---- P4: LN2 over x1: per-lane partial row sums, the 4 lanes of a token (xor 16, 32), then
  // the 4 waves through LDS; two passes (mean, then centred squares) as LN1
  {
    float* red = reinterpret_cast<float*>(lds + CF::OFF_QKV);     // [2][NW][64]
    float mean[4], rstd[4];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < NTW; ++j)
          if (NTP % NW == 0 || w + NW * j < NTP) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float v = pass == 0 ? x1[mi][j][i] : x1[mi][j][i] - mean[mi];
              a += pass == 0 ? v : v * v;
            }
          }
        a += __shfl_xor(a, 16, 64);
        a += __shfl_xor(a, 32, 64);
        if (l < 16) red[pass * NW * 64 + w * 64 + 16 * mi + l] = a;
      }
      __syncthreads();
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int t = 16 * mi + (l & 15);
        float tot = 0.f;
#pragma unroll
        for (int u = 0; u < NW; ++u) tot += red[pass * NW * 64 + u * 64 + t];
        if (pass == 0) mean[mi] = tot * (1.0f / C);
        else rstd[mi] = rsqrtf(tot * (1.0f / C) + 1e-5f);
      }
    }
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      if (NTP % NW == 0 || w + NW * j < NTP) {
        const int c0 = (w + NW * j) * 16 + 4 * (l >> 4);
        const float4 gw = *reinterpret_cast<const float4*>(g.ln2_w + c0);
        const float4 gb = *reinterpret_cast<const float4*>(g.ln2_b + c0);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const int t = 16 * mi + (l & 15);
          uint2 u;
          u.x = pk2bf((x1[mi][j][0] - mean[mi]) * rstd[mi] * gw.x + gb.x,
                      (x1[mi][j][1] - mean[mi]) * rstd[mi] * gw.y + gb.y);
          u.y = pk2bf((x1[mi][j][2] - mean[mi]) * rstd[mi] * gw.z + gb.z,
                      (x1[mi][j][3] - mean[mi]) * rstd[mi] * gw.w + gb.w);
          *reinterpret_cast<uint2*>(sH + t * LD + c0) = u;
        }
      }
    }
  }
  __syncthreads();

  // ---- P5: MLP in hidden chunks of HC: fc1 + GELU(erf) -> HID (LDS) -> fc2 accumulates
  // fc2 accumulates onto x1 + b2 (the residual registers double as the accumulator)
  sw_f32x4 (&acc2)[4][NTW] = x1;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    if (NTP % NW == 0 || w + NW * j < NTP) {
      const float4 bias = *reinterpret_cast<const float4*>(g.b2 + (w + NW * j) * 16 + 4 * (l >> 4));
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        acc2[mi][j][0] += bias.x; acc2[mi][j][1] += bias.y;
        acc2[mi][j][2] += bias.z; acc2[mi][j][3] += bias.w;
      }
    }
  }
  bf16_t* sHID = reinterpret_cast<bf16_t*>(lds + CF::OFF_ATT);
  for (int ch = 0; ch < ((g.dbg & 4) ? 0 : CF::NCH); ++ch) {
    {
      sw_f32x4 acc1[4][3];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc1[mi][j] = sw_f32x4{0.f, 0.f, 0.f, 0.f};
      win_gemm<3, KS, 3 * NW, DA, NW>(sH, LD, pa, g.w1 + (long)ch * 3 * NW * KS * 64, KS, 0, w, acc1);
      wp_prefetch<NTW, NTP, DB, NW>(pb, g.w2, 4 * C / 32, ch * KH, w);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int c0 = (w + NW * j) * 16 + 4 * (l >> 4);
        const float4 bias = *reinterpret_cast<const float4*>(g.b1 + ch * CF::HC + c0);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const int t = 16 * mi + (l & 15);
          float v0 = acc1[mi][j][0] + bias.x, v1 = acc1[mi][j][1] + bias.y;
          float v2 = acc1[mi][j][2] + bias.z, v3 = acc1[mi][j][3] + bias.w;
          if (!(g.dbg & 1)) {
            v0 = gelu_erf_fast(v0); v1 = gelu_erf_fast(v1);
            v2 = gelu_erf_fast(v2); v3 = gelu_erf_fast(v3);
          }
          uint2 u;
          u.x = pk2bf(v0, v1);
          u.y = pk2bf(v2, v3);
          *reinterpret_cast<uint2*>(sHID + t * CF::LDH + c0) = u;
        }
      }
    }
    __syncthreads();
    win_gemm<NTW, KH, NTP, DB, NW>(sHID, CF::LDH, pb, g.w2, 4 * C / 32, ch * KH, w, acc2);
    if (ch + 1 < CF::NCH)
      wp_prefetch<3, 3 * NW, DA, NW>(pa, g.w1 + (long)(ch + 1) * 3 * NW * KS * 64, KS, 0, w);
    __syncthreads();
  }

  // ---- P6: x = x1 + fc2 + bias -> LDS f32 staging -> coalesced float4 row stores (in place)
  float* sX = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    if (NTP % NW == 0 || w + NW * j < NTP) {
      const int c0 = (w + NW * j) * 16 + 4 * (l >> 4);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int t = 16 * mi + (l & 15);
        *reinterpret_cast<float4*>(sX + t * CF::LDX + c0) =
            make_float4(acc2[mi][j][0], acc2[mi][j][1], acc2[mi][j][2], acc2[mi][j][3]);
      }
    }
  }
  __syncthreads();
  {
    const int t = tid / TPT, q = tid % TPT;
    float4* xr = reinterpret_cast<float4*>(g.x + (long)sRow[t] * C);
#pragma unroll
    for (int j = 0; j < C / (4 * TPT); ++j)
      xr[TPT * j + q] = *reinterpret_cast<const float4*>(sX + t * CF::LDX + (TPT * j + q) * 4);
  }
}

}  // namespace zs

using namespace zs;

extern "C" int zs_swin_block(float* x, int B, int H, int W, int C, int heads, int shift,
                             const float* ln1_w, const float* ln1_b, const void* wqkv_packed,
                             const float* bqkv_packed, const float* rel_table,
                             const void* wproj_packed, const float* bproj, const float* ln2_w,
                             const float* ln2_b, const void* w1_packed, const float* b1,
                             const void* w2_packed, const float* b2, void* stream) {
  ZS_REQUIRE(B > 0 && H % 8 == 0 && W % 8 == 0 && H >= 8 && W >= 8,
             "zs_swin_block: H, W multiples of 8 (window 8)");
  ZS_REQUIRE((C == 96 || C == 192 || C == 384) && heads * 24 == C,
             "zs_swin_block: C in {96,192,384}, head dim 24 (C=%d heads=%d)", C, heads);
  ZS_REQUIRE(shift == 0 || shift == 4, "zs_swin_block: shift must be 0 or ws/2 = 4");
  ZS_REQUIRE((long)B * H * W <= (1L << 31) - 1, "zs_swin_block: too many tokens");
  SwinArgs a{x, H, W, shift, ln1_w, ln1_b, (const uint4*)wqkv_packed, bqkv_packed, rel_table,
             (const uint4*)wproj_packed, bproj, ln2_w, ln2_b, (const uint4*)w1_packed, b1,
             (const uint4*)w2_packed, b2, g_swin_dbg};
  dim3 grid(B * (H / 8) * (W / 8));
  hipStream_t st = S(stream);
#define SWL(C_, SH_, O_) \
  hipLaunchKernelGGL((swin_block_kernel<C_, SH_, O_>), grid, dim3(64 * SwinCfg<C_, O_>::NW), 0, st, a)
  if (C == 96 && g_swin_occ3) { if (shift) SWL(96, true, 3); else SWL(96, false, 3); }
  else if (C == 96) { if (shift) SWL(96, true, 2); else SWL(96, false, 2); }
  else if (C == 192) { if (shift) SWL(192, true, 2); else SWL(192, false, 2); }
  else { if (shift) SWL(384, true, 2); else SWL(384, false, 2); }
#undef SWL
  ZS_LAUNCH_CHECK();
  return 0;
}

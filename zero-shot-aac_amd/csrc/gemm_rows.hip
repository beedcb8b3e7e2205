// Row-group GEMM for M <= 64 rows (the GPT-2 decode step at the reference's eval batch of 64,
// the mapper and audio_proj at small batches), bf16 operands, f32 accumulation.
//
// At 64 rows a decode-step GEMM moves 1-5 MB of weights and almost no flops: its time is the
// dependency chain of one launch (dispatch, first loads, reduction, stores), not bandwidth.  The
// split-K skinny kernel (gemm_skinny.hip) pays two extra chip-wide round trips for its slab
// reduction (sc1 slab stores -> atomic ticket -> slab loads by the last arriver).  Here the
// parallelism comes from the ROWS instead: a work unit is (16-row group, NT-column tile) with the
// full K in one workgroup; the K range is split over the workgroup's waves only, whose partials
// are summed through LDS.  No global slabs, no atomics, one round trip from the first load to the
// store.  The 4 row groups of a column tile are consecutive work units on one XCD (bijective
// remap, cdna_hip_programming.md §5 T1), so the weight tile they share crosses HBM once.
//
// LN mode (zs_gemm_ln): the A operand is LayerNorm(x) of the f32 residual stream, computed in the
// prologue: the workgroup loads its 16 rows of x (48 KB at C = 768) while its weight loads are in
// flight, forms mean / variance in registers (two passes over the held values), and writes the
// normalised bf16 rows to LDS, from where the waves read their MFMA A fragments.  This replaces
// GPT-2's ln_1 -> c_attn and ln_2 -> c_fc launch pairs (transformers GPT2Block, eps 1e-5).
//
// MFMA: v_mfma_f32_16x16x32_bf16; lane l holds A[row l&15][k 8(l>>4)..+8] and
// W[n l&15][k 8(l>>4)..+8] (B = W^T), C col = l&15, rows 4(l>>4)+i.
// Per-row arithmetic depends only on (N, K): a row's result does not depend on M or on its row
// group, so a clip's result does not depend on how many clips share the launch.
#include "common.h"

namespace zs {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8r_t;
typedef __attribute__((ext_vector_type(4))) float f32x4r_t;

#ifdef ZS_STAMPS
// diagnostic build only (tools/hip/rows_stamps.cpp): s_memrealtime (100 MHz) stamps of each
// workgroup's phases, written by thread 0 into a buffer no other code reads
__device__ unsigned long long* zs_stamp_buf;
extern "C" int zs_set_stamp_buf(void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(zs_stamp_buf), &p, sizeof(p));
}
#define ZS_STAMP(slot)                                                                           \
  do {                                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    unsigned long long t_;                                                                       \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");              \
    if (threadIdx.x == 0 && zs_stamp_buf) zs_stamp_buf[blockIdx.x * 8 + (slot)] = t_;            \
    __builtin_amdgcn_sched_barrier(0);                                                           \
  } while (0)
#else
#define ZS_STAMP(slot) do {} while (0)
#endif

constexpr int RG = 16;              // rows per group
constexpr int RG_MAX_M = 64;
constexpr int RG_MAX_LOADS = 36;    // 16-byte loads in flight per lane (VGPR budget)

struct RowsArgs {
  int M, N, K;
  const bf16_t* A; int lda;                 // bf16 A operand (plain mode)
  const float* X; int ldx;                  // f32 rows (LN mode)
  const float* ln_w; const float* ln_b; float eps;
  const bf16_t* W; int ldw;
  const float* bias;
  const float* residual; int ldr;
  void* out; int ldo; int out_dtype; int act;
  int rgroups, ntiles;
  const float* Af; const float* Wf;         // f32 operands (gemm_rows_f32_kernel)
};

// 8-wave instances at <= 128 registers (4 waves per SIMD's worth): two of their waves per SIMD
// then fit beside a persistent decode workgroup (4 waves x 256 registers), so a begin's mapper
// GEMM does not wait for a decode grid to end
template <int NT, int WAVES, int LNM, int S>
#ifndef ZS_ROWS_MINB8
#define ZS_ROWS_MINB8 4   // (-DZS_ROWS_MINB8=1: round 4's unbounded registers, for the A/B)
#endif
__global__ __launch_bounds__(64 * WAVES, WAVES == 8 ? ZS_ROWS_MINB8 : 1) void gemm_rows_kernel(RowsArgs g) {
  constexpr bool LN = LNM != 0, AFF = LNM == 1;
  // S = 32-deep k-steps per wave (K = 32 * WAVES * S), a template parameter so that every load
  // is issued unconditionally and up front (a runtime trip count put each load in its own
  // branch and the compiler waited for it there: one round trip per load)
  constexpr int NB = NT / 16;
  constexpr int NTHR = 64 * WAVES;
  constexpr int K = 32 * WAVES * S, KW = K / WAVES;
  static_assert(S * (LN ? NB : NB + 1) <= RG_MAX_LOADS, "rows kernel: VGPR budget");
  // LDS: [LN rows: 16 x (K + 8) bf16] [partials: WAVES x 16 x NT f32]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  ZS_STAMP(0);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // XCD-aware bijective remap: blocks id, id+8, ... share an XCD -> consecutive work units
  const int nwg = gridDim.x, id = blockIdx.x, xcd = id & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
  const int rg = u % g.rgroups, tile = u / g.rgroups;
  const int m0 = rg * RG, n0 = tile * NT;
  const int kw = wid * KW;
  constexpr int ldh = K + 8;                // padded LDS row (conflict-free b128 fragment reads)
  bf16_t* hs = reinterpret_cast<bf16_t*>(smem);
  float* red = reinterpret_cast<float*>(smem + (LN ? RG * ldh * 2 : 0));

  const int fr = lane & 15, fk = 8 * (lane >> 4);
  // rows / columns past M / N load the last valid row / column (every load unconditional);
  // their outputs are never stored
  const int am = min(m0 + fr, g.M - 1);

  // epilogue operands (one column quad of one row per thread), issued before the operand
  // loads (the counted waits below then cover only the operands); loads clamped in range, masked by value
  constexpr int NQ = NT / 4;
  static_assert(RG * NQ <= NTHR, "one epilogue quad per thread");
  const bool epi = threadIdx.x < RG * NQ;
  const int erow = threadIdx.x / NQ, ecq = threadIdx.x % NQ;
  const int em = m0 + erow, en = n0 + 4 * ecq;
  float4 eb = make_float4(0.f, 0.f, 0.f, 0.f), er = eb;
  if (epi) {
    if (g.bias) {
      eb.x = g.bias[min(en, g.N - 1)];     eb.y = g.bias[min(en + 1, g.N - 1)];
      eb.z = g.bias[min(en + 2, g.N - 1)]; eb.w = g.bias[min(en + 3, g.N - 1)];
    }
    if (g.residual) {
      const float* rr = g.residual + (long)min(em, g.M - 1) * g.ldr;
      er.x = rr[min(en, g.N - 1)];     er.y = rr[min(en + 1, g.N - 1)];
      er.z = rr[min(en + 2, g.N - 1)]; er.w = rr[min(en + 3, g.N - 1)];
    }
  }
  // LN operands FIRST (loads return in order: the LayerNorm below then waits only for x, and
  // runs while the weight fragments are still in flight): 16 rows, TPR threads per row, NV
  // float4 per thread (column quads t, t+TPR, ..)
  constexpr int TPR = NTHR / RG, NV = LN ? K / (4 * TPR) : 1;
  static_assert(!LN || K % (4 * TPR) == 0, "LN rows: K % (4 * threads per row)");
  const int lr = threadIdx.x / TPR, lt = threadIdx.x % TPR;
  // (AFF: the LN weight / bias quads of this thread's columns; without AFF the caller folded
  // them into W and the bias, and the 2 x 16 row-threads' redundant loads of them go away)
  float4 xv[NV], lw[AFF ? NV : 1], lb[AFF ? NV : 1];
  if constexpr (LN) {
    const float4* xr = reinterpret_cast<const float4*>(g.X + (long)min(m0 + lr, g.M - 1) * g.ldx);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      xv[i] = xr[lt + TPR * i];
      if constexpr (AFF) {
        lw[i] = reinterpret_cast<const float4*>(g.ln_w)[lt + TPR * i];
        lb[i] = reinterpret_cast<const float4*>(g.ln_b)[lt + TPR * i];
      }
    }
  }
  // weight fragments for every k-step of this wave (straight-line code from here: the LN waits
  // for x alone, the MFMA loop consumes the fragments as they land)
  bf16x8r_t b[S * NB];
  bf16x8r_t a[LN ? 1 : S];
  const bf16_t* wrow[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) wrow[nb] = g.W + (long)min(n0 + 16 * nb + fr, g.N - 1) * g.ldw;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int k = kw + 32 * s + fk;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
      b[s * NB + nb] = *reinterpret_cast<const bf16x8r_t*>(wrow[nb] + k);
    if constexpr (!LN) a[s] = *reinterpret_cast<const bf16x8r_t*>(g.A + (long)am * g.lda + k);
  }
  // keep every load above in flight before any of them is used (the scheduler otherwise sinks
  // loads next to their MFMAs and waits on each group)
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  ZS_STAMP(1);
#ifdef ZS_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ZS_STAMP(2);
#endif

  if constexpr (LN) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += (xv[i].x + xv[i].y) + (xv[i].z + xv[i].w);
#pragma unroll
    for (int o = TPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s * (1.0f / K);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const float a0 = xv[i].x - mean, a1 = xv[i].y - mean, a2 = xv[i].z - mean, a3 = xv[i].w - mean;
      q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
#pragma unroll
    for (int o = TPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = rsqrtf(q * (1.0f / K) + g.eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lt + TPR * i;
      uint2 pk;
      if constexpr (AFF) {
        pk.x = pk2bf((xv[i].x - mean) * rstd * lw[i].x + lb[i].x,
                     (xv[i].y - mean) * rstd * lw[i].y + lb[i].y);
        pk.y = pk2bf((xv[i].z - mean) * rstd * lw[i].z + lb[i].z,
                     (xv[i].w - mean) * rstd * lw[i].w + lb[i].w);
      } else {
        pk.x = pk2bf((xv[i].x - mean) * rstd, (xv[i].y - mean) * rstd);
        pk.y = pk2bf((xv[i].z - mean) * rstd, (xv[i].w - mean) * rstd);
      }
      *reinterpret_cast<uint2*>(hs + lr * ldh + 4 * c) = pk;
    }
    __syncthreads();
  }
  ZS_STAMP(3);

  f32x4r_t acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4r_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < S; ++s) {
    bf16x8r_t af;
    if constexpr (LN)
      af = *reinterpret_cast<const bf16x8r_t*>(hs + fr * ldh + kw + 32 * s + fk);
    else
      af = a[s];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
      acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, b[s * NB + nb], acc[nb], 0, 0, 0);
  }

  // wave partials -> LDS [wave][row][col], summed in wave order
  float* mine = red + wid * RG * NT;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) mine[(4 * (lane >> 4) + i) * NT + 16 * nb + fr] = acc[nb][i];
  ZS_STAMP(4);
  __syncthreads();
  ZS_STAMP(5);
  if (!epi) return;
  float4 sum = *reinterpret_cast<const float4*>(red + erow * NT + 4 * ecq);
#pragma unroll
  for (int w = 1; w < WAVES; ++w) {
    const float4 p = *reinterpret_cast<const float4*>(red + (w * RG + erow) * NT + 4 * ecq);
    sum.x += p.x; sum.y += p.y; sum.z += p.z; sum.w += p.w;
  }
  if (em >= g.M) return;
  float v[4] = {sum.x + eb.x, sum.y + eb.y, sum.z + eb.z, sum.w + eb.w};
  const bool bf = g.out_dtype == ZS_BF16;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = bf ? act_apply_fast(v[j], g.act) : act_apply(v[j], g.act);
  v[0] += er.x; v[1] += er.y; v[2] += er.z; v[3] += er.w;
  if (en + 3 < g.N && (g.ldo & 3) == 0 && ((uintptr_t)g.out & 15) == 0) {
    if (bf) {
      uint2 pk;
      pk.x = pk2bf(v[0], v[1]);
      pk.y = pk2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(g.out) + (long)em * g.ldo + en) = pk;
    } else {
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.out) + (long)em * g.ldo + en) =
          make_float4(v[0], v[1], v[2], v[3]);
    }
  } else {
    for (int j = 0; j < 4; ++j) {
      if (en + j >= g.N) break;
      if (bf) reinterpret_cast<bf16_t*>(g.out)[(long)em * g.ldo + en + j] = f2bf(v[j]);
      else reinterpret_cast<float*>(g.out)[(long)em * g.ldo + en + j] = v[j];
    }
  }
  ZS_STAMP(6);
}

// ------------------------------------------------------------------ f32 operands
// The f32 parity mode's decode GEMMs (exact f32 products, f32 accumulation: v_mfma_f32_16x16x4_f32,
// MI355X_MICROARCH.md: bitwise an fmaf chain).  Same structure as gemm_rows_kernel (row groups of
// 16, full K per workgroup split over its waves, every weight load issued up front, LN prologue
// from the f32 residual stream with the LN affine applied in f32, wave partials summed in LDS).
// A k-step covers 16 k: lane l (fr = l & 15, g = l >> 4) loads 16 bytes of its A row and of its
// weight row at k + 4 g .. + 4; MFMA j (j = 0..3) takes element j of both, i.e. the MFMA's k index
// g stands for k + 4 g + j, so the four MFMAs of a k-step cover its 16 k.
typedef __attribute__((ext_vector_type(4))) float f32x4v_t;

template <int NT, int WAVES, int LNM, int S>
__global__ __launch_bounds__(64 * WAVES) void gemm_rows_f32_kernel(RowsArgs g) {
  constexpr bool LN = LNM != 0;
  constexpr int NB = NT / 16;
  constexpr int NTHR = 64 * WAVES;
  constexpr int K = 16 * WAVES * S, KW = K / WAVES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nwg = gridDim.x, id = blockIdx.x, xcd = id & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
  const int rg = u % g.rgroups, tile = u / g.rgroups;
  const int m0 = rg * RG, n0 = tile * NT;
  const int kw = wid * KW;
  constexpr int ldh = K + 4;                // padded f32 LDS row
  float* hs = reinterpret_cast<float*>(smem);
  float* red = reinterpret_cast<float*>(smem + (LN ? RG * ldh * 4 : 0));
  const int fr = lane & 15, fk = 4 * (lane >> 4);
  const int am = min(m0 + fr, g.M - 1);

  constexpr int NQ = NT / 4;
  static_assert(RG * NQ <= NTHR, "one epilogue quad per thread");
  const bool epi = threadIdx.x < RG * NQ;
  const int erow = threadIdx.x / NQ, ecq = threadIdx.x % NQ;
  const int em = m0 + erow, en = n0 + 4 * ecq;
  float4 eb = make_float4(0.f, 0.f, 0.f, 0.f), er = eb;
  if (epi) {
    if (g.bias) {
      eb.x = g.bias[min(en, g.N - 1)];     eb.y = g.bias[min(en + 1, g.N - 1)];
      eb.z = g.bias[min(en + 2, g.N - 1)]; eb.w = g.bias[min(en + 3, g.N - 1)];
    }
    if (g.residual) {
      const float* rr = g.residual + (long)min(em, g.M - 1) * g.ldr;
      er.x = rr[min(en, g.N - 1)];     er.y = rr[min(en + 1, g.N - 1)];
      er.z = rr[min(en + 2, g.N - 1)]; er.w = rr[min(en + 3, g.N - 1)];
    }
  }
  constexpr int TPR = NTHR / RG, NV = LN ? K / (4 * TPR) : 1;
  static_assert(!LN || K % (4 * TPR) == 0, "LN rows: K % (4 * threads per row)");
  const int lr = threadIdx.x / TPR, lt = threadIdx.x % TPR;
  float4 xv[NV];
  if constexpr (LN) {
    const float4* xr = reinterpret_cast<const float4*>(g.X + (long)min(m0 + lr, g.M - 1) * g.ldx);
#pragma unroll
    for (int i = 0; i < NV; ++i) xv[i] = xr[lt + TPR * i];
  }
  f32x4v_t b[S * NB];
  f32x4v_t a[LN ? 1 : S];
  const float* wrow[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) wrow[nb] = g.Wf + (long)min(n0 + 16 * nb + fr, g.N - 1) * g.ldw;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int k = kw + 16 * s + fk;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) b[s * NB + nb] = *reinterpret_cast<const f32x4v_t*>(wrow[nb] + k);
    if constexpr (!LN) a[s] = *reinterpret_cast<const f32x4v_t*>(g.Af + (long)am * g.lda + k);
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  if constexpr (LN) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += (xv[i].x + xv[i].y) + (xv[i].z + xv[i].w);
#pragma unroll
    for (int o = TPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s * (1.0f / K);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const float a0 = xv[i].x - mean, a1 = xv[i].y - mean, a2 = xv[i].z - mean, a3 = xv[i].w - mean;
      q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
#pragma unroll
    for (int o = TPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = rsqrtf(q * (1.0f / K) + g.eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lt + TPR * i;
      const float4 lw = reinterpret_cast<const float4*>(g.ln_w)[c];
      const float4 lb = reinterpret_cast<const float4*>(g.ln_b)[c];
      *reinterpret_cast<float4*>(hs + lr * ldh + 4 * c) =
          make_float4((xv[i].x - mean) * rstd * lw.x + lb.x, (xv[i].y - mean) * rstd * lw.y + lb.y,
                      (xv[i].z - mean) * rstd * lw.z + lb.z, (xv[i].w - mean) * rstd * lw.w + lb.w);
    }
    __syncthreads();
  }

  f32x4r_t acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4r_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < S; ++s) {
    f32x4v_t af;
    if constexpr (LN)
      af = *reinterpret_cast<const f32x4v_t*>(hs + fr * ldh + kw + 16 * s + fk);
    else
      af = a[s];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[j], b[s * NB + nb][j], acc[nb], 0, 0, 0);
  }
  float* mine = red + wid * RG * NT;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) mine[(4 * (lane >> 4) + i) * NT + 16 * nb + fr] = acc[nb][i];
  __syncthreads();
  if (!epi) return;
  float4 sum = *reinterpret_cast<const float4*>(red + erow * NT + 4 * ecq);
#pragma unroll
  for (int w = 1; w < WAVES; ++w) {
    const float4 p = *reinterpret_cast<const float4*>(red + (w * RG + erow) * NT + 4 * ecq);
    sum.x += p.x; sum.y += p.y; sum.z += p.z; sum.w += p.w;
  }
  if (em >= g.M) return;
  float v[4] = {sum.x + eb.x, sum.y + eb.y, sum.z + eb.z, sum.w + eb.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = act_apply(v[j], g.act);
  v[0] += er.x; v[1] += er.y; v[2] += er.z; v[3] += er.w;
  float* o = reinterpret_cast<float*>(g.out) + (long)em * g.ldo + en;
  if (en + 3 < g.N && (g.ldo & 3) == 0 && ((uintptr_t)g.out & 15) == 0) {
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int j = 0; j < 4; ++j)
      if (en + j < g.N) o[j] = v[j];
  }
}

// f32 plan: 8 waves; LN (K 768 / 1024): 32-column tiles; plain: 16-column tiles, K 768 .. 4096
static int launch_rows_f32(const RowsArgs& g0, bool ln, hipStream_t st) {
  constexpr int W = 8;
  RowsArgs g = g0;
  const int K = g.K;
  if (K % (16 * W)) return 1;
  const int S = K / (16 * W);
  const int nt = ln ? 32 : 16;
  g.rgroups = cdiv(g.M, RG);
  g.ntiles = cdiv(g.N, nt);
  const dim3 grid(g.rgroups * g.ntiles);
  const size_t lds = (ln ? (size_t)RG * (K + 4) * 4 : 0) + (size_t)W * RG * nt * 4;
#define RF(LNM_, NT_, S_) hipLaunchKernelGGL((gemm_rows_f32_kernel<NT_, W, LNM_, S_>), grid, dim3(64 * W), lds, st, g)
  if (ln) {
    if (S == 6) RF(1, 32, 6);
    else if (S == 8) RF(1, 32, 8);
    else return 1;
  } else {
    switch (S) {
      case 6: RF(0, 16, 6); break;
      case 8: RF(0, 16, 8); break;
      case 24: RF(0, 16, 24); break;
      default: return 1;
    }
  }
#undef RF
  ZS_LAUNCH_CHECK();
  return 0;
}

int g_rows_nt48 = 1;  // A/B knob (zs_tune_set "rows_nt48"): 48-column LN tiles (2: 64)
int g_rows_wide = 0;  // A/B knob (zs_tune_set "rows_wide"): 32-column plain tiles at N < 1536
int g_gemm_rows = 1;   // A/B knob (zs_tune_set "gemm_rows"): 0 = skinny split-K kernel for M <= 64

// shape plan: waves (K split), k-steps per wave, column tile; waves < 0 when not covered
struct RowsPlan { int waves, steps, nt; };
static RowsPlan rows_plan(int N, int K, bool ln) {
  const int waves = K >= 2048 ? 8 : 4;
  if (K % (32 * waves)) return {-1, 0, 0};
  const int S = K / (32 * waves);
  const bool ok = ln ? (waves == 4 && (S == 6 || S == 8))
                     : (waves == 4 ? (S == 2 || S == 4 || S == 6 || S == 8 || S == 12)
                                   : (S == 8 || S == 12 || S == 15 || S == 16));
  if (!ok) return {-1, 0, 0};
  const int per = ln ? 2 : 3;               // loads per k-step at NT = 32
  // LN mode: 48-column tiles where N allows (c_fc 64 x 4 = 256 workgroups, c_attn 192: one per
  // CU; at 32 columns c_fc's 384 put two on half the CUs, whose per-CU load bytes set the time)
  // knobs for the concurrent bench (several batches co-running: the bytes each launch pulls
  // through the CUs' load path matter more than its own latency): rows_nt48 = 2 -> 64-column
  // LN tiles; rows_wide = 1 -> 32-column tiles for the N = 768 projections (half the
  // activation re-reads of mproj's 3072-deep rows)
  if (ln && g_rows_nt48 == 2 && N % 64 == 0 && S * 4 <= RG_MAX_LOADS) return {waves, S, 64};
  if (ln && g_rows_nt48 && N % 48 == 0 && S * 3 <= RG_MAX_LOADS) return {waves, S, 48};
  if (S * per <= RG_MAX_LOADS && (N >= 1536 || (!ln && g_rows_wide))) return {waves, S, 32};
  return {waves, S, 16};
}

template <int LNM, int NT, int W, int S>
static void launch_rows_k(const RowsArgs& g, dim3 grid, size_t lds, hipStream_t st) {
  if constexpr (S * (LNM ? NT / 16 : NT / 16 + 1) <= RG_MAX_LOADS)   // rows_plan never asks more
    hipLaunchKernelGGL((gemm_rows_kernel<NT, W, LNM, S>), grid, dim3(64 * W), lds, st, g);
}

template <int LNM, int NT, int W>
static void launch_rows_s(const RowsArgs& g, int S, dim3 grid, size_t lds, hipStream_t st) {
#define RL(S_) launch_rows_k<LNM, NT, W, S_>(g, grid, lds, st)
  if constexpr (LNM) {
    if (S == 6) RL(6); else RL(8);
  } else if constexpr (W == 4) {
    switch (S) { case 2: RL(2); break; case 4: RL(4); break; case 6: RL(6); break;
                 case 8: RL(8); break; default: RL(12); }
  } else {
    switch (S) { case 8: RL(8); break; case 12: RL(12); break; case 15: RL(15); break;
                 default: RL(16); }
  }
#undef RL
}

template <int LNM>
static int launch_rows(const RowsArgs& g0, RowsPlan p, hipStream_t st) {
  constexpr bool LN = LNM != 0;
  RowsArgs g = g0;
  g.rgroups = cdiv(g.M, RG);
  g.ntiles = cdiv(g.N, p.nt);
  const dim3 grid(g.rgroups * g.ntiles);
  const size_t lds = (LN ? (size_t)RG * (g.K + 8) * 2 : 0) + (size_t)p.waves * RG * p.nt * 4;
  if constexpr (LN) {                       // rows_plan: LN at 4 waves only
    if (p.nt == 64) launch_rows_s<LNM, 64, 4>(g, p.steps, grid, lds, st);
    else if (p.nt == 48) launch_rows_s<LNM, 48, 4>(g, p.steps, grid, lds, st);
    else if (p.nt == 32) launch_rows_s<LNM, 32, 4>(g, p.steps, grid, lds, st);
    else launch_rows_s<LNM, 16, 4>(g, p.steps, grid, lds, st);
  } else if (p.nt == 32) {
    if (p.waves == 8) launch_rows_s<0, 32, 8>(g, p.steps, grid, lds, st);
    else launch_rows_s<0, 32, 4>(g, p.steps, grid, lds, st);
  } else {
    if (p.waves == 8) launch_rows_s<0, 16, 8>(g, p.steps, grid, lds, st);
    else launch_rows_s<0, 16, 4>(g, p.steps, grid, lds, st);
  }
  ZS_LAUNCH_CHECK();
  return 0;
}

}  // namespace zs

using namespace zs;

// used by zs_gemm (auto mode) for bf16 M <= 64; returns 1 when the shape is not covered
extern "C" __attribute__((visibility("hidden"))) int zs_gemm_rows_internal(
    int M, int N, int K, const void* A, int lda, const void* W, int ldw, const float* bias,
    const float* residual, int ldr, void* out, int ldo, int out_dtype, int act, void* stream) {
  if (!g_gemm_rows || M > RG_MAX_M || (lda & 7) || (ldw & 7)) return 1;
  const RowsPlan p = rows_plan(N, K, false);
  if (p.waves < 0) return 1;
  RowsArgs g{};
  g.M = M; g.N = N; g.K = K; g.A = (const bf16_t*)A; g.lda = lda; g.W = (const bf16_t*)W;
  g.ldw = ldw; g.bias = bias; g.residual = residual; g.ldr = ldr; g.out = out; g.ldo = ldo;
  g.out_dtype = out_dtype; g.act = act;
  return launch_rows<0>(g, p, S(stream));
}

extern "C" int zs_gemm_ln(int M, int N, int K, const float* x, int ldx, const float* ln_w,
                          const float* ln_b, float eps, const void* W, int ldw, const float* bias,
                          const float* residual, int ldr, void* out, int ldo, int out_dtype,
                          int act, void* stream) {
  ZS_REQUIRE(M > 0 && M <= RG_MAX_M && N > 0 && K > 0, "zs_gemm_ln: M in 1..%d (got M=%d N=%d K=%d)",
             RG_MAX_M, M, N, K);
  // ln_w == ln_b == nullptr: normalise only (the caller folded the LN affine into W and bias)
  ZS_REQUIRE(x && W && out && (ln_w == nullptr) == (ln_b == nullptr), "zs_gemm_ln: null pointer");
  ZS_REQUIRE(ldx % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)ln_w & 15) == 0 &&
             ((uintptr_t)ln_b & 15) == 0, "zs_gemm_ln: x / LN params must be 16-byte aligned");
  ZS_REQUIRE(ldw % 8 == 0 && ((uintptr_t)W & 15) == 0, "zs_gemm_ln: W must be 16-byte aligned");
  ZS_REQUIRE(out_dtype == ZS_BF16 || out_dtype == ZS_F32, "zs_gemm_ln: out dtype");
  const RowsPlan p = rows_plan(N, K, true);
  ZS_REQUIRE(p.waves > 0, "zs_gemm_ln: unsupported K=%d (768 or 1024)", K);
  RowsArgs g{};
  g.M = M; g.N = N; g.K = K; g.X = x; g.ldx = ldx; g.ln_w = ln_w; g.ln_b = ln_b; g.eps = eps;
  g.W = (const bf16_t*)W; g.ldw = ldw; g.bias = bias; g.residual = residual; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.out_dtype = out_dtype; g.act = act;
  return ln_w ? launch_rows<1>(g, p, S(stream)) : launch_rows<2>(g, p, S(stream));
}

extern "C" int zs_gemm_ln_f32(int M, int N, int K, const float* x, int ldx, const float* ln_w,
                              const float* ln_b, float eps, const float* W, int ldw,
                              const float* bias, const float* residual, int ldr, float* out,
                              int ldo, int act, void* stream) {
  ZS_REQUIRE(M > 0 && M <= RG_MAX_M && N > 0 && K > 0,
             "zs_gemm_ln_f32: M in 1..%d (got M=%d N=%d K=%d)", RG_MAX_M, M, N, K);
  // ln_w == ln_b == nullptr: no LayerNorm, out = act(x W^T + b) + residual (the f32 decode's
  // attn.c_proj / mlp.c_proj; K up to 3072)
  ZS_REQUIRE(x && W && out && (ln_w == nullptr) == (ln_b == nullptr), "zs_gemm_ln_f32: null pointer");
  ZS_REQUIRE(ldx % 4 == 0 && ldw % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)W & 15) == 0 &&
             ((uintptr_t)ln_w & 15) == 0 && ((uintptr_t)ln_b & 15) == 0,
             "zs_gemm_ln_f32: x / W / LN params must be 16-byte aligned, ldx / ldw multiples of 4");
  const bool ln = ln_w != nullptr;
  ZS_REQUIRE(ln ? (K == 768 || K == 1024) : (K == 768 || K == 1024 || K == 3072),
             "zs_gemm_ln_f32: unsupported K=%d (768 / 1024, or 3072 without LayerNorm)", K);
  RowsArgs g{};
  g.M = M; g.N = N; g.K = K; g.X = x; g.ldx = ldx; g.ln_w = ln_w; g.ln_b = ln_b; g.eps = eps;
  g.Af = x; g.lda = ldx;
  g.Wf = W; g.ldw = ldw; g.bias = bias; g.residual = residual; g.ldr = ldr;
  g.out = out; g.ldo = ldo; g.out_dtype = ZS_F32; g.act = act;
  return launch_rows_f32(g, ln, S(stream));
}

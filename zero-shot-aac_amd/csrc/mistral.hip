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
typedef __attribute__((ext_vector_type(4))) unsigned u32x4m_t;

int g_fp8_tile = 0;   // zs_tune_set("fp8_tile", v) A/B knob: 1 = 64-column one-shot tiles only,
                      // 2 = one-shot kernel only (no persistent stream kernel), 3 = 128-column
                      // one-shot tiles where the stream kernel does not apply, 4 = 64-column
                      // one-shot tiles below 256 workgroups at M <= 32 (the earlier rule)
int g_fp8_dbg = 0;    // zs_tune_set("fp8_dbg", b): ablations (1 no A loads, 2 no MFMA, 4 no W loads)

constexpr int F8_KC = 1024;   // k per workgroup (one split)
constexpr int F8_MAXM = 64;

// Tile-packed fp8 weights (zsaac/mistral.py fp8_pack_tiles): [K/1024][ntiles = ceil(N/128)][8]
// [16][64 lanes][16 B].  The 1 KiB block of (k split s, 128-column tile t, 16-column group w,
// 64-deep k block j) holds, in lane l, W[128 t + 16 w + (l & 15)][1024 s + 64 j + 16 (l >> 4) ..
// +16] (rows past N zero): each wave-load is one contiguous KiB and an item (s, t) one
// contiguous 128 KiB.  Returns lane l's address of block j = 0 of (s, group nb16 = 8 t + w).
__device__ __forceinline__ const uint8_t* f8_frag(const uint8_t* W8, int ntiles, int split,
                                                  int nb16, int lane) {
  return W8 + ((((long)split * ntiles + (nb16 >> 3)) * 8 + (nb16 & 7)) * 16) * 1024 + lane * 16;
}

// out[split][m][n] = scale[n] * sum_{k in split} A[m][k] * W[n][k]   (M <= 64, W8 tile-packed)
// A workgroup of WAVES waves covers NT = 16 NB WAVES columns x one 1024-deep k split: lane l of a
// wave covers column n = l & 15 of each of its NB 16-column blocks; in each 64-deep k block lane
// group g = l >> 4 holds the 16 consecutive fp8 at k = 64 j + 16 g (one 16-byte load) and feeds
// them as two MFMA k-slices of 8; A is staged once per workgroup in LDS and read with the same k
// assignment, so the products pair up (the sum runs over a permuted k order).  Bytes per
// workgroup: NT x 1024 weight + M x 1024 x 2 activation, so wide tiles (NT = 256 for gate|up)
// keep the activation re-reads at a quarter of the weight stream.
template <int NB, int WAVES, int MB>
__global__ __launch_bounds__(64 * WAVES) void fp8_gemm_rows_kernel(
    const bf16_t* __restrict__ A, int lda, const uint8_t* __restrict__ W8,
    const float* __restrict__ scale, int M, int N, int K, float* __restrict__ out,
    long split_stride, int ldo, int dbg) {
  constexpr int NT = 16 * NB * WAVES, NTHR = 64 * WAVES;
  constexpr int JB = F8_KC / 64;                    // 64-deep k blocks per split
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* as = reinterpret_cast<bf16_t*>(smem);      // [M][F8_KC + 8]
  constexpr int LDA_S = F8_KC + 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * NT + wid * 16 * NB;
  const int split = blockIdx.y, k0 = split * F8_KC;
  constexpr int kc = F8_KC;     // K % 1024 == 0: every load unconditional (a runtime bound put
                                // each weight load in its own branch, waited for there)
  const int fr = lane & 15, g = lane >> 4;
  // the activation chunk's loads are issued FIRST (into registers), the weight stream after
  // them: loads return in order, so the LDS stores below wait only for the A loads while the
  // weight loads stay in flight (issued the other way round, every A load waited behind the
  // whole weight stream and the A copy became a chain of round trips)
  const int per_row = kc / 8;                        // 16-byte pieces per A row
  constexpr int AMAX = MB * (F8_KC / 8) / NTHR;      // pieces per thread at M = MB
  uint4 av[AMAX];
#pragma unroll
  for (int t = 0; t < AMAX; ++t) {
    const int i = threadIdx.x + t * NTHR;
    const int m = min(i / per_row, M - 1), c = (i % per_row) * 8;
    av[t] = *reinterpret_cast<const uint4*>(A + (long)m * lda + k0 + c);
  }
  u32x4m_t wv[NB][JB];   // weights are read once per decode step: non-temporal loads
  const int ntiles = (N + 127) >> 7;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    // groups past the last tile (a 256-column tile over an odd tile count) reread the last
    // group; their columns are >= N and never stored
    const uint8_t* wr = f8_frag(W8, ntiles, split, min((n0 >> 4) + nb, 8 * ntiles - 1), lane);
#pragma unroll
    for (int j = 0; j < JB; ++j)
      wv[nb][j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4m_t*>(wr + 1024 * j));
  }
  // (straight-line code from the first load to here: the compiler's counted waits let these
  // stores wait for the A loads only, the weight stream stays in flight)
#pragma unroll
  for (int t = 0; t < AMAX; ++t) {
    const int i = threadIdx.x + t * NTHR;
    if (i < M * per_row)
      *reinterpret_cast<uint4*>(as + (i / per_row) * LDA_S + (i % per_row) * 8) = av[t];
  }
  __syncthreads();
  const int nrb = (M + 15) / 16;
  f32x4m_t acc[NB][F8_MAXM / 16];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int rb = 0; rb < F8_MAXM / 16; ++rb) acc[nb][rb] = f32x4m_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    bf16x8m_t b0[NB], b1[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const u32x4m_t w = wv[nb][j];
      const bf16x2m_t p0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.x, 1.0f, false);
      const bf16x2m_t p1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.x, 1.0f, true);
      const bf16x2m_t p2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.y, 1.0f, false);
      const bf16x2m_t p3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.y, 1.0f, true);
      b0[nb] = bf16x8m_t{p0[0], p0[1], p1[0], p1[1], p2[0], p2[1], p3[0], p3[1]};
      const bf16x2m_t q0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.z, 1.0f, false);
      const bf16x2m_t q1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.z, 1.0f, true);
      const bf16x2m_t q2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.w, 1.0f, false);
      const bf16x2m_t q3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.w, 1.0f, true);
      b1[nb] = bf16x8m_t{q0[0], q0[1], q1[0], q1[1], q2[0], q2[1], q3[0], q3[1]};
    }
    const int ka = 64 * j + 16 * g;
#pragma unroll
    for (int rb = 0; rb < F8_MAXM / 16; ++rb) {
      if (rb >= nrb) break;
      const int m = min(rb * 16 + fr, M - 1);
      const bf16x8m_t a0 = *reinterpret_cast<const bf16x8m_t*>(as + m * LDA_S + ka);
      const bf16x8m_t a1 = *reinterpret_cast<const bf16x8m_t*>(as + m * LDA_S + ka + 8);
      // transposed product out^T = W A^T: the weight fragment is the A operand, so a lane's
      // accumulators are 4 consecutive output COLUMNS of one row -> one 16-byte slab store
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        acc[nb][rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[nb], a0, acc[nb][rb], 0, 0, 0);
        acc[nb][rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[nb], a1, acc[nb][rb], 0, 0, 0);
      }
    }
  }
  // C layout (transposed product): lane -> output row m = 16 rb + (lane & 15), columns
  // n0 + 16 nb + 4 (lane >> 4) + i, i = 0..3
  float* o = out + split * split_stride;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = n0 + 16 * nb + 4 * g;
    if (n >= N) continue;
    const float4 sc = *reinterpret_cast<const float4*>(scale + n);
#pragma unroll
    for (int rb = 0; rb < F8_MAXM / 16; ++rb) {
      if (rb >= nrb) break;
      const int m = rb * 16 + fr;
      if (m < M)
        *reinterpret_cast<float4*>(o + (long)m * ldo + n) =
            make_float4(acc[nb][rb][0] * sc.x, acc[nb][rb][1] * sc.y, acc[nb][rb][2] * sc.z,
                        acc[nb][rb][3] * sc.w);
    }
  }
}

// Persistent form of the same product for M <= 32 and the long weight streams (gate|up, down):
// gridDim.x workgroups (one per CU) each walk a contiguous, equal-length run of (k split, column
// tile) items in split-major order.  Item i+1's weight fragments are issued into the second
// register buffer before item i's MFMAs, so a CU's weight stream never drains between items (the
// one-shot kernel issues a workgroup's whole slice, waits, computes, stores and exits, and its
// grid of 448 workgroups runs as 1.75 rounds); the LDS activation chunk is reloaded only when the
// run crosses into the next split, before the next item's loads are issued (the counted waits
// are in issue order).  Slab layout and the sum over k are the one-shot kernel's.
template <int WAVES>
struct F8Stream {
  static constexpr int NT = 16 * WAVES, NTHR = 64 * WAVES, JB = F8_KC / 64, MB = 32;
  static constexpr int LDA_S = F8_KC + 8;
  static constexpr int AMAX = MB * (F8_KC / 8) / NTHR;
};

// one item's operands in flight: its weight fragments and the scales of the 4 output columns a
// lane stores (loaded with the item, so the store never waits behind the next item's stream)
struct F8Item {
  u32x4m_t w[F8_KC / 64];
  float4 sc;
};

template <int WAVES>
__device__ __forceinline__ void f8s_issue(F8Item& b, const uint8_t* __restrict__ W8,
                                          const float* __restrict__ scale, int N, int K,
                                          int ntiles, int it) {
  using P = F8Stream<WAVES>;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int split = it / ntiles, tile = it - split * ntiles;     // NT-column item tiles
  const uint8_t* wr = f8_frag(W8, (N + 127) >> 7, split, tile * WAVES + wid, lane);
#pragma unroll
  for (int j = 0; j < P::JB; ++j)
    b.w[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4m_t*>(wr + 1024 * j));
  b.sc = *reinterpret_cast<const float4*>(scale + min(tile * P::NT + wid * 16 + 4 * (lane >> 4), N - 4));
}

template <int WAVES>
__device__ __forceinline__ void f8s_load_a(bf16_t* as, const bf16_t* __restrict__ A, int lda,
                                           int M, int split) {
  using P = F8Stream<WAVES>;
  constexpr int per_row = F8_KC / 8;
  __syncthreads();                     // the previous split's readers are done with `as`
  uint4 av[P::AMAX];
#pragma unroll
  for (int t = 0; t < P::AMAX; ++t) {
    const int i = threadIdx.x + t * P::NTHR;
    const int m = min(i / per_row, M - 1), c = (i % per_row) * 8;
    av[t] = *reinterpret_cast<const uint4*>(A + (long)m * lda + split * F8_KC + c);
  }
#pragma unroll
  for (int t = 0; t < P::AMAX; ++t) {
    const int i = threadIdx.x + t * P::NTHR;
    if (i < M * per_row)
      *reinterpret_cast<uint4*>(as + (i / per_row) * P::LDA_S + (i % per_row) * 8) = av[t];
  }
  __syncthreads();
}

template <int WAVES>
__device__ __forceinline__ void f8s_compute(const F8Item& b, const bf16_t* as, int M, int N,
                                            float* __restrict__ out, long split_stride, int ldo,
                                            int ntiles, int it) {
  using P = F8Stream<WAVES>;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, fr = lane & 15, g = lane >> 4;
  const int split = it / ntiles, tile = it - split * ntiles;
  // both 16-row blocks always run (rows past M read row M - 1, their results are not stored):
  // a data-dependent branch here would make the compiler wait for every load in flight,
  // including the next item's
  f32x4m_t acc[2] = {f32x4m_t{0.f, 0.f, 0.f, 0.f}, f32x4m_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int j = 0; j < P::JB; ++j) {
    const u32x4m_t w = b.w[j];
    const bf16x2m_t p0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.x, 1.0f, false);
    const bf16x2m_t p1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.x, 1.0f, true);
    const bf16x2m_t p2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.y, 1.0f, false);
    const bf16x2m_t p3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.y, 1.0f, true);
    const bf16x8m_t b0 = bf16x8m_t{p0[0], p0[1], p1[0], p1[1], p2[0], p2[1], p3[0], p3[1]};
    const bf16x2m_t q0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.z, 1.0f, false);
    const bf16x2m_t q1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.z, 1.0f, true);
    const bf16x2m_t q2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.w, 1.0f, false);
    const bf16x2m_t q3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.w, 1.0f, true);
    const bf16x8m_t b1 = bf16x8m_t{q0[0], q0[1], q1[0], q1[1], q2[0], q2[1], q3[0], q3[1]};
    const int ka = 64 * j + 16 * g;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int m = min(rb * 16 + fr, M - 1);
      const bf16x8m_t a0 = *reinterpret_cast<const bf16x8m_t*>(as + m * P::LDA_S + ka);
      const bf16x8m_t a1 = *reinterpret_cast<const bf16x8m_t*>(as + m * P::LDA_S + ka + 8);
      acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0, a0, acc[rb], 0, 0, 0);
      acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, a1, acc[rb], 0, 0, 0);
    }
  }
  const int n = tile * P::NT + wid * 16 + 4 * g;
  if (n >= N) return;
  const float4 sc = b.sc;
  float* o = out + split * split_stride;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int m = rb * 16 + fr;
    if (m < M)
      *reinterpret_cast<float4*>(o + (long)m * ldo + n) =
          make_float4(acc[rb][0] * sc.x, acc[rb][1] * sc.y, acc[rb][2] * sc.z, acc[rb][3] * sc.w);
  }
}

// PER items per workgroup, a compile-time count: the loop unrolls and every next-item issue is
// unconditional (a conditional issue makes the compiler's counted waits fall back to waiting for
// every load in flight).  The last workgroup's run is clamped to the final item: it recomputes
// and rewrites identical values.
template <int WAVES, int PER>
__global__ __launch_bounds__(64 * WAVES) void fp8_gemm_stream_kernel(
    const bf16_t* __restrict__ A, int lda, const uint8_t* __restrict__ W8,
    const float* __restrict__ scale, int M, int N, int K, float* __restrict__ out,
    long split_stride, int ldo, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* as = reinterpret_cast<bf16_t*>(smem);
  const int last = ntiles * (K / F8_KC) - 1;
  const int i0 = blockIdx.x * PER;                 // grid = cdiv(items, PER)
  F8Item buf[2];
  int asplit = -1;
  f8s_issue<WAVES>(buf[0], W8, scale, N, K, ntiles, min(i0, last));
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const int it = min(i0 + t, last);
    if (it / ntiles != asplit) { asplit = it / ntiles; f8s_load_a<WAVES>(as, A, lda, M, asplit); }
    if (t + 1 < PER)
      f8s_issue<WAVES>(buf[(t + 1) & 1], W8, scale, N, K, ntiles, min(i0 + t + 1, last));
    // keep the next item's loads ahead of this item's MFMAs (the scheduler would otherwise sink
    // them below the compute to save registers, and the stream would drain every item)
    __builtin_amdgcn_sched_barrier(0);
    f8s_compute<WAVES>(buf[t & 1], as, M, N, out, split_stride, ldo, ntiles, it);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Run kernel (decode, M <= 32): one workgroup per (128-column tile, run of KS consecutive 1024-deep
// k splits), the run's products summed in registers, so a GEMM writes nsplit / KS partial slabs
// instead of nsplit.  Per split the activation chunk is loaded into registers first and the
// split's weight fragments after it (loads return in order), both one split AHEAD of the MFMAs:
// the chunk lands in one of two LDS buffers while the previous split computes from the other, and
// the weight stream of a run never drains.  GLU (KS = nsplit: each workgroup holds complete sums):
// the gate|up matrix is packed with gate and up columns interleaved by 4 (zsaac/mistral.py
// glu_interleave: in every 16-column group, lanes of column quad g = 0 / 2 hold gate columns
// 8 grp + 0..3 / 4..7 and quads 1 / 3 the matching up columns), so lane l's partner is lane l ^ 16
// and the epilogue writes act = silu(gate) * up (bf16, F = N / 2 columns) itself -- no slab, no
// consumer launch (predict_mistralai_multilingual.py's MistralMLP: down(silu(gate(x)) * up(x))).
template <int KH>
struct F8Run {
  static constexpr int WAVES = 8, NTHR = 512, KC = F8_KC / KH, JB = KC / 64, LDA_S = KC + 8;
  static constexpr int PER_ROW = KC / 8, AMAX = 32 * PER_ROW / NTHR;   // M <= 32
  static constexpr int LDS_BYTES = 2 * 32 * LDA_S * 2;
};

template <int KH>
__device__ __forceinline__ void f8r_load_a(uint4 (&av)[F8Run<KH>::AMAX],
                                           const bf16_t* __restrict__ A, int lda, int M, int k0) {
  using P = F8Run<KH>;
#pragma unroll
  for (int t = 0; t < P::AMAX; ++t) {
    const int i = threadIdx.x + t * P::NTHR;
    const int m = min(i / P::PER_ROW, M - 1), c = (i % P::PER_ROW) * 8;
    av[t] = *reinterpret_cast<const uint4*>(A + (long)m * lda + k0 + c);
  }
}

// KH = 2: each workgroup takes one half (512 k) of every split of its run -- twice the workgroups
// and slabs for the short streams (o: 32 tiles x 4 splits = 128 workgroups -> 256)
// rss != NULL: A holds the un-normalised rows x (bf16) of an RMSNorm whose weight is folded into
// W, and rss [nch][32] their partial sums of squares (zs_mistral_add_ss); each output row is
// scaled by rsqrt(sum / K + eps) in the epilogue (the norm's per-row factor moved past the GEMM).
template <int KS, int KH, bool GLU, bool RS>
__global__ __launch_bounds__(512) void fp8_gemm_run_kernel(
    const bf16_t* __restrict__ A, int lda, const uint8_t* __restrict__ W8,
    const float* __restrict__ scale, int M, int N, int K, float* __restrict__ out,
    long split_stride, int ldo, bf16_t* __restrict__ act, int ld_act, int ntiles,
    const float* __restrict__ rss, int nch, float eps) {
  using P = F8Run<KH>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* as = reinterpret_cast<bf16_t*>(smem);                 // [2][32][LDA_S]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, fr = lane & 15, g = lane >> 4;
  const int tile = blockIdx.x % ntiles, rh = blockIdx.x / ntiles;
  const int run = rh / KH, hf = rh % KH, s0 = run * KS;
  const uint8_t* wr0 = f8_frag(W8, ntiles, s0, tile * P::WAVES + wid, lane) + 1024 * P::JB * hf;
  const long split_bytes = (long)ntiles * 128 * 1024;           // one split of every tile
  const int n = tile * 128 + wid * 16 + 4 * g;
  uint4 av[P::AMAX];
  u32x4m_t wv[2][P::JB];
  f8r_load_a<KH>(av, A, lda, M, s0 * F8_KC + hf * P::KC);
#pragma unroll
  for (int j = 0; j < P::JB; ++j)
    wv[0][j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4m_t*>(wr0 + 1024 * j));
  const float4 sc = *reinterpret_cast<const float4*>(scale + min(n, N - 4));
  // the norm's partial sums of squares of the lane's two rows (issued behind split 0's weights,
  // waited for in the epilogue only); chunks past nch read chunk nch - 1 and are not summed
  float rq[2][8];
  if constexpr (RS) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int c = 0; c < 8; ++c) rq[rb][c] = rss[min(c, nch - 1) * 32 + min(rb * 16 + fr, M - 1)];
  }
  f32x4m_t acc[2] = {f32x4m_t{0.f, 0.f, 0.f, 0.f}, f32x4m_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int t = 0; t < KS; ++t) {
    bf16_t* ab = as + (t & 1) * 32 * P::LDA_S;
    // chunk t -> LDS (the compiler's counted wait covers the chunk's loads only: split t's
    // weights and anything issued after stay in flight)
#pragma unroll
    for (int u = 0; u < P::AMAX; ++u) {
      const int i = threadIdx.x + u * P::NTHR;
      *reinterpret_cast<uint4*>(ab + (i / P::PER_ROW) * P::LDA_S + (i % P::PER_ROW) * 8) = av[u];
    }
    if (t + 1 < KS) {                                            // split t + 1 in flight
      f8r_load_a<KH>(av, A, lda, M, (s0 + t + 1) * F8_KC + hf * P::KC);
      const uint8_t* wr = wr0 + (t + 1) * split_bytes;
#pragma unroll
      for (int j = 0; j < P::JB; ++j)
        wv[(t + 1) & 1][j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4m_t*>(wr + 1024 * j));
    }
    // LDS hand-off without waiting on vector memory (a __syncthreads would drain split t + 1)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < P::JB; ++j) {
      const u32x4m_t w = wv[t & 1][j];
      const bf16x2m_t p0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.x, 1.0f, false);
      const bf16x2m_t p1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.x, 1.0f, true);
      const bf16x2m_t p2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.y, 1.0f, false);
      const bf16x2m_t p3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.y, 1.0f, true);
      const bf16x8m_t b0 = bf16x8m_t{p0[0], p0[1], p1[0], p1[1], p2[0], p2[1], p3[0], p3[1]};
      const bf16x2m_t q0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.z, 1.0f, false);
      const bf16x2m_t q1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.z, 1.0f, true);
      const bf16x2m_t q2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.w, 1.0f, false);
      const bf16x2m_t q3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w.w, 1.0f, true);
      const bf16x8m_t b1 = bf16x8m_t{q0[0], q0[1], q1[0], q1[1], q2[0], q2[1], q3[0], q3[1]};
      const int ka = 64 * j + 16 * g;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int m = rb * 16 + fr;             // LDS rows past M hold row M - 1 (clamped loads)
        const bf16x8m_t a0 = *reinterpret_cast<const bf16x8m_t*>(ab + m * P::LDA_S + ka);
        const bf16x8m_t a1 = *reinterpret_cast<const bf16x8m_t*>(ab + m * P::LDA_S + ka + 8);
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0, a0, acc[rb], 0, 0, 0);
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1, a1, acc[rb], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // lane -> row m = 16 rb + fr, columns n .. n + 3 (transposed product, as the one-shot kernel)
  if constexpr (RS) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      float q = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) q += c < nch ? rq[rb][c] : 0.f;
      const float r = rsqrtf(q / K + eps);
      acc[rb][0] *= r; acc[rb][1] *= r; acc[rb][2] *= r; acc[rb][3] *= r;
    }
  }
  if constexpr (GLU) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      float gv[4], uv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float mine = acc[rb][i] * (i == 0 ? sc.x : i == 1 ? sc.y : i == 2 ? sc.z : sc.w);
        const float other = __shfl_xor(mine, 16, 64);
        gv[i] = (g & 1) ? other : mine;
        uv[i] = (g & 1) ? mine : other;
      }
      const int m = rb * 16 + fr;
      if (!(g & 1) && m < M && n < N) {
        const int f = 8 * (tile * P::WAVES + wid) + 4 * (g >> 1);
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = gv[i] / (1.0f + expf(-gv[i])) * uv[i];   // F.silu * up
        st4(act + (long)m * ld_act + f, o[0], o[1], o[2], o[3]);
      }
    }
  } else {
    if (n >= N) return;
    float* o = out + rh * split_stride;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int m = rb * 16 + fr;
      if (m < M)
        *reinterpret_cast<float4*>(o + (long)m * ldo + n) =
            make_float4(acc[rb][0] * sc.x, acc[rb][1] * sc.y, acc[rb][2] * sc.z, acc[rb][3] * sc.w);
    }
  }
}

// Prefill (M > 64 rows) helpers: the tile-packed fp8 codes of one weight matrix unpacked to
// row-major bf16 [N][K] (exact: e4m3 -> bf16 is lossless, the scale is NOT applied) for the
// tiled bf16 MFMA GEMM, whose f32 result columns are then scaled (out[m][n] *= scale[n]).  The
// products and the scaling are the fp8 row kernel's (sum_k a q, then x scale), only the order
// of the k sum differs.  One thread per 16-byte code chunk (16 k of one row).
__global__ __launch_bounds__(256) void fp8_unpack_bf16_kernel(const uint8_t* __restrict__ W8,
                                                              int N, int K,
                                                              bf16_t* __restrict__ out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;   // packed chunk index
  const int ntiles = (N + 127) >> 7;
  const long nchunks = (long)ntiles * 128 * (K / 16);
  if (idx >= nchunks) return;
  // packed order: [split][tile][w][j][lane]
  const int lane = idx & 63;
  long r = idx >> 6;
  const int j = r & 15; r >>= 4;
  const int w = r & 7; r >>= 3;
  const int t = r % ntiles;
  const int split = r / ntiles;
  const int n = t * 128 + w * 16 + (lane & 15);
  if (n >= N) return;
  const int k = split * F8_KC + 64 * j + 16 * (lane >> 4);
  const u32x4m_t c = *reinterpret_cast<const u32x4m_t*>(W8 + idx * 16);
  u32x4m_t lo, hi;
  const unsigned cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const bf16x2m_t a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(cw[q], 1.0f, false);
    const bf16x2m_t b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(cw[q], 1.0f, true);
    const unsigned ua = __builtin_bit_cast(unsigned, a), ub = __builtin_bit_cast(unsigned, b);
    if (q < 2) { lo[2 * q] = ua; lo[2 * q + 1] = ub; }
    else { hi[2 * (q - 2)] = ua; hi[2 * (q - 2) + 1] = ub; }
  }
  u32x4m_t* o = reinterpret_cast<u32x4m_t*>(out + (long)n * K + k);
  o[0] = lo;
  o[1] = hi;
}

__global__ __launch_bounds__(256) void scale_cols_kernel(float* __restrict__ x, int M, int N,
                                                         int ld, const float* __restrict__ scale) {
  const long idx = 4 * ((long)blockIdx.x * 256 + threadIdx.x);
  if (idx >= (long)M * N) return;
  const int m = idx / N, n = idx % N;
  float4* p = reinterpret_cast<float4*>(x + (long)m * ld + n);
  const float4 s = *reinterpret_cast<const float4*>(scale + n);
  float4 v = *p;
  v.x *= s.x; v.y *= s.y; v.z *= s.z; v.w *= s.w;
  *p = v;
}

// ---------------------------------------------------------------- consumers of the slabs
__device__ __forceinline__ float slab_sum(const float* __restrict__ p, int nsplit, long ss) {
  float v = p[0];
  for (int s = 1; s < nsplit; ++s) v += p[s * ss];
  return v;
}

// x[m] += sum_s y[s][m]  (skipped when y == nullptr), then h[m] = w * (x[m] * rsqrt(mean(x^2) +
// eps)) (MistralRMSNorm; w == nullptr: the weight is folded into the next GEMM).  One 1024-thread
// block per row, 4 columns per thread per pass (D <= 4096 in one pass), every split's load issued
// before the adds (a row's slabs are one memory round trip, not one per split).
__device__ __forceinline__ float4 slab_sum4(const float* __restrict__ p, int nsplit, long ss) {
  float4 v = *reinterpret_cast<const float4*>(p);
  int s = 1;
  for (; s + 3 < nsplit; s += 4) {
    const float4 a = *reinterpret_cast<const float4*>(p + s * ss);
    const float4 b = *reinterpret_cast<const float4*>(p + (s + 1) * ss);
    const float4 c = *reinterpret_cast<const float4*>(p + (s + 2) * ss);
    const float4 d = *reinterpret_cast<const float4*>(p + (s + 3) * ss);
    v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
    v.x += c.x; v.y += c.y; v.z += c.z; v.w += c.w;
    v.x += d.x; v.y += d.y; v.z += d.z; v.w += d.w;
  }
  for (; s < nsplit; ++s) {
    const float4 a = *reinterpret_cast<const float4*>(p + s * ss);
    v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
  }
  return v;
}

template <typename T>
__global__ __launch_bounds__(1024) void mistral_add_rmsnorm_kernel(
    float* __restrict__ x, const float* __restrict__ y, int nsplit, long ss, int D, float eps,
    const float* __restrict__ w, T* __restrict__ h) {
  __shared__ float red[16];
  constexpr int CMAX = 4;                              // D <= 4 x 4096 (host-checked)
  const int m = blockIdx.x;
  float* xr = x + (long)m * D;
  float q = 0.f;
  float4 v[CMAX];                                      // the row stays in registers
#pragma unroll
  for (int u = 0; u < CMAX; ++u) {
    const int c = 4 * threadIdx.x + 4096 * u;
    if (c >= D) break;
    v[u] = *reinterpret_cast<const float4*>(xr + c);
    if (y) {
      const float4 a = slab_sum4(y + (long)m * D + c, nsplit, ss);
      v[u].x += a.x; v[u].y += a.y; v[u].z += a.z; v[u].w += a.w;
      *reinterpret_cast<float4*>(xr + c) = v[u];
    }
    q += (v[u].x * v[u].x + v[u].y * v[u].y) + (v[u].z * v[u].z + v[u].w * v[u].w);
  }
  const float r = rsqrtf(block_sum(q, red) / D + eps);
#pragma unroll
  for (int u = 0; u < CMAX; ++u) {
    const int c = 4 * threadIdx.x + 4096 * u;
    if (c >= D) break;
    float o[4] = {v[u].x * r, v[u].y * r, v[u].z * r, v[u].w * r};
    if (w) {
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] *= w[c + t];
    }
    st4(h + (long)m * D + c, o[0], o[1], o[2], o[3]);
  }
}

// Decode form of the residual add + RMSNorm when its consumer is zs_fp8_gemm_run with rss: x[m] +=
// sum_s y[s][m] (y may be NULL), xb[m] = bf16(x[m]) and rss[chunk][m] = the chunk's sum of x^2
// (512 columns per chunk, one 128-thread block per (row, chunk): 256 blocks at 32 rows x 4096,
// where the one-block-per-row norm spreads a step's slab reads over 32 CUs).
__global__ __launch_bounds__(128) void mistral_add_ss_kernel(float* __restrict__ x,
                                                             const float* __restrict__ y,
                                                             int nsplit, long ss, int D,
                                                             bf16_t* __restrict__ xb,
                                                             float* __restrict__ rss) {
  __shared__ float red[2];
  const int m = blockIdx.x, ch = blockIdx.y, c = ch * 512 + 4 * threadIdx.x;
  float* xr = x + (long)m * D + c;
  float4 v = *reinterpret_cast<const float4*>(xr);
  if (y) {
    const float4 a = slab_sum4(y + (long)m * D + c, nsplit, ss);
    v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    *reinterpret_cast<float4*>(xr) = v;
  }
  st4(xb + (long)m * D + c, v.x, v.y, v.z, v.w);
  float q = wave_sum((v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) rss[ch * 32 + m] = red[0] + red[1];
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

// act[m][f] = silu(gate) * up from the gate|up slabs [split][M][2F] (T out), 4 columns per thread;
// the columns are glu-interleaved (fp8_gemm_run_kernel): gate f at 16 (f / 8) + 8 (f / 4 % 2) +
// f % 4, up f four columns after it
template <typename T>
__global__ __launch_bounds__(256) void mistral_silu_mul_kernel(const float* __restrict__ gu,
                                                               int nsplit, long ss, int M, int F,
                                                               T* __restrict__ act) {
  const long idx = 4 * ((long)blockIdx.x * 256 + threadIdx.x);
  if (idx >= (long)M * F) return;
  const int m = idx / F, f = idx % F;
  const long pg = (long)m * 2 * F + 16 * (f >> 3) + 8 * ((f >> 2) & 1);
  const float4 gt = slab_sum4(gu + pg, nsplit, ss);
  const float4 up = slab_sum4(gu + pg + 4, nsplit, ss);
  const float g4[4] = {gt.x, gt.y, gt.z, gt.w}, u4[4] = {up.x, up.y, up.z, up.w};
  float o[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = g4[t] / (1.0f + expf(-g4[t])) * u4[t];   // F.silu * up
  st4(act + idx, o[0], o[1], o[2], o[3]);
}

// in-wave reductions of the attention kernels without LDS round trips (DPP within rows of 16,
// v_permlane16/32_swap across them), the same butterfly order as __shfl_xor 1, 2, 4 / 8, 16, 32
template <int CTRL>
__device__ __forceinline__ float m_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float m_sum8(float s) {          // over lane & 7
  s += m_dpp<0xB1>(s);                                        // quad_perm [1,0,3,2]
  s += m_dpp<0x4E>(s);                                        // quad_perm [2,3,0,1]
  return s + m_dpp<0x141>(s);                                 // row_half_mirror
}
__device__ __forceinline__ float m_pair16(float v) {        // v + lane ^ 16's v
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float m_pair32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float m_max_grp(float v) {       // over lane >> 3
  v = fmaxf(v, m_dpp<0x128>(v));                              // row_ror:8 = lane ^ 8
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float m_add_grp(float v) {
  return m_pair32(m_pair16(v + m_dpp<0x128>(v)));
}

// causal GQA attention, one wave per (query row m, q head h): keys 0..pos[m] of the sequence
// m / rows_per_seq from kv head h / (H / KVH); softmax((q k^T) / sqrt(128)) v, f32 math.
// Lane = (key group grp = lane >> 3, 16-dim slice sub = lane & 7): a wave step scores 8 keys
// (3-shuffle group reductions), 4 steps (32 keys) of K / V loads are issued together, keys past
// pos read a valid row and are masked by value; an online softmax carries across steps and the
// 8 groups' partial outputs are combined at the end.
template <typename T>
__global__ __launch_bounds__(256) void mistral_attn_kernel(const T* __restrict__ q, int M, int H,
                                                           int KVH, const int* __restrict__ pos,
                                                           int rows_per_seq,
                                                           const T* __restrict__ kc,
                                                           const T* __restrict__ vc, int Lmax,
                                                           T* __restrict__ out) {
  constexpr int HD = 128, DPL = 16, U = 4;
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= M * H) return;
  const int grp = lane >> 3, sub = lane & 7;
  const int m = w / H, h = w % H, kvh = h / (H / KVH), seq = m / rows_per_seq;
  const int p = __builtin_amdgcn_readfirstlane(pos[m]);
  const T* qr = q + (long)m * H * HD + h * HD + sub * DPL;
  float qv[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) qv[d] = ldf(qr + d);
  const float scale = 0.08838834764831845f;                      // 128^-0.5 (HF: (q k^T) * s)
  const long base = ((long)seq * KVH + kvh) * Lmax;
  float mx = -INFINITY, l = 0.f, o[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = 0.f;
  for (int j0 = 0; j0 <= p; j0 += 8 * U) {
    float kf[U][DPL], vf[U][DPL];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = min(j0 + 8 * u + grp, p);
      const T* kr = kc + (base + j) * HD + sub * DPL;
      const T* vr = vc + (base + j) * HD + sub * DPL;
#pragma unroll
      for (int d = 0; d < DPL; ++d) { kf[u][d] = ldf(kr + d); vf[u][d] = ldf(vr + d); }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float sv = 0.f;
#pragma unroll
      for (int d = 0; d < DPL; ++d) sv += qv[d] * kf[u][d];
      sv = m_sum8(sv);
      sv = (j0 + 8 * u + grp <= p) ? sv * scale : -INFINITY;
      float pm = m_max_grp(sv);
      const float mn = fmaxf(mx, pm);
      float corr, e;
      if constexpr (sizeof(T) == 4) { corr = expf(mx - mn); e = expf(sv - mn); }   // parity mode
      else { corr = __expf(mx - mn); e = __expf(sv - mn); }
      l = l * corr + e;
#pragma unroll
      for (int d = 0; d < DPL; ++d) o[d] = o[d] * corr + e * vf[u][d];
      mx = mn;
    }
  }
  // combine the 8 key groups (same running max in every group)
  l = m_add_grp(l);
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = m_add_grp(o[d]);
  if (grp == 0) {
    const float inv = 1.0f / l;
    T* orow = out + (long)m * H * HD + h * HD + sub * DPL;
#pragma unroll
    for (int d = 0; d < DPL; ++d) stf(orow + d, o[d] * inv);
  }
}

// Decode step (one new position per sequence, rows_per_seq = 1): RoPE + KV append fused into the
// attention.  Wave (row m, q head h) sums its q slice and its kv head's new k / v slices from the
// qkv slabs, rotates q and k (the dims d and d + 64 of a pair sit in lanes sub and sub ^ 4), scores
// keys 0..p-1 from the caches as mistral_attn_kernel does and key p = pos[m] from registers; the
// first q head of each kv head (group 0 lanes) writes k / v row p to the caches for later steps.
// Same sums, rotation and softmax arithmetic as mistral_rope_kv_kernel + mistral_attn_kernel.
template <typename T>
__global__ __launch_bounds__(256) void mistral_decode_attn_kernel(
    const float* __restrict__ qkv, int nsplit, long ss, int M, int H, int KVH,
    const int* __restrict__ pos, const float* __restrict__ cosb, const float* __restrict__ sinb,
    T* __restrict__ kc, T* __restrict__ vc, int Lmax, T* __restrict__ out) {
  constexpr int HD = 128, HALF = 64, DPL = 16, U = 4;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int w = blockIdx.x * 4 + wid;
  if (w >= M * H) return;
  const int grp = lane >> 3, sub = lane & 7;
  const int m = w / H, h = w % H, kvh = h / (H / KVH);
  const int p = __builtin_amdgcn_readfirstlane(pos[m]);
  const long NQKV = (long)(H + 2 * KVH) * HD;
  const float* src = qkv + m * NQKV + sub * DPL;
  const long base = ((long)m * KVH + kvh) * Lmax;
  // the first 8 U cached keys do not depend on this step's q / k / v: their loads are issued
  // before the slab sums (one memory round trip for both at the usual p <= 8 U... prompt + steps)
  float kf[U][DPL], vf[U][DPL];
  auto load_keys = [&](int j0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = max(min(j0 + 8 * u + grp, p - 1), 0);
      const T* kr = kc + (base + j) * HD + sub * DPL;
      const T* vr = vc + (base + j) * HD + sub * DPL;
#pragma unroll
      for (int d = 0; d < DPL; ++d) { kf[u][d] = ldf(kr + d); vf[u][d] = ldf(vr + d); }
    }
  };
  load_keys(0);
  float qv[DPL], kn[DPL], vn[DPL];
#pragma unroll
  for (int d = 0; d < DPL; d += 4) {
    const float4 a = slab_sum4(src + h * HD + d, nsplit, ss);
    const float4 b = slab_sum4(src + (H + kvh) * HD + d, nsplit, ss);
    const float4 c = slab_sum4(src + (H + KVH + kvh) * HD + d, nsplit, ss);
    qv[d] = a.x; qv[d + 1] = a.y; qv[d + 2] = a.z; qv[d + 3] = a.w;
    kn[d] = b.x; kn[d + 1] = b.y; kn[d + 2] = b.z; kn[d + 3] = b.w;
    vn[d] = c.x; vn[d + 1] = c.y; vn[d + 2] = c.z; vn[d + 3] = c.w;
  }
  {
    // rotary pair (i, i + 64): lo = a c - b s, hi = b c + a s with a = dim i, b = dim i + 64
    const bool lo = sub < 4;
    const float* cr = cosb + (long)p * HALF + (sub & 3) * DPL;
    const float* sr = sinb + (long)p * HALF + (sub & 3) * DPL;
#pragma unroll
    for (int d = 0; d < DPL; ++d) {
      const float c = cr[d], sn = sr[d];
      const float qo = __shfl_xor(qv[d], 4, 64), ko = __shfl_xor(kn[d], 4, 64);
      qv[d] = lo ? qv[d] * c - qo * sn : qv[d] * c + qo * sn;
      kn[d] = lo ? kn[d] * c - ko * sn : kn[d] * c + ko * sn;
    }
  }
  if (h % (H / KVH) == 0 && grp == 0) {
    T* kr = kc + (base + p) * HD + sub * DPL;
    T* vr = vc + (base + p) * HD + sub * DPL;
#pragma unroll
    for (int d = 0; d < DPL; d += 4) {
      st4(kr + d, kn[d], kn[d + 1], kn[d + 2], kn[d + 3]);
      st4(vr + d, vn[d], vn[d + 1], vn[d + 2], vn[d + 3]);
    }
  }
  // the cached operands are T: round q and the new k / v as the unfused path stores them
#pragma unroll
  for (int d = 0; d < DPL; ++d) {
    qv[d] = Cvt<T>::to_f(Cvt<T>::from_f(qv[d]));
    kn[d] = Cvt<T>::to_f(Cvt<T>::from_f(kn[d]));
    vn[d] = Cvt<T>::to_f(Cvt<T>::from_f(vn[d]));
  }
  const float scale = 0.08838834764831845f;                      // 128^-0.5
  float mx = -INFINITY, l = 0.f, o[DPL];
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = 0.f;
  auto update = [&](float sv, const float* vf) {
    float pm = m_max_grp(sv);
    const float mn = fmaxf(mx, pm);
    float corr, e;
    if constexpr (sizeof(T) == 4) { corr = expf(mx - mn); e = expf(sv - mn); }   // parity mode
    else { corr = __expf(mx - mn); e = __expf(sv - mn); }
    l = l * corr + e;
#pragma unroll
    for (int d = 0; d < DPL; ++d) o[d] = o[d] * corr + e * vf[d];
    mx = mn;
  };
  for (int j0 = 0; j0 < p; j0 += 8 * U) {
    if (j0 > 0) load_keys(j0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float sv = 0.f;
#pragma unroll
      for (int d = 0; d < DPL; ++d) sv += qv[d] * kf[u][d];
      sv = m_sum8(sv);
      update((j0 + 8 * u + grp < p) ? sv * scale : -INFINITY, vf[u]);
    }
  }
  {                                                              // key p (group 0 counts it)
    float sv = 0.f;
#pragma unroll
    for (int d = 0; d < DPL; ++d) sv += qv[d] * kn[d];
    sv = m_sum8(sv);
    update(grp == 0 ? sv * scale : -INFINITY, vn);
  }
  l = m_add_grp(l);
#pragma unroll
  for (int d = 0; d < DPL; ++d) o[d] = m_add_grp(o[d]);
  if (grp == 0) {
    const float inv = 1.0f / l;
    T* orow = out + (long)m * H * HD + h * HD + sub * DPL;
#pragma unroll
    for (int d = 0; d < DPL; d += 4)
      st4(orow + d, o[d] * inv, o[d + 1] * inv, o[d + 2] * inv, o[d + 3] * inv);
  }
}

}  // namespace zs

using namespace zs;

extern "C" int zs_fp8_gemm_rows(const void* A, int lda, const void* W8, const float* scale, int M,
                                int N, int K, float* out, long split_stride, int ldo,
                                void* stream) {
  ZS_REQUIRE(M > 0 && M <= F8_MAXM && N > 0 && K > 0 && K % F8_KC == 0,
             "zs_fp8_gemm_rows: 1 <= M <= %d, K %% 1024 == 0 (M=%d N=%d K=%d)", F8_MAXM, M, N, K);
  ZS_REQUIRE(lda % 8 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)W8 & 15) == 0 && K % 16 == 0,
             "zs_fp8_gemm_rows: 16-byte aligned A / W rows");
  ZS_REQUIRE(split_stride >= (long)(M - 1) * ldo + N && ldo >= N && N % 16 == 0 && ldo % 4 == 0 &&
             split_stride % 4 == 0 && ((uintptr_t)out & 15) == 0 && ((uintptr_t)scale & 15) == 0,
             "zs_fp8_gemm_rows: out layout (N %% 16, 16-byte aligned rows and scales)");
  // tile: the widest whose grid still gives >= ~256 workgroups (activation re-reads per weight
  // byte = 2 M / NT), else 64 columns
  const int splits = cdiv(K, F8_KC);
  const size_t lds = (size_t)M * (F8_KC + 8) * 2;
  hipStream_t st = S(stream);
#define F8L(NB_, W_)                                                                            \
  do {                                                                                          \
    if (M <= 32)                                                                                \
      hipLaunchKernelGGL((fp8_gemm_rows_kernel<NB_, W_, 32>), dim3(cdiv(N, 16 * NB_ * W_), splits), \
                         dim3(64 * W_), lds, st, (const bf16_t*)A, lda, (const uint8_t*)W8, scale, \
                         M, N, K, out, split_stride, ldo, g_fp8_dbg);                            \
    else                                                                                        \
      hipLaunchKernelGGL((fp8_gemm_rows_kernel<NB_, W_, 64>), dim3(cdiv(N, 16 * NB_ * W_), splits), \
                         dim3(64 * W_), lds, st, (const bf16_t*)A, lda, (const uint8_t*)W8, scale, \
                         M, N, K, out, split_stride, ldo, g_fp8_dbg);                            \
  } while (0)
  // long streams at M <= 32 (more than one item of 128 columns x 1024 k per CU): persistent kernel
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
  }
  const long items = (long)cdiv(N, 128) * splits;
  if (M <= 32 && (g_fp8_tile == 0 || g_fp8_tile == 4) && items > ncu && items <= 8L * ncu) {
    const long its = items, slots = ncu;
    const long per = (its + slots - 1) / slots;
#define F8S(W_, P_)                                                                             \
  hipLaunchKernelGGL((fp8_gemm_stream_kernel<W_, P_>), dim3((unsigned)((its + P_ - 1) / P_)),   \
                     dim3(64 * W_), (size_t)32 * (F8_KC + 8) * 2, st, (const bf16_t*)A, lda,   \
                     (const uint8_t*)W8, scale, M, N, K, out, split_stride, ldo,               \
                     cdiv(N, 128))
    if (per <= 2) F8S(8, 2);
    else if (per <= 3) F8S(8, 3);
    else if (per <= 4) F8S(8, 4);
    else if (per <= 6) F8S(8, 6);
    else F8S(8, 8);
#undef F8S
  } else if ((long)cdiv(N, 256) * splits >= 256 && g_fp8_tile != 1) F8L(2, 8);
  // 128-column tiles also at M <= 32 with >= 128 workgroups (q|k|v at 192: 11.1 -> 9.8 us)
  else if (((long)cdiv(N, 128) * splits >= (M <= 32 && g_fp8_tile != 4 ? 128 : 256) &&
            g_fp8_tile != 1) ||
           g_fp8_tile == 3)
    F8L(1, 8);
  else F8L(1, 4);
#undef F8L
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_fp8_splits(int K) { return K > 0 ? cdiv(K, F8_KC) : 0; }

extern "C" int zs_fp8_gemm_run(const void* A, int lda, const void* W8, const float* scale, int M,
                               int N, int K, int ks, int kh, float* out, long split_stride,
                               int ldo, void* act, int ld_act, const float* rss, int nch,
                               float eps, void* stream) {
  ZS_REQUIRE(!rss || (nch >= 1 && nch <= 8), "zs_fp8_gemm_run: rss needs 1 <= nch <= 8");
  ZS_REQUIRE(M > 0 && M <= 32 && N > 0 && N % 16 == 0 && K > 0 && K % F8_KC == 0,
             "zs_fp8_gemm_run: 1 <= M <= 32, N %% 16, K %% 1024 (M=%d N=%d K=%d)", M, N, K);
  const int nsplit = K / F8_KC;
  ZS_REQUIRE(ks >= 1 && nsplit % ks == 0 && (ks == 1 || ks == 2 || ks == 4) && (kh == 1 || kh == 2),
             "zs_fp8_gemm_run: ks in {1, 2, 4} dividing the %d splits, kh 1 or 2 (got %d, %d)",
             nsplit, ks, kh);
  ZS_REQUIRE(lda % 8 == 0 && ((uintptr_t)A & 15) == 0 && ((uintptr_t)W8 & 15) == 0 &&
                 ((uintptr_t)scale & 15) == 0,
             "zs_fp8_gemm_run: 16-byte aligned A rows, weights and scales");
  if (act) {
    ZS_REQUIRE(ks == nsplit && kh == 1 && ld_act % 4 == 0 && ld_act >= N / 2 &&
                   ((uintptr_t)act & 7) == 0,
               "zs_fp8_gemm_run: glu needs ks == splits (%d), kh 1, an 8-byte aligned act", nsplit);
  } else {
    ZS_REQUIRE(out && split_stride >= (long)(M - 1) * ldo + N && ldo >= N && ldo % 4 == 0 &&
                   split_stride % 4 == 0 && ((uintptr_t)out & 15) == 0,
               "zs_fp8_gemm_run: out layout (16-byte aligned rows, split stride)");
  }
  const int ntiles = cdiv(N, 128);
  const dim3 grid((unsigned)(ntiles * (nsplit / ks) * kh));
  hipStream_t st = S(stream);
#define F8R(KS_, KH_, GLU_)                                                                     \
  do {                                                                                          \
    if (rss)                                                                                    \
      hipLaunchKernelGGL((fp8_gemm_run_kernel<KS_, KH_, GLU_, true>), grid, dim3(512),          \
                         (size_t)F8Run<KH_>::LDS_BYTES, st, (const bf16_t*)A, lda,              \
                         (const uint8_t*)W8, scale, M, N, K, out, split_stride, ldo,            \
                         (bf16_t*)act, ld_act, ntiles, rss, nch, eps);                          \
    else                                                                                        \
      hipLaunchKernelGGL((fp8_gemm_run_kernel<KS_, KH_, GLU_, false>), grid, dim3(512),         \
                         (size_t)F8Run<KH_>::LDS_BYTES, st, (const bf16_t*)A, lda,              \
                         (const uint8_t*)W8, scale, M, N, K, out, split_stride, ldo,            \
                         (bf16_t*)act, ld_act, ntiles, rss, nch, eps);                          \
  } while (0)
  if (act) {
    if (ks == 4) F8R(4, 1, true);
    else if (ks == 2) F8R(2, 1, true);
    else F8R(1, 1, true);
  } else if (kh == 2) {
    if (ks == 4) F8R(4, 2, false);
    else if (ks == 2) F8R(2, 2, false);
    else F8R(1, 2, false);
  } else {
    if (ks == 4) F8R(4, 1, false);
    else if (ks == 2) F8R(2, 1, false);
    else F8R(1, 1, false);
  }
#undef F8R
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_fp8_unpack_bf16(const void* W8, int N, int K, void* out, void* stream) {
  ZS_REQUIRE(N > 0 && K > 0 && K % F8_KC == 0 && ((uintptr_t)W8 & 15) == 0 &&
                 ((uintptr_t)out & 15) == 0,
             "zs_fp8_unpack_bf16: K %% 1024, 16-byte aligned buffers");
  const long nchunks = (long)cdiv(N, 128) * 128 * (K / 16);
  hipLaunchKernelGGL(fp8_unpack_bf16_kernel, dim3((unsigned)cdiv(nchunks, 256)), dim3(256), 0,
                     S(stream), (const uint8_t*)W8, N, K, (bf16_t*)out);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_scale_cols(float* x, int M, int N, int ld, const float* scale, void* stream) {
  ZS_REQUIRE(M > 0 && N > 0 && N % 4 == 0 && ld % 4 == 0 && ld >= N && ((uintptr_t)x & 15) == 0 &&
                 ((uintptr_t)scale & 15) == 0,
             "zs_scale_cols: N, ld multiples of 4, 16-byte aligned");
  hipLaunchKernelGGL(scale_cols_kernel, dim3((unsigned)cdiv((long)M * N / 4, 256)), dim3(256), 0,
                     S(stream), x, M, N, ld, scale);
  ZS_LAUNCH_CHECK();
  return 0;
}

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
  ZS_REQUIRE(D % 4 == 0 && D <= 16384 && ss % 4 == 0 && ((uintptr_t)x & 15) == 0 &&
                 ((uintptr_t)h & 15) == 0 && (!y || ((uintptr_t)y & 15) == 0),
             "zs_mistral_add_rmsnorm: D <= 16384, D and split stride multiples of 4, 16-byte "
             "aligned rows");
  if (hdtype == ZS_BF16)
    hipLaunchKernelGGL(mistral_add_rmsnorm_kernel<bf16_t>, dim3(M), dim3(1024), 0, S(stream), x,
                       y, nsplit, ss, D, eps, w, (bf16_t*)h);
  else
    hipLaunchKernelGGL(mistral_add_rmsnorm_kernel<float>, dim3(M), dim3(1024), 0, S(stream), x,
                       y, nsplit, ss, D, eps, w, (float*)h);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_mistral_add_ss(float* x, const float* y, int nsplit, long ss, int M, int D,
                                 void* xb, float* rss, void* stream) {
  ZS_REQUIRE(M > 0 && M <= 32 && D > 0 && D % 512 == 0 && D <= 64 * 512 && x && xb && rss &&
                 (y == nullptr || (nsplit >= 1 && ss % 4 == 0 && ((uintptr_t)y & 15) == 0)) &&
                 ((uintptr_t)x & 15) == 0 && ((uintptr_t)xb & 7) == 0,
             "zs_mistral_add_ss: M <= 32, D %% 512 (<= 32768), aligned buffers (M=%d D=%d)", M, D);
  hipLaunchKernelGGL(mistral_add_ss_kernel, dim3(M, D / 512), dim3(128), 0, S(stream), x, y, nsplit,
                     ss, D, (bf16_t*)xb, rss);
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
  ZS_REQUIRE(F % 8 == 0 && ss % 4 == 0 && ((uintptr_t)gu & 15) == 0 && ((uintptr_t)act & 15) == 0,
             "zs_mistral_silu_mul: F %% 8, the split stride %% 4, 16-byte aligned buffers");
  const int nb = cdiv((long)M * F / 4, 256);
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

extern "C" int zs_mistral_decode_attention(const float* qkv, int nsplit, long ss, int M, int H,
                                           int KVH, const int* pos, const float* cosb,
                                           const float* sinb, void* kc, void* vc, int Lmax,
                                           void* out, int dtype, void* stream) {
  ZS_REQUIRE(M > 0 && H > 0 && KVH > 0 && H % KVH == 0 && nsplit >= 1 && Lmax > 0,
             "zs_mistral_decode_attention: bad shape");
  ZS_REQUIRE(ss % 4 == 0 && ((uintptr_t)qkv & 15) == 0 && ((uintptr_t)kc & 15) == 0 &&
                 ((uintptr_t)vc & 15) == 0 && ((uintptr_t)out & 15) == 0,
             "zs_mistral_decode_attention: 16-byte aligned buffers, split stride %% 4");
  const dim3 grid(cdiv((long)M * H, 4));
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(mistral_decode_attn_kernel<bf16_t>, grid, dim3(256), 0, S(stream), qkv,
                       nsplit, ss, M, H, KVH, pos, cosb, sinb, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       (bf16_t*)out);
  else
    hipLaunchKernelGGL(mistral_decode_attn_kernel<float>, grid, dim3(256), 0, S(stream), qkv,
                       nsplit, ss, M, H, KVH, pos, cosb, sinb, (float*)kc, (float*)vc, Lmax,
                       (float*)out);
  ZS_LAUNCH_CHECK();
  return 0;
}

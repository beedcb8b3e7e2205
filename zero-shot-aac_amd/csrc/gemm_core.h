// MFMA GEMM core shared by gemm.hip (Linear / LM head) and cnn.hip (implicit-GEMM conv3x3).
// See gemm.hip for the tiling description.
#pragma once
#include "common.h"

namespace zs {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int BK = 32;

template <typename T> struct GemmTraits;
template <> struct GemmTraits<bf16_t> {
  static constexpr int EPC = 8;    // elements per 16-byte chunk
  static constexpr int PAD = 8;    // 16-byte row pad
};
template <> struct GemmTraits<float> {
  static constexpr int EPC = 4;
  static constexpr int PAD = 4;
};

struct GemmArgs {
  int M, N, K, lda, ldw, ldr, ldo;
  const void* A;
  const void* W;
  const float* bias;
  const float* residual;
  void* out;
  int out_dtype, act, split_k, k_per_split;
  float* ws;
  int dbg;   // experiment knob (zs_tune_set "gemm_dbg"): 1 = skip MFMA, 2 = skip DMA
  int xcd;   // tile order: 1 = XCD-local grouped (zs_tune_set "fast_xcd"), 0 = n-fastest
};

// Loads a ROWS x 32 tile (row-major, K-contiguous) of a [nrows][ld] matrix into registers.
template <typename T, int ROWS>
struct TileLoader {
  static constexpr int EPC = GemmTraits<T>::EPC;
  static constexpr int CPR = BK / EPC;                 // chunks per row
  static constexpr int CHUNKS = ROWS * CPR;
  static constexpr int PER_T = (CHUNKS + 255) / 256;
  uint4 r[PER_T];
  __device__ __forceinline__ void load(const T* base, int row0, int nrows, int ld, int k0) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      int c = threadIdx.x + i * 256;
      int row = c / CPR, col = (c % CPR) * EPC;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (c < CHUNKS && row0 + row < nrows)
        v = *reinterpret_cast<const uint4*>(base + (long)(row0 + row) * ld + k0 + col);
      r[i] = v;
    }
  }
  __device__ __forceinline__ void store(T* lds) {
    constexpr int LDW = BK + GemmTraits<T>::PAD;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      int c = threadIdx.x + i * 256;
      if (c < CHUNKS) {
        int row = c / CPR, col = (c % CPR) * EPC;
        *reinterpret_cast<uint4*>(lds + row * LDW + col) = r[i];
      }
    }
  }
};

// one 32-deep k-tile of MFMAs for a wave: acc[TM][TN] += As(rows) * Ws(rows)^T
template <typename T, int TM, int TN> struct WaveMma;

template <int TM, int TN> struct WaveMma<bf16_t, TM, TN> {
  static __device__ __forceinline__ void run(const bf16_t* As, const bf16_t* Ws, int wr0, int wc0,
                                             f32x16_t (&acc)[TM][TN]) {
    constexpr int LDW = BK + GemmTraits<bf16_t>::PAD;
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[i] = *reinterpret_cast<const bf16x8_t*>(As + (wr0 + i * 32 + r) * LDW + s * 16 + 8 * h);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[j] = *reinterpret_cast<const bf16x8_t*>(Ws + (wc0 + j * 32 + r) * LDW + s * 16 + 8 * h);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
};

template <int TM, int TN> struct WaveMma<float, TM, TN> {
  static __device__ __forceinline__ void run(const float* As, const float* Ws, int wr0, int wc0,
                                             f32x16_t (&acc)[TM][TN]) {
    constexpr int LDW = BK + GemmTraits<float>::PAD;
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    // lane half h owns k in [16h, 16h+16); MFMA step s consumes k = s (half 0) and 16+s (half 1)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[i] = *reinterpret_cast<const float4*>(As + (wr0 + i * 32 + r) * LDW + 16 * h + 4 * q);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[j] = *reinterpret_cast<const float4*>(Ws + (wc0 + j * 32 + r) * LDW + 16 * h + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            float av = e == 0 ? a[i].x : e == 1 ? a[i].y : e == 2 ? a[i].z : a[i].w;
            float bv = e == 0 ? b[j].x : e == 1 ? b[j].y : e == 2 ? b[j].z : b[j].w;
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0);
          }
    }
  }
};

// Dense row-major A operand (the plain GEMM and the LM head)
template <typename T, int BM>
struct DenseA {
  const T* A;
  int lda, M, m0;
  TileLoader<T, BM> t;
  __device__ __forceinline__ void load(int k0) { t.load(A, m0, M, lda, k0); }
  __device__ __forceinline__ void store(T* lds) { t.store(lds); }
};

// main loop shared by the plain GEMM, the LM-head kernel and the implicit-GEMM conv; returns the
// wave's accumulators.  ALoader stages the BM x 32 A tile for a given k0.
template <typename T, int BM, int BN, typename ALoader>
__device__ __forceinline__ void gemm_mainloop(ALoader& la, const T* W, int ldw, int N, int n0,
                                              int kbeg, int kend, T* smem,
                                              f32x16_t (&acc)[BM / 64][BN / 64]) {
  constexpr int LDW = BK + GemmTraits<T>::PAD;
  constexpr int TM = BM / 64, TN = BN / 64;
  T* As[2] = {smem, smem + BM * LDW};
  T* Ws[2] = {smem + 2 * BM * LDW, smem + 2 * BM * LDW + BN * LDW};
  const int wid = threadIdx.x >> 6, wr0 = (wid >> 1) * (BM / 2), wc0 = (wid & 1) * (BN / 2);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  TileLoader<T, BN> lw;
  const int nk = (kend - kbeg) / BK;
  if (nk <= 0) return;
  la.load(kbeg);
  lw.load(W, n0, N, ldw, kbeg);
  la.store(As[0]);
  lw.store(Ws[0]);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      la.load(kbeg + (kt + 1) * BK);
      lw.load(W, n0, N, ldw, kbeg + (kt + 1) * BK);
    }
    WaveMma<T, TM, TN>::run(As[cur], Ws[cur], wr0, wc0, acc);
    if (kt + 1 < nk) {
      la.store(As[cur ^ 1]);
      lw.store(Ws[cur ^ 1]);
    }
    __syncthreads();
  }
}

}  // namespace zs

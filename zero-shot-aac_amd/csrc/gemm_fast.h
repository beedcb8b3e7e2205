// bf16 MFMA GEMM main loop staged by LDS-DMA (global_load_lds_dwordx4), BK = 64.
//
// One LDS stage holds the block's A rows [BM][64] and W rows [BN][64] as 128-byte rows.  A
// glds wave-instruction writes 1 KiB lane-linearly (8 rows x 128 B: lane l -> row l/8, 16-byte
// slot l%8), so the bank swizzle is applied on the SOURCE address: slot s of row r holds the
// logical 16-byte chunk c = s ^ ((r >> 1) & 7), and the MFMA fragment read of chunk c of row r
// reads slot c ^ ((r >> 1) & 7) — the same involution on both sides (cdna_hip_programming.md
// §5.4 rule 21).  A 16-lane ds_read_b128 group reads 16 consecutive rows at one logical chunk;
// (r & 1, (r >> 1) & 7) is then a bijection onto the 16 slots of the 256-byte bank row:
// conflict-free.
//
// Two stages: at the top of k-tile t one barrier (its implicit vmcnt(0) retires stage t's
// DMAs, and every wave has finished reading stage t-1), then the DMAs of tile t+1 are issued
// into the other stage and overlap tile t's MFMAs.  Out-of-range rows and the K tail read a
// 16-byte zero chunk instead (no predicated DMA, no stale LDS), so any M, N and K % 32 == 0 work.
#pragma once
#include "gemm_core.h"

namespace zs {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gptr_t;

constexpr int FBK = 64;   // k per stage

static __device__ __attribute__((aligned(16))) uint4 g_zero_chunk[1];

// rows [row0, nrows) of a row-major bf16 matrix with leading dimension ld
struct DenseRows {
  const bf16_t* p;
  int ld, nrows, row0;
  __device__ __forceinline__ const void* chunk(int r, int k, int kend) const {
    const int row = row0 + r;
    const bool ok = row < nrows && k < kend;       // a select, not a branch
    const bf16_t* q = p + (long)(ok ? row : 0) * ld + (ok ? k : 0);
    return ok ? (const void*)q : (const void*)g_zero_chunk;
  }
};

__device__ __forceinline__ int fswz(int row) { return (row >> 1) & 7; }

template <int BM, int BN>
struct FastTile {
  static constexpr int ROWS = BM + BN;
  static constexpr int STAGE = ROWS * 128;          // bytes
  static constexpr int NI = ROWS / 8;               // DMA instructions per stage
  static_assert(NI % 4 == 0, "rows per stage must be a multiple of 32");
  static constexpr int WM = BM / 2, WN = BN / 2;    // wave tile (2 x 2 waves)
  static constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
};

template <int BM, int BN, typename ASrc, typename BSrc>
__device__ __forceinline__ void fast_issue(const ASrc& A, const BSrc& B, int k0, int kend,
                                           char* stage) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // A rows: BM/8 wave-instructions, then W rows: BN/8 (both multiples of 4: no branch on A/W)
#pragma unroll
  for (int j = 0; j < BM / 32; ++j) {
    const int i = wid + 4 * j;
    const int row = 8 * i + (lane >> 3);
    const int k = k0 + 8 * ((lane & 7) ^ fswz(row));
    __builtin_amdgcn_global_load_lds((gptr_t)A.chunk(row, k, kend), (lds_ptr_t)(stage + i * 1024),
                                     16, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < BN / 32; ++j) {
    const int i = BM / 8 + wid + 4 * j;
    const int row = 8 * i + (lane >> 3);
    const int k = k0 + 8 * ((lane & 7) ^ fswz(row));
    __builtin_amdgcn_global_load_lds((gptr_t)B.chunk(row - BM, k, kend),
                                     (lds_ptr_t)(stage + i * 1024), 16, 0, 0);
  }
}

template <int BM, int BN>
__device__ __forceinline__ void fast_compute(const char* stage,
                                             f32x16_t (&acc)[BM / 64][BN / 64]) {
  using FT = FastTile<BM, BN>;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int wr0 = (wid >> 1) * FT::WM, wc0 = BM + (wid & 1) * FT::WN;
#pragma unroll
  for (int s = 0; s < FBK / 16; ++s) {
    const int c = 2 * s + h;
    bf16x8_t a[FT::TM], b[FT::TN];
#pragma unroll
    for (int i = 0; i < FT::TM; ++i) {
      const int row = wr0 + i * 32 + r;
      a[i] = *reinterpret_cast<const bf16x8_t*>(stage + row * 128 + 16 * (c ^ fswz(row)));
    }
#pragma unroll
    for (int j = 0; j < FT::TN; ++j) {
      const int row = wc0 + j * 32 + r;
      b[j] = *reinterpret_cast<const bf16x8_t*>(stage + row * 128 + 16 * (c ^ fswz(row)));
    }
#pragma unroll
    for (int i = 0; i < FT::TM; ++i)
#pragma unroll
      for (int j = 0; j < FT::TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// acc[i][j] (wave tile (BM/2) x (BN/2) as TM x TN 32x32 fragments; the C/D layout of §3:
// col = lane & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) over k in [kbeg, kend).
//
// NS-stage ring: tiles t+1 .. t+NS-1 stay in flight while tile t is computed.  Per k-tile:
// counted `s_waitcnt vmcnt` retiring this wave's DMAs of tile t (NS-2 younger tiles may stay
// outstanding), a raw s_barrier (every wave's tile-t DMAs retired and every wave done reading
// tile t-1, whose stage is refilled next), the DMAs of tile t+NS-1, then tile t's MFMAs.  A
// __syncthreads() here would drain all DMAs (vmcnt(0)): cdna_hip_programming.md §5
// "Pipelining across barriers".
template <int BM, int BN, int NS = 2, typename ASrc, typename BSrc>
__device__ __forceinline__ void fast_mainloop(const ASrc& A, const BSrc& B, int kbeg, int kend,
                                              char* lds, f32x16_t (&acc)[BM / 64][BN / 64]) {
  using FT = FastTile<BM, BN>;
  constexpr int IPW = FT::NI / 4;                 // DMA instructions per wave per tile
  static_assert(NS >= 2 && (NS - 2) * IPW < 64, "stages");
#pragma unroll
  for (int i = 0; i < FT::TM; ++i)
#pragma unroll
    for (int j = 0; j < FT::TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int nk = (kend - kbeg + FBK - 1) / FBK;
  if (nk <= 0) return;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) fast_issue<BM, BN>(A, B, kbeg + p * FBK, kend, lds + p * FT::STAGE);
  int st = 0;                                     // stage of tile kt
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + NS - 2 < nk) wait_vm<(NS - 2) * IPW>();   // tiles kt+1..kt+NS-2 may stay in flight
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    const int tn = kt + NS - 1;
    if (tn < nk) {
      const int sn = st == 0 ? NS - 1 : st - 1;   // (kt + NS - 1) % NS == stage of tile kt-1
      fast_issue<BM, BN>(A, B, kbeg + tn * FBK, kend, lds + sn * FT::STAGE);
    }
    fast_compute<BM, BN>(lds + st * FT::STAGE, acc);
    st = st == NS - 1 ? 0 : st + 1;
  }
  __syncthreads();   // callers may reuse the LDS for the epilogue
}

}  // namespace zs

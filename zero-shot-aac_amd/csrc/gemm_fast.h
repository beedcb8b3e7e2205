// bf16 MFMA GEMM main loop staged by LDS-DMA (global_load_lds_dwordx4), BK = 32 or 64.
//
// One LDS stage holds the block's A rows [BM][BK] and W rows [BN][BK] as RB = 2*BK-byte rows.
// A glds wave-instruction writes 1 KiB lane-linearly (1024/RB rows; lane l -> row l/(RB/16),
// 16-byte slot l%(RB/16)), so the bank swizzle is applied on the SOURCE address: slot s of row r
// holds the logical 16-byte chunk c = s ^ swz(r) with swz(r) = (r / (256/RB)) % (RB/16), and the
// MFMA fragment read of chunk c of row r reads slot c ^ swz(r) — the same involution on both
// sides (cdna_hip_programming.md §5.4 rule 21).  A 16-lane ds_read_b128 group reads 16
// consecutive rows at one logical chunk; (r % (256/RB), swz(r)) is then a bijection onto the 16
// slots of the 256-byte bank row: conflict-free (SQ_LDS_BANK_CONFLICT = 0 measured).
//
// NS-stage ring with counted `s_waitcnt vmcnt` + raw s_barrier (see fast_mainloop).  Out-of-range
// rows and the K tail read a 16-byte zero chunk instead (no predicated DMA, no stale LDS), so any
// M, N and K % 32 == 0 work.
#pragma once
#include "gemm_core.h"

namespace zs {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gptr_t;

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

// BM x BN block tile computed by WGM x WGN waves, each owning a WM x WN = (BM/WGM) x (BN/WGN)
// wave tile of TM x TN 32x32 MFMA fragments; k staged BK at a time
template <int BM, int BN, int WGM = 2, int WGN = 2, int BK_ = 64>
struct FastTile {
  static constexpr int BKT = BK_;
  static constexpr int RB = 2 * BK_;                // bytes per staged row
  static constexpr int SPR = RB / 16;               // 16-byte slots per row
  static constexpr int RPI = 1024 / RB;             // rows per DMA wave-instruction
  static constexpr int RP256 = 256 / RB;            // rows per 256-byte bank row
  static constexpr int NW = WGM * WGN;              // waves per block
  static constexpr int ROWS = BM + BN;
  static constexpr int STAGE = ROWS * RB;           // bytes
  static constexpr int NI = ROWS / RPI;             // DMA instructions per stage
  static_assert(BK_ == 32 || BK_ == 64 || BK_ == 128, "BK");
  static_assert(BM % (RPI * NW) == 0 && BN % (RPI * NW) == 0, "DMA rows per wave");
  static constexpr int WM = BM / WGM, WN = BN / WGN;
  static constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
  __device__ static __forceinline__ int swz(int row) { return (row / RP256) % SPR; }
};

template <int BM, int BN, int WGM, int WGN, int BK_, typename ASrc, typename BSrc>
__device__ __forceinline__ void fast_issue_t(const ASrc& A, const BSrc& B, int k0, int kend,
                                             char* stage) {
  using FT = FastTile<BM, BN, WGM, WGN, BK_>;
  constexpr int NW = FT::NW;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rsub = lane / FT::SPR, slot = lane % FT::SPR;
  // A rows: BM/RPI wave-instructions, then W rows (both multiples of NW: no branch on A/W)
#pragma unroll
  for (int j = 0; j < BM / (FT::RPI * NW); ++j) {
    const int i = wid + NW * j;
    const int row = FT::RPI * i + rsub;
    const int k = k0 + 8 * (slot ^ FT::swz(row));
    __builtin_amdgcn_global_load_lds((gptr_t)A.chunk(row, k, kend), (lds_ptr_t)(stage + i * 1024),
                                     16, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < BN / (FT::RPI * NW); ++j) {
    const int i = BM / FT::RPI + wid + NW * j;
    const int row = FT::RPI * i + rsub;
    const int k = k0 + 8 * (slot ^ FT::swz(row));
    __builtin_amdgcn_global_load_lds((gptr_t)B.chunk(row - BM, k, kend),
                                     (lds_ptr_t)(stage + i * 1024), 16, 0, 0);
  }
}

// SSQ: also accumulate, per lane, the sum of squares of the B fragments it reads (row
// wc0 + j*32 + (lane & 31), its half of every k-slice): with the xor-32 partner's sum that is
// the squared norm of the B row — the LM head's get_prefix_tokens row norms for free
//
// F32: the staged rows hold f32 (RB bytes = RB / 4 k per row; callers stage an f32 matrix as a
// bf16 one of twice the leading dimension and twice the k range, so the DMA, the swizzle and the
// ring are byte-for-byte the bf16 ones).  A 16-byte chunk is then 4 consecutive k, consumed by 4
// v_mfma_f32_32x32x2f32 (exact f32 products, f32 accumulation): MFMA e of chunk pair s pairs
// k = 4 (2s) + e (lane half 0) with k = 4 (2s + 1) + e (half 1), the same permutation of k on
// the A and B sides.
template <int BM, int BN, int WGM, int WGN, int BK_, bool SSQ = false, bool PRIO = false,
          bool F32 = false>
__device__ __forceinline__ void fast_compute(
    const char* stage,
    f32x16_t (&acc)[FastTile<BM, BN, WGM, WGN, BK_>::TM][FastTile<BM, BN, WGM, WGN, BK_>::TN],
    float* ssq = nullptr) {
  using FT = FastTile<BM, BN, WGM, WGN, BK_>;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const int wr0 = (wid / WGN) * FT::WM, wc0 = BM + (wid % WGN) * FT::WN;
  if constexpr (F32) {
#pragma unroll
    for (int s = 0; s < BK_ / 16; ++s) {
      const int c = 2 * s + h;
      float4 a[FT::TM], b[FT::TN];
#pragma unroll
      for (int i = 0; i < FT::TM; ++i) {
        const int row = wr0 + i * 32 + r;
        a[i] = *reinterpret_cast<const float4*>(stage + row * FT::RB + 16 * (c ^ FT::swz(row)));
      }
#pragma unroll
      for (int j = 0; j < FT::TN; ++j) {
        const int row = wc0 + j * 32 + r;
        b[j] = *reinterpret_cast<const float4*>(stage + row * FT::RB + 16 * (c ^ FT::swz(row)));
        if constexpr (SSQ) ssq[j] += (b[j].x * b[j].x + b[j].y * b[j].y) + (b[j].z * b[j].z + b[j].w * b[j].w);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < FT::TM; ++i)
#pragma unroll
          for (int j = 0; j < FT::TN; ++j) {
            const float av = e == 0 ? a[i].x : e == 1 ? a[i].y : e == 2 ? a[i].z : a[i].w;
            const float bv = e == 0 ? b[j].x : e == 1 ? b[j].y : e == 2 ? b[j].z : b[j].w;
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0);
          }
    }
    return;
  }
#pragma unroll
  for (int s = 0; s < BK_ / 16; ++s) {
    const int c = 2 * s + h;
    bf16x8_t a[FT::TM], b[FT::TN];
#pragma unroll
    for (int i = 0; i < FT::TM; ++i) {
      const int row = wr0 + i * 32 + r;
      a[i] = *reinterpret_cast<const bf16x8_t*>(stage + row * FT::RB + 16 * (c ^ FT::swz(row)));
    }
#pragma unroll
    for (int j = 0; j < FT::TN; ++j) {
      const int row = wc0 + j * 32 + r;
      b[j] = *reinterpret_cast<const bf16x8_t*>(stage + row * FT::RB + 16 * (c ^ FT::swz(row)));
      if constexpr (SSQ) {
#pragma unroll
        for (int u = 0; u < 8; ++u) { const float x = (float)b[j][u]; ssq[j] += x * x; }
      }
    }
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FT::TM; ++i)
#pragma unroll
      for (int j = 0; j < FT::TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// acc[i][j] (wave tile WM x WN as TM x TN 32x32 fragments; the C/D layout of §3:
// col = lane & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) over k in [kbeg, kend).
//
// NS-stage ring: tiles t+1 .. t+NS-1 stay in flight while tile t is computed.  Per k-tile:
// counted `s_waitcnt vmcnt` retiring this wave's DMAs of tile t (NS-2 younger tiles may stay
// outstanding), a raw s_barrier (every wave's tile-t DMAs retired and every wave done reading
// tile t-1, whose stage is refilled next), the DMAs of tile t+NS-1, then tile t's MFMAs.  A
// __syncthreads() here would drain all DMAs (vmcnt(0)): cdna_hip_programming.md §5
// "Pipelining across barriers".  Under full-chip streaming a DMA takes ~2-3 us to land, so the
// ring depth (NS-1 tiles in flight), not the MFMA count, sets the k-loop rate.
// The ring's prologue: tiles 0 .. NS-2 of [kbeg, kend) into stages 0 .. NS-2.
template <int BM, int BN, int NS = 2, int WGM = 2, int WGN = 2, int BK_ = 64, typename ASrc,
          typename BSrc>
__device__ __forceinline__ void fast_prologue(const ASrc& A, const BSrc& B, int kbeg, int kend,
                                              char* lds) {
  using FT = FastTile<BM, BN, WGM, WGN, BK_>;
  const int nk = (kend - kbeg + BK_ - 1) / BK_;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk)
      fast_issue_t<BM, BN, WGM, WGN, BK_>(A, B, kbeg + p * BK_, kend, lds + p * FT::STAGE);
}

// `prologued`: the caller already issued the prologue (fast_prologue), possibly followed by
// other vector-memory operations of this wave — at least XS of them when `xs` is set (a
// persistent tile loop issues the next tile's prologue before the current tile's epilogue
// stores).  vmcnt counts loads, stores and LDS-DMA together in issue order
// (MI355X_MICROARCH.md), so the waits for the prologue stages may leave those XS younger
// operations in flight: the stores then drain under the next tile's first k-steps.
template <int BM, int BN, int NS = 2, int WGM = 2, int WGN = 2, int BK_ = 64, bool SSQ = false,
          int XS = 0, bool F32 = false, typename ASrc, typename BSrc>
__device__ __forceinline__ void fast_mainloop(
    const ASrc& A, const BSrc& B, int kbeg, int kend, char* lds,
    f32x16_t (&acc)[FastTile<BM, BN, WGM, WGN, BK_>::TM][FastTile<BM, BN, WGM, WGN, BK_>::TN],
    int dbg = 0, float* ssq = nullptr, bool prologued = false, bool xs = false) {
  using FT = FastTile<BM, BN, WGM, WGN, BK_>;
  constexpr int IPW = FT::NI / FT::NW;            // DMA instructions per wave per tile
  static_assert(NS >= 2 && (NS - 2) * IPW + XS < 64, "stages");
#pragma unroll
  for (int i = 0; i < FT::TM; ++i)
#pragma unroll
    for (int j = 0; j < FT::TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int nk = (kend - kbeg + BK_ - 1) / BK_;
  if (nk <= 0) return;
  if (!prologued) fast_prologue<BM, BN, NS, WGM, WGN, BK_>(A, B, kbeg, kend, lds);
  int st = 0;                                     // stage of tile kt
  for (int kt = 0; kt < nk; ++kt) {
    const bool young = XS > 0 && xs && kt < NS - 1;   // XS younger ops behind this stage
    if (kt + NS - 2 < nk) {                       // tiles kt+1..kt+NS-2 may stay in flight
      if (young) wait_vm<(NS - 2) * IPW + XS>(); else wait_vm<(NS - 2) * IPW>();
    } else {
      if (young) wait_vm<XS>(); else wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    const int tn = kt + NS - 1;
    if (tn < nk && dbg != 2 && dbg != 3) {
      const int sn = st == 0 ? NS - 1 : st - 1;   // (kt + NS - 1) % NS == stage of tile kt-1
      fast_issue_t<BM, BN, WGM, WGN, BK_>(A, B, kbeg + tn * BK_, kend, lds + sn * FT::STAGE);
    }
    if (dbg != 1 && dbg != 3)
      fast_compute<BM, BN, WGM, WGN, BK_, SSQ, false, F32>(lds + st * FT::STAGE, acc, ssq);
    st = st == NS - 1 ? 0 : st + 1;
  }
  __syncthreads();   // callers may reuse the LDS for the epilogue
}

// Lean variant of the ring (gemm_lean_kernel, lmhead_kernel): the per-lane DMA source pointers
// of the tile's A rows [m0, m0+BM) and W rows [n0, n0+BN) are computed once (rows clamped into
// the matrices; clamped rows only feed outputs the caller's store guard drops) and K % BK == 0,
// so a k-step carries just the counted wait, the raw barrier, IPW pointer adds + DMAs and the
// MFMAs (fast_mainloop's per-chunk zero-chunk selects and 64-bit row products are gone).
template <int BM, int BN, int NS, int WGM, int WGN, int BK_, bool SSQ = false, bool PRIO = false>
__device__ __forceinline__ void lean_mainloop(
    const bf16_t* A, int lda, int M, int m0, const bf16_t* W, int ldw, int N, int n0, int K,
    char* lds,
    f32x16_t (&acc)[FastTile<BM, BN, WGM, WGN, BK_>::TM][FastTile<BM, BN, WGM, WGN, BK_>::TN],
    float* ssq = nullptr) {
  using FT = FastTile<BM, BN, WGM, WGN, BK_>;
  constexpr int NW = FT::NW, IPW = FT::NI / NW;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bf16_t* src[IPW];
  {
    const int rsub = lane / FT::SPR, slot = lane % FT::SPR;
#pragma unroll
    for (int j = 0; j < IPW; ++j) {
      const int i = wid + NW * j;                   // DMA instruction: rows RPI*i .. +RPI
      const int row = FT::RPI * i + rsub;
      const int c = 8 * (slot ^ FT::swz(row));
      if (row < BM) src[j] = A + (long)min(m0 + row, M - 1) * lda + c;   // wave-uniform branch
      else src[j] = W + (long)min(n0 + row - BM, N - 1) * ldw + c;
    }
  }
  auto issue = [&](int stage, int k0) {
#pragma unroll
    for (int j = 0; j < IPW; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(src[j] + k0),
                                       (lds_ptr_t)(lds + stage * FT::STAGE + (wid + NW * j) * 1024),
                                       16, 0, 0);
  };
#pragma unroll
  for (int i = 0; i < FT::TM; ++i)
#pragma unroll
    for (int j = 0; j < FT::TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int nk = K / BK_;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) issue(p, p * BK_);
  int st = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + NS - 2 < nk) wait_vm<(NS - 2) * IPW>(); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + NS - 1 < nk) issue(st == 0 ? NS - 1 : st - 1, (kt + NS - 1) * BK_);
    fast_compute<BM, BN, WGM, WGN, BK_, SSQ, PRIO>(lds + st * FT::STAGE, acc, ssq);
    st = st == NS - 1 ? 0 : st + 1;
  }
  __syncthreads();   // callers may reuse the LDS for the epilogue
}

}  // namespace zs

// MFMA GEMM for every Linear/Conv1D on the hot path, plus the LM-head GEMM with a fused
// per-row max / sum-exp / top-k epilogue (greedy argmax, beam log-softmax top-k,
// get_prefix_tokens cosine argmax).
//
//   out[m][n] = act(sum_k A[m][k] * W[n][k] + bias[n]) + residual[m][n]
//
// Tiles: BM x BN x 32, 256 threads = 4 waves in a 2x2 grid, each wave owning (BM/2) x (BN/2) as
// 32x32 MFMA tiles.  bf16: v_mfma_f32_32x32x16_bf16 (2 per 32-deep k-tile); f32 (parity mode):
// v_mfma_f32_32x32x2f32 with lane-half h owning k in [16h,16h+16) so both dtypes share one LDS
// image ([row][32 + 16B pad], read 16 B per lane).  Global->LDS is register staged and double
// buffered (next tile's loads issued before the current tile's MFMAs).
#include <algorithm>
#include "gemm_fast.h"

namespace zs {

int g_gemm_fast = 1;   // zs_tune_set("gemm_fast", 0) selects the register-staged bf16 loop
int g_gemm_dbg = 0;   // experiments: 1 no MFMA, 2 no DMA, 3 neither, 4 no epilogue, 5 launch
                      // only, 6 no global stores (tools/mbench.py gemm_dbg)
int g_fast_xcd = 1;       // zs_tune_set("fast_xcd", 0): n-fastest tile order

__device__ __forceinline__ void store_out(void* out, int out_dtype, long idx, float v) {
  if (out_dtype == ZS_BF16) reinterpret_cast<bf16_t*>(out)[idx] = f2bf(v);
  else reinterpret_cast<float*>(out)[idx] = v;
}

template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  constexpr int LDW = BK + GemmTraits<T>::PAD;
  __shared__ __attribute__((aligned(16))) T smem[2 * (BM + BN) * LDW];
  constexpr int TM = BM / 64, TN = BN / 64;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM, z = blockIdx.z;
  const int kbeg = z * g.k_per_split, kend = min(g.K, kbeg + g.k_per_split);
  f32x16_t acc[TM][TN];
  DenseA<T, BM> la{(const T*)g.A, g.lda, g.M, m0};
  gemm_mainloop<T, BM, BN>(la, (const T*)g.W, g.ldw, g.N, n0, kbeg, kend, smem, acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr0 = (wid >> 1) * (BM / 2), wc0 = (wid & 1) * (BN / 2);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wc0 + j * 32 + (lane & 31);
      if (n >= g.N) continue;
      const float bias = (g.split_k == 1 && g.bias) ? g.bias[n] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wr0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (m >= g.M) continue;
        float v = acc[i][j][e];
        if (g.split_k > 1) {
          g.ws[((long)z * g.M + m) * g.N + n] = v;
        } else {
          v = act_apply(v + bias, g.act);
          if (g.residual) v += g.residual[(long)m * g.ldr + n];
          store_out(g.out, g.out_dtype, (long)m * g.ldo + n, v);
        }
      }
    }
}

// deterministic split-K reduction: sum slabs in order, then the same epilogue
__global__ void splitk_reduce_kernel(GemmArgs g) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)g.M * g.N;
  if (idx >= total) return;
  int m = idx / g.N, n = idx % g.N;
  float v = 0.f;
  for (int z = 0; z < g.split_k; ++z) v += g.ws[(long)z * total + idx];
  if (g.bias) v += g.bias[n];
  v = act_apply(v, g.act);
  if (g.residual) v += g.residual[(long)m * g.ldr + n];
  store_out(g.out, g.out_dtype, (long)m * g.ldo + n, v);
}

// One wave's parked [32][WN] f32 slab -> out rows mr0..mr0+31, cols nc0..nc0+WN-1: each lane
// owns 8 consecutive columns (two ds_read_b128), so residual loads and the bf16 store are 16 B
// per lane over contiguous row segments; ACT is a template parameter (no per-element switch).
// `bb` (the lane's 8 bias values) is loaded once per tile by the caller, and the slab's residual
// rows are loaded before the slab is read back: a residual load issued after the previous
// row's store would make its wait (vmcnt counts stores too) a full write round trip per row.
template <int ACT, int WN>
__device__ __forceinline__ void epi_slab(const GemmArgs& g, const float* slab, int mr0, int nc0,
                                         int z, bool vec_out, bool vec_res, const float (&bb)[8],
                                         const float4 (&res)[WN / 16][2]) {
  constexpr int Q = WN / 8, IT = 32 * Q / 64;
  static_assert(IT * 64 == 32 * Q, "slab iterations");
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = lane + 64 * it;
    const int r = idx / Q, c = (idx % Q) * 8;
    const int m = mr0 + r, n = nc0 + c;
    if (m >= g.M || n >= g.N) continue;
    const float4 a0 = *reinterpret_cast<const float4*>(slab + r * WN + c);
    const float4 a1 = *reinterpret_cast<const float4*>(slab + r * WN + c + 4);
    float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const int nv = min(8, g.N - n);
    const bool full = nv == 8;
    if (g.split_k > 1) {
      float* dst = g.ws + ((long)z * g.M + m) * g.N + n;
      if (full && g.N % 4 == 0) {
        reinterpret_cast<float4*>(dst)[0] = make_float4(v[0], v[1], v[2], v[3]);
        reinterpret_cast<float4*>(dst)[1] = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        for (int q = 0; q < nv; ++q) dst[q] = v[q];
      }
      continue;
    }
    if constexpr (64 % Q == 0) {   // a lane's 8 columns are the same in every iteration
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = act_apply_fast(v[q] + bb[q], ACT);
    } else {                       // (WN = 96: they move with the iteration)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        v[q] = act_apply_fast(v[q] + ((g.bias && q < nv) ? g.bias[n + q] : 0.f), ACT);
    }
    if (g.residual) {
      if (full && vec_res) {
        const float4 r0 = res[it][0], r1 = res[it][1];
        v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
        v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
      } else {
        const float* rp = g.residual + (long)m * g.ldr + n;
        for (int q = 0; q < nv; ++q) v[q] += rp[q];
      }
    }
    const long o = (long)m * g.ldo + n;
    if (full && vec_out) {
      if (g.out_dtype == ZS_BF16) {
        uint4 u;
        u.x = pk2bf(v[0], v[1]);
        u.y = pk2bf(v[2], v[3]);
        u.z = pk2bf(v[4], v[5]);
        u.w = pk2bf(v[6], v[7]);
        if (g.dbg != 6 || u.x == 0x7fc17fc1u)   // dbg 6 (experiment): no global stores
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g.out) + o) = u;
      } else {
        float4* d = reinterpret_cast<float4*>(reinterpret_cast<float*>(g.out) + o);
        d[0] = make_float4(v[0], v[1], v[2], v[3]);
        d[1] = make_float4(v[4], v[5], v[6], v[7]);
      }
    } else {
      for (int q = 0; q < nv; ++q) store_out(g.out, g.out_dtype, o + q, v[q]);
    }
  }
}

// the residual rows a lane's epi_slab iterations will add (full 8-column segments only)
template <int WN>
__device__ __forceinline__ void epi_res_load(const GemmArgs& g, int mr0, int nc0, bool vec_res,
                                             float4 (&res)[WN / 16][2]) {
  constexpr int Q = WN / 8, IT = 32 * Q / 64;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = lane + 64 * it;
    const int m = mr0 + idx / Q, n = nc0 + (idx % Q) * 8;
    if (g.residual && vec_res && g.split_k == 1 && m < g.M && n + 8 <= g.N) {
      const float4* rp = reinterpret_cast<const float4*>(g.residual + (long)m * g.ldr + n);
      res[it][0] = rp[0];
      res[it][1] = rp[1];
    } else {
      res[it][0] = res[it][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// bf16: the LDS-DMA staged main loop (gemm_fast.h).  Epilogue through LDS: each wave parks one
// 32-row slab of its accumulators ([32][WN] f32, static register indexing), then re-reads it
// row-wise so every lane owns 4 consecutive columns: bias / activation / residual / store move
// 16 B (f32) or 8 B (bf16) per lane in full rows instead of 2-4 B column-strided scalars.
template <int BM, int BN, int NS, int WGM, int WGN, int BK_, bool F32 = false>
// 4-wave tiles are held to 2 waves per SIMD (<= 256 unified VGPRs): two resident blocks per CU,
// so one block's epilogue and DMA waits overlap the other's MFMAs (at 312 registers the 128x128
// tile ran one block per CU)
// F32 (the f32 parity mode): f32 A / W staged as bf16 rows of twice the length (KF = 2 bf16 units
// per f32 element), consumed by v_mfma_f32_32x32x2f32 (fast_compute F32); same ring, tile order
// and epilogue
__global__ __launch_bounds__(64 * WGM * WGN,
                             (WGM * WGN == 4 && NS * FastTile<BM, BN, WGM, WGN, BK_>::STAGE <= 80 * 1024)
                                 ? 2 : 1) void gemm_fast_kernel(GemmArgs g) {
  constexpr int KF = F32 ? 2 : 1;
  using FT = FastTile<BM, BN, WGM, WGN, BK_>;
  __shared__ __attribute__((aligned(16))) char lds[NS * FT::STAGE];
  constexpr int TM = FT::TM, TN = FT::TN, WN = FT::WN;
  if (g.dbg == 5) return;   // experiment: launch cost only
  static_assert(FT::NW * 32 * WN * 4 <= NS * FT::STAGE, "epilogue slab must fit the stage ring");
  // persistent: a grid of (CUs x resident blocks) walks the tiles (n fastest, then m, then the
  // k split), so the per-workgroup dispatch cost is paid once per resident block, not per tile
  const int ntn = cdiv(g.N, BN), ntm = cdiv(g.M, BM);
  const int ntiles = ntn * ntm * g.split_k;
  // XCD-local order: workgroups are placed round-robin on the 8 XCDs (slot v runs on XCD v % 8
  // whenever the grid is a multiple of 8 or one slot per tile), and each XCD has its own L2.
  // Slot v -> u makes the tiles of one XCD a contiguous range (bijective for any count), and u
  // walks groups of gm M-tiles column by column, so a range is a compact gm x (range/gm) patch
  // of the output: its A rows and W rows stay in that XCD's L2 instead of every XCD streaming
  // all of A and W.
  // gm: the patch an XCD works on AT ONCE (its gridDim/8 resident blocks take consecutive u)
  // is about square, so its A rows + W rows fit the XCD's 4 MB L2 (a gm sized for the whole
  // per-XCD range made 39 x 2 patches on 65536 x 3072: 7.5 MB of A rows, 43 % L2 misses)
  const int q8 = ntiles >> 3, r8 = ntiles & 7;
  const int conc = max(1, min(q8, (int)(gridDim.x >> 3)));
  int gm = (int)(sqrtf((float)conc * BN / BM) + 0.5f);
  gm = max(1, min(gm, ntm));
  auto tile = [&](int t, int& m0, int& n0, int& z) {
    if (g.xcd) {
      const int x = t & 7;
      const int u = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + (t >> 3);
      z = u / (ntn * ntm);
      const int w = u - z * (ntn * ntm), per = gm * ntn, grp = w / per, fm = grp * gm;
      const int gs = min(ntm - fm, gm), r = w - grp * per;
      m0 = (fm + r % gs) * BM;
      n0 = (r / gs) * BN;
    } else {
      n0 = (t % ntn) * BN; m0 = ((t / ntn) % ntm) * BM; z = t / (ntn * ntm);
    }
  };
  // Cross-tile prefetch (XPF): the next tile's prologue stages (0 .. NS-2) are issued before this
  // tile's epilogue, whose slab lives in stage NS-1, so the DMA latency of the next tile's first
  // k-steps runs under the epilogue, and its first waits may leave the epilogue's stores in
  // flight (XS = a lower bound on the stores one wave issues for a full tile: >= 1 per slab row
  // iteration).
  constexpr bool XPF = FT::NW * 32 * WN * 4 <= FT::STAGE;
  constexpr int XS = XPF ? TM * (32 * (WN / 8) / 64) : 0;
  int m0, n0, z;
  int t = blockIdx.x;
  if (t < ntiles) tile(t, m0, n0, z);
  bool pre = false, xs = false;
  if (XPF && t < ntiles && g.dbg != 2 && g.dbg != 3) {
    const int kb = z * g.k_per_split;
    fast_prologue<BM, BN, NS, WGM, WGN, BK_>(DenseRows{(const bf16_t*)g.A, KF * g.lda, g.M, m0},
                                             DenseRows{(const bf16_t*)g.W, KF * g.ldw, g.N, n0},
                                             KF * kb, KF * min(g.K, kb + g.k_per_split), lds);
    pre = true;
  }
  for (; t < ntiles; t += gridDim.x) {
  const int kbeg = z * g.k_per_split, kend = min(g.K, kbeg + g.k_per_split);
  f32x16_t acc[TM][TN];
  const DenseRows A{(const bf16_t*)g.A, KF * g.lda, g.M, m0};
  const DenseRows B{(const bf16_t*)g.W, KF * g.ldw, g.N, n0};
  fast_mainloop<BM, BN, NS, WGM, WGN, BK_, false, XS, F32>(A, B, KF * kbeg, KF * kend, lds, acc,
                                                           g.dbg, nullptr, pre, xs);   // ends with a barrier
  const int cm0 = m0, cn0 = n0, cz = z;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr0 = (wid / WGN) * FT::WM, wc0 = (wid % WGN) * WN;
  // 16-byte stores need 8-element (bf16) / 4-element (f32) aligned rows and bias
  const bool vec_out = (g.split_k > 1) ||
                       (g.ldo % 8 == 0 && ((uintptr_t)g.out & 15) == 0);
  const bool vec_res = g.residual == nullptr ||
                       (g.ldr % 4 == 0 && ((uintptr_t)g.residual & 15) == 0);
  // The bias and the first slab's residual rows are loaded BEFORE the next tile's prologue
  // DMAs: vmcnt retires in issue order, so a load issued after those DMAs could only be
  // consumed once the DMAs had landed (a full DMA latency per tile).  The lane's 8 bias columns
  // are the same in every slab of the tile (64 % (WN/8) == 0).
  float bb[8];
  {
    const int n = cn0 + wc0 + (lane % (WN / 8)) * 8, nv = min(8, g.N - n);
    if (g.bias && nv == 8 && ((uintptr_t)(g.bias + n) & 15) == 0) {
      const float4 b0 = reinterpret_cast<const float4*>(g.bias + n)[0];
      const float4 b1 = reinterpret_cast<const float4*>(g.bias + n)[1];
      bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w;
      bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) bb[q] = (g.bias && q < nv) ? g.bias[n + q] : 0.f;
    }
  }
  float4 res0[WN / 16][2];
  epi_res_load<WN>(g, cm0 + wr0, cn0 + wc0, vec_res, res0);
  pre = xs = false;
  if (XPF && t + (int)gridDim.x < ntiles && g.dbg != 2 && g.dbg != 3) {
    tile(t + gridDim.x, m0, n0, z);
    const int kb = z * g.k_per_split;
    fast_prologue<BM, BN, NS, WGM, WGN, BK_>(DenseRows{(const bf16_t*)g.A, KF * g.lda, g.M, m0},
                                             DenseRows{(const bf16_t*)g.W, KF * g.ldw, g.N, n0},
                                             KF * kb, KF * min(g.K, kb + g.k_per_split), lds);
    pre = true;
    xs = g.dbg != 4 && cm0 + BM <= g.M && cn0 + BN <= g.N;   // full tile: >= XS stores follow
  } else if (t + (int)gridDim.x < ntiles) {
    tile(t + gridDim.x, m0, n0, z);
  }
  float* slab = reinterpret_cast<float*>(lds + (XPF ? (NS - 1) * FT::STAGE : 0)) + wid * 32 * WN;
  if (g.dbg == 4) {   // experiment: no epilogue (keep the accumulators alive)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) t += acc[i][j][0];
    if (t == 12345.f) reinterpret_cast<float*>(g.out)[0] = t;
    continue;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mr0 = cm0 + wr0 + i * 32, nc0 = cn0 + wc0;
    float4 res[WN / 16][2];
    if (i == 0) {
#pragma unroll
      for (int q = 0; q < WN / 16; ++q) { res[q][0] = res0[q][0]; res[q][1] = res0[q][1]; }
    } else {
      epi_res_load<WN>(g, mr0, nc0, vec_res, res);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        slab[((e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * WN + j * 32 + (lane & 31)] = acc[i][j][e];
    // the slab is private to this wave and a wave's LDS accesses complete in issue order, so
    // no barrier: a __syncthreads() here would also wait for every outstanding global store
    // (vmcnt(0)) and serialise one full write round trip per row slab
    switch (g.act) {
      case ACT_GELU_ERF: epi_slab<ACT_GELU_ERF, WN>(g, slab, mr0, nc0, cz, vec_out, vec_res, bb, res); break;
      case ACT_GELU_TANH: epi_slab<ACT_GELU_TANH, WN>(g, slab, mr0, nc0, cz, vec_out, vec_res, bb, res); break;
      case ACT_RELU: epi_slab<ACT_RELU, WN>(g, slab, mr0, nc0, cz, vec_out, vec_res, bb, res); break;
      case ACT_TANH: epi_slab<ACT_TANH, WN>(g, slab, mr0, nc0, cz, vec_out, vec_res, bb, res); break;
      default: epi_slab<ACT_NONE, WN>(g, slab, mr0, nc0, cz, vec_out, vec_res, bb, res); break;
    }
  }
  // every wave has read its slab before the next tile's DMAs refill the LDS (LDS-only wait:
  // the stores stay in flight)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  }
}

// ------------------------------------------------------------------ lean tile kernel
// One output tile per workgroup, no persistent loop, no split-K, K % BK == 0: the decode-step
// shapes (M = 256..4096 rows, N = 768..3072, K = 768 / 3072).  Same swizzled LDS-DMA ring as
// gemm_fast_kernel, but the per-lane DMA source pointers are computed ONCE per tile (rows
// clamped into the matrix instead of a per-chunk zero-chunk select; clamped rows only feed
// outputs the store guard drops), and the k-loop carries nothing but the counted wait, the raw
// barrier, IPW pointer adds + DMAs and the MFMAs: gemm_fast_kernel's persistent / cross-tile /
// split-K / experiment control flow spilled SGPRs into VGPR lanes and cost ~300 cycles of
// scalar work per k-step, more than a 64x64 tile's MFMAs.
template <int BM, int BN, int NS, int BK_, int WGM = 2, int WGN = 2>
__global__ __launch_bounds__(64 * WGM * WGN, WGM * WGN == 4 ? 2 : 1) void gemm_lean_kernel(GemmArgs g) {
  using FT = FastTile<BM, BN, WGM, WGN, BK_>;
  constexpr int TM = FT::TM, TN = FT::TN, WN = FT::WN, NW = WGM * WGN;
  static_assert(NW * 32 * WN * 4 <= NS * FT::STAGE, "epilogue slab fits the ring");
  __shared__ __attribute__((aligned(16))) char lds[NS * FT::STAGE];
  const int ntn = cdiv(g.N, BN), ntm = cdiv(g.M, BM), ntiles = ntn * ntm;
  // XCD-local grouped tile order (see gemm_fast_kernel): slot b runs on XCD b % 8
  int m0, n0;
  {
    const int b = blockIdx.x, x = b & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int u = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + (b >> 3);
    const int conc = max(1, min(q8, 64));
    int gm = (int)(sqrtf((float)conc * BN / BM) + 0.5f);
    gm = max(1, min(gm, ntm));
    const int per = gm * ntn, grp = u / per, fm = grp * gm;
    const int gs = min(ntm - fm, gm), r = u - grp * per;
    m0 = (fm + r % gs) * BM;
    n0 = (r / gs) * BN;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  f32x16_t acc[TM][TN];
  // s_setprio(1) around each MFMA cluster (cdna_hip_programming.md T5): -2..-4 % at the
  // 8192-row decode shapes, neutral elsewhere
  lean_mainloop<BM, BN, NS, WGM, WGN, BK_, false, true>((const bf16_t*)g.A, g.lda, g.M, m0,
                                                        (const bf16_t*)g.W, g.ldw, g.N, n0, g.K,
                                                        lds, acc);
  const int wr0 = (wid / WGN) * FT::WM, wc0 = (wid % WGN) * WN;
  const bool vec_out = g.ldo % 8 == 0 && ((uintptr_t)g.out & 15) == 0;
  const bool vec_res = g.residual == nullptr || (g.ldr % 4 == 0 && ((uintptr_t)g.residual & 15) == 0);
  float bb[8];
  {
    const int n = n0 + wc0 + (lane % (WN / 8)) * 8, nv = min(8, g.N - n);
    if (g.bias && nv == 8 && ((uintptr_t)(g.bias + n) & 15) == 0) {
      const float4 b0 = reinterpret_cast<const float4*>(g.bias + n)[0];
      const float4 b1 = reinterpret_cast<const float4*>(g.bias + n)[1];
      bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w;
      bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) bb[q] = (g.bias && q < nv) ? g.bias[n + q] : 0.f;
    }
  }
  float* slab = reinterpret_cast<float*>(lds) + wid * 32 * WN;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mr0 = m0 + wr0 + i * 32, nc0 = n0 + wc0;
    float4 res[WN / 16][2];
    epi_res_load<WN>(g, mr0, nc0, vec_res, res);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        slab[((e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * WN + j * 32 + (lane & 31)] = acc[i][j][e];
    switch (g.act) {
      case ACT_GELU_ERF: epi_slab<ACT_GELU_ERF, WN>(g, slab, mr0, nc0, 0, vec_out, vec_res, bb, res); break;
      case ACT_GELU_TANH: epi_slab<ACT_GELU_TANH, WN>(g, slab, mr0, nc0, 0, vec_out, vec_res, bb, res); break;
      case ACT_RELU: epi_slab<ACT_RELU, WN>(g, slab, mr0, nc0, 0, vec_out, vec_res, bb, res); break;
      case ACT_TANH: epi_slab<ACT_TANH, WN>(g, slab, mr0, nc0, 0, vec_out, vec_res, bb, res); break;
      default: epi_slab<ACT_NONE, WN>(g, slab, mr0, nc0, 0, vec_out, vec_res, bb, res); break;
    }
  }
}

// ------------------------------------------------------------------ 256 x 256 multi-phase tile
// For GEMMs with >= ~1k rows (prefill, the throughput mode, the beam decode at 1280 rows, the
// BERT tower, HTSAT stage 4, the Mistral prefill).  One 512-thread workgroup (8 waves as 2 (M) x
// 4 (N)) per CU owns a 256 x 256 output tile; each wave a 128 x 64 sub-tile as 8 x 4 fragments
// of v_mfma_f32_16x16x32_bf16 (128 accumulator registers).  K in 64-deep tiles, two LDS buffers
// of [256 A rows][256 W rows] x 128 B (128 KiB), staged by LDS-DMA (global_load_lds_dwordx4) with
// the bank swizzle on the source address (FastTile's involution, conflict-free 16-lane reads).
//
// A K-tile is computed in FOUR phases, one output quadrant of every wave each (16 MFMAs):
//   p0 (m0, n0): reads the wave's A rows m0 (4 fragments x 2 k-steps) and W rows n0
//   p1 (m0, n1): reads W rows n1
//   p2 (m1, n1): reads A rows m1
//   p3 (m1, n0): no reads (n0 still in registers)
// so the LDS rows of a K-tile free up in four SETS as their readers finish (A-m0 + W-n0 after p0,
// W-n1 after p1, A-m1 after p2), and each set of K-tile t+2 is staged into the same buffer as
// soon as it is free (p1: A-m0 + W-n0, p2: W-n1, p3: A-m1) — seven phases before it is read.
// Every phase: counted `s_waitcnt vmcnt` retiring this wave's DMAs of the set(s) read in it
// (never vmcnt(0) in steady state), ONE raw s_barrier (RAW: every wave's DMAs of the set landed;
// WAR: every wave's reads of the sets restaged in this phase done — each wave's reads complete
// before its MFMAs of the previous phase), the phase's reads, the restaging DMAs, the MFMAs at
// raised priority (cdna_hip_programming.md §5 "Pipelining across barriers", the 256² template).
namespace big {
constexpr int BM = 256, BN = 256, BKB = 64, RB = 128, BUF = (BM + BN) * RB;
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }
// LDS DMA instruction index (8 rows of 128 B each) of instruction j (0..15) of row set `set`:
// 0 = A rows m0 of both wave rows, 1 = A rows m1, 2 = W rows n0 of the 4 wave columns, 3 = n1
__device__ __forceinline__ int set_instr(int set, int j) {
  if (set < 2) return ((j >> 3) * 128 + set * 64) / 8 + (j & 7);
  return (BM + (j >> 2) * 64 + (set - 2) * 32) / 8 + (j & 3);
}
}  // namespace big

typedef __attribute__((ext_vector_type(4))) float f32x4_t;
// the wave's 128 x 64 accumulators as 4 slabs of 32 rows ([32][64] f32, 8 KiB of LDS each)
template <int ACT>
__device__ __forceinline__ void big_epilogue(const GemmArgs& g, float* slab, int mrw, int nc0,
                                             bool vec_out, bool vec_res, const float (&bb)[8],
                                             const f32x4_t (&acc)[8][4]) {
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) {
    const int mr0 = mrw + 32 * sl;
    float4 res[4][2];
    epi_res_load<64>(g, mr0, nc0, vec_res, res);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          slab[(16 * ii + 4 * fq + e) * 64 + 16 * j + fr] = acc[2 * sl + ii][j][e];
    epi_slab<ACT, 64>(g, slab, mr0, nc0, 0, vec_out, vec_res, bb, res);
  }
}

__global__ __launch_bounds__(512) void gemm_big_kernel(GemmArgs g) {
  using namespace big;
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int ntn = cdiv(g.N, BN), ntm = cdiv(g.M, BM), ntiles = ntn * ntm;
  int m0, n0;
  {  // XCD-local grouped tile order (as gemm_lean_kernel)
    const int b = blockIdx.x, x = b & 7, q8 = ntiles >> 3, r8 = ntiles & 7;
    const int u = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + (b >> 3);
    const int conc = max(1, min(q8, 32));
    int gm = (int)(sqrtf((float)conc) + 0.5f);
    gm = max(1, min(gm, ntm));
    const int per = gm * ntn, grp = u / per, fm = grp * gm;
    const int gs = min(ntm - fm, gm), r = u - grp * per;
    m0 = (fm + r % gs) * BM;
    n0 = (r / gs) * BN;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wr = wid >> 2, wc = wid & 3;
  const bf16_t* A = (const bf16_t*)g.A;
  const bf16_t* W = (const bf16_t*)g.W;
  // per lane: the source of its 2 DMA instructions in each of the 4 sets, as element offsets
  // from A / W (rows clamped into the matrices; clamped rows feed only outputs the store guard
  // drops)
  int src[4][2];
#pragma unroll
  for (int set = 0; set < 4; ++set)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int idx = set_instr(set, wid + 8 * jj);
      const int row = 8 * idx + (lane >> 3);
      const int c = 8 * ((lane & 7) ^ swz(row));
      src[set][jj] = set < 2 ? min(m0 + row, g.M - 1) * g.lda + c
                             : min(n0 + row - BM, g.N - 1) * g.ldw + c;
    }
  auto issue = [&](int set, char* bufp, int k0) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
      __builtin_amdgcn_global_load_lds((gptr_t)((set < 2 ? A : W) + src[set][jj] + k0),
                                       (lds_ptr_t)(bufp + set_instr(set, wid + 8 * jj) * 1024),
                                       16, 0, 0);
  };
  auto tile_issue = [&](char* bufp, int k0) {  // the steady-state order: A-m0, W-n0, W-n1, A-m1
    issue(0, bufp, k0); issue(2, bufp, k0); issue(3, bufp, k0); issue(1, bufp, k0);
  };
  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int nk = g.K / BKB;
  tile_issue(lds, 0);
  if (nk > 1) tile_issue(lds + BUF, BKB);
  const int fr = lane & 15, fq = lane >> 4;
  // fragment rows step by 16 (a multiple of the swizzle period 2 x 8 rows): one swizzle per
  // lane, so a fragment is base + 2048 * i (+ the k-step's chunk), an immediate offset
  const int arow = wr * 128 + fr, brow = BM + wc * 64 + fr;
  int aoff[2], boff[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    aoff[s2] = arow * RB + 16 * ((4 * s2 + fq) ^ swz(arow));
    boff[s2] = brow * RB + 16 * ((4 * s2 + fq) ^ swz(brow));
  }
  bf16x8_t a[4][2], b0[2][2], b1[2][2];
#pragma unroll 1
  for (int t = 0; t < nk; ++t) {
    char* bufp = lds + (t & 1) * BUF;
    const bool pf = t + 2 < nk;                  // this K-tile restages its sets with t + 2
    const int kn = (t + 2) * BKB;
    // ---- p0 (m0, n0)
    if (pf || t + 2 == nk) wait_vm<12>(); else wait_vm<4>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        a[i][s2] = *reinterpret_cast<const bf16x8_t*>(bufp + aoff[s2] + 2048 * i);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        b0[j][s2] = *reinterpret_cast<const bf16x8_t*>(bufp + boff[s2] + 2048 * j);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s2], b0[j][s2], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // ---- p1 (m0, n1)
    if (pf || t + 2 == nk) wait_vm<10>(); else wait_vm<2>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        b1[j][s2] = *reinterpret_cast<const bf16x8_t*>(bufp + boff[s2] + 2048 * (2 + j));
    if (pf) { issue(0, bufp, kn); issue(2, bufp, kn); }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s2], b1[j][s2], acc[i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // ---- p2 (m1, n1)
    if (pf) wait_vm<12>(); else if (t + 2 == nk) wait_vm<8>(); else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        a[i][s2] = *reinterpret_cast<const bf16x8_t*>(bufp + aoff[s2] + 2048 * (4 + i));
    if (pf) issue(3, bufp, kn);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s2], b1[j][s2], acc[4 + i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // ---- p3 (m1, n0): no reads; restage A-m1 (read in p2)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (pf) issue(1, bufp, kn);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s2], b0[j][s2], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  wait_vm<0>();
  __syncthreads();   // the LDS becomes the epilogue's slabs
  // epilogue: 4 slabs of 32 rows per wave ([32][64] f32, 8 KiB), as gemm_lean_kernel
  const bool vec_out = g.ldo % 8 == 0 && ((uintptr_t)g.out & 15) == 0;
  const bool vec_res = g.residual == nullptr || (g.ldr % 4 == 0 && ((uintptr_t)g.residual & 15) == 0);
  const int nc0 = n0 + wc * 64;
  float bb[8];
  {
    const int n = nc0 + (lane % 8) * 8, nv = min(8, g.N - n);
    if (g.bias && nv == 8 && ((uintptr_t)(g.bias + n) & 15) == 0) {
      const float4 c0 = reinterpret_cast<const float4*>(g.bias + n)[0];
      const float4 c1 = reinterpret_cast<const float4*>(g.bias + n)[1];
      bb[0] = c0.x; bb[1] = c0.y; bb[2] = c0.z; bb[3] = c0.w;
      bb[4] = c1.x; bb[5] = c1.y; bb[6] = c1.z; bb[7] = c1.w;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) bb[q] = (g.bias && q < nv) ? g.bias[n + q] : 0.f;
    }
  }
  float* slab = reinterpret_cast<float*>(lds) + wid * 32 * 64;
  const int mrw = m0 + wr * 128;
  switch (g.act) {
    case ACT_GELU_ERF: big_epilogue<ACT_GELU_ERF>(g, slab, mrw, nc0, vec_out, vec_res, bb, acc); break;
    case ACT_GELU_TANH: big_epilogue<ACT_GELU_TANH>(g, slab, mrw, nc0, vec_out, vec_res, bb, acc); break;
    case ACT_RELU: big_epilogue<ACT_RELU>(g, slab, mrw, nc0, vec_out, vec_res, bb, acc); break;
    case ACT_TANH: big_epilogue<ACT_TANH>(g, slab, mrw, nc0, vec_out, vec_res, bb, acc); break;
    default: big_epilogue<ACT_NONE>(g, slab, mrw, nc0, vec_out, vec_res, bb, acc); break;
  }
}

// measured (tools/mbench.py gemm_big, random operands): 1096 TF at 4096^3 and 1252 TF at 8192^3
// against 909 / 968 for the lean 128 x 128 tiles; at K = 768 (every GPT-2 / HTSAT / BERT shape)
// and at grids of < 256 tiles the tile's prologue, 128 KiB epilogue and second-round tail cost
// more than its MFMA efficiency saves (8192 x 3072 x 768: 60 vs 56 us; 1280-1600 rows: 2-4x
// slower), so it is taken only for long K on a full grid
int g_gemm_big = 1;    // zs_tune_set("gemm_big", 0): no 256 x 256 multi-phase tiles
int g_big_min = 256;   // zs_tune_set("big_min", n): 256 x 256 tiles from n tiles up (K >= 2048)

static int launch_big(GemmArgs& g, hipStream_t st) {
  hipLaunchKernelGGL(gemm_big_kernel, dim3(cdiv(g.N, 256) * cdiv(g.M, 256)), dim3(512), 0, st, g);
  ZS_LAUNCH_CHECK();
  return 0;
}

int g_gemm_lean = 1;   // zs_tune_set("gemm_lean", 0): decode-shaped GEMMs on gemm_fast_kernel
int g_lean96 = 0;      // zs_tune_set("lean96", 1): 128x96 tiles for the N = 768 projections
                       // (faster alone, but -2 % end to end with the decode groups co-running)
int g_lean8w = 0;      // zs_tune_set("lean8w", 1): 8-wave 256x128 tile for the 8192-row c_fc
                       // (57.5 vs 60.8 us alone, but -0.6 % end to end: A/B in one box)

template <int BM, int BN, int NS, int BK_, int WGM = 2, int WGN = 2>
static int launch_lean(GemmArgs& g, hipStream_t st) {
  hipLaunchKernelGGL((gemm_lean_kernel<BM, BN, NS, BK_, WGM, WGN>),
                     dim3(cdiv(g.N, BN) * cdiv(g.M, BM)), dim3(64 * WGM * WGN), 0, st, g);
  ZS_LAUNCH_CHECK();
  return 0;
}

int g_fast_persist = 1;   // zs_tune_set("fast_persist", 0): one workgroup per tile

template <int BM, int BN, int NS, int WGM = 2, int WGN = 2, int BK_ = 64, bool F32 = false>
static int launch_fast(GemmArgs& g, hipStream_t st) {
  using FT = FastTile<BM, BN, WGM, WGN, BK_>;
  const long nt = (long)cdiv(g.N, BN) * cdiv(g.M, BM) * g.split_k;
  const int per_cu = max(1, min(160 * 1024 / (NS * FT::STAGE), 8 / FT::NW * 2));
  dim3 grid(g_fast_persist ? (int)std::min<long>(nt, 256L * per_cu) : (int)nt);
  hipLaunchKernelGGL((gemm_fast_kernel<BM, BN, NS, WGM, WGN, BK_, F32>), grid,
                     dim3(64 * WGM * WGN), 0, st, g);
  ZS_LAUNCH_CHECK();
  return 0;
}

static long nblocks(const GemmArgs& g, int bm, int bn) {
  return (long)cdiv(g.M, bm) * cdiv(g.N, bn) * g.split_k;
}

int g_fast_ns = 2;     // zs_tune_set("fast_ns", n): stages of the 128x128 tile (experiment knob)
int g_fast_tile = 0;   // zs_tune_set("fast_tile", t): force a tile (see dispatch_fast)
int g_lean_min128 = 256;  // zs_tune_set("lean_min128", n): 128x128 2-stage tiles from n tiles up
#ifndef ZS_LEAN128_NS
#define ZS_LEAN128_NS 3
#endif
// zs_tune_set("lean128_ns", 3 | 4): stages of the 8-wave 128x128 tile taken at 128 <= n128 < 256
// (3: 96 KiB of LDS, fits beside a grid-decode workgroup; 4: 128 KiB, round 4's tile)
int g_lean128_ns = ZS_LEAN128_NS;

// largest tile that still puts >= 1 block on every CU, else the smallest
static int dispatch_fast(GemmArgs& g, hipStream_t st) {
  switch (g_fast_tile) {
    case 1: return launch_fast<256, 256, 4, 2, 4, 32>(g, st);
    case 2: return launch_fast<256, 128, 4, 4, 2, 32>(g, st);
    case 3: return launch_fast<128, 256, 4, 2, 4, 32>(g, st);
    case 4: return launch_fast<128, 128, 2>(g, st);
    case 5: return launch_fast<128, 128, 4, 2, 2, 32>(g, st);
    case 6: return launch_fast<256, 256, 2, 2, 4, 64>(g, st);
    case 7: return launch_fast<128, 128, 6, 2, 2, 32>(g, st);
    case 8: return launch_fast<128, 64, 3>(g, st);
    case 9: return launch_fast<64, 128, 3>(g, st);
    case 10: return launch_fast<128, 128, 3>(g, st);
    case 11: return launch_fast<128, 128, 2, 2, 2, 32>(g, st);
    case 12: return launch_fast<128, 128, 3, 2, 2, 32>(g, st);
    case 13: return launch_fast<64, 64, 2>(g, st);
    case 14: return launch_fast<128, 128, 4>(g, st);
    case 15: return launch_fast<256, 128, 2, 4, 2, 64>(g, st);
    case 16: return launch_fast<128, 256, 2, 2, 4, 64>(g, st);
    case 17: return launch_fast<64, 64, 2, 2, 2, 128>(g, st);
    default: break;
  }
  if ((g_fast_tile == 18 || (g_gemm_big && g.K >= 2048 && nblocks(g, 256, 256) >= g_big_min)) &&
      g.split_k == 1 && g.K % 64 == 0 && g.lda % 8 == 0 && g.ldw % 8 == 0)
    return launch_big(g, st);
  if (g_gemm_lean && g.split_k == 1 && g.K % 64 == 0) {
    // measured (tools/mbench.py decode_gemm / gemm_dbg; M = 1024..98304 x the GPT-2 and HTSAT
    // shapes): 128x128 for big grids and while it makes 1-2 tiles per 2-block CU slot, 128x64
    // in between (4096-row decode qkv: 28.9 vs 34.3 us) and when 128x128 leaves CUs idle, else
    // 64x64 with a 4-deep ring
    const int lt = g_fast_tile >= 100 ? g_fast_tile - 100 : 0;   // experiment: force a lean tile
    const long n128 = nblocks(g, 128, 128);
    // (re-measured with the s_setprio main loop, tools/mbench.py gemm_dbg at M = 1024..8192 x
    // the GPT-2 shapes: 128x128 beats 128x64 at every n128 >= 256 — 8192x2304x768 46.9 vs 57.2
    // us, 4096x3072x768 30.8 vs 38.1; the 8-wave 256x128 3-stage tile at one block per CU is
    // best for the 8192-row c_fc, 57.5 vs 60.8; the 8-wave 128x128 4-stage tile for
    // 128 <= n128 < 256, 4096x768x3072 32.0 vs 34.8, 1024x3072x768 12.0 vs 13.3)
    if (!lt && g_lean8w && g.N >= 3072 && n128 >= 1024 && n128 <= 4096)
      return launch_lean<256, 128, 3, 64, 2, 4>(g, st);
    // 128x96 (4 waves as 4x1, 32x96 wave tiles) for the N = 768 projections at >= 6144 rows:
    // 8 column tiles, 2 blocks per CU (8192x768x3072 56.4 vs 59.2 us, 6144x768x3072 50.2 vs 53.7)
    if (!lt && g_lean96 && g.N % 96 == 0 && g.N <= 1536 && nblocks(g, 128, 96) >= 384)
      return launch_lean<128, 96, 2, 64, 4, 1>(g, st);
    if (lt == 1 || (!lt && n128 >= g_lean_min128)) return launch_lean<128, 128, 2, 64>(g, st);
    // (3 stages, 96 KiB of LDS: the 4-stage ring's 128 KiB does not fit beside a persistent decode
    // workgroup's 35 KiB, and the prefill would wait for a decode grid to end)
    if (!lt && n128 >= 128)
      return g_lean128_ns == 4 ? launch_lean<128, 128, 4, 64, 2, 4>(g, st)
                               : launch_lean<128, 128, 3, 64, 2, 4>(g, st);
    if (lt == 2 || (!lt && nblocks(g, 128, 64) >= 256))
      return g.M >= g.N ? launch_lean<128, 64, 3, 64>(g, st) : launch_lean<64, 128, 3, 64>(g, st);
    // 64x64 with 128-deep k-steps when a 64x64 grid is still under one tile per CU at >= 512
    // rows (the C3 beam decode's N = 768 projections at 1280 rows: proj 7.1 -> 6.5 us, mproj
    // 19.2 -> 17.7 us, tools/mbench.py gemm_c3)
    if ((lt == 3 || (!lt && g.M >= 512 && nblocks(g, 64, 64) < 256)) && g.K % 128 == 0)
      return launch_lean<64, 64, 2, 128>(g, st);
    // 8-wave tiles at one block per CU (experiments)
    if (lt == 5) return launch_lean<256, 128, 2, 64, 4, 2>(g, st);
    if (lt == 6) return launch_lean<128, 256, 2, 64, 2, 4>(g, st);
    if (lt == 7) return launch_lean<256, 256, 2, 64, 2, 4>(g, st);
    if (lt == 8) return launch_lean<256, 128, 3, 64, 4, 2>(g, st);
    if (lt == 9) return launch_lean<128, 256, 3, 64, 2, 4>(g, st);
    if (lt == 10) return launch_lean<256, 128, 3, 64, 2, 4>(g, st);
    if (lt == 11) return launch_lean<128, 128, 3, 64, 2, 4>(g, st);
    if (lt == 12) return launch_lean<128, 128, 4, 64, 2, 4>(g, st);
    if (lt == 13) return launch_lean<128, 96, 2, 64, 4, 1>(g, st);
    return launch_lean<64, 64, 4, 64>(g, st);
  }
  if (nblocks(g, 128, 128) >= 256) {
    if (g_fast_ns == 3) return launch_fast<128, 128, 3>(g, st);
    if (g_fast_ns == 4) return launch_fast<128, 128, 4>(g, st);
    return launch_fast<128, 128, 2>(g, st);
  }
  if (nblocks(g, 128, 64) >= 256) return g.M >= g.N ? launch_fast<128, 64, 3>(g, st)
                                                     : launch_fast<64, 128, 3>(g, st);
  // small tiles are bound by the per-k-step skeleton (counted wait + barrier + DMA issue,
  // ~300 cycles) rather than by their 4 MFMAs per wave: 128-deep k-steps halve the step count
  // (decode proj / c_proj at 2048 rows: 12.5 -> 11.7 us, 32 -> 28 us)
  if (g.k_per_split % 128 == 0) return launch_fast<64, 64, 2, 2, 2, 128>(g, st);
  return launch_fast<64, 64, 4>(g, st);
}

template <typename T, int BM, int BN>
static int launch_gemm(GemmArgs& g, hipStream_t st) {
  dim3 grid(cdiv(g.N, BN), cdiv(g.M, BM), g.split_k);
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN>), grid, dim3(256), 0, st, g);
  ZS_LAUNCH_CHECK();
  return 0;
}

// f32 parity mode on the LDS-DMA ring (gemm_fast_kernel F32): 32 f32 k per stage, 2 stages at
// 64 KiB (g_f32_tile 8), two blocks per CU; round 4's 16 k per stage x 4 stages at g_f32_tile 0.
// Needs 16-byte rows (K, lda, ldw multiples of 4, aligned bases); else the register-staged
// gemm_kernel<float>.
int g_f32_fast = 1;    // zs_tune_set("f32_fast", 0): f32 GEMMs on the register-staged kernel
// zs_tune_set("f32_tile", t): the f32 tile variant (tools/mbench.py gemm_f32_tiles,
// profiles/r5/f32_gemm_tiles.txt): 8 (default) = 64-k stages, 2 in flight, at every tile size --
// the f32 parity mode's HTSAT + prefill GEMMs 11.15 -> 10.00 ms, bit-identical (same k order);
// 0 = 16-k stages, 4 in flight (round 4); 1-7 = other variants
int g_f32_tile = 8;
static int dispatch_fast_f32(GemmArgs& g, hipStream_t st) {
  if (g_f32_tile >= 7) {     // 64-k stages, 2 in flight, at every tile size
    if (nblocks(g, 128, 128) >= 256) {
      if (g_f32_tile == 10) return launch_fast<128, 128, 2, 2, 2, 128, true>(g, st);
      if (g_f32_tile == 11 && nblocks(g, 256, 128) >= 256)
        return launch_fast<256, 128, 2, 4, 2, 64, true>(g, st);
      return g_f32_tile == 7 ? launch_fast<128, 128, 2, 2, 4, 64, true>(g, st)
                             : launch_fast<128, 128, 2, 2, 2, 64, true>(g, st);
    }
    if (nblocks(g, 128, 64) >= 256)
      return g.M >= g.N ? launch_fast<128, 64, 2, 2, 2, 64, true>(g, st)
                        : launch_fast<64, 128, 2, 2, 2, 64, true>(g, st);
    return launch_fast<64, 64, 2, 2, 2, 64, true>(g, st);
  }
  if (g_f32_tile && nblocks(g, 128, 128) >= 256) {
    switch (g_f32_tile) {
      case 1: return launch_fast<128, 128, 3, 2, 2, 64, true>(g, st);
      case 2: return launch_fast<128, 128, 2, 2, 2, 64, true>(g, st);
      case 3: return launch_fast<256, 128, 4, 4, 2, 32, true>(g, st);
      case 4: return launch_fast<128, 256, 4, 2, 4, 32, true>(g, st);
      case 5: return launch_fast<128, 128, 6, 2, 2, 32, true>(g, st);
      case 6: return launch_fast<128, 128, 4, 2, 4, 32, true>(g, st);
      default: break;
    }
  }
  if (nblocks(g, 128, 128) >= 256) return launch_fast<128, 128, 4, 2, 2, 32, true>(g, st);
  if (nblocks(g, 128, 64) >= 256)
    return g.M >= g.N ? launch_fast<128, 64, 4, 2, 2, 32, true>(g, st)
                      : launch_fast<64, 128, 4, 2, 2, 32, true>(g, st);
  return launch_fast<64, 64, 4, 2, 2, 32, true>(g, st);
}

template <typename T>
static int dispatch_gemm(GemmArgs& g, hipStream_t st) {
  if (sizeof(T) == 2 && g_gemm_fast) return dispatch_fast(g, st);
  if (sizeof(T) == 4 && g_f32_fast && g.K % 4 == 0 && g.lda % 4 == 0 && g.ldw % 4 == 0 &&
      g.k_per_split % 4 == 0 && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.W & 15) == 0)
    return dispatch_fast_f32(g, st);
  const bool small_m = g.M <= 64;
  const bool wide_n = g.N >= 2048 && !small_m;
  if (small_m) return wide_n ? launch_gemm<T, 64, 128>(g, st) : launch_gemm<T, 64, 64>(g, st);
  if (wide_n) return launch_gemm<T, 128, 128>(g, st);
  return launch_gemm<T, 128, 64>(g, st);
}

// ------------------------------------------------------------------ LM head (+ row reductions)
constexpr int LM_BN = 128;
constexpr int MAXK = 8;
int g_lm_prio = 1;   // zs_tune_set("lm_prio", 0): LM head main loop without s_setprio

// RING (f32 only; bf16 always): the LDS-DMA ring main loop and the transposed register epilogue
// (f32 rows staged as bf16 rows of twice the length, fast_compute F32)
template <typename T, int BM, int KMAX, bool RING = sizeof(T) == 2>
__global__ __launch_bounds__(256) void lmhead_kernel(int xcd_order, int M, int K, int V, const T* A, int lda,
                                                     const T* W, int topk, int row_norm,
                                                     float* part_stat, float* part_val,
                                                     int* part_idx, float temp) {
  // temp != 1: logits / temp before the top-k and the softmax statistics (generate2 /
  // generate_beam's `temperature`, gpt2_prefix_eval.py:121, 196); a true division, as the reference
  const bool tdiv = temp != 1.0f;
  constexpr int LDW = BK + GemmTraits<T>::PAD;
  constexpr int TM = BM / 64, TN = LM_BN / 64;
  constexpr int SM_MAIN = 2 * (BM + LM_BN) * LDW * (int)sizeof(T);
  constexpr int SM_EPI = BM * (LM_BN + 1) * 4;
  constexpr bool FAST = RING;
  constexpr int SM_LOOP = FAST ? 2 * FastTile<BM, LM_BN>::STAGE : SM_MAIN;  // 4 waves (2x2)
  constexpr int SM = SM_LOOP > SM_EPI ? SM_LOOP : SM_EPI;
  // ONE __shared__ array (a second object can de-pipeline the DMA loop: §5 item 4(a))
  __shared__ __attribute__((aligned(16))) char smem_raw[SM + BM * 4];
  float* inv_norm = reinterpret_cast<float*>(smem_raw + SM);
  // 1-D grid of nblk x ntm blocks.  XCD-local order: workgroup b runs on XCD b % 8; the remap
  // gives each XCD a contiguous range of u, and u walks the row tiles fastest, so every row tile
  // of a vocab block runs on the same XCD at about the same time: each 128-token W slice is
  // fetched into one L2 once and reused by all row tiles (with the vocab block fastest, the
  // 77 MB of W streamed once per row tile).
  const int ntm = cdiv(M, BM), nblk = cdiv(V, LM_BN), nwg = nblk * ntm;
  int vb, mb;
  if (xcd_order & 1) {
    const int b = blockIdx.x, x = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int u = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + (b >> 3);
    vb = u / ntm;
    mb = u - vb * ntm;
  } else {
    vb = blockIdx.x % nblk;
    mb = blockIdx.x / nblk;
  }
  const int n0 = vb * LM_BN, m0 = mb * BM;
  f32x16_t acc[TM][TN];
  // bf16: transposed product, vocab on the MFMA row axis, so a token's 128 logits of this block
  // sit in registers of one lane pair (see the epilogue below)
  f32x16_t acct[LM_BN / 64][BM / 64];
  float ssq[BM / 64];     // per lane: its half of the squared norm of token wc0 + j*32 + (lane&31)
  if constexpr (FAST && sizeof(T) == 4) {
    const DenseRows ra{(const bf16_t*)A, 2 * lda, M, m0};
    const DenseRows rw{(const bf16_t*)W, 2 * K, V, n0};
#pragma unroll
    for (int j = 0; j < BM / 64; ++j) ssq[j] = 0.f;
    if (row_norm)
      fast_mainloop<LM_BN, BM, 2, 2, 2, 64, true, 0, true>(rw, ra, 0, 2 * K, smem_raw, acct, 0, ssq);
    else
      fast_mainloop<LM_BN, BM, 2, 2, 2, 64, false, 0, true>(rw, ra, 0, 2 * K, smem_raw, acct);
  } else if constexpr (FAST) {
    const DenseRows ra{(const bf16_t*)A, lda, M, m0};
    const DenseRows rw{(const bf16_t*)W, K, V, n0};
#pragma unroll
    for (int j = 0; j < BM / 64; ++j) ssq[j] = 0.f;
    if (K % 64 == 0) {
      if (row_norm)
        lean_mainloop<LM_BN, BM, 2, 2, 2, 64, true>((const bf16_t*)W, K, V, n0, (const bf16_t*)A,
                                                    lda, M, m0, K, smem_raw, acct, ssq);
      else if (xcd_order & 2)   // s_setprio around the MFMA clusters, as gemm_lean_kernel
        lean_mainloop<LM_BN, BM, 2, 2, 2, 64, false, true>((const bf16_t*)W, K, V, n0,
                                                           (const bf16_t*)A, lda, M, m0, K,
                                                           smem_raw, acct);
      else
        lean_mainloop<LM_BN, BM, 2, 2, 2, 64>((const bf16_t*)W, K, V, n0, (const bf16_t*)A, lda,
                                              M, m0, K, smem_raw, acct);
    } else if (row_norm) {
      fast_mainloop<LM_BN, BM, 2, 2, 2, 64, true>(rw, ra, 0, K, smem_raw, acct, 0, ssq);
    } else {
      fast_mainloop<LM_BN, BM>(rw, ra, 0, K, smem_raw, acct);
    }
  } else {
    DenseA<T, BM> la{A, lda, M, m0};
    gemm_mainloop<T, BM, LM_BN>(la, W, K, V, n0, 0, K, (T*)smem_raw, acc);
  }
  // row norms for get_prefix_tokens (normalize(a) . w == (a . w) / max(||a||, 1e-12)); the
  // transposed top-1 path gets them from its own B fragments instead (see below)
  if (row_norm && !FAST) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int r = wid; r < BM; r += 4) {
      float s = 0.f;
      if (m0 + r < M)
        for (int k = lane; k < K; k += 64) {
          float a = ldf(A + (long)(m0 + r) * lda + k);
          s += a * a;
        }
      s = wave_sum(s);
      if (lane == 0) inv_norm[r] = 1.0f / fmaxf(sqrtf(s), 1e-12f);
    }
  }
  __syncthreads();
  if constexpr (FAST) {
    // acct[i][j][e]: vocab n0 + wr0 + i*32 + (e&3) + 8*(e>>2) + 4*(lane>>5), token
    // m0 + wc0 + j*32 + (lane&31).  Per token: a descending top-KMAX list and the sum-exp over the
    // lane's 32 vocab entries in registers, one xor-32 exchange with the partner lane, then the
    // two waves holding the other 64 vocab rows of the same tokens merge through LDS.  Ties keep
    // the lower vocab index (torch argmax / topk order).
    constexpr int TMV = LM_BN / 64, TNT = BM / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wr0 = (wid >> 1) * (LM_BN / 2), wc0 = (wid & 1) * (BM / 2), wg = wid >> 1;
    float* xm = reinterpret_cast<float*>(smem_raw);          // [2][BM] max
    float* xs = xm + 2 * BM;                                  // [2][BM] sum-exp
    float* xv = xs + 2 * BM;                                  // [2][BM][KMAX] top values
    int* xi = reinterpret_cast<int*>(xv + 2 * BM * KMAX);     // [2][BM][KMAX] top indices
    auto better = [](float v, int i, float w, int k) { return v > w || (v == w && i < k); };
#pragma unroll
    for (int j = 0; j < TNT; ++j) {
      const int r = wc0 + j * 32 + (lane & 31);                // token within the block
      float sc = 1.0f;
      if (row_norm) {
        const float t = ssq[j] + __shfl_xor(ssq[j], 32, 64);
        sc = 1.0f / fmaxf(sqrtf(t), 1e-12f);
      }
      float tv[KMAX];
      int ti[KMAX];
#pragma unroll
      for (int q = 0; q < KMAX; ++q) { tv[q] = -INFINITY; ti[q] = 0x7fffffff; }
#pragma unroll
      for (int i = 0; i < TMV; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int n = n0 + wr0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          float cv = n < V ? acct[i][j][e] * sc : -INFINITY;
          if (tdiv) cv = cv / temp;
          int ci = n;
          // n increases with (i, e): strict > keeps the lower index first among equals.  The
          // bubble insertion is select-only (per-element branches became ~500 divergent
          // exec-mask branches per kernel); the outer test skips a value no lane keeps
          if (cv > tv[KMAX - 1]) {
#pragma unroll
            for (int q = 0; q < KMAX; ++q) {
              const bool c = cv > tv[q];
              const float t = tv[q];
              const int u = ti[q];
              tv[q] = c ? cv : t;
              ti[q] = c ? ci : u;
              cv = c ? t : cv;
              ci = c ? u : ci;
            }
          }
        }
      // merge with the partner lane's list (both lanes end with the same top-KMAX)
      float pv[KMAX];
      int pi[KMAX];
#pragma unroll
      for (int q = 0; q < KMAX; ++q) { pv[q] = __shfl_xor(tv[q], 32, 64); pi[q] = __shfl_xor(ti[q], 32, 64); }
      if constexpr (KMAX > 1) {
        // merge of two descending lists, select-only: the partner's entries bubble into this
        // lane's list like new values (the same order as a merge: value desc, then index asc)
#pragma unroll
        for (int p = 0; p < KMAX; ++p) {
          float cv = pv[p];
          int ci = pi[p];
#pragma unroll
          for (int q = 0; q < KMAX; ++q) {
            const bool c = better(cv, ci, tv[q], ti[q]);
            const float t = tv[q];
            const int u = ti[q];
            tv[q] = c ? cv : t;
            ti[q] = c ? ci : u;
            cv = c ? t : cv;
            ci = c ? u : ci;
          }
        }
      } else {
        const bool c = better(pv[0], pi[0], tv[0], ti[0]);
        tv[0] = c ? pv[0] : tv[0];
        ti[0] = c ? pi[0] : ti[0];
      }
      const float bv = tv[0];
      float se = 0.f;
      // the softmax denominator only for callers that need log-probabilities (beam search);
      // greedy argmax and get_prefix_tokens pass part_stat = NULL and skip these 64 exps/lane
      if (part_stat != nullptr && bv != -INFINITY) {
#pragma unroll
        for (int i = 0; i < TMV; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int n = n0 + wr0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
            if (n < V) se += __expf((tdiv ? acct[i][j][e] * sc / temp : acct[i][j][e] * sc) - bv);
          }
        se += __shfl_xor(se, 32, 64);
      }
      if (lane < 32) {
        xm[wg * BM + r] = bv;
        xs[wg * BM + r] = se;
#pragma unroll
        for (int q = 0; q < KMAX; ++q) {
          xv[(wg * BM + r) * KMAX + q] = tv[q];
          xi[(wg * BM + r) * KMAX + q] = ti[q];
        }
      }
    }
    __syncthreads();
    for (int r = threadIdx.x; r < BM; r += 256) {
      const int m = m0 + r;
      if (m >= M) continue;
      const float m0v = xm[r], m1v = xm[BM + r];
      const float g = fmaxf(m0v, m1v);
      const float se = (m0v == -INFINITY ? 0.f : xs[r] * expf(m0v - g)) +
                       (m1v == -INFINITY ? 0.f : xs[BM + r] * expf(m1v - g));
      const long o = (long)m * nblk + vb;
      if (part_stat != nullptr) {
        part_stat[o * 2 + 0] = g;
        part_stat[o * 2 + 1] = se;
      }
      const float* l0v = xv + r * KMAX;
      const int* l0i = xi + r * KMAX;
      const float* l1v = xv + (BM + r) * KMAX;
      const int* l1i = xi + (BM + r) * KMAX;
      int a = 0, b = 0;
      for (int q = 0; q < topk; ++q) {
        const bool ta = b >= KMAX || (a < KMAX && better(l0v[a], l0i[a], l1v[b], l1i[b]));
        part_val[o * topk + q] = ta ? l0v[a] : l1v[b];
        part_idx[o * topk + q] = ta ? l0i[a] : l1i[b];
        if (ta) ++a; else ++b;
      }
    }
    return;
  }
  float* tile = reinterpret_cast<float*>(smem_raw);   // [BM][LM_BN+1]
  {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wr0 = (wid >> 1) * (BM / 2), wc0 = (wid & 1) * (LM_BN / 2);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int r = wr0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          const int c = wc0 + j * 32 + (lane & 31);
          tile[r * (LM_BN + 1) + c] = acc[i][j][e];
        }
  }
  __syncthreads();
  // each row is reduced by TPR threads, each scanning LM_BN/TPR consecutive columns
  constexpr int TPR = 256 / BM;
  constexpr int CPT = LM_BN / TPR;
  const int r = threadIdx.x / TPR, sub = threadIdx.x % TPR;
  const int m = m0 + r;
  const float scale = row_norm ? inv_norm[r] : 1.0f;
  float mx = -INFINITY;
  float tv[KMAX];
  int ti[KMAX];
#pragma unroll
  for (int q = 0; q < KMAX; ++q) { tv[q] = -INFINITY; ti[q] = 0x7fffffff; }
  for (int c = sub * CPT; c < sub * CPT + CPT; ++c) {
    const int n = n0 + c;
    if (n >= V) break;
    float v = tile[r * (LM_BN + 1) + c] * scale;
    if (tdiv) v = v / temp;
    mx = fmaxf(mx, v);
    // insertion into the descending top-k list (strict > keeps the lower index on ties)
    if (KMAX == 1) {
      if (v > tv[0]) { tv[0] = v; ti[0] = n; }
    } else if (v > tv[KMAX - 1]) {
      // bubble the new value up the (static-indexed) list
      float cv = v;
      int ci = n;
#pragma unroll
      for (int q = 0; q < KMAX; ++q) {   // select-only, as the transposed path above
        const bool c = cv > tv[q];
        const float t = tv[q];
        const int u = ti[q];
        tv[q] = c ? cv : t;
        ti[q] = c ? ci : u;
        cv = c ? t : cv;
        ci = c ? u : ci;
      }
    }
  }
  // combine max across the TPR threads of this row (consecutive lanes)
  float gmx = mx;
#pragma unroll
  for (int o = 1; o < TPR; o <<= 1) gmx = fmaxf(gmx, __shfl_xor(gmx, o, 64));
  float se = 0.f;
  for (int c = sub * CPT; part_stat != nullptr && c < sub * CPT + CPT; ++c) {
    const int n = n0 + c;
    if (n >= V) break;
    se += expf((tdiv ? tile[r * (LM_BN + 1) + c] * scale / temp : tile[r * (LM_BN + 1) + c] * scale) - gmx);
  }
#pragma unroll
  for (int o = 1; o < TPR; o <<= 1) se += __shfl_xor(se, o, 64);
  __syncthreads();
  // merge the TPR sorted lists through LDS (reuse the tile area after the barrier)
  float* mv = reinterpret_cast<float*>(smem_raw);
  int* mi = reinterpret_cast<int*>(smem_raw + 256 * MAXK * 4);
#pragma unroll
  for (int q = 0; q < KMAX; ++q) { mv[threadIdx.x * MAXK + q] = tv[q]; mi[threadIdx.x * MAXK + q] = ti[q]; }
  __syncthreads();
  if (sub == 0 && m < M) {
    const long o = ((long)m * nblk + vb);
    if (part_stat != nullptr) {
      part_stat[o * 2 + 0] = gmx;
      part_stat[o * 2 + 1] = se;
    }
    int ptr[TPR];
#pragma unroll
    for (int t = 0; t < TPR; ++t) ptr[t] = 0;
    for (int q = 0; q < topk; ++q) {
      int best = -1;
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int t = 0; t < TPR; ++t) {
        if (ptr[t] >= topk) continue;
        const float v = mv[(threadIdx.x + t) * MAXK + ptr[t]];
        const int ix = mi[(threadIdx.x + t) * MAXK + ptr[t]];
        if (best < 0 || v > bv || (v == bv && ix < bi)) { best = t; bv = v; bi = ix; }
      }
      ptr[best]++;
      part_val[o * topk + q] = bv;
      part_idx[o * topk + q] = bi;
    }
  }
}

}  // namespace zs

using namespace zs;

extern "C" __attribute__((visibility("hidden"))) int zs_gemm_skinny_internal(
    int M, int N, int K, int dtype, const void* A, int lda, const void* W, int ldw,
    const float* bias, const float* residual, int ldr, void* out, int ldo, int out_dtype, int act,
    float* workspace, void* stream);

extern "C" __attribute__((visibility("hidden"))) int zs_gemm_rows_internal(
    int M, int N, int K, const void* A, int lda, const void* W, int ldw, const float* bias,
    const float* residual, int ldr, void* out, int ldo, int out_dtype, int act, void* stream);

extern "C" int zs_gemm(int M, int N, int K, int dtype, const void* A, int lda, const void* W,
                       int ldw, const float* bias, const float* residual, int ldr, void* out,
                       int ldo, int out_dtype, int act, int split_k, float* workspace,
                       void* stream) {
  ZS_REQUIRE(M >= 0 && N > 0 && K > 0, "zs_gemm: bad shape M=%d N=%d K=%d", M, N, K);
  ZS_REQUIRE(K % BK == 0, "zs_gemm: K=%d must be a multiple of 32", K);
  ZS_REQUIRE(lda % 8 == 0 && ldw % 8 == 0, "zs_gemm: lda/ldw must be multiples of 8");
  // the tiled and skinny kernels load A and W rows with 16-byte LDS-DMA / vector loads
  ZS_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0,
             "zs_gemm: A and W must be 16-byte aligned");
  ZS_REQUIRE(split_k >= 0, "zs_gemm: split_k >= 0");
  ZS_REQUIRE(dtype == ZS_F32 || dtype == ZS_BF16, "zs_gemm: dtype");
  if (M == 0) return 0;
  if (split_k == 0 && dtype == ZS_BF16 && M <= 64) {   // decode-sized: row-group kernel
    const int rc = zs_gemm_rows_internal(M, N, K, A, lda, W, ldw, bias, residual, ldr, out, ldo,
                                         out_dtype, act, stream);
    if (rc <= 0) return rc;                             // 1 = shape not covered
  }
  if (split_k == 0) {   // auto: weight-streaming skinny kernel for decode-sized M
    // M <= 64 always; up to 256 rows only where the tiled kernel has too few blocks to cover
    // a long K (mproj-like shapes); everything else goes to the tiled kernel
    const bool few_blocks = (long)cdiv(M, 64) * cdiv(N, 64) < 96 && K >= 2048;
    const bool skinny = M <= 64 || (M <= 256 && (dtype != ZS_BF16 || !g_gemm_fast || few_blocks));
    if (skinny && K % 64 == 0 && workspace != nullptr)
      return zs_gemm_skinny_internal(M, N, K, dtype, A, lda, W, ldw, bias, residual, ldr, out,
                                     ldo, out_dtype, act, workspace, stream);
    split_k = 1;
  }
  GemmArgs g{M, N, K, lda, ldw, ldr, ldo, A, W, bias, residual, out, out_dtype, act, 1, K, workspace,
             g_gemm_dbg, g_fast_xcd};
  if (split_k > 1) {
    int kps = cdiv(cdiv(K, split_k), BK) * BK;
    int s = cdiv(K, kps);
    ZS_REQUIRE(workspace != nullptr, "zs_gemm: split_k needs a workspace");
    g.split_k = s;
    g.k_per_split = kps;
  }
  hipStream_t st = S(stream);
  int rc = dtype == ZS_BF16 ? dispatch_gemm<bf16_t>(g, st) : dispatch_gemm<float>(g, st);
  if (rc) return rc;
  if (g.split_k > 1) {
    long total = (long)M * N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, g);
    ZS_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int zs_lmhead_nblk(int V) { return cdiv(V, LM_BN); }

extern "C" int zs_lmhead_topk(int M, int K, int V, int dtype, const void* A, int lda,
                              const void* W, int topk, int row_norm, float* part_stat,
                              float* part_val, int* part_idx, void* stream) {
  return zs_lmhead_topk_t(M, K, V, dtype, A, lda, W, topk, row_norm, 1.0f, part_stat, part_val,
                          part_idx, stream);
}

extern "C" int zs_lmhead_topk_t(int M, int K, int V, int dtype, const void* A, int lda,
                                const void* W, int topk, int row_norm, float temperature,
                                float* part_stat, float* part_val, int* part_idx, void* stream) {
  ZS_REQUIRE(temperature > 0.f, "zs_lmhead_topk_t: temperature %g (> 0)", temperature);
  ZS_REQUIRE(!row_norm || temperature == 1.0f, "zs_lmhead_topk_t: row_norm with temperature");
  ZS_REQUIRE(M > 0 && K > 0 && V > 0, "zs_lmhead_topk: bad shape");
  ZS_REQUIRE(K % BK == 0 && lda % 8 == 0, "zs_lmhead_topk: K %% 32, lda %% 8");
  ZS_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)W & 15) == 0,
             "zs_lmhead_topk: A and W must be 16-byte aligned");
  ZS_REQUIRE(topk >= 1 && topk <= MAXK, "zs_lmhead_topk: 1 <= topk <= 8");
  hipStream_t st = S(stream);
  const int nblk = cdiv(V, LM_BN);
  // f32 on the LDS-DMA ring when its 16-byte rows allow (lda % 4 already holds: lda % 8)
  const bool ring = dtype != ZS_BF16 && g_f32_fast && K % 4 == 0;
#define LMH(T, BM_, KM_)                                                                     \
  do {                                                                                       \
    if (sizeof(T) == 4 && ring)                                                              \
      hipLaunchKernelGGL((lmhead_kernel<T, BM_, KM_, true>), dim3(nblk * cdiv(M, BM_)), dim3(256), \
                         0, st, (g_fast_xcd ? 1 : 0) | (g_lm_prio ? 2 : 0), M, K, V, (const T*)A, \
                         lda, (const T*)W, topk, row_norm, part_stat, part_val, part_idx,       \
                         temperature);                                                       \
    else                                                                                     \
      hipLaunchKernelGGL((lmhead_kernel<T, BM_, KM_>), dim3(nblk * cdiv(M, BM_)), dim3(256), 0, \
                         st, (g_fast_xcd ? 1 : 0) | (g_lm_prio ? 2 : 0), M, K, V, (const T*)A,  \
                         lda, (const T*)W, topk, row_norm, part_stat, part_val, part_idx,       \
                         temperature);                                                       \
  } while (0)
  // top-k lists of 1 (argmax), 5 (beam <= 5: generate_beam's default) or 8 entries per block
#define LMH_K(T, BM_)                                                                          \
  do {                                                                                         \
    if (topk == 1) LMH(T, BM_, 1);                                                             \
    else if (topk <= 5) LMH(T, BM_, 5);                                                        \
    else LMH(T, BM_, 8);                                                                       \
  } while (0)
  if (M <= 64) {
    if (dtype == ZS_BF16) LMH_K(bf16_t, 64); else LMH_K(float, 64);
  } else {
    if (dtype == ZS_BF16) LMH_K(bf16_t, 128); else LMH_K(float, 128);
  }
#undef LMH_K
#undef LMH
  ZS_LAUNCH_CHECK();
  return 0;
}

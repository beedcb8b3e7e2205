// Weight-streaming GEMM for M <= 256 (GPT-2 decode step over up to 4 row blocks of 64, mapper,
// audio_proj): the weight matrix is streamed from HBM once per launch by ~256-1152 workgroups.
//
//   work unit = (32-column tile, K split, 64-row block);  block = 4 waves;
//   wave w of a workgroup owns k in [k0 + w*KS/4, k0 + (w+1)*KS/4) and computes the full 64x32
//   partial with two 32x32 MFMA tiles, loading its A and W fragments straight from global into
//   registers (all k-steps issued up front: no LDS round trip for a once-read operand,
//   cdna_hip_programming.md §5 "GEMV / M <= 16" row);
//   the 4 wave partials are summed through LDS in wave order; with splits > 1 each workgroup
//   stores its 64x32 f32 slab, and the LAST arriving workgroup of the (row block, column tile)
//   (sc1 write-through slabs + relaxed agent-scope counter, cdna_hip_programming.md §5
//   "In-launch split-K reduction") sums the slabs in split order — deterministic, no atomics on
//   data — and applies the epilogue (bias, activation, residual, dtype) exactly like zs_gemm.
//   Every row's arithmetic (K partition, summation order) depends only on (N, K), never on M or
//   on the row block, so a clip's results do not depend on how many clips share the launch.
//   The row blocks of one (tile, split) are consecutive work units and the linear block id is
//   remapped bijectively so that consecutive units run on the same XCD (each XCD has its own
//   L2): the W slice they share is fetched from HBM once per XCD.
#include <cstring>
#include "common.h"

namespace zs {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8s_t;
typedef __attribute__((ext_vector_type(16))) float f32x16s_t;

constexpr int SK_BN = 32;
constexpr int SK_TILE = 64 * SK_BN;     // floats per slab
// workspace = [SK_MAX_TILES int counters (fixed, so no GEMM shape ever places slabs over another
// shape's counters)][slabs]
constexpr int SK_MAX_TILES = 4096;
constexpr int SK_MAX_M = 256;           // up to 4 row blocks of 64

struct SkinnyArgs {
  int M, N, K, lda, ldw, ldr, ldo, splits, ks;   // ks = K per workgroup
  int rblocks, ntiles;                            // 64-row blocks, 32-column tiles
  const void* A;
  const void* W;
  const float* bias;
  const float* residual;
  void* out;
  int out_dtype, act;
  int* counters;      // [rblocks][ntiles], zero on first use, reset by the reducer
  float* slabs;       // [rblocks][splits][ntiles][64*32]
};

// per-wave partial over kw..kw+len (len % 16 == 0), bf16
__device__ __forceinline__ void wave_partial(const bf16_t* A, int lda, int M, const bf16_t* W,
                                             int ldw, int N, int n0, int kw, int len,
                                             f32x16s_t& c0, f32x16s_t& c1) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int n = n0 + r;
  const bool nv = n < N, m0v = r < M, m1v = r + 32 < M;
  constexpr int MAXS = 8;   // up to 128-deep per wave
  bf16x8s_t a0[MAXS], a1[MAXS], b[MAXS];
  const int steps = len / 16;
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    if (s < steps) {
      const int k = kw + s * 16 + 8 * h;
      b[s] = nv ? *reinterpret_cast<const bf16x8s_t*>(W + (long)n * ldw + k) : bf16x8s_t{};
      a0[s] = m0v ? *reinterpret_cast<const bf16x8s_t*>(A + (long)r * lda + k) : bf16x8s_t{};
      a1[s] = m1v ? *reinterpret_cast<const bf16x8s_t*>(A + (long)(r + 32) * lda + k) : bf16x8s_t{};
    }
  }
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    if (s < steps) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0[s], b[s], c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1[s], b[s], c1, 0, 0, 0);
    }
  }
}

// f32 parity mode: 32x32x2f32, lane half h owns k in [8h, 8h+8) of each 16-deep step
__device__ __forceinline__ void wave_partial(const float* A, int lda, int M, const float* W,
                                             int ldw, int N, int n0, int kw, int len,
                                             f32x16s_t& c0, f32x16s_t& c1) {
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int n = n0 + r;
  const bool nv = n < N, m0v = r < M, m1v = r + 32 < M;
  const int steps = len / 16;
  for (int s0 = 0; s0 < steps; s0 += 4) {
    float4 a0[8], a1[8], b[8];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bool ok = s0 + s < steps;
      const int k = kw + (s0 + s) * 16 + 8 * h;
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        b[2 * s + q] = (ok && nv) ? *reinterpret_cast<const float4*>(W + (long)n * ldw + k + 4 * q) : z;
        a0[2 * s + q] = (ok && m0v) ? *reinterpret_cast<const float4*>(A + (long)r * lda + k + 4 * q) : z;
        a1[2 * s + q] = (ok && m1v) ? *reinterpret_cast<const float4*>(A + (long)(r + 32) * lda + k + 4 * q) : z;
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s0 + s >= steps) break;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float4& va0 = a0[2 * s + e / 4];
        const float4& va1 = a1[2 * s + e / 4];
        const float4& vb = b[2 * s + e / 4];
        const int j = e & 3;
        const float x0 = j == 0 ? va0.x : j == 1 ? va0.y : j == 2 ? va0.z : va0.w;
        const float x1 = j == 0 ? va1.x : j == 1 ? va1.y : j == 2 ? va1.z : va1.w;
        const float y = j == 0 ? vb.x : j == 1 ? vb.y : j == 2 ? vb.z : vb.w;
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, y, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, y, c1, 0, 0, 0);
      }
    }
  }
}

__device__ __forceinline__ void skinny_store(const SkinnyArgs& g, int m, int n, float v) {
  if (g.bias) v += g.bias[n];
  v = act_apply(v, g.act);
  if (g.residual) v += g.residual[(long)m * g.ldr + n];
  if (g.out_dtype == ZS_BF16) reinterpret_cast<bf16_t*>(g.out)[(long)m * g.ldo + n] = f2bf(v);
  else reinterpret_cast<float*>(g.out)[(long)m * g.ldo + n] = v;
}

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

// MODE 0: plain slab stores + agent release fence before the ticket, acquire fence in the reducer
// MODE 1: write-through (sc1) slab stores, no release fence, reducer reads the slabs with sc1
//         loads (cdna_hip_programming.md §5 item 2, "Equally valid and ~0.3-1.0 us cheaper")
template <typename T, int MODE>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(SkinnyArgs g) {
  __shared__ __attribute__((aligned(16))) float red[4 * SK_TILE + 4];   // wave partials + flag
  // XCD-aware bijective remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
  // blocks id, id+8, id+16, ... share an XCD; give them consecutive work units
  const int nwg = gridDim.x, id = blockIdx.x, xcd = id & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
  const int rb = u % g.rblocks, rest = u / g.rblocks;
  const int z = rest % g.splits, tile = rest / g.splits;
  const int n0 = tile * SK_BN;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kq = g.ks / 4;
  const int kw = z * g.ks + wid * kq;
  const int Mr = min(64, g.M - rb * 64);           // rows of this block
  f32x16s_t c0, c1;
#pragma unroll
  for (int e = 0; e < 16; ++e) { c0[e] = 0.f; c1[e] = 0.f; }
  wave_partial((const T*)g.A + (long)rb * 64 * g.lda, g.lda, Mr, (const T*)g.W, g.ldw, g.N, n0,
               kw, kq, c0, c1);
  // wave partial -> LDS [wave][row][col]
  float* mine = red + wid * SK_TILE;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
    const int col = lane & 31;
    mine[row * SK_BN + col] = c0[e];
    mine[(row + 32) * SK_BN + col] = c1[e];
  }
  __syncthreads();
  // each thread owns 8 consecutive tile elements e0..e0+7 (row e0/32, cols e0%32..+7)
  constexpr int PER = SK_TILE / 256;
  const int e0 = threadIdx.x * PER;
  float part[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = e0 + i;
    part[i] = red[e] + red[SK_TILE + e] + red[2 * SK_TILE + e] + red[3 * SK_TILE + e];
  }
  const int m = e0 / SK_BN, nb = n0 + e0 % SK_BN;
  if (g.splits == 1) {
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (m < Mr && nb + i < g.N) skinny_store(g, rb * 64 + m, nb + i, part[i]);
    return;
  }
  const int ntiles = g.ntiles;
  float* slabs = g.slabs + (long)rb * g.splits * ntiles * SK_TILE;
  int* counter = g.counters + rb * ntiles + tile;
  const long slab_off = ((long)z * ntiles + tile) * SK_TILE + e0;
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      slabs, (short)0, g.splits * ntiles * SK_TILE * 4, 0x00020000);
  if (MODE == 1) {
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
      u32x4_t v = {__float_as_uint(part[4 * q]), __float_as_uint(part[4 * q + 1]),
                   __float_as_uint(part[4 * q + 2]), __float_as_uint(part[4 * q + 3])};
      __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, (int)((slab_off + 4 * q) * 4), 0, 16);
    }
  } else {
#pragma unroll
    for (int q = 0; q < PER / 4; ++q)
      *reinterpret_cast<float4*>(slabs + slab_off + 4 * q) =
          make_float4(part[4 * q], part[4 * q + 1], part[4 * q + 2], part[4 * q + 3]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(red + 4 * SK_TILE);
  if (threadIdx.x == 0) {
    if (MODE == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int old = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == g.splits - 1;
    if (last) {
      __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (MODE == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  float v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) v[i] = 0.f;
  for (int s = 0; s < g.splits; ++s) {
    const long off = ((long)s * ntiles + tile) * SK_TILE + e0;
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
      float4 f;
      if (MODE == 1) {
        const u32x4_t u = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)((off + 4 * q) * 4), 0, 16);
        f = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z),
                        __uint_as_float(u.w));
      } else {
        f = *reinterpret_cast<const float4*>(slabs + off + 4 * q);
      }
      v[4 * q] += f.x; v[4 * q + 1] += f.y; v[4 * q + 2] += f.z; v[4 * q + 3] += f.w;
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (m < Mr && nb + i < g.N) skinny_store(g, rb * 64 + m, nb + i, v[i]);
}

static int g_skinny_mode = 1;
extern int g_gemm_fast;     // gemm.hip
extern int g_f32_fast;      // gemm.hip
extern int g_decode_attn5;  // attn.hip
extern int g_window_mfma;   // attn.hip
extern int g_fast_ns;       // gemm.hip
extern int g_fast_tile;     // gemm.hip
extern int g_gemm_dbg;      // gemm.hip
extern int g_fast_persist;  // gemm.hip
extern int g_fast_xcd;      // gemm.hip
extern int g_swin_dbg;      // swin.hip
extern int g_swin_occ3;     // swin.hip
extern int g_gemm_lean;     // gemm.hip
extern int g_row_mfma;      // attn.hip
extern int g_logmel_wave;   // frontend.hip
extern int g_lean96;        // gemm.hip
extern int g_lean8w;        // gemm.hip
extern int g_lean_min128;    // gemm.hip
extern int g_lean128_ns;     // gemm.hip
extern int g_lm_prio;       // gemm.hip
extern int g_gemm_rows;     // gemm_rows.hip
extern int g_rows_nt48;     // gemm_rows.hip
extern int g_fp8_tile;      // mistral.hip
extern int g_rows_wide;     // gemm_rows.hip
extern int g_fp8_dbg;       // mistral.hip
extern int g_attn_split;    // attn.hip
extern int g_small_attn;    // attn.hip
extern int g_small_rmax;    // attn.hip
extern int g_gemm_big;      // gemm.hip
extern int g_big_min;       // gemm.hip
extern int g_dp_spin;       // decode_grid.hip
extern int g_dp_abort;      // decode_grid.hip
extern int g_dg_exp;
extern int g_dg_dynf;       // decode_grid.hip
extern int g_beam_xcd;      // attn.hip
extern int g_f32_tile;      // gemm.hip

// choose K per workgroup: a multiple of 64 dividing K, each wave <= 128 deep, ~256-320 WGs
static int skinny_splits(int N, int K) {
  const int ntiles = cdiv(N, SK_BN);
  int best = -1;
  for (int s = 1; s <= K / 64; ++s) {
    if (K % s) continue;
    const int ks = K / s;
    if (ks % 64 || ks > 512) continue;
    if (best < 0) best = s;
    if (ntiles * s >= 256) { best = s; break; }
    best = s;
  }
  return best;
}

}  // namespace zs

using namespace zs;

extern "C" int zs_tune_set(const char* key, int value) {
  if (!key) return ZS_ERR_ARG;
  if (!strcmp(key, "skinny_mode")) { g_skinny_mode = value; return 0; }
  if (!strcmp(key, "gemm_fast")) { g_gemm_fast = value; return 0; }
  if (!strcmp(key, "f32_fast")) { g_f32_fast = value; return 0; }
  if (!strcmp(key, "decode_attn5")) { g_decode_attn5 = value; return 0; }
  if (!strcmp(key, "window_mfma")) { g_window_mfma = value; return 0; }
  if (!strcmp(key, "fast_ns")) { g_fast_ns = value; return 0; }
  if (!strcmp(key, "fast_tile")) { g_fast_tile = value; return 0; }
  if (!strcmp(key, "gemm_dbg")) { g_gemm_dbg = value; return 0; }
  if (!strcmp(key, "fast_persist")) { g_fast_persist = value; return 0; }
  if (!strcmp(key, "fast_xcd")) { g_fast_xcd = value; return 0; }
  if (!strcmp(key, "swin_dbg")) { g_swin_dbg = value; return 0; }
  if (!strcmp(key, "swin_occ3")) { g_swin_occ3 = value; return 0; }
  if (!strcmp(key, "gemm_lean")) { g_gemm_lean = value; return 0; }
  if (!strcmp(key, "row_mfma")) { g_row_mfma = value; return 0; }
  if (!strcmp(key, "logmel_wave")) { g_logmel_wave = value; return 0; }
  if (!strcmp(key, "lean96")) { g_lean96 = value; return 0; }
  if (!strcmp(key, "lean8w")) { g_lean8w = value; return 0; }
  if (!strcmp(key, "lean_min128")) { g_lean_min128 = value; return 0; }
  if (!strcmp(key, "lean128_ns")) { g_lean128_ns = value; return 0; }
  if (!strcmp(key, "lm_prio")) { g_lm_prio = value; return 0; }
  if (!strcmp(key, "gemm_rows")) { g_gemm_rows = value; return 0; }
  if (!strcmp(key, "rows_nt48")) { g_rows_nt48 = value; return 0; }
  if (!strcmp(key, "fp8_tile")) { g_fp8_tile = value; return 0; }
  if (!strcmp(key, "rows_wide")) { g_rows_wide = value; return 0; }
  if (!strcmp(key, "fp8_dbg")) { g_fp8_dbg = value; return 0; }
  if (!strcmp(key, "attn_split")) { g_attn_split = value; return 0; }
  if (!strcmp(key, "small_attn")) { g_small_attn = value; return 0; }
  if (!strcmp(key, "small_rmax")) { g_small_rmax = value; return 0; }
  if (!strcmp(key, "gemm_big")) { g_gemm_big = value; return 0; }
  if (!strcmp(key, "big_min")) { g_big_min = value; return 0; }
  if (!strcmp(key, "dp_spin")) { g_dp_spin = value; return 0; }
  if (!strcmp(key, "dp_abort_step")) { g_dp_abort = value; return 0; }
  if (!strcmp(key, "dg_exp")) { g_dg_exp = value; return 0; }
  if (!strcmp(key, "dg_dynf")) { g_dg_dynf = value; return 0; }
  if (!strcmp(key, "beam_xcd")) { g_beam_xcd = value; return 0; }
  if (!strcmp(key, "f32_tile")) { g_f32_tile = value; return 0; }
  return fail(ZS_ERR_ARG, "zs_tune_set: unknown key %s", key);
}

extern "C" int zs_gemm_workspace_floats(int M, int N, int K) {
  if (M <= 0 || M > SK_MAX_M) return 0;
  const int s = skinny_splits(N, K);
  if (s < 0) return 0;
  const int ntiles = cdiv(N, SK_BN), rb = cdiv(M, 64);
  if (ntiles * rb > SK_MAX_TILES) return 0;
  return SK_MAX_TILES + rb * s * ntiles * SK_TILE;
}

// internal entry used by zs_gemm for M <= 64 with split_k == 0 (auto)
extern "C" __attribute__((visibility("hidden"))) int zs_gemm_skinny_internal(int M, int N, int K, int dtype, const void* A, int lda,
                                       const void* W, int ldw, const float* bias,
                                       const float* residual, int ldr, void* out, int ldo,
                                       int out_dtype, int act, float* workspace, void* stream) {
  ZS_REQUIRE(M > 0 && M <= SK_MAX_M, "skinny gemm: M <= %d", SK_MAX_M);
  const int s = skinny_splits(N, K);
  ZS_REQUIRE(s > 0, "skinny gemm: K=%d must be a multiple of 64", K);
  const int ntiles = cdiv(N, SK_BN), rb = cdiv(M, 64);
  ZS_REQUIRE(s == 1 || workspace != nullptr, "skinny gemm: needs the zeroed workspace");
  ZS_REQUIRE(ntiles * rb <= SK_MAX_TILES, "skinny gemm: N too large");
  SkinnyArgs g{M, N, K, lda, ldw, ldr, ldo, s, K / s, rb, ntiles, A, W, bias, residual, out,
               out_dtype, act, reinterpret_cast<int*>(workspace), workspace + SK_MAX_TILES};
  dim3 grid(ntiles * s * rb);
#define SKL(T, MODE_) hipLaunchKernelGGL((gemm_skinny_kernel<T, MODE_>), grid, dim3(256), 0, S(stream), g)
  if (dtype == ZS_BF16) {
    if (g_skinny_mode == 1) SKL(bf16_t, 1); else SKL(bf16_t, 0);
  } else {
    if (g_skinny_mode == 1) SKL(float, 1); else SKL(float, 0);
  }
#undef SKL
  ZS_LAUNCH_CHECK();
  return 0;
}

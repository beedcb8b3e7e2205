// GPT-2 greedy decode of ONE eval batch (R <= 64 rows, the reference's bs = 64): every step of
// generate2 after step 0 (gpt2_prefix_eval.py:161-222 over transformers' GPT2LMHeadModel with a
// KV cache) -- 12 blocks, ln_f, the tied LM head with its argmax and the stop / length
// bookkeeping -- on a grid of G 4-wave workgroups, either
//   * persistent: ONE launch runs every remaining step, phases separated by grid barriers
//     (zs_gpt2_decode_persist), or
//   * phase launches: each phase of each step is its own launch (zs_gpt2_decode_phases; the
//     per-step path: no co-residency needed, graph-capturable, the give-up fallback),
// and both run the SAME device code for every phase.
//
// Canonical arithmetic (why the grid size never changes a caption).  Every output element of
// every phase is computed by one fixed sequence of operations whatever G is and whichever mode
// runs it:
//   * a GEMM element out[r][n] = sum_k a[r][k] W[n][k] is four partial sums, one per K quarter
//     (wave w of the workgroup owning the element takes k in [K w / 4, K (w+1) / 4)), each an MFMA
//     16x16x32 chain over its k-steps in increasing order from 0, added as (p0 + p1) + (p2 + p3);
//     then + bias (and the activation / + residual).  The grid only decides WHICH workgroup owns
//     an element (tiles of 16 x 16 are independent in the MFMA);
//   * a LayerNorm row (ln_1 / ln_2 / ln_f) reads bf16(x), sums x and x^2 over each wave's quarter
//     in a fixed in-lane order (v_dot2 over the bf16 pairs), across the 4 lanes of a row by
//     swap-adds, across the waves as (w0 + w1) + (w2 + w3): ONE pass, var = E[x^2] - mean^2,
//     rstd = rsqrt(var + 1e-5) (the f32 parity kernel below is two-pass; the one-pass error on a
//     row with a large mean is bounded in tests/test_ln_onepass.py);
//   * an attention unit (row, head) runs the online softmax over its cached keys in 32-key chunks
//     (8 lane groups x 4 keys), then folds in the new key;
//   * the argmax over the vocabulary is exact (ties -> lower id, as torch.argmax).
// So ids and decode state are identical for G = 48 / 96 / 192 and for the phase launches
// (tests/test_gpu_persist.py asserts it).
//
// Why 4-wave workgroups (half a CU: 256 threads, <= 256 registers per lane, ~41 KB of LDS): a
// persistent grid spends much of each step waiting on hand-offs; at 8 waves x 256 registers a
// grid workgroup held its whole CU, so the other batches' encode / prefill kernels could not use
// it while it waited (DESIGN.md §18 co-residency probe: a begin +50 % beside full-CU grids, +12 %
// beside half-CU ones).  Each wave keeps its K quarter of the activation in registers (B operand
// of a TRANSPOSED product: lane = (row r % 16, 4 consecutive output columns), so a lane's four
// accumulators are 4 consecutive columns of one row: 8 / 16-byte epilogue stores), and the LDS
// holds only the partial-sum slabs of the cross-wave reduction.
//
// Hand-offs (MI355X_MICROARCH.md § Workgroup dispatch, Valid forms row 1: sc1 stores, every
// storing wave's vmcnt(0), a workgroup barrier, one lane's agent-scope add to a counter -- here 8
// sharded counters -- and sc1 polls / loads):
//   A  ln_1 + c_attn -> q [64][768] bf16; k / v straight into the KV cache at each row's pos
//   B  attention (row, head) units -> att [4][24][64][8] bf16 (MFMA fragment order)
//   C  attn.c_proj + residual -> x (f32, held in the owning thread's registers across the whole
//      step; phase launches keep it in the workspace) and its bf16 copy xb (fragment order)
//   D  ln_2 + c_fc + gelu_new -> hid [4][96][64][8] bf16
//   E  mlp.c_proj + residual -> x, xb
//   F  ln_f + LM head over vocab blocks b = w, w + G, ..: per-row best (logit, id) -> a 64-bit
//      agent-scope atomic max of (order-preserving logit bits, ~id).  ln_f's affine is folded into
//      the LM head: logit[v] = y . (g o wte[v]) + (beta . wte[v]) with y the normalised row (the
//      table packed as bf16(g o wte), the per-token bias in f32), as ln_1 / ln_2 into c_attn / c_fc
//   G  every workgroup applies generate2's bookkeeping to its LDS copy of the row state;
//      workgroup 0 commits ids and state to memory after every step (a give-up resumes there)
// 5 barriers per block + 1 after F = 61 per step.
#include <type_traits>

#include "common.h"

// No implicit FP contraction in this file: whether the compiler fuses a multiply into a
// following add depends on the surrounding code, which differs between the grid sizes' template
// instances -- every fused multiply-add below is an explicit fmaf, so each instance rounds alike.
#pragma clang fp contract(off)

namespace zs {
int g_dp_spin = 0;   // zs_tune_set("dp_spin", n): give up a grid-barrier wait after n polls (0 =
                     // the default 2^22, < 0: at the first unmet poll); tests force the give-up
int g_dg_exp = 0;    // zs_tune_set("dg_exp", m): traffic experiments (grid_bench only; ids garbage)
int g_dg_dynf = 1;   // zs_tune_set("dg_dynf", 0): phase F all static in persistent launches too (A/B)
int g_dp_abort = -1; // zs_tune_set("dp_abort_step", k): every workgroup gives up at the start of
                     // decode step k (a mid-launch give-up for the resume test); -1 = never
namespace dg {

constexpr int D = 768, NH = 12, HD = 64, DFF = 3072, NLY = 12, RM = 64, QKVN = 3 * D;
constexpr int NW = 4, NT = 64 * NW;
constexpr int KSD = D / 32, KSF = DFF / 32;          // k-steps of K = 768 / 3072
constexpr int QS = KSD / NW, QF = KSF / NW;          // k-steps of one wave's K quarter: 6 / 24
constexpr int NCB_Q = QKVN / 16, NCB_D = D / 16, NCB_F = DFF / 16;   // 16-column blocks
constexpr unsigned SPIN_MAX = 1u << 22;
#ifndef DG_NSH
#define DG_NSH 8
#endif
constexpr int NSH = DG_NSH;                          // barrier counter shards, one 128-B line each
static_assert(NSH <= 16 && 48 % NSH == 0 && (NSH & (NSH - 1)) == 0,
              "shards: a power of two (bar_arrive takes w & (NSH - 1)) <= 16, dividing every grid");
constexpr int ECH = 4;                               // phase E: k-steps per streamed chunk

// Tiles per workgroup of each GEMM phase: CB column blocks x RB row blocks of 16 (workgroup w
// takes column group w % (blocks / CB) and row group w / (blocks / CB)); PF = column blocks of
// weights prefetched across the barrier (all of them, or one round's).  The grid size changes
// only these ownerships, never the arithmetic of an element.
template <int G> struct Geo;
// ESL: phase E's chunks in flight (tools/grid_bench.py, profiles/r5/esl_ab.txt: 3 / 3 / 4 vs 2 / 2 / 2
// alone 428 / 304 / 252 vs 436 / 313 / 271 us per step, 10 x G48 equal, 5 x G96 +2 %; 4 at G48:
// 484 us alone)
#ifndef DG_ESL48
#define DG_ESL48 3
#endif
#ifndef DG_ESL96
#define DG_ESL96 3
#endif
#ifndef DG_ESL192
#define DG_ESL192 4
#endif
// G = 48: c_attn / c_fc column blocks prefetched across the barrier (the rest: after round 1;
// profiles/r5/pf_ab.txt: all of them, 3 / 4, vs 2 / 2: within noise, ~+1 %)
#ifndef DG_APF48
#define DG_APF48 3
#endif
#ifndef DG_DPF48
#define DG_DPF48 4
#endif
// barrier poll interval (s_sleep units of 64 clocks; profiles/r5/sleep_ab.txt: 3 vs 1, alone -3 %,
// 5 x G48 +1 %)
#ifndef DG_SLEEP
#define DG_SLEEP 3
#endif
// FSL: phase F's vocab blocks in flight
// (profiles/r5/fsl_ab.txt: 4 vs 3 slots, alone -1.5 to -2 %; 6 spills)
#ifndef DG_FSL
#define DG_FSL 4
#endif
template <> struct Geo<48> {
  static constexpr int ACB = 3, ARB = 4, APF = DG_APF48, DCB = 4, DRB = 4, DPF = DG_DPF48, ECB = 2, ERB = 2, ESL = DG_ESL48,
                       FSL = DG_FSL;
};
template <> struct Geo<96> {
  static constexpr int ACB = 3, ARB = 2, APF = 3, DCB = 4, DRB = 2, DPF = 4, ECB = 2, ERB = 1, ESL = DG_ESL96,
                       FSL = DG_FSL;
};
template <> struct Geo<192> {
  static constexpr int ACB = 3, ARB = 1, APF = 3, DCB = 2, DRB = 2, DPF = 2, ECB = 1, ERB = 1, ESL = DG_ESL192,
                       FSL = DG_FSL;
};
template <int G> struct Units {
  static constexpr int UPG = RM * NH / G;   // attention units per workgroup
  static constexpr int KU = UPG / NW;       // per wave
  static constexpr int KC = KU >= 2 ? 4 : 8;   // keys per lane group per loaded chunk (KU KC 8
                                               // registers; a multiple of 4, phase_b)
};

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(3))) int lds_int_t;

// ------------------------------------------------------------------ workspace
constexpr int WS_SH = 0;                          // NSH counters, 128 B apart
constexpr int WS_TMO = NSH * 128;                 // timeout word
constexpr int WS_KEY = WS_TMO + 128;              // u64 [2][64] LM-head argmax keys (step parity)
constexpr int WS_CLM = WS_KEY + 2 * RM * 8;       // tile-claim counters, 128 B apart (persistent)
constexpr int CLM_F = 0;                          // phase F: [step & 1]
constexpr int WS_SYNC_BYTES = 4096;               // zeroed by the launcher
constexpr int WS_Q = WS_SYNC_BYTES;               // bf16 [64][768]
constexpr int WS_ATT = WS_Q + RM * D * 2;         // bf16 [4][24][64][8] (fragment order)
constexpr int WS_XB = WS_ATT + RM * D * 2;        // bf16 [4][24][64][8]
constexpr int WS_HID = WS_XB + RM * D * 2;        // bf16 [4][96][64][8]
constexpr int WS_X = WS_HID + RM * DFF * 2;       // f32  [64][768] (phase launches only)
constexpr int WS_BYTES = WS_X + RM * D * 4;

// ------------------------------------------------------------------ LDS (36,160 B)
constexpr int SM_RED = 0;                         // f32x4 [2048]: partial slabs (32 KiB)
constexpr int SM_LN = SM_RED + 32768;             // f32 [2][4][64]: LayerNorm partials
constexpr int SM_CB = SM_LN + 2048;               // f32 [2][64]: the tile's bias / column sums
constexpr int SM_ST = SM_CB + 512;                // int tok[64], pos[64], done[64], misc[16]
constexpr int SM_TOTAL = SM_ST + (3 * RM + 16) * 4;
constexpr int EXCL_LDS = 80 * 1024 + 512;        // an exclusive launch's LDS per workgroup (> 1/2 CU)

struct Args {
  int R, Lmax, max_steps, stop0, stop1, V, layer, abort_step, exp, dynf;
  unsigned spin_max;
  int kv_bytes;         // bytes of one layer's K (or V) cache
  float temp;
  const bf16_t* wte; const bf16_t* wpe;
  // weights in MFMA fragment order (ops.pack_b_fragments): [N/16][K/32][64][8] bf16
  const bf16_t* wq[NLY]; const float* bq[NLY];     // c_attn (ln_1 affine folded in), bias
  const bf16_t* wo[NLY]; const float* bo[NLY];     // attn.c_proj
  const bf16_t* wf[NLY]; const float* bfc[NLY];    // c_fc (ln_2 affine folded in)
  const bf16_t* wm[NLY]; const float* bm[NLY];     // mlp.c_proj
  const bf16_t* wtep;     // tied LM head with ln_f's weight folded in, fragment order
  const float* lmb;       // beta . wte[v] (ln_f's bias through the LM head), [ceil(V/16) 16]
  bf16_t* kc[NLY]; bf16_t* vc[NLY];
  int* pos; int* next_tok; int* done; int* out_ids; int* out_len; int* step_ctr; int* all_done;
  char* ws;
};

// ------------------------------------------------------------------ memory helpers
struct Rs {
  __amdgpu_buffer_rsrc_t q, att, xb, hid;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk(void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ Rs make_rs(char* ws, int exp) {
  Rs r;
  const int z = (exp & 1) ? 0 : 1;
  r.q = mk(ws + WS_Q, z * RM * D * 2);
  r.att = mk(ws + WS_ATT, z * RM * D * 2);
  r.xb = mk(ws + WS_XB, z * RM * D * 2);
  r.hid = mk(ws + WS_HID, z * RM * DFF * 2);
  return r;
}
// aux 16 = sc1: stores write through, loads bypass this CU's L1 (the hand-off forms)
__device__ __forceinline__ u32x4_t ld16(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, int off, u32x4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
__device__ __forceinline__ void st8(__amdgpu_buffer_rsrc_t r, int off, u32x2_t v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, 16);
}
__device__ __forceinline__ bf16x8_t bf8(u32x4_t u) { return __builtin_bit_cast(bf16x8_t, u); }
// transposed product: A = weight fragment (lane: output column n0 + l % 16), B = activation
// fragment (lane: row l % 16); lane l then holds out[row l % 16][n0 + 4 (l / 16) + i], i < 4
__device__ __forceinline__ f32x4_t mfma(u32x4_t w, u32x4_t a, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf8(w), bf8(a), c, 0, 0, 0);
}
// threadIdx.x through an empty asm: lane arithmetic is recomputed per phase instead of being
// hoisted out of the step loop (and spilled)
__device__ __forceinline__ int otid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float sum8(float s) {     // over the 8 lanes of each 8-lane group
  s += dppf<0xB1>(s);
  s += dppf<0x4E>(s);
  return s + dppf<0x141>(s);
}
__device__ __forceinline__ float xor8(float v) { return dppf<0x128>(v); }   // row_ror:8
// v + the partner lane's v (lane ^ 16 / lane ^ 32), the same value on both lanes
__device__ __forceinline__ float add16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float add32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float max16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// workgroup barrier for LDS hand-offs; waits for nothing in flight in vector memory
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void unpack8(const u32x4_t& u, float (&f)[8]) {
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
  f[4] = __uint_as_float(u.z << 16); f[5] = __uint_as_float(u.z & 0xffff0000u);
  f[6] = __uint_as_float(u.w << 16); f[7] = __uint_as_float(u.w & 0xffff0000u);
}
__device__ __forceinline__ u32x4_t pack8(const float (&f)[8]) {
  return u32x4_t{pk2bf(f[0], f[1]), pk2bf(f[2], f[3]), pk2bf(f[4], f[5]), pk2bf(f[6], f[7])};
}
template <int I, int N, typename F>
__device__ __forceinline__ void static_for_i(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_i<I + 1, N>(f);
  }
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) { static_for_i<0, N>(f); }

// weight fragments (packed [nblk][KS][64][8]) of col blocks cb0 .. cb0 + NB, k-steps s0 .. s0 + S
template <int NB, int S>
__device__ __forceinline__ void ldw(const bf16_t* Wp, int KS, int cb0, int s0, u32x4_t* w) {
  const int lane = otid() & 63;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int s = 0; s < S; ++s)
      w[nb * S + s] =
          *reinterpret_cast<const u32x4_t*>(Wp + ((long)((cb0 + nb) * KS + s0 + s) * 64 + lane) * 8);
}
// handed-off activation fragments ([4][KS][64][8] bf16, sc1): row blocks rb0 .., k-steps s0 ..
template <int NRB, int S>
__device__ __forceinline__ void lda(__amdgpu_buffer_rsrc_t r, int KS, int rb0, int s0, u32x4_t* a) {
  const int lane = otid() & 63;
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
    for (int s = 0; s < S; ++s) a[rb * S + s] = ld16(r, (((rb0 + rb) * KS + s0 + s) * 64 + lane) * 16);
}
// byte offset of element (row, col) (col % 4 == 0) in a fragment-order activation of KS k-steps
__device__ __forceinline__ int frag_off(int row, int col, int KS) {
  return ((((row >> 4) * KS + (col >> 5)) * 64 + (row & 15) + 16 * ((col >> 3) & 3)) * 8 + (col & 7)) * 2;
}

// ------------------------------------------------------------------ diagnostic stamps
// zs_decode_persist_set_stamps(buf, step): thread 0 of every workgroup writes s_memrealtime
// (100 MHz) after each barrier arrive (slot 2i) and wait (2i + 1) of decode step `step`, and at
// its start (127) / end (126), into buf[w][128] (tools/persist_stamps.py).  NULL = off.
// step -2: every persistent workgroup w writes (XCC_ID << 32 | HW_ID) to its launch's workspace at
// WS_X + 8 w instead (tools/placement.py: which CU each workgroup of concurrent grids landed on).
__device__ unsigned long long* dp_stamp_buf;
__device__ int dp_stamp_step;
__device__ const char* dp_stamp_ws;   // only the launch on this workspace (NULL: every launch)
#define DP_NB 64
__device__ __forceinline__ void stamp(unsigned long long* sb, int slot) {
  if (sb != nullptr && threadIdx.x == 0) {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    ((gu64*)sb)[slot] = t;
  }
}

// ------------------------------------------------------------------ grid barrier
// Producer (R1): every storing wave drains its sc1 stores, the workgroup meets, ONE lane adds to
// its shard (w % 8) of the counter.  Consumer: lanes 0..7 of wave 0 poll the 8 shards (relaxed
// sc1 loads), the workgroup meets, then every load of handed-off bytes is an sc1 load.  arrive()
// and wait() are split so a workgroup issues its next phase's weight loads in between.
struct Bar {
  gu32* sh;
  gu32* tmo;
  unsigned n;               // barriers passed
  unsigned per;             // workgroups per shard
  unsigned spin_max;
  unsigned long long* sb;   // this workgroup's stamp row of the traced step (or NULL)
  unsigned n0;
};
__device__ __forceinline__ void bar_arrive(Bar& b, int w) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(b.sh + (w & (NSH - 1)) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  stamp(b.sb, 2 * (b.n - b.n0));
  ++b.n;
}
// (round 6 A/B, tools/grid_bench.py + tools/persist_stamps.py: keeping 3 shard reads in flight --
// a hand-written pipelined poll -- cut no barrier wait under load and took 12 % of ten G48 grids'
// aggregate rate (10.2k vs 11.6k steps/s; loaded step 747 vs 682 us): the extra reads slow the
// co-resident workgroups more than the earlier detection gains.  The poll stays serial.)
__device__ __forceinline__ bool bar_wait(Bar& b, volatile lds_int_t* s_ok) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned target = b.n * b.per;
    unsigned spins = 0;
    int ok = 1;
    for (;;) {
      const unsigned c = lane < NSH
          ? __hip_atomic_load(b.sh + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : target;
      if (__ballot(c < target) == 0) break;
      ++spins;
      // bounded: give up (and tell every other workgroup) after spin_max polls, so a grid that
      // is not co-resident drains instead of hanging
      if (spins > b.spin_max ||
          ((spins & 255) == 0 && __hip_atomic_load(b.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        if (lane == 0) __hip_atomic_store(b.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(DG_SLEEP);
    }
    if (lane == 0) *s_ok = ok;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  stamp(b.sb, 2 * (b.n - b.n0) - 1);
  return *s_ok != 0;
}

// ------------------------------------------------------------------ LDS views
struct Sm {
  f32x4_t* red;
  float* ln;
  float* cb;     // [2][64]: bias, then column sums, of the A / D tile's columns
  int* tok;
  int* pos;
  int* done;
  int* misc;     // [0] rows still decoding, [8] barrier ok flag
  __device__ __forceinline__ explicit Sm(char* s)
      : red(reinterpret_cast<f32x4_t*>(s + SM_RED)), ln(reinterpret_cast<float*>(s + SM_LN)),
        cb(reinterpret_cast<float*>(s + SM_CB)),
        tok(reinterpret_cast<int*>(s + SM_ST)),
        pos(reinterpret_cast<int*>(s + SM_ST) + RM), done(reinterpret_cast<int*>(s + SM_ST) + 2 * RM),
        misc(reinterpret_cast<int*>(s + SM_ST) + 3 * RM) {}
};

// ------------------------------------------------------------------ cross-wave reduction
// The 4 waves' partial tiles (acc[t], t < T: this wave's K quarter) summed as (w0 + w1) + (w2 +
// w3) through LDS; wave v finalises tiles t = 4 j + v: epi(j, t, sum) with the lane's 4 columns
// (j is a compile-time index after unrolling: per-tile operands live in arrays indexed by j).
template <int T, typename Epi>
__device__ __forceinline__ void reduce_tiles(f32x4_t* red, const f32x4_t (&acc)[T], Epi&& epi) {
  static_assert(T * NW * 64 <= 2048, "partial slabs fit the LDS region");
  const int tid = otid(), v = tid >> 6, lane = tid & 63;
  lds_sync();                 // the previous round's readers are done with the slabs
#pragma unroll
  for (int t = 0; t < T; ++t) red[(v * T + t) * 64 + lane] = acc[t];
  lds_sync();
#pragma unroll
  for (int j = 0; j * NW < T; ++j) {
    const int t = NW * j + v;
    if (t < T) {
      const f32x4_t p0 = red[t * 64 + lane], p1 = red[(T + t) * 64 + lane];
      const f32x4_t p2 = red[(2 * T + t) * 64 + lane], p3 = red[(3 * T + t) * 64 + lane];
      epi(j, t, (p0 + p1) + (p2 + p3));
    }
  }
}

// ------------------------------------------------------------------ LayerNorm in registers
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
// x.lo * y.lo + x.hi * y.hi + c over a bf16 pair (v_dot2c_f32_bf16)
__device__ __forceinline__ float dot2bf(unsigned x, unsigned y, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, x), __builtin_bit_cast(bf16x2_t, y),
                                         c, false);
}
// LayerNorm folded into the GEMM that consumes it: with W' = diag(g) W (packed) and
// b' = b + beta W, LN(x) W + b = rstd (x W' - mean cs) + b' where cs[n] = sum_k W'[k][n] -- so the
// MFMAs run on the raw bf16 rows as soon as they land, and only the epilogue needs the row's
// statistics.  ln_stats: this wave's K-quarter fragments of row blocks rb0 .. rb0 + NRB (lane: row
// 16 rb + l % 16, columns 32 (6 v + i) + 8 (l / 16) .. + 8): sum x and sum x^2 over the bf16 pairs
// (v_dot2), then over the row's 4 lanes, into the LDS partials of wave v -- read after the next
// workgroup barrier (every caller has one before its epilogue) by ln_row.
template <int NRB>
__device__ __forceinline__ void ln_stats(const u32x4_t* xf, const Sm& sm, int rb0) {
  const int tid = otid(), v = tid >> 6, lane = tid & 63, fr = lane & 15;
  constexpr unsigned ONE2 = 0x3f803f80u;   // bf16 (1, 1)
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int i = 0; i < QS; ++i) {
      const u32x4_t u = xf[rb * QS + i];
      s = dot2bf(u.x, ONE2, s); q = dot2bf(u.x, u.x, q);
      s = dot2bf(u.y, ONE2, s); q = dot2bf(u.y, u.y, q);
      s = dot2bf(u.z, ONE2, s); q = dot2bf(u.z, u.z, q);
      s = dot2bf(u.w, ONE2, s); q = dot2bf(u.w, u.w, q);
    }
    s = add32(add16(s));
    q = add32(add16(q));
    if (lane < 16) {
      sm.ln[v * RM + 16 * (rb0 + rb) + fr] = s;
      sm.ln[(NW + v) * RM + 16 * (rb0 + rb) + fr] = q;
    }
  }
}
// the row's mean and 1 / sqrt(var + eps) from the 4 waves' partials; var = E[x^2] - mean^2 (the
// residual stream's mean is small against its spread: the one-pass form loses nothing at bf16
// output precision)
__device__ __forceinline__ void ln_row(const Sm& sm, int r, float& mean, float& rstd) {
  const float* l2 = sm.ln + NW * RM;
  mean = ((sm.ln[r] + sm.ln[RM + r]) + (sm.ln[2 * RM + r] + sm.ln[3 * RM + r])) * (1.0f / D);
  const float ex2 = ((l2[r] + l2[RM + r]) + (l2[2 * RM + r] + l2[3 * RM + r])) * (1.0f / D);
  rstd = rsqrtf(fmaxf(fmaf(-mean, mean, ex2), 0.f) + 1e-5f);
}
// the tile's NC columns from n0 of a [2][N] bias (row 0 bias, row 1 column sums) into LDS (read
// after the next workgroup barrier)
template <int NC>
__device__ __forceinline__ void stage_cb(const Sm& sm, const float* b2, int N, int n0) {
  static_assert(NC <= 64, "SM_CB holds 64 columns");
  const int t = otid();
  if (t < NC) sm.cb[t] = b2[n0 + t];
  else if (t >= 64 && t < 64 + NC) sm.cb[t] = b2[N + n0 + t - 64];
}
__device__ __forceinline__ float4 cb_quad(const Sm& sm, int lc, int row1) {
  return *reinterpret_cast<const float4*>(sm.cb + 64 * row1 + lc);
}
// rstd (sum - mean cs) + b for a lane's 4 columns
__device__ __forceinline__ float4 ln_fold(f32x4_t s, float mean, float rstd, float4 cs, float4 b) {
  return make_float4(fmaf(rstd, fmaf(-mean, cs.x, s[0]), b.x), fmaf(rstd, fmaf(-mean, cs.y, s[1]), b.y),
                     fmaf(rstd, fmaf(-mean, cs.z, s[2]), b.z), fmaf(rstd, fmaf(-mean, cs.w, s[3]), b.w));
}

// layer 0's LayerNorm input: bf16(wte[tok] + wpe[pos]) (the f32 sum rounded once)
template <int NRB>
__device__ __forceinline__ void embed_frags(const Args& a, const Sm& sm, int rb0, u32x4_t* xf) {
  const int tid = otid(), v = tid >> 6, lane = tid & 63, fr = lane & 15, fk = 8 * (lane >> 4);
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) {
    const int row = 16 * (rb0 + rb) + fr;
    const bf16_t* te = a.wte + (long)sm.tok[row] * D + fk;
#pragma unroll
    for (int i = 0; i < QS; ++i)
      xf[rb * QS + i] = *reinterpret_cast<const u32x4_t*>(te + 32 * (QS * v + i));
  }
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) {
    const int row = 16 * (rb0 + rb) + fr;
    const bf16_t* pe = a.wpe + (long)sm.pos[row] * D + fk;
    u32x4_t pu[QS];
#pragma unroll
    for (int i = 0; i < QS; ++i) pu[i] = *reinterpret_cast<const u32x4_t*>(pe + 32 * (QS * v + i));
#pragma unroll
    for (int i = 0; i < QS; ++i) {
      float t[8], p[8];
      unpack8(xf[rb * QS + i], t);
      unpack8(pu[i], p);
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] += p[e];
      xf[rb * QS + i] = pack8(t);
    }
  }
}
// the f32 embedding quad (row, col .. col + 3): the residual stream at layer 0
__device__ __forceinline__ float4 embed_quad(const Args& a, const Sm& sm, int row, int col) {
  const uint2 t = *reinterpret_cast<const uint2*>(a.wte + (long)sm.tok[row] * D + col);
  const uint2 p = *reinterpret_cast<const uint2*>(a.wpe + (long)sm.pos[row] * D + col);
  return make_float4(__uint_as_float(t.x << 16) + __uint_as_float(p.x << 16),
                     __uint_as_float(t.x & 0xffff0000u) + __uint_as_float(p.x & 0xffff0000u),
                     __uint_as_float(t.y << 16) + __uint_as_float(p.y << 16),
                     __uint_as_float(t.y & 0xffff0000u) + __uint_as_float(p.y & 0xffff0000u));
}

// ------------------------------------------------------------------ A / D: LayerNorm + GEMM
// The tile's CB col blocks x RB row blocks in rounds of CPR col blocks (<= 8 tiles of slabs);
// weights: PF == CB (all in wpf) or PF == CPR (wpf holds one round; loadw(c, n, wpf) refills it
// with the n col blocks from c after a round's MFMAs).  epi(r, j, c, rb, sum) per finalised quad
// (round r, j as reduce_tiles).
template <int CB, int RB>
struct Rounds {
  static constexpr int CPR = CB < 8 / RB ? CB : 8 / RB;      // col blocks per round
  static constexpr int NR = (CB + CPR - 1) / CPR;             // rounds
  static constexpr int NJ = (CPR * RB + NW - 1) / NW;         // finalised tiles per wave per round
};
template <int CB, int RB, int PF, typename LoadW, typename Epi>
__device__ __forceinline__ void gemm_rounds(const u32x4_t* xf, u32x4_t* wpf, f32x4_t* red,
                                            LoadW&& loadw, Epi&& epi) {
  constexpr int CPR = Rounds<CB, RB>::CPR, NR = Rounds<CB, RB>::NR;
  static_assert(PF == CB || PF == CPR, "weight prefetch rounds");
  static_for<NR>([&](auto rr) {
    constexpr int r = decltype(rr)::value, c0 = r * CPR;
    constexpr int NC = CB - c0 < CPR ? CB - c0 : CPR;
    f32x4_t acc[NC * RB];
#pragma unroll
    for (int t = 0; t < NC * RB; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < QS; ++s)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[c * RB + rb] = mfma(wpf[((PF == CB ? c0 : 0) + c) * QS + s], xf[rb * QS + s], acc[c * RB + rb]);
    if constexpr (PF != CB && c0 + CPR < CB) {
      loadw(c0 + CPR, std::integral_constant<int, (CB - c0 - CPR < CPR ? CB - c0 - CPR : CPR)>{}, wpf);
      __builtin_amdgcn_sched_barrier(0);
    }
    reduce_tiles<NC * RB>(red, acc, [&](int j, int t, f32x4_t s) { epi(r, j, c0 + t / RB, t % RB, s); });
  });
}

// A: ln_1 + c_attn.  q -> WS_Q; k / v -> the KV cache at the row's position (sc1: phase B reads
// them in this step).  wq: the prefetched weights (PM: loaded here).
template <int G, bool PM>
__device__ __forceinline__ void phase_a(const Args& a, const Rs& rs, int l, int w, const Sm& sm,
                                        u32x4_t* wq) {
  using Gm = Geo<G>;
  constexpr int CB = Gm::ACB, RB = Gm::ARB, NCG = NCB_Q / CB;
  const int tid = otid(), v = tid >> 6, lane = tid & 63;
  const int cb0 = (w % NCG) * CB, rb0 = (w / NCG) * RB;
  u32x4_t xf[RB * QS];
  if (l == 0) embed_frags<RB>(a, sm, rb0, xf);
  else lda<RB, QS>(rs.xb, KSD, rb0, QS * v, xf);
  if constexpr (PM) ldw<Gm::APF, QS>(a.wq[l], KSD, cb0, QS * v, wq);
  stage_cb<16 * CB>(sm, a.bq[l], QKVN, 16 * cb0);
  __builtin_amdgcn_sched_barrier(0);
  ln_stats<RB>(xf, sm, rb0);
  const __amdgpu_buffer_rsrc_t rk = mk(a.kc[l], a.kv_bytes), rv = mk(a.vc[l], a.kv_bytes);
  gemm_rounds<CB, RB, Gm::APF>(xf, wq, sm.red,
      [&](int c, auto n, u32x4_t* wr) { ldw<decltype(n)::value, QS>(a.wq[l], KSD, cb0 + c, QS * (otid() >> 6), wr); },
      [&](int r, int j, int c, int rb, f32x4_t s) {
        const int row = 16 * (rb0 + rb) + (lane & 15), col = 16 * (cb0 + c) + 4 * (lane >> 4);
        if (row >= a.R) return;
        float mean, rstd;
        ln_row(sm, row, mean, rstd);
        const int lc = 16 * c + 4 * (lane >> 4);
        const float4 o4 = ln_fold(s, mean, rstd, cb_quad(sm, lc, 1), cb_quad(sm, lc, 0));
        const u32x2_t o{pk2bf(o4.x, o4.y), pk2bf(o4.z, o4.w)};
        if (col < D) {
          st8(rs.q, (row * D + col) * 2, o);
        } else {
          const int j = col - D, kv = j >= D, jj = kv ? j - D : j;
          const int off = ((((row * NH + jj / HD) * a.Lmax) + sm.pos[row]) * HD + (jj % HD)) * 2;
          st8(kv ? rv : rk, off, o);
        }
      });
}

// D: ln_2 + c_fc + gelu_new -> hid (fragment order).  wf: the first round's prefetched weights.
__device__ __forceinline__ float gelu_new_fast(float x) {
  const float u2 = -1.5957691216057308f * fmaf(0.044715f * x * x, x, x);
  return x * __builtin_amdgcn_rcpf(1.0f + __expf(u2));
}
template <int G, bool PM>
__device__ __forceinline__ void phase_d(const Args& a, const Rs& rs, int l, int w, const Sm& sm,
                                        u32x4_t* wf) {
  using Gm = Geo<G>;
  constexpr int CB = Gm::DCB, RB = Gm::DRB, NCG = NCB_F / CB;
  const int tid = otid(), v = tid >> 6, lane = tid & 63;
  const int cb0 = (w % NCG) * CB, rb0 = (w / NCG) * RB;
  u32x4_t xf[RB * QS];
  lda<RB, QS>(rs.xb, KSD, rb0, QS * v, xf);
  if constexpr (PM) ldw<Gm::DPF, QS>(a.wf[l], KSD, cb0, QS * v, wf);
  stage_cb<16 * CB>(sm, a.bfc[l], DFF, 16 * cb0);
  __builtin_amdgcn_sched_barrier(0);
  ln_stats<RB>(xf, sm, rb0);
  gemm_rounds<CB, RB, Gm::DPF>(xf, wf, sm.red,
      [&](int c, auto n, u32x4_t* wr) { ldw<decltype(n)::value, QS>(a.wf[l], KSD, cb0 + c, QS * (otid() >> 6), wr); },
      [&](int r, int j, int c, int rb, f32x4_t s) {
        const int row = 16 * (rb0 + rb) + (lane & 15), col = 16 * (cb0 + c) + 4 * (lane >> 4);
        if (row >= a.R) return;
        float mean, rstd;
        ln_row(sm, row, mean, rstd);
        const int lc = 16 * c + 4 * (lane >> 4);
        const float4 h = ln_fold(s, mean, rstd, cb_quad(sm, lc, 1), cb_quad(sm, lc, 0));
        st8(rs.hid, frag_off(row, col, KSF),
            u32x2_t{pk2bf(gelu_new_fast(h.x), gelu_new_fast(h.y)),
                    pk2bf(gelu_new_fast(h.z), gelu_new_fast(h.w))});
      });
}

// ------------------------------------------------------------------ C / E: projection + residual
// The residual quad this thread owns (tile t = wave v of the C / E tiling; T <= 4 in every
// geometry): x_old from the embedding (layer 0), from the owner's registers (persistent) or from
// the workspace (phase launches); x_new = (sum + bias) + x_old -> registers / workspace and xb.
template <int G>
__device__ __forceinline__ void ce_tile(int w, int t, int& row, int& col) {
  using Gm = Geo<G>;
  constexpr int NCG = NCB_D / Gm::ECB;
  const int lane = otid() & 63;
  const int cb0 = (w % NCG) * Gm::ECB, rb0 = (w / NCG) * Gm::ERB;
  row = 16 * (rb0 + t % Gm::ERB) + (lane & 15);
  col = 16 * (cb0 + t / Gm::ERB) + 4 * (lane >> 4);
}
// (embed: the step's first residual update -- phase C of layer 0 -- whose x_old is the embedding)
template <int G, bool PM>
__device__ __forceinline__ void ce_operands(const Args& a, const Sm& sm, bool embed, int w,
                                            const float* bias, const f32x4_t& xo, float4& b,
                                            float4& xold) {
  constexpr int T = Geo<G>::ECB * Geo<G>::ERB;
  const int v = otid() >> 6;
  b = make_float4(0.f, 0.f, 0.f, 0.f);
  xold = b;
  if (v < T) {
    int row, col;
    ce_tile<G>(w, v, row, col);
    b = *reinterpret_cast<const float4*>(bias + col);
    if (embed) {
      xold = embed_quad(a, sm, row, col);
    } else if constexpr (PM) {
      xold = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.ws + WS_X) + row * D + col);
    } else {
      xold = make_float4(xo[0], xo[1], xo[2], xo[3]);
    }
  }
}
template <int G, bool PM>
__device__ __forceinline__ void ce_epilogue(const Args& a, const Rs& rs, int w, int t, f32x4_t s,
                                            const float4& b, const float4& xold, f32x4_t& xo) {
  int row, col;
  ce_tile<G>(w, t, row, col);
  const f32x4_t o{(s[0] + b.x) + xold.x, (s[1] + b.y) + xold.y, (s[2] + b.z) + xold.z,
                  (s[3] + b.w) + xold.w};
  xo = o;
  if (row < a.R) {
    st8(rs.xb, frag_off(row, col, KSD), u32x2_t{pk2bf(o[0], o[1]), pk2bf(o[2], o[3])});
    if constexpr (PM)
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.ws + WS_X) + row * D + col) =
          make_float4(o[0], o[1], o[2], o[3]);
  }
}

// C: attn.c_proj + residual (K = 768, all 6 k-steps of the quarter at once)
template <int G, bool PM>
__device__ __forceinline__ void phase_c(const Args& a, const Rs& rs, int l, int w, const Sm& sm,
                                        u32x4_t* wo, f32x4_t& xo) {
  using Gm = Geo<G>;
  constexpr int CB = Gm::ECB, RB = Gm::ERB, T = CB * RB, NCG = NCB_D / CB;
  const int v = otid() >> 6;
  const int cb0 = (w % NCG) * CB, rb0 = (w / NCG) * RB;
  u32x4_t af[RB * QS];
  lda<RB, QS>(rs.att, KSD, rb0, QS * v, af);
  if constexpr (PM) ldw<CB, QS>(a.wo[l], KSD, cb0, QS * v, wo);
  float4 b, xold;
  ce_operands<G, PM>(a, sm, l == 0, w, a.bo[l], xo, b, xold);
  __builtin_amdgcn_sched_barrier(0);
  f32x4_t acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < QS; ++s)
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[c * RB + rb] = mfma(wo[c * QS + s], af[rb * QS + s], acc[c * RB + rb]);
  reduce_tiles<T>(sm.red, acc, [&](int, int t, f32x4_t s) { ce_epilogue<G, PM>(a, rs, w, t, s, b, xold, xo); });
}

// E: mlp.c_proj + residual (K = 3072: the quarter's 24 k-steps streamed in chunks of ECH, ESL in
// flight; wm holds the first ESL chunks' weights: prefetched, or loaded here (PM))
template <int G, bool PM>
__device__ __forceinline__ void phase_e(const Args& a, const Rs& rs, int l, int w, const Sm& sm,
                                        u32x4_t* wm, f32x4_t& xo) {
  using Gm = Geo<G>;
  constexpr int CB = Gm::ECB, RB = Gm::ERB, T = CB * RB, NCG = NCB_D / CB, NCH = QF / ECH, ESL = Gm::ESL;
  const int v = otid() >> 6;
  const int cb0 = (w % NCG) * CB, rb0 = (w / NCG) * RB, s0 = QF * v;
  if constexpr (PM) {
#pragma unroll
    for (int k = 0; k < ESL; ++k) ldw<CB, ECH>(a.wm[l], KSF, cb0, s0 + ECH * k, wm + k * CB * ECH);
  }
  u32x4_t af[ESL * RB * ECH];
#pragma unroll
  for (int k = 0; k < ESL; ++k) lda<RB, ECH>(rs.hid, KSF, rb0, s0 + ECH * k, af + k * RB * ECH);
  float4 b, xold;
  ce_operands<G, PM>(a, sm, false, w, a.bm[l], xo, b, xold);
  __builtin_amdgcn_sched_barrier(0);
  f32x4_t acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  static_for<NCH>([&](auto cc) {
    constexpr int c = decltype(cc)::value, sl = c % ESL;
#pragma unroll
    for (int s = 0; s < ECH; ++s)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[cb * RB + rb] = mfma(wm[(sl * CB + cb) * ECH + s], af[(sl * RB + rb) * ECH + s], acc[cb * RB + rb]);
    if constexpr (c + ESL < NCH) {
      ldw<CB, ECH>(a.wm[l], KSF, cb0, s0 + ECH * (c + ESL), wm + sl * CB * ECH);
      lda<RB, ECH>(rs.hid, KSF, rb0, s0 + ECH * (c + ESL), af + sl * RB * ECH);
      __builtin_amdgcn_sched_barrier(0);
    }
  });
  reduce_tiles<T>(sm.red, acc, [&](int, int t, f32x4_t s) { ce_epilogue<G, PM>(a, rs, w, t, s, b, xold, xo); });
}

// ------------------------------------------------------------------ B: attention
// unit u = (row u / 12, head u % 12); wave v of workgroup w takes units w UPG + v KU .. + KU.
// 8 lanes per key (lane sub = l % 8 holds dims 8 sub .. + 8), 8 key groups (grp = l / 8), chunks
// of 8 KC keys; online softmax in f32.  The cached keys 0 .. pos - 1 are read with plain loads
// (chunk 0 issued before the workgroup waits on the c_attn barrier); the new key / value (pos)
// and q are hand-offs (sc1).
__device__ __forceinline__ void attn_unit(const Args& a, const Sm& sm, int u, int& row, int& hh,
                                          int& p, long& base) {
  row = u / NH;
  hh = u % NH;
  const int rr = min(row, a.R - 1);
  p = (a.exp & 2) ? 1 : min(sm.pos[rr], a.Lmax - 1);
  base = ((long)(rr * NH + hh) * a.Lmax) * HD + 8 * ((otid() & 63) & 7);
}
template <int KU, int KC>
__device__ __forceinline__ void attn_load(const Args& a, int l, const Sm& sm, int ub, int cb,
                                          u32x4_t (&kr)[KU][KC], u32x4_t (&vr)[KU][KC]) {
  const int tid = otid(), v = tid >> 6, grp = (tid & 63) >> 3;
  const bf16_t* kc = a.kc[l];
  const bf16_t* vc = a.vc[l];
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    int row, hh, p;
    long base;
    attn_unit(a, sm, ub + KU * v + k, row, hh, p, base);
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const int jc = max(min(cb + 8 * i + grp, p - 1), 0);
      kr[k][i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(kc + base + (long)jc * HD));
      vr[k][i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(vc + base + (long)jc * HD));
    }
  }
}
template <int KU, int KC>
__device__ __forceinline__ void phase_b(const Args& a, const Rs& rs, int l, const Sm& sm, int ub,
                                        u32x4_t (&kr)[KU][KC], u32x4_t (&vr)[KU][KC]) {
  const int tid = otid(), lane = tid & 63, v = tid >> 6, grp = lane >> 3, sub = lane & 7;
  const __amdgpu_buffer_rsrc_t rk = mk(a.kc[l], a.kv_bytes), rv = mk(a.vc[l], a.kv_bytes);
  float m[KU], sum[KU];
  f32x2_t o[KU][4];
  int p[KU], row[KU], hh[KU];
  long base[KU];
  u32x4_t qu[KU], knu[KU], vnu[KU];
  // q and the new key / value (position pos, written by phase A this step) in one round trip
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    attn_unit(a, sm, ub + KU * v + k, row[k], hh[k], p[k], base[k]);
    qu[k] = ld16(rs.q, (min(row[k], a.R - 1) * D + hh[k] * HD + 8 * sub) * 2);
    const int off = (int)((base[k] + (long)p[k] * HD) * 2);
    knu[k] = ld16(rk, off);
    vnu[k] = ld16(rv, off);
  }
  __builtin_amdgcn_sched_barrier(0);
  // q . k over the lane's 8 dims: four bf16-pair dots, then the 8 lanes of the key, / sqrt(64)
  auto qk = [&](const u32x4_t& qv, const u32x4_t& kv) {
    float sv = dot2bf(qv.x, kv.x, 0.f);
    sv = dot2bf(qv.y, kv.y, sv);
    sv = dot2bf(qv.z, kv.z, sv);
    sv = dot2bf(qv.w, kv.w, sv);
    return sum8(sv) * 0.125f;
  };
  // the online softmax starts from the new key (position pos): its score is every lane's running
  // max, and lane group 0 alone carries its weight 1 and its value (the groups are summed at the
  // end), so the new key / value registers are free before the cached keys stream in
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    m[k] = qk(qu[k], knu[k]);
    sum[k] = grp == 0 ? 1.f : 0.f;
    const unsigned w[4] = {vnu[k].x, vnu[k].y, vnu[k].z, vnu[k].w};
#pragma unroll
    for (int t = 0; t < 4; ++t)
      o[k][t] = grp == 0 ? f32x2_t{__uint_as_float(w[t] << 16), __uint_as_float(w[t] & 0xffff0000u)}
                         : f32x2_t{0.f, 0.f};
  }
  auto vacc = [&](f32x2_t (&acc)[4], float e, const u32x4_t& vv) {
    const unsigned w[4] = {vv.x, vv.y, vv.z, vv.w};
    const f32x2_t e2 = {e, e};
#pragma unroll
    for (int t = 0; t < 4; ++t)
      acc[t] = __builtin_elementwise_fma(e2, f32x2_t{__uint_as_float(w[t] << 16),
                                                     __uint_as_float(w[t] & 0xffff0000u)}, acc[t]);
  };
  int pmax = p[0];
#pragma unroll
  for (int k = 1; k < KU; ++k) pmax = max(pmax, p[k]);
  // loads in chunks of 8 KC keys; the online softmax always steps 32 keys at a time (the same
  // recurrence, so the same rounding, whatever KC a grid size loads with)
  for (int cb = 0; cb < pmax; cb += 8 * KC) {
    if (cb > 0) attn_load<KU, KC>(a, l, sm, ub, cb, kr, vr);
#pragma unroll
    for (int h = 0; h < KC / 4; ++h) {
      const int cs = cb + 32 * h;
#pragma unroll
      for (int k = 0; k < KU; ++k) {
        if (cs >= p[k]) continue;                   // wave-uniform
        float sc[4];
        float pm = -INFINITY;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float sv = qk(qu[k], kr[k][4 * h + i]);
          sc[i] = cs + 8 * i + grp < p[k] ? sv : -INFINITY;
          pm = fmaxf(pm, sc[i]);
        }
        pm = fmaxf(pm, xor8(pm));
        pm = max16(pm);
        pm = max32(pm);
        const float mn = fmaxf(m[k], pm);
        const float scale = __expf(m[k] - mn);
        sum[k] *= scale;
        const f32x2_t sc2 = {scale, scale};
#pragma unroll
        for (int t = 0; t < 4; ++t) o[k][t] *= sc2;
        m[k] = mn;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __expf(sc[i] - mn);
          sum[k] += e;
          vacc(o[k], e, vr[k][4 * h + i]);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    const float inv = 1.0f / add32(add16(sum[k] + xor8(sum[k])));
    float of[8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      of[2 * t] = add32(add16(o[k][t].x + xor8(o[k][t].x))) * inv;
      of[2 * t + 1] = add32(add16(o[k][t].y + xor8(o[k][t].y))) * inv;
    }
    if (grp == 0 && row[k] < a.R) {
      // att in fragment order: row r, dims 64 h + 8 sub .. + 8 = k-step 2 h + sub / 4,
      // lane (r & 15) + 16 (sub & 3)
      const int r = row[k];
      st16(rs.att, (((r >> 4) * KSD + 2 * hh[k] + (sub >> 2)) * 64 + (r & 15) + 16 * (sub & 3)) * 16,
           pack8(of));
    }
  }
}

// ------------------------------------------------------------------ F: ln_f + LM head
// Vocab blocks of 16 b = w, w + G, ..; per block each wave multiplies its K quarter (6 KiB of the
// fragment-packed table) into all 64 rows, the 4 partial tiles go through double-buffered slabs,
// and wave v finalises row block v: 4 logits per lane, a running (logit, id) best per lane.
// A ring of FSL blocks of weights per wave is in flight.
// DYN (persistent launches): the vocab blocks are split into a static part -- outer iterations
// u < su of FSL blocks each, block w + G (FSL u + k) -- and a dynamic part of chunks of FSL
// consecutive blocks from d0 = G FSL su, which the workgroups claim from an agent-scope counter
// (fctr, zeroed for this step) three outer iterations ahead: a workgroup that runs slow beside
// other grids claims fewer chunks, so the phase ends with the average workgroup instead of the
// slowest (a logit's arithmetic does not depend on who computes it; the argmax is an exact
// max).  Phase launches (DYN false) take every block statically.
template <int G, bool DYN>
__device__ __forceinline__ void phase_f(const Args& a, const Rs& rs, int w, const Sm& sm, gu64* keys,
                                        gu32* fctr) {
  const int tid = otid(), v = tid >> 6, lane = tid & 63;
  u32x4_t xf[4 * QS];
  lda<4, QS>(rs.xb, KSD, 0, QS * v, xf);
  const int nvb = (a.V + 15) >> 4, lmv = 16 * nvb;    // lmb: [2][16 nvb] bias, then cs
  constexpr int NSL = Geo<G>::FSL;
  int su = (nvb + G * NSL - 1) / (G * NSL);           // static: every block (past nvb: skipped)
  bool dyn = false;
  if constexpr (DYN) {
    // ~5/8 of the blocks static (>= 3 outer iterations: the claims run 3 ahead), the rest claimed
    const int s2 = max(3, (nvb * 5 / 8) / (G * NSL));
    if (G * NSL * s2 <= nvb - G && a.exp == 0 && a.dynf) { su = s2; dyn = true; }
  }
  const int d0 = G * NSL * su, nch = dyn ? (nvb - d0 + NSL - 1) / NSL : 0;   // claimable chunks
  int* const chr = sm.misc + 12;   // LDS ring: the chunk claimed for outer iteration u at [u & 3]
  // first block and block stride of outer iteration u's items (>= nvb: no items; read once per
  // iteration into scalars, so the ring refills do not wait on LDS)
  auto iter_blocks = [&](int u, int& b0, int& st) {
    if (u < su) { b0 = w + G * NSL * u; st = G; }
    else if (dyn) { b0 = d0 + NSL * __builtin_amdgcn_readfirstlane(chr[u & 3]); st = 1; }
    else { b0 = 0x3fffffff; st = 0; }
  };
  // ring of FSL block slots, each this wave's 6 weight fragments of the block; every refill is
  // unconditional (block index clamped to the last block: a conditional load left the compiler
  // counting conservatively, vmcnt(0) before every block, one round trip per block).  The lane's 4
  // per-token biases and column sums of a block are loaded one block ahead (FSL even: the pair a
  // block uses is fixed at compile time)
  static_assert(Geo<G>::FSL % 2 == 0 && Geo<G>::FSL >= 2, "F ring: an even number of slots");
  struct Slot {
    u32x4_t w[QS];
  };
  Slot R[NSL];
  auto fill = [&](int b, Slot& r) { ldw<1, QS>(a.wtep, KSD, min(max(b, 0), nvb - 1), QS * v, r.w); };
  float4 bq[2], cq[2];
  auto fill_b = [&](int b, float4& bb, float4& c) {
    const int bc = min(max(b, 0), nvb - 1);
    bb = *reinterpret_cast<const float4*>(a.lmb + 16 * bc + 4 * (lane >> 4));
    c = *reinterpret_cast<const float4*>(a.lmb + lmv + 16 * bc + 4 * (lane >> 4));
  };
  static_for<NSL>([&](auto k) { fill(w + G * decltype(k)::value, R[decltype(k)::value]); });
  fill_b(w, bq[0], cq[0]);
  __builtin_amdgcn_sched_barrier(0);
  ln_stats<4>(xf, sm, 0);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  const bool tmp = a.temp != 1.0f;
  int buf = 0;
  lds_sync();     // the previous phase's slab readers are done; the row statistics are in
  float mean, rstd;
  ln_row(sm, 16 * v + (lane & 15), mean, rstd);   // wave v finalises row block v
  auto consume = [&](int b, const Slot& r, const float4& rb_, const float4& rc_) {
    f32x4_t acc[4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) acc[rb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < QS; ++s)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[rb] = mfma(r.w[s], xf[rb * QS + s], acc[rb]);
    f32x4_t* red = sm.red + buf * 1024;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) red[(v * 4 + rb) * 64 + lane] = acc[rb];
    lds_sync();
    const f32x4_t sum = (red[v * 64 + lane] + red[(4 + v) * 64 + lane]) +
                        (red[(8 + v) * 64 + lane] + red[(12 + v) * 64 + lane]);
    const int col0 = 16 * b + 4 * (lane >> 4);
    const float4 lg4 = ln_fold(sum, mean, rstd, rc_, rb_);
    const float lgv[4] = {lg4.x, lg4.y, lg4.z, lg4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float lg = lgv[e];
      const float val = tmp ? lg / a.temp : lg;
      if (col0 + e < a.V && val > bv) { bv = val; bi = col0 + e; }
    }
    buf ^= 1;
  };
  // claims (thread 0, dynamic part): at slot 1 of outer iteration u the chunk claimed at u - 1 is
  // published for u + 2, and the chunk for u + 3 claimed -- before slot 1's ring refill, so the
  // next iteration's wait for that refill has also waited for the claim (no extra round trip);
  // the other waves read it after the next consume's workgroup barrier.  Claims only grow, so a
  // workgroup's chunks end at its first invalid one (later claims are discarded; the counter of
  // the other step parity is re-zeroed by workgroup 0 during the next step)
  unsigned pend = 0;
  int bu, stu;
  iter_blocks(0, bu, stu);
  // (an iteration whose first block is past the vocabulary has no items, and neither has any
  // later one: static blocks grow with u, claimed chunks too)
#pragma nounroll
  for (int u = 0; bu < nvb && u < su + nch; ++u) {
    int bn, stn;
    iter_blocks(u + 1, bn, stn);      // (u + 1's chunk: published at u - 1, slot 1)
    static_for<NSL>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      const int b = bu + k * stu;
      if (b < nvb) {                                    // (wave-uniform)
        fill_b(k + 1 < NSL ? b + stu : bn, bq[(k + 1) % 2], cq[(k + 1) % 2]);
        consume(b, R[k], bq[k % 2], cq[k % 2]);
      }
      if constexpr (k == 1) {
        if (dyn && tid == 0 && u >= su - 3) {
          if (u >= su - 2) chr[(u + 2) & 3] = (int)pend;
          pend = __hip_atomic_fetch_add(fctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      fill(bn + k * stn, R[k]);
    });
    bu = bn;
    stu = stn;
  }
  // the 4 lanes of a row (l % 16 equal): larger logit, then the lower id
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  if (lane < 16) {
    const unsigned long long key = ((unsigned long long)f2key(bv) << 32) | (unsigned)(~bi);
    __hip_atomic_fetch_max(keys + 16 * v + lane, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ------------------------------------------------------------------ row state
template <typename A>
__device__ __forceinline__ void load_state(const A& a, const Sm& sm) {
  const int tid = otid();
  if (tid < RM) {
    const bool in = tid < a.R;
    sm.tok[tid] = in ? a.next_tok[tid] : 0;
    sm.pos[tid] = in ? a.pos[tid] : 0;
    sm.done[tid] = in ? a.done[tid] : 1;
  }
}
// generate2's bookkeeping of step `step` from the argmax keys (greedy_step_kernel, gpt2.hip):
// every workgroup updates its LDS copy; `commit`: also ids and the state in memory.  Returns the
// rows still decoding (in sm.misc[0] after the caller's barrier).
template <typename A>
__device__ __forceinline__ void bookkeep(const A& a, const Sm& sm, gu64* keys, int step, bool commit) {
  const int tid = otid();
  int alive = 0;
  if (tid < RM) {
    const unsigned long long key = __hip_atomic_load(keys + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // (a key no workgroup raised -- impossible unless the vocabulary pass skipped a row's every
    // block -- would read as id -1: clamped, so a broken pass shows as wrong ids, never as an
    // out-of-bounds embedding read next step)
    const int t = min(max((int)~(unsigned)key, 0), a.V - 1);
    if (tid < a.R) {
      int d = sm.done[tid];
      if (!d) {
        if (commit) {
          a.out_ids[(long)tid * a.max_steps + step] = t;
          a.out_len[tid] = step + 1;
        }
        if (t == a.stop0 || t == a.stop1) d = 1;
      }
      alive = !d;
      sm.done[tid] = d;
      sm.tok[tid] = t;
      sm.pos[tid] += 1;
      if (commit) {
        a.done[tid] = d;
        a.pos[tid] = sm.pos[tid];
        a.next_tok[tid] = t;
      }
    }
  }
  const unsigned long long bal = __ballot(alive);
  if (tid == 0) sm.misc[0] = (int)__popcll(bal);
}

// a workgroup that gave up waiting (grid not co-resident): all_done = {1, -1} tells the host
template <typename A>
__device__ __forceinline__ void gave_up(const A& a) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(&a.all_done[1], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.all_done[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ------------------------------------------------------------------ persistent kernel
template <int G>
__global__ __launch_bounds__(NT, 2) void dg_persist_kernel(Args a) {
  using Gm = Geo<G>;
  constexpr int KU = Units<G>::KU, KC = Units<G>::KC;
  __shared__ __attribute__((aligned(16))) char smem[SM_TOTAL];
  const Sm sm(smem);
  const int w = blockIdx.x;
  if (a.all_done[0]) return;                 // every row stopped at step 0 (uniform)
  int step = *a.step_ctr;
  if (step >= a.max_steps) return;
  load_state(a, sm);
  __syncthreads();
  const Rs rs = make_rs(a.ws, a.exp);
  Bar bar{(gu32*)(a.ws + WS_SH), (gu32*)(a.ws + WS_TMO), 0, G / NSH, a.spin_max, nullptr, 0};
  gu64* const keys = (gu64*)(a.ws + WS_KEY);
  gu32* const clm = (gu32*)(a.ws + WS_CLM);
  volatile lds_int_t* s_ok = (volatile lds_int_t*)(sm.misc + 8);
  unsigned long long* const stamps =
      (dp_stamp_ws == nullptr || dp_stamp_ws == a.ws) ? dp_stamp_buf : nullptr;
  const int stamp_step = dp_stamp_step;
  if (stamp_step == -2 && threadIdx.x == 0) {   // diagnostic: where this workgroup runs
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    ((gu64*)(a.ws + WS_X))[w] = ((unsigned long long)xcc << 32) | hw;
  }
  const int ub = w * Units<G>::UPG;
  constexpr int ANCG = NCB_Q / Gm::ACB, DNCG = NCB_F / Gm::DCB, ENCG = NCB_D / Gm::ECB;
  const int acb0 = (w % ANCG) * Gm::ACB, dcb0 = (w % DNCG) * Gm::DCB, ecb0 = (w % ENCG) * Gm::ECB;
#define V_ (otid() >> 6)
  u32x4_t wq[Gm::APF * QS];
  ldw<Gm::APF, QS>(a.wq[0], KSD, acb0, QS * V_, wq);
  f32x4_t xo{0.f, 0.f, 0.f, 0.f};
  for (;;) {
    bar.sb = (stamps != nullptr && step == stamp_step) ? stamps + (long)w * 2 * DP_NB : nullptr;
    bar.n0 = bar.n;
    stamp(bar.sb, 2 * DP_NB - 1);
    if (step == a.abort_step) return gave_up(a);    // (test knob: every workgroup, same point)
    for (int l = 0; l < NLY; ++l) {
      phase_a<G, false>(a, rs, l, w, sm, wq);
      bar_arrive(bar, w);
      u32x4_t kr[KU][KC], vr[KU][KC];
      attn_load<KU, KC>(a, l, sm, ub, 0, kr, vr);
      if (!bar_wait(bar, s_ok)) return gave_up(a);
      if (l == 0 && w == 0 && otid() < RM) {  // last step's keys / F claims: every workgroup is done
        __hip_atomic_store(keys + ((step + 1) & 1) * RM + otid(), 0ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        if (otid() == 0)
          __hip_atomic_store(clm + (CLM_F + ((step + 1) & 1)) * 32, 0u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      phase_b<KU, KC>(a, rs, l, sm, ub, kr, vr);
      bar_arrive(bar, w);
      u32x4_t wo[Gm::ECB * QS];
      ldw<Gm::ECB, QS>(a.wo[l], KSD, ecb0, QS * V_, wo);
      if (!bar_wait(bar, s_ok)) return gave_up(a);
      phase_c<G, false>(a, rs, l, w, sm, wo, xo);
      bar_arrive(bar, w);
      u32x4_t wf[Gm::DPF * QS];
      ldw<Gm::DPF, QS>(a.wf[l], KSD, dcb0, QS * V_, wf);
      if (!bar_wait(bar, s_ok)) return gave_up(a);
      phase_d<G, false>(a, rs, l, w, sm, wf);
      bar_arrive(bar, w);
      u32x4_t wm[Gm::ESL * Gm::ECB * ECH];
#pragma unroll
      for (int k = 0; k < Gm::ESL; ++k)
        ldw<Gm::ECB, ECH>(a.wm[l], KSF, ecb0, QF * V_ + ECH * k, wm + k * Gm::ECB * ECH);
      if (!bar_wait(bar, s_ok)) return gave_up(a);
      phase_e<G, false>(a, rs, l, w, sm, wm, xo);
      bar_arrive(bar, w);
      // (the last layer's branch overwrites wq too: otherwise the merge keeps A's operands live
      // through B .. E of every layer)
      if (l + 1 < NLY) ldw<Gm::APF, QS>(a.wq[l + 1], KSD, acb0, QS * V_, wq);
      else for (int i = 0; i < Gm::APF * QS; ++i) wq[i] = u32x4_t{0u, 0u, 0u, 0u};
      if (!bar_wait(bar, s_ok)) return gave_up(a);
    }
    phase_f<G, true>(a, rs, w, sm, keys + (step & 1) * RM, clm + (CLM_F + (step & 1)) * 32);
    bar_arrive(bar, w);
    ldw<Gm::APF, QS>(a.wq[0], KSD, acb0, QS * V_, wq);
    if (!bar_wait(bar, s_ok)) return gave_up(a);
    // ---- every workgroup applies the bookkeeping; workgroup 0 commits it
    bookkeep(a, sm, keys + (step & 1) * RM, step, w == 0);
    __syncthreads();
    stamp(bar.sb, 2 * DP_NB - 2);
    const int total = sm.misc[0];
    const bool fin = total == 0 || step + 1 >= a.max_steps;
    if (w == 0 && otid() == 0) {
      *a.step_ctr = step + 1;
      a.all_done[2] = total;
      if (fin) a.all_done[0] = 1;
    }
    if (fin) return;
    ++step;
    __syncthreads();     // sm.misc is rewritten next step
  }
#undef V_
}

// ------------------------------------------------------------------ phase launches
enum { PH_A = 0, PH_B, PH_C, PH_D, PH_E, PH_F };
template <int G, int PH>
__global__ __launch_bounds__(NT, 2) void dg_phase_kernel(Args a) {
  using Gm = Geo<G>;
  __shared__ __attribute__((aligned(16))) char smem[SM_TOTAL];
  const Sm sm(smem);
  const int w = blockIdx.x, l = a.layer;
  if (a.all_done[0]) return;                 // finished: the rest of a replayed chunk is a no-op
  if (*a.step_ctr >= a.max_steps) return;
  load_state(a, sm);
  __syncthreads();
  const Rs rs = make_rs(a.ws, a.exp);
  if constexpr (PH == PH_A) {
    u32x4_t wq[Gm::APF * QS];
    phase_a<G, true>(a, rs, l, w, sm, wq);
  } else if constexpr (PH == PH_B) {
    constexpr int KU = Units<G>::KU, KC = Units<G>::KC;
    u32x4_t kr[KU][KC], vr[KU][KC];
    attn_load<KU, KC>(a, l, sm, w * Units<G>::UPG, 0, kr, vr);
    phase_b<KU, KC>(a, rs, l, sm, w * Units<G>::UPG, kr, vr);
  } else if constexpr (PH == PH_C) {
    u32x4_t wo[Gm::ECB * QS];
    f32x4_t xo{0.f, 0.f, 0.f, 0.f};
    phase_c<G, true>(a, rs, l, w, sm, wo, xo);
  } else if constexpr (PH == PH_D) {
    u32x4_t wf[Gm::DPF * QS];
    phase_d<G, true>(a, rs, l, w, sm, wf);
  } else if constexpr (PH == PH_E) {
    u32x4_t wm[Gm::ESL * Gm::ECB * ECH];
    f32x4_t xo{0.f, 0.f, 0.f, 0.f};
    phase_e<G, true>(a, rs, l, w, sm, wm, xo);
  } else {
    phase_f<G, false>(a, rs, w, sm, (gu64*)(a.ws + WS_KEY), nullptr);
  }
}
// the step's bookkeeping (phase launches): one workgroup of 64 threads; zeroes the keys
template <typename A>
__global__ __launch_bounds__(64) void dg_book_kernel(A a) {
  __shared__ __attribute__((aligned(16))) char smem[SM_TOTAL];
  const Sm sm(smem);
  if (a.all_done[0]) return;
  const int step = *a.step_ctr;
  if (step >= a.max_steps) return;
  load_state(a, sm);
  __syncthreads();
  gu64* keys = (gu64*)(a.ws + WS_KEY);
  bookkeep(a, sm, keys, step, true);
  __syncthreads();
  if (threadIdx.x < RM) keys[threadIdx.x] = 0ull;
  if (threadIdx.x == 0) {
    const int total = sm.misc[0];
    *a.step_ctr = step + 1;
    a.all_done[2] = total;
    if (total == 0 || step + 1 >= a.max_steps) a.all_done[0] = 1;
  }
}

// ================================================================== f32 parity mode
// The same grid decode in f32 (zs_gpt2_decode_persist_f32 / _phases_f32): f32 weights, f32
// activations, KV cache and hand-offs, exact f32 products (v_mfma_f32_16x16x4_f32: bitwise an fmaf
// chain), two-pass LayerNorms (mean, then the squared deviations) whose affine is folded into the
// consuming GEMM in f32 (W' = W diag(g), b' = b + W beta, the host's f64 sums rounded once; ln_f's
// into the tied LM head plus a per-token bias) -- the normalised row feeds the MFMAs directly.
// A 16-byte lane fragment holds 4 f32 of one row (k-steps of 16: lane l holds k = 16 s + 4 (l / 16)
// .. + 4 of row / column l % 16), so one fragment feeds four MFMAs and a wave's K quarter is 12
// fragments (K = 768) or 48 (K = 3072): twice the bf16 registers, so one geometry, G = 192.  The
// canonical-arithmetic rules of the bf16 kernel hold here too (K quarters, (p0 + p1) + (p2 + p3),
// 32-key softmax steps), so the persistent and the phase launches give identical ids.
namespace f32 {
constexpr int KSD = D / 16, KSF = DFF / 16;      // 16-k fragments of K = 768 / 3072
constexpr int QS = KSD / NW, QF = KSF / NW;      // per wave quarter: 12 / 48
constexpr int G = 192;
// tiles per workgroup: A 3 column blocks x 1 row block (c_attn: 144 blocks / 3 = 48 column groups
// x 4 row groups), C / E 1 x 1 (48 x 4), D 2 x 2 (96 x 2); F one row half (2 row blocks) over the
// vocab blocks (w % 8 + 8 (w / 16)) + 96 i: the two workgroups of a block share an XCD
constexpr int ACB = 3, ARB = 1, DCB = 2, DRB = 2, ECB = 1, ERB = 1;
constexpr int APF = 3;          // c_attn column blocks prefetched across the barrier (the rest: in A)
constexpr int UPG = RM * NH / G, KC = 8;   // attention: UPG / 4 = 1 unit per wave; 8 KC keys loaded per
                                           // chunk, the softmax stepping 32 at a time
constexpr int ESL = 4;                     // E: chunks of ECH k-steps in flight
constexpr int FH = G / 2;                        // LM-head workgroups per row half

constexpr int WS_Q = WS_SYNC_BYTES;              // f32 [64][768]
constexpr int WS_ATT = WS_Q + RM * D * 4;        // f32 [4][48][64][4] (fragment order)
constexpr int WS_XB = WS_ATT + RM * D * 4;       // f32 [4][48][64][4]: the residual stream x
constexpr int WS_HID = WS_XB + RM * D * 4;       // f32 [4][192][64][4]
constexpr int WS_BYTES = WS_HID + RM * DFF * 4;
constexpr int SM_TOTAL32 = SM_TOTAL;

struct Args {
  int R, Lmax, max_steps, stop0, stop1, V, layer, abort_step;
  unsigned spin_max;
  int kv_bytes;
  float temp;
  const float* wte; const float* wpe;
  // per block, weights in f32 fragment order [N/16][K/16][64][4] (ops.pack_f32_fragments), the
  // LayerNorm-fed ones with the affine folded in
  const float* wq[NLY]; const float* bq[NLY];
  const float* wo[NLY]; const float* bo[NLY];
  const float* wf[NLY]; const float* bfc[NLY];
  const float* wm[NLY]; const float* bm[NLY];
  const float* wtep;                             // the tied LM head (g o wte), fragment order
  const float* lmb;                              // beta . wte[v], [ceil(V/16) 16]
  float* kc[NLY]; float* vc[NLY];
  int* pos; int* next_tok; int* done; int* out_ids; int* out_len; int* step_ctr; int* all_done;
  char* ws;
};

struct Rs {
  __amdgpu_buffer_rsrc_t q, att, xb, hid;
};
__device__ __forceinline__ Rs make_rs(char* ws) {
  return Rs{mk(ws + WS_Q, RM * D * 4), mk(ws + WS_ATT, RM * D * 4), mk(ws + WS_XB, RM * D * 4),
            mk(ws + WS_HID, RM * DFF * 4)};
}

// 4 chained MFMAs over a fragment pair: the MFMA's k index g stands for k + 4 g + j in MFMA j
__device__ __forceinline__ f32x4_t mfma4(const u32x4_t& w, const u32x4_t& a, f32x4_t c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.x), __uint_as_float(a.x), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.y), __uint_as_float(a.y), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.z), __uint_as_float(a.z), c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.w), __uint_as_float(a.w), c, 0, 0, 0);
}
// Fragment loads as buffer loads: one VGPR offset (the lane's and the wave's part) and the
// fragment's compile-time part in the scalar offset, so a batch of loads costs no address
// registers (the f32 phases hold up to 60 fragments).  Weights: plain loads; hand-offs: sc1.
template <int NB, int S>
__device__ __forceinline__ void ldw(const float* Wp, int KS, int cb0, int s0, u32x4_t* w) {
  const __amdgpu_buffer_rsrc_t r = mk(const_cast<float*>(Wp), 0x7ffffff0);
  const int vo = ((cb0 * KS + s0) * 64 + (otid() & 63)) * 16;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int s = 0; s < S; ++s) w[nb * S + s] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, (nb * KS + s) * 1024, 0);
}
template <int NRB, int S>
__device__ __forceinline__ void lda(__amdgpu_buffer_rsrc_t r, int KS, int rb0, int s0, u32x4_t* a) {
  const int vo = ((rb0 * KS + s0) * 64 + (otid() & 63)) * 16;
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
    for (int s = 0; s < S; ++s) a[rb * S + s] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, (rb * KS + s) * 1024, 16);
}
// byte offset of the quad (row, col .. col + 3) (col % 4 == 0) in a fragment-order f32 activation
__device__ __forceinline__ int frag_off(int row, int col, int KS) {
  return (((row >> 4) * KS + (col >> 4)) * 64 + (row & 15) + 16 * ((col >> 2) & 3)) * 16;
}
__device__ __forceinline__ u32x4_t u4(const float4& f) {
  return u32x4_t{__float_as_uint(f.x), __float_as_uint(f.y), __float_as_uint(f.z), __float_as_uint(f.w)};
}
__device__ __forceinline__ float4 f4(const u32x4_t& u) {
  return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}
__device__ __forceinline__ float4 add4(const float4& a, const float4& b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// LayerNorm of row blocks rb0 .. rb0 + NRB held in registers (lane: row 16 rb + l % 16, this wave's
// K quarter), in place: mean from the row's 4 lanes and the 4 waves' partials ((w0 + w1) + (w2 +
// w3)), then the squared deviations the same way, rstd = rsqrt(var + 1e-5), y = (x - mean) rstd
// (the affine is in the weights).  Two workgroup barriers.
template <int NRB>
__device__ __forceinline__ void ln_apply(u32x4_t* xf, const Sm& sm, int rb0) {
  const int tid = otid(), v = tid >> 6, lane = tid & 63, fr = lane & 15;
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < QS; ++i) {
      const float4 x = f4(xf[rb * QS + i]);
      s += (x.x + x.y) + (x.z + x.w);
    }
    s = add32(add16(s));
    if (lane < 16) sm.ln[v * RM + 16 * (rb0 + rb) + fr] = s;
  }
  lds_sync();
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) {
    const int r = 16 * (rb0 + rb) + fr;
    const float mean = ((sm.ln[r] + sm.ln[RM + r]) + (sm.ln[2 * RM + r] + sm.ln[3 * RM + r])) * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < QS; ++i) {
      const float4 x = f4(xf[rb * QS + i]);
      const float4 d = make_float4(x.x - mean, x.y - mean, x.z - mean, x.w - mean);
      q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
      xf[rb * QS + i] = u4(d);
    }
    q = add32(add16(q));
    if (lane < 16) sm.ln[(NW + v) * RM + r] = q;
  }
  lds_sync();
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) {
    const int r = 16 * (rb0 + rb) + fr;
    const float* l2 = sm.ln + NW * RM;
    const float var = ((l2[r] + l2[RM + r]) + (l2[2 * RM + r] + l2[3 * RM + r])) * (1.0f / D);
    const float rstd = rsqrtf(var + 1e-5f);
#pragma unroll
    for (int i = 0; i < QS; ++i) {
      const float4 d = f4(xf[rb * QS + i]);
      xf[rb * QS + i] = u4(make_float4(d.x * rstd, d.y * rstd, d.z * rstd, d.w * rstd));
    }
  }
}

// layer 0's input rows: wte[tok] + wpe[pos] (f32)
template <int NRB>
__device__ __forceinline__ void embed_frags(const Args& a, const Sm& sm, int rb0, u32x4_t* xf) {
  const int tid = otid(), v = tid >> 6, lane = tid & 63, fr = lane & 15, fk = 4 * (lane >> 4);
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) {
    const int row = 16 * (rb0 + rb) + fr;
    const float* te = a.wte + (long)sm.tok[row] * D + fk;
    const float* pe = a.wpe + (long)sm.pos[row] * D + fk;
#pragma unroll
    for (int i = 0; i < QS; ++i)
      xf[rb * QS + i] = u4(add4(*reinterpret_cast<const float4*>(te + 16 * (QS * v + i)),
                                *reinterpret_cast<const float4*>(pe + 16 * (QS * v + i))));
  }
}
__device__ __forceinline__ float4 embed_quad(const Args& a, const Sm& sm, int row, int col) {
  return add4(*reinterpret_cast<const float4*>(a.wte + (long)sm.tok[row] * D + col),
              *reinterpret_cast<const float4*>(a.wpe + (long)sm.pos[row] * D + col));
}

// one GEMM round: CB x RB tiles of this wave's K quarter, then the cross-wave sum
template <int CB, int RB, typename Epi>
__device__ __forceinline__ void gemm_tiles(const u32x4_t* xf, const u32x4_t* wr, const Sm& sm, Epi&& epi) {
  f32x4_t acc[CB * RB];
#pragma unroll
  for (int t = 0; t < CB * RB; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < QS; ++s)
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[c * RB + rb] = mfma4(wr[c * QS + s], xf[rb * QS + s], acc[c * RB + rb]);
  reduce_tiles<CB * RB>(sm.red, acc, epi);
}
// the bias quad of the tile wave v finalises (t = v; every phase here has <= 4 tiles)
template <int CB, int RB>
__device__ __forceinline__ float4 bias_quad(const float* b, int cb0) {
  const int tid = otid(), v = tid >> 6, lane = tid & 63;
  if (v >= CB * RB) return make_float4(0.f, 0.f, 0.f, 0.f);
  return *reinterpret_cast<const float4*>(b + 16 * (cb0 + v / RB) + 4 * (lane >> 4));
}

// A: ln_1 + c_attn -> q (WS_Q, row-major), k / v into the KV cache at the row's position
template <bool PM>
__device__ __forceinline__ void phase_a(const Args& a, const Rs& rs, int l, int w, const Sm& sm, u32x4_t* wq) {
  constexpr int CB = ACB, RB = ARB, NCG = NCB_Q / CB;
  const int tid = otid(), v = tid >> 6, lane = tid & 63;
  const int cb0 = (w % NCG) * CB, rb0 = (w / NCG) * RB;
  u32x4_t xf[RB * QS];
  if (l == 0) embed_frags<RB>(a, sm, rb0, xf);
  else lda<RB, QS>(rs.xb, KSD, rb0, QS * v, xf);
  if constexpr (PM) ldw<APF, QS>(a.wq[l], KSD, cb0, QS * v, wq);
  u32x4_t wr[CB * QS];
#pragma unroll
  for (int i = 0; i < APF * QS; ++i) wr[i] = wq[i];
  ldw<CB - APF, QS>(a.wq[l], KSD, cb0 + APF, QS * v, wr + APF * QS);
  const float4 bq = bias_quad<CB, RB>(a.bq[l], cb0);
  __builtin_amdgcn_sched_barrier(0);
  ln_apply<RB>(xf, sm, rb0);
  const __amdgpu_buffer_rsrc_t rk = mk(a.kc[l], a.kv_bytes), rv = mk(a.vc[l], a.kv_bytes);
  gemm_tiles<CB, RB>(xf, wr, sm, [&](int, int t, f32x4_t s) {
    const int row = 16 * (rb0 + t % RB) + (lane & 15), col = 16 * (cb0 + t / RB) + 4 * (lane >> 4);
    if (row >= a.R) return;
    const u32x4_t o = u4(make_float4(s[0] + bq.x, s[1] + bq.y, s[2] + bq.z, s[3] + bq.w));
    if (col < D) {
      st16(rs.q, (row * D + col) * 4, o);
    } else {
      const int j = col - D, kv = j >= D, jj = kv ? j - D : j;
      st16(kv ? rv : rk, ((((row * NH + jj / HD) * a.Lmax) + sm.pos[row]) * HD + (jj % HD)) * 4, o);
    }
  });
}

// D: ln_2 + c_fc + gelu_new -> hid (fragment order)
template <bool PM>
__device__ __forceinline__ void phase_d(const Args& a, const Rs& rs, int l, int w, const Sm& sm, u32x4_t* wf) {
  constexpr int CB = DCB, RB = DRB, NCG = NCB_F / CB;
  const int tid = otid(), v = tid >> 6, lane = tid & 63;
  const int cb0 = (w % NCG) * CB, rb0 = (w / NCG) * RB;
  u32x4_t xf[RB * QS];
  lda<RB, QS>(rs.xb, KSD, rb0, QS * v, xf);
  if constexpr (PM) ldw<CB, QS>(a.wf[l], KSD, cb0, QS * v, wf);
  const float4 bq = bias_quad<CB, RB>(a.bfc[l], cb0);
  __builtin_amdgcn_sched_barrier(0);
  ln_apply<RB>(xf, sm, rb0);
  gemm_tiles<CB, RB>(xf, wf, sm, [&](int, int t, f32x4_t s) {
    const int row = 16 * (rb0 + t % RB) + (lane & 15), col = 16 * (cb0 + t / RB) + 4 * (lane >> 4);
    if (row >= a.R) return;
    st16(rs.hid, frag_off(row, col, KSF),
         u4(make_float4(act_apply(s[0] + bq.x, ACT_GELU_TANH), act_apply(s[1] + bq.y, ACT_GELU_TANH),
                        act_apply(s[2] + bq.z, ACT_GELU_TANH), act_apply(s[3] + bq.w, ACT_GELU_TANH))));
  });
}

// C / E: projection + residual; the C / E tile is one 16 x 16 block per workgroup, finalised by
// wave 0, whose lanes hold the residual quad across the step (persistent) -- the phase launches
// read it back from xb (the f32 stream itself: no separate copy)
__device__ __forceinline__ void ce_tile(int w, int& row, int& col) {
  constexpr int NCG = NCB_D / ECB;
  const int lane = otid() & 63;
  row = 16 * ((w / NCG) * ERB) + (lane & 15);
  col = 16 * ((w % NCG) * ECB) + 4 * (lane >> 4);
}
template <bool PM>
__device__ __forceinline__ void ce_operands(const Args& a, const Rs& rs, const Sm& sm, bool embed, int w,
                                            const float* bias, const f32x4_t& xo, float4& b, float4& xold) {
  const int v = otid() >> 6;
  b = make_float4(0.f, 0.f, 0.f, 0.f);
  xold = b;
  if (v == 0) {
    int row, col;
    ce_tile(w, row, col);
    b = *reinterpret_cast<const float4*>(bias + col);
    if (embed) xold = embed_quad(a, sm, row, col);
    else if constexpr (PM) xold = f4(ld16(rs.xb, frag_off(row, col, KSD)));
    else xold = make_float4(xo[0], xo[1], xo[2], xo[3]);
  }
}
__device__ __forceinline__ void ce_epilogue(const Args& a, const Rs& rs, int w, f32x4_t s, const float4& b,
                                            const float4& xold, f32x4_t& xo) {
  int row, col;
  ce_tile(w, row, col);
  const f32x4_t o{(s[0] + b.x) + xold.x, (s[1] + b.y) + xold.y, (s[2] + b.z) + xold.z, (s[3] + b.w) + xold.w};
  xo = o;
  if (row < a.R) st16(rs.xb, frag_off(row, col, KSD), u4(make_float4(o[0], o[1], o[2], o[3])));
}
template <bool PM>
__device__ __forceinline__ void phase_c(const Args& a, const Rs& rs, int l, int w, const Sm& sm, u32x4_t* wo,
                                        f32x4_t& xo) {
  constexpr int NCG = NCB_D / ECB;
  const int v = otid() >> 6;
  const int cb0 = (w % NCG) * ECB, rb0 = (w / NCG) * ERB;
  u32x4_t af[QS];
  lda<1, QS>(rs.att, KSD, rb0, QS * v, af);
  if constexpr (PM) ldw<1, QS>(a.wo[l], KSD, cb0, QS * v, wo);
  float4 b, xold;
  ce_operands<PM>(a, rs, sm, l == 0, w, a.bo[l], xo, b, xold);
  __builtin_amdgcn_sched_barrier(0);
  gemm_tiles<1, 1>(af, wo, sm, [&](int, int, f32x4_t s) { ce_epilogue(a, rs, w, s, b, xold, xo); });
}
// E: K = 3072, the quarter's 48 k-steps streamed in chunks of ECH, ESL in flight (wm: the first
// ESL chunks' weights, prefetched across the barrier or loaded here (PM))
template <bool PM>
__device__ __forceinline__ void phase_e(const Args& a, const Rs& rs, int l, int w, const Sm& sm, u32x4_t* wm,
                                        f32x4_t& xo) {
  constexpr int NCG = NCB_D / ECB, NCH = QF / ECH;
  const int v = otid() >> 6;
  const int cb0 = (w % NCG) * ECB, rb0 = (w / NCG) * ERB, s0 = QF * v;
  if constexpr (PM) ldw<1, ESL * ECH>(a.wm[l], KSF, cb0, s0, wm);
  u32x4_t af[ESL * ECH];
  lda<1, ESL * ECH>(rs.hid, KSF, rb0, s0, af);
  float4 b, xold;
  ce_operands<PM>(a, rs, sm, false, w, a.bm[l], xo, b, xold);
  __builtin_amdgcn_sched_barrier(0);
  f32x4_t acc[1] = {f32x4_t{0.f, 0.f, 0.f, 0.f}};
  static_for<NCH>([&](auto cc) {
    constexpr int c = decltype(cc)::value, sl = c % ESL;
#pragma unroll
    for (int s = 0; s < ECH; ++s) acc[0] = mfma4(wm[sl * ECH + s], af[sl * ECH + s], acc[0]);
    if constexpr (c + ESL < NCH) {
      ldw<1, ECH>(a.wm[l], KSF, cb0, s0 + ECH * (c + ESL), wm + sl * ECH);
      lda<1, ECH>(rs.hid, KSF, rb0, s0 + ECH * (c + ESL), af + sl * ECH);
      __builtin_amdgcn_sched_barrier(0);
    }
  });
  reduce_tiles<1>(sm.red, acc, [&](int, int, f32x4_t s) { ce_epilogue(a, rs, w, s, b, xold, xo); });
}

// B: attention, unit u = (row u / 12, head u % 12), one per wave; 8 lanes per key (lane sub holds
// dims 8 sub .. + 8: two 16-byte halves), 8 key groups, chunks of 32 keys, online softmax in f32
// starting from the new key, as the bf16 phase_b
__device__ __forceinline__ void attn_unit(const Args& a, const Sm& sm, int u, int& row, int& hh, int& p,
                                          long& base) {
  row = u / NH;
  hh = u % NH;
  const int rr = min(row, a.R - 1);
  p = min(sm.pos[rr], a.Lmax - 1);
  base = ((long)(rr * NH + hh) * a.Lmax) * HD + 8 * ((otid() & 63) & 7);
}
__device__ __forceinline__ void attn_load(const Args& a, int l, const Sm& sm, int ub, int cb,
                                          u32x4_t (&kr)[KC][2], u32x4_t (&vr)[KC][2]) {
  const int tid = otid(), v = tid >> 6, grp = (tid & 63) >> 3;
  int row, hh, p;
  long base;
  attn_unit(a, sm, ub + v, row, hh, p, base);
#pragma unroll
  for (int i = 0; i < KC; ++i) {
    const int jc = max(min(cb + 8 * i + grp, p - 1), 0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      kr[i][h] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(a.kc[l] + base + (long)jc * HD + 4 * h));
      vr[i][h] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(a.vc[l] + base + (long)jc * HD + 4 * h));
    }
  }
}
__device__ __forceinline__ void phase_b(const Args& a, const Rs& rs, int l, const Sm& sm, int ub,
                                        u32x4_t (&kr)[KC][2], u32x4_t (&vr)[KC][2]) {
  const int tid = otid(), lane = tid & 63, v = tid >> 6, grp = lane >> 3, sub = lane & 7;
  const __amdgpu_buffer_rsrc_t rk = mk(a.kc[l], a.kv_bytes), rv = mk(a.vc[l], a.kv_bytes);
  int row, hh, p;
  long base;
  attn_unit(a, sm, ub + v, row, hh, p, base);
  u32x4_t qu[2], knu[2], vnu[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    qu[h] = ld16(rs.q, (min(row, a.R - 1) * D + hh * HD + 8 * sub + 4 * h) * 4);
    const int off = (int)((base + (long)p * HD + 4 * h) * 4);
    knu[h] = ld16(rk, off);
    vnu[h] = ld16(rv, off);
  }
  __builtin_amdgcn_sched_barrier(0);
  const float4 q0 = f4(qu[0]), q1 = f4(qu[1]);
  auto qk = [&](const u32x4_t (&kv)[2]) {
    const float4 k0 = f4(kv[0]), k1 = f4(kv[1]);
    float sv = q0.x * k0.x;
    sv = fmaf(q0.y, k0.y, sv); sv = fmaf(q0.z, k0.z, sv); sv = fmaf(q0.w, k0.w, sv);
    sv = fmaf(q1.x, k1.x, sv); sv = fmaf(q1.y, k1.y, sv); sv = fmaf(q1.z, k1.z, sv); sv = fmaf(q1.w, k1.w, sv);
    return sum8(sv) * 0.125f;
  };
  float m = qk(knu), sum = grp == 0 ? 1.f : 0.f;
  f32x2_t o[4];
  {
    const float4 v0 = f4(vnu[0]), v1 = f4(vnu[1]);
    const bool g0 = grp == 0;
    o[0] = g0 ? f32x2_t{v0.x, v0.y} : f32x2_t{0.f, 0.f};
    o[1] = g0 ? f32x2_t{v0.z, v0.w} : f32x2_t{0.f, 0.f};
    o[2] = g0 ? f32x2_t{v1.x, v1.y} : f32x2_t{0.f, 0.f};
    o[3] = g0 ? f32x2_t{v1.z, v1.w} : f32x2_t{0.f, 0.f};
  }
  // loads in chunks of 8 KC keys; the online softmax steps 32 keys at a time
  for (int cb = 0; cb < p; cb += 8 * KC) {
    if (cb > 0) attn_load(a, l, sm, ub, cb, kr, vr);
#pragma unroll
    for (int hq = 0; hq < KC / 4; ++hq) {
      const int cs = cb + 32 * hq;
      if (cs >= p) break;                          // wave-uniform
      float sc[4];
      float pm = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float sv = qk(kr[4 * hq + i]);
        sc[i] = cs + 8 * i + grp < p ? sv : -INFINITY;
        pm = fmaxf(pm, sc[i]);
      }
      pm = fmaxf(pm, xor8(pm));
      pm = max16(pm);
      pm = max32(pm);
      const float mn = fmaxf(m, pm);
      const float scale = __expf(m - mn);
      sum *= scale;
      const f32x2_t sc2 = {scale, scale};
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] *= sc2;
      m = mn;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = __expf(sc[i] - mn);
        sum += e;
        const f32x2_t e2 = {e, e};
        const float4 v0 = f4(vr[4 * hq + i][0]), v1 = f4(vr[4 * hq + i][1]);
        o[0] = __builtin_elementwise_fma(e2, f32x2_t{v0.x, v0.y}, o[0]);
        o[1] = __builtin_elementwise_fma(e2, f32x2_t{v0.z, v0.w}, o[1]);
        o[2] = __builtin_elementwise_fma(e2, f32x2_t{v1.x, v1.y}, o[2]);
        o[3] = __builtin_elementwise_fma(e2, f32x2_t{v1.z, v1.w}, o[3]);
      }
    }
  }
  const float inv = 1.0f / add32(add16(sum + xor8(sum)));
  float of[8];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    of[2 * t] = add32(add16(o[t].x + xor8(o[t].x))) * inv;
    of[2 * t + 1] = add32(add16(o[t].y + xor8(o[t].y))) * inv;
  }
  if (grp == 0 && row < a.R) {
    const int c0 = hh * HD + 8 * sub;
    st16(rs.att, frag_off(row, c0, KSD), u4(make_float4(of[0], of[1], of[2], of[3])));
    st16(rs.att, frag_off(row, c0 + 4, KSD), u4(make_float4(of[4], of[5], of[6], of[7])));
  }
}

// F: ln_f + LM head.  Workgroup w takes row half h = (w / 8) % 2 (row blocks 2 h .. + 2) and vocab
// blocks wh + 96 i, wh = w % 8 + 8 (w / 16); per block each wave multiplies its K quarter into
// the 32 rows, the 4 partial tiles go through double-buffered slabs, waves 0 / 1 finalise row
// block 2 h + v.  A ring of 2 blocks of weights per wave is in flight.
__device__ __forceinline__ void phase_f(const Args& a, const Rs& rs, int w, const Sm& sm, gu64* keys) {
  const int tid = otid(), v = tid >> 6, lane = tid & 63;
  // the two workgroups of a vocab block (one per row half) are w and w + 8: the same XCD under
  // round-robin dispatch, so the second read of the block hits that XCD's L2
  const int half = (w >> 3) & 1, wh = (w & 7) + 8 * (w >> 4), rb0 = 2 * half;
  u32x4_t xf[2 * QS];
  lda<2, QS>(rs.xb, KSD, rb0, QS * v, xf);
  const int nvb = (a.V + 15) >> 4;
  const int nb = (nvb - wh + FH - 1) / FH;
  // ring of 2 block slots: this wave's 12 fragments of the block and the lane's 4 per-token biases
  struct Slot {
    u32x4_t w[QS];
    float4 b;
  };
  Slot R0, R1;
  auto fill = [&](int i, Slot& r) {
    const int blk = wh + FH * min(i, nb - 1);
    ldw<1, QS>(a.wtep, KSD, blk, QS * v, r.w);
    r.b = *reinterpret_cast<const float4*>(a.lmb + 16 * blk + 4 * (lane >> 4));
  };
  fill(0, R0);
  fill(1, R1);
  __builtin_amdgcn_sched_barrier(0);
  ln_apply<2>(xf, sm, rb0);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  const bool tmp = a.temp != 1.0f;
  int buf = 0;
  auto consume = [&](int i, const Slot& r) {
    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < QS; ++s)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) acc[rb] = mfma4(r.w[s], xf[rb * QS + s], acc[rb]);
    f32x4_t* red = sm.red + buf * 512;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) red[(v * 2 + rb) * 64 + lane] = acc[rb];
    lds_sync();
    if (v < 2) {
      const f32x4_t sum = (red[v * 64 + lane] + red[(2 + v) * 64 + lane]) +
                          (red[(4 + v) * 64 + lane] + red[(6 + v) * 64 + lane]);
      const int col0 = 16 * (wh + FH * i) + 4 * (lane >> 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lg = sum[e] + (e == 0 ? r.b.x : e == 1 ? r.b.y : e == 2 ? r.b.z : r.b.w);
        const float val = tmp ? lg / a.temp : lg;
        if (col0 + e < a.V && val > bv) { bv = val; bi = col0 + e; }
      }
    }
    buf ^= 1;
  };
#pragma nounroll
  for (int i = 0; i < nb; i += 2) {
    consume(i, R0);
    fill(i + 2, R0);
    if (i + 1 < nb) consume(i + 1, R1);     // (wave-uniform)
    fill(i + 3, R1);
  }
  if (v < 2) {
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane < 16) {
      const unsigned long long key = ((unsigned long long)f2key(bv) << 32) | (unsigned)(~bi);
      __hip_atomic_fetch_max(keys + 16 * (rb0 + v) + lane, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ __launch_bounds__(NT, 2) void dg32_persist_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) char smem[SM_TOTAL32];
  const Sm sm(smem);
  const int w = blockIdx.x;
  if (a.all_done[0]) return;
  int step = *a.step_ctr;
  if (step >= a.max_steps) return;
  load_state(a, sm);
  __syncthreads();
  const Rs rs = make_rs(a.ws);
  Bar bar{(gu32*)(a.ws + WS_SH), (gu32*)(a.ws + WS_TMO), 0, G / NSH, a.spin_max, nullptr, 0};
  gu64* const keys = (gu64*)(a.ws + WS_KEY);
  volatile lds_int_t* s_ok = (volatile lds_int_t*)(sm.misc + 8);
  unsigned long long* const stamps =       // (diagnostic stamps, as the bf16 kernel)
      (dp_stamp_ws == nullptr || dp_stamp_ws == a.ws) ? dp_stamp_buf : nullptr;
  const int stamp_step = dp_stamp_step;
  const int ub = w * UPG;
  constexpr int ANCG = NCB_Q / ACB, DNCG = NCB_F / DCB, ENCG = NCB_D / ECB;
  const int acb0 = (w % ANCG) * ACB, dcb0 = (w % DNCG) * DCB, ecb0 = (w % ENCG) * ECB;
#define V_ (otid() >> 6)
  u32x4_t wq[APF * QS];
  ldw<APF, QS>(a.wq[0], KSD, acb0, QS * V_, wq);
  f32x4_t xo{0.f, 0.f, 0.f, 0.f};
  for (;;) {
    bar.sb = (stamps != nullptr && step == stamp_step) ? stamps + (long)w * 2 * DP_NB : nullptr;
    bar.n0 = bar.n;
    stamp(bar.sb, 2 * DP_NB - 1);
    if (step == a.abort_step) return gave_up(a);
    for (int l = 0; l < NLY; ++l) {
      phase_a<false>(a, rs, l, w, sm, wq);
      bar_arrive(bar, w);
      u32x4_t kr[KC][2], vr[KC][2];
      attn_load(a, l, sm, ub, 0, kr, vr);
      if (!bar_wait(bar, s_ok)) return gave_up(a);
      if (l == 0 && w == 0 && otid() < RM)
        __hip_atomic_store(keys + ((step + 1) & 1) * RM + otid(), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      phase_b(a, rs, l, sm, ub, kr, vr);
      bar_arrive(bar, w);
      u32x4_t wo[QS];
      ldw<1, QS>(a.wo[l], KSD, ecb0, QS * V_, wo);
      if (!bar_wait(bar, s_ok)) return gave_up(a);
      phase_c<false>(a, rs, l, w, sm, wo, xo);
      bar_arrive(bar, w);
      u32x4_t wf[DCB * QS];
      ldw<DCB, QS>(a.wf[l], KSD, dcb0, QS * V_, wf);
      if (!bar_wait(bar, s_ok)) return gave_up(a);
      phase_d<false>(a, rs, l, w, sm, wf);
      bar_arrive(bar, w);
      u32x4_t wm[ESL * ECH];
      ldw<1, ESL * ECH>(a.wm[l], KSF, ecb0, QF * V_, wm);
      if (!bar_wait(bar, s_ok)) return gave_up(a);
      phase_e<false>(a, rs, l, w, sm, wm, xo);
      bar_arrive(bar, w);
      // (the last layer's branch overwrites wq too: otherwise the merge keeps A's operands live
      // through B .. E of every layer, and the register allocator spills them)
      if (l + 1 < NLY) ldw<APF, QS>(a.wq[l + 1], KSD, acb0, QS * V_, wq);
      else for (int i = 0; i < APF * QS; ++i) wq[i] = u32x4_t{0u, 0u, 0u, 0u};
      if (!bar_wait(bar, s_ok)) return gave_up(a);
    }
    phase_f(a, rs, w, sm, keys + (step & 1) * RM);
    bar_arrive(bar, w);
    ldw<APF, QS>(a.wq[0], KSD, acb0, QS * V_, wq);
    if (!bar_wait(bar, s_ok)) return gave_up(a);
    bookkeep(a, sm, keys + (step & 1) * RM, step, w == 0);
    __syncthreads();
    stamp(bar.sb, 2 * DP_NB - 2);
    const int total = sm.misc[0];
    const bool fin = total == 0 || step + 1 >= a.max_steps;
    if (w == 0 && otid() == 0) {
      *a.step_ctr = step + 1;
      a.all_done[2] = total;
      if (fin) a.all_done[0] = 1;
    }
    if (fin) return;
    ++step;
    __syncthreads();
  }
#undef V_
}

template <int PH>
__global__ __launch_bounds__(NT, 2) void dg32_phase_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) char smem[SM_TOTAL32];
  const Sm sm(smem);
  const int w = blockIdx.x, l = a.layer;
  if (a.all_done[0]) return;
  if (*a.step_ctr >= a.max_steps) return;
  load_state(a, sm);
  __syncthreads();
  const Rs rs = make_rs(a.ws);
  if constexpr (PH == PH_A) {
    u32x4_t wq[APF * QS];
    phase_a<true>(a, rs, l, w, sm, wq);
  } else if constexpr (PH == PH_B) {
    u32x4_t kr[KC][2], vr[KC][2];
    attn_load(a, l, sm, w * UPG, 0, kr, vr);
    phase_b(a, rs, l, sm, w * UPG, kr, vr);
  } else if constexpr (PH == PH_C) {
    u32x4_t wo[QS];
    f32x4_t xo{0.f, 0.f, 0.f, 0.f};
    phase_c<true>(a, rs, l, w, sm, wo, xo);
  } else if constexpr (PH == PH_D) {
    u32x4_t wf[DCB * QS];
    phase_d<true>(a, rs, l, w, sm, wf);
  } else if constexpr (PH == PH_E) {
    u32x4_t wm[ESL * ECH];
    f32x4_t xo{0.f, 0.f, 0.f, 0.f};
    phase_e<true>(a, rs, l, w, sm, wm, xo);
  } else {
    phase_f(a, rs, w, sm, (gu64*)(a.ws + WS_KEY));
  }
}
}  // namespace f32

}  // namespace dg
}  // namespace zs

using namespace zs;

namespace {
// validation + Args shared by both entry points
int dg_args(dg::Args& a, int R, int Lmax, int max_steps, int stop0, int stop1, int V,
            const void* wte, const void* wpe, const void* wte_packed, float temperature,
            const void* const* layer_w, const float* lm_bias, void* const* kv,
            int* pos, int* next_tok, int* done, int* out_ids, int* out_len, int* step_ctr,
            int* all_done, void* ws, long ws_bytes, int grid) {
  using namespace dg;
  ZS_REQUIRE(grid == 48 || grid == 96 || grid == 192, "zs_gpt2_decode: grid 48, 96 or 192 (got %d)", grid);
  ZS_REQUIRE(R >= 1 && R <= RM, "zs_gpt2_decode: R in 1..%d (got %d)", RM, R);
  ZS_REQUIRE(V >= 16 * grid * 3 && V <= 1 << 24, "zs_gpt2_decode: vocab %d", V);
  ZS_REQUIRE(Lmax >= 2 && max_steps >= 1, "zs_gpt2_decode: Lmax %d max_steps %d", Lmax, max_steps);
  ZS_REQUIRE((long)R * NH * Lmax * HD * 2 < (1L << 31), "zs_gpt2_decode: KV cache too large");
  ZS_REQUIRE(ws && ws_bytes >= WS_BYTES && ((uintptr_t)ws & 255) == 0,
             "zs_gpt2_decode: workspace of %d bytes, 256-byte aligned", WS_BYTES);
  ZS_REQUIRE(temperature > 0.f, "zs_gpt2_decode: temperature %g (> 0)", temperature);
  ZS_REQUIRE(wte_packed && ((uintptr_t)wte_packed & 15) == 0,
             "zs_gpt2_decode: wte_packed null or not 16-byte aligned");
  ZS_REQUIRE(wte && wpe && layer_w && lm_bias && kv && pos && next_tok && done && out_ids &&
             out_len && step_ctr && all_done, "zs_gpt2_decode: null pointer");
  a = Args{};
  a.R = R; a.Lmax = Lmax; a.max_steps = max_steps; a.stop0 = stop0; a.stop1 = stop1; a.V = V;
  a.spin_max = g_dp_spin > 0 ? (unsigned)g_dp_spin : g_dp_spin < 0 ? 0u : SPIN_MAX;
  a.abort_step = g_dp_abort;
  a.exp = g_dg_exp;
  a.dynf = g_dg_dynf;
  a.kv_bytes = R * NH * Lmax * HD * 2;
  a.temp = temperature;
  a.wte = (const bf16_t*)wte; a.wpe = (const bf16_t*)wpe;
  for (int l = 0; l < NLY; ++l) {
    const void* const* p = layer_w + 8 * l;
    for (int k = 0; k < 8; ++k)
      ZS_REQUIRE(p[k] && ((uintptr_t)p[k] & 15) == 0,
                 "zs_gpt2_decode: layer %d pointer %d null or not 16-byte aligned", l, k);
    a.wq[l] = (const bf16_t*)p[0]; a.bq[l] = (const float*)p[1];
    a.wo[l] = (const bf16_t*)p[2]; a.bo[l] = (const float*)p[3];
    a.wf[l] = (const bf16_t*)p[4]; a.bfc[l] = (const float*)p[5];
    a.wm[l] = (const bf16_t*)p[6]; a.bm[l] = (const float*)p[7];
    ZS_REQUIRE(kv[l] && kv[NLY + l] && ((uintptr_t)kv[l] & 127) == 0 && ((uintptr_t)kv[NLY + l] & 127) == 0,
               "zs_gpt2_decode: KV cache pointer of layer %d null or not 128-byte aligned", l);
    a.kc[l] = (bf16_t*)kv[l];
    a.vc[l] = (bf16_t*)kv[NLY + l];
  }
  a.lmb = lm_bias; a.wtep = (const bf16_t*)wte_packed;
  a.pos = pos; a.next_tok = next_tok; a.done = done; a.out_ids = out_ids; a.out_len = out_len;
  a.step_ctr = step_ctr; a.all_done = all_done; a.ws = (char*)ws;
  return 0;
}
}  // namespace

extern "C" int zs_decode_persist_workspace_bytes(void) { return dg::WS_BYTES; }

extern "C" int zs_gpt2_decode_persist(int R, int Lmax, int max_steps, int stop0, int stop1, int V,
                                      const void* wte, const void* wpe, const void* wte_packed,
                                      float temperature, const void* const* layer_w,
                                      const float* lm_bias, void* const* kv,
                                      int* pos, int* next_tok, int* done, int* out_ids,
                                      int* out_len, int* step_ctr, int* all_done, void* ws,
                                      long ws_bytes, int grid, int exclusive, void* stream) {
  dg::Args a;
  const int rc = dg_args(a, R, Lmax, max_steps, stop0, stop1, V, wte, wpe, wte_packed, temperature,
                         layer_w, lm_bias, kv, pos, next_tok, done, out_ids, out_len, step_ctr,
                         all_done, ws, ws_bytes, grid);
  if (rc) return rc;
  // exclusive: dynamic LDS past half a CU's 160 KiB, so no two such workgroups share a CU (the
  // dispatcher otherwise doubles workgroups up on CUs while others idle: tools/placement.py)
  const size_t dyn = exclusive ? (size_t)(dg::EXCL_LDS - dg::SM_TOTAL) : 0;
  static bool attr = false;
  if (exclusive && !attr) {
    ZS_CHECK_HIP(hipFuncSetAttribute((const void*)dg::dg_persist_kernel<48>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, dg::EXCL_LDS - dg::SM_TOTAL));
    ZS_CHECK_HIP(hipFuncSetAttribute((const void*)dg::dg_persist_kernel<96>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, dg::EXCL_LDS - dg::SM_TOTAL));
    ZS_CHECK_HIP(hipFuncSetAttribute((const void*)dg::dg_persist_kernel<192>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, dg::EXCL_LDS - dg::SM_TOTAL));
    attr = true;
  }
  // the barrier shards, timeout word and argmax keys: zeroed before every launch
  ZS_CHECK_HIP(hipMemsetAsync(ws, 0, dg::WS_SYNC_BYTES, S(stream)));
  if (grid == 48) hipLaunchKernelGGL(dg::dg_persist_kernel<48>, dim3(48), dim3(dg::NT), dyn, S(stream), a);
  else if (grid == 96) hipLaunchKernelGGL(dg::dg_persist_kernel<96>, dim3(96), dim3(dg::NT), dyn, S(stream), a);
  else hipLaunchKernelGGL(dg::dg_persist_kernel<192>, dim3(192), dim3(dg::NT), dyn, S(stream), a);
  ZS_LAUNCH_CHECK();
  return 0;
}

namespace {
template <int G>
int dg_phase_step(dg::Args& a, hipStream_t st) {
  using namespace dg;
  for (int l = 0; l < NLY; ++l) {
    a.layer = l;
    hipLaunchKernelGGL((dg_phase_kernel<G, PH_A>), dim3(G), dim3(NT), 0, st, a);
    hipLaunchKernelGGL((dg_phase_kernel<G, PH_B>), dim3(G), dim3(NT), 0, st, a);
    hipLaunchKernelGGL((dg_phase_kernel<G, PH_C>), dim3(G), dim3(NT), 0, st, a);
    hipLaunchKernelGGL((dg_phase_kernel<G, PH_D>), dim3(G), dim3(NT), 0, st, a);
    hipLaunchKernelGGL((dg_phase_kernel<G, PH_E>), dim3(G), dim3(NT), 0, st, a);
  }
  a.layer = 0;
  hipLaunchKernelGGL((dg_phase_kernel<G, PH_F>), dim3(G), dim3(NT), 0, st, a);
  hipLaunchKernelGGL(dg_book_kernel<Args>, dim3(1), dim3(64), 0, st, a);
  ZS_LAUNCH_CHECK();
  return 0;
}
}  // namespace

// `steps` decode steps as phase launches (62 per step), each a no-op once all_done[0] is set
extern "C" int zs_gpt2_decode_phases(int R, int Lmax, int max_steps, int stop0, int stop1, int V,
                                     const void* wte, const void* wpe, const void* wte_packed,
                                     float temperature, const void* const* layer_w,
                                     const float* lm_bias, void* const* kv,
                                     int* pos, int* next_tok, int* done, int* out_ids,
                                     int* out_len, int* step_ctr, int* all_done, void* ws,
                                     long ws_bytes, int steps, int grid, void* stream) {
  dg::Args a;
  const int rc = dg_args(a, R, Lmax, max_steps, stop0, stop1, V, wte, wpe, wte_packed, temperature,
                         layer_w, lm_bias, kv, pos, next_tok, done, out_ids, out_len, step_ctr,
                         all_done, ws, ws_bytes, grid);
  if (rc) return rc;
  ZS_REQUIRE(steps >= 1, "zs_gpt2_decode_phases: steps %d", steps);
  ZS_CHECK_HIP(hipMemsetAsync(ws, 0, dg::WS_SYNC_BYTES, S(stream)));
  for (int s = 0; s < steps; ++s) {
    const int r = grid == 48 ? dg_phase_step<48>(a, S(stream))
                : grid == 96 ? dg_phase_step<96>(a, S(stream)) : dg_phase_step<192>(a, S(stream));
    if (r) return r;
  }
  return 0;
}

// one wave that waits `ticks` of the 100 MHz realtime counter (zs_stream_spin)
__global__ __launch_bounds__(64) void dg_spin_kernel(unsigned long long ticks) {
  unsigned long long t0, t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  do {
    __builtin_amdgcn_s_sleep(32);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  } while (t - t0 < ticks);
}

extern "C" int zs_stream_spin(int us, void* stream) {
  ZS_REQUIRE(us >= 0 && us <= 1000000, "zs_stream_spin: us %d", us);
  if (us == 0) return 0;
  hipLaunchKernelGGL(dg_spin_kernel, dim3(1), dim3(64), 0, S(stream), (unsigned long long)us * 100ull);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_decode_persist_set_stamps(void* buf, int step, const void* ws) {
  ZS_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dg::dp_stamp_buf), &buf, sizeof(buf)));
  ZS_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dg::dp_stamp_ws), &ws, sizeof(ws)));
  ZS_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dg::dp_stamp_step), &step, sizeof(step)));
  return 0;
}

// timeout word of the last launch on this workspace (non-zero: the grid was not co-resident and
// the launch gave up; the state in memory is the last committed step's).  Host-side read.
extern "C" int zs_decode_persist_status(const void* ws, int* timed_out) {
  ZS_REQUIRE(ws && timed_out, "zs_decode_persist_status: null pointer");
  unsigned t = 0;
  ZS_CHECK_HIP(hipMemcpy(&t, (const char*)ws + dg::WS_TMO, 4, hipMemcpyDeviceToHost));
  *timed_out = (int)t;
  return 0;
}

// ------------------------------------------------------------------ f32 parity mode entry points
namespace {
int dg32_args(dg::f32::Args& a, int R, int Lmax, int max_steps, int stop0, int stop1, int V,
              const void* wte, const void* wpe, const void* wte_packed, float temperature,
              const void* const* layer_w, const float* lm_bias, void* const* kv, int* pos,
              int* next_tok, int* done, int* out_ids, int* out_len, int* step_ctr, int* all_done,
              void* ws, long ws_bytes, int grid) {
  using namespace dg;
  ZS_REQUIRE(grid == f32::G, "zs_gpt2_decode_f32: grid %d (got %d)", f32::G, grid);
  ZS_REQUIRE(R >= 1 && R <= RM, "zs_gpt2_decode_f32: R in 1..%d (got %d)", RM, R);
  ZS_REQUIRE(V >= 16 * f32::FH && V <= 1 << 24, "zs_gpt2_decode_f32: vocab %d", V);
  ZS_REQUIRE(Lmax >= 2 && max_steps >= 1, "zs_gpt2_decode_f32: Lmax %d max_steps %d", Lmax, max_steps);
  ZS_REQUIRE((long)R * NH * Lmax * HD * 4 < (1L << 31), "zs_gpt2_decode_f32: KV cache too large");
  ZS_REQUIRE(ws && ws_bytes >= f32::WS_BYTES && ((uintptr_t)ws & 255) == 0,
             "zs_gpt2_decode_f32: workspace of %d bytes, 256-byte aligned", f32::WS_BYTES);
  ZS_REQUIRE(temperature > 0.f, "zs_gpt2_decode_f32: temperature %g (> 0)", temperature);
  ZS_REQUIRE(wte && wpe && wte_packed && lm_bias && layer_w && kv && pos && next_tok && done &&
             out_ids && out_len && step_ctr && all_done, "zs_gpt2_decode_f32: null pointer");
  ZS_REQUIRE(((uintptr_t)wte & 15) == 0 && ((uintptr_t)wpe & 15) == 0 && ((uintptr_t)wte_packed & 15) == 0 &&
             ((uintptr_t)lm_bias & 15) == 0,
             "zs_gpt2_decode_f32: wte / wpe / wte_packed / lm_bias not 16-byte aligned");
  a = f32::Args{};
  a.R = R; a.Lmax = Lmax; a.max_steps = max_steps; a.stop0 = stop0; a.stop1 = stop1; a.V = V;
  a.spin_max = g_dp_spin > 0 ? (unsigned)g_dp_spin : g_dp_spin < 0 ? 0u : SPIN_MAX;
  a.abort_step = g_dp_abort;
  a.kv_bytes = R * NH * Lmax * HD * 4;
  a.temp = temperature;
  a.wte = (const float*)wte; a.wpe = (const float*)wpe; a.wtep = (const float*)wte_packed;
  a.lmb = lm_bias;
  for (int l = 0; l < NLY; ++l) {
    const void* const* p = layer_w + 8 * l;
    for (int k = 0; k < 8; ++k)
      ZS_REQUIRE(p[k] && ((uintptr_t)p[k] & 15) == 0,
                 "zs_gpt2_decode_f32: layer %d pointer %d null or not 16-byte aligned", l, k);
    a.wq[l] = (const float*)p[0]; a.bq[l] = (const float*)p[1];
    a.wo[l] = (const float*)p[2]; a.bo[l] = (const float*)p[3];
    a.wf[l] = (const float*)p[4]; a.bfc[l] = (const float*)p[5];
    a.wm[l] = (const float*)p[6]; a.bm[l] = (const float*)p[7];
    ZS_REQUIRE(kv[l] && kv[NLY + l] && ((uintptr_t)kv[l] & 127) == 0 && ((uintptr_t)kv[NLY + l] & 127) == 0,
               "zs_gpt2_decode_f32: KV cache pointer of layer %d null or not 128-byte aligned", l);
    a.kc[l] = (float*)kv[l];
    a.vc[l] = (float*)kv[NLY + l];
  }
  a.pos = pos; a.next_tok = next_tok; a.done = done; a.out_ids = out_ids; a.out_len = out_len;
  a.step_ctr = step_ctr; a.all_done = all_done; a.ws = (char*)ws;
  return 0;
}
}  // namespace

extern "C" int zs_decode_persist_f32_workspace_bytes(void) { return dg::f32::WS_BYTES; }

extern "C" int zs_gpt2_decode_persist_f32(int R, int Lmax, int max_steps, int stop0, int stop1, int V,
                                          const void* wte, const void* wpe, const void* wte_packed,
                                          float temperature, const void* const* layer_w,
                                          const float* lm_bias, void* const* kv, int* pos,
                                          int* next_tok, int* done, int* out_ids, int* out_len,
                                          int* step_ctr, int* all_done, void* ws, long ws_bytes,
                                          int grid, int exclusive, void* stream) {
  dg::f32::Args a;
  const int rc = dg32_args(a, R, Lmax, max_steps, stop0, stop1, V, wte, wpe, wte_packed, temperature,
                           layer_w, lm_bias, kv, pos, next_tok, done, out_ids, out_len, step_ctr,
                           all_done, ws, ws_bytes, grid);
  if (rc) return rc;
  const size_t dyn = exclusive ? (size_t)(dg::EXCL_LDS - dg::f32::SM_TOTAL32) : 0;
  static bool attr = false;
  if (exclusive && !attr) {
    ZS_CHECK_HIP(hipFuncSetAttribute((const void*)dg::f32::dg32_persist_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     dg::EXCL_LDS - dg::f32::SM_TOTAL32));
    attr = true;
  }
  ZS_CHECK_HIP(hipMemsetAsync(ws, 0, dg::WS_SYNC_BYTES, S(stream)));
  hipLaunchKernelGGL(dg::f32::dg32_persist_kernel, dim3(dg::f32::G), dim3(dg::NT), dyn, S(stream), a);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_gpt2_decode_phases_f32(int R, int Lmax, int max_steps, int stop0, int stop1, int V,
                                         const void* wte, const void* wpe, const void* wte_packed,
                                         float temperature, const void* const* layer_w,
                                         const float* lm_bias, void* const* kv, int* pos,
                                         int* next_tok, int* done, int* out_ids, int* out_len,
                                         int* step_ctr, int* all_done, void* ws, long ws_bytes,
                                         int steps, int grid, void* stream) {
  using namespace dg;
  f32::Args a;
  const int rc = dg32_args(a, R, Lmax, max_steps, stop0, stop1, V, wte, wpe, wte_packed, temperature,
                           layer_w, lm_bias, kv, pos, next_tok, done, out_ids, out_len, step_ctr,
                           all_done, ws, ws_bytes, grid);
  if (rc) return rc;
  ZS_REQUIRE(steps >= 1, "zs_gpt2_decode_phases_f32: steps %d", steps);
  const hipStream_t st = S(stream);
  ZS_CHECK_HIP(hipMemsetAsync(ws, 0, WS_SYNC_BYTES, st));
  for (int s = 0; s < steps; ++s) {
    for (int l = 0; l < NLY; ++l) {
      a.layer = l;
      hipLaunchKernelGGL(f32::dg32_phase_kernel<PH_A>, dim3(f32::G), dim3(NT), 0, st, a);
      hipLaunchKernelGGL(f32::dg32_phase_kernel<PH_B>, dim3(f32::G), dim3(NT), 0, st, a);
      hipLaunchKernelGGL(f32::dg32_phase_kernel<PH_C>, dim3(f32::G), dim3(NT), 0, st, a);
      hipLaunchKernelGGL(f32::dg32_phase_kernel<PH_D>, dim3(f32::G), dim3(NT), 0, st, a);
      hipLaunchKernelGGL(f32::dg32_phase_kernel<PH_E>, dim3(f32::G), dim3(NT), 0, st, a);
    }
    a.layer = 0;
    hipLaunchKernelGGL(f32::dg32_phase_kernel<PH_F>, dim3(f32::G), dim3(NT), 0, st, a);
    hipLaunchKernelGGL(dg_book_kernel<f32::Args>, dim3(1), dim3(64), 0, st, a);
    ZS_LAUNCH_CHECK();
  }
  return 0;
}

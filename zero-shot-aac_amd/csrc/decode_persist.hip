// GPT-2 greedy decode of ONE eval batch (R <= 64 rows, the reference's bs = 64) as ONE persistent
// launch: every remaining step of generate2 (gpt2_prefix_eval.py:161-222 over transformers'
// GPT2LMHeadModel with a KV cache) -- 12 blocks, ln_f, the LM head with its argmax and the stop /
// length bookkeeping -- runs inside the kernel, from the step after the prefill to the last one.
//
// Why: at 64 rows a decode step is ~390 MB of weight + KV-cache reads spread over ~63 dependent
// launches of 1-5 MB each; each launch spends most of its 5-9 us on the kernel boundary and on
// issuing its first weight loads.  Here a fixed set of G workgroups (one per CU)
// owns a fixed slice of every GEMM's columns and of the (row, head) attention units for the whole
// decode.  A phase's inputs arrive through a grid barrier, and the weights of the NEXT phase
// (activation independent) are issued into registers BEFORE the workgroup waits on that barrier,
// so the weight stream overlaps the hand-off instead of following a kernel boundary.
//
// The launch uses G of the chip's 256 CUs, so several eval batches decode at once on disjoint CUs
// (ConcurrentRunner streams): the chip is filled by independent bs = 64 batches, never by merging
// their rows into one GEMM.
//
// Phases of one step (WG w of G = 48, 8 waves; "sc1" = write-through stores / L1-bypassing loads,
// MI355X_MICROARCH.md § Workgroup dispatch, Valid forms row 1):
//   A  ln_1 + c_attn: x [64][768] f32 -> LN (affine folded into W, as the bf16 zs_gemm_ln path)
//      -> bf16 rows in LDS -> qkv[:, 48w .. 48w+48) (bf16); layer 0 embeds wte[tok] + wpe[pos].
//   B  attention: units (row, head) 16w .. 16w+16 (two per wave), keys 0..pos from the cache plus
//      the new k / v from qkv, appended to the cache; out att [64][768] bf16.
//   C  attn.c_proj + residual: x[:, 16w .. 16w+16) += att W^T + b.
//   D  ln_2 + mlp.c_fc + gelu_new: hid[:, 64w .. 64w+64) (bf16).
//   E  mlp.c_proj + residual: x[:, 16w .. 16w+16) += hid W^T + b.
//   F  (after the 12 blocks) ln_f + LM head over vocab rows [wV/G, (w+1)V/G): per row the best
//      (logit, id) of the slice.
//   G  every WG merges the G slices per row (ties -> lower id, torch.argmax) and applies
//      greedy_step's bookkeeping to its LDS copy of (token, position, done); WG 0 writes the
//      state / ids.  Rows past R compute garbage that is never stored.
// Barriers: 5 per block + 1 after F = 61 per step (one monotonic agent-scope counter).
#include <type_traits>

#include "common.h"

namespace zs {
int g_dp_lmil = 1;   // zs_tune_set("dp_lmil", 0): LM-head vocab as one contiguous range per workgroup (A/B)
int g_dp_nt = 2;   // the cached K/V are read non-temporally (round 3 A/B); nt
                   // weight / LM-head loads were slower: the concurrent grids share the weights
                   // through L2 / MALL.  (kept for zs_tune_set compatibility; no other value)
int g_dp_fuse = 0; // zs_tune_set("dp_fuse", 1): the MLP as D' + R (partial sums; measured slower)
int g_dp_spin = 0; // zs_tune_set("dp_spin", n): give up a grid-barrier wait after n polls (0 = the
                   // default 2^22, < 0: at the first unmet poll); tests/test_gpu_persist.py forces
                   // the give-up path with it
namespace dpk {

constexpr int D = 768, NH = 12, HD = 64, DFF = 3072, NLY = 12, RM = 64, QKVN = 3 * D;
constexpr int G = 48;                  // workgroups per batch at CS = 1, one per CU
// CS column slices per workgroup: the grid of one batch is GW = 48 / CS column-slice workgroups
// (x RH row halves).  CS = 2 halves the CUs a batch holds: every workgroup still reads the whole
// handed-off activation once per phase (the same bytes as at CS = 1) but streams twice the
// weight columns, so the CU-time per step falls while the step grows by the weight share only.
template <int CS>
struct Geo {
  static constexpr int GW = G / CS;      // column-slice workgroups
  static constexpr int QN = 48 * CS;     // c_attn columns per workgroup
  static constexpr int PN = 16 * CS;     // attn.c_proj / mlp.c_proj columns
  static constexpr int FN = 64 * CS;     // c_fc columns
  static constexpr int A_KP = 8 / CS;    // phase A waves: A_KP K parts x CS groups of 3 blocks
  static constexpr int SA = 24 / A_KP;   // k-steps per wave in phase A
  static constexpr int D_KP = 4 / CS;    // phase D waves: D_KP K parts x 2 CS groups of 2 blocks
  static constexpr int SD = 24 / D_KP;   // k-steps per wave in phase D
};
constexpr int NW = 8, NT = 64 * NW;    // 8 waves
constexpr int HLD = D + 8;             // bf16 row stride of the normalised rows in LDS
constexpr unsigned SPIN_MAX = 1u << 22;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

// workspace (bytes): the sync block first, zeroed by the launcher before every launch:
//   [0] barrier counter, [4] timeout word, [256..1280) per-row LM-head argmax keys, two step parities
// att and hid are stored in MFMA A-fragment order ([4 row blocks][K/32 k-steps][64 lanes][8]), so
// every A-fragment load of the consuming projection is one contiguous KiB per wave-instruction
constexpr int WS_SYNC = 0;
constexpr int WS_LMKEY = 256;                      // u64  [2][64]
constexpr int WS_SYNC_BYTES = 1280;
constexpr int WS_X = WS_SYNC_BYTES;                // f32  [64][768]
constexpr int WS_QKV = WS_X + RM * D * 4;          // bf16 [64][2304]
constexpr int WS_ATT = WS_QKV + RM * QKVN * 2;     // bf16 fragment-packed [4][24][64][8]
constexpr int WS_HID = WS_ATT + RM * D * 2;        // bf16 fragment-packed [4][96][64][8]
constexpr int WS_XB = WS_HID + RM * DFF * 2;       // bf16 [64][768]: x for the LayerNorms
// fused MLP (FUSE): each workgroup's mlp.c_proj partial sums over its own c_fc columns, in MFMA
// accumulator-tile order [producer w'][row half h][column slice j][row block rb][block bi][64
// lanes][4] (bf16, PART_BF16, or f32), read back by the slice's owner in phase R; sized for the
// 48-workgroup grids (the 24-workgroup grid uses half)
constexpr int PART_BF16 = 1;
constexpr int PART_EB = PART_BF16 ? 8 : 16;       // bytes per lane per tile
constexpr int WS_PART = WS_XB + RM * D * 2;
constexpr int WS_BYTES = WS_PART + G * RM * D * (PART_BF16 ? 2 : 4);

struct Args {
  int R, Lmax, max_steps, stop0, stop1, V, lm_il;
  unsigned spin_max;    // polls before a barrier wait gives up
  const bf16_t* wte; const bf16_t* wpe;
  const bf16_t* wqkv[NLY]; const float* bqkv[NLY];
  const bf16_t* wproj[NLY]; const float* bproj[NLY];
  const bf16_t* wfc[NLY]; const float* bfc[NLY];
  const bf16_t* wmp[NLY]; const float* bmp[NLY];
  const float* lnf_w; const float* lnf_b;
  const bf16_t* wtep;   // wte in B-fragment order [ceil(V/16)][24][64][8] (rows past V zero)
  float temp;           // generate2's temperature (logits / temp before the argmax; 1 = none)
  bf16_t* kc[NLY]; bf16_t* vc[NLY];
  int* pos; int* next_tok; int* done; int* out_ids; int* out_len; int* step_ctr; int* all_done;
  char* ws;
};

// LDS: normalised rows [64][HLD] bf16, aliased by the GEMM partial slabs (<= 98,304 B); argmax
// merge; per-row decode state
constexpr int SM_HS = RM * HLD * 2;
constexpr int SM_AM = 2 * NW * RM * 4;
constexpr int SM_ST = 4 * RM * 4 + 64;
constexpr int SM_LNF = 2 * D * 4;                 // ln_f weight / bias
constexpr int SM_TOTAL = SM_HS + SM_AM + SM_ST + SM_LNF;
static_assert(NW * RM * 48 * 4 <= SM_HS, "QKV partial slabs fit the aliased row buffer");

// ------------------------------------------------------------------ memory helpers
struct Rs {
  __amdgpu_buffer_rsrc_t x, qkv, att, hid, xb, part;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk(char* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, bytes, 0x00020000);
}
// aux 16 = sc1: stores write through (no release fence needed), loads bypass this CU's L1
__device__ __forceinline__ u32x4_t ld16(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}
__device__ __forceinline__ u32x2_t ld8(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 16);
}
__device__ __forceinline__ unsigned ld4(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 16);
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, int off, u32x4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
__device__ __forceinline__ void st8(__amdgpu_buffer_rsrc_t r, int off, u32x2_t v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, 16);
}
__device__ __forceinline__ void st4(__amdgpu_buffer_rsrc_t r, int off, unsigned v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 16);
}
__device__ __forceinline__ float4 u2f4(u32x4_t u) {
  return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z),
                     __uint_as_float(u.w));
}
__device__ __forceinline__ u32x4_t f42u(float a, float b, float c, float d) {
  return u32x4_t{__float_as_uint(a), __float_as_uint(b), __float_as_uint(c), __float_as_uint(d)};
}
__device__ __forceinline__ bf16x8_t bf8(u32x4_t u) { return __builtin_bit_cast(bf16x8_t, u); }
__device__ __forceinline__ f32x4_t mfma(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// threadIdx.x through an empty asm: per-phase lane arithmetic is recomputed in the phase
// instead of being hoisted out of the decode loop by LICM (and spilled: ~200 VGPRs of addresses)
__device__ __forceinline__ int otid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
// in-wave exchanges without LDS: DPP within rows of 16, v_permlane16/32_swap across them
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
// sum over the 8 lanes of each 8-lane group (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror)
__device__ __forceinline__ float sum8(float s) {
  s += dppf<0xB1>(s);
  s += dppf<0x4E>(s);
  return s + dppf<0x141>(s);
}
__device__ __forceinline__ float xor8(float v) { return dppf<0x128>(v); }   // row_ror:8
// v + partner (lane ^ 16 / lane ^ 32), summed in the same order on both lanes
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

// a 16-byte global load, non-temporal (nt: streamed once, evict-first in L2) when NTL
template <bool NTL, typename T>
__device__ __forceinline__ T ldg(const T* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(p);
  else return *p;
}

// weight fragments of NB 16-column blocks x S k-steps (MFMA B operand, W [N][K] row-major);
// only the k-steps [S0, S1) (a prefetch split around a barrier wait)
template <int NB, int S, bool NTL = false, int S0 = 0, int S1 = S>
__device__ __forceinline__ void load_w(const bf16_t* W, int K, int n0, int N, int kbase,
                                       bf16x8_t (&b)[NB * S]) {
  const int lane = otid() & 63, fr = lane & 15, fk = 8 * (lane >> 4);
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const bf16_t* row = W + (long)min(n0 + 16 * nb + fr, N - 1) * K + kbase + fk;
#pragma unroll
    for (int s = S0; s < S1; ++s)
      b[nb * S + s] = ldg<NTL>(reinterpret_cast<const bf16x8_t*>(row + 32 * s));
  }
}

// the blocks [NB0, NB1) of the NB x S fragments load_w would load (a prefetch split by blocks)
template <int NB, int S, int NB0, int NB1, bool NTL = false>
__device__ __forceinline__ void load_w_nb(const bf16_t* W, int K, int n0, int N, int kbase,
                                          bf16x8_t (&b)[NB * S]) {
  const int lane = otid() & 63, fr = lane & 15, fk = 8 * (lane >> 4);
#pragma unroll
  for (int nb = NB0; nb < NB1; ++nb) {
    const bf16_t* row = W + (long)min(n0 + 16 * nb + fr, N - 1) * K + kbase + fk;
#pragma unroll
    for (int s = 0; s < S; ++s)
      b[nb * S + s] = ldg<NTL>(reinterpret_cast<const bf16x8_t*>(row + 32 * s));
  }
}

// ------------------------------------------------------------------ diagnostic stamps
// zs_decode_persist_set_stamps(buf): thread 0 of every workgroup writes s_memrealtime (100 MHz)
// after each barrier arrive and wait of decode step `stamp_step` into buf[w][2 * barrier + {0,1}]
// (tools/persist_stamps.py).  The kernel never reads the buffer; NULL (default) = off.
__device__ unsigned long long* dp_stamp_buf;
__device__ int dp_stamp_step;
#define DP_NB 64                       // stamp slots per (workgroup, step): 61 barriers + spare
__device__ __forceinline__ void stamp(unsigned long long* sb, int slot) {
  if (sb != nullptr && threadIdx.x == 0) {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    ((gu64*)sb)[slot] = t;     // a global (not flat) store
  }
}

// ------------------------------------------------------------------ grid barrier
// Producer side (R1): every storing wave drains its sc1 stores, the workgroup meets, ONE lane adds
// to the counter.  Consumer side: ONE lane polls the counter (relaxed sc1 loads), the workgroup
// meets, then every load of handed-off bytes is an sc1 load.  arrive() and wait() are split so a
// workgroup issues its next phase's weight loads in between.
struct Bar {
  gu32* cnt;
  gu32* tmo;
  unsigned n;
  unsigned long long* sb;   // this workgroup's stamp row of the traced step (or NULL)
  unsigned n0;              // barrier count at the start of the traced step
  unsigned g;               // workgroups in the grid
  unsigned spin_max;        // polls before giving up
};
__device__ __forceinline__ void bar_arrive(Bar& b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(b.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  stamp(b.sb, 2 * (b.n - b.n0));
  ++b.n;
}
typedef __attribute__((address_space(3))) int lds_int_t;
__device__ __forceinline__ bool bar_wait(Bar& b, volatile lds_int_t* s_ok) {
  if (threadIdx.x == 0) {
    const unsigned target = b.n * b.g;
    unsigned spins = 0;
    int ok = 1;
    while (__hip_atomic_load(b.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      ++spins;
      // bounded spin: give up (and tell every other workgroup) after ~2^22 polls, so a grid that
      // is not co-resident drains instead of hanging
      if (spins > b.spin_max ||
          ((spins & 255) == 0 && __hip_atomic_load(b.tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(b.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    *s_ok = ok;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  stamp(b.sb, 2 * (b.n - b.n0) - 1);
  return *s_ok != 0;
}

// ------------------------------------------------------------------ LayerNorm rows -> LDS
// 8 threads per row (row = tid / 8), column quads q + 8i.  MODE 0: x from the workspace;
// 1: the token embedding wte[tok] + wpe[pos] (layer 0; WG w also stores rows r % G == w of x);
// 2: x with the ln_f affine.  The LN affine of ln_1 / ln_2 is folded into c_attn / c_fc.
// NR rows (64, or 32 for a row-split grid) from row r0, TPR = 512 / NR threads per row, NQ column
// quads per thread; rows land at LDS row r - r0.  MODE 1 stores x rows r % gw == w of its range
// (gw = the column-slice workgroups).
struct NoLate {
  __device__ __forceinline__ void operator()() const {}
};
// late(): loads issued right after the handed-off rows' loads (the rest of a weight prefetch
// split around the barrier wait: younger than the rows, so the rows are not waited behind them)
template <int MODE, int NR = RM, bool XB = false, typename Late = NoLate>
__device__ __forceinline__ void ln_rows(const Args& a, const Rs& rs, bf16_t* hs, const int* s_tok,
                                        const int* s_pos, int w, const float* s_lnf = nullptr,
                                        int r0 = 0, int gw = G, Late late = Late()) {
  constexpr int TPR = NT / NR, NQ = D / 4 / TPR;
  const int tid = otid(), rl = tid / TPR, q = tid % TPR, r = r0 + rl;
  const int rr = min(r, a.R - 1);
  if constexpr (XB && MODE != 1) {
    // x handed off in bf16 (the producers' copy, rs.xb): half the bytes of the f32 rows, 16-byte
    // sc1 loads of 8 columns (octets q + TPR i); statistics in f32 over the bf16 values
    constexpr int NO = NQ / 2;
    float xv[NO][8];
    u32x4_t xu[NO];
#pragma unroll
    for (int i = 0; i < NO; ++i) xu[i] = ld16(rs.xb, (rr * D + 8 * (q + TPR * i)) * 2);
    late();
    // all NO loads in flight before the first use (under the LM head's register pressure the
    // compiler otherwise issued them one round trip at a time)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NO; ++i) {
      const u32x4_t u = xu[i];
      xv[i][0] = __uint_as_float(u.x << 16); xv[i][1] = __uint_as_float(u.x & 0xffff0000u);
      xv[i][2] = __uint_as_float(u.y << 16); xv[i][3] = __uint_as_float(u.y & 0xffff0000u);
      xv[i][4] = __uint_as_float(u.z << 16); xv[i][5] = __uint_as_float(u.z & 0xffff0000u);
      xv[i][6] = __uint_as_float(u.w << 16); xv[i][7] = __uint_as_float(u.w & 0xffff0000u);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NO; ++i)
      s += ((xv[i][0] + xv[i][1]) + (xv[i][2] + xv[i][3])) + ((xv[i][4] + xv[i][5]) + (xv[i][6] + xv[i][7]));
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) s += __shfl_xor(s, o, 64);
    const float mean = s * (1.0f / D);
    float qq = 0.f;
#pragma unroll
    for (int i = 0; i < NO; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float d0 = xv[i][t] - mean;
        qq += d0 * d0;
      }
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) qq += __shfl_xor(qq, o, 64);
    const float rstd = rsqrtf(qq * (1.0f / D) + 1e-5f);
#pragma unroll
    for (int i = 0; i < NO; ++i) {
      const int c = 8 * (q + TPR * i);
      float y[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) y[t] = (xv[i][t] - mean) * rstd;
      if constexpr (MODE == 2) {
#pragma unroll
        for (int t = 0; t < 8; ++t) y[t] = y[t] * s_lnf[c + t] + s_lnf[D + c + t];
      }
      *reinterpret_cast<uint4*>(hs + rl * HLD + c) =
          make_uint4(pk2bf(y[0], y[1]), pk2bf(y[2], y[3]), pk2bf(y[4], y[5]), pk2bf(y[6], y[7]));
    }
    return;
  }
  float4 xv[NQ];
  if constexpr (MODE == 1) {
    const bf16_t* te = a.wte + (long)s_tok[r] * D;
    const bf16_t* pe = a.wpe + (long)s_pos[r] * D;
    // halves of NQ / 2 quads (the bf16 pairs of a half are converted before the next is issued)
    constexpr int HQ = NQ / 2;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      uint2 tu[HQ], pu[HQ];
#pragma unroll
      for (int i = 0; i < HQ; ++i) {
        tu[i] = *reinterpret_cast<const uint2*>(te + 4 * (q + TPR * (HQ * hf + i)));
        pu[i] = *reinterpret_cast<const uint2*>(pe + 4 * (q + TPR * (HQ * hf + i)));
      }
#pragma unroll
      for (int i = 0; i < HQ; ++i)
        xv[HQ * hf + i] = make_float4(
            __uint_as_float(tu[i].x << 16) + __uint_as_float(pu[i].x << 16),
            __uint_as_float(tu[i].x & 0xffff0000u) + __uint_as_float(pu[i].x & 0xffff0000u),
            __uint_as_float(tu[i].y << 16) + __uint_as_float(pu[i].y << 16),
            __uint_as_float(tu[i].y & 0xffff0000u) + __uint_as_float(pu[i].y & 0xffff0000u));
      __builtin_amdgcn_sched_barrier(0);
    }
    if (r < a.R && r % gw == w) {
#pragma unroll
      for (int i = 0; i < NQ; ++i)
        st16(rs.x, (r * D + 4 * (q + TPR * i)) * 4, f42u(xv[i].x, xv[i].y, xv[i].z, xv[i].w));
    }
  } else {
#pragma unroll
    for (int i = 0; i < NQ; ++i) xv[i] = u2f4(ld16(rs.x, (rr * D + 4 * (q + TPR * i)) * 4));
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) s += (xv[i].x + xv[i].y) + (xv[i].z + xv[i].w);
#pragma unroll
  for (int o = 1; o < TPR; o <<= 1) s += __shfl_xor(s, o, 64);
  const float mean = s * (1.0f / D);
  float qq = 0.f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const float d0 = xv[i].x - mean, d1 = xv[i].y - mean, d2 = xv[i].z - mean, d3 = xv[i].w - mean;
    qq += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
  }
#pragma unroll
  for (int o = 1; o < TPR; o <<= 1) qq += __shfl_xor(qq, o, 64);
  const float rstd = rsqrtf(qq * (1.0f / D) + 1e-5f);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int c = 4 * (q + TPR * i);
    float y0 = (xv[i].x - mean) * rstd, y1 = (xv[i].y - mean) * rstd;
    float y2 = (xv[i].z - mean) * rstd, y3 = (xv[i].w - mean) * rstd;
    if constexpr (MODE == 2) {   // ln_f params staged in LDS at kernel start (s_lnf)
      const float4 g = *reinterpret_cast<const float4*>(s_lnf + c);
      const float4 bb = *reinterpret_cast<const float4*>(s_lnf + D + c);
      y0 = y0 * g.x + bb.x; y1 = y1 * g.y + bb.y; y2 = y2 * g.z + bb.z; y3 = y3 * g.w + bb.w;
    }
    *reinterpret_cast<uint2*>(hs + rl * HLD + c) = make_uint2(pk2bf(y0, y1), pk2bf(y2, y3));
  }
}

// A fragments from the LDS rows, all 4 row blocks, S k-steps from kbase, NB column blocks
template <int NB, int S, int NRB = 4>
__device__ __forceinline__ void mma_lds(const bf16_t* hs, int kbase, const bf16x8_t (&b)[NB * S],
                                        f32x4_t (&acc)[NRB][NB]) {
  const int lane = otid() & 63, fr = lane & 15, fk = 8 * (lane >> 4);
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[rb][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int rb = 0; rb < NRB; ++rb) {
      const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(hs + (16 * rb + fr) * HLD + kbase + 32 * s + fk);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[rb][nb] = mfma(af, b[nb * S + s], acc[rb][nb]);
    }
}

// partial slab [slab][16 NRB][NC] f32: lane's accumulators of NB column blocks from column col0
template <int NB, int NC, int NRB = 4>
__device__ __forceinline__ void put_partial(float* red, int slab, int col0, const f32x4_t (&acc)[NRB][NB]) {
  const int lane = otid() & 63, fr = lane & 15, r4 = 4 * (lane >> 4);
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        red[(slab * 16 * NRB + 16 * rb + r4 + i) * NC + col0 + 16 * nb + fr] = acc[rb][nb][i];
}

// ------------------------------------------------------------------ phase A: ln_1 + c_attn
// RH = 1: all 64 rows; RH = 2: the 32 rows of half h (row-split grid).  Wave v = (column group
// v / A_KP of 3 blocks, K part v % A_KP); the A_KP partial slabs alias the LN rows (98,304 B at
// every CS).
template <int CS, int RH, bool XB, int RB = 4, typename Late = NoLate>
__device__ __forceinline__ void phase_qkv(const Args& a, const Rs& rs, int l, char* smem,
                                          const int* s_tok, const int* s_pos, int w, int h,
                                          const bf16x8_t (&wq)[3 * Geo<CS>::SA], Late late = Late()) {
  using Gm = Geo<CS>;
  constexpr int NR = 16 * RB / RH, NRB = NR / 16, QN = Gm::QN, KP = Gm::A_KP, QQ = QN / 4;
  constexpr int NQD = (NR * QQ + NT - 1) / NT;      // epilogue quads per thread
  bf16_t* hs = reinterpret_cast<bf16_t*>(smem);
  float* red = reinterpret_cast<float*>(smem);
  const int tid = otid(), v = tid >> 6, r0 = h * NR, ng = v / KP, kp = v % KP;
  if (l == 0) {
    late();
    ln_rows<1, NR>(a, rs, hs, s_tok, s_pos, w, nullptr, r0, Gm::GW);
  } else {
    ln_rows<0, NR, XB>(a, rs, hs, s_tok, s_pos, w, nullptr, r0, Gm::GW, late);
  }
  lds_sync();
  f32x4_t acc[NRB][3];
  mma_lds<3, Gm::SA, NRB>(hs, 32 * Gm::SA * kp, wq, acc);
  // the bias quads are issued after the MFMAs (issued before the LayerNorm they were spilled,
  // and the spill store waited for the load at the top of the phase)
  float4 bq[NQD];
#pragma unroll
  for (int i = 0; i < NQD; ++i)
    bq[i] = *reinterpret_cast<const float4*>(a.bqkv[l] + QN * w + 4 * ((tid + NT * i) % QQ));
  lds_sync();
  put_partial<3, QN, NRB>(red, kp, 48 * ng, acc);
  lds_sync();
#pragma unroll
  for (int i = 0; i < NQD; ++i) {
    const int qd = tid + NT * i;
    if (qd >= NR * QQ) break;
    const int rl = qd / QQ, c = 4 * (qd % QQ), row = r0 + rl;
    const float4 bb = bq[i];
    float4 sm = *reinterpret_cast<const float4*>(red + rl * QN + c);
#pragma unroll
    for (int k = 1; k < KP; ++k) {
      const float4 p = *reinterpret_cast<const float4*>(red + (k * NR + rl) * QN + c);
      sm.x += p.x; sm.y += p.y; sm.z += p.z; sm.w += p.w;
    }
    if (row < a.R)
      st8(rs.qkv, (row * QKVN + QN * w + c) * 2,
          u32x2_t{pk2bf(sm.x + bb.x, sm.y + bb.y), pk2bf(sm.z + bb.z, sm.w + bb.w)});
  }
}

// ------------------------------------------------------------------ phase B: attention
__device__ __forceinline__ void bf8_unpack(const uint4& u, float (&f)[8]) {
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
  f[4] = __uint_as_float(u.z << 16); f[5] = __uint_as_float(u.z & 0xffff0000u);
  f[6] = __uint_as_float(u.w << 16); f[7] = __uint_as_float(u.w & 0xffff0000u);
}
__device__ __forceinline__ uint4 sel4(bool c, const uint4& x, const uint4& y) {
  return make_uint4(c ? x.x : y.x, c ? x.y : y.y, c ? x.z : y.z, c ? x.w : y.w);
}
__device__ __forceinline__ uint4 tou4(u32x4_t u) { return make_uint4(u.x, u.y, u.z, u.w); }

// one wave per KU (row, head) units; keys in chunks of 8 KC (KC keys per 8-lane group, 8 lanes
// per key: lane sub holds dims 8 sub .. 8 sub + 8), online softmax in f32 (decode_attn6
// arithmetic).  The cached keys of the first chunk do not depend on this step's activations:
// attn_load issues them BEFORE the workgroup waits on the c_attn barrier (kr / vr held across it).
// unit u = (row u / 12, head u % 12); wave v of a workgroup whose first unit is ub takes units
// ub + KU v .. + KU (KU = 2: 16 units per workgroup of a 48-grid; 4: 32 per workgroup of a
// 24-grid, in 32-key chunks (KC 4) so the prefetched keys stay at 128 VGPRs; 1: 8 per workgroup
// of a row half, 96-grid)
__device__ __forceinline__ void attn_unit(const Args& a, const int* s_pos, int u,
                                          int& row, int& hh, int& p, long& base) {
  row = u / NH;
  hh = u % NH;
  const int rr = min(row, a.R - 1);
  p = min(s_pos[rr], a.Lmax - 1);
  base = ((long)(rr * NH + hh) * a.Lmax) * HD + 8 * ((otid() & 63) & 7);
}
template <int KU, int KC, bool NTL = false>
__device__ __forceinline__ void attn_load(const Args& a, int l, const int* s_pos, int ub, int cb,
                                          uint4 (&kr)[KU][KC], uint4 (&vr)[KU][KC]) {
  const int tid = otid(), v = tid >> 6, grp = (tid & 63) >> 3;
  const bf16_t* kc = a.kc[l];
  const bf16_t* vc = a.vc[l];
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    int row, hh, p;
    long base;
    attn_unit(a, s_pos, ub + KU * v + k, row, hh, p, base);
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const int jc = max(min(cb + 8 * i + grp, p - 1), 0);
      kr[k][i] = __builtin_bit_cast(uint4, ldg<NTL>(reinterpret_cast<const u32x4_t*>(kc + base + (long)jc * HD)));
      vr[k][i] = __builtin_bit_cast(uint4, ldg<NTL>(reinterpret_cast<const u32x4_t*>(vc + base + (long)jc * HD)));
    }
  }
}
// The new token (key pos, from qkv) is folded in after the cached keys 0..pos-1 (one more
// online-softmax update with its score and v), so the cached chunks need no per-key selects.
template <int KU, int KC, bool NTL = false>
__device__ __forceinline__ void phase_attn(const Args& a, const Rs& rs, int l, const int* s_pos, int ub,
                                           uint4 (&kr)[KU][KC], uint4 (&vr)[KU][KC]) {
  const int tid = otid(), lane = tid & 63, v = tid >> 6, grp = lane >> 3, sub = lane & 7;
  float q[KU][8], o[KU][8], m[KU], sum[KU];
  uint4 knu[KU], vnu[KU];
  int p[KU], row[KU], hh[KU];
  long base[KU];
  // KU = 4: the new token's k / v are loaded after the cached chunks (32 VGPRs less across them)
  constexpr bool LATE_KV = KU > 2;
  // every unit's q (and k / v) load is issued before any is used: one round trip, not KU
  uint4 qu[KU];
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    attn_unit(a, s_pos, ub + KU * v + k, row[k], hh[k], p[k], base[k]);
    const int off = (min(row[k], a.R - 1) * QKVN + hh[k] * HD + 8 * sub) * 2;
    qu[k] = tou4(ld16(rs.qkv, off));
    if constexpr (!LATE_KV) {
      knu[k] = tou4(ld16(rs.qkv, off + 2 * D));
      vnu[k] = tou4(ld16(rs.qkv, off + 4 * D));
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    bf8_unpack(qu[k], q[k]);
#pragma unroll
    for (int t = 0; t < 8; ++t) { q[k][t] *= 0.125f; o[k][t] = 0.f; }
    m[k] = -INFINITY;
    sum[k] = 0.f;
  }
  int pmax = p[0];
#pragma unroll
  for (int k = 1; k < KU; ++k) pmax = max(pmax, p[k]);
  for (int cb = 0; cb < pmax; cb += 8 * KC) {   // cached keys 0 .. p - 1
    if (cb > 0) attn_load<KU, KC, NTL>(a, l, s_pos, ub, cb, kr, vr);
#pragma unroll
    for (int k = 0; k < KU; ++k) {
      if (cb >= p[k]) continue;                   // wave-uniform
      float sc[KC];
      float pm = -INFINITY;
#pragma unroll
      for (int i = 0; i < KC; ++i) {
        float kf[8];
        bf8_unpack(kr[k][i], kf);
        float sv = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) sv += q[k][t] * kf[t];
        sv = sum8(sv);
        sc[i] = cb + 8 * i + grp < p[k] ? sv : -INFINITY;
        pm = fmaxf(pm, sc[i]);
      }
      pm = fmaxf(pm, xor8(pm));       // group-uniform values: row_ror 8 == lane ^ 8
      pm = max16(pm);
      pm = max32(pm);
      const float mn = fmaxf(m[k], pm);
      const float scale = __expf(m[k] - mn);   // 0 on the first chunk (m = -inf)
      sum[k] *= scale;
#pragma unroll
      for (int t = 0; t < 8; ++t) o[k][t] *= scale;
      m[k] = mn;
#pragma unroll
      for (int i = 0; i < KC; ++i) {
        const float e = __expf(sc[i] - mn);     // masked keys: exp(-inf) = 0
        sum[k] += e;
        float vf[8];
        bf8_unpack(vr[k][i], vf);
#pragma unroll
        for (int t = 0; t < 8; ++t) o[k][t] += e * vf[t];
      }
    }
  }
  if constexpr (LATE_KV) {
#pragma unroll
    for (int k = 0; k < KU; ++k) {
      const int off = (min(row[k], a.R - 1) * QKVN + hh[k] * HD + 8 * sub) * 2;
      knu[k] = tou4(ld16(rs.qkv, off + 2 * D));
      vnu[k] = tou4(ld16(rs.qkv, off + 4 * D));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    // over the 8 key groups (lanes sub, sub + 8, ..): same additions on every lane
    sum[k] = add32(add16(sum[k] + xor8(sum[k])));
#pragma unroll
    for (int t = 0; t < 8; ++t) o[k][t] = add32(add16(o[k][t] + xor8(o[k][t])));
    // the new token, key pos: its score from registers
    float kf[8], vf[8];
    bf8_unpack(knu[k], kf);
    bf8_unpack(vnu[k], vf);
    float sn = 0.f;
#pragma unroll
    for (int t = 0; t < 8; ++t) sn += q[k][t] * kf[t];
    sn = sum8(sn);
    const float mn = fmaxf(m[k], sn);
    const float sc = __expf(m[k] - mn), en = __expf(sn - mn);
    const float inv = 1.0f / (sum[k] * sc + en);
    float of[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) of[t] = (o[k][t] * sc + en * vf[t]) * inv;
    if (grp == 0 && row[k] < a.R) {
      u32x4_t pk{pk2bf(of[0], of[1]), pk2bf(of[2], of[3]), pk2bf(of[4], of[5]), pk2bf(of[6], of[7])};
      // att in A-fragment order: row r, dims 64 h + 8 sub .. + 8 = k-step 2 h + sub / 4,
      // lane (r & 15) + 16 (sub & 3)
      const int r = row[k];
      const int fo = (((r >> 4) * (D / 32) + 2 * hh[k] + (sub >> 2)) * 64 + (r & 15) + 16 * (sub & 3)) * 16;
      st16(rs.att, fo, pk);
      // the new token's K / V (read again only by this workgroup, at later steps)
      *reinterpret_cast<uint4*>(a.kc[l] + base[k] + (long)p[k] * HD) = knu[k];
      *reinterpret_cast<uint4*>(a.vc[l] + base[k] + (long)p[k] * HD) = vnu[k];
    }
  }
}

// ------------------------------------------------------------------ phases C / E: projections
// x[:, PN w .. PN w + PN) += A W^T + b (PN = 16 CS columns, NB = CS blocks), A = att (K 768) or
// hid (K 3072) from the workspace in A-fragment order; wave v takes k-steps [v S, (v+1) S), its A
// fragments in chunks of CH k-steps (NIF chunks in flight), each fragment load one contiguous
// KiB, every fragment read by exactly one wave and multiplied into all NB column blocks
template <int S, int CS, int RH, bool XB, int RB = 4, int CH = 4, int NIF = 2, typename Late = NoLate>
__device__ __forceinline__ void phase_proj(const Args& a, const Rs& rs, __amdgpu_buffer_rsrc_t ra,
                                           int K, const float* bias, char* smem, int w, int h,
                                           const bf16x8_t (&wb)[CS * S], Late late = Late()) {
  constexpr int NR = 16 * RB / RH, NRB = NR / 16, NB = CS, PN = 16 * CS, PQ = PN / 4;
  float* red = reinterpret_cast<float*>(smem);
  const int tid = otid(), lane = tid & 63, v = tid >> 6, r0 = h * NR;
  // epilogue operands first: NR rows x PQ quads on threads 0 .. PQ NR - 1 (two threads per
  // 16-byte bf16 copy were tried: the longer per-thread epilogue cost more than the 8-byte stores)
  const int erl = (tid / PQ) % NR, erow = r0 + erl, ec = PN * w + 4 * (tid % PQ);
  float4 eb = make_float4(0.f, 0.f, 0.f, 0.f), ex = eb;
  if (tid < PQ * NR) {
    eb = *reinterpret_cast<const float4*>(bias + ec);
    ex = u2f4(ld16(rs.x, (min(erow, a.R - 1) * D + ec) * 4));
  }
  // fragment (row block rb of the workgroup's rows, k-step s) of this lane at
  // (((r0 / 16 + rb) * K/32 + s) * 64 + lane) * 16 bytes
  int aoff[NRB];
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) aoff[rb] = (((r0 / 16 + rb) * (K / 32) + v * S) * 64 + lane) * 16;
  f32x4_t acc[NRB][NB];
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[rb][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  constexpr int NCH = (S + CH - 1) / CH;
  u32x4_t af[NCH][NRB * CH];
#pragma unroll
  for (int c = 0; c < NCH && c < NIF; ++c)
#pragma unroll
    for (int s = 0; s < CH; ++s)
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
        if (c * CH + s < S) af[c][s * NRB + rb] = ld16(ra, aoff[rb] + 1024 * (c * CH + s));
  late();
  // keep the issued chunks in flight: without the scheduling barriers the compiler sank each
  // fragment load to its MFMA under register pressure (one round trip per k-step)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
#pragma unroll
    for (int s = 0; s < CH; ++s)
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          if (c * CH + s < S)
            acc[rb][nb] = mfma(bf8(af[c][s * NRB + rb]), wb[nb * S + c * CH + s], acc[rb][nb]);
    if (c + NIF < NCH) {
#pragma unroll
      for (int s = 0; s < CH; ++s)
#pragma unroll
        for (int rb = 0; rb < NRB; ++rb)
          if ((c + NIF) * CH + s < S)
            af[c + NIF][s * NRB + rb] = ld16(ra, aoff[rb] + 1024 * ((c + NIF) * CH + s));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  put_partial<NB, PN, NRB>(red, v, 0, acc);
  lds_sync();
  if (tid < PQ * NR) {
    float4 sm = *reinterpret_cast<const float4*>(red + erl * PN + 4 * (tid % PQ));
#pragma unroll
    for (int k = 1; k < NW; ++k) {
      const float4 p = *reinterpret_cast<const float4*>(red + (k * NR + erl) * PN + 4 * (tid % PQ));
      sm.x += p.x; sm.y += p.y; sm.z += p.z; sm.w += p.w;
    }
    if (erow < a.R) {
      const float4 o = make_float4(sm.x + eb.x + ex.x, sm.y + eb.y + ex.y, sm.z + eb.z + ex.z,
                                   sm.w + eb.w + ex.w);
      st16(rs.x, (erow * D + ec) * 4, f42u(o.x, o.y, o.z, o.w));
      if constexpr (XB) st8(rs.xb, (erow * D + ec) * 2, u32x2_t{pk2bf(o.x, o.y), pk2bf(o.z, o.w)});
    }
  }
}

// ------------------------------------------------------------------ phase D: ln_2 + c_fc + gelu
__device__ __forceinline__ float gelu_new_fast(float x) {
  const float u2 = -1.5957691216057308f * (x + 0.044715f * x * x * x);
  return x * __builtin_amdgcn_rcpf(1.0f + __expf(u2));
}
// wave v = (column group v / D_KP of 2 blocks, K part v % D_KP); FN = 64 CS columns per workgroup;
// the D_KP partial slabs (65,536 B at every CS) alias the LN rows
template <int CS, int RH, bool XB, int RB = 4, typename Late = NoLate>
__device__ __forceinline__ void phase_fc(const Args& a, const Rs& rs, int l, char* smem,
                                         const int* s_tok, const int* s_pos, int w, int h,
                                         const bf16x8_t (&wf)[2 * Geo<CS>::SD], Late late = Late()) {
  using Gm = Geo<CS>;
  constexpr int NR = 16 * RB / RH, NRB = NR / 16, FN = Gm::FN, KP = Gm::D_KP, FQ = FN / 4;
  // epilogue quads per thread (same column quad); 16 rows x 16 quads leave half the threads idle
  constexpr int NQD = (NR * FQ + NT - 1) / NT;
  static_assert(NT % FQ == 0, "phase D epilogue mapping");
  bf16_t* hs = reinterpret_cast<bf16_t*>(smem);
  float* red = reinterpret_cast<float*>(smem);
  const int tid = otid(), v = tid >> 6, cg = v / KP, kq = v % KP, r0 = h * NR;
  const int c = 4 * (tid % FQ);
  const float4 bb = *reinterpret_cast<const float4*>(a.bfc[l] + FN * w + c);
  ln_rows<0, NR, XB>(a, rs, hs, s_tok, s_pos, w, nullptr, r0, Gm::GW, late);
  lds_sync();
  f32x4_t acc[NRB][2];
  mma_lds<2, Gm::SD, NRB>(hs, 32 * Gm::SD * kq, wf, acc);
  lds_sync();
  put_partial<2, FN, NRB>(red, kq, 32 * cg, acc);
  lds_sync();
#pragma unroll
  for (int hq = 0; hq < NQD; ++hq) {
    const int rl = tid / FQ + (NT / FQ) * hq, row = r0 + rl;
    if (rl >= NR) break;
    float4 sm = *reinterpret_cast<const float4*>(red + rl * FN + c);
#pragma unroll
    for (int k = 1; k < KP; ++k) {
      const float4 p = *reinterpret_cast<const float4*>(red + (k * NR + rl) * FN + c);
      sm.x += p.x; sm.y += p.y; sm.z += p.z; sm.w += p.w;
    }
    // hid in A-fragment order: column k = FN w + c -> k-step k / 32, lane (row & 15) + 16 ((k / 8) & 3)
    const int k = FN * w + c;
    if (row < a.R)
      st8(rs.hid, ((((row >> 4) * (DFF / 32) + (k >> 5)) * 64 + (row & 15) + 16 * ((k >> 3) & 3)) * 8 + (k & 7)) * 2,
          u32x2_t{pk2bf(gelu_new_fast(sm.x + bb.x), gelu_new_fast(sm.y + bb.y)),
                  pk2bf(gelu_new_fast(sm.z + bb.z), gelu_new_fast(sm.w + bb.w))});
  }
}

// ------------------------------------------------------------------ fused MLP: D' and R
// D' (FUSE): ln_2 + c_fc + gelu_new as phase D, but the workgroup's FN hid columns stay in LDS
// (hl [NR][FN + 8] bf16) and are multiplied at once by the matching FN columns of mlp.c_proj:
// out[rows, 768] = gelu(h[:, FN w ..]) Wmp[:, FN w ..]^T, a K-slice partial of the MLP output that
// the workgroup stores (bf16 tiles, write-through) for the 48 / CS column-slice owners to sum in
// phase R.  Every hid byte then stays on its CU (the unfused E phase had every workgroup read the
// whole 393 KB hid), and R reads 98 KB of partials instead.  mlp.c_proj per wave: columns 96 v ..
// + 96 (6 blocks, two rounds of 3), K = FN (2 CS k-steps), no cross-wave reduction.
template <int CS, int RH>
__device__ __forceinline__ void put_part_tile(const Rs& rs, int w, int h, int rb, int cb,
                                              const f32x4_t& acc) {
  using Gm = Geo<CS>;
  constexpr int NRB = RM / RH / 16;
  const int lane = otid() & 63, j = cb / CS, bi = cb % CS;
  const int off = (((((w * RH + h) * Gm::GW + j) * NRB + rb) * CS + bi) * 64 + lane) * PART_EB;
  if constexpr (PART_BF16) st8(rs.part, off, u32x2_t{pk2bf(acc[0], acc[1]), pk2bf(acc[2], acc[3])});
  else st16(rs.part, off, f42u(acc[0], acc[1], acc[2], acc[3]));
}
template <int CS, int RH, bool XB, typename Late1, typename Mid, typename Late2>
__device__ __forceinline__ void phase_fc_fused(const Args& a, const Rs& rs, int l, char* smem,
                                               const int* s_tok, const int* s_pos, int w, int h,
                                               const bf16x8_t (&wf)[2 * Geo<CS>::SD],
                                               bf16x8_t (&wm)[6 * 2 * CS], Late1 late1, Mid mid,
                                               Late2 late2) {
  using Gm = Geo<CS>;
  constexpr int NR = RM / RH, NRB = NR / 16, FN = Gm::FN, KP = Gm::D_KP, FQ = FN / 4;
  constexpr int NQD = NR * FQ / NT, KS = FN / 32, HL = FN + 8;
  static_assert(NT % FQ == 0 && (NR * FQ) % NT == 0, "phase D epilogue mapping");
  static_assert(KP * NR * FN * 4 + NR * HL * 2 <= SM_HS, "slabs + hid tile fit the row buffer");
  bf16_t* hs = reinterpret_cast<bf16_t*>(smem);
  float* red = reinterpret_cast<float*>(smem);
  bf16_t* hl = reinterpret_cast<bf16_t*>(smem + KP * NR * FN * 4);
  const int tid = otid(), lane = tid & 63, v = tid >> 6, cg = v / KP, kq = v % KP;
  const int c = 4 * (tid % FQ);
  const float4 bb = *reinterpret_cast<const float4*>(a.bfc[l] + FN * w + c);
  ln_rows<0, NR, XB>(a, rs, hs, s_tok, s_pos, w, nullptr, h * NR, Gm::GW, late1);
  lds_sync();
  mid();               // loads after the LN (its row values are dead)
  f32x4_t acc[NRB][2];
  mma_lds<2, Gm::SD, NRB>(hs, 32 * Gm::SD * kq, wf, acc);
  late2();             // loads after c_fc's MFMAs (its fragments are dead)
  lds_sync();
  put_partial<2, FN, NRB>(red, kq, 32 * cg, acc);
  lds_sync();
#pragma unroll
  for (int hq = 0; hq < NQD; ++hq) {
    const int rl = tid / FQ + (NT / FQ) * hq;
    float4 sm = *reinterpret_cast<const float4*>(red + rl * FN + c);
#pragma unroll
    for (int k = 1; k < KP; ++k) {
      const float4 p = *reinterpret_cast<const float4*>(red + (k * NR + rl) * FN + c);
      sm.x += p.x; sm.y += p.y; sm.z += p.z; sm.w += p.w;
    }
    *reinterpret_cast<uint2*>(hl + rl * HL + c) =
        make_uint2(pk2bf(gelu_new_fast(sm.x + bb.x), gelu_new_fast(sm.y + bb.y)),
                   pk2bf(gelu_new_fast(sm.z + bb.z), gelu_new_fast(sm.w + bb.w)));
  }
  lds_sync();
  // mlp.c_proj partial: A = the hid tile (LDS), B = wm (blocks 6 v + 3 nh + nb, k-steps s)
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  bf16x8_t af[NRB][KS];
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2)
      af[rb][s2] = *reinterpret_cast<const bf16x8_t*>(hl + (16 * rb + fr) * HL + 32 * s2 + fk);
#pragma unroll
  for (int nh = 0; nh < 2; ++nh) {
    f32x4_t o[NRB][3];
#pragma unroll
    for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
      for (int nb = 0; nb < 3; ++nb) {
        o[rb][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) o[rb][nb] = mfma(af[rb][s2], wm[(3 * nh + nb) * KS + s2], o[rb][nb]);
      }
#pragma unroll
    for (int rb = 0; rb < NRB; ++rb)
#pragma unroll
      for (int nb = 0; nb < 3; ++nb) put_part_tile<CS, RH>(rs, w, h, rb, 6 * v + 3 * nh + nb, o[rb][nb]);
  }
}

// R (FUSE): the owner of column slice w (PN = 16 CS columns) sums the GW workgroups' partials of
// its tiles in a fixed order (producers in GP groups of PPG, the groups in order), adds the bias
// and the residual: x[:, PN w ..] (f32 and its bf16 copy), as phase E did.
__device__ __forceinline__ void part_unpack(const u32x2_t& v, float (&f)[4]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
}
__device__ __forceinline__ void part_unpack(const u32x4_t& v, float (&f)[4]) {
  f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y);
  f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
}
template <int CS, int RH, bool XB>
__device__ __forceinline__ void phase_red(const Args& a, const Rs& rs, const float* bias, char* smem,
                                          int w, int h) {
  using Gm = Geo<CS>;
  constexpr int NR = RM / RH, NRB = NR / 16, PN = Gm::PN, PQ = PN / 4, GW = Gm::GW;
  constexpr int UNITS = NRB * CS * 64, GP = NT / UNITS, PPG = GW / GP;
  static_assert(NT % UNITS == 0 && GW % GP == 0, "phase R mapping");
  float* red = reinterpret_cast<float*>(smem);
  const int tid = otid(), r0 = h * NR;
  const int u = tid % UNITS, g = tid / UNITS, lane = u & 63, t = u >> 6, rb = t / CS, bi = t % CS;
  // epilogue operands first (as phase_proj)
  const int erl = (tid / PQ) % NR, erow = r0 + erl, ec = PN * w + 4 * (tid % PQ);
  float4 eb = make_float4(0.f, 0.f, 0.f, 0.f), ex = eb;
  if (tid < PQ * NR) {
    eb = *reinterpret_cast<const float4*>(bias + ec);
    ex = u2f4(ld16(rs.x, (min(erow, a.R - 1) * D + ec) * 4));
  }
  typedef std::conditional_t<PART_BF16 != 0, u32x2_t, u32x4_t> pv_t;
  pv_t pv[PPG];
#pragma unroll
  for (int i = 0; i < PPG; ++i) {
    const int wp = g * PPG + i;
    const int off = (((((wp * RH + h) * GW + w) * NRB + rb) * CS + bi) * 64 + lane) * PART_EB;
    if constexpr (PART_BF16) pv[i] = ld8(rs.part, off);
    else pv[i] = ld16(rs.part, off);
  }
  __builtin_amdgcn_sched_barrier(0);
  float sm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < PPG; ++i) {
    float f[4];
    part_unpack(pv[i], f);
#pragma unroll
    for (int e = 0; e < 4; ++e) sm[e] += f[e];
  }
  // group sums -> slab g, rows (16 rb + 4 (lane / 16) + e), column 16 bi + lane % 16
#pragma unroll
  for (int e = 0; e < 4; ++e)
    red[(g * NR + 16 * rb + 4 * (lane >> 4) + e) * PN + 16 * bi + (lane & 15)] = sm[e];
  lds_sync();
  if (tid < PQ * NR) {
    float4 s4 = *reinterpret_cast<const float4*>(red + erl * PN + 4 * (tid % PQ));
#pragma unroll
    for (int k = 1; k < GP; ++k) {
      const float4 p = *reinterpret_cast<const float4*>(red + (k * NR + erl) * PN + 4 * (tid % PQ));
      s4.x += p.x; s4.y += p.y; s4.z += p.z; s4.w += p.w;
    }
    if (erow < a.R) {
      const float4 o = make_float4(s4.x + eb.x + ex.x, s4.y + eb.y + ex.y, s4.z + eb.z + ex.z,
                                   s4.w + eb.w + ex.w);
      st16(rs.x, (erow * D + ec) * 4, f42u(o.x, o.y, o.z, o.w));
      if constexpr (XB) st8(rs.xb, (erow * D + ec) * 2, u32x2_t{pk2bf(o.x, o.y), pk2bf(o.z, o.w)});
    }
  }
}

// ------------------------------------------------------------------ phase F: ln_f + LM head
// vocab blocks of 16 rows [wg nvb / gg, (wg+1) nvb / gg) of this WG (gg = the grid), taken in PAIRS (one A fragment
// read from LDS feeds the MFMAs of both blocks: half the LDS traffic per MFMA); wave v takes
// pairs v, v + 8, ..  A pair's weights (wtep: 24 KiB contiguous per block, one KiB per k-step in
// B-fragment order) arrive as six 4-k-step pieces (both blocks) through a 4-slot register ring:
// three pieces in flight while one is consumed.  Per lane a running (logit, id) best for each of
// its 16 rows.  The WG's best per row goes to a 64-bit agent-scope atomic max of
// key = (order-preserving logit bits, ~id): larger logit wins, then the lower id (torch.argmax),
// whatever order the workgroups arrive in.
template <bool NTL>
__device__ __forceinline__ void lm_piece(const bf16_t* Wp, int b0, int b1, int c, bf16x8_t (&b)[8]) {
  const int lane = otid() & 63;
  const bf16_t* p0 = Wp + ((long)(b0 * (D / 32) + 4 * c) * 64 + lane) * 8;
  const bf16_t* p1 = Wp + ((long)(b1 * (D / 32) + 4 * c) * 64 + lane) * 8;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    b[i] = ldg<NTL>(reinterpret_cast<const bf16x8_t*>(p0 + 512 * i));
    b[4 + i] = ldg<NTL>(reinterpret_cast<const bf16x8_t*>(p1 + 512 * i));
  }
}
__device__ __forceinline__ void lm_consume(const bf16_t* hs, int c, const bf16x8_t (&b)[8],
                                           f32x4_t (&acc)[2][4]) {
  const int lane = otid() & 63, fr = lane & 15, fk = 8 * (lane >> 4);
  // A fragments one k-step ahead of the MFMAs (two register sets)
  const bf16_t* hrow = hs + fr * HLD + 128 * c + fk;
  bf16x8_t af[2][4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) af[0][rb] = *reinterpret_cast<const bf16x8_t*>(hrow + 16 * rb * HLD);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i + 1 < 4) {
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
        af[(i + 1) & 1][rb] = *reinterpret_cast<const bf16x8_t*>(hrow + 16 * rb * HLD + 32 * (i + 1));
    }
    // 4 LDS reads, then the 8 MFMAs of the previous reads (sched_group_barrier: DS read 0x100,
    // MFMA 0x008)
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      acc[0][rb] = mfma(af[i & 1][rb], b[i], acc[0][rb]);
      acc[1][rb] = mfma(af[i & 1][rb], b[4 + i], acc[1][rb]);
    }
  }
}
template <bool XB, bool NTL>
__device__ __forceinline__ void phase_lm(const Args& a, const Rs& rs, char* smem, const int* s_tok,
                                         const int* s_pos, float* am_v, int* am_i, int wg, int gg,
                                         gu64* keys, const float* s_lnf) {
  bf16_t* hs = reinterpret_cast<bf16_t*>(smem);
  const int tid = otid(), lane = tid & 63, v = tid >> 6, fr = lane & 15, r4 = 4 * (lane >> 4);
  ln_rows<2, RM, XB>(a, rs, hs, s_tok, s_pos, wg, s_lnf);
  lds_sync();
  const int nvb = (a.V + 15) / 16;
  const int b_lo = (int)((long)wg * nvb / gg), b_hi = (int)((long)(wg + 1) * nvb / gg);
  const int npair = (b_hi - b_lo + 1) / 2;              // the last pair may hold one block
  // lm_il (A/B): pairs interleaved over the grid (pair (m NW + v) gg + wg for wave v of workgroup
  // wg), so every CU streams pieces of the whole table instead of one contiguous 1.6 MB range
  const int P = (nvb + 1) / 2, x0 = v * gg + wg;
  const int npw = a.lm_il ? (P - x0 + NW * gg - 1) / (NW * gg)
                          : (npair - v + NW - 1) / NW;  // pairs of this wave (>= 1)
  float bv[16];
  int bi[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) { bv[e] = -INFINITY; bi[e] = 0x7fffffff; }
  // blocks of pair m of this wave (clamped into the WG's range: loads past it re-read its last
  // block; their columns are masked below)
  auto blk = [&](int m, int h) {
    if (a.lm_il) return min(2 * ((min(m, npw - 1) * NW) * gg + x0) + h, nvb - 1);
    return min(b_lo + 2 * (v + NW * min(m, npw - 1)) + h, b_hi - 1);
  };
  const bool tmp = a.temp != 1.0f;
  // the running (logit, id) best of pair m's two blocks (blocks in increasing id order within
  // the lane: strict > keeps the lower id on ties)
  auto best = [&](int m, const f32x4_t (&acc)[2][4]) {
    const int p0 = a.lm_il ? 2 * (m * NW * gg + x0) : b_lo + 2 * (v + NW * m);
    const int p_hi = a.lm_il ? nvb : b_hi;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = 16 * (p0 + h) + fr;
      if (p0 + h < p_hi && col < a.V) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float val = tmp ? acc[h][rb][i] / a.temp : acc[h][rb][i];
            if (val > bv[4 * rb + i]) { bv[4 * rb + i] = val; bi[4 * rb + i] = col; }
          }
      }
    }
  };
  // the wave's piece stream j = 6 m + c (pair m, piece c) through a 4-slot register ring, slot
  // j % 4: piece j + 3 is issued before piece j is consumed (three pieces, 24 KiB per wave, in
  // flight); two pairs per iteration make every slot index a constant
  bf16x8_t R0[8], R1[8], R2[8], R3[8];
#define LMP(M_, C_, R_) lm_piece<NTL>(a.wtep, blk(M_, 0), blk(M_, 1), C_, R_)
  LMP(0, 0, R0);
  LMP(0, 1, R1);
  LMP(0, 2, R2);
  for (int m = 0; m < npw; m += 2) {
    f32x4_t acc[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[h][rb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    LMP(m, 3, R3);     lm_consume(hs, 0, R0, acc);
    LMP(m, 4, R0);     lm_consume(hs, 1, R1, acc);
    LMP(m, 5, R1);     lm_consume(hs, 2, R2, acc);
    LMP(m + 1, 0, R2); lm_consume(hs, 3, R3, acc);
    LMP(m + 1, 1, R3); lm_consume(hs, 4, R0, acc);
    LMP(m + 1, 2, R0); lm_consume(hs, 5, R1, acc);
    best(m, acc);
    if (m + 1 < npw) {         // wave-uniform
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) acc[h][rb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      LMP(m + 1, 3, R1); lm_consume(hs, 0, R2, acc);
      LMP(m + 1, 4, R2); lm_consume(hs, 1, R3, acc);
      LMP(m + 1, 5, R3); lm_consume(hs, 2, R0, acc);
      LMP(m + 2, 0, R0); lm_consume(hs, 3, R1, acc);
      LMP(m + 2, 1, R1); lm_consume(hs, 4, R2, acc);
      LMP(m + 2, 2, R2); lm_consume(hs, 5, R3, acc);
      best(m + 1, acc);
    }
  }
#undef LMP
  // over the 16 lanes of each row group (columns), ties -> lower id
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float ov = __shfl_xor(bv[e], o, 64);
      const int oi = __shfl_xor(bi[e], o, 64);
      if (ov > bv[e] || (ov == bv[e] && oi < bi[e])) { bv[e] = ov; bi[e] = oi; }
    }
  if (fr == 0) {
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * rb + r4 + i;
        am_v[v * RM + row] = bv[4 * rb + i];
        am_i[v * RM + row] = bi[4 * rb + i];
      }
  }
  lds_sync();
  if (tid < RM) {
    float best = am_v[tid];
    int bidx = am_i[tid];
#pragma unroll
    for (int k = 1; k < NW; ++k) {
      const float cv = am_v[k * RM + tid];
      const int ci = am_i[k * RM + tid];
      if (cv > best || (cv == best && ci < bidx)) { best = cv; bidx = ci; }
    }
    const unsigned long long key = ((unsigned long long)f2key(best) << 32) | (unsigned)(~bidx);
    __hip_atomic_fetch_max(keys + tid, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// a workgroup that gave up waiting (grid not co-resident): all_done = {1, -1} tells the host
__device__ __forceinline__ void gave_up(const Args& a) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(&a.all_done[1], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.all_done[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ------------------------------------------------------------------ the kernel
// RH = 1: G = 48 workgroups, each owns a column slice of every GEMM for all 64 rows; RH = 2 (the
// row-split grid, 96 workgroups): workgroup (w, h) = the same column slice for rows 32 h .. + 32
// (half the handed-off activation bytes per workgroup, the same weights: blocks b and b + 8 --
// one XCD under round-robin dispatch, speed only -- hold the two halves of a slice), the attention
// units of its rows, and 1/96 of the LM head's vocabulary for all rows.
// XB: the LayerNorm inputs are handed off as a bf16 copy of x (written by phases C / E beside
// the f32 residual stream), halving the bytes every workgroup reads in phases A, D and F.
// NTM: non-temporal loads, bit 0 the weight / LM-head streams, bit 1 the cached K/V
// CS: column slices per workgroup (Geo; grid = 48 / CS x RH workgroups).  FUSE: the MLP as
// phases D' + R (partial mlp.c_proj sums, no hid hand-off) instead of D + E
// RB: row blocks of 16 the grid covers (4: all 64 rows; 2 for batches of <= 32 rows, whose
// phases then read half of the handed-off activations)
template <int CS, int RH, bool XB, int NTM = 0, bool FUSE = false, int RB = 4>
__global__ __launch_bounds__(NT) void decode_persist_kernel(Args a) {
  using Gm = Geo<CS>;
  constexpr bool NTW = NTM & 1, NTK = (NTM >> 1) & 1;
  __shared__ __attribute__((aligned(16))) char smem[SM_TOTAL];
  float* am_v = reinterpret_cast<float*>(smem + SM_HS);
  int* am_i = reinterpret_cast<int*>(smem + SM_HS) + NW * RM;
  int* s_tok = reinterpret_cast<int*>(smem + SM_HS + SM_AM);
  int* s_pos = s_tok + RM;
  int* s_done = s_pos + RM;
  int* s_misc = s_done + RM;     // [0] rows still decoding, [8] barrier ok flag
  constexpr int GW = Gm::GW, GG = GW * RH;
  // attention units (row, head) per workgroup, per wave, the waves that have units, keys per group
  constexpr int UPW = 4 * RB * CS / RH, KU = UPW >= 8 ? UPW / 8 : 1, AW = UPW / KU;
  constexpr int KC = KU > 2 ? 4 : 8;
  static_assert(AW <= NW && AW * KU == UPW, "attention units");
  static_assert(!FUSE || RB == 4, "the fused MLP covers all 64 rows");
  const int wg = blockIdx.x;
  const int w = RH == 1 ? wg : (wg & 7) + 8 * (wg >> 4), h = RH == 1 ? 0 : (wg >> 3) & 1;
  const int ub = (16 * RB * NH / RH) * h + UPW * w;       // first attention unit of this workgroup
  // (a scalar, provably wave-uniform condition; constant true when every wave has units)
  const bool attn_wave = AW == NW || __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) < AW;
  Rs rs;
  rs.x = mk(a.ws + WS_X, RM * D * 4);
  rs.qkv = mk(a.ws + WS_QKV, RM * QKVN * 2);
  rs.att = mk(a.ws + WS_ATT, RM * D * 2);
  rs.hid = mk(a.ws + WS_HID, RM * DFF * 2);
  rs.xb = mk(a.ws + WS_XB, RM * D * 2);
  rs.part = mk(a.ws + WS_PART, G * RM * D * (PART_BF16 ? 2 : 4));
  Bar bar{(gu32*)(a.ws + WS_SYNC), (gu32*)(a.ws + WS_SYNC + 4), 0, nullptr, 0, GG, a.spin_max};
  gu64* const lmkey = (gu64*)(a.ws + WS_LMKEY);
  unsigned long long* const stamps = dp_stamp_buf;
  const int stamp_step = dp_stamp_step;
  // the barrier's ok word, through an LDS-typed pointer (a generic volatile pointer became flat
  // accesses, whose wait is vmcnt(0): every wave then waited for its weight prefetch at each barrier)
  typedef __attribute__((address_space(3))) int lds_int;
  volatile lds_int* s_ok = (volatile lds_int*)(s_misc + 8);
  float* s_lnf = reinterpret_cast<float*>(smem + SM_HS + SM_AM + SM_ST);
  for (int i = otid(); i < D; i += NT) { s_lnf[i] = a.lnf_w[i]; s_lnf[D + i] = a.lnf_b[i]; }

  if (a.all_done[0]) return;                 // every row stopped at step 0 (uniform)
  int step = *a.step_ctr;
  if (step >= a.max_steps) return;
  if (otid() < RM) {
    const int tid = otid();
    const bool in = tid < a.R;
    s_tok[tid] = in ? a.next_tok[tid] : 0;
    s_pos[tid] = in ? a.pos[tid] : 0;
    s_done[tid] = in ? a.done[tid] : 1;
  }
  __syncthreads();

  // weight fragments of this workgroup's column slices (each prefetched across the barrier
  // before its phase): c_attn (3 blocks x SA k-steps), attn.c_proj (CS blocks x 3), c_fc (2 blocks
  // x SD), mlp.c_proj (CS blocks x 12)
  bf16x8_t wq[3 * Gm::SA], wp[CS * 3], wf[2 * Gm::SD], wm[FUSE ? 1 : CS * 12];
#define V_ (otid() >> 6)
  // CS = 2: the big prefetches (c_attn, c_fc, mlp.c_proj: 72-96 VGPRs) are split around the
  // barrier wait -- the first k-steps before it, the rest after -- so the polling wave's wait is
  // not queued behind all of its own weight loads (vector loads return in order)
  constexpr int SPL = CS == 1 ? 1 : 2;
#define LOAD_WQ_H(L_, H_) load_w<3, Gm::SA, NTW, (H_) * Gm::SA / SPL, ((H_) + 1) * Gm::SA / SPL>( \
      a.wqkv[L_], D, Gm::QN * w + 48 * (V_ / Gm::A_KP), QKVN, 32 * Gm::SA * (V_ % Gm::A_KP), wq)
// c_attn: the first part before the barrier wait, the rest inside phase A (after the LN rows'
// loads); at CS = 1 it is all before the wait
#define LOAD_WQ(L_) LOAD_WQ_H(L_, 0)
  LOAD_WQ(0);
  for (;;) {
    bar.sb = (stamps != nullptr && step == stamp_step) ? stamps + (long)wg * 2 * DP_NB : nullptr;
    bar.n0 = bar.n;
    stamp(bar.sb, 2 * DP_NB - 1);   // step start
    for (int l = 0; l < NLY; ++l) {
      phase_qkv<CS, RH, XB, RB>(a, rs, l, smem, s_tok, s_pos, w, h, wq, [&] {
        if constexpr (SPL == 2) LOAD_WQ_H(l, 1);
      });
      bar_arrive(bar);
      uint4 kr[KU][KC], vr[KU][KC];
      if (attn_wave) attn_load<KU, KC, NTK>(a, l, s_pos, ub, 0, kr, vr);
      if (!bar_wait(bar, s_ok)) return gave_up(a);
      if (l == 0 && wg == 0 && otid() < RM)  // the previous step's argmax keys: every WG has read them
        __hip_atomic_store(lmkey + ((step + 1) & 1) * RM + otid(), 0ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);

      if (attn_wave) phase_attn<KU, KC, NTK>(a, rs, l, s_pos, ub, kr, vr);
      bar_arrive(bar);
#define LOAD_WF_H(H_) load_w<2, Gm::SD, NTW, (H_) * Gm::SD / SPL, ((H_) + 1) * Gm::SD / SPL>( \
      a.wfc[l], D, Gm::FN * w + 32 * (V_ / Gm::D_KP), DFF, 32 * Gm::SD * (V_ % Gm::D_KP), wf)
#define LOAD_WF LOAD_WF_H(0); if constexpr (SPL == 2) LOAD_WF_H(1)
      load_w<CS, 3, NTW>(a.wproj[l], D, Gm::PN * w, D, 96 * V_, wp);
      // c_fc's fragments: across phase C at CS = 1 (12 fragments); at CS = 2 (24) they wait for
      // C's barrier (held through C they spilled)
      if constexpr (CS == 1) LOAD_WF;
      if (!bar_wait(bar, s_ok)) return gave_up(a);

      phase_proj<3, CS, RH, XB, RB>(a, rs, rs.att, D, a.bproj[l], smem, w, h, wp);
      bar_arrive(bar);
      if constexpr (CS != 1) LOAD_WF_H(0);
      if (!bar_wait(bar, s_ok)) return gave_up(a);

      if constexpr (FUSE) {
        // D': c_fc + gelu + this workgroup's K-slice of mlp.c_proj (mlp.c_proj fragments: all with
        // the LN rows' loads at CS = 1; at CS = 2 blocks 0-2 after the LN, 3-5 after c_fc's MFMAs)
        bf16x8_t wmf[6 * 2 * CS];
#define LOAD_WMF(B0_, B1_) load_w_nb<6, 2 * CS, B0_, B1_, NTW>(a.wmp[l], DFF, 96 * V_, D, Gm::FN * w, wmf)
        phase_fc_fused<CS, RH, XB>(
            a, rs, l, smem, s_tok, s_pos, w, h, wf, wmf,
            [&] {
              if constexpr (CS != 1) LOAD_WF_H(1);
              else LOAD_WMF(0, 6);
            },
            [&] {
              if constexpr (CS != 1) LOAD_WMF(0, 3);
            },
            [&] {
              if constexpr (CS != 1) LOAD_WMF(3, 6);
            });
#undef LOAD_WMF
        bar_arrive(bar);
        // next block's c_attn (first part), across phase R (few registers there)
        LOAD_WQ(l + 1 < NLY ? l + 1 : 0);
        if (!bar_wait(bar, s_ok)) return gave_up(a);
        phase_red<CS, RH, XB>(a, rs, a.bmp[l], smem, w, h);
        bar_arrive(bar);
        if (!bar_wait(bar, s_ok)) return gave_up(a);
      } else {
        phase_fc<CS, RH, XB, RB>(a, rs, l, smem, s_tok, s_pos, w, h, wf, [&] {
          if constexpr (CS != 1) LOAD_WF_H(1);
        });
        bar_arrive(bar);
        load_w<CS, 12, NTW, 0, 12 / SPL>(a.wmp[l], DFF, Gm::PN * w, D, 384 * V_, wm);
        if (!bar_wait(bar, s_ok)) return gave_up(a);

        // CS = 2: 2-k-step chunks, 3 in flight (the 24 weight fragments leave fewer VGPRs)
        phase_proj<12, CS, RH, XB, RB, (CS == 1 ? 4 : 2), (CS == 1 ? 2 : 3)>(
            a, rs, rs.hid, DFF, a.bmp[l], smem, w, h, wm, [&] {
              if constexpr (SPL == 2) load_w<CS, 12, NTW, 6, 12>(a.wmp[l], DFF, Gm::PN * w, D, 384 * V_, wm);
            });
        bar_arrive(bar);
        // next block's c_attn.  Unconditional (a conditional load keeps the old wq live through
        // the whole block for the path that skips it); after block 11 the value is dead and wq is
        // reloaded after the LM head, which needs the VGPRs
        LOAD_WQ(l + 1 < NLY ? l + 1 : 0);
        if (!bar_wait(bar, s_ok)) return gave_up(a);
      }
#undef LOAD_WF
#undef LOAD_WF_H
    }
    phase_lm<XB, NTW>(a, rs, smem, s_tok, s_pos, am_v, am_i, wg, GG, lmkey + (step & 1) * RM, s_lnf);
    bar_arrive(bar);
    LOAD_WQ(0);
    if (!bar_wait(bar, s_ok)) return gave_up(a);

    // ---- G: every WG reads the per-row argmax (one agent-scope key per row) and applies
    // generate2's bookkeeping (greedy_step_kernel, gpt2.hip) to its copy of the row state
    {
      const int tid = otid();
      int alive = 0;
      if (tid < RM) {
        const unsigned long long key =
            __hip_atomic_load(lmkey + (step & 1) * RM + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int t = (int)~(unsigned)key;
        if (tid < a.R) {
          int d = s_done[tid];
          if (!d) {
            if (wg == 0) {
              a.out_ids[(long)tid * a.max_steps + step] = t;
              a.out_len[tid] = step + 1;
            }
            if (t == a.stop0 || t == a.stop1) d = 1;
          }
          alive = !d;
          s_done[tid] = d;
          s_tok[tid] = t;
          s_pos[tid] += 1;
        }
      }
      // rows 0..63 are the lanes of wave 0: one ballot counts the rows still decoding
      const unsigned long long bal = __ballot(alive);
      if (tid == 0) s_misc[0] = (int)__popcll(bal);
    }
    __syncthreads();
    stamp(bar.sb, 2 * DP_NB - 2);   // step end
    const int total = s_misc[0];
    const bool fin = total == 0 || step + 1 >= a.max_steps;
    if (fin) {
      const int tid = otid();
      if (wg == 0) {
        if (tid < a.R) {
          a.done[tid] = s_done[tid];
          a.pos[tid] = s_pos[tid];
          a.next_tok[tid] = s_tok[tid];
        }
        if (tid == 0) {
          *a.step_ctr = step + 1;
          a.all_done[0] = 1;
          a.all_done[2] = total;
        }
      }
      return;
    }
    ++step;
    __syncthreads();     // s_misc is rewritten next step
  }
}
#undef LOAD_WQ
#undef LOAD_WQ_H
#undef V_

}  // namespace dpk
}  // namespace zs

using namespace zs;

extern "C" int zs_decode_persist_workspace_bytes(void) { return dpk::WS_BYTES; }
extern "C" int zs_decode_persist_grid(void) { return dpk::G; }   // at col_split 1, row_split 1

extern "C" int zs_gpt2_decode_persist(int R, int Lmax, int max_steps, int stop0, int stop1, int V,
                                      const void* wte, const void* wpe, const void* wte_packed,
                                      float temperature, const void* const* layer_w,
                                      const float* lnf_w, const float* lnf_b, void* const* kv,
                                      int* pos, int* next_tok, int* done, int* out_ids,
                                      int* out_len, int* step_ctr, int* all_done, void* ws,
                                      long ws_bytes, int row_split, int col_split, void* stream) {
  using namespace dpk;
  ZS_REQUIRE(row_split == 1 || row_split == 2, "zs_gpt2_decode_persist: row_split 1 or 2 (got %d)",
             row_split);
  ZS_REQUIRE(col_split == 1 || col_split == 2, "zs_gpt2_decode_persist: col_split 1 or 2 (got %d)",
             col_split);
  // batches of <= 32 rows: the grid covers 1 or 2 row blocks (row_split 2 would leave a half
  // without rows; it is taken as 1, a grid no larger than the caller reserved)
  const int rb = R <= 32 ? 2 : 4;     // (one row block, RB 1, spilled 59 VGPRs: not built)
  if (rb < 4) row_split = 1;
  const int grid = G / col_split * row_split;
  ZS_REQUIRE(R >= 1 && R <= RM, "zs_gpt2_decode_persist: R in 1..%d (got %d)", RM, R);
  ZS_REQUIRE(V >= 32 * NW * grid && V <= 1 << 24, "zs_gpt2_decode_persist: vocab %d", V);
  ZS_REQUIRE(Lmax >= 2 && max_steps >= 1, "zs_gpt2_decode_persist: Lmax %d max_steps %d", Lmax, max_steps);
  ZS_REQUIRE(ws && ws_bytes >= WS_BYTES && ((uintptr_t)ws & 255) == 0,
             "zs_gpt2_decode_persist: workspace of %d bytes, 256-byte aligned", WS_BYTES);
  ZS_REQUIRE(temperature > 0.f, "zs_gpt2_decode_persist: temperature %g (> 0)", temperature);
  ZS_REQUIRE(wte_packed && ((uintptr_t)wte_packed & 15) == 0,
             "zs_gpt2_decode_persist: wte_packed null or not 16-byte aligned");
  ZS_REQUIRE(wte && wpe && layer_w && lnf_w && lnf_b && kv && pos && next_tok && done && out_ids &&
             out_len && step_ctr && all_done, "zs_gpt2_decode_persist: null pointer");
  Args a{};
  a.R = R; a.Lmax = Lmax; a.max_steps = max_steps; a.stop0 = stop0; a.stop1 = stop1; a.V = V;
  a.lm_il = g_dp_lmil;
  a.spin_max = g_dp_spin > 0 ? (unsigned)g_dp_spin : g_dp_spin < 0 ? 0u : SPIN_MAX;
  a.wte = (const bf16_t*)wte; a.wpe = (const bf16_t*)wpe;
  for (int l = 0; l < NLY; ++l) {
    const void* const* p = layer_w + 8 * l;
    for (int k = 0; k < 8; ++k)
      ZS_REQUIRE(p[k] && ((uintptr_t)p[k] & 15) == 0,
                 "zs_gpt2_decode_persist: layer %d pointer %d null or not 16-byte aligned", l, k);
    a.wqkv[l] = (const bf16_t*)p[0]; a.bqkv[l] = (const float*)p[1];
    a.wproj[l] = (const bf16_t*)p[2]; a.bproj[l] = (const float*)p[3];
    a.wfc[l] = (const bf16_t*)p[4]; a.bfc[l] = (const float*)p[5];
    a.wmp[l] = (const bf16_t*)p[6]; a.bmp[l] = (const float*)p[7];
    ZS_REQUIRE(kv[l] && kv[NLY + l], "zs_gpt2_decode_persist: KV cache pointer");
    a.kc[l] = (bf16_t*)kv[l];
    a.vc[l] = (bf16_t*)kv[NLY + l];
  }
  a.lnf_w = lnf_w; a.lnf_b = lnf_b; a.wtep = (const bf16_t*)wte_packed; a.temp = temperature;
  a.pos = pos; a.next_tok = next_tok; a.done = done; a.out_ids = out_ids; a.out_len = out_len;
  a.step_ctr = step_ctr; a.all_done = all_done; a.ws = (char*)ws;
  // the barrier counter and timeout word: zeroed before every launch (a memset node under capture)
  ZS_CHECK_HIP(hipMemsetAsync(ws, 0, WS_SYNC_BYTES, S(stream)));
#define DP_K(CS_, RH_, FUSE_, RB_) decode_persist_kernel<CS_, RH_, true, 2, FUSE_, RB_>
#define DP_GO(K_) hipLaunchKernelGGL((K_), dim3(grid), dim3(NT), 0, S(stream), a)
#define DP_LAUNCH(CS_, RH_)                                                                      \
  do {                                                                                           \
    if (rb == 2) DP_GO((DP_K(CS_, RH_, false, 2)));                                              \
    else if (g_dp_fuse) DP_GO((DP_K(CS_, RH_, true, 4)));                                        \
    else DP_GO((DP_K(CS_, RH_, false, 4)));                                                      \
  } while (0)
  if (col_split == 1) {
    if (row_split == 1) DP_LAUNCH(1, 1);
    else DP_GO((DP_K(1, 2, false, 4)));
  } else {
    if (row_split == 1) DP_LAUNCH(2, 1);
    else DP_GO((DP_K(2, 2, false, 4)));
  }
#undef DP_LAUNCH
#undef DP_GO
#undef DP_K
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_decode_persist_set_stamps(void* buf, int step) {
  ZS_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dpk::dp_stamp_buf), &buf, sizeof(buf)));
  ZS_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dpk::dp_stamp_step), &step, sizeof(step)));
  return 0;
}

// timeout word of the last launch on this workspace (non-zero: the grid was not co-resident and
// the launch gave up; the outputs are invalid).  Host-side read, after a synchronisation.
extern "C" int zs_decode_persist_status(const void* ws, int* timed_out) {
  ZS_REQUIRE(ws && timed_out, "zs_decode_persist_status: null pointer");
  unsigned t = 0;
  ZS_CHECK_HIP(hipMemcpy(&t, (const char*)ws + 4, 4, hipMemcpyDeviceToHost));
  *timed_out = (int)t;
  return 0;
}

// Attention kernels:
//  * window_attention  — HTSAT W-MSA / SW-MSA (htsat.py:312-347), roll + partition folded in;
//  * row_attention     — dense per-row attention (TransformerMapper MHA, GPT-2 prompt prefill);
//  * decode_attention  — one new token per row against the KV cache (GPT-2 decode), with an
//                        optional per-position row indirection for beam search;
//  * kv_write          — prefill K/V into the cache.
// Softmax statistics are f32; one wave per query block.
#include "common.h"

namespace zs {

int g_small_attn = 1;     // R <= 128: decode_attn6 with 128-key phases
int g_small_rmax = 128;   // zs_tune_set("small_rmax", r): the row count up to which the small-R
                          // decode attention kernels are taken
int g_beam_xcd = 5;       // zs_tune_set("beam_xcd", g): beam-row groups per XCD (1 = off)
int g_decode_attn5 = 6;   // 6: decode_attn6 16-key phases, DPP reductions; 5: + next-phase prefetch; 4/3/2: decode_attn6 (phases of 16/32/64 keys), 1: decode_attn5, 0: LDS
int g_window_mfma = 1;    // zs_tune_set("window_mfma", 0): VALU window attention for bf16   // zs_tune_set("decode_attn5", 0): LDS-staged decode_attn4 for bf16

// ------------------------------------------------------------------ HTSAT window attention
// grid (B * nWh * nWw, heads), block 64: thread i = token i of the 8x8 window.
template <typename T, int HD>
__global__ __launch_bounds__(64) void window_attn_kernel(const T* __restrict__ qkv, int H, int W,
                                                         int C, int heads, int shift,
                                                         const float* __restrict__ table,
                                                         T* __restrict__ out) {
  constexpr int WS = 8, N = 64;
  __shared__ float Ks[N][HD + 1];
  __shared__ float Vs[N][HD + 1];
  const int nWw = W / WS, nWh = H / WS;
  const int win = blockIdx.x, head = blockIdx.y;
  const int b = win / (nWh * nWw), wyx = win % (nWh * nWw), wy = wyx / nWw, wx = wyx % nWw;
  const int i = threadIdx.x, iy = i / WS, ix = i % WS;
  const int sy = wy * WS + iy, sx = wx * WS + ix;           // coords in the rolled image
  const int hh = (sy + shift) % H, ww = (sx + shift) % W;   // natural coords (roll(-shift))
  const long tok = ((long)b * H + hh) * W + ww;
  const T* row = qkv + tok * 3 * C + head * HD;
  const float scale = rsqrtf((float)HD);
  float q[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    q[d] = ldf(row + d) * scale;
    Ks[i][d] = ldf(row + C + d);
    Vs[i][d] = ldf(row + 2 * C + d);
  }
  // shift-mask region label of this token (htsat.py:406-425 slices on rolled coords)
  auto region = [&](int y, int x) {
    const int ry = y < H - WS ? 0 : (y < H - shift ? 1 : 2);
    const int rx = x < W - WS ? 0 : (x < W - shift ? 1 : 2);
    return ry * 3 + rx;
  };
  const int my_reg = shift > 0 ? region(sy, sx) : 0;
  __syncthreads();
  float s[N];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    float acc = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) acc += q[d] * Ks[j][d];
    const int jy = j / WS, jx = j % WS;
    acc += table[((iy - jy + WS - 1) * (2 * WS - 1) + (ix - jx + WS - 1)) * heads + head];
    if (shift > 0 && region(wy * WS + jy, wx * WS + jx) != my_reg) acc += -100.0f;
    s[j] = acc;
    mx = fmaxf(mx, acc);
  }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    s[j] = expf(s[j] - mx);
    sum += s[j];
  }
  const float inv = 1.0f / sum;
  float o[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) o[d] = 0.f;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const float p = s[j] * inv;
#pragma unroll
    for (int d = 0; d < HD; ++d) o[d] += p * Vs[j][d];
  }
  T* orow = out + tok * C + head * HD;
#pragma unroll
  for (int d = 0; d < HD; ++d) stf(orow + d, o[d]);
}

// MFMA window attention (bf16, head_dim <= 32, zero-padded to 32): one wave per (window, head).
//   S^T[key][query] = K . Q^T           (2x2 tiles of v_mfma_f32_32x32x16_bf16, K-dim = head dim)
//   + rel-pos bias + shift mask, softmax over keys per query column: a lane holds 32 of a query's
//     64 keys, the other 32 sit in lane^32 (one xor-32 exchange)
//   O^T[dim][query] = V^T . P^T         (P^T straight from the S^T accumulators as the B operand)
// The accumulator's key order within a 16-deep k-step is {0-3, 8-11} for lane half 0 and
// {4-7, 12-15} for half 1, so the A operand V^T is read with the same key permutation (the sum
// over keys is order-free).  Q and K are staged [token][32] with the 16-byte slot XOR-swizzled by
// (token >> 2) & 3; V^T [dim][64] with 8-byte key chunks XOR-swizzled by dim & 15: the fragment
// reads are bank-conflict-free.  1/sqrt(hd) is applied to the scores (htsat.py:320 scales q).
typedef __attribute__((ext_vector_type(8))) __bf16 wa_bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float wa_f32x16_t;
constexpr int WA_NW = 4;   // windows-heads (waves) per block
__global__ __launch_bounds__(64 * WA_NW) void window_attn_mfma_kernel(
    const bf16_t* __restrict__ qkv, int H, int W, int C, int heads, int hd, int shift,
    const float* __restrict__ table, bf16_t* __restrict__ out, int total) {
  constexpr int WS = 8, N = 64;
  __shared__ __attribute__((aligned(16))) bf16_t sQ[WA_NW][N * 32];
  __shared__ __attribute__((aligned(16))) bf16_t sK[WA_NW][N * 32];
  __shared__ __attribute__((aligned(16))) bf16_t sVt[WA_NW][32 * N];
  __shared__ float sB[WA_NW][225];
  __shared__ int sReg[WA_NW][N];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int item = blockIdx.x * WA_NW + wv;          // (window, head) index, head fastest
  if (item >= total) return;
  const int head = item % heads, win = item / heads;
  const int nWw = W / WS, nWh = H / WS;
  const int b = win / (nWh * nWw), wyx = win % (nWh * nWw), wy = wyx / nWw, wx = wyx % nWw;
  bf16_t* Q = sQ[wv];
  bf16_t* K = sK[wv];
  bf16_t* Vt = sVt[wv];
  float* Bt = sB[wv];
  int* Rg = sReg[wv];
  // ---- stage: lane = token of the window
  {
    const int i = lane, iy = i / WS, ix = i % WS;
    const int sy = wy * WS + iy, sx = wx * WS + ix;           // coords in the rolled image
    const int hh = (sy + shift) % H, ww = (sx + shift) % W;   // natural coords (roll(-shift))
    const long tok = ((long)b * H + hh) * W + ww;
    const bf16_t* row = qkv + tok * 3 * C + head * hd;
    const int sw = (i >> 2) & 3;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint4 qv = make_uint4(0, 0, 0, 0), kv = make_uint4(0, 0, 0, 0);
      if (8 * c < hd) {
        qv = *reinterpret_cast<const uint4*>(row + 8 * c);
        kv = *reinterpret_cast<const uint4*>(row + C + 8 * c);
      }
      *reinterpret_cast<uint4*>(Q + i * 32 + 8 * (c ^ sw)) = qv;
      *reinterpret_cast<uint4*>(K + i * 32 + 8 * (c ^ sw)) = kv;
    }
    // V^T: element (d, key i) at row d, 4-key chunk (i/4) ^ (d & 15), slot i % 4
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint4 vv = make_uint4(0, 0, 0, 0);
      if (8 * c < hd) vv = *reinterpret_cast<const uint4*>(row + 2 * C + 8 * c);
      const bf16_t* e = reinterpret_cast<const bf16_t*>(&vv);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int d = 8 * c + t;
        Vt[d * N + 4 * ((i >> 2) ^ (d & 15)) + (i & 3)] = e[t];
      }
    }
    for (int r = lane; r < 225; r += 64) Bt[r] = table[r * heads + head];
    int reg = 0;
    if (shift > 0) {
      const int ry = sy < H - WS ? 0 : (sy < H - shift ? 1 : 2);
      const int rx = sx < W - WS ? 0 : (sx < W - shift ? 1 : 2);
      reg = ry * 3 + rx;
    }
    Rg[i] = reg;
  }
  // the staged tiles are private to this wave: its LDS accesses complete in issue order
  const int r = lane & 31, h = lane >> 5;
  // ---- S^T = K . Q^T : tiles (key block kb, query block qb)
  wa_f32x16_t st[2][2];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int e = 0; e < 16; ++e) st[kb][qb][e] = 0.f;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {                    // head-dim slices of 16
    const int c = 2 * ks + h;                         // 16-byte slot of this lane half
    wa_bf16x8_t a[2], bq[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = 32 * t + r;
      a[t] = *reinterpret_cast<const wa_bf16x8_t*>(K + row * 32 + 8 * (c ^ ((row >> 2) & 3)));
      bq[t] = *reinterpret_cast<const wa_bf16x8_t*>(Q + row * 32 + 8 * (c ^ ((row >> 2) & 3)));
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
        st[kb][qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[kb], bq[qb], st[kb][qb], 0, 0, 0);
  }
  // ---- bias + mask + softmax over keys (per query column)
  const float scale = rsqrtf((float)hd);
  wa_f32x16_t ot[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qi = 32 * qb + r, qy = qi / WS, qx = qi % WS, qreg = Rg[qi];
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int kj = 32 * kb + (e & 3) + 8 * (e >> 2) + 4 * h, ky = kj / WS, kx = kj % WS;
        float v = st[kb][qb][e] * scale + Bt[(qy - ky + WS - 1) * (2 * WS - 1) + (qx - kx + WS - 1)];
        if (shift > 0 && Rg[kj] != qreg) v += -100.0f;
        st[kb][qb][e] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float p = expf(st[kb][qb][e] - mx);
        st[kb][qb][e] = p;
        sum += p;
      }
    sum += __shfl_xor(sum, 32, 64);
    // ---- O^T[dim][query] = V^T . P^T over 64 keys (4 k-steps of 16)
#pragma unroll
    for (int e = 0; e < 16; ++e) ot[qb][e] = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        wa_bf16x8_t pb;
#pragma unroll
        for (int u = 0; u < 8; ++u) pb[u] = (__bf16)st[kb][qb][8 * t + u];
        // A: V^T rows d = r, keys 32kb + 16t + {0-3, 8-11} (+4 for half 1)
        const int k0 = 32 * kb + 16 * t + 4 * h;
        const int d = r;
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;
        const bf16x4_t lo = *reinterpret_cast<const bf16x4_t*>(Vt + d * N + 4 * ((k0 >> 2) ^ (d & 15)));
        const bf16x4_t hi = *reinterpret_cast<const bf16x4_t*>(Vt + d * N + 4 * (((k0 + 8) >> 2) ^ (d & 15)));
        wa_bf16x8_t va;
#pragma unroll
        for (int u = 0; u < 4; ++u) { va[u] = lo[u]; va[4 + u] = hi[u]; }
        ot[qb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb, ot[qb], 0, 0, 0);
      }
    // ---- normalise and store: lane holds dims (e&3) + 8(e>>2) + 4h of query qi
    const float inv = 1.0f / sum;
    const int sy = wy * WS + qy, sx = wx * WS + qx;
    const int hh = (sy + shift) % H, ww = (sx + shift) % W;
    bf16_t* orow = out + (((long)b * H + hh) * W + ww) * C + head * hd;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = 8 * g + 4 * h;
      if (d0 < hd) {
        uint2 u;
        u.x = pk2bf(ot[qb][4 * g] * inv, ot[qb][4 * g + 1] * inv);
        u.y = pk2bf(ot[qb][4 * g + 2] * inv, ot[qb][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d0) = u;
      }
    }
  }
}

// ------------------------------------------------------------------ dense row attention
// grid (B, heads, ceil(L/64)), block 64: thread = query i; K/V of the row staged in LDS.
template <typename T, int HD>
__global__ __launch_bounds__(64) void row_attn_kernel(const T* __restrict__ q, int ldq,
                                                      const T* __restrict__ k,
                                                      const T* __restrict__ v, int ldkv, int L,
                                                      const int* __restrict__ lens, int causal,
                                                      float scale, T* __restrict__ out, int ldo) {
  extern __shared__ float sm[];  // K [L][HD] then V [L][HD]
  float* Ks = sm;
  float* Vs = sm + L * HD;
  const int b = blockIdx.x, h = blockIdx.y;
  const int len = lens ? lens[b] : L;
  for (int e = threadIdx.x; e < len * HD; e += 64) {
    const int j = e / HD, d = e % HD;
    const long off = ((long)b * L + j) * ldkv + h * HD + d;
    Ks[e] = ldf(k + off);
    Vs[e] = ldf(v + off);
  }
  __syncthreads();
  const int i = blockIdx.z * 64 + threadIdx.x;
  if (i >= L) return;
  float qr[HD], o[HD];
  const T* qrow = q + ((long)b * L + i) * ldq + h * HD;
#pragma unroll
  for (int d = 0; d < HD; ++d) { qr[d] = ldf(qrow + d); o[d] = 0.f; }
  const int jend = causal ? min(i + 1, len) : len;
  float m = -INFINITY, l = 0.f;
  for (int j = 0; j < jend; ++j) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) s += qr[d] * Ks[j * HD + d];
    s *= scale;
    const float mn = fmaxf(m, s);
    const float corr = expf(m - mn), p = expf(s - mn);
    l = l * corr + p;
#pragma unroll
    for (int d = 0; d < HD; ++d) o[d] = o[d] * corr + p * Vs[j * HD + d];
    m = mn;
  }
  const float inv = l > 0.f ? 1.0f / l : 0.f;
  T* orow = out + ((long)b * L + i) * ldo + h * HD;
#pragma unroll
  for (int d = 0; d < HD; ++d) stf(orow + d, o[d] * inv);
}

// MFMA row attention for short rows (bf16, head dim 64, L <= 32: the GPT-2 prompt prefill, P =
// hard prompt + 10 soft tokens <= 27): one wave per (row, head), 4 per block.
//   S^T[key][query] = K . Q^T   4 x v_mfma_f32_32x32x16_bf16 (head dim in 16-deep steps), both
//                               operands loaded straight from global as 16-byte fragments
//   mask (key < len, causal key <= query), scale, f32 softmax over keys per query column (a lane
//   holds 16 of its query's 32 keys, the other 16 sit in lane ^ 32)
//   O^T[dim][query] = V^T . P^T 2 dim tiles x 2 key steps; P^T straight from the S^T accumulators
//                               (bf16), V^T staged in LDS (swizzled 4-key chunks, 8-byte reads)
// The scalar row_attn_kernel (one thread per query, 64-dim dot products from LDS) ran ~4k VALU
// instructions per thread for what is 8 MFMAs per wave here.
constexpr int RA_NW = 4;
// kc != nullptr (zs_row_attention_kv, the GPT-2 prefill): the wave also stores its (row, head)'s
// L keys and values into the KV cache, slot ((b * row_stride * heads + head) * Lmax + j) * 64 --
// zs_kv_write's layout and values (the bf16 qkv elements as they are), from the fragments it
// loads anyway: one launch and one read of k / v per layer instead of two.
__global__ __launch_bounds__(64 * RA_NW) void row_attn_mfma_kernel(
    const bf16_t* __restrict__ q, int ldq, const bf16_t* __restrict__ k,
    const bf16_t* __restrict__ v, int ldkv, int L, const int* __restrict__ lens, int causal,
    float scale, bf16_t* __restrict__ out, int ldo, int B, int heads,
    bf16_t* __restrict__ kc = nullptr, bf16_t* __restrict__ vc = nullptr, int Lmax = 0,
    int row_stride = 1) {
  __shared__ __attribute__((aligned(16))) bf16_t sVt[RA_NW][64 * 32];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int item = blockIdx.x * RA_NW + wv;
  if (item >= B * heads) return;
  const int b = item / heads, hh = item % heads;
  const int len = lens ? lens[b] : L;
  const int r = lane & 31, h = lane >> 5;
  bf16_t* Vt = sVt[wv];
  // V^T [dim][key]: element (d, key j) at d*32 + 4*((j >> 2) ^ (d & 7)) + (j & 3)
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int j = 8 * it + (lane >> 3), d0 = 8 * (lane & 7);
    uint4 u = make_uint4(0, 0, 0, 0);
    if (j < L) u = *reinterpret_cast<const uint4*>(v + ((long)b * L + j) * ldkv + hh * 64 + d0);
    if (vc && j < L)
      *reinterpret_cast<uint4*>(vc + (((long)b * row_stride * heads + hh) * Lmax + j) * 64 + d0) = u;
    const bf16_t* e = reinterpret_cast<const bf16_t*>(&u);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int d = d0 + t;
      Vt[d * 32 + 4 * ((j >> 2) ^ (d & 7)) + (j & 3)] = e[t];
    }
  }
  // S^T = K . Q^T over the 64 head dims
  wa_f32x16_t st;
#pragma unroll
  for (int e = 0; e < 16; ++e) st[e] = 0.f;
  const bf16_t* krow = k + ((long)b * L + r) * ldkv + hh * 64 + 8 * h;
  const bf16_t* qrow = q + ((long)b * L + r) * ldq + hh * 64 + 8 * h;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    uint4 ku = make_uint4(0, 0, 0, 0), qu = make_uint4(0, 0, 0, 0);
    if (r < L) {
      ku = *reinterpret_cast<const uint4*>(krow + 16 * ks);
      qu = *reinterpret_cast<const uint4*>(qrow + 16 * ks);
      if (kc)
        *reinterpret_cast<uint4*>(kc + (((long)b * row_stride * heads + hh) * Lmax + r) * 64 +
                                  16 * ks + 8 * h) = ku;
    }
    st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(wa_bf16x8_t, ku),
                                                  __builtin_bit_cast(wa_bf16x8_t, qu), st, 0, 0, 0);
  }
  // softmax over the keys of query column r
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int j = (e & 3) + 8 * (e >> 2) + 4 * h;
    const bool ok = j < len && (!causal || j <= r);
    st[e] = ok ? st[e] * scale : -INFINITY;
    mx = fmaxf(mx, st[e]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float p = st[e] == -INFINITY ? 0.f : __expf(st[e] - mx);
    st[e] = p;
    sum += p;
  }
  sum += __shfl_xor(sum, 32, 64);
  // V^T is private to this wave and a wave's LDS accesses complete in issue order: no barrier
  wa_bf16x8_t pb[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 8; ++u) pb[t][u] = (__bf16)st[8 * t + u];
  const float inv = sum > 0.f ? 1.0f / sum : 0.f;
  typedef __attribute__((ext_vector_type(4))) __bf16 ra_bf16x4_t;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    wa_f32x16_t ot;
#pragma unroll
    for (int e = 0; e < 16; ++e) ot[e] = 0.f;
    const int d = 32 * dt + r;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k0 = 16 * t + 4 * h;
      const ra_bf16x4_t lo = *reinterpret_cast<const ra_bf16x4_t*>(Vt + d * 32 + 4 * ((k0 >> 2) ^ (d & 7)));
      const ra_bf16x4_t hi = *reinterpret_cast<const ra_bf16x4_t*>(Vt + d * 32 + 4 * (((k0 + 8) >> 2) ^ (d & 7)));
      wa_bf16x8_t va;
#pragma unroll
      for (int u = 0; u < 4; ++u) { va[u] = lo[u]; va[4 + u] = hi[u]; }
      ot = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb[t], ot, 0, 0, 0);
    }
    if (r < L) {
      bf16_t* orow = out + ((long)b * L + r) * ldo + hh * 64 + 32 * dt;
#pragma unroll
      for (int g = 0; g < 4; ++g) {      // dims 8 g + 4 h .. +3 of this tile
        uint2 u;
        u.x = pk2bf(ot[4 * g] * inv, ot[4 * g + 1] * inv);
        u.y = pk2bf(ot[4 * g + 2] * inv, ot[4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 8 * g + 4 * h) = u;
      }
    }
  }
}

int g_attn_split = 3;   // zs_tune_set("attn_split", v) at R <= 128: 0 one wave per (row, head),
                        // 1 two waves (64-key phases), 3 two waves (32-key), 4 four waves (32-key)
int g_row_mfma = 1;   // zs_tune_set("row_mfma", 0): the scalar row_attn_kernel for bf16 too

// ------------------------------------------------------------------ GPT-2 decode attention
// grid (R, heads), block 256 (hd == 64): append k/v of the new token at pos[r], then attend
// 0..pos[r].  The row's K block ([pos][64], contiguous per (row, head) in the cache) is staged
// into LDS with 16-byte coalesced loads, one thread per key computes its score from LDS, the
// softmax is a block reduction, and P.V reads each V row coalesced (wave w takes keys j = w mod 4).
template <typename T>
__global__ __launch_bounds__(256) void decode_attn4_kernel(const T* __restrict__ qkv, int D,
                                                           int heads, T* __restrict__ kc,
                                                           T* __restrict__ vc, int Lmax,
                                                           const int* __restrict__ pos,
                                                           const int* __restrict__ kvrow,
                                                           T* __restrict__ out) {
  constexpr int HD = 64, KP = HD + 1;
  constexpr int EPC = 16 / sizeof(T);          // elements per 16-byte chunk
  constexpr int CPR = HD / EPC;                // chunks per key row
  extern __shared__ float sm[];
  float* qs = sm;                    // [64]
  float* vnew = sm + 64;             // [64]
  float* red = sm + 128;             // [16]
  float* po = sm + 144;              // [4][64] partial outputs
  float* sc = sm + 144 + 256;        // [Lmax] scores
  float* ks = sc + Lmax;             // [Lmax][65] keys
  const int r = blockIdx.x, h = blockIdx.y, tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int p = min(pos[r], Lmax - 1);
  const T* row = qkv + (long)r * 3 * D + h * HD;
  const long base_rh = ((long)r * heads + h) * Lmax;
  if (tid < HD) {
    qs[tid] = ldf(row + tid) * 0.125f;              // q * 1/sqrt(64) (exact power of two)
    const T kn = row[D + tid], vn = row[2 * D + tid];
    kc[(base_rh + p) * HD + tid] = kn;
    vc[(base_rh + p) * HD + tid] = vn;
    ks[p * KP + tid] = Cvt<T>::to_f(kn);
    vnew[tid] = Cvt<T>::to_f(vn);
  }
  // stage keys 0..p-1
  for (int c = tid; c < p * CPR; c += 256) {
    const int j = c / CPR, part = c % CPR;
    const int pr = kvrow ? kvrow[(long)r * Lmax + j] : r;
    const uint4 u = *reinterpret_cast<const uint4*>(
        kc + ((((long)pr * heads + h) * Lmax + j) * HD) + part * EPC);
    const T* e = reinterpret_cast<const T*>(&u);
#pragma unroll
    for (int q = 0; q < EPC; ++q) ks[j * KP + part * EPC + q] = Cvt<T>::to_f(e[q]);
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int j = tid; j <= p; j += 256) {
    float s = 0.f;
#pragma unroll 16
    for (int e = 0; e < HD; ++e) s += qs[e] * ks[j * KP + e];
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  if (lane == 0) red[wid] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sum = 0.f;
  for (int j = tid; j <= p; j += 256) {
    const float e = expf(sc[j] - mx);
    sc[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if (lane == 0) red[4 + wid] = sum;
  __syncthreads();
  const float inv = 1.0f / (red[4] + red[5] + red[6] + red[7]);
  float o = 0.f;
  for (int j = wid; j < p; j += 4) {
    const int pr = kvrow ? kvrow[(long)r * Lmax + j] : r;
    o += sc[j] * ldf(vc + (((long)pr * heads + h) * Lmax + j) * HD + lane);
  }
  if (wid == (p & 3)) o += sc[p] * vnew[lane];
  po[wid * 64 + lane] = o;
  __syncthreads();
  if (wid == 0)
    stf(out + (long)r * D + h * HD + lane,
        (po[lane] + po[64 + lane] + po[128 + lane] + po[192 + lane]) * inv);
}

// Register-resident decode attention (bf16, Lmax <= DA5_MAXK): one wave per (row, head), 4 heads
// of a row per block.  A lane owns 8 head dims (one 16-byte chunk) of key j = 8*i + lane/8, so one
// wave-instruction reads 8 consecutive cached keys = 1 KiB contiguous (the cache is
// [row][head][pos][64]); every K and V load of the row is issued up front (no LDS, no barrier),
// the q.k partial is reduced over the key's 8 lanes (xor 1,2,4), the softmax statistics and the
// P.V partials over the 8 key groups (xor 8,16,32).  The new token's k/v (position pos[r]) comes
// from the qkv row in registers and is written to the cache for later steps.  HBM-bound on the
// K/V bytes: 2 * (pos+1) * 64 * 2 B per (row, head).
constexpr int DA5_MAXI = 16;                 // key groups of 8 -> up to 128 positions
template <typename T>
__global__ __launch_bounds__(256) void decode_attn5_kernel(const T* __restrict__ qkv, int D,
                                                           int heads, T* __restrict__ kc,
                                                           T* __restrict__ vc, int Lmax,
                                                           const int* __restrict__ pos,
                                                           const int* __restrict__ kvrow,
                                                           T* __restrict__ out,
                                                           const int* __restrict__ rowmap,
                                                           int nphys) {
  static_assert(sizeof(T) == 2, "bf16 only");
  constexpr int HD = 64, EPC = 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.x, h = blockIdx.y * 4 + wid;   // c: compact row of qkv / out
  if (h >= heads) return;
  const int grp = lane >> 3, sub = lane & 7;
  const int r = rowmap ? rowmap[c] : c;                  // r: physical row of pos / cache
  if (r >= nphys) {                                      // padding slot of a compacted step
    if (grp == 0)
      *reinterpret_cast<uint4*>(out + (long)c * D + h * HD + sub * EPC) = make_uint4(0, 0, 0, 0);
    return;
  }
  const int p = min(pos[r], Lmax - 1);
  const T* row = qkv + (long)c * 3 * D + h * HD + sub * EPC;
  const uint4 qu = *reinterpret_cast<const uint4*>(row);
  const uint4 knu = *reinterpret_cast<const uint4*>(row + D);
  const uint4 vnu = *reinterpret_cast<const uint4*>(row + 2 * D);
  const long rh = ((long)r * heads + h) * Lmax;
  if (grp == 0) {        // append this step's k/v to the cache
    *reinterpret_cast<uint4*>(kc + (rh + p) * HD + sub * EPC) = knu;
    *reinterpret_cast<uint4*>(vc + (rh + p) * HD + sub * EPC) = vnu;
  }
  float q[EPC];
  {
    const T* e = reinterpret_cast<const T*>(&qu);
#pragma unroll
    for (int t = 0; t < EPC; ++t) q[t] = ldf(e + t) * 0.125f;   // 1/sqrt(64), exact
  }
  const int nI = (p + 1 + 7) >> 3;
  uint4 kr[DA5_MAXI], vr[DA5_MAXI];
#pragma unroll
  for (int i = 0; i < DA5_MAXI; ++i) {
    const int j = i * 8 + grp;
    kr[i] = make_uint4(0, 0, 0, 0);
    vr[i] = make_uint4(0, 0, 0, 0);
    if (i < nI && j < p) {
      const long src = kvrow ? ((long)kvrow[(long)r * Lmax + j] * heads + h) * Lmax : rh;
      kr[i] = *reinterpret_cast<const uint4*>(kc + (src + j) * HD + sub * EPC);
      vr[i] = *reinterpret_cast<const uint4*>(vc + (src + j) * HD + sub * EPC);
    } else if (j == p) {
      kr[i] = knu;
      vr[i] = vnu;
    }
  }
  float sc[DA5_MAXI];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < DA5_MAXI; ++i) {
    const T* e = reinterpret_cast<const T*>(&kr[i]);
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < EPC; ++t) s += q[t] * ldf(e + t);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    sc[i] = (i * 8 + grp <= p) ? s : -INFINITY;
    mx = fmaxf(mx, sc[i]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 8, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f, o[EPC];
#pragma unroll
  for (int t = 0; t < EPC; ++t) o[t] = 0.f;
#pragma unroll
  for (int i = 0; i < DA5_MAXI; ++i) {
    const float e = (i * 8 + grp <= p) ? expf(sc[i] - mx) : 0.f;
    sum += e;
    const T* v = reinterpret_cast<const T*>(&vr[i]);
#pragma unroll
    for (int t = 0; t < EPC; ++t) o[t] += e * ldf(v + t);
  }
#pragma unroll
  for (int d = 8; d < 64; d <<= 1) {
    sum += __shfl_xor(sum, d, 64);
#pragma unroll
    for (int t = 0; t < EPC; ++t) o[t] += __shfl_xor(o[t], d, 64);
  }
  if (grp == 0) {
    const float inv = 1.0f / sum;
    uint4 ou;
    T* oe = reinterpret_cast<T*>(&ou);
#pragma unroll
    for (int t = 0; t < EPC; ++t) stf(oe + t, o[t] * inv);
    *reinterpret_cast<uint4*>(out + (long)c * D + h * HD + sub * EPC) = ou;
  }
}

// decode_attn6: decode_attn5's wave-per-(row, head) layout with the keys taken in phases of 64
// (8 key groups x 8 keys, one 1 KiB wave-load each for K and V) and an online softmax across
// phases, so a wave holds 64 keys' K/V in registers instead of 128 (~100 VGPRs: 4 waves per
// SIMD instead of 2) and any Lmax works.  The per-slot inputs (rowmap, compact position) are
// loaded together with the qkv row: one dependent round trip before the K/V loads.  With one
// phase (p < 64) the arithmetic equals decode_attn5's.
// DPP lane exchanges for the reductions inside a wave (VALU, no LDS round trip):
// xor 1 / xor 2 = quad_perm [1,0,3,2] / [2,3,0,1]; the other quad of an 8-lane group via
// row_half_mirror (lane i <-> 7 - i), valid once the value is uniform within each quad; the other
// 8-lane group of a 16-lane row via row_mirror (i <-> 15 - i), valid once uniform within groups
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
// sum over the 8 lanes of a group: the same additions, in the same order, as
// s += shfl_xor(s, 1); s += shfl_xor(s, 2); s += shfl_xor(s, 4)  (bitwise equal results)
__device__ __forceinline__ float group8_sum_dpp(float s) {
  s += dpp_f<0xB1>(s);
  s += dpp_f<0x4E>(s);
  return s + dpp_f<0x141>(s);
}

// PF: the next phase's K/V loads are issued before the current phase's math (two phases in
// flight per wave; the wait lands after the math instead of before it).  DPP: the in-group dot
// product reduction and the first step of the cross-group max by DPP instead of ds_bpermute.
// 8 bf16 in a uint4 <-> 8 floats by bit operations (element t in the low / high half of word
// t / 2): no type-punned pointer into a register array, which kept such arrays in scratch memory
__device__ __forceinline__ void bf8_unpack(const uint4& u, float (&f)[8]) {
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
  f[4] = __uint_as_float(u.z << 16); f[5] = __uint_as_float(u.z & 0xffff0000u);
  f[6] = __uint_as_float(u.w << 16); f[7] = __uint_as_float(u.w & 0xffff0000u);
}
// component-wise select (a select of whole uint4 structs went through scratch memory)
__device__ __forceinline__ uint4 sel_u4(bool c, const uint4& a, const uint4& b) {
  return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}
__device__ __forceinline__ uint4 bf8_pack(const float (&f)[8]) {
  return make_uint4(pk2bf(f[0], f[1]),
                    pk2bf(f[2], f[3]),
                    pk2bf(f[4], f[5]),
                    pk2bf(f[6], f[7]));
}

// 8 consecutive elements of a head row as one register packet: one uint4 of bf16, or two of f32
// (the f32 parity mode), with the same unpack / select / pack interface
template <typename T> struct Pk8;
template <> struct Pk8<bf16_t> {
  uint4 u;
  __device__ static Pk8 ld(const bf16_t* p) { return {*reinterpret_cast<const uint4*>(p)}; }
  __device__ void st(bf16_t* p) const { *reinterpret_cast<uint4*>(p) = u; }
  __device__ void unpack(float (&f)[8]) const { bf8_unpack(u, f); }
  __device__ static Pk8 sel(bool c, const Pk8& a, const Pk8& b) { return {sel_u4(c, a.u, b.u)}; }
  __device__ static Pk8 zero() { return {make_uint4(0, 0, 0, 0)}; }
  __device__ static Pk8 pack(const float (&f)[8]) { return {bf8_pack(f)}; }
};
template <> struct Pk8<float> {
  uint4 lo, hi;
  __device__ static Pk8 ld(const float* p) {
    return {*reinterpret_cast<const uint4*>(p), *reinterpret_cast<const uint4*>(p + 4)};
  }
  __device__ void st(float* p) const {
    *reinterpret_cast<uint4*>(p) = lo;
    *reinterpret_cast<uint4*>(p + 4) = hi;
  }
  __device__ void unpack(float (&f)[8]) const {
    f[0] = __uint_as_float(lo.x); f[1] = __uint_as_float(lo.y);
    f[2] = __uint_as_float(lo.z); f[3] = __uint_as_float(lo.w);
    f[4] = __uint_as_float(hi.x); f[5] = __uint_as_float(hi.y);
    f[6] = __uint_as_float(hi.z); f[7] = __uint_as_float(hi.w);
  }
  __device__ static Pk8 sel(bool c, const Pk8& a, const Pk8& b) {
    return {sel_u4(c, a.lo, b.lo), sel_u4(c, a.hi, b.hi)};
  }
  __device__ static Pk8 zero() { return {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)}; }
  __device__ static Pk8 pack(const float (&f)[8]) {
    return {make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]),
                       __float_as_uint(f[3])),
            make_uint4(__float_as_uint(f[4]), __float_as_uint(f[5]), __float_as_uint(f[6]),
                       __float_as_uint(f[7]))};
  }
};

// SPLIT = 2 / 4: the keys of one (row, head) are split over SPLIT waves of the workgroup (slice s
// takes phases s, s + SPLIT, ...; 4 / SPLIT heads per workgroup), whose online-softmax states are
// merged through LDS at the end: SPLIT times the waves for the bs=64 decode's 768 (row, head)
// pairs, each with a shorter chain of phases (requires heads % (4 / SPLIT) == 0, rows without
// rowmap; no early exit before the barrier).
template <typename T, int KPP = 64, bool PF = false, bool DPP = false, int SPLIT = 1>
__global__ __launch_bounds__(256) void decode_attn6_kernel(
    const T* __restrict__ qkv, int D, int heads, T* __restrict__ kc, T* __restrict__ vc, int Lmax,
    const int* __restrict__ pos, const int* __restrict__ kvrow, T* __restrict__ out,
    const int* __restrict__ rowmap, const int* __restrict__ cpos, int nphys, int rgrp) {
  using V8 = Pk8<T>;
  static_assert(SPLIT == 1 || ((SPLIT == 2 || SPLIT == 4) && !PF), "SPLIT 2 / 4 without prefetch");
  constexpr int HD = 64, EPC = 8, NG = KPP / 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int slice = wid % SPLIT;
  // rgrp > 1 (beam search, gridDim.x % (8 rgrp) == 0): rows in groups of rgrp consecutive rows
  // (one clip's beams, whose cached prompt and shared history are the same cache rows through
  // kvrow) go to one XCD at about the same time (workgroups are dealt round-robin over the 8 XCDs:
  // b and b + 8 share one), so a group's shared keys are read from HBM once and from L2 after
  const int c = rgrp > 1 ? ((blockIdx.x & 7) + 8 * ((blockIdx.x >> 3) / rgrp)) * rgrp +
                               (blockIdx.x >> 3) % rgrp
                         : blockIdx.x;
  const int h = blockIdx.y * (4 / SPLIT) + wid / SPLIT;
  __shared__ float merge[SPLIT == 1 ? 1 : 4][66];
  if (SPLIT == 1 && h >= heads) return;
  const int grp = lane >> 3, sub = lane & 7;
  const int r = rowmap ? rowmap[c] : c;
  const int p0 = cpos ? cpos[c] : 0;
  const T* row = qkv + (long)c * 3 * D + h * HD + sub * EPC;
  const V8 qu = V8::ld(row);
  const V8 knu = V8::ld(row + D);
  const V8 vnu = V8::ld(row + 2 * D);
  if (r >= nphys) {
    if (grp == 0) V8::zero().st(out + (long)c * D + h * HD + sub * EPC);
    return;
  }
  // wave-uniform (one (row, head) per wave): scalar branches for the phase loop and prefetch
  const int p = __builtin_amdgcn_readfirstlane(min(cpos ? p0 : pos[r], Lmax - 1));
  const long rh = ((long)r * heads + h) * Lmax;
  // the new token's K/V are stored at the END: the phases never read slot p (they take the new
  // token from registers), and a store here would order every cache load after it -- the qkv
  // load, the store and the cache loads became three dependent round trips instead of two
  float q[EPC];
  qu.unpack(q);
#pragma unroll
  for (int t = 0; t < EPC; ++t) q[t] *= 0.125f;
  float m = -INFINITY, sum = 0.f, o[EPC];
#pragma unroll
  for (int t = 0; t < EPC; ++t) o[t] = 0.f;
  // Branch-free phase load: every lane loads a valid cache slot (keys past p - 1 re-read slot
  // min(j, p - 1), or slot 0 at p == 0) and the key is then chosen by value: cached for j < p,
  // the new token for j == p, zero past it.  (Loads under a divergent `if` were each waited
  // for inside their branch: one round trip per key group instead of one per phase.)
  V8 kr[NG], vr[NG], kx[NG], vx[NG];
  // (beam: the kvrow source rows of the whole phase are loaded first, under one uniform branch)
#define ZS_LOAD_PHASE(BASE, KA, VA)                                                            \
  do {                                                                                         \
    int jc[NG], srow[NG];                                                                      \
    _Pragma("unroll") for (int i = 0; i < NG; ++i) {                                           \
      jc[i] = max(min((BASE) + i * 8 + grp, p - 1), 0);                                        \
      srow[i] = r;                                                                             \
    }                                                                                          \
    if (kvrow) {                                                                               \
      _Pragma("unroll") for (int i = 0; i < NG; ++i) srow[i] = kvrow[(long)r * Lmax + jc[i]];  \
    }                                                                                          \
    _Pragma("unroll") for (int i = 0; i < NG; ++i) {                                           \
      const long src = ((long)srow[i] * heads + h) * Lmax + jc[i];                             \
      KA[i] = V8::ld(kc + src * HD + sub * EPC);                                               \
      VA[i] = V8::ld(vc + src * HD + sub * EPC);                                               \
    }                                                                                          \
  } while (0)
  if (PF) ZS_LOAD_PHASE(0, kr, vr);
  for (int base = slice * KPP; base <= p; base += KPP * SPLIT) {
    if (PF) {
      if (base + KPP <= p) ZS_LOAD_PHASE(base + KPP, kx, vx);
    } else {
      ZS_LOAD_PHASE(base, kr, vr);
    }
    // the by-value key choice, applied where the phase is consumed (a prefetched phase is not
    // waited for early)
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int j = base + i * 8 + grp;
      const V8 z = V8::zero();
      kr[i] = V8::sel(j < p, kr[i], V8::sel(j == p, knu, z));
      vr[i] = V8::sel(j < p, vr[i], V8::sel(j == p, vnu, z));
    }
    float sc[NG];
    float pm = -INFINITY;
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      float kf[EPC];
      kr[i].unpack(kf);
      float sv = 0.f;
#pragma unroll
      for (int t = 0; t < EPC; ++t) sv += q[t] * kf[t];
      if (DPP) {
        sv = group8_sum_dpp(sv);
      } else {
        sv += __shfl_xor(sv, 1, 64);
        sv += __shfl_xor(sv, 2, 64);
        sv += __shfl_xor(sv, 4, 64);
      }
      sc[i] = (base + i * 8 + grp <= p) ? sv : -INFINITY;
      pm = fmaxf(pm, sc[i]);
    }
    pm = fmaxf(pm, DPP ? dpp_f<0x140>(pm) : __shfl_xor(pm, 8, 64));
    pm = fmaxf(pm, __shfl_xor(pm, 16, 64));
    pm = fmaxf(pm, __shfl_xor(pm, 32, 64));
    const float mn = fmaxf(m, pm);
    const float scale = expf(m - mn);       // 0 on the first phase (m = -inf)
    sum *= scale;
#pragma unroll
    for (int t = 0; t < EPC; ++t) o[t] *= scale;
    m = mn;
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const float e = (base + i * 8 + grp <= p) ? expf(sc[i] - m) : 0.f;
      sum += e;
      float vf[EPC];
      vr[i].unpack(vf);
#pragma unroll
      for (int t = 0; t < EPC; ++t) o[t] += e * vf[t];
    }
    if (PF) {
#pragma unroll
      for (int i = 0; i < NG; ++i) { kr[i] = kx[i]; vr[i] = vx[i]; }
    }
  }
#undef ZS_LOAD_PHASE
#pragma unroll
  for (int d = 8; d < 64; d <<= 1) {
    sum += __shfl_xor(sum, d, 64);
#pragma unroll
    for (int t = 0; t < EPC; ++t) o[t] += __shfl_xor(o[t], d, 64);
  }
  if constexpr (SPLIT > 1) {
    // slices 1.. publish (max, sum, o) of their keys; slice 0 merges them, in slice order, into
    // its own (a slice without keys has max -inf and weight 0)
    if (slice != 0 && grp == 0) {
#pragma unroll
      for (int t = 0; t < EPC; ++t) merge[wid][sub * EPC + t] = o[t];
      if (sub == 0) { merge[wid][64] = m; merge[wid][65] = sum; }
    }
    __syncthreads();
    if (slice != 0) return;
    float mm = m;
#pragma unroll
    for (int u = 1; u < SPLIT; ++u) mm = fmaxf(mm, merge[wid + u][64]);
    const float a0 = expf(m - mm);
    sum *= a0;
#pragma unroll
    for (int t = 0; t < EPC; ++t) o[t] *= a0;
#pragma unroll
    for (int u = 1; u < SPLIT; ++u) {
      const float mu = merge[wid + u][64];
      const float au = mu == -INFINITY ? 0.f : expf(mu - mm);
      sum += merge[wid + u][65] * au;
#pragma unroll
      for (int t = 0; t < EPC; ++t) o[t] += merge[wid + u][sub * EPC + t] * au;
    }
  }
  if (grp == 0) {
    const float inv = 1.0f / sum;
    float of[EPC];
#pragma unroll
    for (int t = 0; t < EPC; ++t) of[t] = o[t] * inv;
    V8::pack(of).st(out + (long)c * D + h * HD + sub * EPC);
    knu.st(kc + (rh + p) * HD + sub * EPC);
    vnu.st(vc + (rh + p) * HD + sub * EPC);
  }
}

template <typename T>
__global__ __launch_bounds__(64) void decode_attn_kernel(const T* __restrict__ qkv, int D,
                                                         int heads, T* __restrict__ kc,
                                                         T* __restrict__ vc, int Lmax,
                                                         const int* __restrict__ pos,
                                                         const int* __restrict__ kvrow,
                                                         T* __restrict__ out) {
  constexpr int HD = 64;
  extern __shared__ float sm[];
  float* qs = sm;            // [64]
  float* kn = sm + 64;       // [64]  new key (also written to the cache)
  float* sc = sm + 128;      // [Lmax] scores
  const int r = blockIdx.x, h = blockIdx.y, d = threadIdx.x;
  const int p = min(pos[r], Lmax - 1);   // defensive: callers keep pos < Lmax
  const T* row = qkv + (long)r * 3 * D + h * HD;
  const float qd = ldf(row + d), kd = ldf(row + D + d);
  const T vd = row[2 * D + d];
  const long slot = (((long)r * heads + h) * Lmax + p) * HD + d;
  kc[slot] = row[D + d];
  vc[slot] = vd;
  qs[d] = qd;
  kn[d] = kd;
  __syncthreads();
  const float scale = 0.125f;  // 1/sqrt(64)
  float mx = -INFINITY;
  for (int j = d; j <= p; j += 64) {
    float s = 0.f;
    if (j == p) {
#pragma unroll 8
      for (int e = 0; e < HD; ++e) s += qs[e] * kn[e];
    } else {
      const int pr = kvrow ? kvrow[(long)r * Lmax + j] : r;
      const T* kr = kc + (((long)pr * heads + h) * Lmax + j) * HD;
#pragma unroll 8
      for (int e = 0; e < HD; ++e) s += qs[e] * ldf(kr + e);
    }
    s *= scale;
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = d; j <= p; j += 64) {
    const float e = expf(sc[j] - mx);
    sc[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  const float inv = 1.0f / sum;
  float o = 0.f;
  for (int j = 0; j <= p; ++j) {
    float vv;
    if (j == p) vv = Cvt<T>::to_f(vd);
    else {
      const int pr = kvrow ? kvrow[(long)r * Lmax + j] : r;
      vv = ldf(vc + (((long)pr * heads + h) * Lmax + j) * HD + d);
    }
    o += sc[j] * inv * vv;
  }
  stf(out + (long)r * D + h * HD + d, o);
}

template <typename T>
__global__ void kv_write_kernel(const T* __restrict__ qkv, int R, int n, int D, int heads,
                                const int* __restrict__ pos0, int row_stride, T* __restrict__ kc,
                                T* __restrict__ vc, int Lmax) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)R * n * D;
  if (e >= total) return;
  const int hd = D / heads;
  const int c = e % D;
  const long t = e / D;
  const int i = t % n, r = t / n;
  const int h = c / hd, d = c % hd;
  const int p = (pos0 ? pos0[r] : 0) + i;
  const long slot = (((long)r * row_stride * heads + h) * Lmax + p) * hd + d;
  kc[slot] = qkv[t * 3 * D + D + c];
  vc[slot] = qkv[t * 3 * D + 2 * D + c];
}

// nn.MultiheadAttention's attention core for a few keys (the sound-effect cross-attention of
// caption_model.py:100-206: one CLAP query against the k chosen label embeddings, 4 heads of 256):
// one wave per (batch row b, query i, head h); lane l holds dims l, l+64, ... of the head;
// scores by wave reductions, softmax over the Lk keys in f32, out = sum_j p_j v_j.
template <typename T>
__global__ __launch_bounds__(64) void cross_attn_kernel(const T* __restrict__ q, int ldq,
                                                        const T* __restrict__ k,
                                                        const T* __restrict__ v, int ldkv, int Lq,
                                                        int Lk, int hd, float scale,
                                                        T* __restrict__ out, int ldo) {
  const int bi = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  const int b = bi / Lq;
  const T* qr = q + (long)bi * ldq + h * hd;
  float qv[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) qv[t] = lane + 64 * t < hd ? ldf(qr + lane + 64 * t) : 0.f;
  float s[64];
  float mx = -INFINITY;
  for (int j = 0; j < Lk; ++j) {
    const T* kr = k + ((long)b * Lk + j) * ldkv + h * hd;
    float a = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) if (lane + 64 * t < hd) a += qv[t] * ldf(kr + lane + 64 * t);
    a = wave_sum(a) * scale;
    s[j < 64 ? j : 63] = a;
    mx = fmaxf(mx, a);
  }
  float den = 0.f;
  for (int j = 0; j < Lk; ++j) { s[j] = expf(s[j] - mx); den += s[j]; }
  const float inv = 1.0f / den;
  float o[4] = {0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < Lk; ++j) {
    const T* vr = v + ((long)b * Lk + j) * ldkv + h * hd;
    const float p = s[j] * inv;
#pragma unroll
    for (int t = 0; t < 4; ++t) if (lane + 64 * t < hd) o[t] += p * ldf(vr + lane + 64 * t);
  }
  T* orow = out + (long)bi * ldo + h * hd;
#pragma unroll
  for (int t = 0; t < 4; ++t) if (lane + 64 * t < hd) stf(orow + lane + 64 * t, o[t]);
}

}  // namespace zs

using namespace zs;

extern "C" int zs_window_attention(const void* qkv, int B, int H, int W, int C, int heads, int ws,
                                   int shift, const float* rel_table, void* out, int dtype,
                                   void* stream) {
  ZS_REQUIRE(ws == 8 && H % ws == 0 && W % ws == 0, "zs_window_attention: ws must be 8 and divide H, W");
  ZS_REQUIRE(heads > 0 && C % heads == 0, "zs_window_attention: C %% heads");
  ZS_REQUIRE(shift >= 0 && shift < ws, "zs_window_attention: shift");
  const int hd = C / heads;
  dim3 grid(B * (H / ws) * (W / ws), heads);
  hipStream_t st = S(stream);
  if (dtype == ZS_BF16 && hd <= 32 && hd % 8 == 0 && g_window_mfma) {
    const int total = B * (H / ws) * (W / ws) * heads;
    hipLaunchKernelGGL(window_attn_mfma_kernel, dim3(cdiv(total, WA_NW)), dim3(64 * WA_NW), 0, st,
                       (const bf16_t*)qkv, H, W, C, heads, hd, shift, rel_table, (bf16_t*)out,
                       total);
    ZS_LAUNCH_CHECK();
    return 0;
  }
#define WA(T, HD_)                                                                             \
  hipLaunchKernelGGL((window_attn_kernel<T, HD_>), grid, dim3(64), 0, st, (const T*)qkv, H, W, C, \
                     heads, shift, rel_table, (T*)out)
  if (hd == 24) {
    if (dtype == ZS_BF16) WA(bf16_t, 24); else WA(float, 24);
  } else if (hd == 32) {
    if (dtype == ZS_BF16) WA(bf16_t, 32); else WA(float, 32);
  } else {
    return fail(ZS_ERR_UNSUPPORTED, "zs_window_attention: head_dim %d unsupported (24, 32)", hd);
  }
#undef WA
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_row_attention_kv(const void* qkv, int B, int L, const int* len, int heads,
                                   float scale, void* out, int ldo, void* kc, void* vc, int Lmax,
                                   int row_stride, void* stream) {
  // causal self-attention over the rows of qkv [B*L][3 * heads * 64] bf16 (q | k | v), and the
  // k / v rows stored into the cache as zs_kv_write(qkv, B, L, ..., pos0 = NULL, row_stride)
  ZS_REQUIRE(B > 0 && L > 0 && L <= 32 && heads > 0 && Lmax >= L && row_stride >= 1,
             "zs_row_attention_kv: 1 <= L <= 32 <= Lmax (B=%d L=%d Lmax=%d)", B, L, Lmax);
  ZS_REQUIRE(qkv && out && kc && vc && ldo % 4 == 0 && ((uintptr_t)qkv & 15) == 0 &&
             ((uintptr_t)kc & 15) == 0 && ((uintptr_t)vc & 15) == 0,
             "zs_row_attention_kv: null or misaligned pointer");
  const int D = heads * 64;
  const bf16_t* q = (const bf16_t*)qkv;
  hipLaunchKernelGGL(row_attn_mfma_kernel, dim3(cdiv((long)B * heads, RA_NW)), dim3(64 * RA_NW), 0,
                     S(stream), q, 3 * D, q + D, q + 2 * D, 3 * D, L, len, 1, scale, (bf16_t*)out,
                     ldo, B, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax, row_stride);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_row_attention(const void* q, int ldq, const void* k, const void* v, int ldkv,
                                int B, int L, const int* len, int heads, int hd, int causal,
                                float scale, void* out, int ldo, int dtype, void* stream) {
  ZS_REQUIRE(B > 0 && L > 0 && L <= 256 && heads > 0, "zs_row_attention: bad shape");
  const size_t smem = (size_t)2 * L * hd * sizeof(float);
  ZS_REQUIRE(smem <= 160 * 1024, "zs_row_attention: L*hd too large for LDS");
  dim3 grid(B, heads, cdiv(L, 64));
  hipStream_t st = S(stream);
  if (g_row_mfma && dtype == ZS_BF16 && hd == 64 && L <= 32 && ldq % 8 == 0 && ldkv % 8 == 0 &&
      ldo % 4 == 0) {
    hipLaunchKernelGGL(row_attn_mfma_kernel, dim3(cdiv((long)B * heads, RA_NW)), dim3(64 * RA_NW), 0,
                       st, (const bf16_t*)q, ldq, (const bf16_t*)k, (const bf16_t*)v, ldkv, L, len,
                       causal, scale, (bf16_t*)out, ldo, B, heads);
    ZS_LAUNCH_CHECK();
    return 0;
  }
#define RA(T, HD_)                                                                              \
  hipLaunchKernelGGL((row_attn_kernel<T, HD_>), grid, dim3(64), smem, st, (const T*)q, ldq,       \
                     (const T*)k, (const T*)v, ldkv, L, len, causal, scale, (T*)out, ldo)
  if (hd == 64) {
    if (dtype == ZS_BF16) RA(bf16_t, 64); else RA(float, 64);
  } else if (hd == 96) {
    if (dtype == ZS_BF16) RA(bf16_t, 96); else RA(float, 96);
  } else {
    return fail(ZS_ERR_UNSUPPORTED, "zs_row_attention: head_dim %d unsupported (64, 96)", hd);
  }
#undef RA
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_decode_attention_map(const void* qkv, int R, const int* rowmap, int nphys,
                                       int D, int heads, void* kc, void* vc, int Lmax,
                                       const int* pos, const int* cpos, void* out, int dtype,
                                       void* stream) {
  ZS_REQUIRE(R > 0 && heads > 0 && D / heads == 64 && D % heads == 0 && rowmap && nphys > 0,
             "zs_decode_attention_map: head_dim must be 64");
  ZS_REQUIRE(dtype == ZS_BF16 && Lmax > 0 && Lmax <= 4096,
             "zs_decode_attention_map: bf16 only, Lmax <= 4096");
  // the same kernel (and phase length) as zs_decode_attention picks for this knob setting, so a
  // compacted decode computes exactly what the uncompacted one does
  if (g_decode_attn5 == 1 && cpos == nullptr && Lmax <= 8 * DA5_MAXI) {
    hipLaunchKernelGGL(decode_attn5_kernel<bf16_t>, dim3(R, cdiv(heads, 4)), dim3(256), 0,
                       S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       pos, (const int*)nullptr, (bf16_t*)out, rowmap, nphys);
  } else if (g_decode_attn5 == 2) {
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 64>), dim3(R, cdiv(heads, 4)), dim3(256), 0,
                       S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       pos, (const int*)nullptr, (bf16_t*)out, rowmap, cpos, nphys, 1);
  } else if (g_decode_attn5 == 4) {
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 16>), dim3(R, cdiv(heads, 4)), dim3(256), 0,
                       S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       pos, (const int*)nullptr, (bf16_t*)out, rowmap, cpos, nphys, 1);
  } else if (g_decode_attn5 == 5) {
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 16, true>), dim3(R, cdiv(heads, 4)), dim3(256),
                       0, S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       pos, (const int*)nullptr, (bf16_t*)out, rowmap, cpos, nphys, 1);
  } else if (g_decode_attn5 == 6) {
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 16, false, true>), dim3(R, cdiv(heads, 4)),
                       dim3(256), 0, S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc,
                       (bf16_t*)vc, Lmax, pos, (const int*)nullptr, (bf16_t*)out, rowmap, cpos,
                       nphys, 1);
  } else {
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 32>), dim3(R, cdiv(heads, 4)), dim3(256), 0,
                       S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       pos, (const int*)nullptr, (bf16_t*)out, rowmap, cpos, nphys, 1);
  }
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_cross_attention(const void* q, int ldq, const void* k, const void* v, int ldkv,
                                  int B, int Lq, int Lk, int heads, int hd, float scale, void* out,
                                  int ldo, int dtype, void* stream) {
  ZS_REQUIRE(B > 0 && Lq > 0 && Lk > 0 && Lk <= 64 && heads > 0 && hd > 0 && hd <= 256,
             "zs_cross_attention: Lk <= 64, hd <= 256");
  const dim3 grid(B * Lq, heads);
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(cross_attn_kernel<bf16_t>, grid, dim3(64), 0, S(stream), (const bf16_t*)q,
                       ldq, (const bf16_t*)k, (const bf16_t*)v, ldkv, Lq, Lk, hd, scale,
                       (bf16_t*)out, ldo);
  else
    hipLaunchKernelGGL(cross_attn_kernel<float>, grid, dim3(64), 0, S(stream), (const float*)q, ldq,
                       (const float*)k, (const float*)v, ldkv, Lq, Lk, hd, scale, (float*)out, ldo);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_decode_attention(const void* qkv, int R, int D, int heads, void* kc, void* vc,
                                   int Lmax, const int* pos, const int* kvrow, void* out,
                                   int dtype, void* stream) {
  ZS_REQUIRE(R > 0 && heads > 0 && D / heads == 64 && D % heads == 0,
             "zs_decode_attention: head_dim must be 64");
  ZS_REQUIRE(Lmax > 0 && Lmax <= 4096, "zs_decode_attention: Lmax");
  dim3 grid(R, heads);
  // beam rows (kvrow != NULL): groups of g_beam_xcd consecutive rows per XCD (decode_attn6_kernel)
  const int rg = (kvrow && g_beam_xcd > 1 && R % (8 * g_beam_xcd) == 0) ? g_beam_xcd : 1;
  if (dtype == ZS_F32 && R <= g_small_rmax && g_small_attn && g_attn_split && heads % 2 == 0) {
    // the f32 parity mode's decode: the bf16 path's two-wave split with 32-key phases
    hipLaunchKernelGGL((decode_attn6_kernel<float, 32, false, true, 2>), dim3(R, heads / 2),
                       dim3(256), 0, S(stream), (const float*)qkv, D, heads, (float*)kc,
                       (float*)vc, Lmax, pos, kvrow, (float*)out, (const int*)nullptr,
                       (const int*)nullptr, R, rg);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == ZS_BF16 && R <= g_small_rmax && g_small_attn && g_attn_split == 4) {
    // each (row, head)'s keys over four waves, 32-key phases (one phase per wave at L <= 128)
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 32, false, true, 4>), dim3(R, heads),
                       dim3(256), 0, S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc,
                       (bf16_t*)vc, Lmax, pos, kvrow, (bf16_t*)out, (const int*)nullptr,
                       (const int*)nullptr, R, rg);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == ZS_BF16 && R <= g_small_rmax && g_small_attn && g_attn_split && heads % 2 == 0) {
    // few waves (R x heads): each (row, head)'s keys over two waves, KPP-key phases (64: all
    // keys of L <= 128 in flight at once, half per wave; 32 (attn_split 3): two phases a wave)
    if (g_attn_split == 3)
      hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 32, false, true, 2>), dim3(R, heads / 2),
                         dim3(256), 0, S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc,
                         (bf16_t*)vc, Lmax, pos, kvrow, (bf16_t*)out, (const int*)nullptr,
                         (const int*)nullptr, R, rg);
    else
      hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 64, false, true, 2>), dim3(R, heads / 2),
                         dim3(256), 0, S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc,
                         (bf16_t*)vc, Lmax, pos, kvrow, (bf16_t*)out, (const int*)nullptr,
                         (const int*)nullptr, R, rg);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == ZS_BF16 && R <= g_small_rmax && g_small_attn) {
    // few waves (R x heads): nothing hides a phase's round trip, so take 128-key phases: every
    // key of a row in flight at once, one HBM round trip at L <= 128
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 128, false, true>), dim3(R, cdiv(heads, 4)),
                       dim3(256), 0, S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc,
                       (bf16_t*)vc, Lmax, pos, kvrow, (bf16_t*)out, (const int*)nullptr,
                       (const int*)nullptr, R, rg);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == ZS_BF16 && g_decode_attn5 == 4) {
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 16>), dim3(R, cdiv(heads, 4)), dim3(256), 0,
                       S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       pos, kvrow, (bf16_t*)out, (const int*)nullptr, (const int*)nullptr, R, rg);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == ZS_BF16 && g_decode_attn5 == 6) {
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 16, false, true>), dim3(R, cdiv(heads, 4)),
                       dim3(256), 0, S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc,
                       (bf16_t*)vc, Lmax, pos, kvrow, (bf16_t*)out, (const int*)nullptr,
                       (const int*)nullptr, R, rg);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == ZS_BF16 && g_decode_attn5 == 5) {
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 16, true>), dim3(R, cdiv(heads, 4)), dim3(256),
                       0, S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       pos, kvrow, (bf16_t*)out, (const int*)nullptr, (const int*)nullptr, R, rg);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == ZS_BF16 && g_decode_attn5 == 3) {
    hipLaunchKernelGGL((decode_attn6_kernel<bf16_t, 32>), dim3(R, cdiv(heads, 4)), dim3(256), 0,
                       S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       pos, kvrow, (bf16_t*)out, (const int*)nullptr, (const int*)nullptr, R, rg);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == ZS_BF16 && g_decode_attn5 == 2) {
    hipLaunchKernelGGL(decode_attn6_kernel<bf16_t>, dim3(R, cdiv(heads, 4)), dim3(256), 0,
                       S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       pos, kvrow, (bf16_t*)out, (const int*)nullptr, (const int*)nullptr, R, rg);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == ZS_BF16 && Lmax <= 8 * DA5_MAXI && g_decode_attn5) {
    hipLaunchKernelGGL(decode_attn5_kernel<bf16_t>, dim3(R, cdiv(heads, 4)), dim3(256), 0,
                       S(stream), (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax,
                       pos, kvrow, (bf16_t*)out, (const int*)nullptr, R);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  if (Lmax <= 512) {
    const size_t smem = (400 + 66 * (size_t)Lmax) * sizeof(float);
    if (dtype == ZS_BF16)
      hipLaunchKernelGGL(decode_attn4_kernel<bf16_t>, grid, dim3(256), smem, S(stream),
                         (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax, pos, kvrow,
                         (bf16_t*)out);
    else
      hipLaunchKernelGGL(decode_attn4_kernel<float>, grid, dim3(256), smem, S(stream),
                         (const float*)qkv, D, heads, (float*)kc, (float*)vc, Lmax, pos, kvrow,
                         (float*)out);
    ZS_LAUNCH_CHECK();
    return 0;
  }
  const size_t smem = (128 + (size_t)Lmax) * sizeof(float);
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(decode_attn_kernel<bf16_t>, grid, dim3(64), smem, S(stream),
                       (const bf16_t*)qkv, D, heads, (bf16_t*)kc, (bf16_t*)vc, Lmax, pos, kvrow,
                       (bf16_t*)out);
  else
    hipLaunchKernelGGL(decode_attn_kernel<float>, grid, dim3(64), smem, S(stream),
                       (const float*)qkv, D, heads, (float*)kc, (float*)vc, Lmax, pos, kvrow,
                       (float*)out);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_kv_write(const void* qkv, int R, int n, int D, int heads, const int* pos0,
                           int row_stride, void* kc, void* vc, int Lmax, int dtype,
                           void* stream) {
  ZS_REQUIRE(R > 0 && n > 0 && heads > 0 && D % heads == 0 && n <= Lmax, "zs_kv_write: bad shape");
  const long total = (long)R * n * D;
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(kv_write_kernel<bf16_t>, dim3(cdiv(total, 256)), dim3(256), 0, S(stream),
                       (const bf16_t*)qkv, R, n, D, heads, pos0, row_stride, (bf16_t*)kc, (bf16_t*)vc, Lmax);
  else
    hipLaunchKernelGGL(kv_write_kernel<float>, dim3(cdiv(total, 256)), dim3(256), 0, S(stream),
                       (const float*)qkv, R, n, D, heads, pos0, row_stride, (float*)kc, (float*)vc, Lmax);
  ZS_LAUNCH_CHECK();
  return 0;
}

// GPT-2 decode glue + prompt assembly:
//  * prompt_assemble  — sound_effect_choice + compose_discrete_prompts + padding_captions on
//                       device (utils.py:131-208, dataset/dataset.py:441-453);
//  * prefill_embed    — clap_to_gpt concat (caption_model.py:315-329) + wte/wpe lookup;
//  * embed_tokens     — decode-step input embedding;
//  * argmax_finalize / greedy_step / beam_step — generate2 / generate_beam bookkeeping on device
//    (gpt2_prefix_eval.py:99-158, 161-222) so a captured decode step needs no host round trip.
#include "common.h"

namespace zs {

// ------------------------------------------------------------------ prompt
// sound_effect_choice (utils.py:131-137 / caption_model.py:15-20): the k labels of highest
// similarity emb . label (softmax is monotone, so top-k of the raw similarities), best first,
// ties to the lower label index.
//
// ONE wave per clip, everything in registers: lane l holds e[4 l + 256 u .. + 4), u < 4 (D = 1024;
// other D in 16-byte chunks c = lane + 64 u), each label row is read in the same chunks (four
// rows in flight), the lane partials summed over the wave by DPP row ops and permlane swaps (no
// LDS, no ds_bpermute, no workgroup barrier), and the running top-k kept in uniform registers,
// labels visited in increasing index so a tie keeps the lower one.  (Round 5's 512-thread block
// version -- the embedding staged in LDS, ds_bpermute reductions, a block-wide top-k through LDS
// -- chose different labels now and then while decode grids ran on other streams: 144 of 418k
// clips over 40 rounds, tools/prompt_stress.py grid mode; none alone or beside GEMMs; the cause
// in that kernel was not isolated, this one shares nothing with it.)
constexpr int PK_MAX = 16;          // k <= 16
template <int CTRL>
__device__ __forceinline__ float pdpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
// the sum of v over the 64 lanes, on every lane, in one fixed order
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += pdpp<0xB1>(v);                              // quad_perm [1,0,3,2]
  v += pdpp<0x4E>(v);                              // quad_perm [2,3,0,1]
  v += pdpp<0x141>(v);                             // row_half_mirror: 8-lane sums
  v += pdpp<0x128>(v);                             // row_ror:8: 16-lane sums
  {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// top-k labels of clip blockIdx.x into sel[0..k) (uniform across the wave); K = k (3, the
// reference's sound_effect_num) or PK_MAX (any k <= 16)
template <int K>
__device__ __forceinline__ void label_select_k(const float* __restrict__ emb, int D,
                                               const float* __restrict__ labels, int L, int k,
                                               int (&sel)[PK_MAX]) {
  const int b = blockIdx.x, lane = threadIdx.x & 63;
  float tv[K];
#pragma unroll
  for (int i = 0; i < K; ++i) tv[i] = -INFINITY;
#pragma unroll
  for (int i = 0; i < PK_MAX; ++i) sel[i] = 0x7fffffff;
  auto insert = [&](float sv, int l) {          // strictly better only: ties keep the earlier
    if (K != PK_MAX && !(sv > tv[K - 1])) return;   // (K == k: below the k-th best)
#pragma unroll
    for (int i = 0; i < K; ++i) {
      if (i < k && sv > tv[i]) {
        const float t = tv[i]; const int ti = sel[i];
        tv[i] = sv; sel[i] = l; sv = t; l = ti;
      }
    }
  };
  const float* er = emb + (long)b * D;
  if (D == 1024 && ((uintptr_t)labels & 15) == 0 && ((uintptr_t)er & 15) == 0) {
    float4 e[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) e[u] = reinterpret_cast<const float4*>(er)[lane + 64 * u];
    // four label rows per group, the next group's loads issued before this group's sums
    constexpr int NR = 4;
    auto load = [&](int l0, float4 (&a)[NR][4]) {
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          a[j][u] = reinterpret_cast<const float4*>(labels + (long)min(l0 + j, L - 1) * D)[lane + 64 * u];
    };
    auto consume = [&](int l0, const float4 (&a)[NR][4]) {
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        float sj = 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          sj += (a[j][u].x * e[u].x + a[j][u].y * e[u].y) + (a[j][u].z * e[u].z + a[j][u].w * e[u].w);
        sj = wave_sum_dpp(sj);
        if (l0 + j < L) insert(__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sj))), l0 + j);
      }
    };
    float4 a0[NR][4], a1[NR][4];
    load(0, a0);
    for (int l0 = 0; l0 < L; l0 += 2 * NR) {
      load(l0 + NR, a1);
      consume(l0, a0);
      load(l0 + 2 * NR, a0);
      if (l0 + NR < L) consume(l0 + NR, a1);
    }
  } else {                                         // any D: lane-strided scalar dot products
    for (int l = 0; l < L; ++l) {
      const float* lr = labels + (long)l * D;
      float sj = 0.f;
      for (int d = lane; d < D; d += 64) sj += er[d] * lr[d];
      insert(__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wave_sum_dpp(sj)))), l);
    }
  }
}
__device__ __forceinline__ void label_select_wave(const float* __restrict__ emb, int D,
                                                  const float* __restrict__ labels, int L, int k,
                                                  int (&sel)[PK_MAX]) {
  if (k == 3) label_select_k<3>(emb, D, labels, L, k, sel);
  else label_select_k<PK_MAX>(emb, D, labels, L, k, sel);
}

__global__ __launch_bounds__(64) void prompt_kernel(const float* __restrict__ emb, int D,
                                                     const float* __restrict__ labels, int L,
                                                     int k, const int* __restrict__ ltok,
                                                     const int* __restrict__ llen, int max_tok,
                                                     int* __restrict__ hard_ids, int h_cap,
                                                     int* __restrict__ hard_len,
                                                     int* __restrict__ chosen) {
  int sel[PK_MAX];
  label_select_wave(emb, D, labels, L, k, sel);
  const int b = blockIdx.x, lane = threadIdx.x & 63;
  if (lane == 0) {
    int* out = hard_ids + (long)b * h_cap;
    int n = 0;
    auto put = [&](int id) { if (n < h_cap) out[n] = id; ++n; };
    put(1858); put(389);                    // "There", " are"
    if (k == 0) {
      put(1223);                            // " something"
    } else {
      for (int q = 0; q < k; ++q) {
        const int l = sel[q];
        const int nt = min(llen[l], min(max_tok, 32));
        for (int t = 0; t < nt; ++t) put(ltok[(long)l * max_tok + t]);
        if (q + 1 < k) put(11);             // ","
        if (chosen) chosen[(long)b * k + q] = l;
      }
    }
    put(287); put(428); put(6597); put(13); // " in", " this", " audio", "."
    hard_len[b] = n < h_cap ? n : h_cap;
    for (int t = n; t < h_cap; ++t) out[t] = 0;
  }
}

// the chosen labels' rows gathered: rows[b][q][:] = labels[sel[q]][:] (caption_model.py:15-20,
// sound_effect_embeddings[index].squeeze(1)), and their indices
__global__ __launch_bounds__(64) void label_topk_kernel(const float* __restrict__ emb, int D,
                                                         const float* __restrict__ labels, int L,
                                                         int k, int* __restrict__ idx,
                                                         float* __restrict__ rows) {
  int sel[PK_MAX];
  label_select_wave(emb, D, labels, L, k, sel);
  const int b = blockIdx.x, lane = threadIdx.x & 63;
  for (int q = 0; q < k; ++q) {
    if (idx && lane == 0) idx[(long)b * k + q] = sel[q];
    for (int d = lane; d < D; d += 64) rows[((long)b * k + q) * D + d] = labels[(long)sel[q] * D + d];
  }
}

// ------------------------------------------------------------------ embeddings
template <typename T>
__global__ void prefill_embed_kernel(const int* __restrict__ hard_ids,
                                     const int* __restrict__ hard_len, int h_cap,
                                     const float* __restrict__ soft, int soft_ld, int n_soft,
                                     const T* __restrict__ wte, const T* __restrict__ wpe, int Pmax,
                                     int D, float* __restrict__ embed, float* __restrict__ x,
                                     int* __restrict__ plen, int* __restrict__ last_row) {
  const int b = blockIdx.y, p = blockIdx.x;
  const int H = hard_len[b], P = H + n_soft;
  if (p == 0 && threadIdx.x == 0) {
    plen[b] = P;
    if (last_row) last_row[b] = b * Pmax + P - 1;
  }
  const long o = ((long)b * Pmax + p) * D;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float e = 0.f, xv = 0.f;
    if (p < H) e = ldf(wte + (long)hard_ids[(long)b * h_cap + p] * D + d);
    else if (p < P) e = soft[(long)b * soft_ld + (long)(p - H) * D + d];
    if (p < P) xv = e + ldf(wpe + (long)p * D + d);
    if (embed) embed[o + d] = e;
    x[o + d] = xv;
  }
}

template <typename T>
__global__ void embed_tokens_kernel(const int* __restrict__ tok, const int* __restrict__ pos,
                                    const T* __restrict__ wte, const T* __restrict__ wpe, int D,
                                    float* __restrict__ x, const int* __restrict__ rowmap,
                                    int nphys, int* __restrict__ cpos) {
  const int r = blockIdx.x;                       // compact row (x is compact)
  const int ph = rowmap ? rowmap[r] : r;           // physical decode row (tok/pos are physical)
  if (ph >= nphys) {                               // padding slot of a compacted step
    for (int d = threadIdx.x; d < D; d += blockDim.x) x[(long)r * D + d] = 0.f;
    if (cpos && threadIdx.x == 0) cpos[r] = 0;
    return;
  }
  const int t = tok[ph], p = pos[ph];
  if (cpos && threadIdx.x == 0) cpos[r] = p;     // this step's position, in compact order
  for (int d = threadIdx.x; d < D; d += blockDim.x)
    x[(long)r * D + d] = ldf(wte + (long)t * D + d) + ldf(wpe + (long)p * D + d);
}

// active-row compaction (one 1024-thread block): rowmap[0..n) = the rows with done == 0 in
// increasing order, rowmap[n..nrows) = nrows (padding), *n_active = n.  Deterministic.
__global__ __launch_bounds__(1024) void compact_rows_kernel(const int* __restrict__ done, int nrows,
                                                             int* __restrict__ rowmap,
                                                             int* __restrict__ n_active) {
  __shared__ int wsum[16];
  __shared__ int base;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (int c0 = 0; c0 < nrows; c0 += 1024) {
    const int r = c0 + threadIdx.x;
    const int a = (r < nrows && !done[r]) ? 1 : 0;
    // inclusive scan within the wave
    int inc = a;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int o = __shfl_up(inc, d, 64);
      if (lane >= d) inc += o;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    int off = base;
    for (int w = 0; w < wid; ++w) off += wsum[w];
    if (a) rowmap[off + inc - 1] = r;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int w = 0; w < 16; ++w) t += wsum[w];
      base += t;
    }
    __syncthreads();
  }
  const int n = base;
  for (int r = n + threadIdx.x; r < nrows; r += 1024) rowmap[r] = nrows;
  if (threadIdx.x == 0) *n_active = n;
}

// ------------------------------------------------------------------ argmax over LM-head partials
__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}

__device__ __forceinline__ int row_argmax(const float* pv, const int* pi, int r, int nblk,
                                          int lane) {
  float v = -INFINITY;
  int i = 0x7fffffff;
  for (int k = lane; k < nblk; k += 64) {
    const float cv = pv[(long)r * nblk + k];
    const int ci = pi[(long)r * nblk + k];
    if (cv > v || (cv == v && ci < i)) { v = cv; i = ci; }
  }
  wave_argmax(v, i);
  return i;
}

__global__ void argmax_finalize_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                       int M, int nblk, int* __restrict__ idx) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= M) return;
  const int t = row_argmax(pv, pi, r, nblk, lane);
  if (lane == 0) idx[r] = t;
}

// one wave per row, 4 rows per block.  The blocks combine "rows still alive" and their arrival
// in ONE relaxed agent-scope atomic on all_done[1] (arrivals in the low 16 bits, alive rows in
// the high 16): the block that draws the last ticket knows every block has read *step_ctr and
// added its alive count, so it alone writes all_done[0], advances *step_ctr and re-arms the
// counter (no data hand-off between blocks, so no release/acquire is needed).
__global__ __launch_bounds__(256) void greedy_step_kernel(
    const float* __restrict__ pv, const int* __restrict__ pi, int R, int nblk, int* step_ctr,
    int max_steps, int stop0, int stop1, int* __restrict__ out_ids, int* __restrict__ out_len,
    int* __restrict__ done, int* __restrict__ pos, int* __restrict__ next_tok,
    int* __restrict__ all_done, const int* __restrict__ rowmap, int nphys) {
  __shared__ int s_alive[5];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int step = __hip_atomic_load(step_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int c = blockIdx.x * 4 + wid;             // compact row (partials are compact)
  const int r = c < R ? (rowmap ? rowmap[c] : c) : nphys;   // physical row
  int alive = 0;
  if (c < R && r < nphys) {
    const int t = row_argmax(pv, pi, c, nblk, lane);
    if (lane == 0) {
      int d = done[r];
      if (!d && step < max_steps) {
        out_ids[(long)r * max_steps + step] = t;
        out_len[r] = step + 1;
        if (t == stop0 || t == stop1) d = 1;
        done[r] = d;
      }
      alive = !d;
      next_tok[r] = t;
      if (step < max_steps) pos[r] += 1;   // past entry_length the graph tail re-runs in place
    }
  }
  if (lane == 0) s_alive[wid] = alive;
  __syncthreads();
  if (threadIdx.x == 0) {
    // unsigned: the alive field (bits 16-31) holds up to 65535 rows (R < 65536 at the ABI)
    const unsigned a = s_alive[0] + s_alive[1] + s_alive[2] + s_alive[3];
    const unsigned old = __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(&all_done[1]),
                                                1u + (a << 16), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if ((old & 0xffffu) == gridDim.x - 1) {
      const int total = (int)((old >> 16) + a);
      all_done[0] = (total == 0 || step + 1 >= max_steps) ? 1 : 0;
      all_done[2] = total;             // rows still decoding (sizes the next compacted chunk)
      __hip_atomic_store(step_ctr, step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&all_done[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------ beam search step
// one block per clip, one wave per source row (64 beam threads); beam <= LMB <= 8, topk
// (partials per block) >= beam; LMB = the lane candidate list length
template <int LMB>
__global__ __launch_bounds__(512) void beam_step_kernel(
    const float* __restrict__ pstat, const float* __restrict__ pv, const int* __restrict__ pi,
    int beam, int nblk, int topk, int first, int stop, const int* __restrict__ step_ctr,
    int max_steps, float* __restrict__ scores, float* __restrict__ seq_len,
    int* __restrict__ stopped, int* __restrict__ tokens, int* __restrict__ tokens_tmp,
    int* __restrict__ kvrow, int* __restrict__ kvrow_tmp, int Lmax, int* __restrict__ pos,
    int* __restrict__ next_tok) {
  constexpr int MB = 8;
  __shared__ float c_val[MB * MB];      // candidate values per (source row, rank)
  __shared__ int c_tok[MB * MB];
  __shared__ float c_logp[MB * MB];
  __shared__ int sel_src[MB], sel_tok[MB];
  __shared__ float sel_avg[MB];
  __shared__ int s_skip;
  const int c = blockIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nwv = blockDim.x >> 6, nthr = blockDim.x;
  const int step = *step_ctr;
  const int r0 = c * beam;
  if (threadIdx.x == 0) {
    int all = 1;
    for (int i = 0; i < beam; ++i) all &= stopped[r0 + i];
    s_skip = (!first && all) || step >= max_steps;
  }
  __syncthreads();
  if (s_skip) return;   // finished clip: the reference has left its loop; state is frozen
  const int nsrc = first ? 1 : beam;
  // per source row: lse pieces and its top-`beam` logits (merging the per-block sorted lists)
  for (int i = wid; i < nsrc; i += nwv) {
    const int prow = first ? c : r0 + i;   // partial row (prefill rows are per clip)
    float M = -INFINITY;
    for (int k = lane; k < nblk; k += 64) M = fmaxf(M, pstat[((long)prow * nblk + k) * 2]);
    M = wave_max(M);
    float Ssum = 0.f;
    for (int k = lane; k < nblk; k += 64) {
      const float bm = pstat[((long)prow * nblk + k) * 2];
      Ssum += pstat[((long)prow * nblk + k) * 2 + 1] * expf(bm - M);
    }
    Ssum = wave_sum(Ssum);
    // top-beam over all blocks' lists: each lane first keeps the best MB of its own blocks'
    // candidates in registers (one pass of independent loads, insertion in (value desc, index
    // asc) order), then `beam` rounds of wave argmax over those lane lists (the rounds no longer
    // re-read the candidates from memory)
    float lv[LMB];
    int li[LMB];
#pragma unroll
    for (int t = 0; t < LMB; ++t) { lv[t] = -INFINITY; li[t] = 0x7fffffff; }
    for (int k = lane; k < nblk; k += 64) {
      const long base = ((long)prow * nblk + k) * topk;
      for (int t = 0; t < beam; ++t) {   // only a block's first `beam` can reach the top-beam
        float v = pv[base + t];
        int ix = pi[base + t];
#pragma unroll
        for (int u = 0; u < LMB; ++u) {     // bubble (v, ix) into the sorted lane list
          const bool better = v > lv[u] || (v == lv[u] && ix < li[u]);
          const float tv = better ? lv[u] : v;
          const int ti = better ? li[u] : ix;
          lv[u] = better ? v : lv[u];
          li[u] = better ? ix : li[u];
          v = tv;
          ix = ti;
        }
      }
    }
    float lastv = INFINITY;
    int lasti = -1;
    for (int q = 0; q < beam; ++q) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int t = 0; t < LMB; ++t) {
        const float v = lv[t];
        const int ix = li[t];
        // strictly after the previous pick in (value desc, index asc) order
        const bool after = v < lastv || (v == lastv && ix > lasti);
        if (after && (v > bv || (v == bv && ix < bi))) { bv = v; bi = ix; }
      }
      wave_argmax(bv, bi);
      lastv = bv;
      lasti = bi;
      if (lane == 0) {
        // generate_beam: logits.softmax(-1).log() (gpt2_prefix_eval.py:122)
        const float lp = logf(expf(bv - M) / Ssum);
        c_tok[i * MB + q] = bi;
        c_logp[i * MB + q] = lp;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float newlen[MB];
    if (first) {
      for (int q = 0; q < beam; ++q) {
        sel_src[q] = 0; sel_tok[q] = c_tok[q]; sel_avg[q] = c_logp[q];
      }
    } else {
      // candidates: non-stopped rows -> (score + logp) / (len + 1); stopped rows -> token 0
      // with logp 0 at their unchanged length (gpt2_prefix_eval.py:132-137)
      for (int i = 0; i < beam; ++i) {
        const int r = r0 + i;
        const bool st = stopped[r];
        newlen[i] = st ? seq_len[r] : seq_len[r] + 1.0f;
        if (st) {
          c_val[i * MB] = (scores[r] + 0.0f) / newlen[i];
          c_tok[i * MB] = 0;
          for (int q = 1; q < beam; ++q) c_val[i * MB + q] = -INFINITY;
        } else {
          for (int q = 0; q < beam; ++q) c_val[i * MB + q] = (scores[r] + c_logp[i * MB + q]) / newlen[i];
        }
      }
      // top-beam over beam x beam candidates; ties -> lower flattened index src*V + tok
      unsigned used[MB] = {0};
      for (int q = 0; q < beam; ++q) {
        int bs = -1, bq = -1;
        float bv = -INFINITY;
        long bflat = 0x7fffffffffffffffL;
        for (int i = 0; i < beam; ++i)
          for (int t = 0; t < beam; ++t) {
            if (used[i] & (1u << t)) continue;
            const float v = c_val[i * MB + t];
            const long flat = (long)i * 50257 + c_tok[i * MB + t];
            if (bs < 0 || v > bv || (v == bv && flat < bflat)) { bs = i; bq = t; bv = v; bflat = flat; }
          }
        used[bs] |= 1u << bq;
        sel_src[q] = bs; sel_tok[q] = c_tok[bs * MB + bq]; sel_avg[q] = bv;
      }
      for (int q = 0; q < beam; ++q) c_val[q] = newlen[sel_src[q]];   // reuse: chosen lengths
    }
  }
  __syncthreads();
  // gather histories of the chosen sources into tmp, then write back
  const int P = pos[r0];   // all rows of a clip share the position of this step's token
  for (int q = 0; q < beam; ++q) {
    const int src = first ? r0 : r0 + sel_src[q];
    const int dst = r0 + q;
    for (int s = threadIdx.x; s < step; s += nthr)
      tokens_tmp[(long)dst * max_steps + s] = tokens[(long)src * max_steps + s];
    for (int s = threadIdx.x; s < Lmax; s += nthr) {
      int v;
      if (first) v = s < P ? r0 : -1;                       // prompt lives in clip row r0
      else v = s < P ? kvrow[(long)src * Lmax + s] : (s == P ? src : -1);
      kvrow_tmp[(long)dst * Lmax + s] = v;
    }
  }
  __syncthreads();
  for (int q = 0; q < beam; ++q) {
    const int dst = r0 + q;
    for (int s = threadIdx.x; s < step; s += nthr)
      tokens[(long)dst * max_steps + s] = tokens_tmp[(long)dst * max_steps + s];
    for (int s = threadIdx.x; s < Lmax; s += nthr)
      kvrow[(long)dst * Lmax + s] = kvrow_tmp[(long)dst * Lmax + s];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int st_new[MB];
    float len_new[MB], sc_new[MB];
    for (int q = 0; q < beam; ++q) {
      const int src = r0 + sel_src[q];
      if (first) {
        len_new[q] = 1.0f;
        sc_new[q] = sel_avg[q];
        st_new[q] = 0;
      } else {
        len_new[q] = c_val[q];
        sc_new[q] = sel_avg[q] * len_new[q];   // scores = scores_sum_average * seq_lengths
        st_new[q] = stopped[src];
      }
    }
    for (int q = 0; q < beam; ++q) {
      const int dst = r0 + q;
      const int tok = sel_tok[q];
      tokens[(long)dst * max_steps + step] = tok;
      seq_len[dst] = len_new[q];
      scores[dst] = sc_new[q];
      stopped[dst] = st_new[q] | (tok == stop);
      next_tok[dst] = tok;
      pos[dst] = (first ? P : P + 1);
    }
  }
}

__global__ void beam_advance_kernel(const int* __restrict__ stopped, int R, int* step_ctr,
                                    int max_steps, int* all_done) {
  __shared__ int alive;
  if (threadIdx.x == 0) alive = 0;
  __syncthreads();
  int a = 0;
  for (int r = threadIdx.x; r < R; r += blockDim.x) a |= !stopped[r];
  if (a) atomicOr(&alive, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int s = *step_ctr + 1;
    *step_ctr = s;
    all_done[0] = (!alive || s >= max_steps) ? 1 : 0;
  }
}

}  // namespace zs

using namespace zs;

extern "C" int zs_prompt_assemble(const float* emb, int B, int D, const float* labels, int L,
                                  int k, const int* label_tok, const int* label_len, int max_tok,
                                  int* hard_ids, int h_cap, int* hard_len, int* chosen,
                                  void* stream) {
  ZS_REQUIRE(B > 0 && D > 0 && L > 0 && k >= 0 && k <= 16 && k <= L && max_tok <= 32, "zs_prompt_assemble: bad shape");
  hipLaunchKernelGGL(prompt_kernel, dim3(B), dim3(64), 0, S(stream), emb, D, labels, L, k,
                     label_tok, label_len, max_tok, hard_ids, h_cap, hard_len, chosen);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_label_topk(const float* emb, int B, int D, const float* labels, int L, int k,
                             int* idx, float* rows, void* stream) {
  ZS_REQUIRE(B > 0 && D > 0 && L > 0 && k >= 1 && k <= 16 && k <= L, "zs_label_topk: bad shape");
  ZS_REQUIRE(emb && labels && rows, "zs_label_topk: null pointer");
  hipLaunchKernelGGL(label_topk_kernel, dim3(B), dim3(64), 0, S(stream), emb, D, labels, L, k,
                     idx, rows);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_gpt2_prefill_embed(const int* hard_ids, const int* hard_len, int h_cap,
                                     const float* soft, int soft_ld, int n_soft, const void* wte,
                                     const void* wpe, int B, int Pmax, int D, float* embed,
                                     float* x, int* plen, int* last_row, int dtype, void* stream) {
  ZS_REQUIRE(B > 0 && Pmax > 0 && D > 0, "zs_gpt2_prefill_embed: bad shape");
  dim3 grid(Pmax, B);
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(prefill_embed_kernel<bf16_t>, grid, dim3(256), 0, S(stream), hard_ids,
                       hard_len, h_cap, soft, soft_ld, n_soft, (const bf16_t*)wte, (const bf16_t*)wpe,
                       Pmax, D, embed, x, plen, last_row);
  else
    hipLaunchKernelGGL(prefill_embed_kernel<float>, grid, dim3(256), 0, S(stream), hard_ids,
                       hard_len, h_cap, soft, soft_ld, n_soft, (const float*)wte, (const float*)wpe,
                       Pmax, D, embed, x, plen, last_row);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_embed_tokens(const int* tok, const int* pos, const void* wte, const void* wpe,
                               int R, int D, float* x, int dtype, void* stream) {
  ZS_REQUIRE(R > 0 && D > 0, "zs_embed_tokens: bad shape");
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(embed_tokens_kernel<bf16_t>, dim3(R), dim3(256), 0, S(stream), tok, pos,
                       (const bf16_t*)wte, (const bf16_t*)wpe, D, x, (const int*)nullptr, R, (int*)nullptr);
  else
    hipLaunchKernelGGL(embed_tokens_kernel<float>, dim3(R), dim3(256), 0, S(stream), tok, pos,
                       (const float*)wte, (const float*)wpe, D, x, (const int*)nullptr, R, (int*)nullptr);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_embed_tokens_map(const int* tok, const int* pos, const int* rowmap, int nphys,
                                   const void* wte, const void* wpe, int R, int D, float* x,
                                   int* cpos, int dtype, void* stream) {
  ZS_REQUIRE(R > 0 && D > 0 && rowmap != nullptr && nphys > 0, "zs_embed_tokens_map: bad shape");
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(embed_tokens_kernel<bf16_t>, dim3(R), dim3(256), 0, S(stream), tok, pos,
                       (const bf16_t*)wte, (const bf16_t*)wpe, D, x, rowmap, nphys, cpos);
  else
    hipLaunchKernelGGL(embed_tokens_kernel<float>, dim3(R), dim3(256), 0, S(stream), tok, pos,
                       (const float*)wte, (const float*)wpe, D, x, rowmap, nphys, cpos);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_compact_rows(const int* done, int nrows, int* rowmap, int* n_active,
                               void* stream) {
  ZS_REQUIRE(nrows > 0, "zs_compact_rows: nrows");
  hipLaunchKernelGGL(compact_rows_kernel, dim3(1), dim3(1024), 0, S(stream), done, nrows, rowmap,
                     n_active);
  ZS_LAUNCH_CHECK();
  return 0;
}

// get_prefix_tokens over the soft rows only (see zs_prefix_ids_assemble): row b, position p of
// the [B][Pmax] result = the hard id (p < H_b), the soft-row argmax (H_b <= p < H_b + n_soft) or
// 0 (padding: a zero embedding row's cosines are all 0, argmax = index 0)
__global__ void prefix_ids_kernel(const int* __restrict__ hard_ids, int h_cap,
                                  const int* __restrict__ hard_len, const int* __restrict__ soft_idx,
                                  int n_soft, int B, int Pmax, int* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * Pmax) return;
  const int b = i / Pmax, p = i % Pmax, H = hard_len[b];
  out[i] = p < H ? hard_ids[(long)b * h_cap + p]
                 : (p < H + n_soft ? soft_idx[(long)b * n_soft + p - H] : 0);
}

extern "C" int zs_prefix_ids_assemble(const int* hard_ids, int h_cap, const int* hard_len,
                                      const int* soft_idx, int n_soft, int B, int Pmax, int* out,
                                      void* stream) {
  ZS_REQUIRE(B > 0 && Pmax > 0 && h_cap >= 0 && n_soft >= 0 && h_cap + n_soft <= Pmax,
             "zs_prefix_ids_assemble: bad shape");
  hipLaunchKernelGGL(prefix_ids_kernel, dim3(cdiv((long)B * Pmax, 256)), dim3(256), 0, S(stream),
                     hard_ids, h_cap, hard_len, soft_idx, n_soft, B, Pmax, out);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_argmax_finalize(const float* part_val, const int* part_idx, int M, int nblk,
                                  int* idx, void* stream) {
  ZS_REQUIRE(M > 0 && nblk > 0, "zs_argmax_finalize: bad shape");
  hipLaunchKernelGGL(argmax_finalize_kernel, dim3(cdiv(M, 4)), dim3(256), 0, S(stream), part_val,
                     part_idx, M, nblk, idx);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_greedy_step_map(const float* part_val, const int* part_idx, int R,
                                  const int* rowmap, int nphys, int nblk, int* step_ctr,
                                  int max_steps, int stop0, int stop1, int* out_ids, int* out_len,
                                  int* done, int* pos, int* next_tok, int* all_done,
                                  void* stream) {
  ZS_REQUIRE(R > 0 && R < 65536 && nblk > 0 && max_steps > 0 && rowmap != nullptr && nphys > 0,
             "zs_greedy_step_map: bad shape");
  hipLaunchKernelGGL(greedy_step_kernel, dim3(cdiv(R, 4)), dim3(256), 0, S(stream), part_val,
                     part_idx, R, nblk, step_ctr, max_steps, stop0, stop1, out_ids, out_len, done,
                     pos, next_tok, all_done, rowmap, nphys);
  ZS_LAUNCH_CHECK();
  return 0;
}

// generate2's state before step 0 for R rows: pos = plen - 1, done = out_len = 0, out_ids rows
// zeroed, *step_ctr = 0, all_done = {0, 0, 0} -- one launch instead of six fills and copies
__global__ __launch_bounds__(256) void greedy_init_kernel(int R, const int* __restrict__ plen,
                                                          int* __restrict__ pos,
                                                          int* __restrict__ done,
                                                          int* __restrict__ out_len,
                                                          int* __restrict__ out_ids, int max_steps,
                                                          int* __restrict__ step_ctr,
                                                          int* __restrict__ all_done) {
  const int r = blockIdx.x;
  if (threadIdx.x == 0) {
    pos[r] = plen[r] - 1;
    done[r] = 0;
    out_len[r] = 0;
    if (r == 0) {
      *step_ctr = 0;
      all_done[0] = all_done[1] = all_done[2] = 0;
    }
  }
  for (int t = threadIdx.x; t < max_steps; t += 256) out_ids[(long)r * max_steps + t] = 0;
}

extern "C" int zs_greedy_init(int R, const int* plen, int* pos, int* done, int* out_len,
                              int* out_ids, int max_steps, int* step_ctr, int* all_done,
                              void* stream) {
  ZS_REQUIRE(R > 0 && max_steps > 0 && plen && pos && done && out_len && out_ids && step_ctr &&
             all_done, "zs_greedy_init: bad arguments");
  hipLaunchKernelGGL(greedy_init_kernel, dim3(R), dim3(256), 0, S(stream), R, plen, pos, done,
                     out_len, out_ids, max_steps, step_ctr, all_done);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_greedy_step(const float* part_val, const int* part_idx, int R, int nblk,
                              int* step_ctr, int max_steps, int stop0, int stop1, int* out_ids,
                              int* out_len, int* done, int* pos, int* next_tok, int* all_done,
                              void* stream) {
  ZS_REQUIRE(R > 0 && R < 65536 && nblk > 0 && max_steps > 0, "zs_greedy_step: bad shape");
  hipLaunchKernelGGL(greedy_step_kernel, dim3(cdiv(R, 4)), dim3(256), 0, S(stream), part_val, part_idx, R,
                     nblk, step_ctr, max_steps, stop0, stop1, out_ids, out_len, done, pos,
                     next_tok, all_done, (const int*)nullptr, R);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_beam_step(const float* part_stat, const float* part_val, const int* part_idx,
                            int C, int beam, int nblk, int topk, int first, int stop,
                            int* step_ctr, int max_steps, float* scores, float* seq_len,
                            int* stopped, int* tokens, int* tokens_tmp, int* kvrow,
                            int* kvrow_tmp, int Lmax, int* pos, int* next_tok, int* all_done,
                            void* stream) {
  ZS_REQUIRE(C > 0 && beam >= 1 && beam <= 8 && topk >= beam && nblk > 0,
             "zs_beam_step: 1 <= beam <= 8, topk >= beam");
  // one wave per source row (at least 4 waves for the history gathers)
  const dim3 blk(64 * (beam < 4 ? 4 : beam));
  if (beam <= 5)
    hipLaunchKernelGGL(beam_step_kernel<5>, dim3(C), blk, 0, S(stream), part_stat, part_val,
                       part_idx, beam, nblk, topk, first, stop, step_ctr, max_steps, scores,
                       seq_len, stopped, tokens, tokens_tmp, kvrow, kvrow_tmp, Lmax, pos, next_tok);
  else
    hipLaunchKernelGGL(beam_step_kernel<8>, dim3(C), blk, 0, S(stream), part_stat, part_val,
                       part_idx, beam, nblk, topk, first, stop, step_ctr, max_steps, scores,
                       seq_len, stopped, tokens, tokens_tmp, kvrow, kvrow_tmp, Lmax, pos, next_tok);
  ZS_LAUNCH_CHECK();
  hipLaunchKernelGGL(beam_advance_kernel, dim3(1), dim3(1024), 0, S(stream), stopped, C * beam,
                     step_ctr, max_steps, all_done);
  ZS_LAUNCH_CHECK();
  return 0;
}

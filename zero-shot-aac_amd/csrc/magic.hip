// CLAP-guided ("magic") decoding and the CLAP text tower it runs every step, batched over clips.
//
// Reference (/root/reference): gpt2_prefix_eval.py magic_search 341-393,
// PlugAndPlayContrastiveDecodingOneStepFast 396-469, enlarge/select_past_key_values 471-494,
// plug_and_play_fast_ranking 497-534, compute_audio_text_similarity_* 536-551,
// ComputeMagicScore 553-599, generate_beam_magic 602-689; ASE.encode_text
// retrieval/models/ase_model.py:57-60 over HF BertModel (text_encoder.py:58-68).
//
// Layout.  A batch of C clips decodes b beams per clip (b = 1 for magic_search), each beam
// proposing W candidates.  Candidate c = (clip k, beam j, w) is row c = (k*b + j)*W + w of every
// per-candidate buffer, and c is also the PHYSICAL ROW of the GPT-2 KV cache and of the
// context-hidden store ``ctx`` [rows][Lmax][D] where the candidate's position-p keys / values /
// ln_f hidden state land.  A beam owns no rows: ``kvrow[beam][t]`` names the physical row holding
// position t of its history (the prompt rows of clip k live at row k*b*W, written by the
// prefill), so the reference's enlarge (expand the cache W-fold) and select (gather the chosen
// candidate's cache) become copies of one int row per candidate and one int per beam -- nothing
// of the 12-layer cache moves.  Physical rows are tied to one clip for the whole decode and a
// row only ever receives the positions of its own clip's steps, so no live entry is overwritten.
#include "common.h"

namespace zs {

// ------------------------------------------------------------------ BERT embeddings + LN
// one wave per token row: x = LN(word[id] + pos[j] + type0) (eps 1e-12), f32 out and an optional
// operand copy h (bf16 in the perf mode); rows past a text's length are computed too (their ids
// are [PAD]) and only ever used as masked keys.
template <typename T>
__global__ __launch_bounds__(256) void bert_embed_ln_kernel(
    const int* __restrict__ ids, int rows, int L, const float* __restrict__ word,
    const float* __restrict__ pos, const float* __restrict__ type0, const float* __restrict__ g,
    const float* __restrict__ be, float eps, float* __restrict__ x, T* __restrict__ h) {
  constexpr int D = 768, PL = D / 64;
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int id = ids[r], j = r % L;
  float v[PL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PL; ++i) {
    const int c = lane + 64 * i;
    v[i] = word[(long)id * D + c] + pos[(long)j * D + c] + type0[c];
    s += v[i];
  }
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PL; ++i) { v[i] -= mean; q += v[i] * v[i]; }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
#pragma unroll
  for (int i = 0; i < PL; ++i) {
    const int c = lane + 64 * i;
    const float y = v[i] * rstd * g[c] + be[c];
    x[(long)r * D + c] = y;
    if (h) stf(h + (long)r * D + c, y);
  }
}

// LayerNorm of f32 rows to an f32 copy and an operand copy (BERT's post-LN residual stream and
// the next GEMM's A operand from one read), one wave per row, C = 768.
template <typename T>
__global__ __launch_bounds__(256) void ln_dual_kernel(const float* __restrict__ y, int rows,
                                                      int ldy, const float* __restrict__ g,
                                                      const float* __restrict__ be, float eps,
                                                      float* __restrict__ x, int ldx,
                                                      T* __restrict__ h, int ldh) {
  constexpr int D = 768, PL = D / 64;
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float v[PL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PL; ++i) { v[i] = y[(long)r * ldy + lane + 64 * i]; s += v[i]; }
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PL; ++i) { v[i] -= mean; q += v[i] * v[i]; }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
#pragma unroll
  for (int i = 0; i < PL; ++i) {
    const int c = lane + 64 * i;
    const float o = v[i] * rstd * g[c] + be[c];
    x[(long)r * ldx + c] = o;
    if (h) stf(h + (long)r * ldh + c, o);
  }
}

// ------------------------------------------------------------------ row top-k (+ softmax)
// One 1024-thread block per row of f32 logits [V <= 1024 * TOPK_NPT]: row max and sum of exp,
// then k rounds of a block argmax (ties -> the smaller index, torch.topk's order for distinct
// values); each thread keeps its values in registers and a taken-mask.  mode 0: value =
// log(softmax) (ComputeMagicScore, gpt2_prefix_eval.py:561-562); mode 1: softmax probability
// (PlugAndPlayContrastiveDecodingOneStepFast, 411-413).
constexpr int TOPK_NPT = 50;
__global__ __launch_bounds__(1024) void row_topk_kernel(const float* __restrict__ logits, int V,
                                                        long ld, int k, int mode,
                                                        float* __restrict__ out_val,
                                                        int* __restrict__ out_idx) {
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ int bidx;
  const int r = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const float* row = logits + (long)r * ld;
  float v[TOPK_NPT];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < TOPK_NPT; ++i) {
    const int c = t + 1024 * i;
    v[i] = c < V ? row[c] : -INFINITY;
    mx = fmaxf(mx, v[i]);
  }
  mx = wave_max(mx);
  if (lane == 0) sv[wid] = mx;
  __syncthreads();
  mx = sv[0];
#pragma unroll
  for (int i = 1; i < 16; ++i) mx = fmaxf(mx, sv[i]);
  float se = 0.f;
#pragma unroll
  for (int i = 0; i < TOPK_NPT; ++i) se += __expf(v[i] - mx);
  __syncthreads();
  const float sum = block_sum(se, sv);
  const float lse = mx + __logf(sum);
  uint64_t taken = 0;
  for (int it = 0; it < k; ++it) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < TOPK_NPT; ++i) {
      const int c = t + 1024 * i;
      const bool ok = c < V && !((taken >> i) & 1ull);
      if (ok && (v[i] > bv || (v[i] == bv && c < bi))) { bv = v[i]; bi = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    __syncthreads();
    if (lane == 0) { sv[wid] = bv; si[wid] = bi; }
    __syncthreads();
    if (t == 0) {
      float b = sv[0];
      int bj = si[0];
      for (int w = 1; w < 16; ++w)
        if (sv[w] > b || (sv[w] == b && si[w] < bj)) { b = sv[w]; bj = si[w]; }
      bidx = bj;
      out_idx[(long)r * k + it] = bj;
      out_val[(long)r * k + it] = mode == 0 ? b - lse : __expf(b - mx) / sum;
    }
    __syncthreads();
    const int win = bidx;
    if ((win & 1023) == t) taken |= 1ull << (win >> 10);
  }
}

// ------------------------------------------------------------------ candidate rows
// candidate c inherits its beam's history: kvrow_c[t] = kvrow[beam][t] for t < pos, and the
// beam's position (enlarge_past_key_values, gpt2_prefix_eval.py:471-480, as an index copy)
__global__ __launch_bounds__(128) void magic_expand_kernel(const int* __restrict__ kvrow,
                                                           const int* __restrict__ pos, int W,
                                                           int Lmax, int* __restrict__ kvrow_c,
                                                           int* __restrict__ pos_c) {
  const int c = blockIdx.x, j = c / W;
  const int p = pos[j];
  for (int t = threadIdx.x; t < p; t += blockDim.x)
    kvrow_c[(long)c * Lmax + t] = kvrow[(long)j * Lmax + t];
  if (threadIdx.x == 0) pos_c[c] = p;
}

// max over the beam's context of cos(context hidden, candidate hidden) (plug_and_play_fast_ranking
// 514-520 with prefix_length 1: every position), one wave per candidate; the candidate's own
// ln_f row is then stored at ctx[c][pos] (its position in the context store)
template <typename T>
__global__ __launch_bounds__(256) void magic_maxcos_kernel(const T* __restrict__ hid, int ncand,
                                                           int W, T* __restrict__ ctx, int Lmax,
                                                           const int* __restrict__ kvrow,
                                                           const int* __restrict__ pos,
                                                           float* __restrict__ maxcos) {
  constexpr int D = 768, PL = D / 64;
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= ncand) return;
  const int j = c / W, p = pos[j];
  float h[PL];
  float hh = 0.f;
#pragma unroll
  for (int i = 0; i < PL; ++i) { h[i] = ldf(hid + (long)c * D + lane + 64 * i); hh += h[i] * h[i]; }
  const float hn = sqrtf(wave_sum(hh));
  float best = -INFINITY;
  for (int t = 0; t < p; ++t) {
    const T* cr = ctx + ((long)kvrow[(long)j * Lmax + t] * Lmax + t) * D;
    float d = 0.f, cc = 0.f;
#pragma unroll
    for (int i = 0; i < PL; ++i) {
      const float x = ldf(cr + lane + 64 * i);
      d += x * h[i];
      cc += x * x;
    }
    d = wave_sum(d);
    cc = wave_sum(cc);
    best = fmaxf(best, d / (sqrtf(cc) * hn));
  }
  if (lane == 0) maxcos[c] = best;
  T* own = ctx + ((long)c * Lmax + p) * D;
#pragma unroll
  for (int i = 0; i < PL; ++i) own[lane + 64 * i] = hid[(long)c * D + lane + 64 * i];
}

// ranking score of every candidate of a clip (plug_and_play_fast_ranking 530-533 with the CLAP
// term of compute_audio_text_similarity_via_embeddings 541-547): clap = log_softmax over the
// clip's active candidates of cos(text, audio) / temp; score = (1-alpha) p - alpha maxcos +
// beta clap.  One block per clip; ``nact`` beams of the clip are active (1 at the first step).
__global__ __launch_bounds__(256) void magic_score_kernel(
    const float* __restrict__ pval, const float* __restrict__ maxcos,
    const float* __restrict__ text, const float* __restrict__ audio, int E, int b, int W,
    int nact, float inv_temp, float alpha, float beta, float* __restrict__ score, float stemp) {
  __shared__ float cl[8 * 64];
  const int k = blockIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n = nact * W;
  const float* a = audio + (long)k * E;
  float aa = 0.f;
  for (int e = lane; e < E; e += 64) aa += a[e] * a[e];
  const float an = sqrtf(wave_sum(aa));
  for (int i = wid; i < n; i += 4) {
    const float* tr = text + ((long)k * b * W + i) * E;
    float d = 0.f, tt = 0.f;
    for (int e = lane; e < E; e += 64) { d += tr[e] * a[e]; tt += tr[e] * tr[e]; }
    d = wave_sum(d);
    tt = wave_sum(tt);
    if (lane == 0) cl[i] = d / (sqrtf(tt) * an) * inv_temp;
  }
  __syncthreads();
  if (wid == 0) {
    float mx = -INFINITY;
    for (int i = lane; i < n; i += 64) mx = fmaxf(mx, cl[i]);
    mx = wave_max(mx);
    float s = 0.f;
    for (int i = lane; i < n; i += 64) s += __expf(cl[i] - mx);
    const float lse = mx + __logf(wave_sum(s));
    for (int i = lane; i < n; i += 64) {
      const long c = (long)k * b * W + i;
      const float sc = (1.0f - alpha) * pval[c] - alpha * maxcos[c] + beta * (cl[i] - lse);
      // generate_beam_magic's `temperature` divides the ranking score (gpt2_prefix_eval.py:629)
      score[c] = stemp != 1.0f ? sc / stemp : sc;
    }
  }
}

// ------------------------------------------------------------------ beam bookkeeping
// One block per clip.  beam mode = generate_beam_magic 626-683; greedy mode (b = 1) =
// magic_search's argmax selection 459-468 + stop 386.  A clip whose beams all stopped (or that
// reached its step limit) is frozen, as the reference leaves its loop.  For every beam it
// rewrites the history (kvrow) and token rows from the chosen source beam, sets kvrow[pos] to the
// chosen candidate's row, advances pos, and copies the candidate's ln_f row into sel_h (the next
// step's LM-head input).
constexpr int MAGIC_MAXB = 8, MAGIC_MAXW = 64;
template <typename T>
__global__ __launch_bounds__(256) void magic_step_kernel(
    const float* __restrict__ score, const int* __restrict__ cand, int b, int W, int first,
    int greedy, int stop, int step, const int* __restrict__ max_steps, float* __restrict__ scores,
    float* __restrict__ seq_len, int* __restrict__ stopped, int* __restrict__ tokens, int Smax,
    int* __restrict__ kvrow, int Lmax, int* __restrict__ pos, int* __restrict__ cdone,
    int* __restrict__ ntok, const T* __restrict__ hid, T* __restrict__ sel_h) {
  constexpr int D = 768;
  __shared__ int s_src[MAGIC_MAXB], s_cand[MAGIC_MAXB];
  __shared__ float s_sc[MAGIC_MAXB], s_len[MAGIC_MAXB];
  __shared__ int s_stop[MAGIC_MAXB], s_live;
  const int k = blockIdx.x, t = threadIdx.x;
  const long bw = (long)k * b;
  if (t == 0) {
    s_live = !cdone[k] && step < max_steps[k];
    if (s_live) {
      const float* sc = score + bw * W;
      if (greedy) {                             // magic_search: argmax over the W candidates
        int bi = 0;
        for (int w = 1; w < W; ++w) if (sc[w] > sc[bi]) bi = w;
        s_src[0] = 0; s_cand[0] = bi;
        s_sc[0] = 0.f; s_len[0] = 1.f;
        s_stop[0] = cand[bw * W + bi] == stop;
      } else if (first) {                       // topk(beam) of the single row's W scores
        bool used[MAGIC_MAXW] = {};
        for (int j = 0; j < b; ++j) {
          int bi = -1;
          for (int w = 0; w < W; ++w)
            if (!used[w] && (bi < 0 || sc[w] > sc[bi])) bi = w;
          used[bi] = true;
          s_src[j] = 0; s_cand[j] = bi; s_sc[j] = sc[bi]; s_len[j] = 1.f;
          s_stop[j] = cand[bw * W + bi] == stop;
        }
      } else {                                  // length-normalised topk over beam x W
        float len1[MAGIC_MAXB];
        for (int j = 0; j < b; ++j) len1[j] = seq_len[bw + j] + (stopped[bw + j] ? 0.f : 1.f);
        bool used[MAGIC_MAXB * MAGIC_MAXW] = {};
        for (int q = 0; q < b; ++q) {
          int bi = -1;
          float bv = -INFINITY;
          for (int i = 0; i < b * W; ++i) {
            const int j = i / W, w = i % W;
            float v = sc[i];
            if (stopped[bw + j]) v = w == 0 ? 0.f : -INFINITY;
            const float avg = (scores[bw + j] + v) / len1[j];
            if (!used[i] && (bi < 0 || avg > bv)) { bi = i; bv = avg; }
          }
          used[bi] = true;
          const int j = bi / W;
          s_src[q] = j; s_cand[q] = bi % W;
          s_len[q] = len1[j];
          s_sc[q] = bv * len1[j];
          s_stop[q] = stopped[bw + j] || cand[bw * W + bi] == stop;
        }
      }
    }
  }
  __syncthreads();
  if (!s_live) return;
  // new histories: gather source rows into registers / LDS first (sources are beams of this
  // clip, rewritten below)
  extern __shared__ int sh[];               // [b][Lmax] kvrow, then [b][Smax] tokens
  int* okv = sh;
  int* otk = sh + b * Lmax;
  const int p = pos[bw];
  for (int i = t; i < b * Lmax; i += blockDim.x) okv[i] = kvrow[bw * Lmax + i];
  for (int i = t; i < b * Smax; i += blockDim.x) otk[i] = tokens[bw * Smax + i];
  __syncthreads();
  for (int q = 0; q < b; ++q) {
    const int src = s_src[q];
    const long c = (bw + src) * W + s_cand[q];
    for (int i = t; i < p; i += blockDim.x) kvrow[(bw + q) * Lmax + i] = okv[src * Lmax + i];
    for (int i = t; i < step; i += blockDim.x) tokens[(bw + q) * Smax + i] = otk[src * Smax + i];
    for (int i = t; i < D; i += blockDim.x) sel_h[(bw + q) * D + i] = hid[c * D + i];
    if (t == 0) {
      kvrow[(bw + q) * Lmax + p] = (int)c;
      tokens[(bw + q) * Smax + step] = cand[c];
      scores[bw + q] = s_sc[q];
      seq_len[bw + q] = s_len[q];
      stopped[bw + q] = s_stop[q];
      pos[bw + q] = p + 1;
    }
  }
  if (t == 0) {
    bool all = true;
    for (int q = 0; q < b; ++q) all = all && s_stop[q];
    ntok[k] = step + 1;
    if (all || step + 1 >= max_steps[k]) cdone[k] = 1;
  }
}

}  // namespace zs

using namespace zs;

extern "C" int zs_bert_embed_ln(const int* ids, int rows, int L, const float* word, const float* pos,
                                const float* type0, const float* ln_w, const float* ln_b, float eps,
                                float* x, void* h, int hdtype, void* stream) {
  ZS_REQUIRE(rows > 0 && L > 0 && ids && word && pos && type0 && ln_w && ln_b && x,
             "zs_bert_embed_ln: bad arguments");
  if (hdtype == ZS_BF16)
    hipLaunchKernelGGL(bert_embed_ln_kernel<bf16_t>, dim3(cdiv(rows, 4)), dim3(256), 0, S(stream),
                       ids, rows, L, word, pos, type0, ln_w, ln_b, eps, x, (bf16_t*)h);
  else
    hipLaunchKernelGGL(bert_embed_ln_kernel<float>, dim3(cdiv(rows, 4)), dim3(256), 0, S(stream),
                       ids, rows, L, word, pos, type0, ln_w, ln_b, eps, x, (float*)h);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_layernorm_dual(const float* y, int rows, int C, int ldy, const float* ln_w,
                                 const float* ln_b, float eps, float* x, int ldx, void* h, int ldh,
                                 int hdtype, void* stream) {
  ZS_REQUIRE(rows >= 0 && C == 768 && y && ln_w && ln_b && x, "zs_layernorm_dual: C must be 768");
  if (rows == 0) return 0;
  if (hdtype == ZS_BF16)
    hipLaunchKernelGGL(ln_dual_kernel<bf16_t>, dim3(cdiv(rows, 4)), dim3(256), 0, S(stream), y,
                       rows, ldy, ln_w, ln_b, eps, x, ldx, (bf16_t*)h, ldh);
  else
    hipLaunchKernelGGL(ln_dual_kernel<float>, dim3(cdiv(rows, 4)), dim3(256), 0, S(stream), y,
                       rows, ldy, ln_w, ln_b, eps, x, ldx, (float*)h, ldh);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_row_topk(const float* logits, int R, int V, long ld, int k, int mode,
                           float* out_val, int* out_idx, void* stream) {
  ZS_REQUIRE(R > 0 && V > 0 && V <= 1024 * TOPK_NPT && ld >= V && k >= 1 && k <= 64 && k <= V,
             "zs_row_topk: 0 < V <= %d, 1 <= k <= 64", 1024 * TOPK_NPT);
  ZS_REQUIRE(mode == 0 || mode == 1, "zs_row_topk: mode 0 (log softmax) or 1 (softmax)");
  hipLaunchKernelGGL(row_topk_kernel, dim3(R), dim3(1024), 0, S(stream), logits, V, ld, k, mode,
                     out_val, out_idx);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_magic_expand(const int* kvrow, const int* pos, int nbeams, int W, int Lmax,
                               int* kvrow_c, int* pos_c, void* stream) {
  ZS_REQUIRE(nbeams > 0 && W > 0 && Lmax > 0, "zs_magic_expand: bad shape");
  hipLaunchKernelGGL(magic_expand_kernel, dim3(nbeams * W), dim3(128), 0, S(stream), kvrow, pos, W,
                     Lmax, kvrow_c, pos_c);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_magic_maxcos(const void* hid, int ncand, int W, void* ctx, int Lmax,
                               const int* kvrow, const int* pos, float* maxcos, int dtype,
                               void* stream) {
  ZS_REQUIRE(ncand > 0 && W > 0 && Lmax > 0, "zs_magic_maxcos: bad shape");
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(magic_maxcos_kernel<bf16_t>, dim3(cdiv(ncand, 4)), dim3(256), 0, S(stream),
                       (const bf16_t*)hid, ncand, W, (bf16_t*)ctx, Lmax, kvrow, pos, maxcos);
  else
    hipLaunchKernelGGL(magic_maxcos_kernel<float>, dim3(cdiv(ncand, 4)), dim3(256), 0, S(stream),
                       (const float*)hid, ncand, W, (float*)ctx, Lmax, kvrow, pos, maxcos);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_magic_score(const float* pval, const float* maxcos, const float* text,
                              const float* audio, int C, int E, int b, int W, int nact, float temp,
                              float alpha, float beta, float* score, void* stream) {
  return zs_magic_score_t(pval, maxcos, text, audio, C, E, b, W, nact, temp, alpha, beta, 1.0f,
                          score, stream);
}

extern "C" int zs_magic_score_t(const float* pval, const float* maxcos, const float* text,
                                const float* audio, int C, int E, int b, int W, int nact,
                                float temp, float alpha, float beta, float score_temp,
                                float* score, void* stream) {
  ZS_REQUIRE(score_temp > 0.f, "zs_magic_score_t: temperature %g (> 0)", score_temp);
  ZS_REQUIRE(C > 0 && E > 0 && b >= 1 && b <= MAGIC_MAXB && W >= 1 && W <= MAGIC_MAXW &&
             nact >= 1 && nact <= b && nact * W <= 8 * 64 && temp > 0.f,
             "zs_magic_score: 1 <= beams <= %d, 1 <= width <= %d", MAGIC_MAXB, MAGIC_MAXW);
  hipLaunchKernelGGL(magic_score_kernel, dim3(C), dim3(256), 0, S(stream), pval, maxcos, text,
                     audio, E, b, W, nact, 1.0f / temp, alpha, beta, score, score_temp);
  ZS_LAUNCH_CHECK();
  return 0;
}

extern "C" int zs_magic_step(const float* score, const int* cand, int C, int b, int W, int first,
                             int greedy, int stop, int step, const int* max_steps, float* scores,
                             float* seq_len, int* stopped, int* tokens, int Smax, int* kvrow,
                             int Lmax, int* pos, int* cdone, int* ntok, const void* hid,
                             void* sel_h, int dtype, void* stream) {
  ZS_REQUIRE(C > 0 && b >= 1 && b <= MAGIC_MAXB && W >= b && W <= MAGIC_MAXW && step >= 0 &&
             step < Smax && Lmax > 0 && (!greedy || b == 1),
             "zs_magic_step: 1 <= beams <= min(width, %d), width <= %d, step < Smax",
             MAGIC_MAXB, MAGIC_MAXW);
  const size_t lds = (size_t)b * (Lmax + Smax) * sizeof(int);
  ZS_REQUIRE(lds <= 64 * 1024, "zs_magic_step: beams x (Lmax + Smax) too large");
  if (dtype == ZS_BF16)
    hipLaunchKernelGGL(magic_step_kernel<bf16_t>, dim3(C), dim3(256), lds, S(stream), score, cand,
                       b, W, first, greedy, stop, step, max_steps, scores, seq_len, stopped,
                       tokens, Smax, kvrow, Lmax, pos, cdone, ntok, (const bf16_t*)hid,
                       (bf16_t*)sel_h);
  else
    hipLaunchKernelGGL(magic_step_kernel<float>, dim3(C), dim3(256), lds, S(stream), score, cand,
                       b, W, first, greedy, stop, step, max_steps, scores, seq_len, stopped,
                       tokens, Smax, kvrow, Lmax, pos, cdone, ntok, (const float*)hid,
                       (float*)sel_h);
  ZS_LAUNCH_CHECK();
  return 0;
}

/*
 * zsaac.h — C-ABI of libzsaac_hip.so, the MI355X (gfx950) kernels behind the zero-shot audio
 * captioning hot path of XinMing0411/zero-shot-AAC.
 *
 * Conventions:
 *   - every pointer is a DEVICE pointer owned by the caller (PyTorch caching allocator); the
 *     library never allocates or frees caller memory;
 *   - shapes/strides are explicit ints, element strides (not bytes);
 *   - `dtype` selects the storage/compute type of weights and GEMM operands:
 *       ZS_F32  = parity mode (f32 operands, exact-f32 MFMA 32x32x2f32, f32 accumulate)
 *       ZS_BF16 = perf mode   (bf16 operands, MFMA 32x32x16 bf16, f32 accumulate)
 *     residual streams, softmax, LayerNorm statistics and all reductions are f32 in both modes;
 *   - `stream` is a hipStream_t (pass torch.cuda.current_stream().cuda_stream); every launch is
 *     stream-ordered, allocation-free and sync-free, so a caller may capture it into a hipGraph;
 *   - return 0 on success or a negative zs_status; zs_last_error() gives a thread-local message.
 *
 * Each entry point names the reference code it replaces (paths under the reference repo root).
 */
#ifndef ZSAAC_H
#define ZSAAC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum zs_status { ZS_OK = 0, ZS_ERR_ARG = -1, ZS_ERR_DTYPE = -2, ZS_ERR_HIP = -3, ZS_ERR_UNSUPPORTED = -4 };
enum zs_dtype { ZS_F32 = 0, ZS_BF16 = 1 };
enum zs_act { ZS_ACT_NONE = 0, ZS_ACT_GELU_ERF = 1, ZS_ACT_GELU_TANH = 2, ZS_ACT_RELU = 3, ZS_ACT_TANH = 4 };

/* ------------------------------------------------------------------ runtime */
int zs_version(void);                         /* ABI version, bumped on signature change */
int zs_last_error(char* buf, size_t len);     /* copies the thread-local last error message */
int zs_device_arch(char* buf, size_t len);    /* gcnArchName of the current device (e.g. gfx950) */
int zs_tune_set(const char* key, int value);  /* tuning knobs, e.g. "skinny_mode" (0 fence, 1 sc1) */
/* zs_stream_create: a new non-blocking HIP stream, bound to its hardware queue at once (ROCclr
 * assigns queues round-robin at a stream's first dispatch), so streams created back to back run
 * on distinct hardware queues while GPU_MAX_HW_QUEUES allows.  Used for the concurrent batch
 * streams (two streams sharing a hardware queue serialize).  priority < 0: the device's highest
 * stream priority, > 0: its lowest, 0: the default. */
int zs_stream_create(void** stream, int priority);
/* zs_stream_create_masked: the same, restricted to the CUs whose bits are set in cu_mask
 * (mask_words 32-bit words, bit i = CU i, hipExtStreamCreateWithCUMask): the caption runner's
 * optional split of the chip between the begins (prompt .. step 0) and the decode grids. */
int zs_stream_create_masked(void** stream, const unsigned* cu_mask, int mask_words);
int zs_stream_destroy(void* stream);
/* zs_stream_spin: enqueue a one-wave kernel that holds `stream` for `us` microseconds (s_memrealtime,
 * 100 MHz; nothing written): the caption runner releases the first wave of persistent decode grids
 * one after another, 200 us apart, after a gate they all wait on -- released together, the
 * dispatcher sometimes left one grid without room for all its workgroups until another grid
 * ended (a grid ~40 ms late; profiles/r6/begin_first_ab.txt).  0 <= us <= 1e6; us == 0 enqueues
 * nothing. */
int zs_stream_spin(int us, void* stream);

/* ------------------------------------------------------------------ audio front end
 * zs_logmel: retrieval/models/feature_extractor.py:34-38 (torchlibrosa Spectrogram +
 * LogmelFilterBank, n_fft 1024, hop 320, hann, center/reflect, power 2, 64 Slaney mels,
 * 10*log10(max(x,1e-10))) fused with bn0 (htsat.py:949-951 / cnns.py:176-178):
 *   wav [B][T] f32 -> out [B][n_frames][64] f32, n_frames = T/hop + 1.
 * window[1024], twiddle[1024] = (cos, sin)(-2*pi*k/1024) interleaved for k < 512 (the DFT is a
 * radix-4 FFT in LDS, two real frames packed per complex FFT), melW[64][513] (librosa.filters.mel, row m nonzero on
 * [mel_lo[m], mel_hi[m])), bn_{mean,var,weight,bias}[64] (eval BatchNorm, eps 1e-5; pass NULL
 * bn_mean to skip bn0). */
int zs_logmel(const float* wav, int B, int T, const float* window, const float* twiddle,
              const float* melW,
              const int* mel_lo, const int* mel_hi, const float* bn_mean, const float* bn_var,
              const float* bn_weight, const float* bn_bias, float* out, void* stream);

/* zs_wav2img: htsat.py:908-923 reshape_wav2img — bicubic (A=-0.75, align_corners=True) resize of
 * the time axis T_in -> 1024 and fold (B,1,1024,64) -> (B,256,256).  in [B][T_in][64] f32. */
int zs_wav2img(const float* in, int B, int T_in, float* img, void* stream);

/* zs_pack_clips: ragged mono clips (clip b = flat[offsets[b] .. offsets[b] + lengths[b])) ->
 * out [B][T] f32: each cropped to its first T samples or zero-padded at the end, exactly as
 * data_handing/embeddings_generator.py:53-59 fits clips to max_length * sr before encode_audio.
 * T % 4 == 0; out 16-byte aligned. */
int zs_pack_clips(const float* flat, const long* offsets, const int* lengths, int B, int T,
                  float* out, void* stream);

/* zs_patch_embed: htsat.py:115-125 PatchEmbed (Conv2d 1->96, k4 s4) + LayerNorm(96):
 * img [B][256][256] f32 -> x [B*4096][96] f32 (token = row*64 + col of the 64x64 patch grid). */
int zs_patch_embed(const float* img, int B, const float* w /*[96][16]*/, const float* b,
                   const float* ln_w, const float* ln_b, float* x, void* stream);

/* ------------------------------------------------------------------ generic building blocks
 * zs_layernorm: y[m] = LN(x[rows ? rows[m] : m]) * w + b over C (eps), x f32, y in `ydtype`
 * (ZS_F32/ZS_BF16).  `rows` (int32, may be NULL) gathers rows, e.g. GPT-2 ln_f on the last
 * prompt position of every ragged row. */
int zs_layernorm(const float* x, int M, int C, int ldx, const int* rows, const float* w,
                 const float* b, float eps, void* y, int ldy, int ydtype, void* stream);

/* zs_gemm: out[m][n] = act(sum_k A[m][k] * W[n][k] + bias[n]) + residual[m][n]
 *   A [M][lda], W [N][ldw] in `dtype`; bias f32 or NULL; residual f32 [M][ldr] or NULL (may alias
 *   out); out in `out_dtype`.  K % 32 == 0.  split_k > 1 needs a f32 workspace of
 *   split_k*M*N floats (deterministic slab reduction, no atomics).  split_k == 0 = auto: for
 *   M <= 64 (decode) a weight-streaming split-K kernel whose last-arriving workgroup reduces the
 *   slabs in order (deterministic); it needs a workspace of zs_gemm_workspace_floats(M,N,K) floats
 *   ZEROED ONCE at allocation (its tile counters re-arm themselves).
 *   Replaces every nn.Linear / HF Conv1D on the path (Conv1D weights are repacked to [N][K]). */
int zs_gemm(int M, int N, int K, int dtype, const void* A, int lda, const void* W, int ldw,
            const float* bias, const float* residual, int ldr, void* out, int ldo, int out_dtype,
            int act, int split_k, float* workspace, void* stream);

int zs_gemm_workspace_floats(int M, int N, int K);

/* zs_gemm_ln: out[m][n] = act(sum_k LN(x[m])[k] * W[n][k] + bias[n]) + residual[m][n] for
 *   M <= 64 rows (the GPT-2 decode step at the reference's eval batch of 64): LayerNorm over K
 *   (eps; ln_w / ln_b f32) of the f32 rows x [M][ldx], rounded to bf16, times bf16 W [N][ldw].
 *   Replaces the ln_1 -> attn.c_attn and ln_2 -> mlp.c_fc launch pairs of transformers'
 *   GPT2Block (the zs_layernorm + zs_gemm sequence).  K % 128 == 0, K <= 1024; x, ln_w, ln_b
 *   and W 16-byte aligned.  One launch, no workspace. */
int zs_gemm_ln(int M, int N, int K, const float* x, int ldx, const float* ln_w, const float* ln_b,
               float eps, const void* W, int ldw, const float* bias, const float* residual,
               int ldr, void* out, int ldo, int out_dtype, int act, void* stream);

/* zs_gemm_ln_f32: zs_gemm_ln with f32 W [N][ldw] and f32 out (the f32 parity mode's decode
 *   step): LayerNorm of the f32 rows x with the affine (ln_w, ln_b) applied in f32, exact f32
 *   products and f32 accumulation (v_mfma_f32_16x16x4_f32).  M <= 64, K 768 or 1024; x, W and
 *   the LN params 16-byte aligned.  Replaces GPT2Block's ln_1 -> c_attn / ln_2 -> c_fc pairs.
 *   ln_w == ln_b == NULL: no LayerNorm (out = act(x W^T + b) + residual, K up to 3072: the
 *   attn.c_proj / mlp.c_proj of the same step).  zs_gemm keeps its own f32 kernels, so a row's
 *   zs_gemm result stays independent of how many rows share the launch. */
int zs_gemm_ln_f32(int M, int N, int K, const float* x, int ldx, const float* ln_w,
                   const float* ln_b, float eps, const float* W, int ldw, const float* bias,
                   const float* residual, int ldr, float* out, int ldo, int act, void* stream);

/* zs_l2norm_rows: y = x / max(||x||_2, eps) per row (F.normalize, ase_model.py:54). in-place ok */
int zs_l2norm_rows(const float* x, int M, int C, float eps, float* y, void* stream);

/* ------------------------------------------------------------------ HTSAT
 * zs_window_attention: htsat.py:312-347 W-MSA/SW-MSA for one SwinTransformerBlock, with the
 * cyclic roll (htsat.py:443-463), window partition/reverse and the -100 shift mask (406-425)
 * folded into the indexing.  qkv [B*H*W][3C] (dtype) in natural token order; out [B*H*W][C]
 * (dtype) in natural token order.  head_dim = C/heads (24 in HTSAT), ws*ws == 64.
 * rel_table [(2ws-1)^2][heads] f32. */
int zs_window_attention(const void* qkv, int B, int H, int W, int C, int heads, int ws, int shift,
                        const float* rel_table, void* out, int dtype, void* stream);

/* zs_swin_block: one whole SwinTransformerBlock (htsat.py:427-474, eval) in ONE launch, bf16
 * operands / f32 residual: x += proj(WindowAttention(LN1(x))); x += fc2(GELU(fc1(LN2(x)))),
 * with the roll, window partition/reverse, rel-pos bias and -100 shift mask folded in (replaces
 * the zs_layernorm / zs_gemm / zs_window_attention sequence of one block).  One workgroup per
 * 8x8 window.  x [B*H*W][C] f32, updated in place.  C in {96, 192, 384}, heads = C / 24.
 * Weights are fragment-packed bf16 (see csrc/swin.hip): frag(nt, ks)[lane][j] =
 * W[16 nt + lane%16][32 ks + 8 (lane/16) + j], stored [N/16][K/32][64][8]:
 *   wqkv_packed: qkv.weight regrouped per group of G heads (G = 2 for C <= 192, 4 for C = 384)
 *   as rows [q h0..h(G-1), k h0.., v h0..] x 32 (head dim 24 zero-padded to 32) =
 *   [heads/G][96 G][C], then packed;  bqkv_packed [heads/G][96 G] f32 (same order, zero pad);  wproj [C][C], w1 [4C][C],
 *   w2 [C][4C] packed;  biases / LayerNorm params f32;  rel_table [225][heads] f32. */
int zs_swin_block(float* x, int B, int H, int W, int C, int heads, int shift, const float* ln1_w,
                  const float* ln1_b, const void* wqkv_packed, const float* bqkv_packed,
                  const float* rel_table, const void* wproj_packed, const float* bproj,
                  const float* ln2_w, const float* ln2_b, const void* w1_packed, const float* b1,
                  const void* w2_packed, const float* b2, void* stream);

/* zs_patch_merge_ln: htsat.py:492-511 gather x0..x3 of each 2x2 patch + LayerNorm(4C):
 * x [B][H][W][C] f32 -> y [B*(H/2)*(W/2)][4C] (dtype); the reduction Linear is a zs_gemm. */
int zs_patch_merge_ln(const float* x, int B, int H, int W, int C, const float* ln_w,
                      const float* ln_b, void* y, int dtype, void* stream);

/* zs_ln_meanpool: htsat.py:830,838-847 final LayerNorm + mean over the N tokens -> [B][C] f32. */
int zs_ln_meanpool(const float* x, int B, int N, int C, const float* ln_w, const float* ln_b,
                   float* out, void* stream);

/* ------------------------------------------------------------------ CNN14 (cnns.py:36-78,171-201)
 * zs_conv3x3_bn_relu: NHWC implicit-GEMM conv3x3 pad 1 (no bias) + eval BN + ReLU.
 *   x [B][H][W][Cin] (dtype), w [Cout][3][3][Cin] (dtype), bn folded as scale/shift f32 [Cout]
 *   (y = relu(conv*scale + shift)), out [B][H][W][Cout] (dtype). */
int zs_conv3x3_bn_relu(const void* x, int B, int H, int W, int Cin, const void* w, int Cout,
                       const float* scale, const float* shift, void* out, int dtype, void* stream);
/* zs_avgpool2: 2x2 average pool (floor) NHWC, dtype in/out. */
int zs_avgpool2(const void* x, int B, int H, int W, int C, void* out, int dtype, void* stream);
/* zs_cnn_head: mean over freq (W) then max + mean over time (H): x [B][H][W][C] -> [B][C] f32. */
int zs_cnn_head(const void* x, int B, int H, int W, int C, float* out, int dtype, void* stream);
/* zs_cast: f32 -> dtype element copy (e.g. the bn0'd log-mel as the NHWC C=1 CNN14 input). */
int zs_cast(const float* x, long n, void* y, int dtype, void* stream);

/* ------------------------------------------------------------------ prompt
 * zs_prompt_assemble: dataset/dataset.py:441-453 + utils.py:131-188 on device —
 * sim = emb[b] . labels^T (softmax is monotonic: top-k on sim, ties -> lower index), then
 * ids = head + (label ids + ',')* + tail ("There are l1, l2 in this audio.").
 * label_tok [L][max_tok] int32 with label_len[L]; out hard_ids [B][h_cap] int32 (0-padded,
 * padding_captions utils.py:190-208), hard_len [B], chosen [B][k] int32 (may be NULL). */
int zs_prompt_assemble(const float* emb, int B, int D, const float* labels, int L, int k,
                       const int* label_tok, const int* label_len, int max_tok, int* hard_ids,
                       int h_cap, int* hard_len, int* chosen, void* stream);

/* ------------------------------------------------------------------ mapper / small attention
 * zs_row_attention: per row b, per head h: softmax(scale * q_i . k_j) v_j over j < len[b]
 * (causal: j <= i).  q element (b, i, h, d) at q[(b*L + i)*ldq + h*hd + d], k/v likewise with
 * ldkv, out with ldo (all dtype).  Serves models/mapper.py:49-66 (non-causal, hd 96) and the GPT-2
 * prompt prefill (causal, hd 64).  L <= 128, hd <= 128. */
int zs_row_attention(const void* q, int ldq, const void* k, const void* v, int ldkv, int B, int L,
                     const int* len, int heads, int hd, int causal, float scale, void* out, int ldo,
                     int dtype, void* stream);

/* zs_row_attention_kv: the GPT-2 prompt prefill's attention fused with its KV-cache write
 * (gpt2_prefix_eval.py:99-158 via transformers GPT2Attention with use_cache; replaces the
 * zs_kv_write + zs_row_attention pair of a layer): qkv [B*L][3*heads*64] bf16 (q | k | v, head
 * dim 64), causal over j < len[b], L <= 32; out rows with ldo; k / v of all L rows stored into
 * kc / vc [B*row_stride][heads][Lmax][64] at positions 0..L-1 exactly as zs_kv_write (pos0 NULL)
 * stores them. */
int zs_row_attention_kv(const void* qkv, int B, int L, const int* len, int heads, float scale,
                        void* out, int ldo, void* kc, void* vc, int Lmax, int row_stride,
                        void* stream);

/* zs_cross_attention: nn.MultiheadAttention's core (after in_proj, before out_proj) for short
 * key sets: out(b, i, h) = softmax_j(scale * q(b,i,h) . k(b,j,h)) v(b,j,h), j < Lk; q rows
 * b*Lq + i (ldq), k / v rows b*Lk + j (ldkv), head h at columns h*hd.. (dtype).  Serves the
 * sound-effect cross-attention of ClapCaptionCrossattention[_v2] (models/caption_model.py:100-206,
 * nn.MultiheadAttention(prefix_size, 4)).  Lk <= 64, hd <= 256. */
int zs_cross_attention(const void* q, int ldq, const void* k, const void* v, int ldkv, int B,
                       int Lq, int Lk, int heads, int hd, float scale, void* out, int ldo,
                       int dtype, void* stream);

/* zs_label_topk: sound_effect_choice (caption_model.py:15-20, utils.py:131-137): per row b the
 * k labels (of L, rows of labels [L][D] f32) with the highest similarity emb[b] . label, best
 * first, ties to the lower index (softmax is monotone); idx [B][k] int32 (may be NULL) and the
 * chosen rows gathered into rows [B][k][D] f32.  k <= 16, (D + L) * 4 <= 64 KB. */
int zs_label_topk(const float* emb, int B, int D, const float* labels, int L, int k, int* idx,
                  float* rows, void* stream);

/* ------------------------------------------------------------------ CLAP-guided ("magic") decoding
 * gpt2_prefix_eval.py:341-689 (magic_search, generate_beam_magic and their helpers) batched over C
 * clips, b beams per clip (b = 1: magic_search), W candidates per beam.  Candidate c =
 * (clip*b + beam)*W + w is also the physical row of the GPT-2 KV cache and of the context-hidden
 * store ctx [rows][Lmax][768] that holds its position-pos entries; kvrow [beam][Lmax] names the
 * row holding each position of a beam's history (enlarge/select_past_key_values,
 * gpt2_prefix_eval.py:471-494, as index copies). */

/* zs_bert_embed_ln: HF BertEmbeddings (input_ids, position ids 0..L-1, token type 0) +
 * LayerNorm(eps) for rows = texts*L token rows (ids int32 [rows], row r = text*L + j): x f32
 * [rows][768], and h (hdtype) the same values as the next GEMM's operand (may be NULL).
 * Replaces BertModel's embedding layer under ASE.encode_text (text_encoder.py:64-68). */
int zs_bert_embed_ln(const int* ids, int rows, int L, const float* word, const float* pos,
                     const float* type0, const float* ln_w, const float* ln_b, float eps, float* x,
                     void* h, int hdtype, void* stream);

/* zs_layernorm_dual: LayerNorm of f32 rows y (ldy) into f32 x (ldx) and the operand copy h
 * (hdtype, ldh; may be NULL) -- BERT's post-LN residual stream (BertSelfOutput / BertOutput).
 * C must be 768. */
int zs_layernorm_dual(const float* y, int rows, int C, int ldy, const float* ln_w,
                      const float* ln_b, float eps, float* x, int ldx, void* h, int ldh,
                      int hdtype, void* stream);

/* zs_row_topk: per row of f32 logits [R][V] (row stride ld): the k largest (best first, ties to
 * the lower index) as out_idx [R][k] int32 and out_val [R][k] = log(softmax) (mode 0,
 * ComputeMagicScore gpt2_prefix_eval.py:560-562) or softmax probability (mode 1,
 * PlugAndPlayContrastiveDecodingOneStepFast 411-413).  V <= 51200, k <= 64. */
int zs_row_topk(const float* logits, int R, int V, long ld, int k, int mode, float* out_val,
                int* out_idx, void* stream);

/* zs_magic_expand: candidate c = beam*W + w inherits its beam's history: kvrow_c[c][t] =
 * kvrow[beam][t] for t < pos[beam], pos_c[c] = pos[beam] (enlarge_past_key_values 471-480). */
int zs_magic_expand(const int* kvrow, const int* pos, int nbeams, int W, int Lmax, int* kvrow_c,
                    int* pos_c, void* stream);

/* zs_magic_maxcos: maxcos[c] = max over t < pos[beam] of cos(ctx[kvrow[beam][t]][t], hid[c])
 * (plug_and_play_fast_ranking 514-520, prefix_length 1), hid [ncand][768] = the candidates' ln_f
 * rows (dtype); then stores hid[c] at ctx[c][pos[beam]]. */
int zs_magic_maxcos(const void* hid, int ncand, int W, void* ctx, int Lmax, const int* kvrow,
                    const int* pos, float* maxcos, int dtype, void* stream);

/* zs_magic_score: per clip k, over its first nact*W candidates (nact = 1 at the first beam step):
 * clap = log_softmax_c(cos(text[c], audio[k]) / temp) (gpt2_prefix_eval.py:541-547);
 * score[c] = (1 - alpha) pval[c] - alpha maxcos[c] + beta clap[c] (plug_and_play_fast_ranking
 * 530-531).  text [C*b*W][E], audio [C][E] f32.  b <= 8, W <= 64, nact*W <= 512. */
int zs_magic_score(const float* pval, const float* maxcos, const float* text, const float* audio,
                   int C, int E, int b, int W, int nact, float temp, float alpha, float beta,
                   float* score, void* stream);
/* zs_magic_score_t: zs_magic_score with the score divided by score_temp (> 0):
 * generate_beam_magic's `temperature` (gpt2_prefix_eval.py:629). */
int zs_magic_score_t(const float* pval, const float* maxcos, const float* text, const float* audio,
                     int C, int E, int b, int W, int nact, float temp, float alpha, float beta,
                     float score_temp, float* score, void* stream);

/* zs_magic_step: one selection step per clip (one block each).  greedy = 0: generate_beam_magic
 * 626-683 (first: topk(b) of beam 0's W scores; later: stopped beams keep candidate 0 at zero
 * cost, length-normalised topk over b*W, scores = avg * seq_len); greedy = 1 (b = 1):
 * magic_search's argmax 459-468.  Rewrites each beam's kvrow / token row from its source beam,
 * kvrow[beam][pos] = chosen candidate row, pos += 1, tokens[beam][step] = chosen id, copies the
 * candidate's ln_f row hid[c] to sel_h[beam] (the next LM-head input); a clip is frozen
 * (cdone[k] = 1) once all its beams stopped or step + 1 >= max_steps[k]; ntok[k] = tokens
 * emitted.  tokens [C*b][Smax], kvrow [C*b][Lmax] int32. */
int zs_magic_step(const float* score, const int* cand, int C, int b, int W, int first, int greedy,
                  int stop, int step, const int* max_steps, float* scores, float* seq_len,
                  int* stopped, int* tokens, int Smax, int* kvrow, int Lmax, int* pos, int* cdone,
                  int* ntok, const void* hid, void* sel_h, int dtype, void* stream);

/* ------------------------------------------------------------------ Mistral-7B decoder (C5)
 * predict_mistralai_multilingual.py:97-111 / models/caption_model.py:340-413: batched greedy
 * MistralForCausalLM.generate over inputs_embeds.  head_dim 128, grouped-query attention.
 * Split-K GEMM results are f32 slabs [nsplit][M][N] (split stride ss) summed in order by their
 * consumer (RoPE/KV append, SiLU*up, add+RMSNorm): deterministic, no reduction launch. */

/* zs_fp8_gemm_rows: weight-only fp8 GEMM for M <= 64 rows (decode): out[s][m][n] = scale[n] *
 * sum_{k in split s} A[m][k] W[n][k]; A bf16 [M][lda], W8 the fp8 e4m3 (OCP) codes of W [N][K]
 * TILE-PACKED [K/1024][ceil(N/128)][8][16][64][16 B] (zsaac/mistral.py fp8_pack_tiles: block
 * (s, t, w, j), lane l = W[128 t + 16 w + (l & 15)][1024 s + 64 j + 16 (l >> 4) .. +16], rows past
 * N zero), scale f32 [N] (one per output channel), K % 1024 == 0, splits of 1024 along K
 * (zs_fp8_splits(K) of them), ldo >= N.
 * Replaces the NF4-quantised q/k/v/o/gate/up/down projections of the LoRA-wrapped Mistral
 * (caption_model.py:355-364). */
int zs_fp8_gemm_rows(const void* A, int lda, const void* W8, const float* scale, int M, int N,
                     int K, float* out, long split_stride, int ldo, void* stream);
int zs_fp8_splits(int K);

/* zs_fp8_gemm_run: the same product for M <= 32 with one workgroup per (128-column tile, run of
 * ks consecutive splits, k half of kh), the run summed in registers: out gets
 * zs_fp8_splits(K) / ks * kh slabs (slab (run, half) at index run * kh + half; kh 2 halves each
 * split between two workgroups, for short streams).
 * act != NULL (GLU; ks == zs_fp8_splits(K)): W is the gate|up matrix with rows glu-interleaved
 * (zsaac/mistral.py glu_interleave) and act[m][f] = silu(gate_f) * up_f is written directly as
 * bf16 [M][ld_act] (N / 2 columns; out unused) -- MistralMLP's act_fn(gate_proj(x)) * up_proj(x)
 * (transformers MistralMLP, called from caption_model.py:355-364's generate). */
int zs_fp8_gemm_run(const void* A, int lda, const void* W8, const float* scale, int M, int N,
                    int K, int ks, int kh, float* out, long split_stride, int ldo, void* act,
                    int ld_act, const float* rss, int nch, float eps, void* stream);

/* zs_mistral_add_ss: the decode form of zs_mistral_add_rmsnorm when the next GEMM applies the
 * norm (zs_fp8_gemm_run with rss; MistralRMSNorm's weight folded into that GEMM): x[m] +=
 * sum_s y[s][m] (y may be NULL), xb[m] = bf16(x[m]) and rss[c][m] (row stride 32) = sum of x^2 over
 * columns 512 c .. 512 c + 511; M <= 32, D % 512 == 0.  zs_fp8_gemm_run(..., rss, D / 512 <= 8, eps)
 * then scales output row m by rsqrt(sum_c rss[c][m] / K + eps). */
int zs_mistral_add_ss(float* x, const float* y, int nsplit, long ss, int M, int D, void* xb,
                      float* rss, void* stream);

/* zs_mistral_embed: prefill rows b*P + i (P = H + ns + nt): embed[hard[b][i]] (i < H, pads
 * included as the reference attends them), soft[b][i-H] (ns rows, f32), embed[tail[i-H-ns]]
 * (the language tag); or, with tok != NULL, decode rows embed[tok[m]].  x f32 [M][D]. */
int zs_mistral_embed(const int* hard, int H, const float* soft, int ns, const int* tail, int nt,
                     const int* tok, const void* emb, int D, int M, float* x, int dtype,
                     void* stream);

/* zs_mistral_add_rmsnorm: x[m] += sum_s y[s][m] (y may be NULL), h[m] = w * (x[m] *
 * rsqrt(mean(x[m]^2) + eps)) (MistralRMSNorm; w NULL = folded into the next GEMM). */
int zs_mistral_add_rmsnorm(float* x, const float* y, int nsplit, long ss, int M, int D, float eps,
                           const float* w, void* h, int hdtype, void* stream);

/* zs_mistral_rope_kv: q|k|v slabs [nsplit][M][(H + 2 KVH) * 128] -> rotary-embedded q [M][H*128]
 * and k, plus v, appended to the caches [seq][KVH][Lmax][128] at position pos[m] (seq =
 * m / rows_per_seq); cos / sin [Lmax][64] f32 tables (HF rotary, rotate_half). */
int zs_mistral_rope_kv(const float* qkv, int nsplit, long ss, int M, int H, int KVH,
                       const int* pos, int rows_per_seq, const float* cosb, const float* sinb,
                       void* q, void* kc, void* vc, int Lmax, int dtype, void* stream);

/* zs_fp8_unpack_bf16: the tile-packed fp8 codes of W [N][K] (see zs_fp8_gemm_rows) -> row-major
 * bf16 W-codes [N][K] (exact; the per-channel scale is not applied).  zs_scale_cols:
 * x[m][n] *= scale[n] for an f32 [M][ld] matrix.  Together with zs_gemm they run a prefill's
 * M > 64 rows as one tiled MFMA GEMM (weights read once, not once per 64 rows). */
int zs_fp8_unpack_bf16(const void* W8, int N, int K, void* out, void* stream);
int zs_scale_cols(float* x, int M, int N, int ld, const float* scale, void* stream);

/* zs_mistral_silu_mul: act[m][f] = silu(gate) * up from gate|up slabs [nsplit][M][2F] whose
 * columns are glu-interleaved: gate f at 16 (f / 8) + 8 (f / 4 % 2) + f % 4, up f at that + 4. */
int zs_mistral_silu_mul(const float* gu, int nsplit, long ss, int M, int F, void* act, int dtype,
                        void* stream);

/* zs_mistral_attention: causal GQA attention, query row m against keys 0..pos[m] of sequence
 * m / rows_per_seq, kv head h / (H / KVH), softmax((q k^T) / sqrt(128)) v -> out [M][H*128]. */
int zs_mistral_attention(const void* q, int M, int H, int KVH, const int* pos, int rows_per_seq,
                         const void* kc, const void* vc, int Lmax, void* out, int dtype,
                         void* stream);

/* zs_mistral_decode_attention: one decode step (row m = sequence m, new position pos[m]):
 * zs_mistral_rope_kv + zs_mistral_attention (rows_per_seq 1) in one launch -- q / k / v summed
 * from the slabs and rotated in registers, k / v row pos[m] appended to the caches, keys
 * 0..pos[m]-1 read from them and key pos[m] from registers. */
int zs_mistral_decode_attention(const float* qkv, int nsplit, long ss, int M, int H, int KVH,
                                const int* pos, const float* cosb, const float* sinb, void* kc,
                                void* vc, int Lmax, void* out, int dtype, void* stream);

/* ------------------------------------------------------------------ GPT-2 decode
 * zs_gpt2_prefill_embed: clap_to_gpt (caption_model.py:315-329) + the caller's wte lookup
 * (predict_prompt.py:133) + GPT-2 input embedding:  row b, position p < P_b = hard_len[b]+n_soft:
 *   e = p < H_b ? wte[hard_ids[b][p]] : soft[b][p-H_b]   (prefix_embed, written to `embed`)
 *   x = e + wpe[p]                                         (transformer input, written to `x`)
 * rows padded to Pmax with zeros.  plen[b] = P_b, last_row[b] = b*Pmax + P_b - 1.  wte/wpe in
 * dtype, soft f32 with clip b's n_soft*D prefix at soft + b*soft_ld. */
int zs_gpt2_prefill_embed(const int* hard_ids, const int* hard_len, int h_cap, const float* soft,
                          int soft_ld, int n_soft, const void* wte, const void* wpe, int B,
                          int Pmax, int D, float* embed, float* x, int* plen, int* last_row,
                          int dtype, void* stream);

/* zs_kv_write: copy k,v of `n` tokens per row from qkv [R*n][3D] into the cache
 * kc/vc [rows][heads][Lmax][hd] at cache row r*row_stride, positions pos0[r] + i (pos0 NULL -> 0).
 * row_stride = beam puts a clip's beam-search prompt in its first beam row. */
int zs_kv_write(const void* qkv, int R, int n, int D, int heads, const int* pos0, int row_stride,
                void* kc, void* vc, int Lmax, int dtype, void* stream);

/* zs_decode_attention: one new token per row r at position pos[r]: append its k,v (from
 * qkv[r]) to the cache, attend over positions 0..pos[r] (kv row for position j of row r is
 * kvrow[r*Lmax + j] when kvrow != NULL, else r — the beam-search history indirection),
 * scale 1/sqrt(hd), f32 softmax.  out [R][D] (dtype).  HF GPT2Attention eager semantics. */
int zs_decode_attention(const void* qkv, int R, int D, int heads, void* kc, void* vc, int Lmax,
                        const int* pos, const int* kvrow, void* out, int dtype, void* stream);

/* zs_decode_attention_map: zs_decode_attention over a compacted row set (bf16, no kvrow):
 * qkv/out rows are compact slots c in [0, R); the physical decode row of slot c is rowmap[c]
 * (the cache is indexed physically).  The position of slot c is cpos[c] when cpos != NULL (as
 * written by zs_embed_tokens_map), else pos[rowmap[c]].  rowmap[c] >= nphys marks a padding
 * slot: its out row is zeroed and the cache is untouched. */
int zs_decode_attention_map(const void* qkv, int R, const int* rowmap, int nphys, int D, int heads,
                            void* kc, void* vc, int Lmax, const int* pos, const int* cpos,
                            void* out, int dtype, void* stream);

/* zs_embed_tokens: x[r] = wte[tok[r]] + wpe[pos[r]] (f32 out), optional row gather. */
int zs_embed_tokens(const int* tok, const int* pos, const void* wte, const void* wpe, int R, int D,
                    float* x, int dtype, void* stream);

/* zs_embed_tokens_map: x[c] = wte[tok[rowmap[c]]] + wpe[pos[rowmap[c]]] for compact slots
 * c in [0, R); padding slots (rowmap[c] >= nphys) get x[c] = 0.  cpos (optional, [R]) receives
 * pos[rowmap[c]] (0 for padding) for zs_decode_attention_map. */
int zs_embed_tokens_map(const int* tok, const int* pos, const int* rowmap, int nphys,
                        const void* wte, const void* wpe, int R, int D, float* x, int* cpos,
                        int dtype, void* stream);

/* zs_compact_rows: stable compaction of the rows still decoding.  rowmap[0..n) = the r with
 * done[r] == 0 in increasing order, rowmap[n..nrows) = nrows (padding), *n_active = n.
 * Lets a greedy decode skip the rows that already emitted a stop token (the reference keeps
 * computing them, gpt2_prefix_eval.py:200-215; their outputs are discarded either way). */
int zs_compact_rows(const int* done, int nrows, int* rowmap, int* n_active, void* stream);

/* zs_lmhead_topk: per row m of A [M][K] (dtype) against W [V][K] (dtype; tied wte):
 *   logits = A W^T, split in column blocks of 128; per (row, block) writes the block's max,
 *   sum(exp(logit - max)) and its top-`topk` (value, index) (ties -> lower index).
 *   part_stat [M][nblk][2] f32, part_val [M][nblk][topk] f32, part_idx [M][nblk][topk] int32,
 *   nblk = ceil(V/128).  topk <= 8.  part_stat may be NULL (argmax callers: greedy generate2,
 *   get_prefix_tokens): the max / sum-exp pass is then skipped.  With row_norm != 0 each A row
 *   is L2-normalised first
 *   (get_prefix_tokens, gpt2_prefix_eval.py:271-278: W must then be normalize(wte)). */
int zs_lmhead_topk(int M, int K, int V, int dtype, const void* A, int lda, const void* W,
                   int topk, int row_norm, float* part_stat, float* part_val, int* part_idx,
                   void* stream);
/* zs_lmhead_topk_t: zs_lmhead_topk on logits / temperature (temperature > 0; row_norm needs 1):
 * generate2 / generate_beam's `temperature` (gpt2_prefix_eval.py:121, 196). */
int zs_lmhead_topk_t(int M, int K, int V, int dtype, const void* A, int lda, const void* W,
                     int topk, int row_norm, float temperature, float* part_stat, float* part_val,
                     int* part_idx, void* stream);
int zs_lmhead_nblk(int V);

/* zs_argmax_finalize: merge zs_lmhead_topk partials (topk 1) into idx[M] (lower index on ties). */
int zs_argmax_finalize(const float* part_val, const int* part_idx, int M, int nblk, int* idx,
                       void* stream);

/* zs_prefix_ids_assemble: get_prefix_tokens (gpt2_prefix_eval.py:271-278) with the argmax run
 * only over the soft-prompt rows: out[b][p] = hard_ids[b][p] for p < hard_len[b] (a hard row is
 * wte[id] and its own cosine is the maximum — the caller verifies that every possible hard id
 * beats every other vocabulary row by a margin before taking this path), soft_idx[b][p - H_b]
 * for the n_soft rows after it, 0 for padding rows (zero embeddings: all cosines 0).
 * hard_ids [B][h_cap], soft_idx [B][n_soft], out [B][Pmax] int32. */
int zs_prefix_ids_assemble(const int* hard_ids, int h_cap, const int* hard_len, const int* soft_idx,
                           int n_soft, int B, int Pmax, int* out, void* stream);

/* zs_greedy_step: generate2's per-step bookkeeping (gpt2_prefix_eval.py:208-215) for R rows:
 * tok = argmax(partials); rows already done keep emitting nothing; out_ids[r][step] = tok,
 * out_len[r] = step+1 while not done; done |= tok in {stop0, stop1}; pos[r] += 1 (next position);
 * next_tok[r] = tok.  `step` is read from *step_ctr (device) and *step_ctr += 1 by the last
 * block, so a captured graph replays without host arguments.  all_done[0] = AND(done);
 * all_done[1] is the blocks' arrival counter: zero it once before the first call (every call
 * re-arms it); all_done[2] = the number of rows not done after this step. */
int zs_greedy_step(const float* part_val, const int* part_idx, int R, int nblk, int* step_ctr,
                   int max_steps, int stop0, int stop1, int* out_ids, int* out_len, int* done,
                   int* pos, int* next_tok, int* all_done, void* stream);

/* zs_greedy_init: generate2's state before step 0 (gpt2_prefix_eval.py:186-196) for R rows:
 * pos[r] = plen[r] - 1 (the last prompt position), done = out_len = 0, out_ids[r][0..max_steps)
 * = 0, *step_ctr = 0, all_done[0..2] = 0 -- what zs_greedy_step expects before its first call. */
int zs_greedy_init(int R, const int* plen, int* pos, int* done, int* out_len, int* out_ids,
                   int max_steps, int* step_ctr, int* all_done, void* stream);

/* zs_greedy_step_map: zs_greedy_step where partial row c belongs to physical row rowmap[c]
 * (out_ids, out_len, done, pos, next_tok are physical); padding slots are skipped. */
int zs_greedy_step_map(const float* part_val, const int* part_idx, int R, const int* rowmap,
                       int nphys, int nblk, int* step_ctr, int max_steps, int stop0, int stop1,
                       int* out_ids, int* out_len, int* done, int* pos, int* next_tok,
                       int* all_done, void* stream);

/* zs_gpt2_decode_persist: every remaining step of generate2 (gpt2_prefix_eval.py:161-222: the
 * 67-step loop of model.gpt(inputs_embeds=...) -> argmax -> stop check) for ONE batch of R <= 64
 * rows (the reference's eval batch), bf16, as one persistent launch of `grid` (48, 96 or 192)
 * 256-thread workgroups (half a CU each; the caller keeps the concurrent launches' grids
 * co-resident): per step the 12 GPT2Blocks (ln_1 affine folded into c_attn and ln_2's into c_fc),
 * ln_f, the tied LM head with its argmax (ties -> lower id) and zs_greedy_step's bookkeeping,
 * until every row stopped or max_steps.  Starts from the state zs_greedy_step left after step 0
 * (next_tok, pos, done, out_ids, out_len, *step_ctr, all_done[0]) and commits that state after
 * every step.  layer_w: 12 x 8 device pointers {c_attn W, its bias, attn.c_proj W, bias, c_fc W,
 * its bias, mlp.c_proj W, bias}, each W (= Conv1D weight transposed, [N][K] bf16; c_attn's with
 * ln_1's weight folded in, c_fc's with ln_2's) in MFMA fragment order [N/16][K/32][64][8] (block j,
 * k-step s, lane l = W[16 j + l % 16][32 s + 8 (l / 16) .. + 8]); the c_attn and c_fc biases are f32
 * [2][N]: row 0 the bias with the LayerNorm's beta folded in (b + beta W), row 1 the folded
 * weight's column sums cs[n] = sum_k W'[n][k] -- the LayerNorm runs in the GEMM epilogue as
 * rstd (x W' - mean cs) + b'; the projections' biases are f32 [N].  wte_packed: the tied LM head
 * with ln_f's weight folded in, bf16(g o wte[v]), in the same order, [ceil(V/16)][24][64][8] (rows
 * past V zero); lm_bias f32 [2][ceil(V/16) 16]: beta . wte[v] (ln_f's bias through the head), then
 * the column sums of the folded head; logit[v] = LN(x) . (g o wte[v]) + lm_bias[0][v];
 * temperature > 0 divides the logits before the argmax (gpt2_prefix_eval.py:196);
 * kv: 24 pointers {kc[0..11], vc[0..11]}, each [R][12][Lmax][64] bf16 (zs_kv_write layout),
 * 128-byte aligned.  ws: scratch of zs_decode_persist_workspace_bytes() bytes, 256-byte aligned,
 * private to one launch in flight.  exclusive != 0: each workgroup also requests LDS past half a
 * CU, so no two exclusive workgroups share a CU (the dispatcher otherwise doubles workgroups up
 * while CUs idle); the caller keeps the exclusive workgroups in flight <= the CU count.  Every
 * output element is computed by the same operations
 * whatever `grid` (each GEMM element: four K-quarter MFMA chains summed (p0 + p1) + (p2 + p3);
 * LayerNorm statistics (one pass, sum x and sum x^2), attention and argmax in fixed orders), so ids and state do not depend on the grid
 * and equal zs_gpt2_decode_phases'.  A grid that cannot become co-resident gives up after a
 * bounded wait: all_done[1] = -1, zs_decode_persist_status reports timed_out != 0, and the state
 * in memory is the last committed step's (resume with zs_gpt2_decode_phases). */
int zs_decode_persist_workspace_bytes(void);
int zs_gpt2_decode_persist(int R, int Lmax, int max_steps, int stop0, int stop1, int V,
                           const void* wte, const void* wpe, const void* wte_packed,
                           float temperature, const void* const* layer_w,
                           const float* lm_bias, void* const* kv, int* pos,
                           int* next_tok, int* done, int* out_ids, int* out_len, int* step_ctr,
                           int* all_done, void* ws, long ws_bytes, int grid, int exclusive,
                           void* stream);
/* zs_gpt2_decode_phases: `steps` decode steps of the same computation as separate launches (one
 * per phase of every block, the LM head and the bookkeeping: 62 per step; each a no-op once
 * all_done[0] is set, so a graph-captured chunk can run past the end) -- the per-step path of
 * zs_gpt2_decode_persist (no co-residency needed; the give-up fallback), bit-identical to it. */
int zs_gpt2_decode_phases(int R, int Lmax, int max_steps, int stop0, int stop1, int V,
                          const void* wte, const void* wpe, const void* wte_packed,
                          float temperature, const void* const* layer_w,
                          const float* lm_bias, void* const* kv, int* pos,
                          int* next_tok, int* done, int* out_ids, int* out_len, int* step_ctr,
                          int* all_done, void* ws, long ws_bytes, int steps, int grid,
                          void* stream);
/* zs_gpt2_decode_persist_f32 / zs_gpt2_decode_phases_f32: the same decode in f32 (the parity
 * mode; replaces the same generate2 loop, gpt2_prefix_eval.py:161-222, in fp32): wte / wpe f32
 * [V][768] / [1024][768]; layer_w 12 x 8 pointers in the same order, each W f32 in 16-k fragment
 * order [N/16][K/16][64][4] (block j, k-step s, lane l = W[16 j + l % 16][16 s + 4 (l / 16) .. + 4]),
 * c_attn's / c_fc's with the LayerNorm's weight folded in (W diag(g), f32) and biases f32 [N]
 * (b + W beta); wte_packed f32 g o wte[v] (ln_f's weight) in that order [ceil(V/16)][48][64][4];
 * lm_bias f32 [ceil(V/16) 16] (beta . wte[v]); kv f32 [R][12][Lmax][64]; ws of
 * zs_decode_persist_f32_workspace_bytes().  The LayerNorms are two-pass (mean, then squared
 * deviations) and normalise rows in registers before exact-f32 MFMAs (v_mfma_f32_16x16x4_f32);
 * grid 192 only.  The persistent and phase forms give identical ids, as the bf16 pair. */
int zs_decode_persist_f32_workspace_bytes(void);
int zs_gpt2_decode_persist_f32(int R, int Lmax, int max_steps, int stop0, int stop1, int V,
                               const void* wte, const void* wpe, const void* wte_packed,
                               float temperature, const void* const* layer_w,
                               const float* lm_bias, void* const* kv, int* pos,
                               int* next_tok, int* done, int* out_ids, int* out_len, int* step_ctr,
                               int* all_done, void* ws, long ws_bytes, int grid, int exclusive,
                               void* stream);
int zs_gpt2_decode_phases_f32(int R, int Lmax, int max_steps, int stop0, int stop1, int V,
                              const void* wte, const void* wpe, const void* wte_packed,
                              float temperature, const void* const* layer_w,
                              const float* lm_bias, void* const* kv, int* pos,
                              int* next_tok, int* done, int* out_ids, int* out_len, int* step_ctr,
                              int* all_done, void* ws, long ws_bytes, int steps, int grid,
                              void* stream);
int zs_decode_persist_status(const void* ws, int* timed_out);
/* zs_decode_persist_set_stamps: diagnostic phase timing (tools/persist_stamps.py): with buf !=
 * NULL ([grid][128] u64), thread 0 of every workgroup of later launches writes s_memrealtime
 * (100 MHz) at each barrier arrive (slot 2i) / wait end (2i + 1) of decode step `step`, and at
 * that step's start (127) / end (126); ws != NULL: only the launches on that workspace (one of
 * several concurrent grids).  buf NULL turns it off. */
int zs_decode_persist_set_stamps(void* buf, int step, const void* ws);

/* zs_beam_step: generate_beam's per-step update (gpt2_prefix_eval.py:119-151) for C clips x
 * `beam` rows, from zs_lmhead_topk partials (topk >= beam) with log(softmax) semantics.
 * first != 0: step 0 (row c*beam of each clip is the only live source).  Updates scores,
 * seq_len, stopped, the token history tokens [R][max_steps], the kv-row indirection table
 * kvrow [R][Lmax] (history of the chosen source row + this step's own slot), pos[R],
 * next_tok[R]; all_done[0] = every row stopped. */
int zs_beam_step(const float* part_stat, const float* part_val, const int* part_idx, int C,
                 int beam, int nblk, int topk, int first, int stop, int* step_ctr, int max_steps,
                 float* scores, float* seq_len, int* stopped, int* tokens, int* tokens_tmp,
                 int* kvrow, int* kvrow_tmp, int Lmax, int* pos, int* next_tok, int* all_done,
                 void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ZSAAC_H */

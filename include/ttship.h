/*
 * ttship — MI355X-native Tacotron2-DDC + MultiBand-MelGAN inference path, C ABI.
 *
 * Drop-in boundary. The reference has no FFI/plugin registry: its boundary is
 * nn.Module duck typing. Each entry point below replaces one reference call, cited as
 * path:line relative to the reference checkout:
 *
 *   tts_taco_set_tensor/finalize  <- Tacotron2.load_state_dict(cp['model'])
 *                                    (TTS/server/synthesizer.py:68-79, TTS/tts/utils/io.py:9-24)
 *   tts_taco_infer                <- Tacotron2.inference(text)  (TTS/tts/models/tacotron2.py:142-163)
 *   tts_taco_infer_spk            <- Tacotron2.inference(text, speaker_ids | speaker_embeddings)
 *                                    with decoder.set_r / max_decoder_steps (layers/tacotron2.py:209,156)
 *   tts_taco_encoder              <- embedding + Encoder.inference (models/tacotron2.py:144-145,
 *                                    layers/tacotron2.py:112-119)
 *   tts_taco_postnet              <- Postnet + residual (models/tacotron2.py:159-160)
 *   tts_taco_decoder_state        <- the decoder state the reference leaves on `self` after inference
 *                                    (query, attention_rnn_cell_state, decoder_hidden, decoder_cell,
 *                                    context, attention_weights(_cum): layers/tacotron2.py:217-233,
 *                                    259-298; common_layers.py:251-260): per-stage decoder parity
 *   tts_melgan_set_tensor/finalize<- MultibandMelganGenerator.load_state_dict + remove_weight_norm
 *                                    (TTS/server/synthesizer.py:81-91, melgan_generator.py:91-97)
 *   tts_melgan_infer              <- MultibandMelganGenerator.inference (multiband_melgan_generator.py:32-39)
 *   tts_melgan_infer_strided      <- the same on a (B, M, C) tensor viewed as (B, C, M) (no transposed copy)
 *   tts_melgan_generator          <- MelganGenerator.layers(c) (melgan_generator.py:28-81)
 *   tts_pqmf_synthesis            <- PQMF.synthesis (TTS/vocoder/layers/pqmf.py:51-56)
 *   tts_taco_mbmelgan_infer       <- Tacotron2.inference then MultibandMelganGenerator.inference on its
 *                                    postnet output (TTS/server/synthesizer.py:150-159), one call
 *   tts_taco_mbmelgan_submit/finish <- the same, returning once the decode's results are on the host
 *                                    (the vocoder still running), completed by finish
 *
 * Conventions: every function returns 0 on success and nonzero on failure; the message is
 * available from tts_last_error() (thread-local). Pointers prefixed d_ are device (HIP) memory
 * owned by the caller; h_ are host memory. `stream` is a hipStream_t (NULL = default stream);
 * work is ordered after prior work on `stream` and later work on `stream` is ordered after it.
 * Tensors are fp32, C-contiguous, in the layouts documented per function.
 *
 * Threads: a context may be shared by host threads. Every entry point that takes a context holds
 * that context's (recursive) mutex for the whole call, so calls on one context run one at a time;
 * sequences that must not interleave (load a model then infer with it, glow_encode then
 * glow_decode) need a caller-side lock around them (the Python layer's Engine.lock). Different
 * contexts (one per device) run concurrently. The reference model is not re-entrant at all
 * (per-call state on self: TTS/tts/layers/tacotron2.py:221-233).
 *
 * Host synchronisation: tts_taco_infer(_spk) returns per-utterance step counts and so waits for
 * its work. In the default split-f16 GEMM mode every other compute entry (postnet, melgan,
 * pwgan, glow) also ends with one hipStreamSynchronize on its stream, to read the range flag and
 * re-run the call on the fp32 kernels if an operand left the f16 range (a NaN input counts as out
 * of range and runs the call twice). With tts_set_gemm_mode(ctx, 0) those entries stay
 * stream-asynchronous. INTEGRATION.md §3.
 *
 * Device use: the persistent kernels need every one of their workgroups resident at once (one per
 * CU); another process or stream keeping kernels on the same GPU during a call can delay them
 * past the barrier wait limit below, and the call then fails (retryable).
 *
 * Grid barriers: the persistent decoder / BiLSTM / GE2E kernels give up a barrier wait after
 * TTS_BARRIER_TIMEOUT_MS (environment, default 2000) and the call returns an error; nothing is
 * left half-written that a retry depends on, so retrying the call is safe.
 */
#ifndef TTSHIP_H
#define TTSHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tts_ctx tts_ctx;

int tts_version(void);
const char* tts_last_error(void);

/* One context per (process, device). Owns packed weights, workspace and captured graphs. */
int tts_ctx_create(int device, tts_ctx** out);
int tts_ctx_destroy(tts_ctx* ctx);

/* ---- Tacotron2 (DDC LJSpeech architecture; coarse_decoder.* accepted and ignored) ---- */
/* Register one state_dict tensor by its reference key, fp32 host data. */
int tts_taco_set_tensor(tts_ctx* ctx, const char* name, const float* h_data, const int64_t* shape, int ndim);
/* Fold BatchNorm, permute/swizzle and upload. attn_norm: 0 = sigmoid, 1 = softmax.
   r_init = reduction factor the model was constructed with (projection width 80*r_init). */
int tts_taco_finalize(tts_ctx* ctx, int num_chars, int r_init, int attn_norm);

/* Batched Tacotron2.inference. Output i equals the reference B=1 call on utterance i.
   d_ids      (B, T_max) int64 token ids; row b valid for t < h_lens[b] (1 <= h_lens[b] <= T_max)
   r          reduction factor in use (1 <= r <= r_init)
   h_max_steps per-utterance max_decoder_steps (>= 1); S_cap >= max(h_max_steps)
   d_dec, d_post (B, S_cap*r, 80): frames [0, steps_b*r) valid, rest zero
   d_align    (B, S_cap, T_max);  d_stop (B, S_cap) sigmoid(stop logit)
   h_steps    out: decoder steps taken per utterance; h_status out: 1 stopnet, 2 max steps */
int tts_taco_infer(tts_ctx* ctx, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, int r,
                   const int32_t* h_max_steps, int S_cap, float stop_threshold, float* d_dec, float* d_post,
                   float* d_align, float* d_stop, int32_t* h_steps, int32_t* h_status, void* stream);

/* Multi-speaker Tacotron2.inference(text, speaker_ids=..., speaker_embeddings=...)
   (TTS/tts/models/tacotron2.py:142-156; speaker vector concatenated to the encoder outputs,
   tacotron_abstract.py:213-217). Exactly one of d_spk_ids (int64 (B), rows of the learned
   speaker_embedding table) or d_spk_emb (float (B, spk_dim), external per-sample embeddings) is
   non-null. At most 64 utterances per call, speaker vectors of at most 512 dims. Other arguments
   as tts_taco_infer. */
int tts_taco_infer_spk(tts_ctx* ctx, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, int r,
                       const int32_t* h_max_steps, int S_cap, float stop_threshold, const int64_t* d_spk_ids,
                       const float* d_spk_emb, float* d_dec, float* d_post, float* d_align, float* d_stop,
                       int32_t* h_steps, int32_t* h_status, void* stream);

/* Decoder options that no tensor reveals (layers/tacotron2.py:147-200 -> common_layers.py:196-372):
   attention windowing at inference (attn_win) and forward attention (forward_attn; the transition
   agent is on when decoder.attention.ta.* tensors are loaded). BN prenet is detected from the
   decoder.prenet.linear_layers.N.batch_normalization.* tensors. Variants decode on the persistent
   decoder only. forward_attn_mask keeps the forward alignment to [n-1, n+2] around the shifted
   previous argmax n (common_layers.py:309-318). Set before tts_taco_infer; kept across finalize. */
int tts_taco_set_options(tts_ctx* ctx, int windowing, int forward_attn, int forward_attn_mask);

/* speaker dimension of the finalized model (0 = single speaker) and its learned table size */
int tts_taco_speaker_dim(tts_ctx* ctx, int* spk_dim, int* num_speakers);

/* encoder outputs (B, T_max, 512), zero for t >= h_lens[b] */
int tts_taco_encoder(tts_ctx* ctx, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max,
                     float* d_out, void* stream);

/* postnet(dec) + dec on time-major (B, M_max, 80) frames, valid for t < h_lens[b] */
int tts_taco_postnet(tts_ctx* ctx, const float* d_dec, const int32_t* h_lens, int B, int M_max, float* d_out,
                     void* stream);

/* Decoder state after the last decoder step of the previous tts_taco_infer* call on this context
   (persistent decoder path), rows in the caller's order: attention_rnn h and c (B, 1024),
   decoder_rnn h and c (B, 1024), context (B, 512), attention weights and cumulative weights
   (B, T_max). Rows that stopped before the call's last step hold the state the batched decode left
   in them, not their own final state: compare rows that ran the call's full step count. Any output
   pointer may be NULL (skipped). B and T_max size the caller's buffers and must equal the last
   decode's batch and encoder length (an error otherwise, nothing written). In split-f16 mode
   (tts_set_gemm_mode 1) the persistent decoder publishes attention_rnn h, decoder_rnn h and the
   context pre-split as f16 hi / lo halves; those three outputs are rebuilt as hi + 2^-11 lo, the
   value the next step's GEMMs consume (about 22 significant bits, within ~2^-22 relative of the
   fp32 value), not the unrounded fp32 state. The cell states and attention weights are fp32. */
int tts_taco_decoder_state(tts_ctx* ctx, int B, int T_max, float* d_att_h, float* d_att_c, float* d_dec_h,
                           float* d_dec_c, float* d_context, float* d_alpha, float* d_alpha_cum, void* stream);

/* ---- MultiBand-MelGAN generator ---- */
int tts_melgan_set_tensor(tts_ctx* ctx, const char* name, const float* h_data, const int64_t* shape, int ndim);
/* upsample_factors: n_up entries (even), base_channels, num_res_blocks, out_channels (4 with PQMF) */
int tts_melgan_finalize(tts_ctx* ctx, int in_channels, int out_channels, int base_channels,
                        const int32_t* upsample_factors, int n_up, int num_res_blocks, int use_pqmf);

/* d_mel (B, in_channels, M_max) channel-major, utterance b valid for m < h_lens[b];
   pad = inference_padding (replicate). Requires h_lens[b] + 2*pad >= 4 (ReflectionPad1d(3)).
   d_wav (B, 1, hop*(M_max + 2*pad)), hop = prod(upsample_factors) * (out_channels if PQMF else 1);
   samples past hop*(h_lens[b] + 2*pad) are zero. */
int tts_melgan_infer(tts_ctx* ctx, const float* d_mel, const int32_t* h_lens, int B, int M_max, int pad,
                     float* d_wav, void* stream);
/* the same with d_mel given by element strides (batch, channel, frame), e.g. a Tacotron2 postnet
   output (B, M, in_channels) read in place as (B, in_channels, M): strides (M*in_channels, 1,
   in_channels), no transposed copy. Channel stride 1 needs a frame stride divisible by 4 and a
   16-byte aligned d_mel. */
int tts_melgan_infer_strided(tts_ctx* ctx, const float* d_mel, int64_t stride_b, int64_t stride_c, int64_t stride_t,
                             const int32_t* h_lens, int B, int M_max, int pad, float* d_wav, void* stream);

/* generator layers only: d_out (B, out_channels, up*(M_max + 2*pad)), up = prod(upsample_factors) */
int tts_melgan_generator(tts_ctx* ctx, const float* d_mel, const int32_t* h_lens, int B, int M_max, int pad,
                         float* d_out, void* stream);

/* PQMF synthesis on (B, N, L) subbands with filter d_G (N, taps+1) -> d_y (B, 1, N*L) */
int tts_pqmf_synthesis(tts_ctx* ctx, const float* d_x, int B, int N, int L, const float* d_G, int taps,
                       float* d_y, void* stream);

/* ---- ParallelWaveGAN generator (TTS/vocoder/models/parallel_wavegan_generator.py) ----
   tts_pwgan_set_tensor/finalize <- ParallelWaveganGenerator(...) as setup_generator builds it
                       (vocoder/utils/generic_utils.py:79-92: 64 res / 128 gate / 64 skip / 80 aux
                       channels, kernel 3) + load_state_dict (weight_g / weight_v or folded weight)
   tts_pwgan_infer  <- ParallelWaveganGenerator.inference (:120-125): replicate pad `pad`, ConvUpsample,
                       first_conv on d_noise (B, 1, hop*(M_max + 2*pad)) standard normal, residual
                       blocks, output convs -> d_out (B, 1, hop*(M_max + 2*pad)); row b is zero past
                       hop*(h_lens[b] + 2*pad) */
int tts_pwgan_set_tensor(tts_ctx* ctx, const char* name, const float* host, const int64_t* shape, int ndim);
int tts_pwgan_finalize(tts_ctx* ctx, int num_res_blocks, int stacks, const int32_t* upsample_factors, int n_up);
int tts_pwgan_infer(tts_ctx* ctx, const float* d_mel, const int32_t* h_lens, int B, int M_max, int pad,
                    const float* d_noise, float* d_out, void* stream);

/* ---- Glow-TTS (TTS/tts/models/glow_tts.py, reference configs: gated-conv encoder) ----
   tts_glow_set_tensor/finalize <- GlowTts(...).load_state_dict (enc_layers = 3 + num_layers_enc)
   tts_glow_encode  <- GlowTts.inference up to the durations (glow_tts.py:166-176): encoder,
                       duration predictor, w_ceil; h_ylens out: y_lengths per utterance
   tts_glow_decode  <- the rest (:177-193) for Ty = max(h_ylens): generate_path, expanded means,
                       z = y_mean + d_noise * noise_scale (d_noise (B, 80, Ty) standard normal),
                       reverse flows; d_y (B, 80, 2*floor(Ty/2)), d_ymean (B, 80, Ty),
                       d_attn (B, Ty, T_max), d_logw (B, T_max) = o_dur_log */
int tts_glow_set_tensor(tts_ctx* ctx, const char* name, const float* host, const int64_t* shape, int ndim);
int tts_glow_finalize(tts_ctx* ctx, int num_chars, int enc_layers, int num_flow_blocks, int num_block_layers);
int tts_glow_encode(tts_ctx* ctx, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max,
                    float length_scale, int32_t* h_ylens, void* stream);
/* tts_glow_encode_spk <- GlowTts.inference(x, x_lengths, g) (glow_tts.py:159-176) for a
   multi-speaker model (num_speakers > 1, c_in_channels > 0): h_speaker_ids (B) index emb_g;
   g = F.normalize(emb_g(ids)) joins the duration predictor input (encoder.py:131-135) and, through
   each coupling block's cond_layer, the WN gates of the following tts_glow_decode (glow.py:119-130).
   h_speaker_ids = NULL is tts_glow_encode. Errors as the reference fails: ids given to a model
   without emb_g or cond_layer, no ids for a model with c_in_channels > 0, an id out of range. */
int tts_glow_encode_spk(tts_ctx* ctx, const int64_t* d_ids, const int32_t* h_lens, const int32_t* h_speaker_ids,
                        int B, int T_max, float length_scale, int32_t* h_ylens, void* stream);
int tts_glow_decode(tts_ctx* ctx, const float* d_noise, float noise_scale, int Ty, float* d_y, float* d_ymean,
                    float* d_attn, float* d_logw, void* stream);

/* ---- GE2E speaker encoder (TTS/speaker_encoder/model.py) ----
   tts_ge2e_set_tensor/finalize <- SpeakerEncoder(input_dim, proj_dim, lstm_dim, num_lstm_layers,
                                   use_lstm_with_projection).load_state_dict  (model.py:31-47)
   tts_ge2e_infer               <- SpeakerEncoder.inference(x) (model.py:62-68) on B sequences of
                                   per-sequence length h_lens[b]: d_x (B, T_max, input_dim) fp32,
                                   d_out (B, proj_dim) L2-normalised embeddings. lstm_dim must be 768. */
int tts_ge2e_set_tensor(tts_ctx* ctx, const char* name, const float* host, const int64_t* shape, int ndim);
int tts_ge2e_finalize(tts_ctx* ctx, int input_dim, int proj_dim, int lstm_dim, int num_lstm_layers,
                      int use_lstm_with_projection);
int tts_ge2e_infer(tts_ctx* ctx, const float* d_x, const int32_t* h_lens, int B, int T_max, float* d_out,
                   void* stream);

/* Measurement hook for bench.py: average device time (ms) of `iters` launches of one kernel of the
   last tts_taco_infer configuration, timed with hipEvents on the context's stream.
   which: 0 = decoder LSTM GEMM step kernel (K4), 1 = full decoder step (all 7 kernels). */
int tts_time_decoder_kernel(tts_ctx* ctx, int which, int iters, float* ms_out);

/* Decoder launches of the last tts_taco_infer: path 1 = persistent kernel (one launch per
   batch-tile count, 64 / 48 / 32 / 16 rows, nlaunch <= 4: ms and steps must hold 4 entries;
   ms[i] = hipEvent time of launch i, steps[i] = decoder steps it completed), path 0 = step
   graphs (nlaunch = 0). */
int tts_decoder_stats(tts_ctx* ctx, int* path, int* nlaunch, float* ms, int* steps);

/* GEMM arithmetic of the context's kernels. mode 1 (default) = split-f16 MFMA where a kernel has
   it: every fp32 operand as hi + 2^-11 lo f16 halves, three f16 MFMAs per product accumulated in
   fp32, error equal to the fp32 MFMA GEMM's; a call whose operands leave the f16
   range (|v| >= 65504) is re-run on the fp32 kernels. mode 0 = fp32 MFMA everywhere. The
   environment variable TTS_GEMM=f32 starts contexts in mode 0. tts_gemm_mode reports the mode and
   how many calls fell back to fp32. */
int tts_set_gemm_mode(tts_ctx* ctx, int mode);
int tts_gemm_mode(tts_ctx* ctx, int* mode, int64_t* fallbacks);

/* Tacotron2.inference then MultibandMelganGenerator.inference on its postnet output in ONE call
   (TTS/server/synthesizer.py:150-159 runs the two back to back, the mel lengths passing through
   Python): the decoded lengths h_steps[b] * r go from the decode's status words straight to the
   vocoder launches, which read d_post in place (frame-major). Arguments as tts_taco_infer_spk
   (d_spk_ids / d_spk_emb may both be NULL: single-speaker model) plus the vocoder's inference
   padding `pad` and d_wav, which must hold B * hop * (S_cap * r + 2 pad) floats (hop = 4 x the
   product of the upsample factors). On return its first B * hop * (M + 2 pad) floats, M = r *
   max(h_steps), are the (B, 1, hop * (M + 2 pad)) waveform batch: bit-identical to
   tts_melgan_infer_strided on d_post viewed as (B, 80, M) with strides (S_cap r 80, 1, 80) and
   lengths h_steps * r. The vocoder is launched on the decoded lengths as the decode leaves them on
   the device (rows shorter than the vocoder's reflection pads fail the call), before the host
   reads the decode's status words. Split-f16 range scopes as the two calls: a decode overflow
   re-runs decode and vocoder in fp32, a vocoder overflow the vocoder alone. Returns with the
   call's work done. */
int tts_taco_mbmelgan_infer(tts_ctx* ctx, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, int r,
                            const int32_t* h_max_steps, int S_cap, float thr, const int64_t* d_spk_ids,
                            const float* d_spk_emb, float* d_dec, float* d_post, float* d_align, float* d_stop,
                            int pad, float* d_wav, int32_t* h_steps, int32_t* h_status, void* stream);

/* tts_taco_mbmelgan_infer in two halves, so that a caller can queue the next batch while this
   one's vocoder runs. submit returns when h_steps / h_status are filled and hands out *h_ticket:
   the decode's outputs are done and later work on `stream` is ordered after them, while the
   vocoder may still be running on the library's stream. finish(ticket, stream) waits for that
   vocoder and, if its split-f16 operands left the f16 range, runs it again on the fp32 kernels;
   then d_wav is final and later work on `stream` is ordered after it. Until finish, the caller
   must leave d_post and d_wav untouched and must not read d_wav. At most 4 submissions are outstanding per context: a fifth submit finishes the oldest
   first. finish on a ticket that is already complete returns 0. */
int tts_taco_mbmelgan_submit(tts_ctx* ctx, const int64_t* d_ids, const int32_t* h_lens, int B, int T_max, int r,
                             const int32_t* h_max_steps, int S_cap, float thr, const int64_t* d_spk_ids,
                             const float* d_spk_emb, float* d_dec, float* d_post, float* d_align, float* d_stop,
                             int pad, float* d_wav, int32_t* h_steps, int32_t* h_status, int64_t* h_ticket,
                             void* stream);
int tts_taco_mbmelgan_finish(tts_ctx* ctx, int64_t ticket, void* stream);

/* Test hook (process-wide, off by default): recurrence >= 0 makes one workgroup of that persistent
   BiLSTM recurrence leave before its second grid barrier, so the others time out and the next
   Tacotron2 call reports the encoder barrier error; -1 turns it off. Only tests call it. */
int tts_test_stall_lstm(int recurrence);

#ifdef __cplusplus
}
#endif
#endif

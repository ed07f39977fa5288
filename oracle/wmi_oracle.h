/*
 * wmi_oracle.h — CPU restatement of the reference Whisper path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * or the timed CPU baseline — never as part of the product path.
 *
 * PARITY UNPINNED: the reference (szuwgh/whisper.rs) cannot be built here
 * (no Rust toolchain; its arithmetic crate `galois` is an absent path
 * dependency, Cargo.toml:13) and its tests pin no numbers (main.rs:2077-2118).
 * The mel frontend restates main.rs:1486-1679 operation for operation; the
 * tensor ops restate ggml-1.0.3 semantics, which SURVEY.md §A assumes galois
 * follows; the decoder restates SURVEY.md §A.7 (absent from the reference).
 * See oracle/README.md.
 */
#ifndef WMI_ORACLE_H
#define WMI_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_model or_model;

/* WhisperContext::new + WhisperModel::load (main.rs:366-503, 808-1483).
 * Returns a wmi_status code; err receives the formatted message. */
int or_load(const char *path, or_model **out, char *err, size_t errcap);
void or_free(or_model *m);
void or_get_hparams(const or_model *m, int32_t hp[11]);
/* eot, sot, prev, solm, not, beg, translate, transcribe, is_multilingual */
void or_special_tokens(const or_model *m, int32_t out[9]);
/* prompt tokens; returns count (<= 8) */
int or_prompt(const or_model *m, int32_t *out);

/* 0: ggml AVX2 vec_dot_f16 accumulation order (default); 1: exact double dot
 * products.  The second mode exists only to measure the summation-order noise
 * floor of the arithmetic (tests/test_oracle.py, DESIGN.md "Parity"). */
void or_set_dot_mode(int exact_double);

/* The loader's dequantisation of ggml quantised blocks to f16 (types 2 q4_0,
 * 3 q4_1, 6 q5_0, 7 q5_1, 8 q8_0): w = f16(q * d (+ m)) rounded once. */
int or_dequant(int type, const uint8_t *src, int64_t nel, uint16_t *dst);

/* ggml lookup tables (ggml_init): f16 GELU and f16 exp, 65536 entries each. */
void or_tables(uint16_t *gelu, uint16_t *expt);

/* log_mel_spectrogram + clamp_and_normalize (main.rs:1554-1671).
 * mel may be NULL to query n_len.  mel is [n_mels][n_len]. */
int or_mel(const or_model *m, const float *pcm, size_t n_samples, int n_threads,
           float *mel, int32_t *n_len);

/* The reference's stage checksums (debug prints): {_hann, samples, filters,
 * mel before clamp_and_normalize, the encoder's mel window}, each the
 * sequential f32 sum the reference prints (main.rs:1571, 1686, 1690, 1647,
 * 1832). */
int or_checksums(const or_model *m, const float *pcm, size_t n_samples, int mel_offset, int n_ctx, int n_threads,
                 float out[5]);

/* whisper_encode (main.rs:1799-2063).  enc_out [n_ctx][n_state] f32;
 * cross_k / cross_v [n_text_layer][n_ctx][n_text_state] f16 bits.
 * probe (optional) receives the residual stream after the conv stem + PE and
 * after every encoder layer: [n_audio_layer + 1][n_ctx][n_state]. */
int or_encode(const or_model *m, const float *mel, int32_t n_len, int mel_offset, int n_ctx,
              int n_threads, float *enc_out, uint16_t *cross_k, uint16_t *cross_v, float *probe);

/* Teacher-forced decoder: logits [n_tokens][n_vocab]. */
int or_decode_logits(const or_model *m, const uint16_t *cross_k, const uint16_t *cross_v, int n_ctx,
                     const int32_t *tokens, int n_tokens, int n_threads, float *logits);

/* Greedy decode after the prompt.  tokens_out[max_tokens]; margins (optional)
 * receives top1 - top2 logit per generated token. */
int or_decode_greedy(const or_model *m, const uint16_t *cross_k, const uint16_t *cross_v, int n_ctx,
                     int max_tokens, int suppress_eot, int n_threads,
                     int32_t *tokens_out, int32_t *n_out, float *margins);

/* Beam search (config C5).  Absent from the reference and from whisper.cpp
 * 1.0.3, so the semantics are defined here, after OpenAI whisper's
 * BeamSearchDecoder without length penalty (parity unpinned beyond this
 * restatement):
 *  - K = beam hypotheses; step 0 expands hypothesis 0 (the prompt) only;
 *  - each active hypothesis b contributes its top K+1 tokens by logit
 *    (ties: lower id), scored score_b + (logit - lse_b), lse_b = max +
 *    log(sum exp(logit - max)) in double over all n_vocab logits (EOT at -inf
 *    when suppressed);
 *  - candidates ranked by (score desc, beam asc, rank asc); walking the
 *    ranking, an EOT candidate finishes its hypothesis (kept while fewer than
 *    K have finished), any other fills the next active slot, until K slots
 *    are filled;
 *  - stops when K hypotheses have finished or max_tokens steps ran; the
 *    result is the best score / length (length excludes EOT) among the first
 *    K of: finished hypotheses in order, then active ones in slot order.
 * tokens_out receives the chosen sequence (with its EOT if finished);
 * min_gap (optional) the smallest selection margin met (last kept vs first
 * rejected candidate at every step, best vs second in the final choice);
 * step_gap (optional, [max_tokens]) each step's selection margin (INFINITY
 * where none was met); step_logits (optional, [max_tokens][beam][n_vocab])
 * active hypothesis b's logits at step t before EOT suppression — the same
 * dec_step as or_decode_logits on its history, so teacher-forced logits —
 * and step_sel (optional, [max_tokens][beam][2]) the slots after step t:
 * (parent hypothesis, appended token); entries of inactive slots untouched. */
int or_decode_beam(const or_model *m, const uint16_t *cross_k, const uint16_t *cross_v, int n_ctx, int beam,
                   int max_tokens, int suppress_eot, int n_threads, int32_t *tokens_out, int32_t *n_out,
                   double *score_out, float *min_gap, float *step_gap, float *step_logits, int32_t *step_sel);

#ifdef __cplusplus
}
#endif
#endif

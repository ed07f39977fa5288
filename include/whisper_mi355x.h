/*
 * whisper_mi355x.h — C ABI of the MI355X-native Whisper hot path.
 *
 * This is the drop-in boundary for szuwgh/whisper.rs (snapshot 2024-08-07).
 * Every entry point below names the reference item it replaces
 * (file:line into /root/reference/src/main.rs).  A Rust caller binds this
 * header with a thin `extern "C"` block; the Python mirror
 * whisper.rs_amd/wmi.py binds it with ctypes.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Every array passed in or out is a HOST
 *    array owned by the caller; results are copied out.  Device memory is
 *    owned by the context.
 *  - Every call returns an int status (enum wmi_status).  Nothing aborts.
 *    wmi_last_error() gives the detailed message (tensor name, sizes, ...),
 *    mirroring the formatted WsError variants (main.rs:51-72).
 *  - One context per host thread per GPU; calls are stream-ordered on the
 *    context's HIP stream and synchronous at return (main.rs takes
 *    `&mut WhisperContext`, so the reference is single-caller too).
 *  - Layouts are the reference's: mel [n_mel][n_len] f32 (main.rs:1633),
 *    encoder output [n_ctx][n_state] f32 (ggml ne [n_state, n_ctx]),
 *    cross K/V [n_text_layer][n_ctx][n_state] f16 (main.rs:2018-2030).
 */
#ifndef WHISPER_MI355X_H
#define WHISPER_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* WsError (main.rs:51-72) mapped 1:1, plus device-side codes. */
enum wmi_status {
    WMI_OK = 0,
    WMI_E_IO = 1,             /* WsError::UnexpectIO        main.rs:54-55 */
    WMI_E_BAD_MAGIC = 2,      /* WsError::BadMagic          main.rs:56-57 */
    WMI_E_NO_SPACE = 3,       /* WsError::NotEnoughSpace    main.rs:58-59 */
    WMI_E_UNKNOWN_TENSOR = 4, /* WsError::UnknownTensor     main.rs:60-61 */
    WMI_E_BAD_REF_TENSOR = 5, /* WsError::BadRefTensor      main.rs:62-63 */
    WMI_E_WRONG_SIZE = 6,     /* WsError::WrongSizeTensor   main.rs:64-65 */
    WMI_E_WRONG_SHAPE = 7,    /* WsError::WrongShapeTensor  main.rs:66-67 */
    WMI_E_WRONG_BYTES = 8,    /* WsError::WrongBytesTensor  main.rs:68-69 */
    WMI_E_OP = 9,             /* WsError::WrongGTensor      main.rs:70-71 */
    WMI_E_UNEXPECTED = 10,    /* WsError::Unexpected        main.rs:52-53 */
    WMI_E_HIP = 11,           /* HIP runtime / kernel launch failure */
    WMI_E_RCCL = 12,          /* RCCL failure */
    WMI_E_UNSUPPORTED = 13,   /* valid file, feature not built (e.g. a ggml type other than f32 / f16 / q4_0 / q4_1 / q5_0 / q5_1 / q8_0) */
    WMI_E_INVALID_ARG = 14    /* bad pointer / size / state order */
};

/* WhisperHparams (main.rs:607-619), same field order as the file. */
typedef struct wmi_hparams {
    int32_t n_vocab;
    int32_t n_audio_ctx;
    int32_t n_audio_state;
    int32_t n_audio_head;
    int32_t n_audio_layer;
    int32_t n_text_ctx;
    int32_t n_text_state;
    int32_t n_text_head;
    int32_t n_text_layer;
    int32_t n_mels;
    int32_t f16;
} wmi_hparams;

/* WhisperVocab special ids after the multilingual shift (main.rs:557-575, 433-440). */
typedef struct wmi_special_tokens {
    int32_t eot, sot, prev, solm, not_, beg, translate, transcribe;
    int32_t is_multilingual;
} wmi_special_tokens;

/* Per-stage device times of the last pipeline call, milliseconds (hipEvents).
 * Replaces the never-written t_*_us fields of WhisperContext (main.rs:334-339). */
typedef struct wmi_timings {
    float mel_ms;
    float encode_ms;     /* conv stem -> ln_post */
    float cross_kv_ms;   /* cross-attention K/V precompute */
    float decode_ms;     /* prompt + generated tokens */
    int32_t n_decode_steps;
} wmi_timings;

typedef struct wmi_context wmi_context;

/* ---- lifecycle ------------------------------------------------------ */

/* WhisperContext::new(fname) (main.rs:366-503): open, magic, hparams,
 * filters, vocab (+extra tokens), weights; then upload to `device`.
 * max_clips sizes the device workspace for batched calls (>= 1).  Weight
 * types: f16 and f32 files (hparams.f16 = 1 / 0, main.rs:817-821; f32
 * matrices are kept f32 on the device) and the ggml quantised types. */
int wmi_init_from_file(const char *path, int device, int max_clips, wmi_context **out);
void wmi_free(wmi_context *ctx);
const char *wmi_strerror(int status);
const char *wmi_last_error(const wmi_context *ctx);
/* Library-level last error (for failures before a context exists). */
const char *wmi_last_error_global(void);

int wmi_get_hparams(const wmi_context *ctx, wmi_hparams *out);
int wmi_get_special_tokens(const wmi_context *ctx, wmi_special_tokens *out);
/* WhisperContext.exp_n_audio_ctx (main.rs:362, 1803-1807): 0 = n_audio_ctx. */
int wmi_set_audio_ctx(wmi_context *ctx, int n_audio_ctx);
/* id_to_token (main.rs:578-592, 442-467): copies the token bytes (not NUL
 * terminated) into buf, *len = byte count; WMI_E_NO_SPACE if cap too small. */
int wmi_token_to_bytes(const wmi_context *ctx, int32_t id, char *buf, size_t cap, size_t *len);

/* ---- audio input and text output --------------- */

/* hound::WavReader::open(path) + samples::<i16>() (main.rs:2067-2068):
 * 16-bit integer PCM RIFF/WAVE, samples interleaved as stored.  With
 * samples == NULL only *n_samples (and rate / channels) are filled.
 * WMI_E_IO: missing / malformed file; WMI_E_UNSUPPORTED: not 16-bit PCM;
 * WMI_E_NO_SPACE: cap < *n_samples.  Needs no context or device. */
int wmi_read_wav(const char *path, int16_t *samples, size_t cap, size_t *n_samples, int32_t *sample_rate,
                 int32_t *channels);
/* convert_integer_to_float_audio (main.rs:1673-1679): out[i] = s16[i] / 32768. */
int wmi_pcm16_to_f32(const int16_t *s16, size_t n, float *out);
/* Detokenise: the id_to_token bytes (main.rs:578-592) of the text tokens
 * (id < eot) of ids[0..n), concatenated; special and timestamp tokens are
 * skipped.  *len = byte count; WMI_E_NO_SPACE if cap < *len. */
int wmi_tokens_to_text(const wmi_context *ctx, const int32_t *ids, int n, char *buf, size_t cap, size_t *len);

/* ---- pipeline (reference entry points) ------------------------------ */

/* whisper_pcm_to_mel (main.rs:1681-1707): f32 PCM (s16/32768) -> log-mel. */
int wmi_pcm_to_mel(wmi_context *ctx, const float *pcm, size_t n_samples);
/* Batched form: n_clips independent clips (each <= max_clips). */
int wmi_pcm_to_mel_batch(wmi_context *ctx, int n_clips, const float *const *pcm, const size_t *n_samples);

/* whisper_encode (main.rs:1799-2063): mel window at mel_offset -> conv stem
 * -> encoder blocks -> ln_post -> cross-attention K/V for every decoder
 * layer.  n_threads is accepted and ignored, as in the reference (:1799).
 * Runs on every clip loaded by the last pcm_to_mel call. */
int wmi_encode(wmi_context *ctx, int n_threads, int mel_offset);

/* Greedy decode (the reference declares the decoder but has
 * no forward pass).  Prompt = [SOT] (.en) or [SOT, lang(en), transcribe],
 * then NOT.  Generates up to max_tokens ids per clip; stops a clip at EOT
 * unless suppress_eot != 0 (then exactly max_tokens).  tokens is
 * [n_clips][max_tokens]; n_tokens[c] = ids written for clip c. */
int wmi_decode_greedy(wmi_context *ctx, int max_tokens, int suppress_eot,
                      int32_t *tokens, int32_t *n_tokens);

/* Teacher-forced decoder logits for clip `clip`: feeds tokens[0..n) one at a
 * time from position 0 and writes logits[n][n_vocab] (f32). */
int wmi_decode_logits(wmi_context *ctx, int clip, const int32_t *tokens, int n_tokens, float *logits);

/* Beam search (config C5; absent from the reference, semantics after OpenAI
 * whisper's BeamSearchDecoder without length penalty, stated in
 * oracle/wmi_oracle.h).  beam_size <= 8; one clip at a time, beam_size decoder
 * rows.  tokens is [n_clips][max_tokens]: the best hypothesis (ending in EOT
 * if it finished); n_tokens[c] its length; scores[c] (optional) its summed
 * log-probability. */
int wmi_decode_beam(wmi_context *ctx, int beam_size, int max_tokens, int suppress_eot, int32_t *tokens,
                    int32_t *n_tokens, double *scores);

/* Transcribe: pcm_to_mel -> encode -> decode_greedy for one clip. */
int wmi_full(wmi_context *ctx, const float *pcm, size_t n_samples, int max_tokens,
             int32_t *tokens, int32_t *n_tokens);

/* ---- timestamps, segments, long audio ---------- */

/* WhisperTokenData (main.rs:317-331) as sampled: id, tid = most probable
 * timestamp token, p = P(id), pt = P(tid) / (sum of timestamp
 * probabilities + 1e-10), ptsum = that sum.  Token-level t0 / t1 are not
 * computed (-1) and vlen is 0, as in whisper.cpp-1.0.3 by default. */
typedef struct wmi_token_data {
    int32_t id, tid;
    float p, pt, ptsum;
    int64_t t0, t1;
    float vlen;
} wmi_token_data;

/* One timestamp-decoding window of the encoded clip 0 after `prompt`
 * (whisper.cpp-1.0.3 sampling: the first token is the most probable
 * timestamp > beg; then a timestamp whenever the timestamp probabilities sum
 * above the most probable text token, else the most probable token other
 * than sot / solm / not).  Stops after EOT or max_tokens; out[max_tokens]. */
int wmi_decode_timestamps(wmi_context *ctx, const int32_t *prompt, int n_prompt, int max_tokens,
                          wmi_token_data *out, int32_t *n_out);
/* whisper_full with timestamps over audio of any length: 30 s windows
 * (2 * n_audio_ctx mel frames) advanced by the last timestamp (mel_offset,
 * main.rs:1822-1823), earlier text as prompt context; fills the context's
 * segment list (WhisperSegment, main.rs:599-604; result_all, main.rs:353).
 * max_tokens caps the tokens per window (<= n_text_ctx / 2 - 4). */
int wmi_transcribe(wmi_context *ctx, const float *pcm, size_t n_samples, int max_tokens, int32_t *n_segments);
/* Segment i of the last transcribe: [t0, t1) in 10 ms units, text bytes. */
int wmi_get_segment(const wmi_context *ctx, int i, int64_t *t0, int64_t *t1, char *text, size_t cap, size_t *len);
/* Its tokens (text and timestamp tokens of the segment). */
int wmi_get_segment_tokens(const wmi_context *ctx, int i, wmi_token_data *out, size_t cap, int32_t *n);

/* ---- device-resident benchmark path --------------------------------- */

/* Upload n_clips PCM clips to HBM once (untimed). */
int wmi_stage_pcm(wmi_context *ctx, int n_clips, const float *const *pcm, const size_t *n_samples);
/* mel -> encode -> cross-KV -> decode (n_decode tokens, EOT suppressed) on
 * the staged clips; token ids stay on the device until wmi_get_tokens. */
int wmi_run_staged(wmi_context *ctx, int mel_offset, int n_decode);
/* Same with beam search of beam_size (EOT suppressed, exactly n_decode tokens). */
int wmi_run_staged_beam(wmi_context *ctx, int mel_offset, int n_decode, int beam_size);
int wmi_get_tokens(const wmi_context *ctx, int32_t *tokens, size_t cap, int32_t *n_per_clip);
int wmi_get_timings(const wmi_context *ctx, wmi_timings *out);
/* Block until all work queued on the context's stream is done. */
int wmi_sync(wmi_context *ctx);

/* Re-launch one kernel of the last pipeline call `iters` times between HIP
 * events on the context stream (bench.py's live roofline measurement).
 * which: 14 = the persistent greedy decoder over the staged clips (one launch
 * per 8-row block, as run_staged makes it; algorithmic bytes summed per step),
 * 0 = the kernel chain's logits GEMV + argmax, 1 = encoder MLP-up GEMM of
 * layer 0 (MFMA), 2 = encoder attention of layer 0, 3 = cross-K/V GEMM. */
typedef struct wmi_kernel_bench {
    float avg_us;          /* mean launch duration */
    double alg_bytes;      /* algorithmic HBM bytes per launch */
    double alg_flops;      /* algorithmic FLOPs per launch */
    char name[48];
} wmi_kernel_bench;
int wmi_bench_kernel(wmi_context *ctx, int which, int iters, wmi_kernel_bench *out);

/* Algorithmic bytes and FLOPs of one decode on a model of hparams hp (host
 * only, no device): `steps` decoder steps of `rows` rows; beam != 0: the rows
 * are hypotheses of ONE clip (its cross K/V read once a step), else clips
 * decoded in blocks of 8 rows; q5 != 0: the five q5_1 GEMV matrices (Wqkv,
 * Wo, Wco, W0, W1 = 13 n^2 weights) at 24 bytes a 32-weight block, Wcq and the
 * vocabulary f16.  Every step reads each decoder weight once (shared by the
 * block's rows), each row's cross K/V and self K/V rows [0, pos] and writes
 * its new K/V row.  wmi_bench_kernel 14 and bench.py use this one count. */
int wmi_decode_alg_bytes(const wmi_hparams *hp, int rows, int steps, int beam, int q5, double *bytes, double *flops);

/* Device self-test: the decoder computes ggml's f16 exp table entries
 * instead of looking them up; *n_mismatch = entries (of 31745 non-positive
 * f16 inputs) where the computed value differs from the host-built table. */
int wmi_selftest(wmi_context *ctx, int32_t *n_mismatch);

/* The reference's stage checksums (its debug println!s, each a sequential
 * f32 sum): out5 = {_hann (main.rs:1571-1572), the samples (:1682-1686), the
 * filters (:1688-1690), clip 0's mel before clamp_and_normalize
 * (:1645-1647), clip 0's encoder mel window (:1819-1832)}.  Computed (and
 * printed in the reference's order) only when the context was created with
 * WMI_CHECKSUMS=1; the model-only sums (_hann, filters) always. */
int wmi_get_checksums(const wmi_context *ctx, float *out5);

/* Debug: copy a device buffer of the last decode into out (min of its size
 * and bytes).  which: 0 / 1 = the kernel chain's residual-stream buffers
 * [8][n_text_state] f32, 2 = logits [8][n_vocab] f32 (the persistent
 * decoder fills them only with WMI_PERSIST_LOGITS=1), 3 = the persistent
 * decoder's exchange block (8-byte {tag, value} granules), 4-9 = decoder
 * chain scratch, 10 = this context's tuning knobs (11 int32, host copy; the
 * WMI_* environment is read once per context at wmi_init_from_file),
 * 11 = decodes re-run on the kernel chain (int32, host), 12 = the encoder
 * residual stream, 13 = every position's logits [n_text_ctx][rows][n_vocab]
 * f32 of the last persistent greedy decode (clip b in row b) or beam search
 * (slot s in row s; contexts created with WMI_LOGITS_ALL=1), 14 / 15 = the
 * last beam search's parent slots / tokens [n_text_ctx][8] int32 (its last
 * clip), 16 = the rows of 13 (int32, host: max(8, max_clips)), 17 = the
 * persistent decoder's grid per row count (int32 [9], host; -1 = not sized
 * yet, 0 = kernel chain), 18 = the encoder GELU epilogues' threshold (f32,
 * host: f16 inputs at or above it are computed, the rest read ggml's table;
 * +inf with WMI_GELU_CALC=0). */
int wmi_debug_read(const wmi_context *ctx, int which, void *out, size_t bytes);

/* ---- parity getters (copy device results into caller-owned buffers) --- */

/* ctx.mel (main.rs:1574-1578): [n_mel][n_len] f32. */
int wmi_get_mel(const wmi_context *ctx, int clip, float *out, size_t cap, int32_t *n_mel, int32_t *n_len);
/* ln_post output (main.rs:1977-1986): [n_ctx][n_audio_state] f32. */
int wmi_get_encoder_out(const wmi_context *ctx, int clip, float *out, size_t cap);
/* memory_cross_k / memory_cross_v (main.rs:2018-2030): f16 bit patterns,
 * [n_text_layer][n_ctx][n_text_state] each. */
int wmi_get_cross_kv(const wmi_context *ctx, int clip, uint16_t *k, uint16_t *v, size_t cap);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ------------------ */

/* Size of the opaque RCCL unique id blob (ncclUniqueId). */
size_t wmi_dist_id_size(void);
/* Rank 0 creates the id; every rank passes the same bytes to init. */
int wmi_dist_make_id(void *id_out);
int wmi_dist_init(wmi_context *ctx, int rank, int world, const void *id);
/* Gather every rank's token block to root 0 over RCCL (ncclGather).  A block
 * is [n_clips][1 + n_decode] int32: per clip its token count, then its tokens
 * (-1 padded) — greedy or beam, whichever the last staged run was.  Every
 * rank must have staged the same n_clips and n_decode (checked with an
 * all-reduce first: WMI_E_INVALID_ARG on every rank otherwise).  out (root
 * only; others may pass NULL) is [world][n_clips][1 + n_decode]. */
int wmi_dist_gather_tokens(wmi_context *ctx, int32_t *out, size_t cap);
/* Device-side barrier over the communicator (an RCCL all-reduce of a
 * dedicated int; gathered tokens are never touched). */
int wmi_dist_barrier(wmi_context *ctx);

#ifdef __cplusplus
}
#endif

#endif /* WHISPER_MI355X_H */

// wmi_internal.h — launch interface between the C-ABI host layer
// (wmi_api.cpp) and the gfx950 kernels (wmi_kernels.hip).
//
// Every launcher enqueues on the given stream and returns hipError_t; no
// launcher allocates, copies or synchronises, so a caller may capture any
// sequence of them into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wmi {

// ---- launch-overhead probes: 0 = empty kernel, 1 = 256 x 4 KiB copy ---------
// device exp (decoder attention) vs the host-built ggml exp table, all inputs
hipError_t launch_selftest(hipStream_t s, const uint16_t *exp_tab, int n_exp, uint32_t *mismatch);

// ---- mel frontend (main.rs:1486-1671) ---------------------------------------
// Constant tables built on the host with the reference's exact f32 formulas
// (main.rs:1495, 1537, 1568), uploaded once.
struct MelTables {
    float hann[400];
    float c400[200], s400[200], c200[100], s200[100], c100[50], s100[50], c50[25], s50[25];
    float dc[625], ds[625];
};
static_assert(sizeof(MelTables) % 16 == 0, "k_mel_frames copies MelTables in 16-byte chunks");

// frames -> raw log10 mel [n_mel][n_len] + per-clip ordered-uint max.
// pcm: n_clips pointers (device) with n_samples each (device arrays).
hipError_t launch_mel_frames(hipStream_t s, const MelTables *tabs, const float *filt_t /*[201][n_mel]*/, int n_mel,
                             const float *const *pcm, const int64_t *n_samples, float *mel, int64_t mel_stride,
                             const int64_t *n_len, int64_t max_len, uint32_t *mel_max, int n_clips,
                             const float *filt_c /* compact bank (wmi_api.cpp), or null: LDS copy of filt_t */, int n_fc);
constexpr int MEL_FC_MAX = 4096;  // floats of the compact filterbank k_mel_frames keeps in LDS
// the state a decode run starts from, in one launch instead of a host copy
// and five memsets (each a separate ~5 us fill kernel): zero `n` byte ranges
// (4-byte aligned, sizes multiple of 4) and write feed[0..n_feed) to dfeed
struct ResetArgs {
    void *ptr[8];
    size_t bytes[8];
    int n;
    int32_t *dfeed;
    int n_feed;
    int32_t feed[64];
};
hipError_t launch_dec_reset(hipStream_t s, const ResetArgs &a);
// clamp_and_normalize in place on mel.
hipError_t launch_mel_norm(hipStream_t s, float *mel, int64_t mel_stride, int n_mel, const int64_t *n_len,
                           int64_t max_len, const uint32_t *mel_max, int n_clips);
// mel window (main.rs:1816-1833) -> conv1 input, f16 time-major, zero-padded
// by one frame at each end and to Cp channels: X[b][T2 + 2][Cp].
hipError_t launch_mel_window(hipStream_t s, const float *mel, int64_t mel_stride, int n_mel, const int64_t *n_len,
                             int mel_offset, int T2, int Cp, uint16_t *xconv, int n_clips,
                             float *xconv32 = nullptr, uint16_t *g1 = nullptr, int n = 0);

// ---- LayerNorm (ggml norm + mul(repeat(w)) + add(repeat(b))) ----------------
hipError_t launch_layernorm(hipStream_t s, const float *x, int rows, int n, const float *w, const float *b,
                            uint16_t *y16, float *y32);

// ---- MFMA GEMM: C[M][N] = A[M][K] * B[N][K]^T, f16 in, f32 accumulate -------
enum GemmEpi {
    EPI_F32 = 0,        // out32[m][n] = acc + bias
    EPI_RESID = 1,      // out32[m][n] = (acc + bias) + out32[m][n]
    EPI_GELU16 = 2,     // out16[m][n] = gelu_tab[f16(acc + bias)]
    EPI_QKV = 3,        // q/k [b][h][Tp][64], vt [b][h][64][Tp]   (acc + bias) -> f16
    EPI_CONV1 = 4,      // out16[b][t + 1][n] = gelu_tab[f16(acc + bias)]  (padded time-major)
    EPI_CONV2PE = 5,    // out32[b*T + t][n] = pe[t][n] + gelu_tab[f16(acc + bias)]
    EPI_CROSSKV = 6,    // K: f16(acc * kscale), V: f16(acc + bias) -> [l][b][T][ns]
};

// Tuning knobs of one context (WMI_* environment variables read at
// wmi_init_from_file).  Kernel-argument structs carry a pointer to their
// context's copy; a null pointer means the defaults below.
struct Tune {
    int logits_cap = 512;   // WMI_LOGITS_CAP: chain logits grid cap
    int logits_g = 2;       // (fixed) chain logits rows per lane group
    int gemv_nw = 4;        // (fixed) waves per chain decoder GEMV workgroup
    int xattn_rows = 1;     // WMI_XATTN_ROWS: beam rows share cross-attention phase A (1 auto, 2 always, 0 never)
    int graph_steps = 8;    // WMI_GRAPH_STEPS: chain decoder steps per captured graph
    int enc_attn_nw = 0;    // WMI_ENC_ATTN_NW: 32-query blocks (four key-part waves each) per k_attn_enc4 workgroup (0 auto, 1, 2, 4)
    int gemm_g = 1;         // WMI_GEMM_G: large-M encoder GEMMs on k_gemm_g (LDS-DMA staging); 0: k_gemm
    // WMI_MEL_G=0: the dense-filterbank mel layout (4 two-frame waves, LDS
    // copy of the whole [201][n_mel] bank) that a file whose bank has more
    // than MEL_FC_MAX non-zero weights takes anyway; tested bitwise equal
    int mel_g = 1;
    int epi_staged = 1;     // WMI_GEMM_EPI: GEMM epilogues through LDS, 16 / 8-byte stores (0: per-lane 2 / 4-byte stores)
    int gelu_calc = 1;      // WMI_GELU_CALC: encoder GELU epilogues compute the table's values above the scanned threshold (0: table only)
    int gemm_p = 1;         // WMI_GEMM_P: one-clip encoder GEMMs on k_gemm_p (LDS-DMA ring); 0: k_gemm
};
// (fixed since round 5; their alternatives measured slower and are removed:
// chain logits grid cap at K <= 512, cooperative chain cross-attention up to
// 512 workgroups, k_gemm_g from 240 128 x 128 tiles)
constexpr int CHAIN_LOGITS_CAP2 = 1024, CHAIN_COOP_MAX = 512, GEMM_G_MIN_TILES = 240;
extern const Tune kTuneDefault;
inline const Tune &tune_of(const Tune *t) { return t ? *t : kTuneDefault; }

struct GemmArgs {
    const Tune *tune;   // context knobs (null: defaults)
    const uint16_t *A;  // plain: [M][lda]; conv: X[b][Tin + 2][Cp]
    const uint16_t *B;  // [N][K]
    const float *bias;  // [N] or null
    int M, N, K, lda;
    // implicit-GEMM conv: row m -> (b = m / Tout, t = m % Tout); k -> (tap, c)
    int conv, conv_stride, conv_tin, conv_cp, conv_tout;
    float *out32;
    uint16_t *out16;
    int ldo;
    const uint16_t *gelu_tab;
    float gelu_min = __builtin_huge_valf();  // GELU epilogues compute inputs >= gelu_min (gelu_bits), +inf: table only
    const float *pe;    // EPI_CONV2PE: [T][N]
    int T;              // rows per clip (for b/t split)
    // EPI_QKV
    uint16_t *q, *k, *vt;
    int Tp, n_state;
    // EPI_CROSSKV
    uint16_t *ck, *cv;
    int n_clips;
    float kscale;
    // f32 models (ggml f32 x f32 mul_mat / conv: neither operand rounded):
    // B32 = f32 weights [N][K] selects the f32 MFMA GEMM (wmi_f32.hip); its
    // A operand is A32 (f32) when set, else A (f16: GELU-table outputs, exact)
    const float *A32, *B32;
    int epi_staged;     // set by launch_gemm from the context's knob (Tune::epi_staged)
};
hipError_t launch_gemm(hipStream_t s, int epi, const GemmArgs &a);
// exhaustive scan of gelu_bits' computed path against the table: maxord[0] =
// the largest ord_f32(f) over f16 inputs f whose computed value differs
// (0 if none), maxord[1] = the inputs checked (the caller zeroes both)
hipError_t launch_gelu_scan(hipStream_t s, const uint16_t *gelu_tab, uint32_t *maxord);
hipError_t launch_gemm32(hipStream_t s, int epi, const GemmArgs &a);  // wmi_f32.hip

// ---- encoder self-attention (ggml flash_attn_f16 semantics, exact softmax) --
struct AttnArgs {
    const Tune *tune;  // context knobs (null: defaults)
    const uint16_t *q, *k, *vt;  // [b][h][Tp][64], vt [b][h][64][Tp]
    uint16_t *out;               // [b*T + t][n_state]
    float *out32;                // or f32 output (f32 models: Wo takes it unrounded)
    const uint16_t *exp_tab;     // f16 exp table, negative half
    int n_exp;                   // entries in exp_tab
    int T, Tp, H, n_state, n_clips;
    float scale;
};
hipError_t launch_attn_enc(hipStream_t s, const AttnArgs &a);
// k_attn_enc4 query blocks per workgroup, as launch_attn_enc picks them
int attn_enc_nw(int T, int H, int n_clips, int nw_knob);
int attn_enc_kq(int T, int H);

// ---- decoder step -----------------------------------------
struct DecState {          // device-resident, advanced by the kernels
    int32_t pos;           // position of the token being processed
    int32_t pad[3];
};

enum DecEpi { DEC_QKV = 0, DEC_Q = 1, DEC_GELU = 2, DEC_RESID = 3, DEC_LOGITS = 4 };

struct DecGemvArgs {
    const Tune *tune;  // context knobs (null: defaults)
    const float *x;          // LN input [B][K] f32 (ln != null)
    const float *ln_w, *ln_b;
    const uint16_t *xin16;   // non-LN input [B][K] f16
    const float *parts;      // or: split-key attention partials [B][n_parts][K] f32, summed in order
    int n_parts;
    const uint16_t *W;       // [N][K]
    const uint8_t *Wq5;      // or q5_1 blocks repacked (nibbles [N][K/2], then {5th bits, d | m << 16} [N][K/32])
    const float *bias;       // [N] (null for logits)
    int N, K, B;
    float qscale;            // (n/h)^-0.25
    // outputs
    uint16_t *out16;         // DEC_Q / DEC_GELU / DEC_QKV(q): [B][ldo]
    float *out32;            // DEC_RESID: x [B][N]; DEC_LOGITS: logits [B][N]
    int ldo;
    uint16_t *kcache, *vcache;  // DEC_QKV: [B][n_text_ctx][n]
    int n_text_ctx;
    const DecState *st;
    const uint16_t *gelu_tab;
    unsigned long long *amax;   // DEC_LOGITS: packed argmax, AMAX_SHARDS shards per clip
    int suppress_id;            // DEC_LOGITS: id excluded from argmax (-1 none)
    DecState *st_advance;       // DEC_LOGITS: pos += 1 (block 0)
    // embed prologue (IN = 3, first layer): x = te[tok] + pe[pos], tok from
    // feed[b][pos] while pos < feed_len, else from the previous step's argmax
    const uint16_t *te;
    const float *pe;
    const int32_t *feed;
    int feed_len, feed_stride;
    int32_t *tokens_out;        // [B][out_stride], token of pos - feed_len
    int out_stride;
    float *x_out;               // residual stream written by block 0
    const int32_t *beam_tok;    // beam search: token of row b past the prompt (BeamState::tok), else null
    // f32 models: W32 = f32 weights [N][K] (W / Wq5 unused), te32 = f32 token
    // embedding for IN = 3; activations stay f32 into the dot (wmi_f32.hip)
    const float *W32, *te32;
};
constexpr int AMAX_SHARDS = 64;
constexpr int DEC_ROWS = 8;  // decoder rows per step: clips (greedy) or beam hypotheses
hipError_t launch_dec_gemv(hipStream_t s, int epi, const DecGemvArgs &a);
hipError_t launch_dec_gemv32(hipStream_t s, int epi, const DecGemvArgs &a);  // wmi_f32.hip

struct DecAttnArgs {
    const Tune *tune;  // context knobs (null: defaults)
    const uint16_t *q;       // [B][n]
    const uint16_t *K, *V;   // per clip: rows of n (clip_stride elements apart)
    int64_t clip_stride;     // elements between clips in K/V
    int M_fixed;             // >0: fixed key count (cross); 0: pos + 1 (self)
    int mk;                  // self-attention: key capacity of this launch (64/128/256/512 >= pos + 1)
    const DecState *st;
    float *S;                // scores [B][H][s_stride]
    int s_stride;
    float *cmax;             // per-chunk max [B][H][n_chunks]
    float *opart;            // partial outputs [B][n_chunks][n]
    int n_chunks;            // 128-key chunks in the grid (covers the max M)
    const uint16_t *exp_tab;
    int n_exp, H, n, B;
    unsigned long long *reset_amax;  // self-attn: zero these B * AMAX_SHARDS words (block 0)
    // cross-attention: q = f16((Wq LN(x) + bq) * qscale) computed in the score kernel
    const float *x, *ln_w, *ln_b;
    const uint16_t *Wq;
    const float *bq;
    float qscale;
    // cooperative single-kernel cross-attention: per (clip, head) exchange
    // words for this layer, zeroed at the start of every decode run
    struct XSync *sync;
    uint32_t *err;           // set to 1 if an exchange spin times out
    // beam search: self-attention reads key/value row j < pos of decoder row b
    // from cache slot kv_src[b * kv_src_stride + j] (its hypothesis' history);
    // cross-attention rows b share clip b / clip_div
    const int32_t *kv_src;
    int kv_src_stride;
    int clip_div;
    // self-attention with the output projection fused (Wo null: o_h -> opart):
    // head h writes Wo[:, h*64:(h+1)*64] . f16(o_h) to wo_parts[b][h][n]
    const uint16_t *Wo;
    float *wo_parts;
    // cross-attention prologue (res_parts non-null): x_out = (res_bias +
    // sum_h res_parts[b][h]) + x, the fused self-attention's residual update,
    // then LN(x_out); block (0, 0, b) stores x_out[b] (x_out != x: ping-pong)
    const float *res_parts, *res_bias;
    float *x_out;
};
// exchange words of one (layer, clip, head) for the cooperative kernel
struct XSync {
    uint32_t cnt;            // monotonic arrival counter (target (pos + 1) * n_chunks)
    uint32_t pad[15];
};
hipError_t launch_dec_attn(hipStream_t s, const DecAttnArgs &a);

// ---- beam search (config C5; semantics in oracle/wmi_oracle.h) -------------
constexpr int BEAM_MAX = 8, BEAM_NS = 16, BEAM_TK = BEAM_MAX + 1;
struct BeamPart {            // one vocabulary split of one row
    float m;                 // split max
    float pad;
    double sum;              // sum exp(logit - m) over the split
    float val[BEAM_TK];      // split top-(K+1) by (value desc, id asc)
    int32_t id[BEAM_TK];
};
struct BeamState {
    int32_t n_active, n_fin, done, n_steps;
    double score[BEAM_MAX];      // cumulative log-probability of active slot s
    int32_t tok[BEAM_MAX];       // token slot s feeds at the next step
    int32_t fin_t[BEAM_MAX], fin_beam[BEAM_MAX];
    double fin_score[BEAM_MAX];
};
struct BeamArgs {
    const float *logits;     // [K][V]
    int V, K, suppress_id, eot, feed_len, max_tokens, tctx;
    const DecState *st;
    BeamPart *parts;         // [K][BEAM_NS]
    BeamState *bs;
    int32_t *kv_src;         // [K][tctx]
    int32_t *hist_parent, *hist_tok;  // [max_tokens][BEAM_MAX]
};
hipError_t launch_beam_step(hipStream_t s, const BeamArgs &a);

// ---- timestamp sampling (whisper.cpp-1.0.3 whisper_sample_best /
// whisper_sample_timestamp semantics, restated in oracle/pyoracle.py) --------
struct TsRec {               // WhisperTokenData (main.rs:317-331) as sampled
    int32_t id, tid;
    float p, pt, ptsum;
    int32_t pad;
};
struct TsArgs {
    const float *logits;     // [V] (row 0)
    int V, beg, eot, sot, solm, not_, feed_len, max_rec;
    const DecState *st;      // pos already advanced by the logits launch
    int32_t *tok_out;        // token fed at the next step
    TsRec *rec;              // [max_rec], record t = pos - feed_len
};
hipError_t launch_ts_sample(hipStream_t s, const TsArgs &a);

struct DecEmbedArgs {
    const uint16_t *te;      // [V][n]
    const float *pe;         // [n_text_ctx][n]
    float *x;                // [B][n]
    const int32_t *feed;     // [B][feed_stride] tokens fed while pos < feed_len
    int feed_len, feed_stride;
    unsigned long long *amax;
    int32_t *tokens_out;     // [B][out_stride]
    int out_stride;
    const DecState *st;
    int n, B, record_only;
};
hipError_t launch_dec_embed(hipStream_t s, const DecEmbedArgs &a);

// ---- persistent decoder: one launch runs n_steps greedy decoder steps -------
// (wmi_persist.hip).  Every decoder step is a fixed sequence of phases; the
// workgroups of the launch (all co-resident, one per CU) hand each phase's
// outputs to the next through epoch-tagged 8-byte granules {tag, value}
// written and read with agent-scope (sc1) accesses — the data is its own flag,
// so a seam costs one write-through store plus the consumer's poll, not a
// kernel boundary (MI355X_MICROARCH.md handoff / allgather rows; measured
// 1.8 us per all-to-all seam at 256 workgroups vs 2.1 us per graph kernel
// boundary, scripts/seam_probe.hip).
struct PersistLayer {          // decoder layer weights (device pointers)
    const float *ln1_w, *ln1_b;
    const uint16_t *wqkv; const float *bqkv;   // [3n][n], bias [3n] (zero for K)
    const uint16_t *wo; const float *bo;
    const float *lnc_w, *lnc_b;
    const uint16_t *wcq; const float *bcq;
    const uint16_t *wco; const float *bco;
    const float *ln2_w, *ln2_b;
    const uint16_t *w0; const float *b0;       // [4n][n]
    const uint16_t *w1; const float *b1;       // [n][4n]
    // q5_1 repacks of wqkv, wo, wco, w0, w1 (wmi_api.cpp repack_q5), or null
    const uint8_t *wqkv5, *wo5, *wco5, *w05, *w15;
};

// exchange block layout in granules (host and device agree)
struct XLayout {
    int x1, x2, x3, q, k, v, o, xq, oc, h, s, p, a, ctl, total;
};
constexpr int PX_TASKS = 2048;   // cross-attention (row, head, chunk) tasks
constexpr int PX_GMAX = 256;     // workgroups
__host__ __device__ inline XLayout persist_layout(int n, int H, int T) {
    XLayout L{};
    int o = 0;
    const int R = 8;  // DEC_ROWS
    L.x1 = o; o += R * n;
    L.x2 = o; o += R * n;
    L.x3 = o; o += R * n;
    L.q = o; o += R * n / 2;
    L.k = o; o += R * n / 2;
    L.v = o; o += R * n / 2;
    L.o = o; o += R * n / 2;
    L.xq = o; o += R * n / 2;
    L.oc = o; o += R * n / 2;
    L.h = o; o += R * 2 * n;
    // per (row, head, 128-key sub-chunk) of the cross attention: its max m and
    // its exact exp sum S (a double as lo, hi): [R][H][ceil(T / 128)][3]
    L.s = o; o += 3 * R * H * ((T + 127) / 128);
    L.p = o; o += R * H * ((T + 127) / 128) * 64;  // 128-key P.V partials
    L.a = o; o += R * PX_GMAX * 2;
    L.ctl = o; o += 16;             // ctl[0] low word: abort flag
    L.total = (o + 15) / 16 * 16;   // whole 128-byte lines (memset size a multiple of 16 B)
    return L;
}

struct PersistArgs {
    const PersistLayer *layers;  // device array [L]
    const uint16_t *te;          // token embedding [V][n]
    const float *pe;             // positional embedding [n_text_ctx][n]
    const float *dln_w, *dln_b;  // final LayerNorm
    const uint16_t *gelu_tab;    // ggml GELU table [65536]
    float gelu_min = __builtin_huge_valf();  // phase H computes GELU of f16 inputs >= gelu_min (gelu_bits), +inf: table
    const uint16_t *exp_tab;     // ggml exp table, non-positive half [n_exp]
    int n_exp;
    const uint32_t *exp_fb;      // [64] exp fallback list (launch_exp_fallbacks), 0xffffffff-padded
    uint16_t *kcache, *vcache;   // [L][DEC_ROWS][tctx][n]
    const uint16_t *ck, *cv;     // cross K/V [L][Bt][T][n]; row b uses clip b0 + b
    int L, n, V, B, T, tctx, Bt, b0;
    int nch, cl;                 // cross-attention chunks per (row, head), keys per chunk
    float qscale;                // (n / H)^-0.25
    DecState *st;                // pos advanced by n_steps at the end
    const int32_t *feed;         // [B][feed_stride] prompt tokens
    int feed_len, feed_stride;
    int32_t *tokens_out;         // [B][out_stride] generated tokens (index pos - feed_len)
    int out_stride;
    int32_t *cur_tok;            // [8] last argmax, carried to the next launch
    int suppress_id;
    int n_steps;
    uint64_t *xg;                // exchange block (persist_layout), zeroed before a run
    uint32_t *err;               // bit 3: exchange timeout
    unsigned long long *ptrace;  // WMI_PTRACE: [n_steps][L + 1][16][2] phase-end clocks, or null
    int nres;                    // vocabulary rows per workgroup resident in LDS
    float *logits_out;           // [B][V] logits of every step (debug / teacher forcing), or null
    int64_t lg_stride;           // > 0: position p's logits at logits_out + p * lg_stride (all-step capture)
    // beam search (one step per launch; the beam kernels select between launches):
    // rows are the beam slots of clip b0, step 0 feeds cur_tok (the beam state's
    // tokens), self-attention keys j < pos come from cache row kv_src[b][j], and
    // the launch records no argmax
    int beam;
    const int32_t *kv_src;       // [B][kv_src_stride] or null
    int kv_src_stride;
    int q5;                      // GEMVs of phases A, C, G2, H, I read the layers' q5_1 repacks
    // beam launches (rows = hypotheses of one clip, n > 768): one cross-
    // attention task per (head, key chunk) covers every row (PersistArgs::nch
    // then counts the chunks of one head: H * nch tasks)
    int xshare;
    // fault injection (tests): workgroup stall_wg exits at once, as a
    // workgroup that never became resident — every other workgroup's first
    // poll of its rows runs into the bounded spin, raises the abort word and
    // err bit 3, and the grid drains (-1: none)
    int stall_wg;
    // one-row VALU logits (n = 768): the vocabulary rows past the LDS-resident
    // ones stay in registers for the whole launch (an 8-pass WSet per
    // quarter-wave slot, at most 128 rows a workgroup) instead of streaming
    // every step (0: streamed; past 128 rows the kernel streams them anyway)
    int vreg;
};
hipError_t launch_dec_persist(hipStream_t s, const PersistArgs &a, int G);
// the inputs whose f32 exp is too close to an f16 midpoint, with their table
// values, into list[64] (count in *n; > 64 means the list is unusable)
hipError_t launch_exp_fallbacks(hipStream_t s, const uint16_t *exp_tab, int n_exp, uint32_t *list, uint32_t *n);
// the persistent decoder's exp vs the host ggml table, every non-positive f16 input
hipError_t launch_persist_selftest(hipStream_t s, const uint16_t *exp_tab, int n_exp, const uint32_t *fb,
                                   uint32_t *mismatch);
// largest co-resident grid for the model (0: not supported for this n / B / T)
// and the vocabulary rows per workgroup that fit in LDS beside the phases' data
int persist_grid(int device, int n, int B, int T, int V, int *nres);
// workgroups of each of two concurrent multi-row launches sharing the
// device's G-workgroup grid (0: the rows per workgroup would not fit)
int persist_split_grid(int n, int G);

}  // namespace wmi

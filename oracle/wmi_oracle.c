/*
 * wmi_oracle.c — CPU restatement of the reference Whisper hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see wmi_oracle.h): the parity checker for the HIP
 * path and the timed CPU baseline ("kind": "port").  PARITY UNPINNED — the
 * reference cannot run here and pins no numbers; see oracle/README.md.
 *
 * What each part restates:
 *   loader      WhisperContext::new / WhisperModel::load   main.rs:366-503, 513-535, 578-597, 808-1483
 *   mel         dft / fft / log_mel_spectrogram / clamp_and_normalize
 *                                                         main.rs:1486-1671 (op for op, same f32 order)
 *   encoder     whisper_encode                              main.rs:1799-2063
 *   ops         galois_* call sites main.rs:1709-1797, with ggml-1.0.3 numerics
 *               (assumed): f16 rounding of matmul/conv inputs,
 *               AVX2 vec_dot_f16 accumulation, double-accumulated norm,
 *               f16 GELU/exp lookup tables, flash-attn softmax
 *   decoder     SURVEY.md §A.7 (not present in the reference)
 *
 * Build: oracle/Makefile (gcc -O3 -mavx2 -mfma -mf16c -ffp-contract=off -fopenmp).
 * -ffp-contract=off keeps every f32 multiply/add separately rounded, as Rust
 * compiles main.rs (no implicit FMA contraction).
 */
#define _GNU_SOURCE
#include "wmi_oracle.h"
#include "../include/whisper_mi355x.h"

#include <immintrin.h>
#include <math.h>
#include <omp.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define GGML_MAGIC 0x67676d6cu /* main.rs:46 */
#define SR 16000               /* main.rs:25 */
#define NFFT 400               /* main.rs:26 */
#define HOP 160                /* main.rs:28 */

static inline float h2f(uint16_t h) { return _cvtsh_ss(h); }
static inline uint16_t f2h(float f) { return (uint16_t)_cvtss_sh(f, 0); }

/* ------------------------------------------------------------------------ */
/* ggml lookup tables (ggml_init, ggml-1.0.3)                                */
/* ------------------------------------------------------------------------ */
static uint16_t T_GELU[65536];
static uint16_t T_EXP[65536];
static int g_dot_double = 0; /* WMI_ORACLE_DOT=double: summation-order noise-floor experiment only */
static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

static void init_tables(void) {
    const char *dv = getenv("WMI_ORACLE_DOT");
    g_dot_double = dv && strcmp(dv, "double") == 0;
    const float GELU_COEF_A = 0.044715f;
    const float SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
    for (int i = 0; i < 65536; ++i) {
        const float f = h2f((uint16_t)i);
        T_GELU[i] = f2h(0.5f * f * (1.0f + tanhf(SQRT_2_OVER_PI * f * (1.0f + GELU_COEF_A * f * f))));
        T_EXP[i] = f2h((float)exp((double)f));
    }
}

void or_set_dot_mode(int exact_double) {
    pthread_once(&tables_once, init_tables);
    g_dot_double = exact_double != 0;
}

void or_tables(uint16_t *gelu, uint16_t *expt) {
    pthread_once(&tables_once, init_tables);
    if (gelu) memcpy(gelu, T_GELU, sizeof(T_GELU));
    if (expt) memcpy(expt, T_EXP, sizeof(T_EXP));
}

static inline float gelu_f16(float x) { return h2f(T_GELU[f2h(x)]); }

/* ------------------------------------------------------------------------ */
/* ggml_vec_dot_f16 (AVX2/F16C/FMA build): 4 x 8-wide f32 FMA accumulators    */
/* over 32-element steps, GGML_F32x8_REDUCE, leftovers in double.            */
/* ------------------------------------------------------------------------ */
static inline float dot_f16(int n, const uint16_t *x, const uint16_t *y) {
    if (__builtin_expect(g_dot_double, 0)) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += (double)h2f(x[i]) * (double)h2f(y[i]);
        return (float)s;
    }
    const int np = n & ~31;
    __m256 s0 = _mm256_setzero_ps(), s1 = _mm256_setzero_ps();
    __m256 s2 = _mm256_setzero_ps(), s3 = _mm256_setzero_ps();
    for (int i = 0; i < np; i += 32) {
        s0 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(x + i))),
                             _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(y + i))), s0);
        s1 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(x + i + 8))),
                             _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(y + i + 8))), s1);
        s2 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(x + i + 16))),
                             _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(y + i + 16))), s2);
        s3 = _mm256_fmadd_ps(_mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(x + i + 24))),
                             _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(y + i + 24))), s3);
    }
    s0 = _mm256_add_ps(s0, s1);
    s2 = _mm256_add_ps(s2, s3);
    s0 = _mm256_add_ps(s0, s2);
    __m128 t0 = _mm_add_ps(_mm256_castps256_ps128(s0), _mm256_extractf128_ps(s0, 1));
    __m128 t1 = _mm_hadd_ps(t0, t0);
    double sumf = _mm_cvtss_f32(_mm_hadd_ps(t1, t1));
    for (int i = np; i < n; ++i) sumf += (double)(h2f(x[i]) * h2f(y[i]));
    return (float)sumf;
}

/* ggml_vec_dot_f32 (same AVX2/FMA build): the f16 dot's accumulator layout
 * and reduction over f32 operands, neither rounded (f32 x f32 mul_mat of
 * ftype-0 files, main.rs:817-821) */
static inline float dot_f32(int n, const float *x, const float *y) {
    if (__builtin_expect(g_dot_double, 0)) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += (double)x[i] * (double)y[i];
        return (float)s;
    }
    const int np = n & ~31;
    __m256 s0 = _mm256_setzero_ps(), s1 = _mm256_setzero_ps();
    __m256 s2 = _mm256_setzero_ps(), s3 = _mm256_setzero_ps();
    for (int i = 0; i < np; i += 32) {
        s0 = _mm256_fmadd_ps(_mm256_loadu_ps(x + i), _mm256_loadu_ps(y + i), s0);
        s1 = _mm256_fmadd_ps(_mm256_loadu_ps(x + i + 8), _mm256_loadu_ps(y + i + 8), s1);
        s2 = _mm256_fmadd_ps(_mm256_loadu_ps(x + i + 16), _mm256_loadu_ps(y + i + 16), s2);
        s3 = _mm256_fmadd_ps(_mm256_loadu_ps(x + i + 24), _mm256_loadu_ps(y + i + 24), s3);
    }
    s0 = _mm256_add_ps(s0, s1);
    s2 = _mm256_add_ps(s2, s3);
    s0 = _mm256_add_ps(s0, s2);
    __m128 t0 = _mm_add_ps(_mm256_castps256_ps128(s0), _mm256_extractf128_ps(s0, 1));
    __m128 t1 = _mm_hadd_ps(t0, t0);
    double sumf = _mm_cvtss_f32(_mm_hadd_ps(t1, t1));
    for (int i = np; i < n; ++i) sumf += (double)(x[i] * y[i]);
    return (float)sumf;
}

/* ------------------------------------------------------------------------ */
/* model                                                                     */
/* ------------------------------------------------------------------------ */
typedef struct {
    float *attn_ln_w, *attn_ln_b;
    uint16_t *q_w; float *q_b;
    uint16_t *k_w;
    uint16_t *v_w; float *v_b;
    uint16_t *o_w; float *o_b;
    float *mlp_ln_w, *mlp_ln_b;
    uint16_t *mlp0_w; float *mlp0_b;
    uint16_t *mlp1_w; float *mlp1_b;
} enc_layer;

typedef struct {
    float *attn_ln_w, *attn_ln_b;
    uint16_t *q_w; float *q_b;
    uint16_t *k_w;
    uint16_t *v_w; float *v_b;
    uint16_t *o_w; float *o_b;
    float *cattn_ln_w, *cattn_ln_b;
    uint16_t *cq_w; float *cq_b;
    uint16_t *ck_w;
    uint16_t *cv_w; float *cv_b;
    uint16_t *co_w; float *co_b;
    float *mlp_ln_w, *mlp_ln_b;
    uint16_t *mlp0_w; float *mlp0_b;
    uint16_t *mlp1_w; float *mlp1_b;
} dec_layer;

enum { HP_N_VOCAB, HP_N_AUDIO_CTX, HP_N_AUDIO_STATE, HP_N_AUDIO_HEAD, HP_N_AUDIO_LAYER, HP_N_TEXT_CTX,
       HP_N_TEXT_STATE, HP_N_TEXT_HEAD, HP_N_TEXT_LAYER, HP_N_MELS, HP_F16 };

struct or_model {
    int32_t hp[11];
    int wf32; /* ftype 0 file: the uint16_t matrix pointers below address f32 arrays */
    int32_t n_filt_mel, n_filt_ff;
    float *filters;
    int32_t sp[9]; /* eot sot prev solm not beg translate transcribe multilingual */
    float *e_pe;
    uint16_t *conv1_w; float *conv1_b;
    uint16_t *conv2_w; float *conv2_b;
    float *ln_post_w, *ln_post_b;
    float *d_pe;
    uint16_t *d_te;
    float *d_ln_w, *d_ln_b;
    enc_layer *enc;
    dec_layer *dec;
    void **allocs;
    int n_allocs;
};

typedef struct {
    char name[96];
    int dtype; /* 0 f32, 1 f16 */
    int n_dims;
    int64_t ne[3];
    void **dst;
} reg_entry;

static void set_err(char *err, size_t cap, const char *fmt, ...) {
    if (!err || !cap) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err, cap, fmt, ap);
    va_end(ap);
}

static void *model_alloc(or_model *m, size_t bytes) {
    void *p = calloc(1, bytes ? bytes : 1);
    m->allocs = realloc(m->allocs, sizeof(void *) * (m->n_allocs + 1));
    m->allocs[m->n_allocs++] = p;
    return p;
}

void or_free(or_model *m) {
    if (!m) return;
    for (int i = 0; i < m->n_allocs; ++i) free(m->allocs[i]);
    free(m->allocs);
    free(m->enc);
    free(m->dec);
    free(m->filters);
    free(m);
}

static void reg_add(reg_entry *r, int *n, const char *name, int dtype, int n_dims, int64_t ne0, int64_t ne1,
                    int64_t ne2, void **dst) {
    reg_entry *e = &r[(*n)++];
    snprintf(e->name, sizeof(e->name), "%s", name);
    e->dtype = dtype;
    e->n_dims = n_dims;
    e->ne[0] = ne0;
    e->ne[1] = ne1;
    e->ne[2] = ne2;
    e->dst = dst;
}

/* ggml quantised blocks (QNT version 2 layouts; SURVEY.md §A.8 and §8f
 * item 2: the reference loader rejects them, main.rs:1423-1434).  Weights are
 * dequantised to f16 — w = f16(q * d (+ m)) rounded once, as a fused
 * multiply-add (exact in double here) — and every matmul then follows the f16
 * semantics (§A.4), as ggml's GPU back-ends do (dequantise -> f16 GEMM).  Types: 2 q4_0, 3 q4_1, 6 q5_0,
 * 7 q5_1, 8 q8_0; 32 weights per block. */
static int qblock_bytes(int t) {
    switch (t) {
        case 2: return 18;
        case 3: return 20;
        case 6: return 22;
        case 7: return 24;
        case 8: return 34;
        default: return 0;
    }
}

/* correctly rounded (RNE) double -> f16 */
static uint16_t d2h(double v) {
    uint64_t x;
    memcpy(&x, &v, 8);
    const uint32_t sign = (uint32_t)(x >> 48) & 0x8000u;
    x &= ~(1ull << 63);
    if (x >= 0x7ff0000000000000ull) return (uint16_t)(sign | 0x7c00u | (x > 0x7ff0000000000000ull ? 0x200u : 0u));
    if (x < 0x0010000000000000ull) return (uint16_t)sign;
    const int e = (int)(x >> 52) - 1023;
    const uint64_t mant = (x & ((1ull << 52) - 1)) | (1ull << 52);
    if (e >= 16) return (uint16_t)(sign | 0x7c00u);
    const int shift = e >= -14 ? 42 : 42 + (-14 - e);
    if (shift >= 63) return (uint16_t)sign;
    uint64_t q = mant >> shift;
    const uint64_t rem = mant & ((1ull << shift) - 1), half = 1ull << (shift - 1);
    if (rem > half || (rem == half && (q & 1))) ++q;
    if (e < -14) return (uint16_t)(sign | q);
    uint32_t ex = (uint32_t)(e + 15);
    if (q >> 11) { q >>= 1; ++ex; }
    if (ex >= 31) return (uint16_t)(sign | 0x7c00u);
    return (uint16_t)(sign | (ex << 10) | (uint32_t)(q & 0x3ffu));
}

static void dequant_row_f16(int t, const uint8_t *src, int64_t nel, uint16_t *dst) {
    const int bs = qblock_bytes(t);
    for (int64_t ib = 0; ib < nel / 32; ++ib) {
        const uint8_t *b = src + ib * bs;
        uint16_t *y = dst + ib * 32;
        uint16_t hd, hm;
        memcpy(&hd, b, 2);
        const float d = h2f(hd);
        if (t == 2) { /* q4_0: {d, qs[16]}, (nibble - 8) * d */
            for (int j = 0; j < 16; ++j) {
                y[j] = d2h((double)((b[2 + j] & 0x0F) - 8) * d);
                y[j + 16] = d2h((double)((b[2 + j] >> 4) - 8) * d);
            }
        } else if (t == 3) { /* q4_1: {d, m, qs[16]}, nibble * d + m */
            memcpy(&hm, b + 2, 2);
            const float m = h2f(hm);
            for (int j = 0; j < 16; ++j) {
                y[j] = d2h((double)(b[4 + j] & 0x0F) * d + (double)m);
                y[j + 16] = d2h((double)(b[4 + j] >> 4) * d + (double)m);
            }
        } else if (t == 6 || t == 7) { /* q5_0 {d, qh, qs} (q - 16) * d; q5_1 {d, m, qh, qs} q * d + m */
            const int o = t == 6 ? 2 : 4;
            float m = 0.0f;
            if (t == 7) { memcpy(&hm, b + 2, 2); m = h2f(hm); }
            uint32_t qh;
            memcpy(&qh, b + o, 4);
            const uint8_t *qs = b + o + 4;
            for (int j = 0; j < 16; ++j) {
                const int x0 = (qs[j] & 0x0F) | (((qh >> j) & 1) << 4);
                const int x1 = (qs[j] >> 4) | (((qh >> (j + 16)) & 1) << 4);
                if (t == 6) {
                    y[j] = d2h((double)(x0 - 16) * d);
                    y[j + 16] = d2h((double)(x1 - 16) * d);
                } else {
                    y[j] = d2h((double)x0 * d + (double)m);
                    y[j + 16] = d2h((double)x1 * d + (double)m);
                }
            }
        } else { /* q8_0: {d, int8 qs[32]} */
            for (int j = 0; j < 32; ++j) y[j] = d2h((double)(int8_t)b[2 + j] * d);
        }
    }
}

/* test hook: the loader's dequantisation of nel weights of ggml type t */
int or_dequant(int t, const uint8_t *src, int64_t nel, uint16_t *dst) {
    if (!qblock_bytes(t) || nel % 32) return WMI_E_INVALID_ARG;
    dequant_row_f16(t, src, nel, dst);
    return WMI_OK;
}

/* special token ids (main.rs:557-575) with the multilingual shift
 * (main.rs:433-440); large-v3 (n_vocab 51866, one more language) uses the
 * shift of later whisper.cpp. */
static void init_specials(int32_t n_vocab, int32_t sp[9]) {
    int32_t eot = 50256, sot = 50257, prev = 50360, solm = 50361, not_ = 50362, beg = 50363;
    int32_t translate = 50358, transcribe = 50359;
    const int multilingual = n_vocab >= 51865;
    if (multilingual) {
        const int dt = (n_vocab - 51765 - 1) - 98; /* languages beyond whisper v1/v2's 99 */
        eot += 1; sot += 1;
        prev += 1 + (dt > 1 ? dt - 1 : 0);
        solm += 1 + (dt > 1 ? dt - 1 : 0);
        not_ += 1 + (dt > 1 ? dt - 1 : 0);
        beg += 1 + (dt > 1 ? dt - 1 : 0);
        translate += (dt > 1 ? dt - 1 : 0);
        transcribe += (dt > 1 ? dt - 1 : 0);
    }
    sp[0] = eot; sp[1] = sot; sp[2] = prev; sp[3] = solm; sp[4] = not_; sp[5] = beg;
    sp[6] = translate; sp[7] = transcribe; sp[8] = multilingual;
}

int or_load(const char *path, or_model **out, char *err, size_t errcap) {
    pthread_once(&tables_once, init_tables);
    *out = NULL;
    FILE *f = fopen(path, "rb");
    if (!f) { set_err(err, errcap, "Unexpected IO: cannot open '%s'", path); return WMI_E_IO; }
    fseek(f, 0, SEEK_END);
    const long fsize = ftell(f);
    fseek(f, 0, SEEK_SET);
#define RD(ptr, bytes)                                                                     \
    do {                                                                                   \
        if (fread((ptr), 1, (bytes), f) != (size_t)(bytes)) {                              \
            set_err(err, errcap, "Unexpected IO: short read");                             \
            rc = WMI_E_IO;                                                                 \
            goto fail;                                                                     \
        }                                                                                  \
    } while (0)
    int rc = WMI_OK;
    or_model *m = calloc(1, sizeof(*m));
    reg_entry *reg = NULL;
    uint32_t magic = 0;
    RD(&magic, 4);
    if (magic != GGML_MAGIC) {
        set_err(err, errcap, "invalid model file '%s' (bad magic)", path);
        rc = WMI_E_BAD_MAGIC;
        goto fail;
    }
    RD(m->hp, 44);
    {
        const int32_t *hp = m->hp;
        for (int i = 0; i < 10; ++i)
            if (hp[i] <= 0) { set_err(err, errcap, "Unexpected: bad hparam %d", i); rc = WMI_E_UNEXPECTED; goto fail; }
        if (hp[HP_N_AUDIO_STATE] % hp[HP_N_AUDIO_HEAD] || hp[HP_N_TEXT_STATE] % hp[HP_N_TEXT_HEAD]) {
            set_err(err, errcap, "Unexpected: state not divisible by heads");
            rc = WMI_E_UNEXPECTED;
            goto fail;
        }
    }
    /* filters (main.rs:513-535) */
    RD(&m->n_filt_mel, 4);
    RD(&m->n_filt_ff, 4);
    if (m->n_filt_mel <= 0 || m->n_filt_ff <= 0 || (int64_t)m->n_filt_mel * m->n_filt_ff > (1 << 24)) {
        set_err(err, errcap, "Unexpected: bad filter dims");
        rc = WMI_E_UNEXPECTED;
        goto fail;
    }
    m->filters = malloc(sizeof(float) * m->n_filt_mel * m->n_filt_ff);
    RD(m->filters, sizeof(float) * m->n_filt_mel * m->n_filt_ff);
    /* vocab (main.rs:430, 578-592): skipped by the oracle */
    {
        int32_t nv = 0;
        RD(&nv, 4);
        for (int32_t i = 0; i < nv; ++i) {
            uint32_t len = 0;
            RD(&len, 4);
            if (fseek(f, len, SEEK_CUR) != 0) { set_err(err, errcap, "Unexpected IO: vocab"); rc = WMI_E_IO; goto fail; }
        }
    }
    init_specials(m->hp[HP_N_VOCAB], m->sp);

    /* tensor registry (main.rs:947-1334) */
    {
        const int32_t *hp = m->hp;
        const int64_t n = hp[HP_N_AUDIO_STATE], nt = hp[HP_N_TEXT_STATE];
        const int64_t La = hp[HP_N_AUDIO_LAYER], Lt = hp[HP_N_TEXT_LAYER];
        const int file_ftype = hp[HP_F16] % 1000; /* ggml ftype + 1000 * quantisation version */
        const int W = file_ftype == 0 ? 0 : 1;    /* matrices land as f16 (quantised ones dequantised) */
        const int cap = 16 + 15 * La + 24 * Lt;
        reg = calloc(cap, sizeof(reg_entry));
        int nr = 0;
        m->enc = calloc(La, sizeof(enc_layer));
        m->dec = calloc(Lt, sizeof(dec_layer));
        char nm[96];
        reg_add(reg, &nr, "encoder.positional_embedding", 0, 2, n, hp[HP_N_AUDIO_CTX], 1, (void **)&m->e_pe);
        reg_add(reg, &nr, "encoder.conv1.weight", W, 3, 3, hp[HP_N_MELS], n, (void **)&m->conv1_w);
        reg_add(reg, &nr, "encoder.conv1.bias", 0, 2, 1, n, 1, (void **)&m->conv1_b);
        reg_add(reg, &nr, "encoder.conv2.weight", W, 3, 3, n, n, (void **)&m->conv2_w);
        reg_add(reg, &nr, "encoder.conv2.bias", 0, 2, 1, n, 1, (void **)&m->conv2_b);
        reg_add(reg, &nr, "encoder.ln_post.weight", 0, 1, n, 1, 1, (void **)&m->ln_post_w);
        reg_add(reg, &nr, "encoder.ln_post.bias", 0, 1, n, 1, 1, (void **)&m->ln_post_b);
        for (int i = 0; i < La; ++i) {
            enc_layer *e = &m->enc[i];
#define EREG(suffix, dt, nd, a, b, field)                                  \
    snprintf(nm, sizeof(nm), "encoder.blocks.%d." suffix, i);              \
    reg_add(reg, &nr, nm, dt, nd, a, b, 1, (void **)&e->field)
            EREG("mlp_ln.weight", 0, 1, n, 1, mlp_ln_w);
            EREG("mlp_ln.bias", 0, 1, n, 1, mlp_ln_b);
            EREG("mlp.0.weight", W, 2, n, 4 * n, mlp0_w);
            EREG("mlp.0.bias", 0, 1, 4 * n, 1, mlp0_b);
            EREG("mlp.2.weight", W, 2, 4 * n, n, mlp1_w);
            EREG("mlp.2.bias", 0, 1, n, 1, mlp1_b);
            EREG("attn_ln.weight", 0, 1, n, 1, attn_ln_w);
            EREG("attn_ln.bias", 0, 1, n, 1, attn_ln_b);
            EREG("attn.query.weight", W, 2, n, n, q_w);
            EREG("attn.query.bias", 0, 1, n, 1, q_b);
            EREG("attn.key.weight", W, 2, n, n, k_w);
            EREG("attn.value.weight", W, 2, n, n, v_w);
            EREG("attn.value.bias", 0, 1, n, 1, v_b);
            EREG("attn.out.weight", W, 2, n, n, o_w);
            EREG("attn.out.bias", 0, 1, n, 1, o_b);
#undef EREG
        }
        reg_add(reg, &nr, "decoder.positional_embedding", 0, 2, nt, hp[HP_N_TEXT_CTX], 1, (void **)&m->d_pe);
        reg_add(reg, &nr, "decoder.token_embedding.weight", W, 2, nt, hp[HP_N_VOCAB], 1, (void **)&m->d_te);
        reg_add(reg, &nr, "decoder.ln.weight", 0, 1, nt, 1, 1, (void **)&m->d_ln_w);
        reg_add(reg, &nr, "decoder.ln.bias", 0, 1, nt, 1, 1, (void **)&m->d_ln_b);
        for (int i = 0; i < Lt; ++i) {
            dec_layer *d = &m->dec[i];
#define DREG(suffix, dt, nd, a, b, field)                                  \
    snprintf(nm, sizeof(nm), "decoder.blocks.%d." suffix, i);              \
    reg_add(reg, &nr, nm, dt, nd, a, b, 1, (void **)&d->field)
            DREG("mlp_ln.weight", 0, 1, nt, 1, mlp_ln_w);
            DREG("mlp_ln.bias", 0, 1, nt, 1, mlp_ln_b);
            DREG("mlp.0.weight", W, 2, nt, 4 * nt, mlp0_w);
            DREG("mlp.0.bias", 0, 1, 4 * nt, 1, mlp0_b);
            DREG("mlp.2.weight", W, 2, 4 * nt, nt, mlp1_w);
            DREG("mlp.2.bias", 0, 1, nt, 1, mlp1_b);
            DREG("attn_ln.weight", 0, 1, nt, 1, attn_ln_w);
            DREG("attn_ln.bias", 0, 1, nt, 1, attn_ln_b);
            DREG("attn.query.weight", W, 2, nt, nt, q_w);
            DREG("attn.query.bias", 0, 1, nt, 1, q_b);
            DREG("attn.key.weight", W, 2, nt, nt, k_w);
            DREG("attn.value.weight", W, 2, nt, nt, v_w);
            DREG("attn.value.bias", 0, 1, nt, 1, v_b);
            DREG("attn.out.weight", W, 2, nt, nt, o_w);
            DREG("attn.out.bias", 0, 1, nt, 1, o_b);
            DREG("cross_attn_ln.weight", 0, 1, nt, 1, cattn_ln_w);
            DREG("cross_attn_ln.bias", 0, 1, nt, 1, cattn_ln_b);
            DREG("cross_attn.query.weight", W, 2, nt, nt, cq_w);
            DREG("cross_attn.query.bias", 0, 1, nt, 1, cq_b);
            DREG("cross_attn.key.weight", W, 2, nt, nt, ck_w);
            DREG("cross_attn.value.weight", W, 2, nt, nt, cv_w);
            DREG("cross_attn.value.bias", 0, 1, nt, 1, cv_b);
            DREG("cross_attn.out.weight", W, 2, nt, nt, co_w);
            DREG("cross_attn.out.bias", 0, 1, nt, 1, co_b);
#undef DREG
        }
        /* every tensor exists (zero-filled) even if the file omits it, as
         * the reference's arena allocation does (main.rs:947-1334) */
        for (int i = 0; i < nr; ++i) {
            const int64_t ne = reg[i].ne[0] * reg[i].ne[1] * reg[i].ne[2];
            *reg[i].dst = model_alloc(m, (size_t)ne * (reg[i].dtype ? 2 : 4));
        }
        /* record loop (main.rs:1384-1475): until fewer than 12 bytes remain */
        for (;;) {
            const long pos = ftell(f);
            if (fsize - pos < 12) break;
            int32_t hdr[3];
            RD(hdr, 12);
            const int32_t n_dims = hdr[0], len = hdr[1], ftype = hdr[2];
            if (n_dims < 1 || n_dims > 3 || len <= 0 || len >= 95) {
                set_err(err, errcap, "Unexpected: bad tensor header (n_dims %d, name_len %d)", n_dims, len);
                rc = WMI_E_UNEXPECTED;
                goto fail;
            }
            int64_t ne[3] = {1, 1, 1}, nel = 1;
            for (int i = 0; i < n_dims; ++i) {
                int32_t v;
                RD(&v, 4);
                ne[i] = v;
                nel *= v;
            }
            char name[96] = {0};
            RD(name, len);
            reg_entry *e = NULL;
            for (int i = 0; i < nr; ++i)
                if (strcmp(reg[i].name, name) == 0) { e = &reg[i]; break; }
            if (!e) { set_err(err, errcap, "unknown tensor '%s' in model file", name); rc = WMI_E_UNKNOWN_TENSOR; goto fail; }
            const int64_t want = e->ne[0] * e->ne[1] * e->ne[2];
            if (want != nel) {
                set_err(err, errcap, "tensor %s has wrong size in model file, got:%lld, expected:%lld", name,
                        (long long)want, (long long)nel);
                rc = WMI_E_WRONG_SIZE;
                goto fail;
            }
            for (int i = 0; i < e->n_dims; ++i)
                if (e->ne[i] != ne[i]) {
                    set_err(err, errcap, "tensor %s has wrong shape in model file, got:[%lld, %lld, %lld], expected:[%lld, %lld, %lld]",
                            name, (long long)e->ne[0], (long long)e->ne[1], (long long)e->ne[2], (long long)ne[0],
                            (long long)ne[1], (long long)ne[2]);
                    rc = WMI_E_WRONG_SHAPE;
                    goto fail;
                }
            const int qb = (e->dtype == 1 && e->n_dims == 2 && ne[0] % 32 == 0) ? qblock_bytes(ftype) : 0;
            const int64_t file_bytes = qb ? nel / 32 * qb : nel * (ftype == 0 ? 4 : 2);
            const int64_t nbytes = want * (e->dtype ? 2 : 4);
            if (qb ? 0 : file_bytes != nbytes) {
                set_err(err, errcap, "tensor %s has wrong bytes in model file, got:%lld, expected:%lld", name,
                        (long long)nbytes, (long long)file_bytes);
                rc = WMI_E_WRONG_BYTES;
                goto fail;
            }
            if (qb) {
                uint8_t *raw = malloc((size_t)file_bytes);
                if (fread(raw, 1, (size_t)file_bytes, f) != (size_t)file_bytes) {
                    free(raw);
                    set_err(err, errcap, "Unexpected IO: short read");
                    rc = WMI_E_IO;
                    goto fail;
                }
                dequant_row_f16(ftype, raw, nel, (uint16_t *)*e->dst);
                free(raw);
            } else {
                RD(*e->dst, nbytes);
            }
        }
        {
            const int ft = hp[HP_F16] % 1000, qv = hp[HP_F16] / 1000;
            const int ok = ft == 0 || ft == 1 || ((ft == 2 || ft == 3 || ft == 7 || ft == 8 || ft == 9) && qv == 2);
            if (!ok) {
                set_err(err, errcap, "model ftype %d (hparams.f16 = %d) is not supported by this build", ft, hp[HP_F16]);
                rc = WMI_E_UNSUPPORTED;
                goto fail;
            }
        }
    }
    free(reg);
    fclose(f);
    m->wf32 = m->hp[HP_F16] % 1000 == 0;
    *out = m;
    return WMI_OK;
fail:
    free(reg);
    fclose(f);
    or_free(m);
    return rc;
#undef RD
}

void or_get_hparams(const or_model *m, int32_t hp[11]) { memcpy(hp, m->hp, sizeof(m->hp)); }
void or_special_tokens(const or_model *m, int32_t out[9]) { memcpy(out, m->sp, sizeof(m->sp)); }

int or_prompt(const or_model *m, int32_t *out) {
    int n = 0;
    out[n++] = m->sp[1];
    if (m->sp[8]) {
        out[n++] = m->sp[1] + 1; /* <|en|> */
        out[n++] = m->sp[7];     /* <|transcribe|> */
    }
    out[n++] = m->sp[4]; /* <|notimestamps|> */
    return n;
}

/* ------------------------------------------------------------------------ */
/* mel frontend: main.rs:1486-1671, same f32 operation order                */
/* ------------------------------------------------------------------------ */
#define PI_F 3.14159265358979323846264338327950288f /* std::f32::consts::PI */

typedef struct {
    float c400[200], s400[200], c200[100], s200[100], c100[50], s100[50], c50[25], s50[25];
    float dc[25 * 25], ds[25 * 25];
} fft_tw;

static fft_tw TW;
static pthread_once_t tw_once = PTHREAD_ONCE_INIT;

static void init_tw(void) {
    /* fft: theta = 2.0 * PI * (k as f32) / (n as f32)  (main.rs:1537) */
    for (int k = 0; k < 200; ++k) { float t = 2.0f * PI_F * (float)k / 400.0f; TW.c400[k] = cosf(t); TW.s400[k] = sinf(t); }
    for (int k = 0; k < 100; ++k) { float t = 2.0f * PI_F * (float)k / 200.0f; TW.c200[k] = cosf(t); TW.s200[k] = sinf(t); }
    for (int k = 0; k < 50; ++k) { float t = 2.0f * PI_F * (float)k / 100.0f; TW.c100[k] = cosf(t); TW.s100[k] = sinf(t); }
    for (int k = 0; k < 25; ++k) { float t = 2.0f * PI_F * (float)k / 50.0f; TW.c50[k] = cosf(t); TW.s50[k] = sinf(t); }
    /* dft: angle = 2.0 * PI * (k * n_val) as f32 / n as f32  (main.rs:1495) */
    for (int p = 0; p < 25 * 25; ++p) { float a = 2.0f * PI_F * (float)p / 25.0f; TW.dc[p] = cosf(a); TW.ds[p] = sinf(a); }
}

/* dft (main.rs:1487-1502) */
static void dft(const float *in, int n, float *out) {
    for (int k = 0; k < n; ++k) {
        float re = 0.0f, im = 0.0f;
        for (int j = 0; j < n; ++j) {
            float c, s;
            if (n == 25) { c = TW.dc[k * j]; s = TW.ds[k * j]; }
            else { float a = 2.0f * PI_F * (float)(k * j) / (float)n; c = cosf(a); s = sinf(a); }
            re += in[j] * c;
            im -= in[j] * s;
        }
        out[2 * k] = re;
        out[2 * k + 1] = im;
    }
}

/* fft (main.rs:1505-1551): recursive radix-2 DIT, odd n -> dft */
static void fft(const float *in, int n, float *out) {
    if (n == 1) { out[0] = in[0]; out[1] = 0.0f; return; }
    if (n % 2 == 1) { dft(in, n, out); return; }
    float even[NFFT / 2], odd[NFFT / 2], ef[NFFT], of[NFFT];
    for (int i = 0; i < n; ++i) {
        if (i % 2 == 0) even[i / 2] = in[i];
        else odd[i / 2] = in[i];
    }
    fft(even, n / 2, ef);
    fft(odd, n / 2, of);
    const float *cs = NULL, *sn = NULL;
    if (n == 400) { cs = TW.c400; sn = TW.s400; }
    else if (n == 200) { cs = TW.c200; sn = TW.s200; }
    else if (n == 100) { cs = TW.c100; sn = TW.s100; }
    else if (n == 50) { cs = TW.c50; sn = TW.s50; }
    for (int k = 0; k < n / 2; ++k) {
        float re, im;
        if (cs) { re = cs[k]; im = -sn[k]; }
        else { float t = 2.0f * PI_F * (float)k / (float)n; re = cosf(t); im = -sinf(t); }
        const float re_odd = of[2 * k], im_odd = of[2 * k + 1];
        out[2 * k] = ef[2 * k] + re * re_odd - im * im_odd;
        out[2 * k + 1] = ef[2 * k + 1] + re * im_odd + im * re_odd;
        out[2 * (k + n / 2)] = ef[2 * k] - re * re_odd + im * im_odd;
        out[2 * (k + n / 2) + 1] = ef[2 * k + 1] - re * im_odd - im * re_odd;
    }
}

/* log_mel_spectrogram's frames (main.rs:1575-1644): log10 mel before
 * clamp_and_normalize, [n_mels][n_len] */
static int mel_raw(const or_model *m, const float *pcm, size_t n_samples, int n_threads, float *mel, int64_t n_len) {
    pthread_once(&tw_once, init_tw);
    const int n_mel = m->hp[HP_N_MELS];
    const int n_ff = 1 + NFFT / 2; /* main.rs:1580, speed_up = false */
    if (m->n_filt_mel < n_mel || m->n_filt_mel * m->n_filt_ff < n_mel * n_ff) return WMI_E_UNEXPECTED;
    float hann[NFFT];
    for (int i = 0; i < NFFT; ++i) hann[i] = 0.5f * (1.0f - cosf((2.0f * PI_F * (float)i) / (float)NFFT));
    const float *filt = m->filters;
#pragma omp parallel for num_threads(n_threads) schedule(static)
    for (int64_t i = 0; i < n_len; ++i) {
        float fin[NFFT], fout[2 * NFFT];
        const int64_t off = i * HOP;
        for (int j = 0; j < NFFT; ++j) fin[j] = (off + j < (int64_t)n_samples) ? hann[j] * pcm[off + j] : 0.0f;
        fft(fin, NFFT, fout);
        for (int j = 0; j < NFFT; ++j) fout[j] = fout[2 * j] * fout[2 * j] + fout[2 * j + 1] * fout[2 * j + 1];
        for (int j = 1; j < NFFT / 2; ++j) fout[j] += fout[NFFT - j];
        for (int j = 0; j < n_mel; ++j) {
            float sum = 0.0f;
            for (int k = 0; k < n_ff; ++k) sum += fout[k] * filt[j * n_ff + k];
            if (sum < 1e-10f) sum = 1e-10f;
            mel[(int64_t)j * n_len + i] = log10f(sum);
        }
    }
    return WMI_OK;
}

/* clamp_and_normalize (main.rs:1654-1671) */
static void mel_norm(float *mel, int64_t tot) {
    double mmax = -1e20;
    for (int64_t i = 0; i < tot; ++i)
        if ((double)mel[i] > mmax) mmax = (double)mel[i];
    mmax -= 8.0;
    for (int64_t i = 0; i < tot; ++i) {
        if ((double)mel[i] < mmax) mel[i] = (float)mmax;
        mel[i] = (mel[i] + 4.0f) / 4.0f;
    }
}

int or_mel(const or_model *m, const float *pcm, size_t n_samples, int n_threads, float *mel, int32_t *n_len_out) {
    const int64_t n_len = (int64_t)(n_samples / HOP);
    *n_len_out = (int32_t)n_len;
    if (!mel) return WMI_OK;
    const int rc = mel_raw(m, pcm, n_samples, n_threads, mel, n_len);
    if (rc) return rc;
    mel_norm(mel, (int64_t)m->hp[HP_N_MELS] * n_len);
    return WMI_OK;
}

/* The reference's debug prints, each a sequential f32 sum (Rust
 * iter().sum() / a += loop): "_hann" main.rs:1571-1572, "y" of the samples
 * :1682-1686, "filters" :1688-1690, "x1" of the mel before
 * clamp_and_normalize :1645-1647, "y" of the encoder's mel window
 * :1819-1832 (for mel_offset, n_ctx). */
int or_checksums(const or_model *m, const float *pcm, size_t n_samples, int mel_offset, int n_ctx, int n_threads,
                 float out[5]) {
    const int n_mel = m->hp[HP_N_MELS];
    const int64_t n_len = (int64_t)(n_samples / HOP);
    float hs = 0.0f;
    for (int i = 0; i < NFFT; ++i) hs += 0.5f * (1.0f - cosf((2.0f * PI_F * (float)i) / (float)NFFT));
    float ps = 0.0f;
    for (size_t i = 0; i < n_samples; ++i) ps += pcm[i];
    float fs = 0.0f;
    for (int64_t i = 0; i < (int64_t)m->n_filt_mel * m->n_filt_ff; ++i) fs += m->filters[i];
    float *mel = (float *)malloc(sizeof(float) * (size_t)(n_mel * n_len + 1));
    if (!mel) return WMI_E_UNEXPECTED;
    int rc = mel_raw(m, pcm, n_samples, n_threads, mel, n_len);
    if (rc) { free(mel); return rc; }
    float xs = 0.0f;
    for (int64_t i = 0; i < (int64_t)n_mel * n_len; ++i) xs += mel[i];
    mel_norm(mel, (int64_t)n_mel * n_len);
    const int64_t i0 = mel_offset < n_len ? mel_offset : n_len;
    const int64_t i1 = mel_offset + 2 * (int64_t)n_ctx < n_len ? mel_offset + 2 * (int64_t)n_ctx : n_len;
    float ys = 0.0f;
    for (int j = 0; j < n_mel; ++j)
        for (int64_t c = 0; c < 2 * (int64_t)n_ctx; ++c) {
            const int64_t i = i0 + c;
            ys += i < i1 ? mel[(int64_t)j * n_len + i] : 0.0f;
        }
    free(mel);
    out[0] = hs; out[1] = ps; out[2] = fs; out[3] = xs; out[4] = ys;
    return WMI_OK;
}

/* ------------------------------------------------------------------------ */
/* tensor ops with ggml-1.0.3 semantics                                      */
/* ------------------------------------------------------------------------ */

/* ggml_compute_forward_norm_f32 + mul(repeat(w)) + add(repeat(b)):
 * y = b + w * ((x - mean) * scale) with mean/var accumulated in double. */
static void layer_norm_row(int n, const float *x, const float *w, const float *b, float *y) {
    double mean = 0.0;
    for (int i = 0; i < n; ++i) mean += x[i];
    mean /= n;
    double sum2 = 0.0;
    for (int i = 0; i < n; ++i) {
        const double v = x[i] - mean;
        y[i] = (float)v;
        sum2 += v * v;
    }
    const float scale = (float)(1.0 / sqrt(sum2 / n + 1e-5f));
    for (int i = 0; i < n; ++i) {
        const float t = y[i] * scale;
        y[i] = b[i] + w[i] * t;
    }
}

/* ggml_mul_mat(W f16 [N][K], x f32 [M][K]) with src1 rounded to f16:
 * y[t][o] = vec_dot_f16(W[o], f16(x[t])). x16 is the pre-rounded src1. */
static void matmul_f16(int M, int N, int K, const uint16_t *W, const uint16_t *x16, float *y, int nt) {
    const int OB = 16;
    const int nob = (N + OB - 1) / OB;
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1) collapse(2)
    for (int ob = 0; ob < nob; ++ob)
        for (int tb = 0; tb < (M + 63) / 64; ++tb) {
            const int o1 = (ob + 1) * OB < N ? (ob + 1) * OB : N;
            const int t1 = (tb + 1) * 64 < M ? (tb + 1) * 64 : M;
            for (int t = tb * 64; t < t1; ++t)
                for (int o = ob * OB; o < o1; ++o)
                    y[(int64_t)t * N + o] = dot_f16(K, W + (int64_t)o * K, x16 + (int64_t)t * K);
        }
}

/* ggml_mul_mat(W f32 [N][K], x f32 [M][K]): no rounding of either operand */
static void matmul_f32(int M, int N, int K, const float *W, const float *x, float *y, int nt) {
    const int OB = 16;
    const int nob = (N + OB - 1) / OB;
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1) collapse(2)
    for (int ob = 0; ob < nob; ++ob)
        for (int tb = 0; tb < (M + 63) / 64; ++tb) {
            const int o1 = (ob + 1) * OB < N ? (ob + 1) * OB : N;
            const int t1 = (tb + 1) * 64 < M ? (tb + 1) * 64 : M;
            for (int t = tb * 64; t < t1; ++t)
                for (int o = ob * OB; o < o1; ++o)
                    y[(int64_t)t * N + o] = dot_f32(K, W + (int64_t)o * K, x + (int64_t)t * K);
        }
}

static void to_f16(int64_t n, const float *x, uint16_t *y) {
    for (int64_t i = 0; i < n; ++i) y[i] = f2h(x[i]);
}

/* ggml_compute_forward_conv_1d_{1s,2s}_f16_f32: kernel W[o][c][3] (ggml ne
 * [3, C, O]); src X[c][t] (ne [Tin, C]); output y[o][t] for t < Tin/stride:
 * y = ((0 + v_0) + v_1) + v_2, v_k = vec_dot_f16(Cp, Wk[o][k], xs[t*stride + k])
 * where xs is the f16 time-major source zero-padded by one frame each side and
 * Cp = up32(C) channels (zero-padded, as ggml's ew0). */
static void conv1d(int C, int O, int Tin, int stride, const uint16_t *W, const uint16_t *xs_tm /*[Tin+2][Cp]*/,
                   float *y /*[O][Tout]*/, int nt) {
    const int Cp = (C + 31) & ~31;
    const int Tout = Tin / stride;
    uint16_t *wk = calloc((size_t)O * 3 * Cp, 2);
    for (int o = 0; o < O; ++o)
        for (int c = 0; c < C; ++c)
            for (int k = 0; k < 3; ++k) wk[((size_t)o * 3 + k) * Cp + c] = W[((size_t)o * C + c) * 3 + k];
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int o = 0; o < O; ++o)
        for (int t = 0; t < Tout; ++t) {
            float acc = 0.0f;
            for (int k = 0; k < 3; ++k)
                acc += dot_f16(Cp, wk + ((size_t)o * 3 + k) * Cp, xs_tm + (size_t)(t * stride + k) * Cp);
            y[(size_t)o * Tout + t] = acc;
        }
    free(wk);
}

/* ggml_compute_forward_conv_1d_{1s,2s}_f32: the same kernel / source layout
 * in f32 (ftype-0 files), ggml_vec_dot_f32 per tap */
static void conv1d_f32(int C, int O, int Tin, int stride, const float *W, const float *xs_tm /*[Tin+2][Cp]*/,
                       float *y /*[O][Tout]*/, int nt) {
    const int Cp = (C + 31) & ~31;
    const int Tout = Tin / stride;
    float *wk = calloc((size_t)O * 3 * Cp, 4);
    for (int o = 0; o < O; ++o)
        for (int c = 0; c < C; ++c)
            for (int k = 0; k < 3; ++k) wk[((size_t)o * 3 + k) * Cp + c] = W[((size_t)o * C + c) * 3 + k];
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int o = 0; o < O; ++o)
        for (int t = 0; t < Tout; ++t) {
            float acc = 0.0f;
            for (int k = 0; k < 3; ++k)
                acc += dot_f32(Cp, wk + ((size_t)o * 3 + k) * Cp, xs_tm + (size_t)(t * stride + k) * Cp);
            y[(size_t)o * Tout + t] = acc;
        }
    free(wk);
}

/* ggml_compute_forward_flash_attn_f16 (masked = false), per query row:
 * S = scale * vec_dot_f16(K_j, q); softmax with f16 exp table (sump[j%4] in
 * double, float sum); S16 = f16(S * (1/sum)); out[d] = vec_dot_f16(Vt[d], S16). */
static void flash_attn_row(int D, int M, const uint16_t *q, const uint16_t *K /*[M][ldk]*/, int ldk,
                           const uint16_t *Vt /*[D][ldv]*/, int ldv, float scale, float *S, uint16_t *S16, float *out) {
    const int Mup = (M + 3) & ~3;
    for (int j = 0; j < M; ++j) S[j] = dot_f16(D, K + (int64_t)j * ldk, q);
    for (int j = 0; j < M; ++j) S[j] *= scale;
    for (int j = M; j < Mup; ++j) S[j] = -INFINITY;
    float mx = -INFINITY;
    for (int j = 0; j < M; ++j) mx = S[j] > mx ? S[j] : mx;
    double sump[4] = {0, 0, 0, 0};
    for (int j = 0; j < Mup; ++j) {
        if (S[j] == -INFINITY) { S[j] = 0.0f; continue; }
        const float val = h2f(T_EXP[f2h(S[j] - mx)]);
        sump[j & 3] += val;
        S[j] = val;
    }
    float sum = 0.0f;
    for (int i = 0; i < 4; ++i) sum = (float)(sum + sump[i]);
    sum = (float)(1.0 / sum);
    for (int j = 0; j < M; ++j) S16[j] = f2h(S[j] * sum);
    for (int d = 0; d < D; ++d) out[d] = dot_f16(M, Vt + (int64_t)d * ldv, S16);
}

int or_encode(const or_model *m, const float *mel, int32_t n_len, int mel_offset, int n_ctx, int nt,
              float *enc_out, uint16_t *cross_k, uint16_t *cross_v, float *probe) {
    const int32_t *hp = m->hp;
    const int n = hp[HP_N_AUDIO_STATE], H = hp[HP_N_AUDIO_HEAD], D = n / H, L = hp[HP_N_AUDIO_LAYER];
    const int C = hp[HP_N_MELS];
    if (n_ctx <= 0) n_ctx = hp[HP_N_AUDIO_CTX];
    if (n_ctx > hp[HP_N_AUDIO_CTX] || mel_offset < 0) return WMI_E_INVALID_ARG;
    const int T2 = 2 * n_ctx, T = n_ctx;
    const int Cp = (C + 31) & ~31;

    /* f32 (ftype 0) files: f32 kernels / matrices, nothing rounded to f16
     * before a conv or matmul (ggml's *_f32 forward paths) */
    const int f32 = m->wf32;
    /* mel window (main.rs:1816-1833) -> f16 (f32) time-major padded conv input */
    uint16_t *xs = calloc((size_t)(T2 + 2) * Cp, 2);
    float *xs32 = f32 ? calloc((size_t)(T2 + 2) * Cp, 4) : NULL;
    {
        const int64_t i0 = mel_offset < n_len ? mel_offset : n_len;
        const int64_t i1 = (int64_t)mel_offset + T2 < n_len ? (int64_t)mel_offset + T2 : n_len;
        for (int c = 0; c < C; ++c)
            for (int64_t i = i0; i < i1; ++i) {
                const float v = mel[(int64_t)c * n_len + i];
                xs[(size_t)(i - i0 + 1) * Cp + c] = f2h(v);
                if (f32) xs32[(size_t)(i - i0 + 1) * Cp + c] = v;
            }
    }
    /* conv1 + bias + gelu (main.rs:1834-1855) */
    float *y1 = malloc(sizeof(float) * (size_t)n * T2);
    if (f32) conv1d_f32(C, n, T2, 1, (const float *)m->conv1_w, xs32, y1, nt);
    else conv1d(C, n, T2, 1, m->conv1_w, xs, y1, nt);
    free(xs);
    free(xs32);
    uint16_t *g1 = calloc((size_t)(T2 + 2) * n, 2);
    float *g1f = f32 ? calloc((size_t)(T2 + 2) * n, 4) : NULL; /* the same (f16 table) values in f32 */
    for (int o = 0; o < n; ++o)
        for (int t = 0; t < T2; ++t) {
            const float gv = gelu_f16(m->conv1_b[o] + y1[(size_t)o * T2 + t]);
            g1[(size_t)(t + 1) * n + o] = f2h(gv);
            if (f32) g1f[(size_t)(t + 1) * n + o] = gv;
        }
    free(y1);
    /* conv2 + bias + gelu (main.rs:1856-1860) */
    float *y2 = malloc(sizeof(float) * (size_t)n * T);
    if (f32) conv1d_f32(n, n, T2, 2, (const float *)m->conv2_w, g1f, y2, nt);
    else conv1d(n, n, T2, 2, m->conv2_w, g1, y2, nt);
    free(g1);
    free(g1f);
    /* + positional embedding, transposed (main.rs:1862-1875) */
    float *h = malloc(sizeof(float) * (size_t)T * n);
    for (int t = 0; t < T; ++t)
        for (int c = 0; c < n; ++c)
            h[(size_t)t * n + c] = m->e_pe[(size_t)t * n + c] + gelu_f16(m->conv2_b[c] + y2[(size_t)c * T + t]);
    free(y2);
    if (probe) memcpy(probe, h, sizeof(float) * (size_t)T * n);

    float *xln = malloc(sizeof(float) * (size_t)T * 4 * n);
    uint16_t *x16 = malloc(2 * (size_t)T * 4 * n);
    float *q = malloc(sizeof(float) * (size_t)T * n);
    float *k = malloc(sizeof(float) * (size_t)T * n);
    float *v = malloc(sizeof(float) * (size_t)T * n);
    uint16_t *q16 = malloc(2 * (size_t)T * n), *k16 = malloc(2 * (size_t)T * n), *vt16 = malloc(2 * (size_t)T * n);
    float *att = malloc(sizeof(float) * (size_t)T * n);
    float *y = malloc(sizeof(float) * (size_t)T * 4 * n);
    const float scale = (float)(1.0 / sqrt((double)D));

    for (int l = 0; l < L; ++l) {
        const enc_layer *e = &m->enc[l];
        /* attn_ln (main.rs:1881-1887) */
#pragma omp parallel for num_threads(nt)
        for (int t = 0; t < T; ++t) layer_norm_row(n, h + (size_t)t * n, e->attn_ln_w, e->attn_ln_b, xln + (size_t)t * n);
        /* Q, K, V (main.rs:1891-1897) */
        if (f32) {
            matmul_f32(T, n, n, (const float *)e->q_w, xln, q, nt);
            matmul_f32(T, n, n, (const float *)e->k_w, xln, k, nt);
            matmul_f32(T, n, n, (const float *)e->v_w, xln, v, nt);
        } else {
            to_f16((int64_t)T * n, xln, x16);
            matmul_f16(T, n, n, e->q_w, x16, q, nt);
            matmul_f16(T, n, n, e->k_w, x16, k, nt);
            matmul_f16(T, n, n, e->v_w, x16, v, nt);
        }
        for (int t = 0; t < T; ++t)
            for (int c = 0; c < n; ++c) {
                const size_t i = (size_t)t * n + c;
                q16[i] = f2h(e->q_b[c] + q[i]);
                k16[i] = f2h(k[i]);
                /* V -> f16 [h][d][t] (main.rs:1914-1920) */
                vt16[(size_t)(c / D) * D * T + (size_t)(c % D) * T + t] = f2h(e->v_b[c] + v[i]);
            }
        /* flash attention (main.rs:1922-1929) */
#pragma omp parallel num_threads(nt)
        {
            float *S = malloc(sizeof(float) * (T + 4));
            uint16_t *S16 = malloc(2 * (T + 4));
#pragma omp for collapse(2) schedule(static)
            for (int hh = 0; hh < H; ++hh)
                for (int t = 0; t < T; ++t)
                    flash_attn_row(D, T, q16 + (size_t)t * n + hh * D, k16 + hh * D, n, vt16 + (size_t)hh * D * T, T,
                                   scale, S, S16, att + (size_t)t * n + hh * D);
            free(S);
            free(S16);
        }
        /* out-projection + residual (main.rs:1935-1942) */
        if (f32) {
            matmul_f32(T, n, n, (const float *)e->o_w, att, y, nt);
        } else {
            to_f16((int64_t)T * n, att, x16);
            matmul_f16(T, n, n, e->o_w, x16, y, nt);
        }
        for (int t = 0; t < T; ++t)
            for (int c = 0; c < n; ++c) {
                const size_t i = (size_t)t * n + c;
                h[i] = (e->o_b[c] + y[i]) + h[i];
            }
        /* MLP (main.rs:1945-1968) */
#pragma omp parallel for num_threads(nt)
        for (int t = 0; t < T; ++t) layer_norm_row(n, h + (size_t)t * n, e->mlp_ln_w, e->mlp_ln_b, xln + (size_t)t * n);
        if (f32) {
            matmul_f32(T, 4 * n, n, (const float *)e->mlp0_w, xln, y, nt);
            for (size_t i = 0; i < (size_t)T * 4 * n; ++i) xln[i] = gelu_f16(e->mlp0_b[i % (4 * n)] + y[i]);
            matmul_f32(T, n, 4 * n, (const float *)e->mlp1_w, xln, y, nt);
        } else {
            to_f16((int64_t)T * n, xln, x16);
            matmul_f16(T, 4 * n, n, e->mlp0_w, x16, y, nt);
            for (int t = 0; t < T; ++t)
                for (int c = 0; c < 4 * n; ++c) {
                    const size_t i = (size_t)t * 4 * n + c;
                    x16[i] = f2h(gelu_f16(e->mlp0_b[c] + y[i]));
                }
            matmul_f16(T, n, 4 * n, e->mlp1_w, x16, y, nt);
        }
        for (int t = 0; t < T; ++t)
            for (int c = 0; c < n; ++c) {
                const size_t i = (size_t)t * n + c;
                h[i] = (e->mlp1_b[c] + y[i]) + h[i];
            }
        if (probe) memcpy(probe + (size_t)(l + 1) * T * n, h, sizeof(float) * (size_t)T * n);
    }
    /* ln_post (main.rs:1977-1986) */
#pragma omp parallel for num_threads(nt)
    for (int t = 0; t < T; ++t) layer_norm_row(n, h + (size_t)t * n, m->ln_post_w, m->ln_post_b, enc_out + (size_t)t * n);

    /* cross-attention K/V (main.rs:1990-2060) */
    {
        const int Lt = hp[HP_N_TEXT_LAYER], nt_state = hp[HP_N_TEXT_STATE];
        if (nt_state != n) return WMI_E_UNSUPPORTED;
        const float kscale = powf((float)n / (float)H, -0.25f);
        to_f16((int64_t)T * n, enc_out, x16);
        for (int l = 0; l < Lt; ++l) {
            const dec_layer *d = &m->dec[l];
            if (f32) {
                matmul_f32(T, n, n, (const float *)d->ck_w, enc_out, k, nt);
                matmul_f32(T, n, n, (const float *)d->cv_w, enc_out, v, nt);
            } else {
                matmul_f16(T, n, n, d->ck_w, x16, k, nt);
                matmul_f16(T, n, n, d->cv_w, x16, v, nt);
            }
            uint16_t *ko = cross_k + (size_t)l * T * n, *vo = cross_v + (size_t)l * T * n;
            for (int t = 0; t < T; ++t)
                for (int c = 0; c < n; ++c) {
                    const size_t i = (size_t)t * n + c;
                    ko[i] = f2h(k[i] * kscale);
                    vo[i] = f2h(d->cv_b[c] + v[i]);
                }
        }
    }
    free(h); free(xln); free(x16); free(q); free(k); free(v);
    free(q16); free(k16); free(vt16); free(att); free(y);
    return WMI_OK;
}

/* ------------------------------------------------------------------------ */
/* decoder (whisper.cpp-1.0.3 whisper_decode semantics)         */
/* ------------------------------------------------------------------------ */
typedef struct {
    int n, H, D, L, V, n_text_ctx;
    uint16_t *mk, *mv; /* [L][n_text_ctx][n] f16 */
    float *x, *xl, *buf, *att, *logits_tmp;
    uint16_t *x16, *h16;
    float *h32; /* f32 files: the MLP hidden row (GELU table values) */
    float *S;
    uint16_t *S16, *vcol;
} dec_state;

/* ggml_compute_forward_soft_max_f32 (table exp, double sum) -> f16 probs */
static void softmax_to_f16(int M, float *S, uint16_t *S16) {
    float mx = -INFINITY;
    for (int j = 0; j < M; ++j) mx = S[j] > mx ? S[j] : mx;
    double sum = 0.0;
    for (int j = 0; j < M; ++j) {
        const float val = h2f(T_EXP[f2h(S[j] - mx)]);
        sum += (double)val;
        S[j] = val;
    }
    const float inv = (float)(1.0 / sum);
    for (int j = 0; j < M; ++j) S16[j] = f2h(S[j] * inv);
}

/* one head: scores over M keys K[j][ldk] (pre-scaled f16), probs, out over V[j][ldv] */
static void dec_attn_head(int D, int M, const uint16_t *q16, const uint16_t *K, const uint16_t *V, int ld, dec_state *st,
                          float *out) {
    for (int j = 0; j < M; ++j) st->S[j] = dot_f16(D, K + (int64_t)j * ld, q16);
    softmax_to_f16(M, st->S, st->S16);
    for (int d = 0; d < D; ++d) {
        for (int j = 0; j < M; ++j) st->vcol[j] = V[(int64_t)j * ld + d];
        out[d] = dot_f16(M, st->vcol, st->S16);
    }
}

static void gemv_f16(int N, int K, const uint16_t *W, const uint16_t *x16, float *y, int nt) {
#pragma omp parallel for num_threads(nt) schedule(static)
    for (int o = 0; o < N; ++o) y[o] = dot_f16(K, W + (int64_t)o * K, x16);
}

/* y = W x for the model's matrix type: f16 rows against f16(x) (x16 is
 * filled here), or f32 rows against x unrounded (ftype-0 files) */
static void gemv_w(const or_model *m, int N, int K, const uint16_t *W, const float *x, uint16_t *x16, float *y, int nt) {
    if (m->wf32) {
        const float *W32 = (const float *)W;
#pragma omp parallel for num_threads(nt) schedule(static)
        for (int o = 0; o < N; ++o) y[o] = dot_f32(K, W32 + (int64_t)o * K, x);
        return;
    }
    to_f16(K, x, x16);
    gemv_f16(N, K, W, x16, y, nt);
}

static void dec_step(const or_model *m, dec_state *st, const uint16_t *cross_k, const uint16_t *cross_v, int n_ctx,
                     int32_t tok, int pos, float *logits, int nt) {
    const int n = st->n, H = st->H, D = st->D;
    const float sc = powf((float)n / (float)H, -0.25f);
    float *x = st->x, *xl = st->xl, *buf = st->buf, *att = st->att;
    for (int c = 0; c < n; ++c) {
        const float te = m->wf32 ? ((const float *)m->d_te)[(int64_t)tok * n + c] : h2f(m->d_te[(int64_t)tok * n + c]);
        x[c] = te + m->d_pe[(int64_t)pos * n + c];
    }
    for (int l = 0; l < st->L; ++l) {
        const dec_layer *d = &m->dec[l];
        uint16_t *mk = st->mk + (size_t)l * st->n_text_ctx * n, *mv = st->mv + (size_t)l * st->n_text_ctx * n;
        /* self-attention */
        layer_norm_row(n, x, d->attn_ln_w, d->attn_ln_b, xl);
        gemv_w(m, n, n, d->q_w, xl, st->x16, buf, nt);
        for (int c = 0; c < n; ++c) st->h16[c] = f2h((d->q_b[c] + buf[c]) * sc);
        gemv_w(m, n, n, d->k_w, xl, st->x16, buf, nt);
        for (int c = 0; c < n; ++c) mk[(size_t)pos * n + c] = f2h(buf[c] * sc);
        gemv_w(m, n, n, d->v_w, xl, st->x16, buf, nt);
        for (int c = 0; c < n; ++c) mv[(size_t)pos * n + c] = f2h(d->v_b[c] + buf[c]);
        for (int hh = 0; hh < H; ++hh) dec_attn_head(D, pos + 1, st->h16 + hh * D, mk + hh * D, mv + hh * D, n, st, att + hh * D);
        gemv_w(m, n, n, d->o_w, att, st->x16, buf, nt);
        for (int c = 0; c < n; ++c) x[c] = (d->o_b[c] + buf[c]) + x[c];
        /* cross-attention over memory_cross_k/v[l] */
        layer_norm_row(n, x, d->cattn_ln_w, d->cattn_ln_b, xl);
        gemv_w(m, n, n, d->cq_w, xl, st->x16, buf, nt);
        for (int c = 0; c < n; ++c) st->h16[c] = f2h((d->cq_b[c] + buf[c]) * sc);
        const uint16_t *ck = cross_k + (size_t)l * n_ctx * n, *cv = cross_v + (size_t)l * n_ctx * n;
        for (int hh = 0; hh < H; ++hh) dec_attn_head(D, n_ctx, st->h16 + hh * D, ck + hh * D, cv + hh * D, n, st, att + hh * D);
        gemv_w(m, n, n, d->co_w, att, st->x16, buf, nt);
        for (int c = 0; c < n; ++c) x[c] = (d->co_b[c] + buf[c]) + x[c];
        /* MLP */
        layer_norm_row(n, x, d->mlp_ln_w, d->mlp_ln_b, xl);
        gemv_w(m, 4 * n, n, d->mlp0_w, xl, st->x16, buf, nt);
        for (int c = 0; c < 4 * n; ++c) st->h32[c] = gelu_f16(d->mlp0_b[c] + buf[c]);
        gemv_w(m, n, 4 * n, d->mlp1_w, st->h32, st->x16, buf, nt);
        for (int c = 0; c < n; ++c) x[c] = (d->mlp1_b[c] + buf[c]) + x[c];
    }
    layer_norm_row(n, x, m->d_ln_w, m->d_ln_b, xl);
    gemv_w(m, st->V, n, m->d_te, xl, st->x16, logits, nt);
}

static int dec_init(const or_model *m, dec_state *st, int n_ctx) {
    const int32_t *hp = m->hp;
    memset(st, 0, sizeof(*st));
    st->n = hp[HP_N_TEXT_STATE];
    st->H = hp[HP_N_TEXT_HEAD];
    st->D = st->n / st->H;
    st->L = hp[HP_N_TEXT_LAYER];
    st->V = hp[HP_N_VOCAB];
    st->n_text_ctx = hp[HP_N_TEXT_CTX];
    const int n = st->n;
    const int maxM = (n_ctx > st->n_text_ctx ? n_ctx : st->n_text_ctx) + 8;
    st->mk = calloc((size_t)st->L * st->n_text_ctx * n, 2);
    st->mv = calloc((size_t)st->L * st->n_text_ctx * n, 2);
    st->x = malloc(sizeof(float) * n);
    st->xl = malloc(sizeof(float) * n);
    st->buf = malloc(sizeof(float) * 4 * n);
    st->att = malloc(sizeof(float) * n);
    st->h32 = malloc(sizeof(float) * 4 * n);
    st->x16 = malloc(2 * 4 * n);
    st->h16 = malloc(2 * n);
    st->S = malloc(sizeof(float) * maxM);
    st->S16 = malloc(2 * maxM);
    st->vcol = malloc(2 * maxM);
    return WMI_OK;
}

static void dec_fini(dec_state *st) {
    free(st->mk); free(st->mv); free(st->x); free(st->xl); free(st->buf); free(st->att);
    free(st->x16); free(st->h16); free(st->h32); free(st->S); free(st->S16); free(st->vcol);
}

int or_decode_logits(const or_model *m, const uint16_t *cross_k, const uint16_t *cross_v, int n_ctx,
                     const int32_t *tokens, int n_tokens, int nt, float *logits) {
    if (n_tokens > m->hp[HP_N_TEXT_CTX]) return WMI_E_INVALID_ARG;
    if (n_ctx <= 0) n_ctx = m->hp[HP_N_AUDIO_CTX];
    dec_state st;
    dec_init(m, &st, n_ctx);
    for (int i = 0; i < n_tokens; ++i) {
        if (tokens[i] < 0 || tokens[i] >= st.V) { dec_fini(&st); return WMI_E_INVALID_ARG; }
        dec_step(m, &st, cross_k, cross_v, n_ctx, tokens[i], i, logits + (size_t)i * st.V, nt);
    }
    dec_fini(&st);
    return WMI_OK;
}

int or_decode_greedy(const or_model *m, const uint16_t *cross_k, const uint16_t *cross_v, int n_ctx, int max_tokens,
                     int suppress_eot, int nt, int32_t *tokens_out, int32_t *n_out, float *margins) {
    if (n_ctx <= 0) n_ctx = m->hp[HP_N_AUDIO_CTX];
    int32_t prompt[8];
    const int np = or_prompt(m, prompt);
    if (np + max_tokens > m->hp[HP_N_TEXT_CTX]) return WMI_E_INVALID_ARG;
    dec_state st;
    dec_init(m, &st, n_ctx);
    float *lg = malloc(sizeof(float) * st.V);
    const int eot = m->sp[0];
    int32_t tok = prompt[0];
    int pos = 0, produced = 0;
    for (; pos < np - 1; ++pos) dec_step(m, &st, cross_k, cross_v, n_ctx, prompt[pos], pos, lg, nt);
    tok = prompt[np - 1];
    while (produced < max_tokens) {
        dec_step(m, &st, cross_k, cross_v, n_ctx, tok, pos, lg, nt);
        ++pos;
        if (suppress_eot) lg[eot] = -INFINITY;
        int best = 0;
        float b1 = -INFINITY, b2 = -INFINITY;
        for (int v = 0; v < st.V; ++v) {
            if (lg[v] > b1) { b2 = b1; b1 = lg[v]; best = v; }
            else if (lg[v] > b2) b2 = lg[v];
        }
        tokens_out[produced] = best;
        if (margins) margins[produced] = b1 - b2;
        ++produced;
        tok = best;
        if (!suppress_eot && best == eot) break;
    }
    *n_out = produced;
    free(lg);
    dec_fini(&st);
    return WMI_OK;
}

/* ------------------------------------------------------------------------ */
/* beam search (config C5).  Absent from the reference and from whisper.cpp  */
/* 1.0.3; the semantics are defined in wmi_oracle.h (after OpenAI whisper's  */
/* BeamSearchDecoder without length penalty) and restated by the HIP path.   */
/* ------------------------------------------------------------------------ */
typedef struct {
    double score;
    int beam, rank, id;
} beam_cand;

/* (score desc, beam asc, rank asc): a stable sort of beam-major, top-k-order insertion by score */
static int cand_before(const beam_cand *a, const beam_cand *b) {
    if (a->score != b->score) return a->score > b->score;
    if (a->beam != b->beam) return a->beam < b->beam;
    return a->rank < b->rank;
}

/* top k of lg[0..V) by (value desc, id asc) */
static void topk_row(const float *lg, int V, int k, int *ids) {
    for (int i = 0; i < k; ++i) ids[i] = -1;
    for (int v = 0; v < V; ++v) {
        const float x = lg[v];
        int p = k;
        while (p > 0 && (ids[p - 1] < 0 || x > lg[ids[p - 1]])) --p;
        if (p == k) continue;
        for (int j = k - 1; j > p; --j) ids[j] = ids[j - 1];
        ids[p] = v;
    }
}

static double row_lse(const float *lg, int V) {
    float mx = -INFINITY;
    for (int v = 0; v < V; ++v) mx = lg[v] > mx ? lg[v] : mx;
    double s = 0.0;
    for (int v = 0; v < V; ++v) s += exp((double)lg[v] - (double)mx);
    return (double)mx + log(s);
}

int or_decode_beam(const or_model *m, const uint16_t *cross_k, const uint16_t *cross_v, int n_ctx, int beam,
                   int max_tokens, int suppress_eot, int nt, int32_t *tokens_out, int32_t *n_out, double *score_out,
                   float *min_gap, float *step_gap, float *step_logits, int32_t *step_sel) {
    if (n_ctx <= 0) n_ctx = m->hp[HP_N_AUDIO_CTX];
    if (beam < 1 || beam > 8 || max_tokens < 1) return WMI_E_INVALID_ARG;
    int32_t prompt[8];
    const int np = or_prompt(m, prompt);
    if (np + max_tokens > m->hp[HP_N_TEXT_CTX]) return WMI_E_INVALID_ARG;
    const int K = beam, eot = m->sp[0];
    dec_state *st = calloc(2 * K, sizeof(dec_state));
    for (int i = 0; i < 2 * K; ++i) dec_init(m, &st[i], n_ctx);
    dec_state *cur = st, *nxt = st + K;
    const int V = st[0].V, n = st[0].n, L = st[0].L, tctx = st[0].n_text_ctx;
    float *lg = malloc(sizeof(float) * V * K);
    int32_t *hist = calloc((size_t)K * max_tokens, 4), *nhist = calloc((size_t)K * max_tokens, 4);
    int32_t *fin_tok = calloc((size_t)K * (max_tokens + 1), 4);
    int fin_len[8], n_fin = 0;
    double fin_score[8], score[8], nscore[8];
    int32_t tok[8], ntok[8], parent[8];
    beam_cand *cands = malloc(sizeof(beam_cand) * K * (K + 1));
    float gap = INFINITY;
    int pos = 0;
    for (; pos < np - 1; ++pos) dec_step(m, &cur[0], cross_k, cross_v, n_ctx, prompt[pos], pos, lg, nt);
    int n_active = 1, t = 0;
    tok[0] = prompt[np - 1];
    score[0] = 0.0;
    if (step_gap)
        for (int i = 0; i < max_tokens; ++i) step_gap[i] = INFINITY;
    for (t = 0; t < max_tokens && n_fin < K; ++t, ++pos) {
        int nc = 0;
        for (int b = 0; b < n_active; ++b) {
            float *row = lg + (size_t)b * V;
            dec_step(m, &cur[b], cross_k, cross_v, n_ctx, tok[b], pos, row, nt);
            if (step_logits) memcpy(step_logits + ((size_t)t * K + b) * V, row, sizeof(float) * V);
            if (suppress_eot) row[eot] = -INFINITY;
            const double lse = row_lse(row, V);
            int ids[9];
            topk_row(row, V, K + 1, ids);
            for (int r = 0; r <= K; ++r) {
                cands[nc].score = score[b] + ((double)row[ids[r]] - lse);
                cands[nc].beam = b;
                cands[nc].rank = r;
                cands[nc].id = ids[r];
                ++nc;
            }
        }
        /* insertion sort by the ranking key (nc <= 72) */
        for (int i = 1; i < nc; ++i) {
            beam_cand c = cands[i];
            int j = i;
            while (j > 0 && cand_before(&c, &cands[j - 1])) { cands[j] = cands[j - 1]; --j; }
            cands[j] = c;
        }
        int na = 0, i = 0;
        for (; i < nc && na < K; ++i) {
            const beam_cand *c = &cands[i];
            if (c->id == eot) {
                if (n_fin < K) {
                    memcpy(fin_tok + (size_t)n_fin * (max_tokens + 1), hist + (size_t)c->beam * max_tokens, 4 * t);
                    fin_tok[(size_t)n_fin * (max_tokens + 1) + t] = eot;
                    fin_len[n_fin] = t;
                    fin_score[n_fin] = c->score;
                    ++n_fin;
                }
                continue;
            }
            parent[na] = c->beam;
            ntok[na] = c->id;
            nscore[na] = c->score;
            ++na;
        }
        /* selection margin: last kept active vs the next non-EOT candidate */
        for (; i < nc; ++i)
            if (cands[i].id != eot) {
                const float g = (float)(nscore[na - 1] - cands[i].score);
                gap = g < gap ? g : gap;
                if (step_gap) step_gap[t] = g;
                break;
            }
        for (int s = 0; s < na && step_sel; ++s) {
            step_sel[((size_t)t * K + s) * 2] = parent[s];
            step_sel[((size_t)t * K + s) * 2 + 1] = ntok[s];
        }
        for (int s = 0; s < na; ++s) {
            const int p = parent[s];
            memcpy(nhist + (size_t)s * max_tokens, hist + (size_t)p * max_tokens, 4 * t);
            nhist[(size_t)s * max_tokens + t] = ntok[s];
            for (int l = 0; l < L; ++l) {
                const size_t off = (size_t)l * tctx * n;
                memcpy(nxt[s].mk + off, cur[p].mk + off, (size_t)(pos + 1) * n * 2);
                memcpy(nxt[s].mv + off, cur[p].mv + off, (size_t)(pos + 1) * n * 2);
            }
            tok[s] = ntok[s];
            score[s] = nscore[s];
        }
        dec_state *tmp = cur; cur = nxt; nxt = tmp;
        int32_t *th = hist; hist = nhist; nhist = th;
        n_active = na;
    }
    /* final ranking: finished first (in order), then active in slot order, up to K */
    int best_src = -1, best_i = 0;
    double best = -INFINITY, second = -INFINITY;
    int considered = 0;
    for (int f = 0; f < n_fin && considered < K; ++f, ++considered) {
        const double sc = fin_score[f] / (double)(fin_len[f] > 0 ? fin_len[f] : 1);
        if (sc > best) { second = best; best = sc; best_src = 0; best_i = f; }
        else if (sc > second) second = sc;
    }
    for (int s = 0; s < n_active && considered < K; ++s, ++considered) {
        const double sc = score[s] / (double)(t > 0 ? t : 1);
        if (sc > best) { second = best; best = sc; best_src = 1; best_i = s; }
        else if (sc > second) second = sc;
    }
    int nout;
    if (best_src == 0) {
        nout = fin_len[best_i] + 1;
        memcpy(tokens_out, fin_tok + (size_t)best_i * (max_tokens + 1), 4 * nout);
        if (score_out) *score_out = fin_score[best_i];
    } else {
        nout = t;
        memcpy(tokens_out, hist + (size_t)best_i * max_tokens, 4 * nout);
        if (score_out) *score_out = score[best_i];
    }
    if (isfinite(second)) {
        const float g = (float)(best - second);
        gap = g < gap ? g : gap;
    }
    *n_out = nout;
    if (min_gap) *min_gap = gap;
    for (int i = 0; i < 2 * K; ++i) dec_fini(&st[i]);
    free(st); free(lg); free(hist); free(nhist); free(fin_tok); free(cands);
    return WMI_OK;
}

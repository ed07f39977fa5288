// wmi_kernels.hip — gfx950 (CDNA4) kernels for the Whisper hot path.
//
// Numerics follow the restated reference path (oracle/wmi_oracle.c):
//   * mel: main.rs:1486-1671 operation for operation (f32, unfused), so the
//     frontend matches the CPU restatement bit for bit except where the
//     device log10f differs from glibc's by an ulp;
//   * tensor ops: ggml-1.0.3 rounding points — activations
//     rounded to f16 before every matmul/conv (free: MFMA takes f16),
//     f32 accumulation, f16 GELU/exp lookup tables (uploaded from the host,
//     so the device uses the exact table values), double-accumulated norm,
//     and the flash-attn softmax computed EXACTLY as ggml does (true row max,
//     table exp of f16(s - max), normalise, round to f16, then P·V), which
//     takes three passes over the keys instead of an online softmax.
//
// f32 multiply/add stay separately rounded (no FMA contraction) everywhere a
// reference operation is restated; MFMA and the dot-product accumulations
// are the only places where the summation order differs from the CPU.
#include <utility>
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "wmi_device.h"
#include "wmi_internal.h"
#include "wmi_gemm_epi.h"

#pragma clang fp contract(off)

namespace wmi {


static inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// dynamic LDS above 64 KiB must be opted into per kernel (gfx950 has 160 KiB)
template <typename K>
static hipError_t allow_lds(K *kern, size_t bytes) {
    if (bytes <= 65536) return hipSuccess;
    return hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// ============================================================================
// launch-overhead probes (wmi_bench_kernel 4 / 5)
// ============================================================================
__global__ void k_selftest_exp(const uint16_t *tab, int n_exp, uint32_t *mismatch) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > 0x7c00) return;
    const float x = h2f_bits((uint16_t)(0x8000u | (uint32_t)j));
    const uint16_t got = f2h_bits(exp_f16_exact(x));
    const uint16_t want = j < n_exp ? tab[j] : (uint16_t)0;
    if (got != want) atomicAdd(mismatch, 1u);
}
hipError_t launch_selftest(hipStream_t s, const uint16_t *exp_tab, int n_exp, uint32_t *mismatch) {
    hipLaunchKernelGGL(k_selftest_exp, dim3(cdiv(0x7c01, 256)), dim3(256), 0, s, exp_tab, n_exp, mismatch);
    return hipGetLastError();
}


// ============================================================================
// mel frontend
// ============================================================================
constexpr int MEL_WAVES = 4;
constexpr int MEL_FPW = 2;  // frames per wave
constexpr int MEL_SCRATCH = 2000;  // floats per wave: fin[400], A[800], B[800]

struct cpx {
    float re, im;
};

// one radix-2 combine level of fft (main.rs:1536-1550) for all sub-arrays:
// out sub-array s (size n) = combine(E = in[s], O = in[s + nsub]) where the
// input holds 2*nsub sub-arrays of size n/2.
__device__ __forceinline__ void fft_level(const cpx *in, cpx *out, int n, int nsub, const float *cs, const float *sn,
                                          int lane) {
    const int half = n / 2;
    for (int task = lane; task < nsub * half; task += 64) {
        const int s = task / half, k = task - s * half;
        const cpx E = in[s * half + k], O = in[(s + nsub) * half + k];
        const float re = cs[k], im = -sn[k];
        cpx a, b;
        a.re = E.re + re * O.re - im * O.im;
        a.im = E.im + re * O.im + im * O.re;
        b.re = E.re - re * O.re + im * O.im;
        b.im = E.im - re * O.im - im * O.re;
        out[s * n + k] = a;
        out[s * n + k + half] = b;
    }
}

// MW waves of FPW frames per workgroup; FG: the compact filterbank (each
// mel's non-zero weights, wmi_api.cpp filt_c) in LDS instead of the [201][C]
// copy, so two workgroups of eight one-frame waves fit a CU instead of one of
// four two-frame waves; the same terms in the same order (bitwise equal)
template <int MW, int FPW, bool FG>
__global__ __launch_bounds__(64 * MW) void k_mel_frames(const MelTables *__restrict__ tabs_g, const float *__restrict__ filt_t,
                                                    int n_mel, const float *const *pcm, const int64_t *n_samples,
                                                    float *mel, int64_t mel_stride, const int64_t *n_len,
                                                    uint32_t *mel_max, int n_fc) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int b = blockIdx.y;
    const int64_t nl = n_len[b];
    const int64_t frame0 = (int64_t)blockIdx.x * (MW * FPW);
    if (frame0 >= nl) return;
    MelTables *tabs = (MelTables *)sm;
    float *F = sm + sizeof(MelTables) / 4;
    const int nfc = FG ? n_fc : 203 * n_mel;  // floats of the bank's LDS copy
    float *scratch = F + ((nfc + 3) & ~3);
    {
        // tables + filterbank (~74 KB at 80 mels) -> LDS in 16-byte chunks,
        // eight requests in flight per thread before the first store (a
        // one-load-per-iteration copy loop waited one round trip per chunk)
        const float4 *s1 = (const float4 *)tabs_g, *s2 = (const float4 *)filt_t;
        float4 *dst = (float4 *)tabs;  // tabs, then F (contiguous)
        const int n1 = (int)(sizeof(MelTables) / 16), n2 = nfc / 4, nt = n1 + n2;  // + the ranges
        for (int base = threadIdx.x; base < nt; base += 64 * MW * 8) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = base + 64 * MW * u;
                const int ic = i < nt ? i : nt - 1;
                v[u] = ic < n1 ? s1[ic] : s2[ic - n1];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (base + 64 * MW * u < nt) dst[base + 64 * MW * u] = v[u];
        }
        for (int i = 4 * n2 + (int)threadIdx.x; i < nfc; i += 64 * MW) F[i] = filt_t[i];  // (a size % 4 != 0)
    }
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float *fin = scratch + w * MEL_SCRATCH;
    cpx *A = (cpx *)(fin + 400);
    cpx *Bf = (cpx *)(fin + 1200);
    const float *x = pcm[b];
    const int64_t ns = n_samples[b];
    float lmax = -INFINITY;
    float *melb = mel + (int64_t)b * mel_stride;
    for (int f = 0; f < FPW; ++f) {
        const int64_t i = frame0 + w * FPW + f;
        if (i >= nl) break;
        const int64_t off = i * 160;
        // window, zero past the end (main.rs:1594-1601)
        for (int j = lane; j < 400; j += 64) fin[j] = (off + j < ns) ? tabs->hann[j] * x[off + j] : 0.0f;
        wave_sync();
        // 16 DFT-25 leaves: residue r = in[r + 16 j] (main.rs:1487-1502)
        for (int task = lane; task < 400; task += 64) {
            const int r = task / 25, k = task - r * 25;
            float re = 0.0f, im = 0.0f;
            for (int j = 0; j < 25; ++j) {
                const float v = fin[r + 16 * j];
                re = re + v * tabs->dc[k * j];
                im = im - v * tabs->ds[k * j];
            }
            A[r * 25 + k] = cpx{re, im};
        }
        wave_sync();
        fft_level(A, Bf, 50, 8, tabs->c50, tabs->s50, lane);
        wave_sync();
        fft_level(Bf, A, 100, 4, tabs->c100, tabs->s100, lane);
        wave_sync();
        fft_level(A, Bf, 200, 2, tabs->c200, tabs->s200, lane);
        wave_sync();
        fft_level(Bf, A, 400, 1, tabs->c400, tabs->s400, lane);
        wave_sync();
        // power (main.rs:1603-1606), fold (main.rs:1608-1610)
        for (int j = lane; j < 400; j += 64) fin[j] = A[j].re * A[j].re + A[j].im * A[j].im;
        wave_sync();
        float fold[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = lane + 64 * q;
            fold[q] = (j >= 1 && j < 200) ? fin[j] + fin[400 - j] : 0.0f;
        }
        wave_sync();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = lane + 64 * q;
            if (j >= 1 && j < 200) fin[j] = fold[q];
        }
        wave_sync();
        // filterbank, clamp, log10 (main.rs:1620-1634)
        const int *rng = (const int *)(F + (FG ? 0 : 201 * n_mel));  // per mel: [first, end) of its non-zero weights
        for (int m = lane; m < n_mel; m += 64) {
            float sum = 0.0f;
            const int k0 = rng[(FG ? 4 : 2) * m], k1 = rng[(FG ? 4 : 2) * m + 1];  // outside: weight 0 -> exact +0 terms
            if (FG) {
                const float *wm = F + 4 * n_mel + rng[4 * m + 2] - k0;
                for (int k = k0; k < k1; ++k) sum = sum + fin[k] * wm[k];
            } else {
                for (int k = k0; k < k1; ++k) sum = sum + fin[k] * F[k * n_mel + m];
            }
            if (sum < 1e-10f) sum = 1e-10f;
            // glibc's log10f (what Rust's f32::log10 calls) is within an ulp of
            // the correctly rounded result; the double path lands on the same
            // float for ~96% of inputs, the device log10f for far fewer.
            const float v = (float)log10((double)sum);
            melb[(int64_t)m * nl + i] = v;
            lmax = fmaxf(lmax, v);
        }
        wave_sync();
    }
    lmax = wave_max(lmax);
    if (lane == 0 && lmax > -INFINITY) atomicMax(&mel_max[b], ord_f32(lmax));
}

__global__ void k_mel_norm(float *mel, int64_t mel_stride, int n_mel, const int64_t *n_len, const uint32_t *mel_max) {
    const int b = blockIdx.y;
    const int64_t tot = (int64_t)n_mel * n_len[b];
    const double mmax = (double)unord_f32(mel_max[b]) - 8.0;  // clamp_and_normalize, main.rs:1654-1671
    float *p = mel + (int64_t)b * mel_stride;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (int64_t)gridDim.x * blockDim.x) {
        float v = p[i];
        if ((double)v < mmax) v = (float)mmax;
        p[i] = (v + 4.0f) / 4.0f;
    }
}

__global__ void k_mel_window(const float *mel, int64_t mel_stride, int n_mel, const int64_t *n_len, int mel_offset,
                             int T2, int Cp, uint16_t *xconv, float *xconv32, uint16_t *g1, int n) {
    const int b = blockIdx.y;
    // conv1's output rows 0 and T2 + 1 of this clip are conv2's zero padding
    // (its epilogue writes rows 1..T2): zeroed here instead of a memset of g1
    if (g1)
        for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < 2 * (int64_t)n;
             idx += (int64_t)gridDim.x * blockDim.x)
            g1[((int64_t)b * (T2 + 2) + (idx < n ? 0 : T2 + 1)) * n + (idx < n ? idx : idx - n)] = 0;
    const int64_t nl = n_len[b];
    const int64_t tot = (int64_t)(T2 + 2) * Cp;
    const int64_t i0 = mel_offset < nl ? mel_offset : nl;
    const int64_t i1 = (int64_t)mel_offset + T2 < nl ? (int64_t)mel_offset + T2 : nl;
    const float *p = mel + (int64_t)b * mel_stride;
    uint16_t *o = xconv + (int64_t)b * tot;
    float *o32 = xconv32 ? xconv32 + (int64_t)b * tot : nullptr;  // f32 models: conv1 input unrounded
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < tot; idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = idx / Cp;
        const int c = (int)(idx - row * Cp);
        const int64_t t = row - 1;
        float v = 0.0f;
        if (t >= 0 && t < T2 && c < n_mel && i0 + t < i1) v = p[(int64_t)c * nl + i0 + t];
        if (xconv32) o32[idx] = v;
        else o[idx] = f2h_bits(v);
    }
}

template <int MW, int FPW, bool FG>
static hipError_t mel_frames_launch(hipStream_t s, const MelTables *tabs, const float *filt_t, int n_mel,
                                    const float *const *pcm, const int64_t *n_samples, float *mel, int64_t mel_stride,
                                    const int64_t *n_len, int64_t max_len, uint32_t *mel_max, int n_clips, int n_fc) {
    const size_t lds = sizeof(MelTables) + sizeof(float) * ((((FG ? n_fc : 203 * n_mel) + 3) & ~3) + MW * MEL_SCRATCH);
    dim3 grid(cdiv(max_len, MW * FPW), n_clips);
    hipError_t e = allow_lds(k_mel_frames<MW, FPW, FG>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_mel_frames<MW, FPW, FG>), grid, dim3(64 * MW), lds, s, tabs, filt_t, n_mel, pcm, n_samples, mel,
                       mel_stride, n_len, mel_max, n_fc);
    return hipGetLastError();
}

hipError_t launch_mel_frames(hipStream_t s, const MelTables *tabs, const float *filt_t, int n_mel,
                             const float *const *pcm, const int64_t *n_samples, float *mel, int64_t mel_stride,
                             const int64_t *n_len, int64_t max_len, uint32_t *mel_max, int n_clips,
                             const float *filt_c, int n_fc) {
    if (max_len <= 0) return hipSuccess;
    // (each frame's arithmetic is the same in both variants: bitwise equal)
    if (!filt_c)
        return mel_frames_launch<MEL_WAVES, MEL_FPW, false>(s, tabs, filt_t, n_mel, pcm, n_samples, mel, mel_stride, n_len,
                                                            max_len, mel_max, n_clips, 0);
    return mel_frames_launch<8, 1, true>(s, tabs, filt_c, n_mel, pcm, n_samples, mel, mel_stride, n_len, max_len, mel_max,
                                         n_clips, n_fc);
}

__global__ __launch_bounds__(256) void k_dec_reset(ResetArgs a) {
    const size_t gt = (size_t)blockIdx.x * 256 + threadIdx.x, nt = (size_t)gridDim.x * 256;
    if (gt < (size_t)a.n_feed) a.dfeed[gt] = a.feed[gt];
    for (int r = 0; r < a.n; ++r) {
        uint32_t *p = (uint32_t *)a.ptr[r];
        const size_t nw = a.bytes[r] / 4, n4 = ((uintptr_t)p & 15) ? 0 : nw / 4;
        for (size_t i = gt; i < n4; i += nt) ((uint4 *)p)[i] = make_uint4(0u, 0u, 0u, 0u);
        for (size_t i = 4 * n4 + gt; i < nw; i += nt) p[i] = 0u;
    }
}
hipError_t launch_dec_reset(hipStream_t s, const ResetArgs &a) {
    if (a.n < 0 || a.n > 8 || a.n_feed < 0 || a.n_feed > 64) return hipErrorInvalidValue;
    size_t mx = 0;
    for (int r = 0; r < a.n; ++r) {
        if (((uintptr_t)a.ptr[r] & 3) || (a.bytes[r] & 3)) return hipErrorInvalidValue;
        mx = a.bytes[r] > mx ? a.bytes[r] : mx;
    }
    const int g = (int)std::min<size_t>(1024, std::max<size_t>(1, (mx / 16 + 255) / 256));
    hipLaunchKernelGGL(k_dec_reset, dim3(g), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_mel_norm(hipStream_t s, float *mel, int64_t mel_stride, int n_mel, const int64_t *n_len,
                           int64_t max_len, const uint32_t *mel_max, int n_clips) {
    if (max_len <= 0) return hipSuccess;
    dim3 grid(cdiv((int64_t)n_mel * max_len, 1024) < 512 ? cdiv((int64_t)n_mel * max_len, 1024) : 512, n_clips);
    hipLaunchKernelGGL(k_mel_norm, grid, dim3(256), 0, s, mel, mel_stride, n_mel, n_len, mel_max);
    return hipGetLastError();
}

hipError_t launch_mel_window(hipStream_t s, const float *mel, int64_t mel_stride, int n_mel, const int64_t *n_len,
                             int mel_offset, int T2, int Cp, uint16_t *xconv, int n_clips,
                             float *xconv32, uint16_t *g1, int n) {
    const int64_t tot = (int64_t)(T2 + 2) * Cp;
    dim3 grid(cdiv(tot, 1024) < 512 ? cdiv(tot, 1024) : 512, n_clips);
    hipLaunchKernelGGL(k_mel_window, grid, dim3(256), 0, s, mel, mel_stride, n_mel, n_len, mel_offset, T2, Cp, xconv, xconv32,
                       g1, n);
    return hipGetLastError();
}

// ============================================================================
// LayerNorm: ggml_compute_forward_norm_f32 (double mean / variance, eps 1e-5)
// followed by mul(repeat(w)) and add(repeat(b)) (main.rs:1881-1886)
// ============================================================================
// one wave per row, the row held in registers (n <= 1280, n % 4 == 0): one
// round trip for the loads instead of one per pass over the row
// (LNW_V = n / 256 rounded up, a template constant: no clamped duplicate loads)
constexpr int LNW_VMAX = 5;
template <int LNW_V>
__device__ __forceinline__ void layernorm_wave(const float *x, int n, const float *w, const float *b, uint16_t *y16,
                                               float *y32, int lane) {
    float4 v[LNW_V], gw[LNW_V], gb[LNW_V];
#pragma unroll
    for (int i = 0; i < LNW_V; ++i) {
        const int e = (lane + 64 * i) * 4, ec = e < n ? e : 0;  // clamped, unconditional loads
        v[i] = *(const float4 *)(x + ec);
        gw[i] = *(const float4 *)(w + ec);
        gb[i] = *(const float4 *)(b + ec);
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < LNW_V; ++i)
        if ((lane + 64 * i) * 4 < n) s += ((double)v[i].x + (double)v[i].y) + ((double)v[i].z + (double)v[i].w);
    s = wave_sum(s);
    const double mean = s / n;
    double s2 = 0.0;
#pragma unroll
    for (int i = 0; i < LNW_V; ++i)
        if ((lane + 64 * i) * 4 < n) {
            const double d0 = (double)v[i].x - mean, d1 = (double)v[i].y - mean;
            const double d2 = (double)v[i].z - mean, d3 = (double)v[i].w - mean;
            s2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
        }
    s2 = wave_sum(s2);
    const float scale = (float)(1.0 / sqrt(s2 / n + (double)1e-5f));
#pragma unroll
    for (int i = 0; i < LNW_V; ++i) {
        const int e = (lane + 64 * i) * 4;
        if (e < n) {
            const float xx[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
            const float ww[4] = {gw[i].x, gw[i].y, gw[i].z, gw[i].w}, bb[4] = {gb[i].x, gb[i].y, gb[i].z, gb[i].w};
            float o[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float yv = (float)((double)xx[u] - mean);
                o[u] = bb[u] + ww[u] * (yv * scale);
            }
            if (y16) {
                half4 hv;
                hv[0] = f16_rt(o[0]); hv[1] = f16_rt(o[1]); hv[2] = f16_rt(o[2]); hv[3] = f16_rt(o[3]);
                *(half4 *)(y16 + e) = hv;
            }
            if (y32) *(float4 *)(y32 + e) = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
}

template <int LNW_V>
__global__ __launch_bounds__(256) void k_layernorm(const float *x, int rows, int n, const float *w, const float *b,
                                                   uint16_t *y16, float *y32) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    layernorm_wave<LNW_V>(x + (int64_t)row * n, n, w, b, y16 ? y16 + (int64_t)row * n : nullptr,
                   y32 ? y32 + (int64_t)row * n : nullptr, threadIdx.x & 63);
}

hipError_t launch_layernorm(hipStream_t s, const float *x, int rows, int n, const float *w, const float *b,
                            uint16_t *y16, float *y32) {
    if (n % 4 || n > 256 * LNW_VMAX || n < 4) return hipErrorInvalidValue;
    const dim3 g(cdiv(rows, 4)), t(256);
    switch ((n + 255) / 256) {
        case 1: hipLaunchKernelGGL(k_layernorm<1>, g, t, 0, s, x, rows, n, w, b, y16, y32); break;
        case 2: hipLaunchKernelGGL(k_layernorm<2>, g, t, 0, s, x, rows, n, w, b, y16, y32); break;
        case 3: hipLaunchKernelGGL(k_layernorm<3>, g, t, 0, s, x, rows, n, w, b, y16, y32); break;
        case 4: hipLaunchKernelGGL(k_layernorm<4>, g, t, 0, s, x, rows, n, w, b, y16, y32); break;
        default: hipLaunchKernelGGL(k_layernorm<5>, g, t, 0, s, x, rows, n, w, b, y16, y32); break;
    }
    return hipGetLastError();
}

// ============================================================================
// MFMA GEMM  C[M][N] = A[M][K] * B[N][K]^T   (f16 x f16 -> f32)
// 256 threads = 2x2 waves; each wave owns (BM/2)x(BN/2) built from
// v_mfma_f32_32x32x16_f16 tiles; BK = 32, register-staged double-buffered
// LDS with 80-byte rows (conflict-free ds_read_b128 fragment reads).
// ============================================================================
constexpr int GBK = 32;

template <bool CONV>
__device__ __forceinline__ uint4 gemm_load_a(const GemmArgs &a, int m, int k) {
    if (m >= a.M) return make_uint4(0, 0, 0, 0);
    const uint16_t *p;
    if (CONV) {
        const int b = m / a.conv_tout;
        const int t = m - b * a.conv_tout;
        const int tap = k / a.conv_cp;
        const int c = k - tap * a.conv_cp;
        p = a.A + ((int64_t)b * (a.conv_tin + 2) + (int64_t)t * a.conv_stride + tap) * a.conv_cp + c;
    } else {
        p = a.A + (int64_t)m * a.lda + k;
    }
    return *(const uint4 *)p;
}


// ---- LDS-staged GEMM epilogue -------------------------------------------
// The MFMA accumulators leave a lane as one column n and rows spaced 1, 8 and
// 4 apart: stored straight from them (gemm_epi4) every store is 2 or 4 bytes
// wide and a wave-instruction touches 2 rows x 64-128 bytes — the 8-clip
// encoder GEMMs spent more than half their time there (mlp.0 69.6 vs 30.5 us
// without the stores, cross K/V 212 vs 93).  Here the workgroup's BM x BN f32
// tile goes through LDS (row-major, or column-major for the V^T tiles of the
// QKV projection, whose output runs along m) and every thread then finishes
// 4 consecutive outputs at a time: one 16-byte (f32) or 8-byte (f16) store,
// consecutive threads on consecutive addresses.  The arithmetic per output
// is gemm_epi4's, so the results are bitwise the same.  Needs N % 4 == 0 and
// the caller's LDS free (after the k loop's last barrier).
template <int BM, int BN>
constexpr size_t epi_stage_bytes() {
    return (size_t)4 * (BM * (BN + 4) > BN * (BM + 4) ? BM * (BN + 4) : BN * (BM + 4));
}

// the staged path's shape conditions (workgroup-uniform)
template <int EPI, int BN>
__device__ __forceinline__ bool epi_staged_ok(const GemmArgs &a) {
    return a.epi_staged && a.N % 4 == 0 && a.ldo % 4 == 0 && (EPI != EPI_QKV || a.n_state % BN == 0);
}

template <int EPI, int BM, int BN>
__device__ __forceinline__ void gemm_epi_staged(const GemmArgs &a, const floatx16 (&acc)[BM / 64][BN / 64], float *stg,
                                                int m0, int n0) {
    constexpr int TM = BM / 64, TN = BN / 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
    const int lr = lane & 31, lh = lane >> 5;
    // the QKV projection's V^T tiles (n in [2 ns, 3 ns): whole tiles, ns % BN == 0)
    const bool tr = EPI == EPI_QKV && n0 >= 2 * a.n_state;
    if (!tr) {
        constexpr int LS = BN + 4;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = wm * (BM / 2) + i * 32 + 4 * lh + 8 * (r >> 2) + (r & 3);
                    stg[row * LS + wn * (BN / 2) + j * 32 + lr] = acc[i][j][r];
                }
    } else {
        constexpr int LS = BM + 4;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int col = wn * (BN / 2) + j * 32 + lr, row = wm * (BM / 2) + i * 32 + 4 * lh + 8 * g;
                    *(float4 *)(stg + col * LS + row) =
                        make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
                }
    }
    __syncthreads();
    if (tr) {  // 4 consecutive rows m of one column n -> vt[b][h][d][t .. t + 3]
        constexpr int LS = BM + 4, CPC = BM / 4;
        const int ns = a.n_state, H = ns >> 6;
        for (int c = tid; c < BN * CPC; c += 256) {
            const int nn = c / CPC, m = m0 + 4 * (c - nn * CPC), n = n0 + nn;
            if (n >= a.N || m >= a.M) continue;
            const float4 v = *(const float4 *)(stg + nn * LS + 4 * (c - nn * CPC));
            const float bias = a.bias ? a.bias[n] : 0.0f;
            const int cc = n - 2 * ns, h = cc >> 6, d = cc & 63;
            const int b0 = m / a.T, t0 = m - b0 * a.T;
            const float vv[4] = {v.x, v.y, v.z, v.w};
            if (m + 3 < a.M && t0 + 3 < a.T && (t0 & 3) == 0) {
                half4 hv;
#pragma unroll
                for (int r = 0; r < 4; ++r) hv[r] = f16_rt(vv[r] + bias);
                *(half4 *)(a.vt + (((int64_t)b0 * H + h) * 64 + d) * a.Tp + t0) = hv;
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int mm = m + r;
                    if (mm >= a.M) break;
                    const int b = mm / a.T, t = mm - b * a.T;
                    a.vt[(((int64_t)b * H + h) * 64 + d) * a.Tp + t] = f2h_bits(vv[r] + bias);
                }
            }
        }
        return;
    }
    constexpr int LS = BN + 4, CPR = BN / 4;
    for (int c = tid; c < BM * CPR; c += 256) {
        const int row = c / CPR, n = n0 + 4 * (c - row * CPR), m = m0 + row;
        if (n >= a.N || m >= a.M) continue;
        const float4 v = *(const float4 *)(stg + row * LS + 4 * (c - row * CPR));
        float4 bs = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (EPI != EPI_CROSSKV && a.bias) bs = *(const float4 *)(a.bias + n);
        const float x[4] = {v.x + bs.x, v.y + bs.y, v.z + bs.z, v.w + bs.w};
        if constexpr (EPI == EPI_F32) {
            *(float4 *)(a.out32 + (int64_t)m * a.ldo + n) = make_float4(x[0], x[1], x[2], x[3]);
        } else if constexpr (EPI == EPI_RESID) {
            float4 *p = (float4 *)(a.out32 + (int64_t)m * a.ldo + n);
            const float4 o = *p;
            *p = make_float4(x[0] + o.x, x[1] + o.y, x[2] + o.z, x[3] + o.w);
        } else if constexpr (EPI == EPI_GELU16 || EPI == EPI_CONV1) {
            ushort4 g;
            g.x = gelu_bits(a.gelu_tab, x[0], a.gelu_min);
            g.y = gelu_bits(a.gelu_tab, x[1], a.gelu_min);
            g.z = gelu_bits(a.gelu_tab, x[2], a.gelu_min);
            g.w = gelu_bits(a.gelu_tab, x[3], a.gelu_min);
            int64_t o = (int64_t)m * a.ldo + n;
            if constexpr (EPI == EPI_CONV1) {
                const int b = m / a.T, t = m - b * a.T;
                o = ((int64_t)b * (a.T + 2) + t + 1) * a.ldo + n;
            }
            *(ushort4 *)(a.out16 + o) = g;
        } else if constexpr (EPI == EPI_CONV2PE) {
            const int t = m - (m / a.T) * a.T;
            const float4 pe = *(const float4 *)(a.pe + (int64_t)t * a.ldo + n);
            *(float4 *)(a.out32 + (int64_t)m * a.ldo + n) =
                make_float4(pe.x + h2f_bits(gelu_bits(a.gelu_tab, x[0], a.gelu_min)),
                            pe.y + h2f_bits(gelu_bits(a.gelu_tab, x[1], a.gelu_min)),
                            pe.z + h2f_bits(gelu_bits(a.gelu_tab, x[2], a.gelu_min)),
                            pe.w + h2f_bits(gelu_bits(a.gelu_tab, x[3], a.gelu_min)));
        } else if constexpr (EPI == EPI_CROSSKV) {
            const int ns = a.n_state, l = n / (2 * ns), rr = n - l * 2 * ns;
            const int b = m / a.T, t = m - b * a.T;
            const int64_t base = (((int64_t)l * a.n_clips + b) * a.T + t) * ns;
            ushort4 h;
            if (rr < ns) {
                h.x = f2h_bits(v.x * a.kscale); h.y = f2h_bits(v.y * a.kscale);
                h.z = f2h_bits(v.z * a.kscale); h.w = f2h_bits(v.w * a.kscale);
                *(ushort4 *)(a.ck + base + rr) = h;
            } else {
                const float4 bv = a.bias ? *(const float4 *)(a.bias + n) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                h.x = f2h_bits(v.x + bv.x); h.y = f2h_bits(v.y + bv.y);
                h.z = f2h_bits(v.z + bv.z); h.w = f2h_bits(v.w + bv.w);
                *(ushort4 *)(a.cv + base + rr - ns) = h;
            }
        } else if constexpr (EPI == EPI_QKV) {  // q / k tiles: [b][h][Tp][64]
            const int ns = a.n_state, H = ns >> 6, which = n / ns, cc = n - which * ns, h = cc >> 6, d = cc & 63;
            const int b = m / a.T, t = m - b * a.T;
            ushort4 hv;
            hv.x = f2h_bits(x[0]); hv.y = f2h_bits(x[1]); hv.z = f2h_bits(x[2]); hv.w = f2h_bits(x[3]);
            *(ushort4 *)((which == 0 ? a.q : a.k) + (((int64_t)b * H + h) * a.Tp + t) * 64 + d) = hv;
        }
    }
}

// BK = k per LDS stage.  Small tiles (2-4 MFMAs per wave per 32 k) spend
// their k loop on barriers and LDS round trips, so they take 64 or 128 k per
// stage; the k steps of 16 still run in order, so the result is bitwise the
// same for every BK (and every tile size).
template <int BM, int BN, int BK, int EPI, bool CONV>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs a) {
    constexpr int TM = BM / 64, TN = BN / 64;          // 32x32 tiles per wave (2x2 waves)
    constexpr int LD = BK + 8;                          // halfs per LDS row (16-byte pad)
    constexpr int CPR = BK / 8;                         // 16-byte chunks per row of a stage
    constexpr int ACH = BM * CPR / 256, BCH = BN * CPR / 256;  // chunks per thread per stage
    __shared__ __attribute__((aligned(16))) f16 smem[2 * (BM + BN) * LD];
    // the staged epilogue where the k stages' LDS holds the f32 tile
    constexpr bool STAGED = epi_stage_bytes<BM, BN>() <= sizeof(smem);
    f16 *As = smem;
    f16 *Bs = smem + 2 * BM * LD;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // XCD-aware tile order: consecutive block ids land on different XCDs, so
    // give each XCD a contiguous range of tiles (bijective remap).
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    const int nwg = nbm * nbn;
    int bid = blockIdx.x;
    {
        const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
    }
    const int bn = bid % nbn, bm = bid / nbn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int nk = a.K / BK;

    typedef uint32_t g4 __attribute__((ext_vector_type(4)));  // native vector: stays in registers
    g4 ra[ACH], rb[BCH];
    auto gload = [&](int kt) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int c = tid + i * 256, row = c / CPR, col = (c % CPR) * 8;
            ra[i] = __builtin_bit_cast(g4, gemm_load_a<CONV>(a, m0 + row, kt * BK + col));
        }
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int c = tid + i * 256, row = c / CPR, col = (c % CPR) * 8;
            const int n = n0 + row;
            rb[i] = n < a.N ? *(const g4 *)(a.B + (int64_t)n * a.K + kt * BK + col) : g4{0u, 0u, 0u, 0u};
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int c = tid + i * 256, row = c / CPR, col = (c % CPR) * 8;
            *(g4 *)(As + buf * BM * LD + row * LD + col) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int c = tid + i * 256, row = c / CPR, col = (c % CPR) * 8;
            *(g4 *)(Bs + buf * BN * LD + row * LD + col) = rb[i];
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    gload(0);
    sstore(0);
    __syncthreads();
    const int lr = lane & 31, lh = lane >> 5;
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        gload(kt + 1 < nk ? kt + 1 : kt);  // unconditional (clamped): no undef phi
        const f16 *Ab = As + buf * BM * LD;
        const f16 *Bb = Bs + buf * BN * LD;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            half8 af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                af[i] = *(const half8 *)(Ab + (wm * (BM / 2) + i * 32 + lr) * LD + ks * 16 + lh * 8);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bf[j] = *(const half8 *)(Bb + (wn * (BN / 2) + j * 32 + lr) * LD + ks * 16 + lh * 8);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        sstore(buf ^ 1);  // (after the last stage: a clamped copy, unread)
        __syncthreads();
    }
    if constexpr (STAGED) {
        if (epi_staged_ok<EPI, BN>(a)) {
            gemm_epi_staged<EPI, BM, BN>(a, acc, (float *)smem, m0, n0);
            return;
        }
    }
    // epilogue: lane holds column n, rows (reg&3) + 8(reg>>2) + 4(lane>>5)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * (BN / 2) + j * 32 + lr;
            const int mb = m0 + wm * (BM / 2) + i * 32 + 4 * lh;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                gemm_epi4<EPI>(a, mb + 8 * g, n, v);
            }
        }
}

// ---- large-M GEMM (the 8-clip encoder shapes): a 128 x 128 tile per
// 256-thread workgroup (2 x 2 waves of 64 x 64, v_mfma_f32_32x32x16_f16),
// k staged 64 at a time by global_load_lds (16 bytes a lane, no register
// staging) into a lane-linear LDS image.  A wave-instruction's 1 KB covers 8
// rows of 64 k (128-byte rows); the image's 16-byte chunk c of row r holds the
// row's logical chunk c ^ ((r >> 1) & 7) — the swizzle is applied to the
// per-lane SOURCE address (the DMA destination must stay lane-linear) and
// undone on the read, so a fragment read's 32 rows fall on 16 distinct slots
// of each 256-byte bank row in every 16-lane group (conflict-free
// ds_read_b128).  Two LDS stages: the next tile's DMA is issued before this
// tile's fragment reads and MFMAs, then one vmcnt(0) + barrier per tile.
// The MFMA and the k order (16 at a time, ascending) are k_gemm's, so every
// output is bitwise k_gemm's.
__device__ __forceinline__ int gg_chunk(int r, int c) { return c ^ ((r >> 1) & 7); }

template <int EPI, bool CONV>
__global__ __launch_bounds__(256) void k_gemm_g(GemmArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char gsm[];  // [2][A 128 x 64 | B 128 x 64] f16
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int nbm = (a.M + 127) / 128, nbn = (a.N + 127) / 128;
    const int nwg = nbm * nbn;
    int bid = blockIdx.x;
    {  // XCD-aware bijective tile order (as k_gemm)
        const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
    }
    const int bn = bid % nbn, bm = bid / nbn;
    const int m0 = bm * 128, n0 = bn * 128;
    const int nk = a.K / 64;
    // this lane's DMA rows: wave w, instruction j fills image bytes
    // (4 w + j) KB + 16 lane = row (4 w + j) * 8 + lane / 8, chunk lane % 8
    // (rows past M / N read the last row: their outputs are never stored)
    const uint16_t *srcA[4], *srcB[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = (wave * 4 + j) * 8 + (lane >> 3), lc = gg_chunk(row, lane & 7);
        const int m = m0 + row < a.M ? m0 + row : a.M - 1, n = n0 + row < a.N ? n0 + row : a.N - 1;
        if constexpr (CONV) {
            const int b = m / a.conv_tout, t = m - b * a.conv_tout;
            srcA[j] = a.A + ((int64_t)b * (a.conv_tin + 2) + (int64_t)t * a.conv_stride) * a.conv_cp + lc * 8;
        } else {
            srcA[j] = a.A + (int64_t)m * a.lda + lc * 8;
        }
        srcB[j] = a.B + (int64_t)n * a.K + lc * 8;
    }
    typedef __attribute__((address_space(3))) void lds_t;
    auto stage = [&](int buf, int kt) {
        unsigned char *As = gsm + buf * 32768, *Bs = As + 16384;
        // implicit-GEMM conv: k = tap * Cp + c, a tap's channels contiguous (Cp % 64 == 0)
        int64_t ka = (int64_t)kt * 64;
        if constexpr (CONV) {
            const int tap = (kt * 64) / a.conv_cp, c = kt * 64 - tap * a.conv_cp;
            ka = (int64_t)tap * a.conv_cp + c;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            __builtin_amdgcn_global_load_lds((const void *)(srcA[j] + ka), (lds_t *)(As + (wave * 4 + j) * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *)(srcB[j] + (int64_t)kt * 64), (lds_t *)(Bs + (wave * 4 + j) * 1024),
                                             16, 0, 0);
        }
    };
    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    const int lr = lane & 31, lh = lane >> 5;
    // (three stages with two tiles in flight, a counted vmcnt and a raw
    // s_barrier — 96 KB, one workgroup per CU — measured slower: 8-clip
    // encoder 3.72 vs 3.00 ms, profiles/r04/gemm_g_ab.txt)
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) stage(buf ^ 1, kt + 1);
        const unsigned char *As = gsm + buf * 32768, *Bs = As + 16384;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int c = 2 * ks + lh;
            half8 af[2], bf[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = wm * 64 + i * 32 + lr;
                af[i] = *(const half8 *)(As + r * 128 + gg_chunk(r, c) * 16);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = wn * 64 + j * 32 + lr;
                bf[j] = *(const half8 *)(Bs + r * 128 + gg_chunk(r, c) * 16);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (epi_staged_ok<EPI, 128>(a)) {
        gemm_epi_staged<EPI, 128, 128>(a, acc, (float *)gsm, m0, n0);
        return;
    }
    // epilogue as k_gemm's: lane holds column n, rows (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn * 64 + j * 32 + lr;
            const int mb = m0 + wm * 64 + i * 32 + 4 * lh;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                gemm_epi4<EPI>(a, mb + 8 * g, n, v);
            }
        }
}

__global__ void k_gelu_scan(const uint16_t *tab, uint32_t *maxord) {
    const int h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h > 0xffff) return;
    const float f = h2f_bits((uint16_t)h);
    if (f != f) return;  // NaN inputs always take the table
    if (gelu_calc_bits(f) != tab[h]) atomicMax(maxord, ord_f32(f));
    atomicAdd(maxord + 1, 1u);  // inputs checked (the host expects all 63 490 non-NaN ones)
}

hipError_t launch_gelu_scan(hipStream_t s, const uint16_t *gelu_tab, uint32_t *maxord) {
    hipLaunchKernelGGL(k_gelu_scan, dim3(65536 / 256), dim3(256), 0, s, gelu_tab, maxord);
    return hipGetLastError();
}

// ---- one-clip GEMM (M ~ 1500: 96-384 workgroups, about one per CU): k_gemm's
// BM x BN tiles and MFMA order, but the k stages (64 k) arrive through an
// NST-deep ring of LDS-DMA buffers, NST - 1 stages in flight.  k_gemm holds
// one stage in flight in registers, so with a single workgroup per CU each
// stage cost one load latency (mlp.2 at K = 2048: 32 stages, 23.5 us).  The
// wait is a counted vmcnt + a raw s_barrier in one asm statement:
// __syncthreads() would drain the DMAs still in flight (vmcnt(0)).  The stage
// issued at step kt (clamped to the last stage past the end) goes to the
// buffer read at step kt - 1, which every wave has finished with once it has
// passed step kt's barrier.  LDS image and swizzle as k_gemm_g's (128-byte
// rows, chunk c of row r at c ^ ((r >> 1) & 7)); rows past M / N read the
// last row, whose outputs are never stored.  Every output is bitwise k_gemm's.
template <int BM, int BN, int NST, int EPI, bool CONV>
__global__ __launch_bounds__(256) void k_gemm_p(GemmArgs a) {
    constexpr int TM = BM / 64, TN = BN / 64;
    constexpr int PA = BM / 32, PB = BN / 32, P = PA + PB;  // 1 KB DMA instructions per wave per stage
    constexpr int SB = (BM + BN) * 128;                     // bytes per stage
    extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    const int nwg = nbm * nbn;
    int bid = blockIdx.x;
    {  // XCD-aware bijective tile order (as k_gemm)
        const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
    }
    const int bn = bid % nbn, bm = bid / nbn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int nk = a.K / 64;
    const uint16_t *srcA[PA], *srcB[PB];
#pragma unroll
    for (int j = 0; j < PA; ++j) {
        const int row = (wave * PA + j) * 8 + (lane >> 3), lc = gg_chunk(row, lane & 7);
        const int m = m0 + row < a.M ? m0 + row : a.M - 1;
        if constexpr (CONV) {
            const int b = m / a.conv_tout, t = m - b * a.conv_tout;
            srcA[j] = a.A + ((int64_t)b * (a.conv_tin + 2) + (int64_t)t * a.conv_stride) * a.conv_cp + lc * 8;
        } else {
            srcA[j] = a.A + (int64_t)m * a.lda + lc * 8;
        }
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
        const int row = (wave * PB + j) * 8 + (lane >> 3), lc = gg_chunk(row, lane & 7);
        const int n = n0 + row < a.N ? n0 + row : a.N - 1;
        srcB[j] = a.B + (int64_t)n * a.K + lc * 8;
    }
    typedef __attribute__((address_space(3))) void lds_t;
    // (implicit-GEMM conv: a row's 3 taps x Cp channels are contiguous, k = tap * Cp + c)
    auto stage = [&](int buf, int kt) {
        unsigned char *As = psm + buf * SB, *Bs = As + BM * 128;
#pragma unroll
        for (int j = 0; j < PA; ++j)
            __builtin_amdgcn_global_load_lds((const void *)(srcA[j] + kt * 64), (lds_t *)(As + (wave * PA + j) * 1024), 16, 0, 0);
#pragma unroll
        for (int j = 0; j < PB; ++j)
            __builtin_amdgcn_global_load_lds((const void *)(srcB[j] + kt * 64), (lds_t *)(Bs + (wave * PB + j) * 1024), 16, 0, 0);
    };
    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
    for (int s = 0; s < NST - 1; ++s) stage(s, s < nk ? s : nk - 1);
    for (int kt = 0; kt < nk; ++kt) {
        // stage kt landed (this wave's DMAs; the barrier: every wave's)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"((NST - 2) * P) : "memory");
        {
            const int kn = kt + NST - 1;
            stage(kn % NST, kn < nk ? kn : nk - 1);
        }
        const unsigned char *As = psm + (kt % NST) * SB, *Bs = As + BM * 128;
        // the whole stage's fragments first (one LDS latency a stage, not four)
        half8 af[4][TM], bf[4][TN];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int c = 2 * ks + lh;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int r = wm * (BM / 2) + i * 32 + lr;
                af[ks][i] = *(const half8 *)(As + r * 128 + gg_chunk(r, c) * 16);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int r = wn * (BN / 2) + j * 32 + lr;
                bf[ks][j] = *(const half8 *)(Bs + r * 128 + gg_chunk(r, c) * 16);
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // (the scheduler would sink each read to its MFMA)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[ks][i], bf[ks][j], acc[i][j], 0, 0, 0);
    }
    // the clamped stages past the end are still landing: drain before the
    // staged epilogue reuses the ring
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (epi_staged_ok<EPI, BN>(a)) {
        gemm_epi_staged<EPI, BM, BN>(a, acc, (float *)psm, m0, n0);
        return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * (BN / 2) + j * 32 + lr;
            const int mb = m0 + wm * (BM / 2) + i * 32 + 4 * lh;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                gemm_epi4<EPI>(a, mb + 8 * g, n, v);
            }
        }
}

template <int BM, int BN, int NST, bool CONV>
static hipError_t gemm_p_dispatch(hipStream_t s, int epi, const GemmArgs &a) {
    const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    constexpr size_t ring = (size_t)NST * (BM + BN) * 128, stg = epi_stage_bytes<BM, BN>();
    constexpr size_t lds = ring > stg ? ring : stg;
#define GEMMP_CASE(E)                                                                        \
    case E: {                                                                               \
        hipError_t e = allow_lds(k_gemm_p<BM, BN, NST, E, CONV>, lds);                     \
        if (e != hipSuccess) return e;                                                      \
        hipLaunchKernelGGL((k_gemm_p<BM, BN, NST, E, CONV>), dim3(nwg), dim3(256), lds, s, a); \
        break;                                                                              \
    }
    if constexpr (CONV) {
        switch (epi) {
            GEMMP_CASE(EPI_CONV1)
            GEMMP_CASE(EPI_CONV2PE)
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (epi) {
            GEMMP_CASE(EPI_F32)
            GEMMP_CASE(EPI_RESID)
            GEMMP_CASE(EPI_GELU16)
            GEMMP_CASE(EPI_QKV)
            GEMMP_CASE(EPI_CROSSKV)
            default: return hipErrorInvalidValue;
        }
    }
#undef GEMMP_CASE
    return hipGetLastError();
}

template <bool CONV>
static hipError_t gemm_g_dispatch(hipStream_t s, int epi, const GemmArgs &a) {
    const int nwg = ((a.M + 127) / 128) * ((a.N + 127) / 128);
    constexpr size_t lds = epi_stage_bytes<128, 128>();  // (>= the two 32 KB k stages)
#define GEMMG_CASE(E)                                                                        \
    case E: {                                                                               \
        hipError_t e = allow_lds(k_gemm_g<E, CONV>, lds);                              \
        if (e != hipSuccess) return e;                                                      \
        hipLaunchKernelGGL((k_gemm_g<E, CONV>), dim3(nwg), dim3(256), lds, s, a);      \
        break;                                                                              \
    }
    if constexpr (CONV) {
        switch (epi) {
            GEMMG_CASE(EPI_CONV1)
            GEMMG_CASE(EPI_CONV2PE)
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (epi) {
            GEMMG_CASE(EPI_F32)
            GEMMG_CASE(EPI_RESID)
            GEMMG_CASE(EPI_GELU16)
            GEMMG_CASE(EPI_QKV)
            GEMMG_CASE(EPI_CROSSKV)
            default: return hipErrorInvalidValue;
        }
    }
#undef GEMMG_CASE
    return hipGetLastError();
}

template <int BM, int BN, int BK, bool CONV>
static hipError_t gemm_dispatch_epi(hipStream_t s, int epi, const GemmArgs &a) {
    const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    dim3 grid(nwg), block(256);
#define GEMM_CASE(E)                                                                  \
    case E:                                                                          \
        hipLaunchKernelGGL((k_gemm<BM, BN, BK, E, CONV>), grid, block, 0, s, a);     \
        break;
    if constexpr (CONV) {
        switch (epi) {
            GEMM_CASE(EPI_CONV1)
            GEMM_CASE(EPI_CONV2PE)
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (epi) {
            GEMM_CASE(EPI_F32)
            GEMM_CASE(EPI_RESID)
            GEMM_CASE(EPI_GELU16)
            GEMM_CASE(EPI_QKV)
            GEMM_CASE(EPI_CROSSKV)
            default: return hipErrorInvalidValue;
        }
    }
#undef GEMM_CASE
    return hipGetLastError();
}

hipError_t launch_gemm(hipStream_t s, int epi, const GemmArgs &a0) {
    if (a0.M <= 0 || a0.N <= 0) return hipSuccess;
    GemmArgs a = a0;
    a.epi_staged = tune_of(a0.tune).epi_staged;
    if (a.B32) return launch_gemm32(s, epi, a);
    if (a.K % GBK != 0 || a.K <= 0) return hipErrorInvalidValue;
    if (a.conv && a.conv_cp % GBK != 0) return hipErrorInvalidValue;
    const int64_t t128 = (int64_t)cdiv(a.M, 128) * cdiv(a.N, 128);
    const int64_t t12864 = (int64_t)cdiv(a.M, 128) * cdiv(a.N, 64);
    // k per stage: 64 for the smaller tiles when it divides K (and, for the
    // implicit-GEMM conv, a tap's channel block); LDS stays <= 64 KB
    const bool k64 = (a.conv ? a.conv_cp : a.K) % 64 == 0;
    // large M: the LDS-DMA kernel (bitwise the same outputs)
    // (8-clip encoder 3.10 -> 3.00 ms: conv2 84.6 -> 71.3, Wo 39.7 -> 34.8,
    // mlp.2 77.0 -> 60.2 us; QKV and mlp.0 unchanged)
    // one clip (M <= 2048): every 64-k shape on k_gemm_p's LDS-DMA ring — the
    // same tiles' MFMA order, the k stages 2-3 deep (below); the 128 x 128
    // k_gemm_g keeps the 8-clip shapes
    if (tune_of(a.tune).gemm_p && k64 && a.M <= 2048 && t128 >= 240)
        return a.conv ? gemm_p_dispatch<128, 64, 3, true>(s, epi, a) : gemm_p_dispatch<128, 64, 3, false>(s, epi, a);
    if (t128 >= GEMM_G_MIN_TILES && tune_of(a.tune).gemm_g && a.K % 64 == 0 && (!a.conv || a.conv_cp % 64 == 0))
        return a.conv ? gemm_g_dispatch<true>(s, epi, a) : gemm_g_dispatch<false>(s, epi, a);
    // (128 k a stage for the smaller tiles — half the k steps of these
    // latency-bound one-clip GEMMs, the same MFMA order — measured slower:
    // 1-clip encoder 0.685 -> 0.726 ms, profiles/r06/gemm_bk128_ab_REJECTED.txt)
    // the one-clip shapes: the same tiles with the k stages on an LDS-DMA ring
    // (1-clip encode 0.637 -> 0.541 ms, bitwise equal; measured and not kept:
    // 64 x 64 tiles throughout 0.547, rings of 4 / 6 stages at one workgroup a
    // CU 0.587 vs 0.531, 6 / 8 stages for the <= 256-tile 64 x 64 grids 0.567 /
    // 0.571 vs 0.559; the one-clip shapes of >= 240 128 x 128 tiles on the
    // ring instead of k_gemm_g: small 1.852 -> 1.813 ms, base 0.557 -> 0.548
    // (its cross K / V; 0.533 vs 0.531 in an earlier session): kept, above;
    // the 8-clip shapes on the ring instead: 2.346 -> 2.360 ms, not kept;
    // profiles/r06/gemm_p_ab.txt)
    if (tune_of(a.tune).gemm_p && k64 && t128 < 240) {
        if (t12864 >= 240)
            return a.conv ? gemm_p_dispatch<128, 64, 3, true>(s, epi, a) : gemm_p_dispatch<128, 64, 3, false>(s, epi, a);
        return a.conv ? gemm_p_dispatch<64, 64, 4, true>(s, epi, a) : gemm_p_dispatch<64, 64, 4, false>(s, epi, a);
    }
    if (a.conv) {
        if (t128 >= 240) return gemm_dispatch_epi<128, 128, GBK, true>(s, epi, a);
        if (t12864 >= 240) return k64 ? gemm_dispatch_epi<128, 64, 64, true>(s, epi, a)
                                       : gemm_dispatch_epi<128, 64, GBK, true>(s, epi, a);
        return k64 ? gemm_dispatch_epi<64, 64, 64, true>(s, epi, a) : gemm_dispatch_epi<64, 64, GBK, true>(s, epi, a);
    }
    if (t128 >= 240) return gemm_dispatch_epi<128, 128, GBK, false>(s, epi, a);
    if (t12864 >= 240) return k64 ? gemm_dispatch_epi<128, 64, 64, false>(s, epi, a)
                                  : gemm_dispatch_epi<128, 64, GBK, false>(s, epi, a);
    return k64 ? gemm_dispatch_epi<64, 64, 64, false>(s, epi, a) : gemm_dispatch_epi<64, 64, GBK, false>(s, epi, a);
}

// ============================================================================
// Encoder self-attention, ggml flash_attn_f16 semantics (masked = false):
// S = scale * K q (f16 dot, f32), exact row max, table exp of f16(S - max),
// double sum, P16 = f16(e * (1/sum)), O = P16 V.  (Round 1's k_attn_enc3 —
// 8 waves splitting the keys of one 32-query block, scores in registers — is
// in the git history; k_attn_enc4 replaced it at every batch size.)
// ============================================================================
// NW x 32 queries per workgroup share every K / V tile through LDS
// (128-key tiles, double-buffered, one global->LDS copy per tile for the
// whole workgroup instead of one per 32 queries); KQ = 4 waves share a query
// block, wave kb taking keys kb * 32 .. kb * 32 + 31 of every tile, and the
// softmax runs in three sweeps over the keys instead of holding the scores in
// registers:
//   sweep 0: S = scale * K Q^T (MFMA) -> row max (exact: the parts' maxima
//            meet in LDS)
//   sweep 1: S again -> p = exp_tab[f16(S - max)]: double sum of p (exact,
//            so the parts' sums meet in LDS in any order)
//   sweep 2: S again -> P16 = f16(p * (1 / sum)) -> O += P16 V (MFMA)
// — ggml's rounding points (flash_attn_f16: P16 rounded before P V).  The
// parts' partial O meet in LDS, added in part order.  Recomputing Q K^T costs
// MFMA time the kernel has to spare.  (Round 5's two-sweep form — p V
// unnormalised, O / sum at the end — saved one sweep, 0.69 vs 0.78 ms a clip
// at KQ = 2, but moved the encoder output past its noise floor against the
// oracle: base 1.41e-3 vs floor 1.34e-3; it is in the git history.)
// KQ (2 or 4) key parts per query block: tiles of KT = 32 KQ keys, V^T tile
// rows of KT + 8 halfs in LDS (attn_enc_kq picks KQ per model)
constexpr int AT4_LD = 72;  // halfs per K row in LDS (64 + 8 pad: 144-byte rows)

// 16-byte staging chunks as a native vector (SROA keeps arrays of these in
// registers; the struct uint4 arrays of the staging loop went to scratch)
typedef uint32_t a4vec __attribute__((ext_vector_type(4)));

// this wave's 32-key part kb of a tile in LDS (buffer Kb / Vb) for its 32
// queries.  TAIL: the tile holds keys >= T (masked); full tiles skip every key test.
// Sweep 0 keeps the max of the raw scores (scale > 0 and rounding are
// monotone, so fl(max_raw * scale) is the max of the scaled scores); sweeps
// 1 and 2 clamp the table index to n_exp, where the table holds a 0 (no
// compare / select per element); scale and subtract run as packed f32 pairs,
// as m - S: fl(m - S) = -fl(S - m), so its f16 bits are the table index
// f16(|S - m|) with no mask (m is never -0: the caller adds +0).
typedef float f2v __attribute__((ext_vector_type(2)));
// PASS 3 (sum sweep, one clip): as PASS 1, and the table values p kept in
// pst (registers: the tile's two P fragments); PASS 4: P16 = f16(p * inv)
// from pst — no Q K^T and no table reads — then P16 V
template <int KQ, int PASS, bool TAIL>
__device__ __forceinline__ void attn4_tile(const AttnArgs &a, const f16 *Kb, const f16 *Vb, int key0, int kb,
                                           const uint16_t *tab, const half8 (&qf)[4], float &mx, double &sum,
                                           float m, float inv, floatx16 &o0, floatx16 &o1, half8 (&pst)[2]) {
    constexpr int VLD = 32 * KQ + 8;
    const int lane = threadIdx.x & 63, lr = lane & 31, lh = lane >> 5;
    const int T = a.T;
    const uint32_t n_exp = (uint32_t)a.n_exp;
    const f2v scale2 = {a.scale, a.scale}, m2 = {m, m};
    if constexpr (PASS == 4) {
        half8 pa[2];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < 8; ++i) pa[s][i] = f16_rt((float)pst[s][i] * inv);  // (keys past T: p = 0)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            half8 vb[2];
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const f16 *vp = Vb + (dt * 32 + lr) * VLD + kb * 32 + 16 * s + 4 * lh;
                const half4 v0 = *(const half4 *)vp, v1 = *(const half4 *)(vp + 8);
                vb[dt][0] = v0[0]; vb[dt][1] = v0[1]; vb[dt][2] = v0[2]; vb[dt][3] = v0[3];
                vb[dt][4] = v1[0]; vb[dt][5] = v1[1]; vb[dt][6] = v1[2]; vb[dt][7] = v1[3];
            }
            o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(pa[s], vb[0], o0, 0, 0, 0);
            o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(pa[s], vb[1], o1, 0, 0, 0);
        }
        return;
    }
    {  // this wave's 32-key part kb of the tile
        floatx16 sc;
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = 0.0f;
#pragma unroll
        for (int s = 0; s < 4; ++s)
            sc = __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8 *)(Kb + (kb * 32 + lr) * AT4_LD + 16 * s + 8 * lh),
                                                        qf[s], sc, 0, 0, 0);
        if constexpr (PASS == 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (!TAIL || key < T) mx = fmaxf(mx, sc[r]);
            }
        } else {
            half8 pa[2];
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
                f2v v = {sc[r], sc[r + 1]};
                v = v * scale2;
                v = m2 - v;  // >= +0
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int key = key0 + kb * 32 + ((r + u) & 3) + 8 * ((r + u) >> 2) + 4 * lh;
                    uint32_t i = f2h_bits(v[u]);
                    i = i < n_exp ? i : n_exp;  // v_min: index n_exp holds 0
                    if (TAIL) i = key < T ? i : n_exp;
                    const float e = h2f_bits(tab[i]);  // unguarded read (a guarded one branches per element)
                    if constexpr (PASS == 1 || PASS == 3) sum += (double)e;
                    if constexpr (PASS == 3) pa[(r + u) >> 3][(r + u) & 7] = (f16)e;  // (an f16 value: exact)
                    if constexpr (PASS == 2) pa[(r + u) >> 3][(r + u) & 7] = f16_rt(e * inv);  // P16 = f16(p * (1 / sum))
                }
            }
            if constexpr (PASS == 3) {
                pst[0] = pa[0];
                pst[1] = pa[1];
            }
            if constexpr (PASS == 2) {
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    half8 vb[2];
#pragma unroll
                    for (int dt = 0; dt < 2; ++dt) {
                        const f16 *vp = Vb + (dt * 32 + lr) * VLD + kb * 32 + 16 * s + 4 * lh;
                        const half4 v0 = *(const half4 *)vp, v1 = *(const half4 *)(vp + 8);
                        vb[dt][0] = v0[0]; vb[dt][1] = v0[1]; vb[dt][2] = v0[2]; vb[dt][3] = v0[3];
                        vb[dt][4] = v1[0]; vb[dt][5] = v1[1]; vb[dt][6] = v1[2]; vb[dt][7] = v1[3];
                    }
                    o0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(pa[s], vb[0], o0, 0, 0, 0);
                    o1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(pa[s], vb[1], o1, 0, 0, 0);
                }
            }
        }
    }
}

// One sweep over the key tiles (PASS 0: max, 1: exp sum, 2: P16 V).  Tiles
// go global -> registers -> LDS with two register stages: while tile kt is
// computed from LDS, tile kt + 1 sits in one register set (stored to the
// other LDS buffer after the compute) and tile kt + 2's loads are in flight
// into the other, so a load has two tiles of compute to land (the loop is
// unrolled by two so the register sets are named statically; every load is
// unconditional from a clamped tile, so no undef phi reaches scratch).  The
// partial last tile runs after the loop: a full / tail branch inside it made
// the compiler copy both MFMA accumulators every iteration (32 v_mov a tile).
template <int NW, int KQ, int PASS>
__device__ __forceinline__ void attn4_sweep(const AttnArgs &a, const f16 *K, const f16 *Vt, f16 *Ks, f16 *Vs,
                                            const uint16_t *tab, const half8 (&qf)[4], float &mx, double &sum,
                                            float m, float inv, floatx16 &o0, floatx16 &o1) {
    constexpr int AT4_KT = 32 * KQ, AT4_VLD = AT4_KT + 8;
    const int tid = threadIdx.x;
    const int Tp = a.Tp;
    const int ntiles = (a.T + AT4_KT - 1) / AT4_KT;
    constexpr int NT = 64 * KQ * NW;  // threads: NW query blocks x KQ key parts
    constexpr int SCH = AT4_KT * 8 / NT;  // 16-byte chunks per thread of a K (or V^T) tile
    constexpr int VCH = PASS == 2 ? SCH : 1;
    constexpr int VCPR = AT4_KT / 8;      // 16-byte chunks per V^T tile row
    const int kb = (threadIdx.x >> 6) / NW;  // this wave's 32-key part of every tile
    a4vec kA[SCH], vA[VCH], kB[SCH], vB[VCH];
    // this thread's 16-byte chunks of a tile: K rows (tid >> 3) + (NT / 8) i,
    // column (tid & 7) * 8; V^T rows tid / VCPR + (NT / VCPR) i, column (tid % VCPR) * 8.
    // Keys past Tp (the last tile when T is not a multiple of the tile) are
    // read clamped: masked scores, finite values
    const int crow = tid >> 3, ccol = (tid & 7) * 8;
    const int vrow = tid / VCPR, vcol = (tid % VCPR) * 8;
    half8 pdummy[2];
#define ATT4_GLOAD(KT, KR, VR)                                                                  \
    {                                                                                           \
        const int kt_ = (KT) < ntiles ? (KT) : ntiles - 1;                                      \
        const int key0_ = kt_ * AT4_KT;                                                         \
        _Pragma("unroll") for (int i = 0; i < SCH; ++i) {                                       \
            const int kr_ = key0_ + crow + i * (NT / 8);                                        \
            KR[i] = *(const a4vec *)(K + (int64_t)(kr_ < Tp ? kr_ : Tp - 1) * 64 + ccol);       \
            if constexpr (PASS == 2) {                                                          \
                const int vc_ = key0_ + vcol;                                                   \
                VR[i] = *(const a4vec *)(Vt + (int64_t)(vrow + i * (NT / VCPR)) * Tp + (vc_ < Tp ? vc_ : Tp - 8)); \
            }                                                                                   \
        }                                                                                       \
    }
#define ATT4_SSTORE(BUF, KR, VR)                                                                \
    {                                                                                           \
        _Pragma("unroll") for (int i = 0; i < SCH; ++i) {                                       \
            *(a4vec *)(Ks + ((BUF) * AT4_KT + crow + i * (NT / 8)) * AT4_LD + ccol) = KR[i];    \
            if constexpr (PASS == 2)                                                            \
                *(a4vec *)(Vs + ((BUF) * 64 + vrow + i * (NT / VCPR)) * AT4_VLD + vcol) = VR[i]; \
        }                                                                                       \
    }
    ATT4_GLOAD(0, kA, vA)
    ATT4_SSTORE(0, kA, vA)
    ATT4_GLOAD(1, kB, vB)  // (kB, vB): the next tile, loop-carried
    __syncthreads();
    const int nfull = a.T / AT4_KT;
    for (int kt = 0; kt < nfull; ++kt) {
        const int buf = kt & 1;
        a4vec kF[SCH], vF[VCH];  // tile kt + 2, requested before this tile's compute
        ATT4_GLOAD(kt + 2, kF, vF)
        attn4_tile<KQ, PASS, false>(a, Ks + buf * AT4_KT * AT4_LD, Vs + buf * 64 * AT4_VLD, kt * AT4_KT, kb, tab, qf,
                                    mx, sum, m, inv, o0, o1, pdummy);
        ATT4_SSTORE(buf ^ 1, kB, vB)  // (after the last tile: unread)
        __syncthreads();
#pragma unroll
        for (int i = 0; i < SCH; ++i) kB[i] = kF[i];
#pragma unroll
        for (int i = 0; i < VCH; ++i) vB[i] = vF[i];
    }
    if (nfull < ntiles) {  // the partial tile (stored by the last iteration)
        const int buf = nfull & 1;
        attn4_tile<KQ, PASS, true>(a, Ks + buf * AT4_KT * AT4_LD, Vs + buf * 64 * AT4_VLD, nfull * AT4_KT, kb,
                                   tab, qf, mx, sum, m, inv, o0, o1, pdummy);
        __syncthreads();  // (callers reuse the tile buffers: as after every loop tile)
    }
#undef ATT4_GLOAD
#undef ATT4_SSTORE
}

// The sum sweep keeping p in registers (PASS 3) and the P V sweep reading
// them (PASS 4: only V tiles staged), for one clip's workgroups (NW <= 2:
// the registers for a whole row's p fit beside the sweep's — MAXT tiles x 8
// VGPRs), the tile loop unrolled so every tile's p has its own registers.
// The arithmetic is PASS 1 / PASS 2's, value for value: a clip's output does
// not depend on which form ran (test_enc_attn_nw_parity_and_batch_invariance)
constexpr int AT4_MAXT_REG = 12;  // 128-key tiles held in registers (T <= 1536)
template <int... I, typename F>
__device__ __forceinline__ void static_for(std::integer_sequence<int, I...>, F &&f) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int NW, int KQ, int PASS>
__device__ __forceinline__ void attn4_sweep_reg(const AttnArgs &a, const f16 *K, const f16 *Vt, f16 *Ks, f16 *Vs,
                                                const uint16_t *tab, const half8 (&qf)[4], double &sum, float m,
                                                float inv, floatx16 &o0, floatx16 &o1,
                                                half8 (&ps)[AT4_MAXT_REG][2]) {
    static_assert(PASS == 3 || PASS == 4, "stored-p passes");
    constexpr int AT4_KT = 32 * KQ, AT4_VLD = AT4_KT + 8;
    const int tid = threadIdx.x;
    const int Tp = a.Tp;
    const int ntiles = (a.T + AT4_KT - 1) / AT4_KT, nfull = a.T / AT4_KT;
    constexpr int NT = 64 * KQ * NW;
    constexpr int SCH = AT4_KT * 8 / NT;
    constexpr int VCPR = AT4_KT / 8;
    const int kb = (threadIdx.x >> 6) / NW;
    const int crow = tid >> 3, ccol = (tid & 7) * 8;
    const int vrow = tid / VCPR, vcol = (tid % VCPR) * 8;
    float mx = 0.0f;
    auto gload = [&](int kt, a4vec (&R)[SCH]) {  // PASS 3: K tile rows; PASS 4: V^T tile columns
        const int kt_ = kt < ntiles ? kt : ntiles - 1;
        const int key0 = kt_ * AT4_KT;
#pragma unroll
        for (int i = 0; i < SCH; ++i) {
            if constexpr (PASS == 3) {
                const int kr = key0 + crow + i * (NT / 8);
                R[i] = *(const a4vec *)(K + (int64_t)(kr < Tp ? kr : Tp - 1) * 64 + ccol);
            } else {
                const int vc = key0 + vcol;
                R[i] = *(const a4vec *)(Vt + (int64_t)(vrow + i * (NT / VCPR)) * Tp + (vc < Tp ? vc : Tp - 8));
            }
        }
    };
    auto sstore = [&](int buf, const a4vec (&R)[SCH]) {
#pragma unroll
        for (int i = 0; i < SCH; ++i) {
            if constexpr (PASS == 3) *(a4vec *)(Ks + (buf * AT4_KT + crow + i * (NT / 8)) * AT4_LD + ccol) = R[i];
            else *(a4vec *)(Vs + (buf * 64 + vrow + i * (NT / VCPR)) * AT4_VLD + vcol) = R[i];
        }
    };
    a4vec rA[SCH], rB[SCH];
    gload(0, rA);
    sstore(0, rA);
    gload(1, rB);
    __syncthreads();
    // tile KT as a template step (every tile's p in registers of its own:
    // a runtime-indexed array would live in scratch memory)
    auto step = [&](auto KTc) {
        constexpr int kt = decltype(KTc)::value;
        if (kt >= ntiles) return;  // workgroup-uniform
        a4vec rF[SCH];
        gload(kt + 2, rF);
        const f16 *Kb = Ks + (kt & 1) * AT4_KT * AT4_LD;
        const f16 *Vb = Vs + (kt & 1) * 64 * AT4_VLD;
        if (kt < nfull)
            attn4_tile<KQ, PASS, false>(a, Kb, Vb, kt * AT4_KT, kb, tab, qf, mx, sum, m, inv, o0, o1, ps[kt]);
        else
            attn4_tile<KQ, PASS, true>(a, Kb, Vb, kt * AT4_KT, kb, tab, qf, mx, sum, m, inv, o0, o1, ps[kt]);
        sstore((kt & 1) ^ 1, rB);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < SCH; ++i) rB[i] = rF[i];
    };
    static_for(std::make_integer_sequence<int, AT4_MAXT_REG>{}, step);
}

// Waves w, w + NW, .. w + (KQ - 1) NW share query block w and split every
// tile into its KQ 32-key parts (KQ times the waves per query, for one clip's
// small grid); their maxima, exact double sums and partial P V meet in LDS,
// the partial O added in part order.
template <int NW, int KQ>
__global__ __launch_bounds__(64 * KQ * NW) void k_attn_enc4(AttnArgs a) {
    constexpr int AT4_KT = 32 * KQ;
    extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
    uint16_t *tab = (uint16_t *)smraw;
    const int tab_bytes = (((a.n_exp + 1) * 2 + 15) / 16) * 16;
    f16 *Ks = (f16 *)(smraw + tab_bytes);      // [2][KT keys][AT4_LD]
    f16 *Vs = Ks + 2 * AT4_KT * AT4_LD;        // [2][64 dims][AT4_VLD] (V^T tile)
    const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int lr = lane & 31, lh = lane >> 5;
    const int64_t bh = (int64_t)b * a.H + h;
    const f16 *Q = (const f16 *)a.q + bh * a.Tp * 64;
    const f16 *K = (const f16 *)a.k + bh * a.Tp * 64;
    const f16 *Vt = (const f16 *)a.vt + bh * 64 * a.Tp;
    const int T = a.T;
    const int qw = w % NW, kb = w / NW;  // query block, key part
    const int q0 = (qb * NW + qw) * 32;  // this wave's queries
    half8 qf[4];
    {
        const int qrow = q0 + lr < a.Tp ? q0 + lr : a.Tp - 1;  // rows past T: computed, never stored
#pragma unroll
        for (int s = 0; s < 4; ++s) qf[s] = *(const half8 *)(Q + (int64_t)qrow * 64 + 16 * s + 8 * lh);
    }
    {
        const int nch = (a.n_exp + 1 + 7) / 8;  // through the 0 at index n_exp
        const uint4 *tsrc = (const uint4 *)a.exp_tab;
        for (int i = tid; i < nch; i += 64 * KQ * NW) ((uint4 *)tab)[i] = tsrc[i];
    }
    // exchange slots for the key-part partners (the V buffers: unused until sweep 2)
    float *xm = (float *)Vs;                          // [KQ NW][64]
    double *xd = (double *)(xm + KQ * NW * 64);  // [KQ NW][64]
    float mx = -INFINITY;
    double sum = 0.0;
    floatx16 o0, o1;
#pragma unroll
    for (int r = 0; r < 16; ++r) { o0[r] = 0.0f; o1[r] = 0.0f; }
    attn4_sweep<NW, KQ, 0>(a, K, Vt, Ks, Vs, tab, qf, mx, sum, 0.0f, 0.0f, o0, o1);
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    xm[w * 64 + lane] = mx;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < KQ; ++j) mx = fmaxf(mx, xm[(qw + NW * j) * 64 + lane]);
    const float m = mx * a.scale + 0.0f;  // max of the raw scores, scaled once (never -0)
    // one clip (NW <= 2, four key parts): the sum sweep keeps p in registers
    // and the P V sweep reads them instead of recomputing Q K^T and the table
    constexpr bool REG = KQ == 4 && NW <= 2;
    const bool reg = REG && a.T <= AT4_MAXT_REG * 32 * KQ;
    half8 ps[REG ? AT4_MAXT_REG : 1][2];
    if constexpr (REG) {
        if (reg) attn4_sweep_reg<NW, KQ, 3>(a, K, Vt, Ks, Vs, tab, qf, sum, m, 0.0f, o0, o1, ps);
        else attn4_sweep<NW, KQ, 1>(a, K, Vt, Ks, Vs, tab, qf, mx, sum, m, 0.0f, o0, o1);
    } else {
        attn4_sweep<NW, KQ, 1>(a, K, Vt, Ks, Vs, tab, qf, mx, sum, m, 0.0f, o0, o1);
    }
    sum = sum + __shfl_xor(sum, 32);
    xd[w * 64 + lane] = sum;  // (xd and xm are disjoint: no barrier after the max reads)
    __syncthreads();
    // exact double sums of f16 table values: the total is order-independent;
    // ggml's float sum, then 1 / sum in double rounded to float (the oracle's
    // flash_attn_row)
    double dsum = 0.0;
#pragma unroll
    for (int j = 0; j < KQ; ++j) dsum += xd[(qw + NW * j) * 64 + lane];
    const float inv = (float)(1.0 / (double)(float)dsum);
    // (lane lr's inv belongs to query lr; the P16 operand of lane (lr, lh)
    // row r is query lr too: the score tile is K Q^T, keys in rows)
    __syncthreads();  // (the exchange slots are V buffers in sweep 2)
    if constexpr (REG) {
        if (reg) attn4_sweep_reg<NW, KQ, 4>(a, K, Vt, Ks, Vs, tab, qf, sum, m, inv, o0, o1, ps);
        else attn4_sweep<NW, KQ, 2>(a, K, Vt, Ks, Vs, tab, qf, mx, sum, m, inv, o0, o1);
    } else {
        attn4_sweep<NW, KQ, 2>(a, K, Vt, Ks, Vs, tab, qf, mx, sum, m, inv, o0, o1);
    }
    // key parts 1 .. KQ - 1: partial O -> LDS (the K / V buffers are free
    // now), added to part 0's in part order
    float *xo = (float *)smraw;  // [KQ - 1][NW][32][64] over the table and tiles (free now)
    if (kb) {
        float *xp = xo + (size_t)(kb - 1) * NW * 32 * 64;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int qq = (r & 3) + 8 * (r >> 2) + 4 * lh;
            xp[(qw * 32 + qq) * 64 + lr] = o0[r];
            xp[(qw * 32 + qq) * 64 + 32 + lr] = o1[r];
        }
    }
    __syncthreads();
    if (kb) return;
#pragma unroll
    for (int j = 1; j < KQ; ++j) {
        const float *xp = xo + (size_t)(j - 1) * NW * 32 * 64;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int qq = (r & 3) + 8 * (r >> 2) + 4 * lh;
            o0[r] = o0[r] + xp[(qw * 32 + qq) * 64 + lr];
            o1[r] = o1[r] + xp[(qw * 32 + qq) * 64 + 32 + lr];
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int t = q0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (t < T) {
            const int64_t o = ((int64_t)b * T + t) * a.n_state + h * 64;
            if (a.out32) {  // f32 models: the output projection takes it unrounded
                a.out32[o + lr] = o0[r];
                a.out32[o + 32 + lr] = o1[r];
            } else {
                a.out[o + lr] = f2h_bits(o0[r]);
                a.out[o + 32 + lr] = f2h_bits(o1[r]);
            }
        }
    }
}

template <int NW, int KQ>
static hipError_t attn_enc4_launch(hipStream_t s, const AttnArgs &a) {
    constexpr int AT4_KT = 32 * KQ, AT4_VLD = AT4_KT + 8;
    const size_t tabb = (((a.n_exp + 1) * 2 + 15) / 16) * 16;
    const size_t tiles = (size_t)2 * AT4_KT * AT4_LD * 2 + (size_t)2 * 64 * AT4_VLD * 2;
    const size_t xob = (size_t)(KQ - 1) * NW * 32 * 64 * 4;  // the partial-O exchange (over table + tiles)
    const size_t lds = tabb + tiles > xob ? tabb + tiles : xob;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    hipError_t e = allow_lds(k_attn_enc4<NW, KQ>, lds);
    if (e != hipSuccess) return e;
    dim3 grid(cdiv(a.T, 32 * NW), a.H, a.n_clips);
    hipLaunchKernelGGL((k_attn_enc4<NW, KQ>), grid, dim3(64 * KQ * NW), lds, s, a);
    return hipGetLastError();
}

// Query blocks per workgroup: 4 once the grid holds >= 2 workgroups per CU
// (8 clips of base: 2.38 ms at 2, 2.25-2.30 at 4 — 1024 threads, 20 VGPRs
// spilled — as more waves per CU hide more), else 2.  NW does not change a
// wave's arithmetic, so a clip's result is batch-independent.
int attn_enc_nw(int T, int H, int n_clips, int nw_knob) {
    if (nw_knob == 1 || nw_knob == 2 || nw_knob == 4) return nw_knob;
    return (int64_t)cdiv(T, 128) * H * n_clips >= 512 ? 4 : 2;
}

// Key parts per query block, per model (never per batch: the P V partials'
// order is the arithmetic, so a clip's output stays batch-independent):
// four where one clip's query blocks leave the SIMDs idle (base: 8 heads x
// 47 blocks = 376 -> four-part waves, one clip 0.69 -> 0.645 ms in the
// two-sweep form, profiles/r05/enc_kq4_ab.txt), two where they fill the chip
// by themselves (small: 564, large-v3: 940 blocks).
int attn_enc_kq(int T, int H) { return (int64_t)cdiv(T, 32) * H >= 512 ? 2 : 4; }

hipError_t launch_attn_enc(hipStream_t s, const AttnArgs &a) {
    const Tune &tn = tune_of(a.tune);
    if (a.T < 1 || a.Tp % 64 || a.Tp < a.T) return hipErrorInvalidValue;
    const int nw = attn_enc_nw(a.T, a.H, a.n_clips, tn.enc_attn_nw);
    if (attn_enc_kq(a.T, a.H) == 2) {
        if (nw == 4) return attn_enc4_launch<4, 2>(s, a);
        if (nw == 2) return attn_enc4_launch<2, 2>(s, a);
        return attn_enc4_launch<1, 2>(s, a);
    }
    if (nw == 4) return attn_enc4_launch<4, 4>(s, a);
    if (nw == 2) return attn_enc4_launch<2, 4>(s, a);
    return attn_enc4_launch<1, 4>(s, a);
}

// ============================================================================
// decoder step kernels (batch B <= 8 clips), latency-oriented
// ============================================================================
constexpr int DG_MAXB = 8;

// y[b][o] = W[o] . in[b]  for B <= 8 input rows.  A quarter-wave (16 lanes)
// owns one output row; a wave owns 4*G rows, a workgroup 16*G.  Latency is
// what matters at decode batch sizes, so every global load the kernel needs
// (weight rows, input rows / attention partials, bias, residual) is issued
// before anything waits: the whole kernel costs about one memory round trip.
//   IN = 0: LayerNorm(x) prologue (x rows held in registers, double stats)
//   IN = 1: f16 input vector
//   IN = 2: sum (in chunk order) of split-key attention partials
constexpr int DG_LNV = 5;  // float4 per lane for a LayerNorm row (K <= 1280)

// previous step's greedy token of one clip: max over its AMAX_SHARDS packed
// (ordered logit << 32 | ~id) words; called by a whole wave, result uniform
__device__ __forceinline__ int32_t shard_token(const unsigned long long *sh, int lane) {
    const unsigned long long k = wave_max_u64(sh[lane]);
    return (int32_t)(0xffffffffu - (uint32_t)(k & 0xffffffffull));
}

// v if ok else 0, written so the compiler cannot sink the load of v into a
// branch on ok (a select lets it, and the branch then serialises every load
// behind an s_waitcnt); v must be finite (it is loaded from a clamped, valid
// address)
__device__ __forceinline__ float4 keep4(float4 v, bool ok) {
    const float f = ok ? 1.0f : 0.0f;
    return make_float4(v.x * f, v.y * f, v.z * f, v.w * f);
}
__device__ __forceinline__ float keep1(float v, bool ok) { return v * (ok ? 1.0f : 0.0f); }

// LayerNorm input row as float4 registers: unconditional (clamped) loads so
// every request is in flight before the first wait
template <int L>
__device__ __forceinline__ void ln_load_row(const float *x, int K, int lane, float4 (&xv)[L]) {
    const float4 *xr = (const float4 *)x;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const int idx = lane + 64 * i;
        const bool ok = idx * 4 < K;
        xv[i] = keep4(xr[ok ? idx : 0], ok);
    }
}

// LayerNorm gain / bias as float4 registers
template <int L>
__device__ __forceinline__ void ln_load_params(const float *lw, const float *lb, int K, int lane, float4 (&gw)[L],
                                               float4 (&gb)[L]) {
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const int e = (lane + 64 * i) * 4, ec = e < K ? e : 0;
        gw[i] = keep4(*(const float4 *)(lw + ec), e < K);
        gb[i] = keep4(*(const float4 *)(lb + ec), e < K);
    }
}

// LayerNorm of one K-row held as float4 registers (ggml norm semantics)
template <int L>
__device__ __forceinline__ void ln_regs_to_lds(const float4 (&xv)[L], int K, const float4 (&gw)[L],
                                               const float4 (&gb)[L], f16 *dst, int lane) {
    double s1 = 0.0;
#pragma unroll
    for (int i = 0; i < L; ++i)
        if ((lane + 64 * i) * 4 < K) s1 += ((double)xv[i].x + (double)xv[i].y) + ((double)xv[i].z + (double)xv[i].w);
    s1 = wave_sum(s1);
    const double mean = s1 / K;
    double s2 = 0.0;
#pragma unroll
    for (int i = 0; i < L; ++i)
        if ((lane + 64 * i) * 4 < K) {
            const double d0 = (double)xv[i].x - mean, d1 = (double)xv[i].y - mean;
            const double d2 = (double)xv[i].z - mean, d3 = (double)xv[i].w - mean;
            s2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
        }
    s2 = wave_sum(s2);
    const float scale = (float)(1.0 / sqrt(s2 / K + (double)1e-5f));
#pragma unroll
    for (int i = 0; i < L; ++i) {
        const int e = (lane + 64 * i) * 4;
        if (e < K) {
            const float xx[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
            const float ww[4] = {gw[i].x, gw[i].y, gw[i].z, gw[i].w}, bb4[4] = {gb[i].x, gb[i].y, gb[i].z, gb[i].w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float t = (float)((double)xx[u] - mean) * scale;
                dst[e + u] = f16_rt(bb4[u] + ww[u] * t);
            }
        }
    }
}

// the same with the gain / bias requested here (before the two reductions)
template <int L>
__device__ __forceinline__ void ln_regs_to_lds(const float4 (&xv)[L], int K, const float *lw, const float *lb,
                                               f16 *dst, int lane) {
    float4 gw[L], gb[L];
    ln_load_params(lw, lb, K, lane, gw, gb);
    ln_regs_to_lds(xv, K, gw, gb, dst, lane);
}


// NC = 128-element K chunks a lane prefetches per row (8 for K <= 1024, 16 for
// the MLP-down GEMV at K = 4n <= 2048); longer rows loop.
// decoder weight stream loads (plain loads: the non-temporal policy was
// measured and removed in round 5)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ T wload(const T *p) {
    return *p;
}
__device__ __forceinline__ uint4 wload(const uint4 *p) {
    const u32x4 v = wload((const u32x4 *)p);
    return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ uint2 wload(const uint2 *p) {
    const u32x2 v = wload((const u32x2 *)p);
    return make_uint2(v[0], v[1]);
}

// NW = waves per workgroup: 4 (16 rows per workgroup) for the vocabulary GEMV
// and batched rows; 1 (4 rows) for the small per-layer GEMVs at B <= 2, so
// their 0.5-2 MiB weight streams spread over 4x the CUs (per-CU bytes, not
// chip bandwidth, bound a 2 MiB GEMV spread over 32-128 workgroups)
template <int EPI, int IN, int G, int NC, int WQ, int NW>
__global__ __launch_bounds__(64 * NW) void k_dec_gemv(DecGemvArgs a) {
    // chunk geometry: a quarter-wave covers CW consecutive weights of its row
    // per chunk, a lane LW of them (f16: 8 = one 16-byte load; q5_1: 32 = one
    // block, its 16 nibble bytes + an 8-byte {5th bits, d/m} word)
    constexpr int CW = WQ ? 512 : 128, LW = CW / 16;
    constexpr int DG_NC = NC, DG_KB = NC * CW;
    // the vocabulary GEMV is persistent and software-pipelined over two
    // register sets: row group i + 1's weights are in flight while group i is
    // reduced and written (PIPE); the others run one row group per workgroup
    constexpr bool PIPE = EPI == DEC_LOGITS;
    // LayerNorm row registers: the K <= 512 (NC = 4, f16) instances need 2 float4 per lane
    constexpr int LNV = (NC == 4 && !WQ) ? 2 : DG_LNV;
    extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
    f16 *xs = (f16 *)smraw;  // [B][K]
    __shared__ unsigned long long amax_s[DG_MAXB];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int q = lane >> 4, l16 = lane & 15;
    const int K = a.K, B = a.B, N = a.N;
    const int nrg = (N + 4 * NW * G - 1) / (4 * NW * G);
    auto rbase = [&](int rg) { return (rg * NW + w) * 4 * G; };
    const f16 *W = (const f16 *)a.W;
    const uint8_t *q5n = a.Wq5;
    const uint2 *q5hd = (const uint2 *)(a.Wq5 + (int64_t)N * K / 2);
    struct WSet {
        half8 wv[G][WQ ? 1 : DG_NC];
        uint4 wqn[G][WQ ? DG_NC : 1];
        uint2 wqd[G][WQ ? DG_NC : 1];
        float eb[G], er[G];  // epilogue operands: bias, residual (lane l16 == clip)
    };
    auto load_set = [&](WSet &S, int rb, int k0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int row = rb + g * 4 + q;
#pragma unroll
            for (int c = 0; c < DG_NC; ++c) {
                const int k = k0 + c * CW + l16 * LW;
                if constexpr (WQ) {
                    if (row < N && k < K) {
                        const int64_t e = (int64_t)row * K + k;
                        S.wqn[g][c] = wload((const uint4 *)(q5n + e / 2));
                        S.wqd[g][c] = wload(q5hd + e / 32);
                    } else {
                        S.wqn[g][c] = make_uint4(0u, 0u, 0u, 0u);
                        S.wqd[g][c] = make_uint2(0u, 0u);
                    }
                } else {
                    if (row < N && k < K) S.wv[g][c] = wload((const half8 *)(W + (int64_t)row * K + k));
                    else
#pragma unroll
                        for (int e = 0; e < 8; ++e) S.wv[g][c][e] = (f16)0.0f;
                }
            }
        }
    };
    auto load_epi = [&](WSet &S, int rb) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int o = rb + g * 4 + q;
            S.eb[g] = (a.bias && o < N) ? a.bias[o] : 0.0f;
            S.er[g] = (EPI == DEC_RESID && o < N && l16 < B) ? a.out32[(int64_t)l16 * N + o] : 0.0f;
        }
    };
    auto dot_set = [&](const WSet &S, int k0, float (&acc)[G][DG_MAXB]) {
#pragma unroll
        for (int c = 0; c < DG_NC; ++c) {
            const int k = k0 + c * CW + l16 * LW;
            if constexpr (WQ) {
                if (k < K) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        half8 wc[G];
#pragma unroll
                        for (int g = 0; g < G; ++g) {
                            const uint4 qv = S.wqn[g][c];
                            const uint32_t qn = j == 0 ? qv.x : j == 1 ? qv.y : j == 2 ? qv.z : qv.w;
                            wc[g] = q5_half8(qn, S.wqd[g][c].x, S.wqd[g][c].y, 8 * j);
                        }
#pragma unroll
                        for (int bb = 0; bb < DG_MAXB; ++bb) {
                            if (bb < B) {
                                const half8 xv = *(const half8 *)(xs + bb * K + k + 8 * j);
#pragma unroll
                                for (int g = 0; g < G; ++g) acc[g][bb] = dot8(wc[g], xv, acc[g][bb]);
                            }
                        }
                    }
                }
            } else if (k0 + c * CW < K) {
#pragma unroll
                for (int bb = 0; bb < DG_MAXB; ++bb) {
                    if (bb < B) {
                        const half8 xv = *(const half8 *)(xs + bb * K + k);
#pragma unroll
                        for (int g = 0; g < G; ++g) acc[g][bb] = dot8(S.wv[g][c], xv, acc[g][bb]);
                    }
                }
            }
        }
    };
    // cross-lane reduction and the fused epilogue of one row group
    auto finish = [&](int rb, float (&acc)[G][DG_MAXB], const WSet &S) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int bb = 0; bb < DG_MAXB; ++bb)
                if (bb < B) {
                    float v = acc[g][bb];
                    v = red16_sum(v);
                    acc[g][bb] = v;
                }
        const int pos = (EPI == DEC_QKV) ? a.st->pos : 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int o = rb + g * 4 + q;
            float v = 0.0f;
#pragma unroll
            for (int bb = 0; bb < DG_MAXB; ++bb)
                if (l16 == bb) v = acc[g][bb];
            if (l16 >= B || o >= N) continue;
            const int bb = l16;
            if (EPI == DEC_QKV) {
                const int n = N / 3, which = o / n, c = o - which * n;
                if (which == 0) a.out16[bb * a.ldo + c] = f2h_bits((v + S.eb[g]) * a.qscale);
                else if (which == 1)
                    a.kcache[((int64_t)bb * a.n_text_ctx + pos) * n + c] = f2h_bits(v * a.qscale);
                else a.vcache[((int64_t)bb * a.n_text_ctx + pos) * n + c] = f2h_bits(S.eb[g] + v);
            } else if (EPI == DEC_Q) {
                a.out16[bb * a.ldo + o] = f2h_bits((v + S.eb[g]) * a.qscale);
            } else if (EPI == DEC_GELU) {
                a.out16[bb * a.ldo + o] = a.gelu_tab[f2h_bits(v + S.eb[g])];
            } else if (EPI == DEC_RESID) {
                a.out32[(int64_t)bb * N + o] = (v + S.eb[g]) + S.er[g];
            } else if (EPI == DEC_LOGITS) {
                a.out32[(int64_t)bb * N + o] = v;
                if (a.amax && o != a.suppress_id) {
                    const unsigned long long key =
                        ((unsigned long long)ord_f32(v) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)o);
                    atomicMax(&amax_s[bb], key);
                }
            }
        }
    };
    auto zero = [&](float (&acc)[G][DG_MAXB]) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int bb = 0; bb < DG_MAXB; ++bb) acc[g][bb] = 0.0f;
    };
    // LayerNorm operands of row w first: the LN below then waits for them
    // while the weight stream issued after them is still in flight
    float4 xv0[LNV], gw0[LNV], gb0[LNV];
    if (IN == 0 && w < B) {
        ln_load_row(a.x + (int64_t)w * K, K, lane, xv0);
        ln_load_params(a.ln_w, a.ln_b, K, lane, gw0, gb0);
    }
    // every weight / epilogue request of the first group(s) before the prologue
    WSet S0, S1;
    int rgA = blockIdx.x, rgB = rgA + gridDim.x;
    load_set(S0, rbase(rgA), 0);
    load_epi(S0, rbase(rgA));
    if (PIPE && rgB < nrg) {
        load_set(S1, rbase(rgB), 0);
        load_epi(S1, rbase(rgB));
    }
    if (IN == 0 || IN == 3) {
        // each wave normalises rows w, w + NW, ...
        const int pos = (IN == 3) ? a.st->pos : 0;
#pragma unroll
        for (int rr = 0; rr < DG_MAXB / NW; ++rr) {
            const int rb = w + NW * rr;
            if (rb < B) {
                float4 xv[LNV];
                if (IN == 0 && rr == 0) {
                    ln_regs_to_lds(xv0, K, gw0, gb0, xs + rb * K, lane);
                    continue;
                }
                if (IN == 0) {
                    ln_load_row(a.x + (int64_t)rb * K, K, lane, xv);
                } else {
                    // x = te[tok] + pe[pos] (get_rows f16 -> f32, add)
                    const bool fed = pos < a.feed_len;
                    const int32_t tok = fed ? a.feed[rb * a.feed_stride + pos]
                                            : (a.beam_tok ? a.beam_tok[rb] : shard_token(a.amax + rb * AMAX_SHARDS, lane));
                    const f16 *ter = (const f16 *)a.te + (int64_t)tok * K;
                    const float *per = a.pe + (int64_t)pos * K;
                    half4 tv[LNV];
                    float4 pv[LNV];
#pragma unroll
                    for (int i = 0; i < LNV; ++i) {
                        const int e = (lane + 64 * i) * 4, ec = e < K ? e : 0;
                        tv[i] = *(const half4 *)(ter + ec);
                        pv[i] = *(const float4 *)(per + ec);
                    }
#pragma unroll
                    for (int i = 0; i < LNV; ++i) {
                        const int e = (lane + 64 * i) * 4;
                        xv[i] = keep4(make_float4((float)tv[i][0] + pv[i].x, (float)tv[i][1] + pv[i].y,
                                                  (float)tv[i][2] + pv[i].z, (float)tv[i][3] + pv[i].w),
                                      e < K);
                        if (e < K && blockIdx.x == 0) *(float4 *)(a.x_out + (int64_t)rb * K + e) = xv[i];
                    }
                    if (blockIdx.x == 0 && lane == 0 && !fed && a.tokens_out)
                        a.tokens_out[rb * a.out_stride + (pos - a.feed_len)] = tok;
                }
                ln_regs_to_lds(xv, K, a.ln_w, a.ln_b, xs + rb * K, lane);
            }
        }
    } else if (IN == 1) {
        const uint4 *src = (const uint4 *)a.xin16;
        uint4 *dst = (uint4 *)xs;
        for (int i = tid; i < B * K / 8; i += 64 * NW) dst[i] = src[i];
    } else {
        // partial sums: thread owns 4 consecutive inputs; all chunk loads issued first
        constexpr int CMAXP = 16;
        for (int i4 = tid; i4 < B * K / 4; i4 += 64 * NW) {
            const int bb = (i4 * 4) / K, k = i4 * 4 - bb * K;
            const float *p = a.parts + ((int64_t)bb * a.n_parts) * K + k;
            float4 v[CMAXP];
#pragma unroll
            for (int c = 0; c < CMAXP; ++c)
                v[c] = c < a.n_parts ? *(const float4 *)(p + (int64_t)c * K) : make_float4(0.f, 0.f, 0.f, 0.f);
            float4 sacc = v[0];
#pragma unroll
            for (int c = 1; c < CMAXP; ++c)
                if (c < a.n_parts) {
                    sacc.x = sacc.x + v[c].x; sacc.y = sacc.y + v[c].y;
                    sacc.z = sacc.z + v[c].z; sacc.w = sacc.w + v[c].w;
                }
            half4 hv;
            hv[0] = f16_rt(sacc.x); hv[1] = f16_rt(sacc.y); hv[2] = f16_rt(sacc.z); hv[3] = f16_rt(sacc.w);
            *(half4 *)(xs + bb * K + k) = hv;
        }
    }
    if (EPI == DEC_LOGITS && tid < DG_MAXB) amax_s[tid] = 0ull;
    __syncthreads();
    float acc[G][DG_MAXB];
    if constexpr (PIPE) {  // K <= DG_KB (checked by the launcher)
        for (;;) {
            zero(acc);
            dot_set(S0, 0, acc);
            const int rgC = rgB + gridDim.x;
            if (rgC < nrg) load_set(S0, rbase(rgC), 0);
            finish(rbase(rgA), acc, S0);
            if (rgB >= nrg) break;
            if (rgC < nrg) load_epi(S0, rbase(rgC));
            zero(acc);
            dot_set(S1, 0, acc);
            const int rgD = rgC + gridDim.x;
            if (rgD < nrg) load_set(S1, rbase(rgD), 0);
            finish(rbase(rgB), acc, S1);
            if (rgC >= nrg) break;
            if (rgD < nrg) load_epi(S1, rbase(rgD));
            rgA = rgC;
            rgB = rgD;
        }
    } else {  // one row group, K in DG_KB sweeps
        zero(acc);
        for (int k0 = 0; k0 < K; k0 += DG_KB) {
            if (k0 > 0) load_set(S0, rbase(rgA), k0);
            dot_set(S0, k0, acc);
        }
        finish(rbase(rgA), acc, S0);
    }
    if (EPI == DEC_LOGITS) {
        __syncthreads();
        if (a.amax && tid < B && amax_s[tid]) atomicMax(&a.amax[tid * AMAX_SHARDS + (blockIdx.x & (AMAX_SHARDS - 1))], amax_s[tid]);
        if (blockIdx.x == 0 && tid == 0) a.st_advance->pos += 1;
    }
}

// waves per workgroup of the per-layer GEMVs (Tune::gemv_nw, fixed at 4: one
// wave per workgroup measured mlp0 4.6 -> 10 us at base, B = 1, every
// workgroup repeating the LayerNorm); row groups per register set of the
// vocabulary GEMV at K <= 512 (Tune::logits_g, fixed at 2: base 13.9 us at
// G = 1 -> 12.1 us at G = 2 over 1024 workgroups)

template <int EPI, int IN, int WQ, int NW>
static hipError_t dec_gemv_nw(hipStream_t s, const DecGemvArgs &a) {
    const size_t lds = (size_t)a.B * a.K * 2;
    dim3 block(64 * NW);
    // the vocabulary GEMV runs persistent and pipelined (its K = n_state <=
    // 1280 fits one sweep of either chunk size); the others one group per WG
    const Tune &tn = tune_of(a.tune);
    const int cap = EPI == DEC_LOGITS ? tn.logits_cap : 1 << 30;
    const int nrg = cdiv(a.N, 4 * NW);
    const dim3 grid(nrg < cap ? nrg : cap);
    if constexpr (WQ == 1) {  // q5_1: 4 chunks of 512 weights (K <= 2048 per sweep)
        if (EPI == DEC_LOGITS && a.K > 2048) return hipErrorInvalidValue;
        hipError_t e = allow_lds(k_dec_gemv<EPI, IN, 1, 4, 1, NW>, lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_dec_gemv<EPI, IN, 1, 4, 1, NW>), grid, block, lds, s, a);
    } else if (a.K > 1024) {
        if (EPI == DEC_LOGITS && a.K > 2048) return hipErrorInvalidValue;
        hipError_t e = allow_lds(k_dec_gemv<EPI, IN, 1, 16, 0, NW>, lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_dec_gemv<EPI, IN, 1, 16, 0, NW>), grid, block, lds, s, a);
    } else if (EPI == DEC_LOGITS && a.K <= 512 && tn.logits_g > 1) {
        // K <= 512: 4 chunks cover a row, so each register set can hold G = 2
        // or 4 row groups (more bytes in flight per wave at the same VGPRs)
        // (128 VGPRs at G = 2: four workgroups per CU, hence the larger cap;
        // a balanced grid of equal row-group counts measured slower)
        const int G = tn.logits_g == 2 ? 2 : 4, ng = cdiv(a.N, 4 * NW * G);
        const dim3 grid2(ng < CHAIN_LOGITS_CAP2 ? ng : CHAIN_LOGITS_CAP2);
        if (G == 2) {
            hipError_t e = allow_lds(k_dec_gemv<EPI, IN, 2, 4, 0, NW>, lds);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((k_dec_gemv<EPI, IN, 2, 4, 0, NW>), grid2, block, lds, s, a);
        } else {
            hipError_t e = allow_lds(k_dec_gemv<EPI, IN, 4, 4, 0, NW>, lds);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((k_dec_gemv<EPI, IN, 4, 4, 0, NW>), grid2, block, lds, s, a);
        }
    } else {
        hipError_t e = allow_lds(k_dec_gemv<EPI, IN, 1, 8, 0, NW>, lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_dec_gemv<EPI, IN, 1, 8, 0, NW>), grid, block, lds, s, a);
    }
    return hipGetLastError();
}

template <int EPI, int IN, int WQ>
static hipError_t dec_gemv_g(hipStream_t s, const DecGemvArgs &a) {
    // one wave per workgroup spreads a per-layer GEMV over 4x the CUs; with
    // more rows each wave would normalise B / NW LayerNorm rows serially
    if constexpr (EPI == DEC_LOGITS) {
        return dec_gemv_nw<EPI, IN, WQ, 4>(s, a);
    } else {
        const Tune &tn = tune_of(a.tune);
        const bool one = tn.gemv_nw == 1 || (tn.gemv_nw == 0 && a.B <= 2);
        return one ? dec_gemv_nw<EPI, IN, WQ, 1>(s, a) : dec_gemv_nw<EPI, IN, WQ, 4>(s, a);
    }
}

template <int EPI, int IN>
static hipError_t dec_gemv_w(hipStream_t s, const DecGemvArgs &a) {
    return a.Wq5 ? dec_gemv_g<EPI, IN, 1>(s, a) : dec_gemv_g<EPI, IN, 0>(s, a);
}

// (epilogue, input) pairs the decoder step uses
hipError_t launch_dec_gemv(hipStream_t s, int epi, const DecGemvArgs &a) {
    if (a.B < 1 || a.B > DG_MAXB || a.K % 128) return hipErrorInvalidValue;
    if (a.W32) return launch_dec_gemv32(s, epi, a);
    const int in = a.te ? 3 : (a.ln_w ? 0 : (a.parts ? 2 : 1));
    if (epi == DEC_QKV && in == 3) return dec_gemv_w<DEC_QKV, 3>(s, a);
    if (epi == DEC_QKV && in == 0) return dec_gemv_w<DEC_QKV, 0>(s, a);
    if (epi == DEC_GELU && in == 0) return dec_gemv_w<DEC_GELU, 0>(s, a);
    if (epi == DEC_RESID && in == 1) return dec_gemv_w<DEC_RESID, 1>(s, a);
    if (epi == DEC_RESID && in == 2) return dec_gemv_w<DEC_RESID, 2>(s, a);
    if (epi == DEC_LOGITS && in == 0) return dec_gemv_w<DEC_LOGITS, 0>(s, a);
    return hipErrorInvalidValue;
}

// ---- decoder attention, split over 128-key chunks --------------------------
// ggml_compute_forward_soft_max_f32 semantics need the row max and the row sum
// before any P16 = f16(p * (1/sum)) exists, so the key range is split in two
// passes: (1) scores + per-chunk max; (2) every chunk workgroup recomputes the
// (cheap, L2-resident) global sum from the scores in the same order, so all
// chunks use the identical 1/sum, then writes its partial P16 V.  The partials
// are summed in chunk order by the consumer GEMV's prologue (IN = 2).
constexpr int DA_CK = 128;

// Bounded spin on a monotonic agent-scope counter (cooperative kernels: every
// member must be co-resident, which the launchers guarantee by grid size; on
// timeout the error word is set and the kernel finishes instead of hanging).
__device__ __forceinline__ uint32_t spin_until(uint32_t *p, uint32_t target, uint32_t *err) {
    uint32_t v = 0;
    for (uint32_t it = 0;; ++it) {
        v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v >= target) break;
        if (it > (1u << 22)) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
    return v;
}

// ---- words exchanged between workgroups of one launch ----------------------
// agent-scope relaxed atomics: write-through stores / coherent loads, no cache
// maintenance; ordering comes from s_waitcnt before the arrival counter
template <bool COH>
__device__ __forceinline__ float ld_x(const float *p) {
    if constexpr (COH)
        return __builtin_bit_cast(float, __hip_atomic_load((uint32_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    else
        return *p;
}
template <bool COH>
__device__ __forceinline__ void st_x(float *p, float v) {
    if constexpr (COH)
        __hip_atomic_store((uint32_t *)p, __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}

// Phase B of cross-attention for one 128-key chunk: row max over the chunk
// maxima, the row's exp sum recomputed from all M scores (identical order in
// every chunk workgroup, hence the identical 1/sum), P16 = f16(p / sum) for
// this chunk's keys, partial P16 V -> opart[b][c][h*64 .. +64].  vf holds the
// chunk's V rows: thread (doct = tid & 7, jg = tid >> 3) keys c*128 + jg*4 + u.
template <bool COH>
__device__ __forceinline__ void xattn_pv(const DecAttnArgs &a, int c, int h, int b, int M, const half8 (&vf)[4]) {
    __shared__ double redd[4];
    __shared__ float ow[4][64];
    __shared__ __attribute__((aligned(16))) uint16_t P[DA_CK];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = a.n;
    const int nC = (M + DA_CK - 1) / DA_CK;
    const int64_t bh = (int64_t)b * a.H + h;
    const float *S = a.S + bh * a.s_stride;
    // every request first: the chunk maxima and this thread's scores
    float cm[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) cm[i] = ld_x<COH>(a.cmax + bh * a.n_chunks + (i < nC ? i : 0));
    constexpr int SU = 8;  // M <= 2048 in one unrolled sweep
    float sv[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
        const int j = tid + 256 * u;
        sv[u] = ld_x<COH>(S + (j < M ? j : M - 1));
    }
    float m = cm[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) m = fmaxf(m, cm[i]);
    double sum = 0.0;
    float pmine = 0.0f;
#pragma unroll
    for (int u = 0; u < SU; ++u) {
        const int j = tid + 256 * u;
        const float p = keep1(exp_f16_exact(sv[u] - m), j < M);
        sum += (double)p;
        if (j >= c * DA_CK && j < (c + 1) * DA_CK) pmine = p;
    }
    for (int j = tid + 256 * SU; j < M; j += 256) sum += (double)exp_f16_exact(ld_x<COH>(S + j) - m);
    sum = wave_sum(sum);
    if (lane == 0) redd[w] = sum;
    __syncthreads();
    const float inv = (float)(1.0 / (((redd[0] + redd[1]) + redd[2]) + redd[3]));
#pragma unroll
    for (int u = 0; u < SU; ++u) {
        const int j = tid + 256 * u;
        if (j >= c * DA_CK && j < (c + 1) * DA_CK) P[j - c * DA_CK] = f2h_bits(j < M ? pmine * inv : 0.0f);
    }
    __syncthreads();
    const int doct = tid & 7, jg = tid >> 3;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.0f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const float pj = h2f_bits(P[jg * 4 + u]);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = o[e] + pj * (float)vf[u][e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        o[e] = red_8_16_32(o[e]);
    }
    if (lane < 8)
#pragma unroll
        for (int e = 0; e < 8; ++e) ow[w][lane * 8 + e] = o[e];
    __syncthreads();
    if (tid < 64)
        a.opart[((int64_t)b * a.n_chunks + c) * n + h * 64 + tid] =
            ((ow[0][tid] + ow[1][tid]) + ow[2][tid]) + ow[3][tid];
}

// this chunk's V rows for xattn_pv (clamped rows: every load unconditional)
__device__ __forceinline__ void xattn_load_v(const DecAttnArgs &a, int c, int h, int b, int M, half8 (&vf)[4]) {
    const int tid = threadIdx.x, doct = tid & 7, jg = tid >> 3;
    const f16 *Vb = (const f16 *)a.V + (int64_t)(b / a.clip_div) * a.clip_stride + h * 64 + doct * 8;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int j = c * DA_CK + jg * 4 + u;
        // rows past M repeat row M - 1 (finite); their P16 is 0
        vf[u] = *(const half8 *)(Vb + (int64_t)(j < M ? j : M - 1) * a.n);
    }
}

// Cross-attention for one 128-key chunk of one (clip, head).
// Phase A: q_h = f16((Wq_h LN(x) + bq) * qscale), recomputed by every chunk
// workgroup of the head from L2-resident rows instead of costing a kernel;
// the chunk's scores -> S, its max -> cmax.  MODE 0 stops there (first kernel
// of the two-kernel form, k_dec_attn_pv is the second).  MODE 1 (cooperative,
// all chunk workgroups co-resident): one arrival counter per (layer, clip,
// head) replaces the kernel boundary, then phase B runs in the same launch.
template <int KC, int MODE>
__global__ __launch_bounds__(256) void k_dec_xattn(DecAttnArgs a) {
    constexpr bool COH = MODE == 1;
    const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int q = lane >> 4, l16 = lane & 15;
    const int M = a.M_fixed;
    const int n = a.n;  // == KC * 128
    __shared__ __attribute__((aligned(16))) f16 xs[KC * 128];
    __shared__ __attribute__((aligned(16))) f16 qh[64];
    __shared__ float red[4];
    // ---- every independent load first (all unconditional); the LayerNorm
    // operands (and the fused self-attention's partials) lead, so the LN
    // waits for them while the K / V / Wq requests are still in flight ----
    constexpr int H2 = 2 * KC;  // heads: n / 64
    float4 rp[H2], rbo, rx;
    const bool rpart = a.res_parts != nullptr && tid < n / 4;
    if (rpart) {
        const float *pp = a.res_parts + (int64_t)b * H2 * n + 4 * tid;
#pragma unroll
        for (int hh = 0; hh < H2; ++hh) rp[hh] = *(const float4 *)(pp + (int64_t)hh * n);
        rbo = *(const float4 *)(a.res_bias + 4 * tid);
        rx = *(const float4 *)(a.x + (int64_t)b * n + 4 * tid);
    }
    constexpr int XLNV = (KC * 128 + 255) / 256;  // n = KC * 128
    float4 xv[XLNV], gw[XLNV], gb[XLNV];
    if (w == 0) {
        ln_load_params(a.ln_w, a.ln_b, n, lane, gw, gb);
        if (!a.res_parts) ln_load_row(a.x + (int64_t)b * n, n, lane, xv);
    }
    const int key = c * DA_CK + (tid >> 1), half = tid & 1;
    half8 kf[4];
    {
        const f16 *kr = (const f16 *)a.K + (int64_t)(b / a.clip_div) * a.clip_stride + (int64_t)(key < M ? key : M - 1) * n +
                        h * 64 + half * 32;
#pragma unroll
        for (int i = 0; i < 4; ++i) kf[i] = *(const half8 *)(kr + 8 * i);
    }
    half8 vf[4];
    if (MODE == 1) xattn_load_v(a, c, h, b, M, vf);
    half8 wq[4][KC];
    float bqr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = h * 64 + w * 16 + q * 4 + i;
        const f16 *wr = (const f16 *)a.Wq + (int64_t)r * n + l16 * 8;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) wq[i][kc] = *(const half8 *)(wr + kc * 128);
        bqr[i] = a.bq[r];
    }
    if (a.res_parts) {
        // the fused self-attention's residual update: x + (bo + sum over the
        // H heads of its output-projection partials), in head order; block
        // (0, 0, b) stores it for the rest of the layer (ping-pong buffer)
        __shared__ __attribute__((aligned(16))) float xnew[KC * 128];
        for (int j = tid; j < n / 4; j += 256) {
            if (j != tid) {  // second pass (n > 1024): operands not prefetched
                const float *pp = a.res_parts + (int64_t)b * H2 * n + 4 * j;
#pragma unroll
                for (int hh = 0; hh < H2; ++hh) rp[hh] = *(const float4 *)(pp + (int64_t)hh * n);
                rbo = *(const float4 *)(a.res_bias + 4 * j);
                rx = *(const float4 *)(a.x + (int64_t)b * n + 4 * j);
            }
            float4 sm = rp[0];
#pragma unroll
            for (int hh = 1; hh < H2; ++hh) {
                sm.x = sm.x + rp[hh].x; sm.y = sm.y + rp[hh].y; sm.z = sm.z + rp[hh].z; sm.w = sm.w + rp[hh].w;
            }
            float4 v;
            v.x = (rbo.x + sm.x) + rx.x; v.y = (rbo.y + sm.y) + rx.y;
            v.z = (rbo.z + sm.z) + rx.z; v.w = (rbo.w + sm.w) + rx.w;
            *(float4 *)(xnew + 4 * j) = v;
            if (c == 0 && h == 0) *(float4 *)(a.x_out + (int64_t)b * n + 4 * j) = v;
        }
        __syncthreads();
        if (w == 0) {
            ln_load_row(xnew, n, lane, xv);
            ln_regs_to_lds(xv, n, gw, gb, xs, lane);
        }
    } else if (w == 0) {
        ln_regs_to_lds(xv, n, gw, gb, xs, lane);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float acc = 0.0f;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) acc = dot8(wq[i][kc], *(const half8 *)(xs + kc * 128 + l16 * 8), acc);
        acc = red16_sum(acc);
        if (l16 == 0) qh[w * 16 + q * 4 + i] = f16_rt((acc + bqr[i]) * a.qscale);
    }
    __syncthreads();
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) s = dot8(kf[i], *(const half8 *)(qh + half * 32 + 8 * i), s);
    s = xstep<XSum, 1>(s);
    float *S = a.S + ((int64_t)b * a.H + h) * a.s_stride;
    if (half == 0 && key < M) st_x<COH>(S + key, s);
    float m = (key < M) ? s : -INFINITY;
    m = wave_max(m);
    if (lane == 0) red[w] = m;
    __syncthreads();
    if (tid == 0)
        st_x<COH>(a.cmax + ((int64_t)b * a.H + h) * a.n_chunks + c, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
    if (MODE == 0) {
        return;
    }
    // ---- arrival: this chunk's scores and max are globally visible ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        XSync *sy = a.sync + ((int64_t)b * a.H + h);
        const uint32_t epoch = (uint32_t)a.st->pos + 1u;
        __hip_atomic_fetch_add(&sy->cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        spin_until(&sy->cnt, epoch * (uint32_t)a.n_chunks, a.err);
    }
    __syncthreads();
    xattn_pv<COH>(a, c, h, b, M, vf);
}

// Phase A of cross-attention for beam rows, which all read one clip's cross
// K / V (clip_div == B): one workgroup per (chunk, head) serves every row
// (B <= 8), so the head's 64 Wq rows and the chunk's 128 keys are fetched
// once instead of B times (large-v3 x 5 beams: 197 MB -> 39 MB of Wq reads a
// layer).  Per row the arithmetic is k_dec_xattn<KC, 0>'s, op for op, so S
// and cmax are bit-identical; k_dec_attn_pv follows as in the two-kernel form.
template <int KC>
__global__ __launch_bounds__(256) void k_dec_xattn_rows(DecAttnArgs a) {
    const int c = blockIdx.x, h = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int q = lane >> 4, l16 = lane & 15;
    const int M = a.M_fixed, n = a.n, B = a.B;
    constexpr int H2 = 2 * KC, XLNV = (KC * 128 + 255) / 256;
    __shared__ __attribute__((aligned(16))) f16 xs[8][KC * 128];
    __shared__ __attribute__((aligned(16))) f16 qh[8][64];
    __shared__ __attribute__((aligned(16))) float xnew[4][KC * 128];
    __shared__ float red[8][4];
    // row-shared operands first: the chunk's keys, the head's Wq rows, bq
    const int key = c * DA_CK + (tid >> 1), half = tid & 1;
    half8 kf[4];
    {
        const f16 *kr = (const f16 *)a.K + (int64_t)(key < M ? key : M - 1) * n + h * 64 + half * 32;
#pragma unroll
        for (int i = 0; i < 4; ++i) kf[i] = *(const half8 *)(kr + 8 * i);
    }
    half8 wq[4][KC];
    float bqr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = h * 64 + w * 16 + q * 4 + i;
        const f16 *wr = (const f16 *)a.Wq + (int64_t)r * n + l16 * 8;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) wq[i][kc] = *(const half8 *)(wr + kc * 128);
        bqr[i] = a.bq[r];
    }
    float4 gw[XLNV], gb[XLNV], xv[XLNV];
    ln_load_params(a.ln_w, a.ln_b, n, lane, gw, gb);
    // LayerNorm of every row into xs: wave w takes rows w, w + 4
    for (int r = w; r < B; r += 4) {
        const float *xr = a.x + (int64_t)r * n;
        if (a.res_parts) {  // the fused self-attention's residual update, as in k_dec_xattn
            const float *pp = a.res_parts + (int64_t)r * H2 * n;
            for (int j = lane; j < n / 4; j += 64) {
                float4 rp[H2];
#pragma unroll
                for (int hh = 0; hh < H2; ++hh) rp[hh] = *(const float4 *)(pp + (int64_t)hh * n + 4 * j);
                const float4 rbo = *(const float4 *)(a.res_bias + 4 * j);
                const float4 rx = *(const float4 *)(xr + 4 * j);
                float4 sm = rp[0];
#pragma unroll
                for (int hh = 1; hh < H2; ++hh) {
                    sm.x = sm.x + rp[hh].x; sm.y = sm.y + rp[hh].y; sm.z = sm.z + rp[hh].z; sm.w = sm.w + rp[hh].w;
                }
                float4 v;
                v.x = (rbo.x + sm.x) + rx.x; v.y = (rbo.y + sm.y) + rx.y;
                v.z = (rbo.z + sm.z) + rx.z; v.w = (rbo.w + sm.w) + rx.w;
                *(float4 *)(xnew[w] + 4 * j) = v;
                if (c == 0 && h == 0) *(float4 *)(a.x_out + (int64_t)r * n + 4 * j) = v;
            }
            wave_sync();
            xr = xnew[w];
        }
        ln_load_row(xr, n, lane, xv);
        ln_regs_to_lds(xv, n, gw, gb, xs[r], lane);
        wave_sync();  // xnew[w] is rewritten by this wave's next row
    }
    __syncthreads();
    for (int r = 0; r < B; ++r) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float acc = 0.0f;
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) acc = dot8(wq[i][kc], *(const half8 *)(xs[r] + kc * 128 + l16 * 8), acc);
            acc = red16_sum(acc);
            if (l16 == 0) qh[r][w * 16 + q * 4 + i] = f16_rt((acc + bqr[i]) * a.qscale);
        }
    }
    __syncthreads();
    for (int r = 0; r < B; ++r) {
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) s = dot8(kf[i], *(const half8 *)(qh[r] + half * 32 + 8 * i), s);
        s = xstep<XSum, 1>(s);
        float *S = a.S + ((int64_t)r * a.H + h) * a.s_stride;
        if (half == 0 && key < M) S[key] = s;
        float m = (key < M) ? s : -INFINITY;
        m = wave_max(m);
        if (lane == 0) red[r][w] = m;
    }
    __syncthreads();
    if (tid < B)
        a.cmax[((int64_t)tid * a.H + h) * a.n_chunks + c] =
            fmaxf(fmaxf(red[tid][0], red[tid][1]), fmaxf(red[tid][2], red[tid][3]));
}

__global__ __launch_bounds__(256) void k_dec_attn_pv(DecAttnArgs a) {
    const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int M = a.M_fixed;
    half8 vf[4];
    xattn_load_v(a, c, h, b, M, vf);
    xattn_pv<false>(a, c, h, b, M, vf);
}

// self-attention over the KV cache (M = pos + 1 <= 512 keys): one workgroup
// per (clip, head), every K and V load issued up front.  Output goes to
// opart[b][0][n] (n_parts = 1 for the consumer).
template <int MK>  // keys covered: M = pos + 1 <= MK (64, 128, 256 or 512)
__global__ __launch_bounds__(256) void k_dec_self_attn(DecAttnArgs a) {
    constexpr int RK = MK > 256 ? 2 : 1, NVI = MK / 32;
    const int h = blockIdx.x, b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int M = a.st->pos + 1;
    const int n = a.n;
    __shared__ float redf[4];
    __shared__ double redd[4];
    __shared__ __attribute__((aligned(16))) uint16_t P[MK];
    if (M > MK && tid == 0 && a.err) atomicOr(a.err, 2u);  // host bucketing error: flagged, never silent
    __shared__ float ored[4][64];
    const f16 *qr = (const f16 *)a.q + (int64_t)b * n + h * 64;
    if (a.reset_amax && h == 0 && b == 0 && blockIdx.z == 0)
        for (int i = tid; i < a.B * AMAX_SHARDS; i += 256) a.reset_amax[i] = 0ull;
    // cache row of key j: slot b, or (beam search) the slot holding the
    // hypothesis' history; keys past M load row M - 1 (finite, masked below).
    // Scores: thread t owns keys t and t + 256; PV: thread owns d-octet
    // (tid & 7) and keys (tid >> 3) + 32 i.
    const int doct = tid & 7, jg = tid >> 3;
    int jk[RK], jv[NVI];
    int64_t sk[RK], sv[NVI];
#pragma unroll
    for (int r = 0; r < RK; ++r) jk[r] = min(tid + 256 * r, M - 1);
#pragma unroll
    for (int i = 0; i < NVI; ++i) jv[i] = min(jg + 32 * i, M - 1);
#pragma unroll
    for (int r = 0; r < RK; ++r) sk[r] = b;
#pragma unroll
    for (int i = 0; i < NVI; ++i) sv[i] = b;
    if (a.kv_src) {  // every table load first, then every cache load
        const int32_t *src = a.kv_src + (int64_t)b * a.kv_src_stride;
        int tk[RK], tv[NVI];
#pragma unroll
        for (int r = 0; r < RK; ++r) tk[r] = src[jk[r]];
#pragma unroll
        for (int i = 0; i < NVI; ++i) tv[i] = src[jv[i]];
#pragma unroll
        for (int r = 0; r < RK; ++r) sk[r] = jk[r] < M - 1 ? tk[r] : b;
#pragma unroll
        for (int i = 0; i < NVI; ++i) sv[i] = jv[i] < M - 1 ? tv[i] : b;
    }
    half8 kv[RK][8];
#pragma unroll
    for (int r = 0; r < RK; ++r) {
        const f16 *kr = (const f16 *)a.K + sk[r] * a.clip_stride + (int64_t)jk[r] * n + h * 64;
#pragma unroll
        for (int i = 0; i < 8; ++i) kv[r][i] = *(const half8 *)(kr + 8 * i);
    }
    half8 vv[NVI];
#pragma unroll
    for (int i = 0; i < NVI; ++i)
        vv[i] = *(const half8 *)((const f16 *)a.V + sv[i] * a.clip_stride + (int64_t)jv[i] * n + h * 64 + doct * 8);
    half8 qv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) qv[i] = *(const half8 *)(qr + 8 * i);
    // fused output projection: this head's 64 Wo columns for output rows
    // tid + 256 r (the first two prefetched now, independent of the attention)
    // Split form (gridDim.z = n / 128 > 1): workgroup z owns output rows
    // [128 z, 128 z + 128), two threads per row (32 columns each); the
    // attention itself is recomputed by each of the head's workgroups
    constexpr int WOR = 2;
    const bool wsplit = gridDim.z > 1;
    half8 wov[WOR][8];
    if (a.Wo && wsplit) {
        const int orow = blockIdx.z * 128 + (tid >> 1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            wov[0][i] = wload((const half8 *)(a.Wo + (int64_t)orow * n + h * 64 + 32 * (tid & 1) + 8 * i));
    } else if (a.Wo) {
#pragma unroll
        for (int r = 0; r < WOR; ++r) {
            const int orow = min(tid + 256 * r, n - 1);
#pragma unroll
            for (int i = 0; i < 8; ++i) wov[r][i] = wload((const half8 *)(a.Wo + (int64_t)orow * n + h * 64 + 8 * i));
        }
    }
    float sc[RK];
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < RK; ++r) {
        float s = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s = dot8(kv[r][i], qv[i], s);
        sc[r] = s;
        if (tid + 256 * r < M) mx = fmaxf(mx, s);
    }
    mx = wave_max(mx);
    if (lane == 0) redf[w] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
    double sum = 0.0;
    float p[RK];
#pragma unroll
    for (int r = 0; r < RK; ++r) {
        p[r] = 0.0f;
        if (tid + 256 * r < M) {
            p[r] = exp_f16_exact(sc[r] - mx);
            sum += (double)p[r];
        }
    }
    sum = wave_sum(sum);
    if (lane == 0) redd[w] = sum;
    __syncthreads();
    const float inv = (float)(1.0 / (((redd[0] + redd[1]) + redd[2]) + redd[3]));
#pragma unroll
    for (int r = 0; r < RK; ++r)
        if (tid + 256 * r < MK) P[tid + 256 * r] = f2h_bits(tid + 256 * r < M ? p[r] * inv : 0.0f);
    __syncthreads();
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < NVI; ++i) {
        const float pj = h2f_bits(P[jg + 32 * i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = o[e] + pj * (float)vv[i][e];
    }
    // the wave's 8 key groups by shuffles, then the 4 waves through LDS
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        o[e] = red_8_16_32(o[e]);
    }
    if (lane < 8)
#pragma unroll
        for (int e = 0; e < 8; ++e) ored[w][lane * 8 + e] = o[e];
    __syncthreads();
    if (!a.Wo) {
        if (tid < 64) a.opart[(int64_t)b * n + h * 64 + tid] = ((ored[0][tid] + ored[1][tid]) + ored[2][tid]) + ored[3][tid];
        return;
    }
    __shared__ __attribute__((aligned(16))) f16 oh[64];
    if (tid < 64) oh[tid] = f16_rt(((ored[0][tid] + ored[1][tid]) + ored[2][tid]) + ored[3][tid]);  // f16 input of Wo
    __syncthreads();
    half8 ov[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) ov[i] = *(const half8 *)(oh + 8 * i);
    float *dst = a.wo_parts + ((int64_t)b * a.H + h) * n;
    if (wsplit) {
        const int part = tid & 1;
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) acc = dot8(wov[0][i], part ? ov[4 + i] : ov[i], acc);
        const float other = __uint_as_float(dpp_xor1(__float_as_uint(acc)));
        if (part == 0) dst[blockIdx.z * 128 + (tid >> 1)] = acc + other;  // summed by the next kernel's prologue
        return;
    }
    for (int r = 0; r * 256 < n; ++r) {
        const int orow = tid + 256 * r;
        half8 wr[8];
        if (r < WOR) {
#pragma unroll
            for (int i = 0; i < 8; ++i) wr[i] = r == 0 ? wov[0][i] : wov[1][i];
        } else {
            const int oc = min(orow, n - 1);
#pragma unroll
            for (int i = 0; i < 8; ++i) wr[i] = wload((const half8 *)(a.Wo + (int64_t)oc * n + h * 64 + 8 * i));
        }
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc = dot8(wr[i], ov[i], acc);
        if (orow < n) dst[orow] = acc;  // summed by the next kernel's prologue
    }
}


// Phase A of cross-attention with the query given (f32 models: q =
// f16((Wq LN(x) + bq) * qscale) comes from the DEC_Q GEMV, whose f32 weights
// the score kernels cannot fold in): the chunk's scores -> S, its max -> cmax,
// with k_dec_xattn's key / half-row split and combine; k_dec_attn_pv follows.
__global__ __launch_bounds__(256) void k_dec_xscore_q(DecAttnArgs a) {
    const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int M = a.M_fixed, n = a.n;
    __shared__ float red[4];
    const int key = c * DA_CK + (tid >> 1), half = tid & 1;
    const f16 *kr = (const f16 *)a.K + (int64_t)(b / a.clip_div) * a.clip_stride + (int64_t)(key < M ? key : M - 1) * n +
                    h * 64 + half * 32;
    const f16 *qr = (const f16 *)a.q + (int64_t)b * n + h * 64 + half * 32;
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) s = dot8(*(const half8 *)(kr + 8 * i), *(const half8 *)(qr + 8 * i), s);
    s = xstep<XSum, 1>(s);
    float *S = a.S + ((int64_t)b * a.H + h) * a.s_stride;
    if (half == 0 && key < M) S[key] = s;
    float m = (key < M) ? s : -INFINITY;
    m = wave_max(m);
    if (lane == 0) red[w] = m;
    __syncthreads();
    if (tid == 0) a.cmax[((int64_t)b * a.H + h) * a.n_chunks + c] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

const Tune kTuneDefault{};

hipError_t launch_dec_attn(hipStream_t s, const DecAttnArgs &a) {
    const Tune &tn = tune_of(a.tune);
    if (a.M_fixed == 0) {  // self-attention: M = pos + 1 <= 512
        if (a.n_chunks != 1 || (a.Wo && !a.wo_parts)) return hipErrorInvalidValue;
        // fused output projection split over n / 128 workgroups per head
        const int S = (a.Wo && a.n % 128 == 0) ? a.n / 128 : 1;
        const dim3 grid(a.H, a.B, S);
        switch (a.mk) {
            case 64: hipLaunchKernelGGL(k_dec_self_attn<64>, grid, dim3(256), 0, s, a); break;
            case 128: hipLaunchKernelGGL(k_dec_self_attn<128>, grid, dim3(256), 0, s, a); break;
            case 256: hipLaunchKernelGGL(k_dec_self_attn<256>, grid, dim3(256), 0, s, a); break;
            case 512: hipLaunchKernelGGL(k_dec_self_attn<512>, grid, dim3(256), 0, s, a); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (a.M_fixed > 2048 || a.n_chunks > 16 || a.n_chunks * DA_CK < a.M_fixed || a.n % 128 ||
        (a.res_parts && (a.H * 64 != a.n || !a.res_bias || !a.x_out || a.x_out == a.x)))
        return hipErrorInvalidValue;
    dim3 grid(a.n_chunks, a.H, a.B);
    if (!a.Wq) {  // query precomputed (f32 models)
        if (!a.q || a.res_parts) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_dec_xscore_q, grid, dim3(256), 0, s, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_dec_attn_pv, grid, dim3(256), 0, s, a);
        return hipGetLastError();
    }
    // cooperative single kernel while the grid stays far inside residency
    // (<= 2 workgroups per CU) and the Wq rows fit the register budget;
    // otherwise the two-kernel form
    const bool coop = a.sync && a.n_chunks * a.H * a.B <= CHAIN_COOP_MAX && a.n <= 768;
    // beam rows sharing one clip: phase A once per (chunk, head) for all rows
    // (auto: n > 768, where the head's Wq rows dominate a workgroup's reads —
    // large-v3 x 5 beams 498 -> 448 ms decode; small x 5 beams is faster per
    // row, 122 vs 132 ms, as 144 workgroups serialising 5 rows under-fill)
    if (!coop && (tn.xattn_rows == 2 || (tn.xattn_rows == 1 && a.n > 768)) && a.B > 1 && a.B <= 8 &&
        a.clip_div == a.B) {
        const dim3 g1(a.n_chunks, a.H, 1);
#define XR(KC)                                                                   \
    case KC:                                                                     \
        hipLaunchKernelGGL((k_dec_xattn_rows<KC>), g1, dim3(256), 0, s, a);      \
        break;
        switch (a.n / 128) {
            XR(1) XR(2) XR(3) XR(4) XR(5) XR(6) XR(8) XR(10)
            default: return hipErrorInvalidValue;
        }
#undef XR
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_dec_attn_pv, grid, dim3(256), 0, s, a);
        return hipGetLastError();
    }
#define XA(KC)                                                                                  \
    case KC:                                                                                    \
        if (coop) hipLaunchKernelGGL((k_dec_xattn<KC, 1>), grid, dim3(256), 0, s, a);          \
        else hipLaunchKernelGGL((k_dec_xattn<KC, 0>), grid, dim3(256), 0, s, a);               \
        break;
    switch (a.n / 128) {
        XA(1) XA(2) XA(3) XA(4) XA(5) XA(6) XA(8) XA(10)
        default: return hipErrorInvalidValue;
    }
#undef XA
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || coop) return e;
    hipLaunchKernelGGL(k_dec_attn_pv, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---- timestamp sampling: one workgroup over the vocabulary -----------------
// p_i = exp(l_i - lse) in double.  First generated token: argmax over the
// timestamp ids > beg (whisper_sample_timestamp).  Later: if the summed
// timestamp probability (ids >= beg) exceeds the largest text probability
// (ids < beg) the argmax over ids >= beg, else the argmax over every id but
// sot / solm / not (whisper_sample_best); ties to the lowest id.  Records
// {id, tid = argmax over ids >= beg, p, pt = max_ts / (sum_ts + 1e-10), ptsum}.
__device__ __forceinline__ unsigned long long ts_key(float v, int id) {
    return ((unsigned long long)ord_f32(v) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)id);
}
__device__ __forceinline__ int ts_key_id(unsigned long long k) { return (int)(0xffffffffu - (uint32_t)(k & 0xffffffffu)); }

__global__ __launch_bounds__(1024) void k_ts_sample(TsArgs a) {
    const int pos = a.st->pos;
    if (pos < a.feed_len) return;  // still feeding the prompt
    const int t = pos - a.feed_len;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    __shared__ float smax[16];
    __shared__ double ssum[16], sts[16];
    __shared__ unsigned long long sk[3][16];
    float mx = -INFINITY;
    unsigned long long k_all = 0, k_ts = 0, k_ts1 = 0, k_tx = 0;
    for (int i = tid; i < a.V; i += 1024) {
        const float l = a.logits[i];
        mx = fmaxf(mx, l);
        const unsigned long long k = ts_key(l, i);
        if (i >= a.beg) k_ts = k > k_ts ? k : k_ts;
        else k_tx = k > k_tx ? k : k_tx;
        if (i > a.beg) k_ts1 = k > k_ts1 ? k : k_ts1;
        if (i != a.sot && i != a.solm && i != a.not_) k_all = k > k_all ? k : k_all;
    }
    mx = wave_max(mx);
    k_all = wave_max_u64(k_all);
    k_ts = wave_max_u64(k_ts);
    k_ts1 = wave_max_u64(k_ts1);
    k_tx = wave_max_u64(k_tx);
    __shared__ unsigned long long stx[16];
    if (lane == 0) { smax[w] = mx; sk[0][w] = k_all; sk[1][w] = k_ts; sk[2][w] = k_ts1; stx[w] = k_tx; }
    __syncthreads();
    mx = smax[0];
    k_all = sk[0][0]; k_ts = sk[1][0]; k_ts1 = sk[2][0]; k_tx = stx[0];
    for (int i = 1; i < 16; ++i) {
        mx = fmaxf(mx, smax[i]);
        k_all = sk[0][i] > k_all ? sk[0][i] : k_all;
        k_ts = sk[1][i] > k_ts ? sk[1][i] : k_ts;
        k_ts1 = sk[2][i] > k_ts1 ? sk[2][i] : k_ts1;
        k_tx = stx[i] > k_tx ? stx[i] : k_tx;
    }
    double s = 0.0, st = 0.0;
    for (int i = tid; i < a.V; i += 1024) {
        const double e = exp((double)a.logits[i] - (double)mx);
        s += e;
        if (i >= a.beg) st += e;
    }
    s = wave_sum(s);
    st = wave_sum(st);
    if (lane == 0) { ssum[w] = s; sts[w] = st; }
    __syncthreads();
    if (tid != 0) return;
    double Z = 0.0, TS = 0.0;
    for (int i = 0; i < 16; ++i) { Z += ssum[i]; TS += sts[i]; }
    const int id_ts = ts_key_id(k_ts), id_tx = ts_key_id(k_tx);
    const double p_maxts = exp((double)a.logits[id_ts] - (double)mx) / Z;
    const double p_maxtx = exp((double)a.logits[id_tx] - (double)mx) / Z;
    const double sum_ts = TS / Z;
    int id;
    if (t == 0) id = ts_key_id(k_ts1);
    else if (sum_ts > p_maxtx) id = id_ts;
    else id = ts_key_id(k_all);
    a.tok_out[0] = id;
    if (t < a.max_rec) {
        TsRec r;
        r.id = id;
        r.tid = id_ts;
        r.p = (float)(exp((double)a.logits[id] - (double)mx) / Z);
        r.pt = (float)(p_maxts / (sum_ts + 1e-10));
        r.ptsum = (float)sum_ts;
        r.pad = 0;
        a.rec[t] = r;
    }
}

hipError_t launch_ts_sample(hipStream_t s, const TsArgs &a) {
    if (a.V < a.beg + 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ts_sample, dim3(1), dim3(1024), 0, s, a);
    return hipGetLastError();
}

// records the token produced by the last step (the in-step record happens in
// the first layer's QKV prologue): one wave per clip
__global__ __launch_bounds__(64) void k_dec_record(DecEmbedArgs a) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const int pos = a.st->pos;
    const int32_t tok = shard_token(a.amax + b * AMAX_SHARDS, lane);
    if (lane == 0 && pos >= a.feed_len) a.tokens_out[b * a.out_stride + (pos - a.feed_len)] = tok;
}

hipError_t launch_dec_embed(hipStream_t s, const DecEmbedArgs &a) {
    if (!a.record_only) return hipErrorInvalidValue;  // the embedding is fused into layer 0's QKV kernel
    hipLaunchKernelGGL(k_dec_record, dim3(a.B), dim3(64), 0, s, a);
    return hipGetLastError();
}


// ============================================================================
// beam search step (config C5; semantics in oracle/wmi_oracle.h)
// ============================================================================
// (value desc, id asc) as one unsigned key: larger key = earlier in the order
__device__ __forceinline__ unsigned long long beam_key(float v, int id) {
    return ((unsigned long long)ord_f32(v) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)id);
}


// one vocabulary split of one row: split max, sum exp(logit - max) (double)
// and the split's top-(K+1)
__global__ __launch_bounds__(256) void k_beam_topk(BeamArgs a) {
    const int sp = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (a.st->pos < a.feed_len || a.bs->done || b >= a.bs->n_active) {
        return;
    }
    __shared__ float redf[4];
    __shared__ double redd[4];
    __shared__ unsigned long long redk[4];
    constexpr int U = 16;  // split length <= 4096
    const int chunk = (a.V + BEAM_NS - 1) / BEAM_NS, lo = sp * chunk, hi = min(a.V, lo + chunk);
    const float *row = a.logits + (int64_t)b * a.V;
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = lo + tid + 256 * u;
        v[u] = row[i < hi ? i : lo];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = lo + tid + 256 * u;
        if (i >= hi || i == a.suppress_id) v[u] = -INFINITY;
    }
    float m = -INFINITY;
#pragma unroll
    for (int u = 0; u < U; ++u) m = fmaxf(m, v[u]);
    m = wave_max(m);
    if (lane == 0) redf[w] = m;
    __syncthreads();
    m = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
    double sum = 0.0;
    if (m > -INFINITY)
#pragma unroll
        for (int u = 0; u < U; ++u) sum += exp((double)v[u] - (double)m);
    sum = wave_sum(sum);
    if (lane == 0) redd[w] = sum;
    BeamPart *out = a.parts + (int64_t)b * BEAM_NS + sp;
    uint32_t taken = 0;
    for (int r = 0; r <= a.K; ++r) {
        unsigned long long best = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = lo + tid + 256 * u;
            const unsigned long long k = (i < hi && !((taken >> u) & 1u)) ? beam_key(v[u], i) : 0ull;
            best = k > best ? k : best;
        }
        best = wave_max_u64(best);
        if (lane == 0) redk[w] = best;
        __syncthreads();
        unsigned long long k0 = redk[0];
#pragma unroll
        for (int i = 1; i < 4; ++i) k0 = redk[i] > k0 ? redk[i] : k0;
        const int id = (int)(0xffffffffu - (uint32_t)(k0 & 0xffffffffull));
        const int rel = id - lo;
        if (k0 && (rel & 255) == tid) taken |= 1u << (rel >> 8);
        if (tid == 0) {
            out->val[r] = k0 ? unord_f32((uint32_t)(k0 >> 32)) : -INFINITY;
            out->id[r] = k0 ? id : -1;
        }
        __syncthreads();
    }
    if (tid == 0) {
        out->m = m;
        out->sum = ((redd[0] + redd[1]) + redd[2]) + redd[3];
    }
}

// candidate i before candidate j in the ranking (score desc, beam asc, rank asc)
__device__ __forceinline__ bool cand_before(double si, int bi, int ri, double sj, int bj, int rj) {
    if (si != sj) return si > sj;
    if (bi != bj) return bi < bj;
    return ri < rj;
}

// one workgroup: merge the splits, rank the K x (K+1) candidates, fill the
// next hypotheses, record finished ones, and re-point the KV history table
__global__ __launch_bounds__(256) void k_beam_select(BeamArgs a) {
    BeamState *bs = a.bs;
    const int pos = a.st->pos;
    if (pos < a.feed_len || bs->done) {
        return;
    }
    const int t = pos - a.feed_len, K = a.K, TK = K + 1;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int NC = BEAM_MAX * BEAM_TK;
    __shared__ double lse[BEAM_MAX];
    __shared__ float cval[NC];
    __shared__ int cid[NC];
    __shared__ double cscore[NC];
    __shared__ int order[NC];
    __shared__ int sel_parent[BEAM_MAX], sel_tok[BEAM_MAX], n_new_s;
    __shared__ double sel_score[BEAM_MAX];
    __shared__ int32_t src_old[BEAM_MAX][512];
    const int na_old = bs->n_active;
    // 1. per active row: log-sum-exp and the row's top-(K+1) over the splits
    for (int b = w; b < na_old; b += 4) {
        const BeamPart *pp = a.parts + (int64_t)b * BEAM_NS;
        const float pm = lane < BEAM_NS ? pp[lane].m : -INFINITY;
        const double ps = lane < BEAM_NS ? pp[lane].sum : 0.0;
        const float M = wave_max(pm);
        const double S = wave_sum(pm > -INFINITY ? ps * exp((double)pm - (double)M) : 0.0);
        if (lane == 0) lse[b] = (double)M + log(S);
        unsigned long long key[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int c = lane + 64 * k;
            key[k] = 0ull;
            if (c < BEAM_NS * TK) {
                const int id = pp[c / TK].id[c % TK];
                if (id >= 0) key[k] = beam_key(pp[c / TK].val[c % TK], id);
            }
        }
        for (int r = 0; r < TK; ++r) {
            unsigned long long best = key[0] > key[1] ? key[0] : key[1];
            best = key[2] > best ? key[2] : best;
            best = wave_max_u64(best);
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if (key[k] == best) key[k] = 0ull;
            if (lane == 0) {
                cval[b * TK + r] = unord_f32((uint32_t)(best >> 32));
                cid[b * TK + r] = (int)(0xffffffffu - (uint32_t)(best & 0xffffffffull));
            }
        }
    }
    __syncthreads();
    // 2. scores and ranking
    const int nc = na_old * TK;
    if (tid < nc) cscore[tid] = bs->score[tid / TK] + ((double)cval[tid] - lse[tid / TK]);
    __syncthreads();
    if (tid < nc) {
        int rank = 0;
        const double si = cscore[tid];
        const int bi = tid / TK, ri = tid % TK;
        for (int j = 0; j < nc; ++j)
            if (cand_before(cscore[j], j / TK, j % TK, si, bi, ri)) ++rank;
        order[rank] = tid;
    }
    // history table of the parents, positions < pos - 1
    for (int i = tid; i < na_old * (pos - 1); i += 256) {
        const int r = i / (pos - 1), j = i - r * (pos - 1);
        src_old[r][j] = a.kv_src[r * a.tctx + j];
    }
    __syncthreads();
    // 3. walk the ranking
    if (tid == 0) {
        int na = 0, nf = bs->n_fin;
        for (int k = 0; k < nc && na < K; ++k) {
            const int c = order[k];
            if (cid[c] == a.eot) {
                if (nf < K) {
                    bs->fin_t[nf] = t;
                    bs->fin_beam[nf] = c / TK;
                    bs->fin_score[nf] = cscore[c];
                    ++nf;
                }
                continue;
            }
            sel_parent[na] = c / TK;
            sel_tok[na] = cid[c];
            sel_score[na] = cscore[c];
            ++na;
        }
        n_new_s = na;
        bs->n_fin = nf;
        bs->n_active = na;
        bs->n_steps = t + 1;
        if (nf >= K || t + 1 >= a.max_tokens) bs->done = 1;
    }
    __syncthreads();
    // 4. next hypotheses: scores, fed tokens, back-pointers, KV history table
    const int nn = n_new_s;
    if (tid < nn) {
        bs->score[tid] = sel_score[tid];
        bs->tok[tid] = sel_tok[tid];
        a.hist_parent[t * BEAM_MAX + tid] = sel_parent[tid];
        a.hist_tok[t * BEAM_MAX + tid] = sel_tok[tid];
    }
    for (int i = tid; i < nn * pos; i += 256) {
        const int sl = i / pos, j = i - sl * pos, p = sel_parent[sl];
        a.kv_src[sl * a.tctx + j] = j < pos - 1 ? src_old[p][j] : p;
    }
}

hipError_t launch_beam_step(hipStream_t s, const BeamArgs &a) {
    if (a.K < 1 || a.K > BEAM_MAX || a.tctx > 512 || (a.V + BEAM_NS - 1) / BEAM_NS > 4096)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_beam_topk, dim3(BEAM_NS, a.K), dim3(256), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_beam_select, dim3(1), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace wmi

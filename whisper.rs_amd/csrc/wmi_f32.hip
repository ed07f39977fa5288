// wmi_f32.hip — gfx950 kernels for f32 (ggml ftype 0) Whisper files.
//
// The reference loads f32 weight files (main.rs:817-821, 1423-1427); ggml's
// f32 x f32 mul_mat and conv_1d_*_f32 then round NEITHER operand to f16.  The
// f16 kernels round the activation once in its producer, so f32 files get
// their own matrix kernels here; everything else of the path (mel, LayerNorm,
// flash attention with f16 Q/K/V — main.rs:1898-1920 copies them to F16 for
// every weight type —, the f16 KV caches, beam / timestamp kernels) is shared.
//   * k_gemm32: C = A B^T on v_mfma_f32_32x32x2_f32 (f32 products, f32
//     accumulation), 2x2 waves, BK = 16, double-buffered LDS, the f16 GEMM's
//     fused epilogues (wmi_gemm_epi.h).  A is f32, or f16 where the producer's
//     values are f16 table outputs (GELU), which f32 holds exactly.
//   * k_dec_gemv32: the decoder GEMVs (LayerNorm / embedding / partial-sum
//     prologues, the DEC_* epilogues of k_dec_gemv) streaming f32 rows with
//     the activation rows in LDS as f32.
#include <hip/hip_runtime.h>
#include <math.h>

#include "wmi_device.h"
#include "wmi_gemm_epi.h"
#include "wmi_internal.h"

#pragma clang fp contract(off)

namespace wmi {

static inline int cdiv32(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

template <typename K>
static hipError_t allow_lds32(K *kern, size_t bytes) {
    if (bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// ============================================================================
// f32 MFMA GEMM  C[M][N] = A[M][K] * B[N][K]^T
// ============================================================================
constexpr int FBK = 16;           // k per tile (f32 elements)
constexpr int FLDS = FBK + 4;     // floats per LDS row (80 bytes)

// 4 consecutive A elements of row m from k (never across a conv tap: Cp % 4 == 0)
template <bool CONV, bool AF32>
__device__ __forceinline__ float4 g32_load_a(const GemmArgs &a, int m, int k) {
    if (m >= a.M) return make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t off;
    if (CONV) {
        const int b = m / a.conv_tout;
        const int t = m - b * a.conv_tout;
        const int tap = k / a.conv_cp;
        const int c = k - tap * a.conv_cp;
        off = ((int64_t)b * (a.conv_tin + 2) + (int64_t)t * a.conv_stride + tap) * a.conv_cp + c;
    } else {
        off = (int64_t)m * a.lda + k;
    }
    if constexpr (AF32) {
        return *(const float4 *)(a.A32 + off);
    } else {
        const half4 h = *(const half4 *)((const f16 *)a.A + off);
        return make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
    }
}

template <int BM, int BN, int EPI, bool CONV, bool AF32>
__global__ __launch_bounds__(256) void k_gemm32(GemmArgs a) {
    constexpr int TM = BM / 64, TN = BN / 64;      // 32x32 tiles per wave (2x2 waves)
    constexpr int ACH = BM / 64, BCH = BN / 64;    // float4 chunks per thread per k-tile
    __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * FLDS];
    float *As = smem;
    float *Bs = smem + 2 * BM * FLDS;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.N + BN - 1) / BN;
    const int nwg = nbm * nbn;
    int bid = blockIdx.x;
    {  // XCD-aware tile order (as k_gemm): each XCD gets a contiguous tile range
        const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
    }
    const int bn = bid % nbn, bm = bid / nbn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int nk = a.K / FBK;

    float4 ra[ACH], rb[BCH];
    auto gload = [&](int kt) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int c = tid + i * 256, row = c >> 2, col = (c & 3) * 4;
            ra[i] = g32_load_a<CONV, AF32>(a, m0 + row, kt * FBK + col);
        }
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int c = tid + i * 256, row = c >> 2, col = (c & 3) * 4;
            const int n = n0 + row;
            rb[i] = n < a.N ? *(const float4 *)(a.B32 + (int64_t)n * a.K + kt * FBK + col) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            const int c = tid + i * 256, row = c >> 2, col = (c & 3) * 4;
            *(float4 *)(As + buf * BM * FLDS + row * FLDS + col) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int c = tid + i * 256, row = c >> 2, col = (c & 3) * 4;
            *(float4 *)(Bs + buf * BN * FLDS + row * FLDS + col) = rb[i];
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
    // lane (lr, lh) feeds k = lh * 8 + s of MFMA step s: the A and B operands
    // use the same k order, so the 8 steps cover the tile's 16 k once each
    const int lr = lane & 31, lh = lane >> 5;
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) gload(kt + 1);
        const float *Ab = As + buf * BM * FLDS;
        const float *Bb = Bs + buf * BN * FLDS;
        float4 af[TM][2], bf[TN][2];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const float *p = Ab + (wm * (BM / 2) + i * 32 + lr) * FLDS + lh * 8;
            af[i][0] = *(const float4 *)p;
            af[i][1] = *(const float4 *)(p + 4);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const float *p = Bb + (wn * (BN / 2) + j * 32 + lr) * FLDS + lh * 8;
            bf[j][0] = *(const float4 *)p;
            bf[j][1] = *(const float4 *)(p + 4);
        }
#pragma unroll
        for (int st = 0; st < 8; ++st) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const float4 &av = af[i][st >> 2], &bv = bf[j][st >> 2];
                    const int e = st & 3;
                    const float x = e == 0 ? av.x : e == 1 ? av.y : e == 2 ? av.z : av.w;
                    const float y = e == 0 ? bv.x : e == 1 ? bv.y : e == 2 ? bv.z : bv.w;
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[i][j], 0, 0, 0);
                }
        }
        if (kt + 1 < nk) sstore(buf ^ 1);
        __syncthreads();
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

template <int BM, int BN, bool CONV, bool AF32>
static hipError_t gemm32_epi(hipStream_t s, int epi, const GemmArgs &a) {
    const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    dim3 grid(nwg), block(256);
#define G32_CASE(E)                                                                   \
    case E:                                                                           \
        hipLaunchKernelGGL((k_gemm32<BM, BN, E, CONV, AF32>), grid, block, 0, s, a);  \
        break;
    if constexpr (CONV) {
        switch (epi) {
            G32_CASE(EPI_CONV1)
            G32_CASE(EPI_CONV2PE)
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (epi) {
            G32_CASE(EPI_RESID)
            G32_CASE(EPI_GELU16)
            G32_CASE(EPI_QKV)
            G32_CASE(EPI_CROSSKV)
            default: return hipErrorInvalidValue;
        }
    }
#undef G32_CASE
    return hipGetLastError();
}

template <bool CONV, bool AF32>
static hipError_t gemm32_tiles(hipStream_t s, int epi, const GemmArgs &a) {
    const int64_t t128 = (int64_t)cdiv32(a.M, 128) * cdiv32(a.N, 128);
    if (t128 >= 240) return gemm32_epi<128, 128, CONV, AF32>(s, epi, a);
    return gemm32_epi<64, 64, CONV, AF32>(s, epi, a);
}

hipError_t launch_gemm32(hipStream_t s, int epi, const GemmArgs &a) {
    if (a.M <= 0 || a.N <= 0) return hipSuccess;
    if (!a.B32 || a.K <= 0 || a.K % FBK != 0) return hipErrorInvalidValue;
    if (a.conv && a.conv_cp % 4 != 0) return hipErrorInvalidValue;
    if (!a.A32 && !a.A) return hipErrorInvalidValue;
    if (a.conv) return a.A32 ? gemm32_tiles<true, true>(s, epi, a) : gemm32_tiles<true, false>(s, epi, a);
    return a.A32 ? gemm32_tiles<false, true>(s, epi, a) : gemm32_tiles<false, false>(s, epi, a);
}

// ============================================================================
// Decoder GEMV on f32 rows (SURVEY §A.7 with ggml_vec_dot_f32: the LayerNorm
// output, attention output and embedding stay f32 into the dot).
//   IN = 0: LayerNorm(x) prologue; 1: f16 input vector (GELU table values);
//   2: ordered sum of split-key attention partials; 3: embedding + LayerNorm
// A wave owns one output row at a time (lanes stride K in float4 runs, then a
// fixed butterfly); a workgroup strides over row groups of 4.
// ============================================================================
constexpr int G32_MAXB = 8;

__device__ __forceinline__ int32_t shard_token32(const unsigned long long *sh, int lane) {
    const unsigned long long k = wave_max_u64(sh[lane]);
    return (int32_t)(0xffffffffu - (uint32_t)(k & 0xffffffffull));
}

template <int EPI, int IN>
__global__ __launch_bounds__(256) void k_dec_gemv32(DecGemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
    float *xs = (float *)smraw;          // [B][K] f32 (IN != 1)
    f16 *xh = (f16 *)smraw;              // [B][K] f16 (IN == 1)
    __shared__ unsigned long long amax_s[G32_MAXB];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int K = a.K, B = a.B, N = a.N;
    if (IN == 0 || IN == 3) {
        const int pos = IN == 3 ? a.st->pos : 0;
        for (int rb = w; rb < B; rb += 4) {
            float *xr = xs + rb * K;
            if (IN == 3) {  // x = te[tok] + pe[pos] (get_rows f32, add)
                const bool fed = pos < a.feed_len;
                const int32_t tok = fed ? a.feed[rb * a.feed_stride + pos]
                                        : (a.beam_tok ? a.beam_tok[rb] : shard_token32(a.amax + rb * AMAX_SHARDS, lane));
                for (int k = lane; k < K; k += 64) {
                    const float v = a.te32[(int64_t)tok * K + k] + a.pe[(int64_t)pos * K + k];
                    xr[k] = v;
                    if (blockIdx.x == 0) a.x_out[(int64_t)rb * K + k] = v;
                }
                if (blockIdx.x == 0 && lane == 0 && !fed && a.tokens_out)
                    a.tokens_out[rb * a.out_stride + (pos - a.feed_len)] = tok;
            } else {
                for (int k = lane; k < K; k += 64) xr[k] = a.x[(int64_t)rb * K + k];
            }
            // ggml norm (double mean / variance), then * w + b; row rb is this wave's only
            double s1 = 0.0;
            for (int k = lane; k < K; k += 64) s1 += (double)xr[k];
            s1 = wave_sum(s1);
            const double mean = s1 / K;
            double s2 = 0.0;
            for (int k = lane; k < K; k += 64) {
                const double d = (double)xr[k] - mean;
                s2 += d * d;
            }
            s2 = wave_sum(s2);
            const float scale = (float)(1.0 / sqrt(s2 / K + (double)1e-5f));
            for (int k = lane; k < K; k += 64) {
                const float t = (float)((double)xr[k] - mean) * scale;
                xr[k] = a.ln_b[k] + a.ln_w[k] * t;
            }
        }
    } else if (IN == 1) {
        const uint4 *src = (const uint4 *)a.xin16;
        uint4 *dst = (uint4 *)xh;
        for (int i = tid; i < B * K / 8; i += 256) dst[i] = src[i];
    } else {
        for (int i = tid; i < B * K; i += 256) {
            const int bb = i / K, k = i - bb * K;
            const float *p = a.parts + ((int64_t)bb * a.n_parts) * K + k;
            float sacc = p[0];
            for (int c = 1; c < a.n_parts; ++c) sacc = sacc + p[(int64_t)c * K];
            xs[i] = sacc;
        }
    }
    if (EPI == DEC_LOGITS && tid < G32_MAXB) amax_s[tid] = 0ull;
    __syncthreads();
    const int pos = (EPI == DEC_QKV) ? a.st->pos : 0;
    const int nrg = (N + 3) / 4;
    for (int rg = blockIdx.x; rg < nrg; rg += gridDim.x) {
        const int o = rg * 4 + w;
        if (o >= N) continue;  // wave-uniform
        const float *wr = a.W32 + (int64_t)o * K;
        float acc[G32_MAXB];
#pragma unroll
        for (int bb = 0; bb < G32_MAXB; ++bb) acc[bb] = 0.0f;
        for (int k = 4 * lane; k < K; k += 256) {
            const float4 wv = *(const float4 *)(wr + k);
#pragma unroll
            for (int bb = 0; bb < G32_MAXB; ++bb) {
                if (bb < B) {
                    float4 xv;
                    if (IN == 1) {
                        const half4 h = *(const half4 *)(xh + bb * K + k);
                        xv = make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
                    } else {
                        xv = *(const float4 *)(xs + bb * K + k);
                    }
                    float t = acc[bb];
                    t = fmaf(wv.x, xv.x, t);
                    t = fmaf(wv.y, xv.y, t);
                    t = fmaf(wv.z, xv.z, t);
                    t = fmaf(wv.w, xv.w, t);
                    acc[bb] = t;
                }
            }
        }
        float v = 0.0f;
#pragma unroll
        for (int bb = 0; bb < G32_MAXB; ++bb)
            if (bb < B) {
                const float sm = wave_sum(acc[bb]);
                if (lane == bb) v = sm;
            }
        if (lane >= B) continue;
        const int bb = lane;
        const float bias = a.bias ? a.bias[o] : 0.0f;
        if (EPI == DEC_QKV) {
            const int n = N / 3, which = o / n, c = o - which * n;
            if (which == 0) a.out16[bb * a.ldo + c] = f2h_bits((v + bias) * a.qscale);
            else if (which == 1) a.kcache[((int64_t)bb * a.n_text_ctx + pos) * n + c] = f2h_bits(v * a.qscale);
            else a.vcache[((int64_t)bb * a.n_text_ctx + pos) * n + c] = f2h_bits(bias + v);
        } else if (EPI == DEC_Q) {
            a.out16[bb * a.ldo + o] = f2h_bits((v + bias) * a.qscale);
        } else if (EPI == DEC_GELU) {
            a.out16[bb * a.ldo + o] = a.gelu_tab[f2h_bits(v + bias)];
        } else if (EPI == DEC_RESID) {
            float *p = a.out32 + (int64_t)bb * N + o;
            *p = (v + bias) + *p;
        } else if (EPI == DEC_LOGITS) {
            a.out32[(int64_t)bb * N + o] = v;
            if (a.amax && o != a.suppress_id) {
                const unsigned long long key =
                    ((unsigned long long)ord_f32(v) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)o);
                atomicMax(&amax_s[bb], key);
            }
        }
    }
    if (EPI == DEC_LOGITS) {
        __syncthreads();
        if (a.amax && tid < B && amax_s[tid])
            atomicMax(&a.amax[tid * AMAX_SHARDS + (blockIdx.x & (AMAX_SHARDS - 1))], amax_s[tid]);
        if (blockIdx.x == 0 && tid == 0) a.st_advance->pos += 1;
    }
}

template <int EPI, int IN>
static hipError_t gemv32_launch(hipStream_t s, const DecGemvArgs &a) {
    const size_t lds = (size_t)a.B * a.K * (IN == 1 ? 2 : 4);
    hipError_t e = allow_lds32(k_dec_gemv32<EPI, IN>, lds);
    if (e != hipSuccess) return e;
    const int nrg = cdiv32(a.N, 4);
    const dim3 grid(nrg < 2048 ? nrg : 2048);
    hipLaunchKernelGGL((k_dec_gemv32<EPI, IN>), grid, dim3(256), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_dec_gemv32(hipStream_t s, int epi, const DecGemvArgs &a) {
    if (a.B < 1 || a.B > G32_MAXB || a.K % 128 || !a.W32) return hipErrorInvalidValue;
    const int in = a.te32 ? 3 : (a.ln_w ? 0 : (a.parts ? 2 : 1));
    if (in == 3 && a.te) return hipErrorInvalidValue;
    if (epi == DEC_QKV && in == 3) return gemv32_launch<DEC_QKV, 3>(s, a);
    if (epi == DEC_QKV && in == 0) return gemv32_launch<DEC_QKV, 0>(s, a);
    if (epi == DEC_Q && in == 0) return gemv32_launch<DEC_Q, 0>(s, a);
    if (epi == DEC_GELU && in == 0) return gemv32_launch<DEC_GELU, 0>(s, a);
    if (epi == DEC_RESID && in == 1) return gemv32_launch<DEC_RESID, 1>(s, a);
    if (epi == DEC_RESID && in == 2) return gemv32_launch<DEC_RESID, 2>(s, a);
    if (epi == DEC_LOGITS && in == 0) return gemv32_launch<DEC_LOGITS, 0>(s, a);
    return hipErrorInvalidValue;
}

}  // namespace wmi

// wmi_device.h — device helpers shared by the gfx950 kernel translation units
// (wmi_kernels.hip, wmi_persist.hip): f16 types and bit casts, wave
// reductions, the ggml exp-table value, the f16 dot-product step.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace wmi {

typedef _Float16 f16;
typedef f16 half8 __attribute__((ext_vector_type(8)));
typedef f16 half4 __attribute__((ext_vector_type(4)));
typedef f16 half2v __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// f32 -> f16 of an f32 value, rounded once more (ggml's order: the f32
// result first, then the f16 store).  The backend otherwise folds
// fptrunc(fmul / fadd x, y) into v_fma_mixlo_f16, ONE rounding of the exact
// product / sum — 1-ulp differences in ~1e-4 of the outputs (cross K, the
// decoder's q and P16), whatever -ffp-contract says.  A canonicalize between
// the two blocks the fold and costs no instruction (an empty asm there did
// the same but slowed the decoder's F phase 0.4 us a layer).
__device__ __forceinline__ f16 f16_rt(float x) { return (f16)__builtin_canonicalizef(x); }
__device__ __forceinline__ uint16_t f2h_bits(float x) { return __builtin_bit_cast(uint16_t, f16_rt(x)); }
__device__ __forceinline__ float h2f_bits(uint16_t b) { return (float)__builtin_bit_cast(f16, b); }
// order-preserving map of f32 onto u32 (argmax keys)
__device__ __forceinline__ uint32_t ord_f32(float v) {
    const uint32_t u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
// ---- cross-lane exchange without the LDS ------------------------------------
// __shfl_xor lowers to ds_bpermute_b32, an LDS round trip (~100+ cycles) per
// butterfly step.  These use DPP (row_ror / quad_perm within 16-lane rows) and
// gfx950's v_permlane16_swap / v_permlane32_swap across rows.  Every reduction
// reproduces its __shfl_xor butterfly bit for bit: each step adds (or maxes)
// the same two values in the same order —
//   xor 32 / xor 16: the swap hands every lane its partner's value;
//   xor 8: row_ror 8 IS lane ^ 8 within a 16-lane row;
//   xor 4 after xor 8: values are symmetric under ^ 8, so row_ror 4 (lane - 4
//     mod 16) carries the value of lane ^ 4;
//   xor 2 / xor 1: quad_perm [2,3,0,1] / [1,0,3,2] are exact.
template <int N>
__device__ __forceinline__ uint32_t dpp_ror(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x120 + N, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_xor2(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4e, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_xor1(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xb1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_xor3(uint32_t x) {  // quad_perm [3,2,1,0]
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x1b, 0xf, 0xf, false);
}
// {own, partner} in some order for lane ^ 16 / lane ^ 32
__device__ __forceinline__ void swap16(uint32_t x, uint32_t &a, uint32_t &b) {
    const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    a = p[0];
    b = p[1];
}
__device__ __forceinline__ void swap32(uint32_t x, uint32_t &a, uint32_t &b) {
    const auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    a = p[0];
    b = p[1];
}
// value of lane + 16 (rows 0 and 2 receive rows 1 and 3; rows 1 and 3 get junk)
__device__ __forceinline__ float from_next_row(float v) {
    uint32_t a, b;
    swap16(__float_as_uint(v), a, b);
    return __uint_as_float(b);
}

struct XSum {
    __device__ static float op(float a, float b) { return a + b; }
    __device__ static double op(double a, double b) { return a + b; }
};
struct XMax {
    __device__ static float op(float a, float b) { return fmaxf(a, b); }
};
__device__ __forceinline__ uint32_t lo32(double d) { return (uint32_t)__double_as_longlong(d); }
__device__ __forceinline__ uint32_t hi32(double d) { return (uint32_t)((uint64_t)__double_as_longlong(d) >> 32); }
__device__ __forceinline__ double mk64(uint32_t hi, uint32_t lo) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

template <typename Op, int STEP>
__device__ __forceinline__ float xstep(float v) {
    const uint32_t u = __float_as_uint(v);
    if constexpr (STEP == 32 || STEP == 16) {
        uint32_t a, b;
        if constexpr (STEP == 32) swap32(u, a, b);
        else swap16(u, a, b);
        return Op::op(__uint_as_float(a), __uint_as_float(b));
    } else {
        const uint32_t t = STEP == 8 ? dpp_ror<8>(u) : STEP == 4 ? dpp_ror<4>(u) : STEP == 2 ? dpp_xor2(u) : dpp_xor1(u);
        return Op::op(v, __uint_as_float(t));
    }
}
template <typename Op, int STEP>
__device__ __forceinline__ double xstep(double v) {
    const uint32_t l = lo32(v), h = hi32(v);
    if constexpr (STEP == 32 || STEP == 16) {
        uint32_t la, lb, ha, hb;
        if constexpr (STEP == 32) { swap32(l, la, lb); swap32(h, ha, hb); }
        else { swap16(l, la, lb); swap16(h, ha, hb); }
        return Op::op(mk64(ha, la), mk64(hb, lb));
    } else {
        const uint32_t tl = STEP == 8 ? dpp_ror<8>(l) : STEP == 4 ? dpp_ror<4>(l) : STEP == 2 ? dpp_xor2(l) : dpp_xor1(l);
        const uint32_t th = STEP == 8 ? dpp_ror<8>(h) : STEP == 4 ? dpp_ror<4>(h) : STEP == 2 ? dpp_xor2(h) : dpp_xor1(h);
        return Op::op(v, mk64(th, tl));
    }
}
// sum over the 16 lanes of a row, butterfly order 8, 4, 2, 1
__device__ __forceinline__ float red16_sum(float v) {
    v = xstep<XSum, 8>(v);
    v = xstep<XSum, 4>(v);
    v = xstep<XSum, 2>(v);
    return xstep<XSum, 1>(v);
}
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    v = xstep<XSum, 32>(v);
    v = xstep<XSum, 16>(v);
    v = xstep<XSum, 8>(v);
    v = xstep<XSum, 4>(v);
    v = xstep<XSum, 2>(v);
    return xstep<XSum, 1>(v);
}
__device__ __forceinline__ float wave_max(float v) {
    v = xstep<XMax, 32>(v);
    v = xstep<XMax, 16>(v);
    v = xstep<XMax, 8>(v);
    v = xstep<XMax, 4>(v);
    v = xstep<XMax, 2>(v);
    return xstep<XMax, 1>(v);
}
// the P.V reduction over key groups: xor 8, then 16, then 32
__device__ __forceinline__ float red_8_16_32(float v) {
    v = xstep<XSum, 8>(v);
    v = xstep<XSum, 16>(v);
    return xstep<XSum, 32>(v);
}
// max of 64-bit keys across the wave (order-free)
__device__ __forceinline__ unsigned long long u64max(unsigned long long a, unsigned long long b) { return a > b ? a : b; }
template <int STEP>
__device__ __forceinline__ unsigned long long kstep(unsigned long long k) {
    const uint32_t l = (uint32_t)k, h = (uint32_t)(k >> 32);
    if constexpr (STEP == 32 || STEP == 16) {
        uint32_t la, lb, ha, hb;
        if constexpr (STEP == 32) { swap32(l, la, lb); swap32(h, ha, hb); }
        else { swap16(l, la, lb); swap16(h, ha, hb); }
        return u64max(((unsigned long long)ha << 32) | la, ((unsigned long long)hb << 32) | lb);
    } else {
        const uint32_t tl = STEP == 8 ? dpp_ror<8>(l) : STEP == 4 ? dpp_ror<4>(l) : STEP == 2 ? dpp_xor2(l) : dpp_xor1(l);
        const uint32_t th = STEP == 8 ? dpp_ror<8>(h) : STEP == 4 ? dpp_ror<4>(h) : STEP == 2 ? dpp_xor2(h) : dpp_xor1(h);
        return u64max(k, ((unsigned long long)th << 32) | tl);
    }
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long k) {
    k = kstep<32>(k);
    k = kstep<16>(k);
    k = kstep<8>(k);
    k = kstep<4>(k);
    k = kstep<2>(k);
    return kstep<1>(k);
}
// max over the 4 rows (16-lane quarters) of a wave
__device__ __forceinline__ unsigned long long rows_max_u64(unsigned long long k) {
    k = kstep<16>(k);
    return kstep<32>(k);
}
__device__ __forceinline__ float gelu_lookup(const uint16_t *tab, float x) { return h2f_bits(tab[f2h_bits(x)]); }
// ggml's table_gelu_f16 entry for f16 input f, computed: the host builds the
// table with exactly this f32 expression (build_tables, wmi_api.cpp), one
// rounding per operation.  The device's tanhf is within an ulp of the host's,
// which moves the f16 result only where 1 + tanh cancels (x < -1.8: 235 of
// the 63 488 finite inputs, scripts/gelu_probe.py), so the encoder GEMM
// epilogues compute it for inputs >= gmin — the context's exhaustive device
// scan (k_gelu_scan) puts gmin just above the largest input that differs —
// and read the table below (+inf: the table everywhere).  The table's 128 KB
// of random 2-byte gathers were what bounded the mlp.0 epilogue.
__device__ __forceinline__ uint16_t gelu_calc_bits(float f) {
    const float t = tanhf(0.79788456080286535587989211986876f * f * (1.0f + 0.044715f * f * f));
    return f2h_bits(0.5f * f * (1.0f + t));
}
__device__ __forceinline__ uint16_t gelu_bits(const uint16_t *tab, float x, float gmin) {
    const uint16_t h = f2h_bits(x);
    const float f = h2f_bits(h);
    uint16_t r;
    if (f >= gmin) r = gelu_calc_bits(f);  // (NaN inputs fail the compare: table)
    else r = tab[h];
    return r;
}

// ggml's table_exp_f16 entry for a non-positive f16 argument, computed:
// f16((float)exp((double)x)) — the host builds the table with exactly this
// expression, and a double exp within an ulp of glibc's lands on the same
// float for every f16 input (wmi_selftest checks all of them on the device).
__device__ __forceinline__ float exp_f16_exact(float arg) {
    const f16 h = (f16)arg;
    return (float)(f16)(float)exp((double)(float)h);
}

// f16 x f16 products of 8 lanes accumulated in f32 (ggml_vec_dot_f16 step)
// q5_1 weights (repacked at load: per row K/2 bytes of nibbles in natural
// order, then per 32-block a u32 of 5th bits and a u32 {f16 d, f16 m}):
// eight weights starting at block offset sh, dequantised exactly as the host
// loader does, w = f16(q * d + m) rounded once.  Packed: two quants per dword
// as f16 (1024 + q) via v_perm + bit spread, minus 1024 (exact), then one
// v_pk_fma_f16 per pair.
__device__ __forceinline__ half8 q5_half8(uint32_t qn, uint32_t qh, uint32_t dm, int sh) {
    const uint32_t lo = qn & 0x0F0F0F0Fu, hi = (qn >> 4) & 0x0F0F0F0Fu;  // weights 0,2,4,6 / 1,3,5,7
    const uint32_t hb = qh >> sh;
    const half2v d2 = __builtin_bit_cast(half2v, __builtin_amdgcn_perm(dm, dm, 0x01000100u));
    const half2v m2 = __builtin_bit_cast(half2v, __builtin_amdgcn_perm(dm, dm, 0x03020302u));
    const half2v k1024 = {(f16)1024.0f, (f16)1024.0f};
    half8 w;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t nib = __builtin_amdgcn_perm(hi, lo, 0x0C000C00u | ((uint32_t)(4 + i) << 16) | (uint32_t)i);
        const uint32_t h5 = ((__builtin_amdgcn_ubfe(hb, 2 * i, 2)) * 0x80010u) & 0x100010u;
        const half2v q2 = __builtin_bit_cast(half2v, nib | h5 | 0x64006400u) - k1024;
        const half2v r = __builtin_elementwise_fma(q2, d2, m2);
        w[2 * i] = r[0];
        w[2 * i + 1] = r[1];
    }
    return w;
}

__device__ __forceinline__ float dot8(const half8 w, const half8 x, float acc) {
    acc = __builtin_amdgcn_fdot2(half2v{w[0], w[1]}, half2v{x[0], x[1]}, acc, false);
    acc = __builtin_amdgcn_fdot2(half2v{w[2], w[3]}, half2v{x[2], x[3]}, acc, false);
    acc = __builtin_amdgcn_fdot2(half2v{w[4], w[5]}, half2v{x[4], x[5]}, acc, false);
    acc = __builtin_amdgcn_fdot2(half2v{w[6], w[7]}, half2v{x[6], x[7]}, acc, false);
    return acc;
}

}  // namespace wmi

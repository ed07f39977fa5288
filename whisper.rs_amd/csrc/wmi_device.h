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

__device__ __forceinline__ uint16_t f2h_bits(float x) { return __builtin_bit_cast(uint16_t, (f16)x); }
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
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float gelu_lookup(const uint16_t *tab, float x) { return h2f_bits(tab[f2h_bits(x)]); }

// ggml's table_exp_f16 entry for a non-positive f16 argument, computed:
// f16((float)exp((double)x)) — the host builds the table with exactly this
// expression, and a double exp within an ulp of glibc's lands on the same
// float for every f16 input (wmi_selftest checks all of them on the device).
__device__ __forceinline__ float exp_f16_exact(float arg) {
    const f16 h = (f16)arg;
    return (float)(f16)(float)exp((double)(float)h);
}

// f16 x f16 products of 8 lanes accumulated in f32 (ggml_vec_dot_f16 step)
__device__ __forceinline__ float dot8(const half8 w, const half8 x, float acc) {
    acc = __builtin_amdgcn_fdot2(half2v{w[0], w[1]}, half2v{x[0], x[1]}, acc, false);
    acc = __builtin_amdgcn_fdot2(half2v{w[2], w[3]}, half2v{x[2], x[3]}, acc, false);
    acc = __builtin_amdgcn_fdot2(half2v{w[4], w[5]}, half2v{x[4], x[5]}, acc, false);
    acc = __builtin_amdgcn_fdot2(half2v{w[6], w[7]}, half2v{x[6], x[7]}, acc, false);
    return acc;
}

}  // namespace wmi

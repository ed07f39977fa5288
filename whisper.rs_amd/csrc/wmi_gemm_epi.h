// wmi_gemm_epi.h — fused GEMM epilogues shared by the f16 (wmi_kernels.hip)
// and f32 (wmi_f32.hip) encoder GEMMs: bias, residual, GELU table, conv
// halo rows, positional embedding, head-split Q/K/V^T and cross K/V stores.
#pragma once
#include "wmi_device.h"
#include "wmi_internal.h"

#pragma clang fp contract(off)

namespace wmi {

template <int EPI>
__device__ __forceinline__ void gemm_epi4(const GemmArgs &a, int m, int n, const float *v) {
    // v[0..3] = rows m..m+3 of column n
    if (n >= a.N) return;
    const float bias = a.bias ? a.bias[n] : 0.0f;
    if (EPI == EPI_QKV) {
        const int ns = a.n_state;
        const int which = n / ns, c = n - which * ns, h = c >> 6, d = c & 63;
        const int H = ns >> 6;
        if (which < 2) {
            uint16_t *dst = which == 0 ? a.q : a.k;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int mm = m + r;
                if (mm >= a.M) break;
                const int b = mm / a.T, t = mm - b * a.T;
                dst[(((int64_t)b * H + h) * a.Tp + t) * 64 + d] = f2h_bits(v[r] + bias);
            }
        } else {
            const int b0 = m / a.T, t0 = m - b0 * a.T;
            if (m + 3 < a.M && t0 + 3 < a.T && (t0 & 3) == 0) {
                half4 hv;
#pragma unroll
                for (int r = 0; r < 4; ++r) hv[r] = f16_rt(v[r] + bias);
                *(half4 *)(a.vt + (((int64_t)b0 * H + h) * 64 + d) * a.Tp + t0) = hv;
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int mm = m + r;
                    if (mm >= a.M) break;
                    const int b = mm / a.T, t = mm - b * a.T;
                    a.vt[(((int64_t)b * H + h) * 64 + d) * a.Tp + t] = f2h_bits(v[r] + bias);
                }
            }
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int mm = m + r;
        if (mm >= a.M) break;
        if (EPI == EPI_F32) {
            a.out32[(int64_t)mm * a.ldo + n] = v[r] + bias;
        } else if (EPI == EPI_RESID) {
            float *p = a.out32 + (int64_t)mm * a.ldo + n;
            *p = (v[r] + bias) + *p;
        } else if (EPI == EPI_GELU16) {
            a.out16[(int64_t)mm * a.ldo + n] = gelu_bits(a.gelu_tab, v[r] + bias, a.gelu_min);
        } else if (EPI == EPI_CONV1) {
            const int b = mm / a.T, t = mm - b * a.T;
            a.out16[((int64_t)b * (a.T + 2) + t + 1) * a.ldo + n] = gelu_bits(a.gelu_tab, v[r] + bias, a.gelu_min);
        } else if (EPI == EPI_CONV2PE) {
            const int b = mm / a.T, t = mm - b * a.T;
            (void)b;
            a.out32[(int64_t)mm * a.ldo + n] =
                a.pe[(int64_t)t * a.ldo + n] + h2f_bits(gelu_bits(a.gelu_tab, v[r] + bias, a.gelu_min));
        } else if (EPI == EPI_CROSSKV) {
            const int ns = a.n_state;
            const int l = n / (2 * ns), rr = n - l * 2 * ns;
            const int b = mm / a.T, t = mm - b * a.T;
            const int64_t base = (((int64_t)l * a.n_clips + b) * a.T + t) * ns;
            if (rr < ns) a.ck[base + rr] = f2h_bits(v[r] * a.kscale);
            else a.cv[base + rr - ns] = f2h_bits(v[r] + bias);
        }
    }
}

}  // namespace wmi

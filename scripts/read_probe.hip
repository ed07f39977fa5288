// read_probe.hip — per-CU rate of reading a B x n activation vector that
// every workgroup reads (the all-to-all gather's data movement without any
// hand-off).  Standalone diagnostic (not part of the product library).
//   M0 shared plain : every workgroup reads the same KB bytes, plain 16-B loads
//   M1 shared sc1   : the same with sc1 (L1-bypassing) loads
//   M2 private plain: workgroup b reads its own KB bytes (no sharing)
//   M3 shared plain, round-strided: round r reads a different copy of the
//      data (8 copies), so no line is hot in L2 from the previous round
// Each round: 16-B loads, PU in flight per thread, values summed into LDS.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int M, int PU>
__global__ __launch_bounds__(256, 1) void k_read(const unsigned char *buf, int64_t bytes, int R, float *sink) {
    const int b = blockIdx.x, t = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char *>(buf), (short)0, 0x7fffffff, 0x00020000);
    __shared__ uint32_t acc_s[256];
    uint32_t acc = 0;
    const int nq = (int)(bytes / 16);
    for (int r = 0; r < R; ++r) {
        int64_t base = 0;
        if (M == 2) base = (int64_t)b * bytes;
        if (M == 3) base = (int64_t)(r & 7) * bytes;
        for (int i0 = t; i0 < nq; i0 += 256 * PU) {
            u32x4 v[PU];
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                const int i = i0 + 256 * u;
                if (i < nq) {
                    if (M == 1) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(base + 16ll * i), 0, 16);
                    else v[u] = *(const u32x4 *)(buf + base + 16ll * i);
                } else v[u] = u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < PU; ++u) acc += v[u][0] ^ v[u][3];
        }
        acc_s[t] = acc;
        __syncthreads();
        acc += acc_s[(t + 1) & 255];
        __syncthreads();
    }
    sink[b * 256 + t] = (float)acc;
}

int main() {
    unsigned char *buf;
    float *sink;
    const int64_t cap = 64ll << 20;
    CK(hipMalloc(&buf, cap));
    CK(hipMemset(buf, 1, cap));
    CK(hipMalloc(&sink, 512 * 256 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[] = {"shared plain", "shared sc1", "private plain", "shared 8 copies"};
    auto run = [&](auto kern, int M, int PU, int64_t bytes, int G) {
        const int R = 200;
        std::vector<float> tm;
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(kern, dim3(G), dim3(256), 0, 0, buf, bytes, R, sink);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) tm.push_back(ms * 1000.f / R);
        }
        std::sort(tm.begin(), tm.end());
        printf("G=%3d %6.1f KB %-16s PU=%2d %7.3f us/round = %6.1f GB/s per CU\n", G, bytes / 1024.0, names[M], PU, tm[0],
               bytes / (tm[0] * 1e-6) / 1e9);
        fflush(stdout);
    };
    for (int64_t kb : {8, 25, 50, 100}) {
        const int64_t by = kb * 1024;
        run(k_read<0, 16>, 0, 16, by, 256);
        run(k_read<1, 16>, 1, 16, by, 256);
        run(k_read<2, 16>, 2, 16, by, 256);
        run(k_read<3, 16>, 3, 16, by, 256);
        run(k_read<0, 4>, 0, 4, by, 256);
        run(k_read<1, 4>, 1, 4, by, 256);
    }
    return 0;
}

// read_probe2.hip — is the all-to-all gather slow because its lines are
// fresh, or because every CU fetches the same few lines from memory?
// Standalone diagnostic (not part of the product library).
//
// Every round reads a region no workgroup has read before in the launch (L2
// cold), with sc1 16-byte loads, PU in flight per thread:
//   C0 shared      : all workgroups read the same S bytes of region r
//   C1 8 copies    : workgroup b reads copy b % 8 of region r (copies far apart)
//   C2 32 copies   : copy b % 32
//   C3 private     : workgroup b reads its own S bytes (no sharing at all)
//   C4 shared, L2-warm: all workgroups read region 0 every round (read_probe's M1)
// A fresh variant writes each round's region inside the launch first:
//   F0 fresh shared : round r: every workgroup stores its 1/G share of region r
//                     (sc1), arrives on a counter, waits for all G, then reads
//                     the whole region (the decoder's hand-off without tags)
//   F1 fresh 8 copies: the same, each share stored to all 8 copies, reads copy b % 8
//   FB barrier only  : F0 without the region read (the counter's price)
//   F2 fresh, 2 regions: F0 alternating between two regions (the decoder's
//                     exchange block is rewritten at the same addresses)
//   F3 fresh, 8 regions: F0 cycling over 8 regions
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int NR = 64;  // rounds (distinct regions)

template <int M, int PU>
__global__ __launch_bounds__(256, 1) void k_read2(unsigned char *buf, int64_t S, int64_t cstride, uint32_t *ctr,
                                                  float *sink) {
    const int b = blockIdx.x, t = threadIdx.x, G = gridDim.x;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, 0x7fffffff, 0x00020000);
    __shared__ uint32_t acc_s[256];
    uint32_t acc = 0;
    const int nq = (int)(S / 16);
    for (int r = 0; r < NR; ++r) {
        int64_t base = (int64_t)r * S;  // region r of copy 0
        if (M == 1 || M == 6) base += (int64_t)(b & 7) * cstride;
        if (M == 2) base += (int64_t)(b & 31) * cstride;
        if (M == 3) base = ((int64_t)r * G + b) * S;
        if (M == 4) base = 0;
        if (M == 8) base = (int64_t)(r & 1) * S;
        if (M == 9) base = (int64_t)(r & 7) * S;
        if (M >= 5) {  // fresh: publish this workgroup's share, then a counter wait
            const int per = (nq + G - 1) / G;
            for (int i = t; i < per; i += 256) {
                const int q = b * per + i;
                if (q < nq) {
                    const u32x4 v = {(uint32_t)(r + q), (uint32_t)q, 0u, 1u};
                    if (M == 6) {
#pragma unroll
                        for (int c = 0; c < 8; ++c)
                            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)((int64_t)r * S + c * cstride + 16ll * q), 0, 16);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)(base + 16ll * q), 0, 16);
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) {
                __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t want = (uint32_t)G * (r + 1);
                for (uint32_t it = 0; it < (1u << 24); ++it)
                    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) break;
            }
            __syncthreads();
            if (M == 7) continue;
        }
        for (int i0 = t; i0 < nq; i0 += 256 * PU) {
            u32x4 v[PU];
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                const int i = i0 + 256 * u;
                v[u] = i < nq ? __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(base + 16ll * i), 0, 16)
                              : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                acc += v[u][0] ^ v[u][3];
                // fresh variants: a stale line would show as a wrong value
                if (M >= 5 && i0 + 256 * u < nq && v[u][0] != (uint32_t)(r + i0 + 256 * u)) atomicAdd(ctr + 32, 1u);
            }
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
    uint32_t *ctr;
    const int64_t S_MAX = 100 << 10, cstride = (int64_t)NR * S_MAX + 4096 * 3;
    const int64_t cap = 32 * cstride + (int64_t)NR * 256 * S_MAX;
    CK(hipMalloc(&buf, cap));
    CK(hipMemset(buf, 1, cap));
    CK(hipMalloc(&sink, 512 * 256 * 4));
    CK(hipMalloc(&ctr, 256));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[] = {"cold shared", "cold 8 copies", "cold 32 copies", "cold private", "warm shared",
                           "fresh shared", "fresh 8 copies", "barrier only", "fresh 2 regions", "fresh 8 regions"};
    auto run = [&](auto kern, int M, int PU, int64_t S, int G) {
        std::vector<float> tm;
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipMemset(ctr, 0, 256));
            // overwrite the regions so no launch starts with them cached
            CK(hipMemset(buf, rep, cap));
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(kern, dim3(G), dim3(256), 0, 0, buf, S, cstride, ctr, sink);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) tm.push_back(ms * 1000.f / NR);
        }
        std::sort(tm.begin(), tm.end());
        uint32_t bad = 0;
        CK(hipMemcpy(&bad, ctr + 32, 4, hipMemcpyDeviceToHost));
        printf("G=%3d %6.1f KB %-15s PU=%2d %7.3f us/round = %6.1f GB/s per CU  stale=%u\n", G, S / 1024.0, names[M], PU, tm[0],
               S / (tm[0] * 1e-6) / 1e9, bad);
        fflush(stdout);
    };
    for (int64_t kb : {8, 25, 50, 100}) {
        const int64_t S = kb * 1024;
        run(k_read2<0, 16>, 0, 16, S, 256);
        run(k_read2<1, 16>, 1, 16, S, 256);
        run(k_read2<2, 16>, 2, 16, S, 256);
        run(k_read2<3, 16>, 3, 16, S, 256);
        run(k_read2<4, 16>, 4, 16, S, 256);
        run(k_read2<5, 16>, 5, 16, S, 256);
        run(k_read2<6, 16>, 6, 16, S, 256);
        run(k_read2<7, 16>, 7, 16, S, 256);
        run(k_read2<5, 16>, 5, 16, S, 256);  // (again, next to F2 / F3)
        run(k_read2<8, 16>, 8, 16, S, 256);
        run(k_read2<9, 16>, 9, 16, S, 256);
    }
    return 0;
}

// seam_probe.hip — cost of one all-to-all hand-off ("seam") between the
// workgroups of one persistent launch vs a kernel boundary in a hipGraph.
// Standalone diagnostic (not part of the product library).
//
// Every round each of G workgroups publishes 2 floats (a 2*G vector) and then
// reads the whole vector.  Variants:
//   0 counter8 : sc1 payload stores, vmcnt(0), one agent atomic add per WG on
//                one of 8 shard counters (b % 8); wave 0 polls all 8 shards
//                with one sc1 load per lane; sc1 payload loads
//   1 granule  : payload as {epoch, value} 8-byte sc1 granules, no counter:
//                every thread re-reads its granules until the tags match
//   2 counter1 : one counter for all workgroups
//   3 counter8 with s_sleep(1) in the poll loop
//   9 boundary : one kernel per round, plain loads, in a captured hipGraph
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int NT = 256;
constexpr uint32_t SPIN_MAX = 1u << 20;

__device__ __forceinline__ uint32_t ld_u32(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint64_t ld_u64(const uint64_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_u32(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_u64(uint64_t *p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ __forceinline__ float val(int r, int i) { return (float)(i & 1023) + 0.25f * (float)(r & 63); }

template <int V>
__global__ __launch_bounds__(NT) void k_seam(uint32_t *pay, uint64_t *gran, uint32_t *ctr, uint32_t *err, int R) {
    const int G = gridDim.x, b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int NV = 2 * G;
    __shared__ int bad;
    if (t == 0) bad = 0;
    __syncthreads();
    for (int r = 0; r < R; ++r) {
        const uint32_t e = (uint32_t)r + 1;
        const int buf = (r & 1) * 4096;
        if (V == 1) {
            if (t < 2) {
                const int i = 2 * b + t;
                st_u64(gran + buf + i, ((uint64_t)e << 32) | __float_as_uint(val(r, i)));
            }
            // each thread: granules t, t + 256, ... until every tag == e
            float acc = 0.f;
            for (int i = t; i < NV; i += NT) {
                uint64_t x;
                uint32_t it = 0;
                for (;;) {
                    x = ld_u64(gran + buf + i);
                    if ((uint32_t)(x >> 32) == e) break;
                    if (++it > SPIN_MAX) { atomicOr(err, 1u); bad = 1; break; }
                }
                if (__uint_as_float((uint32_t)x) != val(r, i)) atomicAdd(err + 1, 1u);
                acc += __uint_as_float((uint32_t)x);
            }
            __syncthreads();
            if (bad) break;
            continue;
        }
        if (t < 2) {
            const int i = 2 * b + t;
            st_u32(pay + buf + i, __float_as_uint(val(r, i)));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (V == 2) {
            if (t == 0) {
                __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                uint32_t it = 0;
                while (ld_u32(ctr) < e * (uint32_t)G) {
                    if (++it > SPIN_MAX) { atomicOr(err, 1u); bad = 1; break; }
                }
            }
        } else {
            if (t == 0) __hip_atomic_fetch_add(ctr + (b & 7) * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (w == 0) {
                const int s = lane & 7;
                const uint32_t cnt = (uint32_t)(G / 8 + (s < (G & 7) ? 1 : 0));
                uint32_t it = 0;
                for (;;) {
                    const uint32_t v = ld_u32(ctr + s * 64);
                    if (__all(v >= e * cnt)) break;
                    if (V == 3) __builtin_amdgcn_s_sleep(1);
                    if (++it > SPIN_MAX) { if (lane == 0) { atomicOr(err, 1u); bad = 1; } break; }
                }
            }
        }
        __syncthreads();
        if (bad) break;
        for (int i = t; i < NV; i += NT) {
            const float x = __uint_as_float(ld_u32(pay + buf + i));
            if (x != val(r, i)) atomicAdd(err + 1, 1u);
        }
    }
}

__global__ __launch_bounds__(NT) void k_bound(uint32_t *pay, uint32_t *err, int r) {
    const int G = gridDim.x, b = blockIdx.x, t = threadIdx.x, NV = 2 * G;
    if (r > 0) {
        const int buf = ((r - 1) & 1) * 4096;
        for (int i = t; i < NV; i += NT)
            if (__uint_as_float(pay[buf + i]) != val(r - 1, i)) atomicAdd(err + 1, 1u);
    }
    if (t < 2) {
        const int i = 2 * b + t;
        pay[(r & 1) * 4096 + i] = __float_as_uint(val(r, i));
    }
}

int main(int argc, char **argv) {
    const int R = 200;
    uint32_t *pay, *ctr, *err;
    uint64_t *gran;
    CK(hipMalloc(&pay, 8192 * 4));
    CK(hipMalloc(&gran, 8192 * 8));
    CK(hipMalloc(&ctr, 4096 * 4));
    CK(hipMalloc(&err, 64));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[] = {"counter8", "granule", "counter1", "counter8+sleep"};
    for (int G : {64, 128, 256, 512}) {
        for (int V = 0; V < 4; ++V) {
            std::vector<float> t;
            uint32_t herr[2] = {0, 0};
            for (int rep = 0; rep < 6; ++rep) {
                CK(hipMemsetAsync(pay, 0, 8192 * 4, s));
                CK(hipMemsetAsync(gran, 0, 8192 * 8, s));
                CK(hipMemsetAsync(ctr, 0, 4096 * 4, s));
                CK(hipMemsetAsync(err, 0, 64, s));
                CK(hipEventRecord(e0, s));
                switch (V) {
                    case 0: hipLaunchKernelGGL(k_seam<0>, dim3(G), dim3(NT), 0, s, pay, gran, ctr, err, R); break;
                    case 1: hipLaunchKernelGGL(k_seam<1>, dim3(G), dim3(NT), 0, s, pay, gran, ctr, err, R); break;
                    case 2: hipLaunchKernelGGL(k_seam<2>, dim3(G), dim3(NT), 0, s, pay, gran, ctr, err, R); break;
                    case 3: hipLaunchKernelGGL(k_seam<3>, dim3(G), dim3(NT), 0, s, pay, gran, ctr, err, R); break;
                }
                CK(hipGetLastError());
                CK(hipEventRecord(e1, s));
                CK(hipStreamSynchronize(s));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                uint32_t he[2];
                CK(hipMemcpy(he, err, 8, hipMemcpyDeviceToHost));
                herr[0] |= he[0];
                herr[1] += he[1];
                if (rep) t.push_back(ms * 1000.f / R);
            }
            std::sort(t.begin(), t.end());
            printf("G=%4d %-15s %7.3f us/seam (median %7.3f)  timeout=%u mismatches=%u\n", G, names[V], t[0],
                   t[t.size() / 2], herr[0], herr[1]);
            fflush(stdout);
        }
        // kernel boundary: R dependent launches captured in one graph
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_bound, dim3(G), dim3(NT), 0, s, pay, err, r);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        std::vector<float> t;
        uint32_t mism = 0;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipMemsetAsync(err, 0, 64, s));
            CK(hipEventRecord(e0, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            uint32_t he[2];
            CK(hipMemcpy(he, err, 8, hipMemcpyDeviceToHost));
            mism += he[1];
            if (rep) t.push_back(ms * 1000.f / R);
        }
        std::sort(t.begin(), t.end());
        printf("G=%4d %-15s %7.3f us/seam (median %7.3f)  mismatches=%u\n", G, "graph-boundary", t[0], t[t.size() / 2], mism);
        fflush(stdout);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}

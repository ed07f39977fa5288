// poll_probe.hip — does a workgroup's own weight prefetch delay its seam poll?
// Standalone diagnostic (not part of the product library).
//
// A persistent launch of G workgroups runs R rounds.  Each round a workgroup
// issues its next weight slice (PK 16-byte loads per compute lane, from a
// 64 MiB buffer that stays in the Infinity Cache), then polls a 2G-granule
// all-to-all vector (every workgroup published 2 granules last round), then
// consumes weights + vector and publishes its 2 granules for the next round.
// Loads return in issue order per wave (vmcnt), so a poll issued behind the
// same wave's prefetch cannot complete before the prefetch has landed.
//   V0 same-wave : 4 waves, every lane prefetches then polls (the round-2 decoder)
//   V1 poller-5th: 5 waves; waves 0-3 prefetch, wave 4 (no loads in flight) polls
//   V2 poller-w0 : 4 waves; wave 0 polls only, waves 1-3 prefetch 4/3 as much
//   V3 none      : no prefetch (the bare seam)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr uint32_t SPIN_MAX = 1u << 21;

__device__ __forceinline__ uint64_t ld_u64(const uint64_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_u64(uint64_t *p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// poll cnt granules with nthr lanes starting at lane index `me`; values to LDS
template <int PU>
__device__ __forceinline__ bool poll(const uint64_t *g, int cnt, uint32_t tag, int me, int nthr, float *dst) {
    for (int base = me; base < cnt; base += nthr * PU) {
        uint64_t v[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const int i = base + nthr * u;
            v[u] = i < cnt ? ld_u64(g + i) : ((uint64_t)tag << 32);
        }
        for (uint32_t it = 0;; ++it) {
            bool all = true;
#pragma unroll
            for (int u = 0; u < PU; ++u)
                if ((uint32_t)(v[u] >> 32) != tag) {
                    all = false;
                    v[u] = ld_u64(g + base + nthr * u);
                }
            if (all) break;
            if (it > SPIN_MAX) return false;
        }
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const int i = base + nthr * u;
            if (i < cnt) dst[i] = __uint_as_float((uint32_t)v[u]);
        }
    }
    return true;
}

template <int V, int PK>
__global__ __launch_bounds__(320, 1) void k_poll(const uint4 *wbuf, int64_t nslot, uint64_t *gran, uint32_t *err,
                                                 float *sink, int R) {
    const int G = gridDim.x, b = blockIdx.x, t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int NV = 2 * G;
    __shared__ float vec[1024];
    __shared__ float part[8];
    __shared__ int bad;
    if (V != 1 && t >= 256) return;
    if (t == 0) bad = 0;
    __syncthreads();
    float acc = 0.f;
    for (int r = 0; r < R; ++r) {
        const uint32_t tag = (uint32_t)r + 1;
        const uint64_t *gin = gran + ((r + 1) & 1) * 1024;   // published in round r - 1 (tag r)
        uint64_t *gout = gran + (r & 1) * 1024;
        // ---- prefetch this round's weight slice ----
        constexpr int PKW = V == 2 ? (PK * 4 + 2) / 3 : PK;
        const bool loader = V == 3 ? false : V == 2 ? (w >= 1 && w < 4) : (w < 4);
        uint4 wv[PKW];
#pragma unroll
        for (int k = 0; k < PKW; ++k) wv[k] = make_uint4(0, 0, 0, 0);
        if (loader) {
            const int lt = V == 2 ? t - 64 : t;
            const int nl = V == 2 ? 192 : 256;
            const int64_t s0 = ((int64_t)(r % 16) * G + b) * (int64_t)(PKW * nl);
#pragma unroll
            for (int k = 0; k < PKW; ++k) wv[k] = wbuf[(s0 + k * nl + lt) % nslot];
        }
        asm volatile("" ::: "memory");
        // ---- poll the vector the previous round published ----
        if (r > 0) {
            bool ok = true;
            if (V == 0 || V == 3) ok = poll<4>(gin, NV, tag, t, 256, vec);
            else if (V == 1) { if (w == 4) ok = poll<8>(gin, NV, tag, lane, 64, vec); }
            else { if (w == 0) ok = poll<8>(gin, NV, tag, lane, 64, vec); }
            if (!ok) { atomicOr(err, 1u); bad = 1; }
        }
        __syncthreads();
        if (bad) break;
        // ---- consume: weights + the vector ----
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < PKW; ++k) s += __uint_as_float(wv[k].x & 0x3fffffffu) * 1e-30f;
        if (r > 0 && t < 256) {
            s += vec[t % NV];
            // check a few values: granule i of round r-1 carries i + r
            if (t < NV && vec[t] != (float)(t + r - 1)) atomicAdd(err + 1, 1u);
        }
        acc += s;
        __syncthreads();
        if (t < 2) st_u64(gout + 2 * b + t, ((uint64_t)(tag + 1) << 32) | __float_as_uint((float)(2 * b + t + r)));
    }
    if (t == 0) part[0] = acc;
    sink[b * 320 + t] = acc;
}

int main(int argc, char **argv) {
    const int R = 400;
    const int64_t bytes = 64ll << 20;
    uint4 *wbuf;
    uint64_t *gran;
    uint32_t *err;
    float *sink;
    CK(hipMalloc(&wbuf, bytes));
    CK(hipMemset(wbuf, 0x11, bytes));
    CK(hipMalloc(&gran, 2048 * 8));
    CK(hipMalloc(&err, 64));
    CK(hipMalloc(&sink, 512 * 320 * 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int64_t nslot = bytes / 16;
    const char *names[] = {"same-wave", "poller-5th", "poller-w0", "none"};
    auto run = [&](auto kern, int V, int PK, int G) {
        std::vector<float> t;
        uint32_t herr[2] = {0, 0};
        const int nt = V == 1 ? 320 : 256;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipMemsetAsync(gran, 0, 2048 * 8, s));
            CK(hipMemsetAsync(err, 0, 64, s));
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(kern, dim3(G), dim3(nt), 0, s, (const uint4 *)wbuf, nslot, gran, err, sink, R);
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
        printf("G=%3d PK=%2d (%5.1f KB/WG) %-11s %7.3f us/round (median %7.3f)  timeout=%u mismatches=%u\n", G, PK,
               PK * 256 * 16 / 1024.0, names[V], t[0], t[t.size() / 2], herr[0], herr[1]);
        fflush(stdout);
    };
#define RUN4(PK, G)                      \
    run(k_poll<0, PK>, 0, PK, G);        \
    run(k_poll<1, PK>, 1, PK, G);        \
    run(k_poll<2, PK>, 2, PK, G);
    for (int G : {256, 128}) {
        run(k_poll<3, 1>, 3, 0, G);
        RUN4(1, G)
        RUN4(2, G)
        RUN4(4, G)
        RUN4(8, G)
        RUN4(16, G)
    }
    return 0;
}

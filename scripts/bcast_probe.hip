// bcast_probe.hip — the price of one all-to-all edge of the persistent decoder
// as a function of its size and transport.  Standalone diagnostic (not part of
// the product library).
//
// A persistent launch of G workgroups (256 threads, one per CU) runs R rounds.
// Each round every workgroup publishes its V / G words of a V-word vector and
// then gathers the whole vector (as every decoder phase with a full-vector
// input does: the residual stream x of B rows = B n words, the MLP hidden
// B 4n f16 = B 2n words).  Transports:
//   T0 granule8 : 8-byte {tag, word} granules, sc1 stores / sc1 load polls (the decoder's)
//   T1 granule16: 16-byte {tag, w0, w1, w2} granules (one 16-B sc1 store each)
//   T2 flag     : 16-byte sc1 payload stores, every storing wave's vmcnt(0), a
//                 workgroup barrier, one sc1 flag store per producer; the
//                 consumer's wave 0 polls the G flags (16-B sc1 loads), a
//                 barrier, then every thread loads the payload (16-B sc1 loads)
//   T3 relay     : T0's granules, gathered once per XCD: NRL relay workgroups
//                 per XCD (elected at start by an atomic count per XCC_ID, read
//                 with s_getreg) each poll 1 / NRL of the vector from the
//                 global granules and re-store those granules with PLAIN stores
//                 into their XCD's copy (kept in that XCD's L2); every
//                 workgroup polls its own XCD's copy with sc1 loads
//   T4 flag+acq  : as T2, but the consumer's polling wave runs an agent-scope
//                 acquire after its flag poll and every thread reads the payload
//                 with PLAIN 16-B loads (L2-served for the XCD's other CUs)
//   T5 rel+acq   : as T4 with plain producer stores + an agent release fence
//   T6 counter8  : T2's dense 16-byte sc1 payload, but one agent atomic add per
//                 producer onto ONE of 8 counters (b % 8, each on its own
//                 line); the consumer's lanes 0-7 poll the 8 counters (sc1),
//                 a barrier, then every thread reads the payload (16-B sc1)
//   T7 granule8+sleep: T0 with s_sleep 1 before every re-poll of a granule set
// Every value is checked (word i of round r carries i * 3 + r).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr uint32_t SPIN_MAX = 1u << 20;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t ld8(const uint64_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st8(uint64_t *p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t ld4(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st4(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// 16-byte sc1 (write-through / L1-bypassing) accesses through a buffer resource
__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}

// poll cnt granules g[i] (i = t, t + 256, ...) until every tag matches; values to dst
template <int LDF>
__device__ __forceinline__ uint64_t ldf(const uint64_t *p) {
    if constexpr (LDF == 1) return __builtin_nontemporal_load(p);
    else if constexpr (LDF >= 2) return *(const volatile uint64_t *)p;
    else return ld8(p);
}
template <int PU, int LDF = 0>
__device__ __forceinline__ bool gpoll(const uint64_t *g, int cnt, uint32_t tag, uint32_t *dst, uint32_t *abortw) {
    const int t = threadIdx.x;
    for (int base = t; base < cnt; base += 256 * PU) {
        uint64_t v[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const int i = base + 256 * u;
            v[u] = i < cnt ? ldf<LDF>(g + i) : ((uint64_t)tag << 32);
        }
        for (uint32_t it = 0;; ++it) {
            bool all = true;
#pragma unroll
            for (int u = 0; u < PU; ++u)
                if ((uint32_t)(v[u] >> 32) != tag) {
                    all = false;
                    v[u] = ldf<LDF>(g + base + 256 * u);
                }
            if (all) break;
            if constexpr (LDF == 2) asm volatile("buffer_inv sc0" ::: "memory");
            if ((it & 63) == 63 && ld4(abortw)) return false;
            if (it > SPIN_MAX) { st4(abortw, 1u); return false; }
        }
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const int i = base + 256 * u;
            if (i < cnt) dst[i] = (uint32_t)v[u];
        }
    }
    return true;
}

template <int T, int PU, int NRL = 4, int LDF = 0>
__global__ __launch_bounds__(256, 1) void k_bcast(unsigned char *buf, uint32_t *flags, int V, uint32_t *err, int R,
                                                  float *sink) {
    const int G = gridDim.x, b = blockIdx.x, t = threadIdx.x, w = t >> 6, lane = t & 63;
    extern __shared__ uint32_t vec[];  // [V]
    __shared__ int bad, xcc_s, slot_s;
    if (t == 0) {
        bad = 0;
        if constexpr (T == 3) {
            uint32_t x;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
            xcc_s = (int)(x & 7);
            slot_s = (int)atomicAdd(flags + 1024 + (x & 7), 1u);  // this workgroup's index within its XCD
        }
    }
    __syncthreads();
    uint32_t *abortw = flags + 2048;
    const int per = (V + G - 1) / G;  // words per producer
    const int64_t half = 4ll << 20;   // two buffers of up to 4 MB
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, (int)(2 * half), 0x00020000);
    const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(flags, (short)0, 4096, 0x00020000);
    float acc = 0.f;
    for (int r = 1; r <= R; ++r) {
        const uint32_t tag = (uint32_t)r;
        const int64_t ob = (r & 1) * half;  // this round's buffer
        // ---- publish words [b per, b per + per) of round r ----
        if constexpr (T == 0 || T == 3) {
            uint64_t *g = (uint64_t *)(buf + ob);
            for (int i = t; i < per; i += 256) {
                const int e = b * per + i;
                if (e < V) st8(g + e, ((uint64_t)tag << 32) | (uint32_t)(e * 3 + r));
            }
        } else if constexpr (T == 7) {
            uint64_t *g = (uint64_t *)(buf + ob);
            for (int i = t; i < per; i += 256) {
                const int e = b * per + i;
                if (e < V) st8(g + e, ((uint64_t)tag << 32) | (uint32_t)(e * 3 + r));
            }
        } else if constexpr (T == 1) {
            for (int i = t; i < (per + 2) / 3; i += 256) {
                u32x4 v;
                v[0] = tag;
                for (int k = 0; k < 3; ++k) {
                    const int e = b * per + 3 * i + k;
                    v[k + 1] = (3 * i + k < per && e < V) ? (uint32_t)(e * 3 + r) : 0u;
                }
                const int gi = b * ((per + 2) / 3) + i;  // granule index
                st16(rs, (uint32_t)(ob + 16ll * gi), v);
            }
        } else {
            // payload: per words padded to 4, 16-B stores
            const int per4 = (per + 3) & ~3;
            for (int i = t; i < per4 / 4; i += 256) {
                u32x4 v;
                for (int k = 0; k < 4; ++k) {
                    const int e = b * per + 4 * i + k;
                    v[k] = (4 * i + k < per && e < V) ? (uint32_t)(e * 3 + r) : 0u;
                }
                if constexpr (T == 5) *(u32x4 *)(buf + ob + 4ll * (b * per4 + 4 * i)) = v;
                else st16(rs, (uint32_t)(ob + 4ll * (b * per4 + 4 * i)), v);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) {
                if constexpr (T == 5) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if constexpr (T == 6) __hip_atomic_fetch_add(flags + 3072 + 32 * (b & 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else st4(flags + b, tag);
            }
        }
        // ---- gather the whole vector of round r ----
        if constexpr (T == 3) {
            const uint64_t *g = (const uint64_t *)(buf + ob);
            uint64_t *xl = (uint64_t *)(buf + 2 * half + (int64_t)(r & 1) * (8ll << 20)) + (int64_t)xcc_s * V;  // this XCD's copy
            if (slot_s < NRL) {  // relay part slot_s of the vector into the XCD's copy (plain stores)
                const int p0 = (int)((int64_t)V * slot_s / NRL), p1 = (int)((int64_t)V * (slot_s + 1) / NRL);
                if (!gpoll<PU>(g + p0, p1 - p0, tag, vec + p0, abortw)) bad = 1;
                __syncthreads();
                for (int i = p0 + t; i < p1; i += 256) xl[i] = ((uint64_t)tag << 32) | vec[i];
            }
            if constexpr (LDF == 2) asm volatile("buffer_inv sc0" ::: "memory");
            if (!gpoll<PU, LDF>(xl, V, tag, vec, abortw)) bad = 1;
            if (bad) atomicOr(err, 1u);
        } else if constexpr (T == 0 || T == 7) {
            const uint64_t *g = (const uint64_t *)(buf + ob);
            for (int base = t; base < V; base += 256 * PU) {
                uint64_t v[PU];
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const int i = base + 256 * u;
                    v[u] = i < V ? ld8(g + i) : ((uint64_t)tag << 32);
                }
                for (uint32_t it = 0;; ++it) {
                    bool all = true;
#pragma unroll
                    for (int u = 0; u < PU; ++u)
                        if ((uint32_t)(v[u] >> 32) != tag) {
                            all = false;
                            v[u] = ld8(g + base + 256 * u);
                        }
                    if (all) break;
                    if (it > SPIN_MAX) { bad = 1; atomicOr(err, 1u); break; }
                    if constexpr (T == 7) __builtin_amdgcn_s_sleep(1);
                }
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const int i = base + 256 * u;
                    if (i < V) vec[i] = (uint32_t)v[u];
                }
            }
        } else if constexpr (T == 1) {
            const int pg = (per + 2) / 3, NG = G * pg;
            for (int base = t; base < NG; base += 256 * PU) {
                u32x4 v[PU];
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const int i = base + 256 * u;
                    v[u] = i < NG ? ld16(rs, (uint32_t)(ob + 16ll * i)) : u32x4{tag, 0u, 0u, 0u};
                }
                for (uint32_t it = 0;; ++it) {
                    bool all = true;
#pragma unroll
                    for (int u = 0; u < PU; ++u)
                        if (v[u][0] != tag) {
                            all = false;
                            v[u] = ld16(rs, (uint32_t)(ob + 16ll * (base + 256 * u)));
                        }
                    if (all) break;
                    if (it > SPIN_MAX) { bad = 1; atomicOr(err, 1u); break; }
                }
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const int i = base + 256 * u;
                    if (i < NG) {
                        const int p = i / pg, j = i - p * pg;
                        for (int k = 0; k < 3; ++k) {
                            const int e = p * per + 3 * j + k;
                            if (3 * j + k < per && e < V) vec[e] = v[u][k + 1];
                        }
                    }
                }
            }
        } else {
            if (T == 6 && w == 0) {  // lanes 0-7 poll the 8 counters: G / 8 arrivals per round each
                for (uint32_t it = 0;; ++it) {
                    const bool ok = lane >= 8 || ld4(flags + 3072 + 32 * lane) >= (uint32_t)(G / 8) * (uint32_t)r;
                    if (__all(ok)) break;
                    if (it > SPIN_MAX) { bad = 1; atomicOr(err, 1u); break; }
                }
            } else if (w == 0) {  // poll the G flags, 4 per lane
                for (uint32_t it = 0;; ++it) {
                    bool all = true;
                    for (int f = 4 * lane; f < G; f += 256) {  // G % 4 == 0
                        const u32x4 v = ld16(rf, (uint32_t)(4 * f));
                        all = all && v[0] == tag && v[1] == tag && v[2] == tag && v[3] == tag;
                    }
                    if (__all(all)) break;
                    if (it > SPIN_MAX) { bad = 1; atomicOr(err, 1u); break; }
                }
                if constexpr (T == 4 || T == 5) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            __syncthreads();
            const int per4 = (per + 3) & ~3, NQ = G * per4 / 4;
            for (int base = t; base < NQ; base += 256 * PU) {
                u32x4 v[PU];
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const int i = base + 256 * u;
                    if constexpr (T == 4 || T == 5) v[u] = i < NQ ? *(const u32x4 *)(buf + ob + 16ll * i) : u32x4{0u, 0u, 0u, 0u};
                    else v[u] = i < NQ ? ld16(rs, (uint32_t)(ob + 16ll * i)) : u32x4{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const int i = base + 256 * u;
                    if (i < NQ) {
                        const int p = (4 * i) / per4, j = 4 * i - p * per4;
                        for (int k = 0; k < 4; ++k) {
                            const int e = p * per + j + k;
                            if (j + k < per && e < V) vec[e] = v[u][k];
                        }
                    }
                }
            }
        }
        __syncthreads();
        if (bad) break;
        // check every word, then a token of work on it
        float s = 0.f;
        for (int i = t; i < V; i += 256) {
            if (vec[i] != (uint32_t)(i * 3 + r)) atomicAdd(err + 1, 1u);
            s += (float)(vec[i] & 7);
        }
        acc += s;
        __syncthreads();
    }
    sink[b * 256 + t] = acc;
}

int main(int argc, char **argv) {
    const int R = 200;
    unsigned char *buf;
    uint32_t *flags, *err;
    float *sink;
    CK(hipMalloc(&buf, 24 << 20));
    CK(hipMalloc(&flags, 16384));
    CK(hipMalloc(&err, 64));
    CK(hipMalloc(&sink, 512 * 256 * 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[] = {"granule8", "granule16", "flag+payload", "relay", "flag+acq", "rel+acq", "counter8", "granule8+sleep"};
    auto run = [&](auto kern, int T, int PU, int V, int G, int NRLp = 0) {
        std::vector<float> tm;
        uint32_t herr[2] = {0, 0};
        const size_t lds = (size_t)V * 4;
        CK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipMemsetAsync(buf, 0, 24 << 20, s));
            CK(hipMemsetAsync(flags, 0, 16384, s));
            CK(hipMemsetAsync(err, 0, 64, s));
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(kern, dim3(G), dim3(256), lds, s, buf, flags, V, err, R, sink);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            uint32_t he[2];
            CK(hipMemcpy(he, err, 8, hipMemcpyDeviceToHost));
            herr[0] |= he[0];
            herr[1] += he[1];
            if (rep) tm.push_back(ms * 1000.f / R);
        }
        std::sort(tm.begin(), tm.end());
        printf("G=%3d V=%6d words (%6.1f KB payload) %-13s PU=%2d NRL=%d %7.3f us/round (median %7.3f)  timeout=%u mismatches=%u\n",
               G, V, V * 4 / 1024.0, names[T], PU, NRLp, tm[0], tm[tm.size() / 2], herr[0], herr[1]);
        fflush(stdout);
    };
    for (int V : {2048, 6400, 12800, 25600}) {
        run(k_bcast<0, 16>, 0, 16, V, 256);
        run(k_bcast<7, 16>, 7, 16, V, 256);
        run(k_bcast<2, 16>, 2, 16, V, 256);
        run(k_bcast<6, 16>, 6, 16, V, 256);
        run(k_bcast<6, 4>, 6, 4, V, 256);
    }
    return 0;
}

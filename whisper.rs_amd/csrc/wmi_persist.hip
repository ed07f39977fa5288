// wmi_persist.hip — the whole greedy decoder step as ONE
// persistent launch that runs n_steps steps back to back.
//
// Why: a base decoder step is ~40 dependent operations on ~110 MB that sits in
// the 256 MiB Infinity Cache; as a chain of kernels every seam costs a kernel
// boundary plus the next kernel's cold start (236 us per step in round 1 for a
// 14 us byte roofline).  Here all workgroups stay resident (one per CU) and a
// seam is an all-to-all hand-off of epoch-tagged 8-byte granules {tag, value}:
// the producer stores them write-through (agent-scope relaxed store = `sc1`),
// the consumer re-reads them with `sc1` loads until every tag matches
// (MI355X_MICROARCH.md, Valid forms, R2 granules; cdna_hip_programming.md
// Guideline 16).  Each phase issues its weight loads BEFORE it polls for its
// input, so the weight stream of a phase overlaps the seam in front of it.
//
// Phases of one decoder layer l (rows b < B <= 8; tag = epoch of the phase):
//   A  LN1(x) -> Wqkv rows (all WGs)            -> q, k, v granules + KV cache
//   B  self-attention per (b, head)              -> o (f16 pairs)
//   C  Wo rows + residual                        -> x'
//   D  LNc(x') -> Wcq rows                       -> cross q (f16 pairs)
//      (n <= 768: no D phase — every E task computes its head's q itself)
//   E  cross scores per (b, head, key chunk)     -> scores, chunk max
//   F  exact softmax (global max, double sum) + P16.V per chunk -> partials
//   G1 chunk partials summed in order per (b, head) -> cross o (f16 pairs)
//   G2 Wco rows + residual                       -> x''
//   H  LN2(x'') -> W0 rows -> GELU               -> hidden (f16 pairs)
//   I  W1 rows + residual                        -> x''' (next layer's x)
// then LN_final -> vocabulary rows -> per-WG argmax -> every WG reduces the
// G candidates -> next token -> embedding (te[tok] + pe[pos]).
//
// Numerics are the decoder chain's (wmi_kernels.hip k_dec_*): the same f16
// rounding points, double LayerNorm statistics, ggml exp/GELU tables, exact
// softmax, P.V partials over 128-key chunks summed in chunk order (a task may
// cover several chunks when many rows share the launch; it still publishes
// one partial per 128 keys, so a row's result never depends on the batch).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "wmi_device.h"
#include "wmi_internal.h"

#pragma clang fp contract(off)

namespace wmi {
// the q5_1 instances (PersistArgs::q5) are compiled by wmi_persist_q5.hip,
// which includes this file with WMI_PERSIST_Q5_TU: a second translation unit
// the build runs in parallel
hipError_t launch_persist_q5(hipStream_t s, const PersistArgs &a, int G);
int grid_persist_q5(int device, int n, int B, int V, int *nres);

namespace {

constexpr int PT = 256;                 // threads per workgroup
constexpr uint32_t PSPIN = 1u << 19;    // polls before a seam is declared dead
constexpr int NPH = 11;                 // phases per decoder layer
constexpr int PMAXB = 8;                // decoder rows
constexpr int RNMAX = 16;               // rows of an n-row GEMV per workgroup
// attention / argmax scratch in LDS.  One-row instances use at most ~4.3 KB
// (G1's sub-chunk partials [16][64] + stats; a cross task's q and p values
// 2 KB, the self-attention's q / k / v and P16 1.5 KB, the argmax candidates
// [G][2] 2 KB); the multi-row ones also keep the beam-shared task's [B][4][64]
// P.V partials (from XS_OFF + XS_BYTES) and the MFMA GEMV partials, so the
// one-row instances keep 16 KB more vocabulary rows resident
__host__ __device__ constexpr int scr_bytes(int BT) { return BT == 1 ? 8 * 1024 : 24 * 1024; }
constexpr int NKP = 4;                  // 128-key passes per cross-attention chunk (cl <= 512)
constexpr int EXPFB = 64;               // exp fallback list entries (exp_f16_fast)
constexpr int XS_OFF = 1024;            // cross-attention task scores / p in the LDS scratch
constexpr int XS_BYTES = 8192;          // (a task's p values: rows x keys x 4 B)
constexpr int NSUBM = 16;               // 128-key sub-chunks of a row (T <= 2048)
static_assert(NSUBM * 64 * 4 + NSUBM * 3 * 4 <= scr_bytes(1) && PX_GMAX * 2 * 4 <= scr_bytes(1) &&
                  XS_OFF + 2 * 128 * 4 <= scr_bytes(1) && 512 + 512 * 2 <= scr_bytes(1),
              "one-row scratch: G1 partials, argmax candidates, a cross task's p, P16");

__device__ __forceinline__ uint64_t gld(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gput(uint64_t *p, uint32_t tag, uint32_t v) {
    __hip_atomic_store(p, ((uint64_t)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld32(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st32(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return (uint32_t)f2h_bits(a) | ((uint32_t)f2h_bits(b) << 16);
}
// tags: unique per (position, layer, phase) within a decode run; 0 = never written
__device__ __forceinline__ uint32_t ptag(int pos, int L, int l, int ph) {
    return (uint32_t)(pos * (L * NPH + 2) + l * NPH + ph + 1);
}
__device__ __forceinline__ uint32_t atag(int pos, int L) { return (uint32_t)(pos * (L * NPH + 2) + L * NPH + 1); }

// 16-byte write-through-coherent load (buffer_load_dwordx4 ... sc1): KV-cache
// rows written earlier in this launch by other workgroups
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ half8 bload_sc1(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
    const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
    return __builtin_bit_cast(half8, v);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

// Address-space casts.  Pointers read from memory (the layer table) are
// generic: their loads would be flat loads, which count against lgkmcnt too,
// so every LDS wait or barrier would also wait for the weight prefetch.  The
// layer table is read through the constant address space (scalar loads; the
// host writes it before the launch) and weight pointers are marked global.
// (the host pass only type-checks kernel bodies: no address spaces there)
#if defined(__HIP_DEVICE_COMPILE__)
#define WMI_AS(n) __attribute__((address_space(n)))
#else
#define WMI_AS(n)
#endif
template <typename T>
__device__ __forceinline__ const WMI_AS(1) T *glb(const T *p) {
    return (const WMI_AS(1) T *)p;
}
typedef const WMI_AS(4) PersistLayer ConstLayer;
// once-per-step streams (weight chunks, cross K/V), default cache policy
template <typename T>
__device__ __forceinline__ T sld(const T *p) {
    return *glb(p);
}

struct PShared {
    float xres[PMAXB][RNMAX];   // this workgroup's rows of the residual stream
    int32_t tok[PMAXB];
    float redf[4];
    double redd[4], redd2[4];
    float redfb[PMAXB][4];   // cross tasks: per (row or sub-chunk, wave) score maxima
    double reddb[PMAXB][4];  // and exp sums
    unsigned long long best[4][PMAXB];
    float ored[4][64 * 4];  // per wave: up to NKP 64-float partials
    __attribute__((aligned(16))) uint32_t expfb[EXPFB];  // exp fallback list (exp_f16_fast)
    float kpart[16 * PMAXB];  // split-K GEMV: per (row, k-slice) partials of every decoder row
    int abort_;
};

struct NoPre {
    __device__ void operator()() const {}
};
// Poll cnt granules (granule i at addr(i)) until every tag equals `tag`,
// storing the values to dst[i] (LDS).  Bounded: a dead seam sets the abort
// word (every poller checks it) and err bit 3, so the grid always drains.
// pre() runs once in every thread while its first round of loads is in
// flight (the q5_1 phases dequantise their prefetched weights there, so the
// VALU work overlaps the seam instead of following it).
// T0 / NTH: the threads that poll (threads T0 .. T0 + NTH - 1; NTH a
// multiple of 64: whole waves) — e.g. a wave with few loads of its own queued
// in front of the poll's, since vmcnt retires in order and a poll round
// cannot see its granules before every older load of its wave has landed
template <int PU = 4, int T0 = 0, int NTH = PT, typename F, typename Pre = NoPre>  // PU: granules in flight per thread
__device__ __forceinline__ bool gpoll(int cnt, uint32_t tag, F addr, uint32_t *dst, uint32_t *abortw, uint32_t *err,
                                      Pre pre = Pre{}) {
    bool ok = true, pre_done = false;
    int tid = (int)threadIdx.x - T0;
    asm volatile("" : "+v"(tid));
    const bool mine = tid >= 0 && tid < NTH;
    for (int base = tid; mine && base < cnt && ok; base += NTH * PU) {
        uint64_t v[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const int i = base + NTH * u;
            v[u] = i < cnt ? gld(addr(i)) : ((uint64_t)tag << 32);
        }
        if (!pre_done) {
            pre();
            pre_done = true;
        }
        for (uint32_t it = 0;; ++it) {
            bool all = true;
#pragma unroll
            for (int u = 0; u < PU; ++u)
                if ((uint32_t)(v[u] >> 32) != tag) {
                    all = false;
                    v[u] = gld(addr(base + NTH * u));
                }
            if (all) break;
            if ((it & 15) == 15) {
                if (ld32(abortw)) { ok = false; break; }
                if (it > PSPIN) {
                    st32(abortw, 1u);
                    atomicOr(err, 8u);
                    ok = false;
                    break;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const int i = base + NTH * u;
            if (i < cnt) dst[i] = (uint32_t)v[u];
        }
    }
    if (!pre_done) pre();
    return ok;
}

// ---- a weight matrix [N][K] as the GEMVs read it: f16, or (Q5) the q5_1
// repack of wmi_api.cpp repack_q5 — nibbles of the N*K weights in natural
// order (two per byte), then per 32-weight block a u32 of 5th bits and a u32
// {f16 d, f16 m}.  A lane's chunk is 8 consecutive weights: 16 bytes of f16,
// or 4 nibble bytes + its block's 8-byte word, dequantised at use by
// q5_half8 to exactly the loader's f16 copy (so both read the same weights).
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
struct WMat {
    const uint16_t *w;
    const uint8_t *q;     // nibbles [N * K / 2], or null
    const u32x2v *qd;     // blocks [N * K / 32]
};
__device__ __forceinline__ WMat wmat(const uint16_t *w) { return WMat{w, nullptr, nullptr}; }
__device__ __forceinline__ WMat wmat(const uint16_t *w, const uint8_t *q, int64_t nk) {
    return WMat{w, q, (const u32x2v *)(q + nk / 2)};
}
// a layer matrix: its q5_1 repack in the Q5 instances, else the f16 weights
template <bool Q5>
__device__ __forceinline__ WMat lmat(const uint16_t *w, const uint8_t *q, int64_t nk) {
    if constexpr (Q5) return wmat(w, q, nk);
    else return wmat(w);
}
template <bool Q5>
struct WChunk {
    half8 h;
};
template <>
struct WChunk<true> {
    uint32_t n;
    u32x2v hd;
    half8 h;  // the dequantised weights (wc_pre), read by wc_h8
};
template <bool Q5>
__device__ __forceinline__ void wc_zero(WChunk<Q5> &c) {
    if constexpr (Q5) {
        c.n = 0u;
        c.hd = u32x2v{0u, 0u};  // d = m = 0: dequantises to +0
        c.h = half8{};
    } else {
        c.h = half8{};
    }
}
// weights e .. e + 7 of the matrix (e = row * K + k, k % 8 == 0)
template <bool Q5>
__device__ __forceinline__ void wc_load(WChunk<Q5> &c, const WMat &m, int64_t e) {
    if constexpr (Q5) {
        c.n = sld((const uint32_t *)(m.q + e / 2));
        c.hd = sld(m.qd + e / 32);
    } else {
        c.h = sld((const half8 *)((const f16 *)m.w + e));
    }
}
// sh = e % 32 (a lane's offset inside its block: (l16 & 3) * 8).  q5_1
// chunks are dequantised once by wc_pre (called inside the phase's poll,
// gpoll / poll_ln1 `pre`), to exactly the loader's f16 copy
// (the one-row GEMVs dequantising at use instead, as the MFMA GEMVs do:
// C3 decode 36.2-36.7 -> 38.9 ms, profiles/r06/q5_lazy_one_row_ab_REJECTED.txt)
template <bool Q5>
__device__ __forceinline__ void wc_pre(WChunk<Q5> &c, int sh) {
    if constexpr (Q5) {
        c.h = q5_half8(c.n, c.hd[0], c.hd[1], sh);
        asm volatile("" : "+v"(c.h));  // computed here, not sunk to the first use
    }
}
template <bool Q5>
__device__ __forceinline__ half8 wc_h8(const WChunk<Q5> &c, int) {
    return c.h;
}

// ---- GEMV over this workgroup's rows: quarter-wave (16 lanes) per row, row
// slot = wave * 4 + quarter; pass p covers rows rb + 16 p + slot.  Lane l16
// holds K chunks c * 128 + l16 * 8 (8 weights each), the decoder chain's layout.
template <int KCH, int NP, bool Q5 = false>
struct WSet {
    WChunk<Q5> w[NP][KCH];
    float bias[NP];
};

template <int KCH, int NP, bool Q5>
__device__ __forceinline__ void wset_pre(WSet<KCH, NP, Q5> &S, int l16) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int c = 0; c < KCH; ++c) wc_pre(S.w[p][c], (l16 & 3) * 8);
}

template <int KCH, int NP, bool Q5>
__device__ __forceinline__ void wset_load(WSet<KCH, NP, Q5> &S, const WMat &m, const float *bias, int K, int rb, int r1,
                                          int slot, int l16) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        int row = rb + 16 * p + slot;
        const bool ok = row < r1;  // slots past the rows load nothing (zeros)
        row = ok ? row : 0;
        const int64_t e0 = (int64_t)row * K + l16 * 8;
#pragma unroll
        for (int c = 0; c < KCH; ++c) wc_zero(S.w[p][c]);
        S.bias[p] = 0.0f;
        if (ok) {  // exec-masked loads straight into the zeroed registers
#pragma unroll
            for (int c = 0; c < KCH; ++c) wc_load(S.w[p][c], m, e0 + c * 128);
            if (bias) S.bias[p] = *glb(bias + row);
        }
    }
}

// One row's K chunks c0 .. c0 + N - 1 of xs (lane l16's 8 elements each) in
// registers, every LDS read issued before the first is waited for: one LDS
// latency for the N reads instead of one per dot step (the scheduler
// otherwise interleaves one or two reads with the dots; the values and the
// dot order are unchanged)
// (from 6 K chunks, n >= 768: small 37.3 -> 36.0 ms decode; at n = 512 the
// E tasks' cross-q GEMV measured 0.1 ms slower with it, profiles/r05/preload_*)
constexpr int PRE_GEMV_MIN = 6;  // K chunks from which a one-row GEMV preloads them
template <int N>
__device__ __forceinline__ void xs_chunks(half8 (&xa)[N], const f16 *xs, int c0, int l16) {
#pragma unroll
    for (int c = 0; c < N; ++c) xa[c] = *(const half8 *)(xs + (c0 + c) * 128 + l16 * 8);
#pragma unroll
    for (int c = 0; c < N; ++c) asm volatile("" : "+v"(xa[c]));
}

// epi(row, b, v, bias, valid) is called by EVERY lane (pairing shuffles);
// lane l16 carries the reduced value of row `row` for decoder row b = l16
template <int BT, int KCH, int NP, bool Q5, typename Epi>
__device__ __forceinline__ void wset_dot(const WSet<KCH, NP, Q5> &S, const f16 *xs, int K, int B, int rb, int r1,
                                         int slot, int l16, Epi &&epi) {
    const int sh = (l16 & 3) * 8;
    if constexpr (NP > 1 && BT * KCH <= 32) {
        // the passes' dot chains and reductions interleaved, each xs chunk
        // read once for all passes (every pass computed — the loads behind
        // them are clamped rows — and only valid passes reach the epilogue);
        // each sum keeps its order.  (BT * KCH <= 32: the compiler hoists
        // the xs reads of all chunks; more would spill)
        float acc[NP][BT];
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int b = 0; b < BT; ++b) acc[p][b] = 0.0f;
        if constexpr (BT == 1 && KCH <= 8 && KCH >= PRE_GEMV_MIN) {
            half8 xa[KCH];
            xs_chunks(xa, xs, 0, l16);
#pragma unroll
            for (int c = 0; c < KCH; ++c)
#pragma unroll
                for (int p = 0; p < NP; ++p) acc[p][0] = dot8(wc_h8(S.w[p][c], sh), xa[c], acc[p][0]);
        } else
#pragma unroll
        for (int c = 0; c < KCH; ++c) {
            half8 xv[BT];
#pragma unroll
            for (int b = 0; b < BT; ++b)
                if (b < B) xv[b] = *(const half8 *)(xs + b * K + c * 128 + l16 * 8);
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const half8 wv = wc_h8(S.w[p][c], sh);
#pragma unroll
                for (int b = 0; b < BT; ++b)
                    if (b < B) acc[p][b] = dot8(wv, xv[b], acc[p][b]);
            }
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            float v = 0.0f;
#pragma unroll
            for (int b = 0; b < BT; ++b)
                if (b < B) {
                    const float t = red16_sum(acc[p][b]);
                    if (l16 == b) v = t;
                }
            acc[p][0] = v;
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if (rb + 16 * p >= r1) break;  // workgroup-uniform
            const int row = rb + 16 * p + slot;
            epi(row, l16, acc[p][0], S.bias[p], row < r1 && l16 < B);
        }
        return;
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        if (rb + 16 * p >= r1) break;  // workgroup-uniform
        const int row = rb + 16 * p + slot;
        float acc[BT];
#pragma unroll
        for (int b = 0; b < BT; ++b) acc[b] = 0.0f;
#pragma unroll
        for (int c = 0; c < KCH; ++c) {
            const half8 wv = wc_h8(S.w[p][c], sh);
#pragma unroll
            for (int b = 0; b < BT; ++b)
                if (b < B) acc[b] = dot8(wv, *(const half8 *)(xs + b * K + c * 128 + l16 * 8), acc[b]);
        }
        float v = 0.0f;
#pragma unroll
        for (int b = 0; b < BT; ++b)
            if (b < B) {
                float t = acc[b];
                t = red16_sum(t);
                if (l16 == b) v = t;
            }
        epi(row, l16, v, S.bias[p], row < r1 && l16 < B);
    }
}

// ---- split-K GEMV for phases whose workgroup owns few rows: KS quarter-
// waves per row, quarter ks summing chunks [ks * CQ, ks * CQ + CQ) of the
// row (lane l16 holds c * 128 + l16 * 8 of each, as wset_*), the KS partials
// added in ks order through LDS.  KS depends on n only (rows per workgroup
// at the full grid), so a row's sum never depends on the row count B.
template <int KCH, int KS, bool Q5 = false>
struct WSplit {
    static constexpr int CQ = (KCH + KS - 1) / KS;
    WChunk<Q5> w[CQ];
};
// the grid the row partitions (and so the split-K factors of the GEMV
// phases) are compiled for: min(CUs, PX_GDESIGN) workgroups.  A build with
// -DWMI_GDESIGN=G (G <= PX_GMAX) runs a smaller grid (the grid-size sweep,
// scripts/build_variant.sh)
#ifndef WMI_GDESIGN
#define WMI_GDESIGN PX_GMAX
#endif
constexpr int PX_GDESIGN = WMI_GDESIGN;
static_assert(PX_GDESIGN >= 32 && PX_GDESIGN <= PX_GMAX, "design grid");
// rows per workgroup of an N-row GEMV at the design grid, even
__host__ __device__ constexpr int rows_full(int N) { return (((N + PX_GDESIGN - 1) / PX_GDESIGN) + 1) & ~1; }
// the largest divisor of kch with rows * ks <= 16 (one pass of 16 quarters)
__host__ __device__ constexpr int split_of(int kch, int rows) {
    int best = 1;
    for (int k = 1; k <= kch; ++k)
        if (kch % k == 0 && rows * k <= 16) best = k;
    return best;
}

template <int KCH, int KS, bool Q5>
__device__ __forceinline__ void wsplit_pre(WSplit<KCH, KS, Q5> &S, int l16) {
#pragma unroll
    for (int c = 0; c < WSplit<KCH, KS, Q5>::CQ; ++c) wc_pre(S.w[c], (l16 & 3) * 8);
}

template <int KCH, int KS, bool Q5>
__device__ __forceinline__ void wsplit_load(WSplit<KCH, KS, Q5> &S, const WMat &m, int K, int rb, int r1, int slot,
                                            int l16) {
    constexpr int CQ = WSplit<KCH, KS, Q5>::CQ;
    const int rl = slot / KS, ks = slot - rl * KS, row = rb + rl;
    const bool ok = rl < 16 / KS && row < r1;
    const int64_t e0 = (int64_t)(ok ? row : 0) * K + ks * CQ * 128 + l16 * 8;
#pragma unroll
    for (int c = 0; c < CQ; ++c) wc_zero(S.w[c]);
    if (ok) {
#pragma unroll
        for (int c = 0; c < CQ; ++c) wc_load(S.w[c], m, e0 + c * 128);
    }
}

// In-wave combine (KS = 2, or KS = 4 for epilogues that do not pair rows):
// a row's KS quarters are quarters of ONE wave, so its partials are added
// across lanes (permlane16 / permlane32 swaps) in ks order — bitwise the LDS
// order — with no LDS round trip and no workgroup barrier.  The rows then sit
// in the wave as wsplit_row says (KS = 2: wave w quarters 0 / 1 = rows 2w /
// 2w + 1, adjacent for the pairing epilogues; KS = 4: wave w quarter 0 = row w).
template <int KS, bool PAIR>
constexpr bool wsplit_inwave() { return KS == 2 || (KS == 4 && !PAIR); }
// this lane's row-local index after the in-wave combine, or -1
template <int KS>
__device__ __forceinline__ int wsplit_row(int w, int q) {
    if constexpr (KS == 2) return q < 2 ? 2 * w + q : -1;
    else return q == 0 ? w : -1;
}

// epi(row, b, v, bias, valid) as wset_dot's: called by every lane of the
// first 16 / KS quarters, quarter q carrying row rb + q (lane l16: decoder row
// l16); in-wave (wsplit_inwave): the quarters wsplit_row names
template <int BT, int KCH, int KS, bool Q5, bool PAIR = true, typename Epi>
__device__ __forceinline__ void wsplit_dot(const WSplit<KCH, KS, Q5> &S, const f16 *xs, int K, int B, int rb, int r1,
                                           int slot, int l16, float bias, float *kpart, Epi &&epi) {
    constexpr int CQ = WSplit<KCH, KS, Q5>::CQ;
    const int rl = slot / KS, ks = slot - rl * KS, sh = (l16 & 3) * 8;
    float acc[BT];
#pragma unroll
    for (int b = 0; b < BT; ++b) acc[b] = 0.0f;
    if constexpr (BT == 1 && CQ <= 8 && CQ >= PRE_GEMV_MIN) {
        half8 xa[CQ];
        xs_chunks(xa, xs, ks * CQ, l16);
#pragma unroll
        for (int c = 0; c < CQ; ++c) acc[0] = dot8(wc_h8(S.w[c], sh), xa[c], acc[0]);
    } else
#pragma unroll
    for (int c = 0; c < CQ; ++c) {
        const half8 wv = wc_h8(S.w[c], sh);
#pragma unroll
        for (int b = 0; b < BT; ++b)
            if (b < B) acc[b] = dot8(wv, *(const half8 *)(xs + b * K + (ks * CQ + c) * 128 + l16 * 8), acc[b]);
    }
    float v = 0.0f;
#pragma unroll
    for (int b = 0; b < BT; ++b)
        if (b < B) {
            const float t = red16_sum(acc[b]);
            if (l16 == b) v = t;
        }
    if constexpr (wsplit_inwave<KS, PAIR>()) {
        const int w = slot >> 2, q = slot & 3;
        // (swap16: a0 = quarter 0 / 2's value in quarters 0-1 / 2-3, a1 =
        // quarter 1 / 3's; swap32: c0 = quarter 0 / 1's value in both halves,
        // c1 = quarter 2 / 3's)
        uint32_t a0, a1, c0, c1;
        swap16(__float_as_uint(v), a0, a1);
        float sum;
        if constexpr (KS == 2) {
            sum = v + __uint_as_float(a1);          // quarters 0 / 2: p0 + p1 of rows 2w / 2w + 1
            swap32(__float_as_uint(sum), c0, c1);   // quarter 0 <- quarter 2's sum (c1)
            swap16(c1, a0, a1);                     // quarter 1 <- quarter 0's c1 (a0)
            sum = q == 1 ? __uint_as_float(a0) : sum;
        } else {
            uint32_t d0, d1;
            swap32(__float_as_uint(v), c0, c1);     // quarter 0 <- quarter 2 (p2)
            swap32(a1, d0, d1);                     // quarter 0 <- quarter 2's a1 = p3
            sum = ((v + __uint_as_float(a1)) + __uint_as_float(c1)) + __uint_as_float(d1);
        }
        const int rloc = wsplit_row<KS>(w, q);
        const int row = rb + (rloc < 0 ? 0 : rloc);
        epi(row, l16, sum, bias, rloc >= 0 && row < r1 && l16 < B);
        return;
    }
    if (l16 < PMAXB && rl < 16 / KS) kpart[(rl * KS + ks) * PMAXB + l16] = v;
    __syncthreads();
    const int row = rb + slot;
    float sum = 0.0f;
    if (slot < 16 / KS && l16 < PMAXB) {
        sum = kpart[(slot * KS) * PMAXB + l16];
#pragma unroll
        for (int k = 1; k < KS; ++k) sum = sum + kpart[(slot * KS + k) * PMAXB + l16];
    }
    epi(row, l16, sum, bias, slot < 16 / KS && row < r1 && l16 < B);
}

// a phase's weight set: split-K (KS > 1) or one quarter-wave per row
template <int KCH, int NP, int KS, bool Q5 = false, bool PAIR = true>
struct GSet {
    WSplit<KCH, KS, Q5> s;
    float bias;
    __device__ __forceinline__ void load(const WMat &W, const float *b, int K, int rb, int r1, int slot, int l16) {
        wsplit_load(s, W, K, rb, r1, slot, l16);
        bias = 0.0f;
        // (the row this quarter carries into the epilogue)
        const int rloc = wsplit_inwave<KS, PAIR>() ? wsplit_row<KS>(slot >> 2, slot & 3) : slot < 16 / KS ? slot : -1;
        if (b && rloc >= 0 && rb + rloc < r1) bias = *glb(b + rb + rloc);
    }
    __device__ __forceinline__ void pre(int l16) { wsplit_pre(s, l16); }
    template <int BT, typename Epi>
    __device__ __forceinline__ void dot(const f16 *xs, int K, int B, int rb, int r1, int slot, int l16, float *kpart,
                                        Epi &&epi) const {
        wsplit_dot<BT, KCH, KS, Q5, PAIR>(s, xs, K, B, rb, r1, slot, l16, bias, kpart, epi);
    }
};
template <int KCH, int NP, bool Q5, bool PAIR>
struct GSet<KCH, NP, 1, Q5, PAIR> {
    WSet<KCH, NP, Q5> s;
    __device__ __forceinline__ void load(const WMat &W, const float *b, int K, int rb, int r1, int slot, int l16) {
        wset_load(s, W, b, K, rb, r1, slot, l16);
    }
    __device__ __forceinline__ void pre(int l16) { wset_pre(s, l16); }
    template <int BT, typename Epi>
    __device__ __forceinline__ void dot(const f16 *xs, int K, int B, int rb, int r1, int slot, int l16, float *,
                                        Epi &&epi) const {
        wset_dot<BT>(s, xs, K, B, rb, r1, slot, l16, epi);
    }
};

// ---- MFMA GEMV (n <= 512): a phase's rows [rb, r1) (at most 16 NP) as
// v_mfma_f32_16x16x32_f16 tiles with the decoder rows' inputs as A (rows >= B
// zero) and 16 weight rows as B; wave w takes the 32-k steps
// [w NKQ, (w + 1) NKQ), and the four waves' partials meet in LDS (kp) and
// are added in wave order.  Each (weight row, decoder row) result is one fixed
// chain of MFMAs and additions, independent of B.  The epilogue runs in the
// quarter-wave layout of wset_dot (quarter slot = weight row rb + 16 p +
// slot, lane l16 = decoder row), so the phases' callbacks (and their pairing
// shuffles) are shared with the VALU GEMVs.
template <int KCH, int NP, bool Q5 = false, bool ALDS = false>  // ALDS: A fragments read from LDS per step
struct MSet {
    static constexpr int NKQ = KCH;  // (K / 32) / 4 MFMA steps per wave
    // q5_1 chunks dequantised at each MFMA step, not in the poll: holding
    // every chunk's blocks and its f16 weights until the poll ended spilled
    // the 8-row instance at n = 768 (604 B a lane; 72 B now): small-q5_1 x 8
    // clips 124.7 -> 94.0 ms decode (profiles/r06/q5_lazy_dequant_ab.txt)
    static constexpr bool LAZY = Q5;
    WChunk<Q5> c[NP][NKQ];
    float bias[NP];
    __device__ __forceinline__ void load(const WMat &W, const float *b, int K, int rb, int r1, int slot, int) {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane & 15, lh = lane >> 4;
#pragma unroll
        for (int t = 0; t < NP; ++t) {
            const int row = rb + 16 * t + lr;
            const bool ok = row < r1;
            const int64_t e0 = (int64_t)(ok ? row : 0) * K + 32 * (w * NKQ) + 8 * lh;
#pragma unroll
            for (int i = 0; i < NKQ; ++i) wc_zero(c[t][i]);
            if (ok) {
#pragma unroll
                for (int i = 0; i < NKQ; ++i) wc_load(c[t][i], W, e0 + 32 * i);
            }
            const int r2 = rb + 16 * t + slot;
            bias[t] = 0.0f;
            if (b && r2 < r1) bias[t] = *glb(b + r2);
        }
    }
    __device__ __forceinline__ void pre(int) {
        if constexpr (LAZY) return;
        const int lh = (threadIdx.x & 63) >> 4;
#pragma unroll
        for (int t = 0; t < NP; ++t)
#pragma unroll
            for (int i = 0; i < NKQ; ++i) wc_pre(c[t][i], 8 * lh);
    }
    __device__ __forceinline__ half8 bfrag(int t, int i, int lh) const {
        if constexpr (LAZY) return q5_half8(c[t][i].n, c[t][i].hd[0], c[t][i].hd[1], 8 * lh);
        else return wc_h8(c[t][i], 0);
    }
    // kp: LDS [4][NP][16][8] floats
    template <int BT, typename Epi>
    __device__ __forceinline__ void dot(const f16 *xs, int K, int B, int rb, int r1, int slot, int l16, float *kp,
                                        Epi &&epi) const {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, lr = lane & 15, lh = lane >> 4;
        const half8 z8 = {};
        half8 af[ALDS ? 1 : NKQ];
        auto afrag = [&](int i) {
            const half8 v = *(const half8 *)(xs + (lr < B ? lr : 0) * K + 32 * (w * NKQ + i) + 8 * lh);
            return lr < B ? v : z8;
        };
        if constexpr (!ALDS) {
#pragma unroll
            for (int i = 0; i < NKQ; ++i) af[i] = afrag(i);
        }
#pragma unroll
        for (int t = 0; t < NP; ++t) {
            if (rb + 16 * t >= r1) break;  // workgroup-uniform
            floatx4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < NKQ; ++i)
                d = __builtin_amdgcn_mfma_f32_16x16x32_f16(ALDS ? afrag(i) : af[i], bfrag(t, i, lh), d, 0, 0, 0);
            if (lh < 2)
#pragma unroll
                for (int r = 0; r < 4; ++r) kp[((w * NP + t) * 16 + lr) * 8 + 4 * lh + r] = d[r];
        }
        __syncthreads();
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if (rb + 16 * p >= r1) break;  // workgroup-uniform
            const int row = rb + 16 * p + slot, bq = l16 < 8 ? l16 : 0;
            const float v0 = kp[((0 * NP + p) * 16 + slot) * 8 + bq], v1 = kp[((1 * NP + p) * 16 + slot) * 8 + bq];
            const float v2 = kp[((2 * NP + p) * 16 + slot) * 8 + bq], v3 = kp[((3 * NP + p) * 16 + slot) * 8 + bq];
            const float v = ((v0 + v1) + v2) + v3;
            epi(row, l16, l16 < 8 ? v : 0.0f, bias[p], row < r1 && l16 < B);
        }
    }
};
// a phase's weight set: MFMA for several rows at n <= 512, else VALU.  One
// row keeps the quarter-wave VALU GEMVs: on MFMA its step took 3.6 % longer
// (base 18.56 vs 17.84 ms decode; 8 rows 28.8 vs 32.0 ms, A/B x3,
// profiles/r03/gemv_mfma_ab.txt), so a clip decoded alone and in a batch sum
// its GEMV dots in different (each fixed) orders
// (the K = 4n phase I above n = 512 reads its A fragments from LDS at each
// MFMA step instead of holding all 4n / 128 of them in registers)
// PAIR: the phase's epilogue pairs adjacent rows (f16-pair outputs)
template <int NS, int BT, int KCH, int NP, int KS, bool Q5, bool PAIR = true>
using PSet = typename std::conditional<
    (BT > 1),
    typename std::conditional<(NS <= 512 || KCH <= NS / 128), MSet<KCH, NP, Q5>, MSet<KCH, NP, Q5, true>>::type,
    GSet<KCH, NP, KS, Q5, PAIR>>::type;

// LayerNorm (ggml norm: double mean / variance, eps 1e-5; then * w + b) of
// rows b < B of xf [B][NS] into xs [B][NS] f16 — wave w takes rows w, w + 4.
// One pass: var = E[x^2] - mean^2 in double (the f32 inputs' squares are
// exact in double; against ggml's two-pass sum the variance differs by
// ~1e-16 relative, so the f32 scale is the same unless that double lies
// within 1e-16 of an f32 rounding boundary)
template <int NS>
struct LnP {
    static constexpr int V = (NS + 255) / 256;
    float4 w[V], b[V];
};
template <int NS>
__device__ __forceinline__ void ln_params(const float *lw, const float *lb, LnP<NS> &P, int lane) {
#pragma unroll
    for (int i = 0; i < LnP<NS>::V; ++i) {
        const int e = (lane + 64 * i) * 4, ec = e < NS ? e : 0;
        P.w[i] = *glb((const float4 *)(lw + ec));
        P.b[i] = *glb((const float4 *)(lb + ec));
    }
}
// The multi-row phases' LayerNorm parameters, requested before the phase's
// poll, pass through an empty asm right there (n <= 512): the compiler
// otherwise re-issues these invariant loads where ln_rows first uses them,
// after the poll, and waits for them there with a vmcnt that also covers
// everything requested since (in the logits phase: the streamed vocabulary
// tiles).  C4's shard 8 352 -> 8 506 audio-s/s; above n = 512 the settled
// registers cost more than the late loads (C5 118.1 -> 116.6), and a
// workgroup-wide multi-row LayerNorm there measured far slower (C5 97)
// (profiles/r04/ln_settle_ab.txt)
template <int NS>
__device__ __forceinline__ void ln_params_early(const float *lw, const float *lb, LnP<NS> &P, int lane) {
    ln_params<NS>(lw, lb, P, lane);
    if constexpr (NS <= 512) {
#pragma unroll
        for (int i = 0; i < LnP<NS>::V; ++i) {
            float4 w = P.w[i], b = P.b[i];
            asm volatile("" : "+v"(w.x), "+v"(w.y), "+v"(w.z), "+v"(w.w), "+v"(b.x), "+v"(b.y), "+v"(b.z), "+v"(b.w));
            P.w[i] = w;
            P.b[i] = b;
        }
    }
}
template <int NS>
__device__ __forceinline__ void ln_rows(const float *xf, const LnP<NS> &P, f16 *xs, int B, int w, int lane) {
    constexpr int LV = LnP<NS>::V;
    if (w + 4 < B) {
        // rows w and w + 4 of this wave together (independent chains: twice
        // the ILP of the row-by-row loop); each row's arithmetic as below
        float4 xa[LV], xb[LV];
#pragma unroll
        for (int i = 0; i < LV; ++i) {
            const int e = (lane + 64 * i) * 4, ec = e < NS ? e : 0;
            xa[i] = *(const float4 *)(xf + w * NS + ec);
            xb[i] = *(const float4 *)(xf + (w + 4) * NS + ec);
        }
        double sa1 = 0.0, sa2 = 0.0, sb1 = 0.0, sb2 = 0.0;
#pragma unroll
        for (int i = 0; i < LV; ++i)
            if ((lane + 64 * i) * 4 < NS) {
                const double a0 = xa[i].x, a1 = xa[i].y, a2 = xa[i].z, a3 = xa[i].w;
                const double b0 = xb[i].x, b1 = xb[i].y, b2 = xb[i].z, b3 = xb[i].w;
                sa1 += (a0 + a1) + (a2 + a3);
                sa2 += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
                sb1 += (b0 + b1) + (b2 + b3);
                sb2 += (b0 * b0 + b1 * b1) + (b2 * b2 + b3 * b3);
            }
        sa1 = wave_sum(sa1);
        sb1 = wave_sum(sb1);
        sa2 = wave_sum(sa2);
        sb2 = wave_sum(sb2);
        const double ma = sa1 / NS, mb = sb1 / NS;
        const float ka = (float)(1.0 / sqrt((sa2 / NS - ma * ma) + (double)1e-5f));
        const float kb = (float)(1.0 / sqrt((sb2 / NS - mb * mb) + (double)1e-5f));
#pragma unroll
        for (int i = 0; i < LV; ++i) {
            const int e = (lane + 64 * i) * 4;
            if (e < NS) {
                const float a4[4] = {xa[i].x, xa[i].y, xa[i].z, xa[i].w}, b4[4] = {xb[i].x, xb[i].y, xb[i].z, xb[i].w};
                const float ww[4] = {P.w[i].x, P.w[i].y, P.w[i].z, P.w[i].w};
                const float bb[4] = {P.b[i].x, P.b[i].y, P.b[i].z, P.b[i].w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    xs[w * NS + e + u] = f16_rt(bb[u] + ww[u] * ((float)((double)a4[u] - ma) * ka));
                    xs[(w + 4) * NS + e + u] = f16_rt(bb[u] + ww[u] * ((float)((double)b4[u] - mb) * kb));
                }
            }
        }
        return;
    }
    for (int b = w; b < B; b += 4) {
        float4 xv[LV];
#pragma unroll
        for (int i = 0; i < LV; ++i) {
            const int e = (lane + 64 * i) * 4;
            xv[i] = e < NS ? *(const float4 *)(xf + b * NS + e) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int i = 0; i < LV; ++i)
            if ((lane + 64 * i) * 4 < NS) {
                const double d0 = xv[i].x, d1 = xv[i].y, d2 = xv[i].z, d3 = xv[i].w;
                s1 += (d0 + d1) + (d2 + d3);
                s2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
            }
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        const double mean = s1 / NS;
        const float scale = (float)(1.0 / sqrt((s2 / NS - mean * mean) + (double)1e-5f));
#pragma unroll
        for (int i = 0; i < LV; ++i) {
            const int e = (lane + 64 * i) * 4;
            if (e < NS) {
                const float xx[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
                const float ww[4] = {P.w[i].x, P.w[i].y, P.w[i].z, P.w[i].w};
                const float bb[4] = {P.b[i].x, P.b[i].y, P.b[i].z, P.b[i].w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float t = (float)((double)xx[u] - mean) * scale;
                    xs[b * NS + e + u] = f16_rt(bb[u] + ww[u] * t);
                }
            }
        }
    }
}

// One-row LayerNorm over the whole workgroup (B = 1 instances): thread tid
// holds elements e = tid + PT u — the layout in which a PT-thread poll of NS
// granules receives them — so the statistics start from the poll's registers
// (one partial per thread, a wave sum, one LDS exchange) instead of one wave
// re-reading the row from LDS; same one-pass formula as ln_rows.
template <int NS>
struct Ln1P {
    static constexpr int NE = (NS + PT - 1) / PT;
    float w[NE], b[NE];
};
template <int NS>
__device__ __forceinline__ void ln1_params(const float *lw, const float *lb, Ln1P<NS> &P, int tid) {
#pragma unroll
    for (int u = 0; u < Ln1P<NS>::NE; ++u) {
        const int e = tid + PT * u, ec = e < NS ? e : 0;
        P.w[u] = *glb(lw + ec);
        P.b[u] = *glb(lb + ec);
    }
}
// statistics over the workgroup (every thread calls; sh.abort_ is raised when
// !ok and checked at the one barrier) and xs[e] = f16(b + w * f32(x - mean) * scale)
template <int NS>
__device__ __forceinline__ bool ln1_vals(const float (&xv)[Ln1P<NS>::NE], const Ln1P<NS> &P, f16 *xs, bool ok,
                                         double *r1, double *r2, int *abort_) {
    constexpr int NE = Ln1P<NS>::NE;
    int tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, w = tid >> 6;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int u = 0; u < NE; ++u)
        if (tid + PT * u < NS) {
            const double d = xv[u];
            s1 += d;
            s2 += d * d;
        }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
        r1[w] = s1;
        r2[w] = s2;
    }
    if (!ok) *abort_ = 1;
    __syncthreads();
    if (*abort_) return false;
    const double S1 = ((r1[0] + r1[1]) + r1[2]) + r1[3], S2 = ((r2[0] + r2[1]) + r2[2]) + r2[3];
    const double mean = S1 / NS;
    const float scale = (float)(1.0 / sqrt((S2 / NS - mean * mean) + (double)1e-5f));
#pragma unroll
    for (int u = 0; u < NE; ++u) {
        const int e = tid + PT * u;
        if (e < NS) {
            const float t = (float)((double)xv[u] - mean) * scale;
            xs[e] = f16_rt(P.b[u] + P.w[u] * t);
        }
    }
    return true;
}
// poll one row's NS f32 granules (src[e], tag) into registers and xf, then
// ln1_vals; false: the grid is aborting
template <int NS, typename Pre = NoPre>
__device__ __forceinline__ bool poll_ln1(const uint64_t *src, uint32_t tag, const Ln1P<NS> &P, float *xf, f16 *xs,
                                         uint32_t *abortw, uint32_t *err, double *r1, double *r2, int *abort_,
                                         Pre pre = Pre{}) {
    constexpr int NE = Ln1P<NS>::NE;
    int tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
    uint64_t v[NE];
#pragma unroll
    for (int u = 0; u < NE; ++u) {
        const int e = tid + PT * u;
        v[u] = e < NS ? gld(src + e) : ((uint64_t)tag << 32);
    }
    pre();  // (see gpoll)
    bool ok = true;
    for (uint32_t it = 0;; ++it) {
        bool all = true;
#pragma unroll
        for (int u = 0; u < NE; ++u)
            if ((uint32_t)(v[u] >> 32) != tag) {
                all = false;
                v[u] = gld(src + tid + PT * u);
            }
        if (all) break;
        if ((it & 15) == 15) {
            if (ld32(abortw)) { ok = false; break; }
            if (it > PSPIN) {
                st32(abortw, 1u);
                atomicOr(err, 8u);
                ok = false;
                break;
            }
        }
    }
    float xv[NE];
#pragma unroll
    for (int u = 0; u < NE; ++u) {
        const int e = tid + PT * u;
        xv[u] = __uint_as_float((uint32_t)v[u]);
        if (e < NS) xf[e] = xv[u];
    }
    return ln1_vals<NS>(xv, P, xs, ok, r1, r2, abort_);
}

// ggml's table_exp_f16 value f16(exp(double(f16 x))) for x <= 0 without a
// double exp (whose polynomial constants the compiler would keep live in
// registers across the whole persistent loop): the f32 exp rounds to the same
// f16 unless it lies within 4 f32 ulps of an f16 rounding midpoint.  Those
// inputs (~19 of the 31744 non-positive ones) are found once per context on
// the device (k_exp_fallbacks) and their table values kept in a 64-entry
// list {j << 16 | value} (0xffffffff-padded) that the kernel holds in LDS:
// the rare lane reads it with 16 independent LDS loads instead of waiting
// for a global table load.
__device__ __forceinline__ bool exp_f16_fast_ok(float arg, f16 &hx, float &hv) {
    hx = (f16)arg;
    const float r = expf((float)hx);
    const uint16_t hr = f2h_bits(r);
    hv = h2f_bits(hr);
    const float nb = h2f_bits(r >= hv ? (uint16_t)(hr + 1) : (uint16_t)(hr - 1));
    const float mid = 0.5f * (hv + nb);
    const float ulp = __uint_as_float(__float_as_uint(r) & 0x7f800000u) * 1.1920928955078125e-7f;
    return fabsf(r - mid) > 4.0f * ulp;
}
// The same value branch-free: the fallback inputs sit in a 64-slot table
// addressed by a multiplicative hash of the f16 magnitude j (slot
// (j * K) >> 26, K chosen on the host so the listed inputs get distinct
// slots; an empty slot holds 0xffffffff).  Every lane reads its slot (one
// word per bank: no bank conflicts) and takes the table value when the
// slot's key is j, else the f16 of the f32 exp — no divergent list scan.
__device__ __forceinline__ float exp_f16_hash(float arg, const uint32_t *fbt, uint32_t K) {
    const f16 hx = (f16)arg;
    const float hv = h2f_bits(f2h_bits(expf((float)hx)));
    const uint32_t j = __builtin_bit_cast(uint16_t, hx) & 0x7fff;
    const uint32_t e = fbt[(j * K) >> 26];
    return (e >> 16) == j ? h2f_bits((uint16_t)e) : hv;
}

// Every phase re-derives its lane indices from an opaque copy of threadIdx.x
// behind a compiler memory barrier: __syncthreads() fences only LDS, so
// without it the compiler hoists later phases' weight loads and lane
// addresses into earlier phases and keeps all of them live at once (512
// VGPRs and scratch spills for phases that each need < 256).
#define PHASE_IDS                                                                              \
    int tid = (int)threadIdx.x;                                                                \
    asm volatile("" : "+v"(tid) : : "memory");                                                 \
    const int lane = tid & 63, w = tid >> 6, q = lane >> 4, l16 = lane & 15, slot = w * 4 + q; \
    (void)q; (void)l16; (void)slot;

// WMI_PTRACE: thread 0 of workgroups 0 and G / 2 stamps the 100 MHz device
// clock at the end of every phase of the first launch (host prints averages)
#define PSTAMP(ph)                                                                                    \
    if (a.ptrace && threadIdx.x == 0 && (wg == 0 || wg == G / 2))                                     \
        a.ptrace[(((int64_t)step * (L + 1) + (ph) / 32) * 32 + ((ph) & 31)) * 2 + (wg == 0 ? 0 : 1)] = \
            __builtin_amdgcn_s_memrealtime();

// Weight / operand loads issued ahead of a poll must stay ahead of it: the
// compiler otherwise sinks them to their first use, after the poll, and the
// whole load latency lands behind the seam.  Nothing waits here.
#define PREFETCH_ISSUED asm volatile("" : : : "memory");
// (the workgroup barrier in front of every poll stays even where no LDS
// hazard needs it: without it the waves' polls spread out and the base step
// took 142.5 vs 136.2 us, profiles/r04/prepoll_barrier_ab_REJECTED.txt)

// BT: rows at compile time (1) or at most (8, runtime B); BEAM: beam-search
// launches (self-attention history through kv_src; its index registers stay
// out of the greedy instances)
template <int NS, int BT, bool BEAM, bool Q5>
__global__ __launch_bounds__(PT, 1) void k_dec_persist(PersistArgs a) {
    constexpr int KC = NS / 128;        // 128-element chunks of a K = n row
    constexpr int H = NS / 64;
    constexpr int NPL = KC <= 4 ? 2 : 1;  // logits passes per register set
    // logits on MFMA (n <= 512): v_mfma_f32_16x16x32_f16 with the rows'
    // hidden states as A (rows >= B zero) and 16 vocabulary rows as B
    constexpr bool LMF = KC <= 4;
    // several rows at n > 512: the four waves split K (n / 4 each) over every
    // 16-row tile, partials added in wave order through LDS (the A fragments
    // and a tile's B fragments of all of K would not fit the registers)
    constexpr bool LMF2 = !LMF && BT > 1;
    constexpr bool XQF = KC <= 6;  // cross q computed inside the score tasks (registers allow)
    // 128-key sub-chunks per cross-attention task: one row runs 128-key
    // chunks (H * ceil(T / 128) <= G tasks; 256 on a smaller grid), several
    // rows up to 512 (launch_dec_persist checks)
    constexpr int NKE = BT == 1 ? 2 : NKP;
    // beam rows share one clip's cross K / V tasks (PersistArgs::xshare)
    const bool xsh = BEAM && !XQF && a.xshare;
    // split-K factors of the GEMV phases (quarter-waves per row), from the
    // rows a workgroup owns at the full grid
    constexpr int KS_N = split_of(KC, rows_full(NS)), KS_I = split_of(4 * KC, rows_full(NS));
    constexpr int KS_A = split_of(KC, rows_full(3 * NS)), KS_H = split_of(KC, rows_full(4 * NS));
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ PShared sh;
    const int B = BT == 1 ? 1 : a.B, G = gridDim.x, wg = blockIdx.x;
    if (wg == a.stall_wg) return;  // (fault injection: a workgroup that never ran)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int L = a.L, T = a.T, tctx = a.tctx, nch = a.nch, CL = a.cl;
    const int nsub = (T + 127) >> 7;  // 128-key P.V partials per (row, head)
    // granules in flight per thread for the all-to-all polls (8-byte sc1
    // loads; one round of loads per L2/MALL round trip): the whole vector
    // in one round where registers allow
    constexpr int PUX = BT == 1 ? (NS <= 1024 ? 4 : 8) : 16;   // B x n f32
    constexpr int PUH = BT == 1 ? (NS <= 512 ? 4 : NS <= 1024 ? 8 : 16) : 16;  // B x 2n f16 pairs
    float *xf = (float *)smem;                                          // [B][NS] f32
    f16 *xs = (f16 *)(smem + (size_t)B * NS * 4);                       // [B][4 NS] f16
    unsigned char *scr = smem + (size_t)B * NS * 4 + (size_t)B * NS * 8;  // scr_bytes(BT)
    f16 *vres = (f16 *)(scr + scr_bytes(BT));                              // [nres][NS] resident vocabulary rows
    // exchange offsets as plain scalars (a struct captured by the lambdas
    // below would be kept in scratch memory)
    int oX1, oX2, oX3, oQ, oK, oV, oO, oXQ, oOC, oH, oS, oP, oA;
    {
        const XLayout X = persist_layout(NS, H, T);
        oX1 = X.x1; oX2 = X.x2; oX3 = X.x3; oQ = X.q; oK = X.k; oV = X.v; oO = X.o; oXQ = X.xq;
        oOC = X.oc; oH = X.h; oS = X.s; oP = X.p; oA = X.a;
    }
    uint64_t *xg = a.xg;
    uint32_t *abortw = (uint32_t *)(xg + persist_layout(NS, H, T).ctl);
    const float qs = a.qscale;
    // row partitions (f16-pair outputs need even row starts)
    auto part = [&](int N, bool even, int &r0, int &r1) {
        int rpw = (N + G - 1) / G;
        if (even) rpw = (rpw + 1) & ~1;
        r0 = wg * rpw < N ? wg * rpw : N;
        r1 = r0 + rpw < N ? r0 + rpw : N;
    };
    int rn0, rn1, ra0, ra1, rh0, rh1, rv0, rv1;
    part(NS, true, rn0, rn1);      // Wo / Wcq / Wco / W1 rows = this WG's residual rows
    part(3 * NS, true, ra0, ra1);  // Wqkv rows
    part(4 * NS, true, rh0, rh1);  // W0 rows
    // the GEMV phases' partial sums: LDS scratch for the MFMA GEMVs, else the split-K buffer
    float *kpbuf = BT > 1 ? (float *)scr : sh.kpart;  // (an MSet phase's partials; sh.kpart for GSet's split-K)
    part(a.V, false, rv0, rv1);
    const int rn = rn1 - rn0;
    // this workgroup's first vocabulary rows stay in LDS for the whole launch
    const int rs0 = rv0 + a.nres < rv1 ? rv0 + a.nres : rv1;
    {
        const uint4 *src = (const uint4 *)((const f16 *)a.te + (int64_t)rv0 * NS);
        uint4 *dst = (uint4 *)vres;
        // (MFMA logits: 16-byte chunk c of resident row j at c ^ (j & 15), so
        // the 16 rows of a B fragment read hit distinct banks)
        for (int i = tid; i < (rs0 - rv0) * NS / 8; i += PT) {
            const int j = i / (NS / 8), c = i - j * (NS / 8);
            dst[LMF || LMF2 ? j * (NS / 8) + (c ^ (j & 15)) : i] = src[i];
        }
    }
    // one-row VALU logits (n = 768): the vocabulary rows past the LDS-resident
    // ones (at most 8 per quarter-wave slot) stay in registers for the whole
    // launch (PersistArgs::vreg) instead of streaming from the Infinity Cache
    // every step behind the logits poll.  (The same for the MFMA logits at
    // n <= 512 — five 16-row tiles — measured no faster at base and slower at
    // tiny against the streamed build: profiles/r04b/vs_first_session_*.)
    constexpr bool LREG2 = BT == 1 && !LMF && !LMF2 && KC <= 6;
    const bool lreg2 = LREG2 && a.vreg && rv1 - rs0 <= 128;
    WSet<LREG2 ? KC : 1, LREG2 ? 8 : 1> SR;
    if constexpr (LREG2) wset_load(SR, wmat(a.te), nullptr, NS, rs0, lreg2 ? rv1 : rs0, w * 4 + (lane >> 4), lane & 15);
    if (tid == 0) sh.abort_ = 0;
    if (tid < EXPFB) sh.expfb[tid] = a.exp_fb[tid];
    const uint32_t fbk = a.exp_fb[EXPFB + 1];  // the fallback table's hash multiplier
    __syncthreads();
    auto check = [&](bool ok) -> bool {  // workgroup-uniform abort after a poll
        if (!ok) sh.abort_ = 1;
        __syncthreads();
        return sh.abort_ != 0;
    };
    auto ptr_u64 = [](uint64_t *base) { return [base](int i) { return base + i; }; };

    // every workgroup reduces the G per-workgroup argmax candidates of the
    // logits at position pp: sh.tok[b]
    auto argmax_gather = [&](int pp) -> bool {
        uint32_t *ga = (uint32_t *)scr;  // [B][G][2]
        const bool ok = gpoll<BT == 1 ? 4 : 16>(B * G * 2, atag(pp, L), ptr_u64(xg + oA), ga, abortw, a.err);
        if (check(ok)) return false;
        for (int b = 0; b < B; ++b) {
            unsigned long long k = 0ull;
            if (tid < G) k = ((unsigned long long)ga[(b * G + tid) * 2] << 32) | ga[(b * G + tid) * 2 + 1];
            k = wave_max_u64(k);
            if (lane == 0) sh.best[w][b] = k;
        }
        __syncthreads();
        if (tid < B) {
            unsigned long long k = sh.best[0][tid];
            for (int i = 1; i < 4; ++i) k = sh.best[i][tid] > k ? sh.best[i][tid] : k;
            sh.tok[tid] = (int32_t)(0xffffffffu - (uint32_t)(k & 0xffffffffull));
        }
        __syncthreads();
        return true;
    };

    int pos = a.st->pos;
    for (int step = 0; step < a.n_steps; ++step, ++pos) {
        for (int l = 0; l < L; ++l) {
            ConstLayer &P = ((ConstLayer *)a.layers)[l];
            uint16_t *kc = a.kcache + (size_t)l * DEC_ROWS * tctx * NS;
            uint16_t *vc = a.vcache + (size_t)l * DEC_ROWS * tctx * NS;

            // ---- A: LN1 + QKV rows ------------------------------------
            {
                PHASE_IDS
                const uint32_t tag = ptag(pos, L, l, 0);
                PSet<NS, BT, KC, 2, KS_A, Q5> S;
                const bool act = ra0 < ra1;
                // (layer 0 of a generated position: requested after the
                // argmax gather, which then does not wait for them — they are
                // wanted only after the token's embedding row and its LayerNorm:
                // base 1859 -> 1890 audio-s/s, profiles/r05/l0_weights_after_argmax_ab.txt.
                // Not the q5_1 instances, whose dequantisation right behind the
                // loads would then also hold up the embedding loads)
                const bool late_w = !Q5 && l == 0 && pos >= a.feed_len && step > 0;
                if (!late_w) S.load(lmat<Q5>(P.wqkv, P.wqkv5, 3 * NS * NS), P.bqkv, NS, ra0, ra1, slot, l16);
                LnP<NS> lp;
                Ln1P<NS> l1;
                if constexpr (BT == 1) ln1_params<NS>(P.ln1_w, P.ln1_b, l1, tid);
                else ln_params_early<NS>(P.ln1_w, P.ln1_b, lp, lane);
                PREFETCH_ISSUED
                __syncthreads();
                if (l == 0) {
                    const bool fed = pos < a.feed_len;
                    if (fed) {
                        if (tid < B) sh.tok[tid] = a.feed[tid * a.feed_stride + pos];
                        __syncthreads();
                    } else if (step == 0) {
                        if (tid < B) sh.tok[tid] = a.cur_tok[tid];
                        __syncthreads();
                    } else {
                        if (!argmax_gather(pos - 1)) return;
                        S.load(lmat<Q5>(P.wqkv, P.wqkv5, 3 * NS * NS), P.bqkv, NS, ra0, ra1, slot, l16);
                        if (wg == 0 && tid < B && pos - a.feed_len < a.out_stride)
                            a.tokens_out[tid * a.out_stride + (pos - a.feed_len)] = sh.tok[tid];
                    }
                    S.pre(l16);  // (no poll to hide it behind in layer 0)
                    // x = te[tok] + pe[pos]  (get_rows f16 -> f32, add)
                    for (int i = tid; i < B * NS / 4; i += PT) {
                        const int b = (i * 4) / NS, e = i * 4 - b * NS;
                        const half4 tv = *(const half4 *)((const f16 *)a.te + (int64_t)sh.tok[b] * NS + e);
                        const float4 pv = *(const float4 *)(a.pe + (int64_t)pos * NS + e);
                        *(float4 *)(xf + b * NS + e) = make_float4((float)tv[0] + pv.x, (float)tv[1] + pv.y,
                                                                   (float)tv[2] + pv.z, (float)tv[3] + pv.w);
                    }
                    if constexpr (BT == 1) {
                        __syncthreads();
                        float xv[Ln1P<NS>::NE];
#pragma unroll
                        for (int u = 0; u < Ln1P<NS>::NE; ++u) xv[u] = xf[tid + PT * u < NS ? tid + PT * u : 0];
                        if (!ln1_vals<NS>(xv, l1, xs, true, sh.redd, sh.redd2, &sh.abort_)) return;
                    }
                } else {
                    if constexpr (BT == 1) {
                        if (!poll_ln1<NS>(xg + oX1, ptag(pos, L, l - 1, 10), l1, xf, xs, abortw, a.err, sh.redd, sh.redd2,
                                          &sh.abort_, [&] { S.pre(l16); }))
                            return;
                    } else {
                        const bool ok = gpoll<PUX>(B * NS, ptag(pos, L, l - 1, 10), ptr_u64(xg + oX1), (uint32_t *)xf, abortw, a.err,
                                                   [&] { S.pre(l16); });
                        if (check(ok)) return;
                    }
                PSTAMP(l * 32 + 16)
                }
                __syncthreads();
                for (int i = tid; i < B * rn; i += PT) {
                    const int b = i / rn, r = i - b * rn;
                    sh.xres[b][r] = xf[b * NS + rn0 + r];
                }
                if constexpr (BT > 1) {
                    ln_rows<NS>(xf, lp, xs, B, w, lane);
                    __syncthreads();
                }
                PSTAMP(l * 32 + 27)
                if (act)
                    S.template dot<BT>(xs, NS, B, ra0, ra1, slot, l16, kpbuf, [&](int row, int b, float v, float eb, bool valid) {
                        const float vn = from_next_row(v), ebn = from_next_row(eb);
                        if (!valid || (q & 1)) return;
                        const int which = row / NS, c = row - which * NS;
                        uint32_t pk;
                        if (which == 0) pk = pack2((v + eb) * qs, (vn + ebn) * qs);
                        else if (which == 1) pk = pack2(v * qs, vn * qs);
                        else pk = pack2(eb + v, ebn + vn);
                        const int64_t gi = (which == 0 ? oQ : which == 1 ? oK : oV) + b * (NS / 2) + c / 2;
                        // KV-cache row pos: an sc1 (write-through) store with no
                        // tag.  It is read from step pos + 1 on, by loads issued
                        // after that step's q/k/v poll; every hand-off between
                        // this store and that poll passes through a poll of this
                        // wave (its s_waitcnt vmcnt(0) on gfx9 also drains the
                        // store), so the row is in L2/memory before any granule
                        // that transitively signals it (documented,
                        // no fence — an agent release costs ~1.7 us per phase)
                        if (which > 0)
                            st32((uint32_t *)((which == 1 ? kc : vc) + ((int64_t)b * tctx + pos) * NS + c), pk);
                        gput(xg + gi, tag, pk);
                    });
            }

            PSTAMP(l * 32 + 0)
            // ---- B: self-attention per (row, head) ---------------------
            {
                PHASE_IDS
                const uint32_t tag = ptag(pos, L, l, 1);
                const int M = pos + 1;
                const __amdgpu_buffer_rsrc_t rk = rsrc_of(kc, (uint32_t)(DEC_ROWS * tctx * NS * 2));
                const __amdgpu_buffer_rsrc_t rv = rsrc_of(vc, (uint32_t)(DEC_ROWS * tctx * NS * 2));
                f16 *qn = (f16 *)scr, *kn = qn + 64, *vn = qn + 128;  // this step's q, k, v of the head
                uint16_t *P16 = (uint16_t *)(scr + 512);                 // [512]
                for (int t = wg; t < B * H; t += G) {
                    const int b = t / H, h = t - b * H;
                    const int doct = tid & 7, jg = tid >> 3;
                    // cache rows j < pos (this step's row comes from the granules)
                    half8 kv[2][8];
                    // (every register array is defined on every path — a
                    // conditionally-defined array becomes an undef value carried
                    // around the step loop and stays live across every phase)
                    const half8 z8 = {};
                    // cache row of key j: the row's own, or (beam search) the
                    // slot holding the hypothesis' history of position j
                    int srk[2], srv[16];
#pragma unroll
                    for (int r = 0; r < 2; ++r) srk[r] = b;
#pragma unroll
                    for (int i = 0; i < 16; ++i) srv[i] = b;
                    if (BEAM && a.kv_src) {  // every table load first, then every cache load
                        const int32_t *src = a.kv_src + (int64_t)b * a.kv_src_stride;
#pragma unroll
                        for (int r = 0; r < 2; ++r) {
                            const int j = tid + 256 * r;
                            srk[r] = src[j < pos ? j : 0];
                        }
#pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            const int j = jg + 32 * i;
                            srv[i] = src[j < pos ? j : 0];
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const int j = tid + 256 * r;
                        const uint32_t off = (uint32_t)((((int64_t)srk[r] * tctx + j) * NS + h * 64) * 2);
#pragma unroll
                        for (int i = 0; i < 8; ++i) kv[r][i] = j < pos ? bload_sc1(rk, off + 16 * i) : z8;
                    }
                    // value rows j < pos, in flight across the poll as well
                    half8 vv[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int j = jg + 32 * i;
                        vv[i] = j < pos ? bload_sc1(rv, (uint32_t)((((int64_t)srv[i] * tctx + j) * NS + h * 64 + doct * 8) * 2)) : z8;
                    }
                    PREFETCH_ISSUED
                    __syncthreads();
                    const int64_t hq = b * (NS / 2) + h * 32;  // q, k, v granule blocks lie 4 NS apart
                    // polled by the last wave: its score lanes hold keys >= 192
                    // (no cache-row loads before position 192) and its value
                    // lanes the fewest, so the poll does not wait for the
                    // cache rows the other waves requested (base 121.6 ->
                    // 118.6 us a step, profiles/r05/bpoll_lastwave_ab.txt)
                    const bool ok = gpoll<2, PT - 64, 64>(96, ptag(pos, L, l, 0),
                                          [=](int i) { return xg + oQ + (i >> 5) * (4 * NS) + hq + (i & 31); },
                                          (uint32_t *)qn, abortw, a.err);
                    if (check(ok)) return;
                PSTAMP(l * 32 + 17)
                    // scores: cache rows from registers, this step's row (same
                    // value in every lane) from the granules; no lane guards
                    half8 q8[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) q8[i] = *(const half8 *)(qn + 8 * i);
                    float snew = 0.0f;
#pragma unroll
                    for (int i = 0; i < 8; ++i) snew = dot8(*(const half8 *)(kn + 8 * i), q8[i], snew);
                    float sc[2];
                    float mx = -INFINITY;
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const int j = tid + 256 * r;
                        float s = 0.0f;
                        if (256 * r < pos)  // workgroup-uniform: skip all-zero rows
#pragma unroll
                            for (int i = 0; i < 8; ++i) s = dot8(kv[r][i], q8[i], s);
                        s = j < pos ? s : j == pos ? snew : 0.0f;
                        sc[r] = s;
                        if (j < M) mx = fmaxf(mx, s);
                    }
                    mx = wave_max(mx);
                    if (lane == 0) sh.redf[w] = mx;
                    __syncthreads();
                    mx = fmaxf(fmaxf(sh.redf[0], sh.redf[1]), fmaxf(sh.redf[2], sh.redf[3]));
                PSTAMP(l * 32 + 14)
                    // p = the ggml exp-table value of f16(s - max) (an f16
                    // value: stored exactly), and its double sum (exact in any
                    // order); P.V takes p unnormalised and the sum divides the
                    // result (ggml rounds f16(p / sum) first: the weights
                    // differ by that rounding, one barrier fewer)
                    double sum = 0.0;
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        if (tid + 256 * r < M) {
                            const float pr = exp_f16_hash(sc[r] - mx, sh.expfb, fbk);
                            sum += (double)pr;
                            P16[tid + 256 * r] = f2h_bits(pr);
                        }
                    }
                    sum = wave_sum(sum);
                    if (lane == 0) sh.redd[w] = sum;
                    __syncthreads();
                    const double inv = 1.0 / (((sh.redd[0] + sh.redd[1]) + sh.redd[2]) + sh.redd[3]);
                PSTAMP(l * 32 + 31)
                    // P.V in key order: rows past pos are zero registers and
                    // add exact zeros (o is never -0), so this step's row —
                    // the last key — is added after the loop
                    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                    float pv[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int j = jg + 32 * i;
                        pv[i] = h2f_bits(P16[j]);  // j < 512: inside the buffer
                    }
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        if (32 * i >= pos) break;  // workgroup-uniform: the rest add zeros
                        const int j = jg + 32 * i;
                        const float pj = j < pos ? pv[i] : 0.0f;
#pragma unroll
                        for (int e = 0; e < 8; ++e) o[e] = o[e] + pj * (float)vv[i][e];
                    }
                    if (jg == (pos & 31)) {
                        const float pj = h2f_bits(P16[pos]);
                        const half8 vr = *(const half8 *)(vn + doct * 8);
#pragma unroll
                        for (int e = 0; e < 8; ++e) o[e] = o[e] + pj * (float)vr[e];
                    }
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        o[e] = red_8_16_32(o[e]);
                    }
                    if (lane < 8)
#pragma unroll
                        for (int e = 0; e < 8; ++e) sh.ored[w][lane * 8 + e] = o[e];
                    __syncthreads();
                    if (tid < 32) {
                        const int d = 2 * tid;
                        const float o0 = ((sh.ored[0][d] + sh.ored[1][d]) + sh.ored[2][d]) + sh.ored[3][d];
                        const float o1 = ((sh.ored[0][d + 1] + sh.ored[1][d + 1]) + sh.ored[2][d + 1]) + sh.ored[3][d + 1];
                        gput(xg + oO + b * (NS / 2) + h * 32 + tid, tag, pack2((float)(o0 * inv), (float)(o1 * inv)));
                    }
                }
            }

            PSTAMP(l * 32 + 1)
            // ---- C: Wo rows + residual -> x' ---------------------------
            {
                PHASE_IDS
                const uint32_t tag = ptag(pos, L, l, 2);
                PSet<NS, BT, KC, 1, KS_N, Q5, false> S;
                const bool act = rn0 < rn1;
                S.load(lmat<Q5>(P.wo, P.wo5, NS * NS), P.bo, NS, rn0, rn1, slot, l16);
                PREFETCH_ISSUED
                __syncthreads();
                const bool ok = gpoll<PUX>(B * NS / 2, ptag(pos, L, l, 1), ptr_u64(xg + oO), (uint32_t *)xs, abortw, a.err,
                                           [&] { S.pre(l16); });
                if (check(ok)) return;
                PSTAMP(l * 32 + 18)
                if (act)
                    S.template dot<BT>(xs, NS, B, rn0, rn1, slot, l16, kpbuf, [&](int row, int b, float v, float eb, bool valid) {
                        if (!valid) return;
                        const float x = (v + eb) + sh.xres[b][row - rn0];
                        sh.xres[b][row - rn0] = x;
                        gput(xg + oX2 + b * NS + row, tag, __float_as_uint(x));
                    });
            }

            PSTAMP(l * 32 + 2)
            // ---- D: LNc(x') + Wcq rows -> cross q ------------------------
            // (n <= 768: folded into E, whose tasks compute their head's q)
            if constexpr (!XQF) {
                PHASE_IDS
                const uint32_t tag = ptag(pos, L, l, 3);
                PSet<NS, BT, KC, 1, KS_N, false> S;  // (MFMA with several rows)
                const bool act = rn0 < rn1;
                S.load(wmat(P.wcq), P.bcq, NS, rn0, rn1, slot, l16);
                LnP<NS> lp;
                Ln1P<NS> l1;
                if constexpr (BT == 1) ln1_params<NS>(P.lnc_w, P.lnc_b, l1, tid);
                else ln_params_early<NS>(P.lnc_w, P.lnc_b, lp, lane);
                PREFETCH_ISSUED
                __syncthreads();
                if constexpr (BT == 1) {
                    if (!poll_ln1<NS>(xg + oX2, ptag(pos, L, l, 2), l1, xf, xs, abortw, a.err, sh.redd, sh.redd2, &sh.abort_))
                        return;
                } else {
                    const bool ok = gpoll<PUX>(B * NS, ptag(pos, L, l, 2), ptr_u64(xg + oX2), (uint32_t *)xf, abortw, a.err);
                    if (check(ok)) return;
                    ln_rows<NS>(xf, lp, xs, B, w, lane);
                }
                PSTAMP(l * 32 + 19)
                __syncthreads();
                if (act)
                    S.template dot<BT>(xs, NS, B, rn0, rn1, slot, l16, kpbuf, [&](int row, int b, float v, float eb, bool valid) {
                        const float vn = from_next_row(v), ebn = from_next_row(eb);
                        if (!valid || (q & 1)) return;
                        gput(xg + oXQ + b * (NS / 2) + row / 2, tag, pack2((v + eb) * qs, (vn + ebn) * qs));
                    });
            }

            PSTAMP(l * 32 + 3)
            // ---- E: cross attention of (row, head, key chunk), flash-decoding
            // form.  Per 128-key sub-chunk: the scores s, their max m, p = the
            // ggml exp-table value of f16(s - m), the double sum S of p (f16
            // values in [0, 1]: exact in any order) and the unnormalised
            // o = sum p V; G1 rescales the sub-chunks to the row's max and
            // divides by the total sum.  One hand-off (E -> G1) where the global
            // softmax took two (one row: the scores to F) or three (several rows:
            // chunk maxima, chunk sums); the attention weights differ from
            // ggml's f16(p / S) only by the rounding of f16(s - m) against the
            // sub-chunk's max and the un-rounded division.
            // A sub-chunk's numbers depend only on its keys (one lane layout
            // whatever the task's chunk CL), so a row's cross o does not depend
            // on the row count, the chunking, or beam rows sharing a task.
            {
                PHASE_IDS
                const uint32_t tag = ptag(pos, L, l, 6);  // (G1 polls this tag)
                const int doct = tid & 7, jg = tid >> 3;  // P.V layout: 8 dims x 4 keys a lane
                if (xsh) {
                    // beam rows sharing one clip (cross q from D): one task per
                    // (head, 128-key chunk) covers every row, so a step reads
                    // each K / V chunk once; a row's arithmetic is the per-row
                    // task's, in the same order (launch_dec_persist: CL = 128)
                    f16 *qb = (f16 *)scr;                 // [B][64] this head's cross q of every row
                    float *st = (float *)(scr + XS_OFF);  // [B][128] p
                    const int ntask = H * nch;
                    for (int t = wg; t < ntask; t += G) {
                        const int c = t % nch, h = t / nch;
                        const int j0 = c * CL, j1 = j0 + CL < T ? j0 + CL : T;
                        const int64_t cb = ((int64_t)l * a.Bt + a.b0) * T * NS + h * 64;
                        const f16 *Kb = (const f16 *)a.ck + cb + (tid & 1) * 32;
                        const f16 *Vb = (const f16 *)a.cv + cb + doct * 8;
                        const int key = j0 + (tid >> 1);
                        half8 kf[4], vf[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) kf[i] = sld((const half8 *)(Kb + (int64_t)(key < j1 ? key : j1 - 1) * NS + 8 * i));
                        PREFETCH_ISSUED
                        __syncthreads();
                        const bool ok = gpoll(B * 32, ptag(pos, L, l, 3),
                                              [=](int i) { return xg + oXQ + (i >> 5) * (NS / 2) + h * 32 + (i & 31); },
                                              (uint32_t *)qb, abortw, a.err);
                        // the value rows (wanted after the scores and the exp
                        // sums) behind the poll, which then waits for the key
                        // rows only (vmcnt retires in order)
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int kv = j0 + jg * 4 + u;
                            vf[u] = sld((const half8 *)(Vb + (int64_t)(kv < j1 ? kv : j1 - 1) * NS));
                        }
                        if (check(ok)) return;
                PSTAMP(l * 32 + 20)
                        // (rows unrolled: their dot chains and max reductions interleave)
                        float sc[PMAXB];
#pragma unroll
                        for (int b = 0; b < PMAXB; ++b) {
                            sc[b] = 0.0f;
                            if (b >= B) continue;
                            float sv = 0.0f;
#pragma unroll
                            for (int i = 0; i < 4; ++i) sv = dot8(kf[i], *(const half8 *)(qb + b * 64 + (tid & 1) * 32 + 8 * i), sv);
                            sv = xstep<XSum, 1>(sv);
                            sc[b] = sv;
                            const float m = wave_max(key < j1 ? sv : -INFINITY);
                            if (lane == 0) sh.redfb[b][w] = m;
                        }
                        __syncthreads();
                        const bool own = key < j1 && (tid & 1) == 0;
#pragma unroll
                        for (int b = 0; b < PMAXB; ++b) {
                            if (b >= B) continue;
                            const float m = fmaxf(fmaxf(sh.redfb[b][0], sh.redfb[b][1]), fmaxf(sh.redfb[b][2], sh.redfb[b][3]));
                            const float pj = exp_f16_hash(sc[b] - m, sh.expfb, fbk);
                            if (own) st[b * 128 + key - j0] = pj;
                            const double s = wave_sum(own ? (double)pj : 0.0);
                            if (lane == 0) sh.reddb[b][w] = s;
                        }
                        __syncthreads();
                        float *ob = (float *)(scr + XS_OFF + XS_BYTES);  // [B][4 waves][64]
#pragma unroll
                        for (int b = 0; b < PMAXB; ++b) {
                            if (b >= B) continue;
                            float o[8];
#pragma unroll
                            for (int e = 0; e < 8; ++e) o[e] = 0.0f;
                            float sp[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const int kv = j0 + jg * 4 + u;
                                sp[u] = st[b * 128 + (kv < j1 ? kv : j1 - 1) - j0];
                            }
                            // keys past the chunk add p = 0 (o + 0 == o: o is never -0)
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                const float pj = j0 + jg * 4 + u < j1 ? sp[u] : 0.0f;
#pragma unroll
                                for (int e = 0; e < 8; ++e) o[e] = o[e] + pj * (float)vf[u][e];
                            }
#pragma unroll
                            for (int e = 0; e < 8; ++e) o[e] = red_8_16_32(o[e]);
                            if (lane < 8)
#pragma unroll
                                for (int e = 0; e < 8; ++e) ob[(b * 4 + w) * 64 + lane * 8 + e] = o[e];
                        }
                        __syncthreads();
                        for (int i = tid; i < B * 64; i += PT) {
                            const int b = i >> 6, d = i & 63;
                            const float *q4 = ob + b * 256 + d;
                            gput(xg + oP + (((int64_t)b * H + h) * nsub + c) * 64 + d, tag,
                                 __float_as_uint(((q4[0] + q4[64]) + q4[128]) + q4[192]));
                        }
                        if (tid < B) {
                            const int64_t sb = ((int64_t)tid * H + h) * nsub + c;
                            const double s = ((sh.reddb[tid][0] + sh.reddb[tid][1]) + sh.reddb[tid][2]) + sh.reddb[tid][3];
                            gput(xg + oS + 3 * sb, tag,
                                 __float_as_uint(fmaxf(fmaxf(sh.redfb[tid][0], sh.redfb[tid][1]),
                                                       fmaxf(sh.redfb[tid][2], sh.redfb[tid][3]))));
                            gput(xg + oS + 3 * sb + 1, tag, lo32(s));
                            gput(xg + oS + 3 * sb + 2, tag, hi32(s));
                        }
                    }
                } else {
                    f16 *qh = (f16 *)scr;                 // [64] this task's cross q
                    float *st = (float *)(scr + XS_OFF);  // [NKE][128] p
                    const int ntask = B * H * nch;
                    for (int t = wg; t < ntask; t += G) {
                        const int c = t % nch, bh = t / nch, h = bh % H, b = bh / H;
                        const int j0 = c * CL, j1 = j0 + CL < T ? j0 + CL : T;
                        const int64_t cb = ((int64_t)l * a.Bt + a.b0 + (a.beam ? 0 : b)) * T * NS + h * 64;
                        const f16 *Kb = (const f16 *)a.ck + cb + (tid & 1) * 32;
                        const f16 *Vb = (const f16 *)a.cv + cb + doct * 8;
                        half8 kf[NKE][4], vf[NKE][4];
                        const half8 z8 = {};
#pragma unroll
                        for (int p = 0; p < NKE; ++p) {
                            int key = j0 + 128 * p + (tid >> 1);
                            key = key < j1 ? key : j1 - 1;
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                kf[p][i] = 128 * p < CL ? sld((const half8 *)(Kb + (int64_t)key * NS + 8 * i)) : z8;
                        }
                        auto v_load = [&] {
#pragma unroll
                            for (int p = 0; p < NKE; ++p)
#pragma unroll
                                for (int u = 0; u < 4; ++u) {
                                    int kv = j0 + 128 * p + jg * 4 + u;
                                    kv = kv < j1 ? kv : j1 - 1;
                                    vf[p][u] = 128 * p < CL ? sld((const half8 *)(Vb + (int64_t)kv * NS)) : z8;
                                }
                        };
                        // (the value rows: with the key rows where the task
                        // computes its cross q — the q GEMV covers them — else
                        // behind the poll of q, which then waits for the key
                        // rows only: vmcnt retires in order)
                        if constexpr (XQF) v_load();
                        if constexpr (XQF) {
                            // this head's cross q from x' directly: LNc(x'_b) and
                            // Wcq rows h*64 .. h*64+63, the D phase's arithmetic
                            WSet<KC, 4> S;
                            wset_load(S, wmat(P.wcq), P.bcq, NS, h * 64, h * 64 + 64, slot, l16);
                            Ln1P<NS> l1;  // (the whole workgroup's LayerNorm of row b from the poll registers)
                            ln1_params<NS>(P.lnc_w, P.lnc_b, l1, tid);
                            PREFETCH_ISSUED
                            __syncthreads();
                            if (!poll_ln1<NS>(xg + oX2 + b * NS, ptag(pos, L, l, 2), l1, xf, xs, abortw, a.err, sh.redd,
                                              sh.redd2, &sh.abort_))
                                return;
                PSTAMP(l * 32 + 20)
                            __syncthreads();
                PSTAMP(l * 32 + 29)
                            wset_dot<1>(S, xs, NS, 1, h * 64, h * 64 + 64, slot, l16,
                                        [&](int row, int, float v, float eb, bool valid) {
                                            if (valid) qh[row - h * 64] = f16_rt((v + eb) * qs);
                                        });
                            __syncthreads();
                PSTAMP(l * 32 + 30)
                        } else {
                            PREFETCH_ISSUED
                            __syncthreads();
                            const bool ok = gpoll(32, ptag(pos, L, l, 3),
                                                  [=](int i) { return xg + oXQ + b * (NS / 2) + h * 32 + i; }, (uint32_t *)qh,
                                                  abortw, a.err);
                            v_load();
                            if (check(ok)) return;
                PSTAMP(l * 32 + 20)
                        }
                        // scores and the sub-chunk maxima
                        float sc[NKE];
#pragma unroll
                        for (int p = 0; p < NKE; ++p) {
                            sc[p] = 0.0f;
                            if (j0 + 128 * p < j1) {  // workgroup-uniform
                                const int key = j0 + 128 * p + (tid >> 1);
                                float s = 0.0f;
#pragma unroll
                                for (int i = 0; i < 4; ++i) s = dot8(kf[p][i], *(const half8 *)(qh + (tid & 1) * 32 + 8 * i), s);
                                s = xstep<XSum, 1>(s);
                                sc[p] = s;
                                const float m = wave_max(key < j1 ? s : -INFINITY);
                                if (lane == 0) sh.redfb[p][w] = m;
                            }
                        }
                        __syncthreads();
                        // p against the sub-chunk max, its exact double sum
#pragma unroll
                        for (int p = 0; p < NKE; ++p)
                            if (j0 + 128 * p < j1) {
                                const int key = j0 + 128 * p + (tid >> 1);
                                const float m = fmaxf(fmaxf(sh.redfb[p][0], sh.redfb[p][1]), fmaxf(sh.redfb[p][2], sh.redfb[p][3]));
                                const float pj = exp_f16_hash(sc[p] - m, sh.expfb, fbk);
                                const bool own = key < j1 && (tid & 1) == 0;
                                if (own) st[key - j0] = pj;
                                const double s = wave_sum(own ? (double)pj : 0.0);
                                if (lane == 0) sh.reddb[p][w] = s;
                            }
                        __syncthreads();
                PSTAMP(l * 32 + 11)
                        // unnormalised P.V per 128-key sub-chunk
                        float o[NKE][8];
#pragma unroll
                        for (int p = 0; p < NKE; ++p)
#pragma unroll
                            for (int e = 0; e < 8; ++e) o[p][e] = 0.0f;
#pragma unroll
                        for (int p = 0; p < NKE; ++p)
                            if (j0 + 128 * p < j1) {  // workgroup-uniform
                                float sp[4];
#pragma unroll
                                for (int u = 0; u < 4; ++u) {
                                    const int kv = j0 + 128 * p + jg * 4 + u;
                                    sp[u] = st[(kv < j1 ? kv : j1 - 1) - j0];
                                }
                                // keys past the chunk add p = 0 (o + 0 == o: o is never -0)
#pragma unroll
                                for (int u = 0; u < 4; ++u) {
                                    const float pj = j0 + 128 * p + jg * 4 + u < j1 ? sp[u] : 0.0f;
#pragma unroll
                                    for (int e = 0; e < 8; ++e) o[p][e] = o[p][e] + pj * (float)vf[p][u][e];
                                }
                            }
#pragma unroll
                        for (int p = 0; p < NKE; ++p)
                            if (j0 + 128 * p < j1)
#pragma unroll
                                for (int e = 0; e < 8; ++e) o[p][e] = red_8_16_32(o[p][e]);
                        if (lane < 8)
#pragma unroll
                            for (int p = 0; p < NKE; ++p)
                                if (j0 + 128 * p < j1)
#pragma unroll
                                    for (int e = 0; e < 8; ++e) sh.ored[w][p * 64 + lane * 8 + e] = o[p][e];
                        __syncthreads();
                PSTAMP(l * 32 + 13)
                        const int nsp = (j1 - j0 + 127) >> 7;  // sub-chunks of this task
                        const int64_t sb = (int64_t)bh * nsub + (j0 >> 7);
                        if (tid < 64 * nsp)
                            gput(xg + oP + sb * 64 + tid, tag,
                                 __float_as_uint(((sh.ored[0][tid] + sh.ored[1][tid]) + sh.ored[2][tid]) + sh.ored[3][tid]));
                        if (tid < nsp) {
                            const double s = ((sh.reddb[tid][0] + sh.reddb[tid][1]) + sh.reddb[tid][2]) + sh.reddb[tid][3];
                            gput(xg + oS + 3 * (sb + tid), tag,
                                 __float_as_uint(fmaxf(fmaxf(sh.redfb[tid][0], sh.redfb[tid][1]),
                                                       fmaxf(sh.redfb[tid][2], sh.redfb[tid][3]))));
                            gput(xg + oS + 3 * (sb + tid) + 1, tag, lo32(s));
                            gput(xg + oS + 3 * (sb + tid) + 2, tag, hi32(s));
                        }
                    }
                }
            }

            PSTAMP(l * 32 + 4)
            PSTAMP(l * 32 + 5)
            PSTAMP(l * 32 + 6)
            // ---- G1: the row's sub-chunks combined -> cross o -----------------
            // M = max m_c, o = (sum_c e^(m_c - M) o_c) / (sum_c e^(m_c - M) S_c),
            // both sums in one fixed order
            {
                PHASE_IDS
                const uint32_t tag = ptag(pos, L, l, 7);
                float *pp = (float *)scr;                        // [nsub][64] partial o
                const uint32_t *ps = (const uint32_t *)(pp + nsub * 64);  // [nsub][3] m, S lo, S hi
                const int no = nsub * 64;
                for (int t = wg; t < B * H; t += G) {
                    const int b = t / H, h = t - b * H;
                    __syncthreads();
                    const bool ok = gpoll(no + 3 * nsub, ptag(pos, L, l, 6),
                                          [=](int i) {
                                              return i < no ? xg + oP + (int64_t)t * no + i
                                                            : xg + oS + (int64_t)t * nsub * 3 + (i - no);
                                          },
                                          (uint32_t *)pp, abortw, a.err);
                    if (check(ok)) return;
                PSTAMP(l * 32 + 23)
                    if (tid < 64) {
                        // lane c < nsub: sub-chunk c's max, weight e^(m_c - M)
                        // and weighted sum (one expf a lane, wave reductions in
                        // a fixed order); the weights reach every lane through
                        // readlane; lane d then sums its dimension in chunk order
                        const int cc = lane < nsub ? lane : nsub - 1;
                        const float mcl = __uint_as_float(ps[3 * cc]);
                        const double scl = mk64(ps[3 * cc + 2], ps[3 * cc + 1]);
                        float v[NSUBM];
#pragma unroll
                        for (int c = 0; c < NSUBM; ++c) v[c] = pp[(c < nsub ? c : nsub - 1) * 64 + lane];
                        const float M = wave_max(lane < nsub ? mcl : -INFINITY);
                        const float wcl = lane < nsub ? expf(mcl - M) : 0.0f;
                        const double S = wave_sum(lane < nsub ? (double)wcl * scl : 0.0);
                        float ov = 0.0f;
#pragma unroll
                        for (int c = 0; c < NSUBM; ++c) {
                            const float wc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wcl), c));
                            ov = ov + v[c] * wc;  // (a padded sub-chunk: weight 0)
                        }
                        sh.ored[0][tid] = (float)((double)ov / S);
                    }
                    __syncthreads();
                    if (tid < 32)
                        gput(xg + oOC + b * (NS / 2) + h * 32 + tid, tag, pack2(sh.ored[0][2 * tid], sh.ored[0][2 * tid + 1]));
                }
            }

            PSTAMP(l * 32 + 7)
            // ---- G2: Wco rows + residual -> x'' -------------------------
            {
                PHASE_IDS
                const uint32_t tag = ptag(pos, L, l, 8);
                PSet<NS, BT, KC, 1, KS_N, Q5, false> S;
                const bool act = rn0 < rn1;
                S.load(lmat<Q5>(P.wco, P.wco5, NS * NS), P.bco, NS, rn0, rn1, slot, l16);
                PREFETCH_ISSUED
                __syncthreads();
                const bool ok = gpoll<PUX>(B * NS / 2, ptag(pos, L, l, 7), ptr_u64(xg + oOC), (uint32_t *)xs, abortw, a.err,
                                           [&] { S.pre(l16); });
                if (check(ok)) return;
            PSTAMP(l * 32 + 24)
                if (act)
                    S.template dot<BT>(xs, NS, B, rn0, rn1, slot, l16, kpbuf, [&](int row, int b, float v, float eb, bool valid) {
                        if (!valid) return;
                        const float x = (v + eb) + sh.xres[b][row - rn0];
                        sh.xres[b][row - rn0] = x;
                        gput(xg + oX3 + b * NS + row, tag, __float_as_uint(x));
                    });
            }

            PSTAMP(l * 32 + 8)
            // ---- H: LN2(x'') + W0 rows + GELU -> hidden ---------------------
            {
                PHASE_IDS
                const uint32_t tag = ptag(pos, L, l, 9);
                PSet<NS, BT, KC, 2, KS_H, Q5> S;
                const bool act = rh0 < rh1;
                S.load(lmat<Q5>(P.w0, P.w05, 4 * NS * NS), P.b0, NS, rh0, rh1, slot, l16);
                LnP<NS> lp;
                Ln1P<NS> l1;
                if constexpr (BT == 1) ln1_params<NS>(P.ln2_w, P.ln2_b, l1, tid);
                else ln_params_early<NS>(P.ln2_w, P.ln2_b, lp, lane);
                PREFETCH_ISSUED
                __syncthreads();
                if constexpr (BT == 1) {
                    if (!poll_ln1<NS>(xg + oX3, ptag(pos, L, l, 8), l1, xf, xs, abortw, a.err, sh.redd, sh.redd2, &sh.abort_,
                                      [&] { S.pre(l16); }))
                        return;
                } else {
                    const bool ok = gpoll<PUX>(B * NS, ptag(pos, L, l, 8), ptr_u64(xg + oX3), (uint32_t *)xf, abortw, a.err,
                                               [&] { S.pre(l16); });
                    if (check(ok)) return;
                    ln_rows<NS>(xf, lp, xs, B, w, lane);
                }
                PSTAMP(l * 32 + 25)
                __syncthreads();
                PSTAMP(l * 32 + 28)
                if (act)
                    S.template dot<BT>(xs, NS, B, rh0, rh1, slot, l16, kpbuf, [&](int row, int b, float v, float eb, bool valid) {
                        const float vn = from_next_row(v), ebn = from_next_row(eb);
                        if (!valid || (q & 1)) return;
                        const uint16_t h0 = f2h_bits(v + eb), h1 = f2h_bits(vn + ebn);
                        // (n <= 512: computed where the context's scan allows — no
                        // dependent table gather between the dot and the hand-off: base
                        // decode 15.27 -> 15.10 ms; at n = 768 the tanhf cost more than
                        // the gather, small 34.6 -> 34.8 ms: the table there)
                        uint16_t g0, g1;
                        if constexpr (NS <= 512) {
                            g0 = gelu_bits(a.gelu_tab, h2f_bits(h0), a.gelu_min);
                            g1 = gelu_bits(a.gelu_tab, h2f_bits(h1), a.gelu_min);
                        } else {
                            g0 = a.gelu_tab[h0];
                            g1 = a.gelu_tab[h1];
                        }
                        gput(xg + oH + b * (2 * NS) + row / 2, tag, (uint32_t)g0 | ((uint32_t)g1 << 16));
                    });
            }

            PSTAMP(l * 32 + 9)
            // ---- I: W1 rows + residual -> next layer's x --------------------
            {
                PHASE_IDS
                const uint32_t tag = ptag(pos, L, l, 10);
                PSet<NS, BT, 4 * KC, 1, KS_I, Q5, false> S;
                const bool act = rn0 < rn1;
                S.load(lmat<Q5>(P.w1, P.w15, 4 * NS * NS), P.b1, 4 * NS, rn0, rn1, slot, l16);
                PREFETCH_ISSUED
                __syncthreads();
                const bool ok = gpoll<PUH>(B * 2 * NS, ptag(pos, L, l, 9), ptr_u64(xg + oH), (uint32_t *)xs, abortw, a.err,
                                           [&] { S.pre(l16); });
                if (check(ok)) return;
                PSTAMP(l * 32 + 26)
                if (act)
                    S.template dot<BT>(xs, 4 * NS, B, rn0, rn1, slot, l16, kpbuf, [&](int row, int b, float v, float eb, bool valid) {
                        if (!valid) return;
                        const float x = (v + eb) + sh.xres[b][row - rn0];
                        sh.xres[b][row - rn0] = x;
                        gput(xg + oX1 + b * NS + row, tag, __float_as_uint(x));
                    });
            }
            PSTAMP(l * 32 + 10)
        }

        // ---- logits: LN_final + vocabulary rows + per-WG argmax -------------
        // rows [rv0, rs0) are resident in LDS (loaded once per launch), the
        // rest [rs0, rv1) stream through two register sets issued before the poll
        // (logits_out: this step's [B][V] slab; lg_stride > 0 keeps every
        // position's, for the all-step parity tests)
        float *const lgo = a.logits_out ? a.logits_out + (int64_t)pos * a.lg_stride : nullptr;
        if constexpr (LMF) {
            // MFMA logits: wave w takes the 16-row tiles w, w + 4, ... of the
            // resident rows (B fragments from the swizzled LDS copy), then of
            // the streamed rows (B fragments loaded straight into registers,
            // the next tile's loads in flight during this tile's MFMAs).
            // Lane l: A = hidden row l & 15 (zero for rows >= B), B = vocab
            // row n0 + (l & 15), k = 32 kk + 8 (l >> 4) + 0..7; result D: vocab
            // row n0 + (l & 15), hidden rows 4 (l >> 4) + r.  Each logit is one
            // MFMA chain over k in order: independent of the other rows.
            PHASE_IDS
            constexpr int NK = NS / 32;
            LnP<NS> lp;
            Ln1P<NS> l1;
            if constexpr (BT == 1) ln1_params<NS>(a.dln_w, a.dln_b, l1, tid);
            else ln_params_early<NS>(a.dln_w, a.dln_b, lp, lane);
            PREFETCH_ISSUED
            __syncthreads();
            if constexpr (BT == 1) {
                if (!poll_ln1<NS>(xg + oX1, ptag(pos, L, L - 1, 10), l1, xf, xs, abortw, a.err, sh.redd, sh.redd2, &sh.abort_))
                    return;
            } else {
                const bool ok = gpoll<PUX>(B * NS, ptag(pos, L, L - 1, 10), ptr_u64(xg + oX1), (uint32_t *)xf, abortw, a.err);
                if (check(ok)) return;
            }
                PSTAMP(L * 32 + 16)
            const int lr = lane & 15, lh = lane >> 4;
            // resident tiles cover [rv0, rs0) — the last one partial, its
            // missing rows read clamped and masked — and the streamed tiles
            // start at rs0: at base 139 resident + 64 streamed rows, one
            // streamed tile a wave (round 5: 128 + 75, the fifth tile behind
            // wave 0's resident ones)
            const int rres = rs0, nres_t = rs0 - rv0;  // resident rows end, count
            const int nst = (rv1 - rres + 15) >> 4;    // streamed tiles
            const f16 *te = (const f16 *)a.te;
            const half8 z8 = {};
            auto sload = [&](half8 (&f)[NK], int t) {  // streamed tile t's B fragments
                int row = rres + 16 * t + lr;
                row = row < rv1 ? row : rv1 - 1;
                const f16 *wr = te + (int64_t)row * NS + 8 * lh;
#pragma unroll
                for (int kk = 0; kk < NK; ++kk) f[kk] = t < nst ? sld((const half8 *)(wr + 32 * kk)) : z8;
            };
            half8 bA[NK], bB[NK];
            sload(bA, w);  // (requested after the poll: the resident tiles cover their latency)
            if constexpr (BT > 1) sload(bB, w + 4);  // (one row: behind the resident tiles, measured faster)
            PREFETCH_ISSUED
            if constexpr (BT > 1) ln_rows<NS>(xf, lp, xs, B, w, lane);
            __syncthreads();
            PSTAMP(L * 32 + 1)
            half8 af[NK];
#pragma unroll
            for (int kk = 0; kk < NK; ++kk) {
                const half8 v = *(const half8 *)(xs + (lr < B ? lr : 0) * NS + 32 * kk + 8 * lh);
                af[kk] = lr < B ? v : z8;
            }
            unsigned long long best[4] = {0ull, 0ull, 0ull, 0ull};
            auto epi = [&](const floatx4 &d, int n0, int nend) {
                const int n = n0 + lr;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = 4 * lh + r;
                    const bool valid = m < B && n < nend;
                    if (lgo && valid) lgo[(int64_t)m * a.V + n] = d[r];
                    const unsigned long long k =
                        ((unsigned long long)ord_f32(d[r]) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)n);
                    if (valid && n != a.suppress_id) best[r] = k > best[r] ? k : best[r];
                }
            };
            for (int t = w; 16 * t < nres_t; t += 4) {  // resident tiles
                const int j = 16 * t + lr < nres_t ? 16 * t + lr : nres_t - 1;  // row within the resident copy
                const f16 *wr = vres + j * NS;
                // every B fragment of the tile requested before the first
                // MFMA (one LDS latency a tile, not one per MFMA step: the
                // scheduler otherwise keeps two reads in flight)
                half8 bv[NK];
#pragma unroll
                for (int kk = 0; kk < NK; ++kk) bv[kk] = *(const half8 *)(wr + (((4 * kk + lh) ^ (j & 15)) * 8));
#pragma unroll
                for (int kk = 0; kk < NK; ++kk) asm volatile("" : "+v"(bv[kk]));  // (one wait for all of them)
                floatx4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kk = 0; kk < NK; ++kk) d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[kk], bv[kk], d, 0, 0, 0);
                epi(d, rv0 + 16 * t, rres);
            }
            PSTAMP(L * 32 + 2)
            if constexpr (BT == 1) sload(bB, w + 4);
            PREFETCH_ISSUED
            for (int t = w; t < nst; t += 8) {  // streamed tiles, two register sets in flight
                floatx4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kk = 0; kk < NK; ++kk) d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[kk], bA[kk], d, 0, 0, 0);
                epi(d, rres + 16 * t, rv1);
                if (t + 4 >= nst) break;
                sload(bA, t + 8);
                PREFETCH_ISSUED
                d = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kk = 0; kk < NK; ++kk) d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[kk], bB[kk], d, 0, 0, 0);
                epi(d, rres + 16 * (t + 4), rv1);
                sload(bB, t + 12);
                PREFETCH_ISSUED
            }
            PSTAMP(L * 32 + 3)
            // the 16 lanes of a row group hold rows 4 (l >> 4) + r: reduce them
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                unsigned long long k = best[r];
                k = kstep<8>(k);
                k = kstep<4>(k);
                k = kstep<2>(k);
                k = kstep<1>(k);
                if (lr == 0 && 4 * lh + r < PMAXB) sh.best[w][4 * lh + r] = k;
            }
            __syncthreads();
            if (tid < B) {
                unsigned long long k = sh.best[0][tid];
                for (int i = 1; i < 4; ++i) k = sh.best[i][tid] > k ? sh.best[i][tid] : k;
                const uint32_t tg = atag(pos, L);
                gput(xg + oA + ((int64_t)tid * G + wg) * 2, tg, (uint32_t)(k >> 32));
                gput(xg + oA + ((int64_t)tid * G + wg) * 2 + 1, tg, (uint32_t)k);
            }
        } else if constexpr (LMF2) {
            PHASE_IDS
            constexpr int KQ = NS / 4, NKW = KQ / 32, TG = 8;  // k per wave, MFMA steps per wave, tiles per LDS group
            LnP<NS> lp;
            ln_params_early<NS>(a.dln_w, a.dln_b, lp, lane);
            PREFETCH_ISSUED
            __syncthreads();
            {
                const bool ok = gpoll<PUX>(B * NS, ptag(pos, L, L - 1, 10), ptr_u64(xg + oX1), (uint32_t *)xf, abortw, a.err);
                if (check(ok)) return;
            }
                PSTAMP(L * 32 + 16)
            const int lr = lane & 15, lh = lane >> 4, k0 = w * KQ;
            const int rres = rv0 + ((rs0 - rv0) & ~15);
            const int nres_t = (rres - rv0) >> 4, ntile = nres_t + ((rv1 - rres + 15) >> 4);
            const f16 *te = (const f16 *)a.te;
            const half8 z8 = {};
            auto bload = [&](half8 (&f)[NKW], int t) {  // streamed tile t (t >= nres_t) B fragments of this wave's K
                int row = rv0 + 16 * t + lr;
                row = row < rv1 ? row : rv1 - 1;
                const f16 *wr = te + (int64_t)row * NS + k0 + 8 * lh;
#pragma unroll
                for (int i = 0; i < NKW; ++i) f[i] = t < ntile ? sld((const half8 *)(wr + 32 * i)) : z8;
            };
            half8 bA[NKW], bB[NKW];
            bload(bA, nres_t);
            bload(bB, nres_t + 1);
            PREFETCH_ISSUED
            ln_rows<NS>(xf, lp, xs, B, w, lane);
            __syncthreads();
            PSTAMP(L * 32 + 1)
            half8 af[NKW];
#pragma unroll
            for (int i = 0; i < NKW; ++i) {
                const half8 v = *(const half8 *)(xs + (lr < B ? lr : 0) * NS + k0 + 32 * i + 8 * lh);
                af[i] = lr < B ? v : z8;
            }
            float *kp = (float *)scr;  // [TG][4][16][8]
            unsigned long long best = 0ull;  // this thread's decoder row m = tid & 7
            for (int g0 = 0; g0 < ntile; g0 += TG) {
                for (int t = g0; t < g0 + TG && t < ntile; ++t) {  // workgroup-uniform
                    floatx4 d = {0.f, 0.f, 0.f, 0.f};
                    if (t < nres_t) {
                        const int j = 16 * t + lr;
                        const f16 *wr = vres + j * NS;
                        half8 bv[NKW];  // (all requested before the first MFMA, as in the LMF tiles)
#pragma unroll
                        for (int i = 0; i < NKW; ++i) bv[i] = *(const half8 *)(wr + ((((k0 >> 3) + 4 * i + lh) ^ (j & 15)) * 8));
#pragma unroll
                        for (int i = 0; i < NKW; ++i) asm volatile("" : "+v"(bv[i]));
#pragma unroll
                        for (int i = 0; i < NKW; ++i) d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bv[i], d, 0, 0, 0);
                    } else if (((t - nres_t) & 1) == 0) {
#pragma unroll
                        for (int i = 0; i < NKW; ++i) d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bA[i], d, 0, 0, 0);
                        bload(bA, t + 2);
                        PREFETCH_ISSUED
                    } else {
#pragma unroll
                        for (int i = 0; i < NKW; ++i) d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bB[i], d, 0, 0, 0);
                        bload(bB, t + 2);
                        PREFETCH_ISSUED
                    }
                    if (lh < 2)
#pragma unroll
                        for (int r = 0; r < 4; ++r) kp[(((t - g0) * 4 + w) * 16 + lr) * 8 + 4 * lh + r] = d[r];
                }
                __syncthreads();
                for (int idx = tid; idx < TG * 128; idx += PT) {  // (tile, row, m) with m = tid & 7
                    const int tg = idx >> 7, rr = (idx >> 3) & 15, m = idx & 7, t = g0 + tg;
                    const int n = rv0 + 16 * t + rr;
                    if (t >= ntile || m >= B || n >= rv1) continue;
                    const float v = ((kp[((tg * 4 + 0) * 16 + rr) * 8 + m] + kp[((tg * 4 + 1) * 16 + rr) * 8 + m]) +
                                     kp[((tg * 4 + 2) * 16 + rr) * 8 + m]) +
                                    kp[((tg * 4 + 3) * 16 + rr) * 8 + m];
                    if (lgo) lgo[(int64_t)m * a.V + n] = v;
                    if (n == a.suppress_id) continue;
                    const unsigned long long k =
                        ((unsigned long long)ord_f32(v) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)n);
                    best = k > best ? k : best;
                }
                __syncthreads();  // kp reused by the next group
            }
            PSTAMP(L * 32 + 2)
            PSTAMP(L * 32 + 3)
            // lanes with equal lane & 7 hold the same decoder row: reduce them
            best = kstep<8>(best);
            best = kstep<16>(best);
            best = kstep<32>(best);
            if (lane < PMAXB) sh.best[w][lane] = best;
            __syncthreads();
            if (tid < B) {
                unsigned long long k = sh.best[0][tid];
                for (int i = 1; i < 4; ++i) k = sh.best[i][tid] > k ? sh.best[i][tid] : k;
                const uint32_t tg = atag(pos, L);
                gput(xg + oA + ((int64_t)tid * G + wg) * 2, tg, (uint32_t)(k >> 32));
                gput(xg + oA + ((int64_t)tid * G + wg) * 2 + 1, tg, (uint32_t)k);
            }
        } else {
                PHASE_IDS
            WSet<KC, NPL> S0, S1;
            constexpr int RS = 16 * NPL;  // rows per register set
            LnP<NS> lp;
            Ln1P<NS> l1;
            if constexpr (BT == 1) ln1_params<NS>(a.dln_w, a.dln_b, l1, tid);
            else ln_params_early<NS>(a.dln_w, a.dln_b, lp, lane);
            PREFETCH_ISSUED
            __syncthreads();
            if constexpr (BT == 1) {
                if (!poll_ln1<NS>(xg + oX1, ptag(pos, L, L - 1, 10), l1, xf, xs, abortw, a.err, sh.redd, sh.redd2, &sh.abort_))
                    return;
            } else {
                const bool ok = gpoll<PUX>(B * NS, ptag(pos, L, L - 1, 10), ptr_u64(xg + oX1), (uint32_t *)xf, abortw, a.err);
                if (check(ok)) return;
            }
                PSTAMP(L * 32 + 16)
            // the streamed rows are requested after the poll, not in front of
            // it in the wave's load queue: the LDS-resident rows cover their
            // latency (logits 6.9 -> 5.8 us a step, profiles/r03/ab_r03c.txt)
            wset_load(S0, wmat(a.te), nullptr, NS, rs0, lreg2 ? rs0 : rv1, slot, l16);
            wset_load(S1, wmat(a.te), nullptr, NS, rs0 + RS, lreg2 ? rs0 : rv1, slot, l16);
            PREFETCH_ISSUED
            if constexpr (BT > 1) ln_rows<NS>(xf, lp, xs, B, w, lane);
            __syncthreads();
            PSTAMP(L * 32 + 1)
            unsigned long long best = 0ull;
            auto epi = [&](int row, int b, float v, float eb, bool valid) {
                if (lgo && valid) lgo[(int64_t)b * a.V + row] = v;
                if (!valid || row == a.suppress_id) return;
                const unsigned long long k =
                    ((unsigned long long)ord_f32(v) << 32) | (unsigned long long)(0xffffffffu - (uint32_t)row);
                best = k > best ? k : best;
            };
            // row groups interleaved per iteration; each xs chunk read once for
            // all (as wset_dot: more than 32 xs chunks in registers would spill)
            constexpr int RU = BT == 1 || BT * KC <= 32 ? 4 : 1;
            for (int rb = rv0; rb < rs0; rb += 16 * RU) {  // resident rows
                float acc[RU][BT];
#pragma unroll
                for (int u = 0; u < RU; ++u)
#pragma unroll
                    for (int b = 0; b < BT; ++b) acc[u][b] = 0.0f;
#pragma unroll
                for (int c = 0; c < KC; ++c) {
                    if constexpr (RU > 1) {
                        half8 xv[BT];
#pragma unroll
                        for (int b = 0; b < BT; ++b)
                            if (b < B) xv[b] = *(const half8 *)(xs + b * NS + c * 128 + l16 * 8);
#pragma unroll
                        for (int u = 0; u < RU; ++u) {
                            const int row = rb + 16 * u + slot;
                            const f16 *wr = vres + (row < rs0 ? row - rv0 : 0) * NS + l16 * 8;
                            const half8 wv = *(const half8 *)(wr + c * 128);
#pragma unroll
                            for (int b = 0; b < BT; ++b)
                                if (b < B) acc[u][b] = dot8(wv, xv[b], acc[u][b]);
                        }
                    } else {
                        const int row = rb + slot;
                        const half8 wv = *(const half8 *)(vres + (row < rs0 ? row - rv0 : 0) * NS + l16 * 8 + c * 128);
#pragma unroll
                        for (int b = 0; b < BT; ++b)
                            if (b < B) acc[0][b] = dot8(wv, *(const half8 *)(xs + b * NS + c * 128 + l16 * 8), acc[0][b]);
                    }
                }
#pragma unroll
                for (int u = 0; u < RU; ++u) {
                    const int row = rb + 16 * u + slot;
                    float v = 0.0f;
#pragma unroll
                    for (int b = 0; b < BT; ++b)
                        if (b < B) {
                            const float t = red16_sum(acc[u][b]);
                            if (l16 == b) v = t;
                        }
                    epi(row, l16, v, 0.0f, row < rs0 && l16 < B);
                }
            }
            PSTAMP(L * 32 + 2)
            if (lreg2) {  // register-resident rows (LREG2): the same per-row dot chains
                if constexpr (LREG2) wset_dot<BT>(SR, xs, NS, B, rs0, rv1, slot, l16, epi);
            } else if (rs0 < rv1)
                for (int rb = rs0;;) {
                    wset_dot<BT>(S0, xs, NS, B, rb, rv1, slot, l16, epi);
                    wset_load(S0, wmat(a.te), nullptr, NS, rb + 2 * RS, rv1, slot, l16);
                    PREFETCH_ISSUED
                    if (rb + RS >= rv1) break;
                    wset_dot<BT>(S1, xs, NS, B, rb + RS, rv1, slot, l16, epi);
                    wset_load(S1, wmat(a.te), nullptr, NS, rb + 3 * RS, rv1, slot, l16);
                    PREFETCH_ISSUED
                    rb += 2 * RS;
                    if (rb >= rv1) break;
                }
            PSTAMP(L * 32 + 3)
            // lane l16 = b holds its quarter's best: reduce the 4 quarters, then the waves
            best = rows_max_u64(best);
            if (lane < PMAXB) sh.best[w][lane] = best;
            __syncthreads();
            if (tid < B) {
                unsigned long long k = sh.best[0][tid];
                for (int i = 1; i < 4; ++i) k = sh.best[i][tid] > k ? sh.best[i][tid] : k;
                const uint32_t tg = atag(pos, L);
                gput(xg + oA + ((int64_t)tid * G + wg) * 2, tg, (uint32_t)(k >> 32));
                gput(xg + oA + ((int64_t)tid * G + wg) * 2 + 1, tg, (uint32_t)k);
            }
        }
        PSTAMP(L * 32 + 0)
        if (a.ptrace && threadIdx.x == 0 && (wg == 0 || wg == G / 2))  // shader clock (s_memtime) at the same point
            a.ptrace[(((int64_t)step * (L + 1) + L) * 32 + 4) * 2 + (wg == 0 ? 0 : 1)] = __builtin_amdgcn_s_memtime();
    }
    // the last step's token: recorded by workgroup 0 and carried to the next launch
    if (wg != 0 || a.n_steps < 1) return;
    if (a.beam) {  // the beam kernels select the next tokens
        if (tid == 0) a.st->pos = pos;
        return;
    }
    __syncthreads();
    if (!argmax_gather(pos - 1)) return;
    if (tid < B) {
        if (pos >= a.feed_len && pos - a.feed_len < a.out_stride) a.tokens_out[tid * a.out_stride + (pos - a.feed_len)] = sh.tok[tid];
        a.cur_tok[tid] = sh.tok[tid];
    }
    if (tid == 0) a.st->pos = pos;
}

template <int NS, int BT>
size_t persist_lds(int B) {
    return (size_t)B * NS * 4 + (size_t)B * NS * 8 + scr_bytes(BT);
}
constexpr size_t LDS_CU = 160 * 1024;

template <int NS, int BT, bool BEAM, bool Q5>
hipError_t launch_nsb(hipStream_t s, const PersistArgs &a, int G) {
    // resident vocabulary rows as this instance's LDS holds them (the
    // context's count is sized for the one-row instance at B = 1, whose
    // scratch is smaller than a beam launch's at K = 1)
    static const size_t stat = [] {
        hipFuncAttributes fa;
        return hipFuncGetAttributes(&fa, (const void *)k_dec_persist<NS, BT, BEAM, Q5>) == hipSuccess
                   ? fa.sharedSizeBytes
                   : LDS_CU;
    }();
    const size_t base = persist_lds<NS, BT>(a.B), avail = LDS_CU - stat - 1024;
    if (base > avail) return hipErrorInvalidValue;
    PersistArgs b = a;
    const int maxr = (int)((avail - base) / (NS * 2));
    if (b.nres > maxr) b.nres = maxr;
    const size_t lds = base + (size_t)b.nres * NS * 2;
    hipError_t e = hipFuncSetAttribute((const void *)k_dec_persist<NS, BT, BEAM, Q5>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_dec_persist<NS, BT, BEAM, Q5>), dim3(G), dim3(PT), lds, s, b);
    return hipGetLastError();
}
#ifndef WMI_PERSIST_Q5_TU
// beam launches read the f16 copies (the same weights the q5_1 blocks
// dequantise to); the q5_1 instances live in wmi_persist_q5.hip
template <int NS>
hipError_t launch_ns(hipStream_t s, const PersistArgs &a, int G) {
    if (a.beam) return launch_nsb<NS, PMAXB, true, false>(s, a, G);
    if (a.q5) return launch_persist_q5(s, a, G);
    return a.B == 1 ? launch_nsb<NS, 1, false, false>(s, a, G) : launch_nsb<NS, PMAXB, false, false>(s, a, G);
}
#endif

template <int NS, int BT, bool BEAM, bool Q5>
int grid_nsb(int device, int B, int V, int *nres) {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void *)k_dec_persist<NS, BT, BEAM, Q5>) != hipSuccess) return 0;
    const size_t base = persist_lds<NS, BT>(B), avail = LDS_CU - fa.sharedSizeBytes - 1024;
    if (base > avail) return 0;
    // resident vocabulary rows: as many of a workgroup's rows as the LDS holds
    const int G0 = PX_GDESIGN, rpw = (V + G0 - 1) / G0;
    int nr = (int)((avail - base) / (NS * 2));
    *nres = nr < rpw ? nr : rpw;
    const size_t lds = base + (size_t)*nres * NS * 2;
    if (hipFuncSetAttribute((const void *)k_dec_persist<NS, BT, BEAM, Q5>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
        return 0;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_dec_persist<NS, BT, BEAM, Q5>, PT, lds) != hipSuccess ||
        per_cu < 1)
        return 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 0;
    // the grid must be co-resident: a device that cannot launch cooperatively
    // gives no such guarantee even at one workgroup per CU
    int coop = 0;
    if (hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, device) != hipSuccess || !coop) return 0;
    const int G = prop.multiProcessorCount < PX_GDESIGN ? prop.multiProcessorCount : PX_GDESIGN;
    if (per_cu * prop.multiProcessorCount < G) return 0;
    // row-partition limits of the register sets (see wset_dot users); the
    // split-K phases need the full grid's rows per workgroup
    if ((3 * NS + G - 1) / G > 31 || (4 * NS + G - 1) / G > 31 || (NS + G - 1) / G > RNMAX - 1) return 0;
    auto rows_g = [G](int N) { return (((N + G - 1) / G) + 1) & ~1; };
    if (rows_g(NS) > rows_full(NS) || rows_g(3 * NS) > rows_full(3 * NS) || rows_g(4 * NS) > rows_full(4 * NS)) return 0;
    return G;
}

// the fallback list: every non-positive f16 input whose f32 exp lies too
// close to an f16 rounding midpoint, with its table value (count in *n;
// entries beyond EXPFB are counted, not stored — the host then refuses)
__global__ void k_exp_fallbacks(const uint16_t *tab, int n_exp, uint32_t *list, uint32_t *n) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > 0x7c00) return;
    f16 hx;
    float hv;
    if (exp_f16_fast_ok(h2f_bits((uint16_t)(0x8000u | (uint32_t)j)), hx, hv)) return;
    const uint32_t k = atomicAdd(n, 1u);
    if (k < (uint32_t)EXPFB) list[k] = ((uint32_t)j << 16) | (j < n_exp ? tab[j] : 0u);
}

// exp_f16_fast (with the list) against the host-built ggml exp table over
// every non-positive f16 input
__global__ void k_persist_selftest(const uint16_t *tab, int n_exp, const uint32_t *fb, uint32_t *mismatch) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > 0x7c00) return;
    const float x = h2f_bits((uint16_t)(0x8000u | (uint32_t)j));
    const uint16_t got = f2h_bits(exp_f16_hash(x, fb, fb[EXPFB + 1]));
    const uint16_t want = j < n_exp ? tab[j] : (uint16_t)0;
    if (got != want) atomicAdd(mismatch, 1u);
}

// every instance a context may launch at B rows must fit: grid and resident
// rows are the minimum over them
template <int NS>
int grid_ns(int device, int B, int V, int *nres) {
    int g = PX_GMAX, nr = 1 << 30, ni = 0;
    auto take = [&](int gi) {
        g = gi < g ? gi : g;
        nr = ni < nr ? ni : nr;
    };
    if (B == 1) {
        take(grid_nsb<NS, 1, false, false>(device, B, V, &ni));
    } else {
        take(grid_nsb<NS, PMAXB, false, false>(device, B, V, &ni));
        take(grid_nsb<NS, PMAXB, true, false>(device, B, V, &ni));
    }
    take(grid_persist_q5(device, NS, B, V, &ni));
    *nres = g > 0 ? nr : 0;
    return g;
}

}  // namespace

#ifndef WMI_PERSIST_Q5_TU
hipError_t launch_exp_fallbacks(hipStream_t s, const uint16_t *exp_tab, int n_exp, uint32_t *list, uint32_t *n) {
    hipLaunchKernelGGL(k_exp_fallbacks, dim3((0x7c01 + 255) / 256), dim3(256), 0, s, exp_tab, n_exp, list, n);
    return hipGetLastError();
}

hipError_t launch_persist_selftest(hipStream_t s, const uint16_t *exp_tab, int n_exp, const uint32_t *fb,
                                   uint32_t *mismatch) {
    hipLaunchKernelGGL(k_persist_selftest, dim3((0x7c01 + 255) / 256), dim3(256), 0, s, exp_tab, n_exp, fb, mismatch);
    return hipGetLastError();
}


int persist_grid(int device, int n, int B, int T, int V, int *nres) {
    *nres = 0;
    if (B < 1 || B > PMAXB || T < 1 || T > 2048) return 0;
    switch (n) {
        case 128: return grid_ns<128>(device, B, V, nres);
        case 384: return grid_ns<384>(device, B, V, nres);
        case 512: return grid_ns<512>(device, B, V, nres);
        case 768: return grid_ns<768>(device, B, V, nres);
        case 1024: return grid_ns<1024>(device, B, V, nres);
        case 1280: return grid_ns<1280>(device, B, V, nres);
        default: return 0;
    }
}

int persist_split_grid(int n, int G) {
    // the multi-row instances (MFMA GEMVs: no split-K factors tied to the
    // design grid) at half the grid: every phase's rows per workgroup within
    // the register sets' limits (grid_nsb)
    const int Gh = G / 2;
    if (Gh < 32 || (3 * n + Gh - 1) / Gh > 31 || (4 * n + Gh - 1) / Gh > 31 || (n + Gh - 1) / Gh > RNMAX - 1) return 0;
    return Gh;
}

hipError_t launch_dec_persist(hipStream_t s, const PersistArgs &a, int G) {
    if (G < 1 || G > PX_GMAX || a.B < 1 || a.B > PMAXB || a.T > 2048 || a.nch < 1 || a.nch > 64 ||
        a.cl > 128 * NKP || (int64_t)a.nch * a.cl < a.T || (int64_t)a.B * (a.n / 64) * a.nch > PX_TASKS ||
        a.tctx > 512 || a.cl % 128 || (a.beam && a.n_steps != 1) || (a.kv_src && a.kv_src_stride < a.tctx) ||
        (!a.beam && a.B == 1 && a.cl > 256) ||  // (the one-row instance: two sub-chunks per task)
        (a.xshare && (!a.beam || a.n <= 768 || a.cl != 128)))
        return hipErrorInvalidValue;
    switch (a.n) {
        case 128: return launch_ns<128>(s, a, G);
        case 384: return launch_ns<384>(s, a, G);
        case 512: return launch_ns<512>(s, a, G);
        case 768: return launch_ns<768>(s, a, G);
        case 1024: return launch_ns<1024>(s, a, G);
        case 1280: return launch_ns<1280>(s, a, G);
        default: return hipErrorInvalidValue;
    }
}

#else
hipError_t launch_persist_q5(hipStream_t s, const PersistArgs &a, int G) {
#define WMI_Q5_LAUNCH(NS) \
    case NS: \
        return a.B == 1 ? launch_nsb<NS, 1, false, true>(s, a, G) : launch_nsb<NS, PMAXB, false, true>(s, a, G);
    switch (a.n) {
        WMI_Q5_LAUNCH(128)
        WMI_Q5_LAUNCH(384)
        WMI_Q5_LAUNCH(512)
        WMI_Q5_LAUNCH(768)
        WMI_Q5_LAUNCH(1024)
        WMI_Q5_LAUNCH(1280)
        default: return hipErrorInvalidValue;
    }
#undef WMI_Q5_LAUNCH
}

int grid_persist_q5(int device, int n, int B, int V, int *nres) {
#define WMI_Q5_GRID(NS) \
    case NS: \
        return B == 1 ? grid_nsb<NS, 1, false, true>(device, B, V, nres) \
                      : grid_nsb<NS, PMAXB, false, true>(device, B, V, nres);
    switch (n) {
        WMI_Q5_GRID(128)
        WMI_Q5_GRID(384)
        WMI_Q5_GRID(512)
        WMI_Q5_GRID(768)
        WMI_Q5_GRID(1024)
        WMI_Q5_GRID(1280)
        default: return 0;
    }
#undef WMI_Q5_GRID
}
#endif

}  // namespace wmi

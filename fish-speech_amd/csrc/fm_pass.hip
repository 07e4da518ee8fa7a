// fm_pass.hip -- the persistent batch-1 decode pass: one launch per fast-model pass.
//
// A batch-1 fast pass (forward_generate_fast, llama.py:798-827, 838-843, 947-975) is 4 layers x
// (QKV, attention, Wo, W1||W3, W2) + the codebook head: 17 weight streams of 21-100 MB that the
// launch-per-GEMV path runs as 21 launches, each paying ~3 us of fill, drain and boundary.  Here
// one workgroup per CU runs the whole pass, on the LDS-DMA engine of MI355X_MICROARCH.md's price
// list (rows ldsdma-fill, prefetch-credit, engine-vs-launches):
//
//  * every op is split over the workgroups by OUTPUT ROWS (pairs of outputs; W1||W3 as (w1_j,
//    w3_j) row pairs), whole K per row, so no split-K combine exists; a workgroup's share is one
//    contiguous run of a row-major weight copy, cut into fills of 16 fragments (1 KiB = 512 k of
//    one row each; a fill never spans two ops);
//  * ONE LOADER wave streams the workgroup's fills, op after op, into a ring of 64 KiB of LDS
//    slots (8 x 8 KiB by default) by non-temporal LDS-DMA (global_load_lds_dwordx4), keeping two fills in flight and
//    publishing each behind a counted vmcnt.  It waits only for a FREE slot, never for a hand-off,
//    so the weight stream runs on through every seam until the ring is full;
//  * NC CONSUMER waves take the fills round-robin: dot products (v_dot2c_f32_bf16) of the slot's
//    fragments with the op's input row in LDS, row partials flushed to LDS, the slot freed;
//  * PASS_NWM EXCHANGE waves, once the consumers of an op have all arrived: reduce the row
//    partials (fixed order), run the op's epilogue (bias, residual finalise, SwiGLU, fp32 logits),
//    publish the workgroup's outputs as 8-byte {tag, bf16 pair} granules (write-through agent
//    stores: the data is the flag), sweep the whole vector back from every workgroup into LDS, and
//    build the next op's input row there (RMSNorm, or every head's attention from the gathered
//    q|k|v and the cached K/V rows they staged while the QKV weights streamed);
//  * the roles meet on LDS words only (FULL / FREE per slot, a consumer-arrival counter, the
//    input-ready op count, an exchange-wave counter): no s_barrier after the start, so no wave
//    ever waits for another role's global loads.
// Tags: (generation << 8) + op + 1; the generation word is read at the start and bumped by the
// last workgroup to finish, so granules of an earlier launch never match (no memset per launch).
// Every wait is bounded (pass_spin): a timed-out wait sets err, which the host turns into an error.
#include <type_traits>

#include "fm_attn_dev.h"
#include "fm_kernels.h"
#include "fm_runtime.h"

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef unsigned long long u64;

namespace {

// f(integral_constant<0>) ... f(integral_constant<N - 1>) in order, unrolled at compile time (register
// arrays indexed by the constant stay in VGPRs; #pragma unroll gives up on large bodies)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

enum { OP_QKV = 0, OP_WO = 1, OP_W13 = 2, OP_W2 = 3, OP_HEAD = 4 };
constexpr int PS_FR = 512;     // bf16 elements per fragment: 64 lanes x 8
constexpr int PS_NJ_MAX = 20;  // a vector of at most 256 x 20 pairs (S2-Pro: 4864)
constexpr int PS_NJN = 8;      // pairs per exchange thread of a normalised (dim-wide) row: dim <= 4096

struct Geom {
    const bf16_t* w;  // the workgroup's first weight row
    int K, fpr;       // K and fragments per row
    int o0, nout;     // the workgroup's outputs [o0, o0 + nout) (nout even)
    int rpo;          // weight rows per output (W1||W3: 2)
    int nfr;          // fragments of the workgroup's share
    int kind, layer;
    int s0;           // the op's first fill (sequence number over the whole pass)
};
// The pass's shape as plain scalars, copied out of the kernel argument once: selecting among
// fields of the by-value argument per op makes the compiler copy it to scratch and index it there.
struct Dims {
    const bf16_t *wbase, *head;
    size_t w_layer, off_wo, off_w13, off_w2;
    int L, dim, nq, nqkv, inter, nhead, nwg;
};
__device__ __forceinline__ Dims dims_of(const PassArgs& a) {
    return Dims{a.wbase, a.head, a.w_layer, a.off_wo, a.off_w13, a.off_w2, a.nlayer,
                a.dim,   a.nq,   a.nqkv,    a.inter,  a.nhead,   a.nwg};
}

__device__ __forceinline__ Geom geom(const Dims& d, int o, int wg) {
    Geom g;
    g.layer = o >> 2;
    g.kind = o >= 4 * d.L ? OP_HEAD : (o & 3);
    const bf16_t* lw = d.wbase + (size_t)(g.layer < d.L ? g.layer : d.L - 1) * d.w_layer;
    const int k = g.kind;
    const int N = k == OP_QKV ? d.nqkv : (k == OP_W13 ? d.inter : (k == OP_HEAD ? d.nhead : d.dim));
    g.K = k == OP_WO ? d.nq : (k == OP_W2 ? d.inter : d.dim);
    const bf16_t* W =
        k == OP_HEAD ? d.head : lw + (k == OP_WO ? d.off_wo : (k == OP_W13 ? d.off_w13 : (k == OP_W2 ? d.off_w2 : 0)));
    g.rpo = k == OP_W13 ? 2 : 1;
    const int P = N >> 1;
    const int p0 = P * wg / d.nwg, p1 = P * (wg + 1) / d.nwg;  // P * nwg < 2^31 (host-checked)
    g.o0 = 2 * p0;
    g.nout = 2 * (p1 - p0);
    g.fpr = g.K / PS_FR;
    g.nfr = g.nout * g.rpo * g.fpr;
    g.w = W + (size_t)g.o0 * g.rpo * g.K;
    g.s0 = 0;
    return g;
}

// The per-op geometry as built once per launch into LDS (opt[o][12] ints) by the exchange waves;
// every role reads it with ds_read_b128 + readfirstlane (an LDS wait never waits for a DMA).
__device__ __forceinline__ void opt_put(int* opt, int o, const Geom& g) {
    const uint64_t w = (uint64_t)(uintptr_t)g.w;
    int4* e = reinterpret_cast<int4*>(opt + 12 * o);
    e[0] = make_int4((int)(uint32_t)w, (int)(uint32_t)(w >> 32), g.nfr, g.fpr);
    e[1] = make_int4(g.o0, g.nout, g.kind, g.layer);
    e[2] = make_int4(g.s0, 0, 0, 0);
}
__device__ __forceinline__ Geom opt_get(const int* opt, int o) {
    const int4* e = reinterpret_cast<const int4*>(opt + 12 * o);
    const int4 e0 = e[0], e1 = e[1], e2 = e[2];
    Geom g;
    const uint32_t lo = __builtin_amdgcn_readfirstlane(e0.x), hi = __builtin_amdgcn_readfirstlane(e0.y);
    g.w = reinterpret_cast<const bf16_t*>((uintptr_t)(((uint64_t)hi << 32) | lo));
    g.nfr = __builtin_amdgcn_readfirstlane(e0.z);
    g.fpr = __builtin_amdgcn_readfirstlane(e0.w);
    g.o0 = __builtin_amdgcn_readfirstlane(e1.x);
    g.nout = __builtin_amdgcn_readfirstlane(e1.y);
    g.kind = __builtin_amdgcn_readfirstlane(e1.z);
    g.layer = __builtin_amdgcn_readfirstlane(e1.w);
    g.s0 = __builtin_amdgcn_readfirstlane(e2.x);
    g.rpo = g.kind == OP_W13 ? 2 : 1;
    g.K = g.fpr * PS_FR;
    return g;
}

// acc += w . x over 8 bf16 pairs (v_dot2c_f32_bf16).  The pairs are taken by shufflevector from
// one 8-element view: __builtin_bit_cast of a u32x4 ELEMENT to bf16x2 miscompiles (ROCm 7.2 hipcc
// loads element 0 once and reuses it for all four).
__device__ __forceinline__ float dot8(u32x4_t w, u32x4_t x, float acc) {
    const bf16x8_t wb = __builtin_bit_cast(bf16x8_t, w), xb = __builtin_bit_cast(bf16x8_t, x);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(wb, wb, 0, 1), __builtin_shufflevector(xb, xb, 0, 1),
                                          acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(wb, wb, 2, 3), __builtin_shufflevector(xb, xb, 2, 3),
                                          acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(wb, wb, 4, 5), __builtin_shufflevector(xb, xb, 4, 5),
                                          acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(wb, wb, 6, 7), __builtin_shufflevector(xb, xb, 6, 7),
                                          acc, false);
    return acc;
}

__device__ __forceinline__ float lo_f(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_f(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }
__device__ __forceinline__ unsigned tag_of(unsigned gen, int o) { return (gen << 8) + (unsigned)o + 1u; }

// hand-off words through GLOBAL pointers: the write-through forms of cdna_hip_programming.md §6
// Guideline 16 are measured for global_ / buffer_ sc1 accesses, never flat_
typedef __attribute__((address_space(1))) u64 g_u64;
typedef __attribute__((address_space(1))) unsigned g_u32;
typedef __attribute__((address_space(1))) int g_i32;
// LDS words shared between the roles: volatile LDS accesses (ds_read / ds_write, never cached)
typedef __attribute__((address_space(3))) volatile unsigned lds_vu32;

// the same, default cache policy: a prefetch whose bytes land in a junk LDS slot and stay in L2
// (MALL) for the real (nt) fill that follows
__device__ __forceinline__ void glds16_pf(const void* gsrc, uint32_t lds_base) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_base)
        : "memory");
}

// one 1 KiB fragment by LDS-DMA: lane l's 16 bytes at gsrc -> LDS lds_base + 16 l, non-temporal
// (nt-weights row: each weight byte is read once a pass).  M0 is saved and restored in the same
// statement (compiler-reserved); the DMA is invisible to hipcc's waitcnt bookkeeping, so every
// wait for it is an explicit s_waitcnt vmcnt (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_base) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_base)
        : "memory");
}

// s_sleep with a run-time argument (its operand is an immediate): 64 x n cycles, n in 1 .. 32
__device__ __forceinline__ void sleep_n(int n) {
    if (n <= 1) __builtin_amdgcn_s_sleep(1);
    else if (n <= 2) __builtin_amdgcn_s_sleep(2);
    else if (n <= 4) __builtin_amdgcn_s_sleep(4);
    else if (n <= 8) __builtin_amdgcn_s_sleep(8);
    else if (n <= 16) __builtin_amdgcn_s_sleep(16);
    else __builtin_amdgcn_s_sleep(32);
}

// bounded spin on an LDS word until (word - target) >= 0 as signed (monotonic counters)
__device__ __forceinline__ bool lds_wait_ge(const lds_vu32* w, unsigned target, unsigned limit, int* err) {
    for (unsigned spin = 0;; ++spin) {
        if ((int)(*w - target) >= 0) {
            asm volatile("" ::: "memory");  // no LDS access below is moved above the flag read
            return true;
        }
        if (spin > limit) {
            __hip_atomic_store((g_i32*)err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// Sweep the P granules of one op's vector into dst (bf16 pairs as u32): comm thread t owns pairs
// t, t + 256, ...; every round re-loads all NJ of them (one round trip), keeps those whose tag
// matches; bounded.
template <int NJ>
__device__ __forceinline__ void sweep_nj(const u64* g, int P, unsigned tag, uint32_t* dst, int t, int* err,
                                         unsigned limit, int nap) {
    asm volatile("" : "+v"(t));  // keep the address arithmetic here (not hoisted out of the caller's loop)
    uint32_t pend = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
        if (t + 256 * j < P) pend |= 1u << j;
    for (unsigned spin = 0;; ++spin) {
        u64 v[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {  // only the granules still missing (a poll costs the weight stream)
            v[j] = 0;
            if ((pend >> j) & 1u)
                v[j] = __hip_atomic_load((g_u64*)(g + t + 256 * j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            if ((pend >> j) & 1u) {
                if ((unsigned)(v[j] >> 32) == tag) {
                    dst[t + 256 * j] = (uint32_t)v[j];
                    pend &= ~(1u << j);
                }
            }
        }
        if (!__any(pend != 0u)) break;
        if (spin > limit) {
            __hip_atomic_store((g_i32*)err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        sleep_n(nap);
    }
}
__device__ __forceinline__ void sweep(const u64* g, int P, unsigned tag, uint32_t* dst, int t, int* err,
                                      unsigned limit, int nap) {
    const int nj = (P + 255) >> 8;
    if (nj <= 2) sweep_nj<2>(g, P, tag, dst, t, err, limit, nap);
    else if (nj <= 4) sweep_nj<4>(g, P, tag, dst, t, err, limit, nap);
    else if (nj <= 6) sweep_nj<6>(g, P, tag, dst, t, err, limit, nap);
    else if (nj <= 8) sweep_nj<8>(g, P, tag, dst, t, err, limit, nap);
    else if (nj <= 12) sweep_nj<12>(g, P, tag, dst, t, err, limit, nap);
    else if (nj <= 16) sweep_nj<16>(g, P, tag, dst, t, err, limit, nap);
    else sweep_nj<20>(g, P, tag, dst, t, err, limit, nap);
}

// Fast-model attention of heads hbase .. hbase + 3 (< nh) at position cpos (<= 15): one wave, 16
// lanes per head, lane c owning dims [8c, 8c + 8) (one 16-byte chunk; hd <= 128).  Every operand is
// in LDS: raw = the q|k|v row, kvs = the cached rows [nkv][k|v][cpos][hd], qn / kn = this layer's
// QK-norm weights, tab = the RoPE row at cpos (cos, sin per pair), out = the attention row.
//  * q and k chunks: QK-norm (sum of squares over the head's 16 lanes) and RoPE on the lane's own
//    interleaved pairs, in registers;
//  * scores: per position one 8-wide partial dot (v_dot2c_f32_bf16) per lane, summed across the
//    head's 16-lane row by DPP, kept by lane j;
//  * softmax across the 16 lanes; output: p_j read from lane j, the lane's 8 dims summed over the
//    positions in order.
// The roundings of fast_attn_heads8_lds (fm_attn_dev.h, the launch-per-op path: llama.py:861-975 in
// bf16); the fp32 orders of the dots and of the softmax denominator differ.  store_kv: the lanes
// of each kv group's first q head write the new k / v of cpos to the cache (kc / vc at the slot's
// layer base).
typedef __attribute__((address_space(3))) bf16_t lds_bf16_t;
typedef __attribute__((address_space(3))) float lds_f32_t;
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
typedef __attribute__((address_space(3))) u32x4_t lds_u32x4_t;
struct AttnLds {
    uint32_t raw, kvs, qn, kn, tab, out;
};
template <bool KVG>
__device__ __forceinline__ void pass_attn4(int nh, int nkv, int hd, int cpos, int qk_norm, float eps, float scale,
                                           int hbase, int lane, AttnLds o, bf16_t* kc_base, bf16_t* vc_base,
                                           size_t kv_head_stride, bool store_kv) {
    const lds_u32x4_t* raw = (const lds_u32x4_t*)(size_t)o.raw;
    const lds_u32x4_t* kvs = (const lds_u32x4_t*)(size_t)o.kvs;
    const lds_u32x4_t* qn = (const lds_u32x4_t*)(size_t)o.qn;
    const lds_u32x4_t* kn = (const lds_u32x4_t*)(size_t)o.kn;
    const lds_f32_t* tab = (const lds_f32_t*)(size_t)o.tab;
    lds_u32x4_t* out = (lds_u32x4_t*)(size_t)o.out;
    asm volatile("" : "+v"(lane));  // keep the lane-dependent addressing here (not hoisted out of the caller's op loop)
    const int c = lane & 15, hl = lane >> 4, h = hbase + hl, nck = hd >> 3, g = nh / nkv;
    const bool live = h < nh && c < nck;
    const int hh = h < nh ? h : hbase, kvh = hh / g, cc = c < nck ? c : 0;
    const u32x4_t qw = raw[hh * nck + cc], kw = raw[(nh + kvh) * nck + cc], vw = raw[(nh + nkv + kvh) * nck + cc];
    // QK-norm + RoPE of one chunk; dead lanes hold zeros (they add nothing to the head's sums)
    auto prep = [&](u32x4_t w, const lds_u32x4_t* nwt) {
        float x[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            x[2 * e] = live ? lo_f(w[e]) : 0.f;
            x[2 * e + 1] = live ? hi_f(w[e]) : 0.f;
        }
        if (qk_norm) {
            float ss = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) ss += x[e] * x[e];
            ss = row_sum16(ss);
            const float rs = 1.0f / sqrtf(ss / (float)hd + eps);
            const u32x4_t nv = nwt[cc];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                x[2 * e] = bfround((x[2 * e] * rs) * lo_f(nv[e]));
                x[2 * e + 1] = bfround((x[2 * e + 1] * rs) * hi_f(nv[e]));
            }
        }
        u32x4_t r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float cs = tab[8 * cc + 2 * e], sn = tab[8 * cc + 2 * e + 1];
            r[e] = pack2(bfround(x[2 * e] * cs - x[2 * e + 1] * sn), bfround(x[2 * e + 1] * cs + x[2 * e] * sn));
        }
        return r;
    };
    const u32x4_t qp = prep(qw, qn), kp = prep(kw, kn);
    if (store_kv && live && hh % g == 0) {
        *reinterpret_cast<u32x4_t*>(kc_base + (size_t)kvh * kv_head_stride + (size_t)cpos * hd + 8 * c) = kp;
        *reinterpret_cast<u32x4_t*>(vc_base + (size_t)kvh * kv_head_stride + (size_t)cpos * hd + 8 * c) = vw;
    }
    // scores: position j's 16 partial dots summed across the head's row (DPP), kept by lane j
    const lds_u32x4_t* K = kvs + (size_t)(2 * kvh) * cpos * nck;
    const lds_u32x4_t* V = K + (size_t)cpos * nck;
    // KVG: the cached rows straight from the cache in HBM / L2 (no LDS copy; pass_cfg 5)
    const u32x4_t* Kg = reinterpret_cast<const u32x4_t*>(kc_base + (size_t)kvh * kv_head_stride) + cc;
    const u32x4_t* Vg = reinterpret_cast<const u32x4_t*>(vc_base + (size_t)kvh * kv_head_stride) + cc;
    float sc = -INFINITY;
    for (int jb = 0; jb <= cpos; jb += 4) {  // four positions' rows in flight at once
        u32x4_t kk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            kk[u] = jb + u < cpos ? (KVG ? Kg[(size_t)(jb + u) * nck] : (u32x4_t)K[(jb + u) * nck + cc]) : kp;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float d = row_sum16(dot8(kk[u], qp, 0.f));
            if (c == jb + u && jb + u <= cpos) sc = bfround(bfround(d) * scale);
        }
    }
    const float mx = row_max16(sc);
    const float ex = c <= cpos ? expf(sc - mx) : 0.f;
    const float p = bfround(ex / row_sum16(ex));
    // output: p_j read from lane j of each head's row (four v_readlane, one per row), the lane's
    // 8 dims summed over the positions in order
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int jb = 0; jb <= cpos; jb += 4) {
        u32x4_t vv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            vv[u] = jb + u < cpos ? (KVG ? Vg[(size_t)(jb + u) * nck] : (u32x4_t)V[(jb + u) * nck + cc]) : vw;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = jb + u;
            if (j <= cpos) {
                const float p0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), j));
                const float p1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), 16 + j));
                const float p2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), 32 + j));
                const float p3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), 48 + j));
                const float pj = hl == 0 ? p0 : (hl == 1 ? p1 : (hl == 2 ? p2 : p3));
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    acc[2 * e] += pj * lo_f(vv[u][e]);
                    acc[2 * e + 1] += pj * hi_f(vv[u][e]);
                }
            }
        }
    }
    if (live) {
        u32x4_t r;
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] = pack2(acc[2 * e], acc[2 * e + 1]);
        out[hl * nck + c] = r;
    }
}

}  // namespace

// LDS words of the role hand-offs (u32 offsets inside the flag block)
enum { F_FULL = 0, F_FREE = 16, F_A = 32, F_B = 33, F_X = 34, F_R = 35, F_AT = 36, F_E = 37, F_WORDS = 48 };
// F_R: layers whose q|k|v row is in raw (the attention may start); F_AT: consumer waves' attention
// calls done

// NC consumer waves, a ring of NSLOT slots of PS_FILL 1 KiB fragments, PS_INFL fills in flight.
// SR > 0 (stream form, pass_cfg 6): no loader wave and no LDS ring -- each of the NC STREAM waves
// loads its own contiguous share of every op straight into a ring of SR register fragments
// (non-temporal 16-byte loads, SR KiB in flight per wave, refilled as each fragment is consumed),
// so the weight stream runs on through every seam until SR fragments per wave have landed:
// NC x SR KiB of credit per CU (192 KiB at 4 x 48) instead of the 64-96 KiB LDS ring.  Eight waves
// per workgroup (two per SIMD, 256 VGPRs each).  The exchange waves are unchanged, except that they
// run every head's attention themselves (the stream waves never leave their ring).
// SPLIT (stream form only): stream waves are the workgroup's waves {0, 1, 4, 5} and exchange waves
// {2, 3, 6, 7}: waves go to SIMDs in the order 0, 2, 1, 3 (MI355X_MICROARCH.md, LDS stores), so the
// two roles sit on different SIMDs instead of sharing each one.
template <int NC, int NSLOT, int PS_FILL, int PS_INFL, bool KVG = false, int SR = 0, bool SPLIT = false>
__global__ __launch_bounds__((SR ? 0 : 1) * 64 + (NC + PASS_NWM) * 64, SR ? 2 : 1) void pass_kernel(PassArgs a) {
    static_assert(NSLOT <= 16 && NSLOT > PS_INFL, "ring slots");
    static_assert(SR == 0 || (SR >= 8 && SR <= 56 && SR % 4 == 0), "stream ring: vmcnt is 6 bits; XR divides it");
    constexpr int WL = SR ? 0 : 1;  // loader waves
    auto nfills = [](int nfr) { return (nfr + PS_FILL - 1) / PS_FILL; };
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    bf16_t* xbuf = reinterpret_cast<bf16_t*>(smem + a.off_xbuf);    // the current op's input row
    // residual rows (pre-norm): x (read by Wo's epilogue) and h (read by W2's); two buffers, since
    // one exchange wave finalises Wo from x while the others already sweep h in
    bf16_t* resx = reinterpret_cast<bf16_t*>(smem + a.off_resx);
    bf16_t* resh = reinterpret_cast<bf16_t*>(smem + a.off_resh);
    bf16_t* raw = reinterpret_cast<bf16_t*>(smem + a.off_raw);       // q|k|v row
    bf16_t* kvs = reinterpret_cast<bf16_t*>(smem + a.off_kvs);       // cached K/V rows [nkv][2][cpos][hd]
    float* red = reinterpret_cast<float*>(smem + a.off_red);         // [rows][NC] row partials
    float* ssw = red - 16;                                           // [PASS_NWM] sums of squares
    int* opt = reinterpret_cast<int*>(smem + a.off_opt);             // [nop][12] per-op geometry
    PassLayer* lyt = reinterpret_cast<PassLayer*>(smem + a.off_lyt); // [nlayer] biases / norm weights
    float* atab = reinterpret_cast<float*>(smem + a.off_attc);       // RoPE row at cpos [hd]
    bf16_t* aqn = reinterpret_cast<bf16_t*>(atab + a.hd);            // this layer's q_norm / k_norm [hd]
    bf16_t* akn = aqn + a.hd;
    unsigned char* ring = smem + a.off_ring;                         // [NSLOT][16 KiB] weight fills
    lds_vu32* flg = (lds_vu32*)(smem + a.off_flg);                   // role hand-off words
    unsigned long long* dbg_t = reinterpret_cast<unsigned long long*>(smem + a.off_dbg);  // developer stamps
    auto lds_off = [](const void* p) { return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p; };

    const int wg = blockIdx.x;
    const int pwave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    // role order: [loader], consumers / stream waves, exchange waves
    const int wave = SPLIT ? ((pwave & 2) ? NC : 0) + (((pwave >> 2) << 1) | (pwave & 1)) : pwave;
    const int rtid = wave * 64 + lane;  // thread index in role order
    const unsigned gen = __hip_atomic_load((g_u32*)a.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned limit = 1u << (a.spin_log2 > 0 && a.spin_log2 < 28 ? a.spin_log2 : 16);
    const int nop = a.nop;
    const Dims dm = dims_of(a);

    // ---- start: the exchange waves build the tables and clear the hand-off words
    if (wave >= WL + NC) {
        const int t = rtid - (WL + NC) * 64;
        int s0 = 0;
        for (int o = 0; o < nop; ++o) {  // every thread walks the prefix (nop < 255: cheap)
            Geom g = geom(dm, o, wg);
            g.s0 = s0;
            s0 += nfills(g.nfr);
            if ((o & 255) == t) opt_put(opt, o, g);
        }
        for (int l = t; l < a.nlayer; l += 256) lyt[l] = a.layers[l];
        for (int i = t; i < a.hd; i += 256) atab[i] = a.rope[(size_t)a.cpos * a.hd + i];
        if (t < F_WORDS) flg[t] = 0u;
    }
    __syncthreads();  // the only workgroup barrier

    // one wave's share of a layer's attention: 4 heads per call, wave w8 of nw8 (the exchange waves
    // first, then the consumers); workgroup 0 stores the new k / v of cpos
    auto attention = [&](int layer, bool store_kv, int w8, int nw8) {
        const size_t cb = (size_t)a.row_slot[0] * a.slot_stride + (size_t)layer * a.layer_stride;
        for (int hb = 4 * w8; hb < a.nh; hb += 4 * nw8) {
            AttnLds ao{lds_off(raw), lds_off(kvs), lds_off(aqn), lds_off(akn), lds_off(atab), lds_off(xbuf + (size_t)hb * a.hd)};
            pass_attn4<KVG>(a.nh, a.nkv, a.hd, a.cpos, a.qk_norm, a.eps, a.scale, hb, lane, ao, a.kc + cb, a.vc + cb,
                       (size_t)a.S * a.hd, store_kv);
        }
    };

    if (WL && wave == 0) {
        // ---------------------------------- loader -------------------------------------------
        // fills in sequence; fill s -> slot s % NSLOT once its previous occupant (s - NSLOT) is
        // freed; published (FULL = s + 1) once its 16 DMAs have landed: PS_INFL fills stay in
        // flight, and before waiting for a slot every landed fill is published (a full ring with
        // unpublished fills would deadlock the consumers).
        const uint32_t ring0 = __builtin_amdgcn_readfirstlane(lds_off(ring));
        const uint32_t junk = __builtin_amdgcn_readfirstlane(lds_off(smem + a.off_junk));
        int pub = 0, next = 0;  // fills [pub, next) are issued and not yet published (sequence order)
        // prefetch cursor: while the ring is full (a seam), the fills after it are pulled into L2
        // (op po, fill pfi of it; sequence number pfs), at most a.prefetch fills past the ring
        int po = 0, pfi = 0, pfs = 0;
        Geom pg = opt_get(opt, 0);
        auto prefetch_one = [&](int limit_s) {
            while (po < nop && pfi >= nfills(pg.nfr)) {
                if (++po < nop) pg = opt_get(opt, po);
                pfi = 0;
            }
            if (po >= nop || pfs >= limit_s) return false;
            const int f0 = pfi * PS_FILL;
            const bf16_t* src = pg.w + (size_t)f0 * PS_FR + lane * 8;
#pragma unroll
            for (int i = 0; i < PS_FILL; ++i) {
                const int ok = f0 + i < pg.nfr;
                glds16_pf(src + (ok ? (size_t)i * PS_FR : 0), junk);
            }
            ++pfi;
            ++pfs;
            return true;
        };
        auto publish_oldest = [&]() {
            if (lane == 0) flg[F_FULL + pub % NSLOT] = (unsigned)pub + 1u;
            ++pub;
        };
        for (int o = 0; o < nop; ++o) {
            const Geom g = opt_get(opt, o);
            const int nf = nfills(g.nfr);
            for (int fi = 0; fi < nf; ++fi) {
                const int s = g.s0 + fi, slot = s % NSLOT;
                if (s >= NSLOT && (int)(flg[F_FREE + slot] - (unsigned)(s - NSLOT + 1)) < 0) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    while (pub < next) publish_oldest();
                    // the ring is full: pull the fills after it into L2 while the slot stays taken
                    if (pfs < s) {  // (never re-prefetch what is already in the ring)
                        while (po < nop && pg.s0 + pfi < s) {
                            if (pfi + 1 < nfills(pg.nfr)) ++pfi;
                            else if (++po < nop) { pg = opt_get(opt, po); pfi = 0; }
                        }
                        pfs = s;
                    }
                    int inflight = 0;
                    for (unsigned spin = 0;; ++spin) {
                        if ((int)(flg[F_FREE + slot] - (unsigned)(s - NSLOT + 1)) >= 0) break;
                        if (inflight < 48 / PS_FILL && prefetch_one(s + a.prefetch)) {
                            ++inflight;  // (vmcnt is 6 bits: at most 63 loads outstanding)
                            continue;
                        }
                        if (inflight > 0) {
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                            inflight = 0;
                            continue;
                        }
                        if (spin > limit) {
                            __hip_atomic_store((g_i32*)a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            return;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    asm volatile("" ::: "memory");
                }
                const int f0 = fi * PS_FILL;
                const bf16_t* src = g.w + (size_t)f0 * PS_FR + lane * 8;
                const uint32_t dst = ring0 + (uint32_t)slot * (PS_FILL * 1024);
#pragma unroll
                for (int i = 0; i < PS_FILL; ++i) {  // past the share: fragment 0 of the fill again (cached)
                    const int ok = f0 + i < g.nfr;
                    glds16(src + (ok ? (size_t)i * PS_FR : 0), dst + (uint32_t)(ok ? i : PS_FILL - 1) * 1024);
                }
                next = s + 1;
                if (next - pub > PS_INFL) {
                    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PS_INFL * PS_FILL) : "memory");
                    publish_oldest();
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        while (pub < next) publish_oldest();
        return;
    }

    if constexpr (SR > 0) if (wave < NC) {
        // ------------------------------- stream waves (SR > 0) -------------------------------
        const int c = wave;
        lds_vu32* lerr = flg + F_E;  // a timed-out wait (reported after the loop: no global store in it)
        // this wave's share of every op, as a table in LDS built once: fragments [nfr c / NC,
        // nfr (c + 1) / NC) of the workgroup's contiguous row-major run (a fragment = 512 k of one
        // row; lane l holds k 8 l .. 8 l + 7): {address lo, hi, count, kc0 | fpr << 8 | row0 << 16}
        int4* wt = reinterpret_cast<int4*>(smem + a.off_wtab) + c * nop;
        for (int o = lane; o < nop; o += 64) {
            const Geom g = geom(dm, o, wg);
            const int f0 = (int)(((long long)g.nfr * c) / NC);
            const int m = (int)(((long long)g.nfr * (c + 1)) / NC) - f0;
            const uint64_t p = (uint64_t)(uintptr_t)(g.w + (size_t)f0 * PS_FR);
            const int row0 = f0 / g.fpr;
            wt[o] = make_int4((int)(uint32_t)p, (int)(uint32_t)(p >> 32), m, (f0 - row0 * g.fpr) | (g.fpr << 8) | (row0 << 16));
        }
        if (a.dbg) {
            dbg_t[(NC + c) * 64 + lane] = 0;
            dbg_t[(2 * NC + c) * 64 + lane] = 0;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        auto went = [&](int o, const bf16_t*& p, int& m, int& w) {
            const int4 e = wt[o];
            const uint32_t lo = __builtin_amdgcn_readfirstlane(e.x), hi = __builtin_amdgcn_readfirstlane(e.y);
            p = reinterpret_cast<const bf16_t*>((uintptr_t)(((uint64_t)hi << 32) | lo));
            m = __builtin_amdgcn_readfirstlane(e.z);
            w = __builtin_amdgcn_readfirstlane(e.w);
        };
        // issue cursor: op io, the next fragment's address (lane offset added at the load), the
        // fragments of op io still to issue
        int io = -1, ileft = 0;
        const bf16_t* ip = nullptr;
        auto inext = [&]() {  // the next op with a non-empty share (or nop)
            do {
                if (++io >= nop) break;
                int w;
                went(io, ip, ileft, w);
            } while (ileft == 0);
        };
        inext();
        // past the last op: a fixed 1 KiB of the RoPE table (read by every workgroup: an L2 hit)
        const bf16_t* dummy = reinterpret_cast<const bf16_t*>(a.rope);
        const uint32_t voff = (uint32_t)lane * 16u;
        // The ring is explicit machine code: hipcc's waitcnt pass turns a deep register ring into
        // progressively deeper drains (and vmcnt(0) once the loop holds the op seams), and any copy
        // it inserts of an in-flight register reads garbage.  So each slot is ONE asm statement
        // (wait, MFMA, refills) whose fragment / chunk registers are in-out operands: between two
        // slots those registers are touched by nothing but the asm.  Every vector-memory op of this
        // wave in the loop is a ring load issued in slot order, so slot u's fragment has landed once
        // at most SR - 1 are outstanding; every slot issues exactly one LDS read of the input row
        // (XR fragments ahead), so its chunk is the oldest of at least XR outstanding LDS ops at the
        // wait (other LDS ops only make that wait longer).
        //
        // The dot product runs on the MFMA: the row-major fragment as A (lane l: k 8 l .. 8 l + 7)
        // and the input chunk laid out the same way as B give C[m][n] = sum over the lanes m, m + 16,
        // m + 32, m + 48 of w . x pairings, whose diagonal (m == n) sums to the fragment's dot
        // product; acc4 accumulates a row, and its trace is the row's partial.
        u32x4_t ring[SR];
        auto gbase = [&]() -> uint64_t { return (uint64_t)(uintptr_t)(io < nop ? ip : dummy); };
        auto iadv = [&]() {
            if (io < nop) {
                ip += PS_FR;
                if (--ileft == 0) inext();
            }
        };
        static_for<0, SR>([&](auto u) {
            ring[u] = (u32x4_t){0u, 0u, 0u, 0u};
            asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "+v"(ring[u]) : "v"(voff), "s"(gbase()) : "memory");
            iadv();
        });
        // consume cursor: op co, row / fragment-in-row of the next fragment, fragments left
        int co = -1, cleft = 0, row = 0, kc = 0, fpr = 1;
        int cdone = 0;  // fragments of op co consumed (developer stamps)
        f32x4_t acc4 = {0.f, 0.f, 0.f, 0.f};
        const int dsel = (lane & 15) - 4 * (lane >> 4);  // this lane's diagonal element of C, if any
        bool failed = false;
        // acc4 is only ever defined by asm (tied operands, so the register allocator has no reason
        // to copy it): the MFMAs, the nops that let VALU read an MFMA result, and the clear (an MFMA
        // of zero fragments with SrcC 0)
        const u32x4_t zf = {0u, 0u, 0u, 0u};
        asm volatile("s_nop 7\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %1, 0" : "+v"(acc4) : "v"(zf));  // (VALU-written zeros -> MFMA read)
        auto flush = [&]() {
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(acc4));  // MFMA result -> VALU read
            const float d = dsel == 0 ? acc4[0] : (dsel == 1 ? acc4[1] : (dsel == 2 ? acc4[2] : (dsel == 3 ? acc4[3] : 0.f)));
            const float sm = wave_sum(d);
            if (lane == 0) red[row * NC + c] = sm;
            asm volatile("s_nop 7\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %1, 0" : "+v"(acc4) : "v"(zf));  // (VALU-written zeros -> MFMA read)
        };
        auto arrive = [&](int o) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the row partials are in LDS
            if (a.dbg && lane == 0) dbg_t[c * 64 + (o & 63)] = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) __hip_atomic_fetch_add((unsigned*)(flg + F_A), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        };
        // open the next op: wait for its input row (every op, even an empty share: arrivals stay
        // in op order), arrive at once for an empty share
        auto cnext = [&]() {
            for (++co; co < nop; ++co) {
                if (!(a.mode & 1)) {
                    const unsigned tgt = (unsigned)(co + 1);
                    for (unsigned spin = 0;; ++spin) {
                        if ((int)(flg[F_B] - tgt) >= 0) break;
                        if (spin > limit) {
                            *lerr = 2u;
                            failed = true;
                            co = nop;
                            return;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    asm volatile("" ::: "memory");  // no xbuf read above the flag read
                }
                const bf16_t* p;
                int w;
                went(co, p, cleft, w);
                if (cleft > 0) {
                    kc = w & 255;
                    fpr = (w >> 8) & 255;
                    row = w >> 16;
                    cdone = 0;
                    if (a.dbg && lane == 0) dbg_t[(NC + c) * 64 + (co & 63)] = __builtin_amdgcn_s_memrealtime();
                    return;
                }
                arrive(co);
            }
        };
        constexpr int XR = 4;
        u32x4_t xr[XR];
        const uint32_t xb0 = lds_off(xbuf) + voff;
        int kx = 0;
        auto xaddr = [&]() {
            const uint32_t ad = xb0 + (uint32_t)kx * 1024u;
            kx = kx + 1 == fpr ? 0 : kx + 1;
            return ad;
        };
        // after an op opens: the chunks of its first XR fragments (slot u1 first)
        auto xprime = [&](int u1) {
            kx = kc;
            for (int j = 0; j < XR; ++j) {
                const int t = (u1 + j) % XR;  // xr[t] with constant indices only
                const uint32_t ad = xaddr();
                if (t == 0) asm volatile("ds_read_b128 %0, %1" : "+v"(xr[0]) : "v"(ad) : "memory");
                if (t == 1) asm volatile("ds_read_b128 %0, %1" : "+v"(xr[1]) : "v"(ad) : "memory");
                if (t == 2) asm volatile("ds_read_b128 %0, %1" : "+v"(xr[2]) : "v"(ad) : "memory");
                if (t == 3) asm volatile("ds_read_b128 %0, %1" : "+v"(xr[3]) : "v"(ad) : "memory");
            }
        };
        static_assert(XR == 4, "xprime");
        static_for<0, XR>([&](auto q) { xr[q] = (u32x4_t){0u, 0u, 0u, 0u}; });
        cnext();
        xprime(0);
        while (co < nop) {
            static_for<0, SR>([&](auto u) {
                if (co < nop) {
                    constexpr int ux = (int)u % XR;
                    asm volatile(
                        "s_waitcnt vmcnt(%[nv]) lgkmcnt(%[nl])\n\t"
                        "v_mfma_f32_16x16x32_bf16 %[acc], %[w], %[x], %[acc]\n\t"
                        "ds_read_b128 %[x], %[xa]\n\t"
                        "global_load_dwordx4 %[w], %[vo], %[sb] nt"
                        : [acc] "+v"(acc4), [w] "+v"(ring[u]), [x] "+v"(xr[ux])
                        : [xa] "v"(xaddr()), [vo] "v"(voff), [sb] "s"(gbase()), [nv] "n"(SR - 1), [nl] "n"(XR - 1)
                        : "memory");
                    iadv();
                    if (a.dbg && ++cdone == 32 && lane == 0)  // developer: 32 fragments into the op
                        dbg_t[(2 * NC + c) * 64 + (co & 63)] = __builtin_amdgcn_s_memrealtime();
                    if (++kc == fpr) {
                        flush();
                        ++row;
                        kc = 0;
                    }
                    if (--cleft == 0) {
                        if (kc) flush();
                        arrive(co);
                        cnext();
                        xprime(((int)u + 1) % XR);
                    }
                }
            });
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the ring's tail loads: none left in flight)
        if (failed && lane == 0) __hip_atomic_store((g_i32*)a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.dbg && lane == 0)  // per op: opened (input row seen), 32 fragments in, arrived
            for (int o = 0; o < nop && o < 64; ++o) {
                const unsigned long long t[7] = {dbg_t[(NC + c) * 64 + o], dbg_t[(2 * NC + c) * 64 + o],
                                                 dbg_t[c * 64 + o], 0, 0, 0, 0};
                dbg_record(a.dbg, 0xFB000000u | ((unsigned)wg << 12) | ((unsigned)c << 8) | (unsigned)o, gen, t);
            }
        return;
    }

    if (!SR && wave <= NC) {
        // --------------------------------- consumers -----------------------------------------
        const int c = wave - 1;
        const uint32_t ring0 = lds_off(ring);
        for (int o = 0; o < nop; ++o) {
            const Geom g = opt_get(opt, o);
            if (g.kind == OP_WO && !(a.mode & 1)) {  // heads 16 + 4c ... of this layer's attention
                if (!lds_wait_ge(flg + F_R, (unsigned)g.layer + 1u, limit, a.err)) return;
                attention(g.layer, wg == 0, PASS_NWM + c, PASS_NWM + NC);
                if (lane == 0)
                    __hip_atomic_fetch_add((unsigned*)(flg + F_AT), 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (!(a.mode & 1) && !lds_wait_ge(flg + F_B, (unsigned)(o + 1), limit, a.err)) return;  // op o's input row is in xbuf
            const int nf = nfills(g.nfr);
            float acc = 0.f;
            int cur = -1;
            int fi = ((c - g.s0) % NC + NC) % NC;  // this consumer's fills: s % NC == c
            for (; fi < nf; fi += NC) {
                const int s = g.s0 + fi, slot = s % NSLOT;
                if (!lds_wait_ge(flg + F_FULL + slot, (unsigned)s + 1u, limit, a.err)) return;
                const int f0 = fi * PS_FILL, n = min(PS_FILL, g.nfr - f0);
                int row = f0 / g.fpr, kc = f0 - row * g.fpr;
                if (cur >= 0 && row != cur) {
                    const float sm = wave_sum(acc);
                    if (lane == 0) red[cur * NC + c] = sm;
                    acc = 0.f;
                }
                cur = row;
                const lds_u32x4_t* wsl = (const lds_u32x4_t*)(size_t)(ring0 + (uint32_t)slot * (PS_FILL * 1024)) + lane;
#pragma unroll
                for (int i = 0; i < PS_FILL; ++i) {
                    if (i < n && !(a.mode & 2)) {
                        if (kc == g.fpr) {  // next row of the share
                            const float sm = wave_sum(acc);
                            if (lane == 0) red[cur * NC + c] = sm;
                            acc = 0.f;
                            kc = 0;
                            cur = ++row;
                        }
                        const u32x4_t w = wsl[i * 64];
                        const u32x4_t xv = *reinterpret_cast<const u32x4_t*>(xbuf + kc * PS_FR + lane * 8);
                        acc = dot8(w, xv, acc);
                        ++kc;
                    }
                }
                // the slot's reads have returned (their data fed the dots): free it
                asm volatile("" ::: "memory");
                if (lane == 0) flg[F_FREE + slot] = (unsigned)s + 1u;
            }
            if (cur >= 0) {
                const float sm = wave_sum(acc);
                if (lane == 0) red[cur * NC + c] = sm;
            }
            if (a.dbg && lane == 0) dbg_t[c * 64 + (o & 63)] = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) __hip_atomic_fetch_add((unsigned*)(flg + F_A), 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return;
    }

    // --------------------------------- exchange waves ----------------------------------------
    const int x = wave - NC - WL, t_ = rtid - (WL + NC) * 64;
    const int t = t_;
    const int dim = a.dim, hd = a.hd;
    uint32_t* x32 = reinterpret_cast<uint32_t*>(xbuf);
    uint32_t* rx32 = reinterpret_cast<uint32_t*>(resx);
    uint32_t* rh32 = reinterpret_cast<uint32_t*>(resh);
    unsigned xsync = 0;  // exchange-wave rendezvous count (identical in every exchange wave)
    auto ex_sync = [&]() {
        ++xsync;
        if (lane == 0) __hip_atomic_fetch_add((unsigned*)(flg + F_X), 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        lds_wait_ge(flg + F_X, xsync * PASS_NWM, limit, a.err);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    // this thread's norm weights (pairs t + 256 j of a dim-wide row), loaded ahead of their seam
    // (every helper below takes an opaque copy of t: the compiler would otherwise hoist its
    // t-dependent address arithmetic out of the op loop and spill it)
    uint32_t nw[PS_NJN];
    auto load_nw = [&](const bf16_t* w) {
        int t = t_;
        asm volatile("" : "+v"(t));
        const uint32_t* w32 = reinterpret_cast<const uint32_t*>(w);
#pragma unroll
        for (int j = 0; j < PS_NJN; ++j) nw[j] = w32[min(t + 256 * j, dim / 2 - 1)];
    };
    // sum of squares of this thread's pairs of a residual row (fixed order), staged per wave
    auto stage_ss = [&](const uint32_t* r32) {
        int t = t_;
        asm volatile("" : "+v"(t));
        float ss = 0.f;
        for (int p = t; p < dim / 2; p += 256) {
            const uint32_t w = r32[p];
            const float x0 = lo_f(w), x1 = hi_f(w);
            ss += x0 * x0 + x1 * x1;
        }
        ss = wave_sum(ss);
        if (lane == 0) ssw[x] = ss;
    };
    // xbuf = round(round(r * rs) * w) (RMSNorm.forward, llama.py:989-1000, in bf16)
    auto normalise = [&](const uint32_t* r32) {
        int t = t_;
        asm volatile("" : "+v"(t));
        float tot = 0.f;
#pragma unroll
        for (int i = 0; i < PASS_NWM; ++i) tot += ssw[i];
        const float rs = 1.0f / sqrtf(tot / (float)dim + a.eps);
#pragma unroll
        for (int j = 0; j < PS_NJN; ++j) {
            const int p = t + 256 * j;
            if (p < dim / 2) {
                const uint32_t xv = r32[p], w = nw[j];
                x32[p] = pack2(bfround(bfround(lo_f(xv) * rs) * lo_f(w)), bfround(bfround(hi_f(xv) * rs) * hi_f(w)));
            }
        }
    };
    // cached K/V rows of `layer` (positions < cpos) -> kvs [nkv][k|v][cpos][hd], and its QK-norm
    // weights (the attention reads everything from LDS)
    const int slot = a.row_slot[0];
    auto load_kvs = [&](int layer) {
        int t = t_;
        asm volatile("" : "+v"(t));
        const int cpos = a.cpos, rc = hd / 8, n2 = KVG ? 0 : a.nkv * 2 * cpos * rc;
        const size_t cbase = (size_t)slot * a.slot_stride + (size_t)layer * a.layer_stride;
        for (int i = t; i < n2; i += 256) {
            const int row = i / rc, cc = i - row * rc;
            const int kvh = row / (2 * cpos), rem = row - kvh * 2 * cpos, which = rem / cpos, j = rem - which * cpos;
            const bf16_t* src = (which ? a.vc : a.kc) + cbase + (size_t)kvh * a.S * hd + (size_t)j * hd;
            reinterpret_cast<u32x4_t*>(kvs)[i] = reinterpret_cast<const u32x4_t*>(src)[cc];
        }
        const PassLayer& L = lyt[layer];
        if (a.qk_norm)
            for (int i = t; i < hd; i += 256) {
                aqn[i] = L.qn[i];
                akn[i] = L.kn[i];
            }
    };
    unsigned long long ts[7] = {0, 0, 0, 0, 0, 0, 0}, tatt = 0;
    auto stamp = [&](int i) {
        if (a.dbg && t == 0) ts[i] = __builtin_amdgcn_s_memrealtime();
    };
    auto set_ready = [&](int nready) {  // ops [0, nready) have their input row staged
        ex_sync();
        if ((a.mode & 16) && t == 0) {  // developer: a 20 us seam (the weight rings land meanwhile)
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(8);
        }
        if (t == 0) flg[F_B] = (unsigned)nready;
    };

    if (a.mode & 8) return;  // developer: the weight stream alone (with pass_mode 3)
    // ---- initial seam: the pass input row -> resx, its attention_norm -> xbuf
    {
        const bf16_t* x0 = a.x_in;
        if (a.xidx) {
            int xi = a.xidx[a.xidx_col];
            xi = xi < 0 ? 0 : (xi >= a.xidx_rows ? a.xidx_rows - 1 : xi);
            x0 = a.x_in + (size_t)xi * dim;
        }
        load_nw(lyt[0].an);
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(x0);
        for (int p = t; p < dim / 2; p += 256) rx32[p] = s32[p];
        stage_ss(rx32);
        load_kvs(0);  // (the QK-norm weights even at cpos 0)
        ex_sync();
        normalise(rx32);
        stamp(5);
        set_ready(1);
    }
    for (int o = 0; o < nop; ++o) {
        const Geom g = opt_get(opt, o);
        ts[0] = ts[5];
        lds_wait_ge(flg + F_A, (unsigned)(NC * (o + 1)), limit, a.err);  // op o's consumers all arrived
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        stamp(1);
        // reduce (fixed fill order) + epilogue: thread t < nout owns output o0 + t
        float y = 0.f;
        if (t < g.nout) {
            float s[2] = {0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (q < g.rpo) {
                    const int r = t * g.rpo + q, f0 = r * g.fpr, f1 = f0 + g.fpr - 1;
                    float acc = 0.f;
                    if constexpr (SR > 0) {  // the stream waves whose contiguous shares meet the row, in order
#pragma unroll
                        for (int cw = 0; cw < NC; ++cw) {
                            const int lo = (int)(((long long)g.nfr * cw) / NC), hi = (int)(((long long)g.nfr * (cw + 1)) / NC);
                            if (lo <= f1 && hi > f0) acc += red[r * NC + cw];
                        }
                    } else {
                        for (int fi = f0 / PS_FILL; fi <= f1 / PS_FILL; ++fi) acc += red[r * NC + (g.s0 + fi) % NC];
                    }
                    s[q] = acc;
                }
            }
            const int n = g.o0 + t;
            const PassLayer& L = lyt[g.layer < a.nlayer ? g.layer : a.nlayer - 1];
            if (g.kind == OP_QKV) {  // round(q|k|v + bias)
                y = bfround(s[0] + (L.bqkv ? bf2f(L.bqkv[n]) : 0.f));
            } else if (g.kind == OP_WO) {  // h = x + round(wo . att + bias) (llama.py:841)
                y = bfround(bf2f(resx[n]) + bfround(s[0] + (L.bo ? bf2f(L.bo[n]) : 0.f)));
            } else if (g.kind == OP_W13) {  // round(silu(round(w1 . hn))) * round(w3 . hn) (llama.py:978-986)
                const float ga = bfround(s[0]);
                y = bfround(bfround(ga / (1.0f + expf(-ga))) * bfround(s[1]));
            } else if (g.kind == OP_W2) {  // x = h + round(w2 . act) (llama.py:842)
                y = bfround(bf2f(resh[n]) + bfround(s[0]));
            } else {  // codebook logits, round(head . norm(x)) as fp32
                a.logits[n] = bfround(s[0]);
            }
        }
        const unsigned tag = tag_of(gen, o);
        if (g.kind != OP_HEAD) {
            const float yn = __shfl_down(y, 1);
            if (t < g.nout && !(t & 1))
                __hip_atomic_store((g_u64*)(a.gran + (size_t)o * a.gran_stride + ((g.o0 + t) >> 1)),
                                   ((u64)tag << 32) | pack2(y, yn), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        stamp(2);
        const u64* gv = a.gran + (size_t)o * a.gran_stride;
        if (o + 1 < nop) {
            const Geom gn = opt_get(opt, o + 1);
            if (gn.kind == OP_WO) {  // q|k|v -> raw, then every head's attention -> xbuf
                sweep(gv, a.nqkv / 2, tag, reinterpret_cast<uint32_t*>(raw), t, a.err, limit, a.sweep_nap);
                stamp(3);
                ex_sync();
                stamp(4);
                if (t == 0) flg[F_R] = (unsigned)gn.layer + 1u;  // the consumers take heads 16 ...
                attention(gn.layer, wg == 0, x, SR ? PASS_NWM : PASS_NWM + NC);
                if (a.dbg && t == 0) tatt = __builtin_amdgcn_s_memrealtime() - ts[4];
                if (!SR && !(a.mode & 1)) lds_wait_ge(flg + F_AT, (unsigned)(NC * (gn.layer + 1)), limit, a.err);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            } else if (gn.kind == OP_W2) {  // the SwiGLU row straight in
                sweep(gv, a.inter / 2, tag, x32, t, a.err, limit, a.sweep_nap);
                stamp(3);
                stamp(4);
            } else {  // next layer's QKV, W13, head: the residual row + its RMSNorm
                const PassLayer& L = lyt[gn.layer < a.nlayer ? gn.layer : a.nlayer - 1];
                load_nw(gn.kind == OP_QKV ? L.an : (gn.kind == OP_W13 ? L.fn : a.hnorm));
                uint32_t* r32 = gn.kind == OP_W13 ? rh32 : rx32;
                sweep(gv, dim / 2, tag, r32, t, a.err, limit, a.sweep_nap);
                stage_ss(r32);
                stamp(3);
                ex_sync();
                stamp(4);
                normalise(r32);
            }
            set_ready(o + 2);
            stamp(5);
            // for the op just started: the cached K/V rows (and QK-norm weights) its attention reads
            if (gn.kind == OP_QKV) load_kvs(gn.layer);
        } else if (a.tail_attn) {  // head-less pass ending in a QKV: that layer's K/V store
            if (wg == 0) {
                sweep(gv, a.nqkv / 2, tag, reinterpret_cast<uint32_t*>(raw), t, a.err, limit, a.sweep_nap);
                ex_sync();
                attention(g.layer, true, x, PASS_NWM);  // (the consumers have left)
            }
            stamp(5);
        }
        if (a.dbg && t == 0) {
            unsigned long long mn = ~0ull, mx = 0;
            for (int v = 0; v < NC; ++v) {
                mn = min(mn, dbg_t[v * 64 + (o & 63)]);
                mx = max(mx, dbg_t[v * 64 + (o & 63)]);
            }
            ts[6] = ((mx - mn) << 32) | (tatt & 0xffffffffull);
            dbg_record(a.dbg, 0xFA000000u | ((unsigned)wg << 8) | (unsigned)o, gen, ts);
        }
    }
    // last one out bumps the generation (every workgroup has read it: none can finish before all
    // have published their first op)
    if (t == 0) {
        if (__hip_atomic_fetch_add((g_u32*)(a.sync + 32), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (unsigned)a.nwg - 1) {
            __hip_atomic_store((g_u32*)(a.sync + 32), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store((g_u32*)a.sync, gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
PassLds pass_lds(int kmax, int dim, int nqkv, int nkv, int S, int hd, int maxrows, int nop) {
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    PassLds L;
    size_t o = 0;
    const bool kvg = fm_tuning().pass_cfg == 5;  // K / V read from the cache, the ring takes their LDS
    const bool stream = fm_tuning().pass_cfg >= 6;  // register rings: no LDS ring
    L.ring = (int)o;
    o = al(o + (size_t)(stream ? 0 : (kvg ? 96 : PASS_RING_KB)) * 1024);
    L.xbuf = (int)o;
    o = al(o + (size_t)kmax * 2);
    L.resx = (int)o;
    o = al(o + (size_t)dim * 2);
    L.resh = (int)o;
    o = al(o + (size_t)dim * 2);
    L.raw = (int)o;
    o = al(o + (size_t)nqkv * 2);
    L.kvs = (int)o;
    o = al(o + (kvg ? (size_t)16 : (size_t)nkv * 2 * (S > 1 ? S - 1 : 1) * hd * 2));
    o += 16 * 4;  // the exchange waves' sums of squares, just below red
    L.red = (int)o;
    o = al(o + (size_t)maxrows * PASS_NC * 4);  // [rows][NC]
    L.sc = (int)o;
    o = al(o + 16);  // (spare)
    L.opt = (int)o;
    o = al(o + (size_t)nop * 12 * 4);  // per-op geometry [nop][12]
    L.lyt = (int)o;
    o = al(o + (size_t)((nop + 3) / 4) * sizeof(PassLayer));  // layer table (nlayer <= (nop + 3) / 4)
    L.attc = (int)o;
    o = al(o + (size_t)hd * 4 + 2 * (size_t)hd * 2);  // RoPE row (fp32), q_norm, k_norm
    L.flg = (int)o;
    o = al(o + (size_t)F_WORDS * 4);
    L.junk = (int)o;
    o = al(o + 1024);  // the prefetch DMAs' landing slot
    L.dbg = (int)o;
    o = al(o + (size_t)PASS_NC * 64 * 8 * (stream ? 3 : 1));  // developer stamps (stream: arrive, open, mid)
    L.wtab = (int)o;
    L.bytes = al(o + (stream ? (size_t)PASS_NC * nop * 16 : 0));  // stream waves' per-op shares
    return L;
}

bool pass_shapes_ok(int dim, int nq, int nqkv, int inter, int nhead, int nh, int nkv, int hd, int S, int nwg) {
    // a row spans at most PASS_NC fills of the smallest fill size (8 fragments): each of its
    // partials then comes from a different consumer
    auto k_ok = [](int K) { return K > 0 && K % PS_FR == 0 && K / PS_FR <= 8 * (PASS_NC - 1); };
    auto n_ok = [&](int N) { return N > 0 && N % 2 == 0 && (N / 2) <= 256 * PS_NJ_MAX && N / 2 >= nwg; };
    return nwg > 0 && k_ok(dim) && k_ok(nq) && k_ok(inter) && n_ok(dim) && n_ok(nqkv) && n_ok(inter) &&
           n_ok(nhead) && nq == nh * hd && nqkv == (nh + 2 * nkv) * hd && hd % 16 == 0 && hd <= 128 &&
           nkv > 0 && nh % nkv == 0 && S - 1 < 16 &&
           dim / 2 <= 256 * PS_NJN;
}

void pass_init() {
    static bool done = false;
    if (done) return;
    done = true;
    const void* k[] = {reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 8, 8, 4>),
                       reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 4, 16, 2>),
                       reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 8, 8, 5>),
                       reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 8, 8, 3>),
                       reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 4, 16, 1>),
                       reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 12, 8, 4, true>),
                       reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 1, 8, 0, false, PASS_SR>),
                       reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 1, 8, 0, false, PASS_SR, true>),
                       reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 1, 8, 0, false, 16>),
                       reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 1, 8, 0, false, 32>)};
    for (const void* f : k) HIPCHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
}

static int pass_maxrows(const PassArgs& a) {
    const int mx = std::max({a.nqkv, a.dim, a.inter, a.nhead}) / 2;
    return 2 * 2 * (mx / a.nwg + 1);  // two outputs per pair, two rows per W1||W3 output
}

void launch_pass(hipStream_t s, const PassArgs& a) {
    const PassLds L =
        pass_lds(std::max({a.dim, a.nq, a.inter}), a.dim, a.nqkv, a.nkv, a.S, a.hd, pass_maxrows(a), a.nop);
    FMCHECK(L.bytes <= 160 * 1024 && a.off_ring == L.ring && a.off_xbuf == L.xbuf &&
                a.off_resx == L.resx && a.off_resh == L.resh && a.off_raw == L.raw && a.off_kvs == L.kvs &&
                a.off_red == L.red && a.off_sc == L.sc && a.off_opt == L.opt && a.off_lyt == L.lyt &&
                a.off_attc == L.attc && a.off_flg == L.flg && a.off_junk == L.junk && a.off_dbg == L.dbg &&
                a.off_wtab == L.wtab,
            "pass: LDS layout");
    FMCHECK(a.nop >= 1 && a.nop <= 4 * a.nlayer + 1 && a.nop < 255 && a.cpos >= 0 && a.cpos < a.S,
            "pass: op count / cpos");
    FMCHECK(std::max({a.dim, a.nq, a.inter}) / PS_FR < 256 && pass_maxrows(a) < 32768, "pass: stream table packing");
    FMCHECK(pass_shapes_ok(a.dim, a.nq, a.nqkv, a.inter, a.head ? a.nhead : 2 * a.nwg, a.nh, a.nkv, a.hd, a.S, a.nwg),
            "pass: shapes");
    const dim3 grid(a.nwg), block((1 + PASS_NC + PASS_NWM) * 64);
    FMCHECK((size_t)a.S * a.hd * sizeof(float) >= 1024, "pass: RoPE table under 1 KiB (stream-ring dummy)");
    switch (fm_tuning().pass_cfg) {  // ring of 64 KiB: slots x fill fragments, fills in flight
        case 1: pass_kernel<PASS_NC, 4, 16, 2><<<grid, block, L.bytes, s>>>(a); break;
        case 2: pass_kernel<PASS_NC, 8, 8, 5><<<grid, block, L.bytes, s>>>(a); break;
        case 3: pass_kernel<PASS_NC, 8, 8, 3><<<grid, block, L.bytes, s>>>(a); break;
        case 4: pass_kernel<PASS_NC, 4, 16, 1><<<grid, block, L.bytes, s>>>(a); break;
        case 5: pass_kernel<PASS_NC, 12, 8, 4, true><<<grid, block, L.bytes, s>>>(a); break;  // 96 KiB ring
        case 6:  // stream waves with register rings (no loader wave)
            pass_kernel<PASS_NC, 1, 8, 0, false, PASS_SR><<<grid, dim3((PASS_NC + PASS_NWM) * 64), L.bytes, s>>>(a);
            break;
        case 8:  // stream waves, 16-fragment rings
            pass_kernel<PASS_NC, 1, 8, 0, false, 16><<<grid, dim3((PASS_NC + PASS_NWM) * 64), L.bytes, s>>>(a);
            break;
        case 9:  // stream waves, 32-fragment rings
            pass_kernel<PASS_NC, 1, 8, 0, false, 32><<<grid, dim3((PASS_NC + PASS_NWM) * 64), L.bytes, s>>>(a);
            break;
        case 7:  // the same, stream and exchange waves on different SIMDs
            pass_kernel<PASS_NC, 1, 8, 0, false, PASS_SR, true><<<grid, dim3((PASS_NC + PASS_NWM) * 64), L.bytes, s>>>(a);
            break;
        default: pass_kernel<PASS_NC, 8, 8, 4><<<grid, block, L.bytes, s>>>(a); break;
    }
}

int pass_maxrows_for(int nqkv, int dim, int inter, int nhead, int nwg) {
    PassArgs a{};
    a.nqkv = nqkv;
    a.dim = dim;
    a.inter = inter;
    a.nhead = nhead;
    a.nwg = nwg;
    return pass_maxrows(a);
}

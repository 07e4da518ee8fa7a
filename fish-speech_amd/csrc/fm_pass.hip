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
#include "fm_attn_dev.h"
#include "fm_kernels.h"
#include "fm_runtime.h"

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef unsigned long long u64;

namespace {

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
                                         unsigned limit) {
    asm volatile("" : "+v"(t));  // keep the address arithmetic here (not hoisted out of the caller's loop)
    uint32_t pend = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
        if (t + 256 * j < P) pend |= 1u << j;
    for (unsigned spin = 0;; ++spin) {
        u64 v[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int p = min(t + 256 * j, P - 1);
            v[j] = __hip_atomic_load((g_u64*)(g + p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
        __builtin_amdgcn_s_sleep(1);
    }
}
__device__ __forceinline__ void sweep(const u64* g, int P, unsigned tag, uint32_t* dst, int t, int* err,
                                      unsigned limit) {
    const int nj = (P + 255) >> 8;
    if (nj <= 2) sweep_nj<2>(g, P, tag, dst, t, err, limit);
    else if (nj <= 4) sweep_nj<4>(g, P, tag, dst, t, err, limit);
    else if (nj <= 6) sweep_nj<6>(g, P, tag, dst, t, err, limit);
    else if (nj <= 8) sweep_nj<8>(g, P, tag, dst, t, err, limit);
    else if (nj <= 12) sweep_nj<12>(g, P, tag, dst, t, err, limit);
    else if (nj <= 16) sweep_nj<16>(g, P, tag, dst, t, err, limit);
    else sweep_nj<20>(g, P, tag, dst, t, err, limit);
}

// Fast-model attention of heads hbase .. hbase + 7 (< nh, two whole kv groups when nh / nkv == 4)
// at position cpos: one wave, 8 lanes per head (lane sub owns RoPE pairs sub, sub + 8, ...); every
// operand in LDS, passed as LDS byte offsets so the accesses are ds_ reads out of line: raw = the
// q|k|v row (q and k are rewritten in place after QK-norm + RoPE: a kv group's heads all live in
// this wave), kvs = the cached rows [nkv][k|v][cpos][hd], qn / kn = this layer's QK-norm weights,
// tab = the RoPE row at cpos, pscr = probability scratch [8 heads][16], out = the attention row.
// Scores: lane sub takes positions sub and sub + 8 whole (128-wide dots); softmax across the
// head's 8 lanes; output: lane sub's pairs summed over the positions in order.  The roundings of
// fast_attn_heads8_lds (fm_attn_dev.h, the launch-per-op path: llama.py:861-975 in bf16); the
// fp32 orders of the dots and of the softmax denominator differ.  store_kv: the first q head of
// each kv group writes the new k / v of cpos to the cache (kc / vc at the slot's layer base).
typedef __attribute__((address_space(3))) bf16_t lds_bf16_t;
typedef __attribute__((address_space(3))) float lds_f32_t;
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
typedef __attribute__((address_space(3))) u32x4_t lds_u32x4_t;
struct AttnLds {
    uint32_t raw, kvs, qn, kn, tab, psc, out;
};
__device__ __noinline__ void pass_attn8(int nh, int nkv, int hd, int cpos, int qk_norm, float eps, float scale,
                                        int hbase, int lane, AttnLds o, bf16_t* kc_base, bf16_t* vc_base,
                                        size_t kv_head_stride, bool store_kv) {
    lds_bf16_t* raw = (lds_bf16_t*)(size_t)o.raw;
    const lds_bf16_t* kvs = (const lds_bf16_t*)(size_t)o.kvs;
    const lds_bf16_t* qn = (const lds_bf16_t*)(size_t)o.qn;
    const lds_bf16_t* kn = (const lds_bf16_t*)(size_t)o.kn;
    const lds_f32_t* tab = (const lds_f32_t*)(size_t)o.tab;
    lds_f32_t* psc = (lds_f32_t*)(size_t)o.psc;
    lds_bf16_t* out = (lds_bf16_t*)(size_t)o.out;
    const int g = nh / nkv, PP = hd >> 4;
    const int sub = lane & 7, hl = lane >> 3, h = hbase + hl;
    const bool live = h < nh;
    const int hh = live ? h : hbase, kvh = hh / g;
    const bool kv_writer = live && hh == kvh * g;  // the kv group's first head
    float q0[FATT_MAXPP], q1[FATT_MAXPP], k0[FATT_MAXPP], k1[FATT_MAXPP];
    auto pr = [&](int i) { return 2 * (sub + 8 * (i < PP ? i : 0)); };
    auto ldp = [&](const lds_bf16_t* p, float& x0, float& x1) {
        const uint32_t w = *(const lds_u32_t*)p;
        x0 = lo_f(w);
        x1 = hi_f(w);
    };
    lds_bf16_t* qrow = raw + (size_t)hh * hd;
    lds_bf16_t* krow = raw + (size_t)(nh + kvh) * hd;
    const lds_bf16_t* vrow = raw + (size_t)(nh + nkv + kvh) * hd;
#pragma unroll
    for (int i = 0; i < FATT_MAXPP; ++i) {
        ldp(qrow + pr(i), q0[i], q1[i]);
        ldp(krow + pr(i), k0[i], k1[i]);
        if (i >= PP) q0[i] = q1[i] = k0[i] = k1[i] = 0.f;
    }
    auto sum8 = [](float v) {
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        return v;
    };
    auto prep = [&](float (&x0)[FATT_MAXPP], float (&x1)[FATT_MAXPP], const lds_bf16_t* w) {
        if (qk_norm) {
            float ss = 0.f;
#pragma unroll
            for (int i = 0; i < FATT_MAXPP; ++i) ss += x0[i] * x0[i] + x1[i] * x1[i];
            ss = sum8(ss);
            const float rs = 1.0f / sqrtf(ss / (float)hd + eps);
#pragma unroll
            for (int i = 0; i < FATT_MAXPP; ++i) {
                float w0, w1;
                ldp(w + pr(i), w0, w1);
                x0[i] = bfround((x0[i] * rs) * w0);
                x1[i] = bfround((x1[i] * rs) * w1);
            }
        }
#pragma unroll
        for (int i = 0; i < FATT_MAXPP; ++i) {
            const float c = tab[pr(i)], s = tab[pr(i) + 1];
            const float y0 = bfround(x0[i] * c - x1[i] * s);
            const float y1 = bfround(x1[i] * c + x0[i] * s);
            x0[i] = y0;
            x1[i] = y1;
        }
    };
    prep(q0, q1, qn);
    prep(k0, k1, kn);
    // prepped q / k back into raw (every lane of the wave has read the raw values above)
    if (live) {
#pragma unroll
        for (int i = 0; i < FATT_MAXPP; ++i)
            if (i < PP) *(lds_u32_t*)(qrow + pr(i)) = pack2(q0[i], q1[i]);
    }
    if (kv_writer) {
#pragma unroll
        for (int i = 0; i < FATT_MAXPP; ++i)
            if (i < PP) *(lds_u32_t*)(krow + pr(i)) = pack2(k0[i], k1[i]);
        if (store_kv) {
            bf16_t* kr = kc_base + (size_t)kvh * kv_head_stride + (size_t)cpos * hd;
            bf16_t* vr = vc_base + (size_t)kvh * kv_head_stride + (size_t)cpos * hd;
#pragma unroll
            for (int i = 0; i < FATT_MAXPP; ++i) {
                if (i < PP) {
                    *reinterpret_cast<uint32_t*>(kr + pr(i)) = pack2(k0[i], k1[i]);
                    *reinterpret_cast<uint32_t*>(vr + pr(i)) = *(const lds_u32_t*)(vrow + pr(i));
                }
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // scores: lane sub -> positions j = sub, sub + 8 (clamped reads, masked results)
    const lds_bf16_t* K = kvs + (size_t)(2 * kvh) * cpos * hd;
    const lds_bf16_t* V = K + (size_t)cpos * hd;
    const int nck = hd / 8;  // 16-byte chunks of a row
    float s2[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int j = sub + 8 * r;
        const lds_bf16_t* kr = j < cpos ? K + (size_t)j * hd : krow;
        float d = 0.f;
        for (int c = 0; c < nck; ++c) {
            const u32x4_t qv = *(const lds_u32x4_t*)(qrow + 8 * c);
            const u32x4_t kv = *(const lds_u32x4_t*)(kr + 8 * c);
#pragma unroll
            for (int e = 0; e < 4; ++e) d += lo_f(qv[e]) * lo_f(kv[e]) + hi_f(qv[e]) * hi_f(kv[e]);
        }
        s2[r] = j <= cpos ? bfround(bfround(d) * scale) : -INFINITY;
    }
    auto max8 = [](float v) {
        v = fmaxf(v, __shfl_xor(v, 1));
        v = fmaxf(v, __shfl_xor(v, 2));
        return fmaxf(v, __shfl_xor(v, 4));
    };
    const float mx = max8(fmaxf(s2[0], s2[1]));
    float e2[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) e2[r] = sub + 8 * r <= cpos ? expf(s2[r] - mx) : 0.f;
    const float den = sum8(e2[0] + e2[1]);
    lds_f32_t* ph = psc + hl * 16;
#pragma unroll
    for (int r = 0; r < 2; ++r) ph[sub + 8 * r] = bfround(e2[r] / den);  // 0 past cpos
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // output: lane sub's pairs, positions in order (p = 0 past cpos adds exact zeros)
    float o0[FATT_MAXPP], o1[FATT_MAXPP];
#pragma unroll
    for (int i = 0; i < FATT_MAXPP; ++i) o0[i] = o1[i] = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const float p = ph[j];
        const lds_bf16_t* vr = j < cpos ? V + (size_t)j * hd : vrow;
#pragma unroll
        for (int i = 0; i < FATT_MAXPP; ++i) {
            float v0, v1;
            ldp(vr + pr(i), v0, v1);
            o0[i] += p * v0;
            o1[i] += p * v1;
        }
    }
    if (live) {
        lds_bf16_t* op = out + (size_t)hl * hd;
#pragma unroll
        for (int i = 0; i < FATT_MAXPP; ++i)
            if (i < PP) *(lds_u32_t*)(op + pr(i)) = pack2(o0[i], o1[i]);
    }
}

}  // namespace

// LDS words of the role hand-offs (u32 offsets inside the flag block)
enum { F_FULL = 0, F_FREE = 8, F_A = 16, F_B = 17, F_X = 18, F_WORDS = 32 };

// NC consumer waves, a ring of NSLOT slots of PS_FILL 1 KiB fragments, PS_INFL fills in flight
template <int NC, int NSLOT, int PS_FILL, int PS_INFL>
__global__ __launch_bounds__((1 + NC + PASS_NWM) * 64, 1) void pass_kernel(PassArgs a) {
    static_assert(NSLOT <= 8 && NSLOT > PS_INFL, "ring slots");
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
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const unsigned gen = __hip_atomic_load((g_u32*)a.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned limit = 1u << (a.spin_log2 > 0 && a.spin_log2 < 28 ? a.spin_log2 : 16);
    const int nop = a.nop;
    const Dims dm = dims_of(a);

    // ---- start: the exchange waves build the tables and clear the hand-off words
    if (wave > NC) {
        const int t = (int)threadIdx.x - (1 + NC) * 64;
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

    if (wave == 0) {
        // ---------------------------------- loader -------------------------------------------
        // fills in sequence; fill s -> slot s % NSLOT once its previous occupant (s - NSLOT) is
        // freed; published (FULL = s + 1) once its 16 DMAs have landed: PS_INFL fills stay in
        // flight, and before waiting for a slot every landed fill is published (a full ring with
        // unpublished fills would deadlock the consumers).
        const uint32_t ring0 = __builtin_amdgcn_readfirstlane(lds_off(ring));
        int pend[PS_INFL + 1];
        int np = 0;
        auto publish_oldest = [&]() {
            const int s = pend[0];
#pragma unroll
            for (int i = 0; i < PS_INFL; ++i) pend[i] = pend[i + 1];
            --np;
            if (lane == 0) flg[F_FULL + s % NSLOT] = (unsigned)s + 1u;
        };
        for (int o = 0; o < nop; ++o) {
            const Geom g = opt_get(opt, o);
            const int nf = nfills(g.nfr);
            for (int fi = 0; fi < nf; ++fi) {
                const int s = g.s0 + fi, slot = s % NSLOT;
                if (s >= NSLOT && (int)(flg[F_FREE + slot] - (unsigned)(s - NSLOT + 1)) < 0) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    while (np > 0) publish_oldest();
                    if (!lds_wait_ge(flg + F_FREE + slot, (unsigned)(s - NSLOT + 1), limit, a.err)) return;
                }
                const int f0 = fi * PS_FILL;
                const bf16_t* src = g.w + (size_t)f0 * PS_FR + lane * 8;
                const uint32_t dst = ring0 + (uint32_t)slot * (PS_FILL * 1024);
#pragma unroll
                for (int i = 0; i < PS_FILL; ++i) {  // past the share: fragment 0 of the fill again (cached)
                    const int ok = f0 + i < g.nfr;
                    glds16(src + (ok ? (size_t)i * PS_FR : 0), dst + (uint32_t)(ok ? i : PS_FILL - 1) * 1024);
                }
                pend[np++] = s;
                if (np > PS_INFL) {
                    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PS_INFL * PS_FILL) : "memory");
                    publish_oldest();
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        while (np > 0) publish_oldest();
        return;
    }

    if (wave <= NC) {
        // --------------------------------- consumers -----------------------------------------
        const int c = wave - 1;
        const uint32_t ring0 = lds_off(ring);
        for (int o = 0; o < nop; ++o) {
            if (!(a.mode & 1) && !lds_wait_ge(flg + F_B, (unsigned)(o + 1), limit, a.err)) return;  // op o's input row is in xbuf
            const Geom g = opt_get(opt, o);
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
    const int x = wave - NC - 1, t_ = (int)threadIdx.x - (1 + NC) * 64;
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
        const int cpos = a.cpos, rc = hd / 8, n2 = a.nkv * 2 * cpos * rc;
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
    // every q head's attention (4 exchange waves x 8 heads) from LDS into xbuf; workgroup 0 stores
    // the new k / v of cpos
    auto attention = [&](int layer, bool store_kv) {
        const size_t cb = (size_t)slot * a.slot_stride + (size_t)layer * a.layer_stride;
        for (int hb = 8 * x; hb < a.nh; hb += 8 * PASS_NWM) {
            AttnLds ao{lds_off(raw), lds_off(kvs), lds_off(aqn), lds_off(akn), lds_off(atab),
                       lds_off(smem + a.off_sc) + (uint32_t)(x * 8 * 16 * 4), lds_off(xbuf + (size_t)hb * hd)};
            pass_attn8(a.nh, a.nkv, hd, a.cpos, a.qk_norm, a.eps, a.scale, hb, lane, ao, a.kc + cb, a.vc + cb,
                       (size_t)a.S * hd, store_kv);
        }
    };
    unsigned long long ts[7] = {0, 0, 0, 0, 0, 0, 0}, tatt = 0;
    auto stamp = [&](int i) {
        if (a.dbg && t == 0) ts[i] = __builtin_amdgcn_s_memrealtime();
    };
    auto set_ready = [&](int nready) {  // ops [0, nready) have their input row staged
        ex_sync();
        if (t == 0) flg[F_B] = (unsigned)nready;
    };

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
            for (int q = 0; q < g.rpo; ++q) {
                const int r = t * g.rpo + q, f0 = r * g.fpr, f1 = f0 + g.fpr - 1;
                for (int fi = f0 / PS_FILL; fi <= f1 / PS_FILL; ++fi) s[q] += red[r * NC + (g.s0 + fi) % NC];
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
                sweep(gv, a.nqkv / 2, tag, reinterpret_cast<uint32_t*>(raw), t, a.err, limit);
                stamp(3);
                ex_sync();
                stamp(4);
                attention(gn.layer, wg == 0);
                if (a.dbg && t == 0) tatt = __builtin_amdgcn_s_memrealtime() - ts[4];
            } else if (gn.kind == OP_W2) {  // the SwiGLU row straight in
                sweep(gv, a.inter / 2, tag, x32, t, a.err, limit);
                stamp(3);
                stamp(4);
            } else {  // next layer's QKV, W13, head: the residual row + its RMSNorm
                const PassLayer& L = lyt[gn.layer < a.nlayer ? gn.layer : a.nlayer - 1];
                load_nw(gn.kind == OP_QKV ? L.an : (gn.kind == OP_W13 ? L.fn : a.hnorm));
                uint32_t* r32 = gn.kind == OP_W13 ? rh32 : rx32;
                sweep(gv, dim / 2, tag, r32, t, a.err, limit);
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
                sweep(gv, a.nqkv / 2, tag, reinterpret_cast<uint32_t*>(raw), t, a.err, limit);
                ex_sync();
                attention(g.layer, true);
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
    L.ring = (int)o;
    o = al(o + (size_t)PASS_RING_KB * 1024);
    L.xbuf = (int)o;
    o = al(o + (size_t)kmax * 2);
    L.resx = (int)o;
    o = al(o + (size_t)dim * 2);
    L.resh = (int)o;
    o = al(o + (size_t)dim * 2);
    L.raw = (int)o;
    o = al(o + (size_t)nqkv * 2);
    L.kvs = (int)o;
    o = al(o + (size_t)nkv * 2 * (S > 1 ? S - 1 : 1) * hd * 2);
    o += 16 * 4;  // the exchange waves' sums of squares, just below red
    L.red = (int)o;
    o = al(o + (size_t)maxrows * PASS_NC * 4);  // [rows][NC]
    L.sc = (int)o;
    o = al(o + (size_t)PASS_NWM * 8 * 16 * 4);  // attention probabilities [4 waves][8 heads][16]
    L.opt = (int)o;
    o = al(o + (size_t)nop * 12 * 4);  // per-op geometry [nop][12]
    L.lyt = (int)o;
    o = al(o + (size_t)((nop + 3) / 4) * sizeof(PassLayer));  // layer table (nlayer <= (nop + 3) / 4)
    L.attc = (int)o;
    o = al(o + (size_t)hd * 4 + 2 * (size_t)hd * 2);  // RoPE row (fp32), q_norm, k_norm
    L.flg = (int)o;
    o = al(o + (size_t)F_WORDS * 4);
    L.dbg = (int)o;
    L.bytes = al(o + (size_t)PASS_NC * 64 * 8);  // developer stamps
    return L;
}

bool pass_shapes_ok(int dim, int nq, int nqkv, int inter, int nhead, int nh, int nkv, int hd, int S, int nwg) {
    // a row spans at most PASS_NC fills of the smallest fill size (8 fragments): each of its
    // partials then comes from a different consumer
    auto k_ok = [](int K) { return K > 0 && K % PS_FR == 0 && K / PS_FR <= 8 * (PASS_NC - 1); };
    auto n_ok = [&](int N) { return N > 0 && N % 2 == 0 && (N / 2) <= 256 * PS_NJ_MAX && N / 2 >= nwg; };
    return nwg > 0 && k_ok(dim) && k_ok(nq) && k_ok(inter) && n_ok(dim) && n_ok(nqkv) && n_ok(inter) &&
           n_ok(nhead) && nq == nh * hd && nqkv == (nh + 2 * nkv) * hd && hd % 16 == 0 && hd <= 16 * FATT_MAXPP &&
           nkv > 0 && nh % nkv == 0 && (nh / nkv) * 2 <= 8 && 8 % (nh / nkv) == 0 && S - 1 < 16 &&
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
                       reinterpret_cast<const void*>(&pass_kernel<PASS_NC, 4, 16, 1>)};
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
                a.off_attc == L.attc && a.off_flg == L.flg && a.off_dbg == L.dbg,
            "pass: LDS layout");
    FMCHECK(a.nop >= 1 && a.nop <= 4 * a.nlayer + 1 && a.nop < 255 && a.cpos >= 0 && a.cpos < a.S,
            "pass: op count / cpos");
    FMCHECK(pass_shapes_ok(a.dim, a.nq, a.nqkv, a.inter, a.head ? a.nhead : 2 * a.nwg, a.nh, a.nkv, a.hd, a.S, a.nwg),
            "pass: shapes");
    const dim3 grid(a.nwg), block((1 + PASS_NC + PASS_NWM) * 64);
    switch (fm_tuning().pass_cfg) {  // ring of 64 KiB: slots x fill fragments, fills in flight
        case 1: pass_kernel<PASS_NC, 4, 16, 2><<<grid, block, L.bytes, s>>>(a); break;
        case 2: pass_kernel<PASS_NC, 8, 8, 5><<<grid, block, L.bytes, s>>>(a); break;
        case 3: pass_kernel<PASS_NC, 8, 8, 3><<<grid, block, L.bytes, s>>>(a); break;
        case 4: pass_kernel<PASS_NC, 4, 16, 1><<<grid, block, L.bytes, s>>>(a); break;
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

// Device-side fast-model attention: one (row, q head) per wave for fast_attn2_kernel (fm_attn.hip),
// and the LDS-staged form the Wo GEMV's PRO_FATT prologue runs (fm_gemv.hip).
//
// Fast-model attention at codebook position cpos (llama.py:947-975), every rounding of the
// reference's matmul-softmax-matmul kept: ONE wave per q head, no LDS, no barrier.  Lane l owns
// dimension pairs l, l+64 (RoPE pairs).  Each wave recomputes the new k (qk-norm + RoPE, cheap) so
// waves never wait on each other; the first q head of each kv group writes k/v of cpos to the fast
// cache.
#pragma once
#include "fm_common.h"
#include "fm_kernels.h"

constexpr int FAST_ATTN_MAXJ = 16;  // cached rows a wave keeps in registers (cpos < 16)

// (p[0], p[1]) as floats
template <typename T> __device__ __forceinline__ void ld_pair(const T* p, float& x0, float& x1) {
    if constexpr (sizeof(T) == 2) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
        x0 = __uint_as_float(w << 16);
        x1 = __uint_as_float(w & 0xffff0000u);
    } else {
        x0 = ld(p, 0);
        x1 = ld(p, 1);
    }
}
// elements e, e + 1 of raw projection row r: from the T row, or (qslab) round(sum of the kp fp32
// K-part slabs [kp][R][ld] + bias) -- the one rounding the projection's own epilogue does
template <typename T>
__device__ __forceinline__ void raw_pair(const T* qkv, int ldq, const float* qslab, int kp, int R, const T* bias,
                                         int r, size_t e, float& x0, float& x1) {
    if (qslab) {
        const size_t i = (size_t)r * ldq + e, st = (size_t)R * ldq;
        float a = qslab[i], b = qslab[i + 1];
        for (int q = 1; q < kp; ++q) {
            a += qslab[q * st + i];
            b += qslab[q * st + i + 1];
        }
        if (bias) {
            a += ld(bias, e);
            b += ld(bias, e + 1);
        }
        x0 = rnd<T>(a);
        x1 = rnd<T>(b);
    } else {
        ld_pair<T>(qkv + (size_t)r * ldq + e, x0, x1);
    }
}

template <typename T>
__device__ __forceinline__ void fast_attn_head(const FastFusedArgs<T>& a, int r, int h, int lane,
                                               unsigned long long (&tz)[7]) {
    const int hd = a.hd, g = a.nh / a.nkv, kvh = h / g, cpos = a.cpos, half = hd >> 1;
    const float* tab = a.rope + (size_t)cpos * hd;
    const int slot = a.row_slot[r];
    float q0[2], q1[2], k0[2], k1[2], v0[2], v1[2], qw0[2], qw1[2], kw0[2], kw1[2], c_[2], s_[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int p = lane + 64 * u;
        const bool ok = p < half;
        const int pp = ok ? p : 0;
        raw_pair<T>(a.qkv, a.ldqkv, a.qslab, a.qslab_kp, gridDim.x, a.qbias, r, (size_t)h * hd + 2 * pp, q0[u], q1[u]);
        raw_pair<T>(a.qkv, a.ldqkv, a.qslab, a.qslab_kp, gridDim.x, a.qbias, r, (size_t)(a.nh + kvh) * hd + 2 * pp,
                    k0[u], k1[u]);
        raw_pair<T>(a.qkv, a.ldqkv, a.qslab, a.qslab_kp, gridDim.x, a.qbias, r,
                    (size_t)(a.nh + a.nkv + kvh) * hd + 2 * pp, v0[u], v1[u]);
        qw0[u] = a.qk_norm ? ld(a.qn, 2 * pp) : 1.f;
        qw1[u] = a.qk_norm ? ld(a.qn, 2 * pp + 1) : 1.f;
        kw0[u] = a.qk_norm ? ld(a.kn, 2 * pp) : 1.f;
        kw1[u] = a.qk_norm ? ld(a.kn, 2 * pp + 1) : 1.f;
        c_[u] = tab[2 * pp];
        s_[u] = tab[2 * pp + 1];
        if (!ok) q0[u] = q1[u] = k0[u] = k1[u] = v0[u] = v1[u] = 0.f;
    }
    const size_t base = (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * hd;
    T* kc = a.kc + base;
    T* vc = a.vc + base;
    // cached rows j < cpos: the lane's two pairs of each
    float K0[FAST_ATTN_MAXJ][2], K1[FAST_ATTN_MAXJ][2], V0[FAST_ATTN_MAXJ][2], V1[FAST_ATTN_MAXJ][2];
#pragma unroll
    for (int j = 0; j < FAST_ATTN_MAXJ; ++j) {
        if (j < cpos) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int p = lane + 64 * u;
                const int pp = p < half ? p : 0;
                ld_pair<T>(kc + (size_t)j * hd + 2 * pp, K0[j][u], K1[j][u]);
                ld_pair<T>(vc + (size_t)j * hd + 2 * pp, V0[j][u], V1[j][u]);
                if (p >= half) K0[j][u] = K1[j][u] = V0[j][u] = V1[j][u] = 0.f;
            }
        }
    }
    if (a.dbg) tz[1] = __builtin_amdgcn_s_memrealtime();
    // qk-norm (fp32 incl. weight, one rounding) + RoPE (bf16 table, rounded)
    auto prep = [&](float (&x0)[2], float (&x1)[2], const float (&w0)[2], const float (&w1)[2], bool norm) {
        if (norm) {
            float ss = 0.f;
#pragma unroll
            for (int u = 0; u < 2; ++u) ss += x0[u] * x0[u] + x1[u] * x1[u];
            ss = wave_sum(ss);
            const float rs = 1.0f / sqrtf(ss / (float)hd + a.eps);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                x0[u] = rnd<T>((x0[u] * rs) * w0[u]);
                x1[u] = rnd<T>((x1[u] * rs) * w1[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const float y0 = rnd<T>(x0[u] * c_[u] - x1[u] * s_[u]);
            const float y1 = rnd<T>(x1[u] * c_[u] + x0[u] * s_[u]);
            x0[u] = y0;
            x1[u] = y1;
        }
    };
    prep(q0, q1, qw0, qw1, a.qk_norm);
    prep(k0, k1, kw0, kw1, a.qk_norm);
    if (a.qdbg) {  // per-op test hook only (fm_op_qk_rope)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int p = lane + 64 * u;
            if (p < half) {
                a.qdbg[((size_t)r * a.nh + h) * hd + 2 * p] = q0[u];
                a.qdbg[((size_t)r * a.nh + h) * hd + 2 * p + 1] = q1[u];
            }
        }
    }
    if (a.dbg) tz[2] = __builtin_amdgcn_s_memrealtime();
    if (h == kvh * g) {  // first q head of the group stores the new k / v
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int p = lane + 64 * u;
            if (p < half) {
                st(kc + (size_t)cpos * hd, 2 * p, k0[u]);
                st(kc + (size_t)cpos * hd, 2 * p + 1, k1[u]);
                st(vc + (size_t)cpos * hd, 2 * p, v0[u]);
                st(vc + (size_t)cpos * hd, 2 * p + 1, v1[u]);
            }
        }
    }
    // scores round(round(q.k) * scale), softmax, probabilities rounded (fast SDPA path)
    float sc[FAST_ATTN_MAXJ + 1];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j <= FAST_ATTN_MAXJ; ++j) {
        if (j > cpos) break;
        float d = 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const float a0 = j < cpos ? K0[j < FAST_ATTN_MAXJ ? j : 0][u] : k0[u];
            const float a1 = j < cpos ? K1[j < FAST_ATTN_MAXJ ? j : 0][u] : k1[u];
            d += q0[u] * a0 + q1[u] * a1;
        }
        d = wave_sum(d);
        sc[j] = rnd<T>(rnd<T>(d) * a.scale);
        mx = fmaxf(mx, sc[j]);
    }
    if (a.dbg) tz[3] = __builtin_amdgcn_s_memrealtime();
    float den = 0.f;
#pragma unroll
    for (int j = 0; j <= FAST_ATTN_MAXJ; ++j) {
        if (j > cpos) break;
        sc[j] = expf(sc[j] - mx);
        den += sc[j];
    }
    float o0[2] = {0.f, 0.f}, o1[2] = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j <= FAST_ATTN_MAXJ; ++j) {
        if (j > cpos) break;
        const float p = rnd<T>(sc[j] / den);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            o0[u] += p * (j < cpos ? V0[j < FAST_ATTN_MAXJ ? j : 0][u] : v0[u]);
            o1[u] += p * (j < cpos ? V1[j < FAST_ATTN_MAXJ ? j : 0][u] : v1[u]);
        }
    }
    T* out = a.out + (size_t)r * a.nh * hd + (size_t)h * hd;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int p = lane + 64 * u;
        if (p < half) {
            st(out, 2 * p, o0[u]);
            st(out, 2 * p + 1, o1[u]);
        }
    }
}

// The same fast-model attention for EIGHT q heads at once (one wave: 8 lanes per head, lane sub
// owns RoPE pairs sub, sub+8, ...), every operand already staged in LDS by the Wo GEMV's PRO_FATT
// prologue (fm_gemv.hip): raw = the row's q|k|v projections, kvs = cached rows [nkv][k|v][cpos][hd],
// qn / kn = QK-norm weights, tab = the RoPE row at cpos.  Same roundings as fast_attn_head (the
// fp32 reduction order of the dot products differs).  Heads hbase .. hbase+7 (< hend); head h's
// output goes to out + (h - hbase) * hd.  store_kv: the first q head of each kv group writes the
// new k / v of cpos to the fast cache (one block per launch).
constexpr int FATT_MAXPP = 8;  // RoPE pairs per lane: hd <= 128
template <typename T>
__device__ __forceinline__ void fast_attn_heads8_lds(const FastFusedArgs<T>& a, int hbase, int hend, int lane,
                                                     const T* raw, const T* kvs, const T* qn, const T* kn,
                                                     const float* tab, T* out, bool store_kv, int slot) {
    const int hd = a.hd, g = a.nh / a.nkv, cpos = a.cpos, PP = hd >> 4;
    const int sub = lane & 7, h = hbase + (lane >> 3);
    const bool live = h < hend;
    const int hh = live ? h : hbase, kvh = hh / g;
    float q0[FATT_MAXPP], q1[FATT_MAXPP], k0[FATT_MAXPP], k1[FATT_MAXPP], v0[FATT_MAXPP], v1[FATT_MAXPP];
#pragma unroll
    for (int i = 0; i < FATT_MAXPP; ++i) {
        const int d = 2 * (sub + 8 * (i < PP ? i : 0));
        q0[i] = ld(raw, (size_t)hh * hd + d);
        q1[i] = ld(raw, (size_t)hh * hd + d + 1);
        k0[i] = ld(raw, (size_t)(a.nh + kvh) * hd + d);
        k1[i] = ld(raw, (size_t)(a.nh + kvh) * hd + d + 1);
        v0[i] = ld(raw, (size_t)(a.nh + a.nkv + kvh) * hd + d);
        v1[i] = ld(raw, (size_t)(a.nh + a.nkv + kvh) * hd + d + 1);
        if (i >= PP) q0[i] = q1[i] = k0[i] = k1[i] = v0[i] = v1[i] = 0.f;
    }
    auto sum8 = [](float v) {
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        return v;
    };
    auto prep = [&](float (&x0)[FATT_MAXPP], float (&x1)[FATT_MAXPP], const T* w, bool norm) {
        if (norm) {
            float ss = 0.f;
#pragma unroll
            for (int i = 0; i < FATT_MAXPP; ++i) ss += x0[i] * x0[i] + x1[i] * x1[i];
            ss = sum8(ss);
            const float rs = 1.0f / sqrtf(ss / (float)hd + a.eps);
#pragma unroll
            for (int i = 0; i < FATT_MAXPP; ++i) {
                const int d = 2 * (sub + 8 * (i < PP ? i : 0));
                x0[i] = rnd<T>((x0[i] * rs) * ld(w, d));
                x1[i] = rnd<T>((x1[i] * rs) * ld(w, d + 1));
            }
        }
#pragma unroll
        for (int i = 0; i < FATT_MAXPP; ++i) {
            const int d = 2 * (sub + 8 * (i < PP ? i : 0));
            const float c = tab[d], s = tab[d + 1];
            const float y0 = rnd<T>(x0[i] * c - x1[i] * s);
            const float y1 = rnd<T>(x1[i] * c + x0[i] * s);
            x0[i] = y0;
            x1[i] = y1;
        }
    };
    prep(q0, q1, qn, a.qk_norm);
    prep(k0, k1, kn, a.qk_norm);
    if (store_kv && live && h == kvh * g) {
        const size_t base = (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * hd + (size_t)cpos * hd;
#pragma unroll
        for (int i = 0; i < FATT_MAXPP; ++i) {
            if (i < PP) {
                const int d = 2 * (sub + 8 * i);
                st(a.kc + base, d, k0[i]);
                st(a.kc + base, d + 1, k1[i]);
                st(a.vc + base, d, v0[i]);
                st(a.vc + base, d + 1, v1[i]);
            }
        }
    }
    const T* K = kvs + (size_t)(2 * kvh) * cpos * hd;
    const T* V = K + (size_t)cpos * hd;
    float sc[FAST_ATTN_MAXJ + 1];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j <= FAST_ATTN_MAXJ; ++j) {
        if (j > cpos) break;
        float dd = 0.f;
#pragma unroll
        for (int i = 0; i < FATT_MAXPP; ++i) {
            if (i < PP) {
                const int d = 2 * (sub + 8 * i);
                const float a0 = j < cpos ? ld(K, (size_t)j * hd + d) : k0[i];
                const float a1 = j < cpos ? ld(K, (size_t)j * hd + d + 1) : k1[i];
                dd += q0[i] * a0 + q1[i] * a1;
            }
        }
        dd = sum8(dd);
        sc[j] = rnd<T>(rnd<T>(dd) * a.scale);
        mx = fmaxf(mx, sc[j]);
    }
    float den = 0.f;
#pragma unroll
    for (int j = 0; j <= FAST_ATTN_MAXJ; ++j) {
        if (j > cpos) break;
        sc[j] = expf(sc[j] - mx);
        den += sc[j];
    }
    float o0[FATT_MAXPP], o1[FATT_MAXPP];
#pragma unroll
    for (int i = 0; i < FATT_MAXPP; ++i) o0[i] = o1[i] = 0.f;
#pragma unroll
    for (int j = 0; j <= FAST_ATTN_MAXJ; ++j) {
        if (j > cpos) break;
        const float pj = rnd<T>(sc[j] / den);
#pragma unroll
        for (int i = 0; i < FATT_MAXPP; ++i) {
            if (i < PP) {
                const int d = 2 * (sub + 8 * i);
                o0[i] += pj * (j < cpos ? ld(V, (size_t)j * hd + d) : v0[i]);
                o1[i] += pj * (j < cpos ? ld(V, (size_t)j * hd + d + 1) : v1[i]);
            }
        }
    }
    if (live) {
        T* o = out + (size_t)(h - hbase) * hd;
#pragma unroll
        for (int i = 0; i < FATT_MAXPP; ++i) {
            if (i < PP) {
                const int d = 2 * (sub + 8 * i);
                st(o, d, o0[i]);
                st(o, d + 1, o1[i]);
            }
        }
    }
}

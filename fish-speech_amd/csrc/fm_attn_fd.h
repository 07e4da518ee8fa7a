// fm_attn_fd.h -- the slow model's flash-decode attention body (attn_fd_kernel, fm_attn.hip),
// shared with the fused slow attention + wo launch (fattn_slow_wo_kernel, fm_rowgemv.hip).
// Attention.forward at one query row per slot: /root/reference/fish_speech/models/text2semantic/
// llama.py:883-975 (qk-norm :894-897, RoPE :903-910, KVCache.update :205-214, SDPA :951-969).
#pragma once
#include "fm_common.h"
#include "fm_kernels.h"
#include "fm_attn_dev.h"
#include "fm_frag.h"

// developer stamps (attn_fd_kernel only: the fused launch keeps no stamp registers)
#define FD_TS(n) if (!TX && a.dbg) tz[n] = __builtin_amdgcn_s_memrealtime();

// Slow-model decode attention, flash-decode form (every batch size): grid (R, nkv, maxsplit),
// 256 threads.  A (row, kv head) is cut into nsp <= maxsplit contiguous splits of at least a.cap
// positions, computed on the device from pos (one captured graph serves every frame).  A block
// walks its split in passes of 64 positions (16 per wave, lane layout of attn_dec3: K slice =
// position 16w + (lane & 15), quarter lane >> 4 of hd; V slices = positions 16w + 4it + (lane >> 4),
// dims 8 (lane & 15) .. +8), the next pass's K / V loads in flight while the current one is scored.
// Every wave keeps its own running (max, sum, o) per q head (online softmax: no block barrier in
// the loop); the block folds its waves through LDS and writes the output (nsp == 1) or a
// write-through (m, l, o) partial.  The last-arriving split (relaxed agent ticket) combines the
// partials with every load issued up front: 16 lanes per group = 16 splits, shuffles reduce
// across them (the loop-carried combine of attn_decode2 / attn_dec3 issued its loads one by one).
// The split holding `pos` normalises + ropes the new k (llama.py:894-910), writes k / v to the
// cache (llama.py:205-214) and uses them in place of the cache rows it loaded.
// 16 bytes of T as floats (bf16: 8, fp32: 4)
template <typename T> __device__ __forceinline__ void cvt16(const u32x4_t v, float (&o)[16 / sizeof(T)]) {
    if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o[2 * i] = __uint_as_float(v[i] << 16);
            o[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = __uint_as_float(v[i]);
    }
}

constexpr int FD_GM = 4;
// v summed over the wave's four 16-lane rows (lanes l, l ^ 16, l ^ 32, l ^ 48) by two VALU half
// exchanges (v_permlane32_swap, v_permlane16_swap) instead of LDS-routed shuffles
__device__ __forceinline__ float sum_rows4(float v, int lane) {
    const unsigned u = __float_as_uint(v);
    const auto r32 = __builtin_amdgcn_permlane32_swap(u, u, false, false);  // [0]: vdst, [1]: src
    v += __uint_as_float(lane < 32 ? r32[1] : r32[0]);                   // + lane ^ 32
    const unsigned w = __float_as_uint(v);
    const auto r16 = __builtin_amdgcn_permlane16_swap(w, w, false, false);
    return v + __uint_as_float(((lane >> 4) & 1) ? r16[0] : r16[1]);      // + lane ^ 16
}
// 8 floats (T-exact values) as one MFMA fragment of T
template <typename T> __device__ __forceinline__ typename Frag<T>::f frag_f32(const float* v) {
    typename Frag<T>::f f;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = hi_pair(v[2 * i], v[2 * i + 1]);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f.lo[i] = v[i];
            f.hi[i] = v[4 + i];
        }
    }
    return f;
}
// NW waves per block (4, 8 or 16): 16 NW positions per pass.  The batch-1 launches use wide blocks
// and long splits, so below fd_min16 cached positions one block per kv head needs no cross-block
// combine.
// TX (the fused slow attention + wo, fm_rowgemv.hip fattn_slow_wo_kernel): the output row is not
// stored as T but as tagged 32-bit words (bf16 value << 16 | gen, write-through) into xt [nh * hd],
// which the wo row blocks of the same launch poll; r must be 0 (batch 1).
template <typename T, int HD, int NW, bool TX>
__device__ __forceinline__ void attn_fd_body(const AttnDecArgs<T>& a, const int r, const int kvh, const int sp,
                                             const int gx, const int gz, uint32_t* xt, const uint32_t gen) {
    static_assert(!TX || sizeof(T) == 2, "tagged words carry bf16");
    static_assert(HD % 32 == 0 && HD <= 128, "head_dim a multiple of 32 up to 128");
    constexpr int NT = NW * 64, FD_TILE = 16 * NW;
    constexpr int VL = 8 * (int)sizeof(T) / 16;     // 16-B loads per V slice
    constexpr int half = HD / 2;
    __shared__ __attribute__((aligned(16))) float q_s[FD_GM][HD];
    __shared__ __attribute__((aligned(16))) float kv_new[2][HD];
    __shared__ __attribute__((aligned(16))) float wml[NW][FD_GM][2];
    // PV partials [wave][V position group][head][dim]; 16 waves fold the 4 groups by shuffles first
    constexpr int OG = (NW > 4 || TX) ? 1 : 4;
    __shared__ __attribute__((aligned(16))) float ored[NW][OG][FD_GM][HD];
    __shared__ int flag;
    unsigned long long tz[7] = {0, 0, 0, 0, 0, 0, 0};
    FD_TS(0)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l16 = lane & 15, qq = lane >> 4;
    const int g = a.nh / a.nkv, nitem = g + 2;
    // ---- round trip 1: slot, pos and this wave's raw rows (q heads, then new k, new v); the raw
    // loads do not depend on pos and go out with it (clamped, unconditional)
    const int slot = a.row_slot[r];
    const int pos = a.row_pos[r];
    constexpr int NI = (2 + FD_GM + NW - 1) / NW;  // q heads + new k + new v over the waves
    float x0[NI], x1[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int it = wave + NW * i;
        const int row = it < g ? kvh * g + it : (it == g ? a.nh + kvh : a.nh + a.nkv + kvh);
        const bool ok = it < nitem && lane < half;
        float v0, v1;
        raw_pair<T>(a.qkv, a.ldqkv, a.qslab, a.qslab_kp, gx, a.qbias, r,
                    (size_t)(it < nitem ? row : 0) * HD + 2 * (lane < half ? lane : 0), v0, v1);
        x0[i] = ok ? v0 : 0.f;
        x1[i] = ok ? v1 : 0.f;
    }
    const int npos = pos + 1;
    int nsp = min(gz, (npos + a.cap - 1) / a.cap);
    const int chunk = ((npos + nsp - 1) / nsp + 15) & ~15;
    nsp = (npos + chunk - 1) / chunk;
    if (sp >= nsp) return;
    const int j0 = sp * chunk, jend = min(j0 + chunk, npos);
    const bool owner = jend == npos;
    // ---- round trip 2 (pass 0's K / V), issued before the q-side arithmetic
    const size_t base = (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * HD;
    T* kc = a.kc + base;
    T* vc = a.vc + base;
    const int vd = 8 * l16 < HD ? 8 * l16 : HD - 8;
    // K as MFMA B fragments: lane (l16, qq) holds K[position l16 of its wave's 16][32 ks + 8 qq, + 8)
    using F = Frag<T>;
    constexpr int NKS = HD / 32;
    typename F::f kb[NKS];
    u32x4_t vb[4][VL];
    auto issue_k = [&](int jb) {
        const int jk = min(jb + 16 * wave + l16, jend - 1);
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) kb[ks] = F::load(kc + (size_t)jk * HD + 32 * ks + 8 * qq);
    };
    auto issue_v = [&](int jb) {
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int jv = min(jb + 16 * wave + 4 * it + qq, jend - 1);
            const u32x4_t* pv = reinterpret_cast<const u32x4_t*>(vc + (size_t)jv * HD + vd);
#pragma unroll
            for (int c = 0; c < VL; ++c) vb[it][c] = pv[c];
        }
    };
    auto issue = [&](int jb) {
        issue_k(jb);
        issue_v(jb);
    };
    issue(j0);
    // ---- q heads (+ new k / v in the owner): qk-norm (fp32 incl. weight, one rounding), RoPE
    const float* tab = a.rope + (size_t)pos * HD;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int it = wave + NW * i;
        if (it >= nitem || (it >= g && !owner)) continue;
        const bool isq = it < g, isk = it == g;
        if (a.qk_norm && (isq || isk)) {
            const float ss = wave_sum(x0[i] * x0[i] + x1[i] * x1[i]);
            const float rs = 1.0f / sqrtf(ss / (float)HD + a.eps);
            const T* nw = isq ? a.qn : a.kn;
            if (lane < half) {
                x0[i] = rnd<T>((x0[i] * rs) * ld(nw, 2 * lane));
                x1[i] = rnd<T>((x1[i] * rs) * ld(nw, 2 * lane + 1));
            }
        }
        if (lane < half) {
            float y0 = x0[i], y1 = x1[i];
            if (isq || isk) {
                const float c = tab[2 * lane], sn = tab[2 * lane + 1];
                y0 = rnd<T>(x0[i] * c - x1[i] * sn);
                y1 = rnd<T>(x1[i] * c + x0[i] * sn);
            }
            if (isq) {
                q_s[it][2 * lane] = y0;
                q_s[it][2 * lane + 1] = y1;
                if (a.qdbg && sp == 0) {  // per-op test hook only
                    float* qdp = a.qdbg + ((size_t)r * a.nh + kvh * g + it) * HD;
                    qdp[2 * lane] = y0;
                    qdp[2 * lane + 1] = y1;
                }
            } else {
                kv_new[isk ? 0 : 1][2 * lane] = y0;
                kv_new[isk ? 0 : 1][2 * lane + 1] = y1;
                T* dst = (isk ? kc : vc) + (size_t)pos * HD;
                st(dst, 2 * lane, y0);
                st(dst, 2 * lane + 1, y1);
            }
        }
    }
    lds_barrier();  // q_s / kv_new; pass 0's K / V loads stay in flight
    FD_TS(1)
    // ---- q heads as the MFMA A operand: head h in row 4h (the other rows zero), so that the
    // accumulator's first register holds S[head qq][position l16] in every lane
    const int qh = l16 >> 2;
    const bool qrow = (l16 & 3) == 0 && qh < g;
    typename F::f qa[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        float qv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) qv[e] = qrow ? q_s[qh][32 * ks + 8 * qq + e] : 0.f;
        qa[ks] = frag_f32<T>(qv);
    }
    // ---- passes: S = Q K^T of the wave's 16 positions on one MFMA chain (lane (l16, qq): head qq,
    // position l16), online softmax per head = per 16-lane row (DPP), P through the wave's LDS rows,
    // P V on the VALU in fp32 (lane: positions 4 it + qq, dims vd, every head)
    __shared__ __attribute__((aligned(16))) float p_s[NW][16][FD_GM];
    float m_run = -INFINITY, l_run = 0.f, o[FD_GM][8];
#pragma unroll
    for (int h = 0; h < FD_GM; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) o[h][e] = 0.f;
    const int npass = (jend - j0 + FD_TILE - 1) / FD_TILE;
    for (int pa = 0; pa < npass; ++pa) {
        const int jb = j0 + pa * FD_TILE;
        const int jk = jb + 16 * wave + l16;
        if (owner && jk == pos) {  // the new row from LDS, not the cache row loaded before it was written
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) kb[ks] = frag_f32<T>(&kv_new[0][32 * ks + 8 * qq]);
        }
        f32x4_t sc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) sc = F::mma(qa[ks], kb[ks], sc);
        // (TX: V is converted at its use and the next pass's V loads issue after it -- 32 fewer live
        // registers, so the fused launch's 4-wave occupancy holds without spills)
        float vf[4][8];
        if constexpr (!TX)
#pragma unroll
        for (int it = 0; it < 4; ++it)
#pragma unroll
            for (int c = 0; c < VL; ++c) {
                float t[16 / sizeof(T)];
                cvt16<T>(vb[it][c], t);
#pragma unroll
                for (int u = 0; u < (int)(16 / sizeof(T)); ++u) vf[it][c * (16 / sizeof(T)) + u] = t[u];
            }
        // next pass; none after the last (the fold's barrier would wait for loads nobody reads)
        if (pa + 1 < npass) {
            if constexpr (TX)
                issue_k(jb + FD_TILE);
            else
                issue(jb + FD_TILE);
        }
        if (!TX && owner) {
#pragma unroll
            for (int it = 0; it < 4; ++it)
                if (min(jb + 16 * wave + 4 * it + qq, jend - 1) == pos)
#pragma unroll
                    for (int e = 0; e < 8; ++e) vf[it][e] = kv_new[1][vd + e];
        }
        const bool kval = jk < jend && qq < g;
        {
            const float sv = kval ? sc[0] * a.scale : -INFINITY;
            const float mnew = fmaxf(m_run, row_max16(sv));
            const float alpha = mnew == -INFINITY ? 1.f : expf(m_run - mnew);
            const float p = kval ? expf(sv - mnew) : 0.f;
            m_run = mnew;
            l_run = l_run * alpha + p;
            p_s[wave][l16][qq] = p;
#pragma unroll
            for (int h = 0; h < FD_GM; ++h) {
                if (h >= g) break;
                const float ah = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(alpha), 16 * h));
#pragma unroll
                for (int e = 0; e < 8; ++e) o[h][e] *= ah;
            }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const f32x4_t pv = *reinterpret_cast<const f32x4_t*>(&p_s[wave][4 * it + qq][0]);
            float vt[8];
            if constexpr (TX) {
#pragma unroll
                for (int c = 0; c < VL; ++c) {
                    float t[16 / sizeof(T)];
                    cvt16<T>(vb[it][c], t);
#pragma unroll
                    for (int u = 0; u < (int)(16 / sizeof(T)); ++u) vt[c * (16 / sizeof(T)) + u] = t[u];
                }
                if (owner && min(jb + 16 * wave + 4 * it + qq, jend - 1) == pos)
#pragma unroll
                    for (int e = 0; e < 8; ++e) vt[e] = kv_new[1][vd + e];
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) vt[e] = vf[it][e];
            }
#pragma unroll
            for (int h = 0; h < FD_GM; ++h) {
                if (h >= g) break;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[h][e] += pv[h] * vt[e];
            }
        }
        __builtin_amdgcn_wave_barrier();  // p_s is rewritten by the next pass
        if constexpr (TX)
            if (pa + 1 < npass) issue_v(jb + FD_TILE);
    }
    FD_TS(2)
    // ---- fold the block's waves: PV partials of the 4 V position groups through LDS (no
    // cross-row shuffles), (max, sum) per wave and head
    const float lrow = row_sum16(l_run);  // row qq: head qq's sum
    if (l16 == 0 && qq < g) {
        wml[wave][qq][0] = m_run;
        wml[wave][qq][1] = lrow;
    }
#pragma unroll
    for (int h = 0; h < FD_GM; ++h) {
        if (h >= g) break;
        if constexpr (OG == 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[h][e] = sum_rows4(o[h][e], lane);
        }
        if (8 * l16 < HD && (OG == 4 || qq == 0)) {
            f32x4_t* dst = reinterpret_cast<f32x4_t*>(&ored[wave][OG == 4 ? qq : 0][h][8 * l16]);
            dst[0] = (f32x4_t){o[h][0], o[h][1], o[h][2], o[h][3]};
            dst[1] = (f32x4_t){o[h][4], o[h][5], o[h][6], o[h][7]};
        }
    }
    FD_TS(5)
    lds_barrier();  // ored / wml (the owner's K / V row stores need not have landed)
    FD_TS(3)
    const bool single = nsp == 1;
    for (int idx = threadIdx.x; idx < g * HD; idx += NT) {
        const int h = idx / HD, e = idx - h * HD;
        float M = wml[0][h][0];
#pragma unroll
        for (int w = 1; w < NW; ++w) M = fmaxf(M, wml[w][h][0]);
        float L = 0.f, O = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const float sc = expf(wml[w][h][0] - M);  // a wave with no position: exp(-inf) = 0
            L += sc * wml[w][h][1];
            if constexpr (OG == 4)
                O += sc * ((ored[w][0][h][e] + ored[w][1][h][e]) + (ored[w][2][h][e] + ored[w][3][h][e]));
            else
                O += sc * ored[w][0][h][e];
        }
        if (single) {
            if constexpr (TX)
                __hip_atomic_store(xt + (size_t)(kvh * g + h) * HD + e, ((uint32_t)f2bf(O / L) << 16) | gen,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                st(a.out + (size_t)r * a.nh * HD + (size_t)(kvh * g + h) * HD, e, O / L);
        } else {  // write-through (sc1): read back by the combining block without a fence
            float* pp = a.part + (((size_t)r * a.nh + (size_t)kvh * g + h) * a.maxsplit + sp) * (HD + 2);
            __hip_atomic_store(pp + 2 + e, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (e == 0) {
                __hip_atomic_store(pp, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(pp + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (!TX && a.dbg && threadIdx.x == 0) {
        tz[4] = __builtin_amdgcn_s_memrealtime();
        dbg_record(a.dbg, 0xFFFC, (unsigned)(nsp << 16 | (jend - j0)), tz);
    }
    if (single) return;
    // ---- split combine by the last-arriving block of (row, kv head): sc1 partial stores drained by
    // every wave, a relaxed agent ticket, sc1 loads in the combiner (MI355X_MICROARCH.md hand-off
    // table, first row; no release / acquire fence)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int t = __hip_atomic_fetch_add(a.cnt + (size_t)r * a.nkv + kvh, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        flag = t == nsp - 1;
        if (t == nsp - 1) __hip_atomic_store(a.cnt + (size_t)r * a.nkv + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!flag) return;
    FD_TS(5)
    // lane q of a 16-lane group holds split q; group grp owns PP consecutive (dim pair) items of one
    // head.  Every load is unconditional (split index clamped) and issued before any is used.
    constexpr int PP = FD_GM * HD * 8 / NT;
    const int q = l16, grp = threadIdx.x >> 4;
    const int k0 = grp * PP, h = k0 / half, e0 = 2 * (k0 - h * half);
    if (h >= g) return;  // whole 16-lane groups
    const int qc = q < nsp ? q : nsp - 1;
    const unsigned long long* pp = reinterpret_cast<const unsigned long long*>(
        a.part + (((size_t)r * a.nh + (size_t)kvh * g + h) * a.maxsplit + qc) * (HD + 2));
    const unsigned long long ml = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long ov[PP];
#pragma unroll
    for (int j = 0; j < PP; ++j) ov[j] = __hip_atomic_load(pp + 1 + e0 / 2 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float mq = q < nsp ? __uint_as_float((unsigned)ml) : -INFINITY;
    const float lq = __uint_as_float((unsigned)(ml >> 32));
    float M = mq;
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) M = fmaxf(M, __shfl_xor(M, m));
    const float w = q < nsp ? expf(mq - M) : 0.f;
    float L = w * lq;
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) L += __shfl_xor(L, m);
    T* out = a.out + (size_t)r * a.nh * HD + (size_t)(kvh * g + h) * HD + e0;
#pragma unroll
    for (int j = 0; j < PP; ++j) {
        float o0 = w * __uint_as_float((unsigned)ov[j]), o1 = w * __uint_as_float((unsigned)(ov[j] >> 32));
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) {
            o0 += __shfl_xor(o0, m);
            o1 += __shfl_xor(o1, m);
        }
        if (q == (j & 15)) {
            if constexpr (TX) {
                const uint64_t w = (uint64_t)(((uint32_t)f2bf(o0 / L) << 16) | gen) |
                                   ((uint64_t)(((uint32_t)f2bf(o1 / L) << 16) | gen) << 32);
                __hip_atomic_store(reinterpret_cast<uint64_t*>(xt + (size_t)(kvh * g + h) * HD + e0 + 2 * j), w,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                st(out, 2 * j, o0 / L);
                st(out, 2 * j + 1, o1 / L);
            }
        }
    }
    if (!TX && a.dbg && threadIdx.x == 0) {  // the combiner: {start, .., partials stored, ticket won, end}
        tz[6] = __builtin_amdgcn_s_memrealtime();
        dbg_record(a.dbg, 0xFFFB, (unsigned)nsp, tz);
    }
}

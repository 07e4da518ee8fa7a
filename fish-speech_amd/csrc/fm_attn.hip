// fm_attn.hip -- decode attention with the qk-norm / RoPE / KV-cache write fused in, and the
// radix-select sampler.
//
//   attn_fd_kernel      slow model, every batch size (the default): flash-decode splits of the
//                       context, online softmax per wave, last-arriving split combines.  The split
//                       holding `pos` normalises + ropes k (llama.py:894-910), writes k / v to the
//                       cache (llama.py:205-214) and uses them from LDS; K/V rows are read once
//                       per (row, kv head) and shared by the GQA group (no repeat_interleave,
//                       llama.py:912-913).
//   attn_decode2 / attn_dec3  the same attention for shapes attn_fd does not take (more than 4 q
//                       heads per kv head, head_dim outside {32, 64, 128}).
//   fast_attn_fused     fast model (llama.py:947-975) at codebook position cpos: same fusion,
//                       every rounding of the matmul-softmax-matmul reproduced.
//   sample_radix_kernel top-k via 4-pass radix select on order-preserving keys + rank-by-count
//                       ordering (value desc, token id asc: the order of a stable sort), then
//                       top-p / temperature / multinomial with the shared counter RNG
//                       (inference.py:43-93) and RAS (inference.py:117-144).
#include "fm_kernels.h"
#include "fm_runtime.h"
#include "fm_attn_dev.h"
#include "fm_frag.h"

// normalise (optional) + rope one head held as pairs by a wave (lane p owns pair p, p+64)
template <typename T>
__device__ __forceinline__ void head_prep(const T* src, int hd, bool norm, const T* nw, float eps,
                                          const float* tab, bool do_rope, float (&x0)[2],
                                          float (&x1)[2], int& np, int lane) {
    const int half = hd >> 1;
    np = 0;
    for (int p = lane; p < half; p += 64, ++np) {
        x0[np] = ld(src, 2 * p);
        x1[np] = ld(src, 2 * p + 1);
    }
    if (norm) {
        float ss = 0.f;
        for (int i = 0; i < np; ++i) ss += x0[i] * x0[i] + x1[i] * x1[i];
        ss = wave_sum(ss);
        const float rs = 1.0f / sqrtf(ss / (float)hd + eps);
        for (int i = 0; i < np; ++i) {
            const int p = lane + 64 * i;
            x0[i] = rnd<T>((x0[i] * rs) * ld(nw, 2 * p));
            x1[i] = rnd<T>((x1[i] * rs) * ld(nw, 2 * p + 1));
        }
    }
    if (do_rope) {
        for (int i = 0; i < np; ++i) {
            const int p = lane + 64 * i;
            const float c = tab[2 * p], s = tab[2 * p + 1];
            const float y0 = x0[i] * c - x1[i] * s;
            const float y1 = x1[i] * c + x0[i] * s;
            x0[i] = rnd<T>(y0);
            x1[i] = rnd<T>(y1);
        }
    }
}

// Slow-model decode attention for the small-batch path.  grid (R, nkv, maxs), 512 threads.
// One block normally covers ALL of a row's cached positions for one kv head (up to `cap` rows,
// sized by the host to the LDS budget: 256 at hd 128 bf16), so the common case writes the bf16
// output directly.  Longer contexts split into ceil(npos / cap) blocks whose (m, l, o) partials
// are combined by the last-arriving block (agent-scope release/acquire ticket,
// cdna_hip_programming.md §6 Guideline 16).  Round trips: (slot, pos, raw q/k/v, norm weights)
// then (K/V rows, rope row), all loads issued together; the split owning `pos` normalises/ropes
// the new k and writes k/v to the cache (llama.py:894-914).
template <typename T>
__global__ __launch_bounds__(512) void attn_decode2_kernel(AttnDecArgs<T> a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long tz[7] = {0, 0, 0, 0, 0, 0, 0};
    DBG_TS(tz, 0)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = blockIdx.x, kvh = blockIdx.y, sp = blockIdx.z;
    const int hd = a.hd, g = a.nh / a.nkv, ks = hd + 8, cap = a.cap;
    const int half = hd >> 1;
    const T* raw = a.qkv + (size_t)r * a.ldqkv;
    // ---- round trip 1: everything that does not depend on pos
    const int slot = a.row_slot[r];
    const int pos = a.row_pos[r];
    float q0[2][2], q1[2][2];  // this wave's q heads (wave, wave + 8), pairs lane, lane + 64
    for (int i = 0; i < 2; ++i) {
        const int hh = wave + 8 * i;
        for (int u = 0; u < 2; ++u) {
            const int p = lane + 64 * u;
            const bool ok = hh < g && p < half;
            const T* src = raw + (size_t)(kvh * g + (ok ? hh : 0)) * hd;
            q0[i][u] = ok ? ld(src, 2 * p) : 0.f;
            q1[i][u] = ok ? ld(src, 2 * p + 1) : 0.f;
        }
    }
    const int kvw = wave >= 6;  // waves 6 / 7: new k / v
    float k0[2] = {0.f, 0.f}, k1[2] = {0.f, 0.f};
    if (kvw) {
        const T* src = raw + (size_t)(wave == 6 ? a.nh + kvh : a.nh + a.nkv + kvh) * hd;
        for (int u = 0; u < 2; ++u) {
            const int p = lane + 64 * u;
            if (p < half) {
                k0[u] = ld(src, 2 * p);
                k1[u] = ld(src, 2 * p + 1);
            }
        }
    }
    const int npos = pos + 1;
    const int nsp = (npos + cap - 1) / cap;
    const int chunk = ((npos + nsp - 1) / nsp + 15) & ~15;
    const int j0 = sp * chunk;
    if (sp >= nsp) return;
    const int nj = min(chunk, npos - j0);
    const bool owner = j0 + nj == npos;
    T* Ks = reinterpret_cast<T*>(smem);                  // [cap][hd+8]
    T* Vs = Ks + (size_t)cap * ks;                       // [cap][hd]
    float* qs = reinterpret_cast<float*>(Vs + (size_t)cap * hd);  // [g][hd]
    float* ps = qs + (size_t)g * hd;                     // [g][cap]
    int* flag = reinterpret_cast<int*>(ps + (size_t)g * cap);
    const size_t base = (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * hd;
    T* kc = a.kc + base;
    T* vc = a.vc + base;
    const float* tab = a.rope + (size_t)pos * hd;
    // ---- round trip 2: the block's cached K/V rows (up to 16 x 16 B per thread in flight)
    {
        const int cpr = hd * (int)sizeof(T) / 16;
        const int total = nj * cpr * 2;
        for (int b0 = 0; b0 < total; b0 += 512 * 16) {
            u32x4_t v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int idx = b0 + threadIdx.x + 512 * u;
                if (idx < total) {
                    const int which = idx >= nj * cpr;
                    const int rem = idx - which * nj * cpr;
                    const int j = rem / cpr, c = rem - j * cpr;
                    const T* src = (which ? vc : kc) + (size_t)(j0 + j) * hd;
                    v[u] = *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const char*>(src) + 16 * c);
                }
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int idx = b0 + threadIdx.x + 512 * u;
                if (idx < total) {
                    const int which = idx >= nj * cpr;
                    const int rem = idx - which * nj * cpr;
                    const int j = rem / cpr, c = rem - j * cpr;
                    if (j0 + j == pos) continue;  // the new row comes from waves 6 / 7
                    T* dst = which ? Vs + (size_t)j * hd : Ks + (size_t)j * ks;
                    *reinterpret_cast<u32x4_t*>(reinterpret_cast<char*>(dst) + 16 * c) = v[u];
                }
            }
        }
    }
    DBG_TS(tz, 1)
    // q heads: qk-norm (fp32 incl. weight, one rounding) + RoPE (bf16 table, rounded)
    for (int i = 0; i < 2; ++i) {
        const int hh = wave + 8 * i;
        if (hh >= g) break;
        if (a.qk_norm) {
            float ss = 0.f;
            for (int u = 0; u < 2; ++u) ss += q0[i][u] * q0[i][u] + q1[i][u] * q1[i][u];
            ss = wave_sum(ss);
            const float rs = 1.0f / sqrtf(ss / (float)hd + a.eps);
            for (int u = 0; u < 2; ++u) {
                const int p = lane + 64 * u;
                if (p < half) {
                    q0[i][u] = rnd<T>((q0[i][u] * rs) * ld(a.qn, 2 * p));
                    q1[i][u] = rnd<T>((q1[i][u] * rs) * ld(a.qn, 2 * p + 1));
                }
            }
        }
        for (int u = 0; u < 2; ++u) {
            const int p = lane + 64 * u;
            if (p < half) {
                const float c = tab[2 * p], sn = tab[2 * p + 1];
                qs[hh * hd + 2 * p] = rnd<T>(q0[i][u] * c - q1[i][u] * sn);
                qs[hh * hd + 2 * p + 1] = rnd<T>(q1[i][u] * c + q0[i][u] * sn);
                if (a.qdbg && sp == 0) {  // per-op test hook only
                    float* qd = a.qdbg + ((size_t)r * a.nh + kvh * g + hh) * hd;
                    qd[2 * p] = qs[hh * hd + 2 * p];
                    qd[2 * p + 1] = qs[hh * hd + 2 * p + 1];
                }
            }
        }
    }
    if (kvw && owner) {
        const bool isk = wave == 6;
        if (isk && a.qk_norm) {
            float ss = 0.f;
            for (int u = 0; u < 2; ++u) ss += k0[u] * k0[u] + k1[u] * k1[u];
            ss = wave_sum(ss);
            const float rs = 1.0f / sqrtf(ss / (float)hd + a.eps);
            for (int u = 0; u < 2; ++u) {
                const int p = lane + 64 * u;
                if (p < half) {
                    k0[u] = rnd<T>((k0[u] * rs) * ld(a.kn, 2 * p));
                    k1[u] = rnd<T>((k1[u] * rs) * ld(a.kn, 2 * p + 1));
                }
            }
        }
        T* dst = (isk ? kc : vc) + (size_t)pos * hd;
        T* tile = isk ? Ks + (size_t)(pos - j0) * ks : Vs + (size_t)(pos - j0) * hd;
        for (int u = 0; u < 2; ++u) {
            const int p = lane + 64 * u;
            if (p >= half) break;
            float y0 = k0[u], y1 = k1[u];
            if (isk) {
                const float c = tab[2 * p], sn = tab[2 * p + 1];
                y0 = rnd<T>(k0[u] * c - k1[u] * sn);
                y1 = rnd<T>(k1[u] * c + k0[u] * sn);
            }
            st(dst, 2 * p, y0);
            st(dst, 2 * p + 1, y1);
            st(tile, 2 * p, y0);
            st(tile, 2 * p + 1, y1);
        }
    }
    __syncthreads();
    DBG_TS(tz, 2)
    // ---- scores: item (head, row); a wave's 64 items share one head
    const int rp = (nj + 63) & ~63;
    const float scale = a.scale;
    for (int idx = threadIdx.x; idx < g * rp; idx += 512) {
        const int hh = idx / rp, j = idx - hh * rp;
        if (j < nj) {
            const T* kr = Ks + (size_t)j * ks;
            const float* qv = qs + hh * hd;
            float dot = 0.f;
            for (int e = 0; e < hd; e += 8) {
                float kv[8];
                load8(kr + e, kv);
#pragma unroll
                for (int u = 0; u < 8; ++u) dot += qv[e + u] * kv[u];
            }
            ps[hh * cap + j] = dot * scale;
        }
    }
    __syncthreads();
    DBG_TS(tz, 3)
    // ---- softmax per head (wave per head): p = exp(s - m), l = sum p
    float mh[2], lh[2];
    for (int i = 0; i < 2; ++i) {
        const int hh = wave + 8 * i;
        mh[i] = -INFINITY;
        lh[i] = 0.f;
        if (hh >= g) continue;
        float* pr = ps + hh * cap;
        float mx = -INFINITY;
        for (int j = lane; j < nj; j += 64) mx = fmaxf(mx, pr[j]);
        mx = wave_max(mx);
        float sum = 0.f;
        for (int j = lane; j < nj; j += 64) {
            const float p = expf(pr[j] - mx);
            pr[j] = p;
            sum += p;
        }
        mh[i] = mx;
        lh[i] = wave_sum(sum);
    }
    if (lane == 0)
        for (int i = 0; i < 2; ++i)
            if (wave + 8 * i < g) {
                reinterpret_cast<float*>(flag + 4)[2 * (wave + 8 * i)] = mh[i];
                reinterpret_cast<float*>(flag + 4)[2 * (wave + 8 * i) + 1] = lh[i];
            }
    __syncthreads();
    DBG_TS(tz, 4)
    // ---- PV: item (head, dim pair); two threads per item split the rows (even / odd)
    const int hp = hd >> 1;
    const float* ml = reinterpret_cast<const float*>(flag + 4);
    const bool single = nsp == 1;
    float* part = a.part + (((size_t)r * a.nh + (size_t)kvh * g) * a.maxsplit + sp) * (hd + 2);
    for (int idx = threadIdx.x; idx < g * hp * 2; idx += 512) {
        const int it = idx >> 1, par = idx & 1;
        const int hh = it / hp, e2 = 2 * (it - hh * hp);
        const float* pr = ps + hh * cap;
        float o0 = 0.f, o1 = 0.f;
        for (int j = par; j < nj; j += 2) {
            const float p = pr[j];
            o0 += p * ld(Vs + (size_t)j * hd, e2);
            o1 += p * ld(Vs + (size_t)j * hd, e2 + 1);
        }
        o0 += __shfl_xor(o0, 1);
        o1 += __shfl_xor(o1, 1);
        if (par == 0) {
            if (single) {
                const float il = 1.0f / ml[2 * hh + 1];
                T* out = a.out + (size_t)r * a.nh * hd + (size_t)(kvh * g + hh) * hd;
                st(out, e2, o0 * il);
                st(out, e2 + 1, o1 * il);
            } else {
                // write-through (sc1): the combining block reads them back without a fence
                float* pp = part + (size_t)hh * a.maxsplit * (hd + 2);
                __hip_atomic_store(pp + 2 + e2, o0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(pp + 3 + e2, o1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (e2 == 0) {
                    __hip_atomic_store(pp, ml[2 * hh], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(pp + 1, ml[2 * hh + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
    DBG_TS(tz, 5)
    if (a.dbg && threadIdx.x == 0) {
        tz[6] = __builtin_amdgcn_s_memrealtime();
        dbg_record(a.dbg, 0xFFFD, (unsigned)(nsp << 16 | nj), tz);
    }
    if (single) return;
    // ---- split combine by the last-arriving block of (row, kv head): every wave drains its sc1
    // partial stores, one lane takes a relaxed agent ticket, the last arriver reads the partials
    // with sc1 loads (the write-through hand-off, MI355X_MICROARCH.md; no release / acquire fence)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int t = __hip_atomic_fetch_add(a.cnt + (size_t)r * a.nkv + kvh, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = t == nsp - 1;
        if (t == nsp - 1) __hip_atomic_store(a.cnt + (size_t)r * a.nkv + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!flag[0]) return;
    auto ldp = [](const float* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    const float* p0 = a.part + (((size_t)r * a.nh + (size_t)kvh * g) * a.maxsplit) * (hd + 2);
    for (int idx = threadIdx.x; idx < g * hd; idx += 512) {
        const int hh = idx / hd, e = idx - hh * hd;
        const float* pp = p0 + (size_t)hh * a.maxsplit * (hd + 2);
        float M = -INFINITY;
        for (int q = 0; q < nsp; ++q) M = fmaxf(M, ldp(pp + (size_t)q * (hd + 2)));
        float L = 0.f, O = 0.f;
        for (int q = 0; q < nsp; ++q) {
            const float w = expf(ldp(pp + (size_t)q * (hd + 2)) - M);
            L += w * ldp(pp + (size_t)q * (hd + 2) + 1);
            O += w * ldp(pp + (size_t)q * (hd + 2) + 2 + e);
        }
        st(a.out + (size_t)r * a.nh * hd + (size_t)(kvh * g + hh) * hd, e, O / L);
    }
}

// Slow-model decode attention, v3: grid (R, nkv, maxsplit), 256 threads, ATT3_CH = 64 cached
// positions per block (16 per wave), registers instead of LDS tiles for K / V.
//   round trip 1: slot, pos and the raw q / k / v rows;
//   round trip 2: every lane's K slice (one position, a quarter of hd) and V slice (four
//   positions, eight dims), all loads issued together before the q-side arithmetic;
//   scores: quarter dot products summed across the four 16-lane groups (two xor shuffles);
//   softmax per head over the block's positions (wave per head); PV accumulated in registers per
//   lane, summed across the 16-lane groups and the four waves.
// The split holding `pos` normalises + ropes the new k (llama.py:894-910), writes k / v to the
// cache (llama.py:205-214) and uses them in place of the cache rows it loaded.  One split writes
// the output; several write (m, l, o) partials and the last-arriving one combines them (agent
// release / acquire ticket, as attn_decode2).
constexpr int ATT3_CH = 64;
template <typename T>
__global__ __launch_bounds__(256) void attn_dec3_kernel(AttnDecArgs<T> a) {
    __shared__ float q_s[8][128];        // g <= 8 q heads, hd <= 128, fp32 (T-rounded values)
    __shared__ float kv_new[2][128];     // the new position's k (normed, roped) and v
    __shared__ float ps[8][ATT3_CH];     // scores, then probabilities
    __shared__ float mls[8][2];          // per head (max, sum)
    __shared__ float ored[4][8][128];    // per-wave PV partials
    __shared__ int flag;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = blockIdx.x, kvh = blockIdx.y, sp = blockIdx.z;
    const int hd = a.hd, g = a.nh / a.nkv, half = hd >> 1;
    const int slot = a.row_slot[r];
    const int pos = a.row_pos[r];
    const int npos = pos + 1;
    const int nsp = (npos + ATT3_CH - 1) / ATT3_CH;
    if (sp >= nsp) return;
    const int j0 = sp * ATT3_CH, nj = min(ATT3_CH, npos - j0);
    const bool owner = j0 + nj == npos;
    const T* raw = a.qkv + (size_t)r * a.ldqkv;
    // ---- round trip 1 (raw rows of this wave's items: q heads, then new k, new v) -----------
    float x0[2][2], x1[2][2];
    const int nitem = g + 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int it = wave + 4 * i;
        const int row = it < g ? kvh * g + it : (it == g ? a.nh + kvh : a.nh + a.nkv + kvh);
        const T* src = raw + (size_t)(it < nitem ? row : 0) * hd;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int p = lane + 64 * u;
            const bool ok = it < nitem && p < half;
            x0[i][u] = ok ? ld(src, 2 * p) : 0.f;
            x1[i][u] = ok ? ld(src, 2 * p + 1) : 0.f;
        }
    }
    // ---- round trip 2: K slice (position j0 + 16 w + (lane & 15), dims quarter lane >> 4) and
    // V slices (positions j0 + 16 w + 4 it + (lane >> 4), dims 8 (lane & 15) .. + 8)
    const size_t base = (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * hd;
    T* kc = a.kc + base;
    T* vc = a.vc + base;
    const int qd = hd >> 2;                       // dims per quarter (<= 32)
    const int jk = j0 + 16 * wave + (lane & 15);  // this lane's score position
    const int qq = lane >> 4;
    float kreg[32];
    {
        const T* krow = kc + (size_t)(jk < npos ? jk : npos - 1) * hd + qq * qd;
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (8 * c < qd) load8(krow + 8 * c, *reinterpret_cast<float(*)[8]>(kreg + 8 * c));
    }
    float vreg[4][8];
    const int vd = 8 * (lane & 15);
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int jv = j0 + 16 * wave + 4 * it + (lane >> 4);
        const T* vrow = vc + (size_t)(jv < npos ? jv : npos - 1) * hd + (vd < hd ? vd : 0);
        load8(vrow, vreg[it]);
    }
    const float* tab = a.rope + (size_t)pos * hd;
    // ---- q heads (+ new k / v in the owner): qk-norm (fp32 incl. weight, one rounding), RoPE
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int it = wave + 4 * i;
        if (it >= nitem || (it >= g && !owner)) continue;
        const bool isq = it < g, isk = it == g;
        if (a.qk_norm && (isq || isk)) {
            float ss = 0.f;
            for (int u = 0; u < 2; ++u) ss += x0[i][u] * x0[i][u] + x1[i][u] * x1[i][u];
            ss = wave_sum(ss);
            const float rs = 1.0f / sqrtf(ss / (float)hd + a.eps);
            const T* nw = isq ? a.qn : a.kn;
            for (int u = 0; u < 2; ++u) {
                const int p = lane + 64 * u;
                if (p < half) {
                    x0[i][u] = rnd<T>((x0[i][u] * rs) * ld(nw, 2 * p));
                    x1[i][u] = rnd<T>((x1[i][u] * rs) * ld(nw, 2 * p + 1));
                }
            }
        }
        for (int u = 0; u < 2; ++u) {
            const int p = lane + 64 * u;
            if (p >= half) break;
            float y0 = x0[i][u], y1 = x1[i][u];
            if (isq || isk) {
                const float c = tab[2 * p], sn = tab[2 * p + 1];
                y0 = rnd<T>(x0[i][u] * c - x1[i][u] * sn);
                y1 = rnd<T>(x1[i][u] * c + x0[i][u] * sn);
            }
            if (isq) {
                q_s[it][2 * p] = y0;
                q_s[it][2 * p + 1] = y1;
                if (a.qdbg && sp == 0) {  // per-op test hook only
                    float* qdp = a.qdbg + ((size_t)r * a.nh + kvh * g + it) * hd;
                    qdp[2 * p] = y0;
                    qdp[2 * p + 1] = y1;
                }
            } else {
                kv_new[isk ? 0 : 1][2 * p] = y0;
                kv_new[isk ? 0 : 1][2 * p + 1] = y1;
                T* dst = (isk ? kc : vc) + (size_t)pos * hd;
                st(dst, 2 * p, y0);
                st(dst, 2 * p + 1, y1);
            }
        }
    }
    __syncthreads();
    // ---- scores: the new row comes from kv_new, not the cache rows loaded before it was written
    if (owner && jk == pos) {
#pragma unroll
        for (int c = 0; c < 32; ++c)
            if (c < qd) kreg[c] = kv_new[0][qq * qd + c];
    }
    for (int h = 0; h < g; ++h) {
        float d = 0.f;
#pragma unroll
        for (int c = 0; c < 32; ++c)
            if (c < qd) d += q_s[h][qq * qd + c] * kreg[c];
        d += __shfl_xor(d, 16);
        d += __shfl_xor(d, 32);
        if (qq == 0) ps[h][16 * wave + (lane & 15)] = jk < npos ? d * a.scale : -INFINITY;
    }
    __syncthreads();
    // ---- softmax over the block's positions, wave per head
    for (int h = wave; h < g; h += 4) {
        const float sc = ps[h][lane];
        const float mx = wave_max(sc);
        const float pe = lane < nj ? expf(sc - mx) : 0.f;
        ps[h][lane] = pe;
        const float l = wave_sum(pe);
        if (lane == 0) {
            mls[h][0] = mx;
            mls[h][1] = l;
        }
    }
    __syncthreads();
    // ---- PV: this lane's four V rows x eight dims, every head
    if (owner) {
#pragma unroll
        for (int it = 0; it < 4; ++it)
            if (j0 + 16 * wave + 4 * it + (lane >> 4) == pos)
#pragma unroll
                for (int e = 0; e < 8; ++e) vreg[it][e] = vd + e < hd ? kv_new[1][vd + e] : 0.f;
    }
    for (int h = 0; h < g; ++h) {
        float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const float p = ps[h][16 * wave + 4 * it + (lane >> 4)];
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] += p * vreg[it][e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            o[e] += __shfl_xor(o[e], 16);
            o[e] += __shfl_xor(o[e], 32);
        }
        if (lane < 16 && vd < hd)
#pragma unroll
            for (int e = 0; e < 8; ++e) ored[wave][h][vd + e] = o[e];
    }
    __syncthreads();
    const bool single = nsp == 1;
    float* part = a.part + (((size_t)r * a.nh + (size_t)kvh * g) * a.maxsplit + sp) * (hd + 2);
    for (int idx = threadIdx.x; idx < g * hd; idx += 256) {
        const int h = idx / hd, e = idx - h * hd;
        const float o = (ored[0][h][e] + ored[1][h][e]) + (ored[2][h][e] + ored[3][h][e]);
        if (single) {
            st(a.out + (size_t)r * a.nh * hd + (size_t)(kvh * g + h) * hd, e, o / mls[h][1]);
        } else {  // write-through (sc1): read back by the combining block without a fence
            float* pp = part + (size_t)h * a.maxsplit * (hd + 2);
            __hip_atomic_store(pp + 2 + e, o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (e == 0) {
                __hip_atomic_store(pp, mls[h][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(pp + 1, mls[h][1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (single) return;
    // ---- split combine by the last-arriving block of (row, kv head): sc1 partial stores drained by
    // every wave, a relaxed agent ticket, sc1 loads in the combiner (the write-through hand-off of
    // MI355X_MICROARCH.md, no release / acquire fence)
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
    const float* p0 = a.part + (((size_t)r * a.nh + (size_t)kvh * g) * a.maxsplit) * (hd + 2);
    auto ldp = [](const float* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    for (int idx = threadIdx.x; idx < g * hd; idx += 256) {
        const int h = idx / hd, e = idx - h * hd;
        const float* pp = p0 + (size_t)h * a.maxsplit * (hd + 2);
        float M = -INFINITY;
        for (int q = 0; q < nsp; ++q) M = fmaxf(M, ldp(pp + (size_t)q * (hd + 2)));
        float L = 0.f, O = 0.f;
        for (int q = 0; q < nsp; ++q) {
            const float w = expf(ldp(pp + (size_t)q * (hd + 2)) - M);
            L += w * ldp(pp + (size_t)q * (hd + 2) + 1);
            O += w * ldp(pp + (size_t)q * (hd + 2) + 2 + e);
        }
        st(a.out + (size_t)r * a.nh * hd + (size_t)(kvh * g + h) * hd, e, O / L);
    }
}

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
template <typename T, int HD, int NW>
__global__ __launch_bounds__(NW * 64) void attn_fd_kernel(AttnDecArgs<T> a) {
    static_assert(HD % 32 == 0 && HD <= 128, "head_dim a multiple of 32 up to 128");
    constexpr int NT = NW * 64, FD_TILE = 16 * NW;
    constexpr int VL = 8 * (int)sizeof(T) / 16;     // 16-B loads per V slice
    constexpr int half = HD / 2;
    __shared__ __attribute__((aligned(16))) float q_s[FD_GM][HD];
    __shared__ __attribute__((aligned(16))) float kv_new[2][HD];
    __shared__ __attribute__((aligned(16))) float wml[NW][FD_GM][2];
    // PV partials [wave][V position group][head][dim]; 16 waves fold the 4 groups by shuffles first
    constexpr int OG = NW > 4 ? 1 : 4;
    __shared__ __attribute__((aligned(16))) float ored[NW][OG][FD_GM][HD];
    __shared__ int flag;
    unsigned long long tz[7] = {0, 0, 0, 0, 0, 0, 0};
    DBG_TS(tz, 0)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l16 = lane & 15, qq = lane >> 4;
    const int r = blockIdx.x, kvh = blockIdx.y, sp = blockIdx.z;
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
        raw_pair<T>(a.qkv, a.ldqkv, a.qslab, a.qslab_kp, gridDim.x, a.qbias, r,
                    (size_t)(it < nitem ? row : 0) * HD + 2 * (lane < half ? lane : 0), v0, v1);
        x0[i] = ok ? v0 : 0.f;
        x1[i] = ok ? v1 : 0.f;
    }
    const int npos = pos + 1;
    int nsp = min((int)gridDim.z, (npos + a.cap - 1) / a.cap);
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
    auto issue = [&](int jb) {
        const int jk = min(jb + 16 * wave + l16, jend - 1);
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) kb[ks] = F::load(kc + (size_t)jk * HD + 32 * ks + 8 * qq);
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int jv = min(jb + 16 * wave + 4 * it + qq, jend - 1);
            const u32x4_t* pv = reinterpret_cast<const u32x4_t*>(vc + (size_t)jv * HD + vd);
#pragma unroll
            for (int c = 0; c < VL; ++c) vb[it][c] = pv[c];
        }
    };
    // the RoPE row of pos goes out ahead of pass 0's K / V (vmcnt retires in order: the q-side
    // arithmetic waits for these two floats only, not for the pass's loads)
    const float* tab = a.rope + (size_t)pos * HD;
    const float2 rcs = *reinterpret_cast<const float2*>(tab + 2 * (lane < half ? lane : 0));
    issue(j0);
    // ---- q heads (+ new k / v in the owner): qk-norm (fp32 incl. weight, one rounding), RoPE
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
                const float c = rcs.x, sn = rcs.y;
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
    DBG_TS(tz, 1)
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
        float vf[4][8];
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
        if (pa + 1 < npass) issue(jb + FD_TILE);
        if (owner) {
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
#pragma unroll
            for (int h = 0; h < FD_GM; ++h) {
                if (h >= g) break;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[h][e] += pv[h] * vf[it][e];
            }
        }
        __builtin_amdgcn_wave_barrier();  // p_s is rewritten by the next pass
    }
    DBG_TS(tz, 2)
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
    DBG_TS(tz, 5)
    lds_barrier();  // ored / wml (the owner's K / V row stores need not have landed)
    DBG_TS(tz, 3)
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
    if (a.dbg && threadIdx.x == 0) {
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
    DBG_TS(tz, 5)
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
            st(out, 2 * j, o0 / L);
            st(out, 2 * j + 1, o1 / L);
        }
    }
    if (a.dbg && threadIdx.x == 0) {  // the combiner: {start, .., partials stored, ticket won, end}
        tz[6] = __builtin_amdgcn_s_memrealtime();
        dbg_record(a.dbg, 0xFFFB, (unsigned)nsp, tz);
    }
}

// Fast-model attention at codebook position cpos: grid (R, nh), one wave per q head (body in
// fm_attn_dev.h, shared with the QKV GEMV's fused tail).  Two round trips: (slot, raw q/k/v,
// norm weights, rope row) then (the cpos cached rows).
template <typename T>
__global__ __launch_bounds__(64) void fast_attn2_kernel(FastFusedArgs<T> a) {
    unsigned long long tz[7] = {0, 0, 0, 0, 0, 0, 0};
    DBG_TS(tz, 0)
    fast_attn_head<T>(a, blockIdx.x, blockIdx.y, threadIdx.x, tz);
    if (a.dbg && threadIdx.x == 0) {
        tz[4] = __builtin_amdgcn_s_memrealtime();
        dbg_record(a.dbg, 0xFFFE, (unsigned)a.cpos, tz);
    }
}

// fast model attention at codebook position cpos, fused with qk-norm/rope/cache write.
// grid (R, nkv), block 256 (wave per q head of the GQA group).
template <typename T>
__global__ __launch_bounds__(256) void fast_attn_fused_kernel(FastFusedArgs<T> a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = blockIdx.x, kvh = blockIdx.y;
    const int slot = a.row_slot[r];
    const int hd = a.hd, g = a.nh / a.nkv, C = a.S, cpos = a.cpos;
    float* Kt = reinterpret_cast<float*>(smem);  // [C][hd]
    float* Vt = Kt + (size_t)C * hd;
    float* qs = Vt + (size_t)C * hd;  // [4][hd]
    float* ps = qs + 4 * hd;          // [4][64]
    const size_t base = (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * C * hd;
    T* kc = a.kc + base;
    T* vc = a.vc + base;
    const T* raw = a.qkv + (size_t)r * a.ldqkv;
    const float* tab = a.rope + (size_t)cpos * hd;
    if (wave < 2) {
        float x0[2], x1[2];
        int np;
        const int hk = wave == 0 ? a.nh + kvh : a.nh + a.nkv + kvh;
        head_prep<T>(raw + (size_t)hk * hd, hd, wave == 0 && a.qk_norm, a.kn, a.eps, tab, wave == 0, x0,
                     x1, np, lane);
        T* dst = (wave == 0 ? kc : vc) + (size_t)cpos * hd;
        float* tile = (wave == 0 ? Kt : Vt) + (size_t)cpos * hd;
        for (int i = 0; i < np; ++i) {
            const int p = lane + 64 * i;
            st(dst, 2 * p, x0[i]);
            st(dst, 2 * p + 1, x1[i]);
            tile[2 * p] = x0[i];
            tile[2 * p + 1] = x1[i];
        }
    }
    for (int idx = threadIdx.x; idx < cpos * hd; idx += 256) {
        Kt[idx] = ld(kc, idx);
        Vt[idx] = ld(vc, idx);
    }
    for (int hb = 0; hb < g; hb += 4) {
        const int ql = hb + wave;
        if (ql < g) {
            float x0[2], x1[2];
            int np;
            head_prep<T>(raw + (size_t)(kvh * g + ql) * hd, hd, a.qk_norm, a.qn, a.eps, tab, true, x0,
                         x1, np, lane);
            for (int i = 0; i < np; ++i) {
                const int p = lane + 64 * i;
                qs[wave * hd + 2 * p] = x0[i];
                qs[wave * hd + 2 * p + 1] = x1[i];
            }
        }
        __syncthreads();
        if (ql < g) {
            float sc = -INFINITY;
            if (lane <= cpos) {
                float dot = 0.f;
                for (int e = 0; e < hd; ++e) dot += qs[wave * hd + e] * Kt[(size_t)lane * hd + e];
                sc = rnd<T>(rnd<T>(dot) * a.scale);
            }
            const float mx = wave_max(sc);
            const float ex = lane <= cpos ? expf(sc - mx) : 0.f;
            const float den = wave_sum(ex);
            ps[wave * 64 + lane] = rnd<T>(ex / den);
            __builtin_amdgcn_wave_barrier();
            const int h = kvh * g + ql;
            for (int e = lane; e < hd; e += 64) {
                float o = 0.f;
                for (int j = 0; j <= cpos; ++j) o += ps[wave * 64 + j] * Vt[(size_t)j * hd + e];
                st(a.out, (size_t)r * a.nh * hd + (size_t)h * hd + e, o);
            }
        }
        __syncthreads();
    }
}

// =========================================================================================
// sampler: radix-select top-K
// =========================================================================================
__device__ __forceinline__ uint32_t fkey(float v) {
    const uint32_t u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ bool cbetter(float v, int id, float bv, int bid) {
    return v > bv || (v == bv && id < bid);
}

template <typename T>
__device__ int sample_top(const float* cv, const int* cid, int K, float M, float den, float temperature,
                          float top_p, int top_k, uint64_t seed, uint64_t step, uint32_t draw, int lane) {
    const float v = lane < K ? cv[lane] : -INFINITY;
    const int id = lane < K ? cid[lane] : 0x7fffffff;
    const float p = (v == -INFINITY) ? 0.f : rnd<T>(expf(v - M) / den);
    // the reference's cumsum in rank order: lane k's value read as a scalar (k is uniform), so each
    // step is a readlane + add instead of an LDS-routed shuffle
    float cum = 0.f, mycum = 0.f;
    for (int k = 0; k < K; ++k) {
        cum += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), k));
        if (lane == k) mycum = rnd<T>(cum);
    }
    const float t = rnd<T>(temperature), tp = rnd<T>(top_p);
    const bool keep = lane < K && v != -INFINITY && (lane == 0 || (!(mycum > tp) && lane < top_k));
    const float tt = fmaxf(t, 1e-5f);
    const float lt = keep ? rnd<T>(v / tt) : -INFINITY;
    const float m2 = wave_max(lt);
    const float e = keep ? expf(lt - m2) : 0.f;
    const float d2 = wave_sum(e);
    const float prob = rnd<T>(e / d2);
    float score = -1.f;
    int bid = 0x7fffffff;
    if (keep) {
        const float u = rng_uniform_bf16(seed, step, draw, (uint32_t)id);
        const float qv = rnd<T>(-logf(u));
        score = rnd<T>(prob / qv);
        bid = id;
    }
    // argmax of (score desc, id asc): the wave maximum by DPP, then the smallest id among the lanes
    // holding it (one lane but for exact ties), read as scalars
    const float best = wave_max(score);
    uint64_t hit = __ballot(score == best);
    int tok = 0x7fffffff;
    while (hit) {
        const int l = __ffsll((long long)hit) - 1;
        tok = min(tok, __builtin_amdgcn_readlane(bid, l));
        hit &= hit - 1;
    }
    return tok;
}

// ---- top_k > 64 (the reference's logits_to_probs takes any top_k, inference.py:54-77) ----------
// The row's (key << 32 | ~id) words are sorted descending in LDS by a block bitonic sort (P, a power
// of two >= Nl; padding 0 never ranks), so rank r is the reference's r-th entry of the stable
// descending sort.  Thread 0 runs the reference's cumsum in rank order and finds the kept prefix
// (rank 0, then ranks < top_k whose rounded cumulative probability stays <= top_p); the draw
// argmax(prob / q) over it is a block reduction.  One sort serves both RAS draws.
__device__ __forceinline__ float sw_val(uint64_t k) {
    const uint32_t u = (uint32_t)(k >> 32);
    return __uint_as_float(u & 0x80000000u ? (u & 0x7fffffffu) : ~u);
}
__device__ __forceinline__ int sw_id(uint64_t k) { return (int)~(uint32_t)k; }
__host__ __device__ __forceinline__ int sw_pow2(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

// keys[0, P): filled by the caller (all threads), this sorts them, better first
__device__ void sw_sort(uint64_t* keys, int P) {
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t x = keys[i], y = keys[ixj];
                    const bool desc = (i & k) == 0;
                    if (desc ? (x < y) : (x > y)) {
                        keys[i] = y;
                        keys[ixj] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// one draw over the sorted keys; every thread of the block calls it, every thread gets the token
template <typename T>
__device__ int sw_draw(const uint64_t* keys, int Nl, float M, float den, float temperature, float top_p,
                       int top_k, uint64_t seed, uint64_t step, uint32_t draw, int* sh_i, float* sh_f) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (threadIdx.x == 0) {
        const float tp = rnd<T>(top_p);
        const int lim = top_k < Nl ? top_k : Nl;
        float cum = 0.f;
        int nk = 1;
        for (int r = 0; r < lim; ++r) {
            const float v = sw_val(keys[r]);
            if (v == -INFINITY) break;  // zero probability: never drawn (sample_top's keep)
            cum += rnd<T>(expf(v - M) / den);
            if (r > 0 && rnd<T>(cum) > tp) break;
            nk = r + 1;
        }
        sh_i[0] = nk;
    }
    __syncthreads();
    const int nk = sh_i[0];
    const float tt = fmaxf(rnd<T>(temperature), 1e-5f);
    const float m2 = rnd<T>(sw_val(keys[0]) / tt);  // rank 0 holds the largest scaled logit
    float e = 0.f;
    for (int r = threadIdx.x; r < nk; r += blockDim.x) e += expf(rnd<T>(sw_val(keys[r]) / tt) - m2);
    e = wave_sum(e);
    __syncthreads();
    if (lane == 0) sh_f[wave] = e;
    __syncthreads();
    float d2 = 0.f;
    for (int w = 0; w < nw; ++w) d2 += sh_f[w];
    float best = -1.f;
    int bid = 0x7fffffff;
    for (int r = threadIdx.x; r < nk; r += blockDim.x) {
        const float v = sw_val(keys[r]);
        const int id = sw_id(keys[r]);
        const float prob = rnd<T>(expf(rnd<T>(v / tt) - m2) / d2);
        const float u = rng_uniform_bf16(seed, step, draw, (uint32_t)id);
        const float score = rnd<T>(prob / rnd<T>(-logf(u)));
        if (cbetter(score, id, best, bid)) {
            best = score;
            bid = id;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float os = __shfl_xor(best, o, 64);
        const int oid = __shfl_xor(bid, o, 64);
        if (cbetter(os, oid, best, bid)) {
            best = os;
            bid = oid;
        }
    }
    __syncthreads();
    if (lane == 0) {
        sh_f[wave] = best;
        sh_i[1 + wave] = bid;
    }
    __syncthreads();
    float bb = sh_f[0];
    int bi = sh_i[1];
    for (int w = 1; w < nw; ++w)
        if (cbetter(sh_f[w], sh_i[1 + w], bb, bi)) {
            bb = sh_f[w];
            bi = sh_i[1 + w];
        }
    __syncthreads();
    return bi;
}

// the wide path of both samplers: sort, draw (twice with RAS on the slow head), emit the column
template <typename T>
__device__ void sample_wide(const SampleArgs& a, const SlotParams& sp, int r, int slot, uint64_t* keys, int P,
                            float M, float den) {
    __shared__ int sh_i[1 + 16];
    __shared__ float sh_f[16];
    sw_sort(keys, P);
    const uint64_t step = (uint64_t)sp.step;
    int32_t* col = a.cols + (size_t)r * a.ldc;
    if (a.slow) {
        int tok = sw_draw<T>(keys, a.Nl, M, den, sp.temperature, sp.top_p, sp.top_k, sp.seed, step, 0, sh_i, sh_f);
        const int hi = sw_draw<T>(keys, a.Nl, M, den, 1.0f, 0.9f, sp.top_k, sp.seed, step, 1, sh_i, sh_f);
        if (threadIdx.x != 0) return;
        if (a.ras_enable) {
            const int32_t* prev = a.ras + (size_t)slot * a.ras_stride;
            bool inwin = false;
            for (int j = 0; j < 10; ++j) inwin |= prev[j] == tok;
            if (inwin && tok >= a.sb && tok <= a.se) tok = hi;
        }
        if (!((tok >= a.sb && tok <= a.se) || tok == a.im_end)) tok = a.im_end;
        int c = tok - a.sb;
        c = c < 0 ? 0 : (c > a.cb - 1 ? a.cb - 1 : c);
        if (sp.force) {
            tok = a.force_cols[(size_t)slot * a.ldc];
            c = a.force_cols[(size_t)slot * a.ldc + 1];
        }
        col[0] = tok;
        col[1] = c;
    } else {
        const int code = sw_draw<T>(keys, a.Nl, M, den, sp.temperature, sp.top_p, sp.top_k, sp.seed, step,
                                    (uint32_t)a.draw, sh_i, sh_f);
        if (threadIdx.x == 0)
            col[a.col_idx] = sp.force ? a.force_cols[(size_t)slot * a.ldc + a.col_idx]
                                      : ((code >= 0 && code < a.cb) ? code : 0);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void sample_radix_kernel(SampleArgs a) {
    extern __shared__ __attribute__((aligned(16))) float vals[];  // [Nl]; [P] u64 keys (top_k > 64)
    __shared__ float scratch[16];
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sh_prefix, sh_rem, sh_nstrict, sh_ntie;
    __shared__ float cv[64];
    __shared__ int cid[64];
    __shared__ float sv[64];
    __shared__ int sid[64];
    __shared__ int tid_[256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = blockIdx.x;
    const int slot = a.row_slot[r];
    const SlotParams sp = a.sp[slot];
    const float* lg = a.logits + (size_t)r * a.ldl;
    const int Nl = a.Nl;
    if (sp.force)  // teacher forcing: the logits row as the production graph produced it
        for (int i = threadIdx.x; i < Nl; i += 256) a.tap[(size_t)slot * a.tap_ld + i] = lg[i];
    for (int i = threadIdx.x; i < Nl; i += 256) {
        float v = lg[i];
        if (a.slow && sp.mask_im_end && i == Nl - 1) v = -INFINITY;
        vals[i] = v;
    }
    __syncthreads();
    auto tok_of = [&](int i) { return a.slow ? (i < Nl - 1 ? a.sb + i : a.im_end) : i; };
    float mloc = -INFINITY;
    for (int i = threadIdx.x; i < Nl; i += 256) mloc = fmaxf(mloc, vals[i]);
    const float M = block_max(mloc, scratch);
    float sloc = 0.f;
    for (int i = threadIdx.x; i < Nl; i += 256) sloc += (vals[i] == -INFINITY) ? 0.f : expf(vals[i] - M);
    const float den = block_sum(sloc, scratch);
    if (sp.top_k > 64) {  // block-uniform
        const int P = sw_pow2(Nl);
        uint64_t* keys = reinterpret_cast<uint64_t*>(vals);  // vals are re-read from the row
        __syncthreads();
        for (int i = threadIdx.x; i < P; i += 256) {
            float v = i < Nl ? lg[i] : -INFINITY;
            if (a.slow && sp.mask_im_end && i == Nl - 1) v = -INFINITY;
            keys[i] = i < Nl ? (((uint64_t)fkey(v) << 32) | (uint32_t)~(uint32_t)tok_of(i)) : 0ull;
        }
        sample_wide<T>(a, sp, r, slot, keys, P, M, den);
        return;
    }
    int K = sp.top_k < 1 ? 1 : (sp.top_k > 64 ? 64 : sp.top_k);
    if (K > Nl) K = Nl;

    // ---- radix select: key of the K-th largest element ------------------------------------
    uint32_t prefix = 0, mask = 0, rem = (uint32_t)K;
    for (int shift = 24; shift >= 0; shift -= 8) {
        hist[threadIdx.x] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < Nl; i += 256) {
            const uint32_t k = fkey(vals[i]);
            if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (wave == 0) {
            uint32_t c[4];
            uint32_t s = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                c[q] = hist[255 - 4 * lane - q];
                s += c[q];
            }
            uint32_t incl = s;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(incl, o, 64);
                if (lane >= o) incl += t;
            }
            const uint64_t hit = __ballot(incl >= rem);
            const int L = hit ? __ffsll((long long)hit) - 1 : 63;
            if (lane == L) {
                uint32_t run = incl - s;
                int bin = 255 - 4 * lane - 3;
                uint32_t nrem = rem - run;
                for (int q = 0; q < 4; ++q) {
                    if (run + c[q] >= rem) {
                        bin = 255 - 4 * lane - q;
                        nrem = rem - run;
                        break;
                    }
                    run += c[q];
                }
                sh_prefix = prefix | ((uint32_t)bin << shift);
                sh_rem = nrem;
            }
        }
        __syncthreads();
        prefix = sh_prefix;
        rem = sh_rem;
        mask |= 255u << shift;
    }
    const uint32_t thr = prefix;  // key of the K-th element; take `rem` of the ties
    // ---- gather strict (> thr) and tie (== thr) candidates ----------------------------------
    if (threadIdx.x == 0) {
        sh_nstrict = 0;
        sh_ntie = 0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < Nl; i += 256) {
        const uint32_t k = fkey(vals[i]);
        if (k > thr) {
            const uint32_t at = atomicAdd(&sh_nstrict, 1u);
            if (at < 64) {
                sv[at] = vals[i];
                sid[at] = tok_of(i);
            }
        } else if (k == thr) {
            const uint32_t at = atomicAdd(&sh_ntie, 1u);
            if (at < 256) tid_[at] = tok_of(i);
        }
    }
    __syncthreads();
    if (wave == 0) {
        const int ns = (int)sh_nstrict;  // == K - rem
        const int nt = (int)sh_ntie;
        // strict: rank by counting -> sorted (value desc, id asc)
        if (lane < ns) {
            int rk = 0;
            for (int j = 0; j < ns; ++j) rk += cbetter(sv[j], sid[j], sv[lane], sid[lane]);
            cv[rk] = sv[lane];
            cid[rk] = sid[lane];
        }
        // ties: the `rem` smallest token ids
        float tv = 0.f;
        {
            uint32_t u = thr & 0x80000000u ? (thr & 0x7fffffffu) : ~thr;
            tv = __uint_as_float(u);
        }
        if (nt <= 256) {
            for (int t = lane; t < nt; t += 64) {
                int rk = 0;
                for (int j = 0; j < nt; ++j) rk += tid_[j] < tid_[t];
                if (rk < (int)rem) {
                    cv[ns + rk] = tv;
                    cid[ns + rk] = tid_[t];
                }
            }
        } else if (lane == 0) {  // massive ties (degenerate logits): exact sequential scan by id
            int taken = 0;
            int last = -1;
            while (taken < (int)rem) {
                int best = 0x7fffffff;
                for (int i = 0; i < Nl; ++i) {
                    const int id = tok_of(i);
                    if (fkey(vals[i]) == thr && id > last && id < best) best = id;
                }
                cv[ns + taken] = tv;
                cid[ns + taken] = best;
                last = best;
                ++taken;
            }
        }
        __builtin_amdgcn_wave_barrier();
        const uint64_t step = (uint64_t)sp.step;
        int32_t* col = a.cols + (size_t)r * a.ldc;
        if (a.slow) {
            int tok = sample_top<T>(cv, cid, K, M, den, sp.temperature, sp.top_p, sp.top_k, sp.seed, step,
                                    0, lane);
            const int hi = sample_top<T>(cv, cid, K, M, den, 1.0f, 0.9f, sp.top_k, sp.seed, step, 1, lane);
            if (a.ras_enable) {
                const int32_t* prev = a.ras + (size_t)slot * a.ras_stride;
                bool inwin = false;
                for (int j = 0; j < 10; ++j) inwin |= prev[j] == tok;
                if (inwin && tok >= a.sb && tok <= a.se) tok = hi;
            }
            // never emit an out-of-range id (NaN logits leave no valid candidate): end the stream
            if (!((tok >= a.sb && tok <= a.se) || tok == a.im_end)) tok = a.im_end;
            if (lane == 0) {
                int c = tok - a.sb;
                c = c < 0 ? 0 : (c > a.cb - 1 ? a.cb - 1 : c);
                if (sp.force) {
                    tok = a.force_cols[(size_t)slot * a.ldc];
                    c = a.force_cols[(size_t)slot * a.ldc + 1];
                }
                col[0] = tok;
                col[1] = c;
            }
        } else {
            const int code = sample_top<T>(cv, cid, K, M, den, sp.temperature, sp.top_p, sp.top_k, sp.seed,
                                           step, (uint32_t)a.draw, lane);
            if (lane == 0)
                col[a.col_idx] = sp.force ? a.force_cols[(size_t)slot * a.ldc + a.col_idx]
                                          : ((code >= 0 && code < a.cb) ? code : 0);
        }
    }
}

// Two-stage top-K select (K <= 64) for the decode sampler: per-wave binary radix search for the
// wave's K-th largest key (register-resident values, wave reductions only), block threshold =
// max of the wave thresholds (every global top-K element is >= it, and each wave's elements
// >= it are among that wave's candidates), candidates >= threshold through LDS, then an exact
// select on <= 4*CAP candidates by wave 0.  Degenerate ties (more than CAP candidates in a wave)
// take an exact full scan by wave 0.  Same output order as sample_radix_kernel: value desc,
// token id asc, ties at the K-th value by smallest id.
constexpr int SF_PER = 17;   // values per thread: Nl <= 256 * 17 = 4352 (4097 slow, 4096 fast)
constexpr int SF_CAP = 64;   // candidates kept per wave

// wave total and exclusive lane prefix of a small per-lane count (< 2^B) by bit-plane ballots:
// B scalar popcounts instead of a cross-lane shuffle tree
template <int B>
__device__ __forceinline__ uint32_t sf_wave_count(uint32_t c, uint32_t* excl) {
    uint32_t tot = 0, pre = 0;
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const uint64_t m = __ballot((c >> b) & 1u);
        tot += (uint32_t)__popcll(m) << b;
        if (excl) pre += (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
    }
    if (excl) *excl = pre;
    return tot;
}
constexpr int sf_bits(int n) { return n < 2 ? 1 : 1 + sf_bits(n >> 1); }

template <int N>
__device__ __forceinline__ uint32_t sf_radix_kth(const uint32_t (&k)[N], uint32_t K, uint32_t kmax, uint32_t cap) {
    // a threshold t with K <= #{key >= t} <= cap over the wave's N keys per lane (the exact K-th
    // largest key when ties leave no such t).  Binary search on the key bits; each step counts
    // per lane on the VALU and totals the wave by bit-plane ballots.  Bits that would lift t
    // above the wave maximum `kmax` are skipped (count 0), and the search stops as soon as the
    // count fits in `cap`.
    uint32_t t = 0;
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t c = t | (1u << bit);
        if (c > kmax) continue;
        uint32_t cl = 0;
#pragma unroll
        for (int i = 0; i < N; ++i) cl += k[i] >= c ? 1u : 0u;
        const uint32_t cnt = sf_wave_count<sf_bits(N)>(cl, nullptr);
        if (cnt >= K) {
            t = c;
            if (cnt <= cap) break;
        }
    }
    return t;
}

// wave-wide bitonic sort of one (value, id) per lane into "better first" order (value desc,
// id asc); padding lanes carry (-inf, INT_MAX)
__device__ __forceinline__ void sf_bitonic(float& v, int& id, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const float ov = __shfl_xor(v, j, 64);
            const int oi = __shfl_xor(id, j, 64);
            const bool lower = (lane & j) == 0, dir = (lane & k) == 0;
            const bool other_better = cbetter(ov, oi, v, id);
            if ((lower == dir) == other_better) {
                v = ov;
                id = oi;
            }
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void sample_fast_kernel(SampleArgs a) {
    unsigned long long tsx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define SFTS(n) if (a.dbg) tsx[n] = __builtin_amdgcn_s_memrealtime();
    SFTS(0)
    extern __shared__ __attribute__((aligned(16))) float vals[];  // [Nl] fallback; [P] u64 keys (top_k > 64)
    __shared__ float redm[4], reds[4];
    __shared__ uint32_t wthr[4];
    __shared__ uint32_t ncand[4];
    __shared__ __align__(16) float2 cand[4 * SF_CAP];  // (value, token id bits)
    __shared__ __align__(16) uint64_t ckey[4 * SF_CAP];  // (key << 32 | ~id): larger = better
    __shared__ float cv[64];
    __shared__ int cid[64];
    __shared__ int overflow;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = blockIdx.x;
    const int slot = a.row_slot[r];
    const SlotParams sp = a.sp[slot];
    const float* lg = a.logits + (size_t)r * a.ldl;
    const int Nl = a.Nl;
    if (sp.force)  // teacher forcing: the logits row as the production graph produced it
        for (int i = threadIdx.x; i < Nl; i += 256) a.tap[(size_t)slot * a.tap_ld + i] = lg[i];
    auto tok_of = [&](int i) { return a.slow ? (i < Nl - 1 ? a.sb + i : a.im_end) : i; };
    // this thread's values: indices threadIdx.x + 256 * i (coalesced loads, all in flight)
    float v[SF_PER];
    uint32_t key[SF_PER];
#pragma unroll
    for (int i = 0; i < SF_PER; ++i) {
        const int idx = threadIdx.x + 256 * i;
        float x = idx < Nl ? lg[idx < Nl ? idx : 0] : -INFINITY;
        if (a.slow && sp.mask_im_end && idx == Nl - 1) x = -INFINITY;
        v[i] = x;
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int i = 0; i < SF_PER; ++i) {
        mloc = fmaxf(mloc, v[i]);
        key[i] = threadIdx.x + 256 * i < Nl ? fkey(v[i]) : 0u;  // padding never qualifies
    }
    SFTS(1)
    mloc = wave_max(mloc);
    if (lane == 0) redm[wave] = mloc;
    if (threadIdx.x == 0) overflow = 0;
    // per-wave K-th largest key (the wave holds 64 * SF_PER slots; padding is -inf -> key 0x007fffff)
    int K = sp.top_k < 1 ? 1 : (sp.top_k > 64 ? 64 : sp.top_k);
    if (K > Nl) K = Nl;
    SFTS(2)
    // fast threshold: the K-th largest of the 64 lane maxima t0 has at least K wave keys >= it (the
    // K lanes' maxima), so it is a valid wave threshold whenever those keys fit the candidate cap
    // (else the radix search below)
    uint32_t kth;
    {
        uint32_t lm = 0;
#pragma unroll
        for (int i = 0; i < SF_PER; ++i) lm = key[i] > lm ? key[i] : lm;
        // the K-th largest lane maximum by a binary search on its bits: one ballot + popcount per
        // bit (scalar work) instead of a 21-step shuffle sort of the 64 maxima
        uint32_t t0 = 0;
        for (int bit = 31; bit >= 0; --bit) {
            const uint32_t c = t0 | (1u << bit);
            if ((uint32_t)__popcll(__ballot(lm >= c)) >= (uint32_t)K) t0 = c;
        }
        uint32_t cl = 0;
#pragma unroll
        for (int i = 0; i < SF_PER; ++i) cl += key[i] >= t0 ? 1u : 0u;
        const uint32_t cnt = sf_wave_count<sf_bits(SF_PER)>(cl, nullptr);
        kth = (a.kth_fast && t0 != 0u && cnt >= (uint32_t)K && cnt <= (uint32_t)SF_CAP)
                  ? t0
                  : sf_radix_kth<SF_PER>(key, (uint32_t)K, fkey(mloc), (uint32_t)SF_CAP);
    }
    SFTS(3)
    if (lane == 0) wthr[wave] = kth;
    __syncthreads();
    const float M = fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3]));
    const uint32_t thrT = max(max(wthr[0], wthr[1]), max(wthr[2], wthr[3]));
    float sloc = 0.f;
#pragma unroll
    for (int i = 0; i < SF_PER; ++i) sloc += (v[i] == -INFINITY) ? 0.f : expf(v[i] - M);
    sloc = wave_sum(sloc);
    if (lane == 0) reds[wave] = sloc;
    // candidates >= thrT of this wave -> LDS (order: lane-major, stable)
    uint32_t mine = 0;
#pragma unroll
    for (int i = 0; i < SF_PER; ++i) mine += (key[i] >= thrT && key[i] != 0u) ? 1u : 0u;
    uint32_t excl;
    const uint32_t tot = sf_wave_count<sf_bits(SF_PER)>(mine, &excl);
    if (tot > (uint32_t)SF_CAP) {
        if (lane == 0) overflow = 1;
    } else {
        uint32_t at = excl;
#pragma unroll
        for (int i = 0; i < SF_PER; ++i) {
            if (key[i] >= thrT && key[i] != 0u) {
                const int id = tok_of(threadIdx.x + 256 * i);
                cand[wave * SF_CAP + at] = make_float2(v[i], __int_as_float(id));
                ckey[wave * SF_CAP + at] = ((uint64_t)key[i] << 32) | (uint32_t)~(uint32_t)id;
                ++at;
            }
        }
        // pad the wave's list to a multiple of 8 with entries that never rank above anything
        if (lane >= (int)tot && lane < (int)((tot + 7u) & ~7u))
            ckey[wave * SF_CAP + lane] = 0ull;
    }
    if (lane == 0) ncand[wave] = tot;
    __syncthreads();
    SFTS(4)
    const float den = reds[0] + reds[1] + reds[2] + reds[3];
    if (sp.top_k > 64) {  // block-uniform: the wide path over the whole row (sorted in LDS)
        const int P = sw_pow2(Nl);
        uint64_t* keys = reinterpret_cast<uint64_t*>(vals);
#pragma unroll
        for (int i = 0; i < SF_PER; ++i) {
            const int idx = threadIdx.x + 256 * i;
            if (idx < Nl) keys[idx] = ((uint64_t)fkey(v[i]) << 32) | (uint32_t)~(uint32_t)tok_of(idx);
        }
        for (int i = Nl + threadIdx.x; i < P; i += 256) keys[i] = 0ull;
        sample_wide<T>(a, sp, r, slot, keys, P, M, den);
        return;
    }
    if (overflow) {  // degenerate ties: park everything in LDS for the exact scan below
#pragma unroll
        for (int i = 0; i < SF_PER; ++i) {
            const int idx = threadIdx.x + 256 * i;
            if (idx < Nl) vals[idx] = v[i];
        }
    } else {
        // exact ranks by counting: candidate j's rank is the number of candidates better than it
        // (value desc, id asc -- a total order, ids are unique), so the K best land sorted in cv/cid
        const int n0 = ncand[0], n1 = ncand[1], n2 = ncand[2], n3 = ncand[3];
        const int j = threadIdx.x, nc = n0 + n1 + n2 + n3;
        if (j < nc) {
            const int w = j < n0 ? 0 : (j < n0 + n1 ? 1 : (j < n0 + n1 + n2 ? 2 : 3));
            const int o = j - (w == 0 ? 0 : (w == 1 ? n0 : (w == 2 ? n0 + n1 : n0 + n1 + n2)));
            const float2 me = cand[w * SF_CAP + o];
            const int mid = __float_as_int(me.y);
            int rank = 0;
            const int nw[4] = {n0, n1, n2, n3};
            const uint64_t mk = ckey[w * SF_CAP + o];
#pragma unroll
            for (int w2 = 0; w2 < 4; ++w2) {
                const ulonglong2* cp = reinterpret_cast<const ulonglong2*>(ckey + w2 * SF_CAP);
                const int nq = ((nw[w2] + 7) & ~7) >> 1;  // 16 bytes = two keys
                for (int q = 0; q < nq; q += 4) {  // four independent 16-byte LDS reads per step
                    const ulonglong2 c0 = cp[q], c1 = cp[q + 1], c2 = cp[q + 2], c3 = cp[q + 3];
                    rank += (c0.x > mk) + (c0.y > mk) + (c1.x > mk) + (c1.y > mk) + (c2.x > mk) +
                            (c2.y > mk) + (c3.x > mk) + (c3.y > mk);
                }
            }
            if (rank < K) {
                cv[rank] = me.x;
                cid[rank] = mid;
            }
        }
    }
    __syncthreads();
    if (wave != 0) return;
    // ---- wave 0: sample over the K best (exact full scan first on overflow) ------------------
    int ns = 0;        // strict (> K-th value) count
    uint32_t thr = 0;  // key of the K-th element
    uint32_t rem = 0;  // how many of the K-th value's ties to take
    if (overflow) {
        // exact full scan of vals[] by one wave (rare: massive ties)
        thr = 0;
        for (int bit = 31; bit >= 0; --bit) {
            const uint32_t c = thr | (1u << bit);
            uint32_t cnt = 0;
            for (int i = lane; i < Nl; i += 64) cnt += fkey(vals[i]) >= c ? 1u : 0u;
            cnt = (uint32_t)wave_sum((float)cnt);
            if (cnt >= (uint32_t)K) thr = c;
        }
        uint32_t gt = 0;
        for (int i = lane; i < Nl; i += 64) gt += fkey(vals[i]) > thr ? 1u : 0u;
        ns = (int)wave_sum((float)gt);
        rem = (uint32_t)(K - ns);
        if (lane == 0) {  // strict ones (< 64 of them) by selection, then the smallest tie ids
            int taken = 0;
            float lastv = INFINITY;
            int lasti = -1;
            while (taken < ns) {
                float bv = -INFINITY;
                int bi = 0x7fffffff;
                for (int i = 0; i < Nl; ++i) {
                    const float x = vals[i];
                    const int id = tok_of(i);
                    if (fkey(x) > thr && cbetter(lastv, lasti, x, id) && cbetter(x, id, bv, bi)) {
                        bv = x;
                        bi = id;
                    }
                }
                cv[taken] = bv;
                cid[taken] = bi;
                lastv = bv;
                lasti = bi;
                ++taken;
            }
            int last = -1;
            for (uint32_t t2 = 0; t2 < rem; ++t2) {
                int best = 0x7fffffff;
                float bv = 0.f;
                for (int i = 0; i < Nl; ++i) {
                    const int id = tok_of(i);
                    if (fkey(vals[i]) == thr && id > last && id < best) {
                        best = id;
                        bv = vals[i];
                    }
                }
                cv[ns + t2] = bv;
                cid[ns + t2] = best;
                last = best;
            }
        }
    }
    (void)ns;
    (void)rem;
    __builtin_amdgcn_wave_barrier();
    SFTS(5)
    const uint64_t step = (uint64_t)sp.step;
    int32_t* col = a.cols + (size_t)r * a.ldc;
    // developer stamps {start, values in, max, threshold, candidates, ranks, end} (wave 0, at the end)
    auto record = [&]() {
        if (a.dbg && lane == 0) {
            tsx[6] = __builtin_amdgcn_s_memrealtime();
            const unsigned long long slot2 = atomicAdd(a.dbg, 1ull);
            if (slot2 < (1ull << 20)) {
                unsigned long long* q = a.dbg + 8 + slot2 * 8;
                q[0] = (0xFFFFull << 32) | (unsigned)(ncand[0] + ncand[1] + ncand[2] + ncand[3]) |
                       ((unsigned long long)overflow << 16) | ((unsigned long long)a.slow << 17);
                for (int z = 0; z < 7; ++z) q[1 + z] = tsx[z];
            }
        }
    };
    if (a.slow) {
        int tok = sample_top<T>(cv, cid, K, M, den, sp.temperature, sp.top_p, sp.top_k, sp.seed, step, 0, lane);
        const int hi = sample_top<T>(cv, cid, K, M, den, 1.0f, 0.9f, sp.top_k, sp.seed, step, 1, lane);
        if (a.ras_enable) {
            const int32_t* prev = a.ras + (size_t)slot * a.ras_stride;
            bool inwin = false;
            for (int j = 0; j < 10; ++j) inwin |= prev[j] == tok;
            if (inwin && tok >= a.sb && tok <= a.se) tok = hi;
        }
        if (!((tok >= a.sb && tok <= a.se) || tok == a.im_end)) tok = a.im_end;
        if (lane == 0) {
            int c = tok - a.sb;
            c = c < 0 ? 0 : (c > a.cb - 1 ? a.cb - 1 : c);
            if (sp.force) {
                tok = a.force_cols[(size_t)slot * a.ldc];
                c = a.force_cols[(size_t)slot * a.ldc + 1];
            }
            col[0] = tok;
            col[1] = c;
        }
    } else {
        const int code = sample_top<T>(cv, cid, K, M, den, sp.temperature, sp.top_p, sp.top_k, sp.seed, step,
                                       (uint32_t)a.draw, lane);
        if (lane == 0)
            col[a.col_idx] = sp.force ? a.force_cols[(size_t)slot * a.ldc + a.col_idx]
                                      : ((code >= 0 && code < a.cb) ? code : 0);
    }
    record();
}

// ---------------------------------------------------------------------------------------
template <typename T> void launch_attn_decode2(hipStream_t s, const AttnDecArgs<T>& a, int R) {
    dim3 g1(R, a.nkv, a.maxsplit);
    static bool attr = false;  // > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU)
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_decode2_kernel<T>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    attn_decode2_kernel<T><<<g1, 512, attn2_lds_bytes(a.hd, a.nh / a.nkv, a.cap, sizeof(T)), s>>>(a);
}
template <typename T> void launch_attn_fd(hipStream_t s, const AttnDecArgs<T>& a0, int R) {
    FMCHECK(attn_fd_ok(a0.hd, a0.nh / a0.nkv), "attn_fd: head_dim 32, 64 or 128 and at most 4 q heads per kv head");
    FMCHECK(a0.cap >= 16 && a0.cnt && a0.part && a0.out, "attn_fd: min split >= 16, tickets, partials and output set");
    AttnDecArgs<T> a = a0;
    a.maxsplit = std::min(FD_NSP, FM_CEIL(a.S, a.cap));
    const dim3 grid(R, a.nkv, a.maxsplit);
    if (a.nwb == 16) {
        switch (a.hd) {
            case 32: attn_fd_kernel<T, 32, 16><<<grid, 1024, 0, s>>>(a); break;
            case 64: attn_fd_kernel<T, 64, 16><<<grid, 1024, 0, s>>>(a); break;
            default: attn_fd_kernel<T, 128, 16><<<grid, 1024, 0, s>>>(a); break;
        }
        return;
    }
    if (a.nwb == 8) {
        switch (a.hd) {
            case 32: attn_fd_kernel<T, 32, 8><<<grid, 512, 0, s>>>(a); break;
            case 64: attn_fd_kernel<T, 64, 8><<<grid, 512, 0, s>>>(a); break;
            default: attn_fd_kernel<T, 128, 8><<<grid, 512, 0, s>>>(a); break;
        }
        return;
    }
    switch (a.hd) {
        case 32: attn_fd_kernel<T, 32, 4><<<grid, 256, 0, s>>>(a); break;
        case 64: attn_fd_kernel<T, 64, 4><<<grid, 256, 0, s>>>(a); break;
        default: attn_fd_kernel<T, 128, 4><<<grid, 256, 0, s>>>(a); break;
    }
}
template <typename T> void launch_attn_decode3(hipStream_t s, const AttnDecArgs<T>& a0, int R) {
    FMCHECK(a0.hd % 32 == 0 && a0.hd <= 128 && a0.nh % a0.nkv == 0 && a0.nh / a0.nkv <= 6,
            "attn_dec3: hd a multiple of 32 up to 128, at most 6 q heads per kv head");
    AttnDecArgs<T> a = a0;
    a.maxsplit = FM_CEIL(a.S, ATT3_CH);
    attn_dec3_kernel<T><<<dim3(R, a.nkv, a.maxsplit), 256, 0, s>>>(a);
}
template <typename T> void launch_fast_attn2(hipStream_t s, const FastFusedArgs<T>& a, int R) {
    fast_attn2_kernel<T><<<dim3(R, a.nh), 64, 0, s>>>(a);
}
template <typename T> void launch_fast_attn_fused(hipStream_t s, const FastFusedArgs<T>& a, int R) {
    dim3 g(R, a.nkv);
    const size_t lds = (size_t)2 * a.S * a.hd * 4 + (size_t)4 * a.hd * 4 + 4 * 64 * 4;
    fast_attn_fused_kernel<T><<<g, 256, lds, s>>>(a);
}
template <typename T> void launch_sample_radix(hipStream_t s, const SampleArgs& a, int R) {
    // dynamic LDS: the row's values, or the sorted keys of the top_k > 64 path (top_k lives on the
    // device, per slot, so every launch reserves the larger); the kernels' attributes allow up to
    // 160 KiB (sample_init, run at model finalize outside any capture)
    const size_t lds = std::max(sizeof(float) * a.Nl, sizeof(uint64_t) * (size_t)sw_pow2(a.Nl));
    FMCHECK(lds + 8 * 1024 <= 160 * 1024, "sampler: vocabulary too wide for the LDS row");
    if (a.Nl <= 256 * SF_PER && fm_tuning().sampler_fast) {
        SampleArgs b = a;
        b.kth_fast = fm_tuning().sampler_kth;
        sample_fast_kernel<T><<<R, 256, lds, s>>>(b);
    } else {
        sample_radix_kernel<T><<<R, 256, lds, s>>>(a);
    }
}
template void launch_attn_decode2<bf16_t>(hipStream_t, const AttnDecArgs<bf16_t>&, int);
template void launch_attn_decode2<float>(hipStream_t, const AttnDecArgs<float>&, int);
template void launch_attn_fd<bf16_t>(hipStream_t, const AttnDecArgs<bf16_t>&, int);
template void launch_attn_fd<float>(hipStream_t, const AttnDecArgs<float>&, int);
template void launch_attn_decode3<bf16_t>(hipStream_t, const AttnDecArgs<bf16_t>&, int);
template void launch_attn_decode3<float>(hipStream_t, const AttnDecArgs<float>&, int);
template void launch_fast_attn2<bf16_t>(hipStream_t, const FastFusedArgs<bf16_t>&, int);
template void launch_fast_attn2<float>(hipStream_t, const FastFusedArgs<float>&, int);
template void launch_fast_attn_fused<bf16_t>(hipStream_t, const FastFusedArgs<bf16_t>&, int);
template void launch_fast_attn_fused<float>(hipStream_t, const FastFusedArgs<float>&, int);
void sample_init() {
    const void* k[] = {reinterpret_cast<const void*>(&sample_fast_kernel<bf16_t>),
                       reinterpret_cast<const void*>(&sample_radix_kernel<bf16_t>),
                       reinterpret_cast<const void*>(&sample_fast_kernel<float>),
                       reinterpret_cast<const void*>(&sample_radix_kernel<float>)};
    for (const void* f : k) HIPCHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
}
template void launch_sample_radix<bf16_t>(hipStream_t, const SampleArgs&, int);
template void launch_sample_radix<float>(hipStream_t, const SampleArgs&, int);

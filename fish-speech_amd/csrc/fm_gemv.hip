// fm_gemv.hip -- the decode-step weight-streaming kernel for R <= 8 rows (streams per GPU).
//
// Y[r][n] = sum_k X'[r][k] W[n][k] with the producer/consumer seams of a pre-norm block fused:
//   prologue  PRO_PLAIN   X' = X
//             PRO_NORM    X' = rmsnorm(X)                       (llama.py:989-1000)
//             PRO_PRENORM X' = rmsnorm(X) where X is an already finalised residual row and the
//                         statistic comes from the producer's per-tile sums of squares
//   epilogue  EPI_STORE (T, +bias) | EPI_SWIGLU (round(silu(round(w1 x)))*round(w3 x))
//             | EPI_F32 (logits) | EPI_SLAB (fp32 split-K partial)
//             | EPI_SLABFIN (split-K partial; the tile's last-arriving block finalises
//               x = round(res + round(sum partials)) (llama.py:841-842) and its sum of squares)
//
// Geometry: block = 8 waves, 16 weight rows (one 16x16x32 MFMA row tile; the R<=8 streams are
// MFMA columns), grid = (N/16, KSB).  Weights are pre-packed in MFMA-fragment order
// (fm_kernels.h), so a fragment is 1 KiB of contiguous HBM; wave w owns a contiguous run of the
// block's k-steps and streams them through a ring of U register fragments (predicated tail).
// A decode GEMV gives each wave only 4-16 fragments, so latency rules: the prologue's loads go
// out first (one round trip: x slice, norm weight, tile sums of squares), then the weight ring,
// then the LDS staging, which therefore overlaps the weight flight.
#include "fm_kernels.h"
#include "fm_runtime.h"
#include "fm_attn_dev.h"
#include "fm_frag.h"

__device__ __forceinline__ float silu_g(float a) { return a / (1.0f + expf(-a)); }

// 8 consecutive elements of T as raw 16-byte vectors (bf16: one, fp32: two)
template <typename T> struct C8 {
    u32x4_t v[sizeof(T) / 2];
};
template <typename T> __device__ __forceinline__ C8<T> load_c8(const T* p) {
    C8<T> c;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 2); ++i) c.v[i] = reinterpret_cast<const u32x4_t*>(p)[i];
    return c;
}
template <typename T> __device__ __forceinline__ void c8_to_f(const C8<T>& c, float (&o)[8]) {
    if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o[2 * i] = __uint_as_float(c.v[0][i] << 16);
            o[2 * i + 1] = __uint_as_float(c.v[0][i] & 0xffff0000u);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o[i] = __uint_as_float(c.v[0][i]);
            o[4 + i] = __uint_as_float(c.v[1][i]);
        }
    }
}

constexpr int GEMV_RMAX = 8;  // rows (streams) of the small-batch path
constexpr int GEMV_PRE = 8;   // (row, chunk) items of X preloaded per thread before the weight ring
// occupancy target (waves per SIMD) of the tiled GEMV: the interleaved W1||W3 grid (1216 blocks of
// 4 waves) is resident at 5; the others need 3 (enough for their grids)
constexpr int gemv_wpe(int pro, int epi) { return pro == PRO_PRENORM && epi == EPI_SWIGLU8 ? 5 : (pro == PRO_FATT ? 1 : 3); }

// WPB waves per block share one 16-row tile, each streaming a contiguous run of its k-steps.
// QM 1 (weight-only int8): the weight stream is a.Wq, one ring slot = one 64-k unit (1 KiB per wave,
// as a T fragment is), dequantised exactly to two T fragments in registers; each output is
// round(round(acc) * wscale[row]) (WeightOnlyInt8Linear.forward, quantize.py:228-229).
// QM 2 (weight-only int4, bf16): one ring slot = one 128-k unit of 4-bit codes (1 KiB per wave) plus
// the (scale, zero) of that unit's group for the lane's four accumulator rows (a.wsz, group size a
// multiple of 128).  No per-weight dequantisation: each code becomes the exact bf16 128 + q by one
// mask-and-or per pair (0x4300 | q), the unit's four MFMAs give B = sum x (128 + q) per (row, x row),
// and the unit adds s * B + (z - 136 s) * X_u, X_u = sum x over the unit (staged in LDS by the
// prologue) -- the group's affine map sum x ((q - 8) s + z) applied exactly in fp32.
// ---- chain hand-off (one launch, stages in sequence; cdna_hip_programming.md §6 Guideline 16,
// write-through form): every byte a later stage of the launch reads is stored sc1 and drained
// (s_waitcnt vmcnt(0)) by its storing wave before the block's one arrival on a sharded counter;
// the consumer polls the counter (sc1 loads, one lane per shard), and EVERY load of handed-off
// bytes is an sc1 load (buffer_load_dwordx4 / global_load_dword sc1), so no acquire fence.
// Counter words, one 128-B line each (GEMV_CHAIN_LINE words apart): per stage s, 8 arrival shards
// (block b adds to shard b & 7), a top word that each shard's last arriver increments, and 8 done
// replicas that the top's last arriver sets.  A waiting block polls only the replica of its shard
// (the polls of a thousand waiting blocks spread over 8 lines that nothing else touches).
__device__ __forceinline__ unsigned* chain_word(unsigned* cnt, int s, int k) {
    return cnt + (s * GEMV_CHAIN_SLOTS + k) * GEMV_CHAIN_LINE;
}
struct ChainWait {
    const unsigned* done = nullptr;  // the producing stage's done replica (null: stage 0)
    int sleep = 4;                   // s_sleep between polls (1, 4 or 16)
    int* err = nullptr;              // set on a timed-out wait (host re-zeroes the counters)
};
__device__ __forceinline__ void chain_wait(const ChainWait& cw) {
    if (threadIdx.x == 0) {
        for (unsigned it = 0;; ++it) {
            if (__hip_atomic_load(cw.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
            if (it > (1u << 16)) {  // bounded (~0.1 s; a stage takes tens of us): the host sees err, resets
                __hip_atomic_store(cw.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            if (cw.sleep <= 1)
                __builtin_amdgcn_s_sleep(1);
            else if (cw.sleep <= 4)
                __builtin_amdgcn_s_sleep(4);
            else
                __builtin_amdgcn_s_sleep(16);
        }
    }
    __syncthreads();
}
// 8 elements of T at X + off (elements) as an sc1 load through a buffer descriptor of X
template <typename T> __device__ __forceinline__ C8<T> load_c8_sc1(const T* X, int nbytes, int off) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, nbytes, 0x00020000);
    C8<T> c;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 2); ++i)
        c.v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, off * (int)sizeof(T) + 16 * i, 0, 16);
    return c;
}
template <typename T> __device__ __forceinline__ float ld_sc1(const T* p, size_t i) {
    if constexpr (sizeof(T) == 2) {
        const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t*>(p + (i & ~(size_t)1)), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        return __uint_as_float((i & 1) ? (w & 0xffff0000u) : (w << 16));
    } else {
        return __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// element i of a run of consecutive lanes holding consecutive even-aligned elements, stored
// write-through: bf16 as (even, odd) pairs in one 4-byte store by the even lane.  Every lane of
// the run executes this (the odd lane's value travels by shuffle).
template <typename T> __device__ __forceinline__ void st_sc1_run(T* p, size_t i, float v) {
    if constexpr (sizeof(T) == 2) {
        const float nb = __shfl_down(v, 1);
        if ((i & 1) == 0)
            __hip_atomic_store(reinterpret_cast<uint32_t*>(p + i), (uint32_t)f2bf(v) | ((uint32_t)f2bf(nb) << 16),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        __hip_atomic_store(p + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The GEMV body for block (bxi, ks) of a grid with nks K slices.  CH (chain stage, R == 1, whole
// K per block): the weight ring goes out first, then the wait for the producing stage, then the
// prologue's loads (sc1); outputs a later stage reads are stored sc1 (the caller arrives).
template <typename T, int PRO, int EPI, bool NT, int U, int WPB, int QM, bool CH>
__device__ __forceinline__ void gemv_body(const GemvArgs<T>& a, const int bxi, const int ks, const int nks,
                                          const ChainWait& cw) {
    constexpr bool Q8 = QM == 1, Q4 = QM == 2, QQ = QM != 0;
    static_assert(!(QQ && (EPI == EPI_SWIGLU || EPI == EPI_SLAB || PRO == PRO_FATT)), "no quantized form");
    static_assert(!Q4 || sizeof(T) == 2, "int4: bf16 only");
    static_assert(!CH || (!QQ && (PRO == PRO_PLAIN || PRO == PRO_PRENORM) &&
                          (EPI == EPI_STORE || EPI == EPI_SWIGLU8 || EPI == EPI_SLABFIN || EPI == EPI_F32)),
                  "no chain form");
    // X items preloaded per thread ahead of the weight ring: PRO_PRENORM's operand is one dim-wide
    // row per stream (2 items per thread at R = 1), and its register budget is what lets the
    // 1216-block W1||W3 grid stay resident (5 waves per SIMD)
    constexpr int PRE_N = PRO == PRO_PRENORM ? 3 : GEMV_PRE;
    using G = Frag<T>;
    constexpr int NACC = (EPI == EPI_SWIGLU) ? 2 : 1;
    constexpr int NTH = WPB * 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = bxi * 16;
    const int Kb = a.K / nks;  // host guarantees a multiple of 32 (64 int8, 128 int4)
    const int kbeg = ks * Kb;
    const int R = a.R;
    const int xstride = Kb + 8;  // +16 B per row: conflict-free ds_read_b128 across rows
    T* xs = reinterpret_cast<T*>(smem);
    int* flag = reinterpret_cast<int*>(smem + (size_t)R * xstride * sizeof(T));
    float* red = reinterpret_cast<float*>(flag + 16);  // [NACC][WPB waves][16 rows][R] partials
    float* fin = red + 2 * 8 * 16 * R;                // [R][16] EPI_SLABFIN, ksb == 1
    float* rsl = fin + 16 * R;                        // [8 waves][GEMV_RMAX] PRO_PRENORM 1/rms

    const unsigned long long ts0 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    // EPI_SLABFIN: the residual element this thread will finalise, loaded in the first round trip
    // (unconditional, clamped index: a load under a branch drains vmcnt before the MFMAs)
    float res_pre = 0.f;
    auto load_res = [&]() {
        const int tt = min((int)threadIdx.x, 16 * a.R - 1);
        const int col = tt >> 4, nn = min(bxi * 16 + (tt & 15), a.N - 1);
        int ri = a.residx ? a.residx[(size_t)col * a.xidx_ld + a.xidx_col] : col;
        if (a.residx && a.xidx_rows > 0) ri = ri < 0 ? 0 : (ri >= a.xidx_rows ? a.xidx_rows - 1 : ri);
        if constexpr (CH)
            res_pre = ld_sc1(a.res + (size_t)ri * a.ldr, nn);
        else
            res_pre = ld(a.res + (size_t)ri * a.ldr, nn);
    };
    if constexpr (EPI == EPI_SLABFIN && !CH) load_res();
    // KV prefetch (GemvArgs::pf_kc): slot and pos go out with the prologue's round trip, the sector
    // loads after the weight ring (the ring never waits on them; in-order vmcnt retires them before
    // the ring's refills).  GEMV_PF 4-byte loads per thread, one per 64-B sector, unconditional and
    // clamped to a valid address when off (a load under a branch drains vmcnt before the MFMAs).
    constexpr bool PFOK = !CH && !QQ && (PRO == PRO_NORM || PRO == PRO_PRENORM) && EPI == EPI_STORE;
    constexpr int GEMV_PF = 2;
    int pf_s = 0, pf_p = 0;
    if constexpr (PFOK) {
        const int32_t* ps = a.pf_kc ? a.pf_slot : reinterpret_cast<const int32_t*>(a.X);
        const int32_t* pq = a.pf_kc ? a.pf_pos : reinterpret_cast<const int32_t*>(a.X);
        pf_s = ps[0];
        pf_p = pq[0];
    }
    float pfw[GEMV_PF];
    auto pf_issue = [&]() {
        if constexpr (PFOK) {
            const bool on = a.pf_kc != nullptr;
            const int nkv = on ? a.pf_nkv : 1;
            const int h = bxi % nkv, j = bxi / nkv, nb = ((int)gridDim.x - 1 - h) / nkv + 1;
            const int spr = on ? a.pf_hd * (int)sizeof(T) / 64 : 1;  // 64-B sectors per cached row
            const int np = on ? pf_p + 1 : 0;
            const int total = 2 * np * spr;                            // K rows, then V rows
            const size_t base = on ? (size_t)pf_s * a.pf_slot_stride + a.pf_layer_off + (size_t)h * a.pf_S * a.pf_hd : 0;
#pragma unroll
            for (int q = 0; q < GEMV_PF; ++q) {
                const int i = (j + nb * q) * (WPB * 64) + (int)threadIdx.x;
                const bool ok = i < total;
                const int ii = ok ? i : 0, row = ii / spr, sec = ii - row * spr;
                const bool isv = row >= np;
                const T* src = ok ? (isv ? a.pf_vc : a.pf_kc) + base + (size_t)(isv ? row - np : row) * a.pf_hd : a.X;
                pfw[q] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(src) + (ok ? sec * 64 : 0));
            }
        }
    };
    unsigned long long tsA = 0, tsB = 0;  // PRO_PRENORM: tile sums staged / X' written
    const int r = lane & 15, g = lane >> 4;
    constexpr int KU = Q4 ? 128 : (Q8 ? 64 : 32);  // k per ring slot
    const int S = a.K / KU, Sb = Kb / KU, sb0 = ks * Sb;
    const int wa = (wave * Sb) / WPB, wb = ((wave + 1) * Sb) / WPB, nmy = wb - wa;
    typename G::f fa[QQ ? 1 : U], fb[NACC == 2 ? U : 1];
    u32x4_t fq[QQ ? U : 1];
    u32x4_t fz[Q4 ? U : 1];  // int4: (scale, zero) of the lane's 4 accumulator rows per ring slot
    // Fragment i of the run into ring slot u.  Branch-free on purpose: a load under a branch makes
    // the compiler drain vmcnt(0) before every MFMA (no pipelining at all), so tail slots load a
    // fixed fragment (fm_tune gemv_dummy: one per (block, wave), a cache hit) instead of being
    // predicated off.
    const int ilast = nmy > 0 ? nmy - 1 : 0;
    const size_t run0 = ((size_t)bxi * S + sb0 + (nmy > 0 ? wa : 0)) * (QQ ? 1024 : 512);
    const T* wrun = QQ ? nullptr : a.W + run0;
    const T* wrun2 = (EPI == EPI_SWIGLU) ? a.W2 + run0 : nullptr;
    const unsigned char* qrun = QQ ? a.Wq + run0 : nullptr;
    const uint32_t* zrun = Q4 ? a.wsz + (run0 >> 10) * 16 + 4 * (lane >> 4) : nullptr;
    const bool dtail = a.dummy_tail != 0;
    // dummy_tail 2: the fixed fragment differs per (block, wave) over 256 fragments (no hot line)
    // (bounded by the matrix's own fragment count: ceil(N / 16) tiles x S k-steps)
    const size_t dfr = a.dummy_tail == 2 ? (size_t)((bxi * WPB + wave) & 255) % ((size_t)((a.N + 15) >> 4) * S) : 0;
    auto issue = [&](int i, int u) {
        const size_t ii = (size_t)(i < ilast ? i : ilast);
        const bool past = dtail && i > ilast;  // beyond the run: one fixed (cached) fragment
        if constexpr (QQ) {
            const u32x4_t* p = reinterpret_cast<const u32x4_t*>((past ? a.Wq + dfr * 1024 : qrun + ii * 1024) + lane * 16);
            if constexpr (NT) fq[u] = __builtin_nontemporal_load(p);
            else fq[u] = *p;
            if constexpr (Q4)
                fz[u] = *reinterpret_cast<const u32x4_t*>(past ? a.wsz + dfr * 16 + 4 * (lane >> 4) : zrun + ii * 16);
        } else {
            fa[u] = G::template load_w<NT>(past ? a.W + dfr * 512 : wrun + ii * 512, lane);
            if constexpr (NACC == 2) fb[u] = G::template load_w<NT>(past ? a.W + dfr * 512 : wrun2 + ii * 512, lane);
        }
    };

    // ---------------- prologue: X'[r][kbeg .. kbeg+Kb) -> LDS ----------------------------------
    // Round trip first: this thread's x chunks (and norm weight / tile sums of squares) are loaded
    // BEFORE the weight ring is issued, so the in-order vmcnt waits of the staging below do not
    // queue behind weight bytes.
    if constexpr (PRO == PRO_NORM) {
        // full-row statistic from the row itself (first layer: embeddings / gathered rows).  The
        // weight ring goes out first: the statistic's block reductions use LDS-only barriers, so
        // they do not wait for it
#pragma unroll
        for (int u = 0; u < U; ++u) issue(u, u);
        __shared__ float red_s[16];
        const int nch = a.K >> 3;
        const bool writer = (bxi == 0 && ks == 0);
        for (int rr = 0; rr < R; ++rr) {
            int xi = a.xidx ? a.xidx[(size_t)rr * a.xidx_ld + a.xidx_col] : rr;
            if (a.xidx_rows > 0) xi = xi < 0 ? 0 : (xi >= a.xidx_rows ? a.xidx_rows - 1 : xi);  // defence in depth
            const T* xr = a.X + (size_t)xi * a.ldx;
            float xv[4][8], wv[4][8];
            float ss = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = threadIdx.x + NTH * j;
                if (c < nch) {
                    const int k = 8 * c;
                    if ((k >= kbeg && k < kbeg + Kb) || writer) load8(a.nw + k, wv[j]);
                    load8(xr + k, xv[j]);
#pragma unroll
                    for (int u = 0; u < 8; ++u) ss += xv[j][u] * xv[j][u];
                }
            }
            ss = block_sum_lds(ss, red_s);
            const float rs = 1.0f / sqrtf(ss / (float)a.K + a.eps);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = threadIdx.x + NTH * j;
                if (c >= nch) continue;
                const int k = 8 * c;
                const bool mine = k >= kbeg && k < kbeg + Kb;
                if (!mine && !writer) continue;
                float xn[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) xn[u] = rnd<T>(rnd<T>(xv[j][u] * rs) * wv[j][u]);
                if (mine) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) st(xs, (size_t)rr * xstride + (k - kbeg) + u, xn[u]);
                }
                if (writer && a.xn_out) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) st(a.xn_out, (size_t)rr * a.ldxo + k + u, xn[u]);
                }
            }
            lds_barrier();  // red_s is reused by the next row
        }
        pf_issue();
    } else if constexpr (PRO == PRO_FATT) {
        // One row (host).  Round trip 1: slot, the raw q|k|v row, qk-norm weights, RoPE row; then
        // the weight ring; round trip 2: the cpos cached K/V rows of every kv head (they need the
        // slot).  Then wave-per-head attention from LDS straight into X' (fm_attn_dev.h).
        const FastFusedArgs<T>& at = a.att;
        const int hd = at.hd, cpos = at.cpos, nkv = at.nkv;
        T* raw_s = reinterpret_cast<T*>(smem + a.fatt_off);  // raw row | qn | kn | tab: contiguous
        T* qn_s = raw_s + at.ldqkv;
        T* kn_s = qn_s + hd;
        float* tab_s = reinterpret_cast<float*>(kn_s + hd);
        T* kv_s = reinterpret_cast<T*>(tab_s + hd);
        constexpr int CE = 16 / sizeof(T);  // elements per 16-B chunk
        const int n_raw = at.ldqkv / CE, n_w = hd / CE, n_tab = hd * 4 / 16;
        const int n1 = n_raw + 2 * n_w + n_tab;
        auto src1 = [&](int i) -> const u32x4_t* {
            if (i < n_raw) return reinterpret_cast<const u32x4_t*>(at.qkv) + i;
            i -= n_raw;
            if (i < n_w) return reinterpret_cast<const u32x4_t*>(at.qk_norm ? at.qn : at.qkv) + i;
            i -= n_w;
            if (i < n_w) return reinterpret_cast<const u32x4_t*>(at.qk_norm ? at.kn : at.qkv) + i;
            return reinterpret_cast<const u32x4_t*>(at.rope + (size_t)cpos * hd) + (i - n_w);
        };
        auto dst1 = [&](int i) -> u32x4_t* { return reinterpret_cast<u32x4_t*>(raw_s) + i; };
        constexpr int P1 = 4, P2 = 10;
        u32x4_t c1[P1];
        const int slot = at.row_slot[0];
#pragma unroll
        for (int q = 0; q < P1; ++q) {
            const int i = threadIdx.x + NTH * q;
            if (i < n1) c1[q] = *src1(i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) issue(u, u);
        const int rc = hd / CE, n2 = nkv * 2 * cpos * rc;
        const size_t cbase = (size_t)slot * at.slot_stride + at.layer_off;
        auto src2 = [&](int i) -> const u32x4_t* {
            const int row = i / rc, c = i - row * rc;
            const int kvh = row / (2 * cpos), rem = row - kvh * 2 * cpos, which = rem / cpos, j = rem - which * cpos;
            const T* base = (which ? at.vc : at.kc) + cbase + (size_t)kvh * at.S * hd + (size_t)j * hd;
            return reinterpret_cast<const u32x4_t*>(base) + c;
        };
        u32x4_t c2[P2];
#pragma unroll
        for (int q = 0; q < P2; ++q) {
            const int i = threadIdx.x + NTH * q;
            if (i < n2) c2[q] = *src2(i);
        }
#pragma unroll
        for (int q = 0; q < P1; ++q) {
            const int i = threadIdx.x + NTH * q;
            if (i < n1) *dst1(i) = c1[q];
        }
        for (int i = threadIdx.x + NTH * P1; i < n1; i += NTH) *dst1(i) = *src1(i);
#pragma unroll
        for (int q = 0; q < P2; ++q) {
            const int i = threadIdx.x + NTH * q;
            if (i < n2) reinterpret_cast<u32x4_t*>(kv_s)[i] = c2[q];
        }
        for (int i = threadIdx.x + NTH * P2; i < n2; i += NTH) reinterpret_cast<u32x4_t*>(kv_s)[i] = *src2(i);
        __syncthreads();
        const int h0 = kbeg / hd, h1 = (kbeg + Kb) / hd;
        for (int hb = h0 + 8 * wave; hb < h1; hb += 8 * WPB)
            fast_attn_heads8_lds<T>(at, hb, h1, lane, raw_s, kv_s, qn_s, kn_s, tab_s, xs + (size_t)(hb - h0) * hd,
                                    bxi == 0, slot);
    } else {
        // PRO_PLAIN / PRO_PRENORM: (row, 8-element chunk) items of the slice, up to PRE_N per
        // thread preloaded ahead of the weight ring (the rest, large R x Kb only, after it)
        const int nch = Kb >> 3, nitem = R * nch;
        const int xbytes = (R - 1) * a.ldx * (int)sizeof(T) + a.K * (int)sizeof(T);  // CH: X's descriptor range
        auto ldx8 = [&](int rr, int cc) -> C8<T> {
            if constexpr (CH) return load_c8_sc1(a.X, xbytes, rr * a.ldx + kbeg + 8 * cc);
            else return load_c8(a.X + (size_t)rr * a.ldx + kbeg + 8 * cc);
        };
        if constexpr (CH) {  // chain stage: the weight ring first (no dependency), then the wait
#pragma unroll
            for (int u = 0; u < U; ++u) issue(u, u);
            if (cw.done) chain_wait(cw);
            if constexpr (EPI == EPI_SLABFIN) load_res();
        }
        C8<T> xc[PRE_N], wc[PRO == PRO_PRENORM ? PRE_N : 1];
#pragma unroll
        for (int q = 0; q < PRE_N; ++q) {
            const int it = threadIdx.x + NTH * q;
            if (it < nitem) {
                const int rr = it / nch, cc = it - rr * nch;
                xc[q] = ldx8(rr, cc);
                if constexpr (PRO == PRO_PRENORM) wc[q] = load_c8(a.nw + kbeg + 8 * cc);
            }
        }
        // PRO_PRENORM: the [K/16][R] tile sums of squares, flattened over the block's threads,
        // GEMV_SSQ loads each, unconditional (clamped) and issued before the weight ring so their
        // wait does not queue behind weight bytes (a load under a branch makes the compiler drain
        // vmcnt(0) right there, before the ring is even issued)
        constexpr int GEMV_SSQ = 2;
        const int nss = (a.K >> 4) * R;
        float ssv[PRO == PRO_PRENORM ? GEMV_SSQ : 1];
        if constexpr (PRO == PRO_PRENORM) {
#pragma unroll
            for (int q = 0; q < GEMV_SSQ; ++q) {
                const int e = threadIdx.x + NTH * q;
                if constexpr (CH)
                    ssv[q] = __hip_atomic_load(a.ss_in + (e < nss ? e : nss - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else
                    ssv[q] = a.ss_in[e < nss ? e : nss - 1];
            }
        }
        if constexpr (!CH) {
#pragma unroll
            for (int u = 0; u < U; ++u) issue(u, u);
            pf_issue();
        }
        if constexpr (PRO == PRO_PRENORM) {
            float* rsw = rsl + wave * GEMV_RMAX;
            if (!CH && a.ss_gran == 1) {
                // one row, whole K staged in xc (host-checked): the statistic from the row itself,
                // sum of x^2 per thread, per wave, then over the block's waves in a fixed order
                // (the producer -- fm_rowgemv.hip -- wrote no tile sums)
                float sl = 0.f;
#pragma unroll
                for (int q = 0; q < PRE_N; ++q) {
                    const int it = threadIdx.x + NTH * q;
                    if (it < nitem) {
                        float xv[8];
                        c8_to_f(xc[q], xv);
#pragma unroll
                        for (int u = 0; u < 8; ++u) sl += xv[u] * xv[u];
                    }
                }
                sl = wave_sum(sl);
                if (lane == 0) red[wave] = sl;
                lds_barrier();
                if (a.dbg) tsA = __builtin_amdgcn_s_memrealtime();
                float tot = 0.f;
#pragma unroll
                for (int w = 0; w < WPB; ++w) tot += red[w];
                if (lane == 0) rsw[0] = 1.0f / sqrtf(tot / (float)a.K + a.eps);
            } else {
            // stage the tile sums in `red` (free until the cross-wave reduction), then every wave
            // reduces each row's sums itself: per-row 1/rms in the wave's LDS slot (a register
            // array indexed by the runtime row would be spilled to scratch)
#pragma unroll
            for (int q = 0; q < GEMV_SSQ; ++q) {  // unconditional: the clamped tail re-stores the
                const int e = threadIdx.x + NTH * q;  // last sum (same value), and no branch lets
                red[e < nss ? e : nss - 1] = ssv[q];  // the compiler sink a load past the ring
            }
            for (int e = threadIdx.x + NTH * GEMV_SSQ; e < nss; e += NTH)  // R * K large
                red[e] = CH ? __hip_atomic_load(a.ss_in + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : a.ss_in[e];
            __syncthreads();
            if (a.dbg) tsA = __builtin_amdgcn_s_memrealtime();
            const int nt = a.K >> 4;
#pragma unroll
            for (int rr = 0; rr < GEMV_RMAX; ++rr) {
                if (rr >= R) break;
                float sl = 0.f;
                for (int t = lane; t < nt; t += 64) sl += red[t * R + rr];
                const float v = 1.0f / sqrtf(wave_sum(sl) / (float)a.K + a.eps);
                if (lane == 0) rsw[rr] = v;
            }
            }
            __builtin_amdgcn_wave_barrier();
            const bool writer = bxi == 0 && ks == 0 && a.xn_out;
            auto put = [&](int rr, int cc, const C8<T>& xq, const C8<T>& wq) {
                float xv[8], wv[8];
                c8_to_f(xq, xv);
                c8_to_f(wq, wv);
                const float rs = rsw[rr];
                C8<T> o;
                T* ov = reinterpret_cast<T*>(&o);
#pragma unroll
                for (int u = 0; u < 8; ++u) st(ov, u, rnd<T>(xv[u] * rs) * wv[u]);
                *reinterpret_cast<C8<T>*>(xs + (size_t)rr * xstride + 8 * cc) = o;  // one 16/32-B store
                if (writer) *reinterpret_cast<C8<T>*>(a.xn_out + (size_t)rr * a.ldxo + kbeg + 8 * cc) = o;
            };
#pragma unroll
            for (int q = 0; q < PRE_N; ++q) {
                const int it = threadIdx.x + NTH * q;
                if (it < nitem) put(it / nch, it - (it / nch) * nch, xc[q], wc[q]);
            }
            for (int it = threadIdx.x + NTH * PRE_N; it < nitem; it += NTH) {
                const int rr = it / nch, cc = it - rr * nch;
                put(rr, cc, ldx8(rr, cc), load_c8(a.nw + kbeg + 8 * cc));
            }
            if (a.dbg) tsB = __builtin_amdgcn_s_memrealtime();
        } else {
#pragma unroll
            for (int q = 0; q < PRE_N; ++q) {
                const int it = threadIdx.x + NTH * q;
                if (it < nitem) {
                    const int rr = it / nch, cc = it - rr * nch;
                    *reinterpret_cast<C8<T>*>(xs + (size_t)rr * xstride + 8 * cc) = xc[q];
                }
            }
            for (int it = threadIdx.x + NTH * PRE_N; it < nitem; it += NTH) {  // large R x Kb
                const int rr = it / nch, cc = it - rr * nch;
                *reinterpret_cast<C8<T>*>(xs + (size_t)rr * xstride + 8 * cc) = ldx8(rr, cc);
            }
        }
    }
    lds_barrier();  // X' staged; the weight ring stays in flight (each MFMA waits for its own fragment)
    // int4: X_u = sum of each staged x row over each 128-k unit (one wave per (unit, row), 2 k per lane)
    float* xsum = reinterpret_cast<float*>(smem + a.q4_xsum_off);
    if constexpr (Q4) {
        const int nu = Kb >> 7;
        for (int pr = wave; pr < nu * R; pr += WPB) {
            const int uu = pr / R, rr = pr - uu * R;
            const T* xr = xs + (size_t)rr * xstride + uu * 128 + 2 * lane;
            float v = ld(xr, 0) + ld(xr, 1);
            v = wave_sum(v);
            if (lane == 0) xsum[pr] = v;
        }
        lds_barrier();
    }

    const unsigned long long ts1 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    // ---------------- main loop: ring of U fragments per wave ------------------------------------
    const T* xp = xs + (size_t)(r < R ? r : R - 1) * xstride + (size_t)wa * KU + 8 * g;
    f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < nmy; i += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + u < nmy) {
                if constexpr (Q4) {
                    f32x4_t b = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t w = fq[u][j];
                        typename G::f A;
#pragma unroll
                        for (int p = 0; p < 4; ++p) A[p] = ((w >> (4 * p)) & 0x000F000Fu) | 0x43004300u;
                        b = G::mma(A, G::load(xp + (size_t)(i + u) * 128 + 32 * j), b);
                    }
                    const float xu = xsum[(wa + i + u) * R + (r < R ? r : 0)];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float sc = __uint_as_float(fz[u][e] << 16), zr = __uint_as_float(fz[u][e] & 0xffff0000u);
                        acc0[e] += sc * b[e] + (zr - 136.f * sc) * xu;
                    }
                } else if constexpr (Q8) {
                    typename G::f w0, w1;
                    G::dq8(fq[u], w0, w1);
                    acc0 = G::mma(w0, G::load(xp + (size_t)(i + u) * 64), acc0);
                    acc0 = G::mma(w1, G::load(xp + (size_t)(i + u) * 64 + 32), acc0);
                } else {
                    const typename G::f xb = G::load(xp + (size_t)(i + u) * 32);
                    acc0 = G::mma(fa[u], xb, acc0);
                    if constexpr (NACC == 2) acc1 = G::mma(fb[u], xb, acc1);
                }
            }
            issue(i + u + U, u);
        }
    }
    if constexpr (PFOK) {  // keep the prefetch loads (long retired: the ring's refills were issued after them)
#pragma unroll
        for (int q = 0; q < GEMV_PF; ++q) asm volatile("" ::"v"(pfw[q]));
    }
    // weight-only int8 output: round(round(acc) * scale of the packed row)
    auto wsc = [&](float v, int prow) {
        if constexpr (Q8) return rnd<T>(rnd<T>(v) * ld(a.wscale, prow));
        else return v;
    };
    // cross-wave reduction: only the R live columns of the 16x16 accumulator tile go to LDS
    if ((lane & 15) < R) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = 4 * (lane >> 4) + i, col = lane & 15;
            red[((0 * WPB + wave) * 16 + row) * R + col] = acc0[i];
            if constexpr (NACC == 2) red[((1 * WPB + wave) * 16 + row) * R + col] = acc1[i];
        }
    }
    const unsigned long long ts2 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    __syncthreads();
    // developer timestamps: one record per block {tag, t0 start, t1 staged, t2 streamed, t3 end}
    auto stamp = [&]() {
        if (a.dbg && threadIdx.x == 0) {
            const unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
            const unsigned long long slot = atomicAdd(a.dbg, 1ull);
            if (slot < (1ull << 20)) {
                unsigned long long* q = a.dbg + 8 + slot * 8;
                q[0] = ((unsigned long long)a.N << 32) | ((unsigned long long)ks << 16) | bxi;
                q[1] = ts0;
                q[2] = ts1;
                q[3] = ts2;
                q[4] = t3;
                q[5] = tsA;
                q[6] = tsB;
                q[7] = 0;
            }
        }
    };

    // ---------------- epilogue: 16 rows x R cols -----------------------------------------------
    if constexpr (EPI == EPI_SWIGLU8) {  // rows 0-7 gate, 8-15 up of the same 8 outputs
        for (int o = threadIdx.x; o < 8 * R; o += NTH) {
            const int row = o / R, col = o - row * R;
            const int n = bxi * 8 + row;
            if (!CH && n >= (a.N >> 1)) continue;  // (CH: N % 16 == 0, host-checked)
            float v0 = 0.f, v1 = 0.f;
#pragma unroll
            for (int w = 0; w < WPB; ++w) {
                v0 += red[(w * 16 + row) * R + col];
                v1 += red[(w * 16 + row + 8) * R + col];
            }
            v0 = wsc(v0, n0 + row);
            v1 = wsc(v1, n0 + row + 8);
            const float y = rnd<T>(silu_g(rnd<T>(v0))) * rnd<T>(v1);
            if constexpr (CH)
                st_sc1_run(a.Y, (size_t)col * a.ldy + n, y);
            else
                st(a.Y, (size_t)col * a.ldy + n, y);
        }
        stamp();
        return;
    }
    for (int o = threadIdx.x; o < 16 * R; o += NTH) {
        const int row = o / R, col = o - row * R;
        const int n = n0 + row;
        if (!CH && n >= a.N) continue;  // (CH: N % 16 == 0, host-checked: every lane of a run stores)
        float v0 = 0.f, v1 = 0.f;
#pragma unroll
        for (int w = 0; w < WPB; ++w) {
            v0 += red[((0 * WPB + w) * 16 + row) * R + col];
            if constexpr (NACC == 2) v1 += red[((1 * WPB + w) * 16 + row) * R + col];
        }
        if constexpr (EPI == EPI_SLAB) {
            if (a.bias && ks == 0) v0 += ld(a.bias, n);
            a.Yf[((size_t)ks * R + col) * a.ldy + n] = v0;
        } else if constexpr (EPI == EPI_SLABFIN) {
            if (a.bias && ks == 0) v0 += ld(a.bias, n);
            if (nks == 1) {  // whole K in this block: finalise from LDS below
                fin[col * 16 + (n - n0)] = v0;
            } else {  // write-through (sc1) partial: visible to the tile's reducer without a fence
                __hip_atomic_store(a.Yf + ((size_t)ks * R + col) * a.ldy + n, v0, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            v0 = wsc(v0, n);
            if (a.bias) v0 += ld(a.bias, n);
            const size_t yi = (size_t)col * a.ldy + n;
            if constexpr (EPI == EPI_STORE) {
                if constexpr (CH)
                    st_sc1_run(a.Y, yi, v0);
                else
                    st(a.Y, yi, v0);
            } else if constexpr (EPI == EPI_SWIGLU) {
                const float ga = rnd<T>(v0), ub = rnd<T>(v1);
                st(a.Y, yi, rnd<T>(silu_g(ga)) * ub);
            } else {
                a.Yf[yi] = rnd<T>(v0);
            }
        }
    }
    if constexpr (EPI == EPI_SLABFIN) {
        // The last-arriving K-slice block of this 16-column tile finalises the residual stream:
        // x = round(res + round(sum_q partial_q)) (llama.py:841-842) and the tile's sum of x^2 for
        // the consumer's RMSNorm.  Hand-off in its write-through form (cdna_hip_programming.md §5,
        // split-K recipe): sc1 partial stores drained by every wave, a relaxed agent ticket, sc1
        // loads in the reducer -- no release / acquire fence.  ksb == 1: straight from LDS.
        const int ksb = nks;
        if (ksb > 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (ksb > 1) {
            if (threadIdx.x == 0) {
                const int t = __hip_atomic_fetch_add(a.tickets + bxi, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int last = t == ksb - 1;
                if (last) __hip_atomic_store(a.tickets + bxi, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                flag[0] = last;
            }
            __syncthreads();
            if (!flag[0]) {
                stamp();
                return;
            }
        }
        const int t = threadIdx.x;
        if (t < 16 * R) {
            const int col = t >> 4, n = n0 + (t & 15);
            float y = 0.f;
            if (ksb == 1)
                y = fin[t];
            else
                for (int q = 0; q < ksb; ++q)
                    y += __hip_atomic_load(a.Yf + ((size_t)q * R + col) * a.ldy + n, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            const float x = rnd<T>(res_pre + rnd<T>(wsc(y, n)));
            if constexpr (CH)
                st_sc1_run(a.res_out, (size_t)col * a.ldro + n, x);
            else
                st(a.res_out, (size_t)col * a.ldro + n, x);
            float sq = x * x;
#pragma unroll
            for (int m = 1; m < 16; m <<= 1) sq += __shfl_xor(sq, m);
            if ((t & 15) == 0) {
                if constexpr (CH)
                    __hip_atomic_store(a.ss_out + (size_t)bxi * R + col, sq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else
                    a.ss_out[(size_t)bxi * R + col] = sq;
            }
        }
    }
    stamp();
}

template <typename T, int PRO, int EPI, bool NT, int U, int WPB, int QM>
__global__ __launch_bounds__(WPB * 64) __attribute__((amdgpu_waves_per_eu(gemv_wpe(PRO, EPI))))
void gemv_kernel(GemvArgs<T> a) {
    gemv_body<T, PRO, EPI, NT, U, WPB, QM, false>(a, blockIdx.x, blockIdx.y, gridDim.y, ChainWait{});
}

// One launch running up to GEMV_CHAIN_MAX dependent batch-1 GEMVs (fm_llm.cpp: a layer's wo, w1||w3,
// w2 and the next layer's qkv).  Stage s owns blocks [off[s], off[s+1]) (dispatch is in block
// order, so a waiting block only waits on blocks already resident or done); a stage's blocks
// issue their weight ring, then wait for every block of stage s - 1 to arrive.  The last block of
// the last stage to arrive resets every counter of the launch (all waits have passed by then), so
// the next launch starts from zero (first use: zeroed at allocation).
template <typename T, bool NT, int U, int WPB>
__global__ __launch_bounds__(WPB * 64) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 2 ? 5 : 2)))
void gemv_chain_kernel(GemvChainArgs<T> c) {
    int s = 0;
    while (s + 1 < c.n && (int)blockIdx.x >= c.off[s + 1]) ++s;
    const int bxi = blockIdx.x - c.off[s];
    ChainWait cw;
    if (s > 0) {
        cw.done = chain_word(c.cnt, s - 1, 9 + (blockIdx.x & 7));
        cw.sleep = c.sleep;
        cw.err = c.err;
    }
    const GemvArgs<T>& a = c.st[s];
    switch (c.kind[s]) {
        case GEMV_CHAIN_WO_W2: gemv_body<T, PRO_PLAIN, EPI_SLABFIN, NT, U, WPB, false, true>(a, bxi, 0, 1, cw); break;
        case GEMV_CHAIN_W13: gemv_body<T, PRO_PRENORM, EPI_SWIGLU8, NT, U, WPB, false, true>(a, bxi, 0, 1, cw); break;
        case GEMV_CHAIN_QKV: gemv_body<T, PRO_PRENORM, EPI_STORE, NT, U, WPB, false, true>(a, bxi, 0, 1, cw); break;
        default: gemv_body<T, PRO_PRENORM, EPI_F32, NT, U, WPB, false, true>(a, bxi, 0, 1, cw); break;
    }
    // publish: every storing wave drains its write-through stores, then one arrival per block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int k = blockIdx.x & 7;
        // blocks of this stage in shard k: b in [off[s], off[s+1]) with b % 8 == k
        const unsigned tot = (unsigned)((c.off[s + 1] + 7 - k) / 8 - (c.off[s] + 7 - k) / 8);
        if (__hip_atomic_fetch_add(chain_word(c.cnt, s, k), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tot - 1) {
            const unsigned ne = (unsigned)min(8, c.off[s + 1] - c.off[s]);
            if (__hip_atomic_fetch_add(chain_word(c.cnt, s, 8), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ne - 1) {
                if (s + 1 < c.n) {  // stage complete: release its waiters
                    for (int r = 0; r < 8; ++r)
                        __hip_atomic_store(chain_word(c.cnt, s, 9 + r), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    // the launch is complete and every wait has passed: zero the words for the next one
                    for (int q = 0; q < c.n; ++q)
                        for (int j = 0; j < GEMV_CHAIN_SLOTS; ++j)
                            __hip_atomic_store(chain_word(c.cnt, q, j), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
}

template <typename T, int PRO, int EPI, bool NT, int U, int WPB, int QM = 0>
static void gemv_launch(hipStream_t s, const GemvArgs<T>& a0, dim3 grid, size_t lds) {
    GemvArgs<T> a = a0;
    a.dbg = fm_tuning().dbg;
    static bool big = false;  // > 64 KiB of dynamic LDS (gfx950: 160 KiB per CU)
    if (lds > 64 * 1024 && !big) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemv_kernel<T, PRO, EPI, NT, U, WPB, QM>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        big = true;
    }
    gemv_kernel<T, PRO, EPI, NT, U, WPB, QM><<<grid, WPB * 64, lds, s>>>(a);
}

template <typename T, int PRO, int EPI, bool NT, int U>
static void gemv_go_w(hipStream_t s, const GemvArgs<T>& a, dim3 grid, size_t lds) {
    if (fm_tuning().gemv_wpb == 8)
        gemv_launch<T, PRO, EPI, NT, U, 8>(s, a, grid, lds);
    else
        gemv_launch<T, PRO, EPI, NT, U, 4>(s, a, grid, lds);
}

template <typename T, int PRO, int EPI, bool NT>
static void gemv_go_u(hipStream_t s, const GemvArgs<T>& a, dim3 grid, size_t lds) {
    switch (fm_tuning().gemv_u) {
        case 8: gemv_go_w<T, PRO, EPI, NT, 8>(s, a, grid, lds); break;
        case 2: gemv_go_w<T, PRO, EPI, NT, 2>(s, a, grid, lds); break;
        default: gemv_go_w<T, PRO, EPI, NT, 4>(s, a, grid, lds); break;
    }
}

template <typename T, int PRO, int EPI>
static void gemv_go(hipStream_t s, const GemvArgs<T>& a, int ksb) {
    dim3 grid(FM_CEIL(a.N, 16), ksb);
    const int Kb = a.K / ksb;
    size_t lds = gemv_lds_bytes(a.R, Kb, sizeof(T));
    GemvArgs<T> b = a;
    if constexpr (PRO == PRO_FATT) {
        lds = (lds + 15) & ~(size_t)15;
        b.fatt_off = (int)lds;
        lds += fatt_lds_bytes(a.att.ldqkv, a.att.nkv, a.att.S, a.att.hd, sizeof(T));
    }
    if (fm_tuning().gemv_nt)
        gemv_go_u<T, PRO, EPI, true>(s, b, grid, lds);
    else
        gemv_go_u<T, PRO, EPI, false>(s, b, grid, lds);
}

// weight-only int8: non-temporal, fm_tune q_u units in flight per wave (default 4), 4 waves
template <typename T, int PRO, int EPI>
static void gemv_go_q8(hipStream_t s, const GemvArgs<T>& a, int ksb) {
    FMCHECK(a.K % (64 * ksb) == 0 && a.wscale, "int8 GEMV: K slices must be whole 64-k units, scales set");
    const dim3 grid(FM_CEIL(a.N, 16), ksb);
    const size_t lds = gemv_lds_bytes(a.R, a.K / ksb, sizeof(T));
    if (fm_tuning().q_u == 16) gemv_launch<T, PRO, EPI, true, 16, 4, 1>(s, a, grid, lds);
    else if (fm_tuning().q_u == 8) gemv_launch<T, PRO, EPI, true, 8, 4, 1>(s, a, grid, lds);
    else if (fm_tuning().q_u == 2) gemv_launch<T, PRO, EPI, true, 2, 4, 1>(s, a, grid, lds);
    else gemv_launch<T, PRO, EPI, true, 4, 4, 1>(s, a, grid, lds);
}

// weight-only int4 (bf16): the same configuration over 128-k units
template <typename T, int PRO, int EPI>
static void gemv_go_q4(hipStream_t s, const GemvArgs<T>& a, int ksb) {
    if constexpr (sizeof(T) == 2) {
        FMCHECK(a.K % (128 * ksb) == 0 && a.wsz && !a.wscale, "int4 GEMV: K slices must be whole 128-k units, (scale, zero) set");
        const dim3 grid(FM_CEIL(a.N, 16), ksb);
        GemvArgs<T> b = a;
        b.q4_xsum_off = (int)((gemv_lds_bytes(a.R, a.K / ksb, sizeof(T)) + 15) & ~(size_t)15);
        const size_t lds = b.q4_xsum_off + (size_t)(a.K / ksb / 128) * a.R * 4;
        if (fm_tuning().q_u == 16) gemv_launch<T, PRO, EPI, true, 16, 4, 2>(s, b, grid, lds);
        else if (fm_tuning().q_u == 8) gemv_launch<T, PRO, EPI, true, 8, 4, 2>(s, b, grid, lds);
        else if (fm_tuning().q_u == 2) gemv_launch<T, PRO, EPI, true, 2, 4, 2>(s, b, grid, lds);
        else gemv_launch<T, PRO, EPI, true, 4, 4, 2>(s, b, grid, lds);
    } else {
        FMCHECK(false, "int4 GEMV: bf16 only");
    }
}

template <typename T> void launch_gemv(hipStream_t s, const GemvArgs<T>& a, int pro, int epi, int ksb) {
    // PRO_PRENORM stages the [K/16][R] tile sums in the 256 * R floats of the reduction buffer
    FMCHECK(pro != PRO_PRENORM || (a.K <= 4096 && a.R <= GEMV_RMAX), "PRO_PRENORM needs K <= 4096, R <= 8");
    FMCHECK(pro != PRO_PRENORM || (a.ss_in && (a.ss_gran != 1 || (a.R == 1 && ksb == 1 && a.K <= 3 * 8 * 256))),
            "PRO_PRENORM: ss_in set (also with ss_gran 1: one row, whole K staged)");
    FMCHECK(pro != PRO_FATT || (a.R == 1 && a.att.cpos < FAST_ATTN_MAXJ && a.att.cpos < a.att.S &&
                                (a.K / ksb) % a.att.hd == 0 && a.att.hd % 16 == 0 && a.att.hd <= 16 * FATT_MAXPP &&
                                a.att.ldqkv % 8 == 0),
            "PRO_FATT needs one row, cpos < 16, whole heads per K slice");
    if (a.Wq) {
#define GQ(P, E)                                           \
    if (pro == P && epi == E) {                            \
        if (a.wsz) gemv_go_q4<T, P, E>(s, a, ksb);         \
        else gemv_go_q8<T, P, E>(s, a, ksb);               \
        return;                                            \
    }
        GQ(PRO_PLAIN, EPI_STORE) GQ(PRO_PLAIN, EPI_SLABFIN) GQ(PRO_PLAIN, EPI_F32)
        GQ(PRO_NORM, EPI_STORE) GQ(PRO_NORM, EPI_F32)
        GQ(PRO_PRENORM, EPI_STORE) GQ(PRO_PRENORM, EPI_F32) GQ(PRO_PRENORM, EPI_SWIGLU8)
#undef GQ
        FMCHECK(false, "int8 / int4 GEMV: no kernel for this prologue / epilogue");
    }
#define GO(P, E)                                           \
    if (pro == P && epi == E) {                            \
        gemv_go<T, P, E>(s, a, ksb);                       \
        return;                                            \
    }
    GO(PRO_PLAIN, EPI_STORE) GO(PRO_PLAIN, EPI_SLABFIN) GO(PRO_PLAIN, EPI_F32) GO(PRO_PLAIN, EPI_SLAB)
    GO(PRO_NORM, EPI_STORE) GO(PRO_NORM, EPI_SWIGLU) GO(PRO_NORM, EPI_F32)
    GO(PRO_PRENORM, EPI_STORE) GO(PRO_PRENORM, EPI_SWIGLU) GO(PRO_PRENORM, EPI_F32)
    GO(PRO_PRENORM, EPI_SWIGLU8)
    GO(PRO_FATT, EPI_SLABFIN)
#undef GO
}

template <typename T> void launch_gemv_chain(hipStream_t s, const GemvChainArgs<T>& c0) {
    FMCHECK(c0.n >= 2 && c0.n <= GEMV_CHAIN_MAX && c0.cnt && c0.err, "gemv chain: 2..4 stages, counters set");
    GemvChainArgs<T> c = c0;
    size_t lds = 0;
    c.off[0] = 0;
    for (int i = 0; i < c.n; ++i) {
        GemvArgs<T>& a = c.st[i];
        FMCHECK(a.R == 1 && a.N % 16 == 0 && a.K % 32 == 0 && !a.Wq && !a.xidx,
                "gemv chain: one row, N % 16 == 0, no X gather, no int8");
        FMCHECK(c.kind[i] != GEMV_CHAIN_HEAD || i == c.n - 1, "gemv chain: the fp32 head stage ends the launch");
        FMCHECK(a.K <= 4096 || c.kind[i] == GEMV_CHAIN_WO_W2, "gemv chain: PRO_PRENORM needs K <= 4096");
        a.dbg = fm_tuning().dbg;
        c.off[i + 1] = c.off[i] + a.N / 16;
        lds = std::max(lds, gemv_lds_bytes(1, a.K, sizeof(T)));
    }
    FMCHECK(lds <= 64 * 1024, "gemv chain: LDS budget");
    gemv_chain_kernel<T, true, 8, 4><<<c.off[c.n], 256, lds, s>>>(c);
}

template void launch_gemv_chain<bf16_t>(hipStream_t, const GemvChainArgs<bf16_t>&);
template void launch_gemv_chain<float>(hipStream_t, const GemvChainArgs<float>&);
template void launch_gemv<bf16_t>(hipStream_t, const GemvArgs<bf16_t>&, int, int, int);
template void launch_gemv<float>(hipStream_t, const GemvArgs<float>&, int, int, int);

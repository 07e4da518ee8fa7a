// fm_bstream.hip -- batched decode linears for 8 < R <= 32 rows (BASELINE config 3: 32 concurrent
// utterances per GPU), and the residual finalise + RMSNorm that consumes their split-K slabs.
//
// At R = 32 a decode linear does 32 flop per weight byte: it is an HBM weight stream, not a GEMM.
// Measured on gfx950 (scripts/bgemm_probe.hip, 36 layers of distinct S2-Pro weights):
//   * staging the X slice in LDS caps the block at one per CU, and the in-flight weight bytes
//     with it;
//   * loading X B-fragments from L2 beside every weight fragment (16-row gathers) halves the
//     stream rate;
//   * split-K partials combined by the last-arriving block (ticket) put two memory round trips on
//     every block's tail.
// So X lives in VGPRs instead. Block = NW waves, one block per CU. Wave w owns the k-steps
// [w*Sp/NW, (w+1)*Sp/NW) of the block's K part (at most SPW of them). Their B fragments, both
// 16-column groups, are loaded once. The wave then streams the weight fragments of the block's
// contiguous tile range at those k-steps through a ring of SPW*TPI fragments, the next TPI tiles
// ahead. Per tile, the NW wave partials are summed through LDS (double-buffered, one barrier per
// tile), and the epilogue runs on the full-K sum:
//   EPI_STORE   Y = round(v + bias)                       (QKV, fast_project_in)
//   EPI_SWIGLU8 row-interleaved W1||W3 tile -> 8 outputs round(silu(round(g))) * round(u)
//   EPI_F32     logits as fp32 holding the T-rounded value
//   EPI_SLAB    kparts > 1: fp32 partial slab [kp][R][ldy], no combine here. The consumer
//               (finalize_norm_kernel) sums the slabs, so no block waits on another.
// Weights use the packed fragment layout of fm_kernels.h, shared with the batch-1 GEMV.
#include "fm_kernels.h"
#include "fm_runtime.h"
#include "fm_frag.h"

#include <cmath>

namespace {

constexpr int BS_MAXW = 16;  // waves per block

__device__ __forceinline__ float silu_b(float a) { return a / (1.0f + expf(-a)); }

template <typename T, int SPW, int TPI, int EPI>
__global__ __launch_bounds__(BS_MAXW * 64) void bstream_kernel(BstreamArgs<T> a) {
    using F = Frag<T>;
    __shared__ f32x4_t red[2][BS_MAXW][2][64];
    constexpr int U = SPW * TPI;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, NW = blockDim.x >> 6;
    const int kparts = a.kparts;
    const int kp = blockIdx.x % kparts, gb = blockIdx.x / kparts, Gk = gridDim.x / kparts;
    const int T_ = (a.N + 15) >> 4;
    const int t0 = (int)((long long)gb * T_ / Gk), t1 = (int)((long long)(gb + 1) * T_ / Gk);
    const int ntl = t1 - t0;
    const int S = a.K >> 5, Sp = S / kparts, s0 = kp * Sp;
    const int wa = s0 + wave * Sp / NW, nst = s0 + (wave + 1) * Sp / NW - wa;  // host: 1 <= nst <= SPW
    const int r = lane & 15, g = lane >> 4;
    // this wave's B fragments (rows >= R and steps >= nst are zero; loads clamped, never skipped)
    typename F::f xa[SPW], xb[SPW];
    {
        const int ra = r < a.R ? r : a.R - 1, rb = 16 + r < a.R ? 16 + r : a.R - 1;
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            const int jj = j < nst ? j : nst - 1;
            const size_t k = (size_t)(wa + jj) * 32 + 8 * g;
            xa[j] = F::load(a.X + (size_t)ra * a.ldx + k);
            xb[j] = F::load(a.X + (size_t)rb * a.ldx + k);
            if (j >= nst || r >= a.R) xa[j] = F::zero();
            if (j >= nst || 16 + r >= a.R) xb[j] = F::zero();
        }
    }
    // weight stream: fragment f = (tile f / SPW, step min(f % SPW, nst - 1)); slots past the run
    // re-load its last fragment (a cache hit) so the ring never needs a branch
    const int flast = ntl * SPW - 1;
    const T* wbase = a.W + ((size_t)t0 * S + wa) * 512;
    typename F::f fa[U];
    auto issue = [&](int f, int u) {
        f = f < flast ? f : flast;
        const int t = f / SPW, j = f - t * SPW;
        fa[u] = F::template load_w<true>(wbase + ((size_t)t * S + (j < nst ? j : nst - 1)) * 512, lane);
    };
#pragma unroll
    for (int u = 0; u < U; ++u) issue(u, u);

    for (int t = 0; t < ntl; t += TPI) {
#pragma unroll
        for (int tt = 0; tt < TPI; ++tt) {
            f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
            for (int j = 0; j < SPW; ++j) {
                const int u = tt * SPW + j;
                acc0 = F::mma(fa[u], xa[j], acc0);
                acc1 = F::mma(fa[u], xb[j], acc1);
                issue((t + TPI) * SPW + u, u);
                __builtin_amdgcn_sched_barrier(0);  // each refill right behind its consumer
            }
            const int buf = (t + tt) & 1;
            red[buf][wave][0][lane] = acc0;
            red[buf][wave][1][lane] = acc1;
            __syncthreads();  // buf is rewritten two tiles later, behind the next tile's barrier
            const int tile = t0 + t + tt;
            if (t + tt < ntl) {
                // 16 rows x R columns; C/D map of a 16x16 accumulator: row = 4*(lane>>4)+i, col = lane&15
                if constexpr (EPI == EPI_SWIGLU8) {
                    for (int o = threadIdx.x; o < 8 * a.R; o += blockDim.x) {
                        const int col = o >> 3, row = o & 7;
                        const int cg = col >> 4, i = row & 3;
                        const int lg = 16 * (row >> 2) + (col & 15), lu = 16 * ((row + 8) >> 2) + (col & 15);
                        float vg = 0.f, vu = 0.f;
                        for (int w = 0; w < NW; ++w) {
                            vg += red[buf][w][cg][lg][i];
                            vu += red[buf][w][cg][lu][i];
                        }
                        if (a.wscale) {  // weight-only int8: round(round(acc) * scale) per packed row
                            vg = rnd<T>(rnd<T>(vg) * ld(a.wscale, tile * 16 + row));
                            vu = rnd<T>(rnd<T>(vu) * ld(a.wscale, tile * 16 + 8 + row));
                        }
                        const int n = tile * 8 + row;
                        if (n < (a.N >> 1)) st(a.Y, (size_t)col * a.ldy + n, rnd<T>(silu_b(rnd<T>(vg))) * rnd<T>(vu));
                    }
                } else {
                    for (int o = threadIdx.x; o < 16 * a.R; o += blockDim.x) {
                        const int col = o >> 4, row = o & 15;
                        const int cg = col >> 4, ln = 16 * (row >> 2) + (col & 15), i = row & 3;
                        float v = 0.f;
                        for (int w = 0; w < NW; ++w) v += red[buf][w][cg][ln][i];
                        const int n = tile * 16 + row;
                        if (n >= a.N) continue;
                        if constexpr (EPI == EPI_SLAB) {
                            a.Yf[((size_t)kp * a.R + col) * a.ldy + n] = v;
                        } else {
                            if (a.wscale) v = rnd<T>(rnd<T>(v) * ld(a.wscale, n));
                            if (a.bias) v += ld(a.bias, n);
                            if constexpr (EPI == EPI_STORE)
                                st(a.Y, (size_t)col * a.ldy + n, v);
                            else
                                a.Yf[(size_t)col * a.ldy + n] = rnd<T>(v);
                        }
                    }
                }
            }
        }
    }
}

// 8 bf16 of an X row -> round(round(x * rs) * w) (RMSNorm's two roundings, llama.py:989-1000)
template <typename T>
__device__ __forceinline__ typename Frag<T>::f bs_norm8(typename Frag<T>::f x, float rs, typename Frag<T>::f w) {
    static_assert(sizeof(T) == 2, "bsacc runs bf16");
    typename Frag<T>::f o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float x0 = __uint_as_float(x[i] << 16), x1 = __uint_as_float(x[i] & 0xffff0000u);
        const float w0 = __uint_as_float(w[i] << 16), w1 = __uint_as_float(w[i] & 0xffff0000u);
        const float y0 = rnd<T>(rnd<T>(x0 * rs) * w0), y1 = rnd<T>(rnd<T>(x1 * rs) * w1);
        o[i] = (__float_as_uint(y0) >> 16) | (__float_as_uint(y1) & 0xffff0000u);
    }
    return o;
}

// bsacc_kernel: the same weight stream without a barrier per tile.  Block b takes K part
// b % kparts and a balanced run of tiles (<= NTM); each wave keeps one pair of 16x16 accumulators
// PER TILE in registers, streams its fragments through a ring TPI tiles deep, and only after the
// whole run do the waves meet once: every (tile, wave) partial goes to LDS, then the epilogue of
// all the block's tiles.  kparts is chosen so that tiles * kparts is a whole number of rounds of
// the grid (no block streams twice as much as another).
template <typename T, int SPW, int TPI, int NTM, int EPI, int PRO>
__global__ __launch_bounds__(512) void bsacc_kernel(BstreamArgs<T> a) {
    using F = Frag<T>;
    extern __shared__ __attribute__((aligned(16))) f32x4_t bred[];  // [NTM][NW][2][64]
    constexpr int U = SPW * TPI;
    const unsigned long long ts0 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    unsigned long long ts1 = 0, tsx = 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, NW = blockDim.x >> 6;
    const int kparts = a.kparts;
    const int kp = blockIdx.x % kparts, gb = blockIdx.x / kparts, Gk = gridDim.x / kparts;
    const int T_ = (a.N + 15) >> 4;
    const int t0 = (int)((long long)gb * T_ / Gk), t1 = (int)((long long)(gb + 1) * T_ / Gk);
    const int ntl = t1 - t0;  // host: 1 <= ntl <= NTM
    const int S = a.K >> 5, Sp = S / kparts, s0 = kp * Sp;
    const int wa = s0 + wave * Sp / NW, nst = s0 + (wave + 1) * Sp / NW - wa;  // host: 1 <= nst <= SPW
    const int r = lane & 15, g = lane >> 4;
    const int ra = r < a.R ? r : a.R - 1, rb = 16 + r < a.R ? 16 + r : a.R - 1;
    // weights (they do not depend on X): ring slot u = (t % TPI) * SPW + j holds (tile t, step j)
    const T* wbase = a.W + ((size_t)t0 * S + wa) * 512;
    const int tl = ntl - 1, jl = nst - 1;
    typename F::f fa[U];
    auto issue = [&](int t, int j) {
        const int tt = t < tl ? t : tl, jj = j < jl ? j : jl;
        const bool past = a.dummy_tail && (t > tl || j > jl);  // not this block's: one cached fragment
        const T* dsrc = a.W + (a.dummy_tail == 2 ? (size_t)((blockIdx.x * 8 + wave) & 255) % ((size_t)T_ * S) * 512 : 0);
        fa[(t % TPI) * SPW + j] = F::template load_w<true>(past ? dsrc : wbase + ((size_t)tt * S + jj) * 512, lane);
    };
    // X operands.  PRO_PRENORM also loads the norm weight and the producer's per-tile sums of squares
    // here, laid out [R][K/16] by bsacc's EPI_SLABFIN (rows w + NW * i of wave w, tiles lane + 64 * jj;
    // host: R <= 32, NW == 8, K / 16 <= 192).  a.xfirst (default): these go out before the weight ring,
    // so the first MFMA waits for the first weight fragment, not for the whole ring (in-order vmcnt):
    // B=32 frame 6.48 -> 6.36 ms.  (A per-tile epilogue by each tile's last-arriving wave instead of
    // the one barrier + block epilogue measured 7.8 ms: one wave's stores are issue-bound.)
    typename F::f xa[SPW], xb[SPW], wn[PRO == PRO_PRENORM ? SPW : 1];
    float ssv[PRO == PRO_PRENORM ? 12 : 1];
    auto load_x = [&]() {
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            const int jj = j < nst ? j : nst - 1;
            const size_t k = (size_t)(wa + jj) * 32 + 8 * g;
            xa[j] = F::load(a.X + (size_t)ra * a.ldx + k);
            xb[j] = F::load(a.X + (size_t)rb * a.ldx + k);
            if constexpr (PRO == PRO_PRENORM) wn[j] = F::load(a.nw + k);
        }
        if constexpr (PRO == PRO_PRENORM) {
            const int nt = a.K >> 4;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int jj = 0; jj < 3; ++jj) {
                    const int row = wave + 8 * i, t = lane + 64 * jj;
                    const bool ok = row < a.R && t < nt;
                    const float v = a.ss_in[(size_t)(row < a.R ? row : 0) * nt + (ok ? t : 0)];  // [R][K/16]: coalesced
                    ssv[i * 3 + jj] = ok ? v : 0.f;
                }
        }
    };
    if (a.xfirst) load_x();
#pragma unroll
    for (int t = 0; t < TPI; ++t)
#pragma unroll
        for (int j = 0; j < SPW; ++j) issue(t, j);
    if (!a.xfirst) load_x();
    if constexpr (PRO == PRO_PRENORM) {
        // 1/rms of each X row (wave w: rows w, w + 8, w + 16, w + 24), then every lane's two rows from LDS
        __shared__ float rs_s[32];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float v = 1.0f / sqrtf(wave_sum(ssv[i * 3] + ssv[i * 3 + 1] + ssv[i * 3 + 2]) / (float)a.K + a.eps);
            if (lane == 0 && wave + 8 * i < a.R) rs_s[wave + 8 * i] = v;
        }
        // LDS-only barrier: __syncthreads() would also drain this wave's weight ring (its fence waits
        // for every outstanding global load), serialising the stream behind the norm statistic
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (a.dbg) tsx = __builtin_amdgcn_s_memrealtime();
        const float rsa = rs_s[ra], rsb = rs_s[rb];
#pragma unroll
        for (int j = 0; j < SPW; ++j) {  // round(round(x * rs) * w), llama.py:989-1000
            xa[j] = bs_norm8<T>(xa[j], rsa, wn[j]);
            xb[j] = bs_norm8<T>(xb[j], rsb, wn[j]);
        }
    }
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
        if (j >= nst || r >= a.R) xa[j] = F::zero();
        if (j >= nst || 16 + r >= a.R) xb[j] = F::zero();
    }
    f32x4_t acc[NTM][2];
#pragma unroll
    for (int t = 0; t < NTM; ++t) acc[t][0] = acc[t][1] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < NTM; ++t) {
#pragma unroll
        for (int j = 0; j < SPW; ++j) {
            const int u = (t % TPI) * SPW + j;
            acc[t][0] = F::mma(fa[u], xa[j], acc[t][0]);
            acc[t][1] = F::mma(fa[u], xb[j], acc[t][1]);
            if (t + TPI < NTM) issue(t + TPI, j);
            __builtin_amdgcn_sched_barrier(0);  // each refill right behind its consumer
            if (t == 0 && j == 0 && a.dbg) ts1 = __builtin_amdgcn_s_memrealtime();
        }
    }
    const unsigned long long ts2 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    // tiles >= ntl re-streamed the last tile (clamped loads): their accumulators are never read
#pragma unroll
    for (int t = 0; t < NTM; ++t) {
        bred[((t * NW + wave) * 2 + 0) * 64 + lane] = acc[t][0];
        bred[((t * NW + wave) * 2 + 1) * 64 + lane] = acc[t][1];
    }
    __syncthreads();
    const unsigned long long ts3 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    // developer stamps (scripts/b32_ts.py): {tag = (K << 16 | N >> 4) << 32 | block, start, first
    // MFMA, streamed, end, barrier passed, tiles}, from wave 0 of the block
    auto stamp = [&]() {
        if (a.dbg && threadIdx.x == 0) {
            const unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
            const unsigned long long slot = atomicAdd(a.dbg, 1ull);
            if (slot < (1ull << 20)) {
                unsigned long long* q = a.dbg + 8 + slot * 8;
                q[0] = ((unsigned long long)(((unsigned)a.K << 16) | ((unsigned)a.N >> 4)) << 32) | blockIdx.x;
                q[1] = ts0;
                q[2] = ts1;
                q[3] = ts2;
                q[4] = t4;
                q[5] = ts3;
                q[6] = (unsigned long long)ntl;
                q[7] = tsx;
            }
        }
    };
    // epilogue over the block's tiles: C/D map of a 16x16 accumulator: row = 4*(lane>>4)+i, col = lane&15
    // a.vec_epi: one item = 4 consecutive rows (one accumulator register quad) of one column: NW
    // 16-byte LDS reads (consecutive lanes, consecutive quads: no bank conflict) summed elementwise in
    // wave order (the scalar form's fp32 order: bit-identical), one 8 / 16-byte store
    const bool vec = a.vec_epi && EPI != EPI_SLABFIN && (a.N & 15) == 0 && (a.ldy & 3) == 0;
    auto quad = [&](int t, int cg, int ln) {
        f32x4_t v = bred[((t * NW) * 2 + cg) * 64 + ln];
        for (int w = 1; w < NW; ++w) {
            const f32x4_t p = bred[((t * NW + w) * 2 + cg) * 64 + ln];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] += p[i];
        }
        return v;
    };
    if (vec && EPI == EPI_SWIGLU8) {
        const int no = ntl * 64;  // (tile, column group, gate quad, column)
        for (int o = threadIdx.x; o < no; o += blockDim.x) {
            const int t = o >> 6, cg = (o >> 5) & 1, gq = (o >> 4) & 1, c16 = o & 15, col = 16 * cg + c16;
            if (col >= a.R) continue;
            f32x4_t vg = quad(t, cg, 16 * gq + c16), vu = quad(t, cg, 16 * (gq + 2) + c16);
            const int tile = t0 + t;
            float y[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float g_ = vg[i], u_ = vu[i];
                if (a.wscale) {
                    g_ = rnd<T>(rnd<T>(g_) * ld(a.wscale, tile * 16 + 4 * gq + i));
                    u_ = rnd<T>(rnd<T>(u_) * ld(a.wscale, tile * 16 + 8 + 4 * gq + i));
                }
                y[i] = rnd<T>(silu_b(rnd<T>(g_))) * rnd<T>(u_);
            }
            store4<T>(a.Y + (size_t)col * a.ldy + tile * 8 + 4 * gq, y);
        }
    } else if (vec) {
        const int no = ntl * 128;  // (tile, column group, row quad, column)
        for (int o = threadIdx.x; o < no; o += blockDim.x) {
            const int t = o >> 7, cg = (o >> 6) & 1, q = (o >> 4) & 3, c16 = o & 15, col = 16 * cg + c16;
            if (col >= a.R) continue;
            const f32x4_t v = quad(t, cg, 16 * q + c16);
            const int n = (t0 + t) * 16 + 4 * q;
            if constexpr (EPI == EPI_SLAB) {
                *reinterpret_cast<f32x4_t*>(a.Yf + ((size_t)kp * a.R + col) * a.ldy + n) = v;
            } else {
                float y[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float x = v[i];
                    if (a.wscale) x = rnd<T>(rnd<T>(x) * ld(a.wscale, n + i));
                    if (a.bias) x += ld(a.bias, n + i);
                    y[i] = EPI == EPI_STORE ? x : rnd<T>(x);
                }
                if constexpr (EPI == EPI_STORE)
                    store4<T>(a.Y + (size_t)col * a.ldy + n, y);
                else
                    *reinterpret_cast<f32x4_t*>(a.Yf + (size_t)col * a.ldy + n) = (f32x4_t){y[0], y[1], y[2], y[3]};
            }
        }
    } else if constexpr (EPI == EPI_SWIGLU8) {
        const int no = ntl * 8 * a.R;
        for (int o = threadIdx.x; o < no; o += blockDim.x) {
            const int t = o / (8 * a.R), oo = o - t * 8 * a.R;
            const int col = oo >> 3, row = oo & 7;
            const int cg = col >> 4, i = row & 3;
            const int lg = 16 * (row >> 2) + (col & 15), lu = 16 * ((row + 8) >> 2) + (col & 15);
            float vg = 0.f, vu = 0.f;
            for (int w = 0; w < NW; ++w) {
                vg += bred[((t * NW + w) * 2 + cg) * 64 + lg][i];
                vu += bred[((t * NW + w) * 2 + cg) * 64 + lu][i];
            }
            const int tile = t0 + t;
            if (a.wscale) {
                vg = rnd<T>(rnd<T>(vg) * ld(a.wscale, tile * 16 + row));
                vu = rnd<T>(rnd<T>(vu) * ld(a.wscale, tile * 16 + 8 + row));
            }
            const int n = tile * 8 + row;
            if (n < (a.N >> 1)) st(a.Y, (size_t)col * a.ldy + n, rnd<T>(silu_b(rnd<T>(vg))) * rnd<T>(vu));
        }
    } else {
        const int no = ntl * 16 * a.R;
        for (int o = threadIdx.x; o < no; o += blockDim.x) {
            const int t = o / (16 * a.R), oo = o - t * 16 * a.R;
            const int col = oo >> 4, row = oo & 15;
            const int cg = col >> 4, ln = 16 * (row >> 2) + (col & 15), i = row & 3;
            float v = 0.f;
            for (int w = 0; w < NW; ++w) v += bred[((t * NW + w) * 2 + cg) * 64 + ln][i];
            const int n = (t0 + t) * 16 + row;
            if (n >= a.N) continue;
            if constexpr (EPI == EPI_SLAB) {
                a.Yf[((size_t)kp * a.R + col) * a.ldy + n] = v;
            } else if constexpr (EPI == EPI_SLABFIN) {  // write-through: read by the tile group's last K part
                __hip_atomic_store(a.Yf + ((size_t)kp * a.R + col) * a.ldy + n, v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            } else {
                if (a.wscale) v = rnd<T>(rnd<T>(v) * ld(a.wscale, n));
                if (a.bias) v += ld(a.bias, n);
                if constexpr (EPI == EPI_STORE)
                    st(a.Y, (size_t)col * a.ldy + n, v);
                else
                    a.Yf[(size_t)col * a.ldy + n] = rnd<T>(v);
            }
        }
    }
    if constexpr (EPI == EPI_SLABFIN) {
        // hand-off in the write-through form (cdna_hip_programming.md split-K recipe, as the batch-1
        // GEMV's EPI_SLABFIN): sc1 partial stores drained by every wave, one relaxed agent ticket per
        // tile group, sc1 loads in the last arriver
        __shared__ int last_s;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            const int tk = __hip_atomic_fetch_add(a.tickets + gb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = tk == kparts - 1;
            if (last) __hip_atomic_store(a.tickets + gb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last_s = last;
        }
        __syncthreads();
        if (last_s) {
            // x = round(res + round(sum_kp partial + bias)) (llama.py:841-842; one rounding of the
            // linear output, like finalize_norm_kernel), then each (tile, row of X)'s sum of x^2 over
            // its 16 columns: o's low 4 bits index the column, so a 16-lane group is one tile row.
            // Every partial and residual load of the thread goes out before the first is used
            // (clamped indices, no load under a branch); kparts <= 8, 512 threads (host).
            constexpr int OPT = (NTM * 16 * 32 + 511) / 512;
            const int no = ntl * 16 * a.R;
            float pv[OPT][8], rv[OPT];
#pragma unroll
            for (int u = 0; u < OPT; ++u) {
                const int o0 = threadIdx.x + 512 * u, o = o0 < no ? o0 : no - 1;
                const int t = o / (16 * a.R), oo = o - t * 16 * a.R;
                const int col = oo >> 4, n = min((t0 + t) * 16 + (oo & 15), a.N - 1);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int qq = q < kparts ? q : kparts - 1;
                    pv[u][q] = __hip_atomic_load(a.Yf + ((size_t)qq * a.R + col) * a.ldy + n, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
                }
                rv[u] = ld(a.res, (size_t)col * a.ldr + n);
            }
#pragma unroll
            for (int u = 0; u < OPT; ++u) {
                const int o = threadIdx.x + 512 * u;
                const int t = o / (16 * a.R), oo = o - t * 16 * a.R;
                const int col = oo >> 4, row = oo & 15;
                const int n = (t0 + t) * 16 + row;
                const bool live = o < no && n < a.N;
                float y = 0.f;
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (q < kparts) y += pv[u][q];
                float x = 0.f;
                if (live) {
                    if (a.bias) y += ld(a.bias, n);
                    if (a.wscale) y = rnd<T>(rnd<T>(y) * ld(a.wscale, n));
                    x = rnd<T>(rv[u] + rnd<T>(y));
                    st(a.res_out, (size_t)col * a.ldro + n, x);
                }
                float sq = x * x;
#pragma unroll
                for (int m = 1; m < 16; m <<= 1) sq += __shfl_xor(sq, m);
                if (row == 0 && o < no) a.ss_out[(size_t)col * T_ + t0 + t] = sq;  // [R][N/16] (bsacc layout)
            }
        }
    }
    stamp();
}

// x = round(res + round(sum_kp slab[kp] + bias)) (llama.py:841-842 residual, the split-K sum in fp32
// rounded once like the reference's one linear output), then optionally xn = RMSNorm(x) with two
// roundings (llama.py:989-1000).  One 512-thread block per row: every thread's slab, residual and
// norm-weight loads (<= FN_CPT chunks of 8) are issued together, one round trip, then a block sum.
constexpr int FN_THREADS = 512, FN_CPT = 2;  // d <= 8 * FN_THREADS * FN_CPT
template <typename T>
__global__ __launch_bounds__(FN_THREADS) void finalize_norm_kernel(FinalizeArgs<T> a) {
    __shared__ float red_s[FN_THREADS / 64];
    const int r = blockIdx.x;
    float v[FN_CPT][8], wn[FN_CPT][8];
    float ss = 0.f;
    // the norm weights go out with the slab / residual loads (one round trip, not one per phase)
#pragma unroll
    for (int c = 0; c < FN_CPT; ++c) {
        const int i = 8 * (threadIdx.x + FN_THREADS * c);
        if (a.nw && i < a.d) load8(a.nw + i, wn[c]);
    }
    float x[FN_CPT][8];  // residual rows, also in flight before the slab adds
#pragma unroll
    for (int c = 0; c < FN_CPT; ++c) {
        const int i = 8 * (threadIdx.x + FN_THREADS * c);
        if (i < a.d) load8(a.res + (size_t)r * a.ldr + i, x[c]);
    }
    // slab sums, K parts in order (fp32 add order = the reference restatement's); eight (then
    // four) parts' loads issued before the adds that consume them -- at 8 K parts (the S2-Pro
    // slab linears) one round trip instead of two.  Chunk c = 1 only exists for d > 8 * FN_THREADS.
    float y[FN_CPT][8];
#pragma unroll
    for (int c = 0; c < FN_CPT; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) y[c][j] = 0.f;
    {
        int q = 0;
        auto batch = [&](auto NB) {
            constexpr int B = decltype(NB)::value;
            for (; q + B <= a.kparts; q += B) {
                f32x4_t p[B][FN_CPT][2];
#pragma unroll
                for (int u = 0; u < B; ++u)
#pragma unroll
                    for (int c = 0; c < FN_CPT; ++c) {
                        const int i = 8 * (threadIdx.x + FN_THREADS * c);
                        const float* sp = a.slab + ((size_t)(q + u) * a.R + r) * a.lds + (i < a.d ? i : 0);
                        p[u][c][0] = *reinterpret_cast<const f32x4_t*>(sp);
                        p[u][c][1] = *reinterpret_cast<const f32x4_t*>(sp + 4);
                    }
#pragma unroll
                for (int u = 0; u < B; ++u)
#pragma unroll
                    for (int c = 0; c < FN_CPT; ++c)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            y[c][j] += p[u][c][0][j];
                            y[c][4 + j] += p[u][c][1][j];
                        }
            }
        };
        if (a.d <= 8 * FN_THREADS && a.fin8) {
            // one chunk per thread: the eight parts' 16 loads fit the register budget
            for (; q + 8 <= a.kparts; q += 8) {
                f32x4_t p[8][2];
                const int i = 8 * (int)threadIdx.x;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const float* sp = a.slab + ((size_t)(q + u) * a.R + r) * a.lds + (i < a.d ? i : 0);
                    p[u][0] = *reinterpret_cast<const f32x4_t*>(sp);
                    p[u][1] = *reinterpret_cast<const f32x4_t*>(sp + 4);
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        y[0][j] += p[u][0][j];
                        y[0][4 + j] += p[u][1][j];
                    }
            }
        }
        batch(std::integral_constant<int, 4>{});
        for (; q < a.kparts; ++q) {
#pragma unroll
            for (int c = 0; c < FN_CPT; ++c) {
                const int i = 8 * (threadIdx.x + FN_THREADS * c);
                const float* sp = a.slab + ((size_t)q * a.R + r) * a.lds + (i < a.d ? i : 0);
                const f32x4_t p0 = *reinterpret_cast<const f32x4_t*>(sp);
                const f32x4_t p1 = *reinterpret_cast<const f32x4_t*>(sp + 4);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    y[c][j] += p0[j];
                    y[c][4 + j] += p1[j];
                }
            }
        }
    }
#pragma unroll
    for (int c = 0; c < FN_CPT; ++c) {
        const int i = 8 * (threadIdx.x + FN_THREADS * c);
        if (i < a.d) {
            if (a.bias) {
                float b[8];
                load8(a.bias + i, b);
#pragma unroll
                for (int j = 0; j < 8; ++j) y[c][j] += b[j];
            }
            if (a.wscale) {  // weight-only int8 linear output
                float sc[8];
                load8(a.wscale + i, sc);
#pragma unroll
                for (int j = 0; j < 8; ++j) y[c][j] = rnd<T>(rnd<T>(y[c][j]) * sc[j]);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                v[c][j] = rnd<T>(x[c][j] + rnd<T>(y[c][j]));
                ss += v[c][j] * v[c][j];
            }
            T* xo = a.x_out + (size_t)r * a.ldx + i;
#pragma unroll
            for (int j = 0; j < 8; ++j) st(xo, j, v[c][j]);
        }
    }
    if (!a.nw) return;
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red_s[threadIdx.x >> 6] = ss;
    __syncthreads();
    ss = 0.f;
#pragma unroll
    for (int w = 0; w < FN_THREADS / 64; ++w) ss += red_s[w];
    const float rs = 1.0f / sqrtf(ss / (float)a.d + a.eps);
#pragma unroll
    for (int c = 0; c < FN_CPT; ++c) {
        const int i = 8 * (threadIdx.x + FN_THREADS * c);
        if (i < a.d) {
            T* xn = a.xn_out + (size_t)r * a.ldxn + i;
#pragma unroll
            for (int j = 0; j < 8; ++j) st(xn, j, rnd<T>(rnd<T>(v[c][j] * rs) * wn[c][j]));
        }
    }
}

template <typename T, int SPW, int TPI>
void bs_go(hipStream_t s, const BstreamArgs<T>& a, int epi, int G, int NW) {
    dim3 grid(G), block(NW * 64);
    switch (epi) {
        case EPI_STORE: bstream_kernel<T, SPW, TPI, EPI_STORE><<<grid, block, 0, s>>>(a); break;
        case EPI_SWIGLU8: bstream_kernel<T, SPW, TPI, EPI_SWIGLU8><<<grid, block, 0, s>>>(a); break;
        case EPI_F32: bstream_kernel<T, SPW, TPI, EPI_F32><<<grid, block, 0, s>>>(a); break;
        case EPI_SLAB: bstream_kernel<T, SPW, TPI, EPI_SLAB><<<grid, block, 0, s>>>(a); break;
        default: FMCHECK(false, "bstream: unsupported epilogue");
    }
}

int bs_num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    }
    return n;
}

}  // namespace

// Geometry for one linear (bf16 numbers from scripts/bgemm_probe.hip, S2-Pro shapes):
//   whole-K epilogues: kparts 1, 16 waves, 5 k-steps per wave at K = 2560 (TPI 2);
//   EPI_SLAB: kparts 4 at K = 4096 (8 waves x 4 steps), kparts 8 at K = 9728 (8 waves x 4-5).
// SPW is the smallest instantiated ring width >= ceil(Sp / NW).  fp32 holds twice the VGPRs per
// fragment, so it runs TPI 1 (validation mode only).
// bsacc_kernel geometry: 8 waves per block, one block per CU; K parts (EPI_SLAB only) so that
// tiles * kparts is a whole number of grid rounds, at most NTM tiles per block
static BstreamPlan bsacc_plan(int N, int K, int R, int epi, size_t esz) {
    BstreamPlan p{};
    const int S = K / 32, tiles = (N + 15) / 16, G = bs_num_cus();
    if (R < 1 || R > 32 || K % 32 || S < 1 || esz != 2) return p;
    int kparts = 1;
    if (epi == EPI_SLAB || epi == EPI_SLABFIN) {
        int best = 1;
        double bw = 1e9;
        for (int k = 1; k <= 8; k *= 2) {
            if (S % k || S / k < 8) break;
            const double per = (double)tiles * k / G, waste = std::ceil(per) / per;
            if (std::ceil(per) <= 6 && waste < bw - 1e-3) {
                bw = waste;
                best = k;
            }
        }
        kparts = best;
        const int fk = fm_tuning().bsacc_kparts;  // developer override (subject to the same limits)
        if (fk > 0 && S % fk == 0 && S / fk >= 8 && ((tiles * fk + G - 1) / G) <= 6) kparts = fk;
    }
    const int Sp = S / kparts, NW = std::min(8, Sp);
    const int ntm = (tiles * kparts + G - 1) / G;
    const int spw_need = (Sp + NW - 1) / NW;
    int spw = 0;
    for (int c : {2, 5, 10})
        if (c >= spw_need) {
            spw = c;
            break;
        }
    if (!spw || ntm > 6) return p;
    p.ok = true;
    p.acc = 1;
    p.kparts = kparts;
    p.nw = NW;
    p.spw = spw;
    p.tpi = spw == 2 ? 4 : (spw == 5 ? 2 : 1);
    p.ntm = ntm <= 2 ? 2 : (ntm <= 3 ? 3 : (ntm <= 5 ? 5 : 6));
    p.grid = std::min(G, tiles * kparts) / kparts * kparts;
    return p;
}

BstreamPlan bstream_plan(int N, int K, int R, int epi, size_t esz) {
    BstreamPlan p{};
    const FmTuning& tu = fm_tuning();
    if (tu.bstream_acc) {
        p = bsacc_plan(N, K, R, epi, esz);
        if (p.ok) return p;
    }
    const int S = K / 32, tiles = (N + 15) / 16;
    if (R < 1 || R > 32 || K % 32 || S < 1) return p;
    int kparts = 1;
    if (epi == EPI_SLAB) {
        kparts = tu.bstream_kparts > 0 ? tu.bstream_kparts : (S >= 256 ? 8 : (S >= 128 ? 4 : (S >= 64 ? 2 : 1)));
        while (kparts > 1 && (S % kparts || S / kparts < 8)) kparts /= 2;
    }
    const int Sp = S / kparts;
    int NW = epi == EPI_SLAB ? 8 : 16;
    if (tu.bstream_nw > 0) NW = tu.bstream_nw;
    NW = std::min(NW, Sp);
    const int spw_need = (Sp + NW - 1) / NW;
    const int spws[] = {2, 4, 5, 8};
    int spw = 0;
    for (int c : spws)
        if (c >= spw_need) {
            spw = c;
            break;
        }
    if (!spw) return p;
    int G = std::min(bs_num_cus(), tiles * kparts);
    G = std::max(kparts, G / kparts * kparts);
    p.ok = true;
    p.kparts = kparts;
    p.nw = NW;
    p.spw = spw;
    p.tpi = (esz == 2 && spw <= 5) ? 2 : 1;
    p.grid = G;
    return p;
}

// > 64 KiB of dynamic LDS needs the kernel attribute, which must not be set inside a stream capture
// (the first batched frame is captured): bsacc_init sets it for every instantiation up front
template <typename T, int SPW, int TPI, int NTM, int EPI, int PRO>
static void bsacc_attr() {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bsacc_kernel<T, SPW, TPI, NTM, EPI, PRO>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}
template <typename T, int SPW, int TPI, int NTM>
static void bsacc_attr_all() {
    bsacc_attr<T, SPW, TPI, NTM, EPI_STORE, PRO_PLAIN>();
    bsacc_attr<T, SPW, TPI, NTM, EPI_STORE, PRO_PRENORM>();
    bsacc_attr<T, SPW, TPI, NTM, EPI_SWIGLU8, PRO_PLAIN>();
    bsacc_attr<T, SPW, TPI, NTM, EPI_SWIGLU8, PRO_PRENORM>();
    bsacc_attr<T, SPW, TPI, NTM, EPI_F32, PRO_PLAIN>();
    bsacc_attr<T, SPW, TPI, NTM, EPI_SLAB, PRO_PLAIN>();
    bsacc_attr<T, SPW, TPI, NTM, EPI_SLABFIN, PRO_PLAIN>();
}
template <typename T, int SPW, int TPI, int NTM, int EPI, int PRO>
static void bsacc_launch(hipStream_t s, const BstreamArgs<T>& a, int G, int NW) {
    const size_t lds = (size_t)NTM * NW * 2 * 64 * sizeof(f32x4_t);
    bsacc_kernel<T, SPW, TPI, NTM, EPI, PRO><<<dim3(G), dim3(NW * 64), lds, s>>>(a);
}
template <typename T, int SPW, int TPI, int NTM>
static void bsacc_go(hipStream_t s, const BstreamArgs<T>& a, int epi, int G, int NW) {
    const bool pre = a.pro == PRO_PRENORM;
    FMCHECK(!pre || (a.ss_in && a.nw && a.R <= 32 && NW == 8 && a.K / 16 <= 192 && (epi == EPI_STORE || epi == EPI_SWIGLU8)),
            "bsacc: PRO_PRENORM needs ss_in / nw, R <= 32, 8 waves, K <= 3072 and a STORE or SWIGLU8 epilogue");
    FMCHECK(epi != EPI_SLABFIN || (a.res && a.res_out && a.ss_out && a.tickets && a.Yf && NW == 8 && a.kparts <= 8),
            "bsacc: EPI_SLABFIN needs res / res_out / ss_out / tickets / partials, 8 waves, <= 8 K parts");
    switch (epi) {
        case EPI_STORE:
            if (pre) bsacc_launch<T, SPW, TPI, NTM, EPI_STORE, PRO_PRENORM>(s, a, G, NW);
            else bsacc_launch<T, SPW, TPI, NTM, EPI_STORE, PRO_PLAIN>(s, a, G, NW);
            break;
        case EPI_SWIGLU8:
            if (pre) bsacc_launch<T, SPW, TPI, NTM, EPI_SWIGLU8, PRO_PRENORM>(s, a, G, NW);
            else bsacc_launch<T, SPW, TPI, NTM, EPI_SWIGLU8, PRO_PLAIN>(s, a, G, NW);
            break;
        case EPI_F32: bsacc_launch<T, SPW, TPI, NTM, EPI_F32, PRO_PLAIN>(s, a, G, NW); break;
        case EPI_SLAB: bsacc_launch<T, SPW, TPI, NTM, EPI_SLAB, PRO_PLAIN>(s, a, G, NW); break;
        case EPI_SLABFIN: bsacc_launch<T, SPW, TPI, NTM, EPI_SLABFIN, PRO_PLAIN>(s, a, G, NW); break;
        default: FMCHECK(false, "bsacc: unsupported epilogue");
    }
}

template <typename T> bool launch_bstream(hipStream_t s, const BstreamArgs<T>& a0, int epi, const BstreamPlan& p) {
    if (!p.ok) return false;
    BstreamArgs<T> a = a0;
    a.kparts = p.kparts;
    a.dummy_tail = fm_tuning().bs_dummy;
    a.xfirst = fm_tuning().bs_xfirst;
    a.vec_epi = fm_tuning().bs_vec_epi;
    if (p.acc) {
        if constexpr (sizeof(T) == 2) {
            FMCHECK(epi != EPI_SWIGLU8 || a.N % 16 == 0, "bsacc: SwiGLU8 needs whole interleaved tiles");
#define BSA(SPW, TPI, NTM)                                      \
    if (p.spw == SPW && p.tpi == TPI && p.ntm == NTM) {         \
        bsacc_go<T, SPW, TPI, NTM>(s, a, epi, p.grid, p.nw);    \
        return true;                                            \
    }
            BSA(2, 4, 2) BSA(2, 4, 3) BSA(2, 4, 5) BSA(2, 4, 6) BSA(5, 2, 2) BSA(5, 2, 3) BSA(5, 2, 5)
            BSA(5, 2, 6) BSA(10, 1, 2) BSA(10, 1, 3) BSA(10, 1, 5) BSA(10, 1, 6)
#undef BSA
        }
        return false;
    }
    FMCHECK(epi == EPI_SLAB || p.kparts == 1, "bstream: split K only into slabs");
    FMCHECK(epi != EPI_SWIGLU8 || a.N % 16 == 0, "bstream: SwiGLU8 needs whole interleaved tiles");
#define BSG(SPW, TPI)                                    \
    if (p.spw == SPW && p.tpi == TPI) {                  \
        bs_go<T, SPW, TPI>(s, a, epi, p.grid, p.nw);     \
        return true;                                     \
    }
    BSG(2, 2) BSG(4, 2) BSG(5, 2) BSG(2, 1) BSG(4, 1) BSG(5, 1) BSG(8, 1)
#undef BSG
    return false;
}

void bsacc_init() {
    static bool done = false;
    if (done) return;
    done = true;
#define BSI(SPW, TPI, NTM) bsacc_attr_all<bf16_t, SPW, TPI, NTM>();
    BSI(2, 4, 2) BSI(2, 4, 3) BSI(2, 4, 5) BSI(2, 4, 6) BSI(5, 2, 2) BSI(5, 2, 3) BSI(5, 2, 5) BSI(5, 2, 6)
    BSI(10, 1, 2) BSI(10, 1, 3) BSI(10, 1, 5) BSI(10, 1, 6)
#undef BSI
    (void)hipGetLastError();  // an attribute the runtime declines must not linger as the sticky error
}

// The same finalise + RMSNorm with each row split over `ch` blocks (R * ch blocks: 256 CUs busy at
// R = 32, ch = 8, instead of 32): every block loads only its chunk's K-part slabs, residual and norm
// weights (one round trip), writes x, and publishes its chunk's sum of squares write-through; the
// row's ch blocks then meet on an arrival counter (all resident: R * ch <= 1024 small blocks), read
// the ch partial sums in chunk order (a fixed fp32 order) and normalise their chunk.  The last block
// of a row to read resets the row's two counters, so the next launch starts from zero.
constexpr int FS_THREADS = 64;
template <typename T>
__global__ __launch_bounds__(FS_THREADS) void finalize_split_kernel(FinalizeArgs<T> a) {
    typedef __attribute__((address_space(1))) int g_i32;
    typedef __attribute__((address_space(1))) float g_f32;
    const int r = blockIdx.x / a.ch, c = blockIdx.x - r * a.ch;
    const int per = (a.d / 8 + a.ch - 1) / a.ch;  // 8-element items per chunk
    const int it = c * per + (int)threadIdx.x;    // this thread's item (one per thread: per <= 64)
    const bool live = (int)threadIdx.x < per && it < a.d / 8;
    const int i = 8 * (live ? it : 0);
    float wn[8], x[8], y[8], b[8], v[8];
    if (a.nw) load8(a.nw + i, wn);
    load8(a.res + (size_t)r * a.ldr + i, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = 0.f;
    for (int q = 0; q < a.kparts; ++q) {  // K parts in order (the restatement's fp32 add order)
        const float* sp = a.slab + ((size_t)q * a.R + r) * a.lds + i;
        const f32x4_t p0 = *reinterpret_cast<const f32x4_t*>(sp);
        const f32x4_t p1 = *reinterpret_cast<const f32x4_t*>(sp + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            y[j] += p0[j];
            y[4 + j] += p1[j];
        }
    }
    if (a.bias) {
        load8(a.bias + i, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] += b[j];
    }
    if (a.wscale) {
        float sc[8];
        load8(a.wscale + i, sc);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = rnd<T>(rnd<T>(y[j]) * sc[j]);
    }
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        v[j] = rnd<T>(x[j] + rnd<T>(y[j]));
        ss += v[j] * v[j];
    }
    if (live) {
        T* xo = a.x_out + (size_t)r * a.ldx + i;
#pragma unroll
        for (int j = 0; j < 8; ++j) st(xo, j, v[j]);
    }
    if (!a.nw) return;
    ss = wave_sum(live ? ss : 0.f);
    int* arrive = a.cnt + 2 * r;
    if (threadIdx.x == 0) {
        __hip_atomic_store((g_f32*)(a.ss_part + (size_t)r * a.ch + c), ss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add((g_i32*)arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (unsigned spin = 0;; ++spin) {  // bounded: every block of the row is resident
            if (__hip_atomic_load((g_i32*)arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= a.ch) break;
            if (spin > (1u << 22)) {  // reported (the host throws and resets the counters), never silent
                if (a.err) __hip_atomic_store((g_i32*)a.err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __builtin_amdgcn_wave_barrier();
    float tot = 0.f;
    for (int q = 0; q < a.ch; ++q)  // chunk order: the same sum in every block of the row
        tot += __hip_atomic_load((g_f32*)(a.ss_part + (size_t)r * a.ch + q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float rs = 1.0f / sqrtf(tot / (float)a.d + a.eps);
    if (live) {
        T* xn = a.xn_out + (size_t)r * a.ldxn + i;
#pragma unroll
        for (int j = 0; j < 8; ++j) st(xn, j, rnd<T>(rnd<T>(v[j] * rs) * wn[j]));
    }
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (__hip_atomic_fetch_add((g_i32*)(arrive + 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.ch - 1) {
            __hip_atomic_store((g_i32*)arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store((g_i32*)(arrive + 1), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <typename T> void launch_finalize_norm(hipStream_t s, const FinalizeArgs<T>& a) {
    FMCHECK(a.d % 8 == 0 && a.d <= 8 * FN_THREADS * FN_CPT && a.lds % 4 == 0, "finalize_norm: bad row width");
    if (a.ch > 1 && a.cnt && a.ss_part && a.R * a.ch <= 1024 && (a.d / 8 + a.ch - 1) / a.ch <= FS_THREADS) {
        finalize_split_kernel<T><<<a.R * a.ch, FS_THREADS, 0, s>>>(a);
        return;
    }
    FinalizeArgs<T> b = a;
    b.fin8 = fm_tuning().fin8;
    finalize_norm_kernel<T><<<a.R, FN_THREADS, 0, s>>>(b);
}

template bool launch_bstream<bf16_t>(hipStream_t, const BstreamArgs<bf16_t>&, int, const BstreamPlan&);
template bool launch_bstream<float>(hipStream_t, const BstreamArgs<float>&, int, const BstreamPlan&);
template void launch_finalize_norm<bf16_t>(hipStream_t, const FinalizeArgs<bf16_t>&);
template void launch_finalize_norm<float>(hipStream_t, const FinalizeArgs<float>&);

// fm_gemv.hip -- the decode-step weight-streaming kernel for R <= 8 rows (streams per GPU).
//
// Y[r][n] = sum_k X'[r][k] W[n][k] with the producer/consumer seams of a pre-norm block fused:
//   prologue  PRO_PLAIN   X' = X
//             PRO_NORM    X' = rmsnorm(X)                       (llama.py:989-1000)
//             PRO_RESNORM x  = round(res + round(sum_s slab_s))  (the previous linear's split-K
//                         X' = rmsnorm(x)                        partials + residual add,
//                                                                 llama.py:841-842); block 0
//                                                                 stores x (and X') for later
//   epilogue  EPI_STORE (T, +bias) | EPI_SWIGLU (round(silu(round(w1 x)))*round(w3 x))
//             | EPI_F32 (logits) | EPI_SLAB (fp32 split-K partial, consumed by the next prologue)
//
// Geometry: block = 8 waves, 16 weight rows (one 16x16x32 MFMA row tile; the R<=8 streams are
// MFMA columns), grid = (N/16, KSB).  Wave w takes the block's 32-wide k-steps w, w+8, ...,
// so the 8 waves read 512 contiguous bytes of each row per sweep.  A ring of U register
// fragments keeps U weight loads in flight per wave (prefetch distance U, non-temporal loads:
// each weight byte is read exactly once per frame).  X' is staged once per block in LDS.
#include "fm_kernels.h"

template <typename T> struct GFrag;
template <> struct GFrag<bf16_t> {
    typedef u32x4_t f;
    static __device__ __forceinline__ f load_w(const bf16_t* blk, int lane) {
        return *reinterpret_cast<const u32x4_t*>(blk + lane * 8);
    }
    static __device__ __forceinline__ f load_lds(const bf16_t* p) { return *reinterpret_cast<const u32x4_t*>(p); }
    static __device__ __forceinline__ f32x4_t mma(f a, f b, f32x4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                       __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
    }
};
template <> struct GFrag<float> {
    struct f {
        f32x4_t lo, hi;
    };
    static __device__ __forceinline__ f load_w(const float* blk, int lane) {
        f v;
        v.lo = *reinterpret_cast<const f32x4_t*>(blk + lane * 4);
        v.hi = *reinterpret_cast<const f32x4_t*>(blk + 256 + lane * 4);
        return v;
    }
    static __device__ __forceinline__ f load_lds(const float* p) {
        f v;
        v.lo = *reinterpret_cast<const f32x4_t*>(p);
        v.hi = *reinterpret_cast<const f32x4_t*>(p + 4);
        return v;
    }
    static __device__ __forceinline__ f32x4_t mma(f a, f b, f32x4_t c) {
#pragma unroll
        for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo[j], b.lo[j], c, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi[j], b.hi[j], c, 0, 0, 0);
        return c;
    }
};

__device__ __forceinline__ float silu_g(float a) { return a / (1.0f + expf(-a)); }

// x value of the prologue at (row r, k) before normalisation
template <typename T, int PRO>
__device__ __forceinline__ float pro_x(const GemvArgs<T>& a, const T* xr, const T* resr, int r, int k) {
    if constexpr (PRO == PRO_RESNORM) {
        float s = 0.f;
        for (int q = 0; q < a.nslab; ++q) s += a.slab[((size_t)q * a.R + r) * a.slab_ld + k];
        return rnd<T>(ld(resr, k) + rnd<T>(s));
    } else {
        return ld(xr, k);
    }
}

template <typename T, int PRO, int EPI, int U>
__global__ __launch_bounds__(512) void gemv_kernel(GemvArgs<T> a) {
    using G = GFrag<T>;
    constexpr int NACC = (EPI == EPI_SWIGLU) ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = blockIdx.x * 16;
    const int ks = blockIdx.y;
    const int Kb = a.K / gridDim.y;  // host guarantees a multiple of 32
    const int kbeg = ks * Kb;
    const int R = a.R;
    const int xstride = Kb + 8;  // +16 B per row: conflict-free ds_read_b128 across rows
    T* xs = reinterpret_cast<T*>(smem);
    float* rstd = reinterpret_cast<float*>(smem + (size_t)R * xstride * sizeof(T));
    f32x4_t* red = reinterpret_cast<f32x4_t*>(rstd + 16);

    // ---------------- prologue: stage X'[r][kbeg .. kbeg+Kb) in LDS ---------------------------
    // 16-byte chunks of 8 elements; every thread issues its loads at once (one round trip).
    if constexpr (PRO == PRO_NORM || PRO == PRO_RESNORM) {
        __shared__ float red_s[16];
        const int nch = a.K >> 3;
        const bool writer = (blockIdx.x == 0 && ks == 0);
        for (int r = 0; r < R; ++r) {
            const int xi = a.xidx ? a.xidx[(size_t)r * a.xidx_ld + a.xidx_col] : r;
            const T* xr = a.X + (size_t)xi * a.ldx;
            const int ri = a.residx ? a.residx[(size_t)r * a.xidx_ld + a.xidx_col] : r;
            const T* resr = a.res ? a.res + (size_t)ri * a.ldr : nullptr;
            float xv[2][8];
            float ss = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c = threadIdx.x + 512 * j;
                if (c < nch) {
                    if constexpr (PRO == PRO_RESNORM) {
                        float rv[8], sv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                        load8(resr + 8 * c, rv);
                        for (int q = 0; q < a.nslab; ++q) {
                            const float* sp = a.slab + ((size_t)q * R + r) * a.slab_ld + 8 * c;
                            const f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(sp);
                            const f32x4_t s1 = *reinterpret_cast<const f32x4_t*>(sp + 4);
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                sv[u] += s0[u];
                                sv[4 + u] += s1[u];
                            }
                        }
#pragma unroll
                        for (int u = 0; u < 8; ++u) xv[j][u] = rnd<T>(rv[u] + rnd<T>(sv[u]));
                    } else {
                        load8(xr + 8 * c, xv[j]);
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) ss += xv[j][u] * xv[j][u];
                }
            }
            ss = block_sum(ss, red_s);
            const float rs = 1.0f / sqrtf(ss / (float)a.K + a.eps);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c = threadIdx.x + 512 * j;
                if (c >= nch) continue;
                const int k = 8 * c;
                const bool mine = k >= kbeg && k < kbeg + Kb;
                if (!mine && !writer) continue;
                float wv[8];
                load8(a.nw + k, wv);
                float xn[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) xn[u] = rnd<T>(rnd<T>(xv[j][u] * rs) * wv[u]);
                if (mine) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) st(xs, (size_t)r * xstride + (k - kbeg) + u, xn[u]);
                }
                if (writer) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        if constexpr (PRO == PRO_RESNORM) st(a.res_out, (size_t)r * a.ldro + k + u, xv[j][u]);
                        if (a.xn_out) st(a.xn_out, (size_t)r * a.ldxo + k + u, xn[u]);
                    }
                }
            }
            __syncthreads();
        }
    } else {
        const int nchs = Kb >> 3;
        constexpr int VB = 16 / sizeof(T);  // elements per 16 B
        for (int idx = threadIdx.x; idx < R * nchs * (8 / VB); idx += 512) {
            const int r = idx / (nchs * (8 / VB)), c = idx - r * (nchs * (8 / VB));
            *reinterpret_cast<u32x4_t*>(xs + (size_t)r * xstride + VB * c) =
                *reinterpret_cast<const u32x4_t*>(a.X + (size_t)r * a.ldx + kbeg + VB * c);
        }
    }
    __syncthreads();

    // ---------------- main loop: ring of U weight-fragment loads per wave ------------------------
    // packed weights (fm_kernels.h): the (tile, step) fragment is 512 contiguous elements; wave w
    // streams a contiguous run of the block's steps.
    const int r = lane & 15, g = lane >> 4;
    const int S = a.K >> 5, Sb = Kb >> 5, sb0 = ks * Sb;
    const int wa = (wave * Sb) >> 3, wb = ((wave + 1) * Sb) >> 3, nmy = wb - wa;
    const T* wp = a.W + ((size_t)blockIdx.x * S + sb0 + wa) * 512;
    const T* wp2 = (EPI == EPI_SWIGLU) ? a.W2 + ((size_t)blockIdx.x * S + sb0 + wa) * 512 : nullptr;
    const T* xp = xs + (size_t)(r < R ? r : R - 1) * xstride + (size_t)wa * 32 + 8 * g;
    f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    if (nmy > 0) {
        typename G::f fa[U], fb[U];
        auto boff = [&](int i) { return (size_t)(i < nmy ? i : nmy - 1) * 512; };  // clamped tail
#pragma unroll
        for (int u = 0; u < U; ++u) {
            fa[u] = G::load_w(wp + boff(u), lane);
            if constexpr (NACC == 2) fb[u] = G::load_w(wp2 + boff(u), lane);
        }
        for (int i = 0; i < nmy; i += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (i + u < nmy) {
                    const typename G::f xb = G::load_lds(xp + (size_t)(i + u) * 32);
                    acc0 = G::mma(fa[u], xb, acc0);
                    if constexpr (NACC == 2) acc1 = G::mma(fb[u], xb, acc1);
                }
                fa[u] = G::load_w(wp + boff(i + u + U), lane);
                if constexpr (NACC == 2) fb[u] = G::load_w(wp2 + boff(i + u + U), lane);
            }
        }
    }
    red[(0 * 8 + wave) * 64 + lane] = acc0;
    if constexpr (NACC == 2) red[(1 * 8 + wave) * 64 + lane] = acc1;
    __syncthreads();

    // ---------------- epilogue: 16 rows x R cols; C/D map row = 4*(lane>>4)+i, col = lane&15 ---
    for (int o = threadIdx.x; o < 256; o += 512) {
        const int i = o >> 6, ln = o & 63;
        const int n = n0 + 4 * (ln >> 4) + i;
        const int col = ln & 15;
        if (col >= R || n >= a.N) continue;
        float v0 = 0.f, v1 = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            v0 += red[(0 * 8 + w) * 64 + ln][i];
            if constexpr (NACC == 2) v1 += red[(1 * 8 + w) * 64 + ln][i];
        }
        if constexpr (EPI == EPI_SLAB) {
            if (a.bias && ks == 0) v0 += ld(a.bias, n);
            a.Yf[((size_t)ks * R + col) * a.ldy + n] = v0;
        } else {
            if (a.bias) v0 += ld(a.bias, n);
            const size_t yi = (size_t)col * a.ldy + n;
            if constexpr (EPI == EPI_STORE) {
                st(a.Y, yi, v0);
            } else if constexpr (EPI == EPI_SWIGLU) {
                const float ga = rnd<T>(v0), ub = rnd<T>(v1);
                st(a.Y, yi, rnd<T>(silu_g(ga)) * ub);
            } else {
                a.Yf[yi] = rnd<T>(v0);
            }
        }
    }
}

template <typename T, int PRO, int EPI>
static void gemv_go(hipStream_t s, const GemvArgs<T>& a, int ksb) {
    dim3 grid(FM_CEIL(a.N, 16), ksb);
    const int Kb = a.K / ksb;
    const size_t lds = gemv_lds_bytes(a.R, Kb, sizeof(T));
    gemv_kernel<T, PRO, EPI, 4><<<grid, 512, lds, s>>>(a);
}

template <typename T> void launch_gemv(hipStream_t s, const GemvArgs<T>& a, int pro, int epi, int ksb) {
#define GO(P, E)                                           \
    if (pro == P && epi == E) {                            \
        gemv_go<T, P, E>(s, a, ksb);                       \
        return;                                            \
    }
    GO(PRO_PLAIN, EPI_STORE) GO(PRO_PLAIN, EPI_SLAB) GO(PRO_PLAIN, EPI_F32) GO(PRO_PLAIN, EPI_SWIGLU)
    GO(PRO_NORM, EPI_STORE) GO(PRO_NORM, EPI_SWIGLU) GO(PRO_NORM, EPI_F32) GO(PRO_NORM, EPI_SLAB)
    GO(PRO_RESNORM, EPI_STORE) GO(PRO_RESNORM, EPI_SWIGLU) GO(PRO_RESNORM, EPI_F32)
    GO(PRO_RESNORM, EPI_SLAB)
#undef GO
}

template void launch_gemv<bf16_t>(hipStream_t, const GemvArgs<bf16_t>&, int, int, int);
template void launch_gemv<float>(hipStream_t, const GemvArgs<float>&, int, int, int);

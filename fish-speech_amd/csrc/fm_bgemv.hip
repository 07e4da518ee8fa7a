// fm_bgemv.hip -- decode-step weight streaming for 8 < R <= 32 rows (batched streams, BASELINE
// config 3: B = 32 concurrent utterances per GPU).
//
// Y[r][n] = sum_k X[r][k] W[n][k] (+ bias), epilogue STORE | RESID (Y = res + round(y)) | F32
// (llama.py:838-843 residual, 978-986 / 454-455 linears).  At B = 32 a decode linear still does
// only 32 flop per weight byte, so it is an HBM stream like the batch-1 GEMV (fm_gemv.hip), not a
// GEMM: every weight fragment (16 rows x 32 k, 1 KiB, MFMA A-operand order, fm_kernels.h) is read
// once and multiplied against one or two 16-column groups of X (the streams).
//
// Geometry: block = 8 waves and TPB 16-row tiles (TPB in {1, 2, 4}); wave w streams tile
// (w % TPB) over k-part (w / TPB) of the block's K slice through a branch-free ring of U register
// fragments, issued BEFORE the X slice is staged into LDS, so the staging hides under the weight
// flight.  X is staged once per block and shared by its TPB tiles (X bytes per weight byte =
// R / (16 TPB)).  grid = (tiles / TPB, ksb); ksb > 1 keeps the staged slice within LDS and the
// grid over the CUs: fp32 slice partials are stored write-through (sc1), drained, and the block's
// last-arriving slice (relaxed agent ticket) sums them in slice order and runs the epilogue
// (cdna_hip_programming.md split-K recipe; same hand-off as gemv_kernel EPI_SLABFIN).
#include "fm_kernels.h"
#include "fm_runtime.h"

namespace {

template <typename T> struct BFrag;
template <> struct BFrag<bf16_t> {
    typedef u32x4_t f;
    static __device__ __forceinline__ f load_w(const bf16_t* blk, int lane) {
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(blk + lane * 8));
    }
    static __device__ __forceinline__ f load_lds(const bf16_t* p) { return *reinterpret_cast<const u32x4_t*>(p); }
    static __device__ __forceinline__ f32x4_t mma(f a, f b, f32x4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                       __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
    }
};
template <> struct BFrag<float> {
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
    // lane l holds k = 8*(l>>4) + j of a 32-wide k block; MFMA j covers {8g + j}: exact f32
    static __device__ __forceinline__ f32x4_t mma(f a, f b, f32x4_t c) {
#pragma unroll
        for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo[j], b.lo[j], c, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi[j], b.hi[j], c, 0, 0, 0);
        return c;
    }
};

constexpr int BG_WAVES = 8;

template <typename T, int EPI>
__device__ __forceinline__ void bgemv_epi(const BgemvArgs<T>& a, int n, int col, float v) {
    const size_t yi = (size_t)col * a.ldy + n;
    if (a.bias) v += ld(a.bias, n);
    if constexpr (EPI == EPI_STORE) {
        st(a.Y, yi, v);
    } else if constexpr (EPI == EPI_RESID) {
        st(a.Y, yi, ld(a.res, (size_t)col * a.ldr + n) + rnd<T>(v));
    } else {  // EPI_F32: logits as fp32 holding the T-rounded value
        a.Yf[yi] = rnd<T>(v);
    }
}

template <typename T, int EPI, int NCG, int U>
__global__ __launch_bounds__(BG_WAVES * 64) void bgemv_kernel(BgemvArgs<T> a) {
    using G = BFrag<T>;
    constexpr int NTH = BG_WAVES * 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int TPB = a.tpb, parts = BG_WAVES / TPB;
    const int ksb = gridDim.y, ks = blockIdx.y;
    const int S = a.K >> 5;                 // k-steps of the whole row
    const int Sb = S / ksb, sb0 = ks * Sb;  // host: S % ksb == 0
    const int Kb = Sb * 32, kbeg = sb0 * 32;
    const int R = a.R;
    const int xstride = Kb + 8;  // +16 B per row: conflict-free ds_read_b128 across rows
    T* xs = reinterpret_cast<T*>(smem);
    f32x4_t* red = reinterpret_cast<f32x4_t*>(smem + (size_t)R * xstride * sizeof(T));  // [waves][NCG][64]
    int* flag = reinterpret_cast<int*>(red + BG_WAVES * NCG * 64);

    const int tl = wave % TPB, part = wave / TPB;
    const int tile = blockIdx.x * TPB + tl;
    const int tiles = (a.N + 15) >> 4;
    const bool live = tile < tiles;
    const int wa = (part * Sb) / parts, wb = ((part + 1) * Sb) / parts, nmy = live ? wb - wa : 0;
    const int ilast = nmy > 0 ? nmy - 1 : 0;
    const T* wrun = a.W + ((size_t)(live ? tile : 0) * S + sb0 + wa) * 512;
    typename G::f fa[U];
    // branch-free ring: a load under a branch would drain vmcnt(0) before every MFMA, so tail slots
    // re-load the run's last fragment (a cache hit) instead of being predicated off
    auto issue = [&](int i, int u) { fa[u] = G::load_w(wrun + (size_t)(i < ilast ? i : ilast) * 512, lane); };
#pragma unroll
    for (int u = 0; u < U; ++u) issue(u, u);

    // X[0..R)[kbeg, kbeg + Kb) -> LDS in 16-B chunks (under the weight flight): every thread's
    // first XPRE chunks are loaded before any is stored (one round trip, not one per chunk)
    {
        constexpr int CE = 16 / sizeof(T), XPRE = 12;
        const int nch = Kb / CE, nitem = R * nch;
        u32x4_t xc[XPRE];
#pragma unroll
        for (int q = 0; q < XPRE; ++q) {
            int it = threadIdx.x + NTH * q;
            it = it < nitem ? it : nitem - 1;  // clamped: no branch around the load
            const int rr = it / nch, cc = it - rr * nch;
            xc[q] = *reinterpret_cast<const u32x4_t*>(a.X + (size_t)rr * a.ldx + kbeg + cc * CE);
        }
#pragma unroll
        for (int q = 0; q < XPRE; ++q) {
            int it = threadIdx.x + NTH * q;
            it = it < nitem ? it : nitem - 1;  // the clamped tail re-stores the last chunk (same value)
            const int rr = it / nch, cc = it - rr * nch;
            *reinterpret_cast<u32x4_t*>(xs + (size_t)rr * xstride + cc * CE) = xc[q];
        }
        for (int it = threadIdx.x + NTH * XPRE; it < nitem; it += NTH) {
            const int rr = it / nch, cc = it - rr * nch;
            *reinterpret_cast<u32x4_t*>(xs + (size_t)rr * xstride + cc * CE) =
                *reinterpret_cast<const u32x4_t*>(a.X + (size_t)rr * a.ldx + kbeg + cc * CE);
        }
    }
    __syncthreads();

    const int r = lane & 15, g = lane >> 4;
    const T* xp0 = xs + (size_t)(r < R ? r : R - 1) * xstride + (size_t)wa * 32 + 8 * g;
    const T* xp1 = xs + (size_t)(16 + r < R ? 16 + r : R - 1) * xstride + (size_t)wa * 32 + 8 * g;
    f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < nmy; i += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + u < nmy) {
                acc0 = G::mma(fa[u], G::load_lds(xp0 + (size_t)(i + u) * 32), acc0);
                if constexpr (NCG == 2) acc1 = G::mma(fa[u], G::load_lds(xp1 + (size_t)(i + u) * 32), acc1);
            }
            issue(i + u + U, u);
        }
    }
    red[(wave * NCG + 0) * 64 + lane] = acc0;
    if constexpr (NCG == 2) red[(wave * NCG + 1) * 64 + lane] = acc1;
    __syncthreads();

    // block outputs: TPB tiles x 16 rows x R cols; C/D map: row = 4*(lane>>4)+i, col = lane&15
    const int nout = TPB * 16 * R;
    for (int o = threadIdx.x; o < nout; o += NTH) {
        const int t = o / (16 * R), rem = o - t * 16 * R, row = rem / R, col = rem - row * R;
        const int n = (blockIdx.x * TPB + t) * 16 + row;
        if (n >= a.N) continue;
        const int cg = col >> 4, ln = 16 * (row >> 2) + (col & 15), i = row & 3;
        float v = 0.f;
        for (int p = 0; p < parts; ++p) v += red[((p * TPB + t) * NCG + cg) * 64 + ln][i];
        if (ksb == 1) {
            bgemv_epi<T, EPI>(a, n, col, v);
        } else {
            __hip_atomic_store(a.part + ((size_t)ks * R + col) * a.N + n, v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (ksb == 1) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int tk = __hip_atomic_fetch_add(a.tickets + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = tk == ksb - 1;
        if (last) __hip_atomic_store(a.tickets + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    for (int o = threadIdx.x; o < nout; o += NTH) {
        const int t = o / (16 * R), rem = o - t * 16 * R, row = rem / R, col = rem - row * R;
        const int n = (blockIdx.x * TPB + t) * 16 + row;
        if (n >= a.N) continue;
        float v = 0.f;
        for (int q = 0; q < ksb; ++q)
            v += __hip_atomic_load(a.part + ((size_t)q * R + col) * a.N + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bgemv_epi<T, EPI>(a, n, col, v);
    }
}

template <typename T, int EPI, int NCG, int U>
void bgemv_launch(hipStream_t s, const BgemvArgs<T>& a, dim3 grid, size_t lds) {
    static bool attr = false;  // > 64 KiB of dynamic LDS must be opted into once per kernel
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bgemv_kernel<T, EPI, NCG, U>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    bgemv_kernel<T, EPI, NCG, U><<<grid, BG_WAVES * 64, lds, s>>>(a);
}

template <typename T, int EPI>
void bgemv_go(hipStream_t s, const BgemvArgs<T>& a, dim3 grid, size_t lds) {
    const int u = fm_tuning().bgemv_u;
    if (a.R <= 16) {
        if (u == 4) bgemv_launch<T, EPI, 1, 4>(s, a, grid, lds);
        else bgemv_launch<T, EPI, 1, 8>(s, a, grid, lds);
    } else {
        if (u == 4) bgemv_launch<T, EPI, 2, 4>(s, a, grid, lds);
        else bgemv_launch<T, EPI, 2, 8>(s, a, grid, lds);
    }
}

}  // namespace

BgemvPlan bgemv_plan(int N, int K, int R, size_t esz) {
    const FmTuning& tu = fm_tuning();
    BgemvPlan p;
    const int tiles = (N + 15) / 16, S = K / 32;
    // tiles per block (X staged once for TPB tiles), then K slices: X slice within the LDS
    // budget, the grid over the CUs, and at least two k-steps per wave
    p.tpb = 1;
    while (2 * p.tpb <= tu.bgemv_tpb && tiles >= 2 * p.tpb) p.tpb *= 2;
    const int nbx = (tiles + p.tpb - 1) / p.tpb, parts = 8 / p.tpb;
    p.ksb = 1;
    auto fits = [&](int k) { return (size_t)R * (K / k + 8) * esz <= (size_t)tu.bgemv_lds_kb * 1024; };
    while ((!fits(p.ksb) || nbx * p.ksb < tu.bgemv_fill) && S % (2 * p.ksb) == 0 && S / (2 * p.ksb) >= 2 * parts)
        p.ksb *= 2;
    return p;
}

template <typename T> void launch_bgemv(hipStream_t s, const BgemvArgs<T>& a0, int epi) {
    FMCHECK(a0.R > 0 && a0.R <= 32 && a0.K % 32 == 0, "bgemv: R must be in [1, 32], K a multiple of 32");
    BgemvArgs<T> a = a0;
    const BgemvPlan p = bgemv_plan(a.N, a.K, a.R, sizeof(T));
    a.tpb = p.tpb;
    const int S = a.K / 32;
    FMCHECK(S % p.ksb == 0, "bgemv: K slices must be whole k-steps");
    FMCHECK(p.ksb == 1 || (a.part && a.tickets && (size_t)p.ksb * a.R * a.N <= LINEAR_PART_CAP),
            "bgemv: split-K needs the partial buffer and tickets");
    const int tiles = (a.N + 15) / 16;
    dim3 grid((tiles + p.tpb - 1) / p.tpb, p.ksb);
    const int Kb = a.K / p.ksb, ncg = a.R > 16 ? 2 : 1;
    const size_t lds = (size_t)a.R * (Kb + 8) * sizeof(T) + (size_t)BG_WAVES * ncg * 64 * 16 + 16;
    FMCHECK(lds <= 160 * 1024, "bgemv: LDS budget exceeded");
    switch (epi) {
        case EPI_STORE: bgemv_go<T, EPI_STORE>(s, a, grid, lds); break;
        case EPI_RESID: bgemv_go<T, EPI_RESID>(s, a, grid, lds); break;
        case EPI_F32: bgemv_go<T, EPI_F32>(s, a, grid, lds); break;
        default: FMCHECK(false, "bgemv: unsupported epilogue");
    }
}

template void launch_bgemv<bf16_t>(hipStream_t, const BgemvArgs<bf16_t>&, int);
template void launch_bgemv<float>(hipStream_t, const BgemvArgs<float>&, int);

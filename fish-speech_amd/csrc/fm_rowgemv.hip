// fm_rowgemv.hip -- batch-1 row-block GEMV for the decode linears whose 16-row tile grids leave
// CUs idle or unbalanced.
//
// wo and w2 of a decode layer (TransformerBlock.forward, /root/reference/fish_speech/models/
// text2semantic/llama.py:838-843: h = x + attention(...), out = h + feed_forward(...)) have
// N = dim = 2560 output rows at S2-Pro shapes, and wqkv N = 6144 (Attention.forward, :883-890).  On
// the 16-row MFMA tile kernel (fm_gemv.hip) that is 160 workgroups for 256 CUs (96 CUs idle, each
// busy CU streaming 131 KiB / 311 KiB at the ~26 GB/s per CU its loads in flight sustain) and 384
// workgroups (half the CUs doing two tiles).  Here one 256-thread block owns RP consecutive rows
// (wo / w2: RP = 2, 1280 blocks = 5 per CU; wqkv: RP = 8, 768 blocks = 3 per CU) and reads them
// straight from the row-major weight: for each 256-k chunk of its wave's K range a lane loads 4 bf16
// of each of the RP rows and the matching 4 x values (coalesced 512-B wave loads) and accumulates
// two v_dot2c_f32_bf16 per row.  The whole run of a wave is in flight at once (U chunks,
// U = ceil(K / 256 / 4) <= 12), so there is no ring refill.  No MFMA: at one activation row the
// matrix cores would do 1/16 useful work; the dot2 work is 2 VALU instructions per row per chunk.
//
// Prologue  PLAIN     x as loaded
//           PRENORM   x' = round(round(x * rs) * w_norm), rs = 1 / sqrt(mean(x^2) + eps) over the
//                     whole row (RMSNorm, llama.py:989-1000): each wave sums the squares of its
//                     chunks, one LDS exchange, every block computes the same statistic in the same
//                     order.  x and w_norm are loaded ahead of the weights (in-order vmcnt).
// Epilogue  FIN       y = round(res + round(acc + bias)) into res_out (fm_gemv.hip EPI_SLABFIN
//                     semantics, llama.py:841-842); its RMSNorm consumer takes the statistic from
//                     the row it stages (GemvArgs::ss_gran = 1), so no sums of squares are written
//           STORE     y = round(acc + bias) into Y (wqkv), plus the KV prefetch of fm_gemv.hip
//                     (GemvArgs::pf_kc): the next attention's cached K / V sectors pulled into L2.
#include "fm_common.h"
#include "fm_kernels.h"
#include "fm_runtime.h"

typedef __attribute__((ext_vector_type(2))) uint32_t u32x2_t;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;

// acc += w . x over 4 bf16 (two v_dot2c_f32_bf16); whole-vector bit casts (see fm_pass.hip dot8)
__device__ __forceinline__ float dot4(u32x2_t w, u32x2_t x, float acc) {
    const bf16x4_t wb = __builtin_bit_cast(bf16x4_t, w), xb = __builtin_bit_cast(bf16x4_t, x);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(wb, wb, 0, 1), __builtin_shufflevector(xb, xb, 0, 1),
                                          acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(wb, wb, 2, 3), __builtin_shufflevector(xb, xb, 2, 3),
                                          acc, false);
    return acc;
}
__device__ __forceinline__ float lo16(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi16(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// G: the residual row is gathered (residx; the fast model's first layer), whose index load the
// residual load must wait for -- the compiler hoists that pair ahead of the weight loads (one round
// trip), so the plain form keeps it out of the kernel entirely
template <int U, int RP, bool PRENORM, bool FIN, bool G>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RP == 2 ? 5 : 3)))
void rowgemv_kernel(RowGemvArgs a) {
    __shared__ float red[4 * RP + 4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = blockIdx.x * RP;
    const int nch = a.K >> 8;
    const int wa = (wave * nch) >> 2, nmy = (((wave + 1) * nch) >> 2) - wa;
    const int last = nmy > 0 ? nmy - 1 : 0;
    const unsigned long long ts0 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    // first round trip, unconditional (a load under a branch drains vmcnt): the epilogue's residual
    // and bias elements of row n0 + (thread % RP), then x (and the norm weight) of the wave's chunks
    const int er = n0 + (int)(threadIdx.x % RP);
    int ri = 0;
    if constexpr (G) {
        const int32_t iv = a.residx[a.res_col];
        ri = iv < 0 ? 0 : (iv >= a.res_rows ? a.res_rows - 1 : iv);
    }
    bf16_t rv = 0;
    if constexpr (FIN) rv = a.res[(size_t)ri * a.ldr + er];
    const bf16_t bv = *(a.bias ? a.bias + er : a.X);
    const u32x2_t* xp = reinterpret_cast<const u32x2_t*>(a.X) + (size_t)wa * 64 + lane;
    const u32x2_t* gp = reinterpret_cast<const u32x2_t*>(PRENORM ? a.nw : a.X) + (size_t)wa * 64 + lane;
    u32x2_t xv[U], gv[PRENORM ? U : 1];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int j = (u < last ? u : last) * 64;
        xv[u] = xp[j];
        if constexpr (PRENORM) gv[u] = gp[j];
    }
    // KV prefetch (STORE form, wqkv of the slow model): slot and position ride the first round trip
    constexpr int PF = 2;
    const bool pf_on = !FIN && a.pf_kc != nullptr;
    int pf_s = 0, pf_p = 0;
    if constexpr (!FIN) {
        pf_s = *(pf_on ? a.pf_slot : reinterpret_cast<const int32_t*>(a.X));
        pf_p = *(pf_on ? a.pf_pos : reinterpret_cast<const int32_t*>(a.X));
    }
    asm volatile("" ::: "memory");  // keep the first round trip ahead of the weight loads
    // the block's weights: RP rows of each chunk (tail slots re-load the run's last chunk)
    const u32x2_t* wp = reinterpret_cast<const u32x2_t*>(a.W + (size_t)n0 * a.K) + (size_t)wa * 64 + lane;
    const size_t rs4 = (size_t)(a.K >> 2);  // one row in u32x2 units
    u32x2_t wv[U][RP];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int j = (u < last ? u : last) * 64;
#pragma unroll
        for (int r = 0; r < RP; ++r) wv[u][r] = __builtin_nontemporal_load(wp + r * rs4 + j);
    }
    asm volatile("" ::: "memory");
    float pfw[PF];
    if constexpr (!FIN) {  // GemvArgs::pf_kc: one 4-byte load per 64-B sector, after the weights
        // byte offsets from the K cache (integer selects only: a per-lane pointer select or a
        // load under a branch makes the compiler drain vmcnt)
        const char* kcb = reinterpret_cast<const char*>(pf_on ? a.pf_kc : a.X);
        const long long dv = pf_on ? reinterpret_cast<const char*>(a.pf_vc) - kcb : 0;
        const int nkv = pf_on ? a.pf_nkv : 1;
        const int b = blockIdx.x, h = b % nkv, jb = b / nkv, nb = ((int)gridDim.x - 1 - h) / nkv + 1;
        const int spr = pf_on ? a.pf_hd * 2 / 64 : 1;
        const int np = pf_on ? pf_p + 1 : 0, total = 2 * np * spr;
        const long long base = pf_on ? (long long)pf_s * (long long)a.pf_slot_stride + (long long)a.pf_layer_off +
                                           (long long)h * a.pf_S * a.pf_hd
                                     : 0;
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int i = (jb + nb * q) * 256 + (int)threadIdx.x;
            const bool ok = i < total;
            const int ii = ok ? i : 0, row = ii / spr, sec = ii - row * spr;
            const bool isv = row >= np;
            const long long off = (isv ? dv : 0) + 2 * (base + (long long)(isv ? row - np : row) * a.pf_hd) + sec * 64;
            pfw[q] = *reinterpret_cast<const float*>(kcb + (ok ? off : 0));
        }
    }
    // PRENORM: the row statistic (every block the same sums in the same order), then x'
    if constexpr (PRENORM) {
        float sl = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u < nmy) {
                const float e0 = lo16(xv[u][0]), e1 = hi16(xv[u][0]), e2 = lo16(xv[u][1]), e3 = hi16(xv[u][1]);
                sl += e0 * e0 + e1 * e1 + e2 * e2 + e3 * e3;
            }
        }
        sl = wave_sum(sl);
        if (lane == 0) red[4 * RP + wave] = sl;
        lds_barrier();
        const float tot = ((red[4 * RP] + red[4 * RP + 1]) + red[4 * RP + 2]) + red[4 * RP + 3];
        const float rs = 1.0f / sqrtf(tot / (float)a.K + a.eps);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x2_t o;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float y0 = bfround(bfround(lo16(xv[u][h]) * rs) * lo16(gv[u][h]));
                const float y1 = bfround(bfround(hi16(xv[u][h]) * rs) * hi16(gv[u][h]));
                o[h] = (uint32_t)f2bf(y0) | ((uint32_t)f2bf(y1) << 16);
            }
            xv[u] = o;
        }
    }
    float acc[RP];
#pragma unroll
    for (int r = 0; r < RP; ++r) acc[r] = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (u < nmy) {
#pragma unroll
            for (int r = 0; r < RP; ++r) acc[r] = dot4(wv[u][r], xv[u], acc[r]);
        }
    }
    if constexpr (!FIN) {  // keep the prefetch loads (retired with the weights)
#pragma unroll
        for (int q = 0; q < PF; ++q) asm volatile("" ::"v"(pfw[q]));
    }
    const unsigned long long ts1 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
#pragma unroll
    for (int r = 0; r < RP; ++r) {
        const float v = wave_sum(acc[r]);
        if (lane == 0) red[wave * RP + r] = v;
    }
    __syncthreads();
    if ((int)threadIdx.x < RP) {
        const int t = threadIdx.x;
        float v = ((red[t] + red[RP + t]) + red[2 * RP + t]) + red[3 * RP + t];
        if (a.bias) v += bf2f(bv);
        if constexpr (FIN) {
            a.res_out[er] = f2bf(bfround(bf2f(rv) + bfround(v)));
        } else {
            a.Y[er] = f2bf(v);
        }
    }
    if (a.dbg && threadIdx.x == 0) {
        const unsigned long long t[7] = {ts0, ts1, __builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0};
        dbg_record(a.dbg, 0xFFFA, (unsigned)blockIdx.x, t);
    }
}

// smallest instantiated depth covering a wave's share of the K chunks (0: not eligible)
int rowgemv_u(int K) {
    if (K <= 0 || K % 256) return 0;
    const int need = (K / 256 + 3) / 4;
    for (int u : {2, 3, 4, 5, 6, 8, 10, 12})
        if (need <= u) return u;
    return 0;
}

template <int RP, bool PRENORM, bool FIN>
static void rowgemv_go(hipStream_t s, const RowGemvArgs& a, int U) {
    const dim3 grid(a.N / RP), block(256);
    auto go = [&](void (*plain)(RowGemvArgs), void (*gathered)(RowGemvArgs)) {
        (FIN && a.residx ? gathered : plain)<<<grid, block, 0, s>>>(a);
    };
#define RG(u) go(rowgemv_kernel<u, RP, PRENORM, FIN, false>, rowgemv_kernel<u, RP, PRENORM, FIN, FIN>)
    switch (U) {
        case 2: RG(2); break;
        case 3: RG(3); break;
        case 4: RG(4); break;
        case 5: RG(5); break;
        case 6: RG(6); break;
        case 8: RG(8); break;
        case 10: RG(10); break;
        default: RG(12); break;
    }
#undef RG
}

void launch_rowgemv(hipStream_t s, const RowGemvArgs& a0, int kind) {
    RowGemvArgs a = a0;
    a.dbg = fm_tuning().dbg;
    const int U = rowgemv_u(a.K);
    FMCHECK(U > 0 && a.W && a.X, "row GEMV: K % 256 == 0 and K <= 12288, operands set");
    if (kind == ROWGEMV_FIN) {
        FMCHECK(a.N % 2 == 0 && a.res && a.res_out, "row GEMV (fin): N even, residual rows set");
        rowgemv_go<2, false, true>(s, a, U);
    } else {
        FMCHECK(kind == ROWGEMV_NORM_STORE && a.N % 8 == 0 && a.nw && a.Y, "row GEMV (norm, store): N % 8 == 0, norm weight and output set");
        rowgemv_go<8, true, false>(s, a, U);
    }
}

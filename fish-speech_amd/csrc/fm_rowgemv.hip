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
#include <type_traits>

typedef __attribute__((ext_vector_type(2))) uint32_t u32x2_t;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;

// acc += w . x over 4 bf16 (two v_dot2c_f32_bf16); whole-vector bit casts, so the compiler emits v_dot2c_f32_bf16 on the loaded registers
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
// acc += w . x over 8 bf16 pairs (v_dot2c_f32_bf16); whole-vector bit casts
__device__ __forceinline__ float dot8r(u32x4_t w, u32x4_t x, float acc) {
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
__device__ __forceinline__ void ld_pair_bf(const bf16_t* p, float& x0, float& x1) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
    x0 = lo16(w);
    x1 = hi16(w);
}

// G: the residual row is gathered (residx; the fast model's first layer), whose index load the
// residual load must wait for -- the compiler hoists that pair ahead of the weight loads (one round
// trip), so the plain form keeps it out of the kernel entirely.
// QM 1 (weight-only int8, WeightOnlyInt8Linear, /root/reference/tools/llama/quantize.py:212-240):
// W is the int8 row-major matrix, a chunk is 512 k (8 codes = 8 B per lane per row, x 16 B), the
// codes become floats exactly (byte ^ 0x80 -> v_cvt_f32_ubyte = q + 128, the 128 * sum(x) taken off
// once at the end) and each output is round(round(acc) * scale[row]) (quantize.py:228-229).
// QM 2 (weight-only int4, group size gs a multiple of 8; quantize.py:57-160 group quantization):
// W is the packed row-major code matrix (one 32-bit word = 8 codes, the even ones in the low half),
// a chunk is 512 k (one word per lane per row); each code pair becomes the exact bf16 pair
// (128 + q) by one mask-and-or, two v_dot2c per word pair give B = sum x (128 + q) over the lane's
// 8 k (inside one group), and the group's affine map is applied as s * B + (z - 136 s) * sum x,
// i.e. sum x ((q - 8) s + z) in fp32 (the tile kernel's QM 2 form, fm_gemv.hip).
template <int QM> struct RowT {
    static constexpr int EPL = QM ? 8 : 4;  // elements per lane per chunk
    static constexpr int CE = 64 * EPL;     // k per chunk
    using XV = typename std::conditional<QM != 0, u32x4_t, u32x2_t>::type;  // EPL bf16
    static constexpr int WPL = QM == 2 ? 1 : 2;  // 32-bit words of weights per lane per row per chunk
};

// EPI: 0 STORE (wqkv), 1 FIN (wo / w2), 2 SWIGLU (w1 || w3: rows 4b .. 4b+3 of W1 then of W3 per
// block, outputs y = round(silu(round(g))) * round(u), FeedForward.forward, llama.py:978-986),
// 3 F32 (a head's logits: fp32 holding the T-rounded value).  G: FIN gathers its residual row,
// the other forms their x row (RowGemvArgs::xidx: the fast model's first layer, codebook > 0).
// TX (tagged x, fattn_wo_kernel): x is read after the weights, from 32-bit words (bf16 << 16 | gen)
// that a producer in the same launch stores write-through; the wave re-reads its words (sc1) until
// every tag equals gen (bounded; *err set on timeout).  blk: the row block's index.
template <int U, int RP, bool PRENORM, int EPI, bool G, int QM, bool TX>
__device__ __forceinline__ void rowgemv_body(const RowGemvArgs& a, const int blk, const uint32_t* xt, const uint32_t gen,
                                             int* err) {
    static_assert(!TX || (!PRENORM && EPI == 1), "tagged x: the residual form only");
    constexpr bool FIN = EPI == 1;
    using R = RowT<QM>;
    using XV = typename R::XV;
    constexpr int EPL = R::EPL, NW = EPL / 2;  // NW: 32-bit words of x per lane per chunk
    __shared__ float red[4 * RP + 8];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = blk * RP;
    const int nch = a.K / R::CE;
    const int wa = (wave * nch) >> 2, nmy = (((wave + 1) * nch) >> 2) - wa;
    const int last = nmy > 0 ? nmy - 1 : 0;
    const unsigned long long ts0 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    // first round trip, unconditional (a load under a branch drains vmcnt): the epilogue's residual,
    // bias and (int8) scale elements of row n0 + (thread % RP), then x (and the norm weight)
    const int er = n0 + (int)(threadIdx.x % RP);
    int ri = 0, xi = 0;
    if constexpr (G && FIN) {
        const int32_t iv = a.residx[a.res_col];
        ri = iv < 0 ? 0 : (iv >= a.res_rows ? a.res_rows - 1 : iv);
    } else if constexpr (G) {
        const int32_t iv = a.xidx[a.xcol];
        xi = iv < 0 ? 0 : (iv >= a.xrows ? a.xrows - 1 : iv);
    }
    bf16_t rv = 0;
    if constexpr (FIN) rv = a.res[(size_t)ri * a.ldr + er];
    const bf16_t bv = *(a.bias ? a.bias + er : a.X);
    bf16_t sv = 0;
    if constexpr (QM == 1) sv = a.wscale[er];
    const XV* xp = reinterpret_cast<const XV*>(a.X + (size_t)xi * a.ldx) + (size_t)wa * 64 + lane;
    const XV* gp = reinterpret_cast<const XV*>(PRENORM ? a.nw : a.X) + (size_t)wa * 64 + lane;
    XV xv[U], gv[PRENORM ? U : 1];
    if constexpr (!TX) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = (u < last ? u : last) * 64;
            xv[u] = xp[j];
            if constexpr (PRENORM) gv[u] = gp[j];
        }
    }
    // KV prefetch (STORE form, wqkv of the slow model): slot and position ride the first round trip
    constexpr int PF = 2;
    const bool pf_on = EPI == 0 && a.pf_kc != nullptr;
    int pf_s = 0, pf_p = 0;
    if constexpr (EPI == 0) {
        pf_s = *(pf_on ? a.pf_slot : reinterpret_cast<const int32_t*>(a.X));
        pf_p = *(pf_on ? a.pf_pos : reinterpret_cast<const int32_t*>(a.X));
    }
    asm volatile("" ::: "memory");  // keep the first round trip ahead of the weight loads
    // the block's weights: RP rows of each chunk, 8 B (int4: 4 B) per lane; int4: the lane's group
    // (scale, zero) per row too (tail slots re-load the run's last chunk)
    constexpr int WU = QM == 2 ? 1 : U, WR = QM == 2 ? 1 : RP;
    constexpr int QU = QM == 2 ? U : 1, QR = QM == 2 ? RP : 1;
    u32x2_t wv[WU][WR];
    uint32_t w4[QU][QR], szv[QU][QR];
    if constexpr (QM == 2) {
        const size_t rw = (size_t)(a.K >> 3);  // one row in words
        const int ng = a.K / a.gs;
        const uint32_t* wp = a.Wq4 + (size_t)n0 * rw + (size_t)wa * 64 + lane;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int jc = u < last ? u : last;
#pragma unroll
            for (int r = 0; r < RP; ++r) {
                w4[u][r] = __builtin_nontemporal_load(wp + r * rw + jc * 64);
                szv[u][r] = a.wsz[(size_t)(n0 + r) * ng + ((wa + jc) * 512 + lane * 8) / a.gs];
            }
        }
    } else {
        const unsigned char* wb = QM ? reinterpret_cast<const unsigned char*>(a.Wq) : reinterpret_cast<const unsigned char*>(a.W);
        const size_t rowb = (size_t)a.K * (QM ? 1 : 2);  // bytes per row
        const u32x2_t* wp = reinterpret_cast<const u32x2_t*>(wb + (size_t)n0 * rowb) + (size_t)wa * 64 + lane;
        const size_t rs8 = rowb / 8;  // one row in u32x2 units
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = (u < last ? u : last) * 64;
#pragma unroll
            for (int r = 0; r < RP; ++r) wv[u][r] = __builtin_nontemporal_load(wp + r * rs8 + j);
        }
    }
    asm volatile("" ::: "memory");
    if constexpr (TX) {
        // EPL tagged words per lane per chunk (sc1 loads, 16 B each), re-read until all are current
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)xt, (short)0, a.K * 4, 0x00020000);
        u32x4_t xw[U][EPL / 4];
        for (unsigned it = 0;; ++it) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int jc = u < last ? u : last;
#pragma unroll
                for (int q = 0; q < EPL / 4; ++q)
                    xw[u][q] = __builtin_amdgcn_raw_buffer_load_b128(xr, ((wa + jc) * R::CE + EPL * lane + 4 * q) * 4, 0, 16);
            }
            bool ok = true;
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < EPL / 4; ++q)
#pragma unroll
                    for (int e = 0; e < 4; ++e) ok = ok && ((xw[u][q][e] & 0xffffu) == gen);
            if (__all(ok)) break;
            if (it >= (1u << 14)) {  // bounded: the host sees err and fails the frame
                if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int h = 0; h < NW; ++h) {
                const uint32_t w0 = xw[u][(2 * h) >> 2][(2 * h) & 3], w1 = xw[u][(2 * h + 1) >> 2][(2 * h + 1) & 3];
                xv[u][h] = (w0 >> 16) | (w1 & 0xffff0000u);
            }
    }
    float pfw[PF];
    if constexpr (EPI == 0) {  // GemvArgs::pf_kc: one 4-byte load per 64-B sector, after the weights
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
#pragma unroll
                for (int h = 0; h < NW; ++h) {
                    const float e0 = lo16(xv[u][h]), e1 = hi16(xv[u][h]);
                    sl += e0 * e0 + e1 * e1;
                }
            }
        }
        sl = wave_sum(sl);
        if (lane == 0) red[4 * RP + wave] = sl;
        lds_barrier();
        const float tot = ((red[4 * RP] + red[4 * RP + 1]) + red[4 * RP + 2]) + red[4 * RP + 3];
        const float rs = 1.0f / sqrtf(tot / (float)a.K + a.eps);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            XV o;
#pragma unroll
            for (int h = 0; h < NW; ++h) {
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
    float xs = 0.f;  // int8: this lane's sum of x (the 128 offset of the codes)
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (u < nmy) {
            if constexpr (QM == 0) {
#pragma unroll
                for (int r = 0; r < RP; ++r) acc[r] = dot4(wv[u][r], xv[u], acc[r]);
            } else if constexpr (QM == 2) {
                const u32x4_t ones = {0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
                const float xl = dot8r(ones, xv[u], 0.f);  // sum of the lane's 8 x
#pragma unroll
                for (int r = 0; r < RP; ++r) {
                    const uint32_t w = w4[u][r];
                    u32x4_t A;
#pragma unroll
                    for (int p = 0; p < 4; ++p) A[p] = ((w >> (4 * p)) & 0x000F000Fu) | 0x43004300u;
                    const float B = dot8r(A, xv[u], 0.f);
                    const float sc = lo16(szv[u][r]), zr = hi16(szv[u][r]);
                    acc[r] = fmaf(sc, B, acc[r]);
                    acc[r] = fmaf(zr - 136.f * sc, xl, acc[r]);
                }
            } else {
                float xf[8];
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    xf[2 * h] = lo16(xv[u][h]);
                    xf[2 * h + 1] = hi16(xv[u][h]);
                }
                xs += ((xf[0] + xf[1]) + (xf[2] + xf[3])) + ((xf[4] + xf[5]) + (xf[6] + xf[7]));
#pragma unroll
                for (int r = 0; r < RP; ++r) {
                    const uint32_t c0 = wv[u][r][0] ^ 0x80808080u, c1 = wv[u][r][1] ^ 0x80808080u;
                    float t = acc[r];
#pragma unroll
                    for (int e = 0; e < 4; ++e) t = fmaf((float)((c0 >> (8 * e)) & 0xffu), xf[e], t);
#pragma unroll
                    for (int e = 0; e < 4; ++e) t = fmaf((float)((c1 >> (8 * e)) & 0xffu), xf[4 + e], t);
                    acc[r] = t;
                }
            }
        }
    }
    if constexpr (EPI == 0) {  // keep the prefetch loads (retired with the weights)
#pragma unroll
        for (int q = 0; q < PF; ++q) asm volatile("" ::"v"(pfw[q]));
    }
    const unsigned long long ts1 = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
#pragma unroll
    for (int r = 0; r < RP; ++r) {
        const float v = wave_sum(acc[r]);
        if (lane == 0) red[wave * RP + r] = v;
    }
    if constexpr (QM == 1) {
        const float v = wave_sum(xs);
        if (lane == 0) red[4 * RP + 4 + wave] = v;
    }
    __syncthreads();
    if ((int)threadIdx.x < RP) {
        const int t = threadIdx.x;
        float v = ((red[t] + red[RP + t]) + red[2 * RP + t]) + red[3 * RP + t];
        if constexpr (QM == 1) {
            const float xt = ((red[4 * RP + 4] + red[4 * RP + 5]) + red[4 * RP + 6]) + red[4 * RP + 7];
            v = bfround(bfround(v - 128.f * xt) * bf2f(sv));
        }
        if (a.bias) v += bf2f(bv);
        if constexpr (FIN) {
            a.res_out[er] = f2bf(bfround(bf2f(rv) + bfround(v)));
        } else if constexpr (EPI == 3) {
            a.Yf[er] = bfround(v);
        } else if constexpr (EPI == 2) {  // gate rows t < RP / 2, up rows t >= RP / 2 (same wave)
            const float up = __shfl_down(v, RP / 2, 64);
            if (t < RP / 2) {
                const float g = bfround(v);
                a.Y[blockIdx.x * (RP / 2) + t] = f2bf(bfround(g / (1.0f + expf(-g))) * bfround(up));
            }
        } else {
            a.Y[er] = f2bf(v);
        }
    }
    if (a.dbg && threadIdx.x == 0) {
        const unsigned long long t[7] = {ts0, ts1, __builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0};
        dbg_record(a.dbg, TX ? 0xFFF8u : 0xFFFAu, (unsigned)blk, t);
    }
}

template <int U, int RP, bool PRENORM, int EPI, bool G, int QM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RP == 2 ? 5 : 3)))
void rowgemv_kernel(RowGemvArgs a) {
    rowgemv_body<U, RP, PRENORM, EPI, G, QM, false>(a, blockIdx.x, nullptr, 0u, nullptr);
}

// smallest instantiated depth covering a wave's share of the K chunks (0: not eligible)
int rowgemv_u(int K, int qm) {
    const int ce = qm ? 512 : 256;
    if (K <= 0 || K % ce) return 0;
    const int need = (K / ce + 3) / 4;
    for (int u : {2, 3, 4, 5, 6, 8, 10, 12})
        if (need <= u) return u;
    return 0;
}

template <int RP, bool PRENORM, int EPI, int QM>
static void rowgemv_go(hipStream_t s, const RowGemvArgs& a, int U) {
    const dim3 grid(a.N / RP), block(256);
    auto go = [&](void (*plain)(RowGemvArgs), void (*gathered)(RowGemvArgs)) {
        ((EPI == 1 ? a.residx != nullptr : a.xidx != nullptr) ? gathered : plain)<<<grid, block, 0, s>>>(a);
    };
#define RG(u) go(rowgemv_kernel<u, RP, PRENORM, EPI, false, QM>, rowgemv_kernel<u, RP, PRENORM, EPI, true, QM>)
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
    if (!a.ldx) a.ldx = a.K;
    const int qm = a.Wq4 ? 2 : (a.Wq ? 1 : 0);
    const int U = rowgemv_u(a.K, qm);
    FMCHECK(U > 0 && a.X &&
                (qm == 2 ? (a.wsz && a.gs > 0 && a.gs % 8 == 0 && a.K % a.gs == 0 && !a.bias)
                         : (qm == 1 ? (a.Wq && a.wscale && !a.bias) : a.W != nullptr)),
            "row GEMV: K a whole number of chunks (256 k, int8 / int4 512 k), at most 48 per wave; operands set");
    if (kind == ROWGEMV_FIN) {
        FMCHECK(a.N % 2 == 0 && a.res && a.res_out, "row GEMV (fin): N even, residual rows set");
        if (qm == 2) rowgemv_go<2, false, 1, 2>(s, a, U);
        else if (qm == 1) rowgemv_go<2, false, 1, 1>(s, a, U);
        else rowgemv_go<2, false, 1, 0>(s, a, U);
    } else if (kind == ROWGEMV_NORM_F32) {
        FMCHECK(a.N % 8 == 0 && a.nw && a.Yf && U <= 8 && !a.xidx, "row GEMV (norm, f32): N % 8 == 0, norm weight and output set");
        if (qm == 2) rowgemv_go<8, true, 3, 2>(s, a, U);
        else if (qm == 1) rowgemv_go<8, true, 3, 1>(s, a, U);
        else rowgemv_go<8, true, 3, 0>(s, a, U);
    } else if (kind == ROWGEMV_NORM_SWIGLU) {
        FMCHECK(a.N % 8 == 0 && a.nw && a.Y && U <= 8 && !a.bias,
                "row GEMV (norm, swiglu): N % 8 == 0 (4 + 4 interleaved rows), norm weight and output set");
        if (qm == 2) rowgemv_go<8, true, 2, 2>(s, a, U);
        else if (qm == 1) rowgemv_go<8, true, 2, 1>(s, a, U);
        else rowgemv_go<8, true, 2, 0>(s, a, U);
    } else {
        FMCHECK(kind == ROWGEMV_NORM_STORE && a.N % 8 == 0 && a.nw && a.Y && U <= 8,
                "row GEMV (norm, store): N % 8 == 0, norm weight and output set");
        if (qm == 2) rowgemv_go<8, true, 0, 2>(s, a, U);
        else if (qm == 1) rowgemv_go<8, true, 0, 1>(s, a, U);
        else if (fm_tuning().row_qkv_rp == 4) rowgemv_go<4, true, 0, 0>(s, a, U);
        else if (fm_tuning().row_qkv_rp == 16) rowgemv_go<16, true, 0, 0>(s, a, U);
        else rowgemv_go<8, true, 0, 0>(s, a, U);
    }
}

// =========================================================================================
// Fast-model attention + wo in ONE launch (batch 1, bf16; fm_tune fattn_wo).
//
// The fast model's attention (llama.py:947-975, one query row at codebook position cpos < 16) is
// latency-bound: ~4 us of dependent round trips on 32 of 256 CUs, while the wo GEMV that consumes
// it is a 21 MB weight stream.  Here blocks 0 .. nkv-1 run the attention (one block per kv group,
// one wave per q head, cached K / V rows staged in LDS) and blocks nkv .. nkv + N/2 - 1 are the
// row-pair wo blocks of rowgemv_kernel, which issue their whole weight run first and only then
// wait for the attention output.  The hand-off has no counters and no fences: each attention
// output element is stored write-through (sc1) as one 32-bit word (bf16 value << 16 | gen), gen a
// tag unique among consecutive launches (host: 1 + layer + n_layer * cpos), and a wo wave re-reads
// its x words (sc1 loads) until every tag is current.  Deadlock-free by dispatch order: the
// attention blocks have the lowest indices, so they are resident before any waiting block, and the
// whole grid fits at once (<= 8 blocks of 4 waves per CU, 10 KiB LDS each).  Every wait is bounded
// (FattnWoArgs::err set on timeout; the host throws and resets).
constexpr int FW_MAXJ = 15;   // cached rows staged in LDS (cpos < 16)
constexpr int FW_MAXHD = 128;

template <int U, bool G, int QM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6)))
void fattn_wo_kernel(FattnWoArgs A) {
    __shared__ __attribute__((aligned(16))) bf16_t kvs[2 * FW_MAXJ * FW_MAXHD];
    __shared__ float red[8];
    const FastFusedArgs<bf16_t>& at = A.at;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // the tag: the frame's position (device, constant through the frame's fast passes) times 41
    // plus the launch's index in the frame (1 .. 40): distinct for any two launches less than ~1600
    // frames apart, across requests and slots too, so a stale word never passes for a fresh one
    const uint32_t gen = ((uint32_t)A.at.row_pos[0] * 41u + (uint32_t)A.gen) % 65535u + 1u;
    const unsigned long long ts0 = A.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
    if ((int)blockIdx.x < at.nkv) {
        // ---------------- attention: kv group kvh, q head kvh * g + wave ----------------------
        // top issue priority: the wo waves sharing this CU queue their whole weight run at once
        if (A.prio) __builtin_amdgcn_s_setprio(3);
        const int kvh = blockIdx.x, hd = at.hd, g = at.nh / at.nkv, cpos = at.cpos, half = hd >> 1;
        const int slot = at.row_slot[0];
        const bool live = wave < g;
        const int h = kvh * g + (live ? wave : 0);
        const float* tab = at.rope + (size_t)cpos * hd;
        float q0[2], q1[2], k0[2], k1[2], v0[2], v1[2], qw0[2], qw1[2], kw0[2], kw1[2], c_[2], s_[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int p = lane + 64 * u;
            const int pp = p < half ? p : 0;
            ld_pair_bf(at.qkv + (size_t)h * hd + 2 * pp, q0[u], q1[u]);
            ld_pair_bf(at.qkv + (size_t)(at.nh + kvh) * hd + 2 * pp, k0[u], k1[u]);
            ld_pair_bf(at.qkv + (size_t)(at.nh + at.nkv + kvh) * hd + 2 * pp, v0[u], v1[u]);
            if (at.qk_norm) {
                ld_pair_bf(at.qn + 2 * pp, qw0[u], qw1[u]);
                ld_pair_bf(at.kn + 2 * pp, kw0[u], kw1[u]);
            } else {
                qw0[u] = qw1[u] = kw0[u] = kw1[u] = 1.f;
            }
            c_[u] = tab[2 * pp];
            s_[u] = tab[2 * pp + 1];
            if (p >= half) q0[u] = q1[u] = k0[u] = k1[u] = v0[u] = v1[u] = 0.f;
        }
        // the cached rows j < cpos of this kv head -> LDS (K rows, then V rows), 16 B per thread
        const size_t base = (size_t)slot * at.slot_stride + at.layer_off + (size_t)kvh * at.S * hd;
        const int nck = cpos * hd / 8;
        for (int i = threadIdx.x; i < 2 * nck; i += 256) {
            const bool isv = i >= nck;
            const int c = isv ? i - nck : i;
            const u32x4_t v = *reinterpret_cast<const u32x4_t*>((isv ? at.vc : at.kc) + base + (size_t)c * 8);
            *reinterpret_cast<u32x4_t*>(kvs + (isv ? FW_MAXJ * FW_MAXHD : 0) + c * 8) = v;
        }
        // qk-norm (fp32 incl. weight, one rounding) + RoPE (bf16 table, rounded): fm_attn_dev.h
        auto prep = [&](float (&x0)[2], float (&x1)[2], const float (&w0)[2], const float (&w1)[2]) {
            if (at.qk_norm) {
                float ss = 0.f;
#pragma unroll
                for (int u = 0; u < 2; ++u) ss += x0[u] * x0[u] + x1[u] * x1[u];
                ss = wave_sum(ss);
                const float rs = 1.0f / sqrtf(ss / (float)hd + at.eps);
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    x0[u] = bfround((x0[u] * rs) * w0[u]);
                    x1[u] = bfround((x1[u] * rs) * w1[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float y0 = bfround(x0[u] * c_[u] - x1[u] * s_[u]);
                const float y1 = bfround(x1[u] * c_[u] + x0[u] * s_[u]);
                x0[u] = y0;
                x1[u] = y1;
            }
        };
        prep(q0, q1, qw0, qw1);
        prep(k0, k1, kw0, kw1);
        if (wave == 0) {  // the group's new k / v of cpos into the fast cache
            bf16_t* kd = at.kc + base + (size_t)cpos * hd;
            bf16_t* vd = at.vc + base + (size_t)cpos * hd;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int p = lane + 64 * u;
                if (p < half) {
                    *reinterpret_cast<uint32_t*>(kd + 2 * p) = (uint32_t)f2bf(k0[u]) | ((uint32_t)f2bf(k1[u]) << 16);
                    *reinterpret_cast<uint32_t*>(vd + 2 * p) = (uint32_t)f2bf(v0[u]) | ((uint32_t)f2bf(v1[u]) << 16);
                }
            }
        }
        __syncthreads();  // K / V rows staged
        const unsigned long long ts1 = A.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
        if (!live) return;
        const bf16_t* Ks = kvs;
        const bf16_t* Vs = kvs + FW_MAXJ * FW_MAXHD;
        // scores round(round(q.k) * scale), softmax, probabilities rounded (fast SDPA path)
        float sc[FW_MAXJ + 1];
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j <= FW_MAXJ; ++j) {
            if (j > cpos) break;
            float d = 0.f;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int p = lane + 64 * u;
                const int pp = p < half ? p : 0;
                float a0 = k0[u], a1 = k1[u];
                if (j < cpos) {
                    const uint32_t w = *reinterpret_cast<const uint32_t*>(Ks + j * hd + 2 * pp);
                    a0 = p < half ? lo16(w) : 0.f;
                    a1 = p < half ? hi16(w) : 0.f;
                }
                d += q0[u] * a0 + q1[u] * a1;
            }
            d = wave_sum(d);
            sc[j] = bfround(bfround(d) * at.scale);
            mx = fmaxf(mx, sc[j]);
        }
        float den = 0.f;
#pragma unroll
        for (int j = 0; j <= FW_MAXJ; ++j) {
            if (j > cpos) break;
            sc[j] = expf(sc[j] - mx);
            den += sc[j];
        }
        float o0[2] = {0.f, 0.f}, o1[2] = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j <= FW_MAXJ; ++j) {
            if (j > cpos) break;
            const float pj = bfround(sc[j] / den);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int p = lane + 64 * u;
                const int pp = p < half ? p : 0;
                float b0 = v0[u], b1 = v1[u];
                if (j < cpos) {
                    const uint32_t w = *reinterpret_cast<const uint32_t*>(Vs + j * hd + 2 * pp);
                    b0 = lo16(w);
                    b1 = hi16(w);
                }
                o0[u] += pj * b0;
                o1[u] += pj * b1;
            }
        }
        // tagged write-through store: word = bf16 << 16 | gen
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int p = lane + 64 * u;
            if (p < half) {
                const uint64_t w = (uint64_t)(((uint32_t)f2bf(o0[u]) << 16) | gen) |
                                   ((uint64_t)(((uint32_t)f2bf(o1[u]) << 16) | gen) << 32);
                __hip_atomic_store(reinterpret_cast<uint64_t*>(A.xt + (size_t)h * hd + 2 * p), w, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (A.dbg && lane == 0) {  // developer record per attention wave (tag 0xFFF9): start, staged, stored
            const unsigned long long t[7] = {ts0, ts1, __builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0};
            dbg_record(A.dbg, 0xFFF9, (unsigned)h, t);
        }
        return;
    }
    // ---------------- wo rows 2p, 2p + 1: rowgemv_body FIN with x from the tagged words --------
    rowgemv_body<U, 2, false, 1, G, QM, true>(A.wo, (int)blockIdx.x - at.nkv, A.xt, gen, A.err);
}

bool fattn_wo_ok(int nh, int nkv, int hd, int cpos, int N, int K, int qm) {
    const int U = rowgemv_u(K, qm);
    return nkv > 0 && nh % nkv == 0 && nh / nkv <= 4 && hd % 2 == 0 && hd <= FW_MAXHD && cpos >= 0 &&
           cpos < FW_MAXJ + 1 && K == nh * hd && N % 2 == 0 && U > 0 && U <= 8;
}

void launch_fattn_wo(hipStream_t s, const FattnWoArgs& A0) {
    FattnWoArgs A = A0;
    A.dbg = fm_tuning().dbg;
    A.wo.dbg = A.dbg;
    const FastFusedArgs<bf16_t>& at = A.at;
    const int qm = A.wo.Wq4 ? 2 : (A.wo.Wq ? 1 : 0);
    FMCHECK(fattn_wo_ok(at.nh, at.nkv, at.hd, at.cpos, A.wo.N, A.wo.K, qm) && A.xt && A.err && A.gen > 0 && A.gen <= 40 && at.row_pos &&
                A.wo.res && A.wo.res_out &&
                (qm == 2 ? (A.wo.wsz && A.wo.gs % 8 == 0 && !A.wo.bias) : (qm == 1 ? (A.wo.wscale && !A.wo.bias) : A.wo.W != nullptr)),
            "fused fast attention + wo: shapes, tag and buffers");
    const dim3 grid(at.nkv + A.wo.N / 2), block(256);
    const bool G = A.wo.residx != nullptr;
    auto go = [&](auto q) {
        constexpr int Q = decltype(q)::value;
        switch (rowgemv_u(A.wo.K, Q)) {
#define FW(u) \
    case u: (G ? fattn_wo_kernel<u, true, Q> : fattn_wo_kernel<u, false, Q>)<<<grid, block, 0, s>>>(A); break;
            FW(2) FW(3) FW(4) FW(5) FW(6)
            default: (G ? fattn_wo_kernel<8, true, Q> : fattn_wo_kernel<8, false, Q>)<<<grid, block, 0, s>>>(A); break;
#undef FW
        }
    };
    if (qm == 2) go(std::integral_constant<int, 2>{});
    else if (qm == 1) go(std::integral_constant<int, 1>{});
    else go(std::integral_constant<int, 0>{});
}

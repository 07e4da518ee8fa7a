// fm_llm_kernels.hip -- gfx950 kernels of the Dual-AR decode step (slow 4B llama + fast
// codebook transformer + sampling).  Every kernel is templated on the storage type T
// (bf16_t: production, float: fp32 validation mode) and rounds at the reference's points:
//
//   embed_kernel ............. llama.py:399-420   (fp32 codebook sum, 3 roundings)
//   rmsnorm_kernel ........... llama.py:989-1000  (round(x*rstd) * w, rounded)
//   linear_kernel ............ nn.Linear / F.linear; MFMA 16x16x32 bf16 (or f32 16x16x4),
//                              W streamed once from HBM straight into A fragments, split-K
//                              over 8 waves, fused epilogues (bias, residual, SwiGLU)
//   qk_rope_cache_kernel ..... llama.py:894-910   (qk-norm, RoPE on bf16 table, cache write)
//   attn_split/combine ....... llama.py:915-933   (SDPA over the valid prefix, split-K flash
//                              decode; GQA heads share K/V reads, no repeat_interleave)
//   fast_attn_kernel ......... llama.py:947-975   (matmul-softmax-matmul, rounded per op)
//   sample_kernel ............ inference.py:43-93, 117-144 (top-k / top-p / temperature /
//                              RAS with the reference's rounding; no full-vocab sort)
#include "fm_kernels.h"
#include "fm_frag.h"

// =========================================================================================
// embeddings
// =========================================================================================
template <typename T>
__global__ __launch_bounds__(256) void embed_kernel(const int32_t* __restrict__ tok, int R,
                                                    const T* __restrict__ emb,
                                                    const T* __restrict__ cbemb, int d, int C,
                                                    int cb, int sb, int se, int scale,
                                                    T* __restrict__ x,
                                                    const int* __restrict__ row_slot) {
    // grid (R, ceil(d / 2048)): a thread owns 8 consecutive features; all C + 1 row reads of a
    // thread are in flight together
    const int r = blockIdx.x;
    if (r >= R) return;
    // prefill: tokens per row; decode: the slot's last emitted column (row_slot != null)
    const int32_t* t = tok + (size_t)(row_slot ? row_slot[r] : r) * (C + 1);
    const int i = 8 * (blockIdx.y * 256 + threadIdx.x);
    if (i >= d) return;
    int t0 = t[0];
    t0 = t0 < 0 ? 0 : t0;  // defence in depth: decode tokens come from the sampler (ids <= se)
    if (row_slot) t0 = t0 > se ? se : t0;
    const bool sem = t0 >= sb && t0 <= se;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (sem) {
        for (int q = 0; q < C; ++q) {
            float c8[8];
            int cq = t[1 + q];
            cq = cq < 0 ? 0 : (cq >= cb ? cb - 1 : cq);
            load8(cbemb + (size_t)(cq + q * cb) * d + i, c8);
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] += c8[u];
        }
    }
    float e8[8];
    load8(emb + (size_t)t0 * d + i, e8);
    const float inv = sqrtf((float)(C + 1));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        float e = rnd<T>(e8[u] + (sem ? rnd<T>(v[u]) : 0.f));
        if (scale && sem) e = rnd<T>(e / inv);
        st(x, (size_t)r * d + i + u, e);
    }
}

// x[r] = table[codes[r * ld + col]]  (fast_embeddings lookup, inference.py:154, 173)
template <typename T>
__global__ __launch_bounds__(256) void gather_rows_kernel(const int32_t* __restrict__ codes,
                                                          int ldc, int col, const T* __restrict__ table,
                                                          int d, int rows, T* __restrict__ x) {
    const int r = blockIdx.x;
    int c = codes[(size_t)r * ldc + col];
    c = c < 0 ? 0 : (c >= rows ? rows - 1 : c);  // defence in depth: codes come from the sampler
    for (int i = threadIdx.x; i < d; i += blockDim.x) x[(size_t)r * d + i] = table[(size_t)c * d + i];
}

// =========================================================================================
// RMSNorm (llama.py:989-1000): fp32 mean square, round(x*rstd), * weight, round
// =========================================================================================
// one wave per row (4 rows per block), 8 consecutive features per lane held in registers between
// the sum of squares and the scaled store: one read of x, no block barrier.  Host: d % 8 == 0,
// d <= 512 * RN_MAXC, ldx/ldy multiples of 8 and 16-byte aligned rows.
constexpr int RN_MAXC = 8;
template <typename T>
__global__ __launch_bounds__(256) void rmsnorm_wave_kernel(const T* __restrict__ x, int ldx,
                                                           const T* __restrict__ w, int d, float eps,
                                                           T* __restrict__ y, int ldy, int R) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const T* xr = x + (size_t)r * ldx;
    float v[RN_MAXC][8];
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < RN_MAXC; ++c) {
        const int i = 8 * (c * 64 + lane);
        if (i < d) {
            load8(xr + i, v[c]);
#pragma unroll
            for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
        }
    }
    ss = wave_sum(ss);
    const float rs = 1.0f / sqrtf(ss / (float)d + eps);
    T* yr = y + (size_t)r * ldy;
#pragma unroll
    for (int c = 0; c < RN_MAXC; ++c) {
        const int i = 8 * (c * 64 + lane);
        if (i < d) {
            float g[8], o[8];
            load8(w + i, g);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = rnd<T>(rnd<T>(v[c][j] * rs) * g[j]);
            if constexpr (is_bf16<T>::value) {
                u32x4_t pk;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    pk[j] = (__float_as_uint(o[2 * j]) >> 16) | (__float_as_uint(o[2 * j + 1]) & 0xffff0000u);
                *reinterpret_cast<u32x4_t*>(yr + i) = pk;
            } else {
                *reinterpret_cast<f32x4_t*>(yr + i) = (f32x4_t){o[0], o[1], o[2], o[3]};
                *reinterpret_cast<f32x4_t*>(yr + i + 4) = (f32x4_t){o[4], o[5], o[6], o[7]};
            }
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const T* __restrict__ x, int ldx,
                                                      const T* __restrict__ w, int d, float eps,
                                                      T* __restrict__ y, int ldy) {
    __shared__ float scratch[16];
    const int r = blockIdx.x;
    const T* xr = x + (size_t)r * ldx;
    float ss = 0.f;
    for (int i = threadIdx.x; i < d; i += blockDim.x) {
        float v = ld(xr, i);
        ss += v * v;
    }
    ss = block_sum(ss, scratch);
    const float rs = 1.0f / sqrtf(ss / (float)d + eps);
    for (int i = threadIdx.x; i < d; i += blockDim.x) {
        float v = rnd<T>(ld(xr, i) * rs);
        st(y, (size_t)r * ldy + i, v * ld(w, i));
    }
}

// =========================================================================================
// linear: Y[col][n] = epi( sum_k X[col][k] * W[n][k] )
// =========================================================================================
template <typename T>
__global__ void pack_kernel(const T* __restrict__ src, int N, int K, T* __restrict__ dst) {
    const int S = K >> 5;
    const int64_t nblk = (int64_t)((N + 15) / 16) * S;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nblk * 64; q += stride) {
        const int64_t blk = q >> 6;
        const int l = (int)(q & 63);
        const int t = (int)(blk / S), sidx = (int)(blk - (int64_t)t * S);
        const int row = 16 * t + (l & 15);
        const int k0 = 32 * sidx + 8 * (l >> 4);
        T* d = dst + blk * 512;
        for (int j = 0; j < 8; ++j) {
            const T v = row < N ? src[(size_t)row * K + k0 + j] : (T)0;
            if constexpr (is_bf16<T>::value) d[l * 8 + j] = v;
            else d[j < 4 ? l * 4 + j : 256 + l * 4 + (j - 4)] = v;
        }
    }
}
template <typename T> void launch_pack(hipStream_t s, const T* src, int N, int K, T* dst) {
    const int64_t n = (int64_t)((N + 15) / 16) * (K / 32) * 64;
    const int blocks = (int)std::min<int64_t>(FM_CEIL(n, 256), 16384);
    pack_kernel<T><<<blocks, 256, 0, s>>>(src, N, K, dst);
}
template void launch_pack<bf16_t>(hipStream_t, const bf16_t*, int, int, bf16_t*);

// ---- weight-only int8 (tools/llama/quantize.py) -----------------------------------------------
// One block per row: dynamically_quantize_per_channel (quantize.py:22-52) with quant range
// [-128, 127] on w.float(): the fp32 scale divides, the stored scale is bf16(s) (quantize.py:206 on
// the bf16 model quantize.py loads), held in T.
template <typename T>
__global__ __launch_bounds__(256) void quant_rows_kernel(T* __restrict__ w, int K, int8_t* __restrict__ q,
                                                         T* __restrict__ scale) {
    __shared__ float rmn[8], rmx[8];
    T* wr = w + (size_t)blockIdx.x * K;
    float mn = INFINITY, mx = -INFINITY;
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
        const float v = ld(wr, k);
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, o));
        mx = fmaxf(mx, __shfl_xor(mx, o));
    }
    if ((threadIdx.x & 63) == 0) {
        rmn[threadIdx.x >> 6] = mn;
        rmx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    mn = rmn[0];
    mx = rmx[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
        mn = fminf(mn, rmn[i]);
        mx = fmaxf(mx, rmx[i]);
    }
    const float m = fmaxf(-fminf(mn, 0.f), fmaxf(mx, 0.f));
    const float sc = fmaxf(m / 127.5f, 1.1920928955078125e-07f);  // torch.finfo(float32).eps
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
        const float v = fminf(fmaxf(rintf(ld(wr, k) / sc), -128.f), 127.f);
        q[(size_t)blockIdx.x * K + k] = (int8_t)v;
        st(wr, k, v);
    }
    // quantize.py quantizes the bf16 model (quantize.py:441-446): scales are stored as bf16
    if (threadIdx.x == 0) st(scale, blockIdx.x, rnd<bf16_t>(sc));
}
template <typename T> void launch_quant_rows(hipStream_t s, T* w, int N, int K, int8_t* q, T* scale) {
    quant_rows_kernel<T><<<N, 256, 0, s>>>(w, K, q, scale);
}

template <typename T>
__global__ void i8_to_kernel(const int8_t* __restrict__ q, int64_t n, T* __restrict__ dst) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        st(dst, i, (float)q[i]);
}
template <typename T> void launch_i8_to(hipStream_t s, const int8_t* q, int64_t n, T* dst) {
    i8_to_kernel<T><<<(int)std::min<int64_t>(FM_CEIL(n, 256), 16384), 256, 0, s>>>(q, n, dst);
}

// one thread per (unit, lane): 16 bytes = k-steps 2u and 2u + 1 of row (l & 15), k-offset 8 * (l >> 4)
__global__ void pack_q8_kernel(const int8_t* __restrict__ src, int N, int K, int8_t* __restrict__ dst) {
    const int U = K >> 6;
    const int64_t n = (int64_t)((N + 15) / 16) * U * 64;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t unit = i >> 6;
        const int l = (int)(i & 63);
        const int t = (int)(unit / U), u = (int)(unit - (int64_t)t * U);
        const int row = 16 * t + (l & 15);
        int8_t* d = dst + i * 16;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                d[8 * h + j] = row < N ? src[(size_t)row * K + 64 * u + 32 * h + 8 * (l >> 4) + j] : (int8_t)0;
    }
}
void launch_pack_q8(hipStream_t s, const int8_t* src, int N, int K, int8_t* dst) {
    const int64_t n = (int64_t)((N + 15) / 16) * (K / 64) * 64;
    pack_q8_kernel<<<(int)std::min<int64_t>(FM_CEIL(n, 256), 16384), 256, 0, s>>>(src, N, K, dst);
}
// ---- weight-only int4 (tools/llama/quantize.py:57-160) --------------------------------------
// one thread per (row, group): get_group_qparams + group_quantize_tensor_from_qparams in torch's bf16
// arithmetic (fp32 op, bf16 rounding after every op), then the dequantised bf16 weight in place
__global__ void quant4_kernel(bf16_t* __restrict__ w, int N, int K, int gs, uint8_t* __restrict__ q,
                              uint32_t* __restrict__ sz) {
    const int ng = K / gs;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)N * ng) return;
    const int n = (int)(idx / ng), gi = (int)(idx - (int64_t)n * ng);
    bf16_t* p = w + (size_t)n * K + (size_t)gi * gs;
    uint8_t* qp = q + (size_t)n * K + (size_t)gi * gs;
    auto rb = [](float x) { return bf2f(f2bf(x)); };
    float mn = INFINITY, mx = -INFINITY;
    for (int k = 0; k < gs; ++k) {
        const float v = bf2f(p[k]);
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
    }
    const float d = fmaxf(rb(mx - mn), rb(1e-6f));  // (max - min).clamp(min=1e-6) in bf16
    const float sc = rb(d / 15.f);                   // / max_int
    const float s8 = rb(sc * 8.f);
    const float zr = rb(mn + s8);                    // zeros = min + scales * 2^(n_bit - 1)
    const float lo = rb(zr - s8);                    // min_val of from_qparams
    for (int k = 0; k < gs; ++k) {
        const float x = rb(rb(bf2f(p[k]) - lo) / sc);
        const float qv = fminf(fmaxf(rintf(x), 0.f), 15.f);
        qp[k] = (uint8_t)qv;
        p[k] = f2bf(__fmaf_rn(qv - 8.f, sc, zr));
    }
    sz[idx] = (uint32_t)__builtin_bit_cast(uint16_t, f2bf(sc)) | ((uint32_t)__builtin_bit_cast(uint16_t, f2bf(zr)) << 16);
}
void launch_quant4(hipStream_t s, bf16_t* w, int N, int K, int gs, uint8_t* q, uint32_t* sz) {
    const int64_t n = (int64_t)N * (K / gs);
    quant4_kernel<<<(int)FM_CEIL(n, 256), 256, 0, s>>>(w, N, K, gs, q, sz);
}
// one thread per (unit, lane): word j of its 16 bytes = the 8 codes of k-step j (even e in the low
// half at nibble e / 2, odd e in the high half at nibble (e - 1) / 2)
__global__ void pack_q4_kernel(const uint8_t* __restrict__ q, int N, int K, uint8_t* __restrict__ dst) {
    const int U = K >> 7;
    const int64_t n = (int64_t)((N + 15) / 16) * U * 64;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t unit = i >> 6;
        const int l = (int)(i & 63);
        const int t = (int)(unit / U), u = (int)(unit - (int64_t)t * U);
        const int row = 16 * t + (l & 15);
        uint32_t wd[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t v = 0;
#pragma unroll
            for (int e = 0; e < 8; ++e)
                v |= (uint32_t)(row < N ? q[(size_t)row * K + 128 * u + 32 * j + 8 * (l >> 4) + e] & 15 : 8)
                     << ((e & 1) ? 16 + 4 * (e >> 1) : 4 * (e >> 1));
            wd[j] = v;
        }
        *reinterpret_cast<u32x4_t*>(dst + i * 16) = (u32x4_t){wd[0], wd[1], wd[2], wd[3]};
    }
}
__global__ void pack_q4_rows_kernel(const uint8_t* __restrict__ q, int64_t nw, uint32_t* __restrict__ dst) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t v = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) v |= (uint32_t)(q[i * 8 + e] & 15) << ((e & 1) ? 16 + 4 * (e >> 1) : 4 * (e >> 1));
        dst[i] = v;
    }
}
void launch_pack_q4_rows(hipStream_t s, const uint8_t* q, int N, int K, uint32_t* dst) {
    const int64_t nw = (int64_t)N * (K / 8);
    pack_q4_rows_kernel<<<(int)std::min<int64_t>(FM_CEIL(nw, 256), 16384), 256, 0, s>>>(q, nw, dst);
}
void launch_pack_q4(hipStream_t s, const uint8_t* q, int N, int K, uint8_t* dst) {
    const int64_t n = (int64_t)((N + 15) / 16) * (K / 128) * 64;
    pack_q4_kernel<<<(int)std::min<int64_t>(FM_CEIL(n, 256), 16384), 256, 0, s>>>(q, N, K, dst);
}
__global__ void pack_sz4_kernel(const uint32_t* __restrict__ sz, int N, int K, int gs, uint32_t* __restrict__ dst) {
    const int U = K >> 7, ng = K / gs;
    const int64_t n = (int64_t)((N + 15) / 16) * U * 16;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t tu = i >> 4;
        const int r = (int)(i & 15);
        const int t = (int)(tu / U), u = (int)(tu - (int64_t)t * U);
        const int row = 16 * t + r;
        dst[i] = row < N ? sz[(size_t)row * ng + (128 * u) / gs] : 0u;
    }
}
void launch_pack_sz4(hipStream_t s, const uint32_t* sz, int N, int K, int gs, uint32_t* dst) {
    const int64_t n = (int64_t)((N + 15) / 16) * (K / 128) * 16;
    pack_sz4_kernel<<<(int)std::min<int64_t>(FM_CEIL(n, 256), 16384), 256, 0, s>>>(sz, N, K, gs, dst);
}
template void launch_quant_rows<bf16_t>(hipStream_t, bf16_t*, int, int, int8_t*, bf16_t*);
template void launch_quant_rows<float>(hipStream_t, float*, int, int, int8_t*, float*);
template void launch_i8_to<bf16_t>(hipStream_t, const int8_t*, int64_t, bf16_t*);
template void launch_i8_to<float>(hipStream_t, const int8_t*, int64_t, float*);

template <typename T>
__global__ void swiglu_i8_kernel(const T* __restrict__ t, int ldt, T* __restrict__ act, int lda, int inter, int R) {
    const int64_t n = (int64_t)R * inter;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
        const int r = (int)(q / inter), j = (int)(q - (int64_t)r * inter);
        const T* tr = t + (size_t)r * ldt + 16 * (j >> 3) + (j & 7);
        const float g = ld(tr, 0), u = ld(tr, 8);
        st(act + (size_t)r * lda, j, rnd<T>(g / (1.0f + expf(-g))) * u);
    }
}
template <typename T> void launch_swiglu_i8(hipStream_t s, const T* t, int ldt, T* act, int lda, int inter, int R) {
    const int64_t n = (int64_t)R * inter;
    swiglu_i8_kernel<T><<<(int)std::min<int64_t>(FM_CEIL(n, 256), 16384), 256, 0, s>>>(t, ldt, act, lda, inter, R);
}
template void launch_swiglu_i8<bf16_t>(hipStream_t, const bf16_t*, int, bf16_t*, int, int, int);
template void launch_swiglu_i8<float>(hipStream_t, const float*, int, float*, int, int, int);
template void launch_pack<float>(hipStream_t, const float*, int, int, float*);


__device__ __forceinline__ float silu_f(float a) { return a / (1.0f + expf(-a)); }

template <typename T, int EPI>
__device__ __forceinline__ void linear_epi(const LinearArgs<T>& a, int n, int col, float v0, float v1) {
    const size_t yi = (size_t)col * a.ldy + n;
    if (a.wscale) v0 = rnd<T>(rnd<T>(v0) * ld(a.wscale, n));  // WeightOnlyInt8Linear (no bias)
    if (a.bias) v0 += ld(a.bias, n);
    if constexpr (EPI == EPI_STORE) {
        st(a.Y, yi, v0);
    } else if constexpr (EPI == EPI_RESID) {
        st(a.Y, yi, ld(a.res, (size_t)col * a.ldr + n) + rnd<T>(v0));
    } else if constexpr (EPI == EPI_SWIGLU) {
        const float ga = rnd<T>(v0), ub = rnd<T>(v1);
        st(a.Y, yi, rnd<T>(silu_f(ga)) * ub);
    } else {  // EPI_F32: logits as fp32 holding the T-rounded value
        a.Yf[yi] = rnd<T>(v0);
    }
}

// grid = (N/16 tiles, ksb K-slices).  ksb > 1 (host: R <= 16 * NCG): every block reduces its
// waves in LDS, stores its fp32 tile partial write-through (sc1), drains, takes a relaxed agent
// ticket; the tile's last-arriving block sums the ksb partials in slice order (deterministic)
// with sc1 loads and runs the epilogue (cdna_hip_programming.md split-K recipe, the same hand-off
// as gemv_kernel's EPI_SLABFIN).
template <typename T, int NCG, int EPI, int U>
__global__ __launch_bounds__(512) void linear_kernel(LinearArgs<T> a) {
    using M = Frag<T>;
    constexpr int NACC = (EPI == EPI_SWIGLU) ? 2 : 1;
    __shared__ f32x4_t red[8][NACC * NCG][64];
    __shared__ int last_flag;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = blockIdx.x * 16;
    const int r = lane & 15, g = lane >> 4;
    const int nsteps = a.K >> 5;
    const int ksb = gridDim.y, ks = blockIdx.y;
    const int b0 = (ks * nsteps) / ksb, b1 = ((ks + 1) * nsteps) / ksb;
    const int s0 = b0 + ((wave * (b1 - b0)) >> 3), s1 = b0 + (((wave + 1) * (b1 - b0)) >> 3);
    // packed weights: block (tile, step) = 512 elements
    const T* wp = a.W + (size_t)blockIdx.x * nsteps * 512;
    const T* wp2 = (EPI == EPI_SWIGLU) ? a.W2 + (size_t)blockIdx.x * nsteps * 512 : nullptr;

    for (int c0 = 0; c0 < a.R; c0 += 16 * NCG) {
        f32x4_t acc[NACC][NCG];
        const T* xp[NCG];
#pragma unroll
        for (int c = 0; c < NCG; ++c) {
            int col = c0 + 16 * c + r;
            col = col < a.R ? col : a.R - 1;  // out-of-range columns read a valid row; discarded
            xp[c] = a.X + (size_t)col * a.ldx + 8 * g;
#pragma unroll
            for (int q = 0; q < NACC; ++q) acc[q][c] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        }
        int s = s0;
        for (; s + U <= s1; s += U) {
            typename M::f fa[NACC][U], fb[NCG][U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                fa[0][u] = M::load_w(wp + (size_t)(s + u) * 512, lane);
                if constexpr (NACC == 2) fa[1][u] = M::load_w(wp2 + (size_t)(s + u) * 512, lane);
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < NCG; ++c) fb[c][u] = M::load(xp[c] + (size_t)(s + u) * 32);
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < NCG; ++c)
#pragma unroll
                    for (int q = 0; q < NACC; ++q) acc[q][c] = M::mma(fa[q][u], fb[c][u], acc[q][c]);
        }
        for (; s < s1; ++s) {
            typename M::f fa0 = M::load_w(wp + (size_t)s * 512, lane);
            typename M::f fa1;
            if constexpr (NACC == 2) fa1 = M::load_w(wp2 + (size_t)s * 512, lane);
#pragma unroll
            for (int c = 0; c < NCG; ++c) {
                typename M::f fb = M::load(xp[c] + (size_t)s * 32);
                acc[0][c] = M::mma(fa0, fb, acc[0][c]);
                if constexpr (NACC == 2) acc[1][c] = M::mma(fa1, fb, acc[1][c]);
            }
        }
#pragma unroll
        for (int q = 0; q < NACC; ++q)
#pragma unroll
            for (int c = 0; c < NCG; ++c) red[wave][q * NCG + c][lane] = acc[q][c];
        __syncthreads();
        // 16 rows x (16*NCG) cols; C/D map: row = 4*(lane>>4)+i, col = lane&15
        for (int o = threadIdx.x; o < 256 * NCG; o += 512) {
            const int c = o >> 8, rem = o & 255, i = rem >> 6, ln = rem & 63;
            const int n = n0 + 4 * (ln >> 4) + i;
            const int col = c0 + 16 * c + (ln & 15);
            float v0 = 0.f, v1 = 0.f;
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                v0 += red[w][c][ln][i];
                if constexpr (NACC == 2) v1 += red[w][NCG + c][ln][i];
            }
            if (n < a.N && col < a.R) {
                if (ksb == 1) {
                    linear_epi<T, EPI>(a, n, col, v0, v1);
                } else {
                    float* pp = a.part + (((size_t)ks * NACC) * a.R + col) * a.N + n;
                    __hip_atomic_store(pp, v0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if constexpr (NACC == 2)
                        __hip_atomic_store(pp + (size_t)a.R * a.N, v1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        if (ksb > 1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) {
                const int t = __hip_atomic_fetch_add(a.tickets + blockIdx.x, 1, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                const int last = t == ksb - 1;
                if (last) __hip_atomic_store(a.tickets + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last_flag = last;
            }
            __syncthreads();
            if (!last_flag) return;  // host guarantees a single column group (R <= 16 * NCG)
            for (int o = threadIdx.x; o < 16 * a.R; o += 512) {
                const int col = o >> 4, n = n0 + (o & 15);
                if (n >= a.N) continue;
                float v0 = 0.f, v1 = 0.f;
                for (int q = 0; q < ksb; ++q) {
                    const float* pp = a.part + (((size_t)q * NACC) * a.R + col) * a.N + n;
                    v0 += __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if constexpr (NACC == 2)
                        v1 += __hip_atomic_load(pp + (size_t)a.R * a.N, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                linear_epi<T, EPI>(a, n, col, v0, v1);
            }
        }
        __syncthreads();
    }
}

// =========================================================================================
// qk-norm + RoPE + KV-cache write (llama.py:894-910, 205-214).  One wave per head.
// =========================================================================================
template <typename T>
__global__ __launch_bounds__(256) void qk_rope_cache_kernel(QkArgs<T> a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = blockIdx.x;
    const int head = blockIdx.y * 4 + wave;
    const int nheads = a.nh + 2 * a.nkv;
    if (head >= nheads) return;
    const int pos = a.fixed_pos >= 0 ? a.fixed_pos : a.row_pos[r];
    const int slot = a.row_slot[r];
    const int hd = a.hd, half = hd >> 1;
    const T* src = a.qkv + (size_t)r * a.ldqkv + (size_t)head * hd;
    const int kind = head < a.nh ? 0 : (head < a.nh + a.nkv ? 1 : 2);
    float x0[2], x1[2];
    int np = 0;
    for (int p = lane; p < half; p += 64, ++np) {
        if (a.qslab) {  // round(sum of the K slices + bias): the split-K epilogue's one rounding
            const size_t c = (size_t)head * hd + 2 * p;
            float v0 = 0.f, v1 = 0.f;
            for (int q = 0; q < a.qslab_kp; ++q) {
                const float* sp = a.qslab + ((size_t)q * gridDim.x + r) * a.ldqkv + c;
                v0 += sp[0];
                v1 += sp[1];
            }
            if (a.qbias) {
                v0 += ld(a.qbias, c);
                v1 += ld(a.qbias, c + 1);
            }
            x0[np] = rnd<T>(v0);
            x1[np] = rnd<T>(v1);
        } else {
            x0[np] = ld(src, 2 * p);
            x1[np] = ld(src, 2 * p + 1);
        }
    }
    if (kind < 2 && a.qk_norm) {
        float ss = 0.f;
        for (int i = 0; i < np; ++i) ss += x0[i] * x0[i] + x1[i] * x1[i];
        ss = wave_sum(ss);
        const float rs = 1.0f / sqrtf(ss / (float)hd + a.eps);
        const T* w = kind == 0 ? a.qn : a.kn;
        for (int i = 0; i < np; ++i) {
            const int p = lane + 64 * i;
            x0[i] = rnd<T>((x0[i] * rs) * ld(w, 2 * p));
            x1[i] = rnd<T>((x1[i] * rs) * ld(w, 2 * p + 1));
        }
    }
    if (kind < 2) {
        const float* tab = a.rope + (size_t)pos * hd;
        for (int i = 0; i < np; ++i) {
            const int p = lane + 64 * i;
            const float c = tab[2 * p], s = tab[2 * p + 1];
            const float y0 = x0[i] * c - x1[i] * s;
            const float y1 = x1[i] * c + x0[i] * s;
            x0[i] = rnd<T>(y0);
            x1[i] = rnd<T>(y1);
        }
    }
    T* dst;
    if (kind == 0) {
        dst = a.qout + (size_t)r * a.nh * hd + (size_t)head * hd;
    } else {
        const int kvh = kind == 1 ? head - a.nh : head - a.nh - a.nkv;
        T* base = (kind == 1 ? a.kc : a.vc) + (size_t)slot * a.slot_stride + a.layer_off;
        dst = base + ((size_t)kvh * a.S + pos) * hd;
    }
    for (int i = 0; i < np; ++i) {
        const int p = lane + 64 * i;
        st(dst, 2 * p, x0[i]);
        st(dst, 2 * p + 1, x1[i]);
    }
}

// =========================================================================================
// slow attention: split-K flash decode over the valid prefix [0, pos]
// grid (R, nkv, nsplit); each wave owns q-heads of the GQA group and the KV tile is shared.
// =========================================================================================
template <typename T>
__global__ __launch_bounds__(256) void attn_split_kernel(AttnArgs<T> a) {
    __shared__ float qs[4][256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = blockIdx.x, kvh = blockIdx.y, sp = blockIdx.z;
    const int pos = a.row_pos[r];
    const int j0 = sp * a.split;
    if (j0 > pos) return;
    const int j1 = min(j0 + a.split, pos + 1);
    const int slot = a.row_slot[r];
    const int hd = a.hd;
    const T* kc = a.kc + (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * hd;
    const T* vc = a.vc + (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * hd;
    const int g = a.nh / a.nkv;
    for (int qh = wave; qh < g; qh += 4) {
        const int h = kvh * g + qh;
        const T* q = a.q + (size_t)r * a.nh * hd + (size_t)h * hd;
        for (int e = lane; e < hd; e += 64) qs[wave][e] = ld(q, e);
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        float m = -INFINITY, l = 0.f;
        float o[4] = {0.f, 0.f, 0.f, 0.f};
        for (int jc = j0; jc < j1; jc += 64) {
            const int j = jc + lane;
            float sc = -INFINITY;
            if (j < j1) {
                const T* kr = kc + (size_t)j * hd;
                float dot = 0.f;
                for (int e = 0; e < hd; e += 8) {
                    float kv[8];
                    load8(kr + e, kv);
#pragma unroll
                    for (int u = 0; u < 8; ++u) dot += qs[wave][e + u] * kv[u];
                }
                sc = dot * a.scale;
            }
            const float mn = fmaxf(m, wave_max(sc));
            const float alpha = expf(m - mn);
            const float p = (j < j1) ? expf(sc - mn) : 0.f;
            l = l * alpha + wave_sum(p);
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] *= alpha;
            const int nv = min(64, j1 - jc);
            for (int jj = 0; jj < nv; ++jj) {
                const float pj = __shfl(p, jj, 64);
                const T* vr = vc + (size_t)(jc + jj) * hd;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int e = lane + 64 * i;
                    if (e < hd) o[i] += pj * ld(vr, e);
                }
            }
            m = mn;
        }
        float* out = a.part + (((size_t)r * a.nh + h) * a.maxsplit + sp) * (hd + 2);
        if (lane == 0) {
            out[0] = m;
            out[1] = l;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = lane + 64 * i;
            if (e < hd) out[2 + e] = o[i];
        }
        __builtin_amdgcn_wave_barrier();
    }
}


// =========================================================================================
// prompt attention (causal SDPA of a prefill chunk, llama.py:883-946), bf16, head_dim HD:
// flash form on MFMA.  Block = one kv head x 16 consecutive rows; wave w = q head kvh*g + w of the
// GQA group (g <= 4), so every K/V tile staged in LDS serves the whole group.  Per 32-key tile:
// S = Q K^T (16 x 32, fp32), scale + causal mask, online softmax in fp32 (running max / sum per
// row), P rounded to bf16 for the P V MFMA (as a bf16 SDPA does), O in fp32; out = round(O / l).
// =========================================================================================
template <int HD>
__global__ __launch_bounds__(256) void attn_prefill_kernel(AttnArgs<bf16_t> a, int R, bf16_t* __restrict__ out) {
    using F = Frag<bf16_t>;
    constexpr int KT = 32, KP = HD + 8, VP = KT + 8;
    __shared__ __attribute__((aligned(16))) bf16_t ks[KT][KP];     // K tile [key][dim]
    __shared__ __attribute__((aligned(16))) bf16_t vt[HD][VP];     // V tile transposed [dim][key]
    __shared__ __attribute__((aligned(16))) bf16_t ps[4][16][VP];  // per-wave P [row][key]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kvh = blockIdx.y, r0 = blockIdx.x * 16;
    const int g = a.nh / a.nkv;
    const bool active = wave < g;
    const int h = kvh * g + (active ? wave : 0);
    const int slot = a.row_slot[r0];
    int maxpos = 0;
    for (int i = 0; i < 16; ++i) maxpos = max(maxpos, a.row_pos[min(r0 + i, R - 1)]);
    const bf16_t* kc = a.kc + (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * HD;
    const bf16_t* vc = a.vc + (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * HD;
    // Q as A fragments: lane l -> row r0 + (l & 15), dims 32c + 8 (l >> 4) .. + 8
    const int qa_row = min(r0 + (lane & 15), R - 1);
    F::f qf[HD / 32];
#pragma unroll
    for (int c = 0; c < HD / 32; ++c)
        qf[c] = F::load(a.q + (size_t)qa_row * a.nh * HD + (size_t)h * HD + 32 * c + 8 * (lane >> 4));
    // this lane's S / O rows: 4 (l >> 4) + i
    int prow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) prow[i] = a.row_pos[min(r0 + 4 * (lane >> 4) + i, R - 1)];
    f32x4_t o[HD / 16];
#pragma unroll
    for (int t = 0; t < HD / 16; ++t) o[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    float mrow[4], lrow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        mrow[i] = -INFINITY;
        lrow[i] = 0.f;
    }
    constexpr int CPK = HD / 8;  // 16-B chunks per key row
    for (int j0 = 0; j0 <= maxpos; j0 += KT) {
        __syncthreads();  // the previous tile's LDS reads are done
        for (int c = tid; c < KT * CPK; c += 256) {
            const int key = c / CPK, ch = c - key * CPK, jj = j0 + key;
            const bool ok = jj <= maxpos;
            const size_t off = (size_t)(ok ? jj : 0) * HD + 8 * ch;
            u32x4_t kv = *reinterpret_cast<const u32x4_t*>(kc + off);
            u32x4_t vv = *reinterpret_cast<const u32x4_t*>(vc + off);
            if (!ok) kv = vv = (u32x4_t){0u, 0u, 0u, 0u};
            *reinterpret_cast<u32x4_t*>(&ks[key][8 * ch]) = kv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                reinterpret_cast<uint16_t*>(&vt[8 * ch + 2 * e][key])[0] = (uint16_t)(vv[e] & 0xffffu);
                reinterpret_cast<uint16_t*>(&vt[8 * ch + 2 * e + 1][key])[0] = (uint16_t)(vv[e] >> 16);
            }
        }
        __syncthreads();
        if (!active) continue;
        f32x4_t sc[2];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            sc[hf] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < HD / 32; ++c) {
                const F::f kb = *reinterpret_cast<const u32x4_t*>(&ks[16 * hf + (lane & 15)][32 * c + 8 * (lane >> 4)]);
                sc[hf] = F::mma(qf[c], kb, sc[hf]);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float sv[2];
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int key = j0 + 16 * hf + (lane & 15);
                sv[hf] = key <= prow[i] ? sc[hf][i] * a.scale : -INFINITY;
            }
            float mx = fmaxf(sv[0], sv[1]);
#pragma unroll
            for (int d = 1; d < 16; d <<= 1) mx = fmaxf(mx, __shfl_xor(mx, d, 64));
            const float mn = fmaxf(mrow[i], mx);
            const float al = mn == -INFINITY ? 1.f : expf(mrow[i] - mn);
            const float p0 = sv[0] == -INFINITY ? 0.f : expf(sv[0] - mn);
            const float p1 = sv[1] == -INFINITY ? 0.f : expf(sv[1] - mn);
            float sum = p0 + p1;
#pragma unroll
            for (int d = 1; d < 16; d <<= 1) sum += __shfl_xor(sum, d, 64);
            lrow[i] = lrow[i] * al + sum;
            mrow[i] = mn;
#pragma unroll
            for (int t = 0; t < HD / 16; ++t) o[t][i] *= al;
            const int prr = 4 * (lane >> 4) + i;
            ps[wave][prr][lane & 15] = f2bf(p0);
            ps[wave][prr][16 + (lane & 15)] = f2bf(p1);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const F::f pf = *reinterpret_cast<const u32x4_t*>(&ps[wave][lane & 15][8 * (lane >> 4)]);
#pragma unroll
        for (int t = 0; t < HD / 16; ++t) {
            const F::f vf = *reinterpret_cast<const u32x4_t*>(&vt[16 * t + (lane & 15)][8 * (lane >> 4)]);
            o[t] = F::mma(pf, vf, o[t]);
        }
        __builtin_amdgcn_wave_barrier();  // ps is rewritten by the next tile
    }
    if (!active) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = r0 + 4 * (lane >> 4) + i;
        if (row >= R) continue;
        const float inv = 1.0f / lrow[i];
        bf16_t* orow = out + (size_t)row * a.nh * HD + (size_t)h * HD;
#pragma unroll
        for (int t = 0; t < HD / 16; ++t) st(orow, 16 * t + (lane & 15), o[t][i] * inv);
    }
}

template <typename T>
__global__ __launch_bounds__(64) void attn_combine_kernel(const float* __restrict__ part,
                                                          const int* __restrict__ row_pos, int nh,
                                                          int hd, int split, int maxsplit,
                                                          T* __restrict__ out) {
    const int r = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
    const int ns = row_pos[r] / split + 1;
    const float* p = part + ((size_t)r * nh + h) * maxsplit * (hd + 2);
    float M = -INFINITY;
    for (int s = 0; s < ns; ++s) M = fmaxf(M, p[(size_t)s * (hd + 2)]);
    float L = 0.f;
    for (int s = 0; s < ns; ++s) L += p[(size_t)s * (hd + 2) + 1] * expf(p[(size_t)s * (hd + 2)] - M);
    for (int e = lane; e < hd; e += 64) {
        float o = 0.f;
        for (int s = 0; s < ns; ++s)
            o += p[(size_t)s * (hd + 2) + 2 + e] * expf(p[(size_t)s * (hd + 2)] - M);
        st(out, (size_t)r * nh * hd + (size_t)h * hd + e, o / L);
    }
}

// =========================================================================================
// fast attention (llama.py:947-975): s = round(round(q.k) * scale), masked j > cpos,
// p = round(softmax(s)), y = round(p @ v).  grid (R, nh), one wave.
// =========================================================================================
template <typename T>
__global__ __launch_bounds__(64) void fast_attn_kernel(FastAttnArgs<T> a) {
    const int lane = threadIdx.x;
    const int r = blockIdx.x, h = blockIdx.y;
    const int slot = a.row_slot[r];
    const int hd = a.hd, g = a.nh / a.nkv, kvh = h / g;
    const T* q = a.q + (size_t)r * a.nh * hd + (size_t)h * hd;
    const T* kc = a.kc + (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * hd;
    const T* vc = a.vc + (size_t)slot * a.slot_stride + a.layer_off + (size_t)kvh * a.S * hd;
    float sc = -INFINITY;
    if (lane < a.S && lane <= a.cpos) {
        float dot = 0.f;
        for (int e = 0; e < hd; ++e) dot += ld(q, e) * ld(kc + (size_t)lane * hd, e);
        sc = rnd<T>(rnd<T>(dot) * a.scale);
    }
    __shared__ float ps[64];
    const float mx = wave_max(sc);
    const float ex = (sc == -INFINITY) ? 0.f : expf(sc - mx);
    const float den = wave_sum(ex);
    ps[lane] = rnd<T>(ex / den);
    __syncthreads();
    for (int e = lane; e < hd; e += 64) {
        float o = 0.f;
        for (int j = 0; j < a.S; ++j) o += ps[j] * ld(vc + (size_t)j * hd, e);
        st(a.out, (size_t)r * a.nh * hd + (size_t)h * hd + e, o);
    }
}

// =========================================================================================
// frame bookkeeping: RAS window roll (inference.py:227-230), next input column, pos/step++
// =========================================================================================
__global__ void finish_kernel(int R, const int* __restrict__ row_slot, int* __restrict__ row_pos,
                              const int32_t* __restrict__ cols, int ldc, int32_t* __restrict__ tok_in,
                              int32_t* __restrict__ ras, int ras_stride, int C1, int update_ras,
                              SlotParams* __restrict__ sp) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const int slot = row_slot[r];
    const int32_t* col = cols + (size_t)r * ldc;
    for (int q = 0; q < C1; ++q) tok_in[(size_t)slot * C1 + q] = col[q];
    if (update_ras) {
        int32_t* w = ras + (size_t)slot * ras_stride;
        for (int q = 0; q < C1; ++q) {
            for (int j = 0; j < 9; ++j) w[q * 10 + j] = w[q * 10 + j + 1];
            w[q * 10 + 9] = col[q];
        }
    }
    row_pos[r] += 1;
    sp[slot].step += 1;
}

// =========================================================================================
// synthetic weights (fishmi/synth.py formula) and small utilities
// =========================================================================================
template <typename T>
__global__ void synth_kernel(T* __restrict__ dst, int64_t n, uint64_t base, float center,
                             float scale) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t m = (int64_t)(splitmix64(base + (uint64_t)i) >> 40);
        const float rr = (float)(2 * m - (1 << 24)) * scale;
        const float v = __fadd_rn(center, rr);
        st(dst, i, bfround(v));  // synthetic weights are bf16-valued in both precisions
    }
}

template <typename T>
__global__ void convert_kernel(const void* __restrict__ src, int src_bf16, int64_t n,
                               T* __restrict__ dst) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float v = src_bf16 ? bf2f(((const bf16_t*)src)[i]) : ((const float*)src)[i];
        st(dst, i, v);
    }
}

// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
template <typename T>
void launch_embed(hipStream_t s, const int32_t* tok, int R, const T* emb, const T* cbemb, int d,
                  int C, int cb, int sb, int se, int scale, T* x, const int* row_slot) {
    embed_kernel<T><<<dim3(R, FM_CEIL(d, 2048)), 256, 0, s>>>(tok, R, emb, cbemb, d, C, cb, sb, se, scale, x, row_slot);
}
template <typename T>
void launch_gather_rows(hipStream_t s, const int32_t* codes, int ldc, int col, const T* table,
                        int d, int rows, int R, T* x) {
    gather_rows_kernel<T><<<R, 256, 0, s>>>(codes, ldc, col, table, d, rows, x);
}
template <typename T>
void launch_rmsnorm(hipStream_t s, const T* x, int ldx, const T* w, int d, float eps, T* y,
                    int ldy, int R) {
    const bool vec = d % 8 == 0 && d <= 512 * RN_MAXC && ldx % 8 == 0 && ldy % 8 == 0 &&
                     ((uintptr_t)x | (uintptr_t)w | (uintptr_t)y) % 16 == 0 && !fm_tuning().rmsnorm_block;
    if (vec)
        rmsnorm_wave_kernel<T><<<FM_CEIL(R, 4), 256, 0, s>>>(x, ldx, w, d, eps, y, ldy, R);
    else
        rmsnorm_kernel<T><<<R, 256, 0, s>>>(x, ldx, w, d, eps, y, ldy);
}

// K-slices for the batched decode path: enough blocks to cover the chip (>= tu.linear_fill), each
// slice at least 8 k-steps (one per wave), one column group (R <= 64), partials within the
// caller's buffer (LINEAR_PART_CAP floats)
int linear_ksb(int N, int K, int R, int nacc, bool can_split) {
    const FmTuning& tu = fm_tuning();
    if (!can_split || R > 64 || tu.linear_fill <= 0) return 1;
    const int tiles = FM_CEIL(N, 16), nsteps = K >> 5;
    int ksb = 1;
    while (ksb < 16 && tiles * ksb < tu.linear_fill && nsteps / (2 * ksb) >= 8 &&
           (size_t)2 * ksb * nacc * R * N <= LINEAR_PART_CAP)
        ksb *= 2;
    return ksb;
}

template <typename T, int EPI>
static void linear_dispatch(hipStream_t s, const LinearArgs<T>& a) {
    const int tiles = FM_CEIL(a.N, 16);
    dim3 grid(tiles, linear_ksb(a.N, a.K, a.R, EPI == EPI_SWIGLU ? 2 : 1, a.part != nullptr && a.tickets != nullptr));
    if (a.R <= 16)
        linear_kernel<T, 1, EPI, 8><<<grid, 512, 0, s>>>(a);
    else if (a.R <= 32) {
        if (fm_tuning().linear_u32 == 8)
            linear_kernel<T, 2, EPI, 8><<<grid, 512, 0, s>>>(a);
        else
            linear_kernel<T, 2, EPI, 4><<<grid, 512, 0, s>>>(a);
    } else
        linear_kernel<T, 4, EPI, 4><<<grid, 512, 0, s>>>(a);
}
template <typename T> void launch_linear(hipStream_t s, const LinearArgs<T>& a, int epi) {
    switch (epi) {
        case EPI_STORE: linear_dispatch<T, EPI_STORE>(s, a); break;
        case EPI_RESID: linear_dispatch<T, EPI_RESID>(s, a); break;
        case EPI_SWIGLU: linear_dispatch<T, EPI_SWIGLU>(s, a); break;
        default: linear_dispatch<T, EPI_F32>(s, a); break;
    }
}
template <typename T> void launch_qk_rope_cache(hipStream_t s, const QkArgs<T>& a, int R) {
    dim3 grid(R, FM_CEIL(a.nh + 2 * a.nkv, 4));
    qk_rope_cache_kernel<T><<<grid, 256, 0, s>>>(a);
}
template <typename T> void launch_attn(hipStream_t s, const AttnArgs<T>& a, int R, int nsplit, T* out, bool one_slot) {
    if constexpr (is_bf16<T>::value) {
        if (one_slot && fm_tuning().prefill_attn && a.hd == 128 && a.nh % a.nkv == 0 && a.nh / a.nkv <= 4) {
            attn_prefill_kernel<128><<<dim3(FM_CEIL(R, 16), a.nkv), 256, 0, s>>>(a, R, out);
            return;
        }
    }
    dim3 g1(R, a.nkv, nsplit);
    attn_split_kernel<T><<<g1, 256, 0, s>>>(a);
    dim3 g2(R, a.nh);
    attn_combine_kernel<T><<<g2, 64, 0, s>>>(a.part, a.row_pos, a.nh, a.hd, a.split, a.maxsplit, out);
}
template <typename T>
void launch_attn_combine(hipStream_t s, const float* part, const int* row_pos, int R, int nh, int hd,
                         int split, int maxsplit, T* out) {
    attn_combine_kernel<T><<<dim3(R, nh), 64, 0, s>>>(part, row_pos, nh, hd, split, maxsplit, out);
}
template <typename T> void launch_fast_attn(hipStream_t s, const FastAttnArgs<T>& a, int R) {
    dim3 g(R, a.nh);
    fast_attn_kernel<T><<<g, 64, 0, s>>>(a);
}
void launch_finish(hipStream_t s, int R, const int* row_slot, int* row_pos, const int32_t* cols,
                   int ldc, int32_t* tok_in, int32_t* ras, int ras_stride, int C1, int update_ras,
                   SlotParams* sp) {
    finish_kernel<<<FM_CEIL(R, 64), 64, 0, s>>>(R, row_slot, row_pos, cols, ldc, tok_in, ras,
                                               ras_stride, C1, update_ras, sp);
}
template <typename T>
void launch_synth(hipStream_t s, T* dst, int64_t n, uint64_t seed, uint32_t tid, float center,
                  int log2_half) {
    const uint64_t base = seed * 0xD1B54A32D192ED03ull + (uint64_t)tid * 0x9E3779B97F4A7C15ull;
    const float scale = ldexpf(1.0f, -24 - log2_half);
    int blocks = (int)std::min<int64_t>(FM_CEIL(n, 256), 8192);
    synth_kernel<T><<<blocks, 256, 0, s>>>(dst, n, base, center, scale);
}
template <typename T>
void launch_convert(hipStream_t s, const void* src, int src_bf16, int64_t n, T* dst) {
    int blocks = (int)std::min<int64_t>(FM_CEIL(n, 256), 8192);
    convert_kernel<T><<<blocks, 256, 0, s>>>(src, src_bf16, n, dst);
}

#define INST(T)                                                                                  \
    template void launch_embed<T>(hipStream_t, const int32_t*, int, const T*, const T*, int, int, \
                                  int, int, int, int, T*, const int*);                           \
    template void launch_gather_rows<T>(hipStream_t, const int32_t*, int, int, const T*, int, int, \
                                        int, T*);                                                   \
    template void launch_rmsnorm<T>(hipStream_t, const T*, int, const T*, int, float, T*, int, int); \
    template void launch_linear<T>(hipStream_t, const LinearArgs<T>&, int);                      \
    template void launch_qk_rope_cache<T>(hipStream_t, const QkArgs<T>&, int);                   \
    template void launch_attn<T>(hipStream_t, const AttnArgs<T>&, int, int, T*, bool);           \
    template void launch_fast_attn<T>(hipStream_t, const FastAttnArgs<T>&, int);                 \
    template void launch_attn_combine<T>(hipStream_t, const float*, const int*, int, int, int, int, \
                                         int, T*);                                               \
    template void launch_synth<T>(hipStream_t, T*, int64_t, uint64_t, uint32_t, float, int);    \
    template void launch_convert<T>(hipStream_t, const void*, int, int64_t, T*);
INST(bf16_t)
INST(float)

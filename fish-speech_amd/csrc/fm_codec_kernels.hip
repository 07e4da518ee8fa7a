// fm_codec_kernels.hip -- gfx950 kernels of the modded-DAC decode path (DAC.from_indices,
// modded_dac.py:925-927).  All activations are time-major [t][channel] so that every causal
// conv, transposed conv and linear layer is one implicit GEMM with channels on the MFMA k axis:
//
//   conv_gemm_kernel   out[t*stride+phase][co] = sum_{tap,ci} W[phase][co][tap,ci] x[t-shift][ci]
//                      CausalConvNet (modded_dac.py:521-552): stride 1, taps j, shift (k-1-j)*dil
//                      CausalTransConvNet (modded_dac.py:563-580, rvq.py:100-117): one GEMM per
//                      output phase, taps {0: x[t], 1: x[t-1]} (kernel 2s) or {0} (kernel s)
//                      nn.Linear: one tap.  Epilogues: bias, GELU, LayerScale/residual, SiLU-mul
//                      (SwiGLU), tanh, and Snake1d of the NEXT stage (descript Snake1d:
//                      x + (a+1e-9)^-1 sin^2(a x)) written to a second buffer.
//   rvq_decode_kernel  rvq.py:352-366 + descript ResidualVectorQuantize.from_codes
//   dwconv_ln_kernel   ConvNeXt depthwise causal k7 + LayerNorm (rvq.py:176-178)
//   rope_qk_kernel / window_attn_kernel   WindowLimitedTransformer (modded_dac.py:349-439)
#include <algorithm>

#include "fm_codec.h"
#include "fm_kernels.h"
#include "fm_runtime.h"
#include "fm_frag.h"

// sin^2(x) for the Snake epilogues (descript Snake1d: x + (a+1e-9)^-1 sin^2(a x)), applied to every
// output element, twice per ResidualUnit: the hardware sine (v_sin_f32, argument in revolutions) of
// the fractional revolution x / 2 pi -- three VALU slots and one transcendental instead of a
// Cody-Waite reduction and a polynomial (the epilogues, not the MFMAs, bound the narrow decoder
// stages).  The reduction to [0, 1) keeps the argument inside v_sin_f32's domain at any |x|.
__device__ __forceinline__ float sin2_f(float x) {
    const float s = __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(x * 0.159154943091895336f));
    return s * s;
}
__device__ __forceinline__ float snake_f(float y, float al) {
    return y + (1.0f / (al + 1e-9f)) * sin2_f(al * y);
}
// the same with the channel's reciprocal precomputed (ia = 1.0f / (al + 1e-9f), bit-identical)
__device__ __forceinline__ float snake_fi(float y, float al, float ia) { return y + ia * sin2_f(al * y); }

template <typename T>
__global__ void snake_inv_kernel(const T* __restrict__ alpha, int64_t n, float* __restrict__ ia) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ia[i] = 1.0f / (ld(alpha, i) + 1e-9f);
}

// a.shift[tap] for a per-lane tap as arithmetic on two kernel-argument scalars: every conv here has
// shifts linear in the tap ((k-1-j)*dil causal, j transposed).  Indexing the argument array with a
// lane value makes the compiler fetch it with a vector memory load (and drain vmcnt before it),
// one dependent round trip in front of every X address.
template <typename T> __device__ __forceinline__ int conv_shift(const ConvArgs<T>& a, int tap) {
    return a.shift0 + tap * a.shiftd;
}

// block = 4 waves, block tile 64 time x 64 channels, wave tile 32 x 32 (2x2 MFMA 16x16x32)
template <typename T>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs<T> a) {
    using F = Frag<T>;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tq0 = blockIdx.x * 64 + (wave & 1) * 32;
    const int co0 = blockIdx.y * 64 + (wave >> 1) * 32;
    const int ks = a.ksplit > 1 ? a.ksplit : 1;
    const int phase = blockIdx.z % a.nphase, kz = blockIdx.z / a.nphase;
    if (co0 >= a.Co) return;
    const int r = lane & 15, g = lane >> 4;
    const int Kt = a.ntaps * a.Ci, S = (Kt + 31) >> 5;  // weights zero-padded to 32-multiples
    const int sb = (int)((long long)S * kz / ks), se = (int)((long long)S * (kz + 1) / ks);
    const T* wb = a.w + (size_t)phase * a.wphase;
    const bool c1 = co0 + 16 < a.Co;
    const int ct0 = co0 >> 4;
    f32x4_t acc[2][2];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[c][u] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int tq[2] = {tq0 + r, tq0 + 16 + r};
#pragma unroll 4
    for (int s = sb; s < se; ++s) {
        // this lane's 8-element chunk lies inside one tap (Ci % 8 == 0)
        const int kl = s * 32 + 8 * g;
        int tap = kl / a.Ci;
        const bool kin = tap < a.ntaps;
        tap = kin ? tap : a.ntaps - 1;
        const int ci0 = kin ? kl - tap * a.Ci : 0;
        const int sh = conv_shift(a, tap);
        typename F::f fa0 = F::load_w(wb + ((size_t)ct0 * S + s) * 512, lane);
        typename F::f fa1 = F::load_w(wb + ((size_t)(c1 ? ct0 + 1 : ct0) * S + s) * 512, lane);
        typename F::f fb[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int row = tq[u] - sh;
            const bool valid = kin && row >= a.lo && row < a.Lx;
            const int rc = row < a.lo ? a.lo : (row >= a.Lx ? a.Lx - 1 : row);
            fb[u] = F::load_masked(a.x + (ptrdiff_t)rc * a.ldx + ci0, valid);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            acc[0][u] = F::mma(fa0, fb[u], acc[0][u]);
            acc[1][u] = F::mma(fa1, fb[u], acc[1][u]);
        }
    }
    if (ks > 1) {  // split K: raw fp32 partials, the epilogue runs in conv_splitk_epi_kernel
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (c == 1 && !c1) break;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int t = tq0 + 16 * u + (lane & 15);
                if (t >= a.Lq) continue;
                float* dst = a.slab + ((size_t)(kz * a.nphase + phase) * a.Lq + t) * a.Co + co0 + 16 * c + 4 * (lane >> 4);
                *reinterpret_cast<f32x4_t*>(dst) = acc[c][u];
            }
        }
        return;
    }
    const int fl = a.flags;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (c == 1 && !c1) break;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int t = tq0 + 16 * u + (lane & 15);
            if (t >= a.Lq) continue;
            const int tout = t * a.stride + phase;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int co = co0 + 16 * c + 4 * (lane >> 4) + i;
                if (co >= a.Co) continue;
                float y = acc[c][u][i];
                if (fl & CE_BIAS) y += ld(a.bias, co);
                y = rnd<T>(y);
                if (fl & CE_GELU) y = rnd<T>(0.5f * y * (1.0f + erff(y * 0.70710678118654752f)));
                if (fl & CE_RES) {
                    const float rv = ld(a.res, (size_t)tout * a.ldr + co);
                    if (fl & CE_GAMMA) y = rnd<T>(rv + rnd<T>(ld(a.gamma, co) * y));
                    else y = rnd<T>(rv + y);
                }
                if (fl & CE_TANH) y = tanhf(y);
                if (fl & CE_STORE) {
                    if (fl & CE_F32OUT) reinterpret_cast<float*>(a.out)[(size_t)tout * a.ldo + co] = y;
                    else st(reinterpret_cast<T*>(a.out), (size_t)tout * a.ldo + co, y);
                }
                if (fl & CE_SNAKE) st(a.out2, (size_t)tout * a.ldo2 + co, snake_fi(y, ld(a.alpha2, co), a.ialpha2[co]));
            }
        }
    }
}

// split-K reduction + the conv epilogue on 8 consecutive channels per thread (16-B accesses):
// y = round(sum_kz partial + bias) -> GELU -> residual / LayerScale -> tanh -> store / Snake
// CE_SWIGLU: the GEMM's channels are [W1 rows | W3 rows]; thread (t, n) also sums the partials of
// channel Co/2 + n and writes round(round(silu(g1)) * g3), g = round(sum) -- silu_mul_kernel's
// roundings on the two GEMMs' stored outputs, so the result is bit-identical to the three launches.
// CE_SWIGLU8: the same over the 8-row interleave of the LLM's packed W1 || W3 (thread: gate channels
// 16 cc .. + 8, up channels 16 cc + 8 .. + 8, outputs 8 cc .. + 8), swiglu_i8_kernel's roundings.
template <typename T>
__global__ __launch_bounds__(256) void conv_splitk_epi_kernel(ConvArgs<T> a) {
    const int fl = a.flags;
    const bool sw8 = fl & CE_SWIGLU8;
    // the up channel's offset from the gate's: Co/2 ([W1 | W3]) or 8 (8-row interleave)
    const int half = (fl & CE_SWIGLU) ? a.Co >> 1 : (sw8 ? 8 : 0);
    const int cpr = sw8 ? a.Co >> 4 : ((fl & CE_SWIGLU) ? half : a.Co) >> 3;
    const size_t n = (size_t)a.nphase * a.Lq * cpr;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const int cc = (int)(i % cpr);
        const size_t pt = i / cpr;  // phase * Lq + t
        const int t = (int)(pt % a.Lq), phase = (int)(pt / a.Lq);
        const int co = sw8 ? 16 * cc : 8 * cc;
        float y[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        float u[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int kz = 0; kz < a.ksplit; ++kz) {
            const float* p = a.slab + ((size_t)kz * a.nphase * a.Lq + pt) * a.Co + co;
            const f32x4_t p0 = *reinterpret_cast<const f32x4_t*>(p), p1 = *reinterpret_cast<const f32x4_t*>(p + 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                y[j] += p0[j];
                y[4 + j] += p1[j];
            }
            if (half) {
                const f32x4_t q0 = *reinterpret_cast<const f32x4_t*>(p + half);
                const f32x4_t q1 = *reinterpret_cast<const f32x4_t*>(p + half + 4);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    u[j] += q0[j];
                    u[4 + j] += q1[j];
                }
            }
        }
        if (half) {  // (no bias: the FeedForward linears have none)
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float g = rnd<T>(y[j]);
                o[j] = rnd<T>(rnd<T>(g / (1.0f + expf(-g))) * rnd<T>(u[j]));
            }
            store8(reinterpret_cast<T*>(a.out) + ((size_t)t * a.stride + phase) * a.ldo + 8 * cc, o);
            continue;
        }
        float b[8];
        if (fl & CE_BIAS) load8(a.bias + co, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float v = y[j];
            if (fl & CE_BIAS) v += b[j];
            v = rnd<T>(v);
            if (fl & CE_GELU) v = rnd<T>(0.5f * v * (1.0f + erff(v * 0.70710678118654752f)));
            y[j] = v;
        }
        if ((fl & CE_ROPE) && co < a.rope_nqk) {  // the 8 channels are 4 (even, odd) pairs of one head
            const int half = a.rope_hd >> 1, p0 = (co % a.rope_hd) >> 1;
            const float* cs = a.rope + ((size_t)(t + a.rope_pos0) * half + p0) * 2;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float c = cs[2 * j], sn = cs[2 * j + 1], x0 = y[2 * j], x1 = y[2 * j + 1];
                y[2 * j] = rnd<T>(x0 * c - x1 * sn);
                y[2 * j + 1] = rnd<T>(x1 * c + x0 * sn);
            }
        }
        const size_t tout = (size_t)t * a.stride + phase;
        if (fl & CE_RES) {
            float rv[8], gm[8];
            load8(a.res + tout * a.ldr + co, rv);
            if (fl & CE_GAMMA) load8(a.gamma + co, gm);
#pragma unroll
            for (int j = 0; j < 8; ++j) y[j] = (fl & CE_GAMMA) ? rnd<T>(rv[j] + rnd<T>(gm[j] * y[j])) : rnd<T>(rv[j] + y[j]);
        }
        if (fl & CE_TANH)
#pragma unroll
            for (int j = 0; j < 8; ++j) y[j] = tanhf(y[j]);
        if (fl & CE_STORE) store8(reinterpret_cast<T*>(a.out) + tout * a.ldo + co, y);
        if (fl & CE_SNAKE) {
            float al[8], ia[8], sn[8];
            load8(a.alpha2 + co, al);
            load8(a.ialpha2 + co, ia);
#pragma unroll
            for (int j = 0; j < 8; ++j) sn[j] = rnd<T>(snake_fi(y[j], al[j], ia[j]));
            store8(a.out2 + tout * a.ldo2 + co, sn);
        }
    }
}

// The split-K epilogue of a layer whose output row feeds an RMSNorm (CE_NORM: the transformer's wo
// and w2, modded_dac.py:349-439): 256 / (Co / 8) whole rows per block, y = round(sum + bias) ->
// residual / LayerScale -> store as conv_splitk_epi_kernel, the rounded rows parked in LDS, then the
// first wave of each row sums the squares in rmsnorm_wave_kernel's order (lane l: 8-channel chunks
// l, l + 64, ... in sequence, then wave_sum) and every thread writes round(round(y * rs) * w) to
// out2 -- bit-identical to the rmsnorm launch it replaces.
template <typename T>
__global__ __launch_bounds__(256) void conv_splitk_epi_norm_kernel(ConvArgs<T> a) {
    __shared__ float zrow[256 * 8];
    __shared__ float rss[4];
    const int fl = a.flags;
    const int cpr = a.Co >> 3, rpb = 256 / cpr;  // host: Co % 512 == 0, Co <= 2048
    const int rl = threadIdx.x / cpr, cc = threadIdx.x - rl * cpr, co = 8 * cc;
    const int t = blockIdx.x * rpb + rl;
    const bool live = t < a.Lq;
    const int tt = live ? t : a.Lq - 1;
    float y[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int kz = 0; kz < a.ksplit; ++kz) {
        const float* p = a.slab + ((size_t)kz * a.Lq + tt) * a.Co + co;
        const f32x4_t p0 = *reinterpret_cast<const f32x4_t*>(p), p1 = *reinterpret_cast<const f32x4_t*>(p + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            y[j] += p0[j];
            y[4 + j] += p1[j];
        }
    }
    float b[8];
    if (fl & CE_BIAS) load8(a.bias + co, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = rnd<T>((fl & CE_BIAS) ? y[j] + b[j] : y[j]);
    if (fl & CE_RES) {
        float rv[8], gm[8];
        load8(a.res + (size_t)tt * a.ldr + co, rv);
        if (fl & CE_GAMMA) load8(a.gamma + co, gm);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = (fl & CE_GAMMA) ? rnd<T>(rv[j] + rnd<T>(gm[j] * y[j])) : rnd<T>(rv[j] + y[j]);
    }
    if ((fl & CE_STORE) && live) store8(reinterpret_cast<T*>(a.out) + (size_t)t * a.ldo + co, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) zrow[threadIdx.x * 8 + j] = y[j];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wpr = cpr >> 6;  // waves per row
    if (wv % wpr == 0) {  // the row's first wave: rmsnorm_wave_kernel's sum order
        const float* zr = zrow + (size_t)rl * a.Co;
        float ss = 0.f;
        for (int c = 0; c < wpr; ++c) {
            const float* v = zr + 8 * (c * 64 + lane);
#pragma unroll
            for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
        }
        ss = wave_sum(ss);
        if (lane == 0) rss[rl] = 1.0f / sqrtf(ss / (float)a.Co + a.norm_eps);
    }
    __syncthreads();
    if (!live) return;
    const float rs = rss[rl];
    float g[8], o[8];
    load8(a.normw + co, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = rnd<T>(rnd<T>(y[j] * rs) * g[j]);
    store8(a.out2 + (size_t)t * a.ldo2 + co, o);
}

// SwiGLU helper epilogue: out = silu(round(g)) * y   (modded_dac.py:316-317) -- done by a tiny
// elementwise kernel after the w3 GEMM to keep conv_gemm_kernel's epilogue set small.
template <typename T>
__global__ void silu_mul_kernel(const T* __restrict__ g, T* __restrict__ y, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float a = ld(g, i);
        st(y, i, rnd<T>(a / (1.0f + expf(-a))) * ld(y, i));
    }
}

// z[t][c] = (semantic out_proj(cb[code])) + (sum of residual out_proj(cb_q[code_q]))
template <typename T>
__global__ __launch_bounds__(1024) void rvq_decode_kernel(const int32_t* __restrict__ codes, int Tn, int nq1,
                                                         int sem_size, int cb_size, int cd, RvqPtrs p,
                                                         int D, T* __restrict__ z) {
    // the frame's codebook rows are staged in LDS first (codes, then rows: two round trips for the
    // block instead of two per stage per thread); sums in the reference's order
    __shared__ float erow[16][8];
    const int t = blockIdx.x;
    if (threadIdx.x < nq1 * cd) {
        const int q = threadIdx.x / cd, j = threadIdx.x - q * cd;
        int code = codes[(size_t)q * Tn + t];
        const int mx = (q == 0 ? sem_size : cb_size) - 1;
        code = code > mx ? mx : code;  // rvq.py:354-359 clamps the max only
        erow[q][j] = p.cb[q][(size_t)code * cd + j];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
        float zs = 0.f, zr = 0.f;
#pragma unroll 5
        for (int q = 0; q < nq1; ++q) {
            const float* w = p.w[q] + (size_t)c * cd;
            float acc = 0.f;
            for (int j = 0; j < cd; ++j) acc += w[j] * erow[q][j];
            acc += p.b[q][c];
            if (q == 0) zs += acc;
            else zr += acc;
        }
        st(z, (size_t)t * D + c, zs + zr);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void dwconv_ln_kernel(const T* __restrict__ x, int L, int D,
                                                        const T* __restrict__ dw, const T* __restrict__ db,
                                                        const T* __restrict__ lw, const T* __restrict__ lb,
                                                        T* __restrict__ y, int lo) {
    __shared__ float scratch[16];
    const int t = blockIdx.x;
    float v[8];
    int n = 0;
    float s = 0.f;
    for (int c = threadIdx.x; c < D; c += 256, ++n) {
        float acc = ld(db, c);
        for (int j = 0; j < 7; ++j) {
            const int src = t - 6 + j;
            if (src >= lo) acc += ld(dw, (size_t)c * 7 + j) * ld(x + (ptrdiff_t)src * D, c);
        }
        v[n] = rnd<T>(acc);
        s += v[n];
    }
    const float mu = block_sum(s, scratch) / (float)D;
    float q = 0.f;
    for (int i = 0; i < n; ++i) q += (v[i] - mu) * (v[i] - mu);
    const float var = block_sum(q, scratch) / (float)D;
    const float rs = 1.0f / sqrtf(var + 1e-6f);
    n = 0;
    for (int c = threadIdx.x; c < D; c += 256, ++n)
        st(y, (size_t)t * D + c, (v[n] - mu) * rs * ld(lw, c) + ld(lb, c));
}

template <typename T>
__global__ void rope_qk_kernel(T* __restrict__ qkv, int Tn, int H, int hd, const float* __restrict__ tab,
                               int pos0) {
    const int t = blockIdx.x, tp = t + pos0;
    const int half = hd >> 1;
    for (int idx = threadIdx.x; idx < 2 * H * half; idx += blockDim.x) {
        const int head = idx / half, p = idx - head * half;
        T* v = qkv + (size_t)t * 3 * H * hd + (size_t)head * hd;
        const float x0 = ld(v, 2 * p), x1 = ld(v, 2 * p + 1);
        const float c = tab[((size_t)tp * half + p) * 2], s = tab[((size_t)tp * half + p) * 2 + 1];
        const float y0 = x0 * c - x1 * s;
        const float y1 = x1 * c + x0 * s;
        st(v, 2 * p, y0);
        st(v, 2 * p + 1, y1);
    }
}

// grid (T, H), one wave; window <= 128, hd <= 64
// NS scores per lane: window <= 64 * NS (decode post_module: 128; encoder block: 512)
template <typename T, int NS>
__global__ __launch_bounds__(64) void window_attn_kernel(const T* __restrict__ qkv, int Tn, int H, int hd,
                                                         int window, T* __restrict__ out, int npre) {
    __shared__ float qs[64];
    __shared__ float ps[64 * NS];
    const int lane = threadIdx.x;
    const int t = blockIdx.x, h = blockIdx.y;
    const size_t ld3 = (size_t)3 * H * hd;
    const T* q = qkv + (size_t)t * ld3 + (size_t)h * hd;
    if (lane < hd) qs[lane] = ld(q, lane);
    __syncthreads();
    int j0 = t - window + 1;  // rows [-npre, 0): carried keys / values of the previous chunk
    if (j0 < -npre) j0 = -npre;
    const int nj = t - j0 + 1;
    const float scale = 1.0f / sqrtf((float)hd);
    float sc[NS];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        sc[i] = -INFINITY;
        const int jj = lane + 64 * i;
        if (jj < nj) {
            const T* k = qkv + (ptrdiff_t)(j0 + jj) * (ptrdiff_t)ld3 + (size_t)(H + h) * hd;
            float dot = 0.f;
            for (int e = 0; e < hd; e += 8) {
                float kv[8];
                load8(k + e, kv);
#pragma unroll
                for (int u = 0; u < 8; ++u) dot += qs[e + u] * kv[u];
            }
            sc[i] = dot * scale;
        }
        mx = fmaxf(mx, sc[i]);
    }
    const float m = wave_max(mx);
    float psum = 0.f;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const float p = lane + 64 * i < nj ? expf(sc[i] - m) : 0.f;
        ps[lane + 64 * i] = p;
        psum += p;
    }
    const float l = wave_sum(psum);
    __syncthreads();
    if (lane < hd) {
        float o = 0.f;
        for (int jj = 0; jj < nj; ++jj)
            o += ps[jj] * ld(qkv + (ptrdiff_t)(j0 + jj) * (ptrdiff_t)ld3 + (size_t)(2 * H + h) * hd, lane);
        st(out, (size_t)t * H * hd + (size_t)h * hd + lane, o / l);
    }
}

// mono fp32 samples -> the encoder's [n_pad][8] input (channel 0 live, right pad = causal zeros of
// DAC.encode's pad to a multiple of frame_length, modded_dac.py:906-909)
template <typename T>
__global__ void audio8_kernel(const float* __restrict__ a, int64_t n, int64_t npad, T* __restrict__ y) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npad * 8; i += (int64_t)gridDim.x * blockDim.x)
        st(y, (size_t)i, (i & 7) == 0 && (i >> 3) < n ? a[i >> 3] : 0.f);
}

// Snake1d (descript, restated in oracle/ref_stubs.py) on a time-major [L][C] activation
template <typename T>
__global__ void snake_kernel(const T* __restrict__ x, int C, size_t n, const T* __restrict__ alpha, T* __restrict__ y) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        st(y, i, snake_f(ld(x, i), ld(alpha, (int)(i % C))));
}

// Residual VQ encode (descript 1.0.0 VectorQuantize.forward / decode_latents, eval; rvq.py:
// 303-315 chains the semantic stage then the residual stages on z - semantic_z), fp32.  One
// block per frame t; r (time-major [Tn][D], T) is the running residual, updated in place.
// Stage q: z_e = in_proj(r) (cd outputs); nearest l2-normalised codebook row to the
// l2-normalised z_e (argmax of -(|e|^2 - 2 e.c + |c|^2), lowest index on ties); z_q = z_e +
// (codebook[idx] - z_e); r -= out_proj(z_q).
__global__ __launch_bounds__(256) void vq_encode_kernel_f(float* __restrict__ rf, int Tn, int D, int nst, int cd,
                                                          VqEncPtrs p, int32_t* __restrict__ codes) {
    __shared__ float zs[16], en[16], zq[16];
    __shared__ float bv[256];
    __shared__ int bi[256];
    const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float* r = rf + (size_t)t * D;
    for (int q = 0; q < nst; ++q) {
        for (int j = wave; j < cd; j += 4) {
            const float* w = p.wi[q] + (size_t)j * D;
            float acc = 0.f;
            for (int d = lane; d < D; d += 64) acc += w[d] * r[d];
            acc = wave_sum(acc);
            if (lane == 0) zs[j] = acc + p.bi[q][j];
        }
        __syncthreads();
        if (tid == 0) {
            float ss = 0.f;
            for (int j = 0; j < cd; ++j) ss += zs[j] * zs[j];
            const float nrm = fmaxf(sqrtf(ss), 1e-12f);
            for (int j = 0; j < cd; ++j) en[j] = zs[j] / nrm;
        }
        __syncthreads();
        float e2 = 0.f;
        for (int j = 0; j < cd; ++j) e2 += en[j] * en[j];
        float best = -INFINITY;
        int bidx = 0x7fffffff;
        const float* cb = p.cb[q];
        for (int i = tid; i < p.cbn[q]; i += 256) {
            float ss = 0.f;
            for (int j = 0; j < cd; ++j) ss += cb[(size_t)i * cd + j] * cb[(size_t)i * cd + j];
            const float nrm = fmaxf(sqrtf(ss), 1e-12f);
            float dot = 0.f, c2 = 0.f;
            for (int j = 0; j < cd; ++j) {
                const float cn = cb[(size_t)i * cd + j] / nrm;
                dot += en[j] * cn;
                c2 += cn * cn;
            }
            const float nd = -((e2 - 2.f * dot) + c2);
            if (nd > best) {  // i ascends per thread: strict > keeps the lowest index
                best = nd;
                bidx = i;
            }
        }
        bv[tid] = best;
        bi[tid] = bidx;
        __syncthreads();
        for (int off = 128; off > 0; off >>= 1) {
            if (tid < off) {
                const float ov = bv[tid + off];
                const int oi = bi[tid + off];
                if (ov > bv[tid] || (ov == bv[tid] && oi < bi[tid])) {
                    bv[tid] = ov;
                    bi[tid] = oi;
                }
            }
            __syncthreads();
        }
        const int idx = bi[0];
        if (tid < cd) zq[tid] = zs[tid] + (cb[(size_t)idx * cd + tid] - zs[tid]);
        if (tid == 0) codes[(size_t)q * Tn + t] = idx;
        __syncthreads();
        for (int d = tid; d < D; d += 256) {
            const float* w = p.wo[q] + (size_t)d * cd;
            float acc = 0.f;
            for (int j = 0; j < cd; ++j) acc += w[j] * zq[j];
            r[d] -= acc + p.bo[q][d];
        }
        __syncthreads();
    }
}

// weight norm (torch _weight_norm, dim=0): w = v * (g / ||v||) per leading index
__global__ __launch_bounds__(256) void wn_fold_kernel(const float* __restrict__ g, const float* __restrict__ v,
                                                      int per, float* __restrict__ w) {
    __shared__ float scratch[16];
    const int row = blockIdx.x;
    const float* vr = v + (size_t)row * per;
    float ss = 0.f;
    for (int i = threadIdx.x; i < per; i += 256) ss += vr[i] * vr[i];
    ss = block_sum(ss, scratch);
    const float f = g[row] / sqrtf(ss);
    for (int i = threadIdx.x; i < per; i += 256) w[(size_t)row * per + i] = vr[i] * f;
}

// fp32 conv weights -> row-major [phase][co][tap*Ci + ci] in T.
// kind 0: Conv1d [Co][Ci][k], tap j (shift (k-1-j)*dil set by the host)
// kind 1: ConvTranspose1d [Ci][Co][2s]: phase p, tap0 = W[.][.][p] (x[t]), tap1 = W[.][.][p+s] (x[t-1])
// kind 2: ConvTranspose1d [Ci][Co][s]: phase p, one tap W[.][.][p]
// kind 3: Linear [Co][Ci]
template <typename T>
__global__ void conv_weight_kernel(const float* __restrict__ w, int kind, int Ci, int Co, int k, int s,
                                   T* __restrict__ out) {
    const int ntaps = kind == 0 ? k : (kind == 1 ? 2 : 1);
    const int nph = kind == 0 || kind == 3 ? 1 : s;
    const int64_t Kt = (int64_t)ntaps * Ci;
    const int64_t Kp = (Kt + 31) / 32 * 32;  // zero-padded row length
    const int64_t n = (int64_t)nph * Co * Kp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t ph = i / (Co * Kp);
        const int64_t rem = i - ph * Co * Kp;
        const int co = (int)(rem / Kp);
        const int kk = (int)(rem - (int64_t)co * Kp);
        if (kk >= Kt) {
            st(out, i, 0.f);
            continue;
        }
        const int tap = kk / Ci, ci = kk - tap * Ci;
        float v;
        if (kind == 0) v = w[((size_t)co * Ci + ci) * k + tap];
        else if (kind == 1) v = w[((size_t)ci * Co + co) * (2 * s) + ph + tap * s];
        else if (kind == 2) v = w[((size_t)ci * Co + co) * s + ph];
        else v = w[(size_t)co * Ci + ci];
        st(out, i, v);
    }
}

// ---------------------------------------------------------------------------------------
// conv_gemm2_kernel: the same implicit GEMM (and epilogues) as conv_gemm_kernel with both operands
// staged through LDS.  Block = 4 waves, tile 128 output times x 16*NCO channels; wave w owns times
// [32w, 32w + 32) (two MFMA column tiles) against all NCO channel tiles, so per 32-wide k-step a
// block reads its X rows (8 KB, one 16-B chunk of one row per thread per half) and the NCO packed
// weight fragments once from L2 instead of once per wave.  Double-buffered: the next k-step's
// global loads are in flight while the MFMAs of the current one read LDS; one barrier per step.
// X rows are padded to 40 elements in LDS (80 B for bf16): the B-fragment reads of a wave (16 rows
// x 16 B) spread over all banks.
// Three-stage pipeline: the global loads of k-step s+2 go out before the MFMAs of step s (two
// register staging sets, used alternately), step s+1's set is written to the other LDS buffer after
// them, one barrier per step -- an L2 round trip is hidden behind two steps of MFMAs instead of
// one.  Every staging load is unconditional (clamped step / tile indices): a load under a branch
// makes the compiler drain vmcnt(0), which would serialise the stages again.
// (Measured and dropped: 256-row tiles, 4 row fragments per wave at 2 waves per SIMD, 20-25 % slower
// on every decoder shape; LDS-DMA (global_load_lds) staging of 64-deep k stages, 2 blocks per CU,
// 7-18 % slower on three of the four decoder shapes.  Occupancy, not LDS or L2 bandwidth, decides.)
// Shared epilogue of the LDS-tiled conv GEMMs (128 output times x 16*NCO channels, wave w owning
// times [32w, 32w + 32)), run after the k-loop's last barrier.  Phase 1: each wave parks its
// accumulator tile as T (bias, first rounding, GELU applied) in LDS -- a wave reads back only its own
// rows.  Phase 2: 16-B chunks of 8 consecutive channels of one row per lane: residual / LayerScale,
// tanh, the store and the next stage's Snake with 16-B accesses.
template <typename T, int NCO>
__device__ __forceinline__ void cg_epilogue(const ConvArgs<T>& a, const f32x4_t (&acc)[NCO][2], T* et, int t0,
                                            int co0, int phase, int nct, int wave, int lane) {
    const int fl = a.flags;
    constexpr int EW = 16 * NCO + 8;  // LDS row stride (elements)
    float bsv[NCO][4];
    {
        const T* bp = (fl & CE_BIAS) ? a.bias : a.w;
#pragma unroll
        for (int c = 0; c < NCO; ++c)
#pragma unroll
            for (int i = 0; i < 4; ++i) bsv[c][i] = ld(bp, min(co0 + 16 * c + 4 * (lane >> 4) + i, a.Co - 1));
    }
#pragma unroll
    for (int c = 0; c < NCO; ++c) {
        if (c >= nct) break;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int tl = 32 * wave + 16 * u + (lane & 15), cl = 16 * c + 4 * (lane >> 4);
            float y4[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float y = acc[c][u][i];
                if (fl & CE_BIAS) y += bsv[c][i];
                y = rnd<T>(y);
                if (fl & CE_GELU) y = rnd<T>(0.5f * y * (1.0f + erff(y * 0.70710678118654752f)));
                y4[i] = y;
            }
            if constexpr (is_bf16<T>::value) {  // 4 consecutive channels: one 8-byte LDS store
                uint32_t w0 = (__float_as_uint(y4[0]) >> 16) | (__float_as_uint(y4[1]) & 0xffff0000u);
                uint32_t w1 = (__float_as_uint(y4[2]) >> 16) | (__float_as_uint(y4[3]) & 0xffff0000u);
                *reinterpret_cast<uint2*>(et + (size_t)tl * EW + cl) = make_uint2(w0, w1);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) st(et, (size_t)tl * EW + cl + i, y4[i]);
            }
        }
    }
    constexpr int CPR = 2 * NCO;  // chunks of 8 channels per row
    for (int q = lane; q < 32 * CPR; q += 64) {
        const int tl = 32 * wave + q / CPR, cc = q - (q / CPR) * CPR;
        const int t = t0 + tl;
        if (t >= a.Lq || cc >= 2 * nct) continue;
        const int co = co0 + 8 * cc;
        const size_t tout = (size_t)t * a.stride + phase;
        float y[8];
        load8(et + (size_t)tl * EW + 8 * cc, y);
        if (fl & CE_RES) {
            float rv[8], gm[8];
            load8(a.res + tout * a.ldr + co, rv);
            if (fl & CE_GAMMA) load8(a.gamma + co, gm);
#pragma unroll
            for (int j = 0; j < 8; ++j) y[j] = (fl & CE_GAMMA) ? rnd<T>(rv[j] + rnd<T>(gm[j] * y[j])) : rnd<T>(rv[j] + y[j]);
        }
        if (fl & CE_TANH)
#pragma unroll
            for (int j = 0; j < 8; ++j) y[j] = tanhf(y[j]);
        if (fl & CE_STORE) store8(reinterpret_cast<T*>(a.out) + tout * a.ldo + co, y);
        if (fl & CE_SNAKE) {
            float al[8], ia[8], sn[8];
            load8(a.alpha2 + co, al);
            load8(a.ialpha2 + co, ia);
#pragma unroll
            for (int j = 0; j < 8; ++j) sn[j] = rnd<T>(snake_fi(y[j], al[j], ia[j]));
            store8(a.out2 + tout * a.ldo2 + co, sn);
        }
    }
}

constexpr int CG2_BM = 128, CG2_XS = 40;
// waves per SIMD the register budget targets: the second staging set costs 8 * (XCH + WCH) VGPRs
constexpr int cg2_wpe(int esz, int nco) { return esz == 4 ? 2 : (nco == 8 ? 3 : 4); }
template <typename T, int NCO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(cg2_wpe(sizeof(T), NCO)))) void conv_gemm2_kernel(ConvArgs<T> a) {
    using F = Frag<T>;
    constexpr int XBUF = CG2_BM * CG2_XS, WBUF = NCO * 512;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_cg[];
    T* lds = reinterpret_cast<T*>(smem_cg);  // [2][XBUF + WBUF]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int t0 = blockIdx.x * CG2_BM;
    const int co0 = blockIdx.y * 16 * NCO;
    // grid z = phase + nphase * k-slice (ksplit > 1: fp32 partial slabs, conv_splitk_epi_kernel runs
    // the epilogue); this block's k-steps are [sb, sb + NS)
    const int ks = a.ksplit > 1 ? a.ksplit : 1;
    const int phase = blockIdx.z % a.nphase, kz = blockIdx.z / a.nphase;
    const int Kt = a.ntaps * a.Ci, S = (Kt + 31) >> 5;
    const int sb = (int)((long long)S * kz / ks), NS = (int)((long long)S * (kz + 1) / ks) - sb;
    const T* wb = a.w + (size_t)phase * a.wphase + (size_t)(co0 >> 4) * S * 512;
    const int nct = min(NCO, (a.Co - co0 + 15) >> 4);  // channel tiles present in this block
    constexpr int EC = 16 / (int)sizeof(T);             // elements per 16-B chunk
    constexpr int XCH = CG2_BM * 32 / EC / 256;          // X chunks per thread per step (2 bf16, 4 fp32)
    constexpr int WCH_T = NCO * 512 / EC;                // W chunks per step
    constexpr int WCH = (WCH_T + 255) / 256;
    using XR = u32x4_t[XCH];
    using WR = u32x4_t[WCH];
    using XM = uint32_t[XCH];
    // raw X chunks and their validity masks: the mask is applied when the chunk is written to LDS,
    // so no ALU op consumes a load before the step that stores it (that would drain vmcnt early)
    u32x4_t xr0[XCH], wr0[WCH], xr1[XCH], wr1[WCH];
    uint32_t xm0[XCH], xm1[XCH];
    auto gload = [&](int s, XR& xr, XM& xm, WR& wr) {
        s = sb + (s < NS ? s : NS - 1);
        // the step's first tap once per wave (uniform), then at most one boundary inside the
        // 32-wide step (host: Ci >= 32) -- no per-lane integer division
        const int kb = s * 32, tap0 = kb / a.Ci, ci0 = kb - tap0 * a.Ci;
#pragma unroll
        for (int j = 0; j < XCH; ++j) {
            const int c = tid + 256 * j;
            const int row = c / (32 / EC), kc = c - row * (32 / EC);
            int ci = ci0 + kc * EC, tap = tap0;
            if (ci >= a.Ci) {
                ci -= a.Ci;
                ++tap;
            }
            const bool kin = tap < a.ntaps;
            tap = kin ? tap : a.ntaps - 1;
            const int t = t0 + row, tin = t - conv_shift(a, tap);
            const bool ok = kin && t < a.Lq && tin >= a.lo && tin < a.Lx;
            const int rc = tin < a.lo ? a.lo : (tin >= a.Lx ? a.Lx - 1 : tin);
            xr[j] = *reinterpret_cast<const u32x4_t*>(a.x + (ptrdiff_t)rc * a.ldx + (ok ? ci : 0));
            xm[j] = ok ? 0xffffffffu : 0u;
        }
#pragma unroll
        for (int j = 0; j < WCH; ++j) {
            // tiles past nct are never read by the MFMA loop: clamped re-reads, no branch
            int c = tid + 256 * j;
            c = c < WCH_T ? c : WCH_T - 1;
            int ct = c / (512 / EC);
            const int e = c - ct * (512 / EC);
            ct = ct < nct ? ct : nct - 1;
            wr[j] = *reinterpret_cast<const u32x4_t*>(wb + ((size_t)ct * S + s) * 512 + e * EC);
        }
    };
    auto sstore = [&](int buf, const XR& xr, const XM& xm, const WR& wr) {
        T* xs = lds + (size_t)buf * (XBUF + WBUF);
        T* ws = xs + XBUF;
#pragma unroll
        for (int j = 0; j < XCH; ++j) {
            const int c = tid + 256 * j;
            const int row = c / (32 / EC), kc = c - row * (32 / EC);
            const uint32_t m = xm[j];
            *reinterpret_cast<u32x4_t*>(xs + row * CG2_XS + kc * EC) = (u32x4_t){xr[j][0] & m, xr[j][1] & m, xr[j][2] & m, xr[j][3] & m};
        }
#pragma unroll
        for (int j = 0; j < WCH; ++j) {
            const int c = tid + 256 * j;
            if (c < WCH_T) *reinterpret_cast<u32x4_t*>(ws + (size_t)c * EC) = wr[j];
        }
    };
    f32x4_t acc[NCO][2];
#pragma unroll
    for (int c = 0; c < NCO; ++c) acc[c][0] = acc[c][1] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int xrow0 = 32 * wave + (lane & 15), xk = 8 * (lane >> 4);
    auto mma_step = [&](int buf) {
        const T* xs = lds + (size_t)buf * (XBUF + WBUF);
        const T* ws = xs + XBUF;
        const typename F::f xb0 = F::load(xs + xrow0 * CG2_XS + xk);
        const typename F::f xb1 = F::load(xs + (xrow0 + 16) * CG2_XS + xk);
#pragma unroll
        for (int c = 0; c < NCO; ++c) {
            if (c < nct) {
                const typename F::f wf = F::load_w(ws + c * 512, lane);
                acc[c][0] = F::mma(wf, xb0, acc[c][0]);
                acc[c][1] = F::mma(wf, xb1, acc[c][1]);
            }
        }
    };
    // step s: loads of s+2 into `nx`, MFMAs on LDS buffer s&1, step s+1 (held in `cur`) -> LDS
    auto step = [&](int s, XR& nx, XM& nm, WR& nw, const XR& cur, const XM& cm, const WR& cw) {
        gload(s + 2, nx, nm, nw);
        mma_step(s & 1);
        if (s + 1 < NS) sstore((s + 1) & 1, cur, cm, cw);
        __syncthreads();
    };
    gload(0, xr0, xm0, wr0);
    gload(1, xr1, xm1, wr1);
    sstore(0, xr0, xm0, wr0);
    __syncthreads();
    for (int s = 0; s < NS; s += 4) {  // 4 steps per trip: the loop-header vmcnt drain every 4 steps
        step(s, xr0, xm0, wr0, xr1, xm1, wr1);
        if (s + 1 < NS) step(s + 1, xr1, xm1, wr1, xr0, xm0, wr0);
        if (s + 2 < NS) step(s + 2, xr0, xm0, wr0, xr1, xm1, wr1);
        if (s + 3 < NS) step(s + 3, xr1, xm1, wr1, xr0, xm0, wr0);
    }
    if (ks > 1) {  // raw fp32 partials [kz][phase][Lq][Co]: 4 consecutive channels per lane
#pragma unroll
        for (int c = 0; c < NCO; ++c) {
            if (c >= nct) break;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int t = t0 + 32 * wave + 16 * u + (lane & 15);
                if (t >= a.Lq) continue;
                float* dst = a.slab + ((size_t)(kz * a.nphase + phase) * a.Lq + t) * a.Co + co0 + 16 * c + 4 * (lane >> 4);
                *reinterpret_cast<f32x4_t*>(dst) = acc[c][u];
            }
        }
        return;
    }
    cg_epilogue<T, NCO>(a, acc, lds, t0, co0, phase, nct, wave, lane);
}

template <typename T, int NCO> static void conv2_go(hipStream_t s, const ConvArgs<T>& a) {
    const size_t lds = std::max(2 * ((size_t)CG2_BM * CG2_XS + NCO * 512), (size_t)CG2_BM * (16 * NCO + 8)) * sizeof(T);
    dim3 g(FM_CEIL(a.Lq, CG2_BM), FM_CEIL(a.Co, 16 * NCO), a.nphase * (a.ksplit > 1 ? a.ksplit : 1));
    conv_gemm2_kernel<T, NCO><<<g, 256, lds, s>>>(a);
}



// A split-K layer (PackedW::ks > 1): K slices into fp32 slabs, then conv_splitk_epi_kernel; rows in
// segments that fit the workspace (pointers offset, the carried-context bound lo moved with them)
template <typename T> static void conv_splitk_go(hipStream_t s, const ConvArgs<T>& a) {
    const size_t per_row = (size_t)a.ksplit * a.nphase * a.Co;
    const int seg = (int)std::min<size_t>((size_t)a.Lq, a.slab_cap / per_row / 64 * 64);
    FMCHECK(seg >= 64 || seg == a.Lq, "conv split-K: workspace too small");
    for (int r0 = 0; r0 < a.Lq; r0 += seg) {
        ConvArgs<T> b = a;
        b.Lq = std::min(seg, a.Lq - r0);
        b.x = a.x + (ptrdiff_t)r0 * a.ldx;
        b.Lx = a.Lx - r0;
        b.lo = a.lo - r0;
        b.rope_pos0 = a.rope_pos0 + r0;  // (CE_ROPE: row r0 of the segment is position r0)
        const size_t o = (size_t)r0 * a.stride;
        if (a.out) b.out = (char*)a.out + o * a.ldo * sizeof(T);
        if (a.res) b.res = a.res + o * a.ldr;
        if (a.out2) b.out2 = a.out2 + o * a.ldo2;
        const long long t128 = (long long)FM_CEIL(b.Lq, CG2_BM) * FM_CEIL(b.Co, 128) * b.nphase * b.ksplit;
        if (fm_tuning().conv2 && b.Ci % 8 == 0 && b.Ci >= 32 && b.Co % 16 == 0 && b.Co >= 96 && t128 >= 256) {
            if (b.Co % 128 == 0 || b.Co >= 384)
                conv2_go<T, 8>(s, b);
            else
                conv2_go<T, 6>(s, b);
        } else {
            dim3 g(FM_CEIL(b.Lq, 64), FM_CEIL(b.Co, 64), b.nphase * b.ksplit);
            conv_gemm_kernel<T><<<g, 256, 0, s>>>(b);
        }
        if (b.flags & CE_NORM) {
            FMCHECK(b.nphase == 1 && b.Co % 512 == 0 && b.Co <= 2048 && b.normw && b.out2,
                    "conv: the norm epilogue needs one phase, Co a multiple of 512 up to 2048, weight and out2");
            const int rpb = 256 / (b.Co / 8);
            conv_splitk_epi_norm_kernel<T><<<FM_CEIL(b.Lq, rpb), 256, 0, s>>>(b);
            continue;
        }
        const size_t n = (size_t)b.nphase * b.Lq * (((b.flags & CE_SWIGLU) ? b.Co / 2 : b.Co) / 8);
        conv_splitk_epi_kernel<T><<<(int)std::min<size_t>(FM_CEIL(n, 256), 4096), 256, 0, s>>>(b);
    }
}

template <typename T> void launch_conv_epi(hipStream_t s, const ConvArgs<T>& b) {
    FMCHECK(b.ksplit >= 1 && b.slab && !(b.flags & CE_NORM) && b.Co % 8 == 0, "conv epilogue: slabs, Co % 8, no norm");
    FMCHECK(!(b.flags & CE_SWIGLU8) || (b.Co % 16 == 0 && !(b.flags & (CE_SWIGLU | CE_BIAS))),
            "conv epilogue: the interleaved SwiGLU needs Co % 16 == 0, no bias");
    const size_t n = (size_t)b.nphase * b.Lq *
                     ((b.flags & CE_SWIGLU8) ? b.Co / 16 : (((b.flags & CE_SWIGLU) ? b.Co / 2 : b.Co) / 8));
    conv_splitk_epi_kernel<T><<<(int)std::min<size_t>(FM_CEIL(n, 256), 4096), 256, 0, s>>>(b);
}

template <typename T> void launch_conv_gemm(hipStream_t s, const ConvArgs<T>& a0) {
    ConvArgs<T> a = a0;
    a.shift0 = a.shift[0];
    a.shiftd = a.ntaps > 1 ? a.shift[1] - a.shift[0] : 0;
    for (int j = 0; j < a.ntaps; ++j) FMCHECK(a.shift[j] == a.shift0 + j * a.shiftd, "conv: tap shifts must be linear in the tap");
    // LDS-staged tiles where the channels fill them (every decoder / transformer / upsample GEMM);
    // the few narrow ones (encoder stem, 1-channel output conv) keep the register-only kernel
    // (measured per shape, 10 s decode: 442k x 96 k7 282 vs 292 us, 221k x 192 371 vs 452, 55k x 384
    // 348 vs 370, 6.9k x 768 192 vs 202; at 216-864 rows the LDS tile leaves too few blocks and loses)
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const bool vec_ok = !(a.flags & CE_F32OUT) && al16(a.out) && al16(a.out2) && al16(a.res) && a.ldo % 8 == 0 &&
                        a.ldo2 % 8 == 0 && a.ldr % 8 == 0;  // the coalesced epilogue's 16-B accesses
    if (a.ksplit > 1 && a.slab && vec_ok && a.Co % 8 == 0) {
        conv_splitk_go<T>(s, a);
        return;
    }
    FMCHECK(!(a.flags & (CE_SWIGLU | CE_ROPE | CE_NORM)), "conv: the SwiGLU / RoPE / norm epilogues run on the split-K path only");
    // LDS tiles once they give the chip >= 256 blocks (the 128-row tile, 96-128 channels)
    const long long cg2_blocks = (long long)FM_CEIL(a.Lq, CG2_BM) * FM_CEIL(a.Co, 128) * a.nphase;
    if (fm_tuning().conv2 && vec_ok && a.Ci % 8 == 0 && a.Ci >= 32 && a.Co % 16 == 0 && a.Co >= 96 &&
        (a.Lq >= 4096 || cg2_blocks >= 256)) {
        ConvArgs<T> b = a;
        b.ksplit = 1;
        if (b.Co % 128 == 0 || b.Co >= 384)
            conv2_go<T, 8>(s, b);
        else
            conv2_go<T, 6>(s, b);
        return;
    }
    ConvArgs<T> b = a;
    b.ksplit = 1;
    dim3 g(FM_CEIL(a.Lq, 64), FM_CEIL(a.Co, 64), a.nphase);
    conv_gemm_kernel<T><<<g, 256, 0, s>>>(b);
}

// ---------------------------------------------------------------------------------------
// resunit_kernel: one ResidualUnit (ResUnitArgs, fm_codec.h; decoder and encoder) per launch.
// Block tile: BM output times x all C channels; wave (wt, wc) owns times [16 TT wt, +16 TT) x
// channels [16 CT wc, +16 CT), TT x CT MFMA tiles, so a k-step costs a wave TT X fragments from LDS
// and CT weight fragments from L2 (the k7 weights, 7 C^2 x 2 B, stay L2-resident up to C = 512).
//  1. the input window (rows t0 - 6 dil .. t0 + BM) lands in LDS once by LDS-DMA (16-B slots of a
//     padded row, out-of-range rows from a zero block): every tap reads it at a row offset, so X
//     costs HBM its bytes once instead of once per tap and channel tile;
//  2. k7: k-steps in conv_gemm2_kernel's order (tap-major, 32 channels each), the weights through a
//     three-step register ring;
//  3. h = round(snake(round(acc + b7))) overwrites the window in LDS (bf16 [BM][C + 8]);
//  4. k1 over h, weights again from L2;
//  5. round(acc + b1) parked in LDS, then 16-B chunks: + residual, store, next Snake.
// The variants (RU_VARIANTS) keep LDS and registers at 2-3 blocks per CU, so one block's window
// DMA runs under another's MFMAs (the 384 / 512-channel tiles: one 8-wave block per CU).
namespace {
__device__ __forceinline__ uint32_t ru_lds_off(const void* p) {
    return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p;
}
// one 16-B slot per lane by LDS-DMA: lane l's 16 bytes at gsrc -> LDS lds_base + 16 l (M0 saved
// and restored in the statement; the DMA is invisible to hipcc's waitcnt bookkeeping, so the wait
// for it is an explicit s_waitcnt vmcnt)
__device__ __forceinline__ void ru_glds16(const void* gsrc, uint32_t lds_base) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_base)
        : "memory");
}
constexpr int RU_MAXDIL = 9;
template <int C, int BM, int TT, int CT> constexpr int ru_nw() { return (BM / (16 * TT)) * (C / (16 * CT)); }
template <int C, int BM> constexpr size_t ru_lds() {
    constexpr size_t slots = (size_t)(BM + 6 * RU_MAXDIL) * ((C + 8) / 8);
    constexpr size_t win = (slots + 63) / 64 * 1024;  // whole 64-slot DMA instructions
    constexpr size_t h = (size_t)BM * (C + 8) * 2;
    return win > h ? win : h;
}
}  // namespace

template <int C, int BM, int TT, int WPE, int CT>
__global__ __launch_bounds__((ru_nw<C, BM, TT, CT>() * 64)) __attribute__((amdgpu_waves_per_eu(WPE))) void resunit_kernel(
    ResUnitArgs a) {
    using F = Frag<bf16_t>;
    constexpr int NW = ru_nw<C, BM, TT, CT>(), NT = NW * 64, WCN = C / (16 * CT);
    constexpr int XS = C + 8;     // LDS row stride (elements): 16-B reads of 16 rows spread over the banks
    constexpr int SPR = XS / 8;   // 16-B slots per LDS row (C / 8 data + 1 pad)
    constexpr int SK = C / 32;    // k-steps per tap
    constexpr int S7 = 7 * SK, S1 = SK;
    static_assert(C % (16 * CT) == 0 && C % 32 == 0 && BM % (16 * TT) == 0, "resunit tiling");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_ru[];
    bf16_t* xw = reinterpret_cast<bf16_t*>(smem_ru);
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int wt = wave / WCN, wc = wave - wt * WCN;
    const int t0 = blockIdx.x * BM;
    const int hal = 6 * a.dil, nslot = (BM + hal) * SPR;

    // 1. window -> LDS (wave-uniform instruction bases; lanes past the window write the tail of the
    //    last 1 KiB, which ru_lds reserves)
    {
        const uint32_t x0 = __builtin_amdgcn_readfirstlane(ru_lds_off(xw));
        for (int i0 = wave * 64; i0 < nslot; i0 += NT) {
            const int i = i0 + lane;
            const int r = i / SPR, c = i - r * SPR;
            const int tin = t0 - hal + r;
            const bool ok = i < nslot && c < C / 8 && tin >= a.lo && tin < a.L;
            ru_glds16(ok ? (const void*)(a.x + (ptrdiff_t)tin * C + 8 * c) : (const void*)a.zeros,
                      __builtin_amdgcn_readfirstlane(x0 + 16u * i0));
        }
    }
    // weight ring: fragments (channel tile 3 wc + ct, k-step s), 3 k-steps deep
    const bf16_t* w7 = a.w7 + (size_t)(CT * wc) * S7 * 512;
    const bf16_t* w1 = a.w1 + (size_t)(CT * wc) * S1 * 512;
    u32x4_t wr0[CT], wr1[CT], wr2[CT];
    auto wload = [&](u32x4_t (&w)[CT], const bf16_t* base, int S, int s) {
        s = s < S ? s : S - 1;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) w[ct] = F::load_w(base + ((size_t)ct * S + s) * 512, lane);
    };
    wload(wr0, w7, S7, 0);
    wload(wr1, w7, S7, 1);
    wload(wr2, w7, S7, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    f32x4_t acc[TT][CT];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[tt][ct] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int xr = 16 * TT * wt + (lane & 15), xk = 8 * (lane >> 4);
    // one k-step: 8 X fragments (rows xr + 16 tt + row offset) x the ring's 3 weight fragments
    auto mma8 = [&](const bf16_t* xb, const u32x4_t (&w)[CT]) {
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
            const F::f xf = F::load(xb + (size_t)16 * tt * XS);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) acc[tt][ct] = F::mma(w[ct], xf, acc[tt][ct]);
        }
    };
    // 2. k7: k-step s = tap j, channels [32 q, 32 q + 32); tap j reads input row t - (6 - j) dil =
    //    window row (t - t0) + j dil
    auto step7 = [&](int s, const u32x4_t (&w)[CT]) {
        const int j = s / SK, q = s - j * SK;
        mma8(xw + (size_t)(xr + j * a.dil) * XS + 32 * q + xk, w);
    };
    // (sched_barrier: each refill stays right behind the step that freed its slot; left to itself
    // the compiler sinks all three to the end of the trip and the ring's lookahead is gone)
    // (a trip count that is not a multiple of 3 ends in a guarded partial trip; the guards fold
    // away when it is)
    for (int s = 0; s < S7; s += 3) {
        step7(s, wr0);
        wload(wr0, w7, S7, s + 3);
        __builtin_amdgcn_sched_barrier(0);
        if (S7 % 3 == 0 || s + 1 < S7) {
            step7(s + 1, wr1);
            wload(wr1, w7, S7, s + 4);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (S7 % 3 == 0 || s + 2 < S7) {
            step7(s + 2, wr2);
            wload(wr2, w7, S7, s + 5);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    // the k1 ring goes out before the epilogue (its loads overlap it)
    wload(wr0, w1, S1, 0);
    wload(wr1, w1, S1, 1);
    wload(wr2, w1, S1, 2);
    // 3. h = round(snake_a2(round(acc + b7))) -> LDS over the window (every wave is past its reads)
    const int cl = 16 * CT * wc + 4 * (lane >> 4);  // + 16 ct + i: the lane's accumulator channels
    auto park = [&](const bf16_t* bias, const bf16_t* al, const float* ia) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            float bv[4], av[4], iv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int co = cl + 16 * ct + i;
                bv[i] = bf2f(bias[co]);
                av[i] = al ? bf2f(al[co]) : 0.f;
                iv[i] = al ? ia[co] : 0.f;
            }
#pragma unroll
            for (int tt = 0; tt < TT; ++tt) {
                float y[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    y[i] = bfround(acc[tt][ct][i] + bv[i]);
                    if (al) y[i] = bfround(snake_fi(y[i], av[i], iv[i]));
                }
                const uint32_t w0 = (__float_as_uint(y[0]) >> 16) | (__float_as_uint(y[1]) & 0xffff0000u);
                const uint32_t w1v = (__float_as_uint(y[2]) >> 16) | (__float_as_uint(y[3]) & 0xffff0000u);
                *reinterpret_cast<uint2*>(xw + (size_t)(xr + 16 * tt) * XS + cl + 16 * ct) = make_uint2(w0, w1v);
            }
        }
    };
    __syncthreads();
    park(a.b7, a.a2, a.ia2);
    __syncthreads();
    // 4. k1 over h
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[tt][ct] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const bf16_t* hb = xw + (size_t)xr * XS + xk;
    for (int s = 0; s < S1; s += 3) {
        mma8(hb + 32 * s, wr0);
        wload(wr0, w1, S1, s + 3);
        __builtin_amdgcn_sched_barrier(0);
        if (S1 % 3 == 0 || s + 1 < S1) {
            mma8(hb + 32 * (s + 1), wr1);
            wload(wr1, w1, S1, s + 4);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (S1 % 3 == 0 || s + 2 < S1) {
            mma8(hb + 32 * (s + 2), wr2);
            wload(wr2, w1, S1, s + 5);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    // 5. round(acc + b1) parked over h, then per 16-B chunk: residual, store, next Snake
    __syncthreads();
    park(a.b1, nullptr, nullptr);
    __syncthreads();
    for (int q = threadIdx.x; q < BM * (C / 8); q += NT) {
        const int row = q / (C / 8), cc = q - row * (C / 8);
        const int t = t0 + row;
        if (t >= a.L) continue;
        const int co = 8 * cc;
        float y[8], rv[8], al[8], sn[8];
        load8(xw + (size_t)row * XS + co, y);
        load8(a.res + (size_t)t * C + co, rv);
        load8(a.an + co, al);
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = bfround(rv[j] + y[j]);
        if (a.store_res) store8(a.res + (size_t)t * C + co, y);
#pragma unroll
        for (int j = 0; j < 8; ++j) sn[j] = bfround(snake_fi(y[j], al[j], a.ian[co + j]));
        store8(a.out2 + (size_t)t * C + co, sn);
    }
}

// tile variants: {C, BM, time tiles per wave, waves per SIMD, channel tiles per wave}; decoder
// (fm_tune resunit_cfg picks among the 192 / 96 ones), then encoder widths
#define RU_VARIANTS(X)                                                                                  \
    X(192, 128, 8, 2, 3) X(96, 256, 8, 2, 3) X(192, 64, 4, 3, 3) X(96, 128, 4, 4, 3) X(192, 128, 4, 4, 3) \
    X(96, 128, 8, 2, 3) X(384, 64, 4, 2, 3) X(64, 256, 4, 3, 4) X(128, 128, 4, 3, 4) X(256, 64, 4, 3, 4)  \
    X(512, 64, 4, 2, 4)
void resunit_init() {
    static bool done = false;
    if (done) return;
    done = true;
#define RU_ATTR(C, BM, TT, WPE, CT)                                                                 \
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&resunit_kernel<C, BM, TT, WPE, CT>),   \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)ru_lds<C, BM>());
    RU_VARIANTS(RU_ATTR)
#undef RU_ATTR
    (void)hipGetLastError();
}

bool launch_resunit(hipStream_t s, const ResUnitArgs& a, int C) {
    if (!fm_tuning().codec_fuse || a.dil < 1 || a.dil > RU_MAXDIL || a.L < 1 || a.lo > 0) return false;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    FMCHECK(a.x && a.w7 && a.b7 && a.a2 && a.ia2 && a.w1 && a.b1 && a.res && a.an && a.ian && a.out2 && a.zeros &&
                al16(a.x) && al16(a.res) && al16(a.out2) && a.out2 != a.x,
            "resunit: operands");
    const int cfg = fm_tuning().resunit_cfg;
#define RU_GO(CC, BM, TT, WPE, CT)                                                                   \
    resunit_kernel<CC, BM, TT, WPE, CT>                                                                \
        <<<FM_CEIL(a.L, BM), ru_nw<CC, BM, TT, CT>() * 64, ru_lds<CC, BM>(), s>>>(a);                   \
    return true;
    if (C == 384 && fm_tuning().resunit_384) { RU_GO(384, 64, 4, 2, 3) }
    if (C == 192) {
        if (cfg == 0) { RU_GO(192, 128, 8, 2, 3) }
        if (cfg == 2) { RU_GO(192, 128, 4, 4, 3) }
        RU_GO(192, 64, 4, 3, 3)
    }
    if (C == 96) {
        if (cfg == 0) { RU_GO(96, 256, 8, 2, 3) }
        if (cfg == 2) { RU_GO(96, 128, 8, 2, 3) }
        RU_GO(96, 128, 4, 4, 3)
    }
    if (fm_tuning().resunit_enc) {  // encoder widths (EncoderBlock's units, modded_dac.py:623-667)
        if (C == 64) { RU_GO(64, 256, 4, 3, 4) }
        if (C == 128) { RU_GO(128, 128, 4, 3, 4) }
        if (C == 256) { RU_GO(256, 64, 4, 3, 4) }
        if (C == 512) { RU_GO(512, 64, 4, 2, 4) }
    }
#undef RU_GO
    return false;
}

template <typename T> void launch_snake_inv(hipStream_t s, const T* alpha, int64_t n, float* ialpha) {
    snake_inv_kernel<T><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(alpha, n, ialpha);
}
template <typename T> void launch_silu_mul(hipStream_t s, const T* g, T* y, size_t n) {
    silu_mul_kernel<T><<<(int)std::min<size_t>(FM_CEIL(n, 256), 16384), 256, 0, s>>>(g, y, n);
}
template <typename T>
void launch_rvq_decode(hipStream_t s, const int32_t* codes, int Tn, int nq1, int sem, int cbs, int cd,
                       const RvqPtrs& p, int D, T* z) {
    FMCHECK(nq1 >= 1 && nq1 <= 16 && cd >= 1 && cd <= 8, "rvq decode: at most 16 stages of codebook dim <= 8");
    rvq_decode_kernel<T><<<Tn, 1024, 0, s>>>(codes, Tn, nq1, sem, cbs, cd, p, D, z);
}
template <typename T>
void launch_dwconv_ln(hipStream_t s, const T* x, int L, int D, const T* dw, const T* db, const T* lw,
                      const T* lb, T* y, int lo) {
    dwconv_ln_kernel<T><<<L, 256, 0, s>>>(x, L, D, dw, db, lw, lb, y, lo);
}
template <typename T>
void launch_rope_qk(hipStream_t s, T* qkv, int Tn, int H, int hd, const float* tab, int pos0) {
    rope_qk_kernel<T><<<Tn, 256, 0, s>>>(qkv, Tn, H, hd, tab, pos0);
}
template <typename T>
void launch_window_attn(hipStream_t s, const T* qkv, int Tn, int H, int hd, int window, T* out, int npre) {
    FMCHECK(hd <= 64 && window <= 512, "window attention: head_dim <= 64, window <= 512");
    if (window <= 128)
        window_attn_kernel<T, 2><<<dim3(Tn, H), 64, 0, s>>>(qkv, Tn, H, hd, window, out, npre);
    else
        window_attn_kernel<T, 8><<<dim3(Tn, H), 64, 0, s>>>(qkv, Tn, H, hd, window, out, npre);
}
template <typename T>
void launch_audio8(hipStream_t s, const float* a, int64_t n, int64_t npad, T* y) {
    audio8_kernel<T><<<(unsigned)std::min<int64_t>((npad * 8 + 255) / 256, 8192), 256, 0, s>>>(a, n, npad, y);
}
template <typename T>
void launch_snake(hipStream_t s, const T* x, int C, size_t n, const T* alpha, T* y) {
    snake_kernel<T><<<(unsigned)std::min<size_t>((n + 255) / 256, 8192), 256, 0, s>>>(x, C, n, alpha, y);
}
void launch_vq_encode(hipStream_t s, float* r, int Tn, int D, int nst, int cd, const VqEncPtrs& p, int32_t* codes) {
    FMCHECK(nst >= 1 && nst <= 16 && cd >= 1 && cd <= 16, "vq encode: <= 16 stages, codebook_dim <= 16");
    vq_encode_kernel_f<<<Tn, 256, 0, s>>>(r, Tn, D, nst, cd, p, codes);
}
void launch_wn_fold(hipStream_t s, const float* g, const float* v, int rows, int per, float* w) {
    wn_fold_kernel<<<rows, 256, 0, s>>>(g, v, per, w);
}
template <typename T>
void launch_conv_weight(hipStream_t s, const float* w, int kind, int Ci, int Co, int k, int st_, T* out) {
    conv_weight_kernel<T><<<4096, 256, 0, s>>>(w, kind, Ci, Co, k, st_, out);
}

#define CINST(T)                                                                                     \
    template void launch_conv_gemm<T>(hipStream_t, const ConvArgs<T>&);                              \
    template void launch_conv_epi<T>(hipStream_t, const ConvArgs<T>&);                               \
    template void launch_silu_mul<T>(hipStream_t, const T*, T*, size_t);                             \
    template void launch_rvq_decode<T>(hipStream_t, const int32_t*, int, int, int, int, int,         \
                                       const RvqPtrs&, int, T*);                                     \
    template void launch_dwconv_ln<T>(hipStream_t, const T*, int, int, const T*, const T*, const T*, \
                                      const T*, T*, int);                                            \
    template void launch_rope_qk<T>(hipStream_t, T*, int, int, int, const float*, int);              \
    template void launch_window_attn<T>(hipStream_t, const T*, int, int, int, int, T*, int);         \
    template void launch_snake<T>(hipStream_t, const T*, int, size_t, const T*, T*);                 \
    template void launch_snake_inv<T>(hipStream_t, const T*, int64_t, float*);                       \
    template void launch_audio8<T>(hipStream_t, const float*, int64_t, int64_t, T*);                 \
    template void launch_conv_weight<T>(hipStream_t, const float*, int, int, int, int, int, T*);
CINST(bf16_t)
CINST(float)

// MFMA operand fragments shared by every weight-streaming kernel (decode GEMV, batched linears,
// bstream, codec conv GEMM).
//
// One 16x16x32 MFMA step: lane l holds 8 consecutive k of row (l & 15) at k-offset 8 * (l >> 4).
// Weights are pre-packed fragment by fragment (fm_kernels.h), so a weight fragment is 1 KiB of
// contiguous HBM: lane l reads elements [8l, 8l + 8) (bf16) or [4l, 4l + 4) and [256 + 4l, ..)
// (fp32, which runs the same k-layout as eight exact 16x16x4 f32 MFMAs).
//   load_w<NT>(blk, lane)   packed weight fragment (NT: non-temporal, bf16 only)
//   load(p)                 8 contiguous elements along k (an X row in global memory or LDS)
//   load_masked(p, valid)   the same, zeroed when !valid (the load itself is unconditional)
//   zero()                  an all-zero fragment
//   mma(a, b, c)            c += a . b over the 32-wide k block
//   dq8(raw, f0, f1)        16 int8 weights (one int8 unit of a lane: 8 k of k-step 2u, then 8 k
//                           of k-step 2u + 1) as two exact T fragments (weight-only int8)
#pragma once
#include "fm_common.h"

// (float)(int8) of byte j of w: exact, and exact again in bf16 (|q| <= 128 needs 8 bits)
__device__ __forceinline__ float i8f(uint32_t w, int j) { return (float)(int)(int8_t)(w >> (8 * j)); }
// two floats holding bf16-exact values -> one word of packed bf16 (their high halves)
__device__ __forceinline__ uint32_t hi_pair(float lo, float hi) {
    return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);
}

template <typename T> struct Frag;

template <> struct Frag<bf16_t> {
    typedef u32x4_t f;  // 8 bf16 along k
    template <bool NT = false> static __device__ __forceinline__ f load_w(const bf16_t* blk, int lane) {
        const u32x4_t* p = reinterpret_cast<const u32x4_t*>(blk + lane * 8);
        if constexpr (NT) return __builtin_nontemporal_load(p);
        else return *p;
    }
    static __device__ __forceinline__ f load(const bf16_t* p) { return *reinterpret_cast<const u32x4_t*>(p); }
    static __device__ __forceinline__ f load_masked(const bf16_t* p, bool valid) {
        const u32x4_t v = load(p);
        const uint32_t m = valid ? 0xffffffffu : 0u;
        return (u32x4_t){v[0] & m, v[1] & m, v[2] & m, v[3] & m};
    }
    static __device__ __forceinline__ f zero() { return (u32x4_t){0, 0, 0, 0}; }
    static __device__ __forceinline__ void dq8(u32x4_t raw, f& f0, f& f1) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            f& o = h ? f1 : f0;
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                const uint32_t v = raw[2 * h + w];
                o[2 * w] = hi_pair(i8f(v, 0), i8f(v, 1));
                o[2 * w + 1] = hi_pair(i8f(v, 2), i8f(v, 3));
            }
        }
    }
    // 8 int4 codes (nibble e = k e of the lane's 8) -> 8 bf16 values bf16(fma(q - 8, s, z)), RNE
    // (the weight-only int4 dequantisation, launch_quant4 / quantize.py:139-160's affine form)
    static __device__ __forceinline__ f dq4(uint32_t w, float s, float z) {
        f o;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const float v0 = __fmaf_rn((float)((w >> (8 * p)) & 15u) - 8.f, s, z);
            const float v1 = __fmaf_rn((float)((w >> (8 * p + 4)) & 15u) - 8.f, s, z);
            o[p] = (uint32_t)__builtin_bit_cast(uint16_t, static_cast<__bf16>(v0)) |
                   ((uint32_t)__builtin_bit_cast(uint16_t, static_cast<__bf16>(v1)) << 16);
        }
        return o;
    }
    static __device__ __forceinline__ f32x4_t mma(f a, f b, f32x4_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                       __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
    }
};

template <> struct Frag<float> {
    struct f {
        f32x4_t lo, hi;
    };
    template <bool NT = false> static __device__ __forceinline__ f load_w(const float* blk, int lane) {
        f v;
        v.lo = *reinterpret_cast<const f32x4_t*>(blk + lane * 4);
        v.hi = *reinterpret_cast<const f32x4_t*>(blk + 256 + lane * 4);
        return v;
    }
    static __device__ __forceinline__ f load(const float* p) {
        f v;
        v.lo = *reinterpret_cast<const f32x4_t*>(p);
        v.hi = *reinterpret_cast<const f32x4_t*>(p + 4);
        return v;
    }
    static __device__ __forceinline__ f zero() {
        f v;
        v.lo = v.hi = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        return v;
    }
    static __device__ __forceinline__ void dq8(u32x4_t raw, f& f0, f& f1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            f0.lo[j] = i8f(raw[0], j);
            f0.hi[j] = i8f(raw[1], j);
            f1.lo[j] = i8f(raw[2], j);
            f1.hi[j] = i8f(raw[3], j);
        }
    }
    static __device__ __forceinline__ f load_masked(const float* p, bool valid) {
        f v = load(p);
        if (!valid) v = zero();
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

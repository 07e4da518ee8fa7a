// fm_common.h -- shared device helpers for the gfx950 kernels of libfishmi.
//
// Precision model: every kernel is templated on the storage type T of activations and
// weights: bf16_t (production) or float (fp32 validation mode).  Arithmetic is fp32; rnd<T>()
// rounds to the storage type at the points where the reference rounds (identity for float).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// The in-launch hand-offs (split-K partials, attention split combines, the GEMV chain) are the
// write-through form of cdna_hip_programming.md §6 Guideline 16: sc1 stores drained by
// s_waitcnt vmcnt(0), relaxed agent counters, sc1 loads.  That form is measured on gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "libfishmi kernels are written for gfx950 (MI355X): build with --offload-arch=gfx950"
#endif

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;

template <typename T> struct is_bf16 { static constexpr bool value = false; };
template <> struct is_bf16<bf16_t> { static constexpr bool value = true; };

__device__ __forceinline__ float bf2f(bf16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

// round-to-nearest-even fp32 -> bf16 bits, NaN stays NaN: gfx950's v_cvt_pk_bf16_f32 (one VALU
// op, no NaN branch)
__device__ __forceinline__ bf16_t f2bf(float x) { return __builtin_bit_cast(bf16_t, static_cast<__bf16>(x)); }
__device__ __forceinline__ float bfround(float x) { return bf2f(f2bf(x)); }

template <typename T> __device__ __forceinline__ float rnd(float x) {
    if constexpr (is_bf16<T>::value) return bfround(x);
    else return x;
}
template <typename T> __device__ __forceinline__ float ld(const T* p, size_t i) {
    if constexpr (is_bf16<T>::value) return bf2f(p[i]);
    else return p[i];
}
// store with rounding to T
template <typename T> __device__ __forceinline__ void st(T* p, size_t i, float v) {
    if constexpr (is_bf16<T>::value) p[i] = f2bf(v);
    else p[i] = v;
}

// 4 consecutive elements rounded to T (8 B for bf16, 16 B for float), p aligned to that size
template <typename T> __device__ __forceinline__ void store4(T* p, const float (&v)[4]) {
    if constexpr (is_bf16<T>::value) {
        const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
    } else {
        *reinterpret_cast<f32x4_t*>(p) = (f32x4_t){v[0], v[1], v[2], v[3]};
    }
}

// 8 consecutive elements (16 B for bf16, 32 B for float), p 16-byte aligned
template <typename T> __device__ __forceinline__ void load8(const T* p, float (&o)[8]) {
    if constexpr (is_bf16<T>::value) {
        u32x4_t v = *reinterpret_cast<const u32x4_t*>(p);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            o[2 * j] = __uint_as_float(v[j] << 16);
            o[2 * j + 1] = __uint_as_float(v[j] & 0xffff0000u);
        }
    } else {
        f32x4_t a = *reinterpret_cast<const f32x4_t*>(p);
        f32x4_t b = *reinterpret_cast<const f32x4_t*>(p + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { o[j] = a[j]; o[4 + j] = b[j]; }
    }
}

// 8 floats -> 8 consecutive elements of T (values already T-representable for bf16: rounded here
// by the hardware conversion, which is exact on them)
template <typename T> __device__ __forceinline__ void store8(T* p, const float (&v)[8]) {
    if constexpr (is_bf16<T>::value) {
        u32x4_t o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (uint32_t)f2bf(v[2 * j]) | ((uint32_t)f2bf(v[2 * j + 1]) << 16);
        *reinterpret_cast<u32x4_t*>(p) = o;
    } else {
        *reinterpret_cast<f32x4_t*>(p) = (f32x4_t){v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4_t*>(p + 4) = (f32x4_t){v[4], v[5], v[6], v[7]};
    }
}

// workgroup barrier for LDS hand-offs only: unlike __syncthreads() it does not make the wave
// wait for its outstanding global loads and stores (the release fence's vmcnt(0))
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// developer phase timestamps: one 8-word record {tag << 32 | aux, t0..t6} per call
__device__ __forceinline__ void dbg_record(unsigned long long* dbg, unsigned tag, unsigned aux,
                                           const unsigned long long (&t)[7]) {
    const unsigned long long slot = atomicAdd(dbg, 1ull);
    if (slot < (1ull << 20)) {
        unsigned long long* q = dbg + 8 + slot * 8;
        q[0] = ((unsigned long long)tag << 32) | aux;
        for (int z = 0; z < 7; ++z) q[1 + z] = t[z];
    }
}
#define DBG_TS(arr, n) if (a.dbg) arr[n] = __builtin_amdgcn_s_memrealtime();

// ---- wave (64-lane) reductions ------------------------------------------------------------
// DPP lane exchanges inside each 16-lane row (quad xor 1, quad xor 2, half-row mirror, row
// mirror: after all four every lane holds its row's total), then the four row totals combined
// from v_readlane scalars -- no LDS-unit cross-lane traffic (ds_bpermute) on the critical path.
// Every lane of the wave must be active.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_f<0x141>(v);  // row_half_mirror
    v += dpp_f<0x140>(v);  // row_mirror
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}
// every lane of a 16-lane row gets the row's total / maximum (DPP only, no LDS)
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    return v + dpp_f<0x140>(v);
}
__device__ __forceinline__ float row_max16(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v));
    return fmaxf(v, dpp_f<0x140>(v));
}
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v));
    v = fmaxf(v, dpp_f<0x140>(v));
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
// block-wide sum for blockDim.x <= 1024; scratch: >= 16 floats of LDS
__device__ __forceinline__ float block_sum(float v, float* scratch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) scratch[w] = v;
    __syncthreads();
    float t = 0.f;
    for (int i = 0; i < nw; ++i) t += scratch[i];
    return t;
}
// block_sum over LDS-only barriers: the waves do not wait for their outstanding global loads
__device__ __forceinline__ float block_sum_lds(float v, float* scratch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_sum(v);
    lds_barrier();
    if (lane == 0) scratch[w] = v;
    lds_barrier();
    float t = 0.f;
    for (int i = 0; i < nw; ++i) t += scratch[i];
    return t;
}
__device__ __forceinline__ float block_max(float v, float* scratch) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) scratch[w] = v;
    __syncthreads();
    float t = -INFINITY;
    for (int i = 0; i < nw; ++i) t = fmaxf(t, scratch[i]);
    return t;
}

// ---- counter-based RNG (identical formula in fishmi/synth.py and oracle/fishmi_oracle.c) --
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// sampler uniform in [0,1), truncated to bf16, keyed by (seed, step, draw, index)
__device__ __forceinline__ float rng_uniform_bf16(uint64_t seed, uint64_t step, uint32_t draw,
                                                  uint32_t idx) {
    uint64_t key = seed * 0xD1B54A32D192ED03ull + (step * 64ull + draw) * 0x9E3779B97F4A7C15ull + idx;
    uint32_t m = (uint32_t)(splitmix64(key) >> 40);
    float u = (float)m * (1.0f / 16777216.0f);
    return __uint_as_float(__float_as_uint(u) & 0xffff0000u);
}

#define FM_CEIL(a, b) (((a) + (b) - 1) / (b))

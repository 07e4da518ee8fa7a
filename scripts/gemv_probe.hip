// gemv_probe.hip -- microbenchmark of the decode weight-streaming loop design knobs on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/gemv_probe.hip -o gemv_probe
// Each variant computes y = W x (bf16, R=1) for shapes of the S2-Pro decode step and reports
// achieved GB/s (weight bytes / kernel time, HIP events, median of 20).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

template <bool NT> __device__ __forceinline__ u32x4_t ldw(const u32x4_t* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// WAVES waves split K; INTERLEAVE: wave w takes steps w, w+W, ... else a contiguous range
template <bool NT, bool INTER, int U, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void probe(const uint16_t* W, const uint16_t* X, float* Y, int N, int K) {
    __shared__ f32x4_t red[WAVES][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = blockIdx.x * 16;
    const int ks = blockIdx.y, Kb = K / gridDim.y, kbeg = ks * Kb;
    const int r = lane & 15, g = lane >> 4;
    const int steps = Kb >> 5;
    int nmy, sbeg, sstride;
    if (INTER) { nmy = (steps - wave + WAVES - 1) / WAVES; sbeg = wave; sstride = WAVES; }
    else { int a = wave * steps / WAVES, b = (wave + 1) * steps / WAVES; nmy = b - a; sbeg = a; sstride = 1; }
    const uint16_t* wp = W + (size_t)(n0 + r) * K + kbeg + 8 * g;
    const uint16_t* xp = X + kbeg + 8 * g;
    f32x4_t acc = {0, 0, 0, 0};
    if (nmy > 0) {
        u32x4_t fa[U];
        auto off = [&](int i) { int s = i < nmy ? i : nmy - 1; return (size_t)(sbeg + sstride * s) * 32; };
#pragma unroll
        for (int u = 0; u < U; ++u) fa[u] = ldw<NT>((const u32x4_t*)(wp + off(u)));
        for (int i = 0; i < nmy; i += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (i + u < nmy) {
                    u32x4_t xb = *(const u32x4_t*)(xp + off(i + u));
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[u]),
                                                                  __builtin_bit_cast(bf16x8_t, xb), acc, 0, 0, 0);
                }
                fa[u] = ldw<NT>((const u32x4_t*)(wp + off(i + u + U)));
            }
        }
    }
    red[wave][lane] = acc;
    __syncthreads();
    if (threadIdx.x < 64) {
        f32x4_t s = {0, 0, 0, 0};
        for (int w = 0; w < WAVES; ++w) s += red[w][threadIdx.x];
        if ((threadIdx.x & 15) == 0)
            for (int i = 0; i < 4; ++i) Y[(size_t)ks * N + n0 + 4 * (threadIdx.x >> 4) + i] = s[i];
    }
}

// PACKED layout: tile t (16 rows), step s (32 k): 1 KB block at ((t*steps_total + s)*64 + lane)*8
template <int U, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void probe_packed(const uint16_t* W, const uint16_t* X, float* Y, int N, int K) {
    __shared__ f32x4_t red[WAVES][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t = blockIdx.x;
    const int ks = blockIdx.y, S = K >> 5, Sb = S / gridDim.y, sb0 = ks * Sb;
    const int g = lane >> 4;
    const int a = wave * Sb / WAVES, b = (wave + 1) * Sb / WAVES, nmy = b - a;
    const uint16_t* wp = W + ((size_t)t * S + sb0 + a) * 512 + lane * 8;
    const uint16_t* xp = X + (size_t)(sb0 + a) * 32 + 8 * g;
    f32x4_t acc = {0, 0, 0, 0};
    if (nmy > 0) {
        u32x4_t fa[U];
        auto off = [&](int i) { int s = i < nmy ? i : nmy - 1; return (size_t)s; };
#pragma unroll
        for (int u = 0; u < U; ++u) fa[u] = *(const u32x4_t*)(wp + off(u) * 512);
        for (int i = 0; i < nmy; i += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (i + u < nmy) {
                    u32x4_t xb = *(const u32x4_t*)(xp + off(i + u) * 32);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[u]),
                                                                  __builtin_bit_cast(bf16x8_t, xb), acc, 0, 0, 0);
                }
                fa[u] = *(const u32x4_t*)(wp + off(i + u + U) * 512);
            }
        }
    }
    red[wave][lane] = acc;
    __syncthreads();
    if (threadIdx.x < 64) {
        f32x4_t s = {0, 0, 0, 0};
        for (int w = 0; w < WAVES; ++w) s += red[w][threadIdx.x];
        if ((threadIdx.x & 15) == 0)
            for (int i = 0; i < 4; ++i) Y[(size_t)ks * N + 16 * t + 4 * (threadIdx.x >> 4) + i] = s[i];
    }
}

template <int U, int WAVES>
float runp(const uint16_t* W, const uint16_t* X, float* Y, int N, int K, int ksb, int reps = 20) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> t;
    for (int i = 0; i < reps + 3; ++i) {
        CK(hipEventRecord(a));
        probe_packed<U, WAVES><<<dim3(N / 16, ksb), WAVES * 64>>>(W, X, Y, N, K);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (i >= 3) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

template <bool NT, bool INTER, int U, int WAVES>
float run(const uint16_t* W, const uint16_t* X, float* Y, int N, int K, int ksb, int reps = 20) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> t;
    for (int i = 0; i < reps + 3; ++i) {
        CK(hipEventRecord(a));
        probe<NT, INTER, U, WAVES><<<dim3(N / 16, ksb), WAVES * 64>>>(W, X, Y, N, K);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (i >= 3) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    // a big arena so every call streams from HBM (> 256 MiB Infinity Cache): rotate buffers
    const size_t maxw = (size_t)19456 * 2560;
    const int NB = 8;
    std::vector<uint16_t*> Ws(NB);
    for (auto& w : Ws) { CK(hipMalloc(&w, maxw * 2)); CK(hipMemset(w, 0x3c, maxw * 2)); }
    uint16_t* X; CK(hipMalloc(&X, 16384 * 2)); CK(hipMemset(X, 0x3c, 16384 * 2));
    float* Y; CK(hipMalloc(&Y, (size_t)8 * 19456 * 4));
    struct Shape { const char* name; int N, K; };
    Shape shapes[] = {{"qkv 6144x2560", 6144, 2560}, {"w13 19456x2560", 19456, 2560},
                      {"wo 2560x4096", 2560, 4096}, {"w2 2560x9728", 2560, 9728}};
    int wi = 0;
    auto next = [&]() { wi = (wi + 1) % NB; return Ws[wi]; };
#define V(NT, IN, U, WV, KSB) { \
        float ms = 0; for (int k = 0; k < 3; ++k) ms += run<NT, IN, U, WV>(next(), X, Y, s.N, s.K, KSB) / 3; \
        double gbs = (double)s.N * s.K * 2 / (ms * 1e-3) / 1e9; \
        printf("  %-16s nt=%d inter=%d U=%2d waves=%d ksb=%d : %8.2f us  %7.0f GB/s\n", s.name, NT, IN, U, WV, KSB, ms * 1e3, gbs); }
#define P(U, WV, KSB) { \
        float ms = 0; for (int k = 0; k < 3; ++k) ms += runp<U, WV>(next(), X, Y, s.N, s.K, KSB) / 3; \
        double gbs = (double)s.N * s.K * 2 / (ms * 1e-3) / 1e9; \
        printf("  %-16s PACKED U=%2d waves=%d ksb=%d : %8.2f us  %7.0f GB/s\n", s.name, U, WV, KSB, ms * 1e3, gbs); }
    for (auto& s : shapes) {
        printf("%s\n", s.name);
        P(4, 8, 1) P(8, 8, 1) P(16, 8, 1) P(4, 4, 1) P(8, 4, 1) P(16, 4, 1) P(8, 16, 1) P(4, 16, 1)
        if (s.N <= 6144) { P(8, 8, 2) P(8, 8, 4) P(8, 4, 2) P(8, 4, 4) P(16, 4, 4) P(4, 8, 4) }
    }
    for (auto& s : shapes) {
        printf("%s\n", s.name);
        V(true, true, 8, 8, 1) V(false, true, 8, 8, 1) V(false, false, 8, 8, 1) V(true, false, 8, 8, 1)
        V(false, false, 16, 8, 1) V(false, false, 4, 8, 1) V(false, false, 8, 4, 1) V(false, false, 16, 4, 1)
        if (s.N <= 6144) {
            V(false, false, 8, 8, 2) V(false, false, 8, 8, 4) V(true, true, 8, 8, 4) V(false, true, 8, 8, 4)
            V(false, false, 16, 4, 4) V(false, false, 8, 4, 4)
        }
    }
    return 0;
}

// stream_probe.hip -- pure weight-streaming microbenchmark for the decode GEMV design on gfx950.
// y[n] = sum_k W[n][k] x[k], bf16 W pre-packed in MFMA fragment order ([N/16][K/32] x 1 KiB),
// R = 1, x staged in LDS, no prologue / epilogue fusion.  10 distinct weight buffers are cycled
// so every launch streams from HBM (not the 256 MiB MALL).  Reports GB/s of weight bytes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/stream_probe.hip -o stream_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            printf("%s: %s\n", #x, hipGetErrorString(e));                  \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

template <bool NT> __device__ __forceinline__ u32x4_t ldw(const uint16_t* p) {
    const u32x4_t* q = reinterpret_cast<const u32x4_t*>(p);
    if constexpr (NT) return __builtin_nontemporal_load(q);
    else return *q;
}

// TPB tiles (16 rows each) per block, WPT waves per tile splitting K.
// INTER: wave w of a tile takes k-steps w, w+WPT, ... (neighbouring waves read neighbouring KiB);
// else a contiguous run.  KSB: K split across blocks (grid.y).
template <int U, bool NT, bool INTER, int TPB, int WPT>
__global__ __launch_bounds__(TPB* WPT * 64) void stream_kernel(const uint16_t* __restrict__ W,
                                                               const uint16_t* __restrict__ X, float* Y,
                                                               int N, int K) {
    __shared__ __attribute__((aligned(16))) uint16_t xs[8192 + 64];
    __shared__ f32x4_t red[TPB * WPT][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int tl = wv / WPT, wi = wv - tl * WPT;
    const int tile = blockIdx.x * TPB + tl;
    const int ksb = gridDim.y, Kb = K / ksb, kbeg = blockIdx.y * Kb;
    const int S = K >> 5, Sb = Kb >> 5, sb0 = blockIdx.y * Sb;
    for (int i = threadIdx.x; i < Kb / 8; i += blockDim.x)
        *reinterpret_cast<u32x4_t*>(xs + 8 * i) = *reinterpret_cast<const u32x4_t*>(X + kbeg + 8 * i);
    int nmy, s0, sst;
    if (INTER) {
        nmy = (Sb - wi + WPT - 1) / WPT;
        s0 = wi;
        sst = WPT;
    } else {
        const int a = wi * Sb / WPT, b = (wi + 1) * Sb / WPT;
        nmy = b - a;
        s0 = a;
        sst = 1;
    }
    const uint16_t* wp = W + ((size_t)tile * S + sb0) * 512 + lane * 8;
    const int last = nmy > 0 ? nmy - 1 : 0;
    u32x4_t fa[U];
#pragma unroll
    for (int u = 0; u < U; ++u) fa[u] = ldw<NT>(wp + (size_t)(s0 + sst * (u < last ? u : last)) * 512);
    __syncthreads();
    const int g = lane >> 4;
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < nmy; i += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + u < nmy) {
                const u32x4_t xb = *reinterpret_cast<const u32x4_t*>(xs + (s0 + sst * (i + u)) * 32 + 8 * g);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[u]),
                                                              __builtin_bit_cast(bf16x8_t, xb), acc, 0, 0, 0);
            }
            const int j = i + u + U;
            fa[u] = ldw<NT>(wp + (size_t)(s0 + sst * (j < last ? j : last)) * 512);
        }
    }
    red[wv][lane] = acc;
    __syncthreads();
    if (wi == 0 && lane < 16) {
        float s = 0.f;
        for (int w = 0; w < WPT; ++w) s += red[tl * WPT + w][lane][0];
        Y[(size_t)blockIdx.y * N + tile * 16 + lane] = s;
    }
}

struct Shape {
    const char* name;
    int N, K;
};

static int g_nbuf = 10;  // weight buffers cycled (1 = the same buffer every launch: MALL-resident)

template <int U, bool NT, bool INTER, int TPB, int WPT>
static void run(const char* tag, std::vector<uint16_t*>& Ws, uint16_t* X, float* Y, const Shape& sh, int ksb) {
    const int tiles = sh.N / 16;
    if (tiles % TPB) return;
    if ((sh.K / ksb) > 8192 || (sh.K / ksb) % 32) return;
    dim3 grid(tiles / TPB, ksb);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 10; ++i)
        stream_kernel<U, NT, INTER, TPB, WPT><<<grid, TPB * WPT * 64>>>(Ws[i % g_nbuf], X, Y, sh.N, sh.K);
    CK(hipDeviceSynchronize());
    const int reps = 40;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        stream_kernel<U, NT, INTER, TPB, WPT><<<grid, TPB * WPT * 64>>>(Ws[i % g_nbuf], X, Y, sh.N, sh.K);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps;
    const double bytes = (double)sh.N * sh.K * 2;
    printf("%-10s %-28s nbuf=%d ksb=%d blocks=%5d  %7.2f us  %7.1f GB/s\n", sh.name, tag, g_nbuf, ksb, grid.x * grid.y, us,
           bytes / us / 1e3);
}

int main() {
    const Shape shapes[] = {{"w13(2x)", 19456, 2560}, {"wqkv", 6144, 2560}, {"w2", 2560, 9728}, {"wo", 2560, 4096}};
    size_t maxb = 0;
    for (auto& s : shapes) maxb = std::max(maxb, (size_t)s.N * s.K * 2);
    std::vector<uint16_t*> Ws(10);
    for (auto& w : Ws) {
        CK(hipMalloc(&w, maxb));
        CK(hipMemset(w, 0x3c, maxb));
    }
    uint16_t* X;
    float* Y;
    CK(hipMalloc(&X, 16384 * 2));
    CK(hipMemset(X, 0x3c, 16384 * 2));
    CK(hipMalloc(&Y, 8 * 32768 * 4));
    for (int nb : {10}) {
        g_nbuf = nb;
        for (auto& sh : shapes) {
            for (int ksb : {1, 2, 4, 8}) {
                run<8, true, false, 1, 4>(&"u8 nt run 1x4"[0], Ws, X, Y, sh, ksb);
                run<16, true, false, 1, 4>(&"u16 nt run 1x4"[0], Ws, X, Y, sh, ksb);
                run<8, true, false, 1, 8>(&"u8 nt run 1x8"[0], Ws, X, Y, sh, ksb);
            }
        }
    }
    return 0;
}

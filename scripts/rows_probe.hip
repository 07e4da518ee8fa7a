// rows_probe.hip -- B=1 decode GEMV: 16-row MFMA tiles (the production grid shape, whole K per
// block) against a row-balanced VALU stream (rows split evenly over the grid, no split-K hand-off).
// y[n] = sum_k W[n][k] x[k], bf16, R = 1, x staged in LDS.  10 distinct weight sets are cycled so
// every launch streams from HBM.  Part 1: back-to-back launches per shape; part 2: the four
// dependent GEMVs of one S2-Pro layer (QKV -> Wo -> W13 -> W2) captured in a hipGraph.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/rows_probe.hip -o scripts/rows_probe
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

// production shape: one 16-row tile per block, 4 waves each streaming a contiguous k-run, U in flight
template <int U>
__global__ __launch_bounds__(256) void tile_kernel(const uint16_t* __restrict__ W, const uint16_t* __restrict__ X,
                                                   float* Y, int N, int K) {
    __shared__ __attribute__((aligned(16))) uint16_t xs[9728 + 64];
    __shared__ f32x4_t red[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int tile = blockIdx.x;
    const int S = K >> 5;
    const int a = wv * S / 4, b = (wv + 1) * S / 4, nmy = b - a;
    const uint16_t* wp = W + ((size_t)tile * S + a) * 512 + lane * 8;
    const int last = nmy > 0 ? nmy - 1 : 0;
    u32x4_t fa[U];
#pragma unroll
    for (int u = 0; u < U; ++u) fa[u] = ldw<true>(wp + (size_t)(u < last ? u : last) * 512);
    for (int i = threadIdx.x; i < K / 8; i += blockDim.x)
        *reinterpret_cast<u32x4_t*>(xs + 8 * i) = *reinterpret_cast<const u32x4_t*>(X + 8 * i);
    __syncthreads();
    const int g = lane >> 4;
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < nmy; i += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + u < nmy) {
                const u32x4_t xb = *reinterpret_cast<const u32x4_t*>(xs + (a + i + u) * 32 + 8 * g);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[u]),
                                                              __builtin_bit_cast(bf16x8_t, xb), acc, 0, 0, 0);
            }
            const int j = i + u + U;
            fa[u] = ldw<true>(wp + (size_t)(j < last ? j : last) * 512);
        }
    }
    red[wv][lane] = acc;
    __syncthreads();
    if (wv == 0 && lane < 16) {
        float s = 0.f;
        for (int w = 0; w < 4; ++w) s += red[w][lane][0];
        Y[tile * 16 + lane] = s;
    }
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    return v;
}

__device__ __forceinline__ float dot8(u32x4_t w, u32x4_t x, float acc) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        acc += __uint_as_float(w[i] << 16) * __uint_as_float(x[i] << 16);
        acc += __uint_as_float(w[i] & 0xffff0000u) * __uint_as_float(x[i] & 0xffff0000u);
    }
    return acc;
}

// row-balanced: block b owns rows [b*rb, b*rb+rb); its (row, 512-k chunk) items, row-major, are
// dealt to the WPB waves round-robin (neighbouring waves read neighbouring KiB); each wave keeps
// one running sum and flushes it (wave reduction -> red[row][wave]) when its row changes.
template <int U, int WPB>
__global__ __launch_bounds__(WPB * 64) void rows_kernel(const uint16_t* __restrict__ W,
                                                        const uint16_t* __restrict__ X, float* Y, int N, int K,
                                                        int rb) {
    __shared__ __attribute__((aligned(16))) uint16_t xs[9728 + 64];
    __shared__ float red[128 * WPB];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r0 = blockIdx.x * rb, nr = min(rb, N - r0);
    const int nck = K >> 9;
    const int nit = nr * nck;
    const int nmy = nit > wv ? (nit - wv + WPB - 1) / WPB : 0;
    const int last = nmy > 0 ? nmy - 1 : 0;
    auto item_ptr = [&](int j) {
        const int it = wv + WPB * (j < last ? j : last);
        const int row = it / nck, ck = it - row * nck;
        return W + (size_t)(r0 + row) * K + ck * 512 + lane * 8;
    };
    u32x4_t fa[U];
#pragma unroll
    for (int u = 0; u < U; ++u) fa[u] = ldw<true>(item_ptr(u));
    for (int i = threadIdx.x; i < K / 8; i += blockDim.x)
        *reinterpret_cast<u32x4_t*>(xs + 8 * i) = *reinterpret_cast<const u32x4_t*>(X + 8 * i);
    for (int i = threadIdx.x; i < rb * WPB; i += blockDim.x) red[i] = 0.f;
    __syncthreads();
    float acc = 0.f;
    int cur = nmy > 0 ? wv / nck : 0;
    for (int i = 0; i < nmy; i += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + u < nmy) {
                const int it = wv + WPB * (i + u);
                const int row = it / nck, ck = it - row * nck;
                if (row != cur) {
                    const float s = wsum(acc);
                    if (lane == 0) red[cur * WPB + wv] = s;
                    acc = 0.f;
                    cur = row;
                }
                const u32x4_t xb = *reinterpret_cast<const u32x4_t*>(xs + ck * 512 + lane * 8);
                acc = dot8(fa[u], xb, acc);
            }
            fa[u] = ldw<true>(item_ptr(i + u + U));
        }
    }
    if (nmy > 0) {
        const float s = wsum(acc);
        if (lane == 0) red[cur * WPB + wv] = s;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < nr; t += blockDim.x) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < WPB; ++w) s += red[t * WPB + w];
        Y[r0 + t] = s;
    }
}


// row-pair fragments: fragment (pair q, kf) = rows 2q, 2q+1 x k [256 kf, 256 kf + 256); lane l holds
// row 2q + (m & 1), k 256 kf + 32 (m >> 1) + 8 (l >> 4) .. +8, m = l & 15.  B column c < 8 = the x
// segment c, so D[2s + r][s] summed over s is y[2q + r].  Block = P pairs; wave w streams the kf
// range [w F / WPB, (w + 1) F / WPB) of all P pairs (x fragment reused P times), KA kf ahead.
template <int P, int KA, int WPB>
__global__ __launch_bounds__(WPB * 64) void pair_kernel(const uint16_t* __restrict__ W, const uint16_t* __restrict__ X,
                                                        float* Y, int N, int K) {
    __shared__ __attribute__((aligned(16))) uint16_t xs[9728 + 64];
    __shared__ float red[P][WPB][8][2];
    constexpr int U = KA * P;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int F = K >> 8;
    const int q0 = blockIdx.x * P;
    const int ka = wv * F / WPB, nkf = (wv + 1) * F / WPB - ka;
    const int last = nkf > 0 ? nkf - 1 : 0;
    const uint16_t* wp = W + ((size_t)q0 * F + ka) * 512 + lane * 8;
    u32x4_t fa[U];
    auto issue = [&](int kf, int slot, int p) {
        fa[slot] = ldw<true>(wp + ((size_t)p * F + (kf < last ? kf : last)) * 512);
    };
#pragma unroll
    for (int a = 0; a < KA; ++a)
#pragma unroll
        for (int p = 0; p < P; ++p) issue(a, a * P + p, p);
    for (int i = threadIdx.x; i < K / 8; i += blockDim.x)
        *reinterpret_cast<u32x4_t*>(xs + 8 * i) = *reinterpret_cast<const u32x4_t*>(X + 8 * i);
    __syncthreads();
    const int c = lane & 7, g = lane >> 4;
    f32x4_t acc[P];
#pragma unroll
    for (int p = 0; p < P; ++p) acc[p] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < nkf; i += KA) {
#pragma unroll
        for (int a = 0; a < KA; ++a) {
            if (i + a < nkf) {
                const u32x4_t xb = *reinterpret_cast<const u32x4_t*>(xs + (ka + i + a) * 256 + 32 * c + 8 * g);
#pragma unroll
                for (int p = 0; p < P; ++p)
                    acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[a * P + p]),
                                                                     __builtin_bit_cast(bf16x8_t, xb), acc[p], 0, 0, 0);
            }
#pragma unroll
            for (int p = 0; p < P; ++p) issue(i + a + KA, a * P + p, p);
        }
    }
    const int s = lane & 15;
    if (s < 8 && g == (s >> 1)) {
#pragma unroll
        for (int p = 0; p < P; ++p) {
            red[p][wv][s][0] = (s & 1) ? acc[p][2] : acc[p][0];
            red[p][wv][s][1] = (s & 1) ? acc[p][3] : acc[p][1];
        }
    }
    __syncthreads();
    if (threadIdx.x < 2 * P) {
        const int p = threadIdx.x >> 1, r = threadIdx.x & 1;
        float v = 0.f;
        for (int w = 0; w < WPB; ++w)
            for (int ss = 0; ss < 8; ++ss) v += red[p][w][ss][r];
        Y[2 * (q0 + p) + r] = v;
    }
}

struct Shape {
    const char* name;
    int N, K;
};

struct Launch {
    int kind;  // 0 tile, 1 rows
    int U, WPB, nblk;
};

static void launch(const Launch& L, const uint16_t* W, const uint16_t* X, float* Y, const Shape& sh, hipStream_t s) {
    if (L.kind == 0) {
        if (L.U == 8) tile_kernel<8><<<sh.N / 16, 256, 0, s>>>(W, X, Y, sh.N, sh.K);
        else tile_kernel<16><<<sh.N / 16, 256, 0, s>>>(W, X, Y, sh.N, sh.K);
        return;
    }
    if (L.kind == 2) {
        const int P = L.nblk, grid = sh.N / 2 / P;
        if ((sh.N / 2) % P) { printf("bad P\n"); exit(1); }
#define PK(PP, KK, WW)                                                                              \
        if (P == PP && L.U == KK && L.WPB == WW) {                                                  \
            pair_kernel<PP, KK, WW><<<grid, WW * 64, 0, s>>>(W, X, Y, sh.N, sh.K);                  \
            return;                                                                                 \
        }
        PK(5, 2, 4) PK(5, 3, 4) PK(5, 2, 8) PK(12, 1, 4) PK(12, 2, 4) PK(6, 2, 4) PK(6, 3, 4) PK(12, 1, 8) PK(6, 2, 8)
        PK(38, 1, 4) PK(19, 1, 4) PK(19, 2, 4)
#undef PK
        printf("no pair kernel\n");
        exit(1);
    }
    const int rb = (sh.N + L.nblk - 1) / L.nblk;
    const int nb = (sh.N + rb - 1) / rb;
#define RK(UU, WW)                                                                   \
    if (L.U == UU && L.WPB == WW) {                                                  \
        rows_kernel<UU, WW><<<nb, WW * 64, 0, s>>>(W, X, Y, sh.N, sh.K, rb);         \
        return;                                                                      \
    }
    RK(8, 4) RK(16, 4) RK(8, 8) RK(16, 8) RK(4, 8)
#undef RK
    printf("no kernel\n");
    exit(1);
}

int main() {
    const Shape shapes[] = {{"wqkv", 6144, 2560}, {"wo", 2560, 4096}, {"w13", 19456, 2560}, {"w2", 2560, 9728}};
    const int NSET = 10;
    std::vector<uint16_t*> Ws[4];
    for (int s = 0; s < 4; ++s)
        for (int i = 0; i < NSET; ++i) {
            uint16_t* w;
            const size_t b = (size_t)shapes[s].N * shapes[s].K * 2;
            CK(hipMalloc(&w, b));
            CK(hipMemset(w, 0x3c, b));
            Ws[s].push_back(w);
        }
    uint16_t* X;
    float* Y;
    CK(hipMalloc(&X, 16384 * 2));
    CK(hipMemset(X, 0x3c, 16384 * 2));
    CK(hipMalloc(&Y, 32768 * 4));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    // per shape: {kind, U | KA, WPB, nblk | P}
    std::vector<Launch> vs[4] = {
        {{0, 8, 4, 0}, {2, 1, 4, 12}, {2, 2, 4, 12}, {2, 1, 8, 12}, {2, 2, 4, 6}, {2, 3, 4, 6}, {2, 2, 8, 6}},
        {{0, 8, 4, 0}, {2, 2, 4, 5}, {2, 3, 4, 5}, {2, 2, 8, 5}},
        {{0, 8, 4, 0}, {2, 1, 4, 19}, {2, 2, 4, 19}, {2, 1, 4, 38}},
        {{0, 8, 4, 0}, {2, 2, 4, 5}, {2, 3, 4, 5}, {2, 2, 8, 5}},
    };
    std::vector<Launch> variants = {{0, 8, 4, 0}};
    auto name = [](const Launch& L) {
        static char b[64];
        if (L.kind == 0) snprintf(b, sizeof b, "tile16 U%d", L.U);
        else if (L.kind == 1) snprintf(b, sizeof b, "rows U%d W%d nblk%d", L.U, L.WPB, L.nblk);
        else snprintf(b, sizeof b, "pair P%d KA%d W%d", L.nblk, L.U, L.WPB);
        return b;
    };
    // part 1: per shape, 40 back-to-back launches cycling the weight sets, in one graph
    for (int s = 0; s < 4; ++s) {
        for (const Launch& L : vs[s]) {
            const int reps = 40;
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
            for (int i = 0; i < reps; ++i) launch(L, Ws[s][i % NSET], X, Y, shapes[s], st);
            CK(hipStreamEndCapture(st, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ge, st));
            CK(hipStreamSynchronize(st));
            float best = 1e30f;
            for (int t = 0; t < 5; ++t) {
                CK(hipEventRecord(e0, st));
                CK(hipGraphLaunch(ge, st));
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms);
            }
            const double us = best * 1e3 / reps, bytes = (double)shapes[s].N * shapes[s].K * 2;
            printf("%-5s %-24s %7.2f us %7.1f GB/s\n", shapes[s].name, name(L), us, bytes / us / 1e3);
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
        }
    }
    // part 2: layer chains (QKV -> Wo -> W13 -> W2) x 40 layers, one variant for all four matrices
    const Launch chains[][4] = {
        {{0, 8, 4, 0}, {0, 8, 4, 0}, {0, 8, 4, 0}, {0, 8, 4, 0}},
        {{2, 1, 4, 12}, {2, 2, 4, 5}, {0, 8, 4, 0}, {2, 2, 4, 5}},
        {{2, 2, 4, 6}, {2, 2, 4, 5}, {0, 8, 4, 0}, {2, 2, 4, 5}},
        {{2, 2, 4, 6}, {2, 3, 4, 5}, {2, 1, 4, 19}, {2, 3, 4, 5}},
    };
    for (const auto& C : chains) {
        const Launch& L = C[0];
        const int layers = 40;
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < layers; ++i)
            for (int s = 0; s < 4; ++s) launch(C[s], Ws[s][i % NSET], X, Y, shapes[s], st);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        float best = 1e30f;
        for (int t = 0; t < 5; ++t) {
            CK(hipEventRecord(e0, st));
            CK(hipGraphLaunch(ge, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        double bytes = 0;
        for (int s = 0; s < 4; ++s) bytes += (double)shapes[s].N * shapes[s].K * 2;
        const double us = best * 1e3 / layers;
        printf("layer %-24s|%s %7.2f us per layer %7.1f GB/s\n", name(L), C[1].kind ? "pairs" : "tiles", us, bytes / us / 1e3);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}

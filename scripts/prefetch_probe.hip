// prefetch_probe.hip -- can a weight stream be hidden behind the latency-bound parts of a decode
// frame by pulling the NEXT matrix into the Infinity Cache (MALL, 256 MiB) on a second graph branch?
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/prefetch_probe.hip -o scripts/prefetch_probe
//
//   A  graph-branch concurrency: two 20 us spin kernels on forked capture streams (one block each);
//      replay time ~20 us = branches run concurrently, ~40 us = serialised
//   B  read time of a W-byte buffer by a GEMV-shaped stream kernel (16-row tiles, 1 KiB fragments,
//      4 waves per block, ring of 8): cold (after a 1 GiB flush), after a default-policy prefetch,
//      after an nt prefetch, warm (second read)
//   C  overlap: spin kernel (attention-like latency phase, 8 blocks) || prefetch of the next matrix on
//      P blocks, then the GEMV-shaped read of that matrix; vs the same without the prefetch branch
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e = (x);                                                                       \
        if (e != hipSuccess) {                                                                    \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));               \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

// GEMV-shaped read: block b streams tile b's fragments (K/32 of them) split over 4 waves
template <bool NT>
__global__ __launch_bounds__(256) void tile_read(const u32x4_t* W, int frags_per_tile, unsigned* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int f0 = frags_per_tile * wave / 4, f1 = frags_per_tile * (wave + 1) / 4;
    const u32x4_t* base = W + (size_t)blockIdx.x * frags_per_tile * 64;
    u32x4_t acc = {0, 0, 0, 0}, ring[8];
    const int n = f1 - f0, last = n - 1;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const u32x4_t* p = base + (size_t)(f0 + (u < n ? u : last)) * 64 + lane;
        ring[u] = NT ? __builtin_nontemporal_load(p) : *p;
    }
    for (int i = 0; i < n; i += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            acc ^= ring[u];
            const int j = i + u + 8 < n ? i + u + 8 : last;
            const u32x4_t* p = base + (size_t)(f0 + j) * 64 + lane;
            ring[u] = NT ? __builtin_nontemporal_load(p) : *p;
        }
    }
    const unsigned s = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
    if (s == 0x12345678u) out[blockIdx.x] = s;
}

// prefetch: nb blocks of 256 threads sweep the buffer with 8 x 16 B loads in flight per lane
template <bool NT>
__global__ __launch_bounds__(256) void prefetch(const u32x4_t* W, size_t n16, unsigned* out) {
    const size_t nth = (size_t)gridDim.x * 256, t = (size_t)blockIdx.x * 256 + threadIdx.x;
    u32x4_t acc = {0, 0, 0, 0};
    for (size_t i = t; i < n16; i += 8 * nth) {
        u32x4_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const size_t j = i + u * nth < n16 ? i + u * nth : i;
            v[u] = NT ? __builtin_nontemporal_load(W + j) : W[j];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u];
    }
    const unsigned s = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
    if (s == 0x12345678u) out[t & 1023] = s;
}

__global__ void spin(long long ns, unsigned* out) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) * 10 < ns) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0 && ns < 0) out[0] = 1;
}

__global__ void flush(uint32_t* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i;
}

static float med(std::vector<float> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t e0, e1, ef, ej;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
    unsigned* out;
    CK(hipMalloc(&out, 1 << 20));
    const size_t FL = (size_t)1 << 30;
    uint32_t* F;
    CK(hipMalloc(&F, FL));
    auto doflush = [&]() { flush<<<4096, 256, 0, s0>>>(F, FL / 4); };
    auto timed = [&](auto&& body) {
        CK(hipEventRecord(e0, s0));
        body();
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1e3f;
    };

    // ---- A: graph branch concurrency
    {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
        CK(hipEventRecord(ef, s0));
        CK(hipStreamWaitEvent(s1, ef, 0));
        spin<<<1, 64, 0, s0>>>(20000, out);
        spin<<<1, 64, 0, s1>>>(20000, out);
        CK(hipEventRecord(ej, s1));
        CK(hipStreamWaitEvent(s0, ej, 0));
        CK(hipStreamEndCapture(s0, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        std::vector<float> t;
        for (int i = 0; i < 15; ++i) t.push_back(timed([&] { CK(hipGraphLaunch(ge, s0)); }));
        std::vector<float> t1;
        for (int i = 0; i < 15; ++i) t1.push_back(timed([&] { spin<<<1, 64, 0, s0>>>(20000, out); }));
        printf("A graph: two forked 20 us spins %.1f us (one spin alone %.1f us)\n", med(t), med(t1));
    }

    // ---- B / C per matrix size (S2-Pro shapes: Wo 21 MB, QKV 31.5, W2 49.8, W13 99.6)
    struct Shape { const char* name; int tiles, kfr; };
    const Shape shapes[] = {{"wo", 160, 128}, {"qkv", 384, 80}, {"w2", 160, 304}, {"w13", 1216, 80}};
    for (const Shape& sh : shapes) {
        const size_t bytes = (size_t)sh.tiles * sh.kfr * 1024;
        u32x4_t* W;
        CK(hipMalloc(&W, bytes));
        CK(hipMemset(W, 1, bytes));
        std::vector<float> cold, pdef, pnt, warm;
        for (int rep = 0; rep < 9; ++rep) {
            doflush();
            cold.push_back(timed([&] { tile_read<true><<<sh.tiles, 256, 0, s0>>>(W, sh.kfr, out); }));
            warm.push_back(timed([&] { tile_read<true><<<sh.tiles, 256, 0, s0>>>(W, sh.kfr, out); }));
            doflush();
            prefetch<false><<<1024, 256, 0, s0>>>(W, bytes / 16, out);
            pdef.push_back(timed([&] { tile_read<true><<<sh.tiles, 256, 0, s0>>>(W, sh.kfr, out); }));
            doflush();
            prefetch<true><<<1024, 256, 0, s0>>>(W, bytes / 16, out);
            pnt.push_back(timed([&] { tile_read<true><<<sh.tiles, 256, 0, s0>>>(W, sh.kfr, out); }));
        }
        auto tb = [&](float us) { return bytes / (us * 1e-6) / 1e12; };
        printf("B %-4s %6.1f MB: cold %6.2f us %5.2f TB/s | after default prefetch %6.2f us %5.2f TB/s | after nt prefetch %6.2f us %5.2f TB/s | warm %6.2f us %5.2f TB/s\n",
               sh.name, bytes / 1e6, med(cold), tb(med(cold)), med(pdef), tb(med(pdef)), med(pnt), tb(med(pnt)),
               med(warm), tb(med(warm)));
        // C: latency phase (8 spinning blocks, T us) || prefetch on P blocks, then the read
        for (int T : {6, 12}) {
            for (int P : {0, 16, 32, 64}) {
                hipGraph_t g;
                hipGraphExec_t ge;
                CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
                if (P) {
                    CK(hipEventRecord(ef, s0));
                    CK(hipStreamWaitEvent(s1, ef, 0));
                    prefetch<false><<<P, 256, 0, s1>>>(W, bytes / 16, out);
                }
                spin<<<8, 256, 0, s0>>>((long long)T * 1000, out);
                tile_read<true><<<sh.tiles, 256, 0, s0>>>(W, sh.kfr, out);
                if (P) {
                    CK(hipEventRecord(ej, s1));
                    CK(hipStreamWaitEvent(s0, ej, 0));
                }
                CK(hipStreamEndCapture(s0, &g));
                CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
                std::vector<float> t;
                for (int rep = 0; rep < 9; ++rep) {
                    doflush();
                    t.push_back(timed([&] { CK(hipGraphLaunch(ge, s0)); }));
                }
                printf("C %-4s spin %2d us + read, prefetch branch on %2d blocks: %6.2f us\n", sh.name, T, P, med(t));
                CK(hipGraphExecDestroy(ge));
                CK(hipGraphDestroy(g));
            }
        }
        CK(hipFree(W));
    }
    CK(hipDeviceSynchronize());
    return 0;
}

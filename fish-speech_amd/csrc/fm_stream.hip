// fm_stream.hip -- the measured HBM stream peak the bench line quotes beside the vendor figure
// (SURVEY.md §8d): a non-temporal read-only stream and a float4 copy over buffers far larger than
// the 256 MiB MALL, HIP events around `reps` launches.  Not on any decode path.
#include "fm_common.h"
#include "fm_runtime.h"

#include <algorithm>

namespace {
typedef __attribute__((ext_vector_type(4))) float f4_t;

// every thread sums U float4 per step (non-temporal loads, U in flight); one float per block out
template <int U>
__global__ __launch_bounds__(256) void stream_read_kernel(const f4_t* __restrict__ a, int64_t n4, float* out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float acc = 0.f;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        f4_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += (v[u].x + v[u].y) + (v[u].z + v[u].w);
    }
    for (; i < n4; i += stride) {
        const f4_t v = __builtin_nontemporal_load(a + i);
        acc += (v.x + v.y) + (v.z + v.w);
    }
    if (acc == 1234.5f) out[blockIdx.x] = acc;  // (keeps the loads; never true for the zeroed input)
}

// non-temporal LDS-DMA read stream (global_load_lds_dwordx4 nt, the decode pass's loader form):
// every wave moves 1 KiB chunks into its own LDS slot, INF chunks in flight (vmcnt-throttled)
template <int INF>
__global__ __launch_bounds__(256) void stream_ldsdma_kernel(const char* __restrict__ a, int64_t nchunks) {
    __shared__ __attribute__((aligned(16))) unsigned char slot[4][1024];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const uint32_t dst = (uint32_t)(size_t)(const __attribute__((address_space(3))) unsigned char*)slot[wave];
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(dst);
    int n = 0;
    for (int64_t c = (int64_t)blockIdx.x * 4 + wave; c < nchunks; c += nw) {
        const char* src = a + c * 1024 + lane * 16;
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off nt\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(m0)
            : "memory");
        if (++n >= INF) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INF - 1) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ __launch_bounds__(256) void stream_copy_kernel(const f4_t* __restrict__ a, f4_t* __restrict__ b, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}
}  // namespace

extern "C" int fm_stream_peak(int device, int64_t bytes, int reps, double* read_gbps, double* copy_gbps) {
    return fm_guard([&] {
        FMCHECK(bytes >= (64 << 20) && bytes % 64 == 0 && reps >= 1, "stream_peak: bytes >= 64 MiB, multiple of 64");
        HIPCHK(hipSetDevice(device));
        int ncu = 0;
        HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
        void *a = nullptr, *b = nullptr, *o = nullptr;
        HIPCHK(hipMalloc(&a, bytes));
        HIPCHK(hipMalloc(&b, bytes));
        HIPCHK(hipMalloc(&o, 65536 * sizeof(float)));
        HIPCHK(hipMemset(a, 0, bytes));
        hipEvent_t e0, e1;
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        const int64_t n4 = bytes / 16;
        const int grid = ncu * 8;
        auto time = [&](auto launch) {
            launch();
            HIPCHK(hipEventRecord(e0, nullptr));
            for (int r = 0; r < reps; ++r) launch();
            HIPCHK(hipEventRecord(e1, nullptr));
            HIPCHK(hipEventSynchronize(e1));
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, e0, e1));
            return (double)ms * 1e-3;
        };
        // the best of several forms, so the quoted peak is what the part does, not what one kernel
        // shape reaches: register float4 streams (4 / 8 in flight per thread, 8 / 16 blocks per CU)
        // and non-temporal LDS-DMA streams (16 / 32 KiB in flight per wave)
        double tr = 1e30, tc = 1e30;
        tr = std::min(tr, time([&] {
            stream_read_kernel<4><<<grid, 256>>>(reinterpret_cast<const f4_t*>(a), n4, reinterpret_cast<float*>(o));
        }));
        tr = std::min(tr, time([&] {
            stream_read_kernel<8><<<ncu * 16, 256>>>(reinterpret_cast<const f4_t*>(a), n4, reinterpret_cast<float*>(o));
        }));
        const int64_t nch = bytes / 1024;
        tr = std::min(tr, time([&] {
            stream_ldsdma_kernel<16><<<ncu * 2, 256>>>(reinterpret_cast<const char*>(a), nch);
        }));
        tr = std::min(tr, time([&] {
            stream_ldsdma_kernel<32><<<ncu * 2, 256>>>(reinterpret_cast<const char*>(a), nch);
        }));
        tc = std::min(tc, time([&] {
            stream_copy_kernel<<<grid, 256>>>(reinterpret_cast<const f4_t*>(a), reinterpret_cast<f4_t*>(b), n4);
        }));
        tc = std::min(tc, time([&] {
            stream_copy_kernel<<<ncu * 16, 256>>>(reinterpret_cast<const f4_t*>(a), reinterpret_cast<f4_t*>(b), n4);
        }));
        HIPCHK(hipGetLastError());
        if (read_gbps) *read_gbps = (double)bytes * reps / tr / 1e9;
        if (copy_gbps) *copy_gbps = 2.0 * (double)bytes * reps / tc / 1e9;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipFree(a);
        (void)hipFree(b);
        (void)hipFree(o);
    });
}

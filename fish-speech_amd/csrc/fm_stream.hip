// fm_stream.hip -- the measured HBM stream peak the bench line quotes beside the vendor figure
// (SURVEY.md §8d): a non-temporal read-only stream and a float4 copy over buffers far larger than
// the 256 MiB MALL, HIP events around `reps` launches.  Not on any decode path.
#include "fm_common.h"
#include "fm_runtime.h"

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
        const double tr = time([&] {
            stream_read_kernel<4><<<grid, 256>>>(reinterpret_cast<const f4_t*>(a), n4, reinterpret_cast<float*>(o));
        });
        const double tc = time([&] {
            stream_copy_kernel<<<grid, 256>>>(reinterpret_cast<const f4_t*>(a), reinterpret_cast<f4_t*>(b), n4);
        });
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

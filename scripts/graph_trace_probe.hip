// Developer probe: does rocprofv3 --kernel-trace survive a hipGraph launch on /opt/rocm's HIP
// runtime, for kernels shaped like libfishmi's (by-value argument structs of 64 B .. 2 KiB, dynamic
// LDS past 64 KiB)?  hipcc --offload-arch=gfx950 -O2 scripts/graph_trace_probe.hip -o scripts/graph_trace_probe
// Usage: graph_trace_probe [variant]  (0 all kernels, 1 small args only, 2 big args, 3 big LDS,
// 4 a device-to-device copy node, 5 a memset node, 6 a copy into pinned host memory) [graph launches]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int B> struct Args {
    float* out;
    int v;
    char pad[B - 12];
};
template <int B> __global__ void k_args(Args<B> a) {
    if (threadIdx.x == 0 && blockIdx.x == 0) a.out[0] += (float)a.v + (float)a.pad[B - 13];
}
__global__ void k_lds(float* out) {
    extern __shared__ float sm[];
    sm[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) out[1] += sm[255];
}
#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            printf("%s -> %s\n", #x, hipGetErrorString(e));                          \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

int main(int argc, char** argv) {
    const int variant = argc > 1 ? atoi(argv[1]) : 0;
    float* d;
    CK(hipMalloc(&d, 64));
    CK(hipMemset(d, 0, 64));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_lds), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    Args<64> a64{d, 1, {}};
    Args<464> a464{d, 2, {}};
    Args<1920> a1920{d, 3, {}};
    float* hp = nullptr;
    CK(hipHostMalloc(&hp, 64));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 50; ++i) {
        if (variant == 0 || variant == 1) k_args<64><<<256, 256, 0, s>>>(a64);
        if (variant == 0 || variant == 2) {
            k_args<464><<<256, 256, 0, s>>>(a464);
            k_args<1920><<<256, 256, 0, s>>>(a1920);
        }
        if (variant == 0 || variant == 3) k_lds<<<256, 256, 100 * 1024, s>>>(d);
        if (variant == 4) {
            k_args<64><<<256, 256, 0, s>>>(a64);
            CK(hipMemcpyAsync(d + 8, d, 16, hipMemcpyDeviceToDevice, s));
        }
        if (variant == 5) {
            k_args<64><<<256, 256, 0, s>>>(a64);
            CK(hipMemsetAsync(d + 8, 0, 16, s));
        }
        if (variant == 6) {
            k_args<64><<<256, 256, 0, s>>>(a64);
            CK(hipMemcpyAsync(hp, d, 16, hipMemcpyDeviceToHost, s));
        }
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    const int launches = argc > 2 ? atoi(argv[2]) : 3;
    for (int r = 0; r < launches; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float h[2];
    CK(hipMemcpy(h, d, 8, hipMemcpyDeviceToHost));
    printf("variant %d ok: %.0f %.0f\n", variant, h[0], h[1]);
    return 0;
}

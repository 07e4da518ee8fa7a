// Probe: the row-major dot product on v_mfma_f32_16x16x32_bf16 (A = a 1 KiB fragment of one weight
// row, lane l holding k 8l..8l+7; B = the input chunk laid out the same way): is the trace of C the
// fragment's dot product, and is C's diagonal where the pass kernel's flush reads it?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>
#include <cstring>
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

__global__ void k(const uint16_t* w, const uint16_t* x, int nfrag, float* out, float* cdump) {
    const int lane = threadIdx.x;
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    const u32x4_t zf = {0u, 0u, 0u, 0u};
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %1, 0" : "+v"(acc) : "v"(zf));
    for (int f = 0; f < nfrag; ++f) {
        u32x4_t a = *reinterpret_cast<const u32x4_t*>(w + f * 512 + lane * 8);
        u32x4_t b = *reinterpret_cast<const u32x4_t*>(x + f * 512 + lane * 8);
        asm volatile("s_waitcnt vmcnt(0)\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(acc));
    for (int i = 0; i < 4; ++i) cdump[lane * 4 + i] = acc[i];
    const int dsel = (lane & 15) - 4 * (lane >> 4);
    float d = dsel == 0 ? acc[0] : (dsel == 1 ? acc[1] : (dsel == 2 ? acc[2] : (dsel == 3 ? acc[3] : 0.f)));
    for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o);
    if (lane == 0) out[0] = d;
}

static float bf(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); return f; }

int main() {
    const int nf = 5;
    std::vector<uint16_t> w(nf * 512), x(nf * 512);
    uint32_t s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)((s >> 9) & 0xffff) / 65536.0f - 0.5f; };
    auto tob = [](float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)(u >> 16); };
    double ref = 0;
    for (int i = 0; i < nf * 512; ++i) { w[i] = tob(rnd()); x[i] = tob(rnd()); ref += (double)bf(w[i]) * bf(x[i]); }
    uint16_t *dw, *dx; float *dout, *dc;
    hipMalloc(&dw, w.size() * 2); hipMalloc(&dx, x.size() * 2); hipMalloc(&dout, 4); hipMalloc(&dc, 256 * 4);
    hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dw, dx, nf, dout, dc);
    float out, c[256];
    hipMemcpy(&out, dout, 4, hipMemcpyDeviceToHost);
    hipMemcpy(c, dc, 256 * 4, hipMemcpyDeviceToHost);
    double tr = 0;  // trace under the assumed layout D[4*(l/16)+i][l%16]
    for (int l = 0; l < 64; ++l) for (int i = 0; i < 4; ++i) if (4 * (l / 16) + i == l % 16) tr += c[l * 4 + i];
    printf("ref %.6f  kernel %.6f  host-trace %.6f  (%s)\n", ref, out, tr, fabs(out - ref) < 1e-3 * (1 + fabs(ref)) ? "OK" : "MISMATCH");
    return 0;
}

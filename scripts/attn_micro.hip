// Developer microbenchmark: pass_attn4 (fm_pass.hip) alone on one idle CU, 1 / 4 / 8 waves,
// cycles per call.  hipcc --offload-arch=gfx950 -O3 -I../include -Icsrc scripts/attn_micro.hip
#include "../fish-speech_amd/csrc/fm_pass.hip"
#include <cstdio>

__global__ void attn_micro(int cpos, int nwaves, unsigned long long* out, bf16_t* kc, bf16_t* vc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
    const int nh = 32, nkv = 8, hd = 128;
    bf16_t* raw = reinterpret_cast<bf16_t*>(sm);                  // 48 heads x 128
    bf16_t* kvs = raw + (nh + 2 * nkv) * hd;                       // [8][2][15][128]
    bf16_t* qn = kvs + nkv * 2 * 15 * hd;
    bf16_t* kn = qn + hd;
    float* tab = reinterpret_cast<float*>(kn + hd);
    bf16_t* outp = reinterpret_cast<bf16_t*>(tab + hd);
    for (int i = threadIdx.x; i < (nh + 2 * nkv) * hd; i += blockDim.x) raw[i] = f2bf(0.01f * (i % 97));
    for (int i = threadIdx.x; i < nkv * 2 * 15 * hd; i += blockDim.x) kvs[i] = f2bf(0.02f * (i % 89));
    for (int i = threadIdx.x; i < hd; i += blockDim.x) {
        qn[i] = f2bf(1.0f);
        kn[i] = f2bf(1.0f);
        tab[i] = (i & 1) ? 0.5f : 0.8f;
    }
    __syncthreads();
    auto off = [](const void* p) { return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)p; };
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w >= nwaves) return;
    AttnLds ao{off(raw), off(kvs), off(qn), off(kn), off(tab), off(outp + w * 4 * hd)};
    const unsigned long long t0 = __builtin_readcyclecounter();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int rep = 0; rep < 8; ++rep)
        pass_attn4(nh, nkv, hd, cpos, 1, 1e-6f, 0.088f, (4 * w) % nh, lane, ao, kc, vc, (size_t)16 * hd, false);
    const unsigned long long t1 = __builtin_readcyclecounter();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        out[2 * w] = (t1 - t0) / 8;
        out[2 * w + 1] = (r1 - r0) / 8;
    }
}

FmTuning& fm_tuning() {
    static FmTuning t;
    return t;
}

int main() {
    unsigned long long* d;
    bf16_t *kc, *vc;
    (void)hipMalloc(&d, 64 * sizeof(unsigned long long));
    (void)hipMalloc(&kc, 1 << 20);
    (void)hipMalloc(&vc, 1 << 20);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_micro), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int nw : {1, 4, 8})
        for (int cpos : {1, 5, 9}) {
            attn_micro<<<1, 512, 100 * 1024>>>(cpos, nw, d, kc, vc);
            unsigned long long h[16];
            (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
            printf("waves %d cpos %d: wave0 %llu cycles, %.2f us per call\n", nw, cpos, h[0], h[1] / 100.0);
        }
    return 0;
}

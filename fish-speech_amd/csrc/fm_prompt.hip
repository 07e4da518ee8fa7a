// fm_prompt.hip -- prompt-chunk linears at 32 < R <= 64 rows (bf16): one weight pass for every row.
//
// A prompt chunk (the prefill of a short prompt: config 2's 64 tokens, a speaker turn's text) runs
// each TransformerBlock linear (llama.py:838-843, 883-890, 978-986) on R activation rows.  At
// R <= 64 that is a weight stream, not a GEMM: 2 R flops per weight byte.  The codec's LDS-tiled
// conv GEMMs (fm_codec_kernels.hip) tile M = 128 rows x 96-128 columns and stream the 7.3 GB of
// S2-Pro weights at about 1.15 TB/s there (profiles/r06_prefill64_kernels.md).
//
// Here each wave owns one 16-row weight tile and streams its fragments of the packed layout
// (fm_kernels.h: 1 KiB of contiguous HBM per 16 x 32 fragment, non-temporal) through a two-set
// register ring, 8 k-steps ahead.  The R activation rows are staged through LDS in 128-k chunks
// (double-buffered, LDS-only barriers, so the weight loads stay in flight across them) and serve as
// the MFMA B operands of all 64 rows: 4 accumulators per wave.  Block = 4 waves = 64 weight rows.
// The K range is cut into ks slices (grid y) so the grid fills the chip; each slice writes raw fp32
// partials to the conv split-K slab layout [ks][R][N], and conv_splitk_epi_kernel applies the
// epilogue: round(sum of slices + bias), the residual, the store.  The fp32 sum over slices runs in
// slice order, each slice's MFMA chain in k order.  An unsliced w1 || w3 (act set) applies the
// interleaved SwiGLU itself (no slab, no epilogue launch; swiglu_i8_kernel's roundings).
//
// Measured forms that lost (profiles/r06_prompt_skinny_v3_trace.md, 64-token prefill): loading the
// activation chunks two ahead (6.88 vs 6.57 ms), staging a whole <= 20-step slice at once with a
// 16-deep ring (7.31 ms: 82 KiB of LDS leaves one block per CU), and no LDS at all -- each wave
// loading its 4 activation fragments per k-step from L2 beside its weight fragment (10.03 vs
// 6.05 ms: 4x the weight bytes through L2; w1 || w3 92 vs 34 us, profiles/r06_prompt_skinny_l2direct_trace.md).
// Neutral or slower: 8-step chunks (6.15 vs 6.04 ms, profiles/r06_prompt_chunk8_trace.md), grid
// targets of 384-1024 blocks (6.04-6.30 ms, profiles/r06_prompt_blocks_sweep.txt), and a third weight
// set in the ring (6.25 vs 6.08 ms; w1 || w3 38.9 vs 34 us).
#include "fm_codec.h"
#include "fm_frag.h"
#include "fm_kernels.h"
#include "fm_runtime.h"

namespace {

constexpr int SK_CK = 128;          // k per staged activation chunk (4 MFMA k-steps)
constexpr int SK_XS = SK_CK + 8;    // LDS row stride in bf16 (272 B: 16-B row reads without bank conflicts)

// grid (ceil(N / 64), ks), 256 threads
__global__ __launch_bounds__(256) void prompt_skinny_kernel(PromptSkinnyArgs a) {
    using F = Frag<bf16_t>;
    __shared__ __attribute__((aligned(16))) bf16_t xs[2][64][SK_XS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ntile = (a.N + 15) / 16;
    const int tile = blockIdx.x * 4 + wave;
    const bool live = tile < ntile;
    const int nks = a.K / 32;                    // k-steps of the whole row
    const int kps = nks / (int)gridDim.y;        // k-steps of this slice (host: divides)
    const int s0 = (int)blockIdx.y * kps;
    const int nch = (kps + 3) / 4;
    const bf16_t* wb = a.w + ((size_t)(live ? tile : ntile - 1) * nks + s0) * 512;
    // ---- activation chunk c -> registers: 64 rows x 128 k = 1024 pieces of 16 B, 4 per thread
    u32x4_t xr[4];
    auto xload = [&](int c) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int piece = (int)threadIdx.x + 256 * i;
            const int row = piece >> 4, kq = piece & 15;
            const int kl = 128 * c + 8 * kq;  // k within the slice
            const bool ok = row < a.R && kl < 32 * kps;
            xr[i] = F::load_masked(a.x + (size_t)(ok ? row : 0) * a.ldx + 32 * s0 + (ok ? kl : 0), ok);
        }
    };
    auto xstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int piece = (int)threadIdx.x + 256 * i;
            *reinterpret_cast<u32x4_t*>(&xs[buf][piece >> 4][8 * (piece & 15)]) = xr[i];
        }
    };
    // ---- weight ring: set A holds the even chunk's 4 k-steps, set B the odd chunk's
    u32x4_t wa[4], wbq[4];
    auto wload = [&](u32x4_t (&w)[4], int c) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int st = 4 * c + q;
            w[q] = F::load_w<true>(wb + (size_t)(st < kps ? st : 0) * 512, lane);
        }
    };
    f32x4_t acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    xload(0);      // the first activation chunk goes out ahead of the ring (in-order vmcnt)
    wload(wa, 0);
    if (nch > 1) wload(wbq, 1);
    xstore(0);
    lds_barrier();
    auto chunk = [&](u32x4_t (&w)[4], int c) {
        if (c + 1 < nch) xload(c + 1);  // next chunk's rows in flight under this chunk's MFMAs
        const int buf = c & 1;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (4 * c + q < kps) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const F::f xb = F::load(&xs[buf][16 * t + (lane & 15)][32 * q + 8 * (lane >> 4)]);
                    acc[t] = F::mma(w[q], xb, acc[t]);
                }
            }
        }
        if (c + 2 < nch) wload(w, c + 2);  // the set is free: refill it two chunks ahead
        if (c + 1 < nch) xstore(buf ^ 1);  // that buffer's previous chunk was finished before the last barrier
        lds_barrier();
    };
    for (int c = 0; c < nch; c += 2) {
        chunk(wa, c);
        if (c + 1 < nch) chunk(wbq, c + 1);
    }
    if (a.act) {  // one slice: act[r][8 tile + 4 (lane >> 4) + j] = round(round(silu(g)) * u), g the gate
        // row 16 tile + 4 (lane >> 4) + j (lanes 0-31), u the up row 8 further (lane + 32)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int r = 16 * t + (lane & 15);
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float g = rnd<bf16_t>(acc[t][j]);
                const float u = rnd<bf16_t>(__shfl_xor(acc[t][j], 32));
                o[j] = rnd<bf16_t>(rnd<bf16_t>(g / (1.0f + expf(-g))) * u);
            }
            if (live && lane < 32 && r < a.R) {
                bf16_t* d = a.act + (size_t)r * a.lda + 8 * tile + 4 * (lane >> 4);
#pragma unroll
                for (int j = 0; j < 4; ++j) st(d, j, o[j]);
            }
        }
        return;
    }
    if (!live) return;
    // lane: weight rows 16 tile + 4 (lane >> 4) + j, activation row 16 t + (lane & 15)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int r = 16 * t + (lane & 15);
        if (r < a.R)
            *reinterpret_cast<f32x4_t*>(a.slab + ((size_t)blockIdx.y * a.R + r) * a.N + 16 * tile + 4 * (lane >> 4)) = acc[t];
    }
}

// Fully unrolled form (fm_tune prompt_unroll): NCH chunks as straight-line code, so no load is pending
// across a loop back edge (where the compiler drains vmcnt), with each chunk's activation rows
// loaded two chunks ahead.  Same MFMA chains in the same k order: bit-identical partials.
template <int NCH>
__global__ __launch_bounds__(256) void prompt_skinny_unrolled_kernel(PromptSkinnyArgs a) {
    using F = Frag<bf16_t>;
    __shared__ __attribute__((aligned(16))) bf16_t xs[2][64][SK_XS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ntile = (a.N + 15) / 16;
    const int tile = blockIdx.x * 4 + wave;
    const bool live = tile < ntile;
    const int nks = a.K / 32;
    const int kps = nks / (int)gridDim.y;  // host: (kps + 3) / 4 == NCH
    const int s0 = (int)blockIdx.y * kps;
    const bf16_t* wb = a.w + ((size_t)(live ? tile : ntile - 1) * nks + s0) * 512;
    u32x4_t xr[2][4];
    auto xload = [&](int set, int c) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int piece = (int)threadIdx.x + 256 * i;
            const int row = piece >> 4, kq = piece & 15;
            const int kl = 128 * c + 8 * kq;
            const bool ok = row < a.R && kl < 32 * kps;
            xr[set][i] = F::load_masked(a.x + (size_t)(ok ? row : 0) * a.ldx + 32 * s0 + (ok ? kl : 0), ok);
        }
    };
    auto xstore = [&](int set, int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int piece = (int)threadIdx.x + 256 * i;
            *reinterpret_cast<u32x4_t*>(&xs[buf][piece >> 4][8 * (piece & 15)]) = xr[set][i];
        }
    };
    u32x4_t w[2][4];
    auto wload = [&](int set, int c) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int st = 4 * c + q;
            w[set][q] = F::load_w<true>(wb + (size_t)(st < kps ? st : 0) * 512, lane);
        }
    };
    f32x4_t acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    xload(0, 0);
    if (NCH > 1) xload(1, 1);
    wload(0, 0);
    if (NCH > 1) wload(1, 1);
    xstore(0, 0);
    lds_barrier();
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        if (c + 2 < NCH) xload(c & 1, c + 2);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (4 * c + q < kps) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const F::f xb = F::load(&xs[c & 1][16 * t + (lane & 15)][32 * q + 8 * (lane >> 4)]);
                    acc[t] = F::mma(w[c & 1][q], xb, acc[t]);
                }
            }
        }
        if (c + 2 < NCH) wload(c & 1, c + 2);
        if (c + 1 < NCH) xstore((c + 1) & 1, (c + 1) & 1);
        lds_barrier();
    }
    if (a.act) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int r = 16 * t + (lane & 15);
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float g = rnd<bf16_t>(acc[t][j]);
                const float u = rnd<bf16_t>(__shfl_xor(acc[t][j], 32));
                o[j] = rnd<bf16_t>(rnd<bf16_t>(g / (1.0f + expf(-g))) * u);
            }
            if (live && lane < 32 && r < a.R) {
                bf16_t* d = a.act + (size_t)r * a.lda + 8 * tile + 4 * (lane >> 4);
#pragma unroll
                for (int j = 0; j < 4; ++j) st(d, j, o[j]);
            }
        }
        return;
    }
    if (!live) return;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int r = 16 * t + (lane & 15);
        if (r < a.R)
            *reinterpret_cast<f32x4_t*>(a.slab + ((size_t)blockIdx.y * a.R + r) * a.N + 16 * tile + 4 * (lane >> 4)) = acc[t];
    }
}

}  // namespace

int prompt_skinny_ks(int N, int K, int target) {
    const int groups = (N + 63) / 64, nks = K / 32;
    int ks = 0;
    for (int d = 1; d <= nks; ++d) {
        if (nks % d || nks / d < 8) continue;
        ks = d;
        if ((long long)groups * d >= target) break;
    }
    return ks;  // 0: K too short for a slice of 8 k-steps
}

void launch_prompt_skinny(hipStream_t s, const PromptSkinnyArgs& a, int ks) {
    FMCHECK(a.R > 0 && a.R <= 64 && a.K % 32 == 0 && ks >= 1 && (a.K / 32) % ks == 0 && a.N % 16 == 0 && a.slab &&
                a.ldx % 8 == 0 && ((uintptr_t)a.x & 15) == 0,
            "prompt skinny GEMM: R <= 64, K a multiple of 32 split evenly, N a multiple of 16, 16-B rows, slab set");
    const dim3 grid((a.N + 63) / 64, ks);
    const int nch = (a.K / 32 / ks + 3) / 4;
    if (fm_tuning().prompt_unroll) {
        switch (nch) {
            case 4: prompt_skinny_unrolled_kernel<4><<<grid, 256, 0, s>>>(a); return;
            case 5: prompt_skinny_unrolled_kernel<5><<<grid, 256, 0, s>>>(a); return;
            case 10: prompt_skinny_unrolled_kernel<10><<<grid, 256, 0, s>>>(a); return;
            case 20: prompt_skinny_unrolled_kernel<20><<<grid, 256, 0, s>>>(a); return;
            default: break;
        }
    }
    prompt_skinny_kernel<<<grid, 256, 0, s>>>(a);
}

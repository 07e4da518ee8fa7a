// fm_codec.h -- kernel argument blocks of the modded-DAC decode path (fm_codec_kernels.hip).
#pragma once
#include "fm_kernels.h"

// epilogue flags of conv_gemm_kernel (combined bitwise)
enum {
    CE_BIAS = 1,      // + bias[co]
    CE_GELU = 2,      // exact-erf GELU (nn.GELU, rvq.py:165)
    CE_RES = 4,       // y = res + gamma[co] * y (LayerScale / ConvNeXt gamma) or res + y
    CE_GAMMA = 8,     // with CE_RES: scale by gamma before the add
    CE_STORE = 16,    // store y to out
    CE_SNAKE = 32,    // store snake(y, alpha2) to out2 (the next stage's input)
    CE_TANH = 64,     // y = tanh(y) (decoder output, modded_dac.py:795)
    CE_F32OUT = 128,  // out is fp32 (final waveform)
    CE_SWIGLU = 256,  // split-K epilogue only: out[t][n] = round(round(silu(y[n])) * y[Co/2 + n]) for
                      // n < Co/2 (W1 and W3 of a FeedForward as one GEMM, modded_dac.py:316-317)
    CE_ROPE = 512,    // split-K epilogue only: RoPE on channels [0, rope_nqk) (q and k heads of a wqkv
                      // output) at position t + rope_pos0, as rope_qk_kernel does it
    CE_NORM = 1024,   // split-K epilogue only (one phase, Co % 512 == 0, Co <= 2048): out2 = RMSNorm(y)
                      // with weight normw, the next layer's / stage's norm, as rmsnorm_wave_kernel does it
    CE_SWIGLU8 = 2048,  // split-K epilogue only: CE_SWIGLU over the row-interleaved W1 || W3 (8 rows of
                        // W1, then the same 8 of W3): out[t][8g + e] = round(round(silu(y[16g + e])) *
                        // y[16g + 8 + e]), as swiglu_i8_kernel does it on the stored output (no bias)
};

// out[t_out][co] (time-major, ld = ldo) with t_out = tq * stride + phase, tq in [0, Lq):
//   y = sum_{tap, ci} Wp[phase][co][tap*Ci + ci] * x[tq - shift[tap]][ci]   (x time-major, ldx)
// Wp packed per phase (fm_kernels.h layout), rows = Co, cols = ntaps*Ci.
template <typename T> struct ConvArgs {
    const T* x;
    int ldx, Ci, Lq, Lx;       // input rows available: [0, Lx); rows < 0 are causal zeros
    const T* w;                // packed, phase-major
    size_t wphase;             // elements per phase
    int Co, ntaps, stride, nphase;
    int shift[8];              // per tap
    int shift0, shiftd;        // shift[tap] = shift0 + tap * shiftd (set and checked by the launcher)
    const T* bias;
    const T* gamma;
    const T* res;              // residual [t_out][co], ldr
    int ldr;
    const T* alpha2;           // snake alpha for out2
    const float* ialpha2;      // 1 / (alpha2 + 1e-9) per channel (fp32, computed once at load)
    void* out;
    int ldo;
    T* out2;
    int ldo2;
    int flags;
    int lo;                    // lowest input row read (<= 0): rows [lo, 0) are the carried causal
                               // context of a streamed chunk (buffer prefix), 0 = causal zeros
    float* slab;               // split-K workspace (launcher): fp32 partials [ksplit][nphase][Lq][Co]
    size_t slab_cap;           // its capacity in floats (0: no split-K)
    int ksplit;                // set by the launcher
    const float* rope = nullptr;  // CE_ROPE: the (cos, sin) table [pos][hd / 2][2]
    int rope_pos0 = 0, rope_nqk = 0, rope_hd = 0;
    const T* normw = nullptr;     // CE_NORM: the RMSNorm weight [Co] and eps
    float norm_eps = 0.f;
};

// One decoder ResidualUnit (modded_dac.py:599-620) in one launch, bf16, C in {96, 192, 384}:
//   h   = round(snake_a2(round(conv7_dil(x) + b7)))            (the k7 conv's output, LDS only)
//   y   = round(res + round(conv1(h) + b1))                    (res: stored back when store_res)
//   out2 = round(snake_an(y))                                  (the next unit's / stage's input)
// x = snake_a0 of the unit input, time-major [t][C], rows [lo, 0) the carried context of a streamed
// chunk (buffer prefix), rows < lo causal zeros.  out2 must not alias x (neighbour tiles read x's
// rows behind them).  The k-steps and their fp32 accumulation order are conv_gemm2_kernel's, so
// the result is bit-identical to the two-launch form.
struct ResUnitArgs {
    const bf16_t* x;
    int L, lo, dil;
    const bf16_t* w7;    // packed k7 weights (fm_kernels.h fragment order, K = 7 C as [tap][ci])
    const bf16_t* b7;
    const bf16_t* a2;
    const float* ia2;
    const bf16_t* w1;    // packed k1 weights (K = C)
    const bf16_t* b1;
    bf16_t* res;         // residual [L][C], read, and written back when store_res
    int store_res;
    const bf16_t* an;
    const float* ian;
    bf16_t* out2;        // [L][C]
    const bf16_t* zeros; // >= 16 zero bytes: the LDS-DMA source of rows outside [lo, L)
};
// false: shape not covered (C not 96 / 192 / 384, dil > 9) -- the caller runs the two-launch form
bool launch_resunit(hipStream_t s, const ResUnitArgs& a, int C);
void resunit_init();

struct RvqPtrs {
    const float* cb[16];  // codebooks [size][cd]
    const float* w[16];   // folded out_proj [D][cd]
    const float* b[16];   // out_proj bias [D]
};

template <typename T> void launch_conv_gemm(hipStream_t s, const ConvArgs<T>& a);
// the split-K epilogue alone over a.ksplit slabs in a.slab (the prompt skinny GEMM's finisher)
template <typename T> void launch_conv_epi(hipStream_t s, const ConvArgs<T>& a);
template <typename T> void launch_snake_inv(hipStream_t s, const T* alpha, int64_t n, float* ialpha);
// encode side (fm_codec_encode)
struct VqEncPtrs {
    const float* wi[16];  // folded in_proj [cd][D]
    const float* bi[16];  // in_proj bias [cd]
    const float* cb[16];  // codebooks [cbn][cd]
    const float* wo[16];  // folded out_proj [D][cd]
    const float* bo[16];  // out_proj bias [D]
    int cbn[16];
};
void launch_vq_encode(hipStream_t s, float* r, int Tn, int D, int nst, int cd, const VqEncPtrs& p, int32_t* codes);
template <typename T> void launch_snake(hipStream_t s, const T* x, int C, size_t n, const T* alpha, T* y);
template <typename T> void launch_audio8(hipStream_t s, const float* a, int64_t n, int64_t npad, T* y);
template <typename T> void launch_silu_mul(hipStream_t s, const T* g, T* y, size_t n);
template <typename T>
void launch_rvq_decode(hipStream_t s, const int32_t* codes, int Tn, int nq1, int sem, int cbs, int cd,
                       const RvqPtrs& p, int D, T* z);
// lo <= 0: rows [lo, 0) of x are carried causal context (streamed chunk), else causal zeros
template <typename T>
void launch_dwconv_ln(hipStream_t s, const T* x, int L, int D, const T* dw, const T* db, const T* lw,
                      const T* lb, T* y, int lo = 0);
// pos0: absolute position of row 0 (streamed chunk)
template <typename T>
void launch_rope_qk(hipStream_t s, T* qkv, int Tn, int H, int hd, const float* tab, int pos0 = 0);
// npre: rows [-npre, 0) of qkv hold the carried (post-RoPE) keys / values of earlier frames
template <typename T>
void launch_window_attn(hipStream_t s, const T* qkv, int Tn, int H, int hd, int window, T* out, int npre = 0);
void launch_wn_fold(hipStream_t s, const float* g, const float* v, int rows, int per, float* w);
template <typename T>
void launch_conv_weight(hipStream_t s, const float* w, int kind, int Ci, int Co, int k, int st_, T* out);

// fm_kernels.h -- kernel argument blocks and launchers (host <-> device seam of libfishmi).
#pragma once
#include <algorithm>
#include "fm_common.h"

enum { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_F32 = 3 };

// Packed weight layout used by every GEMM here: a [N][K] nn.Linear weight is stored as
// [ceil(N/16)][K/32] blocks of 512 elements, each block holding one MFMA 16x32 A-fragment in
// lane order (bf16: lane l's 8 elements at l*8; fp32: elements 0-3 at l*4, 4-7 at 256+l*4), so
// every wave-load instruction reads 1 KB of contiguous memory.
// act[r][j] = round(silu(t[r][16*(j/8) + j%8])) * t[r][16*(j/8) + 8 + j%8]: SwiGLU over the output of
// the row-interleaved W1||W3 (batched path)
template <typename T> void launch_swiglu_i8(hipStream_t s, const T* t, int ldt, T* act, int lda, int inter, int R);
template <typename T> void launch_pack(hipStream_t s, const T* src, int N, int K, T* dst);
// Weight-only int8 (tools/llama/quantize.py:22-52, 190-232).
// quant_rows: per row n of a row-major [N][K] weight w (values as T): m = max(-min(min w, 0),
// max(max w, 0)), s = max(m / 127.5, FLT_EPSILON) in fp32, q = clamp(rint(w / s), -128, 127);
// writes q (int8 row-major), scale[n] = bf16(s) (held in T), and rewrites w with T(q) (exact).
template <typename T> void launch_quant_rows(hipStream_t s, T* w, int N, int K, int8_t* q, T* scale);
// int8 row-major -> T row-major (exact), for the kernels that read T fragments of q
template <typename T> void launch_i8_to(hipStream_t s, const int8_t* q, int64_t n, T* dst);
// int8 row-major [N][K] -> the int8 decode-GEMV layout: [ceil(N/16)][K/64] units of 1 KiB, lane l
// (row l & 15, k-offset 8 * (l >> 4)) holding 8 bytes of k-step 2u then 8 bytes of k-step 2u + 1
void launch_pack_q8(hipStream_t s, const int8_t* src, int N, int K, int8_t* dst);
// Weight-only int4, groupwise affine (tools/llama/quantize.py:57-160, WeightOnlyInt4QuantHandler
// :352-418), bf16 only.  quant4: per (row, group of gs along K) of a row-major bf16 [N][K] w, the
// reference's group_quantize_tensor in its bf16 arithmetic (every op computed in fp32 and rounded to
// bf16, as torch does): scale = bf16(bf16(max - min) clamped to bf16(1e-6) / 15), zero =
// bf16(min + scale * 8), q = clamp(round_half_even(bf16(bf16(w - (zero - scale * 8)) / scale)), 0, 15);
// writes q (one code per byte, row-major), sz[n][g] = scale bits | zero bits << 16, and rewrites w
// with bf16(fma(q - 8, scale, zero)) (the dequantised weight every bf16 kernel then reads).
void launch_quant4(hipStream_t s, bf16_t* w, int N, int K, int gs, uint8_t* q, uint32_t* sz);
// codes row-major [N][K] -> the int4 decode-GEMV layout: [ceil(N/16)][K/128] units of 1 KiB, lane l
// (row l & 15, k-offset 8 * (l >> 4)) holding word j = the 8 codes of k-step j of the unit, k =
// 128 u + 32 j + 8 (l >> 4) + e: even e at bits 2e (e / 2 nibbles up), odd e at bits 16 + 2(e - 1),
// so (word >> 4p) & 0x000F000F is the pair (e = 2p, 2p + 1) in bf16 mantissa position
// sz [N][K/gs] -> [ceil(N/16)][K/128][16 rows] (gs a multiple of 128: one group per unit)
void launch_pack_q4(hipStream_t s, const uint8_t* q, int N, int K, uint8_t* dst);
// int4 codes (one per byte) [N][K] -> row-major words [N][K / 8]: word j = codes 8j .. 8j+7, the even
// ones in the low half at nibble e / 2, the odd ones in the high half (fm_rowgemv.hip QM 2)
void launch_pack_q4_rows(hipStream_t s, const uint8_t* q, int N, int K, uint32_t* dst);
void launch_pack_sz4(hipStream_t s, const uint32_t* sz, int N, int K, int gs, uint32_t* dst);

template <typename T> struct LinearArgs {
    const T* W;      // [N(padded to 16)][K] row-major (nn.Linear layout)
    const T* W2;     // second weight for EPI_SWIGLU (w3), same shape
    const T* bias;   // [N] or null
    const T* X;      // [R][ldx]
    int ldx, R, N, K;
    T* Y;            // [R][ldy]
    int ldy;
    const T* res;    // residual [R][ldr] (EPI_RESID)
    int ldr;
    float* Yf;       // fp32 output (EPI_F32)
    // split-K (gridDim.y > 1, R <= 16 * NCG): fp32 tile partials [ksb][NACC][R][N] and one arrival
    // counter per 16-row tile (zero between launches; the last-arriving block resets it)
    float* part = nullptr;
    int* tickets = nullptr;
    // weight-only int8 (tools/llama/quantize.py WeightOnlyInt8Linear): W holds the int8 values
    // exactly and every output is round(round(acc) * wscale[n]) (not with EPI_SWIGLU)
    const T* wscale = nullptr;
};

template <typename T> struct QkArgs {
    const T* qkv;    // [R][ldqkv]
    int ldqkv;
    const int* row_slot;
    const int* row_pos;
    int fixed_pos;   // >= 0: every row at this position (fast model)
    int nh, nkv, hd, qk_norm;
    float eps;
    const T* qn;
    const T* kn;
    const float* rope;  // [S][hd/2][2] (bf16-valued cos/sin)
    T* qout;         // [R][nh*hd]
    T* kc;
    T* vc;
    size_t slot_stride, layer_off;
    int S;
    // prompt chunks on the skinny GEMM: the QKV projection left qslab_kp fp32 K-slice slabs
    // [kp][R][ldqkv] (no bias) instead of qkv; the kernel reads round(sum + qbias) itself
    const float* qslab = nullptr;
    int qslab_kp = 1;
    const T* qbias = nullptr;
};

template <typename T> struct AttnArgs {
    const T* q;      // [R][nh*hd]
    const int* row_slot;
    const int* row_pos;
    const T* kc;
    const T* vc;
    size_t slot_stride, layer_off;
    int S, nh, nkv, hd, split, maxsplit;
    float scale;
    float* part;     // [R][nh][maxsplit][hd+2]
};

template <typename T> struct FastAttnArgs {
    const T* q;
    const int* row_slot;
    const T* kc;
    const T* vc;
    size_t slot_stride, layer_off;
    int S, nh, nkv, hd, cpos;
    float scale;
    T* out;
};

struct SlotParams {
    float temperature, top_p;
    int top_k, mask_im_end;
    uint64_t seed;
    int step;
    int force;  // teacher forcing (fm_llm_force): the samplers emit force_cols[slot] and tap their logits
};

struct SampleArgs {
    const float* logits;  // [R][ldl]
    int ldl, Nl;
    const int* row_slot;
    const SlotParams* sp;
    const int32_t* ras;   // [slot][ras_stride]
    int ras_stride, ras_enable;
    int slow, sb, se, im_end, cb, draw, col_idx;
    unsigned long long* dbg;  // developer timestamps (fm_tune "debug_ts")
    int32_t* cols;        // [R][ldc]
    int ldc;
    // teacher forcing (SlotParams.force): emitted tokens come from force_cols[slot][ldc] and the
    // logits row is copied to tap + slot * tap_ld (parity hook on the production decode graph)
    const int32_t* force_cols;
    float* tap;
    int tap_ld;
    int kth_fast;  // sample_fast_kernel: try the lane-maxima threshold before the radix search (launcher: fm_tune sampler_kth)
};

template <typename T>
void launch_embed(hipStream_t s, const int32_t* tok, int R, const T* emb, const T* cbemb, int d,
                  int C, int cb, int sb, int se, int scale, T* x, const int* row_slot);
template <typename T>
void launch_gather_rows(hipStream_t s, const int32_t* codes, int ldc, int col, const T* table,
                        int d, int rows, int R, T* x);
template <typename T>
void launch_rmsnorm(hipStream_t s, const T* x, int ldx, const T* w, int d, float eps, T* y,
                    int ldy, int R);
template <typename T> void launch_linear(hipStream_t s, const LinearArgs<T>& a, int epi);
constexpr size_t LINEAR_PART_CAP = (size_t)8 << 20;     // floats of split-K partials (= fm_llm skpart)
int linear_ksb(int N, int K, int R, int nacc, bool can_split);
template <typename T> void launch_qk_rope_cache(hipStream_t s, const QkArgs<T>& a, int R);
template <typename T>
void launch_attn(hipStream_t s, const AttnArgs<T>& a, int R, int nsplit, T* out, bool one_slot);  // one_slot: rows of one prompt
template <typename T> void launch_fast_attn(hipStream_t s, const FastAttnArgs<T>& a, int R);
void launch_finish(hipStream_t s, int R, const int* row_slot, int* row_pos, const int32_t* cols,
                   int ldc, int32_t* tok_in, int32_t* ras, int ras_stride, int C1, int update_ras,
                   SlotParams* sp);
template <typename T>
void launch_synth(hipStream_t s, T* dst, int64_t n, uint64_t seed, uint32_t tid, float center,
                  int log2_half);
template <typename T>
void launch_convert(hipStream_t s, const void* src, int src_bf16, int64_t n, T* dst);

// ---- decode weight-streaming path (fm_gemv.hip), R <= 8 rows --------------------------------
enum { PRO_PLAIN = 0, PRO_NORM = 1, PRO_PRENORM = 3, PRO_FATT = 4 };
// PRO_FATT (fast model, one row, cpos < 16): X' is the fast-model attention output, recomputed by
// every block from the raw QKV row and the cached K/V rows staged in LDS (llama.py:947-975), so
// the Wo GEMV needs no separate attention launch; blockIdx.x == 0 writes the new k / v of cpos.
enum { EPI_SLAB = 4, EPI_SLABFIN = 5, EPI_SWIGLU8 = 7 };
// EPI_SWIGLU8: W is the row-interleaved W1||W3 (each 16-row tile = 8 gate rows then the same 8 up
// rows, see pack_w13 in fm_llm.cpp); a tile yields 8 SwiGLU outputs, N = 2 * intermediate.

template <typename T> struct FastFusedArgs {
    const T* qkv;
    int ldqkv;
    const int* row_slot;
    int nh, nkv, hd, qk_norm;
    float eps;
    const T* qn;
    const T* kn;
    const float* rope;   // [C][hd/2][2]
    T* kc;
    T* vc;
    size_t slot_stride, layer_off;
    int S, cpos;         // S = num_codebooks (fast cache length)
    float scale;
    T* out;              // [R][nh*hd]
    unsigned long long* dbg;  // developer timestamps (fm_tune "debug_ts")
    float* qdbg = nullptr;    // per-op test hook (fm_op_qk_rope): q after qk-norm + RoPE [R][nh][hd]
    int nwb = 4;              // attn_fd: waves per block (4, 8 or 16; 16 nwb positions per pass)
    // batched frames (fm_tune bs_qkv_slab): the QKV projection left qslab_kp fp32 K-part slabs
    // [kp][R][ldqkv] (no bias) instead of qkv; the attention reads round(sum + qbias) itself
    const float* qslab = nullptr;
    int qslab_kp = 1;
    const T* qbias = nullptr;
    const int* row_pos = nullptr;  // fattn_wo_kernel: the frame's position (its hand-off tag)
};
template <typename T> struct GemvArgs {
    const T* W;
    const T* W2;             // EPI_SWIGLU: w3
    const T* bias;
    const T* X;              // [R][ldx] (or a table gathered by xidx)
    int ldx;
    const int32_t* xidx;     // optional row gather: X row = xidx[r*xidx_ld + xidx_col]
    int xidx_ld, xidx_col;
    int xidx_rows;           // rows of the gathered table: indices are clamped into it (0: unchecked)
    const int32_t* residx;   // optional row gather for res (same layout as xidx)
    const T* res;            // EPI_SLABFIN residual [R][ldr]
    int ldr;
    const float* ss_in;      // PRO_PRENORM: per-16-column-tile sums of squares of X [K/16][R]
    int ss_gran;             // PRO_PRENORM: 0 ss_in as above; 1 the statistic from the staged row itself (R == 1, whole K)
    const T* nw;             // norm weight [K]
    float eps;
    int R, N, K;
    T* Y;                    // EPI_STORE / EPI_SWIGLU [R][ldy]
    int ldy;                 // also the slab row stride for EPI_SLAB / EPI_F32
    float* Yf;               // EPI_F32 [R][ldy] | EPI_SLAB(FIN) partials [KSB][R][ldy]
    T* res_out;              // EPI_SLABFIN: x = round(res + round(sum of partials)) [R][ldro]
    int ldro;
    float* ss_out;           // EPI_SLABFIN: per-tile sums of squares of x [N/16][R]
    int* tickets;            // EPI_SLABFIN: per-tile arrival counters (zero between launches)
    T* xn_out;               // optional (ksb == 1): block (0,0) stores X' (normalised row) here
    int ldxo;
    unsigned long long* dbg; // developer timestamps (fm_tune "debug_ts"); null in production
    FastFusedArgs<T> att;    // PRO_FATT: the fast-model attention the prologue recomputes
    int fatt_off;            // PRO_FATT: byte offset of the attention staging area in LDS (launcher)
    // weight-only int8: Wq replaces W (packed [tiles][K/64][64 lanes][16 B], fm_kernels.h) and
    // each output is round(round(acc) * wscale[packed row]) (WeightOnlyInt8Linear, quantize.py:228-229)
    const unsigned char* Wq;
    const T* wscale;
    // weight-only int4 (bf16): Wq holds 4-bit codes ([tiles][K/128][64 lanes][16 B], launch_pack_q4)
    // and wsz each (tile, 128-k unit, row)'s group (scale, zero) as bf16 pairs (launch_pack_sz4)
    const uint32_t* wsz;
    int q4_xsum_off;  // int4: LDS byte offset of the per-(128-k unit, x row) sums (launcher)
    // optional KV prefetch (batch-1 QKV GEMV, fm_tune kv_prefetch): while the weights stream, the
    // cached K / V rows the next attention launch reads (positions 0 .. pos of row 0's slot) are
    // pulled into L2: block b loads kv head b % pf_nkv, which under round-robin workgroup placement
    // is the XCD that attention block (kv head h = XCD h) runs on.  Speed only, never correctness.
    const T* pf_kc;          // null: off
    const T* pf_vc;
    const int32_t* pf_slot;  // row 0's slot / position (device, as the attention reads them)
    const int32_t* pf_pos;
    size_t pf_slot_stride, pf_layer_off;
    int pf_S, pf_nkv, pf_hd;
    int dummy_tail;  // ring slots past the wave's run load one fixed fragment (else the run's last)
};
// developer knobs for the decode GEMV (fm_tune): weight load policy and split-K policy
struct FmTuning {
    int gemv_nt = 1;         // 1: non-temporal weight loads (each weight byte is read once a frame)
    int gemv_u = 8;          // weight fragments in flight per wave (2, 4 or 8)
    int gemv_wpb = 4;        // waves per block (4 or 8) sharing one 16-row tile
    int sampler_kth = 1;     // sample_fast_kernel: the K-th lane maximum as the wave threshold when its candidates fit (else the radix search)
    int sampler_fast = 1;    // 1: two-stage register top-K sampler, 0: LDS radix-select sampler
    int attn_cap = 32;       // slow decode attention rows per block cap (0: the LDS-budget maximum)
    int attn_wo = 0;         // 1: fast-model attention recomputed in the Wo GEMV's prologue (PRO_FATT, R == 1; measured 0.37 ms/frame slower)
    int ksb_blocks = 512;    // split K until the grid has at least this many blocks
    int batched_fused_attn = 1;  // batched decode (one row per slot): fused QK-norm/RoPE/KV-write attention kernels
    int attn_cap_batched = 128;  // rows per block of the batched decode attention (one row per slot)
    int linear_u32 = 4;      // linear_kernel weight fragments in flight per wave at 16 < R <= 32 (4 or 8)
    int linear_fill = 0;     // batched linear_kernel: split K until this many blocks (0: never; measured slower)
    int attn3 = 1;           // 1: slow decode attention on attn_dec3_kernel, 0: attn_decode2_kernel
    int attn_fd = 1;         // 1: slow decode attention on attn_fd_kernel (flash-decode splits) where eligible
    int fd_min = 32;         // attn_fd: minimum positions per split at R <= 8
    int fd_min_batched = 512;  // attn_fd: minimum positions per split at R > 8 (B=32: one split below 512)
    int fd_nw = 8;           // attn_fd at R <= 8: waves per block (4, 8 or 16) ...
    int fin_ksb = 0;         // batch-1 wo / w2 (EPI_SLABFIN) split-K factor (0: whole K whenever the x slice fits LDS)
    int fd_nw_batched = 4;   // attn_fd at R > 8: waves per block (4, 8 or 16)
    int fd_min16 = 256;      // ... and splits of at least this many positions (8 or 16 waves; below it
                             // one block per kv head, no cross-block combine)
    int prefill_attn = 1;    // 1: prompt-chunk attention on attn_prefill_kernel (bf16, head_dim 128, flash form)
    int prompt_gemm = 1;     // 1: prompt-chunk linears (R > 32) on the codec's LDS-tiled GEMM kernels
    int prompt_skinny = 1;      // prompt linears at 32 < R <= 64 rows (bf16) on prompt_skinny_kernel ...
    int prompt_skinny_blocks = 256;  // ... with K sliced until its 64-row blocks number >= this
    int prompt_unroll = 1;      // skinny prompt GEMM: the fully unrolled form (5 / 10 / 20-chunk slices)
    int prompt_qkv_slab = 1;    // skinny QKV: slabs summed by qk_rope_cache_kernel (no epilogue launch)
    int prompt_fin = 1;         // skinny wo / w2: slabs finished by finalize_norm with the next RMSNorm
    int prompt_swiglu = 1;      // skinny w1 || w3: the SwiGLU in its split-K epilogue (no separate launch)
    int prompt_ks_tiles = 384;  // prompt GEMM: split K until ceil(R/128) ceil(N/128) ks reaches this ...
    int prompt_ks_max = 8;      // ... or ks this (fp32 slabs + the conv split-K epilogue)
    int conv2 = 1;           // 1: codec GEMMs on the LDS-staged conv_gemm2_kernel, 0: conv_gemm_kernel
    int conv_splitk = 1;     // 1: small-grid codec GEMMs split K into fp32 slabs + a reduce/epilogue kernel
    int resunit_cfg = 1;     // resunit_kernel tile at 192 / 96 channels: 0 (BM 128 / 256, 8 time tiles per wave), 1 (BM 64 / 128, 4 tiles), 2 (128 / 128)
    int resunit_enc = 1;     // 1: the encoder's units (64 / 128 / 256 / 512 channels) fused as well
    int resunit_384 = 1;     // 1: the 384-channel stage's units fused too (BM 64, 8 waves)
    int codec_norm = 1;      // 1: the codec transformer's RMSNorms in the wo / w2 split-K epilogues (no rmsnorm launch)
    int codec_rope = 1;      // 1: the codec transformer's RoPE in the wqkv split-K epilogue (no rope_qk launch)
    int codec_swiglu = 1;    // 1: codec FeedForward W1 | W3 as one split-K GEMM with the SwiGLU epilogue
    int codec_fuse = 1;      // 1: decoder ResidualUnits at 96 / 192 / 384 channels as one resunit_kernel launch (k7 + k1)
    int bstream = 1;         // 1: batched decode linears (8 < R <= 32) on bstream_kernel (fm_bstream.hip)
    int bstream_kparts = 0;  // bstream EPI_SLAB K parts (0: by K)
    int bstream_nw = 0;      // bstream waves per block (0: 16 whole-K, 8 split-K)
    // ring slots past a wave's run (tail of the decode GEMV ring, bsacc tiles / steps a block does
    // not own): 0 re-load the run's last fragment, 1 one fixed fragment, 2 a fixed fragment per
    // (block, wave) over 256 of them.  B=1 frame 4.447 / 4.47 / 4.398 ms, B=32 6.51 / 6.44 / 6.42 ms
    int bs_dummy = 2;
    int gemv_dummy = 2;
    int bs_qkv_slab = 1;     // batched frames: QKV as K-part slabs summed by the attention (balanced
                             // grid: 384 tiles x 2 K parts over 256 CUs; B=32 frame 6.48 -> 6.33 ms)
    int fast_tail = 1;       // 1: codebook 0's fast pass stops its last layer after the K / V cache write (its output is discarded)
    int fkv_prefetch = 0;    // 1: the batch-1 fast-model QKV GEMV pulls the fast attention's cached rows into L2 too
    int kv_prefetch = 1;     // 1: the batch-1 QKV GEMV pulls the next attention's K / V rows into L2
    int bstream_chain = 0;   // 1: bsacc SLABFIN / PRENORM chain instead of finalize_norm launches (measured 6.31 -> 6.75 ms per B=32 frame)
    int bstream_acc = 1;     // 1: bsacc_kernel (per-tile register accumulators, one reduction at the end, balanced K parts); 0: bstream_kernel
    int rmsnorm_block = 0;   // 1: block-per-row RMSNorm (the pre-vectorisation kernel), 0: wave-per-row when shapes allow
    int ksb_balance = 0;     // 1: prefer grids that are whole multiples of 256 blocks (one per CU)
    int chain_max = 4;       // gemv_chain: GEMVs per launch at most (2..4)
    int chain_sleep = 4;     // gemv_chain: s_sleep argument between a waiting block's polls (1, 4 or 16)
    int gemv_chain = 0;      // 1: batch-1 decode runs wo -> w1||w3 -> w2 -> next qkv as one launch (gemv_chain_kernel)
    int bs_xfirst = 1;       // bsacc: X operands before the weight ring (B=32 frame 6.48 -> 6.36 ms)
    int bs_vec_epi = 1;      // bsacc: 4-row epilogue items (bit-identical to the scalar epilogue; B=32 frame 6.31 -> 6.18 ms)
    int bsacc_kparts = 0;    // developer: force the K parts of the batched split-K (slab) linears (0: bsacc_plan's pick)
    int q_u = 4;             // int8 / int4 decode GEMV: ring units in flight per wave (2, 4, 8, 16; int8 frame 3.79 -> 3.59 ms at 8 -> 4)
    int fin8 = 1;            // finalize_norm: all eight K parts' slab loads in one round trip (0: two batches of four)
    int fin_split = 0;       // batched finalize_norm: each row over this many blocks (0 / 1: one block per row)
    int int4_stream = 1;     // weight-only int4: 1 the batch <= 8 GEMVs stream the 4-bit codes, 0 the dequantised bf16 copy
    int fw_delay = 0;        // fattn_wo: FattnWoArgs::delay
    int fw_cheap = 0;        // fattn_wo: FattnWoArgs::cheap
    int fw_prio = 0;         // fattn_wo: FattnWoArgs::prio
    int fattn_wo = 1;        // 1: batch-1 bf16 fast-model attention + wo as one launch (fm_rowgemv.hip fattn_wo_kernel)
    int row_qkv_rp = 8;      // developer: rows per block of the bf16 row-block wqkv (4, 8 or 16)
    int rowgemv_q4 = 31;     // rowgemv's bits for weight-only int4 models (w1 || w3 too: int4 frame 3.06 -> 3.01 ms; bf16 4.07 -> 4.10, int8 3.11 -> 3.20 with it)
    int rowgemv = 27;        // batch-1 decode linears on the row-block GEMV (fm_rowgemv.hip): bit 0 wo / w2, bit 1 wqkv, bit 2 w1 || w3,
                             // bit 3 the codebook head, bit 4 the first layers' wqkv (0: 16-row MFMA tiles; 3 -> 27: 4.066 -> 4.032 ms)
    int row_copies = 1;      // 1: fm_llm_finalize keeps a row-major copy of every linear the row-block GEMV can take, so any
                             // rowgemv bits work later (bf16 S2-Pro: ~3.7 GB beside the packed tiles); 0: only the copies the
                             // rowgemv / rowgemv_q4 bits in force at finalize select (w1 || w3 bf16 / int8: ~3.6 GB saved)
    unsigned long long* dbg = nullptr;  // device buffer of per-block phase timestamps (debug_ts)
};
FmTuning& fm_tuning();
// PRO_FATT staging: raw q|k|v row, cached K/V rows [nkv][2][S-1][hd], qk-norm weights, RoPE row
inline size_t fatt_lds_bytes(int ldqkv, int nkv, int S, int hd, size_t esz) {
    return ((size_t)ldqkv + (size_t)nkv * 2 * (S - 1) * hd + 2 * (size_t)hd) * esz + (size_t)hd * 4 + 64;
}
inline size_t gemv_lds_bytes(int R, int Kb, size_t esz) {
    return (size_t)R * (Kb + 8) * esz + 16 * sizeof(float) + (2 * 8 * 16 + 16) * (size_t)R * sizeof(float) +
           8 * 8 * sizeof(float);
}
template <typename T> void launch_gemv(hipStream_t s, const GemvArgs<T>& a, int pro, int epi, int ksb);
// batch-1 row-block GEMV (fm_rowgemv.hip): row-major bf16 W [N][K], RP rows per 256-thread block.
//   ROWGEMV_FIN        (wo / w2, RP 2): y = round(res + round(W x + bias)) into res_out (its RMSNorm
//                      consumer: GemvArgs::ss_gran = 1)
//   ROWGEMV_NORM_STORE (wqkv, RP 8): x' = RMSNorm(x) * nw in the prologue, y = round(W x' + bias) into
//                      Y, optional KV prefetch (GemvArgs::pf_kc semantics)
//   ROWGEMV_NORM_SWIGLU (w1 || w3, RP 8: rows 8b .. 8b+3 = W1 rows 4b .. 4b+3, rows 8b+4 .. 8b+7 the same
//                      rows of W3): x' = RMSNorm(x) * nw, y[4b + t] = round(silu(round(g))) * round(u) into Y
//   ROWGEMV_NORM_F32   (a head, RP 8): x' = RMSNorm(x) * nw, Yf[n] = fp32 holding round(W x')
enum { ROWGEMV_FIN = 0, ROWGEMV_NORM_STORE = 1, ROWGEMV_NORM_SWIGLU = 2, ROWGEMV_NORM_F32 = 3 };
struct RowGemvArgs {
    const bf16_t* W;
    const int8_t* Wq;         // weight-only int8 (instead of W): row-major codes, output round(round(acc) * wscale)
    const bf16_t* wscale;     // int8: per-row scales [N]
    const uint32_t* Wq4;      // weight-only int4 (instead of W): packed row-major codes [N][K / 8] (launch_pack_q4_rows)
    const uint32_t* wsz;      // int4: (scale, zero) bf16 pairs [N][K / gs]
    int gs;                   // int4: group size
    const bf16_t* X;          // [K] (or a table [.][ldx] gathered by xidx[xcol], clamped to xrows; not FIN)
    int ldx;                  // (0: K)
    const int32_t* xidx;
    int xcol, xrows;
    const bf16_t* bias;       // [N] or null
    const bf16_t* nw;         // NORM: norm weight [K]
    float eps;
    const bf16_t* res;        // FIN: residual table [.][ldr] (row 0, or residx[res_col] clamped to res_rows)
    int ldr;
    const int32_t* residx;
    int res_col, res_rows;
    bf16_t* res_out;          // FIN: [N]
    bf16_t* Y;                // STORE / SWIGLU: [N] ([N / 2])
    float* Yf;                // F32: [N]
    int N, K;
    const bf16_t* pf_kc;      // STORE: KV prefetch (null: off), as GemvArgs
    const bf16_t* pf_vc;
    const int32_t* pf_slot;
    const int32_t* pf_pos;
    size_t pf_slot_stride, pf_layer_off;
    int pf_S, pf_nkv, pf_hd;
    unsigned long long* dbg;  // developer timestamps (launcher: fm_tune debug_ts)
};
int rowgemv_u(int K, int qm);  // per-wave chunk depth for K (qm 1: int8 codes; 0: not eligible)
void launch_rowgemv(hipStream_t s, const RowGemvArgs& a, int kind);
// batch-1 fast-model attention + wo in one launch (fm_rowgemv.hip fattn_wo_kernel; wo in bf16, int8 or int4): the
// attention blocks store their output as tagged words (bf16 << 16 | gen) into xt [nh * hd]; the wo
// row-pair blocks (RowGemvArgs FIN; its X is unused) poll them.  gen: the launch's index in the
// frame, 1..40; the tag is (row_pos[0] * 41 + gen) % 65535 + 1 (at.row_pos: the frame's position);
// err: set when a wait timed out.
struct FattnWoArgs {
    FastFusedArgs<bf16_t> at;
    RowGemvArgs wo;
    uint32_t* xt;
    int gen;
    int* err;
    int delay;                // wo blocks wait this many 10-ns ticks before their weight loads (fm_tune fw_delay)
    int cheap;                // 1: poll one word per 32-element group before the full read (fm_tune fw_cheap)
    int prio;                 // 1: attention waves at s_setprio 3 (fm_tune fw_prio)
    unsigned long long* dbg;  // developer records (launcher: fm_tune debug_ts)
};
bool fattn_wo_ok(int nh, int nkv, int hd, int cpos, int N, int K, int qm);
void launch_fattn_wo(hipStream_t s, const FattnWoArgs& a);
// batch-1 GEMV chain (fm_gemv.hip gemv_chain_kernel): 2..GEMV_CHAIN_MAX dependent GEMVs in one launch,
// whole K per block, one row.  Stage kinds: wo / w2 (PRO_PLAIN, EPI_SLABFIN; the residual may be a
// gathered row), w1||w3 (PRO_PRENORM, EPI_SWIGLU8), qkv (PRO_PRENORM, EPI_STORE), and as the last
// stage only, a head (PRO_PRENORM, EPI_F32; its outputs are read by later launches).  cnt: GEMV_CHAIN_WORDS zeroed words (the launch
// leaves them zeroed); err: set when a wait timed out.
constexpr int GEMV_CHAIN_MAX = 4;
constexpr int GEMV_CHAIN_LINE = 32;  // counter words one 128-B line apart
constexpr int GEMV_CHAIN_SLOTS = 17;  // per stage: 8 arrival shards, 1 top word, 8 done replicas
constexpr int GEMV_CHAIN_WORDS = GEMV_CHAIN_MAX * GEMV_CHAIN_SLOTS * GEMV_CHAIN_LINE;
enum { GEMV_CHAIN_WO_W2 = 0, GEMV_CHAIN_W13 = 1, GEMV_CHAIN_QKV = 2, GEMV_CHAIN_HEAD = 3 };
template <typename T> struct GemvChainArgs {
    GemvArgs<T> st[GEMV_CHAIN_MAX];
    int kind[GEMV_CHAIN_MAX];
    int off[GEMV_CHAIN_MAX + 1];
    int n;
    unsigned* cnt;
    int* err;
    int sleep;  // s_sleep between polls (fm_tune chain_sleep)
};
template <typename T> void launch_gemv_chain(hipStream_t s, const GemvChainArgs<T>& c);

// ---- batched decode weight streaming with register-resident X, 8 < R <= 32 (fm_bstream.hip) ---
template <typename T> struct BstreamArgs {
    const T* W;      // packed MFMA-fragment layout [tiles][K/32][512]
    const T* bias;   // [N] or null (EPI_STORE / EPI_F32; EPI_SLAB leaves it to finalize_norm)
    const T* X;      // [R][ldx]
    int ldx, R, N, K;
    T* Y;            // EPI_STORE / EPI_SWIGLU8 [R][ldy]
    int ldy;         // also the row stride of Yf
    float* Yf;       // EPI_F32 [R][ldy] | EPI_SLAB partial slabs [kparts][R][ldy]
    int kparts = 1;  // set by the launcher from the plan
    const T* wscale = nullptr;  // weight-only int8 row scales (EPI_SLAB: applied by finalize_norm)
    unsigned long long* dbg = nullptr;  // developer per-block timestamps (fm_tune "debug_ts")
    // bsacc_kernel only -- PRO_PRENORM: X' = RMSNorm(X) from the producer's per-tile sums of squares
    // ss_in [R][K/16] and the norm weight nw (llama.py:989-1000); EPI_SLABFIN: the last-arriving K
    // part of each tile group finalises x = round(res + round(sum of partials)) into res_out and
    // its per-tile sums of squares ss_out [R][N/16] (tickets: zero between launches).  (The batch-1
    // GEMV's tile sums are [tiles][R]; the two chains never exchange them.)
    int pro = 0;
    const float* ss_in = nullptr;
    const T* nw = nullptr;
    float eps = 0.f;
    const T* res = nullptr;
    int ldr = 0;
    T* res_out = nullptr;
    int ldro = 0;
    float* ss_out = nullptr;
    int* tickets = nullptr;
    int dummy_tail = 0;  // bsacc: ring slots past the block's tiles / steps load one cached fragment
    int xfirst = 1;      // bsacc: X (and the PRENORM operands) issued before the weight ring (fm_tune bs_xfirst)
    int vec_epi = 1;     // bsacc: epilogue items of 4 rows (16-byte LDS reads, 8 / 16-byte stores; fm_tune bs_vec_epi)
};
struct BstreamPlan {
    bool ok = false;
    int kparts = 1, nw = 0, spw = 0, tpi = 1, grid = 0;
    int acc = 0, ntm = 0;  // bsacc_kernel: tiles per block at most (register accumulators)
};
BstreamPlan bstream_plan(int N, int K, int R, int epi, size_t esz);
void bsacc_init();  // kernel attributes (> 64 KiB LDS) of every bsacc_kernel, outside any capture
template <typename T> bool launch_bstream(hipStream_t s, const BstreamArgs<T>& a, int epi, const BstreamPlan& p);
// x_out = round(res + round(sum of kparts slabs + bias)); if nw: xn_out = RMSNorm(x_out) * nw
template <typename T> struct FinalizeArgs {
    const float* slab;  // [kparts][R][lds]
    int kparts, lds;
    const T* bias;      // [d] or null
    const T* res;       // [R][ldr]
    int ldr;
    T* x_out;           // [R][ldx] (may alias res)
    int ldx;
    const T* nw;        // norm weight [d] or null (no norm)
    float eps;
    T* xn_out;          // [R][ldxn]
    int ldxn, d, R;
    const T* wscale = nullptr;  // weight-only int8: round(res + round(round(sum) * wscale[n]))
    // split form (fm_tune fin_split = ch > 1): each row over ch blocks that meet on cnt[2 r .. 2 r + 1]
    // (zero between launches) after publishing their chunk's sum of squares to ss_part[r][ch]
    int ch = 0;
    int* cnt = nullptr;
    float* ss_part = nullptr;
    int fin8 = 0;       // set by the launcher (fm_tune fin8): eight K parts' slab loads in one round trip
    int* err = nullptr; // split form: set when a row's blocks timed out waiting for each other
};
template <typename T> void launch_finalize_norm(hipStream_t s, const FinalizeArgs<T>& a);

// ---- fused decode attention / sampler (fm_attn.hip) ------------------------------------------
// prompt-chunk linear at 32 < R <= 64 rows, bf16 (fm_prompt.hip): raw fp32 K-slice partials into the
// conv split-K slab layout [ks][R][N]; the conv split-K epilogue finishes it
struct PromptSkinnyArgs {
    const bf16_t* w;   // packed weight [ceil(N/16)][K/32][512]
    const bf16_t* x;   // activation rows [R][ldx]
    int ldx, R, N, K;
    float* slab;       // [ks][R][N]
    // one slice and act set: no slab, the interleaved SwiGLU of the row-interleaved W1 || W3 stored
    // straight to act [R][lda] (swiglu_i8_kernel's roundings)
    bf16_t* act = nullptr;
    int lda = 0;
};
void launch_prompt_skinny(hipStream_t s, const PromptSkinnyArgs& a, int ks);
// K slices: the smallest divisor of K/32 with >= 8 k-steps per slice giving >= target blocks of 64
// rows (the largest such when none does; 0 when K / 32 < 8)
int prompt_skinny_ks(int N, int K, int target);

template <typename T> struct AttnDecArgs {
    const T* qkv;        // raw projections [R][ldqkv] (q heads, k heads, v heads)
    int ldqkv;
    const int* row_slot;
    const int* row_pos;
    int nh, nkv, hd, qk_norm;
    float eps;
    const T* qn;
    const T* kn;
    const float* rope;   // [S][hd/2][2]
    T* kc;
    T* vc;
    size_t slot_stride, layer_off;
    int S, maxsplit;
    float scale;
    float* part;         // [R][nh][maxsplit][hd+2]
    // attn_decode2 only
    int cap;             // rows per block
    int* cnt;            // [R][nkv] arrival tickets (zeroed at allocation, reset by the last block)
    T* out;              // [R][nh*hd]
    unsigned long long* dbg;  // developer timestamps (fm_tune "debug_ts")
    float* qdbg = nullptr;    // per-op test hook (fm_op_qk_rope): q after qk-norm + RoPE [R][nh][hd]
    int nwb = 4;              // attn_fd: waves per block (4, 8 or 16; 16 nwb positions per pass)
    const float* qslab = nullptr;  // as FastFusedArgs: K-part slabs of the QKV projection (attn_fd)
    int qslab_kp = 1;
    const T* qbias = nullptr;
};
// decode attention for the small-batch path (see fm_attn.hip): a.cap rows per block, a.maxsplit =
// ceil(S / cap) blocks per (row, kv head), output straight to a.out (bf16 / T)
template <typename T> void launch_attn_decode2(hipStream_t s, const AttnDecArgs<T>& a, int R);
inline size_t attn2_lds_bytes(int hd, int g, int cap, size_t esz) {
    return (size_t)cap * (hd + 8) * esz + (size_t)cap * hd * esz + (size_t)g * hd * 4 + (size_t)g * cap * 4 +
           16 + 8 * (size_t)g * 4;
}
// rows per attn_decode2 block within ~150 KB of LDS (multiple of 16, <= 256)
inline int attn2_cap(int hd, int g, size_t esz) {
    long budget = 150L * 1024 - 16 - 8L * g * 4 - (long)g * hd * 4;
    long per = (long)(2 * hd + 8) * (long)esz + 4L * g;
    long c = budget / per;
    c = c > 256 ? 256 : c;
    return (int)(c & ~15L);
}
// decode attention v3 (fm_attn.hip attn_dec3_kernel): 64 positions per block in registers,
// maxsplit set by the launcher (ceil(S / 64)); a.part must hold [R][nh][ceil(S / 64)][hd + 2]
// flash-decode attention (fm_attn.hip attn_fd_kernel), every batch size: splits of at least a.cap
// (>= 16) positions, at most FD_NSP per (row, kv head); maxsplit set by the launcher; a.part must
// hold [R][nh][min(FD_NSP, ceil(S / cap))][hd + 2], a.cnt [R][nkv] zeroed tickets
constexpr int FD_NSP = 16;
inline bool attn_fd_ok(int hd, int g) { return (hd == 32 || hd == 64 || hd == 128) && g >= 1 && g <= 4; }
template <typename T> void launch_attn_fd(hipStream_t s, const AttnDecArgs<T>& a, int R);
template <typename T> void launch_attn_decode3(hipStream_t s, const AttnDecArgs<T>& a, int R);
template <typename T> void launch_fast_attn_fused(hipStream_t s, const FastFusedArgs<T>& a, int R);
// fast-model attention, one wave per q head (cpos < 16 cached rows, hd <= 256)
template <typename T> void launch_fast_attn2(hipStream_t s, const FastFusedArgs<T>& a, int R);
template <typename T> void launch_sample_radix(hipStream_t s, const SampleArgs& a, int R);
void sample_init();  // sampler kernel attributes (dynamic LDS past 64 KiB), outside any capture
template <typename T>
void launch_attn_combine(hipStream_t s, const float* part, const int* row_pos, int R, int nh, int hd,
                         int split, int maxsplit, T* out);

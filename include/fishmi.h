/*
 * fishmi.h -- C ABI of libfishmi.so, the MI355X-native Fish-Speech S2-Pro hot path:
 * the Dual-AR text->semantic decode loop and the modded-DAC codec decode.
 *
 * The reference has no FFI/plugin API for this path; its seams are Python
 * callables.  Each entry point below replaces one of them (file:line in the reference,
 * PoTaTo-Mika/fish-speech @ 2026-04-03):
 *
 *   fm_llm_open/set_tensor/finalize  <- DualARTransformer.from_pretrained + init_model +
 *                                       setup_caches           (llama.py:479-593, 307-324,
 *                                                               707-721; inference.py:362-392)
 *   fm_llm_prefill                   <- generate() prefill: decode_one_token_ar(prompt,
 *                                       arange(T))             (inference.py:322-335)
 *   fm_llm_decode                    <- decode_one_token_ar per frame, batched over slots
 *                                                              (inference.py:96-181, 209-234)
 *   fm_llm_decode_frames             <- decode_n_tokens        (inference.py:184-238)
 *   fm_llm_generate                  <- generate()             (inference.py:241-359)
 *   fm_llm_teacher_step              <- forward_generate + forward_generate_fast with given
 *                                       tokens (teacher forcing; parity tests)
 *                                                              (llama.py:390-466, 798-827)
 *   fm_codec_open/set_tensor/...     <- load_codec_model / dac.inference.load_model
 *                                                              (inference.py:395-417;
 *                                                               dac/inference.py:23-47)
 *   fm_codec_decode                  <- DAC.from_indices       (modded_dac.py:925-927)
 *
 * Conventions: every function returns FM_OK (0) or a negative FM_ERR_*; the message of the
 * last failure on the calling thread is fm_last_error().  Nothing throws across the ABI.
 * Buffers are caller-owned host memory.  One handle per GPU; calls on a handle must come from
 * one host thread at a time (the reference's single LLM worker thread, inference.py:748-799).
 * Token matrices are (C+1) x T row-major int32, exactly the reference's prompt layout
 * (row 0 = text/semantic token, rows 1..C = codebooks).
 */
#ifndef FISHMI_H
#define FISHMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FM_OK 0
#define FM_ERR_ARG -1
#define FM_ERR_HIP -2
#define FM_ERR_STATE -3
#define FM_ERR_OOM -4

/* precision of the compute path: bf16 storage + fp32 accumulation (production), or the fp32
   validation mode (same kernels, fp32 storage) used for token-exact parity. */
#define FM_PREC_BF16 0
#define FM_PREC_FP32 1

/* source dtype for fm_*_set_tensor (FM_DT_I8: int8 linear weights, fm_llm_set_quant INT8 only) */
#define FM_DT_F32 0
#define FM_DT_BF16 1
#define FM_DT_I8 2

/* weight-only quantization of the Dual-AR linears (fm_llm_set_quant) */
#define FM_QUANT_NONE 0
#define FM_QUANT_INT8 1
#define FM_QUANT_INT4 2  /* groupwise int4, group size 128 (fm_llm_set_quant_int4 for others) */

/* == DualARModelArgs after from_pretrained (llama.py:27-193); im_end_id from the tokenizer. */
typedef struct fm_model_config {
    int vocab_size, dim, n_layer, n_head, n_local_heads, head_dim, intermediate_size;
    float rope_base, norm_eps;
    int max_seq_len;
    int qkv_bias, o_bias, qk_norm, tie_word_embeddings;
    int codebook_size, num_codebooks, semantic_begin_id, semantic_end_id, im_end_id;
    int scale_codebook_embeddings, norm_fastlayer_input;
    int n_fast_layer, fast_dim, fast_n_head, fast_n_local_heads, fast_head_dim,
        fast_intermediate_size;
    int fast_qkv_bias, fast_o_bias, fast_qk_norm;
} fm_model_config;

/* sampling knobs of decode_one_token_ar; temperature/top_p are applied as tensors of the
   compute dtype like inference.py:305-306.  mask_im_end=1 forbids <|im_end|> (fixed-length
   timing runs). */
typedef struct fm_sampling {
    float temperature, top_p;
    int top_k;
    uint64_t seed;
    int mask_im_end;
} fm_sampling;

typedef struct fm_llm fm_llm;

int fm_device_count(void);
const char* fm_last_error(void);

/* Build provenance: the first 16 hex digits of sha256 over the sources and headers the library was
 * compiled from (fish-speech_amd/Makefile HASHED); fishmi.native.lib() refuses a library whose hash
 * differs from the tree's, so a stale prebuilt libfishmi.so cannot run. */
const char* fm_source_hash(void);
/* Measured HBM stream peak of `device` (no reference counterpart: SURVEY.md §8d's STREAM-like
   figure beside the vendor peak): a non-temporal float4 read stream (GB/s read) and a float4 copy
   (GB/s read + written) over `bytes`-sized buffers (>= 64 MiB; use >> 256 MiB to defeat the MALL),
   `reps` timed launches each. */
int fm_stream_peak(int device, int64_t bytes, int reps, double* read_gbps, double* copy_gbps);

int fm_llm_open(const fm_model_config* cfg, int device, int precision, int max_slots,
                fm_llm** out);
/* Weight-only int8 linears, opt-in (replaces tools/llama/quantize.py WeightOnlyInt8QuantHandler
   .convert_for_runtime + the int8 branch of from_pretrained, llama.py:528-535; quantize.py:190-232).
   Call before any set_tensor.  Every nn.Linear (attention wqkv/wo, feed_forward w1/w2/w3 of both
   stacks, output when untied, fast_project_in, fast_output) then takes either int8 data
   (FM_DT_I8) plus "<module>.scales" [out_features], as quantize.py writes them, or float weights
   that finalize quantizes per output channel with quantize.py's rule.  Outputs are
   round(round(x . q) * scale) like WeightOnlyInt8Linear.forward; the linears' biases are unused
   (that module has none).  Off the bf16 parity contract: parity is against the reference's own
   int8 model. */
int fm_llm_set_quant(fm_llm* h, int mode);
/* Weight-only int4, groupwise affine (replaces tools/llama/quantize.py WeightOnlyInt4QuantHandler
   .create_quantized_state_dict + convert_for_runtime and the int4 branch of from_pretrained,
   llama.py:537-543; quantize.py:57-160, 239-418).  bf16 only; bias-free linears (quantize.py:371);
   groupsize 32, 64, 128 or 256 dividing every in_features.  Every nn.Linear takes float weights, quantized at
   finalize with the reference's group_quantize_tensor (bit-exact, in its bf16 arithmetic); each
   then computes with the weights bf16(fma(q - 8, scale, zero)), and the batch <= 8 decode GEMVs
   stream the 4-bit codes (group size a multiple of 128).  The reference's packed checkpoint format
   (_convert_weight_to_int4pack tiles) is not read: quantize from the bf16 checkpoint instead. */
int fm_llm_set_quant_int4(fm_llm* h, int groupsize);
/* name = reference state_dict key after remap (e.g. "layers.3.attention.wqkv.weight") */
int fm_llm_set_tensor(fm_llm* h, const char* name, const void* host_data, int src_dtype,
                      int64_t numel);
/* deterministic synthetic tensor (fishmi/synth.py formula), generated on the device */
int fm_llm_synth_tensor(fm_llm* h, const char* name, int64_t numel, uint64_t seed, float center,
                        int log2_half);
int fm_llm_finalize(fm_llm* h);
/* n requests prefilled together (each from position 0 of its own slot, slots distinct): tokens
   holds each request's (C+1) x T[i] prompt block back to back, sp one sampling record per request;
   one pass of the slow stack over all prompt rows, one batched first frame; writes n first columns
   (n x (C+1)), the same as n fm_llm_prefill calls (the reference prefills requests one by one:
   inference.py:620-724; this is the serving side's batched form of it). */
int fm_llm_prefill_batch(fm_llm* h, int n, const int32_t* slots, const int32_t* tokens, const int32_t* T,
                         const fm_sampling* sp, int32_t* first_cols);
/* resets slot's caches and runs the prompt; writes the first emitted column (C+1). */
int fm_llm_prefill(fm_llm* h, int slot, const int32_t* tokens, int T, const fm_sampling* sp,
                   int32_t* first_col);
/* one frame for n slots (each continues from its own position); cols: n x (C+1) */
int fm_llm_decode(fm_llm* h, const int32_t* slots, int n, int32_t* cols);
/* nframes frames for the n slots, queued back to back with no host round trip per frame
   (im_end does not stop it: callers drop columns after a slot's <|im_end|>, as the batched
   engine does); cols: nframes x n x (C+1). */
int fm_llm_decode_frames(fm_llm* h, const int32_t* slots, int n, int nframes, int32_t* cols);
/* full generate() for one slot: out (C+1) x max_new row-major; *n_out frames produced
   (stops after emitting <|im_end|> unless mask_im_end). */
int fm_llm_generate(fm_llm* h, int slot, const int32_t* prompt, int T, int max_new,
                    const fm_sampling* sp, int32_t* out, int* n_out);
/* generate() continuing a slot's cached prefix: positions [0, pos0) keep the KV of tokens the
   slot already ran (the previous generate_long batch's prompt and fed columns), the prompt suffix
   ((C+1) x T) is prefilled at pos0 .. pos0 + T - 1, then decoding as fm_llm_generate.  Replaces
   the whole-conversation re-prefill of generate_long (inference.py:620-724) for the shared
   prefix.  pos0 must not exceed fm_llm_slot_pos. */
int fm_llm_generate_at(fm_llm* h, int slot, const int32_t* suffix, int T, int pos0, int max_new,
                       const fm_sampling* sp, int32_t* out, int* n_out);
/* fm_llm_prefill continuing the slot's cached positions [0, pos0): the suffix runs at pos0 .. */
int fm_llm_prefill_at(fm_llm* h, int slot, const int32_t* suffix, int T, int pos0, const fm_sampling* sp,
                      int32_t* first_col);
/* positions of the slot whose KV is written (prompt + fed columns of its last generate) */
int fm_llm_slot_pos(fm_llm* h, int slot, int* pos);
/* teacher forcing for parity: run S positions of x ((C+1) x S) from pos0 on slot (pos0 == 0
   resets the slot), return the last position's slow logits (V, with the semantic bias NOT
   applied), the fast hidden (fast_dim), and -- when next_col != NULL -- the fast logits
   ((C-1) x codebook_size) obtained by feeding next_col's codebook tokens. */
int fm_llm_teacher_step(fm_llm* h, int slot, const int32_t* x, int S, int pos0,
                        const int32_t* next_col, float* slow_logits, float* hidden,
                        float* fast_logits);
/* decode-step accounting for the roofline: algorithmic HBM bytes of one frame at batch n
   (weights read once per frame + KV + embeddings) at cached length `pos`. */
int64_t fm_llm_frame_bytes(fm_llm* h, int n, int pos);
/* per-kernel-class timing (HIP events on the compute stream) */
int fm_llm_profile(fm_llm* h, int enable);
int fm_llm_profile_read(fm_llm* h, const char* kernel_class, double* total_ms, int64_t* launches,
                        int64_t* bytes);
/* roofline hook: runs one decode frame for the last decoded slot set (advancing them one frame)
   while recording the launches of kernel_class ("linear" = the decode GEMVs), then replays
   exactly those launches back to back `reps` times as one graph between two HIP events on the
   compute stream: average duration per launch, launches and algorithmic bytes per frame.
   The replays clobber activation scratch only (KV caches and slot state are untouched). */
int fm_llm_kernel_bench(fm_llm* h, const char* kernel_class, int reps, double* avg_us,
                        int64_t* launches, int64_t* bytes);
int fm_llm_use_graph(fm_llm* h, int enable);
/* developer hook: row 0 of an activation buffer of the decode path ("qkv", "att", "fh", "act",
   "fx", "fx2", "xl", "xnl": bf16/fp32 storage as floats) or slot 0's KV cache of slow layer `index`
   ("kc" / "vc": [n_local_heads][S][head_dim], n <= its size; the prefix-reuse identity tests) */
int fm_llm_debug_vec(fm_llm* h, const char* name, int index, float* out, int64_t n);
/* Teacher forcing on the PRODUCTION decode path (parity with the reference's own teacher-forced
   forward_generate / forward_generate_fast, llama.py:390-466, 798-827): while a slot is forced,
   every sampler of its frames (prefill and decode, graph-replayed or eager, batch-1 GEMV path or
   batched path) emits the given column instead of its draw and copies the logits it was handed
   to a per-slot tap.  col: (C+1) tokens of the next emitted column (row 0 a semantic id or
   <|im_end|>), or NULL to stop forcing; set it before fm_llm_prefill / each fm_llm_decode.
   read_logits: the last forced frame's slow logits (V floats, -inf outside the semantic rows and
   <|im_end|>, bias NOT applied) and fast logits ((C-1) x codebook_size, codebooks 1..C-1). */
int fm_llm_force(fm_llm* h, int slot, const int32_t* col);
int fm_llm_read_logits(fm_llm* h, int slot, float* slow_logits, float* fast_logits);
/* process-wide developer knobs selecting kernel variants (every variant stays under the default
   path's parity bar, tests/test_gpu_knobs.py): decode GEMV "gemv_nt" 0|1, "gemv_u" 2|4|8,
   "gemv_wpb" 4|8, "ksb_blocks" n, "ksb_balance" 0|1, "fin_ksb" n, "kv_prefetch" 0|1, "gemv_dummy" 0|1|2, "gemv_chain" 0|1,
   "chain_max" 2..4, "chain_sleep" 1|4|16; attention "attn_fd" 0|1, "attn3" 0|1,
   "attn_cap" n, "attn_cap_batched" n, "fd_min" n, "fd_min_batched" n, "fd_nw" 4|8|16, "fd_min16" n,
   "fd_nw_batched" 4|8|16, "attn_wo" 0|1,
   "batched_fused_attn" 0|1; batched linears "bstream" 0|1, "bstream_acc" 0|1, "bstream_chain" 0|1, "bstream_kparts" n, "bstream_nw" n, "bs_dummy" 0|1|2, "bs_qkv_slab" 0|1,
   "bs_xfirst" 0|1, "bs_vec_epi" 0|1,
   "linear_u32" n, "linear_fill" n; prompt "prefill_attn", "prompt_gemm"; codec "conv2",
   "conv_splitk"; "sampler_fast" 0|1, "rmsnorm_block" 0|1, "debug_ts" n; batch-1 row-block GEMV
   "rowgemv" / "rowgemv_q4" bits, "row_copies" 0|1 (0: finalize keeps only the row-major weight
   copies those bits select).  They apply to launches
   recorded after the call (graphs captured earlier keep theirs). */
int fm_tune(const char* key, int value);
/* developer hook ("debug_ts" armed): per-block records of 8 words {tag = N<<32 | blockIdx.y<<16 |
   blockIdx.x, start, staged, streamed, end, 3 kernel-specific} of the decode GEMVs,
   s_memrealtime ticks (100 MHz). */
int fm_debug_ts_read(unsigned long long* out, int64_t max_records, int64_t* n_records);
int fm_llm_close(fm_llm* h);

/* ---- per-op parity hooks (tests): one production kernel on caller operands, fp32 host arrays
   in/out (converted to the precision's storage type).  Each replaces nothing in the reference; they
   pin the fused decode kernels to the reference's per-op semantics (tests/golden/ops.npz). */
/* RMSNorm (llama.py:989-1000), R rows of d: mode 0 = the decode GEMV prologue computing the
   statistic from the row (first layer, head), 1 = the prologue fed by the producing GEMV's per-tile
   sums of squares (every later norm of the batch-1 path), 2 = the standalone row kernel (batched /
   prefill path). */
int fm_op_rmsnorm(int device, int precision, int mode, const float* x, const float* w, int R, int d,
                  float eps, float* y);
/* QK-norm (llama.py:861-863) + RoPE with the bf16 table (llama.py:1003-1037) at position pos, as the
   fused decode attention computes them: kernel 0 = slow attn_decode2, 1 = fast-model attention,
   2 = slow attn_dec3, 3 = slow attn_fd (the production kernel).
   qkv: one raw projection row [(nh + 2 nkv) * hd]; q_out [nh * hd], k_out [nkv * hd] (the k row as
   written to the KV cache). */
int fm_op_qk_rope(int device, int precision, int kernel, const float* qkv, int nh, int nkv, int hd,
                  const float* qn, const float* kn, int qk_norm, float eps, float rope_base, int pos,
                  float* q_out, float* k_out);
/* The whole slow-model decode attention as the decode path runs it (llama.py:883-945: QK-norm, RoPE,
   KV-cache write, scaled dot-product attention with the GQA group sharing its kv head) on R rows;
   row r uses slot r of caller caches kcache / vcache [R][nkv][S][hd] holding rows < pos[r].
   kernel 0 = attn_decode2, 2 = attn_dec3, 3 = attn_fd (flash-decode splits of >= min_split
   positions).  out [R][nh * hd]; kc_out / vc_out receive the caches after the kernel's write. */
int fm_op_decode_attn(int device, int precision, int kernel, const float* qkv, int R, int nh, int nkv, int hd,
                      const float* qn, const float* kn, int qk_norm, float eps, float rope_base, const int* pos,
                      const float* kcache, const float* vcache, int S, int min_split, float* out, float* kc_out,
                      float* vc_out);
/* prompt-chunk causal attention (llama.py:883-946, the prefill path after QK-norm / RoPE / KV
   write): q [R][nh * hd] of rows at positions pos0 .. pos0 + R - 1 of one slot, caches
   kcache / vcache [nkv][S][hd] holding every position <= pos0 + R - 1.  kernel 0 = split +
   combine kernels, 1 = attn_prefill_kernel (flash form on MFMA; bf16, head_dim 128, <= 4 q heads
   per kv head).  out [R][nh * hd]. */
int fm_op_prompt_attn(int device, int precision, int kernel, const float* q, int R, int nh, int nkv, int hd, int pos0,
                      const float* kcache, const float* vcache, int S, float* out);
/* Dual-AR input embedding (llama.py:399-420): tok R x (C+1) row-major, x R x dim. */
int fm_op_embed(int device, int precision, const int32_t* tok, int R, const float* emb, int vocab,
                const float* cbemb, int dim, int num_codebooks, int codebook_size, int semantic_begin_id,
                int semantic_end_id, int scale_codebook_embeddings, float* x);
/* Weight-only int4 (fm_llm_set_quant_int4): the device quantizer on a bf16-valued w [N][K] with group
   size gs (quantize.py:57-160 in its bf16 arithmetic): codes q [N][K] (0..15), group scale / zero
   [N][K/gs] and the dequantised weights bf16(fma(q - 8, scale, zero)) [N][K].  With x (R <= 8 rows
   of K), also the decode GEMV y = x . w_deq^T ([R][N] fp32) on the dequantised bf16 weights (y_bf16)
   and, when gs and K are multiples of 128 and y_q4 is given, on the streamed 4-bit codes (y_q4). */
int fm_op_quant4(int device, const float* w, int N, int K, int gs, uint8_t* q, float* scale, float* zero,
                 float* w_deq, const float* x, int R, float* y_q4, float* y_bf16);
/* the RoPE cos/sin table the library builds on the host (precompute_freqs_cis, llama.py:1003-1022):
   out [seq_len][head_dim/2][2], bf16-valued floats.  No device needed. */
int fm_rope_table(int seq_len, int head_dim, float base, float* out);

/* ---- codec (modded DAC decode side, modded_dac_vq.yaml shapes) --------------------- */
typedef struct fm_codec_config {
    int latent, decoder_dim, n_codebooks, codebook_size, semantic_codebook_size, codebook_dim;
    int t_layers, t_heads, t_head_dim, t_inter, window;
    float rope_base, norm_eps;
} fm_codec_config;

typedef struct fm_codec fm_codec;

int fm_codec_open(const fm_codec_config* cfg, int device, int precision, int max_frames,
                  fm_codec** out);
int fm_codec_set_tensor(fm_codec* h, const char* name, const void* host_data, int src_dtype,
                        int64_t numel);
int fm_codec_synth_tensor(fm_codec* h, const char* name, int64_t numel, uint64_t seed,
                          float center, int log2_half);
int fm_codec_finalize(fm_codec* h);
/* codes: (n_codebooks+1) x T row-major (clamped like rvq.py:354-359, input not mutated);
   pcm: 2048*T floats in [-1, 1]. */
int fm_codec_decode(fm_codec* h, const int32_t* codes, int T, float* pcm);
/* Streamed decode (BASELINE config 5: long-form audio vocoded chunk by chunk while the LLM is
   still generating; the reference decodes each generated segment on its own,
   inference_engine/vq_manager.py:16-21).  The codec is causal end to end, so a stream of chunks
   that carries each causal reader's previous rows (conv inputs, the transformer's window of
   keys/values, the RoPE position) reproduces the one-shot fm_codec_decode of the concatenated
   codes exactly.  The handle's own stream: stream_reset starts it, each decode_chunk appends T
   frames (T <= max_frames) and returns their 2048*T samples.  Concurrent streams (one per
   streamed request, several requests on one handle): stream_open gives a new context with its own
   carried rows and position (starting at zero, like a reset), stream_decode appends to it,
   stream_close frees it; stream_rewind zeroes a context for the next request (a context pool
   needs no allocation, and no hipFree device sync, per request).  Calls on one handle are
   serialised by the caller (one host thread at a time); a context switch rebinds pointers only. */
int fm_codec_stream_reset(fm_codec* h);
int fm_codec_decode_chunk(fm_codec* h, const int32_t* codes, int T, float* pcm);
int fm_codec_stream_open(fm_codec* h, int* stream_id);
int fm_codec_stream_decode(fm_codec* h, int stream_id, const int32_t* codes, int T, float* pcm);
int fm_codec_stream_rewind(fm_codec* h, int stream_id);
int fm_codec_stream_close(fm_codec* h, int stream_id);
int fm_codec_profile_read(fm_codec* h, double* total_ms, int64_t* launches, double* flops);
/* test hook: intermediate of the last decode as fp32, time-major (1 transformer out [T][latent],
   2 first upsample [2T][latent], 3 decoder input [4T][latent]); other stages' buffers are
   reused in place and are not readable. */
int fm_codec_debug_read(fm_codec* h, int stage, int T, float* out);
// Codec ENCODE (voice-clone reference audio -> codes), SURVEY.md §8f row 1.  Replaces
// DAC.encode(audio[B,1,N], audio_lengths) -> (codes[B,C,T], lens) (fish_speech/models/dac/
// modded_dac.py:874-923; caller vq_manager.py:24-52 encode_reference).  enable before
// set_tensor/finalize: adds the encode-side tensors (Encoder, quantizer.downsample,
// quantizer.pre_module, VQ in_proj) to the inventory; encoder_dim 64 and enc_layers 4 for
// modded_dac_vq.yaml.  encode: mono 44.1 kHz fp32 samples (n <= 2048 * max_frames), right-padded
// to a multiple of 2048; codes (caller-owned, (n_codebooks+1) x T row-major, T = ceil(n/2048)).
int fm_codec_enable_encoder(fm_codec* h, int encoder_dim, int enc_layers);
int fm_codec_encode(fm_codec* h, const float* audio, int64_t n, int32_t* codes, int* T_out);
int fm_codec_close(fm_codec* h);

#ifdef __cplusplus
}
#endif
#endif /* FISHMI_H */

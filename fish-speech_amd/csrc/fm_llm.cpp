// fm_llm.cpp -- host runtime of the Dual-AR decode path (C ABI in include/fishmi.h).
//
// One handle per GPU owns: the weights (bf16 or fp32), per-slot KV caches, per-slot sampler
// state (temperature/top_p/top_k/seed/step + RAS window), and the activation buffers.  A
// frame (one decode_one_token_ar for n slots, inference.py:96-181) is a fixed kernel sequence
// that reads every dynamic value (tokens, positions, steps) from device memory, so it is
// captured once per batch size into a hipGraph and replayed.
#include <dlfcn.h>
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <signal.h>

#include <algorithm>
#include <array>
#include <memory>

#include "fm_codec.h"
#include "fm_kernels.h"
#include "fm_runtime.h"

// developer: FISHMI_SEGV_TRACE=1 prints the native stack (module + offset per frame) of a host
// fault before the default action (the rocprofv3 fault investigation)
namespace {
void segv_trace(int sig, siginfo_t* si, void*) {
    void* fr[64];
    const int n = backtrace(fr, 64);
    fprintf(stderr, "fishmi: signal %d at address %p, %d frames\n", sig, si ? si->si_addr : nullptr, n);
    for (int i = 0; i < n; ++i) {
        Dl_info d{};
        if (dladdr(fr[i], &d) && d.dli_fname)
            fprintf(stderr, "  #%d %s +0x%lx (%s)\n", i, d.dli_fname,
                    (unsigned long)((const char*)fr[i] - (const char*)d.dli_fbase), d.dli_sname ? d.dli_sname : "?");
        else
            fprintf(stderr, "  #%d %p\n", i, fr[i]);
    }
    fflush(stderr);
    signal(sig, SIG_DFL);
    raise(sig);
}
struct SegvTraceInstaller {
    SegvTraceInstaller() {
        const char* e = getenv("FISHMI_SEGV_TRACE");
        if (!e || e[0] != '1') return;
        struct sigaction sa {};
        sa.sa_sigaction = segv_trace;
        sa.sa_flags = SA_SIGINFO;
        sigaction(SIGSEGV, &sa, nullptr);
        sigaction(SIGBUS, &sa, nullptr);
    }
} g_segv_trace;
}  // namespace

static thread_local std::string g_err;
void fm_set_error(const std::string& s) { g_err = s; }
extern "C" const char* fm_last_error(void) { return g_err.c_str(); }
extern "C" int fm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

static constexpr int PREFILL_CHUNK = 1024;  // prompt rows per slow-stack pass (GEMM M)
static constexpr int ATTN_PIECE = 256;      // prompt rows per attention launch (bounds the split partials)
static constexpr int ATTN_SPLIT = 64;
static constexpr int GEMV_MAX_ROWS = 8;  // frames with <= 8 streams take the fused GEMV path
static constexpr int KSB_MAX = 8;
static constexpr int BS_KPARTS = 8;  // most K parts of a bstream slab (fm_bstream.hip)

// split-K factor across blocks for a GEMV with N output rows: >= ~512 blocks when possible,
// K/(32*ksb) integral, LDS staging within budget.
FmTuning& fm_tuning() {
    static FmTuning t;
    return t;
}

static int pick_ksb(int N, int K, int R, size_t esz) {
    const int nb = (N + 15) / 16;
    const FmTuning& tu = fm_tuning();
    int ksb = 1;
    while (ksb < KSB_MAX && nb * ksb < tu.ksb_blocks && K % (32 * ksb * 2) == 0) ksb *= 2;
    if (tu.ksb_balance) {
        // among the admissible split factors pick the one whose grid wastes the least of its
        // last round of 256 CUs (ties: the smaller split)
        double best = 1e9;
        int bk = ksb;
        for (int k = 1; k <= KSB_MAX && K % (32 * k) == 0; k *= 2) {
            const int b = nb * k;
            if (b < 256) continue;
            const double rounds = (double)((b + 255) / 256), waste = rounds * 256.0 / b;
            if (waste < best - 1e-3) {
                best = waste;
                bk = k;
            }
        }
        ksb = bk;
    }
    while (gemv_lds_bytes(R, K / ksb, esz) > 96 * 1024 && ksb < KSB_MAX && K % (32 * ksb * 2) == 0) ksb *= 2;
    while (K / ksb > 4096 && K % (32 * ksb * 2) == 0) ksb *= 2;  // one 8-element chunk per thread
    return ksb;
}

struct LayerW {
    void *wqkv = nullptr, *bqkv = nullptr, *wo = nullptr, *bo = nullptr, *qn = nullptr, *kn = nullptr;
    void *w13 = nullptr, *w2 = nullptr, *an = nullptr, *fn = nullptr;  // w13: row-interleaved W1||W3
    void *wo_rm = nullptr, *w2_rm = nullptr, *wqkv_rm = nullptr, *w13_rm = nullptr;  // row-major as well (fm_rowgemv.hip)
};

struct StackDims {
    int n_layer, dim, nh, nkv, hd, inter, qkv_bias, o_bias, qk_norm;
    int nq() const { return nh * hd; }
    int nqkv() const { return (nh + 2 * nkv) * hd; }
};

struct fm_llm {
    fm_model_config c{};
    int device = 0, prec = FM_PREC_BF16, max_slots = 1;
    size_t esz = 2;
    hipStream_t stream = nullptr;
    std::map<std::string, DTensor> w;
    bool finalized = false;
    StackDims sd{}, fdm{};
    int S = 0, C = 0, C1 = 0, cb = 0, nsem = 0, Nhead = 0, maxsplit = 0, Rmax = 0;
    std::vector<LayerW> slow, fast;
    void *emb = nullptr, *cbemb = nullptr, *norm = nullptr, *head_c = nullptr, *fproj_w = nullptr,
         *fproj_b = nullptr, *femb = nullptr, *fnorm = nullptr, *fout = nullptr;
    // caches
    void *kc = nullptr, *vc = nullptr, *fkc = nullptr, *fvc = nullptr;
    size_t slot_stride = 0, layer_stride = 0, fslot_stride = 0, flayer_stride = 0;
    float *rope = nullptr, *frope = nullptr;
    // activations
    void *x = nullptr, *h = nullptr, *xn = nullptr, *qkv = nullptr, *q = nullptr, *att = nullptr,
         *act = nullptr;
    void *xl = nullptr, *xnl = nullptr, *fx = nullptr, *fh = nullptr, *fxn = nullptr;
    // batch-1 GEMV chain (fm_tune gemv_chain): layer outputs alternate between x / x2 (fx / fx2), so no
    // launch re-reads a residual row it has already read and a later stage rewrites
    void *x2 = nullptr, *fx2 = nullptr;
    unsigned* chain_cnt = nullptr;  // [GEMV_CHAIN_WORDS] arrival counters (zeroed; each launch re-zeroes them)
    int* chain_err = nullptr;       // a chain wait timed out
    int* h_chain_err = nullptr;     // pinned copy, read after the host's stream sync
    void* plast = nullptr;  // batched prefill: the last prompt row of each request [max_slots][dim]
    float *part = nullptr, *logits = nullptr, *flogits = nullptr;
    void* act2 = nullptr;  // batched path: [R][2 * inter] output of the interleaved W1||W3
    int* attn_cnt = nullptr;
    float *ssX = nullptr, *ssH = nullptr;  // per-16-column tile sums of squares of the residual rows
    int* tickets = nullptr;               // EPI_SLABFIN / linear split-K arrival counters (zero between launches)
    float* skpart = nullptr;              // linear_kernel split-K partial tiles
    long long skpart_cap = 0;             //   floats
    float *slabA = nullptr, *slabB = nullptr;  // split-K partials of wo / w2 (small-batch path)
    float *bsA = nullptr, *bsB = nullptr;      // bstream K-part slabs of wo / w2 (batched path)
    float* bsQ = nullptr;                      // K-part slabs of the batched QKV (fm_tune bs_qkv_slab)
    // rows / slots
    int *frame_slot = nullptr, *frame_pos = nullptr, *prow_slot = nullptr, *prow_pos = nullptr;
    int32_t *tok_in = nullptr, *cols = nullptr, *ptok = nullptr, *ras = nullptr;
    SlotParams* sp = nullptr;
    // teacher forcing on the production graph (fm_llm_force / fm_llm_read_logits)
    int32_t* force_cols = nullptr;              // [max_slots][C1]
    float *tap_slow = nullptr, *tap_fast = nullptr;  // [max_slots][Nhead], [max_slots][C-1][cb]
    std::vector<int> host_force;
    int32_t* h_cols = nullptr;  // pinned [2][max_slots][C1]
    int32_t* h_hist = nullptr;  // pinned, grown on demand: [frames][n][C1] of fm_llm_decode_frames
    size_t h_hist_n = 0;
    std::vector<int> host_pos, host_step;
    std::vector<int> uploaded_slots;
    // graphs
    bool use_graph = true;
    std::map<int, hipGraphExec_t> graphs;
    Profiler prof;
    std::vector<void*> allocs;
    // weight-only int8 (fm_llm_set_quant): packed T pointer of a linear -> its int8 form
    int quant = FM_QUANT_NONE;
    int q4_gs = 0;  // int4: group size along K
    int* fin_cnt = nullptr;   // split finalize_norm: [max rows][2] counters (zero between launches)
    float* fin_ss = nullptr;  //                      [max rows][16] chunk sums of squares
    struct QInfo {
        const unsigned char* q8 = nullptr;  // packed int8 (int4: 4-bit codes) decode-GEMV layout
        const void* scale = nullptr;        // int8: [rows padded to 16] in packed row order
        const uint32_t* sz = nullptr;       // int4: packed (scale, zero) per (tile, 128-k unit, row)
    };
    std::map<const void*, QInfo> qmap;
    std::map<const void*, void*> rowmajor;  // packed wo / w2 / wqkv -> row-major bf16 copy (int8 / int4: codes)
    std::map<const void*, const void*> rowsz;  // int4: packed -> its row-major (scale, zero) table
    std::map<const void*, const void*> rowscale;  // int8 w1 || w3: packed -> its row-block interleaved scales
    bool row_ok = false;                    // every layer of both stacks has wo / w2 row-major
    bool row_qkv_ok = false;                //                         ... and wqkv
    bool row_w13_ok = false;                //                         ... and w1 || w3
    uint32_t* fxt = nullptr;                // fused fast attention + wo: tagged attention words [nh * hd]
    void* fout_rm = nullptr;                // the codebook head row-major (int8 / int4: codes), row-block GEMV
    int32_t* fiota = nullptr;               // [16]: fiota[c] = c - 1 (the fast KV prefetch's last cached row)
    const QInfo* qinfo(const void* W) const {
        auto it = qmap.find(W);
        return it == qmap.end() ? nullptr : &it->second;
    }

    ~fm_llm() {
        if (device >= 0) (void)hipSetDevice(device);
        for (auto& g : graphs) (void)hipGraphExecDestroy(g.second);
        for (auto& kv : w) {
            if (kv.second.p) (void)hipFree(kv.second.p);
            if (kv.second.q) (void)hipFree(kv.second.q);
        }
        for (void* p : allocs) (void)hipFree(p);
        if (h_cols) (void)hipHostFree(h_cols);
        if (h_hist) (void)hipHostFree(h_hist);
        if (h_chain_err) (void)hipHostFree(h_chain_err);
        if (stream) (void)hipStreamDestroy(stream);
    }
    void* dalloc(size_t bytes, bool zero = true) {
        void* p = nullptr;
        if (bytes == 0) bytes = 16;
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess)
            throw FmError{FM_ERR_OOM, "hipMalloc(" + std::to_string(bytes) + ") failed: " + hipGetErrorString(e)};
        if (zero) HIPCHK(hipMemsetAsync(p, 0, bytes, stream));
        allocs.push_back(p);
        return p;
    }
};

// ------------------------------------------------------------------------------------------
// tensor inventory (names = reference state_dict keys after remap; llama.py module tree)
// ------------------------------------------------------------------------------------------
static void add_t(fm_llm* m, const std::string& n, int64_t rows, int64_t cols) {
    DTensor t;
    t.rows = rows;
    t.cols = cols;
    t.numel = rows * cols;
    m->w[n] = t;
}
static void add_stack(fm_llm* m, const std::string& pre, const StackDims& s) {
    for (int i = 0; i < s.n_layer; ++i) {
        std::string p = pre + std::to_string(i) + ".";
        add_t(m, p + "attention.wqkv.weight", s.nqkv(), s.dim);
        if (s.qkv_bias) add_t(m, p + "attention.wqkv.bias", 1, s.nqkv());
        add_t(m, p + "attention.wo.weight", s.dim, s.nq());
        if (s.o_bias) add_t(m, p + "attention.wo.bias", 1, s.dim);
        if (s.qk_norm) {
            add_t(m, p + "attention.q_norm.weight", 1, s.hd);
            add_t(m, p + "attention.k_norm.weight", 1, s.hd);
        }
        add_t(m, p + "feed_forward.w1.weight", s.inter, s.dim);
        add_t(m, p + "feed_forward.w3.weight", s.inter, s.dim);
        add_t(m, p + "feed_forward.w2.weight", s.dim, s.inter);
        add_t(m, p + "ffn_norm.weight", 1, s.dim);
        add_t(m, p + "attention_norm.weight", 1, s.dim);
    }
}

static void build_inventory(fm_llm* m) {
    const fm_model_config& c = m->c;
    m->sd = StackDims{c.n_layer, c.dim, c.n_head, c.n_local_heads, c.head_dim, c.intermediate_size,
                      c.qkv_bias, c.o_bias, c.qk_norm};
    m->fdm = StackDims{c.n_fast_layer, c.fast_dim, c.fast_n_head, c.fast_n_local_heads, c.fast_head_dim,
                       c.fast_intermediate_size, c.fast_qkv_bias, c.fast_o_bias, c.fast_qk_norm};
    add_t(m, "embeddings.weight", c.vocab_size, c.dim);
    add_t(m, "codebook_embeddings.weight", (int64_t)c.codebook_size * c.num_codebooks, c.dim);
    add_stack(m, "layers.", m->sd);
    add_t(m, "norm.weight", 1, c.dim);
    if (!c.tie_word_embeddings) add_t(m, "output.weight", c.vocab_size, c.dim);
    if (c.fast_dim != c.dim) {
        add_t(m, "fast_project_in.weight", c.fast_dim, c.dim);
        add_t(m, "fast_project_in.bias", 1, c.fast_dim);
    }
    add_t(m, "fast_embeddings.weight", c.codebook_size, c.fast_dim);
    add_stack(m, "fast_layers.", m->fdm);
    add_t(m, "fast_norm.weight", 1, c.fast_dim);
    add_t(m, "fast_output.weight", c.codebook_size, c.fast_dim);
}

static DTensor& tensor_for(fm_llm* m, const char* name, int64_t numel) {
    auto it = m->w.find(name);
    FMCHECK(it != m->w.end(), std::string("unknown tensor: ") + name);
    FMCHECK(it->second.numel == numel, std::string("wrong numel for ") + name + ": got " +
                                           std::to_string(numel) + ", want " + std::to_string(it->second.numel));
    DTensor& t = it->second;
    if (!t.p) {
        const int64_t rows = t.rows > 1 ? (t.rows + 15) / 16 * 16 : 1;
        const size_t bytes = (size_t)rows * t.cols * m->esz;
        HIPCHK(hipMalloc(&t.p, bytes));
        HIPCHK(hipMemsetAsync(t.p, 0, bytes, m->stream));
    }
    return t;
}

// ------------------------------------------------------------------------------------------
// kernels on a stack (slow or fast), templated on storage T
// ------------------------------------------------------------------------------------------
template <typename T> struct Run {
    typedef T type_t;
    fm_llm* m;
    hipStream_t s;
    int64_t E;  // element size
    bool rows_distinct_slots = false;  // slow_layers rows are one per slot (batched decode frame)
    explicit Run(fm_llm* mm) : m(mm), s(mm->stream), E(sizeof(T)) {}

    // Prompt chunks (R > 32 rows): a linear is a GEMM, not a weight stream, so it runs on the codec's
    // LDS-tiled implicit-GEMM kernels as a one-tap conv (conv_gemm2_kernel: 128-row x 96-128-column
    // tiles, or the 64 x 64 register tiles with split-K when the grid would not fill the chip).
    // The packed weight layout is the same; epilogues: round(acc + bias) and round(res + round(acc)).
    bool prompt_gemm(const void* W, const void* W2, const void* bias, const void* X, int ldx, int R, int N, int K,
                     void* Y, int ldy, const void* res, int ldr, int epi, const char* cls) {
        if (R <= 32 || W2 || m->qinfo(W) || !fm_tuning().prompt_gemm ||
            (epi != EPI_STORE && epi != EPI_RESID && epi != EPI_SWIGLU8) || N % 16 || K % 32 || N < 96 ||
            (epi == EPI_SWIGLU8 && (bias || N % 16)))
            return false;
        ConvArgs<T> c{};
        c.x = (const T*)X;
        c.ldx = ldx;
        c.Ci = K;
        c.Lq = R;
        c.Lx = R;
        c.w = (const T*)W;
        c.Co = N;
        c.ntaps = 1;
        c.stride = 1;
        c.nphase = 1;
        c.bias = (const T*)bias;
        c.res = epi == EPI_RESID ? (const T*)res : nullptr;
        c.ldr = ldr;
        c.out = Y;
        c.ldo = ldy;
        c.flags = CE_STORE | (bias ? CE_BIAS : 0) | (epi == EPI_RESID ? CE_RES : 0) |
                  (epi == EPI_SWIGLU8 ? CE_SWIGLU8 : 0);  // SWIGLU8: Y = act [R][N/2], ldy = N/2
        hipStream_t st = s;
        const int64_t bytes = (int64_t)N * K * E + (int64_t)R * K * E + (int64_t)R * N * E;
        const double flops = 2.0 * R * N * K;
        if constexpr (sizeof(T) == 2) {
            // R <= 64: one weight pass for all rows (fm_prompt.hip), K slices finished by the conv
            // split-K epilogue (the same roundings as below)
            auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
            const int ks = prompt_skinny_ks(N, K, fm_tuning().prompt_skinny_blocks);
            if (fm_tuning().prompt_skinny && ks > 0 && R <= 64 && ldx % 8 == 0 && al16(X) && al16(Y) && ldy % 8 == 0 &&
                (!c.res || (al16(c.res) && ldr % 8 == 0)) && (long long)ks * R * N <= m->skpart_cap) {
                c.ksplit = ks;
                c.slab = m->skpart;
                c.slab_cap = (size_t)m->skpart_cap;
                PromptSkinnyArgs p{(const bf16_t*)W, (const bf16_t*)X, ldx, R, N, K, m->skpart};
                const bool direct = ks == 1 && epi == EPI_SWIGLU8;  // the kernel stores act itself
                if (direct) {
                    p.act = (bf16_t*)Y;
                    p.lda = ldy;
                }
                auto go = [st, c, p, ks, direct] {
                    launch_prompt_skinny(st, p, ks);
                    if (!direct) launch_conv_epi<T>(st, c);
                };
                m->prof.record(cls, bytes, go);
                run_(cls, bytes, flops, go);
                return true;
            }
        }
        if (epi == EPI_SWIGLU8) return false;  // the conv GEMMs' own epilogues have no interleaved SwiGLU
        // split K (fp32 slabs + the conv split-K epilogue) until the 128 x 128 tiles number >=
        // prompt_ks_tiles (default 384)
        const long long t128 = (long long)FM_CEIL(R, 128) * FM_CEIL(N, 128);
        int ks = 1;
        while (t128 * ks < fm_tuning().prompt_ks_tiles && ks < fm_tuning().prompt_ks_max && K / 32 >= 8 * ks * 2)
            ks *= 2;
        c.ksplit = ks;
        c.slab = m->skpart;
        c.slab_cap = (size_t)m->skpart_cap;
        auto go = [st, c] { launch_conv_gemm<T>(st, c); };
        m->prof.record(cls, bytes, go);
        run_(cls, bytes, flops, go);
        return true;
    }
    // A prompt chunk's wo / w2 (32 < R <= 64, bf16) as raw K-slice partials in m->skpart ([ks][R][N], the
    // finalize_norm slab layout): the residual add, the bias and the next RMSNorm then run in one
    // finalize_norm launch instead of the split-K epilogue + an RMSNorm launch.  false: not eligible.
    bool prompt_slab(const void* W, const void* X, int ldx, int R, int N, int K, int* ks_out) {
        if constexpr (sizeof(T) != 2) {
            return false;
        } else {
            if (!fm_tuning().prompt_fin || !fm_tuning().prompt_skinny || !fm_tuning().prompt_gemm || R <= 32 ||
                R > 64 || m->qinfo(W) || N % 16 || K % 32 || ldx % 8 || ((uintptr_t)X & 15))
                return false;
            const int ks = prompt_skinny_ks(N, K, fm_tuning().prompt_skinny_blocks);
            if (ks <= 0 || (long long)ks * R * N > m->skpart_cap) return false;
            const PromptSkinnyArgs p{(const bf16_t*)W, (const bf16_t*)X, ldx, R, N, K, m->skpart};
            hipStream_t st = s;
            auto go = [st, p, ks] { launch_prompt_skinny(st, p, ks); };
            const int64_t bytes = (int64_t)N * K * E + (int64_t)R * K * E + (int64_t)ks * R * N * 4;
            m->prof.record("linear", bytes, go);
            run_("linear", bytes, 2.0 * R * N * K, go);
            *ks_out = ks;
            return true;
        }
    }
    void linear(const void* W, const void* W2, const void* bias, const void* X, int ldx, int R, int N,
                int K, void* Y, int ldy, const void* res, int ldr, float* Yf, int epi, const char* cls) {
        if (bs_use(R, false) && !W2 && !res && (epi == EPI_F32 || epi == EPI_STORE) &&
            bs_linear(W, bias, X, ldx, R, N, K, Y, ldy, Yf, epi))
            return;  // heads / fast_project_in of a batched frame
        if (prompt_gemm(W, W2, bias, X, ldx, R, N, K, Y, ldy, res, ldr, epi, cls)) return;
        LinearArgs<T> a{(const T*)W, (const T*)W2, (const T*)bias, (const T*)X, ldx, R, N, K, (T*)Y,
                        ldy, (const T*)res, ldr, Yf};
        if (const auto* q = m->qinfo(W)) a.wscale = (const T*)q->scale;
        if (R > GEMV_MAX_ROWS && R <= 64) {  // batched decode: split-K over the idle CUs
            FMCHECK(m->skpart_cap >= (long long)LINEAR_PART_CAP, "split-K partial buffer too small");
            a.part = m->skpart;
            a.tickets = m->tickets;
        }
        const int64_t wbytes = (int64_t)N * K * E * (epi == EPI_SWIGLU ? 2 : 1);
        const int64_t bytes = wbytes + (int64_t)R * K * E + (int64_t)R * N * (epi == EPI_F32 ? 4 : E);
        const double flops = 2.0 * R * N * K * (epi == EPI_SWIGLU ? 2 : 1);
        hipStream_t st = s;
        auto go = [st, a, epi] { launch_linear<T>(st, a, epi); };
        m->prof.record(cls, bytes, go);
        run_(cls, bytes, flops, go);
    }

    // TransformerBlock.forward (llama.py:838-843) on R rows; x is updated in place.
    // ---- batched decode (8 < R <= 32 rows, one per slot) on bstream_kernel (fm_bstream.hip) ----
    // Wo and W2 leave fp32 K-part slabs; finalize_norm_kernel sums them into the residual row and
    // applies the next RMSNorm, so W2's finalise is deferred to the next block's start (or flush()).
    struct BsPending {
        bool on = false;
        const float* slab = nullptr;
        int kparts = 0, d = 0, R = 0;
        void* res = nullptr;  // residual rows (h) ...
        void* out = nullptr;  // ... + round(sum of slabs) -> out (x)
        const void* sc = nullptr;  // weight-only int8 row scales of w2
    } pend;
    // slow-model decode attention: attn_dec3 (registers, 64 positions per block) for the batched
    // frame (B=32: 35.7 vs 38.1 us per layer), attn_decode2 (LDS tiles, 32-row blocks) at B <= 8,
    // where it is the faster of the two (B=1 frame 4.28 vs 4.52 ms)
    void attn_slow(const AttnDecArgs<T>& aa, int R) { attn_slow_on(s, aa, R); }
    static void attn_slow_on(hipStream_t s, const AttnDecArgs<T>& aa, int R) {
        if (fm_tuning().attn_fd && attn_fd_ok(aa.hd, aa.nh / aa.nkv)) {
            AttnDecArgs<T> b = aa;
            b.cap = std::max(16, R > GEMV_MAX_ROWS ? fm_tuning().fd_min_batched : fm_tuning().fd_min);
            if (R <= GEMV_MAX_ROWS && fm_tuning().fd_nw > 4) {
                b.nwb = fm_tuning().fd_nw;
                b.cap = std::max(16, fm_tuning().fd_min16);
            } else if (R > GEMV_MAX_ROWS && fm_tuning().fd_nw_batched > 4) {
                b.nwb = fm_tuning().fd_nw_batched;
            }
            launch_attn_fd<T>(s, b, R);
        } else if (fm_tuning().attn3 && R > GEMV_MAX_ROWS && aa.hd % 32 == 0 && aa.hd <= 128 && aa.nh / aa.nkv <= 6)
            launch_attn_decode3<T>(s, aa, R);
        else
            launch_attn_decode2<T>(s, aa, R);
    }
    bool bs_frame = false;  // inside a batched decode frame (rows are distinct slots)
    bool bs_use(int R, bool) const {
        return fm_tuning().bstream && bs_frame && R > GEMV_MAX_ROWS && R <= 32 && m->bsA;
    }
    // one bstream linear; returns false (nothing launched) when the shape is not eligible
    // bsacc_kernel's fused prologue / epilogue operands (the batched SLABFIN / PRENORM chain)
    struct BsExtra {
        int pro = PRO_PLAIN;
        const float* ss_in = nullptr;
        const void* nw = nullptr;
        const void* res = nullptr;
        void* res_out = nullptr;
        float* ss_out = nullptr;
    };
    bool bs_linear(const void* W, const void* bias, const void* X, int ldx, int R, int N, int K, void* Y, int ldy,
                   float* Yf, int epi, int* kparts_out = nullptr, const BsExtra* ex = nullptr) {
        const BstreamPlan p = bstream_plan(N, K, R, epi, E);
        if (!p.ok || ((epi == EPI_SLABFIN || (ex && ex->pro == PRO_PRENORM)) && !p.acc)) return false;
        BstreamArgs<T> a{(const T*)W, (const T*)bias, (const T*)X, ldx, R, N, K, (T*)Y, ldy, Yf};
        if (const auto* q = m->qinfo(W)) a.wscale = (const T*)q->scale;
        a.dbg = fm_tuning().dbg;
        if (ex) {
            a.pro = ex->pro;
            a.ss_in = ex->ss_in;
            a.nw = (const T*)ex->nw;
            a.eps = m->c.norm_eps;
            a.res = (const T*)ex->res;
            a.ldr = N;
            a.res_out = (T*)ex->res_out;
            a.ldro = N;
            a.ss_out = ex->ss_out;
            a.tickets = m->tickets;
        }
        const int64_t bytes = (int64_t)N * K * E + (int64_t)R * K * E +
                              (int64_t)R * N * (epi == EPI_SLAB ? 4 * p.kparts : (epi == EPI_F32 ? 4 : E));
        const double flops = 2.0 * R * N * K;
        hipStream_t st = s;
        auto go = [st, a, epi, p] { FMCHECK(launch_bstream<T>(st, a, epi, p), "bstream: no kernel for the plan"); };
        m->prof.record("linear", bytes, go);
        run_("linear", bytes, flops, go);
        if (kparts_out) *kparts_out = p.kparts;
        return true;
    }
    const void* wscale(const void* W) const {
        const auto* q = m->qinfo(W);
        return q ? q->scale : nullptr;
    }
    // The batched bf16 chain on bsacc_kernel (fm_tune bstream_chain): Wo and W2 finalise the residual
    // rows and their tile sums of squares (EPI_SLABFIN), QKV and W13 normalise in their prologue
    // (PRO_PRENORM) -- no finalize_norm launches.  Measured slower (B=32 frame 6.31 -> 6.75 ms): the
    // prologue's X rows and tile sums arrive ~7 us into the launch (scripts/b32_ts.py "xready"),
    // 3-4 us later than a plain prologue's, and the last K part's finalise adds 3-5 us to Wo / W2.
    // x_ss: the stack's x rows are final and m->ssX holds their tile sums.
    bool x_ss = false;
    bool bs_chain(const StackDims& d, int R) const {
        if (!fm_tuning().bstream_chain || E != 2 || R > 32) return false;
        auto ok = [&](int N, int K, int epi) { return bstream_plan(N, K, R, epi, E).acc; };
        return ok(d.nqkv(), d.dim, EPI_STORE) && ok(d.dim, d.nq(), EPI_SLABFIN) && ok(2 * d.inter, d.dim, EPI_SWIGLU8) &&
               ok(d.dim, d.inter, EPI_SLABFIN);
    }
    void finalize_norm(const float* slab, int kparts, const void* bias, const void* res, void* out, const void* nw,
                       void* xn, int d, int R, const void* sc) {
        FinalizeArgs<T> f{slab, kparts, d, (const T*)bias, (const T*)res, d, (T*)out, d, (const T*)nw,
                          m->c.norm_eps, (T*)xn, d, d, R, (const T*)sc};
        if (fm_tuning().fin_split > 1 && m->fin_cnt) {
            f.ch = fm_tuning().fin_split;
            f.cnt = m->fin_cnt;
            f.ss_part = m->fin_ss;
            f.err = m->chain_err;
        }
        run_("norm", 0, 0, [&] { launch_finalize_norm<T>(s, f); });
    }
    // finalise a W2 left pending by the last block of a stack (no norm)
    void flush() {
        if (!pend.on) return;
        pend.on = false;
        finalize_norm(pend.slab, pend.kparts, nullptr, pend.res, pend.out, nullptr, nullptr, pend.d, pend.R, pend.sc);
    }
    // the stack's input rows x are final unless a previous block left W2 pending on them
    void bs_norm_in(const StackDims& d, const LayerW& L, int R, void* xb, void* xnb) {
        if (pend.on) {
            FMCHECK(pend.out == xb && pend.R == R && pend.d == d.dim, "bstream: pending residual mismatch");
            pend.on = false;
            finalize_norm(pend.slab, pend.kparts, nullptr, pend.res, xb, L.an, xnb, d.dim, R, pend.sc);
        } else {
            run_("norm", 0, 0, [&] {
                launch_rmsnorm<T>(s, (const T*)xb, d.dim, (const T*)L.an, d.dim, m->c.norm_eps, (T*)xnb, d.dim, R);
            });
        }
    }

    void block(const StackDims& d, const LayerW& L, int R, const int* rslot, const int* rpos,
               int fixed_pos, bool is_fast, void* kc, void* vc, size_t sstride, size_t loff, int Sc,
               const float* rope, void* xb, void* hb, void* xnb) {
        const float eps = m->c.norm_eps;
        const float* qslab = nullptr;  // the QKV projection's K-part slabs (bs_qkv_slab) instead of m->qkv
        int qslab_kp = 1;
        const bool bs = bs_use(R, is_fast);
        const bool chain = bs && bs_chain(d, R);
        if (chain && x_ss) {  // QKV normalises x itself (attention_norm from the tile sums)
            BsExtra e;
            e.pro = PRO_PRENORM;
            e.ss_in = m->ssX;
            e.nw = L.an;
            FMCHECK(bs_linear(L.wqkv, L.bqkv, xb, d.dim, R, d.nqkv(), d.dim, m->qkv, d.nqkv(), nullptr, EPI_STORE,
                              nullptr, &e),
                    "bsacc: no PRENORM QKV plan");
        } else if (bs) {
            bs_norm_in(d, L, R, xb, xnb);
            // fm_tune bs_qkv_slab: K-part slabs (a grid of whole rounds: 384 QKV tiles x 2 parts over
            // 256 CUs) summed + biased + rounded by the fused attention that reads them
            int kp = 0;
            // (bsQ holds BS_KPARTS x 32 rows of either stack's width; the plan never exceeds those)
            // (only where the attention below is one of the fused kernels that read the slabs)
            const bool fused_fast = is_fast && fixed_pos >= 0 && fixed_pos < 16 && d.hd <= 256;
            const bool fused_slow = !is_fast && rows_distinct_slots && fm_tuning().attn_fd &&
                                    attn_fd_ok(d.hd, d.nh / d.nkv);
            // (weight-only int8 keeps the STORE epilogue: its row scales apply before the rounding)
            const bool slab_ok = fm_tuning().bs_qkv_slab && fm_tuning().batched_fused_attn && m->bsQ && R <= 32 &&
                                 (fused_fast || fused_slow) && !m->qinfo(L.wqkv);
            if (slab_ok && bs_linear(L.wqkv, nullptr, xnb, d.dim, R, d.nqkv(), d.dim, nullptr, d.nqkv(), m->bsQ,
                                     EPI_SLAB, &kp)) {
                qslab = m->bsQ;
                qslab_kp = kp;
            } else if (!bs_linear(L.wqkv, L.bqkv, xnb, d.dim, R, d.nqkv(), d.dim, m->qkv, d.nqkv(), nullptr, EPI_STORE))
                linear(L.wqkv, nullptr, L.bqkv, xnb, d.dim, R, d.nqkv(), d.dim, m->qkv, d.nqkv(), nullptr, 0,
                       nullptr, EPI_STORE, "linear");
        } else {
            bs_norm_in(d, L, R, xb, xnb);  // a prompt chunk's pending w2 (prompt_slab) finalised with this norm
            int kq = 0;
            // a prompt chunk's QKV as K-slice slabs, summed by qk_rope_cache_kernel itself (no epilogue launch)
            if (!is_fast && !rows_distinct_slots && fm_tuning().prompt_qkv_slab &&
                prompt_slab(L.wqkv, xnb, d.dim, R, d.nqkv(), d.dim, &kq)) {
                qslab = m->skpart;
                qslab_kp = kq;
            } else {
                linear(L.wqkv, nullptr, L.bqkv, xnb, d.dim, R, d.nqkv(), d.dim, m->qkv, d.nqkv(), nullptr, 0,
                       nullptr, EPI_STORE, "linear");
            }
        }
        const float scale = 1.0f / sqrtf((float)d.hd);
        // One row per slot (batched decode frames, every fast pass): the fused decode attention
        // kernels of the small-batch path do QK-norm, RoPE and the KV write themselves.  Prompt
        // chunks (rows of one slot, causal among themselves) keep the separate write + attention.
        const bool rows_are_slots = is_fast || rows_distinct_slots;
        if (rows_are_slots && !is_fast && fm_tuning().batched_fused_attn) {
            AttnDecArgs<T> aa{(const T*)m->qkv, d.nqkv(), rslot, rpos, d.nh, d.nkv, d.hd, d.qk_norm, eps,
                              (const T*)L.qn, (const T*)L.kn, rope, (T*)kc, (T*)vc, sstride, loff, Sc,
                              m->maxsplit, scale, m->part};
            aa.cap = attn2_cap(d.hd, d.nh / d.nkv, E);
            if (fm_tuning().attn_cap_batched) aa.cap = std::min(aa.cap, fm_tuning().attn_cap_batched);
            aa.maxsplit = FM_CEIL(Sc, aa.cap);
            aa.cnt = m->attn_cnt;
            aa.dbg = fm_tuning().dbg;
            aa.out = (T*)m->att;
            aa.qslab = qslab;
            aa.qslab_kp = qslab_kp;
            aa.qbias = (const T*)L.bqkv;
            FMCHECK(!qslab || (fm_tuning().attn_fd && attn_fd_ok(d.hd, d.nh / d.nkv)), "bs_qkv_slab needs attn_fd");
            hipStream_t st = s;
            auto go = [st, aa, R] { attn_slow_on(st, aa, R); };
            m->prof.record("attn_slow", 0, go);  // the slow model's launches alone (fm_llm_kernel_bench)
            run_rec("attn", go);
        } else if (is_fast && fm_tuning().batched_fused_attn && fixed_pos >= 0 && fixed_pos < 16 && d.hd <= 256) {
            FastFusedArgs<T> fa{(const T*)m->qkv, d.nqkv(), rslot, d.nh, d.nkv, d.hd, d.qk_norm, eps,
                                (const T*)L.qn, (const T*)L.kn, rope, (T*)kc, (T*)vc, sstride, loff, Sc,
                                fixed_pos, scale, (T*)m->att};
            fa.dbg = fm_tuning().dbg;
            fa.qslab = qslab;
            fa.qslab_kp = qslab_kp;
            fa.qbias = (const T*)L.bqkv;
            hipStream_t st = s;
            run_rec("attn", [st, fa, R] { launch_fast_attn2<T>(st, fa, R); });
        } else {
            QkArgs<T> qa{(const T*)m->qkv, d.nqkv(), rslot, rpos, fixed_pos, d.nh, d.nkv, d.hd, d.qk_norm,
                         eps, (const T*)L.qn, (const T*)L.kn, rope, (T*)m->q, (T*)kc, (T*)vc, sstride, loff, Sc};
            qa.qslab = qslab;
            qa.qslab_kp = qslab_kp;
            qa.qbias = (const T*)L.bqkv;
            run_("rope", 0, 0, [&] { launch_qk_rope_cache<T>(s, qa, R); });
            if (!is_fast) {
                // rows [r0, r0 + len) in pieces of <= ATTN_PIECE rows (rows are independent given the cache)
                auto attn_rows = [&](int r0, int len, bool one_slot) {
                    for (int p0 = r0; p0 < r0 + len; p0 += ATTN_PIECE) {
                        const int pn = std::min(ATTN_PIECE, r0 + len - p0);
                        const size_t o = (size_t)p0 * d.nh * d.hd;
                        AttnArgs<T> aa{(const T*)m->q + o, rslot + p0, rpos + p0, (const T*)kc, (const T*)vc, sstride,
                                       loff, Sc, d.nh, d.nkv, d.hd, ATTN_SPLIT, m->maxsplit, scale, m->part};
                        run_("attn", 0, 0, [&] { launch_attn<T>(s, aa, pn, m->maxsplit, (T*)m->att + o, one_slot); });
                    }
                };
                if (!segs.empty())  // a batched prefill chunk: attention per prompt segment
                    for (const auto& sg : segs) attn_rows(sg[0], sg[1], true);
                else
                    attn_rows(0, R, !rows_are_slots);
            } else {
                FastAttnArgs<T> fa{(const T*)m->q, rslot, (const T*)kc, (const T*)vc, sstride, loff, Sc,
                                   d.nh, d.nkv, d.hd, fixed_pos, scale, (T*)m->att};
                run_("attn", 0, 0, [&] { launch_fast_attn<T>(s, fa, R); });
            }
        }
        int kp = 0;
        if (chain) {
            BsExtra eo;  // h = x + wo(att), finalised with its tile sums by the last K part
            eo.res = xb;
            eo.res_out = hb;
            eo.ss_out = m->ssH;
            FMCHECK(bs_linear(L.wo, L.bo, m->att, d.nq(), R, d.dim, d.nq(), nullptr, d.dim, m->bsA, EPI_SLABFIN, &kp, &eo),
                    "bsacc: no SLABFIN wo plan");
            BsExtra e13;  // ffn_norm(h) in W1||W3's prologue
            e13.pro = PRO_PRENORM;
            e13.ss_in = m->ssH;
            e13.nw = L.fn;
            FMCHECK(bs_linear(L.w13, nullptr, hb, d.dim, R, 2 * d.inter, d.dim, m->act, d.inter, nullptr, EPI_SWIGLU8,
                              nullptr, &e13),
                    "bsacc: no PRENORM w13 plan");
            BsExtra e2;  // x = h + w2(act), finalised with its tile sums
            e2.res = hb;
            e2.res_out = xb;
            e2.ss_out = m->ssX;
            FMCHECK(bs_linear(L.w2, nullptr, m->act, d.inter, R, d.dim, d.inter, nullptr, d.dim, m->bsB, EPI_SLABFIN, &kp,
                              &e2),
                    "bsacc: no SLABFIN w2 plan");
            x_ss = true;
            return;
        }
        if (bs && bs_linear(L.wo, nullptr, m->att, d.nq(), R, d.dim, d.nq(), nullptr, d.dim, m->bsA, EPI_SLAB, &kp)) {
            finalize_norm(m->bsA, kp, L.bo, xb, hb, L.fn, xnb, d.dim, R, wscale(L.wo));  // h = x + wo(att); xn = ffn_norm(h)
        } else if (!bs && prompt_slab(L.wo, m->att, d.nq(), R, d.dim, d.nq(), &kp)) {
            finalize_norm(m->skpart, kp, L.bo, xb, hb, L.fn, xnb, d.dim, R, nullptr);  // h = x + wo(att); ffn_norm
        } else {
            linear(L.wo, nullptr, L.bo, m->att, d.nq(), R, d.dim, d.nq(), hb, d.dim, xb, d.dim, nullptr,
                   EPI_RESID, "linear");
            run_("norm", 0, 0, [&] {
                launch_rmsnorm<T>(s, (const T*)hb, d.dim, (const T*)L.fn, d.dim, eps, (T*)xnb, d.dim, R);
            });
        }
        if (!(bs && bs_linear(L.w13, nullptr, xnb, d.dim, R, 2 * d.inter, d.dim, m->act, d.inter, nullptr,
                              EPI_SWIGLU8))) {
            // a prompt chunk's w1 || w3 with the SwiGLU in its split-K epilogue (skinny path), else the
            // stored output and the SwiGLU launch
            if (!(fm_tuning().prompt_swiglu &&
                  prompt_gemm(L.w13, nullptr, nullptr, xnb, d.dim, R, 2 * d.inter, d.dim, m->act, d.inter, nullptr, 0,
                              EPI_SWIGLU8, "linear"))) {
                linear(L.w13, nullptr, nullptr, xnb, d.dim, R, 2 * d.inter, d.dim, m->act2, 2 * d.inter, nullptr, 0,
                       nullptr, EPI_STORE, "linear");
                run_("other", 0, 0, [&] {
                    launch_swiglu_i8<T>(s, (const T*)m->act2, 2 * d.inter, (T*)m->act, d.inter, d.inter, R);
                });
            }
        }
        if (bs && bs_linear(L.w2, nullptr, m->act, d.inter, R, d.dim, d.inter, nullptr, d.dim, m->bsB, EPI_SLAB, &kp)) {
            pend.on = true;  // x = h + w2(act): finalised by the next block's norm, or flush()
            pend.slab = m->bsB;
            pend.kparts = kp;
            pend.d = d.dim;
            pend.R = R;
            pend.res = hb;
            pend.out = xb;
            pend.sc = wscale(L.w2);
        } else if (!bs && prompt_slab(L.w2, m->act, d.inter, R, d.dim, d.inter, &kp)) {
            pend.on = true;  // x = h + w2(act): finalised with the next block's norm, or flush()
            pend.slab = m->skpart;
            pend.kparts = kp;
            pend.d = d.dim;
            pend.R = R;
            pend.res = hb;
            pend.out = xb;
            pend.sc = nullptr;
        } else {
            linear(L.w2, nullptr, nullptr, m->act, d.inter, R, d.dim, d.inter, xb, d.dim, hb, d.dim, nullptr,
                   EPI_RESID, "linear");
        }
    }

    // ---------------- small-batch (<= 8 streams) fused path --------------------------------
    GemvArgs<T> ga() {
        GemvArgs<T> a{};
        a.eps = m->c.norm_eps;
        a.dummy_tail = fm_tuning().gemv_dummy;
        return a;
    }
    // ---- batch-1 GEMV chain: consecutive GEMVs of one row are deferred and launched together
    // (gemv_chain_kernel), up to GEMV_CHAIN_MAX per launch; any other launch flushes them first
    struct ChainSt {
        GemvArgs<T> a;
        int kind;
        int64_t bytes;
        double flops;
    };
    std::vector<ChainSt> chain;
    int chain_kind(const GemvArgs<T>& a, int pro, int epi, int ksb) const {
        const FmTuning& t = fm_tuning();
        if (!t.gemv_chain || m->prof.on || ksb != 1 || a.R != 1 || a.Wq || m->qinfo(a.W) || !t.gemv_nt ||
            t.gemv_u != 8 || t.gemv_wpb != 4 || a.N % 16 || a.xidx)
            return -1;
        if (pro == PRO_PLAIN && epi == EPI_SLABFIN) return GEMV_CHAIN_WO_W2;
        if (a.xn_out || a.K > 4096 || pro != PRO_PRENORM) return a.xn_out && pro == PRO_PRENORM && epi == EPI_F32 &&
                                                                    a.K <= 4096 ? GEMV_CHAIN_HEAD : -1;
        if (epi == EPI_SWIGLU8) return GEMV_CHAIN_W13;
        if (epi == EPI_STORE) return GEMV_CHAIN_QKV;
        if (epi == EPI_F32) return GEMV_CHAIN_HEAD;
        return -1;
    }
    void chain_flush() {
        if (chain.empty()) return;
        std::vector<ChainSt> c;
        c.swap(chain);
        if (c.size() == 1) {
            static const int pro_of[4] = {PRO_PLAIN, PRO_PRENORM, PRO_PRENORM, PRO_PRENORM};
            static const int epi_of[4] = {EPI_SLABFIN, EPI_SWIGLU8, EPI_STORE, EPI_F32};
            gemv_now(c[0].a, pro_of[c[0].kind], epi_of[c[0].kind], 1, "linear");
            return;
        }
        GemvChainArgs<T> g{};
        int64_t bytes = 0;
        double flops = 0;
        g.n = (int)c.size();
        for (int i = 0; i < g.n; ++i) {
            g.st[i] = c[i].a;
            if (!g.st[i].tickets) g.st[i].tickets = m->tickets;
            g.kind[i] = c[i].kind;
            bytes += c[i].bytes;
            flops += c[i].flops;
        }
        g.cnt = m->chain_cnt;
        g.err = m->chain_err;
        g.sleep = fm_tuning().chain_sleep;
        hipStream_t st = s;
        auto go = [st, g] { launch_gemv_chain<T>(st, g); };
        m->prof.record("linear", bytes, go);
        m->prof.run(s, "linear", bytes, flops, go);
    }
    void gemv(GemvArgs<T> a, int pro, int epi, int ksb, const char* cls) {
        const int kind = chain_kind(a, pro, epi, ksb);
        if (kind < 0) {
            chain_flush();
            gemv_now(a, pro, epi, ksb, cls);
            return;
        }
        const size_t E = sizeof(T);
        const int64_t bytes = (int64_t)a.N * a.K * E + (int64_t)a.K * E;
        chain.push_back(ChainSt{a, kind, bytes, 2.0 * a.N * a.K});
        if ((int)chain.size() >= std::min(GEMV_CHAIN_MAX, fm_tuning().chain_max) || kind == GEMV_CHAIN_HEAD)
            chain_flush();
    }
    void gemv_now(GemvArgs<T> a, int pro, int epi, int ksb, const char* cls) {
        int64_t wbytes = (int64_t)a.N * a.K * E * (epi == EPI_SWIGLU ? 2 : 1);
        const auto* q = m->qinfo(a.W);
        if (q && q->sz && !fm_tuning().int4_stream) q = nullptr;  // int4 model on its dequantised bf16 weights
        if (q) {
            a.Wq = q->q8;
            if (q->sz) {  // weight-only int4: 4-bit codes + group (scale, zero), whole 128-k units per slice
                a.wsz = q->sz;
                a.wscale = nullptr;
                while (ksb > 1 && (a.K / ksb) % 128) ksb /= 2;
                wbytes = (int64_t)a.N * a.K / 2 + (int64_t)(a.N + 15) / 16 * 16 * (a.K / 128) * 4;
            } else {  // weight-only int8: the int8 stream, whole 64-k units per slice
                a.wscale = (const T*)q->scale;
                while (ksb > 1 && (a.K / ksb) % 64) ksb /= 2;
                wbytes = (int64_t)a.N * a.K;
            }
        }
        const int64_t bytes = wbytes + (int64_t)a.R * a.K * E;
        const double flops = 2.0 * a.R * a.N * a.K * (epi == EPI_SWIGLU ? 2 : 1);
        hipStream_t st = s;
        if (!a.tickets) a.tickets = m->tickets;
        auto go = [st, a, pro, epi, ksb] { launch_gemv<T>(st, a, pro, epi, ksb); };
        m->prof.record(cls, bytes, go);
        m->prof.run(s, cls, bytes, flops, go);
    }
    // batch-1 bf16 wo / w2 on the row-block GEMV (fm_rowgemv.hip: one block per pair of rows, every
    // CU busy); their RMSNorm consumers then take the statistic from the row they stage (ss_gran 1)
    // the row-block GEMV's enabled linears (fm_tune rowgemv; int4 models: rowgemv_q4)
    int row_bits() const {
        const FmTuning& t = fm_tuning();
        return m->quant == FM_QUANT_INT4 ? t.rowgemv_q4 : t.rowgemv;
    }
    bool row_fin(int n) const {
        const FmTuning& t = fm_tuning();
        return sizeof(T) == 2 && n == 1 && m->row_ok && (row_bits() & 1) && !t.gemv_chain && !t.attn_wo &&
               (m->quant != FM_QUANT_INT4 || t.int4_stream);
    }
    // ... and wqkv (norm prologue, 8 rows per block)
    bool row_qkv(int n) const {
        const FmTuning& t = fm_tuning();
        // (int8: the tile kernel's wqkv measured as fast, 3.12 vs 3.14 ms per frame)
        return sizeof(T) == 2 && n == 1 && m->row_qkv_ok && m->quant != FM_QUANT_INT8 && (row_bits() & 2) &&
               !t.gemv_chain && (m->quant != FM_QUANT_INT4 || t.int4_stream);
    }
    // ... and w1 || w3 (norm prologue, SwiGLU epilogue, 4 + 4 rows per block)
    bool row_w13(int n) const {
        const FmTuning& t = fm_tuning();
        return sizeof(T) == 2 && n == 1 && m->row_w13_ok && (row_bits() & 4) && !t.gemv_chain &&
               (m->quant != FM_QUANT_INT4 || t.int4_stream);
    }
    void rowgemv(const RowGemvArgs& a, int kind) {
        chain_flush();
        const int64_t wbytes = a.Wq4 ? (int64_t)a.N * a.K / 2 + (int64_t)a.N * (a.K / a.gs) * 4
                               : (a.Wq ? (int64_t)a.N * a.K + (int64_t)a.N * 2 : (int64_t)a.N * a.K * 2);
        const int64_t bytes = wbytes + (int64_t)a.K * 2;
        hipStream_t st = s;
        auto go = [st, a, kind] { launch_rowgemv(st, a, kind); };
        m->prof.record("linear", bytes, go);
        m->prof.run(s, "linear", bytes, 2.0 * a.N * a.K, go);
    }
    template <typename F> void run_(const char* cls, int64_t bytes, double flops, F&& f) {
        chain_flush();
        m->prof.run(s, cls, bytes, flops, std::forward<F>(f));
    }
    // run + record for fm_llm_kernel_bench: `go` must capture by value (it is replayed later)
    template <typename F> void run_rec(const char* cls, F go) {
        chain_flush();
        m->prof.record(cls, 0, go);
        m->prof.run(s, cls, 0, 0, go);
    }
    struct KsbPlan {
        int wo, w2;
    };
    // wo / w2 finalise the residual rows (EPI_SLABFIN): whole K per block (local finalise, no
    // cross-block hand-off) whenever the x slice fits the LDS budget, else split K
    KsbPlan plan(const StackDims& d, int n) {
        auto fin_ksb = [&](int N, int K) {
            const int fk = fm_tuning().fin_ksb;  // developer override (split-K factor)
            if (fk > 0 && K % (32 * fk) == 0) return fk;
            // (splitting K further to fill more CUs measured slower at B = 1: 4.37 -> 4.74 ms per
            // frame at 320 blocks, the split-K hand-off costs more than the idle CUs)
            return gemv_lds_bytes(n, K, E) <= 120 * 1024 ? 1 : pick_ksb(N, K, n, E);
        };
        return KsbPlan{fin_ksb(d.dim, d.nq()), fin_ksb(d.dim, d.inter)};
    }
    // one pre-norm block (TransformerBlock.forward, llama.py:838-843) on n rows.  Residual rows
    // are always finalised by the producing GEMV (EPI_SLABFIN: x / h in bf16 plus per-tile sums of
    // squares ssX / ssH), so every RMSNorm consumer is PRO_PRENORM.  x_in: the first layer's input
    // (plain rows, or an embedding table + xidx gather), whose norm is computed in place.
    // xo: where W2 writes the block's output row (xb itself unless the chain alternates buffers)
    void block_small(const StackDims& d, const LayerW& L, int n, bool first, const void* x_in, int ldx_in,
                     const int32_t* xidx, int xcol, void* xb, void* hb, bool is_fast, int cpos, int layer,
                     const KsbPlan& kp, void* xo, bool kv_only = false) {
        const int C1 = m->C1;
        const float scale = 1.0f / sqrtf((float)d.hd);
        FastFusedArgs<T> fa{(const T*)m->qkv, d.nqkv(), m->frame_slot, d.nh, d.nkv, d.hd, d.qk_norm,
                            m->c.norm_eps, (const T*)L.qn, (const T*)L.kn, m->frope, (T*)m->fkc,
                            (T*)m->fvc, m->fslot_stride, (size_t)layer * m->flayer_stride, m->C, cpos,
                            scale, (T*)m->att};
        fa.dbg = fm_tuning().dbg;
        // fast model: attention recomputed by every block of the Wo GEMV (PRO_FATT, one row) --
        // no attention launch (fm_tune attn_wo; measured slower, kept under test)
        const bool rf = row_fin(n);
        // the row-block GEMV's weight: bf16 row-major, or (weight-only int8) the codes + row scales
        auto row_w = [&](RowGemvArgs& r, void* rm, const void* packed) {
            if (m->quant == FM_QUANT_INT4) {
                r.Wq4 = (const uint32_t*)rm;
                r.wsz = (const uint32_t*)m->rowsz.at(packed);
                r.gs = m->q4_gs;
            } else if (m->quant) {
                r.Wq = (const int8_t*)rm;
                auto it = m->rowscale.find(packed);
                r.wscale = (const bf16_t*)(it != m->rowscale.end() ? it->second : m->qinfo(packed)->scale);
            } else {
                r.W = (const bf16_t*)rm;
            }
        };
        // fast model, batch 1: attention and wo as one launch (fm_rowgemv.hip fattn_wo_kernel)
        const int fq = m->quant == FM_QUANT_INT8 ? 1 : (m->quant == FM_QUANT_INT4 ? 2 : 0);
        const bool fw = is_fast && !kv_only && rf && fm_tuning().fattn_wo && m->fxt && m->fdm.n_layer * m->C >= 2 &&
                        m->fdm.n_layer * m->C <= 40 &&
                        fattn_wo_ok(d.nh, d.nkv, d.hd, cpos, d.dim, d.nq(), fq);
        const bool att_wo = is_fast && !kv_only && fm_tuning().attn_wo && !m->quant && n == 1 && cpos < 16 && d.hd % 16 == 0 &&
                            d.hd <= 128 && d.nh % d.nkv == 0 && (d.nq() / kp.wo) % d.hd == 0 && d.nqkv() % 8 == 0;
        // QKV (+ attention_norm)
        {
            GemvArgs<T> a = ga();
            a.W = (const T*)L.wqkv;
            a.bias = (const T*)L.bqkv;
            a.nw = (const T*)L.an;
            a.R = n;
            a.N = d.nqkv();
            a.K = d.dim;
            a.Y = (T*)m->qkv;
            a.ldy = d.nqkv();
            if (!is_fast && n == 1 && fm_tuning().kv_prefetch) {  // the attention's K / V rows into L2
                a.pf_kc = (const T*)m->kc;
                a.pf_vc = (const T*)m->vc;
                a.pf_slot = m->frame_slot;
                a.pf_pos = m->frame_pos;
                a.pf_slot_stride = m->slot_stride;
                a.pf_layer_off = (size_t)layer * m->layer_stride;
                a.pf_S = m->S;
                a.pf_nkv = d.nkv;
                a.pf_hd = d.hd;
            } else if (is_fast && n == 1 && fm_tuning().fkv_prefetch && m->fiota && cpos < 16) {
                // the fast attention's cached rows 0 .. cpos - 1 (fiota[cpos] = cpos - 1)
                a.pf_kc = (const T*)m->fkc;
                a.pf_vc = (const T*)m->fvc;
                a.pf_slot = m->frame_slot;
                a.pf_pos = m->fiota + cpos;
                a.pf_slot_stride = m->fslot_stride;
                a.pf_layer_off = (size_t)layer * m->flayer_stride;
                a.pf_S = m->C;
                a.pf_nkv = d.nkv;
                a.pf_hd = d.hd;
            }
            const int epi = EPI_STORE;
            if (row_qkv(n) && (!first || (row_bits() & 16))) {
                RowGemvArgs r{};
                row_w(r, L.wqkv_rm, L.wqkv);
                if (first) {  // the layer's input row itself (a table row gathered by xidx[xcol] at codebook > 0)
                    r.X = (const bf16_t*)x_in;
                    r.ldx = ldx_in;
                    r.xidx = xidx;
                    r.xcol = xcol;
                    r.xrows = xidx ? m->cb : 0;
                } else {
                    r.X = (const bf16_t*)xb;
                }
                r.bias = (const bf16_t*)L.bqkv;
                r.nw = (const bf16_t*)L.an;
                r.eps = m->c.norm_eps;
                r.Y = (bf16_t*)m->qkv;
                r.N = d.nqkv();
                r.K = d.dim;
                r.pf_kc = (const bf16_t*)a.pf_kc;
                r.pf_vc = (const bf16_t*)a.pf_vc;
                r.pf_slot = a.pf_slot;
                r.pf_pos = a.pf_pos;
                r.pf_slot_stride = a.pf_slot_stride;
                r.pf_layer_off = a.pf_layer_off;
                r.pf_S = a.pf_S;
                r.pf_nkv = a.pf_nkv;
                r.pf_hd = a.pf_hd;
                rowgemv(r, ROWGEMV_NORM_STORE);
            } else if (first) {
                a.X = (const T*)x_in;
                a.ldx = ldx_in;
                a.xidx = xidx;
                a.xidx_ld = C1;
                a.xidx_col = xcol;
                a.xidx_rows = xidx ? m->cb : 0;
                gemv(a, PRO_NORM, epi, 1, "linear");
            } else {
                a.X = (const T*)xb;
                a.ldx = d.dim;
                a.ss_in = m->ssX;
                a.ss_gran = rf ? 1 : 0;
                gemv(a, PRO_PRENORM, epi, 1, "linear");
            }
        }
        if (!is_fast) {
            AttnDecArgs<T> aa{(const T*)m->qkv, d.nqkv(), m->frame_slot, m->frame_pos, d.nh, d.nkv, d.hd,
                              d.qk_norm, m->c.norm_eps, (const T*)L.qn, (const T*)L.kn, m->rope, (T*)m->kc,
                              (T*)m->vc, m->slot_stride, (size_t)layer * m->layer_stride, m->S,
                              m->maxsplit, scale, m->part};
            aa.cap = attn2_cap(d.hd, d.nh / d.nkv, E);
            if (fm_tuning().attn_cap) aa.cap = std::min(aa.cap, fm_tuning().attn_cap);
            aa.maxsplit = FM_CEIL(m->S, aa.cap);
            aa.cnt = m->attn_cnt;
            aa.dbg = fm_tuning().dbg;
            aa.out = (T*)m->att;
            hipStream_t st = s;
            auto go = [st, aa, n] { attn_slow_on(st, aa, n); };
            m->prof.record("attn_slow", 0, go);  // the slow model's launches alone (fm_llm_kernel_bench)
            run_rec("attn", go);
        } else if (!att_wo && !fw) {
            hipStream_t st = s;
            const bool f2 = cpos < 16 && d.hd <= 256;
            run_rec("attn", [st, fa, n, f2] {
                if (f2)
                    launch_fast_attn2<T>(st, fa, n);
                else
                    launch_fast_attn_fused<T>(st, fa, n);
            });
        }
        // kv_only: the layer's K / V rows at cpos are all a later launch reads (the attention above
        // wrote them to the cache); its wo / feed-forward output would be discarded
        if (kv_only) return;
        // wo, split-K; the last block of each tile finalises h = x + wo(att) and its sums of squares
        if (fw) {
            FattnWoArgs A{};
            A.at = *reinterpret_cast<const FastFusedArgs<bf16_t>*>(&fa);
            A.at.dbg = nullptr;
            A.at.row_pos = m->frame_pos;
            RowGemvArgs& r = A.wo;
            row_w(r, L.wo_rm, L.wo);
            r.X = (const bf16_t*)m->att;  // (unused: x comes from the tagged words)
            r.bias = (const bf16_t*)L.bo;
            if (first) {
                r.res = (const bf16_t*)x_in;
                r.ldr = ldx_in;
                r.residx = xidx;
                r.res_col = xcol;
                r.res_rows = xidx ? m->cb : 0;
            } else {
                r.res = (const bf16_t*)xb;
                r.ldr = d.dim;
            }
            r.res_out = (bf16_t*)hb;
            r.N = d.dim;
            r.K = d.nq();
            A.xt = m->fxt;
            A.gen = 1 + layer + m->fdm.n_layer * cpos;  // <= 40 (fattn_wo_ok: cpos < 16, n_layer * C checked)
            A.err = m->chain_err;
            A.delay = fm_tuning().fw_delay;
            A.cheap = fm_tuning().fw_cheap;
            A.prio = fm_tuning().fw_prio;
            chain_flush();
            const int64_t bytes = r.Wq4 ? (int64_t)r.N * r.K / 2 + (int64_t)r.N * (r.K / r.gs) * 4
                                  : (r.Wq ? (int64_t)r.N * r.K + (int64_t)r.N * 2 : (int64_t)r.N * r.K * 2);
            hipStream_t st = s;
            auto go = [st, A] { launch_fattn_wo(st, A); };
            m->prof.record("attn_wo", bytes, go);  // (not "linear": attention + GEMV, reported apart)
            m->prof.run(s, "attn", bytes, 2.0 * r.N * r.K, go);
        } else if (rf) {
            RowGemvArgs r{};
            row_w(r, L.wo_rm, L.wo);
            r.X = (const bf16_t*)m->att;
            r.bias = (const bf16_t*)L.bo;
            if (first) {
                r.res = (const bf16_t*)x_in;
                r.ldr = ldx_in;
                r.residx = xidx;
                r.res_col = xcol;
                r.res_rows = xidx ? m->cb : 0;
            } else {
                r.res = (const bf16_t*)xb;
                r.ldr = d.dim;
            }
            r.res_out = (bf16_t*)hb;
            r.N = d.dim;
            r.K = d.nq();
            rowgemv(r, ROWGEMV_FIN);
        } else {
            GemvArgs<T> a = ga();
            a.W = (const T*)L.wo;
            a.bias = (const T*)L.bo;
            a.X = (const T*)m->att;
            a.ldx = d.nq();
            a.R = n;
            a.N = d.dim;
            a.K = d.nq();
            a.Yf = m->slabA;
            a.ldy = d.dim;
            if (first) {
                a.res = (const T*)x_in;
                a.ldr = ldx_in;
                a.residx = xidx;
                a.xidx_ld = C1;
                a.xidx_col = xcol;
                a.xidx_rows = xidx ? m->cb : 0;
            } else {
                a.res = (const T*)xb;
                a.ldr = d.dim;
            }
            a.res_out = (T*)hb;
            a.ldro = d.dim;
            a.ss_out = m->ssH;
            a.tickets = m->tickets;
            if (att_wo) {
                a.att = fa;
                gemv(a, PRO_FATT, EPI_SLABFIN, kp.wo, "linear");
            } else {
                gemv(a, PRO_PLAIN, EPI_SLABFIN, kp.wo, "linear");
            }
        }
        // W1/W3 (+ ffn_norm) -> SwiGLU act
        if (row_w13(n)) {
            RowGemvArgs r{};
            row_w(r, L.w13_rm, L.w13);
            r.X = (const bf16_t*)hb;
            r.nw = (const bf16_t*)L.fn;
            r.eps = m->c.norm_eps;
            r.Y = (bf16_t*)m->act;
            r.N = 2 * d.inter;
            r.K = d.dim;
            rowgemv(r, ROWGEMV_NORM_SWIGLU);
        } else {
            GemvArgs<T> a = ga();
            a.W = (const T*)L.w13;
            a.nw = (const T*)L.fn;
            a.R = n;
            a.N = 2 * d.inter;
            a.K = d.dim;
            a.X = (const T*)hb;
            a.ldx = d.dim;
            a.ss_in = m->ssH;
            a.ss_gran = rf ? 1 : 0;
            a.Y = (T*)m->act;
            a.ldy = d.inter;
            gemv(a, PRO_PRENORM, EPI_SWIGLU8, 1, "linear");
        }
        // W2, split-K; finalises the block output x = h + w2(act) into xb and its sums of squares
        if (rf) {
            RowGemvArgs r{};
            row_w(r, L.w2_rm, L.w2);
            r.X = (const bf16_t*)m->act;
            r.res = (const bf16_t*)hb;
            r.ldr = d.dim;
            r.res_out = (bf16_t*)xo;
            r.N = d.dim;
            r.K = d.inter;
            rowgemv(r, ROWGEMV_FIN);
        } else {
            GemvArgs<T> a = ga();
            a.W = (const T*)L.w2;
            a.X = (const T*)m->act;
            a.ldx = d.inter;
            a.R = n;
            a.N = d.dim;
            a.K = d.inter;
            a.Yf = m->slabB;
            a.ldy = d.dim;
            a.res = (const T*)hb;
            a.ldr = d.dim;
            a.res_out = (T*)xo;
            a.ldro = d.dim;
            a.ss_out = m->ssX;
            a.tickets = m->tickets;
            gemv(a, PRO_PLAIN, EPI_SLABFIN, kp.w2, "linear");
        }
    }

    // the residual row of layer l: x (in place) or, in chain mode, x / x2 alternating
    void* xbuf(void* x0, void* x1, int l) const { return (fm_tuning().gemv_chain && (l & 1)) ? x1 : x0; }
    void* xfin = nullptr;  // the slow stack's output row (head_small's input when pending)
    void slow_small(int n) {
        const KsbPlan kp = plan(m->sd, n);
        for (int l = 0; l < m->sd.n_layer; ++l)
            block_small(m->sd, m->slow[l], n, l == 0, m->x, m->c.dim, nullptr, 0, xbuf(m->x, m->x2, l), m->h, false, 0,
                        l, kp, xbuf(m->x, m->x2, l + 1));
        xfin = xbuf(m->x, m->x2, m->sd.n_layer);
    }

    // final norm (+ pending residual) -> constrained head logits and the fast-model hidden
    const void* head_small(const void* xlast, bool pending, int n, int ksb_prev) {
        const fm_model_config& c = m->c;
        GemvArgs<T> a = ga();
        a.W = (const T*)m->head_c;
        a.nw = (const T*)m->norm;
        a.R = n;
        a.N = m->Nhead;
        a.K = c.dim;
        a.Yf = m->logits;
        a.ldy = m->Nhead;
        a.xn_out = (T*)m->xnl;
        a.ldxo = c.dim;
        const void* xs = xfin ? xfin : m->x;
        if (pending) {  // the last slow layer's W2 finalised x (xs) and its sums of squares
            a.X = (const T*)xs;
            a.ldx = c.dim;
            a.ss_in = m->ssX;
            a.ss_gran = row_fin(n) ? 1 : 0;
            gemv(a, PRO_PRENORM, EPI_F32, 1, "linear");
        } else {
            a.X = (const T*)xlast;
            a.ldx = c.dim;
            gemv(a, PRO_NORM, EPI_F32, 1, "linear");
        }
        const void* hid = c.norm_fastlayer_input ? m->xnl : (pending ? xs : xlast);
        if (m->fproj_w) {
            GemvArgs<T> p = ga();
            p.W = (const T*)m->fproj_w;
            p.bias = (const T*)m->fproj_b;
            p.X = (const T*)hid;
            p.ldx = c.dim;
            p.R = n;
            p.N = c.fast_dim;
            p.K = c.dim;
            p.Y = (T*)m->xl;
            p.ldy = c.fast_dim;
            gemv(p, PRO_PLAIN, EPI_STORE, 1, "linear");
            return m->xl;
        }
        return hid;
    }

    void fast_small(int n, int cc, bool with_head, const void* hidden) {
        const fm_model_config& c = m->c;
        const KsbPlan kp = plan(m->fdm, n);
        for (int l = 0; l < m->fdm.n_layer; ++l) {
            const bool first = l == 0;
            const void* xin = cc == 0 ? hidden : m->femb;
            const int32_t* xidx = cc == 0 ? nullptr : m->cols;
            // codebook 0's pass (no head: inference.py:148-149 discards its output) only fills the fast
            // KV cache, so its last layer stops once its K / V rows are cached (fm_tune fast_tail)
            const bool kv_only = !with_head && l == m->fdm.n_layer - 1 && fm_tuning().fast_tail;
            block_small(m->fdm, m->fast[l], n, first, xin, c.fast_dim, xidx, cc, xbuf(m->fx, m->fx2, l), m->fh, true,
                        cc, l, kp, xbuf(m->fx, m->fx2, l + 1), kv_only);
        }
        if (with_head && sizeof(T) == 2 && n == 1 && m->fout_rm && (row_bits() & 8) && !fm_tuning().gemv_chain &&
            (m->quant != FM_QUANT_INT4 || fm_tuning().int4_stream)) {
            RowGemvArgs r{};  // the codebook head on the row-block GEMV (norm prologue, fp32 logits)
            auto row_w = [&](RowGemvArgs& rr, void* rm, const void* packed) {
                if (m->quant == FM_QUANT_INT4) {
                    rr.Wq4 = (const uint32_t*)rm;
                    rr.wsz = (const uint32_t*)m->rowsz.at(packed);
                    rr.gs = m->q4_gs;
                } else if (m->quant) {
                    rr.Wq = (const int8_t*)rm;
                    rr.wscale = (const bf16_t*)m->qinfo(packed)->scale;
                } else {
                    rr.W = (const bf16_t*)rm;
                }
            };
            row_w(r, m->fout_rm, m->fout);
            r.X = (const bf16_t*)xbuf(m->fx, m->fx2, m->fdm.n_layer);
            r.nw = (const bf16_t*)m->fnorm;
            r.eps = c.norm_eps;
            r.Yf = m->flogits;
            r.N = m->cb;
            r.K = c.fast_dim;
            rowgemv(r, ROWGEMV_NORM_F32);
        } else if (with_head) {
            GemvArgs<T> a = ga();
            a.W = (const T*)m->fout;
            a.nw = (const T*)m->fnorm;
            a.R = n;
            a.N = m->cb;
            a.K = c.fast_dim;
            a.Yf = m->flogits;
            a.ldy = m->cb;
            a.X = (const T*)xbuf(m->fx, m->fx2, m->fdm.n_layer);
            a.ldx = c.fast_dim;
            a.ss_in = m->ssX;
            a.ss_gran = row_fin(n) ? 1 : 0;
            gemv(a, PRO_PRENORM, EPI_F32, 1, "linear");
        }
    }

    void frame_tail_small(int n, bool ras_enable, bool sample, const void* hidden) {
        if (sample) {
            SampleArgs a = sargs(true, ras_enable, 0);
            run_("sample", 0, 0, [&] { launch_sample_radix<T>(s, a, n); });
        }
        fast_small(n, 0, false, hidden);  // position 0 fills the fast KV cache; logits discarded
        for (int cc = 1; cc < m->C; ++cc) {
            fast_small(n, cc, true, hidden);
            if (sample) {
                SampleArgs a = sargs(false, 0, cc);
                run_("sample", 0, 0, [&] { launch_sample_radix<T>(s, a, n); });
            }
        }
    }

    void decode_frame_small(int n) {
        run_("other", 0, 0, [&] {
            launch_embed<T>(s, m->tok_in, n, (const T*)m->emb, (const T*)m->cbemb, m->c.dim, m->C, m->cb,
                            m->c.semantic_begin_id, m->c.semantic_end_id, m->c.scale_codebook_embeddings,
                            (T*)m->x, m->frame_slot);
        });
        slow_small(n);
        const KsbPlan kp = plan(m->sd, n);
        const void* hid = head_small(nullptr, true, n, kp.w2);
        frame_tail_small(n, true, true, hid);
        chain_flush();
        launch_finish(s, n, m->frame_slot, m->frame_pos, m->cols, m->C1, m->tok_in, m->ras, m->C1 * 10, m->C1,
                      1, m->sp);
    }

    void slow_layers(int R, const int* rslot, const int* rpos) {
        x_ss = false;
        for (int l = 0; l < m->sd.n_layer; ++l)
            block(m->sd, m->slow[l], R, rslot, rpos, -1, false, m->kc, m->vc, m->slot_stride,
                  (size_t)l * m->layer_stride, m->S, m->rope, m->x, m->h, m->xn);
        flush();
    }

    // final norm -> constrained head logits; hidden for the fast model (llama.py:447-466, 826)
    void head_and_hidden(const void* xlast, int n) {
        const fm_model_config& c = m->c;
        chain_flush();
        run_("norm", 0, 0, [&] {
            launch_rmsnorm<T>(s, (const T*)xlast, c.dim, (const T*)m->norm, c.dim, c.norm_eps, (T*)m->xnl,
                              c.dim, n);
        });
        linear(m->head_c, nullptr, nullptr, m->xnl, c.dim, n, m->Nhead, c.dim, nullptr, m->Nhead,
               nullptr, 0, m->logits, EPI_F32, "linear");
        const void* src = c.norm_fastlayer_input ? m->xnl : xlast;
        if (m->fproj_w)
            linear(m->fproj_w, nullptr, m->fproj_b, src, c.dim, n, c.fast_dim, c.dim, m->fx, c.fast_dim,
                   nullptr, 0, nullptr, EPI_STORE, "linear");
        else
            HIPCHK(hipMemcpyAsync(m->fx, src, (size_t)n * c.dim * E, hipMemcpyDeviceToDevice, s));
    }

    void fast_pass(int n, int cpos, bool with_head) {
        const fm_model_config& c = m->c;
        x_ss = false;
        for (int l = 0; l < m->fdm.n_layer; ++l)
            block(m->fdm, m->fast[l], n, m->frame_slot, nullptr, cpos, true, m->fkc, m->fvc,
                  m->fslot_stride, (size_t)l * m->flayer_stride, m->C, m->frope, m->fx, m->fh, m->fxn);
        flush();
        if (with_head) {
            run_("norm", 0, 0, [&] {
                launch_rmsnorm<T>(s, (const T*)m->fx, c.fast_dim, (const T*)m->fnorm, c.fast_dim,
                                  c.norm_eps, (T*)m->fxn, c.fast_dim, n);
            });
            linear(m->fout, nullptr, nullptr, m->fxn, c.fast_dim, n, m->cb, c.fast_dim, nullptr, m->cb,
                   nullptr, 0, m->flogits, EPI_F32, "linear");
        }
    }

    SampleArgs sargs(bool slow, int ras_enable, int c) {
        const fm_model_config& cc = m->c;
        SampleArgs a{};
        a.logits = slow ? m->logits : m->flogits;
        a.ldl = slow ? m->Nhead : m->cb;
        a.Nl = a.ldl;
        a.row_slot = m->frame_slot;
        a.sp = m->sp;
        a.ras = m->ras;
        a.ras_stride = m->C1 * 10;
        a.ras_enable = ras_enable;
        a.slow = slow;
        a.sb = cc.semantic_begin_id;
        a.se = cc.semantic_end_id;
        a.im_end = cc.im_end_id;
        a.cb = m->cb;
        a.draw = 1 + c;
        a.col_idx = c + 1;
        a.cols = m->cols;
        a.ldc = m->C1;
        a.dbg = fm_tuning().dbg;
        a.force_cols = m->force_cols;
        a.tap = slow ? m->tap_slow : m->tap_fast + (size_t)(c - 1) * m->cb;
        a.tap_ld = slow ? m->Nhead : (m->C - 1) * m->cb;
        return a;
    }

    // tail of decode_one_token_ar after the slow forward: sample, fast AR over codebooks
    void frame_tail(int n, bool ras_enable, bool sample) {
        if (sample) {
            SampleArgs a = sargs(true, ras_enable, 0);
            run_("sample", 0, 0, [&] { launch_sample_radix<T>(s, a, n); });
        }
        fast_pass(n, 0, false);  // position 0: fills the fast KV cache, logits discarded
        for (int cc = 1; cc < m->C; ++cc) {
            run_("other", 0, 0, [&] {
                launch_gather_rows<T>(s, m->cols, m->C1, cc, (const T*)m->femb, m->c.fast_dim, m->cb, n, (T*)m->fx);
            });
            fast_pass(n, cc, true);
            if (sample) {
                SampleArgs a = sargs(false, 0, cc);
                run_("sample", 0, 0, [&] { launch_sample_radix<T>(s, a, n); });
            }
        }
    }

    void decode_frame(int n) {
        if (n <= GEMV_MAX_ROWS) {
            decode_frame_small(n);
            return;
        }
        run_("other", 0, 0, [&] {
            launch_embed<T>(s, m->tok_in, n, (const T*)m->emb, (const T*)m->cbemb, m->c.dim, m->C, m->cb,
                            m->c.semantic_begin_id, m->c.semantic_end_id, m->c.scale_codebook_embeddings,
                            (T*)m->x, m->frame_slot);
        });
        rows_distinct_slots = true;
        bs_frame = true;
        slow_layers(n, m->frame_slot, m->frame_pos);
        rows_distinct_slots = false;
        head_and_hidden(m->x, n);
        frame_tail(n, true, true);
        bs_frame = false;
        chain_flush();
        launch_finish(s, n, m->frame_slot, m->frame_pos, m->cols, m->C1, m->tok_in, m->ras, m->C1 * 10,
                      m->C1, 1, m->sp);
    }

    // runs the prompt through the slow model (chunks), leaves the last row in m->x[row]
    const void* prefill_slow(int slot, const int32_t* tokens, int Tn, int pos0) {
        const int C1 = m->C1;
        std::vector<int32_t> rows((size_t)PREFILL_CHUNK * C1);
        std::vector<int> rs(PREFILL_CHUNK, slot), rp(PREFILL_CHUNK);
        int last = 0;
        for (int t0 = 0; t0 < Tn; t0 += PREFILL_CHUNK) {
            const int R = std::min(PREFILL_CHUNK, Tn - t0);
            for (int r = 0; r < R; ++r) {
                for (int q = 0; q < C1; ++q) rows[(size_t)r * C1 + q] = tokens[(size_t)q * Tn + t0 + r];
                rp[r] = pos0 + t0 + r;
            }
            chain_flush();
            HIPCHK(hipMemcpyAsync(m->ptok, rows.data(), (size_t)R * C1 * 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(m->prow_slot, rs.data(), (size_t)R * 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(m->prow_pos, rp.data(), (size_t)R * 4, hipMemcpyHostToDevice, s));
            launch_embed<T>(s, m->ptok, R, (const T*)m->emb, (const T*)m->cbemb, m->c.dim, m->C, m->cb,
                            m->c.semantic_begin_id, m->c.semantic_end_id, m->c.scale_codebook_embeddings,
                            (T*)m->x, nullptr);
            slow_layers(R, m->prow_slot, m->prow_pos);
            last = R - 1;
            HIPCHK(hipStreamSynchronize(s));  // host vectors reused by the next chunk
        }
        return (const char*)m->x + (size_t)last * m->c.dim * E;
    }

    // Several prompts (one slot each, positions from 0) through the slow stack together: their rows
    // packed into PREFILL_CHUNK-row chunks, so every linear is one GEMM over all of them (a prompt
    // may span chunks: its earlier rows are in the KV cache by then); the attention runs per prompt
    // segment (segs); the last row of prompt i is copied to plast row i.
    std::vector<std::array<int, 2>> segs;  // (first row, rows) of each prompt inside the current chunk
    void prefill_multi(int n, const int32_t* slots, const int32_t* const* toks, const int* Ts) {
        const int C1 = m->C1, dim = m->c.dim;
        std::vector<int32_t> rows((size_t)PREFILL_CHUNK * C1);
        std::vector<int> rs(PREFILL_CHUNK), rp(PREFILL_CHUNK);
        int i = 0, t = 0;  // next (prompt, position) to place
        while (i < n) {
            int R = 0;
            segs.clear();
            std::vector<std::array<int, 2>> lasts;  // (prompt, row) of prompts ending in this chunk
            while (R < PREFILL_CHUNK && i < n) {
                const int take = std::min(PREFILL_CHUNK - R, Ts[i] - t);
                segs.push_back({R, take});
                for (int r = 0; r < take; ++r) {
                    for (int q = 0; q < C1; ++q) rows[(size_t)(R + r) * C1 + q] = toks[i][(size_t)q * Ts[i] + t + r];
                    rs[R + r] = slots[i];
                    rp[R + r] = t + r;
                }
                R += take;
                t += take;
                if (t == Ts[i]) {
                    lasts.push_back({i, R - 1});
                    ++i;
                    t = 0;
                }
            }
            chain_flush();
            HIPCHK(hipMemcpyAsync(m->ptok, rows.data(), (size_t)R * C1 * 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(m->prow_slot, rs.data(), (size_t)R * 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(m->prow_pos, rp.data(), (size_t)R * 4, hipMemcpyHostToDevice, s));
            launch_embed<T>(s, m->ptok, R, (const T*)m->emb, (const T*)m->cbemb, dim, m->C, m->cb,
                            m->c.semantic_begin_id, m->c.semantic_end_id, m->c.scale_codebook_embeddings,
                            (T*)m->x, nullptr);
            slow_layers(R, m->prow_slot, m->prow_pos);
            chain_flush();
            for (const auto& l : lasts)
                HIPCHK(hipMemcpyAsync((char*)m->plast + (size_t)l[0] * dim * E, (const char*)m->x + (size_t)l[1] * dim * E,
                                      (size_t)dim * E, hipMemcpyDeviceToDevice, s));
            segs.clear();
            HIPCHK(hipStreamSynchronize(s));  // host vectors reused by the next chunk
        }
    }
};

// ------------------------------------------------------------------------------------------
// finalize: validate weights, derive pointers, allocate caches / buffers
// ------------------------------------------------------------------------------------------
static void* W(fm_llm* m, const std::string& n) {
    auto it = m->w.find(n);
    FMCHECK(it != m->w.end() && it->second.set, "tensor not set: " + n);
    return it->second.p;
}
static void* Wopt(fm_llm* m, const std::string& n) {
    auto it = m->w.find(n);
    return (it != m->w.end() && it->second.set) ? it->second.p : nullptr;
}

static bool is_linear_weight(const std::string& n) {
    auto ends = [&](const char* suf) {
        const size_t L = strlen(suf);
        return n.size() >= L && n.compare(n.size() - L, L, suf) == 0;
    };
    return ends("attention.wqkv.weight") || ends("attention.wo.weight") || ends("feed_forward.w1.weight") ||
           ends("feed_forward.w2.weight") || ends("feed_forward.w3.weight") || n == "fast_output.weight" ||
           n == "fast_project_in.weight";
}

// every nn.Linear of the model (WeightOnlyInt8QuantHandler quantizes them all, quantize.py:190-206);
// the tied head is F.linear on the embedding table, not a module, and stays in T
static bool is_quant_linear(const std::string& n) { return is_linear_weight(n) || n == "output.weight"; }
static std::string base_of(const std::string& n) { return n.substr(0, n.size() - strlen(".weight")); }

// int8 row-major [rows][cols] (rows padded to 16) -> packed int8 decode-GEMV layout
static void* pack_q8_dev(fm_llm* m, const void* q, int rows, int cols) {
    FMCHECK(cols % 64 == 0, "int8 weights need in_features % 64 == 0");
    void* dst = nullptr;
    HIPCHK(hipMalloc(&dst, (size_t)(rows + 15) / 16 * 16 * cols));
    launch_pack_q8(m->stream, (const int8_t*)q, rows, cols, (int8_t*)dst);
    HIPCHK(hipGetLastError());
    m->allocs.push_back(dst);
    return dst;
}

// int4: codes row-major [rows][cols] + sz [rows][cols / gs] -> the packed GEMV stream and its
// (scale, zero) table; none (the bf16 dequantised copy serves every kernel) unless the group size
// and K are whole 128-k units
static fm_llm::QInfo pack_q4_dev(fm_llm* m, const void* q, const void* sz, int rows, int cols) {
    if (m->q4_gs % 128 || cols % 128) return fm_llm::QInfo{};
    const size_t tiles = (size_t)(rows + 15) / 16;
    void* dq = nullptr;
    void* ds = nullptr;
    HIPCHK(hipMalloc(&dq, tiles * 16 * cols / 2));
    HIPCHK(hipMalloc(&ds, tiles * (cols / 128) * 16 * 4));
    launch_pack_q4(m->stream, (const uint8_t*)q, rows, cols, (uint8_t*)dq);
    launch_pack_sz4(m->stream, (const uint32_t*)sz, rows, cols, m->q4_gs, (uint32_t*)ds);
    HIPCHK(hipGetLastError());
    m->allocs.push_back(dq);
    m->allocs.push_back(ds);
    return fm_llm::QInfo{(const unsigned char*)dq, nullptr, (const uint32_t*)ds};
}

// int8 mode, before packing: every quantized linear ends with t.p = T(q) row-major (what the
// T-fragment kernels read), t.q = int8 row-major, t.s = row scales.  int8 checkpoints supply q and
// "<name>.scales"; float weights are quantized here with quantize.py's per-channel rule.
static void quantize_linears(fm_llm* m) {
    if (m->quant == FM_QUANT_INT4) {  // every linear: codes, group (scale, zero), dequantised bf16 in place
        for (auto& kv : m->w) {
            if (!is_quant_linear(kv.first)) continue;
            DTensor& t = kv.second;
            const size_t rp = (size_t)(t.rows + 15) / 16 * 16;
            HIPCHK(hipMalloc(&t.q, rp * t.cols));
            HIPCHK(hipMemsetAsync(t.q, 8, rp * t.cols, m->stream));
            void* sz = nullptr;
            HIPCHK(hipMalloc(&sz, rp * (t.cols / m->q4_gs) * 4));
            HIPCHK(hipMemsetAsync(sz, 0, rp * (t.cols / m->q4_gs) * 4, m->stream));
            t.s = sz;
            launch_quant4(m->stream, (bf16_t*)t.p, (int)t.rows, (int)t.cols, m->q4_gs, (uint8_t*)t.q, (uint32_t*)sz);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipStreamSynchronize(m->stream));
        return;
    }
    for (auto& kv : m->w) {
        if (!is_quant_linear(kv.first)) continue;
        DTensor& t = kv.second;
        const size_t rp = (size_t)(t.rows + 15) / 16 * 16;
        DTensor& sc = m->w.at(base_of(kv.first) + ".scales");
        if (t.q) {
            FMCHECK(sc.set, "int8 weight without scales: " + kv.first);
            FMCHECK(!t.p, "tensor set twice: " + kv.first);
            HIPCHK(hipMalloc(&t.p, rp * t.cols * m->esz));
            if (m->prec == FM_PREC_BF16)
                launch_i8_to<bf16_t>(m->stream, (const int8_t*)t.q, (int64_t)rp * t.cols, (bf16_t*)t.p);
            else
                launch_i8_to<float>(m->stream, (const int8_t*)t.q, (int64_t)rp * t.cols, (float*)t.p);
            t.s = sc.p;
        } else {
            FMCHECK(!sc.set, "scales given with a float weight: " + kv.first);
            HIPCHK(hipMalloc(&t.q, rp * t.cols));
            HIPCHK(hipMemsetAsync(t.q, 0, rp * t.cols, m->stream));
            t.s = m->dalloc(rp * m->esz);
            if (m->prec == FM_PREC_BF16)
                launch_quant_rows<bf16_t>(m->stream, (bf16_t*)t.p, (int)t.rows, (int)t.cols, (int8_t*)t.q, (bf16_t*)t.s);
            else
                launch_quant_rows<float>(m->stream, (float*)t.p, (int)t.rows, (int)t.cols, (int8_t*)t.q, (float*)t.s);
        }
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(m->stream));
}

// row-major [rows][cols] device tensor -> packed fragment layout (fm_kernels.h)
static void* pack_dev(fm_llm* m, const void* src, int rows, int cols) {
    const size_t n = (size_t)(rows + 15) / 16 * 16 * cols;
    void* dst = nullptr;
    HIPCHK(hipMalloc(&dst, n * m->esz));
    if (m->prec == FM_PREC_BF16)
        launch_pack<bf16_t>(m->stream, (const bf16_t*)src, rows, cols, (bf16_t*)dst);
    else
        launch_pack<float>(m->stream, (const float*)src, rows, cols, (float*)dst);
    HIPCHK(hipGetLastError());
    return dst;
}

// bf16 wo / w2 / wqkv whose shapes the row-block GEMV takes keep their row-major copy
// (fm_rowgemv.hip; ~3.7 GB at S2-Pro beside the packed tiles the batched paths read)
// fm_tune row_copies 0: a row-major copy only where the rowgemv bits in force at finalize use it
static bool row_bits(fm_llm* m, int bits) {
    const FmTuning& t = fm_tuning();
    return t.row_copies || ((m->quant == FM_QUANT_INT4 ? t.rowgemv_q4 : t.rowgemv) & bits) != 0;
}
static bool row_keep(fm_llm* m, const std::string& n, int rows, int cols) {
    auto ends = [&](const char* suf) {
        const size_t L = strlen(suf);
        return n.size() >= L && n.compare(n.size() - L, L, suf) == 0;
    };
    // bf16: the T row-major weight; weight-only int8: the int8 row-major codes (rowgemv QM 1)
    const int qm = m->quant == FM_QUANT_INT8 ? 1 : (m->quant == FM_QUANT_INT4 ? 2 : 0);
    if (m->prec != FM_PREC_BF16 || rowgemv_u(cols, qm) == 0) return false;
    if (qm == 2 && (m->q4_gs % 8 || cols % m->q4_gs)) return false;
    if (ends("attention.wo.weight") || ends("feed_forward.w2.weight")) return rows % 2 == 0 && row_bits(m, 1);
    if (n == "fast_output.weight") return rows % 8 == 0 && rowgemv_u(cols, qm) <= 8 && row_bits(m, 8);
    return ends("attention.wqkv.weight") && rows % 8 == 0 && rowgemv_u(cols, qm) <= 8 && row_bits(m, 2 | 16);
}

static bool is_ffn_w13(const std::string& n) {
    auto ends = [&](const char* suf) {
        const size_t L = strlen(suf);
        return n.size() >= L && n.compare(n.size() - L, L, suf) == 0;
    };
    return ends("feed_forward.w1.weight") || ends("feed_forward.w3.weight");
}

// W1 [inter][dim] and W3 -> one packed [2*inter][dim] matrix whose 16-row tiles hold 8 rows of W1
// then the same 8 rows of W3, so one GEMV tile (EPI_SWIGLU8) has both halves of 8 SwiGLU outputs and
// the decode grid is 2*inter/16 single-matrix blocks.  The row-major W1/W3 are freed; their map
// entries keep the shapes (the packed matrix hangs off the w1 entry).
static void* pack_w13(fm_llm* m, const std::string& p, int inter, int dim) {
    FMCHECK(inter % 8 == 0, "intermediate_size must be a multiple of 8");
    DTensor& t1 = m->w.at(p + "feed_forward.w1.weight");
    DTensor& t3 = m->w.at(p + "feed_forward.w3.weight");
    const size_t E = m->esz, rb = (size_t)dim * E;
    void* tmp = nullptr;
    HIPCHK(hipMalloc(&tmp, 2 * (size_t)inter * rb));
    HIPCHK(hipMemcpy2DAsync(tmp, 16 * rb, t1.p, 8 * rb, 8 * rb, inter / 8, hipMemcpyDeviceToDevice, m->stream));
    HIPCHK(hipMemcpy2DAsync((char*)tmp + 8 * rb, 16 * rb, t3.p, 8 * rb, 8 * rb, inter / 8, hipMemcpyDeviceToDevice,
                            m->stream));
    void* pk = pack_dev(m, tmp, 2 * inter, dim);
    // the row-block GEMV's copy (fm_rowgemv.hip ROWGEMV_NORM_SWIGLU): row-major, rows 4b .. 4b+3 of W1
    // then the same rows of W3, per 8-row block (bf16 rows, or int8 codes + scales, or int4 packed
    // code words + (scale, zero) rows)
    const int qm = m->quant == FM_QUANT_INT8 ? 1 : (m->quant == FM_QUANT_INT4 ? 2 : 0);
    const bool rk = m->prec == FM_PREC_BF16 && inter % 4 == 0 && rowgemv_u(dim, qm) > 0 && rowgemv_u(dim, qm) <= 8 &&
                    (qm != 2 || (m->q4_gs % 8 == 0 && dim % m->q4_gs == 0)) && row_bits(m, 4);
    auto il4 = [&](const void* a1, const void* a3, size_t rb4) -> void* {  // rb4: bytes per row
        void* d = m->dalloc(2 * (size_t)inter * rb4, false);
        HIPCHK(hipMemcpy2DAsync(d, 8 * rb4, a1, 4 * rb4, 4 * rb4, inter / 4, hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpy2DAsync((char*)d + 4 * rb4, 8 * rb4, a3, 4 * rb4, 4 * rb4, inter / 4, hipMemcpyDeviceToDevice,
                                m->stream));
        return d;
    };
    if (rk && qm == 0) m->rowmajor[pk] = il4(t1.p, t3.p, rb);
    if (rk && qm == 1) {
        m->rowmajor[pk] = il4(t1.q, t3.q, (size_t)dim);
        m->rowscale[pk] = il4(t1.s, t3.s, E);
    }
    if (rk && qm == 2) {
        void* codes = nullptr;  // one byte per code, interleaved, then packed to row words
        HIPCHK(hipMalloc(&codes, 2 * (size_t)inter * dim));
        HIPCHK(hipMemcpy2DAsync(codes, 8 * (size_t)dim, t1.q, 4 * (size_t)dim, 4 * (size_t)dim, inter / 4,
                                hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpy2DAsync((char*)codes + 4 * (size_t)dim, 8 * (size_t)dim, t3.q, 4 * (size_t)dim, 4 * (size_t)dim,
                                inter / 4, hipMemcpyDeviceToDevice, m->stream));
        void* words = m->dalloc((size_t)inter * dim, false);
        launch_pack_q4_rows(m->stream, (const uint8_t*)codes, 2 * inter, dim, (uint32_t*)words);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(m->stream));
        HIPCHK(hipFree(codes));
        m->rowmajor[pk] = words;
        m->rowsz[pk] = il4(t1.s, t3.s, (size_t)(dim / m->q4_gs) * 4);
    }
    if (m->quant == FM_QUANT_INT4) {  // the same interleave of the code rows and of the (scale, zero) rows
        const size_t gb = (size_t)(dim / m->q4_gs) * 4;
        void* qt = nullptr;
        void* st = nullptr;
        HIPCHK(hipMalloc(&qt, 2 * (size_t)inter * dim));
        HIPCHK(hipMalloc(&st, 2 * (size_t)inter * gb));
        HIPCHK(hipMemcpy2DAsync(qt, 16 * (size_t)dim, t1.q, 8 * (size_t)dim, 8 * (size_t)dim, inter / 8,
                                hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpy2DAsync((char*)qt + 8 * (size_t)dim, 16 * (size_t)dim, t3.q, 8 * (size_t)dim,
                                8 * (size_t)dim, inter / 8, hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpy2DAsync(st, 16 * gb, t1.s, 8 * gb, 8 * gb, inter / 8, hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpy2DAsync((char*)st + 8 * gb, 16 * gb, t3.s, 8 * gb, 8 * gb, inter / 8, hipMemcpyDeviceToDevice,
                                m->stream));
        const fm_llm::QInfo qi = pack_q4_dev(m, qt, st, 2 * inter, dim);
        if (qi.q8) m->qmap[pk] = qi;
        HIPCHK(hipStreamSynchronize(m->stream));
        for (void* p : {qt, st, t1.q, t3.q, t1.s, t3.s}) HIPCHK(hipFree(p));
        t1.q = t3.q = nullptr;
        t1.s = t3.s = nullptr;
    } else if (m->quant) {  // the same interleave of the int8 rows and of the row scales
        void* qt = nullptr;
        HIPCHK(hipMalloc(&qt, 2 * (size_t)inter * dim));
        HIPCHK(hipMemcpy2DAsync(qt, 16 * (size_t)dim, t1.q, 8 * (size_t)dim, 8 * (size_t)dim, inter / 8,
                                hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpy2DAsync((char*)qt + 8 * (size_t)dim, 16 * (size_t)dim, t3.q, 8 * (size_t)dim,
                                8 * (size_t)dim, inter / 8, hipMemcpyDeviceToDevice, m->stream));
        void* s13 = m->dalloc(2 * (size_t)inter * E);
        HIPCHK(hipMemcpy2DAsync(s13, 16 * E, t1.s, 8 * E, 8 * E, inter / 8, hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpy2DAsync((char*)s13 + 8 * E, 16 * E, t3.s, 8 * E, 8 * E, inter / 8, hipMemcpyDeviceToDevice,
                                m->stream));
        m->qmap[pk] = fm_llm::QInfo{(const unsigned char*)pack_q8_dev(m, qt, 2 * inter, dim), s13};
        HIPCHK(hipStreamSynchronize(m->stream));
        HIPCHK(hipFree(qt));
        HIPCHK(hipFree(t1.q));
        HIPCHK(hipFree(t3.q));
        t1.q = t3.q = nullptr;
    }
    HIPCHK(hipStreamSynchronize(m->stream));
    HIPCHK(hipFree(tmp));
    HIPCHK(hipFree(t1.p));
    HIPCHK(hipFree(t3.p));
    t1.p = pk;
    t3.p = nullptr;
    return pk;
}

static void finalize(fm_llm* m) {
    if (m->finalized) return;
    const fm_model_config& c = m->c;
    bsacc_init();
    sample_init();
    for (auto& kv : m->w) FMCHECK(kv.second.set || kv.second.optional, "tensor not set: " + kv.first);
    if (m->quant) quantize_linears(m);
    for (auto& kv : m->w) {
        if (!is_linear_weight(kv.first) || is_ffn_w13(kv.first)) continue;  // W1/W3: pack_w13 below
        DTensor& t = kv.second;
        void* pk = pack_dev(m, t.p, (int)t.rows, (int)t.cols);
        if (m->quant == FM_QUANT_INT4) {
            const fm_llm::QInfo qi = pack_q4_dev(m, t.q, t.s, (int)t.rows, (int)t.cols);
            if (qi.q8) m->qmap[pk] = qi;
            const bool keep = row_keep(m, kv.first, (int)t.rows, (int)t.cols);
            if (keep) {  // the codes as packed row-major words + the row-major (scale, zero) table
                void* rw = m->dalloc((size_t)t.rows * t.cols / 2, false);
                launch_pack_q4_rows(m->stream, (const uint8_t*)t.q, (int)t.rows, (int)t.cols, (uint32_t*)rw);
                HIPCHK(hipGetLastError());
                m->rowmajor[pk] = rw;
                m->rowsz[pk] = t.s;
                m->allocs.push_back(const_cast<void*>(t.s));
            }
            HIPCHK(hipStreamSynchronize(m->stream));
            HIPCHK(hipFree(t.q));
            if (!keep) HIPCHK(hipFree(const_cast<void*>(t.s)));
            t.q = nullptr;
            t.s = nullptr;
        } else if (m->quant) {
            m->qmap[pk] = fm_llm::QInfo{(const unsigned char*)pack_q8_dev(m, t.q, (int)t.rows, (int)t.cols), t.s};
            HIPCHK(hipStreamSynchronize(m->stream));
            if (row_keep(m, kv.first, (int)t.rows, (int)t.cols)) {
                m->rowmajor[pk] = t.q;  // the int8 codes, row-major, for the row-block GEMV
                m->allocs.push_back(t.q);
            } else {
                HIPCHK(hipFree(t.q));
            }
            t.q = nullptr;
        }
        HIPCHK(hipStreamSynchronize(m->stream));
        if (!m->quant && row_keep(m, kv.first, (int)t.rows, (int)t.cols)) {
            m->rowmajor[pk] = t.p;  // kept for the batch-1 row-pair GEMV
            m->allocs.push_back(t.p);
        } else {
            HIPCHK(hipFree(t.p));
        }
        t.p = pk;
    }
    auto stack = [&](const std::string& pre, const StackDims& d, std::vector<LayerW>& out) {
        out.resize(d.n_layer);
        for (int i = 0; i < d.n_layer; ++i) {
            std::string p = pre + std::to_string(i) + ".";
            LayerW& L = out[i];
            L.wqkv = W(m, p + "attention.wqkv.weight");
            L.bqkv = Wopt(m, p + "attention.wqkv.bias");
            L.wo = W(m, p + "attention.wo.weight");
            L.bo = Wopt(m, p + "attention.wo.bias");
            L.qn = Wopt(m, p + "attention.q_norm.weight");
            L.kn = Wopt(m, p + "attention.k_norm.weight");
            L.w13 = pack_w13(m, p, d.inter, d.dim);
            L.w2 = W(m, p + "feed_forward.w2.weight");
            L.an = W(m, p + "attention_norm.weight");
            L.fn = W(m, p + "ffn_norm.weight");
            auto rm = [&](const void* pk) -> void* {
                auto it = m->rowmajor.find(pk);
                return it == m->rowmajor.end() ? nullptr : it->second;
            };
            L.wo_rm = rm(L.wo);
            L.w2_rm = rm(L.w2);
            L.wqkv_rm = rm(L.wqkv);
            L.w13_rm = rm(L.w13);
        }
    };
    stack("layers.", m->sd, m->slow);
    stack("fast_layers.", m->fdm, m->fast);
    {
        int32_t io[16];
        for (int c = 0; c < 16; ++c) io[c] = c - 1;
        m->fiota = (int32_t*)m->dalloc(sizeof(io), false);
        HIPCHK(hipMemcpy(m->fiota, io, sizeof(io), hipMemcpyHostToDevice));
    }
    if (m->prec == FM_PREC_BF16)
        m->fxt = (uint32_t*)m->dalloc((size_t)m->fdm.nh * m->fdm.hd * sizeof(uint32_t));  // tags 0: never current
    m->row_ok = m->row_qkv_ok = m->row_w13_ok = true;
    for (auto* st : {&m->slow, &m->fast})
        for (const LayerW& L : *st) {
            m->row_ok = m->row_ok && L.wo_rm && L.w2_rm;
            m->row_qkv_ok = m->row_qkv_ok && L.wqkv_rm;
            m->row_w13_ok = m->row_w13_ok && L.w13_rm;
        }
    if (m->quant) {  // WeightOnlyInt8Linear has no bias (quantize.py:206-229): the checkpoint's are unused
        for (auto* st : {&m->slow, &m->fast})
            for (LayerW& L : *st) L.bqkv = L.bo = nullptr;
    }
    m->emb = W(m, "embeddings.weight");
    m->cbemb = W(m, "codebook_embeddings.weight");
    m->norm = W(m, "norm.weight");
    m->fproj_w = Wopt(m, "fast_project_in.weight");
    m->fproj_b = m->quant ? nullptr : Wopt(m, "fast_project_in.bias");
    m->femb = W(m, "fast_embeddings.weight");
    m->fnorm = W(m, "fast_norm.weight");
    m->fout = W(m, "fast_output.weight");
    {
        auto it = m->rowmajor.find(m->fout);
        m->fout_rm = it == m->rowmajor.end() ? nullptr : it->second;
    }
    // constrained head (inference.py:308-320): only the semantic rows + <|im_end|> can be
    // finite after the bias, so the LM head streams exactly those rows.
    const void* outw = c.tie_word_embeddings ? m->emb : W(m, "output.weight");
    m->nsem = c.semantic_end_id - c.semantic_begin_id + 1;
    m->Nhead = m->nsem + 1;
    FMCHECK(m->Nhead <= 8192, "constrained head wider than 8192 rows is not supported");
    const size_t rowb = (size_t)c.dim * m->esz;
    void* head_rm = m->dalloc((size_t)(m->Nhead + 15) / 16 * 16 * rowb);
    HIPCHK(hipMemcpyAsync(head_rm, (const char*)outw + (size_t)c.semantic_begin_id * rowb,
                          (size_t)m->nsem * rowb, hipMemcpyDeviceToDevice, m->stream));
    HIPCHK(hipMemcpyAsync((char*)head_rm + (size_t)m->nsem * rowb,
                          (const char*)outw + (size_t)c.im_end_id * rowb, rowb, hipMemcpyDeviceToDevice,
                          m->stream));
    m->head_c = pack_dev(m, head_rm, m->Nhead, c.dim);
    m->allocs.push_back(m->head_c);
    if (m->quant == FM_QUANT_INT4 && !c.tie_word_embeddings) {  // the compact rows of the codes and groups
        DTensor& o = m->w.at("output.weight");
        const size_t gb = (size_t)(c.dim / m->q4_gs) * 4;
        void* hq = nullptr;
        void* hs = nullptr;
        HIPCHK(hipMalloc(&hq, (size_t)(m->Nhead + 15) / 16 * 16 * c.dim));
        HIPCHK(hipMalloc(&hs, (size_t)(m->Nhead + 15) / 16 * 16 * gb));
        HIPCHK(hipMemcpyAsync(hq, (const char*)o.q + (size_t)c.semantic_begin_id * c.dim, (size_t)m->nsem * c.dim,
                              hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpyAsync((char*)hq + (size_t)m->nsem * c.dim, (const char*)o.q + (size_t)c.im_end_id * c.dim,
                              c.dim, hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpyAsync(hs, (const char*)o.s + (size_t)c.semantic_begin_id * gb, (size_t)m->nsem * gb,
                              hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpyAsync((char*)hs + (size_t)m->nsem * gb, (const char*)o.s + (size_t)c.im_end_id * gb, gb,
                              hipMemcpyDeviceToDevice, m->stream));
        const fm_llm::QInfo qi = pack_q4_dev(m, hq, hs, m->Nhead, c.dim);
        if (qi.q8) m->qmap[m->head_c] = qi;
        HIPCHK(hipStreamSynchronize(m->stream));
        for (void* p : {hq, hs, o.q, o.s}) HIPCHK(hipFree(p));
        o.q = o.s = nullptr;
    } else if (m->quant && !c.tie_word_embeddings) {  // the same compact rows of the int8 head and its scales
        DTensor& o = m->w.at("output.weight");
        void* hq = m->dalloc((size_t)(m->Nhead + 15) / 16 * 16 * c.dim);
        HIPCHK(hipMemcpyAsync(hq, (const char*)o.q + (size_t)c.semantic_begin_id * c.dim, (size_t)m->nsem * c.dim,
                              hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpyAsync((char*)hq + (size_t)m->nsem * c.dim, (const char*)o.q + (size_t)c.im_end_id * c.dim,
                              c.dim, hipMemcpyDeviceToDevice, m->stream));
        void* hs = m->dalloc((size_t)(m->Nhead + 15) / 16 * 16 * m->esz);
        HIPCHK(hipMemcpyAsync(hs, (const char*)o.s + (size_t)c.semantic_begin_id * m->esz, (size_t)m->nsem * m->esz,
                              hipMemcpyDeviceToDevice, m->stream));
        HIPCHK(hipMemcpyAsync((char*)hs + (size_t)m->nsem * m->esz, (const char*)o.s + (size_t)c.im_end_id * m->esz,
                              m->esz, hipMemcpyDeviceToDevice, m->stream));
        m->qmap[m->head_c] = fm_llm::QInfo{(const unsigned char*)pack_q8_dev(m, hq, m->Nhead, c.dim), hs};
        HIPCHK(hipStreamSynchronize(m->stream));
        HIPCHK(hipFree(o.q));
        o.q = nullptr;
    }
    // caches [slot][layer][kv][S][hd]
    const StackDims& d = m->sd;
    m->layer_stride = (size_t)d.nkv * m->S * d.hd;
    m->slot_stride = m->layer_stride * d.n_layer;
    m->kc = m->dalloc(m->slot_stride * m->max_slots * m->esz);
    m->vc = m->dalloc(m->slot_stride * m->max_slots * m->esz);
    const StackDims& f = m->fdm;
    m->flayer_stride = (size_t)f.nkv * m->C * f.hd;
    m->fslot_stride = m->flayer_stride * f.n_layer;
    m->fkc = m->dalloc(m->fslot_stride * m->max_slots * m->esz);
    m->fvc = m->dalloc(m->fslot_stride * m->max_slots * m->esz);
    auto rt = rope_table_host(m->S, d.hd, c.rope_base);
    m->rope = (float*)m->dalloc(rt.size() * 4, false);
    HIPCHK(hipMemcpy(m->rope, rt.data(), rt.size() * 4, hipMemcpyHostToDevice));
    auto frt = rope_table_host(m->C, f.hd, c.rope_base);
    m->frope = (float*)m->dalloc(frt.size() * 4, false);
    HIPCHK(hipMemcpy(m->frope, frt.data(), frt.size() * 4, hipMemcpyHostToDevice));
    // activations
    const int R = m->Rmax = std::max(m->max_slots, PREFILL_CHUNK);
    const int dmax = std::max(c.dim, c.fast_dim);
    const int qkvmax = std::max(d.nqkv(), f.nqkv()), qmax = std::max(d.nq(), f.nq());
    const int imax = std::max(d.inter, f.inter);
    const size_t E = m->esz;
    m->x = m->dalloc((size_t)R * dmax * E);
    m->h = m->dalloc((size_t)R * dmax * E);
    m->xn = m->dalloc((size_t)R * dmax * E);
    m->qkv = m->dalloc((size_t)R * qkvmax * E);
    m->q = m->dalloc((size_t)R * qmax * E);
    m->att = m->dalloc((size_t)R * qmax * E);
    m->act = m->dalloc((size_t)R * imax * E);
    m->act2 = m->dalloc((size_t)R * 2 * imax * E);
    const int n = m->max_slots;
    m->xl = m->dalloc((size_t)n * dmax * E);
    m->plast = m->dalloc((size_t)n * dmax * E);
    m->xnl = m->dalloc((size_t)n * dmax * E);
    m->fx = m->dalloc((size_t)n * dmax * E);
    m->fh = m->dalloc((size_t)n * dmax * E);
    m->fxn = m->dalloc((size_t)n * dmax * E);
    m->x2 = m->dalloc((size_t)std::min(n, GEMV_MAX_ROWS) * dmax * E);
    m->fx2 = m->dalloc((size_t)std::min(n, GEMV_MAX_ROWS) * dmax * E);
    m->chain_cnt = (unsigned*)m->dalloc(GEMV_CHAIN_WORDS * sizeof(unsigned));
    m->chain_err = (int*)m->dalloc(16 * sizeof(int));
    HIPCHK(hipHostMalloc((void**)&m->h_chain_err, 16 * sizeof(int), hipHostMallocDefault));
    m->h_chain_err[0] = 0;
    m->maxsplit = FM_CEIL(m->S, ATTN_SPLIT);
    const int Rpart = std::max(m->max_slots, ATTN_PIECE);  // decode rows, or one prompt attention piece
    m->part = (float*)m->dalloc((size_t)Rpart * d.nh * std::max(m->maxsplit, FM_CEIL(m->S, 16)) * (d.hd + 2) * 4, false);
    m->attn_cnt = (int*)m->dalloc((size_t)R * d.nkv * sizeof(int));  // tickets: zeroed
    m->ssX = (float*)m->dalloc((size_t)(dmax / 16) * std::min(n, 32) * 4);  // batched chain: up to 32 rows
    m->ssH = (float*)m->dalloc((size_t)(dmax / 16) * std::min(n, 32) * 4);
    {
        // arrival counters: one per 16-row tile of the largest decode GEMV (the slow head / W13)
        const int maxn = std::max({m->Nhead, 2 * c.intermediate_size, 2 * c.fast_intermediate_size, qkvmax, dmax, m->cb});  // W1||W3 is one 2*I-row linear on the batched path
        m->tickets = (int*)m->dalloc((size_t)(maxn / 16 + 16) * sizeof(int));
        m->fin_cnt = (int*)m->dalloc((size_t)std::max(m->max_slots, 64) * 2 * sizeof(int));
        m->fin_ss = (float*)m->dalloc((size_t)std::max(m->max_slots, 64) * 16 * sizeof(float));
        m->skpart_cap = 16ll << 20;  // 64 MiB of partial tiles (prompt GEMM slabs: 256 rows x 2 x 19456)
        m->skpart = (float*)m->dalloc((size_t)m->skpart_cap * sizeof(float), false);
    }
    HIPCHK(hipMemsetAsync(m->attn_cnt, 0, (size_t)R * d.nkv * sizeof(int), m->stream));
    m->slabA = (float*)m->dalloc((size_t)KSB_MAX * std::min(n, GEMV_MAX_ROWS) * dmax * 4);
    m->slabB = (float*)m->dalloc((size_t)KSB_MAX * std::min(n, GEMV_MAX_ROWS) * dmax * 4);
    if (n > GEMV_MAX_ROWS) {  // [BS_KPARTS][32][dmax] fp32 each
        m->bsA = (float*)m->dalloc((size_t)BS_KPARTS * 32 * dmax * 4, false);
        m->bsB = (float*)m->dalloc((size_t)BS_KPARTS * 32 * dmax * 4, false);
        m->bsQ = (float*)m->dalloc((size_t)BS_KPARTS * 32 * std::max(m->sd.nqkv(), m->fdm.nqkv()) * 4, false);
    }
    m->logits = (float*)m->dalloc((size_t)n * m->Nhead * 4);
    m->flogits = (float*)m->dalloc((size_t)n * m->cb * 4);
    m->frame_slot = (int*)m->dalloc(n * 4);
    m->frame_pos = (int*)m->dalloc(n * 4);
    m->prow_slot = (int*)m->dalloc(PREFILL_CHUNK * 4);
    m->prow_pos = (int*)m->dalloc(PREFILL_CHUNK * 4);
    m->tok_in = (int32_t*)m->dalloc((size_t)n * m->C1 * 4);
    m->cols = (int32_t*)m->dalloc((size_t)n * m->C1 * 4);
    m->ptok = (int32_t*)m->dalloc((size_t)PREFILL_CHUNK * m->C1 * 4);
    m->ras = (int32_t*)m->dalloc((size_t)n * m->C1 * 10 * 4);
    m->sp = (SlotParams*)m->dalloc(sizeof(SlotParams) * n);
    m->force_cols = (int32_t*)m->dalloc((size_t)n * m->C1 * 4);
    m->tap_slow = (float*)m->dalloc((size_t)n * m->Nhead * 4);
    m->tap_fast = (float*)m->dalloc((size_t)n * std::max(m->C - 1, 1) * m->cb * 4);
    m->host_force.assign(n, 0);
    HIPCHK(hipHostMalloc((void**)&m->h_cols, (size_t)2 * n * m->C1 * 4, hipHostMallocDefault));
    m->host_pos.assign(n, 0);
    m->host_step.assign(n, 0);
    HIPCHK(hipStreamSynchronize(m->stream));
    m->finalized = true;
}

template <typename F> static int with_prec(fm_llm* m, F&& f) {
    if (m->prec == FM_PREC_BF16) {
        Run<bf16_t> r(m);
        f(r);
        r.chain_flush();
    } else {
        Run<float> r(m);
        f(r);
        r.chain_flush();
    }
    return 0;
}

static void check_tokens(fm_llm* m, const int32_t* tok, int T) {
    const fm_model_config& c = m->c;
    for (int t = 0; t < T; ++t) {
        const int t0 = tok[t];
        FMCHECK(t0 >= 0 && t0 < c.vocab_size, "token id out of range: " + std::to_string(t0));
        for (int q = 0; q < m->C; ++q) {
            const int v = tok[(size_t)(q + 1) * T + t];
            FMCHECK(v >= 0 && v < m->cb, "codebook token out of range: " + std::to_string(v));
        }
    }
}

static void reset_slot(fm_llm* m, int slot, const fm_sampling* sp) {
    HIPCHK(hipMemsetAsync((char*)m->ras + (size_t)slot * m->C1 * 10 * 4, 0, (size_t)m->C1 * 10 * 4, m->stream));
    SlotParams p{};
    if (sp) {
        // top_k <= 64: register/wave select; larger (the reference takes any, inference.py:54-77):
        // the whole row sorted in LDS (sample_wide)
        FMCHECK(sp->top_k >= 1, "top_k must be >= 1: got " + std::to_string(sp->top_k));
        p.temperature = sp->temperature;
        p.top_p = sp->top_p;
        p.top_k = sp->top_k;
        p.mask_im_end = sp->mask_im_end;
        p.seed = sp->seed;
    } else {
        p.temperature = 0.7f;
        p.top_p = 0.9f;
        p.top_k = 1;
    }
    p.step = 0;
    p.force = m->host_force[slot];
    HIPCHK(hipMemcpyAsync(m->sp + slot, &p, sizeof p, hipMemcpyHostToDevice, m->stream));
    HIPCHK(hipStreamSynchronize(m->stream));
    m->host_step[slot] = 0;
}

static void upload_frame_rows(fm_llm* m, const int32_t* slots, int n) {
    std::vector<int> s(slots, slots + n), p(n);
    if (s == m->uploaded_slots) return;
    for (int i = 0; i < n; ++i) p[i] = m->host_pos[s[i]];
    HIPCHK(hipMemcpyAsync(m->frame_slot, s.data(), (size_t)n * 4, hipMemcpyHostToDevice, m->stream));
    HIPCHK(hipMemcpyAsync(m->frame_pos, p.data(), (size_t)n * 4, hipMemcpyHostToDevice, m->stream));
    HIPCHK(hipStreamSynchronize(m->stream));
    m->uploaded_slots = s;
}

// gemv chain health: the error word travels to pinned memory behind the frames; after the
// host's stream sync, a timed-out hand-off wait (a hang avoided) resets the counters and fails
static void chain_err_async(fm_llm* m) {
    if (fm_tuning().gemv_chain || fm_tuning().fin_split > 1 ||
        (m->fxt && fm_tuning().fattn_wo))
        HIPCHK(hipMemcpyAsync(m->h_chain_err, m->chain_err, sizeof(int), hipMemcpyDeviceToHost, m->stream));
}
static void chain_err_check(fm_llm* m) {
    if (!m->h_chain_err || !m->h_chain_err[0]) return;
    m->h_chain_err[0] = 0;
    HIPCHK(hipMemset(m->chain_cnt, 0, GEMV_CHAIN_WORDS * sizeof(unsigned)));
    HIPCHK(hipMemset(m->chain_err, 0, 16 * sizeof(int)));
    if (m->fin_cnt) HIPCHK(hipMemset(m->fin_cnt, 0, (size_t)std::max(m->max_slots, 64) * 2 * sizeof(int)));
    throw FmError{FM_ERR_STATE,
                  "in-launch hand-off wait timed out (gemv chain / split finalize / fused fast "
                  "attention + wo; counters reset)"};
}

// one decode frame for the uploaded rows (graph replay when enabled), async
static void launch_frame(fm_llm* m, int n) {
    if (m->use_graph && !m->prof.on) {
        auto it = m->graphs.find(n);
        if (it == m->graphs.end()) {
            hipGraph_t g;
            HIPCHK(hipStreamBeginCapture(m->stream, hipStreamCaptureModeThreadLocal));
            with_prec(m, [&](auto& r) { r.decode_frame(n); });
            HIPCHK(hipStreamEndCapture(m->stream, &g));
            hipGraphExec_t ge;
            HIPCHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            HIPCHK(hipGraphDestroy(g));
            it = m->graphs.emplace(n, ge).first;
        }
        HIPCHK(hipGraphLaunch(it->second, m->stream));
    } else {
        with_prec(m, [&](auto& r) { r.decode_frame(n); });
    }
}

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
extern "C" {

int fm_llm_open(const fm_model_config* cfg, int device, int precision, int max_slots, fm_llm** out) {
    return fm_guard([&] {
        FMCHECK(cfg && out, "null argument");
        FMCHECK(precision == FM_PREC_BF16 || precision == FM_PREC_FP32, "bad precision");
        FMCHECK(max_slots >= 1 && max_slots <= 4096, "bad max_slots");
        const fm_model_config& c = *cfg;
        FMCHECK(c.dim % 32 == 0 && c.fast_dim % 32 == 0, "dims must be multiples of 32");
        FMCHECK(c.intermediate_size % 32 == 0 && c.fast_intermediate_size % 32 == 0,
                "intermediate sizes must be multiples of 32");
        FMCHECK((c.n_head * c.head_dim) % 32 == 0 && (c.fast_n_head * c.fast_head_dim) % 32 == 0,
                "n_head*head_dim must be a multiple of 32");
        FMCHECK(c.head_dim % 8 == 0 && c.head_dim <= 256 && c.fast_head_dim <= 256, "bad head_dim");
        FMCHECK(c.n_head % c.n_local_heads == 0 && c.fast_n_head % c.fast_n_local_heads == 0, "bad GQA");
        FMCHECK(c.num_codebooks >= 1 && c.num_codebooks <= 63, "bad num_codebooks");
        FMCHECK(c.codebook_size <= 8192, "codebook_size > 8192 unsupported");
        FMCHECK(c.im_end_id >= 0 && c.im_end_id < c.vocab_size, "im_end_id must be set");
        FMCHECK(c.semantic_begin_id >= 0 && c.semantic_end_id < c.vocab_size &&
                    c.semantic_begin_id <= c.semantic_end_id,
                "bad semantic id range");
        int ndev = fm_device_count();
        FMCHECK(ndev > 0, "no HIP device visible");
        FMCHECK(device >= 0 && device < ndev, "bad device index");
        HIPCHK(hipSetDevice(device));
        std::unique_ptr<fm_llm> m(new fm_llm());
        m->c = c;
        m->device = device;
        m->prec = precision;
        m->esz = precision == FM_PREC_BF16 ? 2 : 4;
        m->max_slots = max_slots;
        m->S = (c.max_seq_len + 7) / 8 * 8;
        m->C = c.num_codebooks;
        m->C1 = c.num_codebooks + 1;
        m->cb = c.codebook_size;
        HIPCHK(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
        const char* g = getenv("FISHMI_GRAPH");  // FISHMI_GRAPH=0: eager launches (profilers)
        m->use_graph = !(g && g[0] == '0');
        build_inventory(m.get());
        *out = m.release();
    });
}

int fm_llm_set_quant_int4(fm_llm* m, int groupsize) {
    return fm_guard([&] {
        FMCHECK(m && (groupsize == 32 || groupsize == 64 || groupsize == 128 || groupsize == 256),
                "int4: groupsize must be 32, 64, 128 or 256 (WeightOnlyInt4QuantHandler, quantize.py:366)");
        FMCHECK(!m->finalized, "weights are frozen after finalize");
        for (auto& kv : m->w) FMCHECK(!kv.second.set, "set the quantization mode before any tensor");
        FMCHECK(m->quant == FM_QUANT_NONE, "quantization mode already set");
        FMCHECK(m->prec == FM_PREC_BF16, "int4: bf16 precision only (the reference quantizes the bf16 weights)");
        const fm_model_config& c = m->c;
        // create_quantized_state_dict asserts bias-free linears (quantize.py:371)
        FMCHECK(!c.qkv_bias && !c.o_bias && !c.fast_qkv_bias && !c.fast_o_bias,
                "int4: the linears must be bias-free (quantize.py:371)");
        for (auto& kv : m->w) {
            if (!is_quant_linear(kv.first)) continue;
            FMCHECK(kv.second.cols % groupsize == 0, "int4: in_features must be a multiple of the group size: " + kv.first);
            FMCHECK(m->w.find(base_of(kv.first) + ".bias") == m->w.end(),
                    "int4: the linears must be bias-free (quantize.py:371): " + kv.first);
        }
        m->quant = FM_QUANT_INT4;
        m->q4_gs = groupsize;
    });
}

int fm_llm_set_quant(fm_llm* m, int mode) {
    if (mode == FM_QUANT_INT4) return fm_llm_set_quant_int4(m, 128);
    return fm_guard([&] {
        FMCHECK(m && (mode == FM_QUANT_NONE || mode == FM_QUANT_INT8), "bad arguments");
        FMCHECK(!m->finalized, "weights are frozen after finalize");
        for (auto& kv : m->w) FMCHECK(!kv.second.set, "set the quantization mode before any tensor");
        if (mode == m->quant) return;
        FMCHECK(m->quant == FM_QUANT_NONE, "quantization mode already set");
        m->quant = mode;
        std::vector<std::pair<std::string, int64_t>> add;
        for (auto& kv : m->w) {
            if (!is_quant_linear(kv.first)) continue;
            FMCHECK(kv.second.cols % 64 == 0, "int8 weights need in_features % 64 == 0: " + kv.first);
            add.emplace_back(base_of(kv.first) + ".scales", kv.second.rows);
            auto b = m->w.find(base_of(kv.first) + ".bias");
            if (b != m->w.end()) b->second.optional = true;
        }
        for (auto& a : add) {
            add_t(m, a.first, 1, a.second);
            m->w[a.first].optional = true;
        }
    });
}

int fm_llm_set_tensor(fm_llm* m, const char* name, const void* data, int dtype, int64_t numel) {
    return fm_guard([&] {
        FMCHECK(m && name && data, "null argument");
        FMCHECK(!m->finalized, "weights are frozen after finalize");
        HIPCHK(hipSetDevice(m->device));
        if (dtype == FM_DT_I8) {  // an int8 checkpoint's weight (WeightOnlyInt8QuantHandler state_dict)
            FMCHECK(m->quant == FM_QUANT_INT8 && is_quant_linear(name), std::string("int8 data for ") + name +
                                                                             " needs fm_llm_set_quant(INT8) and a linear weight");
            auto it = m->w.find(name);
            FMCHECK(it != m->w.end() && it->second.numel == numel, std::string("unknown tensor or wrong numel: ") + name);
            DTensor& t = it->second;
            FMCHECK(!t.set, std::string("tensor set twice: ") + name);
            const size_t bytes = (size_t)(t.rows + 15) / 16 * 16 * t.cols;
            HIPCHK(hipMalloc(&t.q, bytes));
            HIPCHK(hipMemsetAsync(t.q, 0, bytes, m->stream));
            HIPCHK(hipMemcpyAsync(t.q, data, (size_t)numel, hipMemcpyHostToDevice, m->stream));
            HIPCHK(hipStreamSynchronize(m->stream));
            t.set = true;
            return;
        }
        DTensor& t = tensor_for(m, name, numel);
        const size_t sb = dtype == FM_DT_BF16 ? 2 : 4;
        void* tmp = nullptr;
        HIPCHK(hipMalloc(&tmp, (size_t)numel * sb));
        HIPCHK(hipMemcpy(tmp, data, (size_t)numel * sb, hipMemcpyHostToDevice));
        if (m->prec == FM_PREC_BF16)
            launch_convert<bf16_t>(m->stream, tmp, dtype == FM_DT_BF16, numel, (bf16_t*)t.p);
        else
            launch_convert<float>(m->stream, tmp, dtype == FM_DT_BF16, numel, (float*)t.p);
        HIPCHK(hipStreamSynchronize(m->stream));
        HIPCHK(hipFree(tmp));
        t.set = true;
    });
}

int fm_llm_synth_tensor(fm_llm* m, const char* name, int64_t numel, uint64_t seed, float center,
                        int log2_half) {
    return fm_guard([&] {
        FMCHECK(m && name, "null argument");
        FMCHECK(!m->finalized, "weights are frozen after finalize");
        HIPCHK(hipSetDevice(m->device));
        DTensor& t = tensor_for(m, name, numel);
        if (m->prec == FM_PREC_BF16)
            launch_synth<bf16_t>(m->stream, (bf16_t*)t.p, numel, seed, fnv1a32(name), center, log2_half);
        else
            launch_synth<float>(m->stream, (float*)t.p, numel, seed, fnv1a32(name), center, log2_half);
        HIPCHK(hipGetLastError());
        t.set = true;
    });
}

int fm_llm_finalize(fm_llm* m) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
    });
}

// pos0 > 0 continues a slot whose positions [0, pos0) already hold the KV of the same tokens
// (prefix reuse across generate_long batches); the prompt suffix runs at pos0 .. pos0 + T - 1
static void do_prefill(fm_llm* m, int slot, const int32_t* tokens, int T, const fm_sampling* sp,
                       int32_t* first_col, int pos0 = 0) {
    FMCHECK(slot >= 0 && slot < m->max_slots, "bad slot");
    FMCHECK(T >= 1 && pos0 >= 0 && pos0 + T < m->c.max_seq_len, "prompt must end before max_seq_len");
    FMCHECK(pos0 <= m->host_pos[slot], "prefix reuse past the slot's cached positions");
    check_tokens(m, tokens, T);
    reset_slot(m, slot, sp);
    const int32_t one = slot;
    m->uploaded_slots.clear();
    HIPCHK(hipMemcpyAsync(m->frame_slot, &one, 4, hipMemcpyHostToDevice, m->stream));
    with_prec(m, [&](auto& r) {
        const void* last = r.prefill_slow(slot, tokens, T, pos0);
        const void* hid = r.head_small(last, false, 1, 1);
        r.frame_tail_small(1, false, true, hid);
    });
    int pos = pos0 + T - 1;  // finish() advances it: the first decode frame runs at pos0 + T
    HIPCHK(hipMemcpyAsync(m->frame_pos, &pos, 4, hipMemcpyHostToDevice, m->stream));
    launch_finish(m->stream, 1, m->frame_slot, m->frame_pos, m->cols, m->C1, m->tok_in, m->ras,
                  m->C1 * 10, m->C1, 0, m->sp);
    HIPCHK(hipMemcpyAsync(m->h_cols, m->cols, (size_t)m->C1 * 4, hipMemcpyDeviceToHost, m->stream));
    HIPCHK(hipStreamSynchronize(m->stream));
    m->prof.collect();
    m->host_pos[slot] = pos0 + T;
    m->host_step[slot] = 1;
    m->uploaded_slots.clear();
    if (first_col) memcpy(first_col, m->h_cols, (size_t)m->C1 * 4);
}

// Several requests prefilled together (each from position 0 of its own slot): one pass of the slow
// stack over all their prompt rows, then one batched first frame (head + fast model + samplers) for
// their last rows -- the same columns as n separate do_prefill calls.
static void do_prefill_batch(fm_llm* m, int n, const int32_t* slots, const int32_t* tokens, const int32_t* T,
                             const fm_sampling* sps, int32_t* first_cols) {
    FMCHECK(n >= 1 && n <= m->max_slots, "bad request count");
    std::vector<const int32_t*> tk(n);
    size_t off = 0;
    for (int i = 0; i < n; ++i) {
        FMCHECK(slots[i] >= 0 && slots[i] < m->max_slots, "bad slot");
        for (int j = 0; j < i; ++j) FMCHECK(slots[j] != slots[i], "duplicate slot");
        FMCHECK(T[i] >= 1 && T[i] < m->c.max_seq_len, "prompt must end before max_seq_len");
        tk[i] = tokens + off;
        check_tokens(m, tk[i], T[i]);
        off += (size_t)m->C1 * T[i];
    }
    for (int i = 0; i < n; ++i) reset_slot(m, slots[i], sps ? sps + i : nullptr);
    m->uploaded_slots.clear();
    HIPCHK(hipMemcpyAsync(m->frame_slot, slots, (size_t)n * 4, hipMemcpyHostToDevice, m->stream));
    with_prec(m, [&](auto& r) {
        r.prefill_multi(n, slots, tk.data(), T);
        if (n <= GEMV_MAX_ROWS) {
            const void* hid = r.head_small(m->plast, false, n, 1);
            r.frame_tail_small(n, false, true, hid);
        } else {
            r.bs_frame = true;
            r.head_and_hidden(m->plast, n);
            r.frame_tail(n, false, true);
            r.bs_frame = false;
        }
    });
    std::vector<int> pos(n);
    for (int i = 0; i < n; ++i) pos[i] = T[i] - 1;  // finish() advances it
    HIPCHK(hipMemcpyAsync(m->frame_pos, pos.data(), (size_t)n * 4, hipMemcpyHostToDevice, m->stream));
    launch_finish(m->stream, n, m->frame_slot, m->frame_pos, m->cols, m->C1, m->tok_in, m->ras, m->C1 * 10,
                  m->C1, 0, m->sp);
    HIPCHK(hipMemcpyAsync(m->h_cols, m->cols, (size_t)n * m->C1 * 4, hipMemcpyDeviceToHost, m->stream));
    HIPCHK(hipStreamSynchronize(m->stream));
    m->prof.collect();
    for (int i = 0; i < n; ++i) {
        m->host_pos[slots[i]] = T[i];
        m->host_step[slots[i]] = 1;
    }
    m->uploaded_slots.clear();
    if (first_cols) memcpy(first_cols, m->h_cols, (size_t)n * m->C1 * 4);
}

int fm_llm_prefill_batch(fm_llm* m, int n, const int32_t* slots, const int32_t* tokens, const int32_t* T,
                         const fm_sampling* sp, int32_t* first_cols) {
    return fm_guard([&] {
        FMCHECK(m && slots && tokens && T, "null argument");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        do_prefill_batch(m, n, slots, tokens, T, sp, first_cols);
    });
}

int fm_llm_prefill(fm_llm* m, int slot, const int32_t* tokens, int T, const fm_sampling* sp,
                   int32_t* first_col) {
    return fm_guard([&] {
        FMCHECK(m && tokens, "null argument");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        do_prefill(m, slot, tokens, T, sp, first_col);
    });
}

int fm_llm_prefill_at(fm_llm* m, int slot, const int32_t* suffix, int T, int pos0, const fm_sampling* sp,
                      int32_t* first_col) {
    return fm_guard([&] {
        FMCHECK(m && suffix, "null argument");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        do_prefill(m, slot, suffix, T, sp, first_col, pos0);
    });
}

int fm_llm_decode(fm_llm* m, const int32_t* slots, int n, int32_t* cols) {
    return fm_guard([&] {
        FMCHECK(m && slots && n >= 1 && n <= m->max_slots, "bad arguments");
        FMCHECK(m->finalized, "call fm_llm_prefill first");
        HIPCHK(hipSetDevice(m->device));
        for (int i = 0; i < n; ++i) {
            FMCHECK(slots[i] >= 0 && slots[i] < m->max_slots, "bad slot");
            FMCHECK(m->host_pos[slots[i]] < m->c.max_seq_len, "slot reached max_seq_len");
        }
        upload_frame_rows(m, slots, n);
        launch_frame(m, n);
        HIPCHK(hipMemcpyAsync(m->h_cols, m->cols, (size_t)n * m->C1 * 4, hipMemcpyDeviceToHost, m->stream));
        chain_err_async(m);
        HIPCHK(hipStreamSynchronize(m->stream));
        chain_err_check(m);
        m->prof.collect();
        for (int i = 0; i < n; ++i) {
            m->host_pos[slots[i]]++;
            m->host_step[slots[i]]++;
        }
        if (cols) memcpy(cols, m->h_cols, (size_t)n * m->C1 * 4);
    });
}

int fm_llm_decode_frames(fm_llm* m, const int32_t* slots, int n, int nframes, int32_t* cols) {
    return fm_guard([&] {
        FMCHECK(m && slots && cols && n >= 1 && n <= m->max_slots && nframes >= 0, "bad arguments");
        FMCHECK(m->finalized, "call fm_llm_prefill first");
        HIPCHK(hipSetDevice(m->device));
        for (int i = 0; i < n; ++i) {
            FMCHECK(slots[i] >= 0 && slots[i] < m->max_slots, "bad slot");
            for (int j = 0; j < i; ++j) FMCHECK(slots[j] != slots[i], "duplicate slot");
            FMCHECK(m->host_pos[slots[i]] + nframes <= m->c.max_seq_len, "slot would pass max_seq_len");
        }
        if (nframes == 0) return;
        const size_t per = (size_t)n * m->C1;
        if (m->h_hist_n < per * nframes) {
            if (m->h_hist) HIPCHK(hipHostFree(m->h_hist));
            m->h_hist = nullptr;
            m->h_hist_n = 0;
            HIPCHK(hipHostMalloc((void**)&m->h_hist, per * nframes * 4, hipHostMallocDefault));
            m->h_hist_n = per * nframes;
        }
        upload_frame_rows(m, slots, n);
        // every frame is queued back to back; the columns stream to pinned memory behind them
        for (int k = 0; k < nframes; ++k) {
            launch_frame(m, n);
            HIPCHK(hipMemcpyAsync(m->h_hist + per * k, m->cols, per * 4, hipMemcpyDeviceToHost, m->stream));
        }
        chain_err_async(m);
        HIPCHK(hipStreamSynchronize(m->stream));
        chain_err_check(m);
        m->prof.collect();
        for (int i = 0; i < n; ++i) {
            m->host_pos[slots[i]] += nframes;
            m->host_step[slots[i]] += nframes;
        }
        memcpy(cols, m->h_hist, per * nframes * 4);
    });
}

static void do_generate(fm_llm* m, int slot, const int32_t* prompt, int T, int pos0, int max_new,
                        const fm_sampling* sp, int32_t* out, int* n_out) {
        FMCHECK(m && prompt && out && n_out, "null argument");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        const fm_model_config& c = m->c;
        if (max_new <= 0 || pos0 + T + max_new > c.max_seq_len) max_new = c.max_seq_len - pos0 - T;
        FMCHECK(max_new >= 1, "prompt leaves no room to generate");
        const int C1 = m->C1;
        int32_t col[64];
        do_prefill(m, slot, prompt, T, sp, col, pos0);
        for (int q = 0; q < C1; ++q) out[(size_t)q * max_new] = col[q];
        int n = 1;
        upload_frame_rows(m, &slot, 1);
        // pipelined: frame k+1 is queued before frame k's column is inspected on the host
        hipEvent_t ev[2];
        HIPCHK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
        auto issue = [&](int k) {
            launch_frame(m, 1);
            HIPCHK(hipMemcpyAsync(m->h_cols + (size_t)(k & 1) * m->max_slots * C1, m->cols, (size_t)C1 * 4,
                                  hipMemcpyDeviceToHost, m->stream));
            HIPCHK(hipEventRecord(ev[k & 1], m->stream));
        };
        const int steps = max_new - 1;
        int issued = 0;
        if (steps > 0) issue(issued++);
        for (int k = 0; k < steps; ++k) {
            if (issued < steps && issued <= k + 1) issue(issued++);
            HIPCHK(hipEventSynchronize(ev[k & 1]));
            const int32_t* hc = m->h_cols + (size_t)(k & 1) * m->max_slots * C1;
            for (int q = 0; q < C1; ++q) out[(size_t)q * max_new + n] = hc[q];
            n++;
            if (hc[0] == c.im_end_id) break;
        }
        chain_err_async(m);
        HIPCHK(hipStreamSynchronize(m->stream));
        chain_err_check(m);
        m->prof.collect();
        (void)hipEventDestroy(ev[0]);
        (void)hipEventDestroy(ev[1]);
        m->host_pos[slot] = pos0 + T + issued;  // device advanced once per issued frame
        m->host_step[slot] = 1 + issued;
        m->uploaded_slots.clear();
        *n_out = n;
}

int fm_llm_generate(fm_llm* m, int slot, const int32_t* prompt, int T, int max_new, const fm_sampling* sp,
                    int32_t* out, int* n_out) {
    return fm_guard([&] { do_generate(m, slot, prompt, T, 0, max_new, sp, out, n_out); });
}

int fm_llm_generate_at(fm_llm* m, int slot, const int32_t* suffix, int T, int pos0, int max_new,
                       const fm_sampling* sp, int32_t* out, int* n_out) {
    return fm_guard([&] { do_generate(m, slot, suffix, T, pos0, max_new, sp, out, n_out); });
}

int fm_llm_slot_pos(fm_llm* m, int slot, int* pos) {
    return fm_guard([&] {
        FMCHECK(m && pos && slot >= 0 && slot < m->max_slots, "bad arguments");
        *pos = m->host_pos[slot];
    });
}

int fm_llm_teacher_step(fm_llm* m, int slot, const int32_t* x, int S, int pos0, const int32_t* next_col,
                        float* slow_logits, float* hidden, float* fast_logits) {
    return fm_guard([&] {
        FMCHECK(m && x && S >= 1, "bad arguments");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        FMCHECK(slot >= 0 && slot < m->max_slots, "bad slot");
        FMCHECK(pos0 + S <= m->c.max_seq_len, "beyond max_seq_len");
        check_tokens(m, x, S);
        if (next_col)
            for (int q = 1; q < m->C1; ++q)
                FMCHECK(next_col[q] >= 0 && next_col[q] < m->cb, "next_col codebook token out of range");
        if (pos0 == 0) reset_slot(m, slot, nullptr);
        const fm_model_config& c = m->c;
        const int32_t one = slot;
        HIPCHK(hipMemcpyAsync(m->frame_slot, &one, 4, hipMemcpyHostToDevice, m->stream));
        m->uploaded_slots.clear();
        std::vector<float> lg(m->Nhead);
        with_prec(m, [&](auto& r) {
            const void* last = r.prefill_slow(slot, x, S, pos0);
            const void* hid = r.head_small(last, false, 1, 1);
                HIPCHK(hipMemcpyAsync(lg.data(), m->logits, (size_t)m->Nhead * 4, hipMemcpyDeviceToHost, m->stream));
            if (hidden) {
                std::vector<uint8_t> hb((size_t)c.fast_dim * m->esz);
                HIPCHK(hipMemcpyAsync(hb.data(), hid, hb.size(), hipMemcpyDeviceToHost, m->stream));
                HIPCHK(hipStreamSynchronize(m->stream));
                for (int i = 0; i < c.fast_dim; ++i) {
                    if (m->esz == 2) {
                        uint32_t u = ((uint32_t)((uint16_t*)hb.data())[i]) << 16;
                        memcpy(&hidden[i], &u, 4);
                    } else {
                        hidden[i] = ((float*)hb.data())[i];
                    }
                }
            }
            if (next_col) {
                HIPCHK(hipMemcpyAsync(m->cols, next_col, (size_t)m->C1 * 4, hipMemcpyHostToDevice, m->stream));
                r.fast_small(1, 0, false, hid);
                for (int cc = 1; cc < m->C; ++cc) {
                    r.fast_small(1, cc, true, hid);
                                if (fast_logits)
                        HIPCHK(hipMemcpyAsync(fast_logits + (size_t)(cc - 1) * m->cb, m->flogits, (size_t)m->cb * 4,
                                              hipMemcpyDeviceToHost, m->stream));
                }
            }
        });
        HIPCHK(hipStreamSynchronize(m->stream));
        m->prof.collect();
        m->host_pos[slot] = pos0 + S;
        if (slow_logits) {
            for (int i = 0; i < c.vocab_size; ++i) slow_logits[i] = -INFINITY;
            for (int i = 0; i < m->nsem; ++i) slow_logits[c.semantic_begin_id + i] = lg[i];
            slow_logits[c.im_end_id] = lg[m->nsem];
        }
    });
}

int64_t fm_llm_frame_bytes(fm_llm* m, int n, int pos) {
    if (!m) return -1;
    const fm_model_config& c = m->c;
    const int64_t E = (int64_t)m->esz;
    // weight-only int8: one byte per linear weight plus one T scale per output row; int4 (streamed
    // form): half a byte per weight plus one (scale, zero) word per row and 128-k unit
    const bool q4 = m->quant == FM_QUANT_INT4 && m->q4_gs % 128 == 0;
    auto lin = [&](int64_t N, int64_t K) -> int64_t {
        if (q4 && K % 128 == 0) return N * K / 2 + N * (K / 128) * 4;
        if (m->quant == FM_QUANT_INT8) return N * K + N * E;
        return N * K * E;
    };
    auto stack_bytes = [&](const StackDims& d) {
        int64_t per = lin(d.nqkv(), d.dim) + lin(d.dim, d.nq()) + lin(2LL * d.inter, d.dim) + lin(d.dim, d.inter) +
                      2LL * d.dim * E;
        if (d.qk_norm) per += 2LL * d.hd * E;
        return per * d.n_layer;
    };
    int64_t b = stack_bytes(m->sd) + (c.tie_word_embeddings ? (int64_t)m->Nhead * c.dim * E : lin(m->Nhead, c.dim)) +
                (int64_t)c.dim * E;
    b += (int64_t)m->C * stack_bytes(m->fdm) + (int64_t)(m->C - 1) * (lin(m->cb, c.fast_dim) + (int64_t)c.fast_dim * E);
    if (m->fproj_w) b += lin(c.fast_dim, c.dim);
    // per-stream: KV reads (+ the row written), embeddings
    int64_t per_stream = 2LL * m->sd.n_layer * m->sd.nkv * m->sd.hd * E * (pos + 1);
    for (int cc = 0; cc < m->C; ++cc) per_stream += 2LL * m->fdm.n_layer * m->fdm.nkv * m->fdm.hd * E * (cc + 1);
    per_stream += (int64_t)(m->C + 1) * c.dim * E + (int64_t)(m->C - 1) * c.fast_dim * E;
    return b + per_stream * n;
}

int fm_llm_profile(fm_llm* m, int enable) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        m->prof.on = enable != 0;
        if (enable) m->prof.acc.clear();
    });
}

int fm_llm_profile_read(fm_llm* m, const char* cls, double* ms, int64_t* launches, int64_t* bytes) {
    return fm_guard([&] {
        FMCHECK(m && cls, "null argument");
        auto it = m->prof.acc.find(cls);
        Profiler::Acc a = it == m->prof.acc.end() ? Profiler::Acc{} : it->second;
        if (ms) *ms = a.ms;
        if (launches) *launches = a.n;
        if (bytes) *bytes = a.bytes;
    });
}

int fm_tune(const char* key, int value) {
    return fm_guard([&] {
        FMCHECK(key, "null key");
        FmTuning& t = fm_tuning();
        const std::string k = key;
        if (k == "gemv_nt") {
            t.gemv_nt = value != 0;
        } else if (k == "gemv_u") {
            FMCHECK(value == 2 || value == 4 || value == 8, "gemv_u must be 2, 4 or 8");
            t.gemv_u = value;
        } else if (k == "sampler_fast") {
            t.sampler_fast = value != 0;
        } else if (k == "attn_cap") {
            FMCHECK(value == 0 || (value >= 16 && value % 16 == 0), "attn_cap must be 0 or a multiple of 16");
            t.attn_cap = value;
        } else if (k == "prefill_attn") {
            t.prefill_attn = value != 0;
        } else if (k == "prompt_qkv_slab") {
            t.prompt_qkv_slab = value != 0;
        } else if (k == "prompt_unroll") {
            t.prompt_unroll = value != 0;
        } else if (k == "prompt_fin") {
            t.prompt_fin = value != 0;
        } else if (k == "prompt_swiglu") {
            t.prompt_swiglu = value != 0;
        } else if (k == "prompt_skinny") {
            t.prompt_skinny = value != 0;
        } else if (k == "prompt_skinny_blocks") {
            FMCHECK(value >= 1, "prompt_skinny_blocks must be >= 1");
            t.prompt_skinny_blocks = value;
        } else if (k == "prompt_ks_tiles") {
            FMCHECK(value >= 1, "prompt_ks_tiles must be >= 1");
            t.prompt_ks_tiles = value;
        } else if (k == "prompt_ks_max") {
            FMCHECK(value == 1 || value == 2 || value == 4 || value == 8, "prompt_ks_max must be 1, 2, 4 or 8");
            t.prompt_ks_max = value;
        } else if (k == "prompt_gemm") {
            t.prompt_gemm = value != 0;
        } else if (k == "conv2") {
            t.conv2 = value != 0;
        } else if (k == "conv_splitk") {
            t.conv_splitk = value != 0;
        } else if (k == "codec_norm") {
            t.codec_norm = value != 0;
        } else if (k == "codec_rope") {
            t.codec_rope = value != 0;
        } else if (k == "codec_swiglu") {
            t.codec_swiglu = value != 0;
        } else if (k == "codec_fuse") {
            t.codec_fuse = value != 0;
        } else if (k == "resunit_enc") {
            t.resunit_enc = value != 0;
        } else if (k == "resunit_384") {
            t.resunit_384 = value != 0;
        } else if (k == "resunit_cfg") {
            FMCHECK(value >= 0 && value <= 2, "resunit_cfg must be 0..2");
            t.resunit_cfg = value;
        } else if (k == "attn_wo") {
            t.attn_wo = value != 0;
        } else if (k == "gemv_wpb") {
            FMCHECK(value == 4 || value == 8, "gemv_wpb must be 4 or 8");
            t.gemv_wpb = value;
        } else if (k == "ksb_blocks") {
            FMCHECK(value >= 1, "ksb_blocks must be >= 1");
            t.ksb_blocks = value;
        } else if (k == "attn_cap_batched") {
            FMCHECK(value == 0 || (value >= 16 && value % 16 == 0), "attn_cap_batched must be 0 or a multiple of 16");
            t.attn_cap_batched = value;
        } else if (k == "linear_u32") {
            FMCHECK(value == 4 || value == 8, "linear_u32 must be 4 or 8");
            t.linear_u32 = value;
        } else if (k == "batched_fused_attn") {
            t.batched_fused_attn = value != 0;
        } else if (k == "linear_fill") {
            FMCHECK(value >= 0, "linear_fill must be >= 0");
            t.linear_fill = value;
        } else if (k == "ksb_balance") {
            t.ksb_balance = value != 0;
        } else if (k == "attn3") {
            t.attn3 = value != 0;
        } else if (k == "attn_fd") {
            t.attn_fd = value != 0;
        } else if (k == "fd_min") {
            FMCHECK(value >= 16 && value % 16 == 0, "fd_min must be a multiple of 16");
            t.fd_min = value;
        } else if (k == "chain_max") {
            FMCHECK(value >= 2 && value <= GEMV_CHAIN_MAX, "chain_max must be 2..4");
            t.chain_max = value;
        } else if (k == "chain_sleep") {
            FMCHECK(value == 1 || value == 4 || value == 16, "chain_sleep must be 1, 4 or 16");
            t.chain_sleep = value;
        } else if (k == "gemv_chain") {
            t.gemv_chain = value != 0;
        } else if (k == "fd_nw") {
            FMCHECK(value == 4 || value == 8 || value == 16, "fd_nw must be 4, 8 or 16");
            t.fd_nw = value;
        } else if (k == "fin_ksb") {
            FMCHECK(value >= 0 && value <= KSB_MAX, "fin_ksb must be in [0, KSB_MAX]");
            t.fin_ksb = value;
        } else if (k == "fd_nw_batched") {
            FMCHECK(value == 4 || value == 8 || value == 16, "fd_nw_batched must be 4, 8 or 16");
            t.fd_nw_batched = value;
        } else if (k == "fd_min16") {
            FMCHECK(value >= 16 && value % 16 == 0, "fd_min16 must be a multiple of 16");
            t.fd_min16 = value;
        } else if (k == "fd_min_batched") {
            FMCHECK(value >= 16 && value % 16 == 0, "fd_min_batched must be a multiple of 16");
            t.fd_min_batched = value;
        } else if (k == "gemv_dummy") {
            FMCHECK(value >= 0 && value <= 2, "gemv_dummy must be 0, 1 or 2");
            t.gemv_dummy = value;
        } else if (k == "bs_dummy") {
            FMCHECK(value >= 0 && value <= 2, "bs_dummy must be 0, 1 or 2");
            t.bs_dummy = value;
        } else if (k == "bs_qkv_slab") {
            t.bs_qkv_slab = value != 0;
        } else if (k == "fast_tail") {
            t.fast_tail = value != 0;
        } else if (k == "fkv_prefetch") {
            t.fkv_prefetch = value != 0;
        } else if (k == "kv_prefetch") {
            t.kv_prefetch = value != 0;
        } else if (k == "bstream") {
            t.bstream = value != 0;
        } else if (k == "bstream_kparts") {
            FMCHECK(value == 0 || value == 1 || value == 2 || value == 4 || value == 8, "bstream_kparts must be 0, 1, 2, 4 or 8");
            t.bstream_kparts = value;
        } else if (k == "bstream_acc") {
            t.bstream_acc = value;
        } else if (k == "bstream_chain") {
            t.bstream_chain = value;
        } else if (k == "bstream_nw") {
            FMCHECK(value >= 0 && value <= 16, "bstream_nw must be in [0, 16]");
            t.bstream_nw = value;
        } else if (k == "bs_xfirst") {
            t.bs_xfirst = value != 0;
        } else if (k == "bs_vec_epi") {
            t.bs_vec_epi = value != 0;
        } else if (k == "bsacc_kparts") {
            FMCHECK(value == 0 || value == 1 || value == 2 || value == 4 || value == 8, "bsacc_kparts must be 0, 1, 2, 4 or 8");
            t.bsacc_kparts = value;
        } else if (k == "q_u") {
            FMCHECK(value == 2 || value == 4 || value == 8 || value == 16, "q_u must be 2, 4, 8 or 16");
            t.q_u = value;
        } else if (k == "fin8") {
            t.fin8 = value != 0;
        } else if (k == "fin_split") {
            FMCHECK(value >= 0 && value <= 16, "fin_split must be 0..16");
            t.fin_split = value;
        } else if (k == "int4_stream") {
            t.int4_stream = value != 0;
        } else if (k == "fw_delay") {
            FMCHECK(value >= 0 && value <= 1000, "fw_delay must be 0..1000 (10-ns ticks)");
            t.fw_delay = value;
        } else if (k == "fw_prio") {
            t.fw_prio = value != 0;
        } else if (k == "fw_cheap") {
            t.fw_cheap = value != 0;
        } else if (k == "fattn_wo") {
            t.fattn_wo = value != 0;
        } else if (k == "sampler_kth") {
            t.sampler_kth = value != 0;
        } else if (k == "row_qkv_rp") {
            FMCHECK(value == 4 || value == 8 || value == 16, "row_qkv_rp must be 4, 8 or 16");
            t.row_qkv_rp = value;
        } else if (k == "rowgemv_q4") {
            FMCHECK(value >= 0 && value <= 31, "rowgemv_q4 must be 0..31");
            t.rowgemv_q4 = value;
        } else if (k == "row_copies") {
            t.row_copies = value != 0;
        } else if (k == "rowgemv") {
            FMCHECK(value >= 0 && value <= 31, "rowgemv must be 0..31 (bit 0 wo / w2, bit 1 wqkv, bit 2 w1 || w3, bit 3 fast head, bit 4 first-layer wqkv)");
            t.rowgemv = value;
        } else if (k == "rmsnorm_block") {
            t.rmsnorm_block = value != 0;
        } else if (k == "debug_ts") {  // (re)arm the per-block timestamp buffer; 0 frees it
            if (t.dbg) HIPCHK(hipFree(t.dbg));
            t.dbg = nullptr;
            if (value) {
                HIPCHK(hipMalloc(&t.dbg, (8 + 8 * (1 << 20)) * sizeof(unsigned long long)));
                HIPCHK(hipMemset(t.dbg, 0, 8 * sizeof(unsigned long long)));
            }
        } else {
            FMCHECK(false, "unknown tuning key: " + k);
        }
    });
}

int fm_debug_ts_read(unsigned long long* out, int64_t max_records, int64_t* n_records) {
    return fm_guard([&] {
        FMCHECK(out && n_records, "null argument");
        const FmTuning& t = fm_tuning();
        FMCHECK(t.dbg, "debug_ts is not armed");
        HIPCHK(hipDeviceSynchronize());
        unsigned long long n = 0;
        HIPCHK(hipMemcpy(&n, t.dbg, sizeof n, hipMemcpyDeviceToHost));
        n = std::min<unsigned long long>(n, 1ull << 20);
        n = std::min<unsigned long long>(n, (unsigned long long)max_records);
        HIPCHK(hipMemcpy(out, t.dbg + 8, n * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        *n_records = (int64_t)n;
    });
}

int fm_llm_kernel_bench(fm_llm* m, const char* cls, int reps, double* avg_us, int64_t* launches,
                        int64_t* bytes) {
    return fm_guard([&] {
        FMCHECK(m && cls && reps >= 1, "bad arguments");
        FMCHECK(m->finalized && !m->uploaded_slots.empty(), "decode a frame first");
        HIPCHK(hipSetDevice(m->device));
        const int n = (int)m->uploaded_slots.size();
        const bool was_on = m->prof.on;
        // record the class's launches of one eager frame (the frame itself runs normally)
        m->prof.on = false;
        m->prof.rec.clear();
        m->prof.rec_bytes.clear();
        m->prof.rec_cls = cls;
        with_prec(m, [&](auto& r) { r.decode_frame(n); });
        m->prof.rec_cls.clear();
        m->prof.on = was_on;
        HIPCHK(hipStreamSynchronize(m->stream));
        for (int s : m->uploaded_slots) {  // that frame advanced the slots on the device
            m->host_pos[s]++;
            m->host_step[s]++;
        }
        std::vector<std::function<void()>> rec;
        rec.swap(m->prof.rec);
        FMCHECK(!rec.empty(), std::string("no launches of class ") + cls + " in a decode frame");
        int64_t b = 0;
        for (int64_t x : m->prof.rec_bytes) b += x;
        // replay them back to back as one graph, timed by two events on the compute stream
        hipGraph_t g;
        HIPCHK(hipStreamBeginCapture(m->stream, hipStreamCaptureModeThreadLocal));
        for (auto& f : rec) f();
        HIPCHK(hipStreamEndCapture(m->stream, &g));
        hipGraphExec_t ge;
        HIPCHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        HIPCHK(hipGraphDestroy(g));
        hipEvent_t ea, eb;
        HIPCHK(hipEventCreate(&ea));
        HIPCHK(hipEventCreate(&eb));
        HIPCHK(hipGraphLaunch(ge, m->stream));
        HIPCHK(hipEventRecord(ea, m->stream));
        for (int i = 0; i < reps; ++i) HIPCHK(hipGraphLaunch(ge, m->stream));
        HIPCHK(hipEventRecord(eb, m->stream));
        HIPCHK(hipEventSynchronize(eb));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ea, eb));
        (void)hipEventDestroy(ea);
        (void)hipEventDestroy(eb);
        (void)hipGraphExecDestroy(ge);
        if (avg_us) *avg_us = (double)ms * 1e3 / ((double)reps * rec.size());
        if (launches) *launches = (int64_t)rec.size();
        if (bytes) *bytes = b;
    });
}

int fm_llm_force(fm_llm* m, int slot, const int32_t* col) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        FMCHECK(slot >= 0 && slot < m->max_slots, "bad slot");
        const int on = col != nullptr;
        if (on) {
            const fm_model_config& c = m->c;
            // any vocabulary id: the reference's bf16 multinomial draw can emit ids outside the
            // semantic support (torch.rand_like in bf16 yields 0 or 1, and argmax over an all-zero
            // or NaN row is id 0: inference.py:43-46), and teacher forcing replays its streams
            FMCHECK(col[0] >= 0 && col[0] < c.vocab_size, "forced token outside the vocabulary");
            for (int q = 1; q < m->C1; ++q)
                FMCHECK(col[q] >= 0 && col[q] < m->cb, "forced codebook token out of range");
            HIPCHK(hipMemcpyAsync(m->force_cols + (size_t)slot * m->C1, col, (size_t)m->C1 * 4,
                                  hipMemcpyHostToDevice, m->stream));
        }
        m->host_force[slot] = on;
        HIPCHK(hipMemcpyAsync(&m->sp[slot].force, &m->host_force[slot], sizeof(int), hipMemcpyHostToDevice,
                              m->stream));
        HIPCHK(hipStreamSynchronize(m->stream));
    });
}

int fm_llm_read_logits(fm_llm* m, int slot, float* slow_logits, float* fast_logits) {
    return fm_guard([&] {
        FMCHECK(m && m->finalized, "null or unfinalized handle");
        FMCHECK(slot >= 0 && slot < m->max_slots, "bad slot");
        HIPCHK(hipSetDevice(m->device));
        const fm_model_config& c = m->c;
        std::vector<float> lg(m->Nhead);
        HIPCHK(hipMemcpyAsync(lg.data(), m->tap_slow + (size_t)slot * m->Nhead, (size_t)m->Nhead * 4,
                              hipMemcpyDeviceToHost, m->stream));
        if (fast_logits && m->C > 1)
            HIPCHK(hipMemcpyAsync(fast_logits, m->tap_fast + (size_t)slot * (m->C - 1) * m->cb,
                                  (size_t)(m->C - 1) * m->cb * 4, hipMemcpyDeviceToHost, m->stream));
        HIPCHK(hipStreamSynchronize(m->stream));
        if (slow_logits) {
            for (int i = 0; i < c.vocab_size; ++i) slow_logits[i] = -INFINITY;
            for (int i = 0; i < m->nsem; ++i) slow_logits[c.semantic_begin_id + i] = lg[i];
            slow_logits[c.im_end_id] = lg[m->nsem];
        }
    });
}

int fm_llm_use_graph(fm_llm* m, int enable) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        m->use_graph = enable != 0;
        // captured frames are dropped so that the next ones pick up any fm_tune change
        for (auto& g : m->graphs) (void)hipGraphExecDestroy(g.second);
        m->graphs.clear();
    });
}

int fm_llm_debug_vec(fm_llm* m, const char* name, int index, float* out, int64_t n) {
    return fm_guard([&] {
        FMCHECK(m && m->finalized && name && out && n > 0, "bad arguments");
        HIPCHK(hipSetDevice(m->device));
        HIPCHK(hipStreamSynchronize(m->stream));
        const std::string k = name;
        void* p = k == "qkv" ? m->qkv : k == "att" ? m->att : k == "fh" ? m->fh : k == "act" ? m->act
                : k == "fx" ? m->fx : k == "fx2" ? m->fx2 : k == "xl" ? m->xl : k == "xnl" ? m->xnl : nullptr;
        if (k == "kc" || k == "vc") {  // slot 0's slow-layer `index` cache: [nkv][S][hd]
            FMCHECK(index >= 0 && index < m->sd.n_layer, "layer out of range");
            FMCHECK(n <= (int64_t)m->layer_stride, "n past the layer's cache");
            p = (char*)(k == "kc" ? m->kc : m->vc) + (size_t)index * m->layer_stride * m->esz;
        }
        FMCHECK(p, "unknown buffer: " + k);
        if (m->esz == 4) {
            HIPCHK(hipMemcpy(out, p, (size_t)n * 4, hipMemcpyDeviceToHost));
        } else {
            std::vector<uint16_t> v((size_t)n);
            HIPCHK(hipMemcpy(v.data(), p, (size_t)n * 2, hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < n; ++i) {
                const uint32_t u = (uint32_t)v[(size_t)i] << 16;
                memcpy(out + i, &u, 4);
            }
        }
    });
}

int fm_llm_close(fm_llm* m) {
    return fm_guard([&] { delete m; });
}

}  // extern "C"

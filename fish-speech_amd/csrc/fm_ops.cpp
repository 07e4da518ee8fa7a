// fm_ops.cpp -- per-op test hooks of libfishmi (include/fishmi.h, "per-op parity hooks").
//
// Each hook runs ONE production kernel of the decode path on caller-supplied operands, so the
// GPU tests can hold the fused forms to the reference's per-op goldens (tests/golden/ops.npz):
//   fm_op_rmsnorm   RMSNorm (llama.py:989-1000) as the decode path computes it: the GEMV
//                   prologue (first layer / head: statistic from the row itself; later layers:
//                   statistic from the producing GEMV's per-tile sums of squares), or the
//                   standalone row kernel of the batched / prefill path
//   fm_op_qk_rope   QK-norm (llama.py:861-863) + RoPE with the bf16 table (llama.py:1003-1037)
//                   inside the fused decode attention kernels (slow attn_fd / attn_decode2, fast attn2)
//   fm_op_decode_attn  the whole slow decode attention (QK-norm, RoPE, KV write, scaled dot-product
//                   attention over the cache, llama.py:883-945) on R rows with caller K/V caches
//   fm_op_prompt_attn  the prompt-chunk causal attention (llama.py:883-946) over a cache prefix,
//                   on the split kernel or the flash-form attn_prefill_kernel
//   fm_op_embed     the Dual-AR input embedding (llama.py:399-420)
//   fm_rope_table   the host-built bf16 cos/sin table (no device needed)
// Operands are fp32 host arrays, converted to the precision's storage type (bf16 rounding is the
// caller's business: pass bf16-valued floats for bit-level comparisons).
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "fm_kernels.h"
#include "fm_runtime.h"

namespace {

// Every fill, copy and launch of a hook goes to the hook's own non-blocking stream, in order. (A
// non-blocking stream does not wait for the null stream, so a null-stream hipMemset of a buffer
// could land after a kernel on `s` has written it.)
struct DevBufs {
    hipStream_t s;
    std::vector<void*> ptrs;
    explicit DevBufs(hipStream_t st) : s(st) {}
    ~DevBufs() {
        (void)hipStreamSynchronize(s);
        for (void* p : ptrs) (void)hipFree(p);
    }
    void* alloc(size_t bytes) {
        void* p = nullptr;
        HIPCHK(hipMalloc(&p, bytes ? bytes : 16));
        HIPCHK(hipMemsetAsync(p, 0, bytes ? bytes : 16, s));
        ptrs.push_back(p);
        return p;
    }
    void put(void* d, const void* h, size_t bytes) {
        HIPCHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));  // the host array may be a temporary
    }
    // fp32 host -> device storage type T
    template <typename T> T* upload(const float* h, size_t n) {
        float* tmp = (float*)alloc(n * 4);
        put(tmp, h, n * 4);
        T* d = (T*)alloc(n * sizeof(T));
        launch_convert<T>(s, tmp, 0, (int64_t)n, d);
        HIPCHK(hipGetLastError());
        return d;
    }
};

template <typename T> void download(const T* d, size_t n, float* out, hipStream_t s) {
    std::vector<T> h(n);
    HIPCHK(hipMemcpyAsync(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (size_t i = 0; i < n; ++i) {
        if constexpr (sizeof(T) == 2) {
            const uint32_t u = (uint32_t)h[i] << 16;
            memcpy(&out[i], &u, 4);
        } else {
            out[i] = h[i];
        }
    }
}

struct StreamGuard {
    hipStream_t s = nullptr;
    explicit StreamGuard(int device) {
        int n = 0;
        FMCHECK(hipGetDeviceCount(&n) == hipSuccess && n > 0, "no HIP device visible");
        FMCHECK(device >= 0 && device < n, "bad device index");
        HIPCHK(hipSetDevice(device));
        HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    ~StreamGuard() {
        if (s) (void)hipStreamDestroy(s);
    }
};

template <typename T>
void rmsnorm_t(hipStream_t s, int mode, const float* x, const float* w, int R, int d, float eps, float* y) {
    DevBufs b(s);
    T* xd = b.upload<T>(x, (size_t)R * d);
    T* wd = b.upload<T>(w, (size_t)d);
    T* yd = (T*)b.alloc((size_t)R * d * sizeof(T));
    if (mode == 2) {
        launch_rmsnorm<T>(s, xd, d, wd, d, eps, yd, d, R);
    } else {
        // a 16-row GEMV of zeros: only its prologue's X' (stored through xn_out) is looked at
        T* wz = (T*)b.alloc((size_t)16 * d * sizeof(T));
        T* yz = (T*)b.alloc((size_t)R * 16 * sizeof(T));
        int* tickets = (int*)b.alloc(4096);
        GemvArgs<T> a{};
        a.W = wz;
        a.nw = wd;
        a.eps = eps;
        a.R = R;
        a.N = 16;
        a.K = d;
        a.Y = yz;
        a.ldy = 16;
        a.xn_out = yd;
        a.ldxo = d;
        a.tickets = tickets;
        if (mode == 0) {  // PRO_NORM: first layer / head, statistic from the row itself
            a.X = xd;
            a.ldx = d;
            launch_gemv<T>(s, a, PRO_NORM, EPI_STORE, 1);
        } else {
            // PRO_PRENORM: a zero-weight EPI_SLABFIN GEMV finalises x = round(x + round(0)) and
            // its per-16-column sums of squares, exactly as the wo / w2 GEMVs do for the next norm
            T* xz = (T*)b.alloc((size_t)R * 32 * sizeof(T));
            T* wz2 = (T*)b.alloc((size_t)d * 32 * sizeof(T));
            float* slab = (float*)b.alloc((size_t)R * d * 4);
            float* ss = (float*)b.alloc((size_t)(d / 16) * R * 4);
            T* xf = (T*)b.alloc((size_t)R * d * sizeof(T));
            GemvArgs<T> f{};
            f.W = wz2;
            f.X = xz;
            f.ldx = 32;
            f.R = R;
            f.N = d;
            f.K = 32;
            f.Yf = slab;
            f.ldy = d;
            f.res = xd;
            f.ldr = d;
            f.res_out = xf;
            f.ldro = d;
            f.ss_out = ss;
            f.tickets = tickets;
            f.eps = eps;
            launch_gemv<T>(s, f, PRO_PLAIN, EPI_SLABFIN, 1);
            a.X = xf;
            a.ldx = d;
            a.ss_in = ss;
            launch_gemv<T>(s, a, PRO_PRENORM, EPI_STORE, 1);
        }
    }
    HIPCHK(hipGetLastError());
    download<T>(yd, (size_t)R * d, y, s);
}

template <typename T>
void qk_rope_t(hipStream_t s, int kernel, const float* qkv, int nh, int nkv, int hd, const float* qn,
               const float* kn, int qk_norm, float eps, float base, int pos, float* q_out, float* k_out) {
    DevBufs b(s);
    const int ld = (nh + 2 * nkv) * hd;
    T* raw = b.upload<T>(qkv, (size_t)ld);
    T* qnd = qk_norm ? b.upload<T>(qn, (size_t)hd) : (T*)b.alloc((size_t)hd * sizeof(T));
    T* knd = qk_norm ? b.upload<T>(kn, (size_t)hd) : (T*)b.alloc((size_t)hd * sizeof(T));
    const int S = (pos + 1 + 7) / 8 * 8;
    auto tab = rope_table_host(S, hd, base);
    float* rope = (float*)b.alloc(tab.size() * 4);
    b.put(rope, tab.data(), tab.size() * 4);
    const size_t stride = (size_t)nkv * S * hd;
    T* kc = (T*)b.alloc(stride * sizeof(T));
    T* vc = (T*)b.alloc(stride * sizeof(T));
    T* out = (T*)b.alloc((size_t)nh * hd * sizeof(T));
    float* qd = (float*)b.alloc((size_t)nh * hd * 4);
    int* row = (int*)b.alloc(8);
    const int rs[2] = {0, pos};
    b.put(row, rs, 8);
    const float scale = 1.0f / sqrtf((float)hd);
    if (kernel == 0 || kernel == 2 || kernel == 3) {  // slow decode attention
        AttnDecArgs<T> a{raw, ld, row, row + 1, nh, nkv, hd, qk_norm, eps, qnd, knd, rope, kc, vc, stride, 0, S,
                         1, scale, nullptr};
        a.cap = attn2_cap(hd, nh / nkv, sizeof(T));
        a.maxsplit = FM_CEIL(S, std::min(a.cap, 16));  // covers both kernels' split counts
        a.part = (float*)b.alloc((size_t)nh * a.maxsplit * (hd + 2) * 4);
        a.cnt = (int*)b.alloc((size_t)nkv * 4);
        a.out = out;
        a.qdbg = qd;
        // kernel 0: attn_decode2 (the B <= 8 decode path), 2: attn_dec3 (the batched frame)
        if (kernel == 2) {
            launch_attn_decode3<T>(s, a, 1);
        } else if (kernel == 3) {  // attn_fd as the batch-1 decode runs it (8-wave blocks)
            FMCHECK(attn_fd_ok(hd, nh / nkv), "attn_fd: head_dim 32, 64 or 128, at most 4 q heads per kv head");
            a.cap = std::max(16, fm_tuning().fd_min16);
            a.nwb = fm_tuning().fd_nw;
            a.maxsplit = FM_CEIL(S, a.cap);
            launch_attn_fd<T>(s, a, 1);
        } else {
            a.maxsplit = FM_CEIL(S, a.cap);
            launch_attn_decode2<T>(s, a, 1);
        }
    } else {  // fast-model attention (one wave per q head) at codebook position pos
        FMCHECK(pos < 16, "fast attention positions are < 16");
        FastFusedArgs<T> a{raw, ld, row, nh, nkv, hd, qk_norm, eps, qnd, knd, rope, kc, vc, stride, 0, S, pos,
                           scale, out};
        a.qdbg = qd;
        launch_fast_attn2<T>(s, a, 1);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(q_out, qd, (size_t)nh * hd * 4, hipMemcpyDeviceToHost, s));
    for (int h = 0; h < nkv; ++h) download<T>(kc + (size_t)h * S * hd + (size_t)pos * hd, hd, k_out + (size_t)h * hd, s);
    HIPCHK(hipStreamSynchronize(s));
}

// R prompt rows of one slot at positions pos0 .. pos0 + R - 1 over caller caches [nkv][S][hd]
// (keys / values of every position <= pos0 + R - 1 already written, as qk_rope_cache leaves them)
template <typename T>
void prompt_attn_t(hipStream_t s, int kernel, const float* q, int R, int nh, int nkv, int hd, int pos0,
                   const float* kcache, const float* vcache, int S, float* out) {
    DevBufs b(s);
    T* qd = b.upload<T>(q, (size_t)R * nh * hd);
    T* kc = b.upload<T>(kcache, (size_t)nkv * S * hd);
    T* vc = b.upload<T>(vcache, (size_t)nkv * S * hd);
    T* o = (T*)b.alloc((size_t)R * nh * hd * sizeof(T));
    int* rows = (int*)b.alloc((size_t)2 * R * 4);
    std::vector<int> rs(2 * R);
    for (int r = 0; r < R; ++r) {
        rs[r] = 0;
        rs[R + r] = pos0 + r;
    }
    b.put(rows, rs.data(), rs.size() * 4);
    const int split = 64, maxsplit = FM_CEIL(S, split);
    AttnArgs<T> a{qd, rows, rows + R, kc, vc, (size_t)nkv * S * hd, 0, S, nh, nkv, hd, split, maxsplit,
                  1.0f / sqrtf((float)hd), (float*)b.alloc((size_t)R * nh * maxsplit * (hd + 2) * 4)};
    FmTuning& tu = fm_tuning();
    const int keep = tu.prefill_attn;
    tu.prefill_attn = kernel;
    launch_attn<T>(s, a, R, maxsplit, o, true);
    tu.prefill_attn = keep;
    download<T>(o, (size_t)R * nh * hd, out, s);
}

// one decode attention launch over R rows (slot r = row r) with caller K/V caches [R][nkv][S][hd]
// holding rows < pos[r]; the kernel writes row pos[r] (normed + roped k, raw v) itself
template <typename T>
void decode_attn_t(hipStream_t s, int kernel, const float* qkv, int R, int nh, int nkv, int hd, const float* qn,
                   const float* kn, int qk_norm, float eps, float base, const int* pos, const float* kcache,
                   const float* vcache, int S, int min_split, float* out, float* kc_out, float* vc_out) {
    DevBufs b(s);
    const int ld = (nh + 2 * nkv) * hd;
    T* raw = b.upload<T>(qkv, (size_t)R * ld);
    T* qnd = qk_norm ? b.upload<T>(qn, (size_t)hd) : (T*)b.alloc((size_t)hd * sizeof(T));
    T* knd = qk_norm ? b.upload<T>(kn, (size_t)hd) : (T*)b.alloc((size_t)hd * sizeof(T));
    auto tab = rope_table_host(S, hd, base);
    float* rope = (float*)b.alloc(tab.size() * 4);
    b.put(rope, tab.data(), tab.size() * 4);
    const size_t stride = (size_t)nkv * S * hd;
    T* kc = b.upload<T>(kcache, (size_t)R * stride);
    T* vc = b.upload<T>(vcache, (size_t)R * stride);
    T* o = (T*)b.alloc((size_t)R * nh * hd * sizeof(T));
    int* rows = (int*)b.alloc((size_t)2 * R * 4);
    std::vector<int> rs(2 * R);
    for (int r = 0; r < R; ++r) {
        rs[r] = r;
        rs[R + r] = pos[r];
    }
    b.put(rows, rs.data(), rs.size() * 4);
    AttnDecArgs<T> a{raw, ld, rows, rows + R, nh, nkv, hd, qk_norm, eps, qnd, knd, rope, kc, vc, stride, 0, S,
                     1, 1.0f / sqrtf((float)hd), nullptr};
    const int g = nh / nkv;
    a.maxsplit = FM_CEIL(S, 16);
    a.part = (float*)b.alloc((size_t)R * nh * a.maxsplit * (hd + 2) * 4);
    a.cnt = (int*)b.alloc((size_t)R * nkv * 4);
    a.out = o;
    if (kernel == 3) {
        FMCHECK(attn_fd_ok(hd, g), "attn_fd: head_dim 32, 64 or 128 and at most 4 q heads per kv head");
        a.cap = min_split;
        launch_attn_fd<T>(s, a, R);
    } else if (kernel == 2) {
        FMCHECK(hd % 32 == 0 && hd <= 128 && g <= 6, "attn_dec3: hd a multiple of 32 up to 128, g <= 6");
        launch_attn_decode3<T>(s, a, R);
    } else {
        a.cap = std::min(min_split, attn2_cap(hd, g, sizeof(T)));
        a.maxsplit = FM_CEIL(S, a.cap);
        launch_attn_decode2<T>(s, a, R);
    }
    HIPCHK(hipGetLastError());
    download<T>(o, (size_t)R * nh * hd, out, s);
    download<T>(kc, (size_t)R * stride, kc_out, s);
    download<T>(vc, (size_t)R * stride, vc_out, s);
}

template <typename T>
void embed_t(hipStream_t s, const int32_t* tok, int R, const float* emb, int V, const float* cbemb, int d, int C,
             int cb, int sb, int se, int scale, float* x) {
    DevBufs b(s);
    T* e = b.upload<T>(emb, (size_t)V * d);
    T* ce = b.upload<T>(cbemb, (size_t)C * cb * d);
    int32_t* td = (int32_t*)b.alloc((size_t)R * (C + 1) * 4);
    b.put(td, tok, (size_t)R * (C + 1) * 4);
    T* xd = (T*)b.alloc((size_t)R * d * sizeof(T));
    launch_embed<T>(s, td, R, e, ce, d, C, cb, sb, se, scale, xd, nullptr);
    HIPCHK(hipGetLastError());
    download<T>(xd, (size_t)R * d, x, s);
}

}  // namespace

extern "C" {

int fm_op_rmsnorm(int device, int precision, int mode, const float* x, const float* w, int R, int d, float eps,
                  float* y) {
    return fm_guard([&] {
        FMCHECK(x && w && y, "null argument");
        FMCHECK(mode >= 0 && mode <= 2, "mode must be 0 (PRO_NORM), 1 (PRO_PRENORM) or 2 (row kernel)");
        FMCHECK(R >= 1 && d >= 32 && d % 32 == 0, "need R >= 1 and d a multiple of 32");
        FMCHECK(mode == 2 || (R <= 8 && d <= 4096), "GEMV prologue modes need R <= 8 and d <= 4096");
        StreamGuard g(device);
        if (precision == FM_PREC_BF16)
            rmsnorm_t<bf16_t>(g.s, mode, x, w, R, d, eps, y);
        else
            rmsnorm_t<float>(g.s, mode, x, w, R, d, eps, y);
    });
}

int fm_op_prompt_attn(int device, int precision, int kernel, const float* q, int R, int nh, int nkv, int hd, int pos0,
                      const float* kcache, const float* vcache, int S, float* out) {
    return fm_guard([&] {
        FMCHECK(q && kcache && vcache && out, "null argument");
        FMCHECK(kernel == 0 || kernel == 1, "kernel must be 0 (split + combine) or 1 (attn_prefill_kernel)");
        FMCHECK(R >= 1 && R <= 1024 && nh % nkv == 0 && pos0 >= 0 && pos0 + R <= S, "bad rows / positions");
        FMCHECK(kernel == 0 || (precision == FM_PREC_BF16 && hd == 128 && nh / nkv <= 4),
                "attn_prefill_kernel: bf16, head_dim 128, at most 4 q heads per kv head");
        StreamGuard g(device);
        if (precision == FM_PREC_BF16)
            prompt_attn_t<bf16_t>(g.s, kernel, q, R, nh, nkv, hd, pos0, kcache, vcache, S, out);
        else
            prompt_attn_t<float>(g.s, kernel, q, R, nh, nkv, hd, pos0, kcache, vcache, S, out);
    });
}

int fm_op_decode_attn(int device, int precision, int kernel, const float* qkv, int R, int nh, int nkv, int hd,
                      const float* qn, const float* kn, int qk_norm, float eps, float rope_base, const int* pos,
                      const float* kcache, const float* vcache, int S, int min_split, float* out, float* kc_out,
                      float* vc_out) {
    return fm_guard([&] {
        FMCHECK(qkv && pos && kcache && vcache && out && kc_out && vc_out, "null argument");
        FMCHECK(!qk_norm || (qn && kn), "qk_norm needs both norm weights");
        FMCHECK(kernel == 0 || kernel == 2 || kernel == 3, "kernel must be 0 (attn_decode2), 2 (attn_dec3) or 3 (attn_fd)");
        FMCHECK(R >= 1 && R <= 64 && nh >= 1 && nkv >= 1 && nh % nkv == 0, "bad rows / head counts");
        FMCHECK(hd >= 32 && hd <= 128 && hd % 32 == 0, "head_dim a multiple of 32 up to 128");
        FMCHECK(S >= 16 && S <= 65536 && min_split >= 16 && min_split % 16 == 0, "bad S / min_split");
        for (int r = 0; r < R; ++r) FMCHECK(pos[r] >= 0 && pos[r] < S, "position outside the cache");
        StreamGuard g(device);
        if (precision == FM_PREC_BF16)
            decode_attn_t<bf16_t>(g.s, kernel, qkv, R, nh, nkv, hd, qn, kn, qk_norm, eps, rope_base, pos, kcache, vcache,
                                  S, min_split, out, kc_out, vc_out);
        else
            decode_attn_t<float>(g.s, kernel, qkv, R, nh, nkv, hd, qn, kn, qk_norm, eps, rope_base, pos, kcache, vcache,
                                 S, min_split, out, kc_out, vc_out);
    });
}

int fm_op_qk_rope(int device, int precision, int kernel, const float* qkv, int nh, int nkv, int hd, const float* qn,
                  const float* kn, int qk_norm, float eps, float rope_base, int pos, float* q_out, float* k_out) {
    return fm_guard([&] {
        FMCHECK(qkv && q_out && k_out, "null argument");
        FMCHECK(!qk_norm || (qn && kn), "qk_norm needs both norm weights");
        FMCHECK(kernel >= 0 && kernel <= 3,
                "kernel must be 0 (slow attn_decode2), 1 (fast attn2), 2 (slow attn_dec3) or 3 (slow attn_fd)");
        FMCHECK(nh >= 1 && nkv >= 1 && nh % nkv == 0 && nh / nkv <= 16, "bad head counts");
        FMCHECK(hd >= 8 && hd <= 256 && hd % 8 == 0, "bad head_dim");
        FMCHECK(pos >= 0 && pos < 65536, "bad position");
        StreamGuard g(device);
        if (precision == FM_PREC_BF16)
            qk_rope_t<bf16_t>(g.s, kernel, qkv, nh, nkv, hd, qn, kn, qk_norm, eps, rope_base, pos, q_out, k_out);
        else
            qk_rope_t<float>(g.s, kernel, qkv, nh, nkv, hd, qn, kn, qk_norm, eps, rope_base, pos, q_out, k_out);
    });
}

int fm_op_embed(int device, int precision, const int32_t* tok, int R, const float* emb, int vocab,
                const float* cbemb, int dim, int num_codebooks, int codebook_size, int semantic_begin_id,
                int semantic_end_id, int scale_codebook_embeddings, float* x) {
    return fm_guard([&] {
        FMCHECK(tok && emb && cbemb && x && R >= 1 && dim % 8 == 0, "bad arguments");
        for (int r = 0; r < R; ++r) {
            FMCHECK(tok[(size_t)r * (num_codebooks + 1)] >= 0 && tok[(size_t)r * (num_codebooks + 1)] < vocab,
                    "token id out of range");
            for (int q = 1; q <= num_codebooks; ++q) {
                const int v = tok[(size_t)r * (num_codebooks + 1) + q];
                FMCHECK(v >= 0 && v < codebook_size, "codebook token out of range");
            }
        }
        StreamGuard g(device);
        if (precision == FM_PREC_BF16)
            embed_t<bf16_t>(g.s, tok, R, emb, vocab, cbemb, dim, num_codebooks, codebook_size, semantic_begin_id,
                            semantic_end_id, scale_codebook_embeddings, x);
        else
            embed_t<float>(g.s, tok, R, emb, vocab, cbemb, dim, num_codebooks, codebook_size, semantic_begin_id,
                           semantic_end_id, scale_codebook_embeddings, x);
    });
}

// weight-only int4: the device quantizer (launch_quant4) on a caller bf16 matrix, then the decode
// GEMV on R rows of x three ways: the streamed int4 codes (when gs % 128 == 0), the bf16 weights it
// dequantised to, and (for reference) nothing else -- y_q4 / y_bf16 are [R][N] fp32 (EPI_F32)
int fm_op_quant4(int device, const float* w, int N, int K, int gs, uint8_t* q, float* scale, float* zero,
                 float* w_deq, const float* x, int R, float* y_q4, float* y_bf16) {
    return fm_guard([&] {
        FMCHECK(w && q && scale && zero && w_deq && N >= 1 && gs >= 2 && K % gs == 0, "bad arguments");
        FMCHECK(!x || (R >= 1 && R <= 8 && K % 32 == 0 && y_bf16), "bad GEMV arguments");
        StreamGuard g(device);
        DevBufs b(g.s);
        const int Np = (N + 15) / 16 * 16;
        bf16_t* dw = (bf16_t*)b.alloc((size_t)Np * K * 2);
        {
            bf16_t* t = b.upload<bf16_t>(w, (size_t)N * K);
            HIPCHK(hipMemcpyAsync(dw, t, (size_t)N * K * 2, hipMemcpyDeviceToDevice, g.s));
        }
        uint8_t* dq = (uint8_t*)b.alloc((size_t)Np * K);
        uint32_t* dsz = (uint32_t*)b.alloc((size_t)Np * (K / gs) * 4);
        launch_quant4(g.s, dw, N, K, gs, dq, dsz);
        HIPCHK(hipGetLastError());
        std::vector<uint16_t> hw((size_t)N * K);
        std::vector<uint32_t> hs((size_t)N * (K / gs));
        HIPCHK(hipMemcpyAsync(q, dq, (size_t)N * K, hipMemcpyDeviceToHost, g.s));
        HIPCHK(hipMemcpyAsync(hw.data(), dw, hw.size() * 2, hipMemcpyDeviceToHost, g.s));
        HIPCHK(hipMemcpyAsync(hs.data(), dsz, hs.size() * 4, hipMemcpyDeviceToHost, g.s));
        HIPCHK(hipStreamSynchronize(g.s));
        for (size_t i = 0; i < hw.size(); ++i) {
            const uint32_t u = (uint32_t)hw[i] << 16;
            memcpy(&w_deq[i], &u, 4);
        }
        for (size_t i = 0; i < hs.size(); ++i) {
            const uint32_t us = hs[i] << 16, uz = hs[i] & 0xffff0000u;
            memcpy(&scale[i], &us, 4);
            memcpy(&zero[i], &uz, 4);
        }
        if (!x) return;
        // the decode GEMV: packed bf16 fragments of the dequantised weights, and the int4 stream
        bf16_t* pk = (bf16_t*)b.alloc((size_t)Np * K * 2);
        launch_pack<bf16_t>(g.s, dw, N, K, pk);
        bf16_t* dx = b.upload<bf16_t>(x, (size_t)R * K);
        float* dy = (float*)b.alloc((size_t)R * N * 4);
        int* tk = (int*)b.alloc((size_t)(Np / 16 + 16) * 4);
        GemvArgs<bf16_t> a{};
        a.W = pk;
        a.X = dx;
        a.ldx = K;
        a.R = R;
        a.N = N;
        a.K = K;
        a.Yf = dy;
        a.ldy = N;
        a.tickets = tk;
        a.eps = 1e-6f;
        launch_gemv<bf16_t>(g.s, a, PRO_PLAIN, EPI_F32, 1);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(y_bf16, dy, (size_t)R * N * 4, hipMemcpyDeviceToHost, g.s));
        HIPCHK(hipStreamSynchronize(g.s));
        if (y_q4 && gs % 128 == 0 && K % 128 == 0) {
            uint8_t* q4 = (uint8_t*)b.alloc((size_t)Np * K / 2);
            uint32_t* sz4 = (uint32_t*)b.alloc((size_t)(Np / 16) * (K / 128) * 16 * 4);
            launch_pack_q4(g.s, dq, N, K, q4);
            launch_pack_sz4(g.s, dsz, N, K, gs, sz4);
            a.Wq = q4;
            a.wsz = sz4;
            launch_gemv<bf16_t>(g.s, a, PRO_PLAIN, EPI_F32, 1);
            HIPCHK(hipGetLastError());
            HIPCHK(hipMemcpyAsync(y_q4, dy, (size_t)R * N * 4, hipMemcpyDeviceToHost, g.s));
            HIPCHK(hipStreamSynchronize(g.s));
        }
    });
}

int fm_rope_table(int seq_len, int head_dim, float base, float* out) {
    return fm_guard([&] {
        FMCHECK(out && seq_len >= 1 && head_dim >= 2 && head_dim % 2 == 0, "bad arguments");
        auto t = rope_table_host(seq_len, head_dim, base);
        memcpy(out, t.data(), t.size() * 4);
    });
}

}  // extern "C"

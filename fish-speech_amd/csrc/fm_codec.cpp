// fm_codec.cpp -- host runtime of the modded-DAC decode path (C ABI in include/fishmi.h).
//
// DAC.from_indices (modded_dac.py:925-927) = RVQ decode (rvq.py:352-366) -> post_module
// WindowLimitedTransformer (modded_dac.py:349-439) -> upsample 2x[CausalTransConvNet k2s2 +
// ConvNeXtBlock] (rvq.py:263-276) -> Decoder (modded_dac.py:760-801).  Weight norm is folded
// once at finalize; conv weights are re-laid per output phase and packed for the MFMA GEMMs.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <memory>

#include "fm_codec.h"
#include "fm_runtime.h"

struct PackedW {
    void* w = nullptr;
    size_t wphase = 0;
    int Co = 0, Ci = 0, ntaps = 1, nphase = 1, stride = 1;
    int shift[8] = {0};
    void* bias = nullptr;
};

struct TLayer {
    void *an, *fn, *ag, *fg;
    PackedW wqkv, wo, w1, w3, w2;
};
struct RU {
    void *a0, *a2;
    PackedW c7, c1;
};
struct DBlock {
    void* alpha;
    PackedW ct;
    RU ru[3];
};

// Streamed decode (fm_codec_decode_chunk): the codec is causal end to end, so chunk k of a
// stream is decoded exactly like the matching rows of the one-shot decode when every causal
// reader sees the previous chunk's rows it would have read: each conv site's last (k-1)*dil input
// rows, the ConvNeXt depthwise k7 inputs, each transformer layer's window-1 post-RoPE key/value
// rows (and the RoPE position).  Those rows live in per-site state buffers, copied into a prefix
// of the activation buffer before the reader runs and refreshed from it right after.
static constexpr int CODEC_HALO = 128;           // prefix rows of the buffers read with context
static constexpr int CODEC_STREAM_MAX = 1 << 15;  // RoPE positions of one stream (25 min of audio)

struct fm_codec {
    fm_codec_config c{};
    int device = 0, prec = FM_PREC_BF16, max_frames = 0;
    size_t esz = 2;
    hipStream_t stream = nullptr;
    std::map<std::string, DTensor> w;  // raw fp32 tensors
    bool finalized = false;
    std::vector<void*> allocs;
    // prepared
    RvqPtrs rvq{};
    std::vector<TLayer> tl;
    void* tnorm = nullptr;
    PackedW up_ct[2], up_pw1[2], up_pw2[2];
    void *up_dw[2], *up_db[2], *up_lw[2], *up_lb[2], *up_gm[2];
    PackedW conv0, convf;
    DBlock blk[4];
    void* falpha = nullptr;
    float* rope = nullptr;
    // buffers
    int32_t* d_codes = nullptr;
    void *z = nullptr, *xn = nullptr, *qkv = nullptr, *att = nullptr, *g1 = nullptr, *g3 = nullptr;
    void *u0 = nullptr, *u1 = nullptr, *hh = nullptr, *gb = nullptr;
    void *xb = nullptr, *A = nullptr, *B = nullptr, *Cb = nullptr;
    float* wave = nullptr;
    // stream state: carried rows per causal site (zeros at a stream start == causal padding)
    void* st_kv[16] = {};                   // per transformer layer: window-1 qkv rows
    void *st_dw[2] = {}, *st_c0 = nullptr, *st_cf = nullptr;
    void *st_ct[4] = {}, *st_c7[4][3] = {};
    std::vector<std::pair<void*, size_t>> st_all;
    int spos = 0;                           // frames already streamed
    double last_ms = 0, flops = 0, total_ms = 0, total_flops = 0;
    int64_t launches = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;

    ~fm_codec() {
        if (device >= 0) (void)hipSetDevice(device);
        for (auto& kv : w)
            if (kv.second.p) (void)hipFree(kv.second.p);
        for (void* p : allocs) (void)hipFree(p);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (stream) (void)hipStreamDestroy(stream);
    }
    void* dalloc_prefixed(size_t body, size_t prefix) {  // prefix bytes in front of the base
        return (char*)dalloc(prefix + body) + prefix;
    }
    void* dstate(size_t bytes) {
        void* p = dalloc(bytes);
        st_all.emplace_back(p, bytes);
        return p;
    }
    void* dalloc(size_t bytes) {
        void* p = nullptr;
        hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
        if (e != hipSuccess) throw FmError{FM_ERR_OOM, "hipMalloc failed: " + std::string(hipGetErrorString(e))};
        HIPCHK(hipMemsetAsync(p, 0, bytes ? bytes : 16, stream));
        allocs.push_back(p);
        return p;
    }
};

// ---- inventory (decode-side state_dict keys; mirrors fishmi/checkpoint.codec_tensor_shapes) ----
static void add(fm_codec* m, const std::string& n, int64_t numel) {
    DTensor t;
    t.numel = numel;
    t.rows = 1;
    t.cols = numel;
    m->w[n] = t;
}
static void build_inventory(fm_codec* m) {
    const fm_codec_config& c = m->c;
    const int D = c.latent, cd = c.codebook_dim;
    for (int q = 0; q <= c.n_codebooks; ++q) {
        std::string p = q == 0 ? "quantizer.semantic_quantizer.quantizers.0."
                               : "quantizer.quantizer.quantizers." + std::to_string(q - 1) + ".";
        add(m, p + "codebook.weight", (int64_t)(q == 0 ? c.semantic_codebook_size : c.codebook_size) * cd);
        add(m, p + "out_proj.weight_g", D);
        add(m, p + "out_proj.weight_v", (int64_t)D * cd);
        add(m, p + "out_proj.bias", D);
    }
    const int HD = c.t_heads * c.t_head_dim, I = c.t_inter;
    for (int l = 0; l < c.t_layers; ++l) {
        std::string p = "quantizer.post_module.layers." + std::to_string(l) + ".";
        add(m, p + "attention.wqkv.weight", (int64_t)3 * HD * D);
        add(m, p + "attention.wo.weight", (int64_t)D * HD);
        add(m, p + "feed_forward.w1.weight", (int64_t)I * D);
        add(m, p + "feed_forward.w3.weight", (int64_t)I * D);
        add(m, p + "feed_forward.w2.weight", (int64_t)D * I);
        add(m, p + "ffn_norm.weight", D);
        add(m, p + "attention_norm.weight", D);
        add(m, p + "attention_layer_scale.gamma", D);
        add(m, p + "ffn_layer_scale.gamma", D);
    }
    add(m, "quantizer.post_module.norm.weight", D);
    for (int u = 0; u < 2; ++u) {
        std::string p = "quantizer.upsample." + std::to_string(u) + ".";
        add(m, p + "0.conv.weight", (int64_t)D * D * 2);
        add(m, p + "0.conv.bias", D);
        add(m, p + "1.dwconv.conv.weight", (int64_t)D * 7);
        add(m, p + "1.dwconv.conv.bias", D);
        add(m, p + "1.norm.weight", D);
        add(m, p + "1.norm.bias", D);
        add(m, p + "1.pwconv1.weight", (int64_t)4 * D * D);
        add(m, p + "1.pwconv1.bias", 4 * D);
        add(m, p + "1.pwconv2.weight", (int64_t)4 * D * D);
        add(m, p + "1.pwconv2.bias", D);
        add(m, p + "1.gamma", D);
    }
    auto wn = [&](const std::string& p, int co, int ci, int k, bool tr) {
        add(m, p + "conv.parametrizations.weight.original0", tr ? ci : co);
        add(m, p + "conv.parametrizations.weight.original1", (int64_t)co * ci * k);
        add(m, p + "conv.bias", co);
    };
    const int ch = c.decoder_dim;
    wn("decoder.model.0.", ch, D, 7, false);
    int cin = ch;
    const int rates[4] = {8, 8, 4, 2};
    for (int b = 0; b < 4; ++b) {
        const int cout = cin / 2;
        std::string p = "decoder.model." + std::to_string(b + 1) + ".block.";
        add(m, p + "0.alpha", cin);
        wn(p + "1.", cout, cin, 2 * rates[b], true);
        for (int r = 0; r < 3; ++r) {
            std::string rp = p + std::to_string(r + 2) + ".block.";
            add(m, rp + "0.alpha", cout);
            wn(rp + "1.", cout, cout, 7, false);
            add(m, rp + "2.alpha", cout);
            wn(rp + "3.", cout, cout, 1, false);
        }
        cin = cout;
    }
    add(m, "decoder.model.5.alpha", cin);
    wn("decoder.model.6.", 1, cin, 7, false);
}

static float* raw(fm_codec* m, const std::string& n) {
    auto it = m->w.find(n);
    FMCHECK(it != m->w.end() && it->second.set, "codec tensor not set: " + n);
    return (float*)it->second.p;
}

// fp32 -> T copy of a small vector
static void* as_T(fm_codec* m, const float* src, int64_t n) {
    void* d = m->dalloc((size_t)n * m->esz);
    if (m->prec == FM_PREC_BF16)
        launch_convert<bf16_t>(m->stream, src, 0, n, (bf16_t*)d);
    else
        launch_convert<float>(m->stream, src, 0, n, (float*)d);
    return d;
}

// prepare a GEMM weight: kind per conv_weight_kernel; returns phases packed
static PackedW prep(fm_codec* m, const float* w, int kind, int Ci, int Co, int k, int s, int dil,
                    const float* bias) {
    PackedW p;
    p.Co = Co;
    p.Ci = Ci;
    p.ntaps = kind == 0 ? k : (kind == 1 ? 2 : 1);
    p.nphase = (kind == 1 || kind == 2) ? s : 1;
    p.stride = (kind == 1 || kind == 2) ? s : 1;
    FMCHECK(p.ntaps <= 8, "too many taps");
    FMCHECK(Ci % 8 == 0, "codec channel counts must be multiples of 8");
    for (int j = 0; j < p.ntaps; ++j) p.shift[j] = kind == 0 ? (k - 1 - j) * dil : j;
    const int Kt = (p.ntaps * Ci + 31) / 32 * 32;  // padded
    const size_t rm = (size_t)p.nphase * Co * Kt;
    p.wphase = (size_t)(Co + 15) / 16 * 16 * Kt;
    void* tmp = nullptr;
    HIPCHK(hipMalloc(&tmp, rm * m->esz));
    p.w = m->dalloc(p.wphase * p.nphase * m->esz);
    if (m->prec == FM_PREC_BF16) {
        launch_conv_weight<bf16_t>(m->stream, w, kind, Ci, Co, k, s, (bf16_t*)tmp);
        for (int ph = 0; ph < p.nphase; ++ph)
            launch_pack<bf16_t>(m->stream, (const bf16_t*)tmp + (size_t)ph * Co * Kt, Co, Kt,
                                (bf16_t*)p.w + ph * p.wphase);
    } else {
        launch_conv_weight<float>(m->stream, w, kind, Ci, Co, k, s, (float*)tmp);
        for (int ph = 0; ph < p.nphase; ++ph)
            launch_pack<float>(m->stream, (const float*)tmp + (size_t)ph * Co * Kt, Co, Kt,
                               (float*)p.w + ph * p.wphase);
    }
    HIPCHK(hipStreamSynchronize(m->stream));
    HIPCHK(hipFree(tmp));
    p.bias = bias ? as_T(m, bias, Co) : nullptr;
    return p;
}

static const float* fold(fm_codec* m, const std::string& g, const std::string& v, int rows, int per) {
    float* out = (float*)m->dalloc((size_t)rows * per * 4);
    launch_wn_fold(m->stream, raw(m, g), raw(m, v), rows, per, out);
    return out;
}

static PackedW prep_wn_conv(fm_codec* m, const std::string& p, int Ci, int Co, int k, int dil) {
    const float* w = fold(m, p + "conv.parametrizations.weight.original0", p + "conv.parametrizations.weight.original1",
                          Co, Ci * k);
    return prep(m, w, 0, Ci, Co, k, 1, dil, raw(m, p + "conv.bias"));
}

static void finalize(fm_codec* m) {
    if (m->finalized) return;
    for (auto& kv : m->w) FMCHECK(kv.second.set, "codec tensor not set: " + kv.first);
    const fm_codec_config& c = m->c;
    const int D = c.latent, cd = c.codebook_dim, HD = c.t_heads * c.t_head_dim, I = c.t_inter;
    FMCHECK(c.n_codebooks + 1 <= 16, "too many codebooks");
    FMCHECK(c.t_head_dim <= 64 && c.window <= 128, "codec transformer: head_dim <= 64, window <= 128");
    FMCHECK(HD == D, "codec transformer: n_head * head_dim must equal dim");
    for (int q = 0; q <= c.n_codebooks; ++q) {
        std::string p = q == 0 ? "quantizer.semantic_quantizer.quantizers.0."
                               : "quantizer.quantizer.quantizers." + std::to_string(q - 1) + ".";
        m->rvq.cb[q] = raw(m, p + "codebook.weight");
        m->rvq.w[q] = fold(m, p + "out_proj.weight_g", p + "out_proj.weight_v", D, cd);
        m->rvq.b[q] = raw(m, p + "out_proj.bias");
    }
    m->tl.resize(c.t_layers);
    for (int l = 0; l < c.t_layers; ++l) {
        std::string p = "quantizer.post_module.layers." + std::to_string(l) + ".";
        TLayer& L = m->tl[l];
        L.an = as_T(m, raw(m, p + "attention_norm.weight"), D);
        L.fn = as_T(m, raw(m, p + "ffn_norm.weight"), D);
        L.ag = as_T(m, raw(m, p + "attention_layer_scale.gamma"), D);
        L.fg = as_T(m, raw(m, p + "ffn_layer_scale.gamma"), D);
        L.wqkv = prep(m, raw(m, p + "attention.wqkv.weight"), 3, D, 3 * HD, 1, 1, 1, nullptr);
        L.wo = prep(m, raw(m, p + "attention.wo.weight"), 3, HD, D, 1, 1, 1, nullptr);
        L.w1 = prep(m, raw(m, p + "feed_forward.w1.weight"), 3, D, I, 1, 1, 1, nullptr);
        L.w3 = prep(m, raw(m, p + "feed_forward.w3.weight"), 3, D, I, 1, 1, 1, nullptr);
        L.w2 = prep(m, raw(m, p + "feed_forward.w2.weight"), 3, I, D, 1, 1, 1, nullptr);
    }
    m->tnorm = as_T(m, raw(m, "quantizer.post_module.norm.weight"), D);
    for (int u = 0; u < 2; ++u) {
        std::string p = "quantizer.upsample." + std::to_string(u) + ".";
        m->up_ct[u] = prep(m, raw(m, p + "0.conv.weight"), 2, D, D, 2, 2, 1, raw(m, p + "0.conv.bias"));
        m->up_dw[u] = as_T(m, raw(m, p + "1.dwconv.conv.weight"), (int64_t)D * 7);
        m->up_db[u] = as_T(m, raw(m, p + "1.dwconv.conv.bias"), D);
        m->up_lw[u] = as_T(m, raw(m, p + "1.norm.weight"), D);
        m->up_lb[u] = as_T(m, raw(m, p + "1.norm.bias"), D);
        m->up_pw1[u] = prep(m, raw(m, p + "1.pwconv1.weight"), 3, D, 4 * D, 1, 1, 1, raw(m, p + "1.pwconv1.bias"));
        m->up_pw2[u] = prep(m, raw(m, p + "1.pwconv2.weight"), 3, 4 * D, D, 1, 1, 1, raw(m, p + "1.pwconv2.bias"));
        m->up_gm[u] = as_T(m, raw(m, p + "1.gamma"), D);
    }
    const int ch = c.decoder_dim;
    m->conv0 = prep_wn_conv(m, "decoder.model.0.", D, ch, 7, 1);
    int cin = ch;
    const int rates[4] = {8, 8, 4, 2};
    for (int b = 0; b < 4; ++b) {
        const int cout = cin / 2, s = rates[b];
        std::string p = "decoder.model." + std::to_string(b + 1) + ".block.";
        DBlock& B = m->blk[b];
        B.alpha = as_T(m, raw(m, p + "0.alpha"), cin);
        // ConvTranspose1d weight norm: dim 0 is the INPUT channel (norm over (out, k))
        const float* wt = fold(m, p + "1.conv.parametrizations.weight.original0",
                               p + "1.conv.parametrizations.weight.original1", cin, cout * 2 * s);
        B.ct = prep(m, wt, 1, cin, cout, 2 * s, s, 1, raw(m, p + "1.conv.bias"));
        const int dils[3] = {1, 3, 9};
        for (int r = 0; r < 3; ++r) {
            std::string rp = p + std::to_string(r + 2) + ".block.";
            B.ru[r].a0 = as_T(m, raw(m, rp + "0.alpha"), cout);
            B.ru[r].a2 = as_T(m, raw(m, rp + "2.alpha"), cout);
            B.ru[r].c7 = prep_wn_conv(m, rp + "1.", cout, cout, 7, dils[r]);
            B.ru[r].c1 = prep_wn_conv(m, rp + "3.", cout, cout, 1, 1);
        }
        cin = cout;
    }
    m->falpha = as_T(m, raw(m, "decoder.model.5.alpha"), cin);
    m->convf = prep_wn_conv(m, "decoder.model.6.", cin, 1, 7, 1);
    // rope table for the transformer (positions 0..Tmax-1, bf16-valued)
    auto rt = rope_table_host(std::max(m->max_frames, CODEC_STREAM_MAX), c.t_head_dim, c.rope_base);
    m->rope = (float*)m->dalloc(rt.size() * 4);
    HIPCHK(hipMemcpy(m->rope, rt.data(), rt.size() * 4, hipMemcpyHostToDevice));
    // activations
    const size_t Tm = m->max_frames, E = m->esz;
    m->d_codes = (int32_t*)m->dalloc((size_t)(c.n_codebooks + 1) * Tm * 4);
    m->z = m->dalloc(Tm * D * E);
    m->xn = m->dalloc(Tm * D * E);
    m->qkv = m->dalloc_prefixed(Tm * 3 * HD * E, (size_t)CODEC_HALO * 3 * HD * E);
    m->att = m->dalloc(Tm * HD * E);
    m->g1 = m->dalloc(Tm * I * E);
    m->g3 = m->dalloc(Tm * I * E);
    m->u0 = m->dalloc_prefixed(Tm * 2 * D * E, (size_t)CODEC_HALO * D * E);
    m->u1 = m->dalloc_prefixed(Tm * 4 * D * E, (size_t)CODEC_HALO * D * E);
    m->hh = m->dalloc(Tm * 4 * D * E);
    m->gb = m->dalloc(Tm * 4 * 4 * D * E);
    size_t maxact = (size_t)4 * ch;
    {
        int cc = ch, L = 4;
        for (int b = 0; b < 4; ++b) {
            cc /= 2;
            L *= rates[b];
            maxact = std::max(maxact, (size_t)cc * L);
        }
    }
    m->xb = m->dalloc(Tm * maxact * E);
    m->A = m->dalloc_prefixed(Tm * maxact * E, (size_t)CODEC_HALO * std::max(ch, D) * E);
    m->B = m->dalloc_prefixed(Tm * maxact * E, (size_t)CODEC_HALO * std::max(ch, D) * E);
    FMCHECK(c.t_layers <= 16 && c.window - 1 <= CODEC_HALO, "codec stream state: t_layers <= 16, window <= 129");
    for (int l = 0; l < c.t_layers; ++l) m->st_kv[l] = m->dstate((size_t)(c.window - 1) * 3 * HD * E);
    for (int u = 0; u < 2; ++u) m->st_dw[u] = m->dstate((size_t)6 * D * E);
    m->st_c0 = m->dstate((size_t)6 * D * E);
    {
        int cc = ch;
        const int dl[3] = {1, 3, 9};
        for (int b = 0; b < 4; ++b) {
            m->st_ct[b] = m->dstate((size_t)cc * E);
            for (int r = 0; r < 3; ++r) m->st_c7[b][r] = m->dstate((size_t)6 * dl[r] * (cc / 2) * E);
            cc /= 2;
        }
        m->st_cf = m->dstate((size_t)6 * cc * E);
    }
    m->Cb = m->dalloc(Tm * maxact * E);
    m->wave = (float*)m->dalloc(Tm * 2048 * 4);
    HIPCHK(hipEventCreate(&m->e0));
    HIPCHK(hipEventCreate(&m->e1));
    HIPCHK(hipStreamSynchronize(m->stream));
    m->finalized = true;
}

template <typename T> struct CRun {
    fm_codec* m;
    hipStream_t s;
    explicit CRun(fm_codec* mm) : m(mm), s(mm->stream) {}

    void gemm(const PackedW& W, const void* x, int ldx, int Lq, int Lx, void* out, int ldo, int flags,
              const void* res = nullptr, int ldr = 0, const void* gamma = nullptr, const void* alpha2 = nullptr,
              void* out2 = nullptr, int ldo2 = 0, int lo = 0) {
        ConvArgs<T> a{};
        a.x = (const T*)x;
        a.ldx = ldx;
        a.Ci = W.Ci;
        a.Lq = Lq;
        a.Lx = Lx;
        a.w = (const T*)W.w;
        a.wphase = W.wphase;
        a.Co = W.Co;
        a.ntaps = W.ntaps;
        a.stride = W.stride;
        a.nphase = W.nphase;
        for (int j = 0; j < 8; ++j) a.shift[j] = W.shift[j];
        a.bias = (const T*)W.bias;
        a.gamma = (const T*)gamma;
        a.res = (const T*)res;
        a.ldr = ldr;
        a.alpha2 = (const T*)alpha2;
        a.out = out;
        a.ldo = ldo;
        a.out2 = (T*)out2;
        a.ldo2 = ldo2;
        a.flags = flags | (W.bias ? CE_BIAS : 0) | (out2 ? CE_SNAKE : 0);
        a.lo = lo;
        launch_conv_gemm<T>(s, a);
        m->flops += 2.0 * Lq * W.nphase * (double)W.Co * W.ntaps * W.Ci;
        m->launches++;
    }

    // streamed chunk: a causal reader's carried rows -> the prefix of its input buffer, and back
    void site_in(bool on, const void* base, int width, int rows, void* st) {
        if (!on || rows <= 0) return;
        const size_t b = (size_t)rows * width * sizeof(T);
        HIPCHK(hipMemcpyAsync((char*)base - b, st, b, hipMemcpyDeviceToDevice, s));
    }
    void site_out(bool on, const void* base, int width, int rows, int L, void* st) {
        if (!on || rows <= 0) return;
        const size_t b = (size_t)rows * width * sizeof(T);
        HIPCHK(hipMemcpyAsync(st, (const char*)base + ((ptrdiff_t)L - rows) * width * (ptrdiff_t)sizeof(T), b,
                              hipMemcpyDeviceToDevice, s));
    }

    void decode(int Tn, bool stream = false) {
        const fm_codec_config& c = m->c;
        const int D = c.latent, H = c.t_heads, hd = c.t_head_dim, I = c.t_inter;
        const int W1 = c.window - 1, pos0 = stream ? m->spos : 0, npre = stream ? std::min(m->spos, W1) : 0;
        launch_rvq_decode<T>(s, m->d_codes, Tn, c.n_codebooks + 1, c.semantic_codebook_size, c.codebook_size,
                             c.codebook_dim, m->rvq, D, (T*)m->z);
        for (int l = 0; l < c.t_layers; ++l) {
            const TLayer& L = m->tl[l];
            launch_rmsnorm<T>(s, (const T*)m->z, D, (const T*)L.an, D, c.norm_eps, (T*)m->xn, D, Tn);
            gemm(L.wqkv, m->xn, D, Tn, Tn, m->qkv, 3 * H * hd, CE_STORE);
            launch_rope_qk<T>(s, (T*)m->qkv, Tn, H, hd, m->rope, pos0);
            site_in(stream, m->qkv, 3 * H * hd, W1, m->st_kv[l]);
            launch_window_attn<T>(s, (const T*)m->qkv, Tn, H, hd, c.window, (T*)m->att, npre);
            site_out(stream, m->qkv, 3 * H * hd, W1, Tn, m->st_kv[l]);
            gemm(L.wo, m->att, H * hd, Tn, Tn, m->z, D, CE_STORE | CE_RES | CE_GAMMA, m->z, D, L.ag);
            launch_rmsnorm<T>(s, (const T*)m->z, D, (const T*)L.fn, D, c.norm_eps, (T*)m->xn, D, Tn);
            gemm(L.w1, m->xn, D, Tn, Tn, m->g1, I, CE_STORE);
            gemm(L.w3, m->xn, D, Tn, Tn, m->g3, I, CE_STORE);
            launch_silu_mul<T>(s, (const T*)m->g1, (T*)m->g3, (size_t)Tn * I);
            gemm(L.w2, m->g3, I, Tn, Tn, m->z, D, CE_STORE | CE_RES | CE_GAMMA, m->z, D, L.fg);
        }
        launch_rmsnorm<T>(s, (const T*)m->z, D, (const T*)m->tnorm, D, c.norm_eps, (T*)m->xn, D, Tn);
        // upsample x2 x2: CausalTransConvNet(k2 s2) + ConvNeXt
        const void* xin = m->xn;
        int L = Tn;
        void* ubuf[2] = {m->u0, m->u1};
        for (int u = 0; u < 2; ++u) {
            void* uo = ubuf[u];
            gemm(m->up_ct[u], xin, D, L, L, uo, D, CE_STORE);
            L *= 2;
            site_in(stream, uo, D, 6, m->st_dw[u]);
            launch_dwconv_ln<T>(s, (const T*)uo, L, D, (const T*)m->up_dw[u], (const T*)m->up_db[u],
                                (const T*)m->up_lw[u], (const T*)m->up_lb[u], (T*)m->hh, stream ? -6 : 0);
            site_out(stream, uo, D, 6, L, m->st_dw[u]);
            gemm(m->up_pw1[u], m->hh, D, L, L, m->gb, 4 * D, CE_STORE | CE_GELU);
            gemm(m->up_pw2[u], m->gb, 4 * D, L, L, uo, D, CE_STORE | CE_RES | CE_GAMMA, uo, D, m->up_gm[u]);
            xin = uo;
        }
        // decoder
        const int ch = c.decoder_dim;
        site_in(stream, xin, D, 6, m->st_c0);
        gemm(m->conv0, xin, D, L, L, nullptr, 0, 0, nullptr, 0, nullptr, m->blk[0].alpha, m->A, ch, stream ? -6 : 0);
        site_out(stream, xin, D, 6, L, m->st_c0);
        void* in = m->A;
        void* alt = m->B;
        int cin = ch;
        const int rates[4] = {8, 8, 4, 2};
        for (int b = 0; b < 4; ++b) {
            const DBlock& Bk = m->blk[b];
            const int cout = cin / 2, st_ = rates[b];
            site_in(stream, in, cin, 1, m->st_ct[b]);
            gemm(Bk.ct, in, cin, L, L, m->xb, cout, CE_STORE, nullptr, 0, nullptr, Bk.ru[0].a0, alt, cout,
                 stream ? -1 : 0);
            site_out(stream, in, cin, 1, L, m->st_ct[b]);
            L *= st_;
            const int dl[3] = {1, 3, 9};
            for (int r = 0; r < 3; ++r) {
                const RU& R = Bk.ru[r];
                const int hr = 6 * dl[r];
                site_in(stream, alt, cout, hr, m->st_c7[b][r]);
                gemm(R.c7, alt, cout, L, L, nullptr, 0, 0, nullptr, 0, nullptr, R.a2, m->Cb, cout, stream ? -hr : 0);
                site_out(stream, alt, cout, hr, L, m->st_c7[b][r]);
                const void* an = r < 2 ? Bk.ru[r + 1].a0 : (b < 3 ? m->blk[b + 1].alpha : m->falpha);
                gemm(R.c1, m->Cb, cout, L, L, m->xb, cout, (r < 2 ? CE_STORE : 0) | CE_RES, m->xb, cout, nullptr,
                     an, alt, cout);
            }
            std::swap(in, alt);
            cin = cout;
        }
        site_in(stream, in, cin, 6, m->st_cf);
        gemm(m->convf, in, cin, L, L, m->wave, 1, CE_STORE | CE_TANH | CE_F32OUT, nullptr, 0, nullptr, nullptr,
             nullptr, 0, stream ? -6 : 0);
        site_out(stream, in, cin, 6, L, m->st_cf);
    }
};

extern "C" {

int fm_codec_open(const fm_codec_config* cfg, int device, int precision, int max_frames, fm_codec** out) {
    return fm_guard([&] {
        FMCHECK(cfg && out, "null argument");
        FMCHECK(precision == FM_PREC_BF16 || precision == FM_PREC_FP32, "bad precision");
        FMCHECK(max_frames >= 1 && max_frames <= (1 << 16), "bad max_frames");
        int ndev = fm_device_count();
        FMCHECK(ndev > 0, "no HIP device visible");
        FMCHECK(device >= 0 && device < ndev, "bad device index");
        HIPCHK(hipSetDevice(device));
        std::unique_ptr<fm_codec> m(new fm_codec());
        m->c = *cfg;
        m->device = device;
        m->prec = precision;
        m->esz = precision == FM_PREC_BF16 ? 2 : 4;
        m->max_frames = max_frames;
        HIPCHK(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
        build_inventory(m.get());
        *out = m.release();
    });
}

static DTensor& ctensor(fm_codec* m, const char* name, int64_t numel) {
    auto it = m->w.find(name);
    FMCHECK(it != m->w.end(), std::string("unknown codec tensor: ") + name);
    FMCHECK(it->second.numel == numel, std::string("wrong numel for ") + name);
    DTensor& t = it->second;
    if (!t.p) HIPCHK(hipMalloc(&t.p, (size_t)numel * 4));
    return t;
}

int fm_codec_set_tensor(fm_codec* m, const char* name, const void* data, int dtype, int64_t numel) {
    return fm_guard([&] {
        FMCHECK(m && name && data, "null argument");
        FMCHECK(!m->finalized, "weights are frozen after finalize");
        HIPCHK(hipSetDevice(m->device));
        DTensor& t = ctensor(m, name, numel);
        const size_t sb = dtype == FM_DT_BF16 ? 2 : 4;
        void* tmp = nullptr;
        HIPCHK(hipMalloc(&tmp, (size_t)numel * sb));
        HIPCHK(hipMemcpy(tmp, data, (size_t)numel * sb, hipMemcpyHostToDevice));
        launch_convert<float>(m->stream, tmp, dtype == FM_DT_BF16, numel, (float*)t.p);
        HIPCHK(hipStreamSynchronize(m->stream));
        HIPCHK(hipFree(tmp));
        t.set = true;
    });
}

int fm_codec_synth_tensor(fm_codec* m, const char* name, int64_t numel, uint64_t seed, float center, int log2_half) {
    return fm_guard([&] {
        FMCHECK(m && name, "null argument");
        FMCHECK(!m->finalized, "weights are frozen after finalize");
        HIPCHK(hipSetDevice(m->device));
        DTensor& t = ctensor(m, name, numel);
        launch_synth<float>(m->stream, (float*)t.p, numel, seed, fnv1a32(name), center, log2_half);
        HIPCHK(hipGetLastError());
        t.set = true;
    });
}

int fm_codec_finalize(fm_codec* m) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
    });
}

static void codec_decode(fm_codec* m, const int32_t* codes, int T, float* pcm, bool stream);

int fm_codec_decode(fm_codec* m, const int32_t* codes, int T, float* pcm) {
    return fm_guard([&] { codec_decode(m, codes, T, pcm, false); });
}

int fm_codec_stream_reset(fm_codec* m) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        for (auto& pb : m->st_all) HIPCHK(hipMemsetAsync(pb.first, 0, pb.second, m->stream));
        HIPCHK(hipStreamSynchronize(m->stream));
        m->spos = 0;
    });
}

int fm_codec_decode_chunk(fm_codec* m, const int32_t* codes, int T, float* pcm) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        FMCHECK(m->spos + (int64_t)T <= CODEC_STREAM_MAX, "stream longer than the RoPE table: reset it");
        codec_decode(m, codes, T, pcm, true);
        m->spos += T;
    });
}

static void codec_decode(fm_codec* m, const int32_t* codes, int T, float* pcm, bool stream) {
    {
        FMCHECK(m && codes && pcm, "null argument");
        FMCHECK(T >= 1 && T <= m->max_frames, "T must be in [1, max_frames]");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        const int nq1 = m->c.n_codebooks + 1;
        for (int i = 0; i < nq1 * T; ++i) FMCHECK(codes[i] >= 0, "negative code");
        HIPCHK(hipMemcpyAsync(m->d_codes, codes, (size_t)nq1 * T * 4, hipMemcpyHostToDevice, m->stream));
        m->flops = 0;
        HIPCHK(hipEventRecord(m->e0, m->stream));
        if (m->prec == FM_PREC_BF16) {
            CRun<bf16_t> r(m);
            r.decode(T, stream);
        } else {
            CRun<float> r(m);
            r.decode(T, stream);
        }
        HIPCHK(hipEventRecord(m->e1, m->stream));
        HIPCHK(hipMemcpyAsync(pcm, m->wave, (size_t)T * 2048 * 4, hipMemcpyDeviceToHost, m->stream));
        HIPCHK(hipStreamSynchronize(m->stream));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, m->e0, m->e1));
        m->last_ms = ms;
        m->total_ms += ms;
        m->total_flops += m->flops;
    }
}

// test hook: copy an intermediate of the last decode as fp32 (time-major):
// 1 = transformer output [T][D], 2 = upsample-1 [2T][D], 3 = decoder input latent [4T][D]
int fm_codec_debug_read(fm_codec* m, int stage, int T, float* out) {
    return fm_guard([&] {
        FMCHECK(m && out && m->finalized, "bad arguments");
        FMCHECK(stage >= 1 && stage <= 3, "debug stage must be 1..3");
        FMCHECK(T >= 1 && T <= m->max_frames, "bad T");
        const int D = m->c.latent;
        const void* src = stage == 1 ? m->xn : stage == 2 ? m->u0 : m->u1;
        const size_t n = (size_t)(stage == 1 ? 1 : stage == 2 ? 2 : 4) * T * D;
        std::vector<uint8_t> h(n * m->esz);
        HIPCHK(hipMemcpy(h.data(), src, h.size(), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; ++i) {
            if (m->esz == 2) {
                uint32_t u = ((uint32_t)((uint16_t*)h.data())[i]) << 16;
                memcpy(&out[i], &u, 4);
            } else {
                out[i] = ((float*)h.data())[i];
            }
        }
    });
}

int fm_codec_profile_read(fm_codec* m, double* total_ms, int64_t* launches, double* flops) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        if (total_ms) *total_ms = m->total_ms;
        if (launches) *launches = m->launches;
        if (flops) *flops = m->total_flops;
    });
}

int fm_codec_close(fm_codec* m) {
    return fm_guard([&] { delete m; });
}

}  // extern "C"

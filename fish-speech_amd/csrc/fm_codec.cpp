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
    int ks = 1;  // split-K factor (small-M layers; a property of the layer, so every chunking of a
                 // streamed decode sums in the same order as the one-shot decode)
};
// split-K factor of a layer that runs at a few hundred rows: K steps of 32 per slice >= 8, <= 8 slices
static void small_m(PackedW& W) {
    const int S = (W.ntaps * W.Ci + 31) / 32;
    int ks = 1;
    while (ks < 8 && S / (2 * ks) >= 8) ks *= 2;
    W.ks = W.Co % 8 == 0 ? ks : 1;
}

// [A rows | B rows] of two packed one-tap linears over the same input as one PackedW (the packed
// layout is 16-row tile-major, so it is the two buffers back to back)
static PackedW concat_rows(fm_codec* m, const PackedW& A, const PackedW& B);

struct TLayer {
    void *an, *fn, *ag, *fg;
    PackedW wqkv, wo, w1, w3, w2;
    PackedW w13;  // [W1 rows | W3 rows] as one GEMM (CE_SWIGLU split-K epilogue); w null: not built
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
struct EBlock {  // EncoderBlock (modded_dac.py:623-667): 3 residual units, snake, strided conv
    RU ru[3];
    void* a3;
    PackedW down;  // k = 2s, stride s, as a 2-tap conv over the [L/s][s*Ci] view
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
    std::map<const void*, const float*> ialpha;  // Snake alpha (device, T) -> its fp32 reciprocals
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
    void* zeros = nullptr;  // 256 zero bytes (resunit_kernel's DMA source outside the input rows)
    float* wave = nullptr;
    // stream state: carried rows per causal site (zeros at a stream start == causal padding)
    float* ksp = nullptr;                   // split-K workspace (conv_gemm_kernel slabs)
    size_t ksp_cap = 0;                     // floats
    void* st_kv[16] = {};                   // per transformer layer: window-1 qkv rows
    void *st_dw[2] = {}, *st_c0 = nullptr, *st_cf = nullptr;
    void *st_ct[4] = {}, *st_c7[4][3] = {};
    std::vector<std::pair<void*, size_t>> st_all;
    std::vector<void**> st_slots;           // the st_* field each st_all buffer is bound to
    int spos = 0;                           // frames already streamed (active stream)
    // stream contexts (fm_codec_stream_open): each holds its own carried rows + position, so
    // concurrent streamed requests on one handle never share state; id 0 is the handle's own
    struct StreamCtx {
        std::vector<void*> bufs;
        int spos = 0;
    };
    std::map<int, StreamCtx> sctx;
    int active_sid = 0, next_sid = 1;
    // encode side (fm_codec_enable_encoder / fm_codec_encode)
    int enc_dim = 0, enc_layers = 0;        // enc_dim 0: encoder not enabled
    EBlock eblk[4];
    PackedW e_c0, e_cf, ds[2], ds_pw1[2], ds_pw2[2];
    void *e_a5 = nullptr, *ds_dw[2] = {}, *ds_db[2] = {}, *ds_lw[2] = {}, *ds_lb[2] = {}, *ds_gm[2] = {};
    std::vector<TLayer> etl, ptl;
    void *etnorm = nullptr, *ptnorm = nullptr;
    VqEncPtrs vqe{};
    void *e_audio = nullptr, *e_x = nullptr, *e_alt = nullptr, *e_c = nullptr, *e_z = nullptr, *e_xn = nullptr;
    void *e_qkv = nullptr, *e_att = nullptr, *e_g1 = nullptr, *e_g3 = nullptr, *e_zenc = nullptr;
    void *e_u0 = nullptr, *e_u1 = nullptr, *e_zpre = nullptr;
    float* e_r = nullptr;
    float* e_pcm = nullptr;                 // mono input samples (fp32)
    int32_t* e_codes = nullptr;
    double last_ms = 0, flops = 0, total_ms = 0, total_flops = 0;
    int64_t launches = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;

    ~fm_codec() {
        if (device >= 0) (void)hipSetDevice(device);
        for (auto& kv : sctx)
            if (kv.first != 0)
                for (void* p : kv.second.bufs) (void)hipFree(p);
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
    void dstate(void** slot, size_t bytes) {
        void* p = dalloc(bytes);
        st_all.emplace_back(p, bytes);
        st_slots.push_back(slot);
        *slot = p;
    }
    // bind the st_* fields to stream `sid`'s buffers (the active stream's position saved first)
    void activate(int sid) {
        if (sid == active_sid) return;
        auto it = sctx.find(sid);
        FMCHECK(it != sctx.end(), "unknown codec stream id " + std::to_string(sid));
        sctx[active_sid].spos = spos;
        for (size_t i = 0; i < st_slots.size(); ++i) *st_slots[i] = it->second.bufs[i];
        spos = it->second.spos;
        active_sid = sid;
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

// encode-side keys (mirrors fishmi/checkpoint.codec_encoder_tensor_shapes)
static const int ENC_RATES[4] = {2, 4, 8, 8};
static const int ENC_DILS[3] = {1, 3, 9};  // the three ResidualUnits of an EncoderBlock
static constexpr int ENC_WINDOW = 512;  // EncoderBlock transformer: getattr(partial, "window_size", 512)
static void add_tlayers(fm_codec* m, const std::string& pre, int dim, int layers, int HD, int I) {
    for (int l = 0; l < layers; ++l) {
        std::string p = pre + "layers." + std::to_string(l) + ".";
        add(m, p + "attention.wqkv.weight", (int64_t)3 * HD * dim);
        add(m, p + "attention.wo.weight", (int64_t)dim * HD);
        add(m, p + "feed_forward.w1.weight", (int64_t)I * dim);
        add(m, p + "feed_forward.w3.weight", (int64_t)I * dim);
        add(m, p + "feed_forward.w2.weight", (int64_t)dim * I);
        add(m, p + "ffn_norm.weight", dim);
        add(m, p + "attention_norm.weight", dim);
        add(m, p + "attention_layer_scale.gamma", dim);
        add(m, p + "ffn_layer_scale.gamma", dim);
    }
    if (layers) add(m, pre + "norm.weight", dim);
}
static void build_encoder_inventory(fm_codec* m) {
    const fm_codec_config& c = m->c;
    const int D = c.latent, cd = c.codebook_dim;
    auto wn = [&](const std::string& p, int co, int ci, int k) {
        add(m, p + "conv.parametrizations.weight.original0", co);
        add(m, p + "conv.parametrizations.weight.original1", (int64_t)co * ci * k);
        add(m, p + "conv.bias", co);
    };
    wn("encoder.block.0.", m->enc_dim, 1, 7);
    int d = m->enc_dim;
    for (int b = 0; b < 4; ++b) {
        const int h = d;
        d *= 2;
        std::string p = "encoder.block." + std::to_string(b + 1) + ".block.";
        for (int r = 0; r < 3; ++r) {
            std::string rp = p + std::to_string(r) + ".block.";
            add(m, rp + "0.alpha", h);
            wn(rp + "1.", h, h, 7);
            add(m, rp + "2.alpha", h);
            wn(rp + "3.", h, h, 1);
        }
        add(m, p + "3.alpha", h);
        wn(p + "4.", d, h, 2 * ENC_RATES[b]);
        if (b == 3) add_tlayers(m, p + "5.", d, m->enc_layers, d, 3 * d);
    }
    add(m, "encoder.block.5.alpha", d);
    wn("encoder.block.6.", D, d, 3);
    for (int i = 0; i < 2; ++i) {
        std::string p = "quantizer.downsample." + std::to_string(i) + ".";
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
    add_tlayers(m, "quantizer.pre_module.", D, c.t_layers, c.t_heads * c.t_head_dim, c.t_inter);
    for (int q = 0; q <= c.n_codebooks; ++q) {
        std::string p = q == 0 ? "quantizer.semantic_quantizer.quantizers.0."
                               : "quantizer.quantizer.quantizers." + std::to_string(q - 1) + ".";
        add(m, p + "in_proj.weight_g", cd);
        add(m, p + "in_proj.weight_v", (int64_t)cd * D);
        add(m, p + "in_proj.bias", cd);
    }
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

// a Snake alpha vector as T plus its fp32 reciprocals 1 / (alpha + 1e-9) (descript Snake1d, restated
// in oracle/ref_stubs.py), computed once from the T-rounded values so every epilogue multiplies
// by the same fp32 number the per-element division gave
static void* as_snake(fm_codec* m, const float* src, int64_t n) {
    void* d = as_T(m, src, n);
    float* ia = (float*)m->dalloc((size_t)n * sizeof(float));
    if (m->prec == FM_PREC_BF16)
        launch_snake_inv<bf16_t>(m->stream, (const bf16_t*)d, n, ia);
    else
        launch_snake_inv<float>(m->stream, (const float*)d, n, ia);
    m->ialpha[d] = ia;
    return d;
}

// prepare a GEMM weight: kind per conv_weight_kernel; returns phases packed
static PackedW concat_rows(fm_codec* m, const PackedW& A, const PackedW& B) {
    FMCHECK(A.Ci == B.Ci && A.ntaps == 1 && B.ntaps == 1 && A.nphase == 1 && B.nphase == 1 && A.Co % 16 == 0 &&
                A.Co == B.Co && !A.bias && !B.bias && A.ks == B.ks && A.wphase == B.wphase,
            "codec: W1 / W3 concatenation needs two bias-free one-tap linears of one shape");
    PackedW p = A;
    p.Co = A.Co + B.Co;
    p.wphase = A.wphase + B.wphase;
    p.w = m->dalloc(p.wphase * m->esz);
    HIPCHK(hipMemcpyAsync(p.w, A.w, A.wphase * m->esz, hipMemcpyDeviceToDevice, m->stream));
    HIPCHK(hipMemcpyAsync((char*)p.w + A.wphase * m->esz, B.w, B.wphase * m->esz, hipMemcpyDeviceToDevice, m->stream));
    HIPCHK(hipStreamSynchronize(m->stream));
    return p;
}

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

// conv weight rearranged on the host (fp32 [Co][Ci'][k']) then prepared as kind 0
static PackedW prep_host(fm_codec* m, const std::vector<float>& w, int Ci, int Co, int k, const float* bias) {
    float* d = nullptr;
    HIPCHK(hipMalloc(&d, w.size() * 4));
    HIPCHK(hipMemcpy(d, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    PackedW p = prep(m, d, 0, Ci, Co, k, 1, 1, bias);  // prep synchronises before returning
    HIPCHK(hipFree(d));
    return p;
}
static std::vector<float> to_host(fm_codec* m, const float* d, size_t n) {
    std::vector<float> h(n);
    HIPCHK(hipStreamSynchronize(m->stream));
    HIPCHK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
    return h;
}
// causal conv k = 2s, stride s (CausalConvNet, modded_dac.py:59-90; left pad k - s, no right pad
// when L % s == 0): out[t] = sum_j W[j] x[ts + j - s] = tap0 . x'[t-1] + tap1 . x'[t] over the
// contiguous view x'[L/s][s*Ci] of a time-major x, with x'[t][jj*Ci + ci] = x[ts + jj][ci]
static PackedW prep_strided(fm_codec* m, const float* wdev, int Ci, int Co, int s, const float* bias) {
    const std::vector<float> w = to_host(m, wdev, (size_t)Co * Ci * 2 * s);
    std::vector<float> o((size_t)Co * s * Ci * 2);
    for (int co = 0; co < Co; ++co)
        for (int ci = 0; ci < Ci; ++ci)
            for (int jj = 0; jj < s; ++jj)
                for (int tap = 0; tap < 2; ++tap)
                    o[(((size_t)co * s + jj) * Ci + ci) * 2 + tap] = w[((size_t)co * Ci + ci) * 2 * s + tap * s + jj];
    return prep_host(m, o, s * Ci, Co, 2, bias);
}
static void prep_tlayers(fm_codec* m, std::vector<TLayer>& tl, const std::string& pre, int dim, int layers, int HD,
                         int I) {
    tl.resize(layers);
    for (int l = 0; l < layers; ++l) {
        std::string p = pre + "layers." + std::to_string(l) + ".";
        TLayer& L = tl[l];
        L.an = as_T(m, raw(m, p + "attention_norm.weight"), dim);
        L.fn = as_T(m, raw(m, p + "ffn_norm.weight"), dim);
        L.ag = as_T(m, raw(m, p + "attention_layer_scale.gamma"), dim);
        L.fg = as_T(m, raw(m, p + "ffn_layer_scale.gamma"), dim);
        L.wqkv = prep(m, raw(m, p + "attention.wqkv.weight"), 3, dim, 3 * HD, 1, 1, 1, nullptr);
        L.wo = prep(m, raw(m, p + "attention.wo.weight"), 3, HD, dim, 1, 1, 1, nullptr);
        L.w1 = prep(m, raw(m, p + "feed_forward.w1.weight"), 3, dim, I, 1, 1, 1, nullptr);
        L.w3 = prep(m, raw(m, p + "feed_forward.w3.weight"), 3, dim, I, 1, 1, 1, nullptr);
        L.w2 = prep(m, raw(m, p + "feed_forward.w2.weight"), 3, I, dim, 1, 1, 1, nullptr);
    }
}

static void finalize_encoder(fm_codec* m) {
    const fm_codec_config& c = m->c;
    const int D = c.latent, cd = c.codebook_dim;
    FMCHECK(m->enc_dim % 8 == 0, "encoder_dim must be a multiple of 8");
    FMCHECK(c.codebook_dim <= 16 && c.n_codebooks + 1 <= 16, "vq encode: codebook_dim <= 16, <= 16 stages");
    {  // first conv: 1 input channel padded to 8 (the audio buffer is [L][8], channel 0 live)
        const int e = m->enc_dim;
        const float* w = fold(m, "encoder.block.0.conv.parametrizations.weight.original0",
                              "encoder.block.0.conv.parametrizations.weight.original1", e, 7);
        const std::vector<float> h = to_host(m, w, (size_t)e * 7);
        std::vector<float> o((size_t)e * 8 * 7, 0.f);
        for (int co = 0; co < e; ++co)
            for (int j = 0; j < 7; ++j) o[((size_t)co * 8) * 7 + j] = h[(size_t)co * 7 + j];
        m->e_c0 = prep_host(m, o, 8, e, 7, raw(m, "encoder.block.0.conv.bias"));
    }
    int d = m->enc_dim;
    for (int b = 0; b < 4; ++b) {
        const int h = d, st = ENC_RATES[b];
        d *= 2;
        std::string p = "encoder.block." + std::to_string(b + 1) + ".block.";
        EBlock& B = m->eblk[b];
        const int dils[3] = {1, 3, 9};
        for (int r = 0; r < 3; ++r) {
            std::string rp = p + std::to_string(r) + ".block.";
            B.ru[r].a0 = as_snake(m, raw(m, rp + "0.alpha"), h);
            B.ru[r].a2 = as_snake(m, raw(m, rp + "2.alpha"), h);
            B.ru[r].c7 = prep_wn_conv(m, rp + "1.", h, h, 7, dils[r]);
            B.ru[r].c1 = prep_wn_conv(m, rp + "3.", h, h, 1, 1);
        }
        B.a3 = as_snake(m, raw(m, p + "3.alpha"), h);
        const float* w = fold(m, p + "4.conv.parametrizations.weight.original0",
                              p + "4.conv.parametrizations.weight.original1", d, h * 2 * st);
        B.down = prep_strided(m, w, h, d, st, raw(m, p + "4.conv.bias"));
        if (b == 3 && m->enc_layers) {
            FMCHECK(d % 64 == 0, "encoder transformer: dim must be a multiple of 64");
            prep_tlayers(m, m->etl, p + "5.", d, m->enc_layers, d, 3 * d);
            m->etnorm = as_T(m, raw(m, p + "5.norm.weight"), d);
        }
    }
    m->e_a5 = as_snake(m, raw(m, "encoder.block.5.alpha"), d);
    m->e_cf = prep_wn_conv(m, "encoder.block.6.", d, D, 3, 1);
    for (int i = 0; i < 2; ++i) {
        std::string p = "quantizer.downsample." + std::to_string(i) + ".";
        // CausalConvNet(k=2, s=2): no padding, out[t] = W0 x[2t] + W1 x[2t+1] = one tap over [L/2][2D]
        const std::vector<float> w = to_host(m, raw(m, p + "0.conv.weight"), (size_t)D * D * 2);
        std::vector<float> o((size_t)D * 2 * D);
        for (int co = 0; co < D; ++co)
            for (int ci = 0; ci < D; ++ci)
                for (int j = 0; j < 2; ++j) o[((size_t)co * 2 + j) * D + ci] = w[((size_t)co * D + ci) * 2 + j];
        m->ds[i] = prep_host(m, o, 2 * D, D, 1, raw(m, p + "0.conv.bias"));
        m->ds_dw[i] = as_T(m, raw(m, p + "1.dwconv.conv.weight"), (int64_t)D * 7);
        m->ds_db[i] = as_T(m, raw(m, p + "1.dwconv.conv.bias"), D);
        m->ds_lw[i] = as_T(m, raw(m, p + "1.norm.weight"), D);
        m->ds_lb[i] = as_T(m, raw(m, p + "1.norm.bias"), D);
        m->ds_pw1[i] = prep(m, raw(m, p + "1.pwconv1.weight"), 3, D, 4 * D, 1, 1, 1, raw(m, p + "1.pwconv1.bias"));
        m->ds_pw2[i] = prep(m, raw(m, p + "1.pwconv2.weight"), 3, 4 * D, D, 1, 1, 1, raw(m, p + "1.pwconv2.bias"));
        m->ds_gm[i] = as_T(m, raw(m, p + "1.gamma"), D);
    }
    const int HD = c.t_heads * c.t_head_dim;
    prep_tlayers(m, m->ptl, "quantizer.pre_module.", D, c.t_layers, HD, c.t_inter);
    m->ptnorm = as_T(m, raw(m, "quantizer.pre_module.norm.weight"), D);
    for (int q = 0; q <= c.n_codebooks; ++q) {
        std::string p = q == 0 ? "quantizer.semantic_quantizer.quantizers.0."
                               : "quantizer.quantizer.quantizers." + std::to_string(q - 1) + ".";
        m->vqe.wi[q] = fold(m, p + "in_proj.weight_g", p + "in_proj.weight_v", cd, D);
        m->vqe.bi[q] = raw(m, p + "in_proj.bias");
        m->vqe.cb[q] = raw(m, p + "codebook.weight");
        m->vqe.wo[q] = m->rvq.w[q];
        m->vqe.bo[q] = raw(m, p + "out_proj.bias");
        m->vqe.cbn[q] = q == 0 ? c.semantic_codebook_size : c.codebook_size;
    }
    // buffers for max_frames code frames (L0 = 2048 T samples); every encoder stage holds
    // L * channels <= L0 * enc_dim elements
    const size_t Tm = m->max_frames, E = m->esz, L0 = 2048 * Tm, dF = (size_t)m->enc_dim * 16;
    m->e_pcm = (float*)m->dalloc(L0 * 4);
    m->e_audio = m->dalloc(L0 * 8 * E);
    m->e_x = m->dalloc(L0 * m->enc_dim * E);
    m->e_alt = m->dalloc(L0 * m->enc_dim * E);
    m->e_c = m->dalloc(L0 * m->enc_dim * E);
    const size_t R4 = 4 * Tm, wmax = std::max(dF, (size_t)D);
    const size_t imax = std::max(std::max(3 * dF, (size_t)c.t_inter), (size_t)4 * D);
    m->e_z = m->dalloc(R4 * wmax * E);
    m->e_xn = m->dalloc(R4 * wmax * E);
    m->e_qkv = m->dalloc(R4 * 3 * wmax * E);
    m->e_att = m->dalloc(R4 * wmax * E);
    m->e_g1 = m->dalloc(R4 * imax * E);
    m->e_g3 = m->dalloc(R4 * imax * E);
    m->e_zenc = m->dalloc(R4 * D * E);
    m->e_u0 = m->dalloc(2 * Tm * D * E);
    m->e_u1 = m->dalloc(Tm * D * E);
    m->e_zpre = m->dalloc(Tm * D * E);
    m->e_r = (float*)m->dalloc(Tm * D * 4);
    m->e_codes = (int32_t*)m->dalloc((size_t)(c.n_codebooks + 1) * Tm * 4);
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
        for (PackedW* W : {&L.wqkv, &L.wo, &L.w1, &L.w3, &L.w2}) small_m(*W);
        L.w13 = concat_rows(m, L.w1, L.w3);
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
        for (PackedW* W : {&m->up_ct[u], &m->up_pw1[u], &m->up_pw2[u]}) small_m(*W);
    }
    const int ch = c.decoder_dim;
    m->conv0 = prep_wn_conv(m, "decoder.model.0.", D, ch, 7, 1);
    small_m(m->conv0);
    int cin = ch;
    const int rates[4] = {8, 8, 4, 2};
    for (int b = 0; b < 4; ++b) {
        const int cout = cin / 2, s = rates[b];
        std::string p = "decoder.model." + std::to_string(b + 1) + ".block.";
        DBlock& B = m->blk[b];
        B.alpha = as_snake(m, raw(m, p + "0.alpha"), cin);
        // ConvTranspose1d weight norm: dim 0 is the INPUT channel (norm over (out, k))
        const float* wt = fold(m, p + "1.conv.parametrizations.weight.original0",
                               p + "1.conv.parametrizations.weight.original1", cin, cout * 2 * s);
        B.ct = prep(m, wt, 1, cin, cout, 2 * s, s, 1, raw(m, p + "1.conv.bias"));
        const int dils[3] = {1, 3, 9};
        for (int r = 0; r < 3; ++r) {
            std::string rp = p + std::to_string(r + 2) + ".block.";
            B.ru[r].a0 = as_snake(m, raw(m, rp + "0.alpha"), cout);
            B.ru[r].a2 = as_snake(m, raw(m, rp + "2.alpha"), cout);
            B.ru[r].c7 = prep_wn_conv(m, rp + "1.", cout, cout, 7, dils[r]);
            B.ru[r].c1 = prep_wn_conv(m, rp + "3.", cout, cout, 1, 1);
        }
        if (b == 0) {
            // the first stage runs on ~32 x T rows at 768 channels (1.3 LDS tiles per CU): its
            // transposed conv and k7 convs split K in two (a fixed property of the layer, so every
            // chunking of a streamed decode sums in the same order)
            B.ct.ks = 2;
            for (int r = 0; r < 3; ++r) B.ru[r].c7.ks = 2;
        }
        cin = cout;
    }
    m->falpha = as_snake(m, raw(m, "decoder.model.5.alpha"), cin);
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
    for (int l = 0; l < c.t_layers; ++l) m->dstate(&m->st_kv[l], (size_t)(c.window - 1) * 3 * HD * E);
    for (int u = 0; u < 2; ++u) m->dstate(&m->st_dw[u], (size_t)6 * D * E);
    m->dstate(&m->st_c0, (size_t)6 * D * E);
    {
        int cc = ch;
        const int dl[3] = {1, 3, 9};
        for (int b = 0; b < 4; ++b) {
            m->dstate(&m->st_ct[b], (size_t)cc * E);
            for (int r = 0; r < 3; ++r) m->dstate(&m->st_c7[b][r], (size_t)6 * dl[r] * (cc / 2) * E);
            cc /= 2;
        }
        m->dstate(&m->st_cf, (size_t)6 * cc * E);
    }
    {
        auto& c0 = m->sctx[0];
        for (auto& pb : m->st_all) c0.bufs.push_back(pb.first);
    }
    // the k7 output of the two-launch ResidualUnit, or (prefixed: it is a k7 input then) the third
    // buffer the fused units ping-pong with
    m->Cb = m->dalloc_prefixed(Tm * maxact * E, (size_t)CODEC_HALO * std::max(ch, D) * E);
    m->zeros = m->dalloc(256);
    HIPCHK(hipMemset(m->zeros, 0, 256));
    resunit_init();
    m->ksp_cap = (size_t)16 << 20;  // split-K partial slabs of the small-grid codec GEMMs (64 MB)
    m->ksp = (float*)m->dalloc(m->ksp_cap * 4);
    m->wave = (float*)m->dalloc(Tm * 2048 * 4);
    if (m->enc_dim) finalize_encoder(m);
    HIPCHK(hipEventCreate(&m->e0));
    HIPCHK(hipEventCreate(&m->e1));
    HIPCHK(hipStreamSynchronize(m->stream));
    m->finalized = true;
}

template <typename T> struct CRun {
    fm_codec* m;
    hipStream_t s;
    explicit CRun(fm_codec* mm) : m(mm), s(mm->stream) {}
    int rope_pos0_ = 0, rope_nqk_ = 0, rope_hd_ = 0;  // CE_ROPE operands of the next gemm()
    const void* norm_w_ = nullptr;                     // CE_NORM: the norm weight of the next gemm()

    // out = res + gamma * (W x) (the transformer's residual linears), then xn = RMSNorm(out, nw) --
    // in the split-K epilogue when the layer splits K (fm_tune codec_norm), else a rmsnorm launch
    void res_linear_norm(const PackedW& W, const void* x, int ldx, int Tn, void* z, int D, const void* gamma,
                         const void* nw, void* xn) {
        if (fm_tuning().codec_norm && fm_tuning().conv_splitk && W.ks > 1 && W.Co == D && D % 512 == 0 &&
            D <= 2048 && W.nphase == 1) {
            norm_w_ = nw;
            gemm(W, x, ldx, Tn, Tn, z, D, CE_STORE | CE_RES | CE_GAMMA | CE_NORM, z, D, gamma, nullptr, xn, D);
            return;
        }
        gemm(W, x, ldx, Tn, Tn, z, D, CE_STORE | CE_RES | CE_GAMMA, z, D, gamma);
        launch_rmsnorm<T>(s, (const T*)z, D, (const T*)nw, D, m->c.norm_eps, (T*)xn, D, Tn);
    }

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
        if (alpha2) {
            auto it = m->ialpha.find(alpha2);
            FMCHECK(it != m->ialpha.end(), "codec: Snake alpha without reciprocals");
            a.ialpha2 = it->second;
        }
        a.out = out;
        a.ldo = ldo;
        a.out2 = (T*)out2;
        a.ldo2 = ldo2;
        a.flags = flags | (W.bias ? CE_BIAS : 0) | ((out2 && !(flags & CE_NORM)) ? CE_SNAKE : 0);
        if (flags & CE_NORM) {
            a.normw = (const T*)norm_w_;
            a.norm_eps = m->c.norm_eps;
        }
        a.lo = lo;
        a.slab = m->ksp;
        a.slab_cap = m->ksp_cap;
        a.ksplit = fm_tuning().conv_splitk ? W.ks : 1;
        if (flags & CE_ROPE) {
            a.rope = m->rope;
            a.rope_pos0 = rope_pos0_;
            a.rope_nqk = rope_nqk_;
            a.rope_hd = rope_hd_;
        }
        launch_conv_gemm<T>(s, a);
        m->flops += 2.0 * Lq * W.nphase * (double)W.Co * W.ntaps * W.Ci;
        m->launches++;
    }

    // one decoder ResidualUnit (modded_dac.py:599-620) as resunit_kernel (bf16, 96 / 192 / 384 channels):
    // x = snake_a0 of the unit input in `x`, the residual in `res`, snake_an of the output -> out2.
    // false: not covered (fp32, other widths, fm_tune codec_fuse 0) -- the caller runs the two GEMMs
    bool resunit(const RU& R, int dil, const void* x, int L, int lo, bool store_res, const void* an, void* out2,
                 int C, void* res) {
        if constexpr (sizeof(T) != 2) {
            return false;
        } else {
            if (!R.c7.bias || !R.c1.bias || R.c7.ntaps != 7 || R.c7.Ci != C || R.c7.Co != C || R.c1.Ci != C ||
                R.c1.Co != C || R.c7.ks != 1)
                return false;
            auto ia = [&](const void* al) {
                auto it = m->ialpha.find(al);
                FMCHECK(it != m->ialpha.end(), "codec: Snake alpha without reciprocals");
                return (const float*)it->second;
            };
            ResUnitArgs a{};
            a.x = (const bf16_t*)x;
            a.L = L;
            a.lo = lo;
            a.dil = dil;
            a.w7 = (const bf16_t*)R.c7.w;
            a.b7 = (const bf16_t*)R.c7.bias;
            a.a2 = (const bf16_t*)R.a2;
            a.ia2 = ia(R.a2);
            a.w1 = (const bf16_t*)R.c1.w;
            a.b1 = (const bf16_t*)R.c1.bias;
            a.res = (bf16_t*)res;
            a.store_res = store_res;
            a.an = (const bf16_t*)an;
            a.ian = ia(an);
            a.out2 = (bf16_t*)out2;
            a.zeros = (const bf16_t*)m->zeros;
            if (!launch_resunit(s, a, C)) return false;
            m->flops += 2.0 * L * (double)C * 8 * C;  // k7 (K = 7 C) + k1 (K = C)
            m->launches++;
            return true;
        }
    }

    // FeedForward's silu(w1 x) * w3 x (modded_dac.py:316-317) into g3: one GEMM over [W1 | W3] with
    // the SwiGLU split-K epilogue when the layer splits K (bit-identical), else w1, w3, silu_mul
    void ffn13(const TLayer& L, const void* xn, int Dm, int Tn, int I, void* g1, void* g3) {
        const FmTuning& tu = fm_tuning();
        if (L.w13.w && tu.codec_swiglu && tu.conv_splitk && L.w13.ks > 1) {
            gemm(L.w13, xn, Dm, Tn, Tn, g3, I, CE_STORE | CE_SWIGLU);
            return;
        }
        gemm(L.w1, xn, Dm, Tn, Tn, g1, I, CE_STORE);
        gemm(L.w3, xn, Dm, Tn, Tn, g3, I, CE_STORE);
        launch_silu_mul<T>(s, (const T*)g1, (T*)g3, (size_t)Tn * I);
    }

    // WindowLimitedTransformer.forward (modded_dac.py:418-439) on z [Tn][Dm] in place; the final
    // norm goes to xn
    void transformer(const std::vector<TLayer>& tl, const void* norm, int Tn, int Dm, int H, int hd, int I,
                     int window, void* z, void* xn, void* qkv, void* att, void* g1, void* g3) {
        const float eps = m->c.norm_eps;
        for (const TLayer& L : tl) {
            launch_rmsnorm<T>(s, (const T*)z, Dm, (const T*)L.an, Dm, eps, (T*)xn, Dm, Tn);
            gemm(L.wqkv, xn, Dm, Tn, Tn, qkv, 3 * H * hd, CE_STORE);
            launch_rope_qk<T>(s, (T*)qkv, Tn, H, hd, m->rope, 0);
            launch_window_attn<T>(s, (const T*)qkv, Tn, H, hd, window, (T*)att, 0);
            gemm(L.wo, att, H * hd, Tn, Tn, z, Dm, CE_STORE | CE_RES | CE_GAMMA, z, Dm, L.ag);
            launch_rmsnorm<T>(s, (const T*)z, Dm, (const T*)L.fn, Dm, eps, (T*)xn, Dm, Tn);
            ffn13(L, xn, Dm, Tn, I, g1, g3);
            gemm(L.w2, g3, I, Tn, Tn, z, Dm, CE_STORE | CE_RES | CE_GAMMA, z, Dm, L.fg);
        }
        launch_rmsnorm<T>(s, (const T*)z, Dm, (const T*)norm, Dm, eps, (T*)xn, Dm, Tn);
    }

    // ConvNeXtBlock (rvq.py:129-191) of quantizer.downsample.<i> on u [L][D] in place
    void ds_convnext(int i, void* u, int L) {
        const int D = m->c.latent;
        launch_dwconv_ln<T>(s, (const T*)u, L, D, (const T*)m->ds_dw[i], (const T*)m->ds_db[i],
                            (const T*)m->ds_lw[i], (const T*)m->ds_lb[i], (T*)m->e_xn, 0);
        gemm(m->ds_pw1[i], m->e_xn, D, L, L, m->e_g1, 4 * D, CE_STORE | CE_GELU);
        gemm(m->ds_pw2[i], m->e_g1, 4 * D, L, L, u, D, CE_STORE | CE_RES | CE_GAMMA, u, D, m->ds_gm[i]);
    }

    // DAC.encode (modded_dac.py:874-923) on e_audio [2048 Tn][8]: Encoder (modded_dac.py:670-709)
    // -> quantizer.downsample (rvq.py:250-262) -> pre_module -> semantic + residual VQ
    // (rvq.py:303-315) -> e_codes [(nq+1)][Tn]
    void encode(int Tn) {
        const fm_codec_config& c = m->c;
        const int D = c.latent;
        int L = 2048 * Tn, h = m->enc_dim;
        void* alt = m->e_alt;
        void* spare = m->e_c;
        gemm(m->e_c0, m->e_audio, 8, L, L, m->e_x, h, CE_STORE, nullptr, 0, nullptr, m->eblk[0].ru[0].a0, alt, h);
        const void* fin_in = nullptr;  // snake(encoder.block.5) of the last encoder block's output
        for (int b = 0; b < 4; ++b) {
            const EBlock& B = m->eblk[b];
            const int st = ENC_RATES[b], d = 2 * h;
            for (int r = 0; r < 3; ++r) {  // ResidualUnit (modded_dac.py:600-620)
                const RU& R = B.ru[r];
                const void* an = r < 2 ? B.ru[r + 1].a0 : B.a3;
                if (resunit(R, ENC_DILS[r], alt, L, 0, r < 2, an, spare, h, m->e_x)) {
                    std::swap(alt, spare);  // (the unit's output Snake is in `spare` now)
                    continue;
                }
                gemm(R.c7, alt, h, L, L, nullptr, 0, 0, nullptr, 0, nullptr, R.a2, spare, h);
                gemm(R.c1, spare, h, L, L, m->e_x, h, (r < 2 ? CE_STORE : 0) | CE_RES, m->e_x, h, nullptr, an, alt, h);
            }
            const int Lo = L / st;
            if (b < 3) {
                gemm(B.down, alt, st * h, Lo, Lo, m->e_x, d, CE_STORE, nullptr, 0, nullptr, m->eblk[b + 1].ru[0].a0,
                     spare, d);
                std::swap(alt, spare);
            } else if (m->enc_layers) {
                gemm(B.down, alt, st * h, Lo, Lo, m->e_z, d, CE_STORE);
                transformer(m->etl, m->etnorm, Lo, d, d / 64, 64, 3 * d, ENC_WINDOW, m->e_z, m->e_xn, m->e_qkv,
                            m->e_att, m->e_g1, m->e_g3);
                launch_snake<T>(s, (const T*)m->e_xn, d, (size_t)Lo * d, (const T*)m->e_a5, (T*)spare);
                fin_in = spare;
            } else {
                gemm(B.down, alt, st * h, Lo, Lo, nullptr, 0, 0, nullptr, 0, nullptr, m->e_a5, spare, d);
                fin_in = spare;
            }
            L = Lo;
            h = d;
        }
        gemm(m->e_cf, fin_in, h, L, L, m->e_zenc, D, CE_STORE);  // z_enc [4 Tn][D]
        // quantizer.downsample: CausalConvNet(k2 s2) as one tap over the [L/2][2D] view + ConvNeXt
        gemm(m->ds[0], m->e_zenc, 2 * D, L / 2, L / 2, m->e_u0, D, CE_STORE);
        ds_convnext(0, m->e_u0, L / 2);
        gemm(m->ds[1], m->e_u0, 2 * D, L / 4, L / 4, m->e_u1, D, CE_STORE);
        ds_convnext(1, m->e_u1, L / 4);
        transformer(m->ptl, m->ptnorm, Tn, D, c.t_heads, c.t_head_dim, c.t_inter, c.window, m->e_u1, m->e_zpre,
                    m->e_qkv, m->e_att, m->e_g1, m->e_g3);
        launch_convert<float>(s, m->e_zpre, sizeof(T) == 2, (int64_t)Tn * D, m->e_r);
        launch_vq_encode(s, m->e_r, Tn, D, c.n_codebooks + 1, c.codebook_dim, m->vqe, m->e_codes);
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
        // each layer's two norms come out of the residual linears before them (res_linear_norm);
        // only the first attention_norm runs on its own
        if (c.t_layers > 0)
            launch_rmsnorm<T>(s, (const T*)m->z, D, (const T*)m->tl[0].an, D, c.norm_eps, (T*)m->xn, D, Tn);
        for (int l = 0; l < c.t_layers; ++l) {
            const TLayer& L = m->tl[l];
            if (fm_tuning().codec_rope && fm_tuning().conv_splitk && L.wqkv.ks > 1 && hd % 8 == 0) {
                // RoPE in the projection's split-K epilogue (rope_qk_kernel's arithmetic)
                rope_pos0_ = pos0;
                rope_nqk_ = 2 * H * hd;
                rope_hd_ = hd;
                gemm(L.wqkv, m->xn, D, Tn, Tn, m->qkv, 3 * H * hd, CE_STORE | CE_ROPE);
            } else {
                gemm(L.wqkv, m->xn, D, Tn, Tn, m->qkv, 3 * H * hd, CE_STORE);
                launch_rope_qk<T>(s, (T*)m->qkv, Tn, H, hd, m->rope, pos0);
            }
            site_in(stream, m->qkv, 3 * H * hd, W1, m->st_kv[l]);
            launch_window_attn<T>(s, (const T*)m->qkv, Tn, H, hd, c.window, (T*)m->att, npre);
            site_out(stream, m->qkv, 3 * H * hd, W1, Tn, m->st_kv[l]);
            res_linear_norm(L.wo, m->att, H * hd, Tn, m->z, D, L.ag, L.fn, m->xn);
            ffn13(L, m->xn, D, Tn, I, m->g1, m->g3);
            res_linear_norm(L.w2, m->g3, I, Tn, m->z, D, L.fg, l + 1 < c.t_layers ? m->tl[l + 1].an : m->tnorm,
                            m->xn);
        }
        if (c.t_layers == 0)
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
        void* spare = m->Cb;  // fused units: alt -> spare, then the two swap
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
                const void* an = r < 2 ? Bk.ru[r + 1].a0 : (b < 3 ? m->blk[b + 1].alpha : m->falpha);
                site_in(stream, alt, cout, hr, m->st_c7[b][r]);
                if (resunit(R, dl[r], alt, L, stream ? -hr : 0, r < 2, an, spare, cout, m->xb)) {
                    site_out(stream, alt, cout, hr, L, m->st_c7[b][r]);
                    std::swap(alt, spare);
                    continue;
                }
                // two launches: the k7 output goes to `spare` (never alt: after fused units swapped
                // the pair, alt may be m->Cb itself)
                FMCHECK(spare != alt && spare != in, "codec: ResidualUnit scratch aliases its input");
                gemm(R.c7, alt, cout, L, L, nullptr, 0, 0, nullptr, 0, nullptr, R.a2, spare, cout, stream ? -hr : 0);
                site_out(stream, alt, cout, hr, L, m->st_c7[b][r]);
                gemm(R.c1, spare, cout, L, L, m->xb, cout, (r < 2 ? CE_STORE : 0) | CE_RES, m->xb, cout, nullptr,
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

int fm_codec_enable_encoder(fm_codec* m, int encoder_dim, int enc_layers) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        FMCHECK(!m->finalized, "enable the encoder before finalize");
        FMCHECK(!m->enc_dim, "encoder already enabled");
        FMCHECK(encoder_dim >= 8 && encoder_dim % 8 == 0 && enc_layers >= 0 && enc_layers <= 16, "bad encoder shape");
        m->enc_dim = encoder_dim;
        m->enc_layers = enc_layers;
        build_encoder_inventory(m);
    });
}

int fm_codec_encode(fm_codec* m, const float* audio, int64_t n, int32_t* codes, int* T_out) {
    return fm_guard([&] {
        FMCHECK(m && audio && codes && T_out, "null argument");
        FMCHECK(m->enc_dim, "encoder not enabled (fm_codec_enable_encoder)");
        FMCHECK(n >= 1 && n <= (int64_t)m->max_frames * 2048, "audio must hold 1 .. 2048 * max_frames samples");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        const int T = (int)((n + 2047) / 2048);
        // DAC.encode right-pads to a multiple of frame_length (modded_dac.py:906-909); the device
        // expands the mono samples to 8 channels (one live: Ci % 8 == 0 for the implicit-GEMM conv)
        HIPCHK(hipMemcpyAsync(m->e_pcm, audio, (size_t)n * 4, hipMemcpyHostToDevice, m->stream));
        m->flops = 0;
        HIPCHK(hipEventRecord(m->e0, m->stream));
        if (m->prec == FM_PREC_BF16) {
            launch_audio8<bf16_t>(m->stream, m->e_pcm, n, (int64_t)T * 2048, (bf16_t*)m->e_audio);
            CRun<bf16_t> r(m);
            r.encode(T);
        } else {
            launch_audio8<float>(m->stream, m->e_pcm, n, (int64_t)T * 2048, (float*)m->e_audio);
            CRun<float> r(m);
            r.encode(T);
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(m->e1, m->stream));
        const int nq1 = m->c.n_codebooks + 1;
        HIPCHK(hipMemcpyAsync(codes, m->e_codes, (size_t)nq1 * T * 4, hipMemcpyDeviceToHost, m->stream));
        HIPCHK(hipStreamSynchronize(m->stream));
        float ms = 0;  // device time of the encode (fm_codec_profile_read totals decode + encode)
        HIPCHK(hipEventElapsedTime(&ms, m->e0, m->e1));
        m->last_ms = ms;
        m->total_ms += ms;
        m->total_flops += m->flops;
        *T_out = T;
    });
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

static void stream_zero(fm_codec* m) {
    for (size_t i = 0; i < m->st_slots.size(); ++i)
        HIPCHK(hipMemsetAsync(*m->st_slots[i], 0, m->st_all[i].second, m->stream));
    HIPCHK(hipStreamSynchronize(m->stream));
    m->spos = 0;
}

int fm_codec_stream_reset(fm_codec* m) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        m->activate(0);
        stream_zero(m);
    });
}

int fm_codec_decode_chunk(fm_codec* m, const int32_t* codes, int T, float* pcm) {
    return fm_codec_stream_decode(m, 0, codes, T, pcm);
}

int fm_codec_stream_open(fm_codec* m, int* sid) {
    return fm_guard([&] {
        FMCHECK(m && sid, "null argument");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        const int id = m->next_sid++;
        fm_codec::StreamCtx ctx;
        for (auto& pb : m->st_all) {
            void* p = nullptr;
            hipError_t e = hipMalloc(&p, pb.second);
            if (e != hipSuccess) {
                for (void* q : ctx.bufs) (void)hipFree(q);
                throw FmError{FM_ERR_OOM, "codec stream state: hipMalloc failed"};
            }
            ctx.bufs.push_back(p);
            HIPCHK(hipMemsetAsync(p, 0, pb.second, m->stream));
        }
        HIPCHK(hipStreamSynchronize(m->stream));
        m->sctx.emplace(id, std::move(ctx));
        *sid = id;
    });
}

int fm_codec_stream_rewind(fm_codec* m, int sid) {
    return fm_guard([&] {
        FMCHECK(m && sid > 0, "bad stream id (0 is the handle's own stream: stream_reset)");
        FMCHECK(m->sctx.count(sid), "unknown codec stream id " + std::to_string(sid));
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        m->activate(sid);
        stream_zero(m);
    });
}

int fm_codec_stream_close(fm_codec* m, int sid) {
    return fm_guard([&] {
        FMCHECK(m && sid > 0, "bad stream id (0 is the handle's own stream)");
        auto it = m->sctx.find(sid);
        FMCHECK(it != m->sctx.end(), "unknown codec stream id " + std::to_string(sid));
        HIPCHK(hipSetDevice(m->device));
        if (m->active_sid == sid) m->activate(0);
        HIPCHK(hipStreamSynchronize(m->stream));
        for (void* p : it->second.bufs) (void)hipFree(p);
        m->sctx.erase(it);
    });
}

int fm_codec_stream_decode(fm_codec* m, int sid, const int32_t* codes, int T, float* pcm) {
    return fm_guard([&] {
        FMCHECK(m, "null handle");
        HIPCHK(hipSetDevice(m->device));
        finalize(m);
        m->activate(sid);
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

// test hook: copy an intermediate of the last decode / encode as fp32 (time-major):
// 1 = transformer output [T][D], 2 = upsample-1 [2T][D], 3 = decoder input latent [4T][D],
// 10 = encoder output [4T][D], 11 = quantizer input after downsample + pre_module [T][D]
int fm_codec_debug_read(fm_codec* m, int stage, int T, float* out) {
    return fm_guard([&] {
        FMCHECK(m && out && m->finalized, "bad arguments");
        FMCHECK((stage >= 1 && stage <= 3) || ((stage == 10 || stage == 11) && m->enc_dim),
                "debug stage must be 1..3 or 10..11");
        FMCHECK(T >= 1 && T <= m->max_frames, "bad T");
        const int D = m->c.latent;
        const void* src = stage == 1    ? m->xn
                          : stage == 2  ? m->u0
                          : stage == 3  ? m->u1
                          : stage == 10 ? m->e_zenc
                                        : m->e_zpre;
        const size_t n = (size_t)(stage == 1 || stage == 11 ? 1 : stage == 2 ? 2 : 4) * T * D;
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

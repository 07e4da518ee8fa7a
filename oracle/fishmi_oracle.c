/*
 * fishmi_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library,
 * and only as the checker / the timed CPU baseline.  The product path (libfishmi.so) never
 * links or calls it.
 *
 * What it restates (file:line in /root/reference):
 *   Dual-AR decode (text2semantic)
 *     embedding gather/sum/mask/scale ............ llama.py:399-420
 *     RMSNorm (two roundings) ..................... llama.py:989-1000
 *     qk-norm nn.RMSNorm (one rounding) ........... llama.py:861-863, 900-902
 *     RoPE, bf16 cos/sin table .................... llama.py:1003-1037
 *     KV cache write ............................. llama.py:205-214
 *     slow attention (SDPA over the masked cache)  llama.py:915-933
 *     fast attention (matmul-softmax-matmul) ...... llama.py:947-975
 *     SwiGLU FFN, pre-norm residual block ......... llama.py:838-843, 978-986
 *     forward_generate / forward_generate_fast .... llama.py:390-466, 798-827
 *     logits_to_probs / sample / RAS .............. inference.py:43-93, 117-144
 *     decode_one_token_ar ......................... inference.py:96-181
 *     generate / decode_n_tokens (im_end stop) .... inference.py:184-359
 *   Codec decode (modded DAC)
 *     RVQ decode (clamp, codebook gather, WN 1x1) . rvq.py:352-366 + descript from_codes
 *     window-limited causal transformer ........... modded_dac.py:97-347, 349-439
 *     upsample: causal convT k2s2 + ConvNeXt ...... rvq.py:100-191, 263-276
 *     decoder: snake, WN causal conv/convT, RUs ... modded_dac.py:521-620, 712-801
 *
 * Precision: mode 1 ("bf16") rounds to bf16 at exactly the points the reference rounds when
 * run with bf16 weights; mode 0 ("fp32") rounds nowhere.  Accumulations are fp32.
 * Build: see oracle/Makefile (plain C99 + OpenMP, -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------ */
/* bf16 helpers                                                                          */
/* ------------------------------------------------------------------------------------ */
static inline float bf16r(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u)
        u = (u | 0x00400000u) & 0xffff0000u;
    else
        u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
    float r;
    memcpy(&r, &u, 4);
    return r;
}
static inline uint16_t f2bf(float x) {
    float r = bf16r(x);
    uint32_t u;
    memcpy(&u, &r, 4);
    return (uint16_t)(u >> 16);
}
static inline float bf2f(uint16_t b) {
    uint32_t u = ((uint32_t)b) << 16;
    float r;
    memcpy(&r, &u, 4);
    return r;
}

static char g_err[512];
const char* orc_last_error(void) { return g_err; }
static int fail(const char* msg, const char* arg) {
    snprintf(g_err, sizeof g_err, "%s%s%s", msg, arg ? ": " : "", arg ? arg : "");
    return -1;
}

int orc_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------------------------------ */
/* synthetic weights (identical formula in fishmi/synth.py and csrc/fm_common.hip)      */
/* ------------------------------------------------------------------------------------ */
static uint32_t fnv1a32(const char* s) {
    uint32_t h = 0x811C9DC5u;
    for (; *s; ++s) {
        h ^= (uint8_t)*s;
        h *= 0x01000193u;
    }
    return h;
}
static inline uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void synth_fill(float* dst, int64_t n, uint64_t seed, const char* name, float center,
                       int log2_half) {
    const uint64_t base = seed * 0xD1B54A32D192ED03ull + (uint64_t)fnv1a32(name) * 0x9E3779B97F4A7C15ull;
    const float scale = ldexpf(1.0f, -24 - log2_half);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        int64_t m = (int64_t)(splitmix64(base + (uint64_t)i) >> 40);
        float r = (float)(2 * m - (1 << 24)) * scale;
        dst[i] = center + r;
    }
}

/* sampler uniform: bf16 in [0,1) (truncating), keyed by (seed, step, draw, index)      */
static inline float rng_uniform_bf16(uint64_t seed, uint64_t step, uint32_t draw, uint32_t idx) {
    uint64_t key = seed * 0xD1B54A32D192ED03ull + (step * 64ull + draw) * 0x9E3779B97F4A7C15ull + idx;
    uint32_t m = (uint32_t)(splitmix64(key) >> 40);
    float u = (float)m * (1.0f / 16777216.0f);
    uint32_t b;
    memcpy(&b, &u, 4);
    b &= 0xffff0000u;
    memcpy(&u, &b, 4);
    return u;
}

/* ------------------------------------------------------------------------------------ */
/* named tensor store                                                                    */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    char name[160];
    int64_t n;
    float* f;     /* fp32 copy (always present)                         */
    uint16_t* b;  /* bf16 copy (LLM in bf16 mode: used by the matvecs)   */
} tensor_t;

typedef struct {
    tensor_t* t;
    int n, cap;
} store_t;

static tensor_t* store_find(store_t* s, const char* name) {
    for (int i = 0; i < s->n; ++i)
        if (!strcmp(s->t[i].name, name)) return &s->t[i];
    return NULL;
}
static tensor_t* store_put(store_t* s, const char* name, int64_t n) {
    tensor_t* t = store_find(s, name);
    if (t && t->n != n) {
        free(t->f);
        free(t->b);
        t->f = NULL;
        t->b = NULL;
    }
    if (!t) {
        if (s->n == s->cap) {
            s->cap = s->cap ? 2 * s->cap : 256;
            s->t = (tensor_t*)realloc(s->t, sizeof(tensor_t) * s->cap);
        }
        t = &s->t[s->n++];
        memset(t, 0, sizeof *t);
        snprintf(t->name, sizeof t->name, "%s", name);
    }
    t->n = n;
    if (!t->f) t->f = (float*)malloc(sizeof(float) * (n ? n : 1));
    return t;
}
static void store_free(store_t* s) {
    for (int i = 0; i < s->n; ++i) {
        free(s->t[i].f);
        free(s->t[i].b);
    }
    free(s->t);
    memset(s, 0, sizeof *s);
}

/* ------------------------------------------------------------------------------------ */
/* Dual-AR LLM                                                                           */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    int vocab_size, dim, n_layer, n_head, n_local_heads, head_dim, intermediate_size;
    float rope_base, norm_eps;
    int max_seq_len;
    int qkv_bias, o_bias, qk_norm, tie_word_embeddings;
    int codebook_size, num_codebooks, semantic_begin_id, semantic_end_id, im_end_id;
    int scale_codebook_embeddings, norm_fastlayer_input;
    int n_fast_layer, fast_dim, fast_n_head, fast_n_local_heads, fast_head_dim,
        fast_intermediate_size;
    int fast_qkv_bias, fast_o_bias, fast_qk_norm;
} orc_llm_config;

typedef struct {
    float temperature, top_p; /* applied as bf16 tensors, like inference.py:305-306 */
    int top_k;
    uint64_t seed;
    int mask_im_end;          /* fixed-length runs (benchmarks): <|im_end|> also at -inf */
} orc_sampling;

typedef struct {
    int dim, n_head, n_kv, hd, inter, qkv_bias, o_bias, qk_norm;
    /* per layer tensors */
    tensor_t **wqkv, **bqkv, **wo, **bo, **qn, **kn, **w1, **w2, **w3, **an, **fn;
    float *kc, *vc; /* [layer][kv][S][hd] */
    int S;
    float *rope; /* [S][hd/2][2] bf16-valued */
} stack_t;

typedef struct {
    orc_llm_config c;
    int bf16;
    store_t st;
    stack_t slow, fast;
    tensor_t *emb, *cbemb, *norm, *out, *fproj_w, *fproj_b, *femb, *fnorm, *fout;
    int ready;
    /* scratch */
    float *x, *h, *xn, *qkv, *att, *tmp, *g, *u, *act, *hid, *lg;
} orc_llm;

#define R(m, v) ((m)->bf16 ? bf16r(v) : (v))

orc_llm* orc_llm_create(const orc_llm_config* c, int bf16_mode) {
    orc_llm* m = (orc_llm*)calloc(1, sizeof(orc_llm));
    m->c = *c;
    m->bf16 = bf16_mode;
    return m;
}

int orc_llm_set_tensor(orc_llm* m, const char* name, const float* data, int64_t n) {
    tensor_t* t = store_put(&m->st, name, n);
    memcpy(t->f, data, sizeof(float) * n);
    if (m->bf16)
        for (int64_t i = 0; i < n; ++i) t->f[i] = bf16r(t->f[i]);
    m->ready = 0;
    return 0;
}

int orc_llm_synth_tensor(orc_llm* m, const char* name, int64_t n, uint64_t seed, float center,
                         int log2_half) {
    tensor_t* t = store_put(&m->st, name, n);
    synth_fill(t->f, n, seed, name, center, log2_half);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) t->f[i] = bf16r(t->f[i]); /* synthetic weights are bf16 */
    m->ready = 0;
    return 0;
}

static tensor_t* need(orc_llm* m, const char* name, int64_t n, int* bad) {
    tensor_t* t = store_find(&m->st, name);
    if (!t || (n >= 0 && t->n != n)) {
        if (!*bad) fail(t ? "wrong size for tensor" : "missing tensor", name);
        *bad = 1;
        return NULL;
    }
    if (m->bf16 && !t->b) {
        t->b = (uint16_t*)malloc(sizeof(uint16_t) * t->n);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < t->n; ++i) t->b[i] = f2bf(t->f[i]);
    }
    return t;
}

static void rope_table(float* tab, int S, int hd, float base) {
    /* llama.py:1003-1022: freqs = 1/base^(arange(0,hd,2)/hd) (fp32), t*freqs (fp32), polar,
       stacked (cos, sin) cast to bf16. */
    int half = hd / 2;
    for (int i = 0; i < half; ++i) {
        float e = (float)(2 * i) / (float)hd;
        float freq = 1.0f / powf(base, e);
        for (int p = 0; p < S; ++p) {
            float ang = (float)p * freq;
            tab[(p * half + i) * 2 + 0] = bf16r(cosf(ang));
            tab[(p * half + i) * 2 + 1] = bf16r(sinf(ang));
        }
    }
}

static int stack_init(orc_llm* m, stack_t* s, const char* prefix, int nl, int dim, int nh, int nkv,
                      int hd, int inter, int qb, int ob, int qkn, int S) {
    int bad = 0;
    char nm[200];
    s->dim = dim; s->n_head = nh; s->n_kv = nkv; s->hd = hd; s->inter = inter;
    s->qkv_bias = qb; s->o_bias = ob; s->qk_norm = qkn; s->S = S;
#define ALLOC(f) s->f = (tensor_t**)calloc(nl, sizeof(tensor_t*))
    ALLOC(wqkv); ALLOC(bqkv); ALLOC(wo); ALLOC(bo); ALLOC(qn); ALLOC(kn); ALLOC(w1); ALLOC(w2);
    ALLOC(w3); ALLOC(an); ALLOC(fn);
#undef ALLOC
    int nqkv = (nh + 2 * nkv) * hd;
    for (int l = 0; l < nl; ++l) {
#define GET(field, suffix, count)                                           \
    snprintf(nm, sizeof nm, "%s%d.%s", prefix, l, suffix);                  \
    s->field[l] = need(m, nm, count, &bad);
        GET(wqkv, "attention.wqkv.weight", (int64_t)nqkv * dim);
        if (qb) { GET(bqkv, "attention.wqkv.bias", nqkv); }
        GET(wo, "attention.wo.weight", (int64_t)dim * nh * hd);
        if (ob) { GET(bo, "attention.wo.bias", dim); }
        if (qkn) {
            GET(qn, "attention.q_norm.weight", hd);
            GET(kn, "attention.k_norm.weight", hd);
        }
        GET(w1, "feed_forward.w1.weight", (int64_t)inter * dim);
        GET(w3, "feed_forward.w3.weight", (int64_t)inter * dim);
        GET(w2, "feed_forward.w2.weight", (int64_t)dim * inter);
        GET(an, "attention_norm.weight", dim);
        GET(fn, "ffn_norm.weight", dim);
#undef GET
    }
    free(s->kc); free(s->vc); free(s->rope);
    size_t kvn = (size_t)nl * nkv * S * hd;
    s->kc = (float*)calloc(kvn, sizeof(float));
    s->vc = (float*)calloc(kvn, sizeof(float));
    s->rope = (float*)malloc(sizeof(float) * S * hd);
    rope_table(s->rope, S, hd, m->c.rope_base);
    return bad ? -1 : 0;
}

static int llm_finalize(orc_llm* m) {
    if (m->ready) return 0;
    const orc_llm_config* c = &m->c;
    int bad = 0;
    int S = c->max_seq_len;
    if (S % 8) S += 8 - S % 8; /* setup_caches: find_multiple(max_seq_len, 8) */
    if (stack_init(m, &m->slow, "layers.", c->n_layer, c->dim, c->n_head, c->n_local_heads,
                   c->head_dim, c->intermediate_size, c->qkv_bias, c->o_bias, c->qk_norm, S))
        return -1;
    if (stack_init(m, &m->fast, "fast_layers.", c->n_fast_layer, c->fast_dim, c->fast_n_head,
                   c->fast_n_local_heads, c->fast_head_dim, c->fast_intermediate_size,
                   c->fast_qkv_bias, c->fast_o_bias, c->fast_qk_norm, c->num_codebooks))
        return -1;
    m->emb = need(m, "embeddings.weight", (int64_t)c->vocab_size * c->dim, &bad);
    m->cbemb = need(m, "codebook_embeddings.weight",
                    (int64_t)c->codebook_size * c->num_codebooks * c->dim, &bad);
    m->norm = need(m, "norm.weight", c->dim, &bad);
    m->out = c->tie_word_embeddings ? m->emb
                                    : need(m, "output.weight", (int64_t)c->vocab_size * c->dim, &bad);
    if (c->fast_dim != c->dim) {
        m->fproj_w = need(m, "fast_project_in.weight", (int64_t)c->fast_dim * c->dim, &bad);
        m->fproj_b = need(m, "fast_project_in.bias", c->fast_dim, &bad);
    } else {
        m->fproj_w = m->fproj_b = NULL;
    }
    m->femb = need(m, "fast_embeddings.weight", (int64_t)c->codebook_size * c->fast_dim, &bad);
    m->fnorm = need(m, "fast_norm.weight", c->fast_dim, &bad);
    m->fout = need(m, "fast_output.weight", (int64_t)c->codebook_size * c->fast_dim, &bad);
    if (bad) return -1;
    int dmax = c->dim > c->fast_dim ? c->dim : c->fast_dim;
    int imax = c->intermediate_size > c->fast_intermediate_size ? c->intermediate_size
                                                                 : c->fast_intermediate_size;
    int qmax = (c->n_head + 2 * c->n_local_heads) * c->head_dim;
    int qf = (c->fast_n_head + 2 * c->fast_n_local_heads) * c->fast_head_dim;
    if (qf > qmax) qmax = qf;
    int big = dmax > qmax ? dmax : qmax;
    if (imax > big) big = imax;
    free(m->x); free(m->h); free(m->xn); free(m->qkv); free(m->att); free(m->tmp);
    free(m->g); free(m->u); free(m->act); free(m->hid); free(m->lg);
    m->x = malloc(sizeof(float) * big); m->h = malloc(sizeof(float) * big);
    m->xn = malloc(sizeof(float) * big); m->qkv = malloc(sizeof(float) * big);
    m->att = malloc(sizeof(float) * big); m->tmp = malloc(sizeof(float) * big);
    m->g = malloc(sizeof(float) * big); m->u = malloc(sizeof(float) * big);
    m->act = malloc(sizeof(float) * big); m->hid = malloc(sizeof(float) * big);
    int lgn = c->vocab_size > c->codebook_size ? c->vocab_size : c->codebook_size;
    m->lg = malloc(sizeof(float) * lgn);
    m->ready = 1;
    return 0;
}

int orc_llm_reset(orc_llm* m) {
    if (llm_finalize(m)) return -1;
    size_t a = (size_t)m->c.n_layer * m->slow.n_kv * m->slow.S * m->slow.hd;
    size_t b = (size_t)m->c.n_fast_layer * m->fast.n_kv * m->fast.S * m->fast.hd;
    memset(m->slow.kc, 0, a * 4); memset(m->slow.vc, 0, a * 4);
    memset(m->fast.kc, 0, b * 4); memset(m->fast.vc, 0, b * 4);
    return 0;
}

/* y[n] = sum_k W[n,k] x[k] (+ bias[n]); fp32 accumulation, 16 partial sums per row.       */
static void matvec(const orc_llm* m, const tensor_t* W, const tensor_t* bias, const float* x,
                   int N, int K, float* y) {
#pragma omp parallel for schedule(static)
    for (int n = 0; n < N; ++n) {
        float acc[16] = {0};
        int k = 0;
        if (m->bf16) {
            const uint16_t* w = W->b + (size_t)n * K;
            for (; k + 16 <= K; k += 16)
                for (int j = 0; j < 16; ++j) acc[j] += bf2f(w[k + j]) * x[k + j];
            for (; k < K; ++k) acc[0] += bf2f(w[k]) * x[k];
        } else {
            const float* w = W->f + (size_t)n * K;
            for (; k + 16 <= K; k += 16)
                for (int j = 0; j < 16; ++j) acc[j] += w[k + j] * x[k + j];
            for (; k < K; ++k) acc[0] += w[k] * x[k];
        }
        float s = 0.f;
        for (int j = 0; j < 16; ++j) s += acc[j];
        if (bias) s += bias->f[n];
        y[n] = s;
    }
}

/* llama.py:989-1000: (x.float() * rsqrt(mean(x^2)+eps)).type_as(x) * weight               */
static void rmsnorm(const orc_llm* m, const float* x, const tensor_t* w, int n, float* y) {
    float ss = 0.f;
    for (int i = 0; i < n; ++i) ss += x[i] * x[i];
    float r = 1.0f / sqrtf(ss / (float)n + m->c.norm_eps);
    for (int i = 0; i < n; ++i) y[i] = R(m, R(m, x[i] * r) * w->f[i]);
}
/* nn.RMSNorm on a head (torch rms_norm): fp32 compute incl. weight, one rounding           */
static void headnorm(const orc_llm* m, float* x, const tensor_t* w, int n) {
    float ss = 0.f;
    for (int i = 0; i < n; ++i) ss += x[i] * x[i];
    float r = 1.0f / sqrtf(ss / (float)n + m->c.norm_eps);
    for (int i = 0; i < n; ++i) x[i] = R(m, (x[i] * r) * w->f[i]);
}
/* llama.py:1025-1037 interleaved-pair rotation in fp32, rounded to the activation dtype     */
static void rope(const orc_llm* m, float* x, const float* tab, int hd) {
    for (int i = 0; i < hd / 2; ++i) {
        float x0 = x[2 * i], x1 = x[2 * i + 1];
        float c = tab[2 * i], s = tab[2 * i + 1];
        float a = x0 * c;
        float b = x1 * s;
        float d = x1 * c;
        float e = x0 * s;
        x[2 * i] = R(m, a - b);
        x[2 * i + 1] = R(m, d + e);
    }
}
static inline float silu(float a) { return a / (1.0f + expf(-a)); }

/* One transformer block at position pos (TransformerBlock.forward, llama.py:838-843). */
static void block(orc_llm* m, stack_t* s, int l, int pos, int is_fast, float* x) {
    const int d = s->dim, nh = s->n_head, nkv = s->n_kv, hd = s->hd, I = s->inter;
    const int nq = nh * hd, nk = nkv * hd;
    float* xn = m->xn;
    float* qkv = m->qkv;
    rmsnorm(m, x, s->an[l], d, xn);
    matvec(m, s->wqkv[l], s->qkv_bias ? s->bqkv[l] : NULL, xn, nq + 2 * nk, d, qkv);
    for (int i = 0; i < nq + 2 * nk; ++i) qkv[i] = R(m, qkv[i]);
    float* q = qkv;
    float* k = qkv + nq;
    float* v = qkv + nq + nk;
    if (s->qk_norm) {
        for (int h = 0; h < nh; ++h) headnorm(m, q + h * hd, s->qn[l], hd);
        for (int h = 0; h < nkv; ++h) headnorm(m, k + h * hd, s->kn[l], hd);
    }
    const float* tab = s->rope + (size_t)pos * hd;
    for (int h = 0; h < nh; ++h) rope(m, q + h * hd, tab, hd);
    for (int h = 0; h < nkv; ++h) rope(m, k + h * hd, tab, hd);
    size_t lofs = (size_t)l * nkv * s->S * hd;
    for (int h = 0; h < nkv; ++h) {
        memcpy(s->kc + lofs + ((size_t)h * s->S + pos) * hd, k + h * hd, sizeof(float) * hd);
        memcpy(s->vc + lofs + ((size_t)h * s->S + pos) * hd, v + h * hd, sizeof(float) * hd);
    }
    const float scale = 1.0f / sqrtf((float)hd);
    const int g = nh / nkv;
    float* y = m->att;
    int npos = is_fast ? s->S : pos + 1; /* fast: softmax over all C slots, masked */
    float* sc = (float*)malloc(sizeof(float) * (npos > 0 ? npos : 1));
    for (int h = 0; h < nh; ++h) {
        const float* kh = s->kc + lofs + (size_t)(h / g) * s->S * hd;
        const float* vh = s->vc + lofs + (size_t)(h / g) * s->S * hd;
        const float* qh = q + h * hd;
        float mx = -INFINITY;
        for (int j = 0; j < npos; ++j) {
            float dot = 0.f;
            for (int e = 0; e < hd; ++e) dot += qh[e] * kh[(size_t)j * hd + e];
            float sj;
            if (is_fast) /* llama.py:970-971: (q@k^T) rounded, * scale rounded, + bias */
                sj = (j <= pos) ? R(m, R(m, dot) * scale) : -INFINITY;
            else /* SDPA: fp32 scores over the valid prefix (mask kills j > pos) */
                sj = dot * scale;
            sc[j] = sj;
            if (sj > mx) mx = sj;
        }
        float den = 0.f;
        for (int j = 0; j < npos; ++j) {
            sc[j] = (sc[j] == -INFINITY) ? 0.f : expf(sc[j] - mx);
            den += sc[j];
        }
        for (int j = 0; j < npos; ++j) sc[j] = is_fast ? R(m, sc[j] / den) : sc[j] / den;
        for (int e = 0; e < hd; ++e) {
            float acc = 0.f;
            for (int j = 0; j < npos; ++j) acc += sc[j] * vh[(size_t)j * hd + e];
            y[h * hd + e] = R(m, acc);
        }
    }
    free(sc);
    float* t = m->tmp;
    matvec(m, s->wo[l], s->o_bias ? s->bo[l] : NULL, y, d, nq, t);
    float* hbuf = m->h;
    for (int i = 0; i < d; ++i) hbuf[i] = R(m, x[i] + R(m, t[i]));
    rmsnorm(m, hbuf, s->fn[l], d, xn);
    matvec(m, s->w1[l], NULL, xn, I, d, m->g);
    matvec(m, s->w3[l], NULL, xn, I, d, m->u);
    for (int i = 0; i < I; ++i) {
        float a = R(m, m->g[i]);
        float b = R(m, m->u[i]);
        m->act[i] = R(m, R(m, silu(a)) * b);
    }
    matvec(m, s->w2[l], NULL, m->act, d, I, t);
    for (int i = 0; i < d; ++i) x[i] = R(m, hbuf[i] + R(m, t[i]));
}

/* Slow forward over S positions starting at pos0 (tokens: (C+1) x S row-major).
   Writes logits of the LAST position (V) and the hidden state handed to the fast model
   (after fast_project_in), like forward_generate (llama.py:390-466, 818-827). */
int orc_llm_forward(orc_llm* m, const int32_t* tok, int S, int pos0, float* logits, float* hidden) {
    if (llm_finalize(m)) return -1;
    const orc_llm_config* c = &m->c;
    const int d = c->dim, C = c->num_codebooks, cb = c->codebook_size;
    for (int s = 0; s < S; ++s) {
        int pos = pos0 + s;
        if (pos >= m->slow.S) return fail("position beyond max_seq_len", NULL);
        int t0 = tok[s];
        int sem = (t0 >= c->semantic_begin_id) && (t0 <= c->semantic_end_id);
        float* x = m->x;
        /* llama.py:399-420 */
        for (int i = 0; i < d; ++i) {
            float v = 0.f;
            if (sem) {
                for (int q = 0; q < C; ++q) {
                    int id = tok[(q + 1) * S + s] + q * cb;
                    v += m->cbemb->f[(size_t)id * d + i];
                }
                v = R(m, v);
            }
            float e = R(m, m->emb->f[(size_t)t0 * d + i] + v);
            if (c->scale_codebook_embeddings && sem) e = R(m, e / sqrtf((float)(C + 1)));
            x[i] = e;
        }
        for (int l = 0; l < c->n_layer; ++l) block(m, &m->slow, l, pos, 0, x);
    }
    float* xn = m->xn;
    rmsnorm(m, m->x, m->norm, d, xn);
    if (logits) {
        matvec(m, m->out, NULL, xn, c->vocab_size, d, logits);
        for (int i = 0; i < c->vocab_size; ++i) logits[i] = R(m, logits[i]);
    }
    const float* hsrc = c->norm_fastlayer_input ? xn : m->x;
    if (m->fproj_w) {
        matvec(m, m->fproj_w, m->fproj_b, hsrc, c->fast_dim, d, m->hid);
        for (int i = 0; i < c->fast_dim; ++i) m->hid[i] = R(m, m->hid[i]);
    } else {
        memcpy(m->hid, hsrc, sizeof(float) * d);
    }
    if (hidden) memcpy(hidden, m->hid, sizeof(float) * c->fast_dim);
    return 0;
}

/* forward_generate_fast (llama.py:798-816) at codebook position pos.  Input: the slow hidden
   (code < 0) or fast_embeddings[code].  Writes codebook logits (cb) if requested. */
int orc_llm_fast(orc_llm* m, const float* hidden, int code, int pos, float* logits) {
    if (llm_finalize(m)) return -1;
    const orc_llm_config* c = &m->c;
    const int fd = c->fast_dim;
    float* x = m->x;
    if (code < 0)
        memcpy(x, hidden, sizeof(float) * fd);
    else
        memcpy(x, m->femb->f + (size_t)code * fd, sizeof(float) * fd);
    for (int l = 0; l < c->n_fast_layer; ++l) block(m, &m->fast, l, pos, 1, x);
    if (logits) {
        rmsnorm(m, x, m->fnorm, fd, m->xn);
        matvec(m, m->fout, NULL, m->xn, c->codebook_size, fd, logits);
        for (int i = 0; i < c->codebook_size; ++i) logits[i] = R(m, logits[i]);
    }
    return 0;
}

/* ---- sampling: logits_to_probs + multinomial_sample_one_no_sync (inference.py:43-93) ---- */
typedef struct { float v; int i; } kv_t;
static int kv_cmp(const void* a, const void* b) {
    const kv_t* x = (const kv_t*)a;
    const kv_t* y = (const kv_t*)b;
    if (x->v > y->v) return -1;
    if (x->v < y->v) return 1;
    return x->i - y->i; /* stable: ties keep index order (matches torch.sort, golden ops) */
}

/* probs[] (bf16-valued, length n) from logits (bf16-valued; -inf allowed).  Returns kept count. */
int orc_logits_to_probs(const float* logits, int n, float temperature, float top_p, int top_k,
                        int bf16, float* probs) {
#define RB(v) (bf16 ? bf16r(v) : (v))
    kv_t* s = (kv_t*)malloc(sizeof(kv_t) * n);
    for (int i = 0; i < n; ++i) { s[i].v = logits[i]; s[i].i = i; }
    qsort(s, n, sizeof(kv_t), kv_cmp);
    float t = RB(temperature), p = RB(top_p);
    float mx = s[0].v, den = 0.f;
    for (int i = 0; i < n; ++i) den += (s[i].v == -INFINITY) ? 0.f : expf(s[i].v - mx);
    float cum = 0.f;
    unsigned char* keep = (unsigned char*)calloc(n, 1);
    int kept = 0;
    for (int r = 0; r < n; ++r) {
        float pr = RB(((s[r].v == -INFINITY) ? 0.f : expf(s[r].v - mx)) / den);
        cum += pr;
        float cr = RB(cum);
        int remove = (cr > p) || (r >= top_k);
        if (r == 0) remove = 0;
        if (!remove) { keep[s[r].i] = 1; kept++; }
    }
    float tt = t < 1e-5f ? 1e-5f : t;
    float m2 = -INFINITY;
    for (int i = 0; i < n; ++i) {
        probs[i] = keep[i] ? RB(logits[i] / tt) : -INFINITY;
        if (probs[i] > m2) m2 = probs[i];
    }
    float d2 = 0.f;
    for (int i = 0; i < n; ++i) d2 += (probs[i] == -INFINITY) ? 0.f : expf(probs[i] - m2);
    for (int i = 0; i < n; ++i)
        probs[i] = (probs[i] == -INFINITY) ? 0.f : RB(expf(probs[i] - m2) / d2);
    free(keep);
    free(s);
    return kept;
#undef RB
}

/* argmax(probs / bf16(-log(u))) with u the bf16 uniforms of (seed, step, draw). */
int orc_sample(const float* logits, int n, float temperature, float top_p, int top_k, int bf16,
               uint64_t seed, uint64_t step, uint32_t draw) {
    float* probs = (float*)malloc(sizeof(float) * n);
    orc_logits_to_probs(logits, n, temperature, top_p, top_k, bf16, probs);
    int best = 0;
    float bv = -1.f;
    for (int i = 0; i < n; ++i) {
        if (probs[i] <= 0.f) continue;
        float u = rng_uniform_bf16(seed, step, draw, (uint32_t)i);
        float q = bf16 ? bf16r(-logf(u)) : -logf(u);
        float r = bf16 ? bf16r(probs[i] / q) : probs[i] / q;
        if (r > bv) { bv = r; best = i; }
    }
    free(probs);
    return best;
}

/* decode_one_token_ar (inference.py:96-181) on already-computed slow logits/hidden.
   prev: RAS window (C+1) x 10 or NULL.  Writes the (C+1) column. */
static int one_frame(orc_llm* m, const orc_sampling* sp, uint64_t step, const int* prev,
                     int32_t* col) {
    const orc_llm_config* c = &m->c;
    const int V = c->vocab_size, C = c->num_codebooks, cb = c->codebook_size;
    float* lg = m->lg;
    for (int i = 0; i < V; ++i) {
        int allowed = (i >= c->semantic_begin_id && i <= c->semantic_end_id) ||
                      (i == c->im_end_id && !sp->mask_im_end);
        if (!allowed) lg[i] = -INFINITY;
    }
    int tok = orc_sample(lg, V, sp->temperature, sp->top_p, sp->top_k, m->bf16, sp->seed, step, 0);
    int hi = orc_sample(lg, V, 1.0f, 0.9f, sp->top_k, m->bf16, sp->seed, step, 1);
    if (prev) {
        int inwin = 0;
        for (int j = 0; j < 10; ++j) inwin |= (prev[j] == tok);
        int sem = tok >= c->semantic_begin_id && tok <= c->semantic_end_id;
        if (inwin && sem) tok = hi;
    }
    col[0] = tok;
    float* hid = (float*)malloc(sizeof(float) * c->fast_dim);
    memcpy(hid, m->hid, sizeof(float) * c->fast_dim);
    orc_llm_fast(m, hid, -1, 0, NULL);
    free(hid);
    int a = tok - c->semantic_begin_id;
    a = a < 0 ? 0 : (a > cb - 1 ? cb - 1 : a);
    col[1] = a;
    float* fl = (float*)malloc(sizeof(float) * cb);
    for (int q = 1; q < C; ++q) {
        if (orc_llm_fast(m, NULL, a, q, fl)) { free(fl); return -1; }
        a = orc_sample(fl, cb, sp->temperature, sp->top_p, sp->top_k, m->bf16, sp->seed, step, 1 + q);
        col[q + 1] = a;
    }
    free(fl);
    return 0;
}

/* wall time of the last orc_llm_generate: prompt pass + first frame, and the decode frames
   after it (bench.py's cpu_baseline leg reads these to avoid timing the prefill twice). */
static double g_gen_prefill_s, g_gen_frames_s;
void orc_llm_gen_timing(double* prefill_s, double* frames_s) {
    if (prefill_s) *prefill_s = g_gen_prefill_s;
    if (frames_s) *frames_s = g_gen_frames_s;
}

/* generate (inference.py:241-359): prompt (C+1) x T row-major -> out (C+1) x n_new
   row-major (stride max_new), returns n produced (stops after emitting im_end). */
int orc_llm_generate(orc_llm* m, const int32_t* prompt, int T, int max_new, const orc_sampling* sp,
                     int32_t* out) {
    if (orc_llm_reset(m)) return -1;
    const orc_llm_config* c = &m->c;
    const int C = c->num_codebooks;
    int S = m->slow.S;
    if (T >= c->max_seq_len) return fail("prompt longer than max_seq_len", NULL);
    if (max_new <= 0 || T + max_new > c->max_seq_len) max_new = c->max_seq_len - T;
    (void)S;
    int32_t col[64];
    const double t0 = omp_get_wtime();
    if (orc_llm_forward(m, prompt, T, 0, m->lg, NULL)) return -1;
    if (one_frame(m, sp, 0, NULL, col)) return -1;
    const double t1 = omp_get_wtime();
    g_gen_prefill_s = t1 - t0;
    for (int r = 0; r <= C; ++r) out[r * max_new + 0] = col[r];
    int n = 1;
    int* prev = (int*)calloc((size_t)(C + 1) * 10, sizeof(int));
    int32_t xcol[64];
    for (int it = 0; it < max_new - 1; ++it) {
        memcpy(xcol, col, sizeof(int32_t) * (C + 1));
        if (orc_llm_forward(m, xcol, 1, T + it, m->lg, NULL)) { free(prev); return -1; }
        if (one_frame(m, sp, (uint64_t)it + 1, prev, col)) { free(prev); return -1; }
        for (int r = 0; r <= C; ++r) {
            memmove(prev + r * 10, prev + r * 10 + 1, sizeof(int) * 9);
            prev[r * 10 + 9] = col[r];
        }
        for (int r = 0; r <= C; ++r) out[r * max_new + n] = col[r];
        n++;
        if (col[0] == c->im_end_id) break;
    }
    g_gen_frames_s = omp_get_wtime() - t1;
    free(prev);
    return n;
}

void orc_llm_free(orc_llm* m) {
    if (!m) return;
    store_free(&m->st);
    stack_t* ss[2] = {&m->slow, &m->fast};
    for (int i = 0; i < 2; ++i) {
        stack_t* s = ss[i];
        free(s->wqkv); free(s->bqkv); free(s->wo); free(s->bo); free(s->qn); free(s->kn);
        free(s->w1); free(s->w2); free(s->w3); free(s->an); free(s->fn);
        free(s->kc); free(s->vc); free(s->rope);
    }
    free(m->x); free(m->h); free(m->xn); free(m->qkv); free(m->att); free(m->tmp);
    free(m->g); free(m->u); free(m->act); free(m->hid); free(m->lg);
    free(m);
}

/* ------------------------------------------------------------------------------------ */
/* Codec decode (fp32)                                                                   */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    int latent, decoder_dim, n_codebooks, codebook_size, semantic_codebook_size, codebook_dim;
    int t_layers, t_heads, t_head_dim, t_inter, window;
    float rope_base, norm_eps;
} orc_codec_config;

typedef struct {
    orc_codec_config c;
    store_t st;
} orc_codec;

orc_codec* orc_codec_create(const orc_codec_config* c) {
    orc_codec* m = (orc_codec*)calloc(1, sizeof(orc_codec));
    m->c = *c;
    return m;
}
int orc_codec_set_tensor(orc_codec* m, const char* name, const float* data, int64_t n) {
    tensor_t* t = store_put(&m->st, name, n);
    memcpy(t->f, data, sizeof(float) * n);
    return 0;
}
int orc_codec_synth_tensor(orc_codec* m, const char* name, int64_t n, uint64_t seed, float center,
                           int log2_half) {
    tensor_t* t = store_put(&m->st, name, n);
    synth_fill(t->f, n, seed, name, center, log2_half);
    for (int64_t i = 0; i < n; ++i) t->f[i] = bf16r(t->f[i]); /* stored bf16 like the goldens */
    return 0;
}
void orc_codec_free(orc_codec* m) {
    if (!m) return;
    store_free(&m->st);
    free(m);
}

static const float* cget(orc_codec* m, const char* name, int64_t n, int* bad) {
    tensor_t* t = store_find(&m->st, name);
    if (!t || (n >= 0 && t->n != n)) {
        if (!*bad) fail(t ? "wrong size for tensor" : "missing tensor", name);
        *bad = 1;
        return NULL;
    }
    return t->f;
}

/* weight norm w = g * v / ||v||, norm over all dims except dim 0 of the stored layout
   (torch weight_norm dim=0; for ConvTranspose1d dim 0 is the INPUT channel).  rows x per. */
static float* wn_fold(const float* g, const float* v, int rows, int per) {
    float* w = (float*)malloc(sizeof(float) * (size_t)rows * per);
    for (int r = 0; r < rows; ++r) {
        double ss = 0;
        for (int i = 0; i < per; ++i) ss += (double)v[(size_t)r * per + i] * v[(size_t)r * per + i];
        float nrm = (float)sqrt(ss);
        for (int i = 0; i < per; ++i) w[(size_t)r * per + i] = g[r] * (v[(size_t)r * per + i] / nrm);
    }
    return w;
}

static void snake(float* x, const float* alpha, int Cn, int L) {
#pragma omp parallel for schedule(static)
    for (int c = 0; c < Cn; ++c) {
        float a = alpha[c];
        float inv = 1.0f / (a + 1e-9f);
        for (int t = 0; t < L; ++t) {
            float s = sinf(a * x[(size_t)c * L + t]);
            x[(size_t)c * L + t] = x[(size_t)c * L + t] + inv * (s * s);
        }
    }
}

/* causal conv1d stride 1 (CausalConvNet, modded_dac.py:521-552): left pad (k-1)*dil.
   w: [Co][Ci][k].  y: [Co][L] (= + bias) (+= residual when res != NULL) */
static void conv1d_causal(const float* x, int Ci, int L, const float* w, const float* b, int Co,
                          int k, int dil, float* y) {
#pragma omp parallel for schedule(static)
    for (int co = 0; co < Co; ++co) {
        float* yr = y + (size_t)co * L;
        for (int t = 0; t < L; ++t) yr[t] = b ? b[co] : 0.f;
        for (int ci = 0; ci < Ci; ++ci) {
            const float* xr = x + (size_t)ci * L;
            const float* wr = w + ((size_t)co * Ci + ci) * k;
            for (int j = 0; j < k; ++j) {
                int sh = (k - 1 - j) * dil;
                float wv = wr[j];
                for (int t = sh; t < L; ++t) yr[t] += wv * xr[t - sh];
            }
        }
    }
}

/* causal ConvTranspose1d, kernel k in {s, 2s}, stride s, right trim k-s (CausalTransConvNet,
   modded_dac.py:563-580 / rvq.py:100-117): w [Ci][Co][k]; y [Co][L*s] */
static void convT_causal(const float* x, int Ci, int L, const float* w, const float* b, int Co,
                         int s, int k, float* y) {
    const int Lo = L * s;
#pragma omp parallel for schedule(static)
    for (int co = 0; co < Co; ++co) {
        float* yr = y + (size_t)co * Lo;
        for (int t = 0; t < Lo; ++t) yr[t] = b ? b[co] : 0.f;
        for (int ci = 0; ci < Ci; ++ci) {
            const float* xr = x + (size_t)ci * L;
            const float* wr = w + ((size_t)ci * Co + co) * k;
            for (int t = 0; t < Lo; ++t) {
                int tq = t / s, j0 = t - tq * s;
                float acc = wr[j0] * xr[tq];
                if (k == 2 * s && tq >= 1) acc += wr[j0 + s] * xr[tq - 1];
                yr[t] += acc;
            }
        }
    }
}

/* y[T][N] = x[T][K] W[N][K]^T + b */
static void linear_rows(const float* x, int T, int K, const float* W, const float* b, int N, float* y) {
#pragma omp parallel for collapse(2) schedule(static)
    for (int t = 0; t < T; ++t)
        for (int n = 0; n < N; ++n) {
            const float* xr = x + (size_t)t * K;
            const float* wr = W + (size_t)n * K;
            float acc[8] = {0};
            int k = 0;
            for (; k + 8 <= K; k += 8)
                for (int j = 0; j < 8; ++j) acc[j] += xr[k + j] * wr[k + j];
            for (; k < K; ++k) acc[0] += xr[k] * wr[k];
            float s = 0.f;
            for (int j = 0; j < 8; ++j) s += acc[j];
            y[(size_t)t * N + n] = s + (b ? b[n] : 0.f);
        }
}

static void rms_rows(const float* x, int T, int D, const float* w, float eps, float* y) {
    for (int t = 0; t < T; ++t) {
        float ss = 0.f;
        for (int i = 0; i < D; ++i) ss += x[(size_t)t * D + i] * x[(size_t)t * D + i];
        float r = 1.0f / sqrtf(ss / (float)D + eps);
        for (int i = 0; i < D; ++i) y[(size_t)t * D + i] = (x[(size_t)t * D + i] * r) * w[i];
    }
}

/* WindowLimitedTransformer.forward (modded_dac.py:418-439) on x [T][D] in place: layers at
   `pre`layers.<l>., final norm `pre`norm.weight; causal window `window`. */
static int window_transformer_at(orc_codec* m, const char* pre, float* x, int T, int D, int H, int hd,
                                 int I, int nlayers, int window) {
    const orc_codec_config* c = &m->c;
    int bad = 0;
    char nm[200];
    float* xn = (float*)malloc(sizeof(float) * (size_t)T * D);
    float* qkv = (float*)malloc(sizeof(float) * (size_t)T * 3 * H * hd);
    float* y = (float*)malloc(sizeof(float) * (size_t)T * H * hd);
    float* t1 = (float*)malloc(sizeof(float) * (size_t)T * I);
    float* t3 = (float*)malloc(sizeof(float) * (size_t)T * I);
    float* o = (float*)malloc(sizeof(float) * (size_t)T * D);
    float* tab = (float*)malloc(sizeof(float) * (size_t)(T > 0 ? T : 1) * hd);
    /* modded_dac.py:442-452: the 327680-entry table, fp32 math, cast to bf16 */
    {
        int half = hd / 2;
        for (int i = 0; i < half; ++i) {
            float freq = 1.0f / powf(c->rope_base, (float)(2 * i) / (float)hd);
            for (int p = 0; p < T; ++p) {
                float ang = (float)p * freq;
                tab[(p * half + i) * 2] = bf16r(cosf(ang));
                tab[(p * half + i) * 2 + 1] = bf16r(sinf(ang));
            }
        }
    }
    for (int l = 0; l < nlayers; ++l) {
#define CW(var, suffix, cnt) \
    snprintf(nm, sizeof nm, "%slayers.%d.%s", pre, l, suffix); const float* var = cget(m, nm, cnt, &bad);
        CW(an, "attention_norm.weight", D);
        CW(wqkv, "attention.wqkv.weight", (int64_t)3 * H * hd * D);
        CW(wo, "attention.wo.weight", (int64_t)D * H * hd);
        CW(ag, "attention_layer_scale.gamma", D);
        CW(fnw, "ffn_norm.weight", D);
        CW(w1, "feed_forward.w1.weight", (int64_t)I * D);
        CW(w3, "feed_forward.w3.weight", (int64_t)I * D);
        CW(w2, "feed_forward.w2.weight", (int64_t)D * I);
        CW(fg, "ffn_layer_scale.gamma", D);
#undef CW
        if (bad) break;
        rms_rows(x, T, D, an, c->norm_eps, xn);
        linear_rows(xn, T, D, wqkv, NULL, 3 * H * hd, qkv);
        const int ld = 3 * H * hd;
        for (int t = 0; t < T; ++t)
            for (int h = 0; h < 2 * H; ++h) { /* q and k heads */
                float* v = qkv + (size_t)t * ld + h * hd;
                const float* tb = tab + (size_t)t * hd;
                for (int i = 0; i < hd / 2; ++i) {
                    float x0 = v[2 * i], x1 = v[2 * i + 1], cc = tb[2 * i], ss = tb[2 * i + 1];
                    float a = x0 * cc, b2 = x1 * ss, d2 = x1 * cc, e2 = x0 * ss;
                    v[2 * i] = a - b2;
                    v[2 * i + 1] = d2 + e2;
                }
            }
        const float scale = 1.0f / sqrtf((float)hd);
#pragma omp parallel for collapse(2) schedule(static)
        for (int t = 0; t < T; ++t)
            for (int h = 0; h < H; ++h) {
                const float* q = qkv + (size_t)t * ld + h * hd;
                int j0 = t - window + 1;
                if (j0 < 0) j0 = 0;
                float sc[4096];
                float mx = -INFINITY;
                int nj = t - j0 + 1;
                for (int j = 0; j < nj; ++j) {
                    const float* kk = qkv + (size_t)(j0 + j) * ld + (H + h) * hd;
                    float dot = 0.f;
                    for (int e = 0; e < hd; ++e) dot += q[e] * kk[e];
                    sc[j] = dot * scale;
                    if (sc[j] > mx) mx = sc[j];
                }
                float den = 0.f;
                for (int j = 0; j < nj; ++j) { sc[j] = expf(sc[j] - mx); den += sc[j]; }
                for (int e = 0; e < hd; ++e) {
                    float acc = 0.f;
                    for (int j = 0; j < nj; ++j)
                        acc += sc[j] * qkv[(size_t)(j0 + j) * ld + (2 * H + h) * hd + e];
                    y[(size_t)t * H * hd + h * hd + e] = acc / den;
                }
            }
        linear_rows(y, T, H * hd, wo, NULL, D, o);
        for (size_t i = 0; i < (size_t)T * D; ++i) x[i] = x[i] + o[i] * ag[i % D];
        rms_rows(x, T, D, fnw, c->norm_eps, xn);
        linear_rows(xn, T, D, w1, NULL, I, t1);
        linear_rows(xn, T, D, w3, NULL, I, t3);
        for (size_t i = 0; i < (size_t)T * I; ++i) t1[i] = silu(t1[i]) * t3[i];
        linear_rows(t1, T, I, w2, NULL, D, o);
        for (size_t i = 0; i < (size_t)T * D; ++i) x[i] = x[i] + o[i] * fg[i % D];
    }
    if (!bad) {
        snprintf(nm, sizeof nm, "%snorm.weight", pre);
        const float* nw = cget(m, nm, D, &bad);
        if (!bad) {
            rms_rows(x, T, D, nw, c->norm_eps, xn);
            memcpy(x, xn, sizeof(float) * (size_t)T * D);
        }
    }
    free(xn); free(qkv); free(y); free(t1); free(t3); free(o); free(tab);
    return bad ? -1 : 0;
}

static int window_transformer(orc_codec* m, float* x, int T) {
    const orc_codec_config* c = &m->c;
    return window_transformer_at(m, "quantizer.post_module.", x, T, c->latent, c->t_heads, c->t_head_dim,
                                 c->t_inter, c->t_layers, c->window);
}

/* ConvNeXtBlock (rvq.py:129-191) on x [D][L] in place. */
static int convnext(orc_codec* m, const char* pre, float* x, int D, int L) {
    int bad = 0;
    char nm[200];
#define CW(var, suffix, cnt) \
    snprintf(nm, sizeof nm, "%s%s", pre, suffix); const float* var = cget(m, nm, cnt, &bad);
    CW(dw, "dwconv.conv.weight", (int64_t)D * 7);
    CW(db, "dwconv.conv.bias", D);
    CW(lw, "norm.weight", D);
    CW(lb, "norm.bias", D);
    CW(p1w, "pwconv1.weight", (int64_t)4 * D * D);
    CW(p1b, "pwconv1.bias", 4 * D);
    CW(p2w, "pwconv2.weight", (int64_t)4 * D * D);
    CW(p2b, "pwconv2.bias", D);
    CW(gm, "gamma", D);
#undef CW
    if (bad) return -1;
    float* t = (float*)malloc(sizeof(float) * (size_t)L * D);  /* [L][D] */
    float* h = (float*)malloc(sizeof(float) * (size_t)L * 4 * D);
    float* o = (float*)malloc(sizeof(float) * (size_t)L * D);
#pragma omp parallel for schedule(static)
    for (int c = 0; c < D; ++c)
        for (int tt = 0; tt < L; ++tt) {
            float acc = db[c];
            for (int j = 0; j < 7; ++j) {
                int src = tt - 6 + j;
                if (src >= 0) acc += dw[c * 7 + j] * x[(size_t)c * L + src];
            }
            t[(size_t)tt * D + c] = acc;
        }
    for (int tt = 0; tt < L; ++tt) { /* LayerNorm eps 1e-6 over channels */
        float* r = t + (size_t)tt * D;
        float mu = 0.f;
        for (int i = 0; i < D; ++i) mu += r[i];
        mu /= (float)D;
        float var = 0.f;
        for (int i = 0; i < D; ++i) var += (r[i] - mu) * (r[i] - mu);
        var /= (float)D;
        float rs = 1.0f / sqrtf(var + 1e-6f);
        for (int i = 0; i < D; ++i) r[i] = (r[i] - mu) * rs * lw[i] + lb[i];
    }
    linear_rows(t, L, D, p1w, p1b, 4 * D, h);
    for (size_t i = 0; i < (size_t)L * 4 * D; ++i)
        h[i] = 0.5f * h[i] * (1.0f + erff(h[i] * 0.70710678118654752f));
    linear_rows(h, L, 4 * D, p2w, p2b, D, o);
    for (int c = 0; c < D; ++c)
        for (int tt = 0; tt < L; ++tt) x[(size_t)c * L + tt] += gm[c] * o[(size_t)tt * D + c];
    free(t); free(h); free(o);
    return 0;
}

/* CausalWNConv1d at key prefix `pre` (…conv.parametrizations.weight.original0/1, bias). */
static int wn_conv(orc_codec* m, const char* pre, const float* x, int Ci, int L, int Co, int k,
                   int dil, float* y) {
    int bad = 0;
    char nm[220];
    snprintf(nm, sizeof nm, "%sconv.parametrizations.weight.original0", pre);
    const float* g = cget(m, nm, Co, &bad);
    snprintf(nm, sizeof nm, "%sconv.parametrizations.weight.original1", pre);
    const float* v = cget(m, nm, (int64_t)Co * Ci * k, &bad);
    snprintf(nm, sizeof nm, "%sconv.bias", pre);
    const float* b = cget(m, nm, Co, &bad);
    if (bad) return -1;
    float* w = wn_fold(g, v, Co, Ci * k);
    conv1d_causal(x, Ci, L, w, b, Co, k, dil, y);
    free(w);
    return 0;
}

static float* g_dbg_rvq = NULL;  /* optional debug taps: [D][T] after RVQ / after post_module */
static float* g_dbg_post = NULL;
void orc_codec_debug_taps(float* rvq, float* post) { g_dbg_rvq = rvq; g_dbg_post = post; }

/* DAC.from_indices (modded_dac.py:925-927).  codes: (nq+1) x T row-major. */
int orc_codec_decode(orc_codec* m, const int32_t* codes_in, int T, float* wave, float* latent_out) {
    const orc_codec_config* c = &m->c;
    const int D = c->latent, nq = c->n_codebooks, cd = c->codebook_dim;
    int bad = 0;
    char nm[220];
    int32_t* codes = (int32_t*)malloc(sizeof(int32_t) * (nq + 1) * T);
    for (int q = 0; q <= nq; ++q)
        for (int t = 0; t < T; ++t) {
            int v = codes_in[q * T + t];
            int mx = (q == 0 ? c->semantic_codebook_size : c->codebook_size) - 1;
            codes[q * T + t] = v > mx ? mx : v; /* rvq.py:354-359 clamps max only */
        }
    /* RVQ decode: semantic quantizer + residual quantizer, out_proj = WN 1x1 conv (old
       weight_norm: weight_g [D,1,1], weight_v [D,cd,1]) */
    float* zs = (float*)calloc((size_t)D * T, sizeof(float));
    float* zr = (float*)calloc((size_t)D * T, sizeof(float));
    for (int q = 0; q <= nq && !bad; ++q) {
        const char* base = q == 0 ? "quantizer.semantic_quantizer.quantizers.0."
                                  : "quantizer.quantizer.quantizers.";
        char pre[160];
        if (q == 0) snprintf(pre, sizeof pre, "%s", base);
        else snprintf(pre, sizeof pre, "%s%d.", base, q - 1);
        int cbn = q == 0 ? c->semantic_codebook_size : c->codebook_size;
        snprintf(nm, sizeof nm, "%scodebook.weight", pre);
        const float* cbw = cget(m, nm, (int64_t)cbn * cd, &bad);
        snprintf(nm, sizeof nm, "%sout_proj.weight_g", pre);
        const float* g = cget(m, nm, D, &bad);
        snprintf(nm, sizeof nm, "%sout_proj.weight_v", pre);
        const float* v = cget(m, nm, (int64_t)D * cd, &bad);
        snprintf(nm, sizeof nm, "%sout_proj.bias", pre);
        const float* b = cget(m, nm, D, &bad);
        if (bad) break;
        float* w = wn_fold(g, v, D, cd);
        float* z = q == 0 ? zs : zr;
        for (int o = 0; o < D; ++o)
            for (int t = 0; t < T; ++t) {
                const float* e = cbw + (size_t)codes[q * T + t] * cd;
                float acc = 0.f;
                for (int j = 0; j < cd; ++j) acc += w[o * cd + j] * e[j];
                z[(size_t)o * T + t] += acc + b[o];
            }
        free(w);
    }
    free(codes);
    if (bad) { free(zs); free(zr); return -1; }
    /* z = zs + zr, post_module on [T][D] */
    float* xt = (float*)malloc(sizeof(float) * (size_t)T * D);
    for (int o = 0; o < D; ++o)
        for (int t = 0; t < T; ++t) xt[(size_t)t * D + o] = zs[(size_t)o * T + t] + zr[(size_t)o * T + t];
    free(zs); free(zr);
    if (g_dbg_rvq)
        for (int o = 0; o < D; ++o)
            for (int t = 0; t < T; ++t) g_dbg_rvq[(size_t)o * T + t] = xt[(size_t)t * D + o];
    if (window_transformer(m, xt, T)) { free(xt); return -1; }
    float* x = (float*)malloc(sizeof(float) * (size_t)D * T);
    for (int o = 0; o < D; ++o)
        for (int t = 0; t < T; ++t) x[(size_t)o * T + t] = xt[(size_t)t * D + o];
    if (g_dbg_post) memcpy(g_dbg_post, x, sizeof(float) * (size_t)D * T);
    free(xt);
    /* upsample: reversed(enumerate([2,2])) -> upsample.0 then upsample.1, each x2 */
    int L = T;
    for (int u = 0; u < 2; ++u) {
        snprintf(nm, sizeof nm, "quantizer.upsample.%d.0.conv.weight", u);
        const float* w = cget(m, nm, (int64_t)D * D * 2, &bad);
        snprintf(nm, sizeof nm, "quantizer.upsample.%d.0.conv.bias", u);
        const float* b = cget(m, nm, D, &bad);
        if (bad) { free(x); return -1; }
        float* y = (float*)malloc(sizeof(float) * (size_t)D * L * 2);
        convT_causal(x, D, L, w, b, D, 2, 2, y);
        free(x);
        x = y;
        L *= 2;
        snprintf(nm, sizeof nm, "quantizer.upsample.%d.1.", u);
        if (convnext(m, nm, x, D, L)) { free(x); return -1; }
    }
    if (latent_out) memcpy(latent_out, x, sizeof(float) * (size_t)D * L);
    /* Decoder (modded_dac.py:760-801) */
    const int ch = c->decoder_dim;
    float* y = (float*)malloc(sizeof(float) * (size_t)ch * L);
    if (wn_conv(m, "decoder.model.0.", x, D, L, ch, 7, 1, y)) { free(x); free(y); return -1; }
    free(x);
    x = y;
    int Cin = ch;
    const int rates[4] = {8, 8, 4, 2};
    for (int blk = 0; blk < 4; ++blk) {
        int s = rates[blk], Cout = Cin / 2;
        char pre[160];
        snprintf(pre, sizeof pre, "decoder.model.%d.block.", blk + 1);
        snprintf(nm, sizeof nm, "%s0.alpha", pre);
        const float* al = cget(m, nm, Cin, &bad);
        snprintf(nm, sizeof nm, "%s1.conv.parametrizations.weight.original0", pre);
        const float* g = cget(m, nm, Cin, &bad); /* convT weight norm: per INPUT channel */
        snprintf(nm, sizeof nm, "%s1.conv.parametrizations.weight.original1", pre);
        const float* v = cget(m, nm, (int64_t)Cin * Cout * 2 * s, &bad);
        snprintf(nm, sizeof nm, "%s1.conv.bias", pre);
        const float* b = cget(m, nm, Cout, &bad);
        if (bad) { free(x); return -1; }
        snake(x, al, Cin, L);
        float* w = wn_fold(g, v, Cin, Cout * 2 * s);
        y = (float*)malloc(sizeof(float) * (size_t)Cout * L * s);
        convT_causal(x, Cin, L, w, b, Cout, s, 2 * s, y);
        free(w); free(x);
        x = y;
        L *= s;
        const int dils[3] = {1, 3, 9};
        float* t1 = (float*)malloc(sizeof(float) * (size_t)Cout * L);
        float* t2 = (float*)malloc(sizeof(float) * (size_t)Cout * L);
        for (int r = 0; r < 3; ++r) {
            char rp[200];
            snprintf(rp, sizeof rp, "%s%d.block.", pre, r + 2);
            snprintf(nm, sizeof nm, "%s0.alpha", rp);
            const float* a0 = cget(m, nm, Cout, &bad);
            snprintf(nm, sizeof nm, "%s2.alpha", rp);
            const float* a2 = cget(m, nm, Cout, &bad);
            if (bad) break;
            memcpy(t1, x, sizeof(float) * (size_t)Cout * L);
            snake(t1, a0, Cout, L);
            char cp[220];
            snprintf(cp, sizeof cp, "%s1.", rp);
            if (wn_conv(m, cp, t1, Cout, L, Cout, 7, dils[r], t2)) { bad = 1; break; }
            snake(t2, a2, Cout, L);
            snprintf(cp, sizeof cp, "%s3.", rp);
            if (wn_conv(m, cp, t2, Cout, L, Cout, 1, 1, t1)) { bad = 1; break; }
            for (size_t i = 0; i < (size_t)Cout * L; ++i) x[i] += t1[i];
        }
        free(t1); free(t2);
        if (bad) { free(x); return -1; }
        Cin = Cout;
    }
    snprintf(nm, sizeof nm, "decoder.model.5.alpha");
    const float* af = cget(m, nm, Cin, &bad);
    if (bad) { free(x); return -1; }
    snake(x, af, Cin, L);
    if (wn_conv(m, "decoder.model.6.", x, Cin, L, 1, 7, 1, wave)) { free(x); return -1; }
    for (int t = 0; t < L; ++t) wave[t] = tanhf(wave[t]);
    free(x);
    return L;
}

/* ------------------------------------------------------------------------------------ */
/* single-op entry points (pinned by tests/golden/ops.npz)                              */
/* ------------------------------------------------------------------------------------ */
int orc_op_rmsnorm(const float* x, const float* w, int rows, int n, float eps, int bf16, float* y) {
    orc_llm tmp;
    memset(&tmp, 0, sizeof tmp);
    tmp.bf16 = bf16;
    tmp.c.norm_eps = eps;
    tensor_t tw;
    memset(&tw, 0, sizeof tw);
    tw.f = (float*)w;
    for (int r = 0; r < rows; ++r) rmsnorm(&tmp, x + (size_t)r * n, &tw, n, y + (size_t)r * n);
    return 0;
}
int orc_op_headnorm(const float* x, const float* w, int rows, int n, float eps, int bf16, float* y) {
    orc_llm tmp;
    memset(&tmp, 0, sizeof tmp);
    tmp.bf16 = bf16;
    tmp.c.norm_eps = eps;
    tensor_t tw;
    memset(&tw, 0, sizeof tw);
    tw.f = (float*)w;
    memcpy(y, x, sizeof(float) * (size_t)rows * n);
    for (int r = 0; r < rows; ++r) headnorm(&tmp, y + (size_t)r * n, &tw, n);
    return 0;
}
/* table: [S][hd/2][2] as produced by rope_table (bf16 values) */
int orc_op_rope_table(int S, int hd, float base, float* tab) {
    rope_table(tab, S, hd, base);
    return 0;
}
int orc_op_rope(const float* x, const float* tab_rows /* rows x hd */, int rows, int hd, int bf16,
                float* y) {
    orc_llm tmp;
    memset(&tmp, 0, sizeof tmp);
    tmp.bf16 = bf16;
    memcpy(y, x, sizeof(float) * (size_t)rows * hd);
    for (int r = 0; r < rows; ++r) rope(&tmp, y + (size_t)r * hd, tab_rows + (size_t)r * hd, hd);
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* Codec ENCODE (fp32): DAC.encode (modded_dac.py:874-923)                              */
/* ------------------------------------------------------------------------------------ */
/* causal strided conv (CausalConvNet, modded_dac.py:59-90): left pad k - s, L % s == 0 (so no
   extra right pad), Lo = L / s.  w [Co][Ci][k]; y [Co][Lo] */
static void conv1d_causal_strided(const float* x, int Ci, int L, const float* w, const float* b, int Co,
                                  int k, int s, float* y) {
    const int Lo = L / s, pad = k - s;
#pragma omp parallel for schedule(static)
    for (int co = 0; co < Co; ++co) {
        float* yr = y + (size_t)co * Lo;
        for (int t = 0; t < Lo; ++t) yr[t] = b ? b[co] : 0.f;
        for (int ci = 0; ci < Ci; ++ci) {
            const float* xr = x + (size_t)ci * L;
            const float* wr = w + ((size_t)co * Ci + ci) * k;
            for (int t = 0; t < Lo; ++t)
                for (int j = 0; j < k; ++j) {
                    int src = t * s + j - pad;
                    if (src >= 0) yr[t] += wr[j] * xr[src];
                }
        }
    }
}

static int wn_conv_strided(orc_codec* m, const char* pre, const float* x, int Ci, int L, int Co, int k,
                           int s, float* y) {
    int bad = 0;
    char nm[220];
    snprintf(nm, sizeof nm, "%sconv.parametrizations.weight.original0", pre);
    const float* g = cget(m, nm, Co, &bad);
    snprintf(nm, sizeof nm, "%sconv.parametrizations.weight.original1", pre);
    const float* v = cget(m, nm, (int64_t)Co * Ci * k, &bad);
    snprintf(nm, sizeof nm, "%sconv.bias", pre);
    const float* b = cget(m, nm, Co, &bad);
    if (bad) return -1;
    float* w = wn_fold(g, v, Co, Ci * k);
    conv1d_causal_strided(x, Ci, L, w, b, Co, k, s, y);
    free(w);
    return 0;
}

/* ResidualUnit (modded_dac.py:600-620), causal: x += conv1(snake(conv7_dil(snake(x)))) */
static int residual_unit(orc_codec* m, const char* pre, float* x, int C, int L, int dil) {
    int bad = 0;
    char nm[220];
    snprintf(nm, sizeof nm, "%s0.alpha", pre);
    const float* a0 = cget(m, nm, C, &bad);
    snprintf(nm, sizeof nm, "%s2.alpha", pre);
    const float* a2 = cget(m, nm, C, &bad);
    if (bad) return -1;
    float* t = (float*)malloc(sizeof(float) * (size_t)C * L);
    float* u = (float*)malloc(sizeof(float) * (size_t)C * L);
    memcpy(t, x, sizeof(float) * (size_t)C * L);
    snake(t, a0, C, L);
    snprintf(nm, sizeof nm, "%s1.", pre);
    int rc = wn_conv(m, nm, t, C, L, C, 7, dil, u);
    if (!rc) {
        snake(u, a2, C, L);
        snprintf(nm, sizeof nm, "%s3.", pre);
        rc = wn_conv(m, nm, u, C, L, C, 1, 1, t);
    }
    if (!rc)
        for (size_t i = 0; i < (size_t)C * L; ++i) x[i] += t[i];
    free(t); free(u);
    return rc;
}

/* [C][L] <-> [L][C] */
static float* transpose_cl(const float* x, int C, int L) {
    float* y = (float*)malloc(sizeof(float) * (size_t)C * L);
    for (int c = 0; c < C; ++c)
        for (int t = 0; t < L; ++t) y[(size_t)t * C + c] = x[(size_t)c * L + t];
    return y;
}

/* descript 1.0.0 VectorQuantize.forward (restated, eval): z_e = in_proj(r); nearest codebook
   entry of the l2-normalised z_e among the l2-normalised codebook (argmax of -dist, first
   index on ties, dist = |e|^2 - 2 e.c + |c|^2); z_q = z_e + (codebook[idx] - z_e);
   out = out_proj(z_q).  r, out: [D][T]. */
static int vq_stage(orc_codec* m, const char* pre, int cbn, const float* r, int T, int32_t* codes, float* out) {
    const int D = m->c.latent, cd = m->c.codebook_dim;
    int bad = 0;
    char nm[220];
#define QW(var, suffix, cnt) \
    snprintf(nm, sizeof nm, "%s%s", pre, suffix); const float* var = cget(m, nm, cnt, &bad);
    QW(ig, "in_proj.weight_g", cd);
    QW(iv, "in_proj.weight_v", (int64_t)cd * D);
    QW(ib, "in_proj.bias", cd);
    QW(og, "out_proj.weight_g", D);
    QW(ov, "out_proj.weight_v", (int64_t)D * cd);
    QW(ob, "out_proj.bias", D);
    QW(cbw, "codebook.weight", (int64_t)cbn * cd);
#undef QW
    if (bad) return -1;
    float* wi = wn_fold(ig, iv, cd, D);
    float* wo = wn_fold(og, ov, D, cd);
    float* cn = (float*)malloc(sizeof(float) * (size_t)cbn * cd);
    float* cn2 = (float*)malloc(sizeof(float) * cbn);
    for (int i = 0; i < cbn; ++i) {
        float ss = 0.f;
        for (int j = 0; j < cd; ++j) ss += cbw[(size_t)i * cd + j] * cbw[(size_t)i * cd + j];
        float nrm = sqrtf(ss);
        if (nrm < 1e-12f) nrm = 1e-12f;
        float s2 = 0.f;
        for (int j = 0; j < cd; ++j) {
            cn[(size_t)i * cd + j] = cbw[(size_t)i * cd + j] / nrm;
            s2 += cn[(size_t)i * cd + j] * cn[(size_t)i * cd + j];
        }
        cn2[i] = s2;
    }
#pragma omp parallel for schedule(static)
    for (int t = 0; t < T; ++t) {
        float ze[64], en[64], zq[64];
        for (int j = 0; j < cd; ++j) {
            float acc = 0.f;
            for (int d = 0; d < D; ++d) acc += wi[(size_t)j * D + d] * r[(size_t)d * T + t];
            ze[j] = acc + ib[j];
        }
        float ss = 0.f;
        for (int j = 0; j < cd; ++j) ss += ze[j] * ze[j];
        float nrm = sqrtf(ss);
        if (nrm < 1e-12f) nrm = 1e-12f;
        float e2 = 0.f;
        for (int j = 0; j < cd; ++j) { en[j] = ze[j] / nrm; e2 += en[j] * en[j]; }
        int best = 0;
        float bv = -INFINITY;
        for (int i = 0; i < cbn; ++i) {
            float dot = 0.f;
            for (int j = 0; j < cd; ++j) dot += en[j] * cn[(size_t)i * cd + j];
            float nd = -((e2 - 2.f * dot) + cn2[i]);
            if (nd > bv) { bv = nd; best = i; }
        }
        codes[t] = best;
        for (int j = 0; j < cd; ++j) zq[j] = ze[j] + (cbw[(size_t)best * cd + j] - ze[j]);
        for (int d = 0; d < D; ++d) {
            float acc = 0.f;
            for (int j = 0; j < cd; ++j) acc += wo[(size_t)d * cd + j] * zq[j];
            out[(size_t)d * T + t] = acc + ob[d];
        }
    }
    free(wi); free(wo); free(cn); free(cn2);
    return 0;
}

/* DAC.encode: audio (n samples, mono) right-padded to a multiple of 2048 (modded_dac.py:
   906-909); Encoder (modded_dac.py:670-709, strides 2/4/8/8, transformer of enc_layers layers
   in the last block with window enc_window); quantizer: downsample x2 x2 (rvq.py:250-262),
   pre_module (window c->window), semantic VQ then 9 residual VQ stages on z - semantic_z
   (rvq.py:293-315).  codes: (nq+1) x T row-major with T = ceil(n / 2048).  Optional taps:
   z_enc [D][4T], z_pre [D][T].  Returns T or -1. */
int orc_codec_encode(orc_codec* m, const float* audio, int n, int encoder_dim, int enc_layers,
                     int enc_window, int32_t* codes, float* z_enc_out, float* z_pre_out) {
    const orc_codec_config* c = &m->c;
    const int D = c->latent, nq = c->n_codebooks;
    const int rates[4] = {2, 4, 8, 8};
    const int T = (n + 2047) / 2048, L0 = T * 2048;
    char nm[220];
    float* x = (float*)calloc((size_t)L0, sizeof(float));
    memcpy(x, audio, sizeof(float) * (size_t)n);
    float* y = (float*)malloc(sizeof(float) * (size_t)encoder_dim * L0);
    if (wn_conv(m, "encoder.block.0.", x, 1, L0, encoder_dim, 7, 1, y)) { free(x); free(y); return -1; }
    free(x);
    x = y;
    int d = encoder_dim, L = L0;
    for (int b = 0; b < 4; ++b) {
        const int h = d, s = rates[b];
        d *= 2;
        char pre[160];
        const int dils[3] = {1, 3, 9};
        for (int r = 0; r < 3; ++r) {
            snprintf(pre, sizeof pre, "encoder.block.%d.block.%d.block.", b + 1, r);
            if (residual_unit(m, pre, x, h, L, dils[r])) { free(x); return -1; }
        }
        int bad = 0;
        snprintf(nm, sizeof nm, "encoder.block.%d.block.3.alpha", b + 1);
        const float* al = cget(m, nm, h, &bad);
        if (bad) { free(x); return -1; }
        snake(x, al, h, L);
        y = (float*)malloc(sizeof(float) * (size_t)d * (L / s));
        snprintf(pre, sizeof pre, "encoder.block.%d.block.4.", b + 1);
        if (wn_conv_strided(m, pre, x, h, L, d, 2 * s, s, y)) { free(x); free(y); return -1; }
        free(x);
        x = y;
        L /= s;
        if (b == 3 && enc_layers > 0) {
            float* xt = transpose_cl(x, d, L);
            snprintf(pre, sizeof pre, "encoder.block.%d.block.5.", b + 1);
            if (window_transformer_at(m, pre, xt, L, d, d / 64, 64, 3 * d, enc_layers, enc_window)) {
                free(xt); free(x); return -1;
            }
            free(x);
            x = transpose_cl(xt, L, d);
            free(xt);
        }
    }
    {
        int bad = 0;
        const float* al = cget(m, "encoder.block.5.alpha", d, &bad);
        if (bad) { free(x); return -1; }
        snake(x, al, d, L);
        y = (float*)malloc(sizeof(float) * (size_t)D * L);
        if (wn_conv(m, "encoder.block.6.", x, d, L, D, 3, 1, y)) { free(x); free(y); return -1; }
        free(x);
        x = y;
    }
    if (z_enc_out) memcpy(z_enc_out, x, sizeof(float) * (size_t)D * L);
    /* quantizer.downsample: CausalConvNet(k=2, s=2) + ConvNeXtBlock, twice */
    for (int i = 0; i < 2; ++i) {
        int bad = 0;
        snprintf(nm, sizeof nm, "quantizer.downsample.%d.0.conv.weight", i);
        const float* w = cget(m, nm, (int64_t)D * D * 2, &bad);
        snprintf(nm, sizeof nm, "quantizer.downsample.%d.0.conv.bias", i);
        const float* b = cget(m, nm, D, &bad);
        if (bad) { free(x); return -1; }
        y = (float*)malloc(sizeof(float) * (size_t)D * (L / 2));
        conv1d_causal_strided(x, D, L, w, b, D, 2, 2, y);
        free(x);
        x = y;
        L /= 2;
        snprintf(nm, sizeof nm, "quantizer.downsample.%d.1.", i);
        if (convnext(m, nm, x, D, L)) { free(x); return -1; }
    }
    {
        float* xt = transpose_cl(x, D, L);
        if (window_transformer_at(m, "quantizer.pre_module.", xt, L, D, c->t_heads, c->t_head_dim, c->t_inter,
                                  c->t_layers, c->window)) {
            free(xt); free(x); return -1;
        }
        free(x);
        x = transpose_cl(xt, L, D);
        free(xt);
    }
    if (z_pre_out) memcpy(z_pre_out, x, sizeof(float) * (size_t)D * L);
    /* semantic stage on z, then the residual stages on z - semantic_z */
    float* q = (float*)malloc(sizeof(float) * (size_t)D * L);
    int rc = vq_stage(m, "quantizer.semantic_quantizer.quantizers.0.", c->semantic_codebook_size, x, L, codes, q);
    for (size_t i = 0; !rc && i < (size_t)D * L; ++i) x[i] -= q[i];
    for (int k = 0; !rc && k < nq; ++k) {
        char pre[160];
        snprintf(pre, sizeof pre, "quantizer.quantizer.quantizers.%d.", k);
        rc = vq_stage(m, pre, c->codebook_size, x, L, codes + (size_t)(k + 1) * L, q);
        for (size_t i = 0; !rc && i < (size_t)D * L; ++i) x[i] -= q[i];
    }
    free(q); free(x);
    return rc ? -1 : T;
}

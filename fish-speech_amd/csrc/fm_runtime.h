// fm_runtime.h -- host-side helpers shared by the LLM and codec runtimes of libfishmi.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <functional>
#include <map>
#include <string>
#include <vector>

#include "fishmi.h"

struct FmError {
    int code;
    std::string msg;
};

#define HIPCHK(x)                                                                             \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess)                                                                 \
            throw FmError{FM_ERR_HIP, std::string(#x) + " -> " + hipGetErrorString(e_)};      \
    } while (0)

#define FMCHECK(cond, msg)                                                          \
    do {                                                                            \
        if (!(cond)) throw FmError{FM_ERR_ARG, std::string(msg)};                   \
    } while (0)

void fm_set_error(const std::string& s);

template <typename F> int fm_guard(F&& f) {
    try {
        f();
        return FM_OK;
    } catch (const FmError& e) {
        fm_set_error(e.msg);
        return e.code;
    } catch (const std::exception& e) {
        fm_set_error(e.what());
        return FM_ERR_STATE;
    }
}

inline uint32_t fnv1a32(const char* s) {
    uint32_t h = 0x811C9DC5u;
    for (; *s; ++s) {
        h ^= (uint8_t)*s;
        h *= 0x01000193u;
    }
    return h;
}

inline float host_bf16_round(float x) {
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

// RoPE table exactly like llama.py:1003-1022 / modded_dac.py:442-452: fp32 freqs, fp32 angle,
// (cos, sin) cast to bf16.  [S][hd/2][2] floats.
inline std::vector<float> rope_table_host(int S, int hd, float base) {
    std::vector<float> t((size_t)S * hd);
    const int half = hd / 2;
    for (int i = 0; i < half; ++i) {
        const float e = (float)(2 * i) / (float)hd;
        const float freq = 1.0f / powf(base, e);
        for (int p = 0; p < S; ++p) {
            const float ang = (float)p * freq;
            t[((size_t)p * half + i) * 2] = host_bf16_round(cosf(ang));
            t[((size_t)p * half + i) * 2 + 1] = host_bf16_round(sinf(ang));
        }
    }
    return t;
}

// device tensor registry entry
struct DTensor {
    void* p = nullptr;
    int64_t numel = 0;      // logical elements
    int64_t rows = 0, cols = 0;  // 2-D view (rows padded to 16 in the allocation)
    bool set = false;
    bool optional = false;  // may stay unset (int8 mode: scales of float weights, dropped biases)
    void* q = nullptr;      // int8 mode: row-major int8 values [rows padded to 16][cols]
    void* s = nullptr;      //            per-row scales (storage type) [rows padded to 16]
};

// simple per-class profiler on HIP events (the stream the kernels run on)
struct Profiler {
    bool on = false;
    struct Pending {
        std::string cls;
        hipEvent_t a, b;
        int64_t bytes;
        double flops;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    struct Acc {
        double ms = 0;
        int64_t n = 0, bytes = 0;
        double flops = 0;
    };
    std::map<std::string, Acc> acc;
    // launch recording for kernel-class replay timing (fm_llm_kernel_bench)
    std::string rec_cls;
    std::vector<std::function<void()>> rec;
    std::vector<int64_t> rec_bytes;
    template <typename F> void record(const char* cls, int64_t bytes, const F& f) {
        if (!rec_cls.empty() && rec_cls == cls) {
            rec.emplace_back(f);
            rec_bytes.push_back(bytes);
        }
    }
    hipEvent_t get() {
        if (pool.empty()) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            return e;
        }
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    // FISHMI_SYNC_DEBUG=1 (with FISHMI_GRAPH=0): synchronise after every launch and name the class
    // of the first one that fails -- a developer aid for locating a device fault
    int sync_debug = -1;
    template <typename F> void run(hipStream_t s, const char* cls, int64_t bytes, double flops, F&& f) {
        if (sync_debug < 0) {
            const char* e = getenv("FISHMI_SYNC_DEBUG");
            sync_debug = e && e[0] == '1';
        }
        if (sync_debug) {
            f();
            const hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) {
                fprintf(stderr, "FISHMI_SYNC_DEBUG: launch of class '%s' failed: %s\n", cls, hipGetErrorString(e));
                fflush(stderr);
                throw FmError{FM_ERR_HIP, std::string("device fault in class ") + cls};
            }
            return;
        }
        if (!on) {
            f();
            return;
        }
        Pending p{cls, get(), get(), bytes, flops};
        HIPCHK(hipEventRecord(p.a, s));
        f();
        HIPCHK(hipEventRecord(p.b, s));
        pending.push_back(p);
    }
    void collect() {
        for (auto& p : pending) {
            HIPCHK(hipEventSynchronize(p.b));
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
            Acc& a = acc[p.cls];
            a.ms += ms;
            a.n += 1;
            a.bytes += p.bytes;
            a.flops += p.flops;
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.clear();
    }
    ~Profiler() {
        for (auto& e : pool) (void)hipEventDestroy(e);
    }
};

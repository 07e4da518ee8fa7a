// Probe: does hipExtAnyOrderLaunch let a kernel start before its stream predecessor ends on gfx950?
// Kernel A (1 block) polls a flag for at most ~1 ms (bounded by s_memrealtime, 100 MHz);
// kernel B (1 block), launched after A on the SAME stream, sets the flag. If B starts while A runs,
// A sees the flag early; otherwise A times out and B runs after it. Every wait is bounded.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/anyorder_probe scripts/anyorder_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

__global__ void kA(unsigned *flag, unsigned long long *rec, unsigned long long limit) {
  if (threadIdx.x != 0) return;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  unsigned seen = 0;
  while (t - t0 < limit) {
    seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (seen) break;
    __builtin_amdgcn_s_sleep(2);
    t = __builtin_amdgcn_s_memrealtime();
  }
  rec[0] = t0;
  rec[1] = t;
  rec[2] = seen;
}

__global__ void kB(unsigned *flag, unsigned long long *rec) {
  if (threadIdx.x != 0) return;
  rec[3] = __builtin_amdgcn_s_memrealtime();
  __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A chain of dependent "work" kernels to time boundaries: each spins a fixed ~t_ns then stamps.
__global__ void kWork(unsigned long long *rec, int idx, unsigned long long ticks) {
  if (threadIdx.x != 0) return;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  rec[2 * idx] = t0;
  rec[2 * idx + 1] = __builtin_amdgcn_s_memrealtime();
}

static int run(const char *name, hipStream_t s, unsigned *flag, unsigned long long *rec,
               unsigned flagsA, unsigned flagsB, bool graph) {
  CK(hipMemsetAsync(flag, 0, 4, s));
  CK(hipMemsetAsync(rec, 0, 64, s));
  CK(hipStreamSynchronize(s));
  unsigned long long limit = 100000;  // 1 ms at 100 MHz
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  if (graph) CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  hipExtLaunchKernelGGL(kA, dim3(1), dim3(64), 0, s, nullptr, nullptr, flagsA, flag, rec, limit);
  hipExtLaunchKernelGGL(kB, dim3(1), dim3(64), 0, s, nullptr, nullptr, flagsB, flag, rec);
  if (graph) {
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
  }
  CK(hipStreamSynchronize(s));
  unsigned long long h[4];
  CK(hipMemcpy(h, rec, sizeof(h), hipMemcpyDeviceToHost));
  printf("%-40s A waited %8.2f us, saw flag %llu, B start - A start %+9.2f us\n", name,
         (h[1] - h[0]) / 100.0, h[2], ((long long)h[3] - (long long)h[0]) / 100.0);
  if (ge) CK(hipGraphExecDestroy(ge));
  if (g) CK(hipGraphDestroy(g));
  return 0;
}


static int run2(const char *name, hipStream_t s, hipStream_t s2, unsigned *flag, unsigned long long *rec,
                bool graph) {
  CK(hipMemsetAsync(flag, 0, 4, s));
  CK(hipMemsetAsync(rec, 0, 64, s));
  CK(hipStreamSynchronize(s));
  unsigned long long limit = 100000;
  hipEvent_t e1, e2;
  CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  if (graph) CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  CK(hipEventRecord(e1, s));
  CK(hipStreamWaitEvent(s2, e1, 0));
  hipLaunchKernelGGL(kA, dim3(1), dim3(64), 0, s, flag, rec, limit);
  hipLaunchKernelGGL(kB, dim3(1), dim3(64), 0, s2, flag, rec);
  CK(hipEventRecord(e2, s2));
  CK(hipStreamWaitEvent(s, e2, 0));
  if (graph) {
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 2; ++r) {
      CK(hipMemsetAsync(flag, 0, 4, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
    }
  }
  CK(hipStreamSynchronize(s));
  unsigned long long h[4];
  CK(hipMemcpy(h, rec, sizeof(h), hipMemcpyDeviceToHost));
  printf("%-40s A waited %8.2f us, saw flag %llu, B start - A start %+9.2f us\n", name,
         (h[1] - h[0]) / 100.0, h[2], ((long long)h[3] - (long long)h[0]) / 100.0);
  if (ge) CK(hipGraphExecDestroy(ge));
  if (g) CK(hipGraphDestroy(g));
  return 0;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned *flag;
  unsigned long long *rec;
  CK(hipMalloc(&flag, 256));
  CK(hipMalloc(&rec, 4096));
  for (int rep = 0; rep < 2; ++rep) {
    if (run("eager, normal launches", s, flag, rec, 0, 0, false)) return 1;
    if (run("eager, B any-order", s, flag, rec, 0, hipExtAnyOrderLaunch, false)) return 1;
    if (run("eager, A and B any-order", s, flag, rec, hipExtAnyOrderLaunch, hipExtAnyOrderLaunch,
            false)) return 1;
    if (run("graph, B any-order", s, flag, rec, 0, hipExtAnyOrderLaunch, true)) return 1;
    if (run("graph, A and B any-order", s, flag, rec, hipExtAnyOrderLaunch, hipExtAnyOrderLaunch,
            true)) return 1;
  }
  hipStream_t s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  for (int rep = 0; rep < 2; ++rep) {
    if (run2("eager, two streams", s, s2, flag, rec, false)) return 1;
    if (run2("graph, two branches", s, s2, flag, rec, true)) return 1;
  }
  // Boundary timing: 8 dependent 5-us kernels, normal launches.
  for (int mode = 0; mode < 2; ++mode) {
    CK(hipMemsetAsync(rec, 0, 4096, s));
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < 8; ++i)
      hipExtLaunchKernelGGL(kWork, dim3(1), dim3(64), 0, s, nullptr, nullptr,
                            mode ? hipExtAnyOrderLaunch : 0, rec, i, 500ull);
    CK(hipStreamSynchronize(s));
    unsigned long long h[16];
    CK(hipMemcpy(h, rec, sizeof(h), hipMemcpyDeviceToHost));
    printf("work chain (%s): start offsets us:", mode ? "any-order" : "normal");
    for (int i = 0; i < 8; ++i) printf(" %.2f", ((long long)h[2 * i] - (long long)h[0]) / 100.0);
    printf("\n");
  }
  printf("done\n");
  return 0;
}

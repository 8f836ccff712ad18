// Does a captured HIP graph run a forked branch concurrently?  Two kernels
// that each hold one workgroup for ~spin_us, captured (a) in one stream and
// (b) forked onto a second stream and joined; graph replay time of each.
// Build: hipcc --offload-arch=gfx950 -O2 tools/graph_fork_probe.hip -o /tmp/gfp
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void spin(unsigned long long cycles, unsigned* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < cycles) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

int main() {
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  unsigned* out;
  CK(hipMalloc(&out, 4096));
  const unsigned long long cyc = 100ull * 50;  // memrealtime runs at 100 MHz: 50 us
  hipEvent_t fork, join, a, b;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int mode = 0; mode < 2; mode++) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
    spin<<<1, 64, 0, s0>>>(cyc / 5, out);  // a short head
    if (mode == 1) {
      CK(hipEventRecord(fork, s0));
      CK(hipStreamWaitEvent(s1, fork, 0));
      spin<<<1, 64, 0, s1>>>(cyc, out + 64);
      CK(hipEventRecord(join, s1));
      spin<<<1, 64, 0, s0>>>(cyc, out + 128);
      CK(hipStreamWaitEvent(s0, join, 0));
    } else {
      spin<<<1, 64, 0, s0>>>(cyc, out + 64);
      spin<<<1, 64, 0, s0>>>(cyc, out + 128);
    }
    spin<<<1, 64, 0, s0>>>(cyc / 5, out + 192);  // a short tail
    CK(hipStreamEndCapture(s0, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; w++) CK(hipGraphLaunch(ge, s0));
    CK(hipStreamSynchronize(s0));
    const int R = 20;
    CK(hipEventRecord(a, s0));
    for (int r = 0; r < R; r++) CK(hipGraphLaunch(ge, s0));
    CK(hipEventRecord(b, s0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%s: %.1f us per replay (serial would be ~120, concurrent ~70)\n",
           mode ? "forked" : "one stream", 1000.f * ms / R);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}

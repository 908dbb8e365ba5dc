// which part of lu_factor_blocks' fork / join makes hipStreamEndCapture (or the
// instantiation after it) crash under HIP 7.2?  The LU's pattern rebuilt with a trivial kernel, one
// variant per process (argv[1]); tools/gpu_r06c.sh runs them in order from the simplest and stops at
// the first that fails, so the first failing variant names the ingredient.
//
//   1  s0 -> s1 by event, kernels on s1, s1 -> s0 by event                       (plain fork / join)
//   2  1 + per block a second fork s1 -> s2, a kernel on s2, s2's join event waited by s1 next block
//   3  2 with the streams made by hipStreamCreateWithPriority (highest / lowest) as the LU context does
//   4  3 with the events made hipEventDisableTiming, reused every block (the LU context's events)
//   5  4 with the LU's last-block form: the final s2 join waited by s1 after the loop, then s1 -> s0
//   6  5 with the streams and events made once and reused for a second capture (warm-up call before)
//   7  6 with s2's join waited on s1 only after s1 forks the next s2 launch (not the LU's order: a check)
//   8  6 with 80 KB of dynamic LDS per kernel and hipFuncSetAttribute called inside the capture, as
//      lu_factor_blocks does (IADMM_ALLOW_LDS at the top of every call)
//   9  the batch split's shape: s0 forks s1 and s2 by one event, kernels on both, both joined into s0
//  10  the r06 look-ahead under capture: the critical path stays on s0, and every block forks s2 from
//      s0 (kernel on s2, its join waited by s0 at the next block), as 5 without the s0 -> s1 hop
// Finding (gpurun r06f): on torch's bundled HIP runtime (ROCm 7.0.2) variant 1 captures and variant 2
// crashes in hipStreamEndCapture -- a fork from a stream that joined the capture through another
// forked stream; on the system HIP 7.2 runtime all of 1-8 capture, instantiate and replay.
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/capture_probe.hip -o /tmp/capture_probe  (system HIP 7.2, via
// the binary's RPATH), or with -shared -fPIC -DPROBE_LIB into a library that tools/capture_probe_torch.py
// loads into a python process after torch: it then runs on torch's bundled HIP runtime (ROCm 7.0.2),
// the one libiadmm.so binds to in every python caller (same soname, loaded first).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                       \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) {                                                                         \
      std::printf("variant %d: %s failed: %s (line %d)\n", variant, #x, hipGetErrorString(e_), __LINE__); \
      return 1;                                                                                     \
    }                                                                                               \
  } while (0)

__global__ void bump(float* a, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = a[i] * 0.5f + v;
}

__global__ void bump_lds(float* a, int n, float v) {
  extern __shared__ float sh[];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  sh[threadIdx.x] = v;
  __syncthreads();
  if (i < n) a[i] = a[i] * 0.5f + sh[(threadIdx.x + 1) & 255];
}

static int variant = 0;

static void launch(hipStream_t s, float* a, int n, float v) {
  const dim3 g((n + 255) / 256), t(256);
  if (variant >= 8) hipLaunchKernelGGL(bump_lds, g, t, 80 * 1024, s, a, n, v);
  else hipLaunchKernelGGL(bump, g, t, 0, s, a, n, v);
}

struct Ctx {
  hipStream_t s1 = nullptr, s2 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr, ev0 = nullptr, ev1 = nullptr;
};

static int make_ctx(Ctx& c) {
  if (variant >= 3 && variant <= 8) {
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    CK(hipStreamCreateWithPriority(&c.s1, hipStreamNonBlocking, greatest));
    CK(hipStreamCreateWithPriority(&c.s2, hipStreamNonBlocking, least));
  } else {
    CK(hipStreamCreateWithFlags(&c.s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&c.s2, hipStreamNonBlocking));
  }
  hipEvent_t* evs[4] = {&c.fork, &c.join, &c.ev0, &c.ev1};
  for (auto* e : evs) CK(variant >= 4 ? hipEventCreateWithFlags(e, hipEventDisableTiming) : hipEventCreate(e));
  if (variant >= 9) {  // the LU context's priority streams
    CK(hipStreamDestroy(c.s1));
    CK(hipStreamDestroy(c.s2));
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    CK(hipStreamCreateWithPriority(&c.s1, hipStreamNonBlocking, greatest));
    CK(hipStreamCreateWithPriority(&c.s2, hipStreamNonBlocking, least));
  }
  return 0;
}

// The factorization's stream pattern over nb blocks on buffers a (critical path) and b (side work).
static int pattern(const Ctx& c, hipStream_t s0, float* a, float* b, int n, int nb) {
  if (variant == 9) {
    CK(hipEventRecord(c.ev0, s0));
    CK(hipStreamWaitEvent(c.s1, c.ev0, 0));
    CK(hipStreamWaitEvent(c.s2, c.ev0, 0));
    for (int k = 0; k < nb; ++k) {
      launch(c.s1, a, n, (float)k);
      launch(c.s2, b, n, (float)k);
    }
    CK(hipGetLastError());
    CK(hipEventRecord(c.ev1, c.s1));
    CK(hipStreamWaitEvent(s0, c.ev1, 0));
    CK(hipEventRecord(c.join, c.s2));
    CK(hipStreamWaitEvent(s0, c.join, 0));
    return 0;
  }
  if (variant == 10) {
    bool pending = false;
    for (int k = 0; k < nb; ++k) {
      launch(s0, a, n, (float)k);
      if (pending) {
        CK(hipStreamWaitEvent(s0, c.join, 0));
        pending = false;
      }
      if (k + 1 < nb) {
        CK(hipEventRecord(c.fork, s0));
        CK(hipStreamWaitEvent(c.s2, c.fork, 0));
        launch(c.s2, b, n, (float)k);
        CK(hipEventRecord(c.join, c.s2));
        pending = true;
      }
      CK(hipGetLastError());
    }
    if (pending) CK(hipStreamWaitEvent(s0, c.join, 0));
    return 0;
  }
  if (variant >= 8) CK(hipFuncSetAttribute((const void*)bump_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024));
  CK(hipEventRecord(c.ev0, s0));
  CK(hipStreamWaitEvent(c.s1, c.ev0, 0));
  hipStream_t s = c.s1;
  bool pending = false;
  for (int k = 0; k < nb; ++k) {
    launch(s, a, n, (float)k);
    CK(hipGetLastError());
    if (variant >= 2 && k + 1 < nb) {
      if (pending && variant < 7) {
        CK(hipStreamWaitEvent(s, c.join, 0));
        pending = false;
      }
      CK(hipEventRecord(c.fork, s));
      CK(hipStreamWaitEvent(c.s2, c.fork, 0));
      launch(c.s2, b, n, (float)k);
      CK(hipGetLastError());
      if (pending && variant >= 7) {  // the previous side launch joined only now (after the re-record
        CK(hipStreamWaitEvent(s, c.join, 0));  //  of `fork`): the event it waits for is re-recorded below
        pending = false;
      }
      CK(hipEventRecord(c.join, c.s2));
      pending = true;
      if (variant < 5) {  // join at once
        CK(hipStreamWaitEvent(s, c.join, 0));
        pending = false;
      }
    }
  }
  if (pending) CK(hipStreamWaitEvent(s, c.join, 0));
  CK(hipEventRecord(c.ev1, s));
  CK(hipStreamWaitEvent(s0, c.ev1, 0));
  return 0;
}

extern "C" int capture_probe_run(int v) {
  variant = v;
  const int n = 1 << 16, nb = 20;
  float *a = nullptr, *b = nullptr;
  CK(hipMalloc(&a, n * sizeof(float)));
  CK(hipMalloc(&b, n * sizeof(float)));
  CK(hipMemset(a, 0, n * sizeof(float)));
  CK(hipMemset(b, 0, n * sizeof(float)));
  hipStream_t s0;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  Ctx c;
  if (make_ctx(c)) return 1;
  if (variant >= 6 && pattern(c, s0, a, b, n, nb)) return 1;  // eager warm-up with the same objects (6-10)
  CK(hipStreamSynchronize(s0));
  std::printf("variant %d: begin capture\n", variant);
  std::fflush(stdout);
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
  if (pattern(c, s0, a, b, n, nb)) return 1;
  hipGraph_t graph = nullptr;
  std::printf("variant %d: end capture\n", variant);
  std::fflush(stdout);
  CK(hipStreamEndCapture(s0, &graph));
  size_t nodes = 0;
  CK(hipGraphGetNodes(graph, nullptr, &nodes));
  std::printf("variant %d: captured %zu nodes; instantiate\n", variant, nodes);
  std::fflush(stdout);
  hipGraphExec_t exec = nullptr;
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  CK(hipGraphLaunch(exec, s0));
  CK(hipStreamSynchronize(s0));
  std::printf("variant %d: ok\n", variant);
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
  return 0;
}

#ifndef PROBE_LIB
int main(int argc, char** argv) { return capture_probe_run(argc > 1 ? std::atoi(argv[1]) : 1); }
#endif

// Process-level cost of the HIP runtime on the GPU box (diagnostics for the
// s2-porcupine CLI's latency): run with a mode, time the whole process from
// the parent (tools/startup/run.py).
//   0: no HIP call   1: hipGetDeviceCount   2: + stream   3: + 2 GiB hipMalloc
//   4: + a kernel launch   each prints its in-main phases (ms)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <unistd.h>

static double now_ms() {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return 1e3 * t.tv_sec + 1e-6 * t.tv_nsec;
}
__global__ void nop(int* p) { if (p && threadIdx.x == 1234567) p[0] = 1; }

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const bool fast_exit = argc > 2 && atoi(argv[2]) == 1;
  const double t0 = now_ms();
  double t1 = t0, t2 = t0, t3 = t0, t4 = t0;
  int n = 0;
  hipStream_t s = nullptr;
  void* p = nullptr;
  if (mode >= 1) { if (hipGetDeviceCount(&n) != hipSuccess) return 2; t1 = now_ms(); }
  if (mode >= 2) { if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 3; t2 = now_ms(); }
  if (mode >= 3) { if (hipMalloc(&p, 2ull << 30) != hipSuccess) return 4; t3 = now_ms(); }
  if (mode >= 4) {
    hipLaunchKernelGGL(nop, dim3(1), dim3(64), 0, s, (int*)p);
    if (hipStreamSynchronize(s) != hipSuccess) return 5;
    t4 = now_ms();
  }
  printf("{\"mode\":%d,\"init\":%.2f,\"stream\":%.2f,\"malloc\":%.2f,\"kernel\":%.2f,\"main\":%.2f}\n", mode, t1 - t0,
         t2 - t1, t3 - t2, t4 - t3, now_ms() - t0);
  fflush(stdout);
  if (fast_exit) _exit(0);
  return 0;
}

// Cost of the level search's first allocation on a fresh process (diagnostics):
// hipMalloc of two staging arrays of `gib` GiB each, then a 0xFF memset of two
// 512 MiB tables, then a kernel that touches one byte per 2 MiB of the arrays.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

static double now_ms() {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return 1e3 * t.tv_sec + 1e-6 * t.tv_nsec;
}
__global__ void touch(unsigned char* p, size_t n) {
  const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) << 21;
  if (i < n) p[i] = 1;
}
int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 25.0;
  const size_t n = (size_t)(gib * (1ull << 30));
  int dc = 0;
  if (hipGetDeviceCount(&dc) != hipSuccess) return 2;
  void *a = nullptr, *b = nullptr, *t0 = nullptr, *t1 = nullptr;
  double t = now_ms();
  if (hipMalloc(&a, n) != hipSuccess || hipMalloc(&b, n) != hipSuccess) return 3;
  const double t_alloc = now_ms() - t;
  t = now_ms();
  if (hipMalloc(&t0, 512ull << 20) != hipSuccess || hipMalloc(&t1, 512ull << 20) != hipSuccess) return 4;
  hipMemset(t0, 0xFF, 512ull << 20);
  hipMemset(t1, 0xFF, 512ull << 20);
  hipDeviceSynchronize();
  const double t_tables = now_ms() - t;
  t = now_ms();
  const size_t pages = n >> 21;
  hipLaunchKernelGGL(touch, dim3((unsigned)((pages + 255) / 256)), dim3(256), 0, 0, (unsigned char*)a, n);
  hipLaunchKernelGGL(touch, dim3((unsigned)((pages + 255) / 256)), dim3(256), 0, 0, (unsigned char*)b, n);
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  const double t_touch = now_ms() - t;
  t = now_ms();
  hipFree(a); hipFree(b); hipFree(t0); hipFree(t1);
  const double t_free = now_ms() - t;
  printf("{\"gib_each\":%.1f,\"alloc_ms\":%.1f,\"tables_ms\":%.1f,\"touch_ms\":%.1f,\"free_ms\":%.1f}\n", gib, t_alloc,
         t_tables, t_touch, t_free);
  return 0;
}

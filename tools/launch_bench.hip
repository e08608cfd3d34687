// launch_bench.hip — measures the fixed costs the level search's round
// structure pays on this GPU: back-to-back kernel launches of various grid
// sizes (empty, one dependent load, the last-block atomic pattern), graph
// replay of the same, and dependent-load latency (L2 / HBM).
//   hipcc --offload-arch=gfx950 -O3 tools/launch_bench.hip -o /tmp/launch_bench && /tmp/launch_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_empty(int* p) { if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) p[0] = 1; }
__global__ void k_load(const int* __restrict__ flag, int* out) {
  const int v = *flag;  // every wave: one global load, then exit
  if (v == 12345 && threadIdx.x == 0) out[blockIdx.x] = v;
}
__global__ void k_lastblock(unsigned* ctr, int* out) {
  __shared__ unsigned last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(ctr, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) { *ctr = 0; out[0]++; }
}
__global__ void k_lds46k(const int* __restrict__ flag, int* out) {
  __shared__ int big[46080 / 4];
  const int v = *flag;
  big[threadIdx.x] = v;
  __syncthreads();
  if (big[(threadIdx.x + 1) & 255] == 12345) out[blockIdx.x] = 1;
}
// one returning atomicAdd per wave on one counter (no fence)
__global__ void k_atomic_wave(unsigned* ctr, int* out) {
  if ((threadIdx.x & 63) == 0) {
    const unsigned v = atomicAdd(ctr, 8u);
    if (v == 0xFFFFFFFFu) out[0] = 1;
  }
}
// one returning atomicAdd per wave, spread over 64 counters (one per XCD-ish)
__global__ void k_atomic_spread(unsigned* ctr, int* out) {
  if ((threadIdx.x & 63) == 0) {
    const unsigned v = atomicAdd(ctr + 16 * (blockIdx.x & 63), 8u);
    if (v == 0xFFFFFFFFu) out[0] = 1;
  }
}
// a fence per wave
__global__ void k_fence(int* out) {
  if ((threadIdx.x & 63) == 0) {
    __threadfence();
    out[blockIdx.x] = 1;
  }
}
// dependent pointer chase: n steps over a ring of `len` entries with stride
__global__ void k_chase(const unsigned* __restrict__ ring, unsigned steps, unsigned* out, unsigned long long* cyc) {
  unsigned i = 0;
  const unsigned long long t0 = clock64();
  for (unsigned s = 0; s < steps; ++s) i = ring[i];
  const unsigned long long t1 = clock64();
  out[0] = i;
  cyc[0] = t1 - t0;
}

template <typename F>
double time_launches(hipStream_t st, int n, F launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) launch();
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(a, st));
  for (int i = 0; i < n; ++i) launch();
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return 1e3 * ms / n;  // us per launch
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int *flag, *out;
  unsigned* ctr;
  CK(hipMalloc(&flag, 4));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMalloc(&ctr, 64 * 64));
  CK(hipMemset(flag, 0, 4));
  CK(hipMemset(ctr, 0, 64 * 64));
  const int N = 2000;
  const int grids[] = {1, 8, 256, 768, 1792, 2048, 8192};
  for (int g : grids) {
    const double e = time_launches(st, N, [&] { hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, st, out); });
    const double l = time_launches(st, N, [&] { hipLaunchKernelGGL(k_load, dim3(g), dim3(256), 0, st, flag, out); });
    const double lb = time_launches(st, N, [&] { hipLaunchKernelGGL(k_lastblock, dim3(g), dim3(256), 0, st, ctr, out); });
    const double ld = time_launches(st, N, [&] { hipLaunchKernelGGL(k_lds46k, dim3(g), dim3(256), 0, st, flag, out); });
    printf("{\"grid\": %d, \"empty_us\": %.2f, \"one_load_us\": %.2f, \"last_block_atomic_us\": %.2f, \"lds46k_one_load_us\": %.2f}\n",
           g, e, l, lb, ld);
  }
  for (int g : {256, 2048, 8192}) {
    const double a = time_launches(st, 500, [&] { hipLaunchKernelGGL(k_atomic_wave, dim3(g), dim3(256), 0, st, ctr, out); });
    const double b = time_launches(st, 500, [&] { hipLaunchKernelGGL(k_atomic_spread, dim3(g), dim3(256), 0, st, ctr, out); });
    const double f = time_launches(st, 500, [&] { hipLaunchKernelGGL(k_fence, dim3(g), dim3(256), 0, st, out); });
    printf("{\"grid\": %d, \"waves\": %d, \"one_counter_atomic_per_wave_us\": %.2f, \"64_counters_us\": %.2f, \"fence_per_wave_us\": %.2f}\n",
           g, 4 * g, a, b, f);
  }
  // graph replay of 16 x (load kernel 768 blocks + last-block kernel 64 blocks)
  {
    hipGraph_t graph;
    hipGraphExec_t exec;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 16; ++i) {
      hipLaunchKernelGGL(k_load, dim3(768), dim3(256), 0, st, flag, out);
      hipLaunchKernelGGL(k_lastblock, dim3(64), dim3(256), 0, st, ctr, out);
    }
    CK(hipStreamEndCapture(st, &graph));
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    const double t = time_launches(st, 200, [&] { CK(hipGraphLaunch(exec, st)); });
    const double s = time_launches(st, 200, [&] {
      for (int i = 0; i < 16; ++i) {
        hipLaunchKernelGGL(k_load, dim3(768), dim3(256), 0, st, flag, out);
        hipLaunchKernelGGL(k_lastblock, dim3(64), dim3(256), 0, st, ctr, out);
      }
    });
    printf("{\"pair_x16_graph_us_per_pair\": %.2f, \"pair_x16_stream_us_per_pair\": %.2f}\n", t / 16, s / 16);
  }
  // dependent-load latency: a small ring (L2-resident) and a large one (HBM)
  for (size_t len : {(size_t)1 << 12, (size_t)1 << 16, (size_t)1 << 26}) {
    unsigned* h = (unsigned*)malloc(len * 4);
    const size_t stride = 4099;  // co-prime with the power-of-two length: one ring over all entries
    for (size_t i = 0; i < len; ++i) h[i] = (unsigned)((i + stride * 16) % len);
    unsigned* ring;
    unsigned long long* cyc;
    CK(hipMalloc(&ring, len * 4));
    CK(hipMalloc(&cyc, 8));
    CK(hipMemcpy(ring, h, len * 4, hipMemcpyHostToDevice));
    const unsigned steps = 4096;
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(1), 0, st, ring, steps, (unsigned*)out, cyc);
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(1), 0, st, ring, steps, (unsigned*)out, cyc);
    CK(hipStreamSynchronize(st));
    unsigned long long c = 0;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, st));
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(1), 0, st, ring, steps, (unsigned*)out, cyc);
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"chase_bytes\": %zu, \"cycles_per_load\": %.1f, \"ns_per_load\": %.1f}\n", len * 4, (double)c / steps,
           1e6 * ms / steps);
    CK(hipFree(ring));
    CK(hipFree(cyc));
    free(h);
  }
  return 0;
}

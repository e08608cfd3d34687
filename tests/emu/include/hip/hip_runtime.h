// TEST INFRASTRUCTURE ONLY — a CPU stand-in for the slice of the HIP runtime
// that libs2lincheck uses, so the exact kernel source (search_dev.h) can be run
// on the host under AddressSanitizer / ThreadSanitizer: every workgroup is run
// as blockDim.x std::threads sharing `static` "LDS" and a std::barrier.
// Never part of the product build (s2_verification_amd/Makefile uses hipcc).
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <barrier>
#include <thread>
#include <vector>

#define __host__
#define __device__
#define __global__
#define __forceinline__ inline
#define __noinline__
#define __launch_bounds__(...)
#define __shared__ static

struct uint4 { uint32_t x, y, z, w; };
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
struct dim3 {
  uint32_t x, y, z;
  dim3(uint32_t a = 1, uint32_t b = 1, uint32_t c = 1) : x(a), y(b), z(c) {}
};

namespace emu {
inline thread_local uint32_t tid_x = 0, bid_x = 0, bdim_x = 1;
inline std::barrier<>* g_barrier = nullptr;
inline uint8_t* g_dyn_lds = nullptr;
struct Idx { uint32_t x; };
template <typename K, typename... A>
void launch(K kernel, dim3 grid, dim3 block, size_t smem, A... args) {
  std::vector<uint8_t> lds(smem + 16);
  for (uint32_t b = 0; b < grid.x; ++b) {
    memset(lds.data(), 0xA5, lds.size());  // LDS is not zeroed between workgroups either
    g_dyn_lds = (uint8_t*)(((uintptr_t)lds.data() + 15) & ~(uintptr_t)15);
    std::barrier<> bar(block.x);
    g_barrier = &bar;
    std::vector<std::thread> th;
    th.reserve(block.x);
    for (uint32_t t = 0; t < block.x; ++t)
      th.emplace_back([&, t] { tid_x = t; bid_x = b; bdim_x = block.x; kernel(args...); });
    for (auto& x : th) x.join();
  }
}
}  // namespace emu

#define threadIdx (emu::Idx{emu::tid_x})
#define blockIdx (emu::Idx{emu::bid_x})
#define blockDim (emu::Idx{emu::bdim_x})
#define __syncthreads() emu::g_barrier->arrive_and_wait()
namespace emu {
inline std::atomic<int> g_or[2];
inline thread_local int or_phase = 0;
}  // namespace emu
// barrier + OR-reduction of pred over the workgroup (two alternating slots;
// lane 0 clears a slot after everyone has read it)
inline int __syncthreads_or(int pred) {
  const int ph = emu::or_phase;
  emu::or_phase ^= 1;
  if (pred) emu::g_or[ph].store(1);
  emu::g_barrier->arrive_and_wait();
  const int r = emu::g_or[ph].load();
  emu::g_barrier->arrive_and_wait();
  if (emu::tid_x == 0) emu::g_or[ph].store(0);
  return r;
}

template <typename T> inline T min(T a, T b) { return b < a ? b : a; }
template <typename T> inline T max(T a, T b) { return a < b ? b : a; }

inline uint32_t atomicAdd(uint32_t* p, uint32_t v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
  return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST);
}
inline uint32_t atomicCAS(uint32_t* p, uint32_t cmp, uint32_t v) {
  __atomic_compare_exchange_n(p, &cmp, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
  return cmp;
}
inline unsigned long long atomicCAS(unsigned long long* p, unsigned long long cmp, unsigned long long v) {
  __atomic_compare_exchange_n(p, &cmp, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
  return cmp;
}

// ---- runtime API ----
typedef int hipError_t;
enum { hipSuccess = 0, hipErrorOutOfMemory = 2 };
typedef void* hipStream_t;
typedef void* hipEvent_t;
enum hipMemcpyKind { hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice };
enum { hipStreamNonBlocking = 1 };
enum hipDeviceAttribute_t { hipDeviceAttributeMultiprocessorCount };
inline const char* hipGetErrorString(hipError_t) { return "emulated HIP error"; }
inline hipError_t hipGetDeviceCount(int* n) { *n = 1; return hipSuccess; }
inline hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int) { *v = 4; return hipSuccess; }
inline hipError_t hipMemGetInfo(size_t* f, size_t* t) { *f = (size_t)1 << 29; *t = (size_t)1 << 30; return hipSuccess; }
template <typename T> inline hipError_t hipMalloc(T** p, size_t n) {
  *p = (T*)malloc(n ? n : 1);
  if (!*p) return hipErrorOutOfMemory;
  memset((void*)*p, 0xA5, n);  // poison: the device gives no zeroed memory either
  return hipSuccess;
}
inline hipError_t hipFree(void* p) { free(p); return hipSuccess; }
inline hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) { memcpy(d, s, n); return hipSuccess; }
inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) { memcpy(d, s, n); return hipSuccess; }
inline hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t) { memset(d, v, n); return hipSuccess; }
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
inline hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) { *s = (void*)1; return hipSuccess; }
inline hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
inline hipError_t hipEventCreate(hipEvent_t* e) { *e = (void*)1; return hipSuccess; }
inline hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
inline hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
inline hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) { *ms = 0.f; return hipSuccess; }
inline hipError_t hipGetLastError() { return hipSuccess; }
#define hipLaunchKernelGGL(kernel, grid, block, shmem, stream, ...) emu::launch(kernel, grid, block, shmem, __VA_ARGS__)
// LDS-DMA: lane l writes 16 bytes at lds_base + 16*l
#define S2LC_GLDS16(gsrc, lds_base) memcpy((uint8_t*)(lds_base) + 16 * emu::tid_x, (const void*)(gsrc), 16)
#define S2LC_WAIT_ALL() do { } while (0)
// dynamic LDS of the emulated workgroup
#define S2LC_DYNAMIC_LDS(name) uint8_t* name = emu::g_dyn_lds

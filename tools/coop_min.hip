// coop_min: the smallest program that faults at exit under rocprofv3 after a
// cooperative launch, with none of libs2lincheck: one
// hipLaunchCooperativeKernel of a grid-synchronizing kernel, then return.
//   hipcc --offload-arch=gfx950 -O1 tools/coop_min.hip -o tools/coop_min
//   rocprofv3 --kernel-trace --stats -d <dir> -- tools/coop_min [reset]
// "reset": hipDeviceReset() before returning from main.
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <stdio.h>
#include <string.h>

namespace cg = cooperative_groups;

__global__ void coop_kernel(unsigned* out) {
  cg::grid_group g = cg::this_grid();
  if (threadIdx.x == 0) atomicAdd(out, 1u);
  g.sync();
  if (blockIdx.x == 0 && threadIdx.x == 0) out[1] = out[0];
}

int main(int argc, char** argv) {
  unsigned* d = nullptr;
  if (hipMalloc(&d, 8) != hipSuccess) return 2;
  (void)hipMemset(d, 0, 8);
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  void* args[] = {&d};
  hipError_t e = hipLaunchCooperativeKernel((const void*)coop_kernel, dim3(ncu), dim3(64), args, 0, nullptr);
  unsigned h[2] = {0, 0};
  (void)hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
  fprintf(stderr, "coop_min: launch %s, blocks %u (grid %d)\n", hipGetErrorString(e), h[1], ncu);
  (void)hipFree(d);
  if (argc > 1 && !strcmp(argv[1], "reset")) {
    (void)hipDeviceReset();
    fprintf(stderr, "coop_min: device reset\n");
  }
  fprintf(stderr, "coop_min: returning from main\n");
  return 0;
}

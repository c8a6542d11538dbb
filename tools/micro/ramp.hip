// Dispatch ramp probe: duration (launch-recorded events, hipExtLaunchKernelGGL) of a near-empty
// kernel for grid / block / dynamic-LDS shapes of the split rollout (1024 workgroups of 3 waves,
// ~31 KB LDS) and alternatives.  Each wave writes one dword so nothing is optimised away.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/ramp.hip -o build/ramp && ./build/ramp
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void probe(int* out, int spin) {
  extern __shared__ int lds[];
  int v = blockIdx.x;
  for (int i = 0; i < spin; ++i) v = v * 1664525 + 1013904223;  // a little per-wave work
  if ((threadIdx.x & 63) == 0) {
    lds[threadIdx.x >> 6] = v;
    out[blockIdx.x * 16 + (threadIdx.x >> 6)] = lds[threadIdx.x >> 6];
  }
}

int main() {
  int* out;
  hipMalloc(&out, 4096 * 16 * 4);
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  struct Cfg { int grid, block, lds; const char* what; };
  const Cfg cfgs[] = {
      {1024, 64, 0, "1024 x 1 wave, no LDS (per-step kernel shape, C2)"},
      {1024, 64, 13000, "1024 x 1 wave, 13 KB LDS (per-step kernel, C2)"},
      {1024, 192, 31000, "1024 x 3 waves, 31 KB LDS (split rollout, C2)"},
      {512, 384, 62000, "512 x 6 waves, 62 KB LDS"},
      {256, 768, 124000, "256 x 12 waves, 124 KB LDS"},
      {256, 256, 0, "256 x 4 waves, no LDS"},
      {2048, 64, 0, "2048 x 1 wave"},
      {4096, 64, 0, "4096 x 1 wave"},
      {64, 64, 0, "64 x 1 wave"},
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int spin : {0, 200}) {
    for (const Cfg& c : cfgs) {
      std::vector<float> ms;
      for (int r = 0; r < 25; ++r) {
        hipExtLaunchKernelGGL(probe, dim3(c.grid), dim3(c.block), c.lds, 0, e0, e1, 0, out, spin);
        hipEventSynchronize(e1);
        float t = 0;
        hipEventElapsedTime(&t, e0, e1);
        if (r >= 5) ms.push_back(t);
      }
      std::sort(ms.begin(), ms.end());
      printf("spin %3d  %-52s median %6.2f us  min %6.2f us\n", spin, c.what, ms[ms.size() / 2] * 1e3, ms[0] * 1e3);
    }
  }
  return 0;
}

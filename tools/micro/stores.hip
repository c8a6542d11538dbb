// Microbenchmark: cost of writing a wave's 3200-byte block of 64 x 50-byte records
// per "step" on gfx950, by store pattern.  1024 waves x 64 steps (the C2 rollout shape).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int STEPS = 64, WAVES = 1024, REC = 50, BLK = 64 * REC;  // 3200 B per wave-step

// A: 12 scattered dword stores + 1 short per lane (direct record writes)
__global__ void __launch_bounds__(64) k_scatter(unsigned char* out, uint32_t seed) {
  const int l = threadIdx.x;
  uint32_t w[13];
  for (int k = 0; k < 13; ++k) w[k] = seed * (l + 1) + k;
  for (int s = 0; s < STEPS; ++s) {
    unsigned char* rec = out + ((size_t)s * WAVES + blockIdx.x) * BLK + l * REC;
    const bool odd = (l & 1);
    unsigned char* d = rec + (odd ? 2 : 0);
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      uint32_t v = odd ? __builtin_amdgcn_alignbyte(w[j + 1], w[j], 2) : w[j];
      asm volatile("global_store_dword %0, %1, off" :: "v"(d + 4 * j), "v"(v) : "memory");
    }
    *(volatile uint16_t*)(rec + (odd ? 0 : 48)) = (uint16_t)w[0];
    for (int k = 0; k < 13; ++k) w[k] += 7;
  }
}

// B: same bytes as 4 coalesced dwordx4 stores per lane (3.125 really: 200 chunks)
__global__ void __launch_bounds__(64) k_coalesced(unsigned char* out, uint32_t seed) {
  const int l = threadIdx.x;
  uint4 v = make_uint4(seed + l, seed, l, 3);
  for (int s = 0; s < STEPS; ++s) {
    uint4* dst = (uint4*)(out + ((size_t)s * WAVES + blockIdx.x) * BLK);
    for (int i = l; i < BLK / 16; i += 64) dst[i] = v;
    v.x += 1;
  }
}

// C: LDS staging with ds_write2_b32 (6) + b16 (1) per lane, then coalesced copy-out
__global__ void __launch_bounds__(64) k_lds_stage(unsigned char* out, uint32_t seed) {
  __shared__ __align__(16) unsigned char stage[BLK + 16];
  const int l = threadIdx.x;
  uint32_t w[13];
  for (int k = 0; k < 13; ++k) w[k] = seed * (l + 1) + k;
  for (int s = 0; s < STEPS; ++s) {
    const bool odd = (l & 1);
    uint32_t* d = (uint32_t*)(stage + l * REC + (odd ? 2 : 0));
#pragma unroll
    for (int j = 0; j < 12; ++j) d[j] = odd ? __builtin_amdgcn_alignbyte(w[j + 1], w[j], 2) : w[j];
    *(uint16_t*)(stage + l * REC + (odd ? 0 : 48)) = (uint16_t)w[0];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint4* dst = (uint4*)(out + ((size_t)s * WAVES + blockIdx.x) * BLK);
    for (int i = l; i < BLK / 16; i += 64) dst[i] = ((const uint4*)stage)[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int k = 0; k < 13; ++k) w[k] += 7;
  }
}

// D: 5 byte stores + 1 int2 store per lane per step (the per-agent outputs)
__global__ void __launch_bounds__(64) k_small(unsigned char* out, uint32_t seed) {
  const int l = threadIdx.x;
  for (int s = 0; s < STEPS; ++s) {
    size_t o = ((size_t)s * WAVES + blockIdx.x) * 64 + l;
    unsigned char* b = out;
    b[o] = (unsigned char)(seed + s);
    b[(size_t)STEPS * WAVES * 64 + o] = (unsigned char)l;
    b[2 * (size_t)STEPS * WAVES * 64 + o] = (unsigned char)s;
    b[3 * (size_t)STEPS * WAVES * 64 + o] = (unsigned char)(l ^ s);
    ((int2*)(b + 4 * (size_t)STEPS * WAVES * 64))[o] = make_int2(l, s);
  }
}

int main() {
  size_t bytes = (size_t)STEPS * WAVES * BLK + 64;
  unsigned char* out;
  CHECK(hipMalloc(&out, bytes * 2));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[] = {"scatter_dword", "coalesced_x4", "lds_stage", "small_5b+int2"};
  for (int rep = 0; rep < 3; ++rep) {
    for (int k = 0; k < 4; ++k) {
      CHECK(hipEventRecord(e0));
      for (int it = 0; it < 5; ++it) {
        if (k == 0) hipLaunchKernelGGL(k_scatter, dim3(WAVES), dim3(64), 0, 0, out, 7u + it);
        if (k == 1) hipLaunchKernelGGL(k_coalesced, dim3(WAVES), dim3(64), 0, 0, out, 7u + it);
        if (k == 2) hipLaunchKernelGGL(k_lds_stage, dim3(WAVES), dim3(64), 0, 0, out, 7u + it);
        if (k == 3) hipLaunchKernelGGL(k_small, dim3(WAVES), dim3(64), 0, 0, out, 7u + it);
      }
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      double per_step_us = ms * 1e3 / 5 / STEPS;
      double bytes_step = k == 3 ? WAVES * 64.0 * 12 : (double)WAVES * BLK;
      if (rep == 2) printf("%-16s %7.3f us/step  %7.1f GB/s\n", names[k], per_step_us, bytes_step / per_step_us / 1e3);
    }
  }
  return 0;
}

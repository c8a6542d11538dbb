// Microbenchmark: HBM write rate of the C2 runner-rollout output pattern with no
// compute, 1024 one-wave workgroups x 64 steps (4 envs x 16 agents per wave).
// Per wave-step: 3200 B window records, 512 B positions, 4 x 64 B agent bytes,
// 32 B rewards, 16 B t, 4 B term -- each array step-major [T][E][...] like the kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int STEPS = 64, WAVES = 1024;
constexpr size_t REC_STEP = (size_t)WAVES * 3200, POS_STEP = (size_t)WAVES * 512, B_STEP = (size_t)WAVES * 64;
constexpr size_t REW_STEP = (size_t)WAVES * 32, T_STEP = (size_t)WAVES * 16, TERM_STEP = (size_t)WAVES * 4;

struct Out {
  unsigned char *rec, *pos, *node, *edge, *avail, *done, *rew, *tt, *term;
};

// mode 0: every output; 1: records only; 2: everything but records
__global__ void __launch_bounds__(64) k_out(Out o, int mode, uint32_t seed) {
  const int l = threadIdx.x;
  const int w = blockIdx.x;
  uint4 v = make_uint4(seed + l, seed ^ w, l, 3);
  for (int s = 0; s < STEPS; ++s) {
    if (mode != 2) {
      uint4* d = (uint4*)(o.rec + s * REC_STEP + (size_t)w * 3200);
      for (int i = l; i < 200; i += 64) d[i] = v;
    }
    if (mode != 1) {
      if (l < 32) ((uint4*)(o.pos + s * POS_STEP + (size_t)w * 512))[l] = v;
      else if (l < 48) {
        const int a = (l - 32) >> 2, c = (l - 32) & 3;
        unsigned char* arr = a == 0 ? o.node : a == 1 ? o.edge : a == 2 ? o.avail : o.done;
        ((uint4*)(arr + s * B_STEP + (size_t)w * 64))[c] = v;
      } else if (l < 50) {
        ((uint4*)(o.rew + s * REW_STEP + (size_t)w * 32))[l - 48] = v;
      } else if (l == 50) {
        ((uint4*)(o.tt + s * T_STEP + (size_t)w * 16))[0] = v;
      } else if (l == 51) {
        ((uint32_t*)(o.term + s * TERM_STEP + (size_t)w * 4))[0] = v.x;
      }
    }
    v.x += 1;
  }
}

int main() {
  Out o;
  size_t sizes[9] = {REC_STEP, POS_STEP, B_STEP, B_STEP, B_STEP, B_STEP, REW_STEP, T_STEP, TERM_STEP};
  unsigned char** ptrs[9] = {&o.rec, &o.pos, &o.node, &o.edge, &o.avail, &o.done, &o.rew, &o.tt, &o.term};
  double bytes_all = 0, bytes_rec = (double)REC_STEP * STEPS;
  for (int i = 0; i < 9; ++i) {
    CHECK(hipMalloc(ptrs[i], sizes[i] * STEPS));
    bytes_all += (double)sizes[i] * STEPS;
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[] = {"all outputs", "records only", "all but records"};
  for (int rep = 0; rep < 3; ++rep) {
    for (int m = 0; m < 3; ++m) {
      CHECK(hipEventRecord(e0));
      for (int it = 0; it < 8; ++it) hipLaunchKernelGGL(k_out, dim3(WAVES), dim3(64), 0, 0, o, m, 7u + it);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double b = m == 0 ? bytes_all : m == 1 ? bytes_rec : bytes_all - bytes_rec;
      const double us_step = ms * 1e3 / 8 / STEPS;
      if (rep == 2) printf("%-16s %7.3f us/step  %7.1f GB/s\n", names[m], us_step, b / STEPS / us_step / 1e3);
    }
  }
  return 0;
}

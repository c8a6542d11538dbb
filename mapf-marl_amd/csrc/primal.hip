// primal.hip -- MI355X (gfx950) batched PRIMAL sequential dynamics.
//
// MARL-curve-main/src/envs/mapf_primal.py (paths below relative to it):
// MAPFEnv._step((agent_id, action)) :549-637 moves ONE agent against the current
// world (State.moveAgent :103-135: out of bounds -1, wall -2, robot -3, else move;
// status 1 on / reached goal, 2 left goal, 0 otherwise), prices it with the
// reward table :579-596, and returns _observe (:343-386), world.done (:159-166),
// _listNextValidActions (:639-667), on_goal and valid.  Calls are sequential: a
// later call sees the moves of the earlier ones.
//
// One lane group of 16, 32 or 64 lanes per world, 64 / lw worlds per wave.  The
// world lives in LDS as an occupant map (0 empty, id + 1) and an obstacle bitmap;
// for each call the group's first lane resolves the move (the only sequential
// part) and the group builds that agent's 4 x s x s observation (one cell per
// lane), the visible agents' clamped goals (one agent per lane) and the done
// ballot.  The goal-vector magnitude comes from a host
// libm pow LUT, as the reference computes `(dx**2 + dy**2) ** .5` (quirk 8).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>

#include "internal.h"
#include "mapfx.h"
#include "mapfx_primal.h"

namespace {

constexpr double ACTION_COST = -0.3, IDLE_COST = -.5, GOAL_REWARD = 0.0, COLLISION_REWARD = -2.;  // :25

struct QGeo {
  int H, W, N, E, s, map_shared;
  long long map_stride;
  int hw, bits_words, lut_n;
  int lw, lw_shift, wreg;  // lanes per world (16 / 32 / 64), log2, LDS bytes per world
};

struct QArgs {
  int32_t* pos;
  const int32_t* goal;
  const uint8_t* bits;
  const int32_t* ids;
  const int32_t* acts;
  int K;
  double* reward;
  uint8_t* done;
  uint8_t* next_mask;
  uint8_t* on_goal;
  uint8_t* valid;
  uint8_t* obs;
  double* vec;
  int32_t* err;
  const double* pow_lut;  // (double)n ** .5 by host libm pow, n = 0 .. lut_n-1
};

__device__ inline void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline int dir_r(int a) { return a == 2 ? 1 : (a == 4 ? -1 : 0); }  // dirDict :28
__device__ inline int dir_c(int a) { return a == 1 ? 1 : (a == 3 ? -1 : 0); }

// One wave holds 64 / lw worlds, lw lanes each (lw = 16, 32 or 64; the host picks it
// from N and the grid size).  A call is a chain of LDS round trips (move ->
// post-move reads -> goal stamps -> stores), and the waves are too few to hide
// them, so the chain is kept short: every LDS read a step needs is issued in one
// batch (the move's cell and obstacle word, the observation cells of the next
// step, the next-action probes, the agents), the visible-goals plane is a
// per-call stamp (no clearing pass), and the next call's (id, action) is read
// while this one runs.
constexpr int PR_IT = 4;  // observation cells per lane held in registers (s*s <= 4 lw)

// S, LS: observation size and log2(lanes per world) fixed at compile time (0: from
// QGeo).  PRIMAL's default observation_size (10, `:175`) gets specialised kernels:
// the window walk and the planes' store offsets become immediates.
template <int S, int LS>
__global__ void __launch_bounds__(64) primal_act_kernel(QGeo g, QArgs a) {
  extern __shared__ __align__(16) unsigned char lds[];
  const int lws = LS ? LS : g.lw_shift;
  const int lw = 1 << lws, lane = threadIdx.x;
  const int wl = lane >> lws, ag = lane & (lw - 1), lead = wl << lws;
  const int e = blockIdx.x * (64 >> lws) + wl;
  const bool live = e < g.E;
  const uint64_t wmask = (lw == 64 ? ~0ull : ((1ull << lw) - 1ull)) << lead;
  const int N = g.N, H = g.H, W = g.W, s = S ? S : g.s, ss = s * s;
  unsigned char* wr = lds + wl * g.wreg;
  uint8_t* occ = wr;                                           // [H*W] 0 empty, id + 1
  uint32_t* obst = (uint32_t*)(wr + ((g.hw + 15) & ~15));      // [bits_words]
  int2* pos = (int2*)((unsigned char*)obst + ((g.bits_words * 4 + 15) & ~15));  // [N]
  int2* gl = pos + N;                                          // [N]
  int2* pend = gl + N;                                         // [64] goal vector (dx, dy) of a block's calls
  int2* pairL = pend + 64;                                     // [64] a block's (agent id, action)
  int* flag = (int*)(pairL + 64);                              // [4] move status
  int* stamp = flag + 4;                                       // [s*s] call k + 1 marks a visible goal

  if (live) {
    for (int i = ag; i < g.hw; i += lw) occ[i] = 0;
    for (int i = ag; i < ss; i += lw) stamp[i] = 0;
    const uint32_t* src = (const uint32_t*)(a.bits + (g.map_shared ? 0 : (long long)e * g.map_stride));
    for (int w = ag; w < g.bits_words; w += lw) obst[w] = src[w];
    for (int b = ag; b < N; b += lw) {
      pos[b] = ((const int2*)a.pos)[(long long)e * N + b];
      gl[b] = ((const int2*)a.goal)[(long long)e * N + b];
    }
  }
  wave_fence();
  if (live)
    for (int b = ag; b < N; b += lw) occ[pos[b].x * W + pos[b].y] = (uint8_t)(b + 1);
  wave_fence();
  // this lane's first observation cell (ag / s, ag % s) and the step to its next one
  const int r_step = lw / s, c_step = lw % s;
  const int r0 = ag / s, c0 = ag % s;
  const bool probe = ag >= 1 && ag <= 4;  // lanes 1..4 test the next-action directions

  const long long e0k = (long long)e * a.K;
  int kstop = live ? a.K : 0;  // calls of this world from kstop on are not run (bad call)
  for (int kb = 0; kb < a.K; kb += 64) {
    const int kend = min(a.K, kb + 64);
    // the block's (id, action) pairs -> LDS: one load wait per 64 calls (on gfx9
    // vmcnt also counts stores, so a wait drains the earlier calls' outputs)
    if (kb < kstop)
      for (int j = ag; j < kend - kb; j += lw) pairL[j] = make_int2(a.ids[e0k + kb + j], a.acts[e0k + kb + j]);
    wave_fence();
    int2 pa = pairL[0];
    for (int k = kb; k < kend; ++k) {
      const int2 nxt = pairL[min(k + 1 - kb, 63)];  // the next call's pair, read ahead
      const int aid = pa.x - 1, act = pa.y;
      pa = nxt;
      if (k >= kstop) continue;  // (uniform within a world)
      const long long ek = e0k + k;
      if (aid < 0 || aid >= N || act < 0 || act > 4) {  // the reference asserts (:556-558)
        if (ag == 0 && a.err) atomicCAS(a.err, 0, e + 1);
        kstop = k;
        continue;
      }
      // ---- State.moveAgent (:103-135), the world's first lane ----
      if (ag == 0) {
        const int2 p = pos[aid], gg = gl[aid];
        const int nx = p.x + dir_r(act), ny = p.y + dir_c(act);
        const bool inb = nx < H && nx >= 0 && ny < W && ny >= 0;
        const int ci = inb ? nx * W + ny : 0;
        const uint8_t oc = occ[ci];
        const uint32_t ow = obst[ci >> 5];
        // the status chain as selects (one branch, for the move's writes)
        const bool on_old = gg.x == p.x && gg.y == p.y, on_new = gg.x == nx && gg.y == ny;
        const bool wall = ((ow >> (ci & 31)) & 1u) != 0;
        const bool moved = act != 0 && inb && oc == 0 && !wall;
        const int st_move = on_new ? 1 : (on_old ? 2 : 0);
        const int st_blocked = !inb ? -1 : (oc != 0 ? -3 : -2);  // robot before wall: state > 0
        const int status = act == 0 ? (on_old ? 1 : 0) : (moved ? st_move : st_blocked);
        if (moved) {
          occ[p.x * W + p.y] = 0;
          occ[ci] = (uint8_t)(aid + 1);
          pos[aid] = make_int2(nx, ny);
        }
        flag[0] = status;
      }
      wave_fence();
      // ---- one batch of LDS reads on the post-move world ----
      const int status = flag[0];
      const int2 p = pos[aid], gg = gl[aid];
      const int ax = p.x, ay = p.y;
      const int tr = ax - s / 2, tc = ay - s / 2;
      // _observe cells (:343-386) held in registers: occupant and obstacle word
      uint8_t ocv[PR_IT];
      uint32_t obv[PR_IT];
      int cidx[PR_IT];  // map cell, -1 outside the map
      {
        int rr = r0, cc = c0;
#pragma unroll
        for (int it = 0; it < PR_IT; ++it) {
          const int r = tr + rr, c = tc + cc;
          const bool in = ag + it * lw < ss && r < H && r >= 0 && c < W && c >= 0;
          cidx[it] = in ? r * W + c : -1;
          const int ci = in ? r * W + c : 0;
          ocv[it] = occ[ci];  // (unconditional: cell 0 when outside or no obs)
          obv[it] = obst[ci >> 5];
          rr += r_step;
          cc += c_step;
          if (cc >= s) {
            cc -= s;
            ++rr;
          }
        }
      }
      // _listNextValidActions (:639-667): direction ag probed by lane ag of the world
      bool ok = false;
      if (probe) {
        const int nx = ax + dir_r(ag), ny = ay + dir_c(ag);
        const bool inb = nx < H && nx >= 0 && ny < W && ny >= 0;
        const int ci = inb ? nx * W + ny : 0;
        ok = inb && occ[ci] == 0 && !((obst[ci >> 5] >> (ci & 31)) & 1u);
      }
      // agents: done (:159-166) and visible agents' goals, clamped into view (:374-378)
      bool off = false;
      for (int b = ag; b < N; b += lw) {
        const int2 pb = pos[b], gb = gl[b];
        off |= (pb.x != gb.x) || (pb.y != gb.y);
        if (a.obs && b != aid && pb.x >= tr && pb.x < tr + s && pb.y >= tc && pb.y < tc + s) {
          const int mr = max(tr, min(tr + s - 1, gb.x));
          const int mc = max(tc, min(tc + s - 1, gb.y));
          stamp[(mr - tr) * s + (mc - tc)] = k + 1;
        }
      }
      const bool done = (__ballot(off) & wmask) == 0;
      const uint32_t mbits = (uint32_t)(__ballot(ok) >> lead) & 0x1Eu;  // bits 1..4 = actions
      wave_fence();
      if (a.obs) {
        uint8_t* o = a.obs + ek * 4 * ss;
        const int gcell = gg.x * W + gg.y;
        const auto cell = [&](int i, int ci, uint8_t oc, uint32_t ow) {  // branch-free selects
          const bool in = ci >= 0, agent = oc != 0;
          const bool wall = ((ow >> (ci & 31)) & 1u) != 0;
          o[i] = (in && agent) ? 1 : 0;                   // :363-365, 369-372
          o[ss + i] = ci == gcell ? 1 : 0;                // :366-368 (ci = -1 outside)
          o[2 * ss + i] = stamp[i] == k + 1 ? 1 : 0;
          o[3 * ss + i] = (!in || (!agent && wall)) ? 1 : 0;  // outside: obstacle (:356-362)
        };
#pragma unroll
        for (int it = 0; it < PR_IT; ++it) {
          const int i = ag + it * lw;
          if (i < ss) cell(i, cidx[it], ocv[it], obv[it]);
        }
        for (int i = ag + PR_IT * lw; i < ss; i += lw) {  // large windows: the rest
          const int r = tr + i / s, c = tc + i % s;
          const bool in = r < H && r >= 0 && c < W && c >= 0;
          const int ci = in ? r * W + c : 0;
          cell(i, in ? ci : -1, occ[ci], obst[ci >> 5]);
        }
      }
      if (ag == 0) {
        // ---- reward (:579-596), JOINT = False; stay-on-goal blocking term = 0 ----
        const double rew = act == 0 ? (status == 1 ? GOAL_REWARD + 0 : IDLE_COST)
                                    : status == 1 ? GOAL_REWARD : status < 0 ? COLLISION_REWARD : ACTION_COST;
        uint32_t m = 1u | mbits;
        const int opp = act == 1 ? 3 : act == 2 ? 4 : act == 3 ? 1 : act == 4 ? 2 : -1;  // :26
        if (opp > 0) m &= ~(1u << opp);
        if (a.reward) a.reward[ek] = rew;
        if (a.done) a.done[ek] = done ? 1 : 0;
        if (a.next_mask) a.next_mask[ek] = (uint8_t)m;
        if (a.on_goal) a.on_goal[ek] = (ax == gg.x && ay == gg.y) ? 1 : 0;
        if (a.valid) a.valid[ek] = status >= 0 ? 1 : 0;
        // goal vector (:379-384): its magnitude needs a LUT load, so the call's
        // (dx, dy) waits in LDS and the world writes a block's vectors together
        // (one load latency per 64 calls instead of one per call)
        pend[k - kb] = make_int2(gg.x - ax, gg.y - ay);
      }
      wave_fence();
    }
    if (a.vec) {  // the block's goal vectors, calls kb .. min(kend, kstop) - 1
      const int n = min(kend, kstop) - kb;
      for (int j = ag; j < n; j += lw) {
        const int2 d = pend[j];
        const double mag = a.pow_lut[d.x * d.x + d.y * d.y];
        double vx = (double)d.x, vy = (double)d.y;
        if (mag != 0.0) {
          vx = vx / mag;
          vy = vy / mag;
        }
        double* v = a.vec + (e0k + kb + j) * 3;
        v[0] = vx;
        v[1] = vy;
        v[2] = mag;
      }
    }
    wave_fence();
  }
  if (live)
    for (int b = ag; b < N; b += lw) ((int2*)a.pos)[(long long)e * N + b] = pos[b];
}

int perr(int code, const char* msg) { return mapfx_internal_error(code, msg); }

int check_hip(hipError_t err, const char* what) {
  if (err != hipSuccess) {
    char buf[256];
    snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(err));
    return perr(MAPFX_EHIP, buf);
  }
  return MAPFX_OK;
}

}  // namespace

struct mapfx_primal_t {
  QGeo geo;
  double* pow_lut;
  int lds;
};

extern "C" {

int mapfx_primal_create(const mapfx_primal_cfg* cfg, mapfx_primal_t** out) {
  if (!cfg || !out) return perr(MAPFX_EINVAL, "NULL argument");
  *out = nullptr;
  const mapfx_primal_cfg& c = *cfg;
  if (c.H < 1 || c.W < 1 || (long long)c.H * c.W > 16384)
    return perr(MAPFX_EINVAL, "PRIMAL path supports H * W <= 16384");
  if (c.n_agents < 1 || c.n_agents > 255) return perr(MAPFX_EINVAL, "n_agents must be in 1..255");
  if (c.n_envs < 0) return perr(MAPFX_EINVAL, "n_envs < 0");
  if (c.obs_size < 1 || c.obs_size > 32) return perr(MAPFX_EINVAL, "obs_size must be in 1..32");
  mapfx_primal_t* h = new (std::nothrow) mapfx_primal_t();
  if (!h) return perr(MAPFX_ENOMEM, "host allocation failed");
  QGeo& g = h->geo;
  g.H = c.H;
  g.W = c.W;
  g.N = c.n_agents;
  g.E = c.n_envs;
  g.s = c.obs_size;
  g.map_shared = c.map_shared ? 1 : 0;
  g.map_stride = mapfx_map_stride(c.H, c.W);
  g.hw = c.H * c.W;
  g.bits_words = (g.hw + 31) / 32;
  g.lut_n = (c.H - 1) * (c.H - 1) + (c.W - 1) * (c.W - 1) + 1;
  g.wreg = ((g.hw + 15) & ~15) + ((g.bits_words * 4 + 15) & ~15) + 16 * g.N + 64 * 8 + 64 * 8 + 16 +
           ((4 * g.s * g.s + 15) & ~15);
  // Lanes per world: the smallest of 16 / 32 / 64 that covers N, widened while the
  // grid has fewer than 2 waves per SIMD (2048 waves) or the wave's worlds would
  // pass 64 KB of LDS.  Packing worlds saves issue slots (the per-call work is
  // mostly per world, not per cell), more waves hide the call's LDS chain; at
  // 4096 worlds of N = 16 (the bench) 16 / 32 / 64 lanes measured 149 / 120 / 125 us
  // per 64-call launch.
  // MAPFX_PRIMAL_LANES (16 / 32 / 64) overrides the first two rules (tests).
  g.lw_shift = g.N <= 16 ? 4 : g.N <= 32 ? 5 : 6;
  const char* force = getenv("MAPFX_PRIMAL_LANES");
  const int fl = force ? atoi(force) : 0;
  if (fl == 16 || fl == 32 || fl == 64) g.lw_shift = std::max(g.lw_shift, fl == 16 ? 4 : fl == 32 ? 5 : 6);
  else
    while (g.lw_shift < 6 && (long long)(g.E + (64 >> g.lw_shift) - 1) / (64 >> g.lw_shift) < 2048) ++g.lw_shift;
  while (g.lw_shift < 6 && (64 >> g.lw_shift) * g.wreg > 65536) ++g.lw_shift;
  g.lw = 1 << g.lw_shift;
  h->lds = (64 >> g.lw_shift) * g.wreg;
  double* lut = (double*)malloc(sizeof(double) * g.lut_n);
  if (!lut) {
    delete h;
    return perr(MAPFX_ENOMEM, "host allocation failed");
  }
  double (*volatile libm_pow)(double, double) = pow;  // `n ** .5` in Python = libm pow
  for (int i = 0; i < g.lut_n; ++i) lut[i] = libm_pow((double)i, 0.5);
  h->pow_lut = nullptr;
  int rc = check_hip(hipMalloc(&h->pow_lut, sizeof(double) * g.lut_n), "hipMalloc");
  if (!rc) rc = check_hip(hipMemcpy(h->pow_lut, lut, sizeof(double) * g.lut_n, hipMemcpyHostToDevice), "hipMemcpy");
  free(lut);
  if (rc) {
    mapfx_primal_destroy(h);
    return rc;
  }
  *out = h;
  return MAPFX_OK;
}

void mapfx_primal_destroy(mapfx_primal_t* h) {
  if (!h) return;
  if (h->pow_lut) (void)hipFree(h->pow_lut);
  delete h;
}

int mapfx_primal_act(mapfx_primal_t* h, const mapfx_primal_state* st, const int32_t* agent_ids,
                     const int32_t* actions, int32_t K, const mapfx_primal_out* out, void* stream) {
  if (!h) return perr(MAPFX_EINVAL, "NULL handle");
  if (!st || !st->pos || !st->goal || !st->map_bits) return perr(MAPFX_EINVAL, "bad state");
  if (K < 0) return perr(MAPFX_EINVAL, "K < 0");
  if (K == 0 || h->geo.E == 0) return MAPFX_OK;
  if (!agent_ids || !actions) return perr(MAPFX_EINVAL, "NULL agent_ids / actions");
  QArgs a;
  memset(&a, 0, sizeof(a));
  a.pos = st->pos;
  a.goal = st->goal;
  a.bits = st->map_bits;
  a.ids = agent_ids;
  a.acts = actions;
  a.K = K;
  a.pow_lut = h->pow_lut;
  if (out) {
    a.reward = out->reward;
    a.done = out->done;
    a.next_mask = out->next_mask;
    a.on_goal = out->on_goal;
    a.valid = out->valid;
    a.obs = out->obs;
    a.vec = out->vec;
    a.err = out->err;
  }
  const int wpw = 64 >> h->geo.lw_shift;
  const dim3 grid((h->geo.E + wpw - 1) / wpw), block(64);
  const hipStream_t sm = (hipStream_t)stream;
  const QGeo& g = h->geo;
  if (g.s == 10 && g.lw_shift == 4) hipLaunchKernelGGL((primal_act_kernel<10, 4>), grid, block, h->lds, sm, g, a);
  else if (g.s == 10 && g.lw_shift == 5) hipLaunchKernelGGL((primal_act_kernel<10, 5>), grid, block, h->lds, sm, g, a);
  else if (g.s == 10 && g.lw_shift == 6) hipLaunchKernelGGL((primal_act_kernel<10, 6>), grid, block, h->lds, sm, g, a);
  else hipLaunchKernelGGL((primal_act_kernel<0, 0>), grid, block, h->lds, sm, g, a);
  return check_hip(hipGetLastError(), "primal_act_kernel launch");
}

}  // extern "C"

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
// One wavefront per world.  The world lives in LDS as an occupant map (0 empty,
// id + 1) and an obstacle bitmap; for each call lane 0 resolves the move (the
// only sequential part) and the whole wave builds that agent's 4 x s x s
// observation (one cell per lane), the visible agents' clamped goals (one agent
// per lane) and the done ballot.  The goal-vector magnitude comes from a host
// libm pow LUT, as the reference computes `(dx**2 + dy**2) ** .5` (quirk 8).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
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

__global__ void __launch_bounds__(64) primal_act_kernel(QGeo g, QArgs a) {
  extern __shared__ __align__(16) unsigned char lds[];
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = g.N, H = g.H, W = g.W, s = g.s;
  uint8_t* occ = lds;                                   // [H*W] 0 empty, id + 1
  uint32_t* obst = (uint32_t*)(lds + ((g.hw + 15) & ~15));  // [bits_words]
  int2* pos = (int2*)((unsigned char*)obst + ((g.bits_words * 4 + 15) & ~15));  // [N]
  int2* gl = pos + N;                                   // [N]
  uint8_t* goals_plane = (uint8_t*)(gl + N);            // [s*s]
  int* flag = (int*)(goals_plane + ((s * s + 15) & ~15));  // [2]: bad call

  for (int i = lane; i < g.hw; i += 64) occ[i] = 0;
  const uint32_t* src = (const uint32_t*)(a.bits + (g.map_shared ? 0 : (long long)e * g.map_stride));
  for (int w = lane; w < g.bits_words; w += 64) obst[w] = src[w];
  for (int b = lane; b < N; b += 64) {
    pos[b] = ((const int2*)a.pos)[(long long)e * N + b];
    gl[b] = ((const int2*)a.goal)[(long long)e * N + b];
  }
  wave_fence();
  for (int b = lane; b < N; b += 64) occ[pos[b].x * W + pos[b].y] = (uint8_t)(b + 1);
  wave_fence();
  const auto is_obst = [&](int r, int c) { const int i = r * W + c; return (obst[i >> 5] >> (i & 31)) & 1u; };

  // the calls' (agent id, action) pairs: lane l holds call 64 b + l of block b, the
  // next block is loaded while this one runs, and each call reads its pair with
  // v_readlane (uniform index) -- no HBM round trip inside the sequential loop
  const long long e0k = (long long)e * a.K;
  int id_c = 0, act_c = 0, id_n = 0, act_n = 0;
  if (lane < a.K) {
    id_n = a.ids[e0k + lane];
    act_n = a.acts[e0k + lane];
  }
  int pend_dx = 0, pend_dy = 0;
  const auto flush_vec = [&](int kb, int n) {  // calls kb .. kb + n - 1, one per lane
    if (lane < n) {
      const long long ekl = e0k + kb + lane;
      const double mag = a.pow_lut[pend_dx * pend_dx + pend_dy * pend_dy];
      double vx = (double)pend_dx, vy = (double)pend_dy;
      if (mag != 0.0) {
        vx = vx / mag;
        vy = vy / mag;
      }
      a.vec[ekl * 3 + 0] = vx;
      a.vec[ekl * 3 + 1] = vy;
      a.vec[ekl * 3 + 2] = mag;
    }
  };
  for (int k = 0; k < a.K; ++k) {
    const long long ek = e0k + k;
    if ((k & 63) == 0) {
      id_c = id_n;
      act_c = act_n;
      if (k + 64 + lane < a.K) {
        id_n = a.ids[ek + 64 + lane];
        act_n = a.acts[ek + 64 + lane];
      }
    }
    const int aid = __builtin_amdgcn_readlane(id_c, k & 63) - 1;
    const int act = __builtin_amdgcn_readlane(act_c, k & 63);
    if (aid < 0 || aid >= N || act < 0 || act > 4) {  // the reference asserts (:556-558)
      if (lane == 0 && a.err) atomicCAS(a.err, 0, e + 1);
      if (a.vec && (k & 63)) flush_vec(k & ~63, k & 63);  // the block's earlier calls
      break;
    }
    // ---- State.moveAgent (:103-135), lane 0 ----
    int status = 0;
    if (lane == 0) {
      const int ax = pos[aid].x, ay = pos[aid].y;
      const int2 gg = gl[aid];
      if (act == 0) {
        status = (gg.x == ax && gg.y == ay) ? 1 : 0;
      } else {
        const int nx = ax + dir_r(act), ny = ay + dir_c(act);
        if (nx >= H || nx < 0 || ny >= W || ny < 0) status = -1;
        else if (occ[nx * W + ny] != 0) status = -3;   // state > 0 (agents own their cell)
        else if (is_obst(nx, ny)) status = -2;
        else {
          occ[ax * W + ay] = 0;
          occ[nx * W + ny] = (uint8_t)(aid + 1);
          pos[aid] = make_int2(nx, ny);
          if (gg.x == nx && gg.y == ny) status = 1;
          else if (gg.x == ax && gg.y == ay) status = 2;
          else status = 0;
        }
      }
      flag[0] = status;
    }
    wave_fence();
    status = flag[0];
    const int ax = pos[aid].x, ay = pos[aid].y;
    const int2 gg = gl[aid];
    // ---- done: every agent on its goal (:159-166) ----
    bool off = false;
    for (int b = lane; b < N; b += 64) off |= (pos[b].x != gl[b].x) || (pos[b].y != gl[b].y);
    const bool done = __ballot(off) == 0;
    // ---- _observe (:343-386) ----
    const int tr = ax - s / 2, tc = ay - s / 2;
    if (a.obs) {
      for (int i = lane; i < s * s; i += 64) goals_plane[i] = 0;
      wave_fence();
      for (int b = lane; b < N; b += 64) {  // visible agents' goals, clamped into view (:374-378)
        if (b == aid) continue;
        const int br = pos[b].x, bc = pos[b].y;
        if (br >= tr && br < tr + s && bc >= tc && bc < tc + s) {
          const int mr = max(tr, min(tr + s - 1, gl[b].x));
          const int mc = max(tc, min(tc + s - 1, gl[b].y));
          goals_plane[(mr - tr) * s + (mc - tc)] = 1;
        }
      }
      wave_fence();
      uint8_t* o = a.obs + ek * 4 * s * s;
      for (int i = lane; i < s * s; i += 64) {
        const int r = tr + i / s, c = tc + i % s;
        uint8_t poss = 0, goal = 0, ob = 0;
        if (r >= H || r < 0 || c >= W || c < 0) {
          ob = 1;  // :356-359
        } else {
          const bool agent = occ[r * W + c] != 0;
          if (!agent && is_obst(r, c)) ob = 1;    // :360-362
          if (agent) poss = 1;                    // :363-365, 369-372
          if (r == gg.x && c == gg.y) goal = 1;   // :366-368
        }
        o[i] = poss;
        o[s * s + i] = goal;
        o[2 * s * s + i] = goals_plane[i];
        o[3 * s * s + i] = ob;
      }
    }
    if (lane == 0) {
      // ---- reward (:579-596), JOINT = False; stay-on-goal blocking term = 0 ----
      double rew;
      if (act == 0) rew = status == 1 ? GOAL_REWARD + 0 : IDLE_COST;
      else if (status == 1) rew = GOAL_REWARD;
      else if (status < 0) rew = COLLISION_REWARD;
      else rew = ACTION_COST;
      // ---- _listNextValidActions (:639-667) ----
      uint32_t m = 1u;
      for (int b = 1; b <= 4; ++b) {
        const int nx = ax + dir_r(b), ny = ay + dir_c(b);
        if (nx >= H || nx < 0 || ny >= W || ny < 0) continue;
        if (occ[nx * W + ny] != 0 || is_obst(nx, ny)) continue;
        m |= 1u << b;
      }
      const int opp = act == 1 ? 3 : act == 2 ? 4 : act == 3 ? 1 : act == 4 ? 2 : -1;  // :26
      if (opp > 0) m &= ~(1u << opp);
      if (a.reward) a.reward[ek] = rew;
      if (a.done) a.done[ek] = done ? 1 : 0;
      if (a.next_mask) a.next_mask[ek] = (uint8_t)m;
      if (a.on_goal) a.on_goal[ek] = (ax == gg.x && ay == gg.y) ? 1 : 0;
      if (a.valid) a.valid[ek] = status >= 0 ? 1 : 0;
    }
    // goal vector (:379-384): its magnitude needs a LUT load, so lane k & 63 keeps the
    // call's (dx, dy) and the wave writes a block's 64 vectors together (one load
    // latency per 64 calls instead of one per call on the sequential path)
    if (lane == (k & 63)) {
      pend_dx = gg.x - ax;
      pend_dy = gg.y - ay;
    }
    if (a.vec && ((k & 63) == 63 || k + 1 == a.K)) flush_vec(k & ~63, (k & 63) + 1);
    wave_fence();
  }
  wave_fence();
  for (int b = lane; b < N; b += 64) ((int2*)a.pos)[(long long)e * N + b] = pos[b];
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
  h->lds = ((g.hw + 15) & ~15) + ((g.bits_words * 4 + 15) & ~15) + 16 * g.N +
           ((g.s * g.s + 15) & ~15) + 16;
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
  hipLaunchKernelGGL(primal_act_kernel, dim3(h->geo.E), dim3(64), h->lds, (hipStream_t)stream,
                     h->geo, a);
  return check_hip(hipGetLastError(), "primal_act_kernel launch");
}

}  // extern "C"

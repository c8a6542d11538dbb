// partial.hip -- MI355X (gfx950) batched MARL_PARTIAL_ENV step.
//
// The env the reference registers (MARL-curve-main/src/envs/__init__.py:60),
// envs/marl_partial.py (paths below relative to it):
//   step :165-310 -- moves against the PRE-step occupancy (obstacle passable while
//     occupied, :508-512), move / stay / stay-at-goal / env-collision rewards, goal
//     flags, episode limit, BFS-distance "closer" reward (:213-220), node / edge
//     collisions, completion bonus gamma^-(limit - t) (:289-299), fp64 sum in agent
//     order;
//   get_obs :312-375 -- w x w obstacle / agents planes + K nearest agents x 13
//     features (stable sort by L2 distance, self first, -1 padding), float32;
//   get_state :377-387, avail :399-433;
//   goal distances :906-928 -- A* path lengths == BFS levels (bit-parallel BFS).
//
// Layout: one wavefront holds EPW envs (L = pow2ceil(N) lanes per env, lane =
// agent); an env's padded cell map (c = count + 1 - obstacle, c == 0 blocked /
// border) and its dep map (bit 7: obstacle, bits 0-6: the occupant's move) live in
// LDS for the launch; state round-trips HBM between calls.  N > 64 or a side > 256
// (the reference's larger maps and agent counts) take partial_wg_kernel: one
// workgroup per env, the agents' cells in an LDS hash table, the map in HBM.  Every fp64 value is
// computed in the reference's operation order; the completion bonus comes from a host-libm
// LUT (float ** int), sqrt(int) from the device's correctly rounded fp64 sqrt once
// mapfx_partial_create has checked it against host libm on every argument the launch can
// use (else from a host-libm LUT too).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <type_traits>
#include <vector>

#include "internal.h"
#include "mapfx.h"
#include "mapfx_partial.h"


#ifdef PARTIAL_STAMPS
// Diagnostic build only (never the shipped library): s_memtime stamps of partial_kernel's
// phases, block 0 / lane 0, read back with mapfx_partial_debug_stamps().  The stamps stay
// in registers until the end (PST_FLUSH): a store per stamp would make the kernel's
// waits on the vector-memory counter wait for it too.
__device__ unsigned long long g_pstamps[16];
// every wave's s_memrealtime (100 MHz, one clock for the whole device) at stamps 0, 1,
// 8, 10, 11, 13: where the launch's tail comes from
constexpr int PBLK_MAX = 8192, PBLK_N = 6;
__device__ unsigned int g_pblk[PBLK_MAX * PBLK_N];
__device__ __forceinline__ int pblk_slot(int k) {
  return k == 0 ? 0 : k == 1 ? 1 : k == 8 ? 2 : k == 10 ? 3 : k == 11 ? 4 : k == 13 ? 5 : -1;
}
#define PST_DECL uint32_t pst_[14], pbt_[PBLK_N];
#define PST(k)                                                                       \
  do {                                                                               \
    __builtin_amdgcn_sched_barrier(0);                                               \
    unsigned long long t_;                                                           \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");     \
    uint32_t v_;                                                                     \
    asm volatile("v_mov_b32 %0, %1" : "=v"(v_) : "s"((uint32_t)t_));                 \
    if (pblk_slot(k) >= 0) {                                                         \
      unsigned long long r_;                                                         \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r_)::"memory"); \
      uint32_t w_;                                                                   \
      asm volatile("v_mov_b32 %0, %1" : "=v"(w_) : "s"((uint32_t)r_));               \
      pbt_[pblk_slot(k) < 0 ? 0 : pblk_slot(k)] = w_;                                \
    }                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                               \
    pst_[(k)] = v_;                                                                  \
  } while (0)
#define PST_FLUSH()                                                                  \
  do {                                                                               \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                         \
      for (int k_ = 0; k_ < 14; ++k_) g_pstamps[k_] = pst_[k_];                      \
    if (lane64 == 0 && gw < PBLK_MAX)                                                \
      for (int k_ = 0; k_ < PBLK_N; ++k_) g_pblk[gw * PBLK_N + k_] = pbt_[k_];         \
  } while (0)
extern "C" int mapfx_partial_debug_stamps(unsigned long long* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_pstamps), sizeof(unsigned long long) * 16) ==
                 hipSuccess ? 0 : -1;
}
// n_blocks x 6 realtime stamps (diagnostic build)
extern "C" int mapfx_partial_debug_blocks(unsigned int* host_out, int n_blocks) {
  if (n_blocks < 0 || n_blocks > PBLK_MAX) return -1;
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_pblk), sizeof(unsigned int) * PBLK_N * n_blocks) ==
                 hipSuccess ? 0 : -1;
}
#else
#define PST_DECL
#define PST(k) \
  do {         \
  } while (0)
#define PST_FLUSH() \
  do {              \
  } while (0)
#endif

namespace {

constexpr int NF = 13;   // KNN features per agent (:81)
constexpr int FR = 12;   // per-agent feature row in LDS (all but the pairwise distance)
constexpr int BONUS_EXTRA = 65536;  // completion-bonus LUT entries past the episode limit
constexpr int PARTIAL_MAX_WPB = 4;  // partial_kernel: waves per block (g.wpb <= this)

struct PGeo {
  int H, W, N, E;
  int L, lshift, EPW;
  int P, pl, pitch, rows, wpr;       // padded LDS map
  int bits_words, map_shared;
  long long map_stride;
  int map_env_bytes, bits_env_bytes, feat_env_bytes, pos_env_bytes, rew_env_bytes, stage_env_bytes, stage_lanes;
  int off_map, off_dep, off_bits, off_feat, off_pos, off_rew, off_stage, lds;  // off_stage < 0: none
  int off_sqrt;                      // float32 sqrt(0 .. sq_max) per wave (fast path), < 0: none
  int win, K, D, limit, hw;          // window, knn, obs dim, episode limit, H*W
  double move_rew, stay_rew, stay_goal_rew, nc_rew, ec_rew, env_rew;
  int sq_max, bonus_len;             // LUT sizes
  int gd32;                          // goal-distance tables are int32 (H * W > 32767)
  int gd8;                           // ... u8 (H * W <= 255: 255 = -1), else int16
  int big;                           // workgroup-per-env path (N > 64 or H, W > 256), map in HBM
  int hs_log, wg_lds, huge_lds;      // its LDS hash size (log2), block LDS; huge-map BFS LDS
  uint32_t m_wpr;                    // ceil(2^32 / wpr): wi / wpr = umulhi(wi, m_wpr) below rows * wpr
  int wpb;                           // partial_kernel: waves per block (each with g.lds of LDS)
};

struct PArgs {
  int32_t* pos;
  const int32_t* goal;
  const int32_t* init_pos;
  int32_t* steps;
  uint8_t* at_goal;
  uint8_t* done;
  int32_t* goal_cost;
  uint8_t* node;
  int32_t* edge;
  int32_t* t;
  uint8_t* terminated;
  int32_t* total_coll;
  const uint8_t* bits;
  const void* gd;  // u8, int16 or int32 (g.gd8, g.gd32)
  int32_t* pdist;  // [E][N] goal distance of the current cell (carried), or NULL
  int16_t* pnbr;   // [E][N][4] goal distances of its 4 neighbours (carried with pdist), or NULL
  const void* actions;
  int act_dtype;
  int do_step;       // 0: observe only
  const uint8_t* reset_mask;  // reset pass: envs to reset (NULL = all); nullptr when not resetting
  int do_reset;
  double* reward;
  float* obs;
  float* state;
  uint8_t* avail;
  int32_t* err;
  const double* bonus_lut;  // (complete / gamma ** (limit - t)) * fac, t = 0 .. bonus_len-1
  // runner fusion (mapfx_partial_step_rows): observation rows go to obs_rows + e *
  // obs_env_stride (an EpisodeBatch time row) for the envs with obs_mask[e] != 0,
  // instead of the contiguous `obs`
  float* obs_rows;
  long long obs_env_stride;
  const uint8_t* obs_mask;
  // the runner's fused actions (mapfx_partial_step_runner; act_row NULL otherwise)
  mapfx_runner_acts ra;
};

// where env e's observation rows go ([N][D] floats), or nullptr when not written
// (partial_kernel: the caller has read obs_mask[e] with the launch's other loads)
template <bool ROWS = true>
__device__ __forceinline__ float* obs_env_nomask(const PArgs& a, int e, int D, int N) {
  if (ROWS && a.obs_rows) return a.obs_rows + (long long)e * a.obs_env_stride;
  return a.obs ? a.obs + (long long)e * N * D : nullptr;
}
__device__ __forceinline__ float* obs_env(const PArgs& a, int e, int D, int N) {
  if (a.obs_rows) return (a.obs_mask && !a.obs_mask[e]) ? nullptr : a.obs_rows + (long long)e * a.obs_env_stride;
  return a.obs ? a.obs + (long long)e * N * D : nullptr;
}

__device__ inline int load_act(const void* p, int dtype, long long idx) {
  if (dtype == MAPFX_I8) return (int)((const int8_t*)p)[idx];
  if (dtype == MAPFX_I32) return ((const int32_t*)p)[idx];
  const long long v = ((const int64_t*)p)[idx];
  return (v < -1 || v > 5) ? -1 : (int)v;
}

// The step's action of agent `ag` of env `env` (oa = env * N + ag).  The runner's fused
// form (a.ra.act_row): row act_row[env] of the MAC's output, recorded into the
// EpisodeBatch's actions / actions_onehot rows at ts (parallel_runner.py:104-110 and the
// OneHot preprocess); an env outside bs stays (it has terminated: nothing of it is
// recorded again).  Values outside 0..4 come back as -1 (the env is then skipped, :174).
__device__ inline int step_action(const PArgs& a, int env, int ag, long long oa) {
  if (!a.ra.act_row) return load_act(a.actions, a.act_dtype, oa);
  const int row = a.ra.act_row[env];
  if (row < 0) return 4;
  const long long i = (long long)row * a.ra.act_row_stride + ag;
  const long long v = a.act_dtype == MAPFX_I8 ? (long long)((const int8_t*)a.actions)[i]
                      : a.act_dtype == MAPFX_I32 ? (long long)((const int32_t*)a.actions)[i]
                                                 : ((const int64_t*)a.actions)[i];
  if (a.ra.ep_actions)
    a.ra.ep_actions[(long long)env * a.ra.ep_actions_sb + (long long)a.ra.ts * a.ra.ep_actions_st + ag] = v;
  if (a.ra.ep_onehot) {
    float* oh = a.ra.ep_onehot + (long long)env * a.ra.ep_onehot_sb + (long long)a.ra.ts * a.ra.ep_onehot_st +
                (long long)ag * 5;
#pragma unroll
    for (int k = 0; k < 5; ++k) oh[k] = v == k ? 1.0f : 0.0f;
  }
  return (v < 0 || v > 4) ? -1 : (int)v;
}

__device__ inline void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// sqrt(n) of a non-negative integer n <= sq_max in fp64 (math.sqrt of the reference's
// squared distances): the device's correctly rounded sqrt, which mapfx_partial_create
// checks bit for bit against host libm on all of 0 .. sq_max (it refuses the
// configuration otherwise).  Computed, not loaded: a table load here would make every
// later wait on the vector-memory counter also wait for the loads issued before it.
__device__ __forceinline__ double isqrt_f64(int n) { return sqrt((double)n); }

// the action (int64 as (lo, hi), int8 / int32 sign-extended into hi): 0..4, or -1 for
// any value outside 0..4 (the env is then skipped, :174)
__device__ __forceinline__ int act_decode(int lo, int hi) { return ((uint32_t)lo <= 4u && hi == 0) ? lo : -1; }
// the action as the int64 the EpisodeBatch records
__device__ __forceinline__ long long act_value(int lo, int hi) {
  return (long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Cross-lane sums inside an env's L-lane group without the LDS pipeline: DPP moves
// within 16-lane rows (L <= 16: an env's lanes never leave their row), else shuffles.
template <int CTRL>
__device__ __forceinline__ int dpp_mov(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ int group_sum(int x, int L) {
  if (L == 16) {  // row_ror 8, 4, 2, 1
    x += dpp_mov<0x128>(x);
    x += dpp_mov<0x124>(x);
    x += dpp_mov<0x122>(x);
    return x + dpp_mov<0x121>(x);
  }
  if (L == 8) {  // quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror
    x += dpp_mov<0xB1>(x);
    x += dpp_mov<0x4E>(x);
    return x + dpp_mov<0x141>(x);
  }
  if (L == 4) {
    x += dpp_mov<0xB1>(x);
    return x + dpp_mov<0x4E>(x);
  }
  if (L == 2) return x + dpp_mov<0xB1>(x);
  if (L == 1) return x;
  for (int o = 1; o < L; o <<= 1) x += __shfl_xor(x, o);
  return x;
}
// `sum(rewards)` (:310): the naive left fold 0.0 + r[0] + r[1] + ... + r[N-1] in agent
// order, valid in each env's agent-0 lane; r[k] arrives by a DPP row shift (lane i reads
// lane i + k of its row), so L <= 16 (callers fold through LDS otherwise)
template <int K>
__device__ __forceinline__ double row_shl_f64(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const int lo = dpp_mov<0x100 + K>((int)(uint32_t)b);
  const int hi = dpp_mov<0x100 + K>((int)(uint32_t)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo));
}
template <int K>
__device__ __forceinline__ void fold_from(double& R, double x, int N) {
  if constexpr (K < 16) {
    if (K < N) R = R + row_shl_f64<K>(x);
    fold_from<K + 1>(R, x, N);
  }
}
// The same fold over a lane group of LG lanes known at compile time: every lane of the
// group past the env's N agents holds 0.0, and R is never -0.0 (it starts as 0.0 + r[0],
// and in round-to-nearest a sum is -0.0 only when both terms are), so R + 0.0 == R
// exactly and all LG - 1 shifts are folded with no per-term test of N (which cost a
// branch per term)
template <int K, int LG>
__device__ __forceinline__ void fold_all(double& R, double x) {
  if constexpr (K < LG) {
    R = R + row_shl_f64<K>(x);
    fold_all<K + 1, LG>(R, x);
  }
}
// edge collisions against every other lane of a 16-lane row (lane i sees lane (i + k) % 16
// for k = 1..15; lanes past N hold an unmoved cell and never match a moving agent)
template <int K>
__device__ __forceinline__ void dpp_edge_scan(int cur, int nc, int& e) {
  if constexpr (K < 16) {
    const int oj = dpp_mov<0x120 + K>(cur), nj = dpp_mov<0x120 + K>(nc);
    e += (oj == nc) & (nj == cur);
    dpp_edge_scan<K + 1>(cur, nc, e);
  }
}
// LG: the lane group when known at compile time (lanes past N must then hold 0.0), else 0
template <int LG>
__device__ __forceinline__ double row_fold(double x, int N) {
  double R = 0.0 + x;
  if constexpr (LG > 0 && LG <= 16) fold_all<1, LG>(R, x);
  else fold_from<1>(R, x, N);
  return R;
}

// goal distance of neighbour `act` (0 up, 1 down, 2 left, 3 right) from the carried
// pnbr entry (4 x int16 as two words)
__device__ __forceinline__ int nbr_dist(uint2 nb, int act) {
  const uint32_t w = act < 2 ? nb.x : nb.y;
  return (int)(int16_t)(uint16_t)((act & 1) ? (w >> 16) : (w & 0xFFFFu));
}

// entry i of a goal table: u8 while H * W <= 255 (a path is shorter than H * W cells;
// 255 stands for -1, obstacle / unreachable), int16 up to 32767 cells, else int32
__device__ __forceinline__ int gd_entry(const PGeo& g, const void* gd, long long i) {
  if (g.gd8) {
    const int v = ((const uint8_t*)gd)[i];
    return v == 255 ? -1 : v;
  }
  return g.gd32 ? ((const int32_t*)gd)[i] : (int)((const int16_t*)gd)[i];
}
// goal distance of cell `cell` in agent `oa`'s table
__device__ __forceinline__ int goal_dist_at(const PGeo& g, const void* gd, long long oa, int cell) {
  return gd_entry(g, gd, oa * g.hw + cell);
}
// the same with the table width known at compile time (GDE bytes: 1 u8, 2 int16; 0: run
// time): a single load with no branch around it
template <int GDE>
__device__ __forceinline__ int gd_entry_t(const PGeo& g, const void* gd, long long i) {
  if constexpr (GDE == 1) {
    const int v = ((const uint8_t*)gd)[i];
    return v == 255 ? -1 : v;
  } else if constexpr (GDE == 2) {
    return ((const int16_t*)gd)[i];
  } else {
    return gd_entry(g, gd, i);
  }
}

// The step's goal-path distances (:227-233) with the current cell's distance carried in
// the state (mapfx_partial_state.pdist, the reference's _new_pdist of the last step):
// opd is that value, npd = opd unless the agent moved, when it is the table entry of the
// target cell -- looked up speculatively as soon as the position and action are loaded
// (the lookup's latency then overlaps the map build).  Every non-step pass (reset,
// observe: positions may have been rewritten, e.g. by output mode's repair) refreshes
// the carried value from the table; PD_NONE (a state never reset) falls back to it too.
constexpr int PD_NONE = (int)0x80000000;

// The move target of action `act` from (r, c) when it lies on the grid (-1 otherwise):
// the cell whose distance a moving agent's npd is.
__device__ __forceinline__ int move_target(const PGeo& g, int r, int c, int act) {
  if (act < 0 || act > 3) return -1;
  const int tr = r + (act == 0 ? -1 : act == 1 ? 1 : 0);
  const int tc = c + (act == 2 ? -1 : act == 3 ? 1 : 0);
  return (tr < 0 || tr >= g.H || tc < 0 || tc >= g.W) ? -1 : tr * g.W + tc;
}

// ---------------------------------------------------------------------------
// BFS distance tables: one wave per (env, agent), lane r holds row r of the grid
// as a 64-bit mask; each level expands the frontier by shifts (same row) and
// shuffles (rows r-1, r+1).  Distances go to LDS then out, row-major int16.
// ---------------------------------------------------------------------------
template <typename DT>
__global__ void __launch_bounds__(64) partial_bfs_kernel(PGeo g, const uint8_t* bits,
                                                         const int32_t* goal, const uint8_t* mask,
                                                         DT* gd) {
  __shared__ int16_t dist[64 * 64];
  const int pair = blockIdx.x;  // env * N + agent
  const int env = pair / g.N;
  if (mask && !mask[env]) return;  // uniform per block
  const int r = threadIdx.x;
  const int H = g.H, W = g.W;
  const uint64_t wmask = W == 64 ? ~0ull : ((1ull << W) - 1ull);
  // free cells of row r
  uint64_t freem = 0;
  if (r < H) {
    const uint8_t* b = bits + (g.map_shared ? 0 : (long long)env * g.map_stride);
    for (int c = 0; c < W; ++c) {
      const int idx = r * W + c;
      if (!((b[idx >> 3] >> (idx & 7)) & 1)) freem |= 1ull << c;
    }
  }
  for (int i = r; i < H * W; i += 64) dist[i] = -1;
  wave_fence();
  const int gr = goal[2 * pair], gc = goal[2 * pair + 1];
  uint64_t front = (r == gr && ((freem >> gc) & 1)) ? (1ull << gc) : 0ull;
  uint64_t seen = front;
  if (front) dist[r * W + gc] = 0;
  int level = 0;
  while (__ballot(front != 0)) {
    ++level;
    const uint64_t up = __shfl_up(front, 1);    // row r-1
    const uint64_t dn = __shfl_down(front, 1);  // row r+1
    uint64_t nxt = (front << 1) | (front >> 1);
    if (r > 0) nxt |= up;
    if (r < 63) nxt |= dn;
    nxt &= freem & wmask & ~seen;
    if (r >= H) nxt = 0;
    seen |= nxt;
    for (uint64_t m = nxt; m; m &= m - 1) dist[r * W + __builtin_ctzll(m)] = (int16_t)level;
    front = nxt;
  }
  wave_fence();
  DT* out = gd + (long long)pair * g.hw;
  for (int i = r; i < g.hw; i += 64) out[i] = (DT)dist[i];
}

// Maps wider or taller than 64 (up to 256 x 256): one 256-thread workgroup per
// (env, agent); thread r holds row r as four 64-bit masks, the frontier rows are
// exchanged through LDS (double-buffered, one barrier per level), distances go
// straight to the table in global memory (its cells were set to -1 first).
constexpr int BIGW = 4;  // 64-bit words per row: W <= 256
template <typename DT>
__global__ void __launch_bounds__(256) partial_bfs_big_kernel(PGeo g, const uint8_t* bits,
                                                              const int32_t* goal, const uint8_t* mask,
                                                              DT* gd) {
  __shared__ uint64_t front[2][256][BIGW];
  const int pair = blockIdx.x;  // env * N + agent
  const int env = pair / g.N;
  if (mask && !mask[env]) return;  // uniform per block
  const int r = threadIdx.x;
  const int H = g.H, W = g.W;
  DT* out = gd + (long long)pair * g.hw;
  uint64_t freem[BIGW], seen[BIGW], cur[BIGW];
#pragma unroll
  for (int k = 0; k < BIGW; ++k) freem[k] = seen[k] = cur[k] = 0;
  if (r < H) {
    const uint8_t* b = bits + (g.map_shared ? 0 : (long long)env * g.map_stride);
    for (int c = 0; c < W; ++c) {
      const int idx = r * W + c;
      if (!((b[idx >> 3] >> (idx & 7)) & 1)) freem[c >> 6] |= 1ull << (c & 63);
    }
    for (int c = 0; c < W; ++c) out[r * W + c] = -1;
  }
  const int gr = goal[2 * pair], gc = goal[2 * pair + 1];
  if (r == gr && ((freem[gc >> 6] >> (gc & 63)) & 1)) {
    cur[gc >> 6] = 1ull << (gc & 63);
    seen[gc >> 6] = cur[gc >> 6];
    out[r * W + gc] = 0;
  }
#pragma unroll
  for (int k = 0; k < BIGW; ++k) front[0][r][k] = cur[k];
  __syncthreads();
  int level = 0, buf = 0;
  bool any = true;
  while (any) {
    ++level;
    uint64_t nxt[BIGW];
#pragma unroll
    for (int k = 0; k < BIGW; ++k) {
      // same row: cells c-1 / c+1 (carries across the 64-bit words)
      const uint64_t lft = (cur[k] << 1) | (k > 0 ? cur[k - 1] >> 63 : 0ull);
      const uint64_t rgt = (cur[k] >> 1) | (k + 1 < BIGW ? cur[k + 1] << 63 : 0ull);
      const uint64_t up = r > 0 ? front[buf][r - 1][k] : 0ull;
      const uint64_t dn = r + 1 < 256 ? front[buf][r + 1][k] : 0ull;
      nxt[k] = (lft | rgt | up | dn) & freem[k] & ~seen[k];
    }
    if (r >= H) {
#pragma unroll
      for (int k = 0; k < BIGW; ++k) nxt[k] = 0;
    }
    bool mine = false;
#pragma unroll
    for (int k = 0; k < BIGW; ++k) {
      seen[k] |= nxt[k];
      cur[k] = nxt[k];
      front[buf ^ 1][r][k] = nxt[k];
      mine |= nxt[k] != 0;
      for (uint64_t m = nxt[k]; m; m &= m - 1) out[r * W + 64 * k + __builtin_ctzll(m)] = (DT)level;
    }
    buf ^= 1;
    any = __syncthreads_or(mine ? 1 : 0) != 0;
  }
}

// Maps larger than 256 on a side (the reference ships brc202d 481 x 530, orz900d
// 656 x 1491, w_woundedcoast 578 x 642, ...): one 512-thread workgroup per (env,
// agent), thread t owns rows t and t + 512 (H <= 1024), each row as up to 24 64-bit
// words (W <= 1536).  The frontier rows live in LDS (H x words x 8 bytes: 126 KB for
// orz900d); every thread keeps its rows' "free and not yet reached" masks and the
// next frontier in registers, so a level is one LDS read phase, a barrier, one
// write phase and the termination test.  Grid graphs are bipartite and unweighted:
// level-synchronous expansion gives exactly the A* / BFS path lengths (:906-928).
constexpr int HUGE_WORDS = 24;
constexpr int HUGE_THREADS = 512;
template <typename DT>
__global__ void __launch_bounds__(HUGE_THREADS) partial_bfs_huge_kernel(PGeo g, const uint8_t* bits,
                                                                        const int32_t* goal,
                                                                        const uint8_t* mask, DT* gd) {
  extern __shared__ __align__(16) unsigned char lds[];
  uint64_t* front = (uint64_t*)lds;  // [H][WW]
  const int pair = blockIdx.x;       // env * N + agent
  const int env = pair / g.N;
  if (mask && !mask[env]) return;    // uniform per block
  const int tid = threadIdx.x;
  const int H = g.H, W = g.W, WW = (W + 63) >> 6;
  DT* out = gd + (long long)pair * g.hw;
  const uint64_t* b64 = (const uint64_t*)(bits + (g.map_shared ? 0 : (long long)env * g.map_stride));
  const long long nb64 = (g.map_stride + 7) / 8;  // whole u64 words of one env's bitmap
  for (int i = tid; i < g.hw; i += HUGE_THREADS) out[i] = (DT)-1;
  for (int i = tid; i < H * WW; i += HUGE_THREADS) front[i] = 0ull;
  uint64_t allow[2][HUGE_WORDS];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = tid + j * HUGE_THREADS;
#pragma unroll
    for (int k = 0; k < HUGE_WORDS; ++k) {
      allow[j][k] = 0ull;
      if (r < H && k < WW) {  // bits r*W + 64k .. of the bitmap, 1 = obstacle
        const long long p = (long long)r * W + 64 * k;
        const long long wi = p >> 6;
        const int sh = (int)(p & 63);
        const uint64_t lo = b64[wi];
        const uint64_t hi = (sh && wi + 1 < nb64) ? b64[wi + 1] : 0ull;
        const uint64_t word = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
        const int nc = min(64, W - 64 * k);
        const uint64_t cols = nc == 64 ? ~0ull : ((1ull << nc) - 1ull);
        allow[j][k] = ~word & cols;
      }
    }
  }
  __syncthreads();  // the -1 fill and the zeroed frontier come first
  const int gr = goal[2 * pair], gc = goal[2 * pair + 1];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (tid + j * HUGE_THREADS == gr) {
#pragma unroll
      for (int k = 0; k < HUGE_WORDS; ++k) {
        if (k == (gc >> 6) && ((allow[j][k] >> (gc & 63)) & 1ull)) {
          allow[j][k] &= ~(1ull << (gc & 63));
          front[gr * WW + k] = 1ull << (gc & 63);
          out[gr * W + gc] = (DT)0;
        }
      }
    }
  }
  __syncthreads();
  int level = 0;
  bool any = true;
  while (any) {
    ++level;
    uint64_t nxt[2][HUGE_WORDS];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = tid + j * HUGE_THREADS;
#pragma unroll
      for (int k = 0; k < HUGE_WORDS; ++k) {
        nxt[j][k] = 0ull;
        if (r < H && k < WW) {
          const uint64_t* fr = front + r * WW;
          const uint64_t cur = fr[k];
          const uint64_t lft = (cur << 1) | (k > 0 ? fr[k - 1] >> 63 : 0ull);
          const uint64_t rgt = (cur >> 1) | (k + 1 < WW ? fr[k + 1] << 63 : 0ull);
          const uint64_t up = r > 0 ? fr[k - WW] : 0ull;
          const uint64_t dn = r + 1 < H ? fr[k + WW] : 0ull;
          nxt[j][k] = (lft | rgt | up | dn) & allow[j][k];
        }
      }
    }
    __syncthreads();  // every read of this level's frontier is done
    bool mine = false;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = tid + j * HUGE_THREADS;
#pragma unroll
      for (int k = 0; k < HUGE_WORDS; ++k) {
        if (r < H && k < WW) {
          front[r * WW + k] = nxt[j][k];
          allow[j][k] &= ~nxt[j][k];
          mine |= nxt[j][k] != 0ull;
          for (uint64_t m = nxt[j][k]; m; m &= m - 1) out[r * W + 64 * k + __builtin_ctzll(m)] = (DT)level;
        }
      }
    }
    any = __syncthreads_or(mine ? 1 : 0) != 0;
  }
}

// ---------------------------------------------------------------------------
// Workgroup-per-env step for what the wave kernel cannot hold: N > 64 agents or a
// side > 256 cells (SURVEY.md §8(f) F1 at the reference's full range).  One
// 256-thread workgroup per env, thread t owns agents t, t + 256, ... (APL <= 4:
// N <= 1024).  No dense map in LDS: the obstacle bitmap is read from HBM and the
// agents' cells live in an LDS hash table (open addressing, keys = row * W + col,
// >= 4 slots per agent) carrying per cell the PRE-step count, the POST-step count
// and the move of a single pre-step occupant (the edge test's fast case), rebuilt
// every launch.  Same operation order as partial_kernel for every fp64 value.
// ---------------------------------------------------------------------------
constexpr int WG_THREADS = 256;
constexpr uint32_t HEMPTY = 0xFFFFFFFFu;
constexpr uint32_t HPRE = 1u, HPOST = 1u << 11, HDEP_SH = 22;  // val = pre | post << 11 | dep << 22

__device__ __forceinline__ uint32_t hslot0(uint32_t key, int hs_log) {
  return (key * 0x9E3779B1u) >> (32 - hs_log);
}
// the slot of `key`, inserted if absent
__device__ __forceinline__ int hinsert(uint32_t* keys, int hs_log, uint32_t key) {
  const uint32_t msk = (1u << hs_log) - 1u;
  uint32_t s = hslot0(key, hs_log);
  while (true) {
    const uint32_t k = keys[s];
    if (k == key) return (int)s;
    if (k == HEMPTY) {
      const uint32_t old = atomicCAS(&keys[s], HEMPTY, key);
      if (old == HEMPTY || old == key) return (int)s;
    }
    s = (s + 1) & msk;
  }
}
// the value of `key` (0 when absent); all insertions done
__device__ __forceinline__ uint32_t hlookup(const uint32_t* keys, const uint32_t* vals, int hs_log, uint32_t key) {
  const uint32_t msk = (1u << hs_log) - 1u;
  uint32_t s = hslot0(key, hs_log);
  while (true) {
    const uint32_t k = keys[s];
    if (k == key) return vals[s];
    if (k == HEMPTY) return 0u;
    s = (s + 1) & msk;
  }
}

template <int WIN, int APL>
__global__ void __launch_bounds__(WG_THREADS) partial_wg_kernel(PGeo g, PArgs a) {
  extern __shared__ __align__(16) unsigned char lds[];
  constexpr int H2 = WIN / 2, WW = WIN * WIN;
  const int tid = threadIdx.x, env = blockIdx.x, N = g.N, H = g.H, W = g.W;
  const int hs = 1 << g.hs_log;
  uint32_t* keys = (uint32_t*)lds;                    // [hs]
  uint32_t* vals = keys + hs;                         // [hs]
  int* oldL = (int*)(vals + hs);                      // [N] pre-step cell (edge scan)
  int* newL = oldL + N;                               // [N] post-step cell
  int2* posL = (int2*)(newL + N);                     // [N] post-step (row, col) (KNN)
  float* feat = (float*)(posL + N);                   // [N][FR]
  double* rewL = (double*)(((uintptr_t)(feat + N * FR) + 15) & ~(uintptr_t)15);  // [N]
  int* red = (int*)(rewL + N);                        // [8] block reductions
  const uint8_t* bm = a.bits + (g.map_shared ? 0 : (long long)env * g.map_stride);
  const auto obstacle = [&](int rr, int cc) {  // 1 outside the grid or on a static obstacle
    if (rr < 0 || rr >= H || cc < 0 || cc >= W) return 1u;
    const int idx = rr * W + cc;
    return (uint32_t)((bm[idx >> 3] >> (idx & 7)) & 1u);
  };

  int r[APL], c[APL], gr[APL], gc[APL], ir[APL], ic[APL], steps[APL], gcost[APL], edge[APL];
  int pd[APL];  // goal distance of the current cell (carried, see PD_NONE)
  bool has[APL], at_goal[APL], dn[APL];
  uint32_t node[APL];
  const bool reset_me = a.do_reset && (!a.reset_mask || a.reset_mask[env]);
  int tcur = a.t[env], total = a.total_coll[env];
  bool term = a.terminated[env] != 0;
  if (reset_me) {
    tcur = 0;
    term = false;
    total = 0;
  }
#pragma unroll
  for (int k = 0; k < APL; ++k) {
    const int ag = tid + k * WG_THREADS;
    has[k] = ag < N;
    r[k] = c[k] = gr[k] = gc[k] = ir[k] = ic[k] = steps[k] = edge[k] = 0;
    gcost[k] = -1;
    pd[k] = PD_NONE;
    at_goal[k] = dn[k] = false;
    node[k] = 0;
    if (has[k]) {
      const long long oa = (long long)env * N + ag;
      const int2 q = ((const int2*)a.goal)[oa], ip = ((const int2*)a.init_pos)[oa];
      gr[k] = q.x, gc[k] = q.y, ir[k] = ip.x, ic[k] = ip.y;
      if (reset_me) {  // :125-163
        r[k] = ir[k], c[k] = ic[k];
      } else {
        const int2 p = ((const int2*)a.pos)[oa];
        r[k] = p.x, c[k] = p.y;
        steps[k] = a.steps[oa];
        at_goal[k] = a.at_goal[oa] != 0;
        dn[k] = a.done[oa] != 0;
        gcost[k] = a.goal_cost[oa];
        node[k] = a.node[oa];
        edge[k] = a.edge[oa];
        if (a.pdist && a.do_step) pd[k] = a.pdist[oa];
      }
      if (pd[k] == PD_NONE) pd[k] = goal_dist_at(g, a.gd, oa, r[k] * W + c[k]);
    }
  }
  for (int i = tid; i < hs; i += WG_THREADS) {
    keys[i] = HEMPTY;
    vals[i] = 0u;
  }
  if (tid < 8) red[tid] = 0;
  __syncthreads();
  // pre-step counts (the move test reads the PRE-step occupancy, :508-512)
  int oslot[APL];
#pragma unroll
  for (int k = 0; k < APL; ++k) {
    oslot[k] = 0;
    if (has[k]) {
      oslot[k] = hinsert(keys, g.hs_log, (uint32_t)(r[k] * W + c[k]));
      atomicAdd(&vals[oslot[k]], HPRE);
    }
  }
  __syncthreads();

  // ---- step (:165-310) ----
  int act[APL];
  bool bad = false;
#pragma unroll
  for (int k = 0; k < APL; ++k) {
    act[k] = 4;
    if (a.do_step && has[k]) {
      act[k] = step_action(a, env, tid + k * WG_THREADS, (long long)env * N + tid + k * WG_THREADS);
      if (act[k] < 0 || act[k] > 4) bad = true;
    }
  }
  const bool skip = a.do_step && __syncthreads_or(bad ? 1 : 0) != 0;  // the reference asserts (:174)
  if (a.do_step && !skip) {
    ++tcur;  // :178
    double rew[APL];
    bool moved[APL];
    int pre[APL], nr[APL], ncol[APL];
    uint32_t dnew[APL];
#pragma unroll
    for (int k = 0; k < APL; ++k) {
      rew[k] = 0.0;  // rewards[i] = 0 (:183)
      moved[k] = false;
      pre[k] = 0;
      nr[k] = r[k], ncol[k] = c[k];
      if (has[k] && !dn[k]) {  // :193-211
        ++steps[k];
        bool envc = false;
        if (act[k] != 4) {
          const int tr = r[k] + (act[k] == 0 ? -1 : act[k] == 1 ? 1 : 0);
          const int tc = c[k] + (act[k] == 2 ? -1 : act[k] == 3 ? 1 : 0);
          const bool out = tr < 0 || tr >= H || tc < 0 || tc >= W;
          const int cnt = out ? 0 : (int)(hlookup(keys, vals, g.hs_log, (uint32_t)(tr * W + tc)) & 0x7FFu);
          if (out || (obstacle(tr, tc) && cnt == 0)) envc = true;  // obstacle nobody stands on
          else {
            nr[k] = tr, ncol[k] = tc;
            moved[k] = true;
            pre[k] = cnt;
          }
        }
        if (envc) rew[k] = rew[k] + g.env_rew;                          // :203
        if (act[k] != 4) rew[k] = rew[k] + g.move_rew;                  // :207
        else rew[k] = rew[k] + (at_goal[k] ? g.stay_goal_rew : g.stay_rew);  // :209-212
      }
    }
#pragma unroll
    for (int k = 0; k < APL; ++k) {
      if (!has[k]) continue;
      const int ag = tid + k * WG_THREADS;
      at_goal[k] = nr[k] == gr[k] && ncol[k] == gc[k];  // :214-219
      if (at_goal[k]) gcost[k] = tcur;
      if (tcur >= g.limit) {  // :221-225
        term = true;
        dn[k] = true;
      }
      const long long oa = (long long)env * N + ag;
      const int opd = pd[k];  // :227-233
      const int npd = moved[k] ? goal_dist_at(g, a.gd, oa, nr[k] * W + ncol[k]) : opd;
      rew[k] = rew[k] + (double)(opd - npd) / (double)g.limit;
      pd[k] = npd;
      // the single pre-step occupant's move (0..3, 7: stayed) and the post-step count
      atomicOr(&vals[oslot[k]], (moved[k] ? (uint32_t)act[k] : 7u) << HDEP_SH);
      const int ns = hinsert(keys, g.hs_log, (uint32_t)(nr[k] * W + ncol[k]));
      atomicAdd(&vals[ns], HPOST);
      oldL[ag] = r[k] * W + c[k];
      newL[ag] = nr[k] * W + ncol[k];
    }
    __syncthreads();
    // node / edge collisions (:708-727, :822-857); total += (sum(node) + sum(edge)) // 2 (:239)
    int esum = 0;
#pragma unroll
    for (int k = 0; k < APL; ++k) {
      dnew[k] = 0u;
      if (!has[k]) continue;
      const uint32_t v = hlookup(keys, vals, g.hs_log, (uint32_t)(nr[k] * W + ncol[k]));
      node[k] = ((v >> 11) & 0x7FFu) >= 2u ? 1u : 0u;
      edge[k] = 0;
      if (moved[k] && pre[k] > 0) {
        if (pre[k] == 1) {
          edge[k] = (int)((v >> HDEP_SH) & 7u) == (act[k] ^ 1) ? 1 : 0;
        } else {
          const int oc = r[k] * W + c[k], nc = nr[k] * W + ncol[k];
          for (int j = 0; j < N; ++j) edge[k] += (oldL[j] == nc) & (newL[j] == oc);
        }
      }
      esum += (int)node[k] + edge[k];
    }
    if (esum) atomicAdd(&red[0], esum);
    int nat = 0;
#pragma unroll
    for (int k = 0; k < APL; ++k) nat += (has[k] && at_goal[k]) ? 1 : 0;
    if (nat) atomicAdd(&red[1], nat);
    __syncthreads();
    total += red[0] / 2;
    const bool all_at = red[1] == N;  // :283-299
#pragma unroll
    for (int k = 0; k < APL; ++k) {
      if (!has[k]) continue;
      rew[k] = rew[k] + g.nc_rew * (double)node[k];  // :247
      rew[k] = rew[k] + g.ec_rew * (double)edge[k];  // :249
      if (all_at) {
        dn[k] = true;
        rew[k] = rew[k] + a.bonus_lut[min(tcur, g.bonus_len - 1)];
      }
      rewL[tid + k * WG_THREADS] = rew[k];
      r[k] = nr[k], c[k] = ncol[k];
    }
    if (all_at) term = true;
    __syncthreads();
    if (tid == 0) {  // sum(rewards): naive left fold in agent order (:310)
      double R = 0.0;
      for (int j = 0; j < N; ++j) R = R + rewL[j];
      if (a.reward) a.reward[env] = R;
    }
  } else if (a.do_step && tid == 0) {
    if (a.err) atomicCAS(a.err, 0, env + 1);
    if (a.reward) a.reward[env] = 0.0;
  }
  __syncthreads();
  // post-step occupancy: rebuild the table from the current cells (the step's post
  // counts hold it already; a reset / observe pass counts the positions here)
  if (!(a.do_step && !skip)) {
    for (int i = tid; i < hs; i += WG_THREADS) {
      keys[i] = HEMPTY;
      vals[i] = 0u;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < APL; ++k)
      if (has[k]) atomicAdd(&vals[hinsert(keys, g.hs_log, (uint32_t)(r[k] * W + c[k]))], HPOST);
  }
  // ---- observations of the current state (:312-391) ----
#pragma unroll
  for (int k = 0; k < APL; ++k) {
    if (!has[k]) continue;
    const int ag = tid + k * WG_THREADS;
    const int d0 = gr[k] - r[k], d1 = gc[k] - c[k];
    const double nrm = isqrt_f64(d0 * d0 + d1 * d1);   // :937
    const double ux = nrm == 0.0 ? 0.0 : (double)d0 / nrm;   // :938-941
    const double uy = nrm == 0.0 ? 0.0 : (double)d1 / nrm;
    float* fr = feat + ag * FR;
    fr[0] = (float)r[k]; fr[1] = (float)c[k]; fr[2] = (float)ir[k]; fr[3] = (float)ic[k];
    fr[4] = (float)gr[k]; fr[5] = (float)gc[k]; fr[6] = (float)ux; fr[7] = (float)uy;
    fr[8] = (float)nrm; fr[9] = (float)node[k]; fr[10] = (float)edge[k]; fr[11] = (float)steps[k];
    posL[ag] = make_int2(r[k], c[k]);
  }
  int gsum = 0;
#pragma unroll
  for (int k = 0; k < APL; ++k) gsum += has[k] ? gcost[k] : 0;
  if (tid == 0) red[2] = 0;
  __syncthreads();
  if (gsum) atomicAdd(&red[2], gsum);
  float* const env_obs = obs_env(a, env, g.D, N);
  // the c value of a cell: count + 1 - obstacle, 0 = outside / an obstacle nobody stands on
  const auto cval = [&](int rr, int cc) -> uint32_t {
    if (rr < 0 || rr >= H || cc < 0 || cc >= W) return 0u;
    const uint32_t cnt = (hlookup(keys, vals, g.hs_log, (uint32_t)(rr * W + cc)) >> 11) & 0x7FFu;
    return cnt + 1u - obstacle(rr, cc);
  };
#pragma unroll
  for (int k = 0; k < APL; ++k) {
    if (!has[k]) continue;
    const int ag = tid + k * WG_THREADS;
    if (env_obs) {
      float* o = env_obs + (long long)ag * g.D;
      if constexpr (WIN > 0) {  // window planes (:327-342): OOB / obstacle -> 1; agents -> count
        for (int y = 0; y < WIN; ++y)
          for (int x = 0; x < WIN; ++x) {
            const uint32_t cv = cval(r[k] + y - H2, c[k] + x - H2);
            o[y * WIN + x] = cv == 0 ? 1.0f : 0.0f;
            o[WW + y * WIN + x] = cv == 0 ? 0.0f : (float)(cv - 1u);
          }
      }
      // K nearest agents (:346-372): self first, then the k-1 nearest others by L2
      // distance (sorted() is stable: ties by agent index); rows past min(N, K) = -1
      float* kn = o + 2 * WW;
      const int K = g.K, km1 = min(N, K) - 1;
      for (int q = 0; q < 11; ++q) kn[q] = feat[ag * FR + q];
      kn[11] = (float)(H * W);  // distance to itself (:543-545)
      kn[12] = feat[ag * FR + 11];
      long long prev = -1;
      for (int sI = 1; sI <= km1; ++sI) {
        long long best = 0x7FFFFFFFFFFFFFFFll;
        for (int j = 0; j < N; ++j) {
          if (j == ag) continue;
          const int2 pj = posL[j];
          const int dr = r[k] - pj.x, dc = c[k] - pj.y;
          const long long key = (long long)(dr * dr + dc * dc) * 1024 + j;
          if (key > prev && key < best) best = key;
        }
        prev = best;
        const int j = (int)(best & 1023);
        const int sq = (int)(best >> 10);
        float* row = kn + sI * NF;
        for (int q = 0; q < 11; ++q) row[q] = feat[j * FR + q];
        row[11] = (float)isqrt_f64(sq);
        row[12] = feat[j * FR + 11];
      }
      for (int sI = km1 + 1; sI < K; ++sI)
        for (int q = 0; q < NF; ++q) kn[sI * NF + q] = -1.0f;
    }
    if (a.avail) {  // avail (:399-433): neighbour in bounds and not a free-standing obstacle
      uint32_t m = 16u;
      if (cval(r[k] - 1, c[k])) m |= 1u;
      if (cval(r[k] + 1, c[k])) m |= 2u;
      if (cval(r[k], c[k] - 1)) m |= 4u;
      if (cval(r[k], c[k] + 1)) m |= 8u;
      a.avail[(long long)env * N + ag] = (uint8_t)m;
    }
  }
  __syncthreads();
  if (tid == 0 && a.state) {  // state (:377-387): [total collisions, step count, sum(each goal cost)]
    a.state[3 * env + 0] = (float)total;
    a.state[3 * env + 1] = (float)tcur;
    a.state[3 * env + 2] = (float)red[2];
  }
  // ---- state write-back ----
#pragma unroll
  for (int k = 0; k < APL; ++k) {
    if (!has[k]) continue;
    const long long oa = (long long)env * N + tid + k * WG_THREADS;
    ((int2*)a.pos)[oa] = make_int2(r[k], c[k]);
    a.steps[oa] = steps[k];
    a.at_goal[oa] = at_goal[k] ? 1 : 0;
    a.done[oa] = dn[k] ? 1 : 0;
    a.goal_cost[oa] = gcost[k];
    a.node[oa] = (uint8_t)node[k];
    a.edge[oa] = edge[k];
    if (a.pdist) a.pdist[oa] = pd[k];
  }
  if (tid == 0) {
    a.t[env] = tcur;
    a.terminated[env] = term ? 1 : 0;
    a.total_coll[env] = total;
  }
}

// ---------------------------------------------------------------------------
// Step / observe / reset kernel (one launch = one env step or observation pass).
// ---------------------------------------------------------------------------
// KF / LF: K and lanes-per-env fixed at compile time (0: run-time generic path)
// A block is g.wpb independent waves (no barrier between them): bigger blocks let the
// dispatcher start the launch's waves sooner (one wave per block took ~1.4 us to have
// all 1024 waves of the bench shape running).
// GDE: goal-table entry bytes fixed at compile time (1 u8, 2 int16; 0: run time)
// RUN: the runner's fused actions / post pass and EpisodeBatch observation rows compiled
// in (false: the plain step, whose code then holds none of the runner's pointers: 2043
// -> 1747 VALU instructions)
// The runner's `bs` compaction for the next MAC call (runner.hip runner_compact_kernel's
// work) as the extra FIRST workgroup of the runner step's launch (mapfx_runner_acts
// cmp_*): A = cmp_alive (running before this step) is not written by this launch, so the
// compaction runs beside the env workgroups -- dispatched first, it is done long before
// them -- instead of as a launch after them.  Ascending indices of A, padded with the
// first; per-thread chunks (up to 32 flags held as a bit set between the count and the
// write pass, a 16-flag chunk read as one 16-byte load), a shuffle scan per wave and one
// barrier for the wave totals (blockDim = 64 * wpb, 64 .. 256 threads).
__device__ __forceinline__ void runner_compact_block(const mapfx_runner_acts& ra, unsigned char* lds) {
  const int nt = (int)blockDim.x, tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nw = nt >> 6, B = ra.cmp_B;
  const int chunk = (B + nt - 1) / nt;
  const int lo = min(B, tid * chunk), hi = min(B, lo + chunk);
  const bool held = chunk <= 32;
  uint32_t bits = 0;  // flag b - lo (held chunks)
  int c = 0;
  if (held) {
    if (chunk == 16 && hi - lo == 16 && ((uintptr_t)(ra.cmp_alive + lo) & 15) == 0) {
      const uint4 w = *(const uint4*)(ra.cmp_alive + lo);
      const uint32_t ws4[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // bit 7 of each byte: byte != 0
        const uint32_t nz = (((ws4[i] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | ws4[i]) & 0x80808080u;
        const uint32_t m = nz >> 7;
        bits |= ((m | (m >> 7) | (m >> 14) | (m >> 21)) & 0xFu) << (4 * i);
      }
    } else {
      for (int b = lo; b < hi; ++b) bits |= (ra.cmp_alive[b] ? 1u : 0u) << (b - lo);
    }
    c = __popc(bits);
  } else {
    for (int b = lo; b < hi; ++b) c += ra.cmp_alive[b] ? 1 : 0;
  }
  int x = c;  // inclusive scan over the wave's lanes
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  int* ws = (int*)lds;
  if (lane == 63) ws[wv] = x;
  __syncthreads();
  int off = 0, total = 0;
  for (int i = 0; i < nw; ++i) {
    const int v = ws[i];
    off += i < wv ? v : 0;
    total += v;
  }
  int o = off + x - c;  // exclusive prefix of this thread's chunk
  for (int b = lo; b < hi; ++b) {
    const bool in = held ? ((bits >> (b - lo)) & 1u) != 0 : ra.cmp_alive[b] != 0;
    ra.cmp_bs_inv[b] = in ? o : -1;  // where the next MAC call puts env b's row
    if (in) ra.cmp_bs[o++] = b;
  }
  __syncthreads();  // bs[0] written
  const int64_t first = total > 0 ? ra.cmp_bs[0] : 0;
  for (int j = total + tid; j < B; j += nt) ra.cmp_bs[j] = first;
  if (tid == 0) {
    ra.cmp_counts[0] = total;  // len(bs) = the envs running before this step
    ra.cmp_counts[1] = total;  // = the envs running after the previous one
    ra.cmp_env_steps[0] += total;  // the envs this step steps (env_steps_this_run, :142)
    if (ra.cmp_counts_out) {  // possibly pinned host memory
      ra.cmp_counts_out[0] = total;
      ra.cmp_counts_out[1] = total;
    }
  }
}

template <int WIN, int KF, int LF, int GDE = 0, bool RUN = true>
__global__ void __launch_bounds__(64 * PARTIAL_MAX_WPB) partial_kernel(PGeo g_, PArgs a) {
  int blk = (int)blockIdx.x;
  if constexpr (RUN) {  // the runner's fused compaction: the launch's extra first workgroup
    if (a.ra.cmp_bs && blk-- == 0) {
      extern __shared__ __align__(16) unsigned char lds_cmp[];
      runner_compact_block(a.ra, lds_cmp);
      return;
    }
  }
  PGeo g = g_;
  if constexpr (LF > 0) {  // the fast instances' lane group and K as constants (launch() picks
    g.L = LF;              // them only for g.L == LF, g.K == KF)
    g.lshift = __builtin_ctz(LF);
    g.K = KF;
  }
  extern __shared__ __align__(16) unsigned char lds_blk[];
  constexpr int H2 = WIN / 2;
  const int lane64 = threadIdx.x & 63;
  const int gw = blk * g.wpb + (int)(threadIdx.x >> 6);  // this wave's index
  unsigned char* const lds = lds_blk + (threadIdx.x >> 6) * g.lds;
  const int slot = lane64 >> g.lshift;
  const int ag = lane64 & (g.L - 1);
  const int base = slot << g.lshift;
  const int env = gw * g.EPW + slot;
  const int N = g.N;
  const bool env_ok = slot < g.EPW && env < g.E;
  const bool has = env_ok && ag < N;
  const uint64_t envmask = (g.L == 64 ? ~0ull : ((1ull << g.L) - 1ull)) << base;
  const int pitch = g.pitch;
  const int cs = env_ok ? slot : 0;  // LDS slot (idle lanes alias slot 0, write nothing)

  unsigned char* map = lds + g.off_map + cs * g.map_env_bytes;
  uint32_t* map32 = (uint32_t*)map;
  unsigned char* dep = lds + g.off_dep + cs * g.map_env_bytes;
  uint32_t* dep32 = (uint32_t*)dep;
  uint32_t* bitsL = (uint32_t*)(lds + g.off_bits + cs * g.bits_env_bytes);
  float* feat = (float*)(lds + g.off_feat + cs * g.feat_env_bytes);
  int2* posL = (int2*)(lds + g.off_pos + cs * g.pos_env_bytes);
  double* rewL = (double*)(lds + g.off_rew + cs * g.rew_env_bytes);

  PST_DECL
  PST(0);
  const long long oa = (long long)env * N + ag;
  // ---- every global read of the launch issued up front (idle lanes read entry 0),
  // the bitmap's first words first; optional arrays behind uniform branches, and no
  // loaded value used before the map build: a value tested right after its load would
  // put a wait on the vector-memory counter (in-order: on every load before it) into
  // the prologue ----
  const long long oc_ = has ? oa : 0;
  const int ec_ = env_ok ? env : 0;
  const bool runner = RUN && a.do_step && a.ra.act_row != nullptr;
  const bool post = RUN && a.ra.alive != nullptr;  // the runner's post pass, fused
  const bool nb_carry = a.pnbr && a.pdist && !g.gd32;  // neighbour distances carried
  const uint32_t* bsrc = (const uint32_t*)(a.bits + (g.map_shared ? 0 : (long long)ec_ * g.map_stride));
  const uint32_t bw0 = bsrc[ag < g.bits_words ? ag : 0];  // this lane's first bitmap word
  // the step's action: one 8-byte load of the aligned block that holds it (whatever the
  // dtype: the block lies in the element's page), decoded after the map build; the
  // runner's address needs the env's row of the MAC output first
  const int esh = a.act_dtype == MAPFX_I64 ? 3 : a.act_dtype == MAPFX_I32 ? 2 : 0;
  int arow = 0;
  long long ai = oc_;
  if (runner) {
    arow = a.ra.act_row[ec_];
    ai = (has && arow >= 0) ? (long long)arow * a.ra.act_row_stride + ag : 0;
  }
  const uintptr_t abyte = (uintptr_t)(a.do_step ? a.actions : (const void*)a.pos) + ((uintptr_t)ai << esh);
  const uint2 araw = *(const uint2*)(abyte & ~(uintptr_t)7);
  const int2 q = ((const int2*)a.goal)[oc_];
  const int2 ip = ((const int2*)a.init_pos)[oc_];
  const int2 p0 = ((const int2*)a.pos)[oc_];
  int pd_raw = 0;
  if (a.pdist) pd_raw = a.pdist[oc_];
  uint2 nb0 = make_uint2(0u, 0u);
  if (nb_carry && a.do_step) nb0 = ((const uint2*)a.pnbr)[oc_];
  const int steps0 = a.steps[oc_];
  const uint8_t at_goal0 = a.at_goal[oc_], dn0 = a.done[oc_], node0 = a.node[oc_];
  const int gcost0 = a.goal_cost[oc_], edge0 = a.edge[oc_];
  const int t0 = a.t[ec_], total0 = a.total_coll[ec_];
  const uint8_t term0 = a.terminated[ec_];
  uint32_t om_raw = 1, rm_raw = 1, live_raw = 0;
  if (RUN && a.obs_rows && a.obs_mask) om_raw = a.obs_mask[ec_];
  if (a.do_reset && a.reset_mask) rm_raw = a.reset_mask[ec_];
  double epr_raw = 0.0;
  int64_t epl_raw = 0;
  if (post) {
    live_raw = a.ra.alive[ec_];
    epr_raw = a.ra.ep_return[ec_];
    epl_raw = a.ra.ep_length[ec_];
  }
  if constexpr (KF > 0 && LF > 0) {  // float32 sqrt(0 .. sq_max) for the K-nearest rows
    if (g.off_sqrt >= 0) {            // (:352 math.sqrt), while the loads are in flight
      float* sqt = (float*)(lds + g.off_sqrt);
#pragma unroll 1
      for (int i = lane64; i <= g.sq_max; i += 64) sqt[i] = (float)isqrt_f64(i);
    }
  }
  // ---- LDS map (c format) + dep map (obstacle flag in bit 7) ----
  // (staging the bitmap before the state loads are issued measured slower: 15.73 vs
  // 15.42 us per step)
  if (env_ok) {
    if (ag < g.bits_words) bitsL[ag] = bw0;
    for (int w = ag + g.L; w < g.bits_words; w += g.L) bitsL[w] = bsrc[w];  // maps past 16 x 32 words
  }
  PST(1);
  wave_fence();
  if (env_ok) {
    // word wi of the padded map = row pr, cells 4 pw .. 4 pw + 3 (pr = wi / wpr by a
    // multiply-high, exact below rows * wpr: checked at create); each word's 4 obstacle
    // bits from the two bitmap words around its first cell, every read of a group of
    // 4 words issued before any is used (no branch: off-grid cells are masked)
    const int nw = g.rows * g.wpr;
    for (int w0 = ag; w0 < nw; w0 += 4 * g.L) {
      uint32_t blo[4], bhi[4], vm[4];
      int sh[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int wi = w0 + u * g.L;
        const int pr = (int)__umulhi((uint32_t)wi, g.m_wpr), pw = wi - pr * g.wpr;
        const int rr = pr - g.P, cc = pw * 4 - g.pl;  // the word's grid row, first column
        const bool rin = (unsigned)rr < (unsigned)g.H;
        const int idx = (rin ? rr : 0) * g.W + cc;    // bit of the first cell (>= -8)
        const int iw = idx >> 5;
        blo[u] = bitsL[min(max(iw, 0), g.bits_words)];  // (bitsL has a slack word)
        bhi[u] = bitsL[min(max(iw + 1, 0), g.bits_words)];
        sh[u] = idx & 31;
        const int lv = max(0, -cc), hv = min(4, max(0, g.W - cc));  // on-grid cells lv .. hv - 1
        vm[u] = (rin && lv < hv) ? ((1u << hv) - 1u) & ~((1u << lv) - 1u) : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int wi = w0 + u * g.L;
        if (wi < nw) {
          const uint32_t b4 = (uint32_t)((((uint64_t)bhi[u] << 32) | blo[u]) >> sh[u]) & 0xFu;
          const uint32_t ob4 = (b4 & vm[u]) | (~vm[u] & 0xFu);  // obstacle flags (off the grid: 1)
          const uint32_t f = (ob4 * 0x00204081u) & 0x01010101u;  // bit j -> byte j
          map32[wi] = f ^ 0x01010101u;  // c = 1 - obstacle before agents are added
          dep32[wi] = (f << 7) | 0x7F7F7F7Fu;
        }
      }
    }
  }
  wave_fence();
  PST(2);
  // ---- state (:125-163 for a reset env) ----
  const bool reset_me = env_ok && a.do_reset && rm_raw != 0;
  const bool omask = om_raw != 0;
  const uint8_t live0 = live_raw != 0 ? 1 : 0;
  const double epr0 = epr_raw;
  const int64_t epl0 = epl_raw;
  const int gr = q.x, gc = q.y, ir = ip.x, ic = ip.y;
  int r = 0, c = 0, steps = 0, gcost = -1, edge = 0;
  int pd = PD_NONE;  // goal distance of the current cell (carried)
  bool at_goal = false, dn = false;
  uint32_t node = 0;
  if (has) {
    r = reset_me ? ir : p0.x;
    c = reset_me ? ic : p0.y;
    if (!reset_me) {
      steps = steps0;
      at_goal = at_goal0 != 0;
      dn = dn0 != 0;
      gcost = gcost0;
      node = node0;
      edge = edge0;
      pd = a.pdist ? pd_raw : PD_NONE;  // (pd_raw is 0 without pdist)
    }
  }
  int tcur = (env_ok && !reset_me) ? t0 : 0, total = (env_ok && !reset_me) ? total0 : 0;
  bool term = env_ok && !reset_me && term0 != 0;
  // the action (raw int64 as (alo, ahi); int8 / int32 sign-extended); an env outside
  // the runner's bs stays
  const uint32_t aw = (abyte & 4) ? araw.y : araw.x;
  int alo, ahi;
  if (a.act_dtype == MAPFX_I64) {
    alo = (int)araw.x;
    ahi = (int)araw.y;
  } else if (a.act_dtype == MAPFX_I32) {
    alo = (int)aw;
    ahi = alo >> 31;
  } else {
    alo = (int)(int8_t)(uint8_t)(aw >> ((abyte & 3) * 8));
    ahi = alo >> 31;
  }
  int act = 4;
  if (a.do_step && has && !(runner && arow < 0)) act = act_decode(alo, ahi);
  // goal-path distances (:227-233): a moving agent's npd is its target's entry of the
  // carried neighbour distances; without them (no pnbr, int32 tables, a state never reset)
  // the target's table entry is looked up here, and the current cell's when no carried
  // value applies (every non-step pass refreshes it)
  const bool nb_ok = nb_carry && a.do_step && pd != PD_NONE;
  const bool need_cur = has && (!a.do_step || !a.pdist || pd == PD_NONE);
  int npd_t = 0;
  if (has && !nb_ok) {
    const int tgt = (a.do_step && !dn) ? move_target(g, r, c, act) : -1;
    if (tgt >= 0) npd_t = gd_entry_t<GDE>(g, a.gd, oa * g.hw + tgt);
    if (need_cur) pd = gd_entry_t<GDE>(g, a.gd, oa * g.hw + r * g.W + c);
  }
  PST(3);
  int cur = (r + g.P) * pitch + c + g.pl;
  if (has) atomicAdd(&map32[cur >> 2], 1u << ((cur & 3) * 8));
  wave_fence();
  PST(4);

  // ---- step (:165-310) ----
  double Rsum = 0.0;  // sum(rewards) of the env (agent-0 lane)
  if (a.do_step && env_ok) {
    const bool skip = (__ballot(act < 0) & envmask) != 0;  // the reference asserts (:174)
    if (!skip) {
      ++tcur;  // :178
      double rew = 0.0;  // rewards[i] = 0 (:183)
      bool moved = false;
      int nc = cur;
      uint32_t v = 0;
      if (has && !dn) {  // :193-211
        ++steps;
        bool envc = false;
        if (act != 4) {
          const int d = act == 0 ? -pitch : act == 1 ? pitch : act == 2 ? -1 : 1;
          v = map[cur + d];   // PRE-step occupancy: 0 = out of bounds / free-standing obstacle
          if (v == 0) envc = true;
          else {
            nc = cur + d;
            moved = true;
          }
        }
        if (envc) rew = rew + g.env_rew;                    // :203
        if (act != 4) rew = rew + g.move_rew;               // :207
        else rew = rew + (at_goal ? g.stay_goal_rew : g.stay_rew);  // :209-212
      }
      const int nr = r + (moved ? (act == 0 ? -1 : act == 1 ? 1 : 0) : 0);
      const int ncol = c + (moved ? (act == 2 ? -1 : act == 3 ? 1 : 0) : 0);
      at_goal = has && nr == gr && ncol == gc;              // :214-219
      if (at_goal) gcost = tcur;
      if (tcur >= g.limit) {                                // :221-225
        term = true;
        dn = true;
      }
      if (has) {                                            // :227-233
        const int opd = pd;
        const int npd = moved ? (nb_ok ? nbr_dist(nb0, act) : npd_t) : opd;
        rew = rew + (double)(opd - npd) / (double)g.limit;
        pd = npd;
      }
      // counts move; node / edge collisions (:708-727, :822-857)
      if (has) dep[cur] = (unsigned char)((dep[cur] & 0x80u) | (moved ? (uint32_t)act : 0x7Fu));
      wave_fence();
      if (moved) {
        atomicSub(&map32[cur >> 2], 1u << ((cur & 3) * 8));
        atomicAdd(&map32[nc >> 2], 1u << ((nc & 3) * 8));
      }
      wave_fence();
      PST(5);
      const uint32_t dj = has ? dep[nc] : 0x7Fu;
      const uint32_t cn = has ? map[nc] : 0u;
      node = (has && cn + (dj >> 7) >= 3u) ? 1u : 0u;
      const int pre = (int)v - 1 + (int)(dj >> 7);
      edge = 0;
      const bool suspect = moved && pre > 0;
      if (__ballot(suspect)) {
        if (suspect && pre == 1) edge = (dj & 0x7Fu) == (uint32_t)(act ^ 1) ? 1 : 0;
        if (__ballot(suspect && pre > 1)) {  // stacked pre-occupants: scan the env's agents
          if (g.L == 16) {  // the env is one DPP row: rotate its (old, new) cells past each lane
            int e2 = 0;
            dpp_edge_scan<1>(cur, nc, e2);
            if (suspect && pre > 1) edge += e2;
          } else {
            for (int j = 0; j < N; ++j) {
              const int oj = __shfl(cur, base + j);
              const int nj = __shfl(nc, base + j);
              if (suspect && pre > 1) edge += (oj == nc) & (nj == cur);
            }
          }
        }
      }
      // env sums: total collisions += (sum(node) + sum(edge)) // 2  (:239)
      const int esum = group_sum(has ? (int)node + edge : 0, LF > 0 ? LF : g.L);
      total += esum / 2;
      rew = rew + g.nc_rew * (double)node;  // :247
      rew = rew + g.ec_rew * (double)edge;  // :249
      r = nr;
      c = ncol;
      cur = nc;
      // all at goals: dones, terminated, completion bonus (:283-299)
      const bool all_at = (__ballot(has && !at_goal) & envmask) == 0;
      if (all_at) {
        dn = true;
        term = true;
        const int bi = min(tcur, g.bonus_len - 1);
        rew = rew + a.bonus_lut[bi];
      }
      PST(6);
      // sum(rewards): naive left fold in agent order (:310)
      if (g.L <= 16) {
        const double R = row_fold<LF>(has ? rew : 0.0, N);
        if (ag == 0) {
          if (a.reward) a.reward[env] = R;
          Rsum = R;
        }
      } else {
        if (has) rewL[ag] = rew;
        wave_fence();
        if (ag == 0) {
          double R = 0.0;
          for (int j = 0; j < N; ++j) R = R + rewL[j];
          if (a.reward) a.reward[env] = R;
          Rsum = R;
        }
      }
      PST(7);
    } else {
      if (ag == 0 && a.err) atomicCAS(a.err, 0, env + 1);
      if (ag == 0 && a.reward) a.reward[env] = 0.0;
    }
  }
  wave_fence();
  // the goal distances of the (new) cell's neighbours, carried to the next step: issued
  // here, consumed before the staged copy-out (the observation rows hide their latency)
  // -- unconditional loads (idle lanes read agent 0's table at (0, 0), an off-grid
  // neighbour the cell itself; no branch, so no use of a value can move up to its load)
  // (u8 tables, H * W <= 255: the 4 lookups of an agent fall in one 64-byte table, so one
  // memory request; int16 tables span two)
  const long long gi = oc_ * g.hw + r * g.W + c;
  const int nbd0 = gd_entry_t<GDE>(g, a.gd, gi + (r > 0 ? -g.W : 0));
  const int nbd1 = gd_entry_t<GDE>(g, a.gd, gi + (r + 1 < g.H ? g.W : 0));
  const int nbd2 = gd_entry_t<GDE>(g, a.gd, gi + (c > 0 ? -1 : 0));
  const int nbd3 = gd_entry_t<GDE>(g, a.gd, gi + (c + 1 < g.W ? 1 : 0));

  PST(8);
  // ---- the step's results leave before the observation rows are built: their stores
  // then queue ahead of the rows' copy-out instead of behind it ----
  // avail (:399-433): neighbour in bounds and not a free-standing obstacle
  uint32_t am = 16u;
  if (has && (a.avail || (RUN && a.ra.ep_avail))) {
    if (map[cur - pitch]) am |= 1u;
    if (map[cur + pitch]) am |= 2u;
    if (map[cur - 1]) am |= 4u;
    if (map[cur + 1]) am |= 8u;
    if (a.avail) a.avail[oa] = (uint8_t)am;
  }
  // state (:377-387): [total collisions, step count, sum(each goal cost)]
  const int gsum = group_sum(has ? gcost : 0, LF > 0 ? LF : g.L);
  if (env_ok && ag == 0 && a.state) {
    a.state[3 * env + 0] = (float)total;
    a.state[3 * env + 1] = (float)tcur;
    a.state[3 * env + 2] = (float)gsum;
  }
  // ---- state write-back ----
  if (has) {
    ((int2*)a.pos)[oa] = make_int2(r, c);
    a.steps[oa] = steps;
    a.at_goal[oa] = at_goal ? 1 : 0;
    a.done[oa] = dn ? 1 : 0;
    a.goal_cost[oa] = gcost;
    a.node[oa] = (uint8_t)node;
    a.edge[oa] = edge;
    if (a.pdist) a.pdist[oa] = pd;
    if (runner && arow >= 0) {  // the EpisodeBatch's actions / actions_onehot rows at ts
      const long long v = act_value(alo, ahi);
      if (a.ra.ep_actions)
        a.ra.ep_actions[(long long)env * a.ra.ep_actions_sb + (long long)a.ra.ts * a.ra.ep_actions_st + ag] = v;
      if (a.ra.ep_onehot) {
        float* oh = a.ra.ep_onehot + (long long)env * a.ra.ep_onehot_sb +
                    (long long)a.ra.ts * a.ra.ep_onehot_st + (long long)ag * 5;
#pragma unroll
        for (int k = 0; k < 5; ++k) oh[k] = v == k ? 1.0f : 0.0f;
      }
    }
  }
  if (env_ok && ag == 0) {
    a.t[env] = tcur;
    a.terminated[env] = term ? 1 : 0;
    a.total_coll[env] = total;
  }
  if (post && env_ok) {  // runner_post_kernel (runner.hip) for a running env, fused
    const mapfx_runner_acts& ra = a.ra;
    if (live0) {
      if (ag == 0) {
        if (ra.ep_reward) ra.ep_reward[(long long)env * ra.ep_reward_sb + (long long)ra.ts * ra.ep_reward_st] = (float)Rsum;
        // env_terminated = terminated and not info.get("episode_limit") (parallel_runner.py:146-150):
        // MARL_PARTIAL's info has no "episode_limit" key
        if (ra.ep_term) ra.ep_term[(long long)env * ra.ep_term_sb + (long long)ra.ts * ra.ep_term_st] = term ? 1 : 0;
        ra.ep_return[env] = epr0 + Rsum;
        ra.ep_length[env] = epl0 + 1;
        if (!ra.cmp_bs) ra.alive[env] = term ? 0 : 1;  // (fused compaction: A_out below)
        if (ra.ep_state) {  // update(pre_transition_data, bs, ts + 1): state, avail, filled
          float* d = ra.ep_state + (long long)env * ra.ep_state_sb;
          d[0] = (float)total;
          d[1] = (float)tcur;
          d[2] = (float)gsum;
        }
        if (ra.ep_filled) ra.ep_filled[(long long)env * ra.ep_filled_sb] = 1;
      }
      if (has && ra.ep_avail) {
        int32_t* d = ra.ep_avail + (long long)env * ra.ep_avail_sb + ag * 5;
#pragma unroll
        for (int k = 0; k < 5; ++k) d[k] = (int32_t)((am >> k) & 1u);
      }
    }
    // alive_prev: the stale list for the separate compaction, or, with the compaction
    // fused (cmp_bs), A[(ts + 1) & 1] = running after this step, written for every env
    if (ag == 0) ra.alive_prev[env] = ra.cmp_bs ? (uint8_t)(live0 && !term ? 1 : 0) : live0;
  }
  // ---- observations of the current state (:312-391) ----
  // per-agent feature rows: curr, start, goal, unit vec, norm, node, edge, steps
  if (has) {
    const int d0 = gr - r, d1 = gc - c;
    const double nrm = isqrt_f64(d0 * d0 + d1 * d1);   // :937
    const double ux = nrm == 0.0 ? 0.0 : (double)d0 / nrm;   // :938-941
    const double uy = nrm == 0.0 ? 0.0 : (double)d1 / nrm;
    float* fr = feat + ag * FR;
    fr[0] = (float)r; fr[1] = (float)c; fr[2] = (float)ir; fr[3] = (float)ic;
    fr[4] = (float)gr; fr[5] = (float)gc; fr[6] = (float)ux; fr[7] = (float)uy;
    fr[8] = (float)nrm; fr[9] = (float)node; fr[10] = (float)edge; fr[11] = (float)steps;
    posL[ag] = make_int2(r, c);
  }
  wave_fence();
  PST(9);
  constexpr int WW = WIN * WIN;
  constexpr int DF = (KF > 0 && LF > 0) ? 2 * WW + NF * KF : 1;  // fast-path row length
  float o[DF];
  float* const my_obs = (env_ok && omask) ? obs_env_nomask<RUN>(a, env, (KF > 0 && LF > 0) ? DF : g.D, N) : nullptr;
  // Staged copy-out (fast path): the rows of the envs of a staging group (the whole wave,
  // or each half of it) are one contiguous run of the destination (a.obs), or one run
  // per env (EpisodeBatch rows): each run is staged in LDS as its byte image, at the
  // run's own 16-byte misalignment, and copied with lane-contiguous 16-byte stores --
  // per-lane dword stores of 460-byte rows touch 64 lines each.  The images alias the LDS
  // regions the step is done with (dep onwards).  (Sending the window planes first, while
  // the K-nearest rows are built, measured 19.0 vs 15.2 us: chunks of partial lines.)
  constexpr bool FAST = KF > 0 && LF > 0;
  const bool one_run = !RUN || a.obs_rows == nullptr;
  const bool staged = FAST && (a.obs || (RUN && a.obs_rows)) && g.off_stage >= 0;
  // this lane's row of group gi's image (G lanes per group)
  auto stage_row = [&](int gi, int G, int i0, int i1) {
    const int s0 = (G * gi) >> g.lshift;
    if (has && my_obs && lane64 / G == gi) {
      const int kme = slot - s0;  // this lane's env within the group
      const float* rb = one_run ? a.obs + (long long)(gw * g.EPW + s0) * N * DF : my_obs;
      const uint32_t mis = (uint32_t)(uintptr_t)rb & 15u;
      const int k = one_run ? 0 : kme;
      const int ri = (one_run ? kme * N : 0) + ag;  // row within the run
      uint32_t* row = (uint32_t*)(lds + g.off_stage + k * g.stage_env_bytes + mis + ri * (DF * 4));
#pragma unroll
      for (int i = 0; i < DF; ++i)
        if (i >= i0 && i < i1) row[i] = __float_as_uint(o[i]);
    }
  };
  // copy group gi's runs
  auto copy_runs = [&](int gi, int G) {
    const int s0 = (G * gi) >> g.lshift;
    const int ne = max(0, min(min(G >> g.lshift, g.EPW - s0), g.E - (gw * g.EPW + s0)));  // signed
    const int nrun = one_run ? (ne > 0 ? 1 : 0) : ne;
    const int rowB = DF * 4;
    for (int k = 0; k < nrun; ++k) {
      unsigned char* gdst;
      if (one_run) {
        gdst = (unsigned char*)(a.obs + (long long)(gw * g.EPW + s0) * N * DF);
      } else {  // env s0 + k's destination, from its agent-0 lane (NULL: masked)
        const uint64_t pe = (uint64_t)(uintptr_t)my_obs;
        const int src = (s0 + k) << g.lshift;
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)pe, src);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(pe >> 32), src);
        gdst = (unsigned char*)(uintptr_t)(((uint64_t)hi << 32) | lo);
        if (!gdst) continue;
      }
      const uint32_t mis = (uint32_t)(uintptr_t)gdst & 15u;
      const unsigned char* img = lds + g.off_stage + k * g.stage_env_bytes + mis;
      const int nbytes = (one_run ? ne : 1) * N * rowB;
      const int head = mis ? min(16 - (int)mis, nbytes) : 0;  // a multiple of 4
      const int body = (nbytes - head) & ~15;
      if (lane64 < head / 4) ((uint32_t*)gdst)[lane64] = ((const uint32_t*)img)[lane64];
      const uint4* s4 = (const uint4*)(img + head);  // 16-byte aligned: mis + head
      uint4* g4 = (uint4*)(gdst + head);
      const int n16 = body / 16;
      // four LDS reads in flight per lane before their stores
      for (int i = lane64; i < n16; i += 256) {
        const bool b1 = i + 64 < n16, b2 = i + 128 < n16, b3 = i + 192 < n16;
        const uint4 v0 = s4[i];
        uint4 v1, v2, v3;
        if (b1) v1 = s4[i + 64];
        if (b2) v2 = s4[i + 128];
        if (b3) v3 = s4[i + 192];
        g4[i] = v0;
        if (b1) g4[i + 64] = v1;
        if (b2) g4[i + 128] = v2;
        if (b3) g4[i + 192] = v3;
      }
      const int tail = nbytes - head - body;
      if (lane64 < tail / 4)
        ((uint32_t*)(gdst + head + body))[lane64] = ((const uint32_t*)(img + head + body))[lane64];
    }
  };
  if (has && my_obs) {
    if constexpr (FAST) {
      // -------- fast path: the whole row in registers --------
      if constexpr (WIN > 0) {  // window planes (:327-342) from whole map words
        const int wb = (cur - H2 * pitch - H2);
        const int sh = (wb & 3) * 8;
#pragma unroll
        for (int y = 0; y < WIN; ++y) {
          const uint32_t* rowp = map32 + ((wb + y * pitch) >> 2);
          const uint64_t lo = ((uint64_t)rowp[1] << 32) | rowp[0];
          const uint32_t x03 = (uint32_t)(lo >> sh);
          uint32_t x47 = 0u;  // cells 4-7 (WIN > 4)
          if constexpr (WIN > 4) {
            const uint64_t hi = ((uint64_t)rowp[2] << 32) | rowp[1];
            x47 = (uint32_t)(hi >> sh);
          }
#pragma unroll
          for (int x = 0; x < WIN; ++x) {
            const uint32_t cv = ((x < 4 ? x03 : x47) >> (8 * (x & 3))) & 0xFFu;
            o[y * WIN + x] = cv == 0 ? 1.0f : 0.0f;
            o[WW + y * WIN + x] = cv == 0 ? 0.0f : (float)(cv - 1u);  // max(count - obst, 0)
          }
        }
      }
      // K nearest (:346-372): keys = sq distance * 64 + index, selected by repeated min
      uint32_t key[LF];
#pragma unroll
      for (int j = 0; j < LF; ++j) {
        const int2 pj = posL[j];
        const int dr = r - pj.x, dc = c - pj.y;
        key[j] = (j < N && j != ag) ? (uint32_t)(dr * dr + dc * dc) * 64u + (uint32_t)j : 0xFFFFFFFFu;
      }
      const int km1 = min(N, KF) - 1;
      float* k0 = o + 2 * WW;
      const float* me = feat + ag * FR;
#pragma unroll
      for (int q = 0; q < 11; ++q) k0[q] = me[q];
      k0[11] = (float)(g.H * g.W);  // distance to itself (:543-545)
      k0[12] = me[11];
      // round sI takes the smallest key above the last one: keys are distinct, so with
      // prev1 = last + 1 every key <= last wraps to ~2^32 in key - prev1 (an unused
      // slot's 0xFFFFFFFF stays above every real key) and one min over key - prev1 finds
      // it -- a subtract and a third of a min3 per key (was compare, compare, select)
      uint32_t prev1 = 0u;
      const float* sqt = (const float*)(lds + (g.off_sqrt >= 0 ? g.off_sqrt : 0));
      // (a branch per round measured faster than computing every round and selecting -1:
      // 15.2 vs 16.2 us)
      const auto rounds = [&](auto lut) {  // lut: the distances from the wave's table
#pragma unroll
        for (int sI = 1; sI < KF; ++sI) {
          float* row = o + 2 * WW + sI * NF;
          if (sI <= km1) {
            uint32_t m = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < LF; ++j) m = min(m, key[j] - prev1);
            const uint32_t best = m + prev1;
            prev1 = best + 1u;
            const int j = (int)(best & 63u);
            const float* fj = feat + j * FR;
#pragma unroll
            for (int q = 0; q < 11; ++q) row[q] = fj[q];
            if constexpr (decltype(lut)::value) row[11] = sqt[best >> 6];
            else row[11] = (float)isqrt_f64((int)(best >> 6));
            row[12] = fj[11];
          } else {
#pragma unroll
            for (int q = 0; q < NF; ++q) row[q] = -1.0f;
          }
        }
      };
      if (g.off_sqrt >= 0) rounds(std::true_type{});
      else rounds(std::false_type{});
    } else {
      // -------- generic path --------
      float* o = my_obs + ag * g.D;
      if constexpr (WIN > 0) {  // window planes (:327-342): OOB / obstacle -> 1; agents -> count
        for (int y = 0; y < WIN; ++y) {
          for (int x = 0; x < WIN; ++x) {
            const uint32_t cv = map[cur + (y - H2) * pitch + (x - H2)];
            o[y * WIN + x] = cv == 0 ? 1.0f : 0.0f;
            o[WW + y * WIN + x] = cv == 0 ? 0.0f : (float)(cv - 1u);
          }
        }
      }
      // K nearest agents (:346-372): self first, then the k-1 nearest others by L2
      // distance (sorted() is stable: ties by agent index); rows past min(N, K) = -1
      float* kn = o + 2 * WW;
      const int K = g.K;
      const int km1 = min(N, K) - 1;
      for (int q = 0; q < 11; ++q) kn[q] = feat[ag * FR + q];
      kn[11] = (float)(g.H * g.W);  // distance to itself (:543-545)
      kn[12] = feat[ag * FR + 11];
      long long prev = -1;
      for (int sI = 1; sI <= km1; ++sI) {
        long long best = 0x7FFFFFFFFFFFFFFFll;
        for (int j = 0; j < N; ++j) {
          if (j == ag) continue;
          const int2 pj = posL[j];
          const int dr = r - pj.x, dc = c - pj.y;
          const long long key = (long long)(dr * dr + dc * dc) * 64 + j;
          if (key > prev && key < best) best = key;
        }
        prev = best;
        const int j = (int)(best & 63);
        const int sq = (int)(best >> 6);
        float* row = kn + sI * NF;
        for (int q = 0; q < 11; ++q) row[q] = feat[j * FR + q];
        row[11] = (float)isqrt_f64(sq);
        row[12] = feat[j * FR + 11];
      }
      for (int sI = km1 + 1; sI < K; ++sI)
        for (int q = 0; q < NF; ++q) kn[sI * NF + q] = -1.0f;
    }
  }
  PST(10);
  // the carried neighbour distances (their loads have landed by now)
  uint2 nb1 = make_uint2(((uint32_t)nbd0 & 0xFFFFu) | ((uint32_t)nbd1 << 16),
                         ((uint32_t)nbd2 & 0xFFFFu) | ((uint32_t)nbd3 << 16));
  asm volatile("" : "+v"(nb1.x), "+v"(nb1.y));
  if constexpr (FAST) {
    if (g.off_stage < 0 && has && my_obs) {  // rows straight to HBM (per-lane stores)
      uint32_t* d = (uint32_t*)(my_obs + ag * DF);
#pragma unroll
      for (int i = 0; i < DF; ++i) d[i] = __float_as_uint(o[i]);
    }
    if (staged) {
      const int G = g.stage_lanes;  // 64 or 32
      wave_fence();
      for (int gi = 0; gi < 64 / G; ++gi) {
        if (max(0, min(min(G >> g.lshift, g.EPW - ((G * gi) >> g.lshift)),
                       g.E - (gw * g.EPW + ((G * gi) >> g.lshift)))) == 0)
          break;
        stage_row(gi, G, 0, DF);
        wave_fence();
        copy_runs(gi, G);
        wave_fence();  // the next group's rows reuse the images
      }
    }
  }
  PST(11);
  (void)o;
  // the carried neighbour distances are stored last (their loads land during the rows)
  if (has && nb_carry) ((uint2*)a.pnbr)[oa] = nb1;
  PST(12);
#ifdef PARTIAL_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  PST(13);
  PST_FLUSH();
#endif
}

int round_up(int x, int m) { return (x + m - 1) / m * m; }

// A goal-table rebuild makes the carried distances stale: pdist of every (masked) env
// becomes PD_NONE, so its next step looks the current and target cells up in the new
// table (marl_partial.py:228-229 reads _goal_dist afresh every step); pnbr is only read
// while pdist is valid
__global__ void __launch_bounds__(256) pdist_invalidate_kernel(long long total, int N, const uint8_t* env_mask,
                                                               int32_t* pdist) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  if (env_mask && !env_mask[i / N]) return;
  pdist[i] = PD_NONE;
}

// sqrt(i), i = 0 .. n, with the same device sqrt isqrt_f64 uses (mapfx_partial_create
// compares it bit for bit with host libm before the kernels may use it)
__global__ void __launch_bounds__(256) sqrt_probe_kernel(double* out, int n) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i <= n) out[i] = sqrt((double)i);
}

}  // namespace

struct mapfx_partial_t {
  mapfx_partial_cfg cfg;
  PGeo geo;
  double* bonus_lut;
  int device;
  int no_nbcarry;  // diagnostic builds (MAPFX_PARTIAL_DIAG_ENV) only: ignore the state's pnbr
};

namespace {

int perr(int code, const char* msg) { return mapfx_internal_error(code, msg); }

int check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    char buf[256];
    snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    return perr(MAPFX_EHIP, buf);
  }
  return MAPFX_OK;
}

int check_state(const mapfx_partial_t* h, const mapfx_partial_state* st) {
  if (!st) return perr(MAPFX_EINVAL, "NULL state");
  if (!st->pos || !st->goal || !st->init_pos || !st->steps || !st->at_goal || !st->done ||
      !st->goal_cost || !st->node || !st->edge || !st->t || !st->terminated || !st->total_coll ||
      !st->map_bits || !st->goal_dist)
    return perr(MAPFX_EINVAL, "mapfx_partial_state: every pointer is required");
  (void)h;
  return MAPFX_OK;
}

template <int WIN>
void (*pick_wg_apl(int apl))(PGeo, PArgs) {
  if (apl <= 1) return partial_wg_kernel<WIN, 1>;
  if (apl <= 2) return partial_wg_kernel<WIN, 2>;
  return partial_wg_kernel<WIN, 4>;
}

void (*pick_wg(int win, int apl))(PGeo, PArgs) {
  switch (win) {
    case 0: return pick_wg_apl<0>(apl);
    case 1: return pick_wg_apl<1>(apl);
    case 3: return pick_wg_apl<3>(apl);
    case 5: return pick_wg_apl<5>(apl);
    case 7: return pick_wg_apl<7>(apl);
    case 9: return pick_wg_apl<9>(apl);
  }
  return nullptr;
}

int wg_apl(const PGeo& g) { return (g.N + WG_THREADS - 1) / WG_THREADS; }

// the fast-path instance: table width (u8 / int16 / run time) x runner fusion
template <int WIN, int LF>
void (*pick_fast(bool u8, bool i16, bool run))(PGeo, PArgs) {
  if (run) return u8 ? partial_kernel<WIN, 5, LF, 1, true> : i16 ? partial_kernel<WIN, 5, LF, 2, true>
                                                              : partial_kernel<WIN, 5, LF, 0, true>;
  return u8 ? partial_kernel<WIN, 5, LF, 1, false> : i16 ? partial_kernel<WIN, 5, LF, 2, false>
                                                         : partial_kernel<WIN, 5, LF, 0, false>;
}

int launch(mapfx_partial_t* h, PArgs& a, void* stream) {
  const PGeo& g = h->geo;
  if (g.E == 0) return MAPFX_OK;
  a.bonus_lut = h->bonus_lut;
  if (h->no_nbcarry) a.pnbr = nullptr;
  if (g.big) {  // N > 64 or a side > 256: one workgroup per env, map in HBM
    void (*fn)(PGeo, PArgs) = pick_wg(g.win, wg_apl(g));
    if (!fn) return perr(MAPFX_EINVAL, "obs_window must be one of 0, 1, 3, 5, 7, 9");
    hipLaunchKernelGGL(fn, dim3(g.E), dim3(WG_THREADS), g.wg_lds, (hipStream_t)stream, g, a);
    mapfx_note_kernel((const void*)fn);
    return check_hip(hipGetLastError(), "partial_wg_kernel launch");
  }
  const int blocks = (g.E + g.EPW - 1) / g.EPW;
  void (*fn)(PGeo, PArgs) = nullptr;
  const bool u8 = g.gd8 != 0, i16 = !g.gd8 && !g.gd32;  // the table width, as a template argument
  // the runner's fused step, or observation rows to an EpisodeBatch time row
  const bool run = a.ra.act_row != nullptr || a.ra.alive != nullptr || a.obs_rows != nullptr;
  if (g.K == 5 && g.win == 5 && g.L == 16) fn = pick_fast<5, 16>(u8, i16, run);
  else if (g.K == 5 && g.win == 5 && g.L == 8) fn = pick_fast<5, 8>(u8, i16, run);
  else if (g.K == 5 && g.win == 5 && g.L == 32) fn = pick_fast<5, 32>(u8, i16, run);
  else if (g.K == 5 && g.win == 3 && g.L == 16) fn = pick_fast<3, 16>(u8, i16, run);
  else if (g.K == 5 && g.win == 7 && g.L == 16) fn = pick_fast<7, 16>(u8, i16, run);
  else switch (g.win) {
      case 0: fn = partial_kernel<0, 0, 0>; break;
      case 1: fn = partial_kernel<1, 0, 0>; break;
      case 3: fn = partial_kernel<3, 0, 0>; break;
      case 5: fn = partial_kernel<5, 0, 0>; break;
      case 7: fn = partial_kernel<7, 0, 0>; break;
      case 9: fn = partial_kernel<9, 0, 0>; break;
      default: return perr(MAPFX_EINVAL, "obs_window must be one of 0, 1, 3, 5, 7, 9");
    }
  // (+ one workgroup for the runner's fused compaction, partial_kernel's first block)
  const int nblk = (blocks + g.wpb - 1) / g.wpb + (run && a.ra.cmp_bs ? 1 : 0);
  hipLaunchKernelGGL(fn, dim3(nblk), dim3(64 * g.wpb), g.lds * g.wpb, (hipStream_t)stream, g, a);
  mapfx_note_kernel((const void*)fn);
  return check_hip(hipGetLastError(), "partial_kernel launch");
}

void fill_state(PArgs& a, const mapfx_partial_state* st) {
  a.pos = st->pos;
  a.goal = st->goal;
  a.init_pos = st->init_pos;
  a.steps = st->steps;
  a.at_goal = st->at_goal;
  a.done = st->done;
  a.goal_cost = st->goal_cost;
  a.node = st->node;
  a.edge = st->edge;
  a.t = st->t;
  a.terminated = st->terminated;
  a.total_coll = st->total_coll;
  a.bits = st->map_bits;
  a.gd = st->goal_dist;
  a.pdist = st->pdist;
  a.pnbr = st->pnbr;
}

void fill_out(PArgs& a, const mapfx_partial_out* o) {
  if (!o) return;
  a.reward = o->reward;
  a.obs = o->obs;
  a.state = o->state;
  a.avail = o->avail;
  a.err = o->err;
}

}  // namespace

extern "C" {

int mapfx_partial_create(const mapfx_partial_cfg* cfg, mapfx_partial_t** out) {
  if (!cfg || !out) return perr(MAPFX_EINVAL, "NULL argument");
  *out = nullptr;
  const mapfx_partial_cfg& c = *cfg;
  if (c.H < 1 || c.W < 1 || c.H > HUGE_THREADS * 2 || c.W > 64 * HUGE_WORDS)
    return perr(MAPFX_EINVAL, "MARL_PARTIAL path supports 1 <= H <= 1024, 1 <= W <= 1536");
  if (c.n_agents < 1 || c.n_agents > 4 * WG_THREADS) return perr(MAPFX_EINVAL, "n_agents must be in 1..1024");
  if (c.n_envs < 0) return perr(MAPFX_EINVAL, "n_envs < 0");
  if (c.episode_limit < 1) return perr(MAPFX_EINVAL, "episode_limit must be >= 1");
  if (c.obs_knn_agents < 1) return perr(MAPFX_EINVAL, "obs_knn_agents must be >= 1");
  if (c.obs_window < 0 || c.obs_window > 9 || (c.obs_window > 0 && !(c.obs_window & 1)))
    return perr(MAPFX_EINVAL, "obs_window must be 0 or odd <= 9");
  mapfx_partial_t* h = new (std::nothrow) mapfx_partial_t();
  if (!h) return perr(MAPFX_ENOMEM, "host allocation failed");
  h->cfg = c;
  h->bonus_lut = nullptr;
  h->no_nbcarry = 0;
#ifdef MAPFX_PARTIAL_DIAG_ENV  // A/B knobs read from the environment: diagnostic builds only
  if (const char* ev = getenv("MAPFX_PARTIAL_NBCARRY")) h->no_nbcarry = atoi(ev) == 0;
#endif
  if (hipGetDevice(&h->device) != hipSuccess) h->device = 0;
  PGeo& g = h->geo;
  memset(&g, 0, sizeof(g));
  g.H = c.H;
  g.W = c.W;
  g.N = c.n_agents;
  g.E = c.n_envs;
  int L = 1;
  while (L < g.N) L <<= 1;
  g.L = L;
  while ((1 << g.lshift) < L) ++g.lshift;
  g.win = c.obs_window;
  g.K = c.obs_knn_agents;
  g.D = 2 * c.obs_window * c.obs_window + NF * c.obs_knn_agents;
  g.limit = c.episode_limit;
  g.hw = c.H * c.W;
  g.P = std::max(1, c.obs_window / 2);
  g.pl = round_up(g.P, 4);
  g.pitch = round_up(g.pl + c.W + g.P, 4);
  g.rows = c.H + 2 * g.P;
  g.wpr = g.pitch / 4;
  g.m_wpr = (uint32_t)((0x100000000ull + (unsigned long long)g.wpr - 1ull) / (unsigned long long)g.wpr);
  g.bits_words = (c.H * c.W + 31) / 32;
  g.map_shared = c.map_shared ? 1 : 0;
  g.map_stride = mapfx_map_stride(c.H, c.W);
  g.map_env_bytes = round_up(g.rows * g.pitch, 16);
  g.bits_env_bytes = round_up(g.bits_words * 4 + 4, 16);
  g.feat_env_bytes = round_up(L * FR * 4, 16);  // (L lanes per env)
  g.pos_env_bytes = round_up(L * 8, 16);
  g.rew_env_bytes = round_up(L * 8, 16);
  g.gd32 = (long long)c.H * c.W > 32767 ? 1 : 0;  // a path is shorter than H * W cells
  g.gd8 = (long long)c.H * c.W <= 255 ? 1 : 0;
  g.big = (g.N > 64 || c.H > 256 || c.W > 256) ? 1 : 0;
  g.hs_log = 8;
  while ((1 << g.hs_log) < 4 * g.N) ++g.hs_log;
  g.wg_lds = (1 << g.hs_log) * 8 + g.N * (4 + 4 + 8 + FR * 4) + 16 + g.N * 8 + 8 * 4;
  g.huge_lds = (c.H > 256 || c.W > 256) ? c.H * ((c.W + 63) / 64) * 8 : 0;
  g.move_rew = c.move_reward;
  g.stay_rew = c.stay_reward;
  g.stay_goal_rew = c.stay_goal_reward;
  g.nc_rew = c.node_collide_reward;
  g.ec_rew = c.edge_collide_reward;
  g.env_rew = c.env_collide_reward;
  const int per_env = 2 * g.map_env_bytes + g.bits_env_bytes + g.feat_env_bytes + g.pos_env_bytes +
                      g.rew_env_bytes;
  // envs per wave: as many as fit 64 KB of LDS; one env may take up to the CU's
  // 160 KB (maps up to 256 x 256), with the dynamic-LDS limit raised below (the
  // workgroup path keeps no map in LDS)
  int EPW = g.big ? 1 : 64 / L;
  while (EPW > 1 && EPW * per_env > 64 * 1024) --EPW;
#ifdef MAPFX_PARTIAL_DIAG_ENV
  if (const char* ev = getenv("MAPFX_PARTIAL_EPW")) {  // diagnostic / A-B: fewer envs per wave
    const int v = atoi(ev);
    if (v >= 1 && v < EPW) EPW = v;
  }
#endif
  if (!g.big && EPW * per_env > 160 * 1024) {
    delete h;
    return perr(MAPFX_EINVAL, "one env needs more than 160 KB of LDS (map too large)");
  }
  if (g.big && g.huge_lds > 0) {
    // the frontier rows plus the kernel's own static LDS (__syncthreads_or's scratch)
    hipFuncAttributes fa;
    memset(&fa, 0, sizeof fa);
    (void)hipFuncGetAttributes(&fa, g.gd32 ? (const void*)partial_bfs_huge_kernel<int32_t>
                                           : (const void*)partial_bfs_huge_kernel<int16_t>);
    if (g.huge_lds + (int)fa.sharedSizeBytes > 160 * 1024) {
      char msg[240];
      snprintf(msg, sizeof msg,
               "MARL_PARTIAL: the %d x %d map's BFS frontier needs H * ceil(W / 64) * 8 = %d B of "
               "LDS (+ %d B static; the CU has 160 KB: H * ceil(W / 64) must stay below ~20470)",
               c.H, c.W, g.huge_lds, (int)fa.sharedSizeBytes);
      delete h;
      return perr(MAPFX_EINVAL, msg);
    }
  }
  if (g.big && g.wg_lds > 160 * 1024) {
    delete h;
    return perr(MAPFX_EINVAL, "MARL_PARTIAL: the workgroup path needs more than 160 KB of LDS");
  }
  g.EPW = EPW;
  int off = 0;
  g.off_map = off; off += EPW * g.map_env_bytes;
  g.off_dep = off; off += EPW * g.map_env_bytes;
  g.off_bits = off; off += EPW * g.bits_env_bytes;
  g.off_feat = off; off += EPW * g.feat_env_bytes;
  g.off_pos = off; off += EPW * g.pos_env_bytes;
  g.off_rew = off; off += EPW * g.rew_env_bytes;
  // the K-nearest rows' distances sqrt(0 .. sq_max) as float32, one table per wave filled
  // while the state loads are in flight (small maps: sq_max < 512, i.e. sides up to 16)
  g.off_sqrt = -1;
  const long long sq_max_ = 2ll * (std::max(c.H, c.W) - 1) * (std::max(c.H, c.W) - 1);  // = g.sq_max below
  if (sq_max_ < 512) {
    g.off_sqrt = off;
    off += round_up((int)(sq_max_ + 1) * 4, 16);
  }
  // the fast observation path's staging images (one env's rows + 16 bytes of alignment
  // slack each) for a group of 64 lanes (the whole wave) or 32 (each half in turn),
  // aliasing dep onwards; the whole wave while the block stays within 40 KB (4 blocks
  // per CU)
  g.off_stage = -1;
  g.stage_lanes = 0;
  g.stage_env_bytes = round_up(L * g.D * 4 + 16, 16);
  if (g.K == 5 && (g.win == 3 || g.win == 5 || g.win == 7) && L >= 8 && L <= 32) {
    for (int G : {64, 32}) {
      const int st = std::min(EPW, G / L) * g.stage_env_bytes;
      const int need = std::max(off, g.off_dep + st);
      if (need <= (G == 64 ? 40 * 1024 : 64 * 1024)) {
        g.off_stage = g.off_dep;
        g.stage_lanes = G;
        off = need;
        break;
      }
    }
  }
  g.lds = round_up(off, 16);
  // waves per block: up to PARTIAL_MAX_WPB while the block's LDS fits the CU
  g.wpb = 1;
  if (!g.big) {
    g.wpb = PARTIAL_MAX_WPB;
#ifdef MAPFX_PARTIAL_DIAG_ENV
    if (const char* ev = getenv("MAPFX_PARTIAL_WPB")) {  // diagnostic / A-B
      const int v = atoi(ev);
      if (v >= 1 && v <= PARTIAL_MAX_WPB) g.wpb = v;
    }
#endif
    while (g.wpb > 1 && g.wpb * g.lds > 160 * 1024) --g.wpb;
  }
  if (g.big) {
    int rc0 = MAPFX_OK;
    if (g.wg_lds > 64 * 1024)
      rc0 = check_hip(hipFuncSetAttribute((const void*)pick_wg(g.win, wg_apl(g)),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, g.wg_lds),
                      "hipFuncSetAttribute(partial_wg_kernel LDS)");
    if (!rc0 && g.huge_lds > 64 * 1024 &&
        hipFuncSetAttribute(g.gd32 ? (const void*)partial_bfs_huge_kernel<int32_t>
                                   : (const void*)partial_bfs_huge_kernel<int16_t>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, g.huge_lds) != hipSuccess) {
      (void)hipGetLastError();
      char msg[200];
      snprintf(msg, sizeof msg,
               "MARL_PARTIAL: the %d x %d map's BFS frontier (H * ceil(W / 64) * 8 = %d B) exceeds "
               "the LDS a workgroup may allocate", c.H, c.W, g.huge_lds);
      rc0 = perr(MAPFX_EINVAL, msg);
    }
    if (rc0) {
      delete h;
      return rc0;
    }
  } else if (g.lds * g.wpb > 64 * 1024) {
    int rc0 = MAPFX_OK;
    std::vector<void (*)(PGeo, PArgs)> fns = {partial_kernel<0, 0, 0>, partial_kernel<1, 0, 0>,
                                              partial_kernel<3, 0, 0>, partial_kernel<5, 0, 0>,
                                              partial_kernel<7, 0, 0>, partial_kernel<9, 0, 0>};
    for (int t = 0; t < 6; ++t) {  // every fast instance
      const bool u8 = t % 3 == 0, i16 = t % 3 == 1, run = t >= 3;
      fns.push_back(pick_fast<5, 16>(u8, i16, run));
      fns.push_back(pick_fast<5, 8>(u8, i16, run));
      fns.push_back(pick_fast<5, 32>(u8, i16, run));
      fns.push_back(pick_fast<3, 16>(u8, i16, run));
      fns.push_back(pick_fast<7, 16>(u8, i16, run));
    }
    for (auto fn : fns)
      if (!rc0) rc0 = check_hip(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    g.lds * g.wpb),
                                "hipFuncSetAttribute(partial_kernel LDS)");
    if (rc0) {
      delete h;
      return rc0;
    }
  }
  {  // the map build's multiply-high division (partial_kernel) must be exact on its range
    const unsigned long long nw = (unsigned long long)g.rows * g.wpr;
    for (unsigned long long wi = 0; wi < nw; ++wi)
      if (((wi * g.m_wpr) >> 32) != wi / (unsigned long long)g.wpr) {
        delete h;
        return perr(MAPFX_EINVAL, "MARL_PARTIAL: map too large for the padded-map word index");
      }
  }
  // the completion-bonus LUT from host libm (float ** int is correctly rounded there) and
  // the sqrt reference values the device sqrt is checked against
  const int S = std::max(c.H, c.W);
  g.sq_max = 2 * (S - 1) * (S - 1);
  g.bonus_len = c.episode_limit + BONUS_EXTRA;
  double* sq = (double*)malloc(sizeof(double) * (g.sq_max + 1));
  double* bo = (double*)malloc(sizeof(double) * g.bonus_len);
  if (!sq || !bo) {
    free(sq);
    free(bo);
    delete h;
    return perr(MAPFX_ENOMEM, "host allocation failed");
  }
  double (*volatile libm_sqrt)(double) = sqrt;
  double (*volatile libm_pow)(double, double) = pow;
  for (int i = 0; i <= g.sq_max; ++i) sq[i] = libm_sqrt((double)i);
  for (int t = 0; t < g.bonus_len; ++t)  // (complete / (gamma ** (limit - t))) * fac  (:292)
    bo[t] = (c.complete_reward / libm_pow(c.gamma, (double)(c.episode_limit - t))) * c.complete_fac;
  int rc = check_hip(hipMalloc(&h->bonus_lut, sizeof(double) * g.bonus_len), "hipMalloc");
  if (!rc) rc = check_hip(hipMemcpy(h->bonus_lut, bo, sizeof(double) * g.bonus_len, hipMemcpyHostToDevice), "hipMemcpy");
  // the kernels' sqrt (isqrt_f64) must equal host libm on every argument they can use
  double* probe = nullptr;
  double* back = rc ? nullptr : (double*)malloc(sizeof(double) * (g.sq_max + 1));
  if (!rc && !back) rc = perr(MAPFX_ENOMEM, "host allocation failed");
  if (!rc) rc = check_hip(hipMalloc(&probe, sizeof(double) * (g.sq_max + 1)), "hipMalloc");
  if (!rc) {
    hipLaunchKernelGGL(sqrt_probe_kernel, dim3((unsigned)(g.sq_max / 256 + 1)), dim3(256), 0, 0, probe, g.sq_max);
    rc = check_hip(hipGetLastError(), "sqrt_probe_kernel launch");
  }
  if (!rc) rc = check_hip(hipMemcpy(back, probe, sizeof(double) * (g.sq_max + 1), hipMemcpyDeviceToHost), "hipMemcpy");
  if (!rc && memcmp(back, sq, sizeof(double) * (g.sq_max + 1)) != 0)
    rc = perr(MAPFX_EINVAL, "MARL_PARTIAL: the device fp64 sqrt differs from host libm (observations would not match)");
  if (probe) (void)hipFree(probe);
  free(back);
  free(sq);
  free(bo);
  if (rc) {
    mapfx_partial_destroy(h);
    return rc;
  }
  *out = h;
  return MAPFX_OK;
}

void mapfx_partial_destroy(mapfx_partial_t* h) {
  if (!h) return;
  if (h->bonus_lut) (void)hipFree(h->bonus_lut);
  delete h;
}

int32_t mapfx_partial_obs_dim(const mapfx_partial_t* h) { return h ? h->geo.D : -1; }

int32_t mapfx_partial_goal_dist_elem_size(int32_t H, int32_t W) {
  const long long hw = (long long)H * W;
  return hw <= 255 ? 1 : hw > 32767 ? 4 : 2;
}

int mapfx_partial_goal_dist(mapfx_partial_t* h, const mapfx_partial_state* st,
                            const uint8_t* env_mask, void* stream) {
  if (!h) return perr(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st);
  if (rc) return rc;
  const PGeo& g = h->geo;
  if ((long long)g.E * g.N == 0) return MAPFX_OK;
  const hipStream_t sm = (hipStream_t)stream;
  const dim3 grid((unsigned)(g.E * g.N));
  if (g.huge_lds) {
    if (g.gd32)
      hipLaunchKernelGGL(partial_bfs_huge_kernel<int32_t>, grid, dim3(HUGE_THREADS), g.huge_lds, sm, g,
                         st->map_bits, st->goal, env_mask, (int32_t*)st->goal_dist);
    else
      hipLaunchKernelGGL(partial_bfs_huge_kernel<int16_t>, grid, dim3(HUGE_THREADS), g.huge_lds, sm, g,
                         st->map_bits, st->goal, env_mask, (int16_t*)st->goal_dist);
  } else if (g.H <= 64 && g.W <= 64) {
    if (g.gd8)
      hipLaunchKernelGGL(partial_bfs_kernel<uint8_t>, grid, dim3(64), 0, sm, g, st->map_bits, st->goal,
                         env_mask, (uint8_t*)st->goal_dist);
    else
      hipLaunchKernelGGL(partial_bfs_kernel<int16_t>, grid, dim3(64), 0, sm, g, st->map_bits, st->goal,
                         env_mask, (int16_t*)st->goal_dist);
  } else {
    if (g.gd32)
      hipLaunchKernelGGL(partial_bfs_big_kernel<int32_t>, grid, dim3(256), 0, sm, g, st->map_bits,
                         st->goal, env_mask, (int32_t*)st->goal_dist);
    else if (g.gd8)
      hipLaunchKernelGGL(partial_bfs_big_kernel<uint8_t>, grid, dim3(256), 0, sm, g, st->map_bits,
                         st->goal, env_mask, (uint8_t*)st->goal_dist);
    else
      hipLaunchKernelGGL(partial_bfs_big_kernel<int16_t>, grid, dim3(256), 0, sm, g, st->map_bits,
                         st->goal, env_mask, (int16_t*)st->goal_dist);
  }
  rc = check_hip(hipGetLastError(), "partial_bfs_kernel launch");
  if (rc || !st->pdist) return rc;
  const long long total = (long long)g.E * g.N;
  hipLaunchKernelGGL(pdist_invalidate_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, sm, total,
                     g.N, env_mask, st->pdist);
  return check_hip(hipGetLastError(), "pdist_invalidate_kernel launch");
}

int mapfx_partial_reset(mapfx_partial_t* h, const mapfx_partial_state* st, const uint8_t* env_mask,
                        const mapfx_partial_out* out, void* stream) {
  if (!h) return perr(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st);
  if (rc) return rc;
  PArgs a;
  memset(&a, 0, sizeof(a));
  fill_state(a, st);
  fill_out(a, out);
  a.reward = nullptr;
  a.do_reset = 1;
  a.reset_mask = env_mask;
  return launch(h, a, stream);
}

int mapfx_partial_step(mapfx_partial_t* h, const mapfx_partial_state* st, const void* actions,
                       int action_dtype, const mapfx_partial_out* out, void* stream) {
  if (!h) return perr(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st);
  if (rc) return rc;
  if (!actions) return perr(MAPFX_EINVAL, "NULL actions");
  if (action_dtype < MAPFX_I8 || action_dtype > MAPFX_I64) return perr(MAPFX_EINVAL, "bad action_dtype");
  PArgs a;
  memset(&a, 0, sizeof(a));
  fill_state(a, st);
  fill_out(a, out);
  a.actions = actions;
  a.act_dtype = action_dtype;
  a.do_step = 1;
  return launch(h, a, stream);
}

// mapfx_partial_step with the observation rows written to an EpisodeBatch time row
// (obs_rows + e * obs_env_stride floats, envs with obs_mask[e] != 0) instead of
// out->obs: the runner's fused step (runner.hip), internal.h
int mapfx_partial_step_rows(mapfx_partial_t* h, const mapfx_partial_state* st, const void* actions,
                            int action_dtype, const mapfx_partial_out* out, float* obs_rows,
                            long long obs_env_stride, const uint8_t* obs_mask, void* stream) {
  if (!h) return perr(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st);
  if (rc) return rc;
  if (!actions) return perr(MAPFX_EINVAL, "NULL actions");
  if (action_dtype < MAPFX_I8 || action_dtype > MAPFX_I64) return perr(MAPFX_EINVAL, "bad action_dtype");
  PArgs a;
  memset(&a, 0, sizeof(a));
  fill_state(a, st);
  fill_out(a, out);
  a.obs = nullptr;
  a.obs_rows = obs_rows;
  a.obs_env_stride = obs_env_stride;
  a.obs_mask = obs_mask;
  a.actions = actions;
  a.act_dtype = action_dtype;
  a.do_step = 1;
  return launch(h, a, stream);
}

int mapfx_partial_fuses_post(const mapfx_partial_t* h) { return h && !h->geo.big ? 1 : 0; }

int mapfx_partial_step_runner(mapfx_partial_t* h, const mapfx_partial_state* st, const void* actions,
                              int action_dtype, const mapfx_runner_acts* ra, const mapfx_partial_out* out,
                              float* obs_rows, long long obs_env_stride, const uint8_t* obs_mask,
                              void* stream) {
  if (!h) return perr(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st);
  if (rc) return rc;
  if (!actions || !ra || !ra->act_row) return perr(MAPFX_EINVAL, "NULL actions / rows map");
  if (action_dtype < MAPFX_I8 || action_dtype > MAPFX_I64) return perr(MAPFX_EINVAL, "bad action_dtype");
  PArgs a;
  memset(&a, 0, sizeof(a));
  fill_state(a, st);
  fill_out(a, out);
  if (obs_rows) {
    a.obs = nullptr;
    a.obs_rows = obs_rows;
    a.obs_env_stride = obs_env_stride;
    a.obs_mask = obs_mask;
  }
  a.actions = actions;
  a.act_dtype = action_dtype;
  a.ra = *ra;
  a.do_step = 1;
  return launch(h, a, stream);
}

int mapfx_partial_observe(mapfx_partial_t* h, const mapfx_partial_state* st,
                          const mapfx_partial_out* out, void* stream) {
  if (!h) return perr(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st);
  if (rc) return rc;
  PArgs a;
  memset(&a, 0, sizeof(a));
  fill_state(a, st);
  fill_out(a, out);
  a.reward = nullptr;
  return launch(h, a, stream);
}

}  // extern "C"

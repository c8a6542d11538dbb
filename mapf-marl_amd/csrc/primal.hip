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
// world lives in LDS as a PADDED byte map (bit 0 agent, bit 1 wall or outside the
// grid: PRIMAL's state array, :38-45, with the out-of-bounds test of :356-359 as a
// border of walls) and the agents' (position, goal) records; each lane also holds
// its own agents (and, for DIAGONAL_MOVEMENT, their past positions) in registers.
// Per call every lane of the world resolves State.moveAgent itself from broadcast
// LDS reads (no status hand-off), then produces 4 bytes of each observation plane
// with SWAR on one realigned map dword (s even: a plane row of s cells is s / 4
// dwords, so lane m writes cells 4m .. 4m + 3 of each plane with ONE dword store),
// stamps the visible agents' clamped goals into a per-world window image, and the
// world's scalar outputs (reward, done, next-action mask, on_goal, valid, goal
// vector) are staged in LDS and leave once per 64-call block as coalesced runs.
// The goal-vector magnitude comes from a host libm pow LUT, as the reference
// computes `(dx**2 + dy**2) ** .5` (quirk 8).
#include <hip/hip_ext.h>
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
  int P, PW, rows;         // padded byte map: rows x PW, interior at (P, P); P >= max(1, s / 2)
  int off_bm, off_goals, off_ag, off_pair, off_pend, off_rst, off_fst;  // regions of a world
  int diag, nact, apl;     // DIAGONAL_MOVEMENT, actions (5 / 9), agents per lane
  uint64_t m_s, m_ss;      // fastdiv magics (odd s path)
  // primal_seq_kernel (world per wave): LDS regions and size; seq = 0 when not eligible
  int seq, off_gl, off_snap, off_psnap, off_bstr, lds_seq;
};

struct QArgs {
  int32_t* pos;
  const int32_t* goal;
  const uint8_t* bits;
  int32_t* past;
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

// dirDict (:28) as 2-bit fields of (d + 1), action a at bits 2a:
// a:      0  1  2  3  4  5  6  7  8
// row+1:  1  1  2  1  0  2  2  0  0      col+1:  1  2  1  0  1  2  0  0  2
constexpr uint32_t DR1 = 1u | 1u << 2 | 2u << 4 | 1u << 6 | 0u << 8 | 2u << 10 | 2u << 12 | 0u << 14 | 0u << 16;
constexpr uint32_t DC1 = 1u | 2u << 2 | 1u << 4 | 0u << 6 | 1u << 8 | 2u << 10 | 0u << 12 | 0u << 14 | 2u << 16;
__device__ inline int dir_r(int a) { return (int)((DR1 >> (2 * a)) & 3u) - 1; }
__device__ inline int dir_c(int a) { return (int)((DC1 >> (2 * a)) & 3u) - 1; }
// opposite_actions (:26): 1<->3, 2<->4, 5<->7, 6<->8; 0 has none
__device__ inline int opposite(int a) { return a == 0 ? -1 : (a <= 4 ? ((a + 1) & 3) + 1 : ((a - 3) & 3) + 5); }
// the action whose direction is (dr, dc), |dr|, |dc| <= 1 (index (dr + 1) * 3 + dc + 1), 0 for (0, 0)
constexpr uint64_t ACT_OF = 7ull | 4ull << 4 | 8ull << 8 | 3ull << 12 | 0ull << 16 | 1ull << 20 |
                            6ull << 24 | 2ull << 28 | 5ull << 32;

// x / d for 0 <= x < 2^32 with m = ceil(2^48 / d)
__device__ inline int fdiv(int x, uint64_t m) { return (int)(((uint64_t)(uint32_t)x * m) >> 48); }

// S: observation size fixed at compile time (0: g.s); LS: log2(lanes per world);
// DIAG: DIAGONAL_MOVEMENT; MA: agents per lane held in registers (>= g.apl).
template <int S_, int LS, bool DIAG, int MA>
__global__ void __launch_bounds__(64) primal_act_kernel(QGeo g, QArgs a) {
  extern __shared__ __align__(16) unsigned char lds[];
  constexpr int lw = 1 << LS;
  constexpr int NDIR = DIAG ? 8 : 4;
  const int lane = threadIdx.x, wl = lane >> LS, ag = lane & (lw - 1), lead = wl << LS;
  const int e = blockIdx.x * (64 >> LS) + wl;
  const bool live = e < g.E;
  const uint64_t wmask = (lw == 64 ? ~0ull : ((1ull << lw) - 1ull)) << lead;
  const int N = g.N, H = g.H, W = g.W, P = g.P, PW = g.PW;
  const int s = S_ ? S_ : g.s, ss = s * s, h2 = s / 2;
  const int apl = MA == 1 ? 1 : g.apl;
  unsigned char* wr = lds + wl * g.wreg;
  uint8_t* cm = wr;                                   // [rows][PW] agent | wall << 1
  const uint32_t* cm32 = (const uint32_t*)wr;
  uint32_t* bm = (uint32_t*)(wr + g.off_bm);          // obstacle bitmap (set-up only)
  uint8_t* gim = wr + g.off_goals;                    // [s*s] visible goals of the call
  int4* agL = (int4*)(wr + g.off_ag);                 // [N] {row, col, goal row, goal col}
  int2* pairL = (int2*)(wr + g.off_pair);             // [64] a block's (agent id, action)
  int2* pend = (int2*)(wr + g.off_pend);              // [64] goal vector (dx, dy) of a block's calls
  double* rst = (double*)(wr + g.off_rst);            // [64] rewards of a block's calls
  uint8_t* fst = wr + g.off_fst;                      // [5][64] done, on_goal, valid, mask lo / hi

  // ---- agents: lane ag owns agents ag + r * lw (registers) and their LDS records ----
  int px[MA], py[MA], gx[MA], gy[MA], qx[MA], qy[MA];
  bool has[MA];
#pragma unroll
  for (int r = 0; r < MA; ++r) {
    const int b = ag + r * lw;
    has[r] = live && r < apl && b < N;
    px[r] = py[r] = gx[r] = gy[r] = qx[r] = qy[r] = -(1 << 20);  // far outside every window
    if (has[r]) {
      const long long i = (long long)e * N + b;
      const int2 p = ((const int2*)a.pos)[i], q = ((const int2*)a.goal)[i];
      px[r] = p.x, py[r] = p.y, gx[r] = q.x, gy[r] = q.y;
      if constexpr (DIAG) {
        const int2 pp = ((const int2*)a.past)[i];
        qx[r] = pp.x, qy[r] = pp.y;
      }
      agL[b] = make_int4(p.x, p.y, q.x, q.y);
    }
  }
  if (live) {
    const uint32_t* src = (const uint32_t*)(a.bits + (g.map_shared ? 0 : (long long)e * g.map_stride));
    for (int w = ag; w < g.bits_words; w += lw) bm[w] = src[w];
    for (int i = ag; i < (ss + 3) >> 2; i += lw) ((uint32_t*)gim)[i] = 0u;
  }
  wave_fence();
  // ---- the padded map: 4 cells per dword, walls from the bitmap, border = wall ----
  if (live) {
    const int wpr = PW >> 2, nwd = g.rows * wpr;
    for (int wi = ag; wi < nwd; wi += lw) {
      const int pr = wi / wpr;
      const int r = pr - P, c0 = (wi - pr * wpr) * 4 - P;
      uint32_t v = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int c = c0 + t;
        const bool in = r >= 0 && r < H && c >= 0 && c < W;
        const int idx = in ? r * W + c : 0;
        const bool wall = !in || ((bm[idx >> 5] >> (idx & 31)) & 1u);
        v |= (wall ? 2u : 0u) << (8 * t);
      }
      ((uint32_t*)cm)[wi] = v;
    }
  }
  wave_fence();
  int ngoal = 0;  // agents on their goal (State.done :159-166 is ngoal == N)
#pragma unroll
  for (int r = 0; r < MA; ++r) {
    if (has[r]) cm[(px[r] + P) * PW + py[r] + P] = 1;  // agents start on free cells
    ngoal += __popcll(__ballot(has[r] && px[r] == gx[r] && py[r] == gy[r]) & wmask);
  }
  wave_fence();

  // ---- per-lane constants of the observation planes (s even) ----
  // lane m < s*s/4 writes cells 4m .. 4m+3 of each plane: nlow of them in window row
  // y0 from column x0, the rest at the start of row y0 + 1 (o2; = o1 when none)
  const bool even = (s & 1) == 0;
  const int D = even ? ss >> 2 : ss;  // dwords a call writes per plane (even) / per record (odd)
  constexpr int RW = 4;               // rounds held in registers (host: D <= 4 lw for even s)
  int o1[RW], o2[RW];
  uint32_t lom[RW];
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) {
    const int m = ag + rr * lw;
    const int c4 = 4 * m, y0 = c4 / s, x0 = c4 - y0 * s, nlow = min(4, s - x0);
    o1[rr] = y0 * PW + x0;
    o2[rr] = nlow < 4 ? (y0 + 1) * PW + x0 - s : o1[rr];
    lom[rr] = nlow >= 4 ? ~0u : (1u << (8 * nlow)) - 1u;
  }
  const bool probe = ag >= 1 && ag <= NDIR;
  const int pofs = probe ? dir_r(ag) * PW + dir_c(ag) : 0;

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
      if (aid < 0 || aid >= N || act < 0 || act >= g.nact) {  // the reference asserts (:556-558)
        if (ag == 0 && a.err) atomicCAS(a.err, 0, e + 1);
        kstop = k;
        continue;
      }
      // ---- State.moveAgent (:103-135), resolved by every lane of the world ----
      const int4 A = agL[aid];  // broadcast read: aid's (row, col, goal row, goal col)
      const int nx = A.x + dir_r(act), ny = A.y + dir_c(act);
      const bool inb = nx < H && nx >= 0 && ny < W && ny >= 0;
      const uint32_t tv = cm[(nx + P) * PW + ny + P];  // |d| <= 1 <= P: inside the padded map
      bool dcol = false;
      if constexpr (DIAG) {  // diagonalCollision (:77-99) against the PRE-move positions
        const int sx = A.x + nx, sy = A.y + ny;
        bool hit = false;
#pragma unroll
        for (int r = 0; r < MA; ++r)
          hit |= has[r] && ag + r * lw != aid && qx[r] + px[r] == sx && qy[r] + py[r] == sy;
        dcol = (__ballot(hit) & wmask) != 0;
      }
      const bool wall = (tv & 2u) != 0, robot = (tv & 1u) != 0;
      const bool moved = act != 0 && inb && !wall && !robot && !dcol;
      const bool on_old = A.z == A.x && A.w == A.y, on_new = A.z == nx && A.w == ny;
      const int st_blocked = !inb ? -1 : (wall ? -2 : -3);  // out of bounds, wall, robot / diagonal
      const int status = act == 0 ? (on_old ? 1 : 0) : (moved ? (on_new ? 1 : (on_old ? 2 : 0)) : st_blocked);
      const int cx = moved ? nx : A.x, cy = moved ? ny : A.y;
      ngoal += (moved && on_new ? 1 : 0) - (moved && on_old ? 1 : 0);
      if (moved && ag == 0) {
        cm[(A.x + P) * PW + A.y + P] = 0;
        cm[(nx + P) * PW + ny + P] = 1;
        *(int2*)&agL[aid] = make_int2(nx, ny);
      }
#pragma unroll
      for (int r = 0; r < MA; ++r) {
        if (ag + r * lw == aid) {
          if constexpr (DIAG) {
            if (act == 0 || moved) qx[r] = A.x, qy[r] = A.y;  // agents_past (:110-112, :129-131)
          }
          px[r] = cx, py[r] = cy;
        }
      }
      wave_fence();
      // ---- _observe (:343-386) on the post-move world, next valid actions ----
      const int tr = cx - h2, tc = cy - h2;
      const int base = (tr + P) * PW + tc + P;  // first window cell in the padded map
      const int gq = (A.z >= tr && A.z < tr + s && A.w >= tc && A.w < tc + s)
                         ? (A.z - tr) * s + (A.w - tc) : -(1 << 20);  // own goal's window cell
      uint32_t V[RW];
      if (a.obs && even) {
#pragma unroll
        for (int rr = 0; rr < RW; ++rr) {
          V[rr] = 0;
          if (rr * lw < D && ag + rr * lw < D) {
            const int A1 = base + o1[rr], A2 = base + o2[rr];
            const uint32_t v1 = __builtin_amdgcn_alignbyte(cm32[(A1 >> 2) + 1], cm32[A1 >> 2], A1 & 3);
            const uint32_t v2 = __builtin_amdgcn_alignbyte(cm32[(A2 >> 2) + 1], cm32[A2 >> 2], A2 & 3);
            V[rr] = (v1 & lom[rr]) | (v2 & ~lom[rr]);
          }
        }
      }
      bool ok = false;  // _listNextValidActions (:639-667): lane d probes action d
      if (probe) ok = cm[(cx + P) * PW + cy + P + pofs] == 0;  // in bounds, no wall, no robot
      uint32_t dmask = 0;  // DIAG: directions refused by diagonalCollision from (cx, cy)
#pragma unroll
      for (int r = 0; r < MA; ++r) {
        const int b = ag + r * lw;
        if (a.obs && has[r] && b != aid && px[r] >= tr && px[r] < tr + s && py[r] >= tc && py[r] < tc + s) {
          const int mr = max(tr, min(tr + s - 1, gx[r])), mc = max(tc, min(tc + s - 1, gy[r]));
          gim[(mr - tr) * s + (mc - tc)] = 1;  // a visible agent's goal, clamped into view (:374-378)
        }
        if constexpr (DIAG) {
          const int sx = qx[r] + px[r] - 2 * cx, sy = qy[r] + py[r] - 2 * cy;
          if (has[r] && b != aid && sx >= -1 && sx <= 1 && sy >= -1 && sy <= 1)
            dmask |= 1u << (uint32_t)((ACT_OF >> (4 * ((sx + 1) * 3 + sy + 1))) & 0xFu);
        }
      }
      uint32_t mask = 1u | ((uint32_t)(__ballot(ok) >> lead) & (NDIR == 8 ? 0x1FEu : 0x1Eu));
      if constexpr (DIAG) {
#pragma unroll
        for (int d = 1; d <= 8; ++d)
          if (__ballot((dmask >> d) & 1u) & wmask) mask &= ~(1u << d);
      }
      const int opp = opposite(act);
      if (opp > 0) mask &= ~(1u << opp);
      wave_fence();
      if (a.obs) {
        uint8_t* o = a.obs + (e0k + k) * 4 * ss;
        if (even) {
#pragma unroll
          for (int rr = 0; rr < RW; ++rr) {
            const int m = ag + rr * lw;
            if (rr * lw < D && m < D) {
              uint32_t* g32 = (uint32_t*)gim + m;
              const uint32_t gw = *g32;
              *g32 = 0u;  // clear for the next call (in order before its stamps)
              const int d = gq - 4 * m;
              const uint32_t g4 = (uint32_t)d < 4u ? 1u << (8 * d) : 0u;
              uint32_t* o32 = (uint32_t*)(o + 4 * m);
              o32[0] = V[rr] & 0x01010101u;              // poss: own and other agents (:363-372)
              o32[ss >> 2] = g4;                         // goal (:366-368)
              o32[ss >> 1] = gw;                         // goals of visible agents (:374-378)
              o32[3 * (ss >> 2)] = (V[rr] >> 1) & 0x01010101u;  // obstacles, outside = 1 (:356-362)
            }
          }
        } else {  // odd s: record dword m, byte by byte (plane = byte / s^2)
          for (int m = ag; m < ss; m += lw) {
            uint32_t w = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const int b = 4 * m + t;
              const int pl = fdiv(b, g.m_ss), i = b - pl * ss;
              const int y = fdiv(i, g.m_s), x = i - y * s;
              const uint32_t v = cm[base + y * PW + x];
              uint32_t bv;
              if (pl == 0) bv = v & 1u;
              else if (pl == 1) bv = i == gq ? 1u : 0u;
              else if (pl == 2) {
                bv = gim[i];
                gim[i] = 0;
              } else bv = (v >> 1) & 1u;
              w |= bv << (8 * t);
            }
            ((uint32_t*)o)[m] = w;
          }
        }
      }
      if (ag == 0) {
        // ---- reward (:579-596), JOINT = False; stay-on-goal blocking term = 0 ----
        const double rew = act == 0 ? (status == 1 ? GOAL_REWARD + 0 : IDLE_COST)
                                    : status == 1 ? GOAL_REWARD : status < 0 ? COLLISION_REWARD : ACTION_COST;
        const int j = k - kb;
        rst[j] = rew;
        fst[j] = ngoal == N ? 1 : 0;                          // world.done() (:626)
        fst[64 + j] = (cx == A.z && cy == A.w) ? 1 : 0;       // on_goal (:633)
        fst[128 + j] = status >= 0 ? 1 : 0;                   // valid_action (:566)
        fst[192 + j] = (uint8_t)mask;
        if constexpr (DIAG) fst[256 + j] = (uint8_t)(mask >> 8);
        pend[j] = make_int2(A.z - cx, A.w - cy);              // goal vector (:379-384), LUT later
      }
    }
    wave_fence();
    // ---- the block's staged outputs, calls kb .. min(kend, kstop) - 1, as runs ----
    const int n = min(kend, kstop) - kb;
    const long long o0 = e0k + kb;
    for (int j = ag; j < n; j += lw) {
      if (a.reward) a.reward[o0 + j] = rst[j];
      if (a.done) a.done[o0 + j] = fst[j];
      if (a.on_goal) a.on_goal[o0 + j] = fst[64 + j];
      if (a.valid) a.valid[o0 + j] = fst[128 + j];
      if (a.next_mask) {
        if constexpr (DIAG) ((uint16_t*)a.next_mask)[o0 + j] = (uint16_t)(fst[192 + j] | (fst[256 + j] << 8));
        else a.next_mask[o0 + j] = fst[192 + j];
      }
      if (a.vec) {
        const int2 d = pend[j];
        const double mag = a.pow_lut[d.x * d.x + d.y * d.y];
        double vx = (double)d.x, vy = (double)d.y;
        if (mag != 0.0) {
          vx = vx / mag;
          vy = vy / mag;
        }
        double* v = a.vec + (o0 + j) * 3;
        v[0] = vx;
        v[1] = vy;
        v[2] = mag;
      }
    }
    wave_fence();
  }
#pragma unroll
  for (int r = 0; r < MA; ++r) {
    if (!has[r]) continue;
    const long long i = (long long)e * N + ag + r * lw;
    ((int2*)a.pos)[i] = make_int2(px[r], py[r]);
    if constexpr (DIAG) ((int2*)a.past)[i] = make_int2(qx[r], qy[r]);
  }
}

// ---------------------------------------------------------------------------
// primal_seq_kernel<S, DIAG>: one world per wave, the calls of a 64-call block in two
// phases (even s in 4..10, N <= 64, H + 2P <= 64, W + 2P <= 64).
//
// The only truly sequential part of _step is State.moveAgent (:103-135): whether call
// k's move happens depends on the positions the earlier calls left.  Everything else a
// call returns (_observe :343-386, done :159-166, _listNextValidActions :639-667, the
// reward :579-596) is a function of the positions right after the call.  So:
//
//   phase A (the chain, wave-uniform, no LDS on it): lane j holds agent j's position;
//     per call the moved agent's position and the target row's wall mask are
//     v_readlane'd, the robot test is a ballot of lane compares (DIAG: the midpoint
//     test of diagonalCollision :77-99 is a second ballot), the move is a v_cndmask
//     on lane aid.  The call leaves its (old position, moved) in lane k of a log
//     register and every agent's post-call position in a [64][N] u16 LDS snapshot;
//   phase B (parallel, lane k = call k): each lane rebuilds its call's status, reward,
//     done, next-action mask and goal vector from the log and the snapshot, and its
//     call's four observation planes as four S*S-bit masks (walls from padded row
//     masks, agents and clamped goals set bit by bit from the snapshot); the 4*S*S-bit
//     string of call k goes to LDS, and the wave expands strings to bytes (one bit ->
//     one byte, 16 bits per lane-chunk) and writes the block's records as one
//     contiguous run of 16-byte stores.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// acc |= bit idx (idx < 128; 127 is the "nothing" sentinel, masked off later)
__device__ __forceinline__ void set_bit128(uint32_t (&acc)[4], uint32_t idx) {
  const uint32_t b = 1u << (idx & 31u), w = idx >> 5;
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] |= (w == (uint32_t)i) ? b : 0u;
}

// str |= v at compile-time bit offset B (v has no bits at or above `bits`)
template <int B, int NSW>
__device__ __forceinline__ void put_at(uint32_t (&str)[NSW], uint32_t v) {
  constexpr int w = B >> 5, sh = B & 31;
  if constexpr (w < NSW) str[w] |= v << sh;
  if constexpr (sh != 0 && w + 1 < NSW) str[w + 1] |= v >> (32 - sh);
}

template <int P0, int SS, int NSW>
__device__ __forceinline__ void put_plane(uint32_t (&str)[NSW], const uint32_t (&pl)[4]) {
  put_at<P0, NSW>(str, SS >= 32 ? pl[0] : (pl[0] & ((1u << (SS & 31)) - 1u)));
  if constexpr (SS > 32) put_at<P0 + 32, NSW>(str, SS >= 64 ? pl[1] : (pl[1] & ((1u << (SS & 31)) - 1u)));
  if constexpr (SS > 64) put_at<P0 + 64, NSW>(str, SS >= 96 ? pl[2] : (pl[2] & ((1u << (SS & 31)) - 1u)));
  if constexpr (SS > 96) put_at<P0 + 96, NSW>(str, pl[3] & ((1u << (SS & 31)) - 1u));
}

#ifndef MAPFX_QABL
#define MAPFX_QABL 0  // diagnostic builds only: 1 no record stores, 2 no phase B, 4 no move chain
#endif
template <int S, bool DIAG>
__global__ void __launch_bounds__(64) primal_seq_kernel(QGeo g, QArgs a) {
  extern __shared__ __align__(16) unsigned char lds[];
  constexpr int SS = S * S, H2 = S / 2;
  constexpr int CPC = SS / 4;              // 16-byte chunks (= 16-bit string pieces) of one call
  constexpr int NSW = (4 * SS + 31) / 32;  // dwords of a call's bit string
  constexpr int NDIR = DIAG ? 8 : 4;
  static_assert(S % 2 == 0 && S >= 4 && SS <= 100, "even S in 4..10");
  const int lane = threadIdx.x, e = blockIdx.x;
  const int N = g.N, H = g.H, W = g.W, P = g.P;
  uint64_t* rowm = (uint64_t*)lds;                   // [H + 2P] padded wall rows
  uint32_t* gl = (uint32_t*)(lds + g.off_gl);        // [N] biased goal cell
  uint16_t* snap = (uint16_t*)(lds + g.off_snap);    // [65][N] cells before call 0, after calls 0..63
  uint16_t* psnap = (uint16_t*)(lds + g.off_psnap);  // DIAG: agents_past, same rows
  uint16_t* bstr = (uint16_t*)(lds + g.off_bstr);    // the block's bit strings, call k at CPC * k
  const int2* goal2 = (const int2*)a.goal + (long long)e * N;  // wave-uniform reads: SGPRs

  // ---- state: lane j = agent j at its BIASED cell (row + P) | (col + P) << 8 (rows and
  //      columns of the padded map, < 64: the cell is its own u16 snapshot value and a
  //      move is one packed add); other lanes hold a value no cell has ----
  const bool agent = lane < N;
  const uint32_t bias = (uint32_t)P | ((uint32_t)P << 8);
  // block 0's calls are loaded first: their latency overlaps the set-up loads
  int id0 = 0, ac0 = 0;
  if (lane < min(64, a.K)) {
    id0 = a.ids[(long long)e * a.K + lane];
    ac0 = a.acts[(long long)e * a.K + lane];
  }
  uint32_t vpos = 0xFFFFFFFFu, vpast = 0u;
  if (agent) {
    const long long i = (long long)e * N + lane;
    const int2 p = ((const int2*)a.pos)[i], q = goal2[lane];
    vpos = ((uint32_t)p.x | ((uint32_t)p.y << 8)) + bias;
    gl[lane] = ((uint32_t)q.x | ((uint32_t)q.y << 8)) + bias;
    if constexpr (DIAG) {
      const int2 pp = ((const int2*)a.past)[i];
      vpast = ((uint32_t)pp.x | ((uint32_t)pp.y << 8)) + bias;
    }
  }
  uint32_t vsum = vpos + vpast;  // DIAG: past + present, the midpoint test's sum (sentinel off-agent)
  // ---- padded wall rows: lane r = padded row r, bit c + P = wall at column c; outside = 1 ----
  uint64_t vrow = ~0ull;
  {
    const int r = lane - P;
    if (r >= 0 && r < H) {
      const uint32_t* w32 = (const uint32_t*)(a.bits + (g.map_shared ? 0 : (long long)e * g.map_stride));
      const int b0 = r * W, wi = b0 >> 5, sh = b0 & 31, last = (b0 + W - 1) >> 5;
      const uint64_t d0 = w32[wi], d1 = wi + 1 <= last ? w32[wi + 1] : 0u, d2 = wi + 2 <= last ? w32[wi + 2] : 0u;
      uint64_t v = (d0 | (d1 << 32)) >> sh;
      if (sh) v |= d2 << (64 - sh);
      const uint64_t fm = ((1ull << W) - 1ull) << P;
      vrow = (~fm) | ((v << P) & fm);
    }
    if (lane < H + 2 * P) rowm[lane] = vrow;
  }
  const uint32_t vrow_lo = (uint32_t)vrow, vrow_hi = (uint32_t)(vrow >> 32);
  wave_fence();

  const long long e0k = (long long)e * a.K;
  int kstop = a.K;
  for (int kb = 0; kb < kstop; kb += 64) {
    const int nb = min(64, a.K - kb);
    // call kb + lane: agent index, action, and the move as one packed add (cells biased,
    // so a row step never borrows from the column byte); the first bad call ends the
    // world's calls (the reference asserts, :556-558)
    int id = id0, ac = ac0;
    if (kb > 0 && lane < nb) {
      id = a.ids[e0k + kb + lane];
      ac = a.acts[e0k + kb + lane];
    }
    const bool okc = lane < nb && (unsigned)(id - 1) < (unsigned)N && (unsigned)ac < (unsigned)g.nact;
    const uint64_t badm = __ballot(lane < nb && !okc);
    const int nv = badm ? (int)__ffsll((unsigned long long)badm) - 1 : nb;
    const int vaid = okc ? id - 1 : 0, vact = okc ? ac : 0;
    const uint32_t vdel = okc ? (uint32_t)(dir_r(ac) + dir_c(ac) * 256) : 0u;
    // ================= phase A: State.moveAgent, call after call =================
    // snapshot rows: row 0 = the cells before call kb, row kk + 1 = after call kb + kk;
    // agent lanes write slot [row][lane], the others one spare slot past the rows
    uint32_t saddr = agent ? 2u * (uint32_t)lane : 2u * 65u * (uint32_t)N;
    const uint32_t sinc = agent ? 2u * (uint32_t)N : 0u;
    *(uint16_t*)((unsigned char*)snap + saddr) = (uint16_t)vpos;
    if constexpr (DIAG) *(uint16_t*)((unsigned char*)psnap + saddr) = (uint16_t)vpast;
    saddr += sinc;
    for (int kk = 0; kk < nv; ++kk) {
      if (MAPFX_QABL & 4) {
        *(uint16_t*)((unsigned char*)snap + saddr) = (uint16_t)vpos;
        saddr += sinc;
        continue;
      }
      const int aid = __builtin_amdgcn_readlane(vaid, kk);
      const uint32_t d = readlane_u32(vdel, kk);
      const uint32_t o = readlane_u32(vpos, aid), t = o + d;
      const int rs = (int)(t & 0xFFu);  // padded row of the target (outside = wall)
      const uint64_t wr = ((uint64_t)readlane_u32(vrow_hi, rs) << 32) | readlane_u32(vrow_lo, rs);
      // wall / outside, or an agent on the target (a stay hits itself)
      uint64_t blk = ((wr >> (t >> 8)) & 1ull) | __ballot(vpos == t);
      if constexpr (DIAG) blk |= __ballot(vsum == o + t && vpos != o);  // (vpos == o: agent aid)
      uint32_t tm = blk == 0 ? t : o;  // agent aid's cell after the call
      asm volatile("" : "+s"(tm));      // (uniform, computed before the select: no exec branch)
      const bool me = vpos == o;        // (cells are distinct: only lane aid)
      if constexpr (DIAG) vpast = (me && (d == 0u || tm != o)) ? o : vpast;  // agents_past (:110-112, :129-131)
      vpos = me ? tm : vpos;
      if constexpr (DIAG) vsum = vpos + vpast;
      *(uint16_t*)((unsigned char*)snap + saddr) = (uint16_t)vpos;
      if constexpr (DIAG) *(uint16_t*)((unsigned char*)psnap + saddr) = (uint16_t)vpast;
      saddr += sinc;
    }
    if (nv < nb) {
      if (lane == 0 && a.err) atomicCAS(a.err, 0, e + 1);
      kstop = kb + nv;
    }
    wave_fence();
    // ================= phase B: lane k = call kb + k =================
    if (MAPFX_QABL & 2) continue;
    const bool cv = lane < nv;
    const int aid = vaid, act = vact;
    // call k's cell before / after it: snapshot rows k and k + 1 (lanes without a call: the
    // biased (0, 0), so the reads below stay inside the padded map)
    const uint32_t ob = cv ? (uint32_t)snap[lane * N + aid] : bias;
    const uint32_t cb = cv ? (uint32_t)snap[(lane + 1) * N + aid] : bias;
    const uint32_t tb = ob + vdel;
    const bool moved = cb != ob;
    const int cxb = (int)(cb & 0xFFu), cyb = (int)(cb >> 8);
    const bool inb = (unsigned)((int)(tb & 0xFFu) - P) < (unsigned)H && (unsigned)((int)(tb >> 8) - P) < (unsigned)W;
    const uint32_t gA = gl[aid];
    const int gxb = (int)(gA & 0xFFu), gyb = (int)(gA >> 8);
    const int trb = cxb - H2, tcb = cyb - H2;  // window origin in padded coordinates
    // obstacle plane (:356-362, outside = 1) and the walls of the 3 x 3 around the agent
    uint32_t obsp[4] = {0u, 0u, 0u, 0u};
    uint32_t w9 = 0;
#pragma unroll
    for (int y = 0; y < S; ++y) {
      const uint64_t m = rowm[trb + y];
      const uint32_t bits = (uint32_t)(m >> tcb) & ((1u << S) - 1u);
      const int B = S * y;
      obsp[B >> 5] |= bits << (B & 31);
      if ((B & 31) + S > 32) obsp[(B >> 5) + 1] |= bits >> (32 - (B & 31));
      if (y >= H2 - 1 && y <= H2 + 1) w9 |= ((bits >> (H2 - 1)) & 7u) << (3 * (y - H2 + 1));
    }
    // agents at this call: poss plane (:363-372), visible agents' clamped goals
    // (:374-378), agents on their goal (done), DIAG crossing directions
    uint32_t possp[4] = {0u, 0u, 0u, 0u}, goalsp[4] = {0u, 0u, 0u, 0u};
    uint32_t dmask = 0;
    int ngoal = 0;
    const uint16_t* sk = snap + (lane + 1) * N;
    const uint16_t* pk = psnap + (lane + 1) * N;
    for (int j = 0; j < N; ++j) {
      const int2 gj = goal2[j];
      const int gjxb = gj.x + P, gjyb = gj.y + P;
      const uint32_t pj = sk[j];
      ngoal += pj == (uint32_t)(gjxb | (gjyb << 8)) ? 1 : 0;
      const int dx = (int)(pj & 0xFFu) - trb, dy = (int)(pj >> 8) - tcb;
      const bool vis = (unsigned)dx < (unsigned)S && (unsigned)dy < (unsigned)S;
      set_bit128(possp, vis ? (uint32_t)(dx * S + dy) : 127u);
      const int mx = min(max(gjxb - trb, 0), S - 1), my = min(max(gjyb - tcb, 0), S - 1);
      set_bit128(goalsp, (vis && j != aid) ? (uint32_t)(mx * S + my) : 127u);
      if constexpr (DIAG) {
        const uint32_t qj = pk[j];
        const int sx = (int)(qj & 0xFFu) + (int)(pj & 0xFFu) - 2 * cxb;
        const int sy = (int)(qj >> 8) + (int)(pj >> 8) - 2 * cyb;
        if (j != aid && sx >= -1 && sx <= 1 && sy >= -1 && sy <= 1)
          dmask |= 1u << (uint32_t)((ACT_OF >> (4 * ((sx + 1) * 3 + sy + 1))) & 0xFu);
      }
    }
    // the 3 x 3 around the agent is inside the window (S >= 4): its occupied cells are
    // poss-plane bits (the centre is the agent itself, never a probe)
    uint32_t nb9 = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int B = (H2 - 1 + r) * S + H2 - 1;
      uint32_t v = possp[B >> 5] >> (B & 31);
      if ((B & 31) > 29) v |= possp[(B >> 5) + 1] << (32 - (B & 31));
      nb9 |= (v & 7u) << (3 * r);
    }
    uint32_t goalp[4] = {0u, 0u, 0u, 0u};
    {
      const int dx = gxb - trb, dy = gyb - tcb;
      set_bit128(goalp, ((unsigned)dx < (unsigned)S && (unsigned)dy < (unsigned)S) ? (uint32_t)(dx * S + dy) : 127u);
    }
    // status (State.moveAgent), reward (:579-596), next valid actions (:639-667)
    const bool on_old = gA == ob, on_new = gA == tb;
    const int i9 = (dir_r(act) + 1) * 3 + dir_c(act) + 1;  // target in the 3 x 3 (not moved: c = o)
    const bool wallT = ((w9 >> i9) & 1u) != 0;
    const int st_blocked = !inb ? -1 : (wallT ? -2 : -3);
    const int status = act == 0 ? (on_old ? 1 : 0) : (moved ? (on_new ? 1 : (on_old ? 2 : 0)) : st_blocked);
    const uint32_t blocked9 = w9 | nb9;
    uint32_t mask = 1u;
#pragma unroll
    for (int d = 1; d <= NDIR; ++d) {
      const int id9 = (dir_r(d) + 1) * 3 + dir_c(d) + 1;
      mask |= ((~blocked9 >> id9) & 1u) << d;
    }
    const int opp = opposite(act);
    if (opp > 0) mask &= ~(1u << opp);
    if constexpr (DIAG) mask &= ~(dmask & 0x1FEu);
    if (cv) {
      const long long oi = e0k + kb + lane;
      const double rew = act == 0 ? (status == 1 ? GOAL_REWARD + 0 : IDLE_COST)
                                  : status == 1 ? GOAL_REWARD : status < 0 ? COLLISION_REWARD : ACTION_COST;
      if (a.reward) a.reward[oi] = rew;
      if (a.done) a.done[oi] = ngoal == N ? 1 : 0;
      if (a.on_goal) a.on_goal[oi] = gA == cb ? 1 : 0;
      if (a.valid) a.valid[oi] = status >= 0 ? 1 : 0;
      if (a.next_mask) {
        if constexpr (DIAG) ((uint16_t*)a.next_mask)[oi] = (uint16_t)mask;
        else a.next_mask[oi] = (uint8_t)mask;
      }
      if (a.vec) {  // :379-386, magnitude from the host libm pow LUT
        const int dX = gxb - cxb, dY = gyb - cyb;
        const double mag = a.pow_lut[dX * dX + dY * dY];
        double vx = (double)dX, vy = (double)dY;
        if (mag != 0.0) {
          vx = vx / mag;
          vy = vy / mag;
        }
        double* v = a.vec + oi * 3;
        v[0] = vx;
        v[1] = vy;
        v[2] = mag;
      }
    }
    if (a.obs) {
      uint32_t str[NSW];
#pragma unroll
      for (int i = 0; i < NSW; ++i) str[i] = 0u;
      put_plane<0, SS, NSW>(str, possp);
      put_plane<SS, SS, NSW>(str, goalp);
      put_plane<2 * SS, SS, NSW>(str, goalsp);
      put_plane<3 * SS, SS, NSW>(str, obsp);
      // call k's 4 S^2 bits = 16-bit pieces CPC k .. CPC k + CPC - 1 of one contiguous
      // string: the block's records are one run of bytes, piece c -> record bytes 16c ..
      uint16_t* dst = bstr + CPC * lane;
#pragma unroll
      for (int i = 0; i < CPC; ++i) dst[i] = (uint16_t)(str[i >> 1] >> (16 * (i & 1)));
      wave_fence();
      const uint32_t* b32 = (const uint32_t*)bstr;
      uint4* obase = (uint4*)(a.obs + (e0k + kb) * (4 * SS));
      const int nch = nv * CPC;
      for (int i = lane; 2 * i < nch; i += 64) {
        const uint32_t b = b32[i];
        uint4 v0, v1;
        v0.x = ((b & 15u) * 0x00204081u) & 0x01010101u;
        v0.y = (((b >> 4) & 15u) * 0x00204081u) & 0x01010101u;
        v0.z = (((b >> 8) & 15u) * 0x00204081u) & 0x01010101u;
        v0.w = (((b >> 12) & 15u) * 0x00204081u) & 0x01010101u;
        v1.x = (((b >> 16) & 15u) * 0x00204081u) & 0x01010101u;
        v1.y = (((b >> 20) & 15u) * 0x00204081u) & 0x01010101u;
        v1.z = (((b >> 24) & 15u) * 0x00204081u) & 0x01010101u;
        v1.w = ((b >> 28) * 0x00204081u) & 0x01010101u;
        if (MAPFX_QABL & 1) continue;
        obase[2 * i] = v0;
        if (2 * i + 1 < nch) obase[2 * i + 1] = v1;
      }
    }
    wave_fence();
  }
  if (agent) {
    const long long i = (long long)e * N + lane;
    const uint32_t p = vpos - bias;
    ((int2*)a.pos)[i] = make_int2((int)(p & 0xFFu), (int)(p >> 8));
    if constexpr (DIAG) {
      const uint32_t q = vpast - bias;
      ((int2*)a.past)[i] = make_int2((int)(q & 0xFFu), (int)(q >> 8));
    }
  }
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
  QGeo geo;  // (seq layout included)
  double* pow_lut;
  int lds;
};

namespace {

using PrimalFn = void (*)(QGeo, QArgs);

template <int S, int LS, bool DIAG>
PrimalFn pick_ma(int apl) {
  if (apl <= 1) return primal_act_kernel<S, LS, DIAG, 1>;
  return primal_act_kernel<S, LS, DIAG, 4>;
}
template <int S, bool DIAG>
PrimalFn pick_ls(int ls, int apl) {
  if (ls == 4) return pick_ma<S, 4, DIAG>(apl);
  if (ls == 5) return pick_ma<S, 5, DIAG>(apl);
  return pick_ma<S, 6, DIAG>(apl);
}
PrimalFn pick_primal(const QGeo& g) {
  if (g.s == 10) return g.diag ? pick_ls<10, true>(g.lw_shift, g.apl) : pick_ls<10, false>(g.lw_shift, g.apl);
  return g.diag ? pick_ls<0, true>(g.lw_shift, g.apl) : pick_ls<0, false>(g.lw_shift, g.apl);
}

uint64_t magic48(int d) { return ((1ull << 48) + (uint64_t)d - 1) / (uint64_t)d; }
int r16(int x) { return (x + 15) & ~15; }

template <bool DIAG>
PrimalFn pick_seq_s(int s) {
  if (s == 4) return primal_seq_kernel<4, DIAG>;
  if (s == 6) return primal_seq_kernel<6, DIAG>;
  if (s == 8) return primal_seq_kernel<8, DIAG>;
  return primal_seq_kernel<10, DIAG>;
}
PrimalFn pick_seq(const QGeo& g) { return g.diag ? pick_seq_s<true>(g.s) : pick_seq_s<false>(g.s); }

// primal_seq_kernel eligibility and LDS layout of its one world per block: padded wall
// rows (u64), goals (u32), the [64][N] u16 position (and DIAG past) snapshots, the
// [64][16] u32 bit strings.  Returns the size, 0 when the world does not qualify.
int layout_seq(QGeo& g) {
  const bool ok = g.s % 2 == 0 && g.s >= 4 && g.s <= 10 && g.N <= 64 && g.H + 2 * g.P <= 64 &&
                  g.W + 2 * g.P <= 64;
  if (!ok) return 0;
  int o = r16((g.H + 2 * g.P) * 8);
  g.off_gl = o;
  o += r16(4 * g.N);
  g.off_snap = o;
  o += r16(65 * 2 * g.N + 2);  // 65 rows + the spare slot of the non-agent lanes
  g.off_psnap = o;
  if (g.diag) o += r16(65 * 2 * g.N + 2);
  g.off_bstr = o;
  o += 64 * 64;
  return o;
}

// LDS layout of one world for lanes-per-world 1 << ls; returns its size.
int layout(QGeo& g) {
  int o = r16(g.rows * g.PW + 4);  // + the realigning read's overrun
  g.off_bm = o;
  o += r16(g.bits_words * 4);
  g.off_goals = o;
  o += r16(g.s * g.s + 4);
  g.off_ag = o;
  o += 16 * g.N;
  g.off_pair = o;
  o += 64 * 8;
  g.off_pend = o;
  o += 64 * 8;
  g.off_rst = o;
  o += 64 * 8;
  g.off_fst = o;
  o += 5 * 64;
  return r16(o);
}

}  // namespace

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
  memset(&g, 0, sizeof(g));
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
  g.diag = c.diagonal ? 1 : 0;
  g.nact = g.diag ? 9 : 5;
  g.P = std::max(1, g.s / 2);
  g.PW = (c.W + 2 * g.P + 3) & ~3;
  g.rows = c.H + 2 * g.P;
  g.m_s = magic48(g.s);
  g.m_ss = magic48(g.s * g.s);
  // One world per wave, phase A / phase B (primal_seq_kernel) wherever it applies, unless
  // a test pins the lane-group kernel (MAPFX_PRIMAL_LANES, or MAPFX_PRIMAL_PATH=groups).
  {
    const char* lanes = getenv("MAPFX_PRIMAL_LANES");
    const char* path = getenv("MAPFX_PRIMAL_PATH");
    const bool pinned = (lanes && *lanes) || (path && strcmp(path, "groups") == 0);
    g.lds_seq = pinned ? 0 : layout_seq(g);
    g.seq = g.lds_seq > 0 ? 1 : 0;
  }
  const int wreg = layout(g);
  // Lanes per world: the smallest of 16 / 32 / 64 that writes an even-s call's planes
  // in at most 4 rounds (s * s / 4 dwords per plane) and holds the agents in at most
  // 4 registers each, widened while the grid has fewer than 2 waves per SIMD (2048
  // waves: more waves hide the call's LDS round trips) or a wave's worlds would pass
  // 64 KB of LDS.  At 4096 worlds, s = 10 (the bench) this is 32 lanes, 2 worlds a
  // wave.  MAPFX_PRIMAL_LANES (16 / 32 / 64) overrides the wave-count rule (tests).
  const int D = (g.s % 2 == 0) ? g.s * g.s / 4 : 1;
  int ls = 4;
  while (ls < 6 && (D > 4 * (1 << ls) || g.N > 4 * (1 << ls))) ++ls;
  const char* force = getenv("MAPFX_PRIMAL_LANES");
  const int fl = force ? atoi(force) : 0;
  if (fl == 16 || fl == 32 || fl == 64) ls = std::max(ls, fl == 16 ? 4 : fl == 32 ? 5 : 6);
  else
    while (ls < 6 && (long long)(g.E + (64 >> ls) - 1) / (64 >> ls) < 2048) ++ls;
  while (ls < 6 && (64 >> ls) * wreg > 65536) ++ls;
  if ((64 >> ls) * wreg > 160 * 1024) {
    delete h;
    return perr(MAPFX_EINVAL, "PRIMAL world needs too much LDS");
  }
  g.lw_shift = ls;
  g.lw = 1 << ls;
  g.apl = (g.N + g.lw - 1) / g.lw;
  g.wreg = wreg;
  h->lds = (64 >> ls) * wreg;
  if (h->lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)pick_primal(g),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, h->lds);
    if (e != hipSuccess) {
      delete h;
      return check_hip(e, "hipFuncSetAttribute");
    }
  }
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

int mapfx_primal_act_timed(mapfx_primal_t* h, const mapfx_primal_state* st, const int32_t* agent_ids,
                           const int32_t* actions, int32_t K, const mapfx_primal_out* out,
                           void* start_event, void* stop_event, void* stream) {
  if (!h) return perr(MAPFX_EINVAL, "NULL handle");
  if (!st || !st->pos || !st->goal || !st->map_bits) return perr(MAPFX_EINVAL, "bad state");
  if (h->geo.diag && !st->past) return perr(MAPFX_EINVAL, "diagonal movement needs state.past");
  if (K < 0) return perr(MAPFX_EINVAL, "K < 0");
  if (K == 0 || h->geo.E == 0) return MAPFX_OK;
  if (!agent_ids || !actions) return perr(MAPFX_EINVAL, "NULL agent_ids / actions");
  QArgs a;
  memset(&a, 0, sizeof(a));
  a.pos = st->pos;
  a.goal = st->goal;
  a.bits = st->map_bits;
  a.past = st->past;
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
  const QGeo& g = h->geo;
  if (g.seq && ((uintptr_t)a.obs & 15u) == 0) {  // (16-byte record runs)
    if (start_event || stop_event)
      hipExtLaunchKernelGGL(pick_seq(g), dim3(g.E), dim3(64), g.lds_seq, (hipStream_t)stream,
                            (hipEvent_t)start_event, (hipEvent_t)stop_event, 0, g, a);
    else
      hipLaunchKernelGGL(pick_seq(g), dim3(g.E), dim3(64), g.lds_seq, (hipStream_t)stream, g, a);
    mapfx_note_kernel((const void*)pick_seq(g));
    return check_hip(hipGetLastError(), "primal_seq_kernel launch");
  }
  const int wpw = 64 >> g.lw_shift;
  if (start_event || stop_event)
    hipExtLaunchKernelGGL(pick_primal(g), dim3((g.E + wpw - 1) / wpw), dim3(64), h->lds, (hipStream_t)stream,
                          (hipEvent_t)start_event, (hipEvent_t)stop_event, 0, g, a);
  else
    hipLaunchKernelGGL(pick_primal(g), dim3((g.E + wpw - 1) / wpw), dim3(64), h->lds, (hipStream_t)stream, g, a);
  mapfx_note_kernel((const void*)pick_primal(g));
  return check_hip(hipGetLastError(), "primal_act_kernel launch");
}

int mapfx_primal_act(mapfx_primal_t* h, const mapfx_primal_state* st, const int32_t* agent_ids,
                     const int32_t* actions, int32_t K, const mapfx_primal_out* out, void* stream) {
  return mapfx_primal_act_timed(h, st, agent_ids, actions, K, out, nullptr, nullptr, stream);
}

}  // extern "C"

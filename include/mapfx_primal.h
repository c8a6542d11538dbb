/*
 * mapfx_primal.h -- C ABI of PRIMAL's sequential dynamics, batched.
 *
 * Paths relative to MARL-curve-main/src/envs/mapf_primal.py:
 *
 *   reference (one world per object, one agent per call)   this ABI (E worlds per call)
 *   ---------------------------------------------------    --------------------------
 *   MAPFEnv(world0, goals0, observation_size) :175-203      mapfx_primal_create + state
 *   MAPFEnv._step((agent_id, action))         :549-637      mapfx_primal_act (K calls
 *                                                           per world, in order)
 *     State.moveAgent :103-135, reward table :579-596, _observe :343-386,
 *     State.done :159-166, _listNextValidActions :639-667
 *
 * Actions: 0 stay, 1 (0,+1), 2 (+1,0), 3 (0,-1), 4 (-1,0) (dirDict, :28); with
 * cfg.diagonal (DIAGONAL_MOVEMENT, :175) also 5 (1,1), 6 (1,-1), 7 (-1,-1), 8 (-1,1):
 * then every move is also refused (-3) when it crosses another agent's last move
 * (State.diagonalCollision :77-99: equal midpoints of (past, present) and (old, new);
 * with integer coordinates np.isclose of the halves is exact equality of the sums),
 * each agent's past position (agents_past) is part of the state, updated by a stay
 * and by a successful move (:110-112, :129-131), and next_mask has 9 bits (u16).
 * JOINT = False (the reference default, :27).
 * The stay-on-goal blocking term (:583, get_blocking_reward) needs the
 * un-vendored od_mstar3 planner and is defined as 0 (parity unpinned); the
 * `blocking` output of _step is therefore always False and not produced.
 * Agents start on free cells (PRIMAL keeps agents and obstacles in one array).
 *
 * Same conventions as mapfx.h: caller-owned DEVICE pointers, asynchronous on
 * `stream`, 0 / negative MAPFX_E* return codes, messages from mapfx_last_error().
 * Limits: N <= 255, H * W <= 16384, observation size 1..32.
 */
#ifndef MAPFX_PRIMAL_H
#define MAPFX_PRIMAL_H

#include <stdint.h>

#include "mapfx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mapfx_primal_cfg {
  int32_t H, W;          /* grid rows, cols                                      */
  int32_t n_agents;      /* N                                                    */
  int32_t n_envs;        /* E worlds                                             */
  int32_t obs_size;      /* observation_size s (:175)                            */
  int32_t map_shared;    /* 1: one obstacle map for all worlds                   */
  int32_t diagonal;      /* DIAGONAL_MOVEMENT (:175): 9 actions, agents_past     */
} mapfx_primal_cfg;

typedef struct mapfx_primal_state {
  int32_t* pos;             /* [E][N][2] (row, col), updated in place             */
  const int32_t* goal;      /* [E][N][2]                                          */
  const uint8_t* map_bits;  /* [E or 1][mapfx_map_stride(H, W)] obstacle bitmaps  */
  int32_t* past;            /* [E][N][2] agents_past (cfg.diagonal only; updated in
                               place; set it equal to pos for a fresh world, :55-66) */
} mapfx_primal_state;

/* Outputs of the k-th call of world e at index [e][k] (NULL = not produced). */
typedef struct mapfx_primal_out {
  double* reward;        /* [E][K]                                               */
  uint8_t* done;         /* [E][K] world.done() after the call                   */
  uint8_t* next_mask;    /* [E][K] bit a = action a in _listNextValidActions; u8,
                            or u16 ([E][K] uint16_t) with cfg.diagonal (9 bits)   */
  uint8_t* on_goal;      /* [E][K]                                               */
  uint8_t* valid;        /* [E][K] action_status >= 0                            */
  uint8_t* obs;          /* [E][K][4][s][s] _observe maps (poss, goal, goals, obs) */
  double* vec;           /* [E][K][3] _observe goal vector (dx, dy, mag)         */
  int32_t* err;          /* [1] 0, or 1 + index of a world given a bad agent/action */
} mapfx_primal_out;

typedef struct mapfx_primal_t mapfx_primal_t;

int mapfx_primal_create(const mapfx_primal_cfg* cfg, mapfx_primal_t** out_handle);
void mapfx_primal_destroy(mapfx_primal_t* h);

/* K calls of MAPFEnv._step per world, in order: call k of world e is
 * (agent_ids[e][k] (1-based, as the reference), actions[e][k]). */
int mapfx_primal_act(mapfx_primal_t* h, const mapfx_primal_state* st, const int32_t* agent_ids,
                     const int32_t* actions, int32_t K, const mapfx_primal_out* out, void* stream);

/* mapfx_primal_act with the launch's own start / stop timestamps recorded into
 * `start_event` / `stop_event` (hipEvent_t, created by the caller) at the kernel's
 * begin and end (hipExtLaunchKernel): the kernel duration, without the host's
 * launch gaps.  NULL events: plain mapfx_primal_act. */
int mapfx_primal_act_timed(mapfx_primal_t* h, const mapfx_primal_state* st, const int32_t* agent_ids,
                           const int32_t* actions, int32_t K, const mapfx_primal_out* out,
                           void* start_event, void* stop_event, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MAPFX_PRIMAL_H */

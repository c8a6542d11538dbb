/*
 * mapfx_partial.h -- C ABI of the batched MARL_PARTIAL_ENV step.
 *
 * MARL_PARTIAL_ENV is the env the reference actually registers
 * (MARL-curve-main/src/envs/__init__.py:60).  Paths below are relative to
 * MARL-curve-main/src/envs/marl_partial.py:
 *
 *   reference (one env per object)              this ABI (E envs per call)
 *   ------------------------------------------  ------------------------------
 *   MARL_PARTIAL_ENV.__init__  :25-123          mapfx_partial_create
 *   __setup_agent_goal_dist    :906-928         mapfx_partial_goal_dist (BFS)
 *   reset                      :125-163         mapfx_partial_reset
 *   step                       :165-310         mapfx_partial_step
 *   get_obs / get_state / get_avail_actions
 *                              :312-391         mapfx_partial_observe
 *
 * Same conventions as mapfx.h: caller-owned DEVICE pointers, (row, col) int32
 * positions, LSB-first obstacle bitmaps of mapfx_map_stride(H, W) bytes per env,
 * asynchronous on `stream`, 0 / negative MAPFX_E* return codes, messages from
 * mapfx_last_error().  Not restated (out of scope): the `output`
 * mode's random collision repair (:262-275) and the visualisation hooks.
 *
 * Limits: N <= 1024, H <= 1024, W <= 1536, and for a side above 256 the BFS
 * frontier rows must fit LDS: H * ceil(W / 64) * 8 bytes plus the BFS kernel's few
 * bytes of static LDS <= 160 KB, i.e. H * ceil(W / 64) just under 20480 (every map the
 * reference ships fits: orz900d's 656 x 1491 needs 126 KB; a full 1024 x 1536 map
 * would need 196 KB and is refused by mapfx_partial_create).  N <= 64 with H, W <= 256 keeps each env in one wavefront
 * with its cell maps in LDS; otherwise one workgroup steps an env with the agents'
 * cells in an LDS hash table and the obstacle bitmap read from HBM.
 */
#ifndef MAPFX_PARTIAL_H
#define MAPFX_PARTIAL_H

#include <stdint.h>

#include "mapfx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mapfx_partial_cfg {
  int32_t H, W;             /* grid rows, cols                                      */
  int32_t n_agents;         /* N <= 1024                                            */
  int32_t n_envs;           /* E (this rank's shard)                                */
  int64_t env_offset;       /* global id of env 0                                   */
  int32_t episode_limit;    /* :33                                                  */
  int32_t obs_window;       /* W of the window part (:31)                           */
  int32_t obs_knn_agents;   /* K (:32)                                              */
  int32_t map_shared;       /* 1: one obstacle map for all envs                     */
  double move_reward;       /* :35 */
  double stay_reward;       /* :36 */
  double stay_goal_reward;  /* :37 */
  double node_collide_reward, edge_collide_reward, env_collide_reward; /* :38-40 */
  double complete_reward;   /* :41 */
  double complete_fac;      /* :42 */
  double gamma;             /* :45 */
} mapfx_partial_cfg;

/* Caller-owned device state of E envs. */
typedef struct mapfx_partial_state {
  int32_t* pos;             /* [E][N][2] current (row, col)                         */
  const int32_t* goal;      /* [E][N][2]                                            */
  const int32_t* init_pos;  /* [E][N][2]                                            */
  int32_t* steps;           /* [E][N] _agent_step_count                             */
  uint8_t* at_goal;         /* [E][N] _agent_at_goals                               */
  uint8_t* done;            /* [E][N] _agent_dones                                  */
  int32_t* goal_cost;       /* [E][N] _each_goal_cost                               */
  uint8_t* node;            /* [E][N] _node_collision_agents of the last step       */
  int32_t* edge;            /* [E][N] _edge_collision_agents of the last step       */
  int32_t* t;               /* [E] _step_count                                      */
  uint8_t* terminated;      /* [E] _terminated                                      */
  int32_t* total_coll;      /* [E] _total_number_collisions                         */
  const uint8_t* map_bits;  /* [E or 1][mapfx_map_stride(H, W)]                     */
  void* goal_dist;          /* [E][N][H*W] shortest-path lengths to each goal (-1:
                               obstacle / unreachable), filled by
                               mapfx_partial_goal_dist; u8 when H*W <= 255 (255
                               stands for -1; ABI 5), int16 up to 32767 cells, else
                               int32 (mapfx_partial_goal_dist_elem_size)            */
  int32_t* pdist;           /* [E][N] goal_dist of each agent's current cell, carried
                               from step to step (the reference's _new_pdist / next
                               _old_pdist, :227-233): a step reads it as opd and looks
                               up only a moving agent's npd; reset / observe refresh
                               it from the table.  INT32_MIN (never reset) or a NULL
                               pointer: looked up.  Appended in ABI 4.            */
  int16_t* pnbr;            /* [E][N][4] goal_dist of the 4 neighbours (up, down,
                               left, right; an off-grid entry is unused) of each
                               agent's current cell, written with pdist by every
                               launch: a step
                               takes a moving agent's npd from it instead of a
                               dependent table lookup.  Used only with pdist and
                               u8 / int16 tables (H*W <= 32767); NULL: looked up.
                               Appended in ABI 4.                                  */
} mapfx_partial_state;

/* Per-call outputs (device, caller-owned; NULL = not produced). */
typedef struct mapfx_partial_out {
  double* reward;           /* [E] sum(rewards) (:310), fp64 in reference op order  */
  float* obs;               /* [E][N][2*W*W + 13*K] get_obs as float32 (PyMARL)     */
  float* state;             /* [E][3] get_state (:377-387)                          */
  uint8_t* avail;           /* [E][N] 5-bit get_avail_actions mask                  */
  int32_t* err;             /* [1] 0, or 1 + env index given an action outside 0..4 */
} mapfx_partial_out;

typedef struct mapfx_partial_t mapfx_partial_t;

int mapfx_partial_create(const mapfx_partial_cfg* cfg, mapfx_partial_t** out_handle);
void mapfx_partial_destroy(mapfx_partial_t* h);
/* 2*W*W + 13*K (:377 get_obs_size) */
int32_t mapfx_partial_obs_dim(const mapfx_partial_t* h);
/* 1, 2 or 4: bytes per goal_dist entry (a path on H*W cells is shorter than H*W; the
 * u8 form (ABI 5) holds -1 as 255). */
int32_t mapfx_partial_goal_dist_elem_size(int32_t H, int32_t W);

/* BFS distance tables of every (masked) env's goals (:906-928: A* lengths on
 * the 4-connected free-cell graph == BFS levels).  The carried distances of the
 * recomputed envs become stale with their tables, so st->pdist (when non-NULL) is
 * set to INT32_MIN for them: their next step looks the distances up again, as the
 * reference reads _goal_dist afresh every step (:228-229). */
int mapfx_partial_goal_dist(mapfx_partial_t* h, const mapfx_partial_state* st,
                            const uint8_t* env_mask, void* stream);

/* reset (:125-163) of the masked envs (all when env_mask is NULL) to init_pos,
 * then get_obs / get_state / get_avail_actions of every env into `out`. */
int mapfx_partial_reset(mapfx_partial_t* h, const mapfx_partial_state* st,
                        const uint8_t* env_mask, const mapfx_partial_out* out, void* stream);

/* step (:165-310) of all E envs, then the post-step observations. */
int mapfx_partial_step(mapfx_partial_t* h, const mapfx_partial_state* st, const void* actions,
                       int action_dtype, const mapfx_partial_out* out, void* stream);

/* get_obs / get_state / get_avail_actions of the current state. */
int mapfx_partial_observe(mapfx_partial_t* h, const mapfx_partial_state* st,
                          const mapfx_partial_out* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MAPFX_PARTIAL_H */

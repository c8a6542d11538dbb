/*
 * mapfx.h — C ABI of the MI355X-native batched MAPF gridworld step.
 *
 * This is the drop-in boundary beneath the PyMARL env plugin surface of the
 * reference (DongmingShenDS/MAPF-MARL, paths relative to MARL-curve-main/src/):
 *
 *   reference (Python, one env per object)          this ABI (E envs per call)
 *   ---------------------------------------------   ------------------------------
 *   MAPF_GRID.__init__  envs/mapf_gridworld.py:21-68   mapfx_create
 *   MAPF_GRID.reset     envs/mapf_gridworld.py:70-83   mapfx_reset
 *   MAPF_GRID.step      envs/mapf_gridworld.py:85-141  mapfx_step
 *   MAPF_GRID.get_obs / get_state / get_avail_actions
 *                       envs/mapf_gridworld.py:143-224 mapfx_observe
 *   MARL_PARTIAL_ENV.get_obs_agent window part
 *                       envs/marl_partial.py:323-342   mapfx_out.obs_window
 *   MAPFEnv._observe    envs/mapf_primal.py:343-386    mapfx_out.obs_primal/primal_vec
 *   ParallelRunner step loop (T env-steps, random policy)
 *                       runners/parallel_runner.py:91-206  mapfx_rollout
 *
 * Conventions
 *   - Every pointer in mapfx_state / mapfx_out / mapfx_rollout is a DEVICE
 *     pointer owned by the caller (e.g. a torch tensor's data_ptr()).  No call
 *     allocates or frees device memory except mapfx_create / mapfx_destroy.
 *   - Positions are int32 (row, col) pairs, env-major: pos[(e*N + a)*2 + {0,1}],
 *     exactly the reference's (pos[0], pos[1]) = (row, col) convention.
 *   - Obstacle maps are bitmaps: bit (r*W + c) of the env's map (LSB-first in
 *     each byte) is 1 for an obstacle (any map char other than '.',
 *     envs/mapf_gridworld.py:282-288).  Each env's map occupies
 *     mapfx_map_stride(H, W) bytes; with cfg.map_shared one map serves all envs.
 *   - All calls are asynchronous on the given hipStream_t (NULL = default
 *     stream).  Return 0 on success, a negative MAPFX_E* code on error; the
 *     message is available from mapfx_last_error().  No C++ exception crosses
 *     this boundary.  A handle must not be used from two threads at once.
 */
#ifndef MAPFX_H
#define MAPFX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAPFX_ABI_VERSION 6

/* error codes */
#define MAPFX_OK 0
#define MAPFX_EINVAL -1   /* bad argument / unsupported configuration */
#define MAPFX_EHIP -2     /* HIP runtime error (launch / memcpy) */
#define MAPFX_ENOMEM -3   /* device allocation failed in mapfx_create */

/* observation modes (bit mask, cfg.obs_mode) */
#define MAPFX_OBS_FULL 1    /* MAPF_GRID get_obs/get_state: occ map [E][H*W]     */
#define MAPFX_OBS_WINDOW 2  /* marl_partial window [E][N][2][w][w]              */
#define MAPFX_OBS_PRIMAL 4  /* PRIMAL _observe [E][N][4][s][s] u8 + [E][N][3] f64 */

/* action element types */
#define MAPFX_I8 0
#define MAPFX_I32 1
#define MAPFX_I64 2

typedef struct mapfx_cfg {
  int32_t H, W;           /* grid rows, cols (the reference requires H == W)    */
  int32_t n_agents;       /* N, 1..1024                                         */
  int32_t n_envs;         /* E envs handled by this handle (this rank's shard)  */
  int64_t env_offset;     /* global id of env 0 (RNG key; sharding)             */
  int32_t episode_limit;  /* envs/mapf_gridworld.py:26                          */
  double step_reward;     /* envs/mapf_gridworld.py:29 (fp64, exact op order)   */
  double collide_reward;  /* envs/mapf_gridworld.py:30                          */
  int32_t obs_mode;       /* MAPFX_OBS_* mask of modes the handle may produce   */
  int32_t window;         /* marl_partial obs_window (config/envs/marl_partial.yaml:7) */
  int32_t primal_size;    /* PRIMAL observation_size (envs/mapf_primal.py:175)  */
  int32_t map_shared;     /* 1: one obstacle map for all envs                   */
} mapfx_cfg;

/* Caller-owned device state of E envs. */
typedef struct mapfx_state {
  int32_t* pos;             /* [E][N][2] current (row,col), in/out             */
  const int32_t* goal;      /* [E][N][2]                                         */
  const int32_t* init_pos;  /* [E][N][2] restored by reset (may be NULL for step) */
  uint8_t* done;            /* [E][N] per-agent done (_agent_dones)             */
  int32_t* t;               /* [E] env step counter (_step_count)               */
  int32_t* steps;           /* [E][N] _agent_step_count, or NULL (not tracked)  */
  const uint8_t* map_bits;  /* [E or 1][mapfx_map_stride(H,W)] obstacle bitmaps  */
} mapfx_state;

/* Caller-owned device outputs; any pointer may be NULL (not produced).
 * obs_full / obs_window / obs_window_occ are int8 when N <= 127, else int16 (see
 * mapfx_obs_elem_size). */
typedef struct mapfx_out {
  double* reward;        /* [E]  sum(rewards) as the reference folds it (fp64)  */
  float* reward_f32;     /* [E]  same value rounded to fp32                      */
  uint8_t* term;         /* [E]  1 iff every agent is done (episode_done)        */
  uint8_t* node;         /* [E][N] node-collision flag (0/1)                     */
  uint8_t* edge;         /* [E][N] edge-collision count, exact: u8 for N <= 256,
                            u16 above (mapfx_edge_elem_size; ABI 3)              */
  uint8_t* avail;        /* [E][N] 5-bit mask, bit d = action d available        */
  void* obs_full;        /* [E][H*W] occupancy G + counts                        */
  void* obs_window;      /* [E][N][2][w][w] {obstacle, agents} window            */
  uint8_t* obs_primal;   /* [E][N][4][s][s] {poss, goal, goals, obs}             */
  double* primal_vec;    /* [E][N][3] {dx, dy, mag}                              */
  int32_t* traj_pos;     /* [E][N][2] post-step positions (rollout trajectories) */
  uint8_t* traj_done;    /* [E][N]    post-step dones                            */
  int32_t* traj_t;       /* [E]       post-step env step counter                 */
  int32_t* err;          /* [1] 0, or 1 + env index of an env given an action
                            outside 0..4 (that env is left unchanged)            */
  void* obs_window_occ;  /* [E][N][w][w] the same window as ONE plane of occupancy
                            values occ = agents - obstacle (the reference's map
                            value, marl_partial.py:323-342): obstacle plane =
                            (occ == -1), agents plane = max(occ, 0).  Half the bytes
                            of obs_window; for N > 127 (int16 cells) it keeps the
                            0/1 obstacle plane from costing 2 B per cell.  (ABI 2) */
} mapfx_out;

typedef struct mapfx_t mapfx_t;

/* Launch geometry chosen for a configuration (for tests / docs). */
typedef struct mapfx_info {
  int32_t lanes_per_env;   /* L */
  int32_t agents_per_lane; /* ceil(N / L) */
  int32_t envs_per_block;
  int32_t block_threads;
  int32_t lds_bytes;       /* dynamic LDS per block */
  int32_t cell_bytes;      /* 1 (N <= 127) or 2 */
  int32_t pad;             /* border cells around the map in LDS */
} mapfx_info;

int mapfx_abi_version(void);
const char* mapfx_last_error(void);

/* Identity of this build (ABI 5): "src=<first 16 hex of the sha256 over the HIP
 * sources, headers and compile flags> git=<commit the build started from>[+dirty]",
 * fixed at compile time.  A profile records it, so a measurement can refuse a profile
 * taken of another build (bench.py, tools/pmc_traffic.py). */
const char* mapfx_build_id(void);
/* Demangled name of the env kernel the calling thread launched last through this
 * library (the MAPF step / rollout / observe, the MARL_PARTIAL step / reset / observe,
 * the PRIMAL act; not the helper kernels: BFS tables, masked resets, action generation,
 * packing, runner bookkeeping), exactly as rocprofv3 names it; "" before the first
 * launch.  Needs the HIP runtime (a visible device).  ABI 5. */
const char* mapfx_last_kernel(void);

/* Bytes of one env's obstacle bitmap: ceil(H*W/8) rounded up to 16. */
int64_t mapfx_map_stride(int32_t H, int32_t W);
/* 1 or 2: element size of obs_full / obs_window for N agents. */
int32_t mapfx_obs_elem_size(int32_t n_agents);
/* 1 or 2: element size of `edge` for N agents (an edge count is at most N - 1,
 * envs/mapf_gridworld.py:364-383, so u8 holds it while N <= 256).  ABI 3. */
int32_t mapfx_edge_elem_size(int32_t n_agents);

int mapfx_create(const mapfx_cfg* cfg, mapfx_t** out_handle);
void mapfx_destroy(mapfx_t* h);
int mapfx_query(const mapfx_t* h, mapfx_info* info);

/* reset (envs/mapf_gridworld.py:70-83): for every env with env_mask[e] != 0
 * (all envs when env_mask is NULL): pos = init_pos, done = 0, t = 0, steps = 0.
 * If out != NULL, mapfx_observe's outputs (obs, avail, term) of every env's
 * post-reset state are written. */
int mapfx_reset(mapfx_t* h, const mapfx_state* st, const uint8_t* env_mask,
                const mapfx_out* out, void* stream);

/* step (envs/mapf_gridworld.py:85-141) of all E envs.  actions: [E][N] of
 * action_dtype.  Writes the post-step state and every non-NULL output. */
int mapfx_step(mapfx_t* h, const mapfx_state* st, const void* actions, int action_dtype,
               const mapfx_out* out, void* stream);

/* Observations / avail / term of the current state without stepping
 * (get_obs, get_state, get_avail_actions). */
int mapfx_observe(mapfx_t* h, const mapfx_state* st, const mapfx_out* out, void* stream);

/* T fused steps in one launch.  Actions come from `actions` ([T][E][N] of
 * action_dtype) or, when actions == NULL, from the counter-based generator
 * mapfx_action(seed, env_offset + e, t0 + k, a).  Step k's outputs go to slot k
 * of each non-NULL output ([T][...] layouts, i.e. the mapfx_out shapes with a
 * leading T); `err` is shared.  With autoreset, an env whose agents are all done
 * after a step is reset to init_pos before the next one (its t restarts at 0).
 * The result is bit-identical to T successive mapfx_step calls (+ resets). */
int mapfx_rollout(mapfx_t* h, const mapfx_state* st, int32_t T, const void* actions,
                  int action_dtype, uint64_t seed, int32_t t0, int32_t autoreset,
                  const mapfx_out* traj, void* stream);

/* mapfx_rollout with the launch's own start / stop timestamps recorded into
 * `start_event` / `stop_event` (hipEvent_t, created by the caller) at the kernel's
 * begin and end (hipExtLaunchKernel), i.e. the kernel duration rocprofv3 reports,
 * without the event packets' dispatch gaps.  NULL events: plain mapfx_rollout. */
int mapfx_rollout_timed(mapfx_t* h, const mapfx_state* st, int32_t T, const void* actions,
                        int action_dtype, uint64_t seed, int32_t t0, int32_t autoreset,
                        const mapfx_out* traj, void* start_event, void* stop_event, void* stream);

/* Fill out[T][E][N] (int8) with the generator's actions for steps t0..t0+T-1. */
int mapfx_gen_actions(mapfx_t* h, uint64_t seed, int32_t t0, int32_t T, int8_t* out,
                      void* stream);

/* Compact copy of a rollout's trajectory for the gather to rank 0
 * (runners/parallel_runner.py:117-173: the parent collects every env's state each
 * step): cell[T][E][N] = row * W + col of traj_pos (u16; needs H*W <= 65536) and
 * done_bits[T][E][ceil(N/8)] with bit (a & 7) of byte a >> 3 = traj_done[..][a].
 * Together with the env's reward this is the state the obs follow from: rank 0
 * rebuilds any step's window / full / PRIMAL observation with mapfx_observe on the
 * unpacked positions.  ABI 4 addition. */
int mapfx_pack_compact(mapfx_t* h, int32_t T, const int32_t* traj_pos, const uint8_t* traj_done,
                       uint16_t* cell, uint8_t* done_bits, void* stream);

/* The action generator (host reference of the device one):
 * splitmix64(seed ^ env*0xD1B54A32D192ED03 ^ t*0xABC98388FB8FAC03
 *            ^ agent*0x8CB92BA72F3D8DD7) % 5 */
int32_t mapfx_action(uint64_t seed, int64_t env, int32_t t, int32_t agent);

#ifdef __cplusplus
}
#endif
#endif /* MAPFX_H */

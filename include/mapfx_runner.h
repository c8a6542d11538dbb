/*
 * mapfx_runner.h -- C ABI of the batched ParallelRunner's episode writes
 * (SURVEY.md §8(f) F2).
 *
 * The reference collects one transition per env and step through a Pipe and
 * writes it into PyMARL's EpisodeBatch with EpisodeBatch.update
 * (MARL-curve-main/src/runners/parallel_runner.py:62-76 reset, :91-173 run;
 * components/episode_buffer.py:100-134 update).  Here the E = B envs of one
 * MarlPartialBatch are stepped by mapfx_partial_step and these kernels write the
 * step's rows straight into the EpisodeBatch's device tensors, with the runner's
 * bookkeeping (which envs are still running, the MAC's `bs` list, returns,
 * lengths, env-step count) kept on the device -- no per-step host round trip:
 *
 *   reference                                   this ABI
 *   -----------------------------------------   ---------------------------------
 *   reset(): batch.update(pre_transition, ts=0) mapfx_runner_begin
 *   run(): batch.update({"actions"}, bs, ts)    mapfx_runner_actions
 *          (+ the OneHot preprocess of actions)
 *   run(): receive loop, update(post, bs, ts),  mapfx_runner_post (after
 *          update(pre, bs, ts + 1), returns,     mapfx_partial_step)
 *          lengths, envs_not_terminated (:123)
 *
 * Row semantics are the reference's, including its stale list: the MAC and the
 * actions row at step t cover the envs that were running before step t - 1
 * (`bs`), the env step and every other row the envs still running now (`alive`).
 * Tensors are caller-owned DEVICE memory; element strides of the batch (sb) and
 * time (st) dimensions; NULL = field absent.  0 / negative MAPFX_E* return codes.
 */
#ifndef MAPFX_RUNNER_H
#define MAPFX_RUNNER_H

#include <stdint.h>

#include "mapfx_partial.h"

#ifdef __cplusplus
extern "C" {
#endif

/* EpisodeBatch.data.transition_data tensors, [B][max_t][...] (PyMARL's scheme,
 * episode_buffer.py:46-86: obs / state float32, avail_actions int32, actions int64,
 * actions_onehot float32, reward float32, terminated uint8, filled int64). */
typedef struct mapfx_episode_rows {
  int32_t max_t;                                   /* episode_limit + 1          */
  float* obs;          int64_t obs_sb, obs_st;      /* [B][T][N][D]               */
  float* state;        int64_t state_sb, state_st;  /* [B][T][3]                  */
  int32_t* avail;      int64_t avail_sb, avail_st;  /* [B][T][N][5]               */
  int64_t* actions;    int64_t actions_sb, actions_st;       /* [B][T][N][1]      */
  float* onehot;       int64_t onehot_sb, onehot_st;         /* [B][T][N][5]      */
  float* reward;       int64_t reward_sb, reward_st;         /* [B][T][1]         */
  uint8_t* terminated; int64_t terminated_sb, terminated_st; /* [B][T][1]         */
  int64_t* filled;     int64_t filled_sb, filled_st;         /* [B][T][1]         */
} mapfx_episode_rows;

/* The runner's device bookkeeping for B envs of N agents and obs size D. */
typedef struct mapfx_runner_state {
  int32_t B, N, D;
  uint8_t* alive;        /* [B] env not terminated (after the last step)            */
  uint8_t* alive_prev;   /* [B] running before the last step: the stale list        */
                         /* (mapfx_runner_step with the post pass fused -- every map
                            the one-wave-per-env-group kernel takes, N <= 64 and sides
                            <= 256 -- uses the two as A[0] / A[1], A[ts & 1] = running
                            before step ts; ABI 6)                                   */
  int64_t* bs;           /* [B] ascending indices of alive_prev, padded with bs[0]: the
                            MAC's `bs` (parallel_runner.py:91, :123)                 */
  int32_t* counts;       /* [2] len(bs), number alive                               */
  double* ep_return;     /* [B] episode_returns (:139, fp64 like the Python floats)  */
  int64_t* ep_length;    /* [B] episode_lengths (:140)                              */
  int64_t* env_steps;    /* [1] env_steps_this_run (:142)                           */
  int8_t* env_actions;   /* [B][N] the actions the env step reads (mapfx_runner_actions) */
  int32_t* bs_inv;       /* [2][B] row of env b in bs, -1 when b is not in it: the fused
                            step (mapfx_runner_step) reads env b's actions from row
                            bs_inv[ts & 1][b] of the MAC's output and writes its actions
                            rows there, so no separate actions pass runs (appended in
                            ABI 4; two parity halves since ABI 6, the first one used by
                            the unfused forms) */
} mapfx_runner_state;

/* reset(): every env's observations (from `out` of mapfx_partial_reset) into row
 * ts = 0, filled = 1; every env alive, bs = 0..B-1, returns / lengths / steps 0. */
int mapfx_runner_begin(const mapfx_runner_state* rs, const mapfx_partial_out* out,
                       const mapfx_episode_rows* rows, void* stream);

/* The MAC's actions ([counts[0]] rows of N, row j for env bs[j], `row_stride`
 * elements apart, dtype MAPFX_I8 / I32 / I64) into the actions / actions_onehot rows
 * at ts and into env_actions. */
int mapfx_runner_actions(const mapfx_runner_state* rs, const void* actions, int32_t action_dtype,
                         int64_t row_stride, int32_t ts, const mapfx_episode_rows* rows,
                         void* stream);

/* After mapfx_partial_step(env_actions): for every alive env the reward /
 * terminated rows at ts and obs / state / avail_actions / filled at ts + 1 (when
 * ts + 1 < max_t), returns and lengths; then alive_prev = alive, alive &= !terminated,
 * and bs / counts recomputed from alive_prev.  The new counts are also written to
 * `counts_out` (may be pinned host memory: the host polls it behind an event
 * instead of copying; mapfx_host_ring_alloc's dev_ptr), when not NULL. */
int mapfx_runner_post(const mapfx_runner_state* rs, const uint8_t* terminated,
                      const mapfx_partial_out* out, int32_t ts, int32_t* counts_out,
                      const mapfx_episode_rows* rows, void* stream);

/* One runner step in one call: the env step of mapfx_partial_step with every env's
 * actions read from row bs_inv[b] of `actions` (stay for an env not in bs: it is no
 * longer running and nothing of it is recorded), which also writes the actions /
 * actions_onehot rows at ts of the envs in bs -- what mapfx_runner_actions does, in the
 * same launch -- then mapfx_runner_post(rs, st->terminated, out, ...).  When rows->obs
 * is set, the env step writes the observation rows of the envs running before it
 * straight into rows->obs at ts + 1 (out->obs is then not written) and the post kernel
 * copies no observation bytes.
 * One launch (ABI 6) where the env kernel fuses the post pass (mapfx_runner_state
 * alive): the compaction for the next MAC call is its first workgroup, over A[ts & 1]
 * (running before step ts), so counts / counts_out = {len(bs), envs running after step
 * ts - 1}: the running count lags one step more than mapfx_runner_post's. */
int mapfx_runner_step(mapfx_partial_t* h, const mapfx_partial_state* st, const mapfx_partial_out* out,
                      const mapfx_runner_state* rs, const void* actions, int32_t action_dtype,
                      int64_t row_stride, int32_t ts, int32_t* counts_out,
                      const mapfx_episode_rows* rows, void* stream);

/* n int32 of host memory the device writes directly (hipHostMalloc mapped +
 * coherent): *host_ptr for the host, *dev_ptr for kernels (mapfx_runner_post's
 * counts_out).  Free with mapfx_host_ring_free(host_ptr). */
int mapfx_host_ring_alloc(int32_t n, int32_t** host_ptr, int32_t** dev_ptr);
void mapfx_host_ring_free(int32_t* host_ptr);

#ifdef __cplusplus
}
#endif
#endif /* MAPFX_RUNNER_H */

// internal.h -- shared between the translation units of libmapfx.so (not installed).
#ifndef MAPFX_INTERNAL_H
#define MAPFX_INTERNAL_H

#include "mapfx_partial.h"

#ifdef __cplusplus
extern "C" {
#endif
// sets the message returned by mapfx_last_error(); returns `code`
int mapfx_internal_error(int code, const char* msg);
// records the host stub of the kernel the calling thread just launched (mapfx_last_kernel)
void mapfx_note_kernel(const void* fn);
// partial.hip: mapfx_partial_step with the observation rows written to an EpisodeBatch
// time row (obs_rows + e * obs_env_stride floats, only envs with obs_mask[e] != 0)
int mapfx_partial_step_rows(mapfx_partial_t* h, const mapfx_partial_state* st, const void* actions,
                            int action_dtype, const mapfx_partial_out* out, float* obs_rows,
                            long long obs_env_stride, const uint8_t* obs_mask, void* stream);
// The runner's fused step: env e's actions are row act_row[e] (act_row_stride elements
// apart) of `actions`, stay when act_row[e] < 0; the env's actions / one-hot EpisodeBatch
// rows at ts are written where act_row[e] >= 0 (ep_actions / ep_onehot may be NULL).
// obs_rows NULL: observations go to out->obs.
typedef struct mapfx_runner_acts {
  const int32_t* act_row;
  long long act_row_stride;
  int64_t* ep_actions;
  long long ep_actions_sb, ep_actions_st;
  float* ep_onehot;
  long long ep_onehot_sb, ep_onehot_st;
  int ts;
  // runner_post_kernel's work for the envs running before the step (alive[e] != 0),
  // fused into the env step's write-back (alive NULL: not fused): the reward /
  // terminated rows at ts, returns, lengths, alive / alive_prev, and the state /
  // avail_actions / filled rows at ts + 1 (ep_state / ep_avail / ep_filled point at
  // that time row; NULL when ts + 1 == max_t or the field is absent)
  uint8_t* alive;
  uint8_t* alive_prev;
  double* ep_return;
  int64_t* ep_length;
  float* ep_reward;
  long long ep_reward_sb, ep_reward_st;
  uint8_t* ep_term;
  long long ep_term_sb, ep_term_st;
  float* ep_state;
  long long ep_state_sb;
  int32_t* ep_avail;
  long long ep_avail_sb;
  int64_t* ep_filled;
  long long ep_filled_sb;
  // The `bs` compaction for the NEXT MAC call fused into the same launch (cmp_bs NULL:
  // not fused; runner.hip runner_compact_kernel then runs after the step).  The alive
  // flags are double-buffered by step parity: `alive` is A[ts & 1] (running before this
  // step: read, never written) and `alive_prev` is A[(ts + 1) & 1] (written for every env:
  // running after this step), so the launch's last workgroup compacts A[ts & 1] -- the
  // stale list bs(ts + 1) -- while the env workgroups step.  It writes bs, the row map
  // cmp_bs_inv (bs_inv of the next step's parity), counts {len(bs), len(bs)}, env_steps
  // += len(bs) and, when not NULL, counts_out.
  const uint8_t* cmp_alive;
  int64_t* cmp_bs;
  int32_t* cmp_bs_inv;
  int32_t* cmp_counts;
  int64_t* cmp_env_steps;
  int32_t* cmp_counts_out;
  int cmp_B;
} mapfx_runner_acts;
// 1 when mapfx_partial_step_runner can take the post pass (mapfx_runner_acts.alive):
// the one-wave-per-env-group kernel; the workgroup path (N > 64, a side > 256) cannot
int mapfx_partial_fuses_post(const mapfx_partial_t* h);
int mapfx_partial_step_runner(mapfx_partial_t* h, const mapfx_partial_state* st, const void* actions,
                              int action_dtype, const mapfx_runner_acts* ra, const mapfx_partial_out* out,
                              float* obs_rows, long long obs_env_stride, const uint8_t* obs_mask,
                              void* stream);
#ifdef __cplusplus
}
#endif
#endif

// internal.h -- shared between the translation units of libmapfx.so (not installed).
#ifndef MAPFX_INTERNAL_H
#define MAPFX_INTERNAL_H

#include "mapfx_partial.h"

#ifdef __cplusplus
extern "C" {
#endif
// sets the message returned by mapfx_last_error(); returns `code`
int mapfx_internal_error(int code, const char* msg);
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
} mapfx_runner_acts;
int mapfx_partial_step_runner(mapfx_partial_t* h, const mapfx_partial_state* st, const void* actions,
                              int action_dtype, const mapfx_runner_acts* ra, const mapfx_partial_out* out,
                              float* obs_rows, long long obs_env_stride, const uint8_t* obs_mask,
                              void* stream);
#ifdef __cplusplus
}
#endif
#endif

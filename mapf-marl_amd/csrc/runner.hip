// runner.hip — MI355X (gfx950) episode writes of the batched ParallelRunner
// (include/mapfx_runner.h).
//
// The reference's runner loop (MARL-curve-main/src/runners/parallel_runner.py:91-173)
// moves every env's transition through a Pipe and a Python list into PyMARL's
// EpisodeBatch (components/episode_buffer.py:100-134).  These kernels write the
// same rows from the batched env's device outputs into the EpisodeBatch tensors
// and keep the runner's bookkeeping (running envs, the MAC's `bs` list, returns,
// lengths, env-step count) on the device, so a runner step needs no host sync.
//
// Byte-moving work only (HBM-bound): one workgroup per env copies the env's
// N x D float observation row with coalesced dword stores; the `bs` compaction is
// one workgroup's prefix scan.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>

#include "internal.h"
#include "mapfx.h"
#include "mapfx_runner.h"

namespace {

constexpr int RB = 256;  // threads of a row-copy workgroup

int err(int code, const char* msg) { return mapfx_internal_error(code, msg); }

int launch_ok(const char* what) {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MAPFX_OK : err(MAPFX_EHIP, what);
}

// obs / state / avail_actions (+ filled = 1) of env b into time row t
__device__ inline void write_pre(const mapfx_runner_state& rs, const mapfx_partial_out& o,
                                 const mapfx_episode_rows& r, int b, int t) {
  const int ND = rs.N * rs.D;
  if (r.obs) {  // U loads in flight per thread before the stores (restrict: no alias stalls)
    const float* __restrict__ src = o.obs + (int64_t)b * ND;
    float* __restrict__ dst = r.obs + (int64_t)b * r.obs_sb + (int64_t)t * r.obs_st;
    constexpr int U = 8;
    for (int base = 0; base < ND; base += RB * U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * RB + (int)threadIdx.x;
        v[u] = i < ND ? src[i] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * RB + (int)threadIdx.x;
        if (i < ND) dst[i] = v[u];
      }
    }
  }
  if (r.state && threadIdx.x < 3)
    r.state[(int64_t)b * r.state_sb + (int64_t)t * r.state_st + threadIdx.x] = o.state[(int64_t)b * 3 + threadIdx.x];
  if (r.avail) {  // 5-bit mask -> [N][5] int32 (get_avail_actions, marl_partial.py:389-433)
    int32_t* dst = r.avail + (int64_t)b * r.avail_sb + (int64_t)t * r.avail_st;
    for (int i = threadIdx.x; i < rs.N * 5; i += blockDim.x) {
      const int n = i / 5, k = i - 5 * n;
      dst[i] = (o.avail[(int64_t)b * rs.N + n] >> k) & 1;
    }
  }
  if (r.filled && threadIdx.x == 0) r.filled[(int64_t)b * r.filled_sb + (int64_t)t * r.filled_st] = 1;
}

__global__ void __launch_bounds__(RB) runner_begin_kernel(mapfx_runner_state rs, mapfx_partial_out o,
                                                          mapfx_episode_rows r) {
  const int b = blockIdx.x;
  write_pre(rs, o, r, b, 0);  // reset(): update(pre_transition_data, ts=0) (:62-76), all envs
  if (threadIdx.x == 0) {
    rs.alive[b] = 1;
    rs.alive_prev[b] = 1;
    rs.bs[b] = b;
    if (rs.bs_inv) rs.bs_inv[b] = b;
    rs.ep_return[b] = 0.0;
    rs.ep_length[b] = 0;
    if (b == 0) {
      rs.counts[0] = rs.B;
      rs.counts[1] = rs.B;
      rs.env_steps[0] = 0;
    }
  }
  for (int n = threadIdx.x; n < rs.N; n += blockDim.x) rs.env_actions[(int64_t)b * rs.N + n] = 4;
}

__device__ inline int64_t load_act(const void* p, int dtype, int64_t i) {
  if (dtype == MAPFX_I8) return ((const int8_t*)p)[i];
  if (dtype == MAPFX_I32) return ((const int32_t*)p)[i];
  return ((const int64_t*)p)[i];
}

// update({"actions": actions.unsqueeze(1)}, bs=envs_not_terminated, ts) (:104-110) and
// the OneHot preprocess (components/transforms.py) of the same rows
__global__ void runner_actions_kernel(mapfx_runner_state rs, const void* acts, int dtype,
                                      int64_t row_stride, int ts, mapfx_episode_rows r) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = (int)(i / rs.N), n = (int)(i - (int64_t)j * rs.N);
  if (j >= rs.counts[0]) return;
  const int64_t b = rs.bs[j];
  const int64_t a = load_act(acts, dtype, (int64_t)j * row_stride + n);
  if (r.actions) r.actions[b * r.actions_sb + (int64_t)ts * r.actions_st + n] = a;
  if (r.onehot) {
    float* oh = r.onehot + b * r.onehot_sb + (int64_t)ts * r.onehot_st + (int64_t)n * 5;
#pragma unroll
    for (int k = 0; k < 5; ++k) oh[k] = (a == k) ? 1.0f : 0.0f;
  }
  // the env receives only the envs that have not terminated (:116-121); the others
  // are never stepped again, whatever env_actions holds for them
  rs.env_actions[b * rs.N + n] = (int8_t)((a < -128 || a > 127) ? -1 : a);
}

// receive loop of one step (:125-173) for every env still running
__global__ void __launch_bounds__(RB) runner_post_kernel(mapfx_runner_state rs, const uint8_t* term,
                                                         mapfx_partial_out o, int ts,
                                                         mapfx_episode_rows r) {
  const int b = blockIdx.x;
  const uint8_t live = rs.alive[b];
  __syncthreads();  // every thread read alive[b] before thread 0 rewrites it
  if (live) {
    const double R = o.reward[b];
    const uint8_t tn = term[b] ? 1 : 0;
    if (threadIdx.x == 0) {
      if (r.reward) r.reward[(int64_t)b * r.reward_sb + (int64_t)ts * r.reward_st] = (float)R;
      // env_terminated = terminated and not info.get("episode_limit") (:146-150): MARL_PARTIAL's
      // info has no "episode_limit" key
      if (r.terminated) r.terminated[(int64_t)b * r.terminated_sb + (int64_t)ts * r.terminated_st] = tn;
      rs.ep_return[b] = rs.ep_return[b] + R;
      rs.ep_length[b] += 1;
      rs.alive[b] = tn ? 0 : 1;   // (env_steps: counted by the compaction, no atomics here)
    }
    if (ts + 1 < r.max_t) write_pre(rs, o, r, b, ts + 1);
  }
  if (threadIdx.x == 0) rs.alive_prev[b] = live;
}

// envs_not_terminated (:123) for the next MAC call: ascending indices of alive_prev,
// padded with the first one (so a MAC indexing rows by `bs` only sees running envs);
// counts = {len(bs), number alive}.  One workgroup: per-thread chunk counts, a
// shuffle scan inside each wave and one barrier for the 16 wave totals.
constexpr int CT = 1024;
__global__ void __launch_bounds__(CT) runner_compact_kernel(mapfx_runner_state rs, int32_t* counts_out) {
  __shared__ int wsum[CT / 64];
  __shared__ int wsum_a[CT / 64];
  const int chunk = (rs.B + CT - 1) / CT;
  const int lo = threadIdx.x * chunk, hi = min(rs.B, lo + chunk);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int c = 0, ca = 0;
  for (int b = lo; b < hi; ++b) {
    c += rs.alive_prev[b] ? 1 : 0;
    ca += rs.alive[b] ? 1 : 0;
  }
  int x = c;  // inclusive scan over the wave's lanes
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  int xa = ca;  // the wave's alive count
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) xa += __shfl_xor(xa, o);
  if (lane == 63) wsum[wv] = x;
  if (lane == 0) wsum_a[wv] = xa;
  __syncthreads();
  int off = 0, total = 0, total_a = 0;
#pragma unroll
  for (int i = 0; i < CT / 64; ++i) {
    const int v = wsum[i];
    off += i < wv ? v : 0;
    total += v;
    total_a += wsum_a[i];
  }
  int o = off + x - c;  // exclusive prefix of this thread's chunk
  for (int b = lo; b < hi; ++b) {
    const bool in = rs.alive_prev[b] != 0;
    if (rs.bs_inv) rs.bs_inv[b] = in ? o : -1;  // where the next MAC call puts env b's row
    if (in) rs.bs[o++] = b;
  }
  __syncthreads();  // bs[0] written
  const int64_t first = total > 0 ? rs.bs[0] : 0;
  for (int j = total + threadIdx.x; j < rs.B; j += CT) rs.bs[j] = first;
  if (threadIdx.x == 0) {
    rs.counts[0] = total;
    rs.counts[1] = total_a;
    rs.env_steps[0] += total;  // the envs stepped this step: env_steps_this_run (:142)
    if (counts_out) {  // possibly pinned host memory
      counts_out[0] = total;
      counts_out[1] = total_a;
    }
  }
}

int check_rs(const mapfx_runner_state* rs) {
  if (!rs || rs->B < 0 || rs->N < 1 || rs->D < 0 || !rs->alive || !rs->alive_prev || !rs->bs ||
      !rs->counts || !rs->ep_return || !rs->ep_length || !rs->env_steps || !rs->env_actions)
    return err(MAPFX_EINVAL, "runner state: NULL field or bad B/N/D");
  return MAPFX_OK;
}

}  // namespace

extern "C" {

int mapfx_runner_begin(const mapfx_runner_state* rs, const mapfx_partial_out* out,
                       const mapfx_episode_rows* rows, void* stream) {
  int rc = check_rs(rs);
  if (rc) return rc;
  if (!out || !rows || !out->obs || !out->state || !out->avail)
    return err(MAPFX_EINVAL, "runner_begin: NULL out / rows");
  if (rs->B == 0) return MAPFX_OK;
  hipLaunchKernelGGL(runner_begin_kernel, dim3(rs->B), dim3(RB), 0, (hipStream_t)stream, *rs, *out, *rows);
  return launch_ok("runner_begin_kernel launch");
}

int mapfx_runner_actions(const mapfx_runner_state* rs, const void* actions, int32_t action_dtype,
                         int64_t row_stride, int32_t ts, const mapfx_episode_rows* rows,
                         void* stream) {
  int rc = check_rs(rs);
  if (rc) return rc;
  if (!actions || !rows) return err(MAPFX_EINVAL, "runner_actions: NULL actions / rows");
  if (action_dtype < MAPFX_I8 || action_dtype > MAPFX_I64) return err(MAPFX_EINVAL, "runner_actions: bad dtype");
  if (ts < 0 || ts >= rows->max_t) return err(MAPFX_EINVAL, "runner_actions: ts outside the batch");
  const int64_t total = (int64_t)rs->B * rs->N;
  if (total == 0) return MAPFX_OK;
  hipLaunchKernelGGL(runner_actions_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, *rs, actions, (int)action_dtype, row_stride, (int)ts, *rows);
  return launch_ok("runner_actions_kernel launch");
}

int mapfx_runner_post(const mapfx_runner_state* rs, const uint8_t* terminated,
                      const mapfx_partial_out* out, int32_t ts, int32_t* counts_out,
                      const mapfx_episode_rows* rows, void* stream) {
  int rc = check_rs(rs);
  if (rc) return rc;
  if (!terminated || !out || !rows || !out->reward || !out->obs || !out->state || !out->avail)
    return err(MAPFX_EINVAL, "runner_post: NULL terminated / out / rows");
  if (ts < 0 || ts >= rows->max_t) return err(MAPFX_EINVAL, "runner_post: ts outside the batch");
  if (rs->B == 0) return MAPFX_OK;
  hipLaunchKernelGGL(runner_post_kernel, dim3(rs->B), dim3(RB), 0, (hipStream_t)stream, *rs, terminated,
                     *out, (int)ts, *rows);
  if ((rc = launch_ok("runner_post_kernel launch"))) return rc;
  hipLaunchKernelGGL(runner_compact_kernel, dim3(1), dim3(CT), 0, (hipStream_t)stream, *rs, counts_out);
  return launch_ok("runner_compact_kernel launch");
}

int mapfx_runner_step(mapfx_partial_t* h, const mapfx_partial_state* st, const mapfx_partial_out* out,
                      const mapfx_runner_state* rs, const void* actions, int32_t action_dtype,
                      int64_t row_stride, int32_t ts, int32_t* counts_out,
                      const mapfx_episode_rows* rows, void* stream) {
  int rc = check_rs(rs);
  if (rc) return rc;
  if (!rows) return err(MAPFX_EINVAL, "runner_step: NULL rows");
  if (ts < 0 || ts >= rows->max_t) return err(MAPFX_EINVAL, "runner_step: ts outside the batch");
  if (!rs->bs_inv)  // the unfused form: a separate actions pass into env_actions
    return (rc = mapfx_runner_actions(rs, actions, action_dtype, row_stride, ts, rows, stream)) ? rc
           : (rc = mapfx_partial_step(h, st, rs->env_actions, MAPFX_I8, out, stream))
               ? rc : mapfx_runner_post(rs, st->terminated, out, ts, counts_out, rows, stream);
  // the env step reads each env's actions from the MAC's output (row bs_inv[b]) and
  // writes the actions / one-hot rows at ts itself; when the batch has observation rows
  // it also writes those of the envs running before it (rs->alive, updated only by the
  // post kernel) straight into time row ts + 1, so the post kernel moves no observation
  // bytes
  mapfx_runner_acts ra;
  memset(&ra, 0, sizeof ra);
  // the post pass in the env step's write-back too (the one-wave-per-env-group kernel),
  // and with it the compaction for the next MAC call as the launch's last workgroup:
  // alive flags and the row map double-buffered by step parity (alive / alive_prev =
  // A[0] / A[1], bs_inv = [2][B]; A[ts & 1] = running before step ts)
  const bool fpost = mapfx_partial_fuses_post(h) != 0;
  const int par = ts & 1;
  ra.act_row = rs->bs_inv + (fpost ? (int64_t)par * rs->B : 0);
  ra.act_row_stride = row_stride;
  ra.ep_actions = rows->actions;
  ra.ep_actions_sb = rows->actions_sb;
  ra.ep_actions_st = rows->actions_st;
  ra.ep_onehot = rows->onehot;
  ra.ep_onehot_sb = rows->onehot_sb;
  ra.ep_onehot_st = rows->onehot_st;
  ra.ts = ts;
  const bool nxt = ts + 1 < rows->max_t;
  uint8_t* const a_in = par ? rs->alive_prev : rs->alive;   // A[ts & 1]
  uint8_t* const a_out = par ? rs->alive : rs->alive_prev;  // A[(ts + 1) & 1]
  if (fpost) {
    ra.alive = a_in;
    ra.alive_prev = a_out;
    ra.cmp_alive = a_in;
    ra.cmp_bs = rs->bs;
    ra.cmp_bs_inv = rs->bs_inv + (int64_t)(par ^ 1) * rs->B;
    ra.cmp_counts = rs->counts;
    ra.cmp_env_steps = rs->env_steps;
    ra.cmp_counts_out = counts_out;
    ra.cmp_B = rs->B;
    ra.ep_return = rs->ep_return;
    ra.ep_length = rs->ep_length;
    ra.ep_reward = rows->reward;
    ra.ep_reward_sb = rows->reward_sb;
    ra.ep_reward_st = rows->reward_st;
    ra.ep_term = rows->terminated;
    ra.ep_term_sb = rows->terminated_sb;
    ra.ep_term_st = rows->terminated_st;
    ra.ep_state = nxt && rows->state ? rows->state + (int64_t)(ts + 1) * rows->state_st : nullptr;
    ra.ep_state_sb = rows->state_sb;
    ra.ep_avail = nxt && rows->avail ? rows->avail + (int64_t)(ts + 1) * rows->avail_st : nullptr;
    ra.ep_avail_sb = rows->avail_sb;
    ra.ep_filled = nxt && rows->filled ? rows->filled + (int64_t)(ts + 1) * rows->filled_st : nullptr;
    ra.ep_filled_sb = rows->filled_sb;
  }
  float* obs_row = rows->obs && nxt ? rows->obs + (int64_t)(ts + 1) * rows->obs_st : nullptr;
  if ((rc = mapfx_partial_step_runner(h, st, actions, action_dtype, &ra, out, obs_row, rows->obs_sb,
                                      fpost ? a_in : rs->alive, stream)))
    return rc;
  if (fpost) return MAPFX_OK;  // (the compaction ran as the launch's last workgroup)
  if (!rows->obs) return mapfx_runner_post(rs, st->terminated, out, ts, counts_out, rows, stream);
  mapfx_episode_rows r2 = *rows;
  r2.obs = nullptr;
  return mapfx_runner_post(rs, st->terminated, out, ts, counts_out, &r2, stream);
}

int mapfx_host_ring_alloc(int32_t n, int32_t** host_ptr, int32_t** dev_ptr) {
  if (n < 1 || !host_ptr || !dev_ptr) return err(MAPFX_EINVAL, "host_ring_alloc: bad arguments");
  *host_ptr = nullptr;
  *dev_ptr = nullptr;
  void* p = nullptr;
  if (hipHostMalloc(&p, sizeof(int32_t) * (size_t)n, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return err(MAPFX_ENOMEM, "hipHostMalloc (mapped, coherent) failed");
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    (void)hipHostFree(p);
    return err(MAPFX_EHIP, "hipHostGetDevicePointer failed");
  }
  memset(p, 0, sizeof(int32_t) * (size_t)n);
  *host_ptr = (int32_t*)p;
  *dev_ptr = (int32_t*)d;
  return MAPFX_OK;
}

void mapfx_host_ring_free(int32_t* host_ptr) {
  if (host_ptr) (void)hipHostFree(host_ptr);
}

}  // extern "C"

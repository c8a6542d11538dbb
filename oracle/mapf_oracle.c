/*
 * CPU ORACLE (C) — test infrastructure / CPU baseline only, never product code.
 *
 * A direct C restatement of the reference MAPF_GRID step and observations
 * (DongmingShenDS/MAPF-MARL, MARL-curve-main/src/envs/mapf_gridworld.py:85-224),
 * the marl_partial window (envs/marl_partial.py:323-342) and PRIMAL _observe
 * (envs/mapf_primal.py:343-386), batched over E independent envs with OpenMP.
 * Same state layout as include/mapfx.h so tests can compare buffers directly.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library (oracle/liboracle.so), and only as the checker / the timed CPU
 * baseline.  Pinned bit-for-bit against the tests/golden fixtures (reference outputs)
 * by tests/test_oracle_c.py.
 *
 * It deliberately follows the reference's own formulation — unpadded grid,
 * explicit bounds tests, occupancy rebuilt from positions every step, the
 * O(N^2) edge scan of :364-383 — not the HIP kernel's design.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct orc_cfg {
  int32_t H, W, N, E;
  int64_t env_offset;
  int32_t limit;
  double step_rew, collide_rew;
  int32_t map_shared;
  int64_t map_stride; /* bytes per env bitmap */
} orc_cfg;

static const int DR[5] = {-1, 1, 0, 0, 0}; /* :323-332 */
static const int DC[5] = {0, 0, -1, 1, 0};

static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

int orc_action(uint64_t seed, int64_t env, int32_t t, int32_t agent) {
  uint64_t k = seed ^ ((uint64_t)env * 0xD1B54A32D192ED03ull) ^
               ((uint64_t)(uint32_t)t * 0xABC98388FB8FAC03ull) ^
               ((uint64_t)(uint32_t)agent * 0x8CB92BA72F3D8DD7ull);
  return (int)(splitmix64(k) % 5ull);
}

/* G[r][c] = -1 if obstacle else 0  (:282-288) */
static int grid_at(const orc_cfg* c, const uint8_t* bits, int r, int col) {
  int idx = r * c->W + col;
  return ((bits[idx >> 3] >> (idx & 7)) & 1) ? -1 : 0;
}

static const uint8_t* env_bits(const orc_cfg* c, const uint8_t* bits, int64_t e) {
  return bits + (c->map_shared ? 0 : e * c->map_stride);
}

/* occ = G + agent counts (:132-135, 297-299) */
static void build_occ(const orc_cfg* c, const uint8_t* bits, const int32_t* pos, int32_t* occ) {
  for (int r = 0; r < c->H; ++r)
    for (int col = 0; col < c->W; ++col) occ[r * c->W + col] = grid_at(c, bits, r, col);
  for (int a = 0; a < c->N; ++a) occ[pos[2 * a] * c->W + pos[2 * a + 1]] += 1;
}

static int in_bounds(const orc_cfg* c, int r, int col) {
  return 0 <= r && r < c->H && 0 <= col && col < c->W; /* :270-272 */
}

/* One env step (:85-141).  Returns 0, or -1 if an action is outside 0..4
 * (the reference asserts before touching state, :91-92). */
static int step_env(const orc_cfg* c, int64_t e, int32_t* pos, const int32_t* goal, uint8_t* done,
                    int32_t* t, int32_t* steps, const uint8_t* bits, const int32_t* act,
                    double* reward, uint8_t* node_out, uint16_t* edge_out, int32_t* occ,
                    int32_t* newp, double* rew, int32_t* cnt) {
  const int N = c->N, H = c->H, W = c->W;
  for (int i = 0; i < N; ++i)
    if (act[i] < 0 || act[i] > 4) return -1;
  build_occ(c, bits, pos, occ); /* pre-step _full_obs */
  t[0] += 1;                     /* :93 */
  for (int i = 0; i < N; ++i) {  /* :99-118 */
    int r = pos[2 * i], col = pos[2 * i + 1];
    int nr = r, nc = col, envc = 0;
    rew[i] = 0.0;
    if (!done[i]) {
      if (steps) steps[i] += 1;
      if (act[i] != 4) { /* __agent_step :319-342 */
        int cr = r + DR[act[i]], cc = col + DC[act[i]];
        if (!in_bounds(c, cr, cc) || occ[cr * W + cc] == -1)
          envc = 1;
        else {
          nr = cr;
          nc = cc;
        }
      }
      if (envc) rew[i] = rew[i] + c->collide_rew;
      rew[i] = rew[i] + c->step_rew;
    }
    newp[2 * i] = nr;
    newp[2 * i + 1] = nc;
    if (nr == goal[2 * i] && nc == goal[2 * i + 1]) done[i] = 1; /* :112-114 */
    if (t[0] >= c->limit) done[i] = 1;                            /* :116-117 */
  }
  /* __count_node_collision :344-362 */
  memset(cnt, 0, sizeof(int32_t) * H * W);
  for (int i = 0; i < N; ++i) cnt[newp[2 * i] * W + newp[2 * i + 1]] += 1;
  /* __count_edge_collision :364-383, key(p) = H*p[1] + p[0] (:465-468) */
  for (int i = 0; i < N; ++i) {
    const int node = cnt[newp[2 * i] * W + newp[2 * i + 1]] > 1 ? 1 : 0;
    int edge = 0;
    const int64_t oi = (int64_t)H * pos[2 * i + 1] + pos[2 * i];
    const int64_t ni = (int64_t)H * newp[2 * i + 1] + newp[2 * i];
    if (oi != ni) {
      for (int j = 0; j < N; ++j) {
        if (j == i) continue;
        const int64_t oj = (int64_t)H * pos[2 * j + 1] + pos[2 * j];
        const int64_t nj = (int64_t)H * newp[2 * j + 1] + newp[2 * j];
        if (oj == ni && nj == oi && nj != ni) ++edge;
      }
    }
    rew[i] = rew[i] + c->collide_rew * (double)node; /* :127-130 */
    rew[i] = rew[i] + c->collide_rew * (double)edge;
    if (node_out) node_out[i] = (uint8_t)node;
    if (edge_out) edge_out[i] = (uint16_t)edge; /* <= N - 1 < 2^16: exact */
  }
  double R = 0.0; /* sum(rewards): naive left fold (:141, CPython <= 3.11) */
  for (int i = 0; i < N; ++i) R = R + rew[i];
  if (reward) *reward = R;
  memcpy(pos, newp, sizeof(int32_t) * 2 * N);
  (void)e;
  return 0;
}

/* Observations of the current state of one env. */
static void observe_env(const orc_cfg* c, const int32_t* pos, const int32_t* goal,
                        const uint8_t* done, const uint8_t* bits, int32_t* occ, uint8_t* avail,
                        uint8_t* term, void* obs_full, int obs16, void* obs_window, int window,
                        uint8_t* obs_primal, double* primal_vec, int psize, const double* lut) {
  const int N = c->N, H = c->H, W = c->W;
  build_occ(c, bits, pos, occ);
  if (avail) { /* :203-224 */
    for (int i = 0; i < N; ++i) {
      int m = 16;
      for (int d = 0; d < 4; ++d) {
        int r = pos[2 * i] + DR[d], col = pos[2 * i + 1] + DC[d];
        if (in_bounds(c, r, col) && occ[r * W + col] != -1) m |= 1 << d;
      }
      avail[i] = (uint8_t)m;
    }
  }
  if (term) {
    int all = 1;
    for (int i = 0; i < N; ++i) all &= done[i] ? 1 : 0;
    *term = (uint8_t)all;
  }
  if (obs_full) { /* :143-192 */
    for (int k = 0; k < H * W; ++k) {
      if (obs16)
        ((int16_t*)obs_full)[k] = (int16_t)occ[k];
      else
        ((int8_t*)obs_full)[k] = (int8_t)occ[k];
    }
  }
  if (obs_window) { /* marl_partial.py:323-342 */
    const int ww = window * window;
    for (int a = 0; a < N; ++a) {
      const int tr = pos[2 * a] - window / 2, tc = pos[2 * a + 1] - window / 2;
      for (int y = 0; y < window; ++y)
        for (int x = 0; x < window; ++x) {
          int o0 = 0, o1 = 0;
          const int i = tr + y, j = tc + x;
          if (!in_bounds(c, i, j))
            o0 = 1;
          else if (occ[i * W + j] == -1)
            o0 = 1;
          else if (occ[i * W + j] > 0)
            o1 = occ[i * W + j];
          const int64_t b = (int64_t)a * 2 * ww + y * window + x;
          if (obs16) {
            ((int16_t*)obs_window)[b] = (int16_t)o0;
            ((int16_t*)obs_window)[b + ww] = (int16_t)o1;
          } else {
            ((int8_t*)obs_window)[b] = (int8_t)o0;
            ((int8_t*)obs_window)[b + ww] = (int8_t)o1;
          }
        }
    }
  }
  if (obs_primal || primal_vec) { /* mapf_primal.py:343-386 */
    const int S = psize, ss = S * S;
    for (int a = 0; a < N; ++a) {
      const int pr = pos[2 * a], pc = pos[2 * a + 1];
      const int tr = pr - S / 2, tc = pc - S / 2;
      if (obs_primal) {
        uint8_t* m = obs_primal + (int64_t)a * 4 * ss;
        memset(m, 0, 4 * ss);
        for (int i = tr; i < tr + S; ++i)
          for (int j = tc; j < tc + S; ++j) {
            const int q = (i - tr) * S + (j - tc);
            if (i >= H || i < 0 || j >= W || j < 0) {
              m[3 * ss + q] = 1;
              continue;
            }
            const int g = grid_at(c, bits, i, j);
            const int n_here = occ[i * W + j] - g;
            if (g == -1 && n_here == 0) m[3 * ss + q] = 1;
            if (n_here > 0) m[q] = 1;
            if (i == goal[2 * a] && j == goal[2 * a + 1]) m[ss + q] = 1;
          }
        for (int b = 0; b < N; ++b) {
          if (b == a) continue;
          const int br = pos[2 * b], bc = pos[2 * b + 1];
          if (br < tr || br >= tr + S || bc < tc || bc >= tc + S) continue;
          int x = goal[2 * b], y = goal[2 * b + 1];
          x = x < tr ? tr : (x > tr + S - 1 ? tr + S - 1 : x);
          y = y < tc ? tc : (y > tc + S - 1 ? tc + S - 1 : y);
          m[2 * ss + (x - tr) * S + (y - tc)] = 1;
        }
      }
      if (primal_vec) {
        const int dx = goal[2 * a] - pr, dy = goal[2 * a + 1] - pc;
        const double mag = lut ? lut[dx * dx + dy * dy] : pow((double)(dx * dx + dy * dy), 0.5);
        double vx = dx, vy = dy;
        if (mag != 0.0) {
          vx = vx / mag;
          vy = vy / mag;
        }
        primal_vec[3 * a] = vx;
        primal_vec[3 * a + 1] = vy;
        primal_vec[3 * a + 2] = mag;
      }
    }
  }
}

/* Batched step of E envs.  Outputs may be NULL.  Returns the number of envs
 * rejected for an out-of-range action (left unchanged). */
int orc_step(const orc_cfg* c, int32_t* pos, const int32_t* goal, uint8_t* done, int32_t* t,
             int32_t* steps, const uint8_t* bits, const int32_t* actions, double* reward,
             uint8_t* node, uint16_t* edge, int nthreads) {
  const int N = c->N;
  int bad = 0;
#pragma omp parallel num_threads(nthreads) reduction(+ : bad)
  {
    int32_t* occ = (int32_t*)malloc(sizeof(int32_t) * c->H * c->W);
    int32_t* cnt = (int32_t*)malloc(sizeof(int32_t) * c->H * c->W);
    int32_t* newp = (int32_t*)malloc(sizeof(int32_t) * 2 * N);
    double* rew = (double*)malloc(sizeof(double) * N);
#pragma omp for schedule(static)
    for (int64_t e = 0; e < c->E; ++e) {
      int rc = step_env(c, e, pos + e * 2 * N, goal + e * 2 * N, done + e * N, t + e,
                        steps ? steps + e * N : NULL, env_bits(c, bits, e), actions + e * N,
                        reward ? reward + e : NULL, node ? node + e * N : NULL,
                        edge ? edge + e * N : NULL, occ, newp, rew, cnt);
      if (rc) ++bad;
    }
    free(occ);
    free(cnt);
    free(newp);
    free(rew);
  }
  return bad;
}

int orc_observe(const orc_cfg* c, const int32_t* pos, const int32_t* goal, const uint8_t* done,
                const uint8_t* bits, uint8_t* avail, uint8_t* term, void* obs_full,
                void* obs_window, int window, uint8_t* obs_primal, double* primal_vec, int psize,
                int nthreads) {
  const int N = c->N;
  const int obs16 = N > 127;
  const int es = obs16 ? 2 : 1;
  double* lut = NULL;
  if (primal_vec) {
    const int n = (c->H - 1) * (c->H - 1) + (c->W - 1) * (c->W - 1) + 1;
    lut = (double*)malloc(sizeof(double) * n);
    for (int i = 0; i < n; ++i) lut[i] = pow((double)i, 0.5);
  }
#pragma omp parallel num_threads(nthreads)
  {
    int32_t* occ = (int32_t*)malloc(sizeof(int32_t) * c->H * c->W);
#pragma omp for schedule(static)
    for (int64_t e = 0; e < c->E; ++e) {
      observe_env(c, pos + e * 2 * N, goal + e * 2 * N, done + e * N, env_bits(c, bits, e), occ,
                  avail ? avail + e * N : NULL, term ? term + e : NULL,
                  obs_full ? (char*)obs_full + e * (int64_t)c->H * c->W * es : NULL, obs16,
                  obs_window ? (char*)obs_window + e * (int64_t)N * 2 * window * window * es : NULL,
                  window, obs_primal ? obs_primal + e * (int64_t)N * 4 * psize * psize : NULL,
                  primal_vec ? primal_vec + e * (int64_t)N * 3 : NULL, psize, lut);
    }
    free(occ);
  }
  free(lut);
  return 0;
}

/* T steps of every env with generator actions (seed, env_offset + e, t0 + k);
 * after each step the avail mask and the window observation are produced, as
 * the runner loop needs them (runners/parallel_runner.py:227-231).  Used as
 * the timed CPU baseline and for long-horizon parity.  Outputs hold the last
 * step's values. */
int orc_rollout(const orc_cfg* c, int32_t T, uint64_t seed, int32_t t0, int32_t* pos,
                const int32_t* goal, uint8_t* done, int32_t* t, int32_t* steps,
                const uint8_t* bits, double* reward, uint8_t* node, uint16_t* edge,
                uint8_t* avail, void* obs_window, int window, int nthreads) {
  const int N = c->N;
  const int es = N > 127 ? 2 : 1;
#pragma omp parallel num_threads(nthreads)
  {
    int32_t* occ = (int32_t*)malloc(sizeof(int32_t) * c->H * c->W);
    int32_t* cnt = (int32_t*)malloc(sizeof(int32_t) * c->H * c->W);
    int32_t* newp = (int32_t*)malloc(sizeof(int32_t) * 2 * N);
    double* rew = (double*)malloc(sizeof(double) * N);
    int32_t* act = (int32_t*)malloc(sizeof(int32_t) * N);
#pragma omp for schedule(static)
    for (int64_t e = 0; e < c->E; ++e) {
      for (int k = 0; k < T; ++k) {
        for (int a = 0; a < N; ++a) act[a] = orc_action(seed, c->env_offset + e, t0 + k, a);
        step_env(c, e, pos + e * 2 * N, goal + e * 2 * N, done + e * N, t + e,
                 steps ? steps + e * N : NULL, env_bits(c, bits, e), act,
                 reward ? reward + e : NULL, node ? node + e * N : NULL,
                 edge ? edge + e * N : NULL, occ, newp, rew, cnt);
        observe_env(c, pos + e * 2 * N, goal + e * 2 * N, done + e * N, env_bits(c, bits, e), occ,
                    avail ? avail + e * N : NULL, NULL, NULL, es == 2,
                    obs_window ? (char*)obs_window + e * (int64_t)N * 2 * window * window * es
                               : NULL,
                    window, NULL, NULL, 0, NULL);
      }
    }
    free(occ);
    free(cnt);
    free(newp);
    free(rew);
    free(act);
  }
  return 0;
}

int orc_max_threads(void) { return omp_get_max_threads(); }

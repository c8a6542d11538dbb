// mapfx.hip — MI355X (gfx950, CDNA4) batched MAPF gridworld step.
//
// One launch steps E independent envs of the reference's MAPF_GRID
// (MARL-curve-main/src/envs/mapf_gridworld.py:85-141) and emits its
// observations (:143-224), the marl_partial window (envs/marl_partial.py:323-342)
// and the PRIMAL window (envs/mapf_primal.py:343-386).
//
// Execution model:
//   * an env is owned by a lane group of L = pow2ceil(N) lanes (<= 256) of one
//     workgroup; lane l owns agents l, l+L, ... (APL agents per lane);
//     N = 16 puts 4 envs in a wavefront, 16 envs in a 256-thread workgroup;
//   * the env's occupancy lives in LDS as a PADDED cell map: one byte per cell
//     (u16 when N > 127) = obstacle flag (top bit) | agent count.  The border
//     of P cells is "obstacle, 0 agents", which is exactly how the reference
//     treats out-of-bounds cells for moves (:336-337), avail (:209-222) and the
//     windows (marl_partial.py:335-337, mapf_primal.py:356-359), so no bounds
//     test survives in the inner loops.  occ = count - flag.
//   * per step: moves test the PRE-step map (quirk 1: an obstacle is passable
//     while an agent stands on it), agent counts are then moved with LDS
//     atomics, node collisions read the post-step count, edge collisions scan
//     the env's agents only for agents that moved into a pre-occupied cell;
//     rewards are folded in fp64 in agent order by one lane (quirk 4);
//   * window observations are staged in LDS and leave as 16-byte stores.
//
// No MFMA: the step is integer gather/scatter + a short fp64 fold; HBM-bound.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cxxabi.h>
#include <math.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <utility>
#include <new>
#include <string>

#include "mapfx.h"

namespace {

thread_local std::string g_last_error;

// the host stub of the calling thread's most recent launch (mapfx_last_kernel)
thread_local const void* g_last_kernel = nullptr;

int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__host__ __device__ inline int gen_action(uint64_t seed, int64_t env, int32_t t, int32_t agent) {
  uint64_t k = seed ^ ((uint64_t)env * 0xD1B54A32D192ED03ull) ^
               ((uint64_t)(uint32_t)t * 0xABC98388FB8FAC03ull) ^
               ((uint64_t)(uint32_t)agent * 0x8CB92BA72F3D8DD7ull);
  return (int)(splitmix64(k) % 5ull);
}

// x / d for 0 <= x < 2^32, 1 <= d < 2^16, with m = ceil(2^48 / d).
__device__ inline int fastdiv(int x, uint64_t m) {
  return (int)(((uint64_t)(uint32_t)x * m) >> 48);
}

// Launch geometry + env constants (uniform per launch).
struct Geo {
  int H, W, N, E;
  long long env_offset;
  int L, lshift, EPB, BT;
  int P, pl, pitch, rows;  // padded LDS map: rows x pitch cells, interior at (P, pl)
  int map_words;           // u32 words of one env's LDS map
  int bits_words;          // u32 words of the bitmap actually used: ceil(H*W/32)
  long long map_stride;    // bytes per env bitmap in global memory
  int map_shared;
  uint64_t m_wpr;          // fastdiv magic for words-per-padded-row
  uint64_t m_W;            // fastdiv magic for W
  uint64_t m_W4;           // fastdiv magic for W/4
  uint64_t m_pitch;        // fastdiv magic for the padded pitch (cells)
  uint32_t m_pitch24;      // ceil(2^24 / pitch): cell -> row with one v_mul_hi_u32_u24
  int wpr;
  // LDS regions (byte offsets from the dynamic LDS base)
  int off_map, off_bits, off_oldc, off_newc, off_rc, off_goal, off_rew, off_flag;
  int map_env_bytes, bits_env_bytes;
  int gen_lds;             // dynamic LDS of a generic-kernel block
  // deferred reward fold of the generic rollout (one env per block): per-agent reward
  // CODES of the last fold_R steps in an LDS ring at off_rew (fold_R = 0: per-step
  // fold), code_pitch bytes per step, and the fp64 rewards of the codes < 32 at off_ctab
  int fold_R, code_pitch, off_ctab;
  uint64_t m_N, m_w, m_ww, m_wlen;  // fastdiv magics for the block-cooperative window writer
  int window, wlen;        // marl_partial window w, 2*w*w
  int psize;               // PRIMAL observation size s
  int obs_mode;
  int limit;
  double step_rew, collide_rew;
  // wave-local fast path (N <= 64: an env never spans two wavefronts)
  int wave_ok, EPW;
  int wv_off_map, wv_off_dep, wv_off_bits, wv_off_rew, wv_lds;
  int wv_bits_env_bytes, wv_rew_buf, wv_rew_row;  // the reward rows are double-buffered
  int wv_off_split, wv_split_ok;  // store-wave split: its LDS starts at wv_off_split
  int wv_fast;                     // build_map_rows_fast applies (W <= 64, pitch % 8 == 0)
  int nblk;                        // grid size of the launch (set in the kernel from its kernargs)
};
constexpr int MAPFX_FAST_WPR = 24;  // words per padded row handled by build_map_rows_fast

struct Args {
  int32_t* pos;
  const int32_t* goal;
  const int32_t* init_pos;
  uint8_t* done;
  int32_t* t;
  int32_t* steps;
  const uint8_t* bits;
  const void* actions;
  int act_dtype;
  int use_rng;
  uint64_t seed;
  int t0;
  int T;
  int autoreset;
  int do_step;
  double* reward;
  float* reward_f32;
  uint8_t* term;
  uint8_t* node;
  uint8_t* edge;
  uint8_t* avail;
  void* obs_full;
  void* obs_window;
  void* obs_window_occ;
  uint8_t* obs_primal;
  double* primal_vec;
  int32_t* traj_pos;
  uint8_t* traj_done;
  int32_t* traj_t;
  int32_t* err;
  const double* pow_lut;
};

// The pointers a launch reads first also travel as leading scalar kernel parameters:
// built with -amdgpu-kernarg-preload-count=16 they arrive in SGPRs (kernarg preload;
// aggregates are never preloaded), so the state loads issue before the rest of the
// kernargs has been fetched from memory.
#define MAPFX_HOT_PARAMS                                                                     \
  int32_t *hp_pos, const int32_t *hp_goal, uint8_t *hp_done, const uint8_t *hp_bits,       \
      const void *hp_act, int32_t *hp_t, uint32_t hp_geo, uint32_t hp_nm
// ... and what the first loads' addresses need: hp_geo = H | W << 13 | P << 26 |
// wv_fast << 31 (the bitmap stride follows from H, W: mapfx_map_stride) and hp_nm =
// grid size | (T >= 16) << 26 | act_dtype << 27 | do_step << 29 | use_rng << 30 |
// map_shared << 31 (the XCD-aware block order needs the grid size, gridDim comes from
// the implicit kernargs; a rollout of at least 16 steps fetches its first action block
// without a clamp to T, and with every env full E = grid size x envs per block, so the
// first action loads need no kernarg from memory either).  14 dwords: all that
// kernel-argument preload fills next to the kernarg pointer.
#define MAPFX_HOT_APPLY(a, g)                                                                \
  (a).pos = hp_pos, (a).goal = hp_goal, (a).done = hp_done, (a).bits = hp_bits,             \
  (a).actions = hp_act, (a).t = hp_t,                                                       \
  (g).H = (int)(hp_geo & 0x1FFFu), (g).W = (int)((hp_geo >> 13) & 0x1FFFu),                 \
  (g).P = (int)((hp_geo >> 26) & 0x1Fu), (g).wv_fast = (int)(hp_geo >> 31),                \
  (g).bits_words = ((g).H * (g).W + 31) >> 5, (g).map_shared = 0,                           \
  (g).map_stride = (hp_nm >> 31) ? 0 : ((((g).H * (g).W + 7) >> 3) + 15) & ~15,            \
  (g).nblk = (int)(hp_nm & 0x3FFFFFFu), (a).act_dtype = (int)((hp_nm >> 27) & 3u),         \
  (a).do_step = (int)((hp_nm >> 29) & 1u), (a).use_rng = (int)((hp_nm >> 30) & 1u)
#define MAPFX_HOT_ARGS(a, g, nb)                                                             \
  (a).pos, (a).goal, (a).done, (a).bits, (a).actions, (a).t,                                \
      (uint32_t)(g).H | ((uint32_t)(g).W << 13) | ((uint32_t)(g).P << 26) |                 \
          ((uint32_t)(g).wv_fast << 31),                                                    \
      (uint32_t)(nb) | ((a).T >= 16 ? 1u << 26 : 0u) | ((uint32_t)((a).act_dtype & 3) << 27) |   \
          ((a).do_step ? 1u << 29 : 0u) | ((a).use_rng ? 1u << 30 : 0u) | ((g).map_shared ? 1u << 31 : 0u)

template <typename CellT>
struct CellTraits;
template <>
struct CellTraits<uint8_t> {
  static constexpr uint32_t OE = 0x80u;        // obstacle flag, 0 agents
  static constexpr uint32_t CNT = 0x7Fu;
  static constexpr uint32_t OE_WORD = 0x80808080u;
  static constexpr int PER_WORD_SHIFT = 2;     // 4 cells per u32
  __device__ static inline uint32_t inc(int cell) { return 1u << ((cell & 3) * 8); }
};
template <>
struct CellTraits<uint16_t> {
  static constexpr uint32_t OE = 0x8000u;
  static constexpr uint32_t CNT = 0x7FFFu;
  static constexpr uint32_t OE_WORD = 0x80008000u;
  static constexpr int PER_WORD_SHIFT = 1;     // 2 cells per u32
  __device__ static inline uint32_t inc(int cell) { return 1u << ((cell & 1) * 16); }
};

// (row, col) deltas of actions 0..3 (envs/mapf_gridworld.py:323-330)
__device__ inline int act_dr(int a) { return a == 0 ? -1 : (a == 1 ? 1 : 0); }
__device__ inline int act_dc(int a) { return a == 2 ? -1 : (a == 3 ? 1 : 0); }

__device__ inline int load_action(const void* p, int dtype, long long idx) {
  if (dtype == MAPFX_I8) return (int)((const int8_t*)p)[idx];
  if (dtype == MAPFX_I32) {
    return ((const int32_t*)p)[idx];
  }
  long long v = ((const int64_t*)p)[idx];
  return (v < -1 || v > 5) ? -1 : (int)v;  // any out-of-range value is invalid
}

// Bit (r*W + c) of the env's bitmap staged in LDS.
__device__ inline uint32_t map_bit(const uint32_t* bits, int idx) {
  return (bits[idx >> 5] >> (idx & 31)) & 1u;
}

// Build the padded occupancy map of one env from its LDS bitmap (no agents).
template <typename CellT>
__device__ inline void fill_map(const Geo& g, uint32_t* map32, const uint32_t* bits, int lane) {
  using CT = CellTraits<CellT>;
  constexpr int CPW = 1 << CT::PER_WORD_SHIFT;  // cells per word
  for (int wi = lane; wi < g.map_words; wi += g.L) {
    const int pr = fastdiv(wi, g.m_wpr);
    const int pw = wi - pr * g.wpr;
    const int r = pr - g.P;
    uint32_t word;
    if (r < 0 || r >= g.H) {
      word = CT::OE_WORD;
    } else {
      word = 0;
      const int c0 = pw * CPW - g.pl;
#pragma unroll
      for (int j = 0; j < CPW; ++j) {
        const int c = c0 + j;
        uint32_t ob = 1u;
        if (c >= 0 && c < g.W) ob = map_bit(bits, r * g.W + c);
        word |= (ob ? CT::OE : 0u) << (j * (32 / CPW));
      }
    }
    map32[wi] = word;
  }
}

// 32-bit LDS address of a pointer into dynamic shared memory
__device__ __forceinline__ __attribute__((unused)) uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

constexpr int MAPFX_FOLD_R = 8;  // deferred-fold ring depth of the generic rollout (power of two; 0 = off)
constexpr int MAPFX_FOLD_PRIO = 3;  // s_setprio of the deferred fold's chain (0: none)

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations,
// not for its global stores (a __syncthreads() drains every outstanding store --
// a full HBM write latency per barrier).  No value produced in global memory is
// read back inside a launch, so the step loop's barriers need LDS ordering only.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---------------------------------------------------------------------------
// Window observations of a block's envs (marl_partial.py:323-342), written by the
// whole block straight from the post-step LDS maps: the block's output region is
// contiguous ([env0 .. env0 + nenv) x N records), so thread t produces 16-byte
// chunks t, t + BT, ... of it -- every store is a coalesced dwordx4 and no record
// is staged.  Value j of the region is record q = j / VL, element i = j % VL, with
// VL = 2 w^2 (OCC = false: obstacle plane then agents plane, es bytes each) or w^2
// (OCC = true: the occupancy value occ = count - obstacle of each window cell, the
// reference's own map value, from which obstacle = (occ == -1), agents =
// max(occ, 0)).  Out-of-bounds window cells are the border's "obstacle, 0 agents".
// ---------------------------------------------------------------------------
template <typename CellT, bool OCC>
__device__ __forceinline__ int window_elem(uint32_t cv, int plane) {
  using CT = CellTraits<CellT>;
  const int occ = (int)(cv & CT::CNT) - ((cv & CT::OE) ? 1 : 0);
  if (OCC) return occ;
  return plane ? (occ > 0 ? occ : 0) : (occ == -1 ? 1 : 0);
}

template <typename CellT, bool OCC>
__device__ void write_windows(const Geo& g, const unsigned char* lds, const int* newc_blk,
                              unsigned char* dst, int nvals, int tid, int nt) {
  constexpr int es = (int)sizeof(CellT);
  constexpr int VPC = 16 / es;  // values per 16-byte chunk
  constexpr uint32_t VMASK = es == 1 ? 0xFFu : 0xFFFFu;
  const int w = g.window, h = w >> 1, ww = w * w;
  const int VL = OCC ? ww : 2 * ww;
  const uint64_t mVL = OCC ? g.m_ww : g.m_wlen;
  const int pitch = g.pitch;
  const int nchunks = (((uintptr_t)dst & 15) == 0) ? nvals / VPC : 0;
  for (int ch = tid; ch < nchunks; ch += nt) {
    const int v = ch * VPC;
    int q = fastdiv(v, mVL);
    int i = v - q * VL;
    int pl = 0;
    if (!OCC && i >= ww) {
      pl = 1;
      i -= ww;
    }
    int y = fastdiv(i, g.m_w);
    int x = i - y * w;
    int slot = fastdiv(q, g.m_N);
    const CellT* mp = (const CellT*)(lds + g.off_map + slot * g.map_env_bytes);
    int base = newc_blk[q] - h * pitch - h;
    uint32_t pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < VPC; ++j) {
      const uint32_t cv = mp[base + y * pitch + x];
      pk[(j * es) >> 2] |= ((uint32_t)window_elem<CellT, OCC>(cv, pl) & VMASK) << ((j * es * 8) & 31);
      if (j + 1 < VPC && ++x == w) {  // advance to value v + j + 1
        x = 0;
        if (++y == w) {
          y = 0;
          if (!OCC && pl == 0) {
            pl = 1;
          } else {
            pl = 0;
            ++q;
            slot = fastdiv(q, g.m_N);
            mp = (const CellT*)(lds + g.off_map + slot * g.map_env_bytes);
            base = newc_blk[q] - h * pitch - h;
          }
        }
      }
    }
    ((uint4*)dst)[ch] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  }
  // unaligned region or the tail: one value per thread and store
  for (int v = nchunks * VPC + tid; v < nvals; v += nt) {
    const int q = fastdiv(v, mVL);
    int i = v - q * VL;
    int pl = 0;
    if (!OCC && i >= ww) {
      pl = 1;
      i -= ww;
    }
    const int y = fastdiv(i, g.m_w), x = i - y * w;
    const int slot = fastdiv(q, g.m_N);
    const CellT* mp = (const CellT*)(lds + g.off_map + slot * g.map_env_bytes);
    const int e = window_elem<CellT, OCC>(mp[newc_blk[q] + (y - h) * pitch + x - h], pl);
    if (es == 1)
      dst[v] = (unsigned char)e;
    else
      ((int16_t*)dst)[v] = (int16_t)e;
  }
}

// obs_window_occ of u16 cells (N > 127, e.g. BASELINE C5), odd window W <= 7: one
// thread per window ROW of a record (segment (q, y) = W int16 at byte offset
// 2 (q W^2 + y W) of the block's region).  A row is (W + 1) / 2 + 1 LDS dwords
// realigned with v_alignbyte; occ = (cell & 0x7FFF) - (cell >> 15) for two cells at
// a time without a borrow between the halves (offset binary); it leaves as
// (W - 1) / 2 dwords + one u16, aligned either way.  Consecutive threads write
// consecutive rows (10 bytes apart at W = 5), ~5x fewer VALU operations per value
// than the per-value writer above.
template <int W>
__device__ void write_occ16_rows(const Geo& g, const unsigned char* lds, const int* newc_blk,
                                 unsigned char* dst, int nseg, int tid, int nt, int sg_begin = 0) {
  constexpr int NP = (W + 1) / 2;  // cell pairs per row (the last one half used)
  constexpr int h = W / 2;
  constexpr int U = 1;  // rows in flight per thread (2 or 4 measured no faster)
  typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
  const int pitch = g.pitch;
  const bool one_env = g.EPB == 1;
  const uint32_t lbase = lds_addr(lds + g.off_map);
  const bool dalign = (((uintptr_t)dst) & 2u) == 0;
  for (int sg0 = sg_begin + tid; sg0 < nseg; sg0 += U * nt) {
    int q[U], y[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int sg = sg0 + u * nt;
      ok[u] = sg < nseg;
      const int sv = ok[u] ? sg : sg0;
      q[u] = fastdiv(sv, g.m_w);
      y[u] = sv - q[u] * W;
    }
    int nq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) nq[u] = newc_blk[q[u]];
    uint32_t Wd[U][NP + 1], sh[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int slot = one_env ? 0 : fastdiv(q[u], g.m_N);
      const int e0 = nq[u] + (y[u] - h) * pitch - h;  // first cell of the row
      const uint32_t A = lbase + (uint32_t)(slot * g.map_env_bytes) + 2u * (uint32_t)e0;
      lds_cu32* src = (lds_cu32*)(uintptr_t)(A & ~3u);
#pragma unroll
      for (int j = 0; j <= NP; ++j) Wd[u][j] = src[j];
      sh[u] = A & 2u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      uint32_t P[NP];
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const uint32_t c = __builtin_amdgcn_alignbyte(Wd[u][j + 1], Wd[u][j], sh[u]);
        P[j] = (((c & 0x7FFF7FFFu) | 0x80008000u) - ((c >> 15) & 0x00010001u)) ^ 0x80008000u;
      }
      const uint32_t O = 2u * (uint32_t)(q[u] * (W * W) + y[u] * W);
      unsigned char* d = dst + O;
      if (dalign == ((O & 2u) == 0)) {  // parity of the absolute address (dst may be 2 mod 4)
#pragma unroll
        for (int j = 0; j + 1 < NP; ++j) *(uint32_t*)(d + 4 * j) = P[j];
        *(uint16_t*)(d + 4 * (NP - 1)) = (uint16_t)P[NP - 1];
      } else {
        *(uint16_t*)d = (uint16_t)P[0];
#pragma unroll
        for (int j = 0; j + 1 < NP; ++j)
          *(uint32_t*)(d + 2 + 4 * j) = __builtin_amdgcn_alignbyte(P[j + 1], P[j], 2);
      }
    }
  }
}

// obs_window_occ of u16 cells, odd window W <= 7, written as 16-byte stores: thread t
// owns the 8 consecutive window rows 8t .. 8t + 7 of the block's record run (rows of
// W int16: 8 rows = 16 W bytes = W whole 16-byte chunks, aligned when the run is).  Each
// row is read once from the LDS map ((2W + 5) / 4 dwords realigned with v_alignbyte,
// occ = count - obstacle two cells at a time as in write_occ16_rows), rows 2k and
// 2k + 1 are spliced into W dwords (the odd row starts at a half dword: one v_perm and
// alignbyte shifts), and the thread stores W dwordx4 -- against 3 stores (2 dwords +
// one u16) per 10-byte row.  Returns the number of rows it covered (8 per whole group);
// the caller writes the rest with write_occ16_rows.
template <int W>
__device__ int write_occ16_groups(const Geo& g, const unsigned char* lds, const int* newc_blk,
                                  unsigned char* dst, int nseg, int tid, int nt) {
  constexpr int NP = (W + 1) / 2;       // dwords of one row's occ values (the last half used)
  constexpr int NR = (2 * W + 5) / 4;   // LDS dwords covering a row at either alignment
  constexpr int h = W / 2;
  typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  if ((((uintptr_t)dst) & 15u) != 0) return 0;
  const int ngrp = nseg >> 3;
  const int pitch = g.pitch;
  const bool one_env = g.EPB == 1;
  const uint32_t lbase = lds_addr(lds + g.off_map);
  for (int grp = tid; grp < ngrp; grp += nt) {
    const int sg0 = grp << 3;
    int q = fastdiv(sg0, g.m_w);
    int y = sg0 - q * W;
    uint32_t out[4 * W];
#pragma unroll
    for (int pr = 0; pr < 4; ++pr) {
      uint32_t P[2][NP];
#pragma unroll
      for (int j = 0; j < 2; ++j) {  // rows 2 pr + j
        const int slot = one_env ? 0 : fastdiv(q, g.m_N);
        const int e0 = newc_blk[q] + (y - h) * pitch - h;  // first cell of the row
        const uint32_t A = lbase + (uint32_t)(slot * g.map_env_bytes) + 2u * (uint32_t)e0;
        lds_cu32* src = (lds_cu32*)(uintptr_t)(A & ~3u);
        uint32_t Wd[NR + 1];
#pragma unroll
        for (int k = 0; k < NR; ++k) Wd[k] = src[k];
        Wd[NR] = 0u;
        const uint32_t sh = A & 2u;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          const uint32_t c = __builtin_amdgcn_alignbyte(Wd[k + 1], Wd[k], sh);
          P[j][k] = (((c & 0x7FFF7FFFu) | 0x80008000u) - ((c >> 15) & 0x00010001u)) ^ 0x80008000u;
        }
        if (++y == W) {
          y = 0;
          ++q;
        }
      }
      // the pair's W dwords: row 2 pr's NP - 1 full dwords, its last value with the odd
      // row's first, then the odd row's values 1 .. W - 1 shifted down by one u16
      uint32_t* o = out + pr * W;
#pragma unroll
      for (int k = 0; k + 1 < NP; ++k) o[k] = P[0][k];
      o[NP - 1] = __builtin_amdgcn_perm(P[1][0], P[0][NP - 1], 0x05040100u);
#pragma unroll
      for (int k = 0; k + 1 < NP; ++k) o[NP + k] = __builtin_amdgcn_alignbyte(P[1][k + 1], P[1][k], 2);
    }
    u32x4* d = (u32x4*)(dst + 16u * (uint32_t)W * (uint32_t)grp);
#pragma unroll
    for (int k = 0; k < W; ++k) d[k] = u32x4{out[4 * k], out[4 * k + 1], out[4 * k + 2], out[4 * k + 3]};
  }
  return ngrp << 3;
}

// ---------------------------------------------------------------------------
// The step kernel: T fused steps (T = 1 for mapfx_step; do_step = 0 observes).
// FEAT: bit 0 PRIMAL outputs (obs_primal / primal_vec), bit 1 obs_full; the
// window / avail / reward path alone (FEAT 0) keeps its register budget <= 128
// VGPRs, i.e. 4 blocks of 256 threads per CU.
// ---------------------------------------------------------------------------
#ifdef MAPFX_STAMPS
// Diagnostic build only (never the shipped library): per-segment s_memtime stamps
// of block 0 / lane 0, read back with mapfx_debug_stamps().
__device__ unsigned long long g_stamps[256 * 8];
#define STAMP(k)                                                                  \
  do {                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                            \
    unsigned long long t_;                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");  \
    __builtin_amdgcn_sched_barrier(0);                                            \
    if (blockIdx.x == 0 && threadIdx.x == 0 && s < 256) g_stamps[s * 8 + (k)] = t_; \
  } while (0)
// prologue / epilogue stamps of block 0 / lane 0 (row 255 of g_stamps)
#define PSTAMP(k)                                                                 \
  do {                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                            \
    unsigned long long t_;                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");  \
    __builtin_amdgcn_sched_barrier(0);                                            \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[255 * 8 + (k)] = t_;       \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#define PSTAMP(k) \
  do {            \
  } while (0)
#endif

constexpr int FEAT_PRIM = 1, FEAT_FULL = 2;
// FEAT_RUN (rollouts): exactly the runner output set (reward, term, node, edge, avail,
// traj_pos / traj_done / traj_t, a window; no reward_f32 / full / PRIMAL), so the
// per-output tests are compile-time
constexpr int FEAT_RUN = 4;

// The fp64 reward of one agent from its reward code (deferred fold): bit 0 counted
// (not done before the step), bit 1 env collision, bit 2 node collision, bits 3.. the
// edge-collision count -- the op order of the per-step computation below (:94-130).
__device__ inline double code_reward(const Geo& g, uint32_t c) {
  double rr = 0.0;
  if (c & 1u) {
    if (c & 2u) rr = rr + g.collide_rew;
    rr = rr + g.step_rew;
  }
  rr = rr + g.collide_rew * (double)((c >> 2) & 1u);
  rr = rr + g.collide_rew * (double)(c >> 3);
  return rr;
}
template <typename CellT, int APL, bool ROLL, int FEAT>
__device__ __forceinline__ void step_body(const Geo& g, const Args& a) {
  using CT = CellTraits<CellT>;
  constexpr bool RUNF = (FEAT & FEAT_RUN) != 0;  // exact runner output set (rollouts)
  extern __shared__ __align__(16) unsigned char lds[];
  const int tid = threadIdx.x;
  const int slot = tid >> g.lshift;
  const int lane = tid & (g.L - 1);
  const int env0 = blockIdx.x * g.EPB;
  const int env = env0 + slot;
  const bool env_ok = env < g.E;
  const int N = g.N;

  uint32_t* map32 = (uint32_t*)(lds + g.off_map + slot * g.map_env_bytes);
  CellT* map = (CellT*)map32;
  uint32_t* bitsL = (uint32_t*)(lds + g.off_bits + slot * g.bits_env_bytes);
  int* oldc = (int*)(lds + g.off_oldc) + slot * N;
  int* newc = (int*)(lds + g.off_newc) + slot * N;
  int* rcs = (int*)(lds + g.off_rc) + slot * N;
  int* gls = (int*)(lds + g.off_goal) + slot * N;
  double* rew = (double*)(lds + g.off_rew) + slot * N;  // aliases bitsL (used after the build)
  // [slot * 4 + {alldone, bad}]: two slots by step parity
  int* flag = (int*)(lds + g.off_flag) + slot * 12;
  // Deferred fold (rollouts, one env per block): every step stores a u16 reward CODE
  // per agent in a ring of FR rows (aliasing rew / the bitmap); every FR-th step (and
  // the last) lanes 0..FR-1 of wave 0 fold one row each -- the same agent-order chain
  // of fp64 adds per step, FR steps' chains side by side -- so the other steps carry no
  // fold and wave 0 writes window records with the others.
  const int FR = (ROLL && (RUNF || a.do_step)) ? g.fold_R : 0;
  uint16_t* codes = (uint16_t*)(lds + g.off_rew);
  double* ctab = (double*)(lds + g.off_ctab);  // code_reward of the codes < 32
  int* bigrow = (int*)(ctab + 32);              // ring row holds a code >= 32 (edge >= 4)

  // ---- per-lane agent state (registers) ----
  int r[APL], c[APL], gr[APL], gc[APL], st[APL];
  bool dn[APL], has[APL];
#pragma unroll
  for (int k = 0; k < APL; ++k) {
    const int ag = lane + k * g.L;
    has[k] = env_ok && ag < N;
    r[k] = c[k] = gr[k] = gc[k] = st[k] = 0;
    dn[k] = false;
    if (has[k]) {
      const long long i = (long long)env * N + ag;
      const int2 p = ((const int2*)a.pos)[i];
      const int2 q = ((const int2*)a.goal)[i];
      r[k] = p.x;
      c[k] = p.y;
      gr[k] = q.x;
      gc[k] = q.y;
      dn[k] = a.done[i] != 0;
      if (a.steps) st[k] = a.steps[i];
      if constexpr ((FEAT & FEAT_PRIM) != 0) gls[ag] = (q.x << 16) | (q.y & 0xFFFF);
    }
  }
  int tcur = env_ok ? a.t[env] : 0;

  const int T = ROLL ? a.T : 1;
  // actions are loaded one step ahead: step s + 1's load is issued before step s's
  // stores, so waiting for it never waits for them (vmcnt counts both, in order)
  const bool read_act = (RUNF || a.do_step) && !a.use_rng;
  int act_nx[APL];
#pragma unroll
  for (int k = 0; k < APL; ++k)
    act_nx[k] = (has[k] && read_act)
                    ? load_action(a.actions, a.act_dtype, (long long)env * N + lane + k * g.L) : 4;
  // ---- stage the bitmap, build the padded map, add the agents ----
  if (env_ok) {
    const uint32_t* src =
        (const uint32_t*)(a.bits + (g.map_shared ? 0 : (long long)env * g.map_stride));
    for (int w = lane; w < g.bits_words; w += g.L) bitsL[w] = src[w];
  }
  for (int i = lane; i < 12; i += g.L) flag[i] = (i & 3) == 0 ? 1 : 0;  // alldone = 1, bad = 0
  if (FR && tid < 32) ctab[tid] = code_reward(g, (uint32_t)tid);
  if (FR && tid < FR) bigrow[tid] = 0;
  __syncthreads();
  fill_map<CellT>(g, map32, bitsL, lane);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < APL; ++k) {
    if (has[k]) {
      const int cell = (r[k] + g.P) * g.pitch + c[k] + g.pl;
      atomicAdd(&map32[cell >> CT::PER_WORD_SHIFT], CT::inc(cell));
    }
  }
  __syncthreads();

  const int wlen = g.wlen;
  const int es = (int)sizeof(CellT);  // obs element size == cell size
  const long long Elong = g.E;

  for (int s = 0; s < T; ++s) {
    int* fl = flag + (s & 1) * 4;
    int act_in[APL];
#pragma unroll
    for (int k = 0; k < APL; ++k) act_in[k] = act_nx[k];
    if (ROLL && read_act && s + 1 < T) {
#pragma unroll
      for (int k = 0; k < APL; ++k)
        if (has[k])
          act_nx[k] = load_action(a.actions, a.act_dtype,
                                  ((long long)(s + 1) * Elong + env) * N + lane + k * g.L);
    }
    STAMP(0);
    // ================= P0: move decision on the PRE-step map =================
    int oc[APL], nc[APL], act[APL], pre[APL];
    bool moved[APL], envc[APL];
#pragma unroll
    for (int k = 0; k < APL; ++k) {
      const int ag = lane + k * g.L;
      oc[k] = (r[k] + g.P) * g.pitch + c[k] + g.pl;
      nc[k] = oc[k];
      moved[k] = envc[k] = false;
      pre[k] = 0;
      act[k] = 4;
      if (has[k] && (RUNF || a.do_step)) {
        int av;
        if (a.use_rng)
          av = gen_action(a.seed, g.env_offset + env, a.t0 + s, ag);
        else
          av = act_in[k];
        if (av < 0 || av > 4) {
          atomicOr(&fl[1], 1);
          av = 4;
        }
        act[k] = av;
        if (!dn[k] && av != 4) {  // __agent_step :319-342
          const int cand =
              oc[k] + (av == 0 ? -g.pitch : (av == 1 ? g.pitch : (av == 2 ? -1 : 1)));
          const uint32_t v = map[cand];
          const bool blocked = v == CT::OE;
          const int pv = (int)(v & CT::CNT);
          if (blocked) {
            envc[k] = true;       // out of bounds or free-standing obstacle
          } else {
            nc[k] = cand;
            moved[k] = true;
            pre[k] = pv;
          }
        }
        oldc[ag] = oc[k];
        newc[ag] = nc[k];
      }
    }
    lds_barrier();  // B1: every pre-step map read is done (and the bad flag)
    STAMP(1);
    // ================= P1: move the agent counts =================
    const bool skip = (fl[1] != 0) || !(RUNF || a.do_step);
#pragma unroll
    for (int k = 0; k < APL; ++k) {
      if (!has[k]) continue;
      const int ag = lane + k * g.L;
      if (skip) {
        nc[k] = oc[k];
        moved[k] = envc[k] = false;
        newc[ag] = oc[k];
      } else if (moved[k]) {
        atomicSub(&map32[oc[k] >> CT::PER_WORD_SHIFT], CT::inc(oc[k]));
        atomicAdd(&map32[nc[k] >> CT::PER_WORD_SHIFT], CT::inc(nc[k]));
        r[k] += act_dr(act[k]);
        c[k] += act_dc(act[k]);
      }
      if constexpr ((FEAT & FEAT_PRIM) != 0) rcs[ag] = (r[k] << 16) | (c[k] & 0xFFFF);
    }
    if ((RUNF || a.do_step) && !skip && env_ok) ++tcur;
    if (lane == 0) {  // the next step's flags: every read of them (step s - 1's) precedes B1
      int* nf = flag + ((s + 1) & 1) * 4;
      nf[0] = 1;
      nf[1] = 0;
    }
    lds_barrier();  // B2: post-step map complete
    STAMP(2);
    // ================= P2: collisions, rewards, avail, observations =================
    const long long slotE = ROLL ? (long long)s * Elong : 0;  // trajectory slot offset (envs)
    // edge collisions (:364-383): i moved into a cell that had pre-step occupants;
    // count the agents j that moved from that cell into i's old cell.  With whole
    // waves per env (L >= 64) the wave scans the env's agents together for each
    // such i in turn (N/64 reads per lane instead of N by one lane); every lane
    // of the wave takes part, agent or not.
    int edgek[APL];
#pragma unroll
    for (int k = 0; k < APL; ++k) edgek[k] = 0;
    if (g.L >= 64 && (RUNF || a.do_step) && !skip) {
      // the env's (old, new) cells, 64 agents per chunk, read once by a wave that
      // has such an i; each i's count is then one ballot popcount per chunk
      constexpr int NCH = APL * 4;  // N <= APL * 256
      const int l64 = tid & 63;
      const int nch = (N + 63) >> 6;
      uint64_t mk[APL];
      bool any = false;
#pragma unroll
      for (int k = 0; k < APL; ++k) {
        mk[k] = __ballot(has[k] && moved[k] && pre[k] > 0);
        any |= mk[k] != 0;
      }
      if (any) {
        int jo[NCH], jn[NCH];
#pragma unroll
        for (int q = 0; q < NCH; ++q) {
          const int j = q * 64 + l64;
          const bool ok = q < nch && j < N;
          jo[q] = ok ? oldc[j] : -1;
          jn[q] = ok ? newc[j] : -1;
        }
#pragma unroll
        for (int k = 0; k < APL; ++k) {
          uint64_t m = mk[k];
          while (m) {
            const int src = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            // src is wave-uniform (a ballot bit): v_readlane, not two ds_bpermute round trips
            const int tn = __builtin_amdgcn_readlane(nc[k], src);
            const int to = __builtin_amdgcn_readlane(oc[k], src);
            int cnt = 0;
#pragma unroll
            for (int q = 0; q < NCH; ++q)
              if (q < nch) cnt += __popcll(__ballot((jo[q] == tn) & (jn[q] == to)));
            if (l64 == src) edgek[k] = cnt;
          }
        }
      }
    }
    STAMP(3);
#pragma unroll
    for (int k = 0; k < APL; ++k) {
      if (!has[k]) continue;
      const int ag = lane + k * g.L;
      const long long ai = (slotE + env) * N + ag;  // output agent index
      int node = 0, edge = edgek[k];
      if ((RUNF || a.do_step) && !skip) {
        node = ((uint32_t)map[nc[k]] & CT::CNT) > 1u ? 1 : 0;  // :344-362
        if (g.L < 64 && moved[k] && pre[k] > 0) {
          for (int j = 0; j < N; ++j)
            edge += (oldc[j] == nc[k]) & (newc[j] == oc[k]);
        }
        if (FR) {  // the reward's code (code_reward); folded every FR steps
          codes[(s & (FR - 1)) * (g.code_pitch >> 1) + ag] =
              (uint16_t)((dn[k] ? 0u : 1u) | (envc[k] ? 2u : 0u) | ((uint32_t)node << 2) |
                         ((uint32_t)edge << 3));
          if (edge >= 4) bigrow[s & (FR - 1)] = 1;  // the fold takes this row's slow path
          if (!dn[k]) ++st[k];
        } else {
          double rr = 0.0;  // :94-130, exact fp64 op order
          if (!dn[k]) {
            if (envc[k]) rr = rr + g.collide_rew;
            rr = rr + g.step_rew;
            ++st[k];
          }
          rr = rr + g.collide_rew * (double)node;
          rr = rr + g.collide_rew * (double)edge;
          rew[ag] = rr;
        }
        if (r[k] == gr[k] && c[k] == gc[k]) dn[k] = true;  // :112-114
        if (tcur >= g.limit) dn[k] = true;                   // :116-117
      } else if (FR) {
        codes[(s & (FR - 1)) * (g.code_pitch >> 1) + ag] = 0;  // code_reward(0) = 0.0
      } else if ((RUNF || a.do_step)) {
        rew[ag] = 0.0;
      }
      if (!dn[k]) fl[0] = 0;  // every writer stores the same 0: no atomic needed
      if ((RUNF || a.do_step)) {
        if (RUNF || a.node) a.node[ai] = (uint8_t)node;
        if (RUNF || a.edge) {  // u8 while N <= 256 (edge <= N - 1), else u16 (mapfx_edge_elem_size)
          if (N <= 256) a.edge[ai] = (uint8_t)edge;
          else ((uint16_t*)a.edge)[ai] = (uint16_t)edge;
        }
      }
      if (RUNF || a.traj_pos) ((int2*)a.traj_pos)[ai] = make_int2(r[k], c[k]);
      if (RUNF || a.traj_done) a.traj_done[ai] = dn[k] ? 1 : 0;
      if (RUNF || a.avail) {  // :203-224 on the post-step map
        const int cc = nc[k];
        uint32_t m = 16u;
        m |= ((uint32_t)map[cc - g.pitch] != CT::OE) ? 1u : 0u;
        m |= ((uint32_t)map[cc + g.pitch] != CT::OE) ? 2u : 0u;
        m |= ((uint32_t)map[cc - 1] != CT::OE) ? 4u : 0u;
        m |= ((uint32_t)map[cc + 1] != CT::OE) ? 8u : 0u;
        a.avail[ai] = (uint8_t)m;
      }
    }
    // ---- the env's lane-0 tail: the fp64 fold of the rewards, term, t, next flags ----
    auto lane0_tail = [&](bool alldone) {
      if (!env_ok || lane != 0) return;
      if ((RUNF || a.do_step)) {
        if (fl[1] && a.err) atomicCAS(a.err, 0, env + 1);
        double R = 0.0;  // `sum(rewards)`: naive left fold in agent order (:141)
        if (!FR) {
          // the adds are one dependent chain; a ring of 8 LDS reads stays in flight
          // ahead of it (the read of reward j + 8 is issued when reward j is added)
          int j = 0;
          if (N >= 8) {
            double ring[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) ring[i] = rew[i];
            const int n8 = N & ~7;
#pragma nounroll
            for (j = 0; j < n8 - 8; j += 8) {
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                R = R + ring[i];
                ring[i] = rew[j + 8 + i];
                __builtin_amdgcn_sched_barrier(0);  // keep each read where it is issued
              }
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) R = R + ring[i];
            j = n8;
          }
          for (; j < N; ++j) R = R + rew[j];
        }
        if (!FR) {
          if (RUNF || a.reward) a.reward[slotE + env] = R;
          if (!RUNF && a.reward_f32) a.reward_f32[slotE + env] = (float)R;
        }
      }
      if (RUNF || a.term) a.term[slotE + env] = alldone ? 1 : 0;
      if (RUNF || a.traj_t) a.traj_t[slotE + env] = tcur;
    };
    STAMP(4);
    // ---- deferred fold: lane i < FR of wave 0 folds the code row of step s0 + i ----
    const bool fstep = FR && (((s & (FR - 1)) == FR - 1) || s + 1 == T);
    auto fold_ring = [&]() {
      const int s0 = s & ~(FR - 1);
      if (!env_ok || tid > s - s0) return;
      // the fold is one dependent chain of N fp64 adds that competes for issue with the
      // other blocks' window writers on its SIMD: it goes first while it runs
      if (MAPFX_FOLD_PRIO) __builtin_amdgcn_s_setprio(MAPFX_FOLD_PRIO);
      const uint16_t* cs = codes + tid * (g.code_pitch >> 1);
      auto val = [&](uint32_t c) { return c < 32u ? ctab[c] : code_reward(g, c); };
      double R = 0.0;  // `sum(rewards)`: naive left fold in agent order (:141)
      // Rows with only codes < 32 (edge <= 3): groups of 8 codes, software-pipelined
      // over two register sets -- while group q is added, group q + 1's table reads and
      // group q + 2's code read are in flight -- so the adds wait on nothing but the
      // chain.  A row with a larger edge count takes the plain loop below.
      const int ng = bigrow[tid] ? 0 : N >> 3;
      int j = 0;
      if (ng > 0) {
        const uint4* cs4 = (const uint4*)cs;
        auto tab = [&](const uint4& v, double (&t)[8]) {
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] = ctab[(w[i >> 1] >> (16 * (i & 1))) & 31u];
        };
        double tA[8], tB[8];
        uint4 cA = cs4[0], cB = cs4[ng > 1 ? 1 : 0];
        tab(cA, tA);
        for (int q = 0; q < ng; q += 2) {
          if (q + 1 < ng) {
            tab(cB, tB);
            if (q + 2 < ng) cA = cs4[q + 2];
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) R = R + tA[i];
          if (q + 1 < ng) {
            if (q + 2 < ng) {
              tab(cA, tA);
              if (q + 3 < ng) cB = cs4[q + 3];
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) R = R + tB[i];
          }
        }
        j = ng << 3;
      }
      bigrow[tid] = 0;
      for (; j < N; ++j) R = R + val(cs[j]);
      const long long ri = (long long)(s0 + tid) * Elong + env;
      if (RUNF || a.reward) a.reward[ri] = R;
      if (!RUNF && a.reward_f32) a.reward_f32[ri] = (float)R;
      if (MAPFX_FOLD_PRIO) __builtin_amdgcn_s_setprio(0);
    };
    // One env per block over four waves (N > 128): wave 0 runs the tail (the fold is
    // one dependent chain of N adds) while waves 1-3 write the window records; with
    // the deferred fold, wave 0 writes records too except on the fold steps.
    // Without a fold in this step the tail waits until after B3 (no B2b).
    const bool ovl = g.L == 256 && (a.obs_window || a.obs_window_occ);
    const bool tail_early = ovl && (!FR || fstep);
    if (tail_early) {
      lds_barrier();  // B2b: rew[] / codes and the alldone flag complete
      if (tid < 64) {
        lane0_tail(fl[0] != 0);
        if (fstep) fold_ring();
      }
    }
    const int wt0 = tail_early ? 64 : 0;  // first writer thread
    STAMP(5);
    if ((a.obs_window || a.obs_window_occ) && tid >= wt0) {  // :323-342
      const int wtid = tid - wt0, wnt = g.BT - wt0;
      const int nenv = min(g.EPB, g.E - env0);
      const long long rec0 = (slotE + env0) * (long long)N;  // first record of the block
      const int* newc_blk = (const int*)(lds + g.off_newc);
      if (a.obs_window)
        write_windows<CellT, false>(g, lds, newc_blk,
                                    (unsigned char*)a.obs_window + rec0 * wlen * es,
                                    nenv * N * wlen, wtid, wnt);
      if (a.obs_window_occ) {
        unsigned char* dst = (unsigned char*)a.obs_window_occ + rec0 * (wlen / 2) * es;
        bool done_occ = false;
        if constexpr (sizeof(CellT) == 2) {
          const int nseg = nenv * N * g.window;
          done_occ = true;
          // whole 8-row groups as 16-byte stores, the remaining rows one by one
          if (g.window == 5) {
            const int rows = write_occ16_groups<5>(g, lds, newc_blk, dst, nseg, wtid, wnt);
            write_occ16_rows<5>(g, lds, newc_blk, dst, nseg, wtid, wnt, rows);
          } else if (g.window == 3) {
            const int rows = write_occ16_groups<3>(g, lds, newc_blk, dst, nseg, wtid, wnt);
            write_occ16_rows<3>(g, lds, newc_blk, dst, nseg, wtid, wnt, rows);
          } else if (g.window == 7) {
            const int rows = write_occ16_groups<7>(g, lds, newc_blk, dst, nseg, wtid, wnt);
            write_occ16_rows<7>(g, lds, newc_blk, dst, nseg, wtid, wnt, rows);
          } else {
            done_occ = false;
          }
        }
        if (!done_occ)
          write_windows<CellT, true>(g, lds, newc_blk, dst, nenv * N * (wlen / 2), wtid, wnt);
      }
    }
    if ((FEAT & FEAT_PRIM) && (a.obs_primal || a.primal_vec)) {  // rcs[] (P1) visible since B2
#pragma unroll
      for (int k = 0; k < APL; ++k) {
        if (!has[k]) continue;
        const int ag = lane + k * g.L;
        const long long ai = (slotE + env) * N + ag;
        const int S = g.psize, h = S >> 1;
        const int tr = r[k] - h, tc = c[k] - h;
        if (a.obs_primal) {
          // goals channel: goals of visible other agents clamped into the window
          uint64_t gm0 = 0, gm1 = 0;
          for (int j = 0; j < N; ++j) {
            if (j == ag) continue;
            const int rc = rcs[j];
            const int jr = rc >> 16, jc = (int)(int16_t)(rc & 0xFFFF);
            if (jr < tr || jr >= tr + S || jc < tc || jc >= tc + S) continue;
            const int gg = gls[j];
            int xr = gg >> 16, xc = (int)(int16_t)(gg & 0xFFFF);
            xr = max(tr, min(tr + S - 1, xr));
            xc = max(tc, min(tc + S - 1, xc));
            const int q = (xr - tr) * S + (xc - tc);
            if (q < 64) gm0 |= 1ull << q; else gm1 |= 1ull << (q - 64);
          }
          uint8_t* out = a.obs_primal + ai * 4 * S * S;
          const int base = (tr + g.P) * g.pitch + tc + g.pl;
          for (int y = 0; y < S; ++y) {
            for (int x = 0; x < S; ++x) {
              const int q = y * S + x;
              const uint32_t v = map[base + y * g.pitch + x];
              out[q] = (v & CT::CNT) ? 1 : 0;                                  // poss
              out[S * S + q] = (tr + y == gr[k] && tc + x == gc[k]) ? 1 : 0;   // goal
              out[2 * S * S + q] =
                  (uint8_t)(((q < 64 ? gm0 >> q : gm1 >> (q - 64))) & 1ull);   // goals
              out[3 * S * S + q] = (v == CT::OE) ? 1 : 0;                      // obs
            }
          }
        }
        if (a.primal_vec) {  // mapf_primal.py:380-386; mag via host libm pow LUT
          const int dx = gr[k] - r[k], dy = gc[k] - c[k];
          const double mag = a.pow_lut[dx * dx + dy * dy];
          double vx = (double)dx, vy = (double)dy;
          if (mag != 0.0) {
            vx = vx / mag;
            vy = vy / mag;
          }
          double* o = a.primal_vec + ai * 3;
          o[0] = vx;
          o[1] = vy;
          o[2] = mag;
        }
      }
    }
    if ((FEAT & FEAT_FULL) && a.obs_full && env_ok) {  // :143-192: row-major occ = count - flag
      const long long HW = (long long)g.H * g.W;
      unsigned char* outb = (unsigned char*)a.obs_full + (slotE + env) * HW * es;
      if (es == 1 && (g.W & 3) == 0) {
        const int wpr_out = g.W >> 2;
        const int nwords = g.H * wpr_out;
        for (int i = lane; i < nwords; i += g.L) {
          const int rr_ = fastdiv(i, g.m_W4);
          const int cw = i - rr_ * wpr_out;
          const uint32_t v = map32[((rr_ + g.P) * g.pitch + g.pl) / 4 + cw];
          const uint32_t f = (v >> 7) & 0x01010101u;
          const uint32_t o = (((v & 0x7F7F7F7Fu) | 0x80808080u) - f) ^ 0x80808080u;
          ((uint32_t*)outb)[i] = o;
        }
      } else {
        for (int i = lane; i < (int)HW; i += g.L) {
          const int rr_ = fastdiv(i, g.m_W);
          const int cc_ = i - rr_ * g.W;
          const uint32_t v = map[(rr_ + g.P) * g.pitch + cc_ + g.pl];
          const int occ = (int)(v & CT::CNT) - ((v & CT::OE) ? 1 : 0);
          if (es == 1)
            ((int8_t*)outb)[i] = (int8_t)occ;
          else
            ((int16_t*)outb)[i] = (int16_t)occ;
        }
      }
    }
    STAMP(6);
    lds_barrier();  // B3: rew[] and flags complete
    STAMP(7);
    // ================= P3: fold, term, staging copy-out, autoreset =================
    const bool alldone = fl[0] != 0;
    if (!tail_early) {
      lane0_tail(alldone);
      if (fstep && tid < 64) fold_ring();
    }
    // optional autoreset of envs whose agents are all done
#pragma unroll
    for (int k = 0; k < APL; ++k) {
      if (!has[k]) continue;
      const int ag = lane + k * g.L;
      const long long i = (long long)env * N + ag;
      if (a.autoreset && alldone && (RUNF || a.do_step)) {
        const int2 p = ((const int2*)a.init_pos)[i];
        const int ocell = (r[k] + g.P) * g.pitch + c[k] + g.pl;
        const int ncell = (p.x + g.P) * g.pitch + p.y + g.pl;
        atomicSub(&map32[ocell >> CT::PER_WORD_SHIFT], CT::inc(ocell));
        atomicAdd(&map32[ncell >> CT::PER_WORD_SHIFT], CT::inc(ncell));
        r[k] = p.x;
        c[k] = p.y;
        dn[k] = false;
        st[k] = 0;
      }
    }
    if (a.autoreset && alldone && (RUNF || a.do_step)) tcur = 0;
    // B4: the autoreset's map atomics before the next step's reads; without autoreset
    // every hand-off of this step is already ordered by B3 (the tail and the fold read
    // nothing the next step writes before its B1)
    if (ROLL && s + 1 < T && a.autoreset) lds_barrier();
  }

  // ---- write back the env state ----
#pragma unroll
  for (int k = 0; k < APL; ++k) {
    if (!has[k]) continue;
    const int ag = lane + k * g.L;
    const long long i = (long long)env * N + ag;
    ((int2*)a.pos)[i] = make_int2(r[k], c[k]);
    a.done[i] = dn[k] ? 1 : 0;
    if (a.steps) a.steps[i] = st[k];
  }
  if (env_ok && lane == 0) a.t[env] = tcur;
}


// ===========================================================================
// Wave-local fast path (N <= 64).  Every env lives inside ONE wavefront
// (L = pow2ceil(N) lanes, 64/L envs per wave), so a step needs no workgroup
// barrier at all: LDS instructions of a wave execute in order, and cross-lane
// values move with ds_bpermute (__shfl) or wave ballots.  Blocks are one wave;
// waves never wait on each other.  Per step, per agent lane:
//   1 LDS read (candidate cell, PRE-step map) -> 2 LDS atomics (move the count)
//   -> WIN row reads of the POST-step map, turned by SWAR into the window's
//   obstacle / agents planes; node collision and avail fall out of the same
//   rows -> who-map lookup + bpermute only for agents that moved into a
//   pre-occupied cell (edge collisions) -> the 2*WIN*WIN-byte record is packed
//   in registers and staged as u16; one lane per env folds the fp64 rewards in
//   agent order; the wave writes the staged records with 16-byte stores.
// Actions for step s+1 are loaded while step s runs.  All offsets are 32-bit.
// ===========================================================================

// Wave-path cell format: one byte per padded cell = (obstacle << 7) | c with
// c = count + 1 - obstacle (7 bits), so
//   c == 0  <=> obstacle with no agent on it (and every border cell): the move /
//               avail / window "obstacle" test of the reference (:278-280, :209-222,
//               marl_partial.py:335-337) is a zero test of the low 7 bits;
//   agents plane = max(count - obstacle, 0) = c - (c != 0);  occ = c - 1;
//   count = c - 1 + obstacle (bit 7: the static obstacle flag rides with the cell);
// and adding / removing an agent is +-1 with no borrow out of the 7 bits (c >= 1
// under an agent).  The per-cell `dep` byte (move direction of the cell's occupant
// in the current step) is written by every occupant before it is read and needs no
// initialisation.
// Fallback builder (rows wider than build_map_rows_fast handles): one map row per
// lane at a time, border rows / pad words constant, an interior word one 4-bit
// window of the bitmap row (staged in LDS) spread over four cells.
__device__ __forceinline__ uint32_t cells_of_nibble(uint32_t nib) {  // 4 obstacle bits -> 4 cells
  const uint32_t f = (nib * 0x00204081u) & 0x01010101u;
  return (f << 7) | (f ^ 0x01010101u);
}
__device__ inline void build_map_rows_c(const Geo& g, uint32_t* map32, const uint32_t* bitsL, int lane,
                                        int nl) {
  const int wpr = g.wpr, plw = g.pl >> 2;
  const int iw = (g.W + 3) >> 2;  // interior words (the last one may hold border cells)
  const uint32_t last_or = (g.W & 3) ? ((0xFu << (g.W & 3)) & 0xFu) : 0u;
  for (int pr = lane; pr < g.rows; pr += nl) {
    uint32_t* row = map32 + pr * wpr;
    const int rr = pr - g.P;
    if (rr < 0 || rr >= g.H) {
      for (int w = 0; w < wpr; ++w) row[w] = 0x80808080u;
      continue;
    }
    for (int w = 0; w < plw; ++w) row[w] = 0x80808080u;
    // 32 cells (8 map words) per bitmap read pair: the reads of a chunk are waited
    // for once, not once per word
    for (int k0 = 0; k0 < iw; k0 += 8) {
      const int p = rr * g.W + 4 * k0;
      const uint32_t x = __builtin_amdgcn_alignbit(bitsL[(p >> 5) + 1], bitsL[p >> 5], p & 31);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (k0 + j < iw) {
          uint32_t nib = (x >> (4 * j)) & 0xFu;
          if (k0 + j == iw - 1) nib |= last_or;
          row[plw + k0 + j] = cells_of_nibble(nib);
        }
      }
    }
    for (int w = plw + iw; w < wpr; ++w) row[w] = 0x80808080u;
  }
}

// Fast builder for padded rows of at most MAXW words (W <= 64, pitch % 8 == 0):
// each lane builds whole rows, branch-free, from the env's bitmap words read
// straight from global memory (L2 hits after the env's first lane -- no LDS
// staging, no fence), two cell words per ds_write_b64.  The padded row's
// obstacle bits (1 = obstacle, the border included) sit in lo (cells 0-63) / hi.
// The bitmap words of a lane's first RPF rows are loaded by fast_row_prefetch at
// kernel entry, so their latency overlaps the state loads.
template <int RPF>
__device__ __forceinline__ void fast_row_prefetch(const Geo& g, const uint32_t* src, int lane, int nl,
                                                  uint32_t (&pf)[RPF][3]) {
  const int last = g.bits_words - 1;
#pragma unroll
  for (int k = 0; k < RPF; ++k) {
    const int rr = min(max(lane + k * nl - g.P, 0), g.H - 1);  // clamped: always a valid address
    const int i0 = (rr * g.W) >> 5;
    pf[k][0] = src[i0];
    pf[k][1] = src[min(i0 + 1, last)];
    pf[k][2] = src[min(i0 + 2, last)];
  }
}
template <int MAXW, int RPF>
__device__ inline void build_map_rows_fast(const Geo& g, uint32_t* map32, const uint32_t* src, int lane,
                                           int nl, const uint32_t (&pf)[RPF][3], uint32_t* map32b = nullptr) {
  const int wpr = g.wpr, pl = g.pl, e = g.pl + g.W, last = g.bits_words - 1;
  const uint64_t wmask = g.W < 64 ? (1ull << g.W) - 1ull : ~0ull;
  // one padded row from its bitmap words w0..w2 (the words covering bits rr*W ..)
  const auto row = [&](int pr, uint32_t w0, uint32_t w1, uint32_t w2) {
    const int rr = pr - g.P;
    uint64_t lo = ~0ull;
    uint32_t hi = ~0u;
    if (rr >= 0 && rr < g.H) {
      const int sh = (rr * g.W) & 31;
      const uint64_t rb = ((((uint64_t)__builtin_amdgcn_alignbit(w2, w1, sh)) << 32) |
                           __builtin_amdgcn_alignbit(w1, w0, sh)) & wmask;
      lo = (rb << pl) | ((1ull << pl) - 1ull) | (e < 64 ? ~0ull << e : 0ull);  // 1 <= pl <= 32
      hi = (uint32_t)(rb >> (64 - pl)) | (e <= 64 ? ~0u : (e < 96 ? ~0u << (e - 64) : 0u));
    }
    uint2* row2 = (uint2*)(map32 + pr * wpr);
    uint2* row2b = map32b ? (uint2*)(map32b + pr * wpr) : nullptr;  // (the split's second count map)
#pragma unroll
    for (int j = 0; j < MAXW / 2; ++j) {
      if (2 * j < wpr) {
        const int w = 2 * j;  // cells 4w .. 4w+7 of the padded row
        const uint32_t n0 = w < 16 ? (uint32_t)(lo >> (4 * w)) : hi >> (4 * w - 64);
        const uint32_t n1 = w + 1 < 16 ? (uint32_t)(lo >> (4 * w + 4)) : hi >> (4 * w - 60);
        const uint2 cw = make_uint2(cells_of_nibble(n0 & 0xFu), cells_of_nibble(n1 & 0xFu));
        row2[j] = cw;
        if (row2b) row2b[j] = cw;
      }
    }
  };
#pragma unroll
  for (int k = 0; k < RPF; ++k) {
    const int pr = lane + k * nl;
    if (pr < g.rows) row(pr, pf[k][0], pf[k][1], pf[k][2]);
  }
  for (int pr = lane + RPF * nl; pr < g.rows; pr += nl) {
    const int i0 = (min(max(pr - g.P, 0), g.H - 1) * g.W) >> 5;
    row(pr, src[i0], src[min(i0 + 1, last)], src[min(i0 + 2, last)]);
  }
}

// Workgroups are dealt round-robin to the 8 XCDs (block b runs on XCD b % 8), each
// with its own L2.  Renumber them so that XCD x owns one contiguous run of env
// groups: neighbouring groups' small per-step outputs (node / edge / avail / done
// bytes, rewards) share 128-B lines, which then fill in one L2 instead of leaving
// two XCDs as partial-line writes.  Identity when the grid is not a multiple of 8.
__device__ __forceinline__ int xcd_block(int b, int nb) {
  if ((nb & 7) != 0) return b;
  return (b & 7) * (nb >> 3) + (b >> 3);
}

__device__ inline void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 4 cells of the c format (one u32) -> obstacle plane bytes (c == 0) and agents
// plane bytes (c - (c != 0)); c <= 127 so the +0x7F carry never leaves its byte.
__device__ inline void swar_window(uint32_t v, uint32_t& ob, uint32_t& ag) {
  const uint32_t c = v & 0x7F7F7F7Fu;                            // drop the obstacle flags
  const uint32_t nz = ((c + 0x7F7F7F7Fu) >> 7) & 0x01010101u;  // 1 where c >= 1
  ob = nz ^ 0x01010101u;
  ag = c - nz;
}

// OR a chunk of `bits` (<= 56) bits into a little-endian u64 bit stream at `pos`
// (all arguments compile-time after unrolling).
template <int NW>
__device__ __forceinline__ void put_bits(uint64_t (&w)[NW], int pos, int bits, uint64_t chunk) {
  const int wi = pos >> 6, sh = pos & 63;
  w[wi] |= chunk << sh;
  if (sh + bits > 64 && wi + 1 < NW) w[wi + 1] |= chunk >> (64 - sh);
}

// ---- window record packing ------------------------------------------------
// The record of one agent is 2*WIN*WIN bytes: obstacle plane rows then agents
// plane rows.  Row y of a plane lives in two registers: cols 0-3 (R[.. + y]) and
// cols 4-7 (R[.. + WIN + y]).  Register index of record byte b and its byte lane:
template <int WIN>
__host__ __device__ constexpr int rec_reg(int b) {
  const int plane = b / (WIN * WIN), y = (b % (WIN * WIN)) / WIN, x = (b % (WIN * WIN)) % WIN;
  if (WIN == 5 && x == 4) return plane * 2 * WIN + WIN + (y < 4 ? 0 : 1);  // packed column 4
  return plane * 2 * WIN + (x >= 4 ? WIN : 0) + y;
}
template <int WIN>
__host__ __device__ constexpr int rec_lane(int b) {
  const int y = (b % (WIN * WIN)) / WIN, x = (b % (WIN * WIN)) % WIN;
  if (WIN == 5 && x == 4) return y < 4 ? y : 0;
  return x & 3;
}
// Dword k of the record (bytes 4k..4k+3) as at most two v_perm_b32 of register pairs.
struct PermSpec {
  int ra, rb, rc, rd;  // perm(R[rb], R[ra], s1) | perm(R[rd], R[rc], s2); rc < 0: one perm
  uint32_t s1, s2;
};
template <int WIN>
__host__ __device__ constexpr PermSpec perm_spec(int k) {
  constexpr int REC = 2 * WIN * WIN;
  PermSpec sp{-1, -1, -1, -1, 0x0C0C0C0Cu, 0x0C0C0C0Cu};
  for (int j = 0; j < 4; ++j) {
    const int b = 4 * k + j;
    if (b >= REC) continue;
    const int r = rec_reg<WIN>(b), l = rec_lane<WIN>(b);
    const uint32_t clr = ~(0xFFu << (8 * j));
    if (sp.ra < 0 || sp.ra == r) {
      sp.ra = r;
      sp.s1 = (sp.s1 & clr) | ((uint32_t)l << (8 * j));
    } else if (sp.rb < 0 || sp.rb == r) {
      sp.rb = r;
      sp.s1 = (sp.s1 & clr) | ((uint32_t)(4 + l) << (8 * j));
    } else if (sp.rc < 0 || sp.rc == r) {
      sp.rc = r;
      sp.s2 = (sp.s2 & clr) | ((uint32_t)l << (8 * j));
    } else {
      sp.rd = r;
      sp.s2 = (sp.s2 & clr) | ((uint32_t)(4 + l) << (8 * j));
    }
  }
  return sp;
}

// Record word k (bytes 4k..4k+3) from the row registers (<= 2 v_perm_b32).
template <int WIN, int K>
__device__ __forceinline__ uint32_t rec_word(const uint32_t (&R)[4 * WIN]) {
  constexpr PermSpec sp = perm_spec<WIN>(K);
  uint32_t w = __builtin_amdgcn_perm(sp.rb >= 0 ? R[sp.rb >= 0 ? sp.rb : 0] : 0u, R[sp.ra], sp.s1);
  if constexpr (sp.rc >= 0)
    w |= __builtin_amdgcn_perm(sp.rd >= 0 ? R[sp.rd >= 0 ? sp.rd : 0] : 0u, R[sp.rc], sp.s2);
  return w;
}

template <int WIN, int... K>
__device__ __forceinline__ void rec_words(const uint32_t (&R)[4 * WIN], uint32_t* w,
                                          std::integer_sequence<int, K...>) {
  ((w[K] = rec_word<WIN, K>(R)), ...);
}

// Store at a 32-bit byte offset from a uniform base: global_store with saddr
// (every output offset of a launch is < 2^31, checked on the host).
template <typename T>
__device__ __forceinline__ void st_off(void* base, uint32_t off, T v) {
  *(T*)((unsigned char*)base + off) = v;
}

// One agent's 2*WIN*WIN-byte record straight to HBM.  Records are 2-byte aligned
// (2*WIN^2 = 2 mod 4): a record at 2 mod 4 is written as one u16 then dwords
// shifted by two bytes (one v_perm each), one at 0 mod 4 as dwords then one u16,
// so every store is naturally aligned and no byte of a neighbour's record is touched.
template <int WIN>
__device__ __forceinline__ void write_record(const uint32_t (&R)[4 * WIN], void* base, uint32_t off) {
  constexpr int REC = 2 * WIN * WIN;
  constexpr int NW = (REC + 3) / 4;
  constexpr int ND = (REC - 2) / 4;
  uint32_t w[NW];
  rec_words<WIN>(R, w, std::make_integer_sequence<int, NW>{});
  const bool odd = (off & 2) != 0;  // base is 256-byte aligned (torch allocations)
  const uint32_t sel = odd ? 0x05040302u : 0x03020100u;  // bytes 2..5 of {w[j+1], w[j]}
  // one 64-bit base per record: the 12 dwords then merge into dwordx4 stores
  unsigned char* d = (unsigned char*)base + (off + (odd ? 2u : 0u));
#pragma unroll
  for (int j = 0; j < ND; ++j) *(uint32_t*)(d + 4 * j) = __builtin_amdgcn_perm(w[j + 1], w[j], sel);
  st_off(base, off + (odd ? 0u : (uint32_t)(REC - 2)), (uint16_t)(odd ? w[0] : w[NW - 1]));
}


// Stage one agent's 2*WIN*WIN-byte window record in LDS.  Records are 2-byte
// aligned (2*WIN^2 = 2 mod 4 for odd WIN): a record at 2 mod 4 is written as one
// u16 then dwords shifted by two bytes, one at 0 mod 4 as dwords then one u16,
// so every store is naturally aligned (ds_write_b32 / ds_write2_b32, never the
// replayed misaligned forms) and no byte of a neighbour's record is touched.
// The wave then moves its staged block to HBM with coalesced 16-byte stores --
// 13x faster than the same bytes as scattered per-lane dword stores
// (tools/micro/stores.hip: 0.51 vs 6.4 us per 3.2 MB on MI355X).
template <int WIN>
__device__ __forceinline__ void stage_record(const uint32_t (&R)[4 * WIN], unsigned char* rec) {
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  typedef __attribute__((address_space(3))) uint16_t lds_u16;
  constexpr int REC = 2 * WIN * WIN;
  constexpr int NW = (REC + 3) / 4;
  constexpr int ND = (REC - 2) / 4;
  static_assert(REC % 4 == 2, "odd window sizes only");
  uint32_t w[NW];
  rec_words<WIN>(R, w, std::make_integer_sequence<int, NW>{});
  const uint32_t ra = lds_addr(rec);
  const bool odd = (ra & 2) != 0;
  lds_u32* d = (lds_u32*)(uintptr_t)(ra + (odd ? 2 : 0));
#pragma unroll
  for (int j = 0; j < ND; ++j) d[j] = odd ? __builtin_amdgcn_alignbyte(w[j + 1], w[j], 2) : w[j];
  *(lds_u16*)(uintptr_t)(ra + (odd ? 0 : REC - 2)) = (uint16_t)(odd ? w[0] : w[NW - 1]);
}

// One agent's window record registers R ([plane][cols 0-3 | cols 4-7][row]) from its
// raw post-step map rows: qx[y] = cells 0-3, qx[WIN + y] = cells 4-7, qx[2 WIN + y]
// = cells 8-11 of window row y, each starting `o` bytes into the first word.
template <int WIN>
__device__ __forceinline__ void window_regs(const uint32_t* qx, int o, uint32_t (&R)[4 * WIN]) {
  uint32_t X0[WIN];
#pragma unroll
  for (int y = 0; y < WIN; ++y) {
    X0[y] = __builtin_amdgcn_alignbyte(qx[WIN + y], qx[y], o);  // cells 0-3
    swar_window(X0[y], R[y], R[2 * WIN + y]);
    R[WIN + y] = R[3 * WIN + y] = 0;
  }
  if constexpr (WIN == 5) {  // column 4 of rows 0-3 (and of row 4) in one register
    const uint32_t o4 = (uint32_t)o * 0x0101u;
    const uint32_t c0 = __builtin_amdgcn_perm(qx[WIN + 1], qx[WIN + 0], 0x0C0C0400u + o4) |
                        __builtin_amdgcn_perm(qx[WIN + 3], qx[WIN + 2], 0x04000C0Cu + (o4 << 16));
    const uint32_t c1 = __builtin_amdgcn_alignbyte(0u, qx[WIN + 4], o);
    swar_window(c0, R[WIN + 0], R[3 * WIN + 0]);
    swar_window(c1, R[WIN + 1], R[3 * WIN + 1]);
  } else if constexpr (WIN > 5) {
#pragma unroll
    for (int y = 0; y < WIN; ++y)
      swar_window(__builtin_amdgcn_alignbyte(qx[2 * WIN + y], qx[WIN + y], o), R[WIN + y],
                  R[3 * WIN + y]);  // cells 4-7
  }
}

// ---- occupancy window records (obs_window_occ, ABI 2) ------------------------
// The record of one agent is WIN*WIN bytes, one per window cell: occ = c - 1 (the
// reference's map value: -1 for an obstacle nobody stands on or a cell out of
// bounds, else the agent count), marl_partial.py:323-342 as one plane.
__device__ __forceinline__ uint32_t swar_occ(uint32_t v) {  // 4 cells -> 4 occ bytes (c - 1)
  return (((v & 0x7F7F7F7Fu) | 0x80808080u) - 0x01010101u) ^ 0x80808080u;
}
// Record bytes as u32 words from the raw rows (qx as for window_regs).
template <int WIN>
__device__ __forceinline__ void occ_words(const uint32_t* qx, int o, uint32_t (&R)[(WIN * WIN + 3) / 4 + 1]) {
  constexpr int NW64 = (WIN * WIN + 7) / 8;
  uint64_t w[NW64];
#pragma unroll
  for (int i = 0; i < NW64; ++i) w[i] = 0;
#pragma unroll
  for (int y = 0; y < WIN; ++y) {
    const uint32_t lo = swar_occ(__builtin_amdgcn_alignbyte(qx[WIN + y], qx[y], o));  // cells 0-3
    if constexpr (WIN == 3) {
      put_bits<NW64>(w, 24 * y, 24, lo & 0xFFFFFFu);
    } else {
      const uint32_t hi = WIN == 5 ? swar_occ(__builtin_amdgcn_alignbyte(0u, qx[WIN + y], o))
                                   : swar_occ(__builtin_amdgcn_alignbyte(qx[2 * WIN + y], qx[WIN + y], o));
      put_bits<NW64>(w, 8 * WIN * y, 32, lo);
      put_bits<NW64>(w, 8 * WIN * y + 32, 8 * (WIN - 4), hi & ((1u << (8 * (WIN - 4))) - 1u));
    }
  }
#pragma unroll
  for (int k = 0; k < (WIN * WIN + 3) / 4 + 1; ++k)
    R[k] = k / 2 < NW64 ? (uint32_t)(w[k / 2] >> (32 * (k & 1))) : 0u;
}
// Stage one WIN*WIN-byte record at byte `ra` of LDS (odd length, any alignment):
// h = head bytes up to the next dword boundary (0..3), then ND aligned dwords, then
// the tail; with REC = 1 mod 8 the head and tail together are always 5 bytes, so
// every lane issues ND ds_write_b32 + 5 ds_write_b8 (no divergence).
template <int WIN>
__device__ __forceinline__ void stage_occ_record(const uint32_t (&R)[(WIN * WIN + 3) / 4 + 1], uint32_t ra) {
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  typedef __attribute__((address_space(3))) uint8_t lds_u8;
  constexpr int REC = WIN * WIN;
  constexpr int ND = (REC - 3) / 4;
  static_assert(REC - 4 * ND == 5, "odd window: head + tail = 5 bytes");
  const uint32_t h = (4u - (ra & 3u)) & 3u;
  lds_u32* d = (lds_u32*)(uintptr_t)(ra + h);
#pragma unroll
  for (int j = 0; j < ND; ++j) d[j] = __builtin_amdgcn_alignbyte(R[j + 1], R[j], h);
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const bool head = (uint32_t)i < h;
    const uint32_t hv = R[0] >> (8 * (i & 3));                                   // byte i
    const uint32_t tv = R[(4 * ND + i) >> 2] >> (8 * ((4 * ND + i) & 3));      // byte 4 ND + i
    *(lds_u8*)(uintptr_t)(ra + (head ? (uint32_t)i : (uint32_t)(4 * ND + i))) = (uint8_t)(head ? hv : tv);
  }
}

// ---- store-wave split (runner rollout, N = 16) --------------------------------
// A workgroup is three waves.  The "step wave" keeps only the
// dependency chain of a step: moves, LDS count atomics, edge collisions (a cross-lane
// scan) and the dones.  It keeps TWO agent-count maps: map s & 1 holds the counts
// after step s (each step moves an agent's count in that map from where it stood after
// step s - 2 to its new cell), so a step's map stays intact for the whole next barrier
// interval and the store waves read that step's window rows from it themselves.  Per
// agent the step wave hands over a 16-byte info word (new cell, the 4 neighbour bytes,
// flags, t) and, one step later, its edge count.  Two "store waves" take the steps in
// turn (even / odd) and spread each over two barrier intervals: a(q) builds the window
// record (SWAR) and stages it in the wave's LDS image, b(q) stores it with
// lane-contiguous 16-byte stores together with node / edge / avail / done / (row, col) /
// t / term, and every 16th step folds the fp64 rewards of 16 steps x 4 envs from
// per-agent reward codes.  One barrier per step (LDS traffic only), so the step wave
// issues no global store inside its loop and the stores stay in flight across barriers.
// Measured alternatives (a 2-wave form, a single image of raw window rows, a 3-slot ring
// published a barrier late, a MOVE / MAP step side, nontemporal stores) were slower and
// are gone from the source; their numbers are in DESIGN.md §4.1b.
constexpr int SPLIT_WAVES = 3;               // step wave + two store waves
constexpr int SPLIT_DBM_INFO = 2 * 64 * 16;  // info words of two steps
constexpr int SPLIT_DBM_EDGE = 3 * 64;       // edge counts of two steps + the launch's last step
// reward-code table + 32-step code ring: u8 codes (edge <= 15: 16 agents per env) and a
// 256-entry table, or, with 64 agents per env (edge <= 63), u16 codes and 1024 entries
__host__ __device__ constexpr int split_fold_lds(int L) { return L > 16 ? 1024 * 8 + 32 * 64 * 2 : 256 * 8 + 32 * 64; }

// info.z flag bits
constexpr uint32_t SF_DONE = 1, SF_LIVE = 2, SF_DNOLD = 4, SF_ENVC = 8, SF_SKIP = 16, SF_ALLDONE = 64;

// Workgroup barrier that waits for this wave's LDS traffic only: outstanding
// global stores stay in flight (a __syncthreads() would drain them every step).
__device__ __forceinline__ void split_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <typename P, typename V>
__device__ __forceinline__ void split_store(P p, V v) {
  *p = v;
}

// padded LDS cell index -> (row, col); cell < 2^16, pitch < 256
__device__ __forceinline__ int2 padded_cell_rc(const Geo& g, int cell) {
  const uint32_t pr = (uint32_t)(((uint64_t)(((uint32_t)cell << 8) & 0xFFFFFFu) *
                                  (uint64_t)(g.m_pitch24 & 0xFFFFFFu)) >> 32);
  return make_int2((int)pr - g.P, cell - (int)pr * g.pitch - g.pl);
}


// The two store waves.  Wave `par` takes the steps q with q % 2 == par:
//   a(q), the interval after barrier q + 1: step q's info word (written by the step wave
//     in its iteration q) and the agent's window rows read from map q & 1 -- intact until
//     the step wave's iteration q + 2 moves that map's counts again -- to the record, staged
//     in the wave's LDS image, and the node flag;
//   b(q), the interval after barrier q + 2: the edge count (the step wave computes it in
//     iteration q + 1), the reward code, the staged record out with lane-contiguous
//     16-byte stores, every per-agent and per-env output, and every 16th step the fold.
template <int WIN, int LL, bool OCC>
__device__ __forceinline__ void split_store_wave_dbm(const Geo& g, const Args& a, const unsigned char* m0,
                                                     const unsigned char* m1, const unsigned char* info,
                                                     const unsigned char* ering, unsigned char* own,
                                                     double* rtab, unsigned char* codes, int env0,
                                                     int lane, int par) {
  typedef __attribute__((address_space(1))) unsigned char gbyte;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef int i32x2 __attribute__((ext_vector_type(2)));
  constexpr int H2 = WIN / 2, REC = OCC ? WIN * WIN : 2 * WIN * WIN;
  constexpr int RCH = 4 * REC;  // 16-byte chunks of the wave's 64 records
  constexpr int NRC = (RCH + 63) / 64;
  const int T = a.T;
  const uint32_t E = (uint32_t)g.E, EN = E * (uint32_t)LL;
  const int slot = lane / LL, ag = lane % LL;
  // reward codes: node | SF_LIVE | SF_DNOLD | SF_ENVC | edge << 4 -- a byte while the edge
  // count fits 4 bits (16 agents), a u16 for 64 agents (edge <= 63, 1024 table entries)
  constexpr bool WIDE = LL > 16;
  constexpr int NCODE = WIDE ? 1024 : 256;
  typedef typename std::conditional<WIDE, uint16_t, unsigned char>::type code_t;
  code_t* const cring = (code_t*)codes;
  const uint32_t env = (uint32_t)(env0 + slot), ag0 = (uint32_t)env0 * LL;
  const u32x4* ost = (const u32x4*)__builtin_assume_aligned(own, 16);
  const u32x4* inf = (const u32x4*)__builtin_assume_aligned(info, 16);
  const int pitch = g.pitch, wpr = g.pitch >> 2;
  uint32_t k_nc = 0, k_nb = 0, k_fl = 0, k_t = 0, k_node = 0;  // step q's, kept from a to b

  for (int c = lane + 64 * par; c < NCODE; c += 128) {  // the code reward table (as the ALT waves)
    double rr = 0.0;  // exact fp64 op order of the reference
    if (c & SF_LIVE) {
      if (!(c & SF_DNOLD)) {
        if (c & SF_ENVC) rr = rr + g.collide_rew;
        rr = rr + g.step_rew;
      }
      rr = rr + g.collide_rew * (double)(c & 1);
      rr = rr + g.collide_rew * (double)(c >> 4);
    }
    rtab[c] = rr;
  }
  auto fold_batch = [&](uint32_t q0, int cnt) {  // one (env, step) per lane, agent order
    const int j = lane & 15, e = lane >> 4;
    if (j < cnt && e < 64 / LL) {
      double R = 0.0;
      if constexpr (!WIDE) {
        const u32x4 cv = *(const u32x4*)__builtin_assume_aligned(codes + ((q0 + j) & 31) * 64 + e * 16, 16);
        const uint32_t cw[4] = {cv.x, cv.y, cv.z, cv.w};
        double v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = rtab[(cw[i >> 2] >> (8 * (i & 3))) & 0xFFu];
#pragma unroll
        for (int i = 0; i < 16; ++i) R = R + v[i];
      } else {  // the env's 64 agents: 8 x 16 bytes of u16 codes, table reads one group ahead
        const u32x4* cp = (const u32x4*)__builtin_assume_aligned(cring + ((q0 + j) & 31) * 64, 16);
        double v[8];
        u32x4 cv = cp[0];
#pragma unroll
        for (int g8 = 0; g8 < 8; ++g8) {
          const uint32_t cw[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = rtab[(cw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu];
          if (g8 + 1 < 8) cv = cp[g8 + 1];
#pragma unroll
          for (int i = 0; i < 8; ++i) R = R + v[i];
        }
      }
      const uint32_t ei = (q0 + j) * E + (uint32_t)env0 + e;
      split_store((__attribute__((address_space(1))) double*)((gbyte*)a.reward + 8u * ei), R);
      if (a.reward_f32) a.reward_f32[ei] = (float)R;
    }
  };
  auto part_a = [&](uint32_t q) {
    const u32x4 iv = inf[(q & 1) * 64 + lane];
    const uint32_t* m32 = (const uint32_t*)((q & 1) ? m1 : m0) + (slot * g.map_env_bytes >> 2);
    const int nc = (int)iv.x;
    const int w0 = (nc - H2 * pitch - H2) >> 2;
    uint32_t qx[3 * WIN];
#pragma unroll
    for (int y = 0; y < WIN; ++y) {
      qx[y] = m32[w0 + y * wpr];
      qx[WIN + y] = m32[w0 + y * wpr + 1];
      qx[2 * WIN + y] = WIN > 5 ? m32[w0 + y * wpr + 2] : 0u;
    }
    const int o = (nc - H2) & 3;
    if constexpr (OCC) {
      uint32_t R[(WIN * WIN + 3) / 4 + 1];
      occ_words<WIN>(qx, o, R);
      stage_occ_record<WIN>(R, lds_addr(own + lane * REC));
    } else {
      uint32_t R[4 * WIN];
      window_regs<WIN>(qx, o, R);
      stage_record<WIN>(R, own + lane * REC);
    }
    // node collision (:344-362): post-step count = c - 1 + obstacle >= 2 (centre cell)
    const uint32_t ctr = (__builtin_amdgcn_alignbyte(qx[WIN + H2], qx[H2], o) >> (8 * H2)) & 0xFFu;
    k_node = ((ctr & 0x7Fu) + (ctr >> 7) >= 3u && !(iv.z & SF_SKIP)) ? 1u : 0u;
    k_nc = iv.x, k_nb = iv.y, k_fl = iv.z, k_t = iv.w;
  };
  auto part_b = [&](uint32_t q) {
    u32x4 rv[NRC];
#pragma unroll
    for (int k = 0; k < NRC; ++k) rv[k] = ost[(k < NRC - 1 || lane + 64 * k < RCH) ? lane + 64 * k : 0];
    // (the last step's count has its own slot: the step wave writes it while b(T - 3) may
    // still read slot (T - 1) & 1)
    const uint32_t edge = ering[(q + 1 == (uint32_t)T ? 2u : (q & 1)) * 64 + lane];
    cring[(q & 31) * 64 + lane] =
        (code_t)(k_node | (k_fl & (SF_LIVE | SF_DNOLD | SF_ENVC)) | ((edge & (WIDE ? 0x3Fu : 0xFu)) << 4));
    gbyte* rec = (gbyte*)(OCC ? a.obs_window_occ : a.obs_window) + (q * EN + ag0) * (uint32_t)REC;
#pragma unroll
    for (int k = 0; k < NRC; ++k)
      if (k < NRC - 1 || lane + 64 * k < RCH)
        split_store((__attribute__((address_space(1))) u32x4*)(rec + 16u * (lane + 64 * k)), rv[k]);
    const uint32_t fl = k_fl;
    const uint32_t nzn = (((k_nb & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) >> 7) & 0x01010101u;
    const uint32_t availm = __builtin_amdgcn_udot4(nzn, 0x08040201u, 16u, false);
    const uint32_t ai = q * EN + ag0 + lane;
    const int2 rc = padded_cell_rc(g, (int)k_nc);
    split_store((__attribute__((address_space(1))) i32x2*)((gbyte*)a.traj_pos + 8u * ai), i32x2{rc.x, rc.y});
    split_store((gbyte*)a.node + ai, (unsigned char)k_node);
    split_store((gbyte*)a.edge + ai, (unsigned char)edge);
    split_store((gbyte*)a.avail + ai, (unsigned char)availm);
    split_store((gbyte*)a.traj_done + ai, (unsigned char)(fl & SF_DONE));
    if (ag == LL - 1) {
      const uint32_t ei = q * E + env;
      split_store((__attribute__((address_space(1))) int*)((gbyte*)a.traj_t + 4u * ei), (int)k_t);
      split_store((gbyte*)a.term + ei, (unsigned char)((fl & SF_ALLDONE) ? 1 : 0));
      if (a.err && (fl & SF_SKIP)) atomicCAS(a.err, 0, (int)env + 1);
    }
    // the batch ends here: every code of it is in the ring (this wave's b(q) just now,
    // the other wave's b(q - 1) before the last barrier).  Not so for the launch's last
    // step: b(T - 1) runs in the same interval as the other wave's b(T - 2), so that batch
    // is folded after one more barrier, below
    if ((q & 15u) == 15u && q + 1 != (uint32_t)T) {
      wave_fence();
      fold_batch(q & ~15u, 16);
    }
  };

  // T rounds: the launch's last step has its edge count published with its info word
  // (barrier T), so its wave runs a(T - 1) and b(T - 1) back to back in the last interval
  // instead of spending one more barrier interval on b(T - 1) alone
  const int rounds = T > 0 ? T : 0;
  for (int s = 1; s <= rounds; ++s) {
#ifdef MAPFX_STAMPS  // diagnostic: end of round s - 1's work (columns 5 / 7 of row s - 1)
    if (s > 1) {
      unsigned long long t_;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
      if (blockIdx.x == 0 && lane == 0 && s - 1 < 256) g_stamps[(s - 1) * 8 + 5 + 2 * par] = t_;
    }
#endif
    split_barrier();
    const int q = s - 1;  // a(q) now; b(q - 1) by the other parity
    if ((q & 1) == par) {
      part_a((uint32_t)q);
      if (q == T - 1) {  // the last step: its b part right away (own staged record: LDS order)
        wave_fence();
        part_b((uint32_t)q);
      }
    } else if (q >= 1) {
      part_b((uint32_t)(q - 1));
    }
  }
  // barrier T + 1 (the step wave meets it after its state write-back): codes T - 2 (the
  // other wave's) and T - 1 (this wave's) are both in the ring
  split_barrier();
  if (T > 0 && ((T - 1) & 1) == par) fold_batch((uint32_t)(T - 1) & ~15u, ((T - 1) & 15) + 1);
}

// FULLW: every lane owns an agent (N == L and E % EPW == 0) -> no lane masks.
// RUNNER (rollout only): the standard runner outputs are all present (reward,
// term, node, edge, avail, traj_pos/done/t, window obs) -> no per-output tests.
// LL: lanes per env fixed at compile time (0: g.L at run time); with FULLW, N == LL.
//
// Software pipeline (one wave, in-order LDS).  Iteration s runs
//   A  step s's move decision from the carried neighbour bytes, its `dep` write and
//      count atomics                                            (dependency chain)
//   B  issue of step s's post-step window rows, the occupant's move, and the
//      previous-but-one step's reward row (fp64 fold)
//   C  the HEAVY part of step s-1 from registers saved in iteration s-1: window
//      SWAR, record and per-agent stores, node/edge collisions, fp64 reward, and
//      the env outputs of step s-2 -- VALU work that fills B's LDS latency
//   D  step s's neighbour bytes, dones, t and all-done ballot  (dependency chain)
// so only A and D (a few dozen instructions) sit on the serial chain between
// steps.  The last step's heavy part and tails run after the loop.
// Wave priorities of the split (s_setprio): with the ALT store waves and the batched
// reward fold the STEP wave's chain is the longer one (block-0 stamps at C2: step wave
// busy ~2300 cycles per barrier interval, each store wave ~850), so the step wave wins
// issue arbitration against the other blocks' store waves on its SIMD: C2 T = 20
// 25.0 -> 23.5 us (round 3; with the round-2 single store wave the store side was the
// long chain and its priority paid instead).
constexpr int MAPFX_PRIO_STEP = 3;
// ABT: the action block (0: MAPFX_AB); the split kernel has an 8-step instance for short
// launches (T <= MAPFX_AB_SHORT_T): C2 T = 20 21.1 vs 21.9 us, while at T = 64 the 16-step
// block stays faster (52.7 vs 57.0 us; tools/gpucmd_r04q.sh)
template <int WIN, bool ROLL, bool FULLW, bool RUNNER, int LL, bool SPLIT = false, bool OCC = false, int ABT = 0>
// (split: 4 blocks per CU must be resident -- one wave per SIMD of each role -- so the
// register budget is that of SPLIT_WAVES waves per SIMD)
__global__ void __launch_bounds__(SPLIT ? 64 * SPLIT_WAVES : 64, SPLIT ? SPLIT_WAVES : 1)
    mapf_wave_kernel(MAPFX_HOT_PARAMS, Args a0, Geo g0) {
  Args a = a0;
  Geo g = g0;
  MAPFX_HOT_APPLY(a, g);
  extern __shared__ __align__(16) unsigned char lds[];
  static_assert(!SPLIT || (ROLL && FULLW && RUNNER && (LL == 16 || LL == 64) && WIN > 0),
                "split: runner rollout, N = 16 or 64");
  static_assert(!OCC || SPLIT, "occupancy records: the split's store waves");
  if constexpr (SPLIT) {
    if (threadIdx.x >= 64) {  // the output side of the split
      const int e0 = xcd_block(blockIdx.x, g.nblk) * (64 / LL);
      if (g.wv_fast) {  // the store waves build their share of the padded maps (rows
        // ag + 16 w of each env, w = this wave's index: the step wave takes w = 0), then
        // the barrier the step wave meets after its own rows
        const int l64 = threadIdx.x & 63, sl = l64 / LL;
        const uint32_t* src = (const uint32_t*)(a.bits + (g.map_shared ? 0 : (long long)(e0 + sl) * g.map_stride));
        uint32_t pf[1][3];
        const int bl = l64 % LL + LL * (threadIdx.x >> 6);
        fast_row_prefetch<1>(g, src, bl, LL * SPLIT_WAVES, pf);
        __builtin_amdgcn_sched_barrier(0);
        // (as in the step wave, below; + the step wave's LDS offsets, dead here)
        asm volatile("" ::"s"(g0.map_words), "s"(a0.do_step), "s"(g0.wv_off_dep), "s"(g0.wv_off_bits),
                     "s"(g0.wv_off_rew));
        build_map_rows_fast<MAPFX_FAST_WPR, 1>(g, (uint32_t*)(lds + g.wv_off_map + sl * g.map_env_bytes), src,
                                               bl, LL * SPLIT_WAVES, pf,
                                               (uint32_t*)(lds + g.wv_off_split + sl * g.map_env_bytes));
      }
      split_barrier();
      constexpr int RECB = OCC ? WIN * WIN : 2 * WIN * WIN;  // one wave's staged image: 64 * RECB
      const int par = (int)(threadIdx.x >> 6) - 1;            // this wave's step parity
      // [M1: 64 / LL maps][info: 2 steps][edge: 2 steps][staged records: 2 waves][fold]
      unsigned char* m1 = lds + g.wv_off_split;
      unsigned char* inf = m1 + (64 / LL) * g.map_env_bytes;
      unsigned char* eri = inf + SPLIT_DBM_INFO;
      unsigned char* ownd = eri + SPLIT_DBM_EDGE;
      double* rt = (double*)(ownd + 2 * 64 * RECB);
      split_store_wave_dbm<WIN, LL, OCC>(g, a, lds + g.wv_off_map, m1, inf, eri, ownd + par * 64 * RECB, rt,
                                         (unsigned char*)(rt + (LL > 16 ? 1024 : 256)), e0, threadIdx.x & 63, par);
      return;
    }
    if (MAPFX_PRIO_STEP) __builtin_amdgcn_s_setprio(MAPFX_PRIO_STEP);
  }
  constexpr int WW = WIN * WIN;
  constexpr int H2 = WIN / 2;
  constexpr int REC = 2 * WW;  // record bytes per agent
  constexpr int NX = WIN > 0 ? WIN : 1;
  constexpr bool FIXN = FULLW && LL > 0;   // N == LL known at compile time
  constexpr bool FLAT = RUNNER && FULLW;   // env outputs stored by every lane of the env
  PSTAMP(6);
  const int L = LL > 0 ? LL : g.L;
  const int lshift = LL > 0 ? (LL == 64 ? 6 : LL == 32 ? 5 : LL == 16 ? 4 : LL == 8 ? 3 : LL == 4 ? 2 : LL == 2 ? 1 : 0)
                            : g.lshift;
  const int lane64 = threadIdx.x & 63;
  const int slot = lane64 >> lshift;  // env slot within the wave
  const int ag = lane64 & (L - 1);    // agent index
  const int base = slot << lshift;    // first lane of this env
  const int EPW = 64 >> lshift;
  const int env0 = xcd_block(blockIdx.x, g.nblk) * EPW;
  const int env = env0 + slot;
  const int N = FIXN ? LL : g.N;
  const bool env_ok = FULLW || env < g.E;
  const bool has = FULLW || (env_ok && ag < N);
  const bool do_step = ROLL || a.do_step;
  const uint64_t envmask = (L == 64 ? ~0ull : ((1ull << L) - 1ull)) << base;
  const uint32_t oa = (uint32_t)(env * N + ag);  // agent index inside one step slot
  // (every env full: E = grid x EPW, from the preloaded grid size -- the first action
  // loads wait for no kernarg fetch)
  const uint32_t EN = FULLW ? (uint32_t)g.nblk * (uint32_t)(EPW * N) : (uint32_t)(g.E * N);
  const bool t_long = ROLL && ((hp_nm >> 26) & 1u);  // T >= 16 >= AB
  // Actions are fetched for AB steps at a time: one VMEM wait per block instead of
  // one per step (a wait on a per-step load would also drain the step's stores).
  constexpr int MAPFX_AB = 16;
  constexpr int AB = ROLL ? (ABT > 0 ? ABT : MAPFX_AB) : 1;
  static_assert(AB <= 16, "t_long: the first action block lies within T >= 16 steps");
  uint32_t actpk[(AB + 3) / 4];
  // Action blocks from memory are prefetched one block ahead: block 0 is issued
  // first of all (its HBM latency overlaps the state loads and the map build; issued
  // after them, step 0 still waited ~900 cycles for it at C2 T = 20), block b + 1 as
  // soon as block b is unpacked, so the wait at a block boundary finds it arrived.
  int nxt[AB];
  const bool act_mem = do_step && !a.use_rng;
  // block 0 of an int8 launch of >= 16 steps: no clamp to T (a kernarg from memory)
  const bool first_early = act_mem && ROLL && t_long && a.act_dtype == MAPFX_I8;
  if (first_early) {
    const int8_t* ap = (const int8_t*)a.actions;
    const uint32_t oc_ = has ? oa : 0u;
#pragma unroll
    for (int k = 0; k < AB; ++k) nxt[k] = (ap + (uint32_t)k * EN)[oc_];
  }

  // bitmap words of this lane's first map rows (fast build): issued next
  const uint32_t* bsrc = (const uint32_t*)(a.bits + (g.map_shared || !env_ok ? 0 : (long long)env * g.map_stride));
  // (the split kernel's three waves build the rows together: lane ag + 16 w of 48)
  constexpr int RPF = SPLIT ? 1 : 4;
  const int bl = ag, bnl = SPLIT ? LL * SPLIT_WAVES : L;
  uint32_t pfw[RPF][3];
  if (g.wv_fast) fast_row_prefetch<RPF>(g, bsrc, bl, bnl, pfw);
  int tcur = env_ok ? a.t[env] : 0;  // (issued first: its pointer is preloaded)
  int2 p0 = make_int2(0, 0), q0 = make_int2(0, 0);
  bool dn = false;
  if (has) {
    p0 = ((const int2*)a.pos)[oa];
    q0 = ((const int2*)a.goal)[oa];
    dn = a.done[oa] != 0;
  }
  // The kernargs past the preloaded ones are fetched at entry and nothing above waits
  // for them (T and E come from the preloaded dwords).  The dead words of their merged
  // scalar loads stay live up to here, so no register of a load in flight is reused --
  // and waited for -- before the loads above are issued: per-step kernel 5.05 -> 4.98 us
  // (tools/r06/gpu_p.sh; fetched after these loads instead, 5.3 us, gpu_o.sh).
  if constexpr (FULLW && LL > 0) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::"s"(g0.map_words), "s"(a0.do_step));
  }

  const int pitch = g.pitch;
  const int Wd = g.W;
  const bool want_win = WIN > 0 && (RUNNER || a.obs_window);
  const int cell0 = g.P * pitch + g.pl;  // padded index of cell (0, 0)

  unsigned char* map = lds + g.wv_off_map + slot * g.map_env_bytes;
  uint32_t* map32 = (uint32_t*)map;
  unsigned char* dep = lds + g.wv_off_dep + slot * g.map_env_bytes;  // move dir per old cell
  uint32_t* bitsL = (uint32_t*)(lds + g.wv_off_bits + slot * g.wv_bits_env_bytes);
  double* rewL = (double*)(lds + g.wv_off_rew);
  const int rew_buf = g.wv_rew_buf / 8;  // doubles per reward buffer
  const int rew_row = g.wv_rew_row;      // doubles per env row
  const int T = ROLL ? a.T : 1;
  const auto fetch = [&](int s0) {
    // s0 is opaque here: the row offsets are formed at the fetch (scalar row offset +
    // the lane's offset) instead of AB address registers stepped every loop iteration
    int sb = s0;
    asm volatile("" : "+s"(sb));
    if (!ROLL || a.act_dtype != MAPFX_I8) {
#pragma unroll
      for (int k = 0; k < AB; ++k)
        nxt[k] = (has && sb + k < T) ? load_action(a.actions, a.act_dtype, (uint32_t)(sb + k) * EN + oa) : 4;
    } else {  // int8 buffer: AB unconditional loads (clamped addresses)
      const int8_t* ap = (const int8_t*)a.actions;
      const uint32_t oc_ = has ? oa : 0u;
#pragma unroll
      for (int k = 0; k < AB; ++k) nxt[k] = (ap + (uint32_t)min(sb + k, T - 1) * EN)[oc_];
    }
  };
  if (act_mem && ROLL && !first_early) fetch(0);  // (one step: after the state loads -- a
                                                  // non-int8 action is range-checked at its
                                                  // load, which would wait for it here)
  int cur = 0, gcell = -1, st = 0;  // padded cell of the agent / of its goal
  if (has) {
    cur = cell0 + p0.x * pitch + p0.y;
    gcell = cell0 + q0.x * pitch + q0.y;
    if (a.steps) st = a.steps[oa];
  }
  if (act_mem && !ROLL) fetch(0);
  PSTAMP(0);

  // ---- padded map (from the bitmap: global -> registers, or staged in LDS), agents ----
  if (env_ok && !g.wv_fast) {
    for (int w = ag; w < g.bits_words; w += L) bitsL[w] = bsrc[w];
  }
  if (ROLL && !SPLIT) {  // both reward rows start at +0.0 (folds of steps < 0 read them)
    for (int i = lane64; i < 2 * rew_buf; i += 64) rewL[i] = 0.0;
  }
  if (!g.wv_fast) wave_fence();
  PSTAMP(1);
  // the split's second count map M1 (odd steps) of this env, at the start of the split region
  constexpr bool DBM = SPLIT;
  uint32_t* m1_32 = DBM ? (uint32_t*)(lds + g.wv_off_split + slot * g.map_env_bytes) : nullptr;
  if (g.wv_fast) build_map_rows_fast<MAPFX_FAST_WPR, RPF>(g, map32, bsrc, bl, bnl, pfw, m1_32);
  else build_map_rows_c(g, map32, bitsL, ag, L);
  if (DBM && !g.wv_fast) {  // (the fallback builder fills M0 alone: copy it)
    wave_fence();
    for (int w = ag; w < (g.map_env_bytes >> 2); w += L) m1_32[w] = map32[w];
  }
  if constexpr (SPLIT) split_barrier();  // + the store waves' rows
  else wave_fence();
  PSTAMP(2);
  if (has) atomicAdd(&map32[cur >> 2], 1u << ((cur & 3) * 8));
  if (DBM && has) atomicAdd(&m1_32[cur >> 2], 1u << ((cur & 3) * 8));
  wave_fence();

  const auto cell_rc = [&](int cell) {  // padded cell -> (row, col); cell < 2^16, pitch < 256
    const uint32_t pr = (uint32_t)(((uint64_t)(((uint32_t)cell << 8) & 0xFFFFFFu) *
                                    (uint64_t)(g.m_pitch24 & 0xFFFFFFu)) >> 32);
    return make_int2((int)pr - g.P, cell - (int)pr * pitch - g.pl);
  };
  // `sum(rewards)`: naive left fold in agent order (:141) over the env's LDS row
  // (padded with +0.0: adding +0.0 never changes a sum that starts at +0.0)
  auto fold = [&](int buf) {
    const double* rw = rewL + buf * rew_buf + slot * rew_row;
    double R = 0.0;
    if constexpr (FIXN) {
#pragma unroll
      for (int j0 = 0; j0 < LL; j0 += 16) {
        double v[LL < 16 ? LL : 16];
#pragma unroll
        for (int j = 0; j < (LL < 16 ? LL : 16); ++j) v[j] = rw[j0 + j];
#pragma unroll
        for (int j = 0; j < (LL < 16 ? LL : 16); ++j) R = R + v[j];
      }
    } else if (L == 16) {  // all 16 lanes wrote their slot (+0.0 past N)
      double v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = rw[j];
#pragma unroll
      for (int j = 0; j < 16; ++j) R = R + v[j];
    } else {
      for (int j = 0; j < N; ++j) R = R + rw[j];
    }
    return R;
  };
  // env outputs of a step: reward, term, t, f32 copy, error flag, staged window copy-out
  auto tail = [&](int buf, uint32_t se_t, bool skip_t, bool alldone_t, int tcur_t, double R) {
    const uint32_t ei = se_t + env;
    if (FLAT) {  // every lane of the env stores the same values: no lane branch
      st_off(a.reward, ei * 8u, R);
      st_off(a.term, ei, (uint8_t)(alldone_t ? 1 : 0));
      st_off(a.traj_t, ei * 4u, tcur_t);
    } else if (env_ok && ag == 0) {
      if (RUNNER) {
        st_off(a.reward, ei * 8u, R);
        st_off(a.term, ei, (uint8_t)(alldone_t ? 1 : 0));
        st_off(a.traj_t, ei * 4u, tcur_t);
      } else {
        if (do_step && a.reward) a.reward[ei] = R;
        if (a.term) a.term[ei] = alldone_t ? 1 : 0;
        if (a.traj_t) a.traj_t[ei] = tcur_t;
      }
    }
    if (env_ok && ag == 0) {
      if (do_step && a.reward_f32) a.reward_f32[ei] = (float)R;
      if (do_step && a.err && skip_t) atomicCAS(a.err, 0, env + 1);
    }
  };

  // ---- state of step q = s-1 saved for its heavy part (C) ----
  uint32_t qx[3 * NX];  // window rows: [xlo | xhi | xhi2] (WIN == 0: 5 neighbour bytes)
  int q_oc = 0, q_nc = 0, q_act = 4, q_pre = 0, q_tcur = 0;
  uint32_t q_dj = 0xFFu, q_nb = 0;
  bool q_moved = false, q_envc = false, q_dnold = false, q_dn = false, q_live = false;
  bool q_skip = false, q_alldone = false;
  // ---- env outputs of step p = s-2 waiting for their fold ----
  uint32_t p_se = 0;
  bool p_skip = false, p_alldone = false;
  int p_tcur = 0;

  // edge collisions (:364-383) of step q: i moved into a cell X that had pre-step
  // occupants; j counts iff j moved from X back into i's old cell, i.e. in the
  // opposite direction (act ^ 1)
  auto edge_of = [&]() {
    int edge = 0;
    const bool suspect = q_moved && q_pre > 0;
    if (__ballot(suspect)) {
      if (suspect && q_pre == 1) edge = (q_dj & 0x7Fu) == (uint32_t)(q_act ^ 1) ? 1 : 0;
      if (__ballot(suspect && q_pre > 1)) {  // stacked pre-occupants: scan the env
        for (int j = 0; j < N; ++j) {
          const int oj2 = __shfl(q_oc, base + j);
          const int nj2 = __shfl(q_nc, base + j);
          if (suspect && q_pre > 1) edge += (oj2 == q_nc) & (nj2 == q_oc);
        }
      }
    }
    return edge;
  };

  // HEAVY part of step q (slot qs): window, node, edge, reward, per-agent stores.
  auto heavy = [&](int qs) {
    const uint32_t so = ROLL ? (uint32_t)qs * EN : 0u;
    const int buf = ROLL ? (qs & 1) : 0;
    uint32_t node = 0;
    uint32_t R[WIN > 0 ? 4 * WIN : 1];  // [plane][cols 0-3 | cols 4-7][row]
    if constexpr (WIN > 0) {
      const int o = (q_nc - H2) & 3;  // same byte offset in every row (pitch % 4 == 0)
      window_regs<WIN>(qx, o, R);
      // centre cell (H2 <= 3: it lies in cells 0-3 of the middle row)
      const uint32_t ctr = (__builtin_amdgcn_alignbyte(qx[WIN + H2], qx[H2], o) >> (8 * H2)) & 0xFFu;
      node = (ctr & 0x7Fu) + (ctr >> 7) >= 3u ? 1u : 0u;   // count = c - 1 + obstacle >= 2
    } else {
      node = (qx[0] & 0x7Fu) + ((qx[0] >> 7) & 1u) >= 3u ? 1u : 0u;
    }
    if (q_skip) node = 0;
    // avail (:203-224): a neighbour is available iff its c != 0; stay always
    const uint32_t nzn = (((q_nb & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) >> 7) & 0x01010101u;
    const uint32_t availm = __builtin_amdgcn_udot4(nzn, 0x08040201u, 16u, false);
    if constexpr (WIN > 0) {
      if (want_win && has) {
        // the record straight to HBM from registers (records staged in LDS for 16-byte
        // stores measured slower for the per-step launch)
        write_record<WIN>(R, a.obs_window, (so + oa) * (uint32_t)REC);
      }
    }
    const uint32_t ai = so + oa;
    if (has) {
      const int2 rc = cell_rc(q_nc);
      if (RUNNER) {
        a.node[ai] = (uint8_t)node;
        st_off(a.traj_pos, ai * 8u, rc);
        a.traj_done[ai] = q_dn ? 1 : 0;
        a.avail[ai] = (uint8_t)availm;
      } else {
        if (do_step && a.node) a.node[ai] = (uint8_t)node;
        if (a.traj_pos) ((int2*)a.traj_pos)[ai] = rc;
        if (a.traj_done) a.traj_done[ai] = q_dn ? 1 : 0;
        if (a.avail) a.avail[ai] = (uint8_t)availm;
      }
    }
    const int edge = edge_of();
    // reward (:94-130, exact fp64 op order)
    double rr = 0.0;
    if (q_live) {
      if (!q_dnold) {
        if (q_envc) rr = rr + g.collide_rew;
        rr = rr + g.step_rew;
      }
      rr = rr + g.collide_rew * (double)node;
      rr = rr + g.collide_rew * (double)edge;
    }
    if (do_step && (FIXN || ag < rew_row))  // lanes past N pad the row with +0.0
      rewL[buf * rew_buf + slot * rew_row + ag] = has ? rr : 0.0;
    if (has) {
      if (RUNNER || (do_step && a.edge)) a.edge[ai] = (uint8_t)(edge > 255 ? 255 : edge);
    }
  };

  // Retire the state loads here (s_waitcnt vmcnt(0), gfx9 encoding): otherwise the
  // waitcnt pass merges "load pending" into the loop header and re-waits vmcnt(0)
  // -- i.e. drains every outstanding store -- at each use of the state inside the loop.
  __builtin_amdgcn_s_waitcnt(0x0F70);
  // Raw map bytes of the 4 neighbours (byte d = cell of action d), carried from the
  // end of one step (post-step map) to the move decision of the next (pre-step
  // map): the move test needs no LDS round trip.
  uint32_t nb = 0;
  if (has)
    nb = (uint32_t)map[cur - pitch] | ((uint32_t)map[cur + pitch] << 8) |
         ((uint32_t)map[cur - 1] << 16) | ((uint32_t)map[cur + 1] << 24);
  PSTAMP(3);
  // the action of step s: blocks of AB steps unpacked from the prefetch, 4 per u32
  const auto next_action = [&](int s) {
    if ((s & (AB - 1)) == 0) {  // actions of steps s .. s+AB-1, packed 4 per u32
      int v[AB];
      if (!do_step) {  // observation pass: there is no action buffer
#pragma unroll
        for (int k = 0; k < AB; ++k) v[k] = 4;
      } else if (a.use_rng) {
#pragma unroll
        for (int k = 0; k < AB; ++k) v[k] = gen_action(a.seed, g.env_offset + env, a.t0 + s + k, ag);
      } else {  // the prefetched block; the next one is issued right away
#pragma unroll
        for (int k = 0; k < AB; ++k) v[k] = nxt[k];
        if (ROLL && s + AB < T) fetch(s + AB);
      }
#pragma unroll
      for (int k = 0; k < (AB + 3) / 4; ++k) actpk[k] = 0;
#pragma unroll
      for (int k = 0; k < AB; ++k) {
        uint32_t u = (uint32_t)v[k];
        if (!(has && do_step && s + k < T)) u = 4u;
        if (u > 4u) u = 0xFFu;  // invalid action (the reference asserts, :92)
        actpk[k >> 2] |= u << (8 * (k & 3));
      }
    }
    const int act_ = (int)(actpk[0] & 0xFFu);
#pragma unroll
    for (int k = 0; k < (AB + 3) / 4; ++k)  // shift the packed actions down one byte
      actpk[k] = (k + 1 < (AB + 3) / 4) ? __builtin_amdgcn_alignbit(actpk[k + 1], actpk[k], 8)
                                        : (actpk[k] >> 8);
    return act_;
  };

  if constexpr (DBM) {
    // ---- the split's step wave: map s & 1 is moved from the positions after step
    // s - 2 to those after step s; the store waves read step s's window rows from it ----
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    unsigned char* m1 = (unsigned char*)m1_32;
    u32x4* info = (u32x4*)__builtin_assume_aligned(lds + g.wv_off_split + EPW * g.map_env_bytes, 16);
    unsigned char* ering = (unsigned char*)(info + 128);
    int cp0 = cur, cp1 = cur;  // where this lane's agent is counted in M0 / M1
    bool reset_pending = false;
    // The step body below is instanced per (map parity, autoreset, invalid-action check):
    // the parity picks M0 / M1 and cp0 / cp1 at compile time, autoreset is one uniform
    // branch outside the loop, and the per-step ballot for an invalid action (the env
    // skips the step, :91-92) runs only in an action block that holds one (blk_bad, from
    // the block's unpack) -- the step wave's chain paces the launch.
    bool blk_bad = false;
    const auto unpack_block = [&](int s_) __attribute__((always_inline)) {  // steps s .. s+AB-1, 4 per u32
      const int s = __builtin_amdgcn_readfirstlane(s_);  // (wave-uniform)
      int v[AB];
      if (a.use_rng) {
#pragma unroll
        for (int k = 0; k < AB; ++k) v[k] = gen_action(a.seed, g.env_offset + env, a.t0 + s + k, ag);
      } else {  // the prefetched block; the next one is issued right away
#pragma unroll
        for (int k = 0; k < AB; ++k) v[k] = nxt[k];
        if (s + AB < T) fetch(s + AB);
      }
      uint32_t bad = 0;
#pragma unroll
      for (int k = 0; k < (AB + 3) / 4; ++k) actpk[k] = 0;
#pragma unroll
      for (int k = 0; k < AB; ++k) {
        uint32_t u = (uint32_t)v[k];
        if (s + k >= T) u = 4u;
        if (u > 4u) u = 0xFFu;  // invalid action (the reference asserts, :92)
        bad |= u;
        actpk[k >> 2] |= u << (8 * (k & 3));
      }
      blk_bad = __builtin_amdgcn_readfirstlane(__ballot((bad & 0x80u) != 0) != 0 ? 1 : 0) != 0;
    };
    const auto step = [&](auto odd_c, auto ar_c, auto chk_c, int s) __attribute__((always_inline)) {
      constexpr bool ODD = decltype(odd_c)::value;  // map s & 1
      constexpr bool AR = decltype(ar_c)::value;    // autoreset
      constexpr bool CHK = decltype(chk_c)::value;  // the block holds an invalid action
      unsigned char* mp = ODD ? m1 : map;
      uint32_t* mp32 = (uint32_t*)mp;
      int& cpr = ODD ? cp1 : cp0;
      if constexpr (AR) {
        if (__ballot(reset_pending)) {
          // the last step ended these envs' episodes (their agents are back at init_pos,
          // mapf_gridworld.py:70-83): count them there in this step's map -- intact since
          // barrier s - 1's readers are done -- and read their neighbours
          if (reset_pending) {
            const int cpi = cpr;
            atomicAdd(&mp32[cpi >> 2], cpi != cur ? 0u - (1u << ((cpi & 3) * 8)) : 0u);
            atomicAdd(&mp32[cur >> 2], cpi != cur ? 1u << ((cur & 3) * 8) : 0u);
            cpr = cur;
          }
          wave_fence();
          if (reset_pending)
            nb = (uint32_t)mp[cur - pitch] | ((uint32_t)mp[cur + pitch] << 8) |
                 ((uint32_t)mp[cur - 1] << 16) | ((uint32_t)mp[cur + 1] << 24);
          reset_pending = false;
        }
      }
      const int act = (int)(actpk[0] & 0xFFu);
#pragma unroll
      for (int k = 0; k < (AB + 3) / 4; ++k)  // shift the packed actions down one byte
        actpk[k] = (k + 1 < (AB + 3) / 4) ? __builtin_amdgcn_alignbit(actpk[k + 1], actpk[k], 8)
                                          : (actpk[k] >> 8);
      STAMP(0);
      // A: move decision on the pre-step neighbours (:319-342), this map's count moves
      const int oc = cur;
      const bool mv = !dn && (uint32_t)act < 4u;
      const uint32_t v = mv ? ((nb >> ((act & 3) * 8)) & 0xFFu) : 0u;
      const bool envc = mv && (v & 0x7Fu) == 0u;
      const bool skip = CHK && (__ballot(act == 0xFF) & envmask) != 0;
      const bool moved = mv && (v & 0x7Fu) != 0u && !skip;
      int dlt = (act & 2) ? 1 : pitch;
      dlt = (act & 1) ? dlt : -dlt;
      const int nc = moved ? oc + dlt : oc;
      dep[oc] = (unsigned char)(moved ? (uint32_t)act : 0x7Fu);
      const int cpi = cpr;
      atomicAdd(&mp32[cpi >> 2], cpi != nc ? 0u - (1u << ((cpi & 3) * 8)) : 0u);
      atomicAdd(&mp32[nc >> 2], cpi != nc ? 1u << ((nc & 3) * 8) : 0u);
      cpr = nc;
      cur = nc;
      STAMP(2);
      // B: the new cell's 4 neighbours (the next move decision, avail) and the pre-step
      // occupant's move (the edge test)
      const uint32_t n_up = mp[nc - pitch], n_dw = mp[nc + pitch], n_lf = mp[nc - 1], n_rt = mp[nc + 1];
      const uint32_t dj = dep[nc];
      STAMP(1);
      // C: step s - 1's edge count (:364-383), for the store wave's b part (counting it in
      // the store waves' a part instead, from old / new cell, action and the occupant's move
      // in the info word, cut block 0's barrier interval 1904 -> 1700 cycles but measured
      // 25.2 vs 21.6 us at C2 T = 20, gpurun_out/r04o: kept here)
      if (s > 0) {
        const int e = edge_of();
        ering[(ODD ? 0 : 1) * 64 + lane64] = (unsigned char)(e > 255 ? 255 : e);
      }
      STAMP(3);
      // D: dones, t (:112-117), the step's info word
      const uint32_t nbn = n_up | (n_dw << 8) | (n_lf << 16) | (n_rt << 24);
      const bool dn_old = dn;
      const bool live = !skip;
      if (live && nc == gcell) dn = true;
      if (live && tcur + 1 >= g.limit) dn = true;
      if (live && !dn_old) ++st;
      if (!skip) ++tcur;
      const bool alldone = (__ballot(!dn) & envmask) == 0;
      const uint32_t fl = (dn ? SF_DONE : 0u) | (live ? SF_LIVE : 0u) | (dn_old ? SF_DNOLD : 0u) |
                          (envc ? SF_ENVC : 0u) | (skip ? SF_SKIP : 0u) | (alldone ? SF_ALLDONE : 0u);
      info[(ODD ? 1 : 0) * 64 + lane64] = u32x4{(uint32_t)nc, nbn, fl, (uint32_t)tcur};
      q_oc = oc;
      q_nc = nc;
      q_act = act;
      q_pre = (int)(v & 0x7Fu) - 1 + (int)(v >> 7);
      q_dj = dj;
      q_moved = moved;
      nb = nbn;
      if (s == T - 1) {  // the last step's edge count now (slot 2): its b part runs next interval
        const int e = edge_of();
        ering[2 * 64 + lane64] = (unsigned char)(e > 255 ? 255 : e);
      }
      if constexpr (AR) {
        if (alldone) {  // counted at init_pos in the next step's map
          const int2 p = ((const int2*)a.init_pos)[oa];
          cur = cell0 + p.x * pitch + p.y;
          dn = false;
          st = 0;
          tcur = 0;
          reset_pending = true;
        }
      }
      STAMP(4);
      split_barrier();  // info s, map s & 1, edge s - 1 -> store waves
      STAMP(6);
    };
    typedef std::integral_constant<bool, false> F_;
    typedef std::integral_constant<bool, true> T_;
    // two steps (maps 0 and 1) per iteration; AB is even, so both lie in one action block
    const auto run = [&](auto ar_c) __attribute__((always_inline)) {
      for (int s = 0; s < T; s += 2) {
        if ((s & (AB - 1)) == 0) unpack_block(s);
        if (blk_bad) step(F_{}, ar_c, T_{}, s);
        else step(F_{}, ar_c, F_{}, s);
        if (s + 1 < T) {
          if (blk_bad) step(T_{}, ar_c, T_{}, s + 1);
          else step(T_{}, ar_c, F_{}, s + 1);
        }
      }
    };
    if (a.autoreset) run(T_{});
    else run(F_{});
    ((int2*)a.pos)[oa] = cell_rc(cur);
    a.done[oa] = dn ? 1 : 0;
    if (a.steps) a.steps[oa] = st;
    if (ag == 0) a.t[env] = tcur;
    split_barrier();  // barrier T + 1: the store waves' last fold (split_store_wave_dbm)
    return;
  }

  for (int s = 0; s < T; ++s) {
    const int act = next_action(s);
    STAMP(0);
    // ---------------- A: move decision on the PRE-step map (:319-342) ----------------
    const int oc = cur;
    const bool mv = !dn && (uint32_t)act < 4u;  // 4 = stay, 0xFF = invalid (!has: 4)
    const uint32_t v = mv ? ((nb >> ((act & 3) * 8)) & 0xFFu) : 0u;  // pre-step cell (flag | c)
    const bool envc = mv && (v & 0x7Fu) == 0u;  // out of bounds / free-standing obstacle (quirk 1)
    const bool skip = !do_step || ((__ballot(act == 0xFF) & envmask) != 0);
    const bool moved = mv && (v & 0x7Fu) != 0u && !skip;
    int dlt = (act & 2) ? 1 : pitch;  // 0: up, 1: down, 2: left, 3: right
    dlt = (act & 1) ? dlt : -dlt;
    const int nc = moved ? oc + dlt : oc;
    if (has) dep[oc] = (unsigned char)(moved ? (uint32_t)act : 0x7Fu);
    {
      if (FULLW) {  // branch-free: lanes that stay add 0 to their own cell's word
        atomicAdd(&map32[oc >> 2], moved ? 0u - (1u << ((oc & 3) * 8)) : 0u);
        atomicAdd(&map32[nc >> 2], moved ? 1u << ((nc & 3) * 8) : 0u);
      } else if (moved) {
        atomicSub(&map32[oc >> 2], 1u << ((oc & 3) * 8));
        atomicAdd(&map32[nc >> 2], 1u << ((nc & 3) * 8));
      }
    }
    cur = nc;
    STAMP(2);
    // ---------------- B: issue step s's rows, occupant move, fold of step s-2 -------
    uint32_t x[3 * NX];
    if constexpr (WIN > 0) {
      const int w0 = (nc - H2 * pitch - H2) >> 2;
      const int wpr = pitch >> 2;
#pragma unroll
      for (int y = 0; y < WIN; ++y) {
        x[y] = map32[w0 + y * wpr];
        x[WIN + y] = map32[w0 + y * wpr + 1];
        x[2 * WIN + y] = WIN > 5 ? map32[w0 + y * wpr + 2] : 0u;
      }
    } else {
      x[0] = map[nc];  // centre (node), then up / down / left / right
      x[1] = map[nc - pitch];
      x[2] = map[nc + pitch];
    }
    uint32_t xl = 0, xr = 0;
    if constexpr (WIN == 0) {
      xl = map[nc - 1];
      xr = map[nc + 1];
    }
    const uint32_t dj = dep[nc];  // pre-step occupant's move
    const double Rp = (ROLL && do_step) ? fold(s & 1) : 0.0;  // step s-2's row
    STAMP(1);
    // ---------------- C: heavy part of step s-1, env outputs of step s-2 -----------
    if (s > 0) heavy(s - 1);
    if (ROLL && s > 1) tail(s & 1, p_se, p_skip, p_alldone, p_tcur, Rp);
    STAMP(3);
    // ---------------- D: step s's neighbours, dones, t (:112-117) ----------------
    uint32_t nbn;
    if constexpr (WIN > 0) {
      // the 4 neighbours lie in the first 8 bytes of their window rows (o + H2 + 1 <= 7)
      const int o8 = ((nc - H2) & 3) * 8;
      const auto row64 = [&](int y) { return ((uint64_t)x[WIN + y] << 32) | x[y]; };
      const uint32_t up = (uint32_t)(row64(H2 - 1) >> (o8 + 8 * H2)) & 0xFFu;
      const uint32_t dw = (uint32_t)(row64(H2 + 1) >> (o8 + 8 * H2)) & 0xFFu;
      const uint32_t cr = (uint32_t)(row64(H2) >> (o8 + 8 * (H2 - 1)));  // left, centre, right
      nbn = up | (dw << 8) | ((cr & 0xFFu) << 16) | (((cr >> 16) & 0xFFu) << 24);
    } else {
      nbn = (x[1] & 0xFFu) | ((x[2] & 0xFFu) << 8) | ((xl & 0xFFu) << 16) | ((xr & 0xFFu) << 24);
    }
    const bool dn_old = dn;
    const bool live = !skip;
    if (live && nc == gcell) dn = true;          // :112-114 (goal reached)
    if (live && tcur + 1 >= g.limit) dn = true;  // :116-117 (t is incremented below)
    if (live && !dn_old) ++st;
    if (!skip) ++tcur;
    const bool alldone = (__ballot(has && !dn) & envmask) == 0;
    if (!RUNNER && a.obs_full && env_ok) {  // :143-192, row-major occ = count - flag (now:
      // the next step's atomics would change the map)
      const uint32_t se = ROLL ? (uint32_t)s * (uint32_t)g.E : 0u;
      unsigned char* outb = (unsigned char*)a.obs_full + (size_t)(se + env) * g.H * Wd;
      if ((Wd & 3) == 0) {
        const int wpr_out = Wd >> 2;
        const int nwords = g.H * wpr_out;
        for (int i = ag; i < nwords; i += L) {
          const int rr_ = fastdiv(i, g.m_W4);
          const int cw = i - rr_ * wpr_out;
          const uint32_t vv = map32[((rr_ + g.P) * pitch + g.pl) / 4 + cw];
          ((uint32_t*)outb)[i] = (((vv & 0x7F7F7F7Fu) | 0x80808080u) - 0x01010101u) ^ 0x80808080u;  // c - 1
        }
      } else {
        for (int i = ag; i < g.H * Wd; i += L) {
          const int rr_ = fastdiv(i, g.m_W);
          const int cc_ = i - rr_ * Wd;
          ((int8_t*)outb)[i] = (int8_t)((int)(map[(rr_ + g.P) * pitch + cc_ + g.pl] & 0x7F) - 1);
        }
      }
    }
    // save step s for its heavy part / tail
    p_se = ROLL ? (uint32_t)(s - 1) * (uint32_t)g.E : 0u;
    p_skip = q_skip;
    p_alldone = q_alldone;
    p_tcur = q_tcur;
#pragma unroll
    for (int i = 0; i < 3 * NX; ++i) qx[i] = x[i];
    q_oc = oc;
    q_nc = nc;
    q_act = act;
    q_pre = (int)(v & 0x7Fu) - 1 + (int)(v >> 7);  // pre-step occupants of cand (moved lanes)
    q_dj = dj;
    q_nb = nbn;
    q_moved = moved;
    q_envc = envc;
    q_dnold = dn_old;
    q_dn = dn;
    q_live = live;
    q_skip = skip;
    q_alldone = alldone;
    q_tcur = tcur;
    nb = nbn;
    if (ROLL && a.autoreset && alldone) {
      if (has) {
        const int2 p = ((const int2*)a.init_pos)[oa];
        const int ncell = cell0 + p.x * pitch + p.y;
        atomicSub(&map32[cur >> 2], 1u << ((cur & 3) * 8));
        atomicAdd(&map32[ncell >> 2], 1u << ((ncell & 3) * 8));
        cur = ncell;
        dn = false;
        st = 0;
      }
      tcur = 0;
      wave_fence();
      if (has) {
        nb = (uint32_t)map[cur - pitch] | ((uint32_t)map[cur + pitch] << 8) |
             ((uint32_t)map[cur - 1] << 16) | ((uint32_t)map[cur + 1] << 24);
      }
    }
    STAMP(4);
    wave_fence();
    STAMP(6);
  }
  // ---- drain the pipeline: heavy part of the last step, the last two tails ----
  if (T > 0) {
    const double Rp = (ROLL && T > 1) ? fold(T & 1) : 0.0;  // step T-2's row
    heavy(T - 1);
    if (ROLL && T > 1) tail(T & 1, p_se, p_skip, p_alldone, p_tcur, Rp);
    wave_fence();
    const int lb = ROLL ? ((T - 1) & 1) : 0;
    const double Rl = do_step ? fold(lb) : 0.0;
    tail(lb, ROLL ? (uint32_t)(T - 1) * (uint32_t)g.E : 0u, q_skip, q_alldone, q_tcur, Rl);
  }
  if (has) {
    ((int2*)a.pos)[oa] = cell_rc(cur);
    a.done[oa] = dn ? 1 : 0;
    if (a.steps) a.steps[oa] = st;
  }
  if (env_ok && ag == 0) a.t[env] = tcur;
  PSTAMP(4);
#ifdef MAPFX_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  PSTAMP(5);
#endif
}

// One env step (mapfx_step) or an observation pass (mapfx_observe, do_step = 0).
template <typename CellT, int APL, int FEAT>
__global__ void __launch_bounds__(256) mapf_step_kernel(MAPFX_HOT_PARAMS, Args a0, Geo g0) {
  Args a = a0;
  Geo g = g0;
  MAPFX_HOT_APPLY(a, g);
  step_body<CellT, APL, false, FEAT>(g, a);
}

// T fused env steps (mapfx_rollout); state stays in LDS / registers between steps.
template <typename CellT, int APL, int FEAT>
__global__ void __launch_bounds__(256) mapf_rollout_kernel(MAPFX_HOT_PARAMS, Args a0, Geo g0) {
  Args a = a0;
  Geo g = g0;
  MAPFX_HOT_APPLY(a, g);
  step_body<CellT, APL, true, FEAT>(g, a);
}

__global__ void reset_kernel(int E, int N, int32_t* pos, const int32_t* init_pos, uint8_t* done,
                             int32_t* t, int32_t* steps, const uint8_t* mask) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)E * N) return;
  const long long e = i / N;
  if (mask && !mask[e]) return;
  ((int2*)pos)[i] = ((const int2*)init_pos)[i];
  done[i] = 0;
  if (steps) steps[i] = 0;
  if (i % N == 0) t[e] = 0;
}

__global__ void gen_actions_kernel(long long total, int E, int N, long long env_offset,
                                   uint64_t seed, int t0, int8_t* out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long long en = (long long)E * N;
  const int tt = (int)(i / en);
  const long long rem = i - (long long)tt * en;
  const long long e = rem / N;
  const int ag = (int)(rem - e * N);
  out[i] = (int8_t)gen_action(seed, env_offset + e, t0 + tt, ag);
}

// Compact gather payload (mapfx_pack_compact): every agent-step's (row, col) as the
// u16 cell index row * W + col, and the dones as bits.  Thread i owns agent-step i
// of the [T][E][N] trajectory (coalesced 8-B reads, 2-B writes); the thread of agent
// 8k of an env-step packs the done bytes of agents 8k..8k+7 (L1 hits: its neighbours
// read the same line) into bit 0..7 of that env-step's byte k.
__global__ void pack_compact_kernel(long long total, int N, int W, int nbytes, const int2* traj_pos,
                                    const uint8_t* traj_done, uint16_t* cell, uint8_t* done_bits) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int2 p = traj_pos[i];
  cell[i] = (uint16_t)(p.x * W + p.y);
  const long long es = i / N;
  const int ag = (int)(i - es * N);
  if ((ag & 7) == 0) {
    uint32_t b = 0;
    const int m = min(8, N - ag);
    for (int k = 0; k < m; ++k) b |= (traj_done[i + k] ? 1u : 0u) << k;
    done_bits[es * nbytes + (ag >> 3)] = (uint8_t)b;
  }
}

int round_up(int x, int m) { return (x + m - 1) / m * m; }

uint64_t magic48(int d) { return ((1ull << 48) + (uint64_t)d - 1) / (uint64_t)d; }

}  // namespace

struct mapfx_t {
  mapfx_cfg cfg;
  Geo geo;
  int cell_bytes;
  int APL;
  double* pow_lut;  // device
  int lut_len;
  int device;
};

namespace {

using KernelFn = void (*)(int32_t*, const int32_t*, uint8_t*, const uint8_t*, const void*, int32_t*,
                          uint32_t, uint32_t, Args, Geo);

template <typename CellT, int FEAT>
KernelFn pick_kernel_cf(int apl, bool roll) {
  if (roll) {
    if (apl == 1) return mapf_rollout_kernel<CellT, 1, FEAT>;
    if (apl == 2) return mapf_rollout_kernel<CellT, 2, FEAT>;
    return mapf_rollout_kernel<CellT, 4, FEAT>;
  }
  if (apl == 1) return mapf_step_kernel<CellT, 1, FEAT>;
  if (apl == 2) return mapf_step_kernel<CellT, 2, FEAT>;
  return mapf_step_kernel<CellT, 4, FEAT>;
}

// rollouts with exactly the runner output set
template <typename CellT>
KernelFn pick_kernel_run(int apl) {
  if (apl == 1) return mapf_rollout_kernel<CellT, 1, FEAT_RUN>;
  if (apl == 2) return mapf_rollout_kernel<CellT, 2, FEAT_RUN>;
  return mapf_rollout_kernel<CellT, 4, FEAT_RUN>;
}

// feat: 0 (window / avail / rewards), FEAT_FULL, FEAT_FULL | FEAT_PRIM, or FEAT_RUN (rollouts)
template <typename CellT>
KernelFn pick_kernel_c(int apl, bool roll, int feat) {
  if ((feat & FEAT_RUN) && roll) return pick_kernel_run<CellT>(apl);
  if (feat & FEAT_PRIM) return pick_kernel_cf<CellT, FEAT_FULL | FEAT_PRIM>(apl, roll);
  if (feat & FEAT_FULL) return pick_kernel_cf<CellT, FEAT_FULL>(apl, roll);
  return pick_kernel_cf<CellT, 0>(apl, roll);
}

KernelFn pick_kernel(int cell_bytes, int apl, bool roll, int feat) {
  return cell_bytes == 1 ? pick_kernel_c<uint8_t>(apl, roll, feat)
                         : pick_kernel_c<uint16_t>(apl, roll, feat);
}

int check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) return set_error(MAPFX_EHIP, "%s: %s", what, hipGetErrorString(e));
  return MAPFX_OK;
}


constexpr int MAPFX_AB_SHORT_T = 32;
template <int WIN>
KernelFn pick_wave_win(bool roll, bool fullw, bool runner, int L, bool split, bool occ, bool short_t) {
  if (occ) {  // obs_window_occ: only the store-wave split writes it on the wave path
    if constexpr (WIN > 0) {
      if (roll && runner && split && fullw && L == 16)
        return short_t ? mapf_wave_kernel<WIN, true, true, true, 16, true, true, 8>
                       : mapf_wave_kernel<WIN, true, true, true, 16, true, true>;
      if (roll && runner && split && fullw && L == 64)
        return short_t ? mapf_wave_kernel<WIN, true, true, true, 64, true, true, 8>
                       : mapf_wave_kernel<WIN, true, true, true, 64, true, true>;
    }
    return nullptr;
  }
  if (roll) {
    if (runner) {
      if constexpr (WIN > 0) {
        if (split && fullw && L == 16)
          return short_t ? mapf_wave_kernel<WIN, true, true, true, 16, true, false, 8>
                         : mapf_wave_kernel<WIN, true, true, true, 16, true>;
        if (split && fullw && L == 64)
          return short_t ? mapf_wave_kernel<WIN, true, true, true, 64, true, false, 8>
                         : mapf_wave_kernel<WIN, true, true, true, 64, true>;
      }
      if (!fullw) return mapf_wave_kernel<WIN, true, false, true, 0>;
      if (L == 16) return mapf_wave_kernel<WIN, true, true, true, 16>;
      if (L == 64) return mapf_wave_kernel<WIN, true, true, true, 64>;
      return mapf_wave_kernel<WIN, true, true, true, 0>;
    }
    return fullw ? mapf_wave_kernel<WIN, true, true, false, 0> : mapf_wave_kernel<WIN, true, false, false, 0>;
  }
  if (fullw && L == 16) return mapf_wave_kernel<WIN, false, true, false, 16>;
  return fullw ? mapf_wave_kernel<WIN, false, true, false, 0> : mapf_wave_kernel<WIN, false, false, false, 0>;
}

KernelFn pick_wave_kernel(int win, bool roll, bool fullw, bool runner, int L, bool split, bool occ, bool short_t) {
  switch (win) {
    case 0: return pick_wave_win<0>(roll, fullw, runner, L, split, occ, short_t);
    case 3: return pick_wave_win<3>(roll, fullw, runner, L, split, occ, short_t);
    case 5: return pick_wave_win<5>(roll, fullw, runner, L, split, occ, short_t);
    case 7: return pick_wave_win<7>(roll, fullw, runner, L, split, occ, short_t);
  }
  return nullptr;
}

int launch(mapfx_t* h, Args& a, bool roll, hipStream_t stream, hipEvent_t ev0 = nullptr,
           hipEvent_t ev1 = nullptr) {
  const Geo& g = h->geo;
  if (g.E == 0) return MAPFX_OK;
  // wave-local fast path: N <= 64, no PRIMAL output, window 3/5/7 (or none)
  const long long slot_elems = (long long)(roll ? a.T : 1) * g.E * g.N;
  const bool fits32 = slot_elems * std::max(8, 2 * g.window * g.window) < (1ll << 31) &&
                      (long long)(roll ? a.T : 1) * g.E * g.H * g.W < (1ll << 31);
  if (g.wave_ok && fits32 && !a.obs_primal && !a.primal_vec && !(a.obs_window && a.obs_window_occ)) {
    const bool fullw = g.N == g.L && g.E % g.EPW == 0;
    const bool occ = a.obs_window_occ != nullptr;
    const bool runner = roll && a.reward && a.term && a.node && a.edge && a.avail &&
                        a.traj_pos && a.traj_done && a.traj_t && (a.obs_window || occ) && !a.obs_full;
    const uintptr_t al16 = (uintptr_t)a.obs_window | (uintptr_t)a.obs_window_occ | (uintptr_t)a.traj_pos |
                           (uintptr_t)a.node | (uintptr_t)a.edge | (uintptr_t)a.avail |
                           (uintptr_t)a.traj_done | (uintptr_t)a.reward | (uintptr_t)a.traj_t;
    // the split's LDS: M1 (the odd steps' maps of the wave's envs), info + edge rings, the
    // two store waves' staged records, the reward-code table and ring
    const int split_lds = g.wv_lds + g.EPW * g.map_env_bytes + SPLIT_DBM_INFO + SPLIT_DBM_EDGE +
                          2 * 64 * (occ ? g.wlen / 2 : g.wlen) + split_fold_lds(g.L);
    const bool split = runner && fullw && (g.L == 16 || g.L == 64) && g.wv_split_ok &&
                       split_lds <= 64 * 1024 && (al16 & 15) == 0;
    KernelFn fn = pick_wave_kernel((a.obs_window || occ) ? g.window : 0, roll, fullw, runner, g.L, split, occ,
                                   roll && a.T <= MAPFX_AB_SHORT_T);
    if (fn) {
      const int blocks = (g.E + g.EPW - 1) / g.EPW;
      const dim3 bt(split ? 64 * SPLIT_WAVES : 64);
      const unsigned ldsb = split ? split_lds : g.wv_lds;
      if (ev0 || ev1)
        hipExtLaunchKernelGGL(fn, dim3(blocks), bt, ldsb, stream, ev0, ev1, 0, MAPFX_HOT_ARGS(a, g, blocks), a, g);
      else
        hipLaunchKernelGGL(fn, dim3(blocks), bt, ldsb, stream, MAPFX_HOT_ARGS(a, g, blocks), a, g);
      g_last_kernel = (const void*)fn;
      return check_hip(hipGetLastError(), "mapf_wave_kernel launch");
    }
  }
  int feat = (a.obs_primal || a.primal_vec) ? (FEAT_FULL | FEAT_PRIM) : a.obs_full ? FEAT_FULL : 0;
  if (roll && feat == 0 && a.reward && a.term && a.node && a.edge && a.avail && a.traj_pos && a.traj_done &&
      a.traj_t && (a.obs_window || a.obs_window_occ) && !a.reward_f32)
    feat = FEAT_RUN;  // the runner output set: the per-output tests compile away
  KernelFn fn = pick_kernel(h->cell_bytes, h->APL, roll, feat);
  const int blocks = (g.E + g.EPB - 1) / g.EPB;
  const int lds = g.gen_lds;
  if (ev0 || ev1)
    hipExtLaunchKernelGGL(fn, dim3(blocks), dim3(g.BT), lds, stream, ev0, ev1, 0, MAPFX_HOT_ARGS(a, g, blocks), a, g);
  else
    hipLaunchKernelGGL(fn, dim3(blocks), dim3(g.BT), lds, stream, MAPFX_HOT_ARGS(a, g, blocks), a, g);
  g_last_kernel = (const void*)fn;
  return check_hip(hipGetLastError(), roll ? "mapf_rollout_kernel launch" : "mapf_step_kernel launch");
}

void fill_state_args(Args& a, const mapfx_state* st) {
  a.pos = st->pos;
  a.goal = st->goal;
  a.init_pos = st->init_pos;
  a.done = st->done;
  a.t = st->t;
  a.steps = st->steps;
  a.bits = st->map_bits;
}

void fill_out_args(Args& a, const mapfx_out* o) {
  if (!o) return;
  a.reward = o->reward;
  a.reward_f32 = o->reward_f32;
  a.term = o->term;
  a.node = o->node;
  a.edge = o->edge;
  a.avail = o->avail;
  a.obs_full = o->obs_full;
  a.obs_window = o->obs_window;
  a.obs_window_occ = o->obs_window_occ;
  a.obs_primal = o->obs_primal;
  a.primal_vec = o->primal_vec;
  a.traj_pos = o->traj_pos;
  a.traj_done = o->traj_done;
  a.traj_t = o->traj_t;
  a.err = o->err;
}

int check_state(const mapfx_t* h, const mapfx_state* st, bool need_init) {
  if (!st) return set_error(MAPFX_EINVAL, "state is NULL");
  if (h->geo.E == 0) return MAPFX_OK;  // an empty shard: every call is a no-op (empty tensors: NULL)
  if (!st->pos || !st->goal || !st->done || !st->t || !st->map_bits)
    return set_error(MAPFX_EINVAL, "state: pos/goal/done/t/map_bits must be non-NULL");
  if (need_init && !st->init_pos) return set_error(MAPFX_EINVAL, "state: init_pos is NULL");
  return MAPFX_OK;
}

int check_out(const mapfx_t* h, const mapfx_out* o) {
  if (!o) return MAPFX_OK;
  const int m = h->cfg.obs_mode;
  if (o->obs_full && !(m & MAPFX_OBS_FULL))
    return set_error(MAPFX_EINVAL, "obs_full requested but MAPFX_OBS_FULL not in cfg.obs_mode");
  if ((o->obs_window || o->obs_window_occ) && !(m & MAPFX_OBS_WINDOW))
    return set_error(MAPFX_EINVAL, "obs_window requested but MAPFX_OBS_WINDOW not in cfg.obs_mode");
  if ((o->obs_primal || o->primal_vec) && !(m & MAPFX_OBS_PRIMAL))
    return set_error(MAPFX_EINVAL, "PRIMAL obs requested but MAPFX_OBS_PRIMAL not in cfg.obs_mode");
  return MAPFX_OK;
}

}  // namespace

extern "C" {

int mapfx_abi_version(void) { return MAPFX_ABI_VERSION; }

#ifndef MAPFX_BUILD_ID
#define MAPFX_BUILD_ID "src=unknown git=unknown"
#endif
const char* mapfx_build_id(void) { return MAPFX_BUILD_ID; }

void mapfx_note_kernel(const void* fn) { g_last_kernel = fn; }

const char* mapfx_last_kernel(void) {
  thread_local std::string name;
  thread_local const void* named = nullptr;
  if (!g_last_kernel) return "";
  if (named != g_last_kernel) {
    const char* raw = hipKernelNameRefByPtr(g_last_kernel, nullptr);
    name = raw ? raw : "";
    if (raw && raw[0] == '_' && raw[1] == 'Z') {
      int status = 0;
      char* dem = abi::__cxa_demangle(raw, nullptr, nullptr, &status);
      if (status == 0 && dem) name = dem;
      free(dem);
    }
    named = g_last_kernel;
  }
  return name.c_str();
}

// error hook for the other translation unit of the library (partial.hip)
int mapfx_internal_error(int code, const char* msg) { return set_error(code, "%s", msg); }

#ifdef MAPFX_STAMPS
int mapfx_debug_stamps(unsigned long long* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 256 * 8) ==
                 hipSuccess ? 0 : -1;
}
#endif

const char* mapfx_last_error(void) { return g_last_error.c_str(); }

int64_t mapfx_map_stride(int32_t H, int32_t W) {
  const int64_t bytes = ((int64_t)H * W + 7) / 8;
  return (bytes + 15) / 16 * 16;
}

int32_t mapfx_obs_elem_size(int32_t n_agents) { return n_agents <= 127 ? 1 : 2; }

int32_t mapfx_edge_elem_size(int32_t n_agents) { return n_agents <= 256 ? 1 : 2; }

int32_t mapfx_action(uint64_t seed, int64_t env, int32_t t, int32_t agent) {
  return gen_action(seed, env, t, agent);
}

int mapfx_create(const mapfx_cfg* cfg, mapfx_t** out_handle) {
  if (!cfg || !out_handle) return set_error(MAPFX_EINVAL, "NULL cfg/out_handle");
  *out_handle = nullptr;
  const mapfx_cfg& c = *cfg;
  if (c.H < 1 || c.W < 1 || c.H > 4096 || c.W > 4096)
    return set_error(MAPFX_EINVAL, "grid %dx%d out of range", c.H, c.W);
  if (c.n_agents < 1 || c.n_agents > 1024)
    return set_error(MAPFX_EINVAL, "n_agents %d not in 1..1024", c.n_agents);
  if (c.n_envs < 0 || c.n_envs >= (1 << 26))  // the grid size travels in 26 bits (MAPFX_HOT_ARGS)
    return set_error(MAPFX_EINVAL, "n_envs %d not in 0..2^26-1", c.n_envs);
  if ((c.obs_mode & MAPFX_OBS_WINDOW) && (c.window < 1 || c.window > 63))
    return set_error(MAPFX_EINVAL, "window %d not in 1..63", c.window);
  if ((c.obs_mode & MAPFX_OBS_PRIMAL) && (c.primal_size < 1 || c.primal_size > 11))
    return set_error(MAPFX_EINVAL, "primal_size %d not in 1..11", c.primal_size);
  if (c.H >= 32768 || c.W >= 32768) return set_error(MAPFX_EINVAL, "grid too large");

  mapfx_t* h = new (std::nothrow) mapfx_t();
  if (!h) return set_error(MAPFX_ENOMEM, "host allocation failed");
  h->cfg = c;
  h->pow_lut = nullptr;
  h->lut_len = 0;
  if (hipGetDevice(&h->device) != hipSuccess) h->device = 0;

  Geo& g = h->geo;
  memset(&g, 0, sizeof(g));
  const int N = c.n_agents;
  const int es = mapfx_obs_elem_size(N);
  h->cell_bytes = es;
  int L = 1;
  while (L < N && L < 256) L <<= 1;
  int lshift = 0;
  while ((1 << lshift) < L) ++lshift;
  const int APL = (N + L - 1) / L;
  h->APL = APL <= 1 ? 1 : (APL <= 2 ? 2 : 4);

  int P = 1;
  if (c.obs_mode & MAPFX_OBS_WINDOW) {
    P = std::max(P, c.window / 2);
    P = std::max(P, c.window - 1 - c.window / 2);
  }
  if (c.obs_mode & MAPFX_OBS_PRIMAL) {
    P = std::max(P, c.primal_size / 2);
    P = std::max(P, c.primal_size - 1 - c.primal_size / 2);
  }
  const int cpw = 4 / es;  // cells per u32 word
  const int pl = round_up(P, cpw);
  // u8 maps (the wave kernels): rows 8-byte aligned for the ds_write_b64 builds, left
  // and right pads apart.  u16 maps (generic kernel only): the right pad of row r is
  // the left pad of row r + 1 (pitch - W >= pl >= P cells between two rows' interiors),
  // plus a tail of pl + P cells after the last row.
  const int pitch = es == 1 ? round_up(pl + c.W + P, 8 / es) : round_up(c.W + pl, cpw);
  const int rows = c.H + 2 * P;
  const int tail = es == 1 ? 0 : pl + P;

  g.H = c.H;
  g.W = c.W;
  g.N = N;
  g.E = c.n_envs;
  g.env_offset = c.env_offset;
  g.L = L;
  g.lshift = lshift;
  g.P = P;
  g.pl = pl;
  g.pitch = pitch;
  g.rows = rows;
  g.wpr = pitch / cpw;
  g.map_words = (rows * pitch + tail + cpw - 1) / cpw;
  g.m_wpr = magic48(g.wpr);
  g.m_W = magic48(c.W);
  g.m_W4 = magic48(std::max(1, c.W / 4));
  g.m_pitch = magic48(pitch);
  g.m_pitch24 = (uint32_t)(((1u << 24) + pitch - 1) / pitch);
  g.bits_words = (int)(((int64_t)c.H * c.W + 31) / 32);
  g.map_stride = mapfx_map_stride(c.H, c.W);
  g.map_shared = c.map_shared ? 1 : 0;
  g.map_env_bytes = round_up(g.map_words * 4, 16);
  g.bits_env_bytes = round_up(g.bits_words * 4, 16);
  g.window = c.window;
  g.wlen = 2 * c.window * c.window;
  g.psize = c.primal_size;
  g.obs_mode = c.obs_mode;
  g.limit = c.episode_limit;
  g.step_rew = c.step_reward;
  g.collide_rew = c.collide_reward;
  g.m_N = magic48(N);
  g.m_w = magic48(std::max(1, c.window));
  g.m_ww = magic48(std::max(1, c.window * c.window));
  g.m_wlen = magic48(std::max(1, g.wlen));
  const bool prim_arrays = (c.obs_mode & MAPFX_OBS_PRIMAL) != 0;

  if ((int64_t)c.H * c.W >= (1ll << 31) / 8 || g.map_words >= (1 << 30)) {
    delete h;
    return set_error(MAPFX_EINVAL, "grid too large");
  }

  // generic block: maps | oldc | newc | [rc | goal: PRIMAL only] | bits == rew | flags
  auto lds_for = [&](int epb) {
    int off = 0;
    off += epb * g.map_env_bytes;
    off += (prim_arrays ? 4 : 2) * round_up(epb * N * 4, 16);
    off += std::max(epb * g.bits_env_bytes, round_up(epb * N * 8, 16));
    off += round_up(epb * 12 * 4, 16);
    return off;
  };
  int EPB = 256 / L;
  const int LDS_TARGET = 48 * 1024;
  const int LDS_MAX = 160 * 1024;
  while (EPB > 1 && lds_for(EPB) > LDS_TARGET) --EPB;
  if (lds_for(EPB) > LDS_MAX) {
    delete h;
    return set_error(MAPFX_EINVAL, "one env needs %d B of LDS (> %d)", lds_for(1), LDS_MAX);
  }
  g.EPB = EPB;
  g.BT = EPB * L;
  int off = 0;
  g.off_map = off;
  off += EPB * g.map_env_bytes;
  g.off_oldc = off;
  off += round_up(EPB * N * 4, 16);
  g.off_newc = off;
  off += round_up(EPB * N * 4, 16);
  g.off_rc = g.off_goal = -1;
  if (prim_arrays) {
    g.off_rc = off;
    off += round_up(EPB * N * 4, 16);
    g.off_goal = off;
    off += round_up(EPB * N * 4, 16);
  }
  g.off_bits = g.off_rew = off;  // the bitmap is dead once the map is built
  const int rew_bytes = std::max(EPB * g.bits_env_bytes, round_up(EPB * N * 8, 16));
  off += rew_bytes;
  g.off_flag = off;
  off += round_up(EPB * 12 * 4, 16);
  g.gen_lds = off;
  // Deferred fold (rollouts with one env per block): the ring of FOLD_R code rows
  // replaces the fp64 reward row, and is kept only when the block count per CU stays.
  g.fold_R = 0;
  g.code_pitch = round_up(2 * N, 16) + 16;  // +16 B: the fold lanes' rows start on other banks
  g.off_ctab = -1;
  if (MAPFX_FOLD_R > 0 && EPB == 1 && L >= 64 && std::isfinite(c.step_reward) && std::isfinite(c.collide_reward)) {
    constexpr int FOLD_R = MAPFX_FOLD_R;
    const int ring = std::max(rew_bytes, FOLD_R * g.code_pitch);
    const int lds_f = g.gen_lds - rew_bytes + ring + 32 * 8 + FOLD_R * 4;
    if (LDS_MAX / lds_f >= LDS_MAX / g.gen_lds) {
      g.fold_R = FOLD_R;
      g.off_flag = g.off_rew + ring;
      g.off_ctab = g.off_flag + round_up(EPB * 12 * 4, 16);
      g.gen_lds = lds_f;  // step launches share the layout (the ring is unused there)
    }
  }

  // wave-local fast path layout (one wavefront = EPW envs)
  g.wave_ok = 0;
  if (L <= 64 && es == 1) {
    const int EPW = 64 / L;
    g.EPW = EPW;
    g.wv_bits_env_bytes = round_up(g.bits_words * 4 + 4, 16);
    g.wv_fast = (c.W <= 64 && g.wpr <= MAPFX_FAST_WPR && (g.wpr & 1) == 0 && pl >= 1 && pl <= 32) ? 1 : 0;
    int o = 0;
    g.wv_off_map = o;
    o += EPW * g.map_env_bytes;
    g.wv_off_dep = o;
    o += EPW * g.map_env_bytes;
    g.wv_off_bits = o;
    // the fast build reads the bitmap words of its rows straight from global memory (one
    // wide load per lane staged in LDS measured slower: per-step 5.04 -> 6.25 us, C2 T = 20
    // 21.7 -> 23.8 us, gpurun_out/r05c)
    o += g.wv_fast ? 0 : EPW * g.wv_bits_env_bytes;
    // rew rows: one double per LANE of the env (every lane writes its slot, +0.0 past
    // N, and the L = 16 fold reads all 16), rounded up to 2 (16 B), +2 doubles so the
    // envs of a wave start on different banks
    const int rew_base = std::max((N + 1) / 2 * 2, L);
    g.wv_rew_row = rew_base + ((rew_base % 16) == 0 ? 2 : 0);
    g.wv_rew_buf = round_up(EPW * g.wv_rew_row * 8, 16);
    g.wv_off_rew = o;
    o += 2 * g.wv_rew_buf;
    g.wv_lds = o;
    // the store-wave split's LDS (after the wave layout; only that kernel allocates it)
    g.wv_off_split = o;
    g.wv_split_ok = ((L == 16 || L == 64) && (c.window == 3 || c.window == 5 || c.window == 7)) ? 1 : 0;
    g.wave_ok = (o <= 64 * 1024 && pitch < 256 && g.rows * pitch < 65536) ? 1 : 0;
  }

  const int lds_total = g.gen_lds;
  if (lds_total > 64 * 1024) {
    hipError_t e = hipSuccess;
    const int feats[4] = {0, FEAT_FULL, FEAT_FULL | FEAT_PRIM, FEAT_RUN};
    for (int roll = 0; roll < 2 && e == hipSuccess; ++roll)
      for (int fi = 0; fi < 4 && e == hipSuccess; ++fi)
        e = hipFuncSetAttribute((const void*)pick_kernel(es, h->APL, roll != 0, feats[fi]),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds_total);
    if (e != hipSuccess) {
      delete h;
      return set_error(MAPFX_EHIP, "hipFuncSetAttribute(LDS=%d): %s", lds_total,
                       hipGetErrorString(e));
    }
  }

  if (c.obs_mode & MAPFX_OBS_PRIMAL) {
    // mag = (dx**2 + dy**2) ** .5 is libm pow, not sqrt (mapf_primal.py:382, quirk 8):
    // tabulate it on the host with the same libm the reference's CPython calls.
    const int n = (c.H - 1) * (c.H - 1) + (c.W - 1) * (c.W - 1) + 1;
    double* lut = (double*)malloc(sizeof(double) * n);
    if (!lut) {
      delete h;
      return set_error(MAPFX_ENOMEM, "host LUT allocation failed");
    }
    // through a volatile pointer: clang would otherwise rewrite pow(x, 0.5) as sqrt(x)
    double (*volatile libm_pow)(double, double) = pow;
    for (int i = 0; i < n; ++i) lut[i] = libm_pow((double)i, 0.5);
    hipError_t e = hipMalloc((void**)&h->pow_lut, sizeof(double) * n);
    if (e == hipSuccess) e = hipMemcpy(h->pow_lut, lut, sizeof(double) * n, hipMemcpyHostToDevice);
    free(lut);
    if (e != hipSuccess) {
      if (h->pow_lut) (void)hipFree(h->pow_lut);
      delete h;
      return set_error(MAPFX_ENOMEM, "pow LUT: %s", hipGetErrorString(e));
    }
    h->lut_len = n;
  }
  *out_handle = h;
  return MAPFX_OK;
}

void mapfx_destroy(mapfx_t* h) {
  if (!h) return;
  if (h->pow_lut) (void)hipFree(h->pow_lut);
  delete h;
}

int mapfx_query(const mapfx_t* h, mapfx_info* info) {
  if (!h || !info) return set_error(MAPFX_EINVAL, "NULL handle/info");
  const Geo& g = h->geo;
  info->lanes_per_env = g.L;
  info->agents_per_lane = (g.N + g.L - 1) / g.L;
  info->envs_per_block = g.EPB;
  info->block_threads = g.BT;
  info->lds_bytes = g.gen_lds;
  info->cell_bytes = h->cell_bytes;
  info->pad = g.P;
  return MAPFX_OK;
}

int mapfx_reset(mapfx_t* h, const mapfx_state* st, const uint8_t* env_mask, const mapfx_out* out,
                void* stream) {
  if (!h) return set_error(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st, true);
  if (rc) return rc;
  if ((rc = check_out(h, out))) return rc;
  const Geo& g = h->geo;
  const long long total = (long long)g.E * g.N;
  if (total > 0) {
    const int bt = 256;
    hipLaunchKernelGGL(reset_kernel, dim3((unsigned)((total + bt - 1) / bt)), dim3(bt), 0,
                       (hipStream_t)stream, g.E, g.N, st->pos, st->init_pos, st->done, st->t,
                       st->steps, env_mask);
    if ((rc = check_hip(hipGetLastError(), "reset_kernel launch"))) return rc;
  }
  if (out) return mapfx_observe(h, st, out, stream);
  return MAPFX_OK;
}

int mapfx_observe(mapfx_t* h, const mapfx_state* st, const mapfx_out* out, void* stream) {
  if (!h) return set_error(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st, false);
  if (rc) return rc;
  if ((rc = check_out(h, out))) return rc;
  if ((out && (out->obs_primal || out->primal_vec)) && !h->pow_lut)
    return set_error(MAPFX_EINVAL, "PRIMAL LUT missing");
  Args a;
  memset(&a, 0, sizeof(a));
  fill_state_args(a, st);
  if (out) {
    a.term = out->term;
    a.avail = out->avail;
    a.obs_full = out->obs_full;
    a.obs_window = out->obs_window;
    a.obs_window_occ = out->obs_window_occ;
    a.obs_primal = out->obs_primal;
    a.primal_vec = out->primal_vec;
  }
  a.T = 1;
  a.do_step = 0;
  a.pow_lut = h->pow_lut;
  return launch(h, a, false, (hipStream_t)stream);
}

int mapfx_step(mapfx_t* h, const mapfx_state* st, const void* actions, int action_dtype,
               const mapfx_out* out, void* stream) {
  if (!h) return set_error(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st, false);
  if (rc) return rc;
  if ((rc = check_out(h, out))) return rc;
  if (!actions && h->geo.E > 0) return set_error(MAPFX_EINVAL, "NULL actions");
  if (action_dtype < MAPFX_I8 || action_dtype > MAPFX_I64)
    return set_error(MAPFX_EINVAL, "bad action_dtype %d", action_dtype);
  Args a;
  memset(&a, 0, sizeof(a));
  fill_state_args(a, st);
  fill_out_args(a, out);
  a.actions = actions;
  a.act_dtype = action_dtype;
  a.T = 1;
  a.do_step = 1;
  a.pow_lut = h->pow_lut;
  return launch(h, a, false, (hipStream_t)stream);
}

int mapfx_rollout(mapfx_t* h, const mapfx_state* st, int32_t T, const void* actions,
                  int action_dtype, uint64_t seed, int32_t t0, int32_t autoreset,
                  const mapfx_out* traj, void* stream) {
  if (!h) return set_error(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st, autoreset != 0);
  if (rc) return rc;
  if ((rc = check_out(h, traj))) return rc;
  if (T < 0) return set_error(MAPFX_EINVAL, "T < 0");
  if (T == 0) return MAPFX_OK;
  if (actions && (action_dtype < MAPFX_I8 || action_dtype > MAPFX_I64))
    return set_error(MAPFX_EINVAL, "bad action_dtype %d", action_dtype);
  Args a;
  memset(&a, 0, sizeof(a));
  fill_state_args(a, st);
  fill_out_args(a, traj);
  a.actions = actions;
  a.act_dtype = action_dtype;
  a.use_rng = actions ? 0 : 1;
  a.seed = seed;
  a.t0 = t0;
  a.T = T;
  a.autoreset = autoreset ? 1 : 0;
  a.do_step = 1;
  a.pow_lut = h->pow_lut;
  return launch(h, a, true, (hipStream_t)stream);
}

int mapfx_rollout_timed(mapfx_t* h, const mapfx_state* st, int32_t T, const void* actions,
                        int action_dtype, uint64_t seed, int32_t t0, int32_t autoreset,
                        const mapfx_out* traj, void* start_event, void* stop_event, void* stream) {
  if (!h) return set_error(MAPFX_EINVAL, "NULL handle");
  int rc = check_state(h, st, autoreset != 0);
  if (rc) return rc;
  if ((rc = check_out(h, traj))) return rc;
  if (T < 1) return set_error(MAPFX_EINVAL, "T < 1");
  if (actions && (action_dtype < MAPFX_I8 || action_dtype > MAPFX_I64))
    return set_error(MAPFX_EINVAL, "bad action_dtype %d", action_dtype);
  Args a;
  memset(&a, 0, sizeof(a));
  fill_state_args(a, st);
  fill_out_args(a, traj);
  a.actions = actions;
  a.act_dtype = action_dtype;
  a.use_rng = actions ? 0 : 1;
  a.seed = seed;
  a.t0 = t0;
  a.T = T;
  a.autoreset = autoreset ? 1 : 0;
  a.do_step = 1;
  a.pow_lut = h->pow_lut;
  return launch(h, a, true, (hipStream_t)stream, (hipEvent_t)start_event, (hipEvent_t)stop_event);
}

int mapfx_gen_actions(mapfx_t* h, uint64_t seed, int32_t t0, int32_t T, int8_t* out,
                      void* stream) {
  if (!h) return set_error(MAPFX_EINVAL, "NULL handle");
  if (T < 0) return set_error(MAPFX_EINVAL, "T < 0");
  const long long total = (long long)T * h->geo.E * h->geo.N;
  if (total == 0) return MAPFX_OK;
  if (!out) return set_error(MAPFX_EINVAL, "NULL out");
  const int bt = 256;
  hipLaunchKernelGGL(gen_actions_kernel, dim3((unsigned)((total + bt - 1) / bt)), dim3(bt), 0,
                     (hipStream_t)stream, total, h->geo.E, h->geo.N, (long long)h->geo.env_offset,
                     seed, t0, out);
  return check_hip(hipGetLastError(), "gen_actions_kernel launch");
}

int mapfx_pack_compact(mapfx_t* h, int32_t T, const int32_t* traj_pos, const uint8_t* traj_done,
                       uint16_t* cell, uint8_t* done_bits, void* stream) {
  if (!h) return set_error(MAPFX_EINVAL, "NULL handle");
  if (T < 0) return set_error(MAPFX_EINVAL, "T < 0");
  if ((long long)h->cfg.H * h->cfg.W > 65536)
    return set_error(MAPFX_EINVAL, "compact cells are u16: H*W = %lld > 65536",
                     (long long)h->cfg.H * h->cfg.W);
  const long long total = (long long)T * h->geo.E * h->geo.N;
  if (total == 0) return MAPFX_OK;
  if (!traj_pos || !traj_done || !cell || !done_bits) return set_error(MAPFX_EINVAL, "NULL buffer");
  const int bt = 256;
  hipLaunchKernelGGL(pack_compact_kernel, dim3((unsigned)((total + bt - 1) / bt)), dim3(bt), 0,
                     (hipStream_t)stream, total, h->geo.N, h->cfg.W, (h->geo.N + 7) / 8,
                     (const int2*)traj_pos, traj_done, cell, done_bits);
  return check_hip(hipGetLastError(), "pack_compact_kernel launch");
}

}  // extern "C"

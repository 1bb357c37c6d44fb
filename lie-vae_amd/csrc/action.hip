// Host side of the group-action kernels: degree-range planning (segments), launch
// geometry, argument checks and the extern "C" entry points of include/lievae.h.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <array>
#include <atomic>
#include <vector>

#include "action_kernels.h"

namespace lv {
LV_EXTERN_LAUNCHERS(0) LV_EXTERN_LAUNCHERS(1) LV_EXTERN_LAUNCHERS(2) LV_EXTERN_LAUNCHERS(3)
LV_EXTERN_LAUNCHERS(4) LV_EXTERN_LAUNCHERS(5) LV_EXTERN_LAUNCHERS(6) LV_EXTERN_LAUNCHERS(7)
LV_EXTERN_LAUNCHERS(8) LV_EXTERN_LAUNCHERS(9) LV_EXTERN_LAUNCHERS(10) LV_EXTERN_LAUNCHERS(11)
LV_EXTERN_LAUNCHERS(12) LV_EXTERN_LAUNCHERS(13) LV_EXTERN_LAUNCHERS(14) LV_EXTERN_LAUNCHERS(15)
LV_EXTERN_LAUNCHERS(16) LV_EXTERN_LAUNCHERS(17) LV_EXTERN_LAUNCHERS(18) LV_EXTERN_LAUNCHERS(19)
LV_EXTERN_LAUNCHERS(20)
LV_EXTERN_BWD(0) LV_EXTERN_BWD(1) LV_EXTERN_BWD(2) LV_EXTERN_BWD(3) LV_EXTERN_BWD(4)
LV_EXTERN_BWD(5) LV_EXTERN_BWD(6) LV_EXTERN_BWD(7) LV_EXTERN_BWD(8) LV_EXTERN_BWD(9)
LV_EXTERN_BWD(10) LV_EXTERN_BWD(11) LV_EXTERN_BWD(12) LV_EXTERN_BWD(13) LV_EXTERN_BWD(14)
LV_EXTERN_BWD(15) LV_EXTERN_BWD(16) LV_EXTERN_BWD(17) LV_EXTERN_BWD(18) LV_EXTERN_BWD(19)
LV_EXTERN_BWD(20)

// Shared-spectrum gradient: gF[e] = sum over the tile kernel's slabs.  (Round-2 kernel,
// kept for A/B as LV_BWD_REDUCE=1; action_bwd_reduce2_kernel below is the default.)  One block per
// kBwdReduceCols consecutive elements, lane = (slab stream k, column); the block's 16
// waves split the slabs into contiguous runs, and inside a run stream k takes every
// kBwdReduceStreams-th slab (64-byte loads, unrolled).  Against one element per lane this
// is 4x fewer serial loads per lane and 4x the blocks (76 at l = 10, C = 10): 5.1 -> 4.4 us
// at batch 4096.  Partials are added in a fixed order (run, then stream): deterministic.
#ifndef LV_REDUCE_COLS
#define LV_REDUCE_COLS 16
#endif
constexpr int kBwdReduceCols = LV_REDUCE_COLS;
constexpr int kBwdReduceStreams = 64 / kBwdReduceCols;
__global__ __launch_bounds__(64 * kBwdReduceWaves) void action_bwd_reduce_kernel(
    const float* ws_F, float* gF, int64_t MC, int nslab) {
  __shared__ float part[kBwdReduceWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int k = lane / kBwdReduceCols, col = lane - k * kBwdReduceCols;
  const int64_t e = (int64_t)blockIdx.x * kBwdReduceCols + col;
  const int per = (nslab + kBwdReduceWaves - 1) / kBwdReduceWaves;
  const int b0 = min(nslab, w * per), b1 = min(nslab, b0 + per);
  float sum = 0.f;
  if (e < MC) {
    int b = b0 + k;
    constexpr int S = kBwdReduceStreams;
    for (; b + 7 * S < b1; b += 8 * S) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ws_F[(int64_t)(b + u * S) * MC + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) sum += v[u];
    }
    for (; b < b1; b += S) sum += ws_F[(int64_t)b * MC + e];
  }
  part[w][lane] = sum;
  __syncthreads();
  if (threadIdx.x < kBwdReduceCols && e < MC) {
    float r = 0.f;
    for (int ww = 0; ww < kBwdReduceWaves; ++ww) {
      float rw = part[ww][col];
#pragma unroll
      for (int kk = 1; kk < kBwdReduceStreams; ++kk) rw += part[ww][kk * kBwdReduceCols + col];
      r += rw;
    }
    gF[e] = r;
  }
}

// The default since round 3: one block per COLS consecutive elements, 1024
// threads = 1024/COLS slab streams per element; stream k sums slabs k, k + S, k + 2S, ...
// (all of a thread's loads issued together), then the S partials of an element are
// added by a fixed-order halving tree in LDS.  Deterministic; a different (fixed)
// summation order from action_bwd_reduce_kernel.
template <int COLS>
__global__ __launch_bounds__(1024) void action_bwd_reduce2_kernel(const float* ws_F, float* gF, int64_t MC,
                                                                  int nslab) {
  constexpr int S = 1024 / COLS;
  __shared__ float part[S][COLS];
  const int col = (int)threadIdx.x % COLS, k = (int)threadIdx.x / COLS;
  const int64_t e = (int64_t)blockIdx.x * COLS + col;
  float sum = 0.f;
  if (e < MC) {
    int b = k;
    for (; b + 7 * S < nslab; b += 8 * S) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ws_F[(int64_t)(b + u * S) * MC + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) sum += v[u];
    }
    for (; b < nslab; b += S) sum += ws_F[(int64_t)b * MC + e];
  }
  part[k][col] = sum;
#pragma unroll
  for (int h = S / 2; h >= 1; h >>= 1) {
    __syncthreads();
    if (k < h) part[k][col] += part[k + h][col];
  }
  if (k == 0 && e < MC) gF[e] = part[0][col];
}

// Chunk-major slabs (ActionBwdArgs::slab_chunked): one block per 16-element chunk, whose
// gx slabs are one contiguous run of gx * 64 bytes.  Thread t takes quarter q = t % 4 of
// every slab b = t / 4, t / 4 + 256, ... (16-byte loads, all issued together), then the 256
// partials of each quarter are added by a fixed-order halving tree.  Deterministic.
__global__ __launch_bounds__(1024) void action_bwd_reduce3_kernel(const float* ws_F, float* gF, int64_t MC,
                                                                  int nslab, unsigned long long* stamps) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  unsigned long long* rst = stamps ? stamps + kStampBlocks * 16 * 8 + 2 * (int64_t)blockIdx.x : nullptr;
  if (rst && threadIdx.x == 0) rst[0] = __builtin_amdgcn_s_memrealtime();
  __shared__ f4 part[256][4];
  const int q = (int)threadIdx.x & 3, bs = (int)threadIdx.x >> 2;
  const f4* base = reinterpret_cast<const f4*>(ws_F + (int64_t)blockIdx.x * nslab * kSlabChunk) + q;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  int b = bs;
  for (; b + 3 * 256 < nslab; b += 4 * 256) {
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = base[(int64_t)(b + u * 256) * 4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u];
  }
  {
    f4 v[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) v[u] = b + u * 256 < nslab ? base[(int64_t)(b + u * 256) * 4] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (b + u * 256 < nslab) acc += v[u];
  }
  part[bs][q] = acc;
#pragma unroll
  for (int h = 128; h >= 1; h >>= 1) {
    __syncthreads();
    if (bs < h) part[bs][q] += part[bs + h][q];
  }
  if (bs == 0) {
    const f4 r = part[0][q];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t e = (int64_t)blockIdx.x * kSlabChunk + 4 * q + k;
      if (e < MC) gF[e] = r[k];
    }
    if (rst) rst[1] = __builtin_amdgcn_s_memrealtime();
  }
}

// Chunk-major slabs, fewer barriers: as action_bwd_reduce3_kernel, but the 16 slab streams
// of a wave are combined by cross-lane shuffles (xor 4, 8, 16, 32: stream pairs, no
// barrier), then the 16 waves' partials by one barrier and a 16-term sum in wave order.
// Deterministic (a fixed order, different from reduce3's halving tree).
__global__ __launch_bounds__(1024) void action_bwd_reduce4_kernel(const float* ws_F, float* gF, int64_t MC,
                                                                  int nslab) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ f4 part[16][4];
  const int q = (int)threadIdx.x & 3, bs = (int)threadIdx.x >> 2;
  const f4* base = reinterpret_cast<const f4*>(ws_F + (int64_t)blockIdx.x * nslab * kSlabChunk) + q;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  int b = bs;
  for (; b + 3 * 256 < nslab; b += 4 * 256) {
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = base[(int64_t)(b + u * 256) * 4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u];
  }
  {
    f4 v[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) v[u] = b + u * 256 < nslab ? base[(int64_t)(b + u * 256) * 4] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (b + u * 256 < nslab) acc += v[u];
  }
#pragma unroll
  for (int m = 4; m <= 32; m <<= 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += __shfl_xor(acc[k], m, 64);
  }
  const int w = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
  if (lane < 4) part[w][lane] = acc;
  __syncthreads();
  if (threadIdx.x < 4) {
    f4 r = part[0][q];
#pragma unroll
    for (int ww = 1; ww < 16; ++ww) r += part[ww][q];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t e = (int64_t)blockIdx.x * kSlabChunk + 4 * q + k;
      if (e < MC) gF[e] = r[k];
    }
  }
}

// Chunk-major slabs, one 256-thread block per 16-element chunk (the default, LV_BWD_REDUCE=6):
// thread t takes quarter q = t % 4 of slabs t / 4, t / 4 + 64, ... -- up to kR5Loads 16-byte
// loads issued together per round -- then the 64 streams of a quarter are combined by
// cross-lane shuffles inside each wave (xor 4, 8, 16, 32) and the 4 waves' partials in wave
// order after one barrier.  Fewer threads and barriers than reduce3 (1,024 threads, an
// 8-level tree); deterministic in a fixed order of its own.
constexpr int kR5Loads = 12;
// The reduce5 body for one chunk: the modular reduce and the fused VJP launch's reduce blocks
// both call it, so their dF is the same fixed summation order by construction (the bitwise
// fused-vs-modular contract).
__device__ __forceinline__ void reduce5_chunk(const float* ws_F, float* gF, int64_t MC, int nslab, int chunk) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ f4 part[4][4];
  const int q = (int)threadIdx.x & 3, bs = (int)threadIdx.x >> 2;
  const f4* base = reinterpret_cast<const f4*>(ws_F + (int64_t)chunk * nslab * kSlabChunk) + q;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int b0 = bs; b0 < nslab; b0 += 64 * kR5Loads) {
    f4 v[kR5Loads];
#pragma unroll
    for (int u = 0; u < kR5Loads; ++u) {
      const int b = b0 + 64 * u;
      v[u] = b < nslab ? base[(int64_t)b * 4] : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kR5Loads; ++u) acc += v[u];
  }
#pragma unroll
  for (int m = 4; m <= 32; m <<= 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += __shfl_xor(acc[k], m, 64);
  }
  const int w = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
  if (lane < 4) part[w][lane] = acc;
  __syncthreads();
  if (threadIdx.x < 4) {
    f4 r = part[0][q];
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) r += part[ww][q];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t e = (int64_t)chunk * kSlabChunk + 4 * q + k;
      if (e < MC) gF[e] = r[k];
    }
  }
}
__global__ __launch_bounds__(256) void action_bwd_reduce5_kernel(const float* ws_F, float* gF, int64_t MC, int nslab) {
  reduce5_chunk(ws_F, gF, MC, nslab, (int)blockIdx.x);
}

// The persistent backward's fused tail in one launch: blocks [0, nvjp) run the exp -> ZYZ
// VJP (exp_eazyz_vjp_sample, one sample per thread: the same per-sample function as
// lv_exp_eazyz_vjp, so the same bits), blocks [nvjp, nvjp + chunks) the reduce5 dF sum.
// Both read only the persistent kernel's outputs, so they run side by side instead of
// back to back (the VJP is one long dependent chain per sample at one wave per SIMD).
__global__ __launch_bounds__(256) void action_bwd_reduce5_vjp_kernel(const float* ws_F, float* gF, int64_t MC,
                                                                     int nslab, int nvjp, const float* mu,
                                                                     const float* v, const float* gang,
                                                                     float* gmu, float* gv, int64_t n) {
  if ((int)blockIdx.x < nvjp) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
      float av[3], g[3], m[9], gm[9], o[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) { av[k] = v[i * 3 + k]; g[k] = gang[i * 3 + k]; }
      if (mu) {
#pragma unroll
        for (int k = 0; k < 9; ++k) m[k] = mu[i * 9 + k];
      }
      exp_eazyz_vjp_sample(av, mu != nullptr, m, g, gm, o);
      if (mu) {
#pragma unroll
        for (int k = 0; k < 9; ++k) gmu[i * 9 + k] = gm[k];
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) gv[i * 3 + k] = o[k];
    }
    return;
  }
  reduce5_chunk(ws_F, gF, MC, nslab, (int)blockIdx.x - nvjp);
}

namespace {

template <int... Ls>
constexpr std::array<int, sizeof...(Ls)> nnz_table(std::integer_sequence<int, Ls...>) {
  return {j_nnz<Ls>()...};
}
constexpr auto kNnz = nnz_table(std::make_integer_sequence<int, LV_MAX_DEGREE + 1>{});

// Lane-instruction cost of one degree of the chain (FMA-pairs + loads + staging).
inline double degree_cost(int l, bool bwd) {
  const int n = 2 * l + 1;
  const double fwd = 2.0 * kNnz[l] + 6.0 * n + 3.0 * n;
  return bwd ? 2.2 * fwd : fwd;
}

// Split degrees 0..L into nseg contiguous ranges minimising the max range cost
// (prologue cost P charged per range).  Returns seg_lo[0..nseg].  Fixed-size tables: no
// allocation on the launch path.
inline int plan_segments(int L, int nseg, double P, bool bwd, int* seg_lo) {
  constexpr int kD = LV_MAX_DEGREE + 1;
  const int D = L + 1;
  nseg = std::max(1, std::min(nseg, std::min(D, kMaxSeg)));
  double pre[kD + 1];
  pre[0] = 0.0;
  for (int l = 0; l < D; ++l) pre[l + 1] = pre[l] + degree_cost(l, bwd);
  // dp[k][i]: best max cost splitting first i degrees into k ranges
  const double INF = 1e30;
  double dp[kMaxSeg + 1][kD + 1];
  int arg[kMaxSeg + 1][kD + 1];
  for (int k = 0; k <= nseg; ++k)
    for (int i = 0; i <= D; ++i) { dp[k][i] = INF; arg[k][i] = 0; }
  dp[0][0] = 0.0;
  for (int k = 1; k <= nseg; ++k)
    for (int i = 1; i <= D; ++i)
      for (int p = k - 1; p < i; ++p) {
        const double v = std::max(dp[k - 1][p], pre[i] - pre[p] + P);
        if (v < dp[k][i]) { dp[k][i] = v; arg[k][i] = p; }
      }
  int i = D;
  for (int k = nseg; k >= 1; --k) {
    seg_lo[k] = i;
    i = arg[k][i];
  }
  seg_lo[0] = 0;
  return nseg;
}

// Degree sets of the waves, balanced by cost (LPT: degrees in decreasing cost -- decreasing
// l -- each to the least loaded wave, ties to the lowest index).  Contiguous ranges cannot
// balance the high degrees (in-kernel per-degree timings, profiles/r04_timeline_*.txt:
// backward l = 10 segments [0,6) [6,8) [8,10) [10] ran 3.9 / 4.0 / 5.2 / 3.6 us, and every
// wave of a block waits at the barrier for the slowest).  Each degree also carries a fixed
// cost (multiples reads, spectrum column, LDS round trips): kDegFixed, fitted to the same
// timings; the forward's raised from 40 to 80 by the round-6 degree-set A/B
// (profiles/r06_ab_masks_c2.txt, l = 10, 6 waves: degree 0 on the {9} wave instead of the
// {5, 4} one, 7.09 vs 7.19 us, outputs bitwise identical).  At C = 10 (the only C with
// degree sets) that is the one tile plan it changes.
constexpr double kDegFixedFwd = 80.0, kDegFixedBwd = 30.0;
inline double degree_cost_sched(int l, bool bwd) {
  return (bwd ? kDegFixedBwd : kDegFixedFwd) + degree_cost(l, bwd);
}
inline void balance_masks(int L, int nseg, bool bwd, unsigned* masks) {
  double load[kMaxSeg];
  for (int k = 0; k < nseg; ++k) { load[k] = 0.0; masks[k] = 0u; }
  for (int l = L; l >= 0; --l) {
    int best = 0;
    for (int k = 1; k < nseg; ++k)
      if (load[k] < load[best]) best = k;
    masks[best] |= 1u << l;
    load[best] += degree_cost_sched(l, bwd);
  }
  for (int k = nseg; k < kMaxSeg; ++k) masks[k] = 0u;
}
inline void contiguous_masks(const int* seg_lo, int nseg, unsigned* masks) {
  for (int k = 0; k < kMaxSeg; ++k) {
    masks[k] = 0u;
    if (k < nseg)
      for (int l = seg_lo[k]; l < seg_lo[k + 1]; ++l) masks[k] |= 1u << l;
  }
}

// Segments so that the grid has ~2.7 waves per SIMD (1024 SIMDs on MI355X; measured
// best at batch 4096, l = 10: 4 segments), but never more ranges than pay for their
// duplicated prologue.
inline int choose_nseg(int64_t n, int Sw, int L, double P, bool bwd) {
  const int64_t waves = (n + Sw - 1) / Sw;
  const int64_t target = 2732;
  int nseg = (int)std::min<int64_t>(kMaxSeg, std::max<int64_t>(1, (target + waves - 1) / waves));
  // cap: a range should carry at least ~2x its prologue
  double total = 0.0;
  for (int l = 0; l <= L; ++l) total += degree_cost(l, bwd);
  const int cap = std::max(1, (int)(total / (2.0 * P)));
  return std::min(nseg, std::min(cap, L + 1));
}

constexpr double kPrologueFwd = 200.0;
constexpr double kPrologueFused = 250.0;

// Tile kernel (shared spectrum): one block per sample group, one wave per degree
// segment, the prologue once per (sample, slot), output staged in LDS and written as
// whole lines.  Measured on MI355X (tools/fwdbench.hip, l = 10, C = 10,
// profiles/r02_fwd_ab_*.txt): 6-8 segments best at batch 4096, 4 at 65536 (fewer
// segments = fewer waves to hide the chain latency, more = more spectrum staging and a
// bigger block); write-through (sc1) stores best while the output is small enough to be
// written during the kernel (batch 4096, 19.8 MB), nt beyond (65536: 68 vs 81 us).
constexpr size_t kTileMaxLds = 80 * 1024;    // >= 2 blocks per CU
// Per-wave chain cost target by sample groups per CU (round 6, C = 10, l = 10, fp32, same
// box: profiles/r06_ab_nseg_sweep.txt): <= 4 groups per CU 7 waves (batch 4,096: 6.92 us
// against 7.12-7.17 at 6), <= 16 8 waves (8,192: 11.5 vs 12.0; 16,384: 17.6 vs 19.5 at 4),
// beyond 4 waves (65,536: 60.3 vs 62.3-65.1 at 6-8; 32,768 flat from 4 to 8).
constexpr double kTileSegCostFew = 300.0;    // -> 7 waves at l = 10
constexpr double kTileSegCostMid = 260.0;    // -> 8
constexpr double kTileSegCostLarge = 560.0;  // -> 4
constexpr int64_t kTileFewGroupsPerCU = 4, kTileMidGroupsPerCU = 16;
constexpr double kTilePrologue = 60.0;       // per-wave fixed cost: spectrum slice, multiples reads
// round 6 (7 / 8 waves per block): write-through still wins at 6,144 samples (29.7 MB:
// 8.7-8.8 vs 9.0-9.1 us) and loses from 8,192 (39.6 MB: 11.7 vs 11.4; profiles/r06_ab_wt.txt)
constexpr int64_t kWriteThroughMaxBytes = 32ll << 20;

// A/B knobs (LV_TILE=0 disables the tile kernel, LV_TILE_WT=0/1 forces the store policy,
// LV_*_NSEG force segment counts, LV_BWD_FGLOBAL forces the backward's global-spectrum
// mode) exist only in the A/B build (-DLV_AB_KNOBS -> liblievae_hip_ab.so, used by
// tools/ and one bitwise test): the product library never reads the environment, so a
// stray variable cannot change its kernels or its summation order.
#ifdef LV_AB_KNOBS
int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}
#define LV_KNOB(name, dflt) env_int(name, dflt)
// Phase-timestamp buffer of the timeline tool (LV_STAMPS=1, A/B build only): allocated once
// on the first call, read back by lv_ab_stamps_copy.
constexpr size_t kStampBytes = sizeof(unsigned long long) * ((size_t)kStampDegBase + kStampDegBlocks * 16 * 24);
unsigned long long* ab_stamps() {
  static unsigned long long* p = nullptr;
  static bool tried = false;
  if (!tried) {
    tried = true;
    if (env_int("LV_STAMPS", 0) && hipMalloc(&p, kStampBytes) == hipSuccess) (void)hipMemset(p, 0, kStampBytes);
  }
  return p;
}
// LV_TILE_MASKS / LV_BWD_MASKS (A/B): the forward tile kernel's / the compile-time-C
// backward's degree sets as ':'- or ','-separated hex masks (one per wave, in wave order);
// used only when they partition 0..L into exactly the plan's wave count, so a sweep can try
// hand-made sets without a rebuild
bool env_masks(const char* name, int L, int nseg, unsigned* masks) {
  const char* v = std::getenv(name);
  if (!v || !*v) return false;
  unsigned m[kMaxSeg] = {};
  int k = 0;
  unsigned all = 0;
  for (const char* s = v; *s && k < kMaxSeg;) {
    char* e = nullptr;
    m[k] = (unsigned)std::strtoul(s, &e, 16);
    if (e == s || (m[k] & all) || m[k] == 0) return false;
    all |= m[k++];
    s = (*e == ',' || *e == ':') ? e + 1 : e;
  }
  if (k != nseg || all != (1u << (L + 1)) - 1) return false;
  for (int i = 0; i < kMaxSeg; ++i) masks[i] = i < nseg ? m[i] : 0u;
  return true;
}
#else
#define LV_KNOB(name, dflt) (dflt)
inline unsigned long long* ab_stamps() { return nullptr; }
inline bool env_masks(const char*, int, int, unsigned*) { return false; }
#endif

int device_cus();

bool plan_tile(FwdLaunch& p, int L, int out_bytes, int cus) {
  static const int kEnvTile = LV_KNOB("LV_TILE", 1);
  static const int kEnvWT = LV_KNOB("LV_TILE_WT", -1);
  static const int kEnvTileNseg = LV_KNOB("LV_TILE_NSEG", 0);  // A/B testing only
  static const int kEnvPrio = LV_KNOB("LV_TILE_PRIO", 2);      // wave priority phases (ActionArgs)
  // samples per block with compile-time C (A/B knob LV_TILE_SW)
  static const int kEnvSw = LV_KNOB("LV_TILE_SW", 0);
  if (!kEnvTile) return false;
  ActionArgs& a = p.a;
  int Sw = 64 / a.C;
  if (a.C == kTileFastC && kEnvSw >= 2 && kEnvSw < Sw) Sw = kEnvSw;
  const int64_t groups = (a.n + Sw - 1) / Sw;
  double total = 0.0;
  for (int l = 0; l <= L; ++l) total += degree_cost(l, false);
  const double target = groups <= kTileFewGroupsPerCU * cus   ? kTileSegCostFew
                        : groups <= kTileMidGroupsPerCU * cus ? kTileSegCostMid
                                                              : kTileSegCostLarge;
  int nseg = std::max(1, std::min(std::min(8, L + 1), (int)std::ceil(total / target)));
  if (kEnvTileNseg > 0) nseg = std::min(std::min(8, L + 1), kEnvTileNseg);
  // the prologue takes one thread per (sample, slot): 3*Sw threads of the block
  nseg = std::min(L + 1, std::max(nseg, (3 * Sw + 63) / 64));
  if (3 * Sw > 64 * nseg || nseg > 8) return false;
  plan_segments(L, nseg, kTilePrologue, false, a.seg_lo);
  // compile-time C: cost-balanced degree sets; run-time C keeps the contiguous ranges
  // (its spectrum slices are per-wave row ranges)
  static const int kEnvContig = LV_KNOB("LV_SEG_CONTIG", 0);  // A/B: contiguous ranges everywhere
  if (a.C == kTileFastC && env_masks("LV_TILE_MASKS", L, nseg, a.seg_mask)) {
  } else if (a.C == kTileFastC && !kEnvContig) balance_masks(L, nseg, false, a.seg_mask);
  else contiguous_masks(a.seg_lo, nseg, a.seg_mask);
  // spectrum in LDS: C = kTileFastC -> the whole (M, C) once, row-major; other C ->
  // per-wave column-major slices below kTileFGlobalMinL, global memory from there
  int fp = 0;
  if (a.C != kTileFastC && L < kTileFGlobalMinL)
    for (int k = 0; k < nseg; ++k) fp = std::max(fp, fseg_rows(a.seg_lo[k], a.seg_lo[k + 1]) * a.C);
  a.fpitch = (fp + 3) & ~3;
  // (C = kTileFastC with fp32 output: the spectrum sits in the tile's last sample slot)
  const size_t fl = a.C == kTileFastC ? (out_bytes == 4 ? 0 : (size_t)a.MC) : (size_t)nseg * a.fpitch;
  const size_t trig = (size_t)Sw * (6 * ((L + 1 + 3) & ~3) + 4);  // TrigLds<L>::kRow per sample
  const size_t lds = (size_t)tile_stage_bytes(Sw, a.MC, out_bytes) + sizeof(float) * (fl + trig);
  if (lds > kTileMaxLds || groups > 0x7fffffff) return false;
  a.Sw = Sw;
  a.write_through = (int64_t)a.n * a.MC * out_bytes <= kWriteThroughMaxBytes ? 1 : 0;
  if (kEnvWT >= 0) a.write_through = kEnvWT;
  a.prio = kEnvPrio;
  static const int kEnvSpread = LV_KNOB("LV_TILE_SPREAD", 0);  // A/B: prologue tasks over all waves
  a.task_spread = kEnvSpread;
  static const int kEnvAngOrder = LV_KNOB("LV_TILE_ANG_ORDER", 0);  // A/B: 1 = angles after the spectrum loads
  a.ang_order = kEnvAngOrder;
  p.tile = true;
  p.lds = lds;
  p.gx = (int)groups;
  p.gy = nseg;
  return true;
}

template <template <int> class Launcher, int LT = 0>
int dispatch_L(int L, typename Launcher<0>::Args& args) {
  if constexpr (LT > LV_MAX_DEGREE) {
    set_error("l_max %d > %d unsupported", L, LV_MAX_DEGREE);
    return LV_ERR_ARG;
  } else {
    if (L == LT) return Launcher<LT>::run(args);
    return dispatch_L<Launcher, LT + 1>(L, args);
  }
}

int check_common(int64_t n, int L, int C, int dtype) {
  LV_CHECK_ARG(n >= 0, "n must be >= 0 (got %lld)", (long long)n);
  LV_CHECK_ARG(L >= 0 && L <= LV_MAX_DEGREE, "l_max must be in [0, %d] (got %d)", LV_MAX_DEGREE, L);
  LV_CHECK_ARG(C >= 1 && C <= LV_MAX_CHANNELS, "C must be in [1, %d] (got %d)", LV_MAX_CHANNELS, C);
  LV_CHECK_ARG(dtype == LV_DTYPE_F32 || dtype == LV_DTYPE_BF16, "bad out dtype %d", dtype);
  return LV_OK;
}

// Argument checks + launch plan of the forward (host only, no GPU call): the tile
// kernel when its LDS footprint fits, else the grid-stride kernel (gx blocks of
// kWavesPerBlock waves x gy degree segments).  n > 0.
int check_fwd(bool fused, int64_t Fstride, int out_dtype, int64_t n, int L, int C) {
  if (int e = check_common(n, L, C, out_dtype)) return e;
  const int64_t MC = (int64_t)(L + 1) * (L + 1) * C;
  LV_CHECK_ARG(Fstride == 0 || Fstride == MC, "F batch stride must be 0 or M*C=%lld", (long long)MC);
  LV_CHECK_ARG(!fused || Fstride == 0, "the fused path takes a shared spectrum (F batch stride 0)");
  LV_CHECK_ARG(Fstride == 0 || out_dtype == LV_DTYPE_F32, "bf16 output needs a shared spectrum");
  return LV_OK;
}

int plan_fwd(bool fused, int64_t Fstride, int out_dtype, int64_t n, int L, int C, int cus, FwdLaunch& p) {
  if (int e = check_fwd(fused, Fstride, out_dtype, n, L, C)) return e;
  const int64_t MC = (int64_t)(L + 1) * (L + 1) * C;
  p = FwdLaunch{};
  p.a.Fstride = Fstride;
  p.a.n = n;
  p.a.MC = MC;
  p.a.C = C;
  p.a.Sw = 64 / C;
  p.fused = fused;
  p.dtype = out_dtype;
  const int ob = out_dtype == LV_DTYPE_BF16 ? 2 : 4;
  if (Fstride == 0 && plan_tile(p, L, ob, cus)) return LV_OK;
  const double P = fused ? kPrologueFused : kPrologueFwd;
  static const int kEnvFwdNseg = LV_KNOB("LV_FWD_NSEG", 0);  // A/B testing only
  const int nseg = kEnvFwdNseg > 0 ? std::min(kEnvFwdNseg, std::min(L + 1, kMaxSeg))
                                   : choose_nseg(n, p.a.Sw, L, P, false);
  plan_segments(L, nseg, P, false, p.a.seg_lo);
  contiguous_masks(p.a.seg_lo, nseg, p.a.seg_mask);  // (reported by the plan query only)
  const int64_t gx = (n + (int64_t)p.a.Sw * kWavesPerBlock - 1) / ((int64_t)p.a.Sw * kWavesPerBlock);
  LV_CHECK_ARG(gx <= 0x7fffffff, "batch too large");
  p.gx = (int)gx;
  p.gy = nseg;
  // LDS: the widest segment's spectrum slice (shared F), then the per-sample trig tables
  // from kTrigLdsMinL
  int fmax = 0;
  if (Fstride == 0)
    for (int k = 0; k < nseg; ++k)
      fmax = std::max(fmax, (fseg_rows(p.a.seg_lo[k], p.a.seg_lo[k + 1]) * C + 3) & ~3);
  p.a.fpitch = fmax;
  const size_t trig = L >= kTrigLdsMinL ? (size_t)kWavesPerBlock * p.a.Sw * trig_row_floats(L) : 0;
  p.lds = sizeof(float) * ((size_t)fmax + trig);
  return LV_OK;
}

// Per-thread caches of launch plans, keyed by everything the planners read: the segment
// DP and the LDS sizing run once per shape instead of on every call (the eager training
// path calls the same shapes every step).
template <class K, class V, int N = 8>
struct PlanCache {
  K key[N];
  V val[N];
  int used = 0, next = 0;
  const V* find(const K& k) const {
    for (int i = 0; i < used; ++i)
      if (key[i] == k) return &val[i];
    return nullptr;
  }
  void put(const K& k, const V& v) {
    key[next] = k;
    val[next] = v;
    next = (next + 1) % N;
    used = std::min(used + 1, N);
  }
};
using FwdKey = std::array<int64_t, 7>;  // fused, F stride, out dtype, n, L, C, CUs

int plan_fwd_cached(bool fused, int64_t Fstride, int out_dtype, int64_t n, int L, int C, FwdLaunch& p) {
  thread_local PlanCache<FwdKey, FwdLaunch> cache;
  const int cus = device_cus();
  const FwdKey k{fused ? 1 : 0, Fstride, out_dtype, n, L, C, cus};
  if (const FwdLaunch* hit = cache.find(k)) {
    p = *hit;
    return LV_OK;
  }
  if (int e = plan_fwd(fused, Fstride, out_dtype, n, L, C, cus, p)) return e;
  cache.put(k, p);
  return LV_OK;
}

int action_fwd_common(bool fused, const float* ang, const float* mu, const float* v, const float* F,
                      int64_t Fstride, void* out, int out_dtype, float* ang_out, int64_t n, int L,
                      int C, int transpose, hipStream_t stream) {
  clear_error();
  if (int e = check_fwd(fused, Fstride, out_dtype, n, L, C)) return e;
  if (n == 0) return LV_OK;
  LV_CHECK_ARG(F && out, "null F/out");
  LV_CHECK_ARG(fused ? (v != nullptr) : (ang != nullptr), "null input");
  FwdLaunch p;
  if (int e = plan_fwd_cached(fused, Fstride, out_dtype, n, L, C, p)) return e;
  p.a.ang = ang;
  p.a.mu = mu;
  p.a.v = v;
  p.a.F = F;
  p.a.out = out;
  p.a.ang_out = ang_out;
  p.a.transpose = transpose ? 1 : 0;
  p.a.stamps = ab_stamps();
  p.stream = stream;
  return dispatch_L<FwdLauncher>(L, p);
}

// run-time index -> compile-time launcher tables
template <template <int> class Launcher, class Args, int... Is>
constexpr std::array<int (*)(Args&), sizeof...(Is)> launcher_table(std::integer_sequence<int, Is...>) {
  return {&Launcher<Is>::run...};
}
constexpr auto kBwdRun = launcher_table<BwdLauncher, BwdLaunch>(std::make_integer_sequence<int, LV_MAX_DEGREE + 1>{});
constexpr auto kWigRun = launcher_table<WigLauncher, WigLaunch>(std::make_integer_sequence<int, LV_MAX_DEGREE + 1>{});

// Backward plan (action_bwd_tile_kernel): samples per block (Sw <= 64/C, reduced until the
// fp32 gradient tile fits), degree segments as in the forward (the backward chain costs
// ~2.2x), grid capped at kBwdMaxBlocks so the dF workspace stays bounded (blocks then
// loop over groups).
constexpr size_t kBwdMaxLds = 96 * 1024;
constexpr int64_t kBwdMaxBlocks = 4096;
// Per-wave backward chain cost target: the backward kernel is register-heavy (~256 VGPRs,
// 2 waves per SIMD), so few long waves beat many short ones -- measured at batch 4096,
// l = 10 (profiles/r02_bwd_nseg_sweep.txt): 1 / 2 / 3 / 4 / 6 / 8 segments ran
// 40.8 / 32.0 / 42.6 / 39.1 / 44.8 / 45.5 us per call.
constexpr double kBwdSegCost = 2.2 * 1000.0;
// The 3-waves-per-SIMD kernel (bwd_wide in action_bwd.h): half the per-segment cost, 4
// segments at l = 10 (2 / 3 / 4 / 6 / 8 ran 24.2 / 22.2 / 19.5 / 27.8 / 26.9 us per call,
// profiles/r02_bwd_regbudget_sweep.txt).
constexpr double kBwdSegCostWide = 1.1 * 1000.0;
// Compute units of the current device (hipDeviceAttributeMultiprocessorCount, cached per
// device): the persistent backward's grid (3 blocks per CU), and with it the dF summation
// order, follows the part it runs on -- 256 on a full MI355X, fewer on a CPX partition.
// Without a device (CPU-only host planning) the MI355X count.
constexpr int kDefaultCUs = 256;
int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return kDefaultCUs;
  }
  static std::atomic<int> cache[64];
  int cus = cache[dev].load(std::memory_order_relaxed);
  if (cus > 0) return cus;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
    (void)hipGetLastError();
    cus = kDefaultCUs;
  }
  cache[dev].store(cus, std::memory_order_relaxed);
  return cus;
}
// LV_BWD_REDUCE default (see action_bwd_common): 6 = chunk-major slabs + reduce5 (one
// 256-thread block per 16-element chunk).  Same box, backward alone (profiles/r05_reduce_ab.txt):
// 512: 8.93 -> 8.72 us, 4,096: 14.45 -> 13.94, 16,384: 32.2 -> 31.9, 65,536: 103.4 -> 102.5
// against reduce3; a block per quarter chunk (4x the blocks, 16-byte reads at a 64-byte
// stride) was slower: 4,096: 17.2 us.
constexpr int kBwdReduceDefault = 6;
// LV_BWD_VARIANT default (kBwdVar* bits): JIT chain (profiles/r04_bwd_reduce_ab.txt); the
// persistent kernel with one tile buffer at 3 blocks per CU (65,536: 131 -> 114 us against
// the double-buffered 2 blocks per CU, profiles/r05_ab4.txt), its next multiples filled by
// one wave (profiles/r05_ab8.txt), its angle partials summed by one wave from LDS instead of
// a cross-lane tree on every wave (round 6, same box: 65,536 104.0 -> 96.8 us, 262,144 378
// -> 358, 16,384 31.9 -> 30.6; the padded tile, kBwdVarPersistPad, was slower alone and
// with it: 104.5 / 100.2-100.9 us, profiles/r06_ab_persist.txt), and its gradient tile
// by buffer loads to LDS with SGPR round offsets (65,536 99.2-100.5 -> 96.8-97.5 us,
// 4,096 13.7-13.9 -> 13.3-13.5, 262,144 359-360 -> 351-352; profiles/r06_ab_bufdma.txt),
// and its dF slab as 16-byte write-through stores (4,096 13.47-13.52 -> 12.92-13.03 us,
// 16,384 29.9-30.3 -> 29.4-29.5, 2,048 10.4 -> 10.25, 65,536 unchanged; dF bitwise equal;
// profiles/r06_ab_slabwt.txt)
constexpr int kBwdVariantDefault = kBwdVarJit | kBwdVarPersistSingle | kBwdVarPersistTask1 | kBwdVarPersistAng |
                                   kBwdVarPersistBufDma | kBwdVarPersistSlabWT;

// Fallback for tiles that leave no LDS room for the spectrum and the dF slab (large C at
// high l): the whole CU's LDS, the spectrum read from global memory and the slab kept in
// the block's workspace row (kBwdFSharedGlobal); per-sample spectra only need the bigger
// LDS budget.  One block per CU at most, so fewer blocks (and workspace rows) suffice.
constexpr size_t kBwdMaxLdsFallback = 160 * 1024;
constexpr int64_t kBwdMaxBlocksFallback = 1024;

struct BwdPlan {
  int Sw, nseg, gx, fpitch, fmode;
  int persist;            // action_bwd_persist_kernel
  size_t ws_gang_off;     // persist: byte offset of the angle-gradient region (fused VJP)
  int64_t groups;
  int seg_lo[kMaxSeg + 1];
  unsigned seg_mask[kMaxSeg];
  size_t lds, ws;
};

// Persistent backward (action_bwd_persist.h) from more than one 6-sample group per CU (257
// groups = 1,537 samples on MI355X): up to 3 blocks per CU walk the groups, the next
// group's multiples prefetched, one dF slab per block.  Round 5 used it only beyond one
// round of 3 blocks per CU (769 groups; 4,096: 14.26 vs 14.47 us one-group vs persistent,
// profiles/r05_bwd_persist_ab2.txt); with the LDS angle sums it is faster from 342 groups:
// 2,048 samples 11.15 -> 10.5 us, 4,096 14.1 -> 13.8, while at <= one group per CU the
// one-group kernel's 8 segments keep more waves busy (512: 8.5 vs 9.6 us, 1,024: 8.8 vs
// 10.3; profiles/r06_ab_persist_small_batches.txt).

bool plan_bwd(int64_t n, int L, int C, bool sharedF, int cus, BwdPlan& b) {
  static const int kEnvNseg = LV_KNOB("LV_BWD_NSEG", 0);      // A/B testing only
  static const int kEnvGlobal = LV_KNOB("LV_BWD_FGLOBAL", 0);  // force the fallback (tests)
  static const int kEnvPersistMin = LV_KNOB("LV_BWD_PERSIST_MIN", -1);  // A/B; 0 = off, -1 = 3 * CUs + 1
  static const int kEnvVariantP = LV_KNOB("LV_BWD_VARIANT", kBwdVariantDefault);
  const bool single = (kEnvVariantP & kBwdVarPersistSingle) != 0;  // A/B: one tile buffer
  static const int kEnvPersistBpc = LV_KNOB("LV_BWD_PERSIST_BPC", 0);  // A/B: blocks per CU (grid)
  const int64_t persist_blocks =
      (int64_t)cus * (kEnvPersistBpc > 0 ? kEnvPersistBpc : single ? kBwdPersistBlocksPerCU : kBwdPersistBlocksPerCUDB);
  const int64_t persist_min = kEnvPersistMin < 0 ? (int64_t)cus + 1 : kEnvPersistMin;
  b = BwdPlan{};
  const int64_t MC = (int64_t)(L + 1) * (L + 1) * C;
  if (sharedF && C == kTileFastC && L >= kBwdPersistWaves - 1 && L <= kBwdPersistMaxL && !kEnvGlobal &&
      persist_min > 0) {
    const int Sw = 64 / C;
    const int64_t groups = (std::max<int64_t>(n, 1) + Sw - 1) / Sw;
    if (groups >= persist_min) {
      b.persist = 1;
      b.Sw = Sw;
      b.nseg = kBwdPersistWaves;
      b.fmode = kBwdFShared;
      b.groups = groups;
      b.gx = (int)std::min<int64_t>(groups, persist_blocks);
      plan_segments(L, b.nseg, kTilePrologue, true, b.seg_lo);
      if (!env_masks("LV_BWD_MASKS", L, b.nseg, b.seg_mask)) balance_masks(L, b.nseg, true, b.seg_mask);
      const bool pad = single && (kEnvVariantP & kBwdVarPersistPad) != 0;
      b.lds = sizeof(float) * (size_t)persist_lds_floats(L, b.nseg, single ? 1 : 2, pad);
      const size_t slabs = sizeof(float) * (size_t)b.gx * (size_t)(slab_chunks(MC) * kSlabChunk);
      b.ws_gang_off = slabs;
      b.ws = slabs + sizeof(float) * 3 * (size_t)std::max<int64_t>(n, 1);
      return true;
    }
  }
  double total = 0.0;
  for (int l = 0; l <= L; ++l) total += degree_cost(l, true);
  for (int fallback = (kEnvGlobal && sharedF) ? 1 : 0; fallback < 2; ++fallback) {
    const int fmode = !sharedF ? kBwdFSample : (fallback ? kBwdFSharedGlobal : kBwdFShared);
    const size_t cap = fallback ? kBwdMaxLdsFallback : kBwdMaxLds;
    for (int Sw = 64 / C; Sw >= 1; --Sw) {
      const int64_t groups = (std::max<int64_t>(n, 1) + Sw - 1) / Sw;
      const int64_t gx = std::min<int64_t>(groups, fallback ? kBwdMaxBlocksFallback : kBwdMaxBlocks);
      const double seg_cost = bwd_wide(L, C, fmode, groups, gx) ? kBwdSegCostWide : kBwdSegCost;
      int nseg = std::max(1, std::min(std::min(8, L + 1), (int)std::ceil(total / seg_cost)));
      // small batches: at most one group per CU leaves wave slots free, so the chain is
      // split into 8 segments (l = 10: batch 512 4 / 6 / 8 segments 11.9 / 10.5 / 10.3 us;
      // at 2,048 (342 groups) 6 and 8 segments were slower than 4: 19.3 / 18.6 vs 14.9)
      if (bwd_wide(L, C, fmode, groups, gx) && groups <= cus) nseg = std::max(nseg, std::min(8, L + 1));
      if (kEnvNseg > 0) nseg = std::min(std::min(8, L + 1), kEnvNseg);
      nseg = std::min(L + 1, std::max(nseg, (3 * Sw + 63) / 64));
      if (3 * Sw > 64 * nseg || nseg > 8) continue;
      plan_segments(L, nseg, kTilePrologue, true, b.seg_lo);
      // the run-time-C kernel with the spectrum in LDS stages per-wave row ranges: contiguous
      // degree sets; every other kernel takes cost-balanced sets (compile-time C stages the
      // whole spectrum once per block)
      const bool ct = C == kTileFastC && fmode == kBwdFShared;
      static const int kEnvContig = LV_KNOB("LV_SEG_CONTIG", 0);  // A/B: contiguous ranges everywhere
      if ((fmode == kBwdFShared && !ct) || kEnvContig) contiguous_masks(b.seg_lo, nseg, b.seg_mask);
      else if (!(ct && env_masks("LV_BWD_MASKS", L, nseg, b.seg_mask))) balance_masks(L, nseg, true, b.seg_mask);
      int fp = 0;
      if (fmode == kBwdFShared && !ct)
        for (int k = 0; k < nseg; ++k) fp = std::max(fp, fseg_rows(b.seg_lo[k], b.seg_lo[k + 1]) * C);
      b.fpitch = (fp + 3) & ~3;
      const size_t fregion = ct ? (size_t)((MC + 3) & ~3) : (size_t)nseg * b.fpitch;
      const size_t lds = (size_t)tile_stage_bytes(Sw, MC, 4) +
                         sizeof(float) * ((size_t)bwd_trig_floats(Sw, L) + (size_t)nseg * 64 * 3 +
                                          (fmode == kBwdFShared ? (size_t)MC : 0) +
                                          fregion + 12 * (size_t)Sw);
      if (lds > cap) continue;
      b.Sw = Sw;
      b.nseg = nseg;
      b.fmode = fmode;
      b.groups = groups;
      b.gx = (int)std::min<int64_t>(groups, fallback ? kBwdMaxBlocksFallback : kBwdMaxBlocks);
      if (kEnvGlobal && sharedF) b.gx = (int)std::min<int64_t>(groups, kBwdMaxBlocks);
      b.lds = lds;
      // shared spectrum: the dF slabs, then the angle-gradient region of the fused path (its
      // exp -> ZYZ VJP runs beside the reduce, in action_bwd_reduce5_vjp_kernel)
      b.ws_gang_off = sharedF ? sizeof(float) * (size_t)b.gx * (size_t)(slab_chunks(MC) * kSlabChunk) : 0;
      b.ws = sharedF ? b.ws_gang_off + sizeof(float) * 3 * (size_t)std::max<int64_t>(n, 1) : 0;
      return true;
    }
  }
  return false;
}

using BwdKey = std::array<int64_t, 5>;  // n, L, C, shared spectrum, device CUs

bool plan_bwd_cached(int64_t n, int L, int C, bool sharedF, BwdPlan& b) {
  thread_local PlanCache<BwdKey, BwdPlan> cache;
  const int cus = device_cus();
  const BwdKey k{n, L, C, sharedF ? 1 : 0, cus};
  if (const BwdPlan* hit = cache.find(k)) {
    b = *hit;
    return true;
  }
  if (!plan_bwd(n, L, C, sharedF, cus, b)) return false;
  cache.put(k, b);
  return true;
}

}  // namespace
}  // namespace lv

using namespace lv;
static_assert(7 + kMaxSeg + 1 + kMaxSeg == LV_PLAN_LEN, "plan layout (include/lievae.h)");

namespace {
int action_bwd_common(const float* ang, const float* F, int64_t F_batch_stride,
                      const float* gout, float* gang, float* gF, const float* mu, const float* v,
                      float* gmu, float* gv, int64_t n, int L, int C, int transpose,
                      void* workspace, size_t ws_bytes, void* stream) {
  if (int e = check_common(n, L, C, LV_DTYPE_F32)) return e;
  const int64_t MC = (int64_t)(L + 1) * (L + 1) * C;
  LV_CHECK_ARG(F_batch_stride == 0 || F_batch_stride == MC, "F batch stride must be 0 or M*C");
  const bool sharedF = F_batch_stride == 0;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    if (sharedF && gF) (void)hipMemsetAsync(gF, 0, sizeof(float) * MC, st);
    return LV_OK;
  }
  LV_CHECK_ARG(ang && F && gout && gF && (gang || v), "null pointer argument");
  LV_CHECK_ARG(!v || (gv && (!mu || gmu)), "null VJP output");
  BwdPlan b;
  LV_CHECK_ARG(plan_bwd_cached(n, L, C, sharedF, b), "no backward plan fits the LDS budget (l=%d, C=%d)", L, C);
  if (sharedF && (ws_bytes < b.ws || !workspace)) {
    set_error("workspace too small: need %zu bytes", b.ws);
    return LV_ERR_WORKSPACE;
  }
  BwdLaunch p{};
  p.a.ang = ang;
  p.a.F = F;
  p.a.Fstride = F_batch_stride;
  p.a.gout = gout;
  p.a.gang = gang;
  p.a.v = v;
  p.a.mu = mu;
  p.a.gv = gv;
  p.a.gmu = gmu;
  p.a.gF = gF;
  p.a.ws_F = (float*)workspace;
  p.a.n = n;
  p.a.MC = MC;
  p.a.groups = b.groups;
  p.a.C = C;
  p.a.Sw = b.Sw;
  p.a.transpose = transpose ? 1 : 0;
  p.a.fpitch = b.fpitch;
  static const int kEnvBwdPrio = LV_KNOB("LV_BWD_PRIO", 0);  // A/B: 2 = prologue-priority phases
  p.a.prio = kEnvBwdPrio;
  // dF slab reduce: LV_BWD_REDUCE (A/B) 6 = chunk-major slabs + action_bwd_reduce5_kernel
  // (default), 3 / 5 = the same slabs + reduce3 / reduce4, 16 / 8 / 4 = row slabs +
  // action_bwd_reduce2_kernel<COLS>, 1 = the round-2 kernel
  static const int kEnvReduce = LV_KNOB("LV_BWD_REDUCE", kBwdReduceDefault);
  p.a.slab_chunked = b.fmode != kBwdFSample && (kEnvReduce == 3 || kEnvReduce == 5 || kEnvReduce == 6);
  static const int kEnvVariant = LV_KNOB("LV_BWD_VARIANT", kBwdVariantDefault);
  p.a.variant = kEnvVariant;
  p.a.stamps = ab_stamps();
  for (int k = 0; k <= b.nseg; ++k) p.a.seg_lo[k] = b.seg_lo[k];
  for (int k = 0; k < kMaxSeg; ++k) p.a.seg_mask[k] = b.seg_mask[k];
  p.gx = b.gx;
  p.nseg = b.nseg;
  p.fmode = b.fmode;
  p.lds = b.lds;
  p.stream = st;
  p.persist = b.persist;
  if (b.persist) {
    // the persistent kernel writes the angle gradient (the fused path: into the workspace,
    // then the per-sample exp -> ZYZ VJP below) and chunk-major slabs, one per block
    p.a.slab_chunked = 1;
    if (v) p.a.gang = reinterpret_cast<float*>(static_cast<char*>(workspace) + b.ws_gang_off);
    p.a.v = nullptr;
    p.a.mu = nullptr;
    if (int e = kBwdRun[L](p)) return e;
    static const int kEnvReduceP = LV_KNOB("LV_BWD_REDUCE", kBwdReduceDefault);
    static const int kEnvVjpMerge = LV_KNOB("LV_BWD_VJP_MERGE", 1);  // A/B: 0 = separate VJP launch
    if (kEnvReduceP == 6 && v && kEnvVjpMerge) {
      // fused path: the VJP blocks and the dF reduce in one launch (side by side)
      const int nvjp = (int)((n + 255) / 256);
      hipLaunchKernelGGL(action_bwd_reduce5_vjp_kernel, dim3((unsigned)(nvjp + slab_chunks(MC))), dim3(256), 0,
                         st, (const float*)workspace, gF, MC, b.gx, nvjp, mu, v, (const float*)p.a.gang, gmu,
                         gv, n);
      LV_RETURN_LAUNCH("action_bwd_reduce5_vjp_kernel");
    }
    if (kEnvReduceP == 6)
      hipLaunchKernelGGL(action_bwd_reduce5_kernel, dim3((unsigned)slab_chunks(MC)), dim3(256), 0, st,
                         (const float*)workspace, gF, MC, b.gx);
    else
      hipLaunchKernelGGL(action_bwd_reduce3_kernel, dim3((unsigned)slab_chunks(MC)), dim3(1024), 0, st,
                         (const float*)workspace, gF, MC, b.gx, p.a.stamps);
    LV_CHECK_LAUNCH("action_bwd_reduce_kernel");
    if (v) return lv_exp_eazyz_vjp(mu, v, p.a.gang, gmu, gv, n, st);
    return LV_OK;
  }
  // fused path: the tile kernel writes the angle gradient to the workspace and the
  // exp -> ZYZ VJP runs in the reduce's launch, beside it, instead of on wave 0 of every
  // block after its chain (A/B LV_BWD_TAIL_VJP = 1): 4,096 samples 17.2 -> 15.3 us per
  // fused backward, 512: 10.9 -> 9.9 (profiles/r05_tail_vjp_ab.txt)
  static const int kEnvTailVjp = LV_KNOB("LV_BWD_TAIL_VJP", 0);
  const bool vjp_beside = v && sharedF && p.a.slab_chunked && kEnvReduce == 6 && !kEnvTailVjp;
  if (vjp_beside) {
    p.a.gang = reinterpret_cast<float*>(static_cast<char*>(workspace) + b.ws_gang_off);
    p.a.v = nullptr;
    p.a.mu = nullptr;
  }
  if (int e = kBwdRun[L](p)) return e;
  if (!sharedF) return LV_OK;
  if (vjp_beside) {
    const int nvjp = (int)((n + 255) / 256);
    hipLaunchKernelGGL(action_bwd_reduce5_vjp_kernel, dim3((unsigned)(nvjp + slab_chunks(MC))), dim3(256), 0, st,
                       (const float*)workspace, gF, MC, b.gx, nvjp, mu, v, (const float*)p.a.gang, gmu, gv, n);
    LV_RETURN_LAUNCH("action_bwd_reduce5_vjp_kernel");
  }
  // dF slab reduce: chunk-major slabs + action_bwd_reduce5_kernel by default (kBwdReduceDefault;
  // reduce3 before it, profiles/r04_bwd_reduce_ab.txt: 16.0 vs 18.0 us per lv_group_action_bwd call at batch
  // 4,096, 187 vs 191 at 65,536, 9.9 vs 9.8 at 512 against reduce2<16>, the round-3
  // default; an in-kernel reduction by the tile kernel's last blocks -- completion counter,
  // device-scope release fences -- ran 75 us per call at 4,096 and was dropped)
  if (p.a.slab_chunked && kEnvReduce == 6) {
    hipLaunchKernelGGL(action_bwd_reduce5_kernel, dim3((unsigned)slab_chunks(MC)), dim3(256), 0, st,
                       (const float*)workspace, gF, MC, b.gx);
    LV_RETURN_LAUNCH("action_bwd_reduce5_kernel");
  }
  if (p.a.slab_chunked && kEnvReduce == 5) {
    hipLaunchKernelGGL(action_bwd_reduce4_kernel, dim3((unsigned)slab_chunks(MC)), dim3(1024), 0, st,
                       (const float*)workspace, gF, MC, b.gx);
    LV_RETURN_LAUNCH("action_bwd_reduce4_kernel");
  }
  if (p.a.slab_chunked) {
    hipLaunchKernelGGL(action_bwd_reduce3_kernel, dim3((unsigned)slab_chunks(MC)), dim3(1024), 0, st,
                       (const float*)workspace, gF, MC, b.gx, p.a.stamps);
    LV_RETURN_LAUNCH("action_bwd_reduce3_kernel");
  }
  if (kEnvReduce == 8) {
    hipLaunchKernelGGL(action_bwd_reduce2_kernel<8>, dim3(ceil_div(MC, 8)), dim3(1024), 0, st,
                       (const float*)workspace, gF, MC, b.gx);
    LV_RETURN_LAUNCH("action_bwd_reduce2_kernel");
  } else if (kEnvReduce == 16) {
    hipLaunchKernelGGL(action_bwd_reduce2_kernel<16>, dim3(ceil_div(MC, 16)), dim3(1024), 0, st,
                       (const float*)workspace, gF, MC, b.gx);
    LV_RETURN_LAUNCH("action_bwd_reduce2_kernel");
  } else if (kEnvReduce == 4) {
    hipLaunchKernelGGL(action_bwd_reduce2_kernel<4>, dim3(ceil_div(MC, 4)), dim3(1024), 0, st,
                       (const float*)workspace, gF, MC, b.gx);
    LV_RETURN_LAUNCH("action_bwd_reduce2_kernel");
  }
  hipLaunchKernelGGL(action_bwd_reduce_kernel, dim3(ceil_div(MC, kBwdReduceCols)), dim3(64 * kBwdReduceWaves),
                     0, st, (const float*)workspace, gF, MC, b.gx);
  LV_RETURN_LAUNCH("action_bwd_reduce_kernel");
}
}  // namespace

extern "C" {

int lv_group_action_fwd(const float* ang, const float* F, int64_t F_batch_stride, void* out,
                        int out_dtype, int64_t n, int L, int C, int transpose, void* stream) {
  return action_fwd_common(false, ang, nullptr, nullptr, F, F_batch_stride, out, out_dtype,
                           nullptr, n, L, C, transpose, (hipStream_t)stream);
}

int lv_fused_exp_action_fwd(const float* mu, const float* v, const float* F,
                            int64_t F_batch_stride, void* out, int out_dtype, float* ang_out,
                            int64_t n, int L, int C, int transpose, void* stream) {
  return action_fwd_common(true, nullptr, mu, v, F, F_batch_stride, out, out_dtype, ang_out, n,
                           L, C, transpose, (hipStream_t)stream);
}

int lv_fused_exp_action_fwd_repeat(const float* mu, const float* v, const float* F,
                                   int64_t F_batch_stride, void* out, int out_dtype,
                                   float* ang_out, int64_t n, int L, int C, int transpose,
                                   int repeats, void* stream) {
  for (int r = 0; r < repeats; ++r) {
    const int e = action_fwd_common(true, nullptr, mu, v, F, F_batch_stride, out, out_dtype,
                                    ang_out, n, L, C, transpose, (hipStream_t)stream);
    if (e) return e;
  }
  return LV_OK;
}

size_t lv_group_action_bwd_workspace(int64_t n, int L, int C, int shared_F) {
  if (n <= 0 || L < 0 || L > LV_MAX_DEGREE || C < 1 || C > LV_MAX_CHANNELS) return 0;
  BwdPlan b;
  if (!plan_bwd_cached(n, L, C, shared_F != 0, b)) return 0;
  return b.ws;
}


int lv_group_action_bwd(const float* ang, const float* F, int64_t F_batch_stride,
                        const float* gout, float* gang, float* gF, int64_t n, int L, int C,
                        int transpose, void* workspace, size_t ws_bytes, void* stream) {
  clear_error();
  LV_CHECK_ARG(gang, "null gang");
  return action_bwd_common(ang, F, F_batch_stride, gout, gang, gF, nullptr, nullptr, nullptr,
                           nullptr, n, L, C, transpose, workspace, ws_bytes, stream);
}

int lv_fused_exp_action_bwd(const float* mu, const float* v, const float* ang, const float* F,
                            const float* gout, float* gmu, float* gv, float* gF, int64_t n, int L,
                            int C, int transpose, void* workspace, size_t ws_bytes, void* stream) {
  clear_error();
  if (n > 0) LV_CHECK_ARG(v && gv && (!mu || gmu), "null v / gv / gmu");
  return action_bwd_common(ang, F, 0, gout, nullptr, gF, mu, v, gmu, gv, n, L, C, transpose,
                           workspace, ws_bytes, stream);
}

int lv_action_fwd_plan(int fused, int64_t F_batch_stride, int out_dtype, int64_t n, int L, int C,
                       int64_t* plan) {
  clear_error();
  LV_CHECK_ARG(plan, "null plan");
  LV_CHECK_ARG(n > 0, "n must be > 0 (got %lld)", (long long)n);
  FwdLaunch p;
  if (int e = plan_fwd(fused != 0, F_batch_stride, out_dtype, n, L, C, device_cus(), p)) return e;
  plan[0] = p.tile ? 1 : 0;
  plan[1] = p.gx;
  plan[2] = p.gy;
  plan[3] = p.tile ? 64 * p.gy : kThreads;
  plan[4] = (int64_t)p.lds;
  plan[5] = p.a.Sw;
  plan[6] = p.a.write_through;
  for (int k = 0; k <= kMaxSeg; ++k) plan[7 + k] = k <= p.gy ? p.a.seg_lo[k] : -1;
  for (int k = 0; k < kMaxSeg; ++k) plan[8 + kMaxSeg + k] = k < p.gy ? (int64_t)p.a.seg_mask[k] : 0;
  return LV_OK;
}

int lv_group_action_bwd_plan(int64_t n, int L, int C, int shared_F, int64_t* plan) {
  clear_error();
  LV_CHECK_ARG(plan, "null plan");
  LV_CHECK_ARG(n > 0, "n must be > 0 (got %lld)", (long long)n);
  if (int e = check_common(n, L, C, LV_DTYPE_F32)) return e;
  BwdPlan b;
  LV_CHECK_ARG(plan_bwd(n, L, C, shared_F != 0, device_cus(), b), "no backward plan fits the LDS budget (l=%d, C=%d)", L, C);
  plan[0] = b.persist ? 3 : b.fmode;
  plan[1] = b.gx;
  plan[2] = b.nseg;
  plan[3] = 64 * b.nseg;
  plan[4] = (int64_t)b.lds;
  plan[5] = b.Sw;
  plan[6] = (int64_t)b.ws;
  for (int k = 0; k <= kMaxSeg; ++k) plan[7 + k] = k <= b.nseg ? b.seg_lo[k] : -1;
  for (int k = 0; k < kMaxSeg; ++k) plan[8 + kMaxSeg + k] = k < b.nseg ? (int64_t)b.seg_mask[k] : 0;
  return LV_OK;
}

int lv_compute_units(void) { return device_cus(); }

int lv_wigner_d_fwd(const float* ang, float* D, int64_t n, int L, void* stream) {
  clear_error();
  LV_CHECK_ARG(n >= 0, "n must be >= 0");
  LV_CHECK_ARG(L >= 0 && L <= LV_MAX_DEGREE, "l_max out of range");
  if (n == 0) return LV_OK;
  LV_CHECK_ARG(ang && D, "null pointer");
  WigLaunch p{ang, D, n, (L + 1) * (2 * L + 1) * (2 * L + 3) / 3, (hipStream_t)stream};
  for (int l = 0; l <= L; ++l)
    if (int e = kWigRun[l](p)) return e;
  return LV_OK;
}

#ifdef LV_AB_KNOBS
// Timeline tool (A/B build): copy the phase-timestamp buffer to the host after a device
// synchronise; returns the bytes copied (0 without LV_STAMPS=1).
size_t lv_ab_stamps_copy(void* host, size_t bytes) {
  unsigned long long* p = ab_stamps();
  if (!p || !host) return 0;
  bytes = std::min(bytes, kStampBytes);
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(host, p, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return bytes;
}
#endif

}  // extern "C"

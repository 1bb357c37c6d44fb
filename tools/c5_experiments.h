#pragma once
// Config-5 diagnostics (l = 20, bf16 out): the library's tile kernel with parts switched
// off (compile-time bit mask), to split its time.  Never built into the library.
//   1: no flush   2: no chain (y = x)   4: no LDS tile writes   8: no multiples reads
//   16: no spectrum reads (x = the multiples row)   32: spectrum from global (round-2 first try)
#include "action_fwd.h"

namespace lv {

// ------------------------------------------------------- two-phase tile forward
// (round 3 A/B, profiles/r03_c5_tile2.txt: bitwise equal, but 43.0 us at best against the
// library's 39.5 -- the second barrier and the six per-sample flush runs cost more than
// the third block per CU and the phase-A/phase-B overlap gain)
// High degrees (config 5: l = 20, bf16 out): the whole output tile of a 6-sample group
// (53 KB) plus the spectrum and the multiples (74 KB) leave room for only 2 blocks per
// CU, and each block computes, then flushes, in series.  Here the degrees split into two
// phases, [0, L1) and [L1, L], of about equal row counts; the LDS stage holds one phase
// (L1 = 15 at l = 20: 225 / 216 rows, 27 KB), so the block needs 48 KB (3 per CU), and the
// stores of phase A drain while phase B computes.  Each wave owns one degree segment in
// each phase: a.seg_lo[0..nw] (phase A) and a.seg_lo[nw+1..2nw+1] (phase B).  Every
// output element comes from the same arithmetic as fwd_tile_body (bitwise equal).  A
// phase's rows of one sample are one contiguous run in global memory; each run is staged
// at an LDS address congruent to its global address mod 16 and leaves with tile_flush.
__host__ __device__ constexpr int tile2_pitch(int M, int R1, int C, int out_bytes) {
  return ((((R1 > M - R1 ? R1 : M - R1) * C * out_bytes) + 15) & ~15) + 16;
}

template <int LT, bool FUSED, typename OutT>
__device__ __forceinline__ void fwd_tile2_body(const ActionArgs& a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int CT = 10;
  constexpr int kRow = TrigLds<LT>::kRow;
  constexpr int C = CT, Sw = 64 / CT;
  constexpr int M = (LT + 1) * (LT + 1);
  constexpr int64_t MC = (int64_t)M * CT;
  constexpr int E = (int)sizeof(OutT);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nw = (int)(blockDim.x >> 6);
  const int j = lane / C;
  const int c = lane - j * C;
  const int loA = a.seg_lo[wave], hiA = a.seg_lo[wave + 1];
  const int loB = a.seg_lo[nw + 1 + wave], hiB = a.seg_lo[nw + 2 + wave];
  const int L1 = a.seg_lo[nw];
  const int R1 = L1 * L1;
  const int P = tile2_pitch(M, R1, C, E);
  const int64_t s0 = (int64_t)blockIdx.x * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);
  const bool active = j < Sv;
  char* const stage = reinterpret_cast<char*>(lds);
  float* const trig = lds + (Sw * P >> 2);
  float* const Fall = trig + Sw * kRow;
  OutT* const gbase = reinterpret_cast<OutT*>(a.out) + s0 * MC;
  const int tid = (int)threadIdx.x;
  // 1. prologue tasks and this wave's spectrum rows (both phases), as fwd_tile_body
  const bool task = tid < 3 * Sw;
  const int jt = tid / 3, q = tid - 3 * (tid / 3);
  const int64_t st = s0 + min(jt, Sv - 1);
  LaneIn in;
  if (task) lane_load<FUSED>(a, st, in);
  if (task) {
    float c1[3], s1[3];
    lane_angles<FUSED>(a, in, st, jt < Sv, q, FUSED && a.ang_out != nullptr, c1, s1);
    trig_row_fill<LT>(trig + jt * kRow, c1, s1, q, LT);
  }
  for (int e = loA * loA * C + lane; e < hiA * hiA * C; e += 64) Fall[e] = a.F[e];
  for (int e = loB * loB * C + lane; e < hiB * hiB * C; e += 64) Fall[e] = a.F[e];
  block_sync_lds();
  const float* tj = trig + min(j, Sw - 1) * kRow;
  const float* Fl = Fall + c;
  auto chain = [&](int lo, int hi, int rstart) {
    // this lane's stage row pointer for the phase starting at row rstart
    const int mis = (int)(reinterpret_cast<uintptr_t>(gbase + j * MC + rstart * C) & 15);
    OutT* st_lane = reinterpret_cast<OutT*>(stage + j * P + mis) + c;
    sfor<LT + 1>([&](auto Lc) {
      constexpr int l = LV_CV(Lc);
      if (l >= lo && l < hi) {
        constexpr int nn = 2 * l + 1;
        constexpr int r0 = l * l;
        float x[nn], y[nn];
        sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[(r0 + LV_CV(K)) * C]; });
        xrot_lds<l, 2, LT>(tj, x, y);
        jmul<l>(y, x);
        xrot_lds<l, 1, LT>(tj, x, y);
        jmul<l>(y, x);
        xrot_lds<l, 0, LT>(tj, x, y);
        if (active) {
          OutT* d = st_lane + (r0 - rstart) * C;
          sfor<nn>([&](auto I) {
            d[0] = tile_cvt(y[LV_CV(I)], (OutT*)nullptr);
            d += C;
          });
        }
      }
    });
  };
  auto flush = [&](int rstart, int rows) {
    for (int jj = 0; jj < Sv; ++jj) {
      OutT* g = gbase + jj * MC + rstart * C;
      const int mis = (int)(reinterpret_cast<uintptr_t>(g) & 15);
      tile_flush_rt<OutT>(g, stage + jj * P + mis, mis, rows * C * E, a.write_through);
    }
  };
  // 2. phase A, flush A (its stores drain during phase B), phase B, flush B.  One copy
  //    of the chain code in a two-trip loop (two inlined copies double the registers).
  for (int ph = 0; ph < 2; ++ph) {
    const int rstart = ph ? R1 : 0;
    if (ph) block_sync_lds();  // every stage read of flush A has returned: stage is free
    chain(ph ? loB : loA, ph ? hiB : hiA, rstart);
    block_sync_lds();
    flush(rstart, ph ? M - R1 : R1);
  }
}

template <int LT, bool FUSED, typename OutT>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(5))) void action_fwd_tile2_kernel(ActionArgs a) {
  fwd_tile2_body<LT, FUSED, OutT>(a);
}

template <int LT, int DIAG>
__global__ __launch_bounds__(512) void c5_diag_kernel(ActionArgs a) {
  using OutT = __hip_bfloat16;
  constexpr int CT = 10;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int kRow = TrigLds<LT>::kRow;
  const int C = CT, Sw = 64 / CT;
  constexpr int64_t MC = (int64_t)(LT + 1) * (LT + 1) * CT;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int64_t s0 = (int64_t)blockIdx.x * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);
  const bool active = j < Sv;
  const int stage_bytes = tile_stage_bytes(Sw, MC, (int)sizeof(OutT));
  float* trig = lds + (stage_bytes >> 2);
  const int tid = (int)threadIdx.x;
  const bool task = tid < 3 * Sw;
  const int jt = tid / 3, q = tid - 3 * (tid / 3);
  const int64_t st = s0 + min(jt, Sv - 1);
  LaneIn in;
  if (task) lane_load<true>(a, st, in);
  if (task) {
    float c1[3], s1[3];
    lane_angles<true>(a, in, st, jt < Sv, q, false, c1, s1);
    trig_row_fill<LT>(trig + jt * kRow, c1, s1, q, LT);
  }
  float* Fsh = trig + Sw * kRow;  // whole F, row-major, as the library
  if constexpr ((DIAG & 48) == 0) {
    const int rows_lo = lo * lo;
    for (int e = lane; e < (hi * hi - rows_lo) * C; e += 64) Fsh[rows_lo * C + e] = a.F[rows_lo * C + e];
  }
  block_sync_lds();
  OutT* gout = reinterpret_cast<OutT*>(a.out) + s0 * MC;
  const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
  char* stage_b = reinterpret_cast<char*>(lds) + mis;
  OutT* st_lane = reinterpret_cast<OutT*>(stage_b) + j * MC + c;
  const float* tj = trig + min(j, Sw - 1) * kRow;
  const float* Fl = (DIAG & 32) ? a.F + c : (DIAG & 16) ? tj : Fsh + c;
  const int fs = (DIAG & 16) ? 0 : C;
  float keep = 0.f;
  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if (l >= lo && l < hi) {
      constexpr int nn = 2 * l + 1;
      constexpr int r0 = l * l;
      float x[nn], y[nn];
      sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[(r0 + LV_CV(K)) * fs + ((DIAG & 16) ? LV_CV(K) % 8 : 0)]; });
      if constexpr ((DIAG & 2) != 0) {
        sfor<nn>([&](auto K) { y[LV_CV(K)] = x[LV_CV(K)]; });
      } else if constexpr ((DIAG & 8) != 0) {
        TrigTab<l> t;
        sfor<3>([&](auto A) { sfor<l + 1>([&](auto F) { t.c[LV_CV(A)][LV_CV(F)] = x[LV_CV(F)]; t.s[LV_CV(A)][LV_CV(F)] = x[LV_CV(F) + 1]; }); });
        xrot<l, 2>(t, x, y);
        jmul<l>(y, x);
        xrot<l, 1>(t, x, y);
        jmul<l>(y, x);
        xrot<l, 0>(t, x, y);
      } else {
        xrot_lds<l, 2, LT>(tj, x, y);
        jmul<l>(y, x);
        xrot_lds<l, 1, LT>(tj, x, y);
        jmul<l>(y, x);
        xrot_lds<l, 0, LT>(tj, x, y);
      }
      if constexpr ((DIAG & 4) != 0) {
        sfor<nn>([&](auto I) { keep += y[LV_CV(I)]; });
      } else if (active) {
        OutT* d = st_lane + r0 * C;
        sfor<nn>([&](auto I) {
          d[0] = tile_cvt(y[LV_CV(I)], (OutT*)nullptr);
          d += C;
        });
      }
    }
  });
  if constexpr ((DIAG & 4) != 0)
    if (keep == 1234.5f) reinterpret_cast<float*>(a.out)[threadIdx.x] = keep;
  block_sync_lds();
  if constexpr ((DIAG & 1) == 0)
    tile_flush<OutT, 1>(gout, stage_b, mis, Sv * (int)MC * (int)sizeof(OutT), tid, (int)blockDim.x);
}
}  // namespace lv

namespace lv {
// Persistent tile kernel for large l: grid of a few blocks per CU, each looping over
// sample groups; the task lanes prefetch the next group's v while the chain of the
// current group runs, so the per-group prologue latency is not exposed block after block.
template <int LT>
__global__ __launch_bounds__(512) void c5_persist_kernel(ActionArgs a) {
  using OutT = __hip_bfloat16;
  constexpr int CT = 10;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int kRow = TrigLds<LT>::kRow;
  const int C = CT, Sw = 64 / CT;
  constexpr int64_t MC = (int64_t)(LT + 1) * (LT + 1) * CT;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int64_t groups = (a.n + Sw - 1) / Sw;
  const int stage_bytes = tile_stage_bytes(Sw, MC, (int)sizeof(OutT));
  float* trig = lds + (stage_bytes >> 2);
  const int tid = (int)threadIdx.x;
  const bool task = tid < 3 * Sw;
  const int jt = tid / 3, q = tid - 3 * (tid / 3);
  const float* Fl = a.F + c;
  LaneIn in;
  int64_t g = blockIdx.x;
  if (task && g < groups) lane_load<true>(a, min(g * Sw + jt, a.n - 1), in);
  for (; g < groups; g += gridDim.x) {
    const int64_t s0 = g * Sw;
    const int Sv = (int)min((int64_t)Sw, a.n - s0);
    const bool active = j < Sv;
    if (task) {
      float c1[3], s1[3];
      const int64_t st = s0 + min(jt, Sv - 1);
      lane_angles<true>(a, in, st, jt < Sv, q, false, c1, s1);
      trig_row_fill<LT>(trig + jt * kRow, c1, s1, q, LT);
    }
    block_sync_lds();
    const int64_t gn = g + gridDim.x;  // prefetch the next group's inputs
    if (task && gn < groups) lane_load<true>(a, min(gn * Sw + jt, a.n - 1), in);
    OutT* gout = reinterpret_cast<OutT*>(a.out) + s0 * MC;
    const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
    char* stage_b = reinterpret_cast<char*>(lds) + mis;
    OutT* st_lane = reinterpret_cast<OutT*>(stage_b) + j * MC + c;
    const float* tj = trig + min(j, Sw - 1) * kRow;
    sfor<LT + 1>([&](auto Lc) {
      constexpr int l = LV_CV(Lc);
      if (l >= lo && l < hi) {
        constexpr int nn = 2 * l + 1;
        constexpr int r0 = l * l;
        float x[nn], y[nn];
        sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[(r0 + LV_CV(K)) * C]; });
        xrot_lds<l, 2, LT>(tj, x, y);
        jmul<l>(y, x);
        xrot_lds<l, 1, LT>(tj, x, y);
        jmul<l>(y, x);
        xrot_lds<l, 0, LT>(tj, x, y);
        if (active) {
          OutT* d = st_lane + r0 * C;
          sfor<nn>([&](auto I) {
            d[0] = tile_cvt(y[LV_CV(I)], (OutT*)nullptr);
            d += C;
          });
        }
      }
    });
    block_sync_lds();
    tile_flush<OutT, 1>(gout, stage_b, mis, Sv * (int)MC * (int)sizeof(OutT), tid, (int)blockDim.x);
    block_sync_lds();
  }
}
}  // namespace lv

namespace lv {
// Launch floor with the config-5 grid: (0) empty, (1) + the task lanes' v loads and
// prologue maths + one barrier.
template <int MODE>
__global__ __launch_bounds__(512) void c5_floor_kernel(ActionArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if constexpr (MODE == 0) {
    if (a.n < 0) reinterpret_cast<float*>(a.out)[threadIdx.x] = lds[threadIdx.x];
  } else {
    constexpr int LT = 20;
    const int tid = (int)threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * 6;
    if (tid < 18) {
      LaneIn in;
      const int jt = tid / 3, q = tid - 3 * (tid / 3);
      lane_load<true>(a, min(s0 + jt, a.n - 1), in);
      float c1[3], s1[3];
      lane_angles<true>(a, in, s0 + jt, true, q, false, c1, s1);
      trig_row_fill<LT>(lds + jt * TrigLds<LT>::kRow, c1, s1, q, LT);
    }
    block_sync_lds();
    if (lds[threadIdx.x & 63] == 1234.5f) reinterpret_cast<float*>(a.out)[threadIdx.x] = 1.f;
  }
}
template <int LT>
__global__ __launch_bounds__(512) void c5_nomu_kernel(ActionArgs a) {
  fwd_tile_body<LT, 10, true, __hip_bfloat16, false>(a, blockIdx.x);
}

// the two-phase body without the 5-waves-per-SIMD register cap (105 VGPRs, no spills)
template <int LT>
__global__ __launch_bounds__(512) void c5_tile2_free_kernel(ActionArgs a) {
  fwd_tile2_body<LT, true, __hip_bfloat16>(a);
}

}  // namespace lv

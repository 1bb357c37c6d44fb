#pragma once
// Experimental forward variants kept for tools/tilebench.hip A/B runs (never built into
// the library).  v2 shares the per-sample prologue through LDS: it measured slower
// (wave 0's prologue latency serialises the block).
#include "action_fwd.h"

namespace lv {

// Tile forward, v2: the per-sample prologue (load v, exp -> ZYZ (cos, sin), multiples by
// recurrence) runs ONCE per (sample, Euler slot) on wave 0's lanes and is shared through
// an LDS table, instead of on every lane of every segment wave.  The other waves stage
// their spectrum slices meanwhile; one block barrier publishes the table.
__host__ __device__ constexpr int trig_pitch(int LT) { return (LT + 1 + 3) & ~3; }
__host__ __device__ inline int tile2_trig_floats(int Sw, int LT) { return Sw * 6 * trig_pitch(LT); }

template <int LT, bool FUSED, typename OutT, int POL>
__global__ __launch_bounds__(512) void action_fwd_tile2_kernel(ActionArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  LV_STAMP(0);
  constexpr int TP = trig_pitch(LT);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int C = a.C, Sw = a.Sw;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int rows_lo = lo * lo;
  const int frows = fseg_rows(lo, hi);
  const int64_t MC = a.MC;
  const int64_t s0 = (int64_t)blockIdx.x * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);  // >= 1: grid = ceil(n / Sw)
  const bool active = j < Sv;
  const int stage_bytes = tile_stage_bytes(Sw, MC, (int)sizeof(OutT));
  float* trig = lds + (stage_bytes >> 2);
  float* Fw = trig + tile2_trig_floats(Sw, LT) + wave * a.fpitch;
  // spectrum slice loads (every wave)
  constexpr int kFPer = 6;
  float fv[kFPer];
  const int fcnt = (hi * hi - rows_lo) * C;
  const float* fsrc = a.F + rows_lo * C;
#pragma unroll
  for (int k = 0; k < kFPer; ++k) {
    const int e = lane + 64 * k;
    fv[k] = e < fcnt ? fsrc[e] : 0.f;
  }
  if (wave == 0) {
    // task = (sample jj, Euler slot q): full prologue, keep slot q, its multiples
    for (int task = lane; task < Sw * 3; task += 64) {
      const int jj = task / 3, q = task - jj * 3;
      const int64_t s = jj < Sv ? s0 + jj : s0;  // idle slots mirror a valid sample
      LaneIn in;
      lane_load<FUSED>(a, s, in);
      float c1[3], s1[3];
      lane_angles<FUSED>(a, in, s, jj < Sv, q, FUSED && a.ang_out, c1, s1);
      const float cq = q == 0 ? c1[0] : (q == 1 ? c1[1] : c1[2]);
      const float sq = q == 0 ? s1[0] : (q == 1 ? s1[1] : s1[2]);
      float* tc = trig + (jj * 3 + q) * 2 * TP;
      float* ts = tc + TP;
      float cf = 1.f, sf = 0.f;
      tc[0] = 1.f;
      ts[0] = 0.f;
#pragma unroll
      for (int f = 1; f <= LT; ++f) {
        if (f == 1) {
          cf = cq;
          sf = sq;
        } else {
          const float cn = fmaf(cf, cq, -(sf * sq));
          sf = fmaf(sf, cq, cf * sq);
          cf = cn;
        }
        tc[f] = cf;
        ts[f] = sf;
      }
    }
  }
  LV_STAMP(1);
#pragma unroll
  for (int k = 0; k < kFPer; ++k) {
    const int e = lane + 64 * k;
    if (e < fcnt) {
      const int r = e / C, cc = e - r * C;
      Fw[cc * frows + r] = fv[k];
    }
  }
  for (int e = lane + 64 * kFPer; e < fcnt; e += 64) {
    const int r = e / C, cc = e - r * C;
    Fw[cc * frows + r] = fsrc[e];
  }
  __syncthreads();
  LV_STAMP(2);
  TrigTab<LT> t;
  {
    const float* tj = trig + j * 6 * TP;
    sfor<3>([&](auto A) {
      constexpr int q = LV_CV(A);
      sfor<LT + 1>([&](auto Fc) {
        constexpr int f = LV_CV(Fc);
        if (f < hi) {
          t.c[q][f] = tj[(q * 2) * TP + f];
          t.s[q][f] = tj[(q * 2 + 1) * TP + f];
        }
      });
    });
  }

  OutT* gout = reinterpret_cast<OutT*>(a.out) + s0 * MC;
  const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
  char* stage_b = reinterpret_cast<char*>(lds) + mis;  // LDS addr = global addr (mod 16)
  OutT* st_lane = reinterpret_cast<OutT*>(stage_b) + j * MC + c;
  const float* Fl = Fw + c * frows - rows_lo;

  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if (l >= lo && l < hi) {
      constexpr int nn = 2 * l + 1;
      constexpr int r0 = l * l;
      float x[nn], y[nn];
      sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[r0 + LV_CV(K)]; });
      xrot<l, 2>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 1>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 0>(t, x, y);
      if (active) {
        OutT* d = st_lane + r0 * C;
        sfor<nn>([&](auto I) {
          d[0] = tile_cvt(y[LV_CV(I)], (OutT*)nullptr);
          d += C;
        });
      }
    }
  });
  LV_STAMP(5);
  __syncthreads();
  LV_STAMP(3);
  tile_flush<OutT, POL>(gout, stage_b, mis, Sv * (int)MC * (int)sizeof(OutT));
  LV_STAMP(4);
}

// Pipelined (persistent-style) tile forward, kept for tools/tilebench.hip (mode 2/3).
// Measured on MI355X at batch 4096, l = 10: 10.7-18 us vs 7.65 us for the one-shot
// tile kernel: with 4-8 waves per CU every phase of a group is
// latency-bound (stamps: spectrum staging 1.2, shared prologue 1.7, chain 2.2, flush
// issue 1.1 us), so the saving from overlapping stores with compute is lost.

// --------------------------------------------------------- pipelined tile forward
// Persistent-style variant of the tile kernel (shared spectrum).  In the one-shot tile
// kernel every block computes, then every block stores, so the chip alternates between a
// VALU phase with HBM idle and a store phase with VALU idle.  Here a block walks the
// sample groups g = blockIdx.x + k*gridDim.x with two LDS tiles: group k's stores are
// issued (never waited for) and drain while the waves compute group k+1.
//   * The per-sample prologue (v -> ZYZ (cos, sin) -> multiples) runs once per
//     (sample, Euler slot) on wave 0's lanes for a chunk of KC groups and is shared through
//     an LDS table; the other waves never evaluate it.
//   * Wave 0 issues no global stores (waves 1.. flush), so its later v loads never wait
//     behind store traffic (vmcnt retires in order).
//   * Spectrum slices are staged once per block, not once per group.
//   * Barriers are s_barrier + lgkmcnt(0) only (block_sync_lds), never vmcnt.
// Same per-element arithmetic as action_fwd_tile_kernel (trig_fill's recurrence, the
// chain): outputs are bitwise identical.
__host__ __device__ constexpr int trig_row(int LT) { return (LT + 1 + 3) & ~3; }
__host__ __device__ inline int tilep_chunk(int Sw) { return 64 / (3 * Sw) > 0 ? 64 / (3 * Sw) : 1; }
__host__ __device__ inline int tilep_trig_floats(int Sw, int LT) {
  return tilep_chunk(Sw) * Sw * 6 * trig_row(LT);
}

template <int LT, bool FUSED, typename OutT>
__global__ __launch_bounds__(512) void action_fwd_tilep_kernel(ActionArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  LV_STAMP(0);
  constexpr int TP = trig_row(LT);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int C = a.C, Sw = a.Sw;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int rows_lo = lo * lo;
  const int frows = fseg_rows(lo, hi);
  const int64_t MC = a.MC;
  const int64_t groups = (a.n + Sw - 1) / Sw;
  const int64_t G = gridDim.x;
  const int ngb = (int)((groups - blockIdx.x + G - 1) / G);  // >= 1: grid <= groups
  const int KC = tilep_chunk(Sw);
  const int tile_bytes = tile_stage_bytes(Sw, MC, (int)sizeof(OutT));
  char* tiles = reinterpret_cast<char*>(lds);
  float* trig = reinterpret_cast<float*>(tiles + 2 * tile_bytes);
  float* Fw = trig + tilep_trig_floats(Sw, LT) + wave * a.fpitch;

  // this wave's spectrum slice, once
  {
    const int fcnt = (hi * hi - rows_lo) * C;
    const float* fsrc = a.F + rows_lo * C;
    for (int e = lane; e < fcnt; e += 64) {
      const int r = e / C, cc = e - r * C;
      Fw[cc * frows + r] = fsrc[e];
    }
  }
  const float* Fl = Fw + c * frows - rows_lo;
  LV_STAMP(1);

  for (int k = 0; k < ngb; ++k) {
    if (k % KC == 0) {
      if (wave == 0) {
        // task = (group kk of the chunk, sample jj, Euler slot q)
        const int ntask = KC * Sw * 3;
        for (int task = lane; task < ntask; task += 64) {
          const int kk = task / (3 * Sw);
          const int rem = task - kk * 3 * Sw;
          const int jj = rem / 3, q = rem - jj * 3;
          const int64_t g = blockIdx.x + (int64_t)(k + kk) * G;
          int64_t s = g * Sw + jj;
          const bool valid = g < groups && s < a.n;
          if (!valid) s = a.n - 1;  // computed, never used
          LaneIn in;
          lane_load<FUSED>(a, s, in);
          float c1[3], s1[3];
          lane_angles<FUSED>(a, in, s, valid, q, FUSED && a.ang_out, c1, s1);
          const float cq = q == 0 ? c1[0] : (q == 1 ? c1[1] : c1[2]);
          const float sq = q == 0 ? s1[0] : (q == 1 ? s1[1] : s1[2]);
          float* tc = trig + ((kk * Sw + jj) * 6 + 2 * q) * TP;
          float* ts = tc + TP;
          float cf = 1.f, sf = 0.f;
          tc[0] = 1.f;
          ts[0] = 0.f;
#pragma unroll
          for (int f = 1; f <= LT; ++f) {
            if (f == 1) {
              cf = cq;
              sf = sq;
            } else {  // trig_fill's recurrence, same rounding
              const float cn = fmaf(cf, cq, -(sf * sq));
              sf = fmaf(sf, cq, cf * sq);
              cf = cn;
            }
            tc[f] = cf;
            ts[f] = sf;
          }
        }
      }
      block_sync_lds();
    }
    if (k == 0) LV_STAMP(2);
    const int64_t s0 = (blockIdx.x + (int64_t)k * G) * Sw;
    const int Sv = (int)min((int64_t)Sw, a.n - s0);
    const bool active = j < Sv;
    TrigTab<LT> t;
    {
      const float* tj = trig + (((k % KC) * Sw + min(j, Sw - 1)) * 6) * TP;
      sfor<3>([&](auto A) {
        constexpr int q = LV_CV(A);
        sfor<LT + 1>([&](auto Fc) {
          constexpr int f = LV_CV(Fc);
          if (f < hi) {
            t.c[q][f] = tj[(2 * q) * TP + f];
            t.s[q][f] = tj[(2 * q + 1) * TP + f];
          }
        });
      });
    }
    OutT* gout = reinterpret_cast<OutT*>(a.out) + s0 * MC;
    const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
    char* stage_b = tiles + (k & 1) * tile_bytes + mis;  // LDS addr = global addr (mod 16)
    OutT* st_lane = reinterpret_cast<OutT*>(stage_b) + j * MC + c;
    sfor<LT + 1>([&](auto Lc) {
      constexpr int l = LV_CV(Lc);
      if (l >= lo && l < hi) {
        constexpr int nn = 2 * l + 1;
        constexpr int r0 = l * l;
        float x[nn], y[nn];
        sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[r0 + LV_CV(K)]; });
        xrot<l, 2>(t, x, y);
        jmul<l>(y, x);
        xrot<l, 1>(t, x, y);
        jmul<l>(y, x);
        xrot<l, 0>(t, x, y);
        if (active) {
          OutT* d = st_lane + r0 * C;
          sfor<nn>([&](auto I) {
            d[0] = tile_cvt(y[LV_CV(I)], (OutT*)nullptr);
            d += C;
          });
        }
      }
    });
    if (k == 0) LV_STAMP(3);
    block_sync_lds();
    if (k == 0) LV_STAMP(4);
    if (wave > 0)
      tile_flush_rt<OutT>(gout, stage_b, mis, Sv * (int)MC * (int)sizeof(OutT), a.write_through,
                          (int)threadIdx.x - 64, (int)blockDim.x - 64);
    if (k == 0) LV_STAMP(5);
  }
  LV_STAMP(6);
}


}  // namespace lv

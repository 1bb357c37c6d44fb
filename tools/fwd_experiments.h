#pragma once
// Experimental forward variants for tools/fwdbench.hip A/B runs (never built into the
// library).  "Stream" kernels: one block per sample group and one wave per degree
// segment, as the tile kernel, but with NO block barrier -- every wave writes the rows of
// each degree as soon as they are computed, so the store stream overlaps the chain maths
// of the other waves instead of starting after all of it.
//   MODE 0: the degree's rows of the wave's Sv samples are staged in a wave-private LDS
//           chunk ([j][row][c], the global layout) and leave as Sv contiguous runs of
//           8-byte buffer stores (512 contiguous bytes per wave instruction).
//   MODE 1: row-pair stores straight from registers (DPP swap of adjacent lanes), 8-byte
//           buffer stores, no LDS.
#include "action_fwd.h"

namespace lv {

typedef unsigned int lv_u2 __attribute__((ext_vector_type(2)));
template <int POL>
__device__ __forceinline__ void st_b64(__amdgpu_buffer_rsrc_t r, int off, float a, float b) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(lv_u2, make_float2(a, b)), r, off, 0,
                                        POL);
}
template <int POL>
__device__ __forceinline__ void st_b32(__amdgpu_buffer_rsrc_t r, int off, float a) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, a), r, off, 0, POL);
}

__host__ __device__ constexpr int stream_chunk_rows(int LT, int FL) {
  return (2 * LT + 1) > FL * FL ? 2 * LT + 1 : FL * FL;
}
// Per-sample pitch of the staging chunk: >= rows*C and == C (mod 64), so that lanes
// (j, c) of one row write 64 distinct banks; even, for 8-byte reads.
__host__ __device__ constexpr int stream_stage_pitch(int LT, int C, int FL) {
  return stream_chunk_rows(LT, FL) * C + (((C - stream_chunk_rows(LT, FL) * C) % 64) + 64) % 64;
}

template <int LT, int C, bool FUSED, int POL, int MODE, int FL>
__global__ __launch_bounds__(512) void fwd_stream_kernel(ActionArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int Sw = 64 / C;
  constexpr int MC = (LT + 1) * (LT + 1) * C;
  constexpr int SP = stream_stage_pitch(LT, C, FL);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int rows_lo = lo * lo;
  const int frows = fseg_rows(lo, hi);
  const int64_t s0 = (int64_t)blockIdx.x * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);
  const bool active = j < Sv;
  const int64_t s = active ? s0 + j : s0;
  LaneIn in;
  lane_load<FUSED>(a, s, in);
  constexpr int kFPer = 6;
  float fv[kFPer];
  const int fcnt = (hi * hi - rows_lo) * C;
  const float* fsrc = a.F + rows_lo * C;
#pragma unroll
  for (int k = 0; k < kFPer; ++k) {
    const int e = lane + 64 * k;
    fv[k] = e < fcnt ? fsrc[e] : 0.f;
  }
  float c1[3], s1[3];
  TrigTab<LT> t;
  lane_angles<FUSED>(a, in, s, active, c, FUSED && a.ang_out && wave == 0, c1, s1);
  trig_fill<LT>(t, c1, s1, hi - 1);
  const int wfl = a.fpitch + (MODE == 0 ? Sw * SP : 0);  // floats per wave
  float* Fw = lds + wave * wfl;
  float* stage = Fw + a.fpitch;
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
  wave_lds_sync();

  float* gout = reinterpret_cast<float*>(a.out) + s0 * MC;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(gout, 0, Sv * MC * 4, kRawBufferFlags);
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
      if constexpr (MODE == 0) {
        // chunk = rows [R0, (l+1)^2); degrees below FL accumulate from the segment start
        const int R0 = l >= FL ? r0 : rows_lo;
        float* d = stage + j * SP + (r0 - R0) * C + c;
        if (active) sfor<nn>([&](auto I) { d[LV_CV(I) * C] = y[LV_CV(I)]; });
        if (l + 1 == hi || l + 1 >= FL) {
          constexpr int R1 = (l + 1) * (l + 1);
          if constexpr (l >= FL) {
            constexpr int NP = nn * C / 2;
            constexpr int K = (Sw * NP + 63) / 64;
            const int tot = Sv * NP;
#pragma unroll
            for (int k = 0; k < K; ++k) {
              const int e = lane + 64 * k;
              if (e < tot) {
                const int jj = e / NP, w = e - jj * NP;
                const float2 v = *reinterpret_cast<const float2*>(stage + jj * SP + 2 * w);
                st_b64<POL>(rs, (jj * MC + r0 * C + 2 * w) * 4, v.x, v.y);
              }
            }
          } else {
            const int np = (R1 - R0) * C / 2;
            const float inv = 1.f / (float)np;
            const int tot = Sv * np;
            for (int e = lane; e < tot; e += 64) {
              const int jj = (int)(((float)e + 0.5f) * inv), w = e - jj * np;
              const float2 v = *reinterpret_cast<const float2*>(stage + jj * SP + 2 * w);
              st_b64<POL>(rs, (jj * MC + R0 * C + 2 * w) * 4, v.x, v.y);
            }
          }
        }
      } else {
        const bool odd = (c & 1) != 0;
        int off = (j * MC + r0 * C + (odd ? C + c - 1 : c)) * 4;
        sfor<nn / 2>([&](auto P) {
          constexpr int i = 2 * LV_CV(P);
          const float send = odd ? y[i] : y[i + 1];
          const float recv = dpp_swap_adjacent(send);
          const float v0 = odd ? recv : y[i];
          const float v1 = odd ? y[i + 1] : recv;
          if (active) st_b64<POL>(rs, off, v0, v1);
          off += 2 * C * 4;
        });
        if (active) st_b32<POL>(rs, (j * MC + (r0 + nn - 1) * C + c) * 4, y[nn - 1]);
      }
    }
  });
}

}  // namespace lv

namespace lv {
// Tile kernel with parts switched off, to split its time into chain maths and stores:
// (bit mask; 0 = the library's tile kernel with a compile-time C = 10):
//   1: no flush (the tile is computed and parked in LDS, never written out)
//   2: no chain (the spectrum slice is copied through, y = x * cos(a))
//   3: no chain, no LDS tile: the flush writes whatever the tile holds (store floor
//      with the kernel's own launch shape and store pattern)
//   4: trivial prologue (v loaded, no exp -> ZYZ maths)
//   8: no multiples recurrence (every multiple = the angle's own cos / sin)
template <int LT, int POL, int DIAG>
__global__ __launch_bounds__(512) void tile_diag_kernel(ActionArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int C = 10;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int Sw = 64 / C;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int rows_lo = lo * lo;
  const int frows = fseg_rows(lo, hi);
  const int64_t MC = a.MC;
  const int64_t s0 = (int64_t)blockIdx.x * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);
  const bool active = j < Sv;
  const int64_t s = active ? s0 + j : s0;
  LaneIn in;
  lane_load<true>(a, s, in);
  constexpr int kFPer = 6;
  float fv[kFPer];
  const int fcnt = (hi * hi - rows_lo) * C;
  const float* fsrc = a.F + rows_lo * C;
#pragma unroll
  for (int k = 0; k < kFPer; ++k) {
    const int e = lane + 64 * k;
    fv[k] = e < fcnt ? fsrc[e] : 0.f;
  }
  float c1[3], s1[3];
  TrigTab<LT> t;
  if constexpr ((DIAG & 4) != 0) {  // trivial prologue (loads kept)
#pragma unroll
    for (int i = 0; i < 3; ++i) { c1[i] = in.v[i]; s1[i] = in.v[(i + 1) % 3]; }
  } else {
    lane_angles<true>(a, in, s, active, c, false, c1, s1);
  }
  if constexpr ((DIAG & 8) != 0) {  // no multiples recurrence
    sfor<3>([&](auto A) {
      sfor<LT + 1>([&](auto F) {
        t.c[LV_CV(A)][LV_CV(F)] = c1[LV_CV(A)];
        t.s[LV_CV(A)][LV_CV(F)] = s1[LV_CV(A)];
      });
    });
  } else {
    trig_fill<LT>(t, c1, s1, hi - 1);
  }
  const int stage_bytes = tile_stage_bytes(Sw, MC, 4);
  float* Fw = lds + (stage_bytes >> 2) + wave * a.fpitch;
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
  wave_lds_sync();
  float* gout = reinterpret_cast<float*>(a.out) + s0 * MC;
  const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
  char* stage_b = reinterpret_cast<char*>(lds) + mis;
  float* st_lane = reinterpret_cast<float*>(stage_b) + j * MC + c;
  const float* Fl = Fw + c * frows - rows_lo;
  if constexpr ((DIAG & 3) != 3) {
    sfor<LT + 1>([&](auto Lc) {
      constexpr int l = LV_CV(Lc);
      if (l >= lo && l < hi) {
        constexpr int nn = 2 * l + 1;
        constexpr int r0 = l * l;
        float x[nn], y[nn];
        sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[r0 + LV_CV(K)]; });
        if constexpr ((DIAG & 2) != 0) {
          sfor<nn>([&](auto K) { y[LV_CV(K)] = x[LV_CV(K)] * t.c[0][1]; });
        } else {
          xrot<l, 2>(t, x, y);
          jmul<l>(y, x);
          xrot<l, 1>(t, x, y);
          jmul<l>(y, x);
          xrot<l, 0>(t, x, y);
        }
        if (active) {
          float* d = st_lane + r0 * C;
          sfor<nn>([&](auto I) {
            d[0] = y[LV_CV(I)];
            d += C;
          });
        }
      }
    });
  }
  __syncthreads();
  if constexpr ((DIAG & 1) == 0)
    tile_flush<float, POL>(gout, stage_b, mis, Sv * (int)MC * 4, (int)threadIdx.x, (int)blockDim.x);
}
}  // namespace lv

namespace lv {
// Tile kernel v3: the tile kernel with the per-sample prologue computed ONCE per
// (sample, Euler slot) instead of on every lane of every segment wave.  Wave 0's lanes
// t < 3*Sw each take one (sample j, slot q): load v, exp -> ZYZ (cos, sin), then the
// multiples of slot q by the same recurrence as trig_fill (bitwise identical), into an
// LDS table; one block barrier publishes it and every wave reads its sample's rows into
// registers with 16-byte LDS reads.  Compile-time C; the spectrum slice is staged
// row-major ([row][c], no index division).
__host__ __device__ constexpr int t3_tp(int LT) { return (LT + 1 + 3) & ~3; }
__host__ __device__ constexpr int t3_row(int LT) { return 2 * t3_tp(LT); }  // cos | sin

template <int LT, int CT, bool FUSED, typename OutT, int POL>
__global__ __launch_bounds__(512) void tile3_kernel(ActionArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int C = CT, Sw = 64 / C;
  constexpr int MC = (LT + 1) * (LT + 1) * C;
  constexpr int TP = t3_tp(LT), TR = t3_row(LT);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int rows_lo = lo * lo;
  const int64_t s0 = (int64_t)blockIdx.x * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);
  const bool active = j < Sv;
  constexpr int stage_bytes = ((Sw * MC * (int)sizeof(OutT) + 16) + 15) & ~15;
  float* trig = lds + stage_bytes / 4;
  float* Fw = trig + Sw * 3 * TR + wave * a.fpitch;
  // prologue task (wave 0): (sample jt, slot q)
  const bool task = wave == 0 && lane < 3 * Sw;
  const int jt = lane / 3, q = lane - 3 * (lane / 3);
  LaneIn in;
  if (task) lane_load<FUSED>(a, s0 + min(jt, Sv - 1), in);
  // spectrum slice, row-major
  constexpr int kFPer = 6;
  float fv[kFPer];
  const int fcnt = (hi * hi - rows_lo) * C;
  const float* fsrc = a.F + rows_lo * C;
#pragma unroll
  for (int k = 0; k < kFPer; ++k) {
    const int e = lane + 64 * k;
    fv[k] = e < fcnt ? fsrc[e] : 0.f;
  }
  if (task) {
    float c1[3], s1[3];
    lane_angles<FUSED>(a, in, s0 + min(jt, Sv - 1), jt < Sv, q, FUSED && a.ang_out != nullptr,
                       c1, s1);
    const float cq = q == 0 ? c1[0] : (q == 1 ? c1[1] : c1[2]);
    const float sq = q == 0 ? s1[0] : (q == 1 ? s1[1] : s1[2]);
    float* tc = trig + (jt * 3 + q) * TR;
    float* ts = tc + TP;
    tc[0] = 1.f;
    ts[0] = 0.f;
    float cf = cq, sf = sq;
    sfor<LT + 1>([&](auto F) {
      constexpr int f = LV_CV(F);
      if constexpr (f >= 1) {
        if constexpr (f >= 2) {
          const float cn = fmaf(cf, cq, -(sf * sq));
          sf = fmaf(sf, cq, cf * sq);
          cf = cn;
        }
        tc[f] = cf;
        ts[f] = sf;
      }
    });
  }
#pragma unroll
  for (int k = 0; k < kFPer; ++k) {
    const int e = lane + 64 * k;
    if (e < fcnt) Fw[e] = fv[k];
  }
  for (int e = lane + 64 * kFPer; e < fcnt; e += 64) Fw[e] = fsrc[e];
  block_sync_lds();
  TrigTab<LT> t;
  {
    const float* row = trig + min(j, Sw - 1) * 3 * TR;
    sfor<3>([&](auto A) {
      constexpr int q3 = LV_CV(A);
      sfor<TP / 4>([&](auto K) {
        constexpr int k4 = LV_CV(K);
        const lv_f4 cv = *reinterpret_cast<const lv_f4*>(row + q3 * TR + 4 * k4);
        const lv_f4 sv = *reinterpret_cast<const lv_f4*>(row + q3 * TR + TP + 4 * k4);
        sfor<4>([&](auto I) {
          constexpr int f = 4 * k4 + LV_CV(I);
          if constexpr (f <= LT) {
            t.c[q3][f] = cv[LV_CV(I)];
            t.s[q3][f] = sv[LV_CV(I)];
          }
        });
      });
    });
  }
  OutT* gout = reinterpret_cast<OutT*>(a.out) + s0 * MC;
  const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
  char* stage_b = reinterpret_cast<char*>(lds) + mis;
  OutT* st_lane = reinterpret_cast<OutT*>(stage_b) + j * MC + c;
  const float* Fl = Fw + c - rows_lo * C;
  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if (l >= lo && l < hi) {
      constexpr int nn = 2 * l + 1;
      constexpr int r0 = l * l;
      float x[nn], y[nn];
      sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[(r0 + LV_CV(K)) * C]; });
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
  __syncthreads();
  tile_flush<OutT, POL>(gout, stage_b, mis, Sv * MC * (int)sizeof(OutT), (int)threadIdx.x, (int)blockDim.x);
}
}  // namespace lv

namespace lv {
// Launch-floor probes: the tile kernel's grid with (0) nothing, (1) the v + spectrum loads
// only, (2) loads + one 16-byte store per lane of the group's output (first 1 KiB).
template <int MODE>
__global__ __launch_bounds__(512) void floor_kernel(ActionArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t s0 = (int64_t)blockIdx.x * 6;
  if constexpr (MODE == 0) {
    if (a.n < 0) reinterpret_cast<float*>(a.out)[threadIdx.x] = 0.f;
  } else {
    const float v = a.v[s0 * 3 + (lane % 18)] + a.F[threadIdx.x];
    if (MODE == 1) {
      if (v == 12345.f) reinterpret_cast<float*>(a.out)[s0 * a.MC + threadIdx.x] = v;
    } else {
      reinterpret_cast<float4*>(reinterpret_cast<float*>(a.out) + s0 * a.MC)[threadIdx.x & 63] =
          make_float4(v, v, v, v);
    }
  }
}
}  // namespace lv

namespace lv {
// Tile kernel v4 = v3 with G sample groups per block (G * nseg waves): fewer, larger
// blocks (the dispatch floor), one spectrum slice per segment shared by the G groups,
// one prologue table for the block's G*Sw samples, one flush of G contiguous tiles.
template <int LT, int CT, bool FUSED, typename OutT, int POL>
__global__ __launch_bounds__(1024) void tile4_kernel(ActionArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int C = CT, Sw = 64 / C;
  constexpr int MC = (LT + 1) * (LT + 1) * C;
  constexpr int TP = t3_tp(LT), TR = t3_row(LT);
  int nseg = 1;
  while (a.seg_lo[nseg] != LT + 1) ++nseg;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int G = (int)(blockDim.x >> 6) / nseg;
  const int g = wave / nseg, k = wave - g * nseg;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[k], hi = a.seg_lo[k + 1];
  const int rows_lo = lo * lo;
  const int64_t sb = (int64_t)blockIdx.x * G * Sw;       // block's first sample
  const int Sb = (int)min((int64_t)G * Sw, a.n - sb);    // block's valid samples (>= 1)
  const int jl = g * Sw + j;                              // lane's sample within the block
  const bool active = jl < Sb;
  const int tile_bytes = ((G * Sw * MC * (int)sizeof(OutT) + 16) + 15) & ~15;
  float* trig = lds + tile_bytes / 4;
  float* Fw = trig + G * Sw * 3 * TR + k * a.fpitch;
  // prologue tasks: (sample jt, slot q), 3*G*Sw of them on the first lanes of the block
  const int tid = threadIdx.x;
  const bool task = tid < 3 * G * Sw;
  const int jt = tid / 3, q = tid - 3 * (tid / 3);
  LaneIn in;
  if (task) lane_load<FUSED>(a, sb + min(jt, Sb - 1), in);
  constexpr int kFPer = 6;
  float fv[kFPer];
  const int fcnt = (hi * hi - rows_lo) * C;
  const float* fsrc = a.F + rows_lo * C;
  const bool fstage = g == 0;
  if (fstage) {
#pragma unroll
    for (int kk = 0; kk < kFPer; ++kk) {
      const int e = lane + 64 * kk;
      fv[kk] = e < fcnt ? fsrc[e] : 0.f;
    }
  }
  if (task) {
    float c1[3], s1[3];
    lane_angles<FUSED>(a, in, sb + min(jt, Sb - 1), jt < Sb, q, FUSED && a.ang_out != nullptr,
                       c1, s1);
    const float cq = q == 0 ? c1[0] : (q == 1 ? c1[1] : c1[2]);
    const float sq = q == 0 ? s1[0] : (q == 1 ? s1[1] : s1[2]);
    float* tc = trig + (jt * 3 + q) * TR;
    float* ts = tc + TP;
    tc[0] = 1.f;
    ts[0] = 0.f;
    float cf = cq, sf = sq;
    sfor<LT + 1>([&](auto F) {
      constexpr int f = LV_CV(F);
      if constexpr (f >= 1) {
        if constexpr (f >= 2) {
          const float cn = fmaf(cf, cq, -(sf * sq));
          sf = fmaf(sf, cq, cf * sq);
          cf = cn;
        }
        tc[f] = cf;
        ts[f] = sf;
      }
    });
  }
  if (fstage) {
#pragma unroll
    for (int kk = 0; kk < kFPer; ++kk) {
      const int e = lane + 64 * kk;
      if (e < fcnt) Fw[e] = fv[kk];
    }
    for (int e = lane + 64 * kFPer; e < fcnt; e += 64) Fw[e] = fsrc[e];
  }
  block_sync_lds();
  TrigTab<LT> t;
  {
    const float* row = trig + min(jl, Sb - 1) * 3 * TR;
    sfor<3>([&](auto A) {
      constexpr int q3 = LV_CV(A);
      sfor<TP / 4>([&](auto K) {
        constexpr int k4 = LV_CV(K);
        const lv_f4 cv = *reinterpret_cast<const lv_f4*>(row + q3 * TR + 4 * k4);
        const lv_f4 sv = *reinterpret_cast<const lv_f4*>(row + q3 * TR + TP + 4 * k4);
        sfor<4>([&](auto I) {
          constexpr int f = 4 * k4 + LV_CV(I);
          if constexpr (f <= LT) {
            t.c[q3][f] = cv[LV_CV(I)];
            t.s[q3][f] = sv[LV_CV(I)];
          }
        });
      });
    });
  }
  OutT* gout = reinterpret_cast<OutT*>(a.out) + sb * MC;
  const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
  char* stage_b = reinterpret_cast<char*>(lds) + mis;
  OutT* st_lane = reinterpret_cast<OutT*>(stage_b) + jl * MC + c;
  const float* Fl = Fw + c - rows_lo * C;
  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if (l >= lo && l < hi) {
      constexpr int nn = 2 * l + 1;
      constexpr int r0 = l * l;
      float x[nn], y[nn];
      sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[(r0 + LV_CV(K)) * C]; });
      xrot<l, 2>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 1>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 0>(t, x, y);
      if (active && j < Sw) {
        OutT* d = st_lane + r0 * C;
        sfor<nn>([&](auto I) {
          d[0] = tile_cvt(y[LV_CV(I)], (OutT*)nullptr);
          d += C;
        });
      }
    }
  });
  __syncthreads();
  tile_flush<OutT, POL>(gout, stage_b, mis, Sb * MC * (int)sizeof(OutT), (int)threadIdx.x, (int)blockDim.x);
}
}  // namespace lv

namespace lv {
// Tile kernel v5 = v3 with
//   TM 1: the multiples read from the LDS table right before each X product (xrot_lds on
//         the t3 row layout) instead of all held in registers (VGPRs -> occupancy);
//   FM 1: no block barrier at the end: each wave writes its own rows [lo^2, hi^2) of the
//         group's samples as soon as its chain is done (8-byte stores).
template <int l, int A, int LT>
__device__ __forceinline__ void xrot_t3(const float* row, const float (&x)[2 * l + 1],
                                        float (&y)[2 * l + 1]) {
  constexpr int TP = t3_tp(LT), TR = t3_row(LT);
  float cc[l + 1], ss[l + 1];
  sfor<(l + 4) / 4>([&](auto K) {
    constexpr int k4 = LV_CV(K);
    const lv_f4 cv = *reinterpret_cast<const lv_f4*>(row + A * TR + 4 * k4);
    const lv_f4 sv = *reinterpret_cast<const lv_f4*>(row + A * TR + TP + 4 * k4);
    sfor<4>([&](auto I) {
      constexpr int f = 4 * k4 + LV_CV(I);
      if constexpr (f <= l) {
        cc[f] = cv[LV_CV(I)];
        ss[f] = sv[LV_CV(I)];
      }
    });
  });
  sfor<2 * l + 1>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    if constexpr (f == 0) {
      y[i] = x[i];
    } else if constexpr (f > 0) {
      y[i] = fmaf(cc[f], x[i], ss[f] * x[2 * l - i]);
    } else {
      y[i] = fmaf(cc[-f], x[i], -(ss[-f] * x[2 * l - i]));
    }
  });
}

template <int LT, int CT, bool FUSED, typename OutT, int POL, int TM, int FM>
__global__ __launch_bounds__(512) void tile5_kernel(ActionArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int C = CT, Sw = 64 / C;
  constexpr int MC = (LT + 1) * (LT + 1) * C;
  constexpr int TP = t3_tp(LT), TR = t3_row(LT);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int rows_lo = lo * lo;
  const int64_t s0 = (int64_t)blockIdx.x * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);
  const bool active = j < Sv;
  constexpr int stage_bytes = ((Sw * MC * (int)sizeof(OutT) + 16) + 15) & ~15;
  float* trig = lds + stage_bytes / 4;
  float* Fw = trig + Sw * 3 * TR + wave * a.fpitch;
  const bool task = wave == 0 && lane < 3 * Sw;
  const int jt = lane / 3, q = lane - 3 * (lane / 3);
  LaneIn in;
  if (task) lane_load<FUSED>(a, s0 + min(jt, Sv - 1), in);
  constexpr int kFPer = 6;
  float fv[kFPer];
  const int fcnt = (hi * hi - rows_lo) * C;
  const float* fsrc = a.F + rows_lo * C;
#pragma unroll
  for (int k = 0; k < kFPer; ++k) {
    const int e = lane + 64 * k;
    fv[k] = e < fcnt ? fsrc[e] : 0.f;
  }
  if (task) {
    float c1[3], s1[3];
    lane_angles<FUSED>(a, in, s0 + min(jt, Sv - 1), jt < Sv, q, FUSED && a.ang_out != nullptr,
                       c1, s1);
    const float cq = q == 0 ? c1[0] : (q == 1 ? c1[1] : c1[2]);
    const float sq = q == 0 ? s1[0] : (q == 1 ? s1[1] : s1[2]);
    float* tc = trig + (jt * 3 + q) * TR;
    float* ts = tc + TP;
    tc[0] = 1.f;
    ts[0] = 0.f;
    float cf = cq, sf = sq;
    sfor<LT + 1>([&](auto F) {
      constexpr int f = LV_CV(F);
      if constexpr (f >= 1) {
        if constexpr (f >= 2) {
          const float cn = fmaf(cf, cq, -(sf * sq));
          sf = fmaf(sf, cq, cf * sq);
          cf = cn;
        }
        tc[f] = cf;
        ts[f] = sf;
      }
    });
  }
#pragma unroll
  for (int k = 0; k < kFPer; ++k) {
    const int e = lane + 64 * k;
    if (e < fcnt) Fw[e] = fv[k];
  }
  for (int e = lane + 64 * kFPer; e < fcnt; e += 64) Fw[e] = fsrc[e];
  block_sync_lds();
  const float* row = trig + min(j, Sw - 1) * 3 * TR;
  TrigTab<TM == 0 ? LT : 0> t;
  if constexpr (TM == 0) {
    sfor<3>([&](auto A) {
      constexpr int q3 = LV_CV(A);
      sfor<TP / 4>([&](auto K) {
        constexpr int k4 = LV_CV(K);
        const lv_f4 cv = *reinterpret_cast<const lv_f4*>(row + q3 * TR + 4 * k4);
        const lv_f4 sv = *reinterpret_cast<const lv_f4*>(row + q3 * TR + TP + 4 * k4);
        sfor<4>([&](auto I) {
          constexpr int f = 4 * k4 + LV_CV(I);
          if constexpr (f <= LT) {
            t.c[q3][f] = cv[LV_CV(I)];
            t.s[q3][f] = sv[LV_CV(I)];
          }
        });
      });
    });
  }
  OutT* gout = reinterpret_cast<OutT*>(a.out) + s0 * MC;
  const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
  char* stage_b = reinterpret_cast<char*>(lds) + mis;
  OutT* st_lane = reinterpret_cast<OutT*>(stage_b) + j * MC + c;
  const float* Fl = Fw + c - rows_lo * C;
  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if (l >= lo && l < hi) {
      constexpr int nn = 2 * l + 1;
      constexpr int r0 = l * l;
      float x[nn], y[nn];
      sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[(r0 + LV_CV(K)) * C]; });
      if constexpr (TM == 0) {
        xrot<l, 2>(t, x, y);
        jmul<l>(y, x);
        xrot<l, 1>(t, x, y);
        jmul<l>(y, x);
        xrot<l, 0>(t, x, y);
      } else {
        xrot_t3<l, 2, LT>(row, x, y);
        jmul<l>(y, x);
        xrot_t3<l, 1, LT>(row, x, y);
        jmul<l>(y, x);
        xrot_t3<l, 0, LT>(row, x, y);
      }
      if (active) {
        OutT* d = st_lane + r0 * C;
        sfor<nn>([&](auto I) {
          d[0] = tile_cvt(y[LV_CV(I)], (OutT*)nullptr);
          d += C;
        });
      }
    }
  });
  if constexpr (FM == 0) {
    __syncthreads();
    tile_flush<OutT, POL>(gout, stage_b, mis, Sv * MC * (int)sizeof(OutT), (int)threadIdx.x, (int)blockDim.x);
  } else {
    static_assert(sizeof(OutT) == 4, "FM 1: fp32 only");
    wave_lds_sync();
    const int np = (hi * hi - rows_lo) * C / 2;  // pairs per sample
    const float inv = 1.f / (float)np;
    const int tot = Sv * np;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(gout, 0, Sv * MC * 4, kRawBufferFlags);
    for (int e = lane; e < tot; e += 64) {
      const int jj = (int)(((float)e + 0.5f) * inv), w = e - jj * np;
      const int b = (jj * MC + rows_lo * C + 2 * w) * 4;
      const float2 v = *reinterpret_cast<const float2*>(stage_b + b);
      st_b64<POL>(rs, b, v.x, v.y);
    }
  }
}
}  // namespace lv

namespace lv {
// Two-phase tile kernel (experiment): the block first computes degrees [0, L1) (phase A,
// split over its waves by seg_lo[0..nseg]), writes the rows [0, L1^2) of its samples
// (Sv runs, 8-byte stores) and, while those stores drain, computes degrees [L1, L]
// (phase B, seg_lo[nseg+1 .. 2 nseg+1]), then writes rows [L1^2, M).  Otherwise the
// library tile kernel (prologue once per (sample, slot), whole spectrum in LDS).
template <typename OutT, int POL>
__device__ __forceinline__ void flush_rows(OutT* gout, const char* stage_b, int Sv, int MC,
                                           int e0, int e1, int tid, int nthr) {
  // elements [e0, e1) of each of the Sv samples (C even: pairs, 8-B aligned for fp32)
  const int np = (e1 - e0) >> 1;
  const float inv = 1.f / (float)np;
  const int tot = Sv * np;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(gout, 0, Sv * MC * (int)sizeof(OutT), kRawBufferFlags);
  for (int p = tid; p < tot; p += nthr) {
    const int jj = (int)(((float)p + 0.5f) * inv), w = p - jj * np;
    const int b = (jj * MC + e0 + 2 * w) * (int)sizeof(OutT);
    const float2 v = *reinterpret_cast<const float2*>(stage_b + b);
    st_b64<POL>(rs, b, v.x, v.y);
  }
}

template <int LT, int POL>
__global__ __launch_bounds__(512) void tile6_kernel(ActionArgs a) {
  using OutT = float;
  constexpr int CT = 10;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int kRow = TrigLds<LT>::kRow;
  constexpr int C = CT, Sw = 64 / CT;
  constexpr int MC = (LT + 1) * (LT + 1) * CT;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nseg = (int)(blockDim.x >> 6);
  const int j = lane / C;
  const int c = lane - j * C;
  const int loA = a.seg_lo[wave], hiA = a.seg_lo[wave + 1];
  const int loB = a.seg_lo[nseg + 1 + wave], hiB = a.seg_lo[nseg + 2 + wave];
  const int L1 = a.seg_lo[nseg];
  const int64_t s0 = (int64_t)blockIdx.x * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);
  const bool active = j < Sv;
  const int stage_bytes = tile_stage_bytes(Sw, MC, 4);
  float* trig = lds + (stage_bytes >> 2);
  float* Fs = trig + Sw * kRow;  // whole F row-major
  const int tid = (int)threadIdx.x;
  const bool task = tid < 3 * Sw;
  const int jt = tid / 3, q = tid - 3 * (tid / 3);
  const int64_t st = s0 + min(jt, Sv - 1);
  LaneIn in;
  if (task) lane_load<true>(a, st, in);
  // stage both of this wave's spectrum slices
  for (int e = loA * loA * C + lane; e < hiA * hiA * C; e += 64) Fs[e] = a.F[e];
  for (int e = loB * loB * C + lane; e < hiB * hiB * C; e += 64) Fs[e] = a.F[e];
  if (task) {
    float c1[3], s1[3];
    lane_angles<true>(a, in, st, jt < Sv, q, a.ang_out != nullptr, c1, s1);
    trig_row_fill<LT>(trig + jt * kRow, c1, s1, q, LT);
  }
  block_sync_lds();
  float* gout = reinterpret_cast<float*>(a.out) + s0 * MC;
  const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
  char* stage_b = reinterpret_cast<char*>(lds) + mis;
  float* st_lane = reinterpret_cast<float*>(stage_b) + j * MC + c;
  const float* tj = trig + min(j, Sw - 1) * kRow;
  const float* Fl = Fs + c;
  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if (l == L1) {  // phase A done: publish and write its rows, then phase B
      block_sync_lds();
      flush_rows<float, POL>(gout, stage_b, Sv, MC, 0, L1 * L1 * C, tid, (int)blockDim.x);
    }
    if ((l >= loA && l < hiA) || (l >= loB && l < hiB)) {
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
        float* d = st_lane + r0 * C;
        sfor<nn>([&](auto I) {
          d[0] = y[LV_CV(I)];
          d += C;
        });
      }
    }
  });
  block_sync_lds();
  flush_rows<float, POL>(gout, stage_b, Sv, MC, L1 * L1 * C, MC, tid, (int)blockDim.x);
}
// Occupancy / prologue variants of the library tile kernel (same body, fwd_tile_body):
//   nomu: compiled without the mean-rotation (fp64) prologue path (a.mu == null)
//   w8  : register budget for 8 waves per SIMD (64 VGPRs), so 5 blocks of 6 waves fit a CU
template <int LT, int CT, bool MAYMU>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8)))
void tile_w8_kernel(ActionArgs a) {
  fwd_tile_body<LT, CT, true, float, MAYMU>(a, blockIdx.x);
}
template <int LT, int CT>
__global__ __launch_bounds__(512) void tile_nomu_kernel(ActionArgs a) {
  fwd_tile_body<LT, CT, true, float, false>(a, blockIdx.x);
}

}  // namespace lv

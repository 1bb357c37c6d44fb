#pragma once
// Forward group-action kernels for gfx950 (MI355X) + their launchers.
// Instantiated once per l_max in action_inst.hip (-DLV_INST_L=k) so the 21 degree
// variants compile in parallel; host planning lives in action.hip.
//
//   lv_group_action_fwd      block_wigner_matrix_multiply, lie_tools.py:226-253
//   lv_fused_exp_action_fwd  mu@rodrigues(v) -> ZYZ -> block D·F in one pass
//                            (reparameterize.py:269-273, vae.py:182, decoders.py:47-56)
//   lv_wigner_d_fwd          packed D_l blocks (parity / debug only)
//
// Two forward kernels:
//   * action_fwd_tile_kernel (shared spectrum, LDS tile fits): one block per sample
//     group, one wave per degree segment, the group's whole output staged in LDS and
//     written as one contiguous run of 16-byte stores;
//   * action_fwd_kernel (per-sample spectrum, or a tile too large for LDS): blocks of
//     4 waves on one degree segment (gridDim.y), row-pair stores straight from registers.
#include "action_common.h"

namespace lv {

// Output staging.  Degrees are written back in chunks: {0..3} (16 rows), {4, 5} (20 rows),
// then one degree per chunk.  A chunk of a wave's Sw samples sits in LDS as [j][row][c]
// with a per-sample stride SP = C (mod 32) -- lanes (j, c) then hit 64 distinct banks --
// and is written back as Sw contiguous runs of rows*C values with 8-byte stores.
__host__ __device__ constexpr int chunk_first(int l) { return l <= 3 ? 0 : (l <= 5 ? 4 : l); }
__host__ __device__ constexpr int chunk_rows_max(int L) {
  return (L >= 6 ? 2 * L + 1 : 0) > 20 ? 2 * L + 1 : 20;
}
__host__ __device__ inline int stage_stride(int L, int C) {
  return ((chunk_rows_max(L) * C + 31) & ~31) + C;
}
__host__ __device__ inline int stage_floats(int L, int C) { return (64 / C) * stage_stride(L, C); }

// Write a staged chunk back: Sv runs of rows*C values, run j from stage + j*SP to
// out[(s0+j)*MC + row0*C ...].  Latency-tolerant form: every lane first issues all its
// LDS reads (K = at most chunk_rows_max/2 float2 per lane, since Sw*C <= 64), waits
// once, then issues its stores -- 512 contiguous bytes per wave instruction.
template <int K, typename OutT>
__device__ __forceinline__ void flush_chunk(const float* stage, int SP, OutT* out, int64_t s0,
                                            int64_t MC, int row0, int rows, int C, int Sv,
                                            int lane) {
  const int plen = rows * C;
  if ((C & 1) == 0) {
    const int npair = plen >> 1;
    const int total = Sv * npair;
    // (j, w) of element e = lane + 64k, tracked incrementally
    int j = 0, w = lane;
    while (w >= npair) { w -= npair; ++j; }
    float2 v[K];
    int jj[K], ww[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      jj[k] = j;
      ww[k] = w;
      if (lane + 64 * k < total)
        v[k] = *reinterpret_cast<const float2*>(stage + j * SP + 2 * w);
      w += 64;
      while (w >= npair) { w -= npair; ++j; }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (lane + 64 * k < total) {
        OutT* dst = out + (s0 + jj[k]) * MC + (int64_t)row0 * C + 2 * ww[k];
        if constexpr (sizeof(OutT) == 4) {
          *reinterpret_cast<float2*>(dst) = v[k];
        } else {
          __hip_bfloat162 h;
          h.x = __float2bfloat16(v[k].x);
          h.y = __float2bfloat16(v[k].y);
          *reinterpret_cast<__hip_bfloat162*>(dst) = h;
        }
      }
    }
  } else {
    for (int j = 0; j < Sv; ++j) {
      const float* src = stage + j * SP;
      OutT* dst = out + (s0 + j) * MC + (int64_t)row0 * C;
      for (int w = lane; w < plen; w += 64) store_out(dst + w, src[w]);
    }
  }
}

// Forward.  Per degree each lane runs the factored chain on its column and parks its
// (2l+1) outputs in the wave's LDS stage; at the end of a chunk the stage is written back
// as contiguous runs.  There is no global load after the first store (vmcnt retires in
// order, so a later load would wait for every older store): a shared spectrum is staged
// into LDS up front and a per-sample spectrum is prefetched one degree ahead.
#ifndef LV_STAGED_DEFAULT
#define LV_STAGED_DEFAULT false
#endif
template <int LT, bool FUSED, bool SHARED, typename OutT, bool STAGED = LV_STAGED_DEFAULT>
__global__ __launch_bounds__(kThreads) void action_fwd_kernel(ActionArgs a) {
  extern __shared__ float lds[];
  LV_STAMP(0);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int C = a.C, Sw = a.Sw;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[blockIdx.y], hi = a.seg_lo[blockIdx.y + 1];
  const int rows_lo = lo * lo;
  const int frows = SHARED ? fseg_rows(lo, hi) : 0;
  const int64_t s0 = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * Sw;
  const int Sv = (int)max((int64_t)0, min((int64_t)Sw, a.n - s0));
  const bool active = j < Sv;
  const int64_t s = active ? s0 + j : (Sv > 0 ? s0 : 0);  // idle lanes mirror a valid sample
  LaneIn in;
  if (Sv > 0) lane_load<FUSED>(a, s, in);
  // Shared spectrum slice: loads issued now, LDS writes and the barrier after the
  // prologue maths so that both memory latencies overlap the per-lane arithmetic.
  constexpr int kFPer = 8;  // staged values per thread (bounded; a loop covers larger slices)
  float fv[kFPer];
  const int fcnt = SHARED ? (hi * hi - rows_lo) * C : 0;
  const float* fsrc = a.F + rows_lo * C;
  if constexpr (SHARED) {
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {
      const int e = threadIdx.x + k * kThreads;
      fv[k] = e < fcnt ? fsrc[e] : 0.f;
    }
  }
  // l >= kTrigLdsMinL: the per-sample (cos, sin) multiples live in a wave-private LDS table
  // (one row per sample, written by the sample's first three lanes) instead of 6(l+1)
  // VGPRs per lane -- 202 -> ~120 VGPRs at l = 20, i.e. 4 instead of 2 waves per SIMD.
  constexpr bool TL = LT >= kTrigLdsMinL && !STAGED;
  constexpr int kRow = TrigLds<LT>::kRow;
  float* trow = lds + a.fpitch + wave * Sw * kRow;
  float c1[3], s1[3];
  TrigTab<TL ? 0 : LT> t;
  if (Sv > 0) {
    lane_angles<FUSED>(a, in, s, active, c, FUSED && a.ang_out && blockIdx.y == 0, c1, s1);
    if constexpr (TL) {
      if (j < Sw)
        for (int q = c; q < 3; q += C) trig_row_fill<LT>(trow + j * kRow, c1, s1, q, hi - 1);
      if constexpr (!SHARED) wave_lds_sync();
    } else {
      trig_fill<LT>(t, c1, s1, hi - 1);
    }
  }
  const float* tj = trow + min(j, Sw - 1) * kRow;
  LV_STAMP(1);
  if constexpr (SHARED) {
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {
      const int e = threadIdx.x + k * kThreads;
      if (e < fcnt) {
        const int r = e / C, cc = e - r * C;
        lds[cc * frows + r] = fv[k];
      }
    }
    for (int e = threadIdx.x + kFPer * kThreads; e < fcnt; e += kThreads) {
      const int r = e / C, cc = e - r * C;
      lds[cc * frows + r] = fsrc[e];
    }
    __syncthreads();
  }
  LV_STAMP(2);
  if (Sv == 0) return;  // whole wave idle (no block barriers below)

  const int SP = stage_stride(LT, C);
  float* stage = lds + (SHARED ? ((frows * C + 3) & ~3) : 0) + (STAGED ? wave * stage_floats(LT, C) : 0);
  float* stage_lane = stage + j * SP + c;
  OutT* out = reinterpret_cast<OutT*>(a.out);
  const float* Fl = lds + c * frows - rows_lo;                  // shared: LDS column
  const float* Fs = a.F + s * a.Fstride + c;                    // per-sample: global
  float fpre[SHARED ? 1 : 2 * LT + 1];

  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if (l >= lo && l < hi) {
      constexpr int nn = 2 * l + 1;
      constexpr int r0 = l * l;
      float x[nn], y[nn];
      if constexpr (SHARED) {
        sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[r0 + LV_CV(K)]; });
      } else {
        if (l == lo) {
          sfor<nn>([&](auto K) { x[LV_CV(K)] = Fs[(r0 + LV_CV(K)) * C]; });
        } else {
          sfor<nn>([&](auto K) { x[LV_CV(K)] = fpre[LV_CV(K)]; });
        }
        if constexpr (l < LT) {
          if (l + 1 < hi) {
            constexpr int r1 = (l + 1) * (l + 1);
            sfor<nn + 2>([&](auto K) { fpre[LV_CV(K)] = Fs[(r1 + LV_CV(K)) * C]; });
          }
        }
      }
#if LV_STORE_MODE == 3  // diagnostic: no chain, spectrum stored as is
#pragma unroll
      for (int i = 0; i < nn; ++i) y[i] = x[i] * c1[0];
#else
      if constexpr (TL) {
        xrot_lds<l, 2, LT>(tj, x, y);
        jmul<l>(y, x);
        xrot_lds<l, 1, LT>(tj, x, y);
        jmul<l>(y, x);
        xrot_lds<l, 0, LT>(tj, x, y);
      } else {
        xrot<l, 2>(t, x, y);
        jmul<l>(y, x);
        xrot<l, 1>(t, x, y);
        jmul<l>(y, x);
        xrot<l, 0>(t, x, y);
      }
#endif
#if LV_STORE_MODE == 1  // diagnostic: no stores, outputs kept live
#pragma unroll
      for (int i = 0; i < nn; ++i) asm volatile("" ::"v"(y[i]));
#else
      if constexpr (STAGED) {
        // chunk this degree belongs to, clipped to the segment
        constexpr int cf = chunk_first(l);
        const int first = cf > lo ? cf : lo;
        const int crow0 = first * first;
        if (active) {
          float* d = stage_lane + (r0 - crow0) * C;
          sfor<nn>([&](auto I) {
            d[0] = y[LV_CV(I)];
            d += C;
          });
        }
        constexpr bool chunk_end = (l == LT) || (chunk_first(l + 1) == l + 1);
        if (chunk_end || l + 1 == hi) {
          wave_lds_sync();
          flush_chunk<(chunk_rows_max(LT) + 1) / 2, OutT>(stage, SP, out, s0, a.MC, crow0,
                                                           r0 + nn - crow0, C, Sv, lane);
          wave_lds_sync();
        }
      } else if ((C & 1) == 0) {
        // Row pairs: adjacent lanes (c even, c+1) swap one value (DPP quad_perm, no LDS)
        // so that even lanes store (row i, cols c..c+1) and odd lanes (row i+1, cols
        // c-1..c): one 8-byte store per lane writes two whole rows of every sample
        // (80-B runs at C = 10).  A pair never straddles samples since C is even.
        const bool odd = (c & 1) != 0;
        OutT* d = out + s * a.MC + r0 * C + (odd ? C + c - 1 : c);
        sfor<nn / 2>([&](auto P) {
          constexpr int i = 2 * LV_CV(P);
          const float send = odd ? y[i] : y[i + 1];
          const float recv = dpp_swap_adjacent(send);
          const float v0 = odd ? recv : y[i];
          const float v1 = odd ? y[i + 1] : recv;
#ifdef LV_RP_SC1  // diagnostic: write-through row-pair stores
          if (active) {
            if constexpr (sizeof(OutT) == 4)
              __hip_atomic_store(reinterpret_cast<unsigned long long*>(d),
                                 __builtin_bit_cast(unsigned long long, make_float2(v0, v1)),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
              store_out2(d, v0, v1);
          }
#else
          if (active) store_out2(d, v0, v1);
#endif
          d += 2 * C;
        });
        if (active) store_out(out + s * a.MC + (r0 + nn - 1) * C + c, y[nn - 1]);
      } else if (active) {
        // one store per output row: Sw contiguous C-value pieces per instruction; a
        // sample's rows are adjacent, so L2 merges them into whole lines
        OutT* d = out + s * a.MC + r0 * C + c;
        sfor<nn>([&](auto I) {
          store_out(d, y[LV_CV(I)]);
          d += C;
        });
      }
#endif
    }
  });
  LV_STAMP(3);
}

// ------------------------------------------------------------- tile forward
// One block = one sample group (Sw = 64 / C samples, one wave's lanes) x nseg degree
// segments, one wave per segment.  Every wave parks its outputs in the block's LDS tile
// [j][row][c] -- which is exactly the global layout of the group's Sw consecutive
// samples -- so after one block barrier the tile leaves as ONE contiguous run of
// Sw * M * C values: full 16-byte stores, 1 KiB per wave instruction, whole 128-B lines.
// POL selects the store cache policy (buffer-store aux bits on gfx950): 0 plain,
// 1 nt, 16 sc1 (write-through: the bytes leave the XCD's L2 during the kernel instead
// of as dirty lines written back at the kernel boundary), 17 sc0 sc1.
typedef float lv_f4 __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void tile_store16(__amdgpu_buffer_rsrc_t r, int off, lv_f4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, POL);
}
template <int POL>
__device__ __forceinline__ void tile_store_elem(__amdgpu_buffer_rsrc_t r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, off, 0, POL);
}
template <int POL>
__device__ __forceinline__ void tile_store_elem(__amdgpu_buffer_rsrc_t r, int off,
                                                __hip_bfloat16 v) {
  __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(short, v), r, off, 0, POL);
}
__device__ __forceinline__ float tile_cvt(float v, float*) { return v; }
__device__ __forceinline__ __hip_bfloat16 tile_cvt(float v, __hip_bfloat16*) {
  return __float2bfloat16(v);
}

// Buffer descriptor word 3 for raw (untyped) buffer access on gfx9-family parts.
constexpr int kRawBufferFlags = 0x00020000;

// LDS bytes of the tile kernel: the output tile (+16 for the alignment shift) then the
// wave-private spectrum slices.
__host__ __device__ inline int tile_stage_bytes(int Sw, int64_t MC, int out_bytes) {
  return (int)((((int64_t)Sw * MC * out_bytes + 16) + 15) & ~(int64_t)15);
}

// Write a staged tile back: head elements up to the first 16-B boundary, the 16-B
// body (ds_read_b128 -> buffer_store_dwordx4, 1 KiB per wave instruction), tail elements.
// The LDS tile starts `mis` bytes past a 16-B boundary, mis = gout mod 16, so LDS and
// global addresses agree mod 16.
// Threads tid = 0..nthr-1 of the block take part.
template <typename OutT, int POL>
__device__ __forceinline__ void tile_flush(OutT* gout, const char* stage_b, int mis, int nbytes,
                                           int tid, int nthr) {
  const int head = min((16 - mis) & 15, nbytes);
  const int nvec = (nbytes - head) >> 4;
  const int tail0 = head + nvec * 16;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(gout, 0, nbytes, kRawBufferFlags);
  for (int k = tid; k < nvec; k += nthr) {
    const lv_f4 v = *reinterpret_cast<const lv_f4*>(stage_b + head + 16 * k);
    tile_store16<POL>(rs, head + 16 * k, v);
  }
  constexpr int E = (int)sizeof(OutT);
  const int nedge = head / E + (nbytes - tail0) / E;
  if (tid < nedge) {
    const int b = tid < head / E ? tid * E : tail0 + (tid - head / E) * E;
    tile_store_elem<POL>(rs, b, *reinterpret_cast<const OutT*>(stage_b + b));
  }
}
template <typename OutT, int POL>
__device__ __forceinline__ void tile_flush(OutT* gout, const char* stage_b, int mis, int nbytes) {
  tile_flush<OutT, POL>(gout, stage_b, mis, nbytes, (int)threadIdx.x, (int)blockDim.x);
}

// Block barrier for LDS hand-offs only: waits for this wave's LDS operations, never for
// its global stores (a __syncthreads() release fence may emit s_waitcnt vmcnt(0) and
// stall on the previous tile's stores still in flight).
__device__ __forceinline__ void block_sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The store policy picked at run time (uniform branch; aux bits must be immediates).
template <typename OutT>
__device__ __forceinline__ void tile_flush_rt(OutT* gout, const char* stage_b, int mis, int nbytes,
                                              int write_through, int tid, int nthr) {
  if (write_through)
    tile_flush<OutT, 16>(gout, stage_b, mis, nbytes, tid, nthr);
  else
    tile_flush<OutT, 1>(gout, stage_b, mis, nbytes, tid, nthr);
}
template <typename OutT>
__device__ __forceinline__ void tile_flush_rt(OutT* gout, const char* stage_b, int mis, int nbytes,
                                              int write_through) {
  tile_flush_rt<OutT>(gout, stage_b, mis, nbytes, write_through, (int)threadIdx.x,
                      (int)blockDim.x);
}

template <int LT, bool FUSED, typename OutT, int POL, bool WAVEFLUSH = false>
__global__ __launch_bounds__(512) void action_fwd_tile_kernel(ActionArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  LV_STAMP(0);
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
  const int64_t s = active ? s0 + j : s0;  // idle lanes mirror a valid sample
  LaneIn in;
  lane_load<FUSED>(a, s, in);
  // this wave's spectrum slice: loads now, LDS writes after the prologue maths
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
  LV_STAMP(1);
  const int stage_bytes = tile_stage_bytes(Sw, MC, (int)sizeof(OutT));
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
  LV_STAMP(2);

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
#if LV_TILE_DIAG == 2  // diagnostic: no chain
      sfor<nn>([&](auto K) { y[LV_CV(K)] = x[LV_CV(K)] * t.c[0][1]; });
#else
      xrot<l, 2>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 1>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 0>(t, x, y);
#endif
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
  if constexpr (WAVEFLUSH) {
    // each wave writes its own rows [lo^2, hi^2) of every sample: Sv runs, 8-B pieces
    wave_lds_sync();
    LV_STAMP(3);
    constexpr int E = (int)sizeof(OutT);
    const int run = (hi * hi - rows_lo) * C * E;  // bytes per sample
    const int nbytes = Sv * (int)MC * E;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(gout, 0, nbytes, kRawBufferFlags);
    for (int jj = 0; jj < Sv; ++jj) {
      const int b0 = (jj * (int)MC + rows_lo * C) * E;
      if (((mis + b0) & 7) == 0 && (run & 7) == 0) {
        for (int p = lane * 8; p < run; p += 512) {
          const float2 v2 = *reinterpret_cast<const float2*>(stage_b + b0 + p);
          typedef unsigned int lv_u2 __attribute__((ext_vector_type(2)));
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(lv_u2, v2), rs, b0 + p, 0, POL);
        }
      } else {
        for (int p = lane * E; p < run; p += 64 * E)
          tile_store_elem<POL>(rs, b0 + p, *reinterpret_cast<const OutT*>(stage_b + b0 + p));
      }
    }
  } else {
    __syncthreads();
    LV_STAMP(3);
#if LV_TILE_DIAG != 1  // 1: diagnostic, no flush
    if constexpr (POL < 0)
      tile_flush_rt<OutT>(gout, stage_b, mis, Sv * (int)MC * (int)sizeof(OutT), a.write_through);
    else
      tile_flush<OutT, POL>(gout, stage_b, mis, Sv * (int)MC * (int)sizeof(OutT));
#endif
  }
  LV_STAMP(4);
}

// ------------------------------------------------------- paired tile forward (C = 10)
// The tile kernel with each lane owning TWO adjacent columns (c, c+1) of one sample:
// every chain operand is a column pair, so the X rotations and the J products run as
// packed fp32 (v_pk_fma_f32 / v_pk_mul_f32, two columns per VALU slot; the cos/sin
// multiples and J's literal coefficients are broadcast via op_sel).  A wave then holds
// Sw = 12 samples x 5 column pairs, so the per-sample prologue is also amortised over
// twice the samples.  Same rounding sequence per element as the scalar chain.
// C is a compile-time 10 (ActionNet's default rep_copies, the BASELINE configs): spectrum
// reads and LDS tile writes use immediate offsets.
typedef float lv_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ lv_f2 splat2(float v) { return (lv_f2){v, v}; }

template <int l, int A, int LT>
__device__ __forceinline__ void xrot2(const TrigTab<LT>& t, const lv_f2 (&x)[2 * l + 1],
                                      lv_f2 (&y)[2 * l + 1]) {
  sfor<2 * l + 1>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    if constexpr (f == 0) {
      y[i] = x[i];
    } else if constexpr (f > 0) {
      y[i] = __builtin_elementwise_fma(splat2(t.c[A][f]), x[i], splat2(t.s[A][f]) * x[2 * l - i]);
    } else {
      y[i] = __builtin_elementwise_fma(splat2(t.c[A][-f]), x[i],
                                       -(splat2(t.s[A][-f]) * x[2 * l - i]));
    }
  });
}

// xrot2 with the multiples read from a per-sample LDS row (TrigLds layout).
template <int l, int A, int LT>
__device__ __forceinline__ void xrot2_lds(const float* tj, const lv_f2 (&x)[2 * l + 1],
                                          lv_f2 (&y)[2 * l + 1]) {
  constexpr int TP = TrigLds<LT>::TP;
  sfor<2 * l + 1>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    if constexpr (f == 0) {
      y[i] = x[i];
    } else if constexpr (f > 0) {
      y[i] = __builtin_elementwise_fma(splat2(tj[2 * A * TP + f]), x[i],
                                       splat2(tj[(2 * A + 1) * TP + f]) * x[2 * l - i]);
    } else {
      y[i] = __builtin_elementwise_fma(splat2(tj[2 * A * TP - f]), x[i],
                                       -(splat2(tj[(2 * A + 1) * TP - f]) * x[2 * l - i]));
    }
  });
}

template <int l>
__device__ __forceinline__ void jmul2(const lv_f2 (&x)[2 * l + 1], lv_f2 (&y)[2 * l + 1]) {
  constexpr int n = 2 * l + 1;
  constexpr const float* J = lv_j::jtab<l>();
  sfor<n>([&](auto P) {
    constexpr int p = LV_CV(P);
    lv_f2 acc = splat2(0.f);
    sfor<n>([&](auto K) {
      constexpr int k = LV_CV(K);
      constexpr float v = J[p * n + k];
      if constexpr (v != 0.f) acc = __builtin_elementwise_fma(splat2(v), x[k], acc);
    });
    y[p] = acc;
  });
}

constexpr int kPairC = 10;
constexpr int kPairSw = 64 / (kPairC / 2);  // 12 samples per wave
constexpr int kPairMaxL = 12;

template <int LT, bool FUSED, typename OutT>
__global__ __launch_bounds__(512) void action_fwd_tile_pair_kernel(ActionArgs a) {
  constexpr int C = kPairC, CP = C / 2, Sw = kPairSw;
  constexpr int64_t MC = (int64_t)(LT + 1) * (LT + 1) * C;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane / CP;  // 12 for the 4 spare lanes
  const int cp = lane - j * CP;
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int rows_lo = lo * lo;
  const int frows = fseg_rows(lo, hi);
  const int64_t s0 = (int64_t)blockIdx.x * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);  // >= 1: grid = ceil(n / Sw)
  const bool active = j < Sv;
  const int64_t s = active ? s0 + j : s0;  // idle lanes mirror a valid sample
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
  // (cos, sin) multiples: one LDS row per sample, shared by the block's waves.  Every
  // wave fills all rows (lanes cp < 3 one angle each) with identical values, so each wave
  // only needs its own writes to have landed -- no block barrier (the chain would wait
  // for the slowest prologue) and no register table (it would cost 6(l+1) VGPRs).
  constexpr int kRow = TrigLds<LT>::kRow;
  const int stage_bytes = tile_stage_bytes(Sw, MC, (int)sizeof(OutT));
  float* trow = lds + (stage_bytes >> 2) + (int)(blockDim.x >> 6) * a.fpitch;
  {
    float c1[3], s1[3];
    lane_angles<FUSED>(a, in, s, active, cp, FUSED && a.ang_out && wave == 0, c1, s1);
    if (j < Sw)
      for (int q = cp; q < 3; q += CP) trig_row_fill<LT>(trow + j * kRow, c1, s1, q, LT);
  }
  const float* tj = trow + min(j, Sw - 1) * kRow;
  // wave-private spectrum slice as [column pair][row][2]
  float* Fw = lds + (stage_bytes >> 2) + wave * a.fpitch;
#pragma unroll
  for (int k = 0; k < kFPer; ++k) {
    const int e = lane + 64 * k;
    if (e < fcnt) {
      const int r = e / C, cc = e - r * C;
      Fw[((cc >> 1) * frows + r) * 2 + (cc & 1)] = fv[k];
    }
  }
  for (int e = lane + 64 * kFPer; e < fcnt; e += 64) {
    const int r = e / C, cc = e - r * C;
    Fw[((cc >> 1) * frows + r) * 2 + (cc & 1)] = fsrc[e];
  }
  wave_lds_sync();

  OutT* gout = reinterpret_cast<OutT*>(a.out) + s0 * MC;
  const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
  char* stage_b = reinterpret_cast<char*>(lds) + mis;  // LDS addr = global addr (mod 16)
  OutT* st_lane = reinterpret_cast<OutT*>(stage_b) + j * MC + 2 * cp;
  const lv_f2* Fl = reinterpret_cast<const lv_f2*>(Fw + cp * frows * 2) - rows_lo;

  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if (l >= lo && l < hi) {
      constexpr int nn = 2 * l + 1;
      constexpr int r0 = l * l;
      lv_f2 x[nn], y[nn];
      sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[r0 + LV_CV(K)]; });
      xrot2_lds<l, 2, LT>(tj, x, y);
      jmul2<l>(y, x);
      xrot2_lds<l, 1, LT>(tj, x, y);
      jmul2<l>(y, x);
      xrot2_lds<l, 0, LT>(tj, x, y);
      if (active) {
        OutT* d = st_lane + r0 * C;
        sfor<nn>([&](auto I) {
          constexpr int i = LV_CV(I);
          d[i * C] = tile_cvt(y[i].x, (OutT*)nullptr);
          d[i * C + 1] = tile_cvt(y[i].y, (OutT*)nullptr);
        });
      }
    }
  });
  __syncthreads();
  tile_flush_rt<OutT>(gout, stage_b, mis, Sv * (int)MC * (int)sizeof(OutT), a.write_through);
}

// ------------------------------------------------------------ Wigner-D blocks
// Column q of D_l = chain applied to e_q; one thread per (sample, q), one kernel per
// degree.  D is (n, dsz) with block l row-major at offset off.
template <int l>
__global__ void wigner_d_kernel(const float* ang, float* D, int64_t n, int dsz) {
  constexpr int nn = 2 * l + 1;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= n * nn) return;
  const int64_t s = tid / nn;
  const int q = (int)(tid - s * nn);
  float c1[3], s1[3];
  for (int i = 0; i < 3; ++i) sincosf(ang[s * 3 + i], &s1[i], &c1[i]);
  TrigTab<l> t;
  trig_fill<l>(t, c1, s1, l);
  float x[nn], y[nn];
  sfor<nn>([&](auto K) { x[LV_CV(K)] = (LV_CV(K) == q) ? 1.f : 0.f; });
  xrot<l, 2>(t, x, y);
  jmul<l>(y, x);
  xrot<l, 1>(t, x, y);
  jmul<l>(y, x);
  xrot<l, 0>(t, x, y);
  constexpr int off = l * (2 * l - 1) * (2 * l + 1) / 3;  // sum_{k<l} (2k+1)^2
  sfor<nn>([&](auto I) { D[s * dsz + off + LV_CV(I) * nn + q] = y[LV_CV(I)]; });
}

// ------------------------------------------------------------------ host side

struct FwdLaunch {
  ActionArgs a;
  int gx, gy;
  bool fused;
  bool tile;     // tile kernel (shared spectrum; gy = waves per block)
  bool pair;     // ... its paired-column variant (C = 10, l <= kPairMaxL)
  size_t lds;    // tile kernel dynamic LDS bytes
  int dtype;
  hipStream_t stream;
};

template <int LT>
struct FwdLauncher {
  using Args = FwdLaunch;
  static int run(FwdLaunch& p) {
    const bool bf16 = p.dtype == LV_DTYPE_BF16;
    if constexpr (LT <= kPairMaxL) {
      if (p.tile && p.pair) {
        const dim3 grid(p.gx), block(64 * p.gy);
        if (p.fused) {
          if (bf16)
            hipLaunchKernelGGL((action_fwd_tile_pair_kernel<LT, true, __hip_bfloat16>), grid, block, p.lds, p.stream, p.a);
          else
            hipLaunchKernelGGL((action_fwd_tile_pair_kernel<LT, true, float>), grid, block, p.lds, p.stream, p.a);
        } else {
          if (bf16)
            hipLaunchKernelGGL((action_fwd_tile_pair_kernel<LT, false, __hip_bfloat16>), grid, block, p.lds, p.stream, p.a);
          else
            hipLaunchKernelGGL((action_fwd_tile_pair_kernel<LT, false, float>), grid, block, p.lds, p.stream, p.a);
        }
        LV_RETURN_LAUNCH("action_fwd_tile_pair_kernel");
      }
    }
    if (p.tile) {
      const dim3 grid(p.gx), block(64 * p.gy);
      if (p.fused) {
        if (bf16)
          hipLaunchKernelGGL((action_fwd_tile_kernel<LT, true, __hip_bfloat16, -1>), grid, block, p.lds, p.stream, p.a);
        else
          hipLaunchKernelGGL((action_fwd_tile_kernel<LT, true, float, -1>), grid, block, p.lds, p.stream, p.a);
      } else {
        if (bf16)
          hipLaunchKernelGGL((action_fwd_tile_kernel<LT, false, __hip_bfloat16, -1>), grid, block, p.lds, p.stream, p.a);
        else
          hipLaunchKernelGGL((action_fwd_tile_kernel<LT, false, float, -1>), grid, block, p.lds, p.stream, p.a);
      }
      LV_RETURN_LAUNCH("action_fwd_tile_kernel");
    }
    int fmax = 0;
    const bool shared = p.a.Fstride == 0;
    if (shared)
      for (int k = 0; k < p.gy; ++k)
        fmax = max(fmax, (fseg_rows(p.a.seg_lo[k], p.a.seg_lo[k + 1]) * p.a.C + 3) & ~3);
    p.a.fpitch = fmax;  // trig tables follow the spectrum slice (LT >= kTrigLdsMinL)
    const size_t trig = LT >= kTrigLdsMinL && !LV_STAGED_DEFAULT
                            ? (size_t)kWavesPerBlock * p.a.Sw * TrigLds<LT>::kRow : 0;
    const size_t lds = sizeof(float) * ((size_t)fmax + trig + (LV_STAGED_DEFAULT ? (size_t)kWavesPerBlock * stage_floats(LT, p.a.C) : 0));
    const dim3 grid(p.gx, p.gy), block(kThreads);
    if (p.fused) {  // the fused path takes a shared spectrum (ActionNet's item_rep)
      if (bf16)
        hipLaunchKernelGGL((action_fwd_kernel<LT, true, true, __hip_bfloat16>), grid, block, lds, p.stream, p.a);
      else
        hipLaunchKernelGGL((action_fwd_kernel<LT, true, true, float>), grid, block, lds, p.stream, p.a);
    } else if (shared) {
      if (bf16)
        hipLaunchKernelGGL((action_fwd_kernel<LT, false, true, __hip_bfloat16>), grid, block, lds, p.stream, p.a);
      else
        hipLaunchKernelGGL((action_fwd_kernel<LT, false, true, float>), grid, block, lds, p.stream, p.a);
    } else {
      if (bf16) {
        set_error("bf16 output needs a shared spectrum");
        return LV_ERR_ARG;
      }
      hipLaunchKernelGGL((action_fwd_kernel<LT, false, false, float>), grid, block, lds, p.stream, p.a);
    }
    LV_RETURN_LAUNCH("action_fwd_kernel");
  }
};

struct WigLaunch {
  const float* ang;
  float* D;
  int64_t n;
  int dsz;
  hipStream_t stream;
};

template <int l>
struct WigLauncher {
  static int run(WigLaunch& p) {
    const int64_t total = p.n * (2 * l + 1);
    hipLaunchKernelGGL((wigner_d_kernel<l>), dim3(ceil_div(total, 256)), dim3(256), 0, p.stream,
                       p.ang, p.D, p.n, p.dsz);
    LV_RETURN_LAUNCH("wigner_d_kernel");
  }
};

#define LV_EXTERN_LAUNCHERS(L)            \
  extern template struct FwdLauncher<L>;  \
  extern template struct WigLauncher<L>;


}  // namespace lv

#pragma once
#include <type_traits>
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
//     group, one wave per degree segment; the per-sample prologue runs once per
//     (sample, Euler slot) into an LDS table of multiples, the group's whole output is
//     staged in LDS and written as one contiguous run of 16-byte stores;
//   * action_fwd_kernel (per-sample spectrum, or a tile too large for LDS): blocks of
//     4 waves on one degree segment (gridDim.y), row-pair stores straight from registers.
#include "action_common.h"

namespace lv {

// Forward, no LDS tile.  Per degree each lane runs the factored chain on its column and
// stores its (2l+1) outputs straight from registers.  There is no global load after the
// first store (vmcnt retires in order, so a later load would wait for every older store):
// a shared spectrum is staged into LDS up front and a per-sample spectrum is prefetched
// one degree ahead.
template <int LT, bool FUSED, bool SHARED, typename OutT>
__global__ __launch_bounds__(kThreads) void action_fwd_kernel(ActionArgs a) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar branches
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
  constexpr bool TL = LT >= kTrigLdsMinL;
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
  if (Sv == 0) return;  // whole wave idle (no block barriers below)

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
      if ((C & 1) == 0) {
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
          if (active) store_out2(d, v0, v1);
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
    }
  });
}

// ------------------------------------------------------------- tile forward
// Output staging: every wave parks its outputs in the block's LDS tile [j][row][c] --
// exactly the global layout of the group's Sw consecutive samples -- so after one block
// barrier the tile leaves as ONE contiguous run of Sw * M * C values: 16-byte stores,
// 1 KiB per wave instruction, whole 128-B lines.  POL selects the store cache policy
// (buffer-store aux bits on gfx950): 1 nt, 16 sc1 (write-through: the bytes leave the
// XCD's L2 during the kernel instead of as dirty lines written back at the kernel
// boundary; measured best while the output is small, nt beyond).
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

// LDS bytes of the output tile (+16 for the alignment shift).
__host__ __device__ inline int tile_stage_bytes(int Sw, int64_t MC, int out_bytes) {
  return (int)((((int64_t)Sw * MC * out_bytes + 16) + 15) & ~(int64_t)15);
}

// Write a staged tile back: head elements up to the first 16-B boundary, the 16-B
// body (ds_read_b128 -> buffer_store_dwordx4, 1 KiB per wave instruction), tail elements.
// The LDS tile starts `mis` bytes past a 16-B boundary, mis = gout mod 16, so LDS and
// global addresses agree mod 16.
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

// Block barrier for LDS hand-offs only: waits for this wave's LDS operations, never for
// its global stores (a __syncthreads() release fence may emit s_waitcnt vmcnt(0) and
// stall on stores still in flight).
__device__ __forceinline__ void block_sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The store policy picked at run time (uniform branch; aux bits must be immediates).
template <typename OutT>
__device__ __forceinline__ void tile_flush_rt(OutT* gout, const char* stage_b, int mis, int nbytes,
                                              int write_through) {
  if (write_through == 1)
    tile_flush<OutT, 16>(gout, stage_b, mis, nbytes, (int)threadIdx.x, (int)blockDim.x);
  else if (write_through == 2)
    tile_flush<OutT, 0>(gout, stage_b, mis, nbytes, (int)threadIdx.x, (int)blockDim.x);
  else
    tile_flush<OutT, 1>(gout, stage_b, mis, nbytes, (int)threadIdx.x, (int)blockDim.x);
}

// Tile kernel.  One block = one sample group (Sw = 64 / C samples, one wave's lanes) x
// nseg degree segments, one wave per segment.
//   1. Prologue ONCE per (sample j, Euler slot q): the block's first 3*Sw threads each
//      load one sample's v (and mu), run exp -> ZYZ (cos, sin) and the multiples of
//      slot q (trig_row_fill: the same recurrence as trig_fill, bitwise) into the
//      block's LDS table.  Every segment wave used to repeat the whole prologue on all
//      its lanes: 5x the work at batch 4096 and ~40% of the kernel's VALU stream.
//   2. Meanwhile each wave stages its spectrum slice; one barrier publishes both.
//   3. Chain per degree with the multiples read from LDS right before each X product
//      (16-byte reads; low register pressure, 74 VGPRs at l = 10).
//   4. Outputs parked in the LDS tile; barrier; one contiguous flush.
// CT: compile-time C (0 = run-time a.C).  With CT the spectrum slice is staged row-major
// ([row][c], no index division, immediate-offset reads); without it column-major.
// With CT the waves' row-major slices are contiguous: the block holds the whole spectrum
// once (M*C floats, 17.6 KB at l = 20) and each wave stages and reads its own rows.  With
// run-time C from l_max >= kTileFGlobalMinL the spectrum is read from global memory
// instead (no global store precedes the flush, so these loads never wait behind stores);
// that costs ~10 cycles of address processing per wave load instruction, which is why
// the C = 10 path keeps it in LDS (l = 20 bf16: 18.5 -> 5 us of skeleton, tools/c5bench).
// MAYMU = false: compiled without the mean-rotation (mu) prologue (a.mu must be null).
template <int LT, int CT, bool FUSED, typename OutT, bool MAYMU = true>
__device__ __forceinline__ void fwd_tile_body(const ActionArgs& a, int64_t grp) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int kRow = TrigLds<LT>::kRow;
  constexpr bool FG = CT == 0 && LT >= kTileFGlobalMinL;  // spectrum from global, no LDS
  // fp32 tile with compile-time C: the spectrum lives in the tile's LAST sample slot
  // (same [row][c] layout, M*C floats).  A wave reads degree l's spectrum rows into
  // registers before it writes that degree's tile rows, and no other wave touches those
  // rows, so the slot is free to be overwritten; the block saves M*C*4 bytes of LDS
  // (l = 10: 35.7 -> 30.9 KB, 4 -> 5 blocks per CU).
  constexpr bool FT = CT > 0 && std::is_same_v<OutT, float>;
  const int C = CT > 0 ? CT : a.C;
  const int Sw = a.Sw;  // 64 / C, or fewer (plan: LDS per block vs blocks per CU)
  const int64_t MC = CT > 0 ? (int64_t)(LT + 1) * (LT + 1) * CT : a.MC;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar branches
  const int tid = (int)threadIdx.x, nthr = (int)blockDim.x;
  const int j = lane / C;
  const int c = lane - j * C;
  // this wave's degrees: a bit set (compile-time C: any set the planner balanced by cost);
  // run-time C keeps contiguous ranges [lo, hi) for its column-major spectrum slices
  const unsigned dmask = a.seg_mask[wave];
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int rows_lo = lo * lo;
  const int frows = fseg_rows(lo, hi);
  const int64_t s0 = grp * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);  // >= 1: grp < ceil(n / Sw)
  const bool active = j < Sv;
  const int stage_bytes = tile_stage_bytes(Sw, MC, (int)sizeof(OutT));
  float* trig = lds + (stage_bytes >> 2);
  OutT* gout = reinterpret_cast<OutT*>(a.out) + s0 * MC;
  const int mis = (int)(reinterpret_cast<uintptr_t>(gout) & 15);
  char* stage_b = reinterpret_cast<char*>(lds) + mis;  // LDS addr = global addr (mod 16)
  // spectrum in LDS: CT > 0 the whole (M, C) row-major, staged by all threads of the block
  // (FT: in the tile's last sample slot), else per-wave column-major slices of a.fpitch
  float* const Fall = FT ? reinterpret_cast<float*>(stage_b) + (Sw - 1) * MC : trig + Sw * kRow;
  float* Fw = Fall + (CT > 0 ? 0 : wave * a.fpitch);
  // 1. prologue task (sample jt, slot q); the host guarantees 3*Sw <= blockDim.x
  // Wave priority (a.prio, the plan's default 2): the prologue (v / mu loads, exp -> ZYZ,
  // multiples, spectrum staging) issues at s_setprio 3 and the chain at 0, so on a CU that
  // holds blocks in different phases a new block's loads start ahead of the other blocks'
  // FMA streams (tools/gpu_fwd_knobs.sh, profiles/r03_fwd_prio_ab.txt: batch 16,384
  // 20.96 -> 18.27 us, 65,536 63.6 -> 61.1, 262,144 256 -> 252; 4,096, where every block
  // starts at once, unchanged).  1 / 3: A/B variants with the flush raised.
  phase_stamp(a.stamps, wave, 0);
  if (a.prio >= 2) __builtin_amdgcn_s_setprio(3);
  // task_spread: task t on lane t / nw of wave t % nw, so the prologue's serial chains run on
  // every SIMD of the CU instead of all in wave 0
  const int t_task = a.task_spread ? lane * (nthr >> 6) + wave : tid;
  const bool task = t_task < 3 * Sw;
  const int jt = t_task / 3, q = t_task - 3 * (t_task / 3);
  const int64_t st = s0 + min(jt, Sv - 1);  // idle slots mirror a valid sample
  LaneIn in;
  if (task) lane_load<FUSED, MAYMU>(a, st, in);
  // The mu-free fused kernel writes ang_out (the product operator's saved angles) from
  // wave 1, lanes j < Sv, during the prologue -- a wave that only stages spectrum rows
  // there, on another SIMD than the task lanes of wave 0 -- instead of on the q = 0 task
  // lanes, where quat_to_eazyz_fwd's atan2 / acos held wave 0's multiples by ~0.5 us per
  // launch.  Same quaternion (exp_quat), so the same angles bit for bit.  (A one-wave
  // block writes them after its chain.)
  constexpr bool kAngLate = FUSED && !MAYMU;
  const int ang_wave = (nthr >> 6) > 1 ? 1 : 0;
  const bool ang_lane = kAngLate && a.ang_out != nullptr && wave == ang_wave && lane < Sv;
  auto write_ang = [&]() {
    float vang[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) vang[i] = a.v[(s0 + lane) * 3 + i];
    const ExpQuat e = exp_quat(vang);
    float ang[3];
    quat_to_eazyz_fwd(e.qr, ang);
    a.ang_out[(s0 + lane) * 3 + 0] = ang[0];
    a.ang_out[(s0 + lane) * 3 + 1] = ang[1];
    a.ang_out[(s0 + lane) * 3 + 2] = ang[2];
  };
  // a.ang_order 0 (default): wave 1 writes the angles before it issues its spectrum loads,
  // so its two global round trips run back to back and it reaches the prologue barrier last
  // (timeline at 4,096: loads landed 1.08 us after wave start vs 0.52-0.68 on the other
  // waves, barrier at 1.73 with the multiples done at 1.28); 1 (A/B): after them, so the v
  // load and the spectrum loads are in flight together.  A/B at config 2: 7.15 / 7.16 us
  // for 1 against 7.14 / 7.13 for 0 (profiles/r06_ab_ang_order_c2.txt) -- the other waves'
  // chains hide the late wave, so the round-5 order stays
  if (ang_lane && ang_wave == 1 && a.ang_order == 0) write_ang();
  // 2. spectrum staging: every load issued now (before the prologue maths), the LDS writes
  //    after it.  CT > 0: element e = tid + k * nthr of the whole (M, C) spectrum, at most
  //    kFPer per thread for the smallest block the plan makes (2 waves), a batched loop
  //    beyond; else this wave's column-major slice.
  constexpr int kFPer = FG ? 1 : (CT > 0 ? ((LT + 1) * (LT + 1) * (CT > 0 ? CT : 1) + 127) / 128 : 6);
  constexpr int kFPerCap = kFPer < 18 ? kFPer : 18;
  float fv[kFPerCap];
  const int fcnt = FG ? 0 : (CT > 0 ? (int)MC : (hi * hi - rows_lo) * C);
  const int fstr = CT > 0 ? nthr : 64;
  const int fbase = CT > 0 ? tid : lane;
  const float* fsrc = a.F + (CT > 0 ? 0 : rows_lo * C);
#pragma unroll
  for (int k = 0; k < kFPerCap; ++k) {
    const int e = fbase + fstr * k;
    fv[k] = e < fcnt ? fsrc[e] : 0.f;
  }
  if (ang_lane && ang_wave == 1 && a.ang_order != 0) write_ang();
  if (a.stamps) {  // A/B timeline: when this wave's loads (v; spectrum) have landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    phase_stamp(a.stamps, wave, 5);
  }
  if (task) {
    float cq, sq;
    if constexpr (FUSED && !MAYMU) {
      // z = exp(v): this thread's slot only (transpose: slot q takes angle 2 - q, sine negated)
      // ang_out is not written here: wave 1 writes it during the prologue (above; a one-wave
      // block after its chain), since its atan2 / acos kept the multiples waiting on the
      // q = 0 lanes
      float qr[4];
      exp_to_zyz_slot(in.v, a.transpose ? 2 - q : q, cq, sq, qr);
      if (a.transpose) sq = -sq;
    } else {
      float c1[3], s1[3];
      lane_angles<FUSED, MAYMU>(a, in, st, jt < Sv, q, FUSED && a.ang_out != nullptr, c1, s1);
      cq = q == 0 ? c1[0] : (q == 1 ? c1[1] : c1[2]);
      sq = q == 0 ? s1[0] : (q == 1 ? s1[1] : s1[2]);
    }
    if (a.stamps) phase_stamp(a.stamps, wave, 6);
    trig_row_fill1<LT>(trig + jt * kRow, cq, sq, q, LT);
    if (a.stamps) phase_stamp(a.stamps, wave, 7);
  }
  if constexpr (FG) {
  } else if constexpr (CT > 0) {
#pragma unroll
    for (int k = 0; k < kFPerCap; ++k) {
      const int e = fbase + fstr * k;
      if (e < fcnt) Fw[e] = fv[k];
    }
    for (int e0 = fbase + fstr * kFPerCap; e0 < fcnt; e0 += 8 * fstr) {
      float t8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t8[u] = e0 + fstr * u < fcnt ? fsrc[e0 + fstr * u] : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + fstr * u < fcnt) Fw[e0 + fstr * u] = t8[u];
    }
  } else {
#pragma unroll
    for (int k = 0; k < kFPerCap; ++k) {
      const int e = lane + 64 * k;
      if (e < fcnt) {
        const int r = e / C, cc = e - r * C;
        Fw[cc * frows + r] = fv[k];
      }
    }
    for (int e = lane + 64 * kFPerCap; e < fcnt; e += 64) {
      const int r = e / C, cc = e - r * C;
      Fw[cc * frows + r] = fsrc[e];
    }
  }
  block_sync_lds();
  phase_stamp(a.stamps, wave, 1);

  if (a.prio >= 2) __builtin_amdgcn_s_setprio(0);
  OutT* st_lane = reinterpret_cast<OutT*>(stage_b) + j * MC + c;
  const float* tj = trig + min(j, Sw - 1) * kRow;
  // spectrum column: LDS slice, or global (FG)
  const float* Fl = FG ? a.F + c : (CT > 0 ? Fall + c : Fw + c * frows - rows_lo);
  const int fstep = (FG || CT > 0) ? C : 1;  // stride between consecutive rows of a column

  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if ((dmask >> l) & 1u) {
      constexpr int nn = 2 * l + 1;
      constexpr int r0 = l * l;
      float x[nn], y[nn];
      sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[(r0 + LV_CV(K)) * fstep]; });
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
      if (a.stamps) degree_stamp(a.stamps, wave, l);
    }
  });
  if (ang_lane && ang_wave == 0) write_ang();
  phase_stamp(a.stamps, wave, 2);
  block_sync_lds();
  phase_stamp(a.stamps, wave, 3);
  if (a.prio == 1) __builtin_amdgcn_s_setprio(3);  // A/B: the flush ahead of other waves' chains
  else if (a.prio == 3) __builtin_amdgcn_s_setprio(2);
  tile_flush_rt<OutT>(gout, stage_b, mis, Sv * (int)MC * (int)sizeof(OutT), a.write_through);
  phase_stamp(a.stamps, wave, 4);
}

template <int LT, int CT, bool FUSED, typename OutT, bool MAYMU = true>
__global__ __launch_bounds__(512) void action_fwd_tile_kernel(ActionArgs a) {
  fwd_tile_body<LT, CT, FUSED, OutT, MAYMU>(a, blockIdx.x);
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

// Compile-time channel count of the specialised tile kernel (ActionNet's default
// rep_copies, decoders.py:11, and every BASELINE config).
constexpr int kTileFastC = 10;

struct FwdLaunch {
  ActionArgs a;
  int gx, gy;
  bool fused;
  bool tile;     // tile kernel (shared spectrum; gy = waves per block)
  size_t lds;    // tile kernel dynamic LDS bytes
  int dtype;
  hipStream_t stream;
};

// Launchers: run() is defined out of class (not implicitly inline), so that the
// `extern template` declarations in action.hip keep the host TU from instantiating --
// and the device compiler from compiling -- every kernel a second time.
template <int LT>
struct FwdLauncher {
  using Args = FwdLaunch;
  template <int CT>
  static void launch_tile(FwdLaunch& p, bool bf16);
  static int run(FwdLaunch& p);
};

template <int LT>
template <int CT>
void FwdLauncher<LT>::launch_tile(FwdLaunch& p, bool bf16) {
  const dim3 grid(p.gx), block(64 * p.gy);
  if (p.fused && CT > 0 && !p.a.mu) {
    // no mean rotation (the metric path, z = exp(v)): the instantiation without the fp64
    // mu prologue -- 1,660 -> ~700 instructions ahead of the first barrier at l = 10, so
    // fewer cold instruction-cache lines on every block's critical path
    if (bf16)
      hipLaunchKernelGGL((action_fwd_tile_kernel<LT, CT, true, __hip_bfloat16, false>), grid, block, p.lds, p.stream, p.a);
    else
      hipLaunchKernelGGL((action_fwd_tile_kernel<LT, CT, true, float, false>), grid, block, p.lds, p.stream, p.a);
  } else if (p.fused) {
    if (bf16)
      hipLaunchKernelGGL((action_fwd_tile_kernel<LT, CT, true, __hip_bfloat16>), grid, block, p.lds, p.stream, p.a);
    else
      hipLaunchKernelGGL((action_fwd_tile_kernel<LT, CT, true, float>), grid, block, p.lds, p.stream, p.a);
  } else {
    if (bf16)
      hipLaunchKernelGGL((action_fwd_tile_kernel<LT, CT, false, __hip_bfloat16>), grid, block, p.lds, p.stream, p.a);
    else
      hipLaunchKernelGGL((action_fwd_tile_kernel<LT, CT, false, float>), grid, block, p.lds, p.stream, p.a);
  }
}

template <int LT>
int FwdLauncher<LT>::run(FwdLaunch& p) {
  const bool bf16 = p.dtype == LV_DTYPE_BF16;
  if (p.tile) {
    if (p.a.C == kTileFastC)
      launch_tile<kTileFastC>(p, bf16);
    else
      launch_tile<0>(p, bf16);
    LV_RETURN_LAUNCH("action_fwd_tile_kernel");
  }
  const bool shared = p.a.Fstride == 0;
  const size_t lds = p.lds;  // spectrum slice + trig tables (plan_fwd in action.hip)
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

struct WigLaunch {
  const float* ang;
  float* D;
  int64_t n;
  int dsz;
  hipStream_t stream;
};

template <int l>
struct WigLauncher {
  static int run(WigLaunch& p);
};
template <int l>
int WigLauncher<l>::run(WigLaunch& p) {
  const int64_t total = p.n * (2 * l + 1);
  hipLaunchKernelGGL((wigner_d_kernel<l>), dim3(ceil_div(total, 256)), dim3(256), 0, p.stream,
                     p.ang, p.D, p.n, p.dsz);
  LV_RETURN_LAUNCH("wigner_d_kernel");
}

#define LV_EXTERN_LAUNCHERS(L)            \
  extern template struct FwdLauncher<L>;  \
  extern template struct WigLauncher<L>;

}  // namespace lv

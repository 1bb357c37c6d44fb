#pragma once
// Experimental backward variants for tools/bwdbench.hip A/B runs (never built into the
// library).  All are the library's action_bwd_tile_kernel for C = 10, shared spectrum,
// one sample group per block, 3 waves per SIMD (bwd_wide), with switches:
//   kXWaveLocal : no barrier before the chain -- every wave stages ITS OWN rows of the
//                 upstream-gradient tile (8-byte loads, issued first) and runs its own
//                 prologue (sincos + multiples up to its last degree) into a wave-private
//                 table, so no wave waits for another wave's loads or for wave 0's prologue
//   kXSlabUnroll: the per-degree dF slab sum over the group's samples with the compile-
//                 time group size (loads batched) when the group is full
//   kXMultReg   : the X products generate their (cos, sin) multiples in registers from
//                 the slot's (cos, sin) (read once per lane) instead of reading the LDS
//                 table per product: 4 VALU per multiple against 2 LDS bytes... per lane
//   kXGlds      : the upstream-gradient tile goes global -> LDS by LDS-DMA
//                 (global_load_lds: 16-byte body, 4-byte edges; with kXWaveLocal 4-byte
//                 runs of the wave's rows): no VGPRs (nor scratch) hold it in flight
// and diagnostics that drop work (results wrong, timing only):
//   kXDiagNoG   : no upstream-gradient loads (tile left as is)
//   kXDiagNoSlab: no dF slab accumulation
//   kXDiagNoChain: no per-degree chain (loads, prologue, reductions only)
#include "action_bwd.h"

namespace lv {

constexpr int kXWaveLocal = 1, kXSlabUnroll = 2, kXDiagNoG = 4, kXDiagNoSlab = 8,
              kXDiagNoChain = 16, kXGlds = 32, kXMultReg = 64;

// y = X x (T = false) or X^T x (T = true) with the multiples generated in registers by
// trig_row_fill's recurrence from (cos, sin) of the slot's angle: bitwise equal to the
// table version, no LDS reads (4 VALU per multiple instead).
template <int l, bool T>
__device__ __forceinline__ void xm_rec(float c1, float s1, const float (&x)[2 * l + 1],
                                       float (&y)[2 * l + 1]) {
  y[l] = x[l];
  float cf = c1, sf = s1;
  sfor<l>([&](auto F) {
    constexpr int f = LV_CV(F) + 1;
    if constexpr (f >= 2) {
      const float cn = fmaf(cf, c1, -(sf * s1));
      sf = fmaf(sf, c1, cf * s1);
      cf = cn;
    }
    constexpr int i = l - f, i2 = l + f;  // rows with frequency +f and -f
    if constexpr (!T) {
      y[i] = fmaf(cf, x[i], sf * x[2 * l - i]);
      y[i2] = fmaf(cf, x[i2], -(sf * x[2 * l - i2]));
    } else {
      y[i] = fmaf(cf, x[i], -(sf * x[2 * l - i]));
      y[i2] = fmaf(cf, x[i2], sf * x[2 * l - i2]);
    }
  });
}

constexpr int kBwdLoadsPerThread = 8;  // register-staged tile: 16-B loads per thread

__host__ __device__ inline int bwdx_trig_floats(int Sw, int L, int nseg, int var) {
  return (var & kXWaveLocal) ? nseg * bwd_trig_floats(Sw, L) : bwd_trig_floats(Sw, L);
}

template <int LT, int VAR>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(3)))
void bwd_x_kernel(ActionBwdArgs a) {
  constexpr int CT = 10;
  constexpr int Sw = 64 / CT;
  constexpr bool WL = (VAR & kXWaveLocal) != 0;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  typedef float f4 __attribute__((ext_vector_type(4)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  constexpr int kRow = TrigLds<LT>::kRow;
  constexpr int C = CT;
  constexpr int64_t MC = (int64_t)(LT + 1) * (LT + 1) * CT;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tid = (int)threadIdx.x, nthr = (int)blockDim.x;
  const int nw = nthr >> 6;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int rows_lo = lo * lo;
  const int stage_bytes = tile_stage_bytes(Sw, MC, 4);
  float* trig = lds + (stage_bytes >> 2);
  float* trig_w = WL ? trig + wave * bwd_trig_floats(Sw, LT) : trig;
  float* apart = trig + bwdx_trig_floats(Sw, LT, nw, VAR);
  float* slabL = apart + nw * 64 * 3;
  float* Fw = slabL + (int)MC + wave * a.fpitch;
  constexpr int kFPer = 6;
  const int fcnt = (hi * hi - rows_lo) * C;
  const float* fsrc = a.F + rows_lo * C;
  const int64_t g = blockIdx.x;
  const int64_t s0 = g * Sw;
  const int Sv = (int)min((int64_t)Sw, a.n - s0);
  const bool active = j < Sv;
  const int nbytes = Sv * (int)MC * 4;
  const float* gsrc = a.gout + s0 * MC;
  const int mis = (int)(reinterpret_cast<uintptr_t>(gsrc) & 15);
  char* stage_b = reinterpret_cast<char*>(lds) + mis;
  const __amdgpu_buffer_rsrc_t rg =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(gsrc), 0, nbytes, kRawBufferFlags);
  // upstream gradient: block tile (library) or this wave's rows (8-byte loads)
  constexpr int kWLPer = 24;  // 8-byte loads held per lane (covers <= 64*24*2 floats)
  f4 gv[kBwdLoadsPerThread];
  f2 gw[kWLPer];
  const int run = fcnt;  // floats of this wave's rows per sample
  const int npair = Sv * (run >> 1);
  if constexpr ((VAR & kXGlds) && !(VAR & kXDiagNoG)) {
    if constexpr (WL) {
      for (int jj = 0; jj < Sv; ++jj)
        for (int k0 = 0; k0 < run; k0 += 64) {
          const int off = jj * (int)MC + rows_lo * C + k0;
          if (k0 + lane < run)
            __builtin_amdgcn_global_load_lds(gsrc + off + lane, as_lds(stage_b + 4 * off), 4, 0, 0);
        }
    } else {
      const int head = min((16 - mis) & 15, nbytes);
      const int nvec = (nbytes - head) >> 4;
      const int tail0 = head + nvec * 16;
      for (int v0 = wave * 64; v0 < nvec; v0 += nthr)
        if (v0 + lane < nvec)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(gsrc) + head + 16 * (v0 + lane),
                                           as_lds(stage_b + head + 16 * v0), 16, 0, 0);
      if (wave == 0) {
        if (4 * lane < head)
          __builtin_amdgcn_global_load_lds(gsrc + lane, as_lds(stage_b), 4, 0, 0);
        if (tail0 + 4 * lane < nbytes)
          __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(gsrc) + tail0 + 4 * lane,
                                           as_lds(stage_b + tail0), 4, 0, 0);
      }
    }
  } else if constexpr (!(VAR & kXDiagNoG)) {
    if constexpr (WL) {
#pragma unroll
      for (int k = 0; k < kWLPer; ++k) {
        const int p = lane + 64 * k;
        if (p < npair) {
          const int jj = p / (run >> 1), e = 2 * (p - jj * (run >> 1));
          gw[k] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(
                                             rg, (jj * (int)MC + rows_lo * C + e) * 4, 0, 0));
        }
      }
    } else {
      const int head = min((16 - mis) & 15, nbytes);
      const int nvec = (nbytes - head) >> 4;
#pragma unroll
      for (int k = 0; k < kBwdLoadsPerThread; ++k) {
        const int v = tid + k * nthr;
        if (v < nvec)
          gv[k] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rg, head + 16 * v, 0, 0));
      }
    }
  }
  {
    float fv[kFPer];
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {
      const int e = lane + 64 * k;
      fv[k] = e < fcnt ? fsrc[e] : 0.f;
    }
    for (int e = lane; e < fcnt; e += 64) slabL[rows_lo * C + e] = 0.f;
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {
      const int e = lane + 64 * k;
      if (e < fcnt) Fw[e] = fv[k];
    }
    for (int e = lane + 64 * kFPer; e < fcnt; e += 64) Fw[e] = fsrc[e];
  }
  const float* Fl = Fw + c - rows_lo * C;
  // prologue: (sample, slot) tasks -- the block's first 3*Sw threads (library) or the
  // first 3*Sw lanes of every wave, each wave up to its own last degree
  {
    const int t = WL ? lane : tid;
    if (t < 3 * Sw) {
      const int jt = t / 3, q = t - 3 * (t / 3);
      const int64_t st = s0 + min(jt, Sv - 1);
      float cc[3], ss[3], c1[3], s1[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) sincosf(a.ang[st * 3 + i], &ss[i], &cc[i]);
      if (a.transpose) {
        c1[0] = cc[2]; s1[0] = -ss[2];
        c1[1] = cc[1]; s1[1] = -ss[1];
        c1[2] = cc[0]; s1[2] = -ss[0];
      } else {
#pragma unroll
        for (int i = 0; i < 3; ++i) { c1[i] = cc[i]; s1[i] = ss[i]; }
      }
      trig_row_fill<LT>(trig_w + jt * kRow, c1, s1, q, WL ? hi - 1 : LT);
    }
  }
  if constexpr (VAR & kXGlds) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS-DMA writes landed
  } else if constexpr (!(VAR & kXDiagNoG)) {
    if constexpr (WL) {
#pragma unroll
      for (int k = 0; k < kWLPer; ++k) {
        const int p = lane + 64 * k;
        if (p < npair) {
          const int jj = p / (run >> 1), e = 2 * (p - jj * (run >> 1));
          *reinterpret_cast<f2*>(stage_b + (jj * (int)MC + rows_lo * C + e) * 4) = gw[k];
        }
      }
      for (int p = lane + 64 * kWLPer; p < npair; p += 64) {
        const int jj = p / (run >> 1), e = 2 * (p - jj * (run >> 1));
        *reinterpret_cast<f2*>(stage_b + (jj * (int)MC + rows_lo * C + e) * 4) = __builtin_bit_cast(
            f2, __builtin_amdgcn_raw_buffer_load_b64(rg, (jj * (int)MC + rows_lo * C + e) * 4, 0, 0));
      }
    } else {
      const int head = min((16 - mis) & 15, nbytes);
      const int nvec = (nbytes - head) >> 4;
      const int tail0 = head + nvec * 16;
#pragma unroll
      for (int k = 0; k < kBwdLoadsPerThread; ++k) {
        const int v = tid + k * nthr;
        if (v < nvec) *reinterpret_cast<f4*>(stage_b + head + 16 * v) = gv[k];
      }
      for (int v = tid + kBwdLoadsPerThread * nthr; v < nvec; v += nthr)
        *reinterpret_cast<f4*>(stage_b + head + 16 * v) =
            __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rg, head + 16 * v, 0, 0));
      const int nedge = head / 4 + (nbytes - tail0) / 4;
      if (tid < nedge) {
        const int b = tid < head / 4 ? tid * 4 : tail0 + (tid - head / 4) * 4;
        *reinterpret_cast<float*>(stage_b + b) =
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, b, 0, 0));
      }
    }
  }
  if constexpr (WL)
    wave_lds_sync();
  else
    block_sync_lds();

  float* tile_lane = reinterpret_cast<float*>(stage_b) + j * MC + c;
  const float* tj = trig_w + min(j, Sw - 1) * kRow;
  float ga = 0.f, gb = 0.f, gc = 0.f;
  float mc[3], ms[3];  // kXMultReg: (cos, sin) of the three slots, f = 1 of the table
  if constexpr ((VAR & kXMultReg) != 0) {
    constexpr int TP = TrigLds<LT>::TP;
#pragma unroll
    for (int A = 0; A < 3; ++A) {
      mc[A] = tj[2 * A * TP + 1];
      ms[A] = tj[(2 * A + 1) * TP + 1];
    }
  }
  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if (l >= lo && l < hi) {
      constexpr int nn = 2 * l + 1;
      constexpr int r0 = l * l;
      if constexpr (!(VAR & kXDiagNoChain)) {
        float p2[nn], p4[nn], gq[nn], u[nn];
        constexpr bool MR = (VAR & kXMultReg) != 0;
        {
          float f0[nn];
          sfor<nn>([&](auto K) { f0[LV_CV(K)] = Fl[(r0 + LV_CV(K)) * C]; });
          if constexpr (MR) xm_rec<l, false>(mc[2], ms[2], f0, u);
          else xm<l>(mult_lds<l, 2, LT>(tj), f0, u);
        }
        jmul<l>(u, p2);
        if constexpr (MR) xm_rec<l, false>(mc[1], ms[1], p2, u);
        else xm<l>(mult_lds<l, 1, LT>(tj), p2, u);
        jmul<l>(u, p4);
        sfor<nn>([&](auto K) { gq[LV_CV(K)] = active ? tile_lane[(r0 + LV_CV(K)) * C] : 0.f; });
        if constexpr (MR) xm_rec<l, true>(mc[0], ms[0], gq, u);
        else xm_t<l>(mult_lds<l, 0, LT>(tj), gq, u);
        ga += kdot<l>(u, p4);
        jmul<l>(u, p4);
        if constexpr (MR) xm_rec<l, true>(mc[1], ms[1], p4, u);
        else xm_t<l>(mult_lds<l, 1, LT>(tj), p4, u);
        gb += kdot<l>(u, p2);
        jmul<l>(u, p2);
        if constexpr (MR) xm_rec<l, true>(mc[2], ms[2], p2, u);
        else xm_t<l>(mult_lds<l, 2, LT>(tj), p2, u);
        {
          float f0[nn];
          sfor<nn>([&](auto K) { f0[LV_CV(K)] = Fl[(r0 + LV_CV(K)) * C]; });
          gc += kdot<l>(u, f0);
        }
        if (active) sfor<nn>([&](auto I) { tile_lane[(r0 + LV_CV(I)) * C] = u[LV_CV(I)]; });
      }
      if constexpr (!(VAR & kXDiagNoSlab)) {
        wave_lds_sync();
        const float* col0 = reinterpret_cast<const float*>(stage_b) + r0 * C;
        if ((VAR & kXSlabUnroll) && Sv == Sw) {
          for (int e = lane; e < nn * C; e += 64) {
            float v[Sw];
#pragma unroll
            for (int jj = 0; jj < Sw; ++jj) v[jj] = col0[jj * MC + e];
            float sum = v[0];
#pragma unroll
            for (int jj = 1; jj < Sw; ++jj) sum += v[jj];
            slabL[r0 * C + e] += sum;
          }
        } else {
          for (int e = lane; e < nn * C; e += 64) {
            float sum = col0[e];
            for (int jj = 1; jj < Sv; ++jj) sum += col0[jj * MC + e];
            slabL[r0 * C + e] += sum;
          }
        }
      }
    }
  });
  float* ap = apart + wave * 64 * 3;
  if (a.transpose) {
    ap[lane * 3 + 0] = -gc; ap[lane * 3 + 1] = -gb; ap[lane * 3 + 2] = -ga;
  } else {
    ap[lane * 3 + 0] = ga; ap[lane * 3 + 1] = gb; ap[lane * 3 + 2] = gc;
  }
  block_sync_lds();
  if (tid < 3 * Sv) {
    const int js = tid / 3, i = tid - 3 * (tid / 3);
    float r = 0.f;
    for (int w = 0; w < nw; ++w) {
      float sw = 0.f;
      for (int cc2 = 0; cc2 < C; ++cc2) sw += apart[(w * 64 + js * C + cc2) * 3 + i];
      r += sw;
    }
    a.gang[(s0 + js) * 3 + i] = r;
  }
  float* slab = a.ws_F + (int64_t)blockIdx.x * MC;
  for (int e = lane; e < fcnt; e += 64) slab[rows_lo * C + e] = slabL[rows_lo * C + e];
}

}  // namespace lv

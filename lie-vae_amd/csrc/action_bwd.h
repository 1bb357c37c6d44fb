#pragma once
// Backward of the group action (angles + spectrum gradients) for gfx950, one kernel
// per fixed degree range (action_bwd_inst.hip, -DLV_BWD_R=r), plus its launcher.
#include "action_common.h"

namespace lv {

// ---------------------------------------------------------------- backward
// Per lane (sample, column), per degree, with G = gout block column:
//   P1 = Xc F, P2 = J P1, P3 = Xb P2, P4 = J P3           (forward recompute)
//   Q4 = Xa^T G, Q3 = J Q4, Q2 = Xb^T Q3, Q1 = J Q2, dF = Xc^T Q1
//   d/da = <G, Xa' P4>, d/db = <Q3, Xb' P2>, d/dc = <Q1, Xc' F>
// Angle partials are summed over the C lanes of a sample in LDS (fixed order) and
// written per segment to the workspace; dF is summed over the wave's samples and its
// grid-stride loop into a per-wave LDS accumulator, then per block into a slab.
// A second kernel reduces slabs and segments in a fixed order (bitwise reproducible).
struct ActionBwdArgs {
  const float* ang;
  const float* F;
  int64_t Fstride;
  const float* gout;
  float* gF;           // per-sample spectrum: written directly
  float* ws_ang;       // [nranges][n][3]
  float* ws_F;         // [gridX][M*C] (shared F only)
  int64_t n;
  int64_t MC;
  int C, Sw, transpose, groups, L, slot;
};

// Degree ranges of the backward, fixed at compile time and shared by every l_max:
// [0,6) [6,8) then one degree per range up to 20.  Each range is its own kernel (small
// functions: fast to compile, registers sized to the range), launched one after another;
// the range containing l_max is clipped at run time.
constexpr int kNumBwdRanges = 15;
__host__ __device__ constexpr int bwd_range_lo(int r) { return r == 0 ? 0 : (r == 1 ? 6 : r + 6); }
__host__ __device__ constexpr int bwd_range_hi(int r) { return r == 0 ? 6 : (r == 1 ? 8 : r + 7); }
inline int bwd_num_ranges(int L) {
  int n = 0;
  while (n < kNumBwdRanges && bwd_range_lo(n) <= L) ++n;
  return n;
}
inline int bwd_wave_floats(int r, int L, int C, bool sharedF) {
  const int hi = bwd_range_hi(r) < L + 1 ? bwd_range_hi(r) : L + 1;
  const int lo = bwd_range_lo(r);
  const int LT = bwd_range_hi(r) - 1;
  return 64 * (2 * LT + 1) + 64 * 3 + (sharedF ? (hi * hi - lo * lo) * C : 0);
}

template <int R>
__global__ __launch_bounds__(kThreads) void action_bwd_kernel(ActionBwdArgs a) {
  constexpr int LO = bwd_range_lo(R), HI = bwd_range_hi(R), LT = HI - 1;
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int C = a.C, Sw = a.Sw;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = LO, hi = min(HI, a.L + 1);
  const bool sharedF = a.Fstride == 0;
  const int rows_lo = lo * lo, rows_hi = hi * hi;
  const int seg_len = (rows_hi - rows_lo) * C;
  // LDS: per wave [stage 64*(2LT+1)] [angle partials 64*3] [dF accumulator seg_len]
  const int wave_floats = 64 * (2 * LT + 1) + 64 * 3 + (sharedF ? seg_len : 0);
  float* stage = lds + wave * wave_floats;
  float* apart = stage + 64 * (2 * LT + 1);
  float* facc = apart + 64 * 3;
  if (sharedF)
    for (int e = lane; e < seg_len; e += 64) facc[e] = 0.f;
  wave_lds_sync();

  for (int g = blockIdx.x; g < a.groups; g += gridDim.x) {
    const int64_t s0 = ((int64_t)g * kWavesPerBlock + wave) * Sw;
    if (s0 >= a.n) break;
    const int Sv = (int)min((int64_t)Sw, a.n - s0);
    const int64_t s = s0 + j;
    const bool active = j < Sv;
    float cc[3] = {1.f, 1.f, 1.f}, ss[3] = {0.f, 0.f, 0.f};
    if (active)
      for (int i = 0; i < 3; ++i) sincosf(a.ang[s * 3 + i], &ss[i], &cc[i]);
    float c1[3], s1[3];
    if (a.transpose) {
      c1[0] = cc[2]; s1[0] = -ss[2];
      c1[1] = cc[1]; s1[1] = -ss[1];
      c1[2] = cc[0]; s1[2] = -ss[0];
    } else {
      for (int i = 0; i < 3; ++i) { c1[i] = cc[i]; s1[i] = ss[i]; }
    }
    TrigTab<LT> t;
    trig_fill<LT>(t, c1, s1, hi - 1);
    float ga = 0.f, gb = 0.f, gc = 0.f;
    const float* Fbase = a.F + (active ? s * a.Fstride : 0) + c;

    sfor<HI - LO>([&](auto Lc) {
      constexpr int l = LO + LV_CV(Lc);
      if (l < hi) {
        constexpr int nn = 2 * l + 1;
        constexpr int r0 = l * l;
        const int rowlen = nn * C;
        const int total = Sv * rowlen;
        const int q64 = 64 / rowlen, r64 = 64 - q64 * rowlen;
        // stage gout rows (contiguous) into LDS, then read columns
        {
          int jj = lane / rowlen, w = lane - jj * rowlen;
          const float* src0 = a.gout + s0 * a.MC + (int64_t)r0 * C;
          for (int e = lane; e < total; e += 64) {
            stage[e] = src0[jj * a.MC + w];
            jj += q64;
            w += r64;
            if (w >= rowlen) { w -= rowlen; ++jj; }
          }
        }
        wave_lds_sync();
        float f0[nn], p2[nn], p4[nn], gq[nn], u[nn];
        const float* Fp = Fbase + r0 * C;
        sfor<nn>([&](auto K) {
          constexpr int k = LV_CV(K);
          f0[k] = active ? Fp[k * C] : 0.f;
          gq[k] = active ? stage[(j * nn + k) * C + c] : 0.f;
        });
        wave_lds_sync();
        xrot<l, 2>(t, f0, u);
        jmul<l>(u, p2);
        xrot<l, 1>(t, p2, u);
        jmul<l>(u, p4);
        ga += xrot_dot_deriv<l, 0>(t, gq, p4);
        xrot_t<l, 0>(t, gq, u);   // Q4
        jmul<l>(u, p4);           // Q3 (reuse p4)
        gb += xrot_dot_deriv<l, 1>(t, p4, p2);
        xrot_t<l, 1>(t, p4, u);   // Q2
        jmul<l>(u, p2);           // Q1 (reuse p2)
        gc += xrot_dot_deriv<l, 2>(t, p2, f0);
        xrot_t<l, 2>(t, p2, u);   // dF column
        if (sharedF) {
          // sum over the wave's samples: stage [j][i][c], then owners add in order
          if (active) {
            sfor<nn>([&](auto I) {
              constexpr int i = LV_CV(I);
              stage[(j * nn + i) * C + c] = u[i];
            });
          }
          wave_lds_sync();
          float* acc = facc + (r0 - rows_lo) * C;
          for (int e = lane; e < rowlen; e += 64) {
            float sum = acc[e];
            for (int jj = 0; jj < Sv; ++jj) sum += stage[jj * rowlen + e];
            acc[e] = sum;
          }
          wave_lds_sync();
        } else {
          if (active) {
            sfor<nn>([&](auto I) {
              constexpr int i = LV_CV(I);
              stage[(j * nn + i) * C + c] = u[i];
            });
          }
          wave_lds_sync();
          int jj = lane / rowlen, w = lane - jj * rowlen;
          float* dst0 = a.gF + s0 * a.MC + (int64_t)r0 * C;
          for (int e = lane; e < total; e += 64) {
            dst0[jj * a.MC + w] = stage[e];
            jj += q64;
            w += r64;
            if (w >= rowlen) { w -= rowlen; ++jj; }
          }
          wave_lds_sync();
        }
      }
    });
    // angle partials: sum over the C lanes of each sample in column order
    float g3[3];
    if (a.transpose) { g3[0] = -gc; g3[1] = -gb; g3[2] = -ga; }
    else { g3[0] = ga; g3[1] = gb; g3[2] = gc; }
    apart[lane * 3 + 0] = g3[0];
    apart[lane * 3 + 1] = g3[1];
    apart[lane * 3 + 2] = g3[2];
    wave_lds_sync();
    if (active && c == 0) {
      float r[3] = {0.f, 0.f, 0.f};
      for (int cc2 = 0; cc2 < C; ++cc2)
        for (int i = 0; i < 3; ++i) r[i] += apart[(lane + cc2) * 3 + i];
      float* dst = a.ws_ang + ((int64_t)a.slot * a.n + s) * 3;
      dst[0] = r[0]; dst[1] = r[1]; dst[2] = r[2];
    }
    wave_lds_sync();
  }
  if (sharedF) {
    __syncthreads();
    // block slab: sum the 4 wave accumulators in wave order
    const float* acc0 = lds + 64 * (2 * LT + 1) + 64 * 3;
    float* slab = a.ws_F + (int64_t)blockIdx.x * a.MC + (int64_t)rows_lo * C;
    for (int e = threadIdx.x; e < seg_len; e += kThreads) {
      float sum = 0.f;
      for (int w = 0; w < kWavesPerBlock; ++w) sum += acc0[w * wave_floats + e];
      slab[e] = sum;
    }
  }
}

struct BwdLaunch {
  ActionBwdArgs a;
  int gx;
  hipStream_t stream;
};

template <int R>
struct BwdLauncher {
  static int run(BwdLaunch& p) {
    const size_t lds = sizeof(float) * kWavesPerBlock *
                       (size_t)bwd_wave_floats(R, p.a.L, p.a.C, p.a.Fstride == 0);
    hipLaunchKernelGGL((action_bwd_kernel<R>), dim3(p.gx), dim3(kThreads), lds, p.stream, p.a);
    LV_RETURN_LAUNCH("action_bwd_kernel");
  }
};

#define LV_EXTERN_BWD(R) extern template struct BwdLauncher<R>;

}  // namespace lv

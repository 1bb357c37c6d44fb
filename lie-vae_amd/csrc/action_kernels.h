#pragma once
// Group-action decoder kernels for gfx950 (MI355X) -- templates + launchers.
// Instantiated once per l_max in action_inst.hip (-DLV_INST_L=k) so the 21
// degree variants compile in parallel; host planning lives in action.hip.
//
//   lv_group_action_fwd      block_wigner_matrix_multiply, lie_tools.py:226-253
//   lv_fused_exp_action_fwd  mu@rodrigues(v) -> ZYZ -> block D·F in one pass
//                            (reparameterize.py:269-273, vae.py:182, decoders.py:47-56)
//   lv_group_action_bwd      its autograd backward (angles + spectrum gradients)
//   lv_wigner_d_fwd          packed D_l blocks (parity / debug only)
//
// Work decomposition:
//   * lane = (sample slot j, column c): a wave holds Sw = 64 / C samples x C columns;
//   * block = 4 waves, all on the same contiguous range ("segment") of degrees
//     [lo, hi) chosen on the host so that the grid has >= ~2 waves per SIMD even at
//     batch 4096 and the segments cost about the same (cost model: J non-zeros);
//   * per degree each lane runs the factored chain of action_chain.h in registers;
//     the wave stages its Sw x (2l+1) x C output block in LDS and writes it back as
//     contiguous rows (the (n, M, C) layout is row-contiguous per sample and degree).
#include "action_chain.h"
#include "so3_device.h"

namespace lv {

constexpr int kWavesPerBlock = 4;
constexpr int kThreads = 64 * kWavesPerBlock;
constexpr int kMaxSeg = 16;

struct ActionArgs {
  const float* ang;     // (n,3) angles (non-fused)
  const float* mu;      // (n,3,3) or null (fused)
  const float* v;       // (n,3) algebra vector (fused)
  const float* F;       // spectrum
  int64_t Fstride;      // 0 (shared) or M*C
  void* out;            // (n,M,C)
  float* ang_out;       // optional (fused)
  int64_t n;
  int64_t MC;
  int C, Sw, transpose;
  int seg_lo[kMaxSeg + 1];
};

// ZYZ (cos, sin) straight from the quaternion, same function as
// quaternions_to_eazyz (lie_tools.py:160-175) followed by cos/sin: atan2(y, x) ->
// (x, y)/hypot, acos(clamp(w)) -> (w, sqrt((1-w)(1+w))).  atan2(0, 0) edge mirrored.
__device__ __forceinline__ void quat_to_zyz_trig(const float q[4], float c1[3], float s1[3]) {
  const float a1 = q[1] * q[2] - q[0] * q[3];
  const float b1 = q[0] * q[2] + q[1] * q[3];
  const float cb = ((q[3] * q[3] - q[0] * q[0]) - q[1] * q[1]) + q[2] * q[2];
  const float a3 = q[0] * q[3] + q[1] * q[2];
  const float b3 = q[1] * q[3] - q[0] * q[2];
  auto dir = [](float y, float x, float& c, float& s) {
    if (x == 0.f && y == 0.f) {  // atan2(+-0, +-0) in {0, +-pi}
      c = signbit(x) ? -1.f : 1.f;
      s = 0.f;
    } else {
      const float r = rhypotf(x, y);
      c = x * r;
      s = y * r;
    }
  };
  dir(a1, b1, c1[0], s1[0]);
  const float x = fminf(fmaxf(cb, kEazyzLo), kEazyzHi);
  c1[1] = x;
  s1[1] = sqrtf((1.f - x) * (1.f + x));
  dir(a3, b3, c1[2], s1[2]);
}

// Per-lane angle setup; returns (cos, sin) of the three chain angles.  For transpose
// (D^T = X(-c) J X(-b) J X(-a)) the slots are swapped and the sines negated.
template <bool FUSED>
__device__ __forceinline__ void lane_angles(const ActionArgs& a, int64_t s, bool active, int c,
                                            bool write_ang, float c1[3], float s1[3]) {
  float cc[3] = {1.f, 1.f, 1.f}, ss[3] = {0.f, 0.f, 0.f};
  if (active) {
    if constexpr (FUSED) {
      float v[3] = {a.v[s * 3 + 0], a.v[s * 3 + 1], a.v[s * 3 + 2]};
      float R[9], z[9];
      rodrigues_fwd(v, R);
      if (a.mu) {
        float mu[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) mu[i] = a.mu[s * 9 + i];
        matmul3(mu, R, z);
      } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) z[i] = R[i];
      }
      float q[4];
      mat_to_quat_fwd(z, q, nullptr);
      quat_to_zyz_trig(q, cc, ss);
      if (write_ang && c == 0) {
        float ang[3];
        quat_to_eazyz_fwd(q, ang);
        a.ang_out[s * 3 + 0] = ang[0];
        a.ang_out[s * 3 + 1] = ang[1];
        a.ang_out[s * 3 + 2] = ang[2];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i) sincosf(a.ang[s * 3 + i], &ss[i], &cc[i]);
    }
  }
  if (a.transpose) {
    c1[0] = cc[2]; s1[0] = -ss[2];
    c1[1] = cc[1]; s1[1] = -ss[1];
    c1[2] = cc[0]; s1[2] = -ss[0];
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i) { c1[i] = cc[i]; s1[i] = ss[i]; }
  }
}

// Rows of a degree segment's spectrum slice as staged in LDS, column-major
// ([c][row]) so that a lane's column is contiguous (immediate LDS offsets) and padded
// to an odd count so that the C columns fall in different banks.
__host__ __device__ inline int fseg_rows(int lo, int hi) { return (hi * hi - lo * lo) | 1; }

// Forward.  Per degree each lane runs the factored chain on its column and stores its
// (2l+1) outputs straight from registers: one store instruction per output row puts
// Sw contiguous C-float pieces (one per sample) in flight; consecutive rows of a sample
// are adjacent, so L2 merges them into whole lines before they reach HBM.  There is no
// load after the first store (vmcnt retires in order, so a later load would wait for
// every older store): a shared spectrum is staged into LDS up front and a per-sample
// spectrum is prefetched one degree ahead.
template <int LT, bool FUSED, bool SHARED, typename OutT>
__global__ __launch_bounds__(kThreads) void action_fwd_kernel(ActionArgs a) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int C = a.C, Sw = a.Sw;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[blockIdx.y], hi = a.seg_lo[blockIdx.y + 1];
  const int rows_lo = lo * lo;
  const int frows = fseg_rows(lo, hi);
  if constexpr (SHARED) {
    const float* src = a.F + rows_lo * C;
    const int cnt = (hi * hi - rows_lo) * C;
    for (int e = threadIdx.x; e < cnt; e += kThreads) {
      const int r = e / C, cc = e - r * C;
      lds[cc * frows + r] = src[e];
    }
    __syncthreads();
  }
  const int64_t s0 = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * Sw;
  if (s0 >= a.n) return;  // whole wave idle (no block barriers below)
  const int Sv = (int)min((int64_t)Sw, a.n - s0);
  const int64_t s = s0 + j;
  const bool active = j < Sv;

  float c1[3], s1[3];
  lane_angles<FUSED>(a, s, active, c, FUSED && a.ang_out && blockIdx.y == 0, c1, s1);
  TrigTab<LT> t;
  trig_fill<LT>(t, c1, s1, hi - 1);

  OutT* dst = reinterpret_cast<OutT*>(a.out) + (active ? s * a.MC + c : 0);
  const float* Fl = lds + c * frows - rows_lo;                  // shared: LDS column
  // per-sample: global; idle lanes read sample s0's column (valid memory, result unused)
  const float* Fs = a.F + (active ? s : s0) * a.Fstride + c;
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
      xrot<l, 2>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 1>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 0>(t, x, y);
      if (active) {
        OutT* d = dst + r0 * C;
        sfor<nn>([&](auto I) {
          store_out(d, y[LV_CV(I)]);
          d += C;
        });
      }
    }
  });
}

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
  float* gang;         // final (n,3) (written by reduce kernel)
  float* gF;           // final
  float* ws_ang;       // [nseg][n][3]
  float* ws_F;         // [gridX][M*C] (shared F only)
  int64_t n;
  int64_t MC;
  int C, Sw, transpose, nseg, groups;
  int seg_lo[kMaxSeg + 1];
};

template <int LT>
__global__ __launch_bounds__(kThreads) void action_bwd_kernel(ActionBwdArgs a) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int C = a.C, Sw = a.Sw;
  const int j = lane / C;
  const int c = lane - j * C;
  const int lo = a.seg_lo[blockIdx.y], hi = a.seg_lo[blockIdx.y + 1];
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

    sfor<LT + 1>([&](auto Lc) {
      constexpr int l = LV_CV(Lc);
      if (l >= lo && l < hi) {
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
      float* dst = a.ws_ang + ((int64_t)blockIdx.y * a.n + s) * 3;
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

// ------------------------------------------------------------ Wigner-D blocks
// Column q of D_l = chain applied to e_q; one thread per (sample, l, q).
template <int LT>
__global__ void wigner_d_kernel(const float* ang, float* D, int64_t n) {
  constexpr int cols = (LT + 1) * (LT + 1);  // sum_l (2l+1)
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= n * cols) return;
  const int64_t s = tid / cols;
  const int col = (int)(tid - s * cols);
  float c1[3], s1[3];
  for (int i = 0; i < 3; ++i) sincosf(ang[s * 3 + i], &s1[i], &c1[i]);
  TrigTab<LT> t;
  trig_fill<LT>(t, c1, s1, LT);
  constexpr int dsz = (LT + 1) * (2 * LT + 1) * (2 * LT + 3) / 3;
  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    constexpr int nn = 2 * l + 1;
    if (col >= l * l && col < (l + 1) * (l + 1)) {
      const int q = col - l * l;
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
  });
}

// ------------------------------------------------------------------ host side

struct FwdLaunch {
  ActionArgs a;
  int gx, gy;
  bool fused;
  int dtype;
  hipStream_t stream;
};

template <int LT>
struct FwdLauncher {
  using Args = FwdLaunch;
  static int run(FwdLaunch& p) {
    int fmax = 0;
    const bool shared = p.a.Fstride == 0;
    if (shared)
      for (int k = 0; k < p.gy; ++k)
        fmax = max(fmax, fseg_rows(p.a.seg_lo[k], p.a.seg_lo[k + 1]) * p.a.C);
    const size_t lds = sizeof(float) * (size_t)fmax;
    const dim3 grid(p.gx, p.gy), block(kThreads);
    const bool bf16 = p.dtype == LV_DTYPE_BF16;
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

struct BwdLaunch {
  ActionBwdArgs a;
  int gx, gy;
  size_t lds;
  hipStream_t stream;
};

template <int LT>
struct BwdLauncher {
  using Args = BwdLaunch;
  static int run(BwdLaunch& p) {
    hipLaunchKernelGGL((action_bwd_kernel<LT>), dim3(p.gx, p.gy), dim3(kThreads), p.lds, p.stream, p.a);
    LV_RETURN_LAUNCH("action_bwd_kernel");
  }
};

struct WigLaunch {
  const float* ang;
  float* D;
  int64_t n;
  hipStream_t stream;
};

template <int LT>
struct WigLauncher {
  using Args = WigLaunch;
  static int run(WigLaunch& p) {
    const int64_t total = p.n * (int64_t)(LT + 1) * (LT + 1);
    hipLaunchKernelGGL((wigner_d_kernel<LT>), dim3(ceil_div(total, 256)), dim3(256), 0, p.stream,
                       p.ang, p.D, p.n);
    LV_RETURN_LAUNCH("wigner_d_kernel");
  }
};

#define LV_EXTERN_LAUNCHERS(L)            \
  extern template struct FwdLauncher<L>;  \
  extern template struct BwdLauncher<L>;  \
  extern template struct WigLauncher<L>;

}  // namespace lv

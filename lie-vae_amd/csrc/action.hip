// Group-action decoder kernels for gfx950 (MI355X):
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
#include <algorithm>
#include <vector>

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

template <int LT, bool FUSED, typename OutT>
__global__ __launch_bounds__(kThreads) void action_fwd_kernel(ActionArgs a) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int C = a.C, Sw = a.Sw;
  const int j = lane / C;
  const int c = lane - j * C;
  const int64_t s0 = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * Sw;
  if (s0 >= a.n) return;  // whole wave idle (no block barriers below)
  const int Sv = (int)min((int64_t)Sw, a.n - s0);
  const int64_t s = s0 + j;
  const bool active = j < Sv;
  const int lo = a.seg_lo[blockIdx.y], hi = a.seg_lo[blockIdx.y + 1];

  float c1[3], s1[3];
  lane_angles<FUSED>(a, s, active, c, FUSED && a.ang_out && blockIdx.y == 0, c1, s1);
  TrigTab<LT> t;
  trig_fill<LT>(t, c1, s1, hi - 1);

  float* stage = lds + wave * (64 * (2 * LT + 1));
  OutT* out = reinterpret_cast<OutT*>(a.out);
  const float* Fbase = a.F + (active ? s * a.Fstride : 0) + c;

  sfor<LT + 1>([&](auto Lc) {
    constexpr int l = LV_CV(Lc);
    if (l >= lo && l < hi) {
      constexpr int nn = 2 * l + 1;
      constexpr int r0 = l * l;
      float x[nn], y[nn];
      const float* Fp = Fbase + r0 * C;
      sfor<nn>([&](auto K) {
        constexpr int k = LV_CV(K);
        x[k] = active ? Fp[k * C] : 0.f;
      });
      xrot<l, 2>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 1>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 0>(t, x, y);
      if (active) {
        sfor<nn>([&](auto I) {
          constexpr int i = LV_CV(I);
          stage[(j * nn + i) * C + c] = y[i];
        });
      }
      wave_lds_sync();
      // contiguous write-back: Sv rows of nn*C values at out[s0 + jj, r0*C ...]
      const int rowlen = nn * C;
      const int total = Sv * rowlen;
      const int q64 = 64 / rowlen, r64 = 64 - q64 * rowlen;
      int jj = lane / rowlen, w = lane - jj * rowlen;
      OutT* dst0 = out + s0 * a.MC + (int64_t)r0 * C;
      for (int e = lane; e < total; e += 64) {
        store_out(dst0 + jj * a.MC + w, stage[e]);
        jj += q64;
        w += r64;
        if (w >= rowlen) { w -= rowlen; ++jj; }
      }
      wave_lds_sync();
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

__global__ void action_bwd_reduce_kernel(const float* ws_ang, const float* ws_F, float* gang,
                                         float* gF, int64_t n, int64_t MC, int nseg, int gridX,
                                         int sharedF) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n * 3) {
    float sum = 0.f;
    for (int sg = 0; sg < nseg; ++sg) sum += ws_ang[(int64_t)sg * n * 3 + t];
    gang[t] = sum;
  }
  if (sharedF && t < MC) {
    float sum = 0.f;
    for (int b = 0; b < gridX; ++b) sum += ws_F[(int64_t)b * MC + t];
    gF[t] = sum;
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
// (prologue cost P charged per range).  Returns seg_lo[0..nseg].
inline int plan_segments(int L, int nseg, double P, bool bwd, int* seg_lo) {
  const int D = L + 1;
  nseg = std::max(1, std::min(nseg, std::min(D, kMaxSeg)));
  std::vector<double> pre(D + 1, 0.0);
  for (int l = 0; l < D; ++l) pre[l + 1] = pre[l] + degree_cost(l, bwd);
  // dp[k][i]: best max cost splitting first i degrees into k ranges
  const double INF = 1e30;
  std::vector<std::vector<double>> dp(nseg + 1, std::vector<double>(D + 1, INF));
  std::vector<std::vector<int>> arg(nseg + 1, std::vector<int>(D + 1, 0));
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

// Segments so that the grid has ~2 waves per SIMD (1024 SIMDs on MI355X), but never
// more ranges than pay for their duplicated prologue.
inline int choose_nseg(int64_t n, int Sw, int L, double P, bool bwd) {
  const int64_t waves = (n + Sw - 1) / Sw;
  const int64_t target = 2048;
  int nseg = (int)std::min<int64_t>(kMaxSeg, std::max<int64_t>(1, (target + waves - 1) / waves));
  // cap: a range should carry at least ~2x its prologue
  double total = 0.0;
  for (int l = 0; l <= L; ++l) total += degree_cost(l, bwd);
  const int cap = std::max(1, (int)(total / (2.0 * P)));
  return std::min(nseg, std::min(cap, L + 1));
}

constexpr double kPrologueFwd = 220.0;
constexpr double kPrologueFused = 420.0;

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
    const size_t lds = sizeof(float) * kWavesPerBlock * 64 * (2 * LT + 1);
    dim3 grid(p.gx, p.gy), block(kThreads);
    if (p.fused) {
      if (p.dtype == LV_DTYPE_BF16)
        hipLaunchKernelGGL((action_fwd_kernel<LT, true, __hip_bfloat16>), grid, block, lds, p.stream, p.a);
      else
        hipLaunchKernelGGL((action_fwd_kernel<LT, true, float>), grid, block, lds, p.stream, p.a);
    } else {
      if (p.dtype == LV_DTYPE_BF16)
        hipLaunchKernelGGL((action_fwd_kernel<LT, false, __hip_bfloat16>), grid, block, lds, p.stream, p.a);
      else
        hipLaunchKernelGGL((action_fwd_kernel<LT, false, float>), grid, block, lds, p.stream, p.a);
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

int check_common(int64_t n, int L, int C, int dtype) {
  LV_CHECK_ARG(n >= 0, "n must be >= 0 (got %lld)", (long long)n);
  LV_CHECK_ARG(L >= 0 && L <= LV_MAX_DEGREE, "l_max must be in [0, %d] (got %d)", LV_MAX_DEGREE, L);
  LV_CHECK_ARG(C >= 1 && C <= LV_MAX_CHANNELS, "C must be in [1, %d] (got %d)", LV_MAX_CHANNELS, C);
  LV_CHECK_ARG(dtype == LV_DTYPE_F32 || dtype == LV_DTYPE_BF16, "bad out dtype %d", dtype);
  return LV_OK;
}

int action_fwd_common(bool fused, const float* ang, const float* mu, const float* v, const float* F,
                      int64_t Fstride, void* out, int out_dtype, float* ang_out, int64_t n, int L,
                      int C, int transpose, hipStream_t stream) {
  clear_error();
  if (int e = check_common(n, L, C, out_dtype)) return e;
  const int64_t MC = (int64_t)(L + 1) * (L + 1) * C;
  LV_CHECK_ARG(Fstride == 0 || Fstride == MC, "F batch stride must be 0 or M*C=%lld", (long long)MC);
  if (n == 0) return LV_OK;
  LV_CHECK_ARG(F && out, "null F/out");
  LV_CHECK_ARG(fused ? (v != nullptr) : (ang != nullptr), "null input");
  FwdLaunch p{};
  p.a.ang = ang;
  p.a.mu = mu;
  p.a.v = v;
  p.a.F = F;
  p.a.Fstride = Fstride;
  p.a.out = out;
  p.a.ang_out = ang_out;
  p.a.n = n;
  p.a.MC = MC;
  p.a.C = C;
  p.a.Sw = 64 / C;
  p.a.transpose = transpose ? 1 : 0;
  const double P = fused ? kPrologueFused : kPrologueFwd;
  const int nseg = choose_nseg(n, p.a.Sw, L, P, false);
  plan_segments(L, nseg, P, false, p.a.seg_lo);
  const int64_t gx = (n + (int64_t)p.a.Sw * kWavesPerBlock - 1) / ((int64_t)p.a.Sw * kWavesPerBlock);
  LV_CHECK_ARG(gx <= 0x7fffffff, "batch too large");
  p.gx = (int)gx;
  p.gy = nseg;
  p.fused = fused;
  p.dtype = out_dtype;
  p.stream = stream;
  return dispatch_L<FwdLauncher>(L, p);
}

struct BwdPlan {
  int nseg, gx, groups, Sw;
  int seg_lo[kMaxSeg + 1];
  size_t lds, ws_ang, ws_F;
};

BwdPlan plan_bwd(int64_t n, int L, int C, bool sharedF) {
  BwdPlan b{};
  b.Sw = 64 / C;
  b.nseg = choose_nseg(n, b.Sw, L, kPrologueFwd, true);
  plan_segments(L, b.nseg, kPrologueFwd, true, b.seg_lo);
  b.groups = (int)((n + (int64_t)b.Sw * kWavesPerBlock - 1) / ((int64_t)b.Sw * kWavesPerBlock));
  // bound the slab count: each block walks several sample groups
  b.gx = std::max(1, std::min(b.groups, sharedF ? 512 : 1 << 30));
  int max_seg_rows = 0;
  for (int k = 0; k < b.nseg; ++k)
    max_seg_rows = std::max(max_seg_rows, b.seg_lo[k + 1] * b.seg_lo[k + 1] - b.seg_lo[k] * b.seg_lo[k]);
  const size_t wave_floats = 64 * (2 * L + 1) + 64 * 3 + (sharedF ? (size_t)max_seg_rows * C : 0);
  b.lds = sizeof(float) * kWavesPerBlock * wave_floats;
  b.ws_ang = sizeof(float) * (size_t)b.nseg * (size_t)n * 3;
  const size_t MC = (size_t)(L + 1) * (L + 1) * C;
  b.ws_F = sharedF ? sizeof(float) * (size_t)b.gx * MC : 0;
  return b;
}

}  // namespace
}  // namespace lv

using namespace lv;

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
  const BwdPlan b = plan_bwd(n, L, C, shared_F != 0);
  return b.ws_ang + b.ws_F;
}

int lv_group_action_bwd(const float* ang, const float* F, int64_t F_batch_stride,
                        const float* gout, float* gang, float* gF, int64_t n, int L, int C,
                        int transpose, void* workspace, size_t ws_bytes, void* stream) {
  clear_error();
  if (int e = check_common(n, L, C, LV_DTYPE_F32)) return e;
  const int64_t MC = (int64_t)(L + 1) * (L + 1) * C;
  LV_CHECK_ARG(F_batch_stride == 0 || F_batch_stride == MC, "F batch stride must be 0 or M*C");
  const bool sharedF = F_batch_stride == 0;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    if (sharedF && gF) hipMemsetAsync(gF, 0, sizeof(float) * MC, st);
    return LV_OK;
  }
  LV_CHECK_ARG(ang && F && gout && gang && gF, "null pointer argument");
  const BwdPlan b = plan_bwd(n, L, C, sharedF);
  if (ws_bytes < b.ws_ang + b.ws_F || !workspace) {
    set_error("workspace too small: need %zu bytes", b.ws_ang + b.ws_F);
    return LV_ERR_WORKSPACE;
  }
  BwdLaunch p{};
  p.a.ang = ang;
  p.a.F = F;
  p.a.Fstride = F_batch_stride;
  p.a.gout = gout;
  p.a.gang = gang;
  p.a.gF = gF;
  p.a.ws_ang = (float*)workspace;
  p.a.ws_F = (float*)((char*)workspace + b.ws_ang);
  p.a.n = n;
  p.a.MC = MC;
  p.a.C = C;
  p.a.Sw = b.Sw;
  p.a.transpose = transpose ? 1 : 0;
  p.a.nseg = b.nseg;
  p.a.groups = b.groups;
  for (int k = 0; k <= kMaxSeg; ++k) p.a.seg_lo[k] = b.seg_lo[k];
  p.gx = b.gx;
  p.gy = b.nseg;
  p.lds = b.lds;
  p.stream = st;
  LV_CHECK_ARG(b.lds <= 160 * 1024, "LDS plan too large (%zu B)", b.lds);
  if (int e = dispatch_L<BwdLauncher>(L, p)) return e;
  const int64_t work = std::max<int64_t>(n * 3, sharedF ? MC : 0);
  hipLaunchKernelGGL(action_bwd_reduce_kernel, dim3(ceil_div(work, 256)), dim3(256), 0, st,
                     p.a.ws_ang, p.a.ws_F, gang, gF, n, MC, b.nseg, b.gx, sharedF ? 1 : 0);
  LV_RETURN_LAUNCH("action_bwd_reduce_kernel");
}

int lv_wigner_d_fwd(const float* ang, float* D, int64_t n, int L, void* stream) {
  clear_error();
  LV_CHECK_ARG(n >= 0, "n must be >= 0");
  LV_CHECK_ARG(L >= 0 && L <= LV_MAX_DEGREE, "l_max out of range");
  if (n == 0) return LV_OK;
  LV_CHECK_ARG(ang && D, "null pointer");
  WigLaunch p{ang, D, n, (hipStream_t)stream};
  return dispatch_L<WigLauncher>(L, p);
}

}  // extern "C"

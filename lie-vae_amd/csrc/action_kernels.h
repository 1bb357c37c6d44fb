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

// Diagnostic timestamps (tools/kbench.hip builds with -DLV_STAMPS; never in the library).
#ifndef LV_STORE_MODE
#define LV_STORE_MODE 0
#endif
#ifndef LV_PROLOGUE_MODE
#define LV_PROLOGUE_MODE 0
#endif
#ifdef LV_STAMPS
__device__ unsigned long long* lv_stamp_buf;
#define LV_STAMP(slot)                                                                  \
  do {                                                                                  \
    if ((threadIdx.x & 63) == 0) {                                                      \
      const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                   \
      const unsigned long long w_ = ((unsigned long long)blockIdx.y * gridDim.x + blockIdx.x) * \
                                    (blockDim.x >> 6) + (threadIdx.x >> 6);             \
      lv_stamp_buf[w_ * 8 + (slot)] = t_;                                               \
    }                                                                                   \
  } while (0)
#else
#define LV_STAMP(slot) do {} while (0)
#endif

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

// ---- fused-prologue maths (per lane, registers).

// ZYZ (cos, sin) straight from the quaternion: the function quaternions_to_eazyz
// (lie_tools.py:160-175) followed by cos/sin.  atan2(y, x) -> (x, y)/|(x, y)| with the
// atan2(+-0, +-0) edge mirrored; acos(clamp(w)) -> (w, sqrt((1-w)(1+w))).
__device__ __forceinline__ void quat_to_zyz_trig(const float q[4], float c1[3], float s1[3]) {
  const float a1 = q[1] * q[2] - q[0] * q[3];
  const float b1 = q[0] * q[2] + q[1] * q[3];
  const float cb = ((q[3] * q[3] - q[0] * q[0]) - q[1] * q[1]) + q[2] * q[2];
  const float a3 = q[0] * q[3] + q[1] * q[2];
  const float b3 = q[1] * q[3] - q[0] * q[2];
  auto dir = [](float y, float x, float& c, float& s) {
    const float r2 = x * x + y * y;
    if (r2 == 0.f) {  // atan2(+-0, +-0) in {0, +-pi}
      c = signbit(x) ? -1.f : 1.f;
      s = 0.f;
    } else {
      const float r = rsqrtf(r2);
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

// The same (cos, sin) for z = exp(v) straight from the axis-angle form, at better than
// fp32-reference accuracy.  The reference's q = group_matrix_to_quaternions(rodrigues(v))
// is, in exact arithmetic, the unit quaternion q* = (-u sin(t/2), cos(t/2)) of R(v) (its
// matrix is the transpose of the active one) with the trace method's epsilon applied to
// the largest component k: q_k -> d = sqrt(q_k^2 + 2.5e-7), q_j -> sign(q_k) q_j |q_k| / d
// (lie_tools.py:126-156).  cos(beta) = 1 - (1 - cb) is formed in "one-minus" form so that
// sin(beta) = sqrt((1-cb)(1+cb)) keeps full relative accuracy near beta = 0 / pi, where the
// reference's fp32 acos(cb) loses it (the clamp to +-(1 - 1e-6) is mirrored exactly).
__device__ __forceinline__ void exp_to_zyz_trig(const float v[3], float c1[3], float s1[3],
                                                float qr[4]) {
  const float vv = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  const float inv = rsqrtf(vv);  // NaN downstream at v = 0, as the reference
  const float th = vv * inv;
  float sh, ch;
  sincosf(0.5f * th, &sh, &ch);
  const float m = -sh * inv;
  const float qt[4] = {v[0] * m, v[1] * m, v[2] * m, ch};
  int k = 0;
  float best = fabsf(qt[0]);
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (fabsf(qt[i]) > best) { best = fabsf(qt[i]); k = i; }
  const float qk = k == 0 ? qt[0] : (k == 1 ? qt[1] : (k == 2 ? qt[2] : qt[3]));
  constexpr float eps = 2.5e-7f;
  const float qk2 = qk * qk;
  const float d = sqrtf(qk2 + eps);
  const float sc = copysignf(best / d, qk);
#pragma unroll
  for (int i = 0; i < 4; ++i) qr[i] = (i == k) ? d : qt[i] * sc;
  const float oms = eps * (1.f - 2.f * qk2 - eps) / (qk2 + eps);  // 1 - |q_ref|^2
  float omc = fmaf(2.f, qr[0] * qr[0] + qr[1] * qr[1], oms);        // 1 - cos(beta)
  float opc = fmaf(2.f, qr[2] * qr[2] + qr[3] * qr[3], oms);        // 1 + cos(beta)
  constexpr float kDelta = 1.f - kEazyzHi;                          // exact in fp32
  if (omc < kDelta) { omc = kDelta; opc = 2.f - kDelta; }
  else if (opc < kDelta) { opc = kDelta; omc = 2.f - kDelta; }
  c1[1] = omc <= opc ? 1.f - omc : opc - 1.f;
  s1[1] = sqrtf(omc * opc);
  auto dir = [](float y, float x, float& c, float& s) {
    const float r2 = x * x + y * y;
    if (r2 == 0.f) {  // atan2(+-0, +-0) in {0, +-pi}
      c = signbit(x) ? -1.f : 1.f;
      s = 0.f;
    } else {
      const float r = rsqrtf(r2);
      c = x * r;
      s = y * r;
    }
  };
  dir(qr[1] * qr[2] - qr[0] * qr[3], qr[0] * qr[2] + qr[1] * qr[3], c1[0], s1[0]);
  dir(qr[0] * qr[3] + qr[1] * qr[2], qr[1] * qr[3] - qr[0] * qr[2], c1[2], s1[2]);
}

// General mean (z = mu @ exp(v)): the reference's op sequence (rodrigues, matmul, trace
// method with its 1e-6 epsilon and first-argmax case, quaternion -> ZYZ) evaluated in
// fp64 and rounded once to fp32 (cos, sin).  Near beta = 0 / pi the fp32 reference is
// ill-conditioned (a 1-ulp change of z moves D by ~1e-5); fp64 keeps this path within
// the reference's own fp64 evaluation.  Off the config-2 metric path (no mu there).
__device__ __forceinline__ void mu_exp_to_zyz_trig(const float mu[9], const float vf[3],
                                                   float c1[3], float s1[3], float qf[4]) {
  const double v[3] = {vf[0], vf[1], vf[2]};
  const double th = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  const double u[3] = {v[0] / th, v[1] / th, v[2] / th};
  double sn, cs;
  sincos(th, &sn, &cs);
  const double omc = 1.0 - cs;
  const double K[9] = {0, -u[2], u[1], u[2], 0, -u[0], -u[1], u[0], 0};
  const double K2[9] = {-u[2] * u[2] - u[1] * u[1], u[1] * u[0], u[2] * u[0],
                        u[0] * u[1], -u[2] * u[2] - u[0] * u[0], u[2] * u[1],
                        u[0] * u[2], u[1] * u[2], -u[1] * u[1] - u[0] * u[0]};
  double R[9], z[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = ((i % 4 == 0) ? 1.0 : 0.0) + sn * K[i] + omc * K2[i];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      z[i * 3 + j] = (double)mu[i * 3] * R[j] + (double)mu[i * 3 + 1] * R[3 + j] +
                     (double)mu[i * 3 + 2] * R[6 + j];
  const double a = z[0], b = z[4], c = z[8];
  const double pre[4] = {1 + a - b - c, 1 - a + b - c, 1 - a - b + c, 1 + a + b + c};
  int k = 0;
  double best = 0.5 * sqrt(1e-6 + fabs(pre[0]));
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    const double d = 0.5 * sqrt(1e-6 + fabs(pre[i]));
    if (d > best) { best = d; k = i; }
  }
  const double s01 = z[1] + z[3], s02 = z[2] + z[6], s12 = z[5] + z[7];
  const double d12 = z[5] - z[7], d20 = z[6] - z[2], d01 = z[1] - z[3];
  const double r4 = 1.0 / (4.0 * best);
  double q[4];
  switch (k) {
    case 0: q[0] = best; q[1] = s01 * r4; q[2] = s02 * r4; q[3] = d12 * r4; break;
    case 1: q[0] = s01 * r4; q[1] = best; q[2] = s12 * r4; q[3] = d20 * r4; break;
    case 2: q[0] = s02 * r4; q[1] = s12 * r4; q[2] = best; q[3] = d01 * r4; break;
    default: q[0] = d12 * r4; q[1] = d20 * r4; q[2] = d01 * r4; q[3] = best; break;
  }
  double cb = ((q[3] * q[3] - q[0] * q[0]) - q[1] * q[1]) + q[2] * q[2];
  cb = fmin(fmax(cb, (double)kEazyzLo), (double)kEazyzHi);
  c1[1] = (float)cb;
  s1[1] = (float)sqrt((1.0 - cb) * (1.0 + cb));
  auto dir = [](double y, double x, float& cf, float& sf) {
    const double r2 = x * x + y * y;
    if (r2 == 0.0) {
      cf = signbit(x) ? -1.f : 1.f;
      sf = 0.f;
    } else {
      const double r = 1.0 / sqrt(r2);
      cf = (float)(x * r);
      sf = (float)(y * r);
    }
  };
  dir(q[1] * q[2] - q[0] * q[3], q[0] * q[2] + q[1] * q[3], c1[0], s1[0]);
  dir(q[0] * q[3] + q[1] * q[2], q[1] * q[3] - q[0] * q[2], c1[2], s1[2]);
#pragma unroll
  for (int i = 0; i < 4; ++i) qf[i] = (float)q[i];
}

// Per-lane inputs, loaded before the block barrier so that their latency overlaps the
// spectrum staging.
struct LaneIn {
  float v[3];
  float mu[9];
};

template <bool FUSED>
__device__ __forceinline__ void lane_load(const ActionArgs& a, int64_t s, LaneIn& in) {
  if constexpr (FUSED) {
#pragma unroll
    for (int i = 0; i < 3; ++i) in.v[i] = a.v[s * 3 + i];
    if (a.mu) {
#pragma unroll
      for (int i = 0; i < 9; ++i) in.mu[i] = a.mu[s * 9 + i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i) in.v[i] = a.ang[s * 3 + i];
  }
}

// (cos, sin) of the three chain angles.  For transpose (D^T = X(-c) J X(-b) J X(-a)) the
// slots are swapped and the sines negated.
template <bool FUSED>
__device__ __forceinline__ void lane_angles(const ActionArgs& a, const LaneIn& in, int64_t s,
                                            bool active, int c, bool write_ang, float c1[3],
                                            float s1[3]) {
  float cc[3], ss[3];
#if LV_PROLOGUE_MODE == 1  // diagnostic: trivial angles (loads kept)
  if (true) {
#pragma unroll
    for (int i = 0; i < 3; ++i) { cc[i] = in.v[i]; ss[i] = in.v[(i + 1) % 3]; }
  } else
#endif
  if constexpr (FUSED) {
    float q[4];
    if (a.mu) {
      mu_exp_to_zyz_trig(in.mu, in.v, cc, ss, q);
    } else {
      exp_to_zyz_trig(in.v, cc, ss, q);
    }
    if (write_ang && active && c == 0) {
      float ang[3];
      quat_to_eazyz_fwd(q, ang);
      a.ang_out[s * 3 + 0] = ang[0];
      a.ang_out[s * 3 + 1] = ang[1];
      a.ang_out[s * 3 + 2] = ang[2];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i) sincosf(in.v[i], &ss[i], &cc[i]);
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
  float c1[3], s1[3];
  TrigTab<LT> t;
  if (Sv > 0) {
    lane_angles<FUSED>(a, in, s, active, c, FUSED && a.ang_out && blockIdx.y == 0, c1, s1);
    trig_fill<LT>(t, c1, s1, hi - 1);
  }
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
      xrot<l, 2>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 1>(t, x, y);
      jmul<l>(y, x);
      xrot<l, 0>(t, x, y);
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
#endif
    }
  });
  LV_STAMP(3);
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
        fmax = max(fmax, (fseg_rows(p.a.seg_lo[k], p.a.seg_lo[k + 1]) * p.a.C + 3) & ~3);
    const size_t lds = sizeof(float) * ((size_t)fmax + (LV_STAGED_DEFAULT ? (size_t)kWavesPerBlock * stage_floats(LT, p.a.C) : 0));
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
#define LV_EXTERN_BWD(R) extern template struct BwdLauncher<R>;

}  // namespace lv

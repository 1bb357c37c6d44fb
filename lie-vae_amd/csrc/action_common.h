#pragma once
// Shared pieces of the group-action kernels for gfx950 (MI355X): launch arguments, the
// fused prologue maths (z = mu·exp(v) -> ZYZ (cos, sin)) and per-lane input staging.
// Forward kernels: action_fwd.h; backward: action_bwd.h; host planning: action.hip.
#include "action_chain.h"
#include "so3_device.h"

namespace lv {

constexpr int kWavesPerBlock = 4;
constexpr int kThreads = 64 * kWavesPerBlock;
constexpr int kMaxSeg = 16;
constexpr int kTrigLdsMinL = 13;  // action_fwd_kernel keeps its trig table in LDS from here
constexpr int kTileFGlobalMinL = 13;  // the tile kernel reads the spectrum from global from here

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
  int fpitch;           // tile kernel: floats per wave-private spectrum slice in LDS
  int write_through;    // tile kernel: 1 = sc1 (write-through) stores, 0 = nt stores, 2 = plain (A/B)
  int prio;             // tile kernel wave priority: 2 = prologue at s_setprio 3, chain at 0
                        // (default); A/B: 0 off, 1 flush at 3, 3 = 2 + flush at 2
  int task_spread;      // tile kernel: prologue task t on lane t / nw of wave t % nw (1) instead
                        // of thread t (0: all tasks in wave 0)
  int ang_order;        // tile kernel, mu-free fused: 0 = angles written before the spectrum
                        // loads are issued (default), 1 = after them (A/B)
  unsigned long long* stamps;  // phase timestamps (A/B timeline tool; null in the product)
  int seg_lo[kMaxSeg + 1];      // non-tile kernel / run-time-C tile: contiguous degree ranges
  unsigned seg_mask[kMaxSeg];   // tile kernel: degree set of wave k (bit l = degree l)
};

// Phase timestamps for tools/timeline.py (the A/B build's LV_STAMPS=1; the product passes
// null): lane 0 of each wave writes the 100 MHz real-time counter at phase k, slot
// [block][wave < 16][k < 8].
constexpr int64_t kStampBlocks = 16384;
__device__ __forceinline__ void phase_stamp(unsigned long long* st, int wave, int k) {
  if (st && (threadIdx.x & 63) == 0 && blockIdx.x < kStampBlocks)
    st[((int64_t)blockIdx.x * 16 + wave) * 8 + k] = __builtin_amdgcn_s_memrealtime();
}
// ... and at the end of each degree l of the chain, slot [block < 2048][wave][l < 24] after
// the phase slots and the reduce kernel's 2 x 4096 (per-degree cost calibration).
constexpr int64_t kStampDegBlocks = 2048;
constexpr int64_t kStampDegBase = kStampBlocks * 16 * 8 + 2 * 4096;
__device__ __forceinline__ void degree_stamp(unsigned long long* st, int wave, int l) {
  if (st && (threadIdx.x & 63) == 0 && blockIdx.x < kStampDegBlocks)
    st[kStampDegBase + ((int64_t)blockIdx.x * 16 + wave) * 24 + l] = __builtin_amdgcn_s_memrealtime();
}


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
// sin and cos of x as straight-line code: Cody-Waite reduction by pi/2 (three-part fp32
// constant, FMA) into [-pi/4, pi/4], minimax polynomials (the Cephes sinf / cosf
// coefficients) and the quadrant by k & 3; <= 1.6 ulp for |x| <= 1e5 (checked against fp64
// on 430k points).  Larger |x| (a rotation vector beyond 2e5 rad) and NaN take sincosf on a
// cold branch.  The library's sincosf inlines its large-argument reduction in the middle of
// the code, and in the tile kernels' prologue -- one serial chain per (sample, slot) that
// every wave of the block waits for -- the jumps around it land on cold instruction-cache
// lines.
__device__ __forceinline__ void lv_sincos(float x, float& s, float& c) {
  const float k = rintf(x * 0.63661977236758134f);
  float r = fmaf(k, -1.5707963705062866f, x);
  r = fmaf(k, 4.371138828673793e-08f, r);
  r = fmaf(k, 1.7151245100058819e-15f, r);
  const float r2 = r * r;
  const float ps = fmaf(r2, fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f), -1.6666654611e-1f) * r2;
  const float sn = fmaf(r, ps, r);
  const float pc = fmaf(r2, fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f), 4.166664568298827e-2f);
  const float cs = fmaf(r2 * r2, pc, fmaf(r2, -0.5f, 1.f));
  const int q = (int)k & 3;
  s = (q & 1) ? cs : sn;
  c = (q & 1) ? sn : cs;
  if (q == 1 || q == 2) c = -c;
  if (q >= 2) s = -s;
  if (__builtin_expect(!(fabsf(x) <= 1.0e5f), 0)) sincosf(x, &s, &c);
}

// The quaternion part of exp_to_zyz_trig: q_ref of z = exp(v) (see exp_to_zyz_trig), and the
// quantities the angle formulas reuse.
struct ExpQuat {
  float qr[4];
  float qk2, rd;  // the largest component squared, rsqrt(qk2 + eps)
};
__device__ __forceinline__ ExpQuat exp_quat(const float v[3]) {
  ExpQuat e;
  const float vv = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  const float inv = rsqrtf(vv);  // NaN downstream at v = 0, as the reference
  const float th = vv * inv;
  float sh, ch;
  lv_sincos(0.5f * th, sh, ch);
  const float m = -sh * inv;
  const float qt[4] = {v[0] * m, v[1] * m, v[2] * m, ch};
  int k = 0;
  float best = fabsf(qt[0]);
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (fabsf(qt[i]) > best) { best = fabsf(qt[i]); k = i; }
  const float qk = k == 0 ? qt[0] : (k == 1 ? qt[1] : (k == 2 ? qt[2] : qt[3]));
  constexpr float eps = 2.5e-7f;
  e.qk2 = qk * qk;
  // d = sqrt(qk^2 + eps), best / d as reciprocal-square-root products (<= 2 ulp)
  e.rd = rsqrtf(e.qk2 + eps);
  const float d = (e.qk2 + eps) * e.rd;
  const float sc = copysignf(best * e.rd, qk);
#pragma unroll
  for (int i = 0; i < 4; ++i) e.qr[i] = (i == k) ? d : qt[i] * sc;
  return e;
}
// (cos, sin) of beta: cos from the "one-minus" forms, the clamp to +-(1 - 1e-6) mirrored
__device__ __forceinline__ void exp_beta(const ExpQuat& e, float& c, float& s) {
  constexpr float eps = 2.5e-7f;
  const float* qr = e.qr;
  const float oms = eps * (1.f - 2.f * e.qk2 - eps) * (e.rd * e.rd);  // 1 - |q_ref|^2
  float omc = fmaf(2.f, qr[0] * qr[0] + qr[1] * qr[1], oms);          // 1 - cos(beta)
  float opc = fmaf(2.f, qr[2] * qr[2] + qr[3] * qr[3], oms);          // 1 + cos(beta)
  constexpr float kDelta = 1.f - kEazyzHi;
  const bool clo = omc < kDelta, chi = !clo && opc < kDelta;
  omc = clo ? kDelta : (chi ? 2.f - kDelta : omc);
  opc = clo ? 2.f - kDelta : (chi ? kDelta : opc);
  c = omc <= opc ? 1.f - omc : opc - 1.f;
  s = __builtin_amdgcn_sqrtf(omc * opc);  // v_sqrt_f32 (1 ulp)
}
// (cos, sin) of alpha (ai = 0) or gamma (ai = 2): the direction of (x, y), atan2(+-0, +-0)
// in {0, +-pi} mirrored
__device__ __forceinline__ void exp_dir(const ExpQuat& e, int ai, float& c, float& s) {
  const float* qr = e.qr;
  const float y = ai == 0 ? qr[1] * qr[2] - qr[0] * qr[3] : qr[0] * qr[3] + qr[1] * qr[2];
  const float x = ai == 0 ? qr[0] * qr[2] + qr[1] * qr[3] : qr[1] * qr[3] - qr[0] * qr[2];
  const float r2 = x * x + y * y;
  const float rr = rsqrtf(r2);
  c = r2 == 0.f ? (signbit(x) ? -1.f : 1.f) : x * rr;
  s = r2 == 0.f ? 0.f : y * rr;
}

// (cos, sin) of the three ZYZ angles of z = exp(v) straight from the axis-angle form, at
// better than fp32-reference accuracy.  The reference's q = group_matrix_to_quaternions(
// rodrigues(v)) is, in exact arithmetic, the unit quaternion q* = (-u sin(t/2), cos(t/2))
// of R(v) (its matrix is the transpose of the active one) with the trace method's epsilon
// applied to the largest component k: q_k -> d = sqrt(q_k^2 + 2.5e-7), q_j -> sign(q_k)
// q_j |q_k| / d (lie_tools.py:126-156).  cos(beta) = 1 - (1 - cb) is formed in "one-minus"
// form so that sin(beta) = sqrt((1-cb)(1+cb)) keeps full relative accuracy near beta = 0 /
// pi, where the reference's fp32 acos(cb) loses it (the clamp to +-(1 - 1e-6) is mirrored
// exactly).  Every fused kernel evaluates these same expressions (bitwise equal across the
// tile and non-tile kernels).
__device__ __forceinline__ void exp_to_zyz_trig(const float v[3], float c1[3], float s1[3],
                                                float qr[4]) {
  const ExpQuat e = exp_quat(v);
  exp_dir(e, 0, c1[0], s1[0]);
  exp_beta(e, c1[1], s1[1]);
  exp_dir(e, 2, c1[2], s1[2]);
#pragma unroll
  for (int i = 0; i < 4; ++i) qr[i] = e.qr[i];
}

// One slot (angle index ai: 0 = alpha, 1 = beta, 2 = gamma) of exp_to_zyz_trig, straight-
// line (selects, no divergent branches): each prologue thread of the tile kernel fills one
// slot's multiples, so it computes that slot's (cos, sin) only (and the quaternion, for
// ang_out).  Bitwise the values exp_to_zyz_trig returns for that slot.
__device__ __forceinline__ void exp_to_zyz_slot(const float v[3], int ai, float& c, float& s, float qr[4]) {
  const ExpQuat e = exp_quat(v);
  float cb, sb, cd, sd;
  exp_beta(e, cb, sb);
  exp_dir(e, ai, cd, sd);
  c = ai == 1 ? cb : cd;
  s = ai == 1 ? sb : sd;
#pragma unroll
  for (int i = 0; i < 4; ++i) qr[i] = e.qr[i];
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

// MAYMU = false: the caller guarantees a.mu == nullptr (compiled without the mu path).
template <bool FUSED, bool MAYMU = true>
__device__ __forceinline__ void lane_load(const ActionArgs& a, int64_t s, LaneIn& in) {
  if constexpr (FUSED) {
#pragma unroll
    for (int i = 0; i < 3; ++i) in.v[i] = a.v[s * 3 + i];
    if (MAYMU && a.mu) {
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
template <bool FUSED, bool MAYMU = true>
__device__ __forceinline__ void lane_angles(const ActionArgs& a, const LaneIn& in, int64_t s,
                                            bool active, int c, bool write_ang, float c1[3],
                                            float s1[3]) {
  float cc[3], ss[3];
  if constexpr (FUSED) {
    float q[4];
    if (MAYMU && a.mu) {
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


}  // namespace lv

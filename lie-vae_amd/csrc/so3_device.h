// Per-sample SO(3) math, forward and hand-derived backward, in registers.
//
// Every function restates one reference op (file:line under the reference root) and
// keeps its evaluation order (the library is built with -ffp-contract=off, so nothing
// here is silently fused into an FMA).  Backward functions return the gradient autograd
// would produce for the same composition of torch ops.  The maps are templates on the
// scalar type T: the reference's maps follow their input dtype (v.new_tensor,
// eye(dtype=v.dtype), lie_tools.py:28-38,61), so fp64 inputs get fp64 kernels; T = T
// is the hot path and compiles to exactly the former fp32 code.
#pragma once
#include <hip/hip_runtime.h>

namespace lv {

// Scalar-type helpers: overloads so that one template body gives the fp32 code
// (sincosf) for float and the fp64 code (sincos) for double.
template <typename T>
struct lv_nondeduced { using type = T; };
__device__ __forceinline__ void lv_sincos(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ __forceinline__ void lv_sincos(double x, double* s, double* c) { sincos(x, s, c); }

// ---------------------------------------------------------------- rodrigues
// lie_tools.py:17-43 (hat) and :56-64 (rodrigues).  K = hat(u), K2 = K@K.
template <typename T>
__device__ __forceinline__ void hat_sq(const T u[3], T K[9], T K2[9]) {
  K[0] = T(0.);   K[1] = -u[2]; K[2] = u[1];
  K[3] = u[2];  K[4] = T(0.);   K[5] = -u[0];
  K[6] = -u[1]; K[7] = u[0];  K[8] = T(0.);
  // (K@K)_ij summed k = 0..2 exactly as the matmul does (zero products drop out).
  K2[0] = -u[2] * u[2] - u[1] * u[1];
  K2[1] = u[1] * u[0];
  K2[2] = u[2] * u[0];
  K2[3] = u[0] * u[1];
  K2[4] = -u[2] * u[2] - u[0] * u[0];
  K2[5] = u[2] * u[1];
  K2[6] = u[0] * u[2];
  K2[7] = u[1] * u[2];
  K2[8] = -u[1] * u[1] - u[0] * u[0];
}

template <typename T>
__device__ __forceinline__ T norm3(const T v[3]) {
  return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
}

// The angle-dependent pieces rodrigues_fwd and rodrigues_bwd both start from, computed
// once when a caller needs both (exp_eazyz_vjp_sample): the same operations, so the same
// bits as computing them twice.
template <typename T>
struct RodPrep {
  T th, u[3], K[9], K2[9], s, c;
};
template <typename T>
__device__ __forceinline__ void rodrigues_prep(const T v[3], RodPrep<T>& p) {
  p.th = norm3(v);
  p.u[0] = v[0] / p.th;  // NaN at th == 0, like the reference
  p.u[1] = v[1] / p.th;
  p.u[2] = v[2] / p.th;
  hat_sq(p.u, p.K, p.K2);
  lv_sincos(p.th, &p.s, &p.c);
}
template <typename T>
__device__ __forceinline__ void rodrigues_fwd_p(const RodPrep<T>& p, T R[9]) {
  const T omc = T(1.) - p.c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const T eye = (i == 0 || i == 4 || i == 8) ? T(1.) : T(0.);
    R[i] = (eye + p.s * p.K[i]) + omc * p.K2[i];
  }
}
template <typename T>
__device__ __forceinline__ void rodrigues_fwd(const T v[3], T R[9]) {
  RodPrep<T> p;
  rodrigues_prep(v, p);
  rodrigues_fwd_p(p, R);
}

// d/du of <g, s K(u) + w (u u^T - |u|^2 I)>
template <typename T>
__device__ __forceinline__ void hat_sq_vjp(const T u[3], const T g[9], T s, T w,
                                           T gu[3]) {
  const T tr = g[0] + g[4] + g[8];
  T gsym_u[3];
#pragma unroll
  for (int m = 0; m < 3; ++m)
    gsym_u[m] = (g[m * 3 + 0] + g[0 * 3 + m]) * u[0] + (g[m * 3 + 1] + g[1 * 3 + m]) * u[1] +
                (g[m * 3 + 2] + g[2 * 3 + m]) * u[2];
  gu[0] = s * (g[7] - g[5]) + w * (gsym_u[0] - T(2.) * tr * u[0]);
  gu[1] = s * (g[2] - g[6]) + w * (gsym_u[1] - T(2.) * tr * u[1]);
  gu[2] = s * (g[3] - g[1]) + w * (gsym_u[2] - T(2.) * tr * u[2]);
}

// (theta, u = v/theta) -> v chain rule.
template <typename T>
__device__ __forceinline__ void polar_vjp(const T v[3], T th, const T gu[3], T gth,
                                          T gv[3]) {
  const T dot = gu[0] * v[0] + gu[1] * v[1] + gu[2] * v[2];
  const T inv = T(1.) / th;
  const T inv3 = inv * inv * inv;
#pragma unroll
  for (int i = 0; i < 3; ++i) gv[i] = gu[i] * inv - dot * v[i] * inv3 + gth * v[i] * inv;
}

template <typename T>
__device__ __forceinline__ void rodrigues_bwd_p(const T v[3], const RodPrep<T>& p, const T gR[9], T gv[3]) {
  T gth = T(0.);
#pragma unroll
  for (int i = 0; i < 9; ++i) gth += gR[i] * (p.c * p.K[i] + p.s * p.K2[i]);
  T gu[3];
  hat_sq_vjp(p.u, gR, p.s, T(1.) - p.c, gu);
  polar_vjp(v, p.th, gu, gth, gv);
}
template <typename T>
__device__ __forceinline__ void rodrigues_bwd(const T v[3], const T gR[9], T gv[3]) {
  RodPrep<T> p;
  rodrigues_prep(v, p);
  rodrigues_bwd_p(v, p, gR, gv);
}

// ------------------------------------------------------------------ 3x3 ops
template <typename T>
__device__ __forceinline__ void matmul3(const T A[9], const T B[9], T C[9]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[i * 3 + j] = (A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j]) +
                     A[i * 3 + 2] * B[2 * 3 + j];
}
// C = A^T B
template <typename T>
__device__ __forceinline__ void matmul3_tn(const T A[9], const T B[9], T C[9]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[i * 3 + j] = A[0 * 3 + i] * B[0 * 3 + j] + A[1 * 3 + i] * B[1 * 3 + j] +
                     A[2 * 3 + i] * B[2 * 3 + j];
}
// C = A B^T
template <typename T>
__device__ __forceinline__ void matmul3_nt(const T A[9], const T B[9], T C[9]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[i * 3 + j] = A[i * 3 + 0] * B[j * 3 + 0] + A[i * 3 + 1] * B[j * 3 + 1] +
                     A[i * 3 + 2] * B[j * 3 + 2];
}

// ----------------------------------------------- group_matrix_to_quaternions
// lie_tools.py:112-157: 4-case trace method, eps 1e-6, case = first argmax.
template <typename T>
struct QuatCase {
  T pre[4];
  T den[4];
  int k;
};

template <typename T>
__device__ __forceinline__ void mat_to_quat_fwd(const T r[9], T q[4],
                                                typename lv_nondeduced<QuatCase<T>>::type* qc) {
  const T a = r[0], b = r[4], c = r[8];
  T pre[4] = {((T(1.) + a) - b) - c, ((T(1.) - a) + b) - c, ((T(1.) - a) - b) + c,
                  ((T(1.) + a) + b) + c};
  T den[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) den[i] = T(0.5) * sqrt(T(1e-6) + fabs(pre[i]));
  int k = 0;
  T best = den[0];
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (den[i] > best) { best = den[i]; k = i; }
  const T s01 = r[1] + r[3], s02 = r[2] + r[6], s12 = r[5] + r[7];
  const T d12 = r[5] - r[7], d20 = r[6] - r[2], d01 = r[1] - r[3];
  const T d4 = T(4.) * best;
  switch (k) {
    case 0: q[0] = best;      q[1] = s01 / d4;  q[2] = s02 / d4;  q[3] = d12 / d4; break;
    case 1: q[0] = s01 / d4;  q[1] = best;      q[2] = s12 / d4;  q[3] = d20 / d4; break;
    case 2: q[0] = s02 / d4;  q[1] = s12 / d4;  q[2] = best;      q[3] = d01 / d4; break;
    default: q[0] = d12 / d4; q[1] = d20 / d4;  q[2] = d01 / d4;  q[3] = best; break;
  }
  if (qc) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { qc->pre[i] = pre[i]; qc->den[i] = den[i]; }
    qc->k = k;
  }
}

// The backward from the forward's own q and case (mat_to_quat_fwd(r, q, &qc) already run).
// Written without run-time indexing of small arrays (case tables, q[k], den[k]): those put
// the arrays in scratch memory, a dependent global round trip on the VJP's serial chain.
// Every gr entry receives exactly one term, 0 + g or 0 - g, so the selects below give the
// same bits as the per-case accumulation.
template <typename T>
__device__ __forceinline__ T sel4(int k, T a0, T a1, T a2, T a3) {
  return k == 0 ? a0 : (k == 1 ? a1 : (k == 2 ? a2 : a3));
}
template <typename T>
__device__ __forceinline__ void mat_to_quat_bwd_qc(const T q[4], const QuatCase<T>& qc, const T gq[4], T gr[9]) {
  const int k = qc.k;
  const T d = sel4(k, qc.den[0], qc.den[1], qc.den[2], qc.den[3]);
  const T inv4d = T(1.) / (T(4.) * d);
  // gradient into the denominator: q_k = d, q_j = N_j / (4 d)
  T gd = sel4(k, gq[0], gq[1], gq[2], gq[3]);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j != k) gd -= gq[j] * q[j] / d;
  // N_j partials.  Numerators per case: case0 (s01, s02, d12) at q1..q3; case1 (s01, s12,
  // d20) at q0, q2, q3; case2 (s02, s12, d01) at q0, q1, q3; case3 (d12, d20, d01) at q0..q2;
  // s01 = r01 + r10, s02 = r02 + r20, s12 = r12 + r21, d12 = r12 - r21, d20 = r20 - r02,
  // d01 = r01 - r10.
  T g[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) g[jj] = gq[jj] * inv4d;
  const T z = T(0.);
  gr[1] = z + sel4(k, g[1], g[0], g[3], g[2]);                      // s01 | d01
  gr[3] = k < 2 ? z + sel4(k, g[1], g[0], g[0], g[0]) : z - sel4(k, g[0], g[0], g[3], g[2]);
  gr[2] = (k == 0 || k == 2) ? z + sel4(k, g[2], g[2], g[0], g[0]) : z - sel4(k, g[3], g[3], g[3], g[1]);
  gr[6] = z + sel4(k, g[2], g[3], g[0], g[1]);                      // s02 | d20
  gr[5] = z + sel4(k, g[3], g[2], g[1], g[0]);                      // d12 | s12
  gr[7] = (k == 1 || k == 2) ? z + sel4(k, g[2], g[2], g[1], g[2]) : z - sel4(k, g[3], g[3], g[3], g[0]);
  // d = 0.5 sqrt(1e-6 + |pre_k|)
  const T p = sel4(k, qc.pre[0], qc.pre[1], qc.pre[2], qc.pre[3]);
  const T t = sqrt(T(1e-6) + fabs(p));
  const T sg = (p > T(0.)) ? T(1.) : ((p < T(0.)) ? -T(1.) : T(0.));
  const T gpre = gd * T(0.25) / t * sg;
  // coef[k][i] = +1 if k == 3 or k == i, else -1
  gr[0] = z + ((k == 3 || k == 0) ? gpre : -gpre);
  gr[4] = z + ((k == 3 || k == 1) ? gpre : -gpre);
  gr[8] = z + ((k == 3 || k == 2) ? gpre : -gpre);
}
template <typename T>
__device__ __forceinline__ void mat_to_quat_bwd(const T r[9], const T gq[4], T gr[9]) {
  T q[4];
  QuatCase<T> qc;
  mat_to_quat_fwd(r, q, &qc);
  mat_to_quat_bwd_qc(q, qc, gq, gr);
}

// ----------------------------------------------------- quaternions_to_eazyz
// lie_tools.py:160-175 (q scalar-last; beta clamped to [-1+1e-6, 1-1e-6]).
constexpr float kEazyzLo = (float)(-1.0 + 1e-6);
constexpr float kEazyzHi = (float)(1.0 - 1e-6);
template <typename T>
__device__ __forceinline__ T eazyz_lo() { return (T)(-1.0 + 1e-6); }
template <typename T>
__device__ __forceinline__ T eazyz_hi() { return (T)(1.0 - 1e-6); }

template <typename T>
__device__ __forceinline__ void quat_to_eazyz_fwd(const T q[4], T ang[3]) {
  const T a1 = q[1] * q[2] - q[0] * q[3];
  const T b1 = q[0] * q[2] + q[1] * q[3];
  const T cb = ((q[3] * q[3] - q[0] * q[0]) - q[1] * q[1]) + q[2] * q[2];
  const T a3 = q[0] * q[3] + q[1] * q[2];
  const T b3 = q[1] * q[3] - q[0] * q[2];
  ang[0] = atan2(a1, b1);
  ang[1] = acos(fmin(fmax(cb, eazyz_lo<T>()), eazyz_hi<T>()));
  ang[2] = atan2(a3, b3);
}

template <typename T>
__device__ __forceinline__ void quat_to_eazyz_bwd(const T q[4], const T ga[3], T gq[4]) {
  const T a1 = q[1] * q[2] - q[0] * q[3];
  const T b1 = q[0] * q[2] + q[1] * q[3];
  const T cb = ((q[3] * q[3] - q[0] * q[0]) - q[1] * q[1]) + q[2] * q[2];
  const T a3 = q[0] * q[3] + q[1] * q[2];
  const T b3 = q[1] * q[3] - q[0] * q[2];
  const T r1 = a1 * a1 + b1 * b1, r3 = a3 * a3 + b3 * b3;
  const T ga1 = ga[0] * b1 / r1, gb1 = ga[0] * -a1 / r1;
  const T ga3 = ga[2] * b3 / r3, gb3 = ga[2] * -a3 / r3;
  const T x = fmin(fmax(cb, eazyz_lo<T>()), eazyz_hi<T>());
  const bool pass = (cb >= eazyz_lo<T>()) && (cb <= eazyz_hi<T>());
  const T gcb = pass ? (-ga[1] / sqrt(T(1.) - x * x)) : T(0.);
  gq[0] = -q[3] * ga1 + q[2] * gb1 + q[3] * ga3 - q[2] * gb3 - T(2.) * q[0] * gcb;
  gq[1] = q[2] * ga1 + q[3] * gb1 + q[2] * ga3 + q[3] * gb3 - T(2.) * q[1] * gcb;
  gq[2] = q[1] * ga1 + q[0] * gb1 + q[1] * ga3 - q[0] * gb3 + T(2.) * q[2] * gcb;
  gq[3] = -q[0] * ga1 + q[1] * gb1 + q[0] * ga3 + q[1] * gb3 + T(2.) * q[3] * gcb;
}

// ------------------------------------------------ quaternions_to_group_matrix
// lie_tools.py:183-192: normalise, then the reference's (transposed-active) matrix.
template <typename T>
__device__ __forceinline__ void quat_to_mat_fwd(const T q0[4], T R[9]) {
  const T nrm = sqrt(q0[0] * q0[0] + q0[1] * q0[1] + q0[2] * q0[2] + q0[3] * q0[3]);
  const T x = q0[0] / nrm, y = q0[1] / nrm, z = q0[2] / nrm, w = q0[3] / nrm;
  R[0] = ((x * x - y * y) - z * z) + w * w;
  R[1] = T(2.) * (x * y + z * w);
  R[2] = T(2.) * (x * z - y * w);
  R[3] = T(2.) * (x * y - z * w);
  R[4] = ((-x * x + y * y) - z * z) + w * w;
  R[5] = T(2.) * (y * z + x * w);
  R[6] = T(2.) * (x * z + y * w);
  R[7] = T(2.) * (y * z - x * w);
  R[8] = ((-x * x - y * y) + z * z) + w * w;
}

template <typename T>
__device__ __forceinline__ void quat_to_mat_bwd(const T q0[4], const T g[9], T gq[4]) {
  const T nrm = sqrt(q0[0] * q0[0] + q0[1] * q0[1] + q0[2] * q0[2] + q0[3] * q0[3]);
  const T x = q0[0] / nrm, y = q0[1] / nrm, z = q0[2] / nrm, w = q0[3] / nrm;
  T gn[4];
  gn[0] = T(2.) * (x * (g[0] - g[4] - g[8]) + y * (g[1] + g[3]) + z * (g[2] + g[6]) + w * (g[5] - g[7]));
  gn[1] = T(2.) * (-y * (g[0] - g[4] + g[8]) + x * (g[1] + g[3]) - w * (g[2] - g[6]) + z * (g[5] + g[7]));
  gn[2] = T(2.) * (-z * (g[0] + g[4] - g[8]) + w * (g[1] - g[3]) + x * (g[2] + g[6]) + y * (g[5] + g[7]));
  gn[3] = T(2.) * (w * (g[0] + g[4] + g[8]) + z * (g[1] - g[3]) - y * (g[2] - g[6]) + x * (g[5] - g[7]));
  const T dot = gn[0] * x + gn[1] * y + gn[2] * z + gn[3] * w;
  gq[0] = (gn[0] - dot * x) / nrm;
  gq[1] = (gn[1] - dot * y) / nrm;
  gq[2] = (gn[2] - dot * z) / nrm;
  gq[3] = (gn[3] - dot * w) / nrm;
}

// ------------------------------------------------- exp -> ZYZ vector-Jacobian product
// The autograd backward of z = mu @ rodrigues(v) (or z = rodrigues(v)) followed by
// group_matrix_to_eazyz (reparameterize.py:269-273, lie_tools.py:56-64,112-180): g = dL/d
// angles -> gm = dL/dmu (when m != nullptr), gv = dL/dv, in the same operation order as
// the modular kernels lv_so3_exp_fwd + lv_mat_to_eazyz_bwd + lv_so3_exp_bwd (or the
// so3_sample pair), hence bitwise equal to them.  Shared by lv_exp_eazyz_vjp and the
// fused backward tile kernel's tail.
// has_m selects the mu path (a flag, not a nullable pointer: selecting between a local
// array's address and nullptr forces the array into scratch memory).
template <typename T>
__device__ __forceinline__ void exp_eazyz_vjp_sample(const T a[3], bool has_m, const T m[9], const T g[3],
                                                     T gm[9], T gv[3]) {
  // the Rodrigues and quaternion intermediates are computed once and shared by the forward
  // and backward steps (the same operations the modular kernels repeat: same bits)
  T r[9], z[9], q[4], gq[4], gz[9];
  RodPrep<T> rp;
  rodrigues_prep(a, rp);
  rodrigues_fwd_p(rp, r);
  if (has_m) {
    matmul3(m, r, z);
  } else {
#pragma unroll
    for (int k = 0; k < 9; ++k) z[k] = r[k];
  }
  QuatCase<T> qc;
  mat_to_quat_fwd(z, q, &qc);
  quat_to_eazyz_bwd(q, g, gq);
  mat_to_quat_bwd_qc(q, qc, gq, gz);
  if (has_m) {
    T t[9], gr[9];
    matmul3_nt(gz, r, t);
#pragma unroll
    for (int k = 0; k < 9; ++k) gm[k] = T(0) + t[k];
    matmul3_tn(m, gz, gr);
    rodrigues_bwd_p(a, rp, gr, gv);
  } else {
    rodrigues_bwd_p(a, rp, gz, gv);
  }
}

// ------------------------------------------------------------- s2s1rodrigues
// lie_tools.py:67-78: R = I + sin K + (1 - cos) K@K, K = hat(axis), (cos, sin) given.
template <typename T>
__device__ __forceinline__ void s2s1_fwd(const T a[3], const T cs[2], T R[9]) {
  T K[9], K2[9];
  hat_sq(a, K, K2);
  const T omc = T(1.) - cs[0];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const T eye = (i == 0 || i == 4 || i == 8) ? T(1.) : T(0.);
    R[i] = (eye + cs[1] * K[i]) + omc * K2[i];
  }
}

template <typename T>
__device__ __forceinline__ void s2s1_bwd(const T a[3], const T cs[2], const T g[9],
                                         T ga[3], T gcs[2]) {
  T K[9], K2[9];
  hat_sq(a, K, K2);
  T gs = T(0.), gc = T(0.);
#pragma unroll
  for (int i = 0; i < 9; ++i) { gs += g[i] * K[i]; gc -= g[i] * K2[i]; }
  hat_sq_vjp(a, g, cs[1], T(1.) - cs[0], ga);
  gcs[0] = gc;
  gcs[1] = gs;
}

// ------------------------------------------------- s2s2_gram_schmidt (fp64)
// lie_tools.py:81-89 (cross product along the last axis).
__device__ __forceinline__ void cross3d(const double a[3], const double b[3], double c[3]) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

struct S2S2State {
  double n1, n1c, e1[3], dot, u2[3], n2, n2c, e2[3], e3[3];
};

__device__ __forceinline__ void s2s2_fwd(const double v1[3], const double v2[3], S2S2State& st) {
  st.n1 = sqrt(v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2]);
  st.n1c = fmax(st.n1, 1e-5);
  for (int i = 0; i < 3; ++i) st.e1[i] = v1[i] / st.n1c;
  st.dot = (st.e1[0] * v2[0] + st.e1[1] * v2[1]) + st.e1[2] * v2[2];
  for (int i = 0; i < 3; ++i) st.u2[i] = v2[i] - st.dot * st.e1[i];
  st.n2 = sqrt(st.u2[0] * st.u2[0] + st.u2[1] * st.u2[1] + st.u2[2] * st.u2[2]);
  st.n2c = fmax(st.n2, 1e-5);
  for (int i = 0; i < 3; ++i) st.e2[i] = st.u2[i] / st.n2c;
  cross3d(st.e1, st.e2, st.e3);
}

__device__ __forceinline__ void s2s2_bwd(const double v1[3], const double v2[3], const double g[9],
                                         double gv1[3], double gv2[3]) {
  S2S2State st;
  s2s2_fwd(v1, v2, st);
  double ge1[3] = {g[0], g[1], g[2]}, ge2[3] = {g[3], g[4], g[5]};
  const double ge3[3] = {g[6], g[7], g[8]};
  double t[3];
  cross3d(st.e2, ge3, t);  // d(e1 x e2)/de1 . g = e2 x g
  for (int i = 0; i < 3; ++i) ge1[i] += t[i];
  cross3d(ge3, st.e1, t);  // d/de2 = g x e1
  for (int i = 0; i < 3; ++i) ge2[i] += t[i];
  // e2 = u2 / clamp(|u2|, 1e-5)
  double gu2[3];
  const double de2 = ge2[0] * st.e2[0] + ge2[1] * st.e2[1] + ge2[2] * st.e2[2];
  const bool pass2 = st.n2 >= 1e-5;
  for (int i = 0; i < 3; ++i) gu2[i] = (ge2[i] - (pass2 ? de2 * st.e2[i] : 0.0)) / st.n2c;
  // u2 = v2 - dot e1 ; dot = <e1, v2>
  double gdot = 0.0;
  for (int i = 0; i < 3; ++i) {
    gv2[i] = gu2[i];
    gdot -= gu2[i] * st.e1[i];
    ge1[i] -= st.dot * gu2[i];
  }
  for (int i = 0; i < 3; ++i) {
    ge1[i] += gdot * v2[i];
    gv2[i] += gdot * st.e1[i];
  }
  // e1 = v1 / clamp(|v1|, 1e-5)
  const double de1 = ge1[0] * st.e1[0] + ge1[1] * st.e1[1] + ge1[2] * st.e1[2];
  const bool pass1 = st.n1 >= 1e-5;
  for (int i = 0; i < 3; ++i) gv1[i] = (ge1[i] - (pass1 ? de1 * st.e1[i] : 0.0)) / st.n1c;
}

}  // namespace lv

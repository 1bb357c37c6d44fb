// Per-sample SO(3) math, forward and hand-derived backward, in registers.
//
// Every function restates one reference op (file:line under the reference root) and
// keeps its fp32 evaluation order (the library is built with -ffp-contract=off, so
// nothing here is silently fused into an FMA).  Backward functions return the
// gradient autograd would produce for the same composition of torch ops.
#pragma once
#include <hip/hip_runtime.h>

namespace lv {

// ---------------------------------------------------------------- rodrigues
// lie_tools.py:17-43 (hat) and :56-64 (rodrigues).  K = hat(u), K2 = K@K.
__device__ __forceinline__ void hat_sq(const float u[3], float K[9], float K2[9]) {
  K[0] = 0.f;   K[1] = -u[2]; K[2] = u[1];
  K[3] = u[2];  K[4] = 0.f;   K[5] = -u[0];
  K[6] = -u[1]; K[7] = u[0];  K[8] = 0.f;
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

__device__ __forceinline__ float norm3(const float v[3]) {
  return sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
}

__device__ __forceinline__ void rodrigues_fwd(const float v[3], float R[9]) {
  const float th = norm3(v);
  const float u[3] = {v[0] / th, v[1] / th, v[2] / th};  // NaN at th == 0, like the reference
  float K[9], K2[9];
  hat_sq(u, K, K2);
  float s, c;
  sincosf(th, &s, &c);
  const float omc = 1.f - c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float eye = (i == 0 || i == 4 || i == 8) ? 1.f : 0.f;
    R[i] = (eye + s * K[i]) + omc * K2[i];
  }
}

// d/du of <g, s K(u) + w (u u^T - |u|^2 I)>
__device__ __forceinline__ void hat_sq_vjp(const float u[3], const float g[9], float s, float w,
                                           float gu[3]) {
  const float tr = g[0] + g[4] + g[8];
  float gsym_u[3];
#pragma unroll
  for (int m = 0; m < 3; ++m)
    gsym_u[m] = (g[m * 3 + 0] + g[0 * 3 + m]) * u[0] + (g[m * 3 + 1] + g[1 * 3 + m]) * u[1] +
                (g[m * 3 + 2] + g[2 * 3 + m]) * u[2];
  gu[0] = s * (g[7] - g[5]) + w * (gsym_u[0] - 2.f * tr * u[0]);
  gu[1] = s * (g[2] - g[6]) + w * (gsym_u[1] - 2.f * tr * u[1]);
  gu[2] = s * (g[3] - g[1]) + w * (gsym_u[2] - 2.f * tr * u[2]);
}

// (theta, u = v/theta) -> v chain rule.
__device__ __forceinline__ void polar_vjp(const float v[3], float th, const float gu[3], float gth,
                                          float gv[3]) {
  const float dot = gu[0] * v[0] + gu[1] * v[1] + gu[2] * v[2];
  const float inv = 1.f / th;
  const float inv3 = inv * inv * inv;
#pragma unroll
  for (int i = 0; i < 3; ++i) gv[i] = gu[i] * inv - dot * v[i] * inv3 + gth * v[i] * inv;
}

__device__ __forceinline__ void rodrigues_bwd(const float v[3], const float gR[9], float gv[3]) {
  const float th = norm3(v);
  const float u[3] = {v[0] / th, v[1] / th, v[2] / th};
  float K[9], K2[9];
  hat_sq(u, K, K2);
  float s, c;
  sincosf(th, &s, &c);
  float gth = 0.f;
#pragma unroll
  for (int i = 0; i < 9; ++i) gth += gR[i] * (c * K[i] + s * K2[i]);
  float gu[3];
  hat_sq_vjp(u, gR, s, 1.f - c, gu);
  polar_vjp(v, th, gu, gth, gv);
}

// ------------------------------------------------------------------ 3x3 ops
__device__ __forceinline__ void matmul3(const float A[9], const float B[9], float C[9]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[i * 3 + j] = (A[i * 3 + 0] * B[0 * 3 + j] + A[i * 3 + 1] * B[1 * 3 + j]) +
                     A[i * 3 + 2] * B[2 * 3 + j];
}
// C = A^T B
__device__ __forceinline__ void matmul3_tn(const float A[9], const float B[9], float C[9]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[i * 3 + j] = A[0 * 3 + i] * B[0 * 3 + j] + A[1 * 3 + i] * B[1 * 3 + j] +
                     A[2 * 3 + i] * B[2 * 3 + j];
}
// C = A B^T
__device__ __forceinline__ void matmul3_nt(const float A[9], const float B[9], float C[9]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[i * 3 + j] = A[i * 3 + 0] * B[j * 3 + 0] + A[i * 3 + 1] * B[j * 3 + 1] +
                     A[i * 3 + 2] * B[j * 3 + 2];
}

// ----------------------------------------------- group_matrix_to_quaternions
// lie_tools.py:112-157: 4-case trace method, eps 1e-6, case = first argmax.
struct QuatCase {
  float pre[4];
  float den[4];
  int k;
};

__device__ __forceinline__ void mat_to_quat_fwd(const float r[9], float q[4], QuatCase* qc) {
  const float a = r[0], b = r[4], c = r[8];
  float pre[4] = {((1.f + a) - b) - c, ((1.f - a) + b) - c, ((1.f - a) - b) + c,
                  ((1.f + a) + b) + c};
  float den[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) den[i] = 0.5f * sqrtf(1e-6f + fabsf(pre[i]));
  int k = 0;
  float best = den[0];
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (den[i] > best) { best = den[i]; k = i; }
  const float s01 = r[1] + r[3], s02 = r[2] + r[6], s12 = r[5] + r[7];
  const float d12 = r[5] - r[7], d20 = r[6] - r[2], d01 = r[1] - r[3];
  const float d4 = 4.f * best;
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

__device__ __forceinline__ void mat_to_quat_bwd(const float r[9], const float gq[4], float gr[9]) {
  float q[4];
  QuatCase qc;
  mat_to_quat_fwd(r, q, &qc);
  const int k = qc.k;
  const float d = qc.den[k];
  const float inv4d = 1.f / (4.f * d);
#pragma unroll
  for (int i = 0; i < 9; ++i) gr[i] = 0.f;
  // gradient into the denominator: q_k = d, q_j = N_j / (4 d)
  float gd = gq[k];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j != k) gd -= gq[j] * q[j] / d;
  // N_j partials: index pairs (p, m, sign of second) for s01, s02, s12, d12, d20, d01
  auto addN = [&](int which, float g) {
    switch (which) {
      case 0: gr[1] += g; gr[3] += g; break;   // s01
      case 1: gr[2] += g; gr[6] += g; break;   // s02
      case 2: gr[5] += g; gr[7] += g; break;   // s12
      case 3: gr[5] += g; gr[7] -= g; break;   // d12 = r12 - r21
      case 4: gr[6] += g; gr[2] -= g; break;   // d20 = r20 - r02
      default: gr[1] += g; gr[3] -= g; break;  // d01 = r01 - r10
    }
  };
  // numerators used per case: case0 (s01,s02,d12) at q1..q3; case1 (s01,s12,d20) at q0,q2,q3;
  // case2 (s02,s12,d01) at q0,q1,q3; case3 (d12,d20,d01) at q0..q2
  const int tab[4][4] = {{-1, 0, 1, 3}, {0, -1, 2, 4}, {1, 2, -1, 5}, {3, 4, 5, -1}};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j != k) addN(tab[k][j], gq[j] * inv4d);
  // d = 0.5 sqrt(1e-6 + |pre_k|)
  const float t = sqrtf(1e-6f + fabsf(qc.pre[k]));
  const float p = qc.pre[k];
  const float sg = (p > 0.f) ? 1.f : ((p < 0.f) ? -1.f : 0.f);
  const float gpre = gd * 0.25f / t * sg;
  const float coef[4][3] = {{1.f, -1.f, -1.f}, {-1.f, 1.f, -1.f}, {-1.f, -1.f, 1.f}, {1.f, 1.f, 1.f}};
  gr[0] += gpre * coef[k][0];
  gr[4] += gpre * coef[k][1];
  gr[8] += gpre * coef[k][2];
}

// ----------------------------------------------------- quaternions_to_eazyz
// lie_tools.py:160-175 (q scalar-last; beta clamped to [-1+1e-6, 1-1e-6]).
constexpr float kEazyzLo = (float)(-1.0 + 1e-6);
constexpr float kEazyzHi = (float)(1.0 - 1e-6);

__device__ __forceinline__ void quat_to_eazyz_fwd(const float q[4], float ang[3]) {
  const float a1 = q[1] * q[2] - q[0] * q[3];
  const float b1 = q[0] * q[2] + q[1] * q[3];
  const float cb = ((q[3] * q[3] - q[0] * q[0]) - q[1] * q[1]) + q[2] * q[2];
  const float a3 = q[0] * q[3] + q[1] * q[2];
  const float b3 = q[1] * q[3] - q[0] * q[2];
  ang[0] = atan2f(a1, b1);
  ang[1] = acosf(fminf(fmaxf(cb, kEazyzLo), kEazyzHi));
  ang[2] = atan2f(a3, b3);
}

__device__ __forceinline__ void quat_to_eazyz_bwd(const float q[4], const float ga[3], float gq[4]) {
  const float a1 = q[1] * q[2] - q[0] * q[3];
  const float b1 = q[0] * q[2] + q[1] * q[3];
  const float cb = ((q[3] * q[3] - q[0] * q[0]) - q[1] * q[1]) + q[2] * q[2];
  const float a3 = q[0] * q[3] + q[1] * q[2];
  const float b3 = q[1] * q[3] - q[0] * q[2];
  const float r1 = a1 * a1 + b1 * b1, r3 = a3 * a3 + b3 * b3;
  const float ga1 = ga[0] * b1 / r1, gb1 = ga[0] * -a1 / r1;
  const float ga3 = ga[2] * b3 / r3, gb3 = ga[2] * -a3 / r3;
  const float x = fminf(fmaxf(cb, kEazyzLo), kEazyzHi);
  const bool pass = (cb >= kEazyzLo) && (cb <= kEazyzHi);
  const float gcb = pass ? (-ga[1] / sqrtf(1.f - x * x)) : 0.f;
  gq[0] = -q[3] * ga1 + q[2] * gb1 + q[3] * ga3 - q[2] * gb3 - 2.f * q[0] * gcb;
  gq[1] = q[2] * ga1 + q[3] * gb1 + q[2] * ga3 + q[3] * gb3 - 2.f * q[1] * gcb;
  gq[2] = q[1] * ga1 + q[0] * gb1 + q[1] * ga3 - q[0] * gb3 + 2.f * q[2] * gcb;
  gq[3] = -q[0] * ga1 + q[1] * gb1 + q[0] * ga3 + q[1] * gb3 + 2.f * q[3] * gcb;
}

// ------------------------------------------------ quaternions_to_group_matrix
// lie_tools.py:183-192: normalise, then the reference's (transposed-active) matrix.
__device__ __forceinline__ void quat_to_mat_fwd(const float q0[4], float R[9]) {
  const float nrm = sqrtf(q0[0] * q0[0] + q0[1] * q0[1] + q0[2] * q0[2] + q0[3] * q0[3]);
  const float x = q0[0] / nrm, y = q0[1] / nrm, z = q0[2] / nrm, w = q0[3] / nrm;
  R[0] = ((x * x - y * y) - z * z) + w * w;
  R[1] = 2.f * (x * y + z * w);
  R[2] = 2.f * (x * z - y * w);
  R[3] = 2.f * (x * y - z * w);
  R[4] = ((-x * x + y * y) - z * z) + w * w;
  R[5] = 2.f * (y * z + x * w);
  R[6] = 2.f * (x * z + y * w);
  R[7] = 2.f * (y * z - x * w);
  R[8] = ((-x * x - y * y) + z * z) + w * w;
}

__device__ __forceinline__ void quat_to_mat_bwd(const float q0[4], const float g[9], float gq[4]) {
  const float nrm = sqrtf(q0[0] * q0[0] + q0[1] * q0[1] + q0[2] * q0[2] + q0[3] * q0[3]);
  const float x = q0[0] / nrm, y = q0[1] / nrm, z = q0[2] / nrm, w = q0[3] / nrm;
  float gn[4];
  gn[0] = 2.f * (x * (g[0] - g[4] - g[8]) + y * (g[1] + g[3]) + z * (g[2] + g[6]) + w * (g[5] - g[7]));
  gn[1] = 2.f * (-y * (g[0] - g[4] + g[8]) + x * (g[1] + g[3]) - w * (g[2] - g[6]) + z * (g[5] + g[7]));
  gn[2] = 2.f * (-z * (g[0] + g[4] - g[8]) + w * (g[1] - g[3]) + x * (g[2] + g[6]) + y * (g[5] + g[7]));
  gn[3] = 2.f * (w * (g[0] + g[4] + g[8]) + z * (g[1] - g[3]) - y * (g[2] - g[6]) + x * (g[5] - g[7]));
  const float dot = gn[0] * x + gn[1] * y + gn[2] * z + gn[3] * w;
  gq[0] = (gn[0] - dot * x) / nrm;
  gq[1] = (gn[1] - dot * y) / nrm;
  gq[2] = (gn[2] - dot * z) / nrm;
  gq[3] = (gn[3] - dot * w) / nrm;
}

// ------------------------------------------------------------- s2s1rodrigues
// lie_tools.py:67-78: R = I + sin K + (1 - cos) K@K, K = hat(axis), (cos, sin) given.
__device__ __forceinline__ void s2s1_fwd(const float a[3], const float cs[2], float R[9]) {
  float K[9], K2[9];
  hat_sq(a, K, K2);
  const float omc = 1.f - cs[0];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float eye = (i == 0 || i == 4 || i == 8) ? 1.f : 0.f;
    R[i] = (eye + cs[1] * K[i]) + omc * K2[i];
  }
}

__device__ __forceinline__ void s2s1_bwd(const float a[3], const float cs[2], const float g[9],
                                         float ga[3], float gcs[2]) {
  float K[9], K2[9];
  hat_sq(a, K, K2);
  float gs = 0.f, gc = 0.f;
#pragma unroll
  for (int i = 0; i < 9; ++i) { gs += g[i] * K[i]; gc -= g[i] * K2[i]; }
  hat_sq_vjp(a, g, cs[1], 1.f - cs[0], ga);
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

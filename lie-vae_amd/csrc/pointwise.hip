// Per-sample SO(3) conversions and reparameterisation kernels (forward + backward).
// One thread per sample; all state in registers (so3_device.h).  These are
// latency-trivial, byte-bound maps; they exist so the whole latent path runs on the
// GPU through the C ABI rather than as chains of tiny torch ops.
#include <cmath>
#include <cstdarg>
#include <cstring>

#include "lv_common.h"
#include "so3_device.h"

namespace lv {

namespace {
thread_local char g_err[512] = {0};
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
void clear_error() { g_err[0] = 0; }

constexpr int kBlock = 256;

inline dim3 grid_for(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  if (b > 65536) b = 65536;  // grid-stride beyond
  return dim3((unsigned)b);
}

#define LV_FOR_EACH(i, n) \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

template <typename T, int K>
__device__ __forceinline__ void ld(const T* p, T (&x)[K]) {
#pragma unroll
  for (int i = 0; i < K; ++i) x[i] = p[i];
}
template <typename T, int K>
__device__ __forceinline__ void st(T* p, const T (&x)[K]) {
#pragma unroll
  for (int i = 0; i < K; ++i) p[i] = x[i];
}

template <typename T>
__global__ void so3_exp_fwd_k(const T* v, T* R, int64_t n) {
  LV_FOR_EACH(i, n) {
    T a[3], r[9];
    ld(v + i * 3, a);
    rodrigues_fwd(a, r);
    st(R + i * 9, r);
  }
}
template <typename T>
__global__ void so3_exp_bwd_k(const T* v, const T* gR, T* gv, int64_t n) {
  LV_FOR_EACH(i, n) {
    T a[3], g[9], o[3];
    ld(v + i * 3, a);
    ld(gR + i * 9, g);
    rodrigues_bwd(a, g, o);
    st(gv + i * 3, o);
  }
}

// z[s,b] = mu[b] @ exp(v[s,b])
template <typename T>
__global__ void so3_sample_fwd_k(const T* mu, const T* v, T* z, int64_t ns, int64_t B) {
  LV_FOR_EACH(i, ns * B) {
    const int64_t b = i % B;
    T a[3], r[9], m[9], o[9];
    ld(v + i * 3, a);
    ld(mu + b * 9, m);
    rodrigues_fwd(a, r);
    matmul3(m, r, o);
    st(z + i * 9, o);
  }
}
// gv[s,b] via exp backward of mu^T gz; gmu[b] = sum_s gz R^T (fixed order)
template <typename T>
__global__ void so3_sample_bwd_k(const T* mu, const T* v, const T* gz, T* gmu,
                                 T* gv, int64_t ns, int64_t B) {
  LV_FOR_EACH(b, B) {
    T m[9], acc[9];
    ld(mu + b * 9, m);
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[k] = T(0);
    for (int64_t s = 0; s < ns; ++s) {
      const int64_t i = s * B + b;
      T a[3], r[9], g[9], gr[9], t[9], o[3];
      ld(v + i * 3, a);
      ld(gz + i * 9, g);
      rodrigues_fwd(a, r);
      matmul3_nt(g, r, t);
#pragma unroll
      for (int k = 0; k < 9; ++k) acc[k] += t[k];
      matmul3_tn(m, g, gr);
      rodrigues_bwd(a, gr, o);
      st(gv + i * 3, o);
    }
    st(gmu + b * 9, acc);
  }
}

// Backward of the fused path's prologue, z = mu @ exp(v) (mu optional) -> ZYZ angles, in
// one pass per sample: the composition of so3_sample_fwd/so3_exp_fwd, mat_to_eazyz_bwd
// and so3_sample_bwd/so3_exp_bwd above (same device functions, same operation order,
// hence bitwise the same gradients) without the three launches and the (n,3,3)
// round trips through memory.  reparameterize.py:269-273 + vae.py:182 (autograd in the
// reference).
template <typename T>
__global__ void exp_eazyz_vjp_k(const T* mu, const T* v, const T* ga, T* gmu,
                                T* gv, int64_t n) {
  LV_FOR_EACH(i, n) {
    T a[3], g[3], m[9], gm[9], o[3];
    ld(v + i * 3, a);
    ld(ga + i * 3, g);
    if (mu) ld(mu + i * 9, m);
    exp_eazyz_vjp_sample(a, mu != nullptr, m, g, gm, o);
    if (mu) st(gmu + i * 9, gm);
    st(gv + i * 3, o);
  }
}

template <typename T>
__global__ void quat_to_mat_fwd_k(const T* q, T* R, int64_t n) {
  LV_FOR_EACH(i, n) {
    T a[4], r[9];
    ld(q + i * 4, a);
    quat_to_mat_fwd(a, r);
    st(R + i * 9, r);
  }
}
template <typename T>
__global__ void quat_to_mat_bwd_k(const T* q, const T* gR, T* gq, int64_t n) {
  LV_FOR_EACH(i, n) {
    T a[4], g[9], o[4];
    ld(q + i * 4, a);
    ld(gR + i * 9, g);
    quat_to_mat_bwd(a, g, o);
    st(gq + i * 4, o);
  }
}

template <typename T>
__global__ void mat_to_quat_fwd_k(const T* R, T* q, int64_t n) {
  LV_FOR_EACH(i, n) {
    T r[9], o[4];
    ld(R + i * 9, r);
    mat_to_quat_fwd(r, o, nullptr);
    st(q + i * 4, o);
  }
}
template <typename T>
__global__ void mat_to_quat_bwd_k(const T* R, const T* gq, T* gR, int64_t n) {
  LV_FOR_EACH(i, n) {
    T r[9], g[4], o[9];
    ld(R + i * 9, r);
    ld(gq + i * 4, g);
    mat_to_quat_bwd(r, g, o);
    st(gR + i * 9, o);
  }
}

template <typename T>
__global__ void quat_to_eazyz_fwd_k(const T* q, T* ang, int64_t n) {
  LV_FOR_EACH(i, n) {
    T a[4], o[3];
    ld(q + i * 4, a);
    quat_to_eazyz_fwd(a, o);
    st(ang + i * 3, o);
  }
}
template <typename T>
__global__ void quat_to_eazyz_bwd_k(const T* q, const T* ga, T* gq, int64_t n) {
  LV_FOR_EACH(i, n) {
    T a[4], g[3], o[4];
    ld(q + i * 4, a);
    ld(ga + i * 3, g);
    quat_to_eazyz_bwd(a, g, o);
    st(gq + i * 4, o);
  }
}

template <typename T>
__global__ void mat_to_eazyz_fwd_k(const T* R, T* ang, int64_t n) {
  LV_FOR_EACH(i, n) {
    T r[9], q[4], o[3];
    ld(R + i * 9, r);
    mat_to_quat_fwd(r, q, nullptr);
    quat_to_eazyz_fwd(q, o);
    st(ang + i * 3, o);
  }
}
template <typename T>
__global__ void mat_to_eazyz_bwd_k(const T* R, const T* ga, T* gR, int64_t n) {
  LV_FOR_EACH(i, n) {
    T r[9], q[4], g[3], gq[4], o[9];
    ld(R + i * 9, r);
    ld(ga + i * 3, g);
    mat_to_quat_fwd(r, q, nullptr);
    quat_to_eazyz_bwd(q, g, gq);
    mat_to_quat_bwd(r, gq, o);
    st(gR + i * 9, o);
  }
}

template <typename T>
__global__ void s2s1_fwd_k(const T* ax, const T* cs, T* R, int64_t n) {
  LV_FOR_EACH(i, n) {
    T a[3], c[2], r[9];
    ld(ax + i * 3, a);
    ld(cs + i * 2, c);
    s2s1_fwd(a, c, r);
    st(R + i * 9, r);
  }
}
template <typename T>
__global__ void s2s1_bwd_k(const T* ax, const T* cs, const T* gR, T* gax,
                           T* gcs, int64_t n) {
  LV_FOR_EACH(i, n) {
    T a[3], c[2], g[9], oa[3], oc[2];
    ld(ax + i * 3, a);
    ld(cs + i * 2, c);
    ld(gR + i * 9, g);
    s2s1_bwd(a, c, g, oa, oc);
    st(gax + i * 3, oa);
    st(gcs + i * 2, oc);
  }
}

__global__ void s2s2_fwd_k(const double* v1, const double* v2, double* R, int64_t n) {
  LV_FOR_EACH(i, n) {
    double a[3], b[3];
    for (int k = 0; k < 3; ++k) { a[k] = v1[i * 3 + k]; b[k] = v2[i * 3 + k]; }
    S2S2State s;
    s2s2_fwd(a, b, s);
    for (int k = 0; k < 3; ++k) {
      R[i * 9 + k] = s.e1[k];
      R[i * 9 + 3 + k] = s.e2[k];
      R[i * 9 + 6 + k] = s.e3[k];
    }
  }
}
__global__ void s2s2_bwd_k(const double* v1, const double* v2, const double* gR, double* g1,
                           double* g2, int64_t n) {
  LV_FOR_EACH(i, n) {
    double a[3], b[3], g[9], o1[3], o2[3];
    for (int k = 0; k < 3; ++k) { a[k] = v1[i * 3 + k]; b[k] = v2[i * 3 + k]; }
    for (int k = 0; k < 9; ++k) g[k] = gR[i * 9 + k];
    s2s2_bwd(a, b, g, o1, o2);
    for (int k = 0; k < 3; ++k) { g1[i * 3 + k] = o1[k]; g2[i * 3 + k] = o2[k]; }
  }
}

// ---------------------------------------------------------------- N0 + SO(3) density
// softplus(x) = log1p(exp(x)), identity above threshold 20 (torch defaults).
__global__ void softplus_fwd_k(const float* h, float* s, int64_t n) {
  LV_FOR_EACH(i, n) {
    const float x = h[i];
    s[i] = x > 20.f ? x : log1pf(expf(x));
  }
}
__global__ void softplus_bwd_k(const float* h, const float* gs, float* gh, int64_t n) {
  LV_FOR_EACH(i, n) {
    const float x = h[i];
    const float z = expf(x);
    gh[i] = x > 20.f ? gs[i] : gs[i] * z / (z + 1.f);
  }
}
__global__ void n0_sample_fwd_k(const float* sigma, const float* eps, float* v, int64_t ns, int64_t B) {
  LV_FOR_EACH(i, ns * B * 3) {
    const int64_t bj = i % (B * 3);
    v[i] = eps[i] * sigma[bj];
  }
}
__global__ void n0_sample_bwd_k(const float* eps, const float* gv, float* gs, int64_t ns, int64_t B) {
  LV_FOR_EACH(bj, B * 3) {
    float acc = 0.f;
    for (int64_t s = 0; s < ns; ++s) acc += gv[s * B * 3 + bj] * eps[s * B * 3 + bj];
    gs[bj] = acc;
  }
}

// log q(z|x) for z = exp(v): reparameterize.py:233-263 with torch.distributions.Normal
// log_prob (loc 0) and the max-shifted logsumexp of lie_vae/utils.py:4-26.
constexpr float kTwoPi = 6.283185307179586f;
constexpr float kHalfLog2Pi = 0.9189385332046727f;  // log(sqrt(2 pi))

constexpr int kMaxWrap = 64;

// One wrapped term l_t of the density (reparameterize.py:240-260), logs of sigma hoisted.
__device__ __forceinline__ float logpost_term(int t, float th, const float u[3],
                                              const float var[3], const float logsig[3]) {
  const float thk = th + (float)t * kTwoPi;
  float lp = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float x = u[j] * thk;
    const float term = (-(x * x) / (2.f * var[j]) - logsig[j]) - kHalfLog2Pi;
    lp = (j == 0) ? term : lp + term;
  }
  const float th2 = fmaxf(thk * thk, 1e-3f);
  const float den = fmaxf(2.f - 2.f * cosf(thk), 1e-3f);
  return lp + logf(th2 / den);
}

// max-shifted logsumexp over t = -k..k (lie_vae/utils.py:4-26), two passes.
__device__ __forceinline__ float logpost_lse(float th, const float u[3], const float var[3],
                                             const float logsig[3], int k) {
  float m = -INFINITY;
  for (int t = -k; t <= k; ++t) m = fmaxf(m, logpost_term(t, th, u, var, logsig));
  float sum = 0.f;
  for (int t = -k; t <= k; ++t) sum += expf(logpost_term(t, th, u, var, logsig) - m);
  return m + logf(sum);
}

__global__ void so3_logpost_fwd_k(const float* v, const float* sigma, float* out, int64_t ns,
                                  int64_t B, int k) {
  LV_FOR_EACH(i, ns * B) {
    const int64_t b = i % B;
    float a[3], sg[3], var[3], ls[3];
    ld(v + i * 3, a);
    ld(sigma + b * 3, sg);
    for (int j = 0; j < 3; ++j) { var[j] = sg[j] * sg[j]; ls[j] = logf(sg[j]); }
    const float th = norm3(a);
    const float u[3] = {a[0] / th, a[1] / th, a[2] / th};
    out[i] = logpost_lse(th, u, var, ls, k);
  }
}

__global__ void so3_logpost_bwd_k(const float* v, const float* sigma, const float* gout, float* gv,
                                  float* gsig, int64_t ns, int64_t B, int k) {
  LV_FOR_EACH(b, B) {
    float sg[3], var[3], ls[3];
    ld(sigma + b * 3, sg);
    for (int j = 0; j < 3; ++j) { var[j] = sg[j] * sg[j]; ls[j] = logf(sg[j]); }
    float gsacc[3] = {0.f, 0.f, 0.f};
    for (int64_t s = 0; s < ns; ++s) {
      const int64_t i = s * B + b;
      float a[3];
      ld(v + i * 3, a);
      const float th = norm3(a);
      const float u[3] = {a[0] / th, a[1] / th, a[2] / th};
      const float lse = logpost_lse(th, u, var, ls, k);
      const float g = gout[i];
      float gth = 0.f, gu[3] = {0.f, 0.f, 0.f};
      for (int t = -k; t <= k; ++t) {
        const float w = g * expf(logpost_term(t, th, u, var, ls) - lse);
        const float thk = th + (float)t * kTwoPi;
        float dth = 0.f;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const float x = u[j] * thk;
          dth -= x * u[j] / var[j];
          gu[j] -= w * x * thk / var[j];
          gsacc[j] += w * ((x * x) / (var[j] * sg[j]) - 1.f / sg[j]);
        }
        if (thk * thk >= 1e-3f) dth += 2.f * thk / (thk * thk);
        const float den = 2.f - 2.f * cosf(thk);
        if (den >= 1e-3f) dth -= 2.f * sinf(thk) / den;
        gth += w * dth;
      }
      float o[3];
      polar_vjp(a, th, gu, gth, o);
      st(gv + i * 3, o);
    }
    st(gsig + b * 3, gsacc);
  }
}

// Wave-per-element variants: lane t holds wrapped term t - k (2k+1 <= 64), max and sum
// over the terms by cross-lane reductions.  The thread-per-element kernels above run the
// 2k+1 terms (x2 passes, x3 in backward) serially per thread: at training sizes
// (ns * B = 512) that is a latency chain of ~60 transcendental terms on a few waves.
// Same per-term arithmetic; only the order of the exp-sum (and gradient sums) differs.
constexpr int kWaveMaxK = 31;
constexpr int64_t kWaveMaxElems = 1 << 16;  // beyond: enough elements to fill the chip per thread

__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
  return x;
}
__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

#define LV_FOR_EACH_WAVE(i, n)                                                          \
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < (n);        \
       i += ((int64_t)gridDim.x * blockDim.x) >> 6)

__global__ void so3_logpost_fwd_wave_k(const float* v, const float* sigma, float* out, int64_t ns,
                                       int64_t B, int k) {
  const int lane = threadIdx.x & 63;
  const bool on = lane < 2 * k + 1;
  LV_FOR_EACH_WAVE(i, ns * B) {
    const int64_t b = i % B;
    float a[3], sg[3], var[3], ls[3];
    ld(v + i * 3, a);
    ld(sigma + b * 3, sg);
    for (int j = 0; j < 3; ++j) { var[j] = sg[j] * sg[j]; ls[j] = logf(sg[j]); }
    const float th = norm3(a);
    const float u[3] = {a[0] / th, a[1] / th, a[2] / th};
    const float term = on ? logpost_term(lane - k, th, u, var, ls) : -INFINITY;
    const float m = wave_max(term);
    const float sum = wave_sum(on ? expf(term - m) : 0.f);
    if (lane == 0) out[i] = m + logf(sum);
  }
}

__global__ void so3_logpost_bwd_wave_k(const float* v, const float* sigma, const float* gout,
                                       float* gv, float* gsig, int64_t ns, int64_t B, int k) {
  const int lane = threadIdx.x & 63;
  const bool on = lane < 2 * k + 1;
  const int t = lane - k;
  LV_FOR_EACH_WAVE(b, B) {
    float sg[3], var[3], ls[3];
    ld(sigma + b * 3, sg);
    for (int j = 0; j < 3; ++j) { var[j] = sg[j] * sg[j]; ls[j] = logf(sg[j]); }
    float gsacc[3] = {0.f, 0.f, 0.f};
    for (int64_t s = 0; s < ns; ++s) {
      const int64_t i = s * B + b;
      float a[3];
      ld(v + i * 3, a);
      const float th = norm3(a);
      const float u[3] = {a[0] / th, a[1] / th, a[2] / th};
      const float term = on ? logpost_term(t, th, u, var, ls) : -INFINITY;
      const float m = wave_max(term);
      const float lse = m + logf(wave_sum(on ? expf(term - m) : 0.f));
      float gth = 0.f, gu[3] = {0.f, 0.f, 0.f};
      if (on) {
        const float w = gout[i] * expf(term - lse);
        const float thk = th + (float)t * kTwoPi;
        float dth = 0.f;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const float x = u[j] * thk;
          dth -= x * u[j] / var[j];
          gu[j] = -(w * x * thk / var[j]);
          gsacc[j] += w * ((x * x) / (var[j] * sg[j]) - 1.f / sg[j]);
        }
        if (thk * thk >= 1e-3f) dth += 2.f * thk / (thk * thk);
        const float den = 2.f - 2.f * cosf(thk);
        if (den >= 1e-3f) dth -= 2.f * sinf(thk) / den;
        gth = w * dth;
      }
      gth = wave_sum(gth);
#pragma unroll
      for (int j = 0; j < 3; ++j) gu[j] = wave_sum(gu[j]);
      if (lane == 0) {
        float o[3];
        polar_vjp(a, th, gu, gth, o);
        st(gv + i * 3, o);
      }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) gsacc[j] = wave_sum(gsacc[j]);
    if (lane == 0) st(gsig + b * 3, gsacc);
  }
}

inline dim3 grid_for_waves(int64_t nwaves) {
  int64_t b = (nwaves * 64 + kBlock - 1) / kBlock;
  if (b > 65536) b = 65536;
  return dim3((unsigned)b);
}

}  // namespace lv

using namespace lv;

#define LV_PTRS(...) LV_CHECK_ARG(n == 0 || (__VA_ARGS__), "null pointer argument")
#define LV_LAUNCH1(kern, n, ...)                                                     \
  do {                                                                               \
    clear_error();                                                                   \
    LV_CHECK_ARG((n) >= 0, "n must be >= 0");                                        \
    if ((n) == 0) return LV_OK;                                                      \
    hipLaunchKernelGGL(kern, grid_for(n), dim3(kBlock), 0, (hipStream_t)stream, __VA_ARGS__); \
    LV_RETURN_LAUNCH(#kern);                                                         \
  } while (0)

extern "C" {

int lv_abi_version(void) { return 1; }
const char* lv_last_error(void) { return g_err; }
int lv_max_degree(void) { return LV_MAX_DEGREE; }

int lv_so3_exp_fwd(const float* v, float* R, int64_t n, void* stream) {
  LV_PTRS(v && R);
  LV_LAUNCH1(so3_exp_fwd_k<float>, n, v, R, n);
}
int lv_so3_exp_bwd(const float* v, const float* gR, float* gv, int64_t n, void* stream) {
  LV_PTRS(v && gR && gv);
  LV_LAUNCH1(so3_exp_bwd_k<float>, n, v, gR, gv, n);
}
int lv_so3_sample_fwd(const float* mu, const float* v, float* z, int64_t ns, int64_t B, void* stream) {
  const int64_t n = ns * B;
  LV_CHECK_ARG(ns >= 0 && B >= 0, "bad sizes");
  LV_PTRS(mu && v && z);
  LV_LAUNCH1(so3_sample_fwd_k<float>, n, mu, v, z, ns, B);
}
int lv_so3_sample_bwd(const float* mu, const float* v, const float* gz, float* gmu, float* gv,
                      int64_t ns, int64_t B, void* stream) {
  const int64_t n = B;
  LV_CHECK_ARG(ns >= 0 && B >= 0, "bad sizes");
  LV_PTRS(mu && v && gz && gmu && gv);
  if (ns == 0) {
    (void)hipMemsetAsync(gmu, 0, sizeof(float) * 9 * B, (hipStream_t)stream);
    return LV_OK;
  }
  LV_LAUNCH1(so3_sample_bwd_k<float>, n, mu, v, gz, gmu, gv, ns, B);
}
int lv_exp_eazyz_vjp(const float* mu, const float* v, const float* gang, float* gmu, float* gv,
                     int64_t n, void* stream) {
  LV_PTRS(v && gang && gv && (!mu || gmu));
  LV_LAUNCH1(exp_eazyz_vjp_k<float>, n, mu, v, gang, gmu, gv, n);
}
int lv_quat_to_mat_fwd(const float* q, float* R, int64_t n, void* stream) {
  LV_PTRS(q && R);
  LV_LAUNCH1(quat_to_mat_fwd_k<float>, n, q, R, n);
}
int lv_quat_to_mat_bwd(const float* q, const float* gR, float* gq, int64_t n, void* stream) {
  LV_PTRS(q && gR && gq);
  LV_LAUNCH1(quat_to_mat_bwd_k<float>, n, q, gR, gq, n);
}
int lv_mat_to_quat_fwd(const float* R, float* q, int64_t n, void* stream) {
  LV_PTRS(R && q);
  LV_LAUNCH1(mat_to_quat_fwd_k<float>, n, R, q, n);
}
int lv_mat_to_quat_bwd(const float* R, const float* gq, float* gR, int64_t n, void* stream) {
  LV_PTRS(R && gq && gR);
  LV_LAUNCH1(mat_to_quat_bwd_k<float>, n, R, gq, gR, n);
}
int lv_quat_to_eazyz_fwd(const float* q, float* ang, int64_t n, void* stream) {
  LV_PTRS(q && ang);
  LV_LAUNCH1(quat_to_eazyz_fwd_k<float>, n, q, ang, n);
}
int lv_quat_to_eazyz_bwd(const float* q, const float* gang, float* gq, int64_t n, void* stream) {
  LV_PTRS(q && gang && gq);
  LV_LAUNCH1(quat_to_eazyz_bwd_k<float>, n, q, gang, gq, n);
}
int lv_mat_to_eazyz_fwd(const float* R, float* ang, int64_t n, void* stream) {
  LV_PTRS(R && ang);
  LV_LAUNCH1(mat_to_eazyz_fwd_k<float>, n, R, ang, n);
}
int lv_mat_to_eazyz_bwd(const float* R, const float* gang, float* gR, int64_t n, void* stream) {
  LV_PTRS(R && gang && gR);
  LV_LAUNCH1(mat_to_eazyz_bwd_k<float>, n, R, gang, gR, n);
}
int lv_s2s1_fwd(const float* axis, const float* cs, float* R, int64_t n, void* stream) {
  LV_PTRS(axis && cs && R);
  LV_LAUNCH1(s2s1_fwd_k<float>, n, axis, cs, R, n);
}
int lv_s2s1_bwd(const float* axis, const float* cs, const float* gR, float* gaxis, float* gcs,
                int64_t n, void* stream) {
  LV_PTRS(axis && cs && gR && gaxis && gcs);
  LV_LAUNCH1(s2s1_bwd_k<float>, n, axis, cs, gR, gaxis, gcs, n);
}
// fp64 twins of the per-sample maps above: the reference's maps follow the input dtype
// (lie_tools.py:28-38,61 -- new_tensor / eye(dtype=v.dtype)), and its own self-tests run
// them in fp64 (lie_tools.py:271-291).  Same templates, T = double.
int lv_so3_exp_fwd_f64(const double* v, double* R, int64_t n, void* stream) {
  LV_PTRS(v && R);
  LV_LAUNCH1(so3_exp_fwd_k<double>, n, v, R, n);
}
int lv_so3_exp_bwd_f64(const double* v, const double* gR, double* gv, int64_t n, void* stream) {
  LV_PTRS(v && gR && gv);
  LV_LAUNCH1(so3_exp_bwd_k<double>, n, v, gR, gv, n);
}
int lv_so3_sample_fwd_f64(const double* mu, const double* v, double* z, int64_t ns, int64_t B, void* stream) {
  const int64_t n = ns * B;
  LV_CHECK_ARG(ns >= 0 && B >= 0, "bad sizes");
  LV_PTRS(mu && v && z);
  LV_LAUNCH1(so3_sample_fwd_k<double>, n, mu, v, z, ns, B);
}
int lv_so3_sample_bwd_f64(const double* mu, const double* v, const double* gz, double* gmu, double* gv,
                      int64_t ns, int64_t B, void* stream) {
  const int64_t n = B;
  LV_CHECK_ARG(ns >= 0 && B >= 0, "bad sizes");
  LV_PTRS(mu && v && gz && gmu && gv);
  if (ns == 0) {
    (void)hipMemsetAsync(gmu, 0, sizeof(double) * 9 * B, (hipStream_t)stream);
    return LV_OK;
  }
  LV_LAUNCH1(so3_sample_bwd_k<double>, n, mu, v, gz, gmu, gv, ns, B);
}
int lv_exp_eazyz_vjp_f64(const double* mu, const double* v, const double* gang, double* gmu, double* gv,
                     int64_t n, void* stream) {
  LV_PTRS(v && gang && gv && (!mu || gmu));
  LV_LAUNCH1(exp_eazyz_vjp_k<double>, n, mu, v, gang, gmu, gv, n);
}
int lv_quat_to_mat_fwd_f64(const double* q, double* R, int64_t n, void* stream) {
  LV_PTRS(q && R);
  LV_LAUNCH1(quat_to_mat_fwd_k<double>, n, q, R, n);
}
int lv_quat_to_mat_bwd_f64(const double* q, const double* gR, double* gq, int64_t n, void* stream) {
  LV_PTRS(q && gR && gq);
  LV_LAUNCH1(quat_to_mat_bwd_k<double>, n, q, gR, gq, n);
}
int lv_mat_to_quat_fwd_f64(const double* R, double* q, int64_t n, void* stream) {
  LV_PTRS(R && q);
  LV_LAUNCH1(mat_to_quat_fwd_k<double>, n, R, q, n);
}
int lv_mat_to_quat_bwd_f64(const double* R, const double* gq, double* gR, int64_t n, void* stream) {
  LV_PTRS(R && gq && gR);
  LV_LAUNCH1(mat_to_quat_bwd_k<double>, n, R, gq, gR, n);
}
int lv_quat_to_eazyz_fwd_f64(const double* q, double* ang, int64_t n, void* stream) {
  LV_PTRS(q && ang);
  LV_LAUNCH1(quat_to_eazyz_fwd_k<double>, n, q, ang, n);
}
int lv_quat_to_eazyz_bwd_f64(const double* q, const double* gang, double* gq, int64_t n, void* stream) {
  LV_PTRS(q && gang && gq);
  LV_LAUNCH1(quat_to_eazyz_bwd_k<double>, n, q, gang, gq, n);
}
int lv_mat_to_eazyz_fwd_f64(const double* R, double* ang, int64_t n, void* stream) {
  LV_PTRS(R && ang);
  LV_LAUNCH1(mat_to_eazyz_fwd_k<double>, n, R, ang, n);
}
int lv_mat_to_eazyz_bwd_f64(const double* R, const double* gang, double* gR, int64_t n, void* stream) {
  LV_PTRS(R && gang && gR);
  LV_LAUNCH1(mat_to_eazyz_bwd_k<double>, n, R, gang, gR, n);
}
int lv_s2s1_fwd_f64(const double* axis, const double* cs, double* R, int64_t n, void* stream) {
  LV_PTRS(axis && cs && R);
  LV_LAUNCH1(s2s1_fwd_k<double>, n, axis, cs, R, n);
}
int lv_s2s1_bwd_f64(const double* axis, const double* cs, const double* gR, double* gaxis, double* gcs,
                int64_t n, void* stream) {
  LV_PTRS(axis && cs && gR && gaxis && gcs);
  LV_LAUNCH1(s2s1_bwd_k<double>, n, axis, cs, gR, gaxis, gcs, n);
}
int lv_s2s2_fwd_f64(const double* v1, const double* v2, double* R, int64_t n, void* stream) {
  LV_PTRS(v1 && v2 && R);
  LV_LAUNCH1(s2s2_fwd_k, n, v1, v2, R, n);
}
int lv_s2s2_bwd_f64(const double* v1, const double* v2, const double* gR, double* gv1,
                    double* gv2, int64_t n, void* stream) {
  LV_PTRS(v1 && v2 && gR && gv1 && gv2);
  LV_LAUNCH1(s2s2_bwd_k, n, v1, v2, gR, gv1, gv2, n);
}
int lv_softplus_fwd(const float* h, float* sigma, int64_t n, void* stream) {
  LV_PTRS(h && sigma);
  LV_LAUNCH1(softplus_fwd_k, n, h, sigma, n);
}
int lv_softplus_bwd(const float* h, const float* gsigma, float* gh, int64_t n, void* stream) {
  LV_PTRS(h && gsigma && gh);
  LV_LAUNCH1(softplus_bwd_k, n, h, gsigma, gh, n);
}
int lv_n0_sample_fwd(const float* sigma, const float* eps, float* v, int64_t ns, int64_t B,
                     void* stream) {
  const int64_t n = ns * B * 3;
  LV_CHECK_ARG(ns >= 0 && B >= 0, "bad sizes");
  LV_PTRS(sigma && eps && v);
  LV_LAUNCH1(n0_sample_fwd_k, n, sigma, eps, v, ns, B);
}
int lv_n0_sample_bwd(const float* eps, const float* gv, float* gsigma, int64_t ns, int64_t B,
                     void* stream) {
  const int64_t n = B * 3;
  LV_CHECK_ARG(ns >= 0 && B >= 0, "bad sizes");
  LV_PTRS(eps && gv && gsigma);
  LV_LAUNCH1(n0_sample_bwd_k, n, eps, gv, gsigma, ns, B);
}
int lv_so3_log_posterior_fwd(const float* v, const float* sigma, float* out, int64_t ns,
                             int64_t B, int k, void* stream) {
  const int64_t n = ns * B;
  LV_CHECK_ARG(ns >= 0 && B >= 0, "bad sizes");
  LV_CHECK_ARG(k >= 0 && k <= kMaxWrap, "k must be in [0, %d]", kMaxWrap);
  LV_PTRS(v && sigma && out);
  if (n > 0 && k <= kWaveMaxK && n <= kWaveMaxElems) {
    clear_error();
    hipLaunchKernelGGL(so3_logpost_fwd_wave_k, grid_for_waves(n), dim3(kBlock), 0,
                       (hipStream_t)stream, v, sigma, out, ns, B, k);
    LV_RETURN_LAUNCH("so3_logpost_fwd_wave_k");
  }
  LV_LAUNCH1(so3_logpost_fwd_k, n, v, sigma, out, ns, B, k);
}
int lv_so3_log_posterior_bwd(const float* v, const float* sigma, const float* gout, float* gv,
                             float* gsigma, int64_t ns, int64_t B, int k, void* stream) {
  const int64_t n = B;
  LV_CHECK_ARG(ns >= 0 && B >= 0, "bad sizes");
  LV_CHECK_ARG(k >= 0 && k <= kMaxWrap, "k must be in [0, %d]", kMaxWrap);
  LV_PTRS(v && sigma && gout && gv && gsigma);
  if (ns == 0) {
    (void)hipMemsetAsync(gsigma, 0, sizeof(float) * 3 * B, (hipStream_t)stream);
    return LV_OK;
  }
  if (n > 0 && k <= kWaveMaxK && n <= kWaveMaxElems) {
    clear_error();
    hipLaunchKernelGGL(so3_logpost_bwd_wave_k, grid_for_waves(n), dim3(kBlock), 0,
                       (hipStream_t)stream, v, sigma, gout, gv, gsigma, ns, B, k);
    LV_RETURN_LAUNCH("so3_logpost_bwd_wave_k");
  }
  LV_LAUNCH1(so3_logpost_bwd_k, n, v, sigma, gout, gv, gsigma, ns, B, k);
}

}  // extern "C"

// Microbenchmark: the group-action backward chain (P1..P4 recompute, Q4..dF, three kdots,
// every degree 0..LT) per lane-item, one spectrum column per lane (float) vs two columns
// of the same sample per lane (float2: v_pk_fma_f32 / v_pk_mul_f32, J literals splat from
// SGPRs).  Operands come from LDS as in the persistent kernel; the figure is ns per
// (sample, column) item at 3 (float) / 2 (float2) waves per SIMD.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
//         -I lie-vae_amd/csrc tools/chain_pk.hip -o gpurun_out/chain_pk && gpurun_out/chain_pk
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "action_chain.h"

using namespace lv;
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <typename T> __device__ __forceinline__ T sp(float v) { return (T)v; }
template <typename T> __device__ __forceinline__ T vfma(T a, T b, T c) { return __builtin_elementwise_fma(a, b, c); }

template <int l>
struct MultS { float c[l + 1], s[l + 1]; };
template <int l, int A, int LT>
__device__ __forceinline__ MultS<l> mlds(const float* tj) {
  constexpr int TP = TrigLds<LT>::TP;
  MultS<l> m;
  sfor<(l + 4) / 4>([&](auto K) {
    constexpr int k4 = LV_CV(K);
    const f4 cv = *reinterpret_cast<const f4*>(tj + 2 * A * TP + 4 * k4);
    const f4 sv = *reinterpret_cast<const f4*>(tj + (2 * A + 1) * TP + 4 * k4);
    sfor<4>([&](auto I) {
      constexpr int f = 4 * k4 + LV_CV(I);
      if constexpr (f <= l) { m.c[f] = cv[LV_CV(I)]; m.s[f] = sv[LV_CV(I)]; }
    });
  });
  return m;
}
template <int l, bool TR, typename T>
__device__ __forceinline__ void xmT(const MultS<l>& m, const T (&x)[2 * l + 1], T (&y)[2 * l + 1]) {
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    const T a = x[i], b = x[2 * l - i];
    const T c = sp<T>(m.c[f]), s = sp<T>(m.s[f]);
    if constexpr (TR) { y[i] = vfma(c, a, -(s * b)); y[2 * l - i] = vfma(c, b, s * a); }
    else { y[i] = vfma(c, a, s * b); y[2 * l - i] = vfma(c, b, -(s * a)); }
  });
  y[l] = x[l];
}
template <int l, bool TR, typename T>
__device__ __forceinline__ void xm_memT(const MultS<l>& m, const float* x, int stride, T (&y)[2 * l + 1]) {
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    const T a = *reinterpret_cast<const T*>(x + i * stride), b = *reinterpret_cast<const T*>(x + (2 * l - i) * stride);
    const T c = sp<T>(m.c[f]), s = sp<T>(m.s[f]);
    if constexpr (TR) { y[i] = vfma(c, a, -(s * b)); y[2 * l - i] = vfma(c, b, s * a); }
    else { y[i] = vfma(c, a, s * b); y[2 * l - i] = vfma(c, b, -(s * a)); }
  });
  y[l] = *reinterpret_cast<const T*>(x + l * stride);
}
template <int l, typename T>
__device__ __forceinline__ T kdotT(const T (&av)[2 * l + 1], const T (&bv)[2 * l + 1]) {
  T acc = sp<T>(0.f);
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    const T t = vfma(av[i], bv[2 * l - i], -(av[2 * l - i] * bv[i]));
    acc = vfma(sp<T>((float)f), t, acc);
  });
  return acc;
}
template <int l, typename T>
__device__ __forceinline__ void jmulT(const T (&x)[2 * l + 1], T (&y)[2 * l + 1]) {
  constexpr int n = 2 * l + 1;
  constexpr const float* J = lv_j::jtab<l>();
  sfor<n>([&](auto P) {
    constexpr int p = LV_CV(P);
    T acc = sp<T>(0.f);
    bool first = true;
    sfor<n>([&](auto K) {
      constexpr int k = LV_CV(K);
      constexpr float v = J[p * n + k];
      if constexpr (v != 0.f) {
        if (first) acc = sp<T>(v) * x[k];
        else acc = vfma(sp<T>(v), x[k], acc);
        first = false;
      }
    });
    y[p] = acc;
  });
}


// ---- pair layout (one column per lane): x as (x_i, x_{2l-i}) pairs + the middle element;
// X products as v_pk_mul_f32 + v_pk_fma_f32 with the multiples taken from their LDS
// vectors by op_sel (no register moves), J products and kdots on the halves.
template <int l>
struct VP { f2 p[l > 0 ? l : 1]; float m; };
template <int l, int k>
__device__ __forceinline__ float vget(const VP<l>& v) {
  if constexpr (k < l) return v.p[k].x;
  else if constexpr (k > l) return v.p[2 * l - k].y;
  else return v.m;
}
template <int l, int k>
__device__ __forceinline__ void vset(VP<l>& v, float x) {
  if constexpr (k < l) v.p[k].x = x;
  else if constexpr (k > l) v.p[2 * l - k].y = x;
  else v.m = x;
}
template <int l>
struct MultP { f4 c[(l + 4) / 4], s[(l + 4) / 4]; };
template <int l, int A, int LT>
__device__ __forceinline__ MultP<l> mldsP(const float* tj) {
  constexpr int TP = TrigLds<LT>::TP;
  MultP<l> m;
  sfor<(l + 4) / 4>([&](auto K) {
    constexpr int k4 = LV_CV(K);
    m.c[k4] = *reinterpret_cast<const f4*>(tj + 2 * A * TP + 4 * k4);
    m.s[k4] = *reinterpret_cast<const f4*>(tj + (2 * A + 1) * TP + 4 * k4);
  });
  return m;
}
template <int f>
__device__ __forceinline__ f2 half_of(const f4& v) {
  if constexpr ((f & 3) < 2) return v.xy; else return v.zw;
}
// (y_i, y_{2l-i}) = (c a + s b, c b - s a)  [TR: (c a - s b, c b + s a)], (a, b) = x pair i
template <int f, bool TR>
__device__ __forceinline__ f2 xpair(f2 cp, f2 sp, f2 x) {
  f2 prod, y;
  if constexpr (f & 1) {
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(prod) : "v"(sp), "v"(x));
    if constexpr (TR) asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,1] neg_lo:[0,0,1]" : "=v"(y) : "v"(cp), "v"(x), "v"(prod));
    else asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,1] neg_hi:[0,0,1]" : "=v"(y) : "v"(cp), "v"(x), "v"(prod));
  } else {
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,0]" : "=v"(prod) : "v"(sp), "v"(x));
    if constexpr (TR) asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[0,1,1] neg_lo:[0,0,1]" : "=v"(y) : "v"(cp), "v"(x), "v"(prod));
    else asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[0,1,1] neg_hi:[0,0,1]" : "=v"(y) : "v"(cp), "v"(x), "v"(prod));
  }
  return y;
}
template <int l, bool TR>
__device__ __forceinline__ void xmP(const MultP<l>& m, const VP<l>& x, VP<l>& y) {
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    y.p[i] = xpair<f, TR>(half_of<f>(m.c[f / 4]), half_of<f>(m.s[f / 4]), x.p[i]);
  });
  y.m = x.m;
}
template <int l, bool TR>
__device__ __forceinline__ void xm_memP(const MultP<l>& m, const float* x, int stride, VP<l>& y) {
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    const f2 ab = {x[i * stride], x[(2 * l - i) * stride]};
    y.p[i] = xpair<f, TR>(half_of<f>(m.c[f / 4]), half_of<f>(m.s[f / 4]), ab);
  });
  y.m = x[l * stride];
}
template <int l>
__device__ __forceinline__ float kdotP(const VP<l>& a, const VP<l>& b) {
  float acc = 0.f;
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    const float t = fmaf(a.p[i].x, b.p[i].y, -(a.p[i].y * b.p[i].x));
    acc = fmaf((float)f, t, acc);
  });
  return acc;
}
template <int l>
__device__ __forceinline__ void jmulP(const VP<l>& x, VP<l>& y) {
  constexpr int n = 2 * l + 1;
  constexpr const float* J = lv_j::jtab<l>();
  sfor<n>([&](auto P) {
    constexpr int p = LV_CV(P);
    float acc = 0.f;
    bool first = true;
    sfor<n>([&](auto K) {
      constexpr int k = LV_CV(K);
      constexpr float v = J[p * n + k];
      if constexpr (v != 0.f) {
        if (first) acc = v * vget<l, k>(x);
        else acc = fmaf(v, vget<l, k>(x), acc);
        first = false;
      }
    });
    vset<l, p>(y, acc);
  });
}

constexpr int LT = 10, C = 10, MC = (LT + 1) * (LT + 1) * C;
constexpr int kRow = TrigLds<LT>::kRow;

// W = 1: lane = (sample j < 6, column c); W = 2: lane = (sample j < 12, columns 2cp, 2cp+1)
template <int W, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
void chain_kernel(const float* gtrig, const float* gF, const float* gtile, float* out, int reps, unsigned dmask) {
  typedef typename std::conditional<W == 1, float, f2>::type T;
  constexpr int Sw = W == 1 ? 6 : 12, CL = C / W;
  __shared__ __attribute__((aligned(16))) float trig[12 * kRow];
  __shared__ __attribute__((aligned(16))) float Fs[MC];
  __shared__ __attribute__((aligned(16))) float tile[4][MC];  // one sample's tile per wave (synthetic)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < 12 * kRow; e += 256) trig[e] = gtrig[e];
  for (int e = tid; e < MC; e += 256) Fs[e] = gF[e];
  for (int e = tid; e < 4 * MC; e += 256) (&tile[0][0])[e] = gtile[e % MC];
  __syncthreads();
  const int j = min(lane / CL, Sw - 1), c = (lane % CL) * W;
  const float* tj = trig + j * kRow;
  const float* Fl = Fs + c;
  float* tl = &tile[wave][0] + c;
  T ga = sp<T>(0.f), gb = ga, gc = ga;
  for (int r = 0; r < reps; ++r) {
    // opaque pointers: keep the LDS operand reads inside the repetition (no hoisting)
    asm volatile("" : "+v"(tj), "+v"(Fl), "+v"(tl));
    sfor<LT + 1>([&](auto Lc) {
      constexpr int l = LT - LV_CV(Lc);
      constexpr int nn = 2 * l + 1, r0 = l * l;
      if (!((dmask >> l) & 1u)) return;  // run-time degree set (one basic block per degree)
      T p2[nn], p4[nn], u[nn];
      xm_memT<l, false>(mlds<l, 2, LT>(tj), Fl + r0 * C, C, u);
      jmulT<l>(u, p2);
      xmT<l, false>(mlds<l, 1, LT>(tj), p2, u);
      jmulT<l>(u, p4);
      xm_memT<l, true>(mlds<l, 0, LT>(tj), tl + r0 * C, C, u);
      ga += kdotT<l>(u, p4);
      jmulT<l>(u, p4);
      xmT<l, true>(mlds<l, 1, LT>(tj), p4, u);
      gb += kdotT<l>(u, p2);
      jmulT<l>(u, p2);
      xmT<l, true>(mlds<l, 2, LT>(tj), p2, u);
      gc += kdotT<l>(u, p2);
      if (lane < 60) sfor<nn>([&](auto I) { *reinterpret_cast<T*>(tl + (r0 + LV_CV(I)) * C) = u[LV_CV(I)]; });
    });
  }
  T s = ga + gb + gc;
  float v;
  if constexpr (W == 1) v = s; else v = s.x + s.y;
  out[blockIdx.x * 256 + tid] = v;
}


template <int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
void chainP_kernel(const float* gtrig, const float* gF, const float* gtile, float* out, int reps, unsigned dmask) {
  constexpr int Sw = 6;
  __shared__ __attribute__((aligned(16))) float trig[12 * kRow];
  __shared__ __attribute__((aligned(16))) float Fs[MC];
  __shared__ __attribute__((aligned(16))) float tile[4][MC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < 12 * kRow; e += 256) trig[e] = gtrig[e];
  for (int e = tid; e < MC; e += 256) Fs[e] = gF[e];
  for (int e = tid; e < 4 * MC; e += 256) (&tile[0][0])[e] = gtile[e % MC];
  __syncthreads();
  const int j = min(lane / C, Sw - 1), c = lane % C;
  const float* tj = trig + j * kRow;
  const float* Fl = Fs + c;
  float* tl = &tile[wave][0] + c;
  float ga = 0.f, gb = 0.f, gc = 0.f;
  for (int r = 0; r < reps; ++r) {
    asm volatile("" : "+v"(tj), "+v"(Fl), "+v"(tl));
    sfor<LT + 1>([&](auto Lc) {
      constexpr int l = LT - LV_CV(Lc);
      constexpr int r0 = l * l;
      if (!((dmask >> l) & 1u)) return;
      if constexpr (l == 0) {
        const float u = tl[0];
        if (lane < 60) tl[0] = u * Fl[0];
      } else {
        VP<l> p2, p4, u;
        xm_memP<l, false>(mldsP<l, 2, LT>(tj), Fl + r0 * C, C, u);
        jmulP<l>(u, p2);
        xmP<l, false>(mldsP<l, 1, LT>(tj), p2, u);
        jmulP<l>(u, p4);
        xm_memP<l, true>(mldsP<l, 0, LT>(tj), tl + r0 * C, C, u);
        ga += kdotP<l>(u, p4);
        jmulP<l>(u, p4);
        xmP<l, true>(mldsP<l, 1, LT>(tj), p4, u);
        gb += kdotP<l>(u, p2);
        jmulP<l>(u, p2);
        xmP<l, true>(mldsP<l, 2, LT>(tj), p2, u);
        gc += kdotP<l>(u, p2);
        if (lane < 60) sfor<2 * l + 1>([&](auto I) { tl[(r0 + LV_CV(I)) * C] = vget<l, LV_CV(I)>(u); });
      }
    });
  }
  out[blockIdx.x * 256 + tid] = ga + gb + gc;
}

// ---- forward chain (X(c) F -> J -> X(b) -> J -> X(a)), degrees 0..20, 8 waves per block at
// 2 blocks per CU (config 5's shape); scalar vs pair layout with the sines stored as
// interleaved (s, -s) pairs so that each X pair is v_pk_mul_f32 + v_pk_fma_f32 from
// compiler intrinsics (op_sel folds the swap and the cosine splat).
constexpr int LT2 = 20, MC2 = (LT2 + 1) * (LT2 + 1) * C;
constexpr int TP2 = TrigLds<LT2>::TP;
constexpr int kRowS = 6 * TP2 + 4, kRowP = 9 * TP2 + 4;

template <int l, int A>
__device__ __forceinline__ void xrotS(const float* tj, const float (&x)[2 * l + 1], float (&y)[2 * l + 1]) {
  float cc[l + 1], ss[l + 1];
  sfor<(l + 4) / 4>([&](auto K) {
    constexpr int k4 = LV_CV(K);
    const f4 cv = *reinterpret_cast<const f4*>(tj + 2 * A * TP2 + 4 * k4);
    const f4 sv = *reinterpret_cast<const f4*>(tj + (2 * A + 1) * TP2 + 4 * k4);
    sfor<4>([&](auto I) {
      constexpr int f = 4 * k4 + LV_CV(I);
      if constexpr (f <= l) { cc[f] = cv[LV_CV(I)]; ss[f] = sv[LV_CV(I)]; }
    });
  });
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    y[i] = fmaf(cc[f], x[i], ss[f] * x[2 * l - i]);
    y[2 * l - i] = fmaf(cc[f], x[2 * l - i], -(ss[f] * x[i]));
  });
  y[l] = x[l];
}
// pair layout: slot A's cosines at 3*A*TP, its (s, -s) pairs at 3*A*TP + TP
template <int l, int A>
__device__ __forceinline__ void xrotP2(const float* tj, const VP<l>& x, VP<l>& y) {
  f4 cv[(l + 4) / 4];
  f4 sn[(2 * l + 5) / 4];
  sfor<(l + 4) / 4>([&](auto K) { cv[LV_CV(K)] = *reinterpret_cast<const f4*>(tj + 3 * A * TP2 + 4 * LV_CV(K)); });
  sfor<(2 * l + 5) / 4>([&](auto K) { sn[LV_CV(K)] = *reinterpret_cast<const f4*>(tj + 3 * A * TP2 + TP2 + 4 * LV_CV(K)); });
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    const float c = cv[f / 4][f % 4];
    const f4 s4 = sn[(2 * f) / 4];
    const f2 sp = (f & 1) ? s4.zw : s4.xy;
    const f2 sw = __builtin_shufflevector(x.p[i], x.p[i], 1, 0);
    y.p[i] = __builtin_elementwise_fma((f2)(c), x.p[i], sp * sw);
  });
  y.m = x.m;
}

template <bool PAIR>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
void fwd_kernel(const float* gtrig, const float* gF, float* out, int reps, unsigned dmask) {
  constexpr int kRow = PAIR ? kRowP : kRowS;
  __shared__ __attribute__((aligned(16))) float trig[6 * kRowP];
  __shared__ __attribute__((aligned(16))) float Fs[MC2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < 6 * kRowP; e += 512) trig[e] = gtrig[e % 64];
  for (int e = tid; e < MC2; e += 512) Fs[e] = gF[e % MC];
  __syncthreads();
  const int j = min(lane / C, 5), c = lane % C;
  const float* tj = trig + j * kRow;
  const float* Fl = Fs + c;
  float acc = 0.f;
  // degrees spread over the 8 waves by cost: wave w takes l with (l * 7) % 8 == w (a fixed mix)
  const unsigned wm = dmask & [&] { unsigned m = 0; for (int l = 0; l <= LT2; ++l) if ((l * 5 + l / 8) % 8 == wave) m |= 1u << l; return m; }();
  for (int r = 0; r < reps; ++r) {
    asm volatile("" : "+v"(tj), "+v"(Fl));
    sfor<LT2 + 1>([&](auto Lc) {
      constexpr int l = LV_CV(Lc);
      constexpr int nn = 2 * l + 1, r0 = l * l;
      if (!((wm >> l) & 1u)) return;
      if constexpr (l == 0) {
        acc += Fl[0];
      } else if constexpr (PAIR) {
        VP<l> x, y;
        sfor<l>([&](auto I) { x.p[LV_CV(I)] = f2{Fl[(r0 + LV_CV(I)) * C], Fl[(r0 + 2 * l - LV_CV(I)) * C]}; });
        x.m = Fl[(r0 + l) * C];
        xrotP2<l, 2>(tj, x, y);
        jmulP<l>(y, x);
        xrotP2<l, 1>(tj, x, y);
        jmulP<l>(y, x);
        xrotP2<l, 0>(tj, x, y);
        float sacc = y.m;
        sfor<l>([&](auto I) { sacc += y.p[LV_CV(I)].x * y.p[LV_CV(I)].y; });
        acc += sacc;
      } else {
        float x[nn], y[nn];
        sfor<nn>([&](auto K) { x[LV_CV(K)] = Fl[(r0 + LV_CV(K)) * C]; });
        xrotS<l, 2>(tj, x, y);
        jmul<l>(y, x);
        xrotS<l, 1>(tj, x, y);
        jmul<l>(y, x);
        xrotS<l, 0>(tj, x, y);
        float sacc = y[l];
        sfor<l>([&](auto I) { sacc += y[LV_CV(I)] * y[2 * l - LV_CV(I)]; });
        acc += sacc;
      }
    });
  }
  out[blockIdx.x * 512 + tid] = acc;
}

int main() {
  std::vector<float> trig(12 * kRow), F(MC), tile(MC);
  for (size_t i = 0; i < trig.size(); ++i) trig[i] = 0.1f + 0.01f * (float)(i % 29);
  for (size_t i = 0; i < F.size(); ++i) F[i] = 0.001f * (i % 17), tile[i] = 0.002f * (i % 13);
  float *dt, *dF, *dtile, *dout;
  const int blocks = 256 * 3;
  hipMalloc(&dt, trig.size() * 4); hipMalloc(&dF, MC * 4); hipMalloc(&dtile, MC * 4);
  hipMalloc(&dout, blocks * 256 * 4);
  hipMemcpy(dt, trig.data(), trig.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dF, F.data(), MC * 4, hipMemcpyHostToDevice);
  hipMemcpy(dtile, tile.data(), MC * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int reps = 40;
  auto run = [&](auto kern, int nblk, int items_per_block, const char* name) {
    for (int w = 0; w < 3; ++w) kern<<<nblk, 256>>>(dt, dF, dtile, dout, reps, 0x7ffu);
    hipEventRecord(e0);
    for (int it = 0; it < 10; ++it) kern<<<nblk, 256>>>(dt, dF, dtile, dout, reps, 0x7ffu);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double items = (double)nblk * items_per_block * reps * 10;
    printf("%-28s blocks %4d  %.3f ms  %.4f ns per (sample,column) item\n", name, nblk, ms / 10, ms * 1e6 / items);
  };
  run(chain_kernel<1, 3>, 768, 240, "float  (1 col/lane, 3 w/SIMD)");
  run(chain_kernel<1, 2>, 512, 240, "float  (1 col/lane, 2 w/SIMD)");
  run(chain_kernel<2, 2>, 512, 480, "float2 (2 col/lane, 2 w/SIMD)");
  run(chain_kernel<2, 3>, 768, 480, "float2 (2 col/lane, 3 w/SIMD)");
  run(chain_kernel<2, 1>, 256, 480, "float2 (2 col/lane, 1 w/SIMD)");
  run(chainP_kernel<3>, 768, 240, "pairs  (1 col/lane, 3 w/SIMD)");
  run(chainP_kernel<2>, 512, 240, "pairs  (1 col/lane, 2 w/SIMD)");
  run(chain_kernel<1, 2>, 512, 240, "float  (1 col/lane, 2 w/SIMD)");
  run(chain_kernel<1, 3>, 768, 240, "float  (1 col/lane, 3 w/SIMD)");
  run(chain_kernel<2, 2>, 512, 480, "float2 (2 col/lane, 2 w/SIMD)");
  {
    float* dout2;
    hipMalloc(&dout2, 512 * 512 * 4);
    auto runf = [&](auto kern, const char* name) {
      for (int w = 0; w < 3; ++w) kern<<<512, 512>>>(dt, dF, dout2, reps, 0x1fffffu);
      hipEventRecord(e0);
      for (int it = 0; it < 10; ++it) kern<<<512, 512>>>(dt, dF, dout2, reps, 0x1fffffu);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%-28s %.3f ms per launch (512 blocks x 8 waves, l <= 20)\n", name, ms / 10);
    };
    runf(fwd_kernel<false>, "fwd scalar");
    runf(fwd_kernel<true>, "fwd pairs (s,-s)");
    runf(fwd_kernel<false>, "fwd scalar");
    runf(fwd_kernel<true>, "fwd pairs (s,-s)");
  }
  // pair layout vs one column per lane: same operations, bitwise equal sums
  std::vector<float> o1(512 * 256), o2(512 * 256);
  chain_kernel<1, 2><<<512, 256>>>(dt, dF, dtile, dout, 3, 0x7feu);
  hipMemcpy(o1.data(), dout, o1.size() * 4, hipMemcpyDeviceToHost);
  chainP_kernel<2><<<512, 256>>>(dt, dF, dtile, dout, 3, 0x7feu);
  hipMemcpy(o2.data(), dout, o2.size() * 4, hipMemcpyDeviceToHost);
  int ndiff = 0;
  for (size_t i = 0; i < o1.size(); ++i) ndiff += o1[i] != o2[i];
  printf("pair layout vs scalar: %d of %zu sums differ (o1[0]=%g o2[0]=%g)\n", ndiff, o1.size(), o1[0], o2[0]);
  printf("err %d\n", (int)hipGetLastError());
  return 0;
}

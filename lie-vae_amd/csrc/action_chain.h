// The per-degree factored Wigner chain shared by the forward and backward kernels.
//
// The reference evaluates D_l = X(a)·J·X(b)·J·X(c) as four dense bmm's per degree and
// then D_l·F (lie_tools.py:211-253).  Here one lane owns one column c of one sample's
// spectrum block and applies the factors right-to-left to that column, never forming D:
//
//   y = X(a) · J · X(b) · J · X(c) · F[:, c]
//
// X(θ) has two non-zeros per row (cos on the diagonal, sin on the anti-diagonal,
// frequency l-i for row i, lie_tools.py:195-208) and J_l is a compile-time constant
// table (~1/4 dense), so each product is a short chain of register FMAs with literal
// coefficients: ~2·nnz(J_l) + 6(2l+1) FLOP-pairs per column instead of the reference's
// 8(2l+1)^3 + 2(2l+1)^2·C per sample.
#pragma once
#include "j_tables.h"
#include "lv_common.h"

#define LV_CV(x) decltype(x)::value

namespace lv {

// cos/sin of f·angle for the three Euler slots (0 = a, 1 = b, 2 = c), f = 0..LT.
template <int LT>
struct TrigTab {
  float c[3][LT + 1];
  float s[3][LT + 1];
};

// Fill multiples by the rotation recurrence from exact (cos, sin) of each angle.
// Error grows ~f·ulp: at f = 20 it is below the reference's own fp32 sin(f·θ) error.
template <int LT>
__device__ __forceinline__ void trig_fill(TrigTab<LT>& t, const float c1[3], const float s1[3],
                                          int upto) {
  sfor<3>([&](auto A) {
    constexpr int a = LV_CV(A);
    t.c[a][0] = 1.f;
    t.s[a][0] = 0.f;
    if constexpr (LT >= 1) {
      t.c[a][1] = c1[a];
      t.s[a][1] = s1[a];
    }
    sfor<LT + 1>([&](auto F) {
      constexpr int f = LV_CV(F);
      if constexpr (f >= 2) {
        if (f <= upto) {
          t.c[a][f] = fmaf(t.c[a][f - 1], c1[a], -(t.s[a][f - 1] * s1[a]));
          t.s[a][f] = fmaf(t.s[a][f - 1], c1[a], t.c[a][f - 1] * s1[a]);
        }
      }
    });
  });
}

// y = X_l(θ_A) x      (row i: cos(fθ) x_i + sin(fθ) x_{2l-i}, f = l - i)
template <int l, int A, int LT>
__device__ __forceinline__ void xrot(const TrigTab<LT>& t, const float (&x)[2 * l + 1],
                                     float (&y)[2 * l + 1]) {
  sfor<2 * l + 1>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    if constexpr (f == 0) {
      y[i] = x[i];
    } else if constexpr (f > 0) {
      y[i] = fmaf(t.c[A][f], x[i], t.s[A][f] * x[2 * l - i]);
    } else {
      y[i] = fmaf(t.c[A][-f], x[i], -(t.s[A][-f] * x[2 * l - i]));
    }
  });
}

// The same multiples kept in LDS instead of registers (the register table is 6(l+1)
// VGPRs).  Row of one sample: [2A][f] = cos(f θ_A), [2A+1][f] = sin(f θ_A),
// f = 0..TP-1 (TP a multiple of 4: 16-byte aligned reads); kRow floats per sample
// (padded so the samples of a wave fall in different LDS banks).
template <int LT>
struct TrigLds {
  static constexpr int TP = (LT + 1 + 3) & ~3;
  static constexpr int kRow = 6 * TP + 4;
};
// Run-time twin of TrigLds<L>::kRow (host launch planning).
__host__ __device__ constexpr int trig_row_floats(int L) { return 6 * ((L + 1 + 3) & ~3) + 4; }
static_assert(trig_row_floats(10) == TrigLds<10>::kRow && trig_row_floats(20) == TrigLds<20>::kRow,
              "trig row layout");

// Write slot q's multiples f = 0..upto (trig_fill's recurrence, same rounding).
template <int LT>
__device__ __forceinline__ void trig_row_fill(float* tj, const float c1[3], const float s1[3],
                                              int q, int upto) {
  constexpr int TP = TrigLds<LT>::TP;
  const float cq = q == 0 ? c1[0] : (q == 1 ? c1[1] : c1[2]);
  const float sq = q == 0 ? s1[0] : (q == 1 ? s1[1] : s1[2]);
  float* tc = tj + 2 * q * TP;
  float* ts = tc + TP;
  tc[0] = 1.f;
  ts[0] = 0.f;
  float cf = cq, sf = sq;
  sfor<LT + 1>([&](auto F) {
    constexpr int f = LV_CV(F);
    if constexpr (f >= 1) {
      if (f <= upto) {
        if constexpr (f >= 2) {
          const float cn = fmaf(cf, cq, -(sf * sq));
          sf = fmaf(sf, cq, cf * sq);
          cf = cn;
        }
        tc[f] = cf;
        ts[f] = sf;
      }
    }
  });
}

// The same for one slot whose (cos, sin) the caller already picked (bitwise equal).  The
// row is written with 16-byte LDS stores once the recurrence is done (entries past `upto`
// and up to TP - 1 are zero): 2 * TP / 4 stores instead of 2 * (upto + 1) scalar ones on
// the prologue's critical path.
template <int LT>
__device__ __forceinline__ void trig_row_fill1(float* tj, float cq, float sq, int q, int upto) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int TP = TrigLds<LT>::TP;
  float cv[TP], sv[TP];
  cv[0] = 1.f;
  sv[0] = 0.f;
  float cf = cq, sf = sq;
  sfor<TP>([&](auto F) {
    constexpr int f = LV_CV(F);
    if constexpr (f >= 1) {
      if (f <= LT && f <= upto) {
        if constexpr (f >= 2) {
          const float cn = fmaf(cf, cq, -(sf * sq));
          sf = fmaf(sf, cq, cf * sq);
          cf = cn;
        }
        cv[f] = cf;
        sv[f] = sf;
      } else {
        cv[f] = 0.f;
        sv[f] = 0.f;
      }
    }
  });
  f4* tc = reinterpret_cast<f4*>(tj + 2 * q * TP);
  f4* ts = reinterpret_cast<f4*>(tj + (2 * q + 1) * TP);
  sfor<TP / 4>([&](auto K) {
    constexpr int k = LV_CV(K);
    tc[k] = f4{cv[4 * k], cv[4 * k + 1], cv[4 * k + 2], cv[4 * k + 3]};
    ts[k] = f4{sv[4 * k], sv[4 * k + 1], sv[4 * k + 2], sv[4 * k + 3]};
  });
}

// y = X_l(θ_A) x with the multiples read from an LDS row (bitwise equal to xrot): the
// l+1 needed (cos, sin) pairs are fetched with 16-byte reads right before the product,
// so they occupy registers only while it runs.
template <int l, int A, int LT>
__device__ __forceinline__ void xrot_lds(const float* tj, const float (&x)[2 * l + 1],
                                         float (&y)[2 * l + 1]) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int TP = TrigLds<LT>::TP;
  float cc[l + 1], ss[l + 1];
  sfor<(l + 4) / 4>([&](auto K) {
    constexpr int k4 = LV_CV(K);
    const f4 cv = *reinterpret_cast<const f4*>(tj + 2 * A * TP + 4 * k4);
    const f4 sv = *reinterpret_cast<const f4*>(tj + (2 * A + 1) * TP + 4 * k4);
    sfor<4>([&](auto I) {
      constexpr int f = 4 * k4 + LV_CV(I);
      if constexpr (f <= l) {
        cc[f] = cv[LV_CV(I)];
        ss[f] = sv[LV_CV(I)];
      }
    });
  });
  sfor<2 * l + 1>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    if constexpr (f == 0) {
      y[i] = x[i];
    } else if constexpr (f > 0) {
      y[i] = fmaf(cc[f], x[i], ss[f] * x[2 * l - i]);
    } else {
      y[i] = fmaf(cc[-f], x[i], -(ss[-f] * x[2 * l - i]));
    }
  });
}

// y = X_l(θ_A)^T x = X_l(-θ_A) x
template <int l, int A, int LT>
__device__ __forceinline__ void xrot_t(const TrigTab<LT>& t, const float (&x)[2 * l + 1],
                                       float (&y)[2 * l + 1]) {
  sfor<2 * l + 1>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    if constexpr (f == 0) {
      y[i] = x[i];
    } else if constexpr (f > 0) {
      y[i] = fmaf(t.c[A][f], x[i], -(t.s[A][f] * x[2 * l - i]));
    } else {
      y[i] = fmaf(t.c[A][-f], x[i], t.s[A][-f] * x[2 * l - i]);
    }
  });
}

// <g, dX_l(θ_A)/dθ · x>: row i of dX/dθ is (-f sin(fθ) at i, f cos(fθ) at 2l-i).
template <int l, int A, int LT>
__device__ __forceinline__ float xrot_dot_deriv(const TrigTab<LT>& t, const float (&g)[2 * l + 1],
                                                const float (&x)[2 * l + 1]) {
  float acc = 0.f;
  sfor<2 * l + 1>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    if constexpr (f > 0) {
      const float d = fmaf(-t.s[A][f], x[i], t.c[A][f] * x[2 * l - i]);
      acc = fmaf(g[i], (float)f * d, acc);
    } else if constexpr (f < 0) {
      // sin(fθ) = -sin(|f|θ), cos(fθ) = cos(|f|θ)
      const float d = fmaf(t.s[A][-f], x[i], t.c[A][-f] * x[2 * l - i]);
      acc = fmaf(g[i], (float)f * d, acc);
    }
  });
  return acc;
}

// y = J_l x with J_l's non-zeros as literal coefficients (J is symmetric: J^T = J).
#ifndef LV_JMUL_MUL
#define LV_JMUL_MUL 1
#endif
template <int l>
__device__ __forceinline__ void jmul(const float (&x)[2 * l + 1], float (&y)[2 * l + 1]) {
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
        // LV_JMUL_MUL: the row's first term as a multiply (v_mul_f32 takes the literal;
        // fma(v, x, 0) needs it in an SGPR, one s_mov per row) -- equal except for the
        // sign of an all-zero row's result
        if (LV_JMUL_MUL && first) acc = v * x[k];
        else acc = fmaf(v, x[k], acc);
        first = false;
      }
    });
    y[p] = acc;
  });
}

// Number of structural non-zeros of J_l (host-side cost model).
template <int l>
constexpr int j_nnz() {
  constexpr int n = 2 * l + 1;
  constexpr const float* J = lv_j::jtab<l>();
  int c = 0;
  for (int i = 0; i < n * n; ++i) c += (J[i] != 0.f);
  return c;
}

// Make this wave's LDS writes visible to its own later reads (cross-lane, same wave).
// Only LDS is waited for: a workgroup-scope release fence would also emit
// s_waitcnt vmcnt(0) and stall on every global store still in flight.  The "memory"
// clobber keeps the compiler from moving LDS or global accesses across this point.
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

}  // namespace lv

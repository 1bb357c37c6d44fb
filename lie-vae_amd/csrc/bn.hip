// Encoder BatchNorm2d + LeakyReLU on channels-last bf16 activations: the
// ConvNetBN stack (reference nets.py:33-57) follows every strided conv with
// BatchNorm2d(width) and LeakyReLU(0.2).  PyTorch's channels-last kernels for these four
// layers took ~1.1 ms of the 6.7 ms config-3 bf16 step at 0.2-0.5 TB/s
// (profiles/r03_train_config3_bf16_mfma_steady_kernels.txt); the layers are pure HBM
// streams, so the floor is the bytes: 3 passes forward (stats read, apply read + write)
// and 5 backward (reduce reads g, x; apply reads g, x, writes gx).
//
// Layout.  x is a flat (P, C) bf16 array (P = N·H·W pixels, channels innermost), read as
// 16-byte vectors of 8 elements.  The channel of element j of vector v is (8v + j) mod C,
// which repeats every T = C / gcd(C, 8) vectors.  The reductions give thread (rho, phi) of
// a block the vectors g·T + phi of the period groups g = rho, rho + R, ... (R = 256 / T),
// so each of its 8 accumulators stays on ONE channel; the block then folds its R x 8T
// accumulators into per-channel sums in a fixed order, and a second kernel adds the
// per-block partials in block order -- deterministic, no atomics.  Statistics are
// accumulated around a per-channel shift (x of pixel 0) so E[(x-K)^2] - E[x-K]^2 does not
// cancel.  The elementwise kernels walk the vectors grid-stride with a running channel
// offset and keep the per-channel coefficients in LDS.
//
// Semantics follow torch.nn.BatchNorm2d (training: biased variance normalises, the
// running variance takes the unbiased one, running = (1 - m)·running + m·batch) and
// torch.nn.LeakyReLU: y = z if z > 0 else slope·z, gz = g if z > 0 else slope·g.
#include <algorithm>

#include "lv_common.h"

namespace lv {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBnThreads = 256;
constexpr int kBnMaxBlocks = 512;

__device__ __forceinline__ void unpack8(const u32x4 v, float (&f)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = __uint_as_float(v[e] << 16);
    f[2 * e + 1] = __uint_as_float(v[e] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float (&f)[8]) {
  u32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const unsigned lo = __bfloat16_as_ushort(__float2bfloat16(f[2 * e]));
    const unsigned hi = __bfloat16_as_ushort(__float2bfloat16(f[2 * e + 1]));
    v[e] = lo | (hi << 16);
  }
  return v;
}

struct BnGeom {
  int C, T, R;           // channels, vectors per period, periods per block pass
  int64_t groups;        // period groups in the tensor
  int64_t per_blk;       // groups per reduction block
  int nblk;              // reduction blocks
};

// Per-block partial sums of the two per-channel quantities of a reduction.
//   MODE 0 (forward statistics): s1 = x - K, s2 = (x - K)^2, K = x[0, c]
//   MODE 1 (backward):           s1 = gz,    s2 = gz · xhat,  gz = g·(z > 0 ? 1 : slope)
// coef (MODE 1): [a | b | mean | invstd] per channel, z = a x + b, xhat = (x - mean) invstd
template <int MODE>
__global__ __launch_bounds__(kBnThreads) void bn_reduce_part_kernel(const __hip_bfloat16* x, const __hip_bfloat16* g,
                                                                    const float* coef, float slope, BnGeom geo,
                                                                    float* part) {
  __shared__ float red[2][kBnThreads * 8];
  const int tid = (int)threadIdx.x, C = geo.C, T = geo.T, R = geo.R;
  const int phi = tid % T, rho = tid / T;
  const bool active = rho < R;
  float s1[8], s2[8], k0[8], k1[8], k2[8], k3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s1[j] = s2[j] = 0.f;
    int c = (8 * phi + j) % C;
    if (MODE == 0) {
      k0[j] = __bfloat162float(x[c]);
    } else {
      k0[j] = coef[c];
      k1[j] = coef[C + c];
      k2[j] = coef[2 * C + c];
      k3[j] = coef[3 * C + c];
    }
  }
  if (active) {
    const int64_t g0 = (int64_t)blockIdx.x * geo.per_blk;
    const int64_t g1 = min(geo.groups, g0 + geo.per_blk);
    auto acc = [&](const u32x4 xv, const u32x4 gv) {
      float xf[8], gf[8];
      unpack8(xv, xf);
      if (MODE == 1) unpack8(gv, gf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (MODE == 0) {
          const float d = xf[j] - k0[j];
          s1[j] += d;
          s2[j] += d * d;
        } else {
          const float z = xf[j] * k0[j] + k1[j];
          const float gz = z > 0.f ? gf[j] : gf[j] * slope;
          s1[j] += gz;
          s2[j] += gz * ((xf[j] - k2[j]) * k3[j]);
        }
      }
    };
    int64_t gi = g0 + rho;
    for (; gi + 3 * R < g1; gi += 4 * R) {  // four vectors (per operand) in flight
      u32x4 xv[4], gv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t off = ((gi + u * R) * T + phi) * 8;
        xv[u] = *reinterpret_cast<const u32x4*>(x + off);
        if (MODE == 1) gv[u] = *reinterpret_cast<const u32x4*>(g + off);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc(xv[u], gv[u]);
    }
    for (; gi < g1; gi += R) {
      const int64_t off = (gi * T + phi) * 8;
      const u32x4 xv = *reinterpret_cast<const u32x4*>(x + off);
      u32x4 gv = xv;
      if (MODE == 1) gv = *reinterpret_cast<const u32x4*>(g + off);
      acc(xv, gv);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][rho * 8 * T + 8 * phi + j] = s1[j];
      red[1][rho * 8 * T + 8 * phi + j] = s2[j];
    }
  }
  __syncthreads();
  // channel c collects slot c + m·C (m < 8T / C) of every rho, in a fixed order
  const int reps = 8 * T / C;
  for (int c = tid; c < C; c += kBnThreads) {
    float t1 = 0.f, t2 = 0.f;
    for (int r = 0; r < R; ++r)
      for (int m = 0; m < reps; ++m) {
        t1 += red[0][r * 8 * T + c + m * C];
        t2 += red[1][r * 8 * T + c + m * C];
      }
    part[(int64_t)blockIdx.x * 2 * C + c] = t1;
    part[(int64_t)blockIdx.x * 2 * C + C + c] = t2;
  }
}

// Fixed-order sum of the block partials: 64 channels per block, 16 slices of blocks (slice sl
// takes blocks sl, sl + 16, ..., 4-way unrolled), the 16 slice sums added by a fixed
// halving tree, then the per-channel epilogue in slice 0.  (Round 3: 16 slices instead of 4
// -- the kernel runs on ceil(C / 64) blocks only, so its time is the partials' load latency.)
//   MODE 0: batch mean / biased var -> save_mean, save_invstd, running stats, coef = [a | b]
//   MODE 1: ggamma, gbeta and coef2 = [gamma·invstd | sum gz / P | sum gz·xhat / P]
constexpr int kBnFinSlices = 16;
template <int MODE>
__global__ __launch_bounds__(64 * kBnFinSlices) void bn_finalize_kernel(const float* part, int nblk, int C, int64_t P,
                                                          const __hip_bfloat16* x, const float* gamma,
                                                          const float* beta, float eps, float momentum,
                                                          float* running_mean, float* running_var, float* save_mean,
                                                          float* save_invstd, float* coef, float* ggamma,
                                                          float* gbeta) {
  constexpr int SL = kBnFinSlices;
  __shared__ float red[2][SL][64];
  const int t = (int)threadIdx.x, el = t & 63, sl = t >> 6;
  const int c = blockIdx.x * 64 + el;
  float a1[4] = {0.f, 0.f, 0.f, 0.f}, a2[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int b = sl;
    for (; b + 3 * SL < nblk; b += 4 * SL) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a1[u] += part[(int64_t)(b + SL * u) * 2 * C + c];
        a2[u] += part[(int64_t)(b + SL * u) * 2 * C + C + c];
      }
    }
    for (; b < nblk; b += SL) {
      a1[0] += part[(int64_t)b * 2 * C + c];
      a2[0] += part[(int64_t)b * 2 * C + C + c];
    }
  }
  red[0][sl][el] = (a1[0] + a1[1]) + (a1[2] + a1[3]);
  red[1][sl][el] = (a2[0] + a2[1]) + (a2[2] + a2[3]);
#pragma unroll
  for (int h = SL / 2; h >= 1; h >>= 1) {
    __syncthreads();
    if (sl < h) {
      red[0][sl][el] += red[0][sl + h][el];
      red[1][sl][el] += red[1][sl + h][el];
    }
  }
  __syncthreads();
  if (sl != 0 || c >= C) return;
  const float S1 = red[0][0][el];
  const float S2 = red[1][0][el];
  const float n = (float)P;
  const float gm = gamma ? gamma[c] : 1.f;
  if (MODE == 0) {
    const float md = S1 / n;
    const float var = fmaxf(S2 / n - md * md, 0.f);
    const float mean = __bfloat162float(x[c]) + md;
    const float invstd = 1.f / sqrtf(var + eps);
    save_mean[c] = mean;
    save_invstd[c] = invstd;
    const float a = gm * invstd;
    coef[c] = a;
    coef[C + c] = (beta ? beta[c] : 0.f) - mean * a;
    if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
    if (running_var) {
      const float unb = P > 1 ? var * n / (n - 1.f) : var;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
    }
  } else {
    if (ggamma) ggamma[c] = S2;
    if (gbeta) gbeta[c] = S1;
    coef[c] = gm * save_invstd[c];
    coef[C + c] = S1 / n;
    coef[2 * C + c] = S2 / n;
  }
}

// Elementwise passes over the 16-byte vectors (grid-stride, running channel offset).
//   MODE 0 (forward, training or eval): y = lrelu(a x + b)        tab = [a | b]
//   MODE 2 (backward): gx = k1 (gz - k2 - xhat k3)               tab = [a | b | mean | invstd | k1 | k2 | k3]
template <int MODE>
__global__ __launch_bounds__(kBnThreads) void bn_apply_kernel(const __hip_bfloat16* x, const __hip_bfloat16* g,
                                                              const float* tab, int ntab, float slope, int C,
                                                              int64_t nvec, __hip_bfloat16* out) {
  extern __shared__ float st[];   // [ntab][C]
  for (int i = threadIdx.x; i < ntab * C; i += kBnThreads) st[i] = tab[i];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kBnThreads;
  const int step = (int)((stride * 8) % C);
  int64_t v = (int64_t)blockIdx.x * kBnThreads + threadIdx.x;
  int c0 = (int)((v * 8) % C);
  for (; v < nvec; v += stride) {
    float xf[8], o[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + v * 8), xf);
    float gf[8];
    if (MODE == 2) unpack8(*reinterpret_cast<const u32x4*>(g + v * 8), gf);
    int c = c0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float z = xf[j] * st[c] + st[C + c];
      if (MODE == 2) {
        const float gz = z > 0.f ? gf[j] : gf[j] * slope;
        const float xh = (xf[j] - st[2 * C + c]) * st[3 * C + c];
        o[j] = st[4 * C + c] * (gz - st[5 * C + c] - xh * st[6 * C + c]);
      } else {
        o[j] = z > 0.f ? z : z * slope;
      }
      if (++c == C) c = 0;
    }
    *reinterpret_cast<u32x4*>(out + v * 8) = pack8(o);
    c0 += step;
    if (c0 >= C) c0 -= C;
  }
}

// eval-mode coefficients from the running statistics
__global__ void bn_eval_coef_kernel(const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                                    int C, float* coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float a = (gamma ? gamma[c] : 1.f) / sqrtf(rv[c] + eps);
  coef[c] = a;
  coef[C + c] = (beta ? beta[c] : 0.f) - rm[c] * a;
}

// bwd coefficient table [a | b | mean | invstd] for the reduce and apply passes
__global__ void bn_bwd_coef_kernel(const float* gamma, const float* beta, const float* mean, const float* invstd,
                                   int C, float* coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float a = (gamma ? gamma[c] : 1.f) * invstd[c];
  coef[c] = a;
  coef[C + c] = (beta ? beta[c] : 0.f) - mean[c] * a;
  coef[2 * C + c] = mean[c];
  coef[3 * C + c] = invstd[c];
}

int gcd_int(int a, int b) {
  while (b) {
    const int t = a % b;
    a = b;
    b = t;
  }
  return a;
}

bool bn_geom(int64_t P, int C, BnGeom* g) {
  if (C < 8 || P <= 0) return false;
  const int T = C / gcd_int(C, 8);
  if (T > kBnThreads) return false;
  const int64_t pix_per_group = 8 * (int64_t)T / C;
  if (P % pix_per_group) return false;
  g->C = C;
  g->T = T;
  g->R = kBnThreads / T;
  g->groups = P / pix_per_group;
  g->nblk = (int)std::min<int64_t>(kBnMaxBlocks, (g->groups + 4 * g->R - 1) / (4 * g->R));
  g->per_blk = (g->groups + g->nblk - 1) / g->nblk;
  g->nblk = (int)((g->groups + g->per_blk - 1) / g->per_blk);
  return true;
}

// acc[i] += g[i] (bf16 -> fp32): a parameter's bf16 gradient (the autocast copy's) added
// into its fp32 master gradient in one pass, 10 bytes per element.  The first `head` (< 4)
// elements are peeled so that acc + head is 16-byte aligned (gradient-bucket views start
// anywhere); the body moves 4 elements per lane: one 16-byte fp32 access and, by g's
// alignment there, one 8-byte (GA = 8), two 4-byte (GA = 4) or four 2-byte (GA = 2) reads.
__device__ __forceinline__ float bf16_bits_to_float(unsigned short b) { return __uint_as_float((unsigned)b << 16); }

template <int GA>
__global__ __launch_bounds__(256) void accumulate_bf16_f32_kernel(const __hip_bfloat16* __restrict__ g,
                                                                  float* __restrict__ acc, int64_t n, int head) {
  const unsigned short* gb = reinterpret_cast<const unsigned short*>(g);
  const int tid0 = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (blockIdx.x == 0 && (int)threadIdx.x < head && threadIdx.x < n)
    acc[threadIdx.x] += bf16_bits_to_float(gb[threadIdx.x]);
  const int64_t nv = (n - head) / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float4* a4 = reinterpret_cast<float4*>(acc + head);
  const unsigned short* gh = gb + head;
  for (int64_t i = tid0; i < nv; i += stride) {
    float x0, x1, x2, x3;
    if constexpr (GA == 8) {
      const uint2 v = reinterpret_cast<const uint2*>(gh)[i];
      x0 = __uint_as_float(v.x << 16), x1 = __uint_as_float(v.x & 0xffff0000u);
      x2 = __uint_as_float(v.y << 16), x3 = __uint_as_float(v.y & 0xffff0000u);
    } else if constexpr (GA == 4) {
      const unsigned v0 = reinterpret_cast<const unsigned*>(gh)[2 * i];
      const unsigned v1 = reinterpret_cast<const unsigned*>(gh)[2 * i + 1];
      x0 = __uint_as_float(v0 << 16), x1 = __uint_as_float(v0 & 0xffff0000u);
      x2 = __uint_as_float(v1 << 16), x3 = __uint_as_float(v1 & 0xffff0000u);
    } else {
      x0 = bf16_bits_to_float(gh[4 * i]), x1 = bf16_bits_to_float(gh[4 * i + 1]);
      x2 = bf16_bits_to_float(gh[4 * i + 2]), x3 = bf16_bits_to_float(gh[4 * i + 3]);
    }
    float4 a = a4[i];
    a.x += x0, a.y += x1, a.z += x2, a.w += x3;
    a4[i] = a;
  }
  const int64_t t = head + nv * 4 + tid0;  // the last (n - head) % 4 elements
  if (blockIdx.x == 0 && t < n) acc[t] += bf16_bits_to_float(gb[t]);
}

int apply_blocks(int64_t nvec) { return (int)std::max<int64_t>(1, std::min<int64_t>(2048, (nvec + kBnThreads - 1) / kBnThreads)); }

}  // namespace
}  // namespace lv

using namespace lv;

extern "C" {

int lv_accumulate_bf16_f32(const void* g, float* acc, int64_t n, void* stream) {
  clear_error();
  LV_CHECK_ARG(n >= 0, "n < 0");
  if (n == 0) return LV_OK;
  LV_CHECK_ARG(g && acc, "null pointer");
  LV_CHECK_ARG((reinterpret_cast<uintptr_t>(g) & 1) == 0 && (reinterpret_cast<uintptr_t>(acc) & 3) == 0,
               "misaligned element pointers");
  const int head = (int)std::min<int64_t>(n, ((16 - (reinterpret_cast<uintptr_t>(acc) & 15)) & 15) / 4);
  const uintptr_t gh = reinterpret_cast<uintptr_t>(g) + 2 * head;
  const int64_t units = (n - head) / 4;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(2048, (units + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  const __hip_bfloat16* gp = (const __hip_bfloat16*)g;
  if ((gh & 7) == 0)
    hipLaunchKernelGGL(accumulate_bf16_f32_kernel<8>, dim3(blocks), dim3(256), 0, st, gp, acc, n, head);
  else if ((gh & 3) == 0)
    hipLaunchKernelGGL(accumulate_bf16_f32_kernel<4>, dim3(blocks), dim3(256), 0, st, gp, acc, n, head);
  else
    hipLaunchKernelGGL(accumulate_bf16_f32_kernel<2>, dim3(blocks), dim3(256), 0, st, gp, acc, n, head);
  LV_RETURN_LAUNCH("accumulate_bf16_f32_kernel");
}

int lv_bn_supported(int64_t P, int C) {
  BnGeom g;
  return bn_geom(P, C, &g) ? 1 : 0;
}

size_t lv_bn_workspace_elems(int64_t P, int C) {
  BnGeom g;
  if (!bn_geom(P, C, &g)) return 0;
  return (size_t)g.nblk * 2 * C + 7 * (size_t)C;
}

int lv_bn_lrelu_fwd_bf16(const void* x, const float* gamma, const float* beta, float* running_mean,
                         float* running_var, int training, float momentum, float eps, float slope, void* y,
                         float* save_mean, float* save_invstd, float* ws, int64_t P, int C, void* stream) {
  clear_error();
  BnGeom geo;
  LV_CHECK_ARG(bn_geom(P, C, &geo), "unsupported shape P=%lld C=%d (lv_bn_supported)", (long long)P, C);
  LV_CHECK_ARG(x && y && ws, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  float* coef = ws + (size_t)geo.nblk * 2 * C;
  if (training) {
    LV_CHECK_ARG(save_mean && save_invstd, "training needs save_mean / save_invstd");
    hipLaunchKernelGGL(bn_reduce_part_kernel<0>, dim3(geo.nblk), dim3(kBnThreads), 0, st, (const __hip_bfloat16*)x,
                       (const __hip_bfloat16*)nullptr, (const float*)nullptr, slope, geo, ws);
    LV_CHECK_LAUNCH("bn_reduce_part_kernel<0>");
    hipLaunchKernelGGL(bn_finalize_kernel<0>, dim3(ceil_div(C, 64)), dim3(64 * kBnFinSlices), 0, st, ws, geo.nblk, C, P,
                       (const __hip_bfloat16*)x, gamma, beta, eps, momentum, running_mean, running_var, save_mean,
                       save_invstd, coef, (float*)nullptr, (float*)nullptr);
    LV_CHECK_LAUNCH("bn_finalize_kernel<0>");
  } else {
    LV_CHECK_ARG(running_mean && running_var, "eval needs the running statistics");
    hipLaunchKernelGGL(bn_eval_coef_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, st, gamma, beta, running_mean,
                       running_var, eps, C, coef);
    LV_CHECK_LAUNCH("bn_eval_coef_kernel");
  }
  const int64_t nvec = P * C / 8;
  hipLaunchKernelGGL(bn_apply_kernel<0>, dim3(apply_blocks(nvec)), dim3(kBnThreads), 2 * C * sizeof(float), st,
                     (const __hip_bfloat16*)x, (const __hip_bfloat16*)nullptr, coef, 2, slope, C, nvec,
                     (__hip_bfloat16*)y);
  LV_RETURN_LAUNCH("bn_apply_kernel<0>");
}

int lv_bn_lrelu_bwd_bf16(const void* g, const void* x, const float* gamma, const float* beta, const float* save_mean,
                         const float* save_invstd, float slope, void* gx, float* ggamma, float* gbeta, float* ws,
                         int64_t P, int C, void* stream) {
  clear_error();
  BnGeom geo;
  LV_CHECK_ARG(bn_geom(P, C, &geo), "unsupported shape P=%lld C=%d (lv_bn_supported)", (long long)P, C);
  LV_CHECK_ARG(g && x && save_mean && save_invstd && gx && ws, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  float* coef = ws + (size_t)geo.nblk * 2 * C;   // [a | b | mean | invstd | k1 | k2 | k3]
  hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, st, gamma, beta, save_mean,
                     save_invstd, C, coef);
  LV_CHECK_LAUNCH("bn_bwd_coef_kernel");
  hipLaunchKernelGGL(bn_reduce_part_kernel<1>, dim3(geo.nblk), dim3(kBnThreads), 0, st, (const __hip_bfloat16*)x,
                     (const __hip_bfloat16*)g, (const float*)coef, slope, geo, ws);
  LV_CHECK_LAUNCH("bn_reduce_part_kernel<1>");
  hipLaunchKernelGGL(bn_finalize_kernel<1>, dim3(ceil_div(C, 64)), dim3(64 * kBnFinSlices), 0, st, ws, geo.nblk, C, P,
                     (const __hip_bfloat16*)x, gamma, beta, 0.f, 0.f, (float*)nullptr, (float*)nullptr,
                     (float*)save_mean, (float*)save_invstd, coef + 4 * C, ggamma, gbeta);
  LV_CHECK_LAUNCH("bn_finalize_kernel<1>");
  const int64_t nvec = P * C / 8;
  hipLaunchKernelGGL(bn_apply_kernel<2>, dim3(apply_blocks(nvec)), dim3(kBnThreads), 7 * C * sizeof(float), st,
                     (const __hip_bfloat16*)x, (const __hip_bfloat16*)g, coef, 7, slope, C, nvec,
                     (__hip_bfloat16*)gx);
  LV_RETURN_LAUNCH("bn_apply_kernel<2>");
}

}  // extern "C"

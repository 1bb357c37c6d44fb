// Decoder transposed convolution on MFMA: ConvTranspose2d(Cin, Cout,
// kernel 4, stride 2, padding 1) forward, bf16 NHWC, fp32 accumulate -- the three
// hidden 200 -> 200 upsampling layers of DeconvNet (reference nets.py:60-75; config 3/4
// decoder).  MIOpen runs these as backward-data convolutions at ~12% of the bf16 MFMA
// peak (profiles/r03_train_config3_bf16_steady_kernels.txt); here each layer is four
// implicit GEMMs, one per output phase.
//
// Sub-pixel decomposition.  Output pixel (2a + r, 2b + s) only sees input pixels
// (a + di, b + dj) with di in {r - 1, r}, dj in {s - 1, s}, through kernel tap
// (ku, kv) = (1 - 2 di + r, 1 - 2 dj + s).  So phase p = 2r + s is a GEMM
//   Y_p[m, o] = sum_k A_p[m, k] Wt_p[o, k],   m = (n, a, b),  k = t * Cin + c,
// t = 2 (di - r + 1) + (dj - s + 1) the 2x2 tap, A_p[m, t*Cin + c] = x[n, a+di, b+dj, c]
// (zero outside the image): M = N·H·W, K = 4·Cin, N = Cout, with no zero taps.  The
// weight is repacked once per call into Wt[p][o][k] (o padded to kBN with zeros), so a
// lane's 8 consecutive k of one output channel are one 16-byte load.
//
// Tiling (gfx950, v_mfma_f32_16x16x32_bf16): a block of BM / 32 waves (BM = 256 by
// default: the weight tile is read from L2 once per 256 pixels; 128 ran 1.1-1.8x slower)
// computes a BM-pixel x kBN-channel tile of one phase; wave w owns pixel rows [32w, 32w+32)
// x all channels (2 x 13 accumulator tiles of 16x16, 104 fp32 registers).  K steps of 32:
// the next step's A (BM x 32) and B (kBN x 32) pieces are loaded to registers while the current
// step's MFMAs run, then written to the other LDS buffer (row pitch 80 B: the 16-byte
// fragment reads of 8 consecutive rows fall in distinct banks).  Epilogue: + bias, round
// to bf16, stage the tile in LDS, 16-byte stores of whole 2·Cout-byte output rows.
#include <map>
#include <mutex>
#include <tuple>
#include <algorithm>

#include "lv_common.h"

namespace lv {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// g where x > 0 (ReLU backward against its output x), 8 packed bf16: x > 0 <=> the signed
// 16-bit pattern is positive (a +NaN x also passes; the reference's mask would drop it).
__device__ __forceinline__ u32x4 relu_mask_bf16x8(u32x4 g, u32x4 x) {
  const s16x8 keep = __builtin_bit_cast(s16x8, x) > s16x8(0);  // lanes of -1 / 0
  return g & __builtin_bit_cast(u32x4, keep);
}

constexpr int kBN = 208;               // output channels per tile (13 x 16; Cout <= kBN)
constexpr int kNT = kBN / 16;          // 16-wide channel tiles
constexpr int kBK = 32;                // K per step (one MFMA)
constexpr int kPitch = kBK + 8;        // LDS row pitch in bf16 (80 B)
constexpr int kBPieces = kBN * kBK / 8;   // 16-byte pieces per B step (832)
// BM pixels per block tile, BM / 32 waves (each 32 pixel rows x kBN channels)
template <int BM>
struct DeconvTile {
  static constexpr int kThreads = BM * 2;
  static constexpr int kAPer = BM * kBK / 8 / kThreads;                 // 2
  static constexpr int kBPer = (kBPieces + kThreads - 1) / kThreads;    // 4 / 2
  static constexpr int kStageRows = BM <= 128 ? BM : 128;               // epilogue pass rows
  static constexpr size_t kLds = 2 * (size_t)(BM + kBN) * kPitch * 2;   // 53,760 / 74,240 B
  static_assert((size_t)kStageRows * kBN * 2 <= kLds, "epilogue stage fits the A/B buffers");
};

// Wt[p][o][t*Cin + c] = w[c][o][ku][kv] for o < Cout, 0 for Cout <= o < kBN.  One thread
// per 8 consecutive k of one (phase, channel): 8 gathered 2-byte reads of the (L2-resident)
// weight, one 16-byte store.
__global__ void deconv_pack_kernel(const __hip_bfloat16* w, __hip_bfloat16* wt, int Cin, int Cout) {
  const int K = 4 * Cin, kg = K / 8;
  const int total = 4 * kBN * kg;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int g = i % kg, o = (i / kg) % kBN, p = i / (kg * kBN);
    const int k0 = 8 * g, t = k0 / Cin, c0 = k0 - t * Cin;
    const int r = p >> 1, s = p & 1;
    const int di = r - 1 + (t >> 1), dj = s - 1 + (t & 1);
    const int tap = (1 - 2 * di + r) * 4 + (1 - 2 * dj + s);
    __hip_bfloat16 v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] = o < Cout ? w[((c0 + e) * Cout + o) * 16 + tap] : __float2bfloat16(0.f);
    *reinterpret_cast<u32x4*>(wt + ((int64_t)(p * kBN + o) * K + k0)) = *reinterpret_cast<const u32x4*>(v);
  }
  // 64 zero bytes after the packed weight: the v2 kernel's source for taps outside the image
  if (blockIdx.x == 0 && threadIdx.x < 4)
    *reinterpret_cast<u32x4*>(wt + (int64_t)4 * kBN * K + 8 * threadIdx.x) = u32x4{0u, 0u, 0u, 0u};
}

struct DeconvArgs {
  const __hip_bfloat16* x;   // (N, H, W, Cin) bf16, channels-last
  const __hip_bfloat16* wt;  // (4, kBN, 4*Cin) bf16, deconv_pack_kernel
  const float* bias;         // (Cout) or null
  __hip_bfloat16* y;         // (N, 2H, 2W, Cout) bf16, channels-last
  int64_t M;                 // N*H*W pixels per phase
  int H, W, Cin, Cout;
  int relu;                  // epilogue max(0, .) (the decoder's ReLU after the layer)
};

template <int BM>
__global__ __launch_bounds__(BM * 2) void deconv_mfma_kernel(DeconvArgs a) {
  using T = DeconvTile<BM>;
  constexpr int kThreads = T::kThreads, kAPer = T::kAPer, kBPer = T::kBPer;
  constexpr int kBM = BM;
  extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
  __hip_bfloat16* As = smem;                       // [2][kBM][kPitch]
  __hip_bfloat16* Bs = smem + 2 * kBM * kPitch;    // [2][kBN][kPitch]
  const int tid = (int)threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = blockIdx.y, r = p >> 1, s = p & 1;
  const int64_t m0 = (int64_t)blockIdx.x * kBM;
  const int K = 4 * a.Cin;
  const int nk = K / kBK;
  const __hip_bfloat16* wtp = a.wt + (int64_t)p * kBN * K;

  // A pieces of this thread: pixel row and the 8-channel group inside the K step
  int64_t abase[kAPer];  // element offset of (pixel, tap 0 origin) or -1 outside M
  int arow[kAPer], aq[kAPer], aa[kAPer], ab[kAPer];
#pragma unroll
  for (int i = 0; i < kAPer; ++i) {
    const int pid = tid + kThreads * i;
    arow[i] = pid >> 2;
    aq[i] = pid & 3;
    const int64_t m = m0 + arow[i];
    if (m < a.M) {
      const int b = (int)(m % a.W);
      const int64_t na = m / a.W;
      aa[i] = (int)(na % a.H);
      ab[i] = b;
      abase[i] = (na / a.H) * a.H;  // n * H
    } else {
      abase[i] = -1;
      aa[i] = ab[i] = 0;
    }
  }
  auto load_a = [&](int ks, u32x4 (&ra)[kAPer]) {
#pragma unroll
    for (int i = 0; i < kAPer; ++i) {
      const int k0 = ks * kBK + aq[i] * 8;
      const int t = k0 / a.Cin, c = k0 - t * a.Cin;
      const int ia = aa[i] + r - 1 + (t >> 1), ib = ab[i] + s - 1 + (t & 1);
      ra[i] = u32x4{0u, 0u, 0u, 0u};
      if (abase[i] >= 0 && ia >= 0 && ia < a.H && ib >= 0 && ib < a.W)
        ra[i] = *reinterpret_cast<const u32x4*>(a.x + ((abase[i] + ia) * a.W + ib) * a.Cin + c);
    }
  };
  auto load_b = [&](int ks, u32x4 (&rb)[kBPer]) {
#pragma unroll
    for (int i = 0; i < kBPer; ++i) {
      const int pid = tid + kThreads * i;
      if (pid < kBPieces) {
        const int o = pid >> 2, q = pid & 3;
        rb[i] = *reinterpret_cast<const u32x4*>(wtp + (int64_t)o * K + ks * kBK + q * 8);
      }
    }
  };
  auto store_ab = [&](int buf, const u32x4 (&ra)[kAPer], const u32x4 (&rb)[kBPer]) {
#pragma unroll
    for (int i = 0; i < kAPer; ++i)
      *reinterpret_cast<u32x4*>(As + (buf * kBM + arow[i]) * kPitch + aq[i] * 8) = ra[i];
#pragma unroll
    for (int i = 0; i < kBPer; ++i) {
      const int pid = tid + kThreads * i;
      if (pid < kBPieces)
        *reinterpret_cast<u32x4*>(Bs + (buf * kBN + (pid >> 2)) * kPitch + (pid & 3) * 8) = rb[i];
    }
  };

  f32x4 acc[2][kNT];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < kNT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[kAPer], rb[kBPer];
  load_a(0, ra);
  load_b(0, rb);
  store_ab(0, ra, rb);
  __syncthreads();
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) {  // next step's pieces in flight during this step's MFMAs
      load_a(ks + 1, ra);
      load_b(ks + 1, rb);
    }
    const __hip_bfloat16* Ab = As + (buf * kBM + wave * 32) * kPitch;
    const __hip_bfloat16* Bb = Bs + buf * kBN * kPitch;
    bf16x8 af[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
      af[mt] = *reinterpret_cast<const bf16x8*>(Ab + (mt * 16 + fr) * kPitch + fk);
#pragma unroll
    for (int nt = 0; nt < kNT; ++nt) {
      const bf16x8 bf = *reinterpret_cast<const bf16x8*>(Bb + (nt * 16 + fr) * kPitch + fk);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bf, acc[mt][nt], 0, 0, 0);
    }
    if (ks + 1 < nk) {
      store_ab(buf ^ 1, ra, rb);  // the other buffer: last read one step ago
      __syncthreads();
    }
  }
  // epilogue: + bias, bf16, stage [rows][kBN] in LDS (reuses the A/B buffers) in passes
  // of kStageRows pixel rows, then 16-byte stores of whole output rows (Cout % 8 == 0)
  __hip_bfloat16* Cs = smem;
  const int cq = (lane >> 4) * 4;
  const int pieces = a.Cout / 8;
  const int H2 = 2 * a.H, W2 = 2 * a.W;
  constexpr int SR = T::kStageRows;
#pragma unroll
  for (int pass = 0; pass < kBM / SR; ++pass) {
    __syncthreads();
    if (wave * 32 / SR == pass) {
#pragma unroll
      for (int nt = 0; nt < kNT; ++nt) {
        const int o = nt * 16 + fr;
        const float bo = (a.bias && o < a.Cout) ? a.bias[o] : 0.f;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v = acc[mt][nt][j] + bo;
            if (a.relu) v = fmaxf(v, 0.f);
            Cs[(wave * 32 - pass * SR + mt * 16 + cq + j) * kBN + o] = __float2bfloat16(v);
          }
      }
    }
    __syncthreads();
    for (int e = tid; e < SR * pieces; e += kThreads) {
      const int row = e / pieces, q = e - row * pieces;
      const int64_t m = m0 + pass * SR + row;
      if (m >= a.M) continue;
      const int b = (int)(m % a.W);
      const int64_t na = m / a.W;
      const int aa_ = (int)(na % a.H);
      const int64_t n = na / a.H;
      __hip_bfloat16* dst = a.y + (((n * H2 + 2 * aa_ + r) * W2 + 2 * b + s) * a.Cout) + q * 8;
      *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(Cs + row * kBN + q * 8);
    }
  }
}


// v2 of the same GEMMs: the block's A (BM x 32) and B (kBN x 32) pieces go global -> LDS
// by LDS-DMA (global_load_lds, 16 B per lane, no register staging) into an S-stage ring
// issued S - 1 K-steps ahead, and the 8 waves tile the 256 x 208 block tile as 4 (rows) x 2
// (channels): wave (wm, wn) owns 64 pixel rows x 7 | 6 channel tiles, so per K-step a wave
// reads 4 A + 7 B fragments for 28 MFMAs (v1: 2 + 13 for 26).  The DMA writes 16 rows x
// 64 B per wave instruction, so rows are unpadded and the 16-B k-chunks are XOR-swizzled
// (chunk ^ (row >> 2) & 3): the 16 rows of a fragment read fall in 16 distinct 4-bank
// groups.  Taps outside the image read 64 zero bytes kept after the packed weight.  Same
// MFMA sequence per output element as v1: bitwise equal.
// BM = 256: 4 x 2 waves (64 rows x 7 | 6 channel tiles), 159 VGPRs, one block per CU;
// BM = 128: 2 x 4 waves (64 rows x 3 | 3 | 3 | 4 tiles), for two blocks per CU.
template <int S, int BM = 256>
struct DeconvV2 {
  static constexpr int kWM = BM / 64, kWN = 8 / kWM;                // wave grid
  static constexpr int kNW = (kNT + kWN - 1) / kWN;                  // max channel tiles per wave
  static constexpr int kAI = BM / 128;                               // A DMA instructions per wave
  static constexpr int kSR = BM / 2;                                 // epilogue rows per pass
  static constexpr int kA = BM * kBK, kB = kBN * kBK;                // bf16 per stage
  static constexpr size_t kLds = (size_t)S * (kA + kB) * 2;          // BM 256, S = 2: 59,392 B
  static_assert((size_t)kSR * kBN * 2 <= kLds, "epilogue stage fits the ring");
};
__device__ __forceinline__ int v2_swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }
__device__ __forceinline__ void vm_wait(int n) {  // s_waitcnt vmcnt(n), n wave-uniform
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
  }
}

// XCD: 1-D grid whose consecutive block ids are dealt round-robin over the 8 XCDs; the four
// phases of a pixel tile get ids b, b + 8, b + 16, b + 24, i.e. the same XCD at about the
// same time, so the tile's input pixels come from HBM into that XCD's L2 once, not 4 times.
template <int S, bool XCD, int BM = 256, bool RM = false>
__global__ __launch_bounds__(512) void deconv_mfma2_kernel(DeconvArgs a) {
  using T = DeconvV2<S, BM>;
  constexpr int kV2BM = BM, kV2NW = T::kNW;
  extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 smem[];
  const int tid = (int)threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // RM: SIMD-balanced wave tiling, as in deconv_mfma_f32_kernel
  const int wm = RM ? wave % T::kWM : wave / T::kWN, wn = RM ? wave / T::kWM : wave % T::kWN;
  const int t0 = wn * kNT / T::kWN, ntw = (wn + 1) * kNT / T::kWN - t0;  // this wave's channel tiles
  int p, tile;
  if constexpr (XCD) {
    const int bid = (int)blockIdx.x, slot = bid >> 3;
    p = slot & 3;
    tile = (bid & 7) + 8 * (slot >> 2);
    if ((int64_t)tile * kV2BM >= a.M) return;  // grid padded to whole groups of 8 tiles
  } else {
    p = blockIdx.y;
    tile = blockIdx.x;
  }
  const int r = p >> 1, s = p & 1;
  const int64_t m0 = (int64_t)tile * kV2BM;
  const int K = 4 * a.Cin;
  const int nk = K / kBK;
  const __hip_bfloat16* wtp = a.wt + (int64_t)p * kBN * K;
  const __hip_bfloat16* zero16 = a.wt + (int64_t)4 * kBN * K;
  const int lrow = lane >> 2, lslot = lane & 3;
  // A DMA: rows (BM / 8) wave + 16 i + lrow (i < kAI)
  int64_t abase[T::kAI];
  int aa[T::kAI], ab[T::kAI], achunk[T::kAI];
#pragma unroll
  for (int i = 0; i < T::kAI; ++i) {
    const int row = (BM / 8) * wave + 16 * i + lrow;
    achunk[i] = v2_swz(row, lslot);
    const int64_t m = m0 + row;
    if (m < a.M) {
      const int64_t na = m / a.W;
      ab[i] = (int)(m - na * a.W);
      aa[i] = (int)(na % a.H);
      abase[i] = (na / a.H) * a.H;
    } else {
      abase[i] = -1;
      aa[i] = ab[i] = 0;
    }
  }
  // B DMA: 16-row groups g = wave, wave + 8 (< kNT)
  const int nbg = wave + 8 < kNT ? 2 : 1;
  const int bchunk = v2_swz(lrow, lslot);  // (16 g + lrow) >> 2 & 3 == lrow >> 2 & 3
  auto issue = [&](int ks, int stage) {
    __hip_bfloat16* As = smem + stage * (T::kA + T::kB);
    __hip_bfloat16* Bs = As + T::kA;
#pragma unroll
    for (int i = 0; i < T::kAI; ++i) {
      const int k0 = ks * kBK + achunk[i] * 8;
      const int t = k0 / a.Cin, c = k0 - t * a.Cin;
      const int ia = aa[i] + r - 1 + (t >> 1), ib = ab[i] + s - 1 + (t & 1);
      const __hip_bfloat16* src = (abase[i] >= 0 && ia >= 0 && ia < a.H && ib >= 0 && ib < a.W)
                                      ? a.x + ((abase[i] + ia) * a.W + ib) * a.Cin + c
                                      : zero16;
      __builtin_amdgcn_global_load_lds(src, as_lds(As + ((BM / 8) * wave + 16 * i) * kBK), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j < nbg) {
        const int g = wave + 8 * j;
        const __hip_bfloat16* src = wtp + (int64_t)(16 * g + lrow) * K + ks * kBK + bchunk * 8;
        __builtin_amdgcn_global_load_lds(src, as_lds(Bs + 16 * g * kBK), 16, 0, 0);
      }
    }
  };

  f32x4 acc[4][kV2NW];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < kV2NW; ++j) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < S - 1; ++st)
    if (st < nk) issue(st, st);
  const int per = T::kAI + nbg;  // DMA instructions per stage of this wave
  const int fr = lane & 15, kc = lane >> 4;
  for (int ks = 0; ks < nk; ++ks) {
    const int stage = ks % S;
    vm_wait(per * min(S - 2, nk - 1 - ks));  // this wave's pieces of step ks have landed
    // everyone's have; stage (ks - 1) % S is free.  Not __syncthreads(): its fence waits for
    // vmcnt(0), i.e. for the DMA of the steps still in flight, which undoes the ring.
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (ks + S - 1 < nk) issue(ks + S - 1, (ks + S - 1) % S);
    const __hip_bfloat16* As = smem + stage * (T::kA + T::kB);
    const __hip_bfloat16* Bs = As + T::kA;
    bf16x8 af[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int row = wm * 64 + mt * 16 + fr;
      af[mt] = *reinterpret_cast<const bf16x8*>(As + row * kBK + v2_swz(row, kc) * 8);
    }
#pragma unroll
    for (int j = 0; j < kV2NW; ++j) {
      if (j < ntw) {
        const int row = (t0 + j) * 16 + fr;
        const bf16x8 bf = *reinterpret_cast<const bf16x8*>(Bs + row * kBK + v2_swz(row, kc) * 8);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bf, acc[mt][j], 0, 0, 0);
      }
    }
  }
  // epilogue: + bias (+ ReLU), bf16, staged [128 rows][kBN] in LDS per pass, 16-byte stores
  __hip_bfloat16* Cs = smem;
  const int cq = (lane >> 4) * 4;
  const int pieces = a.Cout / 8;
  const int H2 = 2 * a.H, W2 = 2 * a.W;
  constexpr int SR = T::kSR;
#pragma unroll
  for (int pass = 0; pass < kV2BM / SR; ++pass) {
    __syncthreads();
    if (wm * 64 / SR == pass) {
#pragma unroll
      for (int j = 0; j < kV2NW; ++j) {
        if (j < ntw) {
          const int o = (t0 + j) * 16 + fr;
          const float bo = (a.bias && o < a.Cout) ? a.bias[o] : 0.f;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              float v = acc[mt][j][q] + bo;
              if (a.relu) v = fmaxf(v, 0.f);
              Cs[(wm * 64 - pass * SR + mt * 16 + cq + q) * kBN + o] = __float2bfloat16(v);
            }
        }
      }
    }
    __syncthreads();
    if (pieces * 8 == a.Cout) {
      for (int e = tid; e < SR * pieces; e += 512) {
        const int row = e / pieces, q = e - row * pieces;
        const int64_t m = m0 + pass * SR + row;
        if (m >= a.M) continue;
        const int b = (int)(m % a.W);
        const int64_t na = m / a.W;
        const int aa_ = (int)(na % a.H);
        const int64_t n = na / a.H;
        __hip_bfloat16* dst = a.y + (((n * H2 + 2 * aa_ + r) * W2 + 2 * b + s) * a.Cout) + q * 8;
        *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(Cs + row * kBN + q * 8);
      }
    } else {  // Cout % 4 == 0: 8-byte pieces (e.g. an encoder conv's dgrad to 100 channels)
      const int p4 = a.Cout / 4;
      for (int e = tid; e < SR * p4; e += 512) {
        const int row = e / p4, q = e - row * p4;
        const int64_t m = m0 + pass * SR + row;
        if (m >= a.M) continue;
        const int b = (int)(m % a.W);
        const int64_t na = m / a.W;
        const int aa_ = (int)(na % a.H);
        const int64_t n = na / a.H;
        __hip_bfloat16* dst = a.y + (((n * H2 + 2 * aa_ + r) * W2 + 2 * b + s) * a.Cout) + q * 4;
        *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(Cs + row * kBN + q * 4);
      }
    }
  }
}

// ----------------------------------------------------- fp32 (the reference's precision)
// The same four sub-pixel GEMMs for fp32 operands on v_mfma_f32_16x16x4_f32 (exact fp32
// products, fp32 accumulation), for the fp32 training step (reference unsupervised.py:108-117
// trains in fp32), where MIOpen runs these layers at 53% of the fp32 peak
// (profiles/r06_conv_layers_f32.txt).  x is channels-last (N, H, W, Cin) fp32, y NCHW fp32
// (the layout of the fp32 network around it).  The v2 structure with fp32 elements: K steps
// of 16 (64-byte rows per stage, as the bf16 kernel's 32), LDS-DMA ring of 2 stages with the
// same XOR-swizzled 16-byte chunks, 8 waves as (BM / 64) x (8 / (BM / 64)), XCD-grouped
// phases.  A lane's 16-byte fragment (k = 4 kc .. 4 kc + 3 of its row) feeds four MFMAs:
// MFMA `sub` takes k = 4 kc + sub from lane group kc, in A and B alike.  The epilogue stages
// one 64-row band per pass in LDS (pitch kBN + 1: conflict-free reads) and writes NCHW
// with one 4-byte store per element, consecutive lanes on consecutive pixels.
constexpr int kBKf = 16;
template <int BM, int S = 2>
struct DeconvF32 {
  static constexpr int kWM = BM / 64, kWN = 8 / kWM;
  static constexpr int kNW = (kNT + kWN - 1) / kWN;
  static constexpr int kAI = BM / 128;                     // A DMA instructions per wave
  static constexpr int kA = BM * kBKf, kB = kBN * kBKf;    // floats per stage
  static constexpr int kSP = kBN + 1;                      // epilogue stage pitch (floats)
  static constexpr size_t kRing = S * (size_t)(kA + kB) * 4;
  static constexpr size_t kStage = 64 * (size_t)kSP * 4;
  static constexpr size_t kLds = kRing > kStage ? kRing : kStage;  // BM 128: 53,504 B
};

// Wt[p][o][t*Cin + c] = w[c][o][ku][kv] in fp32 (deconv_pack_kernel's layout), 4 k per thread
// (one 16-byte store), + 16 zero floats after it (the source of taps outside the image).
__global__ void deconv_pack_f32_kernel(const float* w, float* wt, int Cin, int Cout) {
  const int K = 4 * Cin, kg = K / 4;
  const int total = 4 * kBN * kg;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int g = i % kg, o = (i / kg) % kBN, p = i / (kg * kBN);
    const int k0 = 4 * g, t = k0 / Cin, c0 = k0 - t * Cin;
    const int r = p >> 1, s = p & 1;
    const int di = r - 1 + (t >> 1), dj = s - 1 + (t & 1);
    const int tap = (1 - 2 * di + r) * 4 + (1 - 2 * dj + s);
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = o < Cout ? w[((c0 + e) * Cout + o) * 16 + tap] : 0.f;
    *reinterpret_cast<f32x4*>(wt + ((int64_t)(p * kBN + o) * K + k0)) = v;
  }
  if (blockIdx.x == 0 && threadIdx.x < 4)
    *reinterpret_cast<f32x4*>(wt + (int64_t)4 * kBN * K + 4 * threadIdx.x) = f32x4{0.f, 0.f, 0.f, 0.f};
}

struct DeconvF32Args {
  const float* x;     // (N, H, W, Cin) fp32, channels-last
  const float* wt;    // (4, kBN, 4*Cin) fp32, deconv_pack_f32_kernel
  const float* bias;  // (Cout) or null
  float* y;           // (N, Cout, 2H, 2W) fp32, NCHW
  float* y_cl;        // the same values channels-last (N, 2H, 2W, Cout), or null
  int64_t M;          // N*H*W pixels per phase
  int H, W, Cin, Cout;
  int relu;
};

template <int BM, int S, bool RM = false>
__global__ __launch_bounds__(512) void deconv_mfma_f32_kernel(DeconvF32Args a) {
  using T = DeconvF32<BM, S>;
  extern __shared__ __attribute__((aligned(16))) float smf[];
  const int tid = (int)threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // RM: wave w -> (wm, wn) = (w % kWM, w / kWM).  A block's waves go round-robin to the
  // CU's 4 SIMDs (SIMD = w % 4), and the 13 channel tiles split 3 | 3 | 3 | 4 over wn: with
  // wn = w % 4 one SIMD holds both 4-tile waves (8 tile-units against 6), with RM the SIMDs
  // hold 6 / 6 / 7 / 7 -- the block's per-step barrier waits for the busiest SIMD
  const int wm = RM ? wave % T::kWM : wave / T::kWN, wn = RM ? wave / T::kWM : wave % T::kWN;
  const int t0 = wn * kNT / T::kWN, ntw = (wn + 1) * kNT / T::kWN - t0;
  // XCD-grouped 1-D grid (deconv_mfma2_kernel): phases of a tile on one XCD
  const int bid = (int)blockIdx.x, slot = bid >> 3;
  const int p = slot & 3;
  const int tile = (bid & 7) + 8 * (slot >> 2);
  if ((int64_t)tile * BM >= a.M) return;
  const int r = p >> 1, s = p & 1;
  const int64_t m0 = (int64_t)tile * BM;
  const int K = 4 * a.Cin;
  const int nk = K / kBKf;
  const float* wtp = a.wt + (int64_t)p * kBN * K;
  const float* zero16 = a.wt + (int64_t)4 * kBN * K;
  const int lrow = lane >> 2, lslot = lane & 3;
  int64_t abase[T::kAI];
  int aa[T::kAI], ab[T::kAI], achunk[T::kAI];
#pragma unroll
  for (int i = 0; i < T::kAI; ++i) {
    const int row = (BM / 8) * wave + 16 * i + lrow;
    achunk[i] = v2_swz(row, lslot);
    const int64_t m = m0 + row;
    if (m < a.M) {
      const int64_t na = m / a.W;
      ab[i] = (int)(m - na * a.W);
      aa[i] = (int)(na % a.H);
      abase[i] = (na / a.H) * a.H;
    } else {
      abase[i] = -1;
      aa[i] = ab[i] = 0;
    }
  }
  const int nbg = wave + 8 < kNT ? 2 : 1;
  const int bchunk = v2_swz(lrow, lslot);
  auto issue = [&](int ks, int stage) {
    float* As = smf + stage * (T::kA + T::kB);
    float* Bs = As + T::kA;
#pragma unroll
    for (int i = 0; i < T::kAI; ++i) {
      const int k0 = ks * kBKf + achunk[i] * 4;
      const int t = k0 / a.Cin, c = k0 - t * a.Cin;
      const int ia = aa[i] + r - 1 + (t >> 1), ib = ab[i] + s - 1 + (t & 1);
      const float* src = (abase[i] >= 0 && ia >= 0 && ia < a.H && ib >= 0 && ib < a.W)
                             ? a.x + ((abase[i] + ia) * a.W + ib) * a.Cin + c
                             : zero16;
      __builtin_amdgcn_global_load_lds(src, as_lds(As + ((BM / 8) * wave + 16 * i) * kBKf), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j < nbg) {
        const int g = wave + 8 * j;
        const float* src = wtp + (int64_t)(16 * g + lrow) * K + ks * kBKf + bchunk * 4;
        __builtin_amdgcn_global_load_lds(src, as_lds(Bs + 16 * g * kBKf), 16, 0, 0);
      }
    }
  };

  f32x4 acc[4][T::kNW];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int j = 0; j < T::kNW; ++j) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < S - 1; ++st)
    if (st < nk) issue(st, st);
  const int per = T::kAI + nbg;  // DMA instructions per stage of this wave
  const int fr = lane & 15, kc = lane >> 4;
  for (int ks = 0; ks < nk; ++ks) {
    const int stage = ks % S;
    vm_wait(per * min(S - 2, nk - 1 - ks));  // this wave's pieces of step ks have landed
    // everyone's have; stage (ks - 1) % S is free
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (ks + S - 1 < nk) issue(ks + S - 1, (ks + S - 1) % S);
    const float* As = smf + stage * (T::kA + T::kB);
    const float* Bs = As + T::kA;
    f32x4 af[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int row = wm * 64 + mt * 16 + fr;
      af[mt] = *reinterpret_cast<const f32x4*>(As + row * kBKf + v2_swz(row, kc) * 4);
    }
#pragma unroll
    for (int j = 0; j < T::kNW; ++j) {
      if (j < ntw) {
        const int row = (t0 + j) * 16 + fr;
        const f32x4 bf = *reinterpret_cast<const f32x4*>(Bs + row * kBKf + v2_swz(row, kc) * 4);
#pragma unroll
        for (int sub = 0; sub < 4; ++sub)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mt][sub], bf[sub], acc[mt][j], 0, 0, 0);
      }
    }
  }
  // epilogue: + bias (+ ReLU), one 64-row band (wave row wm) per pass staged [row][o], then
  // NCHW stores: element e of the band -> (o = e / 64, row = e % 64)
  float* Cs = smf;
  const int cq = (lane >> 4) * 4;
  const int H2 = 2 * a.H, W2 = 2 * a.W;
  for (int pass = 0; pass < T::kWM; ++pass) {
    __syncthreads();
    if (wm == pass) {
#pragma unroll
      for (int j = 0; j < T::kNW; ++j) {
        if (j < ntw) {
          const int o = (t0 + j) * 16 + fr;
          const float bo = (a.bias && o < a.Cout) ? a.bias[o] : 0.f;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              float v = acc[mt][j][q] + bo;
              if (a.relu) v = fmaxf(v, 0.f);
              Cs[(mt * 16 + cq + q) * T::kSP + o] = v;
            }
        }
      }
    }
    __syncthreads();
    for (int e = tid; e < 64 * a.Cout; e += 512) {
      const int row = e & 63, o = e >> 6;
      const int64_t m = m0 + pass * 64 + row;
      if (m >= a.M) continue;
      const int64_t na = m / a.W;
      const int b = (int)(m - na * a.W);
      const int aa_ = (int)(na % a.H);
      const int64_t n = na / a.H;
      a.y[((n * a.Cout + o) * H2 + 2 * aa_ + r) * W2 + 2 * b + s] = Cs[row * T::kSP + o];
    }
    if (a.y_cl) {  // channels-last twin (the next layer's input): 16-byte pieces of 4 channels
      const int q4 = a.Cout >> 2;
      for (int e = tid; e < 64 * q4; e += 512) {
        const int row = e / q4, q = e - row * q4;
        const int64_t m = m0 + pass * 64 + row;
        if (m >= a.M) continue;
        const int64_t na = m / a.W;
        const int b = (int)(m - na * a.W);
        const int aa_ = (int)(na % a.H);
        const int64_t n = na / a.H;
        const float* src = Cs + row * T::kSP + 4 * q;
        *reinterpret_cast<f32x4*>(a.y_cl + ((n * H2 + 2 * aa_ + r) * W2 + 2 * b + s) * a.Cout + 4 * q) =
            f32x4{src[0], src[1], src[2], src[3]};
      }
    }
  }
}

// ----------------------------------------------------- small-Cout decoder layer
// The decoder's last layer ConvTranspose2d(200, 3, 4, 2, 1) (nets.py:74): an N = 3
// GEMM per phase wastes an MFMA tile and MIOpen runs it at ~10 TFLOP/s (1 ms per forward
// at batch 512, profiles/r03_conv_layers.txt).  Here one GEMM row is an output QUAD
// (2a + r, 2b + s), r, s in {0, 1}: its four pixels see only the 3x3 input neighbourhood
// of (a, b), so
//   Y[quad, (p, o)] = sum_{nbr, c} X[a + na - 1, b + nb - 1, c] Wq[nbr, c, (p, o)],
// with Wq[nbr, c, (p, o)] = w[c, o, ku, kv] when nbr = (na, nb) is a tap of phase p (else
// 0): K = 9 x Cin, N = 4·Cout <= 16 -- one 16x16x32 MFMA column tile for all phases.
// A block covers 8 x 16 quads of one image; per 32-channel chunk the 10 x 18 input pixels
// of that region are staged once in LDS and the nine neighbour offsets are nine K steps
// read from it (no im2col), so each input byte crosses HBM once (+ a halo).  Channels
// beyond Cin read as zero (K padded to a multiple of 32 per neighbour).
constexpr int kSqH = 8, kSqW = 16;                      // quads per block
constexpr int kSiH = kSqH + 2, kSiW = kSqW + 2;         // staged input pixels
constexpr int kSPitch = 40;                              // bf16 per staged pixel (32 + pad)
constexpr int kSmallThreads = 256;
constexpr int kSmallMaxCout = 4;

// Wq[chunk][nbr][n][32] (n = p * Cout + o padded to 16), zeros where nbr is not a tap of p
__global__ void deconv_small_pack_kernel(const __hip_bfloat16* w, __hip_bfloat16* wq, int Cin, int Cout) {
  const int nch = (Cin + 31) / 32;
  const int total = nch * 9 * 16 * 32;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cl = i % 32, n = (i / 32) % 16, nbr = (i / 512) % 9, ch = i / (512 * 9);
    const int c = ch * 32 + cl;
    const int p = n / Cout, o = n - p * Cout;
    float v = 0.f;
    if (c < Cin && p < 4) {
      const int r = p >> 1, s = p & 1;
      const int di = nbr / 3 - 1, dj = nbr % 3 - 1;           // input offset of the neighbour
      if ((di == r - 1 || di == r) && (dj == s - 1 || dj == s)) {
        const int ku = 1 - 2 * di + r, kv = 1 - 2 * dj + s;
        v = __bfloat162float(w[((c * Cout + o) * 4 + ku) * 4 + kv]);
      }
    }
    wq[i] = __float2bfloat16(v);
  }
}

struct DeconvSmallArgs {
  const __hip_bfloat16* x;    // (N, H, W, Cin) bf16 channels-last
  const __hip_bfloat16* wq;   // deconv_small_pack_kernel
  const float* bias;          // (Cout) or null
  __hip_bfloat16* y;          // (N, 2H, 2W, Cout) bf16 channels-last
  int H, W, Cin, Cout, tiles_w;
};

__global__ __launch_bounds__(kSmallThreads) void deconv_small_kernel(DeconvSmallArgs a) {
  __shared__ __attribute__((aligned(16))) __hip_bfloat16 xs[2][kSiH * kSiW * kSPitch];  // 2 x 14.4 KB
  __shared__ __attribute__((aligned(16))) __hip_bfloat16 ws[2][9 * 16 * kSPitch];         // 2 x 11.5 KB
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_img = blockIdx.y;
  const int ta = blockIdx.x / a.tiles_w, tb = blockIdx.x - ta * a.tiles_w;
  const int a0 = ta * kSqH, b0 = tb * kSqW;
  const int nch = (a.Cin + 31) / 32;
  const __hip_bfloat16* ximg = a.x + (int64_t)n_img * a.H * a.W * a.Cin;
  constexpr int kXPieces = kSiH * kSiW * 4;   // 16-byte pieces of an input chunk (720)
  constexpr int kWPieces = 9 * 16 * 4;        // ... of a weight chunk (576)
  constexpr int kXPer = (kXPieces + kSmallThreads - 1) / kSmallThreads;  // 3
  constexpr int kWPer = (kWPieces + kSmallThreads - 1) / kSmallThreads;  // 3
  u32x4 rx[kXPer], rw[kWPer];
  auto load = [&](int ch) {
#pragma unroll
    for (int i = 0; i < kXPer; ++i) {
      const int pid = tid + kSmallThreads * i;
      rx[i] = u32x4{0u, 0u, 0u, 0u};
      if (pid < kXPieces) {
        const int px = pid >> 2, q = pid & 3;
        const int ia = a0 - 1 + px / kSiW, ib = b0 - 1 + px % kSiW;
        const int c = ch * 32 + q * 8;
        if (ia >= 0 && ia < a.H && ib >= 0 && ib < a.W && c < a.Cin) {
          rx[i] = *reinterpret_cast<const u32x4*>(ximg + ((int64_t)ia * a.W + ib) * a.Cin + c);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kWPer; ++i) {
      const int pid = tid + kSmallThreads * i;
      if (pid < kWPieces) rw[i] = *reinterpret_cast<const u32x4*>(a.wq + ((int64_t)ch * kWPieces + pid) * 8);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < kXPer; ++i) {
      const int pid = tid + kSmallThreads * i;
      if (pid < kXPieces) *reinterpret_cast<u32x4*>(&xs[buf][(pid >> 2) * kSPitch + (pid & 3) * 8]) = rx[i];
    }
#pragma unroll
    for (int i = 0; i < kWPer; ++i) {
      const int pid = tid + kSmallThreads * i;
      if (pid < kWPieces) *reinterpret_cast<u32x4*>(&ws[buf][(pid >> 2) * kSPitch + (pid & 3) * 8]) = rw[i];
    }
  };
  // wave w: quad rows 2w, 2w + 1 (one 16-quad M tile each); lane row = quad column
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  load(0);
  store(0);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nch) load(ch + 1);
#pragma unroll
    for (int nbr = 0; nbr < 9; ++nbr) {
      const int na = nbr / 3, nb = nbr % 3;
      const bf16x8 bf = *reinterpret_cast<const bf16x8*>(&ws[buf][(nbr * 16 + fr) * kSPitch + fk]);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int qr = 2 * wave + mt;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(
            &xs[buf][((qr + na) * kSiW + fr + nb) * kSPitch + fk]);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[mt], 0, 0, 0);
      }
    }
    if (ch + 1 < nch) {
      store(buf ^ 1);
      __syncthreads();
    }
  }
  // epilogue: C column n = fr -> (phase p, channel o); rows -> quad columns (lane>>4)*4 + j.
  // Stage the block's (2 kSqH) x (2 kSqW) x Cout output pixels in LDS (xs buffer), then
  // write each output row's 2 kSqW * Cout contiguous values.
  __syncthreads();
  __hip_bfloat16* os = &xs[0][0];
  const int Co = a.Cout, OW = 2 * kSqW;
  const int p = fr / Co, o = fr - p * Co;
  if (p < 4) {
    const float bo = a.bias ? a.bias[o] : 0.f;
    const int r = p >> 1, s = p & 1;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qr = 2 * wave + mt, qc = (lane >> 4) * 4 + j;
        os[((2 * qr + r) * OW + 2 * qc + s) * Co + o] = __float2bfloat16(acc[mt][j] + bo);
      }
  }
  __syncthreads();
  const int H2 = 2 * a.H, W2 = 2 * a.W;
  const int ocols = min(OW, W2 - 2 * b0);   // valid output columns of this tile
  const int orows = min(2 * kSqH, H2 - 2 * a0);
  const int rowel = ocols * Co;             // contiguous elements per output row
  for (int e = tid; e < orows * rowel; e += kSmallThreads) {
    const int rr = e / rowel, k = e - rr * rowel;
    a.y[(((int64_t)n_img * H2 + 2 * a0 + rr) * W2 + 2 * b0) * Co + k] = os[rr * OW * Co + k];
  }
}

// ----------------------------------------------------- small-Cout decoder layer, backward
// With the quad view of the forward (Y[quad, n] = sum_{nbr, c} X[quad + nbr - 1, c]
// Wq[nbr, c, n], n = p·Cout + o), input pixel (a, b) meets quad (a - na + 1, b - nb + 1)
// through neighbour nbr = (na, nb), so
//   dgrad  gX[(a, b), c]   = sum_{nbr, n} gYq[(a, b) - nbr + 1, n] Wq[nbr, c, n]   (K = 9 x 16)
//   wgrad  gWq[nbr, c, n]  = sum_{(a, b)} X[(a, b), c] gYq[(a, b) - nbr + 1, n]   (K = pixels)
//   bias   gb[o]           = sum_{quads, p} gYq[quad, p·Cout + o]
// Both kernels walk tiles of kBwTA x kBwTB input pixels of one image and stage the
// (kBwTA + 2) x (kBwTB + 2) gradient quads around the tile in LDS as [quad][16] bf16.
// dgrad writes 2·Cin bytes per pixel (the layer's HBM floor), wgrad reads them: each is a
// single pass over the 2·N·H·W·Cin-byte activation.
constexpr int kBwTA = 2, kBwTB = 32;                      // input pixels per tile (rows x cols)
constexpr int kBwPix = kBwTA * kBwTB;                     // 64 = 4 MFMA tiles of 16 pixels
constexpr int kBwQW = kBwTB + 2, kBwQuads = (kBwTA + 2) * kBwQW;   // 136 staged quads
constexpr int kBwMaxCt = 16;                              // 16-channel tiles (Cin + 1 <= 256)
constexpr int kDgThreads = 256, kWgThreads = 512;
constexpr int kDgK = 160;                                 // dgrad K: 9 nbr x 16, padded to 5 x 32

struct DeconvSmallBwdArgs {
  const __hip_bfloat16* x;    // (N, H, W, Cin) channels-last
  const __hip_bfloat16* gy;   // (N, 2H, 2W, Cout) channels-last
  const __hip_bfloat16* wd;   // dgrad weight [nct·16][kDgK]
  __hip_bfloat16* gx;         // (N, H, W, Cin) channels-last
  float* part;                // wgrad partials [blocks][Cin·Cout·16 + 4·Cout]
  int H, W, Cin, Cout, nct, tiles_w;
  int tiles_img;              // tiles per image
  int64_t ntiles;
};

// wd[c][nbr·16 + n] = Wq[nbr, c, n] (0 past Cin, past 4·Cout and for nbr = 9): the dgrad
// A operand, 8 consecutive K of one channel per 16-byte load
__global__ void deconv_small_pack_dgrad_kernel(const __hip_bfloat16* w, __hip_bfloat16* wd, int Cin, int Cout,
                                               int rows) {
  const int total = rows * kDgK;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i / kDgK, k = i - c * kDgK, nbr = k >> 4, n = k & 15;
    const int p = n / Cout, o = n - p * Cout;
    float v = 0.f;
    if (c < Cin && p < 4 && nbr < 9) {
      const int r = p >> 1, s = p & 1, di = nbr / 3 - 1, dj = nbr % 3 - 1;
      if ((di == r - 1 || di == r) && (dj == s - 1 || dj == s))
        v = __bfloat162float(w[((c * Cout + (n - p * Cout)) * 4 + 1 - 2 * di + r) * 4 + 1 - 2 * dj + s]);
    }
    (void)o;
    wd[i] = __float2bfloat16(v);
  }
}

// gYq of the quads around one tile: (kBwTA + 2) quad rows = 2 (kBwTA + 2) gradient rows,
// each a contiguous run of 2 (kBwTB + 2) Cout values; zero outside the image.  load() takes
// a tile's values into registers (issued a tile ahead, so the loads fly during the current
// tile's MFMAs), store() writes them to the [quad][16] LDS image.
template <int Co, int NTHR>
struct QuadStage {
  static constexpr int L = 2 * kBwQW * Co;
  static constexpr int kN = 2 * (kBwTA + 2) * L;
  static constexpr int kPer = (kN + NTHR - 1) / NTHR;
  __hip_bfloat16 v[kPer];
  __device__ __forceinline__ void load(const DeconvSmallBwdArgs& a, int64_t n_img, int a0, int b0, int tid) {
    const int H2 = 2 * a.H, W2 = 2 * a.W;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * NTHR;
      const int row = e / L, k = e - row * L;
      const int qi = row >> 1, r = row & 1, pix = k / Co, o = k - pix * Co, qj = pix >> 1, s = pix & 1;
      const int qa = a0 - 1 + qi, qb = b0 - 1 + qj;
      v[i] = __float2bfloat16(0.f);
      if (e < kN && qa >= 0 && qa < a.H && qb >= 0 && qb < a.W)
        v[i] = a.gy[((n_img * H2 + 2 * qa + r) * W2 + 2 * qb + s) * Co + o];
    }
  }
  __device__ __forceinline__ void store(__hip_bfloat16* qs, int tid) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * NTHR;
      const int row = e / L, k = e - row * L;
      const int qi = row >> 1, r = row & 1, pix = k / Co, o = k - pix * Co, qj = pix >> 1, s = pix & 1;
      if (e < kN) qs[(qi * kBwQW + qj) * 16 + (2 * r + s) * Co + o] = v[i];
    }
  }
};

struct TileAt {
  int64_t n;
  int a0, b0;
};
__device__ __forceinline__ TileAt tile_at(const DeconvSmallBwdArgs& a, int64_t tile) {
  const int64_t n = tile / a.tiles_img;
  const int t = (int)(tile - n * a.tiles_img);
  return TileAt{n, (t / a.tiles_w) * kBwTA, (t % a.tiles_w) * kBwTB};
}

// dgrad.  4 waves; wave w owns channel tiles w, w + 4, ... and keeps their weight
// fragments in registers for the whole (persistent) block.  Per 16-pixel MFMA tile: five
// 16-byte quad reads (B operand: K = 8 consecutive (nbr, n) of one pixel), five MFMAs per
// channel tile (C rows = 4 consecutive channels per lane -> one 8-byte LDS store), then the
// staged [64 pixels][Cin] tile leaves as 16-byte stores of whole pixel rows.
// MASK: gx is masked by x > 0 (the ReLU in front of the layer,
// LV_DECONV_MASK_GX); the tile's x pieces are loaded right after the quad stage, so their
// latency hides under the tile's MFMAs.
template <int CO, bool MASK>
__global__ __launch_bounds__(kDgThreads) void deconv_small_dgrad_kernel(DeconvSmallBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 sm[];
  __hip_bfloat16* qs = sm;                               // [kBwQuads + 1][16], last = zeros
  __hip_bfloat16* os = sm + (kBwQuads + 1) * 16;         // [kBwPix][pitch]
  const int pitch = a.nct * 16 + 8;
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  for (int i = tid; i < (kBwQuads + 1) * 2; i += kDgThreads)
    reinterpret_cast<u32x4*>(qs)[i] = u32x4{0u, 0u, 0u, 0u};
  constexpr int kPer = kBwMaxCt / 4;
  bf16x8 wf[kPer][5];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int ct = wave + 4 * i;
    if (ct < a.nct) {
#pragma unroll
      for (int st = 0; st < 5; ++st)
        wf[i][st] = *reinterpret_cast<const bf16x8*>(a.wd + (ct * 16 + fr) * kDgK + st * 32 + g * 8);
    }
  }
  // per lane: the quad offsets (elements) of its B fragments, relative to the pixel's quad
  int boff[5];
#pragma unroll
  for (int st = 0; st < 5; ++st) {
    const int nbr = 2 * st + (g >> 1);
    const int na = nbr / 3, nb = nbr % 3;
    boff[st] = nbr < 9 ? ((2 - na) * kBwQW + (2 - nb)) * 16 + 8 * (g & 1) : -1;
  }
  const int G8 = a.Cin / 8;
  QuadStage<CO, kDgThreads> qst;
  int64_t tile = blockIdx.x;
  TileAt at = tile_at(a, tile);
  if (tile < a.ntiles) qst.load(a, at.n, at.a0, at.b0, tid);
  __syncthreads();  // the zeroed quad image
  constexpr int kXm = MASK ? (kBwPix * kBwMaxCt * 2 + kDgThreads - 1) / kDgThreads : 1;  // 8
  u32x4 xm[kXm];
  for (; tile < a.ntiles; tile += gridDim.x) {
    const int64_t n_img = at.n;
    const int a0 = at.a0, b0 = at.b0;
    qst.store(qs, tid);
    __syncthreads();
    if constexpr (MASK) {  // this tile's x pieces, in the store loop's order
#pragma unroll
      for (int i = 0; i < kXm; ++i) {
        const int e = tid + i * kDgThreads;
        const int px = e / G8, q = e - px * G8;
        const int ia = a0 + px / kBwTB, ib = b0 + px % kBwTB;
        xm[i] = u32x4{0u, 0u, 0u, 0u};
        if (e < kBwPix * G8 && ia < a.H && ib < a.W)
          xm[i] = *reinterpret_cast<const u32x4*>(a.x + ((n_img * a.H + ia) * a.W + ib) * a.Cin + 8 * q);
      }
    }
    if (tile + gridDim.x < a.ntiles) {  // next tile's quads in flight during this tile's MFMAs
      at = tile_at(a, tile + gridDim.x);
      qst.load(a, at.n, at.a0, at.b0, tid);
    }
#pragma unroll
    for (int mt = 0; mt < kBwPix / 16; ++mt) {
      const int ta = mt >> 1, tb = 16 * (mt & 1) + fr;
      const int qbase = (ta * kBwQW + tb) * 16;
      bf16x8 gf[5];
#pragma unroll
      for (int st = 0; st < 5; ++st)
        gf[st] = *reinterpret_cast<const bf16x8*>(qs + (boff[st] >= 0 ? qbase + boff[st] : kBwQuads * 16));
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int ct = wave + 4 * i;
        if (ct < a.nct) {
          f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int st = 0; st < 5; ++st) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][st], gf[st], acc, 0, 0, 0);
          __hip_bfloat16 v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = __float2bfloat16(acc[j]);
          *reinterpret_cast<uint2*>(os + (mt * 16 + fr) * pitch + ct * 16 + 4 * g) = *reinterpret_cast<const uint2*>(v);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kXm; ++i) {
      const int e = tid + i * kDgThreads;
      if (e >= kBwPix * G8) break;
      const int px = e / G8, q = e - px * G8;
      const int ia = a0 + px / kBwTB, ib = b0 + px % kBwTB;
      if (ia < a.H && ib < a.W) {
        const int64_t off = ((n_img * a.H + ia) * a.W + ib) * a.Cin + 8 * q;
        u32x4 v = *reinterpret_cast<const u32x4*>(os + px * pitch + 8 * q);
        if constexpr (MASK) v = relu_mask_bf16x8(v, xm[i]);
        *reinterpret_cast<u32x4*>(a.gx + off) = v;
      }
    }
    if constexpr (!MASK) {  // kXm = 1 covers only the first pass: the rest of the tile
      for (int e = tid + kDgThreads; e < kBwPix * G8; e += kDgThreads) {
        const int px = e / G8, q = e - px * G8;
        const int ia = a0 + px / kBwTB, ib = b0 + px % kBwTB;
        if (ia < a.H && ib < a.W)
          *reinterpret_cast<u32x4*>(a.gx + ((n_img * a.H + ia) * a.W + ib) * a.Cin + 8 * q) =
              *reinterpret_cast<const u32x4*>(os + px * pitch + 8 * q);
      }
    }
  }
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// 8 K values (pixels) of one column from two 4-row transposed reads (ds_read_b64_tr_b16):
// lane 4q + p of each 16-lane group names row q, columns 4p..4p+3 of a 4 x 16 block; lane i
// of the group receives column i of the 4 rows.  `addr0`/`addr1` are this lane's element
// addresses for the rows k0 + q and k0 + 4 + q.
__device__ __forceinline__ bf16x8 tr_read8(const __hip_bfloat16* addr0, const __hip_bfloat16* addr1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(as_lds(addr0)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(as_lds(addr1)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// wgrad + bias.  8 waves; wave w accumulates channel tiles w and w + 8 against all nine
// neighbours (18 16x16 fp32 tiles).  Per tile row of 32 pixels (one MFMA K step): the A
// operand (32 pixels x 16 channels of X, pixel-major in LDS) and the B operands (32 pixels
// x 16 quad values per neighbour) are transposed reads.  Column Cin of the staged X is 1
// on valid pixels, so channel row Cin of the centre neighbour accumulates the bias
// gradient.  The block's sums leave once, in gw order, as fp32 partials.
template <int CO>
__global__ __launch_bounds__(kWgThreads) void deconv_small_wgrad_kernel(DeconvSmallBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) __hip_bfloat16 sm[];
  __hip_bfloat16* qs = sm;                          // [kBwQuads][16]
  __hip_bfloat16* xs = sm + kBwQuads * 16;          // [kBwPix][xpitch]
  const int xpitch = a.nct * 16 + 8;
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4, q4 = fr >> 2, p4 = fr & 3;
  constexpr int kPer = kBwMaxCt / 8;
  f32x4 acc[kPer][9];
#pragma unroll
  for (int i = 0; i < kPer; ++i)
#pragma unroll
    for (int nb = 0; nb < 9; ++nb) acc[i][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int G8 = a.nct * 2;   // 8-channel pieces per staged pixel
  constexpr int kXPer = kBwPix * 2 * kBwMaxCt / kWgThreads;
  u32x4 xv[kXPer];
  auto load_x = [&](const TileAt& t) {
#pragma unroll
    for (int i = 0; i < kXPer; ++i) {
      const int e = tid + i * kWgThreads;
      const int px = e / G8, c = 8 * (e - px * G8);
      const int ia = t.a0 + px / kBwTB, ib = t.b0 + px % kBwTB;
      xv[i] = u32x4{0u, 0u, 0u, 0u};
      if (e < kBwPix * G8 && ia < a.H && ib < a.W) {
        if (c < a.Cin) {
          xv[i] = *reinterpret_cast<const u32x4*>(a.x + ((t.n * a.H + ia) * a.W + ib) * a.Cin + c);
        }
        else if (c == a.Cin)
          xv[i][0] = 0x3f80u;  // bf16 1.0 in element 0 (channel Cin)
      }
    }
  };
  QuadStage<CO, kWgThreads> qst;
  int64_t tile = blockIdx.x;
  TileAt at = tile_at(a, tile);
  if (tile < a.ntiles) {
    qst.load(a, at.n, at.a0, at.b0, tid);
    load_x(at);
  }
  for (; tile < a.ntiles; tile += gridDim.x) {
    qst.store(qs, tid);
#pragma unroll
    for (int i = 0; i < kXPer; ++i) {
      const int e = tid + i * kWgThreads;
      const int px = e / G8, c = 8 * (e - px * G8);
      if (e < kBwPix * G8) *reinterpret_cast<u32x4*>(xs + px * xpitch + c) = xv[i];
    }
    __syncthreads();
    if (tile + gridDim.x < a.ntiles) {  // next tile in flight during this tile's MFMAs
      at = tile_at(a, tile + gridDim.x);
      qst.load(a, at.n, at.a0, at.b0, tid);
      load_x(at);
    }
#pragma unroll
    for (int ks = 0; ks < kBwTA; ++ks) {
      bf16x8 af[kPer];
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int ct = wave + 8 * i;
        if (ct < a.nct) {
          const __hip_bfloat16* base = xs + (ks * kBwTB + 8 * g + q4) * xpitch + ct * 16 + 4 * p4;
          af[i] = tr_read8(base, base + 4 * xpitch);
        }
      }
#pragma unroll
      for (int nbr = 0; nbr < 9; ++nbr) {
        const int na = nbr / 3, nb = nbr % 3;
        const __hip_bfloat16* base = qs + ((ks - na + 2) * kBwQW + 8 * g + q4 - nb + 2) * 16 + 4 * p4;
        const bf16x8 bfr = tr_read8(base, base + 4 * 16);
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
          const int ct = wave + 8 * i;
          if (ct < a.nct) acc[i][nbr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][nbr], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // C: column n = fr -> (phase p, channel o); rows c = ct·16 + 4g + j
  constexpr int Co = CO;
  const int p = fr / Co, o = fr - p * Co;
  if (p >= 4) return;
  const int r = p >> 1, s = p & 1;
  float* part = a.part + (int64_t)blockIdx.x * ((int64_t)a.Cin * Co * 16 + 4 * Co);
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int ct = wave + 8 * i;
    if (ct >= a.nct) continue;
#pragma unroll
    for (int nbr = 0; nbr < 9; ++nbr) {
      const int di = nbr / 3 - 1, dj = nbr % 3 - 1;
      if (!((di == r - 1 || di == r) && (dj == s - 1 || dj == s))) continue;
      const int ku = 1 - 2 * di + r, kv = 1 - 2 * dj + s;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = ct * 16 + 4 * g + j;
        if (c < a.Cin)
          part[((c * Co + o) * 4 + ku) * 4 + kv] = acc[i][nbr][j];
        else if (c == a.Cin && nbr == 4)
          part[a.Cin * Co * 16 + p * Co + o] = acc[i][nbr][j];
      }
    }
  }
}

// out[e] = sum_{b < nblk} part[b·stride + e] for e < E, in a fixed order: four slices
// (b mod 4), each an 8-way unrolled sum (8 independent loads in flight per thread), then
// the slices added in order.  64 consecutive outputs per block: coalesced 256-byte rows.
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* part, int nblk, int64_t stride, int E,
                                                           float* out) {
  __shared__ float red[4][64];
  const int t = (int)threadIdx.x, el = t & 63, sl = t >> 6;
  const int e = blockIdx.x * 64 + el;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (e < E) {
    int b = sl;
    for (; b + 28 < nblk; b += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += part[(int64_t)(b + 4 * u) * stride + e];
    }
    for (; b < nblk; b += 4) acc[0] += part[(int64_t)b * stride + e];
  }
  red[sl][el] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (sl == 0 && e < E) out[e] = (red[0][el] + red[1][el]) + (red[2][el] + red[3][el]);
}

// gw (bf16, the weight's layout) and gb[o] = sum_p of the reduced wgrad sums
__global__ void deconv_small_wgrad_finish_kernel(const float* red, int Cin, int Cout, __hip_bfloat16* gw, float* gb) {
  const int nw = Cin * Cout * 16;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nw) {
    gw[e] = __float2bfloat16(red[e]);
  } else if (e < nw + Cout && gb) {
    const int o = e - nw;
    gb[o] = ((red[nw + o] + red[nw + Cout + o]) + red[nw + 2 * Cout + o]) + red[nw + 3 * Cout + o];
  }
}

// ----------------------------------------------------- per-channel sum (bias gradient)
// out[c] = sum_p g[p, c] over a channels-last (P, C) bf16 tensor, C % 8 == 0: each block
// sums a contiguous row range (thread = 8 channels x every R-th row), a fixed-order LDS
// combine, then a second kernel adds the per-block partials in block order.
constexpr int kCsThreads = 256, kCsMaxBlocks = 1024;

__global__ __launch_bounds__(kCsThreads) void channel_sum_part_kernel(const __hip_bfloat16* g, float* part, int64_t P,
                                                                      int C, int64_t rows_per_blk) {
  __shared__ float red[kCsThreads * 8];
  const int G = C / 8, R = kCsThreads / G;
  const int tid = (int)threadIdx.x, cg = tid % G, rr = tid / G;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk, r1 = min(P, r0 + rows_per_blk);
  if (rr < R) {
    auto add = [&](const u32x4 v) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[2 * e] += __uint_as_float(v[e] << 16);
        s[2 * e + 1] += __uint_as_float(v[e] & 0xffff0000u);
      }
    };
    int64_t row = r0 + rr;
    for (; row + 3 * R < r1; row += 4 * R) {  // four rows in flight
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const u32x4*>(g + (row + u * R) * C + 8 * cg);
#pragma unroll
      for (int u = 0; u < 4; ++u) add(v[u]);
    }
    for (; row < r1; row += R) add(*reinterpret_cast<const u32x4*>(g + row * C + 8 * cg));
#pragma unroll
    for (int e = 0; e < 8; ++e) red[rr * C + 8 * cg + e] = s[e];
  }
  __syncthreads();
  for (int c = tid; c < C; c += kCsThreads) {
    float t = 0.f;
    for (int k = 0; k < R; ++k) t += red[k * C + c];
    part[(int64_t)blockIdx.x * C + c] = t;
  }
}

}  // namespace
}  // namespace lv

using namespace lv;

// default forward variant: v2 with 128-row block tiles (2 x 4 waves, 104 VGPRs: two blocks
// per CU, so one block's epilogue stores overlap the other's MFMAs), 2-stage LDS-DMA ring,
// XCD-grouped phases.  Batch 512, 200 -> 200 at H = 4 / 8 / 16: 26 / 65 / 260 us against
// 256-row tiles' 38 / 74 / 284 and v1's 43 / 88 / 344, all bitwise equal
// (profiles/r03_deconv_v2.txt).
constexpr int kDeconvAutoBM = 6;
// fp32 default: 128-row tiles, 2-stage ring, SIMD-balanced wave tiling (variant 5): 16 -> 32
// 1,684-1,693 -> 1,600-1,607 us, 8 -> 16 463-471 -> 451-453, 4 -> 8 144 -> 132-134
// (profiles/r06_ab_deconv_f32_rm.txt); the same remap is neutral on the bf16 kernel (bm = 8)
constexpr int kDeconvF32Default = 5;
#ifdef LV_AB_KNOBS
int deconv_env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}
#define LV_DECONV_KNOB(name, dflt) deconv_env_int(name, dflt)
#else
#define LV_DECONV_KNOB(name, dflt) (dflt)
#endif

namespace {
template <int S, bool XCD, int BM = 256, bool RM = false>
int launch_deconv_v2(const DeconvArgs& a, hipStream_t st) {
  const int64_t tiles = (a.M + BM - 1) / BM;
  if constexpr (XCD)
    hipLaunchKernelGGL((deconv_mfma2_kernel<S, true, BM, RM>), dim3((unsigned)(4 * ((tiles + 7) / 8 * 8))), dim3(512),
                       (DeconvV2<S, BM>::kLds), st, a);
  else
    hipLaunchKernelGGL((deconv_mfma2_kernel<S, false, BM>), dim3((unsigned)tiles, 4), dim3(512),
                       (DeconvV2<S, BM>::kLds), st, a);
  LV_RETURN_LAUNCH("deconv_mfma2_kernel");
}
template <int BM, int S, bool RM = false>
int launch_deconv_f32(const DeconvF32Args& a, hipStream_t st) {
  const int64_t tiles = (a.M + BM - 1) / BM;
  hipLaunchKernelGGL((deconv_mfma_f32_kernel<BM, S, RM>), dim3((unsigned)(4 * ((tiles + 7) / 8 * 8))), dim3(512),
                     (DeconvF32<BM, S>::kLds), st, a);
  LV_RETURN_LAUNCH("deconv_mfma_f32_kernel");
}
template <int BM>
int launch_deconv(const DeconvArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(deconv_mfma_kernel<BM>, dim3((unsigned)((a.M + BM - 1) / BM), 4),
                     dim3(DeconvTile<BM>::kThreads), DeconvTile<BM>::kLds, st, a);
  LV_RETURN_LAUNCH("deconv_mfma_kernel");
}
}  // namespace

extern "C" {
#ifdef LV_AB_KNOBS
// A/B build only (liblievae_hip_ab.so, tools/deconv_bench.py): an explicit kernel variant
int lv_deconv4s2_fwd_bf16_tile(const void* x, const void* wt, const float* bias, void* y, int64_t N,
                               int H, int W, int Cin, int Cout, int bm, void* stream);
#endif

size_t lv_deconv4s2_packed_weight_elems(int Cin) { return 4 * (size_t)kBN * 4 * (size_t)Cin + 32; }

int lv_deconv4s2_pack_weight_bf16(const void* w, void* wt, int Cin, int Cout, void* stream) {
  clear_error();
  LV_CHECK_ARG(w && wt, "null pointer");
  LV_CHECK_ARG(Cin > 0 && Cin % 8 == 0, "Cin must be a positive multiple of 8 (got %d)", Cin);
  LV_CHECK_ARG(Cout > 0 && Cout <= kBN && Cout % 4 == 0, "Cout must be a multiple of 4 in [4, %d] (got %d)", kBN, Cout);
  LV_CHECK_ARG((int64_t)Cin * Cout * 16 < (1ll << 31), "weight too large");
  hipLaunchKernelGGL(deconv_pack_kernel, dim3(ceil_div(4 * kBN * (Cin / 2), 256)), dim3(256), 0, (hipStream_t)stream,
                     (const __hip_bfloat16*)w, (__hip_bfloat16*)wt, Cin, Cout);
  LV_RETURN_LAUNCH("deconv_pack_kernel");
}

int lv_deconv4s2_fwd_bf16(const void* x, const void* wt, const float* bias, void* y, int64_t N,
                          int H, int W, int Cin, int Cout, void* stream) {
  return lv_deconv4s2_fwd_bf16_ex(x, wt, bias, y, N, H, W, Cin, Cout, 0, stream);
}

static int deconv_fwd(const void* x, const void* wt, const float* bias, void* y, int64_t N, int H, int W,
                      int Cin, int Cout, int bm, int flags, void* stream) {
  clear_error();
  LV_CHECK_ARG((flags & ~LV_DECONV_RELU_OUT) == 0, "flags: only LV_DECONV_RELU_OUT for this layer");
  LV_CHECK_ARG(N >= 0 && H > 0 && W > 0, "bad shape");
  LV_CHECK_ARG(Cin > 0 && Cin % 8 == 0, "Cin must be a positive multiple of 8 (got %d)", Cin);
  LV_CHECK_ARG(Cout > 0 && Cout <= kBN && Cout % 4 == 0, "Cout must be a multiple of 4 in [4, %d] (got %d)", kBN, Cout);
  if (N == 0) return LV_OK;
  LV_CHECK_ARG(x && wt && y, "null pointer");
  const int64_t M = N * H * W;
  LV_CHECK_ARG((M + 127) / 128 <= 0x7fffffff, "batch too large");
  LV_CHECK_ARG(bm == 0 || bm == 128 || bm == 256 || (bm >= 2 && bm <= 8),
               "variant must be 0 (auto), 128 / 256 (v1 tile rows) or 2 / 3 (v2 stages), 4 / 5 (+ XCD order)");
  DeconvArgs a{(const __hip_bfloat16*)x, (const __hip_bfloat16*)wt, bias, (__hip_bfloat16*)y, M, H, W, Cin, Cout,
               (flags & LV_DECONV_RELU_OUT) ? 1 : 0};
  if (bm == 0) bm = kDeconvAutoBM;
  LV_CHECK_ARG(Cout % 8 == 0 || (bm >= 2 && bm <= 8), "the v1 kernels need Cout %% 8 == 0 (got %d)", Cout);
  if (bm == 2) return launch_deconv_v2<2, false>(a, (hipStream_t)stream);
  if (bm == 3) return launch_deconv_v2<3, false>(a, (hipStream_t)stream);
  if (bm == 4) return launch_deconv_v2<2, true>(a, (hipStream_t)stream);
  if (bm == 5) return launch_deconv_v2<3, true>(a, (hipStream_t)stream);
  if (bm == 6) return launch_deconv_v2<2, true, 128>(a, (hipStream_t)stream);
  if (bm == 7) return launch_deconv_v2<3, true, 128>(a, (hipStream_t)stream);
  if (bm == 8) return launch_deconv_v2<2, true, 128, true>(a, (hipStream_t)stream);
  return bm == 256 ? launch_deconv<256>(a, (hipStream_t)stream) : launch_deconv<128>(a, (hipStream_t)stream);
}
#ifdef LV_AB_KNOBS
// bm: 0 = the default, 128 / 256 = v1 (register-staged double buffer) with that pixel-tile
// height, 2 / 3 = v2 (LDS-DMA ring of that many stages, 4 x 2 wave tiling), 4 / 5 = v2 with
// 2 / 3 stages and XCD-grouped phases, 6 / 7 = the same with 128-row block tiles, 8 = 6 with
// SIMD-balanced wave tiling
int lv_deconv4s2_fwd_bf16_tile(const void* x, const void* wt, const float* bias, void* y, int64_t N,
                               int H, int W, int Cin, int Cout, int bm, void* stream) {
  return deconv_fwd(x, wt, bias, y, N, H, W, Cin, Cout, bm, 0, stream);
}
#endif
int lv_deconv4s2_fwd_bf16_ex(const void* x, const void* wt, const float* bias, void* y, int64_t N,
                             int H, int W, int Cin, int Cout, int flags, void* stream) {
  return deconv_fwd(x, wt, bias, y, N, H, W, Cin, Cout, 0, flags, stream);
}

size_t lv_deconv4s2_packed_weight_elems_f32(int Cin) { return 4 * (size_t)kBN * 4 * (size_t)Cin + 16; }

int lv_deconv4s2_pack_weight_f32(const float* w, float* wt, int Cin, int Cout, void* stream) {
  clear_error();
  LV_CHECK_ARG(w && wt, "null pointer");
  LV_CHECK_ARG(Cin > 0 && Cin % 4 == 0, "Cin must be a positive multiple of 4 (got %d)", Cin);
  LV_CHECK_ARG(Cout > 0 && Cout <= kBN, "Cout must be in [1, %d] (got %d)", kBN, Cout);
  LV_CHECK_ARG((int64_t)Cin * Cout * 16 < (1ll << 31), "weight too large");
  hipLaunchKernelGGL(deconv_pack_f32_kernel, dim3(ceil_div(4 * kBN * Cin, 256)), dim3(256), 0, (hipStream_t)stream,
                     w, wt, Cin, Cout);
  LV_RETURN_LAUNCH("deconv_pack_f32_kernel");
}

int lv_deconv4s2_fwd_f32(const float* x, const float* wt, const float* bias, float* y, float* y_cl, int64_t N,
                         int H, int W, int Cin, int Cout, int flags, void* stream) {
  clear_error();
  LV_CHECK_ARG((flags & ~LV_DECONV_RELU_OUT) == 0, "flags: only LV_DECONV_RELU_OUT for this layer");
  LV_CHECK_ARG(N >= 0 && H > 0 && W > 0, "bad shape");
  LV_CHECK_ARG(Cin > 0 && Cin % 4 == 0, "Cin must be a positive multiple of 4 (got %d)", Cin);
  LV_CHECK_ARG(Cout > 0 && Cout <= kBN, "Cout must be in [1, %d] (got %d)", kBN, Cout);
  if (N == 0) return LV_OK;
  LV_CHECK_ARG(x && wt && y, "null pointer");
  LV_CHECK_ARG(!y_cl || Cout % 4 == 0, "the channels-last twin needs Cout %% 4 == 0 (got %d)", Cout);
  const int64_t M = N * H * W;
  LV_CHECK_ARG(N * Cout * 4 * H * W < (1ll << 40) && (M + 127) / 128 * 4 + 32 <= 0x7fffffff, "batch too large");
  DeconvF32Args a{x, wt, bias, y, y_cl, M, H, W, Cin, Cout, (flags & LV_DECONV_RELU_OUT) ? 1 : 0};
  // A/B build: LV_DECONV_F32_VARIANT 1 = 128-row tiles, 2-stage ring (the default); 2 = 3
  // stages; 3 = 256-row tiles, 2 stages; 4 = 256 rows, 3 stages; 5 = 1 with SIMD-balanced
  // wave tiling (RM, the default); 6 = 3 with RM
  static const int kVar = LV_DECONV_KNOB("LV_DECONV_F32_VARIANT", kDeconvF32Default);
  switch (kVar) {
    case 2: return launch_deconv_f32<128, 3>(a, (hipStream_t)stream);
    case 3: return launch_deconv_f32<256, 2>(a, (hipStream_t)stream);
    case 4: return launch_deconv_f32<256, 3>(a, (hipStream_t)stream);
    case 5: return launch_deconv_f32<128, 2, true>(a, (hipStream_t)stream);
    case 6: return launch_deconv_f32<256, 2, true>(a, (hipStream_t)stream);
    default: return launch_deconv_f32<128, 2>(a, (hipStream_t)stream);
  }
}

size_t lv_deconv4s2_small_packed_weight_elems(int Cin) { return (size_t)((Cin + 31) / 32) * 9 * 16 * 32; }

int lv_deconv4s2_small_pack_weight_bf16(const void* w, void* wq, int Cin, int Cout, void* stream) {
  clear_error();
  LV_CHECK_ARG(w && wq, "null pointer");
  LV_CHECK_ARG(Cin > 0 && Cin % 8 == 0, "Cin must be a positive multiple of 8 (got %d)", Cin);
  LV_CHECK_ARG(Cout >= 1 && Cout <= kSmallMaxCout, "Cout must be in [1, %d] (got %d)", kSmallMaxCout, Cout);
  const int total = (int)lv_deconv4s2_small_packed_weight_elems(Cin);
  hipLaunchKernelGGL(deconv_small_pack_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream,
                     (const __hip_bfloat16*)w, (__hip_bfloat16*)wq, Cin, Cout);
  LV_RETURN_LAUNCH("deconv_small_pack_kernel");
}

int lv_deconv4s2_small_fwd_bf16(const void* x, const void* wq, const float* bias, void* y, int64_t N,
                                int H, int W, int Cin, int Cout, void* stream) {
  clear_error();
  LV_CHECK_ARG(N >= 0 && H > 0 && W > 0, "bad shape");
  LV_CHECK_ARG(Cin > 0 && Cin % 8 == 0, "Cin must be a positive multiple of 8 (got %d)", Cin);
  LV_CHECK_ARG(Cout >= 1 && Cout <= kSmallMaxCout, "Cout must be in [1, %d] (got %d)", kSmallMaxCout, Cout);
  LV_CHECK_ARG(N <= 65535, "batch must be <= 65535 (grid y)");
  if (N == 0) return LV_OK;
  LV_CHECK_ARG(x && wq && y, "null pointer");
  const int th = (H + kSqH - 1) / kSqH, tw = (W + kSqW - 1) / kSqW;
  DeconvSmallArgs a{(const __hip_bfloat16*)x, (const __hip_bfloat16*)wq, bias, (__hip_bfloat16*)y, H, W, Cin, Cout, tw};
  hipLaunchKernelGGL(deconv_small_kernel, dim3(th * tw, (unsigned)N), dim3(kSmallThreads), 0,
                     (hipStream_t)stream, a);
  LV_RETURN_LAUNCH("deconv_small_kernel");
}

static int small_bwd_nct(int Cin) { return (Cin + 1 + 15) / 16; }  // + the bias "ones" channel

size_t lv_deconv4s2_small_dgrad_weight_elems(int Cin) { return (size_t)small_bwd_nct(Cin) * 16 * kDgK; }

int lv_deconv4s2_small_pack_dgrad_weight_bf16(const void* w, void* wd, int Cin, int Cout, void* stream) {
  clear_error();
  LV_CHECK_ARG(w && wd, "null pointer");
  LV_CHECK_ARG(Cin > 0 && Cin % 8 == 0 && small_bwd_nct(Cin) <= kBwMaxCt,
               "Cin must be a positive multiple of 8 below %d (got %d)", 16 * kBwMaxCt, Cin);
  LV_CHECK_ARG(Cout >= 1 && Cout <= kSmallMaxCout, "Cout must be in [1, %d] (got %d)", kSmallMaxCout, Cout);
  const int rows = small_bwd_nct(Cin) * 16;
  hipLaunchKernelGGL(deconv_small_pack_dgrad_kernel, dim3(ceil_div(rows * kDgK, 256)), dim3(256), 0,
                     (hipStream_t)stream, (const __hip_bfloat16*)w, (__hip_bfloat16*)wd, Cin, Cout, rows);
  LV_RETURN_LAUNCH("deconv_small_pack_dgrad_kernel");
}

constexpr int kWgMaxBlocks = 512;  // wgrad partial slabs (workspace bound)
static int small_wgrad_blocks(int64_t ntiles) { return (int)std::min<int64_t>(ntiles, kWgMaxBlocks); }

// resident blocks of a persistent kernel on the current device (all CUs x its
// occupancy), cached per (device, kernel, threads, LDS bytes) under a mutex: launches may
// come from several host threads and devices
static int resident_blocks(const void* kern, int threads, size_t lds) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, int, size_t>, int> cache;
  const auto key = std::make_tuple(dev, kern, threads, lds);
  {
    std::lock_guard<std::mutex> lock(mu);
    const auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) != hipSuccess) per_cu = 1;
  if (dev < 0 || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  const int v = std::max(1, per_cu) * std::max(1, cus);
  std::lock_guard<std::mutex> lock(mu);
  cache[key] = v;
  return v;
}

size_t lv_deconv4s2_small_bwd_workspace_elems(int64_t N, int H, int W, int Cin, int Cout) {
  if (N <= 0 || H <= 0 || W <= 0) return 0;
  const int64_t ntiles = N * ((H + kBwTA - 1) / kBwTA) * ((W + kBwTB - 1) / kBwTB);
  return ((size_t)small_wgrad_blocks(ntiles) + 1) * ((size_t)Cin * Cout * 16 + 4 * (size_t)Cout);
}

int lv_deconv4s2_small_bwd_bf16(const void* x, const void* gy, const void* wd, void* gx, void* gw, float* gb,
                                float* ws, int64_t N, int H, int W, int Cin, int Cout, void* stream) {
  return lv_deconv4s2_small_bwd_bf16_ex(x, gy, wd, gx, gw, gb, ws, N, H, W, Cin, Cout, 0, stream);
}
int lv_deconv4s2_small_bwd_bf16_ex(const void* x, const void* gy, const void* wd, void* gx, void* gw, float* gb,
                                   float* ws, int64_t N, int H, int W, int Cin, int Cout, int flags,
                                   void* stream) {
  clear_error();
  LV_CHECK_ARG((flags & ~LV_DECONV_MASK_GX) == 0, "flags: only LV_DECONV_MASK_GX for this layer");
  LV_CHECK_ARG(N >= 0 && H > 0 && W > 0, "bad shape");
  LV_CHECK_ARG(Cin > 0 && Cin % 8 == 0 && small_bwd_nct(Cin) <= kBwMaxCt,
               "Cin must be a positive multiple of 8 below %d (got %d)", 16 * kBwMaxCt, Cin);
  LV_CHECK_ARG(Cout >= 1 && Cout <= kSmallMaxCout, "Cout must be in [1, %d] (got %d)", kSmallMaxCout, Cout);
  LV_CHECK_ARG(x && gy, "null pointer");
  LV_CHECK_ARG(!gx || wd, "gx needs the packed dgrad weight");
  LV_CHECK_ARG(!gw || ws, "gw needs the workspace");
  hipStream_t st = (hipStream_t)stream;
  const int tw = (W + kBwTB - 1) / kBwTB, th = (H + kBwTA - 1) / kBwTA;
  const int64_t ntiles = N * th * tw;
  DeconvSmallBwdArgs a{(const __hip_bfloat16*)x, (const __hip_bfloat16*)gy, (const __hip_bfloat16*)wd,
                       (__hip_bfloat16*)gx, ws, H, W, Cin, Cout, small_bwd_nct(Cin), tw, th * tw, ntiles};
  const int nw = Cin * Cout * 16;
  if (ntiles == 0) {  // empty batch: zero gradients
    if (gw) LV_CHECK_HIP(hipMemsetAsync(gw, 0, (size_t)nw * 2, st));
    if (gb) LV_CHECK_HIP(hipMemsetAsync(gb, 0, (size_t)Cout * 4, st));
    return LV_OK;
  }
  if (gx) {
    const size_t lds = ((size_t)(kBwQuads + 1) * 16 + (size_t)kBwPix * (a.nct * 16 + 8)) * 2;
    const bool mask = (flags & LV_DECONV_MASK_GX) != 0;
    auto k = mask ? (Cout == 1 ? deconv_small_dgrad_kernel<1, true> : Cout == 2 ? deconv_small_dgrad_kernel<2, true>
                     : Cout == 3 ? deconv_small_dgrad_kernel<3, true> : deconv_small_dgrad_kernel<4, true>)
                  : (Cout == 1 ? deconv_small_dgrad_kernel<1, false> : Cout == 2 ? deconv_small_dgrad_kernel<2, false>
                     : Cout == 3 ? deconv_small_dgrad_kernel<3, false> : deconv_small_dgrad_kernel<4, false>);
    const int blocks = (int)std::min<int64_t>(ntiles, resident_blocks((const void*)k, kDgThreads, lds));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(kDgThreads), lds, st, a);
    LV_CHECK_LAUNCH("deconv_small_dgrad_kernel");
  }
  LV_CHECK_ARG(gw || !gb, "gb is computed with gw");
  if (gw) {
    const size_t lds = ((size_t)kBwQuads * 16 + (size_t)kBwPix * (a.nct * 16 + 8)) * 2;
    auto k = Cout == 1 ? deconv_small_wgrad_kernel<1> : Cout == 2 ? deconv_small_wgrad_kernel<2>
           : Cout == 3 ? deconv_small_wgrad_kernel<3> : deconv_small_wgrad_kernel<4>;
    const int blocks = std::min(small_wgrad_blocks(ntiles), resident_blocks((const void*)k, kWgThreads, lds));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(kWgThreads), lds, st, a);
    LV_CHECK_LAUNCH("deconv_small_wgrad_kernel");
    const int E = nw + 4 * Cout;
    float* red = ws + (size_t)blocks * E;
    hipLaunchKernelGGL(sum_partials_kernel, dim3(ceil_div(E, 64)), dim3(256), 0, st, ws, blocks, (int64_t)E, E, red);
    LV_CHECK_LAUNCH("sum_partials_kernel");
    hipLaunchKernelGGL(deconv_small_wgrad_finish_kernel, dim3(ceil_div(nw + Cout, 256)), dim3(256), 0, st, red, Cin,
                       Cout, (__hip_bfloat16*)gw, gb);
    LV_RETURN_LAUNCH("deconv_small_wgrad_finish_kernel");
  }
  return LV_OK;
}

size_t lv_channel_sum_workspace_elems(int64_t P, int C) {
  if (P <= 0 || C <= 0) return 0;
  return ((size_t)std::min<int64_t>(kCsMaxBlocks, (P + 255) / 256) + 1) * C;
}

int lv_channel_sum_bf16(const void* g, float* out, float* ws, int64_t P, int C, void* stream) {
  clear_error();
  LV_CHECK_ARG(P >= 0 && C > 0 && C % 8 == 0 && C / 8 <= kCsThreads, "C must be a multiple of 8 in [8, %d] (got %d)",
               8 * kCsThreads, C);
  LV_CHECK_ARG(out, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (P == 0) {
    LV_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)C * 4, st));
    return LV_OK;
  }
  LV_CHECK_ARG(g && ws, "null pointer");
  const int nblk = (int)std::min<int64_t>(kCsMaxBlocks, (P + 255) / 256);
  const int64_t rows = (P + nblk - 1) / nblk;
  hipLaunchKernelGGL(channel_sum_part_kernel, dim3(nblk), dim3(kCsThreads), 0, st, (const __hip_bfloat16*)g, ws, P, C,
                     rows);
  LV_CHECK_LAUNCH("channel_sum_part_kernel");
  hipLaunchKernelGGL(sum_partials_kernel, dim3(ceil_div(C, 64)), dim3(256), 0, st, ws, nblk, (int64_t)C, C, out);
  LV_RETURN_LAUNCH("sum_partials_kernel");
}

}  // extern "C"

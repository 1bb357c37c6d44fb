#pragma once
// Backward of the group action (angle + spectrum gradients) for gfx950, instantiated once
// per l_max in action_bwd_inst.hip (-DLV_INST_L=k), plus the deterministic reduction of
// the shared-spectrum gradient.  The reference gets these from autograd through
// lie_tools.py:211-253 (wigner_d_matrix, block_wigner_matrix_multiply).
#include "action_fwd.h"

namespace lv {

// ---------------------------------------------------------------- backward
// Same decomposition as the forward tile kernel: one block per group of Sw samples, one
// wave per degree segment.  The group's upstream gradient (Sw*M*C contiguous values) is
// loaded into an LDS tile with 16-byte loads issued first thing; the per-sample
// prologue (sincos of the three angles, multiples by recurrence) runs once per
// (sample, slot) into an LDS table.  Per lane (sample, column), per degree, with
// G = gout block column:
//   P1 = Xc F, P2 = J P1, P3 = Xb P2, P4 = J P3           (forward recompute)
//   Q4 = Xa^T G, Q3 = J Q4, Q2 = Xb^T Q3, Q1 = J Q2, dF = Xc^T Q1
//   d/da = <G, Xa' P4> = <Q4, K P4>, d/db = <Q2, K P2>, d/dc = <dF, K F> (kdot)
// The dF column overwrites the lane's own G values in the tile (each degree's rows
// belong to one wave).  Angle gradients: the C lanes of a sample and the segment waves
// are summed in a fixed order in LDS and written straight to gang.  dF: per-sample
// spectrum -> the tile leaves as gF with one contiguous flush; shared spectrum -> each
// wave sums its rows over the group's samples (fixed order) into the block's LDS slab;
// blocks loop over groups (grid capped so the workspace stays
// bounded), write their slab to the workspace once, and action_bwd_reduce_kernel sums
// the slabs in block order.  No atomics: bitwise reproducible.
// FM (spectrum mode): kBwdFSample per-sample spectrum, kBwdFShared shared spectrum with
// its slices and the dF slab in LDS, kBwdFSharedGlobal shared spectrum read from global
// memory and the slab accumulated in place in the block's workspace row -- the fallback
// for tiles too large to leave room for both (large C at high l); same summation order,
// so bitwise equal to kBwdFShared for the same plan.
constexpr int kBwdFSample = 0, kBwdFShared = 1, kBwdFSharedGlobal = 2;
constexpr int kBwdVarJit = 1;  // ActionBwdArgs::variant: row-pair reads of F and G (wide kernel)
// one-group blocks' post-chain slab pass (A/B): flat element list over the wave's degrees
// (else one pass set per degree), and write-through (sc1) slab stores (else plain)
constexpr int kBwdVarSlabFlat = 2, kBwdVarSlabWT = 4;
// one-group compile-time-C blocks: the barrier after the prologue split in two, so each
// wave's first (largest) degree computes its forward recompute P1..P4 -- which needs the
// multiples and the spectrum, not the gradient tile -- while the tile's LDS-DMA is in flight
constexpr int kBwdVarSplit = 8;
// prologue tasks spread over the block's waves (see action_bwd_tile_kernel)
constexpr int kBwdVarSpread = 16;
struct ActionBwdArgs {
  const float* ang;
  const float* F;
  int64_t Fstride;
  const float* gout;
  float* gang;         // may be null when v is set (fused: the angle gradient stays in LDS)
  const float* v;      // fused exp -> ZYZ VJP in the tail (lv_fused_exp_action_bwd), or null
  const float* mu;     // (n,3,3) or null
  float* gv;
  float* gmu;
  float* gF;           // per-sample spectrum: written directly
  float* ws_F;         // [gridDim.x][M*C] (shared F only)
  int64_t n;
  int64_t MC;
  int64_t groups;      // ceil(n / Sw); block b takes groups b, b + gridDim.x, ...
  int C, Sw, transpose;
  int fpitch;          // floats per wave-private spectrum slice in LDS
  int prio;            // 2: group load + prologue at s_setprio 3, chain at 0 (A/B: 0 off)
  int slab_chunked;    // kBwdFShared slab layout: 0 [block][M*C], 1 [M*C/16][block][16]
  int variant;         // kernel variant bits (kBwdVar*)
  unsigned long long* stamps;  // phase timestamps (A/B timeline tool; null in the product)
  int seg_lo[kMaxSeg + 1];      // contiguous degree ranges (run-time-C kernel, LDS spectrum)
  unsigned seg_mask[kMaxSeg];   // degree set of wave k (bit l = degree l)
};

// Chunk-major dF slabs (slab_chunked): element e of block b at
// ((e / 16) * gridDim.x + b) * 16 + e % 16, so that the reduce reads each 16-element chunk's
// slabs as one contiguous run (action_bwd_reduce3_kernel).
constexpr int kSlabChunk = 16;
__host__ __device__ inline int64_t slab_chunks(int64_t MC) { return (MC + kSlabChunk - 1) / kSlabChunk; }

// LDS floats of the backward tile kernel beyond the gout tile.
__host__ __device__ inline int bwd_trig_floats(int Sw, int L) {
  return Sw * (6 * ((L + 1 + 3) & ~3) + 4);  // TrigLds<L>::kRow per sample
}

// One Euler slot's multiples for degree l (f <= l), fetched from the LDS table with
// 16-byte reads right before use, so that at most one slot's are live in registers.
template <int l>
struct Mult {
  float c[l + 1], s[l + 1];
};
template <int l, int A, int LT>
__device__ __forceinline__ Mult<l> mult_lds(const float* tj) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int TP = TrigLds<LT>::TP;
  Mult<l> m;
  sfor<(l + 4) / 4>([&](auto K) {
    constexpr int k4 = LV_CV(K);
    const f4 cv = *reinterpret_cast<const f4*>(tj + 2 * A * TP + 4 * k4);
    const f4 sv = *reinterpret_cast<const f4*>(tj + (2 * A + 1) * TP + 4 * k4);
    sfor<4>([&](auto I) {
      constexpr int f = 4 * k4 + LV_CV(I);
      if constexpr (f <= l) {
        m.c[f] = cv[LV_CV(I)];
        m.s[f] = sv[LV_CV(I)];
      }
    });
  });
  return m;
}
// y = X x, y = X^T x and <g, X' x> on one slot's multiples (the arithmetic of xrot,
// xrot_t and xrot_dot_deriv in action_chain.h, operation for operation).
template <int l>
__device__ __forceinline__ void xm(const Mult<l>& m, const float (&x)[2 * l + 1], float (&y)[2 * l + 1]) {
  sfor<2 * l + 1>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    if constexpr (f == 0) y[i] = x[i];
    else if constexpr (f > 0) y[i] = fmaf(m.c[f], x[i], m.s[f] * x[2 * l - i]);
    else y[i] = fmaf(m.c[-f], x[i], -(m.s[-f] * x[2 * l - i]));
  });
}
template <int l>
__device__ __forceinline__ void xm_t(const Mult<l>& m, const float (&x)[2 * l + 1], float (&y)[2 * l + 1]) {
  sfor<2 * l + 1>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    if constexpr (f == 0) y[i] = x[i];
    else if constexpr (f > 0) y[i] = fmaf(m.c[f], x[i], -(m.s[f] * x[2 * l - i]));
    else y[i] = fmaf(m.c[-f], x[i], m.s[-f] * x[2 * l - i]);
  });
}
// y = X x / y = X^T x with x read from memory (LDS) in row pairs (i, 2l-i) right where the
// product needs them: no (2l+1)-register copy of x stays live beside the chain's arrays.
// Same arithmetic as xm / xm_t.
template <int l, bool T>
__device__ __forceinline__ void xm_mem(const Mult<l>& m, const float* x, int stride, float (&y)[2 * l + 1]) {
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    const float a = x[i * stride], b = x[(2 * l - i) * stride];
    if constexpr (T) {
      y[i] = fmaf(m.c[f], a, -(m.s[f] * b));
      y[2 * l - i] = fmaf(m.c[f], b, m.s[f] * a);
    } else {
      y[i] = fmaf(m.c[f], a, m.s[f] * b);
      y[2 * l - i] = fmaf(m.c[f], b, -(m.s[f] * a));
    }
  });
  y[l] = x[l * stride];
}
// <a, K x> with x read from memory in row pairs (kdot's arithmetic)
template <int l>
__device__ __forceinline__ float kdot_mem(const float (&av)[2 * l + 1], const float* x, int stride) {
  float acc = 0.f;
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    const float t = fmaf(av[i], x[(2 * l - i) * stride], -(av[2 * l - i] * x[i * stride]));
    acc = fmaf((float)f, t, acc);
  });
  return acc;
}

// <a, K b> with K = X(θ)^{-1} dX/dθ, the so(2) generator of the degree-l block: row i
// of K has f_i = l - i at column 2l-i (X = C + S P with P the row reversal, so
// dX/dθ = diag(f cos) P - diag(f sin) = X diag(f) P).  Hence <g, X' x> = <X^T g, K x>:
// each angle gradient is a dot product of two vectors the chain computes anyway, paired
// as f_i (a_i b_{2l-i} - a_{2l-i} b_i), with no multiples.
template <int l>
__device__ __forceinline__ float kdot(const float (&av)[2 * l + 1], const float (&bv)[2 * l + 1]) {
  float acc = 0.f;
  sfor<l>([&](auto I) {
    constexpr int i = LV_CV(I);
    constexpr int f = l - i;
    const float t = fmaf(av[i], bv[2 * l - i], -(av[2 * l - i] * bv[i]));
    acc = fmaf((float)f, t, acc);
  });
  return acc;
}

// Up to l_max = kBwdWideMaxL the C = 10, one-group-per-block kernel fits 168 VGPRs
// without spilling (156 at l = 10), so it has a twin built for 3 waves per SIMD
// (WPE = 3) that the plan gives twice the segments: 26.9 -> 19.5 us per
// call at batch 4096 (profiles/r02_bwd_regbudget_sweep.txt).  Every other variant (group
// loop, run-time C, higher degrees) spills at 168 and keeps the 256-VGPR budget.
constexpr int kBwdWideMaxL = 10;
__host__ __device__ constexpr bool bwd_wide(int L, int C, int fmode, int64_t groups, int64_t gx) {
  return L <= kBwdWideMaxL && C == kTileFastC && fmode == kBwdFShared && gx >= groups;
}

// This block's dF slab elements [g0, g0 + cnt) (a wave's rows) from LDS to the workspace,
// row layout ([block][M*C]) or chunk-major (slab_chunked).
__device__ __forceinline__ void write_slab_rows(const ActionBwdArgs& a, const float* slabL, int g0, int cnt,
                                                int lane) {
  if (a.slab_chunked) {
    float* ws = a.ws_F + (int64_t)blockIdx.x * kSlabChunk;
    const int64_t cstride = (int64_t)gridDim.x * kSlabChunk;
    for (int e = lane; e < cnt; e += 64) {
      const int g = g0 + e;
      ws[(g / kSlabChunk) * cstride + g % kSlabChunk] = slabL[g];
    }
  } else {
    float* slab = a.ws_F + (int64_t)blockIdx.x * a.MC;
    for (int e = lane; e < cnt; e += 64) slab[g0 + e] = slabL[g0 + e];
  }
}

// LOOP: blocks loop over sample groups (grid capped, bounded workspace).  Without it each
// block takes exactly one group (grid = groups): the group loop made the compiler hoist
// loop-invariant addresses and hold them across the whole chain (256 VGPRs + 240 B/lane of
// spills at l = 10 vs 220 VGPRs and none; 31.4 -> 28.0 us per call at batch 4096,
// profiles/r02_bwd_regbudget_sweep.txt), so the launcher uses it whenever the grid covers
// the batch.
// WPE: waves per SIMD the register budget is sized for (3 only for the bwd_wide case).
// JIT: the spectrum column and G read in row pairs inside the products (A/B variant bit
// kBwdVarJit of ActionBwdArgs::variant; wide kernel only).
template <int LT, int CT, int FM, bool LOOP = true, int WPE = 2, bool JIT = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE)))
void action_bwd_tile_kernel(ActionBwdArgs a) {
  constexpr bool SHAREDF = FM != kBwdFSample;
  constexpr bool GSLAB = FM == kBwdFSharedGlobal;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int kRow = TrigLds<LT>::kRow;
  const int C = CT > 0 ? CT : a.C;
  const int Sw = a.Sw;
  const int64_t MC = CT > 0 ? (int64_t)(LT + 1) * (LT + 1) * CT : a.MC;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar branches
  const int tid = (int)threadIdx.x, nthr = (int)blockDim.x;
  const int j = lane / C;
  const int c = lane - j * C;
  // this wave's degrees: a bit set (balanced by cost in the planner); the run-time-C kernel
  // with the spectrum in LDS keeps contiguous ranges [lo, hi) for its column-major slices
  const unsigned dmask = a.seg_mask[wave];
  const int lo = a.seg_lo[wave], hi = a.seg_lo[wave + 1];
  const int rows_lo = lo * lo;
  const int frows = fseg_rows(lo, hi);
  auto each_degree = [&](auto&& fn) {  // the wave's degrees, ascending (scalar loop)
    for (unsigned m = dmask; m; m &= m - 1) fn(__builtin_ctz(m));
  };
  const int stage_bytes = tile_stage_bytes(Sw, MC, 4);
  // LDS: [gout / dF tile][multiples table][angle partials][dF slab (shared F)][spectrum:
  //      CT > 0 the whole (M, C) row-major, else per-wave column-major slices]
  //      [fused path: the group's v (and mu), Sw * 12 floats]
  float* trig = lds + (stage_bytes >> 2);
  float* apart = trig + bwd_trig_floats(Sw, LT);               // [nseg][64][3]
  // dF slab: LDS [M*C] (kBwdFShared), or this block's workspace row (kBwdFSharedGlobal)
  float* slabL = GSLAB ? a.ws_F + (int64_t)blockIdx.x * MC : apart + (nthr >> 6) * 64 * 3;
  // slab element g: LDS (kBwdFShared), or this block's workspace slab in the row or the
  // chunk-major layout (kBwdFSharedGlobal; the layout the reduce kernel reads)
  auto slab_at = [&](int g) -> float& {
    if constexpr (GSLAB) {
      if (a.slab_chunked)
        return a.ws_F[((int64_t)(g / kSlabChunk) * gridDim.x + blockIdx.x) * kSlabChunk + g % kSlabChunk];
    }
    return slabL[g];
  };
  float* const Fbase = apart + (nthr >> 6) * 64 * 3 + (FM == kBwdFShared ? (int)MC : 0);
  const int fsize = CT > 0 ? (((int)MC + 3) & ~3) : (nthr >> 6) * a.fpitch;
  float* Fw = Fbase + (CT > 0 ? 0 : wave * a.fpitch);
  // spectrum (shared F): once per block -- CT > 0: element e = tid + k * nthr of the whole
  // (M, C) by every thread, loads issued together; else this wave's column-major slice
  constexpr int kFPer = CT > 0 ? ((LT + 1) * (LT + 1) * (CT > 0 ? CT : 1) + 255) / 256 : 6;
  constexpr int kFPerCap = kFPer < 16 ? kFPer : 16;
  const int fcnt = SHAREDF ? (CT > 0 ? (int)MC : (hi * hi - rows_lo) * C) : 0;
  const int fstr = CT > 0 ? nthr : 64;
  const int fbase = CT > 0 ? tid : lane;
  const float* fsrc = a.F + (CT > 0 ? 0 : rows_lo * C);
  // Degrees walked largest first (every instantiation, so that all spectrum modes and the
  // looping kernel add a sample's angle-gradient partials in the same order); kDesc: the
  // one-group compile-time-C kernel also loads its prologue inputs ahead of the tile DMA
  // and may split the prologue barrier (kBwdVarSplit: the largest degree's forward
  // recompute overlapping the tile DMA)
  constexpr bool kDesc = CT > 0 && !LOOP && FM == kBwdFShared;
  // kBwdVarSpread: task t on lane t / nw of wave t % nw (the prologue's serial chains on
  // every SIMD), else thread t (all tasks in wave 0); the host guarantees 3*Sw <= blockDim.x
  const int t_task = (a.variant & kBwdVarSpread) ? lane * (nthr >> 6) + wave : tid;
  const bool task = t_task < 3 * Sw;
  const int jt = t_task / 3, q = t_task - 3 * (t_task / 3);
  // kDesc: the prologue's angle and the VJP tail's v / mu loaded before the spectrum, so
  // the spectrum staging's wait covers them and nothing after the tile DMA waits in vmcnt
  // order behind it
  float ang0 = 0.f, vmu0 = 0.f;
  if constexpr (kDesc) {
    const int64_t s0e = (int64_t)blockIdx.x * Sw;
    const int Sve = (int)min((int64_t)Sw, a.n - s0e);
    if (task) ang0 = a.ang[(s0e + min(jt, Sve - 1)) * 3 + (a.transpose ? 2 - q : q)];
    if (a.v && tid < 12 * Sve && 12 * Sve <= nthr) {  // else the loop after the DMA
      const int js = tid / 12, k = tid - 12 * js;
      vmu0 = k < 3 ? a.v[(s0e + js) * 3 + k] : (a.mu ? a.mu[(s0e + js) * 9 + (k - 3)] : 0.f);
    }
  }
  if constexpr (GSLAB) {
    each_degree([&](int l) {  // this wave's rows
      for (int e = lane; e < (2 * l + 1) * C; e += 64) slab_at(l * l * C + e) = 0.f;
    });
  } else if constexpr (SHAREDF) {
    float fv[kFPerCap];
#pragma unroll
    for (int k = 0; k < kFPerCap; ++k) {
      const int e = fbase + fstr * k;
      fv[k] = e < fcnt ? fsrc[e] : 0.f;
    }
    if constexpr (LOOP)
      each_degree([&](int l) {  // this wave's rows
        for (int e = lane; e < (2 * l + 1) * C; e += 64) slabL[l * l * C + e] = 0.f;
      });
    if constexpr (CT > 0) {
#pragma unroll
      for (int k = 0; k < kFPerCap; ++k) {
        const int e = fbase + fstr * k;
        if (e < fcnt) Fw[e] = fv[k];
      }
      for (int e0 = fbase + fstr * kFPerCap; e0 < fcnt; e0 += 8 * fstr) {
        float t8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t8[u] = e0 + fstr * u < fcnt ? fsrc[e0 + fstr * u] : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (e0 + fstr * u < fcnt) Fw[e0 + fstr * u] = t8[u];
      }
    } else {
#pragma unroll
      for (int k = 0; k < kFPerCap; ++k) {
        const int e = lane + 64 * k;
        if (e < fcnt) {
          const int r = e / C, cc2 = e - r * C;
          Fw[cc2 * frows + r] = fv[k];
        }
      }
      for (int e = lane + 64 * kFPerCap; e < fcnt; e += 64) {
        const int r = e / C, cc2 = e - r * C;
        Fw[cc2 * frows + r] = fsrc[e];
      }
    }
  }
  // fused path: the exp -> ZYZ VJP's inputs, loaded by the prologue threads so that the
  // tail does not wait on global loads (after the spectrum)
  float* vmu = Fbase + fsize;
  const float* Fl = GSLAB ? a.F + c : (CT > 0 ? Fw + c : Fw + c * frows - rows_lo);
  const int fstep = (GSLAB || CT > 0) ? C : 1;

  phase_stamp(a.stamps, wave, 0);
  for (int64_t g = blockIdx.x; g < a.groups; g += LOOP ? gridDim.x : a.groups) {
    const int64_t s0 = g * Sw;
    const int Sv = (int)min((int64_t)Sw, a.n - s0);
    const bool active = j < Sv;
    const int nbytes = Sv * (int)MC * 4;
    if (a.prio >= 2) __builtin_amdgcn_s_setprio(3);
    // 1. upstream-gradient tile: global -> LDS by LDS-DMA (global_load_lds, 16-byte body,
    //    4-byte head/tail), issued first thing.  No VGPR holds the tile in flight: the
    //    register-staged form kept 32 VGPRs of loads live across the prologue, which the
    //    3-waves-per-SIMD build spilled to scratch (96 B/lane; tools/bwdbench.hip: 13.5 ->
    //    12.2 us at batch 4096, bitwise equal).
    const float* gsrc = a.gout + s0 * MC;
    const int mis = (int)(reinterpret_cast<uintptr_t>(gsrc) & 15);
    char* stage_b = reinterpret_cast<char*>(lds) + mis;  // LDS addr = global addr (mod 16)
    {
      const int head = min((16 - mis) & 15, nbytes);
      const int nvec = (nbytes - head) >> 4;
      const int tail0 = head + nvec * 16;
      const char* gb = reinterpret_cast<const char*>(gsrc);
      for (int v0 = wave * 64; v0 < nvec; v0 += nthr)
        if (v0 + lane < nvec)
          __builtin_amdgcn_global_load_lds(gb + head + 16 * (v0 + lane), as_lds(stage_b + head + 16 * v0),
                                           16, 0, 0);
      if (wave == 0) {
        if (4 * lane < head) __builtin_amdgcn_global_load_lds(gsrc + lane, as_lds(stage_b), 4, 0, 0);
        if (tail0 + 4 * lane < nbytes)
          __builtin_amdgcn_global_load_lds(gb + tail0 + 4 * lane, as_lds(stage_b + tail0), 4, 0, 0);
      }
    }
    // 2. prologue task (sample jt, slot q): sincos, multiples of slot q
    if (task) {
      const int64_t st = s0 + min(jt, Sv - 1);  // idle slots mirror a valid sample
      // only this slot's angle (transpose: slot q takes angle 2 - q, sine negated)
      float cq, sq;
      if constexpr (kDesc) (void)st;
      sincosf(kDesc ? ang0 : a.ang[st * 3 + (a.transpose ? 2 - q : q)], &sq, &cq);
      if (a.transpose) sq = -sq;
      trig_row_fill1<LT>(trig + jt * kRow, cq, sq, q, LT);
    }
    if (kDesc && a.v && 12 * Sv <= nthr) {
      if (tid < 12 * Sv) vmu[tid] = vmu0;
    } else if (a.v) {  // v (3) and mu (9) of the group's samples for the VJP tail (12 * Sv
                       // may exceed the block: 252 values at C = 3)
      for (int t = tid; t < 12 * Sv; t += nthr) {
        const int js = t / 12, k = t - 12 * js;
        if (k < 3) vmu[js * 12 + k] = a.v[(s0 + js) * 3 + k];
        else if (a.mu) vmu[js * 12 + k] = a.mu[(s0 + js) * 9 + (k - 3)];
      }
    }
    // 3. the LDS-DMA writes of this wave have landed (an LDS-DMA is counted in vmcnt);
    //    kBwdVarSplit: only the multiples, the spectrum and v / mu here (LDS writes), the
    //    tile after the first degree's forward recompute
    bool split_pending = kDesc && (a.variant & kBwdVarSplit) != 0;
    if (!split_pending) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    block_sync_lds();
    phase_stamp(a.stamps, wave, 1);

    if (a.prio >= 2) __builtin_amdgcn_s_setprio(0);
    float* tile_lane = reinterpret_cast<float*>(stage_b) + j * MC + c;
    const float* tj = trig + min(j, Sw - 1) * kRow;
    const float* Fs = a.F + (s0 + min(j, Sv - 1)) * a.Fstride + c;  // per-sample spectrum
    float ga = 0.f, gb = 0.f, gc = 0.f;
    sfor<LT + 1>([&](auto Lc) {
      constexpr int l = LT - LV_CV(Lc);
      if ((dmask >> l) & 1u) {
        constexpr int nn = 2 * l + 1;
        constexpr int r0 = l * l;
        // live arrays kept to three or four of 2l+1: the spectrum column and G are
        // re-read from LDS where they are needed again
        float p2[nn], p4[nn], u[nn];
        const float* fcol = SHAREDF ? Fl + r0 * fstep : Fs + r0 * C;
        const int fst = SHAREDF ? fstep : C;
        if constexpr (JIT) {
          // the spectrum column and G read in row pairs inside the products that use them
          // (xm_mem), on every lane: an idle lane's addresses stay inside the block's LDS
          // and its results are never used
          xm_mem<l, false>(mult_lds<l, 2, LT>(tj), fcol, fst, u);  // P1
        } else {
          float f0[nn];
          sfor<nn>([&](auto K) { f0[LV_CV(K)] = fcol[LV_CV(K) * fst]; });
          xm<l>(mult_lds<l, 2, LT>(tj), f0, u);   // P1
        }
        jmul<l>(u, p2);                           // P2
        xm<l>(mult_lds<l, 1, LT>(tj), p2, u);     // P3
        jmul<l>(u, p4);                           // P4
        if (split_pending) {  // the wave's first degree: now the tile
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          block_sync_lds();
          split_pending = false;
        }
        if constexpr (JIT) {
          xm_mem<l, true>(mult_lds<l, 0, LT>(tj), tile_lane + r0 * C, C, u);  // Q4
        } else {
          float gq[nn];
          sfor<nn>([&](auto K) { gq[LV_CV(K)] = active ? tile_lane[(r0 + LV_CV(K)) * C] : 0.f; });
          xm_t<l>(mult_lds<l, 0, LT>(tj), gq, u);  // Q4
        }
        ga += kdot<l>(u, p4);                     // <G, Xa' P4> = <Q4, K P4>
        jmul<l>(u, p4);                           // Q3 (reuse p4)
        xm_t<l>(mult_lds<l, 1, LT>(tj), p4, u);  // Q2
        gb += kdot<l>(u, p2);                     // <Q3, Xb' P2> = <Q2, K P2>
        jmul<l>(u, p2);                           // Q1 (reuse p2)
        xm_t<l>(mult_lds<l, 2, LT>(tj), p2, u);  // dF column
        if constexpr (JIT) {
          gc += kdot_mem<l>(u, fcol, fst);        // <Q1, Xc' F> = <dF, K F>
        } else {
          float f0[nn];
          sfor<nn>([&](auto K) { f0[LV_CV(K)] = fcol[LV_CV(K) * fst]; });
          gc += kdot<l>(u, f0);
        }
        if (active) sfor<nn>([&](auto I) { tile_lane[(r0 + LV_CV(I)) * C] = u[LV_CV(I)]; });
        if constexpr (SHAREDF && (LOOP || FM != kBwdFShared)) {
          // this degree's rows summed over the group's samples in sample order, added to
          // the block's slab (groups in order)
          wave_lds_sync();
          const float* col0 = reinterpret_cast<const float*>(stage_b) + r0 * C;
          constexpr int kSw = CT > 0 ? 64 / CT : 1;
          if (CT > 0 && Sv == kSw && Sw == kSw) {
            // full group, compile-time size: the Sw loads of an element are issued
            // together (one LDS round trip), summed in the same sample order
            for (int e = lane; e < nn * C; e += 64) {
              float v[kSw];
#pragma unroll
              for (int jj = 0; jj < kSw; ++jj) v[jj] = col0[jj * MC + e];
              float sum = v[0];
#pragma unroll
              for (int jj = 1; jj < kSw; ++jj) sum += v[jj];
              slab_at(r0 * C + e) += sum;
            }
          } else {
            for (int e = lane; e < nn * C; e += 64) {
              float sum = col0[e];
              for (int jj = 1; jj < Sv; ++jj) sum += col0[jj * MC + e];
              slab_at(r0 * C + e) += sum;
            }
          }
        }
        if (a.stamps) degree_stamp(a.stamps, wave, l);
      }
    });
    if (split_pending) {  // a wave without degrees still takes the tile barrier
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      block_sync_lds();
    }
    phase_stamp(a.stamps, wave, 2);
    if constexpr (FM == kBwdFShared && !LOOP) {
      // one group per block: this wave's rows of the slab are the group's dF rows summed
      // over its samples in sample order (the same sums as the looping path's per-degree
      // slab adds, whose 0 + sum only differs in the sign of a zero, which the reduce's
      // 0 + ... erases), taken once after the whole chain -- one LDS wait instead of one
      // per degree -- and stored straight to the workspace, ahead of the angle tail
      wave_lds_sync();
      const float* t0 = reinterpret_cast<const float*>(stage_b);
      constexpr int kSw = CT > 0 ? 64 / CT : 1;
      const bool full = CT > 0 && Sv == kSw && Sw == kSw;
      // write-through (sc1, kBwdVarSlabWT) or plain slab stores
      const int64_t slab_floats = (int64_t)gridDim.x * (a.slab_chunked ? slab_chunks(MC) * kSlabChunk : MC);
      const __amdgpu_buffer_rsrc_t wrs =
          __builtin_amdgcn_make_buffer_rsrc(a.ws_F, 0, (int)(slab_floats * 4), kRawBufferFlags);
      const int64_t cstride = (int64_t)gridDim.x * kSlabChunk;
      const bool wt = (a.variant & kBwdVarSlabWT) != 0;
      auto put = [&](int g, float sum) {
        const int64_t idx = a.slab_chunked ? (g / kSlabChunk) * cstride + (int64_t)blockIdx.x * kSlabChunk + g % kSlabChunk
                                           : (int64_t)blockIdx.x * MC + g;
        if (wt) tile_store_elem<16>(wrs, (int)(idx * 4), sum);
        else a.ws_F[idx] = sum;
      };
      // a range [g0, g0 + cnt) of slab elements, kU per lane per pass with all their LDS
      // loads issued before any sum or store; idx maps a range position to the element
      auto sum_range = [&](int cnt, auto&& idx) {
        if (full) {
          constexpr int kU = 4;
          for (int e0 = lane; e0 < cnt; e0 += kU * 64) {
            float v[kU][kSw];
            int gg[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
              gg[u] = idx(min(e0 + 64 * u, cnt - 1));  // clamped: in-range reads
#pragma unroll
              for (int jj = 0; jj < kSw; ++jj) v[u][jj] = t0[jj * MC + gg[u]];
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
              float sum = v[u][0];
#pragma unroll
              for (int jj = 1; jj < kSw; ++jj) sum += v[u][jj];
              if (e0 + 64 * u < cnt) put(gg[u], sum);
            }
          }
        } else {
          for (int e = lane; e < cnt; e += 64) {
            const int g = idx(e);
            float sum = t0[g];
            for (int jj = 1; jj < Sv; ++jj) sum += t0[jj * MC + g];
            put(g, sum);
          }
        }
      };
      if (a.variant & kBwdVarSlabFlat) {
        // the wave's elements as one flat list over its degrees (ascending)
        int tot = 0;
        each_degree([&](int l) { tot += (2 * l + 1) * C; });
        sum_range(tot, [&](int e) {
          int off = 0, g = 0;
          each_degree([&](int l) {
            const int cnt = (2 * l + 1) * C;
            if (e >= off && e < off + cnt) g = l * l * C + (e - off);
            off += cnt;
          });
          return g;
        });
      } else {
        each_degree([&](int l) { sum_range((2 * l + 1) * C, [&](int e) { return l * l * C + e; }); });
      }
    }
    phase_stamp(a.stamps, wave, 3);
    // angle gradients: sum over the C lanes of a sample (column order), then segments
    float* ap = apart + wave * 64 * 3;
    if (a.transpose) {
      ap[lane * 3 + 0] = -gc; ap[lane * 3 + 1] = -gb; ap[lane * 3 + 2] = -ga;
    } else {
      ap[lane * 3 + 0] = ga; ap[lane * 3 + 1] = gb; ap[lane * 3 + 2] = gc;
    }
    block_sync_lds();
    phase_stamp(a.stamps, wave, 4);
    if (tid < 3 * Sv) {
      const int js = tid / 3, i = tid - 3 * (tid / 3);
      const int nw = nthr >> 6;
      float r = 0.f;
      for (int w = 0; w < nw; ++w) {
        float sw = 0.f;
        for (int cc2 = 0; cc2 < C; ++cc2) sw += apart[(w * 64 + js * C + cc2) * 3 + i];
        r += sw;
      }
      if (a.gang) a.gang[(s0 + js) * 3 + i] = r;
      if (a.v) trig[js * 3 + i] = r;  // the chains are done: the table is free
    }
    if (!LOOP && SHAREDF && wave > 0) {  // the tail below is wave 0's (tid < 3 * Sw)
      phase_stamp(a.stamps, wave, 5);
      return;
    }
    if (a.v) {  // fused path: exp -> ZYZ VJP of the group's samples (exp_eazyz_vjp_sample)
      if constexpr (!LOOP && SHAREDF) wave_lds_sync();  // wave 0 alone from here
      else block_sync_lds();
      if (tid < Sv) {
        const int64_t s = s0 + tid;
        float av[3], g[3], m[9], gm[9], o[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) { av[k] = vmu[tid * 12 + k]; g[k] = trig[tid * 3 + k]; }
        if (a.mu) {
#pragma unroll
          for (int k = 0; k < 9; ++k) m[k] = vmu[tid * 12 + 3 + k];
        }
        exp_eazyz_vjp_sample(av, a.mu != nullptr, m, g, gm, o);
        if (a.mu) {
#pragma unroll
          for (int k = 0; k < 9; ++k) a.gmu[s * 9 + k] = gm[k];
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) a.gv[s * 3 + k] = o[k];
      }
    }
    if constexpr (!SHAREDF)
      tile_flush<float, 1>(a.gF + s0 * MC, stage_b, mis, nbytes, tid, nthr);
    if constexpr (!LOOP && SHAREDF) {
      phase_stamp(a.stamps, wave, 5);
      return;
    }
    block_sync_lds();  // the next group overwrites the tile, the table and the partials
  }
  if constexpr (FM == kBwdFShared)
    each_degree([&](int l) { write_slab_rows(a, slabL, l * l * C, (2 * l + 1) * C, lane); });
}

}  // namespace lv
#include "action_bwd_persist.h"
namespace lv {

// Slab count per block of action_bwd_reduce_kernel (defined in action.hip).
constexpr int kBwdReduceWaves = 16;

struct BwdLaunch {
  ActionBwdArgs a;
  int gx, nseg, fmode;
  int persist;  // action_bwd_persist_kernel (large batches, C = 10, shared spectrum)
  size_t lds;
  hipStream_t stream;
};

template <int LT>
struct BwdLauncher {
  static int run(BwdLaunch& p);  // out of class: see FwdLauncher
};
template <int LT>
int BwdLauncher<LT>::run(BwdLaunch& p) {
  const dim3 grid(p.gx), block(64 * p.nseg);
  if (p.persist) {
    if constexpr (LT <= kBwdPersistMaxL) {
      const bool single = (p.a.variant & kBwdVarPersistSingle) != 0;
      const int pv = ((p.a.variant & kBwdVarPersistPad) ? 1 : 0) | ((p.a.variant & kBwdVarPersistAng) ? 2 : 0) |
                     ((p.a.variant & kBwdVarPersistBufDma) ? 4 : 0) | ((p.a.variant & kBwdVarPersistLaneMap) ? 8 : 0) |
                     ((p.a.variant & kBwdVarPersistSlabWT) ? 16 : 0);
      // built single-buffer variants: 0 (round 5), 2 (LDS angle sums), 3 (+ padded tile),
      // 6 (+ buffer DMA), 7 (padded tile by buffer DMA), 14 (+ lane map), 22 (6 + write-through
      // slab stores); the A/B library refuses other combinations
      if (single && pv == 22)
        hipLaunchKernelGGL((action_bwd_persist_kernel<LT, kBwdPersistWaves, false, true, 3, 22>), grid, block, p.lds, p.stream, p.a);
      else if (single && pv == 7)
        hipLaunchKernelGGL((action_bwd_persist_kernel<LT, kBwdPersistWaves, false, true, 3, 7>), grid, block, p.lds, p.stream, p.a);
      else if (single && pv == 14)
        hipLaunchKernelGGL((action_bwd_persist_kernel<LT, kBwdPersistWaves, false, true, 3, 14>), grid, block, p.lds, p.stream, p.a);
      else if (single && pv == 6)
        hipLaunchKernelGGL((action_bwd_persist_kernel<LT, kBwdPersistWaves, false, true, 3, 6>), grid, block, p.lds, p.stream, p.a);
      else if (single && pv == 3)
        hipLaunchKernelGGL((action_bwd_persist_kernel<LT, kBwdPersistWaves, false, true, 3, 3>), grid, block, p.lds, p.stream, p.a);
      else if (single && pv == 2)
        hipLaunchKernelGGL((action_bwd_persist_kernel<LT, kBwdPersistWaves, false, true, 3, 2>), grid, block, p.lds, p.stream, p.a);
      else if (single && pv == 0)
        hipLaunchKernelGGL((action_bwd_persist_kernel<LT, kBwdPersistWaves, false, true>), grid, block, p.lds, p.stream, p.a);
      else if (single) {
        set_error("persistent backward variant %d not built", pv);
        return LV_ERR_ARG;
      }
      else
        hipLaunchKernelGGL((action_bwd_persist_kernel<LT, kBwdPersistWaves>), grid, block, p.lds, p.stream, p.a);
    }
    LV_RETURN_LAUNCH("action_bwd_persist_kernel");
  }
  if (p.fmode == kBwdFSample)
    hipLaunchKernelGGL((action_bwd_tile_kernel<LT, 0, kBwdFSample>), grid, block, p.lds, p.stream, p.a);
  else if (p.fmode == kBwdFSharedGlobal)
    hipLaunchKernelGGL((action_bwd_tile_kernel<LT, 0, kBwdFSharedGlobal>), grid, block, p.lds, p.stream, p.a);
  else if (bwd_wide(LT, p.a.C, p.fmode, p.a.groups, p.gx)) {
    if constexpr (LT <= kBwdWideMaxL) {
      if (p.a.variant & kBwdVarJit)
        hipLaunchKernelGGL((action_bwd_tile_kernel<LT, kTileFastC, kBwdFShared, false, 3, true>), grid, block, p.lds, p.stream, p.a);
      else
        hipLaunchKernelGGL((action_bwd_tile_kernel<LT, kTileFastC, kBwdFShared, false, 3>), grid, block, p.lds, p.stream, p.a);
    }
  } else if (p.a.C == kTileFastC && p.gx >= p.a.groups)
    hipLaunchKernelGGL((action_bwd_tile_kernel<LT, kTileFastC, kBwdFShared, false>), grid, block, p.lds, p.stream, p.a);
  else if (p.a.C == kTileFastC)
    hipLaunchKernelGGL((action_bwd_tile_kernel<LT, kTileFastC, kBwdFShared>), grid, block, p.lds, p.stream, p.a);
  else
    hipLaunchKernelGGL((action_bwd_tile_kernel<LT, 0, kBwdFShared>), grid, block, p.lds, p.stream, p.a);
  LV_RETURN_LAUNCH("action_bwd_tile_kernel");
}

#define LV_EXTERN_BWD(L) extern template struct BwdLauncher<L>;

}  // namespace lv

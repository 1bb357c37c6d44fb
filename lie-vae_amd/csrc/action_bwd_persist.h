#pragma once
// Persistent group-action backward for large batches (compile-time C = 10, shared spectrum,
// l_max <= kBwdPersistMaxL): the reference's autograd through lie_tools.py:211-253
// (wigner_d_matrix, block_wigner_matrix_multiply) for the training direction.
//
// The one-group tile kernel (action_bwd.h) runs one 6-sample group per block, so every
// block pays its whole phase chain -- gradient-tile load, prologue, chain, per-group dF slab
// pass, angle barrier -- back to back, and writes one 4.8 KB dF slab per 6 samples (a
// third of the gradient tile's bytes again at l = 10, read back by the reduce).  Beyond
// 4,096 groups the grid was capped and blocks looped over groups in a 256-VGPR build.
//
// Here a grid of 3 blocks per CU walks the groups (block b: groups b, b + P, b + 2P, ...):
//   * the prologue of group k+1 (sincos of the stored angle, multiples of one (sample,
//     slot) per task lane, tasks spread over the block's waves) runs after each wave's
//     chain, into the second of two multiples tables, its angle loads issued at the top;
//   * each wave adds its degrees' dF rows, summed over the group's samples, into the
//     block's LDS slab (its own rows only: no race); the slab leaves once per block;
//   * one barrier per group publishes the angle partials and the next multiples and
//     frees the gradient tile, which then takes the next group by LDS-DMA (no VGPR holds
//     it in flight) before a second barrier.
// DB = true double-buffers the gradient tile instead (the next tile's DMA under the current
// chain, one barrier per group) at 2 blocks per CU; measured slower than 3 blocks per CU
// with one buffer (65,536: 131 vs 114 us, profiles/r05_ab4.txt), kept as A/B variant.
// The chain itself (P1..P4 forward recompute, Q4..dF transposed chain, angle gradients as
// <Q4, K P4>, <Q2, K P2>, <dF, K F>) is the one-group kernel's JIT chain, operation for
// operation.  Summation orders are fixed by the plan (degree set per wave, groups per
// block): reproducible bit for bit, and within fp32 rounding of the one-group kernel.
// The angle gradient goes to a.gang (the caller's, or a workspace region for the fused
// exp -> ZYZ VJP, which the host then runs beside the dF reduce, in
// action_bwd_reduce5_vjp_kernel).
// Included by action_bwd.h after the one-group kernel and its helpers.

namespace lv {

constexpr int kBwdPersistMaxL = 10;
constexpr int kBwdPersistWaves = 4;      // degree-set waves per block
constexpr int kBwdPersistBlocksPerCU = 3;    // one gradient-tile buffer (the product)
constexpr int kBwdPersistBlocksPerCUDB = 2;  // double-buffered tile (A/B)
// A/B variant bits of the persistent kernel (ActionBwdArgs::variant, A/B build only):
// single gradient-tile buffer at 3 blocks per CU (3 waves per SIMD; the next tile is
// loaded after the group's barrier); the next group's multiples filled by the 18 first lanes
// of the last wave instead of 4-5 lanes of every wave (every wave then ran the whole
// sincos + recurrence; 65,536: 110.3 -> 107.9 us, 262,144: 390 -> 376 us; both are the
// product default).  (The non-JIT chain, 5 waves per block and one buffer at 2 blocks per
// CU built for 2 waves per SIMD were slower: profiles/r05_bwd_persist_ab2.txt, r05_ab4.txt,
// r05_ab8.txt.)
constexpr int kBwdVarPersistSingle = 32, kBwdVarPersistTask1 = 512;
// Round 6 (single-buffer kernel, template parameter PV): kBwdVarPersistPad = the padded
// gradient tile (persist_pad); kBwdVarPersistAng = the angle partials leave every lane by
// three LDS stores and one wave sums each sample's 4 x 10 (wave, column) partials after
// the group barrier, instead of a 4-step cross-lane tree (12 ds_bpermute + ~67 VALU) on
// every wave.
constexpr int kBwdVarPersistPad = 1024, kBwdVarPersistAng = 2048;
// kBwdVarPersistBufDma: the gradient tile by buffer loads to LDS (buffer_load_dwordx4 ...
// lds): the group's rows as a buffer resource, each lane's byte offset fixed for the whole
// walk and the round's offset in an SGPR, so a full round of 16-byte pieces costs no VALU
// (global_load_lds needs a 64-bit VGPR address per lane: ~5 VALU per wave instruction, ~140
// per group); only the last, partial round keeps a per-lane bound.
constexpr int kBwdVarPersistBufDma = 4096;
// kBwdVarPersistLaneMap (with the LDS angle sums): lanes take (sample, column) pairs in the
// order below instead of lane = 10 j + c.  With the unpadded tile at l = 10 (1,210 floats =
// 26 mod 32 between samples) every ds_read_b32 / ds_write_b32 of the chain's tile rows had
// 4 banks 2-way in each 32-lane half; residues 2, 3, 8, 9 hold three (j, c) pairs each, so
// one half must keep a 2-way bank, and this assignment (found by search) leaves exactly
// that: 1 extra LDS cycle per tile access instead of 2.  Entries are 16 j + c; lanes 60-63
// are idle (j = 6).  Used where M*C = 26 mod 32 (l = 4, 10).
constexpr int kBwdVarPersistLaneMap = 8192;
// kBwdVarPersistSlabWT: the block's dF slab leaves as whole 16-byte pieces with write-through
// (sc1) buffer stores after one block barrier, instead of each wave's rows as 4-byte stores
// left dirty in the XCD's L2 for the end-of-kernel write-back.
constexpr int kBwdVarPersistSlabWT = 16384;
static __constant__ unsigned char kPersistLaneJC[64] = {
    0, 1, 2, 3, 5, 6, 7, 8, 9, 17, 18, 19, 21, 24, 32, 34, 37, 38, 49, 52, 53, 55,
    57, 66, 70, 72, 73, 81, 82, 86, 87, 89, 4, 16, 20, 22, 23, 25, 33, 35, 36, 39,
    40, 41, 48, 50, 51, 54, 56, 64, 65, 67, 68, 69, 71, 80, 83, 84, 85, 88, 96, 97, 98, 99};

// LDS floats of the persistent kernel: NB gradient tiles (2: double-buffered), 2
// multiples tables, 2 angle-partial buffers, the dF slab and the spectrum.
// Unpadded (PAD = false), samples of the gradient tile sit M*C floats apart in LDS, exactly
// as in global memory, so one LDS-DMA instruction moves 1 KiB of any sample(s) and the tile
// takes ~29 of them, spread evenly over the waves.  At l = 10 that stride (1,210 floats,
// 26 mod 32 banks) puts the 10 column lanes of adjacent samples on 4 shared banks in each
// 32-lane half of every ds_read_b32 / ds_write_b32 of the chain (Q4 reads, dF writes): 2
// extra LDS cycles per instruction, ~480 per group (0.64 conflict cycles per LDS
// instruction, profiles/r05_pmc_persist_65536.txt).
// PAD (kBwdVarPersistPad): samples persist_pad(L) floats further apart (l = 10: 1,226 =
// 10 mod 32, so the six samples' 10-lane windows tile both halves without a shared bank).
// The pad is a multiple of 16 bytes, so every sample's LDS image stays congruent to its
// global image mod 16 and the tile still moves as flat 16-byte LDS-DMA pieces: a piece's
// source is its LDS offset minus pad bytes per preceding sample (pieces in a pad read the
// neighbouring sample's bytes into the pad, never read).
__host__ __device__ constexpr int persist_pad(int L) {
  return ((10 - (L + 1) * (L + 1) * 10) % 32 + 32) % 32 % 4 == 0 ? ((10 - (L + 1) * (L + 1) * 10) % 32 + 32) % 32 : 0;
}
__host__ __device__ constexpr int persist_stride(int L, bool pad = false) {
  return (L + 1) * (L + 1) * 10 + (pad ? persist_pad(L) : 0);
}
__host__ __device__ constexpr int persist_tile_floats(int L, bool pad = false) {
  return (((64 / 10) * persist_stride(L, pad) * 4 + 16 + 15) & ~15) / 4;
}
__host__ __device__ constexpr int persist_lds_floats(int L, int NW, int NB = 2, bool pad = false) {
  return NB * persist_tile_floats(L, pad) + 2 * (64 / 10) * trig_row_floats(L) + 2 * 3 * (NW * 64 + 4) +
         2 * ((((L + 1) * (L + 1) * 10) + 3) & ~3);
}
static_assert(persist_stride(10, true) % 32 == 10 && persist_pad(10) % 4 == 0, "l = 10 pad");

// DB: double-buffered gradient tile (2 blocks per CU); else one buffer at 3 blocks per CU.
// JIT: spectrum / gradient columns read in row pairs inside the products.
template <int LT, int NW, bool DB = true, bool JIT = true, int WPE = (DB ? 2 : 3), int PV = 0>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(WPE)))
void action_bwd_persist_kernel(ActionBwdArgs a) {
  constexpr bool PAD = (PV & 1) != 0 && persist_pad(LT) > 0;
  constexpr bool ANGL = (PV & 2) != 0;
  constexpr bool BUFDMA = (PV & 4) != 0 && !((PV & 1) != 0 && persist_pad(LT) > 0);
  constexpr bool PADBUF = (PV & 4) != 0 && PAD;  // padded tile by buffer loads to LDS
  constexpr bool SLABWT = (PV & 16) != 0;
  constexpr bool LMAP = (PV & 8) != 0 && ANGL && !((PV & 1) != 0 && persist_pad(LT) > 0) &&
                        ((LT + 1) * (LT + 1) * 10) % 32 == 26;
  constexpr int C = kTileFastC;
  constexpr int Sw = 64 / C;
  constexpr int MC = (LT + 1) * (LT + 1) * C;
  constexpr int MC4 = (MC + 3) & ~3;
  constexpr int kRow = TrigLds<LT>::kRow;
  constexpr int kTile = persist_tile_floats(LT, PAD);
  constexpr int kStride = persist_stride(LT, PAD);  // floats between samples of the tile
  constexpr int kPadB = 4 * (kStride - MC);         // pad bytes per sample
  constexpr int kTrig = Sw * kRow;
  // angle partials per buffer: [wave][sample][3] (tree), or (ANGL) three planes [wave][lane]
  // kPl floats apart -- 4 floats more than a plane, so that the summing lanes' 8-byte reads
  // of the three planes fall in distinct banks
  constexpr int kPl = NW * 64 + 4;
  constexpr int kAp = ANGL ? 3 * kPl : NW * 64 * 3;
  constexpr int nthr = 64 * NW;
  constexpr int NB = DB ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* const tiles = lds;                 // [NB][kTile]
  float* const trig = tiles + NB * kTile;   // [2][Sw][kRow]
  float* const apart = trig + 2 * kTrig;    // [2][NW][64][3]
  float* const slab = apart + 2 * kAp;      // [MC4]
  float* const Fsp = slab + MC4;            // [MC4], row-major (M, C)

  const int tid = (int)threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int j, c;
  if constexpr (LMAP) {
    const int jc = kPersistLaneJC[lane];
    j = jc >> 4;
    c = jc & 15;
  } else {
    j = lane / C;
    c = lane - j * C;
  }
  const unsigned dmask = a.seg_mask[wave];
  const int64_t P = gridDim.x;
  const int64_t groups = a.groups;
  const int64_t n = a.n;
  // prologue task of this thread: task t = lane * NW + wave (spread over the waves), or
  // (A/B) t = lane of the last wave; the angle sums (step 7) keep the spread numbering
  const int t_task = lane * NW + wave;
  const int t_fill = (a.variant & kBwdVarPersistTask1) ? (wave == NW - 1 ? lane : 64) : t_task;
  const bool task = t_fill < 3 * Sw;
  const int jt = t_fill / 3, q = t_fill - 3 * (t_fill / 3);
  // A/B timeline (LV_STAMPS=1): phase stamps of the block's 5th group (steady state)
  auto st = [&](int kk, int ph) {
    if (kk == 4 && a.stamps) phase_stamp(a.stamps, wave, ph);
  };
  // all groups' tiles sit at the same offset mod 16 (Sw * MC * 4 = 29,040 B at l = 10)
  const int mis = (int)(reinterpret_cast<uintptr_t>(a.gout) & 15);

  // the group's gradient tile, global -> LDS by LDS-DMA: 16-byte pieces (1 KiB per wave
  // instruction) spread over the waves, 4-byte head / tail pieces
  auto issue_tile = [&](int64_t g, int buf) {
    const int64_t s0 = g * Sw;
    const int Sv = (int)min((int64_t)Sw, n - s0);
    const int nbytes = Sv * MC * 4;
    const char* gb = reinterpret_cast<const char*>(a.gout + s0 * MC);
    char* stage_b = reinterpret_cast<char*>(tiles + buf * kTile) + mis;
    if constexpr (PAD) {
      // LDS span of the padded tile: up to the last sample's data end
      const int span = (Sv - 1) * kStride * 4 + MC * 4;
      const int head = min((16 - mis) & 15, span);
      const int nvec = (span - head) >> 4;
      const int tail0 = head + nvec * 16;
      if constexpr (PADBUF) {
        // the same pieces by buffer loads: the group's bytes as a buffer resource, a piece's
        // source offset from its LDS offset by one constant division (no 64-bit address)
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(gb), 0, nbytes, kRawBufferFlags);
        for (int v0 = wave * 64; v0 < nvec; v0 += nthr)
          if (v0 + lane < nvec) {
            const int rel = head + 16 * (v0 + lane);
            const int jp = (rel + 15) / (kStride * 4);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, as_lds(stage_b + head + 16 * v0), 16, rel - jp * kPadB, 0, 0, 0);
          }
        if (wave == NW - 1) {
          if (4 * lane < head) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, as_lds(stage_b), 4, 4 * lane, 0, 0, 0);
          const int tb = tail0 + 4 * lane;
          if (tb < span)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, as_lds(stage_b + tail0), 4, tb - (Sv - 1) * kPadB, 0, 0, 0);
        }
        return;
      }
      for (int v0 = wave * 64; v0 < nvec; v0 += nthr)
        if (v0 + lane < nvec) {
          // piece at LDS offset rel: the sample holding its last byte, its global bytes
          // (a piece in a pad reads the neighbouring sample's bytes: in bounds, never used)
          const int rel = head + 16 * (v0 + lane);
          const int jp = (rel + 15) / (kStride * 4);
          __builtin_amdgcn_global_load_lds(gb + rel - jp * kPadB, as_lds(stage_b + head + 16 * v0), 16, 0, 0);
        }
      if (wave == NW - 1) {
        // head: the first sample's bytes (no pad before it); tail: the last sample's
        if (4 * lane < head) __builtin_amdgcn_global_load_lds(gb + 4 * lane, as_lds(stage_b), 4, 0, 0);
        const int tb = tail0 + 4 * lane;
        if (tb < span)
          __builtin_amdgcn_global_load_lds(gb + tb - (Sv - 1) * kPadB, as_lds(stage_b + tail0), 4, 0, 0);
      }
      (void)nbytes;
      return;
    }
    const int head = min((16 - mis) & 15, nbytes);
    const int nvec = (nbytes - head) >> 4;
    const int tail0 = head + nvec * 16;
    if constexpr (BUFDMA) {
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(gb), 0, nbytes, kRawBufferFlags);
      const int vo = head + 16 * (wave * 64 + lane);  // this lane's piece in round 0
      char* const ldsw = stage_b + head + 16 * (wave * 64);
      const int nfull = nvec / nthr;  // rounds in which every lane of every wave has a piece
      for (int it = 0; it < nfull; ++it)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, as_lds(ldsw + it * nthr * 16), 16, vo, it * nthr * 16, 0, 0);
      if (nfull * nthr + wave * 64 + lane < nvec)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, as_lds(ldsw + nfull * nthr * 16), 16, vo, nfull * nthr * 16, 0, 0);
      if (wave == NW - 1) {
        if (4 * lane < head) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, as_lds(stage_b), 4, 4 * lane, 0, 0, 0);
        if (tail0 + 4 * lane < nbytes)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, as_lds(stage_b + tail0), 4, 4 * lane, tail0, 0, 0);
      }
      return;
    }
    for (int v0 = wave * 64; v0 < nvec; v0 += nthr)
      if (v0 + lane < nvec)
        __builtin_amdgcn_global_load_lds(gb + head + 16 * (v0 + lane), as_lds(stage_b + head + 16 * v0), 16, 0, 0);
    if (wave == NW - 1) {
      if (4 * lane < head) __builtin_amdgcn_global_load_lds(gb + 4 * lane, as_lds(stage_b), 4, 0, 0);
      if (tail0 + 4 * lane < nbytes)
        __builtin_amdgcn_global_load_lds(gb + tail0 + 4 * lane, as_lds(stage_b + tail0), 4, 0, 0);
    }
  };
  // the stored angle a task's slot uses (transpose: slot q takes angle 2 - q)
  auto task_angle = [&](int64_t g) -> float {
    const int64_t s0 = g * Sw;
    const int Sv = (int)min((int64_t)Sw, n - s0);
    return a.ang[(s0 + min(jt, Sv - 1)) * 3 + (a.transpose ? 2 - q : q)];
  };
  auto task_fill = [&](float ang, int buf) {
    // straight-line sincos (Cody-Waite + minimax, <= 1.6 ulp; action_common.h): the
    // library sincosf's range-reduction branches sat on every group's prologue path
    float cq, sq;
    lv_sincos(ang, sq, cq);
    if (a.transpose) sq = -sq;
    trig_row_fill1<LT>(trig + buf * kTrig + jt * kRow, cq, sq, q, LT);
  };

  int64_t g = blockIdx.x;
  // ---- first group: its tile, its multiples; the spectrum; the zeroed slab
  float ang_next = 0.f;
  if (task) ang_next = task_angle(g);
  issue_tile(g, 0);
  {
    constexpr int kFPer = (MC + nthr - 1) / nthr;
    float fv[kFPer];
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {
      const int e = tid + nthr * k;
      fv[k] = e < MC ? a.F[e] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < kFPer; ++k) {
      const int e = tid + nthr * k;
      if (e < MC) {
        Fsp[e] = fv[k];
        slab[e] = 0.f;
      }
    }
  }
  if (task) task_fill(ang_next, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  block_sync_lds();

  const float* Fl = Fsp + c;
  // the flat slab pass (step 3): this wave's element pairs, the tile's 8-byte alignment
  constexpr int kPR = 3;
  int npairs = 0;
  for (unsigned m = dmask; m; m &= m - 1) npairs += 5 * (2 * __builtin_ctz(m) + 1);
  const bool pair_ok = (mis & 7) == 0 && npairs <= 64 * kPR;
  // this lane's pair offsets in the wave's rows (-1: none), fixed for the whole walk
  int poff[kPR];
#pragma unroll
  for (int uu = 0; uu < kPR; ++uu) {
    const int pp = lane + 64 * uu;
    int o = 0, acc = 0;
    for (unsigned m = dmask; m; m &= m - 1) {
      const int l = __builtin_ctz(m);
      const int np = 5 * (2 * l + 1);
      if (pp >= acc && pp < acc + np) o = l * l * C + 2 * (pp - acc);
      acc += np;
    }
    poff[uu] = pp < npairs ? o : -1;
  }
  for (int k = 0; g < groups; ++k, g += P) {
    const int cur = k & 1, nxt = cur ^ 1;
    const int tcur = DB ? cur : 0;
    const int64_t gn = g + P;
    const bool has_next = gn < groups;
    st(k, 0);
    // 1. next group's angle loads (task lanes), then (double buffer) its gradient tile by
    //    LDS-DMA; a single buffer is refilled after this group's barrier (step 7)
    if (task && has_next) ang_next = task_angle(gn);
    if (DB && has_next) issue_tile(gn, nxt);

    // 2. this group's chain over the wave's degrees, largest first
    const int64_t s0 = g * Sw;
    const int Sv = (int)min((int64_t)Sw, n - s0);
    const bool active = j < Sv;
    char* stage_b = reinterpret_cast<char*>(tiles + tcur * kTile) + mis;
    float* tile_lane = reinterpret_cast<float*>(stage_b) + j * kStride + c;
    const float* tj = trig + cur * kTrig + min(j, Sw - 1) * kRow;
    float ga = 0.f, gb = 0.f, gc = 0.f;
    sfor<LT + 1>([&](auto Lc) {
      constexpr int l = LT - LV_CV(Lc);
      if ((dmask >> l) & 1u) {
        constexpr int nn = 2 * l + 1;
        constexpr int r0 = l * l;
        float p2[nn], p4[nn], u[nn];
        const float* fcol = Fl + r0 * C;
        if constexpr (JIT) {
          xm_mem<l, false>(mult_lds<l, 2, LT>(tj), fcol, C, u);           // P1
        } else {
          float f0[nn];
          sfor<nn>([&](auto K) { f0[LV_CV(K)] = fcol[LV_CV(K) * C]; });
          xm<l>(mult_lds<l, 2, LT>(tj), f0, u);
        }
        jmul<l>(u, p2);                                                    // P2
        xm<l>(mult_lds<l, 1, LT>(tj), p2, u);                              // P3
        jmul<l>(u, p4);                                                    // P4
        if constexpr (JIT) {
          xm_mem<l, true>(mult_lds<l, 0, LT>(tj), tile_lane + r0 * C, C, u);  // Q4
        } else {
          float gq[nn];
          sfor<nn>([&](auto K) { gq[LV_CV(K)] = tile_lane[(r0 + LV_CV(K)) * C]; });
          xm_t<l>(mult_lds<l, 0, LT>(tj), gq, u);
        }
        ga += kdot<l>(u, p4);
        jmul<l>(u, p4);                                                    // Q3
        xm_t<l>(mult_lds<l, 1, LT>(tj), p4, u);                            // Q2
        gb += kdot<l>(u, p2);
        jmul<l>(u, p2);                                                    // Q1
        xm_t<l>(mult_lds<l, 2, LT>(tj), p2, u);                            // dF column
        if constexpr (JIT) {
          gc += kdot_mem<l>(u, fcol, C);
        } else {
          float f0[nn];
          sfor<nn>([&](auto K) { f0[LV_CV(K)] = fcol[LV_CV(K) * C]; });
          gc += kdot<l>(u, f0);
        }
        if (active) sfor<nn>([&](auto I) { tile_lane[(r0 + LV_CV(I)) * C] = u[LV_CV(I)]; });
      }
    });
    st(k, 1);
    // 3. this wave's dF rows summed over the group's samples (sample order), added to the
    //    block's slab (groups in the block's order)
    wave_lds_sync();
    if (pair_ok && Sv == Sw) {
      // full group, 8-byte aligned tile: the wave's rows as ONE flat list of element pairs
      // (a degree's 10 (2l+1) elements are whole pairs), up to kPR rounds of 64 pairs with
      // every 8-byte load issued before any sum: one LDS round trip for the loads, one for
      // the slab's read-modify-write (the per-degree passes took 3-6)
      typedef float f2 __attribute__((ext_vector_type(2)));
      const float* t0 = reinterpret_cast<const float*>(stage_b);
      f2 v[kPR][Sw];
      const int* off = poff;
#pragma unroll
      for (int uu = 0; uu < kPR; ++uu) {
#pragma unroll
        for (int jj = 0; jj < Sw; ++jj)
          v[uu][jj] = *reinterpret_cast<const f2*>(t0 + jj * kStride + (off[uu] < 0 ? 0 : off[uu]));
      }
#pragma unroll
      for (int uu = 0; uu < kPR; ++uu) {
        f2 sum = v[uu][0];
#pragma unroll
        for (int jj = 1; jj < Sw; ++jj) sum += v[uu][jj];
        if (off[uu] >= 0) *reinterpret_cast<f2*>(slab + off[uu]) += sum;
      }
    } else {
      const float* t0 = reinterpret_cast<const float*>(stage_b);
      for (unsigned m = dmask; m; m &= m - 1) {
        const int l = __builtin_ctz(m);
        const int base = l * l * C, cnt = (2 * l + 1) * C;
        if (Sv == Sw) {
          constexpr int kU = 4;
          for (int e0 = lane; e0 < cnt; e0 += kU * 64) {
            float v[kU][Sw];
#pragma unroll
            for (int uu = 0; uu < kU; ++uu) {
              const int e = base + min(e0 + 64 * uu, cnt - 1);
#pragma unroll
              for (int jj = 0; jj < Sw; ++jj) v[uu][jj] = t0[jj * kStride + e];
            }
#pragma unroll
            for (int uu = 0; uu < kU; ++uu) {
              float sum = v[uu][0];
#pragma unroll
              for (int jj = 1; jj < Sw; ++jj) sum += v[uu][jj];
              if (e0 + 64 * uu < cnt) slab[base + e0 + 64 * uu] += sum;
            }
          }
        } else {
          for (int e = lane; e < cnt; e += 64) {
            float sum = t0[base + e];
            for (int jj = 1; jj < Sv; ++jj) sum += t0[jj * kStride + base + e];
            slab[base + e] += sum;
          }
        }
      }
    }
    st(k, 2);
    // 4. (double buffer) the next group's multiples (its angles have long landed)
    if (DB && task && has_next) task_fill(ang_next, nxt);
    // 5. angle partials: the C column lanes of each sample summed by a segmented
    //    cross-lane tree (((c0 + c1) + (c2 + c3)) + ((c4 + c5) + (c6 + c7))) + (c8 + c9), then
    //    one (sample, angle) value per wave into the partial buffer; (ANGL) every lane's
    //    three partials straight to the buffer, [angle][wave][lane]
    if constexpr (ANGL) {
      float* ap = apart + cur * kAp + wave * 64 + (j * C + c);  // [angle][wave][sample][column]
      ap[0] = ga;
      ap[kPl] = gb;
      ap[2 * kPl] = gc;
    } else {
      float v0 = ga, v1 = gb, v2 = gc;
#pragma unroll
      for (int off = 1; off < C; off <<= 1) {
        const float t0 = __shfl_down(v0, off, 64), t1 = __shfl_down(v1, off, 64), t2 = __shfl_down(v2, off, 64);
        if ((c & (2 * off - 1)) == 0 && c + off < C) {
          v0 += t0;
          v1 += t1;
          v2 += t2;
        }
      }
      if (c == 0 && j < Sw) {
        float* ap = apart + cur * kAp + (wave * Sw + j) * 3;
        if (a.transpose) {
          ap[0] = -v2; ap[1] = -v1; ap[2] = -v0;
        } else {
          ap[0] = v0; ap[1] = v1; ap[2] = v2;
        }
      }
    }
    if constexpr (DB) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's share of the next tile
    st(k, 3);
    block_sync_lds();
    st(k, 4);
    // 6. (one buffer) every wave is past this group's chain and slab pass: the tile takes
    //    the next group now, and the angle sums and the next multiples run under its DMA
    if (!DB && has_next) issue_tile(gn, 0);
    // 7. the group's angle gradients (waves in order), output t on lane t / NW of wave t % NW;
    //    (ANGL) output t = (sample, angle) on lane t of wave 0: its 4 waves x 10 columns of
    //    partials read as 8-byte pairs, summed column-pairwise then over the waves
    if constexpr (ANGL) {
      if (wave == 0 && lane < 3 * Sv) {
        const int js = lane / 3, i = lane - 3 * (lane / 3);
        // transpose: angle i is the negated sum of stored component 2 - i
        const int ci = a.transpose ? 2 - i : i;
        typedef float f2 __attribute__((ext_vector_type(2)));
        const float* apc = apart + cur * kAp + ci * kPl + js * C;
        f2 pv[NW][C / 2];
#pragma unroll
        for (int w = 0; w < NW; ++w)
#pragma unroll
          for (int k = 0; k < C / 2; ++k) pv[w][k] = *reinterpret_cast<const f2*>(apc + w * 64 + 2 * k);
        float r = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          f2 t = pv[w][0];
#pragma unroll
          for (int k = 1; k < C / 2; ++k) t += pv[w][k];
          r += t[0] + t[1];
        }
        a.gang[(s0 + js) * 3 + i] = a.transpose ? -r : r;
      }
    } else if (t_task < 3 * Sv) {
      const int js = t_task / 3, i = t_task - 3 * (t_task / 3);
      const float* apc = apart + cur * kAp;
      float r = apc[js * 3 + i];
#pragma unroll
      for (int w = 1; w < NW; ++w) r += apc[(w * Sw + js) * 3 + i];
      a.gang[(s0 + js) * 3 + i] = r;
    }
    if constexpr (!DB) {
      if (has_next) {
        if (task) task_fill(ang_next, nxt);
        st(k, 5);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st(k, 6);
        block_sync_lds();
        st(k, 7);
      }
    }
  }
  // ---- the block's slab (each wave its own rows) to the workspace, chunk-major
  if constexpr (SLABWT) {
    block_sync_lds();  // every wave's slab rows are final
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int nch = (MC + kSlabChunk - 1) / kSlabChunk;
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(a.ws_F, 0, nch * (int)gridDim.x * kSlabChunk * 4, kRawBufferFlags);
    // piece (chunk q, quarter k): slab[16 q + 4 k ..] -> ws_F[q * grid * 16 + block * 16 + 4 k ..]
    // (the last chunk's pad reads the next LDS floats: summed by reduce5, never stored to gF)
    for (int pc = tid; pc < 4 * nch; pc += nthr) {
      const int q = pc >> 2, k = pc & 3;
      const f4 v = *reinterpret_cast<const f4*>(slab + kSlabChunk * q + 4 * k);
      __builtin_amdgcn_raw_buffer_store_b128(v, rw, ((q * (int)gridDim.x + (int)blockIdx.x) * kSlabChunk + 4 * k) * 4,
                                             0, 16);
    }
    return;
  }
  for (unsigned m = dmask; m; m &= m - 1) {
    const int l = __builtin_ctz(m);
    const int g0 = l * l * C, cnt = (2 * l + 1) * C;
    float* ws = a.ws_F + (int64_t)blockIdx.x * kSlabChunk;
    const int64_t cstride = (int64_t)gridDim.x * kSlabChunk;
    for (int e = lane; e < cnt; e += 64) {
      const int gg = g0 + e;
      ws[(gg / kSlabChunk) * cstride + gg % kSlabChunk] = slab[gg];
    }
  }
}

}  // namespace lv

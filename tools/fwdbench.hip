// Standalone A/B harness for the config-2 forward (l = 10, C = 10, fp32, fused exp):
// the library's tile kernel against the stream kernels of tools/fwd_experiments.h, every
// variant checked bitwise against the tile kernel, then timed over back-to-back launches
// with HIP events.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
//     -I lie-vae_amd/csrc tools/fwdbench.hip -o tools/kbench_fwd
//   ./tools/kbench_fwd [n] [reps] [occ]
#include <algorithm>
#include <string>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fwd_experiments.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

using namespace lv;
constexpr int L = 10, C = 10;

template <int... Ls>
constexpr std::array<int, sizeof...(Ls)> nnz_tab(std::integer_sequence<int, Ls...>) { return {j_nnz<Ls>()...}; }

static void plan(int nseg, double P, int* seg) {
  auto nnz = nnz_tab(std::make_integer_sequence<int, L + 1>{});
  const int D = L + 1;
  std::vector<double> pre(D + 1, 0);
  for (int l = 0; l < D; ++l) pre[l + 1] = pre[l] + 2.0 * nnz[l] + 9.0 * (2 * l + 1);
  std::vector<std::vector<double>> dp(nseg + 1, std::vector<double>(D + 1, 1e30));
  std::vector<std::vector<int>> arg(nseg + 1, std::vector<int>(D + 1, 0));
  dp[0][0] = 0;
  for (int k = 1; k <= nseg; ++k)
    for (int i = 1; i <= D; ++i)
      for (int p = k - 1; p < i; ++p) {
        double v = std::max(dp[k - 1][p], pre[i] - pre[p] + P);
        if (v < dp[k][i]) { dp[k][i] = v; arg[k][i] = p; }
      }
  int i = D;
  for (int k = nseg; k >= 1; --k) { seg[k] = i; i = arg[k][i]; }
  seg[0] = 0;
}

static int fslice(const ActionArgs& a, int nseg) {
  int fp = 0;
  for (int k = 0; k < nseg; ++k) fp = std::max(fp, fseg_rows(a.seg_lo[k], a.seg_lo[k + 1]) * C);
  return (fp + 3) & ~3;
}

typedef void (*Kern)(ActionArgs);

// Every launch is checked: a block larger than the kernel's __launch_bounds__ (or an LDS
// request beyond the CU) fails to launch, and timing such "launches" measures nothing.
static double timeit(Kern k, dim3 g, dim3 b, size_t lds, const ActionArgs& a, int reps) {
  for (int w = 0; w < 20; ++w) {
    hipLaunchKernelGGL(k, g, b, lds, 0, a);
    if (hipGetLastError() != hipSuccess) return -1.0;  // invalid configuration: no row
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(k, g, b, lds, 0, a);
    CK(hipGetLastError());
  }
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  return ms * 1e3 / reps;
}

static size_t check(Kern k, dim3 g, dim3 b, size_t lds, const ActionArgs& a, int64_t n,
                    const std::vector<float>& ref) {
  const size_t cnt = (size_t)n * a.MC;
  CK(hipMemset(a.out, 0xff, cnt * 4));
  hipLaunchKernelGGL(k, g, b, lds, 0, a);
  CK(hipDeviceSynchronize());
  std::vector<float> h(cnt);
  CK(hipMemcpy(h.data(), a.out, cnt * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < cnt; ++i) bad += memcmp(&h[i], &ref[i], 4) != 0;
  return bad;
}

template <int POL, int MODE, int FL>
static void run_stream(ActionArgs a, int64_t n, int nseg, int reps, const std::vector<float>& ref,
                       double bytes, const char* tag) {
  plan(nseg, 250.0, a.seg_lo);
  a.fpitch = fslice(a, nseg);
  const int wfl = a.fpitch + (MODE == 0 ? (64 / C) * stream_stage_pitch(L, C, FL) : 0);
  const size_t lds = 4 * (size_t)nseg * wfl;
  const int gx = (int)((n + a.Sw - 1) / a.Sw);
  Kern k = fwd_stream_kernel<L, C, true, POL, MODE, FL>;
  const size_t bad = check(k, dim3(gx), dim3(64 * nseg), lds, a, n, ref);
  const double us = timeit(k, dim3(gx), dim3(64 * nseg), lds, a, reps);
  printf("n=%lld %-10s mode=%d FL=%d pol=%2d nseg=%d lds=%5zu: %8.2f us %6.0f GB/s %s\n",
         (long long)n, tag, MODE, FL, POL, nseg, lds, us, bytes / us / 1e3,
         bad ? "MISMATCH" : "bitwise-ok");
  if (bad) printf("   %zu elements differ\n", bad);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 4096;
  const int reps = argc > 2 ? atoi(argv[2]) : 500;
  const int M = (L + 1) * (L + 1);
  std::vector<float> hv(n * 3), hF(M * C);
  srand(1);
  for (auto& x : hv) x = (rand() / (float)RAND_MAX - 0.5f) * 3.f;
  for (auto& x : hF) x = rand() / (float)RAND_MAX - 0.5f;
  float *v, *F, *out;
  CK(hipMalloc(&v, n * 3 * 4));
  CK(hipMalloc(&F, M * C * 4));
  CK(hipMalloc(&out, (size_t)n * M * C * 4 + 64));
  CK(hipMemcpy(v, hv.data(), n * 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(F, hF.data(), M * C * 4, hipMemcpyHostToDevice));
  ActionArgs a{};
  a.v = v; a.F = F; a.Fstride = 0; a.out = out; a.n = n; a.MC = M * C; a.C = C; a.Sw = 64 / C;
  const double bytes = (double)n * (12 + M * C * 4) + M * C * 4;
  const int gx = (int)((n + a.Sw - 1) / a.Sw);

  // floor_kernel is __launch_bounds__(512): at most 8 waves per block
  for (int nw : {4, 5, 8}) {
    const int gb = std::max(1, gx * 4 / nw);
    const double f0 = timeit(floor_kernel<0>, dim3(gb), dim3(64 * nw), 0, a, reps);
    const double f1 = timeit(floor_kernel<1>, dim3(gb), dim3(64 * nw), 0, a, reps);
    if (f0 < 0 || f1 < 0) { printf("floor %d waves/block: launch failed\n", nw); continue; }
    printf("n=%lld floor %d waves/block x %d blocks: empty %.2f  loads %.2f us\n", (long long)n, nw, gb, f0, f1);
  }
  // reference + baseline: the library's tile kernel (C = 10 specialisation)
  std::vector<float> ref((size_t)n * M * C);
  auto lib_tile = [&](int nseg, int wt, bool keep, size_t pad = 0) {
    ActionArgs b = a;
    plan(nseg, 60.0, b.seg_lo);
    b.fpitch = fslice(b, nseg);
    b.write_through = wt;
    const size_t lds = pad + tile_stage_bytes(b.Sw, b.MC, 4) + 4 * ((size_t)b.Sw * TrigLds<L>::kRow);  // spectrum in the tile
    Kern k = action_fwd_tile_kernel<L, C, true, float>;
    if (keep) {
      hipLaunchKernelGGL(k, dim3(gx), dim3(64 * nseg), lds, 0, b);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(ref.data(), out, ref.size() * 4, hipMemcpyDeviceToHost));
    }
    return timeit(k, dim3(gx), dim3(64 * nseg), lds, b, reps);
  };
  lib_tile(4, 1, true);
  if (argc > 3 && std::string(argv[3]) == "occ") {
    // occupancy sensitivity: pad the block's LDS so fewer blocks fit per CU (160 KB)
    const size_t base = tile_stage_bytes(a.Sw, a.MC, 4) + 4 * ((size_t)a.Sw * TrigLds<L>::kRow);
    for (int per_cu : {5, 4, 2})
      for (int nseg : {4, 5, 6}) {
        const size_t want = 160 * 1024 / per_cu - 64;
        const size_t pad = per_cu == 5 ? 0 : ((want - base) & ~(size_t)15);
        printf("n=%lld occ blocks/CU<=%d (lds %zu) nseg=%d: sc1 %8.2f us  nt %8.2f us\n", (long long)n,
               per_cu, base + pad, nseg, lib_tile(nseg, 1, false, pad), lib_tile(nseg, 0, false, pad));
      }
    return 0;
  }
  const int wt = n * M * C * 4 <= (24ll << 20) ? 1 : 0;  // the library's store policy
  for (int nseg : {4, 5, 6, 7, 8})
    printf("n=%lld lib tile nseg=%d: %s %8.2f us\n", (long long)n, nseg, wt ? "sc1" : "nt", lib_tile(nseg, wt, false));
  auto occ = [&](Kern k, int nseg) {
    ActionArgs b = a;
    plan(nseg, 60.0, b.seg_lo);
    b.fpitch = fslice(b, nseg);
    b.write_through = wt;
    const size_t lds = tile_stage_bytes(b.Sw, b.MC, 4) + 4 * ((size_t)b.Sw * TrigLds<L>::kRow);
    const size_t bad = check(k, dim3(gx), dim3(64 * nseg), lds, b, n, ref);
    const double t = timeit(k, dim3(gx), dim3(64 * nseg), lds, b, reps);
    return std::make_pair(t, bad);
  };
  for (int nseg : {4, 5, 6}) {
    auto a0 = occ(action_fwd_tile_kernel<L, C, true, float>, nseg);
    auto a1 = occ(tile_nomu_kernel<L, C>, nseg);
    auto a2 = occ(tile_w8_kernel<L, C, true>, nseg);
    auto a3 = occ(tile_w8_kernel<L, C, false>, nseg);
    printf("n=%lld nseg=%d: lib %7.2f | nomu %7.2f%s | w8 %7.2f%s | nomu+w8 %7.2f%s us\n", (long long)n, nseg,
           a0.first, a1.first, a1.second ? " DIFF" : "", a2.first, a2.second ? " DIFF" : "", a3.first,
           a3.second ? " DIFF" : "");
  }
  if (!(argc > 3 && std::string(argv[3]) == "twophase")) return 0;
  // two-phase tile kernel: degrees [0, L1) then [L1, L], the first part's rows written
  // while the second part computes
  auto plan_range = [&](int lo, int hi, int nseg, int* seg) {
    auto nnz = nnz_tab(std::make_integer_sequence<int, L + 1>{});
    std::vector<double> cost;
    for (int l = lo; l < hi; ++l) cost.push_back(2.0 * nnz[l] + 12.0 * l + 10.0);
    double tot = 0; for (double x : cost) tot += x;
    int k = 0; double acc = 0; seg[0] = lo;
    for (int l = lo; l < hi && k < nseg - 1; ++l) {
      acc += cost[l - lo];
      if (acc >= tot * (k + 1) / nseg) { seg[++k] = l + 1; }
    }
    while (k < nseg - 1) { seg[k + 1] = seg[k]; ++k; }
    seg[nseg] = hi;
  };
  for (int L1 : {6, 7, 8})
    for (int nseg : {4, 5, 6, 7}) {
      ActionArgs b = a;
      plan_range(0, L1, nseg, b.seg_lo);
      plan_range(L1, L + 1, nseg, b.seg_lo + nseg + 1);
      const size_t l6 = tile_stage_bytes(b.Sw, b.MC, 4) + 4 * ((size_t)b.MC + (size_t)b.Sw * TrigLds<L>::kRow);
      const dim3 g(gx), bl(64 * nseg);
      const size_t bad = check(tile6_kernel<L, 16>, g, bl, l6, b, n, ref);
      const double t16 = timeit(tile6_kernel<L, 16>, g, bl, l6, b, reps);
      const double t1 = timeit(tile6_kernel<L, 1>, g, bl, l6, b, reps);
      printf("n=%lld two-phase L1=%d nseg=%d: sc1 %8.2f  nt %8.2f us  %s\n", (long long)n, L1, nseg, t16, t1,
             bad ? "MISMATCH" : "bitwise-ok");
    }
  return 0;
  // tile v5: trig from LDS per degree (TM 1), per-wave flush (FM 1)
  auto t5 = [&](auto tm, auto fm, int nseg, const char* tag) {
    constexpr int TM = decltype(tm)::value, FM = decltype(fm)::value;
    ActionArgs b = a;
    plan(nseg, 60.0, b.seg_lo);
    b.fpitch = (fslice(b, nseg) + 3) & ~3;
    const size_t l3 = ((64 / C) * M * C * 4 + 16 + 15) / 16 * 16 + 4 * (size_t)(64 / C) * 3 * t3_row(L) +
                      4 * (size_t)nseg * b.fpitch;
    const dim3 g(gx), bl(64 * nseg);
    const size_t bad = check(tile5_kernel<L, C, true, float, 16, TM, FM>, g, bl, l3, b, n, ref);
    const double t16 = timeit(tile5_kernel<L, C, true, float, 16, TM, FM>, g, bl, l3, b, reps);
    const double t1 = timeit(tile5_kernel<L, C, true, float, 1, TM, FM>, g, bl, l3, b, reps);
    const double t0 = timeit(tile5_kernel<L, C, true, float, 0, TM, FM>, g, bl, l3, b, reps);
    printf("n=%lld tile5 %s nseg=%d: sc1 %8.2f  nt %8.2f  plain %8.2f us (best %.0f GB/s) %s\n", (long long)n, tag, nseg,
           t16, t1, t0, bytes / std::min(std::min(t1, t16), t0) / 1e3, bad ? "MISMATCH" : "bitwise-ok");
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  for (int nseg : {3, 4, 5, 6, 8}) {
    t5(I1{}, I0{}, nseg, "ldstrig      ");
    t5(I0{}, I1{}, nseg, "waveflush    ");
    t5(I1{}, I1{}, nseg, "ldstrig+wflsh");
  }
  return 0;
}

// Standalone harness: row-pair forward (action_fwd_kernel) vs tile forward
// (action_fwd_tile_kernel) at l_max = 10, C = 10, fp32, with the tile kernel's store
// cache policy and segment count swept.  Checks the tile outputs bitwise against the
// row-pair kernel, then times back-to-back launches with HIP events.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
//     -I lie-vae_amd/csrc tools/tilebench.hip -o tools/kbench_tile
//   ./tools/kbench_tile [n] [reps]
#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "tile_experiments.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

using namespace lv;
constexpr int L = 10;

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

template <int POL, int V = 1, bool WF = false>
static double run_tile(ActionArgs a, int nseg, int reps, float* out, std::vector<float>& ref, int64_t n, bool check) {
  plan(nseg, V == 1 ? 250.0 : 40.0, a.seg_lo);
  int fp = 0;
  for (int k = 0; k < nseg; ++k) fp = std::max(fp, fseg_rows(a.seg_lo[k], a.seg_lo[k + 1]) * a.C);
  a.fpitch = (fp + 3) & ~3;
  const size_t lds = tile_stage_bytes(a.Sw, a.MC, 4) + 4 * (size_t)nseg * a.fpitch +
                     (V == 2 ? 4 * (size_t)tile2_trig_floats(a.Sw, L) : 0);
  const int gx = (int)((n + a.Sw - 1) / a.Sw);
  auto k = V == 1 ? action_fwd_tile_kernel<L, true, float, POL, WF> : action_fwd_tile2_kernel<L, true, float, POL>;
  if (check) {
    CK(hipMemset(out, 0, (size_t)n * a.MC * 4));
    hipLaunchKernelGGL(k, dim3(gx), dim3(64 * nseg), lds, 0, a);
    CK(hipDeviceSynchronize());
    std::vector<float> h((size_t)n * a.MC);
    CK(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < h.size(); ++i) bad += memcmp(&h[i], &ref[i], 4) != 0;
    if (bad) printf("  MISMATCH v%d pol=%d nseg=%d: %zu of %zu differ\n", V, POL, nseg, bad, h.size());
  }
  for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k, dim3(gx), dim3(64 * nseg), lds, 0, a);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(gx), dim3(64 * nseg), lds, 0, a);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / reps;
}

// pipelined tile kernel: nseg waves per block, grid G blocks (0 = one block per group)
static double run_tilep(ActionArgs a, int nseg, int G, int wt, int reps, float* out,
                        std::vector<float>& ref, int64_t n, bool check) {
  plan(nseg, 40.0, a.seg_lo);
  int fp = 0;
  for (int k = 0; k < nseg; ++k) fp = std::max(fp, fseg_rows(a.seg_lo[k], a.seg_lo[k + 1]) * a.C);
  a.fpitch = (fp + 3) & ~3;
  a.write_through = wt;
  const size_t lds = 2 * (size_t)tile_stage_bytes(a.Sw, a.MC, 4) +
                     4 * (size_t)tilep_trig_floats(a.Sw, L) + 4 * (size_t)nseg * a.fpitch;
  const int groups = (int)((n + a.Sw - 1) / a.Sw);
  const int gx = G <= 0 ? groups : std::min(G, groups);
  auto k = action_fwd_tilep_kernel<L, true, float>;
  if (check) {
    CK(hipMemset(out, 0, (size_t)n * a.MC * 4));
    hipLaunchKernelGGL(k, dim3(gx), dim3(64 * nseg), lds, 0, a);
    CK(hipDeviceSynchronize());
    std::vector<float> h((size_t)n * a.MC);
    CK(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < h.size(); ++i) bad += memcmp(&h[i], &ref[i], 4) != 0;
    if (bad) printf("  MISMATCH tilep nseg=%d G=%d: %zu of %zu differ\n", nseg, gx, bad, h.size());
  }
  for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k, dim3(gx), dim3(64 * nseg), lds, 0, a);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(gx), dim3(64 * nseg), lds, 0, a);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / reps;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 4096;
  const int reps = argc > 2 ? atoi(argv[2]) : 500;
  const int only = argc > 3 ? atoi(argv[3]) : 0;  // 1: tile v1 nseg 4 sc1 only (profiling)
  const int C = 10, M = (L + 1) * (L + 1);
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
#ifdef LV_STAMPS
  {  // every stamped kernel needs a valid buffer: size for the largest grid used below
    const size_t w = (size_t)((n + a.Sw - 1) / a.Sw) * 16 + 64;
    unsigned long long* sb0;
    CK(hipMalloc(&sb0, w * 64));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(lv_stamp_buf), &sb0, sizeof(sb0)));
  }
#endif

  // row-pair kernel, 4 segments (the library's plan at batch 4096)
  {
    ActionArgs b = a;
    const int nseg = 4;
    plan(nseg, 250.0, b.seg_lo);
    const int gx = (int)((n + b.Sw * kWavesPerBlock - 1) / (b.Sw * kWavesPerBlock));
    int fmax = 0;
    for (int k = 0; k < nseg; ++k) fmax = std::max(fmax, (fseg_rows(b.seg_lo[k], b.seg_lo[k + 1]) * C + 3) & ~3);
    auto k = action_fwd_kernel<L, true, true, float>;
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k, dim3(gx, nseg), dim3(kThreads), 4 * fmax, 0, b);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(gx, nseg), dim3(kThreads), 4 * fmax, 0, b);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("n=%lld rowpair nseg=4: %.2f us  %.0f GB/s\n", (long long)n, us, bytes / us / 1e3);
  }
  std::vector<float> ref((size_t)n * M * C);
  CK(hipMemcpy(ref.data(), out, ref.size() * 4, hipMemcpyDeviceToHost));

  if (only == 1) {
    std::vector<float> dummy;
    printf("tile v1 nseg=4 sc1: %.2f us\n", run_tile<16, 1>(a, 4, reps, out, dummy, n, false));
    return 0;
  }
  if (only == 2) {  // pipelined tile kernel sweep vs the library's tile kernel (5 seg, sc1)
    printf("n=%lld tile nseg=5 sc1: %.2f us\n", (long long)n,
           run_tile<16, 1>(a, 5, reps, out, ref, n, true));
    const int groups = (int)((n + a.Sw - 1) / a.Sw);
    for (int nseg : {4, 6, 8})
      for (int G : {256, 512, 1024, 0}) {
        if (G > groups) continue;
        const double t1 = run_tilep(a, nseg, G, 1, reps, out, ref, n, true);
        const double t0 = run_tilep(a, nseg, G, 0, reps, out, ref, n, false);
        printf("n=%lld tilep nseg=%d G=%d: sc1 %.2f  nt %.2f us  (best %.0f GB/s)\n", (long long)n,
               nseg, G ? G : groups, t1, t0, bytes / std::min(t0, t1) / 1e3);
      }
    return 0;
  }
#ifdef LV_STAMPS
  if (only == 3) {  // tilep phase stamps (first group of each block)
    for (int nseg : {4, 8})
      for (int G : {256, 683}) {
        const int waves = G * nseg;
        unsigned long long* sb;
        CK(hipMalloc(&sb, (size_t)waves * 64));
        CK(hipMemset(sb, 0, (size_t)waves * 64));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(lv_stamp_buf), &sb, sizeof(sb)));
        const double us = run_tilep(a, nseg, G, 1, 50, out, ref, n, false);
        std::vector<unsigned long long> hs((size_t)waves * 8);
        CK(hipMemcpy(hs.data(), sb, hs.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, tend = 0;
        for (int w = 0; w < waves; ++w) { t0 = std::min(t0, hs[w * 8]); tend = std::max(tend, hs[w * 8 + 6]); }
        printf("tilep nseg=%d G=%d: %.2f us/launch, stamped span %.2f us\n", nseg, G, us, (tend - t0) * 0.01);
        const char* names[7] = {"start", "F stage", "prologue", "chain0", "barrier0", "flush0", "rest"};
        const int from[7] = {-1, 0, 1, 2, 3, 4, 5}, to[7] = {0, 1, 2, 3, 4, 5, 6};
        for (int ph = 0; ph < 7; ++ph) {
          std::vector<double> v;
          for (int w = 0; w < waves; ++w) {
            auto* p = &hs[w * 8];
            v.push_back(from[ph] < 0 ? (p[0] - t0) * 0.01 : ((double)p[to[ph]] - (double)p[from[ph]]) * 0.01);
          }
          std::sort(v.begin(), v.end());
          printf("  %-9s min %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", names[ph], v[0], v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
        }
        CK(hipFree(sb));
      }
    return 0;
  }
  for (int ver : {1, 2})
  for (int nseg : {4, 5, 6}) {
    const int waves = (int)((n + a.Sw - 1) / a.Sw) * nseg;
    unsigned long long* sb;
    CK(hipMalloc(&sb, (size_t)waves * 64));
    CK(hipMemset(sb, 0, (size_t)waves * 64));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(lv_stamp_buf), &sb, sizeof(sb)));
    if (ver == 1) run_tile<16, 1>(a, nseg, 50, out, ref, n, false);
    else run_tile<16, 2>(a, nseg, 50, out, ref, n, false);
    std::vector<unsigned long long> hs((size_t)waves * 8);
    CK(hipMemcpy(hs.data(), sb, hs.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, tend = 0;
    for (int w = 0; w < waves; ++w) { t0 = std::min(t0, hs[w * 8]); tend = std::max(tend, hs[w * 8 + 4]); }
    const char* names[6] = {"start", "prologue", "F->LDS/b1", "chain", "barrier", "flush"};
    const int from[6] = {-1, 0, 1, 2, 5, 3}, to[6] = {0, 1, 2, 5, 3, 4};
    printf("v%d nseg=%d waves=%d span %.2f us (last launch of 50)\n", ver, nseg, waves, (tend - t0) * 0.01);
    for (int ph = 0; ph < 6; ++ph) {
      std::vector<double> v;
      for (int w = 0; w < waves; ++w) {
        auto* p = &hs[w * 8];
        v.push_back(from[ph] < 0 ? (p[0] - t0) * 0.01 : ((double)p[to[ph]] - (double)p[from[ph]]) * 0.01);
      }
      std::sort(v.begin(), v.end());
      printf("  %-9s min %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", names[ph], v[0], v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
    }
    std::vector<double> en;
    for (int w = 0; w < waves; ++w) en.push_back((hs[w * 8 + 4] - t0) * 0.01);
    std::sort(en.begin(), en.end());
    printf("  end       min %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", en[0], en[en.size() / 10], en[en.size() / 2], en[en.size() * 9 / 10], en.back());
    CK(hipFree(sb));
  }
  return 0;
#endif
  for (int nseg : {2, 3, 4, 5, 6, 8}) {
    double t0 = run_tile<0>(a, nseg, reps, out, ref, n, true);
    double t1 = run_tile<1>(a, nseg, reps, out, ref, n, false);
    double t16 = run_tile<16>(a, nseg, reps, out, ref, n, true);
    double t17 = run_tile<17>(a, nseg, reps, out, ref, n, false);
    printf("n=%lld tile nseg=%d: plain %.2f  nt %.2f  sc1 %.2f  sc0sc1 %.2f us   (best %.0f GB/s)\n",
           (long long)n, nseg, t0, t1, t16, t17, bytes / std::min(std::min(t0, t1), std::min(t16, t17)) / 1e3);
  }
  for (int nseg : {3, 4, 5, 6}) {
    double t0 = run_tile<0, 1, true>(a, nseg, reps, out, ref, n, true);
    double t1 = run_tile<1, 1, true>(a, nseg, reps, out, ref, n, false);
    double t16 = run_tile<16, 1, true>(a, nseg, reps, out, ref, n, true);
    double t17 = run_tile<17, 1, true>(a, nseg, reps, out, ref, n, false);
    printf("n=%lld tile-waveflush nseg=%d: plain %.2f  nt %.2f  sc1 %.2f  sc0sc1 %.2f us\n",
           (long long)n, nseg, t0, t1, t16, t17);
  }
  for (int nseg : {3, 4, 5, 6, 7, 8}) {
    double t0 = run_tile<0, 2>(a, nseg, reps, out, ref, n, true);
    double t1 = run_tile<1, 2>(a, nseg, reps, out, ref, n, false);
    double t16 = run_tile<16, 2>(a, nseg, reps, out, ref, n, true);
    printf("n=%lld tile2 nseg=%d: plain %.2f  nt %.2f  sc1 %.2f us   (best %.0f GB/s)\n",
           (long long)n, nseg, t0, t1, t16, bytes / std::min(std::min(t0, t1), t16) / 1e3);
  }
  return 0;
}

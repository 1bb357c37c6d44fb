// Standalone A/B harness for the config-2 backward (l = 10, C = 10, batch n, shared
// spectrum): the library's action_bwd_tile_kernel (C = 10, one group per block, 3 waves
// per SIMD) against the variants of tools/bwd_experiments.h.  Every variant that claims
// the same arithmetic is checked bit for bit (angle gradients and dF slabs) against the
// library's output; diagnostics (work dropped) are timed only.  Back-to-back launches,
// HIP events, every launch checked.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I lie-vae_amd/csrc \
//     tools/bwdbench.hip -o tools/kbench_bwd -L lie-vae_amd/lie_vae -llievae_hip \
//     -Wl,-rpath,'$ORIGIN/../lie-vae_amd/lie_vae'
//   ./tools/kbench_bwd [n] [reps]
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../tools/bwd_experiments.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

using namespace lv;
constexpr int L = 10, C = 10;

template <int... Ls>
constexpr std::array<int, sizeof...(Ls)> nnz_tab(std::integer_sequence<int, Ls...>) { return {j_nnz<Ls>()...}; }

// the library's segment DP (action.hip plan_segments, backward cost, prologue 60)
static void plan(int nseg, int* seg) {
  auto nnz = nnz_tab(std::make_integer_sequence<int, L + 1>{});
  const int D = L + 1;
  const double P = 60.0;
  std::vector<double> pre(D + 1, 0);
  for (int l = 0; l < D; ++l) pre[l + 1] = pre[l] + 2.2 * (2.0 * nnz[l] + 9.0 * (2 * l + 1));
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

typedef void (*Kern)(ActionBwdArgs);

static double timeit(Kern k, dim3 g, dim3 b, size_t lds, const ActionBwdArgs& a, int reps) {
  for (int w = 0; w < 20; ++w) {
    hipLaunchKernelGGL(k, g, b, lds, 0, a);
    if (hipGetLastError() != hipSuccess) return -1.0;
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

struct Out {
  std::vector<float> gang, ws;
};

static Out run_once(Kern k, dim3 g, dim3 b, size_t lds, const ActionBwdArgs& a, int64_t n, int64_t MC) {
  CK(hipMemset(a.gang, 0xff, n * 12));
  CK(hipMemset(a.ws_F, 0xff, (size_t)g.x * MC * 4));
  hipLaunchKernelGGL(k, g, b, lds, 0, a);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  Out o{std::vector<float>(n * 3), std::vector<float>((size_t)g.x * MC)};
  CK(hipMemcpy(o.gang.data(), a.gang, n * 12, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o.ws.data(), a.ws_F, o.ws.size() * 4, hipMemcpyDeviceToHost));
  return o;
}

static size_t ndiff(const std::vector<float>& x, const std::vector<float>& y) {
  size_t d = 0;
  for (size_t i = 0; i < x.size(); ++i) d += memcmp(&x[i], &y[i], 4) != 0;
  return d;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 4096;
  const int reps = argc > 2 ? atoi(argv[2]) : 300;
  const int M = (L + 1) * (L + 1);
  const int64_t MC = (int64_t)M * C;
  const int Sw = 64 / C;
  const int gx = (int)((n + Sw - 1) / Sw);
  std::vector<float> hang(n * 3), hF(MC), hg((size_t)n * MC);
  srand(3);
  for (auto& x : hang) x = (rand() / (float)RAND_MAX - 0.5f) * 6.2f;
  for (auto& x : hF) x = rand() / (float)RAND_MAX - 0.5f;
  for (auto& x : hg) x = rand() / (float)RAND_MAX - 0.5f;
  float *ang, *F, *gout, *gang, *ws, *gF;
  CK(hipMalloc(&ang, n * 12));
  CK(hipMalloc(&F, MC * 4));
  CK(hipMalloc(&gout, (size_t)n * MC * 4));
  CK(hipMalloc(&gang, n * 12));
  CK(hipMalloc(&ws, (size_t)gx * MC * 4));
  CK(hipMalloc(&gF, MC * 4));
  CK(hipMemcpy(ang, hang.data(), n * 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(F, hF.data(), MC * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(gout, hg.data(), (size_t)n * MC * 4, hipMemcpyHostToDevice));
  ActionBwdArgs a{};
  a.ang = ang; a.F = F; a.Fstride = 0; a.gout = gout; a.gang = gang; a.gF = gF; a.ws_F = ws;
  a.n = n; a.MC = MC; a.groups = gx; a.C = C; a.Sw = Sw; a.transpose = 0;
  const double bytes = (double)n * (12 + MC * 4 + 12) + 2.0 * MC * 4 + 2.0 * gx * MC * 4;

  for (int nseg : {4, 3, 5, 6}) {
    ActionBwdArgs b = a;
    plan(nseg, b.seg_lo);
    int fp = 0;
    for (int k = 0; k < nseg; ++k) fp = std::max(fp, fseg_rows(b.seg_lo[k], b.seg_lo[k + 1]) * C);
    b.fpitch = (fp + 3) & ~3;
    const size_t base = tile_stage_bytes(Sw, MC, 4) +
                        4 * ((size_t)nseg * 64 * 3 + (size_t)MC + (size_t)nseg * b.fpitch);
    const size_t lds_lib = base + 4 * (size_t)bwd_trig_floats(Sw, L);
    const dim3 g(gx), bl(64 * nseg);
    printf("n=%lld nseg=%d seg_lo:", (long long)n, nseg);
    for (int k = 0; k <= nseg; ++k) printf(" %d", b.seg_lo[k]);
    printf("\n");
    Kern lib = action_bwd_tile_kernel<L, C, kBwdFShared, false, 3>;
    const Out ref = run_once(lib, g, bl, lds_lib, b, n, MC);
    const double tl = timeit(lib, g, bl, lds_lib, b, reps);
    printf("  lib tile kernel        %8.2f us  (%.0f GB/s incl. slabs)\n", tl, bytes / tl / 1e3);
    auto var = [&](Kern k, int v, const char* tag, bool exact) {
      const size_t lds = base + 4 * (size_t)bwdx_trig_floats(Sw, L, nseg, v);
      const Out o = run_once(k, g, bl, lds, b, n, MC);
      const double t = timeit(k, g, bl, lds, b, reps);
      if (exact)
        printf("  %-22s %8.2f us  lds %zu  gang %s slabs %s\n", tag, t, lds,
               ndiff(o.gang, ref.gang) ? "DIFF" : "bitwise", ndiff(o.ws, ref.ws) ? "DIFF" : "bitwise");
      else
        printf("  %-22s %8.2f us  lds %zu  (diagnostic)\n", tag, t, lds);
    };
    var(bwd_x_kernel<L, 0>, 0, "x baseline", true);
    var(bwd_x_kernel<L, kXSlabUnroll>, kXSlabUnroll, "slab unroll", true);
    var(bwd_x_kernel<L, kXWaveLocal>, kXWaveLocal, "wave-local", true);
    var(bwd_x_kernel<L, kXWaveLocal | kXSlabUnroll>, kXWaveLocal | kXSlabUnroll, "wave-local+unroll", true);
    var(bwd_x_kernel<L, kXGlds>, kXGlds, "glds", true);
    var(bwd_x_kernel<L, kXGlds | kXSlabUnroll>, kXGlds | kXSlabUnroll, "glds+unroll", true);
    var(bwd_x_kernel<L, kXGlds | kXWaveLocal | kXSlabUnroll>, kXGlds | kXWaveLocal | kXSlabUnroll,
        "glds wave-local+unroll", true);
    constexpr int GU = kXGlds | kXSlabUnroll;
    var(bwd_x_kernel<L, GU | kXMultReg>, GU | kXMultReg, "glds+unroll+multreg", true);
    var(bwd_x_kernel<L, GU | kXDiagNoSlab>, GU | kXDiagNoSlab, "glds+unroll no slab", false);
    var(bwd_x_kernel<L, GU | kXDiagNoChain>, GU | kXDiagNoChain, "glds+unroll no chain", false);
    var(bwd_x_kernel<L, GU | kXMultReg | kXDiagNoSlab>, GU | kXMultReg | kXDiagNoSlab,
        "glds+unroll+multreg no slab", false);
    var(bwd_x_kernel<L, kXDiagNoG>, kXDiagNoG, "diag no G", false);
    var(bwd_x_kernel<L, kXDiagNoSlab>, kXDiagNoSlab, "diag no slab", false);
    var(bwd_x_kernel<L, kXDiagNoChain>, kXDiagNoChain, "diag no chain", false);
    var(bwd_x_kernel<L, kXDiagNoChain | kXDiagNoSlab>, kXDiagNoChain | kXDiagNoSlab, "diag no chain/slab", false);
    var(bwd_x_kernel<L, kXDiagNoChain | kXDiagNoSlab | kXDiagNoG>, kXDiagNoChain | kXDiagNoSlab | kXDiagNoG,
        "diag skeleton", false);
  }
  return 0;
}

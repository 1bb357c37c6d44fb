// Standalone harness for the fused action kernel (l_max = 10): timing with HIP events
// and, with -DLV_STAMPS, per-wave phase timestamps (s_memrealtime, 100 MHz).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DLV_STAMPS \
//     -I lie-vae_amd/csrc tools/kbench.hip -o kbench
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#include "action_kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

using namespace lv;

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 4096;
  const int nseg = argc > 2 ? atoi(argv[2]) : 2;
  const int reps = argc > 3 ? atoi(argv[3]) : 200;
  constexpr int L = 10;
  const int C = 10, M = (L + 1) * (L + 1);
  std::vector<float> hv(n * 3), hF(M * C);
  srand(1);
  for (auto& x : hv) x = (rand() / (float)RAND_MAX - 0.5f) * 3.f;
  for (auto& x : hF) x = rand() / (float)RAND_MAX - 0.5f;
  float *v, *F, *out;
  CK(hipMalloc(&v, n * 3 * 4));
  CK(hipMalloc(&F, M * C * 4));
  CK(hipMalloc(&out, (size_t)n * M * C * 4));
  CK(hipMemcpy(v, hv.data(), n * 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(F, hF.data(), M * C * 4, hipMemcpyHostToDevice));
  ActionArgs a{};
  a.v = v; a.F = F; a.Fstride = 0; a.out = out; a.n = n; a.MC = M * C; a.C = C; a.Sw = 64 / C;
  // degree segments: balanced by hand for nseg in {1,2,3,4}
  const int segs[5][6] = {{0, 11}, {0, 8, 11}, {0, 7, 9, 11}, {0, 6, 8, 10, 11}, {}};
  for (int k = 0; k <= nseg; ++k) a.seg_lo[k] = segs[nseg - 1][k];
  const int gx = (int)((n + a.Sw * kWavesPerBlock - 1) / (a.Sw * kWavesPerBlock));
  int fmax = 0;
  for (int k = 0; k < nseg; ++k) fmax = std::max(fmax, (fseg_rows(a.seg_lo[k], a.seg_lo[k + 1]) * C + 3) & ~3);
  const size_t lds = 4 * ((size_t)fmax + (LV_STAGED_DEFAULT ? (size_t)kWavesPerBlock * stage_floats(L, C) : 0));
  const int waves = gx * nseg * kWavesPerBlock;
#ifdef LV_STAMPS
  unsigned long long* sb;
  CK(hipMalloc(&sb, (size_t)waves * 8 * 8));
  CK(hipMemset(sb, 0, (size_t)waves * 64));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(lv_stamp_buf), &sb, sizeof(sb)));
#endif
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 20; ++w)
    hipLaunchKernelGGL((action_fwd_kernel<L, true, true, float>), dim3(gx, nseg), dim3(kThreads), lds, 0, a);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((action_fwd_kernel<L, true, true, float>), dim3(gx, nseg), dim3(kThreads), lds, 0, a);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double bytes = (double)n * (12 + M * C * 4) + M * C * 4;
  printf("n=%lld nseg=%d waves=%d lds=%zu  %.2f us/launch  %.0f GB/s\n", (long long)n, nseg, waves, lds, us, bytes / us / 1e3);
#ifdef LV_STAMPS
  // one more launch, then analyse its stamps
  hipLaunchKernelGGL((action_fwd_kernel<L, true, true, float>), dim3(gx, nseg), dim3(kThreads), lds, 0, a);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> hs((size_t)waves * 8);
  CK(hipMemcpy(hs.data(), sb, hs.size() * 8, hipMemcpyDeviceToHost));
  unsigned long long t0 = ~0ull, tend = 0;
  for (int w = 0; w < waves; ++w) if (hs[w * 8 + 3]) { t0 = std::min(t0, hs[w * 8]); tend = std::max(tend, hs[w * 8 + 3]); }
  std::vector<double> st, ph1, ph2, ph3, en;
  for (int w = 0; w < waves; ++w) {
    auto* p = &hs[w * 8];
    if (!p[3]) continue;
    st.push_back((p[0] - t0) * 0.01); ph1.push_back((p[1] - p[0]) * 0.01);
    ph2.push_back((p[2] - p[1]) * 0.01); ph3.push_back((p[3] - p[2]) * 0.01); en.push_back((p[3] - t0) * 0.01);
  }
  auto pr = [](const char* name, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    printf("  %-22s min %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f us\n", name, v[0], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
  };
  printf("stamped waves %zu, span %.2f us\n", st.size(), (tend - t0) * 0.01);
  pr("start", st); pr("loads+prologue", ph1); pr("F LDS+barrier", ph2); pr("chain+stores", ph3); pr("end", en);
#endif
  return 0;
}

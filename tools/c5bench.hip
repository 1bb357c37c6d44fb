// Config-5 split: l = 20, batch 8192, C = 10, bf16 output, fused exp, shared spectrum.
// The library's tile kernel (bitwise reference), then c5_diag_kernel variants.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I lie-vae_amd/csrc \
//     tools/c5bench.hip -o tools/kbench_c5
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "c5_experiments.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)
using namespace lv;
constexpr int L = 20, C = 10;
typedef void (*Kern)(ActionArgs);

static double timeit(Kern k, dim3 g, dim3 b, size_t lds, const ActionArgs& a, int reps) {
  for (int w = 0; w < 10; ++w) hipLaunchKernelGGL(k, g, b, lds, 0, a);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, g, b, lds, 0, a);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / reps;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 8192;
  const int reps = argc > 2 ? atoi(argv[2]) : 200;
  const int M = (L + 1) * (L + 1);
  std::vector<float> hv(n * 3), hF(M * C);
  srand(1);
  for (auto& x : hv) x = (rand() / (float)RAND_MAX - 0.5f) * 3.f;
  for (auto& x : hF) x = rand() / (float)RAND_MAX - 0.5f;
  float *v, *F; void* out;
  CK(hipMalloc(&v, n * 12)); CK(hipMalloc(&F, M * C * 4)); CK(hipMalloc(&out, (size_t)n * M * C * 2 + 64));
  CK(hipMemcpy(v, hv.data(), n * 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(F, hF.data(), M * C * 4, hipMemcpyHostToDevice));
  const int gx = (int)((n + 5) / 6);
  std::vector<unsigned short> ref((size_t)n * M * C), got((size_t)n * M * C);
  for (int nseg : {5, 6, 8}) {
    ActionArgs a{};
    a.v = v; a.F = F; a.out = out; a.n = n; a.MC = M * C; a.C = C; a.Sw = 6; a.write_through = 0;
    // equal-ish segments by cost: split degrees so sum (2 nnz + 12 l) balances (rough)
    const int cuts8[9] = {0, 8, 11, 13, 15, 16, 18, 19, 21};
    const int cuts6[7] = {0, 10, 13, 15, 17, 19, 21};
    const int cuts5[6] = {0, 11, 14, 17, 19, 21};
    for (int k = 0; k <= nseg; ++k) a.seg_lo[k] = nseg == 8 ? cuts8[k] : (nseg == 6 ? cuts6[k] : cuts5[k]);
    const size_t lds = tile_stage_bytes(6, a.MC, 2) + 4 * (size_t)6 * TrigLds<L>::kRow;
    const size_t lds_lib = lds + 4 * (size_t)a.MC;  // the library kernel stages the whole F
    const dim3 g(gx), b(64 * nseg);
    double lib = timeit(action_fwd_tile_kernel<L, C, true, __hip_bfloat16>, g, b, lds_lib, a, reps);
    CK(hipMemcpy(ref.data(), out, ref.size() * 2, hipMemcpyDeviceToHost));
    {
      Kern kn = c5_nomu_kernel<L>;
      CK(hipMemset(out, 0xff, ref.size() * 2));
      hipLaunchKernelGGL(kn, g, b, lds_lib, 0, a);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), out, got.size() * 2, hipMemcpyDeviceToHost));
      printf("nseg=%d library %.2f us | no-mu build %.2f us %s\n", nseg, lib, timeit(kn, g, b, lds_lib, a, reps),
             memcmp(ref.data(), got.data(), ref.size() * 2) ? "MISMATCH" : "bitwise-ok");
    }
    // two-phase tile kernel: degrees [0, L1) then [L1, L], nw waves, one segment per phase each
    for (int L1 : {14, 15, 16})
      for (int nw : {5, 6, 7}) {
        if (L + 1 - L1 < nw) continue;
        ActionArgs t = a;
        auto cost = [](int l) { return (2.0 * l + 1) * (2.0 * l + 1) / 2 + 6.0 * (2 * l + 1) + 20; };
        auto split = [&](int lo, int hi, int k, int* seg) {  // greedy equal-cost split
          double tot = 0; for (int l = lo; l < hi; ++l) tot += cost(l);
          int m = 0; double acc = 0; seg[0] = lo;
          for (int l = lo; l < hi && m < k - 1; ++l) {
            acc += cost(l);
            if (acc >= tot * (m + 1) / k || hi - (l + 1) == k - 1 - m) seg[++m] = l + 1;
          }
          while (m < k - 1) { seg[m + 1] = seg[m] + 1; ++m; }
          seg[k] = hi;
        };
        split(0, L1, nw, t.seg_lo);
        split(L1, L + 1, nw, t.seg_lo + nw + 1);
        const int P = tile2_pitch(M, L1 * L1, C, 2);
        const size_t l2 = (size_t)6 * P + 4 * ((size_t)6 * TrigLds<L>::kRow + (size_t)M * C);
        Kern k2 = action_fwd_tile2_kernel<L, true, __hip_bfloat16>;
        CK(hipMemset(out, 0xff, ref.size() * 2));
        hipLaunchKernelGGL(k2, dim3(gx), dim3(64 * nw), l2, 0, t);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), out, got.size() * 2, hipMemcpyDeviceToHost));
        const bool ok = !memcmp(ref.data(), got.data(), ref.size() * 2);
        printf("   two-phase L1=%d waves=%d lds=%zu: capped %.2f us, uncapped %.2f us %s\n", L1, nw, l2,
               timeit(k2, dim3(gx), dim3(64 * nw), l2, t, reps),
               timeit(c5_tile2_free_kernel<L>, dim3(gx), dim3(64 * nw), l2, t, reps), ok ? "bitwise-ok" : "MISMATCH");
      }
    if (argc > 3) continue;  // A/B rows only
    CK(hipMemset(out, 0xff, ref.size() * 2));
    hipLaunchKernelGGL(c5_persist_kernel<L>, dim3(std::min(512, gx)), b, lds, 0, a);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), out, got.size() * 2, hipMemcpyDeviceToHost));
    printf("persistent vs library: %s\n", memcmp(ref.data(), got.data(), ref.size() * 2) ? "MISMATCH" : "bitwise-ok");
    double d0 = timeit(c5_diag_kernel<L, 0>, g, b, lds_lib, a, reps);
    double d1 = timeit(c5_diag_kernel<L, 1>, g, b, lds_lib, a, reps);
    double d2 = timeit(c5_diag_kernel<L, 2>, g, b, lds_lib, a, reps);
    double d3 = timeit(c5_diag_kernel<L, 3>, g, b, lds_lib, a, reps);
    double d7 = timeit(c5_diag_kernel<L, 7>, g, b, lds_lib, a, reps);
    double d23 = timeit(c5_diag_kernel<L, 16 | 7>, g, b, lds_lib, a, reps);
    double d39 = timeit(c5_diag_kernel<L, 32 | 7>, g, b, lds_lib, a, reps);
    double d17 = timeit(c5_diag_kernel<L, 16 | 1>, g, b, lds_lib, a, reps);
    double d5 = timeit(c5_diag_kernel<L, 5>, g, b, lds_lib, a, reps);
    printf("nseg=%d lib %.2f | diag0 %.2f  no-flush %.2f  no-chain %.2f  no-chain-no-flush %.2f | "
           "skeleton(F LDS) %.2f  skeleton(no F) %.2f  skeleton(F global) %.2f | chain, no F, no flush %.2f  chain no-tile no-flush %.2f us\n",
           nseg, lib, d0, d1, d2, d3, d7, d23, d39, d17, d5);
    for (size_t ll : {(size_t)0, (size_t)16384, lds}) {
      const double f0 = timeit(c5_floor_kernel<0>, g, b, ll, a, reps);
      const double f1 = timeit(c5_floor_kernel<1>, g, b, std::max(ll, (size_t)4096), a, reps);
      printf("   nseg=%d floor lds=%zu: empty %.2f  prologue+barrier %.2f us\n", nseg, ll, f0, f1);
    }
  }
  return 0;
}

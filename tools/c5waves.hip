// Config 5 (l = 20, batch 8192, C = 10, bf16 out, fused): the library's tile body at more
// waves per block than the product's 8 (launch bounds 1024) and with a VGPR cap
// (amdgpu_waves_per_eu = 5 / 6), against the library kernel (bitwise reference).
// Segments: equal-cost split of degrees 0..20 under the library's cost model.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I lie-vae_amd/csrc \
//     tools/c5waves.hip -o tools/kbench_c5waves
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "action_fwd.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)
using namespace lv;
constexpr int L = 20, C = 10;
typedef void (*Kern)(ActionArgs);

template <int WPE>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(WPE))) void tile_wpe(ActionArgs a) {
  fwd_tile_body<L, C, true, __hip_bfloat16>(a, blockIdx.x);
}
__global__ __launch_bounds__(1024) void tile_free(ActionArgs a) {
  fwd_tile_body<L, C, true, __hip_bfloat16>(a, blockIdx.x);
}

template <int... Ls>
constexpr std::array<int, sizeof...(Ls)> nnz_tab(std::integer_sequence<int, Ls...>) { return {j_nnz<Ls>()...}; }
constexpr auto kNnz = nnz_tab(std::make_integer_sequence<int, L + 1>{});

// min-max contiguous split of degrees 0..L into k segments (cost 2 nnz + 9(2l+1) + P)
static void plan(int k, int* seg) {
  const int D = L + 1;
  double pre[D + 1]; pre[0] = 0;
  for (int l = 0; l < D; ++l) pre[l + 1] = pre[l] + 2.0 * kNnz[l] + 9.0 * (2 * l + 1);
  const double P = 60.0, INF = 1e30;
  static double dp[17][22]; static int arg[17][22];
  for (int a = 0; a <= k; ++a) for (int i = 0; i <= D; ++i) dp[a][i] = INF;
  dp[0][0] = 0;
  for (int a = 1; a <= k; ++a)
    for (int i = 1; i <= D; ++i)
      for (int p = a - 1; p < i; ++p) {
        const double v = std::max(dp[a - 1][p], pre[i] - pre[p] + P);
        if (v < dp[a][i]) { dp[a][i] = v; arg[a][i] = p; }
      }
  int i = D;
  for (int a = k; a >= 1; --a) { seg[a] = i; i = arg[a][i]; }
  seg[0] = 0;
}

static double timeit(Kern k, dim3 g, dim3 b, size_t lds, const ActionArgs& a, int reps) {
  for (int w = 0; w < 10; ++w) hipLaunchKernelGGL(k, g, b, lds, 0, a);
  CK(hipGetLastError());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, g, b, lds, 0, a);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  CK(hipGetLastError());
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / reps;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 8192;
  const int reps = argc > 2 ? atoi(argv[2]) : 300;
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
  const size_t lds = tile_stage_bytes(6, (int64_t)M * C, 2) + 4 * ((size_t)6 * TrigLds<L>::kRow + (size_t)M * C);
  auto args = [&](int nseg) {
    ActionArgs a{};
    a.v = v; a.F = F; a.out = out; a.n = n; a.MC = M * C; a.C = C; a.Sw = 6; a.write_through = 0;
    plan(nseg, a.seg_lo);
    return a;
  };
  {
    ActionArgs a = args(8);
    hipLaunchKernelGGL((action_fwd_tile_kernel<L, C, true, __hip_bfloat16>), dim3(gx), dim3(512), lds, 0, a);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), out, ref.size() * 2, hipMemcpyDeviceToHost));
    printf("library tile kernel nseg=8 (lds %zu): %.2f us\n", lds,
           timeit(action_fwd_tile_kernel<L, C, true, __hip_bfloat16>, dim3(gx), dim3(512), lds, a, reps));
  }
  struct V { const char* name; Kern k; };
  const V vars[] = {{"free", tile_free}, {"wpe5", tile_wpe<5>}, {"wpe6", tile_wpe<6>}};
  for (int nseg : {8, 10, 12, 14, 16}) {
    ActionArgs a = args(nseg);
    printf("nseg=%2d seg_lo:", nseg);
    for (int k = 0; k <= nseg; ++k) printf(" %d", a.seg_lo[k]);
    printf("\n");
    for (const V& var : vars) {
      CK(hipMemset(out, 0xff, ref.size() * 2));
      hipLaunchKernelGGL(var.k, dim3(gx), dim3(64 * nseg), lds, 0, a);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), out, got.size() * 2, hipMemcpyDeviceToHost));
      const bool ok = !memcmp(ref.data(), got.data(), ref.size() * 2);
      printf("   %-5s %7.2f us %s\n", var.name, timeit(var.k, dim3(gx), dim3(64 * nseg), lds, a, reps),
             ok ? "bitwise-ok" : "MISMATCH");
    }
  }
  return 0;
}

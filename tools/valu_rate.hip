// VALU issue-rate probe for gfx950: v_fma_f32 vs v_pk_fma_f32 (two fp32 FMAs per lane)
// vs v_pk_mul_f32, 8 independent chains per lane, 8 waves per SIMD.  Decides whether
// packing the group-action chain over column pairs halves its vector-issue time.
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) k_fma(float* out, int iters, float a, float b) {
  float x[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 1e-3f + k;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[k]) : "v"(a), "v"(b));
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_pkfma(float* out, int iters, float a, float b) {
  f2 x[8];
  f2 av = {a, a}, bv = {b, b};
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = f2{threadIdx.x * 1e-3f + k, (float)k};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(x[k]) : "v"(av), "v"(bv));
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k].x + x[k].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// broadcast scalar coefficient: both halves read the low half of av (op_sel_hi:[0,1,1])
__global__ void __launch_bounds__(256) k_pkfma_bc(float* out, int iters, float a, float b) {
  f2 x[8];
  f2 av = {a, 0.f}, bv = {b, b};
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = f2{threadIdx.x * 1e-3f + k, (float)k};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(x[k]) : "v"(av), "v"(bv));
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k].x + x[k].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// scalar-register coefficient (SGPR) on the packed FMA
__global__ void __launch_bounds__(256) k_pkfma_s(float* out, int iters, float a, float b) {
  f2 x[8];
  f2 bv = {b, b};
  f2 as = {a, a};
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = f2{threadIdx.x * 1e-3f + k, (float)k};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(x[k]) : "s"(as), "v"(bv));
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += x[k].x + x[k].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  const int blocks = 256 * 4 * 8 / 4;  // 8 waves per SIMD
  const int iters = 4096;
  float* out;
  hipMalloc(&out, blocks * 256 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, void (*k)(float*, int, float, float), double flop_per_inst) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f, 1e-7f);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f, 1e-7f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double inst = 5.0 * blocks * 4.0 * iters * 8;  // wave instructions
    const double s = ms / 1e3;
    printf("%-12s %8.3f ms  %7.2f TFLOP/s  %6.2f wave-inst/ns  cycles/inst/SIMD @2.4GHz %.2f\n", name, ms,
           inst * 64 * flop_per_inst / s / 1e12, inst / s / 1e9, 1024.0 * 2.4e9 * s / inst);
  };
  run("v_fma_f32", k_fma, 2);
  run("v_pk_fma", k_pkfma, 4);
  run("v_pk_fma_bc", k_pkfma_bc, 4);
  run("v_pk_fma_s", k_pkfma_s, 4);
  return 0;
}

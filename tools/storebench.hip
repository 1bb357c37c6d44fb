// Store-pattern calibration: write n*MC floats (MC = 1210) in several lane patterns.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

// (a) contiguous dword per lane, grid-stride
__global__ void st_dword(float* o, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = (float)i;
}
// (b) contiguous dwordx4 per lane
__global__ void st_dwordx4(float4* o, int64_t total4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = make_float4(i, i, i, i);
}
// (c) the action kernel's pattern: lane = (sample j < 6, column c < 10); per row r a
//     store of out[s][r][c] (6 pieces of 40 B per wave-instruction), rows 0..120.
__global__ void st_pieces(float* o, int64_t n, int MC, int C) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int Sw = 64 / C, j = lane / C, c = lane - j * C;
  const int64_t s0 = ((int64_t)blockIdx.x * 4 + wave) * Sw;
  const int64_t s = s0 + j;
  if (j >= Sw || s >= n) return;
  float* d = o + s * MC + c;
  for (int r = 0; r < MC / C; ++r) { d[0] = (float)r; d += C; }
}
// (d) row pairs per instruction: lane (j, c) writes float2 of rows (r, r+1): even c ->
//     (row r, cols c, c+1), odd c -> (row r+1, cols c-1, c): 80-B pieces per sample.
__global__ void st_pieces80(float* o, int64_t n, int MC, int C) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int Sw = 64 / C, j = lane / C, c = lane - j * C;
  const int64_t s0 = ((int64_t)blockIdx.x * 4 + wave) * Sw;
  const int64_t s = s0 + j;
  if (j >= Sw || s >= n) return;
  const int odd = c & 1;
  float* d = o + s * MC + (odd ? C + c - 1 : c);
  const int rows = MC / C;
  for (int r = 0; r + 1 < rows; r += 2) { *reinterpret_cast<float2*>(d) = make_float2(r, r); d += 2 * C; }
}
// (e) the tile kernel's flush: block b writes its contiguous run of S samples (S*MC
//     floats) with 16-B buffer stores, cache policy POL (0 default, 1 nt, 16 sc1)
typedef float f4v __attribute__((ext_vector_type(4)));
template <int POL>
__global__ __launch_bounds__(1024) void st_chunk(float* o, int64_t n, int MC, int S) {
  const int64_t s0 = (int64_t)blockIdx.x * S;
  const int Sv = (int)min((int64_t)S, n - s0);
  const int nbytes = Sv * MC * 4;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(o + s0 * MC, 0, nbytes, 0x00020000);
  const float v = (float)blockIdx.x;
  for (int k = threadIdx.x; k < nbytes / 16; k += blockDim.x)
    __builtin_amdgcn_raw_buffer_store_b128(f4v{v, v, v, v}, r, 16 * k, 0, POL);
}
int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 65536;
  const int MC = 1210, C = 10;
  const int64_t total = n * MC;
  float* o;
  CK(hipMalloc(&o, total * 4 + 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 5; ++w) launch();
    CK(hipDeviceSynchronize());
    const int reps = 50;
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    printf("%-28s n=%lld  %8.2f us  %6.0f GB/s\n", name, (long long)n, us, total * 4.0 / us / 1e3);
  };
  for (int g : {1024, 2048, 4096, 16384}) {
    char nm[64]; snprintf(nm, 64, "dword grid=%d", g);
    run(nm, [&] { hipLaunchKernelGGL(st_dword, dim3(g), dim3(256), 0, 0, o, total); });
    snprintf(nm, 64, "dwordx4 grid=%d", g);
    run(nm, [&] { hipLaunchKernelGGL(st_dwordx4, dim3(g), dim3(256), 0, 0, (float4*)o, total / 4); });
  }
  const int blocks = (int)((n + 23) / 24);
  run("pieces40B", [&] { hipLaunchKernelGGL(st_pieces, dim3(blocks), dim3(256), 0, 0, o, n, MC, C); });
  run("pieces80B float2", [&] { hipLaunchKernelGGL(st_pieces80, dim3(blocks), dim3(256), 0, 0, o, n, MC, C); });
  for (int S : {6, 12, 24, 48})
    for (int nw : {4, 8, 16}) {
      const int g = (int)((n + S - 1) / S);
      char nm[64];
      snprintf(nm, 64, "chunk S=%d w=%d def", S, nw);
      run(nm, [&] { hipLaunchKernelGGL(st_chunk<0>, dim3(g), dim3(64 * nw), 0, 0, o, n, MC, S); });
      snprintf(nm, 64, "chunk S=%d w=%d nt", S, nw);
      run(nm, [&] { hipLaunchKernelGGL(st_chunk<1>, dim3(g), dim3(64 * nw), 0, 0, o, n, MC, S); });
      snprintf(nm, 64, "chunk S=%d w=%d sc1", S, nw);
      run(nm, [&] { hipLaunchKernelGGL(st_chunk<16>, dim3(g), dim3(64 * nw), 0, 0, o, n, MC, S); });
    }
  return 0;
}

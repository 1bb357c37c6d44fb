// Common plumbing for the lie-vae MI355X kernels: error state, dtype tags,
// compile-time loops.  gfx950 only; no CUDA/HIP dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdint>
#include <cstdio>
#include <utility>

#include "../../include/lievae.h"

namespace lv {

// Thread-local last-error text (lv_last_error()).
void set_error(const char* fmt, ...);
void clear_error();

#define LV_CHECK_ARG(cond, ...)                      \
  do {                                               \
    if (!(cond)) {                                   \
      ::lv::set_error(__VA_ARGS__);                  \
      return LV_ERR_ARG;                             \
    }                                                \
  } while (0)

#define LV_RETURN_LAUNCH(kname)                                               \
  do {                                                                        \
    hipError_t e_ = hipGetLastError();                                        \
    if (e_ != hipSuccess) {                                                   \
      ::lv::set_error("%s: launch failed: %s", kname, hipGetErrorString(e_)); \
      return LV_ERR_HIP;                                                      \
    }                                                                         \
    return LV_OK;                                                             \
  } while (0)

// Like LV_RETURN_LAUNCH, but falls through on success (more work follows).
#define LV_CHECK_LAUNCH(kname)                                                \
  do {                                                                        \
    hipError_t e_ = hipGetLastError();                                        \
    if (e_ != hipSuccess) {                                                   \
      ::lv::set_error("%s: launch failed: %s", kname, hipGetErrorString(e_)); \
      return LV_ERR_HIP;                                                      \
    }                                                                         \
  } while (0)

#define LV_CHECK_HIP(call)                                                    \
  do {                                                                        \
    hipError_t e_ = (call);                                                   \
    if (e_ != hipSuccess) {                                                   \
      ::lv::set_error("%s: %s", #call, hipGetErrorString(e_));                \
      return LV_ERR_HIP;                                                      \
    }                                                                         \
  } while (0)

// ---------------------------------------------------------------- static_for
template <class F, int... Is>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// ---------------------------------------------------------------- out types
__device__ __forceinline__ void store_out(float* p, float v) { *p = v; }
__device__ __forceinline__ void store_out(__hip_bfloat16* p, float v) { *p = __float2bfloat16(v); }
__device__ __forceinline__ float load_in(const float* p) { return *p; }
__device__ __forceinline__ float load_in(const __hip_bfloat16* p) { return __bfloat162float(*p); }

__device__ __forceinline__ void store_out2(float* p, float a, float b) {
  *reinterpret_cast<float2*>(p) = make_float2(a, b);
}
__device__ __forceinline__ void store_out2(__hip_bfloat16* p, float a, float b) {
  __hip_bfloat162 h;
  h.x = __float2bfloat16(a);
  h.y = __float2bfloat16(b);
  *reinterpret_cast<__hip_bfloat162*>(p) = h;
}

// Exchange a value with the adjacent lane (0<->1, 2<->3, ...): DPP quad_perm [1,0,3,2].
__device__ __forceinline__ float dpp_swap_adjacent(float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// LDS pointer for __builtin_amdgcn_global_load_lds (global -> LDS DMA; the destination is
// the wave-uniform base + lane * size).
typedef __attribute__((address_space(3))) void* lds_vp;
__device__ __forceinline__ lds_vp as_lds(const void* p) { return (lds_vp)(p); }

}  // namespace lv

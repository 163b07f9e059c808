// Internal helpers shared by the acquisition and tracking translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "gsdr.h"

namespace gsdr
{

void set_error(const char* fmt, ...);

// Map a HIP status to GSDR_E_DEVICE with a message naming the call site.
#define GSDR_HIP(call)                                                                              \
    do                                                                                              \
        {                                                                                           \
            hipError_t e_ = (call);                                                                 \
            if (e_ != hipSuccess)                                                                   \
                {                                                                                   \
                    ::gsdr::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
                    return GSDR_E_DEVICE;                                                           \
                }                                                                                   \
        }                                                                                           \
    while (0)

#define GSDR_REQUIRE(cond, code, ...)                \
    do                                               \
        {                                            \
            if (!(cond))                             \
                {                                    \
                    ::gsdr::set_error(__VA_ARGS__);  \
                    return (code);                   \
                }                                    \
        }                                            \
    while (0)

// RAII device switch: the ABI is called from arbitrary host threads.
struct DeviceGuard
{
    int prev{-1};
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Single-rounding float operations that the backend may not fuse into an FMA
// (the reference's code index floor(step*n + (shift - rem)) flips
// at chip boundaries, so each product and sum must round exactly as on x86).
// HIP's __fmul_rn/__fadd_rn are plain operators whose contraction follows the
// caller's context; these carry an explicit contract(off).
__device__ __forceinline__ float mul_rn(float a, float b)
{
#pragma clang fp contract(off)
    return a * b;
}
__device__ __forceinline__ float add_rn(float a, float b)
{
#pragma clang fp contract(off)
    return a + b;
}
__device__ __forceinline__ float sub_rn(float a, float b)
{
#pragma clang fp contract(off)
    return a - b;
}

// Replace *stream (if any) with a new non-blocking stream on the current device,
// restricted to the CUs in mask[0..n_words) (all CUs when n_words == 0).
int replace_stream(hipStream_t* stream, const uint32_t* mask, int n_words);

// Inverse regularised lower incomplete gamma for integer shape a:
// returns x with P(a, x) = p.  (Boost gamma_p_inv, used by calculate_threshold.)
double gamma_p_inv_int(int a, double p);

// Wave64 maximum of a float by DPP lane moves (no LDS, no index arithmetic):
// quad swaps, half-row and row mirrors give each 16-lane row its maximum, the
// row broadcasts carry rows 0..2 into lane 63.  fmaxf keeps the float rule
// (a NaN operand yields the other value).  The result is read from lane 63 and is
// wave-uniform.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_max_step(float x)
{
    const int o = __builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), CTRL, ROW_MASK, 0xf, false);
    return __builtin_fmaxf(x, __int_as_float(o));
}

__device__ __forceinline__ float wave_max(float v)
{
    v = dpp_max_step<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_max_step<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_max_step<0x141, 0xf>(v);  // row_half_mirror
    v = dpp_max_step<0x140, 0xf>(v);  // row_mirror
    v = dpp_max_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    v = dpp_max_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Wave64 sum by the same DPP lane moves (no LDS round trips, unlike __shfl_xor's
// ds_bpermute): the disabled rows of the two row broadcasts read 0, so they keep
// their value.  The total is valid in lane 63 only (rows 0..2 hold partial sums).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_add_step(float x)
{
    const int o = __builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROW_MASK, 0xf, false);
    return x + __int_as_float(o);
}

__device__ __forceinline__ float wave_sum_lane63(float v)
{
    v = dpp_add_step<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_add_step<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_add_step<0x141, 0xf>(v);  // row_half_mirror
    v = dpp_add_step<0x140, 0xf>(v);  // row_mirror
    v = dpp_add_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    v = dpp_add_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
    return v;
}

}  // namespace gsdr

// pointer types of __builtin_amdgcn_global_load_lds (global source, LDS destination)
typedef __attribute__((address_space(1))) void gsdr_gvoid;
typedef __attribute__((address_space(3))) void gsdr_lvoid;


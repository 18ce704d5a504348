// common.hpp -- shared device/host helpers for the gfx950 hot-path kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <string>

#include "../../include/dpvo_hot.h"

namespace dpvo {

// ---------------------------------------------------------------------------
// error reporting through the C ABI
// ---------------------------------------------------------------------------
void set_error(const std::string& msg);

#define DPVO_CHECK_ARG(cond, msg)                                   \
    do {                                                            \
        if (!(cond)) {                                              \
            ::dpvo::set_error(std::string(__func__) + ": " + (msg)); \
            return -1;                                              \
        }                                                           \
    } while (0)

#define DPVO_CHECK_LAUNCH()                                                              \
    do {                                                                                 \
        hipError_t _e = hipGetLastError();                                               \
        if (_e != hipSuccess) {                                                          \
            ::dpvo::set_error(std::string(__func__) + ": launch failed: " + hipGetErrorString(_e)); \
            return -2;                                                                   \
        }                                                                                \
    } while (0)

#define DPVO_CHECK_HIP(expr)                                                               \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess) {                                                            \
            ::dpvo::set_error(std::string(__func__) + ": " #expr ": " + hipGetErrorString(_e)); \
            return -2;                                                                     \
        }                                                                                  \
    } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline unsigned grid_for(int64_t n, int block, int64_t cap = 1 << 20)
{
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// ---------------------------------------------------------------------------
// vector types
// ---------------------------------------------------------------------------
typedef _Float16 half_t;
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));

// CUDA/AMD cvt.rzi.s32.f32 semantics for (int)floorf(v): NaN -> 0, saturate.
__device__ __forceinline__ int floor_to_int_sat(float v)
{
    float f = floorf(v);
    if (!(f == f)) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (int)0x80000000u;
    return (int)f;
}
__device__ __forceinline__ int wrap_add(int a, int b) { return (int)((unsigned)a + (unsigned)b); }

// ---------------------------------------------------------------------------
// wave64 reductions (DPP row rotations + readlanes)
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_rot(float v)
{
    // (no "old" operand: every lane of a row rotation is written; update_dpp
    // with old = 0 cost a v_mov of that 0 per rotation)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
// all-reduce over a DPP row (16 lanes): every lane of the row gets the row's sum
__device__ __forceinline__ float row16_sum(float s)
{
    s += dpp_rot<0x128>(s);
    s += dpp_rot<0x124>(s);
    s += dpp_rot<0x122>(s);
    s += dpp_rot<0x121>(s);
    return s;
}
// sum over all 64 lanes (wave-uniform result)
__device__ __forceinline__ float wave64_sum(float s)
{
    s = row16_sum(s);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 0)) +
           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 16)) +
           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 32)) +
           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 48));
}

}  // namespace dpvo

// corrmfma.hpp -- the matrix-core altcorr's parameters and its bilinear
// step (corrmfma.hip: one wave per edge, windows read through the
// vector-memory path).
#pragma once

#include "common.hpp"

namespace dpvo {

namespace cm {
constexpr int R = 3, D = 8, DO = 7, NP = 9, C = 128, BOXMAX = 12, WAVES = 4;
constexpr int RS = 148;           // LDS row per patch pixel: the box's <= 144 pixels (+ pad: rows 4 apart, 16 banks apart)
constexpr int RL = NP * RS;       // per level
constexpr unsigned OOB = 0x80000000u;   // a buffer offset past every descriptor's range: the load returns 0
}  // namespace cm

struct CorrMfmaParams {
    const half_t* gt;   // [N1][9][128] transposed patch features
    int N1;
    const float* coords;
    int64_t c_s[5];
    const int64_t* ii;
    const int64_t* jj;
    int E;
    const half_t* fmap[2];
    int64_t f_s1[2];
    int N2[2], H2[2], W2[2];
    int64_t rowb[2];          // row stride in bytes
    int pixb[2];              // pixel stride in bytes
    int rowext[2];            // bytes from a row's first pixel to the end of its last
    int frameext[2];          // bytes from a frame's first pixel to the end of its last
    float scale[2];
    half_t* out;
    int64_t o_e;
    const int* order;   // optional edge visiting order (edges grouped by target frame), NULL = 0..E-1
};

// The fp32 bilinear 8x8 -> 7x7 step of one output (correlation_kernel.cu:221-232's
// four terms) as one explicit chain, so it rounds the same way whatever the
// compiler would contract:
// w = {(1-dx)(1-dy), dx(1-dy), (1-dx)dy, dx dy}, r = the 2 x 2 products
__device__ __forceinline__ float cm_bilinear(float w0, float w1, float w2, float w3, float r00, float r01, float r10,
                                             float r11)
{
    float v = __builtin_fmaf(w3, r11, __builtin_fmaf(w2, r10, __builtin_fmaf(w1, r01, w0 * r00)));
    // an fp32 value, rounded to fp16 by the caller's conversion: without this
    // the compiler may fuse the last fma into the conversion (v_fma_mix*_f16:
    // one rounding instead of two)
    asm volatile("" : "+v"(v));
    return v;
}

// dpvo_corr_pyramid_mfma's argument checks and parameter block (0, or -1 with the error set)
int corr_mfma_setup(CorrMfmaParams& p, const void* table, int64_t num_patches, const void* const* fmaps,
                    const int64_t* fmap_sizes, const int64_t* fmap_strides, const float* level_scale,
                    const float* coords, const int64_t* coords_size, const int64_t* coords_stride, const int64_t* ii,
                    const int64_t* jj, void* corr, int64_t edge_stride, const int* order);
// corr_mfma_kernel over the order's slots
int corr_mfma_launch(const CorrMfmaParams& p, hipStream_t s);

}  // namespace dpvo

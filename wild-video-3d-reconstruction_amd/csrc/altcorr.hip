// altcorr.hip -- patch <-> frame local correlation for gfx950.
//
// Replaces the reference's cuda_corr extension
// (dpvo/altcorr/correlation.cpp:57-62, correlation_kernel.cu).
//
// Arithmetic contract: for fp16 inputs the result is bit-identical to the
// reference, whose kernel accumulates `s += f1*f2` in c10::Half (each product
// and each sum rounded to binary16, channel order 0..C-1;
// correlation_kernel.cu:121-131) and whose ATen epilogue rounds every
// elementwise op to binary16 (:221-232).  Native v_pk_mul_f16/v_pk_add_f16
// round exactly like "fp32 op, then round to half" for binary16 operands, so
// the chain is emulated with packed fp16 VALU ops.  This file is compiled with
// -ffp-contract=off: a fused multiply-add would change the bits.
//
// Fast path (fp16, radius 3, 3x3 patches, channel-last fmap, C % 8 == 0):
//   one workgroup per (batch, edge); 128 lanes per pyramid level.  The nine
//   8x8 windows of a patch overlap: when their floor() offsets spread by at
//   most 2 pixels they lie in one 10x10 box.  Lane u owns box pixel u, streams
//   its C channels from HBM exactly once (16-byte loads), and runs the
//   reference's fp16 chain for all nine patch pixels at once, two chains per
//   packed op: (f1[p][c], f1[p'][c]) x (W[u][c], W[u][c]).  The per-pixel raw
//   8x8 tiles are then gathered from LDS, bilinearly combined with the
//   reference's exact rounding sequence and written in the caller's layout.
//   Boxes wider than 10x10 fall back, inside the same kernel, to one 8x8
//   window per patch pixel.
#include "common.hpp"

namespace dpvo {

namespace corr {
constexpr int R = 3, D = 8, DO = 7, PS = 3, NP = 9, BOX = 10, NPAIR = 5;
}

struct CorrFastParams {
    const half_t* gmap;
    int64_t g_s[5];
    int N1, C;
    const float* coords;
    int64_t c_s[5];
    const int64_t* ii;
    const int64_t* jj;
    int B, E;
    const half_t* fmap[2];
    int64_t f_s0[2], f_s1[2], f_s3[2], f_s4[2];
    int N2[2], H2[2], W2[2];
    float scale[2];
    half_t* out;
    int64_t o_b, o_e, o_l, o_x, o_y, o_p;
};

__device__ __forceinline__ half2_t as_h2(uint32_t v) { return __builtin_bit_cast(half2_t, v); }

// exact binary16 ops (contraction is off for this file)
__device__ __forceinline__ half_t hmul(half_t a, half_t b) { return a * b; }
__device__ __forceinline__ half_t hadd(half_t a, half_t b) { return a + b; }

template <int NLEV>
__global__ __launch_bounds__(128 * NLEV) void corr_fast_kernel(CorrFastParams p)
{
    using namespace corr;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // LDS carve: f1 pairs [C][8] dwords (5 used) | raw tiles [NLEV][NP][BOX*BOX] half
    uint32_t* f1pk = reinterpret_cast<uint32_t*>(smem);
    half_t* raw_all = reinterpret_cast<half_t*>(smem + (size_t)p.C * 8 * 4);

    const int be = blockIdx.x;
    const int b = be / p.E, e = be - b * p.E;
    const int tid = threadIdx.x;
    const int lev = tid >> 7;
    const int t = tid & 127;
    const int C = p.C;

    const int ix = (int)p.ii[e];
    const int jx = (int)p.jj[e];
    const bool ix_ok = ix >= 0 && ix < p.N1;

    // ---- patch features -> packed pairs (p0,p1) (p2,p3) (p4,p5) (p6,p7) (p8,0)
    {
        const half_t* g = p.gmap + b * p.g_s[0] + (int64_t)ix * p.g_s[1];
        for (int i = tid; i < C * NPAIR; i += 128 * NLEV) {
            const int c = i / NPAIR, q = i - c * NPAIR;
            const int pa = 2 * q, pb = 2 * q + 1;
            half_t lo = (half_t)0, hi = (half_t)0;
            if (ix_ok) {
                lo = g[c * p.g_s[2] + (pa / PS) * p.g_s[3] + (pa % PS) * p.g_s[4]];
                if (pb < NP) hi = g[c * p.g_s[2] + (pb / PS) * p.g_s[3] + (pb % PS) * p.g_s[4]];
            }
            half2_t v = {lo, hi};
            f1pk[c * 8 + q] = __builtin_bit_cast(uint32_t, v);
        }
    }

    // ---- this level's coordinates (uniform per wave)
    const float sc = p.scale[lev];
    const int N2 = p.N2[lev], H2 = p.H2[lev], W2 = p.W2[lev];
    const bool idx_ok = ix_ok && jx >= 0 && jx < N2;
    float xs[NP], ys[NP];
    int fy[NP], fx[NP];
    int ymin = 0x7fffffff, ymax = (int)0x80000000u, xmin = 0x7fffffff, xmax = (int)0x80000000u;
    const float* cb = p.coords + b * p.c_s[0] + (int64_t)e * p.c_s[1];
#pragma unroll
    for (int q = 0; q < NP; q++) {
        const int64_t o = (q / PS) * p.c_s[3] + (q % PS) * p.c_s[4];
        xs[q] = cb[o] / sc;
        ys[q] = cb[p.c_s[2] + o] / sc;
        fy[q] = floor_to_int_sat(ys[q]);
        fx[q] = floor_to_int_sat(xs[q]);
        ymin = min(ymin, fy[q]); ymax = max(ymax, fy[q]);
        xmin = min(xmin, fx[q]); xmax = max(xmax, fx[q]);
    }
    const bool fast = ((int64_t)ymax - ymin) <= 2 && ((int64_t)xmax - xmin) <= 2;

    const half_t* fm = p.fmap[lev] + b * p.f_s0[lev] + (int64_t)jx * p.f_s1[lev];
    const int64_t fs3 = p.f_s3[lev], fs4 = p.f_s4[lev];
    half_t* raw = raw_all + lev * NP * BOX * BOX;

    __syncthreads();  // f1pk complete

    // one pass computes every chain of box pixel u for all nine patch pixels
    auto run_box = [&](int oy, int ox, int bw, int bh, int only_p) {
        const int uy = t / bw, ux = t - uy * bw;
        const bool act = t < bw * bh;
        const int gy = wrap_add(oy, uy), gx = wrap_add(ox, ux);
        const bool inb = act && idx_ok && gy >= 0 && gy < H2 && gx >= 0 && gx < W2;
        half2_t acc[NPAIR];
#pragma unroll
        for (int q = 0; q < NPAIR; q++) acc[q] = (half2_t){(half_t)0, (half_t)0};
        const uint4* wp = reinterpret_cast<const uint4*>(fm + (int64_t)(inb ? gy : 0) * fs3 + (int64_t)(inb ? gx : 0) * fs4);
        const int C8 = C >> 3;
        uint4 w = inb ? wp[0] : make_uint4(0, 0, 0, 0);
        for (int c8 = 0; c8 < C8; c8++) {
            const uint4 cur = w;
            if (c8 + 1 < C8) w = inb ? wp[c8 + 1] : make_uint4(0, 0, 0, 0);
            const uint32_t wd[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const half2_t wv = as_h2(wd[k]);
#pragma unroll
                for (int hsel = 0; hsel < 2; hsel++) {
                    const int c = c8 * 8 + 2 * k + hsel;
                    const half_t ws = hsel ? wv.y : wv.x;
                    const half2_t wb = {ws, ws};
                    const uint4 f03 = *reinterpret_cast<const uint4*>(f1pk + c * 8);
                    const uint32_t f4 = f1pk[c * 8 + 4];
                    acc[0] = acc[0] + wb * as_h2(f03.x);
                    acc[1] = acc[1] + wb * as_h2(f03.y);
                    acc[2] = acc[2] + wb * as_h2(f03.z);
                    acc[3] = acc[3] + wb * as_h2(f03.w);
                    acc[4] = acc[4] + wb * as_h2(f4);
                }
            }
        }
        if (act) {
            // out-of-image positions are exactly +0 in the reference (never accumulated)
            const half_t z = (half_t)0;
            const half_t s[NP] = {acc[0].x, acc[0].y, acc[1].x, acc[1].y, acc[2].x,
                                  acc[2].y, acc[3].x, acc[3].y, acc[4].x};
            if (only_p < 0) {
#pragma unroll
                for (int q = 0; q < NP; q++) raw[q * BOX * BOX + t] = inb ? s[q] : z;
            } else {
                half_t v = z;
#pragma unroll
                for (int q = 0; q < NP; q++) if (q == only_p) v = s[q];
                raw[only_p * BOX * BOX + t] = inb ? v : z;
            }
        }
    };

    if (fast) {
        run_box(wrap_add(ymin, -R), wrap_add(xmin, -R), BOX, BOX, -1);
    } else {
        // rare: the nine windows do not share a 10x10 box
        for (int q = 0; q < NP; q++) run_box(wrap_add(fy[q], -R), wrap_add(fx[q], -R), D, D, q);
    }
    __syncthreads();

    // ---- bilinear epilogue, exact rounding sequence of correlation_kernel.cu:221-232
    half_t* ob = p.out + b * p.o_b + (int64_t)e * p.o_e + lev * p.o_l;
    for (int o = t; o < NP * DO * DO; o += 128) {
        const int q = o / (DO * DO), r = o - q * (DO * DO);
        const int a = r / DO, bx = r - a * DO;  // a: y offset, bx: x offset
        // raw tile of patch pixel q: inside the shared 10x10 box at its floor
        // offset (fast), or its own 8x8 window (fallback)
        const int bw = fast ? BOX : D;
        int oy = 0, ox = 0;
        if (fast) {
#pragma unroll
            for (int k = 0; k < NP; k++)
                if (k == q) { oy = fy[k] - ymin; ox = fx[k] - xmin; }
        }
        const int base = q * BOX * BOX + (oy + a) * bw + (ox + bx);
        const half_t c00 = raw[base], c01 = raw[base + 1], c10 = raw[base + bw], c11 = raw[base + bw + 1];
        float xq = 0.f, yq = 0.f;
#pragma unroll
        for (int k = 0; k < NP; k++)
            if (k == q) { xq = xs[k]; yq = ys[k]; }
        const half_t dx = (half_t)(xq - floorf(xq));
        const half_t dy = (half_t)(yq - floorf(yq));
        const half_t one = (half_t)1.0f;
        const half_t omdx = one - dx, omdy = one - dy;
        half_t v = hmul(hmul(omdx, omdy), c00);
        v = hadd(v, hmul(hmul(dx, omdy), c01));
        v = hadd(v, hmul(hmul(omdx, dy), c10));
        v = hadd(v, hmul(hmul(dx, dy), c11));
        ob[bx * p.o_x + a * p.o_y + q * p.o_p] = v;
    }
}

// ---------------------------------------------------------------------------
// generic path: any float dtype / radius / patch size / strides.
// One thread per output element; the four raw chains it needs are recomputed
// (the reference's channel order and rounding per dtype).
// ---------------------------------------------------------------------------
struct CorrGenParams {
    const void* gmap;
    int64_t g_s[5];
    int N1, C, PH, PW;
    const void* fmap;
    int64_t f_s[5];
    int N2, H2, W2;
    const float* coords;
    int64_t c_s[5];
    const int64_t* ii;
    const int64_t* jj;
    int B, E, radius;
    float scale;
    void* out;
    int64_t o_b, o_e, o_x, o_y, o_i, o_j;
    int64_t total;
};

template <typename T>
__device__ __forceinline__ T chain_step(T s, T a, T b) { return s + a * b; }
template <>
__device__ __forceinline__ float chain_step<float>(float s, float a, float b) { return fmaf(a, b, s); }  // nvcc contracts `s += a*b`
template <>
__device__ __forceinline__ double chain_step<double>(double s, double a, double b) { return fma(a, b, s); }

template <typename T>
__device__ T raw_corr(const CorrGenParams& p, int b, int ix, int jx, int i0, int j0, int fy, int fx, int a, int c)
{
    const int i1 = wrap_add(fy, a - p.radius), j1 = wrap_add(fx, c - p.radius);
    T s = (T)0;
    if (ix < 0 || ix >= p.N1 || jx < 0 || jx >= p.N2) return s;
    if (!(i1 >= 0 && i1 < p.H2 && j1 >= 0 && j1 < p.W2)) return s;
    const T* f1 = (const T*)p.gmap + b * p.g_s[0] + (int64_t)ix * p.g_s[1] + i0 * p.g_s[3] + j0 * p.g_s[4];
    const T* f2 = (const T*)p.fmap + b * p.f_s[0] + (int64_t)jx * p.f_s[1] + (int64_t)i1 * p.f_s[3] + (int64_t)j1 * p.f_s[4];
    for (int k = 0; k < p.C; k++) s = chain_step<T>(s, f1[k * p.g_s[2]], f2[k * p.f_s[2]]);
    return s;
}

template <typename T>
__global__ __launch_bounds__(256) void corr_generic_kernel(CorrGenParams p)
{
    const int Do = 2 * p.radius + 1;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < p.total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        int64_t n = idx;
        const int j0 = n % p.PW; n /= p.PW;
        const int i0 = n % p.PH; n /= p.PH;
        const int bx = n % Do; n /= Do;
        const int a = n % Do; n /= Do;
        const int e = n % p.E; n /= p.E;
        const int b = (int)n;
        const int ix = (int)p.ii[e], jx = (int)p.jj[e];
        const float* cb = p.coords + b * p.c_s[0] + (int64_t)e * p.c_s[1] + i0 * p.c_s[3] + j0 * p.c_s[4];
        const float x = cb[0] / p.scale, y = cb[p.c_s[2]] / p.scale;
        const int fy = floor_to_int_sat(y), fx = floor_to_int_sat(x);
        const T c00 = raw_corr<T>(p, b, ix, jx, i0, j0, fy, fx, a, bx);
        const T c01 = raw_corr<T>(p, b, ix, jx, i0, j0, fy, fx, a, bx + 1);
        const T c10 = raw_corr<T>(p, b, ix, jx, i0, j0, fy, fx, a + 1, bx);
        const T c11 = raw_corr<T>(p, b, ix, jx, i0, j0, fy, fx, a + 1, bx + 1);
        const T dx = (T)(x - floorf(x)), dy = (T)(y - floorf(y));
        const T one = (T)1;
        const T omdx = one - dx, omdy = one - dy;
        T v = (omdx * omdy) * c00;
        v = v + (dx * omdy) * c01;
        v = v + (omdx * dy) * c10;
        v = v + (dx * dy) * c11;
        ((T*)p.out)[b * p.o_b + (int64_t)e * p.o_e + bx * p.o_x + a * p.o_y + i0 * p.o_i + j0 * p.o_j] = v;
    }
}

// ---------------------------------------------------------------------------
// backward (training surface): atomics into fp32/fp64 grads
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void corr_backward_kernel(const T* gmap, int N1, int C, int PH, int PW,
                                                            const T* fmap, int N2, int H2, int W2,
                                                            const float* coords, const int64_t* ii,
                                                            const int64_t* jj, const float* grad, int B, int E,
                                                            int radius, T* g1, T* g2, int64_t total)
{
    const int D = 2 * radius + 2, Do = D - 1;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        int64_t n = idx;
        const int j0 = n % PW; n /= PW;
        const int i0 = n % PH; n /= PH;
        const int c = n % D; n /= D;   // x offset in the raw window
        const int a = n % D; n /= D;   // y offset
        const int e = n % E; n /= E;
        const int b = (int)n;
        const float* cb = coords + (((int64_t)b * E + e) * 2) * PH * PW + i0 * PW + j0;
        const float x = cb[0], y = cb[PH * PW];
        const float dx = x - floorf(x), dy = y - floorf(y);
        // raw-window gradient = sum of the bilinear taps that read (a, c)
        float g = 0.f;
        auto G = [&](int aa, int cc) -> float {
            if (aa < 0 || aa >= Do || cc < 0 || cc >= Do) return 0.f;
            // grad layout: [B][E][x][y][PH][PW]
            return grad[((((int64_t)b * E + e) * Do + cc) * Do + aa) * PH * PW + i0 * PW + j0];
        };
        g += (1 - dx) * (1 - dy) * G(a, c);
        g += dx * (1 - dy) * G(a, c - 1);
        g += (1 - dx) * dy * G(a - 1, c);
        g += dx * dy * G(a - 1, c - 1);
        if (g == 0.f) continue;
        const int ix = (int)ii[e], jx = (int)jj[e];
        if (ix < 0 || ix >= N1 || jx < 0 || jx >= N2) continue;
        const int i1 = wrap_add(floor_to_int_sat(y), a - radius), j1 = wrap_add(floor_to_int_sat(x), c - radius);
        if (!(i1 >= 0 && i1 < H2 && j1 >= 0 && j1 < W2)) continue;
        const T* f1 = gmap + (((int64_t)b * N1 + ix) * C) * PH * PW + i0 * PW + j0;
        const T* f2 = fmap + (((int64_t)b * N2 + jx) * C) * H2 * W2 + (int64_t)i1 * W2 + j1;
        T* d1 = g1 + (((int64_t)b * N1 + ix) * C) * PH * PW + i0 * PW + j0;
        T* d2 = g2 + (((int64_t)b * N2 + jx) * C) * H2 * W2 + (int64_t)i1 * W2 + j1;
        for (int k = 0; k < C; k++) {
            atomicAdd(d1 + (int64_t)k * PH * PW, (T)g * f2[(int64_t)k * H2 * W2]);
            atomicAdd(d2 + (int64_t)k * H2 * W2, (T)g * f1[(int64_t)k * PH * PW]);
        }
    }
}

// ---------------------------------------------------------------------------
// patchify
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void patchify_forward_kernel(const T* net, int64_t s0, int64_t s1, int64_t s2,
                                                               int64_t s3, int B, int C, int H, int W,
                                                               const float* coords, int M, int radius, T* out,
                                                               int64_t total)
{
    const int D = 2 * radius + 2;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        int64_t n = idx;
        const int bb = n % D; n /= D;
        const int a = n % D; n /= D;
        const int k = n % C; n /= C;
        const int m = n % M; n /= M;
        const int b = (int)n;
        const float x = coords[((int64_t)b * M + m) * 2 + 0], y = coords[((int64_t)b * M + m) * 2 + 1];
        const int i = wrap_add(floor_to_int_sat(y), a - radius), j = wrap_add(floor_to_int_sat(x), bb - radius);
        T v = (T)0;
        if (i >= 0 && i < H && j >= 0 && j < W) v = net[b * s0 + k * s1 + (int64_t)i * s2 + (int64_t)j * s3];
        out[idx] = v;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void patchify_backward_kernel(int B, int C, int H, int W, const float* coords,
                                                                int M, int radius, const T* grad, T* net_grad,
                                                                int64_t total)
{
    const int D = 2 * radius + 2;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        int64_t n = idx;
        const int bb = n % D; n /= D;
        const int a = n % D; n /= D;
        const int k = n % C; n /= C;
        const int m = n % M; n /= M;
        const int b = (int)n;
        const float x = coords[((int64_t)b * M + m) * 2 + 0], y = coords[((int64_t)b * M + m) * 2 + 1];
        const int i = wrap_add(floor_to_int_sat(y), a - radius), j = wrap_add(floor_to_int_sat(x), bb - radius);
        if (i >= 0 && i < H && j >= 0 && j < W)
            atomicAdd(net_grad + (((int64_t)b * C + k) * H + i) * W + j, grad[idx]);
    }
}

}  // namespace dpvo

using namespace dpvo;

namespace {

bool fast_path_ok(int dtype, const int64_t* gsz, const int64_t* fsz, const int64_t* fst, const int64_t* csz,
                  int radius)
{
    if (dtype != DPVO_F16 || radius != corr::R) return false;
    if (gsz[3] != corr::PS || gsz[4] != corr::PS || csz[3] != corr::PS || csz[4] != corr::PS) return false;
    if (gsz[2] % 8 != 0 || gsz[2] > 512 || fsz[2] != gsz[2]) return false;
    if (fst[2] != 1) return false;  // channel-last storage
    if (fst[0] % 8 || fst[1] % 8 || fst[3] % 8 || fst[4] % 8) return false;  // 16-byte aligned pixels
    return true;
}

int launch_fast(int nlev, const void* gmap, const int64_t* gsz, const int64_t* gst, const void* const* fmaps,
                const int64_t* fsz, const int64_t* fst, const float* scales, const float* coords, const int64_t* csz,
                const int64_t* cst, const int64_t* ii, const int64_t* jj, void* out, const int64_t* ostr,
                hipStream_t stream)
{
    CorrFastParams p{};
    p.gmap = (const half_t*)gmap;
    for (int i = 0; i < 5; i++) { p.g_s[i] = gst[i]; p.c_s[i] = cst[i]; }
    p.N1 = (int)gsz[1];
    p.C = (int)gsz[2];
    p.coords = coords;
    p.ii = ii;
    p.jj = jj;
    p.B = (int)csz[0];
    p.E = (int)csz[1];
    for (int l = 0; l < nlev; l++) {
        if (reinterpret_cast<uintptr_t>(fmaps[l]) % 16) return 1;  // not 16-byte aligned: caller falls back
        p.fmap[l] = (const half_t*)fmaps[l];
        p.f_s0[l] = fst[l * 5 + 0];
        p.f_s1[l] = fst[l * 5 + 1];
        p.f_s3[l] = fst[l * 5 + 3];
        p.f_s4[l] = fst[l * 5 + 4];
        p.N2[l] = (int)fsz[l * 5 + 1];
        p.H2[l] = (int)fsz[l * 5 + 3];
        p.W2[l] = (int)fsz[l * 5 + 4];
        p.scale[l] = scales[l];
    }
    p.out = (half_t*)out;
    p.o_b = ostr[0]; p.o_e = ostr[1]; p.o_l = ostr[2]; p.o_x = ostr[3]; p.o_y = ostr[4]; p.o_p = ostr[5];
    const int64_t nblk = (int64_t)p.B * p.E;
    if (nblk == 0) return 0;
    const size_t lds = (size_t)p.C * 8 * 4 + (size_t)nlev * corr::NP * corr::BOX * corr::BOX * sizeof(half_t);
    if (nlev == 2)
        hipLaunchKernelGGL(corr_fast_kernel<2>, dim3((unsigned)nblk), dim3(256), lds, stream, p);
    else
        hipLaunchKernelGGL(corr_fast_kernel<1>, dim3((unsigned)nblk), dim3(128), lds, stream, p);
    return 0;
}

int launch_generic(int dtype, const void* gmap, const int64_t* gsz, const int64_t* gst, const void* fmap,
                   const int64_t* fsz, const int64_t* fst, float scale, const float* coords, const int64_t* csz,
                   const int64_t* cst, const int64_t* ii, const int64_t* jj, int radius, void* out,
                   const int64_t* ostr, hipStream_t stream)
{
    CorrGenParams p{};
    p.gmap = gmap;
    p.fmap = fmap;
    for (int i = 0; i < 5; i++) { p.g_s[i] = gst[i]; p.f_s[i] = fst[i]; p.c_s[i] = cst[i]; }
    p.N1 = (int)gsz[1]; p.C = (int)gsz[2]; p.PH = (int)csz[3]; p.PW = (int)csz[4];
    p.N2 = (int)fsz[1]; p.H2 = (int)fsz[3]; p.W2 = (int)fsz[4];
    p.coords = coords; p.ii = ii; p.jj = jj;
    p.B = (int)csz[0]; p.E = (int)csz[1]; p.radius = radius; p.scale = scale;
    p.out = out;
    p.o_b = ostr[0]; p.o_e = ostr[1]; p.o_x = ostr[2]; p.o_y = ostr[3]; p.o_i = ostr[4]; p.o_j = ostr[5];
    const int Do = 2 * radius + 1;
    p.total = (int64_t)p.B * p.E * Do * Do * p.PH * p.PW;
    if (p.total == 0) return 0;
    const unsigned grid = grid_for(p.total, 256, 65536);
    if (dtype == DPVO_F16)
        hipLaunchKernelGGL(corr_generic_kernel<half_t>, dim3(grid), dim3(256), 0, stream, p);
    else if (dtype == DPVO_F32)
        hipLaunchKernelGGL(corr_generic_kernel<float>, dim3(grid), dim3(256), 0, stream, p);
    else
        hipLaunchKernelGGL(corr_generic_kernel<double>, dim3(grid), dim3(256), 0, stream, p);
    return 0;
}

int check_common(int dtype, const void* gmap, const int64_t* gsz, const int64_t* csz, const int64_t* ii,
                 const int64_t* jj, int radius, const void* out)
{
    if (dtype != DPVO_F16 && dtype != DPVO_F32 && dtype != DPVO_F64) return 0;
    if (radius < 0 || radius > 64) return 0;
    if (csz[2] != 2 || gsz[0] != csz[0] || gsz[3] != csz[3] || gsz[4] != csz[4]) return 0;
    if (csz[1] > 0 && (!gmap || !ii || !jj || !out)) return 0;
    if (csz[0] * csz[1] > 0x7fffffff) return 0;
    return 1;
}

}  // namespace

extern "C" int dpvo_corr_forward(int dtype, const void* gmap, const int64_t* gmap_size, const int64_t* gmap_stride,
                                 const void* fmap, const int64_t* fmap_size, const int64_t* fmap_stride,
                                 const float* coords, const int64_t* coords_size, const int64_t* coords_stride,
                                 const int64_t* ii, const int64_t* jj, int radius, void* corr, void* stream)
{
    DPVO_CHECK_ARG(check_common(dtype, gmap, gmap_size, coords_size, ii, jj, radius, corr),
                   "invalid arguments (dtype/radius/shapes)");
    DPVO_CHECK_ARG(fmap_size[0] == coords_size[0] && fmap_size[2] == gmap_size[2], "fmap shape mismatch");
    const int Do = 2 * radius + 1;
    const int64_t P2 = coords_size[3] * coords_size[4];
    const int64_t E = coords_size[1];
    // output memory: contiguous [B][E][y][x][P][P]
    if (fast_path_ok(dtype, gmap_size, fmap_size, fmap_stride, coords_size, radius)) {
        const int64_t ostr[6] = {E * Do * Do * P2, Do * Do * P2, 0, P2, Do * P2, 1};
        const void* fm[1] = {fmap};
        const float sc[1] = {1.0f};
        const int rc = launch_fast(1, gmap, gmap_size, gmap_stride, fm, fmap_size, fmap_stride, sc, coords,
                                   coords_size, coords_stride, ii, jj, corr, ostr, as_stream(stream));
        if (rc == 0) { DPVO_CHECK_LAUNCH(); return 0; }
    }
    const int64_t ostr[6] = {E * Do * Do * P2, Do * Do * P2, P2, Do * P2, coords_size[4], 1};
    launch_generic(dtype, gmap, gmap_size, gmap_stride, fmap, fmap_size, fmap_stride, 1.0f, coords, coords_size,
                   coords_stride, ii, jj, radius, corr, ostr, as_stream(stream));
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_corr_forward_pyramid(int dtype, const void* gmap, const int64_t* gmap_size,
                                         const int64_t* gmap_stride, int nlev, const void* const* fmaps,
                                         const int64_t* fmap_sizes, const int64_t* fmap_strides,
                                         const float* level_scale, const float* coords, const int64_t* coords_size,
                                         const int64_t* coords_stride, const int64_t* ii, const int64_t* jj,
                                         int radius, void* corr, void* stream)
{
    DPVO_CHECK_ARG(check_common(dtype, gmap, gmap_size, coords_size, ii, jj, radius, corr),
                   "invalid arguments (dtype/radius/shapes)");
    DPVO_CHECK_ARG(nlev >= 1 && nlev <= 8 && fmaps && level_scale, "nlev must be 1..8");
    const int Do = 2 * radius + 1;
    const int64_t P2 = coords_size[3] * coords_size[4];
    const int64_t E = coords_size[1];
    // output: [B][E][x][y][P][P][L]
    const int64_t o_e = (int64_t)Do * Do * P2 * nlev;
    bool all_fast = nlev <= 2;
    for (int l = 0; l < nlev && all_fast; l++)
        all_fast = fast_path_ok(dtype, gmap_size, fmap_sizes + 5 * l, fmap_strides + 5 * l, coords_size, radius) &&
                   fmap_sizes[5 * l] == coords_size[0];
    if (all_fast) {
        const int64_t ostr[6] = {E * o_e, o_e, 1, Do * P2 * nlev, P2 * nlev, nlev};
        const int rc = launch_fast(nlev, gmap, gmap_size, gmap_stride, fmaps, fmap_sizes, fmap_strides, level_scale,
                                   coords, coords_size, coords_stride, ii, jj, corr, ostr, as_stream(stream));
        if (rc == 0) { DPVO_CHECK_LAUNCH(); return 0; }
    }
    for (int l = 0; l < nlev; l++) {
        DPVO_CHECK_ARG(fmap_sizes[5 * l] == coords_size[0] && fmap_sizes[5 * l + 2] == gmap_size[2],
                       "fmap shape mismatch");
        const size_t esz = dtype == DPVO_F16 ? 2 : dtype == DPVO_F32 ? 4 : 8;
        void* o = (char*)corr + l * esz;
        const int64_t ostr[6] = {E * o_e, o_e, Do * P2 * nlev, P2 * nlev, coords_size[4] * nlev, nlev};
        launch_generic(dtype, gmap, gmap_size, gmap_stride, fmaps[l], fmap_sizes + 5 * l, fmap_strides + 5 * l,
                       level_scale[l], coords, coords_size, coords_stride, ii, jj, radius, o, ostr,
                       as_stream(stream));
        DPVO_CHECK_LAUNCH();
    }
    return 0;
}

extern "C" int dpvo_corr_backward(int dtype, const void* gmap, const int64_t* gsz, const void* fmap,
                                  const int64_t* fsz, const float* coords, const int64_t* csz, const int64_t* ii,
                                  const int64_t* jj, const float* grad, int radius, void* gmap_grad, void* fmap_grad,
                                  void* stream)
{
    DPVO_CHECK_ARG(dtype == DPVO_F32 || dtype == DPVO_F64, "backward supports float32/float64 feature maps");
    DPVO_CHECK_ARG(csz[2] == 2 && radius >= 0, "bad coords / radius");
    const int D = 2 * radius + 2;
    const int64_t total = csz[0] * csz[1] * D * D * csz[3] * csz[4];
    if (total == 0) return 0;
    const unsigned grid = grid_for(total, 256, 65536);
    if (dtype == DPVO_F32)
        hipLaunchKernelGGL(corr_backward_kernel<float>, dim3(grid), dim3(256), 0, as_stream(stream),
                           (const float*)gmap, (int)gsz[1], (int)gsz[2], (int)csz[3], (int)csz[4],
                           (const float*)fmap, (int)fsz[1], (int)fsz[3], (int)fsz[4], coords, ii, jj, grad,
                           (int)csz[0], (int)csz[1], radius, (float*)gmap_grad, (float*)fmap_grad, total);
    else
        hipLaunchKernelGGL(corr_backward_kernel<double>, dim3(grid), dim3(256), 0, as_stream(stream),
                           (const double*)gmap, (int)gsz[1], (int)gsz[2], (int)csz[3], (int)csz[4],
                           (const double*)fmap, (int)fsz[1], (int)fsz[3], (int)fsz[4], coords, ii, jj, grad,
                           (int)csz[0], (int)csz[1], radius, (double*)gmap_grad, (double*)fmap_grad, total);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_patchify_forward(int dtype, const void* net, const int64_t* nsz, const int64_t* nst,
                                     const float* coords, int64_t M, int radius, void* out, void* stream)
{
    DPVO_CHECK_ARG(radius >= 0 && radius <= 64, "bad radius");
    const int D = 2 * radius + 2;
    const int64_t total = nsz[0] * M * nsz[1] * D * D;
    if (total == 0) return 0;
    const unsigned grid = grid_for(total, 256, 65536);
#define PF_LAUNCH(T)                                                                                        \
    hipLaunchKernelGGL(patchify_forward_kernel<T>, dim3(grid), dim3(256), 0, as_stream(stream), (const T*)net, \
                       nst[0], nst[1], nst[2], nst[3], (int)nsz[0], (int)nsz[1], (int)nsz[2], (int)nsz[3], coords, \
                       (int)M, radius, (T*)out, total)
    if (dtype == DPVO_F16) PF_LAUNCH(half_t);
    else if (dtype == DPVO_F32) PF_LAUNCH(float);
    else if (dtype == DPVO_F64) PF_LAUNCH(double);
    else DPVO_CHECK_ARG(false, "unsupported dtype");
#undef PF_LAUNCH
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_patchify_backward(int dtype, const int64_t* nsz, const float* coords, int64_t M, int radius,
                                      const void* grad, void* net_grad, void* stream)
{
    DPVO_CHECK_ARG(dtype == DPVO_F32 || dtype == DPVO_F64, "patchify backward supports float32/float64");
    const int D = 2 * radius + 2;
    const int64_t total = nsz[0] * M * nsz[1] * D * D;
    if (total == 0) return 0;
    const unsigned grid = grid_for(total, 256, 65536);
    if (dtype == DPVO_F32)
        hipLaunchKernelGGL(patchify_backward_kernel<float>, dim3(grid), dim3(256), 0, as_stream(stream),
                           (int)nsz[0], (int)nsz[1], (int)nsz[2], (int)nsz[3], coords, (int)M, radius,
                           (const float*)grad, (float*)net_grad, total);
    else
        hipLaunchKernelGGL(patchify_backward_kernel<double>, dim3(grid), dim3(256), 0, as_stream(stream),
                           (int)nsz[0], (int)nsz[1], (int)nsz[2], (int)nsz[3], coords, (int)M, radius,
                           (const double*)grad, (double*)net_grad, total);
    DPVO_CHECK_LAUNCH();
    return 0;
}

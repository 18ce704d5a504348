// corrmfma.hip -- DPVO's two-level patch correlation on the gfx950 matrix cores.
//
// The same quantity as DPVO.corr (reference dpvo/dpvo.py:326-333 ->
// correlation_kernel.cu:83-135 + the ATen bilinear epilogue :221-232):
// for each edge, the 3x3 patch's 128-channel features dotted with every pixel
// of an 8x8 window around each of the nine reprojected patch pixels, at two
// pyramid levels, bilinearly reduced to 7x7 and stacked as one 882-wide row
// [x][y][P][P][level].  Here the dot products are one small GEMM per edge and
// level -- (9 patch pixels, zero-padded to 16) x 128 channels x (the box of
// pixels covering the nine windows) -- on v_mfma_f32_16x16x32_f16: fp16
// operands, fp32 accumulation, fp32 bilinear epilogue, one rounding to fp16 at
// the output.  That is more accurate than the reference, which accumulates the
// 128 products in fp16 (the bit-exact emulation of it stays in altcorr.hip);
// tests/test_gpu_corr_mfma.py bounds the difference against the oracle's fp16
// and fp64 modes.
//
// Layout: one wave per edge, four edges per workgroup.  The patch features
// come from a transposed copy of the gmap ring, [patch][pixel][channel]
// (dpvo_corr_pack_mfma), so each lane's A fragment is one 16-byte load; the
// fmap ring is channel-last, so each lane's B fragment (8 channels of one box
// pixel) is one 16-byte load too.  The raw 16x16 tiles go to a per-wave LDS
// scratch, from which the bilinear epilogue writes 256-byte coalesced rows.
#include "common.hpp"

namespace dpvo {

namespace cm {
constexpr int R = 3, D = 8, DO = 7, NP = 9, C = 128, BOXMAX = 12, WAVES = 4;
constexpr int RS = 148;   // raw row stride (>= 144 box slots; 4 rows apart land 16 banks apart)
}  // namespace cm

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f4m_t __attribute__((ext_vector_type(4)));

struct CorrMfmaParams {
    const half_t* gt;   // [N1][9][128] transposed patch features
    int N1;
    const float* coords;
    int64_t c_s[5];
    const int64_t* ii;
    const int64_t* jj;
    int E;
    const half_t* fmap[2];
    int64_t f_s1[2], f_s3[2], f_s4[2];
    int N2[2], H2[2], W2[2];
    float scale[2];
    half_t* out;
    int64_t o_e;
};

struct CorrMfmaMeta {
    float xs[2][cm::NP], ys[2][cm::NP];
    int fy[2][cm::NP], fx[2][cm::NP];
    int oy[2], ox[2], bw[2], bh[2], fast[2], ntiles[2];
};

__device__ __forceinline__ void cm_wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// blocks b, b + 8, ... share an XCD under round-robin dispatch: give each XCD a
// contiguous run of edges (consecutive edges mostly share a target frame)
__device__ __forceinline__ int cm_xcd_swizzle(int b, int nblk)
{
    const int main = nblk & ~7;
    if (b >= main) return b;
    return (b & 7) * (main >> 3) + (b >> 3);
}

__global__ __launch_bounds__(64 * cm::WAVES) void corr_mfma_kernel(CorrMfmaParams p)
{
    using namespace cm;
    __shared__ float raw[WAVES][2][NP][RS];
    __shared__ CorrMfmaMeta meta[WAVES];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int e = cm_xcd_swizzle(blockIdx.x, gridDim.x) * WAVES + wave;
    if (e >= p.E) return;   // the whole wave; nothing below synchronises across waves
    CorrMfmaMeta& m = meta[wave];
    float (*rw)[NP][RS] = raw[wave];
    const int ix = (int)p.ii[e], jx = (int)p.jj[e];
    const bool ix_ok = ix >= 0 && ix < p.N1;

    // ---- coordinates, floors, and per level the box covering the nine windows
    if (lane < 2 * NP) {
        const int lev = lane / NP, q = lane - lev * NP;
        const float* cb = p.coords + (int64_t)e * p.c_s[1];
        const int64_t o = (q / 3) * p.c_s[3] + (q % 3) * p.c_s[4];
        const float x = cb[o] / p.scale[lev], y = cb[p.c_s[2] + o] / p.scale[lev];
        m.xs[lev][q] = x;
        m.ys[lev][q] = y;
        m.fy[lev][q] = floor_to_int_sat(y);
        m.fx[lev][q] = floor_to_int_sat(x);
    }
    cm_wave_fence();
    if (lane < 2) {
        const int lev = lane;
        int ymin = 0x7fffffff, ymax = (int)0x80000000u, xmin = 0x7fffffff, xmax = (int)0x80000000u;
#pragma unroll
        for (int q = 0; q < NP; q++) {
            ymin = min(ymin, m.fy[lev][q]); ymax = max(ymax, m.fy[lev][q]);
            xmin = min(xmin, m.fx[lev][q]); xmax = max(xmax, m.fx[lev][q]);
        }
        const bool fast = ((int64_t)ymax - ymin) <= BOXMAX - D && ((int64_t)xmax - xmin) <= BOXMAX - D;
        m.fast[lev] = fast;
        m.oy[lev] = wrap_add(ymin, -R);
        m.ox[lev] = wrap_add(xmin, -R);
        m.bh[lev] = fast ? ymax - ymin + D : D;
        m.bw[lev] = fast ? xmax - xmin + D : D;
        // wide spreads: one 8x8 window per patch pixel, 4 tiles each
        m.ntiles[lev] = fast ? (m.bh[lev] * m.bw[lev] + 15) / 16 : NP * 4;
    }
    cm_wave_fence();

    // ---- A fragments: patch pixel (lane & 15) x 8 channels of each 32-channel step
    const int q16 = lane & 15, kc = lane >> 4;
    const h8_t hz = (h8_t)(_Float16)0;
    h8_t a[4];
    {
        const bool ok = ix_ok && q16 < NP;
        const half_t* ga = p.gt + ((int64_t)(ok ? ix : 0) * NP + (ok ? q16 : 0)) * C + 8 * kc;
#pragma unroll
        for (int ks = 0; ks < 4; ks++) a[ks] = ok ? *(const h8_t*)(ga + 32 * ks) : hz;
    }

    // ---- the box tiles of both levels, one flat pipelined sequence
    const int nt0 = m.ntiles[0], ntot = nt0 + m.ntiles[1];
    struct Src { const h8_t* ptr; bool inb; int lev, n, qq; };
    auto locate = [&](int t) {
        Src s;
        s.lev = t >= nt0 ? 1 : 0;
        const int tl = s.lev ? t - nt0 : t;
        const int bw = m.bw[s.lev];
        int gy, gx;
        bool valid;
        if (m.fast[s.lev]) {
            s.n = tl * 16 + q16;
            s.qq = -1;
            const int by = s.n / bw, bx = s.n - by * bw;
            valid = s.n < bw * m.bh[s.lev];
            gy = wrap_add(m.oy[s.lev], by);
            gx = wrap_add(m.ox[s.lev], bx);
        } else {
            s.qq = tl >> 2;
            s.n = (tl & 3) * 16 + q16;
            gy = wrap_add(m.fy[s.lev][s.qq], (s.n >> 3) - R);
            gx = wrap_add(m.fx[s.lev][s.qq], (s.n & 7) - R);
            valid = true;
        }
        const int lv = s.lev;
        s.inb = valid && ix_ok && jx >= 0 && jx < p.N2[lv] && gy >= 0 && gy < p.H2[lv] && gx >= 0 && gx < p.W2[lv];
        s.ptr = reinterpret_cast<const h8_t*>(
            p.fmap[lv] + (s.inb ? (int64_t)jx * p.f_s1[lv] + (int64_t)gy * p.f_s3[lv] + (int64_t)gx * p.f_s4[lv] : 0) +
            8 * kc);
        return s;
    };
    Src cur = locate(0);
    h8_t b[4], bn[4] = {hz, hz, hz, hz};
#pragma unroll
    for (int ks = 0; ks < 4; ks++) b[ks] = cur.inb ? cur.ptr[4 * ks] : hz;
    for (int t = 0; t < ntot; t++) {
        Src nxt = cur;
        if (t + 1 < ntot) {
            nxt = locate(t + 1);
#pragma unroll
            for (int ks = 0; ks < 4; ks++) bn[ks] = nxt.inb ? nxt.ptr[4 * ks] : hz;
        }
        f4m_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ks++) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ks], b[ks], acc, 0, 0, 0);
        // acc[r] = patch pixel 4 kc + r . box slot cur.n (out-of-box slots are zero and unread)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int row = 4 * kc + r;
            if (row < NP && (cur.qq < 0 || row == cur.qq)) rw[cur.lev][row][cur.n] = acc[r];
        }
        cur = nxt;
#pragma unroll
        for (int ks = 0; ks < 4; ks++) b[ks] = bn[ks];
    }
    cm_wave_fence();

    // ---- bilinear 8x8 -> 7x7 per pixel and level (fp32), stacked row [x][y][P][P][level]
    half_t* orow = p.out + (int64_t)e * p.o_e;
    for (int t = lane; t < DO * DO * NP; t += 64) {
        const int pos = t / NP, q = t - pos * NP;
        const int bxo = pos / DO, ay = pos - bxo * DO;   // x offset (outer), y offset
        float v[2];
#pragma unroll
        for (int lev = 0; lev < 2; lev++) {
            const float x = m.xs[lev][q], y = m.ys[lev][q];
            const float dx = x - floorf(x), dy = y - floorf(y);
            int base, st;
            if (m.fast[lev]) {
                st = m.bw[lev];
                base = (m.fy[lev][q] - wrap_add(m.oy[lev], R)) * st + (m.fx[lev][q] - wrap_add(m.ox[lev], R));
            } else {
                st = D;
                base = 0;
            }
            const float* r0 = &rw[lev][q][base + ay * st + bxo];
            v[lev] = (1.f - dx) * (1.f - dy) * r0[0] + dx * (1.f - dy) * r0[1] + (1.f - dx) * dy * r0[st] +
                     dx * dy * r0[st + 1];
        }
        *(half2_t*)(orow + 2 * t) = half2_t{(half_t)v[0], (half_t)v[1]};
    }
}

// gmap [N1][C][3][3] (any strides) -> [N1][9][C] contiguous
__global__ __launch_bounds__(256) void corr_pack_mfma_kernel(const half_t* __restrict__ gmap, int64_t gs1, int64_t gs2,
                                                             int64_t gs3, int64_t gs4, int N1, half_t* __restrict__ gt)
{
    const int64_t total = (int64_t)N1 * cm::C;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(t % cm::C);
        const int64_t n = t / cm::C;
        const half_t* g = gmap + n * gs1 + c * gs2;
#pragma unroll
        for (int q = 0; q < cm::NP; q++) gt[(n * cm::NP + q) * cm::C + c] = g[(q / 3) * gs3 + (q % 3) * gs4];
    }
}

}  // namespace dpvo

using namespace dpvo;

extern "C" size_t dpvo_corr_pack_mfma_bytes(const int64_t* gmap_size)
{
    return (size_t)gmap_size[0] * gmap_size[1] * cm::NP * cm::C * 2;
}

extern "C" int dpvo_corr_pack_mfma(const void* gmap, const int64_t* gmap_size, const int64_t* gmap_stride,
                                   void* table, void* stream)
{
    DPVO_CHECK_ARG(gmap_size[0] == 1 && gmap_size[2] == cm::C && gmap_size[3] == 3 && gmap_size[4] == 3,
                   "gmap must be [1][N1][128][3][3]");
    const int N1 = (int)gmap_size[1];
    if (N1 == 0) return 0;
    const int64_t total = (int64_t)N1 * cm::C;
    hipLaunchKernelGGL(corr_pack_mfma_kernel, dim3(grid_for(total, 256, 8192)), dim3(256), 0, as_stream(stream),
                       (const half_t*)gmap, gmap_stride[1], gmap_stride[2], gmap_stride[3], gmap_stride[4], N1,
                       (half_t*)table);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_corr_pyramid_mfma(const void* table, int64_t num_patches, const void* const* fmaps,
                                      const int64_t* fmap_sizes, const int64_t* fmap_strides,
                                      const float* level_scale, const float* coords, const int64_t* coords_size,
                                      const int64_t* coords_stride, const int64_t* ii, const int64_t* jj, void* corr,
                                      int64_t edge_stride, void* stream)
{
    DPVO_CHECK_ARG(coords_size[0] == 1 && coords_size[2] == 2 && coords_size[3] == 3 && coords_size[4] == 3,
                   "coords must be [1][E][2][3][3]");
    DPVO_CHECK_ARG(edge_stride == 0 || edge_stride >= 882, "edge_stride smaller than one edge's 882 features");
    const int64_t E = coords_size[1];
    DPVO_CHECK_ARG(E < 0x7fffffff && num_patches < 0x7fffffff, "too many edges / patches");
    CorrMfmaParams p{};
    p.gt = (const half_t*)table;
    p.N1 = (int)num_patches;
    p.coords = coords;
    for (int i = 0; i < 5; i++) p.c_s[i] = coords_stride[i];
    p.ii = ii;
    p.jj = jj;
    p.E = (int)E;
    for (int l = 0; l < 2; l++) {
        const int64_t* fs = fmap_sizes + 5 * l;
        const int64_t* ft = fmap_strides + 5 * l;
        DPVO_CHECK_ARG(fs[0] == 1 && fs[2] == cm::C, "fmaps must be [1][N2][128][H][W]");
        DPVO_CHECK_ARG(ft[2] == 1 && ft[1] % 8 == 0 && ft[3] % 8 == 0 && ft[4] % 8 == 0 &&
                           reinterpret_cast<uintptr_t>(fmaps[l]) % 16 == 0,
                       "fmaps must be channel-last with 16-byte aligned pixels");
        p.fmap[l] = (const half_t*)fmaps[l];
        p.f_s1[l] = ft[1];
        p.f_s3[l] = ft[3];
        p.f_s4[l] = ft[4];
        p.N2[l] = (int)fs[1];
        p.H2[l] = (int)fs[3];
        p.W2[l] = (int)fs[4];
        p.scale[l] = level_scale[l];
    }
    DPVO_CHECK_ARG(reinterpret_cast<uintptr_t>(table) % 16 == 0, "table must be 16-byte aligned");
    p.out = (half_t*)corr;
    p.o_e = edge_stride ? edge_stride : 882;
    DPVO_CHECK_ARG(reinterpret_cast<uintptr_t>(corr) % 4 == 0 && p.o_e % 2 == 0, "corr rows must be 4-byte aligned");
    if (E == 0) return 0;
    const unsigned grid = (unsigned)((E + cm::WAVES - 1) / cm::WAVES);
    hipLaunchKernelGGL(corr_mfma_kernel, dim3(grid), dim3(64 * cm::WAVES), 0, as_stream(stream), p);
    DPVO_CHECK_LAUNCH();
    return 0;
}

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
#include <algorithm>

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
    const int* order;   // optional edge visiting order (edges grouped by target frame), NULL = 0..E-1
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

// per-edge prologue operands, loaded one edge ahead
struct CmEdgeIn {
    int e, ix, jx;
    float cx[1], cy[1];   // lane < 9: patch pixel q's coordinates (x, y) -- level scaling applied later
};

__device__ __forceinline__ CmEdgeIn cm_load_edge(const CorrMfmaParams& p, int slot, int lane)
{
    CmEdgeIn in;
    in.e = p.order ? p.order[slot] : slot;
    in.ix = (int)p.ii[in.e];
    in.jx = (int)p.jj[in.e];
    const int q = lane < cm::NP ? lane : 0;
    const float* cb = p.coords + (int64_t)in.e * p.c_s[1] + (q / 3) * p.c_s[3] + (q % 3) * p.c_s[4];
    in.cx[0] = cb[0];
    in.cy[0] = cb[p.c_s[2]];
    return in;
}

// One wave per edge, persistent over a grid-stride range of edge slots.  The
// next edge's indices and coordinates are in flight while the current edge
// runs; the box tiles of both levels are one flat sequence whose B fragments
// are loaded three tiles ahead (a static register ring), so about 12 KB per
// wave is in flight at any time.
__global__ __launch_bounds__(64 * cm::WAVES) void corr_mfma_kernel(CorrMfmaParams p)
{
    using namespace cm;
    __shared__ float raw[WAVES][2][NP][RS];
    __shared__ CorrMfmaMeta meta[WAVES];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nwaves = gridDim.x * WAVES;
    int slot = cm_xcd_swizzle(blockIdx.x, gridDim.x) * WAVES + wave;
    if (slot >= p.E) return;   // the whole wave; nothing below synchronises across waves
    CorrMfmaMeta& m = meta[wave];
    float (*rw)[NP][RS] = raw[wave];
    const int q16 = lane & 15, kc = lane >> 4;
    const h8_t hz = (h8_t)(_Float16)0;
    CmEdgeIn nin = cm_load_edge(p, slot, lane);

    for (; slot < p.E; slot += nwaves) {
        const CmEdgeIn in = nin;
        if (slot + nwaves < p.E) nin = cm_load_edge(p, slot + nwaves, lane);
        const int e = in.e, ix = in.ix, jx = in.jx;
        const bool ix_ok = ix >= 0 && ix < p.N1;

        // ---- coordinates, floors, and per level the box covering the nine windows
        cm_wave_fence();   // the previous edge's epilogue has read meta / raw
        if (lane < 2 * NP) {
            const int lev = lane / NP, q = lane - lev * NP;
            const float xr = __shfl(in.cx[0], q), yr = __shfl(in.cy[0], q);
            const float x = xr / p.scale[lev], y = yr / p.scale[lev];
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
        h8_t a[4];
        {
            const bool ok = ix_ok && q16 < NP;
            const half_t* ga = p.gt + ((int64_t)(ok ? ix : 0) * NP + (ok ? q16 : 0)) * C + 8 * kc;
#pragma unroll
            for (int ks = 0; ks < 4; ks++) a[ks] = ok ? *(const h8_t*)(ga + 32 * ks) : hz;
        }

        // ---- box tiles of both levels.  Per-level constants are selected, never
        // indexed by the runtime level: an indexed kernel argument is a memory
        // load whose vmcnt(0) wait would drain the prefetched tiles every step.
        const int nt0 = m.ntiles[0], ntot = nt0 + m.ntiles[1];
        struct Lev { const half_t* base; int64_t s3, s4; int H, W, fast, bw, bh, oy, ox; bool ok; };
        Lev L0, L1;
#pragma unroll
        for (int l = 0; l < 2; l++) {
            Lev& L = l ? L1 : L0;
            const bool jok = jx >= 0 && jx < p.N2[l];
            L.base = p.fmap[l] + (jok ? (int64_t)jx * p.f_s1[l] : 0) + 8 * kc;
            L.s3 = p.f_s3[l];
            L.s4 = p.f_s4[l];
            L.H = p.H2[l];
            L.W = p.W2[l];
            L.fast = m.fast[l];
            L.bw = m.bw[l];
            L.bh = m.bh[l];
            L.oy = m.oy[l];
            L.ox = m.ox[l];
            L.ok = jok && ix_ok;
        }
        struct Src { const h8_t* ptr; bool inb; int lev, n, qq; };
        auto locate = [&](int t) {
            Src s;
            s.lev = t >= nt0 ? 1 : 0;
            const Lev& L = s.lev ? L1 : L0;
            const int tl = s.lev ? t - nt0 : t;
            int gy, gx;
            bool valid;
            if (L.fast) {
                s.n = tl * 16 + q16;
                s.qq = -1;
                const int by = s.n / L.bw, bx = s.n - by * L.bw;
                valid = s.n < L.bw * L.bh;
                gy = wrap_add(L.oy, by);
                gx = wrap_add(L.ox, bx);
            } else {
                s.qq = tl >> 2;
                s.n = (tl & 3) * 16 + q16;
                gy = wrap_add(m.fy[s.lev][s.qq], (s.n >> 3) - R);
                gx = wrap_add(m.fx[s.lev][s.qq], (s.n & 7) - R);
                valid = true;
            }
            s.inb = t < ntot && valid && L.ok && gy >= 0 && gy < L.H && gx >= 0 && gx < L.W;
            s.ptr = reinterpret_cast<const h8_t*>(L.base + (s.inb ? (int64_t)gy * L.s3 + (int64_t)gx * L.s4 : 0));
            return s;
        };
        // loads are unconditional (an out-of-box slot reads the map's first pixel)
        // and masked at the MFMA: a load under a branch makes the wait counter
        // unknown at the loop head, and the compiler then waits for everything
        auto fetch = [&](const Src& s, h8_t* b) {
#pragma unroll
            for (int ks = 0; ks < 4; ks++) b[ks] = s.ptr[4 * ks];
        };
        auto consume = [&](const Src& s, const h8_t* b) {
            f4m_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 4; ks++)
                acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ks], s.inb ? b[ks] : hz, acc, 0, 0, 0);
            // acc[r] = patch pixel 4 kc + r . box slot s.n (out-of-box slots are zero and unread)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = 4 * kc + r;
                if (row < NP && (s.qq < 0 || row == s.qq)) rw[s.lev][row][s.n] = acc[r];
            }
        };
        Src s0 = locate(0), s1 = locate(1), s2 = locate(2);
        h8_t b0[4], b1[4], b2[4];
        // issue order must match consume order, or the wait at the loop head
        // (merged over the entry and the back edge) drains the whole ring
        fetch(s0, b0);
        __builtin_amdgcn_sched_barrier(0);
        fetch(s1, b1);
        __builtin_amdgcn_sched_barrier(0);
        fetch(s2, b2);
        __builtin_amdgcn_sched_barrier(0);
        for (int t = 0; t < ntot; t += 3) {
            consume(s0, b0);
            s0 = locate(t + 3);
            fetch(s0, b0);
            if (t + 1 < ntot) consume(s1, b1);
            s1 = locate(t + 4);
            fetch(s1, b1);
            if (t + 2 < ntot) consume(s2, b2);
            s2 = locate(t + 5);
            fetch(s2, b2);
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
}

// edge visiting order grouped by target frame (counting sort; the order inside
// a frame's group is arbitrary -- it only affects which edges share an L2)
__global__ __launch_bounds__(256) void edge_hist_kernel(const int64_t* __restrict__ jj, int64_t E, int nb,
                                                        int* __restrict__ count)
{
    extern __shared__ int h[];
    for (int i = threadIdx.x; i <= nb; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = jj[e];
        atomicAdd(&h[(j >= 0 && j < nb) ? (int)j : nb], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= nb; i += blockDim.x)
        if (h[i]) atomicAdd(&count[i], h[i]);
}

// scatter: each workgroup counts its chunk per bucket in LDS, reserves one
// contiguous run per bucket with a single global atomic, then fills it
// (every thread adding to a few shared global cursors serialises: ~0.4 ms)
__global__ __launch_bounds__(256) void edge_scatter_kernel(const int64_t* __restrict__ jj, int64_t E, int nb,
                                                           const int* __restrict__ count, int* __restrict__ cursor,
                                                           int* __restrict__ order)
{
    extern __shared__ int sh[];
    int* base = sh;              // [nb + 1] global start of this workgroup's run per bucket
    int* loc = sh + (nb + 1);    // [nb + 1] local counts, then local cursors
    const int64_t chunk = (E + gridDim.x - 1) / gridDim.x;
    const int64_t e0 = blockIdx.x * chunk, e1 = min(E, e0 + chunk);
    for (int i = threadIdx.x; i <= nb; i += blockDim.x) loc[i] = 0;
    __syncthreads();
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const int64_t j = jj[e];
        atomicAdd(&loc[(j >= 0 && j < nb) ? (int)j : nb], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;
        for (int i = 0; i <= nb; i++) {
            const int c = count[i];
            base[i] = loc[i] ? s + atomicAdd(&cursor[i], loc[i]) : 0;
            s += c;
            loc[i] = 0;
        }
    }
    __syncthreads();
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const int64_t j = jj[e];
        const int b = (j >= 0 && j < nb) ? (int)j : nb;
        order[base[b] + atomicAdd(&loc[b], 1)] = (int)e;
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

extern "C" size_t dpvo_edge_order_workspace_bytes(int num_buckets) { return (size_t)2 * (num_buckets + 1) * 4; }

extern "C" int dpvo_edge_order(const int64_t* jj, int64_t num_edges, int num_buckets, int* order, void* workspace,
                               size_t workspace_bytes, void* stream)
{
    DPVO_CHECK_ARG(num_buckets >= 1 && num_buckets <= 16384, "num_buckets must be 1..16384");
    DPVO_CHECK_ARG(num_edges >= 0 && num_edges < 0x7fffffff, "bad edge count");
    DPVO_CHECK_ARG(workspace && workspace_bytes >= dpvo_edge_order_workspace_bytes(num_buckets), "workspace too small");
    if (num_edges == 0) return 0;
    hipStream_t s = as_stream(stream);
    int* count = (int*)workspace;
    int* cursor = count + num_buckets + 1;
    DPVO_CHECK_HIP(hipMemsetAsync(workspace, 0, dpvo_edge_order_workspace_bytes(num_buckets), s));
    const size_t lds = (size_t)(num_buckets + 1) * 4;
    const unsigned g = grid_for(num_edges, 256, 512);
    hipLaunchKernelGGL(edge_hist_kernel, dim3(g), dim3(256), lds, s, jj, num_edges, num_buckets, count);
    const unsigned gs = grid_for(num_edges, 2048, 256);
    hipLaunchKernelGGL(edge_scatter_kernel, dim3(gs), dim3(256), 2 * lds, s, jj, num_edges, num_buckets, count,
                       cursor, order);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_corr_pyramid_mfma(const void* table, int64_t num_patches, const void* const* fmaps,
                                      const int64_t* fmap_sizes, const int64_t* fmap_strides,
                                      const float* level_scale, const float* coords, const int64_t* coords_size,
                                      const int64_t* coords_stride, const int64_t* ii, const int64_t* jj, void* corr,
                                      int64_t edge_stride, const int* order, void* stream)
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
    p.order = order;
    DPVO_CHECK_ARG(reinterpret_cast<uintptr_t>(corr) % 4 == 0 && p.o_e % 2 == 0, "corr rows must be 4-byte aligned");
    if (E == 0) return 0;
    // persistent: a few workgroups per CU, each wave walking a grid-stride range of edges
    const unsigned grid = (unsigned)std::min<int64_t>((E + cm::WAVES - 1) / cm::WAVES, 256 * 3);  // LDS: 3 per CU
    hipLaunchKernelGGL(corr_mfma_kernel, dim3(grid), dim3(64 * cm::WAVES), 0, as_stream(stream), p);
    DPVO_CHECK_LAUNCH();
    return 0;
}

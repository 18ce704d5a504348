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
#include <cstdlib>

#include "corrmfma.hpp"

namespace dpvo {


typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f4m_t __attribute__((ext_vector_type(4)));



__device__ __forceinline__ void cm_wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Edge slots per wave.  Workgroups are dispatched to the 8 XCDs round-robin
// (block b on XCD b % 8), each with its own L2: give each XCD one contiguous
// eighth of the (target-frame-grouped) edge sequence, walked by all of its
// waves in step, so an XCD streams through a few target frames' maps instead
// of every XCD touching every frame.
struct CmRange { int slot, end, stride; };
__device__ __forceinline__ CmRange cm_range(int E, int wave)
{
    const int nblk = gridDim.x, b = blockIdx.x;
    CmRange r;
    if (nblk >= 8 && (nblk & 7) == 0) {
        const int x = b & 7, per = nblk >> 3;
        const int lo = (int)((int64_t)E * x / 8);
        r.end = (int)((int64_t)E * (x + 1) / 8);
        r.slot = lo + (b >> 3) * cm::WAVES + wave;
        r.stride = per * cm::WAVES;
    } else {
        r.slot = b * cm::WAVES + wave;
        r.end = E;
        r.stride = nblk * cm::WAVES;
    }
    return r;
}

// The loaded registers l[ks] hold, in lane (q16, kc), chunk
// 8 (ks >> 1) + 4 (q16 & 1) + kc of pixel (q16 & ~1) + (ks & 1).  The MFMA
// operand m[j] must hold chunk 4 j + kc of pixel q16 in every lane:
//   m[2h]     = even lane: l[2h] (own)        odd lane: l[2h+1] of lane - 1
//   m[2h + 1] = even lane: l[2h] of lane + 1  odd lane: l[2h+1] (own)
// (DPP quad_perm(0,0,2,2) / (1,1,3,3) fetch the pair partner's register).
// The DPP moves carry no "old" operand (every lane of a quad_perm is
// written): a DPP move and a select per dword.  (update_dpp with an explicit
// old value of 0 cost a v_mov of that 0 as well: with the OOB change in the
// tile loads below, the loop went from ~98 to ~74 VALU instructions per tile,
// 0.364 -> 0.354 ms at C3, bit-identical.  Folding the DPP into the select
// (v_cndmask_b32_dpp, 58 per tile) measured no faster: the loop is not bound
// by VALU issue alone; profiles/r6/NOTES.md.)
__device__ __forceinline__ void cm_pair_operands(const h8_t* l, h8_t* m, bool odd)
{
    typedef unsigned u4_t __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const u4_t e = __builtin_bit_cast(u4_t, l[2 * h]), o = __builtin_bit_cast(u4_t, l[2 * h + 1]);
        u4_t m0, m1;
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const unsigned from_o = (unsigned)__builtin_amdgcn_mov_dpp((int)o[d], 0xA0, 0xF, 0xF, false);
            const unsigned from_e = (unsigned)__builtin_amdgcn_mov_dpp((int)e[d], 0xF5, 0xF, 0xF, false);
            m0[d] = odd ? from_o : e[d];
            m1[d] = odd ? o[d] : from_e;
        }
        m[2 * h] = __builtin_bit_cast(h8_t, m0);
        m[2 * h + 1] = __builtin_bit_cast(h8_t, m1);
    }
}

// per-edge prologue operands, loaded one edge ahead
struct CmEdgeIn {
    int e, ix, jx;
    float cx, cy;   // patch pixel (lane & 15)'s coordinates (x, y) when < 9 -- level scaling applied later
};

// The edge's slot, index and frame indices are wave-uniform: read through the
// scalar cache (constant address space: s_load), so the next edge's dependent
// index chain waits on lgkmcnt only.  As vector loads, the wait for the order
// entry before the ii / jj loads was a vmcnt(0) -- every edge drained the
// previous edge's epilogue stores before its own work could start.
typedef const __attribute__((address_space(4))) int cm_cint;
typedef const __attribute__((address_space(4))) int64_t cm_cint64;
__device__ __forceinline__ CmEdgeIn cm_load_edge(const CorrMfmaParams& p, int slot, int q16)
{
    CmEdgeIn in;
    slot = __builtin_amdgcn_readfirstlane(slot);
    in.e = p.order ? ((cm_cint*)p.order)[slot] : slot;
    in.ix = (int)((cm_cint64*)p.ii)[in.e];
    in.jx = (int)((cm_cint64*)p.jj)[in.e];
    const int q = q16 < cm::NP ? q16 : 0;
    const float* cb = p.coords + (int64_t)in.e * p.c_s[1] + (q / 3) * p.c_s[3] + (q % 3) * p.c_s[4];
    in.cx = cb[0];
    in.cy = cb[p.c_s[2]];
    return in;
}

// Per edge and level: the pixels the nine 8x8 windows need.  When the nine
// floors lie within 4 of each other ("fast") that is one box of at most 12x12
// pixels, enumerated row-major and visited 16 pixels per tile: every lane of
// every tile loads a box pixel (only the last tile has a tail), which keeps the
// vector-memory address work -- what bounds this kernel -- at the box's size.
// Each lane walks its pixel (box row, column) by increments.  Otherwise each
// patch pixel's own window is visited, two window rows (16 pixels) per tile.
// Either way the product of tile pixel n and patch pixel q lands at
// raw[level][q][16 tile + n]: four consecutive floats per lane.
struct CmLevel {
    const char* frame;    // this target frame's map (byte pointer), wave-uniform
    int64_t rowb;         // row stride in bytes
    int H, W, pixb, frameext;
    int fast, oy, ox, bw, npx, ntiles;
    int by, bx;           // per lane: box pixel (lane & 15) of the first tile (fast)
    int fy, fx;           // per lane: floors of patch pixel (lane & 15)
};

// One wave per edge, persistent over a contiguous per-XCD range of edge
// slots.  The next edge's indices and coordinates are in flight while the
// current edge runs; the tiles of both levels are one flat sequence whose A
// fragments are loaded four tiles ahead (a static register ring).  Products
// land in a per-wave LDS box [level][patch pixel][RS] (fp32), from which the
// bilinear epilogue reads each pixel's window and writes 256-byte coalesced rows.
// Tile loads read full 128-B lines: instruction ks gives lane (q16, kc) 16 B
// of the EVEN (ks = 0, 2) or ODD (ks = 1, 3) pixel of its lane pair, chunk
// 8 (ks >> 1) + 4 (q16 & 1) + kc of the pixel's 16 chunks -- eight pixels x 128 B
// per wave-instruction instead of sixteen pixels x 64 B, the fragment shape
// that costs the texture addresser twice the cycles (557 -> 388 us measured
// with the loads alone changed).  Two DPP quad permutations and a select per
// dword then rebuild the MFMA operand (lane (q16, kc): pixel q16, chunk
// 4 j + kc): an exchange between the lanes of each pair (cm_pair_operands).
__global__ __launch_bounds__(64 * cm::WAVES) void corr_mfma_kernel(CorrMfmaParams p)
{
    using namespace cm;
    __shared__ __attribute__((aligned(16))) float raw[WAVES][2 * RL];
    __shared__ float wts[WAVES][2][4][16];   // bilinear weights per level and patch pixel
    __shared__ int ebase[WAVES][2][16];      // window origin of each patch pixel inside its raw row
    __shared__ int estr[WAVES][2];           // raw row stride of the window (box width, or 8)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const CmRange rg = cm_range(p.E, wave);
    int slot = rg.slot;
    if (slot >= rg.end) return;   // the whole wave; nothing below synchronises across waves
    float* rw = raw[wave];
    const int q16 = lane & 15, kc = lane >> 4;
    const bool qv = q16 < NP;

    // epilogue: output t = lane + 64 i is (x offset, y offset, patch pixel) = ((t / 9) / 7, (t / 9) % 7, t % 9)
    int eq[7], ex[7], ey[7];
#pragma unroll
    for (int i = 0; i < 7; i++) {
        const int t = min(lane + 64 * i, DO * DO * NP - 1);
        const int pos = t / NP, q = t - pos * NP;
        const int bxo = pos / DO, ay = pos - bxo * DO;
        eq[i] = q;
        ex[i] = bxo;
        ey[i] = ay;
    }

    CmEdgeIn nin = cm_load_edge(p, slot, q16);
    for (; slot < rg.end; slot += rg.stride) {
        const CmEdgeIn in = nin;
        if (slot + rg.stride < rg.end) nin = cm_load_edge(p, slot + rg.stride, q16);
        const int e = __builtin_amdgcn_readfirstlane(in.e);
        const int ix = __builtin_amdgcn_readfirstlane(in.ix);
        const int jx = __builtin_amdgcn_readfirstlane(in.jx);
        const bool ix_ok = ix >= 0 && ix < p.N1;

        // ---- B fragments: patch pixel (lane & 15) x 8 channels of each 32-channel step
        h8_t bq[4];
        {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<half_t*>(p.gt + (ix_ok ? (int64_t)ix * NP * C : 0)), (short)0, ix_ok ? NP * C * 2 : 0,
                0x00020000);
            const unsigned voff = qv ? (unsigned)(q16 * C * 2 + 16 * kc) : OOB;
#pragma unroll
            for (int ks = 0; ks < 4; ks++)
                bq[ks] = __builtin_bit_cast(h8_t, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 64 * ks, 0, 0));
        }

        // ---- per level: scaled coordinates, floors, box, per-lane walk start
        cm_wave_fence();   // the previous edge's epilogue has read wts / raw / ebase
        CmLevel L0, L1;
#pragma unroll
        for (int l = 0; l < 2; l++) {
            CmLevel& L = l ? L1 : L0;
            const float x = in.cx / p.scale[l], y = in.cy / p.scale[l];
            L.fy = floor_to_int_sat(y);
            L.fx = floor_to_int_sat(x);
            int ymin = __builtin_amdgcn_readlane(L.fy, 0), ymax = ymin;
            int xmin = __builtin_amdgcn_readlane(L.fx, 0), xmax = xmin;
#pragma unroll
            for (int q = 1; q < NP; q++) {
                const int vy = __builtin_amdgcn_readlane(L.fy, q), vx = __builtin_amdgcn_readlane(L.fx, q);
                ymin = min(ymin, vy); ymax = max(ymax, vy);
                xmin = min(xmin, vx); xmax = max(xmax, vx);
            }
            const bool jok = jx >= 0 && jx < p.N2[l];
            L.frame = reinterpret_cast<const char*>(p.fmap[l] + (jok ? (int64_t)jx * p.f_s1[l] : 0));
            L.rowb = p.rowb[l];
            L.H = p.H2[l];
            L.W = p.W2[l];
            L.pixb = p.pixb[l];
            L.frameext = jok && ix_ok ? p.frameext[l] : 0;
            L.fast = ((int64_t)ymax - ymin) <= BOXMAX - D && ((int64_t)xmax - xmin) <= BOXMAX - D;
            L.oy = wrap_add(ymin, -R);
            L.ox = wrap_add(xmin, -R);
            L.bw = L.fast ? xmax - xmin + D : D;
            const int bh = L.fast ? ymax - ymin + D : D;
            L.npx = L.bw * bh;
            L.ntiles = L.fast ? (L.npx + 15) / 16 : NP * 4;
            L.by = q16 / L.bw;
            L.bx = q16 - L.by * L.bw;
            if (lane < NP) {
                const float dx = x - floorf(x), dy = y - floorf(y);
                wts[wave][l][0][lane] = (1.f - dx) * (1.f - dy);
                wts[wave][l][1][lane] = dx * (1.f - dy);
                wts[wave][l][2][lane] = (1.f - dx) * dy;
                wts[wave][l][3][lane] = dx * dy;
                // the window of pixel q starts at box (fy - ymin, fx - xmin); wide: its own 8 x 8
                ebase[wave][l][lane] = L.fast ? (L.fy - ymin) * L.bw + (L.fx - xmin) : 0;
            }
            if (lane == 0) estr[wave][l] = L.bw;
        }

        // ---- tiles of both levels: A = 16 box pixels (or two window rows), B = the patch.
        const int ntot = L0.ntiles + L1.ntiles;
        struct FCur {
            int lev, tl, ntl, fast, oy, ox, bw, npx, H, W, pixb, num;
            int64_t rowb;
            const char* frame;
            int by, bx, fy, fx;   // per lane
        };
        auto fstart = [&](const CmLevel& L, int lev) {
            FCur c;
            c.lev = lev;
            c.tl = 0;
            c.ntl = L.ntiles;
            c.fast = L.fast;
            c.oy = L.oy;
            c.ox = L.ox;
            c.bw = L.bw;
            c.npx = L.npx;
            c.H = L.H;
            c.W = L.W;
            c.pixb = L.pixb;
            c.num = L.frameext;
            c.rowb = L.rowb;
            c.frame = L.frame;
            c.by = L.by;
            c.bx = L.bx;
            c.fy = L.fy;
            c.fx = L.fx;
            return c;
        };
        FCur fc = fstart(L0, 0);
        auto fetch = [&](h8_t* a) {
            if (fc.tl == fc.ntl) {
                if (fc.lev == 0) {
                    fc = fstart(L1, 1);
                } else {   // past the last tile: nothing to read
                    fc.lev = 2;
                    fc.num = 0;
                    fc.ntl = 0x7fffffff;
                }
            }
            int gy, gx;
            bool inb;
            if (fc.fast) {
                gy = wrap_add(fc.oy, fc.by);
                gx = wrap_add(fc.ox, fc.bx);
                inb = 16 * fc.tl + q16 < fc.npx;
                // next tile: 16 pixels on (the box is at least 8 wide: at most two row wraps)
                fc.bx += 16;
                if (fc.bx >= fc.bw) { fc.bx -= fc.bw; fc.by++; }
                if (fc.bx >= fc.bw) { fc.bx -= fc.bw; fc.by++; }
            } else {
                const int qq = fc.tl >> 2, tt = fc.tl & 3;
                gy = wrap_add(__builtin_amdgcn_readlane(fc.fy, qq), 2 * tt + (q16 >> 3) - R);
                gx = wrap_add(__builtin_amdgcn_readlane(fc.fx, qq), (q16 & 7) - R);
                inb = true;
            }
            inb = inb && gy >= 0 && gy < fc.H && gx >= 0 && gx < fc.W;
            const int pix = inb ? gy * (int)fc.rowb + gx * fc.pixb : (int)OOB;   // this lane's pixel
            fc.tl++;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(fc.frame), (short)0, fc.num, 0x00020000);
            // full-line loads (see cm_pair_operands): the lane pair's even / odd
            // pixel, + the lane's 16-byte chunk.  An out-of-map pixel's OOB
            // (2^31) plus the chunk (< 256) stays past every descriptor's range
            // (frameext < 2^31 - 256, corr_mfma_setup), so it needs no select
            // of its own, and the 128-byte half goes to the immediate offset.
            const unsigned ch = 16u * (unsigned)((q16 & 1) * 4 + kc);
            const unsigned pe = (unsigned)__builtin_amdgcn_mov_dpp(pix, 0xA0, 0xF, 0xF, false) + ch;   // quad_perm(0,0,2,2)
            const unsigned po = (unsigned)__builtin_amdgcn_mov_dpp(pix, 0xF5, 0xF, 0xF, false) + ch;   // quad_perm(1,1,3,3)
#pragma unroll
            for (int ks = 0; ks < 4; ks++)
                a[ks] = __builtin_bit_cast(h8_t, __builtin_amdgcn_raw_buffer_load_b128(rs, ((ks & 1) ? po : pe) + 128u * (ks >> 1), 0, 0));
        };
        int clev = 0, ctl = 0, cntl = L0.ntiles;
        auto consume = [&](int t, const h8_t* a) {
            if (t >= ntot) return;
            f4m_t acc = {0.f, 0.f, 0.f, 0.f};
            h8_t m[4];
            cm_pair_operands(a, m, (q16 & 1) != 0);
#pragma unroll
            for (int ks = 0; ks < 4; ks++) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(m[ks], bq[ks], acc, 0, 0, 0);
            // acc[r] = tile pixel 4 kc + r . patch pixel (lane & 15)
            if (ctl == cntl) {
                clev = 1;
                ctl = 0;
                cntl = L1.ntiles;
            }
            const bool fast = clev ? L1.fast : L0.fast;
            // wide path: tile ctl holds rows 2 (ctl & 3) .. + 1 of pixel ctl / 4's window only
            if (qv && (fast || q16 == (ctl >> 2))) {
                const int n = fast ? 16 * ctl : 16 * (ctl & 3);
                *(f4m_t*)(rw + clev * RL + q16 * RS + n + 4 * kc) = acc;
            }
            ctl++;
        };
        // issue order must match consume order, or the wait at the loop head
        // (merged over the entry and the back edge) drains the whole ring
        h8_t b0[4], b1[4], b2[4], b3[4];
        fetch(b0);
        __builtin_amdgcn_sched_barrier(0);
        fetch(b1);
        __builtin_amdgcn_sched_barrier(0);
        fetch(b2);
        __builtin_amdgcn_sched_barrier(0);
        fetch(b3);
        __builtin_amdgcn_sched_barrier(0);
        for (int t = 0; t < ntot; t += 4) {
            consume(t, b0);
            fetch(b0);
            consume(t + 1, b1);
            fetch(b1);
            consume(t + 2, b2);
            fetch(b2);
            consume(t + 3, b3);
            fetch(b3);
        }
        cm_wave_fence();

        // ---- bilinear 8x8 -> 7x7 per pixel and level (fp32), stacked row [x][y][P][P][level]
        half_t* orow = p.out + (int64_t)e * p.o_e;
        const int st0 = estr[wave][0], st1 = estr[wave][1];
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const int t = lane + 64 * i;
            if (t < DO * DO * NP) {
                const int q = eq[i];
                float v[2];
#pragma unroll
                for (int lev = 0; lev < 2; lev++) {
                    const int st = lev ? st1 : st0;
                    const float* r0 = rw + lev * RL + q * RS + ebase[wave][lev][q] + ey[i] * st + ex[i];
                    v[lev] = cm_bilinear(wts[wave][lev][0][q], wts[wave][lev][1][q], wts[wave][lev][2][q],
                                         wts[wave][lev][3][q], r0[0], r0[1], r0[st], r0[st + 1]);
                }
                *(half2_t*)(orow + 2 * t) = half2_t{(half_t)v[0], (half_t)v[1]};
            }
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

namespace dpvo {

int corr_mfma_setup(CorrMfmaParams& p, const void* table, int64_t num_patches, const void* const* fmaps,
                    const int64_t* fmap_sizes, const int64_t* fmap_strides, const float* level_scale,
                    const float* coords, const int64_t* coords_size, const int64_t* coords_stride, const int64_t* ii,
                    const int64_t* jj, void* corr, int64_t edge_stride, const int* order)
{
    DPVO_CHECK_ARG(coords_size[0] == 1 && coords_size[2] == 2 && coords_size[3] == 3 && coords_size[4] == 3,
                   "coords must be [1][E][2][3][3]");
    DPVO_CHECK_ARG(edge_stride == 0 || edge_stride >= 882, "edge_stride smaller than one edge's 882 features");
    const int64_t E = coords_size[1];
    DPVO_CHECK_ARG(E < 0x7fffffff && num_patches < 0x7fffffff, "too many edges / patches");
    p = CorrMfmaParams{};
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
        p.N2[l] = (int)fs[1];
        p.H2[l] = (int)fs[3];
        p.W2[l] = (int)fs[4];
        // buffer offsets are 32-bit with OOB = 2^31 as "nothing": every pixel of a frame must lie below it
        const int64_t rowext = fs[4] > 0 ? ((fs[4] - 1) * ft[4] + cm::C) * 2 : 0;
        const int64_t frameext = fs[3] > 0 && fs[4] > 0 ? (fs[3] - 1) * ft[3] * 2 + rowext : 0;
        DPVO_CHECK_ARG(frameext < (int64_t)cm::OOB - 256 && ft[3] * 2 < (int64_t)cm::OOB,
                       "one frame of a feature map must span less than 2 GiB");
        p.rowb[l] = ft[3] * 2;
        p.pixb[l] = (int)(ft[4] * 2);
        p.rowext[l] = (int)rowext;
        p.frameext[l] = (int)frameext;
        p.scale[l] = level_scale[l];
    }
    DPVO_CHECK_ARG(reinterpret_cast<uintptr_t>(table) % 16 == 0, "table must be 16-byte aligned");
    p.out = (half_t*)corr;
    p.o_e = edge_stride ? edge_stride : 882;
    p.order = order;
    DPVO_CHECK_ARG(reinterpret_cast<uintptr_t>(corr) % 4 == 0 && p.o_e % 2 == 0, "corr rows must be 4-byte aligned");
    return 0;
}

int corr_mfma_launch(const CorrMfmaParams& p, hipStream_t s)
{
    if (p.E == 0) return 0;
    // persistent: a few workgroups per CU, each wave walking a grid-stride range of edges
    // (a multiple of 8 once there are 8 workgroups' worth of edges: see cm_range)
    int64_t g = std::min<int64_t>((p.E + cm::WAVES - 1) / cm::WAVES, 256 * 3);   // LDS and VGPRs: 3 per CU
    if (g > 8) g &= ~int64_t(7);
    hipLaunchKernelGGL(corr_mfma_kernel, dim3((unsigned)g), dim3(64 * cm::WAVES), 0, s, p);
    DPVO_CHECK_LAUNCH();
    return 0;
}

}  // namespace dpvo

extern "C" int dpvo_corr_pyramid_mfma(const void* table, int64_t num_patches, const void* const* fmaps,
                                      const int64_t* fmap_sizes, const int64_t* fmap_strides,
                                      const float* level_scale, const float* coords, const int64_t* coords_size,
                                      const int64_t* coords_stride, const int64_t* ii, const int64_t* jj, void* corr,
                                      int64_t edge_stride, const int* order, void* stream)
{
    CorrMfmaParams p;
    if (corr_mfma_setup(p, table, num_patches, fmaps, fmap_sizes, fmap_strides, level_scale, coords, coords_size,
                        coords_stride, ii, jj, corr, edge_stride, order))
        return -1;
    return corr_mfma_launch(p, as_stream(stream));
}

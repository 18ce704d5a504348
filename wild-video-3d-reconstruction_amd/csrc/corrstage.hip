// corrstage.hip -- DPVO's two-level patch correlation on the matrix cores with
// the target frames' windows staged in LDS.
//
// Same quantity and the same bits as corr_mfma_kernel (corrmfma.hip; reference
// dpvo/dpvo.py:326-333 -> correlation_kernel.cu:83-135 + the ATen bilinear
// epilogue :221-232): per edge and level the nine patch pixels' 128-channel
// features against the box of pixels covering their nine 8x8 windows, on
// v_mfma_f32_16x16x32_f16 in the same channel order, then the same fp32
// bilinear epilogue.  What changes is where the box pixels come from.
//
// corr_mfma_kernel reads every edge's boxes (~100 level-1 and ~70 level-2
// pixels of 256 B) through the vector-memory address path, and that path
// bounds it: ~2,700 edges per update read windows of each target frame, so
// every level-2 pixel is addressed ~250 times.  Here the edges are binned by
// (target frame, 8x8-pixel cell of the level-1 map) on the device, and one
// workgroup per CU walks a contiguous range of bins: per bin it stages the
// cell's 17x17-pixel level-1 region and 11x11-pixel level-2 region in LDS
// once (contiguous 1 KB loads per wave instruction) and every edge of the bin
// reads its MFMA operands from there.  The staging of the next bin is issued
// into registers while the current bin's edges compute.
//
// An edge is binned only when both of its boxes lie inside its cell's
// regions (the box is at most 12x12: the "fast" case of corr_mfma_kernel)
// and its indices and coordinates are valid and finite; the rest (wide
// patches, edges far outside the map, bad indices) are the fallback bin,
// which corr_mfma_kernel processes after the staged launch.  Either way each
// edge's output row is computed by the same arithmetic, so the result does
// not depend on the binning (tests/test_gpu_corr_stage.py checks bit
// identity with corr_mfma_kernel).
#include <algorithm>
#include <cmath>

#include "corrmfma.hpp"

namespace dpvo {

constexpr int CS_MAX_GRID = 4096;
constexpr int CS_MAX_BINS = 1 << 15;   // (frame, cell) bins + 1: the scan's register budget
constexpr int CS_SCAN_PER = CS_MAX_BINS / 1024;

namespace cs {
constexpr int WAVES = 8, THREADS = 64 * WAVES;
constexpr int CELL = 8;                        // level-1 cell pitch (pixels)
constexpr int R1 = 17, O1 = -4;                // level-1 region of cell c: [8c - 4, 8c + 12]
constexpr int R2 = 11, O2 = -4;                // level-2 region of cell c: [2c - 4, 2c + 6]
constexpr int NPX1 = R1 * R1, NPX2 = R2 * R2;  // 289, 121 pixels
constexpr int PIXB = cm::C * 2 + 16;           // 256 B per pixel + 16: pixel p's 64-B quarters start
                                               // 4 banks after pixel p - 1's, so the 16 pixels of an MFMA
                                               // tile reading one quarter spread over the banks (no swizzle)
constexpr int CH1 = (NPX1 * 16 + 63) / 64 * 64;   // level-1 16-byte chunks, padded to whole wave instructions
constexpr int CH2 = NPX2 * 16;
constexpr int LOADS = (CH1 + CH2 + THREADS - 1) / THREADS;   // staging loads per lane
constexpr int REG1_OFF = 0;
constexpr int REG2_OFF = NPX1 * PIXB;                          // 78,608
constexpr int RAW_OFF = REG2_OFF + NPX2 * PIXB;                // 111,520
constexpr int REC = 32;                                        // ints per binned edge record (128 B)
constexpr int RAW_W = cm::NP * cm::RS * 4;                     // 5,328 B per wave (one level at a time)
constexpr int WTS_OFF = RAW_OFF + WAVES * RAW_W;
constexpr int EB_OFF = WTS_OFF + WAVES * 4 * 16 * 4;
constexpr int LDS = EB_OFF + WAVES * 16 * 4;
static_assert(LDS <= 163840, "LDS budget of one workgroup per CU");
static_assert(CH1 % 64 == 0, "every staging wave-instruction reads one level");
}  // namespace cs

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f4m_t __attribute__((ext_vector_type(4)));
typedef unsigned u4_t __attribute__((ext_vector_type(4)));

// Bins: frame * ncell + (cy + 1) * ncx + (cx + 1) for level-1 cells cy in
// [-1, ncy - 1), cx in [-1, ncx - 1); bin nb - 1 is the fallback.
struct CsGeom {
    int ncy, ncx, ncell, nb;
    float iscale[2];   // 1 / level scale
    int pow2s;         // both scales powers of two: x * iscale == x / scale exactly
};

__device__ __forceinline__ int cs_floor8(int v) { return v >> 3; }   // floor(v / 8), v small

// An edge's floors at both levels (the staged kernel's boxes) and its bin.
struct CsBox {
    int y0[2], x0[2], y1[2], x1[2];
    int bin;
};
__device__ __forceinline__ CsBox cs_edge_box(const CorrMfmaParams& p, const CsGeom& g, int e)
{
    CsBox bx;
    bx.bin = g.nb - 1;
    const int64_t ix = p.ii[e], jx = p.jj[e];
    if (!(ix >= 0 && ix < p.N1 && jx >= 0 && jx < p.N2[0] && jx < p.N2[1])) return bx;
#pragma unroll
    for (int l = 0; l < 2; l++) {
        bx.y0[l] = bx.x0[l] = 0x7fffffff;
        bx.y1[l] = bx.x1[l] = -0x7fffffff;
    }
    bool fin = true;
    const float* cb = p.coords + (int64_t)e * p.c_s[1];
#pragma unroll
    for (int q = 0; q < cm::NP; q++) {
        const float* c = cb + (q / 3) * p.c_s[3] + (q % 3) * p.c_s[4];
        const float cx = c[0], cy = c[p.c_s[2]];
        // finite and well inside int range (the floors below are the kernel's own)
        fin = fin && fabsf(cx) < 1e6f && fabsf(cy) < 1e6f;
#pragma unroll
        for (int l = 0; l < 2; l++) {
            // (x * 2^-k == x / 2^k exactly)
            const float sy = g.pow2s ? cy * g.iscale[l] : cy / p.scale[l];
            const float sx = g.pow2s ? cx * g.iscale[l] : cx / p.scale[l];
            const int fy = floor_to_int_sat(sy), fx = floor_to_int_sat(sx);
            bx.y0[l] = min(bx.y0[l], fy); bx.y1[l] = max(bx.y1[l], fy);
            bx.x0[l] = min(bx.x0[l], fx); bx.x1[l] = max(bx.x1[l], fx);
        }
    }
    if (!fin || bx.y1[0] - bx.y0[0] > cm::BOXMAX - cm::D || bx.x1[0] - bx.x0[0] > cm::BOXMAX - cm::D) return bx;
    // the cell whose region's top-left corner is the last one at or above the
    // box's: region [8c - 4, 8c + 12] holds rows fy0 - 3 .. fy1 + 4 iff fy1 <= 8c + 8
    const int cy = cs_floor8(bx.y0[0] + 1), cx = cs_floor8(bx.x0[0] + 1);
    bool ok = cy >= -1 && cy < g.ncy - 1 && cx >= -1 && cx < g.ncx - 1;
    ok = ok && bx.y1[0] <= cs::CELL * cy + 8 && bx.x1[0] <= cs::CELL * cx + 8;
    // level 2: box rows gy0 - 3 .. gy1 + 4 inside [2c - 4, 2c + 6]
    ok = ok && bx.y0[1] >= 2 * cy - 1 && bx.y1[1] <= 2 * cy + 2 && bx.x0[1] >= 2 * cx - 1 && bx.x1[1] <= 2 * cx + 2;
    if (ok) bx.bin = (int)jx * g.ncell + (cy + 1) * g.ncx + (cx + 1);
    return bx;
}

// per edge: its bin and the bin's count.  The fallback bin collects a few
// percent of all edges: its count is added once per wave (one address hit by
// every such edge serialised the atomics: 38 us at C3)
__global__ __launch_bounds__(256) void cs_bin_kernel(CorrMfmaParams p, CsGeom g, int* __restrict__ bin,
                                                     int* __restrict__ count)
{
    const int e = blockIdx.x * 256 + threadIdx.x;
    const bool valid = e < p.E;
    const int b = valid ? cs_edge_box(p, g, e).bin : -1;
    if (valid) bin[e] = b;
    const bool fb = b == g.nb - 1;
    const uint64_t m = __ballot(fb);
    if (fb) {
        if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)m) - 1) atomicAdd(&count[b], __popcll(m));
    } else if (valid) {
        atomicAdd(&count[b], 1);
    }
}

// The staged kernel's cost of a task of c edges, in units of ~5k wave cycles
// (in-kernel stamps, DPVO_STAMPS): staging + barriers ~3, each pass of the
// eight waves over its edges ~2.
__device__ __forceinline__ int cs_task_cost(int c) { return 3 + 2 * ((c + cs::WAVES - 1) / cs::WAVES); }

// One workgroup: exclusive offsets of the bins (offs[nb] = E), the counts
// turned into scatter cursors, the non-empty staged bins as a task list
// (task_bin, task_off[ntask + 1]: task_off[ntask] = the fallback bin's start),
// and the tasks split over the staged kernel's G workgroups by cost: workgroup
// lw runs the whole tasks wg_first[lw] .. wg_first[lw + 1] - 1, those whose
// cost prefix c0 lies in [C lw / G, C (lw + 1) / G) -- wg_first[lw] is the
// number of tasks with floor(c0 G / C) < lw.
__global__ __launch_bounds__(1024) void cs_scan_kernel(CsGeom g, int G, int* __restrict__ count,
                                                       int* __restrict__ offs, int* __restrict__ task_bin,
                                                       int* __restrict__ task_off, int* __restrict__ ntask,
                                                       int* __restrict__ wg_first)
{
    __shared__ int wsum[16][3];
    __shared__ int hist[CS_MAX_GRID];
    const int nb = g.nb, t = threadIdx.x, lane = t & 63, w = t >> 6;
    // bins per thread: CS_SCAN_PER at most (the counts of a thread's bins are
    // loaded together, one round trip; CS_MAX_BINS / 1024 bins at most)
    const int per = (nb + 1023) / 1024;
    const int b0 = min(nb, t * per), b1 = min(nb, b0 + per);
    for (int k = t; k < G; k += 1024) hist[k] = 0;
    int cnt[CS_SCAN_PER];
#pragma unroll
    for (int j = 0; j < CS_SCAN_PER; j++) cnt[j] = b0 + j < b1 ? count[b0 + j] : 0;
    int s = 0, ne = 0, cs_ = 0;
#pragma unroll
    for (int j = 0; j < CS_SCAN_PER; j++) {
        const int c = cnt[j];
        s += c;
        if (c > 0 && b0 + j < nb - 1) {
            ne++;
            cs_ += cs_task_cost(c);
        }
    }
    // inclusive wave scans of (edges, tasks, cost)
    int is = s, in = ne, ic = cs_;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int ys = __shfl_up(is, d, 64), yn = __shfl_up(in, d, 64), yc = __shfl_up(ic, d, 64);
        if (lane >= d) { is += ys; in += yn; ic += yc; }
    }
    if (lane == 63) { wsum[w][0] = is; wsum[w][1] = in; wsum[w][2] = ic; }
    __syncthreads();
    int bs = 0, bn = 0, bc = 0, tot = 0, ctot = 0;
    for (int k = 0; k < 16; k++) {
        if (k < w) { bs += wsum[k][0]; bn += wsum[k][1]; bc += wsum[k][2]; }
        tot += wsum[k][1];
        ctot += wsum[k][2];
    }
    int o = bs + is - s, tk = bn + in - ne, c0 = bc + ic - cs_;
#pragma unroll
    for (int j = 0; j < CS_SCAN_PER; j++) {
        const int b = b0 + j;
        if (b >= b1) break;
        const int c = cnt[j];
        offs[b] = o;
        count[b] = o;   // the scatter's cursor
        if (b == nb - 1) {   // the fallback bin closes the task list
            task_off[tot] = o;
            *ntask = tot;
            offs[nb] = o + c;
        } else if (c > 0) {
            task_bin[tk] = b;
            task_off[tk] = o;
            atomicAdd(&hist[(int)((int64_t)c0 * G / ctot)], 1);
            c0 += cs_task_cost(c);
            tk++;
        }
        o += c;
    }
    __syncthreads();
    // wg_first[lw] = hist[0] + .. + hist[lw - 1]: one wave scans it in 64-wide chunks
    if (w == 0) {
        int run = 0;
        for (int k0 = 0; k0 < G; k0 += 64) {
            const int v = k0 + lane < G ? hist[k0 + lane] : 0;
            int x = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int y = __shfl_up(x, d, 64);
                if (lane >= d) x += y;
            }
            if (k0 + lane < G) wg_first[k0 + lane] = run + x - v;
            run += __shfl(x, 63, 64);
        }
        if (lane == 0) wg_first[G] = tot;
    }
}

// order[slot] = e, and the staged kernel's per-slot record (cs::REC ints):
// e, ii, both levels' box corner and size, the 18 coordinates -- scalar loads
// there (lgkmcnt), outside the vmcnt queue its region prefetch occupies, with
// no dependent load chain.  Fallback slots: one returning atomic per wave.
__global__ __launch_bounds__(256) void cs_scatter_kernel(CorrMfmaParams p, CsGeom g, const int* __restrict__ bin,
                                                         int* __restrict__ cursor, int* __restrict__ order,
                                                         int* __restrict__ rec)
{
    const int e = blockIdx.x * 256 + threadIdx.x;
    const bool valid = e < p.E;
    const int b = valid ? bin[e] : -1;
    const bool fb = b == g.nb - 1;
    const uint64_t m = __ballot(fb);
    int pos = 0;
    if (m) {
        const int lead = __ffsll((unsigned long long)m) - 1;
        int base = 0;
        if ((int)(threadIdx.x & 63) == lead) base = atomicAdd(&cursor[g.nb - 1], __popcll(m));
        base = __shfl(base, lead, 64);
        const int below = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
        pos = base + below;
    }
    if (!valid) return;
    if (!fb) pos = atomicAdd(&cursor[b], 1);
    order[pos] = e;
    if (fb) return;
    const CsBox bx = cs_edge_box(p, g, e);
    int* r = rec + (int64_t)pos * cs::REC;
    typedef int i4_t __attribute__((ext_vector_type(4)));
    *(i4_t*)(r + 0) = i4_t{e, (int)p.ii[e], bx.y0[0], bx.x0[0]};
    *(i4_t*)(r + 4) = i4_t{bx.x1[0] - bx.x0[0] + cm::D, bx.y1[0] - bx.y0[0] + cm::D, bx.y0[1], bx.x0[1]};
    *(i4_t*)(r + 8) = i4_t{bx.x1[1] - bx.x0[1] + cm::D, bx.y1[1] - bx.y0[1] + cm::D, 0, 0};
    const float* cb = p.coords + (int64_t)e * 18;   // contiguous (checked on the host)
#pragma unroll
    for (int q = 0; q < 18; q++) r[14 + q] = __float_as_int(cb[q]);
}

// a wave-uniform zero the compiler cannot see through: address arithmetic
// that depends on it is recomputed where it is used instead of being hoisted
// out of the task loop into ~100 long-lived registers
__device__ __forceinline__ int cs_opaque_zero()
{
    int z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    return z;
}

__device__ __forceinline__ void cs_wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// LDS byte address of 16-byte chunk cc of region pixel px (padded pixel stride)
__device__ __forceinline__ int cs_chunk(int base, int px, int cc) { return base + px * cs::PIXB + (cc << 4); }

#ifdef DPVO_STAMPS
// Diagnostic build only (never the product library): per-wave cycle sums of
// the staged kernel's phases, s_memtime stamps.  dpvo_cs_stamps[block][wave][seg]:
// 0 barriers + region write, 1 edge inputs + prefetch issue, 2 level 2, 3 level 1,
// 4 output stores, 5 whole kernel, 6 tasks, 7 edges; per level (summed): 8 setup,
// 9 tile loop, 10 epilogue, 11 tiles
__device__ unsigned long long dpvo_cs_stamps[4096 * cs::WAVES * 16];
#define CS_STAMP(v)                                                                            \
    unsigned long long v;                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");                  \
    __builtin_amdgcn_sched_barrier(0);
#define CS_ACC(seg, a, b) cst[seg] += (b) - (a);
#else
#define CS_STAMP(v)
#define CS_ACC(seg, a, b)
#endif

struct CsEdge {
    int e;
    int y0[2], x0[2], bw[2], bh[2];   // per level: the box's first pixel (floors' minimum) and size
    float cx, cy;                     // patch pixel (lane & 15)'s coordinates when < 9
    h8_t bq[4];                       // B fragments: patch pixel (lane & 15) x 8 channels of each 32-channel step
};

// One workgroup per CU, 8 waves.  Workgroup b (logical index: each XCD owns
// one contiguous eighth) takes an equal share of the binned edge slots and
// walks the bins (tasks) that share covers.  Per task: stage the regions,
// then each wave takes the task's edges wave, wave + 8, ...; per edge, level
// 2 then level 1 (one per-wave product box, reused), exactly the tile / MFMA /
// bilinear arithmetic of corr_mfma_kernel's fast path.
__global__ __launch_bounds__(cs::THREADS, 1) void corr_stage_kernel(CorrMfmaParams p, CsGeom g,
                                                                    const int* __restrict__ rec,
                                                                    const int* __restrict__ task_bin,
                                                                    const int* __restrict__ task_off,
                                                                    const int* __restrict__ ntask_p,
                                                                    const int* __restrict__ wg_first)
{
    using namespace cm;
    __shared__ __attribute__((aligned(16))) char smem[cs::LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int G = gridDim.x, bid = blockIdx.x;
    const int lw = (G >= 8 && (G & 7) == 0) ? (bid & 7) * (G >> 3) + (bid >> 3) : bid;
    const int ntask = *ntask_p;
    if (ntask == 0) return;
    int task = wg_first[lw];              // this workgroup's whole tasks (cs_scan_kernel: split by cost)
    const int task_end = wg_first[lw + 1];
    if (task >= task_end) return;         // the whole workgroup
#ifdef DPVO_STAMPS
    unsigned long long cst[16] = {};
#endif
    const bool pow2s = g.pow2s != 0;
    const float iscale[2] = {g.iscale[0], g.iscale[1]};
    float* rw = reinterpret_cast<float*>(smem + cs::RAW_OFF + wave * cs::RAW_W);
    float* wts = reinterpret_cast<float*>(smem + cs::WTS_OFF) + wave * 64;     // [16][4]: patch pixel's 4 weights
    int* ebase = reinterpret_cast<int*>(smem + cs::EB_OFF) + wave * 16;        // [16]
    const int q16 = lane & 15, kc = lane >> 4;
    const bool qv = q16 < NP;


    // ---- staging: this lane's chunks of the two regions, in registers
    u4_t st[cs::LOADS];
    auto region_of = [&](int bin, int& frame, int& oy1, int& ox1, int& oy2, int& ox2) __attribute__((always_inline)) {
        frame = bin / g.ncell;
        const int cell = bin - frame * g.ncell;
        const int cy = cell / g.ncx - 1, cx = cell - (cy + 1) * g.ncx - 1;
        oy1 = cs::CELL * cy + cs::O1;
        ox1 = cs::CELL * cx + cs::O1;
        oy2 = 2 * cy + cs::O2;
        ox2 = 2 * cx + cs::O2;
    };
    // the maps' geometry as plain scalars (indexing p's arrays by a runtime
    // level became a serialised kernel-argument load per staging load)
    const int H_0 = p.H2[0], H_1 = p.H2[1], W_0 = p.W2[0], W_1 = p.W2[1];
    const int rb_0 = (int)p.rowb[0], rb_1 = (int)p.rowb[1], pb_0 = p.pixb[0], pb_1 = p.pixb[1];
    // (straight-line: one load per j whatever its level -- branches between the
    // loads made the compiler wait for each before issuing the next)
    auto stage_issue = [&](int bin, bool on) __attribute__((always_inline)) {
        int frame, oy1, ox1, oy2, ox2;
        region_of(bin, frame, oy1, ox1, oy2, ox2);
        const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<half_t*>(p.fmap[0] + (int64_t)frame * p.f_s1[0]), (short)0, p.frameext[0], 0x00020000);
        const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<half_t*>(p.fmap[1] + (int64_t)frame * p.f_s1[1]), (short)0, p.frameext[1], 0x00020000);
        const int w64 = 64 * wave + cs_opaque_zero();
#pragma unroll
        for (int j = 0; j < cs::LOADS; j++) {
            const int kb = cs::THREADS * j + w64;   // wave-uniform: which level this instruction reads
            const bool l2 = kb >= cs::CH1;
            const int k = (l2 ? kb - cs::CH1 : kb) + lane, px = k >> 4, cc = k & 15;
            const int ry = l2 ? px / cs::R2 : px / cs::R1;
            const int rx = px - ry * (l2 ? cs::R2 : cs::R1);
            const int gy = (l2 ? oy2 : oy1) + ry, gx = (l2 ? ox2 : ox1) + rx;
            const bool ok = on && px < (l2 ? cs::NPX2 : cs::NPX1) && gy >= 0 && gy < (l2 ? H_1 : H_0) && gx >= 0 &&
                            gx < (l2 ? W_1 : W_0);
            const unsigned o = (unsigned)(gy * (l2 ? rb_1 : rb_0) + gx * (l2 ? pb_1 : pb_0) + 16 * cc);
            st[j] = __builtin_bit_cast(u4_t, __builtin_amdgcn_raw_buffer_load_b128(l2 ? r2 : r1, ok ? o : OOB, 0, 0));
        }
    };
    auto stage_write = [&]() __attribute__((always_inline)) {
        const int w64 = 64 * wave + cs_opaque_zero();
#pragma unroll
        for (int j = 0; j < cs::LOADS; j++) {
            const int kb = cs::THREADS * j + w64;
            const bool l2 = kb >= cs::CH1;
            const int k = (l2 ? kb - cs::CH1 : kb) + lane, px = k >> 4, cc = k & 15;
            if (px < (l2 ? cs::NPX2 : cs::NPX1))
                *(u4_t*)(smem + cs_chunk(l2 ? cs::REG2_OFF : cs::REG1_OFF, px, cc)) = st[j];
        }
    };
    // The edge records (cs_scatter_kernel) of a wave's two edges of a task sit
    // in one VGPR: lanes 0-31 hold record A's 32 ints, lanes 32-63 record B's.
    // They are loaded right behind the region prefetch of the task before, so
    // they have landed when that task's staging has (no wait of their own).
    auto load_recs = [&](int slot_a, int slot_b) __attribute__((always_inline)) -> int {
        const int slot = lane < 32 ? slot_a : slot_b;
        return rec[(int64_t)slot * cs::REC + (lane & 31)];
    };
    auto take_edge = [&](int recv, int half) __attribute__((always_inline)) {
        CsEdge in;
        const int b = 32 * half;
        in.e = __builtin_amdgcn_readlane(recv, b + 0);
        const int ix = __builtin_amdgcn_readlane(recv, b + 1);
#pragma unroll
        for (int l = 0; l < 2; l++) {
            in.y0[l] = __builtin_amdgcn_readlane(recv, b + 2 + 4 * l);
            in.x0[l] = __builtin_amdgcn_readlane(recv, b + 3 + 4 * l);
            in.bw[l] = __builtin_amdgcn_readlane(recv, b + 4 + 4 * l);
            in.bh[l] = __builtin_amdgcn_readlane(recv, b + 5 + 4 * l);
        }
        const int q = qv ? q16 : 0;
        in.cx = __int_as_float(__shfl(recv, b + 14 + q, 64));
        in.cy = __int_as_float(__shfl(recv, b + 23 + q, 64));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<half_t*>(p.gt + (int64_t)ix * NP * C), (short)0, NP * C * 2, 0x00020000);
        const unsigned voff = qv ? (unsigned)(q16 * C * 2 + 16 * kc) : OOB;
#pragma unroll
        for (int ks = 0; ks < 4; ks++)
            in.bq[ks] = __builtin_bit_cast(h8_t, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 64 * ks, 0, 0));
        return in;
    };

    // one level of one edge: tiles from the LDS region -> product box -> 7 bilinear outputs per lane
    auto level = [&](const CsEdge& in, int l, int reg_off, int RW, int oyl, int oxl, float* v) __attribute__((always_inline)) {
        CS_STAMP(l0)
        // (x * 2^-k == x / 2^k exactly: the host passes 1 / scale only for powers of two)
        const float x = pow2s ? in.cx * iscale[l] : in.cx / p.scale[l];
        const float y = pow2s ? in.cy * iscale[l] : in.cy / p.scale[l];
        const int fy = floor_to_int_sat(y), fx = floor_to_int_sat(x);
        const int ymin = in.y0[l], xmin = in.x0[l], bw = in.bw[l], bh = in.bh[l];
        const int npx = bw * bh, ntiles = (npx + 15) >> 4;
        // the box's origin (ymin - R, xmin - R) in region coordinates
        const int boy = ymin - R - oyl, box = xmin - R - oxl;
        cs_wave_fence();   // the previous level's epilogue has read wts / raw / ebase
        if (lane < NP) {
            const float dx = x - floorf(x), dy = y - floorf(y);
            *(f4m_t*)(wts + 4 * lane) = f4m_t{(1.f - dx) * (1.f - dy), dx * (1.f - dy), (1.f - dx) * dy, dx * dy};
            // the window of pixel q starts at box (fy - ymin, fx - xmin)
            ebase[lane] = (fy - ymin) * bw + (fx - xmin);
        }
        // lane's box pixel 16 t + q16 as a region pixel, walked by increments
        // (16 pixels on = one or two box-row wraps: the box is 8 .. 12 wide)
        int bx = q16 - (q16 >= bw ? bw : 0);
        int px = (boy + (q16 >= bw ? 1 : 0)) * RW + box + bx;
        const int pmax = RW * RW - 1;
        const int wrap = RW - bw;
        auto tile_load = [&](h8_t* a) __attribute__((always_inline)) {
            const char* src = smem + reg_off + min(px, pmax) * cs::PIXB + 16 * kc;
#pragma unroll
            for (int ks = 0; ks < 4; ks++) a[ks] = *(const h8_t*)(src + 64 * ks);
            bx += 16;
            px += 16;
            if (bx >= bw) { bx -= bw; px += wrap; }
            if (bx >= bw) { bx -= bw; px += wrap; }
        };
        auto tile_mma = [&](const h8_t* a, int t) __attribute__((always_inline)) {
            f4m_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 4; ks++) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ks], in.bq[ks], acc, 0, 0, 0);
            // acc[r] = tile pixel 4 kc + r . patch pixel (lane & 15)
            if (qv) *(f4m_t*)(rw + q16 * RS + 16 * t + 4 * kc) = acc;
        };
        CS_STAMP(l1)
        h8_t a0[4], a1[4];
        tile_load(a0);
        for (int t = 0; t < ntiles; t += 2) {
            if (t + 1 < ntiles) tile_load(a1);
            tile_mma(a0, t);
            if (t + 1 < ntiles) {
                if (t + 2 < ntiles) tile_load(a0);
                tile_mma(a1, t + 1);
            }
        }
        cs_wave_fence();
        CS_STAMP(l2)
        // bilinear 8x8 -> 7x7 per patch pixel (fp32); output t = lane + 64 i is
        // (x offset, y offset, patch pixel) = ((t / 9) / 7, (t / 9) % 7, t % 9).
        // In three batches (window origins, then all weights and products, then
        // the arithmetic) so the LDS reads overlap instead of paying two
        // dependent round trips per output.
        int qi[7], off[7];
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const int t = min(lane + 64 * i, DO * DO * NP - 1);
            const int pos = t / NP, q = t - pos * NP;
            const int exi = pos / DO, eyi = pos - exi * DO;
            qi[i] = q;
            off[i] = q * RS + eyi * bw + exi + ebase[q];
        }
        float w[7][4], r[7][4];
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const float* r0 = rw + off[i];
            r[i][0] = r0[0];
            r[i][1] = r0[1];
            r[i][2] = r0[bw];
            r[i][3] = r0[bw + 1];
            const f4m_t wq = *(const f4m_t*)(wts + 4 * qi[i]);
#pragma unroll
            for (int k = 0; k < 4; k++) w[i][k] = wq[k];
        }
#pragma unroll
        for (int i = 0; i < 7; i++) v[i] = cm_bilinear(w[i][0], w[i][1], w[i][2], w[i][3], r[i][0], r[i][1], r[i][2], r[i][3]);
#ifdef DPVO_STAMPS
        asm volatile("" ::"v"(v[0]), "v"(v[6]));
        CS_STAMP(l3)
        CS_ACC(8, l0, l1) CS_ACC(9, l1, l2) CS_ACC(10, l2, l3)
        cst[11] += ntiles;
#endif
    };

    CS_STAMP(k0)
    int bin = task_bin[task];
    stage_issue(bin, true);
    int recs;
    {
        const int seg0 = task_off[task], seg1 = task_off[task + 1];
        recs = load_recs(min(seg0 + wave, seg1 - 1), min(seg0 + wave + cs::WAVES, seg1 - 1));
    }
    for (;;) {
        const int seg0 = task_off[task], seg1 = task_off[task + 1];
        int frame, oy1, ox1, oy2, ox2;
        region_of(bin, frame, oy1, ox1, oy2, ox2);
        (void)frame;
        CS_STAMP(a0)
        __syncthreads();   // every wave is done with the previous task's regions
        stage_write();
        __syncthreads();
        CS_STAMP(a1)
        CS_ACC(0, a0, a1)
#ifdef DPVO_STAMPS
        cst[6]++;
#endif
        const bool more = task + 1 < task_end;
        const int nbin = more ? task_bin[task + 1] : bin;
        // Straight-line vector loads, so the compiler's vmcnt counts are exact:
        // the patch features of this wave's first two edges (a wave with fewer
        // uses a valid slot and skips it), the next task's regions (all-zero
        // loads when there is none) and records, then the two edges'
        // arithmetic, which waits for its own inputs only.  Edges past the
        // second (crowded cells) load after the prefetch and wait for it.
        const int s0 = seg0 + wave, s1 = s0 + cs::WAVES;
        const CsEdge ea = take_edge(recs, 0);
        const CsEdge eb = take_edge(recs, 1);
        stage_issue(nbin, more);
        {
            const int n0 = more ? task_off[task + 1] : seg0, n1 = more ? task_off[task + 2] : seg1;
            recs = load_recs(min(n0 + wave, n1 - 1), min(n0 + wave + cs::WAVES, n1 - 1));
        }
        CS_STAMP(a2)
        CS_ACC(1, a1, a2)
        auto run = [&](const CsEdge& in) __attribute__((always_inline)) {
            float v1[7], v2[7];
            CS_STAMP(b0)
            level(in, 1, cs::REG2_OFF, cs::R2, oy2, ox2, v2);
            CS_STAMP(b1)
            level(in, 0, cs::REG1_OFF, cs::R1, oy1, ox1, v1);
            CS_STAMP(b2)
            half_t* orow = p.out + (int64_t)in.e * p.o_e;
#pragma unroll
            for (int i = 0; i < 7; i++) {
                const int t = lane + 64 * i;
                if (t < DO * DO * NP) *(half2_t*)(orow + 2 * t) = half2_t{(half_t)v1[i], (half_t)v2[i]};
            }
            CS_STAMP(b3)
            CS_ACC(2, b0, b1) CS_ACC(3, b1, b2) CS_ACC(4, b2, b3)
#ifdef DPVO_STAMPS
            cst[7]++;
#endif
        };
        if (s0 < seg1) run(ea);
        if (s1 < seg1) run(eb);
        for (int slot = s1 + cs::WAVES; slot < seg1; slot += cs::WAVES) {
            const int rv = load_recs(slot, slot);
            run(take_edge(rv, 0));
        }
        if (!more) break;
        task++;
        bin = nbin;
    }
#ifdef DPVO_STAMPS
    CS_STAMP(k1)
    CS_ACC(5, k0, k1)
    if (lane == 0)
        for (int k = 0; k < 16; k++) dpvo_cs_stamps[((int64_t)blockIdx.x * cs::WAVES + wave) * 16 + k] = cst[k];
#endif
}

static int g_cs_cus = 0;

static CsGeom cs_geom(const CorrMfmaParams& p)
{
    CsGeom g;
    g.ncy = (p.H2[0] + cs::CELL - 1) / cs::CELL + 2;
    g.ncx = (p.W2[0] + cs::CELL - 1) / cs::CELL + 2;
    g.ncell = g.ncy * g.ncx;
    g.nb = (int)std::min<int64_t>((int64_t)std::min(p.N2[0], p.N2[1]) * g.ncell + 1, 0x7fffffff);
    g.pow2s = 1;
    for (int l = 0; l < 2; l++) {
        int ex = 0;
        const float m = std::frexp(p.scale[l], &ex);
        g.pow2s &= m == 0.5f && ex > -100 && ex < 100;
        g.iscale[l] = 1.0f / p.scale[l];
    }
    return g;
}

struct CsLayout {
    size_t count, offs, task_bin, task_off, ntask, wg_first, bin, order, rec, total;
};
static CsLayout cs_layout(int64_t E, int nb)
{
    CsLayout L;
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t at = o; o += (bytes + 255) / 256 * 256; return at; };
    L.count = take((size_t)nb * 4);
    L.offs = take((size_t)(nb + 1) * 4);
    L.task_bin = take((size_t)nb * 4);
    L.task_off = take((size_t)(nb + 1) * 4);
    L.ntask = take(4);
    L.wg_first = take((size_t)(CS_MAX_GRID + 1) * 4);
    L.bin = take((size_t)std::max<int64_t>(E, 1) * 4);
    L.order = take((size_t)std::max<int64_t>(E, 1) * 4);
    L.rec = take((size_t)std::max<int64_t>(E, 1) * cs::REC * 4);
    L.total = o;
    return L;
}


}  // namespace dpvo

using namespace dpvo;

#ifdef DPVO_STAMPS
extern "C" int dpvo_diag_cs_stamps(void* host, size_t bytes)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(dpvo_cs_stamps), std::min(bytes, sizeof(dpvo_cs_stamps)), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" size_t dpvo_corr_staged_workspace_bytes(int64_t num_edges, int64_t num_frames, int64_t height,
                                                   int64_t width)
{
    if (num_edges < 0 || num_frames < 0 || height < 0 || width < 0) return 0;
    const int64_t ncy = (height + cs::CELL - 1) / cs::CELL + 2, ncx = (width + cs::CELL - 1) / cs::CELL + 2;
    const int64_t nb = num_frames * ncy * ncx + 1;
    if (nb > CS_MAX_BINS) return 0;
    return cs_layout(num_edges, (int)nb).total;
}

extern "C" int dpvo_corr_pyramid_staged(const void* table, int64_t num_patches, const void* const* fmaps,
                                        const int64_t* fmap_sizes, const int64_t* fmap_strides,
                                        const float* level_scale, const float* coords, const int64_t* coords_size,
                                        const int64_t* coords_stride, const int64_t* ii, const int64_t* jj,
                                        void* corr, int64_t edge_stride, void* workspace, size_t workspace_bytes,
                                        void* stream)
{
    CorrMfmaParams p;
    if (corr_mfma_setup(p, table, num_patches, fmaps, fmap_sizes, fmap_strides, level_scale, coords, coords_size,
                        coords_stride, ii, jj, corr, edge_stride, nullptr))
        return -1;
    DPVO_CHECK_ARG(coords_stride[4] == 1 && coords_stride[3] == 3 && coords_stride[2] == 9 && coords_stride[1] == 18,
                   "the staged kernel reads contiguous coords [1][E][2][3][3]");
    const CsGeom g = cs_geom(p);
    DPVO_CHECK_ARG((int64_t)std::min(p.N2[0], p.N2[1]) * g.ncell + 1 <= CS_MAX_BINS,
                   "too many (frame, cell) bins for the staged kernel");
    const CsLayout L = cs_layout(p.E, g.nb);
    DPVO_CHECK_ARG(workspace && workspace_bytes >= L.total, "workspace too small (dpvo_corr_staged_workspace_bytes)");
    if (p.E == 0) return 0;
    hipStream_t s = as_stream(stream);
    char* ws = (char*)workspace;
    int* count = (int*)(ws + L.count);
    int* offs = (int*)(ws + L.offs);
    int* task_bin = (int*)(ws + L.task_bin);
    int* task_off = (int*)(ws + L.task_off);
    int* ntask = (int*)(ws + L.ntask);
    int* wg_first = (int*)(ws + L.wg_first);
    int* bin = (int*)(ws + L.bin);
    int* order = (int*)(ws + L.order);
    int* rec = (int*)(ws + L.rec);
    if (g_cs_cus == 0) {
        int dev = 0;
        DPVO_CHECK_HIP(hipGetDevice(&dev));
        DPVO_CHECK_HIP(hipDeviceGetAttribute(&g_cs_cus, hipDeviceAttributeMultiprocessorCount, dev));
        if (g_cs_cus <= 0) g_cs_cus = 256;
        g_cs_cus = std::min(g_cs_cus, CS_MAX_GRID);
    }
    const int G = g_cs_cus;   // one workgroup per CU (LDS)
    DPVO_CHECK_HIP(hipMemsetAsync(count, 0, (size_t)g.nb * 4, s));
    const unsigned ge = grid_for(p.E, 256);
    hipLaunchKernelGGL(cs_bin_kernel, dim3(ge), dim3(256), 0, s, p, g, bin, count);
    hipLaunchKernelGGL(cs_scan_kernel, dim3(1), dim3(1024), 0, s, g, G, count, offs, task_bin, task_off, ntask,
                       wg_first);
    hipLaunchKernelGGL(cs_scatter_kernel, dim3(ge), dim3(256), 0, s, p, g, bin, count, order, rec);
    hipLaunchKernelGGL(corr_stage_kernel, dim3((unsigned)G), dim3(cs::THREADS), 0, s, p, g, rec, task_bin,
                       task_off, ntask, wg_first);
    DPVO_CHECK_LAUNCH();
    // the fallback bin: order slots [offs[nb - 1], E) through the per-edge kernel
    CorrMfmaParams pf = p;
    pf.order = order;
    pf.dev_begin = offs + (g.nb - 1);
    return corr_mfma_launch(pf, s);
}

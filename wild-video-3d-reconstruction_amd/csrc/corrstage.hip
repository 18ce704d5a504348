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

#include "corrmfma.hpp"

namespace dpvo {

namespace cs {
constexpr int WAVES = 8, THREADS = 64 * WAVES;
constexpr int CELL = 8;                        // level-1 cell pitch (pixels)
constexpr int R1 = 17, O1 = -4;                // level-1 region of cell c: [8c - 4, 8c + 12]
constexpr int R2 = 11, O2 = -4;                // level-2 region of cell c: [2c - 4, 2c + 6]
constexpr int NPX1 = R1 * R1, NPX2 = R2 * R2;  // 289, 121 pixels
constexpr int PIXB = cm::C * 2;                // 256 B per pixel
constexpr int CH1 = (NPX1 * 16 + 63) / 64 * 64;   // level-1 16-byte chunks, padded to whole wave instructions
constexpr int CH2 = NPX2 * 16;
constexpr int LOADS = (CH1 + CH2 + THREADS - 1) / THREADS;   // staging loads per lane
constexpr int REG1_OFF = 0;
constexpr int REG2_OFF = NPX1 * PIXB;                          // 73,984
constexpr int RAW_OFF = REG2_OFF + NPX2 * PIXB;                // 104,960
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
};

__device__ __forceinline__ int cs_floor8(int v) { return v >> 3; }   // floor(v / 8), v small

// per edge: its bin (see above) and the bin's count
__global__ __launch_bounds__(256) void cs_bin_kernel(CorrMfmaParams p, CsGeom g, int* __restrict__ bin,
                                                     int* __restrict__ count)
{
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= p.E) return;
    int b = g.nb - 1;
    const int64_t ix = p.ii[e], jx = p.jj[e];
    if (ix >= 0 && ix < p.N1 && jx >= 0 && jx < p.N2[0] && jx < p.N2[1]) {
        int fy0 = 0x7fffffff, fy1 = -0x7fffffff, fx0 = 0x7fffffff, fx1 = -0x7fffffff;
        int gy0 = 0x7fffffff, gy1 = -0x7fffffff, gx0 = 0x7fffffff, gx1 = -0x7fffffff;
        bool fin = true;
        const float* cb = p.coords + (int64_t)e * p.c_s[1];
#pragma unroll
        for (int q = 0; q < cm::NP; q++) {
            const float* c = cb + (q / 3) * p.c_s[3] + (q % 3) * p.c_s[4];
            const float cx = c[0], cy = c[p.c_s[2]];
            // finite and well inside int range (the floors below are the kernel's own)
            fin = fin && fabsf(cx) < 1e6f && fabsf(cy) < 1e6f;
            const int fy = floor_to_int_sat(cy / p.scale[0]), fx = floor_to_int_sat(cx / p.scale[0]);
            const int gy = floor_to_int_sat(cy / p.scale[1]), gx = floor_to_int_sat(cx / p.scale[1]);
            fy0 = min(fy0, fy); fy1 = max(fy1, fy); fx0 = min(fx0, fx); fx1 = max(fx1, fx);
            gy0 = min(gy0, gy); gy1 = max(gy1, gy); gx0 = min(gx0, gx); gx1 = max(gx1, gx);
        }
        if (fin && fy1 - fy0 <= cm::BOXMAX - cm::D && fx1 - fx0 <= cm::BOXMAX - cm::D) {
            // the cell whose region's top-left corner is the last one at or
            // above the box's: region [8c - 4, 8c + 12] holds rows fy0 - 3 ..
            // fy1 + 4 iff fy1 <= 8c + 8
            const int cy = cs_floor8(fy0 + 1), cx = cs_floor8(fx0 + 1);
            bool ok = cy >= -1 && cy < g.ncy - 1 && cx >= -1 && cx < g.ncx - 1;
            ok = ok && fy1 <= cs::CELL * cy + 8 && fx1 <= cs::CELL * cx + 8;
            // level 2: box rows gy0 - 3 .. gy1 + 4 inside [2c - 4, 2c + 6]
            ok = ok && gy0 >= 2 * cy - 1 && gy1 <= 2 * cy + 2 && gx0 >= 2 * cx - 1 && gx1 <= 2 * cx + 2;
            if (ok) b = (int)jx * g.ncell + (cy + 1) * g.ncx + (cx + 1);
        }
    }
    bin[e] = b;
    atomicAdd(&count[b], 1);
}

// One workgroup: exclusive offsets of the bins (offs[nb] = E), the counts
// turned into scatter cursors, and the non-empty staged bins as a task list
// (task_bin, task_off[ntask + 1]: task_off[ntask] = the fallback bin's start).
__global__ __launch_bounds__(1024) void cs_scan_kernel(CsGeom g, int* __restrict__ count, int* __restrict__ offs,
                                                       int* __restrict__ task_bin, int* __restrict__ task_off,
                                                       int* __restrict__ ntask)
{
    __shared__ int wsum[16][2];
    const int nb = g.nb, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int per = (nb + 1023) / 1024;
    const int b0 = min(nb, t * per), b1 = min(nb, b0 + per);
    int s = 0, ne = 0;
    for (int b = b0; b < b1; b++) {
        const int c = count[b];
        s += c;
        ne += (c > 0 && b < nb - 1);
    }
    // inclusive wave scans of (s, ne)
    int is = s, in = ne;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int ys = __shfl_up(is, d, 64), yn = __shfl_up(in, d, 64);
        if (lane >= d) { is += ys; in += yn; }
    }
    if (lane == 63) { wsum[w][0] = is; wsum[w][1] = in; }
    __syncthreads();
    int bs = 0, bn = 0, tot = 0;
    for (int k = 0; k < 16; k++) {
        if (k < w) { bs += wsum[k][0]; bn += wsum[k][1]; }
        tot += wsum[k][1];
    }
    int o = bs + is - s, tk = bn + in - ne;
    for (int b = b0; b < b1; b++) {
        const int c = count[b];
        offs[b] = o;
        count[b] = o;   // the scatter's cursor
        if (b == nb - 1) {   // the fallback bin closes the task list
            task_off[tot] = o;
            *ntask = tot;
            offs[nb] = o + c;
        } else if (c > 0) {
            task_bin[tk] = b;
            task_off[tk] = o;
            tk++;
        }
        o += c;
    }
}

__global__ __launch_bounds__(256) void cs_scatter_kernel(int E, const int* __restrict__ bin, int* __restrict__ cursor,
                                                         int* __restrict__ order)
{
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    order[atomicAdd(&cursor[bin[e]], 1)] = e;
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

// LDS byte address of 16-byte chunk cc of region pixel px: chunks XOR-swizzled
// by the pixel's low 4 bits, so the 16 pixels of an MFMA tile reading the same
// chunk spread over the banks
__device__ __forceinline__ int cs_chunk(int base, int px, int cc) { return base + px * cs::PIXB + ((cc ^ (px & 15)) << 4); }

struct CsEdge {
    int e, ix;
    float cx, cy;   // patch pixel (lane & 15)'s coordinates when < 9
    h8_t bq[4];     // B fragments: patch pixel (lane & 15) x 8 channels of each 32-channel step
};

// One workgroup per CU, 8 waves.  Workgroup b (logical index: each XCD owns
// one contiguous eighth) takes an equal share of the binned edge slots and
// walks the bins (tasks) that share covers.  Per task: stage the regions,
// then each wave takes the task's edges wave, wave + 8, ...; per edge, level
// 2 then level 1 (one per-wave product box, reused), exactly the tile / MFMA /
// bilinear arithmetic of corr_mfma_kernel's fast path.
__global__ __launch_bounds__(cs::THREADS, 1) void corr_stage_kernel(CorrMfmaParams p, CsGeom g,
                                                                    const int* __restrict__ order,
                                                                    const int* __restrict__ task_bin,
                                                                    const int* __restrict__ task_off,
                                                                    const int* __restrict__ ntask_p)
{
    using namespace cm;
    __shared__ __attribute__((aligned(16))) char smem[cs::LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int G = gridDim.x, bid = blockIdx.x;
    const int lw = (G >= 8 && (G & 7) == 0) ? (bid & 7) * (G >> 3) + (bid >> 3) : bid;
    const int ntask = *ntask_p;
    if (ntask == 0) return;
    const int Eb = task_off[ntask];   // binned edges (the fallback bin follows)
    const int s_begin = (int)((int64_t)Eb * lw / G), s_end = (int)((int64_t)Eb * (lw + 1) / G);
    if (s_begin >= s_end) return;     // the whole workgroup
    // the task holding slot s_begin: the last with task_off <= s_begin
    int lo = 0, hi = ntask - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (task_off[mid] <= s_begin) lo = mid; else hi = mid - 1;
    }
    int task = lo;

    float* rw = reinterpret_cast<float*>(smem + cs::RAW_OFF + wave * cs::RAW_W);
    float* wts = reinterpret_cast<float*>(smem + cs::WTS_OFF) + wave * 64;     // [4][16]
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
    auto stage_issue = [&](int bin) __attribute__((always_inline)) {
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
            if (kb < cs::CH1) {
                const int k = kb + lane, px = k >> 4, cc = k & 15;
                const int ry = px / cs::R1, rx = px - ry * cs::R1;
                const int gy = oy1 + ry, gx = ox1 + rx;
                const bool ok = px < cs::NPX1 && gy >= 0 && gy < p.H2[0] && gx >= 0 && gx < p.W2[0];
                const unsigned off = ok ? (unsigned)(gy * (int)p.rowb[0] + gx * p.pixb[0] + 16 * cc) : OOB;
                st[j] = __builtin_bit_cast(u4_t, __builtin_amdgcn_raw_buffer_load_b128(r1, off, 0, 0));
            } else if (kb < cs::CH1 + cs::CH2) {
                const int k = kb - cs::CH1 + lane, px = k >> 4, cc = k & 15;
                const int ry = px / cs::R2, rx = px - ry * cs::R2;
                const int gy = oy2 + ry, gx = ox2 + rx;
                const bool ok = px < cs::NPX2 && gy >= 0 && gy < p.H2[1] && gx >= 0 && gx < p.W2[1];
                const unsigned off = ok ? (unsigned)(gy * (int)p.rowb[1] + gx * p.pixb[1] + 16 * cc) : OOB;
                st[j] = __builtin_bit_cast(u4_t, __builtin_amdgcn_raw_buffer_load_b128(r2, off, 0, 0));
            }
        }
    };
    auto stage_write = [&]() __attribute__((always_inline)) {
        const int w64 = 64 * wave + cs_opaque_zero();
#pragma unroll
        for (int j = 0; j < cs::LOADS; j++) {
            const int kb = cs::THREADS * j + w64;
            if (kb < cs::CH1) {
                const int k = kb + lane, px = k >> 4, cc = k & 15;
                if (px < cs::NPX1) *(u4_t*)(smem + cs_chunk(cs::REG1_OFF, px, cc)) = st[j];
            } else if (kb < cs::CH1 + cs::CH2) {
                const int k = kb - cs::CH1 + lane, px = k >> 4, cc = k & 15;
                if (px < cs::NPX2) *(u4_t*)(smem + cs_chunk(cs::REG2_OFF, px, cc)) = st[j];
            }
        }
    };
    auto load_edge = [&](int slot) __attribute__((always_inline)) {
        CsEdge in;
        in.e = __builtin_amdgcn_readfirstlane(order[slot]);
        in.ix = __builtin_amdgcn_readfirstlane((int)p.ii[in.e]);
        const int q = qv ? q16 : 0;
        const float* cb = p.coords + (int64_t)in.e * p.c_s[1] + (q / 3) * p.c_s[3] + (q % 3) * p.c_s[4];
        in.cx = cb[0];
        in.cy = cb[p.c_s[2]];
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<half_t*>(p.gt + (int64_t)in.ix * NP * C), (short)0, NP * C * 2, 0x00020000);
        const unsigned voff = qv ? (unsigned)(q16 * C * 2 + 16 * kc) : OOB;
#pragma unroll
        for (int ks = 0; ks < 4; ks++)
            in.bq[ks] = __builtin_bit_cast(h8_t, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 64 * ks, 0, 0));
        return in;
    };

    // one level of one edge: tiles from the LDS region -> product box -> 7 bilinear outputs per lane
    auto level = [&](const CsEdge& in, int l, int reg_off, int RW, int oyl, int oxl, float* v) __attribute__((always_inline)) {
        const float x = in.cx / p.scale[l], y = in.cy / p.scale[l];
        const int fy = floor_to_int_sat(y), fx = floor_to_int_sat(x);
        int ymin = __builtin_amdgcn_readlane(fy, 0), ymax = ymin;
        int xmin = __builtin_amdgcn_readlane(fx, 0), xmax = xmin;
#pragma unroll
        for (int q = 1; q < NP; q++) {
            const int vy = __builtin_amdgcn_readlane(fy, q), vx = __builtin_amdgcn_readlane(fx, q);
            ymin = min(ymin, vy); ymax = max(ymax, vy);
            xmin = min(xmin, vx); xmax = max(xmax, vx);
        }
        const int bw = xmax - xmin + D, bh = ymax - ymin + D;
        const int npx = bw * bh, ntiles = (npx + 15) >> 4;
        // the box's origin (ymin - R, xmin - R) in region coordinates
        const int boy = ymin - R - oyl, box = xmin - R - oxl;
        cs_wave_fence();   // the previous level's epilogue has read wts / raw / ebase
        if (lane < NP) {
            const float dx = x - floorf(x), dy = y - floorf(y);
            wts[0 * 16 + lane] = (1.f - dx) * (1.f - dy);
            wts[1 * 16 + lane] = dx * (1.f - dy);
            wts[2 * 16 + lane] = (1.f - dx) * dy;
            wts[3 * 16 + lane] = dx * dy;
            ebase[lane] = (fy - ymin) * bw + (fx - xmin);
        }
        // lane's box pixel 16 t + q16, walked by increments (the box is >= 8 wide)
        int by = q16 / bw, bx = q16 - (q16 / bw) * bw;
        const int pmax = RW * RW - 1;
        auto tile_load = [&](h8_t* a) __attribute__((always_inline)) {
            const int px = min((boy + by) * RW + box + bx, pmax);
#pragma unroll
            for (int ks = 0; ks < 4; ks++) a[ks] = *(const h8_t*)(smem + cs_chunk(reg_off, px, 4 * ks + kc));
            bx += 16;
            if (bx >= bw) { bx -= bw; by++; }
            if (bx >= bw) { bx -= bw; by++; }
        };
        auto tile_mma = [&](const h8_t* a, int t) __attribute__((always_inline)) {
            f4m_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 4; ks++) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[ks], in.bq[ks], acc, 0, 0, 0);
            // acc[r] = tile pixel 4 kc + r . patch pixel (lane & 15)
            if (qv) *(f4m_t*)(rw + q16 * RS + 16 * t + 4 * kc) = acc;
        };
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
        // bilinear 8x8 -> 7x7 per patch pixel (fp32)
#pragma unroll
        for (int i = 0; i < 7; i++) {
            // output t = lane + 64 i is (x offset, y offset, patch pixel) = ((t / 9) / 7, (t / 9) % 7, t % 9)
            const int t = min(lane + 64 * i, DO * DO * NP - 1);
            const int pos = t / NP, q = t - pos * NP;
            const int exi = pos / DO, eyi = pos - exi * DO;
            const float* r0 = rw + q * RS + ebase[q] + eyi * bw + exi;
            v[i] = cm_bilinear(wts[0 * 16 + q], wts[1 * 16 + q], wts[2 * 16 + q], wts[3 * 16 + q], r0[0], r0[1],
                               r0[bw], r0[bw + 1]);
        }
    };

    int t_next = task;
    int bin = task_bin[task];
    stage_issue(bin);
    for (;;) {
        const int seg0 = max(s_begin, task_off[task]), seg1 = min(s_end, task_off[task + 1]);
        int frame, oy1, ox1, oy2, ox2;
        region_of(bin, frame, oy1, ox1, oy2, ox2);
        (void)frame;
        __syncthreads();   // every wave is done with the previous task's regions
        stage_write();
        __syncthreads();
        const bool more = seg1 < s_end && task + 1 < ntask;
        t_next = task + 1;
        int slot = seg0 + wave;
        CsEdge cur;
        if (slot < seg1) cur = load_edge(slot);
        int nbin = 0;
        if (more) {
            nbin = task_bin[t_next];
            stage_issue(nbin);   // the next task's regions load while this one computes
        }
        for (; slot < seg1; slot += cs::WAVES) {
            CsEdge nxt;
            if (slot + cs::WAVES < seg1) nxt = load_edge(slot + cs::WAVES);
            float v1[7], v2[7];
            level(cur, 1, cs::REG2_OFF, cs::R2, oy2, ox2, v2);
            level(cur, 0, cs::REG1_OFF, cs::R1, oy1, ox1, v1);
            half_t* orow = p.out + (int64_t)cur.e * p.o_e;
#pragma unroll
            for (int i = 0; i < 7; i++) {
                const int t = lane + 64 * i;
                if (t < DO * DO * NP) *(half2_t*)(orow + 2 * t) = half2_t{(half_t)v1[i], (half_t)v2[i]};
            }
            cur = nxt;
        }
        if (!more) break;
        task = t_next;
        bin = nbin;
    }
}

static int g_cs_cus = 0;

static CsGeom cs_geom(const CorrMfmaParams& p)
{
    CsGeom g;
    g.ncy = (p.H2[0] + cs::CELL - 1) / cs::CELL + 2;
    g.ncx = (p.W2[0] + cs::CELL - 1) / cs::CELL + 2;
    g.ncell = g.ncy * g.ncx;
    g.nb = (int)std::min<int64_t>((int64_t)std::min(p.N2[0], p.N2[1]) * g.ncell + 1, 0x7fffffff);
    return g;
}

struct CsLayout {
    size_t count, offs, task_bin, task_off, ntask, bin, order, total;
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
    L.bin = take((size_t)std::max<int64_t>(E, 1) * 4);
    L.order = take((size_t)std::max<int64_t>(E, 1) * 4);
    L.total = o;
    return L;
}

constexpr int CS_MAX_BINS = 1 << 20;

}  // namespace dpvo

using namespace dpvo;

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
    int* bin = (int*)(ws + L.bin);
    int* order = (int*)(ws + L.order);
    DPVO_CHECK_HIP(hipMemsetAsync(count, 0, (size_t)g.nb * 4, s));
    const unsigned ge = grid_for(p.E, 256);
    hipLaunchKernelGGL(cs_bin_kernel, dim3(ge), dim3(256), 0, s, p, g, bin, count);
    hipLaunchKernelGGL(cs_scan_kernel, dim3(1), dim3(1024), 0, s, g, count, offs, task_bin, task_off, ntask);
    hipLaunchKernelGGL(cs_scatter_kernel, dim3(ge), dim3(256), 0, s, p.E, bin, count, order);
    if (g_cs_cus == 0) {
        int dev = 0;
        DPVO_CHECK_HIP(hipGetDevice(&dev));
        DPVO_CHECK_HIP(hipDeviceGetAttribute(&g_cs_cus, hipDeviceAttributeMultiprocessorCount, dev));
        if (g_cs_cus <= 0) g_cs_cus = 256;
    }
    hipLaunchKernelGGL(corr_stage_kernel, dim3((unsigned)g_cs_cus), dim3(cs::THREADS), 0, s, p, g, order, task_bin,
                       task_off, ntask);
    DPVO_CHECK_LAUNCH();
    // the fallback bin: order slots [offs[nb - 1], E) through the per-edge kernel
    CorrMfmaParams pf = p;
    pf.order = order;
    pf.dev_begin = offs + (g.nb - 1);
    return corr_mfma_launch(pf, s);
}

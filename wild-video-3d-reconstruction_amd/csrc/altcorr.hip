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
#include <stdlib.h>

#include "common.hpp"

namespace dpvo {

namespace corr {
constexpr int R = 3, D = 8, DO = 7, PS = 3, NP = 9, NPAIR = 5;
// v3's shared box: floor spreads up to 4 px (12 x 12).  At level 1 about 1 edge
// in 9 of the C3 workload spreads by 3 px (perspective scale ~1.4 between
// frames up to 35 apart); per-pixel windows would cost it 4x the common pass.
constexpr int SBOX = 12;
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
    const uint32_t* f1tab;   // [B*N1][C][5] packed patch-feature pairs (corr_pack_kernel)
};

__device__ __forceinline__ half2_t as_h2(uint32_t v) { return __builtin_bit_cast(half2_t, v); }
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// exact binary16 ops (contraction is off for this file)
__device__ __forceinline__ half_t hmul(half_t a, half_t b) { return a * b; }
__device__ __forceinline__ half_t hadd(half_t a, half_t b) { return a + b; }

// Block -> edge map that gives each XCD a contiguous run of edges (blocks
// b, b+8, ... share an XCD under round-robin dispatch), so consecutive edges --
// which mostly share a target frame -- reuse that XCD's L2 (speed only).
__device__ __forceinline__ int xcd_swizzle(int b, int nblk)
{
    const int main = nblk & ~7;
    if (b >= main) return b;
    return (b & 7) * (main >> 3) + (b >> 3);
}

template <int NLEV>
struct FastThreads {
    static constexpr int value = NLEV == 2 ? 192 : 128;
};

// per-level metadata, uniform over the workgroup (kept in LDS so that runtime
// level / pixel indices never force register arrays to scratch)
struct LevelMeta {
    int fy[corr::NP], fx[corr::NP];
    float xs[corr::NP], ys[corr::NP];
    int fast, oy, ox, bw, bh, nslots, first_slot, pad;
    float rbw;   // 1 / bw (v3 decode: exact floor((loc + 0.5) / bw) for loc < 256, bw <= 12)
};

// ---------------------------------------------------------------------------
// v3 fast path: the patch features are uniform over the workgroup, so they are
// read as SCALAR operands (s_load from a per-call packed table) instead of LDS
// broadcasts -- no ds_read latency in the chain, 40 fewer VGPRs (occupancy).
// ---------------------------------------------------------------------------
typedef unsigned int u32x16 __attribute__((ext_vector_type(16)));

// gmap [B][N1][C][3][3] -> table [B*N1][C][5] dwords: (p0,p1)(p2,p3)(p4,p5)(p6,p7)(p8,0)
__global__ __launch_bounds__(256) void corr_pack_kernel(const half_t* __restrict__ gmap, int64_t gs0, int64_t gs1,
                                                        int64_t gs2, int64_t gs3, int64_t gs4, int B, int N1, int C,
                                                        uint32_t* __restrict__ tab)
{
    const int64_t total = (int64_t)B * N1 * C;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(t % C);
        const int64_t bn = t / C;
        const int n = (int)(bn % N1), b = (int)(bn / N1);
        const half_t* g = gmap + b * gs0 + n * gs1 + c * gs2;
        half_t v[10];
#pragma unroll
        for (int q = 0; q < 9; q++) v[q] = g[(q / 3) * gs3 + (q % 3) * gs4];
        v[9] = (half_t)0;
        uint32_t* o = tab + t * 5;
#pragma unroll
        for (int q = 0; q < 5; q++) o[q] = __builtin_bit_cast(uint32_t, (half2_t){v[2 * q], v[2 * q + 1]});
    }
}

template <int NLEV, int C8>
__global__ __launch_bounds__(FastThreads<NLEV>::value) void corr_sfast_kernel(CorrFastParams p)
{
    using namespace corr;
    constexpr int NT = FastThreads<NLEV>::value;
    constexpr int C = C8 * 8;
    __shared__ half_t raw[NLEV][NP][SBOX * SBOX];
    __shared__ LevelMeta meta[NLEV];
    // per (patch pixel, level): the reference's bilinear weights (each product
    // rounded to binary16 exactly as correlation_kernel.cu:221-232 forms them)
    // and the raw-tile offset of the window origin
    struct EpiQ { half_t w00, w01, w10, w11; int base, bw; };
    __shared__ EpiQ epq[NP * NLEV];

    const int bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const int b = bid / p.E, e = bid - b * p.E;
    const int tid = threadIdx.x;
    const int ix = (int)p.ii[e];
    const int jx = (int)p.jj[e];
    const bool ix_ok = ix >= 0 && ix < p.N1;

    // ---- per-(level, patch pixel) coordinates and floors: 9*NLEV threads
    if (tid < NLEV * NP) {
        const int lev = tid / NP, q = tid - lev * NP;
        const float sc = p.scale[lev];
        const float* cb = p.coords + b * p.c_s[0] + (int64_t)e * p.c_s[1];
        const int64_t o = (q / PS) * p.c_s[3] + (q % PS) * p.c_s[4];
        const float x = cb[o] / sc, y = cb[p.c_s[2] + o] / sc;
        LevelMeta& m = meta[lev];
        m.xs[q] = x; m.ys[q] = y;
        m.fy[q] = floor_to_int_sat(y);
        m.fx[q] = floor_to_int_sat(x);
    }
    __syncthreads();
    if (tid < NLEV) {
        LevelMeta& m = meta[tid];
        int ymin = 0x7fffffff, ymax = (int)0x80000000u, xmin = 0x7fffffff, xmax = (int)0x80000000u;
#pragma unroll
        for (int q = 0; q < NP; q++) {
            ymin = min(ymin, m.fy[q]); ymax = max(ymax, m.fy[q]);
            xmin = min(xmin, m.fx[q]); xmax = max(xmax, m.fx[q]);
        }
        m.fast = ((int64_t)ymax - ymin) <= SBOX - D && ((int64_t)xmax - xmin) <= SBOX - D;
        m.oy = wrap_add(ymin, -R);
        m.ox = wrap_add(xmin, -R);
        m.bh = m.fast ? (ymax - ymin) + D : D;
        m.bw = m.fast ? (xmax - xmin) + D : D;
        m.nslots = m.fast ? m.bh * m.bw : NP * D * D;
        m.rbw = 1.0f / (float)m.bw;
    }
    __syncthreads();
    if (tid < NP * NLEV) {   // epilogue constants, index qi = q * NLEV + lev (output order)
        const int q = tid / NLEV, lev = tid - q * NLEV;
        const LevelMeta& m = meta[lev];
        const int bw = m.fast ? m.bw : D;
        const int oy = m.fast ? m.fy[q] - (int)wrap_add(m.oy, R) : 0;
        const int ox = m.fast ? m.fx[q] - (int)wrap_add(m.ox, R) : 0;
        const float xq = m.xs[q], yq = m.ys[q];
        const half_t dx = (half_t)(xq - floorf(xq));
        const half_t dy = (half_t)(yq - floorf(yq));
        const half_t one = (half_t)1.0f;
        const half_t omdx = one - dx, omdy = one - dy;
        EpiQ& t = epq[tid];
        t.w00 = hmul(omdx, omdy);
        t.w01 = hmul(dx, omdy);
        t.w10 = hmul(omdx, dy);
        t.w11 = hmul(dx, dy);
        t.base = oy * bw + ox;
        t.bw = bw;
    }
    const int n0 = meta[0].nslots;
    const int total = NLEV == 2 ? n0 + meta[NLEV - 1].nslots : n0;

    struct Slot { int lev, q_only, u; bool act, inb; const uint4* ptr; };
    auto decode = [&](int slot) {
        Slot s{0, -1, 0, false, false, nullptr};
        s.act = slot < total;
        const int sl = s.act ? slot : 0;
        s.lev = (NLEV == 2 && sl >= n0) ? NLEV - 1 : 0;
        const LevelMeta& m = meta[s.lev];
        const int loc = s.lev ? sl - n0 : sl;
        int gy, gx;
        if (m.fast) {
            const int uy = (int)(((float)loc + 0.5f) * m.rbw), ux = loc - uy * m.bw;
            gy = wrap_add(m.oy, uy); gx = wrap_add(m.ox, ux);
            s.u = loc;
        } else {
            const int q = loc / (D * D), u = loc - q * (D * D);
            const int uy = u / D, ux = u - uy * D;
            gy = wrap_add(m.fy[q], uy - R); gx = wrap_add(m.fx[q], ux - R);
            s.q_only = q;
            s.u = u;
        }
        const int lv = s.lev;
        s.inb = s.act && ix_ok && jx >= 0 && jx < p.N2[lv] && gy >= 0 && gy < p.H2[lv] && gx >= 0 && gx < p.W2[lv];
        const half_t* base = p.fmap[lv] + b * p.f_s0[lv];
        s.ptr = reinterpret_cast<const uint4*>(
            s.inb ? base + (int64_t)jx * p.f_s1[lv] + (int64_t)gy * p.f_s3[lv] + (int64_t)gx * p.f_s4[lv] : base);
        return s;
    };

    // this patch's packed features: 4 channels = 20 dwords (s_load x16 + x4)
    const uint32_t* T = p.f1tab + ((int64_t)b * p.N1 + (ix_ok ? ix : 0)) * C * 5;

    for (int base = 0; base < total; base += NT) {
        if (base + (tid & ~63) >= total) continue;   // a wave with no slot in this pass skips it
        const Slot cur = decode(base + tid);
        half2_t acc[NPAIR];
#pragma unroll
        for (int q = 0; q < NPAIR; q++) acc[q] = (half2_t){(half_t)0, (half_t)0};
        // Hand-scheduled: pixel-row chunks by asm global loads (4 in flight,
        // counted vmcnt), patch features by asm scalar loads one 4-channel step
        // ahead (SMEM returns out of order: lgkmcnt(0) per step).
        u32x4 w[C8];
        u32x16 fa16, fb16;
        u32x4 fa4, fb4;
#pragma unroll
        for (int k = 0; k < 4; k++)
            asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(w[k]) : "v"(cur.ptr), "i"(k * 16));
        asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx4 %1, %2, 0x40"
                     : "=s"(fa16), "=s"(fa4) : "s"(T));
#pragma unroll
        for (int k = 0; k < C8; k++) {
            // chunk k holds channels 8k..8k+7 = steps 2k, 2k+1
            switch (C8 - 1 - k < 3 ? C8 - 1 - k : 3) {   // outstanding younger chunks
            case 3: asm volatile("s_waitcnt vmcnt(3)" : "+v"(w[k])); break;
            case 2: asm volatile("s_waitcnt vmcnt(2)" : "+v"(w[k])); break;
            case 1: asm volatile("s_waitcnt vmcnt(1)" : "+v"(w[k])); break;
            default: asm volatile("s_waitcnt vmcnt(0)" : "+v"(w[k])); break;
            }
            if (k + 4 < C8)
                asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(w[k + 4]) : "v"(cur.ptr), "i"((k + 4) * 16));
#pragma unroll
            for (int hs = 0; hs < 2; hs++) {
                const int step = 2 * k + hs;
                u32x16& c16 = (step & 1) ? fb16 : fa16;
                u32x4& c4 = (step & 1) ? fb4 : fa4;
                u32x16& n16 = (step & 1) ? fa16 : fb16;
                u32x4& n4 = (step & 1) ? fa4 : fb4;
                asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(c16), "+s"(c4));
                if (step + 1 < 2 * C8)
                    asm volatile("s_load_dwordx16 %0, %2, %3\n\ts_load_dwordx4 %1, %2, %4"
                                 : "=s"(n16), "=s"(n4) : "s"(T), "i"((step + 1) * 80), "i"((step + 1) * 80 + 64));
                const uint32_t fs[20] = {c16[0], c16[1], c16[2], c16[3], c16[4], c16[5], c16[6], c16[7],
                                         c16[8], c16[9], c16[10], c16[11], c16[12], c16[13], c16[14], c16[15],
                                         c4[0], c4[1], c4[2], c4[3]};
                const uint32_t wd[2] = {hs ? w[k][2] : w[k][0], hs ? w[k][3] : w[k][1]};
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    const half2_t wv = as_h2(wd[j]);
#pragma unroll
                    for (int hsel = 0; hsel < 2; hsel++) {
                        const int c = 2 * j + hsel;
                        const half_t ws = hsel ? wv.y : wv.x;
                        const half2_t wb = {ws, ws};
                        // all five products first, then the five sums (same per-op
                        // rounding): a product feeding the very next instruction costs
                        // an s_nop on gfx950 when its src0 carries op_sel_hi = 1 (the
                        // hi-half broadcast), ~300 wait states per pass otherwise
                        half2_t pr[NPAIR];
#pragma unroll
                        for (int q = 0; q < NPAIR; q++) pr[q] = wb * as_h2(fs[c * 5 + q]);
                        __builtin_amdgcn_sched_barrier(0);   // (an asm fence would itself cost the s_nop)
#pragma unroll
                        for (int q = 0; q < NPAIR; q++) acc[q] = acc[q] + pr[q];
                    }
                }
                // keep this step's arithmetic ahead of the next step's (volatile) loads:
                // LLVM otherwise sinks the pure VALU chain and spills the SGPR operands
                asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (cur.act) {
            const half_t z = (half_t)0;
            const half_t sv[NP] = {acc[0].x, acc[0].y, acc[1].x, acc[1].y, acc[2].x,
                                   acc[2].y, acc[3].x, acc[3].y, acc[4].x};
            if (cur.q_only < 0) {
#pragma unroll
                for (int q = 0; q < NP; q++) raw[cur.lev][q][cur.u] = cur.inb ? sv[q] : z;
            } else {
                half_t v = z;
#pragma unroll
                for (int q = 0; q < NP; q++) if (q == cur.q_only) v = sv[q];
                raw[cur.lev][cur.q_only][cur.u] = cur.inb ? v : z;
            }
        }
    }
    __syncthreads();

    half_t* ob = p.out + b * p.o_b + (int64_t)e * p.o_e;
    // DPVO's stacked row [x][y][P][P][level] (dpvo.py:333; what corr_pyramid
    // writes): thread t owns the two levels of output pair t = (x, y, pixel), one
    // half2 op per bilinear step (each lane rounds exactly like the scalar
    // sequence) and one 4-byte store; a wave stores 256 contiguous bytes.
    const bool stacked = NLEV == 2 && p.o_l == 1 && p.o_p == 2 && p.o_y == 18 && p.o_x == 126 &&
                         ((uintptr_t)ob & 3) == 0;
    if (stacked) {
        for (int t = tid; t < DO * DO * NP; t += NT) {
            const int pos = t / NP, q = t - pos * NP;
            const int bx = pos / DO, a = pos - bx * DO;
            const EpiQ t0 = epq[q * NLEV], t1 = epq[q * NLEV + 1];
            const half_t* c0 = &raw[0][q][t0.base + a * t0.bw + bx];
            const half_t* c1 = &raw[NLEV - 1][q][t1.base + a * t1.bw + bx];
            half2_t v = half2_t{t0.w00, t1.w00} * half2_t{c0[0], c1[0]};
            v = v + half2_t{t0.w01, t1.w01} * half2_t{c0[1], c1[1]};
            v = v + half2_t{t0.w10, t1.w10} * half2_t{c0[t0.bw], c1[t1.bw]};
            v = v + half2_t{t0.w11, t1.w11} * half2_t{c0[t0.bw + 1], c1[t1.bw + 1]};
            *(half2_t*)(ob + 2 * t) = v;
        }
        return;
    }
    // general strides: thread -> fixed (patch pixel, level) qi, walking the 49 window positions
    constexpr int NQ = NP * NLEV, GR = NT / NQ;
    if (tid < NQ * GR) {
        const int qi = tid % NQ, g = tid / NQ;
        const int q = qi / NLEV, lev = qi - q * NLEV;
        const EpiQ t = epq[qi];
        const half_t* rt = &raw[lev][q][t.base];
        half_t* oq = ob + q * p.o_p + lev * p.o_l;
        for (int pos = g; pos < DO * DO; pos += GR) {
            const int bx = pos / DO, a = pos - bx * DO;
            const half_t* c = rt + a * t.bw + bx;
            half_t v = hmul(t.w00, c[0]);
            v = hadd(v, hmul(t.w01, c[1]));
            v = hadd(v, hmul(t.w10, c[t.bw]));
            v = hadd(v, hmul(t.w11, c[t.bw + 1]));
            oq[bx * p.o_x + a * p.o_y] = v;
        }
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
    if (gsz[2] != 128 || fsz[2] != gsz[2]) return false;
    if (fst[2] != 1) return false;  // channel-last storage
    if (fst[0] % 8 || fst[1] % 8 || fst[3] % 8 || fst[4] % 8) return false;  // 16-byte aligned pixels
    return true;
}

int launch_fast(int nlev, const void* gmap, const int64_t* gsz, const int64_t* gst, const void* const* fmaps,
                const int64_t* fsz, const int64_t* fst, const float* scales, const float* coords, const int64_t* csz,
                const int64_t* cst, const int64_t* ii, const int64_t* jj, void* out, const int64_t* ostr,
                hipStream_t stream, const void* table = nullptr)
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
    {
        // patch features as a scalar-load table: the caller's (dpvo_corr_pack), or
        // packed here into stream-ordered scratch
        void* tab = nullptr;
        if (table) {
            p.f1tab = (const uint32_t*)table;
        } else {
            const size_t tab_bytes = (size_t)p.B * p.N1 * p.C * 5 * 4;
            if (hipMallocAsync(&tab, tab_bytes, stream) != hipSuccess) return 2;
            const int64_t np = (int64_t)p.B * p.N1 * p.C;
            hipLaunchKernelGGL(corr_pack_kernel, dim3(grid_for(np, 256, 8192)), dim3(256), 0, stream, p.gmap,
                               p.g_s[0], p.g_s[1], p.g_s[2], p.g_s[3], p.g_s[4], p.B, p.N1, p.C, (uint32_t*)tab);
            p.f1tab = (const uint32_t*)tab;
        }
        if (nlev == 2)
            hipLaunchKernelGGL((corr_sfast_kernel<2, 16>), dim3((unsigned)nblk), dim3(FastThreads<2>::value), 0,
                               stream, p);
        else
            hipLaunchKernelGGL((corr_sfast_kernel<1, 16>), dim3((unsigned)nblk), dim3(FastThreads<1>::value), 0,
                               stream, p);
        if (tab) (void)hipFreeAsync(tab, stream);
    }
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
    return dpvo_corr_forward_pyramid_ld(dtype, gmap, gmap_size, gmap_stride, nlev, fmaps, fmap_sizes, fmap_strides,
                                        level_scale, coords, coords_size, coords_stride, ii, jj, radius, corr, 0,
                                        nullptr, stream);
}

extern "C" int dpvo_corr_forward_pyramid_ld(int dtype, const void* gmap, const int64_t* gmap_size,
                                            const int64_t* gmap_stride, int nlev, const void* const* fmaps,
                                            const int64_t* fmap_sizes, const int64_t* fmap_strides,
                                            const float* level_scale, const float* coords,
                                            const int64_t* coords_size, const int64_t* coords_stride,
                                            const int64_t* ii, const int64_t* jj, int radius, void* corr,
                                            int64_t edge_stride, const void* table, void* stream)
{
    DPVO_CHECK_ARG(check_common(dtype, gmap, gmap_size, coords_size, ii, jj, radius, corr),
                   "invalid arguments (dtype/radius/shapes)");
    DPVO_CHECK_ARG(nlev >= 1 && nlev <= 8 && fmaps && level_scale, "nlev must be 1..8");
    const int Do = 2 * radius + 1;
    const int64_t P2 = coords_size[3] * coords_size[4];
    const int64_t E = coords_size[1];
    // output: [B][E][x][y][P][P][L], edges edge_stride elements apart (0: packed)
    const int64_t o_row = (int64_t)Do * Do * P2 * nlev;
    DPVO_CHECK_ARG(edge_stride == 0 || edge_stride >= o_row, "edge_stride smaller than one edge's features");
    const int64_t o_e = edge_stride ? edge_stride : o_row;
    bool all_fast = nlev <= 2;
    for (int l = 0; l < nlev && all_fast; l++)
        all_fast = fast_path_ok(dtype, gmap_size, fmap_sizes + 5 * l, fmap_strides + 5 * l, coords_size, radius) &&
                   fmap_sizes[5 * l] == coords_size[0];
    if (all_fast) {
        const int64_t ostr[6] = {E * o_e, o_e, 1, Do * P2 * nlev, P2 * nlev, nlev};
        const int rc = launch_fast(nlev, gmap, gmap_size, gmap_stride, fmaps, fmap_sizes, fmap_strides, level_scale,
                                   coords, coords_size, coords_stride, ii, jj, corr, ostr, as_stream(stream), table);
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

extern "C" size_t dpvo_corr_table_bytes(const int64_t* gmap_size)
{
    return (size_t)(gmap_size[0] * gmap_size[1] * gmap_size[2]) * 5 * 4;
}

extern "C" int dpvo_corr_pack(const void* gmap, const int64_t* gmap_size, const int64_t* gmap_stride, void* table,
                              void* stream)
{
    DPVO_CHECK_ARG(gmap && table, "null pointer");
    DPVO_CHECK_ARG(gmap_size[3] == 3 && gmap_size[4] == 3, "the packed table is for 3x3 patches");
    DPVO_CHECK_ARG(((uintptr_t)table & 15) == 0, "table must be 16-byte aligned");
    const int64_t np = gmap_size[0] * gmap_size[1] * gmap_size[2];
    if (np == 0) return 0;
    hipLaunchKernelGGL(corr_pack_kernel, dim3(grid_for(np, 256, 8192)), dim3(256), 0, as_stream(stream),
                       (const half_t*)gmap, gmap_stride[0], gmap_stride[1], gmap_stride[2], gmap_stride[3],
                       gmap_stride[4], (int)gmap_size[0], (int)gmap_size[1], (int)gmap_size[2], (uint32_t*)table);
    DPVO_CHECK_LAUNCH();
    return 0;
}

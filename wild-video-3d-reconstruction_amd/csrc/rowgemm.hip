// rowgemm.hip -- full-row MFMA GEMM with fused update-operator epilogues (gfx950).
//
// The learned update operator (reference dpvo/net.py:75-93, blocks.py) is a
// chain of Linear(384 -> 384) layers over E ~ 95k edge rows, glued by
// LayerNorm, ReLU/sigmoid, residual adds, gating and row gathers.  Under the
// reference's autocast every Linear is an fp16 GEMM (fp32 accumulate, fp16
// output) and every glue op is its own elementwise pass over E x 384 fp32.
//
// Here one kernel computes   Y = A W^T + b   for a tile of 128 rows and ALL
// 384 output columns, so any row-wise op can run in the epilogue:
//   y16 = fp16(acc + b)  [-> relu | sigmoid]          (autocast Linear output)
//   v   = y  | res32 + res16[idx] + y | res32 + fp16(gate16 * y)
//   v   = LayerNorm(v) [-> relu]                       (fp32, as autocast)
//   heads: d = W_d relu(v) + b_d, w = sigmoid(W_w relu(v) + b_w)  (fp16 out)
//   out32 = v, out16 = fp16(v)
// A rows may be gathered through an index (idx < 0 -> a zero row), which
// fuses `mask_ix * net[:, ix]` (net.py:82-85) into the GEMM's operand load.
//
// Tiling: 512 threads = 8 waves as 2 (M) x 4 (N); wave tile 64 x 96 =
// 4 x 6 mfma_f32_16x16x32_f16 accumulators.  BK = 64; A (16 KB) and W (48 KB)
// stages are staged global -> LDS by global_load_lds (16 B per lane, source
// pre-swizzled, conflict-free ds_read_b128 fragment reads), two stages in
// flight.  Persistent blocks walk a flat (tile, k-stage) sequence, so the next
// tile's first stage loads during the current tile's epilogue.
#include "common.hpp"

#include <algorithm>
#include <stdlib.h>
#include <type_traits>

namespace dpvo {
namespace {

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

constexpr int RG_BM = 128, RG_BN = 384, RG_BK = 64, RG_THREADS = 512;
constexpr int RG_A_STAGE = RG_BM * RG_BK * 2;   // 16 KB
constexpr int RG_W_STAGE = RG_BN * RG_BK * 2;   // 48 KB

enum {
    RG_RELU = DPVO_RG_RELU, RG_SIGMOID = DPVO_RG_SIGMOID, RG_RES = DPVO_RG_RES, RG_GATE = DPVO_RG_GATE,
    RG_LN = DPVO_RG_LN, RG_LN_RELU = DPVO_RG_LN_RELU, RG_HEADS = DPVO_RG_HEADS,
    RG_NOADD = 1 << 20   // (device side only) RES without a res16 addend: + 0 in its place, no loads
};

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));   // (no old operand)
}
// all-reduce over a DPP row (16 lanes) by rotations: every lane gets the sum
__device__ __forceinline__ float rowsum16(float s)
{
    s += dpp_f<0x128>(s);
    s += dpp_f<0x124>(s);
    s += dpp_f<0x122>(s);
    s += dpp_f<0x121>(s);
    return s;
}

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base)
{
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ float hround(float v) { return (float)(half_t)v; }


__device__ __forceinline__ float fast_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// ---- the row epilogue with two rows per wave (v3 / rowchain): half h = lane/32
// takes row 2i + h, lane s = lane%32 of the half owns columns 4s + 128j (j < 3),
// so every global access is a 16-byte (fp32) or 8-byte (fp16) vector -- half
// the store instructions of the one-row-per-wave layout above, whose
// completions every next-tile k-step wait includes (one vmcnt for loads and
// stores).  Row sums: a DPP row reduce plus one gfx950 lane swap (a + b == b + a,
// so every lane of the half agrees).
typedef float ep_f4 __attribute__((ext_vector_type(4)));
typedef _Float16 ep_h4 __attribute__((ext_vector_type(4)));

struct EpiConsts2 {
    ep_f4 g[3], b[3];     // LayerNorm weight / bias at this lane's columns
    ep_f4 hw[4][3];       // head weights (fp16 values)
    float hb[4];
};

template <int FLAGS>
__device__ __forceinline__ void load_consts2(const dpvo_rowgemm_args& p, int lane, EpiConsts2& k)
{
    const int s = lane & 31;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const int c = 128 * j + 4 * s;
        if (FLAGS & RG_LN) {
            k.g[j] = *(const ep_f4*)(p.ln_g + c);
            k.b[j] = *(const ep_f4*)(p.ln_b + c);
        }
        if (FLAGS & RG_HEADS) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const ep_h4 w = *(const ep_h4*)((const half_t*)p.head_w + q * RG_BN + c);
                k.hw[q][j] = ep_f4{(float)w[0], (float)w[1], (float)w[2], (float)w[3]};
            }
        }
    }
    if (FLAGS & RG_HEADS) {
#pragma unroll
        for (int q = 0; q < 4; q++) k.hb[q] = (float)((const half_t*)p.head_b)[q];
    }
}

__device__ __forceinline__ float half_sum(float x)
{
    x = rowsum16(x);
    auto h = __builtin_amdgcn_permlane16_swap(__float_as_int(x), __float_as_int(x), false, false);
    return __int_as_float(h[0]) + __int_as_float(h[1]);
}

template <int R>   // R rows = R/2 row pairs
struct EpiOps2 {
    ep_f4 base[R / 2][3];   // res32
    ep_h4 add[R / 2][3];    // res16[idx] or gate16
};

// A row of zeros the epilogue reads in place of an absent res16 row: the add
// registers are then always load destinations (a zero-fill branch beside the
// load made the compiler drain every outstanding load -- the chain's W / A
// prefetch included -- before each OVL batch, to order the zero writes after
// the registers' previous loads).
__device__ half_t g_epi_zero_row[RG_BN];   // (device globals start zeroed)

template <int FLAGS, int R>
__device__ __forceinline__ void epi2_load(const dpvo_rowgemm_args& p, int64_t M, int64_t row0, int lane, EpiOps2<R>& o)
{
    if (!(FLAGS & (RG_RES | RG_GATE))) return;
    const int h = lane >> 5, s = lane & 31;
#pragma unroll
    for (int i = 0; i < R / 2; i++) {
        const int64_t rr = row0 + 2 * i + h;
        const int64_t row = rr < M ? rr : M - 1;   // clamped for loads; stores skip rows >= M
        const float* r32 = (const float*)p.res32 + row * p.ldr;
        const half_t* r16 = g_epi_zero_row;
        if (FLAGS & RG_GATE) {
            r16 = (const half_t*)p.gate16 + row * RG_BN;
        } else if (p.res16) {
            const int64_t src = p.res16_idx ? p.res16_idx[row] : row;
            if (src >= 0) r16 = (const half_t*)p.res16 + src * RG_BN;
        }
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int c = 128 * j + 4 * s;
            o.base[i][j] = *(const ep_f4*)(r32 + c);
            if (!(FLAGS & RG_NOADD)) o.add[i][j] = *(const ep_h4*)(r16 + c);
        }
    }
}

// yget(i, j): the fp16 y of row 2 i + h, columns 128 j + 4 s .. + 3 (from the
// y tile in LDS, or from registers in the warp-specialised chain)
template <int FLAGS, int R, typename YGet>
__device__ __forceinline__ void epi2_finish(const dpvo_rowgemm_args& p, int64_t M, YGet yget, int64_t row0, int lane,
                                            const EpiConsts2& k, const EpiOps2<R>& o)
{
    const int h = lane >> 5, s = lane & 31;
    ep_f4 v[R / 2][3];
#pragma unroll
    for (int i = 0; i < R / 2; i++) {
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const ep_h4 y = yget(i, j);
            v[i][j] = ep_f4{(float)y[0], (float)y[1], (float)y[2], (float)y[3]};
        }
    }
    if (FLAGS & (RG_RES | RG_GATE)) {
#pragma unroll
        for (int i = 0; i < R / 2; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) {
                // (NOADD: + 0.f as the zero row's addend -- -0 + 0 is +0, kept bit for bit)
                const ep_f4 add = (FLAGS & RG_NOADD) ? ep_f4{0.f, 0.f, 0.f, 0.f}
                                                     : ep_f4{(float)o.add[i][j][0], (float)o.add[i][j][1],
                                                             (float)o.add[i][j][2], (float)o.add[i][j][3]};
                if (FLAGS & RG_GATE) {   // x + fp16(gate * res)   (blocks.py:30, fp16 product)
#pragma unroll
                    for (int t = 0; t < 4; t++) v[i][j][t] = o.base[i][j][t] + hround(add[t] * v[i][j][t]);
                } else {                 // (res32 + res16) + y
                    v[i][j] = (o.base[i][j] + add) + v[i][j];
                }
            }
    }
    if (FLAGS & RG_LN) {
#pragma unroll
        for (int i = 0; i < R / 2; i++) {
            float sm = 0.f;
#pragma unroll
            for (int j = 0; j < 3; j++) sm += (v[i][j][0] + v[i][j][1]) + (v[i][j][2] + v[i][j][3]);
            const float mean = half_sum(sm) * (1.f / RG_BN);
            float sq = 0.f;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const ep_f4 d = v[i][j] - mean;
                sq += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
            }
            const float rstd = rsqrtf(half_sum(sq) * (1.f / RG_BN) + p.ln_eps);
#pragma unroll
            for (int j = 0; j < 3; j++) {
                v[i][j] = (v[i][j] - mean) * rstd * k.g[j] + k.b[j];
                if (FLAGS & RG_LN_RELU)
#pragma unroll
                    for (int t = 0; t < 4; t++) v[i][j][t] = fmaxf(v[i][j][t], 0.f);
            }
        }
    }
    if (FLAGS & RG_HEADS) {
        // d = W_d relu(v) + b_d ; w = sigmoid(W_w relu(v) + b_w)   (fp16 operands, fp32 accumulate)
#pragma unroll
        for (int i = 0; i < R / 2; i++) {
            float d[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 3; j++)
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const float x = hround(fmaxf(v[i][j][t], 0.f));
#pragma unroll
                    for (int q = 0; q < 4; q++) d[q] += x * k.hw[q][j][t];
                }
            half_t ho[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                float z = hround(half_sum(d[q]) + k.hb[q]);
                if (q >= 2) z = hround(fast_sigmoid(z));
                ho[q] = (half_t)z;
            }
            const int64_t row = row0 + 2 * i + h;
            if (s == 0 && row < M) *(ep_h4*)((half_t*)p.head_out + row * 4) = ep_h4{ho[0], ho[1], ho[2], ho[3]};
        }
    }
#pragma unroll
    for (int i = 0; i < R / 2; i++) {
        const int64_t row = row0 + 2 * i + h;
        if (row >= M) continue;
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int c = 128 * j + 4 * s;
            if (p.out32) *(ep_f4*)((float*)p.out32 + row * p.ldo32 + c) = v[i][j];
            if (p.out16)
                *(ep_h4*)((half_t*)p.out16 + row * p.ldo16 + c) =
                    ep_h4{(half_t)v[i][j][0], (half_t)v[i][j][1], (half_t)v[i][j][2], (half_t)v[i][j][3]};
        }
    }
}

template <int FLAGS, int R, typename YMap>
__device__ __forceinline__ void epilogue_rows2(const dpvo_rowgemm_args& p, int64_t M, const char* smem, YMap ym,
                                               int lrow0, int64_t row0, int lane, const EpiConsts2& k)
{
    EpiOps2<R> o;
    epi2_load<FLAGS, R>(p, M, row0, lane, o);
    const int h = lane >> 5, s = lane & 31;
    epi2_finish<FLAGS, R>(
        p, M, [&](int i, int j) { return *(const ep_h4*)(smem + ym.off(lrow0 + 2 * i + h, (128 * j + 4 * s) * 2)); },
        row0, lane, k, o);
}


// ---------------------------------------------------------------------------
// v3: the v1 tiling (128 x 384, 8 waves, BK = 64) with the A stream prefetched
// TWO stages ahead instead of one.  A (the activations, 73 MB per layer at C3)
// is the HBM stream; W (295 KB) is L2-resident.  In v1 a stage holds A and W
// together, so one stage of lookahead leaves only 16 KB of A in flight per CU
// (4 MB chip-wide, ~2 TB/s at HBM latency).  Here W has 2 slots (48 KB) and A
// a ring of 3 (16 KB), issued in the order W(i+1), A(i+2): the wait for step i
// (vmcnt 10) then leaves A(i+1) and A(i+2) in flight.  The 96 KB y tile no
// longer fits beside the rings, so the epilogue runs in two 64-row halves
// through the consumed W slot.
// ---------------------------------------------------------------------------
constexpr int R3_W_SLOT = RG_W_STAGE;            // 48 KB
constexpr int R3_A_BASE = 2 * R3_W_SLOT;         // A ring after the two W slots
constexpr int R3_LDS = R3_A_BASE + 3 * RG_A_STAGE;   // 144 KB

struct YMapSlot {   // 64 rows x 768 B in one W slot, 32-B granules XOR (row/4)&3
    int base;
    __device__ int off(int r, int byte) const { return base + r * 768 + (byte ^ (((r >> 2) & 3) << 5)); }
};

template <int FLAGS, bool DUAL = false>
__global__ __launch_bounds__(RG_THREADS, 1) void rowgemm3_kernel(dpvo_rowgemm_args p, dpvo_rowgemm_args p2)
{
    __shared__ __attribute__((aligned(16))) char smem[R3_LDS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int K = p.K;
    const int ksteps = K / RG_BK;
    const int64_t Mrows = p.M_dev ? min(*p.M_dev, p.M) : p.M;
    const int64_t ntiles = (Mrows + RG_BM - 1) / RG_BM;
    if ((int64_t)blockIdx.x >= ntiles) return;
    // DUAL: a second GEMM on the same A (p2's W, bias, outputs): every tile runs
    // twice in a row, the second pass's A stream hitting L2
    const int64_t my_tiles = ((ntiles - 1 - blockIdx.x) / gridDim.x + 1) << (DUAL ? 1 : 0);
    const int64_t total = my_tiles * ksteps;
    const int64_t wdelta = DUAL ? (const half_t*)p2.W - (const half_t*)p.W : 0;

    const half_t* __restrict__ Wt = (const half_t*)p.W;
    const half_t* __restrict__ zero = (const half_t*)p.zero_row;
    const int srow = lane >> 3, pch = lane & 7;
    const half_t* wsrc[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const int n = (wave * 6 + j) * 8 + srow;
        wsrc[j] = Wt + (int64_t)n * K + 8 * (pch ^ ((n >> 1) & 7));
    }
    // A rows of the tile a flat step belongs to (two tiles can be in flight)
    auto a_src = [&](int64_t tile, int j) {
        const int r = (wave * 2 + j) * 8 + srow;
        const int64_t m = tile * RG_BM + r;
        const half_t* row = zero;
        if (m < Mrows) {
            const int64_t s = p.a_idx ? p.a_idx[m] : m;
            if (s >= 0 && s < p.a_rows) row = (const half_t*)p.A + s * p.lda;
        }
        return row + 8 * (pch ^ ((r >> 1) & 7));
    };
    // flat step f -> (tile, k-step) of this block
    auto tile_of = [&](int64_t f) { return (int64_t)blockIdx.x + ((f / ksteps) >> (DUAL ? 1 : 0)) * gridDim.x; };
    auto second = [&](int64_t f) { return DUAL && ((f / ksteps) & 1); };
    const half_t* asrc[2];
    int64_t asrc_tile = -1;
    auto issue_a = [&](int64_t f) {
        const int64_t t = tile_of(f);
        if (t != asrc_tile) {
            asrc[0] = a_src(t, 0);
            asrc[1] = a_src(t, 1);
            asrc_tile = t;
        }
        char* sA = smem + R3_A_BASE + (int)(f % 3) * RG_A_STAGE;
        const int k0 = (int)(f % ksteps) * RG_BK;
        glds16(asrc[0] + k0, sA + (wave * 2 + 0) * 1024);
        glds16(asrc[1] + k0, sA + (wave * 2 + 1) * 1024);
    };
    auto issue_w = [&](int64_t f) {
        char* sW = smem + (int)(f & 1) * R3_W_SLOT;
        const int64_t k0 = (f % ksteps) * RG_BK + (second(f) ? wdelta : 0);
#pragma unroll
        for (int j = 0; j < 6; j++) glds16(wsrc[j] + k0, sW + (wave * 6 + j) * 1024);
    };

    f4_t acc[4][6];
#pragma unroll
    for (int mt = 0; mt < 4; mt++)
#pragma unroll
        for (int nt = 0; nt < 6; nt++) acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fq = lane >> 4;
    int a_off[4], w_off[6], a_sw[4], w_sw[6];
#pragma unroll
    for (int mt = 0; mt < 4; mt++) {
        const int row = wm * 64 + mt * 16 + fr;
        a_off[mt] = row * 128;
        a_sw[mt] = (row >> 1) & 7;
    }
#pragma unroll
    for (int nt = 0; nt < 6; nt++) {
        const int n = wn * 96 + nt * 16 + fr;
        w_off[nt] = n * 128;
        w_sw[nt] = (n >> 1) & 7;
    }

    EpiConsts2 kc;
    load_consts2<FLAGS>(p, lane, kc);
    // prologue: A(0), W(0), A(1) -- then every step issues W(i+1), A(i+2)
    issue_a(0);
    issue_w(0);
    if (total > 1) issue_a(1);
    for (int64_t i = 0; i < total; i++) {
        const bool w_next = i + 1 < total, a_next = i + 2 < total;
        if (w_next) issue_w(i + 1);
        if (a_next) issue_a(i + 2);
        // outstanding after W(i): A(i+1) [2], W(i+1) [6], A(i+2) [2]
        if (a_next)
            asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        else if (w_next)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* sA = smem + R3_A_BASE + (int)(i % 3) * RG_A_STAGE;
        const char* sW = smem + (int)(i & 1) * R3_W_SLOT;
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
            const int c = kk * 4 + fq;
            h8_t a[4], b[6];
#pragma unroll
            for (int mt = 0; mt < 4; mt++) a[mt] = *(const h8_t*)(sA + a_off[mt] + 16 * (c ^ a_sw[mt]));
#pragma unroll
            for (int nt = 0; nt < 6; nt++) b[nt] = *(const h8_t*)(sW + w_off[nt] + 16 * (c ^ w_sw[nt]));
            // W as the first operand: the accumulator is the transposed tile, lane
            // (fr, fq) holding row fr, columns 4 fq .. 4 fq + 3 of each 16 x 16 block
#pragma unroll
            for (int mt = 0; mt < 4; mt++)
#pragma unroll
                for (int nt = 0; nt < 6; nt++)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[nt], a[mt], acc[mt][nt], 0, 0, 0);
        }
        __builtin_amdgcn_s_barrier();
        if ((int)(i % ksteps) != ksteps - 1) continue;

        // ---- epilogue of tile t.  y16 = act(fp16(acc + b)): four consecutive
        // columns of one row per (m-tile, n-tile) and lane.
        const int64_t cur_tile = tile_of(i);
        const bool sec = second(i);
        const dpvo_rowgemm_args& pe = sec ? p2 : p;
        typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
        h4_t y16[4][6];
#pragma unroll
        for (int nt = 0; nt < 6; nt++) {
            const h4_t bias = *(const h4_t*)((const half_t*)pe.bias + wn * 96 + nt * 16 + 4 * fq);
#pragma unroll
            for (int mt = 0; mt < 4; mt++) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    half_t y = (half_t)(acc[mt][nt][r] + (float)bias[r]);
                    if (FLAGS & RG_RELU) y = y > (half_t)0 ? y : (half_t)0;
                    if (FLAGS & RG_SIGMOID) y = (half_t)fast_sigmoid((float)y);
                    y16[mt][nt][r] = y;
                    acc[mt][nt][r] = 0.f;
                }
            }
        }
        // Two 64-row halves through the consumed W slot (whole-row stores are
        // coalesced; 8-byte stores straight from the accumulator layout measured
        // slower even with no row-wise op).  Half h holds tile rows
        // {64 w + 32 h + [0, 32)}, w = 0, 1: every wave writes its m-tiles 2h,
        // 2h+1, so only half of y16 stays live across the first half's row pass.
        const YMapSlot ym{(int)(i & 1) * R3_W_SLOT};
#pragma unroll
        for (int h = 0; h < 2; h++) {
#pragma unroll
            for (int nt = 0; nt < 6; nt++) {
                const int col = wn * 96 + nt * 16 + 4 * fq;
#pragma unroll
                for (int mm = 0; mm < 2; mm++)
                    *(h4_t*)(smem + ym.off(wm * 32 + mm * 16 + fr, col * 2)) = y16[2 * h + mm][nt];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            // rows per batch (register budget: half of y16 is still live here)
            constexpr int RB = (FLAGS & (RG_RES | RG_GATE | RG_LN)) ? ((FLAGS & (RG_LN | RG_HEADS)) ? 2 : 4) : 8;
            const int lr = wave * 8;                                             // 8 rows inside one 32-row block
            const int64_t row0 = cur_tile * RG_BM + (lr >> 5) * 64 + h * 32 + (lr & 31);
#pragma unroll
            for (int q0 = 0; q0 < 8; q0 += RB)
                epilogue_rows2<FLAGS, RB>(pe, Mrows, smem, ym, lr + q0, row0 + q0, lane, kc);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
    }
}

// ---------------------------------------------------------------------------
// Chained pair: Y = epi2(act1(A W1^T + b1) W2^T + b2) with the 128 x 384
// intermediate kept in LDS -- the update operator's Linear -> ReLU -> Linear
// pairs (corr0/corr1, c1, c2, the GRU res branches; net.py:53-56,
// blocks.py:27-30), whose 73 MB intermediates otherwise round-trip HBM.
// (rowchain5_kernel below; the y tile is GEMM2's A operand, then its output
// for the row epilogue.)
// ---------------------------------------------------------------------------


// chunk swizzle of the BK = 32 stage rows (64 B = four 16-byte chunks): the
// physical chunk p of row r holds logical chunk p ^ rc_sw(r), with rc_sw =
// [0, 2, 3, 1][(r >> 2) & 3].  Each ds_read_b128 lane group ({0-3, 12-15,
// 20-27}, ...) reads rows fr = lane & 15 at chunk fq = lane >> 4; with this
// permutation its 16 lanes hit 16 distinct 16-byte bank slots (the plain
// (r >> 2) & 3 xor put two lanes on each slot: 2-way conflicts on every
// fragment read, 46 % of the chain kernels' LDS cycles).
__device__ __forceinline__ int rc_sw(int r) { return (0x78 >> (((r >> 2) & 3) << 1)) & 3; }

#ifdef DPVO_STAMPS
// Diagnostic build only (never the product library): per-wave cycle sums of
// the chain kernels' k-loop segments, s_memtime stamps (cdna guide, In-kernel
// stamps).  dpvo_stamps[block][wave][segment].
constexpr int ST_SEGS = 16;
__device__ unsigned long long dpvo_stamps[1024 * 8 * ST_SEGS];
#define RC_STAMP(v)                                                                            \
    unsigned long long v;                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");                  \
    __builtin_amdgcn_sched_barrier(0);
#define RC_ACC(seg, a, b) st_sum[seg] += (b) - (a);
#else
#define RC_STAMP(v)
#define RC_ACC(seg, a, b)
#endif

struct YMapChunk {   // 128 rows x 768 B, 16-byte chunks XOR (row & 15): conflict-free
    // ds_read_b128 fragment reads down 16 rows and 256-byte row sweeps
    __device__ int off(int r, int byte) const { return r * 768 + (((byte >> 4) ^ (r & 15)) << 4) + (byte & 15); }
};

// GATED (the GRU's GatedResidual, blocks.py:27-30): after GEMM2 has put y in
// the y tile, a third GEMM on the same A (re-read from L2) gives
// gate = sigmoid(A Wg^T + bg) in the accumulators, and every lane rewrites its
// own y tile elements as fp16(gate * y) -- the epilogue then adds them to the
// residual like RES, which is bit-for-bit the GATE epilogue's
// x + fp16(gate * y) without the 73 MB gate16 round trip (nor a gate held in
// registers across the GEMMs).
// TRI (the corr MLP of net.py:54-61 and the `norm(net + inp + corr(.))` of
// :78-79 in one launch): pg is then the MIDDLE Linear -- GEMM2 runs with pg's
// W and bias, its y tile gets pg's row epilogue in place (LayerNorm -> ReLU,
// rounded to fp16: the A operand the next Linear casts to under autocast),
// then a third GEMM on that tile with p's W and bias feeds p's epilogue.
// Bit-identical to rowchain (corr0, corr1, LN|LN_RELU) -> fp16 rows ->
// rowgemm (corr2, RES|LN): the same MFMA k order and the same epilogue code.
// ---------------------------------------------------------------------------
// v5 (round 4): the plain GEMM (flags 0 / RELU / SIGMOID) with a k-blocked W
// and no LDS-DMA:
//   * 8 waves as 1 (M) x 8 (N), wave tile 128 x 48 (8 x 3 accumulators), BK 32:
//     every W fragment is read by one wave only (24 KB per k-step and CU from
//     L2; the 2 x 4 layout read each twice: 93 -> 85 us for the SoftAgg pair);
//   * W ([K/32][384][32]: a fragment = one contiguous 1 KB, whole lines)
//     streams from L2 straight into registers, two k-steps ahead -- no LDS
//     traffic for W;
//   * A (128 rows x 64 B per k-step) goes global -> registers -> a 4-slot LDS
//     ring (register staging, four k-steps ahead; rc_sw chunk swizzle,
//     conflict-free fragment reads);
//   * one barrier per TWO k-steps (in-kernel stamps: with one per k-step the
//     waves of a SIMD met at every step, the younger ~500 cycles behind); every
//     wait is the compiler's exact count of the wave's own loads and stores;
//   * the row epilogue stages y16 through a 96 KB LDS tile and stores whole
//     rows, with the next tile's first loads already in flight ahead of it.
// (Measured and not kept: W / A prefetched three or four k-steps ahead -- the
// vmcnt waits are ~10 % of a k-step, no gain; the next k-step's fragments read
// between this one's MFMAs -- 79 -> 91 us.)
// Persistent blocks walk a flat (tile, pass, k-step) sequence; DUAL runs a
// second GEMM (p2's W, bias, out16) on the same A tile right after the first.
// Per output element the MFMA k order is rowgemm3's: the same bits.
// ---------------------------------------------------------------------------
// f(integral_constant<int, K>) for K = B .. E-1, expanded at compile time
template <int B, int E>
struct bd_steps {
    template <class F>
    __device__ __forceinline__ static void run(F&& f)
    {
        if constexpr (B < E) {
            f(std::integral_constant<int, B>{});
            bd_steps<B + 1, E>::run(f);
        }
    }
};
constexpr int R5_THREADS = 512, R5_BK = 32;
constexpr int R5_Y = RG_BM * 768;                  // 96 KB
constexpr int R5_ASLOT = RG_BM * R5_BK * 2;        // 8 KB
constexpr int R5_LDS = R5_Y + 4 * R5_ASLOT;        // 128 KB

// (tile, pass, k-step) of a flat step, advanced one step at a time (no
// 64-bit divisions); past the end it stays on the last step
struct R5Cursor {
    int64_t f, t;
    int k, q;
    __device__ __forceinline__ void next(int64_t total, int nks, int np, unsigned grid)
    {
        if (f + 1 >= total) return;
        f++;
        if (++k == nks) {
            k = 0;
            if (++q == np) {
                q = 0;
                t += grid;
            }
        }
    }
};

// PRE (dpvo_rowgemm_pair_pre): the A rows are formed while they are staged,
// A[m] = fp16(pre.a[m] + pre.b16[pre.b_idx[m]]) -- rowadd_ln's fp32 add and
// rounding (net + agg_kk(net), net.py:87 -> the agg_ij SoftAgg's f / g
// operand) without its 73 MB fp16 rows round-tripping HBM.
struct R5PreRaw {
    f4_t lo, hi;   // 8 fp32 of pre.a
    h8_t b;        // 8 fp16 of the gathered addend, or -0 (a row without one)
};
// The addend of a row without one: -0, so that v + b == v for every v (rowadd_ln
// then adds nothing; a +0 would turn -0 into +0)
struct R5NegZeroRow {
    unsigned short v[RG_BN];
    constexpr R5NegZeroRow() : v{}
    {
        for (int i = 0; i < RG_BN; i++) v[i] = 0x8000;
    }
};
// (a non-const __device__ object: global address space, so that a pointer to
// it or to an addend row stays a global pointer -- a constant one made the
// loads through it flat loads)
__device__ R5NegZeroRow g_pre_negzero = R5NegZeroRow{};
constexpr int R5_PRE_IDX_TILES = 8;   // PRE: tiles per block whose addend sources sit in LDS
template <bool PRE>
using r5_areg_t = std::conditional_t<PRE, R5PreRaw, h8_t>;
__device__ __forceinline__ h8_t r5_cvt(const h8_t& x) { return x; }
__device__ __forceinline__ h8_t r5_cvt(const R5PreRaw& x)
{
    h8_t y;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        y[i] = (half_t)(x.lo[i] + (float)x.b[i]);
        y[4 + i] = (half_t)(x.hi[i] + (float)x.b[4 + i]);
    }
    return y;
}

template <int FLAGS, bool DUAL>
__global__ __launch_bounds__(R5_THREADS, 1) void rowgemm5_kernel(dpvo_rowgemm_args p, dpvo_rowgemm_args p2)
{
    static_assert((FLAGS & ~(RG_RELU | RG_SIGMOID)) == 0, "v5: plain GEMMs only");
    __shared__ __attribute__((aligned(16))) char smem[R5_LDS];
    typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int K = p.K, nks = K / R5_BK;
    const int64_t Mrows = p.M_dev ? min(*p.M_dev, p.M) : p.M;
    const int64_t ntiles = (Mrows + RG_BM - 1) / RG_BM;
    if ((int64_t)blockIdx.x >= ntiles) return;
    constexpr int NP = DUAL ? 2 : 1;
    const int64_t my_tiles = (ntiles - 1 - blockIdx.x) / gridDim.x + 1;
    const int64_t total = my_tiles * NP * nks;   // flat k-steps of this block
    const YMapChunk ym;
    const int fr = lane & 15, fq = lane >> 4;
    const half_t* __restrict__ zero = (const half_t*)p.zero_row;
    // ---- A staging: lane holds row 16 w + (lane >> 2), logical chunk lane & 3
    const int ar = 16 * w + (lane >> 2), ac = lane & 3;

    int64_t a_tile = -1;
    const half_t* arow = zero;
    auto a_row = [&](int64_t t) __attribute__((always_inline)) {
        if (t == a_tile) return;
        a_tile = t;
        const int64_t m = t * RG_BM + ar;
        const half_t* row = zero;
        if (p.a_idx) {   // (the index load's wait inside the branch, not at the join)
            if (m < Mrows) {
                const int64_t src = p.a_idx[m];
                if (src >= 0 && src < p.a_rows) row = (const half_t*)p.A + src * p.lda;
            }
        } else if (m < Mrows && m < p.a_rows) {
            row = (const half_t*)p.A + m * p.lda;
        }
        arow = row + 8 * ac;
    };
    h8_t areg[2];
    auto load_a = [&](const R5Cursor& c) __attribute__((always_inline)) -> h8_t {
        a_row(c.t);
        return *(const h8_t*)(arow + c.k * R5_BK);
    };
    // slot image: row r, physical chunk ac ^ rc_sw(r) holds logical chunk ac
    const int aw_off = ar * 64 + 16 * (ac ^ rc_sw(ar));
    // ---- W fragments: column 48 w + 16 nt + fr, k 8 fq .. 8 fq + 7 of the step
    h8_t wreg[2][3];
    const half_t* W1 = (const half_t*)p.W;
    const half_t* W2 = DUAL ? (const half_t*)p2.W : W1;
    const int wcol = (48 * w + fr) * R5_BK + 8 * fq;
    auto load_w = [&](const R5Cursor& c, h8_t (&r)[3]) __attribute__((always_inline)) {
        const half_t* src = (DUAL && c.q ? W2 : W1) + (int64_t)c.k * (RG_BN * R5_BK) + wcol;
#pragma unroll
        for (int nt = 0; nt < 3; nt++) r[nt] = *(const h8_t*)(src + nt * 16 * R5_BK);
    };
    // ---- biases of this wave's columns, both passes
    h4_t bias[NP][3];
#pragma unroll
    for (int q = 0; q < NP; q++)
#pragma unroll
        for (int nt = 0; nt < 3; nt++)
            bias[q][nt] = *(const h4_t*)((const half_t*)(q ? p2.bias : p.bias) + 48 * w + 16 * nt + 4 * fq);
    f4_t acc[8][3];
#pragma unroll
    for (int mt = 0; mt < 8; mt++)
#pragma unroll
        for (int nt = 0; nt < 3; nt++) acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
    const int ar_off = fr * 64 + 16 * (fq ^ rc_sw(fr));   // + 1024 mt: row 16 mt + fr

    auto epilogue = [&](int64_t t, auto qc) __attribute__((always_inline)) {
        constexpr int q = decltype(qc)::value;
        const dpvo_rowgemm_args& pe = q ? p2 : p;
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
            const int col = 48 * w + 16 * nt + 4 * fq;
            const h4_t bq = bias[q][nt];
#pragma unroll
            for (int mt = 0; mt < 8; mt++) {
                h4_t y;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    half_t v = (half_t)(acc[mt][nt][r] + (float)bq[r]);
                    if (FLAGS & RG_RELU) v = v > (half_t)0 ? v : (half_t)0;
                    if (FLAGS & RG_SIGMOID) v = (half_t)fast_sigmoid((float)v);
                    y[r] = v;
                }
                acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
                *(h4_t*)(smem + ym.off(16 * mt + fr, col * 2)) = y;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        // whole rows out: wave w stores rows 16 w .. 16 w + 15, one 768-byte
        // row per instruction (lanes 0-47, 16 bytes each: 16 stores per lane
        // instead of 24 of 8 bytes)
        half_t* out = (half_t*)pe.out16;
        if (((uintptr_t)out & 15) == 0 && (pe.ldo16 & 7) == 0) {
            if (lane < 48) {
#pragma unroll 4
                for (int i = 0; i < 16; i++) {
                    const int lr = 16 * w + i;
                    const int64_t row = t * RG_BM + lr;
                    const h8_t v = *(const h8_t*)(smem + ym.off(lr, 16 * lane));
                    if (row < Mrows) *(h8_t*)(out + row * pe.ldo16 + 8 * lane) = v;
                }
            }
        } else {   // 8-byte aligned rows: two rows per pass, 8 bytes per lane
            const int h = lane >> 5, s = lane & 31;
#pragma unroll 2
            for (int i = 0; i < 8; i++) {
                const int lr = 16 * w + 2 * i + h;
                const int64_t row = t * RG_BM + lr;
                ep_h4 v[3];
#pragma unroll
                for (int j = 0; j < 3; j++) v[j] = *(const ep_h4*)(smem + ym.off(lr, (128 * j + 4 * s) * 2));
                if (row < Mrows) {
#pragma unroll
                    for (int j = 0; j < 3; j++) *(ep_h4*)(out + row * pe.ldo16 + 128 * j + 4 * s) = v[j];
                }
            }
        }
    };

    // ---- prologue: stages 0, 1 into slots 0, 1; stages 2, 3 in registers
    // (stage g: slot g % 4, register set g % 2); W stages 0, 1 (stage f in
    // wreg[f % 2])
    const unsigned G = gridDim.x;
    R5Cursor cur{0, (int64_t)blockIdx.x, 0, 0};   // step f
    R5Cursor cw = cur, ca = cur;                   // W / A prefetch cursors
#pragma unroll
    for (int r = 0; r < 2; r++) {
        load_w(cw, wreg[r]);
        cw.next(total, nks, NP, G);
    }
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const h8_t x = load_a(ca);
        *(h8_t*)(smem + R5_Y + r * R5_ASLOT + aw_off) = x;
        ca.next(total, nks, NP, G);
    }
#pragma unroll
    for (int r = 0; r < 2; r++) {
        areg[r] = load_a(ca);
        ca.next(total, nks, NP, G);
    }
#ifdef DPVO_STAMPS
    unsigned long long st_sum[ST_SEGS] = {};
    RC_STAMP(t_begin)
#endif
    // one k-step, PH = f mod 4: stage f is read from slot f % 4 and, after
    // the MFMAs, stage f + 2 written into slot (f + 2) % 4.  One barrier per
    // TWO k-steps (even f): it makes stages f, f + 1 visible (written at the
    // ends of f - 2, f - 1) and frees slots (f + 2) % 4, (f + 3) % 4 (stages
    // f - 2, f - 1, read at f - 2, f - 1), so the waves of a SIMD may drift a
    // k-step apart between them.
    auto step = [&](auto ph) __attribute__((always_inline)) {
        constexpr int PH = decltype(ph)::value;
        constexpr int PR = PH & 1;
        RC_STAMP(s0)
        if (PR == 0) {
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_s_barrier();
        }
        RC_STAMP(s1)
#ifdef DPVO_STAMPS
        asm volatile("" ::"v"(wreg[PR][0]), "v"(wreg[PR][1]), "v"(wreg[PR][2]));
#endif
        RC_STAMP(s2)
        const char* sa = smem + R5_Y + PH * R5_ASLOT;
        h8_t a[8];
#pragma unroll
        for (int mt = 0; mt < 8; mt++) a[mt] = *(const h8_t*)(sa + ar_off + 1024 * mt);
#pragma unroll
        for (int nt = 0; nt < 3; nt++)
#pragma unroll
            for (int mt = 0; mt < 8; mt++)
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wreg[PR][nt], a[mt], acc[mt][nt], 0, 0, 0);
        // W(f + 2) is issued BEFORE A(f + 4): the MFMAs' wait on W(f) at step f
        // then never covers an HBM A load; only the ring write (after this
        // step's MFMAs) waits on its A stage
        load_w(cw, wreg[PR]);                                                  // W stage f + 2
        cw.next(total, nks, NP, G);
        __builtin_amdgcn_sched_barrier(0);
        *(h8_t*)(smem + R5_Y + ((PH + 2) & 3) * R5_ASLOT + aw_off) = areg[PR];   // stage f + 2
        areg[PR] = load_a(ca);                                                         // stage f + 4
        ca.next(total, nks, NP, G);
        RC_STAMP(s3)
        RC_ACC(0, s0, s1) RC_ACC(1, s1, s2) RC_ACC(2, s2, s3)
        if (cur.k == nks - 1) {
            if (DUAL && cur.q)
                epilogue(cur.t, std::integral_constant<int, DUAL ? 1 : 0>{});
            else
                epilogue(cur.t, std::integral_constant<int, 0>{});
            RC_STAMP(s4)
            RC_ACC(3, s3, s4)
        }
        cur.next(total, nks, NP, G);
    };
    for (int64_t f = 0; f < total; f += 4) {
        bd_steps<0, 4>::run([&](auto pc) __attribute__((always_inline)) {
            if (f + decltype(pc)::value < total) step(pc);
        });
    }
#ifdef DPVO_STAMPS
    RC_STAMP(t_end)
    st_sum[10] += t_end - t_begin;
    if (lane == 0)
        for (int k = 0; k < ST_SEGS; k++) dpvo_stamps[((int64_t)blockIdx.x * 8 + w) * ST_SEGS + k] = st_sum[k];
#endif
}

// ---------------------------------------------------------------------------
// rowpair6 (round 6): SoftAgg's f / g pair (rowgemm5 DUAL, K <= 384) with the
// whole A tile resident in LDS.  rowgemm5 streams A through a 4-slot ring and
// reads it twice, once per pass; the second read comes back from past L2 (the
// round-5 counters: 152 MB fetched for agg_kk's 73 MB operand, 345 MB for
// pair_pre's).  Here pass 0 stages every k-step of the tile into its own 8 KB
// slot (96 KB at K = 384), pass 1 runs on those slots with no loads and no
// barriers, and each pass's row epilogue goes out through half a y tile (48 KB,
// 64 rows at a time).  During pass 1 the next tile's first two A stages load
// into the registers the ring protocol uses; they reach slots 0 / 1 after pass
// 1's epilogue.  Same MFMA operands in the same k order, the same epilogue
// arithmetic: bit-identical to rowgemm5.
// ---------------------------------------------------------------------------
constexpr int P6_MAXK = 12;                                      // k-steps (K <= 384)
constexpr int P6_YH = P6_MAXK * R5_ASLOT;                        // half y tile after the A tile
constexpr int P6_IDX = P6_YH + 64 * 768;                         // PRE: addend sources
constexpr int P6_BIAS = P6_IDX + R5_PRE_IDX_TILES * RG_BM * 8;   // PRE: both passes' biases
constexpr int P6_LDS = P6_BIAS + 2 * RG_BN * 2;                  // 153.5 KB

template <bool PRE>
__global__ __launch_bounds__(R5_THREADS, 1) void rowpair6_kernel(dpvo_rowgemm_args p, dpvo_rowgemm_args p2,
                                                                 dpvo_rowadd_args pre)
{
    __shared__ __attribute__((aligned(16))) char smem[P6_LDS];
    typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nks = p.K / R5_BK;   // even, 4 .. 12 (host-checked)
    const int64_t Mrows = p.M_dev ? min(*p.M_dev, p.M) : p.M;
    const int64_t ntiles = (Mrows + RG_BM - 1) / RG_BM;
    if ((int64_t)blockIdx.x >= ntiles) return;
    const unsigned G = gridDim.x;
    const int64_t my_tiles = (ntiles - 1 - blockIdx.x) / G + 1;
    const int64_t total_w = my_tiles * 2 * nks;
    const YMapChunk ym;
    const int fr = lane & 15, fq = lane >> 4;
    const half_t* __restrict__ zero = (const half_t*)p.zero_row;
    int64_t* idx_lds = (int64_t*)(smem + P6_IDX);
    auto pre_src = [&](int64_t m) __attribute__((always_inline)) -> int64_t {
        return (m < Mrows && pre.b16) ? (pre.b_idx ? pre.b_idx[m] : m) : -1;
    };
    // ---- A staging (rowgemm5's): lane holds row 16 w + (lane >> 2), chunk lane & 3
    const int ar = 16 * w + (lane >> 2), ac = lane & 3;
    int64_t a_tile = -1;
    int a_lt = -1;
    const half_t* arow = zero;
    const float* arow32 = nullptr;
    auto pre_set = [&](int64_t t, int64_t s) __attribute__((always_inline)) {
        const int64_t m = t * RG_BM + ar;
        arow32 = (const float*)pre.a + (m < Mrows ? m : 0) * pre.lda + 8 * ac;
        const half_t* b = (const half_t*)g_pre_negzero.v;
        if (s >= 0 && s < pre.b_rows) b = (const half_t*)pre.b16 + s * RG_BN;
        arow = b + 8 * ac;
    };
    if constexpr (PRE) {
        a_tile = blockIdx.x;
        a_lt = 0;
        pre_set(a_tile, pre_src(a_tile * RG_BM + ar));
    }
    auto a_row = [&](int64_t t) __attribute__((always_inline)) {
        if (t == a_tile) return;
        a_tile = t;
        const int64_t m = t * RG_BM + ar;
        if constexpr (PRE) {
            a_lt++;
            pre_set(t, idx_lds[a_lt * RG_BM + ar]);
        } else {
            const half_t* row = zero;
            if (p.a_idx) {
                if (m < Mrows) {
                    const int64_t src = p.a_idx[m];
                    if (src >= 0 && src < p.a_rows) row = (const half_t*)p.A + src * p.lda;
                }
            } else if (m < Mrows && m < p.a_rows) {
                row = (const half_t*)p.A + m * p.lda;
            }
            arow = row + 8 * ac;
        }
    };
    r5_areg_t<PRE> areg[2];
    auto load_a = [&](int64_t t, int k) __attribute__((always_inline)) -> r5_areg_t<PRE> {
        a_row(t);
        if constexpr (PRE) {
            R5PreRaw x;
            x.lo = *(const f4_t*)(arow32 + k * R5_BK);
            x.hi = *(const f4_t*)(arow32 + k * R5_BK + 4);
            x.b = *(const h8_t*)(arow + k * R5_BK);
            return x;
        } else {
            return *(const h8_t*)(arow + k * R5_BK);
        }
    };
    const int aw_off = ar * 64 + 16 * (ac ^ rc_sw(ar));
    auto put_a = [&](int slot, const r5_areg_t<PRE>& x) __attribute__((always_inline)) {
        *(h8_t*)(smem + slot * R5_ASLOT + aw_off) = r5_cvt(x);
    };
    // ---- W fragments (rowgemm5's flat (tile, pass, k-step) stream, two ahead)
    h8_t wreg[2][3];
    const half_t* W1 = (const half_t*)p.W;
    const half_t* W2 = (const half_t*)p2.W;
    const int wcol = (48 * w + fr) * R5_BK + 8 * fq;
    auto load_w = [&](const R5Cursor& c, h8_t (&r)[3]) __attribute__((always_inline)) {
        const half_t* src = (c.q ? W2 : W1) + (int64_t)c.k * (RG_BN * R5_BK) + wcol;
#pragma unroll
        for (int nt = 0; nt < 3; nt++) r[nt] = *(const h8_t*)(src + nt * 16 * R5_BK);
    };
    h4_t bias[PRE ? 1 : 2][3];
    if constexpr (PRE) {
        if (threadIdx.x < 2 * 96) {
            const int b = threadIdx.x / 96, c = 4 * (threadIdx.x % 96);
            *(h4_t*)(smem + P6_BIAS + b * RG_BN * 2 + 2 * c) = *(const h4_t*)((const half_t*)(b ? p2.bias : p.bias) + c);
        }
    } else {
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
            for (int nt = 0; nt < 3; nt++)
                bias[q][nt] = *(const h4_t*)((const half_t*)(q ? p2.bias : p.bias) + 48 * w + 16 * nt + 4 * fq);
    }
    f4_t acc[8][3];
#pragma unroll
    for (int mt = 0; mt < 8; mt++)
#pragma unroll
        for (int nt = 0; nt < 3; nt++) acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
    const int ar_off = fr * 64 + 16 * (fq ^ rc_sw(fr));   // + 1024 mt: row 16 mt + fr
    auto sync = [&]() __attribute__((always_inline)) {
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
    };
    // pass q's rows out, 64 at a time through the half y tile (rowgemm5's
    // conversion and whole-row stores); ends on a barrier
    auto epilogue = [&](int64_t t, auto qc) __attribute__((always_inline)) {
        constexpr int q = decltype(qc)::value;
        const dpvo_rowgemm_args& pe = q ? p2 : p;
        half_t* out = (half_t*)pe.out16;
        const bool al16 = ((uintptr_t)out & 15) == 0 && (pe.ldo16 & 7) == 0;
#pragma unroll
        for (int hh = 0; hh < 2; hh++) {
#pragma unroll
            for (int nt = 0; nt < 3; nt++) {
                const int col = 48 * w + 16 * nt + 4 * fq;
                h4_t bq;
                if constexpr (PRE)
                    bq = *(const h4_t*)(smem + P6_BIAS + q * RG_BN * 2 + 2 * col);
                else
                    bq = bias[q][nt];
#pragma unroll
                for (int m4 = 0; m4 < 4; m4++) {
                    const int mt = 4 * hh + m4;
                    h4_t y;
#pragma unroll
                    for (int r = 0; r < 4; r++) y[r] = (half_t)(acc[mt][nt][r] + (float)bq[r]);
                    acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
                    *(h4_t*)(smem + P6_YH + ym.off(16 * m4 + fr, col * 2)) = y;
                }
            }
            sync();
            const int64_t row0 = t * RG_BM + 64 * hh;
            if (al16) {   // wave w: rows 8 w .. 8 w + 7 of the half, one 768-byte row per instruction
                if (lane < 48) {
#pragma unroll 4
                    for (int i = 0; i < 8; i++) {
                        const int lr = 8 * w + i;
                        const h8_t v = *(const h8_t*)(smem + P6_YH + ym.off(lr, 16 * lane));
                        if (row0 + lr < Mrows) *(h8_t*)(out + (row0 + lr) * pe.ldo16 + 8 * lane) = v;
                    }
                }
            } else {   // 8-byte aligned rows: two rows per pass
                const int h = lane >> 5, s = lane & 31;
#pragma unroll 2
                for (int i = 0; i < 4; i++) {
                    const int lr = 8 * w + 2 * i + h;
                    ep_h4 v[3];
#pragma unroll
                    for (int j = 0; j < 3; j++) v[j] = *(const ep_h4*)(smem + P6_YH + ym.off(lr, (128 * j + 4 * s) * 2));
                    if (row0 + lr < Mrows) {
#pragma unroll
                        for (int j = 0; j < 3; j++) *(ep_h4*)(out + (row0 + lr) * pe.ldo16 + 128 * j + 4 * s) = v[j];
                    }
                }
            }
            sync();
        }
    };

    // ---- prologue: W steps 0, 1; the first tile's A stages 0, 1 in slots 0, 1, 2, 3 in registers
    R5Cursor cw{0, (int64_t)blockIdx.x, 0, 0};
    auto wnext = [&]() __attribute__((always_inline)) { cw.next(total_w, nks, 2, G); };
    load_w(cw, wreg[0]);
    wnext();
    load_w(cw, wreg[1]);
    wnext();
    put_a(0, load_a(blockIdx.x, 0));
    put_a(1, load_a(blockIdx.x, 1));
    areg[0] = load_a(blockIdx.x, 2);
    areg[1] = load_a(blockIdx.x, 3);
    if constexpr (PRE) {
        for (int i = RG_BM + threadIdx.x; i < (int)my_tiles * RG_BM; i += blockDim.x)
            idx_lds[i] = pre_src(((int64_t)blockIdx.x + (int64_t)(i / RG_BM) * G) * RG_BM + i % RG_BM);
    }
    auto mfmas = [&](int slot, const h8_t (&wr)[3]) __attribute__((always_inline)) {
        const char* sa = smem + slot * R5_ASLOT;
        h8_t a[8];
#pragma unroll
        for (int mt = 0; mt < 8; mt++) a[mt] = *(const h8_t*)(sa + ar_off + 1024 * mt);
#pragma unroll
        for (int nt = 0; nt < 3; nt++)
#pragma unroll
            for (int mt = 0; mt < 8; mt++)
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[nt], a[mt], acc[mt][nt], 0, 0, 0);
    };
#ifdef DPVO_STAMPS
    // segments: 0 pass-0 barrier waits, 1 pass-0 k-steps otherwise, 2 pass-0
    // epilogue, 3 pass 1, 4 pass-1 epilogue + next stages, 10 total, 11 tiles
    unsigned long long st_sum[ST_SEGS] = {};
    RC_STAMP(p_begin)
#endif
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += G) {
        const bool more = tile + G < ntiles;
#ifdef DPVO_STAMPS
        st_sum[11] += 1;
        RC_STAMP(q0)
#endif
        // ---- pass 0: k-step ks reads slot ks, then stage ks + 2 goes from its
        // register set into slot ks + 2 and stage ks + 4 is loaded; one barrier
        // per two k-steps makes stages ks, ks + 1 visible (no slot is reused
        // within the tile, so no barrier guards a rewrite)
#pragma unroll 1
        for (int ks = 0; ks < nks; ks += 2) {
            bd_steps<0, 2>::run([&](auto pc) __attribute__((always_inline)) {
                constexpr int PH = decltype(pc)::value;
                const int k = ks + PH;
                RC_STAMP(b0)
                if (PH == 0) sync();
                RC_STAMP(b1)
                RC_ACC(0, b0, b1)
                mfmas(k, wreg[PH]);
                load_w(cw, wreg[PH]);
                wnext();
                __builtin_amdgcn_sched_barrier(0);
                if (k + 2 < nks) {
                    put_a(k + 2, areg[PH]);
                    if (k + 4 < nks) areg[PH] = load_a(tile, k + 4);
                }
            });
        }
#ifdef DPVO_STAMPS
        RC_STAMP(q1)
        st_sum[1] += q1 - q0;
#endif
        epilogue(tile, std::integral_constant<int, 0>{});
#ifdef DPVO_STAMPS
        RC_STAMP(q2)
        RC_ACC(2, q1, q2)
#endif
        // ---- pass 1 on the resident tile; the next tile's stages 0, 1 load meanwhile
#pragma unroll 1
        for (int ks = 0; ks < nks; ks += 2) {
            bd_steps<0, 2>::run([&](auto pc) __attribute__((always_inline)) {
                constexpr int PH = decltype(pc)::value;
                mfmas(ks + PH, wreg[PH]);
                load_w(cw, wreg[PH]);
                wnext();
                if (ks == 0 && more) areg[PH] = load_a(tile + G, PH);
            });
        }
#ifdef DPVO_STAMPS
        RC_STAMP(q3)
        RC_ACC(3, q2, q3)
#endif
        epilogue(tile, std::integral_constant<int, 1>{});
        if (more) {   // (every wave is past its pass-1 reads: the epilogue's barriers)
            put_a(0, areg[0]);
            put_a(1, areg[1]);
            areg[0] = load_a(tile + G, 2);
            areg[1] = load_a(tile + G, 3);
        }
#ifdef DPVO_STAMPS
        RC_STAMP(q4)
        RC_ACC(4, q3, q4)
#endif
    }
#ifdef DPVO_STAMPS
    RC_STAMP(p_end)
    st_sum[1] -= st_sum[0];   // (segment 1 held the whole pass 0)
    st_sum[10] += p_end - p_begin;
    if (lane == 0)
        for (int k = 0; k < ST_SEGS; k++) dpvo_stamps[((int64_t)blockIdx.x * 8 + w) * ST_SEGS + k] = st_sum[k];
#endif
}

// ---------------------------------------------------------------------------
// v5 chains (round 4): the chain dataflow -- GEMM1 -> y tile -> GEMM2
// [-> LayerNorm -> GEMM3 (TRI) | gate GEMM (GATED)] -> row epilogue -- on
// rowgemm5's machinery: every W (k-blocked) streams from L2 into registers two
// W-steps ahead over one flat per-block sequence (W1, then W2, then W3 / Wg),
// A goes through registers into the 4-slot ring (GEMM1 and the gate pass; one
// barrier per two A-steps), the GEMMs over the y tile read it in place and
// need no barrier at all.  8 waves as 1 (M) x 8 (N), wave tile 128 x 48.
// K1 % 64 == 0 keeps the register-set parities of both sequences equal to the
// k-step's.  The biases sit in LDS (read at the y-tile writes without waiting
// behind the prefetch's vmcnt; in registers the LN chains spilled).
// OVL (residual-only epilogues): tile t's row epilogue runs inside tile
// t + 1's GEMM1 k-loop on every wave (8 batches of 2 rows, each batch's loads
// one k-step ahead of its arithmetic) -- GEMM1 never touches the y tile.
// (Measured at C3 shapes: 151 us with it, 156 without; two batches in flight
// spill.)  Per output element the MFMA k order and the epilogue arithmetic are
// rowgemm3's: bit-identical to the unchained launches.
// ---------------------------------------------------------------------------
// PRELN's row operands: R rows (R / 2 row pairs, half a wave per row, lane s
// of the half at columns 4 s + 128 j: rowadd_ln's and epi2's layout)
template <int R>
struct PreOps {
    ep_f4 a[R / 2][3];
    ep_h4 b[R / 2][3], c[R / 2][3];
};
template <int R>
__device__ __forceinline__ void preln_issue(const dpvo_rowadd_args& pre, int64_t M, int64_t row0, int lane, PreOps<R>& o)
{
    const int h = lane >> 5, s = lane & 31;
    const half_t* negzero = (const half_t*)g_pre_negzero.v;
#pragma unroll
    for (int i = 0; i < R / 2; i++) {
        const int64_t rr = row0 + 2 * i + h;
        const int64_t row = rr < M ? rr : M - 1;   // clamped for loads; stores skip rows >= M
        const int64_t sb = pre.b_idx ? pre.b_idx[row] : row;
        const int64_t sc = pre.c_idx ? pre.c_idx[row] : row;
        const half_t* b = pre.b16 && sb >= 0 && sb < pre.b_rows ? (const half_t*)pre.b16 + sb * RG_BN : negzero;
        const half_t* c = pre.c16 && sc >= 0 && sc < pre.c_rows ? (const half_t*)pre.c16 + sc * RG_BN : negzero;
        const float* a = (const float*)pre.a + row * pre.lda;
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int col = 128 * j + 4 * s;
            o.a[i][j] = *(const ep_f4*)(a + col);
            o.b[i][j] = *(const ep_h4*)(b + col);
            o.c[i][j] = *(const ep_h4*)(c + col);
        }
    }
}
// base = rowadd_ln(a, b16, c16, LN)'s out32 rows, operation for operation:
// ((a + b) + c), the 12 values of a lane summed in order, half-wave sums,
// then (v - mean) * rstd * g + beta
template <int R>
__device__ __forceinline__ void preln_rows(const dpvo_rowadd_args& pre, int lane, const PreOps<R>& o, EpiOps2<R>& e)
{
    const int s = lane & 31;
#pragma unroll
    for (int i = 0; i < R / 2; i++) {
        float v[12];
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int t = 0; t < 4; t++) v[4 * j + t] = o.a[i][j][t];
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int t = 0; t < 4; t++) v[4 * j + t] += (float)o.b[i][j][t];
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int t = 0; t < 4; t++) v[4 * j + t] += (float)o.c[i][j][t];
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < 12; j++) sm += v[j];
        const float mean = half_sum(sm) * (1.f / RG_BN);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 12; j++) q += (v[j] - mean) * (v[j] - mean);
        const float rstd = rsqrtf(half_sum(q) * (1.f / RG_BN) + pre.ln_eps);
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const ep_f4 g = *(const ep_f4*)(pre.ln_g + 128 * j + 4 * s);
            const ep_f4 bt = *(const ep_f4*)(pre.ln_b + 128 * j + 4 * s);
#pragma unroll
            for (int t = 0; t < 4; t++) e.base[i][j][t] = (v[4 * j + t] - mean) * rstd * g[t] + bt[t];
        }
    }
}

constexpr int R5_IDX_TILES = 8;   // rowchain5: tiles per block whose row sources sit in LDS

struct R5WCursor {   // (tile, segment, k-step) of the flat W-step sequence
    int64_t f, t;
    int s, k;
    __device__ __forceinline__ void next(int64_t total, int n0, int n1, int n2, int nseg, unsigned grid)
    {
        if (f + 1 >= total) return;
        f++;
        if (++k == (s == 0 ? n0 : s == 1 ? n1 : n2)) {
            k = 0;
            if (++s == nseg) {
                s = 0;
                t += grid;
            }
        }
    }
};

// F1: GEMM1's activation as a compile-time constant (RG_RELU: every chain of
// the update operator), or -1 to read it from p1.flags.  With the runtime
// flags the y-tile conversion evaluates the sigmoid (exp + rcp per element)
// beside the ReLU and selects: ~10k cycles per tile, an eighth of a c1 tile.
// PRELN (the first GRU's gated chain, dpvo_rowchain_gated_pre): the
// residual base is not read from res32 but formed in the row epilogue as
// LayerNorm(pre.a + pre.b16[b_idx] + pre.c16[c_idx]) with rowadd_ln's fp32
// arithmetic in its order (preln_rows below) -- the rows rowadd_ln would have
// written as out32 (net.py:90-91: net + agg_kk + agg_ij -> norm), without
// their 147 MB write and re-read.
template <int F2, bool GATED = false, int FMID = 0, int F1 = -1, bool PRELN = false>
__global__ __launch_bounds__(R5_THREADS, 1) void rowchain5_kernel(dpvo_rowgemm_args p1, dpvo_rowgemm_args p,
                                                                  dpvo_rowgemm_args pg, dpvo_rowadd_args pre)
{
    static_assert(!PRELN || (GATED && (F2 & RG_NOADD) && (F2 & RG_LN)), "PRELN: the gated LN chain");
    constexpr bool TRI = FMID != 0;
    static_assert(!(TRI && GATED), "a chain is either gated or three GEMMs long");
    // (RES | LN overlapped the same way -- the corr chain, the gated LN chain --
    // measured 188 -> 197 us and 150 -> 150 us: its batches' loads queue ahead
    // of the A stream's in the in-order vmcnt; profiles/r6/experiments/)
    constexpr bool OVL = (F2 & ~RG_NOADD) == RG_RES;
    constexpr int NSEG = (TRI || GATED) ? 3 : 2;
    constexpr int NPA = GATED ? 2 : 1;   // A passes per tile
    constexpr int nk2 = RG_BN / R5_BK;
    constexpr int BIAS_OFF = R5_LDS;   // the three biases, 768 B each, after the A ring
    constexpr int IDX_OFF = BIAS_OFF + 3 * RG_BN * 2;   // the gathered rows' sources, R5_IDX_TILES tiles
    __shared__ __attribute__((aligned(16))) char smem[R5_LDS + 3 * RG_BN * 2 + (!GATED && !TRI ? R5_IDX_TILES * RG_BM * 8 : 0)];
    typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int fr = lane & 15, fq = lane >> 4;
    const int nk1 = p1.K / R5_BK;
    const int64_t Mrows = p1.M_dev ? min(*p1.M_dev, p1.M) : p1.M;
    const int64_t ntiles = (Mrows + RG_BM - 1) / RG_BM;
    if ((int64_t)blockIdx.x >= ntiles) return;
    const unsigned G = gridDim.x;
    const int64_t my_tiles = (ntiles - 1 - blockIdx.x) / G + 1;
    const int64_t total_a = my_tiles * NPA * nk1;
    const int n2 = TRI ? nk2 : nk1;
    const int64_t total_w = my_tiles * (nk1 + nk2 + (NSEG == 3 ? n2 : 0));
    const YMapChunk ym;
    const half_t* __restrict__ zero = (const half_t*)p1.zero_row;
    // ---- the gathered rows' sources (p1.a_idx): the first tile's read
    // directly in the prologue, the block's later tiles' from an LDS table
    // filled after the prologue's loads are issued (published by GEMM1's first
    // barrier), so crossing into the next tile inside the k-loop waits on LDS,
    // not (vmcnt 0) on every load the wave has in flight -- the W / A prefetch
    // and the OVL epilogue's.  (K1 = 64: the prologue's four A stages already
    // cross, so the whole table is filled first.)  The host sizes the grid so
    // that a block has <= R5_IDX_TILES tiles.  The two-GEMM chains only (c1 /
    // c2 gather); the gated and three-GEMM chains keep the direct read, their
    // registers are full.
    constexpr bool IDX_LDS = !GATED && !TRI;
    int64_t* idx_lds = (int64_t*)(smem + IDX_OFF);
    const bool idx_tab = IDX_LDS && p1.a_idx, idx_early = idx_tab && nk1 < 4;
    auto idx_fill = [&](int i0) __attribute__((always_inline)) {
        for (int i = i0 + threadIdx.x; i < (int)my_tiles * RG_BM; i += blockDim.x) {
            const int64_t m = ((int64_t)blockIdx.x + (int64_t)(i / RG_BM) * G) * RG_BM + i % RG_BM;
            idx_lds[i] = m < Mrows ? p1.a_idx[m] : -1;
        }
    };
    if (idx_early) {
        idx_fill(0);
        __syncthreads();
    }
    // ---- A staging (rowgemm5's): lane holds row 16 w + (lane >> 2), chunk lane & 3
    const int ar = 16 * w + (lane >> 2), ac = lane & 3;

    int64_t a_tile = -1;
    int a_lt = -1;   // the block-local index of a_tile (the cursor moves a tile at a time)
    const half_t* arow = zero;
    auto a_set = [&](int64_t m, int64_t src) __attribute__((always_inline)) {
        const half_t* row = zero;
        if (m < Mrows && src >= 0 && src < p1.a_rows) row = (const half_t*)p1.A + src * p1.lda;
        arow = row + 8 * ac;
    };
    if (idx_tab && !idx_early) {   // the first tile, from global (the table is filled after the prologue)
        a_tile = blockIdx.x;
        a_lt = 0;
        const int64_t m0 = a_tile * RG_BM + ar;
        a_set(m0, m0 < Mrows ? p1.a_idx[m0] : -1);
    }
    auto a_row = [&](int64_t t) __attribute__((always_inline)) {
        if (t == a_tile) return;
        a_tile = t;
        if constexpr (!GATED && !TRI) a_lt++;
        const int64_t m = t * RG_BM + ar;
        if constexpr (IDX_LDS) {
            a_set(m, !p1.a_idx ? m : idx_lds[a_lt * RG_BM + ar]);
        } else if (p1.a_idx) {   // (the load's wait stays inside this branch: a wait at
            a_set(m, m < Mrows ? p1.a_idx[m] : -1);   // the join would drain the queue on every path)
        } else {
            a_set(m, m);
        }
    };
    h8_t areg[2];
    auto load_a = [&](const R5Cursor& c) __attribute__((always_inline)) -> h8_t {
        a_row(c.t);
        return *(const h8_t*)(arow + c.k * R5_BK);
    };
    const int aw_off = ar * 64 + 16 * (ac ^ rc_sw(ar));
    // ---- W: segment 0 = W1, 1 = the middle (TRI) or second Linear, 2 = the
    // last (TRI) or the gate (GATED); fragments at column 48 w + 16 nt + fr
    const half_t* Ws0 = (const half_t*)p1.W;
    const half_t* Ws1 = (const half_t*)(TRI ? pg.W : p.W);
    const half_t* Ws2 = (const half_t*)(TRI ? p.W : pg.W);
    h8_t wreg[2][3];
    const int wcol = (48 * w + fr) * R5_BK + 8 * fq;
    auto load_w = [&](const R5WCursor& c, h8_t (&r)[3]) __attribute__((always_inline)) {
        const half_t* base = c.s == 0 ? Ws0 : (c.s == 1 ? Ws1 : Ws2);
        const half_t* src = base + (int64_t)c.k * (RG_BN * R5_BK) + wcol;
#pragma unroll
        for (int nt = 0; nt < 3; nt++) r[nt] = *(const h8_t*)(src + nt * 16 * R5_BK);
    };
    // ---- the biases (GEMM1, GEMM2, GEMM3 / gate) into LDS: read at the
    // y-tile writes without waiting behind the W / A prefetch's vmcnt
    if (threadIdx.x < 3 * 96) {
        const int b = threadIdx.x / 96, c = 4 * (threadIdx.x % 96);
        const void* src = b == 0 ? p1.bias : (b == 1 ? (TRI ? pg.bias : p.bias) : (TRI ? p.bias : pg.bias));
        if (b < NSEG) *(h4_t*)(smem + BIAS_OFF + b * RG_BN * 2 + 2 * c) = *(const h4_t*)((const half_t*)src + c);
    }
    f4_t acc[8][3];
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int mt = 0; mt < 8; mt++)
#pragma unroll
            for (int nt = 0; nt < 3; nt++) acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
    };
    const int ar_off = fr * 64 + 16 * (fq ^ rc_sw(fr));   // + 1024 mt: row 16 mt + fr
    auto sync = [&]() __attribute__((always_inline)) {
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
    };
    // acc + bias (LDS copy bi) -> act -> fp16 -> y tile
    auto acc_to_y = [&](int bi, bool relu, bool sigm) __attribute__((always_inline)) {
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
            const int col = 48 * w + 16 * nt + 4 * fq;
            const h4_t b = *(const h4_t*)(smem + BIAS_OFF + bi * RG_BN * 2 + 2 * col);
#pragma unroll
            for (int mt = 0; mt < 8; mt++) {
                h4_t y;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    half_t v = (half_t)(acc[mt][nt][r] + (float)b[r]);
                    if (relu) v = v > (half_t)0 ? v : (half_t)0;
                    if (sigm) v = (half_t)fast_sigmoid((float)v);
                    y[r] = v;
                }
                *(h4_t*)(smem + ym.off(16 * mt + fr, col * 2)) = y;
            }
        }
    };
    const unsigned bid = blockIdx.x;
    R5Cursor ca{0, (int64_t)bid, 0, 0};
    R5WCursor cw{0, (int64_t)bid, 0, 0};
    auto wnext = [&]() __attribute__((always_inline)) { cw.next(total_w, nk1, nk2, n2, NSEG, G); };
    auto anext = [&]() __attribute__((always_inline)) { ca.next(total_a, nk1, NPA, G); };
    // one A-step (GEMM1 or the gate pass): stage g in slot g & 1, g + 1 in
    // areg[(g + 1) & 1], g + 2 in areg[g & 1]; PH = g & 1 = the W-step's parity
    // one A-step g (GEMM1 or the gate pass), PH = g & 1: stage g from slot
    // g % 4; after the MFMAs stage g + 2 (register set PH) into slot
    // (g + 2) % 4 and stage g + 4 loaded into set PH.  One barrier per two A-steps (even g): it makes
    // stages g, g + 1 visible and frees the slots of stages g - 2, g - 1.
    int ga = 0;
    auto step_a = [&](auto ph) __attribute__((always_inline)) {
        constexpr int PH = decltype(ph)::value;
        if (PH == 0) sync();
        const char* sa = smem + R5_Y + (ga & 3) * R5_ASLOT;
        h8_t a[8];
#pragma unroll
        for (int mt = 0; mt < 8; mt++) a[mt] = *(const h8_t*)(sa + ar_off + 1024 * mt);
#pragma unroll
        for (int nt = 0; nt < 3; nt++)
#pragma unroll
            for (int mt = 0; mt < 8; mt++)
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wreg[PH][nt], a[mt], acc[mt][nt], 0, 0, 0);
        // (W before A, the ring write after the MFMAs: as in rowgemm5)
        load_w(cw, wreg[PH]);
        wnext();
        __builtin_amdgcn_sched_barrier(0);
        *(h8_t*)(smem + R5_Y + ((ga + 2) & 3) * R5_ASLOT + aw_off) = areg[PH];
        areg[PH] = load_a(ca);
        anext();
        ga++;
    };
    // one k-step of a GEMM over the y tile (read in place; no barrier)
    auto step_y = [&](auto ph, int ks) __attribute__((always_inline)) {
        constexpr int PH = decltype(ph)::value;
        h8_t a[8];
#pragma unroll
        for (int mt = 0; mt < 8; mt++) a[mt] = *(const h8_t*)(smem + ym.off(16 * mt + fr, (ks * 4 + fq) * 16));
#pragma unroll
        for (int nt = 0; nt < 3; nt++)
#pragma unroll
            for (int mt = 0; mt < 8; mt++)
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wreg[PH][nt], a[mt], acc[mt][nt], 0, 0, 0);
        load_w(cw, wreg[PH]);
        wnext();
    };
    auto gemm_y = [&]() __attribute__((always_inline)) {
        zero_acc();
#pragma unroll 1
        for (int ks = 0; ks < nk2; ks += 2) {
            step_y(std::integral_constant<int, 0>{}, ks);
            step_y(std::integral_constant<int, 1>{}, ks + 1);
        }
    };
    // TRI: LayerNorm (+ ReLU) of the y tile's rows in place, rounded to fp16
    // (epi2_finish's LN arithmetic)
    auto mid_rows = [&](const dpvo_rowgemm_args& pm) __attribute__((always_inline)) {
        EpiConsts2 km;
        load_consts2<FMID>(pm, lane, km);
        const int h = lane >> 5, s = lane & 31;
#pragma unroll 1
        for (int i = 0; i < 8; i++) {
            const int r = w * 16 + 2 * i + h;
            ep_f4 v[3];
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const ep_h4 y = *(const ep_h4*)(smem + ym.off(r, (128 * j + 4 * s) * 2));
                v[j] = ep_f4{(float)y[0], (float)y[1], (float)y[2], (float)y[3]};
            }
            float sm = 0.f;
#pragma unroll
            for (int j = 0; j < 3; j++) sm += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
            const float mean = half_sum(sm) * (1.f / RG_BN);
            float sq = 0.f;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const ep_f4 d = v[j] - mean;
                sq += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
            }
            const float rstd = rsqrtf(half_sum(sq) * (1.f / RG_BN) + pm.ln_eps);
#pragma unroll
            for (int j = 0; j < 3; j++) {
                v[j] = (v[j] - mean) * rstd * km.g[j] + km.b[j];
                if (FMID & RG_LN_RELU)
#pragma unroll
                    for (int t = 0; t < 4; t++) v[j][t] = fmaxf(v[j][t], 0.f);
                *(ep_h4*)(smem + ym.off(r, (128 * j + 4 * s) * 2)) =
                    ep_h4{(half_t)v[j][0], (half_t)v[j][1], (half_t)v[j][2], (half_t)v[j][3]};
            }
        }
    };
    // the row epilogue in batches of R rows: local rows lr .. lr + R - 1 of tile et
    auto epi_issue = [&](int64_t et, int lr, auto& o) __attribute__((always_inline)) {
        constexpr int R = sizeof(o.add) / sizeof(o.add[0][0]) / 3 * 2;
        epi2_load<F2, R>(p, Mrows, et * RG_BM + lr, lane, o);
    };
    auto epi_done = [&](int64_t et, int lr, const EpiConsts2& kc, const auto& o) __attribute__((always_inline)) {
        constexpr int R = sizeof(o.add) / sizeof(o.add[0][0]) / 3 * 2;
        const int hh = lane >> 5, ss = lane & 31;
        epi2_finish<F2, R>(
            p, Mrows,
            [&](int i, int j) { return *(const ep_h4*)(smem + ym.off(lr + 2 * i + hh, (128 * j + 4 * ss) * 2)); },
            et * RG_BM + lr, lane, kc, o);
    };

    // ---- prologue: W-steps 0, 1 in registers; A stages 0, 1 in slots 0, 1,
    // 2 and 3 in register sets 0, 1
    load_w(cw, wreg[0]);
    wnext();
    load_w(cw, wreg[1]);
    wnext();
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const h8_t x = load_a(ca);
        *(h8_t*)(smem + R5_Y + r * R5_ASLOT + aw_off) = x;
        anext();
    }
#pragma unroll
    for (int r = 0; r < 2; r++) {
        areg[r] = load_a(ca);
        anext();
    }
    if (idx_tab && !idx_early) idx_fill(RG_BM);   // (tiles 1.. : read after GEMM1's first barrier)
    int64_t etile = -1;   // OVL: the tile whose row epilogue is still pending
#ifdef DPVO_STAMPS
    // chain segments: 0 GEMM1 k-loop (+ OVL epilogue), 1 GEMM1 -> y tile + sync,
    // 2 GEMM2 (+ TRI: mid rows + GEMM3) + syncs, 3 y-tile write (+ gate pass) + sync,
    // 4 row epilogue (non-OVL / last tile), 10 total, 11 tiles
    unsigned long long st_sum[ST_SEGS] = {};
    RC_STAMP(c_begin)
#endif
    for (int64_t tile = bid; tile < ntiles; tile += G) {
#ifdef DPVO_STAMPS
        RC_STAMP(c0)
        st_sum[11] += 1;
#endif
        const bool more = tile + G < ntiles;
        // ---- GEMM1 (+ OVL: the previous tile's row epilogue, rows 16 w .. 16 w + 15
        // in 8 batches of 2: batch b's loads after k-step L(b) = b (nk1 - 4) / 7,
        // its y-tile reads and arithmetic after k-step L(b) + 1 <= nk1 - 3.
        // Barriers come at the even k-steps only, so the last batch must finish
        // before the barrier of k-step nk1 - 2: that barrier is the only one
        // between a wave's last read of tile t's y rows and the other waves'
        // acc_to_y writes of tile t + 1 after k-step nk1 - 1.  (Round 4 to 5
        // scheduled the last batch's reads after k-step nk1 - 2, with no barrier
        // before those writes: a wave running ahead could overwrite y-tile
        // columns a slower wave had not read yet -- the intermittent last-bit
        // differences of the round-5 graph-replay test.)
        {
            constexpr int OR = 2, NB = 16 / OR;   // rows per batch, batches
            // (4-row batches: the same time, 248 registers)
            EpiOps2<OR> st;
            int bi = 0, bd = 0;
            auto ovl = [&](int ks) __attribute__((always_inline)) {
                if (!OVL || etile < 0) return;
                if (bd < bi) {
                    EpiConsts2 kc;
                    load_consts2<F2>(p, lane, kc);
                    epi_done(etile, 16 * w + OR * bd, kc, st);
                    bd++;
                }
                __builtin_amdgcn_sched_barrier(0);
                if (bi < NB && (bi * (nk1 - 4)) / (NB - 1) == ks) {
                    epi_issue(etile, 16 * w + OR * bi, st);
                    bi++;
                }
            };
            zero_acc();
#pragma unroll 1
            for (int ks = 0; ks < nk1; ks += 2) {
                step_a(std::integral_constant<int, 0>{});
                ovl(ks);
                step_a(std::integral_constant<int, 1>{});
                ovl(ks + 1);
            }
        }
        etile = -1;
#ifdef DPVO_STAMPS
        RC_STAMP(c1)
#endif
        if constexpr (F1 >= 0)
            acc_to_y(0, (F1 & RG_RELU) != 0, (F1 & RG_SIGMOID) != 0);
        else
            acc_to_y(0, p1.flags & RG_RELU, p1.flags & RG_SIGMOID);
        sync();
#ifdef DPVO_STAMPS
        RC_STAMP(c2)
#endif
        gemm_y();
        sync();   // every wave is done reading the y tile
        if (TRI) {
            acc_to_y(1, false, false);
            sync();
            mid_rows(pg);
            sync();
            gemm_y();
            sync();
            acc_to_y(2, F2 & RG_RELU, F2 & RG_SIGMOID);
        } else {
#ifdef DPVO_STAMPS
            RC_STAMP(c3t)
            RC_ACC(2, c2, c3t)
#endif
            acc_to_y(1, F2 & RG_RELU, F2 & RG_SIGMOID);
        }
        if (GATED) {
            // gate = sigmoid(A Wg^T + bg) (rowgemm's SIGMOID rounding); y = fp16(gate * y)
            zero_acc();
#pragma unroll 1
            for (int ks = 0; ks < nk1; ks += 2) {
                step_a(std::integral_constant<int, 0>{});
                step_a(std::integral_constant<int, 1>{});
            }
#pragma unroll
            for (int nt = 0; nt < 3; nt++) {
                const int col = 48 * w + 16 * nt + 4 * fq;
                const h4_t b = *(const h4_t*)(smem + BIAS_OFF + 2 * RG_BN * 2 + 2 * col);
#pragma unroll
                for (int mt = 0; mt < 8; mt++) {
                    h4_t* yp = (h4_t*)(smem + ym.off(16 * mt + fr, col * 2));
                    h4_t y = *yp;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const half_t g = (half_t)fast_sigmoid((float)(half_t)(acc[mt][nt][r] + (float)b[r]));
                        y[r] = (half_t)((float)g * (float)y[r]);
                    }
                    *yp = y;
                }
            }
        }
        sync();
#ifdef DPVO_STAMPS
        RC_STAMP(c4)
        RC_ACC(0, c0, c1) RC_ACC(1, c1, c2) RC_ACC(3, c2, c4)
#endif
        if (OVL && more && nk1 >= 12) {   // (12 k-steps fit the 8 batches' schedule)
            etile = tile;   // runs inside the next tile's GEMM1
            continue;
        }
        // the row epilogue now: rows 16 w .. 16 w + 15 (the next tile's y
        // tile writes follow its GEMM1 k-steps' barriers)
        // (the accumulators are dead here: the next batch's loads are issued
        // before this batch's arithmetic, two batches live)
        EpiConsts2 kc;
        load_consts2<F2>(p, lane, kc);
        if constexpr (OVL) {   // (only the last tile: one batch live, no spill beside the deferred state)
#pragma unroll 1
            for (int q0 = 0; q0 < 16; q0 += 4) {
                EpiOps2<4> st;
                epi_issue(tile, 16 * w + q0, st);
                epi_done(tile, 16 * w + q0, kc, st);
            }
        } else if constexpr (PRELN) {
            PreOps<4> st[2];
            preln_issue<4>(pre, Mrows, tile * RG_BM + 16 * w, lane, st[0]);
            bd_steps<0, 4>::run([&](auto bc) __attribute__((always_inline)) {
                constexpr int b = decltype(bc)::value;
                if constexpr (b + 1 < 4) preln_issue<4>(pre, Mrows, tile * RG_BM + 16 * w + 4 * (b + 1), lane, st[(b + 1) & 1]);
                EpiOps2<4> o;
                preln_rows<4>(pre, lane, st[b & 1], o);
                epi_done(tile, 16 * w + 4 * b, kc, o);
            });
        } else {
            EpiOps2<4> st[2];
            epi_issue(tile, 16 * w, st[0]);
            bd_steps<0, 4>::run([&](auto bc) __attribute__((always_inline)) {
                constexpr int b = decltype(bc)::value;
                if constexpr (b + 1 < 4) epi_issue(tile, 16 * w + 4 * (b + 1), st[(b + 1) & 1]);
                epi_done(tile, 16 * w + 4 * b, kc, st[b & 1]);
            });
        }
#ifdef DPVO_STAMPS
        RC_STAMP(c5)
        RC_ACC(4, c4, c5)
#endif
    }
#ifdef DPVO_STAMPS
    RC_STAMP(c_end)
    st_sum[10] += c_end - c_begin;
    if (lane == 0)
        for (int k = 0; k < ST_SEGS; k++) dpvo_stamps[((int64_t)blockIdx.x * 8 + w) * ST_SEGS + k] = st_sum[k];
#endif
}

// v = a32[row] (+ b16[idx[row]]) -> [LayerNorm] -> out32 / out16
// Half a wave per row: lane l of the half covers columns 4l + 128j (j < 3), so
// every access is a 16-byte (fp32) or 8-byte (fp16) vector and one wave keeps
// two rows' loads in flight.  HBM-bound: 4 B x 384 in, 6 B x 384 out per row.
typedef float rl_f4 __attribute__((ext_vector_type(4)));
typedef half_t rl_h4 __attribute__((ext_vector_type(4)));

// Every load of a row is issued before the first use: the two row-source
// indices together, then the a, b and c rows together (absent addends read a
// row of -0, so v + b == v exactly, as the skipped add; the fp16 / fp32 choice
// of a is a template parameter).  Branching per load had the compiler wait on
// each in turn: ~7 dependent HBM round trips per row, 67 us at C3.
template <bool A16>
__global__ __launch_bounds__(256) void rowadd_ln_kernel(dpvo_rowadd_args p)
{
    const int sub = threadIdx.x & 31;
    float g[12], bt[12];
    if (p.ln_g) {
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const rl_f4 gg = *(const rl_f4*)((const float*)p.ln_g + 128 * j + 4 * sub);
            const rl_f4 bb = *(const rl_f4*)((const float*)p.ln_b + 128 * j + 4 * sub);
#pragma unroll
            for (int t = 0; t < 4; t++) {
                g[4 * j + t] = gg[t];
                bt[4 * j + t] = bb[t];
            }
        }
    }
    const half_t* negzero = (const half_t*)g_pre_negzero.v;
    for (int64_t row = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 5; row < p.M;
         row += ((int64_t)gridDim.x * blockDim.x) >> 5) {
        float v[12];
        const int64_t sb = p.b_idx ? p.b_idx[row] : row;
        const int64_t sc = p.c_idx ? p.c_idx[row] : row;
        const half_t* b = p.b16 && sb >= 0 && sb < p.b_rows ? (const half_t*)p.b16 + sb * RG_BN : negzero;
        const half_t* c2 = p.c16 && sc >= 0 && sc < p.c_rows ? (const half_t*)p.c16 + sc * RG_BN : negzero;
        rl_h4 hb[3], hc[3];
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int c = 128 * j + 4 * sub;
            if constexpr (A16) {
                const rl_h4 h = *(const rl_h4*)((const half_t*)p.a + row * p.lda + c);
#pragma unroll
                for (int t = 0; t < 4; t++) v[4 * j + t] = (float)h[t];
            } else {
                const rl_f4 a = *(const rl_f4*)((const float*)p.a + row * p.lda + c);
#pragma unroll
                for (int t = 0; t < 4; t++) v[4 * j + t] = a[t];
            }
            hb[j] = *(const rl_h4*)(b + c);
            hc[j] = *(const rl_h4*)(c2 + c);
        }
        // ((a + b) + c: the two row adds of consecutive rowadd_ln calls, in order)
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int t = 0; t < 4; t++) v[4 * j + t] += (float)hb[j][t];
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int t = 0; t < 4; t++) v[4 * j + t] += (float)hc[j][t];
        if (p.ln_g) {
            // half-wave sums with DPP rotations and a gfx950 lane swap: VALU
            // only (a + b == b + a, so both lanes of a swapped pair agree)
            auto halfsum = [](float x) {
                x = rowsum16(x);
                auto h = __builtin_amdgcn_permlane16_swap(__float_as_int(x), __float_as_int(x), false, false);
                return __int_as_float(h[0]) + __int_as_float(h[1]);
            };
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 12; j++) s += v[j];
            const float mean = halfsum(s) * (1.f / RG_BN);
            float q = 0.f;
#pragma unroll
            for (int j = 0; j < 12; j++) q += (v[j] - mean) * (v[j] - mean);
            const float rstd = rsqrtf(halfsum(q) * (1.f / RG_BN) + p.ln_eps);
#pragma unroll
            for (int j = 0; j < 12; j++) v[j] = (v[j] - mean) * rstd * g[j] + bt[j];
        }
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int c = 128 * j + 4 * sub;
            if (p.out32) *(rl_f4*)((float*)p.out32 + row * RG_BN + c) = rl_f4{v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]};
            if (p.out16)
                *(rl_h4*)((half_t*)p.out16 + row * RG_BN + c) =
                    rl_h4{(half_t)v[4 * j], (half_t)v[4 * j + 1], (half_t)v[4 * j + 2], (half_t)v[4 * j + 3]};
        }
    }
}

// ---------------------------------------------------------------------------
// Narrow tiles (round 6) for the device-counted GEMMs -- SoftAgg's h Linear
// on the groups (`rowgemm(y, *ph, M_dev=G)`, net.py): G (~4.4k patch groups,
// a few hundred frame-pair groups at C3) is known only on the device, so
// rowgemm5 launched for the upper bound put it on 35 / 4 busy workgroups of
// 128 rows: 15 us a launch, bound by each workgroup's L1 traffic (the whole
// 288 KB W per tile).  Here a workgroup takes 32 rows x 192 columns (two per
// row tile; 4 waves x 48 columns, 2 x 3 accumulators): the A tile is loaded
// once into LDS (XOR-swizzled 16-byte chunks: conflict-free fragment reads),
// each wave streams its W fragments from L2 two k-steps ahead, and each lane
// stores its 4 columns of each row.  Same 16 x 16 x 32 blocks in the same k
// order, the same epilogue rounding: bit-identical to rowgemm5.
// ---------------------------------------------------------------------------
// (RN_WD: W k-steps in flight; 4 measured the same as 2, 7.17 vs 7.11 us)
constexpr int RN_BM = 32, RN_THREADS = 256, RN_MAXK = 896, RN_WD = 2;

template <int FLAGS, int KC>   // KC = K / 64: the A chunks each thread stages
__global__ __launch_bounds__(RN_THREADS) void rowgemm_narrow_kernel(dpvo_rowgemm_args p)
{
    static_assert((FLAGS & ~(RG_RELU | RG_SIGMOID)) == 0, "narrow: plain GEMMs only");
    __shared__ __attribute__((aligned(16))) char sA[RN_BM * RN_MAXK * 2];
    typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int fr = lane & 15, fq = lane >> 4;
    constexpr int K = 64 * KC, nks = K / R5_BK, rowb = 2 * K;
    static_assert(K <= RN_MAXK && K % 128 == 0, "narrow: the A tile's swizzle needs K % 128 == 0");
    static_assert(nks % RN_WD == 0, "narrow: whole groups of W k-steps");
    const int64_t Mrows = p.M_dev ? min(*p.M_dev, p.M) : p.M;
    const int64_t ntiles = (Mrows + RN_BM - 1) / RN_BM;
    const int c0 = 192 * (blockIdx.x & 1) + 48 * w;   // this wave's first column
    const half_t* __restrict__ W = (const half_t*)p.W + (c0 + fr) * R5_BK + 8 * fq;
    half_t* out = (half_t*)p.out16;
    auto soff = [&](int r, int c) __attribute__((always_inline)) { return r * rowb + ((c ^ (r & 15)) << 4); };
    h4_t bias[3];
#pragma unroll
    for (int nt = 0; nt < 3; nt++) bias[nt] = *(const h4_t*)((const half_t*)p.bias + c0 + 16 * nt + 4 * fq);
    const int ar = threadIdx.x >> 3, ac = threadIdx.x & 7;   // staging: row ar, chunks ac + 8 j
    for (int64_t t = blockIdx.x >> 1; t < ntiles; t += gridDim.x >> 1) {
        // ---- the A tile into LDS: all KC loads of a thread in flight together
        const int64_t m = t * RN_BM + ar;
        const half_t* row = (const half_t*)p.zero_row;
        if (m < Mrows) {
            const int64_t src = p.a_idx ? p.a_idx[m] : m;
            if (src >= 0 && src < p.a_rows) row = (const half_t*)p.A + src * p.lda;
        }
        h8_t st[KC];
#pragma unroll
        for (int j = 0; j < KC; j++) st[j] = *(const h8_t*)(row + 8 * (ac + 8 * j));
#pragma unroll
        for (int j = 0; j < KC; j++) *(h8_t*)(sA + soff(ar, ac + 8 * j)) = st[j];
        __syncthreads();
        f4_t acc[2][3];
#pragma unroll
        for (int mt = 0; mt < 2; mt++)
#pragma unroll
            for (int nt = 0; nt < 3; nt++) acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
        h8_t wf[RN_WD][3];
        auto load_w = [&](int ks, h8_t (&wr)[3]) __attribute__((always_inline)) {
#pragma unroll
            for (int nt = 0; nt < 3; nt++) wr[nt] = *(const h8_t*)(W + (int64_t)ks * (RG_BN * R5_BK) + nt * 16 * R5_BK);
        };
#pragma unroll
        for (int d = 0; d < RN_WD; d++) load_w(d, wf[d]);
#pragma unroll 1
        for (int ks = 0; ks < nks; ks += RN_WD) {
            bd_steps<0, RN_WD>::run([&](auto pc) __attribute__((always_inline)) {
                constexpr int S = decltype(pc)::value;
                h8_t a[2];
#pragma unroll
                for (int mt = 0; mt < 2; mt++) a[mt] = *(const h8_t*)(sA + soff(16 * mt + fr, 4 * (ks + S) + fq));
#pragma unroll
                for (int nt = 0; nt < 3; nt++)
#pragma unroll
                    for (int mt = 0; mt < 2; mt++)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[S][nt], a[mt], acc[mt][nt], 0, 0, 0);
                load_w(min(ks + S + RN_WD, nks - 1), wf[S]);   // (unconditional: exact wait counts)
            });
        }
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
            const int col = c0 + 16 * nt + 4 * fq;
#pragma unroll
            for (int mt = 0; mt < 2; mt++) {
                h4_t y;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    half_t v = (half_t)(acc[mt][nt][r] + (float)bias[nt][r]);
                    if (FLAGS & RG_RELU) v = v > (half_t)0 ? v : (half_t)0;
                    if (FLAGS & RG_SIGMOID) v = (half_t)fast_sigmoid((float)v);
                    y[r] = v;
                }
                const int64_t row = t * RN_BM + 16 * mt + fr;
                if (row < Mrows) *(h4_t*)(out + row * p.ldo16 + col) = y;
            }
        }
        __syncthreads();   // (every wave's A reads before the next tile's writes)
    }
}

int g_num_cus = 0;

}  // namespace
}  // namespace dpvo

using namespace dpvo;

static int validate_rowgemm(const dpvo_rowgemm_args* a)
{
    DPVO_CHECK_ARG(a != nullptr, "null args");
    DPVO_CHECK_ARG(a->N == RG_BN, "rowgemm: output width must be 384");
    if (a->flags & DPVO_RG_WKB) {
        DPVO_CHECK_ARG((a->flags & ~(DPVO_RG_WKB | DPVO_RG_RELU | DPVO_RG_SIGMOID)) == 0,
                       "rowgemm: k-blocked W (WKB) takes only RELU / SIGMOID");
        // K a multiple of 2 k-steps: every tile's last k-step is then odd, so the
        // even step after it (one barrier per two steps) separates a tile's
        // y-tile reads from the next tile's y-tile writes (K = 32 would race)
        DPVO_CHECK_ARG(a->K > 0 && a->K % (2 * R5_BK) == 0, "rowgemm: K must be a positive multiple of 64 with WKB");
        DPVO_CHECK_ARG(a->out16 && a->ldo16 % 4 == 0 && ((uintptr_t)a->out16 & 7) == 0 && !a->out32,
                       "rowgemm: WKB writes out16 only (8-byte aligned rows)");
    } else {
        DPVO_CHECK_ARG(a->K > 0 && a->K % RG_BK == 0, "rowgemm: K must be a positive multiple of 64 (pad W with zeros)");
    }
    // (v2 stages K in steps of 32; every multiple of 64 is one)
    DPVO_CHECK_ARG(a->A && a->W && a->bias && a->zero_row, "rowgemm: A, W, bias and zero_row are required");
    DPVO_CHECK_ARG(a->lda >= a->K && a->lda % 8 == 0, "rowgemm: lda must be >= K and a multiple of 8");
    DPVO_CHECK_ARG(((uintptr_t)a->A & 15) == 0 && ((uintptr_t)a->W & 15) == 0 && ((uintptr_t)a->zero_row & 15) == 0,
                   "rowgemm: A, W and zero_row must be 16-byte aligned");
    const int f = a->flags;
    DPVO_CHECK_ARG(!((f & DPVO_RG_RES) || (f & DPVO_RG_GATE)) || a->res32, "rowgemm: residual input missing");
    DPVO_CHECK_ARG(!(f & DPVO_RG_GATE) || a->gate16, "rowgemm: gate input missing");
    DPVO_CHECK_ARG(!(f & DPVO_RG_LN) || (a->ln_g && a->ln_b), "rowgemm: LayerNorm weights missing");
    DPVO_CHECK_ARG(!(f & DPVO_RG_HEADS) || (a->head_w && a->head_b && a->head_out), "rowgemm: head weights missing");
    DPVO_CHECK_ARG(!a->out16 || (a->ldo16 % 4 == 0 && ((uintptr_t)a->out16 & 7) == 0),
                   "rowgemm: out16 needs 8-byte aligned rows (ldo16 % 4 == 0)");
    DPVO_CHECK_ARG(!a->out32 || (a->ldo32 % 4 == 0 && ((uintptr_t)a->out32 & 15) == 0),
                   "rowgemm: out32 needs 16-byte aligned rows (ldo32 % 4 == 0)");
    DPVO_CHECK_ARG(((uintptr_t)a->bias & 7) == 0, "rowgemm: bias must be 8-byte aligned");
    return 0;
}

static int ensure_num_cus()
{
    if (g_num_cus == 0) {
        int dev = 0;
        DPVO_CHECK_HIP(hipGetDevice(&dev));
        DPVO_CHECK_HIP(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
        if (g_num_cus <= 0) g_num_cus = 256;
    }
    return 0;
}

extern "C" int dpvo_rowgemm_pair(const dpvo_rowgemm_args* a, const dpvo_rowgemm_args* b, void* stream)
{
    if (validate_rowgemm(a) || validate_rowgemm(b)) return -1;
    DPVO_CHECK_ARG((a->flags == 0 && b->flags == 0) || (a->flags == DPVO_RG_WKB && b->flags == DPVO_RG_WKB),
                   "rowgemm_pair: plain GEMMs only (flags 0, or WKB on both)");
    DPVO_CHECK_ARG(a->A == b->A && a->lda == b->lda && a->a_idx == b->a_idx && a->a_rows == b->a_rows &&
                       a->K == b->K && a->M == b->M && a->M_dev == b->M_dev,
                   "rowgemm_pair: both GEMMs must share A, K and M");
    if (a->M <= 0) return 0;
    if (ensure_num_cus()) return -1;
    const int64_t ntiles = (a->M + RG_BM - 1) / RG_BM;
    const unsigned grid = (unsigned)std::min<int64_t>(ntiles, g_num_cus);
    if ((a->flags & DPVO_RG_WKB) && a->K / R5_BK <= P6_MAXK && a->K / R5_BK >= 4)   // (the A tile fits LDS)
        hipLaunchKernelGGL((rowpair6_kernel<false>), dim3(grid), dim3(R5_THREADS), 0, as_stream(stream), *a, *b,
                           dpvo_rowadd_args{});
    else if (a->flags & DPVO_RG_WKB)
        hipLaunchKernelGGL((rowgemm5_kernel<0, true>), dim3(grid), dim3(R5_THREADS), 0, as_stream(stream), *a, *b);
    else
        hipLaunchKernelGGL((rowgemm3_kernel<0, true>), dim3(grid), dim3(RG_THREADS), 0, as_stream(stream), *a, *b);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_rowgemm_pair_pre(const dpvo_rowgemm_args* a, const dpvo_rowgemm_args* b,
                                     const dpvo_rowadd_args* pre, void* stream)
{
    DPVO_CHECK_ARG(pre != nullptr && pre->a != nullptr && !pre->a_f16 && pre->lda >= 384 && pre->lda % 4 == 0 &&
                       ((uintptr_t)pre->a & 15) == 0,
                   "rowgemm_pair_pre: pre.a must be fp32 rows of >= 384 (16-byte aligned)");
    DPVO_CHECK_ARG(!pre->b16 || ((uintptr_t)pre->b16 & 15) == 0, "rowgemm_pair_pre: pre.b16 must be 16-byte aligned");
    DPVO_CHECK_ARG(!pre->ln_g && !pre->c16 && !pre->out32 && !pre->out16,
                   "rowgemm_pair_pre: pre is the row add only (no LayerNorm, second addend or outputs)");
    if (validate_rowgemm(a) || validate_rowgemm(b)) return -1;
    DPVO_CHECK_ARG(a->flags == DPVO_RG_WKB && b->flags == DPVO_RG_WKB, "rowgemm_pair_pre: k-blocked W on both");
    DPVO_CHECK_ARG(a->K == 384 && b->K == 384 && a->M == b->M && a->M == pre->M && a->M_dev == b->M_dev &&
                       !a->a_idx && !b->a_idx,
                   "rowgemm_pair_pre: K = 384, one M, no row gather (the rows are pre's)");
    if (a->M <= 0) return 0;
    if (ensure_num_cus()) return -1;
    const int64_t ntiles = (a->M + RG_BM - 1) / RG_BM;
    // (at least ntiles / R5_PRE_IDX_TILES blocks: a block's addend sources fit its LDS table)
    const unsigned grid =
        (unsigned)std::max<int64_t>(std::min<int64_t>(ntiles, g_num_cus), (ntiles + R5_PRE_IDX_TILES - 1) / R5_PRE_IDX_TILES);
    hipLaunchKernelGGL((rowpair6_kernel<true>), dim3(grid), dim3(R5_THREADS), 0, as_stream(stream), *a, *b, *pre);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_rowgemm(const dpvo_rowgemm_args* a, void* stream)
{
    if (validate_rowgemm(a)) return -1;
    const int f = a->flags;
    if (a->M <= 0) return 0;
    if (ensure_num_cus()) return -1;
    const int64_t ntiles = (a->M + RG_BM - 1) / RG_BM;
    const unsigned grid = (unsigned)std::min<int64_t>(ntiles, g_num_cus);
    // a device row count (the SoftAgg group GEMMs: G rows of an upper bound M,
    // G << M) takes the narrow 32-row tiles
    const unsigned grid_n = 2 * (unsigned)std::min<int64_t>((a->M + RN_BM - 1) / RN_BM, 2 * (int64_t)g_num_cus);
    const bool narrow = a->M_dev && (a->K == 384 || a->K == 896);
    switch (f) {
#define R5_CASE(F)                                                                                                    \
    case (F) | DPVO_RG_WKB:                                                                                           \
        if (narrow && a->K == 384)                                                                                    \
            hipLaunchKernelGGL((rowgemm_narrow_kernel<(F), 6>), dim3(grid_n), dim3(RN_THREADS), 0, as_stream(stream), \
                               *a);                                                                                   \
        else if (narrow)                                                                                              \
            hipLaunchKernelGGL((rowgemm_narrow_kernel<(F), 14>), dim3(grid_n), dim3(RN_THREADS), 0,                   \
                               as_stream(stream), *a);                                                                \
        else                                                                                                          \
            hipLaunchKernelGGL((rowgemm5_kernel<(F), false>), dim3(grid), dim3(R5_THREADS), 0, as_stream(stream), *a, \
                               *a);                                                                                   \
        break;
        R5_CASE(0)
        R5_CASE(DPVO_RG_RELU)
        R5_CASE(DPVO_RG_SIGMOID)
#undef R5_CASE
#define R3_CASE(F)                                                                                            \
    case (F):                                                                                                 \
        hipLaunchKernelGGL(rowgemm3_kernel<(F)>, dim3(grid), dim3(RG_THREADS), 0, as_stream(stream), *a, *a); \
        break;
        R3_CASE(0)
        R3_CASE(DPVO_RG_RELU)
        R3_CASE(DPVO_RG_SIGMOID)
        R3_CASE(DPVO_RG_LN | DPVO_RG_LN_RELU)
        R3_CASE(DPVO_RG_RES)
        R3_CASE(DPVO_RG_RES | DPVO_RG_LN)
        R3_CASE(DPVO_RG_GATE | DPVO_RG_LN)
        R3_CASE(DPVO_RG_GATE | DPVO_RG_HEADS)
        R3_CASE(DPVO_RG_GATE)
#undef R3_CASE
    default:
        set_error("dpvo_rowgemm: unsupported epilogue flag combination " + std::to_string(f));
        return -1;
    }
    DPVO_CHECK_LAUNCH();
    return 0;
}

static int rowchain_launch(const dpvo_rowgemm_args* g1, const dpvo_rowgemm_args* g2, const dpvo_rowgemm_args* gate,
                           void* stream, const dpvo_rowadd_args* pre = nullptr)
{
    DPVO_CHECK_ARG(g1 != nullptr && g2 != nullptr, "null args");
    DPVO_CHECK_ARG(g1->N == RG_BN && g2->N == RG_BN, "rowchain: output widths must be 384");
    DPVO_CHECK_ARG(g1->K > 0 && g1->K % 64 == 0, "rowchain: K1 must be a positive multiple of 64");
    DPVO_CHECK_ARG(g2->K == RG_BN, "rowchain: the second GEMM's K must be 384 (the intermediate width)");
    DPVO_CHECK_ARG(g1->A && g1->W && g1->bias && g1->zero_row && g2->W && g2->bias,
                   "rowchain: A, W1, W2, both biases and zero_row are required");
    DPVO_CHECK_ARG(g1->lda >= g1->K && g1->lda % 8 == 0, "rowchain: lda must be >= K1 and a multiple of 8");
    DPVO_CHECK_ARG(((uintptr_t)g1->A & 15) == 0 && ((uintptr_t)g1->W & 15) == 0 && ((uintptr_t)g2->W & 15) == 0 &&
                       ((uintptr_t)g1->zero_row & 15) == 0,
                   "rowchain: A, W1, W2 and zero_row must be 16-byte aligned");
    DPVO_CHECK_ARG(((uintptr_t)g1->bias & 7) == 0 && ((uintptr_t)g2->bias & 7) == 0,
                   "rowchain: biases must be 8-byte aligned");
    DPVO_CHECK_ARG((g1->flags & ~(DPVO_RG_RELU | DPVO_RG_SIGMOID)) == 0,
                   "rowchain: the first GEMM takes only an activation");
    const int f = g2->flags;
    DPVO_CHECK_ARG(!((f & DPVO_RG_RES) || (f & DPVO_RG_GATE)) || g2->res32, "rowchain: residual input missing");
    DPVO_CHECK_ARG(!(f & DPVO_RG_GATE) || g2->gate16 || gate, "rowchain: gate input missing");
    if (gate) {
        DPVO_CHECK_ARG(f & DPVO_RG_GATE, "rowchain_gated: the second GEMM's flags must include DPVO_RG_GATE");
        DPVO_CHECK_ARG(!g2->gate16, "rowchain_gated: gate16 must be NULL (the gate is computed on chip)");
        DPVO_CHECK_ARG(gate->W && gate->bias && ((uintptr_t)gate->W & 15) == 0 && ((uintptr_t)gate->bias & 7) == 0,
                       "rowchain_gated: gate W (16-byte aligned) and bias (8-byte aligned) are required");
        DPVO_CHECK_ARG(gate->K == g1->K && gate->N == RG_BN, "rowchain_gated: gate W must be [384][K1] like W1");
    }
    DPVO_CHECK_ARG(!(f & DPVO_RG_LN) || (g2->ln_g && g2->ln_b), "rowchain: LayerNorm weights missing");
    DPVO_CHECK_ARG(!(f & DPVO_RG_HEADS) || (g2->head_w && g2->head_b && g2->head_out), "rowchain: head weights missing");
    if (g1->M <= 0) return 0;
    if (ensure_num_cus()) return -1;
    const int64_t ntiles = (g1->M + RG_BM - 1) / RG_BM;
    // (at least ntiles / R5_IDX_TILES blocks: a block's row sources fit its LDS table)
    const unsigned grid = (unsigned)std::max<int64_t>(std::min<int64_t>(ntiles, g_num_cus), (ntiles + R5_IDX_TILES - 1) / R5_IDX_TILES);
    dpvo_rowgemm_args a2 = *g2;
    a2.M = g1->M;
    a2.M_dev = g1->M_dev;
    const bool relu1 = g1->flags == DPVO_RG_RELU;   // (the compile-time activation)
    if (pre) {   // the first GRU chain: the residual base is LayerNorm(pre rows), formed in the epilogue
        DPVO_CHECK_ARG(gate && f == (DPVO_RG_GATE | DPVO_RG_LN) && relu1,
                       "rowchain_gated_pre: a gated GATE | LN chain with a ReLU first GEMM");
        a2.gate16 = nullptr;
        a2.res16 = nullptr;
        hipLaunchKernelGGL((rowchain5_kernel<DPVO_RG_RES | DPVO_RG_LN | RG_NOADD, true, 0, RG_RELU, true>), dim3(grid),
                           dim3(R5_THREADS), 0, as_stream(stream), *g1, a2, *gate, *pre);
        DPVO_CHECK_LAUNCH();
        return 0;
    }
    if (gate) {
        // the gated y goes through the RES epilogue (res16 none): x + fp16(gate * y)
        a2.gate16 = nullptr;
        a2.res16 = nullptr;
        switch (f) {
// (no res16 in a gated chain: the addend loads compiled out, RG_NOADD)
#define RCG_NA RG_NOADD
#define RCG_CASE(F)                                                                                                   \
    case (F):                                                                                                         \
        if (relu1)                                                                                                    \
            hipLaunchKernelGGL((rowchain5_kernel<((F) & ~DPVO_RG_GATE) | DPVO_RG_RES | RCG_NA, true, 0, RG_RELU>),    \
                               dim3(grid), dim3(R5_THREADS), 0, as_stream(stream), *g1, a2, *gate, dpvo_rowadd_args{});                   \
        else                                                                                                          \
            hipLaunchKernelGGL((rowchain5_kernel<((F) & ~DPVO_RG_GATE) | DPVO_RG_RES | RCG_NA, true>), dim3(grid),    \
                               dim3(R5_THREADS), 0, as_stream(stream), *g1, a2, *gate, dpvo_rowadd_args{});                               \
        break;
            RCG_CASE(DPVO_RG_GATE | DPVO_RG_LN)
            RCG_CASE(DPVO_RG_GATE | DPVO_RG_HEADS)
#undef RCG_CASE
#undef RCG_NA
        default:
            set_error("dpvo_rowchain_gated: unsupported epilogue flag combination " + std::to_string(f));
            return -1;
        }
        DPVO_CHECK_LAUNCH();
        return 0;
    }
    if (f == DPVO_RG_RES && !g2->res16) {   // (c1 / c2: no addend loads, + 0 in their place)
        if (relu1)
            hipLaunchKernelGGL((rowchain5_kernel<DPVO_RG_RES | RG_NOADD, false, 0, RG_RELU>), dim3(grid),
                               dim3(R5_THREADS), 0, as_stream(stream), *g1, a2, a2, dpvo_rowadd_args{});
        else
            hipLaunchKernelGGL((rowchain5_kernel<DPVO_RG_RES | RG_NOADD>), dim3(grid), dim3(R5_THREADS), 0,
                               as_stream(stream), *g1, a2, a2, dpvo_rowadd_args{});
        DPVO_CHECK_LAUNCH();
        return 0;
    }
    switch (f) {
#define RCH_CASE(F)                                                                                                   \
    case (F):                                                                                                         \
        if (relu1)                                                                                                    \
            hipLaunchKernelGGL((rowchain5_kernel<(F), false, 0, RG_RELU>), dim3(grid), dim3(R5_THREADS), 0,           \
                               as_stream(stream), *g1, a2, a2, dpvo_rowadd_args{});                                   \
        else                                                                                                          \
            hipLaunchKernelGGL(rowchain5_kernel<(F)>, dim3(grid), dim3(R5_THREADS), 0, as_stream(stream), *g1, a2,   \
                               a2, dpvo_rowadd_args{});                                                               \
        break;
        RCH_CASE(DPVO_RG_LN | DPVO_RG_LN_RELU)
        RCH_CASE(DPVO_RG_RES)
        RCH_CASE(DPVO_RG_GATE | DPVO_RG_LN)
        RCH_CASE(DPVO_RG_GATE | DPVO_RG_HEADS)
#undef RCH_CASE
    default:
        set_error("dpvo_rowchain: unsupported epilogue flag combination " + std::to_string(f));
        return -1;
    }
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_rowchain(const dpvo_rowgemm_args* g1, const dpvo_rowgemm_args* g2, void* stream)
{
    return rowchain_launch(g1, g2, nullptr, stream);
}

extern "C" int dpvo_rowchain3(const dpvo_rowgemm_args* g1, const dpvo_rowgemm_args* g2, const dpvo_rowgemm_args* g3,
                              void* stream)
{
    DPVO_CHECK_ARG(g1 != nullptr && g2 != nullptr && g3 != nullptr, "rowchain3: null args");
    DPVO_CHECK_ARG(g2->N == RG_BN && g2->K == RG_BN && g2->W && g2->bias && ((uintptr_t)g2->W & 15) == 0 &&
                       ((uintptr_t)g2->bias & 7) == 0,
                   "rowchain3: the middle Linear needs W [384][384] (16-byte aligned) and bias (8-byte aligned)");
    DPVO_CHECK_ARG(g2->flags == (DPVO_RG_LN | DPVO_RG_LN_RELU) && g2->ln_g && g2->ln_b &&
                       ((uintptr_t)g2->ln_g & 15) == 0 && ((uintptr_t)g2->ln_b & 15) == 0,
                   "rowchain3: the middle epilogue must be LN | LN_RELU with 16-byte aligned LayerNorm parameters");
    DPVO_CHECK_ARG(g3->flags == (DPVO_RG_RES | DPVO_RG_LN), "rowchain3: the last epilogue must be RES | LN");
    DPVO_CHECK_ARG(g1->N == RG_BN && g3->N == RG_BN, "rowchain3: output widths must be 384");
    DPVO_CHECK_ARG(g1->K > 0 && g1->K % 64 == 0, "rowchain3: K1 must be a positive multiple of 64");
    DPVO_CHECK_ARG(g3->K == RG_BN, "rowchain3: the last GEMM's K must be 384");
    DPVO_CHECK_ARG(g1->A && g1->W && g1->bias && g1->zero_row && g3->W && g3->bias,
                   "rowchain3: A, the three W, the biases and zero_row are required");
    DPVO_CHECK_ARG(g1->lda >= g1->K && g1->lda % 8 == 0, "rowchain3: lda must be >= K1 and a multiple of 8");
    DPVO_CHECK_ARG(((uintptr_t)g1->A & 15) == 0 && ((uintptr_t)g1->W & 15) == 0 && ((uintptr_t)g3->W & 15) == 0 &&
                       ((uintptr_t)g1->zero_row & 15) == 0,
                   "rowchain3: A, W1, W3 and zero_row must be 16-byte aligned");
    DPVO_CHECK_ARG(((uintptr_t)g1->bias & 7) == 0 && ((uintptr_t)g3->bias & 7) == 0,
                   "rowchain3: biases must be 8-byte aligned");
    DPVO_CHECK_ARG((g1->flags & ~(DPVO_RG_RELU | DPVO_RG_SIGMOID)) == 0,
                   "rowchain3: the first GEMM takes only an activation");
    DPVO_CHECK_ARG(g3->res32 && g3->ln_g && g3->ln_b, "rowchain3: residual input / LayerNorm weights missing");
    DPVO_CHECK_ARG(!g3->out16 || (g3->ldo16 % 4 == 0 && ((uintptr_t)g3->out16 & 7) == 0),
                   "rowchain3: out16 needs 8-byte aligned rows (ldo16 % 4 == 0)");
    DPVO_CHECK_ARG(!g3->out32 || (g3->ldo32 % 4 == 0 && ((uintptr_t)g3->out32 & 15) == 0),
                   "rowchain3: out32 needs 16-byte aligned rows (ldo32 % 4 == 0)");
    if (g1->M <= 0) return 0;
    if (ensure_num_cus()) return -1;
    const int64_t ntiles = (g1->M + RG_BM - 1) / RG_BM;
    // (at least ntiles / R5_IDX_TILES blocks: a block's row sources fit its LDS table)
    const unsigned grid = (unsigned)std::max<int64_t>(std::min<int64_t>(ntiles, g_num_cus), (ntiles + R5_IDX_TILES - 1) / R5_IDX_TILES);
    dpvo_rowgemm_args a3 = *g3;
    a3.M = g1->M;
    a3.M_dev = g1->M_dev;
    if (g1->flags == DPVO_RG_RELU)
        hipLaunchKernelGGL((rowchain5_kernel<DPVO_RG_RES | DPVO_RG_LN, false, DPVO_RG_LN | DPVO_RG_LN_RELU, RG_RELU>),
                           dim3(grid), dim3(R5_THREADS), 0, as_stream(stream), *g1, a3, *g2, dpvo_rowadd_args{});
    else
        hipLaunchKernelGGL((rowchain5_kernel<DPVO_RG_RES | DPVO_RG_LN, false, DPVO_RG_LN | DPVO_RG_LN_RELU>),
                           dim3(grid), dim3(R5_THREADS), 0, as_stream(stream), *g1, a3, *g2, dpvo_rowadd_args{});
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_rowchain_gated(const dpvo_rowgemm_args* gate, const dpvo_rowgemm_args* g1,
                                   const dpvo_rowgemm_args* g2, void* stream)
{
    DPVO_CHECK_ARG(gate != nullptr, "rowchain_gated: gate args missing");
    return rowchain_launch(g1, g2, gate, stream);
}

extern "C" int dpvo_rowchain_gated_pre(const dpvo_rowgemm_args* gate, const dpvo_rowgemm_args* g1,
                                       const dpvo_rowgemm_args* g2, const dpvo_rowadd_args* pre, void* stream)
{
    DPVO_CHECK_ARG(gate != nullptr && pre != nullptr, "rowchain_gated_pre: gate / pre args missing");
    DPVO_CHECK_ARG(pre->a && !pre->a_f16 && pre->lda >= RG_BN && pre->lda % 4 == 0 && ((uintptr_t)pre->a & 15) == 0,
                   "rowchain_gated_pre: pre.a must be fp32 rows of >= 384 (16-byte aligned)");
    DPVO_CHECK_ARG(pre->ln_g && pre->ln_b && ((uintptr_t)pre->ln_g & 15) == 0 && ((uintptr_t)pre->ln_b & 15) == 0,
                   "rowchain_gated_pre: pre.ln_g / ln_b (16-byte aligned) are required");
    DPVO_CHECK_ARG((!pre->b16 || ((uintptr_t)pre->b16 & 7) == 0) && (!pre->c16 || ((uintptr_t)pre->c16 & 7) == 0),
                   "rowchain_gated_pre: pre.b16 / c16 must be 8-byte aligned");
    DPVO_CHECK_ARG(!pre->c16 || pre->b16, "rowchain_gated_pre: c16 needs b16");
    DPVO_CHECK_ARG(pre->M == g1->M && !g1->M_dev, "rowchain_gated_pre: pre.M must be the chain's row count");
    DPVO_CHECK_ARG(!g2->res32 && !g2->res16, "rowchain_gated_pre: the residual comes from pre (res32 / res16 NULL)");
    dpvo_rowgemm_args b2 = *g2;
    b2.res32 = pre->a;   // (rowchain_launch's residual check; the kernel reads pre)
    b2.ldr = pre->lda;
    return rowchain_launch(g1, &b2, gate, stream, pre);
}

#ifdef DPVO_STAMPS
extern "C" int dpvo_diag_stamps(void* host, size_t bytes)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(dpvo_stamps), std::min(bytes, sizeof(dpvo_stamps)), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int dpvo_rowadd_ln(const dpvo_rowadd_args* a, void* stream)
{
    DPVO_CHECK_ARG(a != nullptr, "rowadd_ln: args missing");
    if (a->M <= 0) return 0;   // (empty tensors may carry null data pointers)
    DPVO_CHECK_ARG(a->a != nullptr, "rowadd_ln: input missing");
    DPVO_CHECK_ARG(a->lda >= RG_BN && a->lda % 4 == 0, "rowadd_ln: lda must be a multiple of 4 and >= 384");
    DPVO_CHECK_ARG((uintptr_t)a->a % (a->a_f16 ? 8 : 16) == 0, "rowadd_ln: input rows must be vector aligned");
    DPVO_CHECK_ARG(!a->b16 || (uintptr_t)a->b16 % 8 == 0, "rowadd_ln: b16 must be 8-byte aligned");
    DPVO_CHECK_ARG(!a->c16 || (uintptr_t)a->c16 % 8 == 0, "rowadd_ln: c16 must be 8-byte aligned");
    DPVO_CHECK_ARG(!a->c16 || a->b16, "rowadd_ln: c16 needs b16 (the second addend follows the first)");
    DPVO_CHECK_ARG(!a->ln_g || ((uintptr_t)a->ln_g % 16 == 0 && (uintptr_t)a->ln_b % 16 == 0),
                   "rowadd_ln: LayerNorm parameters must be 16-byte aligned");
    DPVO_CHECK_ARG((!a->out32 || (uintptr_t)a->out32 % 16 == 0) && (!a->out16 || (uintptr_t)a->out16 % 8 == 0),
                   "rowadd_ln: outputs must be vector aligned");
    DPVO_CHECK_ARG(a->out32 || a->out16, "rowadd_ln: no output");
    DPVO_CHECK_ARG(!a->ln_g == !a->ln_b, "rowadd_ln: LayerNorm needs both weight and bias");
    if (a->M <= 0) return 0;
    const unsigned grid = grid_for(a->M * 32, 256, 16384);
    if (a->a_f16)
        hipLaunchKernelGGL(rowadd_ln_kernel<true>, dim3(grid), dim3(256), 0, as_stream(stream), *a);
    else
        hipLaunchKernelGGL(rowadd_ln_kernel<false>, dim3(grid), dim3(256), 0, as_stream(stream), *a);
    DPVO_CHECK_LAUNCH();
    return 0;
}

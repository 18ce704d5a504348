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
constexpr int RG_STAGE = RG_A_STAGE + RG_W_STAGE;
constexpr int RG_EXTRA = 32 * 1024;             // + the consumed stage = the 96 KB y tile
constexpr int RG_LDS = 2 * RG_STAGE + RG_EXTRA;  // 160 KB: the whole CU

enum {
    RG_RELU = DPVO_RG_RELU, RG_SIGMOID = DPVO_RG_SIGMOID, RG_RES = DPVO_RG_RES, RG_GATE = DPVO_RG_GATE,
    RG_LN = DPVO_RG_LN, RG_LN_RELU = DPVO_RG_LN_RELU, RG_HEADS = DPVO_RG_HEADS
};

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
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

// sum over the 64 lanes, broadcast (DPP row reduce + 4 readlanes)
__device__ __forceinline__ float wave_sum(float s)
{
    s = rowsum16(s);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 0)) +
           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 16)) +
           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 32)) +
           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 48));
}

// y tile: 128 rows x 768 B (fp16 row-major) spread over the consumed stage
// buffer (64 KB) and the extra region (32 KB); 32-B granules XOR-swizzled by
// (row/4)&3 so the C-layout b16 writes of 4 row groups hit distinct banks.
__device__ __forceinline__ int ytile_off(int cur_buf, int r, int byte)
{
    const int o = r * 768 + (byte ^ (((r >> 2) & 3) << 5));
    return o < 65536 ? cur_buf * 65536 + o : 2 * RG_STAGE + (o - 65536);
}

__device__ __forceinline__ float fast_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

struct EpiConsts {
    float2_t g[3], b[3];     // LayerNorm weight / bias at this lane's columns
    float2_t hw[4][3];       // head weights (fp16 values)
    float hb[4];
};

template <int FLAGS>
__device__ __forceinline__ void load_consts(const dpvo_rowgemm_args& p, int lane, EpiConsts& k)
{
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const int c = 128 * j + 2 * lane;
        if (FLAGS & RG_LN) {
            k.g[j] = *(const float2_t*)(p.ln_g + c);
            k.b[j] = *(const float2_t*)(p.ln_b + c);
        }
        if (FLAGS & RG_HEADS) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const half2_t w = *(const half2_t*)((const half_t*)p.head_w + q * RG_BN + c);
                k.hw[q][j] = float2_t{(float)w.x, (float)w.y};
            }
        }
    }
    if (FLAGS & RG_HEADS) {
#pragma unroll
        for (int q = 0; q < 4; q++) k.hb[q] = (float)((const half_t*)p.head_b)[q];
    }
}

// R whole output rows per wave (lane owns columns 2*lane + 128*j, j < 3):
// all of the batch's loads are issued before any row's reductions.
struct YMapFull {   // v1: 128-row tile over the consumed stage + extra region
    int cur_buf;
    __device__ int off(int r, int byte) const { return ytile_off(cur_buf, r, byte); }
};

// The row epilogue in two halves: epi_load issues a batch's residual / gate
// operand loads, epi_finish combines them with y and runs LN / heads / stores.
// (v4 issues batch b + 1's loads before finishing batch b.)
template <int R>
struct EpiOps {
    float2_t base[R][3];   // res32
    half2_t add[R][3];     // res16[idx] or gate16
};

template <int FLAGS, int R>
__device__ __forceinline__ void epi_load(const dpvo_rowgemm_args& p, int64_t M, int64_t row0, int lane, EpiOps<R>& o)
{
    if (!(FLAGS & (RG_RES | RG_GATE))) return;
#pragma unroll
    for (int q = 0; q < R; q++) {
        const int64_t row = row0 + q < M ? row0 + q : M - 1;   // clamped for loads; stores skip rows >= M
        const float* r32 = (const float*)p.res32 + row * p.ldr;
        const half_t* r16 = nullptr;
        if (FLAGS & RG_GATE) {
            r16 = (const half_t*)p.gate16 + row * RG_BN;
        } else if (p.res16) {
            const int64_t s = p.res16_idx ? p.res16_idx[row] : row;
            r16 = s >= 0 ? (const half_t*)p.res16 + s * RG_BN : nullptr;
        }
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int c = 128 * j + 2 * lane;
            o.base[q][j] = *(const float2_t*)(r32 + c);
            o.add[q][j] = r16 ? *(const half2_t*)(r16 + c) : half2_t{(half_t)0, (half_t)0};
        }
    }
}

template <int FLAGS, int R, typename YMap>
__device__ __forceinline__ void epi_finish(const dpvo_rowgemm_args& p, int64_t M, const char* smem, YMap ym, int lrow0,
                                           int64_t row0, int lane, const EpiConsts& k, const EpiOps<R>& o)
{
    float2_t v[R][3];
#pragma unroll
    for (int q = 0; q < R; q++) {
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const half2_t y = *(const half2_t*)(smem + ym.off(lrow0 + q, (128 * j + 2 * lane) * 2));
            v[q][j] = float2_t{(float)y.x, (float)y.y};
        }
    }
    if (FLAGS & (RG_RES | RG_GATE)) {
#pragma unroll
        for (int q = 0; q < R; q++)
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const float2_t add = float2_t{(float)o.add[q][j].x, (float)o.add[q][j].y};
                if (FLAGS & RG_GATE)   // x + fp16(gate * res)   (blocks.py:30, fp16 product)
                    v[q][j] = o.base[q][j] + float2_t{hround(add.x * v[q][j].x), hround(add.y * v[q][j].y)};
                else                   // (res32 + res16) + y
                    v[q][j] = (o.base[q][j] + add) + v[q][j];
            }
    }
    if (FLAGS & RG_LN) {
        float mean[R];
#pragma unroll
        for (int q = 0; q < R; q++) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 3; j++) s += v[q][j].x + v[q][j].y;
            mean[q] = wave_sum(s) * (1.f / RG_BN);
        }
#pragma unroll
        for (int q = 0; q < R; q++) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const float2_t d = v[q][j] - mean[q];
                s += d.x * d.x + d.y * d.y;
            }
            const float rstd = rsqrtf(wave_sum(s) * (1.f / RG_BN) + p.ln_eps);
#pragma unroll
            for (int j = 0; j < 3; j++) {
                v[q][j] = (v[q][j] - mean[q]) * rstd * k.g[j] + k.b[j];
                if (FLAGS & RG_LN_RELU) v[q][j] = float2_t{fmaxf(v[q][j].x, 0.f), fmaxf(v[q][j].y, 0.f)};
            }
        }
    }
    if (FLAGS & RG_HEADS) {
        // d = W_d relu(v) + b_d ; w = sigmoid(W_w relu(v) + b_w)   (fp16 operands, fp32 accumulate)
#pragma unroll
        for (int q = 0; q < R; q++) {
            float d[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const float x0 = hround(fmaxf(v[q][j].x, 0.f)), x1 = hround(fmaxf(v[q][j].y, 0.f));
#pragma unroll
                for (int h = 0; h < 4; h++) d[h] += x0 * k.hw[h][j].x + x1 * k.hw[h][j].y;
            }
            half_t o[4];
#pragma unroll
            for (int h = 0; h < 4; h++) {
                float z = hround(wave_sum(d[h]) + k.hb[h]);
                if (h >= 2) z = hround(fast_sigmoid(z));
                o[h] = (half_t)z;
            }
            if (lane == 0 && row0 + q < M) {
                typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
                *(h4_t*)((half_t*)p.head_out + (row0 + q) * 4) = h4_t{o[0], o[1], o[2], o[3]};
            }
        }
    }
#pragma unroll
    for (int q = 0; q < R; q++) {
        if (row0 + q >= M) continue;
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int c = 128 * j + 2 * lane;
            if (p.out32) *(float2_t*)((float*)p.out32 + (row0 + q) * p.ldo32 + c) = v[q][j];
            if (p.out16)
                *(half2_t*)((half_t*)p.out16 + (row0 + q) * p.ldo16 + c) = half2_t{(half_t)v[q][j].x, (half_t)v[q][j].y};
        }
    }
}


template <int FLAGS, int R, typename YMap>
__device__ __forceinline__ void epilogue_rows(const dpvo_rowgemm_args& p, int64_t M, const char* smem, YMap ym,
                                              int lrow0, int64_t row0, int lane, const EpiConsts& k)
{
    EpiOps<R> o;
    epi_load<FLAGS, R>(p, M, row0, lane, o);
    epi_finish<FLAGS, R>(p, M, smem, ym, lrow0, row0, lane, k, o);
}

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
        const half_t* r16 = nullptr;
        if (FLAGS & RG_GATE) {
            r16 = (const half_t*)p.gate16 + row * RG_BN;
        } else if (p.res16) {
            const int64_t src = p.res16_idx ? p.res16_idx[row] : row;
            r16 = src >= 0 ? (const half_t*)p.res16 + src * RG_BN : nullptr;
        }
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int c = 128 * j + 4 * s;
            o.base[i][j] = *(const ep_f4*)(r32 + c);
            o.add[i][j] = r16 ? *(const ep_h4*)(r16 + c) : ep_h4{(half_t)0, (half_t)0, (half_t)0, (half_t)0};
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
                const ep_f4 add = ep_f4{(float)o.add[i][j][0], (float)o.add[i][j][1], (float)o.add[i][j][2],
                                        (float)o.add[i][j][3]};
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

template <int FLAGS>
__global__ __launch_bounds__(RG_THREADS, 1) void rowgemm_kernel(dpvo_rowgemm_args p)
{
    __shared__ __attribute__((aligned(16))) char smem[RG_LDS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int K = p.K;
    const int ksteps = K / RG_BK;
    const int64_t Mrows = p.M_dev ? min(*p.M_dev, p.M) : p.M;
    const int64_t ntiles = (Mrows + RG_BM - 1) / RG_BM;
    if ((int64_t)blockIdx.x >= ntiles) return;
    const int64_t my_tiles = (ntiles - 1 - blockIdx.x) / gridDim.x + 1;
    const int64_t total = my_tiles * ksteps;

    const half_t* __restrict__ Wt = (const half_t*)p.W;
    const half_t* __restrict__ zero = (const half_t*)p.zero_row;

    // staging sources: lane L of a wave-instruction fills LDS row base+L/8,
    // physical 16-B chunk L%8, holding logical chunk (L%8) ^ ((row>>1)&7)
    const int srow = lane >> 3, pch = lane & 7;
    const half_t* wsrc[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const int n = (wave * 6 + j) * 8 + srow;
        wsrc[j] = Wt + (int64_t)n * K + 8 * (pch ^ ((n >> 1) & 7));
    }
    const half_t* asrc[2];
    auto set_tile_a = [&](int64_t tile) {
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int r = (wave * 2 + j) * 8 + srow;
            const int64_t m = tile * RG_BM + r;
            const half_t* row = zero;
            if (m < Mrows) {
                const int64_t s = p.a_idx ? p.a_idx[m] : m;
                if (s >= 0 && s < p.a_rows) row = (const half_t*)p.A + s * p.lda;
            }
            asrc[j] = row + 8 * (pch ^ ((r >> 1) & 7));
        }
    };
    // stage s (0..ksteps) of the block's j-th tile -> buffer parity of the flat index
    auto issue = [&](int ks, int64_t tile, int buf) {
        if (ks == 0) set_tile_a(tile);
        char* sA = smem + buf * RG_STAGE;
        char* sW = sA + RG_A_STAGE;
        const int k0 = ks * RG_BK;
        glds16(asrc[0] + k0, sA + (wave * 2 + 0) * 1024);
        glds16(asrc[1] + k0, sA + (wave * 2 + 1) * 1024);
#pragma unroll
        for (int j = 0; j < 6; j++) glds16(wsrc[j] + k0, sW + (wave * 6 + j) * 1024);
    };

    f4_t acc[4][6];
#pragma unroll
    for (int mt = 0; mt < 4; mt++)
#pragma unroll
        for (int nt = 0; nt < 6; nt++) acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};

    // fragment read offsets (bytes within a stage), k-step independent part
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
        w_off[nt] = RG_A_STAGE + n * 128;
        w_sw[nt] = (n >> 1) & 7;
    }

    EpiConsts kc;
    load_consts<FLAGS>(p, lane, kc);
    int64_t tile = blockIdx.x;
    int ks = 0, buf = 0;
    issue(0, tile, 0);
    for (int64_t i = 0; i < total; i++) {
        // the flat sequence's next (tile, stage)
        int nks = ks + 1;
        int64_t ntile = tile;
        if (nks == ksteps) {
            nks = 0;
            ntile += gridDim.x;
        }
        if (i + 1 < total) {
            issue(nks, ntile, buf ^ 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* st = smem + buf * RG_STAGE;
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
            const int c = kk * 4 + fq;
            h8_t a[4], b[6];
#pragma unroll
            for (int mt = 0; mt < 4; mt++) a[mt] = *(const h8_t*)(st + a_off[mt] + 16 * (c ^ a_sw[mt]));
#pragma unroll
            for (int nt = 0; nt < 6; nt++) b[nt] = *(const h8_t*)(st + w_off[nt] + 16 * (c ^ w_sw[nt]));
#pragma unroll
            for (int mt = 0; mt < 4; mt++)
#pragma unroll
                for (int nt = 0; nt < 6; nt++)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
        }
        __builtin_amdgcn_s_barrier();
        const int cur_buf = buf;
        const int64_t cur_tile = tile;
        const bool last = ks == ksteps - 1;
        ks = nks;
        tile = ntile;
        buf ^= 1;
        if (!last) continue;

        // ------------------------------ epilogue ------------------------------
        // Every wave writes y16 = fp16(acc + b) [act] of its 64x96 block into
        // the y tile (consumed stage buffer + extra region), then finishes 16
        // whole rows: lanes over columns, coalesced loads/stores, DPP+readlane
        // row reductions.  The other stage buffer is loading the next tile.
#pragma unroll
        for (int nt = 0; nt < 6; nt++) {
            const int cl = wn * 96 + nt * 16 + fr;
            const float bias = (float)((const half_t*)p.bias)[cl];
#pragma unroll
            for (int mt = 0; mt < 4; mt++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    half_t y = (half_t)(acc[mt][nt][r] + bias);
                    if (FLAGS & RG_RELU) y = y > (half_t)0 ? y : (half_t)0;
                    if (FLAGS & RG_SIGMOID) y = (half_t)fast_sigmoid((float)y);
                    *(half_t*)(smem + ytile_off(cur_buf, wm * 64 + mt * 16 + fq * 4 + r, cl * 2)) = y;
                    acc[mt][nt][r] = 0.f;
                }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        epilogue_rows<FLAGS, 8>(p, Mrows, smem, YMapFull{cur_buf}, wave * 16, cur_tile * RG_BM + wave * 16, lane, kc);
        __builtin_amdgcn_sched_barrier(0);
        epilogue_rows<FLAGS, 8>(p, Mrows, smem, YMapFull{cur_buf}, wave * 16 + 8, cur_tile * RG_BM + wave * 16 + 8,
                                lane, kc);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
}


// ---------------------------------------------------------------------------
// v2: two workgroups per CU.  BM = 64 rows, 4 waves (each 64 rows x 96 columns,
// the same 4 x 6 accumulators), BK = 32 stages (A 4 KB + W 24 KB), 56 KB of
// LDS per workgroup.  The epilogue stages 32-row halves of y through the
// consumed stage buffer.  With two resident workgroups one's HBM-bound
// epilogue overlaps the other's MFMA loop.
// ---------------------------------------------------------------------------
constexpr int R2_BM = 64, R2_BK = 32, R2_THREADS = 256;
constexpr int R2_A_STAGE = R2_BM * R2_BK * 2;    // 4 KB
constexpr int R2_W_STAGE = RG_BN * R2_BK * 2;    // 24 KB
constexpr int R2_STAGE = R2_A_STAGE + R2_W_STAGE;
constexpr int R2_LDS = 2 * R2_STAGE;             // 56 KB

struct YMapHalf {   // v2: 32 rows x 768 B in one stage buffer, 32-B granules XOR (row/4)&3
    int base;
    __device__ int off(int r, int byte) const { return base + r * 768 + (byte ^ (((r >> 2) & 3) << 5)); }
};

template <int FLAGS>
__global__ __launch_bounds__(R2_THREADS, 2) void rowgemm2_kernel(dpvo_rowgemm_args p)
{
    __shared__ __attribute__((aligned(16))) char smem[R2_LDS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int K = p.K;
    const int ksteps = K / R2_BK;
    const int64_t Mrows = p.M_dev ? min(*p.M_dev, p.M) : p.M;
    const int64_t ntiles = (Mrows + R2_BM - 1) / R2_BM;
    if ((int64_t)blockIdx.x >= ntiles) return;
    const int64_t my_tiles = (ntiles - 1 - blockIdx.x) / gridDim.x + 1;
    const int64_t total = my_tiles * ksteps;

    const half_t* __restrict__ Wt = (const half_t*)p.W;
    const half_t* __restrict__ zero = (const half_t*)p.zero_row;
    // staging: lane L of a wave-instruction fills LDS row base + L/4, physical 16-B
    // chunk L%4, holding logical chunk (L%4) ^ ((row>>2)&3)
    const int srow = lane >> 2, pch = lane & 3;
    const half_t* wsrc[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const int n = (wave * 6 + j) * 16 + srow;
        wsrc[j] = Wt + (int64_t)n * K + 8 * (pch ^ ((n >> 2) & 3));
    }
    const half_t* asrc;
    auto set_tile_a = [&](int64_t tile) {
        const int r = wave * 16 + srow;
        const int64_t m = tile * R2_BM + r;
        const half_t* row = zero;
        if (m < Mrows) {
            const int64_t s = p.a_idx ? p.a_idx[m] : m;
            if (s >= 0 && s < p.a_rows) row = (const half_t*)p.A + s * p.lda;
        }
        asrc = row + 8 * (pch ^ ((r >> 2) & 3));
    };
    auto issue = [&](int ks, int64_t tile, int buf) {
        if (ks == 0) set_tile_a(tile);
        char* sA = smem + buf * R2_STAGE;
        char* sW = sA + R2_A_STAGE;
        const int k0 = ks * R2_BK;
        glds16(asrc + k0, sA + wave * 1024);
#pragma unroll
        for (int j = 0; j < 6; j++) glds16(wsrc[j] + k0, sW + (wave * 6 + j) * 1024);
    };

    f4_t acc[4][6];
#pragma unroll
    for (int mt = 0; mt < 4; mt++)
#pragma unroll
        for (int nt = 0; nt < 6; nt++) acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fq = lane >> 4;
    int a_off[4], w_off[6];
#pragma unroll
    for (int mt = 0; mt < 4; mt++) {
        const int row = mt * 16 + fr;
        a_off[mt] = row * 64 + 16 * (fq ^ ((row >> 2) & 3));
    }
#pragma unroll
    for (int nt = 0; nt < 6; nt++) {
        const int n = wave * 96 + nt * 16 + fr;
        w_off[nt] = R2_A_STAGE + n * 64 + 16 * (fq ^ ((n >> 2) & 3));
    }
    EpiConsts kc;
    load_consts<FLAGS>(p, lane, kc);

    int64_t tile = blockIdx.x;
    int ks = 0, buf = 0;
    issue(0, tile, 0);
    for (int64_t i = 0; i < total; i++) {
        int nks = ks + 1;
        int64_t ntile = tile;
        if (nks == ksteps) {
            nks = 0;
            ntile += gridDim.x;
        }
        if (i + 1 < total) {
            issue(nks, ntile, buf ^ 1);
            asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* st = smem + buf * R2_STAGE;
        h8_t a[4], b[6];
#pragma unroll
        for (int mt = 0; mt < 4; mt++) a[mt] = *(const h8_t*)(st + a_off[mt]);
#pragma unroll
        for (int nt = 0; nt < 6; nt++) b[nt] = *(const h8_t*)(st + w_off[nt]);
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
#pragma unroll
            for (int nt = 0; nt < 6; nt++)
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
        __builtin_amdgcn_s_barrier();
        const int cur_buf = buf;
        const int64_t cur_tile = tile;
        const bool last = ks == ksteps - 1;
        ks = nks;
        tile = ntile;
        buf ^= 1;
        if (!last) continue;

        // epilogue in two 32-row halves through the consumed stage buffer
#pragma unroll
        for (int h = 0; h < 2; h++) {
#pragma unroll
            for (int nt = 0; nt < 6; nt++) {
                const int cl = wave * 96 + nt * 16 + fr;
                const float bias = (float)((const half_t*)p.bias)[cl];
#pragma unroll
                for (int mm = 0; mm < 2; mm++) {
                    const int mt = 2 * h + mm;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        half_t y = (half_t)(acc[mt][nt][r] + bias);
                        if (FLAGS & RG_RELU) y = y > (half_t)0 ? y : (half_t)0;
                        if (FLAGS & RG_SIGMOID) y = (half_t)fast_sigmoid((float)y);
                        *(half_t*)(smem + YMapHalf{cur_buf * R2_STAGE}.off(mm * 16 + fq * 4 + r, cl * 2)) = y;
                        acc[mt][nt][r] = 0.f;
                    }
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            constexpr int RB = (FLAGS & (RG_RES | RG_GATE)) ? 4 : 8;   // rows per batch (register budget)
#pragma unroll
            for (int q0 = 0; q0 < 8; q0 += RB)
                epilogue_rows<FLAGS, RB>(p, Mrows, smem, YMapHalf{cur_buf * R2_STAGE}, wave * 8 + q0,
                                         cur_tile * R2_BM + h * 32 + wave * 8 + q0, lane, kc);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
    }
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
// LDS: the y tile (96 KB; GEMM2's A operand, then its output for the row
// epilogue) + two 32 KB stages (BK = 32: A 8 KB | W 24 KB for GEMM1, W only
// for GEMM2).  Transposed accumulators as in v3.
// ---------------------------------------------------------------------------
constexpr int RC_BK = 32;
constexpr int RC_A_STAGE = RG_BM * RC_BK * 2;      // 8 KB
constexpr int RC_W_STAGE = RG_BN * RC_BK * 2;      // 24 KB
constexpr int RC_STAGE = RC_A_STAGE + RC_W_STAGE;  // 32 KB
constexpr int RC_Y = RG_BM * 768;                  // 96 KB
constexpr int RC_LDS = RC_Y + 2 * RC_STAGE;        // 160 KB

constexpr int RC_RN = 6, RC_RD = RC_RN - 2;   // A ring: 6 x 16 KB slots in the y-tile region, 4 stages ahead

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
// DBG (timing experiments only, DPVO_RC_DBG, flag RES; scripts/bench_rc_dbg.py):
// 1 no row pass, 2 no MFMA, 3 neither; 256 GEMM1's A through a ring in the y-tile region;
// 512 ping-pong wave groups
template <int F2, bool GATED = false, int DBG = 0, int FMID = 0>
__global__ __launch_bounds__(RG_THREADS, 1) void rowchain_kernel(dpvo_rowgemm_args p1, dpvo_rowgemm_args p,
                                                                 dpvo_rowgemm_args pg)
{
    constexpr bool TRI = FMID != 0;
    static_assert(!(TRI && GATED), "a chain is either gated or three GEMMs long");
    __shared__ __attribute__((aligned(16))) char smem[RC_LDS];
    typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int K1 = p1.K, ks1 = K1 / RC_BK, ks2 = RG_BN / RC_BK;
    const int64_t Mrows = p1.M_dev ? min(*p1.M_dev, p1.M) : p1.M;
    const int64_t ntiles = (Mrows + RG_BM - 1) / RG_BM;
    if ((int64_t)blockIdx.x >= ntiles) return;
    const half_t* __restrict__ W1 = (const half_t*)p1.W;
    const half_t* __restrict__ W2 = (const half_t*)(TRI ? pg.W : p.W);
    const half_t* __restrict__ zero = (const half_t*)p1.zero_row;
    // TRI: the third GEMM's W stages come from p.W ([384][384] like W2)
    const int64_t w3delta = TRI ? (const half_t*)p.W - W2 : 0;
    const YMapChunk ym;
    // piece (1 KB = 16 rows x 64 B) lane mapping: row base + L/4, physical chunk
    // L%4 holding logical chunk (L%4) ^ ((row>>2)&3)
    const int srow = lane >> 2, pch = lane & 3;
    // GEMM1 stage: pieces 4 wave .. 4 wave + 3 of 32 (0-7 A rows, 8-31 W1 rows)
    const half_t* g1src[4];
    auto set_tile = [&](int64_t tile) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int pc = 4 * wave + j;
            if (pc < 8) {
                const int r = pc * 16 + srow;
                const int64_t m = tile * RG_BM + r;
                const half_t* row = zero;
                if (m < Mrows) {
                    const int64_t s = p1.a_idx ? p1.a_idx[m] : m;
                    if (s >= 0 && s < p1.a_rows) row = (const half_t*)p1.A + s * p1.lda;
                }
                g1src[j] = row + 8 * (pch ^ ((r >> 2) & 3));
            }
        }
    };
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int pc = 4 * wave + j;   // A pieces then W pieces, contiguous within the stage
        if (pc >= 8) {   // W1 k-blocked [K1/32][384][32]: a stage's 384 rows are one contiguous block
            const int n = (pc - 8) * 16 + srow;
            g1src[j] = W1 + (int64_t)n * RC_BK + 8 * (pch ^ ((n >> 2) & 3));
        }
    }
    // GEMM2 stage: W2 pieces 3 wave .. 3 wave + 2 of 24
    const half_t* w2src[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const int n = (3 * wave + j) * 16 + srow;
        w2src[j] = W2 + (int64_t)n * RC_BK + 8 * (pch ^ ((n >> 2) & 3));   // k-blocked like W1
    }
    // gate pass: the same stage layout, W pieces from Wg ([384][K1] like W1)
    const int64_t gdelta = GATED ? (const half_t*)pg.W - W1 : 0;
    // A pieces advance 32 columns per stage, k-blocked W pieces one 384 x 32 block
    // WROT (DPVO_RC_DBG=1024, timing only, wrong results): every block walks the
    // W stages in a k order rotated by its index, so the CUs of an XCD do not
    // all request the same 24 KB W block from L2 at the same time
    constexpr bool WROT = (DBG & 1024) != 0;
    auto wrot = [&](int ks, int nks) { return WROT ? (ks + (int)(blockIdx.x % (unsigned)nks)) % nks : ks; };
    auto issue1 = [&](int ks, int buf, bool gate = false) {
        char* st = smem + RC_Y + buf * RC_STAGE;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const bool wp = 4 * wave + j >= 8;
            const int64_t k0 = wp ? (int64_t)wrot(ks, ks1) * (RG_BN * RC_BK) : ks * RC_BK;
            glds16(g1src[j] + k0 + (GATED && gate && wp ? gdelta : 0), st + (4 * wave + j) * 1024);
        }
    };
    auto issue2 = [&](int ks, int buf, int64_t wdelta = 0) {
        char* st = smem + RC_Y + buf * RC_STAGE + RC_A_STAGE;
        const int64_t k0 = (int64_t)wrot(ks, ks2) * (RG_BN * RC_BK) + wdelta;
#pragma unroll
        for (int j = 0; j < 3; j++) glds16(w2src[j] + k0, st + (3 * wave + j) * 1024);
    };
    auto sync_lds = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    // ---- ping-pong k-loops (PP, DPVO_RC_DBG=512; measured no faster: the
    // k-loops are bound by the per-CU LDS-DMA fill rate, profiles/r3/NOTES.md):
    // the waves run as two groups,
    // G0 = waves 0-3 and G1 = waves 4-7 (one of each per SIMD), G1 one barrier
    // behind, so on every SIMD one wave's MFMAs run while the other wave reads
    // its fragments -- with both in step (DPVO_RC_DBG=512) each k-step costs
    // MFMA + LDS reads + DMA one after the other.  G0 issues every stage's
    // LDS-DMA (8 pieces per wave for GEMM1, 6 for the W-only stages) at the
    // start of its read phase and waits for it before the barrier that opens
    // its next read phase; G1 reads a stage one phase after G0.
    constexpr bool PP = (DBG & 512) != 0;
    const bool G0 = wave < 4;
    // G0 wave w issues stage pieces 2w, 2w+1 (A rows) and 8 + 6w .. + 5 (W rows;
    // one base pointer: the pieces are 512 elements apart in the k-blocked W)
    const half_t* qa[2];
    const int wq = ((6 * (wave & 3)) * 16 + srow) * RC_BK + 8 * (pch ^ ((srow >> 2) & 3));
    auto set_tile_pp = [&](int64_t tile) {
        if (!PP || !G0) return;
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int r = (2 * wave + j) * 16 + srow;
            const int64_t m = tile * RG_BM + r;
            const half_t* row = zero;
            if (m < Mrows) {
                const int64_t s = p1.a_idx ? p1.a_idx[m] : m;
                if (s >= 0 && s < p1.a_rows) row = (const half_t*)p1.A + s * p1.lda;
            }
            qa[j] = row + 8 * (pch ^ ((r >> 2) & 3));
        }
    };
    auto issue1_pp = [&](int ks, int buf, bool gate) {
        char* st = smem + RC_Y + buf * RC_STAGE;
#pragma unroll
        for (int j = 0; j < 2; j++) glds16(qa[j] + ks * RC_BK, st + (2 * wave + j) * 1024);
        const half_t* w = W1 + wq + (int64_t)ks * (RG_BN * RC_BK) + (GATED && gate ? gdelta : 0);
#pragma unroll
        for (int j = 0; j < 6; j++) glds16(w + 512 * j, st + (8 + 6 * wave + j) * 1024);
    };
    auto issue2_pp = [&](int ks, int buf, int64_t wdelta) {
        char* st = smem + RC_Y + buf * RC_STAGE + RC_A_STAGE;
        const half_t* w = W2 + wq + (int64_t)ks * (RG_BN * RC_BK) + wdelta;
#pragma unroll
        for (int j = 0; j < 6; j++) glds16(w + 512 * j, st + (6 * wave + j) * 1024);
    };
    auto bar = []() {
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    // ---- GEMM1's A stream through a ring in the (then unused) y-tile region
    // (RING, DPVO_RC_DBG=256): stages of 64 k (128 rows x 128 B = 16 KB, whole
    // lines), RC_RD stages in flight, issued by waves 0-3 only while waves 4-7
    // issue the W stages: vmcnt counts each wave's own loads in order, so the
    // W waves wait for one W stage and the A waves for the A stage issued
    // RC_RD stages back -- the gathered rows' HBM latency leaves the k-step.
    // Piece j of wave w (0-3) holds rows 8 (4 w + j) .. + 7, lane L row
    // 8 (4 w + j) + L / 8, physical chunk L % 8 = logical chunk ^ ((row >> 1) & 7).
    // measured slower than the stage-buffer A stream (c1 chain 157 vs 147 us,
    // k-loops alone 94 vs 85: profiles/r3/NOTES.md): timing experiment only
    constexpr bool RING = (DBG & 256) != 0;
    const bool awave = wave < 4;
    const half_t* rsrc[4];
    auto set_ring_tile = [&](int64_t tile) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int r = 8 * (4 * (wave & 3) + j) + (lane >> 3);
            const int64_t m = tile * RG_BM + r;
            const half_t* row = zero;
            if (m < Mrows) {
                const int64_t s = p1.a_idx ? p1.a_idx[m] : m;
                if (s >= 0 && s < p1.a_rows) row = (const half_t*)p1.A + s * p1.lda;
            }
            rsrc[j] = row + 8 * ((lane & 7) ^ ((r >> 1) & 7));
        }
    };
    auto issue_ring = [&](int st) {   // A stage st (k = 64 st ..) into ring slot st % RC_RN
        char* dst = smem + (st % RC_RN) * 16384 + (4 * (wave & 3)) * 1024;
#pragma unroll
        for (int j = 0; j < 4; j++) glds16(rsrc[j] + 64 * st, dst + j * 1024);
    };
    // W waves 4-7: the stage's 24 pieces, 6 each, into the W part of stage buffer buf
    auto issue_wonly = [&](int ks, int buf) {
        char* st = smem + RC_Y + buf * RC_STAGE;
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const int pc = 6 * (wave - 4) + j;   // W piece 0 .. 23 = stage piece 8 + pc
            const int n = pc * 16 + (lane >> 2);
            const half_t* src = W1 + (int64_t)n * RC_BK + 8 * ((lane & 3) ^ ((n >> 2) & 3));
            glds16(src + (int64_t)ks * (RG_BN * RC_BK), st + (8 + pc) * 1024);
        }
    };

    f4_t acc[4][6];
    const int fr = lane & 15, fq = lane >> 4;
    int a_off[4], w_off[6];
#pragma unroll
    for (int mt = 0; mt < 4; mt++) {
        const int row = wm * 64 + mt * 16 + fr;
        a_off[mt] = row * 64 + 16 * (fq ^ ((row >> 2) & 3));
    }
#pragma unroll
    for (int nt = 0; nt < 6; nt++) {
        const int n = wn * 96 + nt * 16 + fr;
        w_off[nt] = RC_A_STAGE + n * 64 + 16 * (fq ^ ((n >> 2) & 3));
    }
    auto zero_acc = [&]() {
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
#pragma unroll
            for (int nt = 0; nt < 6; nt++) acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
    };
    auto mfma_step = [&](const h8_t (&a)[4], const h8_t (&b)[6]) {
        if (DBG & 2) {
            acc[0][0][0] += (float)a[0][0] + (float)b[0][0];
            return;
        }
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
#pragma unroll
            for (int nt = 0; nt < 6; nt++)
                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[nt], a[mt], acc[mt][nt], 0, 0, 0);
    };
    // acc + bias -> act -> fp16 -> y tile (row mt*16+fr, columns 4 fq.. of block nt)
    // (called before any stage prefetch is in flight: its bias loads would
    // otherwise wait behind the prefetch in the in-order vmcnt)
    auto acc_to_y = [&](const half_t* bias_p, bool relu, bool sigm) {
#pragma unroll
        for (int nt = 0; nt < 6; nt++) {
            const int col = wn * 96 + nt * 16 + 4 * fq;
            const h4_t bias = *(const h4_t*)(bias_p + col);
#pragma unroll
            for (int mt = 0; mt < 4; mt++) {
                h4_t y;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    half_t v = (half_t)(acc[mt][nt][r] + (float)bias[r]);
                    if (relu) v = v > (half_t)0 ? v : (half_t)0;
                    if (sigm) v = (half_t)fast_sigmoid((float)v);
                    y[r] = v;
                }
                *(h4_t*)(smem + ym.off(wm * 64 + mt * 16 + fr, col * 2)) = y;
            }
        }
    };
    // TRI: LayerNorm (+ ReLU) of the y tile's rows in place, rounded to fp16 --
    // epi2_finish's LN arithmetic (two rows per wave pass, lane s of half h
    // owning columns 4 s + 128 j), the result written back instead of stored
    auto mid_rows = [&](const dpvo_rowgemm_args& pm) {
        if (!TRI) return;
        EpiConsts2 km;
        load_consts2<FMID>(pm, lane, km);
        const int h = lane >> 5, s = lane & 31;
#pragma unroll 1
        for (int i = 0; i < 8; i++) {
            const int r = wave * 16 + 2 * i + h;
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
    // One ping-pong GEMM: stage 0 issued (any mapping) into buffer 0 by the caller.
    auto pp_loop = [&](int nks, auto issue, auto read) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's stage-0 pieces
        bar();
        if (!G0) bar();   // G1: one phase behind
#pragma unroll 1
        for (int ks = 0; ks < nks; ks++) {
            // read phase (G0: during G1's MFMAs of the previous step)
            if (G0 && ks + 1 < nks) issue(ks + 1, (ks + 1) & 1);
            h8_t a[4], b[6];
            read(ks, ks & 1, a, b);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            // (pinned: the scheduler would move MFMAs -- not memory operations --
            // across the barrier, into the read phase)
            __builtin_amdgcn_sched_barrier(0);
            bar();
            __builtin_amdgcn_sched_barrier(0);
            // MFMA phase (G0: during G1's read phase)
            mfma_step(a, b);
            __builtin_amdgcn_sched_barrier(0);
            if (G0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // stage ks+1 landed
            bar();
            __builtin_amdgcn_sched_barrier(0);
        }
        if (G0) bar();   // back in step: every read and MFMA of the loop is done
    };
    auto read1 = [&](int, int buf, h8_t (&a)[4], h8_t (&b)[6]) {
        const char* st = smem + RC_Y + buf * RC_STAGE;
#pragma unroll
        for (int mt = 0; mt < 4; mt++) a[mt] = *(const h8_t*)(st + a_off[mt]);
#pragma unroll
        for (int nt = 0; nt < 6; nt++) b[nt] = *(const h8_t*)(st + w_off[nt]);
    };
    // GEMM1 with the A ring (not the gate pass: the y tile is in use then).
    // Caller: W stage 0 issued by the W waves into buffer 0, nothing of A.
    int ring_off[4];
#pragma unroll
    for (int mt = 0; mt < 4; mt++) {
        const int row = wm * 64 + mt * 16 + fr;
        ring_off[mt] = row * 128 + 16 * (fq ^ ((row >> 1) & 7));   // + 16 * 4 (ks & 1) via the xor below
    }
    auto gemm1_ring = [&]() {
        const int nst = ks1 / 2;   // A stages (K1 % 64 == 0 on this path)
        if (awave) {
#pragma unroll
            for (int st = 0; st < RC_RD; st++)
                if (st < nst) issue_ring(st);
        }
#pragma unroll 1
        for (int ks = 0; ks < ks1; ks++) {
            if (!awave) {
                if (ks + 1 < ks1) {
                    issue_wonly(ks + 1, (ks + 1) & 1);
                    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            } else if ((ks & 1) == 0) {
                // A stage ks/2 landed: the stages issued after it may fly (4 pieces each)
                const int st = ks >> 1, after = min(RC_RD - 1, nst - 1 - st);
                if (after >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
                else if (after == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                // the slot of stage st + RC_RD held stage st - 2 (RC_RN = RC_RD + 2),
                // read by every wave before the previous step's barriers
                if (st + RC_RD < nst) issue_ring(st + RC_RD);
            }
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const char* sa = smem + ((ks >> 1) % RC_RN) * 16384;
            const char* st = smem + RC_Y + (ks & 1) * RC_STAGE;
            const int sub = (ks & 1) * 64;   // logical chunks 4 (ks & 1) + fq: xor-ing 4 flips bit 2 only
            h8_t a[4], b[6];
#pragma unroll
            for (int mt = 0; mt < 4; mt++) a[mt] = *(const h8_t*)(sa + (ring_off[mt] ^ sub));
#pragma unroll
            for (int nt = 0; nt < 6; nt++) b[nt] = *(const h8_t*)(st + w_off[nt]);
            mfma_step(a, b);
            __builtin_amdgcn_s_barrier();
        }
    };
    // DEEP (DPVO_RC_DBG=2048): GEMM1 with four stages in flight instead of one.
    // The y tile is free until GEMM1's result goes there, so it holds three
    // more 32 KB stage slots beside the two stage buffers: slot s at
    // RC_Y + s RC_STAGE (s < 2) or (s - 2) RC_STAGE.  Stage 0 is in slot 0
    // (issued under the previous tile's epilogue); stage ks + 5 is issued into
    // the slot of stage ks once every wave has passed step ks's trailing barrier.
    constexpr bool DEEP = (DBG & 2048) != 0;
    constexpr int DS = 5, DD = DS - 1;
    auto slot1 = [](int sl) { return sl < 2 ? RC_Y + sl * RC_STAGE : (sl - 2) * RC_STAGE; };
    auto issue1o = [&](int ks, int off) {
        char* st = smem + off;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const bool wp = 4 * wave + j >= 8;
            const int64_t k0 = wp ? (int64_t)wrot(ks, ks1) * (RG_BN * RC_BK) : ks * RC_BK;
            glds16(g1src[j] + k0, st + (4 * wave + j) * 1024);
        }
    };
    auto gemm1_deep = [&]() {
#pragma unroll
        for (int s2 = 1; s2 <= DD; s2++)
            if (s2 < ks1) issue1o(s2, slot1(s2));
#pragma unroll 1
        for (int ks = 0; ks < ks1; ks++) {
            // stages ks+1 .. min(ks+DD, ks1-1) may stay in flight, 4 loads each
            const int ahead = min(DD, ks1 - 1 - ks);
            if (ahead >= 4) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            else if (ahead == 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else if (ahead == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const char* st = smem + slot1(ks % DS);
            h8_t a[4], b[6];
#pragma unroll
            for (int mt = 0; mt < 4; mt++) a[mt] = *(const h8_t*)(st + a_off[mt]);
#pragma unroll
            for (int nt = 0; nt < 6; nt++) b[nt] = *(const h8_t*)(st + w_off[nt]);
            mfma_step(a, b);
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (ks + DS < ks1) issue1o(ks + DS, slot1(ks % DS));
        }
    };
    auto gemm1 = [&](bool gate) {
        if (PP) {
            pp_loop(ks1, [&](int ks, int buf) { issue1_pp(ks, buf, gate); }, read1);
            return;
        }
        for (int ks = 0; ks < ks1; ks++) {
            if (ks + 1 < ks1) {
                issue1(ks + 1, (ks + 1) & 1, gate);
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const char* st = smem + RC_Y + (ks & 1) * RC_STAGE;
            h8_t a[4], b[6];
#pragma unroll
            for (int mt = 0; mt < 4; mt++) a[mt] = *(const h8_t*)(st + a_off[mt]);
#pragma unroll
            for (int nt = 0; nt < 6; nt++) b[nt] = *(const h8_t*)(st + w_off[nt]);
            mfma_step(a, b);
            __builtin_amdgcn_s_barrier();
        }
    };
    int64_t tile = blockIdx.x;
    if (RING) {
        set_ring_tile(tile);
        if (GATED) set_tile(tile);   // the gate pass streams A through the stages
        if (!awave) issue_wonly(0, 0);
    } else {
        set_tile(tile);
        set_tile_pp(tile);
        issue1(0, 0);
    }
    for (; tile < ntiles; tile += gridDim.x) {
        const bool more = tile + gridDim.x < ntiles;
        // ---- GEMM1: A (global, gathered) x W1
        zero_acc();
        if (RING) gemm1_ring();
        else if (DEEP) gemm1_deep();
        else gemm1(false);
        // ---- intermediate -> y tile; W2's first stage into the released stage 0
        acc_to_y((const half_t*)p1.bias, p1.flags & RG_RELU, p1.flags & RG_SIGMOID);
        issue2(0, 0);
        sync_lds();
        // ---- GEMM2: y tile x W2 (stage 0 already issued); wdelta selects W3
        auto gemm_y = [&](int64_t wdelta) {
            zero_acc();
            if (PP) {
                pp_loop(
                    ks2, [&](int ks, int buf) { issue2_pp(ks, buf, wdelta); },
                    [&](int ks, int buf, h8_t (&a)[4], h8_t (&b)[6]) {
                        const char* st = smem + RC_Y + buf * RC_STAGE;
#pragma unroll
                        for (int mt = 0; mt < 4; mt++)
                            a[mt] = *(const h8_t*)(smem + ym.off(wm * 64 + mt * 16 + fr, (ks * 4 + fq) * 16));
#pragma unroll
                        for (int nt = 0; nt < 6; nt++) b[nt] = *(const h8_t*)(st + w_off[nt]);
                    });
                return;
            }
#pragma unroll 1
            for (int ks = 0; ks < ks2; ks++) {
                if (ks + 1 < ks2) {
                    issue2(ks + 1, (ks + 1) & 1, wdelta);
                    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                const char* st = smem + RC_Y + (ks & 1) * RC_STAGE;
                h8_t a[4], b[6];
#pragma unroll
                for (int mt = 0; mt < 4; mt++)
                    a[mt] = *(const h8_t*)(smem + ym.off(wm * 64 + mt * 16 + fr, (ks * 4 + fq) * 16));
#pragma unroll
                for (int nt = 0; nt < 6; nt++) b[nt] = *(const h8_t*)(st + w_off[nt]);
                mfma_step(a, b);
                __builtin_amdgcn_s_barrier();
            }
        };
        gemm_y(0);
        if (TRI) {
            // the middle Linear's output -> its row epilogue (LayerNorm, ReLU) in
            // place on the y tile -> the third GEMM's A operand
            acc_to_y((const half_t*)pg.bias, false, false);
            issue2(0, 0, w3delta);   // stage 0 of W3 loads under the row pass
            sync_lds();
            mid_rows(pg);
            sync_lds();
            gemm_y(w3delta);
        }
        acc_to_y((const half_t*)p.bias, F2 & RG_RELU, F2 & RG_SIGMOID);
        if (GATED) {
            // ---- gate: A x Wg -> sigmoid (rowgemm's SIGMOID rounding) -> y = fp16(gate * y)
            issue1(0, 0, true);
            zero_acc();
            gemm1(true);
#pragma unroll
            for (int nt = 0; nt < 6; nt++) {
                const int col = wn * 96 + nt * 16 + 4 * fq;
                const h4_t bias = *(const h4_t*)((const half_t*)pg.bias + col);
#pragma unroll
                for (int mt = 0; mt < 4; mt++) {
                    h4_t* yp = (h4_t*)(smem + ym.off(wm * 64 + mt * 16 + fr, col * 2));
                    h4_t y = *yp;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const half_t g = (half_t)fast_sigmoid((float)(half_t)(acc[mt][nt][r] + (float)bias[r]));
                        y[r] = (half_t)((float)g * (float)y[r]);
                    }
                    *yp = y;
                }
            }
        }
        // ---- the next tile's first GEMM1 stage loads under this epilogue
        if (more) {
            if (RING) {
                set_ring_tile(tile + gridDim.x);
                if (GATED) set_tile(tile + gridDim.x);
                if (!awave) issue_wonly(0, 0);
            } else {
                set_tile(tile + gridDim.x);
                set_tile_pp(tile + gridDim.x);
                issue1(0, 0);
            }
        }
        sync_lds();
        // LayerNorm / head constants loaded per tile, not held across the GEMMs
        // (the gated chain's gate already holds 48 VGPRs there)
        EpiConsts2 kc;
        load_consts2<F2>(p, lane, kc);
        constexpr int RB = (F2 & (RG_RES | RG_GATE | RG_LN)) ? 4 : 8;
        dpvo_rowgemm_args pd = p;
        if (DBG & 32) pd.out32 = pd.out16 = nullptr;   // timing experiment: no row stores
        constexpr int FE = (DBG & 16) ? (F2 & ~RG_RES) : F2;   // timing experiment: no residual loads
#pragma unroll 1
        for (int q0 = 0; q0 < 16 && !(DBG & 1); q0 += RB)   // one batch live at a time (register budget)
            epilogue_rows2<FE, RB>(pd, Mrows, smem, ym, wave * 16 + q0, tile * RG_BM + wave * 16 + q0, lane, kc);
        sync_lds();
    }
}

// ---------------------------------------------------------------------------
// rowchain_ws: the chains whose first GEMM has K1 = 384 (c1 / c2 and the GRU's
// gated residuals, net.py:80-85, blocks.py:27-30), warp-specialised.
// rowchain_kernel runs the k-loops (latency / address-path bound) and the row
// epilogue (HBM bound: the residual in, out32 / out16 out) one after the
// other in the same waves -- measured on the c1 chain: 80 us of k-loop and
// 67 us of epilogue, in series -- and its next tile's first stage load waits
// behind the epilogue's stores (one in-order vmcnt per wave).  Here a
// 512-thread workgroup (one per CU) has two roles:
//   G, waves 0-3: the GEMMs of tile t (64 rows x 384; wave w owns columns
//     96 w .. + 96, acc 4 x 6 MFMA tiles) and every LDS-DMA;
//   E, waves 4-7: the row epilogue of tile t-1 (16 rows each), whose fp16
//     y rows they copied from LDS into registers when tile t began.
// Both roles pass the same barriers; E's loads and stores never enter G's
// vmcnt.
// LDS (144 KB): two 48 KB tiles T0 / T1 (YMapG layout: [3 column groups of
// 256 B][64 rows][256 B], 16-byte chunks XOR (row & 15)) and two 24 KB W
// stages (all 384 output rows x 32 k of the k-blocked W).  Tile t uses
// T[t & 1]: its A rows (gathered as whole 128-B lines during tile t-1, one
// piece per k-step), then GEMM1's activation (GEMM2's A), then GEMM2's
// output, which E copies out at the start of tile t+1.
// Per output element the MFMAs, their k order and the epilogue arithmetic are
// rowchain_kernel's: bit-identical results.
// GATED: the gate GEMM runs first on A; gate = fp16(sigmoid(fp16(A Wg^T +
// bg))) waits in G's registers and multiplies GEMM2's fp16 output as
// rowchain_kernel's gate pass does.
// ---------------------------------------------------------------------------
constexpr int WS_BM = 64, WS_THREADS = 512;
constexpr int WS_T = WS_BM * 768;                  // 48 KB
constexpr int WS_WST = RG_BN * RC_BK * 2;          // 24 KB
constexpr int WS_LDS = 2 * WS_T + 2 * WS_WST + 64; // 144 KB + the sync counters

struct YMapG {   // [byte / 256][64 rows][256 B], 16-byte chunks XOR (row & 15): conflict-free
    // fragment reads down 16 rows, C-layout writes and 256-byte row sweeps
    __device__ int off(int r, int byte) const
    {
        return (byte >> 8) * (WS_BM * 256) + r * 256 + ((((byte >> 4) & 15) ^ (r & 15)) << 4) + (byte & 15);
    }
};

// DBG (timing experiments, DPVO_RCWS_DBG, flag RES; results wrong): 2 no A loads
// after the first tile, 4 no W stream, 8 no E work
template <int F2, bool GATED, int DBG = 0>
__global__ __launch_bounds__(WS_THREADS, 1) void rowchain_ws_kernel(dpvo_rowgemm_args p1, dpvo_rowgemm_args p,
                                                                    dpvo_rowgemm_args pg)
{
    __shared__ __attribute__((aligned(16))) char smem[WS_LDS];
    typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t Mrows = p1.M_dev ? min(*p1.M_dev, p1.M) : p1.M;
    const int64_t ntiles = (Mrows + WS_BM - 1) / WS_BM;
    if ((int64_t)blockIdx.x >= ntiles) return;
    const int nmine = (int)((ntiles - 1 - blockIdx.x) / gridDim.x + 1);
    const YMapG ym;
    // the tile's GEMM k-steps (12 per GEMM); GEMM1 ends at G1END
    constexpr int NS = GATED ? 36 : 24;
    constexpr int G1END = GATED ? 23 : 11;
    // ---- synchronisation: counters in LDS, no workgroup barrier after the
    // first (a barrier would tie the roles' paces together).  Every counter
    // only grows; a waiter spins (s_sleep) until it reaches its target.
    //   ctr[0]  G step counter: a G wave adds 1 when its pieces of the current
    //           W stage have landed and its reads of the previous stage are done
    //   ctr[1]  y ready: a G wave adds 1 after writing its part of a tile's y
    //   ctr[2]  T free: an E wave adds 1 after copying its rows of a tile's y
    //   ctr[3]  abort: a spin that timed out (the kernel then drains and exits;
    //           results are wrong but no wave hangs)
    // (the counter accesses are inline asm with their own lgkmcnt waits: as
    // atomics the compiler would add vmcnt(0) waits, draining the LDS-DMA that
    // is meant to stay in flight)
    const unsigned cbase = (unsigned)(uintptr_t)(smem + WS_LDS - 64);
    if (tid < 4) ((int*)(smem + WS_LDS - 64))[tid] = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    auto add = [&](int i) {
        // this wave's LDS writes (and reads) first; one lane adds
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) asm volatile("ds_add_u32 %0, %1" ::"v"(cbase + 4 * i), "v"(1) : "memory");
    };
    auto ld = [&](int i) {
        int v;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(cbase + 4 * i) : "memory");
        return __builtin_amdgcn_readfirstlane(v);
    };
    auto wait = [&](int i, int target) {
        for (int n = 0;; n++) {
            if (ld(i) >= target || ld(3)) break;
            if (n > (1 << 22)) {   // ~0.2 s: give up (wrong results, no hang)
                add(3);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        asm volatile("" ::: "memory");
    };

    if (wave < 4) {
        // =========================== G role ===========================
        const int wn = wave;
        const int fr = lane & 15, fq = lane >> 4;
        const half_t* __restrict__ zero = (const half_t*)p1.zero_row;
        const half_t* W1 = (const half_t*)p1.W;
        const half_t* W2 = (const half_t*)p.W;
        const half_t* Wg = (const half_t*)pg.W;
        // W stage pieces 6 wave .. 6 wave + 5 of 24 (16 rows x 64 B each); the
        // swizzle ((n >> 2) & 3) does not depend on the piece: one base offset
        const int wsrc0 = [&] {
            const int srow = lane >> 2, pch = lane & 3, n = 96 * wave + srow;
            return n * RC_BK + 8 * (pch ^ ((n >> 2) & 3));
        }();
        // the W of step s (0 .. NS-1) of a tile: gate (GATED), W1, W2
        auto wmat = [&](int s) {
            const int g = s / 12;
            if (GATED) return g == 0 ? Wg : (g == 1 ? W1 : W2);
            return g == 0 ? W1 : W2;
        };
        auto issue_w = [&](int s, int buf) {
            if (DBG & 4) return;
            const half_t* base = wmat(s) + (int64_t)(s % 12) * (RG_BN * RC_BK);
            char* st = smem + 2 * WS_T + buf * WS_WST;
#pragma unroll
            for (int j = 0; j < 6; j++) glds16(base + wsrc0 + 512 * j, st + (6 * wave + j) * 1024);
        };
        // A rows of a tile into T[b]: piece (g, k) = rows 4 wave + 16 k .. + 3 of
        // column group g; lane L: row 4 wave + 16 k + L / 16, chunk L % 16
        int64_t arow[4];   // element offsets of this lane's four A rows (-1: zero row)
        auto load_rows = [&](int64_t tile) {
            const int r0 = 4 * wave + (lane >> 4);
            int64_t sidx[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int64_t m = tile * WS_BM + r0 + 16 * k;
                sidx[k] = m < Mrows ? m : Mrows - 1;
            }
            if (p1.a_idx) {   // all four loads before any use
#pragma unroll
                for (int k = 0; k < 4; k++) sidx[k] = p1.a_idx[sidx[k]];
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const bool ok = tile * WS_BM + r0 + 16 * k < Mrows && sidx[k] >= 0 && sidx[k] < p1.a_rows;
                arow[k] = ok ? sidx[k] * p1.lda : -1;
            }
        };
        auto issue_a = [&](int q, int b) {   // piece q = 4 g + k of this wave
            const int g = q >> 2, k = q & 3;
            const int r = 4 * wave + 16 * k + (lane >> 4);
            const half_t* row = arow[k] >= 0 ? (const half_t*)p1.A + arow[k] : zero;
            glds16(row + 128 * g + 8 * ((lane & 15) ^ (r & 15)),
                   smem + b * WS_T + g * (WS_BM * 256) + (r - (lane >> 4)) * 256);
        };
        // W fragment nt of this wave: row n = 96 wn + 16 nt + fr (the swizzle
        // ((n >> 2) & 3) is fr's)
        const int w_off0 = (wn * 96 + fr) * 64 + 16 * (fq ^ ((fr >> 2) & 3));
        f4_t acc[4][6];
        h4_t gsv[4][6];
        auto zero_acc = [&]() {
#pragma unroll
            for (int mt = 0; mt < 4; mt++)
#pragma unroll
                for (int nt = 0; nt < 6; nt++) acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
        };
        // acc + bias -> act -> fp16 (-> x gate) -> T[b]
        auto acc_to_t = [&](int b, const half_t* bias_p, bool relu, bool sigm, bool gated) {
#pragma unroll
            for (int nt = 0; nt < 6; nt++) {
                const int col = wn * 96 + nt * 16 + 4 * fq;
                const h4_t bias = *(const h4_t*)(bias_p + col);
#pragma unroll
                for (int mt = 0; mt < 4; mt++) {
                    h4_t y;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        half_t v = (half_t)(acc[mt][nt][r] + (float)bias[r]);
                        if (relu) v = v > (half_t)0 ? v : (half_t)0;
                        if (sigm) v = (half_t)fast_sigmoid((float)v);
                        if (GATED && gated) v = (half_t)((float)gsv[mt][nt][r] * (float)v);
                        y[r] = v;
                    }
                    *(h4_t*)(smem + b * WS_T + ym.off(mt * 16 + fr, col * 2)) = y;
                }
            }
        };
        int gsync = 0;   // G-sync rounds passed
        auto gbar = [&]() {
            add(0);
            wait(0, 4 * ++gsync);
        };

        // Software-pipelined k-loop (one G wave per SIMD: nothing else hides
        // the LDS reads): step g starts with stage g's fragments in registers
        // and stage g+1's DMA in flight; it waits for that DMA, syncs the G
        // waves once (stage g+1 landed everywhere, stage g read everywhere),
        // issues stage g+2's DMA into stage g's buffer, and reads stage g+1's
        // fragments between its MFMAs (each W fragment right after the four
        // MFMAs that used it).  Tiles chain: the flat step sequence runs over
        // this workgroup's tiles.
        h8_t acur[4], anxt[4], b[6];
        auto read_a = [&](const char* Tb, int ks, h8_t (&a)[4]) {
#pragma unroll
            for (int mt = 0; mt < 4; mt++) a[mt] = *(const h8_t*)(Tb + ym.off(mt * 16 + fr, (ks * 4 + fq) * 16));
        };
        auto read_b = [&](int buf, int nt) { return *(const h8_t*)(smem + 2 * WS_T + buf * WS_WST + w_off0 + 1024 * nt); };
        load_rows(blockIdx.x);
#pragma unroll
        for (int q = 0; q < 12; q++) issue_a(q, 0);
        issue_w(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        gbar();
        issue_w(1 % NS, 1);   // (NS > 1)
        read_a(smem, 0, acur);
#pragma unroll
        for (int nt = 0; nt < 6; nt++) b[nt] = read_b(0, nt);
        for (int it = 0; it < nmine; it++) {
            const int64_t tile = blockIdx.x + (int64_t)it * gridDim.x;
            const bool next = it + 1 < nmine;
            const int cur = it & 1;
            const char* T = smem + cur * WS_T;
            if (next) load_rows(tile + gridDim.x);   // (plain loads: waited for at their first use)
            zero_acc();
#pragma unroll 1
            for (int s = 0; s < NS; s++) {
                const bool more = s + 1 < NS || next;   // a stage g+1 exists
                // stage g's fragments in registers before the sync (the uses tell
                // the compiler, which then adds no wait covering later reads)
#pragma unroll
                for (int nt = 0; nt < 6; nt++) asm volatile("" ::"v"(b[nt]));
#pragma unroll
                for (int mt = 0; mt < 4; mt++) asm volatile("" ::"v"(acur[mt]));
                if (more) {
                    // stage g+1 landed (the newest A piece of the previous step may fly)
                    const bool aprev = next && s >= 2 && s <= 13 && !(DBG & 2);
                    if (aprev) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    gbar();
                    // stage g+2 into stage g's buffer; one piece of the next tile's
                    // A rows on steps 1 .. 12 (into T[cur ^ 1], which E has copied
                    // tile it-1's y out of)
                    if (s + 2 < NS || next) issue_w((s + 2) % NS, s & 1);
                    if (next && s >= 1 && s <= 12 && !(DBG & 2)) {
                        if (s == 1) wait(2, 4 * it);
                        issue_a(s - 1, cur ^ 1);
                    }
                }
                // stage g+1's fragments (read unconditionally: past the last stage,
                // or at the GEMM1 -> GEMM2 boundary where GEMM1's output is not in
                // T yet, they are harmless in-range reads, replaced below)
                read_a(s + 1 < NS ? T : smem + (cur ^ 1) * WS_T, (s + 1) % 12, anxt);
#pragma unroll
                for (int nt = 0; nt < 6; nt++) {
#pragma unroll
                    for (int mt = 0; mt < 4; mt++)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[nt], acur[mt], acc[mt][nt], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                    b[nt] = read_b((s + 1) & 1, nt);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (GATED && s == 11) {   // gate -> registers
#pragma unroll
                    for (int nt = 0; nt < 6; nt++) {
                        const h4_t bias = *(const h4_t*)((const half_t*)pg.bias + wn * 96 + nt * 16 + 4 * fq);
#pragma unroll
                        for (int mt = 0; mt < 4; mt++)
#pragma unroll
                            for (int r = 0; r < 4; r++)
                                gsv[mt][nt][r] = (half_t)fast_sigmoid((float)(half_t)(acc[mt][nt][r] + (float)bias[r]));
                    }
                    zero_acc();
                } else if (s == G1END) {   // GEMM1's activation -> T once every G wave is done reading A
                    gbar();
                    acc_to_t(cur, (const half_t*)p1.bias, p1.flags & RG_RELU, p1.flags & RG_SIGMOID, false);
                    zero_acc();
                    gbar();
                    read_a(T, 0, anxt);
                } else if (s == NS - 1) {  // GEMM2's output (x gate) -> T, then E may take it
                    gbar();
                    acc_to_t(cur, (const half_t*)p.bias, F2 & RG_RELU, F2 & RG_SIGMOID, true);
                    add(1);
                }
#pragma unroll
                for (int mt = 0; mt < 4; mt++) acur[mt] = anxt[mt];
            }
        }
    } else {
        // =========================== E role ===========================
        const int e = wave - 4;   // rows 16 e .. 16 e + 15 of a tile
        const int hh = lane >> 5, sl = lane & 31;
        ep_h4 yr[8][3];   // pair i: row 16 e + 2 i + hh, columns 128 j + 4 sl ..
        EpiConsts2 kc;
        load_consts2<F2>(p, lane, kc);
        for (int it = 0; it < nmine; it++) {
            const int64_t row0 = (blockIdx.x + (int64_t)it * gridDim.x) * WS_BM + 16 * e;
            wait(1, 4 * (it + 1));   // tile it's y is in T[it & 1]
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int j = 0; j < 3; j++)
                    yr[i][j] = *(const ep_h4*)(smem + (it & 1) * WS_T + ym.off(16 * e + 2 * i + hh, (128 * j + 4 * sl) * 2));
            add(2);   // (add waits for the reads)
            if (DBG & 8) continue;
            // the rows: pair i + 1's loads in flight while pair i finishes
            EpiOps2<2> ops[2];
            epi2_load<F2, 2>(p, Mrows, row0, lane, ops[0]);
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (i + 1 < 8) epi2_load<F2, 2>(p, Mrows, row0 + 2 * (i + 1), lane, ops[(i + 1) & 1]);
                epi2_finish<F2, 2>(
                    p, Mrows, [&](int, int j) { return yr[i][j]; }, row0 + 2 * i, lane, kc, ops[i & 1]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// v4: one GEMM, or two chained (CHAIN), per 128-row tile, with the operand
// streams decoupled from the MFMA waves.  v1-v3 stage W through LDS next to A
// and synchronise all eight waves twice per k-step: every k-step then pays one
// load latency (one stage in flight) and the waves' LDS reads and MFMAs run in
// lockstep instead of overlapping.  Here
//   - W never touches LDS: wave w owns output columns [48 w, 48 w + 48) and
//     loads its own W fragments (3 x 16 B per lane per 32-wide k-step) straight
//     into a 4-step register ring (W is L2-resident: 295 KB per layer);
//   - A (the HBM stream, rows gathered through a_idx) goes global -> LDS by
//     LDS-DMA into an 8-stage ring (8 KB per 32-wide stage), issued 3 groups of
//     2 stages ahead, one barrier per group;
//   - the 128 x 384 fp16 y tile (96 KB) holds GEMM1's activation (GEMM2's A
//     operand) and the final y for the row epilogue (epilogue_rows, as v1-v3).
// The flat sequence of (tile, k-step) runs persistently per workgroup, so the
// next tile's first A stages and W fragments load under this tile's epilogue.
// LDS: 96 KB + 64 KB = 160 KB (one workgroup, 8 waves, per CU).
// ---------------------------------------------------------------------------
constexpr int R4_BK = 32, R4_NS = 8, R4_G = 2, R4_AD = 3, R4_WD = 4;
constexpr int R4_A_STAGE = RG_BM * R4_BK * 2;        // 8 KB
constexpr int R4_Y = RG_BM * 768;                    // 96 KB
constexpr int R4_LDS = R4_Y + R4_NS * R4_A_STAGE;    // 160 KB
static_assert(R4_NS == (R4_AD + 1) * R4_G, "A ring = the groups in flight + the one being read");

// DBG (timing experiments only, DPVO_RG4_DBG): 1 no epilogue, 2 no MFMA, 4 no A loads, 8 no W loads,
// 16 no row pass (acc -> y tile only)
template <int F2, bool CHAIN, int DBG = 0>
__global__ __launch_bounds__(RG_THREADS, 1) void rowgemm4_kernel(dpvo_rowgemm_args p1, dpvo_rowgemm_args p)
{
    __shared__ __attribute__((aligned(16))) char smem[R4_LDS];
    typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int K1 = p1.K;
    const int S1 = K1 / R4_BK, S2 = CHAIN ? RG_BN / R4_BK : 0, S = S1 + S2;
    const int GPT = S / R4_G;   // groups per tile
    const int64_t Mrows = p1.M_dev ? min(*p1.M_dev, p1.M) : p1.M;
    const int64_t ntiles = (Mrows + RG_BM - 1) / RG_BM;
    if ((int64_t)blockIdx.x >= ntiles) return;
    const int64_t my_tiles = (ntiles - 1 - blockIdx.x) / gridDim.x + 1;
    const int64_t total_groups = my_tiles * GPT;
    const YMapChunk ym;

    // ---- W fragment streams: lane (fr, fq) of n-tile nt reads W row 48 w + 16 nt + fr, k 8 fq .. + 8
    const half_t* w1b[3];
    const half_t* w2b[3];
#pragma unroll
    for (int nt = 0; nt < 3; nt++) {
        const int n = 48 * wave + 16 * nt + fr;
        w1b[nt] = (const half_t*)p1.W + (int64_t)n * K1 + 8 * fq;
        w2b[nt] = CHAIN ? (const half_t*)p.W + (int64_t)n * RG_BN + 8 * fq : w1b[nt];
    }
    const __amdgpu_buffer_rsrc_t nothing = __builtin_amdgcn_make_buffer_rsrc((void*)p1.bias, (short)0, 0, 0x00020000);
    h8_t wr[R4_WD][3];
    int wstep = 0;   // k-step (0 .. S-1) of the next W fetch, periodic: W does not depend on the tile
    // W loads are issued by inline asm and waited for with counted vmcnt: the
    // compiler's own wait placement goes conservative (vmcnt(0)) across the
    // persistent loop's branches and would drain the ring every group.  Every
    // k-step issues exactly 3 of them and every group start exactly 2 A-stream
    // operations, so a fixed count covers the steady state (see step / group).
    auto fetch_w = [&](h8_t (&dst)[3]) __attribute__((always_inline)) {
        const bool g1 = wstep < S1;
        const int k0 = R4_BK * (g1 ? wstep : wstep - S1);
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
            if (DBG & 8)
                __builtin_amdgcn_raw_buffer_store_b32(0, nothing, 0, 0, 0);
            else
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst[nt]) : "v"((g1 ? w1b[nt] : w2b[nt]) + k0));
        }
        wstep = wstep + 1 == S ? 0 : wstep + 1;
    };

    // ---- A stream: LDS-DMA of 32-wide k-stages; wave w fills rows 16 w .. 16 w + 15
    // (lane L: row 16 w + L / 4, 16-byte chunk L % 4), stage slots in issue order.
    // Every group start issues exactly 3 vm operations -- 2 stage loads or 2
    // dummies, and the next tile's gather index or a dummy -- so the counted
    // waits below hold.  Dummies are stores through a zero-range descriptor:
    // they count in vmcnt, touch no memory and, unlike a dummy load, leave no
    // in-flight write to a register the compiler may have handed to something else.
    const int arow = 16 * wave + (lane >> 2);
    auto dummy_a = [&]() __attribute__((always_inline)) { __builtin_amdgcn_raw_buffer_store_b32(0, nothing, 0, 0, 0); };
    // the next tile's gather index, loaded a whole tile (>= 3 groups) before its
    // use, by asm: a compiler-visible load would get a compiler wait at the use,
    // counted over the compiler's own loads only, i.e. a vmcnt(0) draining
    // every stream once per tile.  The group-start wait covers it.
    int64_t idx_next = 0;
    auto fetch_idx = [&](int64_t t_ord) __attribute__((always_inline)) {
        const int64_t m = (blockIdx.x + t_ord * gridDim.x) * RG_BM + arow;
        if (p1.a_idx && t_ord < my_tiles && m < Mrows)
            asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(idx_next) : "v"(p1.a_idx + m));
        else
            dummy_a();
    };
    auto row_of = [&](int64_t t_ord, int64_t idx) __attribute__((always_inline)) {
        const int64_t m = (blockIdx.x + t_ord * gridDim.x) * RG_BM + arow;
        const half_t* row = (const half_t*)p1.zero_row;
        if (m < Mrows) {
            const int64_t src = p1.a_idx ? idx : m;
            if (src >= 0 && src < p1.a_rows) row = (const half_t*)p1.A + src * p1.lda;
        }
        return row + 8 * (lane & 3);
    };
    const half_t* asrc = nullptr;
    int astage = 0;
    int64_t ai_t = 0;   // tile ordinal (0 .. my_tiles) of the A cursor
    int ac_gs = 0;      // its tile-local group
    // advance the A cursor by one flat group: its stage loads when that group is
    // a GEMM1 group, and on entering a tile the index fetch for the tile after
    auto a_cursor_step = [&]() __attribute__((always_inline)) {
        if (ac_gs < S1 / R4_G && ai_t < my_tiles) {
            if (ac_gs == 0) {
                if (GPT < 3) asm volatile("s_waitcnt vmcnt(0)" : "+v"(idx_next));   // fetched < 3 groups ago
                asrc = row_of(ai_t, idx_next);
            }
#pragma unroll
            for (int st = 0; st < R4_G; st++) {
                const int k0 = R4_BK * (R4_G * ac_gs + st);
                if (DBG & 4)
                    dummy_a();
                else
                    glds16(asrc + k0, smem + R4_Y + (astage % R4_NS) * R4_A_STAGE + wave * 1024);
                astage++;
            }
        } else {
            dummy_a();
            dummy_a();
        }
        if (ac_gs == 0)
            fetch_idx(ai_t + 1);
        else
            dummy_a();
        if (++ac_gs == GPT) {
            ac_gs = 0;
            ai_t++;
        }
    };

    f4_t acc[8][3];
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int mt = 0; mt < 8; mt++)
#pragma unroll
            for (int nt = 0; nt < 3; nt++) acc[mt][nt] = f4_t{0.f, 0.f, 0.f, 0.f};
    };
    // acc + bias -> act -> fp16 -> y tile: lane (fr, fq) holds row 16 mt + fr, columns 48 w + 16 nt + 4 fq + r
    auto acc_to_y = [&](const h4_t (&bias)[3], bool relu, bool sigm) __attribute__((always_inline)) {
#pragma unroll
        for (int nt = 0; nt < 3; nt++) {
            const int col = 48 * wave + 16 * nt + 4 * fq;
#pragma unroll
            for (int mt = 0; mt < 8; mt++) {
                h4_t y;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    half_t v = (half_t)(acc[mt][nt][r] + (float)bias[nt][r]);
                    if (relu) v = v > (half_t)0 ? v : (half_t)0;
                    if (sigm) v = (half_t)fast_sigmoid((float)v);
                    y[r] = v;
                }
                *(h4_t*)(smem + ym.off(16 * mt + fr, col * 2)) = y;
            }
        }
    };
    auto sync_lds = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    // biases preloaded (a load at a GEMM's end would wait for every stream)
    h4_t bias1[3], bias2[3];
#pragma unroll
    for (int nt = 0; nt < 3; nt++) {
        const int col = 48 * wave + 16 * nt + 4 * fq;
        bias1[nt] = *(const h4_t*)((const half_t*)p1.bias + col);
        bias2[nt] = *(const h4_t*)((const half_t*)p.bias + col);
    }

    // ---- one k-step: A fragments (ring stage or y tile) x W fragments of ring slot SL
    int cstage = 0;   // A stages consumed
    auto step = [&](auto SLC, bool g1, int k2) __attribute__((always_inline)) {
        constexpr int SL = decltype(SLC)::value;
        // W(f) was issued R4_WD steps ago; 3 (R4_WD - 1) W loads and two group
        // starts' 3 A-stream operations have been issued since (more around a
        // tile's epilogue, which only makes this wait conservative)
        asm volatile("s_waitcnt vmcnt(15)" : "+v"(wr[SL][0]), "+v"(wr[SL][1]), "+v"(wr[SL][2]));
        h8_t a[8];
        if (g1) {
            const char* st = smem + R4_Y + (cstage % R4_NS) * R4_A_STAGE + fr * 64 + 16 * fq;
#pragma unroll
            for (int mt = 0; mt < 8; mt++) a[mt] = *(const h8_t*)(st + mt * 1024);
            cstage++;
        } else {
#pragma unroll
            for (int mt = 0; mt < 8; mt++) a[mt] = *(const h8_t*)(smem + ym.off(16 * mt + fr, (4 * k2 + fq) * 16));
        }
        if (!(DBG & 2)) {
#pragma unroll
            for (int mt = 0; mt < 8; mt++)
#pragma unroll
                for (int nt = 0; nt < 3; nt++)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[SL][nt], a[mt], acc[mt][nt], 0, 0, 0);
        } else {
#pragma unroll
            for (int mt = 0; mt < 8; mt++) acc[mt][0][0] += (float)a[mt][0] + (float)wr[SL][0][0];
        }
        // the refill goes after the MFMAs that read the slot: hoisted above them it
        // would need fresh registers, and the wait for the slot's old loads would
        // then also wait for the refill just issued
        __builtin_amdgcn_sched_barrier(0);
        fetch_w(wr[SL]);   // this slot's next use is R4_WD steps ahead
        __builtin_amdgcn_sched_barrier(0);
    };

    // prologue: tile 0's gather index, W for steps 0 .. WD-1, A for flat groups 0 .. AD-1
    fetch_idx(0);
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(idx_next));
#pragma unroll
    for (int i = 0; i < R4_WD; i++) fetch_w(wr[i]);
    for (int i = 0; i < R4_AD; i++) a_cursor_step();
    zero_acc();

    int64_t ti = 0;   // tile ordinal of the current group
    int gs = 0;       // tile-local group
    auto group = [&](auto PC, int64_t g) __attribute__((always_inline)) {
        constexpr int P = decltype(PC)::value;
        // this group's A stages were issued R4_AD groups ago; every group since
        // issued 2 x 3 W fetches after them (the prologue is the exception)
        // (lgkmcnt: acc_to_y's y-tile writes are published by this barrier)
        if (g < R4_AD)
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(18) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        a_cursor_step();   // the ring slot it fills was read before this barrier
        const bool g1 = gs < S1 / R4_G;
        const int k2 = R4_G * (gs - S1 / R4_G);
        step(std::integral_constant<int, 2 * P>{}, g1, k2);
        step(std::integral_constant<int, 2 * P + 1>{}, g1, k2 + 1);
        const int64_t tile = blockIdx.x + ti * gridDim.x;
        if (CHAIN && gs == S1 / R4_G - 1) {
            // GEMM1 done: its activation becomes GEMM2's A operand (the next
            // group's barrier publishes it; nothing reads y until then)
            acc_to_y(bias1, p1.flags & RG_RELU, p1.flags & RG_SIGMOID);
            zero_acc();
        }
        if (gs == GPT - 1 && (DBG & 1)) zero_acc();
        if (gs == GPT - 1 && !(DBG & 1)) {
            if (CHAIN) sync_lds();   // every wave's last GEMM2 read of y is done
            acc_to_y(CHAIN ? bias2 : bias1, F2 & RG_RELU, F2 & RG_SIGMOID);
            sync_lds();
            if (!(DBG & 16)) {
            EpiConsts kc;   // loaded here, not held across the k-loop (register budget)
            load_consts<F2>(p, lane, kc);
            // the wave's 16 rows in 4 batches, each batch's residual / gate loads
            // issued one batch ahead (a dependent gather index costs one more trip)
            const int64_t r0 = tile * RG_BM + 16 * __builtin_amdgcn_readfirstlane(wave);
            EpiOps<4> ops[2];
            epi_load<F2, 4>(p, Mrows, r0, lane, ops[0]);
#pragma unroll
            for (int b = 0; b < 4; b++) {
                if (b + 1 < 4) epi_load<F2, 4>(p, Mrows, r0 + 4 * (b + 1), lane, ops[(b + 1) & 1]);
                epi_finish<F2, 4>(p, Mrows, smem, ym, wave * 16 + 4 * b, r0 + 4 * b, lane, kc, ops[b & 1]);
            }
            }
            zero_acc();
        }
        if (++gs == GPT) {
            gs = 0;
            ti++;
        }
    };
    for (int64_t g = 0; g < total_groups; g += 2) {
        group(std::integral_constant<int, 0>{}, g);
        if (g + 1 < total_groups) group(std::integral_constant<int, 1>{}, g + 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // trailing W prefetches
}

// v = a32[row] (+ b16[idx[row]]) -> [LayerNorm] -> out32 / out16
// Half a wave per row: lane l of the half covers columns 4l + 128j (j < 3), so
// every access is a 16-byte (fp32) or 8-byte (fp16) vector and one wave keeps
// two rows' loads in flight.  HBM-bound: 4 B x 384 in, 6 B x 384 out per row.
typedef float rl_f4 __attribute__((ext_vector_type(4)));
typedef half_t rl_h4 __attribute__((ext_vector_type(4)));

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
    for (int64_t row = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 5; row < p.M;
         row += ((int64_t)gridDim.x * blockDim.x) >> 5) {
        float v[12];
        const half_t* b = nullptr;
        const half_t* c2 = nullptr;
        if (p.b16) {
            const int64_t s = p.b_idx ? p.b_idx[row] : row;
            if (s >= 0 && s < p.b_rows) b = (const half_t*)p.b16 + s * RG_BN;
        }
        if (p.c16) {
            const int64_t s = p.c_idx ? p.c_idx[row] : row;
            if (s >= 0 && s < p.c_rows) c2 = (const half_t*)p.c16 + s * RG_BN;
        }
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int c = 128 * j + 4 * sub;
            if (p.a_f16) {
                const rl_h4 h = *(const rl_h4*)((const half_t*)p.a + row * p.lda + c);
#pragma unroll
                for (int t = 0; t < 4; t++) v[4 * j + t] = (float)h[t];
            } else {
                const rl_f4 a = *(const rl_f4*)((const float*)p.a + row * p.lda + c);
#pragma unroll
                for (int t = 0; t < 4; t++) v[4 * j + t] = a[t];
            }
        }
        if (b) {
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const rl_h4 h = *(const rl_h4*)(b + 128 * j + 4 * sub);
#pragma unroll
                for (int t = 0; t < 4; t++) v[4 * j + t] += (float)h[t];
            }
        }
        if (c2) {   // ((a + b) + c: the two row adds of consecutive rowadd_ln calls, in order)
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const rl_h4 h = *(const rl_h4*)(c2 + 128 * j + 4 * sub);
#pragma unroll
                for (int t = 0; t < 4; t++) v[4 * j + t] += (float)h[t];
            }
        }
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

int g_num_cus = 0;

}  // namespace
}  // namespace dpvo

using namespace dpvo;

#define RG_CASE(F)                                                                                   \
    case (F):                                                                                        \
        hipLaunchKernelGGL(rowgemm_kernel<(F)>, dim3(grid), dim3(RG_THREADS), 0, as_stream(stream), *a); \
        break;

static int validate_rowgemm(const dpvo_rowgemm_args* a)
{
    DPVO_CHECK_ARG(a != nullptr, "null args");
    DPVO_CHECK_ARG(a->N == RG_BN, "rowgemm: output width must be 384");
    DPVO_CHECK_ARG(a->K > 0 && a->K % RG_BK == 0, "rowgemm: K must be a positive multiple of 64 (pad W with zeros)");
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
    DPVO_CHECK_ARG(a->flags == 0 && b->flags == 0, "rowgemm_pair: plain GEMMs only (flags 0)");
    DPVO_CHECK_ARG(a->A == b->A && a->lda == b->lda && a->a_idx == b->a_idx && a->a_rows == b->a_rows &&
                       a->K == b->K && a->M == b->M && a->M_dev == b->M_dev,
                   "rowgemm_pair: both GEMMs must share A, K and M");
    if (a->M <= 0) return 0;
    if (ensure_num_cus()) return -1;
    const int64_t ntiles = (a->M + RG_BM - 1) / RG_BM;
    const unsigned grid = (unsigned)std::min<int64_t>(ntiles, g_num_cus);
    hipLaunchKernelGGL((rowgemm3_kernel<0, true>), dim3(grid), dim3(RG_THREADS), 0, as_stream(stream), *a, *b);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_rowgemm(const dpvo_rowgemm_args* a, void* stream)
{
    if (validate_rowgemm(a)) return -1;
    const int f = a->flags;
    if (a->M <= 0) return 0;
    if (g_num_cus == 0) {
        int dev = 0;
        DPVO_CHECK_HIP(hipGetDevice(&dev));
        DPVO_CHECK_HIP(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
        if (g_num_cus <= 0) g_num_cus = 256;
    }
    static const int version = [] {
        // 1: one 128-row workgroup per CU; 2: two 64-row workgroups per CU;
        // 3 (default): v1 tiling, A stream two stages ahead, transposed accumulators;
        // 4: W fragments streamed to registers, 8-stage A ring (rowgemm4_kernel) --
        // measured no faster at C3 (profiles/r2/NOTES.md), kept for the experiment.
        // (Measured and dropped: stage fills through registers instead of LDS-DMA,
        // and v2 + register fills -- neither beat v3 on the C3 update operator.)
        const char* v = getenv("DPVO_ROWGEMM");
        return v ? atoi(v) : 3;
    }();
    if (version == 4) {
        const int64_t ntiles = (a->M + RG_BM - 1) / RG_BM;
        const unsigned grid = (unsigned)std::min<int64_t>(ntiles, g_num_cus);
        const char* dbgs = getenv("DPVO_RG4_DBG");   // read per call: timing experiments switch it in-process
        const int dbg = dbgs ? atoi(dbgs) : 0;
        if (dbg && f == 0) {   // timing experiments (scripts/bench_rg4_dbg.py)
            warn_debug_knob("DPVO_RG4_DBG");
            switch (dbg) {
#define R4D_CASE(D)                                                                                                  \
    case (D):                                                                                                        \
        hipLaunchKernelGGL((rowgemm4_kernel<0, false, (D)>), dim3(grid), dim3(RG_THREADS), 0, as_stream(stream), *a, \
                           *a);                                                                                      \
        break;
                R4D_CASE(1) R4D_CASE(2) R4D_CASE(3) R4D_CASE(4) R4D_CASE(5) R4D_CASE(6) R4D_CASE(8) R4D_CASE(9)
                R4D_CASE(12) R4D_CASE(13) R4D_CASE(14) R4D_CASE(15) R4D_CASE(16) R4D_CASE(22) R4D_CASE(30)
#undef R4D_CASE
            default:
                set_error("DPVO_RG4_DBG: unsupported value");
                return -1;
            }
            DPVO_CHECK_LAUNCH();
            return 0;
        }
        switch (f) {
#define R4_CASE(F)                                                                                                \
    case (F):                                                                                                     \
        hipLaunchKernelGGL((rowgemm4_kernel<(F), false>), dim3(grid), dim3(RG_THREADS), 0, as_stream(stream), *a, \
                           *a);                                                                                   \
        break;
            R4_CASE(0)
            R4_CASE(DPVO_RG_RELU)
            R4_CASE(DPVO_RG_SIGMOID)
            R4_CASE(DPVO_RG_LN | DPVO_RG_LN_RELU)
            R4_CASE(DPVO_RG_RES)
            R4_CASE(DPVO_RG_RES | DPVO_RG_LN)
            R4_CASE(DPVO_RG_GATE | DPVO_RG_LN)
            R4_CASE(DPVO_RG_GATE | DPVO_RG_HEADS)
            R4_CASE(DPVO_RG_GATE)
#undef R4_CASE
        default:
            set_error("dpvo_rowgemm: unsupported epilogue flag combination " + std::to_string(f));
            return -1;
        }
        DPVO_CHECK_LAUNCH();
        return 0;
    }
    if (version == 2) {
        const int64_t nt2 = (a->M + R2_BM - 1) / R2_BM;
        const unsigned grid = (unsigned)std::min<int64_t>(nt2, 2 * (int64_t)g_num_cus);
        switch (f) {
#define R2_CASE(F)                                                                                           \
    case (F):                                                                                                \
        hipLaunchKernelGGL(rowgemm2_kernel<(F)>, dim3(grid), dim3(R2_THREADS), 0, as_stream(stream), *a); \
        break;
            R2_CASE(0)
            R2_CASE(DPVO_RG_RELU)
            R2_CASE(DPVO_RG_SIGMOID)
            R2_CASE(DPVO_RG_LN | DPVO_RG_LN_RELU)
            R2_CASE(DPVO_RG_RES)
            R2_CASE(DPVO_RG_RES | DPVO_RG_LN)
            R2_CASE(DPVO_RG_GATE | DPVO_RG_LN)
            R2_CASE(DPVO_RG_GATE | DPVO_RG_HEADS)
            R2_CASE(DPVO_RG_GATE)
#undef R2_CASE
        default:
            set_error("dpvo_rowgemm: unsupported epilogue flag combination " + std::to_string(f));
            return -1;
        }
        DPVO_CHECK_LAUNCH();
        return 0;
    }
    const int64_t ntiles = (a->M + RG_BM - 1) / RG_BM;
    const unsigned grid = (unsigned)std::min<int64_t>(ntiles, g_num_cus);
    if (version == 3) {
        switch (f) {
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
    switch (f) {
        RG_CASE(0)
        RG_CASE(DPVO_RG_RELU)
        RG_CASE(DPVO_RG_SIGMOID)
        RG_CASE(DPVO_RG_LN | DPVO_RG_LN_RELU)
        RG_CASE(DPVO_RG_RES)
        RG_CASE(DPVO_RG_RES | DPVO_RG_LN)
        RG_CASE(DPVO_RG_GATE | DPVO_RG_LN)
        RG_CASE(DPVO_RG_GATE | DPVO_RG_HEADS)
        RG_CASE(DPVO_RG_GATE)
    default:
        set_error("dpvo_rowgemm: unsupported epilogue flag combination " + std::to_string(f));
        return -1;
    }
    DPVO_CHECK_LAUNCH();
    return 0;
}

static int rowchain_launch(const dpvo_rowgemm_args* g1, const dpvo_rowgemm_args* g2, const dpvo_rowgemm_args* gate,
                           void* stream)
{
    DPVO_CHECK_ARG(g1 != nullptr && g2 != nullptr, "null args");
    DPVO_CHECK_ARG(g1->N == RG_BN && g2->N == RG_BN, "rowchain: output widths must be 384");
    DPVO_CHECK_ARG(g1->K > 0 && g1->K % RC_BK == 0, "rowchain: K1 must be a positive multiple of 32");
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
    if (g_num_cus == 0) {
        int dev = 0;
        DPVO_CHECK_HIP(hipGetDevice(&dev));
        DPVO_CHECK_HIP(hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev));
        if (g_num_cus <= 0) g_num_cus = 256;
    }
    const int64_t ntiles = (g1->M + RG_BM - 1) / RG_BM;
    const unsigned grid = (unsigned)std::min<int64_t>(ntiles, g_num_cus);
    dpvo_rowgemm_args a2 = *g2;
    a2.M = g1->M;
    a2.M_dev = g1->M_dev;
    static const bool v4 = [] {
        const char* v = getenv("DPVO_ROWGEMM");
        return v && atoi(v) == 4;
    }();
    if (v4 && !gate && g1->K % 64 == 0) {
        switch (f) {
#define RC4_CASE(F)                                                                                              \
    case (F):                                                                                                    \
        hipLaunchKernelGGL((rowgemm4_kernel<(F), true>), dim3(grid), dim3(RG_THREADS), 0, as_stream(stream), *g1, \
                           a2);                                                                                  \
        break;
            RC4_CASE(DPVO_RG_LN | DPVO_RG_LN_RELU)
            RC4_CASE(DPVO_RG_RES)
            RC4_CASE(DPVO_RG_GATE | DPVO_RG_LN)
            RC4_CASE(DPVO_RG_GATE | DPVO_RG_HEADS)
#undef RC4_CASE
        default:
            set_error("dpvo_rowchain: unsupported epilogue flag combination " + std::to_string(f));
            return -1;
        }
        DPVO_CHECK_LAUNCH();
        return 0;
    }
    static const bool ws = [] {
        // 1: the warp-specialised 64-row chains (measured slower at C3 so far:
        // profiles/r3/NOTES.md); default: the one-role 128-row chain kernel
        const char* v = getenv("DPVO_RCWS");
        return v && atoi(v) == 1;
    }();
    if (const char* d = getenv("DPVO_RCWS_DBG"); ws && g1->K == RG_BN && d && f == DPVO_RG_RES && !gate) {
        warn_debug_knob("DPVO_RCWS_DBG");
        const unsigned gws = (unsigned)std::min<int64_t>((g1->M + WS_BM - 1) / WS_BM, g_num_cus);
        switch (atoi(d)) {
#define RCWSD_CASE(D)                                                                                       \
    case (D):                                                                                               \
        hipLaunchKernelGGL((rowchain_ws_kernel<DPVO_RG_RES, false, (D)>), dim3(gws), dim3(WS_THREADS), 0,   \
                           as_stream(stream), *g1, a2, a2);                                                 \
        break;
            RCWSD_CASE(0) RCWSD_CASE(2) RCWSD_CASE(4) RCWSD_CASE(6) RCWSD_CASE(8) RCWSD_CASE(14)
#undef RCWSD_CASE
        default:
            set_error("DPVO_RCWS_DBG: unsupported value");
            return -1;
        }
        DPVO_CHECK_LAUNCH();
        return 0;
    }
    if (ws && g1->K == RG_BN) {
        const int64_t ntw = (g1->M + WS_BM - 1) / WS_BM;
        const unsigned gws = (unsigned)std::min<int64_t>(ntw, g_num_cus);
        if (gate) {
            a2.gate16 = nullptr;
            a2.res16 = nullptr;
        }
        switch (f | (gate ? 1024 : 0)) {
#define RCWS_CASE(F)                                                                                              \
    case (F):                                                                                                     \
        hipLaunchKernelGGL((rowchain_ws_kernel<(F), false>), dim3(gws), dim3(WS_THREADS), 0, as_stream(stream), *g1, \
                           a2, a2);                                                                                \
        break;
#define RCWSG_CASE(F)                                                                                              \
    case ((F) | 1024):                                                                                             \
        hipLaunchKernelGGL((rowchain_ws_kernel<((F) & ~DPVO_RG_GATE) | DPVO_RG_RES, true>), dim3(gws),             \
                           dim3(WS_THREADS), 0, as_stream(stream), *g1, a2, *gate);                                \
        break;
            RCWS_CASE(DPVO_RG_LN | DPVO_RG_LN_RELU)
            RCWS_CASE(DPVO_RG_RES)
            RCWS_CASE(DPVO_RG_GATE | DPVO_RG_LN)
            RCWS_CASE(DPVO_RG_GATE | DPVO_RG_HEADS)
            RCWSG_CASE(DPVO_RG_GATE | DPVO_RG_LN)
            RCWSG_CASE(DPVO_RG_GATE | DPVO_RG_HEADS)
#undef RCWS_CASE
#undef RCWSG_CASE
        default:
            set_error("dpvo_rowchain: unsupported epilogue flag combination " + std::to_string(f));
            return -1;
        }
        DPVO_CHECK_LAUNCH();
        return 0;
    }
    if (gate) {
        // the gated y goes through the RES epilogue (res16 none): x + fp16(gate * y)
        a2.gate16 = nullptr;
        a2.res16 = nullptr;
        switch (f) {
#define RCG_CASE(F)                                                                                                   \
    case (F):                                                                                                         \
        hipLaunchKernelGGL((rowchain_kernel<((F) & ~DPVO_RG_GATE) | DPVO_RG_RES, true>), dim3(grid), dim3(RG_THREADS), \
                           0, as_stream(stream), *g1, a2, *gate);                                                     \
        break;
            RCG_CASE(DPVO_RG_GATE | DPVO_RG_LN)
            RCG_CASE(DPVO_RG_GATE | DPVO_RG_HEADS)
#undef RCG_CASE
        default:
            set_error("dpvo_rowchain_gated: unsupported epilogue flag combination " + std::to_string(f));
            return -1;
        }
        DPVO_CHECK_LAUNCH();
        return 0;
    }
    if (const char* dbgs = getenv("DPVO_RC_DBG"); dbgs && f == DPVO_RG_RES && !gate) {   // timing experiments
        if (atoi(dbgs)) warn_debug_knob("DPVO_RC_DBG");
        switch (atoi(dbgs)) {
#define RCD_CASE(D)                                                                                               \
    case (D):                                                                                                     \
        hipLaunchKernelGGL((rowchain_kernel<DPVO_RG_RES, false, (D)>), dim3(grid), dim3(RG_THREADS), 0,            \
                           as_stream(stream), *g1, a2, a2);                                                       \
        break;
            RCD_CASE(0) RCD_CASE(1) RCD_CASE(2) RCD_CASE(3) RCD_CASE(16) RCD_CASE(32) RCD_CASE(48) RCD_CASE(256) RCD_CASE(257) RCD_CASE(512) RCD_CASE(513) RCD_CASE(1024) RCD_CASE(1025) RCD_CASE(2048) RCD_CASE(2049)
#undef RCD_CASE
        default:
            set_error("DPVO_RC_DBG: unsupported value");
            return -1;
        }
        DPVO_CHECK_LAUNCH();
        return 0;
    }
    switch (f) {
#define RCH_CASE(F)                                                                                                   \
    case (F):                                                                                                         \
        hipLaunchKernelGGL(rowchain_kernel<(F)>, dim3(grid), dim3(RG_THREADS), 0, as_stream(stream), *g1, a2, a2); \
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
    DPVO_CHECK_ARG(g1->K > 0 && g1->K % RC_BK == 0, "rowchain3: K1 must be a positive multiple of 32");
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
    const unsigned grid = (unsigned)std::min<int64_t>(ntiles, g_num_cus);
    dpvo_rowgemm_args a3 = *g3;
    a3.M = g1->M;
    a3.M_dev = g1->M_dev;
    hipLaunchKernelGGL((rowchain_kernel<DPVO_RG_RES | DPVO_RG_LN, false, 0, DPVO_RG_LN | DPVO_RG_LN_RELU>), dim3(grid),
                       dim3(RG_THREADS), 0, as_stream(stream), *g1, a3, *g2);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_rowchain_gated(const dpvo_rowgemm_args* gate, const dpvo_rowgemm_args* g1,
                                   const dpvo_rowgemm_args* g2, void* stream)
{
    DPVO_CHECK_ARG(gate != nullptr, "rowchain_gated: gate args missing");
    return rowchain_launch(g1, g2, gate, stream);
}

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
    hipLaunchKernelGGL(rowadd_ln_kernel, dim3(grid), dim3(256), 0, as_stream(stream), *a);
    DPVO_CHECK_LAUNCH();
    return 0;
}

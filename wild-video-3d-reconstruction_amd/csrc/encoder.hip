// encoder.hip -- the Patchifier's two BasicEncoder4 networks (reference
// dpvo/extractor.py:200-264, ResidualBlock :6-53; called twice per frame from
// dpvo/net.py:121-122) as 11 MFMA launches per frame instead of ~100
// MIOpen / elementwise launches.
//
// Design (gfx950):
//  * Activations are fp16 NHWC (channel-last): one pixel's 32 / 64 channels are
//    64 / 128 contiguous bytes, the 16-byte MFMA operand is 8 channels.
//  * Every convolution is an implicit GEMM on v_mfma_f32_16x16x32_f16: the
//    weights are the first operand (16 output channels), 16 output pixels of
//    one tile row the second; K runs over (tap, 32 input channels).  A 256-thread
//    workgroup owns an 8 x 16 output tile: its input halo (normalised on load)
//    and the layer's whole weight tensor sit in LDS, each wave computes two
//    tile rows x all output channels.
//  * Nothing between two convolutions is a separate pass.  Instance norm,
//    ReLU and the residual add of a ResidualBlock are applied when the NEXT
//    convolution loads its input (x = relu(relu(IN(y)) + res)); the convolution
//    that first reads a block output also writes it (the residual of the next
//    block).  Instance-norm statistics: each producing workgroup writes its
//    tile's per-channel (sum, sum of squares); every consuming workgroup
//    reduces all tiles' partials itself, in one fixed order (fp64), while its
//    weight DMA is in flight.  No cross-workgroup synchronisation, no extra
//    launch, identical (rstd, -mean rstd) in every workgroup, deterministic.
//    (A last-workgroup-reduces scheme measured 19 us more per layer: the
//    device-scope counter and release fences serialise the 768 workgroups.)
//  * Both encoders run in the same launches (blockIdx.y = encoder: fnet with
//    instance norm, inet with none), so every launch has twice the workgroups.
//  * The inet's final 1x1 convolution (64 -> 384) is evaluated only at the
//    patch centres the Patchifier gathers (net.py:301-303: imap is sampled at
//    integer centres with radius 0), not over the whole map.
// Rounding follows the reference under fp16 autocast: conv outputs rounded to
// fp16, the normalised value rounded to fp16, the residual sum rounded to fp16.
#include "common.hpp"

namespace dpvo {
namespace {

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
typedef float f4_t __attribute__((ext_vector_type(4)));

constexpr int EN_TH = 8, EN_TW = 16, EN_THREADS = 256;

struct EncBatch {
    dpvo_conv_args e[2];
    int Hi, Wi, Ho, Wo, tiles_x, ntiles;
};

__device__ __forceinline__ h8_t load_h8(const half_t* p) { return *(const h8_t*)p; }

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;
// global -> LDS DMA: lane l's 16 bytes land at lds_base + 16 l
__device__ __forceinline__ void wlds16(const void* src, char* lds_base)
{
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_base, 16, 0, 0);
}
// weight row r (32 K halves, 64 B) in LDS: its four 16-byte chunks are stored
// XOR-swizzled by (r >> 2) & 3 (encoder_ops.pack_conv does the swizzle), so
// the 16 rows of an MFMA operand read hit 16 distinct bank groups
__device__ __forceinline__ int wrow(int r, int chunk) { return r * 32 + 8 * (chunk ^ ((r >> 2) & 3)); }

// x = relu(IN(a)) [+ res, relu]  for 8 channels (XMODE 1 / 2); XMODE 0: x = a
template <int XMODE>
__device__ __forceinline__ h8_t xform(h8_t a, const float (&as)[16], bool a_norm, h8_t r, const float (&rs)[16],
                                      bool r_norm)
{
    if (XMODE == 0) return a;
    h8_t o;
#pragma unroll
    for (int c = 0; c < 8; c++) {
        half_t n = a_norm ? (half_t)((float)a[c] * as[2 * c] + as[2 * c + 1]) : a[c];
        n = n > (half_t)0 ? n : (half_t)0;
        if (XMODE == 2) {
            const half_t rr = r_norm ? (half_t)((float)r[c] * rs[2 * c] + rs[2 * c + 1]) : r[c];
            n = (half_t)((float)n + (float)rr);
            n = n > (half_t)0 ? n : (half_t)0;
        }
        o[c] = n;
    }
    return o;
}

// acc (+ bias) -> fp16 -> out; instance-norm partial sums of the stored
// values -> part[tile] (sum, sumsq interleaved per channel).
template <int COUT>
__device__ void conv_epilogue(const dpvo_conv_args& e, f4_t (&acc)[2][COUT / 16], int Ho, int Wo, int oy0, int ox0,
                              int tile, float (*sred)[2 * COUT])
{
    constexpr int NT = COUT / 16;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fq = lane >> 4;
    const bool stats = e.part != nullptr;
    const half_t* bias = (const half_t*)e.bias;
    half_t* out = (half_t*)e.out;
    float ssum[NT][4], ssq[NT][4];
#pragma unroll
    for (int mt = 0; mt < NT; mt++)
#pragma unroll
        for (int r = 0; r < 4; r++) ssum[mt][r] = ssq[mt][r] = 0.f;
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const int oy = oy0 + 2 * wave + i, ox = ox0 + (lane & 15);
        const bool valid = oy < Ho && ox < Wo;
        half_t* op = out + ((int64_t)oy * Wo + ox) * e.o_ps + e.o_co;
#pragma unroll
        for (int mt = 0; mt < NT; mt++) {
            const int co = mt * 16 + 4 * fq;
            const h4_t b = *(const h4_t*)(bias + co);
            h4_t v;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                half_t h = (half_t)(acc[i][mt][r] + (float)b[r]);
                if (e.out_scale != 1.f) h = (half_t)((float)h * e.out_scale);
                v[r] = h;
                const float s = valid ? (float)h : 0.f;
                ssum[mt][r] += s;
                ssq[mt][r] += s * s;
            }
            if (valid) *(h4_t*)(op + co) = v;
        }
    }
    if (!stats) return;
#pragma unroll
    for (int mt = 0; mt < NT; mt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const float s = row16_sum(ssum[mt][r]), q = row16_sum(ssq[mt][r]);
            if ((lane & 15) == 0) {
                sred[wave][2 * (mt * 16 + 4 * fq + r)] = s;
                sred[wave][2 * (mt * 16 + 4 * fq + r) + 1] = q;
            }
        }
    __syncthreads();
    constexpr int V = 2 * COUT;
    for (int t = tid; t < V; t += EN_THREADS)
        e.part[(int64_t)tile * V + t] = ((sred[0][t] + sred[1][t]) + sred[2][t]) + sred[3][t];
}

// Instance-norm pairs (rstd, -mean rstd) of C channels [co, co + C) of a
// producer's output from its per-tile partials (st: [tiles][ld] floats, (sum,
// sumsq) per channel) over n pixels -> ss[2 C] in LDS.  Thread t sums the
// quad t % (2C/4) of tiles t / (2C/4) + SL i (loads issued B tiles at a time),
// the SL slices are summed in slice order: the same fixed order in every
// workgroup.  Ends with a barrier.
template <int C>
__device__ void reduce_stats(const float* st, int tiles, int ld, int co, double n, float eps, float* ss, double* dred)
{
    constexpr int V = 2 * C, Q4 = V / 4, SL = EN_THREADS / Q4;
    const int tid = threadIdx.x, q = tid % Q4, s = tid / Q4;
    const float* base = st + 2 * co + 4 * q;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    constexpr int B = 8;   // tiles per thread per batch
    for (int g0 = s; g0 < tiles; g0 += B * SL) {
        float4 v[B];
#pragma unroll
        for (int u = 0; u < B; u++) {
            const int g = g0 + u * SL;
            v[u] = g < tiles ? *(const float4*)(base + (int64_t)g * ld) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < B; u++) {
            a[0] += (double)v[u].x;
            a[1] += (double)v[u].y;
            a[2] += (double)v[u].z;
            a[3] += (double)v[u].w;
        }
    }
#pragma unroll
    for (int c = 0; c < 4; c++) dred[s * V + 4 * q + c] = a[c];
    __syncthreads();
    if (tid < C) {
        double S = 0.0, Q = 0.0;
        for (int k = 0; k < SL; k++) {
            S += dred[k * V + 2 * tid];
            Q += dred[k * V + 2 * tid + 1];
        }
        const double mean = S / n;
        double var = Q / n - mean * mean;
        var = var > 0.0 ? var : 0.0;
        const float rstd = 1.f / sqrtf((float)var + eps);
        ss[2 * tid] = rstd;
        ss[2 * tid + 1] = (float)(-mean) * rstd;
    }
    __syncthreads();
}

// 3x3 (pad 1) or 1x1 (pad 0) convolution, stride S, CIN -> COUT channels, over
// the transformed input x = xform(a, r).  DS (the stride-2 block of layer2):
// output channels [COUT/2, COUT) are the block's 1x1 stride-2 downsample
// (extractor.py:43-44), packed as the centre tap of a 3x3 kernel; its MFMAs run
// at that tap only.
template <int KS, int S, int CIN, int COUT, int XMODE, bool DS>
__global__ __launch_bounds__(EN_THREADS) void enc_conv_kernel(EncBatch p)
{
    constexpr int PAD = KS / 2, IH = (EN_TH - 1) * S + KS, IW = (EN_TW - 1) * S + KS;
    constexpr int CP = CIN + 8, KC = CIN / 32, NT = COUT / 16, TAPS = KS * KS;
    __shared__ __attribute__((aligned(16))) half_t sW[TAPS * KC * COUT * 32];
    __shared__ __attribute__((aligned(16))) half_t sX[IH * IW * CP];
    __shared__ float sred[4][2 * COUT];
    __shared__ double dred[4 * EN_THREADS];
    __shared__ float sss[2][2 * CIN];

    const dpvo_conv_args& e = p.e[blockIdx.y];
    const int tile = blockIdx.x;
    const int oy0 = (tile / p.tiles_x) * EN_TH, ox0 = (tile % p.tiles_x) * EN_TW;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fq = lane >> 4;

    // Every global read of the prologue is in flight before the first is
    // used: the weights go global -> LDS by DMA (1 KB per wave instruction;
    // the host packs them pre-swizzled, see wrow()), the halo loads fill a
    // fully unrolled register batch.
    {
        constexpr int NP = TAPS * KC * COUT / 16;   // 1 KB pieces
        const char* w = (const char*)e.w;
        for (int pc = wave; pc < NP; pc += 4) wlds16(w + pc * 1024 + lane * 16, (char*)sW + pc * 1024);
    }
    // instance-norm pairs of the input (and residual): reduced while the
    // weight DMA is in flight, before the halo batch occupies registers
    const bool a_norm = XMODE != 0 && e.a_st != nullptr, r_norm = XMODE == 2 && e.r_st != nullptr;
    const double n_in = (double)p.Hi * p.Wi;
    if (a_norm) reduce_stats<CIN>(e.a_st, e.a_st_tiles, e.a_st_ld, e.a_co, n_in, e.eps, sss[0], dred);
    if (r_norm) reduce_stats<CIN>(e.r_st, e.r_st_tiles, e.r_st_ld, e.r_co, n_in, e.eps, sss[1], dred);
    constexpr int CJ = CIN / 8;                   // 16-byte chunks per pixel; tid % CJ is fixed per thread
    constexpr int NX = (IH * IW * CJ + EN_THREADS - 1) / EN_THREADS;
    const int j = tid % CJ;
    const int gy0 = oy0 * S - PAD, gx0 = ox0 * S - PAD;
    const half_t* A = (const half_t*)e.a;
    const half_t* R = (const half_t*)e.r;
    h8_t va[NX], vr[XMODE == 2 ? NX : 1];
#pragma unroll
    for (int u = 0; u < NX; u++) {
        const int it = tid + u * EN_THREADS, q = it / CJ;
        const int gy = gy0 + q / IW, gx = gx0 + q % IW;
        const bool ok = it < IH * IW * CJ && gy >= 0 && gy < p.Hi && gx >= 0 && gx < p.Wi;
        const int64_t pix = ok ? (int64_t)gy * p.Wi + gx : 0;
        va[u] = ok ? load_h8(A + pix * e.a_ps + e.a_co + 8 * j) : (h8_t)(half_t)0;
        if (XMODE == 2) vr[u] = ok ? load_h8(R + pix * e.r_ps + e.r_co + 8 * j) : (h8_t)(half_t)0;
    }
    float as[16], rs[16];
#pragma unroll
    for (int c = 0; c < 16; c++) {
        as[c] = a_norm ? sss[0][16 * j + c] : 0.f;
        rs[c] = r_norm ? sss[1][16 * j + c] : 0.f;
    }
    {
        half_t* X = (half_t*)e.xout;
#pragma unroll
        for (int u = 0; u < NX; u++) {
            const int it = tid + u * EN_THREADS, q = it / CJ, qy = q / IW, qx = q % IW;
            if (it >= IH * IW * CJ) break;
            const int gy = gy0 + qy, gx = gx0 + qx;
            const bool ok = gy >= 0 && gy < p.Hi && gx >= 0 && gx < p.Wi;
            h8_t v = (h8_t)(half_t)0;
            if (ok) v = xform<XMODE>(va[u], as, a_norm, XMODE == 2 ? vr[u] : va[u], rs, r_norm);
            // the block output this conv reads is the next block's residual:
            // written once, by the tile whose interior holds the pixel
            if (S == 1 && X != nullptr && ok && qy >= PAD && qy < PAD + EN_TH && qx >= PAD && qx < PAD + EN_TW)
                *(h8_t*)(X + ((int64_t)gy * p.Wi + gx) * e.x_ps + 8 * j) = v;
            *(h8_t*)(sX + q * CP + 8 * j) = v;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the weight DMA
    __syncthreads();

    f4_t acc[2][NT];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int mt = 0; mt < NT; mt++) acc[i][mt] = f4_t{0.f, 0.f, 0.f, 0.f};
    const int px = lane & 15;
#pragma unroll
    for (int tap = 0; tap < TAPS; tap++) {
        const int ky = tap / KS, kx = tap % KS;
#pragma unroll
        for (int kc = 0; kc < KC; kc++) {
            h8_t bx[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int q = ((2 * wave + i) * S + ky) * IW + px * S + kx;
                bx[i] = *(const h8_t*)(sX + q * CP + kc * 32 + 8 * fq);
            }
#pragma unroll
            for (int mt = 0; mt < NT; mt++) {
                if (DS && mt >= NT / 2 && tap != TAPS / 2) continue;   // downsample: centre tap only
                const h8_t wa = *(const h8_t*)(sW + wrow((tap * KC + kc) * COUT + mt * 16 + px, fq));
#pragma unroll
                for (int i = 0; i < 2; i++) acc[i][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa, bx[i], acc[i][mt], 0, 0, 0);
            }
        }
    }
    conv_epilogue<COUT>(e, acc, p.Ho, p.Wo, oy0, ox0, tile, sred);
}

// conv1 of BasicEncoder4 (7x7, stride 2, pad 3, 3 -> 32) on the uint8 frame,
// with the Patchifier's 2 (x / 255) - 0.5 (net.py:116) applied on load and
// rounded to fp16 as autocast's input cast does.  K = 3 x 49 = 147 padded to
// 160 (five 32-wide chunks), im2col in LDS.
constexpr int ST_K = 160, ST_KP = 168, ST_IH = 2 * (EN_TH - 1) + 7, ST_IW = 2 * (EN_TW - 1) + 7;

template <int K0>   // im2col of K entries [K0, K0 + 80) of one output pixel (offsets compile-time)
__device__ __forceinline__ void stem_im2col(const half_t* sI, int py, int px, half_t* dst)
{
    const half_t* src = sI + 2 * py * ST_IW + 2 * px;
#pragma unroll
    for (int g = 0; g < 80; g += 8) {
        h8_t v;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int k = K0 + g + i;
            v[i] = k < 147 ? src[(k / 49) * ST_IH * ST_IW + ((k % 49) / 7) * ST_IW + k % 7] : (half_t)0;
        }
        *(h8_t*)(dst + K0 + g) = v;
    }
}

__global__ __launch_bounds__(EN_THREADS) void enc_stem_kernel(EncBatch p, const uint8_t* image)
{
    __shared__ __attribute__((aligned(16))) half_t sA[EN_TH * EN_TW * ST_KP];
    __shared__ __attribute__((aligned(16))) half_t sW[32 * ST_K];
    __shared__ half_t sI[3 * ST_IH * ST_IW];
    __shared__ float sred[4][64];

    const dpvo_conv_args& e = p.e[blockIdx.y];
    const int tile = blockIdx.x;
    const int oy0 = (tile / p.tiles_x) * EN_TH, ox0 = (tile % p.tiles_x) * EN_TW;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fq = lane >> 4;
    // weights [5 chunks][32 rows][32] (wrow-swizzled): 10 KB by DMA
    for (int pc = wave; pc < 32 * ST_K / 512; pc += 4)
        wlds16((const char*)e.w + pc * 1024 + lane * 16, (char*)sW + pc * 1024);
    // the 3 x 21 x 37 input window: every byte load in flight, then converted
    constexpr int NI = 3 * ST_IH * ST_IW, NB = (NI + EN_THREADS - 1) / EN_THREADS;
    const int gy0 = 2 * oy0 - 3, gx0 = 2 * ox0 - 3;
    uint8_t b[NB];
#pragma unroll
    for (int u = 0; u < NB; u++) {
        const int it = tid + u * EN_THREADS, c = it / (ST_IH * ST_IW), q = it % (ST_IH * ST_IW);
        const int gy = gy0 + q / ST_IW, gx = gx0 + q % ST_IW;
        const bool ok = it < NI && gy >= 0 && gy < p.Hi && gx >= 0 && gx < p.Wi;
        b[u] = ok ? image[((int64_t)c * p.Hi + gy) * p.Wi + gx] : 0;
    }
#pragma unroll
    for (int u = 0; u < NB; u++) {
        const int it = tid + u * EN_THREADS, q = it % (ST_IH * ST_IW);
        if (it >= NI) break;
        const int gy = gy0 + q / ST_IW, gx = gx0 + q % ST_IW;
        const bool ok = gy >= 0 && gy < p.Hi && gx >= 0 && gx < p.Wi;
        sI[it] = ok ? (half_t)(2.f * ((float)b[u] / 255.f) - 0.5f) : (half_t)0;
    }
    __syncthreads();
    {
        const int pix = tid & 127;
        if (tid < 128) stem_im2col<0>(sI, pix / EN_TW, pix % EN_TW, sA + pix * ST_KP);
        else stem_im2col<80>(sI, pix / EN_TW, pix % EN_TW, sA + pix * ST_KP);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the weight DMA
    __syncthreads();
    f4_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int mt = 0; mt < 2; mt++) acc[i][mt] = f4_t{0.f, 0.f, 0.f, 0.f};
    const int px = lane & 15;
#pragma unroll
    for (int kc = 0; kc < ST_K / 32; kc++) {
        h8_t bx[2];
#pragma unroll
        for (int i = 0; i < 2; i++) bx[i] = *(const h8_t*)(sA + ((2 * wave + i) * EN_TW + px) * ST_KP + kc * 32 + 8 * fq);
#pragma unroll
        for (int mt = 0; mt < 2; mt++) {
            const h8_t wa = *(const h8_t*)(sW + wrow(kc * 32 + mt * 16 + px, fq));
#pragma unroll
            for (int i = 0; i < 2; i++) acc[i][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa, bx[i], acc[i][mt], 0, 0, 0);
        }
    }
    conv_epilogue<32>(e, acc, p.Ho, p.Wo, oy0, ox0, tile, sred);
}

// The final 1x1 convolution (64 -> cout) at given pixels only: out[m] =
// W x(y[m], x[m]) + b, x = relu(relu(IN(a)) + res) (the last block's output),
// rounded to fp16 and scaled.  One workgroup per point.
__global__ __launch_bounds__(EN_THREADS) void enc_head_at_kernel(dpvo_conv_args e, int cout, int Hi, int Wi,
                                                                 const int64_t* xs, const int64_t* ys, int64_t M)
{
    __shared__ float sx[64];
    __shared__ double dred[4 * EN_THREADS];
    __shared__ float sss[2][128];
    const int64_t m = blockIdx.x;
    if (m >= M) return;
    const int tid = threadIdx.x;
    const int64_t yy = ys[m], xx = xs[m];
    if (e.a_st) reduce_stats<64>(e.a_st, e.a_st_tiles, e.a_st_ld, e.a_co, (double)Hi * Wi, e.eps, sss[0], dred);
    if (e.r_st) reduce_stats<64>(e.r_st, e.r_st_tiles, e.r_st_ld, e.r_co, (double)Hi * Wi, e.eps, sss[1], dred);
    if (tid < 64) {
        float v = 0.f;
        if (yy >= 0 && yy < Hi && xx >= 0 && xx < Wi) {
            const int64_t pix = yy * Wi + xx;
            half_t a = ((const half_t*)e.a)[pix * e.a_ps + e.a_co + tid];
            if (e.a_st) a = (half_t)((float)a * sss[0][2 * tid] + sss[0][2 * tid + 1]);
            a = a > (half_t)0 ? a : (half_t)0;
            half_t r = ((const half_t*)e.r)[pix * e.r_ps + e.r_co + tid];
            if (e.r_st) r = (half_t)((float)r * sss[1][2 * tid] + sss[1][2 * tid + 1]);
            half_t s = (half_t)((float)a + (float)r);
            v = s > (half_t)0 ? (float)s : 0.f;
        }
        sx[tid] = v;
    }
    __syncthreads();
    const half_t* W = (const half_t*)e.w;
    const half_t* B = (const half_t*)e.bias;
    for (int co = tid; co < cout; co += EN_THREADS) {
        const half_t* w = W + (int64_t)co * 64;
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < 64; k += 8) {
            const h8_t wv = load_h8(w + k);
#pragma unroll
            for (int c = 0; c < 8; c++) a += (float)wv[c] * sx[k + c];
        }
        half_t h = (half_t)(a + (float)B[co]);
        h = (half_t)((float)h * e.out_scale);
        ((half_t*)e.out)[m * e.o_ps + e.o_co + co] = h;
    }
}

int conv_out(int n, int ks, int s) { return (n + 2 * (ks / 2) - ks) / s + 1; }

int fill_batch(EncBatch& b, const dpvo_conv_args* enc, int n_enc, int Hi, int Wi, int ks, int s)
{
    DPVO_CHECK_ARG(n_enc == 1 || n_enc == 2, "n_enc must be 1 or 2");
    DPVO_CHECK_ARG(Hi > 0 && Wi > 0, "empty input");
    b.e[0] = enc[0];
    b.e[1] = enc[n_enc - 1];
    b.Hi = Hi;
    b.Wi = Wi;
    b.Ho = conv_out(Hi, ks, s);
    b.Wo = conv_out(Wi, ks, s);
    b.tiles_x = (b.Wo + EN_TW - 1) / EN_TW;
    b.ntiles = b.tiles_x * ((b.Ho + EN_TH - 1) / EN_TH);
    for (int i = 0; i < n_enc; i++) {
        DPVO_CHECK_ARG(enc[i].w && enc[i].bias && enc[i].out, "w, bias and out are required");
        DPVO_CHECK_ARG(!enc[i].a_st || (enc[i].a_st_tiles > 0 && enc[i].a_st_ld % 4 == 0 && enc[i].a_co % 8 == 0),
                       "a_st: tiles > 0, row length a multiple of 4");
        DPVO_CHECK_ARG(!enc[i].r_st || (enc[i].r_st_tiles > 0 && enc[i].r_st_ld % 4 == 0 && enc[i].r_co % 8 == 0),
                       "r_st: tiles > 0, row length a multiple of 4");
        DPVO_CHECK_ARG(((uintptr_t)enc[i].out & 7) == 0 && enc[i].o_ps % 4 == 0 && enc[i].o_co % 4 == 0,
                       "out must allow 8-byte stores");
    }
    return 0;
}


// The Patchifier's gathers at the M patch centres (net.py:301-315), one
// workgroup per patch, in one launch instead of ~80 torch launches:
//   gmap    = patchify(fmap, c, 1)            [M][128][3][3]
//   imap    = inet at c (head_at's rows)      [M][dim]
//   patches = patchify(grid(x, y, 1), c, 1)   [M][3][3][3]
//   clr     = patchify(image', 4 (c + 0.5), 0) [M][3], image' = lut[u8]
// Each patchify gathers the (2r+2)^2 window at floor(c) - r (zero outside
// the map, correlation_kernel.cu:288-308) and reduces it bilinearly with
// frac(c) as correlation.py:51-69 does -- ((w00 p00 + w01 p01) + w10 p10) +
// w11 p11, w00 = (1-dy)(1-dx), w01 = (1-dy) dx, w10 = dy (1-dx), w11 = dy dx --
// in fp32 with every product and sum rounded on its own (the torch
// composition's separate kernels: bit-identical).
struct PgWin {
    float w00, w01, w10, w11;
    int x0, y0;   // floor(c)
};

__device__ __forceinline__ PgWin pg_window(float cx, float cy)
{
    const float dx = __fsub_rn(cx, floorf(cx)), dy = __fsub_rn(cy, floorf(cy));
    const float ux = __fsub_rn(1.f, dx), uy = __fsub_rn(1.f, dy);
    return {__fmul_rn(uy, ux), __fmul_rn(uy, dx), __fmul_rn(dy, ux), __fmul_rn(dy, dx), floor_to_int_sat(cx),
            floor_to_int_sat(cy)};
}

__device__ __forceinline__ float pg_bilinear(const PgWin& w, float p00, float p01, float p10, float p11)
{
    return __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(w.w00, p00), __fmul_rn(w.w01, p01)), __fmul_rn(w.w10, p10)),
                     __fmul_rn(w.w11, p11));
}

struct PgArgs {
    const half_t* fmap; int64_t f_sc, f_sy, f_sx; int h, w;
    const half_t* imap_at; int dim;
    const uint8_t* image; int H, W; const float* lut;
    const int64_t* xs; const int64_t* ys;
    float* gmap; float* imap; float* patches; float* clr;
};

__global__ __launch_bounds__(256) void patch_gather_kernel(PgArgs a, int64_t M)
{
    const int64_t m = blockIdx.x;
    if (m >= M) return;
    const int tid = threadIdx.x;
    const float cx = (float)a.xs[m], cy = (float)a.ys[m];
    const PgWin g = pg_window(cx, cy);
    // gmap: channel fastest, so a wave reads whole pixel rows of the NHWC map
    for (int idx = tid; idx < 9 * 128; idx += 256) {
        const int c = idx & 127, ab = idx >> 7, ia = ab / 3, ib = ab - 3 * ia;
        float p[2][2];
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int v = 0; v < 2; v++) {
                const int i = wrap_add(g.y0, ia + u - 1), j = wrap_add(g.x0, ib + v - 1);
                p[u][v] = (i >= 0 && i < a.h && j >= 0 && j < a.w)
                              ? (float)a.fmap[c * a.f_sc + (int64_t)i * a.f_sy + (int64_t)j * a.f_sx] : 0.f;
            }
        a.gmap[m * 1152 + c * 9 + ab] = pg_bilinear(g, p[0][0], p[0][1], p[1][0], p[1][1]);
    }
    for (int k = tid; k < a.dim; k += 256) a.imap[m * a.dim + k] = (float)a.imap_at[m * a.dim + k];
    if (tid < 27) {   // the (x, y, 1) grid of the stride-4 map
        const int ch = tid / 9, ab = tid - 9 * ch, ia = ab / 3, ib = ab - 3 * ia;
        float p[2][2];
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int v = 0; v < 2; v++) {
                const int i = wrap_add(g.y0, ia + u - 1), j = wrap_add(g.x0, ib + v - 1);
                const bool in = i >= 0 && i < a.h && j >= 0 && j < a.w;
                p[u][v] = !in ? 0.f : ch == 0 ? (float)j : ch == 1 ? (float)i : 1.f;
            }
        a.patches[m * 27 + tid] = pg_bilinear(g, p[0][0], p[0][1], p[1][0], p[1][1]);
    } else if (a.clr && tid >= 64 && tid < 67) {   // colour at 4 (c + 0.5) of the full frame
        const int ch = tid - 64;
        const PgWin q = pg_window(__fmul_rn(4.f, __fadd_rn(cx, 0.5f)), __fmul_rn(4.f, __fadd_rn(cy, 0.5f)));
        float p[2][2];
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int v = 0; v < 2; v++) {
                const int i = wrap_add(q.y0, u), j = wrap_add(q.x0, v);
                p[u][v] = (i >= 0 && i < a.H && j >= 0 && j < a.W)
                              ? a.lut[a.image[((int64_t)ch * a.H + i) * a.W + j]] : 0.f;
            }
        a.clr[m * 3 + ch] = pg_bilinear(q, p[0][0], p[0][1], p[1][0], p[1][1]);
    }
}

}  // namespace
}  // namespace dpvo

using namespace dpvo;

extern "C" int64_t dpvo_encoder_tiles(int Hi, int Wi, int ks, int stride)
{
    const int Ho = conv_out(Hi, ks, stride), Wo = conv_out(Wi, ks, stride);
    return (int64_t)((Wo + EN_TW - 1) / EN_TW) * ((Ho + EN_TH - 1) / EN_TH);
}

extern "C" int dpvo_encoder_stem(const uint8_t* image, int H, int W, const dpvo_conv_args* enc, int n_enc,
                                 void* stream)
{
    DPVO_CHECK_ARG(image != nullptr, "image is required");
    EncBatch b;
    if (fill_batch(b, enc, n_enc, H, W, 7, 2)) return -1;
    hipLaunchKernelGGL(enc_stem_kernel, dim3(b.ntiles, n_enc), dim3(EN_THREADS), 0, as_stream(stream), b, image);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_encoder_conv(int ks, int stride, int cin, int cout, int xmode, int Hi, int Wi,
                                 const dpvo_conv_args* enc, int n_enc, void* stream)
{
    EncBatch b;
    if (fill_batch(b, enc, n_enc, Hi, Wi, ks, stride)) return -1;
    for (int i = 0; i < n_enc; i++) {
        DPVO_CHECK_ARG(enc[i].a && enc[i].a_ps % 8 == 0 && enc[i].a_co % 8 == 0, "a must allow 16-byte loads");
        DPVO_CHECK_ARG(xmode != 2 || (enc[i].r && enc[i].r_ps % 8 == 0 && enc[i].r_co % 8 == 0),
                       "xmode 2 needs a residual allowing 16-byte loads");
        DPVO_CHECK_ARG(!enc[i].xout || (stride == 1 && ks == 3 && enc[i].x_ps % 8 == 0),
                       "xout: stride-1 3x3 convolutions only");
    }
    const dim3 grid(b.ntiles, n_enc), block(EN_THREADS);
    hipStream_t s = as_stream(stream);
#define ENC_CASE(KS, S, CI, CO, XM, DS)                                                        \
    if (ks == KS && stride == S && cin == CI && cout == CO && xmode == XM) {                   \
        hipLaunchKernelGGL((enc_conv_kernel<KS, S, CI, CO, XM, DS>), grid, block, 0, s, b);    \
        DPVO_CHECK_LAUNCH();                                                                   \
        return 0;                                                                              \
    }
    ENC_CASE(3, 1, 32, 32, 1, false)
    ENC_CASE(3, 1, 32, 32, 2, false)
    ENC_CASE(3, 2, 32, 128, 2, true)
    ENC_CASE(3, 1, 64, 64, 1, false)
    ENC_CASE(3, 1, 64, 64, 2, false)
    ENC_CASE(1, 1, 64, 128, 2, false)
#undef ENC_CASE
    set_error("dpvo_encoder_conv: unsupported layer shape (ks " + std::to_string(ks) + ", stride " +
              std::to_string(stride) + ", " + std::to_string(cin) + " -> " + std::to_string(cout) + ", xmode " +
              std::to_string(xmode) + ")");
    return -1;
}

extern "C" int dpvo_encoder_head_at(const dpvo_conv_args* e, int cout, int Hi, int Wi, const int64_t* x,
                                    const int64_t* y, int64_t M, void* stream)
{
    DPVO_CHECK_ARG(e && e->a && e->r && e->w && e->bias && e->out, "a, r, w, bias and out are required");
    DPVO_CHECK_ARG(x && y && M >= 0, "x, y and M >= 0 are required");
    DPVO_CHECK_ARG(((uintptr_t)e->w & 15) == 0, "w must be 16-byte aligned");
    if (M == 0) return 0;
    hipLaunchKernelGGL(enc_head_at_kernel, dim3((unsigned)M), dim3(EN_THREADS), 0, as_stream(stream), *e, cout, Hi, Wi,
                       x, y, M);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_patch_gather(const void* fmap, const int64_t* fmap_strides, int h, int w, const void* imap_at,
                                 int dim, const uint8_t* image, int H, int W, const float* lut, const int64_t* x,
                                 const int64_t* y, int64_t M, float* gmap, float* imap, float* patches, float* clr,
                                 void* stream)
{
    DPVO_CHECK_ARG(fmap && fmap_strides && imap_at && x && y && gmap && imap && patches, "null pointer");
    DPVO_CHECK_ARG(M >= 0 && h > 0 && w > 0 && dim >= 0, "M >= 0, a non-empty map and dim >= 0 are required");
    DPVO_CHECK_ARG(!clr || (image && lut && H > 0 && W > 0), "clr needs image, lut and the frame size");
    if (M == 0) return 0;
    PgArgs a{(const half_t*)fmap, fmap_strides[0], fmap_strides[1], fmap_strides[2], h, w,
             (const half_t*)imap_at, dim, image, H, W, lut, x, y, gmap, imap, patches, clr};
    hipLaunchKernelGGL(patch_gather_kernel, dim3((unsigned)M), dim3(256), 0, as_stream(stream), a, M);
    DPVO_CHECK_LAUNCH();
    return 0;
}

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
//    block).  Instance-norm statistics are per-workgroup partial sums in the
//    producing epilogue; the last workgroup to finish (one device-scope
//    counter) reduces them in a fixed order (fp64) and leaves the per-channel
//    (rstd, -mean rstd) pairs for the consumer -- deterministic, no extra
//    launch.
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
constexpr int EN_WROW = 40;   // LDS weight row: 32 K halves + 8 pad (conflict-free 16-B reads)

struct EncBatch {
    dpvo_conv_args e[2];
    int Hi, Wi, Ho, Wo, tiles_x, ntiles;
};

__device__ __forceinline__ h8_t load_h8(const half_t* p) { return *(const h8_t*)p; }

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
// values -> part[tile]; the last tile reduces them into ss_out.
template <int COUT>
__device__ void conv_epilogue(const dpvo_conv_args& e, f4_t (&acc)[2][COUT / 16], int Ho, int Wo, int oy0, int ox0,
                              int tile, int ntiles, float (*sred)[2 * COUT], double* dred, int* flag)
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
    constexpr int V = 2 * COUT;   // (sum, sumsq) interleaved per channel
    for (int t = tid; t < V; t += EN_THREADS)
        e.part[(int64_t)tile * V + t] = ((sred[0][t] + sred[1][t]) + sred[2][t]) + sred[3][t];
    __threadfence();
    __syncthreads();
    if (tid == 0) *flag = atomicAdd(e.counter, 1u) == (unsigned)(ntiles - 1);
    __syncthreads();
    if (!*flag) return;
    // last workgroup: fixed-order fp64 reduction of every tile's partials.
    // Thread t owns the float4 quad t % (V/4) of tiles t / (V/4) + SL i: its
    // loads are independent and issued 8 at a time (one L2 round trip per 8
    // tiles, not per tile); the SL slices are then summed in slice order.
    __threadfence();
    constexpr int Q4 = V / 4, SL = EN_THREADS / Q4;
    {
        const int q = tid % Q4, s = tid / Q4;
        const float4* P = (const float4*)e.part;
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        for (int g0 = s; g0 < ntiles; g0 += 8 * SL) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int g = g0 + u * SL;
                v[u] = g < ntiles ? P[(int64_t)g * Q4 + q] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                a0 += (double)v[u].x;
                a1 += (double)v[u].y;
                a2 += (double)v[u].z;
                a3 += (double)v[u].w;
            }
        }
        dred[s * V + 4 * q + 0] = a0;
        dred[s * V + 4 * q + 1] = a1;
        dred[s * V + 4 * q + 2] = a2;
        dred[s * V + 4 * q + 3] = a3;
    }
    __syncthreads();
    if (tid < COUT) {
        double S = 0.0, Q = 0.0;
        for (int s = 0; s < SL; s++) {
            S += dred[s * V + 2 * tid];
            Q += dred[s * V + 2 * tid + 1];
        }
        const double n = (double)Ho * Wo, mean = S / n;
        double var = Q / n - mean * mean;
        var = var > 0.0 ? var : 0.0;
        const float rstd = 1.f / sqrtf((float)var + e.eps);
        e.ss_out[2 * tid] = rstd;
        e.ss_out[2 * tid + 1] = (float)(-mean) * rstd;
    }
    if (tid == 0) *e.counter = 0u;   // ready for the next frame (and graph replays)
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
    __shared__ __attribute__((aligned(16))) half_t sW[TAPS * KC * COUT * EN_WROW];
    __shared__ __attribute__((aligned(16))) half_t sX[IH * IW * CP];
    __shared__ float sred[4][2 * COUT];
    __shared__ double dred[4 * EN_THREADS];
    __shared__ int flag;

    const dpvo_conv_args& e = p.e[blockIdx.y];
    const int tile = blockIdx.x;
    const int oy0 = (tile / p.tiles_x) * EN_TH, ox0 = (tile % p.tiles_x) * EN_TW;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fq = lane >> 4;

    // weights: global [tap][kc][co][32] -> LDS rows of 40 halves
    {
        const half_t* w = (const half_t*)e.w;
        constexpr int CH = TAPS * KC * COUT * 4;
        for (int c = tid; c < CH; c += EN_THREADS)
            *(h8_t*)(sW + (c >> 2) * EN_WROW + (c & 3) * 8) = load_h8(w + (int64_t)c * 8);
    }
    // input halo, transformed on load (zero outside the map: the conv pads x)
    {
        constexpr int CJ = CIN / 8;   // 16-byte chunks per pixel; tid % CJ is fixed per thread
        const int j = tid % CJ;
        float as[16], rs[16];
        const bool a_norm = XMODE != 0 && e.a_ss != nullptr, r_norm = XMODE == 2 && e.r_ss != nullptr;
#pragma unroll
        for (int c = 0; c < 16; c++) {
            as[c] = a_norm ? e.a_ss[16 * j + c] : 0.f;
            rs[c] = r_norm ? e.r_ss[16 * j + c] : 0.f;
        }
        const half_t* A = (const half_t*)e.a;
        const half_t* R = (const half_t*)e.r;
        half_t* X = (half_t*)e.xout;
        const int gy0 = oy0 * S - PAD, gx0 = ox0 * S - PAD;
        for (int it = tid; it < IH * IW * CJ; it += EN_THREADS) {
            const int q = it / CJ, qy = q / IW, qx = q % IW;
            const int gy = gy0 + qy, gx = gx0 + qx;
            h8_t v = (h8_t)(half_t)0;
            if (gy >= 0 && gy < p.Hi && gx >= 0 && gx < p.Wi) {
                const int64_t pix = (int64_t)gy * p.Wi + gx;
                const h8_t a = load_h8(A + pix * e.a_ps + e.a_co + 8 * j);
                h8_t r = (h8_t)(half_t)0;
                if (XMODE == 2) r = load_h8(R + pix * e.r_ps + e.r_co + 8 * j);
                v = xform<XMODE>(a, as, a_norm, r, rs, r_norm);
                // the block output this conv reads is the next block's residual:
                // written once, by the tile whose interior holds the pixel
                if (S == 1 && X != nullptr && qy >= PAD && qy < PAD + EN_TH && qx >= PAD && qx < PAD + EN_TW)
                    *(h8_t*)(X + pix * e.x_ps + 8 * j) = v;
            }
            *(h8_t*)(sX + q * CP + 8 * j) = v;
        }
    }
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
                const h8_t wa = *(const h8_t*)(sW + ((tap * KC + kc) * COUT + mt * 16 + px) * EN_WROW + 8 * fq);
#pragma unroll
                for (int i = 0; i < 2; i++) acc[i][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa, bx[i], acc[i][mt], 0, 0, 0);
            }
        }
    }
    conv_epilogue<COUT>(e, acc, p.Ho, p.Wo, oy0, ox0, tile, p.ntiles, sred, dred, &flag);
}

// conv1 of BasicEncoder4 (7x7, stride 2, pad 3, 3 -> 32) on the uint8 frame,
// with the Patchifier's 2 (x / 255) - 0.5 (net.py:116) applied on load and
// rounded to fp16 as autocast's input cast does.  K = 3 x 49 = 147 padded to
// 160 (five 32-wide chunks), im2col in LDS.
constexpr int ST_K = 160, ST_KP = 168, ST_IH = 2 * (EN_TH - 1) + 7, ST_IW = 2 * (EN_TW - 1) + 7;

__global__ __launch_bounds__(EN_THREADS) void enc_stem_kernel(EncBatch p, const uint8_t* image)
{
    __shared__ __attribute__((aligned(16))) half_t sA[EN_TH * EN_TW * ST_KP];
    __shared__ __attribute__((aligned(16))) half_t sW[32 * ST_KP];
    __shared__ half_t sI[3 * ST_IH * ST_IW];
    __shared__ float sred[4][64];
    __shared__ double dred[4 * EN_THREADS];
    __shared__ int flag;

    const dpvo_conv_args& e = p.e[blockIdx.y];
    const int tile = blockIdx.x;
    const int oy0 = (tile / p.tiles_x) * EN_TH, ox0 = (tile % p.tiles_x) * EN_TW;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fq = lane >> 4;
    {
        const half_t* w = (const half_t*)e.w;
        for (int c = tid; c < 32 * ST_K / 8; c += EN_THREADS)
            *(h8_t*)(sW + (c / (ST_K / 8)) * ST_KP + (c % (ST_K / 8)) * 8) = load_h8(w + (int64_t)c * 8);
    }
    const int gy0 = 2 * oy0 - 3, gx0 = 2 * ox0 - 3;
    for (int it = tid; it < 3 * ST_IH * ST_IW; it += EN_THREADS) {
        const int c = it / (ST_IH * ST_IW), q = it % (ST_IH * ST_IW);
        const int gy = gy0 + q / ST_IW, gx = gx0 + q % ST_IW;
        half_t v = (half_t)0;
        if (gy >= 0 && gy < p.Hi && gx >= 0 && gx < p.Wi) {
            const float u = (float)image[((int64_t)c * p.Hi + gy) * p.Wi + gx];
            v = (half_t)(2.f * (u / 255.f) - 0.5f);
        }
        sI[it] = v;
    }
    __syncthreads();
    for (int it = tid; it < EN_TH * EN_TW * ST_K; it += EN_THREADS) {
        const int pix = it / ST_K, k = it % ST_K;
        half_t v = (half_t)0;
        if (k < 147) {
            const int c = k / 49, ky = (k % 49) / 7, kx = k % 7;
            v = sI[(c * ST_IH + 2 * (pix / EN_TW) + ky) * ST_IW + 2 * (pix % EN_TW) + kx];
        }
        sA[pix * ST_KP + k] = v;
    }
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
            const h8_t wa = *(const h8_t*)(sW + (mt * 16 + px) * ST_KP + kc * 32 + 8 * fq);
#pragma unroll
            for (int i = 0; i < 2; i++) acc[i][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa, bx[i], acc[i][mt], 0, 0, 0);
        }
    }
    conv_epilogue<32>(e, acc, p.Ho, p.Wo, oy0, ox0, tile, p.ntiles, sred, dred, &flag);
}

// The final 1x1 convolution (64 -> cout) at given pixels only: out[m] =
// W x(y[m], x[m]) + b, x = relu(relu(IN(a)) + res) (the last block's output),
// rounded to fp16 and scaled.  One workgroup per point.
__global__ __launch_bounds__(EN_THREADS) void enc_head_at_kernel(dpvo_conv_args e, int cout, int Hi, int Wi,
                                                                 const int64_t* xs, const int64_t* ys, int64_t M)
{
    __shared__ float sx[64];
    const int64_t m = blockIdx.x;
    if (m >= M) return;
    const int tid = threadIdx.x;
    const int64_t yy = ys[m], xx = xs[m];
    if (tid < 64) {
        float v = 0.f;
        if (yy >= 0 && yy < Hi && xx >= 0 && xx < Wi) {
            const int64_t pix = yy * Wi + xx;
            half_t a = ((const half_t*)e.a)[pix * e.a_ps + e.a_co + tid];
            if (e.a_ss) a = (half_t)((float)a * e.a_ss[2 * tid] + e.a_ss[2 * tid + 1]);
            a = a > (half_t)0 ? a : (half_t)0;
            half_t r = ((const half_t*)e.r)[pix * e.r_ps + e.r_co + tid];
            if (e.r_ss) r = (half_t)((float)r * e.r_ss[2 * tid] + e.r_ss[2 * tid + 1]);
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
        DPVO_CHECK_ARG(!enc[i].part || (enc[i].counter && enc[i].ss_out), "statistics need counter and ss_out");
        DPVO_CHECK_ARG(((uintptr_t)enc[i].out & 7) == 0 && enc[i].o_ps % 4 == 0 && enc[i].o_co % 4 == 0,
                       "out must allow 8-byte stores");
    }
    return 0;
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

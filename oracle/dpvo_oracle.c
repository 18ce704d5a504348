/*
 * dpvo_oracle.c -- CPU restatement of the reference DPVO patch-graph hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: it may be
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
 * and nowhere else.  The product path (wild-video-3d-reconstruction_amd/)
 * never links or calls it.
 *
 * Every routine restates one reference routine; citations are relative to
 * the reference repository root (ljjTYJR/Wild-video-3d-reconstruction).
 *
 *   oracle_corr_forward     dpvo/altcorr/correlation_kernel.cu:83-135 (kernel)
 *                           + :221-232 (ATen bilinear epilogue)
 *   oracle_patchify_forward dpvo/altcorr/correlation_kernel.cu:17-47
 *   oracle_ba_forward       dpvo/fastba/ba_cuda.cu:18-211 (device math),
 *                           :214-365 (Hessian), :422-540 (driver)
 *   oracle_reproject        dpvo/fastba/ba_cuda.cu:368-418
 *   oracle_lie_*            dpvo/lietorch/include/so3.h, se3.h, rxso3.h, sim3.h
 *   oracle_transform        dpvo/projective_ops.py:19-68
 *   oracle_point_cloud      dpvo/projective_ops.py:106-108
 *   oracle_neighbors        dpvo/fastba/ba.cpp:113-158
 *
 * Arithmetic conventions
 *  - binary16 is emulated exactly: every c10::Half operation of the reference
 *    ("compute in fp32, round to nearest even") is reproduced op by op, which
 *    makes mode ORACLE_F16 bit-exact with the reference CUDA kernel.
 *  - Build with -ffp-contract=off so no FMA is introduced behind our back.
 */
#include <math.h>
#include <stdint.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* binary16 <-> binary32                                                */
/* ------------------------------------------------------------------ */
static inline float h2f(uint16_t h)
{
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, bits;
    if (e == 0) {
        float f = (float)m * 5.9604644775390625e-08f; /* m * 2^-24, exact */
        return sign ? -f : f;
    } else if (e == 31) {
        bits = sign | 0x7f800000u | (m << 13);
    } else {
        bits = sign | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

/* round-to-nearest-even, the behaviour of __float2half_rn / c10::Half(float) */
static inline uint16_t f2h(float f)
{
    uint32_t x;
    memcpy(&x, &f, 4);
    uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
    uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) {
        if (ax > 0x7f800000u) return (uint16_t)(sign | 0x7e00u);
        return (uint16_t)(sign | 0x7c00u);
    }
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* >= 65520 */
    if (ax < 0x38800000u) {                                   /* < 2^-14 */
        float v;
        memcpy(&v, &ax, 4);
        float r = rintf(v * 16777216.0f); /* exact scale, RNE to integer */
        return (uint16_t)(sign | (uint16_t)r);
    }
    uint32_t e = (ax >> 23) - 112u, m = ax & 0x7fffffu;
    uint32_t h = (e << 10) | (m >> 13), rem = m & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h += 1u;
    return (uint16_t)(sign | h);
}

/* c10::Half arithmetic: fp32 op then round */
static inline uint16_t hmul(uint16_t a, uint16_t b) { return f2h(h2f(a) * h2f(b)); }
static inline uint16_t hadd(uint16_t a, uint16_t b) { return f2h(h2f(a) + h2f(b)); }
static inline uint16_t hsub(uint16_t a, uint16_t b) { return f2h(h2f(a) - h2f(b)); }

void oracle_f32_to_f16(const float* in, uint16_t* out, int64_t n)
{
    for (int64_t i = 0; i < n; i++) out[i] = f2h(in[i]);
}
void oracle_f16_to_f32(const uint16_t* in, float* out, int64_t n)
{
    for (int64_t i = 0; i < n; i++) out[i] = h2f(in[i]);
}

/* CUDA cvt.rzi.s32.f32: NaN -> 0, saturating */
static inline int32_t cvt_i32(float f)
{
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT32_MAX;
    if (f <= -2147483648.0f) return INT32_MIN;
    return (int32_t)f;
}
/* 32-bit wrapping add, as the device int arithmetic does */
static inline int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }

/* ------------------------------------------------------------------ */
/* altcorr                                                              */
/* ------------------------------------------------------------------ */
enum { ORACLE_F16 = 0, ORACLE_F32 = 1, ORACLE_F64 = 2, ORACLE_F16_ACC64 = 3 };

/*
 * fmap1: [B][N1][C][H][W] (the gmap of patch features, H=W=P)
 * fmap2: [B][N2][C][H2][W2] (one pyramid level of the frame features)
 * coords: [B][M][2][H][W] float
 * out: contiguous [B][M][D-1][D-1][H][W] -- the memory of the reference's
 *      pre-permute tensor (correlation_kernel.cu:226-232); the reference
 *      returns it as .permute(0,1,3,2,4,5).
 * mode ORACLE_F16: fmaps/out are binary16 bit patterns, reference arithmetic.
 * mode ORACLE_F32: fmaps/out float; dot product as fmaf chain (nvcc contracts
 *      `s += a*b`), epilogue as separate float ops.
 * mode ORACLE_F64: fmaps/out double.
 * mode ORACLE_F16_ACC64: fmaps binary16, everything else in double (accuracy
 *      reference), out double.
 */
int oracle_corr_forward(int mode, const void* fmap1, const int64_t* s1sz, const int64_t* s1st,
                        const void* fmap2, const int64_t* s2sz, const int64_t* s2st,
                        const float* coords, const int64_t* csz, const int64_t* cst,
                        const int64_t* ii, const int64_t* jj, int radius, void* out)
{
    const int R = radius, D = 2 * radius + 2, Do = D - 1;
    const int64_t B = csz[0], M = csz[1], H = csz[3], W = csz[4];
    const int64_t C = s1sz[2], N1 = s1sz[1], N2 = s2sz[1], H2 = s2sz[3], W2 = s2sz[4];
    int status = 0;
    /* edges are independent: OpenMP over (b, m) when built with -fopenmp
     * (each edge is computed by one thread in the same order either way) */
#pragma omp parallel
    {
    double* raw = (double*)malloc(sizeof(double) * D * D);
    uint16_t* rawh = (uint16_t*)malloc(sizeof(uint16_t) * D * D);
    if (!raw || !rawh) {
#pragma omp atomic write
        status = -1;
    }
#pragma omp for schedule(dynamic, 4)
    for (int64_t bm = 0; bm < B * M; bm++)
    for (int64_t i0 = 0; i0 < H; i0++)
    for (int64_t j0 = 0; j0 < W; j0++) {
        const int64_t b = bm / M, m = bm % M;
        if (!raw || !rawh) continue;
        const int64_t ix = (int32_t)ii[m], jx = (int32_t)jj[m];
        const int valid_idx = ix >= 0 && ix < N1 && jx >= 0 && jx < N2;
        const float x = coords[b * cst[0] + m * cst[1] + 0 * cst[2] + i0 * cst[3] + j0 * cst[4]];
        const float y = coords[b * cst[0] + m * cst[1] + 1 * cst[2] + i0 * cst[3] + j0 * cst[4]];
        const int32_t fy = cvt_i32(floorf(y)), fx = cvt_i32(floorf(x));
        for (int a = 0; a < D; a++)
        for (int bb = 0; bb < D; bb++) {
            const int32_t i1 = wadd(fy, a - R), j1 = wadd(fx, bb - R);
            const int inb = valid_idx && i1 >= 0 && i1 < H2 && j1 >= 0 && j1 < W2;
            const int64_t o1 = b * s1st[0] + ix * s1st[1] + i0 * s1st[3] + j0 * s1st[4];
            const int64_t o2 = b * s2st[0] + jx * s2st[1] + (int64_t)i1 * s2st[3] + (int64_t)j1 * s2st[4];
            if (mode == ORACLE_F16) {
                uint16_t s = 0;
                if (inb) {
                    const uint16_t* f1 = (const uint16_t*)fmap1;
                    const uint16_t* f2 = (const uint16_t*)fmap2;
                    for (int64_t c = 0; c < C; c++)
                        s = hadd(s, hmul(f1[o1 + c * s1st[2]], f2[o2 + c * s2st[2]]));
                }
                rawh[a * D + bb] = s;
            } else if (mode == ORACLE_F32) {
                float s = 0.f;
                if (inb) {
                    const float* f1 = (const float*)fmap1;
                    const float* f2 = (const float*)fmap2;
                    for (int64_t c = 0; c < C; c++) s = fmaf(f1[o1 + c * s1st[2]], f2[o2 + c * s2st[2]], s);
                }
                raw[a * D + bb] = s;
            } else if (mode == ORACLE_F64) {
                double s = 0.0;
                if (inb) {
                    const double* f1 = (const double*)fmap1;
                    const double* f2 = (const double*)fmap2;
                    for (int64_t c = 0; c < C; c++) s = fma(f1[o1 + c * s1st[2]], f2[o2 + c * s2st[2]], s);
                }
                raw[a * D + bb] = s;
            } else {
                double s = 0.0;
                if (inb) {
                    const uint16_t* f1 = (const uint16_t*)fmap1;
                    const uint16_t* f2 = (const uint16_t*)fmap2;
                    for (int64_t c = 0; c < C; c++)
                        s += (double)h2f(f1[o1 + c * s1st[2]]) * (double)h2f(f2[o2 + c * s2st[2]]);
                }
                raw[a * D + bb] = s;
            }
        }
        /* bilinear epilogue, correlation_kernel.cu:221-232 */
        const float dxf = x - floorf(x), dyf = y - floorf(y);
        for (int a = 0; a < Do; a++)
        for (int bb = 0; bb < Do; bb++) {
            const int64_t oo = ((((b * M + m) * Do + a) * Do + bb) * H + i0) * W + j0;
            if (mode == ORACLE_F16) {
                const uint16_t one = 0x3c00, dx = f2h(dxf), dy = f2h(dyf);
                const uint16_t omdx = hsub(one, dx), omdy = hsub(one, dy);
                uint16_t o = hmul(hmul(omdx, omdy), rawh[a * D + bb]);
                o = hadd(o, hmul(hmul(dx, omdy), rawh[a * D + bb + 1]));
                o = hadd(o, hmul(hmul(omdx, dy), rawh[(a + 1) * D + bb]));
                o = hadd(o, hmul(hmul(dx, dy), rawh[(a + 1) * D + bb + 1]));
                ((uint16_t*)out)[oo] = o;
            } else if (mode == ORACLE_F32) {
                const float dx = dxf, dy = dyf, omdx = 1.f - dx, omdy = 1.f - dy;
                float o = (omdx * omdy) * (float)raw[a * D + bb];
                o = o + (dx * omdy) * (float)raw[a * D + bb + 1];
                o = o + (omdx * dy) * (float)raw[(a + 1) * D + bb];
                o = o + (dx * dy) * (float)raw[(a + 1) * D + bb + 1];
                ((float*)out)[oo] = o;
            } else {
                const double dx = dxf, dy = dyf, omdx = 1.0 - dx, omdy = 1.0 - dy;
                double o = (omdx * omdy) * raw[a * D + bb];
                o += (dx * omdy) * raw[a * D + bb + 1];
                o += (omdx * dy) * raw[(a + 1) * D + bb];
                o += (dx * dy) * raw[(a + 1) * D + bb + 1];
                ((double*)out)[oo] = o;
            }
        }
    }
    free(raw);
    free(rawh);
    }
    return status;
}

/* OpenMP threads of the parallel oracle loops (1 = the scalar port) */
void oracle_set_threads(int n)
{
#ifdef _OPENMP
    omp_set_num_threads(n > 0 ? n : 1);
#else
    (void)n;
#endif
}

int oracle_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------------ */
/* patchify (correlation_kernel.cu:17-47)                               */
/* ------------------------------------------------------------------ */
/* net: [B][C][H][W]; coords: contiguous [B][M][2]; out: contiguous
 * [B][M][C][D][D], pre-zeroed by the caller. elem_bytes 2, 4 or 8. */
int oracle_patchify_forward(int elem_bytes, const void* net, const int64_t* nsz, const int64_t* nst,
                            const float* coords, int64_t M, int radius, void* out)
{
    const int R = radius, D = 2 * radius + 2;
    const int64_t B = nsz[0], C = nsz[1], H = nsz[2], W = nsz[3];
    for (int64_t n = 0; n < B; n++)
    for (int64_t m = 0; m < M; m++)
    for (int a = 0; a < D; a++)
    for (int b = 0; b < D; b++) {
        const float x = coords[(n * M + m) * 2 + 0], y = coords[(n * M + m) * 2 + 1];
        const int32_t i = wadd(cvt_i32(floorf(y)), a - R), j = wadd(cvt_i32(floorf(x)), b - R);
        if (!(i >= 0 && i < H && j >= 0 && j < W)) continue;
        for (int64_t k = 0; k < C; k++) {
            const int64_t src = n * nst[0] + k * nst[1] + (int64_t)i * nst[2] + (int64_t)j * nst[3];
            const int64_t dst = (((n * M + m) * C + k) * D + a) * D + b;
            memcpy((char*)out + dst * elem_bytes, (const char*)net + src * elem_bytes, elem_bytes);
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* fastba device math, restated in float (ba_cuda.cu:18-156)            */
/* ------------------------------------------------------------------ */
static void actSO3f(const float* q, const float* X, float* Y)
{
    float uv[3];
    uv[0] = 2.0f * (q[1] * X[2] - q[2] * X[1]);
    uv[1] = 2.0f * (q[2] * X[0] - q[0] * X[2]);
    uv[2] = 2.0f * (q[0] * X[1] - q[1] * X[0]);
    Y[0] = X[0] + q[3] * uv[0] + (q[1] * uv[2] - q[2] * uv[1]);
    Y[1] = X[1] + q[3] * uv[1] + (q[2] * uv[0] - q[0] * uv[2]);
    Y[2] = X[2] + q[3] * uv[2] + (q[0] * uv[1] - q[1] * uv[0]);
}
static void actSE3f(const float* t, const float* q, const float* X, float* Y)
{
    actSO3f(q, X, Y);
    Y[3] = X[3];
    Y[0] += X[3] * t[0];
    Y[1] += X[3] * t[1];
    Y[2] += X[3] * t[2];
}
static void adjSE3f(const float* t, const float* q, const float* X, float* Y)
{
    const float qinv[4] = {-q[0], -q[1], -q[2], q[3]};
    float u[3], v[3];
    actSO3f(qinv, &X[0], &Y[0]);
    actSO3f(qinv, &X[3], &Y[3]);
    u[0] = t[2] * X[1] - t[1] * X[2];
    u[1] = t[0] * X[2] - t[2] * X[0];
    u[2] = t[1] * X[0] - t[0] * X[1];
    actSO3f(qinv, u, v);
    Y[3] += v[0];
    Y[4] += v[1];
    Y[5] += v[2];
}
static void relSE3f(const float* ti, const float* qi, const float* tj, const float* qj, float* tij, float* qij)
{
    qij[0] = -qj[3] * qi[0] + qj[0] * qi[3] - qj[1] * qi[2] + qj[2] * qi[1];
    qij[1] = -qj[3] * qi[1] + qj[1] * qi[3] - qj[2] * qi[0] + qj[0] * qi[2];
    qij[2] = -qj[3] * qi[2] + qj[2] * qi[3] - qj[0] * qi[1] + qj[1] * qi[0];
    qij[3] = qj[3] * qi[3] + qj[0] * qi[0] + qj[1] * qi[1] + qj[2] * qi[2];
    actSO3f(qij, ti, tij);
    tij[0] = tj[0] - tij[0];
    tij[1] = tj[1] - tij[1];
    tij[2] = tj[2] - tij[2];
}
static void expSO3f(const float* phi, float* q)
{
    const float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
    const float theta_p4 = theta_sq * theta_sq;
    const float theta = sqrtf(theta_sq);
    float imag, real;
    if (theta_sq < 1e-8) {
        imag = (float)(0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_p4);
        real = (float)(1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_p4);
    } else {
        imag = sinf(0.5f * theta) / theta;
        real = cosf(0.5f * theta);
    }
    q[0] = imag * phi[0];
    q[1] = imag * phi[1];
    q[2] = imag * phi[2];
    q[3] = real;
}
static void crossInplacef(const float* a, float* b)
{
    const float x[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    b[0] = x[0];
    b[1] = x[1];
    b[2] = x[2];
}
static void expSE3f(const float* xi, float* t, float* q)
{
    expSO3f(xi + 3, q);
    float tau[3] = {xi[0], xi[1], xi[2]};
    const float phi[3] = {xi[3], xi[4], xi[5]};
    const float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
    const float theta = sqrtf(theta_sq);
    t[0] = tau[0];
    t[1] = tau[1];
    t[2] = tau[2];
    if (theta > 1e-4) {
        const float a = (1 - cosf(theta)) / theta_sq;
        crossInplacef(phi, tau);
        t[0] += a * tau[0];
        t[1] += a * tau[1];
        t[2] += a * tau[2];
        const float b = (theta - sinf(theta)) / (theta * theta_sq);
        crossInplacef(phi, tau);
        t[0] += b * tau[0];
        t[1] += b * tau[1];
        t[2] += b * tau[2];
    }
}
static void retrSE3f(const float* xi, const float* t, const float* q, float* t1, float* q1)
{
    float dt[3] = {0, 0, 0}, dq[4] = {0, 0, 0, 1};
    expSE3f(xi, dt, dq);
    q1[0] = dq[3] * q[0] + dq[0] * q[3] + dq[1] * q[2] - dq[2] * q[1];
    q1[1] = dq[3] * q[1] + dq[1] * q[3] + dq[2] * q[0] - dq[0] * q[2];
    q1[2] = dq[3] * q[2] + dq[2] * q[3] + dq[0] * q[1] - dq[1] * q[0];
    q1[3] = dq[3] * q[3] - dq[0] * q[0] - dq[1] * q[1] - dq[2] * q[2];
    actSO3f(dq, t, t1);
    t1[0] += dt[0];
    t1[1] += dt[1];
    t1[2] += dt[2];
}

static int cmp_i64(const void* a, const void* b)
{
    const int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return (x > y) - (x < y);
}

/* torch::_unique(kk, sorted=true, return_inverse=true) */
static int64_t unique_sorted(const int64_t* kk, int64_t E, int64_t** kx_out, int64_t** ku_out)
{
    int64_t* tmp = (int64_t*)malloc(sizeof(int64_t) * (E > 0 ? E : 1));
    int64_t* ku = (int64_t*)malloc(sizeof(int64_t) * (E > 0 ? E : 1));
    memcpy(tmp, kk, sizeof(int64_t) * E);
    qsort(tmp, E, sizeof(int64_t), cmp_i64);
    int64_t Mu = 0;
    for (int64_t i = 0; i < E; i++)
        if (i == 0 || tmp[i] != tmp[i - 1]) tmp[Mu++] = tmp[i];
    for (int64_t e = 0; e < E; e++) {
        int64_t lo = 0, hi = Mu - 1;
        while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if (tmp[mid] < kk[e]) lo = mid + 1; else hi = mid;
        }
        ku[e] = lo;
    }
    *kx_out = tmp;
    *ku_out = ku;
    return Mu;
}

/* dense Cholesky (lower) in double; returns 0 on success, k+1 if the leading
 * minor of order k+1 is not positive definite (torch.linalg.cholesky info).
 * Row i's leading zeros (columns < first[i]) stay zero in L, so the inner
 * products start at the later of the two rows' first nonzero: the terms
 * skipped are exact zeros and the result equals the plain dense loop's. */
static int cholesky_d(double* A, int n)
{
    int* first = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        int f = i;
        for (int k = 0; k < i; k++)
            if (A[i * n + k] != 0.0) { f = k; break; }
        first[i] = f;
    }
    for (int j = 0; j < n; j++) {
        double s = A[j * n + j];
        for (int k = first[j]; k < j; k++) s -= A[j * n + k] * A[j * n + k];
        if (!(s > 0.0)) { free(first); return j + 1; }
        const double l = sqrt(s);
        A[j * n + j] = l;
        for (int i = j + 1; i < n; i++) {
            if (first[i] > j) continue; /* A[i][j] is and stays 0 */
            double t = A[i * n + j];
            for (int k = first[i] > first[j] ? first[i] : first[j]; k < j; k++) t -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = t / l;
        }
    }
    free(first);
    return 0;
}

/*
 * fastba.BA (dpvo/fastba/ba.py:7-8 -> ba_cuda.cu:422-540), restated on the
 * CPU.  poses [*][7] and patches [*][3][P][P] are updated in place.
 * Accumulations happen in float in edge order (one admissible order of the
 * reference's float atomics); the Schur complement, Cholesky and back
 * substitution are carried in double (the reference uses fp32 cuBLAS /
 * cuSOLVER) and rounded to float.
 * Returns 0, or the Cholesky info (>0) of the failing iteration -- the
 * reference raises at that point (torch::linalg::cholesky), leaving the
 * state of the earlier iterations.
 */
int oracle_ba_forward(float* poses, float* patches, const float* intrinsics, const float* target,
                      const float* weight, float lmbda, const int64_t* ii, const int64_t* jj,
                      const int64_t* kk, int64_t E, int P, int t0, int t1, int iterations)
{
    int64_t *kx, *ku;
    const int64_t Mu = unique_sorted(kk, E, &kx, &ku);
    const int N = t1 - t0, n6 = 6 * N;
    const int64_t PP = (int64_t)P * P, c = (P / 2) * P + P / 2; /* centre pixel [1][1] */
    float* Bm = (float*)calloc((size_t)n6 * n6 + 1, sizeof(float));
    float* Em = (float*)calloc((size_t)n6 * (Mu > 0 ? Mu : 1) + 1, sizeof(float));
    float* Cv = (float*)calloc((size_t)Mu + 1, sizeof(float));
    float* v = (float*)calloc((size_t)n6 + 1, sizeof(float));
    float* u = (float*)calloc((size_t)Mu + 1, sizeof(float));
    double* S = (double*)calloc((size_t)n6 * n6 + 1, sizeof(double));
    double* y = (double*)calloc((size_t)n6 + 1, sizeof(double));
    float* dX = (float*)calloc((size_t)n6 + 1, sizeof(float));
    float* dZ = (float*)calloc((size_t)Mu + 1, sizeof(float));
    float* Q = (float*)calloc((size_t)Mu + 1, sizeof(float));
    int* rows = (int*)calloc((size_t)n6 + 1, sizeof(int));
    int status = 0;
    const float fx = intrinsics[0], fy = intrinsics[1], cx = intrinsics[2], cy = intrinsics[3];

    for (int itr = 0; itr < iterations && status == 0; itr++) {
        memset(Bm, 0, sizeof(float) * n6 * n6);
        memset(Em, 0, sizeof(float) * n6 * Mu);
        memset(Cv, 0, sizeof(float) * Mu);
        memset(v, 0, sizeof(float) * n6);
        memset(u, 0, sizeof(float) * Mu);

        for (int64_t n = 0; n < E; n++) {
            const int64_t k = ku[n];
            int64_t ix = ii[n], jx = jj[n];
            const int64_t kxn = kk[n];
            const float ti[3] = {poses[ix * 7 + 0], poses[ix * 7 + 1], poses[ix * 7 + 2]};
            const float tj[3] = {poses[jx * 7 + 0], poses[jx * 7 + 1], poses[jx * 7 + 2]};
            const float qi[4] = {poses[ix * 7 + 3], poses[ix * 7 + 4], poses[ix * 7 + 5], poses[ix * 7 + 6]};
            const float qj[4] = {poses[jx * 7 + 3], poses[jx * 7 + 4], poses[jx * 7 + 5], poses[jx * 7 + 6]};
            float Xi[4], Xj[4], tij[3], qij[4];
            Xi[0] = (patches[(kxn * 3 + 0) * PP + c] - cx) / fx;
            Xi[1] = (patches[(kxn * 3 + 1) * PP + c] - cy) / fy;
            Xi[2] = 1.0f;
            Xi[3] = patches[(kxn * 3 + 2) * PP + c];
            relSE3f(ti, qi, tj, qj, tij, qij);
            actSE3f(tij, qij, Xi, Xj);
            const float X = Xj[0], Y = Xj[1], Z = Xj[2], Wh = Xj[3];
            const float d = (Z >= 0.2f) ? 1.0f / Z : 0.0f;
            const float d2 = d * d;
            const float x1 = fx * (X / Z) + cx, y1 = fy * (Y / Z) + cy;
            const float rx = target[n * 2 + 0] - x1, ry = target[n * 2 + 1] - y1;
            const int in_bounds = (sqrtf(rx * rx + ry * ry) < 128) && (Z > 0.2f) && (x1 > -64) && (y1 > -64) &&
                                  (x1 < 2 * cx + 64) && (y1 < 2 * cy + 64);
            const float mask = in_bounds ? 1.0f : 0.0f;
            ix -= t0;
            jx -= t0;
            const int iv = ix >= 0 && ix < N, jv = jx >= 0 && jx < N;
            for (int row = 0; row < 2; row++) {
                const float r = row == 0 ? rx : ry;
                const float w = mask * weight[n * 2 + row];
                float Jz, Ji[6], Jj[6];
                if (row == 0) {
                    Jz = fx * (tij[0] * d - tij[2] * (X * d2));
                    const float J[6] = {fx * Wh * d, 0, fx * -X * Wh * d2, fx * -X * Y * d2, fx * (1 + X * X * d2), fx * -Y * d};
                    memcpy(Jj, J, sizeof J);
                } else {
                    Jz = fy * (tij[1] * d - tij[2] * (Y * d2));
                    const float J[6] = {0, fy * Wh * d, fy * -Y * Wh * d2, fy * (-1 - Y * Y * d2), fy * (X * Y * d2), fy * X * d};
                    memcpy(Jj, J, sizeof J);
                }
                adjSE3f(tij, qij, Jj, Ji);
                for (int a = 0; a < 6; a++)
                for (int b = 0; b < 6; b++) {
                    if (iv) Bm[(6 * ix + a) * n6 + 6 * ix + b] += w * Ji[a] * Ji[b];
                    if (jv) Bm[(6 * jx + a) * n6 + 6 * jx + b] += w * Jj[a] * Jj[b];
                    if (iv && jv) {
                        Bm[(6 * ix + a) * n6 + 6 * jx + b] += -w * Ji[a] * Jj[b];
                        Bm[(6 * jx + a) * n6 + 6 * ix + b] += -w * Jj[a] * Ji[b];
                    }
                }
                for (int a = 0; a < 6; a++) {
                    if (iv) Em[(6 * ix + a) * Mu + k] += -w * Jz * Ji[a];
                    if (jv) Em[(6 * jx + a) * Mu + k] += w * Jz * Jj[a];
                }
                for (int a = 0; a < 6; a++) {
                    if (iv) v[6 * ix + a] += -w * r * Ji[a];
                    if (jv) v[6 * jx + a] += w * r * Jj[a];
                }
                Cv[k] += w * Jz * Jz;
                u[k] += w * r * Jz;
            }
        }

        for (int64_t k = 0; k < Mu; k++) Q[k] = 1.0f / (Cv[k] + lmbda);

        if (N == 0) {
            for (int64_t k = 0; k < Mu; k++) dZ[k] = Q[k] * u[k];
        } else {
            /* S = B - (E Q) E^T, y = v - (E Q) u (ba_cuda.cu:510-515), summed
             * over patches k in ascending order as the dense loop does, but
             * visiting only each patch's nonzero E rows (the skipped products
             * are exact zeros, so every sum is the dense loop's) */
            memset(S, 0, sizeof(double) * n6 * n6);
            memset(y, 0, sizeof(double) * n6);
            for (int64_t k = 0; k < Mu; k++) {
                int nr = 0;
                for (int a = 0; a < n6; a++)
                    if (Em[a * Mu + k] != 0.0f) rows[nr++] = a;
                for (int i = 0; i < nr; i++) {
                    const int a = rows[i];
                    const double ea = (double)(Em[a * Mu + k] * Q[k]);
                    for (int j = 0; j < nr; j++) S[a * n6 + rows[j]] += ea * Em[rows[j] * Mu + k];
                    y[a] += ea * u[k];
                }
            }
            for (int a = 0; a < n6; a++) {
                for (int b = 0; b < n6; b++) S[a * n6 + b] = (double)Bm[a * n6 + b] - S[a * n6 + b];
                y[a] = (double)v[a] - y[a];
            }
            for (int a = 0; a < n6; a++) S[a * n6 + a] += 1e-4 * S[a * n6 + a] + 1.0;
            const int info = cholesky_d(S, n6);
            if (info) { status = info; break; }
            /* forward / back substitution: L L^T dX = y */
            for (int a = 0; a < n6; a++) {
                double t = y[a];
                for (int b = 0; b < a; b++) t -= S[a * n6 + b] * y[b];
                y[a] = t / S[a * n6 + a];
            }
            for (int a = n6 - 1; a >= 0; a--) {
                double t = y[a];
                for (int b = a + 1; b < n6; b++) t -= S[b * n6 + a] * y[b];
                y[a] = t / S[a * n6 + a];
            }
            for (int a = 0; a < n6; a++) dX[a] = (float)y[a];
            for (int64_t k = 0; k < Mu; k++) {
                double s = 0.0;
                for (int a = 0; a < n6; a++) s += (double)Em[a * Mu + k] * dX[a];
                dZ[k] = Q[k] * (float)((double)u[k] - s);
            }
            for (int i = 0; i < N; i++) {
                float* pt = poses + (int64_t)(t0 + i) * 7;
                const float tt[3] = {pt[0], pt[1], pt[2]}, qq[4] = {pt[3], pt[4], pt[5], pt[6]};
                float t1o[3], q1o[4];
                retrSE3f(dX + 6 * i, tt, qq, t1o, q1o);
                pt[0] = t1o[0]; pt[1] = t1o[1]; pt[2] = t1o[2];
                pt[3] = q1o[0]; pt[4] = q1o[1]; pt[5] = q1o[2]; pt[6] = q1o[3];
            }
        }
        /* patch_retr_kernel, ba_cuda.cu:191-211 */
        for (int64_t n = 0; n < Mu; n++) {
            float* pd = patches + (kx[n] * 3 + 2) * PP;
            float dd = pd[0] + dZ[n];
            dd = (dd > 20) ? 1.0f : dd;
            dd = dd > 1e-4f ? dd : (float)1e-4;
            for (int64_t q = 0; q < PP; q++) pd[q] = dd;
        }
    }
    free(Bm); free(Em); free(Cv); free(v); free(u); free(S); free(y); free(dX); free(dZ); free(Q); free(rows);
    free(kx); free(ku);
    return status;
}

/* fastba.reproject (ba_cuda.cu:368-418): coords [E][2][P][P], no Z clamp */
int oracle_reproject(const float* poses, const float* patches, const float* intrinsics, const int64_t* ii,
                     const int64_t* jj, const int64_t* kk, int64_t E, int P, float* coords)
{
    const float fx = intrinsics[0], fy = intrinsics[1], cx = intrinsics[2], cy = intrinsics[3];
    const int64_t PP = (int64_t)P * P;
    for (int64_t n = 0; n < E; n++) {
        const int64_t ix = ii[n], jx = jj[n], kxn = kk[n];
        const float ti[3] = {poses[ix * 7 + 0], poses[ix * 7 + 1], poses[ix * 7 + 2]};
        const float tj[3] = {poses[jx * 7 + 0], poses[jx * 7 + 1], poses[jx * 7 + 2]};
        const float qi[4] = {poses[ix * 7 + 3], poses[ix * 7 + 4], poses[ix * 7 + 5], poses[ix * 7 + 6]};
        const float qj[4] = {poses[jx * 7 + 3], poses[jx * 7 + 4], poses[jx * 7 + 5], poses[jx * 7 + 6]};
        float tij[3], qij[4], Xi[4], Xj[4];
        relSE3f(ti, qi, tj, qj, tij, qij);
        for (int64_t p = 0; p < PP; p++) {
            Xi[0] = (patches[(kxn * 3 + 0) * PP + p] - cx) / fx;
            Xi[1] = (patches[(kxn * 3 + 1) * PP + p] - cy) / fy;
            Xi[2] = 1.0f;
            Xi[3] = patches[(kxn * 3 + 2) * PP + p];
            actSE3f(tij, qij, Xi, Xj);
            coords[(n * 2 + 0) * PP + p] = fx * (Xj[0] / Xj[2]) + cx;
            coords[(n * 2 + 1) * PP + p] = fy * (Xj[1] / Xj[2]) + cy;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* lietorch SO3 / SE3 in double (so3.h, se3.h)                          */
/* ------------------------------------------------------------------ */
#define LIE_EPS 1e-6
#define LIE_PI 3.14159265358979323846

typedef struct { double x, y, z, w; } quat;

static quat q_load(const double* d) /* SO3(const Scalar*) normalises */
{
    quat q = {d[0], d[1], d[2], d[3]};
    const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    if (n > 0) { q.x /= n; q.y /= n; q.z /= n; q.w /= n; }
    return q;
}
static quat q_norm(quat q)
{
    const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    if (n > 0) { q.x /= n; q.y /= n; q.z /= n; q.w /= n; }
    return q;
}
static quat q_mul(quat a, quat b) /* Eigen quaternion product */
{
    quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}
static quat q_conj(quat q) { quat r = {-q.x, -q.y, -q.z, q.w}; return r; }
static void q_act(quat q, const double* p, double* o) /* so3.h:67-72 */
{
    double uv[3] = {q.y * p[2] - q.z * p[1], q.z * p[0] - q.x * p[2], q.x * p[1] - q.y * p[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    o[0] = p[0] + q.w * uv[0] + (q.y * uv[2] - q.z * uv[1]);
    o[1] = p[1] + q.w * uv[1] + (q.z * uv[0] - q.x * uv[2]);
    o[2] = p[2] + q.w * uv[2] + (q.x * uv[1] - q.y * uv[0]);
}
static void q_mat(quat q, double* R) /* Eigen toRotationMatrix, row-major 3x3 */
{
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
static void hat3(const double* p, double* M)
{
    M[0] = 0; M[1] = -p[2]; M[2] = p[1];
    M[3] = p[2]; M[4] = 0; M[5] = -p[0];
    M[6] = -p[1]; M[7] = p[0]; M[8] = 0;
}
static void mm3(const double* A, const double* B, double* C)
{
    double T[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
    memcpy(C, T, sizeof T);
}
static quat so3_exp(const double* phi) /* so3.h:165-182 */
{
    const double theta2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2], theta = sqrt(theta2);
    double imag, real;
    if (theta < LIE_EPS) {
        const double theta4 = theta2 * theta2;
        imag = 0.5 - (1.0 / 48.0) * theta2 + (1.0 / 3840.0) * theta4;
        real = 1.0 - (1.0 / 8.0) * theta2 + (1.0 / 384.0) * theta4;
    } else {
        imag = sin(0.5 * theta) / theta;
        real = cos(0.5 * theta);
    }
    quat q = {imag * phi[0], imag * phi[1], imag * phi[2], real};
    return q_norm(q);
}
static void so3_log(quat q, double* phi) /* so3.h:127-163 */
{
    const double sn = q.x * q.x + q.y * q.y + q.z * q.z, w = q.w;
    double f;
    if (sn < LIE_EPS * LIE_EPS) {
        f = 2.0 / w - (2.0 / 3.0) * sn / (w * w * w);
    } else {
        const double n = sqrt(sn);
        if (fabs(w) < LIE_EPS) f = (w > 0 ? LIE_PI : -LIE_PI) / n;
        else f = 2.0 * atan(n / w) / n;
    }
    phi[0] = f * q.x; phi[1] = f * q.y; phi[2] = f * q.z;
}
static void so3_left_jacobian(const double* phi, double* J) /* so3.h:184-202 */
{
    double Ph[9], Ph2[9];
    hat3(phi, Ph);
    mm3(Ph, Ph, Ph2);
    const double t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2], t = sqrt(t2);
    const double c1 = t < LIE_EPS ? 0.5 - (1.0 / 24.0) * t2 : (1.0 - cos(t)) / t2;
    const double c2 = t < LIE_EPS ? 1.0 / 6.0 - (1.0 / 120.0) * t2 : (t - sin(t)) / (t2 * t);
    for (int i = 0; i < 9; i++) J[i] = (i % 4 == 0 ? 1.0 : 0.0) + c1 * Ph[i] + c2 * Ph2[i];
}
static void so3_left_jacobian_inverse(const double* phi, double* J) /* so3.h:204-220 */
{
    double Ph[9], Ph2[9];
    hat3(phi, Ph);
    mm3(Ph, Ph, Ph2);
    const double t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2], t = sqrt(t2), ht = 0.5 * t;
    const double c2 = t < LIE_EPS ? 1.0 / 12.0 : (1.0 - t * cos(ht) / (2.0 * sin(ht))) / (t * t);
    for (int i = 0; i < 9; i++) J[i] = (i % 4 == 0 ? 1.0 : 0.0) - 0.5 * Ph[i] + c2 * Ph2[i];
}
static void se3_calcQ(const double* xi, double* Qm) /* se3.h:385-414 */
{
    double Ta[9], Ph[9], A[9], Bm[9], Cm[9], T1[9], T2[9];
    hat3(xi, Ta);
    hat3(xi + 3, Ph);
    const double t = sqrt(xi[3] * xi[3] + xi[4] * xi[4] + xi[5] * xi[5]), t2 = t * t, t4 = t2 * t2;
    const double c1 = t < LIE_EPS ? 1.0 / 6.0 - (1.0 / 120.0) * t2 : (t - sin(t)) / (t2 * t);
    const double c2 = t < LIE_EPS ? 1.0 / 24.0 - (1.0 / 720.0) * t2 : (t2 + 2 * cos(t) - 2) / (2 * t4);
    const double c3 = t < LIE_EPS ? 1.0 / 120.0 - (1.0 / 2520.0) * t2 : (2 * t - 3 * sin(t) + t * cos(t)) / (2 * t4 * t);
    /* A = Ph*Ta + Ta*Ph + Ph*Ta*Ph */
    mm3(Ph, Ta, T1); mm3(Ta, Ph, T2); mm3(T1, Ph, Cm);
    for (int i = 0; i < 9; i++) A[i] = T1[i] + T2[i] + Cm[i];
    /* B = Ph*Ph*Ta + Ta*Ph*Ph - 3*Ph*Ta*Ph */
    double PP2[9], PPT[9], TPP[9];
    mm3(Ph, Ph, PP2); mm3(PP2, Ta, PPT); mm3(Ta, PP2, TPP);
    for (int i = 0; i < 9; i++) Bm[i] = PPT[i] + TPP[i] - 3 * Cm[i];
    /* C = Ph*Ta*Ph*Ph + Ph*Ph*Ta*Ph */
    double X1[9], X2[9];
    mm3(Cm, Ph, X1); mm3(PPT, Ph, X2);
    for (int i = 0; i < 9; i++) Qm[i] = 0.5 * Ta[i] + c1 * A[i] + c2 * Bm[i] + c3 * (X1[i] + X2[i]);
}

/* group ids as dispatch.h:16-31 */
enum { G_SO3 = 1, G_RXSO3 = 2, G_SE3 = 3, G_SIM3 = 4 };
enum { OP_EXP = 0, OP_LOG, OP_INV, OP_MUL, OP_ADJ, OP_ADJT, OP_ACT, OP_ACT4, OP_MATRIX, OP_PROJECTOR, OP_JINV };

typedef struct { quat q; double t[3]; } se3;
static se3 se3_load(const double* d)
{
    se3 g;
    g.t[0] = d[0]; g.t[1] = d[1]; g.t[2] = d[2];
    g.q = q_load(d + 3);
    return g;
}
static void se3_store(se3 g, double* d)
{
    d[0] = g.t[0]; d[1] = g.t[1]; d[2] = g.t[2];
    d[3] = g.q.x; d[4] = g.q.y; d[5] = g.q.z; d[6] = g.q.w;
}
static void se3_adj_matrix(se3 g, double* Ad) /* se3.h:299-308, row-major 6x6 */
{
    double R[9], tx[9], tR[9];
    q_mat(g.q, R);
    hat3(g.t, tx);
    mm3(tx, R, tR);
    memset(Ad, 0, sizeof(double) * 36);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            Ad[i * 6 + j] = R[i * 3 + j];
            Ad[i * 6 + 3 + j] = tR[i * 3 + j];
            Ad[(3 + i) * 6 + 3 + j] = R[i * 3 + j];
        }
}
static void se3_log(se3 g, double* xi)
{
    double phi[3], Vinv[9];
    so3_log(g.q, phi);
    so3_left_jacobian_inverse(phi, Vinv);
    for (int i = 0; i < 3; i++) xi[i] = Vinv[i * 3] * g.t[0] + Vinv[i * 3 + 1] * g.t[1] + Vinv[i * 3 + 2] * g.t[2];
    xi[3] = phi[0]; xi[4] = phi[1]; xi[5] = phi[2];
}


/* ------------------------------------------------------------------ */
/* RxSO3 [qx qy qz qw s] and Sim3 [t q s] in double (rxso3.h, sim3.h)   */
/* ------------------------------------------------------------------ */
typedef struct { quat q; double s; } rxso3;
typedef struct { rxso3 r; double t[3]; } sim3;

static rxso3 rx_load(const double* d) { rxso3 g; g.q = q_load(d); g.s = d[4]; return g; }
static void rx_store(rxso3 g, double* d) { d[0] = g.q.x; d[1] = g.q.y; d[2] = g.q.z; d[3] = g.q.w; d[4] = g.s; }
static rxso3 rx_inv(rxso3 g) { rxso3 h; h.q = q_norm(q_conj(g.q)); h.s = 1.0 / g.s; return h; }
static rxso3 rx_mul(rxso3 a, rxso3 b) { rxso3 c; c.q = q_norm(q_mul(a.q, b.q)); c.s = a.s * b.s; return c; }
static void rx_act(rxso3 g, const double* p, double* o) /* s (R p) */
{
    q_act(g.q, p, o);
    o[0] *= g.s; o[1] *= g.s; o[2] *= g.s;
}
static void rx_log(rxso3 g, double* ps) { so3_log(g.q, ps); ps[3] = log(g.s); }
static rxso3 rx_exp(const double* ps) { rxso3 g; g.q = so3_exp(ps); g.s = exp(ps[3]); return g; }
static void rx_calcW(const double* ps, double* W) /* rxso3.h calcW, row-major 3x3 */
{
    double Ph[9], Ph2[9];
    hat3(ps, Ph);
    mm3(Ph, Ph, Ph2);
    const double sigma = ps[3], theta = sqrt(ps[0] * ps[0] + ps[1] * ps[1] + ps[2] * ps[2]), sc = exp(sigma);
    double A, B, C;
    if (fabs(sigma) < LIE_EPS) {
        C = 1.0;
        if (fabs(theta) < LIE_EPS) { A = 0.5; B = 1.0 / 6.0; }
        else { A = (1.0 - cos(theta)) / (theta * theta); B = (theta - sin(theta)) / (theta * theta * theta); }
    } else {
        C = (sc - 1.0) / sigma;
        if (fabs(theta) < LIE_EPS) {
            const double s2 = sigma * sigma;
            A = ((sigma - 1.0) * sc + 1.0) / s2;
            B = (sc * 0.5 * s2 + sc - 1.0 - sigma * sc) / (s2 * sigma);
        } else {
            const double t2 = theta * theta, a = sc * sin(theta), b = sc * cos(theta), c = t2 + sigma * sigma;
            A = (a * sigma + (1.0 - b) * theta) / (theta * c);
            B = (C - ((b - 1.0) * sigma + a * theta) / c) / t2;
        }
    }
    for (int i = 0; i < 9; i++) W[i] = A * Ph[i] + B * Ph2[i] + (i % 4 == 0 ? C : 0.0);
}
static void inv3d(const double* A, double* B) /* adjugate / determinant */
{
    const double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8], c02 = A[3] * A[7] - A[4] * A[6];
    const double det = A[0] * c00 + A[1] * c01 + A[2] * c02, id = 1.0 / det;
    B[0] = c00 * id; B[1] = (A[2] * A[7] - A[1] * A[8]) * id; B[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    B[3] = c01 * id; B[4] = (A[0] * A[8] - A[2] * A[6]) * id; B[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    B[6] = c02 * id; B[7] = (A[1] * A[6] - A[0] * A[7]) * id; B[8] = (A[0] * A[4] - A[1] * A[3]) * id;
}
static sim3 sim3_load(const double* d) { sim3 g; g.t[0] = d[0]; g.t[1] = d[1]; g.t[2] = d[2]; g.r = rx_load(d + 3); return g; }
static void sim3_store(sim3 g, double* d) { d[0] = g.t[0]; d[1] = g.t[1]; d[2] = g.t[2]; rx_store(g.r, d + 3); }
static void sim3_log(sim3 g, double* xi) /* [W^-1 t, phi, sigma] */
{
    double W[9], Wi[9];
    rx_log(g.r, xi + 3);
    rx_calcW(xi + 3, W);
    inv3d(W, Wi);
    for (int i = 0; i < 3; i++) xi[i] = Wi[i * 3] * g.t[0] + Wi[i * 3 + 1] * g.t[1] + Wi[i * 3 + 2] * g.t[2];
}
static void sim3_adj_matrix(sim3 g, double* Ad) /* sim3.h Adj, row-major 7x7 */
{
    double R[9], tx[9], tR[9];
    q_mat(g.r.q, R);
    hat3(g.t, tx);
    mm3(tx, R, tR);
    memset(Ad, 0, sizeof(double) * 49);
    for (int i = 0; i < 7; i++) Ad[i * 7 + i] = 1;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) {
            Ad[i * 7 + j] = g.r.s * R[i * 3 + j];
            Ad[i * 7 + 3 + j] = tR[i * 3 + j];
            Ad[(3 + i) * 7 + 3 + j] = R[i * 3 + j];
        }
        Ad[i * 7 + 6] = -g.t[i];
    }
}
static void sim3_ad(const double* a, double* A) /* sim3.h adj */
{
    double Ta[9], Ph[9];
    hat3(a, Ta);
    hat3(a + 3, Ph);
    memset(A, 0, sizeof(double) * 49);
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) {
            A[i * 7 + j] = Ph[i * 3 + j] + (i == j ? a[6] : 0.0);
            A[i * 7 + 3 + j] = Ta[i * 3 + j];
            A[(3 + i) * 7 + 3 + j] = Ph[i * 3 + j];
        }
        A[i * 7 + 6] = -a[i];
    }
}
static void mm7(const double* A, const double* B, double* C)
{
    double T[49];
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) {
            double s = 0;
            for (int k = 0; k < 7; k++) s += A[i * 7 + k] * B[k * 7 + j];
            T[i * 7 + j] = s;
        }
    memcpy(C, T, sizeof T);
}
static void sim3_left_jacobian_inverse(const double* xi, double* J) /* I - X/2 + X^2/12 - X^4/720 */
{
    double X[49], X2[49], X4[49];
    sim3_ad(xi, X);
    mm7(X, X, X2);
    mm7(X2, X2, X4);
    for (int i = 0; i < 49; i++) J[i] = (i % 8 == 0 ? 1.0 : 0.0) - 0.5 * X[i] + X2[i] / 12.0 - X4[i] / 720.0;
}

static int lie_forward_scaled(int op, int group, const double* X, const double* Y, double* out, int64_t n)
{
    for (int64_t i = 0; i < n; i++) {
        if (group == G_RXSO3) {
            const double* x = X + i * 5;
            switch (op) {
            case OP_EXP: rx_store(rx_exp(X + i * 4), out + i * 5); break;
            case OP_LOG: rx_log(rx_load(x), out + i * 4); break;
            case OP_INV: rx_store(rx_inv(rx_load(x)), out + i * 5); break;
            case OP_MUL: rx_store(rx_mul(rx_load(x), rx_load(Y + i * 5)), out + i * 5); break;
            case OP_ADJ: case OP_ADJT: { /* Adj = diag(R, 1) */
                double R[9]; q_mat(rx_load(x).q, R);
                const double* a = Y + i * 4; double* o = out + i * 4;
                for (int r = 0; r < 3; r++) o[r] = op == OP_ADJ ? R[r * 3] * a[0] + R[r * 3 + 1] * a[1] + R[r * 3 + 2] * a[2]
                                                           : R[r] * a[0] + R[3 + r] * a[1] + R[6 + r] * a[2];
                o[3] = a[3];
                break;
            }
            case OP_ACT: rx_act(rx_load(x), Y + i * 3, out + i * 3); break;
            case OP_ACT4: rx_act(rx_load(x), Y + i * 4, out + i * 4); out[i * 4 + 3] = Y[i * 4 + 3]; break;
            case OP_MATRIX: {
                rxso3 g = rx_load(x); double R[9]; q_mat(g.q, R); double* o = out + i * 16;
                memset(o, 0, sizeof(double) * 16);
                for (int r = 0; r < 3; r++) for (int cc = 0; cc < 3; cc++) o[r * 4 + cc] = g.s * R[r * 3 + cc];
                o[15] = 1; break;
            }
            case OP_PROJECTOR: { /* rxso3.h orthogonal_projector, 5x5 */
                rxso3 g = rx_load(x); double* o = out + i * 25; memset(o, 0, sizeof(double) * 25);
                const double v[3] = {-g.q.x, -g.q.y, -g.q.z}; double H[9]; hat3(v, H);
                for (int r = 0; r < 3; r++) for (int cc = 0; cc < 3; cc++) o[r * 5 + cc] = 0.5 * ((r == cc ? g.q.w : 0) + H[r * 3 + cc]);
                for (int cc = 0; cc < 3; cc++) o[3 * 5 + cc] = 0.5 * v[cc];
                o[4 * 5 + 3] = g.s;
                break;
            }
            case OP_JINV: { /* diag(so3 Jl^-1, 1) at Log(X) */
                double ps[4], J[9]; rx_log(rx_load(x), ps); so3_left_jacobian_inverse(ps, J);
                const double* a = Y + i * 4; double* o = out + i * 4;
                for (int r = 0; r < 3; r++) o[r] = J[r * 3] * a[0] + J[r * 3 + 1] * a[1] + J[r * 3 + 2] * a[2];
                o[3] = a[3];
                break;
            }
            default: return -1;
            }
        } else {
            const double* x = X + i * 8;
            switch (op) {
            case OP_EXP: {
                const double* xi = X + i * 7; sim3 g; double W[9];
                g.r = rx_exp(xi + 3); rx_calcW(xi + 3, W);
                for (int r = 0; r < 3; r++) g.t[r] = W[r * 3] * xi[0] + W[r * 3 + 1] * xi[1] + W[r * 3 + 2] * xi[2];
                sim3_store(g, out + i * 8); break;
            }
            case OP_LOG: sim3_log(sim3_load(x), out + i * 7); break;
            case OP_INV: {
                sim3 g = sim3_load(x), h; double tt[3]; h.r = rx_inv(g.r); rx_act(h.r, g.t, tt);
                h.t[0] = -tt[0]; h.t[1] = -tt[1]; h.t[2] = -tt[2];
                sim3_store(h, out + i * 8); break;
            }
            case OP_MUL: {
                sim3 a = sim3_load(x), b = sim3_load(Y + i * 8), c; double tt[3];
                c.r = rx_mul(a.r, b.r); rx_act(a.r, b.t, tt);
                c.t[0] = a.t[0] + tt[0]; c.t[1] = a.t[1] + tt[1]; c.t[2] = a.t[2] + tt[2];
                sim3_store(c, out + i * 8); break;
            }
            case OP_ADJ: case OP_ADJT: {
                double Ad[49]; sim3_adj_matrix(sim3_load(x), Ad);
                const double* a = Y + i * 7; double* o = out + i * 7;
                for (int r = 0; r < 7; r++) {
                    double sum = 0; for (int cc = 0; cc < 7; cc++) sum += (op == OP_ADJ ? Ad[r * 7 + cc] : Ad[cc * 7 + r]) * a[cc];
                    o[r] = sum;
                }
                break;
            }
            case OP_ACT: { sim3 g = sim3_load(x); double* o = out + i * 3; rx_act(g.r, Y + i * 3, o); o[0] += g.t[0]; o[1] += g.t[1]; o[2] += g.t[2]; break; }
            case OP_ACT4: {
                sim3 g = sim3_load(x); const double* p = Y + i * 4; double* o = out + i * 4; rx_act(g.r, p, o);
                o[0] += p[3] * g.t[0]; o[1] += p[3] * g.t[1]; o[2] += p[3] * g.t[2]; o[3] = p[3]; break;
            }
            case OP_MATRIX: {
                sim3 g = sim3_load(x); double R[9]; q_mat(g.r.q, R); double* o = out + i * 16; memset(o, 0, sizeof(double) * 16);
                for (int r = 0; r < 3; r++) { for (int cc = 0; cc < 3; cc++) o[r * 4 + cc] = g.r.s * R[r * 3 + cc]; o[r * 4 + 3] = g.t[r]; }
                o[15] = 1; break;
            }
            case OP_PROJECTOR: { /* sim3.h orthogonal_projector, 8x8 */
                sim3 g = sim3_load(x); double* o = out + i * 64; memset(o, 0, sizeof(double) * 64);
                const double mt[3] = {-g.t[0], -g.t[1], -g.t[2]}; double H[9]; hat3(mt, H);
                for (int r = 0; r < 3; r++) {
                    o[r * 8 + r] = 1;
                    for (int cc = 0; cc < 3; cc++) o[r * 8 + 3 + cc] = H[r * 3 + cc];
                    o[r * 8 + 6] = g.t[r];
                }
                const double v[3] = {-g.r.q.x, -g.r.q.y, -g.r.q.z}; double Hq[9]; hat3(v, Hq);
                for (int r = 0; r < 3; r++) for (int cc = 0; cc < 3; cc++) o[(3 + r) * 8 + 3 + cc] = 0.5 * ((r == cc ? g.r.q.w : 0) + Hq[r * 3 + cc]);
                for (int cc = 0; cc < 3; cc++) o[6 * 8 + 3 + cc] = 0.5 * v[cc];
                o[7 * 8 + 6] = g.r.s;
                break;
            }
            case OP_JINV: {
                double xi[7], J[49]; sim3_log(sim3_load(x), xi); sim3_left_jacobian_inverse(xi, J);
                const double* a = Y + i * 7; double* o = out + i * 7;
                for (int r = 0; r < 7; r++) { double sum = 0; for (int cc = 0; cc < 7; cc++) sum += J[r * 7 + cc] * a[cc]; o[r] = sum; }
                break;
            }
            default: return -1;
            }
        }
    }
    return 0;
}

/*
 * Forward group operators on flat [n][dim] double arrays (lietorch.cpp:18-283
 * semantics; inputs already broadcast).  RxSO3 / Sim3 go to
 * lie_forward_scaled (rxso3.h / sim3.h).
 * Returns 0, or -1 for an unsupported (group, op).
 */
int oracle_lie_forward(int op, int group, const double* X, const double* Y, double* out, int64_t n)
{
    if (group == G_RXSO3 || group == G_SIM3) return lie_forward_scaled(op, group, X, Y, out, n);
    if (group != G_SO3 && group != G_SE3) return -1;
    for (int64_t i = 0; i < n; i++) {
        if (group == G_SO3) {
            const double* x = X + i * 4;
            switch (op) {
            case OP_EXP: { quat q = so3_exp(X + i * 3); double* o = out + i * 4; o[0] = q.x; o[1] = q.y; o[2] = q.z; o[3] = q.w; break; }
            case OP_LOG: so3_log(q_load(x), out + i * 3); break;
            case OP_INV: { quat q = q_norm(q_conj(q_load(x))); double* o = out + i * 4; o[0] = q.x; o[1] = q.y; o[2] = q.z; o[3] = q.w; break; }
            case OP_MUL: { quat q = q_norm(q_mul(q_load(x), q_load(Y + i * 4))); double* o = out + i * 4; o[0] = q.x; o[1] = q.y; o[2] = q.z; o[3] = q.w; break; }
            case OP_ADJ: case OP_ADJT: {
                double R[9]; q_mat(q_load(x), R);
                const double* a = Y + i * 3; double* o = out + i * 3;
                for (int r = 0; r < 3; r++) o[r] = op == OP_ADJ ? R[r * 3] * a[0] + R[r * 3 + 1] * a[1] + R[r * 3 + 2] * a[2]
                                                           : R[r] * a[0] + R[3 + r] * a[1] + R[6 + r] * a[2];
                break;
            }
            case OP_ACT: q_act(q_load(x), Y + i * 3, out + i * 3); break;
            case OP_ACT4: q_act(q_load(x), Y + i * 4, out + i * 4); out[i * 4 + 3] = Y[i * 4 + 3]; break;
            case OP_MATRIX: {
                double R[9]; q_mat(q_load(x), R); double* o = out + i * 16;
                memset(o, 0, sizeof(double) * 16);
                for (int r = 0; r < 3; r++) for (int cc = 0; cc < 3; cc++) o[r * 4 + cc] = R[r * 3 + cc];
                o[15] = 1; break;
            }
            case OP_PROJECTOR: { /* so3.h:93-103 */
                quat q = q_load(x); double* o = out + i * 16; memset(o, 0, sizeof(double) * 16);
                const double v[3] = {-q.x, -q.y, -q.z}; double H[9]; hat3(v, H);
                for (int r = 0; r < 3; r++) for (int cc = 0; cc < 3; cc++) o[r * 4 + cc] = 0.5 * ((r == cc ? q.w : 0) + H[r * 3 + cc]);
                for (int cc = 0; cc < 3; cc++) o[12 + cc] = 0.5 * v[cc];
                break;
            }
            case OP_JINV: {
                double phi[3], J[9]; so3_log(q_load(x), phi); so3_left_jacobian_inverse(phi, J);
                const double* a = Y + i * 3; double* o = out + i * 3;
                for (int r = 0; r < 3; r++) o[r] = J[r * 3] * a[0] + J[r * 3 + 1] * a[1] + J[r * 3 + 2] * a[2];
                break;
            }
            default: return -1;
            }
        } else {
            const double* x = X + i * 7;
            switch (op) {
            case OP_EXP: { /* se3.h:375-383 */
                const double* xi = X + i * 6; se3 g; double J[9];
                g.q = so3_exp(xi + 3); so3_left_jacobian(xi + 3, J);
                for (int r = 0; r < 3; r++) g.t[r] = J[r * 3] * xi[0] + J[r * 3 + 1] * xi[1] + J[r * 3 + 2] * xi[2];
                se3_store(g, out + i * 7); break;
            }
            case OP_LOG: se3_log(se3_load(x), out + i * 6); break;
            case OP_INV: { /* se3.h:277-279 */
                se3 g = se3_load(x), h; h.q = q_norm(q_conj(g.q));
                double tt[3]; q_act(h.q, g.t, tt); h.t[0] = -tt[0]; h.t[1] = -tt[1]; h.t[2] = -tt[2];
                se3_store(h, out + i * 7); break;
            }
            case OP_MUL: { /* se3.h:286-288 */
                se3 a = se3_load(x), b = se3_load(Y + i * 7), c; double tt[3];
                c.q = q_norm(q_mul(a.q, b.q)); q_act(a.q, b.t, tt);
                c.t[0] = a.t[0] + tt[0]; c.t[1] = a.t[1] + tt[1]; c.t[2] = a.t[2] + tt[2];
                se3_store(c, out + i * 7); break;
            }
            case OP_ADJ: case OP_ADJT: {
                double Ad[36]; se3_adj_matrix(se3_load(x), Ad);
                const double* a = Y + i * 6; double* o = out + i * 6;
                for (int r = 0; r < 6; r++) {
                    double s = 0; for (int cc = 0; cc < 6; cc++) s += (op == OP_ADJ ? Ad[r * 6 + cc] : Ad[cc * 6 + r]) * a[cc];
                    o[r] = s;
                }
                break;
            }
            case OP_ACT: { se3 g = se3_load(x); double* o = out + i * 3; q_act(g.q, Y + i * 3, o); o[0] += g.t[0]; o[1] += g.t[1]; o[2] += g.t[2]; break; }
            case OP_ACT4: { /* se3.h:294-297 */
                se3 g = se3_load(x); const double* p = Y + i * 4; double* o = out + i * 4; q_act(g.q, p, o);
                o[0] += g.t[0] * p[3]; o[1] += g.t[1] * p[3]; o[2] += g.t[2] * p[3]; o[3] = p[3]; break;
            }
            case OP_MATRIX: {
                se3 g = se3_load(x); double R[9]; q_mat(g.q, R); double* o = out + i * 16; memset(o, 0, sizeof(double) * 16);
                for (int r = 0; r < 3; r++) { for (int cc = 0; cc < 3; cc++) o[r * 4 + cc] = R[r * 3 + cc]; o[r * 4 + 3] = g.t[r]; }
                o[15] = 1; break;
            }
            case OP_PROJECTOR: { /* se3.h:355-363 */
                se3 g = se3_load(x); double* o = out + i * 49; memset(o, 0, sizeof(double) * 49);
                const double mt[3] = {-g.t[0], -g.t[1], -g.t[2]}; double H[9]; hat3(mt, H);
                for (int r = 0; r < 3; r++) { o[r * 7 + r] = 1; for (int cc = 0; cc < 3; cc++) o[r * 7 + 3 + cc] = H[r * 3 + cc]; }
                const double v[3] = {-g.q.x, -g.q.y, -g.q.z}; double Hq[9]; hat3(v, Hq);
                for (int r = 0; r < 3; r++) for (int cc = 0; cc < 3; cc++) o[(3 + r) * 7 + 3 + cc] = 0.5 * ((r == cc ? g.q.w : 0) + Hq[r * 3 + cc]);
                for (int cc = 0; cc < 3; cc++) o[6 * 7 + 3 + cc] = 0.5 * v[cc];
                break;
            }
            case OP_JINV: { /* se3.h:429-442 applied to Log(X) */
                double xi[6], Ji[9], Qm[9], T[9], JQJ[9];
                se3_log(se3_load(x), xi); so3_left_jacobian_inverse(xi + 3, Ji); se3_calcQ(xi, Qm);
                mm3(Ji, Qm, T); mm3(T, Ji, JQJ);
                const double* a = Y + i * 6; double* o = out + i * 6;
                for (int r = 0; r < 3; r++) {
                    o[r] = 0; o[3 + r] = 0;
                    for (int cc = 0; cc < 3; cc++) {
                        o[r] += Ji[r * 3 + cc] * a[cc] - JQJ[r * 3 + cc] * a[3 + cc];
                        o[3 + r] += Ji[r * 3 + cc] * a[3 + cc];
                    }
                }
                break;
            }
            default: return -1;
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* projective_ops.transform / point_cloud (double geometry)             */
/* ------------------------------------------------------------------ */
/*
 * poses [*][7], patches [*][3][P][P], intrinsics [*][4] (per frame), all
 * double.  coords out [E][P][P][2 + depth]; valid out [E][P][P] (Z > 0.2)
 * when non-NULL.  Semantics of projective_ops.py:53-68 + proj :32-50.
 */
int oracle_transform(const double* poses, const double* patches, const double* intrinsics, const int64_t* ii,
                     const int64_t* jj, const int64_t* kk, int64_t E, int P, int depth, int tonly, double* coords,
                     double* valid)
{
    const int64_t PP = (int64_t)P * P;
    const int od = depth ? 3 : 2;
    for (int64_t e = 0; e < E; e++) {
        se3 gi = se3_load(poses + ii[e] * 7), gj = se3_load(poses + jj[e] * 7), giv, g;
        double tt[3];
        giv.q = q_norm(q_conj(gi.q));
        q_act(giv.q, gi.t, tt);
        giv.t[0] = -tt[0]; giv.t[1] = -tt[1]; giv.t[2] = -tt[2];
        g.q = q_norm(q_mul(gj.q, giv.q));
        q_act(gj.q, giv.t, tt);
        g.t[0] = gj.t[0] + tt[0]; g.t[1] = gj.t[1] + tt[1]; g.t[2] = gj.t[2] + tt[2];
        if (tonly) { g.q.x = 0; g.q.y = 0; g.q.z = 0; g.q.w = 1; }
        const double* ki = intrinsics + ii[e] * 4;
        const double* kj = intrinsics + jj[e] * 4;
        for (int64_t p = 0; p < PP; p++) {
            const double* pa = patches + kk[e] * 3 * PP;
            const double X0[4] = {(pa[p] - ki[2]) / ki[0], (pa[PP + p] - ki[3]) / ki[1], 1.0, pa[2 * PP + p]};
            double X1[3];
            q_act(g.q, X0, X1);
            X1[0] += g.t[0] * X0[3]; X1[1] += g.t[1] * X0[3]; X1[2] += g.t[2] * X0[3];
            const double Zc = X1[2] < 0.1 ? 0.1 : X1[2];
            const double d = 1.0 / Zc;
            double* o = coords + (e * PP + p) * od;
            o[0] = kj[0] * (d * X1[0]) + kj[2];
            o[1] = kj[1] * (d * X1[1]) + kj[3];
            if (depth) o[2] = d;
            if (valid) valid[e * PP + p] = X1[2] > 0.2 ? 1.0 : 0.0;
        }
    }
    return 0;
}

/* point_cloud centre pixel divided by w (dpvo/dpvo.py:747-749): out [m][3] */
int oracle_point_cloud_centre(const double* poses, const double* patches, const double* intrinsics,
                              const int64_t* ix, int64_t m, int P, double* out)
{
    const int64_t PP = (int64_t)P * P, c = (P / 2) * P + P / 2;
    for (int64_t k = 0; k < m; k++) {
        se3 g = se3_load(poses + ix[k] * 7), gi;
        double tt[3];
        gi.q = q_norm(q_conj(g.q));
        q_act(gi.q, g.t, tt);
        gi.t[0] = -tt[0]; gi.t[1] = -tt[1]; gi.t[2] = -tt[2];
        const double* in = intrinsics + ix[k] * 4;
        const double* pa = patches + k * 3 * PP;
        const double X0[4] = {(pa[c] - in[2]) / in[0], (pa[PP + c] - in[3]) / in[1], 1.0, pa[2 * PP + c]};
        double X1[3];
        q_act(gi.q, X0, X1);
        for (int r = 0; r < 3; r++) out[k * 3 + r] = (X1[r] + gi.t[r] * X0[3]) / X0[3];
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* neighbors (ba.cpp:113-158)                                           */
/* ------------------------------------------------------------------ */
typedef struct { int64_t key, sub, idx; } triple;
static int cmp_triple(const void* a, const void* b)
{
    const triple *x = (const triple*)a, *y = (const triple*)b;
    if (x->key != y->key) return (x->key > y->key) - (x->key < y->key);
    if (x->sub != y->sub) return (x->sub > y->sub) - (x->sub < y->sub);
    return (x->idx > y->idx) - (x->idx < y->idx); /* stable */
}
int oracle_neighbors(const int64_t* ii, const int64_t* jj, int64_t E, int64_t* ix, int64_t* jx)
{
    triple* t = (triple*)malloc(sizeof(triple) * (E > 0 ? E : 1));
    for (int64_t e = 0; e < E; e++) { t[e].key = ii[e]; t[e].sub = jj[e]; t[e].idx = e; }
    qsort(t, E, sizeof(triple), cmp_triple);
    for (int64_t s = 0; s < E; s++) {
        const int first = s == 0 || t[s - 1].key != t[s].key;
        const int last = s == E - 1 || t[s + 1].key != t[s].key;
        ix[t[s].idx] = first ? -1 : t[s - 1].idx;
        jx[t[s].idx] = last ? -1 : t[s + 1].idx;
    }
    free(t);
    return 0;
}

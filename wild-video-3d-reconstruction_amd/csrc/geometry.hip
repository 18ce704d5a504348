// geometry.hip -- fused projective ops of dpvo/projective_ops.py for gfx950,
// plus the library's runtime entry points (ABI version, error string).
//
// The reference composes transform() from ~30 ATen/lietorch launches and
// materialises E*9 broadcast pose copies (lietorch/broadcasting.py:21-29);
// here one thread handles one edge: Gij = poses[jj] * poses[ii]^-1 once, then
// the P*P patch pixels, with lietorch's normalise-on-load semantics.
#include <algorithm>
#include <string>

#include <mutex>
#include <set>

#include "common.hpp"
#include "liegroups.hpp"

namespace dpvo {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

using G3 = lie::SE3<float>;

// PC: the patch size as a compile-time constant (3, every tracker preset) or
// 0 for a run-time P.  The operands are __restrict__ (coords / valid never
// alias the inputs) and, with PC, every patch value and both intrinsics are
// loaded before the first store: the previous loop, with possible aliasing,
// reloaded them after each pixel's stores -- a dependent L2 round trip per
// pixel (17 us at C3).
template <int PC>
__global__ __launch_bounds__(256) void transform_kernel(const float* __restrict__ poses,
                                                       const float* __restrict__ patches, int P,
                                                       const float* __restrict__ intr, const int64_t* __restrict__ ii,
                                                       const int64_t* __restrict__ jj, const int64_t* __restrict__ kk,
                                                       int64_t E, int flags, float* __restrict__ coords,
                                                       float* __restrict__ valid)
{
    const bool depth = flags & DPVO_TF_DEPTH, tonly = flags & DPVO_TF_TONLY, chw = flags & DPVO_TF_CHW;
    const int od = depth ? 3 : 2;
    const int64_t PP = PC ? PC * PC : (int64_t)P * P;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = ii[e], j = jj[e], k = kk[e];   // (the three index loads together)
        __builtin_amdgcn_sched_barrier(0);
        const float* pa = patches + k * 3 * PP;
        // Gij = poses[jj] * poses[ii].inv()   (projective_ops.py:60); raw pose
        // words first (G3::load normalizes: arithmetic on the loaded values)
        float rj[7], ri[7];
#pragma unroll
        for (int t = 0; t < 7; t++) {
            rj[t] = poses[j * 7 + t];
            ri[t] = poses[i * 7 + t];
        }
        float ki[4], kj[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            ki[t] = intr[i * 4 + t];
            kj[t] = intr[j * 4 + t];
        }
        float pv[3][PC ? PC * PC : 1];
        if constexpr (PC > 0) {
#pragma unroll
            for (int c = 0; c < 3; c++)
#pragma unroll
                for (int q = 0; q < PC * PC; q++) pv[c][q] = pa[c * PC * PC + q];
        }
        __builtin_amdgcn_sched_barrier(0);   // (every operand load issued before the arithmetic)
        G3 g = G3::load(rj).mul(G3::load(ri).inv());
        if (tonly) { g.so3.q.x = 0.f; g.so3.q.y = 0.f; g.so3.q.z = 0.f; g.so3.q.w = 1.f; }
        auto pixel = [&](int64_t q, float px, float py, float pd) __attribute__((always_inline)) {
            // iproj (projective_ops.py:19-29)
            const float X0[4] = {(px - ki[2]) / ki[0], (py - ki[3]) / ki[1], 1.0f, pd};
            float X1[4];
            g.act4(X0, X1);
            // proj with Z clamped to >= 0.1 (projective_ops.py:32-50)
            const float d = 1.0f / fmaxf(X1[2], 0.1f);
            const float x = kj[0] * (d * X1[0]) + kj[2];
            const float y = kj[1] * (d * X1[1]) + kj[3];
            if (chw) {
                coords[(e * od + 0) * PP + q] = x;
                coords[(e * od + 1) * PP + q] = y;
                if (depth) coords[(e * od + 2) * PP + q] = d;
            } else {
                coords[(e * PP + q) * od + 0] = x;
                coords[(e * PP + q) * od + 1] = y;
                if (depth) coords[(e * PP + q) * od + 2] = d;
            }
            if (valid) valid[e * PP + q] = X1[2] > 0.2f ? 1.0f : 0.0f;
        };
        if constexpr (PC > 0) {
#pragma unroll
            for (int q = 0; q < PC * PC; q++) pixel(q, pv[0][q], pv[1][q], pv[2][q]);
        } else {
            for (int64_t q = 0; q < PP; q++) pixel(q, pa[q], pa[PP + q], pa[2 * PP + q]);
        }
    }
}

__global__ __launch_bounds__(256) void point_cloud_kernel(const float* __restrict__ poses,
                                                         const float* __restrict__ patches, int P,
                                                         const float* __restrict__ intr,
                                                         const int64_t* __restrict__ ix, int64_t m, int centre_only,
                                                         float* __restrict__ out)
{
    const int64_t PP = (int64_t)P * P, centre = (P / 2) * P + P / 2;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t f = ix[k];
        const float* K = intr + f * 4;
        const float* pa = patches + k * 3 * PP;
        if (centre_only) {
            // every operand load issued before the arithmetic (G3::load normalizes)
            float rp[7], kv[4], c[3];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < 7; t++) rp[t] = poses[f * 7 + t];
#pragma unroll
            for (int t = 0; t < 4; t++) kv[t] = K[t];
#pragma unroll
            for (int t = 0; t < 3; t++) c[t] = pa[t * PP + centre];
            __builtin_amdgcn_sched_barrier(0);
            const G3 g = G3::load(rp).inv();
            const float X0[4] = {(c[0] - kv[2]) / kv[0], (c[1] - kv[3]) / kv[1], 1.0f, c[2]};
            float X1[4];
            g.act4(X0, X1);
            out[k * 3 + 0] = X1[0] / X1[3];
            out[k * 3 + 1] = X1[1] / X1[3];
            out[k * 3 + 2] = X1[2] / X1[3];
        } else {
            const G3 g = G3::load(poses + f * 7).inv();
            for (int64_t q = 0; q < PP; q++) {
                const float X0[4] = {(pa[q] - K[2]) / K[0], (pa[PP + q] - K[3]) / K[1], 1.0f, pa[2 * PP + q]};
                g.act4(X0, out + (k * PP + q) * 4);
            }
        }
    }
}

// transform_kernel's per-pixel projection (iproj -> act4 -> proj, Z >= 0.1)
__device__ __forceinline__ void project_px(const G3& g, const float* ki, const float* kj, const float* pa,
                                           int64_t PP, int64_t q, float& x, float& y)
{
    const float X0[4] = {(pa[q] - ki[2]) / ki[0], (pa[PP + q] - ki[3]) / ki[1], 1.0f, pa[2 * PP + q]};
    float X1[4];
    g.act4(X0, X1);
    const float d = 1.0f / fmaxf(X1[2], 0.1f);
    x = kj[0] * (d * X1[0]) + kj[2];
    y = kj[1] * (d * X1[1]) + kj[3];
}

// DPVO.motionmag (dpvo.py:507-514) for the two directions keyframe() reads
// (i -> j and j -> i, :609): mean over the matching edges and their P*P
// pixels of flow_mag (projective_ops.py:111-121) = beta |x(Gij) - x(Gii)| +
// (1 - beta) |x(t-only Gij) - x(Gii)|.  One workgroup scans the edge list
// (no mask -> index -> gather round trip, no host sync for the match count),
// per-thread partial sums are reduced in a fixed tree order (deterministic).
// out[d] = NaN when direction d has no edge (torch's mean of an empty tensor).
constexpr int MM_THREADS = 1024;
__global__ __launch_bounds__(MM_THREADS) void motion_mag_kernel(const float* poses, const float* patches, int P,
                                                               const float* intr, const int64_t* ii,
                                                               const int64_t* jj, const int64_t* kk, int64_t E,
                                                               int64_t fi, int64_t fj, float beta, float* out)
{
    __shared__ float s_sum[2][MM_THREADS];
    __shared__ int s_cnt[2][MM_THREADS];
    const int t = threadIdx.x;
    const int64_t PP = (int64_t)P * P;
    float sum[2] = {0.f, 0.f};
    int cnt[2] = {0, 0};
    for (int64_t e = t; e < E; e += MM_THREADS) {
        const int64_t a = ii[e], b = jj[e];
        const int dir = (a == fi && b == fj) ? 0 : (a == fj && b == fi) ? 1 : -1;
        if (dir < 0) continue;
        const G3 Pa = G3::load(poses + a * 7), Pb = G3::load(poses + b * 7);
        const G3 g0 = Pa.mul(Pa.inv());
        const G3 g1 = Pb.mul(Pa.inv());
        G3 g2 = g1;
        g2.so3.q.x = 0.f; g2.so3.q.y = 0.f; g2.so3.q.z = 0.f; g2.so3.q.w = 1.f;
        const float *ka = intr + a * 4, *kb = intr + b * 4;
        const float* pa = patches + kk[e] * 3 * PP;
        for (int64_t q = 0; q < PP; q++) {
            float x0, y0, x1, y1, x2, y2;
            project_px(g0, ka, ka, pa, PP, q, x0, y0);
            project_px(g1, ka, kb, pa, PP, q, x1, y1);
            project_px(g2, ka, kb, pa, PP, q, x2, y2);
            const float f1 = sqrtf((x1 - x0) * (x1 - x0) + (y1 - y0) * (y1 - y0));
            const float f2 = sqrtf((x2 - x0) * (x2 - x0) + (y2 - y0) * (y2 - y0));
            sum[dir] += beta * f1 + (1.0f - beta) * f2;
        }
        cnt[dir]++;
    }
    for (int d = 0; d < 2; d++) { s_sum[d][t] = sum[d]; s_cnt[d][t] = cnt[d]; }
    __syncthreads();
    for (int w = MM_THREADS / 2; w > 0; w >>= 1) {
        if (t < w)
            for (int d = 0; d < 2; d++) { s_sum[d][t] += s_sum[d][t + w]; s_cnt[d][t] += s_cnt[d][t + w]; }
        __syncthreads();
    }
    if (t < 2) out[t] = s_cnt[t][0] ? s_sum[t][0] / (float)((int64_t)s_cnt[t][0] * PP) : __builtin_nanf("");
}

// The same two means over many workgroups (the single-workgroup scan of the
// ~95k-edge list takes ~80 us, a latency chain of dependent index loads per
// thread): one edge per thread (grid-stride past MM2_MAXBLK blocks), each
// workgroup reduces its threads in a fixed tree order into part[block] =
// (sum, count) per direction, and motion_mag_final_kernel adds the partials in
// a fixed order too (deterministic).
constexpr int MM2_THREADS = 256, MM2_MAXBLK = 4096;
template <int PT>   // PT = P * P when known at compile time (the P*P pixel loop unrolls), else 0
__global__ __launch_bounds__(MM2_THREADS) void motion_mag_part_kernel(const float* poses, const float* patches, int P,
                                                                     const float* intr, const int64_t* ii,
                                                                     const int64_t* jj, const int64_t* kk, int64_t E,
                                                                     int64_t fi, int64_t fj, float beta, float* part)
{
    __shared__ float s_sum[2][MM2_THREADS];
    __shared__ int s_cnt[2][MM2_THREADS];
    const int t = threadIdx.x;
    const int64_t PP = PT ? PT : (int64_t)P * P;
    float sum[2] = {0.f, 0.f};
    int cnt[2] = {0, 0};
    for (int64_t e = blockIdx.x * (int64_t)MM2_THREADS + t; e < E; e += (int64_t)gridDim.x * MM2_THREADS) {
        const int64_t a = ii[e], b = jj[e];
        const int dir = (a == fi && b == fj) ? 0 : (a == fj && b == fi) ? 1 : -1;
        if (dir < 0) continue;
        const G3 Pa = G3::load(poses + a * 7), Pb = G3::load(poses + b * 7);
        const G3 g0 = Pa.mul(Pa.inv());
        const G3 g1 = Pb.mul(Pa.inv());
        G3 g2 = g1;
        g2.so3.q.x = 0.f; g2.so3.q.y = 0.f; g2.so3.q.z = 0.f; g2.so3.q.w = 1.f;
        const float *ka = intr + a * 4, *kb = intr + b * 4;
        const float* pa = patches + kk[e] * 3 * PP;
        float s = 0.f;
        for (int64_t q = 0; q < PP; q++) {   // (PP = P * P at run time: not unrolled)
            float x0, y0, x1, y1, x2, y2;
            project_px(g0, ka, ka, pa, PP, q, x0, y0);
            project_px(g1, ka, kb, pa, PP, q, x1, y1);
            project_px(g2, ka, kb, pa, PP, q, x2, y2);
            const float f1 = sqrtf((x1 - x0) * (x1 - x0) + (y1 - y0) * (y1 - y0));
            const float f2 = sqrtf((x2 - x0) * (x2 - x0) + (y2 - y0) * (y2 - y0));
            s += beta * f1 + (1.0f - beta) * f2;
        }
        sum[dir] += s;
        cnt[dir]++;
    }
    for (int d = 0; d < 2; d++) { s_sum[d][t] = sum[d]; s_cnt[d][t] = cnt[d]; }
    __syncthreads();
    for (int w = MM2_THREADS / 2; w > 0; w >>= 1) {
        if (t < w)
            for (int d = 0; d < 2; d++) { s_sum[d][t] += s_sum[d][t + w]; s_cnt[d][t] += s_cnt[d][t + w]; }
        __syncthreads();
    }
    if (t < 2) {
        part[blockIdx.x * 4 + 2 * t] = s_sum[t][0];
        part[blockIdx.x * 4 + 2 * t + 1] = __int_as_float(s_cnt[t][0]);
    }
}

// partials of nblk workgroups -> the two means; 256 threads take strided
// partials, then a fixed tree (deterministic for a given nblk)
__global__ __launch_bounds__(MM2_THREADS) void motion_mag_final_kernel(const float* part, int nblk, int64_t PP, float* out)
{
    __shared__ float s_sum[2][MM2_THREADS];
    __shared__ int s_cnt[2][MM2_THREADS];
    const int t = threadIdx.x;
    float sm[2] = {0.f, 0.f};
    int c[2] = {0, 0};
    for (int b = t; b < nblk; b += MM2_THREADS)
        for (int d = 0; d < 2; d++) {
            sm[d] += part[b * 4 + 2 * d];
            c[d] += __float_as_int(part[b * 4 + 2 * d + 1]);
        }
    for (int d = 0; d < 2; d++) { s_sum[d][t] = sm[d]; s_cnt[d][t] = c[d]; }
    __syncthreads();
    for (int w = MM2_THREADS / 2; w > 0; w >>= 1) {
        if (t < w)
            for (int d = 0; d < 2; d++) { s_sum[d][t] += s_sum[d][t + w]; s_cnt[d][t] += s_cnt[d][t + w]; }
        __syncthreads();
    }
    if (t < 2) out[t] = s_cnt[t][0] ? s_sum[t][0] / (float)((int64_t)s_cnt[t][0] * PP) : __builtin_nanf("");
}

// Keyframe distance matrix for the global BA's distance-based edges
// (dpvo.py:383-429 compute_keyframe_distance / get_distance_based_edges, which
// call flow_mag twice and .item() once per frame pair -- O(n^2) host syncs).
// dist[a][b] = mean over frame a's M patches and P*P pixels of flow_mag(a -> b)
// (projective_ops.py:111-121), the same per-pixel arithmetic as
// motion_mag_kernel.  One workgroup per (a, block of KF_TB targets): frame a's
// back-projected pixels and their Gaa projection are staged in LDS once, each
// target's sum is reduced in a fixed tree order (deterministic).
constexpr int KF_THREADS = 256, KF_TB = 16;
__global__ __launch_bounds__(KF_THREADS) void keyframe_flow_kernel(const float* poses, const float* patches, int P,
                                                                  const float* intr, int64_t n, int64_t M,
                                                                  float beta, float* dist)
{
    extern __shared__ float kf_sh[];
    __shared__ float red[KF_THREADS];
    const int t = threadIdx.x;
    const int64_t a = blockIdx.x, b0 = (int64_t)blockIdx.y * KF_TB;
    const int64_t PP = (int64_t)P * P, NPX = M * PP;
    float* X0s = kf_sh;            // [4][NPX]
    float* c0s = kf_sh + 4 * NPX;  // [2][NPX]
    const G3 Pa = G3::load(poses + a * 7);
    const G3 Pai = Pa.inv();
    const G3 g0 = Pa.mul(Pai);     // transform(ii, ii): Gaa, as the reference composes it
    const float* ka = intr + a * 4;
    for (int64_t px = t; px < NPX; px += KF_THREADS) {
        const int64_t k = px / PP, q = px - k * PP;
        const float* pa = patches + (M * a + k) * 3 * PP;
        const float X0[4] = {(pa[q] - ka[2]) / ka[0], (pa[PP + q] - ka[3]) / ka[1], 1.0f, pa[2 * PP + q]};
        float X1[4];
        g0.act4(X0, X1);
        const float d = 1.0f / fmaxf(X1[2], 0.1f);
#pragma unroll
        for (int c = 0; c < 4; c++) X0s[c * NPX + px] = X0[c];
        c0s[px] = ka[0] * (d * X1[0]) + ka[2];
        c0s[NPX + px] = ka[1] * (d * X1[1]) + ka[3];
    }
    __syncthreads();
    for (int bi = 0; bi < KF_TB; bi++) {
        const int64_t b = b0 + bi;
        if (b >= n) break;
        const G3 g1 = G3::load(poses + b * 7).mul(Pai);
        G3 g2 = g1;
        g2.so3.q.x = 0.f; g2.so3.q.y = 0.f; g2.so3.q.z = 0.f; g2.so3.q.w = 1.f;
        const float* kb = intr + b * 4;
        float sum = 0.f;
        for (int64_t px = t; px < NPX; px += KF_THREADS) {
            const float X0[4] = {X0s[px], X0s[NPX + px], X0s[2 * NPX + px], X0s[3 * NPX + px]};
            const float x0 = c0s[px], y0 = c0s[NPX + px];
            float X1[4], X2[4];
            g1.act4(X0, X1);
            g2.act4(X0, X2);
            const float d1 = 1.0f / fmaxf(X1[2], 0.1f), d2 = 1.0f / fmaxf(X2[2], 0.1f);
            const float x1 = kb[0] * (d1 * X1[0]) + kb[2], y1 = kb[1] * (d1 * X1[1]) + kb[3];
            const float x2 = kb[0] * (d2 * X2[0]) + kb[2], y2 = kb[1] * (d2 * X2[1]) + kb[3];
            const float f1 = sqrtf((x1 - x0) * (x1 - x0) + (y1 - y0) * (y1 - y0));
            const float f2 = sqrtf((x2 - x0) * (x2 - x0) + (y2 - y0) * (y2 - y0));
            sum += beta * f1 + (1.0f - beta) * f2;
        }
        red[t] = sum;
        __syncthreads();
        for (int w = KF_THREADS / 2; w > 0; w >>= 1) {
            if (t < w) red[t] += red[t + w];
            __syncthreads();
        }
        if (t == 0) dist[a * n + b] = red[0] / (float)NPX;
        __syncthreads();
    }
}


// ---------------------------------------------------------------------------
// keyframe() device work (dpvo.py:605-658), both outcomes before the decision.
// Per edge e (patch kk from frame ii, target jj), k the candidate frame:
//   old_keep = ix[kk] < n - RW                        (keep: :654-658)
//   drop     = ii == k || jj == k                     (drop: :616-617)
//   kk_d = ii > k ? kk - M : kk,  ii_d = ii > k ? ii - 1 : ii,  jj_d = jj > k ? jj - 1 : jj
//   old_d    = ix[kk_d] < n - 1 - RW && !drop         (retirement after the drop)
//   rm_d     = old_d || drop
// masks u8 [3][E] (old_keep, old_d, rm_d), idx [3][E] (ii_d, jj_d, kk_d),
// part[b][4]: block b's counts of the three masks.  kk outside [0, ix_len)
// reads no index and counts as not old.
constexpr int KM_THREADS = 256, KM_MAXBLK = 512;

__global__ __launch_bounds__(KM_THREADS) void kf_masks_kernel(const int64_t* ii, const int64_t* jj,
                                                              const int64_t* kk, const int64_t* ix, int64_t ix_len,
                                                              int64_t E, int64_t k, int64_t M, int64_t n, int64_t RW,
                                                              uint8_t* masks, int64_t* idx, int* part)
{
    __shared__ int red[3][KM_THREADS / 64];
    int c0 = 0, c1 = 0, c2 = 0;
    for (int64_t e = blockIdx.x * (int64_t)KM_THREADS + threadIdx.x; e < E; e += (int64_t)gridDim.x * KM_THREADS) {
        const int64_t a = ii[e], b = jj[e], p = kk[e];
        const bool later = a > k, drop = a == k || b == k;
        const int64_t pd = later ? p - M : p;
        const bool keep_old = p >= 0 && p < ix_len && ix[p] < n - RW;
        const bool old_d = !drop && pd >= 0 && pd < ix_len && ix[pd] < n - 1 - RW;
        const bool rm_d = old_d || drop;
        masks[e] = keep_old;
        masks[E + e] = old_d;
        masks[2 * E + e] = rm_d;
        idx[e] = later ? a - 1 : a;
        idx[E + e] = b > k ? b - 1 : b;
        idx[2 * E + e] = pd;
        c0 += keep_old;
        c1 += old_d;
        c2 += rm_d;
    }
    for (int o = 32; o > 0; o >>= 1) {
        c0 += __shfl_xor(c0, o);
        c1 += __shfl_xor(c1, o);
        c2 += __shfl_xor(c2, o);
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) { red[0][wv] = c0; red[1][wv] = c1; red[2][wv] = c2; }
    __syncthreads();
    if (threadIdx.x < 3) {
        int t = 0;
        for (int w = 0; w < KM_THREADS / 64; w++) t += red[threadIdx.x][w];
        part[blockIdx.x * 4 + threadIdx.x] = t;
    }
}

// vals = [mm[0], mm[1], ba_fail, any(isnan(pose_k)), n_old_keep, n_old_d, n_rm_d]
// as doubles: keyframe()'s one host read (dpvo.py:609, :647, the compaction sizes)
__global__ __launch_bounds__(64) void kf_pack_kernel(const int* part, int nblk, const float* mm,
                                                     const int* ba_fail, const float* pose_k, double* vals)
{
    const int t = threadIdx.x;
    long long c[3] = {0, 0, 0};
    for (int b = t; b < nblk; b += 64)
        for (int q = 0; q < 3; q++) c[q] += part[b * 4 + q];
    for (int o = 32; o > 0; o >>= 1)
        for (int q = 0; q < 3; q++) c[q] += __shfl_xor(c[q], o);
    if (t == 0) {
        bool nan = false;
        for (int q = 0; q < 7; q++) nan = nan || isnan(pose_k[q]);
        vals[0] = (double)mm[0];
        vals[1] = (double)mm[1];
        vals[2] = (double)ba_fail[0];
        vals[3] = nan ? 1.0 : 0.0;
        vals[4] = (double)c[0];
        vals[5] = (double)c[1];
        vals[6] = (double)c[2];
    }
}

// A keyframe drop moves frames k+1 .. n-1 down by one slot in every per-frame
// buffer (dpvo.py:626-639).  Segment s: slots of slot_bytes at base, frame f
// in slot f % ring (ring 0: slot f).  Each thread owns one word offset of every
// slot and walks the frames upwards, so it reads slot f+1 before it writes it:
// the same result as the reference's loop, in one launch for all buffers.
struct FsSeg {
    char* base;
    int64_t slot_bytes, ring;
    int unit;   // 16, 4 or 1 bytes per word
};
constexpr int FS_MAXSEG = 16;
struct FsArgs {
    FsSeg seg[FS_MAXSEG];
    int nseg;
};

__global__ __launch_bounds__(256) void frame_shift_kernel(FsArgs a, int64_t k, int64_t n)
{
    const FsSeg s = a.seg[blockIdx.y];
    const int64_t words = s.slot_bytes / s.unit;
    for (int64_t w = blockIdx.x * 256ll + threadIdx.x; w < words; w += (int64_t)gridDim.x * 256) {
        for (int64_t f = k; f + 1 < n; f++) {
            const int64_t d = s.ring ? f % s.ring : f, r = s.ring ? (f + 1) % s.ring : f + 1;
            char* dst = s.base + d * s.slot_bytes + w * s.unit;
            const char* src = s.base + r * s.slot_bytes + w * s.unit;
            if (s.unit == 16) *(uint4*)dst = *(const uint4*)src;
            else if (s.unit == 4) *(uint32_t*)dst = *(const uint32_t*)src;
            else *dst = *src;
        }
    }
}


// ---------------------------------------------------------------------------
// Edge-state compaction of keyframe() / remove_factors (dpvo.py:349-364):
// edges with rm[e] == 0 keep their order at the front of the kept arrays;
// edges with store[e] != 0 (a subset of the removed ones; store_mode 1: all
// removed edges) are appended, in order, to the inactive lists.  Two launches:
// per-block counts, then each block adds up the counts before it, ranks its
// edges with wave ballots and moves them -- the index fields, the (weight,
// target) rows and the edge-state rows (row_words 16-byte words each).
constexpr int CE_THREADS = 256, CE_EDGES = 256;   // one edge per thread: E / 256 blocks

struct CeArgs {
    int64_t E;
    const uint8_t* rm; const uint8_t* store; int store_mode;
    const int64_t* ii; const int64_t* jj; const int64_t* kk;
    const char* w; const char* t; int wt_bytes;          // weight / target rows, wt_bytes each
    const uint4* net; int64_t row_words;                  // edge-state rows
    int64_t* ii_k; int64_t* jj_k; int64_t* kk_k; char* w_k; char* t_k; uint4* net_k;
    int64_t* ii_s; int64_t* jj_s; int64_t* kk_s; char* w_s; char* t_s;
    int* part;
};

__device__ __forceinline__ bool ce_store(const CeArgs& a, int64_t e, bool rm)
{
    return a.store_mode == 1 ? rm : a.store_mode == 2 ? a.store[e] != 0 : false;
}

__device__ __forceinline__ void ce_row(char* d, const char* sp, int bytes)
{
    if (bytes % 8 == 0 && ((uintptr_t)d & 7) == 0 && ((uintptr_t)sp & 7) == 0)
        for (int b = 0; b < bytes; b += 8) *(uint2*)(d + b) = *(const uint2*)(sp + b);
    else
        for (int b = 0; b < bytes; b++) d[b] = sp[b];
}

__global__ __launch_bounds__(CE_THREADS) void ce_count_kernel(CeArgs a)
{
    __shared__ int red[2][CE_THREADS / 64];
    int ck = 0, cs = 0;
    const int64_t e0 = (int64_t)blockIdx.x * CE_EDGES;
    for (int i = threadIdx.x; i < CE_EDGES; i += CE_THREADS) {
        const int64_t e = e0 + i;
        if (e < a.E) {
            const bool rm = a.rm[e] != 0;
            ck += !rm;
            cs += ce_store(a, e, rm);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        ck += __shfl_xor(ck, o);
        cs += __shfl_xor(cs, o);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = ck;
        red[1][threadIdx.x >> 6] = cs;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        int t = 0;
        for (int w = 0; w < CE_THREADS / 64; w++) t += red[threadIdx.x][w];
        a.part[blockIdx.x * 2 + threadIdx.x] = t;
    }
}

__global__ __launch_bounds__(CE_THREADS) void ce_move_kernel(CeArgs a)
{
    __shared__ int base[2];
    __shared__ int wsum[2][CE_THREADS / 64];
    __shared__ int64_t src[CE_EDGES], dst[CE_EDGES];
    __shared__ int nk_s;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // counts of the blocks before this one
    {
        int bk = 0, bs = 0;
        for (int b = tid; b < (int)blockIdx.x; b += CE_THREADS) {
            bk += a.part[2 * b];
            bs += a.part[2 * b + 1];
        }
        for (int o = 32; o > 0; o >>= 1) {
            bk += __shfl_xor(bk, o);
            bs += __shfl_xor(bs, o);
        }
        if (lane == 0) { wsum[0][wv] = bk; wsum[1][wv] = bs; }
        __syncthreads();
        if (tid < 2) {
            int t = 0;
            for (int w = 0; w < CE_THREADS / 64; w++) t += wsum[tid][w];
            base[tid] = t;
        }
        __syncthreads();
    }
    const int64_t e0 = (int64_t)blockIdx.x * CE_EDGES;
    int64_t ok = base[0], os = base[1];   // running output positions (block-uniform)
    int nk = 0;                           // kept edges of this block so far
    for (int c = 0; c < CE_EDGES; c += CE_THREADS) {
        const int64_t e = e0 + c + tid;
        const bool in = e < a.E;
        const bool rm = in && a.rm[e] != 0;
        const bool keep = in && !rm, st = in && ce_store(a, e, rm);
        const uint64_t bk = __ballot(keep), bs = __ballot(st);
        const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
        const int rk = __popcll(bk & below), rs = __popcll(bs & below);
        if (lane == 0) { wsum[0][wv] = __popcll(bk); wsum[1][wv] = __popcll(bs); }
        __syncthreads();
        int pk = 0, ps = 0, tk = 0, ts = 0;
        for (int w = 0; w < CE_THREADS / 64; w++) {
            pk += w < wv ? wsum[0][w] : 0;
            ps += w < wv ? wsum[1][w] : 0;
            tk += wsum[0][w];
            ts += wsum[1][w];
        }
        if (keep) {
            const int64_t d = ok + pk + rk;
            a.ii_k[d] = a.ii[e];
            a.jj_k[d] = a.jj[e];
            a.kk_k[d] = a.kk[e];
            ce_row(a.w_k + d * a.wt_bytes, a.w + e * a.wt_bytes, a.wt_bytes);
            ce_row(a.t_k + d * a.wt_bytes, a.t + e * a.wt_bytes, a.wt_bytes);
            src[nk + pk + rk] = e;
            dst[nk + pk + rk] = d;
        }
        if (st) {
            const int64_t d = os + ps + rs;
            a.ii_s[d] = a.ii[e];
            a.jj_s[d] = a.jj[e];
            a.kk_s[d] = a.kk[e];
            ce_row(a.w_s + d * a.wt_bytes, a.w + e * a.wt_bytes, a.wt_bytes);
            ce_row(a.t_s + d * a.wt_bytes, a.t + e * a.wt_bytes, a.wt_bytes);
        }
        ok += tk;
        os += ts;
        nk += tk;
        __syncthreads();   // wsum reused by the next chunk
    }
    if (tid == 0) nk_s = nk;
    __syncthreads();
    // the kept edge-state rows: each wave moves groups of 8 rows as one flat
    // range of 16-byte words, all of a lane's loads issued before its stores
    // (12 per lane for 1,536-byte rows: enough bytes in flight for HBM)
    const int rw = (int)a.row_words;
    constexpr int G = 8, U = 12;
    for (int r0 = wv * G; r0 < nk_s; r0 += (CE_THREADS / 64) * G) {
        const int total = min(G, nk_s - r0) * rw;
        uint4 v[U];
        int64_t to[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const int q = lane + 64 * j;
            if (q < total) {
                const int r = q / rw, wd = q - r * rw;
                v[j] = a.net[src[r0 + r] * rw + wd];
                to[j] = dst[r0 + r] * rw + wd;
            }
        }
#pragma unroll
        for (int j = 0; j < U; j++)
            if (lane + 64 * j < total) a.net_k[to[j]] = v[j];
        for (int q = lane + 64 * U; q < total; q += 64) {   // rows wider than 96 words
            const int r = q / rw, wd = q - r * rw;
            a.net_k[dst[r0 + r] * rw + wd] = a.net[src[r0 + r] * rw + wd];
        }
    }
}

}  // namespace dpvo

using namespace dpvo;

extern "C" int dpvo_hot_abi_version(void) { return DPVO_HOT_ABI_VERSION; }
extern "C" const char* dpvo_hot_last_error(void) { return g_last_error.c_str(); }

extern "C" int dpvo_transform(const float* poses, const float* patches, int P, const float* intrinsics,
                              const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t num_edges, int flags,
                              float* coords, float* valid, void* stream)
{
    DPVO_CHECK_ARG(P >= 1, "bad patch size");
    if (num_edges == 0) return 0;
    DPVO_CHECK_ARG(poses && patches && intrinsics && ii && jj && kk && coords, "null operand");
    if (P == 3)
        hipLaunchKernelGGL(transform_kernel<3>, dim3(grid_for(num_edges, 256)), dim3(256), 0, as_stream(stream), poses,
                           patches, P, intrinsics, ii, jj, kk, num_edges, flags, coords, valid);
    else
        hipLaunchKernelGGL(transform_kernel<0>, dim3(grid_for(num_edges, 256)), dim3(256), 0, as_stream(stream), poses,
                           patches, P, intrinsics, ii, jj, kk, num_edges, flags, coords, valid);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_point_cloud(const float* poses, const float* patches, int P, const float* intrinsics,
                                const int64_t* ix, int64_t m, int centre_only, float* out, void* stream)
{
    DPVO_CHECK_ARG(P >= 1, "bad patch size");
    if (m == 0) return 0;
    DPVO_CHECK_ARG(poses && patches && intrinsics && ix && out, "null operand");
    hipLaunchKernelGGL(point_cloud_kernel, dim3(grid_for(m, 256)), dim3(256), 0, as_stream(stream), poses, patches,
                       P, intrinsics, ix, m, centre_only, out);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_motion_mag(const float* poses, const float* patches, int P, const float* intrinsics,
                               const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t num_edges, int64_t i,
                               int64_t j, float beta, float* out, void* stream)
{
    DPVO_CHECK_ARG(P >= 1, "bad patch size");
    DPVO_CHECK_ARG(num_edges >= 0, "negative edge count");
    DPVO_CHECK_ARG(out && (num_edges == 0 || (poses && patches && intrinsics && ii && jj && kk)), "null operand");
    hipLaunchKernelGGL(motion_mag_kernel, dim3(1), dim3(MM_THREADS), 0, as_stream(stream), poses, patches, P,
                       intrinsics, ii, jj, kk, num_edges, i, j, beta, out);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" size_t dpvo_keyframe_flow_lds_bytes(int P, int64_t patches_per_frame)
{
    return (size_t)6 * P * P * patches_per_frame * sizeof(float);
}

extern "C" int dpvo_keyframe_flow(const float* poses, const float* patches, int P, const float* intrinsics,
                                  int64_t num_frames, int64_t patches_per_frame, float beta, float* dist, void* stream)
{
    DPVO_CHECK_ARG(P >= 1 && num_frames >= 0 && patches_per_frame >= 1, "bad sizes");
    DPVO_CHECK_ARG(num_frames < 65536 * (int64_t)KF_TB, "too many frames");
    if (num_frames == 0) return 0;
    DPVO_CHECK_ARG(poses && patches && intrinsics && dist, "null operand");
    const size_t lds = dpvo_keyframe_flow_lds_bytes(P, patches_per_frame);
    DPVO_CHECK_ARG(lds + KF_THREADS * sizeof(float) <= 160 * 1024, "one frame's patches do not fit in LDS");
    const dim3 grid((unsigned)num_frames, (unsigned)((num_frames + KF_TB - 1) / KF_TB));
    hipLaunchKernelGGL(keyframe_flow_kernel, grid, dim3(KF_THREADS), lds, as_stream(stream), poses, patches, P,
                       intrinsics, num_frames, patches_per_frame, beta, dist);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" size_t dpvo_motion_mag_workspace_bytes(int64_t num_edges)
{
    (void)num_edges;
    return (size_t)MM2_MAXBLK * 4 * sizeof(float);
}

extern "C" int dpvo_motion_mag_ws(const float* poses, const float* patches, int P, const float* intrinsics,
                                  const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t num_edges, int64_t i,
                                  int64_t j, float beta, float* out, void* workspace, size_t workspace_bytes,
                                  void* stream)
{
    DPVO_CHECK_ARG(P >= 1, "bad patch size");
    DPVO_CHECK_ARG(num_edges >= 0, "negative edge count");
    DPVO_CHECK_ARG(out && (num_edges == 0 || (poses && patches && intrinsics && ii && jj && kk)), "null operand");
    DPVO_CHECK_ARG(workspace && workspace_bytes >= dpvo_motion_mag_workspace_bytes(num_edges), "workspace too small");
    const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>((num_edges + MM2_THREADS - 1) / MM2_THREADS,
                                                                  MM2_MAXBLK));
    if (P == 3)
        hipLaunchKernelGGL(motion_mag_part_kernel<9>, dim3(nblk), dim3(MM2_THREADS), 0, as_stream(stream), poses,
                           patches, P, intrinsics, ii, jj, kk, num_edges, i, j, beta, (float*)workspace);
    else
        hipLaunchKernelGGL(motion_mag_part_kernel<0>, dim3(nblk), dim3(MM2_THREADS), 0, as_stream(stream), poses,
                           patches, P, intrinsics, ii, jj, kk, num_edges, i, j, beta, (float*)workspace);
    hipLaunchKernelGGL(motion_mag_final_kernel, dim3(1), dim3(MM2_THREADS), 0, as_stream(stream),
                       (const float*)workspace, nblk, (int64_t)P * P, out);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" size_t dpvo_keyframe_masks_workspace_bytes(int64_t num_edges)
{
    (void)num_edges;
    return (size_t)KM_MAXBLK * 4 * sizeof(int);
}

extern "C" int dpvo_keyframe_masks(const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t num_edges,
                                   const int64_t* ix, int64_t ix_len, int64_t k, int64_t M, int64_t n, int64_t RW,
                                   const float* mm, const int* ba_fail, const float* pose_k, uint8_t* masks,
                                   int64_t* idx, double* vals, void* workspace, size_t workspace_bytes, void* stream)
{
    DPVO_CHECK_ARG(num_edges >= 0 && ix_len >= 0, "negative size");
    DPVO_CHECK_ARG(mm && ba_fail && pose_k && vals, "null operand");
    DPVO_CHECK_ARG(num_edges == 0 || (ii && jj && kk && ix && masks && idx), "null operand");
    DPVO_CHECK_ARG(workspace && workspace_bytes >= dpvo_keyframe_masks_workspace_bytes(num_edges),
                   "workspace too small");
    const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>((num_edges + KM_THREADS - 1) / KM_THREADS,
                                                                  KM_MAXBLK));
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(kf_masks_kernel, dim3(nblk), dim3(KM_THREADS), 0, st, ii, jj, kk, ix, ix_len, num_edges, k, M,
                       n, RW, masks, idx, (int*)workspace);
    hipLaunchKernelGGL(kf_pack_kernel, dim3(1), dim3(64), 0, st, (const int*)workspace, nblk, mm, ba_fail, pose_k,
                       vals);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_frame_shift(void* const* bases, const int64_t* slot_bytes, const int64_t* rings, int nseg,
                                int64_t k, int64_t n, void* stream)
{
    DPVO_CHECK_ARG(nseg >= 0 && nseg <= FS_MAXSEG, "at most 16 buffers");
    DPVO_CHECK_ARG(nseg == 0 || (bases && slot_bytes && rings), "null operand");
    if (nseg == 0 || n - 1 <= k) return 0;
    DPVO_CHECK_ARG(k >= 0, "k must be >= 0");
    FsArgs a{};
    a.nseg = nseg;
    int64_t most = 0;
    for (int i = 0; i < nseg; i++) {
        DPVO_CHECK_ARG(bases[i] && slot_bytes[i] > 0 && rings[i] >= 0, "bad buffer");
        DPVO_CHECK_ARG(rings[i] == 0 || n - k <= rings[i], "the moved frames must fit in the ring");
        const uintptr_t b = (uintptr_t)bases[i];
        const int unit = (b % 16 == 0 && slot_bytes[i] % 16 == 0) ? 16 : (b % 4 == 0 && slot_bytes[i] % 4 == 0) ? 4 : 1;
        a.seg[i] = {(char*)bases[i], slot_bytes[i], rings[i], unit};
        most = std::max<int64_t>(most, slot_bytes[i] / unit);
    }
    const unsigned gx = (unsigned)std::min<int64_t>((most + 255) / 256, 2048);
    hipLaunchKernelGGL(frame_shift_kernel, dim3(gx, nseg), dim3(256), 0, as_stream(stream), a, k, n);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" size_t dpvo_compact_edges_workspace_bytes(int64_t num_edges)
{
    return (size_t)std::max<int64_t>(1, (num_edges + CE_EDGES - 1) / CE_EDGES) * 2 * sizeof(int);
}

extern "C" int dpvo_compact_edges(int64_t num_edges, const uint8_t* rm, const uint8_t* store, int store_mode,
                                  const int64_t* ii, const int64_t* jj, const int64_t* kk, const void* weight,
                                  const void* target, int wt_bytes, const void* net, int64_t row_bytes,
                                  int64_t* ii_k, int64_t* jj_k, int64_t* kk_k, void* weight_k, void* target_k,
                                  void* net_k, int64_t* ii_s, int64_t* jj_s, int64_t* kk_s, void* weight_s,
                                  void* target_s, void* workspace, size_t workspace_bytes, void* stream)
{
    DPVO_CHECK_ARG(num_edges >= 0 && store_mode >= 0 && store_mode <= 2, "bad size or store mode");
    if (num_edges == 0) return 0;
    DPVO_CHECK_ARG(rm && ii && jj && kk && weight && target && net, "null operand");
    DPVO_CHECK_ARG(ii_k && jj_k && kk_k && weight_k && target_k && net_k, "null kept output");
    DPVO_CHECK_ARG(store_mode != 2 || store, "store_mode 2 needs the store mask");
    DPVO_CHECK_ARG(store_mode == 0 || (ii_s && jj_s && kk_s && weight_s && target_s), "null inactive output");
    DPVO_CHECK_ARG(wt_bytes > 0 && row_bytes > 0 && row_bytes % 16 == 0, "row sizes: edge-state rows of 16-byte words");
    DPVO_CHECK_ARG(((uintptr_t)net & 15) == 0 && ((uintptr_t)net_k & 15) == 0, "edge-state rows must be 16-byte aligned");
    DPVO_CHECK_ARG(workspace && workspace_bytes >= dpvo_compact_edges_workspace_bytes(num_edges), "workspace too small");
    const unsigned nblk = (unsigned)((num_edges + CE_EDGES - 1) / CE_EDGES);
    CeArgs a{num_edges, rm, store, store_mode, ii, jj, kk, (const char*)weight, (const char*)target, wt_bytes,
             (const uint4*)net, row_bytes / 16, ii_k, jj_k, kk_k, (char*)weight_k, (char*)target_k, (uint4*)net_k,
             ii_s, jj_s, kk_s, (char*)weight_s, (char*)target_s, (int*)workspace};
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(ce_count_kernel, dim3(nblk), dim3(CE_THREADS), 0, st, a);
    hipLaunchKernelGGL(ce_move_kernel, dim3(nblk), dim3(CE_THREADS), 0, st, a);
    DPVO_CHECK_LAUNCH();
    return 0;
}

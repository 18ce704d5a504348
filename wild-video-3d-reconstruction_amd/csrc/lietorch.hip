// lietorch.hip -- SO3 / RxSO3 / SE3 / Sim3 group operators for gfx950.
//
// Replaces the GPU half of the reference's lietorch_backends extension
// (dpvo/lietorch/src/lietorch.cpp:286-316, lietorch_gpu.cu:21-601): one
// thread per group element, flat [n][dim] operands.  Backward outputs follow
// the reference's convention of writing the K-dim tangent gradient into the
// first K slots of each N-dim row (lietorch_gpu.cu:87-92, 116-120, ...).
#include "common.hpp"
#include "liegroups.hpp"

namespace dpvo {

using lie::SE3;
using lie::SO3;

#define GRID_LOOP(i, n) for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

template <class G, typename T>
__global__ __launch_bounds__(256) void lie_fwd_kernel(int op, const T* X, const T* Y, T* out, int64_t n)
{
    constexpr int K = G::K, N = G::N;
    GRID_LOOP(i, n)
    {
        switch (op) {
        case DPVO_LIE_EXP: G::Exp(X + i * K).store(out + i * N); break;
        case DPVO_LIE_LOG: G::load(X + i * N).Log(out + i * K); break;
        case DPVO_LIE_INV: G::load(X + i * N).inv().store(out + i * N); break;
        case DPVO_LIE_MUL: G::load(X + i * N).mul(G::load(Y + i * N)).store(out + i * N); break;
        case DPVO_LIE_ADJ:
        case DPVO_LIE_ADJT: {
            T A[K][K];
            G::load(X + i * N).Adj(A);
            const T* a = Y + i * K;
            for (int r = 0; r < K; r++) {
                T s = 0;
                for (int c = 0; c < K; c++) s += (op == DPVO_LIE_ADJ ? A[r][c] : A[c][r]) * a[c];
                out[i * K + r] = s;
            }
            break;
        }
        case DPVO_LIE_ACT: G::load(X + i * N).act(Y + i * 3, out + i * 3); break;
        case DPVO_LIE_ACT4: G::load(X + i * N).act4(Y + i * 4, out + i * 4); break;
        case DPVO_LIE_MATRIX: {
            T M[4][4];
            G::load(X + i * N).matrix4(M);
            for (int r = 0; r < 4; r++)
                for (int c = 0; c < 4; c++) out[i * 16 + r * 4 + c] = M[r][c];
            break;
        }
        case DPVO_LIE_PROJECTOR: G::load(X + i * N).projector(out + i * N * N); break;
        case DPVO_LIE_JINV: {
            T a[K], J[K][K];
            G::load(X + i * N).Log(a);
            G::left_jacobian_inverse(a, J);
            const T* v = Y + i * K;
            for (int r = 0; r < K; r++) {
                T s = 0;
                for (int c = 0; c < K; c++) s += J[r][c] * v[c];
                out[i * K + r] = s;
            }
            break;
        }
        default: break;
        }
    }
}

// row vector (1 x R) times matrix (R x C)
template <typename T, int R, int C>
__device__ __forceinline__ void rowmul(const T* v, const T M[R][C], T* o)
{
    for (int c = 0; c < C; c++) {
        T s = 0;
        for (int r = 0; r < R; r++) s += v[r] * M[r][c];
        o[c] = s;
    }
}

template <class G, typename T>
__global__ __launch_bounds__(256) void lie_bwd_kernel(int op, const T* grad, const T* X, const T* Y, T* dX, T* dY,
                                                     int64_t n)
{
    constexpr int K = G::K, N = G::N;
    GRID_LOOP(i, n)
    {
        switch (op) {
        case DPVO_LIE_EXP: {  // lietorch_gpu.cu:31-43
            T J[K][K];
            G::left_jacobian(X + i * K, J);
            rowmul<T, K, K>(grad + i * N, J, dX + i * K);
            break;
        }
        case DPVO_LIE_LOG: {  // :59-71
            T a[K], J[K][K];
            G::load(X + i * N).Log(a);
            G::left_jacobian_inverse(a, J);
            rowmul<T, K, K>(grad + i * K, J, dX + i * N);
            break;
        }
        case DPVO_LIE_INV: {  // :86-98
            T A[K][K], v[K];
            G::load(X + i * N).inv().Adj(A);
            rowmul<T, K, K>(grad + i * N, A, v);
            for (int k = 0; k < K; k++) dX[i * N + k] = -v[k];
            break;
        }
        case DPVO_LIE_MUL: {  // :113-127
            T A[K][K];
            for (int k = 0; k < K; k++) dX[i * N + k] = grad[i * N + k];
            G::load(X + i * N).Adj(A);
            rowmul<T, K, K>(grad + i * N, A, dY + i * N);
            break;
        }
        case DPVO_LIE_ADJ: {  // :141-159
            T A[K][K], b[K], ad[K][K], v[K];
            G::load(X + i * N).Adj(A);
            const T* a = Y + i * K;
            for (int r = 0; r < K; r++) { b[r] = 0; for (int c = 0; c < K; c++) b[r] += A[r][c] * a[c]; }
            rowmul<T, K, K>(grad + i * K, A, dY + i * K);
            G::ad(b, ad);
            rowmul<T, K, K>(grad + i * K, ad, v);
            for (int k = 0; k < K; k++) dX[i * N + k] = -v[k];
            break;
        }
        case DPVO_LIE_ADJT: {  // :177-192
            T A[K][K], b[K], ad[K][K], v[K];
            G::load(X + i * N).Adj(A);
            const T* db = grad + i * K;
            for (int r = 0; r < K; r++) { b[r] = 0; for (int c = 0; c < K; c++) b[r] += A[r][c] * db[c]; }
            for (int k = 0; k < K; k++) dY[i * K + k] = b[k];
            G::ad(b, ad);
            rowmul<T, K, K>(Y + i * K, ad, v);
            for (int k = 0; k < K; k++) dX[i * N + k] = -v[k];
            break;
        }
        case DPVO_LIE_ACT: {  // :209-226
            const G g = G::load(X + i * N);
            T M[4][4], R3[3][3], q[3], J[3][K];
            g.matrix4(M);
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++) R3[r][c] = M[r][c];
            rowmul<T, 3, 3>(grad + i * 3, R3, dY + i * 3);
            g.act(Y + i * 3, q);
            G::act_jacobian(q, J);
            rowmul<T, 3, K>(grad + i * 3, J, dX + i * N);
            break;
        }
        case DPVO_LIE_ACT4: {  // :243-260
            const G g = G::load(X + i * N);
            T M[4][4], q[4], J[4][K];
            g.matrix4(M);
            rowmul<T, 4, 4>(grad + i * 4, M, dY + i * 4);
            g.act4(Y + i * 4, q);
            G::act4_jacobian(q, J);
            rowmul<T, 4, K>(grad + i * 4, J, dX + i * N);
            break;
        }
        default: break;
        }
    }
}

}  // namespace dpvo

using namespace dpvo;

namespace {
template <template <typename> class G>
int lie_dispatch_fwd(int op, int dtype, const void* X, const void* Y, void* out, int64_t n, hipStream_t s)
{
    const unsigned grid = grid_for(n, 256, 65536);
    if (dtype == DPVO_F32)
        hipLaunchKernelGGL((lie_fwd_kernel<G<float>, float>), dim3(grid), dim3(256), 0, s, op, (const float*)X,
                           (const float*)Y, (float*)out, n);
    else
        hipLaunchKernelGGL((lie_fwd_kernel<G<double>, double>), dim3(grid), dim3(256), 0, s, op, (const double*)X,
                           (const double*)Y, (double*)out, n);
    return 0;
}
template <template <typename> class G>
int lie_dispatch_bwd(int op, int dtype, const void* g, const void* X, const void* Y, void* dX, void* dY, int64_t n,
                     hipStream_t s)
{
    const unsigned grid = grid_for(n, 256, 65536);
    if (dtype == DPVO_F32)
        hipLaunchKernelGGL((lie_bwd_kernel<G<float>, float>), dim3(grid), dim3(256), 0, s, op, (const float*)g,
                           (const float*)X, (const float*)Y, (float*)dX, (float*)dY, n);
    else
        hipLaunchKernelGGL((lie_bwd_kernel<G<double>, double>), dim3(grid), dim3(256), 0, s, op, (const double*)g,
                           (const double*)X, (const double*)Y, (double*)dX, (double*)dY, n);
    return 0;
}
}  // namespace

extern "C" int dpvo_lie_forward(int op, int group, int dtype, const void* X, const void* Y, void* out, int64_t n,
                                void* stream)
{
    DPVO_CHECK_ARG(group >= 1 && group <= 4, "group id must be 1 (SO3), 2 (RxSO3), 3 (SE3) or 4 (Sim3)");
    DPVO_CHECK_ARG(dtype == DPVO_F32 || dtype == DPVO_F64, "lietorch ops take float32 or float64");
    DPVO_CHECK_ARG(op >= DPVO_LIE_EXP && op <= DPVO_LIE_JINV, "unknown operator");
    if (n == 0) return 0;
    const bool binary = op == DPVO_LIE_MUL || op == DPVO_LIE_ADJ || op == DPVO_LIE_ADJT || op == DPVO_LIE_ACT ||
                        op == DPVO_LIE_ACT4 || op == DPVO_LIE_JINV;
    DPVO_CHECK_ARG(X && out && (!binary || Y), "null operand");
    switch (group) {
    case 1: lie_dispatch_fwd<lie::SO3>(op, dtype, X, Y, out, n, as_stream(stream)); break;
    case 2: lie_dispatch_fwd<lie::RxSO3>(op, dtype, X, Y, out, n, as_stream(stream)); break;
    case 3: lie_dispatch_fwd<lie::SE3>(op, dtype, X, Y, out, n, as_stream(stream)); break;
    default: lie_dispatch_fwd<lie::Sim3>(op, dtype, X, Y, out, n, as_stream(stream)); break;
    }
    DPVO_CHECK_LAUNCH();
    return 0;
}

// DPVO.__call__'s DAMPED_LINEAR motion model (dpvo.py:816-825) in one
// launch instead of five lietorch calls from Python (inv, mul, log, the scalar
// product, exp, mul): poses[n] = Exp(s Log(poses[n-1] poses[n-2]^-1)) poses[n-1],
// s = MOTION_DAMPING * dt ratio rounded to fp32 (as torch rounds the scalar).
// The same SE3 functions the lietorch kernels use, values kept in registers
// between them (fp32 either way).
__global__ void pose_extrapolate_kernel(float* poses, int64_t n, float s)
{
    const SE3<float> P1 = SE3<float>::load(poses + (n - 1) * 7), P2 = SE3<float>::load(poses + (n - 2) * 7);
    float xi[6];
    P1.mul(P2.inv()).Log(xi);
    for (int k = 0; k < 6; k++) xi[k] = xi[k] * s;
    SE3<float>::Exp(xi).mul(P1).store(poses + n * 7);
}

// keyframe()'s relative pose of a dropped frame (dpvo.py:613): out = a b^-1
__global__ void pose_relative_kernel(const float* a, const float* b, float* out)
{
    SE3<float>::load(a).mul(SE3<float>::load(b).inv()).store(out);
}

extern "C" int dpvo_pose_extrapolate(float* poses, int64_t n, float s, void* stream)
{
    DPVO_CHECK_ARG(poses != nullptr && n >= 2, "poses[n-2], poses[n-1] needed (n >= 2)");
    hipLaunchKernelGGL(pose_extrapolate_kernel, dim3(1), dim3(1), 0, as_stream(stream), poses, n, s);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_pose_relative(const float* a, const float* b, float* out, void* stream)
{
    DPVO_CHECK_ARG(a && b && out, "null operand");
    hipLaunchKernelGGL(pose_relative_kernel, dim3(1), dim3(1), 0, as_stream(stream), a, b, out);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_lie_backward(int op, int group, int dtype, const void* grad, const void* X, const void* Y,
                                 void* dX, void* dY, int64_t n, void* stream)
{
    DPVO_CHECK_ARG(group >= 1 && group <= 4, "group id must be 1 (SO3), 2 (RxSO3), 3 (SE3) or 4 (Sim3)");
    DPVO_CHECK_ARG(dtype == DPVO_F32 || dtype == DPVO_F64, "lietorch ops take float32 or float64");
    DPVO_CHECK_ARG(op >= DPVO_LIE_EXP && op <= DPVO_LIE_ACT4, "operator has no backward");
    if (n == 0) return 0;
    switch (group) {
    case 1: lie_dispatch_bwd<lie::SO3>(op, dtype, grad, X, Y, dX, dY, n, as_stream(stream)); break;
    case 2: lie_dispatch_bwd<lie::RxSO3>(op, dtype, grad, X, Y, dX, dY, n, as_stream(stream)); break;
    case 3: lie_dispatch_bwd<lie::SE3>(op, dtype, grad, X, Y, dX, dY, n, as_stream(stream)); break;
    default: lie_dispatch_bwd<lie::Sim3>(op, dtype, grad, X, Y, dX, dY, n, as_stream(stream)); break;
    }
    DPVO_CHECK_LAUNCH();
    return 0;
}

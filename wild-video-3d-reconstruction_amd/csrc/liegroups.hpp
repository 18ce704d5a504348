// liegroups.hpp -- SO3 / RxSO3 / SE3 / Sim3 on the device, no Eigen.
//
// Restates the group algebra of the reference's lietorch headers
// (dpvo/lietorch/include/so3.h, rxso3.h, se3.h, sim3.h) with explicit
// small-matrix code: element data [qx,qy,qz,qw] (SO3), [qx,qy,qz,qw,s]
// (RxSO3), [tx,ty,tz,qx,qy,qz,qw] (SE3) and [tx,ty,tz,qx,qy,qz,qw,s] (Sim3);
// the quaternion is normalised on every load exactly as SO3(const Scalar*)
// does (so3.h:47-49); EPS = 1e-6 small-angle branches (common.h:7).
#pragma once

#include <hip/hip_runtime.h>

namespace dpvo {
namespace lie {

template <typename T>
struct Quat {
    T x, y, z, w;
};

template <typename T>
__device__ __forceinline__ T lie_eps() { return (T)1e-6; }

template <typename T>
__device__ __forceinline__ Quat<T> qnormalize(Quat<T> q)
{
    const T n2 = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
    if (n2 > (T)0) {
        const T n = sqrt(n2);
        q.x /= n; q.y /= n; q.z /= n; q.w /= n;
    }
    return q;
}
template <typename T>
__device__ __forceinline__ Quat<T> qmul(const Quat<T>& a, const Quat<T>& b)
{
    Quat<T> r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}
template <typename T>
__device__ __forceinline__ void qact(const Quat<T>& q, const T* p, T* o)  // so3.h:67-72
{
    T uv0 = q.y * p[2] - q.z * p[1], uv1 = q.z * p[0] - q.x * p[2], uv2 = q.x * p[1] - q.y * p[0];
    uv0 += uv0; uv1 += uv1; uv2 += uv2;
    const T o0 = p[0] + q.w * uv0 + (q.y * uv2 - q.z * uv1);
    const T o1 = p[1] + q.w * uv1 + (q.z * uv0 - q.x * uv2);
    const T o2 = p[2] + q.w * uv2 + (q.x * uv1 - q.y * uv0);
    o[0] = o0; o[1] = o1; o[2] = o2;
}
template <typename T>
__device__ __forceinline__ void qmat(const Quat<T>& q, T R[3][3])  // Eigen toRotationMatrix
{
    const T tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const T twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const T txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const T tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz;       R[0][2] = txz + twy;
    R[1][0] = txy + twz;       R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
    R[2][0] = txz - twy;       R[2][1] = tyz + twx;       R[2][2] = 1 - (txx + tyy);
}
template <typename T>
__device__ __forceinline__ void hat(const T* p, T M[3][3])
{
    M[0][0] = 0; M[0][1] = -p[2]; M[0][2] = p[1];
    M[1][0] = p[2]; M[1][1] = 0; M[1][2] = -p[0];
    M[2][0] = -p[1]; M[2][1] = p[0]; M[2][2] = 0;
}
template <typename T>
__device__ __forceinline__ void mm3(const T A[3][3], const T B[3][3], T C[3][3])
{
    T R[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C[i][j] = R[i][j];
}

// ---------------------------------------------------------------------------
template <typename T>
struct SO3 {
    static constexpr int K = 3, N = 4;
    Quat<T> q;

    __device__ static SO3 load(const T* d) { SO3 g; g.q = qnormalize(Quat<T>{d[0], d[1], d[2], d[3]}); return g; }
    __device__ void store(T* d) const { d[0] = q.x; d[1] = q.y; d[2] = q.z; d[3] = q.w; }
    __device__ SO3 inv() const { SO3 g; g.q = qnormalize(Quat<T>{-q.x, -q.y, -q.z, q.w}); return g; }
    __device__ SO3 mul(const SO3& o) const { SO3 g; g.q = qnormalize(qmul(q, o.q)); return g; }
    __device__ void act(const T* p, T* o) const { qact(q, p, o); }
    __device__ void act4(const T* p, T* o) const { qact(q, p, o); o[3] = p[3]; }
    __device__ void Adj(T A[K][K]) const { qmat(q, A); }
    __device__ void matrix4(T M[4][4]) const
    {
        T R[3][3];
        qmat(q, R);
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) M[i][j] = (i < 3 && j < 3) ? R[i][j] : (T)(i == j ? 1 : 0);
    }
    __device__ void projector(T* P) const  // so3.h:93-103, row-major N x N
    {
        for (int i = 0; i < 16; i++) P[i] = 0;
        const T v[3] = {-q.x, -q.y, -q.z};
        T H[3][3];
        hat(v, H);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) P[i * 4 + j] = (T)0.5 * ((i == j ? q.w : (T)0) + H[i][j]);
        for (int j = 0; j < 3; j++) P[12 + j] = (T)0.5 * v[j];
    }
    __device__ void Log(T* phi) const  // so3.h:127-163
    {
        const T sn = q.x * q.x + q.y * q.y + q.z * q.z, w = q.w;
        T f;
        const T eps = lie_eps<T>();
        if (sn < eps * eps) {
            f = (T)2 / w - (T)(2.0 / 3.0) * sn / (w * (w * w));
        } else {
            const T n = sqrt(sn);
            if (fabs(w) < eps) f = (w > (T)0 ? (T)3.14159265358979323846 : -(T)3.14159265358979323846) / n;
            else f = (T)2 * atan(n / w) / n;
        }
        phi[0] = f * q.x; phi[1] = f * q.y; phi[2] = f * q.z;
    }
    __device__ static SO3 Exp(const T* phi)  // so3.h:165-182
    {
        const T t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2], t = sqrt(t2);
        T im, re;
        if (t < lie_eps<T>()) {
            const T t4 = t2 * t2;
            im = (T)0.5 - (T)(1.0 / 48.0) * t2 + (T)(1.0 / 3840.0) * t4;
            re = (T)1 - (T)(1.0 / 8.0) * t2 + (T)(1.0 / 384.0) * t4;
        } else {
            im = sin((T)0.5 * t) / t;
            re = cos((T)0.5 * t);
        }
        SO3 g;
        g.q = qnormalize(Quat<T>{im * phi[0], im * phi[1], im * phi[2], re});
        return g;
    }
    __device__ static void left_jacobian(const T* phi, T J[3][3])  // so3.h:184-202
    {
        T Ph[3][3], Ph2[3][3];
        hat(phi, Ph);
        mm3(Ph, Ph, Ph2);
        const T t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2], t = sqrt(t2);
        const T c1 = t < lie_eps<T>() ? (T)0.5 - (T)(1.0 / 24.0) * t2 : ((T)1 - cos(t)) / t2;
        const T c2 = t < lie_eps<T>() ? (T)(1.0 / 6.0) - (T)(1.0 / 120.0) * t2 : (t - sin(t)) / (t2 * t);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) J[i][j] = (T)(i == j) + c1 * Ph[i][j] + c2 * Ph2[i][j];
    }
    __device__ static void left_jacobian_inverse(const T* phi, T J[3][3])  // so3.h:204-220
    {
        T Ph[3][3], Ph2[3][3];
        hat(phi, Ph);
        mm3(Ph, Ph, Ph2);
        const T t2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2], t = sqrt(t2), ht = (T)0.5 * t;
        const T c2 = t < lie_eps<T>() ? (T)(1.0 / 12.0) : ((T)1 - t * cos(ht) / ((T)2 * sin(ht))) / (t * t);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) J[i][j] = (T)(i == j) - (T)0.5 * Ph[i][j] + c2 * Ph2[i][j];
    }
    __device__ static void ad(const T* a, T A[3][3]) { hat(a, A); }
    __device__ static void act_jacobian(const T* p, T J[3][3])
    {
        const T m[3] = {-p[0], -p[1], -p[2]};
        hat(m, J);
    }
    __device__ static void act4_jacobian(const T* p, T J[4][3])
    {
        const T m[3] = {-p[0], -p[1], -p[2]};
        T H[3][3];
        hat(m, H);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) J[i][j] = H[i][j];
        for (int j = 0; j < 3; j++) J[3][j] = 0;
    }
};

// ---------------------------------------------------------------------------
template <typename T>
struct SE3 {
    static constexpr int K = 6, N = 7;
    SO3<T> so3;
    T t[3];

    __device__ static SE3 load(const T* d)
    {
        SE3 g;
        g.t[0] = d[0]; g.t[1] = d[1]; g.t[2] = d[2];
        g.so3 = SO3<T>::load(d + 3);
        return g;
    }
    __device__ void store(T* d) const { d[0] = t[0]; d[1] = t[1]; d[2] = t[2]; so3.store(d + 3); }
    __device__ SE3 inv() const  // se3.h:277-279
    {
        SE3 g;
        g.so3 = so3.inv();
        T tt[3];
        g.so3.act(t, tt);
        g.t[0] = -tt[0]; g.t[1] = -tt[1]; g.t[2] = -tt[2];
        return g;
    }
    __device__ SE3 mul(const SE3& o) const  // se3.h:286-288
    {
        SE3 g;
        g.so3 = so3.mul(o.so3);
        T tt[3];
        so3.act(o.t, tt);
        g.t[0] = t[0] + tt[0]; g.t[1] = t[1] + tt[1]; g.t[2] = t[2] + tt[2];
        return g;
    }
    __device__ void act(const T* p, T* o) const
    {
        so3.act(p, o);
        o[0] += t[0]; o[1] += t[1]; o[2] += t[2];
    }
    __device__ void act4(const T* p, T* o) const  // se3.h:294-297
    {
        T r[3];
        so3.act(p, r);
        o[0] = r[0] + t[0] * p[3];
        o[1] = r[1] + t[1] * p[3];
        o[2] = r[2] + t[2] * p[3];
        o[3] = p[3];
    }
    __device__ void Adj(T A[6][6]) const  // se3.h:299-308
    {
        T R[3][3], tx[3][3], tR[3][3];
        qmat(so3.q, R);
        hat(t, tx);
        mm3(tx, R, tR);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                A[i][j] = R[i][j]; A[i][j + 3] = tR[i][j];
                A[i + 3][j] = 0; A[i + 3][j + 3] = R[i][j];
            }
    }
    __device__ void matrix4(T M[4][4]) const
    {
        T R[3][3];
        qmat(so3.q, R);
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) M[i][j] = R[i][j];
            M[i][3] = t[i];
        }
        M[3][0] = 0; M[3][1] = 0; M[3][2] = 0; M[3][3] = 1;
    }
    __device__ void projector(T* P) const  // se3.h:355-363, 7x7 row-major
    {
        for (int i = 0; i < 49; i++) P[i] = 0;
        const T mt[3] = {-t[0], -t[1], -t[2]};
        T H[3][3];
        hat(mt, H);
        for (int i = 0; i < 3; i++) {
            P[i * 7 + i] = 1;
            for (int j = 0; j < 3; j++) P[i * 7 + 3 + j] = H[i][j];
        }
        T Pq[16];
        so3.projector(Pq);
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) P[(3 + i) * 7 + 3 + j] = Pq[i * 4 + j];
    }
    __device__ static void calcQ(const T* xi, T Qm[3][3])  // se3.h:385-414
    {
        T Ta[3][3], Ph[3][3];
        hat(xi, Ta);
        hat(xi + 3, Ph);
        const T th = sqrt(xi[3] * xi[3] + xi[4] * xi[4] + xi[5] * xi[5]);
        const T t2 = th * th, t4 = t2 * t2;
        const bool small = th < lie_eps<T>();
        const T c1 = small ? (T)(1.0 / 6.0) - (T)(1.0 / 120.0) * t2 : (th - sin(th)) / (t2 * th);
        const T c2 = small ? (T)(1.0 / 24.0) - (T)(1.0 / 720.0) * t2 : (t2 + 2 * cos(th) - 2) / (2 * t4);
        const T c3 = small ? (T)(1.0 / 120.0) - (T)(1.0 / 2520.0) * t2
                           : (2 * th - 3 * sin(th) + th * cos(th)) / (2 * t4 * th);
        T PT[3][3], TP[3][3], PTP[3][3], PP[3][3], PPT[3][3], TPP[3][3], PTPP[3][3], PPTP[3][3];
        mm3(Ph, Ta, PT); mm3(Ta, Ph, TP); mm3(PT, Ph, PTP); mm3(Ph, Ph, PP);
        mm3(PP, Ta, PPT); mm3(Ta, PP, TPP); mm3(PTP, Ph, PTPP); mm3(PPT, Ph, PPTP);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                Qm[i][j] = (T)0.5 * Ta[i][j] + c1 * (PT[i][j] + TP[i][j] + PTP[i][j]) +
                           c2 * (PPT[i][j] + TPP[i][j] - 3 * PTP[i][j]) + c3 * (PTPP[i][j] + PPTP[i][j]);
    }
    __device__ void Log(T* xi) const  // se3.h:365-373
    {
        T phi[3], Vi[3][3];
        so3.Log(phi);
        SO3<T>::left_jacobian_inverse(phi, Vi);
        for (int i = 0; i < 3; i++) xi[i] = Vi[i][0] * t[0] + Vi[i][1] * t[1] + Vi[i][2] * t[2];
        xi[3] = phi[0]; xi[4] = phi[1]; xi[5] = phi[2];
    }
    __device__ static SE3 Exp(const T* xi)  // se3.h:375-383
    {
        SE3 g;
        g.so3 = SO3<T>::Exp(xi + 3);
        T J[3][3];
        SO3<T>::left_jacobian(xi + 3, J);
        for (int i = 0; i < 3; i++) g.t[i] = J[i][0] * xi[0] + J[i][1] * xi[1] + J[i][2] * xi[2];
        return g;
    }
    __device__ static void left_jacobian(const T* xi, T J[6][6])  // se3.h:416-427
    {
        T Js[3][3], Qm[3][3];
        SO3<T>::left_jacobian(xi + 3, Js);
        calcQ(xi, Qm);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                J[i][j] = Js[i][j]; J[i][j + 3] = Qm[i][j];
                J[i + 3][j] = 0; J[i + 3][j + 3] = Js[i][j];
            }
    }
    __device__ static void left_jacobian_inverse(const T* xi, T J[6][6])  // se3.h:429-442
    {
        T Ji[3][3], Qm[3][3], A[3][3], B[3][3];
        SO3<T>::left_jacobian_inverse(xi + 3, Ji);
        calcQ(xi, Qm);
        mm3(Ji, Qm, A);
        mm3(A, Ji, B);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                J[i][j] = Ji[i][j]; J[i][j + 3] = -B[i][j];
                J[i + 3][j] = 0; J[i + 3][j + 3] = Ji[i][j];
            }
    }
    __device__ static void ad(const T* a, T A[6][6])  // se3.h:341-353
    {
        T Ta[3][3], Ph[3][3];
        hat(a, Ta);
        hat(a + 3, Ph);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                A[i][j] = Ph[i][j]; A[i][j + 3] = Ta[i][j];
                A[i + 3][j] = 0; A[i + 3][j + 3] = Ph[i][j];
            }
    }
    __device__ static void act_jacobian(const T* p, T J[3][6])
    {
        const T m[3] = {-p[0], -p[1], -p[2]};
        T H[3][3];
        hat(m, H);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) { J[i][j] = (T)(i == j); J[i][j + 3] = H[i][j]; }
    }
    __device__ static void act4_jacobian(const T* p, T J[4][6])
    {
        const T m[3] = {-p[0], -p[1], -p[2]};
        T H[3][3];
        hat(m, H);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) { J[i][j] = i == j ? p[3] : (T)0; J[i][j + 3] = H[i][j]; }
        for (int j = 0; j < 6; j++) J[3][j] = 0;
    }
};

// ---------------------------------------------------------------------------
// small dense helpers for the 4x4 / 7x7 tangent-space matrices
template <typename T, int K>
__device__ __forceinline__ void mmk(const T A[K][K], const T B[K][K], T C[K][K])
{
    T R[K][K];
    for (int i = 0; i < K; i++)
        for (int j = 0; j < K; j++) {
            T s = 0;
            for (int k = 0; k < K; k++) s += A[i][k] * B[k][j];
            R[i][j] = s;
        }
    for (int i = 0; i < K; i++)
        for (int j = 0; j < K; j++) C[i][j] = R[i][j];
}
template <typename T>
__device__ __forceinline__ void inv3(const T A[3][3], T B[3][3])  // cofactors / determinant (Eigen's 3x3 inverse)
{
    const T c00 = A[1][1] * A[2][2] - A[1][2] * A[2][1];
    const T c01 = A[1][2] * A[2][0] - A[1][0] * A[2][2];
    const T c02 = A[1][0] * A[2][1] - A[1][1] * A[2][0];
    const T det = A[0][0] * c00 + A[0][1] * c01 + A[0][2] * c02;
    const T id = (T)1 / det;
    B[0][0] = c00 * id; B[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) * id; B[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) * id;
    B[1][0] = c01 * id; B[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) * id; B[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) * id;
    B[2][0] = c02 * id; B[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) * id; B[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) * id;
}

// ---------------------------------------------------------------------------
// RxSO3: rotation and positive scale, data [qx,qy,qz,qw,s] (rxso3.h)
template <typename T>
struct RxSO3 {
    static constexpr int K = 4, N = 5;
    SO3<T> so3;
    T s;

    __device__ static RxSO3 load(const T* d) { RxSO3 g; g.so3 = SO3<T>::load(d); g.s = d[4]; return g; }
    __device__ void store(T* d) const { so3.store(d); d[4] = s; }
    __device__ RxSO3 inv() const { RxSO3 g; g.so3 = so3.inv(); g.s = (T)1 / s; return g; }
    __device__ RxSO3 mul(const RxSO3& o) const { RxSO3 g; g.so3 = so3.mul(o.so3); g.s = s * o.s; return g; }
    __device__ void act(const T* p, T* o) const
    {
        so3.act(p, o);
        o[0] *= s; o[1] *= s; o[2] *= s;
    }
    __device__ void act4(const T* p, T* o) const { act(p, o); o[3] = p[3]; }
    __device__ void Adj(T A[4][4]) const  // rotation block, scale untouched
    {
        T R[3][3];
        qmat(so3.q, R);
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) A[i][j] = (i < 3 && j < 3) ? R[i][j] : (T)(i == j);
    }
    __device__ void matrix4(T M[4][4]) const
    {
        T R[3][3];
        qmat(so3.q, R);
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) M[i][j] = (i < 3 && j < 3) ? s * R[i][j] : (T)(i == j);
    }
    __device__ void projector(T* P) const  // rxso3.h orthogonal_projector, 5x5 row-major
    {
        T Pq[16];
        so3.projector(Pq);
        for (int i = 0; i < 25; i++) P[i] = 0;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 3; j++) P[i * 5 + j] = Pq[i * 4 + j];
        P[4 * 5 + 3] = s;
    }
    __device__ void Log(T* ps) const
    {
        so3.Log(ps);
        ps[3] = log(s);
    }
    __device__ static RxSO3 Exp(const T* ps)
    {
        RxSO3 g;
        g.so3 = SO3<T>::Exp(ps);
        g.s = exp(ps[3]);
        return g;
    }
    // W(phi, sigma): the translation part of Sim3's exp (rxso3.h calcW)
    __device__ static void calcW(const T* ps, T W[3][3])
    {
        T Ph[3][3], Ph2[3][3];
        hat(ps, Ph);
        mm3(Ph, Ph, Ph2);
        const T sigma = ps[3], theta = sqrt(ps[0] * ps[0] + ps[1] * ps[1] + ps[2] * ps[2]), sc = exp(sigma);
        const T eps = lie_eps<T>(), one = 1, half = (T)0.5;
        T A, B, C;
        if (fabs(sigma) < eps) {
            C = one;
            if (fabs(theta) < eps) {
                A = half;
                B = (T)(1. / 6.);
            } else {
                const T t2 = theta * theta;
                A = (one - cos(theta)) / t2;
                B = (theta - sin(theta)) / (t2 * theta);
            }
        } else {
            C = (sc - one) / sigma;
            if (fabs(theta) < eps) {
                const T s2 = sigma * sigma;
                A = ((sigma - one) * sc + one) / s2;
                B = (sc * half * s2 + sc - one - sigma * sc) / (s2 * sigma);
            } else {
                const T t2 = theta * theta, a = sc * sin(theta), b = sc * cos(theta), c = t2 + sigma * sigma;
                A = (a * sigma + (one - b) * theta) / (theta * c);
                B = (C - ((b - one) * sigma + a * theta) / c) * one / t2;
            }
        }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) W[i][j] = A * Ph[i][j] + B * Ph2[i][j] + (i == j ? C : (T)0);
    }
    __device__ static void left_jacobian(const T* ps, T J[4][4])
    {
        T Js[3][3];
        SO3<T>::left_jacobian(ps, Js);
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) J[i][j] = (i < 3 && j < 3) ? Js[i][j] : (T)(i == j);
    }
    __device__ static void left_jacobian_inverse(const T* ps, T J[4][4])
    {
        T Js[3][3];
        SO3<T>::left_jacobian_inverse(ps, Js);
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) J[i][j] = (i < 3 && j < 3) ? Js[i][j] : (T)(i == j);
    }
    __device__ static void ad(const T* a, T A[4][4])
    {
        T H[3][3];
        hat(a, H);
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) A[i][j] = (i < 3 && j < 3) ? H[i][j] : (T)0;
    }
    __device__ static void act_jacobian(const T* p, T J[3][4])
    {
        const T m[3] = {-p[0], -p[1], -p[2]};
        T H[3][3];
        hat(m, H);
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) J[i][j] = H[i][j];
            J[i][3] = p[i];
        }
    }
    __device__ static void act4_jacobian(const T* p, T J[4][4])
    {
        const T m[3] = {-p[0], -p[1], -p[2]};
        T H[3][3];
        hat(m, H);
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) J[i][j] = H[i][j];
            J[i][3] = p[i];
        }
        for (int j = 0; j < 4; j++) J[3][j] = 0;
    }
};

// ---------------------------------------------------------------------------
// Sim3: similarity, data [tx,ty,tz,qx,qy,qz,qw,s] (sim3.h)
template <typename T>
struct Sim3 {
    static constexpr int K = 7, N = 8;
    RxSO3<T> r;
    T t[3];

    __device__ static Sim3 load(const T* d)
    {
        Sim3 g;
        g.t[0] = d[0]; g.t[1] = d[1]; g.t[2] = d[2];
        g.r = RxSO3<T>::load(d + 3);
        return g;
    }
    __device__ void store(T* d) const { d[0] = t[0]; d[1] = t[1]; d[2] = t[2]; r.store(d + 3); }
    __device__ Sim3 inv() const
    {
        Sim3 g;
        g.r = r.inv();
        T tt[3];
        g.r.act(t, tt);
        g.t[0] = -tt[0]; g.t[1] = -tt[1]; g.t[2] = -tt[2];
        return g;
    }
    __device__ Sim3 mul(const Sim3& o) const
    {
        Sim3 g;
        g.r = r.mul(o.r);
        T tt[3];
        r.act(o.t, tt);
        g.t[0] = t[0] + tt[0]; g.t[1] = t[1] + tt[1]; g.t[2] = t[2] + tt[2];
        return g;
    }
    __device__ void act(const T* p, T* o) const
    {
        r.act(p, o);
        o[0] += t[0]; o[1] += t[1]; o[2] += t[2];
    }
    __device__ void act4(const T* p, T* o) const
    {
        T q[3];
        r.act(p, q);
        o[0] = q[0] + p[3] * t[0];
        o[1] = q[1] + p[3] * t[1];
        o[2] = q[2] + p[3] * t[2];
        o[3] = p[3];
    }
    __device__ void matrix4(T M[4][4]) const
    {
        r.matrix4(M);
        M[0][3] = t[0]; M[1][3] = t[1]; M[2][3] = t[2];
    }
    __device__ void Adj(T A[7][7]) const  // sim3.h Adj
    {
        T R[3][3], tx[3][3], tR[3][3];
        qmat(r.so3.q, R);
        hat(t, tx);
        mm3(tx, R, tR);
        for (int i = 0; i < 7; i++)
            for (int j = 0; j < 7; j++) A[i][j] = (T)(i == j);
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) {
                A[i][j] = r.s * R[i][j];
                A[i][j + 3] = tR[i][j];
                A[i + 3][j + 3] = R[i][j];
            }
            A[i][6] = -t[i];
        }
    }
    __device__ void projector(T* P) const  // sim3.h orthogonal_projector, 8x8 row-major
    {
        for (int i = 0; i < 64; i++) P[i] = 0;
        const T mt[3] = {-t[0], -t[1], -t[2]};
        T H[3][3];
        hat(mt, H);
        for (int i = 0; i < 3; i++) {
            P[i * 8 + i] = 1;
            for (int j = 0; j < 3; j++) P[i * 8 + 3 + j] = H[i][j];
            P[i * 8 + 6] = t[i];
        }
        T Pr[25];
        r.projector(Pr);
        for (int i = 0; i < 5; i++)
            for (int j = 0; j < 5; j++) P[(3 + i) * 8 + 3 + j] = Pr[i * 5 + j];
    }
    __device__ void Log(T* xi) const  // [W^-1 t, phi, sigma]
    {
        r.Log(xi + 3);
        T W[3][3], Wi[3][3];
        RxSO3<T>::calcW(xi + 3, W);
        inv3(W, Wi);
        for (int i = 0; i < 3; i++) xi[i] = Wi[i][0] * t[0] + Wi[i][1] * t[1] + Wi[i][2] * t[2];
    }
    __device__ static Sim3 Exp(const T* xi)
    {
        Sim3 g;
        g.r = RxSO3<T>::Exp(xi + 3);
        T W[3][3];
        RxSO3<T>::calcW(xi + 3, W);
        for (int i = 0; i < 3; i++) g.t[i] = W[i][0] * xi[0] + W[i][1] * xi[1] + W[i][2] * xi[2];
        return g;
    }
    __device__ static void ad(const T* a, T A[7][7])  // sim3.h adj
    {
        T Ta[3][3], Ph[3][3];
        hat(a, Ta);
        hat(a + 3, Ph);
        for (int i = 0; i < 7; i++)
            for (int j = 0; j < 7; j++) A[i][j] = 0;
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) {
                A[i][j] = Ph[i][j] + (i == j ? a[6] : (T)0);
                A[i][j + 3] = Ta[i][j];
                A[i + 3][j + 3] = Ph[i][j];
            }
            A[i][6] = -a[i];
        }
    }
    // sim3.h left_jacobian: I + X/2 + X^2/6 + X^3/24 + X^4/120 (its 1/720 X^5
    // term sits after the statement's semicolon in the reference: not applied)
    __device__ static void left_jacobian(const T* xi, T J[7][7])
    {
        T X[7][7], X2[7][7], X3[7][7], X4[7][7];
        ad(xi, X);
        mmk<T, 7>(X, X, X2);
        mmk<T, 7>(X, X2, X3);
        mmk<T, 7>(X2, X2, X4);
        for (int i = 0; i < 7; i++)
            for (int j = 0; j < 7; j++)
                J[i][j] = (T)(i == j) + (T)(1.0 / 2.0) * X[i][j] + (T)(1.0 / 6.0) * X2[i][j] +
                          (T)(1.0 / 24.0) * X3[i][j] + (T)(1.0 / 120.0) * X4[i][j];
    }
    __device__ static void left_jacobian_inverse(const T* xi, T J[7][7])
    {
        T X[7][7], X2[7][7], X4[7][7];
        ad(xi, X);
        mmk<T, 7>(X, X, X2);
        mmk<T, 7>(X2, X2, X4);
        for (int i = 0; i < 7; i++)
            for (int j = 0; j < 7; j++)
                J[i][j] = (T)(i == j) - (T)(1.0 / 2.0) * X[i][j] + (T)(1.0 / 12.0) * X2[i][j] -
                          (T)(1.0 / 720.0) * X4[i][j];
    }
    __device__ static void act_jacobian(const T* p, T J[3][7])
    {
        const T m[3] = {-p[0], -p[1], -p[2]};
        T H[3][3];
        hat(m, H);
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) { J[i][j] = (T)(i == j); J[i][j + 3] = H[i][j]; }
            J[i][6] = p[i];
        }
    }
    __device__ static void act4_jacobian(const T* p, T J[4][7])
    {
        const T m[3] = {-p[0], -p[1], -p[2]};
        T H[3][3];
        hat(m, H);
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) { J[i][j] = i == j ? p[3] : (T)0; J[i][j + 3] = H[i][j]; }
            J[i][6] = p[i];
        }
        for (int j = 0; j < 7; j++) J[3][j] = 0;
    }
};

}  // namespace lie
}  // namespace dpvo

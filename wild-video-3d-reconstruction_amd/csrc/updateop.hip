// updateop.hip -- native glue of the learned update operator (gfx950).
//
// SoftAgg (reference dpvo/blocks.py:40-48) aggregates edge features over
// groups of edges sharing a key with torch_scatter 2.1.2's scatter_softmax +
// scatter_sum.  torch_scatter is absent on ROCm and ATen's scatter_reduce
// "amax" path is a same-address atomic storm (~2.4 ms per call at C3), so the
// whole softmax-weighted sum is one streaming pass here:
//
//   1. CSR of the group labels: count (atomics on G counters), one-block
//      exclusive scan, fill (atomic cursor per group);
//   2. one wave64 per (group, 128-channel slice): the wave sorts its edge
//      list in LDS (ascending edge index -> deterministic fp32 sums), then
//      streams the f/s rows 8 edges at a time with a batched online softmax
//      (one rescale per 8 edges), and writes y = acc / (l + eps).
//
// Bytes per edge: 2 rows x D x sizeof(T) read once (+12 B of CSR traffic);
// the kernel is HBM-bound like the GEMMs around it.
#include <climits>

#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "common.hpp"

namespace dpvo {
namespace {

constexpr int SA_WAVES = 4;          // waves per block in the reduce kernel
constexpr int SA_UNROLL = 8;         // edges in flight per online-softmax step
constexpr int SA_CAP = DPVO_SOFTAGG_SORT_CAP;

struct SaLayout {
    int64_t count, offs, cursor, perm, total;
};

inline int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }

SaLayout sa_layout(int64_t E, int64_t G)
{
    SaLayout L;
    int64_t o = 0;
    L.count = o;  o += align256(4 * G);
    L.offs = o;   o += align256(4 * (G + 1));
    L.cursor = o; o += align256(4 * G);
    L.perm = o;   o += align256(4 * E);
    L.total = o;
    return L;
}

__global__ __launch_bounds__(256) void sa_count_kernel(const int64_t* __restrict__ group, int64_t E, int64_t G,
                                                       int* __restrict__ count)
{
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = group[e];
        if (g >= 0 && g < G) atomicAdd(&count[g], 1);
    }
}

// exclusive scan of count[0..G) -> offs[0..G], cursor = offs (single block)
__global__ __launch_bounds__(1024) void sa_scan_kernel(const int* __restrict__ count, int64_t G,
                                                       int* __restrict__ offs, int* __restrict__ cursor)
{
    __shared__ int part[1024];
    const int tid = threadIdx.x;
    const int64_t per = (G + 1023) / 1024;
    const int64_t g0 = tid * per, g1 = min(G, g0 + per);
    int sum = 0;
    for (int64_t g = g0; g < g1; g++) sum += count[g];
    part[tid] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const int add = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += add;
        __syncthreads();
    }
    int base = part[tid] - sum;
    for (int64_t g = g0; g < g1; g++) {
        offs[g] = base;
        cursor[g] = base;
        base += count[g];
    }
    if (tid == 1023) offs[G] = part[1023];
}

__global__ __launch_bounds__(256) void sa_fill_kernel(const int64_t* __restrict__ group, int64_t E, int64_t G,
                                                      int* __restrict__ cursor, int* __restrict__ perm)
{
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = group[e];
        if (g < 0 || g >= G) continue;
        perm[atomicAdd(&cursor[g], 1)] = (int)e;
    }
}

template <typename T> struct Pair;
template <> struct Pair<half_t> {
    typedef half2_t V;
    static __device__ __forceinline__ float2_t load(const half_t* p) { V v = *(const V*)p; return {(float)v.x, (float)v.y}; }
    static __device__ __forceinline__ void store(half_t* p, float2_t v) { *(V*)p = V{(half_t)v.x, (half_t)v.y}; }
};
template <> struct Pair<float> {
    static __device__ __forceinline__ float2_t load(const float* p) { return *(const float2_t*)p; }
    static __device__ __forceinline__ void store(float* p, float2_t v) { *(float2_t*)p = v; }
};
template <> struct Pair<double> {
    static __device__ __forceinline__ float2_t load(const double* p) { return {(float)p[0], (float)p[1]}; }
    static __device__ __forceinline__ void store(double* p, float2_t v) { p[0] = v.x; p[1] = v.y; }
};

// Online softmax-weighted sum over rows order[i0 .. i1) for the lane's two
// channels, in SA_UNROLL batches from i0 (sa_reduce_csr_kernel's arithmetic).
template <typename T>
__device__ __forceinline__ void sa_online(const T* __restrict__ f, int64_t ldf, const T* __restrict__ s, int64_t lds,
                                          const int* order, int i0b, int i1, int cc, float2_t& m, float2_t& l,
                                          float2_t& acc)
{
    for (int i0 = i0b; i0 < i1; i0 += SA_UNROLL) {
        float2_t sv[SA_UNROLL], fv[SA_UNROLL];
#pragma unroll
        for (int u = 0; u < SA_UNROLL; u++) {
            const int64_t e = order[min(i0 + u, i1 - 1)];
            sv[u] = Pair<T>::load(s + e * lds + cc);
            fv[u] = Pair<T>::load(f + e * ldf + cc);
        }
        float2_t mb = m;
#pragma unroll
        for (int u = 0; u < SA_UNROLL; u++)
            if (i0 + u < i1) {
                mb.x = fmaxf(mb.x, sv[u].x);
                mb.y = fmaxf(mb.y, sv[u].y);
            }
        const float ax = __expf(m.x - mb.x), ay = __expf(m.y - mb.y);
        l.x *= ax; l.y *= ay; acc.x *= ax; acc.y *= ay;
#pragma unroll
        for (int u = 0; u < SA_UNROLL; u++)
            if (i0 + u < i1) {
                const float px = __expf(sv[u].x - mb.x), py = __expf(sv[u].y - mb.y);
                l.x += px; l.y += py;
                acc.x += px * fv[u].x; acc.y += py * fv[u].y;
            }
        m = mb;
    }
}

// One wave per (group, 128-channel slice).  Lane owns channels c, c+1.
template <typename T>
__global__ __launch_bounds__(64 * SA_WAVES) void sa_reduce_kernel(const T* __restrict__ f, int64_t ldf,
                                                                  const T* __restrict__ s, int64_t lds,
                                                                  const int* __restrict__ offs,
                                                                  const int* __restrict__ perm, int64_t G, int D,
                                                                  int slices, float eps, T* __restrict__ y)
{
    __shared__ int lst[SA_WAVES][2][SA_CAP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t task = (int64_t)blockIdx.x * SA_WAVES + w;
    if (task >= G * slices) return;
    const int64_t g = task / slices;
    const int c = (int)(task % slices) * 128 + 2 * lane;
    const int b = offs[g], S = offs[g + 1] - b;
    const bool act = c < D;
    const int cc = act ? c : 0;
    float2_t m = {-INFINITY, -INFINITY}, l = {0.f, 0.f}, acc = {0.f, 0.f};

    // ascending edge order within the group (ranks of distinct edge ids).  The
    // online pass is instantiated once per source of the order -- the wave's
    // LDS list or global perm -- never through one pointer that may be either:
    // such a generic pointer compiles to flat loads, and a flat load of the
    // LDS list is not ordered after the ds_write that stored it (another lane's
    // rank), so the pass could read a stale slot of the sorted list -- the
    // round-5 intermittent "csr != dense" SoftAgg mismatch.
    if (S <= SA_CAP) {
        int* raw = lst[w][0];
        int* srt = lst[w][1];
        for (int i = lane; i < S; i += 64) raw[i] = perm[b + i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int i = lane; i < S; i += 64) {
            const int v = raw[i];
            int r = 0;
            for (int j = 0; j < S; j++) r += raw[j] < v;
            srt[r] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        sa_online<T>(f, ldf, s, lds, srt, 0, S, cc, m, l, acc);
    } else {
        sa_online<T>(f, ldf, s, lds, perm + b, 0, S, cc, m, l, acc);
    }
    if (act) Pair<T>::store(y + g * (int64_t)D + c, float2_t{acc.x / (l.x + eps), acc.y / (l.y + eps)});
}

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void gather_rows_kernel(const TI* __restrict__ x, int64_t ldx, int64_t rows,
                                                          const int64_t* __restrict__ idx, int64_t n, int D,
                                                          TO* __restrict__ out)
{
    // one wave per output row, 2 channels per lane per step
    const int lane = threadIdx.x & 63;
    for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; r < n;
         r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const int64_t src = idx[r];
        const bool ok = src >= 0 && src < rows;
        for (int c = 2 * lane; c < D; c += 128) {
            float2_t v = {0.f, 0.f};
            if (ok) v = Pair<TI>::load(x + src * ldx + c);
            Pair<TO>::store(out + r * (int64_t)D + c, v);
        }
    }
}

template <typename TI>
int gather_dispatch_out(const TI* x, int64_t ldx, int64_t rows, const int64_t* idx, int64_t n, int D, int out_dtype,
                        void* out, hipStream_t s)
{
    const unsigned grid = grid_for(n * 64, 256, 8192);
    switch (out_dtype) {
    case DPVO_F16: hipLaunchKernelGGL((gather_rows_kernel<TI, half_t>), dim3(grid), dim3(256), 0, s, x, ldx, rows, idx, n, D, (half_t*)out); break;
    case DPVO_F32: hipLaunchKernelGGL((gather_rows_kernel<TI, float>), dim3(grid), dim3(256), 0, s, x, ldx, rows, idx, n, D, (float*)out); break;
    case DPVO_F64: hipLaunchKernelGGL((gather_rows_kernel<TI, double>), dim3(grid), dim3(256), 0, s, x, ldx, rows, idx, n, D, (double*)out); break;
    default: return -1;
    }
    return 0;
}

// ---------------------------------------------------------------------------
// sync-free group-by (torch.unique(key, return_inverse=True) + CSR)
// ---------------------------------------------------------------------------
// keys as unsigned radix-sort keys: 32-bit when the caller's bound fits
// (fewer radix passes), 64-bit otherwise (any int64 key; negative keys sort
// after the non-negative ones but still group by equality)
template <typename K>
__global__ __launch_bounds__(256) void gb_keys_kernel(const int64_t* __restrict__ key, int64_t n,
                                                      K* __restrict__ kout, int* __restrict__ idx)
{
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        kout[e] = (K)key[e];
        idx[e] = (int)e;
    }
}

template <typename K>
__global__ __launch_bounds__(256) void gb_flags_kernel(const K* __restrict__ sk, int64_t n, int* __restrict__ flag)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        flag[i] = (i == 0 || sk[i] != sk[i - 1]) ? 1 : 0;
}

__global__ __launch_bounds__(256) void gb_finish_kernel(const int* __restrict__ flag, const int* __restrict__ incl,
                                                        const int* __restrict__ perm, int64_t n,
                                                        int64_t* __restrict__ gid, int* __restrict__ offs,
                                                        int64_t* __restrict__ groups)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int r = incl[i] - 1;
        gid[perm[i]] = r;
        if (flag[i]) offs[r] = (int)i;
        if (i == n - 1) {
            offs[r + 1] = (int)n;
            *groups = r + 1;
        }
    }
}

struct GbLayout {
    int64_t k_in, k_out, v_in, flag, incl, tmp, tmp_bytes, total;
};

size_t gb_tmp_bytes(int64_t n)
{
    size_t a = 0, a64 = 0, b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (uint32_t*)nullptr, (uint32_t*)nullptr, (int*)nullptr,
                                             (int*)nullptr, (int)n);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a64, (uint64_t*)nullptr, (uint64_t*)nullptr, (int*)nullptr,
                                             (int*)nullptr, (int)n);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, (int*)nullptr, (int*)nullptr, (int)n);
    return std::max(std::max(a, a64), b);
}

GbLayout gb_layout(int64_t n)
{
    GbLayout L;
    int64_t o = 0;
    L.k_in = o;  o += align256(8 * n);
    L.k_out = o; o += align256(8 * n);
    L.v_in = o;  o += align256(4 * n);
    L.flag = o;  o += align256(4 * n);
    L.incl = o;  o += align256(4 * n);
    L.tmp = o;
    L.tmp_bytes = (int64_t)gb_tmp_bytes(n);
    o += align256(L.tmp_bytes);
    L.total = o;
    return L;
}

// Counting-sort group-by for keys bounded by 2^key_bits <= 2^22 (the tracker's
// kk < N M and its dense (ii, jj) pair key): a histogram with atomic slots, one
// exclusive scan over the bins carrying (start, group index) together, a
// scatter, and a per-group fix-up that restores ascending edge order inside
// each group (the atomic slots are arrival order) -- the same outputs as the
// stable radix sort, in 5 launches instead of ~12 (the radix path's merge
// passes, flags, scan and finish kernels).
constexpr int CB_MAX_BITS = 22;

struct CbLayout {
    int64_t hist, pre, slot, ptmp, tmp, tmp_bytes, total;
};

struct CbCombine {
    __host__ __device__ int64_t operator()(int c) const { return (int64_t)c | ((int64_t)(c > 0) << 32); }
};

CbLayout cb_layout(int64_t n, int key_bits)
{
    const int64_t B = int64_t(1) << key_bits;
    CbLayout L;
    int64_t o = 0;
    L.hist = o; o += align256(4 * B);
    L.pre = o;  o += align256(8 * B);
    L.slot = o; o += align256(4 * n);
    L.ptmp = o; o += align256(4 * n);
    L.tmp = o;
    size_t tb = 0;
    hipcub::TransformInputIterator<int64_t, CbCombine, const int*> it(nullptr, CbCombine());
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, it, (int64_t*)nullptr, (int)B);
    L.tmp_bytes = (int64_t)tb;
    o += align256(L.tmp_bytes);
    L.total = o;
    return L;
}

// runs of equal keys inside a wave take one atomic per run (the run head's),
// so bins hit by many consecutive edges do not serialise on one address.
// Called by whole waves (uniform trip counts); valid lanes are a prefix.
__device__ __forceinline__ int cb_run_slot(uint32_t k, bool valid, int lane, int* __restrict__ hist)
{
    const uint32_t prev = __shfl_up(k, 1);
    const bool head = valid && (lane == 0 || prev != k);
    const uint64_t hm = __ballot(head), vm = __ballot(valid);
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int hl = 63 - __clzll(hm & upto);                  // my run's head lane
    const uint64_t above = hm & ~upto;
    const int end = above ? __ffsll((long long)above) - 1 : 64 - __clzll(vm);
    int base = 0;
    if (head) base = atomicAdd(&hist[k], end - lane);
    base = __shfl(base, valid ? hl : 0);
    return base + (lane - hl);
}

__global__ __launch_bounds__(256) void cb_hist_kernel(const int64_t* __restrict__ key, int64_t n, uint32_t mask,
                                                      int* __restrict__ hist, int* __restrict__ slot)
{
    const int lane = threadIdx.x & 63;
    for (int64_t e0 = blockIdx.x * (int64_t)blockDim.x; e0 < n; e0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = e0 + threadIdx.x;   // uniform trip count: whole waves stay converged
        const bool valid = e < n;
        const uint32_t k = valid ? (uint32_t)key[e] & mask : 0xffffffffu;
        const int s = cb_run_slot(k, valid, lane, hist);
        if (valid) slot[e] = s;
    }
}

__global__ __launch_bounds__(256) void cb_scatter_kernel(const int64_t* __restrict__ key, int64_t n, uint32_t mask,
                                                         const int* __restrict__ hist, const int64_t* __restrict__ pre,
                                                         const int* __restrict__ slot, int* __restrict__ ptmp,
                                                         int64_t* __restrict__ gid, int* __restrict__ offs,
                                                         int64_t* __restrict__ groups)
{
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = pre[(uint32_t)key[e] & mask];
        const int start = (int)(p & 0xffffffff), g = (int)(p >> 32), s = slot[e];
        ptmp[start + s] = (int)e;
        gid[e] = g;
        if (s == 0) offs[g] = start;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int64_t last = pre[mask] + CbCombine()(hist[mask]);
        const int64_t G = last >> 32;
        *groups = G;
        offs[G] = (int)n;
    }
}

// one wave per group: members back into ascending edge order (ranks by
// comparison; edge ids are distinct, so the ranks are a permutation).  Groups
// of <= 64 rank in registers (readlane broadcasts), up to CB_CAP members
// through the wave's LDS slice (16-byte broadcast reads), larger ones from
// global memory (L2).
constexpr int CB_CAP = 2048;
constexpr int CB_WAVES = 4;

__device__ __forceinline__ void cb_fix_group(int64_t g, const int* __restrict__ ptmp, const int* __restrict__ offs,
                                             const int64_t* __restrict__ gid, int64_t n, int* __restrict__ perm,
                                             int* __restrict__ mine, int lane)
{
    const int b = offs[g], S = offs[g + 1] - b;
    if (S <= 64) {
        const int v = lane < S ? ptmp[b + lane] : INT_MAX;
        int rank = 0;
        for (int j = 0; j < S; j++) rank += __builtin_amdgcn_readlane(v, j) < v;
        if (lane < S) perm[b + rank] = v;
    } else if (S <= CB_CAP) {
        for (int i = lane; i < S; i += 64) mine[i] = ptmp[b + i];
        for (int i = S + lane; i < ((S + 3) & ~3); i += 64) mine[i] = INT_MAX;   // pad the last int4
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int i = lane; i < S; i += 64) {
            const int v = mine[i];
            int rank = 0;
            for (int j = 0; j < S; j += 4) {
                const int4 q = *(const int4*)(mine + j);
                rank += (q.x < v) + (q.y < v) + (q.z < v) + (q.w < v);
            }
            perm[b + rank] = v;
        }
        __builtin_amdgcn_wave_barrier();   // every lane's reads before the next group's writes
    } else {
        // more than CB_CAP members: they are the edges e with gid[e] == g, so a
        // scan of gid over [first member, last member] in ascending e emits
        // them in order -- O(span / 64) per group, at most n / CB_CAP such
        // groups (a rank by comparison would be O(S^2))
        int lo = INT_MAX, hi = -1;
        for (int i = lane; i < S; i += 64) {
            const int v = ptmp[b + i];
            lo = min(lo, v);
            hi = max(hi, v);
        }
        for (int o = 32; o > 0; o >>= 1) {
            lo = min(lo, __shfl_xor(lo, o));
            hi = max(hi, __shfl_xor(hi, o));
        }
        int w = b;
        for (int64_t e0 = lo; e0 <= hi; e0 += 64) {
            const int64_t e = e0 + lane;
            const bool m = e <= hi && e < n && gid[e] == g;
            const uint64_t bal = __ballot(m);
            if (m) perm[w + __popcll(bal & ((1ull << lane) - 1))] = (int)e;
            w += __popcll(bal);
        }
    }
}

__global__ __launch_bounds__(64 * CB_WAVES) void cb_fix_kernel(const int* __restrict__ ptmp,
                                                               const int* __restrict__ offs,
                                                               const int64_t* __restrict__ groups,
                                                               const int64_t* __restrict__ gid, int64_t n,
                                                               int* __restrict__ perm)
{
    __shared__ __attribute__((aligned(16))) int buf[CB_WAVES][CB_CAP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t G = *groups;
    for (int64_t g = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; g < G;
         g += ((int64_t)gridDim.x * blockDim.x) >> 6)
        cb_fix_group(g, ptmp, offs, gid, n, perm, buf[w], lane);
}

// SoftAgg over a prebuilt CSR whose group count lives on the device.  Group
// members are already in ascending edge order (stable sort): no LDS sort.
template <typename T>
__global__ __launch_bounds__(256) void sa_reduce_csr_kernel(const T* __restrict__ f, int64_t ldf,
                                                            const T* __restrict__ s, int64_t lds,
                                                            const int* __restrict__ offs,
                                                            const int* __restrict__ perm,
                                                            const int64_t* __restrict__ groups, int D, int slices,
                                                            float eps, T* __restrict__ y)
{
    const int lane = threadIdx.x & 63;
    const int64_t ntask = *groups * slices;
    for (int64_t task = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; task < ntask;
         task += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const int64_t g = task / slices;
        const int c = (int)(task % slices) * 128 + 2 * lane;
        const int b = offs[g], S = offs[g + 1] - b;
        const int* order = perm + b;
        const bool act = c < D;
        const int cc = act ? c : 0;
        float2_t m = {-INFINITY, -INFINITY}, l = {0.f, 0.f}, acc = {0.f, 0.f};
        for (int i0 = 0; i0 < S; i0 += SA_UNROLL) {
            float2_t sv[SA_UNROLL], fv[SA_UNROLL];
#pragma unroll
            for (int u = 0; u < SA_UNROLL; u++) {
                const int64_t e = order[min(i0 + u, S - 1)];
                sv[u] = Pair<T>::load(s + e * lds + cc);
                fv[u] = Pair<T>::load(f + e * ldf + cc);
            }
            float2_t mb = m;
#pragma unroll
            for (int u = 0; u < SA_UNROLL; u++)
                if (i0 + u < S) {
                    mb.x = fmaxf(mb.x, sv[u].x);
                    mb.y = fmaxf(mb.y, sv[u].y);
                }
            const float ax = __expf(m.x - mb.x), ay = __expf(m.y - mb.y);
            l.x *= ax; l.y *= ay; acc.x *= ax; acc.y *= ay;
#pragma unroll
            for (int u = 0; u < SA_UNROLL; u++)
                if (i0 + u < S) {
                    const float px = __expf(sv[u].x - mb.x), py = __expf(sv[u].y - mb.y);
                    l.x += px; l.y += py;
                    acc.x += px * fv[u].x; acc.y += py * fv[u].y;
                }
            m = mb;
        }
        if (act) Pair<T>::store(y + g * (int64_t)D + c, float2_t{acc.x / (l.x + eps), acc.y / (l.y + eps)});
    }
}

// sa_reduce_csr_kernel with a workgroup per (group, 128-channel slice): groups
// of at least SA_SPLIT rows are cut into four contiguous row ranges, one per
// wave, whose (max, sum, weighted sum) states are merged in wave order -- the
// long frame-pair groups (~190 rows at C3) run four times shorter chains of
// dependent loads.  Shorter groups run on wave 0 alone with exactly
// sa_reduce_csr_kernel's arithmetic (same bits).  Deterministic either way.
constexpr int SA_SPLIT = 64;
template <typename T>
__global__ __launch_bounds__(256) void sa_reduce_csr_split_kernel(const T* __restrict__ f, int64_t ldf,
                                                                  const T* __restrict__ s, int64_t lds,
                                                                  const int* __restrict__ offs,
                                                                  const int* __restrict__ perm,
                                                                  const int64_t* __restrict__ groups, int D,
                                                                  int slices, float eps, T* __restrict__ y)
{
    __shared__ float2_t st[4][3][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t ntask = *groups * slices;
    for (int64_t task = blockIdx.x; task < ntask; task += gridDim.x) {
        const int64_t g = task / slices;
        const int c = (int)(task % slices) * 128 + 2 * lane;
        const int b = offs[g], S = offs[g + 1] - b;
        const int* order = perm + b;
        const bool act = c < D;
        const int cc = act ? c : 0;
        float2_t m = {-INFINITY, -INFINITY}, l = {0.f, 0.f}, acc = {0.f, 0.f};
        if (S < SA_SPLIT) {
            if (wave == 0) {
                sa_online<T>(f, ldf, s, lds, order, 0, S, cc, m, l, acc);
                if (act) Pair<T>::store(y + g * (int64_t)D + c, float2_t{acc.x / (l.x + eps), acc.y / (l.y + eps)});
            }
            continue;   // S is uniform over the workgroup: every wave skips the barriers below together
        }
        const int q = (S + 3) / 4, r0 = min(S, wave * q), r1 = min(S, r0 + q);
        sa_online<T>(f, ldf, s, lds, order, r0, r1, cc, m, l, acc);
        st[wave][0][lane] = m;
        st[wave][1][lane] = l;
        st[wave][2][lane] = acc;
        __syncthreads();
        if (wave == 0) {
            float2_t M = st[0][0][lane];
#pragma unroll
            for (int w = 1; w < 4; w++) {
                M.x = fmaxf(M.x, st[w][0][lane].x);
                M.y = fmaxf(M.y, st[w][0][lane].y);
            }
            float2_t L = {0.f, 0.f}, A = {0.f, 0.f};
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const float2_t mw = st[w][0][lane];
                if (mw.x != -INFINITY) {
                    const float a = __expf(mw.x - M.x);
                    L.x += st[w][1][lane].x * a;
                    A.x += st[w][2][lane].x * a;
                }
                if (mw.y != -INFINITY) {
                    const float a = __expf(mw.y - M.y);
                    L.y += st[w][1][lane].y * a;
                    A.y += st[w][2][lane].y * a;
                }
            }
            if (act) Pair<T>::store(y + g * (int64_t)D + c, float2_t{A.x / (L.x + eps), A.y / (L.y + eps)});
        }
        __syncthreads();   // the states are read before the next task overwrites them
    }
}

}  // namespace
}  // namespace dpvo

using namespace dpvo;

extern "C" size_t dpvo_softagg_workspace_bytes(int64_t num_edges, int64_t groups)
{
    return (size_t)sa_layout(num_edges < 0 ? 0 : num_edges, groups < 0 ? 0 : groups).total + 256;
}

extern "C" int dpvo_softagg_forward(int dtype, const void* f, int64_t ldf, const void* s, int64_t lds,
                                    const int64_t* group, int64_t num_edges, int D, int64_t groups, float eps,
                                    void* y, void* workspace, size_t workspace_bytes, void* stream)
{
    DPVO_CHECK_ARG(D > 0 && D % 2 == 0, "feature dim must be even and positive");
    DPVO_CHECK_ARG(num_edges >= 0 && groups >= 0 && num_edges < (int64_t(1) << 31), "bad sizes");
    DPVO_CHECK_ARG(ldf >= D && lds >= D && ldf % 2 == 0 && lds % 2 == 0, "row strides must be even and >= D");
    DPVO_CHECK_ARG(dtype == DPVO_F16 || dtype == DPVO_F32 || dtype == DPVO_F64, "unsupported dtype");
    if (groups == 0) return 0;
    DPVO_CHECK_ARG(num_edges > 0, "groups without edges");
    const SaLayout L = sa_layout(num_edges, groups);
    DPVO_CHECK_ARG(workspace != nullptr && workspace_bytes >= (size_t)L.total + 256, "workspace too small");
    hipStream_t st = as_stream(stream);
    char* ws = (char*)(((uintptr_t)workspace + 255) & ~uintptr_t(255));
    int* count = (int*)(ws + L.count);
    int* offs = (int*)(ws + L.offs);
    int* cursor = (int*)(ws + L.cursor);
    int* perm = (int*)(ws + L.perm);
    DPVO_CHECK_HIP(hipMemsetAsync(count, 0, 4 * groups, st));
    const unsigned gE = grid_for(num_edges, 256, 4096);
    hipLaunchKernelGGL(sa_count_kernel, dim3(gE), dim3(256), 0, st, group, num_edges, groups, count);
    hipLaunchKernelGGL(sa_scan_kernel, dim3(1), dim3(1024), 0, st, count, groups, offs, cursor);
    hipLaunchKernelGGL(sa_fill_kernel, dim3(gE), dim3(256), 0, st, group, num_edges, groups, cursor, perm);
    const int slices = (D + 127) / 128;
    const unsigned gR = (unsigned)((groups * slices + SA_WAVES - 1) / SA_WAVES);
    switch (dtype) {
    case DPVO_F16:
        hipLaunchKernelGGL(sa_reduce_kernel<half_t>, dim3(gR), dim3(64 * SA_WAVES), 0, st, (const half_t*)f, ldf,
                           (const half_t*)s, lds, offs, perm, groups, D, slices, eps, (half_t*)y);
        break;
    case DPVO_F32:
        hipLaunchKernelGGL(sa_reduce_kernel<float>, dim3(gR), dim3(64 * SA_WAVES), 0, st, (const float*)f, ldf,
                           (const float*)s, lds, offs, perm, groups, D, slices, eps, (float*)y);
        break;
    default:
        hipLaunchKernelGGL(sa_reduce_kernel<double>, dim3(gR), dim3(64 * SA_WAVES), 0, st, (const double*)f, ldf,
                           (const double*)s, lds, offs, perm, groups, D, slices, eps, (double*)y);
    }
    DPVO_CHECK_LAUNCH();
    return 0;
}

// The tracker's per-update edge keys in one pass (DPVO.update: _kk_groups,
// _ij_groups and the context-row index of dpvo.py:718), instead of ~6 torch
// elementwise launches: key_kk = kk - M base, key_ij = (ii - base) * 64 +
// (jj - base), ctx = kk mod ring (the patch ring slot: DPVO.corr's and the
// context gather's index), jslot = jj mod frames (the frame ring slot).
// flag (optional): set to -2 (unless already non-zero) when an edge lies
// outside the 64-frame key window, so a violated invariant fails loudly at the
// tracker's next status read instead of mis-grouping silently.
__global__ __launch_bounds__(256) void window_keys_kernel(const int64_t* __restrict__ ii,
                                                          const int64_t* __restrict__ jj,
                                                          const int64_t* __restrict__ kk, int64_t E, int64_t M,
                                                          int64_t base, int64_t ring, int64_t frames,
                                                          int64_t* __restrict__ key_kk, int64_t* __restrict__ key_ij,
                                                          int64_t* __restrict__ ctx, int64_t* __restrict__ jslot,
                                                          int* __restrict__ flag)
{
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = kk[e];
        const int64_t a = ii[e] - base, b = jj[e] - base, kr = k - M * base;
        key_kk[e] = kr;
        key_ij[e] = a * 64 + b;
        if (flag && (a < 0 || a >= 64 || b < 0 || b >= 64 || kr < 0 || kr >= 64 * M)) atomicCAS(flag, 0, -2);
        const int64_t r = k % ring, f = jj[e] % frames;
        ctx[e] = r < 0 ? r + ring : r;   // Python's modulo (kk, jj >= 0 in the tracker)
        jslot[e] = f < 0 ? f + frames : f;
    }
}

// The tracker's whole per-update grouping -- window_keys_kernel's outputs plus
// the counting-sort group-bys of key_kk (2^kk_bits bins) and key_ij (4096
// bins) -- in one memset and four launches instead of thirteen (DPVO.update's
// window keys, then dpvo_group_by twice, each a memset, a histogram, a
// two-kernel device scan, a scatter and a fix-up).  The launches are short
// (~5 us) and back to back, so their count, not their bytes, sets the cost.
// Outputs are dpvo_group_by's exactly (same masking of out-of-window keys).
constexpr int WG_IJ_BITS = 12;

struct WgLayout {
    int64_t hist, pre_kk, pre_ij, pre_j, slot_kk, slot_ij, ptmp_kk, ptmp_ij, key_kk, key_ij, total;
};

WgLayout wg_layout(int64_t n, int kk_bits)
{
    const int64_t Bkk = int64_t(1) << kk_bits, Bij = int64_t(1) << WG_IJ_BITS;
    WgLayout L;
    int64_t o = 0;
    L.hist = o;    o += align256(4 * (Bkk + Bij));   // kk bins then ij bins: one memset
    L.pre_kk = o;  o += align256(8 * Bkk);
    L.pre_ij = o;  o += align256(8 * Bij);
    L.pre_j = o;   o += align256(4 * Bij);           // ij bins' starts in jj-major order
    L.slot_kk = o; o += align256(4 * n);
    L.slot_ij = o; o += align256(4 * n);
    L.ptmp_kk = o; o += align256(4 * n);
    L.ptmp_ij = o; o += align256(4 * n);
    L.key_kk = o;  o += align256(4 * n);
    L.key_ij = o;  o += align256(4 * n);
    L.total = o;
    return L;
}

__global__ __launch_bounds__(256) void wg_hist_kernel(const int64_t* __restrict__ ii, const int64_t* __restrict__ jj,
                                                      const int64_t* __restrict__ kk, int64_t E, int64_t M,
                                                      int64_t base, int64_t ring, int64_t frames, uint32_t mask_kk,
                                                      int64_t* __restrict__ ctx, int64_t* __restrict__ jslot,
                                                      int* __restrict__ flag, int* __restrict__ hist_kk,
                                                      int* __restrict__ hist_ij, int* __restrict__ slot_kk,
                                                      int* __restrict__ slot_ij, uint32_t* __restrict__ key_kk,
                                                      uint32_t* __restrict__ key_ij)
{
    // the (ii, jj) keys: a patch's edges go to different frame pairs, so a
    // wave's lanes rarely share one and ~500 bins took every edge's atomic; a
    // workgroup ranks its edges in an LDS histogram instead and reserves each
    // touched bin's range with one global atomic (the slots within a bin are
    // ordered by wg_fix afterwards, as before).  The kk keys come in runs (a
    // patch's edges are adjacent): one atomic per run, cb_run_slot.
    constexpr int BIJ = 1 << WG_IJ_BITS;
    __shared__ int lh[BIJ];
    const int lane = threadIdx.x & 63;
    for (int64_t e0 = blockIdx.x * (int64_t)blockDim.x; e0 < E; e0 += (int64_t)gridDim.x * blockDim.x) {
        for (int i = threadIdx.x; i < BIJ; i += blockDim.x) lh[i] = 0;
        __syncthreads();
        const int64_t e = e0 + threadIdx.x;   // uniform trip count: whole waves stay converged
        const bool valid = e < E;
        uint32_t kk_k = 0xffffffffu, ij_k = 0xffffffffu;
        if (valid) {
            const int64_t k = kk[e], j = jj[e];
            const int64_t a = ii[e] - base, b = j - base, kr = k - M * base;
            kk_k = (uint32_t)kr & mask_kk;
            ij_k = (uint32_t)(a * 64 + b) & (BIJ - 1);
            if (flag && (a < 0 || a >= 64 || b < 0 || b >= 64 || kr < 0 || kr >= 64 * M)) atomicCAS(flag, 0, -2);
            const int64_t r = k % ring, f = j % frames;
            ctx[e] = r < 0 ? r + ring : r;
            jslot[e] = f < 0 ? f + frames : f;
            key_kk[e] = kk_k;
            key_ij[e] = ij_k;
        }
        const int s_kk = cb_run_slot(kk_k, valid, lane, hist_kk);
        const int l_ij = valid ? atomicAdd(&lh[ij_k], 1) : 0;   // rank within this workgroup's share
        __syncthreads();
        for (int i = threadIdx.x; i < BIJ; i += blockDim.x) {
            const int c = lh[i];
            if (c) lh[i] = atomicAdd(&hist_ij[i], c);   // the workgroup's base in bin i
        }
        __syncthreads();
        if (valid) {
            slot_kk[e] = s_kk;
            slot_ij[e] = lh[ij_k] + l_ij;
        }
        __syncthreads();   // (lh is cleared for the next round)
    }
}

// block 0 scans the kk bins, block 1 the ij bins: (start, group index) per
// bin, the group count and offs[G] = E.  8192 bins per round: thread t loads
// bins 8t .. 8t+7 (two 16-byte loads, coalesced), scans them in registers,
// one block scan of the thread sums, 64-byte coalesced stores of the results.
// (16 bins per thread, C3's 16384 kk bins in one round: 11.8 vs 11.4 us.)
__global__ __launch_bounds__(1024) void wg_scan_kernel(const int* __restrict__ hist, int Bkk, int64_t* __restrict__ pre_kk,
                                                       int64_t* __restrict__ pre_ij, int* __restrict__ offs_kk,
                                                       int* __restrict__ offs_ij, int64_t* __restrict__ groups_kk,
                                                       int64_t* __restrict__ groups_ij, int n,
                                                       int* __restrict__ pre_j)
{
    __shared__ int64_t wsum[16];
    if (blockIdx.x == 2) {
        // the (ii, jj) bins visited jj-major (bin a * 64 + b at transposed
        // position b * 64 + a): their starts give altcorr's target-frame order
        // from the ij slots, with no histogram of its own
        const int* h = hist + Bkk;
        const int t = threadIdx.x, lane = t & 63, w = t >> 6;
        int c[4], loc[4], sum = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int tix = 4 * t + j, b = tix >> 6, a = tix & 63;
            c[j] = h[a * 64 + b];
            loc[j] = sum;
            sum += c[j];
        }
        int x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        int off = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) off += i < w ? (int)wsum[i] : 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int tix = 4 * t + j, b = tix >> 6, a = tix & 63;
            pre_j[a * 64 + b] = off + x - sum + loc[j];
        }
        return;
    }
    const bool ij = blockIdx.x != 0;
    const int B = ij ? (1 << WG_IJ_BITS) : Bkk;
    const int* h = ij ? hist + Bkk : hist;
    int64_t* pre = ij ? pre_ij : pre_kk;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    constexpr int PT = 8;   // bins per thread
    int64_t carry = 0;
    for (int base = 0; base < B; base += 1024 * PT) {
        const int b0 = base + PT * t;
        int c[PT];
        if (b0 + PT <= B && ((uintptr_t)(h + b0) & 15) == 0) {
#pragma unroll
            for (int q = 0; q < PT / 4; q++) {
                const int4 x = *(const int4*)(h + b0 + 4 * q);
                c[4 * q] = x.x; c[4 * q + 1] = x.y; c[4 * q + 2] = x.z; c[4 * q + 3] = x.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < PT; j++) c[j] = b0 + j < B ? h[b0 + j] : 0;
        }
        int64_t loc[PT], s = 0;
#pragma unroll
        for (int j = 0; j < PT; j++) {
            loc[j] = s;
            s += CbCombine()(c[j]);
        }
        int64_t x = s;   // inclusive scan over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        int64_t off = carry, tot = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int64_t v = wsum[i];
            off += i < w ? v : 0;
            tot += v;
        }
        const int64_t ex = off + x - s;
#pragma unroll
        for (int j = 0; j < PT; j++)
            if (b0 + j < B) pre[b0 + j] = ex + loc[j];
        carry += tot;
        __syncthreads();   // wsum is rewritten next round
    }
    if (t == 0) {   // carry = the grand total
        const int64_t G = carry >> 32;
        *(ij ? groups_ij : groups_kk) = G;
        (ij ? offs_ij : offs_kk)[G] = n;
    }
}

__global__ __launch_bounds__(256) void wg_scatter_kernel(int64_t E, const uint32_t* __restrict__ key_kk,
                                                         const uint32_t* __restrict__ key_ij,
                                                         const int64_t* __restrict__ pre_kk,
                                                         const int64_t* __restrict__ pre_ij,
                                                         const int* __restrict__ slot_kk,
                                                         const int* __restrict__ slot_ij, int* __restrict__ ptmp_kk,
                                                         int* __restrict__ ptmp_ij, int64_t* __restrict__ gid_kk,
                                                         int64_t* __restrict__ gid_ij, int* __restrict__ offs_kk,
                                                         int* __restrict__ offs_ij, const int* __restrict__ pre_j,
                                                         int* __restrict__ order_j)
{
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        if (order_j) order_j[pre_j[key_ij[e]] + slot_ij[e]] = (int)e;
        const int64_t p = pre_kk[key_kk[e]], q = pre_ij[key_ij[e]];
        const int sp = slot_kk[e], sq = slot_ij[e];
        const int ps = (int)(p & 0xffffffff), pg = (int)(p >> 32), qs = (int)(q & 0xffffffff), qg = (int)(q >> 32);
        ptmp_kk[ps + sp] = (int)e;
        ptmp_ij[qs + sq] = (int)e;
        gid_kk[e] = pg;
        gid_ij[e] = qg;
        if (sp == 0) offs_kk[pg] = ps;
        if (sq == 0) offs_ij[qg] = qs;
    }
}

// one wave per group, the (larger) ij groups first
__global__ __launch_bounds__(64 * CB_WAVES) void wg_fix_kernel(int64_t n, const int* __restrict__ ptmp_kk,
                                                               const int* __restrict__ offs_kk,
                                                               const int64_t* __restrict__ groups_kk,
                                                               const int64_t* __restrict__ gid_kk,
                                                               int* __restrict__ perm_kk,
                                                               const int* __restrict__ ptmp_ij,
                                                               const int* __restrict__ offs_ij,
                                                               const int64_t* __restrict__ groups_ij,
                                                               const int64_t* __restrict__ gid_ij,
                                                               int* __restrict__ perm_ij)
{
    __shared__ __attribute__((aligned(16))) int buf[CB_WAVES][CB_CAP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t Gi = *groups_ij, G = Gi + *groups_kk;
    for (int64_t g = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; g < G;
         g += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        if (g < Gi)
            cb_fix_group(g, ptmp_ij, offs_ij, gid_ij, n, perm_ij, buf[w], lane);
        else
            cb_fix_group(g - Gi, ptmp_kk, offs_kk, gid_kk, n, perm_kk, buf[w], lane);
    }
}

// DPVO.__call__'s edge append (dpvo.py:756-769, 799-800): the old edge list
// followed by the forward edges (patches of frames [n - r, n - 1) into frame
// n - 1) and the backward edges (frame n - 1's patches into frames
// [n - r, n), patch-major as flatmeshgrid(indexing="ij") lists them), with
// ii = ix[kk] -- one launch instead of two aranges + meshgrid per direction,
// the concatenations and the ix gather.  n: the frame count after the new
// frame was added.
__global__ __launch_bounds__(256) void append_edges_kernel(const int64_t* __restrict__ ii, const int64_t* __restrict__ jj,
                                                           const int64_t* __restrict__ kk, int64_t E,
                                                           const int64_t* __restrict__ ix, int64_t n, int64_t M,
                                                           int64_t r, int64_t* __restrict__ ii_o,
                                                           int64_t* __restrict__ jj_o, int64_t* __restrict__ kk_o)
{
    const int64_t f0 = M * (n - r > 0 ? n - r : 0), f1 = M * (n - 1 > 0 ? n - 1 : 0);
    const int64_t nf = f1 - f0;
    const int64_t b0 = f1, j0 = n - r > 0 ? n - r : 0, nj = n - j0;
    const int64_t nb = (M * n - b0) * nj;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E + nf + nb;
         e += (int64_t)gridDim.x * blockDim.x) {
        int64_t i, j, k;
        if (e < E) {
            i = ii[e], j = jj[e], k = kk[e];
        } else if (e < E + nf) {
            k = f0 + (e - E), j = n - 1, i = ix[k];
        } else {
            const int64_t t = e - E - nf;
            k = b0 + t / nj, j = j0 + t % nj, i = ix[k];
        }
        ii_o[e] = i;
        jj_o[e] = j;
        kk_o[e] = k;
    }
}

// target = coords[..., P/2, P/2] + float(delta), weight = float(w) for every
// edge (DPVO.update after the update operator, dpvo.py:724-727), one launch
// instead of three.  delta / w: fp16 rows with their own strides (the fused
// operator's [E][4] head rows); c: the patch centre's x at c + e * cs, y at
// c + e * cs + cc.
__global__ __launch_bounds__(256) void edge_targets_kernel(const half_t* __restrict__ delta, int64_t ds,
                                                           const half_t* __restrict__ w, int64_t ws,
                                                           const float* __restrict__ c, int64_t cs, int64_t cc,
                                                           int64_t E, float* __restrict__ target,
                                                           float* __restrict__ weight)
{
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        target[2 * e] = c[e * cs] + (float)delta[e * ds];
        target[2 * e + 1] = c[e * cs + cc] + (float)delta[e * ds + 1];
        weight[2 * e] = (float)w[e * ws];
        weight[2 * e + 1] = (float)w[e * ws + 1];
    }
}

extern "C" int dpvo_gather_rows(int in_dtype, const void* x, int64_t ldx, int64_t rows, const int64_t* idx, int64_t n,
                                int D, int out_dtype, void* out, void* stream)
{
    DPVO_CHECK_ARG(D > 0 && D % 2 == 0 && ldx >= D && ldx % 2 == 0, "feature dim / row stride must be even");
    DPVO_CHECK_ARG(n >= 0 && rows >= 0, "bad sizes");
    if (n == 0) return 0;
    hipStream_t s = as_stream(stream);
    int rc;
    switch (in_dtype) {
    case DPVO_F16: rc = gather_dispatch_out((const half_t*)x, ldx, rows, idx, n, D, out_dtype, out, s); break;
    case DPVO_F32: rc = gather_dispatch_out((const float*)x, ldx, rows, idx, n, D, out_dtype, out, s); break;
    case DPVO_F64: rc = gather_dispatch_out((const double*)x, ldx, rows, idx, n, D, out_dtype, out, s); break;
    default: rc = -1;
    }
    DPVO_CHECK_ARG(rc == 0, "unsupported dtype");
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" size_t dpvo_group_by_workspace_bytes(int64_t n)
{
    return (size_t)gb_layout(n > 0 ? n : 1).total + 256;
}

extern "C" size_t dpvo_group_by_workspace_bytes_for(int64_t n, int key_bits)
{
    size_t r = dpvo_group_by_workspace_bytes(n);
    if (key_bits >= 1 && key_bits <= CB_MAX_BITS) r = std::max(r, (size_t)cb_layout(n > 0 ? n : 1, key_bits).total + 256);
    return r;
}

extern "C" int dpvo_group_by(const int64_t* key, int64_t n, int key_bits, int64_t* gid, int* offs, int* perm,
                             int64_t* groups, void* workspace, size_t workspace_bytes, void* stream)
{
    DPVO_CHECK_ARG(n >= 0 && n < (int64_t(1) << 31), "bad size");
    DPVO_CHECK_ARG(key_bits >= 1 && key_bits <= 64, "key_bits must be 1..64");
    DPVO_CHECK_ARG(groups != nullptr, "groups output missing");
    hipStream_t st = as_stream(stream);
    if (n == 0) {
        DPVO_CHECK_HIP(hipMemsetAsync(groups, 0, sizeof(int64_t), st));
        DPVO_CHECK_HIP(hipMemsetAsync(offs, 0, sizeof(int), st));
        return 0;
    }
    char* ws = (char*)(((uintptr_t)workspace + 255) & ~uintptr_t(255));
    if (key_bits <= CB_MAX_BITS && workspace != nullptr) {
        const CbLayout C = cb_layout(n, key_bits);
        if (workspace_bytes >= (size_t)C.total + 256) {   // else: the radix path below
            const int64_t B = int64_t(1) << key_bits;
            const uint32_t mask = (uint32_t)(B - 1);
            int* hist = (int*)(ws + C.hist);
            int64_t* pre = (int64_t*)(ws + C.pre);
            int* slot = (int*)(ws + C.slot);
            int* ptmp = (int*)(ws + C.ptmp);
            const unsigned gn = grid_for(n, 256, 2048);
            DPVO_CHECK_HIP(hipMemsetAsync(hist, 0, 4 * B, st));
            hipLaunchKernelGGL(cb_hist_kernel, dim3(gn), dim3(256), 0, st, key, n, mask, hist, slot);
            size_t tb = (size_t)C.tmp_bytes;
            hipcub::TransformInputIterator<int64_t, CbCombine, const int*> it(hist, CbCombine());
            DPVO_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(ws + C.tmp, tb, it, pre, (int)B, st));
            hipLaunchKernelGGL(cb_scatter_kernel, dim3(gn), dim3(256), 0, st, key, n, mask, hist, pre, slot, ptmp, gid,
                               offs, groups);
            const unsigned gf = grid_for(std::min<int64_t>(n, B) * 64, 64 * CB_WAVES, 2048);
            hipLaunchKernelGGL(cb_fix_kernel, dim3(gf), dim3(64 * CB_WAVES), 0, st, ptmp, offs, groups, gid, n, perm);
            DPVO_CHECK_LAUNCH();
            return 0;
        }
    }
    const GbLayout L = gb_layout(n);
    DPVO_CHECK_ARG(workspace != nullptr && workspace_bytes >= (size_t)L.total + 256, "workspace too small");
    int* v_in = (int*)(ws + L.v_in);
    int* flag = (int*)(ws + L.flag);
    int* incl = (int*)(ws + L.incl);
    size_t tmp_bytes = (size_t)L.tmp_bytes;
    const unsigned g = grid_for(n, 256, 2048);
    auto sort = [&](auto* k_in, auto* k_out) -> int {
        using K = std::remove_pointer_t<decltype(k_in)>;
        hipLaunchKernelGGL(gb_keys_kernel<K>, dim3(g), dim3(256), 0, st, key, n, k_in, v_in);
        DPVO_CHECK_LAUNCH();
        DPVO_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(ws + L.tmp, tmp_bytes, k_in, k_out, v_in, perm, (int)n, 0,
                                                          key_bits, st));
        hipLaunchKernelGGL(gb_flags_kernel<K>, dim3(g), dim3(256), 0, st, k_out, n, flag);
        return 0;
    };
    if (key_bits <= 32)
        sort((uint32_t*)(ws + L.k_in), (uint32_t*)(ws + L.k_out));
    else
        sort((uint64_t*)(ws + L.k_in), (uint64_t*)(ws + L.k_out));
    tmp_bytes = (size_t)L.tmp_bytes;
    DPVO_CHECK_HIP(hipcub::DeviceScan::InclusiveSum(ws + L.tmp, tmp_bytes, flag, incl, (int)n, st));
    hipLaunchKernelGGL(gb_finish_kernel, dim3(g), dim3(256), 0, st, flag, incl, perm, n, gid, offs, groups);
    DPVO_CHECK_LAUNCH();
    return 0;
}

// neighbors over the kk group-by CSR: one wave per group; member i's
// predecessor / successor in (jj, edge) order by an O(s^2) scan of the group
// (s ~ 25 in DPVO's steady state), 64 members at a time, broadcast by shuffles.
__global__ __launch_bounds__(256) void nb_csr_kernel(const int64_t* __restrict__ jj, const int* __restrict__ offs,
                                                     const int* __restrict__ perm, const int64_t* __restrict__ groups,
                                                     int64_t max_groups, int64_t* __restrict__ ix,
                                                     int64_t* __restrict__ jx)
{
    const int lane = threadIdx.x & 63;
    const int64_t G = min(*groups, max_groups);
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t g = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; g < G; g += nw) {
        const int start = offs[g], s = offs[g + 1] - start;
        for (int i0 = 0; i0 < s; i0 += 64) {
            const bool mine = i0 + lane < s;
            const int ei = mine ? perm[start + i0 + lane] : 0;
            const int64_t ji = mine ? jj[ei] : 0;
            // best predecessor (largest key below mine) / successor (smallest above)
            int64_t pj = INT64_MIN, nj = INT64_MAX;
            int pe = -1, ne = -1;
            for (int t0 = 0; t0 < s; t0 += 64) {
                const int cnt = min(64, s - t0);
                const int et = t0 + lane < s ? perm[start + t0 + lane] : 0;
                const int64_t jt = t0 + lane < s ? jj[et] : 0;
                for (int k = 0; k < cnt; k++) {
                    const int ek = __shfl(et, k);
                    const int64_t jk = __shfl(jt, k);
                    const bool below = jk < ji || (jk == ji && ek < ei);
                    const bool above = jk > ji || (jk == ji && ek > ei);
                    if (below && (jk > pj || (jk == pj && ek > pe))) { pj = jk; pe = ek; }
                    if (above && (jk < nj || (jk == nj && ek < ne))) { nj = jk; ne = ek; }
                }
            }
            if (mine) {
                ix[ei] = pe;
                jx[ei] = ne;
            }
        }
    }
}

extern "C" int dpvo_neighbors_csr(const int64_t* jj, const int* offs, const int* perm, const int64_t* groups,
                                  int64_t max_groups, int64_t num_edges, int64_t* ix, int64_t* jx, void* stream)
{
    DPVO_CHECK_ARG(groups != nullptr && offs != nullptr && perm != nullptr, "CSR missing");
    DPVO_CHECK_ARG(num_edges >= 0 && num_edges < (int64_t(1) << 31), "bad size");
    if (num_edges == 0 || max_groups <= 0) return 0;
    const unsigned grid = grid_for(max_groups * 64, 256, 4096);
    hipLaunchKernelGGL(nb_csr_kernel, dim3(grid), dim3(256), 0, as_stream(stream), jj, offs, perm, groups,
                       max_groups, ix, jx);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_softagg_csr(int dtype, const void* f, int64_t ldf, const void* s, int64_t lds, const int* offs,
                                const int* perm, const int64_t* groups, int64_t max_groups, int D, float eps, void* y,
                                void* stream)
{
    DPVO_CHECK_ARG(D > 0 && D % 2 == 0, "feature dim must be even and positive");
    DPVO_CHECK_ARG(ldf >= D && lds >= D && ldf % 2 == 0 && lds % 2 == 0, "row strides must be even and >= D");
    DPVO_CHECK_ARG(groups != nullptr && offs != nullptr && perm != nullptr, "CSR missing");
    if (max_groups <= 0) return 0;
    hipStream_t st = as_stream(stream);
    const int slices = (D + 127) / 128;
    const unsigned grid = grid_for(max_groups * slices * 64, 256, 4096);
    switch (dtype) {
    case DPVO_F16:
        hipLaunchKernelGGL(sa_reduce_csr_kernel<half_t>, dim3(grid), dim3(256), 0, st, (const half_t*)f, ldf,
                           (const half_t*)s, lds, offs, perm, groups, D, slices, eps, (half_t*)y);
        break;
    case DPVO_F32:
        hipLaunchKernelGGL(sa_reduce_csr_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)f, ldf,
                           (const float*)s, lds, offs, perm, groups, D, slices, eps, (float*)y);
        break;
    case DPVO_F64:
        hipLaunchKernelGGL(sa_reduce_csr_kernel<double>, dim3(grid), dim3(256), 0, st, (const double*)f, ldf,
                           (const double*)s, lds, offs, perm, groups, D, slices, eps, (double*)y);
        break;
    default:
        set_error("dpvo_softagg_csr: unsupported dtype");
        return -1;
    }
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_window_keys(const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t E, int64_t M,
                                int64_t base, int64_t ring, int64_t frames, int64_t* key_kk, int64_t* key_ij,
                                int64_t* ctx, int64_t* jslot, int* flag, void* stream)
{
    DPVO_CHECK_ARG(E >= 0 && M > 0 && ring > 0 && frames > 0, "E >= 0, M > 0, ring > 0 and frames > 0 required");
    if (E == 0) return 0;
    DPVO_CHECK_ARG(ii && jj && kk && key_kk && key_ij && ctx && jslot, "null operand");
    hipLaunchKernelGGL(window_keys_kernel, dim3(grid_for(E, 256, 4096)), dim3(256), 0, as_stream(stream), ii, jj, kk,
                       E, M, base, ring, frames, key_kk, key_ij, ctx, jslot, flag);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" size_t dpvo_window_group_by_workspace_bytes(int64_t E, int kk_bits)
{
    if (kk_bits < 1 || kk_bits > CB_MAX_BITS) return 0;
    return (size_t)wg_layout(E > 0 ? E : 1, kk_bits).total + 256;
}

extern "C" int dpvo_window_group_by(const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t E, int64_t M,
                                    int64_t base, int64_t ring, int64_t frames, int kk_bits, int64_t* ctx,
                                    int64_t* jslot, int* flag, int64_t* kk_gid, int* kk_offs, int* kk_perm,
                                    int64_t* kk_groups, int64_t* ij_gid, int* ij_offs, int* ij_perm,
                                    int64_t* ij_groups, int* jj_order, void* workspace, size_t workspace_bytes,
                                    void* stream)
{
    DPVO_CHECK_ARG(E >= 0 && E < (int64_t(1) << 31), "bad size");
    DPVO_CHECK_ARG(M > 0 && ring > 0 && frames > 0, "M > 0, ring > 0 and frames > 0 required");
    DPVO_CHECK_ARG(kk_bits >= 1 && kk_bits <= CB_MAX_BITS, "kk_bits must be 1..22");
    DPVO_CHECK_ARG(kk_groups && kk_offs && ij_groups && ij_offs, "CSR outputs missing");
    hipStream_t st = as_stream(stream);
    if (E == 0) {
        DPVO_CHECK_HIP(hipMemsetAsync(kk_groups, 0, sizeof(int64_t), st));
        DPVO_CHECK_HIP(hipMemsetAsync(kk_offs, 0, sizeof(int), st));
        DPVO_CHECK_HIP(hipMemsetAsync(ij_groups, 0, sizeof(int64_t), st));
        DPVO_CHECK_HIP(hipMemsetAsync(ij_offs, 0, sizeof(int), st));
        return 0;
    }
    DPVO_CHECK_ARG(ii && jj && kk && ctx && jslot && kk_gid && kk_perm && ij_gid && ij_perm, "null operand");
    const WgLayout L = wg_layout(E, kk_bits);
    DPVO_CHECK_ARG(workspace != nullptr && workspace_bytes >= (size_t)L.total + 256, "workspace too small");
    char* ws = (char*)(((uintptr_t)workspace + 255) & ~uintptr_t(255));
    const int Bkk = 1 << kk_bits;
    int* hist = (int*)(ws + L.hist);
    int64_t* pre_kk = (int64_t*)(ws + L.pre_kk);
    int64_t* pre_ij = (int64_t*)(ws + L.pre_ij);
    int* slot_kk = (int*)(ws + L.slot_kk);
    int* slot_ij = (int*)(ws + L.slot_ij);
    int* ptmp_kk = (int*)(ws + L.ptmp_kk);
    int* ptmp_ij = (int*)(ws + L.ptmp_ij);
    uint32_t* key_kk = (uint32_t*)(ws + L.key_kk);
    uint32_t* key_ij = (uint32_t*)(ws + L.key_ij);
    int* pre_j = (int*)(ws + L.pre_j);
    const unsigned gn = grid_for(E, 256, 2048);
    DPVO_CHECK_HIP(hipMemsetAsync(hist, 0, 4 * (size_t)(Bkk + (1 << WG_IJ_BITS)), st));
    hipLaunchKernelGGL(wg_hist_kernel, dim3(gn), dim3(256), 0, st, ii, jj, kk, E, M, base, ring, frames,
                       (uint32_t)(Bkk - 1), ctx, jslot, flag, hist, hist + Bkk, slot_kk, slot_ij, key_kk, key_ij);
    hipLaunchKernelGGL(wg_scan_kernel, dim3(jj_order ? 3 : 2), dim3(1024), 0, st, hist, Bkk, pre_kk, pre_ij, kk_offs,
                       ij_offs, kk_groups, ij_groups, (int)E, pre_j);
    hipLaunchKernelGGL(wg_scatter_kernel, dim3(gn), dim3(256), 0, st, E, key_kk, key_ij, pre_kk, pre_ij, slot_kk,
                       slot_ij, ptmp_kk, ptmp_ij, kk_gid, ij_gid, kk_offs, ij_offs, pre_j, jj_order);
    const int64_t waves = std::min<int64_t>(E, Bkk) + std::min<int64_t>(E, 1 << WG_IJ_BITS);
    const unsigned gf = grid_for(waves * 64, 64 * CB_WAVES, 2048);
    hipLaunchKernelGGL(wg_fix_kernel, dim3(gf), dim3(64 * CB_WAVES), 0, st, E, ptmp_kk, kk_offs, kk_groups, kk_gid,
                       kk_perm, ptmp_ij, ij_offs, ij_groups, ij_gid, ij_perm);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int64_t dpvo_append_edges_count(int64_t n, int64_t M, int64_t r)
{
    if (n < 1 || M < 1 || r < 1) return -1;
    const int64_t f0 = M * (n - r > 0 ? n - r : 0), f1 = M * (n - 1 > 0 ? n - 1 : 0), j0 = n - r > 0 ? n - r : 0;
    return (f1 - f0) + (M * n - f1) * (n - j0);
}

extern "C" int dpvo_append_edges(const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t E, const int64_t* ix,
                                 int64_t n, int64_t M, int64_t r, int64_t* ii_out, int64_t* jj_out, int64_t* kk_out,
                                 void* stream)
{
    const int64_t add = dpvo_append_edges_count(n, M, r);
    DPVO_CHECK_ARG(add >= 0 && E >= 0, "n >= 1, M >= 1, PATCH_LIFETIME >= 1 and E >= 0 required");
    DPVO_CHECK_ARG(ix && ii_out && jj_out && kk_out && (E == 0 || (ii && jj && kk)), "null operand");
    if (E + add == 0) return 0;
    hipLaunchKernelGGL(append_edges_kernel, dim3(grid_for(E + add, 256, 4096)), dim3(256), 0, as_stream(stream), ii,
                       jj, kk, E, ix, n, M, r, ii_out, jj_out, kk_out);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_edge_targets(const void* delta, int64_t delta_stride, const void* w, int64_t w_stride,
                                 const float* centre, int64_t centre_stride, int64_t centre_comp, int64_t E,
                                 float* target, float* weight, void* stream)
{
    DPVO_CHECK_ARG(E >= 0, "E >= 0 required");
    if (E == 0) return 0;
    DPVO_CHECK_ARG(delta && w && centre && target && weight, "null operand");
    hipLaunchKernelGGL(edge_targets_kernel, dim3(grid_for(E, 256, 4096)), dim3(256), 0, as_stream(stream),
                       (const half_t*)delta, delta_stride, (const half_t*)w, w_stride, centre, centre_stride,
                       centre_comp, E, target, weight);
    DPVO_CHECK_LAUNCH();
    return 0;
}

extern "C" int dpvo_softagg_csr_long(int dtype, const void* f, int64_t ldf, const void* s, int64_t lds,
                                     const int* offs, const int* perm, const int64_t* groups, int64_t max_groups,
                                     int D, float eps, void* y, void* stream)
{
    DPVO_CHECK_ARG(D > 0 && D % 2 == 0, "feature dim must be even and positive");
    DPVO_CHECK_ARG(ldf >= D && lds >= D && ldf % 2 == 0 && lds % 2 == 0, "row strides must be even and >= D");
    DPVO_CHECK_ARG(groups != nullptr && offs != nullptr && perm != nullptr, "CSR missing");
    DPVO_CHECK_ARG(dtype == DPVO_F16 || dtype == DPVO_F32, "dtype must be fp16 or fp32");
    if (max_groups <= 0) return 0;
    const int slices = (D + 127) / 128;
    const unsigned grid = grid_for(max_groups * slices, 1, 8192);
    if (dtype == DPVO_F16)
        hipLaunchKernelGGL(sa_reduce_csr_split_kernel<half_t>, dim3(grid), dim3(256), 0, as_stream(stream),
                           (const half_t*)f, ldf, (const half_t*)s, lds, offs, perm, groups, D, slices, eps,
                           (half_t*)y);
    else
        hipLaunchKernelGGL(sa_reduce_csr_split_kernel<float>, dim3(grid), dim3(256), 0, as_stream(stream),
                           (const float*)f, ldf, (const float*)s, lds, offs, perm, groups, D, slices, eps, (float*)y);
    DPVO_CHECK_LAUNCH();
    return 0;
}

// ---------------------------------------------------------------------------
// torch_scatter 2.1.2 reductions (scatter_sum / mean / max / softmax) over the
// CSR of dpvo_group_by(index): the reference's SoftAgg (blocks.py:42-43), its
// Python BA (ba.py:40-56) and loop closure (long_term.py:134) call them.
// src is viewed as [outer][E][inner] (the scatter dim in the middle) and the
// index is 1-D along it.  One thread per (group, outer x inner column) walks
// the group's members in ascending edge order: deterministic, no atomics.
// ---------------------------------------------------------------------------
namespace {
enum { SC_SUM = 0, SC_MEAN = 1, SC_MAX = 2, SC_SOFTMAX = 3 };

template <typename T> struct ScAcc { typedef float type; };
template <> struct ScAcc<double> { typedef double type; };

template <typename T, int OP>
__global__ __launch_bounds__(256) void scatter_csr_kernel(const T* __restrict__ src, int64_t outer, int64_t E,
                                                          int64_t inner, const int64_t* __restrict__ index,
                                                          const int* __restrict__ offs, const int* __restrict__ perm,
                                                          const int64_t* __restrict__ groups, int64_t max_groups,
                                                          float eps, T* __restrict__ out, int64_t out_rows,
                                                          int64_t* __restrict__ arg)
{
    typedef typename ScAcc<T>::type A;
    const int64_t G = min(*groups, max_groups);
    const int64_t cols = outer * inner;
    const int64_t cblocks = (cols + 255) / 256;
    for (int64_t w = blockIdx.x; w < G * cblocks; w += gridDim.x) {
        const int64_t g = w / cblocks;
        const int64_t col = (w % cblocks) * 256 + threadIdx.x;
        if (col >= cols) continue;
        const int64_t o = col / inner, c = col % inner;
        const int b = offs[g], s = offs[g + 1] - b;
        const T* sp = src + o * E * inner + c;
        if (OP == SC_SUM || OP == SC_MEAN) {
            A a = 0;
            for (int i = 0; i < s; i++) a += (A)sp[(int64_t)perm[b + i] * inner];
            const int64_t key = index[perm[b]];
            if (key < 0 || key >= out_rows) continue;
            T* op = out + (o * out_rows + key) * inner + c;
            A v = (A)*op + a;
            if (OP == SC_MEAN) v = v / (A)s;
            *op = (T)v;
        } else if (OP == SC_MAX) {
            A m = 0;
            int64_t am = -1;
            for (int i = 0; i < s; i++) {
                const int e = perm[b + i];
                const A v = (A)sp[(int64_t)e * inner];
                if (am < 0 || v > m) {
                    m = v;
                    am = e;
                }
            }
            const int64_t key = index[perm[b]];
            if (key < 0 || key >= out_rows) continue;
            out[(o * out_rows + key) * inner + c] = (T)m;
            arg[(o * out_rows + key) * inner + c] = am;
        } else {   // SOFTMAX: recentre on the group max, exp, / (sum + eps)   (composite/softmax.py)
            A m = 0;
            for (int i = 0; i < s; i++) {
                const A v = (A)sp[(int64_t)perm[b + i] * inner];
                m = (i == 0 || v > m) ? v : m;
            }
            A den = 0;
            for (int i = 0; i < s; i++) den += exp((A)sp[(int64_t)perm[b + i] * inner] - m);
            den += (A)eps;
            T* op = out + o * E * inner + c;
            for (int i = 0; i < s; i++) {
                const int64_t e = perm[b + i];
                op[e * inner] = (T)(exp((A)sp[e * inner] - m) / den);
            }
        }
    }
}

template <typename T>
int scatter_dispatch(int op, const T* src, int64_t outer, int64_t E, int64_t inner, const int64_t* index,
                     const int* offs, const int* perm, const int64_t* groups, int64_t max_groups, float eps, T* out,
                     int64_t out_rows, int64_t* arg, hipStream_t st)
{
    const int64_t cblocks = (outer * inner + 255) / 256;
    const unsigned grid = grid_for(max_groups * cblocks, 1, 16384);
#define SC_LAUNCH(OPV)                                                                                          \
    hipLaunchKernelGGL((scatter_csr_kernel<T, OPV>), dim3(grid), dim3(256), 0, st, src, outer, E, inner, index, \
                       offs, perm, groups, max_groups, eps, out, out_rows, arg)
    switch (op) {
    case SC_SUM: SC_LAUNCH(SC_SUM); break;
    case SC_MEAN: SC_LAUNCH(SC_MEAN); break;
    case SC_MAX: SC_LAUNCH(SC_MAX); break;
    case SC_SOFTMAX: SC_LAUNCH(SC_SOFTMAX); break;
    default: return -1;
    }
#undef SC_LAUNCH
    return 0;
}
}  // namespace

extern "C" int dpvo_scatter_csr(int op, int dtype, const void* src, int64_t outer, int64_t E, int64_t inner,
                                const int64_t* index, const int* offs, const int* perm, const int64_t* groups,
                                int64_t max_groups, float eps, void* out, int64_t out_rows, int64_t* argmax,
                                void* stream)
{
    DPVO_CHECK_ARG(op >= SC_SUM && op <= SC_SOFTMAX, "op must be 0 (sum), 1 (mean), 2 (max) or 3 (softmax)");
    DPVO_CHECK_ARG(outer >= 0 && E >= 0 && inner >= 0 && out_rows >= 0, "bad sizes");
    DPVO_CHECK_ARG(E < (int64_t(1) << 31), "at most 2^31 - 1 elements along the scatter dim");
    DPVO_CHECK_ARG(op != SC_MAX || argmax != nullptr, "scatter max needs the argmax output");
    if (E == 0 || outer == 0 || inner == 0 || max_groups <= 0) return 0;
    DPVO_CHECK_ARG(src && index && offs && perm && groups && out, "null operand");
    hipStream_t st = as_stream(stream);
    int rc;
    switch (dtype) {
    case DPVO_F16:
        rc = scatter_dispatch(op, (const half_t*)src, outer, E, inner, index, offs, perm, groups, max_groups, eps,
                              (half_t*)out, out_rows, argmax, st);
        break;
    case DPVO_F32:
        rc = scatter_dispatch(op, (const float*)src, outer, E, inner, index, offs, perm, groups, max_groups, eps,
                              (float*)out, out_rows, argmax, st);
        break;
    case DPVO_F64:
        rc = scatter_dispatch(op, (const double*)src, outer, E, inner, index, offs, perm, groups, max_groups, eps,
                              (double*)out, out_rows, argmax, st);
        break;
    default: rc = -1;
    }
    DPVO_CHECK_ARG(rc == 0, "unsupported dtype");
    DPVO_CHECK_LAUNCH();
    return 0;
}

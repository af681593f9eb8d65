// Top-k of 64-bit keys and the stable rank sort, for gfx950.
//
// Replaces the library top-k of the ProposalLayer (tf.nn.top_k(scores,
// pre_nms_limit, sorted=True) at core/models.py:403-404; rocprim merge-path
// sort behind torch.topk before round 5) and the single-workgroup bitonic sort
// of m3d_nms3d's candidates.
//
//   select: radix select of the k-th largest key, six digit passes over the
//           keys (11, 11, 11, 11, 11, 9 bits from the top).  Every pass counts
//           the next digit of the keys that share the threshold's prefix in an
//           LDS histogram (wave-aggregated adds: the first digits of score keys
//           are few) added to the pass's global one; a one-block kernel then
//           scans it (2048 bins, largest first) for the next digit of the
//           prefix and the keys still needed below it.
//           The keys are read once per pass (33 MB per pass at 256^3's 4.2 M
//           anchors); no sort of the n keys.
//   gather: the keys >= the threshold (exactly k of them for distinct keys)
//           with their positions, unordered (per-block LDS compaction, one
//           atomic per block for the output offset).
//   rank:   out[rank(i)] = key(i) with rank(i) = #{j : u_j > u_i or (u_j == u_i
//           and j < i)} (descending; ascending for the NMS form) -- an O(k^2)
//           count split over (target block, source chunk) workgroups with
//           integer atomics (exact, so the result does not depend on arrival
//           order), then a scatter.  15000 keys: 59 x 8 workgroups of 2048
//           comparisons per lane instead of 105 barrier-separated bitonic
//           stages in one workgroup.
//
// Keys are signed int64 in the m3d_topk_keys API (the orderable score keys of
// m3d_score_keys); they are compared as u = key ^ 2^63 (unsigned order ==
// signed order).
#include "common.h"

namespace m3d {

constexpr int TK_PASSES = 6;
constexpr int TK_BINS = 2048;
__device__ __host__ constexpr int tk_shift(int p) { return p < 5 ? 53 - 11 * p : 0; }
__device__ __host__ constexpr int tk_width(int p) { return p < 5 ? 11 : 9; }

// Selection state after each digit pass: the threshold's digit prefix (bits
// at and above the pass's shift) and how many keys are still needed among the
// keys sharing it.  st[0] = (0, k); st[p + 1] = tk_state_kernel(st[p], hist[p]).
struct TkState {
    uint64_t prefix;
    int64_t need;
};

// one 256-thread block: the digit of pass `pass` holding the need-th largest
// key below the prefix (a suffix scan over the pass's histogram, largest digit
// first), written to st[pass + 1]
__global__ __launch_bounds__(256) void tk_state_kernel(const uint32_t* __restrict__ hists, int pass, int64_t k,
                                                       TkState* __restrict__ st) {
    __shared__ uint32_t part[256];
    const int t = threadIdx.x;
    const TkState cur = pass ? st[pass] : TkState{0, k};
    const uint32_t* h = hists + (size_t)pass * TK_BINS;
    const int nb = 1 << tk_width(pass);
    const int per = nb / 256;                          // 8 bins per thread (2 in the 9-bit pass)
    const int hi = nb - per * t;                       // thread t owns bins [hi - per, hi): t = 0 the largest
    uint32_t sum = 0;
    for (int b = hi - per; b < hi; ++b) sum += h[b];
    part[t] = sum;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {         // inclusive prefix over threads, Hillis-Steele
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const int64_t need = cur.need;
    const uint32_t before = t ? part[t - 1] : 0u;      // keys in larger digits than this thread's bins
    if ((int64_t)before < need && need <= (int64_t)part[t]) {
        uint32_t c = before;
        for (int b = hi - 1; b >= hi - per; --b) {
            if (need <= (int64_t)(c + h[b])) {
                st[pass + 1] = TkState{cur.prefix | ((uint64_t)b << tk_shift(pass)), need - (int64_t)c};
                break;
            }
            c += h[b];
        }
    }
}

// LDS histogram of the pass's digit over the keys sharing the prefix; the
// first pass's digits are few (the scores' sign / exponent bits), so the adds
// of a wave are aggregated per distinct digit (up to 4 rounds of readfirstlane
// + ballot) before the per-lane fallback
__global__ __launch_bounds__(256) void topk_hist_kernel(const int64_t* __restrict__ keys, int64_t n,
                                                        const TkState* __restrict__ st, uint32_t* __restrict__ hists,
                                                        int pass) {
    __shared__ uint32_t lh[TK_BINS];
    const uint64_t prefix = pass ? st[pass].prefix : 0;
    const int nb = 1 << tk_width(pass);
    for (int b = threadIdx.x; b < nb; b += 256) lh[b] = 0;
    __syncthreads();
    const int sh = tk_shift(pass);
    const uint64_t dmask = (uint64_t)nb - 1;
    const int hsh = pass ? tk_shift(pass - 1) : 64;    // bits at and above hsh must match the prefix
    const uint64_t want = hsh < 64 ? (prefix >> hsh) : 0;
    const int lane = threadIdx.x & 63;
    for (int64_t i0 = (int64_t)blockIdx.x * 256; i0 < n; i0 += (int64_t)gridDim.x * 256) {   // block-uniform trip
        const int64_t i = i0 + threadIdx.x;
        bool live = false;
        uint32_t bin = 0;
        if (i < n) {
            const uint64_t u = (uint64_t)keys[i] ^ 0x8000000000000000ull;
            live = hsh == 64 || (u >> hsh) == want;
            bin = (uint32_t)((u >> sh) & dmask);
        }
#pragma unroll
        for (int round = 0; round < 4; ++round) {
            const uint64_t act = __ballot(live);
            if (!act) break;
            const int leader = __ffsll((long long)act) - 1;
            const uint32_t lb = (uint32_t)__shfl(bin, leader);
            const uint64_t same = __ballot(live && bin == lb);
            if (lane == leader) atomicAdd(&lh[lb], (uint32_t)__popcll(same));
            if (live && bin == lb) live = false;
        }
        if (live) atomicAdd(&lh[bin], 1u);
    }
    __syncthreads();
    uint32_t* gh = hists + (size_t)pass * TK_BINS;
    for (int b = threadIdx.x; b < nb; b += 256)
        if (lh[b]) atomicAdd(&gh[b], lh[b]);
}

// the keys >= the threshold, unordered; among keys EQUAL to the threshold only
// the `need` first to claim a slot are taken (distinct keys: exactly one)
__global__ __launch_bounds__(256) void topk_gather_kernel(const int64_t* __restrict__ keys, int64_t n,
                                                          const TkState* __restrict__ st,
                                                          unsigned long long* __restrict__ counters,
                                                          uint64_t* __restrict__ sel_u, int64_t* __restrict__ sel_pos) {
    const uint64_t thr = st[TK_PASSES].prefix;
    const int64_t need = st[TK_PASSES].need;
    __shared__ uint32_t cnt, base;
    __shared__ uint64_t su[256];
    __shared__ int64_t sp[256];
    for (int64_t i0 = (int64_t)blockIdx.x * 256; i0 < n; i0 += (int64_t)gridDim.x * 256) {
        if (threadIdx.x == 0) cnt = 0;
        __syncthreads();
        const int64_t i = i0 + threadIdx.x;
        if (i < n) {
            const uint64_t u = (uint64_t)keys[i] ^ 0x8000000000000000ull;
            bool take = u > thr;
            if (u == thr) take = atomicAdd(&counters[1], 1ull) < (unsigned long long)need;
            if (take) {
                const uint32_t s = atomicAdd(&cnt, 1u);
                su[s] = u;
                sp[s] = i;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0 && cnt) base = (uint32_t)atomicAdd(&counters[0], (unsigned long long)cnt);
        __syncthreads();
        if (threadIdx.x < cnt) {
            sel_u[base + threadIdx.x] = su[threadIdx.x];
            sel_pos[base + threadIdx.x] = sp[threadIdx.x];
        }
        __syncthreads();
    }
}

constexpr int RS_CHUNK = 2048;

// rank[i] += #{j in this block's chunk : u_j before u_i} (DESC: larger first;
// ties by position, lower first)
template <bool DESC>
__global__ __launch_bounds__(256) void rank_count_kernel(const uint64_t* __restrict__ u, int64_t n,
                                                         uint32_t* __restrict__ rank) {
    __shared__ __attribute__((aligned(16))) uint64_t su[RS_CHUNK];
    const int64_t c0 = (int64_t)blockIdx.y * RS_CHUNK;
    const int cn = (int)((n - c0) < RS_CHUNK ? (n - c0) : RS_CHUNK);
    const int cp = (cn + 7) & ~7;
    // padding never counts: DESC pads 0 (never above a key; an equal 0 sits at j >= jt),
    // ascending pads ~0
    for (int j = threadIdx.x; j < cp; j += 256) su[j] = j < cn ? u[c0 + j] : (DESC ? 0ull : ~0ull);
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t ui = u[i];
    // chunk positions j < jt are below i: equal keys there come first (stable)
    const int64_t jt64 = i - c0;
    const int jt = jt64 < 0 ? 0 : (jt64 > cn ? cn : (int)jt64);
    uint32_t r = 0;
    const ulonglong2* s2 = reinterpret_cast<const ulonglong2*>(su);
    for (int j = 0; j < cp; j += 8) {                  // 4 x ds_read_b128 in flight per step
        ulonglong2 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = s2[(j >> 1) + q];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int ja = j + 2 * q;
            if constexpr (DESC) {
                r += (v[q].x > ui) | ((v[q].x == ui) & (ja < jt));
                r += (v[q].y > ui) | ((v[q].y == ui) & (ja + 1 < jt));
            } else {
                r += (v[q].x < ui) | ((v[q].x == ui) & (ja < jt));
                r += (v[q].y < ui) | ((v[q].y == ui) & (ja + 1 < jt));
            }
        }
    }
    if (gridDim.y == 1) rank[i] = r;
    else if (r) atomicAdd(&rank[i], r);
}

__global__ void rank_scatter_kernel(const uint64_t* __restrict__ u, const int64_t* __restrict__ pos,
                                    const uint32_t* __restrict__ rank, int64_t n, int signed_out,
                                    uint64_t* __restrict__ out_u, int64_t* __restrict__ out_pos) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = rank[i];
    out_u[r] = signed_out ? (u[i] ^ 0x8000000000000000ull) : u[i];
    if (out_pos) out_pos[r] = pos ? pos[i] : i;
}

// Beyond RS_MAX keys the O(n^2) count costs more than a bitonic network: a
// permutation p (padded to a power of two with -1 = "after every key") is
// sorted by (key, position) with global compare-exchange passes, then
// scattered.
constexpr int64_t RS_MAX = 32768;

__global__ void perm_init_kernel(int32_t* __restrict__ p, int64_t n, int64_t npad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < npad) p[i] = i < n ? (int32_t)i : -1;
}

template <bool DESC>
__device__ __forceinline__ bool perm_before(const uint64_t* u, int32_t a, int32_t b) {
    if (a < 0) return false;
    if (b < 0) return true;
    const uint64_t ua = u[a], ub = u[b];
    if (ua != ub) return DESC ? ua > ub : ua < ub;
    return a < b;
}

template <bool DESC>
__global__ void bitonic_perm_kernel(const uint64_t* __restrict__ u, int32_t* __restrict__ p, int64_t npad,
                                    int64_t kk, int64_t j) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (npad >> 1)) return;
    const int64_t i = 2 * t - (t & (j - 1));
    const int64_t q = i + j;
    const bool up = (i & kk) == 0;
    const int32_t a = p[i], b = p[q];
    const bool swap = up ? perm_before<DESC>(u, b, a) : perm_before<DESC>(u, a, b);
    if (swap) { p[i] = b; p[q] = a; }
}

__global__ void perm_scatter_kernel(const uint64_t* __restrict__ u, const int64_t* __restrict__ pos,
                                    const int32_t* __restrict__ p, int64_t n, int signed_out,
                                    uint64_t* __restrict__ out_u, int64_t* __restrict__ out_pos) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int32_t i = p[r];
    out_u[r] = signed_out ? (u[i] ^ 0x8000000000000000ull) : u[i];
    if (out_pos) out_pos[r] = pos ? pos[i] : i;
}

static int64_t pow2_ge(int64_t n) {
    int64_t q = 1;
    while (q < n) q <<= 1;
    return q;
}

// scratch (rank) bytes the sort of n keys needs
size_t rank_sort_scratch_bytes(int64_t n) {
    if (n <= RS_MAX) return sizeof(uint32_t) * (size_t)(n > 0 ? n : 1);
    return sizeof(int32_t) * (size_t)pow2_ge(n);
}

// Stable sort of n uint64 keys (ascending, or descending with desc) into
// out_u, positions (pos[i], or i) into out_pos (nullable); rank: n uint32 of
// device scratch.  Used by m3d_nms3d (ascending keys) and m3d_topk_keys.
int rank_sort_u64(const uint64_t* u, const int64_t* pos, int64_t n, bool desc, bool signed_out, uint32_t* rank,
                  uint64_t* out_u, int64_t* out_pos, hipStream_t s) {
    if (n <= 0) return M3D_OK;
    if (n > RS_MAX) {
        int32_t* p = reinterpret_cast<int32_t*>(rank);
        const int64_t npad = pow2_ge(n);
        hipLaunchKernelGGL(perm_init_kernel, dim3(grid_for(npad, 256)), dim3(256), 0, s, p, n, npad);
        for (int64_t kk = 2; kk <= npad; kk <<= 1)
            for (int64_t j = kk >> 1; j > 0; j >>= 1) {
                if (desc)
                    hipLaunchKernelGGL(bitonic_perm_kernel<true>, dim3(grid_for(npad / 2, 256)), dim3(256), 0, s, u,
                                       p, npad, kk, j);
                else
                    hipLaunchKernelGGL(bitonic_perm_kernel<false>, dim3(grid_for(npad / 2, 256)), dim3(256), 0, s,
                                       u, p, npad, kk, j);
            }
        int rc = check_launch("bitonic_perm_kernel");
        if (rc) return rc;
        hipLaunchKernelGGL(perm_scatter_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, u, pos, p, n,
                           signed_out ? 1 : 0, out_u, out_pos);
        return check_launch("perm_scatter_kernel");
    }
    const unsigned chunks = (unsigned)((n + RS_CHUNK - 1) / RS_CHUNK);
    if (chunks > 1 && hipMemsetAsync(rank, 0, sizeof(uint32_t) * n, s) != hipSuccess)
        return check_launch("rank_sort: memset");
    const dim3 grid((unsigned)((n + 255) / 256), chunks);
    if (desc)
        hipLaunchKernelGGL(rank_count_kernel<true>, grid, dim3(256), 0, s, u, n, rank);
    else
        hipLaunchKernelGGL(rank_count_kernel<false>, grid, dim3(256), 0, s, u, n, rank);
    int rc = check_launch("rank_count_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(rank_scatter_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, u, pos, rank, n,
                       signed_out ? 1 : 0, out_u, out_pos);
    return check_launch("rank_scatter_kernel");
}

struct TopkWs {
    uint32_t* hists;
    unsigned long long* counters;
    TkState* st;
    uint64_t* sel_u;
    int64_t* sel_pos;
    uint32_t* rank;
    size_t bytes;
};

static TopkWs topk_ws(int64_t k, void* base) {
    TopkWs w{};
    char* p = (char*)base;
    size_t off = 0;
    auto take = [&](size_t b) {
        size_t o = off;
        off += (b + 255) & ~(size_t)255;
        return p ? p + o : nullptr;
    };
    const int64_t kk = k > 0 ? k : 1;
    w.hists = (uint32_t*)take(sizeof(uint32_t) * TK_PASSES * TK_BINS + 2 * sizeof(unsigned long long));
    w.counters = w.hists ? (unsigned long long*)(w.hists + TK_PASSES * TK_BINS) : nullptr;
    w.st = (TkState*)take(sizeof(TkState) * (TK_PASSES + 1));
    w.sel_u = (uint64_t*)take(sizeof(uint64_t) * kk);
    w.sel_pos = (int64_t*)take(sizeof(int64_t) * kk);
    w.rank = (uint32_t*)take(rank_sort_scratch_bytes(kk));
    w.bytes = off;
    return w;
}

}  // namespace m3d

using namespace m3d;

extern "C" size_t m3d_topk_workspace_bytes(int64_t n, int64_t k) {
    (void)n;
    return topk_ws(k, nullptr).bytes;
}

extern "C" int m3d_topk_keys(const int64_t* keys, int64_t n, int64_t k, int64_t* out_keys, int64_t* out_pos,
                             void* workspace, size_t ws_bytes, m3d_stream_t s) {
    if (n < 0 || k < 0) return einval("topk: negative size");
    if (k > n) return einval("input must have at least k columns");    // tf.nn.top_k's InvalidArgument
    if (n > 0xFFFFFFFFll) return einval("topk: more than 2^32 keys");
    if (k == 0) return M3D_OK;
    if (!keys || !out_keys) return einval("topk: null pointer");
    const TopkWs need = topk_ws(k, nullptr);
    if (!workspace || ws_bytes < need.bytes) return einval("topk: workspace too small");
    TopkWs w = topk_ws(k, workspace);
    if (hipMemsetAsync(w.hists, 0, sizeof(uint32_t) * TK_PASSES * TK_BINS + 2 * sizeof(unsigned long long), st(s)) !=
        hipSuccess)
        return check_launch("topk: memset");
    const unsigned grid = (unsigned)std::min<int64_t>((n + 1023) / 1024, 1024);
    for (int p = 0; p < TK_PASSES; ++p) {
        hipLaunchKernelGGL(topk_hist_kernel, dim3(grid), dim3(256), 0, st(s), keys, n, w.st, w.hists, p);
        hipLaunchKernelGGL(tk_state_kernel, dim3(1), dim3(256), 0, st(s), w.hists, p, k, w.st);
        int rc = check_launch("topk_hist_kernel");
        if (rc) return rc;
    }
    hipLaunchKernelGGL(topk_gather_kernel, dim3(grid), dim3(256), 0, st(s), keys, n, w.st, w.counters,
                       w.sel_u, w.sel_pos);
    int rc = check_launch("topk_gather_kernel");
    if (rc) return rc;
    return rank_sort_u64(w.sel_u, w.sel_pos, k, true, true, w.rank, reinterpret_cast<uint64_t*>(out_keys),
                         out_pos, st(s));
}

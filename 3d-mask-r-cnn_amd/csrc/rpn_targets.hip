// build_rpn_targets (ATSS variant, core/data_generators.py:2031-2178) on gfx950.
//
// The reference runs this per training volume in host numpy over the full
// [A x G] IoU matrix (A = 4.19 M anchors at 256^3); here it is a handful of
// launches over the device-resident anchors, no [A x G] matrix:
//   K1 rpn_iou_kernel      per anchor: IoU with every GT (compute_overlaps_3d
//                          order), max + first argmax; per GT: first-max
//                          anchor (64-bit atomicMax of (iou, ~index)) and the
//                          list of anchors with IoU > 0 (the only possible
//                          members of a top-k unless a GT has fewer than k).
//   K2 rpn_label_kernel    rpn_match = gt-argmax -> 1, < neg -> -1, >= pos -> 1
//   K3 atss_kernel         one workgroup per GT: exact top-k of its list by
//                          (IoU desc, index asc) with an 8-pass 8-bit radix
//                          select, mean / std over the k IoUs (missing = 0),
//                          thr = max(pos, mu + sd), marks IoU >= thr (or the
//                          top ATSS_MIN_POS when fewer) positive.
//   balancing              keep the RPN_TRAIN_ANCHORS_PER_IMAGE * ratio
//                          positives with the largest IoU max (index asc on
//                          ties), and a seeded random subset of the negatives
//                          (replaces np.random.choice): both via a global
//                          radix select over 64-bit keys.
//   deltas                 positives in anchor order (block scan), box
//                          refinement / RPN_BBOX_STD_DEV into rpn_bbox.
// Tie rules where the reference is implementation-defined (np.argpartition /
// unstable argsort order) are: larger IoU first, then smaller anchor index.
#include <float.h>

#include <vector>

#include "common.h"

namespace m3d {

constexpr int RT_MAX_G = 256;

struct G6 { float v[6]; };

__device__ __forceinline__ float iou_np(const float* a0, const float* b0) {
    // core/utils.py:78-143 compute_overlaps_3d: corners normalised by min/max,
    // union floored at 1e-10, result clipped to [0, 1]; float32 op order kept.
    float a[6], b[6];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        a[q] = smin(a0[q], a0[q + 3]); a[q + 3] = smax(a0[q], a0[q + 3]);
        b[q] = smin(b0[q], b0[q + 3]); b[q + 3] = smax(b0[q], b0[q + 3]);
    }
    const float y1 = smax(a[0], b[0]), x1 = smax(a[1], b[1]), z1 = smax(a[2], b[2]);
    const float y2 = smin(a[3], b[3]), x2 = smin(a[4], b[4]), z2 = smin(a[5], b[5]);
    const float inter = smax(y2 - y1, 0.0f) * smax(x2 - x1, 0.0f) * smax(z2 - z1, 0.0f);
    const float va = (a[3] - a[0]) * (a[4] - a[1]) * (a[5] - a[2]);
    const float vb = (b[3] - b[0]) * (b[4] - b[1]) * (b[5] - b[2]);
    const float uni = smax(va + vb - inter, 1e-10f);
    return smin(smax(inter / uni, 0.0f), 1.0f);
}

__device__ __forceinline__ uint64_t iou_key(float iou, int64_t i) {
    return ((uint64_t)__float_as_uint(iou) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
}

// Per-GT maxima and list appends are aggregated per workgroup in LDS (one
// global atomic per GT per workgroup); the appends reserve a range per GT and
// a second sweep (IoUs recomputed) writes the entries.
__global__ __launch_bounds__(256) void rpn_iou_kernel(const float* __restrict__ anchors, int64_t A,
                                                      const float* __restrict__ gt, int G,
                                                      float* __restrict__ iou_max, int32_t* __restrict__ arg,
                                                      unsigned long long* __restrict__ gt_best,
                                                      uint64_t* __restrict__ lists, int32_t* __restrict__ list_n,
                                                      int cap) {
    __shared__ float sg[RT_MAX_G][6];
    __shared__ unsigned long long sbest[RT_MAX_G];
    __shared__ int scount[RT_MAX_G], sbase[RT_MAX_G];
    for (int q = threadIdx.x; q < G * 6; q += blockDim.x) sg[q / 6][q % 6] = gt[q];
    for (int q = threadIdx.x; q < G; q += blockDim.x) { sbest[q] = 0ull; scount[q] = 0; }
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < A;
    float a[6] = {0, 0, 0, 0, 0, 0};
    if (live) {
#pragma unroll
        for (int q = 0; q < 6; ++q) a[q] = anchors[i * 6 + q];
        float best = -1.0f;
        int bg = 0;
        for (int g = 0; g < G; ++g) {
            const float v = iou_np(a, sg[g]);
            if (v > best) { best = v; bg = g; }             // np.argmax: first max
            atomicMax(&sbest[g], (unsigned long long)iou_key(v, i));
            if (v > 0.0f) atomicAdd(&scount[g], 1);
        }
        iou_max[i] = best;
        arg[i] = bg;
    }
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
        atomicMax(gt_best + g, sbest[g]);
        sbase[g] = scount[g] ? atomicAdd(list_n + g, scount[g]) : 0;
        scount[g] = 0;
    }
    __syncthreads();
    if (!live) return;
    for (int g = 0; g < G; ++g) {
        const float v = iou_np(a, sg[g]);
        if (v > 0.0f) {
            const int slot = sbase[g] + atomicAdd(&scount[g], 1);
            if (slot < cap) lists[(int64_t)g * cap + slot] = iou_key(v, i);
        }
    }
}

__global__ __launch_bounds__(256) void rpn_label_kernel(const float* __restrict__ iou_max, int64_t A,
                                                        float pos_thr, float neg_thr,
                                                        int8_t* __restrict__ match) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A) return;
    const float m = iou_max[i];
    int8_t v = match[i];                                    // 1 where a GT's best anchor
    if (m < neg_thr) v = -1;                                // float32 compares (numpy
    if (m >= pos_thr) v = 1;                                // casts the Python threshold)
    match[i] = v;
}

__global__ void rpn_gt_best_kernel(const unsigned long long* __restrict__ gt_best, int G,
                                   int8_t* __restrict__ match) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    match[0xFFFFFFFFu - (uint32_t)(gt_best[g] & 0xFFFFFFFFull)] = 1;
}

// Top-k prefilter: a GT's IoU > 0 list holds ~10^5 anchors at 128^3, and one
// workgroup per GT radix-selecting over all of it (contended LDS histogram
// atomics, G workgroups on a 256-CU chip) took ~10 ms.  The global top-k
// keys lie in the union of every 4096-entry chunk's top-k, so the chunks'
// top-k (k rounds of a block max; keys are unique, 0 = empty slot) run in
// parallel first, and the per-GT kernel selects over their union.
constexpr int ATSS_CH = 4096, ATSS_KMAX = 64;

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t t = __shfl_xor(v, o);
        v = t > v ? t : v;
    }
    return v;
}

__global__ __launch_bounds__(256) void atss_chunk_topk_kernel(const uint64_t* __restrict__ lists,
                                                              const int32_t* __restrict__ list_n, int cap,
                                                              int k, int nch, uint64_t* __restrict__ cand) {
    __shared__ uint64_t red[4];
    const int g = blockIdx.y, c = blockIdx.x, tid = threadIdx.x;
    const int n = list_n[g] < cap ? list_n[g] : cap;
    uint64_t* out = cand + ((int64_t)g * nch + c) * k;
    const int64_t base = (int64_t)c * ATSS_CH;
    if (base >= n) {                                        // past the list: empty slots
        for (int r = tid; r < k; r += 256) out[r] = 0ull;
        return;
    }
    uint64_t v[ATSS_CH / 256];
#pragma unroll
    for (int q = 0; q < ATSS_CH / 256; ++q) {
        const int64_t j = base + tid + 256 * q;
        v[q] = j < n ? lists[(int64_t)g * cap + j] : 0ull;
    }
    uint64_t last = ~0ull;
    for (int r = 0; r < k; ++r) {
        uint64_t best = 0;
#pragma unroll
        for (int q = 0; q < ATSS_CH / 256; ++q)
            if (v[q] < last && v[q] > best) best = v[q];
        best = wave_max_u64(best);
        if ((tid & 63) == 0) red[tid >> 6] = best;
        __syncthreads();
        uint64_t m = red[0];
        for (int w = 1; w < 4; ++w) m = red[w] > m ? red[w] : m;
        if (tid == 0) out[r] = m;
        last = m;
        __syncthreads();
    }
}

// sum over a 256-thread block: wave butterfly, then the four waves in order
__device__ __forceinline__ double block_sum_d(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const double r = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    return r;
}

// One workgroup per GT: k-th largest key of its list (radix select, 8-bit
// digits, over the chunk top-k union `cand` when given), stats over the
// top-k, ATSS marking.
__global__ __launch_bounds__(256) void atss_kernel(const uint64_t* __restrict__ lists,
                                                   const int32_t* __restrict__ list_n, int cap,
                                                   int64_t A, int topk_cfg, int min_pos, double pos_thr,
                                                   const uint64_t* __restrict__ cand_all, int ncand,
                                                   int8_t* __restrict__ match) {
    const int g = blockIdx.x;
    const uint64_t* L = lists + (int64_t)g * cap;
    const int n = list_n[g] < cap ? list_n[g] : cap;
    if (n == 0) return;                                     // `not np.any(ious_g > 0)`: skip
    const uint64_t* S = cand_all ? cand_all + (int64_t)g * ncand : L;   // selection set
    const int ns = cand_all ? ncand : n;
    const int k = (int)(topk_cfg < A ? topk_cfg : A);
    __shared__ unsigned hist[256];
    __shared__ uint64_t s_prefix;
    __shared__ int s_need;
    __shared__ double s_red[4];
    __shared__ int s_cand;
    const int tid = threadIdx.x;
    // threshold key K* = k-th largest key (or the smallest key if n <= k)
    const int kk = k < n ? k : n;
    if (tid == 0) { s_prefix = 0; s_need = kk; s_cand = 0; }
    __syncthreads();
    for (int pass = 0; pass < 8; ++pass) {
        const int shift = 56 - 8 * pass;
        for (int q = tid; q < 256; q += blockDim.x) hist[q] = 0;
        __syncthreads();
        const uint64_t pre = s_prefix;
        const uint64_t pmask = pass ? (~0ull << (64 - 8 * pass)) : 0ull;
        for (int j = tid; j < ns; j += blockDim.x) {
            const uint64_t key = S[j];
            if (key && (key & pmask) == pre) atomicAdd(&hist[(key >> shift) & 0xFF], 1u);
        }
        __syncthreads();
        if (tid == 0) {
            int need = s_need;
            int d = 255;
            for (; d > 0; --d) {
                if ((int)hist[d] >= need) break;
                need -= (int)hist[d];
            }
            s_prefix = pre | ((uint64_t)d << shift);
            s_need = need;
        }
        __syncthreads();
    }
    const uint64_t kth = s_prefix;                          // exact: keys are unique
    // mean / std over the top-k IoUs (entries beyond the list are zeros)
    // sums in a fixed order (per-thread strided, then a fixed tree): the same
    // mean / std on every run, unlike shared-memory atomics
    double sum = 0.0;
    for (int j = tid; j < n; j += blockDim.x)
        if (L[j] >= kth) sum += (double)__uint_as_float((uint32_t)(L[j] >> 32));
    const double mu = block_sum_d(sum, s_red) / (double)k;
    double sq = 0.0;
    for (int j = tid; j < n; j += blockDim.x)
        if (L[j] >= kth) {
            const double dv = (double)__uint_as_float((uint32_t)(L[j] >> 32)) - mu;
            sq += dv * dv;
        }
    const double ssq = block_sum_d(sq, s_red);
    const double zeros = (double)(k - kk);                  // top-k members with IoU 0
    const double sd = sqrt((ssq + zeros * mu * mu) / (double)k);
    // np.mean / np.std return float32; thr = max(pos, mu + sd) in Python
    // float; `ious_g >= thr` compares in float32
    const double s32 = (double)(float)mu + (double)(float)sd;
    const float thr = (float)(pos_thr > s32 ? pos_thr : s32);
    int c = 0;
    for (int j = tid; j < n; j += blockDim.x)
        if (__uint_as_float((uint32_t)(L[j] >> 32)) >= thr) ++c;
    atomicAdd(&s_cand, c);
    __syncthreads();
    if (s_cand >= min_pos) {
        for (int j = tid; j < n; j += blockDim.x)
            if (__uint_as_float((uint32_t)(L[j] >> 32)) >= thr)
                match[0xFFFFFFFFu - (uint32_t)(L[j] & 0xFFFFFFFFull)] = 1;
        return;
    }
    // fewer than ATSS_MIN_POS candidates: the min_pos best of the top-k
    // (IoU desc, index asc); if the list is shorter, the smallest-index
    // zero-IoU anchors complete it.
    const int mp = min_pos < k ? min_pos : k;
    if (tid == 0) {
        int taken = 0;
        uint64_t last = ~0ull;
        while (taken < mp && taken < n) {                   // selection by repeated max (mp small)
            uint64_t bestk = 0;
            for (int j = 0; j < ns; ++j)                    // the mp <= k best are in the selection set
                if (S[j] < last && S[j] > bestk) bestk = S[j];
            match[0xFFFFFFFFu - (uint32_t)(bestk & 0xFFFFFFFFull)] = 1;
            last = bestk;
            ++taken;
        }
        for (int64_t a = 0; taken < mp && a < A; ++a) {
            bool inlist = false;
            for (int j = 0; j < n && !inlist; ++j)
                inlist = (0xFFFFFFFFu - (uint32_t)(L[j] & 0xFFFFFFFFull)) == (uint32_t)a;
            if (!inlist) { match[a] = 1; ++taken; }
        }
    }
}

// ---- global top-k by key among flagged anchors (radix select, 8 passes) ----
struct SelState {
    uint64_t prefix;
    long long need;
    int active;                  // this balancing stage drops anchors
    unsigned long long hist[256];
};

// Balancing stage set-up on the device (no host round trip): stage 0 keeps
// the target_pos positives with the largest keys when there are more;
// stage 1 keeps min(total - positives, negatives) of the negatives.
__global__ void sel_init_kernel(const unsigned long long* __restrict__ cnt, int stage, int target_pos,
                                int total, SelState* st) {
    if (threadIdx.x == 0) {
        long long keep;
        bool active;
        if (stage == 0) {
            keep = target_pos;
            active = (long long)cnt[0] > keep;
        } else {
            keep = (long long)total - (long long)cnt[0];
            if (keep > (long long)cnt[1]) keep = (long long)cnt[1];
            active = (long long)cnt[1] > keep;
        }
        st->active = active ? 1 : 0;
        if (keep <= 0) {
            st->need = 0;
            st->prefix = stage == 0 ? ~0ull : 0ull;   // keep none (keys < ~0; hash keys > 0)
        } else {
            st->need = keep;
            st->prefix = 0;
        }
    }
    for (int q = threadIdx.x; q < 256; q += blockDim.x) st->hist[q] = 0;
}

// key of anchor i for the balancing selections: positives by (iou max, ~i),
// negatives by a seeded random 32-bit hash (then ~i)
__device__ __forceinline__ uint32_t mix32r(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint64_t sel_key(int mode, const float* iou_max, int64_t i, uint32_t seed) {
    if (mode == 0) return iou_key(iou_max[i], i);
    return ((uint64_t)mix32r((uint32_t)i * 0x9E3779B9u ^ seed) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
}

__global__ __launch_bounds__(256) void sel_hist_kernel(const int8_t* __restrict__ match, int64_t A, int want,
                                                       int mode, const float* __restrict__ iou_max,
                                                       uint32_t seed, int pass, SelState* st) {
    __shared__ unsigned h[256];
    for (int q = threadIdx.x; q < 256; q += blockDim.x) h[q] = 0;
    __syncthreads();
    const uint64_t pre = st->prefix;
    const int shift = 56 - 8 * pass;
    const uint64_t pmask = pass ? (~0ull << (64 - 8 * pass)) : 0ull;
    if (st->active && st->need > 0) {
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A;
             i += (int64_t)gridDim.x * blockDim.x) {
            if (match[i] != want) continue;
            const uint64_t key = sel_key(mode, iou_max, i, seed);
            if ((key & pmask) == pre) atomicAdd(&h[(key >> shift) & 0xFF], 1u);
        }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < 256; q += blockDim.x)
        if (h[q]) atomicAdd(&st->hist[q], (unsigned long long)h[q]);
}

// picks the digit holding the need-th largest key; mode 0 keeps the
// largest keys, mode 1 keeps the SMALLEST hash keys (need counted from below)
__global__ void sel_pick_kernel(SelState* st, int pass, int from_below) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    long long need = st->need;
    const int shift = 56 - 8 * pass;
    if (st->active && need > 0) {
        int d;
        if (!from_below) {
            for (d = 255; d > 0; --d) {
                if ((long long)st->hist[d] >= need) break;
                need -= (long long)st->hist[d];
            }
        } else {
            for (d = 0; d < 255; ++d) {
                if ((long long)st->hist[d] >= need) break;
                need -= (long long)st->hist[d];
            }
        }
        st->prefix |= (uint64_t)d << shift;
        st->need = need;
    }
    for (int q = 0; q < 256; ++q) st->hist[q] = 0;
}

// drop (set 0) the flagged anchors outside the kept set
__global__ __launch_bounds__(256) void sel_apply_kernel(int8_t* __restrict__ match, int64_t A, int want,
                                                        int mode, const float* __restrict__ iou_max,
                                                        uint32_t seed, const SelState* st, int from_below) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A || !st->active || match[i] != want) return;
    const uint64_t key = sel_key(mode, iou_max, i, seed);
    const uint64_t kth = st->prefix;
    const bool keep = from_below ? key <= kth : key >= kth;
    if (!keep) match[i] = 0;
}

__global__ __launch_bounds__(256) void count_kernel(const int8_t* __restrict__ match, int64_t A,
                                                    unsigned long long* __restrict__ cnt) {
    __shared__ unsigned cp, cn;
    if (threadIdx.x == 0) { cp = 0; cn = 0; }
    __syncthreads();
    unsigned p = 0, q = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A; i += (int64_t)gridDim.x * blockDim.x) {
        p += match[i] == 1;
        q += match[i] == -1;
    }
    atomicAdd(&cp, p);
    atomicAdd(&cn, q);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(cnt, (unsigned long long)cp);
        atomicAdd(cnt + 1, (unsigned long long)cn);
    }
}

// counts_dev[0..2] = positives, negatives, 1 if a GT's IoU>0 list overflowed list_cap
__global__ void counts_out_kernel(const unsigned long long* __restrict__ cnt, const int32_t* __restrict__ list_n,
                                  int G, int cap, int32_t* __restrict__ out) {
    if (threadIdx.x != 0) return;
    int over = 0;
    for (int g = 0; g < G; ++g) over |= list_n[g] > cap;
    out[0] = (int32_t)cnt[0];
    out[1] = (int32_t)cnt[1];
    out[2] = over;
}

// rpn_bbox rows: positives in ascending anchor order.  Block-level counts
// -> exclusive scan in one block -> write.
constexpr int SCAN_CHUNK = 4096;

__global__ __launch_bounds__(256) void pos_block_count_kernel(const int8_t* __restrict__ match, int64_t A,
                                                              int32_t* __restrict__ bcount) {
    __shared__ int c;
    if (threadIdx.x == 0) c = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * SCAN_CHUNK;
    int p = 0;
    for (int j = threadIdx.x; j < SCAN_CHUNK; j += blockDim.x) {
        const int64_t i = base + j;
        if (i < A && match[i] == 1) ++p;
    }
    atomicAdd(&c, p);
    __syncthreads();
    if (threadIdx.x == 0) bcount[blockIdx.x] = c;
}

__global__ void scan_kernel(int32_t* __restrict__ v, int n) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int s = 0;
    for (int j = 0; j < n; ++j) { const int t = v[j]; v[j] = s; s += t; }
}

__global__ __launch_bounds__(256) void pos_deltas_kernel(const int8_t* __restrict__ match, int64_t A,
                                                         const int32_t* __restrict__ boff,
                                                         const float* __restrict__ anchors,
                                                         const float* __restrict__ gt,
                                                         const int32_t* __restrict__ arg, G6 std6, int total,
                                                         float* __restrict__ rpn_bbox) {
    // one thread walks the block's chunk in order (positives are sparse)
    __shared__ int flags[SCAN_CHUNK];
    const int64_t base = (int64_t)blockIdx.x * SCAN_CHUNK;
    for (int j = threadIdx.x; j < SCAN_CHUNK; j += blockDim.x) {
        const int64_t i = base + j;
        flags[j] = (i < A && match[i] == 1) ? 1 : 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {                                  // in-LDS exclusive scan (sparse)
        int s = boff[blockIdx.x];
        for (int j = 0; j < SCAN_CHUNK; ++j) {
            const int f = flags[j];
            flags[j] = f ? s : -1;
            s += f;
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < SCAN_CHUNK; j += blockDim.x) {
        const int row = flags[j];
        if (row < 0 || row >= total) continue;
        const int64_t i = base + j;
        const float* an = anchors + i * 6;
        const float* g = gt + arg[i] * 6;
        const float eps = 1e-6f;
        const float ah = an[3] - an[0], aw = an[4] - an[1], ad = an[5] - an[2];
        const float acy = an[0] + 0.5f * ah, acx = an[1] + 0.5f * aw, acz = an[2] + 0.5f * ad;
        const float gh = g[3] - g[0], gw = g[4] - g[1], gd = g[5] - g[2];
        const float gcy = g[0] + 0.5f * gh, gcx = g[1] + 0.5f * gw, gcz = g[2] + 0.5f * gd;
        float d[6];
        d[0] = (gcy - acy) / smax(ah, eps);
        d[1] = (gcx - acx) / smax(aw, eps);
        d[2] = (gcz - acz) / smax(ad, eps);
        d[3] = logf(smax(gh, eps) / smax(ah, eps));
        d[4] = logf(smax(gw, eps) / smax(aw, eps));
        d[5] = logf(smax(gd, eps) / smax(ad, eps));
        for (int q = 0; q < 6; ++q) rpn_bbox[(int64_t)row * 6 + q] = d[q] / std6.v[q];
    }
}

}  // namespace m3d

using namespace m3d;

struct RtWs {
    float* iou_max;
    int32_t* arg;
    unsigned long long* gt_best;
    int32_t* list_n;
    uint64_t* lists;
    SelState* st;
    unsigned long long* cnt;
    int32_t* bcount;
    int32_t* cdev;
    uint64_t* cand;              // [G][nch][k] chunk top-k (k <= ATSS_KMAX)
};

static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

static size_t rt_layout(int64_t A, int64_t G, int64_t cap, char* base, RtWs* w) {
    size_t off = 0;
    auto take = [&](size_t bytes) { char* p = base ? base + off : nullptr; off += al256(bytes); return p; };
    const int64_t nb = (A + SCAN_CHUNK - 1) / SCAN_CHUNK;
    RtWs t{};
    t.iou_max = (float*)take(sizeof(float) * A);
    t.arg = (int32_t*)take(sizeof(int32_t) * A);
    t.gt_best = (unsigned long long*)take(sizeof(unsigned long long) * (G > 0 ? G : 1));
    t.list_n = (int32_t*)take(sizeof(int32_t) * (G > 0 ? G : 1));
    t.lists = (uint64_t*)take(sizeof(uint64_t) * (size_t)(G > 0 ? G : 1) * cap);
    t.st = (SelState*)take(sizeof(SelState));
    t.cnt = (unsigned long long*)take(sizeof(unsigned long long) * 2);
    t.bcount = (int32_t*)take(sizeof(int32_t) * (nb > 0 ? nb : 1));
    t.cdev = (int32_t*)take(sizeof(int32_t) * 3);
    t.cand = (uint64_t*)take(sizeof(uint64_t) * (size_t)(G > 0 ? G : 1) * ((cap + ATSS_CH - 1) / ATSS_CH) * ATSS_KMAX);
    if (w) *w = t;
    return off;
}

extern "C" size_t m3d_rpn_targets_workspace_bytes(int64_t A, int64_t G, int64_t list_cap) {
    return rt_layout(A, G, list_cap, nullptr, nullptr);
}

// Stream-ordered, no host round trip: the balancing stages are set up on the
// device from the label counts (sel_init_kernel), so a training step can build
// its targets on the GPU each iteration.  counts_dev (device int32[3], may be
// NULL): final positives, negatives, and 1 if a GT overlapped more than
// list_cap anchors (its ATSS candidate list was truncated; the synchronous
// m3d_rpn_targets reports that as M3D_EINVAL).
static int rpn_targets_impl(const float* anchors, int64_t A, const float* gt_boxes, int64_t G, float pos_iou,
                            float neg_iou, int32_t total, float positive_ratio, int32_t atss_topk,
                            int32_t atss_min_pos, const float rpn_bbox_std_dev[6], uint32_t seed,
                            int8_t* rpn_match, float* rpn_bbox, int64_t list_cap, void* workspace,
                            size_t ws_bytes, int32_t* counts_dev, hipStream_t hs) {
    if (A <= 0 || G < 0 || G > RT_MAX_G) return einval("rpn_targets: need A > 0 and 0 <= G <= 256");
    if (A > 0xFFFFFFFFll) return einval("rpn_targets: more than 2^32 anchors");
    if (total <= 0) return einval("rpn_targets: RPN_TRAIN_ANCHORS_PER_IMAGE must be positive");
    if (list_cap <= 0 || list_cap > 0x7FFFFFFF) return einval("rpn_targets: list_cap must be in [1, 2^31)");
    if (ws_bytes < m3d_rpn_targets_workspace_bytes(A, G, list_cap)) return einval("rpn_targets: workspace too small");
    RtWs w{};
    rt_layout(A, G, list_cap, (char*)workspace, &w);
    if (hipMemsetAsync(rpn_bbox, 0, sizeof(float) * 6 * (size_t)total, hs) != hipSuccess)
        return check_launch("memset rpn_bbox");
    if (G == 0) {                                            // empty GT: everything negative
        if (hipMemsetAsync(rpn_match, 0xFF, (size_t)A, hs) != hipSuccess) return check_launch("memset");
        if (counts_dev) {
            if (hipMemsetAsync(w.cnt, 0, sizeof(unsigned long long) * 2, hs) != hipSuccess)
                return check_launch("memset");
            hipLaunchKernelGGL(count_kernel, dim3(1024), dim3(256), 0, hs, rpn_match, A, w.cnt);
            hipLaunchKernelGGL(counts_out_kernel, dim3(1), dim3(64), 0, hs, w.cnt, w.list_n, 0, (int)list_cap,
                               counts_dev);
            return check_launch("rpn_targets counts");
        }
        return M3D_OK;
    }
    if (hipMemsetAsync(rpn_match, 0, (size_t)A, hs) != hipSuccess ||
        hipMemsetAsync(w.gt_best, 0, sizeof(unsigned long long) * G, hs) != hipSuccess ||
        hipMemsetAsync(w.list_n, 0, sizeof(int32_t) * G, hs) != hipSuccess)
        return check_launch("memset");
    const unsigned gA = grid_for(A, 256);
    hipLaunchKernelGGL(rpn_iou_kernel, dim3(gA), dim3(256), 0, hs, anchors, A, gt_boxes, (int)G, w.iou_max, w.arg,
                       w.gt_best, w.lists, w.list_n, (int)list_cap);
    hipLaunchKernelGGL(rpn_gt_best_kernel, dim3(1), dim3(RT_MAX_G), 0, hs, w.gt_best, (int)G, rpn_match);
    hipLaunchKernelGGL(rpn_label_kernel, dim3(gA), dim3(256), 0, hs, w.iou_max, A, pos_iou, neg_iou, rpn_match);
    const int kk = (int)(atss_topk < A ? atss_topk : A);
    const int nch = (int)((list_cap + ATSS_CH - 1) / ATSS_CH);
    const bool pre = kk >= 1 && kk <= ATSS_KMAX && nch > 1;
    if (pre)
        hipLaunchKernelGGL(atss_chunk_topk_kernel, dim3((unsigned)nch, (unsigned)G), dim3(256), 0, hs, w.lists,
                           w.list_n, (int)list_cap, kk, nch, w.cand);
    hipLaunchKernelGGL(atss_kernel, dim3((unsigned)G), dim3(256), 0, hs, w.lists, w.list_n, (int)list_cap, A,
                       (int)atss_topk, (int)atss_min_pos, (double)pos_iou, pre ? w.cand : nullptr, nch * kk,
                       rpn_match);
    int rc = check_launch("rpn_targets labels");
    if (rc) return rc;
    // balancing (core/data_generators.py:2150-2165)
    const int target_pos = (int)nearbyint((double)total * (double)positive_ratio);   // round() half-even
    auto count = [&]() {
        if (hipMemsetAsync(w.cnt, 0, sizeof(unsigned long long) * 2, hs) != hipSuccess) return check_launch("memset");
        hipLaunchKernelGGL(count_kernel, dim3(1024), dim3(256), 0, hs, rpn_match, A, w.cnt);
        return check_launch("count_kernel");
    };
    auto stage = [&](int st_id, int want, int mode, int from_below) {
        hipLaunchKernelGGL(sel_init_kernel, dim3(1), dim3(256), 0, hs, w.cnt, st_id, target_pos, (int)total, w.st);
        for (int pass = 0; pass < 8; ++pass) {
            hipLaunchKernelGGL(sel_hist_kernel, dim3(1024), dim3(256), 0, hs, rpn_match, A, want, mode, w.iou_max,
                               seed, pass, w.st);
            hipLaunchKernelGGL(sel_pick_kernel, dim3(1), dim3(64), 0, hs, w.st, pass, from_below);
        }
        hipLaunchKernelGGL(sel_apply_kernel, dim3(gA), dim3(256), 0, hs, rpn_match, A, want, mode, w.iou_max, seed,
                           w.st, from_below);
        return check_launch("rpn_targets balancing");
    };
    if ((rc = count()) || (rc = stage(0, 1, 0, 0)) || (rc = count()) || (rc = stage(1, -1, 1, 1))) return rc;
    // deltas of the positives in anchor order
    const unsigned nb = (unsigned)((A + SCAN_CHUNK - 1) / SCAN_CHUNK);
    hipLaunchKernelGGL(pos_block_count_kernel, dim3(nb), dim3(256), 0, hs, rpn_match, A, w.bcount);
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(64), 0, hs, w.bcount, (int)nb);
    G6 sd{};
    for (int q = 0; q < 6; ++q) sd.v[q] = rpn_bbox_std_dev[q];
    hipLaunchKernelGGL(pos_deltas_kernel, dim3(nb), dim3(256), 0, hs, rpn_match, A, w.bcount, anchors, gt_boxes,
                       w.arg, sd, (int)total, rpn_bbox);
    if ((rc = check_launch("rpn_targets deltas"))) return rc;
    if (counts_dev) {
        if ((rc = count())) return rc;
        hipLaunchKernelGGL(counts_out_kernel, dim3(1), dim3(64), 0, hs, w.cnt, w.list_n, (int)G, (int)list_cap,
                           counts_dev);
        return check_launch("rpn_targets counts");
    }
    return M3D_OK;
}

extern "C" int m3d_rpn_targets_async(const float* anchors, int64_t A, const float* gt_boxes, int64_t G,
                                     float pos_iou, float neg_iou, int32_t total, float positive_ratio,
                                     int32_t atss_topk, int32_t atss_min_pos, const float rpn_bbox_std_dev[6],
                                     uint32_t seed, int8_t* rpn_match, float* rpn_bbox, int64_t list_cap,
                                     void* workspace, size_t ws_bytes, int32_t* counts_dev, m3d_stream_t s) {
    return rpn_targets_impl(anchors, A, gt_boxes, G, pos_iou, neg_iou, total, positive_ratio, atss_topk,
                            atss_min_pos, rpn_bbox_std_dev, seed, rpn_match, rpn_bbox, list_cap, workspace,
                            ws_bytes, counts_dev, st(s));
}

// The data-loader form (the reference runs build_rpn_targets in numpy in its
// generator): the async path, then the counts read back once (stream sync)
// and a truncated candidate list reported as M3D_EINVAL.
extern "C" int m3d_rpn_targets(const float* anchors, int64_t A, const float* gt_boxes, int64_t G,
                               float pos_iou, float neg_iou, int32_t total, float positive_ratio,
                               int32_t atss_topk, int32_t atss_min_pos, const float rpn_bbox_std_dev[6],
                               uint32_t seed, int8_t* rpn_match, float* rpn_bbox, int64_t list_cap,
                               void* workspace, size_t ws_bytes, int32_t* counts_out, m3d_stream_t s) {
    hipStream_t hs = st(s);
    int rc = rpn_targets_impl(anchors, A, gt_boxes, G, pos_iou, neg_iou, total, positive_ratio, atss_topk,
                              atss_min_pos, rpn_bbox_std_dev, seed, rpn_match, rpn_bbox, list_cap, workspace,
                              ws_bytes, nullptr, hs);
    if (rc) return rc;
    RtWs w{};
    rt_layout(A, G, list_cap, (char*)workspace, &w);
    if (hipMemsetAsync(w.cnt, 0, sizeof(unsigned long long) * 2, hs) != hipSuccess) return check_launch("memset");
    hipLaunchKernelGGL(count_kernel, dim3(1024), dim3(256), 0, hs, rpn_match, A, w.cnt);
    hipLaunchKernelGGL(counts_out_kernel, dim3(1), dim3(64), 0, hs, w.cnt, w.list_n, (int)G, (int)list_cap, w.cdev);
    int32_t hc[3];
    if (hipMemcpyAsync(hc, w.cdev, sizeof(hc), hipMemcpyDeviceToHost, hs) != hipSuccess ||
        hipStreamSynchronize(hs) != hipSuccess)
        return check_launch("rpn_targets counts");
    if (hc[2]) {
        set_error("rpn_targets: a GT overlaps more than list_cap=%lld anchors", (long long)list_cap);
        return M3D_EINVAL;
    }
    if (counts_out) {
        counts_out[0] = hc[0];
        counts_out[1] = hc[1];
    }
    return M3D_OK;
}

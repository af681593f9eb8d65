// 3-D non-max suppression and ProposalLayer kernels for gfx950.
//
// Replaces NonMaxSuppression3D of the vendored wheel (CPU-only; SURVEY.md
// 2.1, Appendix A.3) and the per-image TF glue of ProposalLayer
// (core/models.py:369-503).
//
// Pipeline for m3d_nms3d (all stream-ordered, no host sync):
//   1. keys:   64-bit (desc-orderable score << 32 | index); candidates with
//              score <= -FLT_MAX or NaN get the all-ones key (sorted last);
//              -0.0 is folded onto +0.0 so ties compare like floats.
//   2. sort:   ascending == (score desc, index asc), i.e. the pop order of
//              the reference's priority queue (A.3): the stable rank sort of
//              topk.hip (an O(N^2) parallel count up to 32768 keys -- 15000
//              candidates in ~20 us instead of 147 us for the single-workgroup
//              LDS bitonic network it replaced -- a bitonic permutation network
//              beyond).
//   3. mask:   64x64 tiles, one wave per tile, boxes of the column block
//              staged in LDS; bit j of word (i, jb) = IoU(i, j) > thr, j > i.
//              IoU op order is IOU<float> @0xb500 (compiled -ffp-contract=off,
//              IEEE divide) so the bits are identical to the reference's
//              comparisons.
//   4. reduce: one workgroup; per 64-row block wave 0 resolves the
//              intra-block dependencies in registers (readlane loop), then
//              all threads OR the kept rows into the LDS-resident removed
//              mask.  Kept original indices are written in selection order.
#include <float.h>
#include <stdlib.h>

#include "common.h"

namespace m3d {

__device__ __forceinline__ uint32_t float_ord(float f) {
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void nms_keys_kernel(const float* __restrict__ scores, int64_t N, int64_t Npad,
                                uint64_t* __restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Npad) return;
    uint64_t k = ~0ull;
    if (i < N) {
        float s = scores[i];
        if (s > -FLT_MAX) {
            if (s == 0.0f) s = 0.0f;  // fold -0.0
            k = ((uint64_t)(~float_ord(s)) << 32) | (uint64_t)(uint32_t)i;
        }
    }
    keys[i] = k;
}

__global__ void nms_gather_kernel(const float* __restrict__ boxes, const uint64_t* __restrict__ keys,
                                  int64_t N, int cols, float* __restrict__ sboxes) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const uint64_t k = keys[i];
    const uint32_t idx = (uint32_t)k;
    const bool valid = (k >> 32) != 0xFFFFFFFFull;
    for (int q = 0; q < 6; ++q)
        sboxes[i * 6 + q] = (valid && q < cols) ? boxes[(int64_t)idx * cols + q] : 0.0f;
}

// IOU<float> (@0xb500-0xb656) -- op order is load-bearing.
__device__ __forceinline__ float iou3d(const float* bi, const float* bj) {
    const float ymin_i = smin(bi[0], bi[3]), ymax_i = smax(bi[0], bi[3]);
    const float xmin_i = smin(bi[1], bi[4]), xmax_i = smax(bi[1], bi[4]);
    const float zmin_i = smin(bi[2], bi[5]), zmax_i = smax(bi[2], bi[5]);
    const float ymin_j = smin(bj[0], bj[3]), ymax_j = smax(bj[0], bj[3]);
    const float xmin_j = smin(bj[1], bj[4]), xmax_j = smax(bj[1], bj[4]);
    const float zmin_j = smin(bj[2], bj[5]), zmax_j = smax(bj[2], bj[5]);
    const float area_i = ((ymax_i - ymin_i) * (xmax_i - xmin_i)) * (zmax_i - zmin_i);
    const float area_j = ((ymax_j - ymin_j) * (xmax_j - xmin_j)) * (zmax_j - zmin_j);
    if (area_i <= 0 || area_j <= 0) return 0.0f;
    const float iymin = smax(ymin_i, ymin_j), iymax = smin(ymax_i, ymax_j);
    const float ixmin = smax(xmin_i, xmin_j), ixmax = smin(xmax_i, xmax_j);
    const float izmin = smax(zmin_i, zmin_j), izmax = smin(zmax_i, zmax_j);
    const float inter =
        (smax(iymax - iymin, 0.0f) * smax(ixmax - ixmin, 0.0f)) * smax(izmax - izmin, 0.0f);
    return inter / ((area_i + area_j) - inter);
}

// TF 2.2 IOU<float> on (y1,x1,y2,x2) rows (stored in the first 4 of 6 slots).
__device__ __forceinline__ float iou2d(const float* bi, const float* bj) {
    const float ymin_i = smin(bi[0], bi[2]), ymax_i = smax(bi[0], bi[2]);
    const float xmin_i = smin(bi[1], bi[3]), xmax_i = smax(bi[1], bi[3]);
    const float ymin_j = smin(bj[0], bj[2]), ymax_j = smax(bj[0], bj[2]);
    const float xmin_j = smin(bj[1], bj[3]), xmax_j = smax(bj[1], bj[3]);
    const float area_i = (ymax_i - ymin_i) * (xmax_i - xmin_i);
    const float area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j);
    if (area_i <= 0 || area_j <= 0) return 0.0f;
    const float iymin = smax(ymin_i, ymin_j), iymax = smin(ymax_i, ymax_j);
    const float ixmin = smax(xmin_i, xmin_j), ixmax = smin(xmax_i, xmax_j);
    const float inter = smax(iymax - iymin, 0.0f) * smax(ixmax - ixmin, 0.0f);
    return inter / ((area_i + area_j) - inter);
}

__global__ __launch_bounds__(64) void nms_mask_kernel(const float* __restrict__ sboxes, int64_t N,
                                                      int64_t cb, float thr, int mode,
                                                      uint64_t* __restrict__ mask) {
    const int64_t ib = blockIdx.y, jb = blockIdx.x;
    if (jb < ib) return;
    __shared__ float cbox[64 * 6];
    const int t = threadIdx.x;
    const int64_t j0 = jb * 64;
    for (int q = t; q < 64 * 6; q += 64) {
        const int64_t g = j0 * 6 + q;
        cbox[q] = (g < N * 6) ? sboxes[g] : 0.0f;
    }
    __syncthreads();
    const int64_t i = ib * 64 + t;
    if (i >= N) return;
    float bi[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) bi[q] = sboxes[i * 6 + q];
    uint64_t bits = 0;
    const int start = (jb == ib) ? t + 1 : 0;
    for (int q = start; q < 64; ++q) {
        const int64_t j = j0 + q;
        if (j >= N) break;
        const float sim = mode == 1 ? iou2d(bi, cbox + q * 6) : iou3d(bi, cbox + q * 6);
        if (sim > thr) bits |= (1ull << q);
    }
    mask[i * cb + jb] = bits;
}

// Greedy reduction.  removed[] lives in LDS (cb words, cb <= 16384).
// Per 64-row block: wave 0 resolves the block serially in registers
// (readlane over the diagonal mask words), then ALL threads OR the kept rows'
// mask words into removed[] -- one independent global load per (kept row,
// word) pair, folded with LDS 64-bit atomic ORs, so the global latency is paid
// once per block instead of once per kept row.
__global__ __launch_bounds__(1024) void nms_reduce_kernel(const uint64_t* __restrict__ mask,
                                                          const uint64_t* __restrict__ keys,
                                                          int64_t N, int64_t cb, int max_out,
                                                          int32_t* __restrict__ keep,
                                                          int32_t* __restrict__ num_keep) {
    extern __shared__ __attribute__((aligned(16))) uint64_t removed[];
    __shared__ int kept_rows[64];
    __shared__ int nkept_sh, nkeep_sh, stop_sh;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int64_t w = tid; w < cb; w += blockDim.x) removed[w] = 0;
    if (tid == 0) { nkeep_sh = 0; stop_sh = 0; nkept_sh = 0; }
    __syncthreads();
    // wave 0 keeps the next block's keys / diagonal words in flight across the
    // OR phase (the mask is read-only), hiding one global round trip per block
    uint64_t key_n = 0, diag_n = 0;
    if (wave == 0) {
        key_n = lane < N ? keys[lane] : ~0ull;
        diag_n = lane < N ? mask[(int64_t)lane * cb] : 0ull;
    }
    for (int64_t blk = 0; blk < cb; ++blk) {
        if (wave == 0) {
            const int64_t row = blk * 64 + lane;
            const uint64_t key = key_n;
            const bool valid = row < N && (key >> 32) != 0xFFFFFFFFull;
            const uint64_t diag = valid ? diag_n : 0ull;
            if (blk + 1 < cb) {
                const int64_t rn = row + 64;
                key_n = rn < N ? keys[rn] : ~0ull;
                diag_n = rn < N ? mask[rn * cb + blk + 1] : 0ull;
            }
            const uint64_t vmask = __ballot(valid);
            uint64_t rem = removed[blk];
            uint64_t kept = 0;
            const int nk0 = nkeep_sh;
            int nk = nk0;
            const uint32_t dlo = (uint32_t)diag, dhi = (uint32_t)(diag >> 32);
            for (int r = 0; r < 64; ++r) {
                if (!((vmask >> r) & 1ull)) break;            // sorted: rest invalid
                if (nk >= max_out) break;
                if (!((rem >> r) & 1ull)) {
                    kept |= (1ull << r);
                    ++nk;
                    const uint64_t d = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(dlo, r) |
                                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(dhi, r) << 32);
                    rem |= d;
                }
            }
            if ((kept >> lane) & 1ull) {
                const int j = __popcll(kept & ((1ull << lane) - 1ull));
                keep[nk0 + j] = (int32_t)(uint32_t)key;
                kept_rows[j] = lane;
            }
            if (lane == 0) {
                nkept_sh = nk - nk0;
                nkeep_sh = nk;
                if (nk >= max_out || vmask != ~0ull) stop_sh = 1;
            }
        }
        __syncthreads();
        if (stop_sh) break;
        const int nkb = nkept_sh;
        const int64_t w0 = blk + 1, nw = cb - w0;
        const int64_t total = (int64_t)nkb * nw;
        const uint64_t* mrow = mask + (blk * 64) * cb;
        for (int64_t p0 = tid; p0 < total; p0 += 4 * (int64_t)blockDim.x) {
            uint64_t v[4];
            int64_t wi[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t p = p0 + (int64_t)u * blockDim.x;
                v[u] = 0;
                wi[u] = -1;
                if (p < total) {
                    const int i = (int)(p / nw);
                    wi[u] = w0 + p % nw;
                    v[u] = mrow[(int64_t)kept_rows[i] * cb + wi[u]];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (v[u]) atomicOr((unsigned long long*)&removed[wi[u]], (unsigned long long)v[u]);
        }
        __syncthreads();
    }
    if (tid == 0) *num_keep = nkeep_sh;
}

// Greedy reduction for cb <= 256 (N <= 16384, every ProposalLayer shape of the
// configs): thread (g, w) owns mask word w of the block rows g, g+G, ... (G =
// 1024 / cb row groups), so the OR phase needs no index arithmetic beyond the
// launch, and the NEXT block's rows are loaded into the second register buffer
// while wave 0 resolves the current block -- one global round trip per block
// is hidden instead of paid.  Same greedy result as nms_reduce_kernel.
constexpr int NR_RPG = 16;   // rows per group held per buffer (G >= 4)

__device__ __forceinline__ void nr_load(const uint64_t* __restrict__ mask, int64_t N, int64_t cb, int64_t blk,
                                        int g, int G, int w, bool own, uint64_t (&v)[NR_RPG]) {
#pragma unroll
    for (int k = 0; k < NR_RPG; ++k) {
        const int r = g + G * k;
        const int64_t row = blk * 64 + r;
        v[k] = (own && r < 64 && row < N && w > blk) ? mask[row * cb + w] : 0ull;
    }
}

__global__ __launch_bounds__(1024) void nms_reduce_pf_kernel(const uint64_t* __restrict__ mask,
                                                             const uint64_t* __restrict__ keys,
                                                             int64_t N, int64_t cb, int max_out,
                                                             int32_t* __restrict__ keep,
                                                             int32_t* __restrict__ num_keep) {
    __shared__ uint64_t removed[256];
    __shared__ uint64_t kept_sh;
    __shared__ int nkeep_sh, stop_sh;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = 1024 / (int)cb < 64 ? 1024 / (int)cb : 64;
    const int g = tid / (int)cb, w = tid % (int)cb;
    const bool own = g < G;
    for (int64_t q = tid; q < cb; q += blockDim.x) removed[q] = 0;
    if (tid == 0) { nkeep_sh = 0; stop_sh = 0; kept_sh = 0; }
    uint64_t va[NR_RPG], vb[NR_RPG];
    nr_load(mask, N, cb, 0, g, G, w, own, va);
    __syncthreads();
    uint64_t key_n = 0, diag_n = 0;
    if (wave == 0) {
        key_n = lane < N ? keys[lane] : ~0ull;
        diag_n = lane < N ? mask[(int64_t)lane * cb] : 0ull;
    }
    // one block: resolve (wave 0), then OR the kept rows of cur into removed[]
    auto block = [&](int64_t blk, const uint64_t (&cur)[NR_RPG]) -> bool {
        if (wave == 0) {
            const int64_t row = blk * 64 + lane;
            const uint64_t key = key_n;
            const bool valid = row < N && (key >> 32) != 0xFFFFFFFFull;
            const uint64_t diag = valid ? diag_n : 0ull;
            if (blk + 1 < cb) {
                const int64_t rn = row + 64;
                key_n = rn < N ? keys[rn] : ~0ull;
                diag_n = rn < N ? mask[rn * cb + blk + 1] : 0ull;
            }
            const uint64_t vmask = __ballot(valid);
            uint64_t rem = removed[blk];
            uint64_t kept = 0;
            const int nk0 = nkeep_sh;
            int nk = nk0;
            const uint32_t dlo = (uint32_t)diag, dhi = (uint32_t)(diag >> 32);
            for (int r = 0; r < 64; ++r) {
                if (!((vmask >> r) & 1ull)) break;
                if (nk >= max_out) break;
                if (!((rem >> r) & 1ull)) {
                    kept |= (1ull << r);
                    ++nk;
                    const uint64_t d = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(dlo, r) |
                                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(dhi, r) << 32);
                    rem |= d;
                }
            }
            if ((kept >> lane) & 1ull) {
                const int j = __popcll(kept & ((1ull << lane) - 1ull));
                keep[nk0 + j] = (int32_t)(uint32_t)key;
            }
            if (lane == 0) {
                kept_sh = kept;
                nkeep_sh = nk;
                if (nk >= max_out || vmask != ~0ull) stop_sh = 1;
            }
        }
        lds_barrier();              // orders LDS only (kept_sh / stop_sh); the prefetched rows stay in flight
        if (stop_sh) return false;
        const uint64_t kept = kept_sh;
        uint64_t acc = 0;
#pragma unroll
        for (int k = 0; k < NR_RPG; ++k) {
            const int r = g + G * k;
            if (r < 64 && ((kept >> r) & 1ull)) acc |= cur[k];
        }
        if (own && acc) atomicOr((unsigned long long*)&removed[w], (unsigned long long)acc);
        lds_barrier();              // orders LDS only (removed[])
        return true;
    };
    for (int64_t blk = 0; blk < cb; blk += 2) {
        if (blk + 1 < cb) nr_load(mask, N, cb, blk + 1, g, G, w, own, vb);
        if (!block(blk, va)) break;
        if (blk + 1 >= cb) break;
        if (blk + 2 < cb) nr_load(mask, N, cb, blk + 2, g, G, w, own, va);
        if (!block(blk + 1, vb)) break;
    }
    if (tid == 0) *num_keep = nkeep_sh;
}

// ---- ProposalLayer ----------------------------------------------------------
// gidx (optional): the anchor's index in the whole volume's anchor list when
// this rank holds a depth slab of it (the key then sorts in global order).
__global__ void score_keys_kernel(const float* __restrict__ probs, int64_t A,
                                  const int64_t* __restrict__ gidx, int64_t* __restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A) return;
    float s = probs[i * 2 + 1];
    if (s == 0.0f) s = 0.0f;
    const uint32_t o = float_ord(s) ^ 0x80000000u;   // signed-orderable
    const uint32_t idx = (uint32_t)(gidx ? gidx[i] : i);
    const uint64_t k = ((uint64_t)o << 32) | (uint64_t)(0xFFFFFFFFu - idx);
    keys[i] = (int64_t)k;
}

struct Std6 { float v[6]; };

// exp of a float32 through float64: (float)exp((double)x).  The oracle
// (oracle/ops_ref.py) computes the same expression with numpy's float64 exp, so
// the decoded boxes -- and the NMS keep set on them -- agree bit for bit (the
// two double exps differ at most in the last double bit, which changes the
// float rounding only within 2^-29 of a float tie).
__device__ __forceinline__ float exp_via_f64(float x) { return (float)exp((double)x); }

// core/models.py:391-447 with apply_box_deltas_graph (280-337).  order[j] must
// be < A (the anchor rows): an index outside [0, A) is never read; its row is
// written as a zero box with score -FLT_MAX (NMS never selects it) and *err is
// set to 1 for the caller's next synchronisation point.
__global__ void proposal_decode_kernel(const float* __restrict__ probs,
                                       const float* __restrict__ deltas,
                                       const float* __restrict__ anchors, int64_t A,
                                       const int64_t* __restrict__ order, int64_t k, Std6 sd,
                                       float image_depth, float* __restrict__ boxes,
                                       float* __restrict__ scores, int32_t* __restrict__ err) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    const int64_t a = order[j];
    if (a < 0 || a >= A) {
        scores[j] = -3.402823466e38f;
#pragma unroll
        for (int q = 0; q < 6; ++q) boxes[j * 6 + q] = 0.0f;
        if (err) *err = 1;
        return;
    }
    scores[j] = probs[a * 2 + 1];
    float d[6], an[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        float v = deltas[a * 6 + q] * sd.v[q];
        v = smax(smin(v, 3.0f), -3.0f);     // ProposalLayer clip
        d[q] = smax(smin(v, 3.0f), -3.0f);  // apply_box_deltas_graph clip
        an[q] = anchors[a * 6 + q];
    }
    float height = an[3] - an[0], width = an[4] - an[1], depth = an[5] - an[2];
    float cy = an[0] + 0.5f * height, cx = an[1] + 0.5f * width, cz = an[2] + 0.5f * depth;
    cy = cy + d[0] * height;
    cx = cx + d[1] * width;
    cz = cz + d[2] * depth;
    height = height * exp_via_f64(d[3]);
    width = width * exp_via_f64(d[4]);
    depth = depth * exp_via_f64(d[5]);
    const float y1 = cy - 0.5f * height, x1 = cx - 0.5f * width, z1 = cz - 0.5f * depth;
    float r[6] = {y1, x1, z1, y1 + height, x1 + width, z1 + depth};
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        r[q] = smax(smin(r[q], 1.0f), 0.0f);   // clip_by_value(result, 0, 1)
        r[q] = smax(smin(r[q], 1.0f), 0.0f);   // clip_boxes_graph(window [0,0,0,1,1,1])
    }
    const float eps = 1e-6f;
    const float img_depth = smax(image_depth, 1.0f);
    const float min_d = smax(1.0f / img_depth, 1e-4f);
    r[3] = smax(r[3], r[0] + eps);
    r[4] = smax(r[4], r[1] + eps);
    r[5] = smax(r[5], r[2] + min_d);
#pragma unroll
    for (int q = 0; q < 6; ++q) boxes[j * 6 + q] = r[q];
}

__global__ void proposal_gather_kernel(const float* __restrict__ boxes,
                                       const int32_t* __restrict__ keep,
                                       const int32_t* __restrict__ num_keep, int P,
                                       float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int nk = *num_keep;
    for (int q = 0; q < 6; ++q) out[(int64_t)i * 6 + q] = i < nk ? boxes[(int64_t)keep[i] * 6 + q] : 0.0f;
}

static int64_t pow2_at_least(int64_t n) {
    int64_t p = 1;
    while (p < n) p <<= 1;
    return p;
}

struct NmsWs {
    uint64_t* keys;      // unsorted keys, then the sort's output goes to skeys
    uint64_t* skeys;
    uint32_t* rank;
    float* sboxes;
    uint64_t* mask;
    size_t bytes;
};

static NmsWs nms_ws_layout(int64_t N, void* base) {
    NmsWs w{};
    const int64_t npad = pow2_at_least(N < 2 ? 2 : N);
    const int64_t cb = (N + 63) / 64;
    char* p = (char*)base;
    size_t off = 0;
    // sizing pass (base == nullptr): offsets only, no arithmetic on a null pointer
    auto take = [&](size_t b) {
        size_t o = off;
        off += (b + 255) & ~(size_t)255;
        return p ? p + o : nullptr;
    };
    w.keys = (uint64_t*)take(sizeof(uint64_t) * npad);
    w.skeys = (uint64_t*)take(sizeof(uint64_t) * npad);
    w.rank = (uint32_t*)take(rank_sort_scratch_bytes(N > 0 ? N : 1));
    w.sboxes = (float*)take(sizeof(float) * 6 * (N > 0 ? N : 1));
    w.mask = (uint64_t*)take(sizeof(uint64_t) * (size_t)(N > 0 ? N : 1) * (cb > 0 ? cb : 1));
    w.bytes = off;
    return w;
}

}  // namespace m3d

using namespace m3d;

extern "C" size_t m3d_nms3d_workspace_bytes(int64_t N) { return nms_ws_layout(N, nullptr).bytes; }

extern "C" int m3d_nms3d(const float* boxes, const float* scores, int64_t N, int32_t max_out,
                         float iou_thr, int32_t mode, int32_t* keep, int32_t* num_keep,
                         void* workspace, size_t ws_bytes, m3d_stream_t s) {
    if (!(iou_thr >= 0.0f && iou_thr <= 1.0f)) return einval("iou_threshold must be in [0, 1]");
    if (mode != 0 && mode != 1) return einval("mode must be 0 (3-D) or 1 (2-D)");
    if (N < 0) return einval("boxes must be 2-D");
    if (N > (int64_t)0x7FFFFFFF) return einval("too many boxes");
    const int64_t cb = (N + 63) / 64;
    if (cb > 16384) return einval("too many boxes for the LDS-resident reduction (max 1048576)");
    const bool work = N > 0 && max_out > 0;
    if (work && ws_bytes < nms_ws_layout(N, nullptr).bytes) return einval("workspace too small");
    if (hipMemsetAsync(num_keep, 0, sizeof(int32_t), st(s)) != hipSuccess)
        return check_launch("memset num_keep");
    if (!work) return M3D_OK;
    NmsWs w = nms_ws_layout(N, workspace);
    const int64_t npad = pow2_at_least(N < 2 ? 2 : N);
    hipLaunchKernelGGL(nms_keys_kernel, dim3(grid_for(npad, 256)), dim3(256), 0, st(s), scores, N,
                       npad, w.keys);
    int rc = check_launch("nms_keys_kernel");
    if (rc) return rc;
    rc = rank_sort_u64(w.keys, nullptr, N, false, false, w.rank, w.skeys, nullptr, st(s));
    if (rc) return rc;
    hipLaunchKernelGGL(nms_gather_kernel, dim3(grid_for(N, 256)), dim3(256), 0, st(s), boxes,
                       w.skeys, N, mode == 1 ? 4 : 6, w.sboxes);
    rc = check_launch("nms_gather_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(nms_mask_kernel, dim3((unsigned)cb, (unsigned)cb), dim3(64), 0, st(s),
                       w.sboxes, N, cb, iou_thr, mode, w.mask);
    rc = check_launch("nms_mask_kernel");
    if (rc) return rc;
    // up to 16384 boxes: the prefetching form (1.10 -> 0.84 ms at 15000 -> 6000)
    if (cb <= 256) {
        hipLaunchKernelGGL(nms_reduce_pf_kernel, dim3(1), dim3(1024), 0, st(s), w.mask, w.skeys, N, cb, max_out,
                           keep, num_keep);
        return check_launch("nms_reduce_pf_kernel");
    }
    hipLaunchKernelGGL(nms_reduce_kernel, dim3(1), dim3(1024), sizeof(uint64_t) * cb, st(s),
                       w.mask, w.skeys, N, cb, max_out, keep, num_keep);
    return check_launch("nms_reduce_kernel");
}

extern "C" int m3d_score_keys(const float* probs, int64_t A, int64_t* keys, m3d_stream_t s) {
    return m3d_score_keys_mapped(probs, A, nullptr, keys, s);
}

extern "C" int m3d_score_keys_mapped(const float* probs, int64_t A, const int64_t* gidx,
                                     int64_t* keys, m3d_stream_t s) {
    if (A < 0) return einval("score_keys: negative anchor count");
    if (A == 0) return M3D_OK;
    if (A > 0xFFFFFFFFll) return einval("score_keys: more than 2^32 anchors");
    hipLaunchKernelGGL(score_keys_kernel, dim3(grid_for(A, 256)), dim3(256), 0, st(s), probs, A,
                       gidx, keys);
    return check_launch("score_keys_kernel");
}

extern "C" int m3d_proposal_decode(const float* probs, const float* deltas, const float* anchors,
                                   int64_t n_anchors, const int64_t* order, int64_t k,
                                   const float std_dev[6], float image_depth, float* boxes,
                                   float* scores, int32_t* err, m3d_stream_t s) {
    if (k < 0) return einval("proposal_decode: negative proposal count");
    if (n_anchors < 0) return einval("proposal_decode: negative anchor count");
    if (k > n_anchors) return einval("proposal_decode: more proposals than anchors");
    if (k == 0) return M3D_OK;
    if (!probs || !deltas || !anchors || !order || !boxes || !scores || !std_dev)
        return einval("proposal_decode: null pointer");
    Std6 sd{};
    for (int q = 0; q < 6; ++q) sd.v[q] = std_dev[q];
    hipLaunchKernelGGL(proposal_decode_kernel, dim3(grid_for(k, 256)), dim3(256), 0, st(s), probs,
                       deltas, anchors, n_anchors, order, k, sd, image_depth, boxes, scores, err);
    return check_launch("proposal_decode_kernel");
}

extern "C" int m3d_proposal_gather(const float* boxes, const int32_t* keep,
                                   const int32_t* num_keep, int32_t P, float* proposals,
                                   m3d_stream_t s) {
    if (P < 0) return einval("proposal_gather: negative proposal count");
    if (P == 0) return M3D_OK;
    hipLaunchKernelGGL(proposal_gather_kernel, dim3(grid_for(P, 256)), dim3(256), 0, st(s), boxes,
                       keep, num_keep, P, proposals);
    return check_launch("proposal_gather_kernel");
}

// On-device batched NMS (utils/util.py:123-169 + torchvision.ops.nms contract).
//
// Reference algorithm, per image (util.py:136-169):
//   pairs (anchor a, class c) with score y[4+c][a] > conf, row-major order
//   (util.py:147, nonzero over (anchor, class)); boxes = wh2xy(cx,cy,w,h)
//   (util.py:76-82,145); sort by score descending, keep the first max_nms
//   (util.py:157); offset boxes by class*max_wh (util.py:160-161); greedy NMS
//   with IoU = inter / (area_i + area_j - inter) > iou (torchvision, util.py:162);
//   first max_det kept (util.py:163).
// Deterministic restatement: ties in score are broken by the lower pair index
// a*nc + c (the reference's argsort is unstable, so any tie order is valid
// there); no wall-clock cutoff (util.py:166-167 is dropped).
//
// Design (gfx950):
//   nms_emit   grid (A/256, B), 8 class groups per block: the census of the pairs
//              above conf: the image's count and its 2048-bin score histogram.
//   nms_gather 8 workgroups per image: the first batch = the top whole score bins
//              (>= FIRST_TARGET pairs, <= 4096), each pair as a 56-bit key (score bits
//              << 26 | (2^26-1 - pair); larger key = earlier in the reference order),
//              made from the scores (for_pairs).
//   nms_prep   one 1024-thread workgroup per image: the first batch bitonic-sorted in
//              LDS, each entry decoded once into the workspace.
//   nms_mask   the first batches' lower-triangular IoU bitmasks, one wave per 64 x 64
//              tile, the tiles of all images strided over one grid.
//   nms_finish one workgroup per image: one wave resolves the greedy order from the
//              mask, 64 entries per step; the kept entries are written in parallel.
//              Later batches (an image whose first batch keeps < max_det with
//              candidates left, or a bin > 4096 keys: radix select with 4 x 14-bit
//              digit histograms) run greedy NMS on 256-key sub-batches in the same
//              workgroup: parallel test against the kept set, a 256x256 IoU bitmask
//              and parallel resolve rounds. Stops at max_det kept or max_nms processed.
#include "common.h"
#include "dtypes.h"

#pragma clang fp contract(off)

// phase stamps of the diagnostic build (make EXTRA=-DYH_ABLATION, tools/nms_trace.py);
// compiled out of the shipped library
#ifdef YH_ABLATION
#define NMS_TRACE (p.trace)
#define NMS_DBG(bit) (p.dbg & (bit))
#else
#define NMS_TRACE ((unsigned long long*)nullptr)
#define NMS_DBG(bit) 0
#endif

namespace yh {

namespace {

constexpr int NMS_T = 1024;
constexpr int CAP = 4096;      // keys sorted per batch
constexpr int SB = 256;        // sub-batch for the greedy pass
constexpr int DBITS = 14;
constexpr int HBINS = 1 << DBITS;
constexpr int PBITS = 26;
constexpr unsigned PMASK = (1u << PBITS) - 1;
constexpr int MAXDET = 1024;

__device__ __forceinline__ unsigned long long make_key(float s, unsigned pair) {
    const unsigned bits = __float_as_uint(s) & 0x3FFFFFFFu;
    return ((unsigned long long)bits << PBITS) | (unsigned long long)(PMASK - pair);
}

constexpr int NBINS = 2048;  // coarse score bins = top 16 bits of the fp32 score, offset by the threshold's
// Keys the first batch takes at least (whole score bins, <= CAP): the greedy of a typical image
// reaches max_det = 300 kept within its first 400-620 keys (v11_n bf16 synthetic scenes); with
// 640 an image continued into the single-workgroup sub-batch path in about every second batch of
// 32 (nms_finish 10 -> 70 us). 960 still sorts as one 1024-key register bitonic (nms_prep).
constexpr int FIRST_TARGET = 960;

__device__ __forceinline__ int score_bin(float s, int base) {
    const int b = (int)(__float_as_uint(s) >> 16) - base;
    return b < 0 ? 0 : (b >= NBINS ? NBINS - 1 : b);
}

// Candidate census: a block covers 256 anchors (32 chunks of 8 consecutive anchors,
// one 16-B load per class row) x 8 class groups; thread (chunk, group) loads the group's
// class rows, counts the passing (anchor, class) pairs (util.py:147, score > conf) and adds
// each to the block's LDS score-bin histogram; one atomic per block for the image's count,
// one merge of the histogram. No keys are written: nms_gather makes the first batch's keys
// from the scores again (its bins are known by then), and the rare later batches
// (nms_rest) enumerate the pairs from the scores the same way (for_pairs). Writing every
// candidate's 8-byte key here (up to 30 k per image) cost more than reading the scores twice.
constexpr int EMIT_APT = 8;            // anchors per thread (one 16-B chunk)
constexpr int EMIT_CHUNKS = 32;        // anchor chunks per block
constexpr int EMIT_GROUPS = 8;         // class groups per block

template <typename T>
__device__ __forceinline__ void load_scores(const T* src, bool full, int n_ok, float (&v)[EMIT_APT]) {
    if (full) {
        chunk_to_f(ld_chunk(src), v);
    } else {
#pragma unroll
        for (int e = 0; e < EMIT_APT; ++e) v[e] = e < n_ok ? tof(src[e]) : -1.0f;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void nms_emit(const NmsArgs p) {
    __shared__ unsigned lhist[NBINS];
    __shared__ int wtot[4];
    for (int i = threadIdx.x; i < NBINS; i += 256) lhist[i] = 0;
    __syncthreads();   // at entry: no load is in flight yet
    const int n = blockIdx.y;
    const int chunk = threadIdx.x & (EMIT_CHUNKS - 1), grp = threadIdx.x / EMIT_CHUNKS;
    const int a0 = (blockIdx.x * EMIT_CHUNKS + chunk) * EMIT_APT;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int cpg = (p.nc + EMIT_GROUPS - 1) / EMIT_GROUPS;
    const int c_lo = grp * cpg, c_hi = min(p.nc, c_lo + cpg);
    const T* y = reinterpret_cast<const T*>(p.y) + (long long)n * (4 + p.nc) * p.A;
    const bool full = a0 + EMIT_APT <= p.A && (p.A % EMIT_APT) == 0;
    int cnt = 0;
    if (a0 < p.A) {
        constexpr int U = 5;   // rows in flight per thread (55 VGPRs: 8 waves per SIMD)
        for (int c0 = c_lo; c0 < c_hi; c0 += U) {
            float v[U][EMIT_APT];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (c0 + u < c_hi) load_scores(y + (long long)(4 + c0 + u) * p.A + a0, full, p.A - a0, v[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (c0 + u >= c_hi) continue;
#pragma unroll
                for (int e = 0; e < EMIT_APT; ++e)
                    if (v[u][e] > p.conf) {
                        ++cnt;
                        atomicAdd(&lhist[score_bin(v[u][e], p.bin_base)], 1u);
                    }
            }
        }
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) cnt += __shfl_xor(cnt, d);
    if (lane == 0) wtot[wave] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int t = wtot[0] + wtot[1] + wtot[2] + wtot[3];
        if (t) atomicAdd(&p.counts[n], t);
    }
    unsigned* gh = p.hist + (long long)n * NBINS;
    for (int i = threadIdx.x; i < NBINS; i += 256)
        if (lhist[i]) atomicAdd(&gh[i], lhist[i]);
}

// Every candidate pair of image n (score > conf) in units [u0, u1) of one class row's 8
// consecutive anchors (unit u = class * nq + chunk, nq = ceil(A / 8)), units strided by
// `step` from `first`: fn(key, score) for each, in no particular order. The keys are
// make_key's, bit for bit the ones nms_emit used to write.
template <typename T, int U = 4, typename F>   // U: units in flight per thread
__device__ __forceinline__ void for_pairs(const NmsArgs& p, const T* y, int u0, int u1, int first, int step, F fn) {
    const int nq = (p.A + EMIT_APT - 1) / EMIT_APT;
    const bool aligned = (p.A % EMIT_APT) == 0;
    for (int ub = u0 + first; ub < u1; ub += U * step) {
        float v[U][EMIT_APT];
        int a0[U], c[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int u = ub + k * step;
            c[k] = u / nq;
            a0[k] = (u - c[k] * nq) * EMIT_APT;
            if (u < u1) load_scores(y + (long long)(4 + c[k]) * p.A + a0[k], aligned, p.A - a0[k], v[k]);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (ub + k * step >= u1) continue;
#pragma unroll
            for (int e = 0; e < EMIT_APT; ++e)
                if (v[k][e] > p.conf) fn(make_key(v[k][e], (unsigned)((a0[k] + e) * p.nc + c[k])));
        }
    }
}

// Zeroes the per-image candidate counts, score histograms and gather counters (one
// launch instead of three memsets).
__global__ __launch_bounds__(256) void nms_zero(int* counts, unsigned* hist, unsigned long long* state, int B) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < B * NBINS) hist[i] = 0u;
    if (i < B) {
        counts[i] = 0;
        state[(long long)i * 8 + 4] = 0ull;   // gather counter (STW = 8)
    }
}

// IoU test "RN(inter / union) > thr" (fp32 division, torchvision contract) without
// the division. For thr >= 0 a pair without positive intersection never passes
// (0 / union is +-0 or NaN). Otherwise, with union > 0 finite, RN(q) > t <=>
// RN(q) >= t+ (next float) <=> q > m or (q == m and the tie rounds up to t+),
// m = (t + t+) / 2. inter, union are floats and m has <= 25 significant bits,
// so m * union is exact in double and the comparison is exact. Degenerate unions
// (<= 0, inf, NaN) take the division.
struct IouThr {
    float t;
    double m;
    bool tie_up, nonneg;
};

__device__ __forceinline__ IouThr make_thr(float t) {
    IouThr r;
    r.t = t;
    r.nonneg = t >= 0.0f && t < 3.0e38f;
    const float tp = __uint_as_float(__float_as_uint(t) + 1u);   // next float above t (t >= 0)
    r.m = ((double)t + (double)tp) * 0.5;
    r.tie_up = (__float_as_uint(t) & 1u) != 0;                   // t odd -> tie goes to even t+
    return r;
}

__device__ __forceinline__ bool iou_above(float ax1, float ay1, float ax2, float ay2, float aa,
                                          float bx1, float by1, float bx2, float by2, float ba, const IouThr& th) {
    const float xx1 = fmaxf(ax1, bx1), yy1 = fmaxf(ay1, by1);
    const float xx2 = fminf(ax2, bx2), yy2 = fminf(ay2, by2);
    const float w = fmaxf(0.0f, xx2 - xx1), h = fmaxf(0.0f, yy2 - yy1);
    const float inter = w * h;
    const float uni = aa + ba - inter;
    if (th.nonneg) {
        if (!(inter > 0.0f)) return false;
        if (uni > 0.0f && uni < 3.0e38f && inter < 3.0e38f) {
            const double lhs = (double)inter, rhs = th.m * (double)uni;
            return lhs > rhs || (lhs == rhs && th.tie_up);
        }
    }
    const float ovr = inter / uni;
    return ovr > th.t;
}

struct NmsSmem {
    unsigned hist[HBINS + 1];
    unsigned long long bkeys[CAP];
    float sb[SB][4];        // class-offset boxes of the sub-batch
    float sarea[SB];
    float sraw[SB][4];      // plain boxes (output)
    float sscore[SB];
    float scls[SB];
    unsigned long long smask[SB][4];
    unsigned supp[SB / 32];
    unsigned long long und[4], kep[4];   // parallel-resolve state (bit i = sub-batch entry i)
    int nslow;
    float kb[MAXDET][4];
    float karea[MAXDET];
    float kcls[MAXDET];
    // plain-coordinate extent of every entry processed so far (finite: no inf / NaN): with
    // rhi - rlo <= max_wh / 2 boxes of different classes cannot intersect (class offsets)
    float rlo, rhi;
    int rfin;
    float wlo[NMS_T / 64], whi[NMS_T / 64];
    int wfin[NMS_T / 64];
    unsigned wsum[NMS_T / 64];
    unsigned long long sel_prefix;
    int sel_need, sel_bin, gcount, kept;
};

template <typename T>
__device__ __forceinline__ float round_t(float v) { return tof(fromf<T>(v)); }

// A sorted key's entry: the box by wh2xy (util.py:76-82) in the input dtype, the same box
// offset by class * max_wh (util.py:160-161) and its area, the score and the class.
template <typename T>
__device__ __forceinline__ void decode_key(const NmsArgs& p, const T* y, unsigned long long key, float (&ob)[4],
                                           float (&raw)[4], float& area, float& score, float& cls) {
    const unsigned pair = PMASK - (unsigned)(key & PMASK);
    const int a = (int)(pair / (unsigned)p.nc), c = (int)(pair - (unsigned)a * p.nc);
    const float cx = tof(y[a]), cy = tof(y[(long long)p.A + a]);
    const float w = tof(y[2LL * p.A + a]), h = tof(y[3LL * p.A + a]);
    raw[0] = round_t<T>(cx - w / 2.0f); raw[1] = round_t<T>(cy - h / 2.0f);
    raw[2] = round_t<T>(cx + w / 2.0f); raw[3] = round_t<T>(cy + h / 2.0f);
    const float off = (float)c * p.max_wh;
    ob[0] = raw[0] + off; ob[1] = raw[1] + off; ob[2] = raw[2] + off; ob[3] = raw[3] + off;
    area = (ob[2] - ob[0]) * (ob[3] - ob[1]);
    score = tof(y[(long long)(4 + c) * p.A + a]);
    cls = (float)c;
}


// Bitonic sort (descending) of bkeys[0, count), count <= CAP, padded with zero
// keys to a power of two P. The keys live in registers: wave w owns indices
// [w*64E, (w+1)*64E), element e of lane l being index w*64E + e*64 + l
// (E = P / NMS_T, at least 1). Compare-exchange partners i ^ j are then
// reached by a lane shuffle (j < 64), inside the thread (j < 64E), or through
// LDS with a workgroup barrier (larger j: 10 of the 66 stages at P = 2048).
__device__ __forceinline__ unsigned long long shfl_xor64(unsigned long long v, int m) {
    const unsigned lo = __shfl_xor((unsigned)v, m), hi = __shfl_xor((unsigned)(v >> 32), m);
    return ((unsigned long long)hi << 32) | lo;
}

template <int E>
__device__ void sort_regs(NmsSmem& S, int count, int P, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
    const int base = wave * 64 * E;
    const bool active = base < P;
    unsigned long long v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = base + e * 64 + lane;
        v[e] = active && i < count ? S.bkeys[i] : 0ull;   // pad with the smallest key
    }
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j < 64) {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const unsigned long long o = shfl_xor64(v[e], j);
                    const int i = base + e * 64 + lane;
                    const bool lower = (lane & j) == 0, desc = (i & k) == 0;
                    const bool take_max = lower == desc;
                    v[e] = take_max ? (v[e] > o ? v[e] : o) : (v[e] < o ? v[e] : o);
                }
            } else if (j < 64 * E) {
                const int jj = j >> 6;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    if (e & jj) continue;
                    const int i = base + e * 64 + lane;
                    const bool desc = (i & k) == 0;
                    const unsigned long long a = v[e], b = v[e | jj];
                    const bool sw = desc ? (a < b) : (a > b);
                    v[e] = sw ? b : a;
                    v[e | jj] = sw ? a : b;
                }
            } else {
                __syncthreads();   // previous LDS readers are done
                if (active)
#pragma unroll
                    for (int e = 0; e < E; ++e) S.bkeys[base + e * 64 + lane] = v[e];
                __syncthreads();
                if (active) {
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const int i = base + e * 64 + lane;
                        const unsigned long long o = S.bkeys[i ^ j];
                        const bool lower = (i & j) == 0, desc = (i & k) == 0;
                        const bool take_max = lower == desc;
                        v[e] = take_max ? (v[e] > o ? v[e] : o) : (v[e] < o ? v[e] : o);
                    }
                }
            }
        }
    }
    __syncthreads();
    if (active)
#pragma unroll
        for (int e = 0; e < E; ++e) S.bkeys[base + e * 64 + lane] = v[e];
    __syncthreads();
}

__device__ void sort_batch(NmsSmem& S, int count, int tid) {
    int P = 64;
    while (P < count) P <<= 1;
    if (P <= NMS_T) sort_regs<1>(S, count, P, tid);
    else if (P <= 2 * NMS_T) sort_regs<2>(S, count, P, tid);
    else sort_regs<4>(S, count, P, tid);
}

// Greedy NMS over the first `want` keys of the sorted batch (sub-batches of SB).
// Pair test without branches for the common case; degenerate unions (<= 0, inf,
// NaN) are flagged and resolved by the division in a rare second pass.
__device__ __forceinline__ bool iou_fast(float ax1, float ay1, float ax2, float ay2, float aa,
                                         float bx1, float by1, float bx2, float by2, float ba,
                                         const IouThr& th, bool& slow) {
    const float xx1 = fmaxf(ax1, bx1), yy1 = fmaxf(ay1, by1);
    const float xx2 = fminf(ax2, bx2), yy2 = fminf(ay2, by2);
    const float w = fmaxf(0.0f, xx2 - xx1), h = fmaxf(0.0f, yy2 - yy1);
    const float inter = w * h;
    // most pairs do not intersect (every class is offset by c * max_wh): they skip the fp64
    // test (wave-uniform when no lane of the wave intersects)
    if (!(inter > 0.0f)) return false;
    const float uni = aa + ba - inter;
    const double lhs = (double)inter, rhs = th.m * (double)uni;
    const bool good = (uni > 0.0f) & (uni < 3.0e38f) & (inter < 3.0e38f);
    slow |= !good;
    return good & ((lhs > rhs) | ((lhs == rhs) & th.tie_up));
}

// Greedy NMS over the first `want` keys of the sorted batch, in sub-batches of SB
// entries (torchvision nms semantics, util.py:162-163):
//   1. decode the sub-batch's boxes (wh2xy in the input dtype, class offset);
//   2. flag entries suppressed by an already-kept box (4 threads per entry);
//   3. lower-triangular IoU bitmask: bit j of row i <=> j < i and IoU(i, j) > thr;
//   4. resolve the greedy order in parallel rounds: an undecided entry with a kept
//      suppressor is removed, one whose suppressors are all decided (and none
//      kept) is kept. The first undecided entry always resolves, so this ends;
//      it equals the sequential greedy, and truncating to the first
//      max_det - kept keeps equals stopping the greedy there.
template <typename T>
__device__ void nms_batch(NmsSmem& S, const NmsArgs& p, const T* y, float* dets, int want, int tid, int lane, int wave) {
        const int n = blockIdx.x;
        int sbi = 0;
        const IouThr th = make_thr(p.iou);
        // diagnostic builds: ticks of each part summed over all sub-batches (slots 12 decode, 13 kept
        // test + pairwise mask, 14 resolve, 15 outputs; 15's bits 40+ count the sub-batches)
        unsigned long long tprev = 0;
#define SB_MARK(k)                                                                               \
    do {                                                                                         \
        if (NMS_TRACE && tid == 0) {                                                             \
            const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                      \
            if ((k) >= 12) NMS_TRACE[n * 16 + (k)] += t_ - tprev + ((k) == 15 ? (1ull << 40) : 0ull); \
            tprev = t_;                                                                          \
        }                                                                                        \
    } while (0)
        for (int s0 = 0; s0 < want && S.kept < p.max_det; s0 += SB) {
            SB_MARK(0);
            const int ns = min(SB, want - s0);
            float lo = INFINITY, hi = -INFINITY;
            bool fin = true;
            if (tid < ns) {
                float ob[4], raw[4], area, score, cls;
                decode_key<T>(p, y, S.bkeys[s0 + tid], ob, raw, area, score, cls);
                S.sb[tid][0] = ob[0]; S.sb[tid][1] = ob[1]; S.sb[tid][2] = ob[2]; S.sb[tid][3] = ob[3];
                S.sarea[tid] = area;
                S.sraw[tid][0] = raw[0]; S.sraw[tid][1] = raw[1]; S.sraw[tid][2] = raw[2]; S.sraw[tid][3] = raw[3];
                S.sscore[tid] = score;
                S.scls[tid] = cls;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    fin &= fabsf(raw[k]) < 3.0e38f;
                    lo = fminf(lo, raw[k]);
                    hi = fmaxf(hi, raw[k]);
                }
            }
#pragma unroll
            for (int d = 32; d > 0; d >>= 1) {
                lo = fminf(lo, __shfl_xor(lo, d));
                hi = fmaxf(hi, __shfl_xor(hi, d));
            }
            fin = __ballot(!fin) == 0ull;
            if (lane == 0) { S.wlo[wave] = lo; S.whi[wave] = hi; S.wfin[wave] = fin; }
            if (tid < SB / 32) S.supp[tid] = 0;
            if (tid == 0) S.nslow = 0;
            __syncthreads();
            SB_MARK(12);
            const int kept0 = S.kept;
            lo = S.rlo; hi = S.rhi; fin = S.rfin != 0;
#pragma unroll
            for (int w = 0; w < NMS_T / 64; ++w) {
                lo = fminf(lo, S.wlo[w]);
                hi = fmaxf(hi, S.whi[w]);
                fin &= S.wfin[w] != 0;
            }
            // classes separable over the kept set and this sub-batch: test same-class pairs only.
            // Only for thresholds >= 0: with thr < 0 a disjoint pair (IoU 0) still suppresses.
            const bool sep = th.nonneg && fin && p.max_wh > 0.0f && p.max_wh < 3.0e38f && hi - lo <= 0.5f * p.max_wh;
            bool slow = !th.nonneg;
            {   // 2. suppressed by an already-kept box? 4 threads per entry, 4 kept boxes per step
                const int e = tid >> 2, part = tid & 3;
                if (e < ns) {
                    const float ex1 = S.sb[e][0], ey1 = S.sb[e][1], ex2 = S.sb[e][2], ey2 = S.sb[e][3], ea = S.sarea[e];
                    const float ec = S.scls[e];
                    bool sup = false;
                    for (int k0 = 0; k0 < kept0 && !sup; k0 += 16) {
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int k = k0 + 4 * u + part;
                            if (k < kept0 && (!sep || S.kcls[k] == ec))
                                sup |= iou_fast(S.kb[k][0], S.kb[k][1], S.kb[k][2], S.kb[k][3], S.karea[k],
                                                ex1, ey1, ex2, ey2, ea, th, slow);
                        }
                    }
                    if (sup) atomicOr(&S.supp[e >> 5], 1u << (e & 31));
                }
            }
            {   // 3. lower-triangular pairwise mask, 64 columns per thread
                const int i = tid >> 2, wd = tid & 3;
                unsigned long long m = 0;
                if (i < ns && wd * 64 < i) {
                    const float ix1 = S.sb[i][0], iy1 = S.sb[i][1], ix2 = S.sb[i][2], iy2 = S.sb[i][3], ia = S.sarea[i];
                    const float ic = S.scls[i];
#pragma unroll 8
                    for (int jj = 0; jj < 64; ++jj) {
                        const int j = wd * 64 + jj;
                        if (sep && S.scls[j] != ic) continue;
                        const bool hit = iou_fast(ix1, iy1, ix2, iy2, ia, S.sb[j][0], S.sb[j][1], S.sb[j][2], S.sb[j][3],
                                                  S.sarea[j], th, slow);
                        m |= (unsigned long long)hit << jj;
                    }
                    const int lim = i - wd * 64;   // columns j < i only
                    if (lim < 64) m &= (1ull << lim) - 1ull;
                }
                S.smask[i][wd] = m;
            }
            if (slow) atomicAdd(&S.nslow, 1);
            __syncthreads();
            if (S.nslow) {
                // rare: degenerate unions somewhere in this sub-batch -> exact division path
                const int e = tid >> 2, part = tid & 3;
                if (e < ns) {
                    bool sup = false;
                    for (int k = part; k < kept0 && !sup; k += 4)
                        sup = iou_above(S.kb[k][0], S.kb[k][1], S.kb[k][2], S.kb[k][3], S.karea[k],
                                        S.sb[e][0], S.sb[e][1], S.sb[e][2], S.sb[e][3], S.sarea[e], th);
                    if (sup) atomicOr(&S.supp[e >> 5], 1u << (e & 31));
                }
                const int i = e, wd = part;
                unsigned long long m = 0;
                if (i < ns) {
                    for (int jj = 0; jj < 64; ++jj) {
                        const int j = wd * 64 + jj;
                        if (j < i && iou_above(S.sb[i][0], S.sb[i][1], S.sb[i][2], S.sb[i][3], S.sarea[i],
                                               S.sb[j][0], S.sb[j][1], S.sb[j][2], S.sb[j][3], S.sarea[j], th))
                            m |= 1ull << jj;
                    }
                }
                S.smask[i][wd] = m;
                __syncthreads();
            }
            SB_MARK(13);
            // 4. parallel rounds (waves 0..3, one entry per thread)
            unsigned long long low[4] = {0ull, 0ull, 0ull, 0ull};
            bool undec = false, iskept = false;
            if (tid < SB) {
#pragma unroll
                for (int w = 0; w < 4; ++w) low[w] = S.smask[tid][w];
                undec = tid < ns && !((S.supp[tid >> 5] >> (tid & 31)) & 1u);
                const unsigned long long bu = __ballot(undec);
                if (lane == 0) { S.und[wave] = bu; S.kep[wave] = 0ull; }
            }
            __syncthreads();
            for (;;) {
                unsigned long long U[4], K[4];
#pragma unroll
                for (int w = 0; w < 4; ++w) { U[w] = S.und[w]; K[w] = S.kep[w]; }
                if ((U[0] | U[1] | U[2] | U[3]) == 0ull) break;
                bool nk = false, nr = false;
                if (undec) {
                    const unsigned long long hk = (low[0] & K[0]) | (low[1] & K[1]) | (low[2] & K[2]) | (low[3] & K[3]);
                    const unsigned long long hu = (low[0] & U[0]) | (low[1] & U[1]) | (low[2] & U[2]) | (low[3] & U[3]);
                    nr = hk != 0ull;
                    nk = !nr && hu == 0ull;
                }
                __syncthreads();   // all reads of U, K done
                if (tid < SB) {
                    undec = undec && !nk && !nr;
                    iskept = iskept || nk;
                    const unsigned long long bu = __ballot(undec), bk = __ballot(iskept);
                    if (lane == 0) { S.und[wave] = bu; S.kep[wave] = bk; }
                }
                __syncthreads();
            }
            SB_MARK(14);
            {   // outputs: rank of each kept entry among this sub-batch's kept
                unsigned long long K[4];
#pragma unroll
                for (int w = 0; w < 4; ++w) K[w] = S.kep[w];
                const int budget = p.max_det - kept0;
                const int total = __popcll(K[0]) + __popcll(K[1]) + __popcll(K[2]) + __popcll(K[3]);
                if (tid < SB && iskept) {
                    int r = 0;
#pragma unroll
                    for (int w = 0; w < 4; ++w)
                        r += w < wave ? __popcll(K[w]) : (w == wave ? __popcll(K[w] & ((1ull << lane) - 1ull)) : 0);
                    if (r < budget) {
                        const int o = kept0 + r;
                        S.kb[o][0] = S.sb[tid][0]; S.kb[o][1] = S.sb[tid][1];
                        S.kb[o][2] = S.sb[tid][2]; S.kb[o][3] = S.sb[tid][3];
                        S.karea[o] = S.sarea[tid];
                        S.kcls[o] = S.scls[tid];
                        float* d = dets + o * 6;
                        d[0] = S.sraw[tid][0]; d[1] = S.sraw[tid][1]; d[2] = S.sraw[tid][2]; d[3] = S.sraw[tid][3];
                        d[4] = S.sscore[tid]; d[5] = S.scls[tid];
                    }
                }
                __syncthreads();
                if (tid == 0) {
                    S.kept = kept0 + min(total, budget);
                    S.rlo = lo; S.rhi = hi; S.rfin = fin;
                }
            }
            __syncthreads();
            SB_MARK(15);
            ++sbi;
        }
}

// Append every candidate key of image n with pred(key) to bkeys (order irrelevant: the batch
// is sorted next), enumerating the pairs from the scores (for_pairs) over units [u0, u1).
template <typename T, int U = 4, typename SM, typename Pred>
__device__ __forceinline__ void gather_pairs(SM& S, const NmsArgs& p, const T* y, int u0, int u1, int tid, Pred pred) {
    for_pairs<T, U>(p, y, u0, u1, tid, NMS_T, [&](unsigned long long k) {
        if (pred(k)) {
            const int pos = atomicAdd(&S.gcount, 1);
            if (pos < CAP) S.bkeys[pos] = k;
        }
    });
}

// block-wide inclusive scan of one value per thread (1024 threads)
template <typename SM>
__device__ unsigned block_scan_incl(SM& S, unsigned v, int lane, int wave) {
    unsigned incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) S.wsum[wave] = incl;
    __syncthreads();
    unsigned before = 0;
    for (int w = 0; w < wave; ++w) before += S.wsum[w];
    __syncthreads();
    return incl + before;
}

#define NMS_MARK(k)                                                                       \
    do {                                                                                  \
        if (NMS_TRACE && tid == 0) NMS_TRACE[n * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// ---- split greedy for the first batch (the only batch on typical images):
//   nms_prep    one workgroup per image: score-bin selection, gather and sort of the
//               first batch (as before), then every entry decoded once into the scratch
//   nms_mask    the batch's lower-triangular IoU bitmask, one wave per 64 x 64 tile (row i,
//               word w: bit jj <=> j = 64 w + jj < i and IoU > thr), all images in one grid
//   nms_finish  one workgroup per image: one wave resolves the greedy order 64 entries at a
//               time from the mask (LDS copy), all threads write the kept entries; later
//               batches (rare) continue with the single-workgroup path above
// The first batch no longer waits on one CU's 256-entry sub-batches: the n^2 / 2 pair
// tests spread over the whole chip.
constexpr int ENT = CAP;                      // entries of the first batch in the scratch
constexpr int MASKW = 64 * 64 * 65 / 2;       // triangular mask words for ENT entries
constexpr int NB_LDS = 19;                    // row blocks of the mask the resolve stages in LDS

__device__ __forceinline__ int tri(int b) { return 32 * b * (b + 1); }   // first word of row block b

// NmsArgs::state per image (8 words): [0] ub (every key < ub is unprocessed), [1] entries of
// the first batch, [2] score bin to continue from, [3] flags (bit 0: general path, bit 1:
// nothing left), [4] keys gathered so far (u32, zeroed by nms_zero), [5] keys selected for the
// first batch, [6] the batch's upper bin, [7] plain-coordinate extent of the batch (nms_prep)
constexpr int STW = 8;

__device__ __forceinline__ bool sep_of(unsigned long long ext, float max_wh) {
    const float lo = __uint_as_float((unsigned)ext), hi = __uint_as_float((unsigned)(ext >> 32));
    return max_wh > 0.0f && max_wh < 3.0e38f && hi - lo <= 0.5f * max_wh;   // false for the NaN pattern
}

// C[b] = number of candidates in score bins >= b (suffix sums of the emitted histogram)
template <typename SM>
__device__ void bin_suffix(SM& S, const NmsArgs& p, int n, int tid, int lane, int wave) {
    unsigned* C = S.hist;  // C[0..NBINS], C[NBINS] = 0
    const unsigned* gh = p.hist + (long long)n * NBINS;
    const int r0 = 2 * tid, r1 = 2 * tid + 1;  // reversed bin index: b = NBINS-1-r
    const unsigned h0 = gh[NBINS - 1 - r0], h1 = gh[NBINS - 1 - r1];
    const unsigned incl = block_scan_incl(S, h0 + h1, lane, wave);
    C[NBINS - 1 - r1] = incl;
    C[NBINS - 1 - r0] = incl - h1;
    if (tid == 0) C[NBINS] = 0;
    __syncthreads();
}

// The first batch: whole score bins (blo, bin_hi] holding >= FIRST_TARGET keys (or everything left),
// at most CAP; bcnt = 0 with flags bit 0: one bin alone exceeds CAP, bit 1: nothing to do.
template <typename SM>
__device__ void select_first(SM& S, int ktot, int tid, int& blo, int& bin_hi, int& bcnt, int& flags) {
    const unsigned* C = S.hist;
    bin_hi = NBINS - 1;
    bcnt = 0;
    blo = -1;
    flags = ktot > 0 ? 0 : 2;
    while (ktot > 0) {
        const unsigned c0 = C[bin_hi + 1];
        const unsigned target = c0 + (unsigned)FIRST_TARGET, cap = c0 + (unsigned)CAP;
        if (tid == 0) {  // default: everything that is left fits the minimum batch
            S.sel_bin = -1;
            S.sel_need = (int)(C[0] - c0);
        }
        __syncthreads();
        if (C[0] >= target) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int b = 2 * tid + e;
                if (b <= bin_hi && C[b + 1] < target && target <= C[b]) {
                    if (C[b] <= cap) { S.sel_bin = b - 1; S.sel_need = (int)(C[b] - c0); }
                    else { S.sel_bin = b; S.sel_need = (int)(C[b + 1] - c0); }
                }
            }
        }
        __syncthreads();
        blo = S.sel_bin;
        bcnt = S.sel_need;
        __syncthreads();
        if (bcnt == 0) {
            if (C[0] == c0) { flags = 2; break; }           // every candidate processed
            if (blo == bin_hi) { flags = 1; break; }        // one bin alone exceeds CAP
            bin_hi = blo;                                 // skip empty bins
            if (bin_hi < 0) { flags = 2; break; }
            continue;
        }
        break;
    }
}

// Gather of the first batch's keys, GATHER_G workgroups per image over slices of the
// candidate list (each recomputes the bin selection from the 8 KB histogram); matches are
// collected in LDS and appended to the image's gather buffer with one atomic per workgroup.
struct GatherSmem {
    unsigned hist[NBINS + 1];
    unsigned long long bkeys[CAP];
    unsigned wsum[NMS_T / 64];
    int sel_bin, sel_need, gcount, gbase;
};
constexpr int GATHER_G = 16;   // workgroups per image (each scans 1/16 of its scores)

template <typename T>
__global__ __launch_bounds__(NMS_T) void nms_gather(const NmsArgs p) {
    __shared__ GatherSmem S;
    const int n = blockIdx.y, g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nall = p.counts[n];
    const int ktot = min(nall, p.max_nms);
    if (tid == 0) S.gcount = 0;
    bin_suffix(S, p, n, tid, lane, wave);
    int blo, bin_hi, bcnt, flags;
    select_first(S, ktot, tid, blo, bin_hi, bcnt, flags);
    unsigned long long* st = p.state + (long long)n * STW;
    if (g == 0 && tid == 0) {
        st[2] = (unsigned long long)(long long)blo;
        st[3] = (unsigned long long)flags;
        st[5] = (unsigned long long)bcnt;
        st[6] = (unsigned long long)(long long)bin_hi;
    }
    if (bcnt == 0) return;
    // this workgroup's slice of the image's (class row, 8-anchor chunk) units
    const T* y = reinterpret_cast<const T*>(p.y) + (long long)n * (4 + p.nc) * p.A;
    const int nu = p.nc * ((p.A + EMIT_APT - 1) / EMIT_APT);
    const int per = (nu + gridDim.x - 1) / gridDim.x;
    const int u0 = g * per, u1 = min(nu, u0 + per);
    gather_pairs<T>(S, p, y, u0, u1, tid, [&](unsigned long long k) {
        const int bb = score_bin(__uint_as_float((unsigned)(k >> PBITS)), p.bin_base);
        return bb > blo && bb <= bin_hi;
    });
    __syncthreads();
    const int m = min(S.gcount, CAP);
    if (tid == 0) S.gbase = m ? (int)atomicAdd(reinterpret_cast<unsigned*>(st + 4), (unsigned)m) : 0;
    __syncthreads();
    unsigned long long* gk = p.gkeys + (long long)n * CAP;
    for (int t = tid; t < m; t += NMS_T)
        if (S.gbase + t < CAP) gk[S.gbase + t] = S.bkeys[t];
}

// Sort of the gathered first batch (bitonic in LDS), every entry decoded once.
template <typename T>
__global__ __launch_bounds__(NMS_T) void nms_prep(const NmsArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    NmsSmem& S = *reinterpret_cast<NmsSmem*>(smem_raw);
    const int n = blockIdx.x, tid = threadIdx.x;
    const T* y = reinterpret_cast<const T*>(p.y) + (long long)n * (4 + p.nc) * p.A;
    const int nall = p.counts[n];
    const int ktot = min(nall, p.max_nms);
    unsigned long long* st = p.state + (long long)n * STW;
    NMS_MARK(0);
    NMS_MARK(1);
    if (NMS_TRACE && tid == 0) NMS_TRACE[n * 16 + 7] = __builtin_amdgcn_s_memtime();
    const int bcnt = (int)st[5];
    const int want = min(bcnt, ktot);
    if (bcnt > 0) {
        const unsigned long long* gk = p.gkeys + (long long)n * CAP;
        for (int t = tid; t < bcnt; t += NMS_T) S.bkeys[t] = gk[t];
        __syncthreads();
        NMS_MARK(2);
        sort_batch(S, bcnt, tid);
    }
    float4* E = reinterpret_cast<float4*>(p.ents) + (long long)n * 3 * ENT;
    // class separability: with every plain coordinate of the batch in [lo, hi] and
    // hi - lo <= max_wh / 2, boxes of different classes (offset by c * max_wh, rounding
    // monotonic) cannot intersect, so nms_mask tests same-class pairs only (sep_of)
    float lo = INFINITY, hi = -INFINITY;
    bool finite = true;
    for (int t = tid; t < want; t += NMS_T) {
        float ob[4], raw[4], area, score, cls;
        decode_key<T>(p, y, S.bkeys[t], ob, raw, area, score, cls);
        E[t] = make_float4(ob[0], ob[1], ob[2], ob[3]);
        E[ENT + t] = make_float4(raw[0], raw[1], raw[2], raw[3]);
        E[2 * ENT + t] = make_float4(area, score, cls, 0.0f);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            finite &= fabsf(raw[k]) < 3.0e38f;   // false for inf and NaN
            lo = fminf(lo, raw[k]);
            hi = fmaxf(hi, raw[k]);
        }
    }
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, d));
        hi = fmaxf(hi, __shfl_xor(hi, d));
    }
    const bool wfin = __ballot(!finite) == 0ull;
    __shared__ float wlo[NMS_T / 64], whi[NMS_T / 64];
    __shared__ int wok[NMS_T / 64];
    if (lane == 0) { wlo[wave] = lo; whi[wave] = hi; wok[wave] = wfin; }
    __syncthreads();
    if (tid == 0) {
        bool ok = true;
        for (int w = 0; w < NMS_T / 64; ++w) {
            lo = fminf(lo, wlo[w]);
            hi = fmaxf(hi, whi[w]);
            ok &= wok[w] != 0;
        }
        // [7]: the batch's plain-coordinate extent (lo, hi) as float bits, all ones if not finite
        st[7] = ok ? ((unsigned long long)__float_as_uint(hi) << 32) | __float_as_uint(lo) : ~0ull;
        st[0] = want > 0 ? S.bkeys[want - 1] : ~0ull;
        st[1] = (unsigned long long)want;
        if (want == 0) st[2] = (unsigned long long)(long long)(int)st[6];   // no batch: bin_hi unchanged
    }
    NMS_MARK(3);
}

// One wave per 64 x 64 tile of a triangle (row block rb, word w <= rb); the tiles of every
// image of the batch are numbered globally and strided over the grid, so one image's large
// first batch spreads over the whole chip. Lane r holds row entry 64 rb + r; the tile's 64
// column entries are staged in LDS. A lane tests only the columns that can hit: those of
// its own class when the image's classes are separable (most pairs: other classes), else all.
constexpr int MASK_T = 256;

__global__ __launch_bounds__(MASK_T) void nms_mask(const NmsArgs p) {
    extern __shared__ int pre[];   // [B + 1]: first global tile of image n
    __shared__ float4 colb[MASK_T / 64][64];
    __shared__ float cola[MASK_T / 64][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (wave == 0) {
        int carry = 0;
        for (int c0 = 0; c0 < p.B; c0 += 64) {
            const int n = c0 + lane;
            int v = 0;
            if (n < p.B) {
                const int nb = ((int)p.state[(long long)n * STW + 1] + 63) >> 6;
                v = nb * (nb + 1) / 2;
            }
            int incl = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int o = __shfl_up(incl, d);
                if (lane >= d) incl += o;
            }
            if (n < p.B) pre[n + 1] = carry + incl;
            carry += __shfl(incl, 63);
        }
        if (lane == 0) pre[0] = 0;
    }
    __syncthreads();
    const int total = pre[p.B];
    const IouThr th = make_thr(p.iou);
    for (int t = blockIdx.x * (MASK_T / 64) + wave; t < total; t += gridDim.x * (MASK_T / 64)) {
        int lo = 0, hi = p.B - 1;   // image: the last n with pre[n] <= t
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pre[mid] <= t) lo = mid;
            else hi = mid - 1;
        }
        const int n = lo, q = t - pre[n];
        const int want = (int)p.state[(long long)n * STW + 1];
        const bool sep = th.nonneg && sep_of(p.state[(long long)n * STW + 7], p.max_wh);   // thr < 0: all pairs
        int rb = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
        while (rb * (rb + 1) / 2 > q) --rb;
        while ((rb + 1) * (rb + 2) / 2 <= q) ++rb;
        const int w = q - rb * (rb + 1) / 2;
        const float4* E = reinterpret_cast<const float4*>(p.ents) + (long long)n * 3 * ENT;
        const int i = rb * 64 + lane, j = w * 64 + lane;
        const int ic = min(i, want - 1), jc = min(j, want - 1);
        const float4 bi = E[ic], xi = E[2 * ENT + ic];
        const float4 bj = E[jc], xj = E[2 * ENT + jc];
        colb[wave][lane] = bj;
        cola[wave][lane] = xj.x;
        const int jlim = min(i, want) - w * 64;   // columns jj < jlim (j < i, j < want)
        unsigned long long cm = jlim >= 64 ? ~0ull : (jlim > 0 ? (1ull << jlim) - 1ull : 0ull);
        if (sep) {
            const int ci = (int)xi.z, cj = (int)xj.z;
            unsigned long long same = 0;
#pragma unroll
            for (int jj = 0; jj < 64; ++jj) same |= (unsigned long long)(__builtin_amdgcn_readlane(cj, jj) == ci) << jj;
            cm &= same;
        }
        if (i >= want) cm = 0;
        unsigned long long m = 0;
        while (cm) {   // the wave runs max-over-lanes candidate columns
            const int jj = __ffsll((long long)cm) - 1;
            cm &= cm - 1ull;
            const float4 b = colb[wave][jj];
            const float a = cola[wave][jj];
            bool hit;
            if (th.nonneg) {
                bool slow = false;
                hit = iou_fast(bi.x, bi.y, bi.z, bi.w, xi.x, b.x, b.y, b.z, b.w, a, th, slow);
                if (slow) hit = iou_above(bi.x, bi.y, bi.z, bi.w, xi.x, b.x, b.y, b.z, b.w, a, th);
            } else {
                hit = iou_above(bi.x, bi.y, bi.z, bi.w, xi.x, b.x, b.y, b.z, b.w, a, th);
            }
            m |= (unsigned long long)hit << jj;
        }
        p.mask[(long long)n * MASKW + tri(rb) + w * 64 + lane] = m;
    }
}

// The greedy over the first batch from its mask, then (rarely) the later batches.
template <typename T>
__device__ void nms_rest(NmsSmem& S, const NmsArgs& p, const T* y, float* dets,
                         int nall, int ktot, int processed, unsigned long long ub, int bin_hi, bool fallback,
                         int tid, int lane, int wave) {
    const int n = blockIdx.x;
    const int nu = p.nc * ((p.A + EMIT_APT - 1) / EMIT_APT);   // the image's (class row, chunk) units
    unsigned* C = S.hist;
    {
        const unsigned* gh = p.hist + (long long)n * NBINS;
        const int r0 = 2 * tid, r1 = 2 * tid + 1;
        const unsigned h0 = gh[NBINS - 1 - r0], h1 = gh[NBINS - 1 - r1];
        const unsigned incl = block_scan_incl(S, h0 + h1, lane, wave);
        C[NBINS - 1 - r1] = incl;
        C[NBINS - 1 - r0] = incl - h1;
        if (tid == 0) C[NBINS] = 0;
    }
    __syncthreads();
    NMS_MARK(8);
    // ---- fast path: batches of whole score bins, ~1024..CAP keys, exact order by an LDS sort
    while (!fallback && processed < ktot && S.kept < p.max_det && bin_hi >= 0) {
        const unsigned c0 = C[bin_hi + 1];
        const unsigned target = c0 + 640u, cap = c0 + (unsigned)CAP;
        if (tid == 0) {
            S.sel_bin = -1;
            S.sel_need = (int)(C[0] - c0);
        }
        __syncthreads();
        if (C[0] >= target) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int b = 2 * tid + e;
                if (b <= bin_hi && C[b + 1] < target && target <= C[b]) {
                    if (C[b] <= cap) { S.sel_bin = b - 1; S.sel_need = (int)(C[b] - c0); }
                    else { S.sel_bin = b; S.sel_need = (int)(C[b + 1] - c0); }
                }
            }
        }
        __syncthreads();
        const int blo = S.sel_bin, bcnt = S.sel_need;
        __syncthreads();
        if (bcnt == 0) {
            if (C[0] == c0) break;                        // every candidate processed
            if (blo == bin_hi) { fallback = true; break; }  // one bin alone exceeds CAP
            bin_hi = blo;                                 // skip empty bins
            continue;
        }
        if (tid == 0) S.gcount = 0;
        __syncthreads();
        const unsigned long long tg0 = NMS_TRACE ? __builtin_amdgcn_s_memrealtime() : 0ull;
        gather_pairs<T, 2>(S, p, y, 0, nu, tid, [&](unsigned long long k) {
            const int bb = score_bin(__uint_as_float((unsigned)(k >> PBITS)), p.bin_base);
            return bb > blo && bb <= bin_hi;
        });
        __syncthreads();
        // diagnostic builds: slot 9 sums the batches' score scans (bits 40+: batches), 11 their sorts
        const unsigned long long tg1 = NMS_TRACE ? __builtin_amdgcn_s_memrealtime() : 0ull;
        const int want = min(bcnt, ktot - processed);
        sort_batch(S, bcnt, tid);
        if (NMS_TRACE && tid == 0) {
            NMS_TRACE[n * 16 + 9] += tg1 - tg0 + (1ull << 40);
            NMS_TRACE[n * 16 + 11] += __builtin_amdgcn_s_memrealtime() - tg1;
        }
        nms_batch<T>(S, p, y, dets, want, tid, lane, wave);
        processed += want;
        ub = S.bkeys[want - 1];
        bin_hi = blo;
        __syncthreads();
    }
    if (fallback) {
        // ---- general path: radix-select the next <= CAP keys below ub (exact for any ties)
        while (processed < ktot && S.kept < p.max_det) {
            int want = min(CAP, ktot - processed);
            const unsigned long long tf0 = NMS_TRACE ? __builtin_amdgcn_s_memrealtime() : 0ull;
            if (tid == 0) S.gcount = 0;
            __syncthreads();
            {
                int c = 0;
                for_pairs<T, 2>(p, y, 0, nu, tid, NMS_T, [&](unsigned long long k) { c += k < ub; });
                atomicAdd(&S.gcount, c);
            }
            __syncthreads();
            const int remaining = S.gcount;
            __syncthreads();
            if (remaining == 0) break;
            unsigned long long lo = 0;
            if (remaining > want) {
                unsigned long long prefix = 0;
                int need = want;
                for (int lvl = 0; lvl < 4; ++lvl) {
                    const int shift = 56 - DBITS * (lvl + 1);
                    for (int i = tid; i < HBINS; i += NMS_T) S.hist[i] = 0;
                    __syncthreads();
                    for_pairs<T, 2>(p, y, 0, nu, tid, NMS_T, [&](unsigned long long k) {
                        if (k < ub && (lvl == 0 || (k >> (shift + DBITS)) == prefix))
                            atomicAdd(&S.hist[(k >> shift) & (HBINS - 1)], 1u);
                    });
                    __syncthreads();
                    constexpr int PER = HBINS / NMS_T;
                    unsigned local = 0;
#pragma unroll
                    for (int b = 0; b < PER; ++b) local += S.hist[tid * PER + b];
                    unsigned incl = local;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const unsigned o = __shfl_down(incl, d);
                        if (lane + d < 64) incl += o;
                    }
                    if (lane == 0) S.wsum[wave] = incl;
                    __syncthreads();
                    unsigned above = 0;
                    for (int w2 = wave + 1; w2 < NMS_T / 64; ++w2) above += S.wsum[w2];
                    above += incl - local;
                    if (above < (unsigned)need && above + local >= (unsigned)need) {
                        unsigned cum = above;
                        for (int b = PER - 1; b >= 0; --b) {
                            const unsigned h = S.hist[tid * PER + b];
                            if (cum + h >= (unsigned)need) {
                                S.sel_bin = tid * PER + b;
                                S.sel_need = need - (int)cum;
                                break;
                            }
                            cum += h;
                        }
                    }
                    __syncthreads();
                    prefix = (prefix << DBITS) | (unsigned long long)S.sel_bin;
                    need = S.sel_need;
                    __syncthreads();
                }
                lo = prefix;
            } else {
                want = remaining;
            }
            if (tid == 0) S.gcount = 0;
            __syncthreads();
            gather_pairs<T, 2>(S, p, y, 0, nu, tid, [&](unsigned long long k) { return k >= lo && k < ub; });
            __syncthreads();
            const unsigned long long tf1 = NMS_TRACE ? __builtin_amdgcn_s_memrealtime() : 0ull;
            sort_batch(S, want, tid);
            if (NMS_TRACE && tid == 0) {
                NMS_TRACE[n * 16 + 9] += tf1 - tf0 + (1ull << 40);
                NMS_TRACE[n * 16 + 11] += __builtin_amdgcn_s_memrealtime() - tf1;
            }
            nms_batch<T>(S, p, y, dets, want, tid, lane, wave);
            processed += want;
            ub = lo;
            __syncthreads();
        }
    }
}

template <typename T>
__global__ __launch_bounds__(NMS_T) void nms_finish(const NmsArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    NmsSmem& S = *reinterpret_cast<NmsSmem*>(smem_raw);
    __shared__ unsigned long long Kw[64];   // kept entries of row block b (bit r = entry 64 b + r)
    __shared__ int Kpre[65];                // kept entries before block b
    __shared__ int nbd_s;
    const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const T* y = reinterpret_cast<const T*>(p.y) + (long long)n * (4 + p.nc) * p.A;
    float* dets = p.dets + (long long)n * p.max_det * 6;
    const int nall = p.counts[n];
    const int ktot = min(nall, p.max_nms);
    const unsigned long long* st = p.state + (long long)n * STW;
    const unsigned long long ub = st[0];
    const int want = (int)st[1], bin_hi = (int)(long long)st[2], flags = (int)st[3];
    NMS_MARK(4);
    if (tid == 0) {
        S.kept = 0;
        const unsigned long long ext = want > 0 ? st[7] : 0xff800000'7f800000ull;   // (+inf, -inf): empty
        S.rlo = __uint_as_float((unsigned)ext);
        S.rhi = __uint_as_float((unsigned)(ext >> 32));
        S.rfin = ext != ~0ull;
    }
    if (want > 0) {
        // the mask's first NB_LDS row blocks into LDS (over the histogram and key areas, unused
        // until a later batch), the rest read from the scratch
        unsigned long long* ML = reinterpret_cast<unsigned long long*>(smem_raw);
        static_assert(64 * NB_LDS * (NB_LDS + 1) / 2 * 8 <= offsetof(NmsSmem, sb), "mask LDS overlay too large");
        const unsigned long long* MG = p.mask + (long long)n * MASKW;
        const int nb = (want + 63) >> 6, nbl = min(nb, NB_LDS);
        for (int x = tid; x < tri(nbl); x += NMS_T) ML[x] = MG[x];
        __syncthreads();
        if (wave == 0) {
            // block b: entry i = 64 b + r is suppressed by a kept entry of an earlier block (its
            // row's words w < b against Kw[w]) or of this block (its diagonal word, resolved in
            // order; entries without an in-block suppressor are decided at once)
            int kacc = 0, nbd = nb;
            for (int b = 0; b < nb; ++b) {
                const int i = b * 64 + lane;
                const bool valid = i < want;
                bool sup = false;
                unsigned long long diag = 0;
                if (valid) {
                    unsigned long long acc = 0;
                    if (b < NB_LDS) {
                        const unsigned long long* src = ML + tri(b) + lane;
#pragma unroll 8
                        for (int w = 0; w < b; ++w) acc |= src[w * 64] & Kw[w];
                        diag = src[b * 64];
                    } else {
                        const unsigned long long* src = MG + tri(b) + lane;
#pragma unroll 8
                        for (int w = 0; w < b; ++w) acc |= src[w * 64] & Kw[w];
                        diag = src[b * 64];
                    }
                    sup = acc != 0ull;
                }
                const unsigned long long vm = __ballot(valid), sm = __ballot(sup), dm = __ballot(diag != 0ull);
                unsigned long long kb = vm & ~sm & ~dm, todo = vm & ~sm & dm;
                const unsigned dlo = (unsigned)diag, dhi = (unsigned)(diag >> 32);
                while (todo) {
                    const int r = __ffsll((long long)todo) - 1;
                    // (readlane returns int: widen through unsigned, not by sign extension)
                    const unsigned long long d = (unsigned long long)(unsigned)__builtin_amdgcn_readlane(dlo, r) |
                                                 ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(dhi, r) << 32);
                    if (!(d & kb)) kb |= 1ull << r;
                    todo &= todo - 1ull;
                }
                int c = __popcll(kb);
                const int need = p.max_det - kacc;
                if (c >= need) {   // the greedy stops at max_det kept: the first `need` of this block
                    unsigned long long keep = 0, rest = kb;
                    for (int k = 0; k < need; ++k) {
                        keep |= rest & (~rest + 1ull);
                        rest &= rest - 1ull;
                    }
                    kb = keep;
                    c = need;
                }
                if (lane == 0) { Kw[b] = kb; Kpre[b] = kacc; }
                kacc += c;
                if (kacc >= p.max_det) { nbd = b + 1; break; }
            }
            if (lane == 0) { Kpre[nbd] = kacc; nbd_s = nbd; S.kept = kacc; }
        }
        __syncthreads();
        NMS_MARK(5);
        const int nbd = nbd_s;
        const float4* E = reinterpret_cast<const float4*>(p.ents) + (long long)n * 3 * ENT;
        for (int t = tid; t < want && t < nbd * 64; t += NMS_T) {
            const int b = t >> 6, r = t & 63;
            const unsigned long long K = Kw[b];
            if ((K >> r) & 1ull) {
                const int o = Kpre[b] + __popcll(K & ((1ull << r) - 1ull));
                const float4 ob = E[t], raw = E[ENT + t], ax = E[2 * ENT + t];
                S.kb[o][0] = ob.x; S.kb[o][1] = ob.y; S.kb[o][2] = ob.z; S.kb[o][3] = ob.w;
                S.karea[o] = ax.x;
                S.kcls[o] = ax.z;
                float* d = dets + o * 6;
                d[0] = raw.x; d[1] = raw.y; d[2] = raw.z; d[3] = raw.w;
                d[4] = ax.y; d[5] = ax.z;
            }
        }
    }
    __syncthreads();
    const bool fallback = (flags & 1) != 0;
    const bool more = !(flags & 2) && want < ktot && S.kept < p.max_det && (fallback || bin_hi >= 0);
    if (more) nms_rest<T>(S, p, y, dets, nall, ktot, want, ub, bin_hi, fallback, tid, lane, wave);
    NMS_MARK(6);
    if (NMS_TRACE && tid == 0) NMS_TRACE[n * 16 + 10] = __builtin_amdgcn_s_memtime();
    if (tid == 0) p.ndet[n] = S.kept;
}

template <typename T>
int launch_nms_t(const NmsArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(nms_zero, dim3((a.B * NBINS + 255) / 256), dim3(256), 0, s, a.counts, a.hist, a.state, a.B);
    const int per_block = EMIT_CHUNKS * EMIT_APT;
    hipLaunchKernelGGL((nms_emit<T>), dim3((a.A + per_block - 1) / per_block, a.B), dim3(256), 0, s, a);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&nms_prep<T>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(NmsSmem));
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&nms_finish<T>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(NmsSmem));
        attr = true;
    }
    hipLaunchKernelGGL((nms_gather<T>), dim3(GATHER_G, a.B), dim3(NMS_T), 0, s, a);
    hipLaunchKernelGGL((nms_prep<T>), dim3(a.B), dim3(NMS_T), sizeof(NmsSmem), s, a);
    // about one 64 x 64 tile per wave at the typical first batch (~1000 entries: 136 tiles per image)
    hipLaunchKernelGGL(nms_mask, dim3(std::min(4096, 32 * a.B)), dim3(MASK_T), (a.B + 1) * sizeof(int), s, a);
    hipLaunchKernelGGL((nms_finish<T>), dim3(a.B), dim3(NMS_T), sizeof(NmsSmem), s, a);
    return (int)hipGetLastError();
}

}  // namespace

int launch_nms(int dtype, const NmsArgs& a, hipStream_t s) {
    if (a.max_det > MAXDET || (long long)a.A * a.nc > (long long)PMASK) return (int)hipErrorInvalidValue;
    switch (dtype) {
        case F32: return launch_nms_t<float>(a, s);
        case F16: return launch_nms_t<_Float16>(a, s);
        case BF16: return launch_nms_t<__bf16>(a, s);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace yh

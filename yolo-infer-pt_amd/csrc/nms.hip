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
//   nms_emit   grid (A/256, B): every pair above conf becomes a 56-bit key
//              (score bits << 26 | (2^26-1 - pair)); larger key = earlier in the
//              reference order. Block-scanned, one atomic per block.
//   nms_image  one 1024-thread workgroup per image: repeatedly radix-selects the
//              next <= 4096 keys (4 x 14-bit digit histograms in LDS), gathers and
//              bitonic-sorts them in LDS, then runs greedy NMS on 256-key
//              sub-batches: parallel test against the kept set, a 256x256 IoU
//              bitmask, and a one-wave sequential resolve. Stops at max_det kept
//              or max_nms processed, so typical images touch one batch only.
#include "common.h"
#include "dtypes.h"

#pragma clang fp contract(off)

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

__device__ __forceinline__ int score_bin(float s, int base) {
    const int b = (int)(__float_as_uint(s) >> 16) - base;
    return b < 0 ? 0 : (b >= NBINS ? NBINS - 1 : b);
}

template <typename T>
__global__ __launch_bounds__(256) void nms_emit(const NmsArgs p) {
    __shared__ int wtot[4];
    __shared__ int sbase;
    __shared__ unsigned lhist[NBINS];
    for (int i = threadIdx.x; i < NBINS; i += 256) lhist[i] = 0;
    const int n = blockIdx.y;
    const int a = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const T* y = reinterpret_cast<const T*>(p.y) + (long long)n * (4 + p.nc) * p.A;
    int cnt = 0;
    if (a < p.A)
        for (int c = 0; c < p.nc; ++c) cnt += tof(y[(long long)(4 + c) * p.A + a]) > p.conf;
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    if (threadIdx.x == 0) sbase = atomicAdd(&p.counts[n], wtot[0] + wtot[1] + wtot[2] + wtot[3]);
    __syncthreads();
    int off = sbase + incl - cnt;
    for (int w = 0; w < wave; ++w) off += wtot[w];
    if (a < p.A && cnt) {
        unsigned long long* keys = p.keys + (long long)n * p.A * p.nc;
        for (int c = 0; c < p.nc; ++c) {
            const float s = tof(y[(long long)(4 + c) * p.A + a]);
            if (s > p.conf) {
                keys[off++] = make_key(s, (unsigned)(a * p.nc + c));
                atomicAdd(&lhist[score_bin(s, p.bin_base)], 1u);
            }
        }
    }
    __syncthreads();
    unsigned* gh = p.hist + (long long)n * NBINS;
    for (int i = threadIdx.x; i < NBINS; i += 256)
        if (lhist[i]) atomicAdd(&gh[i], lhist[i]);
}

__device__ __forceinline__ bool iou_above(float ax1, float ay1, float ax2, float ay2, float aa,
                                          float bx1, float by1, float bx2, float by2, float ba, float thr) {
    const float xx1 = fmaxf(ax1, bx1), yy1 = fmaxf(ay1, by1);
    const float xx2 = fminf(ax2, bx2), yy2 = fminf(ay2, by2);
    const float w = fmaxf(0.0f, xx2 - xx1), h = fmaxf(0.0f, yy2 - yy1);
    const float inter = w * h;
    const float ovr = inter / (aa + ba - inter);
    return ovr > thr;
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
    float kb[MAXDET][4];
    float karea[MAXDET];
    unsigned wsum[NMS_T / 64];
    unsigned long long sel_prefix;
    int sel_need, sel_bin, gcount, kept;
};

template <typename T>
__device__ __forceinline__ float round_t(float v) { return tof(fromf<T>(v)); }


__device__ void sort_batch(NmsSmem& S, int count, int tid) {
    int P = 1;
    while (P < count) P <<= 1;
    for (int i = count + tid; i < P; i += NMS_T) S.bkeys[i] = 0;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P; i += NMS_T) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long a = S.bkeys[i], b = S.bkeys[ixj];
                    const bool desc = (i & k) == 0;
                    if (desc ? (a < b) : (a > b)) { S.bkeys[i] = b; S.bkeys[ixj] = a; }
                }
            }
            __syncthreads();
        }
    }
}

// Greedy NMS over the first `want` keys of the sorted batch (sub-batches of SB).
template <typename T>
__device__ void nms_batch(NmsSmem& S, const NmsArgs& p, const T* y, float* dets, int want, int tid, int lane, int wave) {
        for (int s0 = 0; s0 < want && S.kept < p.max_det; s0 += SB) {
            const int ns = min(SB, want - s0);
            if (tid < ns) {
                const unsigned long long key = S.bkeys[s0 + tid];
                const unsigned pair = PMASK - (unsigned)(key & PMASK);
                const int a = (int)(pair / (unsigned)p.nc), c = (int)(pair - (unsigned)a * p.nc);
                const float cx = tof(y[a]), cy = tof(y[(long long)p.A + a]);
                const float w = tof(y[2LL * p.A + a]), h = tof(y[3LL * p.A + a]);
                // wh2xy (util.py:76-82) in the input dtype
                const float x1 = round_t<T>(cx - w / 2.0f), y1 = round_t<T>(cy - h / 2.0f);
                const float x2 = round_t<T>(cx + w / 2.0f), y2 = round_t<T>(cy + h / 2.0f);
                const float off = (float)c * p.max_wh;
                const float bx1 = x1 + off, by1 = y1 + off, bx2 = x2 + off, by2 = y2 + off;
                S.sb[tid][0] = bx1; S.sb[tid][1] = by1; S.sb[tid][2] = bx2; S.sb[tid][3] = by2;
                S.sarea[tid] = (bx2 - bx1) * (by2 - by1);
                S.sraw[tid][0] = x1; S.sraw[tid][1] = y1; S.sraw[tid][2] = x2; S.sraw[tid][3] = y2;
                S.sscore[tid] = tof(y[(long long)(4 + c) * p.A + a]);
                S.scls[tid] = (float)c;
            }
            if (tid < SB / 32) S.supp[tid] = 0;
            __syncthreads();
            const int kept0 = S.kept;
            {   // suppressed by an already-kept box? 4 threads per entry
                const int e = tid >> 2, part = tid & 3;
                if (e < ns) {
                    bool sup = false;
                    for (int k = part; k < kept0 && !sup; k += 4)
                        sup = iou_above(S.kb[k][0], S.kb[k][1], S.kb[k][2], S.kb[k][3], S.karea[k],
                                        S.sb[e][0], S.sb[e][1], S.sb[e][2], S.sb[e][3], S.sarea[e], p.iou);
                    if (sup) atomicOr(&S.supp[e >> 5], 1u << (e & 31));
                }
            }
            {   // pairwise mask: bit j of row i set if j > i and IoU(i, j) > thr
                const int i = tid >> 2, wd = tid & 3;
                unsigned long long m = 0;
                if (i < ns) {
                    const float ix1 = S.sb[i][0], iy1 = S.sb[i][1], ix2 = S.sb[i][2], iy2 = S.sb[i][3], ia = S.sarea[i];
                    for (int jj = 0; jj < 64; ++jj) {
                        const int j = wd * 64 + jj;
                        if (j > i && j < ns &&
                            iou_above(ix1, iy1, ix2, iy2, ia, S.sb[j][0], S.sb[j][1], S.sb[j][2], S.sb[j][3], S.sarea[j], p.iou))
                            m |= 1ull << jj;
                    }
                }
                S.smask[i][wd] = m;
            }
            __syncthreads();
            if (wave == 0) {
                unsigned long long removed = 0;
                if (lane < 4) removed = (unsigned long long)S.supp[2 * lane] | ((unsigned long long)S.supp[2 * lane + 1] << 32);
                int kept = kept0;
                for (int i = 0; i < ns && kept < p.max_det; ++i) {
                    const unsigned long long rw = __shfl(removed, i >> 6);
                    if ((rw >> (i & 63)) & 1ull) continue;
                    if (lane < 4) {
                        S.kb[kept][lane] = S.sb[i][lane];
                        removed |= S.smask[i][lane];
                    }
                    if (lane == 0) S.karea[kept] = S.sarea[i];
                    if (lane < 6) {
                        const float v = lane < 4 ? S.sraw[i][lane] : (lane == 4 ? S.sscore[i] : S.scls[i]);
                        dets[kept * 6 + lane] = v;
                    }
                    ++kept;
                }
                if (lane == 0) S.kept = kept;
            }
            __syncthreads();
        }
}

// block-wide inclusive scan of one value per thread (1024 threads)
__device__ unsigned block_scan_incl(NmsSmem& S, unsigned v, int lane, int wave) {
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

template <typename T>
__global__ __launch_bounds__(NMS_T) void nms_image(const NmsArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    NmsSmem& S = *reinterpret_cast<NmsSmem*>(smem_raw);
    const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const T* y = reinterpret_cast<const T*>(p.y) + (long long)n * (4 + p.nc) * p.A;
    const unsigned long long* keys = p.keys + (long long)n * p.A * p.nc;
    float* dets = p.dets + (long long)n * p.max_det * 6;
    const int nall = p.counts[n];
    const int ktot = min(nall, p.max_nms);
    if (tid == 0) S.kept = 0;

    // C[b] = number of candidates in score bins >= b (suffix sums of the emitted histogram)
    unsigned* C = S.hist;  // C[0..NBINS], C[NBINS] = 0
    {
        const unsigned* gh = p.hist + (long long)n * NBINS;
        const int r0 = 2 * tid, r1 = 2 * tid + 1;  // reversed bin index: b = NBINS-1-r
        const unsigned h0 = gh[NBINS - 1 - r0], h1 = gh[NBINS - 1 - r1];
        const unsigned incl = block_scan_incl(S, h0 + h1, lane, wave);
        C[NBINS - 1 - r1] = incl;
        C[NBINS - 1 - r0] = incl - h1;
        if (tid == 0) C[NBINS] = 0;
    }
    __syncthreads();

    int processed = 0;
    unsigned long long ub = ~0ull;  // every key < ub is still unprocessed
    // ---- fast path: batches of whole score bins, ~1024..CAP keys, exact order by an LDS sort
    int bin_hi = NBINS - 1;
    bool fallback = false;
    while (processed < ktot && S.kept < p.max_det && bin_hi >= 0) {
        const unsigned c0 = C[bin_hi + 1];
        const unsigned target = c0 + 1024u, cap = c0 + (unsigned)CAP;
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
        for (int i0 = 0; i0 < nall; i0 += NMS_T) {
            const int i = i0 + tid;
            unsigned long long k = 0;
            bool hit = false;
            if (i < nall) {
                k = keys[i];
                const int bb = score_bin(__uint_as_float((unsigned)(k >> PBITS)), p.bin_base);
                hit = bb > blo && bb <= bin_hi;
            }
            const unsigned long long bal = __ballot(hit);
            if (bal) {
                const int leader = __ffsll((long long)bal) - 1;
                int base = 0;
                if (lane == leader) base = atomicAdd(&S.gcount, __popcll(bal));
                base = __shfl(base, leader);
                if (hit) {
                    const int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
                    if (pos < CAP) S.bkeys[pos] = k;
                }
            }
        }
        __syncthreads();
        const int want = min(bcnt, ktot - processed);
        sort_batch(S, bcnt, tid);
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
            if (tid == 0) S.gcount = 0;
            __syncthreads();
            {
                int c = 0;
                for (int i = tid; i < nall; i += NMS_T) c += keys[i] < ub;
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
                    for (int i = tid; i < nall; i += NMS_T) {
                        const unsigned long long k = keys[i];
                        if (k < ub && (lvl == 0 || (k >> (shift + DBITS)) == prefix))
                            atomicAdd(&S.hist[(k >> shift) & (HBINS - 1)], 1u);
                    }
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
            for (int i0 = 0; i0 < nall; i0 += NMS_T) {
                const int i = i0 + tid;
                unsigned long long k = 0;
                bool hit = false;
                if (i < nall) { k = keys[i]; hit = k >= lo && k < ub; }
                const unsigned long long bal = __ballot(hit);
                if (bal) {
                    const int leader = __ffsll((long long)bal) - 1;
                    int base = 0;
                    if (lane == leader) base = atomicAdd(&S.gcount, __popcll(bal));
                    base = __shfl(base, leader);
                    if (hit) {
                        const int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
                        if (pos < CAP) S.bkeys[pos] = k;
                    }
                }
            }
            __syncthreads();
            sort_batch(S, want, tid);
            nms_batch<T>(S, p, y, dets, want, tid, lane, wave);
            processed += want;
            ub = lo;
            __syncthreads();
        }
    }
    if (tid == 0) p.ndet[n] = S.kept;
}

template <typename T>
int launch_nms_t(const NmsArgs& a, hipStream_t s) {
    hipError_t e = hipMemsetAsync(a.counts, 0, sizeof(int) * a.B, s);
    if (e != hipSuccess) return (int)e;
    e = hipMemsetAsync(a.hist, 0, sizeof(unsigned) * NBINS * a.B, s);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL((nms_emit<T>), dim3((a.A + 255) / 256, a.B), dim3(256), 0, s, a);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&nms_image<T>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(NmsSmem));
        attr = true;
    }
    hipLaunchKernelGGL((nms_image<T>), dim3(a.B), dim3(NMS_T), sizeof(NmsSmem), s, a);
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
